// Trimesh terrain on the device (setup time): isaacgym terrain_utils.convert_heightfield_to_trimesh
// as legged_gym calls it for mesh_type 'trimesh' (terrain.py:70-73, slope_treshold of
// legged_robot_config.py:68; the mesh is added at legged_robot.py:629-643), plus the contact table
// the physics kernel reads (lgx_buffers.hf_trimesh).  One thread per vertex: the moves of the slope
// correction compare the vertex with its x / y / diagonal neighbours; the contact flag ORs the
// moves of the 4 x 4 vertex block (rows i-1 .. i+2, cols j-1 .. j+2), recomputed per vertex from
// the heights (no second pass).  HBM-bound byte work: 2 B read (x ~25 with neighbour re-reads from
// L1/L2) and 12 + 12 + 1 B written per vertex.
#include <stdint.h>

#include "lgx_internal.h"

namespace {

inline double __dmul_rn_host(double a, double b) { return a * b; }

// move (dx, dy) of vertex (i, j): +1 toward a neighbour higher by more than thr, -1 toward a
// previous neighbour higher by more than thr; the diagonal move applies where the axis move is 0
// (integer height differences compared with the threshold in double, as numpy compares them)
__device__ __forceinline__ void tm_move(const int16_t* __restrict__ hf, int rows, int cols, double thr, int i, int j,
                                        int* dx, int* dy) {
  const int h = hf[(int64_t)i * cols + j];
  int mx = 0, my = 0, mc = 0;
  if (i + 1 < rows && (double)(hf[(int64_t)(i + 1) * cols + j] - h) > thr) mx += 1;
  if (i > 0 && (double)(hf[(int64_t)(i - 1) * cols + j] - h) > thr) mx -= 1;
  if (j + 1 < cols && (double)(hf[(int64_t)i * cols + j + 1] - h) > thr) my += 1;
  if (j > 0 && (double)(hf[(int64_t)i * cols + j - 1] - h) > thr) my -= 1;
  if (i + 1 < rows && j + 1 < cols && (double)(hf[(int64_t)(i + 1) * cols + j + 1] - h) > thr) mc += 1;
  if (i > 0 && j > 0 && (double)(hf[(int64_t)(i - 1) * cols + j - 1] - h) > thr) mc -= 1;
  *dx = mx + (mx == 0 ? mc : 0);
  *dy = my + (my == 0 ? mc : 0);
}

__global__ void __launch_bounds__(256) lgx_trimesh_kernel(const int16_t* __restrict__ hf, int rows, int cols, double hs,
                                                          double vs, double thr, double xstep, double ystep,
                                                          float* __restrict__ vert, uint32_t* __restrict__ tri,
                                                          int8_t* __restrict__ table) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= (int64_t)rows * cols) return;
  const int i = (int)(v / cols), j = (int)(v % cols);
  int dx = 0, dy = 0;
  if (thr >= 0.0) tm_move(hf, rows, cols, thr, i, j, &dx, &dy);
  if (vert) {
    // np.linspace(0, (n - 1) hs, n): i * step in double, the last point exactly the stop value;
    // then + move * hs in double (two roundings, as numpy) and the float32 cast
    const double gx = i == rows - 1 ? __dmul_rn((double)(rows - 1), hs) : __dmul_rn((double)i, xstep);
    const double gy = j == cols - 1 ? __dmul_rn((double)(cols - 1), hs) : __dmul_rn((double)j, ystep);
    vert[3 * v + 0] = (float)__dadd_rn(gx, __dmul_rn((double)dx, hs));
    vert[3 * v + 1] = (float)__dadd_rn(gy, __dmul_rn((double)dy, hs));
    vert[3 * v + 2] = (float)__dmul_rn((double)hf[v], vs);
  }
  if (tri && i + 1 < rows && j + 1 < cols) {
    const uint32_t i0 = (uint32_t)v, i1 = i0 + 1, i2 = i0 + (uint32_t)cols, i3 = i2 + 1;
    const int64_t t = 2 * ((int64_t)i * (cols - 1) + j);
    uint32_t* o = tri + 3 * t;
    o[0] = i0; o[1] = i3; o[2] = i1;
    o[3] = i0; o[4] = i2; o[5] = i3;
  }
  if (table) {
    int flag = 0;
    if (thr >= 0.0)
      for (int a = max(i - 1, 0); a <= min(i + 2, rows - 1) && !flag; ++a)
        for (int b = max(j - 1, 0); b <= min(j + 2, cols - 1); ++b) {
          int mx, my;
          tm_move(hf, rows, cols, thr, a, b, &mx, &my);
          if (mx | my) { flag = 1; break; }
        }
    table[v] = (int8_t)(((dx + 1) * 3 + (dy + 1)) | (flag << 4));
  }
}

}  // namespace

extern "C" int lgx_trimesh_build(const int16_t* hf, int32_t rows, int32_t cols, double hs, double vs, double height_threshold,
                                 float* vertices, uint32_t* triangles, int8_t* table, void* stream) {
  if (!hf || rows < 2 || cols < 2 || !(hs > 0.0) || !(vs > 0.0) || (int64_t)rows * cols >= (1ll << 31) / 3)
    return lgx_fail(LGX_EINVAL, "lgx_trimesh_build: bad arguments");
  // np.linspace's step: delta / div in double
  const double xstep = __dmul_rn_host((double)(rows - 1), hs) / (double)(rows - 1);
  const double ystep = __dmul_rn_host((double)(cols - 1), hs) / (double)(cols - 1);
  const int64_t n = (int64_t)rows * cols;
  hipLaunchKernelGGL(lgx_trimesh_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, hf, rows,
                     cols, hs, vs, height_threshold, xstep, ystep, vertices, triangles, table);
  return lgx_hip_status("lgx_trimesh_build");
}
