// Pipelined split-bf16 GEMM of the PPO update (lgx_gemm_nt with a pre-split B operand):
//   C[z][m][n] = epi( sum_k A[z][m][k] * B[z][n][k] ),  K % 32 == 0, N % 128 == 0.
//
// Same arithmetic as gemm_nt_x3_kernel (lgx_gemm_split.hip: three RNE bf16 limbs per f32
// operand, the six limb products of order <= 2 on v_mfma_f32_32x32x16_bf16, f32 accumulation),
// restructured around the load pipeline, which is what bounded that kernel: with one K stage of
// register-staged prefetch and a barrier pair per 32-k stage, its loads were exposed once per
// stage (measured: the kernel without its MFMAs took as long as the MFMA floor).
//
//   * 256 x 128 output tile per workgroup; one workgroup per CU (149 KB of LDS), persistent over
//     XCD-contiguous tile ranges (consecutive tiles share A rows: L2 reuse on one XCD).  Wave
//     layouts (template NWV): 4 waves = one per SIMD, 64 x 128 each (2 x 4 transposed 32x32
//     accumulators) - no second wave competes for the SIMD's issue, so the barrier that closes
//     every 32-k slot does not wait on a starved wave; 8 waves = two per SIMD, 32 x 128 each
//     (X3P_WGN; measured with s_memtime stamps: the younger wave of each SIMD loses issue
//     arbitration and the older one idles ~35 % of every slot at the barrier);
//   * every global -> LDS copy is an LDS-DMA load (global_load_lds_dwordx4): no staging
//     registers, no LDS write pass.  A (f32 activations) goes through a 3-deep ring of 32 KB
//     stages, its 16-byte chunks placed at chunk ^ ((row >> 1) & 7) by the per-lane SOURCE
//     address (the DMA writes lane-linear); B (pre-split weights, L2-resident) through a 2-deep
//     ring of 24 KB stages copied verbatim - lgx_split_bf16 / the Adam limb mirrors already write
//     the LDS image (x3_limb_off).  The A load of slot q+2 and the B load of slot q+1 are issued
//     while slot q computes, across tile boundaries; one raw s_barrier per 32-k slot, counted
//     vmcnt (the A stage still in flight stays in flight across the barrier); the DMA is
//     inline asm, invisible to the compiler's own waits (which would otherwise drain it);
//   * A is split into its limbs after the fragment read (8 floats per lane per 16 k: 12
//     v_cvt_pk_bf16_f32 + exact f32 subtractions);
//   * epilogues: bias + ELU / plain deferred into the next tile's slots (16-byte row stores of the
//     transposed accumulators, a few per slot, under the MFMAs); ELU' + bias-gradient column sums
//     (the backward dA) at each tile's end from non-transposed accumulators (lane = column: the
//     column sums stay in registers), Y read there (dA2 101-103 -> 89-93 us vs the
//     register-staged gemm_nt_x3_kernel).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "lgx_gemm_common.h"
#include "lgx_internal.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float fx2 __attribute__((ext_vector_type(2)));
typedef float f32x16v __attribute__((ext_vector_type(16)));

constexpr int PN = 128, PK = 32;
constexpr int LGX_X3P_MAX_LDS = 160 * 1024;   // LDS per CU (one workgroup per CU)
constexpr int B_ST = 3 * PN * PK * 2;        // 24 KB: limb B stage ([limb][128 n][64 B])
constexpr int NSA = 3, NSB = 2;              // ring depths
constexpr int B_BLK = 3 * 128 * 32;             // bf16 per pre-split (128 n x 32 k) block

// X3P_WGN: waves along N of the 8-wave 256-row tile.  1 (default): 8 x 1 waves of 32 x 128, each
// wave splits only its own 32 A rows (the 4 x 2 layout of 64 x 64 waves split every A row in
// two waves) for twice the B fragment reads (LDS has the slack): layer-1 forward 81.8 -> 75-77 us
#ifndef X3P_WGN
#define X3P_WGN 1
#endif
#ifndef X3P_BOLD
#define X3P_BOLD 1
#endif
// Tile of PM = 256 rows (the default) or 128 rows (half tiles: the layer whose 256-row tile count
// leaves a fractional last round on the CUs, e.g. 384 tiles on 256 CUs -> 768 half tiles = 3 rounds)
template <int NWV, int PM>
struct XC {
  static constexpr int A_ST = PM * PK * 4;               // f32 A stage (PM rows x 128 B): 32 | 16 KB
  static constexpr int OFF_B = NSA * A_ST;
  static constexpr int OFF_BIAS = OFF_B + NSB * B_ST;    // 3 x 1 KB: bias of the pending / current / next tile
  static constexpr int P_LDS = OFF_BIAS + 4 * 1024;      // 151,552 | 102,400 B (DELU: 4 KB column-sum scratch)
  // LGX_GEMM_DELU with the deferred epilogue: in place of the bias / scratch area, one 16-byte Y run
  // per lane and per deferred store run of a slot (gps), wave-private (wave w's runs at w * gps KB)
  static constexpr int y_lds(int gps) { return OFF_BIAS + NWV * gps * 1024; }
  static constexpr int WGN = NWV == 8 && (PM == 128 || X3P_WGN == 2) ? 2 : 1;   // waves along N
  static constexpr int WGM = NWV / WGN;                  // waves along M (4 | 8)
  static constexpr int WI = PM / WGM / 32;               // 32-row accumulator tiles per wave (2 | 1)
  static constexpr int WJ = PN / WGN / 32;               // 32-column accumulator tiles per wave (2 | 4)
  static constexpr int PT = 64 * NWV;
  static constexpr int A_GL = A_ST / (PT * 16);          // LDS-DMA loads per thread per A stage (4 | 8; 2)
  static constexpr int B_GL = B_ST / (PT * 16);          // per B stage (3 | 6)
  static constexpr int GROUPS = WI * WJ * 4;             // float4 output runs per lane (16 | 32; 8)
  static constexpr int NB = 2 * WI * WJ;                 // MFMA blocks per slot (two 16-k halves)
  static constexpr int ITEMS = B_GL + 1 + A_GL;          // side items per slot: B loads, bias, A loads
  static constexpr int IPB = (ITEMS + NB - 1) / NB;      // side items per MFMA block
  // BOLD: the older half of the waves (0 .. NWV/2-1, which win issue arbitration and then idle at
  // the slot barrier) issues the whole B stage, 2 B_GL loads each; the younger half only its A rows.
  // Half tiles only (isolated, 3 alternated runs: 512 -> 256 forward 90.1 -> 87.2 us; the 256-row
  // tiles' K = 256 forwards 71.8 -> 72.8 and 32.4 -> 34.3 us: a longer pipeline prologue per tile)
  static constexpr bool BOLD = X3P_BOLD && PM == 128;
  static constexpr int ITEMS_O = 2 * B_GL + 1 + A_GL, IPB_O = (ITEMS_O + NB - 1) / NB;
  static constexpr int IPB_Y = (A_GL + NB - 1) / NB;
  // B-stage byte offset of wave w's loads
  static __device__ __forceinline__ int bw_off(int w) {
    return BOLD ? (w < NWV / 2 ? w * (2 * B_GL * 1024) : 0) : w * (B_GL * 1024);
  }
  static_assert((WGM == 4 || WGM == 8) && (WI == 1 || WI == 2), "wave rows of 32 WI rows");
};

struct PArgs {
  int64_t M;
  int32_t N, K, batch, kb;   // kb = K / 32
  const float* A;
  int64_t lda, sa;
  const uint16_t* Bs;
  int64_t sbs;               // batch stride of Bs (bf16 elements)
  float* C;
  int64_t ldc, sc;
  const float* bias;
  const float* Y;
  float* partials;
  int32_t tiles, ntn;
};

struct PTile {
  int32_t mt, nt, z;
};

__device__ __forceinline__ PTile ptile(const PArgs& g, int32_t t) {
  PTile T;
  T.nt = t % g.ntn;
  const int32_t r = t / g.ntn;
  T.z = r % g.batch;
  T.mt = r / g.batch;
  return T;
}

// vmcnt-only waits (expcnt / lgkmcnt left alone)
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void p_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void split2(float x0, float x1, uint32_t& l0, uint32_t& l1, uint32_t& l2) {
  lgx_split2(x0, x1, l0, l1, l2);   // (lgx_internal.h)
}

__device__ __forceinline__ void split8(const float4& x, const float4& y, bf16x8 (&o)[3]) {
  uint4 u0, u1, u2;
  split2(x.x, x.y, u0.x, u1.x, u2.x);
  split2(x.z, x.w, u0.y, u1.y, u2.y);
  split2(y.x, y.y, u0.z, u1.z, u2.z);
  split2(y.z, y.w, u0.w, u1.w, u2.w);
  o[0] = __builtin_bit_cast(bf16x8, u0);
  o[1] = __builtin_bit_cast(bf16x8, u1);
  o[2] = __builtin_bit_cast(bf16x8, u2);
}

// One LDS-DMA load (global_load_lds_dwordx4): 16 bytes per lane from base + voff to LDS address
// lds + 16 * lane.  Inline asm, so the compiler neither orders nor waits on it (its own waits
// would drain the ring: it treats every later LDS-DMA / LDS read as aliasing a pending one);
// the kernel counts vmcnt itself.  M0 is saved and restored around it.
__device__ __forceinline__ void glds16(const char* base, uint32_t voff, uint32_t lds) {
  uint32_t sv;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %2, %3\n\ts_mov_b32 m0, %0"
               : "=&s"(sv)
               : "s"(lds), "v"(voff), "s"(base)
               : "memory");
}

__device__ __forceinline__ const char* uniform_ptr(const void* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const char*>(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)(p));
}

// Per-lane A source offsets (bytes from the batch entry's base) of one tile's DMA loads: LDS
// block b = A_GL * wave + i (1 KB) holds tile rows 8b .. 8b + 7; lane l writes row 8b + l / 8 at
// chunk l % 8, which holds k-chunk (l % 8) ^ ((row >> 1) & 7).
template <int NWV, int PM>
struct AOffs {
  uint32_t o[XC<NWV, PM>::A_GL];
};

template <int NWV, int PM>
__device__ __forceinline__ void a_offs(AOffs<NWV, PM>& a, const PArgs& g, int32_t mt, int tid) {
  constexpr int AG = XC<NWV, PM>::A_GL;
  const int w = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int i = 0; i < AG; ++i) {
    const int r = 8 * (AG * w + i) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int64_t m = min((int64_t)mt * PM + r, g.M - 1);   // rows past M load row M-1 (never stored)
    a.o[i] = (uint32_t)((m * g.lda + 4 * c) * 4);
  }
}

// A / B stage issue split into its single loads: prepare once (uniform addresses), then load(i)
struct DmaPlan {
  const char* src;
  uint32_t dst;
};

template <int NWV, int PM>
__device__ __forceinline__ DmaPlan plan_a(uint32_t lds0, int buf, const PArgs& g, int z, int ks, int tid) {
  using X = XC<NWV, PM>;
  return DmaPlan{uniform_ptr(reinterpret_cast<const char*>(g.A + z * g.sa) + ks * (PK * 4)),
                 (uint32_t)__builtin_amdgcn_readfirstlane(lds0 + buf * X::A_ST + (tid >> 6) * (X::A_GL * 1024))};
}

template <int NWV, int PM>
__device__ __forceinline__ DmaPlan plan_b(uint32_t lds0, int buf, const PArgs& g, const PTile& T, int ks, int tid) {
  using X = XC<NWV, PM>;
  constexpr int BG = X::B_GL;
  (void)BG;
  return DmaPlan{uniform_ptr(reinterpret_cast<const char*>(g.Bs + T.z * g.sbs + (int64_t)(T.nt * g.kb + ks) * B_BLK) +
                             X::bw_off(tid >> 6)),
                 (uint32_t)__builtin_amdgcn_readfirstlane(lds0 + X::OFF_B + buf * B_ST + X::bw_off(tid >> 6))};
}

template <int NWV, int PM>
__device__ __forceinline__ void issue_a(uint32_t lds0, int buf, const PArgs& g, const AOffs<NWV, PM>& a, int z,
                                        int ks, int tid) {
  using X = XC<NWV, PM>;
  constexpr int AG = X::A_GL;
  const char* src = uniform_ptr(reinterpret_cast<const char*>(g.A + z * g.sa) + ks * (PK * 4));
  const uint32_t dst = __builtin_amdgcn_readfirstlane(lds0 + buf * X::A_ST + (tid >> 6) * (AG * 1024));
#pragma unroll
  for (int i = 0; i < AG; ++i) glds16(src, a.o[i], dst + i * 1024);
}

// B stage of slot (T, ks); with `bias` (BIAS_ELU, a tile's first stage, wave 0 only) also the
// tile's 128 bias values into bias buffer `bbuf` (lanes 32-63 duplicate lanes 0-31).  The extra
// load is issued with the B stage, so every vmcnt count of the pipeline stays the same.
template <int NWV, int PM>
__device__ __forceinline__ void issue_b(uint32_t lds0, int buf, const PArgs& g, const PTile& T, int ks, int tid,
                                        bool bias, int bbuf) {
  using X = XC<NWV, PM>;
  constexpr int BG = X::B_GL;
  const int w = tid >> 6, lane = tid & 63;
  const char* src = uniform_ptr(g.Bs + T.z * g.sbs + (int64_t)(T.nt * g.kb + ks) * B_BLK);
  const uint32_t dst = __builtin_amdgcn_readfirstlane(lds0 + X::OFF_B + buf * B_ST + X::bw_off(w));
  if (!X::BOLD || __builtin_amdgcn_readfirstlane(w) < NWV / 2) {
#pragma unroll
    for (int i = 0; i < (X::BOLD ? 2 * BG : BG); ++i)
      glds16(src, (uint32_t)(X::bw_off(w) + i * 1024 + lane * 16), dst + i * 1024);
  }
  if (bias)
    glds16(uniform_ptr(g.bias + (int64_t)T.z * g.N + T.nt * PN), (uint32_t)((lane & 31) * 16),
           __builtin_amdgcn_readfirstlane(lds0 + X::OFF_BIAS + bbuf * 1024));
}

// One 32-k slot of a wave's WI x WJ accumulators: per 16-k half, its A row tiles are read (f32)
// and split into limbs, its B column tiles read (limbs), 6 MFMAs per accumulator (small limb
// products first).  Conflict-free reads: A chunk c of row R at c ^ ((R >> 1) & 7); B chunk c of
// column n at c ^ ((n >> 2) & 3).
//
// side(b) runs after accumulator block b (b = 0 .. 2 WI WJ - 1 in issue order): the slot's DMA
// issues and deferred stores are spread between the MFMA blocks, where a DMA issue that waits for
// the texture unit to accept it costs no MFMA time (issued in one burst before the compute, the 14
// DMA loads of a 4-wave slot took ~950 cycles of the wave's ~5600).
template <int NWV, int PM, bool TRANS, typename Side>
__device__ __forceinline__ void compute_slot(const char* __restrict__ la, const char* __restrict__ lb, int wm, int wn,
                                             int r, int h, f32x16v (&acc)[XC<NWV, PM>::WI][XC<NWV, PM>::WJ],
                                             Side&& side) {
  constexpr int WI = XC<NWV, PM>::WI, WJ = XC<NWV, PM>::WJ;
  const int sa = (r >> 1) & 7, sb = (r >> 2) & 3;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int ca = 4 * s + 2 * h, cb = 2 * s + h;
    bf16x8 a[WI][3], b[WJ][3];
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const char* row = la + (wm * 32 * WI + 32 * i + r) * (PK * 4);
      const float4 x = *reinterpret_cast<const float4*>(row + 16 * (ca ^ sa));
      const float4 y = *reinterpret_cast<const float4*>(row + 16 * ((ca + 1) ^ sa));
#ifndef X3P_NO_SPLIT
      split8(x, y, a[i]);
#else   // A/B: raw bits as limbs (wrong results; measures the split's VALU cost)
      a[i][0] = __builtin_bit_cast(bf16x8, x);
      a[i][1] = __builtin_bit_cast(bf16x8, y);
      a[i][2] = __builtin_bit_cast(bf16x8, x);
#endif
    }
#pragma unroll
    for (int j = 0; j < WJ; ++j)
#pragma unroll
      for (int l = 0; l < 3; ++l)
        b[j][l] =
            *reinterpret_cast<const bf16x8*>(lb + l * (PN * 64) + (wn * 32 * WJ + 32 * j + r) * 64 + 16 * (cb ^ sb));
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int j = 0; j < WJ; ++j) {
#ifdef X3P_NO_MFMA   // A/B: keep the fragment reads / split alive, no MFMA
        acc[i][j][0] += (float)a[i][0][0] + (float)a[i][1][1] + (float)a[i][2][2] + (float)b[j][0][0] +
                        (float)b[j][1][3] + (float)b[j][2][5];
        continue;
#endif
        f32x16v c = acc[i][j];
        if constexpr (TRANS) {   // weights first: lane = output row, 4 runs of 4 columns
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][2], a[i][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][1], a[i][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][0], a[i][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][1], a[i][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][0], a[i][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][0], a[i][0], c, 0, 0, 0);
        } else {                 // rows first: lane = output column (column sums in registers)
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][0], c, 0, 0, 0);
        }
        acc[i][j] = c;
        side((s * WI + i) * WJ + j);
      }
  }
}

__device__ __forceinline__ float4 q4(const f32x16v& v, int q) {
  return make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

// Bias + ELU (or plain) output of float4 run gi = (i, j, q), gi = 4 (WJ i + j) + q, of a lane.
template <int EPI, int NWV, int PM>
__device__ __forceinline__ void p_store_group(const PArgs& g, const f32x16v (&pend)[XC<NWV, PM>::WI][XC<NWV, PM>::WJ],
                                              const PTile& T, int wm, int wn, int r, int h, const float* bias_lds,
                                              int gi) {
  constexpr int WI = XC<NWV, PM>::WI, WJ = XC<NWV, PM>::WJ;
  const int q = gi & 3, j = (gi >> 2) % WJ, i = (gi >> 2) / WJ;
  const int64_t row = (int64_t)T.mt * PM + wm * 32 * WI + 32 * i + r;
  const int cn = wn * 32 * WJ + 32 * j + 8 * q + 4 * h;
  float4 v = q4(pend[i][j], q);
  if (EPI == LGX_GEMM_BIAS_ELU) {
    const float4 bq = *reinterpret_cast<const float4*>(bias_lds + cn);
    v.x = elu_f(v.x + bq.x);
    v.y = elu_f(v.y + bq.y);
    v.z = elu_f(v.z + bq.z);
    v.w = elu_f(v.w + bq.w);
    // keep the bias read and the ELU ahead of the row test: sunk into the branch, the read waited
    // on its own LDS round trip inside it
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
  }
  // (LGX_GEMM_DELU: the run was multiplied by ELU'(Y) in place before - delu_apply)
  if (row < g.M) *reinterpret_cast<float4*>(g.C + T.z * g.sc + row * g.ldc + T.nt * PN + cn) = v;
}

// LGX_GEMM_DELU on transposed accumulators (lane = row, runs of 4 columns, as p_store_group): the
// Y run of output run gi (16-byte load from a clamped row: unconditional), and the run multiplied
// by ELU'(Y) in place
template <int NWV, int PM>
__device__ __forceinline__ const float* delu_addr(const PArgs& g, const PTile& T, int wm, int wn, int r, int h, int gi) {
  constexpr int WI = XC<NWV, PM>::WI, WJ = XC<NWV, PM>::WJ;
  const int q = gi & 3, j = (gi >> 2) % WJ, i = (gi >> 2) / WJ;
  const int64_t row = min((int64_t)T.mt * PM + wm * 32 * WI + 32 * i + r, g.M - 1);
  const int cn = wn * 32 * WJ + 32 * j + 8 * q + 4 * h;
  return g.Y + T.z * g.sc + row * g.ldc + T.nt * PN + cn;
}

template <int NWV, int PM>
__device__ __forceinline__ float4 delu_load(const PArgs& g, const PTile& T, int wm, int wn, int r, int h, int gi) {
  return *reinterpret_cast<const float4*>(delu_addr<NWV, PM>(g, T, wm, wn, r, h, gi));
}



template <int NWV, int PM>
__device__ __forceinline__ void delu_apply(int gi, const float4& y, f32x16v (&pend)[XC<NWV, PM>::WI][XC<NWV, PM>::WJ]) {
  constexpr int WJ = XC<NWV, PM>::WJ;
  const int q = gi & 3, j = (gi >> 2) % WJ, i = (gi >> 2) / WJ;
  pend[i][j][4 * q] *= elu_grad_from_out(y.x);
  pend[i][j][4 * q + 1] *= elu_grad_from_out(y.y);
  pend[i][j][4 * q + 2] *= elu_grad_from_out(y.z);
  pend[i][j][4 * q + 3] *= elu_grad_from_out(y.w);
}

// every run of a tile at once (the last tile, or the runtime-K kernels): all Y loads in flight,
// then multiply and store
template <int NWV, int PM>
__device__ __forceinline__ void delu_tile(const PArgs& g, f32x16v (&acc)[XC<NWV, PM>::WI][XC<NWV, PM>::WJ],
                                          const PTile& T, int wm, int wn, int r, int h) {
  constexpr int GROUPS = XC<NWV, PM>::GROUPS;
  float4 y[GROUPS];
#pragma unroll
  for (int gi = 0; gi < GROUPS; ++gi) y[gi] = delu_load<NWV, PM>(g, T, wm, wn, r, h, gi);
#pragma unroll
  for (int gi = 0; gi < GROUPS; ++gi) {
    delu_apply<NWV, PM>(gi, y[gi], acc);
    p_store_group<LGX_GEMM_DELU, NWV, PM>(g, acc, T, wm, wn, r, h, nullptr, gi);
  }
}

// ELU' + bias-gradient column sums at a tile's end (non-transposed accumulators: lane = column
// 32 j + r of the wave's 32 WI rows, acc[i][j][e] = row 32 i + 8 (e >> 2) + 4 h + (e & 3)):
// D = acc * elu'(Y) with 128-byte row segments per load / store, column sums in registers, then
// across the lane halves and, in a fixed order, across the waves of each 128-row partial block
// (partials[m / 128][z][n], the layout of gemm_nt_x3_kernel's).  scratch: [NWV][128] floats.
template <int NWV, int PM>
__device__ __forceinline__ void delu_epilogue(const PArgs& g, const f32x16v (&acc)[XC<NWV, PM>::WI][XC<NWV, PM>::WJ],
                                              const PTile& T, int wave, int wm, int wn, int r, int h,
                                              float* scratch) {
  using X = XC<NWV, PM>;
  constexpr int WI = X::WI, WJ = X::WJ;
  const int64_t m0 = (int64_t)T.mt * PM + wm * 32 * WI;
  const int cl = wn * 32 * WJ;                         // the wave's first column in the tile
  const int64_t n0 = (int64_t)T.nt * PN + cl;
  const float* Y = g.Y + T.z * g.sc;
  float* C = g.C + T.z * g.sc;
  float cs[WJ];
#pragma unroll
  for (int j = 0; j < WJ; ++j) cs[j] = 0.f;
#pragma unroll
  for (int i = 0; i < WI; ++i)
#pragma unroll
    for (int e0 = 0; e0 < 16; e0 += 4) {   // 4 WJ loads of Y in flight, then the stores
      float y[4][WJ];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
          const int64_t row = min(m0 + 32 * i + 8 * ((e0 + e) >> 2) + 4 * h + ((e0 + e) & 3), g.M - 1);
          y[e][j] = Y[row * g.ldc + n0 + 32 * j + r];
        }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
          const int64_t row = m0 + 32 * i + 8 * ((e0 + e) >> 2) + 4 * h + ((e0 + e) & 3);
          const float d = acc[i][j][e0 + e] * elu_grad_from_out(y[e][j]);
          if (row < g.M) {
            C[row * g.ldc + n0 + 32 * j + r] = d;
            cs[j] += d;
          }
        }
    }
#pragma unroll
  for (int j = 0; j < WJ; ++j) cs[j] += __shfl_xor(cs[j], 32);
  if (h == 0) {
#pragma unroll
    for (int j = 0; j < WJ; ++j) scratch[wave * 128 + cl + 32 * j + r] = cs[j];
  }
  __syncthreads();
  // wave w of the first X::WGN * (128 / (32 WI)) waves... : one 128-row block = 128 / (32 WI)
  // wave rows; the waves of wave row 0 of each block write its partial row
  constexpr int BLOCK_WM = 128 / (32 * WI);            // wave rows per 128-row partial block
  if (wm % BLOCK_WM == 0 && h == 0) {
    const int64_t mb = ((int64_t)T.mt * PM + wm * 32 * WI) / 128;
    if (mb * 128 < g.M) {
      float* P = g.partials + mb * ((int64_t)g.batch * g.N) + (int64_t)T.z * g.N;
#pragma unroll
      for (int j = 0; j < WJ; ++j) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < BLOCK_WM; ++w) v += scratch[((wm + w) * X::WGN + wn) * 128 + cl + 32 * j + r];   // fixed order
        P[n0 + 32 * j + r] = v;
      }
    }
  }
}

#ifdef X3P_CLOCK   // A/B instrumentation: per-slot s_memtime stamps of workgroup 0 into g.partials
#define X3P_STAMP(e) \
  if (clk && q < 32) clk[(wave * 32 + q) * 8 + (e)] = __builtin_amdgcn_s_memtime()
#else
#define X3P_STAMP(e)
#endif

// Slot q = (the workgroup's j-th tile, K stage k), q = j * kb + k.  Iteration q: wait for slot q's
// A and B stages (the A stage of slot q+1, issued after them, and the deferred stores issued after
// that, stay in flight: vmcnt is an in-order count), barrier (every wave's DMA for slot q landed;
// every wave is done with slot q-1's buffers), issue B(q+1) and A(q+2) into the buffers slot q-1
// used, write this slot's share of the previous tile's output, compute slot q.
//
// KBT > 0: K = 32 KBT known at compile time, the k loop unrolled and the BIAS_ELU / PLAIN
// epilogue deferred into the next tile's slots (GROUPS / KBT store runs per slot: constant
// register indices).  KBT == 0: the epilogue runs at the tile's end (after waiting for the next
// slot's stages, so its stores do not sit in front of them).  (ELU' + column sums: the
// register-staged gemm_nt_x3_kernel, measured equal or faster for the dA shapes.)
template <int EPI, int KBT, int NWV, int PM>
__global__ void __launch_bounds__(64 * NWV, 1) gemm_nt_x3p_kernel(PArgs g) {
  using X = XC<NWV, PM>;
  constexpr int WI = X::WI, WJ = X::WJ, AG = X::A_GL;
  constexpr int A_ST = X::A_ST, OFF_B = X::OFF_B, OFF_BIAS = X::OFF_BIAS;
  extern __shared__ __attribute__((aligned(16))) char plds[];
  constexpr bool DELU = EPI == LGX_GEMM_DELU_COLSUM;
  // LGX_GEMM_DELU: transposed accumulators like the forward, the output deferred into the next
  // tile's slots; the Y runs of a slot's stores are loaded one slot ahead (before that slot's
  // B stage, so the pipeline's vmcnt counts are unchanged) and multiplied in after its barrier
  constexpr bool DELU_T = EPI == LGX_GEMM_DELU;
  // deferred store runs per slot (slots k with k * GPS < GROUPS store GPS runs each)
  constexpr int GPS0 = KBT > 0 ? (X::GROUPS >= KBT ? X::GROUPS / KBT : 1) : 0;
  // (DELU: deferred only where the Y runs of a slot fit the LDS beside the rings)
  constexpr bool DEFER = KBT > 0 && !DELU && !(DELU_T && X::y_lds(GPS0) > LGX_X3P_MAX_LDS);
  constexpr int GPS = DEFER ? GPS0 : 0;
  static_assert(!DEFER || X::GROUPS % GPS == 0, "every storing slot issues exactly GPS runs (vmcnt counts)");
  constexpr int UNR = KBT > 0 ? KBT : 1;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave / X::WGN, wn = wave % X::WGN;
  const int xcd = blockIdx.x & 7;
  const int32_t stride = gridDim.x >> 3;   // grid is a multiple of 8
  const int32_t lo = (int32_t)((int64_t)xcd * g.tiles / 8), hi = (int32_t)((int64_t)(xcd + 1) * g.tiles / 8);
  const int32_t t0 = lo + (blockIdx.x >> 3);
  if (t0 >= hi) return;
  const int32_t ntiles = (hi - t0 + stride - 1) / stride;
  const int kb = KBT > 0 ? KBT : g.kb;
  const int32_t nslots = ntiles * kb;
  const uint32_t lds0 = lds_addr(plds);
#ifdef X3P_CLOCK
  uint64_t* clk = (blockIdx.x == 0 && lane == 0) ? reinterpret_cast<uint64_t*>(g.partials) : nullptr;
#endif

  // A issue iterator (runs 2 slots ahead), B issue iterator (1 slot ahead)
  int32_t ja = 0, jb = 0;
  PTile Ta = ptile(g, t0), Tb = Ta;
  int ka = 0, kbb = 0;
  AOffs<NWV, PM> ao;
  a_offs<NWV, PM>(ao, g, Ta.mt, tid);
  auto next_a = [&]() {
    if (++ka == kb) {
      ka = 0;
      Ta = ptile(g, t0 + (++ja) * stride);
      a_offs<NWV, PM>(ao, g, Ta.mt, tid);
    }
  };
  auto next_b = [&]() {
    if (++kbb == kb) {
      kbb = 0;
      Tb = ptile(g, t0 + (++jb) * stride);
    }
  };
  // prologue: A(0), B(0), A(1)
  constexpr bool BIAS = EPI == LGX_GEMM_BIAS_ELU;
  const bool w0 = __builtin_amdgcn_readfirstlane(wave) == 0;
  issue_a<NWV, PM>(lds0, 0, g, ao, Ta.z, ka, tid);
  next_a();
  issue_b<NWV, PM>(lds0, 0, g, Tb, kbb, tid, BIAS && w0, 0);
  next_b();
  if (nslots > 1) {
    issue_a<NWV, PM>(lds0, 1, g, ao, Ta.z, ka, tid);
    next_a();
  }

  f32x16v acc[WI][WJ], pend[WI][WJ];
#pragma unroll
  for (int i = 0; i < WI; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = pend[i][j][e] = 0.f;
  PTile Tp{0, 0, 0};           // tile whose output is pending (DEFER)
  bool pending = false, pend_full = false;
  int32_t q = 0;
  bool waited = false;         // (!DEFER) the epilogue already waited for the next slot's stages
  bool stores = false;         // (DEFER) GPS deferred stores issued in the previous iteration
  // KBT > 0: every unrolled slot's issue targets are compile-time (stage (k + 2) % KBT / (k + 1) %
  // KBT of this tile or the next), so the next tile's coordinates and A row offsets are computed
  // once per tile instead of the iterators' per-slot wrap tests (measured: ~230 scalar / VALU
  // instructions between the barrier and the first MFMA of every slot)
  static_assert(KBT == 0 || (KBT >= 2 && KBT % 2 == 0), "A runs two slots ahead: at most one tile boundary; "
                "an even K step count keeps the B ring index compile-time");
  AOffs<NWV, PM> aon = ao;
  PTile T = ptile(g, t0);
  // (KBT > 0) the DMA plans of a slot from per-tile uniform bases and running ring offsets: the
  // per-slot plan arithmetic (64-bit address products, ring indices modulo 3, readfirstlanes) took
  // 300-500 cycles between the barrier and the first MFMA of every slot (X3P_CLOCK)
  constexpr int BG0 = X::B_GL;
  const uint32_t lds_aw = (uint32_t)__builtin_amdgcn_readfirstlane(lds0 + (tid >> 6) * (AG * 1024));
  const uint32_t lds_bw = (uint32_t)__builtin_amdgcn_readfirstlane(lds0 + OFF_B + X::bw_off(tid >> 6));
  const bool older = __builtin_amdgcn_readfirstlane(tid >> 6) < NWV / 2;
  (void)BG0;
  uint32_t off_ac = 0, off_ai = 2 * A_ST;   // A ring byte offsets of slot q (compute) and q + 2 (issue)
  const char* a_nxt = uniform_ptr(reinterpret_cast<const char*>(g.A + T.z * g.sa));
  const char* b_nxt = uniform_ptr(reinterpret_cast<const char*>(g.Bs + T.z * g.sbs + (int64_t)(T.nt * g.kb) * B_BLK) +
                                  X::bw_off(tid >> 6));
  for (int32_t tj = 0; tj < ntiles; ++tj) {
    if (KBT == 0) T = ptile(g, t0 + tj * stride);
    PTile Tn = T;
    const char* a_cur = a_nxt;
    const char* b_cur = b_nxt;
    const bool last_tile = tj + 1 == ntiles;
    if constexpr (KBT > 0) {
      Tn = ptile(g, t0 + (tj + 1) * stride);   // (past the last tile: bases computed, never loaded)
      if (!last_tile) a_offs<NWV, PM>(aon, g, Tn.mt, tid);
      a_nxt = uniform_ptr(reinterpret_cast<const char*>(g.A + Tn.z * g.sa));
      b_nxt = uniform_ptr(reinterpret_cast<const char*>(g.Bs + Tn.z * g.sbs + (int64_t)(Tn.nt * g.kb) * B_BLK) +
                          X::bw_off(tid >> 6));
    }
#pragma unroll UNR
    for (int k = 0; k < kb; ++k, ++q) {
      X3P_STAMP(0);
      // slots q + 1 / q + 2 exist (KBT > 0: compile-time except in the last tile's last slots)
      const bool more1 = KBT > 0 ? !(last_tile && k + 1 >= KBT) : q + 1 < nslots;
      const bool more2 = KBT > 0 ? !(last_tile && k + 2 >= KBT) : q + 2 < nslots;
      if (!waited) {
        // slot q's stages; A(q+1) (AG loads) and last iteration's stores may stay in flight
        if (more1) {
          if (DEFER && stores) wait_vm<AG + GPS>();
          else wait_vm<AG>();
        } else {
          if (DEFER && stores) wait_vm<GPS>();
          else wait_vm<0>();
        }
      }
      waited = false;
      X3P_STAMP(1);
      p_barrier();
      X3P_STAMP(2);
      // slot q+1's B stage and slot q+2's A stage (same order as always: B, bias, A), and this
      // slot's share of the pending output, spread over the MFMA blocks of compute(q)
      const bool a_next = KBT > 0 && k + 2 >= KBT, b_next = KBT > 0 && k + 1 >= KBT;
      const bool do_b = more1, do_a = more2;
      const bool do_bias = BIAS && w0 && (KBT > 0 ? b_next : kbb == 0) && do_b;
      const int bbuf = KBT > 0 ? (tj + (b_next ? 1 : 0)) % 3 : jb % 3;
      DmaPlan pb{nullptr, 0}, pa{nullptr, 0};
      const PTile Tbias = KBT > 0 ? (b_next ? Tn : T) : Tb;
      if constexpr (KBT > 0) {   // (KBT even: the B ring index (q + 1) % 2 is (k + 1) % 2)
        pb = DmaPlan{(b_next ? b_nxt : b_cur) + ((k + 1) % KBT) * (B_BLK * 2), lds_bw + ((k + 1) % NSB) * B_ST};
        pa = DmaPlan{(a_next ? a_nxt : a_cur) + ((k + 2) % KBT) * (PK * 4), lds_aw + off_ai};
      } else {
        if (do_b) pb = plan_b<NWV, PM>(lds0, (q + 1) % NSB, g, Tbias, kbb, tid);
        if (do_a) pa = plan_a<NWV, PM>(lds0, (q + 2) % NSA, g, Ta.z, ka, tid);
      }
      const AOffs<NWV, PM> aoq = KBT > 0 && a_next ? aon : ao;
      if (KBT == 0) {
        if (do_b) next_b();
        if (do_a) next_a();
      }
      X3P_STAMP(3);
      const bool st_now = DEFER && pending && k * GPS < X::GROUPS;
      if constexpr (DELU_T && DEFER) {
        // this slot's runs of the pending tile: Y staged by the previous slot's LDS-DMA into this
        // wave's private runs (the slot-top vmcnt wait covers it: issued before that slot's B stage)
        const char* ylds = plds + X::OFF_BIAS + wave * (GPS * 1024) + lane * 16;
        if (st_now) {
#pragma unroll
          for (int u = 0; u < GPS; ++u)
            if (k * GPS + u < X::GROUPS)
              delu_apply<NWV, PM>(k * GPS + u, *reinterpret_cast<const float4*>(ylds + u * 1024), pend);
        }
        // the next slot's runs (of the pending tile within this tile; of this tile, pending from the
        // next tile on, in its last slot) into the same runs once this slot's reads have completed
        const bool last = k + 1 == KBT;
        const bool ld = last ? tj + 1 < ntiles : (pending && (k + 1) * GPS < X::GROUPS);
        if (ld) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const PTile& Ty = last ? T : Tp;
          const char* yb = uniform_ptr(g.Y + Ty.z * g.sc + ((int64_t)Ty.mt * PM) * g.ldc + Ty.nt * PN);
          const uint32_t ydst = (uint32_t)__builtin_amdgcn_readfirstlane(lds0 + X::OFF_BIAS + wave * (GPS * 1024));
#pragma unroll
          for (int u = 0; u < GPS; ++u) {
            const int gi = (last ? 0 : (k + 1) * GPS) + u;
            if (gi < X::GROUPS) {
              const int q4i = gi & 3, jj = (gi >> 2) % WJ, ii = (gi >> 2) / WJ;
              const int64_t rt = min((int64_t)wm * 32 * WI + 32 * ii + r, g.M - 1 - (int64_t)Ty.mt * PM);
              const int cn = wn * 32 * WJ + 32 * jj + 8 * q4i + 4 * h;
              glds16(yb, (uint32_t)((rt * g.ldc + cn) * 4), ydst + u * 1024);
            }
          }
        }
      }
      stores = DEFER && st_now && pend_full;
      const float* bias_prev = reinterpret_cast<const float*>(plds + OFF_BIAS + ((tj + 2) % 3) * 1024);
      constexpr int BG = X::B_GL;
      auto side = [&](int blk) {
        // side items (IPB per MFMA block, in this order): BG B loads, the bias, AG A loads; then
        // the stores
        if (!X::BOLD || older) {
          constexpr int NBW = X::BOLD ? 2 * BG : BG, IPBW = X::BOLD ? X::IPB_O : X::IPB;
#pragma unroll
          for (int e = 0; e < IPBW; ++e) {
            const int it = blk * IPBW + e;
            if (it < NBW) {
              if (do_b) glds16(pb.src, (uint32_t)(lane * 16 + it * 1024), pb.dst + it * 1024);
            } else if (it == NBW) {
              if (do_bias)
                glds16(uniform_ptr(g.bias + (int64_t)Tbias.z * g.N + Tbias.nt * PN), (uint32_t)((lane & 31) * 16),
                       __builtin_amdgcn_readfirstlane(lds0 + OFF_BIAS + bbuf * 1024));
            } else if (it <= NBW + AG) {
              if (do_a) glds16(pa.src, aoq.o[it - NBW - 1], pa.dst + (it - NBW - 1) * 1024);
            }
          }
        } else {
#pragma unroll
          for (int e = 0; e < X::IPB_Y; ++e) {
            const int it = blk * X::IPB_Y + e;
            if (it < AG && do_a) glds16(pa.src, aoq.o[it], pa.dst + it * 1024);
          }
        }
        if constexpr (DEFER) {
          constexpr int NB = X::NB;
          static_assert(NB >= GPS, "every store run gets a block");
          // the stores after the last GPS blocks (they may interleave with A(q+2)'s loads: the
          // next wait only needs B(q+1), which precedes both)
          const int u = blk - (NB - GPS);
          if (st_now && u >= 0 && u < GPS)
            p_store_group<EPI, NWV, PM>(g, pend, Tp, wm, wn, r, h, bias_prev, k * GPS + u);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      X3P_STAMP(4);
#ifndef X3P_NO_COMPUTE
      compute_slot<NWV, PM, !DELU>(plds + (KBT > 0 ? off_ac : (q % NSA) * A_ST),
                                   plds + OFF_B + (KBT > 0 ? k % NSB : q % NSB) * B_ST, wm, wn, r, h, acc, side);
#else
      for (int blk = 0; blk < X::NB; ++blk) side(blk);
#endif
      X3P_STAMP(5);
      off_ac = off_ac == (NSA - 1) * A_ST ? 0u : off_ac + A_ST;
      off_ai = off_ai == (NSA - 1) * A_ST ? 0u : off_ai + A_ST;
    }
    // ---- tile end
    if constexpr (DEFER) {
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int j = 0; j < WJ; ++j) pend[i][j] = acc[i][j];
      Tp = T;
      pending = true;
      pend_full = (int64_t)T.mt * PM + PM <= g.M;
    } else {
      if (q + 1 < nslots) wait_vm<AG>();   // (q = the next slot) its stages; A(q+1) may stay in flight
      else wait_vm<0>();
      waited = true;
#ifndef X3P_NO_EPI
      if constexpr (DELU) {
        delu_epilogue<NWV, PM>(g, acc, T, wave, wm, wn, r, h, reinterpret_cast<float*>(plds + OFF_BIAS));
      } else if constexpr (DELU_T) {
        delu_tile<NWV, PM>(g, acc, T, wm, wn, r, h);
      } else {
#pragma unroll
        for (int gi = 0; gi < X::GROUPS; ++gi)
          p_store_group<EPI, NWV, PM>(g, acc, T, wm, wn, r, h,
                                      reinterpret_cast<const float*>(plds + OFF_BIAS + (tj % 3) * 1024), gi);
      }
#else
      if (acc[0][0][0] == 1234.5f) g.C[tid] = acc[WI - 1][1][3] + acc[0][1][2] + acc[WI - 1][0][1];
#endif
    }
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int j = 0; j < WJ; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    if constexpr (KBT > 0) {
      ao = aon;
      T = Tn;
    }
  }
  if constexpr (DEFER) {   // the last tile's output (no further slots to spread it over)
#ifndef X3P_NO_EPI
    if constexpr (DELU_T) {
      delu_tile<NWV, PM>(g, pend, Tp, wm, wn, r, h);
    } else {
#pragma unroll
      for (int gi = 0; gi < X::GROUPS; ++gi)
        p_store_group<EPI, NWV, PM>(g, pend, Tp, wm, wn, r, h,
                                    reinterpret_cast<const float*>(plds + OFF_BIAS + ((ntiles - 1) % 3) * 1024), gi);
    }
#else
    if (pend[0][0][0] == 1234.5f) g.C[tid] = pend[WI - 1][1][3] + pend[0][1][2] + pend[WI - 1][0][1];
#endif
  }
}

typedef void (*x3p_fn)(PArgs);

// [epilogue (PLAIN, BIAS_ELU, DELU_COLSUM, DELU)][KBT index: 0 (runtime K), 4, 8, 16]
template <int NWV, int PM>
struct X3PTable {
  static constexpr x3p_fn k[4][4] = {
      {&gemm_nt_x3p_kernel<LGX_GEMM_PLAIN, 0, NWV, PM>, &gemm_nt_x3p_kernel<LGX_GEMM_PLAIN, 4, NWV, PM>,
       &gemm_nt_x3p_kernel<LGX_GEMM_PLAIN, 8, NWV, PM>, &gemm_nt_x3p_kernel<LGX_GEMM_PLAIN, 16, NWV, PM>},
      {&gemm_nt_x3p_kernel<LGX_GEMM_BIAS_ELU, 0, NWV, PM>, &gemm_nt_x3p_kernel<LGX_GEMM_BIAS_ELU, 4, NWV, PM>,
       &gemm_nt_x3p_kernel<LGX_GEMM_BIAS_ELU, 8, NWV, PM>, &gemm_nt_x3p_kernel<LGX_GEMM_BIAS_ELU, 16, NWV, PM>},
      {&gemm_nt_x3p_kernel<LGX_GEMM_DELU_COLSUM, 0, NWV, PM>, &gemm_nt_x3p_kernel<LGX_GEMM_DELU_COLSUM, 4, NWV, PM>,
       &gemm_nt_x3p_kernel<LGX_GEMM_DELU_COLSUM, 8, NWV, PM>, &gemm_nt_x3p_kernel<LGX_GEMM_DELU_COLSUM, 16, NWV, PM>},
      {&gemm_nt_x3p_kernel<LGX_GEMM_DELU, 0, NWV, PM>, &gemm_nt_x3p_kernel<LGX_GEMM_DELU, 4, NWV, PM>,
       &gemm_nt_x3p_kernel<LGX_GEMM_DELU, 8, NWV, PM>, &gemm_nt_x3p_kernel<LGX_GEMM_DELU, 16, NWV, PM>}};
};

template <int NWV, int PM>
bool x3p_attrs() {
  bool ok = true;
  for (const auto& row : X3PTable<NWV, PM>::k)
    for (x3p_fn f : row)
      if (f)
        ok &= hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LGX_X3P_MAX_LDS) == hipSuccess;
  return ok;
}

// Dynamic LDS of an instantiation: the rings + bias / scratch area, or for the deferred
// LGX_GEMM_DELU (where its Y runs fit; the kernel decides alike) the rings + the Y runs
template <int NWV, int PM>
int x3p_lds(int epi, int kbt) {
  using X = XC<NWV, PM>;
  if (epi == LGX_GEMM_DELU && kbt > 0) {
    const int yl = X::y_lds(X::GROUPS >= kbt ? X::GROUPS / kbt : 1);
    if (yl <= LGX_X3P_MAX_LDS) return std::max(X::P_LDS, yl);
  }
  return X::P_LDS;
}

// Tile height: 256 rows, or 128 when that fills the CUs' rounds better: cost = rounds of persistent
// tiles x tile time, a half tile measured 0.55-0.62 of a full one (e.g. the 512 -> 256 layer at
// M = 24576: 384 full tiles = 2 rounds on 256 CUs, 768 half tiles = 3 rounds of 0.6: 100 -> 93 us).
// lgx_gemm_args.tile_rows = 128 / 256 forces one (tests of both heights).
int pick_pm(int64_t M, int ntn, int batch, int cus, int forced) {
  if (forced == 128 || forced == 256) return forced;
  const int64_t t256 = (M + 255) / 256 * ntn * batch, t128 = (M + 127) / 128 * ntn * batch;
  const double c256 = (double)((t256 + cus - 1) / cus), c128 = 0.6 * (double)((t128 + cus - 1) / cus);
  return c128 < c256 ? 128 : 256;
}

}  // namespace

// lgx_gemm_nt with a pre-split B (x3_limb_off layout), K % 32 == 0 (checked by the caller)
int lgx_gemm_nt_x3p(const lgx_gemm_args& a, int cus, void* stream_) {
  const hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  PArgs g;
  g.M = a.M;
  g.N = a.N;
  g.K = a.K;
  g.batch = a.batch;
  g.kb = a.K / PK;
  g.A = a.A;
  g.lda = a.lda;
  g.sa = a.sa;
  g.Bs = a.Bs;
  g.sbs = (int64_t)a.N * g.kb * 96;
  g.C = a.C;
  g.ldc = a.ldc;
  g.sc = a.sc;
  g.bias = a.bias;
  g.Y = a.Y;
  g.partials = a.partials;
  g.ntn = a.N / PN;
  if (((uintptr_t)a.Bs & 15) || a.M * a.lda * 4 >= (1ll << 32))
    return lgx_fail(LGX_EINVAL, "lgx_gemm_nt: pre-split B must be 16-byte aligned; A < 4 GB per batch entry");
  // K = 128 / 256 / 512 (the PPO-update layers): the k loop unrolled, the epilogue deferred into
  // the next tile; other K: the runtime loop with the epilogue at the tile's end.  Eight waves (two
  // per SIMD; four measured 2-8 % slower on the update shapes).
  constexpr int nwv = 8;
  static const bool attrs = x3p_attrs<8, 256>() && x3p_attrs<8, 128>();
  if (!attrs) return lgx_fail(LGX_EHIP, "lgx_gemm_nt: hipFuncSetAttribute (dynamic LDS) failed");
  if (a.tile_rows != 0 && a.tile_rows != 128 && a.tile_rows != 256)
    return lgx_fail(LGX_EINVAL, "lgx_gemm_nt: tile_rows must be 0 (automatic), 128 or 256");
  const int pm = pick_pm(a.M, g.ntn, a.batch, cus, a.tile_rows);
  const int64_t tiles = ((a.M + pm - 1) / pm) * g.ntn * a.batch;
  if (tiles >= (1ll << 31) / 8) return lgx_fail(LGX_EINVAL, "lgx_gemm_nt: too many tiles");
  g.tiles = (int32_t)tiles;
  const int kbt = (g.kb == 4 || g.kb == 8 || g.kb == 16) ? g.kb : 0;
  const int ki = kbt == 0 ? 0 : kbt == 4 ? 1 : kbt == 8 ? 2 : 3;
  const x3p_fn f = pm == 128 ? X3PTable<8, 128>::k[a.epi][ki] : X3PTable<8, 256>::k[a.epi][ki];
  const int lds = pm == 128 ? x3p_lds<8, 128>(a.epi, kbt) : x3p_lds<8, 256>(a.epi, kbt);
  // persistent: one workgroup per CU, a multiple of 8 (XCD tile ranges)
  const int64_t per_xcd = (g.tiles + 7) / 8;
  const int64_t wgs = 8 * std::min<int64_t>(per_xcd, std::max(1, cus / 8));
  LGX_LAUNCH(f, dim3((unsigned)wgs), dim3(64 * nwv), lds, stream, g);
  return lgx_hip_status("lgx_gemm_nt");
}
