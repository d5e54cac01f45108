// Go1 actuator network body (weight-stationary f32 MFMA), shared by the standalone launch
// (lgx_mlp.hip) and the post-physics launch that runs it on workgroups of its own
// (lgx_envlogic.hip).  Needs lgx_device.h.
#pragma once

// ---------------------------------------------------------------- weight-stationary narrow MLP
// Go1 actuator net (30-128-128-128-3, tanh): every wave keeps its 32-column slice of all three
// 128-wide layers in VGPRs for the whole launch (B fragments of v_mfma_f32_32x32x2f32: 16 + 64 +
// 64 floats per lane) and persistent workgroups stream 32-row tiles through LDS, so the inner
// loops issue only LDS reads and MFMAs.  The 128->3 output layer runs on the VALU.
// 32x32x2 f32 operand layout (lane l): A[row l&31][k l>>5], B[k l>>5][col l&31],
// D reg i: row 8*(i/4) + 4*(l>>5) + i%4, col l&31.
typedef float lgx_f32x16 __attribute__((ext_vector_type(16)));
#define WS_BM 32
#define WS_H 128
#define WS_IN 30
#define WS_S0 33            // input tile stride (odd: conflict-free A reads)
#define WS_S1 129           // hidden tile stride

struct WsArgs {
  const float* x;
  float* y;
  int64_t rows;
  const float* w;           // packed [W0t b0 W1t b1 W2t b2 W3t b3]
  const float* out_scale;   // [3] or null
};

// tanh(x) = 1 - 2 / (exp(2x) + 1) with the hardware exp and reciprocal (v_exp_f32, v_rcp_f32, ~1 ulp
// each: |error| <= ~3e-7 absolute; exact +-1 saturation: rcp(inf) = 0, rcp(1) = 1).  The IEEE
// division it replaces expanded to ~12 instructions (v_div_scale / v_div_fmas / v_div_fixup) per
// value, 48 values per lane and tile
LGX_DEV float fast_tanh(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * x) + 1.f); }

LGX_DEV void ws_layer_epilogue(const lgx_f32x16& acc, float bb, float* __restrict__ out, int wave, int lane) {
  const int col = wave * 32 + (lane & 31);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3);
    out[row * WS_S1 + col] = fast_tanh(acc[i] + bb);
  }
}

// wg / nwg: this workgroup's index among the nwg persistent workgroups that share the rows
LGX_DEV void actuator_ws_body(const WsArgs& a, int wg, int nwg) {
  __shared__ float act0[WS_BM * WS_S1];
  __shared__ float act1[WS_BM * WS_S1];
  __shared__ float w3[WS_H * 3 + 3];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* W0 = a.w;
  const float* b0 = W0 + WS_IN * WS_H;
  const float* W1 = b0 + WS_H;
  const float* b1 = W1 + WS_H * WS_H;
  const float* W2 = b1 + WS_H;
  const float* b2 = W2 + WS_H * WS_H;
  const float* W3 = b2 + WS_H;        // [128][3]
  const float* b3 = W3 + WS_H * 3;
  const int col = wave * 32 + (lane & 31);
  const int kh = lane >> 5;
  float wr0[16], wr1[64], wr2[64];
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const int k = 2 * ks + kh;
    wr0[ks] = k < WS_IN ? W0[k * WS_H + col] : 0.f;
  }
#pragma unroll
  for (int ks = 0; ks < 64; ++ks) {
    wr1[ks] = W1[(2 * ks + kh) * WS_H + col];
    wr2[ks] = W2[(2 * ks + kh) * WS_H + col];
  }
  for (int i = tid; i < WS_H * 3 + 3; i += 256) w3[i] = i < WS_H * 3 ? W3[i] : b3[i - WS_H * 3];
  // this lane's bias of each hidden layer and the output scale, in registers for the whole launch:
  // a global load inside the tile loop would make its wait (vmcnt 0) also drain the next tile's
  // prefetch
  const float bb0 = b0[col], bb1 = b1[col], bb2 = b2[col];
  const float osc = a.out_scale ? a.out_scale[min(tid & 7, 2)] : 1.f;
  const int64_t ntiles = (a.rows + WS_BM - 1) / WS_BM;
  // next tile's input rows are prefetched into registers while the current tile computes
  float pre[4];
  auto fetch = [&](int64_t tile) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + 256 * j, r = i >> 5, k = i & 31;
      const int64_t gr = tile * WS_BM + r;
      pre[j] = (tile < ntiles && k < WS_IN && gr < a.rows) ? a.x[gr * WS_IN + k] : 0.f;
    }
  };
  fetch(wg);
  for (int64_t tile = wg; tile < ntiles; tile += nwg) {
    const int64_t r0 = tile * WS_BM;
    __syncthreads();  // previous tile's readers of act0/act1 are done
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + 256 * j;
      act0[(i >> 5) * WS_S0 + (i & 31)] = pre[j];
    }
    fetch(tile + nwg);
    __syncthreads();
    lgx_f32x16 acc;
    // layer 0: 30 (padded 32) -> 128
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(act0[(lane & 31) * WS_S0 + 2 * ks + kh], wr0[ks], acc, 0, 0, 0);
    ws_layer_epilogue(acc, bb0, act1, wave, lane);
    __syncthreads();
    // layer 1: 128 -> 128
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 64; ++ks)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(act1[(lane & 31) * WS_S1 + 2 * ks + kh], wr1[ks], acc, 0, 0, 0);
    ws_layer_epilogue(acc, bb1, act0, wave, lane);  // act0 (layer-0 input) is no longer read
    __syncthreads();
    // layer 2: 128 -> 128
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 64; ++ks)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(act0[(lane & 31) * WS_S1 + 2 * ks + kh], wr2[ks], acc, 0, 0, 0);
    ws_layer_epilogue(acc, bb2, act1, wave, lane);
    __syncthreads();
    // layer 3: 128 -> 3 on the VALU; thread = (row, 16-wide k slice), 8-lane shuffle reduction
    {
      const int r = tid >> 3, part = tid & 7;
      const float* h = act1 + r * WS_S1 + 16 * part;
      const float* wk = w3 + 16 * part * 3;
      float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float v = h[k];
        s0 += v * wk[3 * k]; s1 += v * wk[3 * k + 1]; s2 += v * wk[3 * k + 2];
      }
#pragma unroll
      for (int m = 1; m < 8; m <<= 1) {
        s0 += __shfl_xor(s0, m); s1 += __shfl_xor(s1, m); s2 += __shfl_xor(s2, m);
      }
      const int64_t gr = r0 + r;
      if (part < 3 && gr < a.rows) {
        const float sv = part == 0 ? s0 : (part == 1 ? s1 : s2);
        a.y[gr * 3 + part] = (sv + w3[WS_H * 3 + part]) * osc;
      }
    }
  }
}
