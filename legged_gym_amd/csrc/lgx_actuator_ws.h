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

// tanh(x) = 1 - 2 / (exp(2x) + 1): |error| <= ~1.5e-7 absolute (fast exp), exact +-1 saturation
LGX_DEV float fast_tanh(float x) { return 1.f - 2.f / (__expf(2.f * x) + 1.f); }

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

// ---------------------------------------------------------------- split-bf16 weight-stationary variant
// The same network on v_mfma_f32_32x32x16_bf16 with three RNE bf16 limbs per f32 operand and the
// six limb products of order <= 2 (f32-accurate, lgx_gemm_split.hip), 2.67x fewer MFMA cycles
// than the f32 MFMA.  A wave's 32-column slice of layers 0-2 lives in VGPRs as bf16 limb B
// fragments (24 + 96 + 96 registers: one wave per SIMD, so this body runs in a launch of its own,
// lgx_actuator_x3_kernel, not inside the post-physics launch's 256-register budget).  Weights are
// the MFMA's first operand: each lane ends with one row and 4 runs of 4 consecutive columns, so
// the tanh outputs are split once and stored as 8-byte limb runs of the next layer's LDS image
// [limb][32 rows][K] (no per-fragment split); layer 2 writes f32 rows for the VALU 128 -> 3 layer.
typedef __bf16 ax_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 ax_bf16x2 __attribute__((ext_vector_type(2)));
typedef float ax_fx2 __attribute__((ext_vector_type(2)));
#define AX_RS0 (32 * 2 + 16)     // layer-0 input image row stride (bytes): K = 32 + pad
#define AX_RS1 (128 * 2 + 16)    // hidden image row stride

LGX_DEV void ax_split2(float x0, float x1, uint32_t& l0, uint32_t& l1, uint32_t& l2) {
  l0 = __builtin_bit_cast(uint32_t, __builtin_convertvector((ax_fx2){x0, x1}, ax_bf16x2));
  float r0 = x0 - __uint_as_float(l0 << 16), r1 = x1 - __uint_as_float(l0 & 0xffff0000u);
  l1 = __builtin_bit_cast(uint32_t, __builtin_convertvector((ax_fx2){r0, r1}, ax_bf16x2));
  r0 -= __uint_as_float(l1 << 16);
  r1 -= __uint_as_float(l1 & 0xffff0000u);
  l2 = __builtin_bit_cast(uint32_t, __builtin_convertvector((ax_fx2){r0, r1}, ax_bf16x2));
}

// B fragment limbs of W^t [K][128] (row k, column n): lane (r, h) holds column n0 + r, k = 16 kb + 8 h ..
template <int KB>
LGX_DEV void ax_load_w(const float* __restrict__ Wt, int K, int n, int h, ax_bf16x8 (&w)[KB][3]) {
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = 16 * kb + 8 * h + i;
      v[i] = k < K ? Wt[k * WS_H + n] : 0.f;
    }
    uint4 u0, u1, u2;
    ax_split2(v[0], v[1], u0.x, u1.x, u2.x);
    ax_split2(v[2], v[3], u0.y, u1.y, u2.y);
    ax_split2(v[4], v[5], u0.z, u1.z, u2.z);
    ax_split2(v[6], v[7], u0.w, u1.w, u2.w);
    w[kb][0] = __builtin_bit_cast(ax_bf16x8, u0);
    w[kb][1] = __builtin_bit_cast(ax_bf16x8, u1);
    w[kb][2] = __builtin_bit_cast(ax_bf16x8, u2);
  }
}

// acc (transposed: lane row r, columns 8 q + 4 h + i of the wave's 32) += W . X over KB k blocks
template <int KB>
LGX_DEV void ax_layer(const char* __restrict__ img, int rs, const ax_bf16x8 (&w)[KB][3], int r, int h,
                      lgx_f32x16& acc) {
  const int limb = WS_BM * rs;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const char* p = img + r * rs + (16 * kb + 8 * h) * 2;
    const ax_bf16x8 a0 = *reinterpret_cast<const ax_bf16x8*>(p);
    const ax_bf16x8 a1 = *reinterpret_cast<const ax_bf16x8*>(p + limb);
    const ax_bf16x8 a2 = *reinterpret_cast<const ax_bf16x8*>(p + 2 * limb);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[kb][2], a0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[kb][1], a1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[kb][0], a2, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[kb][1], a0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[kb][0], a1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[kb][0], a0, acc, 0, 0, 0);
  }
}

// tanh(acc + b) of the lane's row into the next layer's limb image (8-byte runs of 4 columns)
LGX_DEV void ax_epilogue_limbs(const lgx_f32x16& acc, const float (&bb)[16], char* __restrict__ img, int wave, int r,
                               int h) {
  const int limb = WS_BM * AX_RS1;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = fast_tanh(acc[4 * q + i] + bb[4 * q + i]);
    uint32_t a0, a1, a2, b0, b1, b2;
    ax_split2(v[0], v[1], a0, a1, a2);
    ax_split2(v[2], v[3], b0, b1, b2);
    char* p = img + r * AX_RS1 + (wave * 32 + 8 * q + 4 * h) * 2;
    *reinterpret_cast<uint2*>(p) = make_uint2(a0, b0);
    *reinterpret_cast<uint2*>(p + limb) = make_uint2(a1, b1);
    *reinterpret_cast<uint2*>(p + 2 * limb) = make_uint2(a2, b2);
  }
}

LGX_DEV void actuator_x3_body(const WsArgs& a, int wg, int nwg) {
  __shared__ __attribute__((aligned(16))) char img0[3 * WS_BM * AX_RS0];   // layer-0 input (K 32)
  __shared__ __attribute__((aligned(16))) char img1[3 * WS_BM * AX_RS1];   // layer-0 output
  __shared__ __attribute__((aligned(16))) char img2[3 * WS_BM * AX_RS1];   // layer-1 output
  __shared__ float act2[WS_BM * WS_S1];                                     // layer-2 output (f32)
  __shared__ float w3[WS_H * 3 + 3];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const float* W0 = a.w;
  const float* b0 = W0 + WS_IN * WS_H;
  const float* W1 = b0 + WS_H;
  const float* b1 = W1 + WS_H * WS_H;
  const float* W2 = b1 + WS_H;
  const float* b2 = W2 + WS_H * WS_H;
  const float* W3 = b2 + WS_H;        // [128][3]
  const float* b3 = W3 + WS_H * 3;
  const int n = wave * 32 + r;        // this lane's weight column
  ax_bf16x8 wl0[2][3], wl1[8][3], wl2[8][3];
  ax_load_w<2>(W0, WS_IN, n, h, wl0);
  ax_load_w<8>(W1, WS_H, n, h, wl1);
  ax_load_w<8>(W2, WS_H, n, h, wl2);
  for (int i = tid; i < WS_H * 3 + 3; i += 256) w3[i] = i < WS_H * 3 ? W3[i] : b3[i - WS_H * 3];
  // the lane's bias values: columns wave * 32 + 8 q + 4 h + i (transposed accumulator layout)
  float bb0[16], bb1[16], bb2[16];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = wave * 32 + 8 * q + 4 * h + i;
      bb0[4 * q + i] = b0[c];
      bb1[4 * q + i] = b1[c];
      bb2[4 * q + i] = b2[c];
    }
  const float osc = a.out_scale ? a.out_scale[min(tid & 7, 2)] : 1.f;
  const int64_t ntiles = (a.rows + WS_BM - 1) / WS_BM;
  // the next tile's input rows (32 x 32, zero past column 30) are prefetched during this tile:
  // thread t holds row t >> 3, columns 4 (t & 7) .. + 3
  float pre[4];
  auto fetch = [&](int64_t tile) {
    const int row = tid >> 3, c0 = 4 * (tid & 7);
    const int64_t gr = min(tile * WS_BM + row, a.rows - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) pre[i] = a.x[gr * WS_IN + min(c0 + i, WS_IN - 1)];
  };
  fetch(wg);
  for (int64_t tile = wg; tile < ntiles; tile += nwg) {
    const int64_t r0 = tile * WS_BM;
    __syncthreads();   // the previous tile's readers of the images are done
    {
      const int row = tid >> 3, c0 = 4 * (tid & 7);
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (c0 + i < WS_IN && r0 + row < a.rows) ? pre[i] : 0.f;
      uint32_t a0, a1, a2, b0_, b1_, b2_;
      ax_split2(v[0], v[1], a0, a1, a2);
      ax_split2(v[2], v[3], b0_, b1_, b2_);
      char* p = img0 + row * AX_RS0 + c0 * 2;
      *reinterpret_cast<uint2*>(p) = make_uint2(a0, b0_);
      *reinterpret_cast<uint2*>(p + WS_BM * AX_RS0) = make_uint2(a1, b1_);
      *reinterpret_cast<uint2*>(p + 2 * WS_BM * AX_RS0) = make_uint2(a2, b2_);
    }
    fetch(tile + nwg < ntiles ? tile + nwg : tile);
    __syncthreads();
    lgx_f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    ax_layer<2>(img0, AX_RS0, wl0, r, h, acc);           // layer 0: 30 (padded 32) -> 128
    ax_epilogue_limbs(acc, bb0, img1, wave, r, h);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    ax_layer<8>(img1, AX_RS1, wl1, r, h, acc);           // layer 1: 128 -> 128
    ax_epilogue_limbs(acc, bb1, img2, wave, r, h);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    ax_layer<8>(img2, AX_RS1, wl2, r, h, acc);           // layer 2: 128 -> 128, f32 rows for layer 3
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        act2[r * WS_S1 + wave * 32 + 8 * q + 4 * h + i] = fast_tanh(acc[4 * q + i] + bb2[4 * q + i]);
    __syncthreads();
    // layer 3: 128 -> 3 on the VALU; thread = (row, 16-wide k slice), 8-lane shuffle reduction
    {
      const int rr = tid >> 3, part = tid & 7;
      const float* hrow = act2 + rr * WS_S1 + 16 * part;
      const float* wk = w3 + 16 * part * 3;
      float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float v = hrow[k];
        s0 += v * wk[3 * k]; s1 += v * wk[3 * k + 1]; s2 += v * wk[3 * k + 2];
      }
#pragma unroll
      for (int m = 1; m < 8; m <<= 1) {
        s0 += __shfl_xor(s0, m); s1 += __shfl_xor(s1, m); s2 += __shfl_xor(s2, m);
      }
      const int64_t gr = r0 + rr;
      if (part < 3 && gr < a.rows) {
        const float sv = part == 0 ? s0 : (part == 1 ? s1 : s2);
        a.y[gr * 3 + part] = (sv + w3[WS_H * 3 + part]) * osc;
      }
    }
  }
}
