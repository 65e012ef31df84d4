// Sigma MLP (tcnn FullyFusedMLP 32 -> 64 ReLU -> 1(pad 16), no bias) on gfx950 MFMA.
//
// One wave computes a tile of 16 samples with v_mfma_f32_16x16x32_f16 (fp16 operands, fp32
// accumulate).  Operand maps (cdna_hip_programming.md §3): lane l, g = l>>4 holds
// A[row l&15][k 8g+j], B[k 8g+j][col l&15]; D[row 4g+r][col l&15].
//
// Forward computes H^T = W0 * Enc^T so the accumulator (hid on rows, sample on the lane) is
// directly usable as the B operand of the backward product dEnc^T = W0^T * dH^T with the k index
// permuted as hid(s,g,j) = 32s + 16(j>>2) + 4g + (j&3) — the permutation is applied to the W0^T
// operand once at load time, so no LDS round trip is needed between the two products.
// The 64->1 output layer is a per-lane dot product + two xor-shuffles (only row 0 of the padded
// 16-row W1 contributes to sigma).
#pragma once
#include "common.hpp"

namespace lnr {

struct SigmaWeights {
  half8_t a0[4];     // layer-0 A operand per hid tile t: W0[16t + (l&15)][8g + j]
  half8_t bt[2][2];  // backward A operand [in tile m][k-step s]: W0[hid(s,g,j)][16m + (l&15)]
  half8_t w1h[2];    // W1[0][16t + 4g + r] at index k = 4t + r, as fp16 (the weight's own precision)
  __device__ __forceinline__ float w1(int k) const { return (float)w1h[k >> 3][k & 7]; }
  __device__ __forceinline__ half8_t A0(int t) const { return a0[t]; }
  __device__ __forceinline__ half8_t BT(int m, int s) const { return bt[m][s]; }
};

// The same operands kept in LDS (one copy per workgroup, [operand][64 lanes] of 16 B: conflict-free
// ds_read_b128) and read where used: 32 fewer registers per lane for a register-bound kernel.
struct SigmaWeightsLds {
  const half8_t* a0;  // [4][64]
  const half8_t* bt;  // [2 m][2 s][64]
  half8_t w1h[2];
  __device__ __forceinline__ float w1(int k) const { return (float)w1h[k >> 3][k & 7]; }
  __device__ __forceinline__ half8_t A0(int t) const { return a0[t * 64 + (threadIdx.x & 63)]; }
  __device__ __forceinline__ half8_t BT(int m, int s) const { return bt[(2 * m + s) * 64 + (threadIdx.x & 63)]; }
  // stage from registers (every wave writes the same values: wave 0's write suffices; the caller syncs)
  __device__ __forceinline__ void stage(half8_t* lds, const struct SigmaWeights& sw);
};

// The hidden layer of one 16-sample tile, fp16 (tcnn stores it so): h[k] = relu(H)[hid 16t + 4g + r][sample
// l&15] at k = 4t + r, as packed halves (8 registers, not 16)
struct SigmaHidden {
  half8_t q[2];
  __device__ __forceinline__ float operator[](int k) const { return (float)q[k >> 3][k & 7]; }
};

__device__ __forceinline__ int hid_perm(int s, int g, int j) { return 32 * s + 16 * (j >> 2) + 4 * g + (j & 3); }

__device__ __forceinline__ void load_sigma_weights(const uint16_t* __restrict__ w, SigmaWeights& sw) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const uint16_t* w0 = w;                  // (64, 32)
  const uint16_t* w1 = w + LNR_SIGMA_W0;   // (16, 64), row 0 used
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint16_t* row = w0 + (16 * t + c) * 32 + 8 * g;
#pragma unroll
    for (int j = 0; j < 8; ++j) sw.a0[t][j] = __builtin_bit_cast(_Float16, row[j]);
  }
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) sw.bt[m][s][j] = __builtin_bit_cast(_Float16, w0[hid_perm(s, g, j) * 32 + 16 * m + c]);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      sw.w1h[(4 * t + r) >> 3][(4 * t + r) & 7] = __builtin_bit_cast(_Float16, w1[16 * t + 4 * g + r]);
}

__device__ __forceinline__ void SigmaWeightsLds::stage(half8_t* lds, const SigmaWeights& sw) {
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < 64) {
#pragma unroll
    for (int t = 0; t < 4; ++t) lds[t * 64 + lane] = sw.a0[t];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int q = 0; q < 2; ++q) lds[(4 + 2 * m + q) * 64 + lane] = sw.bt[m][q];
  }
  a0 = lds;
  bt = lds + 4 * 64;
  w1h[0] = sw.w1h[0];
  w1h[1] = sw.w1h[1];
}

// B operand of the forward product for sample n (lane column): features 8g..8g+7 = levels 4g..4g+3.
__device__ __forceinline__ half8_t load_enc_operand(const uint32_t* __restrict__ enc, int64_t stride, int64_t n,
                                                    bool valid) {
  const int g = (threadIdx.x & 63) >> 4;
  half8_t b;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t v = valid ? enc[(int64_t)(4 * g + q) * stride + n] : 0u;
    b[2 * q + 0] = __builtin_bit_cast(_Float16, (uint16_t)(v & 0xFFFFu));
    b[2 * q + 1] = __builtin_bit_cast(_Float16, (uint16_t)(v >> 16));
  }
  return b;
}

// Forward of one 16-sample tile.  h[4t+r] = fp16(relu(H))[hid 16t+4g+r][sample l&15];
// returns sigma for sample l&15 (fp32 accumulate of fp16 operands, NOT yet rounded).
// The ReLU on the rounded halves (pk_relu: one v_cvt_pk + one v_pk_max per two values) is the rounding of the
// ReLU; a -0 it may leave adds nothing below and counts as inactive everywhere (h > 0, pk_nonzero_mask).
template <class W>
__device__ __forceinline__ float sigma_tile_fwd(const W& sw, const half8_t& benc, SigmaHidden& h) {
  float4_t acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(sw.A0(t), benc, (float4_t){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  uint32_t hw[8];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    hw[2 * t] = pk_relu(acc[t][0], acc[t][1]);
    hw[2 * t + 1] = pk_relu(acc[t][2], acc[t][3]);
  }
  h.q[0] = __builtin_bit_cast(half8_t, (u32x4){hw[0], hw[1], hw[2], hw[3]});
  h.q[1] = __builtin_bit_cast(half8_t, (u32x4){hw[4], hw[5], hw[6], hw[7]});
  float part = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) part = fmaf(sw.w1(k), (k & 1) ? pk_hi(hw[k >> 1]) : pk_lo(hw[k >> 1]), part);
  part += __shfl_xor(part, 16, 64);
  part += __shfl_xor(part, 32, 64);
  return part;
}

// tcnn returns fp16; DecoupledNeRF then replaces non-finite values (nerf_tcnn.py:74-78):
// nan_to_num(posinf=65504, neginf=-65504) — NaN becomes 0.
__device__ __forceinline__ float sigma_to_f16(float s) {
  float r = round_f16(s);
  if (isnan(r)) return 0.f;
  if (isinf(r)) return r > 0 ? 65504.f : -65504.f;
  return r;
}

// Power-of-two scale that lifts the largest |value| of the wave to ~2^13 for fp16 MFMA operands.
__device__ __forceinline__ float grad_scale(float maxabs) {
  if (!(maxabs > 0.f) || !isfinite(maxabs)) return 1.f;
  int e;
  frexpf(maxabs, &e);  // maxabs = m * 2^e, m in [0.5,1)
  int k = 13 - e;
  k = k > 100 ? 100 : (k < -100 ? -100 : k);
  return ldexpf(1.f, k);
}

// Backward of one tile for d_sigma = 1: dH^T[hid][s] = w1[hid] * (h > 0) is exact in fp16, so the
// MFMA result is exact up to fp32 accumulation; the caller multiplies by the sample's d_sigma.
// d[m][r] = dEnc[sample l&15][in 16m + 4g + r] / d_sigma.
template <class W>
__device__ __forceinline__ void sigma_tile_bwd_denc(const W& sw, const SigmaHidden& h, float (&d)[2][4]) {
  half8_t b[2];  // (k-step s, j) holds hidden unit k = 8 s + j: mask * w1 in one select per half
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) b[s][j] = h.q[s][j] > (_Float16)0.f ? sw.w1h[s][j] : (_Float16)0.f;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    float4_t acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(sw.BT(m, 0), b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(sw.BT(m, 1), b[1], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) d[m][r] = acc[r];
  }
}

// dW0 accumulation for a PAIR of tiles (32 samples) through a per-wave LDS transpose.
// lds: 64*32 + 32*32 halves (6 KB) per wave.  acc[t][m][r] += dW0[16t+4g+r][16m+(l&15)].
struct DW0Acc {
  float v[4][2][4];
};

__device__ __forceinline__ void dw0_pair(_Float16* __restrict__ lds, const SigmaWeights& sw, const SigmaHidden& h0,
                                         const SigmaHidden& h1, const half8_t& e0, const half8_t& e1, float ds0,
                                         float ds1, float scale, DW0Acc& acc) {
  // dW0[hid][in] = w1[hid] * sum_s mask[hid][s] * (ds_s * Enc[s][in]); the mask operand is exact,
  // ds_s * Enc is lifted by a per-pair power of two for the fp16 operand.
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  _Float16* mk = lds;             // [64 hid][32 samples] ReLU mask
  _Float16* ens = lds + 64 * 32;  // [32 in][32 samples] scaled ds * Enc
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int hid = 16 * t + 4 * g + r;
      mk[hid * 32 + c] = (_Float16)((h0[4 * t + r] > 0.f) ? 1.f : 0.f);
      mk[hid * 32 + 16 + c] = (_Float16)((h1[4 * t + r] > 0.f) ? 1.f : 0.f);
    }
  const float s0 = ds0 * scale, s1 = ds1 * scale;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ens[(8 * g + j) * 32 + c] = (_Float16)((float)e0[j] * s0);
    ens[(8 * g + j) * 32 + 16 + c] = (_Float16)((float)e1[j] * s1);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-local hand-off through LDS
  __builtin_amdgcn_wave_barrier();
  const float inv = 1.f / scale;
  half8_t a[4], b[2];
#pragma unroll
  for (int t = 0; t < 4; ++t) a[t] = *reinterpret_cast<const half8_t*>(mk + (16 * t + c) * 32 + 8 * g);
#pragma unroll
  for (int m = 0; m < 2; ++m) b[m] = *reinterpret_cast<const half8_t*>(ens + (16 * m + c) * 32 + 8 * g);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      float4_t d = {0.f, 0.f, 0.f, 0.f};
      d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], b[m], d, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc.v[t][m][r] = fmaf(d[r], sw.w1(4 * t + r) * inv, acc.v[t][m][r]);
    }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
}

// dW0 accumulated in the MFMA accumulators themselves (C operand), at a running power-of-two operand
// scale 2^kc that only decreases: a pair whose ds * Enc needs a smaller scale first rescales the sums
// (exact: a power of two).  No per-pair fp32 FMAs and no per-pair result registers; w1 and 2^-kc are
// applied once, in finish().  Pairs whose ds are all zero add nothing and are skipped.
struct DW0Mfma {
  float4_t v[4][2];
  int kc;  // running exponent (kUnset before the first non-zero pair)
  static constexpr int kUnset = 1 << 20;
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int m = 0; m < 2; ++m) v[t][m] = float4_t{0.f, 0.f, 0.f, 0.f};
    kc = kUnset;
  }
  // acc.v[t][m][r] * w1[4t + r] * 2^-kc: dW0[16t + 4g + r][16m + (l&15)], as DW0Acc for write_dw_slab
  template <class W>
  __device__ __forceinline__ void finish(const W& sw, DW0Acc& out) const {
    const float inv = kc == kUnset ? 0.f : ldexpf(1.f, -kc);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) out.v[t][m][r] = v[t][m][r] * (sw.w1(4 * t + r) * inv);
  }
};

__device__ __forceinline__ void dw0_pair_mfma(_Float16* __restrict__ lds, const SigmaHidden& h0, const SigmaHidden& h1,
                                              const half8_t& e0, const half8_t& e1, float ds0, float ds1, float maxabs,
                                              DW0Mfma& acc) {
  if (!(maxabs > 0.f) || !isfinite(maxabs)) return;  // (wave-uniform) nothing to add
  int e;
  frexpf(maxabs, &e);
  int k = 13 - e;
  k = k > 100 ? 100 : (k < -100 ? -100 : k);
  if (k < acc.kc) {  // a larger pair: the sums so far move to the smaller scale
    if (acc.kc != DW0Mfma::kUnset) {
      const float f = ldexpf(1.f, k - acc.kc);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int m = 0; m < 2; ++m) acc.v[t][m] *= f;
    }
    acc.kc = k;
  }
  const float scale = ldexpf(1.f, acc.kc);
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  _Float16* mk = lds;             // [64 hid][32 samples] ReLU mask
  _Float16* ens = lds + 64 * 32;  // [32 in][32 samples] scaled ds * Enc
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = 8 * q + j, hid = 16 * (kk >> 2) + 4 * g + (kk & 3);
      mk[hid * 32 + c] = h0.q[q][j] > (_Float16)0.f ? (_Float16)1.f : (_Float16)0.f;
      mk[hid * 32 + 16 + c] = h1.q[q][j] > (_Float16)0.f ? (_Float16)1.f : (_Float16)0.f;
    }
  const float s0 = ds0 * scale, s1 = ds1 * scale;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#ifdef LNR_DW0_DOUBLE_ROUND
    float p0 = (float)e0[j] * s0, p1 = (float)e1[j] * s1;
    asm volatile("" : "+v"(p0), "+v"(p1));
    ens[(8 * g + j) * 32 + c] = (_Float16)p0;
    ens[(8 * g + j) * 32 + 16 + c] = (_Float16)p1;
#else
    ens[(8 * g + j) * 32 + c] = (_Float16)((float)e0[j] * s0);
    ens[(8 * g + j) * 32 + 16 + c] = (_Float16)((float)e1[j] * s1);
#endif
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-local hand-off through LDS
  __builtin_amdgcn_wave_barrier();
  half8_t a[4], b[2];
#pragma unroll
  for (int t = 0; t < 4; ++t) a[t] = *reinterpret_cast<const half8_t*>(mk + (16 * t + c) * 32 + 8 * g);
#pragma unroll
  for (int m = 0; m < 2; ++m) b[m] = *reinterpret_cast<const half8_t*>(ens + (16 * m + c) * 32 + 8 * g);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int m = 0; m < 2; ++m) acc.v[t][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], b[m], acc.v[t][m], 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
}

// dw0_pair_mfma in three parts, so a tile's hidden layer and encoding can be handed to the LDS right
// after its own use and the two tiles are never live together (same operands, same MFMAs: bitwise
// the same sums).  dw0_scale: the pair's operand scale from max |ds * Enc| over both tiles (an input
// property, known before the forward), false when the pair adds nothing; dw0_stage: tile half's mask
// and scaled ds * Enc into the wave's LDS; dw0_mfma: the 8 MFMAs once both halves are staged.
__device__ __forceinline__ bool dw0_scale(float maxabs, DW0Mfma& acc, float& scale) {
  if (!(maxabs > 0.f) || !isfinite(maxabs)) return false;  // (wave-uniform) nothing to add
  int e;
  frexpf(maxabs, &e);
  int k = 13 - e;
  k = k > 100 ? 100 : (k < -100 ? -100 : k);
  if (k < acc.kc) {
    if (acc.kc != DW0Mfma::kUnset) {
      const float f = ldexpf(1.f, k - acc.kc);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int m = 0; m < 2; ++m) acc.v[t][m] *= f;
    }
    acc.kc = k;
  }
  scale = ldexpf(1.f, acc.kc);
  return true;
}
__device__ __forceinline__ void dw0_stage(_Float16* __restrict__ lds, int half, const SigmaHidden& h, const half8_t& e,
                                          float ds_scaled) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  _Float16* mk = lds + 16 * half;
  _Float16* ens = lds + 64 * 32 + 16 * half;
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = 8 * q + j, hid = 16 * (kk >> 2) + 4 * g + (kk & 3);
      mk[hid * 32 + c] = h.q[q][j] > (_Float16)0.f ? (_Float16)1.f : (_Float16)0.f;
    }
#pragma unroll
  for (int j = 0; j < 8; ++j) ens[(8 * g + j) * 32 + c] = (_Float16)((float)e[j] * ds_scaled);
}
__device__ __forceinline__ void dw0_mfma(const _Float16* __restrict__ lds, DW0Mfma& acc) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const _Float16* mk = lds;
  const _Float16* ens = lds + 64 * 32;
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-local hand-off through LDS
  __builtin_amdgcn_wave_barrier();
  half8_t a[4], b[2];
#pragma unroll
  for (int t = 0; t < 4; ++t) a[t] = *reinterpret_cast<const half8_t*>(mk + (16 * t + c) * 32 + 8 * g);
#pragma unroll
  for (int m = 0; m < 2; ++m) b[m] = *reinterpret_cast<const half8_t*>(ens + (16 * m + c) * 32 + 8 * g);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int m = 0; m < 2; ++m) acc.v[t][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], b[m], acc.v[t][m], 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
}

// Block-level write of the per-block dW slab (3072 fp32, layout W0 (64,32) then W1 (16,64)).
// red: LDS scratch of 3072 floats.  dw1 is per-lane (hid 16t+4g+r) summed over the lane's samples.
template <int NT>
__device__ __forceinline__ void write_dw_slab(float* __restrict__ red, const DW0Acc& acc, const float (&dw1)[16],
                                              float* __restrict__ slab) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15, wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < LNR_SIGMA_MLP_PARAMS; i += NT) red[i] = 0.f;
  __syncthreads();
  float v1[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float x = dw1[i];
    x += __shfl_xor(x, 1, 64);
    x += __shfl_xor(x, 2, 64);
    x += __shfl_xor(x, 4, 64);
    x += __shfl_xor(x, 8, 64);
    v1[i] = x;
  }
  for (int w = 0; w < NT / 64; ++w) {
    if (wid == w) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[(16 * t + 4 * g + r) * 32 + 16 * m + c] += acc.v[t][m][r];
      if (c == 0) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[LNR_SIGMA_W0 + 16 * t + 4 * g + r] += v1[4 * t + r];
      }
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < LNR_SIGMA_MLP_PARAMS; i += NT) slab[i] = red[i];
}


// dW[i] += (or, overwrite, =) the sum over the nb per-workgroup slabs of slab[b][i], in a FIXED order (bitwise
// reproducible): workgroup x owns 64 consecutive i, each of its kSlabWaves waves sums a contiguous
// range of slabs (256-B coalesced rows), then the wave partials are added in wave order.
constexpr int kSlabWaves = 16;
__device__ __forceinline__ void reduce_slabs_fixed(const float* __restrict__ slab, int nb, float* __restrict__ dw,
                                                   bool overwrite = false) {
  __shared__ float part[kSlabWaves][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const int per = (nb + kSlabWaves - 1) / kSlabWaves;
  const int b0 = wid * per, b1 = b0 + per < nb ? b0 + per : nb;
  float s = 0.f;
  if (i < LNR_SIGMA_MLP_PARAMS) {
    int b = b0;
    for (; b + 32 <= b1; b += 32) {  // 32 rows in flight (a wave's whole range at 512 slabs: one load latency)
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = slab[(int64_t)(b + u) * LNR_SIGMA_MLP_PARAMS + i];
#pragma unroll
      for (int u = 0; u < 32; ++u) s += v[u];
    }
    for (; b + 8 <= b1; b += 8) {  // 8 rows in flight
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slab[(int64_t)(b + u) * LNR_SIGMA_MLP_PARAMS + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < b1; ++b) s += slab[(int64_t)b * LNR_SIGMA_MLP_PARAMS + i];
  }
  part[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && i < LNR_SIGMA_MLP_PARAMS) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kSlabWaves; ++w) t += part[w][lane];
    dw[i] = overwrite ? t : dw[i] + t;
  }
}

}  // namespace lnr
