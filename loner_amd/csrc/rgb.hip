// Colour head forward + colour compositing, fused (inference, C3 shape).
//
// Reference: DecoupledNeRF.forward with sigma_only=False (src/models/nerf_tcnn.py:80-95):
//   h_x   = colour HashGrid(pos01)                           (L=16, F=2, T=2^19: 32 features)
//   h_d   = SphericalHarmonics(deg 4)((viewdir + 1) / 2)     (16 features)
//   h_c   = FullyFusedMLP([h_x, h_d])  48 -> 64 (ReLU) -> ... -> 3 (padded 16), fp16, no bias
//   color = sigmoid(h_c)                                      (fp16)
// and raw2outputs' colour map (src/models/rendering_tcnn.py:283-289):
//   rgb = sum_i w_i * color_i + (1 - sum_i w_i)   (white background, rendering_tcnn.py:288-289)
// with the weights of the sigma pass (lnr_field_render), the direction repeated per sample
// (rendering_tcnn.py:319-320: the view direction, rays[:, 6:9]).
//
// One wave per ray, 16-sample tiles on v_mfma_f32_16x16x32_f16.  The first layer's 48 inputs are two
// k-steps: the 32 colour-grid features, and the 16 SH values (constant along the ray, one B operand
// per ray) zero-padded to 32.  Hidden activations are rounded to fp16 (tcnn keeps
// them in fp16) and stay in registers between layers: a layer's accumulator (hid on rows, sample on
// the lane) is the next layer's B operand when the next layer's weights are read with the k index
// permuted by hid_perm (mlp.hpp).  Weights of every layer live in registers (NH hidden-to-hidden
// layers, template).  The colour encodings are read once (64 B per sample): the kernel is bound by
// the MFMA chain (8 + 8 * NH + 2 MFMAs per 16 samples) and that read.
#include "rgb.hpp"

namespace lnr {



template <int NH, bool TRAIN>
__global__ void __launch_bounds__(64 * kRgbWaves) k_rgb_render(RgbArgs a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  if (TRAIN && a.denc_max && blockIdx.x == 0 && threadIdx.x < 16) a.denc_max[threadIdx.x] = 0.f;  // before k_rgb_bwd_tiles
  RgbWeights<NH> rw;
  load_rgb_weights<NH>(a.w, rw);
  for (int64_t r = (int64_t)blockIdx.x * kRgbWaves + wid; r < a.n_rays; r += (int64_t)gridDim.x * kRgbWaves) {
    const float* ry = a.rays + 13 * r;
    // dir = (viewdir + 1) / 2 (nerf_tcnn.py:83), SH degree 4 rounded to fp16 (tcnn encodings are fp16)
    float sh[16];
    sh_eval<4>((ry[6] + 1.0f) / 2.0f, (ry[7] + 1.0f) / 2.0f, (ry[8] + 1.0f) / 2.0f, sh);
    // B operand of the SH k-step: the same 16 fp16 values for every sample column, zero padding
    half8_t bsh = {};
    if (g < 2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) bsh[j] = (_Float16)sh[8 * g + j];
    }
    float acc_c[3] = {0.f, 0.f, 0.f}, acc_w = 0.f;
    const int64_t base = r * a.S;
    for (int tb = 0; tb < a.S; tb += 16) {
      const float w = a.weights[base + tb + c];
      // a tile whose 16 weights are all exactly 0 adds nothing to rgb (w * colour = 0): skipped
      // (its encodings may be the zeros of lnr_hashgrid_fwd_rays_live)
      if (__ballot(w != 0.f) == 0ull) continue;
      const half8_t benc = load_enc_operand(a.enc, a.enc_stride, base + tb + c, true);
      float h[16];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float4_t acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.a0[t], benc, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.as[t], bsh, acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) h[4 * t + q] = round_f16(fmaxf(acc[q], 0.f));
      }
#pragma unroll
      for (int l = 0; l < NH; ++l) {
        const half8_t b0 = hid_operand(h, 0), b1 = hid_operand(h, 1);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          float4_t acc = {0.f, 0.f, 0.f, 0.f};
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.ah[l][t][0], b0, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.ah[l][t][1], b1, acc, 0, 0, 0);
#pragma unroll
          for (int q = 0; q < 4; ++q) h[4 * t + q] = round_f16(fmaxf(acc[q], 0.f));
        }
      }
      float4_t o = {0.f, 0.f, 0.f, 0.f};
      o = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.ao[0], hid_operand(h, 0), o, 0, 0, 0);
      o = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.ao[1], hid_operand(h, 1), o, 0, 0, 0);
      if (g == 0) {  // rows 0..2 = the three colour channels of sample tb + c
        acc_w += w;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float hc = round_f16(o[k]);                             // tcnn fp16 output
          const float col = round_f16(1.0f / (1.0f + expf(-hc)));       // torch.sigmoid on fp16
          acc_c[k] = fmaf(w, col, acc_c[k]);
        }
      }
    }
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) {  // lanes 0..15 hold the partial sums
      acc_w += __shfl_xor(acc_w, off, 64);
#pragma unroll
      for (int k = 0; k < 3; ++k) acc_c[k] += __shfl_xor(acc_c[k], off, 64);
    }
    if (lane < 3) a.rgb[3 * r + lane] = (lane == 0 ? acc_c[0] : lane == 1 ? acc_c[1] : acc_c[2]) + (1.0f - acc_w);
    if (TRAIN && lane == 0) {  // nn.functional.l1_loss(rgb.reshape(-1, 1), gt.reshape(-1, 1)) (optimizer.py:883-884)
      float l = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float d = acc_c[k] + (1.0f - acc_w) - a.gt[3 * r + k];
        a.g[3 * r + k] = (d > 0.f ? a.inv_count : (d < 0.f ? -a.inv_count : 0.f));  // torch.sign
        l += fabsf(d);
      }
      a.ray_loss[r] = l;
    }
  }
}


// ------------------------------------------------------------------ colour-head training backward
// Camera phase of the reference (optimizer.py:541-688, compute_loss_camera :861-894): sigma frozen
// and detached, so dL/dlogit_i = g_ray * w_i * col_i * (1 - col_i) with g_ray = dL/drgb from
// k_rgb_render<NH, true>.  One workgroup = 4 waves, one 16-sample tile per wave per iteration:
//   1. each wave re-runs its tile's forward (bit-identical to the render), then the backward chain
//      dO -> dH_NH -> ... -> dH_0 -> d_enc on MFMA with per-wave power-of-two scaling of the fp16
//      operands (the chain's scale is tracked per layer); d_enc goes to HBM (level-major float2,
//      as lnr_field_train's) for the colour-grid backward;
//   2. every layer's input X_l (fp16) and scaled output gradient dY_l (fp16) are staged in LDS;
//   3. after a barrier, matrix l's weight gradient dW_l = sum_s dY_l[:, s] X_l[:, s]^T is
//      accumulated by ONE owner wave (16x16x16 MFMA per source wave, unscaled by that wave's
//      factor in fp32), so the 16 weight tiles of a matrix live in one wave's registers;
//   4. at the end each owner writes its tiles to the workgroup's slab; k_rgb_reduce_slabs sums the
//      slabs in a fixed order (bitwise reproducible).
// Hidden-layer operands (forward, and transposed with the hid_perm k order) are pre-arranged in LDS
// so each is one conflict-free 16-B read per lane.
constexpr int kRgbBwdWaves = 4;
constexpr int kRgbXRows = 48;                       // colour-grid features (32) + SH (16)
constexpr int kRgbCols = 16 * kRgbBwdWaves;         // samples per workgroup iteration
constexpr int kRgbLd = kRgbCols + 8;                // halfs per staged row

template <int NH>
struct RgbBwdLds {
  static constexpr int kOps = 8 * NH;                        // hidden operands per direction
  static constexpr int kXRows = kRgbXRows + 64 * (NH + 1);   // X_0 = [enc; SH], X_{l+1} = H_l
  static constexpr int kYRows = 64 * (NH + 1) + 16;          // dH_0 .. dH_NH, dO (16 rows)
  _Float16 w[2 * (kOps > 0 ? kOps : 1) * 512];
  _Float16 x[kXRows * kRgbLd];
  _Float16 y[kYRows * kRgbLd];
  float inv[kRgbBwdWaves][NH + 2];                           // 1 / scale of dY_l per source wave
  int valid[kRgbBwdWaves];
};


__device__ __forceinline__ void scale_chain(float (&v)[16], float& scale) {
  float mx = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) mx = fmaxf(mx, fabsf(v[k]));
  const float k2 = grad_scale(wave_max_nonneg(mx));
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] *= k2;
  scale *= k2;
}


// Owner accumulation for matrix i.  KIND 0: hidden (64 x 64, acc tiles 4t + m), 1: W0 (64 x 48, acc
// tiles 3t + m), 2: output (16 x 64, acc tiles 12 + m; its owner never also owns a hidden matrix).
template <int KIND>
struct RgbOwnerShape {
  static constexpr int rt = KIND == 2 ? 1 : 4, ct = KIND == 1 ? 3 : 4;
  static constexpr int ld = KIND == 1 ? kRgbIn : kRgbWidth;
  __device__ static constexpr int slot(int t, int m) { return KIND == 0 ? 4 * t + m : (KIND == 1 ? 3 * t + m : 12 + m); }
};

// The owner's tiles accumulate in the MFMA accumulators themselves, at a running power-of-two scale
// `run` (values held = true x run): a source tile whose own scale s is larger is shifted down by
// run / s <= 1 in fp16 (exact, or into subnormals for tiles far below the running maximum); a tile
// that needs a smaller scale first rescales the accumulators (rare: the running maximum only grows).
template <int NH, int KIND>
__device__ __forceinline__ void rgb_owner(const RgbBwdLds<NH>& sm, int i, float4_t (&acc)[16], float& run) {
  using Sh = RgbOwnerShape<KIND>;
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int ybase = 64 * i;  // dO sits at 64 (NH + 1) = 64 i for the output
  const int xbase = i == 0 ? 0 : kRgbXRows + 64 * (i - 1);
  float imax = 0.f;  // 1 / the smallest scale of this iteration's tiles
#pragma unroll
  for (int sw = 0; sw < kRgbBwdWaves; ++sw)
    if (sm.valid[sw]) imax = fmaxf(imax, sm.inv[sw][i]);
  if (imax == 0.f) return;
  const float s_new = 1.0f / imax;
  if (s_new < run) {  // wave-uniform
    if (run != INFINITY) {
      const float f = s_new / run;
#pragma unroll
      for (int t = 0; t < Sh::rt; ++t)
#pragma unroll
        for (int m = 0; m < Sh::ct; ++m) acc[Sh::slot(t, m)] *= f;
    }
    run = s_new;
  }
  for (int sw = 0; sw < kRgbBwdWaves; ++sw) {
    if (!sm.valid[sw]) continue;
    const _Float16 r = (_Float16)(run * sm.inv[sw][i]);  // run / s_sw = 2^-k, k >= 0
    const half4_t rv = {r, r, r, r};
    const int cs = 16 * sw + 4 * g;
    half4_t ya[Sh::rt], xb[Sh::ct];
#pragma unroll
    for (int t = 0; t < Sh::rt; ++t)
      ya[t] = *reinterpret_cast<const half4_t*>(&sm.y[(ybase + 16 * t + c) * kRgbLd + cs]) * rv;
#pragma unroll
    for (int m = 0; m < Sh::ct; ++m) xb[m] = *reinterpret_cast<const half4_t*>(&sm.x[(xbase + 16 * m + c) * kRgbLd + cs]);
#pragma unroll
    for (int t = 0; t < Sh::rt; ++t)
#pragma unroll
      for (int m = 0; m < Sh::ct; ++m)
        acc[Sh::slot(t, m)] = __builtin_amdgcn_mfma_f32_16x16x16f16(ya[t], xb[m], acc[Sh::slot(t, m)], 0, 0, 0);
  }
}

template <int NH, int KIND>
__device__ __forceinline__ void rgb_owner_store(float* __restrict__ sb, int i, const float4_t (&acc)[16], float run) {
  using Sh = RgbOwnerShape<KIND>;
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  float* mat = sb + rgb_layer_offset<NH>(i);
  const float inv = run == INFINITY ? 0.f : 1.0f / run;
#pragma unroll
  for (int t = 0; t < Sh::rt; ++t)
#pragma unroll
    for (int m = 0; m < Sh::ct; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) mat[(16 * t + 4 * g + q) * Sh::ld + 16 * m + c] = acc[Sh::slot(t, m)][q] * inv;
}

template <int NH>
__global__ void __launch_bounds__(64 * kRgbBwdWaves) k_rgb_bwd_tiles(RgbArgs a, float* __restrict__ d_enc,
                                                                     float* __restrict__ slab) {
  __shared__ RgbBwdLds<NH> sm;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  // ---- weights: layer 0 / output in registers, hidden operands in LDS
  const uint16_t* w0 = a.w;
  half8_t a0[4], as[4], b0t[2][2];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    a0[t] = ld_half8(w0 + (16 * t + c) * kRgbIn + 8 * g);
    const half8_t z = {};
    as[t] = g < 2 ? ld_half8(w0 + (16 * t + c) * kRgbIn + 32 + 8 * g) : z;
  }
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        b0t[m][s2][j] = __builtin_bit_cast(_Float16, w0[hid_perm(s2, g, j) * kRgbIn + 16 * m + c]);
  const uint16_t* wo = a.w + rgb_layer_offset<NH>(NH + 1);  // (16, 64)
  half8_t ao[2], aot[4];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) ao[s2] = ld_half8_perm(wo + c * kRgbWidth, s2, g);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j)  // A = Wout^T: [hid 16t + c][k = output 8g + j], outputs 0..2 only
      aot[t][j] = (g == 0 && j < 3) ? __builtin_bit_cast(_Float16, wo[j * kRgbWidth + 16 * t + c]) : (_Float16)0.f;
  for (int op = wid; op < 2 * RgbBwdLds<NH>::kOps; op += kRgbBwdWaves) {
    const bool tr = op >= RgbBwdLds<NH>::kOps;
    const int o = tr ? op - RgbBwdLds<NH>::kOps : op;
    const int l = o >> 3, t = (o >> 1) & 3, s2 = o & 1;  // hidden matrix l + 1
    const uint16_t* wl = a.w + rgb_layer_offset<NH>(l + 1);
    half8_t v;
    if (!tr) {
      v = ld_half8_perm(wl + (16 * t + c) * kRgbWidth, s2, g);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __builtin_bit_cast(_Float16, wl[hid_perm(s2, g, j) * kRgbWidth + 16 * t + c]);
    }
    *reinterpret_cast<half8_t*>(&sm.w[op * 512 + lane * 8]) = v;
  }
  // ---- owner jobs: matrix i (0 = W0, 1..NH hidden, NH + 1 = output) -> wave i, the 5th to wave 0
  float4_t acc[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = float4_t{0.f, 0.f, 0.f, 0.f};
  float run_a = INFINITY, run_b = INFINITY;  // running scales of the (up to two) owned matrices
  __syncthreads();

  const int64_t n_tiles = a.n_rays * (int64_t)(a.S / 16);
  const int64_t per_iter = (int64_t)gridDim.x * kRgbBwdWaves;
  const int64_t n_iter = (n_tiles + per_iter - 1) / per_iter;
  float2* denc = reinterpret_cast<float2*>(d_enc);
  float lmax[4] = {0.f, 0.f, 0.f, 0.f};  // max |d_enc| of this lane's levels 2g, 2g + 1, 8 + 2g, 9 + 2g
  // software pipelining: the next tile's HBM inputs are in flight while this tile computes (one wave
  // per SIMD at this LDS footprint, so latency is hidden by ILP only)
  uint32_t nx[4];
  float nw = 0.f, ng[3] = {0.f, 0.f, 0.f}, nd[3] = {0.f, 0.f, 0.f};
  auto prefetch = [&](int64_t tl) {
    if (tl >= n_tiles) return;
    const int64_t m0 = tl * 16, rr = m0 / a.S;
#pragma unroll
    for (int q = 0; q < 4; ++q) nx[q] = a.enc[(int64_t)(4 * g + q) * a.enc_stride + m0 + c];
    nw = a.weights[m0 + c];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      ng[k] = a.g[3 * rr + k];
      nd[k] = a.rays[13 * rr + 6 + k];
    }
  };
  prefetch((int64_t)blockIdx.x * kRgbBwdWaves + wid);
  for (int64_t it = 0; it < n_iter; ++it) {
    const int64_t tile = it * per_iter + (int64_t)blockIdx.x * kRgbBwdWaves + wid;
    const bool valid = tile < n_tiles;
    bool skip = false;
    half8_t benc;
    float w_s = 0.f, g_r[3] = {0.f, 0.f, 0.f}, sh[16];
    if (valid) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        benc[2 * q + 0] = __builtin_bit_cast(_Float16, (uint16_t)(nx[q] & 0xFFFFu));
        benc[2 * q + 1] = __builtin_bit_cast(_Float16, (uint16_t)(nx[q] >> 16));
      }
      w_s = nw;
#pragma unroll
      for (int k = 0; k < 3; ++k) g_r[k] = ng[k];
      sh_eval<4>((nd[0] + 1.0f) / 2.0f, (nd[1] + 1.0f) / 2.0f, (nd[2] + 1.0f) / 2.0f, sh);
      prefetch(tile + per_iter);
      skip = __ballot(w_s != 0.f) == 0ull;  // all 16 weights exactly 0: no gradient anywhere in the tile
    }
    if (valid && skip) {
      const int64_t n0 = tile * 16;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int lvl = 8 * m + 2 * g;
        denc[(int64_t)lvl * a.enc_stride + n0 + c] = make_float2(0.f, 0.f);
        denc[(int64_t)(lvl + 1) * a.enc_stride + n0 + c] = make_float2(0.f, 0.f);
      }
    }
    if (valid && !skip) {
      const int64_t n0 = tile * 16;
      half8_t bsh = {};
      if (g < 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bsh[j] = (_Float16)sh[8 * g + j];
      }
      const int col = 16 * wid + c;
#pragma unroll
      for (int j = 0; j < 8; ++j) sm.x[(8 * g + j) * kRgbLd + col] = benc[j];
      if (g < 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sm.x[(32 + 8 * g + j) * kRgbLd + col] = bsh[j];
      }
      // forward (as k_rgb_render), H_l staged as X_{l+1}, ReLU masks kept as bits
      float h[16];
      uint32_t mask[NH + 1];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float4_t ac = {0.f, 0.f, 0.f, 0.f};
        ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[t], benc, ac, 0, 0, 0);
        ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(as[t], bsh, ac, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) h[4 * t + q] = round_f16(fmaxf(ac[q], 0.f));
      }
#pragma unroll
      for (int l = 0; l <= NH; ++l) {
        uint32_t mk = 0;
        _Float16* xr = sm.x + (kRgbXRows + 64 * l) * kRgbLd + col;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int hid = 16 * (k >> 2) + 4 * g + (k & 3);
          xr[hid * kRgbLd] = (_Float16)h[k];
          mk |= (h[k] > 0.f ? 1u : 0u) << k;
        }
        mask[l] = mk;
        if (l == NH) break;
        const half8_t b0 = hid_operand(h, 0), b1 = hid_operand(h, 1);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const half8_t w_0 = *reinterpret_cast<const half8_t*>(&sm.w[((8 * l + 2 * t) + 0) * 512 + lane * 8]);
          const half8_t w_1 = *reinterpret_cast<const half8_t*>(&sm.w[((8 * l + 2 * t) + 1) * 512 + lane * 8]);
          float4_t ac = {0.f, 0.f, 0.f, 0.f};
          ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(w_0, b0, ac, 0, 0, 0);
          ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(w_1, b1, ac, 0, 0, 0);
#pragma unroll
          for (int q = 0; q < 4; ++q) h[4 * t + q] = round_f16(fmaxf(ac[q], 0.f));
        }
      }
      float4_t o = {0.f, 0.f, 0.f, 0.f};
      o = __builtin_amdgcn_mfma_f32_16x16x32_f16(ao[0], hid_operand(h, 0), o, 0, 0, 0);
      o = __builtin_amdgcn_mfma_f32_16x16x32_f16(ao[1], hid_operand(h, 1), o, 0, 0, 0);
      // dL/dlogit (rows 0..2 of the padded output, lanes g == 0)
      float dl[3] = {0.f, 0.f, 0.f};
      if (g == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float hc = round_f16(o[k]);
          const float cl = round_f16(1.0f / (1.0f + expf(-hc)));
          dl[k] = g_r[k] * w_s * cl * (1.0f - cl);
        }
      }
      float mx = fmaxf(fabsf(dl[0]), fmaxf(fabsf(dl[1]), fabsf(dl[2])));
      float scale = grad_scale(wave_max_nonneg(mx));
      {
        _Float16* yr = sm.y + (64 * (NH + 1)) * kRgbLd + col;
#pragma unroll
        for (int q = 0; q < 4; ++q) yr[(4 * g + q) * kRgbLd] = (_Float16)(q < 3 && g == 0 ? dl[q < 3 ? q : 0] * scale : 0.f);
        if (lane == 0) sm.inv[wid][NH + 1] = 1.0f / scale;
      }
      half8_t bo = {};
      if (g == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) bo[k] = (_Float16)(dl[k] * scale);
      }
      float dh[16];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float4_t ac = {0.f, 0.f, 0.f, 0.f};
        ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(aot[t], bo, ac, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) dh[4 * t + q] = ((mask[NH] >> (4 * t + q)) & 1u) ? ac[q] : 0.f;
      }
      // dH_NH .. dH_0: rescale, stage, propagate
#pragma unroll
      for (int l = NH; l >= 0; --l) {
        scale_chain(dh, scale);
        _Float16* yr = sm.y + (64 * l) * kRgbLd + col;
#pragma unroll
        for (int k = 0; k < 16; ++k) yr[(16 * (k >> 2) + 4 * g + (k & 3)) * kRgbLd] = (_Float16)dh[k];
        if (lane == 0) sm.inv[wid][l] = 1.0f / scale;
        if (l == 0) break;
        const half8_t b0 = hid_operand(dh, 0), b1 = hid_operand(dh, 1);
        float nd[16];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int base = RgbBwdLds<NH>::kOps + 8 * (l - 1) + 2 * t;
          const half8_t w_0 = *reinterpret_cast<const half8_t*>(&sm.w[(base + 0) * 512 + lane * 8]);
          const half8_t w_1 = *reinterpret_cast<const half8_t*>(&sm.w[(base + 1) * 512 + lane * 8]);
          float4_t ac = {0.f, 0.f, 0.f, 0.f};
          ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(w_0, b0, ac, 0, 0, 0);
          ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(w_1, b1, ac, 0, 0, 0);
#pragma unroll
          for (int q = 0; q < 4; ++q) nd[4 * t + q] = ((mask[l - 1] >> (4 * t + q)) & 1u) ? ac[q] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) dh[k] = nd[k];
      }
      // d_enc = W0[:, :32]^T dH_0 (true value: / scale)
      {
        const half8_t b0 = hid_operand(dh, 0), b1 = hid_operand(dh, 1);
        const float inv = 1.0f / scale;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          float4_t ac = {0.f, 0.f, 0.f, 0.f};
          ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0t[m][0], b0, ac, 0, 0, 0);
          ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0t[m][1], b1, ac, 0, 0, 0);
          const int lvl = 8 * m + 2 * g;
          const float2 q0 = make_float2(ac[0] * inv, ac[1] * inv), q1 = make_float2(ac[2] * inv, ac[3] * inv);
          denc[(int64_t)lvl * a.enc_stride + n0 + c] = q0;
          denc[(int64_t)(lvl + 1) * a.enc_stride + n0 + c] = q1;
          lmax[2 * m] = fmaxf(lmax[2 * m], fmaxf(fabsf(q0.x), fabsf(q0.y)));
          lmax[2 * m + 1] = fmaxf(lmax[2 * m + 1], fmaxf(fabsf(q1.x), fabsf(q1.y)));
        }
      }
    }
    if (lane == 0) sm.valid[wid] = (valid && !skip) ? 1 : 0;
    lds_barrier();  // LDS only: the d_enc stores and the next tile's loads stay in flight
    // owners: dW_i += dY_i X_i^T over the 4 source waves' samples
    if (wid == 0) rgb_owner<NH, 1>(sm, 0, acc, run_a);                       // W0
    if (wid >= 1 && wid <= NH) rgb_owner<NH, 0>(sm, wid, acc, run_a);        // hidden
    if (wid == (NH + 1) % kRgbBwdWaves) rgb_owner<NH, 2>(sm, NH + 1, acc, run_b);  // output
    lds_barrier();
  }
  float* sb = slab + (int64_t)blockIdx.x * rgb_mlp_params<NH>();
  if (wid == 0) rgb_owner_store<NH, 1>(sb, 0, acc, run_a);
  if (wid >= 1 && wid <= NH) rgb_owner_store<NH, 0>(sb, wid, acc, run_a);
  if (wid == (NH + 1) % kRgbBwdWaves) rgb_owner_store<NH, 2>(sb, NH + 1, acc, run_b);
  if (a.denc_max) {  // the colour grid backward's record scales: 16-lane row max, one atomicMax per wave and level
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = lmax[q];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
      if (c == 0 && v > 0.f)
        atomicMax(reinterpret_cast<uint32_t*>(a.denc_max) + (q >> 1) * 8 + 2 * g + (q & 1), __float_as_uint(v));
    }
  }
}

// d_w[i] = sum over the nb slabs, fixed order (as reduce_slabs_fixed, any parameter count)
__global__ void __launch_bounds__(64 * kSlabWaves) k_rgb_reduce_slabs(const float* __restrict__ slab, int nb, int P,
                                                                      float* __restrict__ dw) {
  __shared__ float part[kSlabWaves][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const int per = (nb + kSlabWaves - 1) / kSlabWaves;
  const int b0 = wid * per, b1 = b0 + per < nb ? b0 + per : nb;
  float s = 0.f;
  if (i < P) {
    int b = b0;
    for (; b + 16 <= b1; b += 16) {  // 16 rows in flight, added in order
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = slab[(int64_t)(b + u) * P + i];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; b < b1; ++b) s += slab[(int64_t)b * P + i];
  }
  part[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && i < P) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kSlabWaves; ++w) t += part[w][lane];
    dw[i] = t;
  }
}

// loss = inv_count * sum_r ray_loss[r], one workgroup, fixed order
__global__ void __launch_bounds__(1024) k_rgb_loss_sum(const float* __restrict__ ray_loss, int64_t n, float inv,
                                                       float* out) {
  __shared__ float red[16];
  float v = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) v += ray_loss[i];
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += red[w];
    out[0] = t * inv;
  }
}

constexpr int kRgbBwdMaxBlocks = 256;

}  // namespace lnr

using namespace lnr;

extern "C" int lnr_rgb_render(const uint16_t* w_rgb, int32_t n_hidden_layers, const uint32_t* enc_rgb,
                              int64_t enc_stride, const float* rays, const float* weights, int64_t n_rays,
                              int32_t n_samples, float* rgb, void* stream) {
  LNR_REQUIRE(n_hidden_layers >= 1 && n_hidden_layers <= 4,
              "lnr_rgb_render: n_hidden_layers=%d not supported (1..4, 64 neurons)", n_hidden_layers);
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && n_samples % 16 == 0,
              "lnr_rgb_render: n_samples=%d must be a positive multiple of 16", n_samples);
  LNR_REQUIRE(enc_stride >= n_rays * (int64_t)n_samples, "lnr_rgb_render: enc_stride too small");
  if (n_rays == 0) return LNR_OK;
  LNR_REQUIRE(w_rgb && enc_rgb && rays && weights && rgb, "lnr_rgb_render: null pointer");
  RgbArgs a{};
  a.w = w_rgb; a.enc = enc_rgb; a.enc_stride = enc_stride; a.rays = rays; a.weights = weights; a.n_rays = n_rays;
  a.S = n_samples; a.rgb = rgb;
  const int64_t nb = (n_rays + kRgbWaves - 1) / kRgbWaves;
  const dim3 grid((unsigned)(nb < 4096 ? nb : 4096)), block(64 * kRgbWaves);
  hipStream_t st = as_stream(stream);
  switch (n_hidden_layers - 1) {
    case 0: hipLaunchKernelGGL((k_rgb_render<0, false>), grid, block, 0, st, a); break;
    case 1: hipLaunchKernelGGL((k_rgb_render<1, false>), grid, block, 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_rgb_render<2, false>), grid, block, 0, st, a); break;
    default: hipLaunchKernelGGL((k_rgb_render<3, false>), grid, block, 0, st, a); break;
  }
  LNR_RETURN_LAUNCH("lnr_rgb_render");
}

extern "C" int64_t lnr_rgb_mlp_params(int32_t n_hidden_layers) {
  return 64 * kRgbIn + (int64_t)(n_hidden_layers - 1) * 64 * 64 + kRgbOutPad * 64;
}

extern "C" int64_t lnr_rgb_train_workspace_bytes(int32_t n_hidden_layers, int64_t n_rays) {
  const int64_t P = lnr_rgb_mlp_params(n_hidden_layers);
  return (int64_t)kRgbBwdMaxBlocks * P * 4 + ((3 * n_rays + 63) / 64) * 64 * 4 + ((n_rays + 63) / 64) * 64 * 4;
}

// The colour-head backward kernel: 2 (default) k_rgb_bwd2, 1 round 4's k_rgb_bwd_tiles (LONER_RGB_BWD, read
// at every launch)
static int rgb_bwd_version() {
  const char* e = getenv("LONER_RGB_BWD");
  return e ? atoi(e) : 2;
}
static int kRgbBwdTileWaves(int v) { return v == 1 ? kRgbBwdWaves : kRgbBwd2Waves; }

template <int NH>
static int rgb_train_launch(RgbArgs a, float* d_enc, float* d_w, float* slab, float* loss, hipStream_t st) {
  const int64_t nb_r = (a.n_rays + kRgbWaves - 1) / kRgbWaves;
  hipLaunchKernelGGL((k_rgb_render<NH, true>), dim3((unsigned)(nb_r < 4096 ? nb_r : 4096)), dim3(64 * kRgbWaves), 0,
                     st, a);
  const int64_t tiles = a.n_rays * (int64_t)(a.S / 16);
  const int v = rgb_bwd_version();
  const int64_t want = (tiles + kRgbBwdTileWaves(v) - 1) / kRgbBwdTileWaves(v);  // a tile per wave per iteration
  const int nb = (int)(want < kRgbBwdMaxBlocks ? want : kRgbBwdMaxBlocks);
  if (v == 1)
    hipLaunchKernelGGL(k_rgb_bwd_tiles<NH>, dim3(nb), dim3(64 * kRgbBwdWaves), 0, st, a, d_enc, slab);
  else
    launch_rgb_bwd2(NH, a, d_enc, slab, nb, st);
  const int P = rgb_mlp_params<NH>();
  hipLaunchKernelGGL(k_rgb_reduce_slabs, dim3((P + 63) / 64), dim3(64 * kSlabWaves), 0, st, slab, nb, P, d_w);
  if (loss) hipLaunchKernelGGL(k_rgb_loss_sum, dim3(1), dim3(1024), 0, st, a.ray_loss, a.n_rays, a.inv_count, loss);
  return LNR_OK;
}

extern "C" int lnr_rgb_train(const uint16_t* w_rgb, int32_t n_hidden_layers, const uint32_t* enc_rgb,
                             int64_t enc_stride, const float* rays, const float* weights, const float* intensities,
                             int64_t n_rays, int32_t n_samples, float inv_count, float* rgb, float* loss,
                             float* d_enc, float* d_w, void* workspace, int64_t workspace_bytes,
                             float* d_enc_level_max, void* stream) {
  LNR_REQUIRE(n_hidden_layers >= 1 && n_hidden_layers <= 4,
              "lnr_rgb_train: n_hidden_layers=%d not supported (1..4, 64 neurons)", n_hidden_layers);
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && n_samples % 16 == 0,
              "lnr_rgb_train: n_samples=%d must be a positive multiple of 16", n_samples);
  LNR_REQUIRE(enc_stride >= n_rays * (int64_t)n_samples, "lnr_rgb_train: enc_stride too small");
  LNR_REQUIRE(workspace_bytes >= lnr_rgb_train_workspace_bytes(n_hidden_layers, n_rays),
              "lnr_rgb_train: workspace too small (%lld < %lld bytes)", (long long)workspace_bytes,
              (long long)lnr_rgb_train_workspace_bytes(n_hidden_layers, n_rays));
  if (n_rays == 0) return LNR_OK;
  LNR_REQUIRE(w_rgb && enc_rgb && rays && weights && intensities && rgb && d_enc && d_w && workspace,
              "lnr_rgb_train: null pointer");
  const int64_t P = lnr_rgb_mlp_params(n_hidden_layers);
  float* slab = reinterpret_cast<float*>(workspace);
  float* g = slab + (int64_t)kRgbBwdMaxBlocks * P;
  float* ray_loss = g + ((3 * n_rays + 63) / 64) * 64;
  RgbArgs a{};
  a.w = w_rgb; a.enc = enc_rgb; a.enc_stride = enc_stride; a.rays = rays; a.weights = weights; a.n_rays = n_rays;
  a.S = n_samples; a.rgb = rgb; a.gt = intensities; a.g = g; a.ray_loss = ray_loss; a.inv_count = inv_count;
  a.denc_max = d_enc_level_max;
  hipStream_t st = as_stream(stream);
  switch (n_hidden_layers - 1) {
    case 0: rgb_train_launch<0>(a, d_enc, d_w, slab, loss, st); break;
    case 1: rgb_train_launch<1>(a, d_enc, d_w, slab, loss, st); break;
    case 2: rgb_train_launch<2>(a, d_enc, d_w, slab, loss, st); break;
    default: rgb_train_launch<3>(a, d_enc, d_w, slab, loss, st); break;
  }
  LNR_RETURN_LAUNCH("lnr_rgb_train");
}
