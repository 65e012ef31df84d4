// Per-ray fused kernels: sigma MLP -> volume compositing -> LiDAR loss -> compositing backward ->
// MLP backward, one 256-thread workgroup per ray (persistent over rays).
//
// Reference semantics (file:line in /root/reference):
//   raw2outputs            src/models/rendering_tcnn.py:219-295  (default; noise active, far term)
//   raw2outputs_adjusted   src/models/rendering_tcnn.py:70-214   (T <= 0.5 crossing; overrides inert)
//   compute_loss (LiDAR)   src/mapping/optimizer.py:718-844, losses.py:29-51, JS/KL optimizer.py:913-925
//   autograd of the above  replaced by the division-free reverse affine scan documented in
//                          oracle/render.py::composite_backward
// Every per-sample intermediate (alpha, T, w, w_gt, dL/dw, dL/dsigma, hidden activations) lives in
// registers/LDS; HBM sees z, the level-major encodings in, d_enc out and per-ray scalars.
#include "common.hpp"
#include "mlp.hpp"

namespace lnr {

constexpr int NT = 256;  // threads per ray-block
constexpr int NW = NT / 64;

enum SigmaSrc { kSigmaGiven = 0, kSigmaMLP = 1 };

struct FieldArgs {
  const float* rays;
  const float* z;
  const float* sigma_in;   // kSigmaGiven
  const uint16_t* w;       // kSigmaMLP
  const uint32_t* enc;
  int64_t enc_stride;
  const float* depth_gt;
  const float* noise;
  int64_t n_rays;
  int32_t S;
  float noise_std;
  uint32_t key;
  int64_t ray_offset;
  lnr_loss_params lp;
  // outputs
  float* weights;
  float* depth;
  float* opacity;
  float* variance;
  float* d_sigma;     // kSigmaGiven + train
  float* d_enc;       // kSigmaMLP + train
  float* dw_slab;     // kSigmaMLP + train: [gridDim.x][3072]
  float* denc_max;    // optional: [16] max |d_enc| per level (float bits, atomicMax; zeroed by the ray phase)
  uint32_t* d_jac;    // optional, replaces d_enc: d sigma / d enc as level-major fp16 pairs (d_enc = d_sigma J)
  float* ray_stats;   // train: [R][LNR_RAY_STATS]
  // kLossExternal: upstream gradients of the render outputs (any may be NULL = zero)
  const float* g_weights;   // (R,S)
  const float* g_depth;     // (R)
  const float* g_opacity;   // (R)
  const float* g_variance;  // (R)
  float* d_ray;             // optional (R,2): [dL/d|d|, dL/dfar] (the render's dependence on the ray itself)
};

// lnr_loss_params.kind for the plain autograd backward of the render (no loss inside the kernel)
constexpr int32_t kLossExternal = 100;

// Graph replay: the step's key, los_lambda and los_eps from device memory (lnr_step_scalars).
__device__ __forceinline__ uint32_t step_key_of(const FieldArgs& a) { return a.lp.dev_step ? a.lp.dev_step->key : a.key; }
__device__ __forceinline__ lnr_loss_params step_lp(const lnr_loss_params& in) {
  lnr_loss_params lp = in;
  if (lp.dev_step) {
    lp.los_lambda = lp.dev_step->los_lambda;
    lp.los_eps = lp.dev_step->los_eps;
  }
  return lp;
}

struct RayShared {
  float* sig;        // [S] sigma, then dL/dsigma
  float* red;        // reduction scratch [16 * NW]
  double* dscan;     // [NW] wave products
  float* fscan;      // [2 * NW] affine wave totals
  float* lastT;      // [NT]
  float* slot;       // [4]
  _Float16* mlp;     // [NW][64*32 + 32*32]
};

// ---------------------------------------------------------------- block scans
// Exclusive multiplicative scan of per-thread doubles across the block.
__device__ __forceinline__ double block_excl_prod(double p, double* dscan) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double inc = p;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    double q = __shfl_up(inc, o, 64);
    if (lane >= o) inc *= q;
  }
  if (lane == 63) dscan[wid] = inc;
  __syncthreads();
  double pre = 1.0;
  for (int w = 0; w < wid; ++w) pre *= dscan[w];
  double excl = __shfl_up(inc, 1, 64);
  if (lane == 0) excl = 1.0;
  __syncthreads();
  return pre * excl;
}

// Reverse (suffix) scan of affine maps F_t(x) = A x + B; returns X_t = (F_{t+1} o ... o F_last)(0).
__device__ __forceinline__ float block_suffix_affine(float A, float B, float* fscan) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float qa = A, qb = B;  // inclusive suffix composition Q_t = F_t o Q_{t+1}
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    float na = __shfl_down(qa, o, 64), nb = __shfl_down(qb, o, 64);
    if (lane + o < 64) {
      qb = qa * nb + qb;
      qa = qa * na;
    }
  }
  if (lane == 0) {
    fscan[2 * wid] = qa;
    fscan[2 * wid + 1] = qb;
  }
  __syncthreads();
  // value entering this wave from the right: (W_{w+1} o ... o W_last)(0)
  float xw = 0.f;
  for (int w = NW - 1; w > wid; --w) xw = fscan[2 * w] * xw + fscan[2 * w + 1];
  float na = __shfl_down(qa, 1, 64), nb = __shfl_down(qb, 1, 64);
  float x = (lane == 63) ? xw : na * xw + nb;
  __syncthreads();
  return x;
}

// ---------------------------------------------------------------- compositing + loss for one ray
template <int C, bool TRAIN, bool ADJ>
__device__ void composite_ray(const FieldArgs& a, const RayShared& sh, int64_t r) {
  const int t = threadIdx.x;
  const int S = a.S;
  const int i0 = t * C;
  const bool active = i0 < S;
  const float* ry = a.rays + 13 * r;
  const float dx = ry[3], dy = ry[4], dz = ry[5];
  const float far = ry[12];
  const float dnorm = sqrtf(dx * dx + dy * dy + dz * dz);
  const float* zr = a.z + r * S;
  const int64_t gr = a.ray_offset + r;

  float z[C], alpha[C], s[C], delta[C], x[C], w[C], dlr[C];
  double tl[C];
  double P = 1.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int i = i0 + c;
    dlr[c] = 0.f;
    if (active && i < S) {
      z[c] = zr[i];
      const float zn = (i + 1 < S) ? zr[i + 1] : 0.f;
      const float dl = (i + 1 < S) ? (zn - z[c]) : 1e10f;
      dlr[c] = dl;
      delta[c] = dl * dnorm;
      float nz = 0.f;
      if (!ADJ) {
        if (a.noise) nz = a.noise[r * S + i] * a.noise_std;
        else if (a.noise_std > 0.f) nz = rand_normal(step_key_of(a), kStreamNoise, (uint32_t)gr, (uint32_t)i) * a.noise_std;
      }
      x[c] = sh.sig[i] + nz;
      const float sr = fmaxf(x[c], 0.f);
      alpha[c] = 1.0f - expf(-(delta[c] * sr));
      s[c] = (1.0f - alpha[c]) + 1e-10f;
    } else {
      z[c] = 0.f; delta[c] = 0.f; x[c] = 0.f; alpha[c] = 0.f; s[c] = 1.f;
    }
    tl[c] = P;
    P *= (double)s[c];
  }
  const double T0 = block_excl_prod(P, sh.dscan);
  float T[C];
  float sw = 0.f;
  double acc_w = 0.0, acc_wz = 0.0, acc_wzs = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    T[c] = (float)(T0 * tl[c]);
    w[c] = alpha[c] * T[c];
    if (active && i0 + c < S) {
      acc_w += (double)w[c];
      acc_wz += (double)(w[c] * z[c]);
      if (TRAIN) acc_wzs += (double)((z[c] * a.lp.scale) * w[c]);
    }
  }
  (void)sw;
  float redA[3] = {(float)acc_w, (float)acc_wz, (float)acc_wzs};
  // block sums in double-rounded float: wave sums of per-thread doubles cast to float are exact
  // enough for S <= 4096 (see DESIGN.md numerics); the reference sums fp32 products.
  block_sum<NT, 3>(redA, sh.red);
  const float wsum = redA[0];
  float depth;
  if (ADJ) {
    if (t == 0) sh.slot[0] = 0.f;
    float lt = 1.0f;
#pragma unroll
    for (int c = 0; c < C; ++c)
      if (active && i0 + c < S) lt = T[c];
    sh.lastT[t] = lt;
    __syncthreads();
    float Tprev = (t == 0) ? 1.0f : sh.lastT[t - 1];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (active && i0 + c < S) {
        if (!(T[c] > 0.5f) && (Tprev > 0.5f)) sh.slot[0] = z[c];
        Tprev = T[c];
      }
    }
    __syncthreads();
    depth = sh.slot[0];
    __syncthreads();
  } else {
    const float tail = (1.0f - wsum) * far;
    depth = (float)((double)redA[1] + (double)tail);
  }
  const float opacity = wsum;

  // pass B: variance of the render, and the loss-side weighted variance
  const float wden = wsum + 1e-10f;
  const float mean = TRAIN ? redA[2] / wden : 0.f;
  double acc_var = 0.0, acc_lv = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    if (active && i0 + c < S) {
      const float dd = depth - z[c];
      acc_var += (double)(w[c] * (dd * dd));
      if (TRAIN) {
        const float e = z[c] * a.lp.scale - mean;
        acc_lv += (double)((e * e) * w[c]);
      }
    }
  }
  float redB[2] = {(float)acc_var, (float)acc_lv};
  block_sum<NT, 2>(redB, sh.red);
  const float variance = redB[0];

  if (t == 0) {
    if (a.depth) a.depth[r] = depth;
    if (a.opacity) a.opacity[r] = opacity;
    if (a.variance) a.variance[r] = variance;
  }
  if (!TRAIN) {
    if (a.weights && active)
#pragma unroll
      for (int c = 0; c < C; ++c)
        if (i0 + c < S) a.weights[r * S + i0 + c] = w[c];
    return;
  }

  const lnr_loss_params lp = step_lp(a.lp);
  if (lp.kind == kLossExternal) {
    // autograd of raw2outputs(_adjusted) w.r.t. sigma given dL/d{weights, depth, opacity, variance}
    // (rendering_tcnn.py:262-293): variance = sum w (depth - z)^2 feeds w directly and via depth;
    // depth = sum w z + (1 - sum w) far feeds w_k with (z_k - far).  The adjusted depth is a
    // piecewise-constant pick of z, so it passes no gradient (:130-132).
    const float gv = a.g_variance ? a.g_variance[r] : 0.f;
    const float gd = ADJ ? 0.f : (a.g_depth ? a.g_depth[r] : 0.f) + gv * 2.0f * (depth * opacity - redA[1]);
    const float go = a.g_opacity ? a.g_opacity[r] : 0.f;
    float G[C];
    float FA = 1.f, FB = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      G[c] = 0.f;
      if (active && i0 + c < S) {
        const float dd = depth - z[c];
        const float gw = a.g_weights ? a.g_weights[r * S + i0 + c] : 0.f;
        G[c] = gw + gv * (dd * dd) + (ADJ ? 0.f : gd * (z[c] - far)) + go;
      }
    }
#pragma unroll
    for (int c = C - 1; c >= 0; --c) {
      if (active && i0 + c < S) {
        FB = G[c] * alpha[c] + s[c] * FB;
        FA = s[c] * FA;
      }
    }
    float X = block_suffix_affine(FA, FB, sh.fscan);
    double acc_dn = 0.0;
#pragma unroll
    for (int c = C - 1; c >= 0; --c) {
      if (active && i0 + c < S) {
        const float dA = T[c] * (G[c] - X);
        X = G[c] * alpha[c] + s[c] * X;
        const float sr = fmaxf(x[c], 0.f);
        const float ex = expf(-(delta[c] * sr));
        const float dsig = (x[c] > 0.f) ? dA * (delta[c] * ex) : 0.f;
        sh.sig[i0 + c] = dsig;
        if (a.d_sigma) a.d_sigma[r * S + i0 + c] = dsig;
        // deltas = dl * |d| (rendering_tcnn.py:248): d alpha / d |d| = dl * relu(sigma + noise) * exp(-delta sr)
        acc_dn += (double)((dA * (ex * sr)) * dlr[c]);
      }
    }
    if (a.d_ray) {  // (block-uniform branch)
      float rd[1] = {(float)acc_dn};
      block_sum<NT, 1>(rd, sh.red);
      if (t == 0) {
        a.d_ray[2 * r + 0] = rd[0];
        // depth = sum w z + (1 - sum w) far (rendering_tcnn.py:274-278); the adjusted depth ignores far
        a.d_ray[2 * r + 1] = ADJ ? 0.f : gd * (1.0f - wsum);
      }
    }
    __syncthreads();
    return;
  }

  // ------------------------------------------------ loss (optimizer.py:718-844)
  const float inv_nop = lp.dev_n_opaque ? 1.0f / fmaxf(lp.dev_n_opaque[0], 1.0f) : lp.inv_n_opaque;
  const float dgt = a.depth_gt[r];
  const float g = dgt * lp.scale;
  const float far_ref = lp.dev_far_ref ? lp.dev_far_ref[0] : lp.far_ref;
  const bool opaque = (dgt > 0.f) && !(dgt > far_ref);
  const float lvar = redB[1] / wden + 1e-10f;
  const float stdv = sqrtf(lvar);
  float eps;
  if (lp.kind == LNR_LOSS_L1_JS || lp.kind == LNR_LOSS_L2_JS) {
    const float s1 = lp.min_depth_eps / 3.0f;
    const float mm = 0.5f * (g + mean);
    const float smv = 0.5f * sqrtf(s1 * s1 + stdv * stdv);
    const float v2 = smv * smv;
    const float kl1 = logf(smv / s1) + (s1 * s1 + (g - mm) * (g - mm)) / (2.0f * v2) - 0.5f;
    const float kl2 = logf(smv / stdv) + (stdv * stdv + (mean - mm) * (mean - mm)) / (2.0f * v2) - 0.5f;
    float js = 0.5f * kl1 + 0.5f * kl2;
    if (js < lp.min_js) js = 0.f;
    if (js > lp.max_js) js = lp.max_js;
    eps = lp.min_depth_eps * (1.0f + lp.js_alpha * js);
  } else {
    eps = lp.los_eps;
  }
  // truncated Gaussian target (losses.py:29-51)
  const float sg = eps / 9.0f;
  const float clip_a = ((g - eps) - g) / sg;
  const float clip_b = ((g + eps) - g) / sg;
  const float cdf_a = 0.5f * (1.0f + erff(clip_a / 1.4142135623730951f));
  const float cdf_b = 0.5f * (1.0f + erff(clip_b / 1.4142135623730951f));
  const float zden = cdf_b - cdf_a;
  float wgt[C];
  double acc_gt = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    wgt[c] = 0.f;
    if (active && i0 + c < S) {
      const float sm = z[c] * lp.scale;
      const float xx = (sm - g) / sg;
      const float pdf = 0.3989422804014327f * expf(-0.5f * (xx * xx));
      const float v = pdf / sg / zden;
      const bool inside = ((sm - (g - eps)) > 0.f) && (((g + eps) - sm) > 0.f);
      wgt[c] = inside ? v : 0.f;
      acc_gt += (double)wgt[c];
    }
  }
  float redC[1] = {(float)acc_gt};
  block_sum<NT, 1>(redC, sh.red);
  const float gt_den = redC[0] + 1e-6f;
  const bool l1 = (lp.kind == LNR_LOSS_L1_JS || lp.kind == LNR_LOSS_L1_LOS);
  const float d_euc = depth * lp.scale;
  const float ddiff = d_euc - g;
  const float g_depth = opaque ? lp.depthloss_lambda * 2.0f * ddiff * lp.scale * inv_nop : 0.f;
  const float operr = opacity - 1.0f;
  const float g_op = opaque ? ((operr > 0.f) ? 1.f : (operr < 0.f ? -1.f : 0.f)) * inv_nop : 0.f;
  float G[C];
  double acc_los = 0.0;
  float FA = 1.f, FB = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    G[c] = 0.f;
    if (active && i0 + c < S) {
      const float wg = opaque ? wgt[c] / gt_den : 0.f;
      const float dw = w[c] - wg;
      float gw;
      if (l1) {
        gw = lp.los_lambda * ((dw > 0.f) ? 1.f : (dw < 0.f ? -1.f : 0.f)) * lp.inv_rs;
        acc_los += (double)fabsf(dw);
      } else {
        gw = lp.los_lambda * 2.0f * dw * lp.inv_rs;
        acc_los += (double)(dw * dw);
      }
      G[c] = gw + g_depth * (z[c] - far) + g_op;
    }
  }
  // F_t composed right-to-left over the chunk: x <- G_k alpha_k + s_k x
#pragma unroll
  for (int c = C - 1; c >= 0; --c) {
    if (active && i0 + c < S) {
      FB = G[c] * alpha[c] + s[c] * FB;
      FA = s[c] * FA;
    }
  }
  float redD[1] = {(float)acc_los};
  block_sum<NT, 1>(redD, sh.red);
  float X = block_suffix_affine(FA, FB, sh.fscan);
  double acc_dn = 0.0;
#pragma unroll
  for (int c = C - 1; c >= 0; --c) {
    if (active && i0 + c < S) {
      const float dA = T[c] * (G[c] - X);
      X = G[c] * alpha[c] + s[c] * X;
      const float sr = fmaxf(x[c], 0.f);
      const float ex = expf(-(delta[c] * sr));
      const float dsig = (x[c] > 0.f) ? dA * (delta[c] * ex) : 0.f;
      sh.sig[i0 + c] = dsig;
      if (a.d_sigma) a.d_sigma[r * S + i0 + c] = dsig;
      acc_dn += (double)((dA * (ex * sr)) * dlr[c]);
    }
  }
  if (a.d_ray) {  // the loss's dependence on the ray (poses under optimisation): see composite_loss_wave
    float rd[1] = {(float)acc_dn};
    block_sum<NT, 1>(rd, sh.red);
    if (t == 0) {
      a.d_ray[2 * r + 0] = rd[0];
      a.d_ray[2 * r + 1] = ADJ ? 0.f : g_depth * (1.0f - wsum);
    }
  }
  if (a.weights && active)
#pragma unroll
    for (int c = 0; c < C; ++c)
      if (i0 + c < S) a.weights[r * S + i0 + c] = w[c];
  if (t == 0) {
    float* st = a.ray_stats + r * LNR_RAY_STATS;
    st[0] = opaque ? ddiff * ddiff : 0.f;
    st[1] = redD[0];
    st[2] = opaque ? fabsf(operr) : 0.f;
    st[3] = eps;
    st[4] = opaque ? 1.f : 0.f;
  }
  __syncthreads();
}

// ---------------------------------------------------------------- MLP phases
__device__ __forceinline__ void mlp_forward_ray(const FieldArgs& a, const RayShared& sh, const SigmaWeights& sw,
                                                int64_t r) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int per_wave = a.S / NW;
  for (int tb = wid * per_wave; tb < (wid + 1) * per_wave; tb += 16) {
    const int64_t n = r * a.S + tb + c;
    half8_t b = load_enc_operand(a.enc, a.enc_stride, n, true);
    SigmaHidden h;
    const float sg = sigma_tile_fwd(sw, b, h);
    if (g == 0) sh.sig[tb + c] = sigma_to_f16(sg);
    if (a.lp.dev_status && __any(!isfinite(round_f16(sg))) && lane == 0) atomicOr(a.lp.dev_status, LNR_STATUS_SIGMA_CLIPPED);
  }
  __syncthreads();
}

__device__ __forceinline__ void mlp_backward_ray(const FieldArgs& a, const RayShared& sh, const SigmaWeights& sw,
                                                 int64_t r, DW0Acc& acc, float (&dw1)[16]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int per_wave = a.S / NW;
  _Float16* lds = sh.mlp + wid * (64 * 32 + 32 * 32);
  float2* denc = reinterpret_cast<float2*>(a.d_enc);
  for (int tb = wid * per_wave; tb < (wid + 1) * per_wave; tb += 32) {
    SigmaHidden h0, h1;
    half8_t e0, e1;
    float ds0, ds1;
    {
      const int64_t n = r * a.S + tb + c;
      e0 = load_enc_operand(a.enc, a.enc_stride, n, true);
      (void)sigma_tile_fwd(sw, e0, h0);
      ds0 = sh.sig[tb + c];
    }
    const bool second = tb + 16 < (wid + 1) * per_wave;
    {
      const int64_t n = r * a.S + tb + 16 + c;
      e1 = load_enc_operand(a.enc, a.enc_stride, n, second);
      (void)sigma_tile_fwd(sw, e1, h1);
      ds1 = second ? sh.sig[tb + 16 + c] : 0.f;
    }
    float mx = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      dw1[k] = fmaf(ds0, h0[k], dw1[k]);
      dw1[k] = fmaf(ds1, h1[k], dw1[k]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fmaxf(fabsf((float)e0[j] * ds0), fabsf((float)e1[j] * ds1)));
    const float scale = grad_scale(wave_max(mx));
    float d[2][4];
    sigma_tile_bwd_denc(sw, h0, d);
    {
      const int64_t n = r * a.S + tb + c;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int lvl = 8 * m + 2 * g;
        denc[(int64_t)lvl * a.enc_stride + n] = make_float2(d[m][0] * ds0, d[m][1] * ds0);
        denc[(int64_t)(lvl + 1) * a.enc_stride + n] = make_float2(d[m][2] * ds0, d[m][3] * ds0);
      }
    }
    sigma_tile_bwd_denc(sw, h1, d);
    if (second) {
      const int64_t n = r * a.S + tb + 16 + c;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int lvl = 8 * m + 2 * g;
        denc[(int64_t)lvl * a.enc_stride + n] = make_float2(d[m][0] * ds1, d[m][1] * ds1);
        denc[(int64_t)(lvl + 1) * a.enc_stride + n] = make_float2(d[m][2] * ds1, d[m][3] * ds1);
      }
    }
    dw0_pair(lds, sw, h0, h1, e0, e1, ds0, ds1, scale, acc);
  }
}

// ---------------------------------------------------------------- kernels
template <int C, bool TRAIN, bool ADJ, int SRC>
__global__ void __launch_bounds__(NT) k_field(FieldArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  RayShared sh;
  {
    char* p = smem;
    sh.sig = reinterpret_cast<float*>(p);
    p += ((a.S * 4 + 15) / 16) * 16;
    sh.red = reinterpret_cast<float*>(p);
    p += 16 * NW * 4;
    sh.dscan = reinterpret_cast<double*>(p);
    p += NW * 8;
    sh.fscan = reinterpret_cast<float*>(p);
    p += 2 * NW * 4;
    sh.lastT = reinterpret_cast<float*>(p);
    p += NT * 4;
    sh.slot = reinterpret_cast<float*>(p);
    p += 16;
    sh.mlp = reinterpret_cast<_Float16*>(p);
  }
  SigmaWeights sw;
  DW0Acc acc;
  float dw1[16];
  if (SRC == kSigmaMLP) {
    load_sigma_weights(a.w, sw);
    if (TRAIN) {
#pragma unroll
      for (int k = 0; k < 16; ++k) dw1[k] = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc.v[t][m][q] = 0.f;
    }
  }
  for (int64_t r = blockIdx.x; r < a.n_rays; r += gridDim.x) {
    if (SRC == kSigmaMLP) {
      mlp_forward_ray(a, sh, sw, r);
    } else {
      for (int i = threadIdx.x; i < a.S; i += NT) sh.sig[i] = a.sigma_in[r * a.S + i];
      __syncthreads();
    }
    composite_ray<C, TRAIN, ADJ>(a, sh, r);
    if (SRC == kSigmaMLP && TRAIN) mlp_backward_ray(a, sh, sw, r, acc, dw1);
    __syncthreads();
  }
  if (SRC == kSigmaMLP && TRAIN) {
    write_dw_slab<NT>(reinterpret_cast<float*>(smem), acc, dw1, a.dw_slab + (int64_t)blockIdx.x * LNR_SIGMA_MLP_PARAMS);
  }
}

// ---------------------------------------------------------------- wave-per-ray training kernel
// The training hot path (lnr_field_train: sigma MLP, default compositing, LiDAR loss, backward)
// with ONE WAVE PER RAY: S = 64 * C samples, lane l holds samples [C*l, C*l + C).  Scans and sums
// are wave-level shuffles, so a ray needs no workgroup barrier; the 4 waves of a workgroup work on
// 4 rays independently and meet once, at the end, to reduce their dW slabs.  Same arithmetic as
// composite_ray<C, true, false> (the block version), reassociated only in the cross-lane sums.
constexpr int kWavesPerBlock = NT / 64;
#ifndef LNR_MLP_BWD_BLOCKS
#define LNR_MLP_BWD_BLOCKS 512  // workgroups of k_mlp_bwd_tiles (and dW slabs), at most: one resident round (C2: 178.8 + 7.7 us slab reduce at 1024, 175.5 + 4.9 at 512)
#endif
constexpr int kMlpBwdBlocks = LNR_MLP_BWD_BLOCKS;
#ifndef LNR_FIELD_SPLIT
#define LNR_FIELD_SPLIT 1  // lnr_field_train: MLP forward and compositing as two kernels (k_sigma_fwd_tiles, k_composite_wave)
#endif
constexpr int kSigmaLevels = 16;  // the sigma MLP's 32 inputs: 16 levels x 2 features

__device__ __forceinline__ double wave_excl_prod(double p) {
  const int lane = threadIdx.x & 63;
  double inc = p;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double q = __shfl_up(inc, o, 64);
    if (lane >= o) inc *= q;
  }
  const double ex = __shfl_up(inc, 1, 64);
  return lane == 0 ? 1.0 : ex;
}

// X_t = (F_{t+1} o ... o F_63)(0) for per-lane affine maps F(x) = A x + B.
__device__ __forceinline__ float wave_suffix_affine(float A, float B) {
  const int lane = threadIdx.x & 63;
  float qa = A, qb = B;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float na = __shfl_down(qa, o, 64), nb = __shfl_down(qb, o, 64);
    if (lane + o < 64) {
      qb = qa * nb + qb;
      qa = qa * na;
    }
  }
  const float na = __shfl_down(qa, 1, 64), nb = __shfl_down(qb, 1, 64);
  return (lane == 63) ? 0.f : na * 0.f + nb;
}

__device__ __forceinline__ void wave_lds_handoff() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
}

template <int C>
__device__ void composite_loss_wave(const FieldArgs& a, float* sig, int64_t r) {
  const int lane = threadIdx.x & 63;
  const int S = a.S;
  const int i0 = lane * C;
  const float* ry = a.rays + 13 * r;
  const float dx = ry[3], dy = ry[4], dz = ry[5];
  const float far = ry[12];
  const float dnorm = sqrtf(dx * dx + dy * dy + dz * dz);
  const float* zr = a.z + r * S;
  const int64_t gr = a.ray_offset + r;
  const lnr_loss_params lp = step_lp(a.lp);

  float z[C], alpha[C], s[C], delta[C], x[C], T[C], w[C];
  double tl[C];
#pragma unroll
  for (int c = 0; c < C; ++c) z[c] = zr[i0 + c];
  const float z_next = __shfl_down(z[0], 1, 64);  // first sample of the next lane
  double P = 1.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int i = i0 + c;
    const float zn = (c + 1 < C) ? z[c + 1] : z_next;
    const float dl = (i + 1 < S) ? (zn - z[c]) : 1e10f;
    delta[c] = dl * dnorm;
    float nz = 0.f;
    if (a.noise) nz = a.noise[r * S + i] * a.noise_std;
    else if (a.noise_std > 0.f) nz = rand_normal(step_key_of(a), kStreamNoise, (uint32_t)gr, (uint32_t)i) * a.noise_std;
    x[c] = sig[i] + nz;
    const float sr = fmaxf(x[c], 0.f);
    alpha[c] = 1.0f - expf(-(delta[c] * sr));
    s[c] = (1.0f - alpha[c]) + 1e-10f;
    tl[c] = P;
    P *= (double)s[c];
  }
  const double T0 = wave_excl_prod(P);
  double acc_w = 0.0, acc_wz = 0.0, acc_wzs = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    T[c] = (float)(T0 * tl[c]);
    w[c] = alpha[c] * T[c];
    acc_w += (double)w[c];
    acc_wz += (double)(w[c] * z[c]);
    acc_wzs += (double)((z[c] * lp.scale) * w[c]);
  }
  if (lp.dev_term_hist && S % 64 == 0) {
    // where the ray terminates (lnr_loss_params.dev_term_hist): its samples after which the transmittance product
    // (the one above, in double) is still >= the early-ray-termination threshold
    int live = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) live += (T0 * tl[c] * (double)s[c] >= LNR_ERT_T_MIN) ? 1 : 0;
    const int cnt = (int)wave_sum((float)live);  // (exact: at most 512)
    if (lane == 0) atomicAdd(lp.dev_term_hist + (r % LNR_TERM_HIST_SLOTS) * (S / 64 + 1) + cnt / 64, 1u);
  }
  const float wsum = wave_sum((float)acc_w);
  const float wzsum = wave_sum((float)acc_wz);
  const float wzssum = wave_sum((float)acc_wzs);
  const float tail = (1.0f - wsum) * far;
  const float depth = (float)((double)wzsum + (double)tail);
  const float opacity = wsum;
  const float wden = wsum + 1e-10f;
  const float mean = wzssum / wden;
  double acc_lv = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float e = z[c] * lp.scale - mean;
    acc_lv += (double)((e * e) * w[c]);
  }
  const float lvsum = wave_sum((float)acc_lv);
  if (lane == 0) {
    if (a.depth) a.depth[r] = depth;
    if (a.opacity) a.opacity[r] = opacity;
  }
  // ------------------------------------------------ loss (optimizer.py:718-844)
  const float inv_nop = lp.dev_n_opaque ? 1.0f / fmaxf(lp.dev_n_opaque[0], 1.0f) : lp.inv_n_opaque;
  const float dgt = a.depth_gt[r];
  const float g = dgt * lp.scale;
  const float far_ref = lp.dev_far_ref ? lp.dev_far_ref[0] : lp.far_ref;
  const bool opaque = (dgt > 0.f) && !(dgt > far_ref);
  const float lvar = lvsum / wden + 1e-10f;
  const float stdv = sqrtf(lvar);
  float eps;
  if (lp.kind == LNR_LOSS_L1_JS || lp.kind == LNR_LOSS_L2_JS) {
    const float s1 = lp.min_depth_eps / 3.0f;
    const float mm = 0.5f * (g + mean);
    const float smv = 0.5f * sqrtf(s1 * s1 + stdv * stdv);
    const float v2 = smv * smv;
    const float kl1 = logf(smv / s1) + (s1 * s1 + (g - mm) * (g - mm)) / (2.0f * v2) - 0.5f;
    const float kl2 = logf(smv / stdv) + (stdv * stdv + (mean - mm) * (mean - mm)) / (2.0f * v2) - 0.5f;
    float js = 0.5f * kl1 + 0.5f * kl2;
    if (js < lp.min_js) js = 0.f;
    if (js > lp.max_js) js = lp.max_js;
    eps = lp.min_depth_eps * (1.0f + lp.js_alpha * js);
  } else {
    eps = lp.los_eps;
  }
  // truncated Gaussian target (losses.py:29-51)
  const float sg = eps / 9.0f;
  const float clip_a = ((g - eps) - g) / sg;
  const float clip_b = ((g + eps) - g) / sg;
  const float cdf_a = 0.5f * (1.0f + erff(clip_a / 1.4142135623730951f));
  const float cdf_b = 0.5f * (1.0f + erff(clip_b / 1.4142135623730951f));
  const float zden = cdf_b - cdf_a;
  float wgt[C];
  double acc_gt = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float sm = z[c] * lp.scale;
    const float xx = (sm - g) / sg;
    const float pdf = 0.3989422804014327f * expf(-0.5f * (xx * xx));
    const float v = pdf / sg / zden;
    const bool inside = ((sm - (g - eps)) > 0.f) && (((g + eps) - sm) > 0.f);
    wgt[c] = inside ? v : 0.f;
    acc_gt += (double)wgt[c];
  }
  const float gt_den = wave_sum((float)acc_gt) + 1e-6f;
  const bool l1 = (lp.kind == LNR_LOSS_L1_JS || lp.kind == LNR_LOSS_L1_LOS);
  const float d_euc = depth * lp.scale;
  const float ddiff = d_euc - g;
  const float g_depth = opaque ? lp.depthloss_lambda * 2.0f * ddiff * lp.scale * inv_nop : 0.f;
  const float operr = opacity - 1.0f;
  const float g_op = opaque ? ((operr > 0.f) ? 1.f : (operr < 0.f ? -1.f : 0.f)) * inv_nop : 0.f;
  float G[C];
  double acc_los = 0.0;
  float FA = 1.f, FB = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float wg = opaque ? wgt[c] / gt_den : 0.f;
    const float dw = w[c] - wg;
    float gw;
    if (l1) {
      gw = lp.los_lambda * ((dw > 0.f) ? 1.f : (dw < 0.f ? -1.f : 0.f)) * lp.inv_rs;
      acc_los += (double)fabsf(dw);
    } else {
      gw = lp.los_lambda * 2.0f * dw * lp.inv_rs;
      acc_los += (double)(dw * dw);
    }
    G[c] = gw + g_depth * (z[c] - far) + g_op;
  }
#pragma unroll
  for (int c = C - 1; c >= 0; --c) {
    FB = G[c] * alpha[c] + s[c] * FB;
    FA = s[c] * FA;
  }
  const float los = wave_sum((float)acc_los);
  float X = wave_suffix_affine(FA, FB);
  if (a.d_ray) {
    // poses under optimisation (optimizer.py:258-262): the loss's dependence on the ray itself.  deltas =
    // dl * |d| (rendering_tcnn.py:248), so dL/d|d| = sum dA * dl * relu(x) * exp(-delta relu(x)); depth =
    // sum w z + (1 - sum w) far (:274-278), so dL/dfar = g_depth (1 - sum w).  The z are detached
    // (ray_sampling.py:75-90 samples under no_grad).  (A wave-uniform branch: the default step keeps
    // the loop below.)
    double acc_dn = 0.0;
    const float inv_dn = dnorm > 0.f ? 1.0f / dnorm : 0.f;
#pragma unroll
    for (int c = C - 1; c >= 0; --c) {
      const float dA = T[c] * (G[c] - X);
      X = G[c] * alpha[c] + s[c] * X;
      const float sr = fmaxf(x[c], 0.f);
      const float ex = expf(-(delta[c] * sr));
      sig[i0 + c] = (x[c] > 0.f) ? dA * (delta[c] * ex) : 0.f;
      acc_dn += (double)((dA * (ex * sr)) * (delta[c] * inv_dn));
    }
    const float dn = wave_sum((float)acc_dn);
    if (lane == 0) {
      a.d_ray[2 * r + 0] = dn;
      a.d_ray[2 * r + 1] = g_depth * (1.0f - wsum);
    }
  } else {
#pragma unroll
    for (int c = C - 1; c >= 0; --c) {
      const float dA = T[c] * (G[c] - X);
      X = G[c] * alpha[c] + s[c] * X;
      const float sr = fmaxf(x[c], 0.f);
      sig[i0 + c] = (x[c] > 0.f) ? dA * (delta[c] * expf(-(delta[c] * sr))) : 0.f;
    }
  }
  if (a.weights)
#pragma unroll
    for (int c = 0; c < C; ++c) a.weights[r * S + i0 + c] = w[c];
  if (lane == 0) {
    float* st = a.ray_stats + r * LNR_RAY_STATS;
    st[0] = opaque ? ddiff * ddiff : 0.f;
    st[1] = los;
    st[2] = opaque ? fabsf(operr) : 0.f;
    st[3] = eps;
    st[4] = opaque ? 1.f : 0.f;
  }
}

// Phase 1, one wave per ray: sigma MLP forward -> compositing -> loss -> compositing backward;
// writes dL/dsigma (R, S) fp32 for phase 2.
template <int C>
__global__ void __launch_bounds__(NT) k_field_wave(FieldArgs a) {
  if (a.denc_max && blockIdx.x == 0 && threadIdx.x < kSigmaLevels) a.denc_max[threadIdx.x] = 0.f;  // before k_mlp_bwd_tiles
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  constexpr int S = 64 * C;  // == a.S (checked at launch)
  float* sig = reinterpret_cast<float*>(smem) + wid * S;  // this wave's ray: sigma, then dL/dsigma
  SigmaWeights sw;
  load_sigma_weights(a.w, sw);
  for (int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + wid; r < a.n_rays; r += (int64_t)gridDim.x * kWavesPerBlock) {
#pragma unroll 8
    for (int tb = 0; tb < S; tb += 16) {
      SigmaHidden h;
      const float sgm = sigma_tile_fwd(sw, load_enc_operand(a.enc, a.enc_stride, r * S + tb + c, true), h);
      if (g == 0) sig[tb + c] = sigma_to_f16(sgm);
      if (a.lp.dev_status && __any(!isfinite(round_f16(sgm))) && lane == 0) atomicOr(a.lp.dev_status, LNR_STATUS_SIGMA_CLIPPED);
    }
    wave_lds_handoff();
    composite_loss_wave<C>(a, sig, r);
    wave_lds_handoff();
#pragma unroll
    for (int k = 0; k < C; ++k) a.d_sigma[r * S + 64 * k + lane] = sig[64 * k + lane];  // coalesced
    wave_lds_handoff();  // sig is rewritten by the next ray
  }
}

// The same phase split in two, so neither kernel carries the other's registers (k_field_wave<8>: 211
// registers, 2 waves per SIMD, its encoding loads exposed between rays).
// Phase 1a, tile-parallel: sigma MLP forward over 64-sample units (4 tiles per wave trip, every load
// first), sigma (fp16-rounded, as tcnn returns it) into a.d_sigma.
constexpr int kSigmaFwdUnit = 64;
__global__ void __launch_bounds__(NT) k_sigma_fwd_tiles(FieldArgs a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  SigmaWeights sw;
  load_sigma_weights(a.w, sw);
  const int64_t n_units = a.n_rays * (int64_t)a.S / kSigmaFwdUnit;
  for (int64_t u = (int64_t)blockIdx.x * kWavesPerBlock + wid; u < n_units; u += (int64_t)gridDim.x * kWavesPerBlock) {
    const int64_t n0 = u * kSigmaFwdUnit;
    half8_t b[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) b[t] = load_enc_operand(a.enc, a.enc_stride, n0 + 16 * t + c, true);
    bool clipped = false;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      SigmaHidden h;
      const float sgm = sigma_tile_fwd(sw, b[t], h);
      if (g == 0) a.d_sigma[n0 + 16 * t + c] = sigma_to_f16(sgm);
      clipped |= !isfinite(round_f16(sgm));
    }
    if (a.lp.dev_status && __any(clipped) && lane == 0) atomicOr(a.lp.dev_status, LNR_STATUS_SIGMA_CLIPPED);
  }
}

// Early ray termination (lnr_field_sigma_phase).  A sample behind enough opaque ones has transmittance exactly 0
// in the compositing (T = (float) of a double product, rendering_tcnn.py:262-266): its weight alpha T is 0 whatever
// its sigma, so it contributes nothing to the render, the loss or any gradient (dL/dalpha = T (G - X) = 0), and its
// sigma need not be evaluated -- nor its encoding gathered.  The step evaluates a ray in phases of samples [lo, hi):
// after each phase the ray's product of s = 1 - alpha + 1e-10 over its samples so far (the compositing's own
// per-sample float arithmetic, in double); a ray whose product fell below kErtTMin skips the later phases, and its
// later samples' sigma is set to 0 where it falls (the compositing reads it), so alpha there stays finite and T
// stays 0 (s <= 1); the composite kernel itself carries no test for it (a per-sample select there cost 11 us at C4).  The compositing's double products associate differently but agree to ~1e-13 relative, so
// every later sample's float T is 0 there too.  The margin (1e-50 against float's 1.4e-45) also keeps the later
// samples' alpha, which still enters the suffix sums X of the samples before them through factors below 1e-50 / T,
// out of every float result in practice (tests/test_gpu_live.py: bitwise the step without termination).
constexpr double kErtTMin = LNR_ERT_T_MIN;

// The sigma of one phase, one wave per listed ray (list null: every ray; grid-stride, a block past the list leaves
// at once), its 64-sample units in order.  When hi < S the wave also takes the ray's transmittance times the product
// of s over the phase (per lane over its units, then across the lanes; every lane holds the product), and a ray
// that falls below t_min gets sigma 0 at its samples [hi, S) (the compositing's input); keep[e] = r for a surviving
// ray, ~0 for the others (k_ert_compact lists them).  sigma_tile_fwd leaves sample 16 t + c's sigma in every lane c + 16 g, so lane l finds its own sample's in
// tile t = l / 16.
__global__ void __launch_bounds__(NT) k_sigma_phase(FieldArgs a, const uint32_t* __restrict__ list,
                                                    const uint32_t* __restrict__ count, int32_t lo, int32_t hi,
                                                    double* __restrict__ trans, uint32_t* __restrict__ keep,
                                                    double t_min) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  const int S = a.S;
  const bool upd = hi < S;
  const int64_t n_e = list ? (int64_t)count[0] : a.n_rays;
  if ((int64_t)blockIdx.x * kWavesPerBlock >= n_e) return;  // (block-uniform) past the listed rays
  SigmaWeights sw;
  load_sigma_weights(a.w, sw);
  bool clipped = false;
  for (int64_t e = (int64_t)blockIdx.x * kWavesPerBlock + wid; e < n_e; e += (int64_t)gridDim.x * kWavesPerBlock) {
    const int64_t r = list ? (int64_t)list[e] : e;
    const float* ry = a.rays + 13 * r;
    const float dx = ry[3], dy = ry[4], dz = ry[5];
    const float dnorm = sqrtf(dx * dx + dy * dy + dz * dz);
    const float* zr = a.z + r * S;
    const uint32_t gr = (uint32_t)(a.ray_offset + r);
    double P = 1.0;
    for (int u0 = lo; u0 < hi; u0 += kSigmaFwdUnit) {
      const int64_t n0 = r * S + u0;
      half8_t b[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) b[t] = load_enc_operand(a.enc, a.enc_stride, n0 + 16 * t + c, true);
      float mine = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        SigmaHidden h;
        const float sgm = sigma_tile_fwd(sw, b[t], h);
        const float sg16 = sigma_to_f16(sgm);
        if (g == 0) a.d_sigma[n0 + 16 * t + c] = sg16;
        if (g == t) mine = sg16;
        clipped |= !isfinite(round_f16(sgm));
      }
      if (upd) {  // the compositing's per-sample arithmetic (composite_loss_wave)
        const int i = u0 + lane;
        const float zi = zr[i];
        const float dl = (i + 1 < S) ? (zr[i + 1] - zi) : 1e10f;
        const float delta = dl * dnorm;
        float nz = 0.f;
        if (a.noise) nz = a.noise[r * S + i] * a.noise_std;
        else if (a.noise_std > 0.f) nz = rand_normal(step_key_of(a), kStreamNoise, gr, (uint32_t)i) * a.noise_std;
        const float sr = fmaxf(mine + nz, 0.f);
        const float alpha = 1.0f - expf(-(delta * sr));
        P *= (double)((1.0f - alpha) + 1e-10f);
      }
    }
    if (upd) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) P *= __shfl_xor(P, o, 64);
      const double t = (lo == 0 ? 1.0 : trans[r]) * P;  // (every lane: the butterfly left P in all of them)
      const bool al = t >= t_min;
      if (lane == 0) {
        trans[r] = t;
        keep[e] = al ? (uint32_t)r : ~0u;
      }
      if (!al)  // (wave-uniform) terminated here: sigma 0 for the samples no later phase evaluates
        for (int i = hi + lane; i < S; i += 64) a.d_sigma[r * S + i] = 0.f;
    }
  }
  if (a.lp.dev_status && __any(clipped) && lane == 0) atomicOr(a.lp.dev_status, LNR_STATUS_SIGMA_CLIPPED);
}

// The surviving rays of a phase listed in list order: keep[e] (k_sigma_phase) != ~0 over the phase's entries, one
// workgroup, 8 consecutive entries per thread (every load first), a block-wide exclusive scan per 8192 entries.
constexpr int kErtCompactThreads = 1024, kErtCompactPer = 8;
__global__ void __launch_bounds__(kErtCompactThreads) k_ert_compact(const uint32_t* __restrict__ keep,
                                                                     const uint32_t* __restrict__ count_in, int64_t n_rays,
                                                                     uint32_t* __restrict__ list_out,
                                                                     uint32_t* __restrict__ count_out) {
  __shared__ uint32_t wsum[kErtCompactThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int64_t n_e = count_in ? (int64_t)count_in[0] : n_rays;
  uint32_t base = 0;
  for (int64_t c0 = 0; c0 < n_e; c0 += (int64_t)kErtCompactThreads * kErtCompactPer) {
    uint32_t r[kErtCompactPer];
    uint32_t mine = 0;
#pragma unroll
    for (int j = 0; j < kErtCompactPer; ++j) {
      const int64_t e = c0 + (int64_t)t * kErtCompactPer + j;
      r[j] = e < n_e ? keep[e] : ~0u;
    }
#pragma unroll
    for (int j = 0; j < kErtCompactPer; ++j) mine += r[j] != ~0u ? 1u : 0u;
    uint32_t inc = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t off = base + inc - mine, tot = 0;
    for (int w = 0; w < kErtCompactThreads / 64; ++w) {
      const uint32_t v = wsum[w];
      if (w < wid) off += v;
      tot += v;
    }
#pragma unroll
    for (int j = 0; j < kErtCompactPer; ++j)
      if (r[j] != ~0u) list_out[off++] = r[j];
    base += tot;
    __syncthreads();  // wsum is rewritten by the next chunk
  }
  if (t == 0) count_out[0] = base;
}

// Phase 1b, one wave per ray: compositing -> loss -> compositing backward on the sigma of phase 1a,
// dL/dsigma written over it (a.d_sigma, (R, S) fp32).
template <int C>
__global__ void __launch_bounds__(NT) k_composite_wave(FieldArgs a) {
  if (a.denc_max && blockIdx.x == 0 && threadIdx.x < kSigmaLevels) a.denc_max[threadIdx.x] = 0.f;  // before k_mlp_bwd_tiles
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int S = 64 * C;  // == a.S (checked at launch)
  float* sig = reinterpret_cast<float*>(smem) + wid * S;
  for (int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + wid; r < a.n_rays; r += (int64_t)gridDim.x * kWavesPerBlock) {
    // (early ray termination: the samples from term[r] on were not evaluated, their sigma is 0)
#pragma unroll
    for (int k = 0; k < C; ++k) sig[64 * k + lane] = a.d_sigma[r * S + 64 * k + lane];  // coalesced
    wave_lds_handoff();
    composite_loss_wave<C>(a, sig, r);
    wave_lds_handoff();
#pragma unroll
    for (int k = 0; k < C; ++k) a.d_sigma[r * S + 64 * k + lane] = sig[64 * k + lane];
    wave_lds_handoff();  // sig is rewritten by the next ray
  }
}

// Element access at a 32-bit byte offset from a (uniform) base pointer
template <class T>
__device__ __forceinline__ T ld_off(const T* base, uint32_t byte_off) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}
template <class T>
__device__ __forceinline__ void st_off(T* base, uint32_t byte_off, T v) {
  *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + byte_off) = v;
}

// fp16 pair (round to nearest) in one word, low half first
__device__ __forceinline__ uint32_t pack_h2(float x, float y) {
  const half2v_t h = {(_Float16)x, (_Float16)y};  // (one v_cvt_pk_f16_f32)
  return __builtin_bit_cast(uint32_t, h);
}

// Packed-half pair for k_mlp_bwd_tiles (LNR_MLP_PK): the hidden layer kept as 8 fp16-pair words per tile
// (v_cvt_pk + v_pk_max: the ReLU of the rounded value), the ReLU masks taken from those words by integer ops
// (pk_nonzero_mask), and dW0's operands staged as [sample][neuron] rows of 8-byte chunks read back transposed
// (ds_read_b64_tr_b16) instead of one 2-byte LDS store per value.  Same operands at the same MFMA k
// positions as dw0_pair_mfma (the k order matters: tools/ubench/ubench_mfma_korder.hip), bitwise the same sums
// except where the scaled ds * Enc operand rounds a tie differently (below).
// Wave image of a pair: the ReLU mask (1.0 / 0.0), 32 sample rows x 16 chunks (64 hid), and ds * Enc at the
// pair's scale, 32 rows x 8 chunks (32 inputs).  Chunk swizzles (MI355X_MICROARCH.md LDS table: stores bank
// on (a/4) mod 32 in 16-lane groups for b64 and 8-lane groups for b128, the transposed reads on (a/4) mod 64 in
// 32-lane halves): a store instruction's 16 rows of one chunk, or 8 rows of one 16-byte chunk pair, and a
// transposed read's rows 8g + q (g = 0, 1 or 2, 3; q = 0..3 or 4..7) x 4 chunks all meet distinct banks.
// Mask image: chunk ch of row r at ch ^ f(r), f = the bits (r3, r1, r2, r0) of r mod 16 (r3 r1 set the chunk's
// 4-group for the reads, the whole permutation spreads the stores); ds * Enc image: ch ^ (2 r1 + 4 (r2 ^ r3)).
__device__ __forceinline__ uint32_t mk_dw(uint32_t r, uint32_t ch) {
  const uint32_t f = (((r >> 3) & 1u) << 3) | (((r >> 1) & 1u) << 2) | (((r >> 2) & 1u) << 1) | (r & 1u);
  return 32u * r + 2u * (ch ^ f);
}
__device__ __forceinline__ uint32_t en_dw(uint32_t r, uint32_t ch) {
  return 1024u + 16u * r + 2u * (ch ^ ((((r >> 1) & 1u) << 1) | ((((r >> 2) ^ (r >> 3)) & 1u) << 2)));
}
// forward of one tile: hw[2t + (r >> 1)] holds relu(H)[hid 16t + 4g + r] (r = 0..3) for sample l & 15
template <class W>
__device__ __forceinline__ void sigma_tile_fwd_pk(const W& sw, const uint32_t (&x)[4], uint32_t (&hw)[8]) {
  const half8_t e = __builtin_bit_cast(half8_t, (u32x4){x[0], x[1], x[2], x[3]});
  float4_t acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(sw.A0(t), e, (float4_t){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    hw[2 * t] = pk_relu(acc[t][0], acc[t][1]);
    hw[2 * t + 1] = pk_relu(acc[t][2], acc[t][3]);
  }
}
// max |e_j| over a tile's 8 encoding halves (non-negative halves order as their bits), as fp32
__device__ __forceinline__ float enc_absmax(const uint32_t (&x)[4]) {
  u16x2v_t m = __builtin_bit_cast(u16x2v_t, x[0] & 0x7FFF7FFFu);
#pragma unroll
  for (int q = 1; q < 4; ++q) m = __builtin_elementwise_max(m, __builtin_bit_cast(u16x2v_t, x[q] & 0x7FFF7FFFu));
  return h2f(m[0] > m[1] ? m[0] : m[1]);
}

// Phase 2, tile-parallel: sigma MLP backward over 32-sample tile pairs (no per-ray structure):
// d_enc (level-major float2) and the per-block dW slab.
// (2 waves per SIMD at its 242 VGPRs; forcing 3 or 4 spills 45 / 116 VGPRs: 0.18 -> 0.56 / 0.76 ms)
#ifndef LNR_MLP_PREFETCH
#define LNR_MLP_PREFETCH 1  // tile pairs loaded ahead in k_mlp_bwd_tiles (1 or 2; C2: 271 against 279 us)
#endif
#ifndef LNR_MLP_W_LDS
#define LNR_MLP_W_LDS 0  // the layer-0 weight operands in LDS instead of registers (k_mlp_bwd_tiles)
#endif
#ifndef LNR_MLP_SPLIT_PAIR
#define LNR_MLP_SPLIT_PAIR 0  // k_mlp_bwd_tiles: one tile of the pair live at a time (pair_split)
#endif
#ifndef LNR_MLP_PK
#define LNR_MLP_PK 1  // k_mlp_bwd_tiles: the packed-half pair (pair_pk)
#endif
#ifndef LNR_MLP_BWD_WAVES
#define LNR_MLP_BWD_WAVES 2  // waves per SIMD (3 spills 113 registers with the weights in registers)
#endif
template <bool JAC>  // JAC: write d sigma / d enc (fp16 pairs) instead of d_enc
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(LNR_MLP_BWD_WAVES, LNR_MLP_BWD_WAVES))) k_mlp_bwd_tiles(FieldArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  _Float16* lds = reinterpret_cast<_Float16*>(smem) + wid * (64 * 32 + 32 * 32);
#if LNR_MLP_W_LDS
  SigmaWeightsLds sw;
  {
    SigmaWeights swr;
    load_sigma_weights(a.w, swr);
    sw.stage(reinterpret_cast<half8_t*>(reinterpret_cast<_Float16*>(smem) + kWavesPerBlock * (64 * 32 + 32 * 32)), swr);
  }
  __syncthreads();
#else
  SigmaWeights sw;
  load_sigma_weights(a.w, sw);
#endif
  DW0Mfma acc;
  acc.init();
  float dw1[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) dw1[k] = 0.f;
  float2* denc = reinterpret_cast<float2*>(a.d_enc);
  float lmax[4] = {0.f, 0.f, 0.f, 0.f};  // max |d_enc| of this lane's levels 2g, 2g + 1, 8 + 2g, 9 + 2g
  const int64_t N = a.n_rays * (int64_t)a.S;  // a multiple of 64
  // software-pipelined two tile pairs deep: the loads of the next two pairs (enc, dsigma) are in flight
  // while this one computes (2 waves per SIMD at this register count: latency is hidden by ILP)
  const int64_t step = (int64_t)gridDim.x * kWavesPerBlock * 32;
  int64_t n0 = ((int64_t)blockIdx.x * kWavesPerBlock + wid) * 32;
  struct Pre {
    uint32_t x0[4], x1[4];
    float d0, d1;
  };
  // 32-bit byte offsets from uniform bases (the launcher checks 16 levels x stride x 4 B < 4 GB): one
  // register per address instead of a 64-bit pair, and no hoisted per-level 64-bit row addresses
  const uint32_t st4 = (uint32_t)a.enc_stride * 4u;
  const uint32_t row_e = 4u * (uint32_t)g * st4, row_j = 2u * (uint32_t)g * st4;  // this lane group's rows
  auto prefetch = [&](int64_t m, Pre& p) {
    const uint32_t mb = (uint32_t)((m < N ? m : 0) + c) * 4u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      p.x0[q] = ld_off(a.enc, row_e + (uint32_t)q * st4 + mb);
      p.x1[q] = ld_off(a.enc, row_e + (uint32_t)q * st4 + mb + 64u);
    }
    p.d0 = ld_off(a.d_sigma, mb);
    p.d1 = ld_off(a.d_sigma, mb + 64u);
  };
  auto pair = [&](int64_t n0, const Pre& p) {
    SigmaHidden h0, h1;
    half8_t e0, e1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      e0[2 * q + 0] = __builtin_bit_cast(_Float16, (uint16_t)(p.x0[q] & 0xFFFFu));
      e0[2 * q + 1] = __builtin_bit_cast(_Float16, (uint16_t)(p.x0[q] >> 16));
      e1[2 * q + 0] = __builtin_bit_cast(_Float16, (uint16_t)(p.x1[q] & 0xFFFFu));
      e1[2 * q + 1] = __builtin_bit_cast(_Float16, (uint16_t)(p.x1[q] >> 16));
    }
    const float ds0 = p.d0, ds1 = p.d1;
    (void)sigma_tile_fwd(sw, e0, h0);
    (void)sigma_tile_fwd(sw, e1, h1);
    float mx = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      dw1[k] = fmaf(ds0, h0[k], dw1[k]);
      dw1[k] = fmaf(ds1, h1[k], dw1[k]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fmaxf(fabsf((float)e0[j] * ds0), fabsf((float)e1[j] * ds1)));
    const float pair_max = wave_max(mx);
    float d[2][4];
    sigma_tile_bwd_denc(sw, h0, d);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int lvl = 8 * m + 2 * g;
      const float2 q0 = make_float2(d[m][0] * ds0, d[m][1] * ds0), q1 = make_float2(d[m][2] * ds0, d[m][3] * ds0);
      if (JAC) {
        const uint32_t o = row_j + 8u * (uint32_t)m * st4 + (uint32_t)(n0 + c) * 4u;
        st_off(a.d_jac, o, pack_h2(d[m][0], d[m][1]));
        st_off(a.d_jac, o + st4, pack_h2(d[m][2], d[m][3]));
      } else {
        denc[(int64_t)lvl * a.enc_stride + n0 + c] = q0;
        denc[(int64_t)(lvl + 1) * a.enc_stride + n0 + c] = q1;
      }
      lmax[2 * m] = fmaxf(lmax[2 * m], fmaxf(fabsf(q0.x), fabsf(q0.y)));
      lmax[2 * m + 1] = fmaxf(lmax[2 * m + 1], fmaxf(fabsf(q1.x), fabsf(q1.y)));
    }
    sigma_tile_bwd_denc(sw, h1, d);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int lvl = 8 * m + 2 * g;
      const float2 q0 = make_float2(d[m][0] * ds1, d[m][1] * ds1), q1 = make_float2(d[m][2] * ds1, d[m][3] * ds1);
      if (JAC) {
        const uint32_t o = row_j + 8u * (uint32_t)m * st4 + (uint32_t)(n0 + 16 + c) * 4u;
        st_off(a.d_jac, o, pack_h2(d[m][0], d[m][1]));
        st_off(a.d_jac, o + st4, pack_h2(d[m][2], d[m][3]));
      } else {
        denc[(int64_t)lvl * a.enc_stride + n0 + 16 + c] = q0;
        denc[(int64_t)(lvl + 1) * a.enc_stride + n0 + 16 + c] = q1;
      }
      lmax[2 * m] = fmaxf(lmax[2 * m], fmaxf(fabsf(q0.x), fabsf(q0.y)));
      lmax[2 * m + 1] = fmaxf(lmax[2 * m + 1], fmaxf(fabsf(q1.x), fabsf(q1.y)));
    }
    dw0_pair_mfma(lds, h0, h1, e0, e1, ds0, ds1, pair_max, acc);
  };
  // the same pair with one tile live at a time: the pair's operand scale first (from the inputs), then
  // per tile the forward, dW1, its dW0 operands staged in LDS, its d_enc; the dW0 MFMAs last
  auto pair_split = [&](int64_t n0, const Pre& p) {
    float mx = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float a0 = (float)__builtin_bit_cast(_Float16, (uint16_t)(p.x0[q] & 0xFFFFu));
      const float b0 = (float)__builtin_bit_cast(_Float16, (uint16_t)(p.x0[q] >> 16));
      const float a1 = (float)__builtin_bit_cast(_Float16, (uint16_t)(p.x1[q] & 0xFFFFu));
      const float b1 = (float)__builtin_bit_cast(_Float16, (uint16_t)(p.x1[q] >> 16));
      mx = fmaxf(mx, fmaxf(fabsf(a0 * p.d0), fabsf(a1 * p.d1)));
      mx = fmaxf(mx, fmaxf(fabsf(b0 * p.d0), fabsf(b1 * p.d1)));
    }
    float scale = 1.f;
    const bool dw0 = dw0_scale(wave_max(mx), acc, scale);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      half8_t e;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t x = t ? p.x1[q] : p.x0[q];
        e[2 * q + 0] = __builtin_bit_cast(_Float16, (uint16_t)(x & 0xFFFFu));
        e[2 * q + 1] = __builtin_bit_cast(_Float16, (uint16_t)(x >> 16));
      }
      const float ds = t ? p.d1 : p.d0;
      SigmaHidden h;
      (void)sigma_tile_fwd(sw, e, h);
#pragma unroll
      for (int k = 0; k < 16; ++k) dw1[k] = fmaf(ds, h[k], dw1[k]);
      if (dw0) dw0_stage(lds, t, h, e, ds * scale);
      float d[2][4];
      sigma_tile_bwd_denc(sw, h, d);
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int lvl = 8 * m + 2 * g;
        const float2 q0 = make_float2(d[m][0] * ds, d[m][1] * ds), q1 = make_float2(d[m][2] * ds, d[m][3] * ds);
        if (JAC) {
          const uint32_t o = row_j + 8u * (uint32_t)m * st4 + (uint32_t)(n0 + 16 * t + c) * 4u;
          st_off(a.d_jac, o, pack_h2(d[m][0], d[m][1]));
          st_off(a.d_jac, o + st4, pack_h2(d[m][2], d[m][3]));
        } else {
          denc[(int64_t)lvl * a.enc_stride + n0 + 16 * t + c] = q0;
          denc[(int64_t)(lvl + 1) * a.enc_stride + n0 + 16 * t + c] = q1;
        }
        lmax[2 * m] = fmaxf(lmax[2 * m], fmaxf(fabsf(q0.x), fabsf(q0.y)));
        lmax[2 * m + 1] = fmaxf(lmax[2 * m + 1], fmaxf(fabsf(q1.x), fabsf(q1.y)));
      }
    }
    if (dw0) dw0_mfma(lds, acc);
  };
  auto pair_pk = [&](int64_t n0, const Pre& p) {
    uint32_t hw[2][8];
    sigma_tile_fwd_pk(sw, p.x0, hw[0]);
    sigma_tile_fwd_pk(sw, p.x1, hw[1]);
    const float ds[2] = {p.d0, p.d1};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float h0 = (k & 1) ? pk_hi(hw[0][k >> 1]) : pk_lo(hw[0][k >> 1]);
      const float h1 = (k & 1) ? pk_hi(hw[1][k >> 1]) : pk_lo(hw[1][k >> 1]);
      dw1[k] = fmaf(ds[0], h0, dw1[k]);
      dw1[k] = fmaf(ds[1], h1, dw1[k]);
    }
    // max |e ds| over the pair: |ds| max |e| (rounding is monotonic: the same value)
    // (on DPP, wave-uniform; the same value as dw0_pair_mfma's wave_max for finite inputs)
    const float pair_max = wave_max_nonneg(fmaxf(enc_absmax(p.x0) * fabsf(ds[0]), enc_absmax(p.x1) * fabsf(ds[1])));
    const uint32_t* w1w = reinterpret_cast<const uint32_t*>(&sw.w1h[0]);
    uint32_t mk[2][8];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int i = 0; i < 8; ++i) mk[t][i] = pk_nonzero_mask(hw[t][i]);
      uint32_t bw[8];  // the backward's B operand: w1 where the hidden unit is live
#pragma unroll
      for (int i = 0; i < 8; ++i) bw[i] = mk[t][i] & w1w[i];
      const half8_t b0 = __builtin_bit_cast(half8_t, (u32x4){bw[0], bw[1], bw[2], bw[3]});
      const half8_t b1 = __builtin_bit_cast(half8_t, (u32x4){bw[4], bw[5], bw[6], bw[7]});
      const float dst = ds[t];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        float4_t acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(sw.BT(m, 0), b0, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(sw.BT(m, 1), b1, acc, 0, 0, 0);
        const int lvl = 8 * m + 2 * g;
        if (JAC) {
          const uint32_t o = row_j + 8u * (uint32_t)m * st4 + (uint32_t)(n0 + 16 * t + c) * 4u;
          st_off(a.d_jac, o, pack_h2(acc[0], acc[1]));
          st_off(a.d_jac, o + st4, pack_h2(acc[2], acc[3]));
          // max |d ds| = |ds| max |d| (monotonic rounding)
          const float ads = fabsf(dst);
          lmax[2 * m] = fmaxf(lmax[2 * m], fmaxf(fabsf(acc[0]), fabsf(acc[1])) * ads);
          lmax[2 * m + 1] = fmaxf(lmax[2 * m + 1], fmaxf(fabsf(acc[2]), fabsf(acc[3])) * ads);
        } else {
          const float2 q0 = make_float2(acc[0] * dst, acc[1] * dst), q1 = make_float2(acc[2] * dst, acc[3] * dst);
          denc[(int64_t)lvl * a.enc_stride + n0 + 16 * t + c] = q0;
          denc[(int64_t)(lvl + 1) * a.enc_stride + n0 + 16 * t + c] = q1;
          lmax[2 * m] = fmaxf(lmax[2 * m], fmaxf(fabsf(q0.x), fabsf(q0.y)));
          lmax[2 * m + 1] = fmaxf(lmax[2 * m + 1], fmaxf(fabsf(q1.x), fabsf(q1.y)));
        }
      }
    }
#ifdef LNR_MLP_PK_OLDDW0
    {
      SigmaHidden H[2];
      half8_t E[2];
      for (int t = 0; t < 2; ++t) {
        H[t].q[0] = __builtin_bit_cast(half8_t, (u32x4){hw[t][0], hw[t][1], hw[t][2], hw[t][3]});
        H[t].q[1] = __builtin_bit_cast(half8_t, (u32x4){hw[t][4], hw[t][5], hw[t][6], hw[t][7]});
        const uint32_t* x = t ? p.x1 : p.x0;
        E[t] = __builtin_bit_cast(half8_t, (u32x4){x[0], x[1], x[2], x[3]});
      }
      dw0_pair_mfma(lds, H[0], H[1], E[0], E[1], ds[0], ds[1], pair_max, acc);
      return;
    }
#endif
    float scale = 1.f;
    if (!dw0_scale(pair_max, acc, scale)) return;  // (wave-uniform) the pair adds nothing to dW0
    uint32_t* img = reinterpret_cast<uint32_t*>(lds);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint32_t r = 16u * t + c;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)  // hid 16 tt + 4 g .. + 3: chunk 4 tt + g
        *reinterpret_cast<u32x2*>(&img[mk_dw(r, 4u * tt + g)]) =
            (u32x2){mk[t][2 * tt] & 0x3C003C00u, mk[t][2 * tt + 1] & 0x3C003C00u};
      const float st = ds[t] * scale;
      const uint32_t* x = t ? p.x1 : p.x0;
      // (fp32 product, then rounded to fp16, as written: dw0_pair_mfma's same expression compiles to v_fma_mixlo,
      // one rounding of the exact product, so a rare tie rounds differently there: tools/mlp_bwd_dump.py)
      const half8_t e = __builtin_bit_cast(half8_t, (u32x4){x[0], x[1], x[2], x[3]});
      half8_t es;
#pragma unroll
      for (int j = 0; j < 8; ++j) es[j] = (_Float16)((float)e[j] * st);
      *reinterpret_cast<half8_t*>(&img[en_dw(r, 2u * g)]) = es;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-local hand-off through LDS
    __builtin_amdgcn_wave_barrier();
    const uint32_t tq = ((uint32_t)lane >> 2) & 3u, tp = (uint32_t)lane & 3u;
    const uint32_t r0 = 8u * g + tq;
    half8_t av[4], bv[2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const half4_t lo = lds_tr16(&img[mk_dw(r0, 4u * t + tp)]), hi = lds_tr16(&img[mk_dw(r0 + 4u, 4u * t + tp)]);
      av[t] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const half4_t lo = lds_tr16(&img[en_dw(r0, 4u * m + tp)]), hi = lds_tr16(&img[en_dw(r0 + 4u, 4u * m + tp)]);
      bv[m] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int m = 0; m < 2; ++m) acc.v[t][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[t], bv[m], acc.v[t][m], 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  };
#if LNR_MLP_PK
#define LNR_MLP_PAIR pair_pk
#elif LNR_MLP_SPLIT_PAIR
#define LNR_MLP_PAIR pair_split
#else
#define LNR_MLP_PAIR pair
#endif
#if LNR_MLP_PREFETCH == 2
  Pre pa, pb;
  prefetch(n0, pa);
  prefetch(n0 + step, pb);
  for (; n0 < N; n0 += 2 * step) {
    {
      const Pre cur = pa;
      prefetch(n0 + 2 * step, pa);
      LNR_MLP_PAIR(n0, cur);
    }
    if (n0 + step < N) {  // (wave-uniform)
      const Pre cur = pb;
      prefetch(n0 + 3 * step, pb);
      LNR_MLP_PAIR(n0 + step, cur);
    }
  }
#else
  // A pair whose 32 d sigma are all 0 (relu(sigma + noise) = 0 for every sample: most pairs of a trained field's
  // free space) adds exact zeros to dW1 and to the level maxima and nothing to dW0 (dw0_scale refuses a zero
  // pair_max), and its d_enc is 0: it is skipped, its encodings not even loaded and its J not written (consumers
  // form d sigma * J as 0 there, hashgrid.hpp GradJac).  The wave finds its live pairs 16 at a time (lane l reads 8
  // of pair l / 4's d sigma: one load round trip per 16 pairs, not per pair) and walks them with the next live
  // pair's loads in flight during this one's work.
  // Round k of the walk gives wave w the pair k W + (w + 7 k) mod W (W waves): every round still covers W
  // consecutive pairs once, but a wave's position within the rays (16 pairs of 512 samples) changes from round to
  // round.  With the plain k W + w (W a multiple of 16) a wave met one position in every ray, and the live pairs,
  // which sit at the positions near the surfaces, went to a few waves (C2 trained: 74 us for 21 % live pairs).
  const int64_t W = (int64_t)gridDim.x * kWavesPerBlock, w0 = (int64_t)blockIdx.x * kWavesPerBlock + wid;
  const int64_t npairs = N / 32;
  auto pair_at = [&](int64_t k) { return 32 * (k * W + (w0 + 7 * k) % W); };  // its first sample
  int64_t lb = -16;  // the wave's current batch of 16 rounds
  uint32_t pm = 0u;  // its live pairs not yet taken
  auto next_live = [&]() -> int64_t {
    while (pm == 0u) {
      lb += 16;
      if (lb * W >= npairs) return -1;  // (wave-uniform)
      const int64_t m = pair_at(lb + (lane >> 2));
      bool lv = false;
      if (m < N) {
        const float* dp = a.d_sigma + m + 8 * (lane & 3);
#pragma unroll
        for (int k = 0; k < 8; ++k) lv = lv || dp[k] != 0.f;
      }
      const unsigned long long bl = __ballot(lv);
      uint32_t q = 0u;
#pragma unroll
      for (int j = 0; j < 16; ++j) q |= ((bl >> (4 * j)) & 0xFull) ? (1u << j) : 0u;
      pm = q;
    }
    const int j = __builtin_ctz(pm);
    pm &= pm - 1u;
    return pair_at(lb + j);
  };
  Pre pa{};
  int64_t nm = next_live();
  if (nm >= 0) prefetch(nm, pa);
  while (nm >= 0) {
    const Pre cur = pa;
    const int64_t m = nm;
    nm = next_live();
    if (nm >= 0) prefetch(nm, pa);
    LNR_MLP_PAIR(m, cur);
  }
#endif
#undef LNR_MLP_PAIR
  __syncthreads();
  {
    DW0Acc out;
    acc.finish(sw, out);
    write_dw_slab<NT>(reinterpret_cast<float*>(smem), out, dw1, a.dw_slab + (int64_t)blockIdx.x * LNR_SIGMA_MLP_PARAMS);
  }
  if (a.denc_max) {  // the level maxima (hash-grid backward record scales): 16-lane row max, then the block's
    __shared__ float bm[kWavesPerBlock][kSigmaLevels];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = lmax[q];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
      if (c == 0) bm[wid][(q >> 1) * 8 + 2 * g + (q & 1)] = v;
    }
    __syncthreads();
    if (threadIdx.x < kSigmaLevels) {
      float v = 0.f;
      for (int w = 0; w < kWavesPerBlock; ++w) v = fmaxf(v, bm[w][threadIdx.x]);
      if (v > 0.f) atomicMax(reinterpret_cast<uint32_t*>(a.denc_max) + threadIdx.x, __float_as_uint(v));
    }
  }
}

// max |d_enc| per level for the per-ray field path (grid (256, 16), zeroed before)
__global__ void __launch_bounds__(256) k_denc_max(const float2* __restrict__ d_enc, int64_t stride, int64_t n,
                                                  float* __restrict__ out) {
  __shared__ float red[4];
  const float2* src = d_enc + (int64_t)blockIdx.y * stride;
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float2 q = src[i];
    m = fmaxf(m, fmaxf(fabsf(q.x), fabsf(q.y)));
  }
  m = wave_max_nonneg(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (m > 0.f) atomicMax(reinterpret_cast<uint32_t*>(out) + blockIdx.y, __float_as_uint(m));
  }
}

static size_t wave_smem_bytes(int S) { return (size_t)kWavesPerBlock * S * 4; }
static size_t bwd_tiles_smem_bytes() {
  // per-wave dW0 staging, then (LNR_MLP_W_LDS) the 8 weight operands x 64 lanes x 16 B
  const size_t b = (size_t)kWavesPerBlock * (64 * 32 + 32 * 32) * 2 + (LNR_MLP_W_LDS ? 8 * 64 * 16 : 0);
  return b < LNR_SIGMA_MLP_PARAMS * 4 ? LNR_SIGMA_MLP_PARAMS * 4 : b;
}

constexpr int kReduceThreads = 1024;  // single-workgroup reductions over rays: latency, not bandwidth

// lnr_loss_finalize's body (one workgroup of kReduceThreads): per-ray partials -> the loss scalars
__device__ __forceinline__ void loss_finalize_block(const float* __restrict__ st, int64_t n, const lnr_loss_params& lp_in,
                                                    float* out) {
  const lnr_loss_params lp = step_lp(lp_in);
  __shared__ float red[5 * kReduceThreads / 64];
  double a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0;
  for (int64_t r = threadIdx.x; r < n; r += blockDim.x) {
    const float* s = st + r * LNR_RAY_STATS;
    a0 += s[0];
    a1 += s[1];
    a2 += s[2];
    a3 += s[3];
    a4 += s[4];
  }
  float v[5] = {(float)a0, (float)a1, (float)a2, (float)a3, (float)a4};
  block_sum<kReduceThreads, 5>(v, red);
  if (threadIdx.x == 0) {
    const float inv_nop = lp.dev_n_opaque ? 1.0f / fmaxf(lp.dev_n_opaque[0], 1.0f) : lp.inv_n_opaque;
    const float dterm = v[0] * inv_nop;
    const float lterm = v[1] * lp.inv_rs;
    const float oterm = v[2] * inv_nop;
    out[0] = lp.depthloss_lambda * dterm + lp.los_lambda * lterm + oterm;
    if (lp.dev_status) {
      const uint32_t bits = (isnan(out[0]) ? LNR_STATUS_NAN_LOSS : 0u) | (isinf(out[0]) ? LNR_STATUS_INF_LOSS : 0u);
      if (bits) atomicOr(lp.dev_status, bits);
    }
    out[1] = n > 0 ? v[3] / (float)n : 0.f;
    out[2] = dterm;
    out[3] = lterm;
    out[4] = oterm;
    out[5] = v[4];
  }
}

// dW (+)= the per-workgroup slabs, fixed summation order (mlp.hpp reduce_slabs_fixed).  With
// lp.dev_loss_out, one more workgroup (the last) finalizes the loss from the per-ray partials.
static_assert(64 * kSlabWaves == kReduceThreads, "the loss-finalize workgroup shares the launch shape");
__global__ void __launch_bounds__(64 * kSlabWaves) k_reduce_slabs(const float* __restrict__ slab, int nb, float* __restrict__ dw,
                                                                  bool overwrite, const float* __restrict__ ray_stats,
                                                                  int64_t n_rays, lnr_loss_params lp) {
  if (blockIdx.x == (LNR_SIGMA_MLP_PARAMS + 63) / 64) {
    loss_finalize_block(ray_stats, n_rays, lp, lp.dev_loss_out);
    return;
  }
  reduce_slabs_fixed(slab, nb, dw, overwrite);
}

__global__ void __launch_bounds__(kReduceThreads) k_loss_finalize(const float* __restrict__ st, int64_t n,
                                                                  lnr_loss_params lp, float* out) {
  loss_finalize_block(st, n, lp, out);
}

static int chunk_for(int S) {
  int c = (S + NT - 1) / NT;
  int p = 1;
  while (p < c) p <<= 1;
  return p;
}

static size_t smem_bytes(int S, bool mlp_train) {
  size_t b = ((size_t)S * 4 + 15) / 16 * 16 + 16 * NW * 4 + NW * 8 + 2 * NW * 4 + NT * 4 + 16;
  b = (b + 15) / 16 * 16;
  if (mlp_train) b += (size_t)NW * (64 * 32 + 32 * 32) * 2;
  if (mlp_train && b < LNR_SIGMA_MLP_PARAMS * 4) b = LNR_SIGMA_MLP_PARAMS * 4;
  return b;
}

template <bool TRAIN, bool ADJ, int SRC>
static int launch_field(const FieldArgs& a, int nblocks, hipStream_t st, const char* who) {
  const int C = chunk_for(a.S);
  const size_t sm = smem_bytes(a.S, SRC == kSigmaMLP && TRAIN);
  dim3 grid(nblocks), block(NT);
  switch (C) {
    case 1: hipLaunchKernelGGL((k_field<1, TRAIN, ADJ, SRC>), grid, block, sm, st, a); break;
    case 2: hipLaunchKernelGGL((k_field<2, TRAIN, ADJ, SRC>), grid, block, sm, st, a); break;
    case 4: hipLaunchKernelGGL((k_field<4, TRAIN, ADJ, SRC>), grid, block, sm, st, a); break;
    case 8: hipLaunchKernelGGL((k_field<8, TRAIN, ADJ, SRC>), grid, block, sm, st, a); break;
    case 16: hipLaunchKernelGGL((k_field<16, TRAIN, ADJ, SRC>), grid, block, sm, st, a); break;
    default: set_error("%s: n_samples=%d too large (max 4096)", who, a.S); return LNR_ERR_ARG;
  }
  LNR_RETURN_LAUNCH(who);
}

static int field_blocks(int64_t n_rays) { return (int)(n_rays < 1024 ? n_rays : 1024); }

}  // namespace lnr

using namespace lnr;

extern "C" int64_t lnr_dw_workspace_words(int64_t n_rows) {
  int64_t nb = n_rows < 1024 ? n_rows : 1024;
  if (nb < 1) nb = 1;
  return nb * LNR_SIGMA_MLP_PARAMS;
}

extern "C" int64_t lnr_field_train_workspace_words(int64_t n_rays, int32_t n_samples) {
  if (n_rays < 0 || n_samples < 0) return -1;
  return lnr_dw_workspace_words(n_rays) + n_rays * (int64_t)n_samples;
}

static int check_rays(const float* rays, const float* z, int64_t n_rays, int32_t S, const char* who) {
  LNR_REQUIRE(n_rays >= 0, "%s: n_rays=%lld", who, (long long)n_rays);
  LNR_REQUIRE(S >= 2 && S <= 4096, "%s: n_samples=%d not in [2,4096]", who, S);
  LNR_REQUIRE(n_rays == 0 || (rays && z), "%s: null rays/z", who);
  return LNR_OK;
}

extern "C" int lnr_composite(const float* rays, const float* z, const float* sigma, int64_t n_rays, int32_t n_samples,
                             int32_t strategy, float noise_std, const float* noise, uint32_t key, int64_t ray_offset,
                             float* weights, float* depth, float* opacity, float* variance, void* stream) {
  if (int e = check_rays(rays, z, n_rays, n_samples, "lnr_composite")) return e;
  LNR_REQUIRE(strategy == LNR_RENDER_DEFAULT || strategy == LNR_RENDER_ADJUSTED,
              "Unknown render strategy: %d", strategy);  // rendering_tcnn.py:403-404 raises ValueError
  if (n_rays == 0) return LNR_OK;
  LNR_REQUIRE(sigma && depth, "lnr_composite: null sigma/depth");
  FieldArgs a{};
  a.rays = rays; a.z = z; a.sigma_in = sigma; a.n_rays = n_rays; a.S = n_samples;
  a.noise_std = noise_std; a.noise = noise; a.key = key; a.ray_offset = ray_offset;
  a.weights = weights; a.depth = depth; a.opacity = opacity; a.variance = variance;
  const int nb = field_blocks(n_rays);
  if (strategy == LNR_RENDER_ADJUSTED)
    return launch_field<false, true, kSigmaGiven>(a, nb, as_stream(stream), "lnr_composite");
  return launch_field<false, false, kSigmaGiven>(a, nb, as_stream(stream), "lnr_composite");
}

static int check_lp(const lnr_loss_params* lp, const char* who) {
  LNR_REQUIRE(lp != nullptr, "%s: null loss params", who);
  LNR_REQUIRE(lp->kind >= 0 && lp->kind <= 3, "Can't use unknown Loss %d", lp->kind);
  return LNR_OK;
}

extern "C" int lnr_composite_loss_bwd(const float* rays, const float* z, const float* sigma, const float* depth_gt,
                                      int64_t n_rays, int32_t n_samples, float noise_std, const float* noise,
                                      uint32_t key, int64_t ray_offset, const lnr_loss_params* lp, float* weights,
                                      float* depth, float* opacity, float* d_sigma, float* ray_stats, void* stream) {
  if (int e = check_rays(rays, z, n_rays, n_samples, "lnr_composite_loss_bwd")) return e;
  if (int e = check_lp(lp, "lnr_composite_loss_bwd")) return e;
  if (n_rays == 0) return LNR_OK;
  LNR_REQUIRE(sigma && depth_gt && d_sigma && ray_stats, "lnr_composite_loss_bwd: null pointer");
  FieldArgs a{};
  a.rays = rays; a.z = z; a.sigma_in = sigma; a.depth_gt = depth_gt; a.n_rays = n_rays; a.S = n_samples;
  a.noise_std = noise_std; a.noise = noise; a.key = key; a.ray_offset = ray_offset; a.lp = *lp;
  a.weights = weights; a.depth = depth; a.opacity = opacity; a.d_sigma = d_sigma; a.ray_stats = ray_stats;
  return launch_field<true, false, kSigmaGiven>(a, field_blocks(n_rays), as_stream(stream), "lnr_composite_loss_bwd");
}

extern "C" int lnr_composite_bwd(const float* rays, const float* z, const float* sigma, int64_t n_rays,
                                 int32_t n_samples, int32_t strategy, float noise_std, const float* noise, uint32_t key,
                                 int64_t ray_offset, const float* g_weights, const float* g_depth,
                                 const float* g_opacity, const float* g_variance, float* d_sigma, float* d_ray,
                                 void* stream) {
  if (int e = check_rays(rays, z, n_rays, n_samples, "lnr_composite_bwd")) return e;
  LNR_REQUIRE(strategy == LNR_RENDER_DEFAULT || strategy == LNR_RENDER_ADJUSTED,
              "Unknown render strategy: %d", strategy);
  if (n_rays == 0) return LNR_OK;
  LNR_REQUIRE(sigma && d_sigma, "lnr_composite_bwd: null sigma/d_sigma");
  FieldArgs a{};
  a.rays = rays; a.z = z; a.sigma_in = sigma; a.n_rays = n_rays; a.S = n_samples;
  a.noise_std = noise_std; a.noise = noise; a.key = key; a.ray_offset = ray_offset;
  a.lp.kind = kLossExternal;
  a.g_weights = g_weights; a.g_depth = g_depth; a.g_opacity = g_opacity; a.g_variance = g_variance;
  a.d_sigma = d_sigma;
  a.d_ray = d_ray;
  const int nb = field_blocks(n_rays);
  if (strategy == LNR_RENDER_ADJUSTED)
    return launch_field<true, true, kSigmaGiven>(a, nb, as_stream(stream), "lnr_composite_bwd");
  return launch_field<true, false, kSigmaGiven>(a, nb, as_stream(stream), "lnr_composite_bwd");
}

extern "C" int lnr_field_train(const uint16_t* w, const uint32_t* enc, int64_t enc_stride, const float* rays,
                               const float* z, const float* depth_gt, int64_t n_rays, int32_t n_samples,
                               float noise_std, const float* noise, uint32_t key, int64_t ray_offset,
                               const lnr_loss_params* lp, float* d_enc, float* d_w, float* workspace,
                               float* ray_stats, float* depth, float* opacity, float* weights,
                               float* d_enc_level_max, uint32_t* d_enc_jac, void* stream) {
  if (int e = check_rays(rays, z, n_rays, n_samples, "lnr_field_train")) return e;
  if (int e = check_lp(lp, "lnr_field_train")) return e;
  LNR_REQUIRE(n_samples % 64 == 0, "lnr_field_train: n_samples=%d must be a multiple of 64", n_samples);
  LNR_REQUIRE(enc_stride >= n_rays * (int64_t)n_samples, "lnr_field_train: enc_stride too small");
  if (n_rays == 0) {
    // an empty batch (e.g. one rank's share of a tiny global batch) still has outputs: the stored MLP
    // gradient is zero, the level maxima are zero, and the loss scalars are finalized (loss 0)
    hipStream_t st = as_stream(stream);
    if (d_w && (lp->flags & LNR_LP_DW_OVERWRITE))
      LNR_REQUIRE(hipMemsetAsync(d_w, 0, LNR_SIGMA_MLP_PARAMS * sizeof(float), st) == hipSuccess,
                  "lnr_field_train: memset failed");
    if (d_enc_level_max)
      LNR_REQUIRE(hipMemsetAsync(d_enc_level_max, 0, kSigmaLevels * sizeof(float), st) == hipSuccess,
                  "lnr_field_train: memset failed");
    if (lp->dev_loss_out)
      hipLaunchKernelGGL(k_loss_finalize, dim3(1), dim3(kReduceThreads), 0, st, ray_stats, (int64_t)0, *lp,
                         lp->dev_loss_out);
    LNR_RETURN_LAUNCH("lnr_field_train(empty)");
  }
  LNR_REQUIRE(w && enc && depth_gt && (d_enc || d_enc_jac) && d_w && workspace && ray_stats,
              "lnr_field_train: null pointer");
  LNR_REQUIRE(!d_enc_jac || n_samples == 64 || n_samples == 128 || n_samples == 256 || n_samples == 512,
              "lnr_field_train: d_enc_jac needs n_samples in {64, 128, 256, 512} (got %d)", n_samples);
  LNR_REQUIRE(enc_stride < (int64_t(1) << 26), "lnr_field_train: enc_stride=%lld over 2^26 (32-bit level offsets)",
              (long long)enc_stride);
  FieldArgs a{};
  a.w = w; a.enc = enc; a.enc_stride = enc_stride; a.rays = rays; a.z = z; a.depth_gt = depth_gt;
  a.n_rays = n_rays; a.S = n_samples; a.noise_std = noise_std; a.noise = noise; a.key = key;
  a.ray_offset = ray_offset; a.lp = *lp; a.d_enc = d_enc; a.dw_slab = workspace; a.ray_stats = ray_stats;
  a.depth = depth; a.opacity = opacity; a.weights = weights; a.denc_max = d_enc_level_max; a.d_jac = d_enc_jac;
  a.d_ray = lp->dev_d_ray;
  hipStream_t st = as_stream(stream);
  int nb;
  const int C = n_samples / 64;
  float* dsig_ws = workspace + lnr_dw_workspace_words(n_rays);
  const bool fwd_only = (lp->flags & LNR_LP_FORWARD_ONLY) != 0, bwd_only = (lp->flags & LNR_LP_BACKWARD_ONLY) != 0;
  LNR_REQUIRE(!(fwd_only || bwd_only) || (d_enc_jac && (C == 1 || C == 2 || C == 4 || C == 8) && !(fwd_only && bwd_only)),
              "lnr_field_train: LNR_LP_FORWARD_ONLY / BACKWARD_ONLY need d_enc_jac, n_samples in {64 .. 512}, one of them");
  if ((C == 1 || C == 2 || C == 4 || C == 8) && dsig_ws) {
    // one wave per ray (the reference's 512 samples: C = 8), then the tile-parallel MLP backward
    a.d_sigma = dsig_ws;
    const int64_t want = (n_rays + kWavesPerBlock - 1) / kWavesPerBlock;
    const int nr = (int)(want < 2048 ? want : 2048);
    const size_t sm = wave_smem_bytes(n_samples);
#if LNR_FIELD_SPLIT
    if (!bwd_only) {
    if (!(lp->flags & LNR_LP_SIGMA_READY)) {  // (early ray termination: lnr_field_sigma_phase wrote sigma)
      const int64_t units = n_rays * (int64_t)n_samples / kSigmaFwdUnit;
      const int64_t wantu = (units + kWavesPerBlock - 1) / kWavesPerBlock;
      hipLaunchKernelGGL(k_sigma_fwd_tiles, dim3((int)(wantu < 8192 ? wantu : 8192)), dim3(NT), 0, st, a);
    }
    switch (C) {
      case 1: hipLaunchKernelGGL(k_composite_wave<1>, dim3(nr), dim3(NT), sm, st, a); break;
      case 2: hipLaunchKernelGGL(k_composite_wave<2>, dim3(nr), dim3(NT), sm, st, a); break;
      case 4: hipLaunchKernelGGL(k_composite_wave<4>, dim3(nr), dim3(NT), sm, st, a); break;
      default: hipLaunchKernelGGL(k_composite_wave<8>, dim3(nr), dim3(NT), sm, st, a); break;
    }
    }
    if (fwd_only) LNR_RETURN_LAUNCH("lnr_field_train(forward)");
#else
    switch (C) {
      case 1: hipLaunchKernelGGL(k_field_wave<1>, dim3(nr), dim3(NT), sm, st, a); break;
      case 2: hipLaunchKernelGGL(k_field_wave<2>, dim3(nr), dim3(NT), sm, st, a); break;
      case 4: hipLaunchKernelGGL(k_field_wave<4>, dim3(nr), dim3(NT), sm, st, a); break;
      default: hipLaunchKernelGGL(k_field_wave<8>, dim3(nr), dim3(NT), sm, st, a); break;
    }
#endif
    const int64_t pairs = (n_rays * (int64_t)n_samples) / 32;
    const int64_t wantb = (pairs + kWavesPerBlock - 1) / kWavesPerBlock;
    const int64_t slabs = lnr_dw_workspace_words(n_rays) / LNR_SIGMA_MLP_PARAMS;  // one dW slab per block
    nb = (int)(wantb < slabs ? wantb : slabs);
    if (nb > kMlpBwdBlocks) nb = kMlpBwdBlocks;
    if (d_enc_jac)
      hipLaunchKernelGGL(k_mlp_bwd_tiles<true>, dim3(nb), dim3(NT), bwd_tiles_smem_bytes(), st, a);
    else
      hipLaunchKernelGGL(k_mlp_bwd_tiles<false>, dim3(nb), dim3(NT), bwd_tiles_smem_bytes(), st, a);
  } else {
    nb = field_blocks(n_rays);
    int e = launch_field<true, false, kSigmaMLP>(a, nb, st, "lnr_field_train");
    if (e) return e;
    if (d_enc_level_max) {
      LNR_REQUIRE(hipMemsetAsync(d_enc_level_max, 0, kSigmaLevels * sizeof(float), st) == hipSuccess,
                  "lnr_field_train: memset failed");
      hipLaunchKernelGGL(k_denc_max, dim3(256, kSigmaLevels), dim3(256), 0, st, reinterpret_cast<const float2*>(d_enc),
                         enc_stride, n_rays * (int64_t)n_samples, d_enc_level_max);
    }
  }
  const int nred = (LNR_SIGMA_MLP_PARAMS + 63) / 64 + (lp->dev_loss_out ? 1 : 0);
  hipLaunchKernelGGL(k_reduce_slabs, dim3(nred), dim3(64 * kSlabWaves), 0, st, workspace, nb, d_w,
                     (lp->flags & LNR_LP_DW_OVERWRITE) != 0, ray_stats, n_rays, *lp);
  LNR_RETURN_LAUNCH("lnr_field_train(reduce)");
}

extern "C" int lnr_field_sigma_phase(const uint16_t* w, const uint32_t* enc, int64_t enc_stride, const float* rays,
                                     const float* z, int64_t n_rays, int32_t n_samples, int32_t lo, int32_t hi,
                                     float noise_std, const float* noise, uint32_t key, int64_t ray_offset,
                                     const lnr_loss_params* lp, float* workspace, const uint32_t* list_in,
                                     const uint32_t* count_in, uint32_t* list_out, uint32_t* count_out,
                                     double* transmittance, void* scratch, void* stream) {
  if (int e = check_rays(rays, z, n_rays, n_samples, "lnr_field_sigma_phase")) return e;
  LNR_REQUIRE(n_samples % 64 == 0 && lo >= 0 && lo < hi && hi <= n_samples && lo % 64 == 0 && hi % 64 == 0,
              "lnr_field_sigma_phase: phase [%d, %d) of %d samples must be whole 64-sample waves", lo, hi, n_samples);
  LNR_REQUIRE(enc_stride >= n_rays * (int64_t)n_samples && enc_stride < (int64_t(1) << 26),
              "lnr_field_sigma_phase: bad enc_stride");
  LNR_REQUIRE(n_rays < (int64_t(1) << 31), "lnr_field_sigma_phase: too many rays");
  if (n_rays == 0) return LNR_OK;
  LNR_REQUIRE(w && enc && workspace && (lo == 0 || (list_in && count_in)) && (!list_in || count_in),
              "lnr_field_sigma_phase: null pointer (a phase after the first needs the list of rays still alive)");
  LNR_REQUIRE(hi == n_samples || (list_out && count_out && transmittance && scratch),
              "lnr_field_sigma_phase: null pointer (the phase's transmittance update)");
  FieldArgs a{};
  a.w = w; a.enc = enc; a.enc_stride = enc_stride; a.rays = rays; a.z = z; a.n_rays = n_rays; a.S = n_samples;
  a.noise_std = noise_std; a.noise = noise; a.key = key; a.ray_offset = ray_offset;
  if (lp) a.lp = *lp;
  a.d_sigma = workspace + lnr_dw_workspace_words(n_rays);
  hipStream_t st = as_stream(stream);
  const uint32_t* lin = lo == 0 ? nullptr : list_in;
  const uint32_t* cin = lo == 0 ? nullptr : count_in;
  uint32_t* keep = reinterpret_cast<uint32_t*>(scratch);  // one word per entry
  const int64_t want = (n_rays + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(k_sigma_phase, dim3((unsigned)(want < 8192 ? want : 8192)), dim3(NT), 0, st, a, lin, cin, lo, hi,
                     transmittance, keep, kErtTMin);
  if (hi < n_samples)
    hipLaunchKernelGGL(k_ert_compact, dim3(1), dim3(kErtCompactThreads), 0, st, keep, cin, n_rays, list_out, count_out);
  LNR_RETURN_LAUNCH("lnr_field_sigma_phase");
}

extern "C" int lnr_field_render(const uint16_t* w, const uint32_t* enc, int64_t enc_stride, const float* rays,
                                const float* z, int64_t n_rays, int32_t n_samples, int32_t strategy, float noise_std,
                                const float* noise, uint32_t key, int64_t ray_offset, float* depth, float* opacity,
                                float* variance, float* weights, void* stream) {
  if (int e = check_rays(rays, z, n_rays, n_samples, "lnr_field_render")) return e;
  LNR_REQUIRE(strategy == LNR_RENDER_DEFAULT || strategy == LNR_RENDER_ADJUSTED,
              "Unknown render strategy: %d", strategy);
  LNR_REQUIRE(n_samples % 64 == 0, "lnr_field_render: n_samples=%d must be a multiple of 64", n_samples);
  LNR_REQUIRE(enc_stride >= n_rays * (int64_t)n_samples, "lnr_field_render: enc_stride too small");
  if (n_rays == 0) return LNR_OK;
  LNR_REQUIRE(w && enc && depth, "lnr_field_render: null pointer");
  FieldArgs a{};
  a.w = w; a.enc = enc; a.enc_stride = enc_stride; a.rays = rays; a.z = z; a.n_rays = n_rays; a.S = n_samples;
  a.noise_std = noise_std; a.noise = noise; a.key = key; a.ray_offset = ray_offset;
  a.depth = depth; a.opacity = opacity; a.variance = variance; a.weights = weights;
  const int nb = field_blocks(n_rays);
#if LNR_FIELD_SPLIT
  if (weights) {
    // the sigma MLP tile-parallel first (k_sigma_fwd_tiles), its sigma staged in the weights buffer,
    // which the compositing reads into LDS one ray at a time before it writes that ray's weights
    hipStream_t st = as_stream(stream);
    a.d_sigma = weights;
    const int64_t units = n_rays * (int64_t)n_samples / kSigmaFwdUnit;
    const int64_t wantu = (units + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(k_sigma_fwd_tiles, dim3((int)(wantu < 8192 ? wantu : 8192)), dim3(NT), 0, st, a);
    a.d_sigma = nullptr;
    a.sigma_in = weights;
    if (strategy == LNR_RENDER_ADJUSTED) return launch_field<false, true, kSigmaGiven>(a, nb, st, "lnr_field_render");
    return launch_field<false, false, kSigmaGiven>(a, nb, st, "lnr_field_render");
  }
#endif
  if (strategy == LNR_RENDER_ADJUSTED)
    return launch_field<false, true, kSigmaMLP>(a, nb, as_stream(stream), "lnr_field_render");
  return launch_field<false, false, kSigmaMLP>(a, nb, as_stream(stream), "lnr_field_render");
}

__global__ void __launch_bounds__(kReduceThreads) k_count_opaque(const float* __restrict__ dgt, int64_t n,
                                                                 float far_ref_h, const float* dev_far_ref, float* out) {
  const float far_ref = dev_far_ref ? dev_far_ref[0] : far_ref_h;
  __shared__ float red[kReduceThreads / 64];
  float c = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) c += (dgt[i] > 0.f && !(dgt[i] > far_ref)) ? 1.f : 0.f;
  float v[1] = {c};
  block_sum<kReduceThreads, 1>(v, red);
  if (threadIdx.x == 0) out[0] = v[0];
}

extern "C" int lnr_count_opaque(const float* depth_gt, int64_t n_rays, float far_ref, const float* dev_far_ref,
                                float* out, void* stream) {
  LNR_REQUIRE(n_rays >= 0 && out, "lnr_count_opaque: bad arguments");
  LNR_REQUIRE(n_rays == 0 || depth_gt, "lnr_count_opaque: null depth_gt");
  hipLaunchKernelGGL(k_count_opaque, dim3(1), dim3(kReduceThreads), 0, as_stream(stream), depth_gt, n_rays, far_ref, dev_far_ref, out);
  LNR_RETURN_LAUNCH("lnr_count_opaque");
}

extern "C" int lnr_loss_finalize(const float* ray_stats, int64_t n_rays, const lnr_loss_params* lp, float* out,
                                 void* stream) {
  if (int e = check_lp(lp, "lnr_loss_finalize")) return e;
  LNR_REQUIRE(ray_stats && out, "lnr_loss_finalize: null pointer");
  hipLaunchKernelGGL(k_loss_finalize, dim3(1), dim3(kReduceThreads), 0, as_stream(stream), ray_stats, n_rays, *lp, out);
  LNR_RETURN_LAUNCH("lnr_loss_finalize");
}
