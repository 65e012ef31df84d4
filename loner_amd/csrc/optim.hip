// Optimiser-side kernels: fused Adam over the flat sigma parameters, the occupancy-grid (OGM)
// update, parameter init and dtype conversion.
//
// Adam  : torch.optim.Adam as constructed per window at src/mapping/optimizer.py:255-265 and
//         stepped at :460 (betas 0.9/0.999, eps 1e-8, no weight decay) on fp32 master params,
//         writing the fp16 forward shadow in the same pass (tcnn forwards with fp16 params).
// OGM   : Optimizer._step_occupancy_grid src/mapping/optimizer.py:897-908 — grid_sample backward of
//         get_logits_grad (src/models/losses.py:54-62) followed by SGD (lr from occ_model.lr).
#include "common.hpp"

namespace lnr {

__device__ __forceinline__ void adam_range(float* __restrict__ p, uint16_t* __restrict__ shadow,
                                           const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
                                           int64_t n, float one_minus_b1, float b2, float one_minus_b2,
                                           float step_size, float bc2_sqrt, float eps, uint32_t bx, uint32_t nbx) {
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)nbx * blockDim.x;
  for (int64_t i = (int64_t)bx * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* pa = &pp.x;
    const float* ga = &gg.x;
    float* ma = &mm.x;
    float* va = &vv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ma[k] = ma[k] + one_minus_b1 * (ga[k] - ma[k]);           // exp_avg.lerp_(grad, 1-b1)
      va[k] = va[k] * b2 + one_minus_b2 * ga[k] * ga[k];         // mul_(b2).addcmul_(g, g, 1-b2)
      const float denom = sqrtf(va[k]) / bc2_sqrt + eps;
      pa[k] = pa[k] + (-step_size) * (ma[k] / denom);           // addcdiv_(m, denom, -step_size)
    }
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (shadow) {
      uint2 h;
      h.x = (uint32_t)f2h(pa[0]) | ((uint32_t)f2h(pa[1]) << 16);
      h.y = (uint32_t)f2h(pa[2]) | ((uint32_t)f2h(pa[3]) << 16);
      reinterpret_cast<uint2*>(shadow)[i] = h;
    }
  }
  // tail
  if (bx == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = n4 * 4 + threadIdx.x;
    float mk = m[i] + one_minus_b1 * (g[i] - m[i]);
    float vk = v[i] * b2 + one_minus_b2 * g[i] * g[i];
    float pk = p[i] + (-step_size) * (mk / (sqrtf(vk) / bc2_sqrt + eps));
    m[i] = mk;
    v[i] = vk;
    p[i] = pk;
    if (shadow) shadow[i] = f2h(pk);
  }
}

__global__ void __launch_bounds__(256) k_adam(float* __restrict__ p, uint16_t* __restrict__ shadow,
                                              const float* __restrict__ g, float* __restrict__ m,
                                              float* __restrict__ v, int64_t n, float one_minus_b1, float b2,
                                              float one_minus_b2, float step_size, float bc2_sqrt, float eps,
                                              const lnr_step_scalars* dev_step) {
  if (dev_step) {  // graph replay: this step's coefficients from device memory
    step_size = dev_step->adam_step_size;
    bc2_sqrt = dev_step->adam_bc2_sqrt;
  }
  adam_range(p, shadow, g, m, v, n, one_minus_b1, b2, one_minus_b2, step_size, bc2_sqrt, eps, blockIdx.x, gridDim.x);
}

// Several ranges in one launch (the sharded optimiser's chunks, one per level range): blockIdx.y
// is the range.
struct AdamRanges {
  lnr_adam_range r[LNR_ADAM_MAX_RANGES];
};
__global__ void __launch_bounds__(256) k_adam_ranges(AdamRanges rs, float one_minus_b1, float b2, float one_minus_b2,
                                                     float step_size, float bc2_sqrt, float eps,
                                                     const lnr_step_scalars* dev_step) {
  if (dev_step) {
    step_size = dev_step->adam_step_size;
    bc2_sqrt = dev_step->adam_bc2_sqrt;
  }
  const lnr_adam_range& r = rs.r[blockIdx.y];
  adam_range(r.param, r.shadow, r.grad, r.m, r.v, r.n, one_minus_b1, b2, one_minus_b2, step_size, bc2_sqrt, eps,
             blockIdx.x, gridDim.x);
}

// logits "gradient" of losses.py:54-62 with eps=2, l_free=0.25, l_occ=2.5; H(0)=0.
__device__ __forceinline__ float logits_grad(float x) {
  const float eps = 2.0f;
  const float fr = ((-x - eps) > 0.f) ? 1.f : 0.f;
  const float oc = (((x + eps) > 0.f) ? 1.f : 0.f) * (((eps - x) > 0.f) ? 1.f : 0.f);
  return 0.25f * fr - 2.5f * oc;
}

// The splat accumulates in int64 fixed point, so the grid gradient does not depend on the atomics'
// order: bitwise reproducible.  The OGM update's unit is 2^-28 (a sample adds |w g| <= 2.5, so 2^31
// samples stay below 2^63); the generic grid_sample backward (lnr_grid_sample3d_bwd) takes its unit
// from max |dout| and the point count (fix_exp below).  Workspace (floats): [0, V) the float result,
// then n_rep int64 replicas.
constexpr int32_t kOgmReplicas = 3;
constexpr int kOgmFixExp = 28;
constexpr uint32_t kInfBits = 0x7F800000u;  // +inf's bits: k_abs_max's value at or above it = non-finite

// The OGM update's points: sample i of ray r, xyz = o + d z, logits gradient of its depth error.
struct OgmRaySamples {
  const float* rays;
  const float* z;
  const float* dgt;
  int32_t S;
  float scale;
  __device__ __forceinline__ void at(int64_t i, float& px, float& py, float& pz, float& g) const {
    const int64_t r = i / S;
    const float* ry = rays + 13 * r;
    const float t = z[i];
    px = ry[0] + ry[3] * t;
    py = ry[1] + ry[4] * t;
    pz = ry[2] + ry[5] * t;
    g = logits_grad(t * scale - dgt[r] * scale);
  }
};

// grid_sample's backward for given points and output gradients (OccupancyGridModel.interpolate).
struct PointGrads {
  const float* pts;   // (n, 3)
  const float* dout;  // (n)
  __device__ __forceinline__ void at(int64_t i, float& px, float& py, float& pz, float& g) const {
    px = pts[3 * i];
    py = pts[3 * i + 1];
    pz = pts[3 * i + 2];
    g = dout[i];
  }
};

// Fixed-point exponent of the generic backward: every per-voxel sum of |w g| <= n max|g| < 2^62.
__device__ __forceinline__ int fix_exp(const uint32_t* amax_bits, int64_t n) {
  if (amax_bits == nullptr) return kOgmFixExp;
  if (*amax_bits >= kInfBits) return 0;  // non-finite: k_sum_replicas writes NaN
  const float m = __uint_as_float(*amax_bits);
  if (!(m > 0.f)) return 0;  // nothing to add
  int em, en = 0;
  frexpf(m, &em);  // m < 2^em
  while ((int64_t(1) << en) < n && en < 62) ++en;
  const int e = 62 - em - en;
  return e < -120 ? -120 : (e > 120 ? 120 : e);
}

template <class Src>
__global__ void __launch_bounds__(256) k_ogm_grad(Src src, int64_t n, unsigned long long* __restrict__ grad,
                                                  int32_t R, int32_t n_rep, const uint32_t* amax_bits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // replica of the grid this workgroup adds into: the rays of one keyframe share their first
  // voxels, so one copy would serialise hundreds of same-address atomics at the memory side
  grad += (int64_t)(blockIdx.x % (uint32_t)n_rep) * R * R * R;
  const float fix = ldexpf(1.f, fix_exp(amax_bits, n));
  const int lane = threadIdx.x & 63;
  const bool valid = i < n;
  float gval = 0.f, px = 0.f, py = 0.f, pz = 0.f;
  if (valid) src.at(i, px, py, pz, gval);
  const float ix = ((px + 1.f) * (float)R - 1.f) / 2.f;
  const float iy = ((py + 1.f) * (float)R - 1.f) / 2.f;
  const float iz = ((pz + 1.f) * (float)R - 1.f) / 2.f;
  const float fx = floorf(ix), fy = floorf(iy), fz = floorf(iz);
  const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
  const float wx[2] = {(float)(x0 + 1) - ix, ix - (float)x0};
  const float wy[2] = {(float)(y0 + 1) - iy, iy - (float)y0};
  const float wz[2] = {(float)(z0 + 1) - iz, iz - (float)z0};
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int bx = c & 1, by = (c >> 1) & 1, bz = (c >> 2) & 1;
    const int cx = x0 + bx, cy = y0 + by, cz = z0 + bz;
    const bool inb = valid && gval != 0.f && cx >= 0 && cx < R && cy >= 0 && cy < R && cz >= 0 && cz < R;
    const int64_t idx = inb ? (((int64_t)cz * R + cy) * R + cx) : -1;
    float p = inb ? wx[bx] * wy[by] * wz[bz] * gval : 0.f;
    // merge runs of equal voxel indices across consecutive samples before the atomic
    const int64_t prev = __shfl_up(idx, 1, 64);
    const bool head = (lane == 0) || (prev != idx);
    const unsigned long long heads = __ballot(head);
    const int head_lane = 63 - __clzll(heads & ((2ull << lane) - 1ull));
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float q = __shfl_up(p, o, 64);
      if (lane - o >= head_lane) p += q;
    }
    const bool tail = (lane == 63) || ((heads >> (lane + 1)) & 1ull);
    if (tail && idx >= 0) atomicAdd(&grad[idx], (unsigned long long)__float2ll_rn(p * fix));
  }
}

// out = (sum of the int64 replicas) / 2^e (exact integer sum, one rounding).  A non-finite output
// gradient (k_abs_max's bits >= +inf's) cannot be carried in fixed point: the whole grid gradient is
// then NaN, so the non-finite value propagates (torch's grid_sample backward would give NaN / inf at the
// voxels the point touches) instead of turning into arbitrary integers.
__global__ void k_sum_replicas(const unsigned long long* __restrict__ g, int64_t nv, int32_t n_rep,
                               float* __restrict__ out, const uint32_t* amax_bits, int64_t n_pts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nv) return;
  if (amax_bits && *amax_bits >= kInfBits) {
    out[i] = __builtin_nanf("");
    return;
  }
  long long s = 0;
  for (int k = 0; k < n_rep; ++k) s += (long long)g[(int64_t)k * nv + i];
  out[i] = (float)ldexp((double)s, -fix_exp(amax_bits, n_pts));
}

// max |x| of n floats into *amax_bits (zeroed before), as bits: non-negative floats order as their bits,
// +inf is 0x7F800000 and every NaN (sign cleared) lies above it, so a non-finite x is never skipped (fmaxf
// would drop a NaN)
__global__ void __launch_bounds__(256) k_abs_max(const float* __restrict__ x, int64_t n, uint32_t* amax_bits) {
  uint32_t m = 0u;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = max(m, __float_as_uint(x[i]) & 0x7FFFFFFFu);
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0 && m > 0u) atomicMax(amax_bits, m);
}

__global__ void __launch_bounds__(256) k_grid_sample3d(const float* __restrict__ grid, int32_t R,
                                                       const float* __restrict__ pts, int64_t n, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = occ_grid_sample(grid, R, pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
}

static int ogm_grad_launch(const float* rays, const float* z, const float* depth_gt, int64_t n_rays, int32_t n_samples,
                           float scale, float* grad_ws, int64_t ws_words, int32_t occ_res, hipStream_t st,
                           const char* who) {
  const int64_t nv = (int64_t)occ_res * occ_res * occ_res;
  LNR_REQUIRE(ws_words >= 3 * nv, "%s: grad_ws holds %lld words, needs >= %lld (3 res^3)", who, (long long)ws_words,
              (long long)(3 * nv));
  const int64_t rep = (ws_words / nv - 1) / 2;  // int64 replicas after the float result
  const int32_t n_rep = (int32_t)(rep > kOgmReplicas ? kOgmReplicas : rep);
  unsigned long long* g64 = reinterpret_cast<unsigned long long*>(grad_ws + nv + (nv & 1));  // 8-B aligned
  LNR_REQUIRE((nv + (nv & 1)) + 2 * n_rep * nv <= ws_words, "%s: grad_ws too small", who);
  if (hipMemsetAsync(g64, 0, (size_t)n_rep * nv * sizeof(unsigned long long), st) != hipSuccess) {
    set_error("%s: hipMemsetAsync failed", who);
    return LNR_ERR_HIP;
  }
  const int64_t n = n_rays * (int64_t)n_samples;
  if (n > 0) {
    LNR_REQUIRE(rays && z && depth_gt, "%s: null pointer", who);
    const OgmRaySamples src{rays, z, depth_gt, n_samples, scale};
    hipLaunchKernelGGL(k_ogm_grad<OgmRaySamples>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, n, g64,
                       occ_res, n_rep, (const uint32_t*)nullptr);
  }
  hipLaunchKernelGGL(k_sum_replicas, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, g64, nv, n_rep, grad_ws,
                     (const uint32_t*)nullptr, n);
  return LNR_OK;
}

__global__ void k_sgd(float* __restrict__ p, const float* __restrict__ g, int64_t n, float lr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] + (-lr) * g[i];
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void k_fill_uniform(float* __restrict__ dst, int64_t n, uint32_t seed, float lo, float hi, int64_t start) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = splitmix64(((uint64_t)seed << 32) + (uint64_t)(start + i));
  const float u = (float)(h >> 40) * 5.9604644775390625e-08f;
  dst[i] = lo + (hi - lo) * u;
}

__global__ void k_f32_to_f16(const float* __restrict__ s, uint16_t* __restrict__ d, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = f2h(s[i]);
}

static unsigned grid1d(int64_t n, int64_t cap = 1 << 20) {
  int64_t b = (n + 255) / 256;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace lnr

using namespace lnr;

struct StepScalarsArg {
  lnr_step_scalars v[4];
};
__global__ void k_step_scalars_set(StepScalarsArg values, int32_t n, lnr_step_scalars* __restrict__ out) {
  if (threadIdx.x < (uint32_t)n) out[threadIdx.x] = values.v[threadIdx.x];
}

extern "C" int lnr_step_scalars_set(const lnr_step_scalars* values, int32_t n, lnr_step_scalars* dev, void* stream) {
  LNR_REQUIRE(values && dev && n >= 1 && n <= 4, "lnr_step_scalars_set: bad arguments (n=%d, at most 4)", n);
  StepScalarsArg arg{};
  for (int i = 0; i < n; ++i) arg.v[i] = values[i];
  hipLaunchKernelGGL(k_step_scalars_set, dim3(1), dim3(64), 0, as_stream(stream), arg, n, dev);
  LNR_RETURN_LAUNCH("lnr_step_scalars_set");
}

// the hyper-parameters arrive as doubles (Python floats) and every derived scalar is formed in double
// before its single rounding to fp32, as torch.optim.Adam forms them (1 - beta2 from the float 0.999f
// would be 1.3e-5 off)
extern "C" int lnr_adam_coefficients(int32_t step, double lr, double beta1, double beta2, float* step_size,
                                     float* bc2_sqrt) {
  LNR_REQUIRE(step >= 1 && step_size && bc2_sqrt, "lnr_adam_coefficients: step=%d", step);
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  *step_size = (float)(lr / bc1);
  *bc2_sqrt = (float)std::sqrt(bc2);
  return LNR_OK;
}

extern "C" int lnr_adam_step(float* param, uint16_t* shadow, const float* grad, float* m, float* v, int64_t n,
                             int32_t step, double lr, double beta1, double beta2, double eps,
                             const lnr_step_scalars* dev_step, void* stream) {
  LNR_REQUIRE(n >= 0 && step >= 1, "lnr_adam_step: n=%lld step=%d", (long long)n, step);
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(param && grad && m && v, "lnr_adam_step: null pointer");
  LNR_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) % 16 == 0 &&
                  (shadow == nullptr || (uintptr_t)shadow % 8 == 0),
              "lnr_adam_step: buffers must be 16-byte aligned");
  float step_size, bc2_sqrt;
  if (int e = lnr_adam_coefficients(step, lr, beta1, beta2, &step_size, &bc2_sqrt)) return e;
  hipLaunchKernelGGL(k_adam, dim3(grid1d(n / 4, 8192)), dim3(256), 0, as_stream(stream), param, shadow, grad, m, v, n,
                     (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), step_size, bc2_sqrt, (float)eps, dev_step);
  LNR_RETURN_LAUNCH("lnr_adam_step");
}

extern "C" int lnr_adam_step_ranges(const lnr_adam_range* ranges, int32_t n_ranges, int32_t step, double lr,
                                    double beta1, double beta2, double eps, const lnr_step_scalars* dev_step,
                                    void* stream) {
  LNR_REQUIRE(n_ranges >= 0 && n_ranges <= LNR_ADAM_MAX_RANGES && step >= 1,
              "lnr_adam_step_ranges: n_ranges=%d (at most %d) step=%d", n_ranges, LNR_ADAM_MAX_RANGES, step);
  if (n_ranges == 0) return LNR_OK;
  LNR_REQUIRE(ranges != nullptr, "lnr_adam_step_ranges: null ranges");
  AdamRanges rs{};
  int64_t nmax = 0;
  for (int i = 0; i < n_ranges; ++i) {
    const lnr_adam_range& r = ranges[i];
    LNR_REQUIRE(r.n >= 0, "lnr_adam_step_ranges: range %d: n < 0", i);
    LNR_REQUIRE(r.n == 0 || (r.param && r.grad && r.m && r.v), "lnr_adam_step_ranges: range %d: null pointer", i);
    LNR_REQUIRE(((uintptr_t)r.param | (uintptr_t)r.grad | (uintptr_t)r.m | (uintptr_t)r.v) % 16 == 0 &&
                    (r.shadow == nullptr || (uintptr_t)r.shadow % 8 == 0),
                "lnr_adam_step_ranges: range %d: buffers must be 16-byte aligned", i);
    rs.r[i] = r;
    nmax = r.n > nmax ? r.n : nmax;
  }
  if (nmax == 0) return LNR_OK;
  float step_size, bc2_sqrt;
  if (int e = lnr_adam_coefficients(step, lr, beta1, beta2, &step_size, &bc2_sqrt)) return e;
  hipLaunchKernelGGL(k_adam_ranges, dim3(grid1d(nmax / 4, 8192), n_ranges), dim3(256), 0, as_stream(stream), rs,
                     (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), step_size, bc2_sqrt, (float)eps, dev_step);
  LNR_RETURN_LAUNCH("lnr_adam_step_ranges");
}

extern "C" int64_t lnr_ogm_workspace_words(int32_t occ_res) {
  if (occ_res < 1) return -1;
  const int64_t nv = (int64_t)occ_res * occ_res * occ_res;
  return nv + (nv & 1) + 2 * kOgmReplicas * nv;  // float result + int64 replicas
}

extern "C" int lnr_ogm_update(const float* rays, const float* z, const float* depth_gt, int64_t n_rays,
                              int32_t n_samples, float scale, float lr, float* occ, float* grad_ws, int64_t ws_words,
                              int32_t occ_res, void* stream) {
  LNR_REQUIRE(n_rays >= 0 && n_samples >= 1 && occ_res >= 1, "lnr_ogm_update: bad sizes");
  LNR_REQUIRE(occ && grad_ws, "lnr_ogm_update: null grid");
  const int64_t nv = (int64_t)occ_res * occ_res * occ_res;
  hipStream_t st = as_stream(stream);
  if (int e = ogm_grad_launch(rays, z, depth_gt, n_rays, n_samples, scale, grad_ws, ws_words, occ_res, st,
                              "lnr_ogm_update"))
    return e;
  hipLaunchKernelGGL(k_sgd, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, occ, grad_ws, nv, lr);
  LNR_RETURN_LAUNCH("lnr_ogm_update");
}

extern "C" int lnr_ogm_grad(const float* rays, const float* z, const float* depth_gt, int64_t n_rays,
                            int32_t n_samples, float scale, float* grad_ws, int64_t ws_words, int32_t occ_res,
                            void* stream) {
  LNR_REQUIRE(n_rays >= 0 && n_samples >= 1 && occ_res >= 1 && grad_ws, "lnr_ogm_grad: bad arguments");
  if (int e = ogm_grad_launch(rays, z, depth_gt, n_rays, n_samples, scale, grad_ws, ws_words, occ_res,
                              as_stream(stream), "lnr_ogm_grad"))
    return e;
  LNR_RETURN_LAUNCH("lnr_ogm_grad");
}

extern "C" int lnr_grid_sample3d(const float* grid, int32_t res, const float* pts, int64_t n, float* out,
                                 void* stream) {
  LNR_REQUIRE(res >= 1 && n >= 0, "lnr_grid_sample3d: bad sizes");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(grid && pts && out, "lnr_grid_sample3d: null pointer");
  hipLaunchKernelGGL(k_grid_sample3d, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), grid, res, pts,
                     n, out);
  LNR_RETURN_LAUNCH("lnr_grid_sample3d");
}

extern "C" int64_t lnr_grid_sample3d_bwd_workspace_words(int32_t res) {
  if (res < 1) return -1;
  return 2 + 2 * (int64_t)kOgmReplicas * res * res * res;  // max |dout| (8-B slot) + int64 replicas
}

extern "C" int lnr_grid_sample3d_bwd(const float* pts, const float* dout, int64_t n, int32_t res, float* dgrid,
                                     float* ws, int64_t ws_words, void* stream) {
  LNR_REQUIRE(res >= 1 && n >= 0, "lnr_grid_sample3d_bwd: bad sizes");
  LNR_REQUIRE(n < (int64_t(1) << 40), "lnr_grid_sample3d_bwd: n=%lld too large", (long long)n);
  LNR_REQUIRE(dgrid && ws, "lnr_grid_sample3d_bwd: null pointer");
  LNR_REQUIRE(n == 0 || (pts && dout), "lnr_grid_sample3d_bwd: null pointer");
  LNR_REQUIRE(((uintptr_t)ws & 7) == 0, "lnr_grid_sample3d_bwd: workspace must be 8-byte aligned");
  const int64_t nv = (int64_t)res * res * res;
  const int64_t rep = (ws_words - 2) / (2 * nv);
  LNR_REQUIRE(rep >= 1, "lnr_grid_sample3d_bwd: workspace holds %lld words, needs >= %lld", (long long)ws_words,
              (long long)(2 + 2 * nv));
  const int32_t n_rep = (int32_t)(rep > kOgmReplicas ? kOgmReplicas : rep);
  uint32_t* amax = reinterpret_cast<uint32_t*>(ws);
  unsigned long long* g64 = reinterpret_cast<unsigned long long*>(ws + 2);
  hipStream_t st = as_stream(stream);
  if (hipMemsetAsync(ws, 0, (size_t)(2 + 2 * n_rep * nv) * sizeof(float), st) != hipSuccess) {
    set_error("lnr_grid_sample3d_bwd: hipMemsetAsync failed");
    return LNR_ERR_HIP;
  }
  if (n > 0) {
    hipLaunchKernelGGL(k_abs_max, dim3(grid1d(n, 1024)), dim3(256), 0, st, dout, n, amax);
    const PointGrads src{pts, dout};
    hipLaunchKernelGGL(k_ogm_grad<PointGrads>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, n, g64, res,
                       n_rep, (const uint32_t*)amax);
  }
  hipLaunchKernelGGL(k_sum_replicas, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, g64, nv, n_rep, dgrid,
                     (const uint32_t*)amax, n);
  LNR_RETURN_LAUNCH("lnr_grid_sample3d_bwd");
}

extern "C" int lnr_sgd_step(float* param, const float* grad, int64_t n, float lr, void* stream) {
  LNR_REQUIRE(n >= 0, "lnr_sgd_step: n < 0");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(param && grad, "lnr_sgd_step: null pointer");
  hipLaunchKernelGGL(k_sgd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), param, grad, n, lr);
  LNR_RETURN_LAUNCH("lnr_sgd_step");
}

extern "C" int lnr_fill_uniform(float* dst, int64_t n, uint32_t seed, float lo, float hi, int64_t start, void* stream) {
  LNR_REQUIRE(n >= 0, "lnr_fill_uniform: n < 0");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(dst, "lnr_fill_uniform: null pointer");
  hipLaunchKernelGGL(k_fill_uniform, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), dst, n, seed,
                     lo, hi, start);
  LNR_RETURN_LAUNCH("lnr_fill_uniform");
}

extern "C" int lnr_f32_to_f16(const float* src, uint16_t* dst, int64_t n, void* stream) {
  LNR_REQUIRE(n >= 0, "lnr_f32_to_f16: n < 0");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(src && dst, "lnr_f32_to_f16: null pointer");
  hipLaunchKernelGGL(k_f32_to_f16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), src, dst, n);
  LNR_RETURN_LAUNCH("lnr_f32_to_f16");
}

// ------------------------------------------------------------------ status scan
// rendering_tcnn.py:419-424 (DEBUG): every result tensor is scanned for nan/inf on the host.  Here
// one launch ORs `bit` into the device status word when any of the n values is not finite.
__global__ void __launch_bounds__(256) k_status_scan(const float* __restrict__ x, int64_t n, uint32_t bit,
                                                     uint32_t* status) {
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bad |= !isfinite(x[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(status, bit);
}

extern "C" int lnr_status_scan(const float* values, int64_t n, uint32_t bit, uint32_t* status, void* stream) {
  LNR_REQUIRE(n >= 0 && status != nullptr, "lnr_status_scan: bad arguments");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(values != nullptr, "lnr_status_scan: null values");
  const int64_t want = (n + 255) / 256;
  hipLaunchKernelGGL(k_status_scan, dim3((unsigned)(want < 1024 ? want : 1024)), dim3(256), 0, as_stream(stream), values,
                     n, bit, status);
  LNR_RETURN_LAUNCH("lnr_status_scan");
}
