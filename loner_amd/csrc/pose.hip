// Joint pose + map: the per-keyframe pose gradient of a step and the poses' Adam step, on the device.
//
// The reference optimises every un-anchored keyframe's pose tensor [t, axis-angle] in the map's Adam
// (src/mapping/optimizer.py:235-262, lrate_pose); the rays depend on it through
// LidarRayDirections.build_lidar_rays (src/common/ray_utils.py:269-322):
//   o = (t + shift) / scale,  d = R v / |R v|,  far = min(r_max / scale, get_far_val(o, d))   (:31-60)
// with R = axis_angle_to_matrix(axis-angle) (pytorch3d, src/common/pose_utils.py:354-368); sky rays use the
// detached pose (src/mapping/keyframe.py:98).  The step hands over per sample dL/dpos01 (the hash grid's
// input gradient) and per ray [dL/d|d|, dL/dfar] (the compositing's ray terms); loner_amd/pose.py states
// the chain and restates it in torch (the test reference for these kernels):
//   k_pose_rays    one wave per ray: dL/do = sum dpos / 2, dL/dd = sum z dpos / 2 + dL/d|d| d, plus the far
//                  term through get_far_val (torch autograd's choices at the min / max / clamp: first index
//                  on ties, minimum's even split); the ray's contributions to its keyframe's dL/dt (dL/do)
//                  and dL/dR (the (I - d d^T) dL/dd d^T part; dL/dR = that R, loner_amd/pose.py)
//   k_pose_reduce  one workgroup per keyframe, a fixed-order sum over its rays (deterministic), then
//                  dL/dt = sum / scale and dL/d(axis-angle) from dL/dR (closed form, double)
//   k_pose_adam    torch.optim.Adam's step (foreach arithmetic, as lnr_adam_step) on the (K, 6) tensors and the
//                  window's pose rows [R | t] rewritten from them (grad NULL: the rows only)
#include "common.hpp"

namespace lnr {

constexpr int kPoseThreads = 256;
constexpr int kPoseWaves = kPoseThreads / 64;

// far = min(far_range, min_i max(clamp0(t_lo_i), clamp0(t_hi_i))), t = (+-1 - o_i) / (d_i + 1e-15): the axis and
// plane torch's autograd routes the gradient through, and d far / d{o, d} there (0 where far = far_range).
__device__ __forceinline__ void far_grad(const float o[3], const float d[3], float far_range, float g_far, float go[3],
                                         float gd[3]) {
  float best = 0.f, tsel = 0.f, dsel = 1.f;
  int axis = -1;
  bool pass = false;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float dd = d[i] + 1e-15f;
    const float tl = (-1.0f - o[i]) / dd, th = (1.0f - o[i]) / dd;
    const float cl = fmaxf(tl, 0.f), ch = fmaxf(th, 0.f);
    // max over the two planes: the first (-1) on ties; clamp(min=0) passes the gradient where t >= 0
    const bool hi_wins = ch > cl;
    const float m = hi_wins ? ch : cl;
    const float t = hi_wins ? th : tl;
    if (axis < 0 || m < best) {  // min over the axes: the first on ties
      best = m;
      axis = i;
      tsel = t;
      dsel = dd;
      pass = t >= 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) go[i] = gd[i] = 0.f;
  // torch.minimum(far_range, clip): the gradient to clip is 1 below the range, 1/2 on a tie, 0 above
  const float share = best < far_range ? 1.f : (best == far_range ? 0.5f : 0.f);
  if (share == 0.f || !pass) return;
  const float g = g_far * share;
  go[axis] = -g / dsel;           // t = (s - o_i) / (d_i + 1e-15)
  gd[axis] = -g * tsel / dsel;
}

__global__ void __launch_bounds__(kPoseThreads) k_pose_rays(const float* __restrict__ rays, const float* __restrict__ z,
                                                            const float* __restrict__ d_pos, const float* __restrict__ d_ray,
                                                            int64_t n_rays, int32_t S, const int64_t* __restrict__ slots,
                                                            int64_t slot0, const float* __restrict__ slot_pose,
                                                            float far_range, float* __restrict__ ray_ws) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t r = (int64_t)blockIdx.x * kPoseWaves + wid; r < n_rays; r += (int64_t)gridDim.x * kPoseWaves) {
    const int64_t slot = slots ? slots[r] : slot0 + r;
    const float w = slot_pose[slot];
    float so[3] = {0.f, 0.f, 0.f}, sz[3] = {0.f, 0.f, 0.f};
    if (w != 0.f) {  // (wave-uniform) sky rays and anchored keyframes carry no pose gradient
      for (int i = lane; i < S; i += 64) {
        const int64_t n = r * S + i;
        const float zi = z[n];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float p = d_pos[3 * n + k];
          so[k] += p;
          sz[k] += zi * p;
        }
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          so[k] += __shfl_xor(so[k], off, 64);
          sz[k] += __shfl_xor(sz[k], off, 64);
        }
      }
    }
    if (lane == 0) {
      float* out = ray_ws + 12 * r;
      if (w == 0.f) {
#pragma unroll
        for (int k = 0; k < 12; ++k) out[k] = 0.f;
      } else {
        const float* ry = rays + 13 * r;
        const float o[3] = {ry[0], ry[1], ry[2]}, d[3] = {ry[3], ry[4], ry[5]};
        const float dn = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        float go[3], gd[3];
        far_grad(o, d, far_range, d_ray[2 * r + 1], go, gd);
        float g_o[3], g_d[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          g_o[k] = 0.5f * so[k] + go[k];
          g_d[k] = 0.5f * sz[k] + d_ray[2 * r] * (d[k] / dn) + gd[k];
        }
        // dL/dR contribution (before the right factor R): (I - d d^T) g_d d^T
        const float dg = d[0] * g_d[0] + d[1] * g_d[1] + d[2] * g_d[2];
        float gp[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) gp[k] = g_d[k] - d[k] * dg;
#pragma unroll
        for (int k = 0; k < 3; ++k) out[k] = w * g_o[k];
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
          for (int b = 0; b < 3; ++b) out[3 + 3 * a + b] = w * gp[a] * d[b];
      }
    }
  }
}

__device__ __forceinline__ void rodrigues(const double w[3], double R[3][3]) {
  // axis_angle_to_matrix (pytorch3d: through the unit quaternion (cos h, w sin(h)/|w|), h = |w| / 2)
  const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  const double h = 0.5 * th;
  const double sh = th < 1e-6 ? 0.5 - th * th / 48.0 : sin(h) / th;
  const double q[4] = {cos(h), w[0] * sh, w[1] * sh, w[2] * sh};
  const double n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  const double s = 2.0 / n2;
  const double r = q[0], i = q[1], j = q[2], k = q[3];
  R[0][0] = 1 - s * (j * j + k * k); R[0][1] = s * (i * j - k * r); R[0][2] = s * (i * k + j * r);
  R[1][0] = s * (i * j + k * r); R[1][1] = 1 - s * (i * i + k * k); R[1][2] = s * (j * k - i * r);
  R[2][0] = s * (i * k - j * r); R[2][1] = s * (j * k + i * r); R[2][2] = 1 - s * (i * i + j * j);
}

// One workgroup per keyframe: dL/dt and dL/d(axis-angle) of keyframe k from the rays' contributions.
__global__ void __launch_bounds__(kPoseThreads) k_pose_reduce(const float* __restrict__ ray_ws, int64_t n_rays,
                                                              const int64_t* __restrict__ slots, int64_t slot0,
                                                              const int32_t* __restrict__ slot_kf,
                                                              const float* __restrict__ pose6, float scale,
                                                              float* __restrict__ grad) {
  const int k = blockIdx.x;
  __shared__ double part[kPoseThreads][12];
  double acc[12];
#pragma unroll
  for (int c = 0; c < 12; ++c) acc[c] = 0.0;
  for (int64_t r = threadIdx.x; r < n_rays; r += kPoseThreads) {
    const int64_t slot = slots ? slots[r] : slot0 + r;
    if (slot_kf[slot] != k) continue;
#pragma unroll
    for (int c = 0; c < 12; ++c) acc[c] += (double)ray_ws[12 * r + c];
  }
#pragma unroll
  for (int c = 0; c < 12; ++c) part[threadIdx.x][c] = acc[c];
  __syncthreads();
  for (int s = kPoseThreads / 2; s > 0; s >>= 1) {  // fixed-order tree: deterministic
    if ((int)threadIdx.x < s)
#pragma unroll
      for (int c = 0; c < 12; ++c) part[threadIdx.x][c] += part[threadIdx.x + s][c];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const float* p = pose6 + 6 * k;
  const double w[3] = {p[3], p[4], p[5]};
  double R[3][3];
  rodrigues(w, R);
  // dL/dR = M R, M = sum (I - d d^T) g_d d^T
  double G[3][3];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) {
      double s = 0.0;
      for (int c = 0; c < 3; ++c) s += part[0][3 + 3 * a + c] * R[c][b];
      G[a][b] = s;
    }
  // dL/dw_i = sum_ab G_ab dR_ab/dw_i, dR/dw_i = (w_i [w]x + [w x ((I - R) e_i)]x) R / |w|^2 (Gallego & Yezzi,
  // J. Math. Imaging Vis. 2015); [e_i]x R's first-order form below |w| = 1e-6 (where R = I + [w]x + O(|w|^2))
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  for (int i = 0; i < 3; ++i) {
    double A[3][3];  // the skew-symmetric factor
    double v[3];
    if (th2 < 1e-12) {
      v[0] = v[1] = v[2] = 0.0;
      v[i] = 1.0;
    } else {
      double u[3];  // (I - R) e_i
      for (int a = 0; a < 3; ++a) u[a] = (a == i ? 1.0 : 0.0) - R[a][i];
      const double x[3] = {w[1] * u[2] - w[2] * u[1], w[2] * u[0] - w[0] * u[2], w[0] * u[1] - w[1] * u[0]};
      for (int a = 0; a < 3; ++a) v[a] = (w[i] * w[a] + x[a]) / th2;
    }
    A[0][0] = 0.0; A[0][1] = -v[2]; A[0][2] = v[1];
    A[1][0] = v[2]; A[1][1] = 0.0; A[1][2] = -v[0];
    A[2][0] = -v[1]; A[2][1] = v[0]; A[2][2] = 0.0;
    double s = 0.0;
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        double dr = 0.0;
        for (int c = 0; c < 3; ++c) dr += A[a][c] * R[c][b];
        s += G[a][b] * dr;
      }
    grad[6 * k + 3 + i] = (float)s;
  }
  for (int a = 0; a < 3; ++a) grad[6 * k + a] = (float)(part[0][a] / (double)scale);
}

__global__ void k_pose_adam(float* __restrict__ pose6, float* __restrict__ m, float* __restrict__ v,
                            const float* __restrict__ grad, const uint8_t* __restrict__ optimise, int32_t n_kf,
                            float one_minus_b1, float b2, float one_minus_b2, float step_size, float bc2_sqrt, float eps,
                            float* __restrict__ rows) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_kf) return;
  float* p = pose6 + 6 * k;
  if (grad != nullptr && (optimise == nullptr || optimise[k])) {
    for (int c = 0; c < 6; ++c) {  // torch.optim.Adam's foreach step (lnr_adam_step's arithmetic)
      const float g = grad[6 * k + c];
      float mm = m[6 * k + c], vv = v[6 * k + c];
      mm = mm + one_minus_b1 * (g - mm);
      vv = vv * b2 + one_minus_b2 * g * g;
      const float denom = sqrtf(vv) / bc2_sqrt + eps;
      p[c] = p[c] + (-step_size) * (mm / denom);
      m[6 * k + c] = mm;
      v[6 * k + c] = vv;
    }
  }
  if (rows) {
    const double w[3] = {p[3], p[4], p[5]};
    double R[3][3];
    rodrigues(w, R);
    float* o = rows + 12 * k;
    for (int a = 0; a < 3; ++a) {
      for (int b = 0; b < 3; ++b) o[4 * a + b] = (float)R[a][b];
      o[4 * a + 3] = p[a];
    }
  }
}

}  // namespace lnr

using namespace lnr;

extern "C" int lnr_pose_grad(const float* rays, const float* z, const float* d_pos, const float* d_ray, int64_t n_rays,
                             int32_t n_samples, const int64_t* slots, int64_t slot0, const int32_t* slot_kf,
                             const float* slot_pose, const float* pose6, int32_t n_kf, float scale, float far_range,
                             float* ray_ws, float* grad, void* stream) {
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && n_kf > 0 && scale > 0.f, "lnr_pose_grad: bad sizes");
  LNR_REQUIRE(grad && pose6 && slot_kf && slot_pose && (n_rays == 0 || (rays && z && d_pos && d_ray && ray_ws)),
              "lnr_pose_grad: null pointer");
  hipStream_t st = as_stream(stream);
  if (n_rays > 0) {
    const int64_t want = (n_rays + kPoseWaves - 1) / kPoseWaves;
    hipLaunchKernelGGL(k_pose_rays, dim3((unsigned)(want < 4096 ? want : 4096)), dim3(kPoseThreads), 0, st, rays, z,
                       d_pos, d_ray, n_rays, n_samples, slots, slot0, slot_pose, far_range, ray_ws);
  }
  hipLaunchKernelGGL(k_pose_reduce, dim3((unsigned)n_kf), dim3(kPoseThreads), 0, st, ray_ws, n_rays, slots, slot0,
                     slot_kf, pose6, scale, grad);
  LNR_RETURN_LAUNCH("lnr_pose_grad");
}

extern "C" int lnr_pose_adam(float* pose6, float* m, float* v, const float* grad, const uint8_t* optimise,
                             int32_t n_kf, int64_t step, float lr, float beta1, float beta2, float eps, float* rows,
                             void* stream) {
  LNR_REQUIRE(n_kf > 0 && (step >= 1 || grad == nullptr), "lnr_pose_adam: bad sizes");
  LNR_REQUIRE(pose6 && (grad == nullptr || (m && v)) && (grad || rows), "lnr_pose_adam: null pointer");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  hipLaunchKernelGGL(k_pose_adam, dim3((unsigned)((n_kf + 63) / 64)), dim3(64), 0, as_stream(stream), pose6, m, v, grad,
                     optimise, n_kf, 1.0f - beta1, beta2, 1.0f - beta2, (float)((double)lr / bc1), (float)sqrt(bc2), eps,
                     rows);
  LNR_RETURN_LAUNCH("lnr_pose_adam");
}
