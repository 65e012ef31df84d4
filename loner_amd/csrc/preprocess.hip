// Per-keyframe scan preprocessing of the north-star driver, on the device
// (examples/fdt_optimize_implicit_map.py:594-607, once per keyframe before it joins the window):
//
//   lnr_motion_compensate   LidarScan.motion_compensate (src/common/sensors.py:169-231): each point
//                           is re-expressed in the target frame from the sensor pose interpolated at
//                           its timestamp (translation lerp, rotation start_R * exp(s * log(R0^T R1))).
//   lnr_sky_rays            compute_sky_rays (examples/fdt_optimize_implicit_map_utils.py:38-77): the
//                           scan's (elevation x azimuth) occupancy image at 1-degree bins, closed by a
//                           3x3 dilation + erosion (kornia.morphology, geodesic borders), top 3 rows
//                           forced occupied; each empty bin becomes a direction, rotated by the pose
//                           rotation, kept when more than 10 degrees above the horizon.
//
// The reference runs both through torch (+ pytorch3d / kornia) per keyframe; here the motion
// compensation is one elementwise kernel and the sky image lives in one workgroup's LDS (at most
// 181 x 360 one-byte bins; occupancy, dilation and closing as bits of one byte), so a scan's sky rays cost one single-workgroup launch.
#include "common.hpp"

namespace lnr {

// ------------------------------------------------------------------ motion compensation
__device__ __forceinline__ void rodrigues(const float* axis, float ang, float (&R)[9]) {
  const float c = cosf(ang), s = sinf(ang), t = 1.0f - c;
  const float x = axis[0], y = axis[1], z = axis[2];
  R[0] = t * x * x + c;     R[1] = t * x * y - s * z; R[2] = t * x * z + s * y;
  R[3] = t * x * y + s * z; R[4] = t * y * y + c;     R[5] = t * y * z - s * x;
  R[6] = t * x * z - s * y; R[7] = t * y * z + s * x; R[8] = t * z * z + c;
}

__global__ void __launch_bounds__(256) k_motion_compensate(lnr_motion_comp mc, const float* __restrict__ ts,
                                                           float* __restrict__ dirs, float* __restrict__ dists,
                                                           int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float s = (ts[i] - mc.t0) / (mc.t1 - mc.t0);
  float Ri[9];
  if (mc.identity) {
    for (int k = 0; k < 9; ++k) Ri[k] = (k % 4 == 0) ? 1.f : 0.f;
  } else {
    rodrigues(mc.axis, mc.angle * s, Ri);
  }
  float R[9];  // start_R @ R_interp
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      R[3 * r + c] = mc.start_rot[3 * r + 0] * Ri[c] + mc.start_rot[3 * r + 1] * Ri[3 + c] + mc.start_rot[3 * r + 2] * Ri[6 + c];
  float t[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) t[k] = mc.delta_t[k] * s + mc.start_t[k];
  const float d = dists[i];
  const float p[3] = {dirs[3 * i + 0] * d, dirs[3 * i + 1] * d, dirs[3 * i + 2] * d};
  float w[3];  // world = R p + t
#pragma unroll
  for (int r = 0; r < 3; ++r) w[r] = R[3 * r + 0] * p[0] + R[3 * r + 1] * p[1] + R[3 * r + 2] * p[2] + t[r];
  float q[3];  // target frame = inv(T_world_to_target) w
#pragma unroll
  for (int r = 0; r < 3; ++r)
    q[r] = mc.target_inv[4 * r + 0] * w[0] + mc.target_inv[4 * r + 1] * w[1] + mc.target_inv[4 * r + 2] * w[2] +
           mc.target_inv[4 * r + 3];
  const float nrm = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
  dists[i] = nrm;
#pragma unroll
  for (int k = 0; k < 3; ++k) dirs[3 * i + k] = q[k] / nrm;
}

// ------------------------------------------------------------------ sky rays
constexpr int kSkyRows = 181, kSkyCols = 360, kSkyThreads = 1024;

__device__ __forceinline__ void sky_bins(const float* d, int& theta, int& phi) {
  const float x = d[0], y = d[1], z = d[2];
  constexpr float kDeg = 57.29577951308232f;  // torch.rad2deg
  theta = (int)rintf(atan2f(y, x) * kDeg);     // .round(): half to even
  phi = (int)rintf(atan2f(sqrtf(x * x + y * y), z) * kDeg);
}

__global__ void __launch_bounds__(kSkyThreads) k_sky_rays(const float* __restrict__ dirs, int64_t n, lnr_sky_params sp,
                                                          float* __restrict__ out, int64_t cap, int32_t* count) {
  __shared__ uint8_t img[kSkyRows * kSkyCols];  // bit 0 occupied, bit 1 dilated, bit 2 closed
  __shared__ int32_t red[3][kSkyThreads / 64];
  __shared__ int32_t wsum[kSkyThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  // 1. bin ranges
  int pmin = 1 << 30, pmax = -(1 << 30), tmin = 1 << 30;
  for (int64_t i = t; i < n; i += kSkyThreads) {
    int th, ph;
    sky_bins(dirs + 3 * i, th, ph);
    pmin = min(pmin, ph);
    pmax = max(pmax, ph);
    tmin = min(tmin, th);
  }
  for (int o = 32; o >= 1; o >>= 1) {
    pmin = min(pmin, __shfl_xor(pmin, o, 64));
    pmax = max(pmax, __shfl_xor(pmax, o, 64));
    tmin = min(tmin, __shfl_xor(tmin, o, 64));
  }
  if (lane == 0) {
    red[0][wid] = pmin;
    red[1][wid] = pmax;
    red[2][wid] = tmin;
  }
  for (int k = t; k < kSkyRows * kSkyCols; k += kSkyThreads) img[k] = 0;
  __syncthreads();
  pmin = red[0][0];
  pmax = red[1][0];
  tmin = red[2][0];
  for (int w = 1; w < kSkyThreads / 64; ++w) {
    pmin = min(pmin, red[0][w]);
    pmax = max(pmax, red[1][w]);
    tmin = min(tmin, red[2][w]);
  }
  const int H = pmax - pmin + 1;  // <= 181 (phi in [0, 180])
  // 2. occupied bins (theta_img == 360 wraps to 0)
  for (int64_t i = t; i < n; i += kSkyThreads) {
    int th, ph;
    sky_bins(dirs + 3 * i, th, ph);
    int c = th - tmin;
    if (c == 360) c = 0;
    img[(ph - pmin) * kSkyCols + c] = 1;
  }
  __syncthreads();
  // 3. 3x3 dilation then erosion, geodesic borders (out-of-image neighbours ignored)
  for (int k = t; k < H * kSkyCols; k += kSkyThreads) {
    const int r = k / kSkyCols, c = k % kSkyCols;
    uint8_t m = 0;
    for (int dr = -1; dr <= 1; ++dr)
      for (int dc = -1; dc <= 1; ++dc) {
        const int rr = r + dr, cc = c + dc;
        if (rr >= 0 && rr < H && cc >= 0 && cc < kSkyCols) m = max(m, (uint8_t)(img[rr * kSkyCols + cc] & 1u));
      }
    img[k] |= (uint8_t)(m << 1);
  }
  __syncthreads();
  for (int k = t; k < H * kSkyCols; k += kSkyThreads) {
    const int r = k / kSkyCols, c = k % kSkyCols;
    uint8_t m = 1;
    for (int dr = -1; dr <= 1; ++dr)
      for (int dc = -1; dc <= 1; ++dc) {
        const int rr = r + dr, cc = c + dc;
        if (rr >= 0 && rr < H && cc >= 0 && cc < kSkyCols) m = min(m, (uint8_t)((img[rr * kSkyCols + cc] >> 1) & 1u));
      }
    img[k] |= (uint8_t)(((r < sp.top_rows) ? 1 : m) << 2);  // depth_img[:TOP_ROWS] = 1
  }
  __syncthreads();
  // 4. empty bins -> directions -> world rotation -> elevation filter, compacted in row-major order
  const int total = H * kSkyCols;
  const int per = (total + kSkyThreads - 1) / kSkyThreads;
  const int k0 = t * per;
  auto dir_of = [&](int k, float (&o)[3]) -> bool {
    const int r = k / kSkyCols, c = k % kSkyCols;
    constexpr float kRad = 0.017453292519943295f;  // torch.deg2rad
    const float ph = (float)(r + pmin) * kRad, th = (float)(c + tmin) * kRad;
    const float z = cosf(ph), y = sinf(ph) * sinf(th), x = sinf(ph) * cosf(th);
#pragma unroll
    for (int q = 0; q < 3; ++q) o[q] = sp.rot[3 * q + 0] * x + sp.rot[3 * q + 1] * y + sp.rot[3 * q + 2] * z;
    const float phw = 90.0f - atan2f(sqrtf(o[0] * o[0] + o[1] * o[1]), o[2]) * 57.29577951308232f;
    return phw > sp.horizon_deg;
  };
  int cnt = 0;
  for (int k = k0; k < k0 + per && k < total; ++k) {
    float o[3];
    if (!(img[k] & 4u) && dir_of(k, o)) ++cnt;
  }
  int inc = cnt;
  for (int o = 1; o < 64; o <<= 1) {
    const int q = __shfl_up(inc, o, 64);
    if (lane >= o) inc += q;
  }
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wid; ++w) base += wsum[w];
  int pos = base + inc - cnt;
  for (int k = k0; k < k0 + per && k < total; ++k) {
    float o[3];
    if (!(img[k] & 4u) && dir_of(k, o)) {
      if (pos < cap) {
        out[3 * pos + 0] = o[0];
        out[3 * pos + 1] = o[1];
        out[3 * pos + 2] = o[2];
      }
      ++pos;
    }
  }
  if (t == kSkyThreads - 1) count[0] = pos;
}

}  // namespace lnr

using namespace lnr;

extern "C" int lnr_motion_compensate(const lnr_motion_comp* mc, const float* timestamps, float* dirs, float* dists,
                                     int64_t n_points, void* stream) {
  LNR_REQUIRE(mc != nullptr && n_points >= 0, "lnr_motion_compensate: bad arguments");
  LNR_REQUIRE(mc->t1 != mc->t0, "lnr_motion_compensate: start and end timestamps are equal");
  if (n_points == 0) return LNR_OK;
  LNR_REQUIRE(timestamps && dirs && dists, "lnr_motion_compensate: null pointer");
  hipLaunchKernelGGL(k_motion_compensate, dim3((unsigned)((n_points + 255) / 256)), dim3(256), 0, as_stream(stream),
                     *mc, timestamps, dirs, dists, n_points);
  LNR_RETURN_LAUNCH("lnr_motion_compensate");
}

extern "C" int64_t lnr_sky_rays_capacity(void) { return (int64_t)kSkyRows * kSkyCols; }

extern "C" int lnr_sky_rays(const float* dirs, int64_t n_points, const lnr_sky_params* sp, float* out, int64_t cap,
                            int32_t* count, void* stream) {
  LNR_REQUIRE(sp != nullptr && n_points >= 1, "lnr_sky_rays: needs at least one scan point");
  LNR_REQUIRE(dirs && out && count && cap >= 0, "lnr_sky_rays: null pointer");
  hipLaunchKernelGGL(k_sky_rays, dim3(1), dim3(kSkyThreads), 0, as_stream(stream), dirs, n_points, *sp, out, cap,
                     count);
  LNR_RETURN_LAUNCH("lnr_sky_rays");
}
