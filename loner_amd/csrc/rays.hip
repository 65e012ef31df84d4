// On-device LiDAR ray selection and ray building: the per-step data preparation of
// Optimizer._do_iterate_optimizer (src/mapping/optimizer.py:363-424), which the reference runs on
// the CPU (data_prep_on_cpu, cfg/defaults.yaml:39) and copies to the GPU keyframe by keyframe.
//
//   selection  RANDOM  torch.randint(len(scan), (n,))                       optimizer.py:365-366
//              MASK    75 % of the slots from the "trunk" points (0.5 < z_sensor < 8 m), 25 % from
//                      the rest, each without replacement (randperm prefix)  optimizer.py:367-379
//              sky     torch.randint(0, n_sky_dirs, (num_samples.sky,))     optimizer.py:383-386
//   building   KeyFrame.build_lidar_rays (src/mapping/keyframe.py:75-105) ->
//              LidarRayDirections.build_lidar_rays (src/common/ray_utils.py:269-322) + get_far_val
//              (:31-60): 13-column rays, depth = range / scale, sky depth = r_max + 1
//              (keyframe.py:96), validity far > near + 1 m / scale (ray_utils.py:319-322).
//
// One thread per output slot.  The window's scans stay resident in HBM for the whole window; a
// step reads only the selected points (52 B of ray + 4 B of depth written per slot).  Draws come
// from the counter-based generator keyed by (step key, stream, keyframe, slot), so a rank that
// builds a slice of the slots gets exactly the rays the unsharded build puts there.
// "Without replacement" is a keyed Feistel permutation of [0, n) (cycle-walking on the next
// even power of two): slot j takes element perm(j), so slots never collide and each costs O(1).
#include "common.hpp"

namespace lnr {

enum : uint32_t { kStreamSelect = 5, kStreamSky = 6 };

__host__ __device__ __forceinline__ uint32_t ceil_log2_u32(uint32_t n) {
  uint32_t b = 0;
  while (b < 31 && (1u << b) < n) ++b;
  return b;
}

// Keyed permutation of [0, n), n >= 1: 4-round balanced Feistel network on 2h bits (2^(2h) >= n,
// h >= 1), cycle-walked back into range.  oracle/rays.py: feistel_perm.
__host__ __device__ __forceinline__ uint32_t feistel_perm(uint32_t j, uint32_t n, uint32_t key, uint32_t kf,
                                                          uint32_t part) {
  if (n <= 1u) return 0u;
  uint32_t bits = ceil_log2_u32(n);
  if (bits < 2) bits = 2;
  bits += bits & 1u;
  const uint32_t h = bits >> 1, mask = (1u << h) - 1u;
  uint32_t rk[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) rk[r] = rand_u32(key, kStreamSelect, kf, 0x80000000u | (part << 2) | (uint32_t)r);
  uint32_t x = j;
  do {  // terminates: x walks the permutation cycle that contains j < n
    uint32_t L = x >> h, R = x & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t F = mix32(R ^ rk[r]) & mask;
      const uint32_t nl = R;
      R = L ^ F;
      L = nl;
    }
    x = (L << h) | R;
  } while (x >= n);
  return x;
}

// torch.randint(0, n): an unbiased-enough multiply-shift of one 32-bit draw (n < 2^31).
__device__ __forceinline__ uint32_t draw_index(uint32_t key, uint32_t stream, uint32_t kf, uint32_t j, uint32_t n) {
  return (uint32_t)(((uint64_t)rand_u32(key, stream, kf, j) * (uint64_t)n) >> 32);
}

struct BuiltRay {
  float o[3], d[3], near_, far_, depth;
  bool valid;
};

// LidarRayDirections.build_lidar_rays for one point (ray_utils.py:284-322), fp32, op order of the
// reference's torch code (compiled with -ffp-contract=off).
__device__ __forceinline__ BuiltRay build_one(const lnr_ray_window& w, const float* P, float sx, float sy, float sz,
                                              float dist) {
  BuiltRay b;
  const float sc = w.scale;
  b.depth = dist / sc;
  b.o[0] = (P[3] + w.shift[0]) / sc;
  b.o[1] = (P[7] + w.shift[1]) / sc;
  b.o[2] = (P[11] + w.shift[2]) / sc;
  float d[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) d[r] = (P[4 * r + 0] * sx + P[4 * r + 1] * sy) + P[4 * r + 2] * sz;
  const float nrm = sqrtf((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
#pragma unroll
  for (int r = 0; r < 3; ++r) b.d[r] = d[r] / nrm;
  b.near_ = w.r_min / sc;
  const float far_range = w.r_max / sc;
  // get_far_val(no_nan=True): t = (+-1 - o) / (d + 1e-15), clamp(min=0), max over +-1, min over axes
  float far_clip = INFINITY;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const float dd = b.d[r] + 1e-15f;
    const float t0 = fmaxf((-1.0f - b.o[r]) / dd, 0.0f);
    const float t1 = fmaxf((1.0f - b.o[r]) / dd, 0.0f);
    far_clip = fminf(far_clip, fmaxf(t0, t1));
  }
  b.far_ = fminf(far_range, far_clip);
  b.valid = b.far_ > (b.near_ + 1.0f / sc);
  return b;
}

struct SlotPoint {
  const float* dir;
  float dist;
  int32_t local;
  int32_t kf;
};

// Which scan point feeds global slot g (selection rules above).
__device__ __forceinline__ SlotPoint slot_point(const lnr_ray_window& w, int32_t select, const int32_t* given,
                                                uint32_t key, int64_t g) {
  // keyframe k with ray_off[k] <= g < ray_off[k + 1]
  int32_t lo = 0, hi = w.n_kf;
  while (hi - lo > 1) {
    const int32_t mid = (lo + hi) >> 1;
    if ((int64_t)w.ray_off[mid] <= g) lo = mid;
    else hi = mid;
  }
  const int32_t k = lo;
  const uint32_t j = (uint32_t)(g - w.ray_off[k]);
  const uint32_t n_sel = (uint32_t)w.n_sel[k];
  SlotPoint p;
  p.kf = k;
  if (j < n_sel) {  // LiDAR point
    const int32_t s0 = w.scan_off[k];
    const uint32_t P = (uint32_t)(w.scan_off[k + 1] - s0);
    uint32_t loc;
    if (select == LNR_SELECT_GIVEN) {
      loc = (uint32_t)given[g];
    } else if (select == LNR_SELECT_ALL) {
      loc = j;
    } else if (select == LNR_SELECT_MASK) {
      const uint32_t nt = (uint32_t)w.n_trunk[k], ts = (uint32_t)w.n_sel_trunk[k];
      loc = j < ts ? (uint32_t)w.order[s0 + feistel_perm(j, nt, key, (uint32_t)k, 0u)]
                   : (uint32_t)w.order[s0 + nt + feistel_perm(j - ts, P - nt, key, (uint32_t)k, 1u)];
    } else {
      loc = draw_index(key, kStreamSelect, (uint32_t)k, j, P);
    }
    loc = loc < P ? loc : P - 1u;  // GIVEN indices out of range clamp instead of faulting (P >= 1: host check)
    p.local = (int32_t)loc;
    p.dir = w.dirs + 3 * ((int64_t)s0 + loc);
    p.dist = w.dists[s0 + loc];
  } else {  // sky ray: LidarScan.get_sky_scan(r_max + 1) (keyframe.py:96, sensors.py:164-167)
    const uint32_t js = j - n_sel;
    const int32_t q0 = w.sky_off[k];
    const uint32_t Q = (uint32_t)(w.sky_off[k + 1] - q0);
    uint32_t loc = select == LNR_SELECT_GIVEN ? (uint32_t)given[g]
                   : select == LNR_SELECT_ALL ? js
                                              : draw_index(key, kStreamSky, (uint32_t)k, js, Q);
    loc = loc < Q ? loc : Q - 1u;
    p.local = (int32_t)loc;
    p.dir = w.sky_dirs + 3 * ((int64_t)q0 + loc);
    p.dist = w.r_max + 1.0f;
  }
  return p;
}

// The per-keyframe tables (offsets, counts, poses) of windows of up to kKfLds keyframes are copied to
// LDS once per workgroup: a slot's keyframe search and its table reads then cost LDS latency, not a
// chain of dependent global loads (the kernel is latency-bound: a few thousand slots).
constexpr int kKfLds = 64;
struct KfTables {
  int32_t ray_off[kKfLds + 1], scan_off[kKfLds + 1], sky_off[kKfLds + 1];
  int32_t n_sel[kKfLds], n_trunk[kKfLds], n_sel_trunk[kKfLds];
  float poses[12 * kKfLds];
};

__global__ void __launch_bounds__(256) k_build_rays(lnr_ray_window w, int32_t select, const int32_t* __restrict__ given,
                                                    uint32_t key, int64_t slot0, int64_t n, float* __restrict__ rays,
                                                    float* __restrict__ depth, uint8_t* __restrict__ valid,
                                                    int32_t* __restrict__ point_index, float* __restrict__ far_ref) {
  if (w.dev_step) key = w.dev_step->key;  // graph replay: this step's key from device memory
  __shared__ KfTables tb;
  if (w.n_kf <= kKfLds) {  // (uniform)
    const int K = w.n_kf;
    for (int i = threadIdx.x; i <= K; i += blockDim.x) {
      tb.ray_off[i] = w.ray_off[i];
      tb.scan_off[i] = w.scan_off[i];
      if (w.sky_off) tb.sky_off[i] = w.sky_off[i];
      if (i < K) {
        tb.n_sel[i] = w.n_sel[i];
        if (w.n_trunk) tb.n_trunk[i] = w.n_trunk[i];
        if (w.n_sel_trunk) tb.n_sel_trunk[i] = w.n_sel_trunk[i];
      }
    }
    for (int i = threadIdx.x; i < 12 * K; i += blockDim.x) tb.poses[i] = w.poses[i];
    __syncthreads();
    w.ray_off = tb.ray_off;
    w.scan_off = tb.scan_off;
    w.n_sel = tb.n_sel;
    w.poses = tb.poses;
    if (w.sky_off) w.sky_off = tb.sky_off;
    if (w.n_trunk) w.n_trunk = tb.n_trunk;
    if (w.n_sel_trunk) w.n_sel_trunk = tb.n_sel_trunk;
  }
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (far_ref != nullptr && t == 0) {
    // far bound of the first valid ray of the whole batch (global ray 0 after the validity filter;
    // optimizer.py:724 compares every ray's depth with it)
    const int64_t total = w.ray_off[w.n_kf];
    float f = 0.f;
    for (int64_t g = 0; g < total; ++g) {
      const SlotPoint p = slot_point(w, select, given, key, g);
      const BuiltRay b = build_one(w, w.poses + 12 * p.kf, p.dir[0], p.dir[1], p.dir[2], p.dist);
      if (b.valid) {
        f = b.far_;
        break;
      }
    }
    far_ref[0] = f;
  }
  if (t >= n) return;
  const int64_t g = slot0 + t;
  const SlotPoint p = slot_point(w, select, given, key, g);
  const BuiltRay b = build_one(w, w.poses + 12 * p.kf, p.dir[0], p.dir[1], p.dir[2], p.dist);
  float* ry = rays + 13 * t;
  ry[0] = b.o[0];
  ry[1] = b.o[1];
  ry[2] = b.o[2];
  ry[3] = b.d[0];
  ry[4] = b.d[1];
  ry[5] = b.d[2];
  ry[6] = -b.d[0];
  ry[7] = -b.d[1];
  ry[8] = -b.d[2];
  ry[9] = 0.f;
  ry[10] = 0.f;
  ry[11] = b.near_;
  ry[12] = b.far_;
  depth[t] = b.depth;
  if (valid) valid[t] = b.valid ? 1 : 0;
  if (point_index) point_index[t] = p.local;
}

}  // namespace lnr

using namespace lnr;

extern "C" int lnr_build_lidar_rays(const lnr_ray_window* w, int32_t select, const int32_t* given, uint32_t key,
                                    int64_t slot0, int64_t n_slots, float* rays, float* depth, uint8_t* valid,
                                    int32_t* point_index, float* far_ref, void* stream) {
  LNR_REQUIRE(w != nullptr && w->n_kf >= 1, "lnr_build_lidar_rays: empty window");
  LNR_REQUIRE(select >= LNR_SELECT_RANDOM && select <= LNR_SELECT_GIVEN, "lnr_build_lidar_rays: bad select %d",
              select);
  LNR_REQUIRE(slot0 >= 0 && n_slots >= 0, "lnr_build_lidar_rays: bad slot range");
  LNR_REQUIRE(w->scale > 0.f, "lnr_build_lidar_rays: world-cube scale must be positive");
  LNR_REQUIRE(w->poses && w->dirs && w->dists && w->scan_off && w->ray_off && w->n_sel,
              "lnr_build_lidar_rays: null window array");
  LNR_REQUIRE(select != LNR_SELECT_MASK || (w->order && w->n_trunk && w->n_sel_trunk),
              "lnr_build_lidar_rays: MASK selection needs order / n_trunk / n_sel_trunk");
  LNR_REQUIRE(select != LNR_SELECT_GIVEN || given != nullptr, "lnr_build_lidar_rays: GIVEN selection needs indices");
  LNR_REQUIRE(n_slots == 0 || (rays && depth), "lnr_build_lidar_rays: null output");
  if (n_slots == 0 && far_ref == nullptr) return LNR_OK;
  const unsigned blocks = (unsigned)((n_slots + 255) / 256 > 0 ? (n_slots + 255) / 256 : 1);
  hipLaunchKernelGGL(k_build_rays, dim3(blocks), dim3(256), 0, as_stream(stream), *w, select, given, key, slot0,
                     n_slots, rays, depth, valid, point_index, far_ref);
  LNR_RETURN_LAUNCH("lnr_build_lidar_rays");
}

// ------------------------------------------------------------------ camera rays
// KeyFrame.build_camera_rays -> CameraRayDirections.build_rays (src/mapping/keyframe.py:108-127,
// src/common/ray_utils.py:175-212): pixel p = j * W + i of the undistorted per-pixel directions
// table, rotated by the camera pose, normalised; origin = (t + shift) / scale; view direction = -d;
// near = r_min / scale; far = get_far_val(o, d, no_nan=True) (NOT clipped by r_max here); the
// intensities are the image row p.  fp32 in the reference's operation order.
__device__ __forceinline__ void camera_ray(const lnr_camera_desc& cam, const float* __restrict__ dirs,
                                           const float* __restrict__ image, int64_t p, int64_t k,
                                           float* __restrict__ rays, float* __restrict__ intens) {
  const float sc = cam.scale;
  float o[3], d[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) o[r] = (cam.pose[4 * r + 3] + cam.shift[r]) / sc;
  const float dx = dirs[3 * p + 0], dy = dirs[3 * p + 1], dz = dirs[3 * p + 2];
#pragma unroll
  for (int r = 0; r < 3; ++r) d[r] = (dx * cam.pose[4 * r + 0] + dy * cam.pose[4 * r + 1]) + dz * cam.pose[4 * r + 2];
  const float nrm = sqrtf((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
#pragma unroll
  for (int r = 0; r < 3; ++r) d[r] = d[r] / nrm;
  float far_clip = INFINITY;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const float dd = d[r] + 1e-15f;
    const float t0 = fmaxf((-1.0f - o[r]) / dd, 0.0f);
    const float t1 = fmaxf((1.0f - o[r]) / dd, 0.0f);
    far_clip = fminf(far_clip, fmaxf(t0, t1));
  }
  float* ry = rays + 13 * k;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    ry[r] = o[r];
    ry[3 + r] = d[r];
    ry[6 + r] = -d[r];
  }
  ry[9] = (float)(p % cam.width);
  ry[10] = (float)(p / cam.width);
  ry[11] = cam.r_min / sc;
  ry[12] = far_clip;
  if (intens)
    for (int c = 0; c < cam.channels; ++c) intens[k * cam.channels + c] = image[p * cam.channels + c];
}

__global__ void __launch_bounds__(256) k_build_camera_rays(lnr_camera_desc cam, const float* __restrict__ dirs,
                                                           const float* __restrict__ image,
                                                           const int64_t* __restrict__ pixels, int64_t n,
                                                           float* __restrict__ rays, float* __restrict__ intens) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  camera_ray(cam, dirs, image, pixels[k], k, rays, intens);
}

// every frame of a camera window in one launch: frame f's slots [f n_per, (f + 1) n_per) take its
// pixels[f stride + first + j]
__global__ void __launch_bounds__(256) k_build_camera_rays_window(const lnr_camera_frame* __restrict__ frames,
                                                                  int32_t n_frames, const float* __restrict__ dirs,
                                                                  const int64_t* __restrict__ pixels, int64_t stride,
                                                                  int64_t first, int64_t n_per,
                                                                  float* __restrict__ rays, float* __restrict__ intens) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (int64_t)n_frames * n_per) return;
  const int64_t f = k / n_per, j = k - f * n_per;
  const lnr_camera_frame fr = frames[f];
  camera_ray(fr.cam, dirs, fr.image, pixels[f * stride + first + j], k, rays, intens);
}

extern "C" int lnr_build_camera_rays(const lnr_camera_desc* cam, const float* dirs, const float* image,
                                     const int64_t* pixels, int64_t n, float* rays, float* intensities,
                                     void* stream) {
  LNR_REQUIRE(cam != nullptr && n >= 0, "lnr_build_camera_rays: bad arguments");
  LNR_REQUIRE(cam->width > 0 && cam->height > 0 && cam->channels > 0 && cam->scale > 0.f,
              "lnr_build_camera_rays: bad camera description");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(dirs && pixels && rays && (intensities == nullptr || image), "lnr_build_camera_rays: null pointer");
  hipLaunchKernelGGL(k_build_camera_rays, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), *cam,
                     dirs, image, pixels, n, rays, intensities);
  LNR_RETURN_LAUNCH("lnr_build_camera_rays");
}

extern "C" int lnr_build_camera_rays_window(const lnr_camera_frame* frames, int32_t n_frames, const float* dirs,
                                            const int64_t* pixels, int64_t stride, int64_t first, int64_t n_per_frame,
                                            float* rays, float* intensities, void* stream) {
  LNR_REQUIRE(n_frames >= 0 && n_per_frame >= 0 && first >= 0 && first + n_per_frame <= stride,
              "lnr_build_camera_rays_window: bad sizes");
  const int64_t n = (int64_t)n_frames * n_per_frame;
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(frames && dirs && pixels && rays, "lnr_build_camera_rays_window: null pointer");
  hipLaunchKernelGGL(k_build_camera_rays_window, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                     frames, n_frames, dirs, pixels, stride, first, n_per_frame, rays, intensities);
  LNR_RETURN_LAUNCH("lnr_build_camera_rays_window");
}
