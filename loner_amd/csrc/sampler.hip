// Per-ray depth sampling: stratified (jittered) + occupancy-grid importance sampling, sorted.
//
// Reference: OccGridRaySampler.get_samples   src/models/ray_sampling.py:53-92
//            UniformRaySampler.get_samples   src/models/ray_sampling.py:22-43
//            OccupancyGridModel.interpolate  src/models/model_tcnn.py:126-134 (grid_sample 3-D,
//                                            trilinear, align_corners=False, zeros padding)
//            sample_pdf                      src/models/rendering_tcnn.py:19-68 (det=False)
// One 256-thread workgroup per ray (grid-stride over rays).  The 100^3 fp32 occupancy grid (4 MB)
// stays L2/MALL resident; the cdf, bins and the bitonic sort buffer live in LDS.
#include "common.hpp"

namespace lnr {

constexpr int SNT = 256;

__device__ __forceinline__ float linspace01(int i, int n) {
  // torch linspace(0, 1, n): start + step*i for i < n/2, end - step*(n-1-i) otherwise
  const float step = 1.0f / (float)(n - 1);
  return (i < n / 2) ? (0.0f + step * (float)i) : (1.0f - step * (float)(n - 1 - i));
}

struct SamplerArgs {
  const float* rays;
  int64_t n_rays;
  int32_t S;       // total samples per ray
  int32_t H;       // stratified samples (S/2 for OGM, S for uniform)
  const float* occ;
  int32_t occ_res;
  float perturb;
  const float* u_jitter;
  const float* u_pdf;
  uint32_t key;
  int64_t ray_offset;
  float* z;
  int32_t P2;      // next power of two >= S (sort width)
  const lnr_step_scalars* dev_step;  // optional: the key from device memory (graph replay)
};

template <bool OGM>
__global__ void __launch_bounds__(SNT) k_sampler(SamplerArgs a) {
  if (a.dev_step) a.key = a.dev_step->key;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* zs = reinterpret_cast<float*>(smem);  // [H] stratified (jittered)
  float* cdf = zs + a.H;                       // [H-1]
  float* prob = cdf + a.H;                     // [H]
  float* buf = prob + a.H;                     // [P2] sort buffer
  double* red = reinterpret_cast<double*>(smem + ((((size_t)3 * a.H + a.P2) * 4 + 7) & ~(size_t)7));  // [SNT/64+2]
  const int H = a.H, S = a.S, t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  for (int64_t r = blockIdx.x; r < a.n_rays; r += gridDim.x) {
    const float* ry = a.rays + 13 * r;
    const float near = ry[11], far = ry[12];
    const uint32_t gr = (uint32_t)(a.ray_offset + r);
    // 1. linspace + jitter (ray_sampling.py:59-72)
    for (int i = t; i < H; i += SNT) {
      const float tt = linspace01(i, H);
      zs[i] = near * (1.0f - tt) + far * tt;
    }
    __syncthreads();
    float zj[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = t + k * SNT;
      float z = 0.f;
      if (i < H) {
        z = zs[i];
        if (a.perturb > 0.f) {
          const float zl = zs[i > 0 ? i - 1 : 0], zu = zs[i + 1 < H ? i + 1 : H - 1];
          const float upper = (i + 1 < H) ? 0.5f * (z + zu) : z;
          const float lower = (i > 0) ? 0.5f * (zl + z) : z;
          const float u = a.u_jitter ? a.u_jitter[r * H + i] : rand_uniform(a.key, kStreamJitter, gr, (uint32_t)i);
          z = lower + (upper - lower) * (a.perturb * u);
        }
      }
      zj[k] = z;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = t + k * SNT;
      if (i < H) zs[i] = zj[k];
    }
    __syncthreads();
    if (!OGM) {
      for (int i = t; i < S; i += SNT) a.z[r * S + i] = zs[i];
      __syncthreads();
      continue;
    }
    // 2. occupancy probabilities at the stratified points (ray_sampling.py:74-81)
    for (int i = t; i < H; i += SNT) {
      const float z = zs[i];
      const float px = ry[0] + ry[3] * z, py = ry[1] + ry[4] * z, pz = ry[2] + ry[5] * z;
      const float l = occ_grid_sample(a.occ, a.occ_res, px, py, pz);
      float p = 1.0f / (1.0f + expf(-l));
      p = 2.0f * (fminf(fmaxf(p, 0.5f), 1.0f) - 0.5f);
      prob[i] = p;
    }
    __syncthreads();
    // 3. sample_pdf over bins = midpoints (H-1), weights = prob[1:H-1] (H-2 values) + 1e-5
    const int M = H - 2;
    double wsum = 0.0;
    for (int i = t; i < M; i += SNT) wsum += (double)(prob[i + 1] + 1e-5f);
    {
      float v[1] = {(float)wsum};
      // block sum in float of per-thread doubles (reference: torch.sum fp32)
      block_sum<SNT, 1>(v, reinterpret_cast<float*>(red));
      wsum = v[0];
    }
    const float wtot = (float)wsum;
    // inclusive cumsum of pdf in double, per contiguous chunk per thread
    const int K = (M + SNT - 1) / SNT;
    const int j0 = t * K;
    double loc = 0.0;
    for (int k = 0; k < K; ++k) {
      const int j = j0 + k;
      if (j < M) loc += (double)((prob[j + 1] + 1e-5f) / wtot);
    }
    double inc = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      double q = __shfl_up(inc, o, 64);
      if (lane >= o) inc += q;
    }
    if (lane == 63) red[wid] = inc;
    __syncthreads();
    double pre = 0.0;
    for (int w = 0; w < wid; ++w) pre += red[w];
    double run = pre + inc - loc;
    for (int k = 0; k < K; ++k) {
      const int j = j0 + k;
      if (j < M) {
        run += (double)((prob[j + 1] + 1e-5f) / wtot);
        cdf[j + 1] = (float)run;
      }
    }
    if (t == 0) cdf[0] = 0.f;
    __syncthreads();
    // bins (midpoints of the jittered stratified depths) reuse prob[]
    for (int i = t; i < H - 1; i += SNT) prob[i] = 0.5f * (zs[i] + zs[i + 1]);
    __syncthreads();
    // 4. inverse CDF (searchsorted right=True over H-1 cdf entries)
    for (int i = t; i < H; i += SNT) {
      const float u = a.u_pdf ? a.u_pdf[r * H + i] : rand_uniform(a.key, kStreamPdf, gr, (uint32_t)i);
      int lo = 0, hi = H - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cdf[mid] <= u) lo = mid + 1;
        else hi = mid;
      }
      const int below = lo - 1 > 0 ? lo - 1 : 0;
      const int above = lo < M ? lo : M;
      const float c0 = cdf[below], c1 = cdf[above];
      const float b0 = prob[below], b1 = prob[above];
      float denom = c1 - c0;
      if (denom < 1e-5f) denom = 1.0f;
      buf[H + i] = b0 + (u - c0) / denom * (b1 - b0);
      buf[i] = zs[i];
    }
    for (int i = S + t; i < a.P2; i += SNT) buf[i] = INFINITY;
    __syncthreads();
    // 5. bitonic sort of P2 values (torch.sort(..., -1), ray_sampling.py:90)
    for (int k = 2; k <= a.P2; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int q = t; q < a.P2 / 2; q += SNT) {
          const int i = 2 * j * (q / j) + (q % j);
          const int l = i + j;
          const bool up = (i & k) == 0;
          const float x = buf[i], y = buf[l];
          if ((x > y) == up) {
            buf[i] = y;
            buf[l] = x;
          }
        }
        __syncthreads();
      }
    }
    for (int i = t; i < S; i += SNT) a.z[r * S + i] = buf[i];
    __syncthreads();
  }
}


// ---------------------------------------------------------------------------------------------
// OGM sampler, one wave per ray (S/2 a multiple of 64, next power of two of S <= 2048): no
// workgroup barriers.  Lane l owns the stratified indices [l*Q, (l+1)*Q) (Q = S/128); the cdf and
// the bins live in this wave's LDS slice; the S depths are sorted by a bitonic network in registers
// (E = P2/64 per lane, lane l holding sorted positions [l*E, (l+1)*E)): in-lane exchanges for
// distances < E, __shfl_xor across lanes for the rest.  Same arithmetic as k_sampler<true>.
template <int E>
__device__ __forceinline__ void wave_bitonic_sort(float (&v)[E]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 2; k <= 64 * E; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= E) {  // partner in lane ^ (j / E), same register
        const int dl = j / E;
        const bool lower = (lane & dl) == 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int pos = lane * E + e;
          const bool up = (pos & k) == 0;
          const float o = __shfl_xor(v[e], dl, 64);
          // the lower position keeps the min when ascending
          v[e] = (lower == up) ? fminf(v[e], o) : fmaxf(v[e], o);
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if ((e & j) == 0) {
            const int pos = lane * E + e;
            const bool up = (pos & k) == 0;
            const float x = v[e], y = v[e + j];
            v[e] = up ? fminf(x, y) : fmaxf(x, y);
            v[e + j] = up ? fmaxf(x, y) : fminf(x, y);
          }
        }
      }
    }
  }
}

// The last stage of the bitonic sort alone: a bitonic sequence of 64 E values (ascending, then
// descending) merged into ascending order, the same compare-exchanges as wave_bitonic_sort's stage
// k = 64 E.
template <int E>
__device__ __forceinline__ void wave_bitonic_merge(float (&v)[E]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 32 * E; j > 0; j >>= 1) {
    if (j >= E) {
      const int dl = j / E;
      const bool lower = (lane & dl) == 0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float o = __shfl_xor(v[e], dl, 64);
        v[e] = lower ? fminf(v[e], o) : fmaxf(v[e], o);
      }
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if ((e & j) == 0) {
          const float x = v[e], y = v[e + j];
          v[e] = fminf(x, y);
          v[e + j] = fmaxf(x, y);
        }
      }
    }
  }
}

#ifndef LNR_SAMPLER_MERGE
// LONER_SAMPLER_MERGE: 0 the full bitonic sort; 1 the importance draws' bitonic sort + one merge stage with the
// strata; 2 (default) the draws sorted before the inverse CDF, merged by rank (k_sampler_rank, from 4 depths
// per lane; 2 per lane fall back to 1)
#define LNR_SAMPLER_MERGE 2
#endif
#ifndef LNR_SAMPLER_RANK_MIN_RAYS
// fewest rays for the rank merge (smaller launches take the bitonic merge).  With both forms' occupancy lookups
// lane-contiguous: C4 shard of 8 (1152 rays) 0.0246 ms either way, C2 0.053 -> 0.049, C3 0.178 -> 0.160
#define LNR_SAMPLER_RANK_MIN_RAYS 0
#endif
static int64_t sampler_rank_min_rays() {  // LONER_SAMPLER_RANK_MIN_RAYS, read at every launch
  const char* e = getenv("LONER_SAMPLER_RANK_MIN_RAYS");
  return e ? atoll(e) : (int64_t)LNR_SAMPLER_RANK_MIN_RAYS;
}
static int sampler_merge() {  // read at every launch
  const char* e = getenv("LONER_SAMPLER_MERGE");
  return e ? atoi(e) : LNR_SAMPLER_MERGE;
}

constexpr int kSamplerWaves = 4;

template <int E, bool MERGE>
__global__ void __launch_bounds__(64 * kSamplerWaves) k_sampler_wave(SamplerArgs a) {
  if (a.dev_step) a.key = a.dev_step->key;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int QMAX = E / 2;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int H = a.H, S = a.S, Q = H / 64, M = H - 2;
  float* base = reinterpret_cast<float*>(smem) + (size_t)wid * (64 * E + 2 * H);
  float* buf = base;              // [P2] stratified, then importance, then +inf padding
  float* cdf = base + 64 * E;     // [H - 1]
  float* bins = cdf + H;          // [H - 1]
  for (int64_t r = (int64_t)blockIdx.x * kSamplerWaves + wid; r < a.n_rays; r += (int64_t)gridDim.x * kSamplerWaves) {
    const float* ry = a.rays + 13 * r;
    const float near = ry[11], far = ry[12];
    const float ox = ry[0], oy = ry[1], oz = ry[2], dx = ry[3], dy = ry[4], dz = ry[5];
    const uint32_t gr = (uint32_t)(a.ray_offset + r);
    // 1. linspace + jitter (ray_sampling.py:59-72); neighbours recomputed, not exchanged.  Computed
    // lane-contiguous (stratum 64 q + lane: one gather instruction's lanes read neighbouring strata, mostly the
    // same voxels), then transposed through LDS (bins: free until step 3) to this lane's range [l Q, (l + 1) Q)
    for (int q = 0; q < Q; ++q) {
      const int i = q * 64 + lane;
      const float tt = linspace01(i, H);
      float z = near * (1.0f - tt) + far * tt;
      if (a.perturb > 0.f) {
        const float tl = linspace01(i > 0 ? i - 1 : 0, H), tu = linspace01(i + 1 < H ? i + 1 : H - 1, H);
        const float zl = near * (1.0f - tl) + far * tl, zu = near * (1.0f - tu) + far * tu;
        const float upper = (i + 1 < H) ? 0.5f * (z + zu) : z;
        const float lower = (i > 0) ? 0.5f * (zl + z) : z;
        const float u = a.u_jitter ? a.u_jitter[r * H + i] : rand_uniform(a.key, kStreamJitter, gr, (uint32_t)i);
        z = lower + (upper - lower) * (a.perturb * u);
      }
      buf[i] = z;
      // 2. occupancy probability (ray_sampling.py:74-81)
      const float l = occ_grid_sample(a.occ, a.occ_res, ox + dx * z, oy + dy * z, oz + dz * z);
      float p = 1.0f / (1.0f + expf(-l));
      p = 2.0f * (fminf(fmaxf(p, 0.5f), 1.0f) - 0.5f);
      bins[i] = p;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
    float zq[QMAX], pq[QMAX];
    double wl = 0.0;
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      if (q >= Q) break;
      const int i = lane * Q + q;
      zq[q] = buf[i];
      pq[q] = bins[i];
      if (i >= 1 && i <= M) wl += (double)(pq[q] + 1e-5f);  // weights = prob[1:-1] + eps
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");  // (bins is rewritten in step 3)
    // 3. sample_pdf (rendering_tcnn.py:19-68): wtot, cdf = cumsum(pdf) in double
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) wl += __shfl_xor(wl, o, 64);
    const float wtot = (float)wl;
    double loc = 0.0;
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      if (q >= Q) break;
      const int i = lane * Q + q;
      if (i >= 1 && i <= M) loc += (double)((pq[q] + 1e-5f) / wtot);
    }
    double inc = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    double run = inc - loc;
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      if (q >= Q) break;
      const int i = lane * Q + q;
      if (i >= 1 && i <= M) {
        run += (double)((pq[q] + 1e-5f) / wtot);
        cdf[i] = (float)run;
      }
    }
    if (lane == 0) cdf[0] = 0.f;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    // bins = midpoints of the jittered stratified depths (needs the next lane's first depth)
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      if (q >= Q) break;
      const int i = lane * Q + q;
      if (i < H - 1) bins[i] = 0.5f * (zq[q] + buf[i + 1]);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
    // 4. inverse CDF, searchsorted(cdf, u, right=True)
    for (int i = lane; i < H; i += 64) {
      const float u = a.u_pdf ? a.u_pdf[r * H + i] : rand_uniform(a.key, kStreamPdf, gr, (uint32_t)i);
      int lo = 0, hi = H - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cdf[mid] <= u) lo = mid + 1;
        else hi = mid;
      }
      const int below = lo - 1 > 0 ? lo - 1 : 0;
      const int above = lo < M ? lo : M;
      const float c0 = cdf[below], c1 = cdf[above];
      const float b0 = bins[below], b1 = bins[above];
      float denom = c1 - c0;
      if (denom < 1e-5f) denom = 1.0f;
      buf[H + i] = b0 + (u - c0) / denom * (b1 - b0);
    }
    for (int i = S + lane; i < 64 * E; i += 64) buf[i] = INFINITY;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
    // 5. sort (torch.sort, ray_sampling.py:90) and store
    float v[E];
    if constexpr (MERGE) {
    // the jittered strata are ascending unless rounding crossed two of them (checked, wave-uniform):
    // then only the H importance draws need sorting, and one bitonic merge stage finishes the sort.
    // Same values in the same places as the full sort (depths are positive: no -0 / NaN ties)
    bool strat_sorted = 2 * H == 64 * E;  // no padding
    {
      float prev = -INFINITY;
#pragma unroll
      for (int q = 0; q < QMAX; ++q) {
        if (q >= Q) break;
        strat_sorted = strat_sorted && !(zq[q] < prev);
        prev = zq[q];
      }
      const float next_first = __shfl_down(zq[0], 1, 64);
      if (lane < 63) strat_sorted = strat_sorted && !(next_first < prev);
    }
    if (__all(strat_sorted)) {
      constexpr int E2 = E / 2;
      float vi[E2];
#pragma unroll
      for (int e = 0; e < E2; ++e) vi[e] = buf[H + lane * E2 + e];
      wave_bitonic_sort<E2>(vi);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
#pragma unroll
      for (int e = 0; e < E2; ++e) buf[2 * H - 1 - (lane * E2 + e)] = vi[e];  // descending after the strata
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] = buf[lane * E + e];
      wave_bitonic_merge<E>(v);
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] = buf[lane * E + e];
      wave_bitonic_sort<E>(v);
    }
    } else {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = buf[lane * E + e];
    wave_bitonic_sort<E>(v);
    }
    float* zr = a.z + r * S;
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (lane * E + e < S) zr[lane * E + e] = v[e];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");  // buf is rewritten by the next ray
  }
}

#ifndef LNR_GALLOP_JS
#define LNR_GALLOP_JS 0
#endif
#ifndef LNR_GALLOP_JT
#define LNR_GALLOP_JT 1
#endif
#ifndef LNR_GALLOP_CDF
#define LNR_GALLOP_CDF 0
#endif
#ifndef LNR_SAMPLER_MERGE_FILL
// the merge places the depths (each one's stratum count from the linspace, corrected by a short walk: no chain
// of searches) and fills the other positions with the strata in order (a mark per position, a wave scan)
#define LNR_SAMPLER_MERGE_FILL 1
#endif
#ifndef LNR_SAMPLER_CDF_LIFT
#define LNR_SAMPLER_CDF_LIFT 1
#endif
#ifndef LNR_SAMPLER_LOOKUP_UNROLL
#define LNR_SAMPLER_LOOKUP_UNROLL 4
#endif
// ---------------------------------------------------------------------------------------------
// OGM sampler, one wave per ray, the importance draws sorted BEFORE the inverse CDF (LONER_SAMPLER_MERGE=2,
// the default from 256 samples): the inverse CDF is non-decreasing in u, so sorting the draws u and mapping
// them in order gives the sorted importance depths, and the draws are uniform on [0, 1), which a counting
// sort handles in a few passes instead of a bitonic network (k_sampler_wave's 2048-sample sort is 88 % of its
// VALU work).  Then:
//  * counting sort of the H draws into 2H buckets (LDS atomics, a wave scan), the few bucket mates put in
//    order by odd-even transposition passes in registers;
//  * the inverse CDF per sorted draw, its searchsorted answer walked on from the previous draw's;
//  * strata and importance depths merged by rank: stratum i goes to i + #{importance depths < it}, depth j
//    to j + #{strata <= it} (positions unique; equal values are interchangeable);
//  * if the strata are not ascending (jitter rounding, checked as k_sampler_wave does) or the mapped depths
//    are not (one rounding at a bin edge can put a depth an ulp above the next bin's first), the same values
//    go through the full bitonic sort instead.
// Either way the output is the sorted multiset of k_sampler_wave's values: bit for bit the same depths
// (test_ogm_sampler_merge_equals_full_sort).  Q = E / 2 >= 2 strata and draws per lane, lane l holding
// positions [l Q, (l + 1) Q); the per-wave LDS slice is k_sampler_wave's.
__device__ __forceinline__ int lower_bound_from(const float* arr, int lo, int n, float x) {  // first j >= lo: arr[j] >= x
  if (lo >= n || !(arr[lo] < x)) return lo;
  int hi = n;
  ++lo;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (arr[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int upper_bound_from(const float* arr, int lo, int n, float x) {  // first j >= lo: arr[j] > x
  if (lo >= n || arr[lo] > x) return lo;
  int hi = n;
  ++lo;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (arr[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// The same searches when the answer is known to lie just after lo (the previous, smaller key's answer):
// exponential steps lo + 1, + 2, + 4, ... then a binary search in the last step's interval: about 2 log2 of the
// distance LDS reads instead of log2 (n - lo).  UPPER: first j >= lo with arr[j] > x, else arr[j] >= x.
template <bool UPPER>
__device__ __forceinline__ int gallop_from(const float* arr, int lo, int n, float x) {
  auto after = [&](int j) { return UPPER ? !(arr[j] > x) : (arr[j] < x); };  // the answer lies after j
  if (lo >= n || !after(lo)) return lo;
  int last = lo, hi = n;
  for (int b = 1;; b <<= 1) {
    const int j = lo + b;
    if (j >= n) break;
    if (!after(j)) {
      hi = j;
      break;
    }
    last = j;
  }
  int l2 = last + 1;
  while (l2 < hi) {
    const int mid = (l2 + hi) >> 1;
    if (after(mid)) l2 = mid + 1;
    else hi = mid;
  }
  return l2;
}
// #{j < N : !(arr[j] > x)} for ascending arr (upper_bound over [0, N)) by binary lifting: a fixed number of steps,
// no branch, so several independent searches interleave their LDS reads
template <int N>
__device__ __forceinline__ int upper_count_lift(const float* arr, float x) {
  int cnt = 0;
#pragma unroll
  for (int st = 1 << (31 - __builtin_clz(N)); st >= 1; st >>= 1) {
    const int j = cnt + st;
    if (j <= N && !(arr[j - 1] > x)) cnt = j;
  }
  return cnt;
}
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
}

template <int E>
__global__ void __launch_bounds__(64 * kSamplerWaves) k_sampler_rank(SamplerArgs a) {
  static_assert(E >= 4, "two or more strata per lane");
  if (a.dev_step) a.key = a.dev_step->key;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int Q = E / 2, H = 32 * E, NBK = 2 * H;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int M = H - 2;
  float* base = reinterpret_cast<float*>(smem) + (size_t)wid * (4 * H);
  float* strat = base;                                        // [H] strata
  float* imp = base + H;                                      // [H] bucketed draws, then importance depths
  float* cdf = base + 2 * H;                                  // [H - 1]
  float* bins = cdf + H;                                      // [H - 1]
  uint32_t* cnt = reinterpret_cast<uint32_t*>(base + 2 * H);  // [2H] bucket counters (before the cdf)
  float* out = base + 2 * H;                                  // [2H] merged depths (after the inverse CDF)
  for (int64_t r = (int64_t)blockIdx.x * kSamplerWaves + wid; r < a.n_rays; r += (int64_t)gridDim.x * kSamplerWaves) {
    const float* ry = a.rays + 13 * r;
    const float near = ry[11], far = ry[12];
    const float ox = ry[0], oy = ry[1], oz = ry[2], dx = ry[3], dy = ry[4], dz = ry[5];
    const uint32_t gr = (uint32_t)(a.ray_offset + r);
    LNR_STAMP(t0);
    // 1. the draws' counting sort (first, while no stratum is held in registers): bucket counters, ranks within a
    // bucket, bucket offsets, scatter
#pragma unroll
    for (int e = 0; e < E; e += 4) *reinterpret_cast<uint4*>(&cnt[lane * E + e]) = make_uint4(0u, 0u, 0u, 0u);
    wave_lds_fence();
    auto bucket = [&](float u) {
      const uint32_t k = (uint32_t)(u * (float)NBK);
      return k < (uint32_t)NBK ? k : (uint32_t)NBK - 1u;
    };
    float uq[Q];
    uint32_t rk[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int i = lane * Q + q;
      uq[q] = a.u_pdf ? a.u_pdf[r * H + i] : rand_uniform(a.key, kStreamPdf, gr, (uint32_t)i);
      rk[q] = atomicAdd(&cnt[bucket(uq[q])], 1u);
    }
    wave_lds_fence();
    {  // exclusive scan of the counters, this lane's E of them in two passes of 16-byte reads
      uint32_t run = 0;
#pragma unroll
      for (int e = 0; e < E; e += 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(&cnt[lane * E + e]);
        run += v.x + v.y + v.z + v.w;
      }
      uint32_t ex = wave_incl_scan_u32(run) - run;
#pragma unroll
      for (int e = 0; e < E; e += 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(&cnt[lane * E + e]);
        const uint4 o = make_uint4(ex, ex + v.x, ex + v.x + v.y, ex + v.x + v.y + v.z);
        ex += v.x + v.y + v.z + v.w;
        *reinterpret_cast<uint4*>(&cnt[lane * E + e]) = o;
      }
    }
    wave_lds_fence();
#pragma unroll
    for (int q = 0; q < Q; ++q) imp[cnt[bucket(uq[q])] + rk[q]] = uq[q];
    wave_lds_fence();
    float su[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) su[q] = imp[lane * Q + q];
    // bucket mates into order: odd-even transposition passes until the wave's draws ascend
    while (true) {
      bool asc = true;
#pragma unroll
      for (int q = 0; q + 1 < Q; ++q) asc = asc && !(su[q + 1] < su[q]);
      const float nf = __shfl_down(su[0], 1, 64);
      if (lane < 63) asc = asc && !(nf < su[Q - 1]);
      if (__all(asc)) break;
#pragma unroll
      for (int q = 0; q + 1 < Q; q += 2) {
        const float x = su[q], y = su[q + 1];
        su[q] = fminf(x, y);
        su[q + 1] = fmaxf(x, y);
      }
#pragma unroll
      for (int q = 1; q + 1 < Q; q += 2) {
        const float x = su[q], y = su[q + 1];
        su[q] = fminf(x, y);
        su[q + 1] = fmaxf(x, y);
      }
      const float pl = __shfl_up(su[Q - 1], 1, 64), nx = __shfl_down(su[0], 1, 64);
      if (lane < 63) su[Q - 1] = fminf(su[Q - 1], nx);
      if (lane > 0) su[0] = fmaxf(su[0], pl);
    }
    wave_lds_fence();  // (the counters' reads are done: the strata's probabilities overwrite them)
    LNR_STAMP(t1);
    // 2. strata and occupancy probabilities (k_sampler_wave step 1-2), computed lane-contiguous (stratum
    // 64 q + lane: one gather instruction's lanes read neighbouring strata, mostly the same voxels), then
    // transposed through LDS to this lane's positions [l Q, (l + 1) Q)
    float* pscr = bins;  // [H] the probabilities in stratum order (free until step 3)
#pragma unroll LNR_SAMPLER_LOOKUP_UNROLL
    for (int q = 0; q < Q; ++q) {  // (a few strata's gathers in flight per lane: all Q of them cost E = 32 its occupancy)
      const int i = q * 64 + lane;
      const float tt = linspace01(i, H);
      float z = near * (1.0f - tt) + far * tt;
      if (a.perturb > 0.f) {
        const float tl = linspace01(i > 0 ? i - 1 : 0, H), tu = linspace01(i + 1 < H ? i + 1 : H - 1, H);
        const float zl = near * (1.0f - tl) + far * tl, zu = near * (1.0f - tu) + far * tu;
        const float upper = (i + 1 < H) ? 0.5f * (z + zu) : z;
        const float lower = (i > 0) ? 0.5f * (zl + z) : z;
        const float u = a.u_jitter ? a.u_jitter[r * H + i] : rand_uniform(a.key, kStreamJitter, gr, (uint32_t)i);
        z = lower + (upper - lower) * (a.perturb * u);
      }
      strat[i] = z;
      const float l = occ_grid_sample(a.occ, a.occ_res, ox + dx * z, oy + dy * z, oz + dz * z);
      float p = 1.0f / (1.0f + expf(-l));
      p = 2.0f * (fminf(fmaxf(p, 0.5f), 1.0f) - 0.5f);
      pscr[i] = p;
    }
    wave_lds_fence();
    float zq[Q], pq[Q];
    double wl = 0.0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int i = lane * Q + q;
      zq[q] = strat[i];
      pq[q] = pscr[i];
      if (i >= 1 && i <= M) wl += (double)(pq[q] + 1e-5f);
    }
    bool strat_sorted = true;
#pragma unroll
    for (int q = 0; q + 1 < Q; ++q) strat_sorted = strat_sorted && !(zq[q + 1] < zq[q]);
    {
      const float next_first = __shfl_down(zq[0], 1, 64);
      if (lane < 63) strat_sorted = strat_sorted && !(next_first < zq[Q - 1]);
    }
    wave_lds_fence();
    LNR_STAMP(t2);
    // 3. sample_pdf's cdf and bins (k_sampler_wave step 3)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) wl += __shfl_xor(wl, o, 64);
    const float wtot = (float)wl;
    double loc = 0.0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int i = lane * Q + q;
      if (i >= 1 && i <= M) loc += (double)((pq[q] + 1e-5f) / wtot);
    }
    double inc = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    double run = inc - loc;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int i = lane * Q + q;
      if (i >= 1 && i <= M) {
        run += (double)((pq[q] + 1e-5f) / wtot);
        cdf[i] = (float)run;
      }
    }
    if (lane == 0) cdf[0] = 0.f;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int i = lane * Q + q;
      if (i < H - 1) bins[i] = 0.5f * (zq[q] + strat[i + 1]);
    }
    wave_lds_fence();
    LNR_STAMP(t3);
    // 4. inverse CDF of the sorted draws (searchsorted(cdf, u, right=True) over [0, H - 1])
    float fq[Q];
    int lo = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const float u = su[q];
      // the previous draw's answer, or the first cdf entry above u after it (the answer capped at H - 1)
      // (LNR_SAMPLER_CDF_LIFT: each draw's search from scratch, fixed steps, so the Q searches overlap; else
      // walked on from the previous draw's answer)
      lo = LNR_SAMPLER_CDF_LIFT ? upper_count_lift<H - 1>(cdf, u)
           : LNR_GALLOP_CDF     ? gallop_from<true>(cdf, lo, H - 1, u)
                                : upper_bound_from(cdf, lo, H - 1, u);
      const int below = lo - 1 > 0 ? lo - 1 : 0;
      const int above = lo < M ? lo : M;
      const float c0 = cdf[below], c1 = cdf[above];
      const float b0 = bins[below], b1 = bins[above];
      float denom = c1 - c0;
      if (denom < 1e-5f) denom = 1.0f;
      fq[q] = b0 + (u - c0) / denom * (b1 - b0);
    }
    bool f_asc = true;
#pragma unroll
    for (int q = 0; q + 1 < Q; ++q) f_asc = f_asc && !(fq[q + 1] < fq[q]);
    {
      const float nf = __shfl_down(fq[0], 1, 64);
      if (lane < 63) f_asc = f_asc && !(nf < fq[Q - 1]);
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) imp[lane * Q + q] = fq[q];
    wave_lds_fence();
    float* zr = a.z + r * (int64_t)(2 * H);
    LNR_STAMP(t4);
    if (LNR_SAMPLER_MERGE_FILL && __all(strat_sorted && f_asc)) {
      // 5. merge into out, then coalesced stores (out overlays the cdf and bins, whose reads ended before the
      // fence above).  Depth j goes to j + #{strata <= it}: the strata are the linspace's jittered within their
      // bins, so the count is the linspace position's, up to the stratum of the bin holding the depth (a walk
      // of a step or two over the sorted strata makes it exact).  Stratum i goes to the i-th position no depth
      // took (= i + #{depths < it}: the same merge, ties included): positions are marked in a bit per
      // position (imp's words: the depths are in registers now), and a lane's E positions take their strata
      // after a wave scan of the marks' counts.
      uint32_t* mk = reinterpret_cast<uint32_t*>(imp);
      constexpr int NW = 2 * H / 32;
      for (int w = lane; w < NW; w += 64) mk[w] = 0u;
      const float span = far - near;
      const float per = span > 0.f ? (float)(H - 1) / span : 0.f;
      wave_lds_fence();
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const float f = fq[q];
        int e;
        if (span > 0.f) {  // (wave-uniform: one ray per wave)
          e = (int)fminf(fmaxf((f - near) * per + 1.0f, 0.0f), (float)H);
          while (e > 0 && strat[e - 1] > f) --e;
          while (e < H && !(strat[e] > f)) ++e;
        } else {  // no linspace estimate (far <= near): the same count by binary lifting, not a walk of up to H steps
          e = upper_count_lift<H>(strat, f);
        }
        const int pos = lane * Q + q + e;
        out[pos] = f;
        atomicOr(&mk[pos >> 5], 1u << (pos & 31));
      }
      wave_lds_fence();
      const uint32_t bits = (mk[(lane * E) >> 5] >> ((lane * E) & 31)) & (E >= 32 ? 0xFFFFFFFFu : ((1u << E) - 1u));
      const uint32_t nd = (uint32_t)__popc(bits);
      int k = lane * E - (int)(wave_incl_scan_u32(nd) - nd);  // the stratum of this lane's first free position
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (!((bits >> e) & 1u)) {
          out[lane * E + e] = strat[k];
          ++k;
        }
      }
      wave_lds_fence();
#pragma unroll
      for (int e = 0; e < E; ++e) zr[e * 64 + lane] = out[e * 64 + lane];
    } else if (__all(strat_sorted && f_asc)) {
      // 5. merge by rank into out, then coalesced stores
      // (out overlays the cdf and bins, whose reads ended before the fence above)
      int js = 0, jt = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        js = (q == 0 || !LNR_GALLOP_JS) ? lower_bound_from(imp, js, H, zq[q]) : gallop_from<false>(imp, js, H, zq[q]);
        out[lane * Q + q + js] = zq[q];
        jt = (q == 0 || !LNR_GALLOP_JT) ? upper_bound_from(strat, jt, H, fq[q]) : gallop_from<true>(strat, jt, H, fq[q]);
        out[lane * Q + q + jt] = fq[q];
      }
      wave_lds_fence();
#pragma unroll
      for (int e = 0; e < E; ++e) zr[e * 64 + lane] = out[e * 64 + lane];
    } else {
      // the full bitonic sort of the same values (strata in strat, depths in imp: one contiguous buffer)
      float v[E];
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] = base[lane * E + e];
      wave_bitonic_sort<E>(v);
#pragma unroll
      for (int e = 0; e < E; ++e) zr[lane * E + e] = v[e];
    }
    wave_lds_fence();  // this wave's slice is rewritten by its next ray
    LNR_STAMP(t5);
    LNR_PHASE(0, t1, t0);
    LNR_PHASE(1, t2, t1);
    LNR_PHASE(2, t3, t2);
    LNR_PHASE(3, t4, t3);
    LNR_PHASE(4, t5, t4);
  }
}

static size_t sampler_wave_smem(int E, int H) { return (size_t)kSamplerWaves * (64 * E + 2 * H) * 4; }

static size_t sampler_smem(int H, int P2) { return ((size_t)3 * H + P2 + 2) * 4 + (SNT / 64 + 2) * 8 + 16; }

}  // namespace lnr

using namespace lnr;

LNR_PHASE_EXPORT(sampler)

extern "C" uint32_t lnr_step_key(uint32_t seed, uint32_t step) { return mix32(mix32(seed) ^ step); }

extern "C" int lnr_sample_ogm(const float* rays, int64_t n_rays, int32_t n_samples, const float* occ, int32_t occ_res,
                              float perturb, const float* u_jitter, const float* u_pdf, uint32_t key, int64_t ray_offset,
                              float* z, const lnr_step_scalars* dev_step, void* stream) {
  LNR_REQUIRE(n_rays >= 0, "lnr_sample_ogm: n_rays < 0");
  LNR_REQUIRE(n_samples >= 8 && n_samples % 2 == 0 && n_samples <= 4096,
              "lnr_sample_ogm: n_samples=%d must be even in [8,4096]", n_samples);
  LNR_REQUIRE(occ_res >= 1, "lnr_sample_ogm: occ_res=%d", occ_res);
  if (n_rays == 0) return LNR_OK;
  LNR_REQUIRE(rays && occ && z, "lnr_sample_ogm: null pointer");
  SamplerArgs a{};
  a.rays = rays; a.n_rays = n_rays; a.S = n_samples; a.H = n_samples / 2; a.occ = occ; a.occ_res = occ_res;
  a.perturb = perturb; a.u_jitter = u_jitter; a.u_pdf = u_pdf; a.key = key; a.ray_offset = ray_offset; a.z = z;
  a.dev_step = dev_step;
  int p2 = 1;
  while (p2 < n_samples) p2 <<= 1;
  a.P2 = p2;
  LNR_REQUIRE(a.H <= 8 * SNT, "lnr_sample_ogm: too many samples");
  if (a.H % 64 == 0 && p2 >= 128 && p2 <= 2048) {  // one wave per ray
    const int E = p2 / 64;
    const int mode = sampler_merge();
    const bool merge = mode != 0;
    const int64_t nbw = (n_rays + kSamplerWaves - 1) / kSamplerWaves;
    const dim3 g((unsigned)(nbw < 8192 ? nbw : 8192)), b(64 * kSamplerWaves);
    const size_t sm = sampler_wave_smem(E, a.H);
    if (mode == 2 && E >= 4 && 2 * a.H == 64 * E && n_rays >= sampler_rank_min_rays()) {
      switch (E) {
        case 4: hipLaunchKernelGGL(k_sampler_rank<4>, g, b, sm, as_stream(stream), a); break;
        case 8: hipLaunchKernelGGL(k_sampler_rank<8>, g, b, sm, as_stream(stream), a); break;
        case 16: hipLaunchKernelGGL(k_sampler_rank<16>, g, b, sm, as_stream(stream), a); break;
        default: hipLaunchKernelGGL(k_sampler_rank<32>, g, b, sm, as_stream(stream), a); break;
      }
      LNR_RETURN_LAUNCH("lnr_sample_ogm");
    }
    switch (E) {
      case 2: hipLaunchKernelGGL((merge ? k_sampler_wave<2, true> : k_sampler_wave<2, false>), g, b, sm, as_stream(stream), a); break;
      case 4: hipLaunchKernelGGL((merge ? k_sampler_wave<4, true> : k_sampler_wave<4, false>), g, b, sm, as_stream(stream), a); break;
      case 8: hipLaunchKernelGGL((merge ? k_sampler_wave<8, true> : k_sampler_wave<8, false>), g, b, sm, as_stream(stream), a); break;
      case 16: hipLaunchKernelGGL((merge ? k_sampler_wave<16, true> : k_sampler_wave<16, false>), g, b, sm, as_stream(stream), a); break;
      default: hipLaunchKernelGGL((merge ? k_sampler_wave<32, true> : k_sampler_wave<32, false>), g, b, sm, as_stream(stream), a); break;
    }
    LNR_RETURN_LAUNCH("lnr_sample_ogm");
  }
  const int nb = (int)(n_rays < 4096 ? n_rays : 4096);
  hipLaunchKernelGGL(k_sampler<true>, dim3(nb), dim3(SNT), sampler_smem(a.H, p2), as_stream(stream), a);
  LNR_RETURN_LAUNCH("lnr_sample_ogm");
}

extern "C" int lnr_sample_uniform(const float* rays, int64_t n_rays, int32_t n_samples, float perturb,
                                  const float* u_jitter, uint32_t key, int64_t ray_offset, float* z,
                                  const lnr_step_scalars* dev_step, void* stream) {
  LNR_REQUIRE(n_rays >= 0, "lnr_sample_uniform: n_rays < 0");
  LNR_REQUIRE(n_samples >= 2 && n_samples <= 2048, "lnr_sample_uniform: n_samples=%d not in [2,2048]", n_samples);
  if (n_rays == 0) return LNR_OK;
  LNR_REQUIRE(rays && z, "lnr_sample_uniform: null pointer");
  SamplerArgs a{};
  a.rays = rays; a.n_rays = n_rays; a.S = n_samples; a.H = n_samples; a.perturb = perturb; a.u_jitter = u_jitter;
  a.key = key; a.ray_offset = ray_offset; a.z = z; a.P2 = 0; a.dev_step = dev_step;
  const int nb = (int)(n_rays < 4096 ? n_rays : 4096);
  hipLaunchKernelGGL(k_sampler<false>, dim3(nb), dim3(SNT), sampler_smem(a.H, 0), as_stream(stream), a);
  LNR_RETURN_LAUNCH("lnr_sample_uniform");
}
