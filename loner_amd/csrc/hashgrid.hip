// Multi-resolution hash-grid encoding (tiny-cuda-nn v1.7 HashGrid semantics) for gfx950: forward.
//
// Replaces tcnn's kernel_grid behind tcnn.NetworkWithInputEncoding (src/models/nerf_tcnn.py:35-38,
// 68, 71) and tcnn.Encoding (:40, 64).  The backward lives in hashgrid_bwd.hip.
//
// Launch shape: grid (ceil(N / kSB), n_levels / G) of kSB-thread workgroups (kSB = 512 samples, one
// histogram row each), each taking G levels y, y + L/G, y + 2 L/G, ... (G = 2 from 512 rows, 4 from
// 2048, see enc_levels_per_group; the live-masked eval launch: G = 1, kSB / 2 threads of two samples).  The
// level group is the slow grid dimension, so the dispatcher walks group by group and the live gather
// footprint is one group's table slices (<= 4 MB fp16, about an XCD's L2) instead of the whole
// 14.8 MB table; and every group mixes coherent levels (position decoding, run detection: VALU) with
// fine ones (hashed gathers: the texture addresser), so the two bottlenecks overlap.
// Output layout is level-major half2 (enc[l * stride + n]) so every store is a coalesced 4 B/lane.
// In training mode the forward also emits the backward's per-block record histogram (same
// corners), which removes a full corner-recompute pass from the backward.
#include "hashgrid.hpp"

namespace lnr {

// The encoding is written once, as whole lines, and read by the field kernels after this launch: a
// nontemporal store keeps it out of the way of the table slices in L2 (step -0.01 ms at C2; plain stores
// re-measured in round 5 within the noise)
__device__ __forceinline__ void store_enc(uint32_t* p, uint32_t v) { __builtin_nontemporal_store(v, p); }

// The 8 corners of a fine (hashed, power-of-two) level: the x-pairs e, e ^ d of the four y/z edges.
// What bounds this gather is the texture addresser: TA busy 0.78 of the launch at C2 with the level-grouped
// encode (profiles/r04_l2req_C2.txt; 0.85 before the grouping, profiles/r03_l2req_C2.txt), about 40 TA cycles
// per wave-wide gather of scattered entries.  Reading an
// x-pair through one 16-B load of its aligned quad (3/4 of the pairs; tried) cut the vector-L1 line
// accesses from 426 M to 288 M per launch but left TA busy where it was (0.743 against 0.720 ms);
// 8-B pair loads ran 0.86 ms.  Plain dword gathers (here, or lane-paired below).
__device__ __forceinline__ void fine_gather(const uint32_t* __restrict__ tl, const FineCell& c, uint32_t (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = tl[c.e[j]];
    v[2 * j + 1] = tl[c.e[j] ^ c.d];
  }
}

// The same 8 corners with lanes paired (2m, 2m + 1): in one instruction both lanes of a pair read
// the two x-corners of one sample's edge (the even lane corner e, the odd lane e ^ d), so the pair
// shares a cache line (94 % of the x-pairs do) and a wave-wide gather touches 32 lines instead of 64.
// Slot 0 of each edge serves the even lane's sample, slot 1 the odd lane's; one DPP swap per edge
// hands each lane the corner its partner read for it.  C2 encode 0.721 -> 0.691 ms: the texture
// addresser does not charge purely by lines.  Every lane of the wave must take
// part (the swaps): the loads, not the lanes, are predicated on ``use``, and a dead lane still gathers
// for a live partner, which is why the live-masked eval launch keeps fine_gather.  Same entries in the
// same corner order: the encoding is bit-identical to fine_gather's.
#ifndef LNR_ENC_PAIRED
#define LNR_ENC_PAIRED true  // the training / plain eval encode's fine gathers lane-paired (C2: 0.721 -> 0.691 ms)
#endif
__device__ __forceinline__ uint32_t dpp_pair_swap(uint32_t v) {  // quad_perm [1, 0, 3, 2]
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ void fine_gather_paired(const uint32_t* __restrict__ tl, const FineCell& c, bool use,
                                                   uint32_t (&v)[8]) {
  const bool odd = (threadIdx.x & 1) != 0;
  const uint32_t pd = dpp_pair_swap(c.d);
  const bool puse = dpp_pair_swap(use ? 1u : 0u) != 0u;
  const uint32_t d_even = odd ? pd : c.d, d_odd = odd ? c.d : pd;
  const bool use_even = odd ? puse : use, use_odd = odd ? use : puse;
  uint32_t s0[4], s1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t pe = dpp_pair_swap(c.e[j]);
    const uint32_t e_even = odd ? pe : c.e[j], e_odd = odd ? c.e[j] : pe;
    const uint32_t a0 = odd ? (e_even ^ d_even) : e_even;  // slot 0: the even lane's sample
    const uint32_t a1 = odd ? (e_odd ^ d_odd) : e_odd;     // slot 1: the odd lane's sample
    s0[j] = use_even ? tl[a0] : 0u;
    s1[j] = use_odd ? tl[a1] : 0u;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t r = dpp_pair_swap(odd ? s0[j] : s1[j]);  // what the partner read for this lane
    v[2 * j] = odd ? r : s0[j];
    v[2 * j + 1] = odd ? s1[j] : r;
  }
}

#ifndef LNR_ENC_SPT2_MIN_N
#define LNR_ENC_SPT2_MIN_N (1 << 18)  // the live-masked eval encode: two samples per thread from this many
                                      // samples (C3 colour encode 0.48 -> 0.43 ms); below it one
#endif

// One kernel for the training encode (ws.hist set: also the backward's record histogram) and the
// eval encode (ws.hist null; ``live`` optional).  The flag is a runtime, block-uniform one on
// purpose: a separate no-count instantiation compiles to a shape whose fine and dense gathers share
// one load block, and that runs 14 % slower (C2: 838 against 722 us; tools/exp_overlap.py).
// One workgroup per histogram row (kSB samples) and level, kEncSpt samples per thread: thread t
// takes samples t and t + kSB / 2 of the row, so each wave still covers 64-sample groups (the
// coherent levels' run merging sees the lanes the scatter sees), and a fine level's gathers of both
// samples are in flight together.
#ifndef LNR_ENC_LPB
#define LNR_ENC_LPB 4  // most levels per workgroup of the training / plain eval encode (1, 2 or 4)
#endif
#ifndef LNR_ENC_GROUP_MIN_ROWS
#define LNR_ENC_GROUP_MIN_ROWS 512  // fewer rows: one level per workgroup (C1's 64 rows need the workgroups)
#endif
// Levels per workgroup for n levels and n_sb rows: G levels y, y + n/G, ... share a workgroup.
// Measured at C2 (encode ms, tools/gpu_ab_libs.sh): one level 0.677; two consecutive levels 0.662;
// two levels y, y + 8 0.618; four consecutive 0.720 (a 4 MB working set of fine levels); four levels
// y, y + 4, y + 8, y + 12 0.605-0.612; eight 0.767, sixteen 0.890.  C3's sigma encode 1.188 / 1.135 /
// 0.965 / 0.960 for one / two consecutive / two strided / four strided.
// A group's fine levels must fit an XCD's 4 MB L2 together: four 1 MB levels of the sigma grid (2^18
// entries), two 2 MB levels of the colour grid (2^19: CAM's colour encode 0.33 ms at one level per
// workgroup, 0.37 at four).
#ifndef LNR_ENC_GROUP4_MIN_ROWS
// Groups of four from 2048 rows: at 1152 (C4, one rank of eight) pairs encode 0.0975 ms against 0.0993
// with fours, bitwise the same (tools/gpu_ab_libs.sh, three interleaved runs each).
#define LNR_ENC_GROUP4_MIN_ROWS 2048  // rows from which groups of four are allowed (fewer: at most two)
#endif
inline int enc_levels_per_group(const lnr_grid_desc* d, int64_t n_sb) {
  if (n_sb < LNR_ENC_GROUP_MIN_ROWS) return 1;
  const int64_t level_bytes = (int64_t)4 << d->log2_hashmap_size;
  for (int g = LNR_ENC_LPB; g > 1; g /= 2)
    if (d->n_levels % g == 0 && g * level_bytes <= ((int64_t)4 << 20) && (g < 4 || n_sb >= LNR_ENC_GROUP4_MIN_ROWS))
      return g;
  return 1;
}
// Early ray termination (lnr_hashgrid_fwd_rays_phase): the encode of samples [lo, hi) of the listed rays (the
// rays still alive, ascending; every ray in the first phase).  With the record histogram (the first phase, for a
// full backward, which places every sample's records) the grid is the plain one, every sample's records are
// counted and only the phase's samples gather; without it (the live backward counts its own) the grid covers the
// phase's samples of the listed rays (``compact``: workgroup sample g -> ray list[g / (hi - lo)], ray sample
// lo + g % (hi - lo); a wave stays within one ray, as lo and hi are multiples of 64), sized for every ray, and its
// samples past the list's end (count x width) leave at once.
struct EncPhase {
  const uint32_t* list;   // the rays of the phase (compact only); null: every ray
  const uint32_t* count;  // DEVICE: how many
  int32_t lo, hi;         // ray-local sample range; hi == 0: no phase (every sample)
  int32_t S;              // samples per ray
  bool compact;
  __device__ __forceinline__ bool on() const { return hi > 0; }
  template <bool LISTED>
  __device__ __forceinline__ int64_t sample(int64_t g) const {
    if (!compact) return g;
    if constexpr (LISTED) {
      const uint32_t w = (uint32_t)(hi - lo), e = (uint32_t)g / w;
      return (int64_t)list[e] * S + lo + ((uint32_t)g - e * w);
    } else {
      const int32_t w = hi - lo;
      return (g / w) * S + lo + g % w;
    }
  }
};

// Early ray termination's sparse phases: fewer expected rows than this take the one-level row-walking grid
#ifndef LNR_ENC_SPARSE_ROWS
#define LNR_ENC_SPARSE_ROWS 512
#endif
constexpr int64_t kEncSparseRows = LNR_ENC_SPARSE_ROWS;
#ifndef LNR_ENC_SPARSE_LPB
#define LNR_ENC_SPARSE_LPB 2  // levels per workgroup of a sparse phase's row-walking grid (C2: 4 and 1 within
                              // the noise, 4 spills two VGPRs in the loop; tools/gpu_ab_libs.sh, three rounds)
#endif
#ifndef LNR_ENC_WAVES
#define LNR_ENC_WAVES 8  // waves per SIMD asked of the encode (68 registers would allow 7)
#endif
// One row (kSB samples) of the encode at the workgroup's levels (the body of k_hashgrid_fwd); false: this thread's
// samples lie past the end (it has nothing more to do).
template <class PosFn, int kEncSpt, bool PAIRED, int LPB, bool LISTED>
__device__ __forceinline__ bool enc_row(const GridArgs& a, PosFn pos, int64_t n, const uint32_t* __restrict__ table,
                                        uint32_t* __restrict__ enc, int64_t stride, const BwdWorkspace& ws,
                                        const float* __restrict__ live, const EncPhase& ph, int64_t row) {
  constexpr int H = kSB / kEncSpt;
  const int64_t g0 = row * kSB + threadIdx.x;  // (the compact phase grid: g0 < n counts its samples)
  const bool count = ws.hist != nullptr;
  const int64_t n_in = ph.compact ? (int64_t)(n / (ph.hi - ph.lo)) * ph.S : n;  // pos.wave's bound (every ray)
  if constexpr (LISTED) n = (int64_t)ph.count[0] * (ph.hi - ph.lo);  // the listed rays' samples
  if (!count && (g0 & ~(int64_t)1) >= n) return false;  // (lane pairs leave together: fine_gather_paired)
  __shared__ uint32_t hist[kMaxChunksPerLevel];
  bool in[kEncSpt], use[kEncSpt], cnt[kEncSpt];
  float x[kEncSpt], y[kEncSpt], z[kEncSpt];
#pragma unroll
  for (int h = 0; h < kEncSpt; ++h) {
    const int64_t i = ph.template sample<LISTED>(g0 + h * H);
    in[h] = (g0 + h * H) < n;
    // live: samples whose weight is exactly 0 get a zero encoding and issue no gathers; when counting
    // too, they emit no records at the fine levels (the scatter skips them by the same mask)
    use[h] = in[h] && (live == nullptr || live[i] != 0.f);
    cnt[h] = use[h];
    if (ph.on()) {  // early ray termination: the phase's samples of the listed rays gather, every sample counts
      const int32_t j = (int32_t)(i % ph.S);
      use[h] = in[h] && j >= ph.lo && j < ph.hi;
      cnt[h] = in[h];
    }
    x[h] = y[h] = z[h] = 0.f;
    pos.wave(i, n_in, in[h], x[h], y[h], z[h]);
  }
  if (ph.on() && !count) {
    bool any = false;
#pragma unroll
    for (int h = 0; h < kEncSpt; ++h) any |= use[h];
    if (!__any(any)) return true;  // a terminated ray's wave (no histogram: no barriers to keep)
  }
  // dead samples (live, use = false) get a zero encoding only where their aligned 16-sample tile holds a live
  // sample: the colour kernels skip a tile whose weights are all 0 and read every encoding of the others
  // (lnr_hashgrid_fwd_rays_live's contract, include/loner_amd.h)
  bool zero[kEncSpt];
#pragma unroll
  for (int h = 0; h < kEncSpt; ++h) {
    const unsigned long long lv = __ballot(use[h]);
    zero[h] = in[h] && ((lv >> (threadIdx.x & 48)) & 0xFFFFull) != 0ull;
  }
  // LPB levels per workgroup, y, y + L/LPB, y + 2 L/LPB, ... (grid.y = L / LPB), in level order: the
  // sample's position is decoded and its depth loaded once for them, and a coherent level's VALU-heavy
  // work runs beside a fine level's gathers (head comment)
  for (int li = 0; li < LPB; ++li) {
  const uint32_t l = blockIdx.y + li * gridDim.y;
  if (count) {
    if (li > 0) lds_barrier();  // the previous level's histogram is published
    for (int b = threadIdx.x; b < kMaxChunksPerLevel; b += blockDim.x) hist[b] = 0;
  }
  const LevelParams& lv = a.lv[l];
  if (lv.fine) {  // block-uniform
    FineCell c[kEncSpt];
    uint32_t v[kEncSpt][8];
    const uint32_t* tl = table + lv.offset;
#pragma unroll
    for (int h = 0; h < kEncSpt; ++h) fine_cell(lv, x[h], y[h], z[h], c[h]);
    if constexpr (PAIRED) {
#pragma unroll
      for (int h = 0; h < kEncSpt; ++h) fine_gather_paired(tl, c[h], use[h], v[h]);
    } else {
#pragma unroll
      for (int h = 0; h < kEncSpt; ++h)
        if (use[h]) fine_gather(tl, c[h], v[h]);
    }
#pragma unroll
    for (int h = 0; h < kEncSpt; ++h) {
      uint32_t* dst = enc + (int64_t)l * stride + ph.template sample<LISTED>(g0 + h * H);
      if (use[h]) {
        float f0 = 0.f, f1 = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float w = fine_weight(c[h], k >> 1, k & 1);
          const float2 t = half2_to_float2(v[h][k]);
          f0 = fmaf(w, t.x, f0);
          f1 = fmaf(w, t.y, f1);
        }
        store_enc(dst, (uint32_t)f2h(f0) | ((uint32_t)f2h(f1) << 16));
      } else if (zero[h]) {
        *dst = 0u;
      }
    }
    if (count) {
      lds_barrier();
#pragma unroll
      for (int h = 0; h < kEncSpt; ++h) count_fine_add(c[h], cnt[h], hist);
      lds_barrier();
      publish_block_counts(a, l, hist, ws);
    }
    continue;
  }
  // (the coherent levels' gathers once per run of lanes in one cell, handed to the run's lanes by ds_bpermute,
  // measured no faster: the texture addresser charges the lanes' shared lines once either way; removed in round
  // 6, history before commit e32a0b7)
#pragma unroll
  for (int h = 0; h < kEncSpt; ++h) {
    Corners c;
    level_corners(lv, x[h], y[h], z[h], c);
    uint32_t* dst = enc + (int64_t)l * stride + ph.template sample<LISTED>(g0 + h * H);
    if (use[h]) {
      uint32_t v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = table[c.idx[k]];
      float f0 = 0.f, f1 = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float2 t = half2_to_float2(v[k]);
        f0 = fmaf(c.w[k], t.x, f0);
        f1 = fmaf(c.w[k], t.y, f1);
      }
      store_enc(dst, (uint32_t)f2h(f0) | ((uint32_t)f2h(f1) << 16));
    } else if (zero[h]) {
      *dst = 0u;
    }
    if (count) {
      if (h == 0) lds_barrier();  // the zeroed histogram
      count_add(a, l, c, in[h], cnt[h], hist);
    }
  }
  if (count) {
    lds_barrier();
    publish_block_counts(a, l, hist, ws);
  }
  }
  return true;
}

// The training / eval encode (see above); LOOP (early ray termination's later phases over a list of rays): a grid
// smaller than the rows walks them, a workgroup taking rows blockIdx.x, + gridDim.x, ... until past the list's end.
template <class PosFn, int kEncSpt, bool PAIRED, int LPB = 1, bool LISTED = false, bool LOOP = false>
__global__ void __launch_bounds__(kSB / kEncSpt) __attribute__((amdgpu_waves_per_eu(LNR_ENC_WAVES, LNR_ENC_WAVES))) k_hashgrid_fwd(GridArgs a, PosFn pos, int64_t n,
                                                               const uint32_t* __restrict__ table,
                                                               uint32_t* __restrict__ enc, int64_t stride,
                                                               BwdWorkspace ws, const float* __restrict__ live,
                                                               EncPhase ph) {
  if constexpr (!LOOP) {
    enc_row<PosFn, kEncSpt, PAIRED, LPB, LISTED>(a, pos, n, table, enc, stride, ws, live, ph, blockIdx.x);
  } else {
    for (int64_t row = blockIdx.x;
         enc_row<PosFn, kEncSpt, PAIRED, LPB, LISTED>(a, pos, n, table, enc, stride, ws, live, ph, row);
         row += gridDim.x) {
    }
  }
}

// Backward with fp32 atomics.  Levels whose cells span several consecutive samples merge equal
// corner indices across neighbouring lanes first (segmented wave reduction), so only run heads
// issue atomics; fine hashed levels issue one atomic pair per corner.
template <class PosFn>
__global__ void __launch_bounds__(256) k_hashgrid_bwd(GridArgs a, PosFn pos, int64_t n, const float2* __restrict__ d_enc,
                                                      int64_t stride, float* __restrict__ d_table) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t l = blockIdx.y;
  const bool valid = i < n;
  float x = 0.f, y = 0.f, z = 0.f;
  float2 g = make_float2(0.f, 0.f);
  if (valid) {
    pos(i, x, y, z);
    g = d_enc[(int64_t)l * stride + i];
  }
  Corners c;
  level_corners(a.lv[l], x, y, z, c);
  if (l < a.merge_levels) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t idx = valid ? c.idx[k] : 0xFFFFFFFFu;
      float p0 = c.w[k] * g.x, p1 = c.w[k] * g.y;
      // runs of equal idx are contiguous in lane order (samples sorted along the ray)
      const RunInfo ri = lane_runs(idx);
      run_sum(ri, p0, p1);
      if (ri.tail && idx != 0xFFFFFFFFu) {
        atomicAdd(&d_table[2 * (int64_t)idx + 0], p0);
        atomicAdd(&d_table[2 * (int64_t)idx + 1], p1);
      }
    }
  } else if (valid) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      atomicAdd(&d_table[2 * (int64_t)c.idx[k] + 0], c.w[k] * g.x);
      atomicAdd(&d_table[2 * (int64_t)c.idx[k] + 1], c.w[k] * g.y);
    }
  }
}

__global__ void k_enc_to_aos(const uint32_t* __restrict__ enc, int64_t stride, int64_t n, uint32_t L,
                             uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * L) return;
  const int64_t s = i / L;
  const uint32_t l = (uint32_t)(i % L);
  out[i] = enc[(int64_t)l * stride + s];
}

__global__ void k_aos_grad_to_enc(const uint16_t* __restrict__ g16, const float* __restrict__ g32, int64_t n, uint32_t L,
                                  float2* __restrict__ d_enc, int64_t stride) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * L) return;
  const int64_t s = i / L;
  const uint32_t l = (uint32_t)(i % L);
  float2 v;
  if (g16) {
    v = make_float2(h2f(g16[2 * i]), h2f(g16[2 * i + 1]));
  } else {
    v = make_float2(g32[2 * i], g32[2 * i + 1]);
  }
  d_enc[(int64_t)l * stride + s] = v;
}


}  // namespace lnr

using namespace lnr;

extern "C" int lnr_grid_desc_init(lnr_grid_desc* d, uint32_t n_levels, uint32_t n_features, uint32_t log2_hashmap_size,
                                  uint32_t base_resolution, float per_level_scale) {
  LNR_REQUIRE(d != nullptr, "lnr_grid_desc_init: null descriptor");
  LNR_REQUIRE(n_levels >= 1 && n_levels <= LNR_MAX_LEVELS, "lnr_grid_desc_init: n_levels=%u out of [1,%d]", n_levels,
              LNR_MAX_LEVELS);
  LNR_REQUIRE(n_features == 2, "lnr_grid_desc_init: only n_features_per_level=2 is supported (got %u)", n_features);
  LNR_REQUIRE(log2_hashmap_size >= 4 && log2_hashmap_size <= 28, "lnr_grid_desc_init: log2_hashmap_size=%u",
              log2_hashmap_size);
  LNR_REQUIRE(base_resolution >= 1, "lnr_grid_desc_init: base_resolution=%u", base_resolution);
  d->n_levels = n_levels;
  d->n_features = n_features;
  d->log2_hashmap_size = log2_hashmap_size;
  d->base_resolution = base_resolution;
  d->per_level_scale = per_level_scale;
  const float l2s = std::log2(per_level_scale);
  uint32_t offset = 0;
  const uint32_t max_params = 0xFFFFFFFFu / 2;
  for (uint32_t l = 0; l < n_levels; ++l) {
    const float scale = std::exp2((float)l * l2s) * (float)base_resolution - 1.0f;
    const uint32_t res = (uint32_t)std::ceil(scale) + 1;
    uint32_t dense;
    if (std::pow((float)res, 3.0f) > (float)max_params)
      dense = max_params;
    else
      dense = res * res * res;
    uint32_t size = ((dense + 7u) / 8u) * 8u;
    const uint32_t cap = 1u << log2_hashmap_size;
    if (size > cap) size = cap;
    d->scale[l] = scale;
    d->resolution[l] = res;
    d->size[l] = size;
    d->offset[l] = offset;
    offset += size;
  }
  d->offset[n_levels] = offset;
  d->n_entries = offset;
  return LNR_OK;
}

static int check_desc(const lnr_grid_desc* d, const char* who) {
  LNR_REQUIRE(d != nullptr && d->n_levels >= 1 && d->n_levels <= LNR_MAX_LEVELS && d->n_features == 2,
              "%s: invalid grid descriptor", who);
  return LNR_OK;
}

// Levels per workgroup of the live-masked eval encode (C3's colour encode): LONER_ENC_LIVE_LPB 2 (default:
// strided pairs, the colour grid's two 2 MB levels per group, one sample per thread) or 1 (one level, two
// samples per thread), read at every launch.  C3 colour encode 0.435 -> 0.408 ms, bitwise the same
// (test_hashgrid_fwd_live_mask_matches_full_encode).
static int live_lpb() {
  const char* e = getenv("LONER_ENC_LIVE_LPB");
  return e ? atoi(e) : 2;
}

template <class PosFn>
static int launch_fwd(const lnr_grid_desc* d, PosFn pos, int64_t n, const uint16_t* table, uint32_t* enc,
                      int64_t enc_stride, void* bwd_ws, int64_t bwd_ws_bytes, hipStream_t st, const char* who,
                      const float* live = nullptr, EncPhase ph = EncPhase{nullptr, nullptr, 0, 0, 1, false},
                      int64_t expect_rays = 0) {
  GridArgs a = make_args(d, pos.samples_per_ray());
  LNR_REQUIRE(n < (int64_t(1) << 31), "%s: n=%lld samples exceeds 2^31", who, (long long)n);
  // training and plain eval launches: one sample per thread, lane-paired fine gathers; the eval launch
  // with a ``live`` mask (C3's colour encode, most samples dead): plain gathers, so dead lanes issue
  // none, two samples per thread from LNR_ENC_SPT2_MIN_N samples
  const bool spt2 = n >= (int64_t)LNR_ENC_SPT2_MIN_N;
  const int lpb = enc_levels_per_group(d, (n + kSB - 1) / kSB);
  auto enc_kernel = [&]() {
    return lpb == 4 ? k_hashgrid_fwd<PosFn, 1, LNR_ENC_PAIRED, 4>
         : lpb == 2 ? k_hashgrid_fwd<PosFn, 1, LNR_ENC_PAIRED, 2>
                    : k_hashgrid_fwd<PosFn, 1, LNR_ENC_PAIRED, 1>;
  };
  BwdWorkspace w{};
  if (bwd_ws) {
    LNR_REQUIRE(bwd_ws_bytes >= bwd_workspace_bytes(d, n), "%s: backward workspace too small", who);
    LNR_REQUIRE(a.n_buckets <= (uint32_t)kMaxBuckets, "%s: too many table chunks (%u)", who, a.n_buckets);
    for (uint32_t l = 0; l < d->n_levels; ++l)
      LNR_REQUIRE(a.bucket_base[l + 1] - a.bucket_base[l] <= (uint32_t)kMaxChunksPerLevel,
                  "%s: level %u has more than %d table chunks", who, l, kMaxChunksPerLevel);
    w = carve_workspace(bwd_ws, a, d, n);
  }
  // one workgroup per histogram row (kSB samples), so a counted row is written whole (and kSB-sample
  // workgroups for the plain eval launch too: C2-size eval 1011 us at 256 one-sample threads, 836 at 512)
  const unsigned rows = (unsigned)((n + kSB - 1) / kSB);
  const uint32_t* tb = reinterpret_cast<const uint32_t*>(table);
  const dim3 grid(rows, d->n_levels);
  if (ph.compact) {  // a phase of early ray termination: the grid covers the phase's samples only
    const int64_t ng = (n / ph.S) * (ph.hi - ph.lo);
    const unsigned rows_c = (unsigned)((ng + kSB - 1) / kSB);
    const int lpb_c = enc_levels_per_group(d, rows_c);
    const unsigned groups = d->n_levels / lpb_c;
    const int64_t exp_rows = (expect_rays * (ph.hi - ph.lo) + kSB - 1) / kSB;
    if (ph.list && expect_rays > 0 && exp_rows < kEncSparseRows) {
      // a sparse phase (few rays still alive, by the caller's estimate): latency-bound, its rows fit in one round of
      // resident workgroups, so a grid of about the expected rows (x 1.25) walks the listed rows, LNR_ENC_SPARSE_LPB
      // levels per workgroup (a grid sized for every ray launches workgroups only to leave)
      const unsigned gx = (unsigned)std::min<int64_t>(rows_c, exp_rows + exp_rows / 4 + 8);
      const int lpb_s = d->n_levels % LNR_ENC_SPARSE_LPB == 0 ? LNR_ENC_SPARSE_LPB : 1;
      auto k = lpb_s == LNR_ENC_SPARSE_LPB ? k_hashgrid_fwd<PosFn, 1, LNR_ENC_PAIRED, LNR_ENC_SPARSE_LPB, true, true>
                                           : k_hashgrid_fwd<PosFn, 1, LNR_ENC_PAIRED, 1, true, true>;
      hipLaunchKernelGGL(k, dim3(gx, d->n_levels / lpb_s), dim3(kSB), 0, st, a, pos, ng, tb, enc, enc_stride,
                         BwdWorkspace{}, nullptr, ph);
      LNR_RETURN_LAUNCH(who);
    }
    if (ph.list) {
      auto k = lpb_c == 4 ? k_hashgrid_fwd<PosFn, 1, LNR_ENC_PAIRED, 4, true>
             : lpb_c == 2 ? k_hashgrid_fwd<PosFn, 1, LNR_ENC_PAIRED, 2, true>
                          : k_hashgrid_fwd<PosFn, 1, LNR_ENC_PAIRED, 1, true>;
      hipLaunchKernelGGL(k, dim3(rows_c, groups), dim3(kSB), 0, st, a, pos, ng, tb, enc, enc_stride,
                         BwdWorkspace{}, nullptr, ph);
      LNR_RETURN_LAUNCH(who);
    }
    auto k = lpb_c == 4 ? k_hashgrid_fwd<PosFn, 1, LNR_ENC_PAIRED, 4>
           : lpb_c == 2 ? k_hashgrid_fwd<PosFn, 1, LNR_ENC_PAIRED, 2>
                        : k_hashgrid_fwd<PosFn, 1, LNR_ENC_PAIRED, 1>;
    hipLaunchKernelGGL(k, dim3(rows_c, groups), dim3(kSB), 0, st, a, pos, ng, tb, enc, enc_stride,
                       BwdWorkspace{}, nullptr, ph);
    LNR_RETURN_LAUNCH(who);
  }
  if (live == nullptr)
    hipLaunchKernelGGL(enc_kernel(), dim3(rows, d->n_levels / lpb), dim3(kSB), 0, st, a, pos, n, tb, enc, enc_stride, w,
                       live, ph);
  else if (spt2 && live_lpb() == 2 && d->n_levels % 2 == 0 && enc_levels_per_group(d, rows) >= 2)
    // (two samples per thread over two levels spill at eight waves per SIMD: one sample per thread)
    hipLaunchKernelGGL((k_hashgrid_fwd<PosFn, 1, false, 2>), dim3(rows, d->n_levels / 2), dim3(kSB), 0, st, a, pos, n,
                       tb, enc, enc_stride, w, live, ph);
  else if (spt2)
    hipLaunchKernelGGL((k_hashgrid_fwd<PosFn, 2, false>), grid, dim3(kSB / 2), 0, st, a, pos, n, tb, enc, enc_stride, w,
                       live, ph);
  else
    hipLaunchKernelGGL((k_hashgrid_fwd<PosFn, 1, false>), grid, dim3(kSB), 0, st, a, pos, n, tb, enc, enc_stride, w,
                       live, ph);
  LNR_RETURN_LAUNCH(who);
}

extern "C" int lnr_hashgrid_fwd(const lnr_grid_desc* d, const float* pos01, int64_t n, const uint16_t* table,
                                uint32_t* enc, int64_t enc_stride, void* bwd_ws, int64_t bwd_ws_bytes,
                                void* stream) {
  if (int e = check_desc(d, "lnr_hashgrid_fwd")) return e;
  LNR_REQUIRE(n >= 0 && enc_stride >= n, "lnr_hashgrid_fwd: n=%lld stride=%lld", (long long)n, (long long)enc_stride);
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(pos01 && table && enc, "lnr_hashgrid_fwd: null pointer");
  return launch_fwd(d, PosFromArray{pos01}, n, table, enc, enc_stride, bwd_ws, bwd_ws_bytes, as_stream(stream),
                    "lnr_hashgrid_fwd");
}

extern "C" int lnr_hashgrid_fwd_rays(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                     int32_t n_samples, const uint16_t* table, uint32_t* enc, int64_t enc_stride,
                                     void* bwd_ws, int64_t bwd_ws_bytes, void* stream) {
  if (int e = check_desc(d, "lnr_hashgrid_fwd_rays")) return e;
  const int64_t n = n_rays * (int64_t)n_samples;
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && enc_stride >= n, "lnr_hashgrid_fwd_rays: bad sizes");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(rays && z && table && enc, "lnr_hashgrid_fwd_rays: null pointer");
  return launch_fwd(d, PosFromRays{rays, z, n_samples}, n, table, enc, enc_stride, bwd_ws, bwd_ws_bytes,
                    as_stream(stream), "lnr_hashgrid_fwd_rays");
}

extern "C" int lnr_hashgrid_fwd_rays_phase(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                           int32_t n_samples, const uint16_t* table, uint32_t* enc, int64_t enc_stride,
                                           void* bwd_ws, int64_t bwd_ws_bytes, const uint32_t* ray_list,
                                           const uint32_t* ray_count, int64_t expect_rays, int32_t lo, int32_t hi,
                                           void* stream) {
  if (int e = check_desc(d, "lnr_hashgrid_fwd_rays_phase")) return e;
  const int64_t n = n_rays * (int64_t)n_samples;
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && enc_stride >= n, "lnr_hashgrid_fwd_rays_phase: bad sizes");
  LNR_REQUIRE(n_samples % 64 == 0 && lo >= 0 && lo < hi && hi <= n_samples && lo % 64 == 0 && hi % 64 == 0,
              "lnr_hashgrid_fwd_rays_phase: phase [%d, %d) of %d samples must be whole 64-sample waves", lo, hi,
              n_samples);
  LNR_REQUIRE(bwd_ws == nullptr || (lo == 0 && ray_list == nullptr),
              "lnr_hashgrid_fwd_rays_phase: the record histogram comes with the first phase, over every ray");
  LNR_REQUIRE(ray_list == nullptr || ray_count != nullptr, "lnr_hashgrid_fwd_rays_phase: a ray list needs its count");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(rays && z && table && enc, "lnr_hashgrid_fwd_rays_phase: null pointer");
  const EncPhase ph{ray_list, ray_count, lo, hi, n_samples, bwd_ws == nullptr};
  return launch_fwd(d, PosFromRays{rays, z, n_samples}, n, table, enc, enc_stride, bwd_ws, bwd_ws_bytes,
                    as_stream(stream), "lnr_hashgrid_fwd_rays_phase", nullptr, ph, expect_rays);
}

extern "C" int lnr_hashgrid_fwd_rays_live(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                          int32_t n_samples, const uint16_t* table, const float* live, uint32_t* enc,
                                          int64_t enc_stride, void* stream) {
  if (int e = check_desc(d, "lnr_hashgrid_fwd_rays_live")) return e;
  const int64_t n = n_rays * (int64_t)n_samples;
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && enc_stride >= n, "lnr_hashgrid_fwd_rays_live: bad sizes");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(rays && z && table && enc && live, "lnr_hashgrid_fwd_rays_live: null pointer");
  return launch_fwd(d, PosFromRays{rays, z, n_samples}, n, table, enc, enc_stride, nullptr, 0, as_stream(stream),
                    "lnr_hashgrid_fwd_rays_live", live);
}

extern "C" int lnr_hashgrid_fwd_rays_live_ws(const lnr_grid_desc* d, const float* rays, const float* z,
                                             int64_t n_rays, int32_t n_samples, const uint16_t* table,
                                             const float* live, uint32_t* enc, int64_t enc_stride, void* bwd_ws,
                                             int64_t bwd_ws_bytes, void* stream) {
  if (int e = check_desc(d, "lnr_hashgrid_fwd_rays_live_ws")) return e;
  const int64_t n = n_rays * (int64_t)n_samples;
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && enc_stride >= n, "lnr_hashgrid_fwd_rays_live_ws: bad sizes");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(rays && z && table && enc && live && bwd_ws, "lnr_hashgrid_fwd_rays_live_ws: null pointer");
  return launch_fwd(d, PosFromRays{rays, z, n_samples}, n, table, enc, enc_stride, bwd_ws, bwd_ws_bytes,
                    as_stream(stream), "lnr_hashgrid_fwd_rays_live_ws", live);
}

extern "C" int lnr_hashgrid_bwd_atomic(const lnr_grid_desc* d, const float* pos01, int64_t n, const float* d_enc,
                                       int64_t enc_stride, float* d_table, void* stream) {
  if (int e = check_desc(d, "lnr_hashgrid_bwd_atomic")) return e;
  LNR_REQUIRE(n >= 0 && enc_stride >= n, "lnr_hashgrid_bwd: bad sizes");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(pos01 && d_enc && d_table, "lnr_hashgrid_bwd: null pointer");
  dim3 grid((unsigned)((n + 255) / 256), d->n_levels);
  hipLaunchKernelGGL(k_hashgrid_bwd<PosFromArray>, grid, dim3(256), 0, as_stream(stream), make_args(d),
                     PosFromArray{pos01}, n, reinterpret_cast<const float2*>(d_enc), enc_stride, d_table);
  LNR_RETURN_LAUNCH("lnr_hashgrid_bwd_atomic");
}

extern "C" int lnr_hashgrid_bwd_rays_atomic(const lnr_grid_desc* d, const float* rays, const float* z,
                                            int64_t n_rays, int32_t n_samples, const float* d_enc, int64_t enc_stride,
                                            float* d_table, void* stream) {
  if (int e = check_desc(d, "lnr_hashgrid_bwd_rays_atomic")) return e;
  const int64_t n = n_rays * (int64_t)n_samples;
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && enc_stride >= n, "lnr_hashgrid_bwd_rays: bad sizes");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(rays && z && d_enc && d_table, "lnr_hashgrid_bwd_rays: null pointer");
  dim3 grid((unsigned)((n + 255) / 256), d->n_levels);
  hipLaunchKernelGGL(k_hashgrid_bwd<PosFromRays>, grid, dim3(256), 0, as_stream(stream), make_args(d),
                     PosFromRays{rays, z, n_samples}, n, reinterpret_cast<const float2*>(d_enc), enc_stride, d_table);
  LNR_RETURN_LAUNCH("lnr_hashgrid_bwd_rays_atomic");
}

extern "C" int lnr_enc_to_aos(const uint32_t* enc, int64_t enc_stride, int64_t n, uint32_t n_levels, uint16_t* out,
                              void* stream) {
  LNR_REQUIRE(n >= 0 && enc_stride >= n && n_levels >= 1, "lnr_enc_to_aos: bad sizes");
  if (n == 0) return LNR_OK;
  const int64_t tot = n * n_levels;
  hipLaunchKernelGGL(k_enc_to_aos, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, as_stream(stream), enc,
                     enc_stride, n, n_levels, reinterpret_cast<uint32_t*>(out));
  LNR_RETURN_LAUNCH("lnr_enc_to_aos");
}

extern "C" int lnr_aos_grad_to_enc(const uint16_t* g16, const float* g32, int64_t n, uint32_t n_levels, float* d_enc,
                                   int64_t enc_stride, void* stream) {
  LNR_REQUIRE(n >= 0 && enc_stride >= n && n_levels >= 1, "lnr_aos_grad_to_enc: bad sizes");
  LNR_REQUIRE((g16 != nullptr) != (g32 != nullptr), "lnr_aos_grad_to_enc: exactly one of g16/g32 must be given");
  if (n == 0) return LNR_OK;
  const int64_t tot = n * n_levels;
  hipLaunchKernelGGL(k_aos_grad_to_enc, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, as_stream(stream), g16, g32,
                     n, n_levels, reinterpret_cast<float2*>(d_enc), enc_stride);
  LNR_RETURN_LAUNCH("lnr_aos_grad_to_enc");
}
