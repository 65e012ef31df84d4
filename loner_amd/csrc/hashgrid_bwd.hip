// Hash-grid backward (tcnn kernel_grid_backward semantics) as an atomic-free binned scatter.
//
// Measured on MI355X: scattered fp32 global atomics run at ~20 G lane-ops/s (memory-side
// execution) and LDS ds_add_f32 at only 0.33 lanes/clk/CU whatever the address pattern, while
// ds_add_u64 runs at 4.8 lanes/clk/CU (scratch/ubench_*.hip).  So the backward is
//   count   per (256-sample block, level) record histogram per 4096-entry table chunk
//           (emitted by the training forward, or by k_bwd_count)
//   scan    column prefix over blocks -> exact record offsets (no global atomics, no capacity guess)
//   scatter records {idx in chunk, g0, g1 as fp25} staged in LDS in bucket order and written
//           as coalesced runs; per-block max |g| for the fixed-point scale
//   accum   one workgroup per (bucket, slice): int64 fixed-point sums in a 64 KB LDS chunk with
//           ds_add_u64, converted back to fp32 and stored; a bucket split over several slices
//           stores per-slice int64 partial chunks that k_bwd_finalize adds exactly
// No float atomics anywhere: the result is bitwise reproducible, and d_table is overwritten.
// Coherent coarse levels merge runs of equal corner indices across lanes before emitting.
#include "hashgrid.hpp"

namespace lnr {

__device__ __forceinline__ uint32_t f32_to_f25(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x3Fu + ((u >> 7) & 1u);
  return u >> 7;
}
__device__ __forceinline__ float f25_to_f32(uint32_t v) { return __uint_as_float(v << 7); }

template <class PosFn>
__global__ void __launch_bounds__(kSB) k_bwd_count(GridArgs a, PosFn pos, int64_t n, BwdWorkspace ws) {
  __shared__ uint32_t hist[kMaxChunksPerLevel];
  const uint32_t l = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * kSB + threadIdx.x;
  const bool in = i < n;
  for (int b = threadIdx.x; b < kMaxChunksPerLevel; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  float x = 0.f, y = 0.f, z = 0.f;
  if (in) pos(i, x, y, z);
  Corners c;
  level_corners(a.lv[l], x, y, z, c);
  count_block_records(a, l, c, in, hist, ws);
}

// Exclusive prefix of every bucket column over the histogram rows of one scan chunk, offset by
// the preceding chunks' sums; chunk 0 also writes the bucket totals.  One thread per column,
// rows read whole (coalesced); grid (n_chunks, L).
__global__ void __launch_bounds__(kMaxChunksPerLevel) k_bwd_scan_rows(GridArgs a, BwdWorkspace ws) {
  const uint32_t l = blockIdx.y, ch = blockIdx.x, c = threadIdx.x;
  const uint32_t nb = a.bucket_base[l + 1] - a.bucket_base[l];
  if (c >= nb) return;
  const uint32_t* cs = ws.chunk_sum + (int64_t)l * ws.n_chunks * kMaxChunksPerLevel + c;
  uint32_t base = 0;
  for (uint32_t k = 0; k < ch; ++k) base += cs[(int64_t)k * kMaxChunksPerLevel];
  if (ch == 0) {
    uint32_t tot = 0;
    for (int64_t k = 0; k < ws.n_chunks; ++k) tot += cs[k * kMaxChunksPerLevel];
    ws.counts[a.bucket_base[l] + c] = tot;
  }
  uint32_t* col = ws.hist + (int64_t)a.bucket_base[l] * ws.n_sb + c;
  const int64_t r0 = (int64_t)ch * kRowsPerChunk;
  const int64_t r1 = r0 + kRowsPerChunk < ws.n_sb ? r0 + kRowsPerChunk : ws.n_sb;
  for (int64_t r = r0; r < r1; r += 16) {  // 16 row loads in flight
    uint32_t v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = r + u < r1 ? col[(r + u) * nb] : 0u;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (r + u < r1) col[(r + u) * nb] = base;
      base += v[u];
    }
  }
}

// Bucket segment starts, work-item (slice) prefix and split-bucket partial prefix.
__global__ void __launch_bounds__(1024) k_bwd_scan_buckets(BwdWorkspace ws, uint32_t n_buckets) {
  __shared__ uint64_t w_seg[16];
  __shared__ uint32_t w_sl[16], w_pp[16];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  // two buckets per thread (n_buckets <= kMaxBuckets = 2048)
  uint64_t seg[2];
  uint32_t sl[2], pp[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const uint32_t b = 2 * t + q;
    const uint32_t c = b < n_buckets ? ws.counts[b] : 0u;
    const uint32_t k = (uint32_t)((c + kSliceRecords - 1) / kSliceRecords);
    seg[q] = c;
    sl[q] = b < n_buckets ? (k > 0 ? k : 1) : 0u;
    pp[q] = b < n_buckets && k > 1 ? k : 0u;
  }
  uint64_t iseg = seg[0] + seg[1];
  uint32_t isl = sl[0] + sl[1], ipp = pp[0] + pp[1];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t a0 = __shfl_up(iseg, o, 64);
    const uint32_t a1 = __shfl_up(isl, o, 64), a2 = __shfl_up(ipp, o, 64);
    if (lane >= o) {
      iseg += a0;
      isl += a1;
      ipp += a2;
    }
  }
  if (lane == 63) {
    w_seg[wid] = iseg;
    w_sl[wid] = isl;
    w_pp[wid] = ipp;
  }
  __syncthreads();
  uint64_t bseg = 0;
  uint32_t bsl = 0, bpp = 0;
  for (int w = 0; w < wid; ++w) {
    bseg += w_seg[w];
    bsl += w_sl[w];
    bpp += w_pp[w];
  }
  // exclusive values at this thread's first bucket
  uint64_t e_seg = bseg + iseg - seg[0] - seg[1];
  uint32_t e_sl = bsl + isl - sl[0] - sl[1], e_pp = bpp + ipp - pp[0] - pp[1];
  if (t == 1023) {  // totals (n_buckets may equal 2 * blockDim)
    ws.seg_start[n_buckets] = bseg + iseg;
    ws.slice_pre[n_buckets] = bsl + isl;
    ws.part_pre[n_buckets] = bpp + ipp;
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const uint32_t b = 2 * t + q;
    if (b < n_buckets) {
      ws.seg_start[b] = e_seg;
      ws.slice_pre[b] = e_sl;
      ws.part_pre[b] = e_pp;
    }
    e_seg += seg[q];
    e_sl += sl[q];
    e_pp += pp[q];
  }
}

// One workgroup per (histogram row, level): kSB samples, 8 records each, staged in LDS in bucket
// order and written as one contiguous run per bucket.
template <class PosFn>
__global__ void __launch_bounds__(kSB) k_bwd_scatter(GridArgs a, PosFn pos, int64_t n, const float2* __restrict__ d_enc,
                                                     int64_t stride, BwdWorkspace ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t* stage = reinterpret_cast<uint64_t*>(smem);                // [8 * kSB]
  uint64_t* gbase = stage + 8 * kSB;                                  // [kMaxChunksPerLevel]
  uint32_t* hist = reinterpret_cast<uint32_t*>(gbase + kMaxChunksPerLevel);  // [kMaxChunksPerLevel]
  uint32_t* start = hist + kMaxChunksPerLevel;                        // [kMaxChunksPerLevel + 1]
  float* wmax = reinterpret_cast<float*>(start + kMaxChunksPerLevel + 1);    // [kSB / 64]
  uint8_t* sbk = reinterpret_cast<uint8_t*>(wmax + kSB / 64);         // [8 * kSB]
  const uint32_t l = blockIdx.y;
  const int64_t sb = blockIdx.x;
  const int64_t i = sb * kSB + threadIdx.x;
  const bool in = i < n;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t b0 = a.bucket_base[l];
  const uint32_t nb = a.bucket_base[l + 1] - b0;
  const uint32_t* row = hist_row(a, ws, l, sb);
  for (uint32_t b = threadIdx.x; b < kMaxChunksPerLevel; b += kSB) {
    hist[b] = 0;
    if (b < nb) gbase[b] = ws.seg_start[b0 + b] + row[b];
  }
  __syncthreads();
  float x = 0.f, y = 0.f, z = 0.f;
  float2 g = make_float2(0.f, 0.f);
  if (in) {
    pos(i, x, y, z);
    g = d_enc[(int64_t)l * stride + i];
  }
  Corners c;
  level_corners(a.lv[l], x, y, z, c);
  const bool coherent = l < a.merge_levels;
  const uint32_t off = a.lv[l].offset;
  uint32_t e[8], rank[8];
  uint64_t rec[8];
  bool valid[8];
  float m = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t idx = in ? c.idx[k] : 0xFFFFFFFFu;
    float v0 = c.w[k] * g.x, v1 = c.w[k] * g.y;
    valid[k] = in;
    if (coherent) {
      const RunInfo ri = lane_runs(idx);
      run_sum(ri, v0, v1);
      valid[k] = in && ri.tail;
    }
    e[k] = valid[k] ? idx - off : 0u;
    rank[k] = wave_bucket_rank(hist, e[k] >> kChunkLog2, valid[k], coherent);
    const uint32_t q0 = f32_to_f25(v0), q1 = f32_to_f25(v1);
    rec[k] = (uint64_t)(e[k] & (kChunk - 1)) | ((uint64_t)q0 << 13) | ((uint64_t)q1 << 38);
    if (valid[k]) m = fmaxf(m, fmaxf(fabsf(f25_to_f32(q0)), fabsf(f25_to_f32(q1))));
  }
  m = wave_max(m);
  if (lane == 0) wmax[wid] = m;
  __syncthreads();
  if (wid == 0) {  // exclusive prefix of the (<= 128) bucket counts: 2 per lane + a wave scan
    const uint32_t c0 = 2 * lane < nb ? hist[2 * lane] : 0u;
    const uint32_t c1 = 2 * lane + 1 < nb ? hist[2 * lane + 1] : 0u;
    uint32_t inc = c0 + c1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t q = __shfl_up(inc, o, 64);
      if (lane >= o) inc += q;
    }
    const uint32_t ex = inc - c0 - c1;
    if (2 * lane <= nb) start[2 * lane] = ex;
    if (2 * lane + 1 <= nb) start[2 * lane + 1] = ex + c0;
    if (lane == 63) start[nb] = inc;  // the total (nb = 128 has no lane whose pair reaches it)
    float mm = lane < kSB / 64 ? wmax[lane] : 0.f;
    mm = wave_max(mm);
    if (lane == 0) ws.blockmax[(int64_t)l * ws.n_sb + sb] = mm;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (valid[k]) {
      const uint32_t ch = e[k] >> kChunkLog2;
      const uint32_t slot = start[ch] + rank[k];
      if (slot < 8 * kSB) {  // always true when counts and ranks agree; guards the LDS stage
        stage[slot] = rec[k];
        sbk[slot] = (uint8_t)ch;
      }
    }
  }
  __syncthreads();
  const uint32_t total = start[nb] < 8u * kSB ? start[nb] : 8u * kSB;
  for (uint32_t t = threadIdx.x; t < total; t += kSB) {
    const uint32_t ch = sbk[t];
    __builtin_nontemporal_store(stage[t], &ws.records[gbase[ch] + (t - start[ch])]);  // read once, later
  }
}

constexpr size_t kScatterLds = 8 * kSB * 8 + kMaxChunksPerLevel * 8 + kMaxChunksPerLevel * 4 +
                               (kMaxChunksPerLevel + 1) * 4 + (kSB / 64) * 4 + 8 * kSB;

__global__ void __launch_bounds__(256) k_bwd_level_max(BwdWorkspace ws) {
  __shared__ float red[4];
  const float* col = ws.blockmax + (int64_t)blockIdx.x * ws.n_sb;
  float m = 0.f;
  for (int64_t j = threadIdx.x; j < ws.n_sb; j += 256) m = fmaxf(m, col[j]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) ws.level_max[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

constexpr int kAccumThreads = 1024;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(kAccumThreads) k_bwd_accum(GridArgs a, BwdWorkspace ws, float* __restrict__ d_table) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem);  // [kChunk][2] int64 fixed point
  const uint32_t nbk = a.n_buckets;
  const uint32_t total = ws.slice_pre[nbk];
  const int lane = threadIdx.x & 63;
  for (uint32_t s = blockIdx.x; s < total; s += gridDim.x) {
    uint32_t lo = 0, hi = nbk;  // bucket b with slice_pre[b] <= s < slice_pre[b+1]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (ws.slice_pre[mid] <= s) lo = mid;
      else hi = mid;
    }
    const uint32_t b = lo;
    const uint32_t nsl = ws.slice_pre[b + 1] - ws.slice_pre[b];
    const uint32_t j = s - ws.slice_pre[b];
    const uint64_t beg = ws.seg_start[b] + (uint64_t)j * kSliceRecords;
    uint64_t end = ws.seg_start[b + 1];
    if (beg + kSliceRecords < end) end = beg + kSliceRecords;
    uint32_t l = 0;
    while (l + 1 < a.n_levels && a.bucket_base[l + 1] <= b) ++l;
    const uint32_t chunk = b - a.bucket_base[l];
    const uint32_t ent0 = chunk * kChunk;
    const uint32_t nent = (a.lv[l].size - ent0) < (uint32_t)kChunk ? (a.lv[l].size - ent0) : (uint32_t)kChunk;
    // fixed-point scale: |v| < 2^E, at most `cnt` records in the whole bucket -> |sum| < 2^62
    // (one scale per bucket, so split buckets' int64 partials add exactly)
    int E;
    frexpf(ws.level_max[l], &E);
    const uint64_t bcnt = ws.seg_start[b + 1] - ws.seg_start[b];
    const uint64_t cnt = bcnt > 0 ? bcnt : 1;
    const int lg = 64 - __clzll((long long)cnt);  // ceil-ish log2(cnt + 1)
    int k2 = 62 - lg - E;
    k2 = k2 > 120 ? 120 : (k2 < -120 ? -120 : k2);
    const float scale = ldexpf(1.f, k2);
    for (int t = threadIdx.x; t < 2 * kChunk; t += blockDim.x) acc[t] = 0ull;
    __syncthreads();
    const bool coherent = l < a.merge_levels;
#ifdef LNR_EXP_NO_LDS_ATOMICS
    long long dummy = 0;
#endif
    const uint64_t* rec = ws.records;
    // 16-B loads (2 records per lane), 4 in flight: 8 KB per wave trip; a lane's two records are
    // handled as two lane-ordered streams (merging of equal entries is an optimisation only)
    const uint64_t beg2 = beg & ~1ull;
    for (uint64_t rb = beg2 + 2 * (threadIdx.x & ~63u); rb < end; rb += 8 * kAccumThreads) {  // wave-uniform
      u64x2 q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t rr = rb + 2 * lane + (uint64_t)u * 2 * kAccumThreads;
        q[u] = rr < end ? __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(&rec[rr])) : u64x2{~0ull, ~0ull};
        if (rr < beg) q[u].x = ~0ull;
        if (rr + 1 >= end) q[u].y = ~0ull;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint64_t v = (u & 1) ? q[u >> 1].y : q[u >> 1].x;
        const bool ok = v != ~0ull;
        const uint32_t ee = ok ? (uint32_t)(v & (kChunk - 1)) : 0xFFFFFFFFu;
        const float v0 = ok ? f25_to_f32((uint32_t)(v >> 13) & 0x1FFFFFFu) : 0.f;
        const float v1 = ok ? f25_to_f32((uint32_t)(v >> 38) & 0x1FFFFFFu) : 0.f;
        long long i0 = __float2ll_rn(v0 * scale), i1 = __float2ll_rn(v1 * scale);
        bool emit = ok;
        if (coherent) {  // records of coherent levels arrive in runs of equal entries; merged in
          const RunInfo ri = lane_runs(ee);  // int64 so the sum does not depend on record order
          run_sum_i64(ri, i0, i1);
          emit = ok && ri.tail;
        }
#ifdef LNR_EXP_NO_LDS_ATOMICS
        if (emit) dummy += i0 + i1 + ee;
#else
        if (emit) {
          atomicAdd(&acc[2 * ee + 0], (unsigned long long)i0);
          atomicAdd(&acc[2 * ee + 1], (unsigned long long)i1);
        }
#endif
      }
    }
#ifdef LNR_EXP_NO_LDS_ATOMICS
    if (dummy == 0x123456789LL) acc[threadIdx.x] = dummy;
#endif
    __syncthreads();
    if (nsl == 1) {  // the final values
      const float inv = ldexpf(1.f, -k2);
      float* dst = d_table + 2 * ((int64_t)a.lv[l].offset + ent0);
      for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x) dst[t] = (float)(long long)acc[t] * inv;
    } else {  // this slice's int64 partial chunk
      long long* dst = ws.partial + (int64_t)(ws.part_pre[b] + j) * (2 * kChunk);
      for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x) dst[t] = (long long)acc[t];
    }
    __syncthreads();
  }
}

// Split buckets: d_table = sum of the slices' partial chunks, in slice order (deterministic).
__global__ void __launch_bounds__(256) k_bwd_finalize(GridArgs a, BwdWorkspace ws, float* __restrict__ d_table) {
  const uint32_t b = blockIdx.x;
  const uint32_t nsl = ws.part_pre[b + 1] - ws.part_pre[b];
  if (nsl == 0) return;
  uint32_t l = 0;
  while (l + 1 < a.n_levels && a.bucket_base[l + 1] <= b) ++l;
  const uint32_t ent0 = (b - a.bucket_base[l]) * kChunk;
  const uint32_t nent = (a.lv[l].size - ent0) < (uint32_t)kChunk ? (a.lv[l].size - ent0) : (uint32_t)kChunk;
  // the accumulate kernel's per-bucket scale
  int E;
  frexpf(ws.level_max[l], &E);
  const uint64_t bcnt = ws.seg_start[b + 1] - ws.seg_start[b];
  const int lg = 64 - __clzll((long long)(bcnt > 0 ? bcnt : 1));
  int k2 = 62 - lg - E;
  k2 = k2 > 120 ? 120 : (k2 < -120 ? -120 : k2);
  const float inv = ldexpf(1.f, -k2);
  const long long* src = ws.partial + (int64_t)ws.part_pre[b] * (2 * kChunk);
  float* dst = d_table + 2 * ((int64_t)a.lv[l].offset + ent0);
  for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x) {
    long long v = 0;
    for (uint32_t k = 0; k < nsl; ++k) v += src[(int64_t)k * (2 * kChunk) + t];
    dst[t] = (float)v * inv;
  }
}

template <class PosFn>
static int launch_bwd_bucketed(const lnr_grid_desc* d, PosFn pos, int64_t n, const float* d_enc, int64_t stride,
                               float* d_table, void* workspace, int64_t ws_bytes, int32_t flags, hipStream_t st,
                               const char* who) {
  GridArgs a = make_args(d);
  LNR_REQUIRE(a.n_buckets <= (uint32_t)kMaxBuckets, "%s: too many table chunks (%u)", who, a.n_buckets);
  for (uint32_t l = 0; l < d->n_levels; ++l)
    LNR_REQUIRE(a.bucket_base[l + 1] - a.bucket_base[l] <= (uint32_t)kMaxChunksPerLevel,
                "%s: level %u has more than %d table chunks", who, l, kMaxChunksPerLevel);
  LNR_REQUIRE(workspace != nullptr && ws_bytes >= bwd_workspace_bytes(d, n),
              "%s: workspace too small (%lld < %lld bytes)", who, (long long)ws_bytes,
              (long long)bwd_workspace_bytes(d, n));
  LNR_REQUIRE(n < (int64_t(1) << 31), "%s: n=%lld samples exceeds 2^31", who, (long long)n);
  BwdWorkspace w = carve_workspace(workspace, a, d, n);
  static bool lds_attr = false;  // scatter stages 8 records per sample of its row in LDS (> 64 KB)
  if (!lds_attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_bwd_scatter<PosFn>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kScatterLds) != hipSuccess) {
      set_error("%s: cannot raise the scatter kernel's LDS limit to %zu bytes", who, kScatterLds);
      return LNR_ERR_HIP;
    }
    lds_attr = true;
  }
  dim3 grid((unsigned)w.n_sb, d->n_levels);
  if (!(flags & LNR_BWD_COUNTS_READY)) {
    int64_t off, bytes;
    chunk_sum_range(d, n, &off, &bytes);
    if (hipMemsetAsync(reinterpret_cast<char*>(workspace) + off, 0, bytes, st) != hipSuccess) {
      set_error("%s: hipMemsetAsync failed", who);
      return LNR_ERR_HIP;
    }
    hipLaunchKernelGGL(k_bwd_count<PosFn>, grid, dim3(kSB), 0, st, a, pos, n, w);
  }
  hipLaunchKernelGGL(k_bwd_scan_rows, dim3((unsigned)w.n_chunks, d->n_levels), dim3(kMaxChunksPerLevel), 0, st, a, w);
  hipLaunchKernelGGL(k_bwd_scan_buckets, dim3(1), dim3(1024), 0, st, w, a.n_buckets);
  hipLaunchKernelGGL(k_bwd_scatter<PosFn>, grid, dim3(kSB), kScatterLds, st, a, pos, n,
                     reinterpret_cast<const float2*>(d_enc), stride, w);
  hipLaunchKernelGGL(k_bwd_level_max, dim3(d->n_levels), dim3(256), 0, st, w);
  const int64_t max_slices = a.n_buckets + (8 * n * (int64_t)d->n_levels) / kSliceRecords + 1;
  const unsigned g = (unsigned)(max_slices < 4096 ? max_slices : 4096);
  hipLaunchKernelGGL(k_bwd_accum, dim3(g), dim3(kAccumThreads), 2 * kChunk * sizeof(unsigned long long), st, a, w, d_table);
  hipLaunchKernelGGL(k_bwd_finalize, dim3(a.n_buckets), dim3(256), 0, st, a, w, d_table);
  LNR_RETURN_LAUNCH(who);
}

static int check_desc_bwd(const lnr_grid_desc* d, const char* who) {
  LNR_REQUIRE(d != nullptr && d->n_levels >= 1 && d->n_levels <= LNR_MAX_LEVELS && d->n_features == 2,
              "%s: invalid grid descriptor", who);
  return LNR_OK;
}

}  // namespace lnr

using namespace lnr;

extern "C" int64_t lnr_hashgrid_bwd_workspace_bytes(const lnr_grid_desc* d, int64_t n) {
  if (d == nullptr || n < 0) return -1;
  return bwd_workspace_bytes(d, n);
}

extern "C" int lnr_hashgrid_bwd(const lnr_grid_desc* d, const float* pos01, int64_t n, const float* d_enc,
                                int64_t enc_stride, float* d_table, void* workspace, int64_t workspace_bytes,
                                int32_t flags, void* stream) {
  if (int e = check_desc_bwd(d, "lnr_hashgrid_bwd")) return e;
  LNR_REQUIRE(n >= 0 && enc_stride >= n, "lnr_hashgrid_bwd: bad sizes");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(pos01 && d_enc && d_table, "lnr_hashgrid_bwd: null pointer");
  return launch_bwd_bucketed(d, PosFromArray{pos01}, n, d_enc, enc_stride, d_table, workspace, workspace_bytes, flags,
                             as_stream(stream), "lnr_hashgrid_bwd");
}

extern "C" int lnr_hashgrid_bwd_rays(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                     int32_t n_samples, const float* d_enc, int64_t enc_stride, float* d_table,
                                     void* workspace, int64_t workspace_bytes, int32_t flags, void* stream) {
  if (int e = check_desc_bwd(d, "lnr_hashgrid_bwd_rays")) return e;
  const int64_t n = n_rays * (int64_t)n_samples;
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && enc_stride >= n, "lnr_hashgrid_bwd_rays: bad sizes");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(rays && z && d_enc && d_table, "lnr_hashgrid_bwd_rays: null pointer");
  return launch_bwd_bucketed(d, PosFromRays{rays, z, n_samples}, n, d_enc, enc_stride, d_table, workspace,
                             workspace_bytes, flags, as_stream(stream), "lnr_hashgrid_bwd_rays");
}
