// Hash-grid backward (tcnn kernel_grid_backward semantics) as an atomic-free binned scatter.
//
// Measured on MI355X: scattered fp32 global atomics run at ~20 G lane-ops/s (memory-side
// execution) and LDS ds_add_f32 at only 0.33 lanes/clk/CU whatever the address pattern, while
// ds_add_u64 runs at 4.8 lanes/clk/CU.  So the backward is
//   count    per (512-sample row, level) record histogram over the level's 4096-entry table chunks
//            (buckets), emitted by the training forward (k_hashgrid_fwd given the workspace) or by k_bwd_count
//   scan     k_bwd_chunk_sums + k_bwd_scan_rows (column prefix over 64-row chunks) + k_bwd_scan_buckets:
//            exact per-row record offsets in every bucket (no global atomics, no capacity guess)
//   scatter  k_bwd_scatter_rows: one workgroup per row walks all 16 levels; 8-byte records {word,
//            fp16 value pair at the level's power-of-two scale} (hashgrid.hpp "Backward records": one
//            per x-pair of corners at fine levels, one per corner of a run of lanes in one cell at the
//            coherent levels) are ranked with LDS atomics, staged in bucket order and copied out as
//            runs; a (row, level) with more records than the stage holds writes each to its slot
//   accum    k_bwd_accum: the records of a bucket range split evenly over 512 workgroups, each adding
//            its pieces into a 64 KB LDS chunk of int64 fixed point (ds_add_u64) and storing fp32 (a
//            whole bucket) or an int64 partial chunk (a bucket its range boundaries cut) that
//            k_bwd_finalize adds in workgroup order.  Small batches take k_bwd_accum_buckets instead:
//            one workgroup per whole bucket, no partials and no finalize (accum_buckets_max_n); mid-size
//            ones (a data-parallel shard) k_bwd_accum_units: a work list of whole buckets and equal
//            pieces of the large ones, so only those leave partial chunks (accum_units).
// No float atomics anywhere: the result is bitwise reproducible, and d_table is overwritten.
#include "hashgrid.hpp"

namespace lnr {

// Histogram after the MLP backward: samples whose d_enc is zero at a non-coherent level (ReLU'd
// sigma: relu(sigma + noise) = 0 gives dL/dsigma = 0 exactly, typically half the samples) emit no
// records there; the scatter skips them the same way (skip_zero).
template <class PosFn, class GradFn>
__global__ void __launch_bounds__(kSB) k_bwd_count(GridArgs a, PosFn pos, int64_t n, GradFn grad, BwdWorkspace ws) {
  __shared__ uint32_t hist[kMaxChunksPerLevel];
  const uint32_t l = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * kSB + threadIdx.x;
  const bool in = i < n;
  for (int b = threadIdx.x; b < kMaxChunksPerLevel; b += blockDim.x) hist[b] = 0;
  float x = 0.f, y = 0.f, z = 0.f;
  bool act = false;
  if (in) {
    pos(i, x, y, z);
    const float2 g = grad.load(l, i);
    act = grad.live_at(i) && (g.x != 0.f || g.y != 0.f);
  }
  lds_barrier();
  if (a.lv[l].fine) {
    FineCell c;
    fine_cell(a.lv[l], x, y, z, c);
    count_block_records_fine(a, l, c, act, hist, ws);
  } else {
    Corners c;
    level_corners(a.lv[l], x, y, z, c);
    count_block_records(a, l, c, in, l < a.merge_levels ? in : act, hist, ws);
  }
}

// Column sums of the histogram rows of one scan chunk (kRowsPerChunk rows); grid (n_chunks, L).
__global__ void __launch_bounds__(kMaxChunksPerLevel) k_bwd_chunk_sums(GridArgs a, BwdWorkspace ws) {
  const uint32_t l = blockIdx.y, ch = blockIdx.x, c = threadIdx.x;
  const uint32_t nb = a.bucket_base[l + 1] - a.bucket_base[l];
  if (c >= nb) return;
  const uint32_t* col = ws.hist + (int64_t)a.bucket_base[l] * ws.n_sb + c;
  const int64_t nrows = ws.use_live ? (int64_t)ws.live[1] : ws.n_sb;  // (the live histogram's rows)
  const int64_t r0 = (int64_t)ch * kRowsPerChunk;
  const int64_t r1 = r0 + kRowsPerChunk < nrows ? r0 + kRowsPerChunk : nrows;
  uint32_t s = 0;
  for (int64_t r = r0; r < r1; r += 16) {  // 16 row loads in flight
    uint32_t v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = r + u < r1 ? col[(r + u) * nb] : 0u;
#pragma unroll
    for (int u = 0; u < 16; ++u) s += v[u];
  }
  ws.chunk_sum[((int64_t)l * ws.n_chunks + ch) * kMaxChunksPerLevel + c] = s;
}

// Exclusive prefix of every bucket column over the histogram rows of one scan chunk, offset by
// the preceding chunks' sums; chunk 0 also writes the bucket totals.  One thread per column,
// rows read whole (coalesced); grid (n_chunks, L).
__global__ void __launch_bounds__(kMaxChunksPerLevel) k_bwd_scan_rows(GridArgs a, BwdWorkspace ws) {
  const uint32_t l = blockIdx.y, ch = blockIdx.x, c = threadIdx.x;
  const uint32_t nb = a.bucket_base[l + 1] - a.bucket_base[l];
  if (c >= nb) return;
  const uint32_t* cs = ws.chunk_sum + (int64_t)l * ws.n_chunks * kMaxChunksPerLevel + c;
  uint32_t base = 0, tot = 0;  // the preceding chunks' sum; all chunks' (the bucket total, chunk 0)
  const int64_t nrows = ws.use_live ? (int64_t)ws.live[1] : ws.n_sb;  // (the live histogram's rows)
  // one chunk (a small batch): no k_bwd_chunk_sums launch, the total is this chunk's own column sum
  const int64_t kend = ws.n_chunks == 1 ? 0 : ch == 0 ? ws.n_chunks : ch;
  if (ws.n_chunks == 1) {
    const uint32_t* col = ws.hist + (int64_t)a.bucket_base[l] * ws.n_sb + c;
    for (int64_t r = 0; r < nrows; r += 16) {
      uint32_t v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = r + u < nrows ? col[(r + u) * nb] : 0u;
#pragma unroll
      for (int u = 0; u < 16; ++u) tot += v[u];
    }
  }
  for (int64_t k = 0; k < kend; k += 16) {  // 16 loads in flight (L2 hits)
    uint32_t v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = k + u < kend ? cs[(k + u) * kMaxChunksPerLevel] : 0u;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (k + u < (int64_t)ch) base += v[u];
      tot += v[u];
    }
  }
  if (ch == 0) ws.counts[a.bucket_base[l] + c] = tot;
  uint32_t* col = ws.hist + (int64_t)a.bucket_base[l] * ws.n_sb + c;
  const int64_t r0 = (int64_t)ch * kRowsPerChunk;
  const int64_t r1 = r0 + kRowsPerChunk < nrows ? r0 + kRowsPerChunk : nrows;
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

// The unit accumulation's work list for buckets [b0, b0 + nb) holding R records (see UnitTable):
// thread t's buckets are b0 + 2t and b0 + 2t + 1, with record counts cnt.  One 1024-thread block.
constexpr uint64_t kUnitMinRecords = 2048;  // one accumulate tile (kTile): no smaller pieces
__device__ __forceinline__ void build_units(UnitTable* ut, uint32_t b0, uint32_t nb, const uint64_t (&cnt)[2],
                                            uint64_t R, uint64_t* scratch /* LDS [16] */) {
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const uint64_t T0 = (R + kAccumGroups - 1) / kAccumGroups;
  const uint64_t T = T0 > kUnitMinRecords ? T0 : kUnitMinRecords;
  uint32_t P[2];
  uint64_t pk[2];  // packed counters: units (bits 0-20), partial chunks (21-41), cut buckets (42-)
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    P[q] = 2 * t + q < (int)nb ? (cnt[q] <= T ? 1u : (uint32_t)((cnt[q] + T - 1) / T)) : 0u;
    pk[q] = (uint64_t)P[q] | ((uint64_t)(P[q] > 1 ? P[q] : 0u) << 21) | ((uint64_t)(P[q] > 1 ? 1u : 0u) << 42);
  }
  uint64_t inc = pk[0] + pk[1];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  if (lane == 63) scratch[wid] = inc;
  lds_barrier();
  uint64_t ex = inc - pk[0] - pk[1], tot = 0;
  for (int w = 0; w < 16; ++w) {
    if (w < wid) ex += scratch[w];
    tot += scratch[w];
  }
  constexpr uint64_t m21 = (1ull << 21) - 1;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (P[q]) {
      const uint32_t b = b0 + 2 * t + q, u0 = (uint32_t)(ex & m21), s0 = (uint32_t)((ex >> 21) & m21);
      for (uint32_t k = 0; k < P[q]; ++k) ut->unit[u0 + k] = make_uint2(b, (k << 16) | P[q]);
      if (P[q] > 1) {
        ut->slot[b] = s0;
        ut->cut[ex >> 42] = make_uint2(b, P[q]);
      }
    }
    ex += pk[q];
  }
  if (t == 0) {
    ut->n_units = (uint32_t)(tot & m21);
    ut->n_cut = (uint32_t)(tot >> 42);
  }
}

// Bucket segment starts: exclusive prefix of the bucket totals (records are laid out bucket-major),
// and the unit accumulation's work list over all buckets.
__global__ void __launch_bounds__(1024) k_bwd_scan_buckets(BwdWorkspace ws, uint32_t n_buckets) {
  __shared__ uint64_t w_seg[16], w_units[16];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  uint64_t seg[2];  // two buckets per thread (n_buckets <= kMaxBuckets = 2048)
#pragma unroll
  for (int q = 0; q < 2; ++q) seg[q] = 2 * t + q < (int)n_buckets ? ws.counts[2 * t + q] : 0u;
  uint64_t iseg = seg[0] + seg[1];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t a0 = __shfl_up(iseg, o, 64);
    if (lane >= o) iseg += a0;
  }
  if (lane == 63) w_seg[wid] = iseg;
  lds_barrier();
  uint64_t bseg = 0, total = 0;
  for (int w = 0; w < 16; ++w) {
    if (w < wid) bseg += w_seg[w];
    total += w_seg[w];
  }
  uint64_t e_seg = bseg + iseg - seg[0] - seg[1];  // exclusive value at this thread's first bucket
  if (t == 1023) ws.seg_start[n_buckets] = bseg + iseg;  // total (n_buckets may equal 2 * blockDim)
  ws.bucket_done[2 * t] = 0u;  // k_bwd_accum<true>'s arrival counters (kMaxBuckets = 2 * blockDim)
  ws.bucket_done[2 * t + 1] = 0u;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (2 * t + q < (int)n_buckets) ws.seg_start[2 * t + q] = e_seg;
    e_seg += seg[q];
  }
  build_units(ws.units, 0, n_buckets, seg, total, w_units);
}

// The work list for a sub-range [b0, b1) of the buckets (the accumulation by level range, for the
// bucketed gradient exchange); k_bwd_scan_buckets made the whole range's.
__global__ void __launch_bounds__(1024) k_bwd_units(BwdWorkspace ws, uint32_t b0, uint32_t b1) {
  __shared__ uint64_t w_r[16], w_units[16];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const uint32_t nb = b1 - b0;
  uint64_t cnt[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) cnt[q] = 2 * t + q < (int)nb ? ws.counts[b0 + 2 * t + q] : 0u;
  uint64_t r = cnt[0] + cnt[1];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) r += __shfl_xor(r, o, 64);
  if (lane == 0) w_r[wid] = r;
  lds_barrier();
  uint64_t R = 0;
  for (int w = 0; w < 16; ++w) R += w_r[w];
  build_units(ws.units, b0, nb, cnt, R, w_units);
}

// ---------------------------------------------------------------- the live backward (LNR_BWD_LIVE)
// A sample whose dL/dsigma is exactly 0 (relu(sigma + noise) = 0, rendering_tcnn.py:252,260: most of a trained
// field's free-space samples) adds exactly 0 to every table entry.  The live backward places records only for the
// live samples: fine levels emit a sample's records iff dL/dsigma != 0, coherent levels a run's records iff the run
// holds a live lane, and a wave without a live lane skips all of its work.  Everything else is the full
// backward's: the same rows, the same run merging over the same lanes (dead lanes add zeros), the same record
// values, and the same fixed-point unit (bwd_fixed_k2: from N, not from the counts), so the int64 sums, and the
// gradient, are bitwise those of the full backward.  It counts its own records (k_bwd_count_live): the forward
// need not record a histogram for it.

// Whether lane's run [head_lane, lane] holds a live lane (wl: the wave's live lanes)
__device__ __forceinline__ bool run_live(unsigned long long wl, const RunInfo& ri) {
  const int lane = threadIdx.x & 63;
  const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  return (wl & upto & ~((1ull << ri.head_lane) - 1ull)) != 0ull;
}

// The live waves: wflags[w] = some sample of the 64-sample group w has dL/dsigma != 0 (16 threads of 4 samples
// per group), then k_bwd_live_list lists them in order and counts them (ws.live: waves, rows of 8).
__global__ void __launch_bounds__(256) k_bwd_live_flags(const float* __restrict__ dsig, int64_t n, BwdWorkspace ws) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t i = 4 * t;
  bool lv = false;
#pragma unroll
  for (int k = 0; k < 4; ++k) lv = lv || (i + k < n && dsig[i + k] != 0.f);
  const unsigned long long b = __ballot(lv);
  const int lane = threadIdx.x & 63;
  if ((lane & 15) == 0 && i < n) ws.wflags[t >> 4] = ((b >> lane) & 0xFFFFull) != 0ull ? 1 : 0;
}
// One workgroup: passes of 1024 x 64 wave flags, each thread listing the live ones among its 64 in order.
__global__ void __launch_bounds__(1024) k_bwd_live_list(int64_t n_waves, BwdWorkspace ws) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  if (t == 0) carry = 0u;
  for (int64_t p0 = 0; p0 < n_waves; p0 += 1024 * 64) {
    const int64_t f0 = p0 + 64 * (int64_t)t;
    unsigned long long m = 0ull;
    if (f0 + 64 <= n_waves) {  // 64 flags in four 16-B loads (the flags array is 256-B aligned)
      uint4 q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = reinterpret_cast<const uint4*>(ws.wflags + f0)[k];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t wd = k % 4 == 0 ? q[k / 4].x : k % 4 == 1 ? q[k / 4].y : k % 4 == 2 ? q[k / 4].z : q[k / 4].w;
#pragma unroll
        for (int b = 0; b < 4; ++b) m |= ((wd >> (8 * b)) & 0xFFu) ? 1ull << (4 * k + b) : 0ull;
      }
    } else {
      for (int k = 0; k < 64; ++k)
        if (f0 + k < n_waves && ws.wflags[f0 + k]) m |= 1ull << k;
    }
    const uint32_t c = (uint32_t)__popcll(m);
    const uint32_t inc = wave_incl_scan_u32(c);
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t off = carry, tot = carry;
    for (int w = 0; w < 16; ++w) {
      if (w < wid) off += wsum[w];
      tot += wsum[w];
    }
    off += inc - c;
    while (m) {
      const int k = __builtin_ctzll(m);
      m &= m - 1ull;
      ws.wlist[off++] = (uint32_t)(f0 + k);
    }
    __syncthreads();
    if (t == 0) carry = tot;
    __syncthreads();
  }
  if (t == 0) {
    ws.live[0] = carry;
    ws.live[1] = (carry + 7u) / 8u;
  }
}

// The live backward's histogram: row r = the live waves 8r .. 8r + 7 (one per wave of the workgroup), every level,
// the records k_bwd_scatter_rows<LIVE> places (above).  NL levels, the first NM coherent, at most NB buckets per
// level.  Rows past the live ones return at once (the scans stop at ws.live[1]).
template <class PosFn, int NL, int NM, int NB>
__global__ void __launch_bounds__(kSB) k_bwd_count_live(GridArgs a, PosFn pos, int64_t n, const float* __restrict__ dsig,
                                                        BwdWorkspace ws) {
  __shared__ uint32_t hist[NL * NB];
  const int64_t sb = blockIdx.x;
  if (sb >= (int64_t)ws.live[1]) return;  // (block-uniform)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t wi = 8u * (uint32_t)sb + (uint32_t)wid;
  const bool wok = wi < ws.live[0];
  const int64_t i = (int64_t)(wok ? ws.wlist[wi] : 0u) * 64 + lane;
  const bool in = wok && i < n;
  const int64_t ic = in ? i : n - 1;
  for (int t = threadIdx.x; t < NL * NB; t += kSB) hist[t] = 0u;
  const typename PosFn::Raw raw = pos.load(ic);  // (with d sigma: one round trip)
  const bool live = in && dsig[ic] != 0.f;
  const unsigned long long wl = __ballot(live);
  lds_barrier();
  if (wl) {  // (wave-uniform) the row's tail waves hold no live sample
    float x = 0.f, y = 0.f, z = 0.f;
    pos.eval(raw, x, y, z);
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const LevelParams& lv = a.lv[l];
      uint32_t* h = hist + l * NB;
      if (l < NM) {
        Corners c;
        level_corners<true>(lv, x, y, z, c);
        const RunInfo ri = cell_runs_dpp(in, c.cx, c.cy, c.cz);
        if (in && ri.tail && run_live(wl, ri)) {
#pragma unroll
          for (int k = 0; k < 8; ++k) atomicAdd(&h[(c.idx[k] - lv.offset) >> kChunkLog2], 1u);
        }
      } else {
        FineCell c;
        fine_cell(lv, x, y, z, c);
        count_fine_add(c, live, h);
      }
    }
  }
  lds_barrier();
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const uint32_t nb = a.bucket_base[l + 1] - a.bucket_base[l];
    uint32_t* row = hist_row(a, ws, l, sb);
    for (uint32_t b = threadIdx.x; b < nb; b += kSB) row[b] = hist[l * NB + b];
  }
}

// One workgroup per (histogram row, level): kSB samples, up to 8 records each (hashgrid.hpp).
// The row's per-bucket record counts are known before it starts (the forward's histogram, scanned
// into per-row offsets), so every record's place is known the moment its bucket rank is: staged
// rows write records in bucket order into LDS and copy whole bucket runs out, coalesced.  Rows with
// more than kCap records (coherent levels whose runs did not merge) write each record straight
// to its global slot instead.
constexpr int kCap = 4 * kSB + 256;

// Histogram row of scatter workgroup bx.  Workgroups are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md, workgroup dispatch), so row r+1 would run on the XCD after row r's.  Rows r
// and r+1 write adjacent runs in every bucket: their boundary lines are completed in one XCD's L2
// only if both rows run there.  So XCD x takes the contiguous rows [x n/8, (x+1) n/8), in order.
__device__ __forceinline__ int64_t xcd_row(uint32_t bx, uint32_t n) {
#ifndef LNR_EXP_NO_XCD_ROWS
  if ((n & 7u) == 0) return (int64_t)(bx & 7u) * (n >> 3) + (bx >> 3);
#endif
  return bx;
}  // 4 records per sample at fine levels, plus slack
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// KIND: the levels one launch covers, so each gets only its own code and registers.
// kLevelsAny: one launch over every level, grid.x = rows x levels with the level fastest, so each CU
// interleaves VALU-heavy coherent-level rows with store-heavy fine-level rows; consecutive rows of
// one level are L blocks apart, i.e. on the same XCD when L is a multiple of 8 (see xcd_row).
enum : int { kLevelsCoherent = 0, kLevelsFine = 1, kLevelsGeneric = 2, kLevelsAny = 3 };

#ifndef LNR_SCATTER_WAVES_PER_EU
#define LNR_SCATTER_WAVES_PER_EU 1
#endif
// One (histogram row sb, level l) of the scatter; KIND as below, kLevelsAny meaning "any level".
template <class PosFn, class GradFn, int KIND>
__device__ __forceinline__ void scatter_row_level(const GridArgs& a, const PosFn& pos, int64_t n, const GradFn& grad,
                                                  const BwdWorkspace& ws, uint32_t l, int64_t sb, bool skip_zero,
                                                  char* smem) {
  uint32_t* stage_v = reinterpret_cast<uint32_t*>(smem);                     // [kCap] fp16 value pairs
  uint64_t* gbase = reinterpret_cast<uint64_t*>(stage_v + kCap);             // [kMaxChunksPerLevel]
  uint32_t* stage_w = reinterpret_cast<uint32_t*>(gbase + kMaxChunksPerLevel);  // [kCap]
  uint32_t* rank_ctr = stage_w + kCap;                                       // [kMaxChunksPerLevel]
  uint32_t* start = rank_ctr + kMaxChunksPerLevel;                           // [kMaxChunksPerLevel + 1]
  uint8_t* sbk = reinterpret_cast<uint8_t*>(start + kMaxChunksPerLevel + 1);  // [kCap] bucket of each staged record
  const int kind = KIND != kLevelsAny ? KIND
                   : a.lv[l].fine           ? kLevelsFine
                   : l < a.merge_levels     ? kLevelsCoherent
                                            : kLevelsGeneric;
  const int64_t i = sb * kSB + threadIdx.x;
  const bool in = i < n;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t b0 = a.bucket_base[l];
  const uint32_t nb = a.bucket_base[l + 1] - b0;
  const LevelParams& lv = a.lv[l];
  const float rs = ldexpf(1.f, rec_exp_for(ws.level_max[l]));  // record scale
  static_assert(kMaxChunksPerLevel <= 128, "two buckets per lane of wave 0");
  LNR_STAMP(t0);
  // 1. Global loads, all unconditional (clamped indices) so nothing waits for them before it must:
  //    the sample's position inputs and d_enc, and (wave 0) the row's offsets.
  const int64_t ic = in ? i : n - 1;
  const typename PosFn::Raw raw = pos.load(ic);
  // d_enc is read once: a nontemporal load keeps it from displacing the L2 lines in which adjacent
  // rows' bucket runs combine (scatter -1.5 % at C2)
  const float2 g_raw = grad.load_nt(l, ic);
  uint32_t h0[2] = {0u, 0u}, h1[2] = {0u, 0u};
  uint64_t seg[2] = {0ull, 0ull};
  const bool last = sb + 1 >= ws.n_sb;
  {  // every wave loads (L2 hits): a branch around the loads would make its exit wait for them
    const uint32_t* row = hist_row(a, ws, l, sb);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint32_t b = min(2u * lane + q, nb - 1u);
      h0[q] = row[b];
      h1[q] = (last ? ws.counts + b0 : row + nb)[b];  // next row's offset, or the bucket total
      seg[q] = ws.seg_start[b0 + b];
    }
  }
  // wave 0 turns the offsets into the row's bucket starts and global bases (called where its loads
  // have had the most time to land)
  auto row_starts = [&]() {
    if (wid != 0) return;
    const uint32_t c0 = 2 * lane < nb ? h1[0] - h0[0] : 0u;
    const uint32_t c1 = 2 * lane + 1 < nb ? h1[1] - h0[1] : 0u;
    uint32_t inc = c0 + c1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t q = __shfl_up(inc, o, 64);
      if (lane >= o) inc += q;
    }
    const uint32_t ex = inc - c0 - c1;
    if (2 * lane < nb) {
      start[2 * lane] = ex;
      gbase[2 * lane] = seg[0] + h0[0];
    }
    if (2 * lane + 1 < nb) {
      start[2 * lane + 1] = ex + c0;
      gbase[2 * lane + 1] = seg[1] + h0[1];
    }
    if (lane == 63) start[nb] = inc;
  };
  if (threadIdx.x < kMaxChunksPerLevel) rank_ctr[threadIdx.x] = 0;
  if (kind == kLevelsCoherent) row_starts();  // coherent rows place as they rank
  lds_barrier();
  LNR_STAMP(t1);
  float x = 0.f, y = 0.f, z = 0.f;
  pos.eval(raw, x, y, z);
  const float2 g = in ? g_raw : make_float2(0.f, 0.f);
  // fine / generic levels: samples with a zero gradient emit nothing when the histogram was
  // counted after the MLP backward (k_bwd_count, same predicate); coherent levels keep every lane
  const bool act = in && grad.live_at(ic) && (!skip_zero || g.x != 0.f || g.y != 0.f);
  bool staged = true;
  auto place = [&](bool valid, uint32_t bk, uint32_t rank, uint32_t word, float2 val) {
    if (!valid) return;
    const uint32_t h = rec_half2(val.x, val.y, rs);
    if (staged) {
      const uint32_t t = start[bk] + rank;
      stage_w[t] = word;
      stage_v[t] = h;
      sbk[t] = (uint8_t)bk;
    } else {
      ws.rec[gbase[bk] + rank] = make_uint2(word, h);
    }
  };
  // 2. records: rank, then place (hashgrid.hpp "Backward records")
  if (kind == kLevelsFine) {
    // ranks first (LDS counters only), placement after wave 0 has published the starts
    FineCell c;
    fine_cell(lv, x, y, z, c);
    const bool split = c.d >= (uint32_t)kChunk;
    const uint32_t code = ((uint32_t)__popc(c.d) << kChunkLog2) | (tx_unorm16(c.tx) << 16);
    uint32_t rank[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) rank[j] = act ? atomicAdd(&rank_ctr[c.e[j] >> kChunkLog2], 1u) : 0u;
    row_starts();
    LNR_STAMP(t1b);
    lds_barrier();
    LNR_PHASE_BY(sb, 5 * kind + 4, t1b, t1);
    staged = start[nb] <= (uint32_t)kCap;  // block-uniform
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t e0 = c.e[j];
      const float wyz = ((j & 1) ? c.ty : 1.0f - c.ty) * ((j & 2) ? c.tz : 1.0f - c.tz);
      const float w0 = split ? fine_weight(c, j, 0) : wyz;
      place(act, e0 >> kChunkLog2, rank[j], (e0 & (kChunk - 1)) | (split ? 0u : code), make_float2(w0 * g.x, w0 * g.y));
    }
    if (__ballot(act && split)) {  // pairs spanning two chunks: the second corners on their own
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t e1 = c.e[j] ^ c.d;
        const float w1 = fine_weight(c, j, 1);
        const bool v = act && split;
        const uint32_t r = v ? atomicAdd(&rank_ctr[e1 >> kChunkLog2], 1u) : 0u;
        place(v, e1 >> kChunkLog2, r, e1 & (kChunk - 1), make_float2(w1 * g.x, w1 * g.y));
      }
    }
  } else {
    Corners c;
    level_corners(lv, x, y, z, c);
    const uint32_t off = lv.offset;
    if (kind == kLevelsCoherent) {  // corner k summed over the run of lanes that share it
      staged = start[nb] <= (uint32_t)kCap;
      RunInfo ri;
      float v[16];
      coherent_run_values(c, in, g.x, g.y, ri, v);
      const bool valid = in && ri.tail;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t e = valid ? c.idx[k] - off : 0u;
        const uint32_t bk = e >> kChunkLog2;
        const uint32_t rank = valid ? atomicAdd(&rank_ctr[bk], 1u) : 0u;  // run tails only: few lanes
        place(valid, bk, rank, e & (kChunk - 1), make_float2(v[2 * k], v[2 * k + 1]));
      }
    } else {  // generic non-coherent levels (configurations without power-of-two hashed tables)
      row_starts();
      lds_barrier();
      staged = start[nb] <= (uint32_t)kCap;
      const uint32_t txq = tx_unorm16(c.tx);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t e0 = c.idx[2 * j] - off, e1 = c.idx[2 * j + 1] - off;
        const bool pair = pairable(e0, e1);
        const float wyz = ((j & 1) ? c.ty : 1.0f - c.ty) * ((j & 2) ? c.tz : 1.0f - c.tz);
        const float w0 = pair ? wyz : c.w[2 * j];
        const uint32_t r0 = act ? atomicAdd(&rank_ctr[e0 >> kChunkLog2], 1u) : 0u;
        place(act, e0 >> kChunkLog2, r0, pair ? pair_word(e0, e1, txq) : (e0 & (kChunk - 1)),
              make_float2(w0 * g.x, w0 * g.y));
        const bool v1 = act && !pair;
        const uint32_t r1 = v1 ? atomicAdd(&rank_ctr[e1 >> kChunkLog2], 1u) : 0u;
        place(v1, e1 >> kChunkLog2, r1, e1 & (kChunk - 1), make_float2(c.w[2 * j + 1] * g.x, c.w[2 * j + 1] * g.y));
      }
    }
  }
  LNR_STAMP(t2);
  lds_barrier();
  LNR_STAMP(t3);
  // 3. copy the staged row out in bucket order (consecutive lanes -> consecutive slots of a run)
  if (staged) {
    const uint32_t total = start[nb];
    for (uint32_t t = threadIdx.x; t < total; t += kSB) {
      const uint32_t bk = sbk[t];
      const uint64_t dst = gbase[bk] + (t - start[bk]);
      ws.rec[dst] = make_uint2(stage_w[t], stage_v[t]);
    }
  }
  LNR_STAMP(t4);
  LNR_PHASE_BY(sb, 5 * kind + 0, t1, t0);
  LNR_PHASE_BY(sb, 5 * kind + 1, t2, t1);
  LNR_PHASE_BY(sb, 5 * kind + 2, t3, t2);
  LNR_PHASE_BY(sb, 5 * kind + 3, t4, t3);
}

template <class PosFn, class GradFn, int KIND>
__global__ void __launch_bounds__(kSB, LNR_SCATTER_WAVES_PER_EU) k_bwd_scatter(GridArgs a, PosFn pos, int64_t n,
                                                                             GradFn grad, BwdWorkspace ws, uint32_t l0,
                                                                             bool skip_zero) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t l = KIND == kLevelsAny ? blockIdx.x % a.n_levels : l0 + blockIdx.y;
  const int64_t sb = KIND == kLevelsAny ? (int64_t)(blockIdx.x / a.n_levels) : xcd_row(blockIdx.x, gridDim.x);
  scatter_row_level<PosFn, GradFn, KIND>(a, pos, n, grad, ws, l, sb, skip_zero, smem);
}

// Level-looped scatter: one workgroup per histogram row walks every level, so a sample's position is
// loaded and decoded once (not once per level), the next level's d_enc and histogram row are in
// flight while this level ranks and places, and the copy-out of level l - 1 overlaps the ranking of
// level l (double-buffered staging, one barrier per level).  A level's bucket starts come from the
// forward's histogram alone, so wave 0 computes them one level ahead and every record is placed the
// moment its rank returns.  Same records, counts and blockmax as k_bwd_scatter.
// ---------------------------------------------------------------------------------------------
// Level-looped scatter: one workgroup per histogram row walks every level.
//  * All global loads happen in the prologue: the sample's position, its encoding gradient at every
//    level (GradJac: 16 registers of fp16 pairs) and, wave w, the histogram rows of levels 2w and
//    2w + 1, turned at once into every level's bucket starts.  The level loop then issues only LDS
//    operations and the copy-out stores, so nothing in it ever waits on global memory.
//  * Each record is ranked (returning LDS atomic) and placed at once, 16 B {word, global slot, v0,
//    v1} in bucket order; then the level's stage is copied out (kRowsStages).
//  * A (row, level) with more than kRowsCap records (coherent rows whose runs did not merge) writes
//    every record straight to its global slot instead (same slots, unstaged).
// Same records, counts and blockmax as k_bwd_scatter.
constexpr int kRowsCap = 2176;  // 4.25 records per sample: fine rows hold 4 + the rare split pairs
// Stages: 1, one stage with the copy-out after each level's placement: 44 KB of LDS and 80 VGPRs
// (GradJac: the Jacobian held as fp16 pairs), so 3 workgroups (6 waves per SIMD) share a CU; 2, a
// double-buffered stage with the copy-out of level l - 1 overlapping level l, 79 KB, 2 workgroups
// per CU (C2: 670 against 627 us).  GradF32's float2 gradients need 16 more registers: they keep
// the double-buffered stage at 4 waves per SIMD (one stage would spill), except with 128 chunks
// per level (the colour grid), whose tables leave room for one stage only.
#ifndef LNR_SCATTER_STAGES
#define LNR_SCATTER_STAGES 0  // 0: per gradient source as above; 1 or 2: forced (experiments)
#endif
template <class GradFn, int NB>
constexpr int rows_stages() {
  return LNR_SCATTER_STAGES ? LNR_SCATTER_STAGES : (sizeof(typename GradFn::Raw) <= 4 || NB > 64 ? 1 : 2);
}
#ifndef LNR_ROWS_WIDE_WAVES
// One stage with float2 gradients (GradF32: the colour grid's backward): 6 waves cap it at 80 VGPRs
// and it spilled 12; at 5 it does not (CAM backward stage 0.455-0.459 -> 0.449-0.454 ms, bitwise).
#define LNR_ROWS_WIDE_WAVES 5
#endif
template <class GradFn, int NB>
constexpr int rows_waves() {
  return rows_stages<GradFn, NB>() == 2 ? 4 : (sizeof(typename GradFn::Raw) > 4 ? LNR_ROWS_WIDE_WAVES : 6);
}
#ifndef LNR_PRESCALE
#define LNR_PRESCALE 1
#endif
#ifndef LNR_ROWS_NB128
#define LNR_ROWS_NB128 1  // the level-looped scatter for grids with up to 128 chunks per level too
#endif
#ifndef LNR_ROWS_SOA
#define LNR_ROWS_SOA 1
#endif
template <int NL, int NB, int STG>
struct RowsLds {  // the small tables first: their addresses fit the 16-bit LDS instruction offset
  uint2 sg[NL][NB];           // per level and bucket: {start in the stage, global slot of the run}
  uint32_t total[NL];         // records of the row at each level
  uint32_t ctr[2][NB];        // rank counters
  LevelParams lv[NL];         // the level table (kernel arguments indexed per level would be loads)
#if LNR_ROWS_SOA
  // staged records in bucket order, one array per field: a record's three stores go to bank slot mod 32 each
  // (with 16-byte records a store's 32 lanes, at random slots, met only 8 banks: 4 slot mod 8 + field)
  uint32_t st_word[STG][kRowsCap], st_slot[STG][kRowsCap], st_val[STG][kRowsCap];
#else
  uint4 stage[STG][kRowsCap];  // staged records {word, global slot, fp16 value pair, -}, bucket order
#endif
};

// NL levels, the first NM coherent (run-merging) and the rest fine, at most NB buckets per level:
// compile-time, so the level loop unrolls into straight-line code.  Record slots are 32-bit (the
// launcher checks 8 N L < 2^32).
// The body walks levels [LB, LB + NL) of histogram row sb (local level l is level LB + l).
// LIVE (GradJac only): the live backward (k_bwd_count_live above): records only for samples with dL/dsigma != 0
// (coherent levels: runs holding one), and a wave without a live lane skips its loads and corner work.
template <class PosFn, class GradFn, int LB, int NL, int NM, int NB, int kRowsStages, bool LIVE = false>
__device__ __forceinline__ void scatter_rows_body(RowsLds<NL, NB, kRowsStages>& sm, const GridArgs& a, const PosFn& pos,
                                                  int64_t n, const GradFn& grad, const BwdWorkspace& ws, bool skip_zero,
                                                  int64_t sb) {
  static_assert(NL <= 2 * (kSB / 64), "wave w prepares levels 2w and 2w + 1");
  static_assert(NB <= 128, "two buckets per lane");
  static_assert(kRowsStages == 1 || kRowsStages == 2, "one or two stages");
  static_assert(NM <= NL, "coherent levels come first");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // LIVE: row sb = the live waves 8 sb .. 8 sb + 7 (ws.wlist), each wave its own 64-sample group: the coherent
  // levels' runs and sums see the lanes the full backward's wave sees
  const uint32_t wi = 8u * (uint32_t)sb + (uint32_t)wid;
  const bool wok = !LIVE || wi < ws.live[0];
  const int64_t i = LIVE ? (int64_t)(wok ? ws.wlist[wi] : 0u) * 64 + lane : sb * kSB + threadIdx.x;
  const bool in = wok && i < n;
  const bool last = sb + 1 >= (LIVE ? (int64_t)ws.live[1] : ws.n_sb);
  const int64_t ic = in ? i : n - 1;
  const uint32_t spare = (uint32_t)(8 * n * (int64_t)a.n_levels);  // one of the 2 slack records past the last slot

  // prologue 1: the level table and zero rank counters
  if (threadIdx.x < NL * (sizeof(LevelParams) / 4))
    reinterpret_cast<uint32_t*>(sm.lv)[threadIdx.x] = reinterpret_cast<const uint32_t*>(a.lv + LB)[threadIdx.x];
  if (threadIdx.x < 2 * NB) (&sm.ctr[0][0])[threadIdx.x] = 0u;
  // prologue 2: every global load of the kernel
  const typename PosFn::Raw raw = pos.load(ic);
  static_assert(!LIVE || GradFn::kScaled, "the live backward takes its criterion from dL/dsigma");
  const float gsc = grad.scale(ic);
  const bool live = grad.live_at(ic);  // (GradF32's live mask, when the forward counted with it)
  // LIVE: this lane's sample has dL/dsigma != 0, and the wave's live lanes (wave-uniform)
  const bool lv_live = in && (!GradFn::kScaled || gsc != 0.f);
  const unsigned long long wl = LIVE ? __ballot(lv_live) : ~0ull;
  typename GradFn::Raw g[NL];  // (GradJac: the fp16 pair, scaled by d sigma at use: half the registers)
  if (!LIVE || wl) {
#pragma unroll
    for (int l = 0; l < NL; ++l) g[l] = grad.load_raw_nt(LB + l, ic);  // read once: nontemporal, so they do not
                                                                  // displace the runs' L2 lines
  } else {
#pragma unroll
    for (int l = 0; l < NL; ++l) g[l] = typename GradFn::Raw{};
  }
  uint32_t h0[2][2], h1[2][2];
  uint64_t seg[2][2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const uint32_t l = 2 * wid + p;
    if (l < (uint32_t)NL) {
      const uint32_t b0 = a.bucket_base[LB + l], nb = a.bucket_base[LB + l + 1] - b0;
      const uint32_t* row = ws.hist + (int64_t)b0 * ws.n_sb + sb * nb;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint32_t b = min(2u * lane + q, nb - 1u);
        h0[p][q] = row[b];
        h1[p][q] = (last ? ws.counts + b0 : row + nb)[b];  // next row's offset, or the bucket total
        seg[p][q] = ws.seg_start[b0 + b];
      }
    }
  }
  float rsc[NL];  // per-level record scales (uniform: scalar loads)
#pragma unroll
  for (int l = 0; l < NL; ++l) rsc[l] = ldexpf(1.f, rec_exp_for(ws.level_max[LB + l]));
  float x = 0.f, y = 0.f, z = 0.f;
  pos.eval(raw, x, y, z);
  // prologue 3: wave w's levels' bucket starts (a wave prefix over the buckets, two per lane)
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const uint32_t l = 2 * wid + p;
    if (l < (uint32_t)NL) {
      const uint32_t nb = a.bucket_base[LB + l + 1] - a.bucket_base[LB + l];
      const uint32_t c0 = 2 * lane < nb ? h1[p][0] - h0[p][0] : 0u;
      const uint32_t c1 = 2 * lane + 1 < nb ? h1[p][1] - h0[p][1] : 0u;
      const uint32_t inc = wave_incl_scan_u32(c0 + c1);
      const uint32_t ex = inc - c0 - c1;
      if (2 * lane < nb) sm.sg[l][2 * lane] = make_uint2(ex, (uint32_t)(seg[p][0] + h0[p][0]));
      if (2 * lane + 1 < nb) sm.sg[l][2 * lane + 1] = make_uint2(ex + c0, (uint32_t)(seg[p][1] + h0[p][1]));
      if (lane == 63) sm.total[l] = inc;
    }
  }
  lds_barrier();

  // staged record t of stage b as {word, global slot, fp16 pair, -}
  auto staged_rec = [&](int b, uint32_t t) {
#if LNR_ROWS_SOA
    return make_uint4(sm.st_word[b][t], sm.st_slot[b][t], sm.st_val[b][t], 0u);
#else
    return sm.stage[b][t];
#endif
  };
  // copy level l's staged row out (consecutive threads -> consecutive slots of a run)
  auto copy_out = [&](uint32_t l) {
    const int sbuf = kRowsStages == 2 ? (l & 1) : 0;
    const uint32_t total = sm.total[l];
    const uint32_t lim = total <= (uint32_t)kRowsCap ? total : 0u;
#if LNR_COPY_ALL_TRIPS
#pragma unroll
    for (int u = 0; u < (kRowsCap + kSB - 1) / kSB; ++u) {
      const uint32_t t = threadIdx.x + u * kSB;
      const uint4 q = staged_rec(sbuf, t < (uint32_t)kRowsCap ? t : kRowsCap - 1);
      const uint32_t d = t < lim && q.y < spare ? q.y : spare;  // (the bound: never a store outside the records)
      ws.rec[d] = make_uint2(q.x, q.z);
    }
#else
    // only the trips the row's records need (block-uniform: a merged coherent row holds far fewer
    // than kRowsCap), and only the lanes holding a record store
#pragma unroll
    for (int u = 0; u < (kRowsCap + kSB - 1) / kSB; ++u) {
      if ((uint32_t)(u * kSB) < lim) {
        const uint32_t t = threadIdx.x + u * kSB;
        if (t < lim) {
          const uint4 q = staged_rec(sbuf, t);
          const uint32_t d = q.y < spare ? q.y : spare;  // (the bound: never a store outside the records)
          ws.rec[d] = make_uint2(q.x, q.z);
        }
      }
    }
#endif
  };

#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const int sbuf = l & 1;  // rank counters (and, with two stages, the stage)
    const int stg = kRowsStages == 2 ? sbuf : 0;
    const LevelParams lv = sm.lv[l];
    const bool staged = sm.total[l] <= (uint32_t)kRowsCap;  // block-uniform
    uint32_t* ctr = sm.ctr[sbuf];
    const uint2* sgl = sm.sg[l];
    const float2 gl = GradFn::finish(g[l], gsc);
#if LNR_PRESCALE
    // the level's record scale applied to the gradient once, not to every record value: a power of
    // two, so w (g 2^k) rounds exactly as (w g) 2^k
    const float2 gv = in ? make_float2(gl.x * rsc[l], gl.y * rsc[l]) : make_float2(0.f, 0.f);
#else
    const float2 gv = in ? gl : make_float2(0.f, 0.f);
#endif
    const bool act = LIVE ? lv_live : in && live && (!skip_zero || gv.x != 0.f || gv.y != 0.f);
    const float rs = LNR_PRESCALE ? 1.0f : rsc[l];
    // rank (returning LDS atomics) and place: all start reads, then all atomics, then all writes
    // (one lane-level branch for the 4 records: they share their validity)
    auto place = [&](bool valid, const uint32_t (&bk)[4], const uint32_t (&word)[4], const float2 (&val)[4]) {
      if (valid) {
        uint2 s4[4];
        uint32_t rank[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) s4[k] = sgl[bk[k]];
#pragma unroll
        for (int k = 0; k < 4; ++k) rank[k] = atomicAdd(&ctr[bk[k]], 1u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t slot = s4[k].y + rank[k];
          const uint32_t h = rec_half2(val[k].x, val[k].y, rs);
          if (staged) {
#if LNR_ROWS_SOA
            const uint32_t t = s4[k].x + rank[k];
            sm.st_word[stg][t] = word[k];
            sm.st_slot[stg][t] = slot;
            sm.st_val[stg][t] = h;
#else
            // three 32-bit fields (ds_write2_b32 + ds_write_b32: no register moves for a b128 quad)
            uint32_t* q = reinterpret_cast<uint32_t*>(&sm.stage[stg][s4[k].x + rank[k]]);
            q[0] = word[k];
            q[1] = slot;
            q[2] = h;
#endif
          } else {  // (block-uniform) more records than the stage holds: each straight to its global slot
            ws.rec[slot < spare ? slot : spare] = make_uint2(word[k], h);
          }
        }
      }
    };
    uint32_t bk4[4], w4[4];
    float2 val4[4];
    if (LIVE && !wl) {
      // (wave-uniform) LIVE: no live lane, nothing to place
    } else if (l >= NM) {  // fine: one record per x-pair (hashgrid.hpp "Backward records")
      FineCell c;
      fine_cell(lv, x, y, z, c);
      const bool split = c.d >= (uint32_t)kChunk;
      const uint32_t code = ((uint32_t)__popc(c.d) << kChunkLog2) | (tx_unorm16(c.tx) << 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t e0 = c.e[j];
        const float wyz = ((j & 1) ? c.ty : 1.0f - c.ty) * ((j & 2) ? c.tz : 1.0f - c.tz);
        const float w0 = split ? fine_weight(c, j, 0) : wyz;
        bk4[j] = e0 >> kChunkLog2;
        w4[j] = (e0 & (kChunk - 1)) | (split ? 0u : code);
        val4[j] = make_float2(w0 * gv.x, w0 * gv.y);
      }
      place(act, bk4, w4, val4);
      if (__ballot(act && split)) {  // pairs spanning two chunks: the second corners on their own
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t e1 = c.e[j] ^ c.d;
          const float w1 = fine_weight(c, j, 1);
          bk4[j] = e1 >> kChunkLog2;
          w4[j] = e1 & (kChunk - 1);
          val4[j] = make_float2(w1 * gv.x, w1 * gv.y);
        }
        place(act && split, bk4, w4, val4);
      }
    } else {  // coherent: corner k summed over the run of lanes that share it, 4 corners at a time
      Corners c;
      level_corners<true>(lv, x, y, z, c);
      const uint32_t off = lv.offset;
      RunInfo ri;
      float v[16];
      coherent_run_values(c, in, gv.x, gv.y, ri, v);
      const bool valid = in && ri.tail && (!LIVE || run_live(wl, ri));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int k = 4 * h + kk;
          const uint32_t e = c.idx[k] - off;
          bk4[kk] = e >> kChunkLog2;
          w4[kk] = e & (kChunk - 1);
          val4[kk] = make_float2(v[2 * k], v[2 * k + 1]);
        }
        place(valid, bk4, w4, val4);
      }
    }
    if (threadIdx.x < NB) sm.ctr[sbuf ^ 1][threadIdx.x] = 0u;  // level l + 1's counters (last used by l - 1)
    if (kRowsStages == 2) {
      if (l >= 1) copy_out(l - 1);
      lds_barrier();
    } else {
      lds_barrier();  // level l placed
      copy_out(l);
      if (l + 1 < NL) lds_barrier();  // the stage is free for level l + 1
    }
  }
  if (kRowsStages == 2) copy_out(NL - 1);
}

template <class PosFn, class GradFn, int NL, int NM, int NB, bool LIVE = false>
__global__ void __launch_bounds__(kSB)
__attribute__((amdgpu_waves_per_eu(rows_waves<GradFn, NB>(), rows_waves<GradFn, NB>())))
k_bwd_scatter_rows(GridArgs a, PosFn pos, int64_t n, GradFn grad, BwdWorkspace ws, bool skip_zero) {
  __shared__ RowsLds<NL, NB, rows_stages<GradFn, NB>()> sm;
  int64_t sb = xcd_row(blockIdx.x, gridDim.x);
  if (LIVE) {  // the live rows only, XCD x taking the contiguous rows [x r/8, (x+1) r/8) of them (see xcd_row)
    const uint32_t r = ws.live[1], r8 = (r + 7u) & ~7u;
    if (blockIdx.x >= r8) return;
    sb = (int64_t)(blockIdx.x & 7u) * (r8 >> 3) + (blockIdx.x >> 3);
    if (sb >= (int64_t)r) return;
  }
  scatter_rows_body<PosFn, GradFn, 0, NL, NM, NB, rows_stages<GradFn, NB>(), LIVE>(sm, a, pos, n, grad, ws, skip_zero, sb);
}

constexpr size_t kScatterLds = (size_t)kCap * 4 + kMaxChunksPerLevel * 8 + (size_t)kCap * 4 + kMaxChunksPerLevel * 4 +
                               (kMaxChunksPerLevel + 1) * 4 + kCap;
static_assert(kScatterLds <= 65536, "scatter LDS within the default dynamic limit");

// Max |d_enc| per level (the record scales): grid (kMaxBlocks, L), grid-stride float2 loads, one
// atomicMax per workgroup on the float's bits (non-negative floats order as their bit patterns).
// ws.level_max is zeroed before.
constexpr int kMaxBlocks = 256;
template <class GradFn>
__global__ void __launch_bounds__(256) k_denc_level_max(GradFn grad, int64_t n, BwdWorkspace ws) {
  __shared__ float red[4];
  const uint32_t l = blockIdx.y;
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)kMaxBlocks * 256) {
    const float2 g = grad.load(l, i);
    m = fmaxf(m, fmaxf(fabsf(g.x), fabsf(g.y)));
  }
  m = wave_max_nonneg(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  lds_barrier();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (m > 0.f) atomicMax(reinterpret_cast<uint32_t*>(ws.level_max) + l, __float_as_uint(m));
  }
}

#ifndef LNR_ACCUM_THREADS
#define LNR_ACCUM_THREADS 1024
#endif
constexpr int kAccumThreads = LNR_ACCUM_THREADS;

// Fixed-point exponent of bucket b, in the records' scaled units: ws.k2 = bwd_fixed_k2(N) for every bucket
// (hashgrid.hpp: every partial or total sum stays below 2^62 from the records' magnitudes alone, and each converted
// value below 2^51, the exact range of the double conversion below).  The unit is 2^-30 of the scaled units at C2,
// 2^-39 of the level's largest record.  (Precision here matters beyond the gradients' own: Adam's eps = 1e-8 turns
// a one-unit difference of a near-zero gradient entry into a visible step, so two runs must round alike far below
// the gradients' scale; they do, as the unit depends on N alone, not on which records a backward places.)
// (Rounds 1-5 took 47 - lg(count) per bucket, which needed every sample's count, i.e. the forward's record
// histogram, for the live backward to round like the full one; history before this commit.)
__device__ __forceinline__ int bucket_k2(const BwdWorkspace& ws, uint32_t) { return ws.k2; }
// 2^-(k2 + k_l): fixed-point units back to gradient units (double: the exponent may pass fp32's range)
__device__ __forceinline__ double unit_back(const GridArgs& a, const BwdWorkspace& ws, uint32_t l, int k2) {
  return ldexp(1.0, -(k2 + rec_exp_for(ws.level_max[l])));
}
// round(x) as int64 for |x| < 2^51: x + 1.5 2^52 in double places the rounded integer in the low
// mantissa bits, and the constant's low word is 0, so only the high word needs the subtraction.
__device__ __forceinline__ unsigned long long fixed_i64(float x) {
  const double d = (double)x + 6755399441055744.0;
  const unsigned long long bits = (unsigned long long)__double_as_longlong(d);
  return bits - 0x4338000000000000ull;
}

#ifndef LNR_SCATTER_ROWS_MIN
#define LNR_SCATTER_ROWS_MIN 256
#endif
#ifndef LNR_ACCUM_BUCKETS_MAX_N
#define LNR_ACCUM_BUCKETS_MAX_N (1 << 17)  // C1 (32 K samples): 103 -> 76 us for the backward stage; the C4 shard of 8 GPUs (590 K): 219 -> 229 us
#endif
#ifndef LNR_ACCUM_WAVES_PER_EU
#define LNR_ACCUM_WAVES_PER_EU 8
#endif
#ifndef LNR_ACCUM_TRIP
#define LNR_ACCUM_TRIP 2
#endif
constexpr int kAccumTrip = LNR_ACCUM_TRIP;        // tiles per trip of the accumulate loop (loads ahead)
constexpr int kTile = 2 * kAccumThreads;         // records per tile: 2 per thread
static_assert(kTile == 2048, "the stage's swizzle and the strided reads assume 64-lane waves x 16 x 2");
// the stage position of tile record q: bits 1-4 XOR bits 5-8 (record pairs stay adjacent: the stores
// are 16 B), so a wave's reads of records 32 apart spread over the banks
__device__ __forceinline__ uint32_t stage_pos(uint32_t q) { return q ^ (((q >> 5) & 15u) << 1); }
// Workgroup i's record range [range_at(i), range_at(i + 1)) of the R records from r0: an even split.
__device__ __forceinline__ uint64_t range_at(uint64_t r0, uint64_t R, uint32_t i) {
  return r0 + (R * i) / kAccumGroups;
}
// The workgroup whose range holds record p (r0 <= p < r0 + R): the last i with range_at(i) <= p.
__device__ __forceinline__ uint32_t group_of(uint64_t r0, uint64_t R, uint64_t p) {
  uint32_t i = (uint32_t)(((p - r0) * kAccumGroups) / R);
  while (i + 1 < (uint32_t)kAccumGroups && range_at(r0, R, i + 1) <= p) ++i;
  while (i > 0 && range_at(r0, R, i) > p) --i;
  return i;
}
__device__ __forceinline__ uint32_t level_of_bucket(const GridArgs& a, uint32_t b) {
  uint32_t l = 0;
  while (l + 1 < a.n_levels && a.bucket_base[l + 1] <= b) ++l;
  return l;
}


// The records [beg, end) of one bucket, added into the workgroup's LDS chunk (zeroed before).
// Tiles of kTile records pass through LDS: each thread loads 2 consecutive records (one 16-B load,
// coalesced) and stores them to the tile stage; then lane L of wave w takes records 32 L + 2 w and
// + 1 of the tile, so one atomic instruction holds records 32 apart.  Adjacent records of a bucket
// are one ray's consecutive samples (equal or neighbouring corners), and equal addresses
// serialise within one LDS instruction; this way they meet in one only by a hash collision.
// The stage is XOR-swizzled (stage_pos) so those strided reads spread over the banks.
// Loads run kAccumTrip tiles ahead (registers).
// A pair record (p > 0) adds (1 - tx) v to corner e0 and tx v to e1 = e0 ^ (2^p - 1), a single
// record (p = 0, tx = 0) adds v to e0.  int64 sums: the result does not depend on the order.
// fs = 2^k2, the bucket's fixed-point scale (the records carry 2^k_l already).
// (Measured and dropped, round 5: walking the tiles from the range's end, for the Infinity Cache, and plain
// instead of nontemporal record loads, both within the noise; adding each thread's own records without the
// tile stage from some level on, +0.21 ms at C2 from same-entry conflicts.  History before commit e32a0b7.)
__device__ __forceinline__ void accum_records(unsigned long long* acc, uint2* stage, const BwdWorkspace& ws,
                                              uint64_t beg, uint64_t end, float fs) {
  const int lane = threadIdx.x & 63;
  const uint64_t beg2 = beg & ~1ull;
  const float ftx = fs * kInvU16;
  const uint64_t n_tiles = (end - beg2 + kTile - 1) / kTile;
  auto load_tile = [&](uint64_t tile) {  // this thread's 2 records of a tile: {w0, v0, w1, v1}
    const uint64_t rr = beg2 + (tile < n_tiles ? tile : 0) * kTile + 2 * threadIdx.x;
    const uint64_t rc = rr < end ? rr : beg2;  // unconditional loads; read once: nontemporal
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(&ws.rec[rc]));
  };
  const uint32_t q0 = 32u * lane + 2u * (threadIdx.x >> 6);  // this lane's records in a tile
  auto run_tile = [&](uint64_t tile, const u32x4& cur) {
    lds_barrier();  // the previous tile's stage reads are done
    *reinterpret_cast<u32x4*>(&stage[stage_pos(2 * threadIdx.x)]) = cur;
    lds_barrier();
    const uint64_t base = beg2 + tile * kTile;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const uint2 rec = stage[stage_pos(q0 + r)];
      const uint64_t rr = base + q0 + r;
      if (rr >= beg && rr < end) {
        const uint32_t w = rec.x;
        const float v0 = rec_v0(rec.y), v1 = rec_v1(rec.y);
        const uint32_t e0 = w & (kChunk - 1);
        const uint32_t p = (w >> kChunkLog2) & 15u;
        const float tx = (float)(w >> 16) * ftx;  // 0 for single-corner records; pre-scaled
        const float s0 = fs - tx;
        atomicAdd(&acc[e0], fixed_i64(s0 * v0));
        atomicAdd(&acc[kChunk + e0], fixed_i64(s0 * v1));
        if (p) {
          // Invariant: the scatter writes p <= 12 (kChunkLog2) for every record, so e1 stays inside
          // this chunk.  A corrupted record with p in 13..15 would put e1 up to 32767, which still
          // lands inside this workgroup's LDS (the second feature array or the tile stage) and
          // would corrupt sums silently; the mask is not applied in the product build because it
          // cost 10 % of the kernel (408 -> 450 us at C2).  -DLNR_BWD_CHECK traps instead.
#ifdef LNR_BWD_CHECK
          if (p > kChunkLog2) __builtin_trap();
#endif
          const uint32_t e1 = e0 ^ ((1u << p) - 1u);
          atomicAdd(&acc[e1], fixed_i64(tx * v0));
          atomicAdd(&acc[kChunk + e1], fixed_i64(tx * v1));
        }
      }
    }
  };
  // kAccumTrip tiles per trip, each in a register set of its own (the unrolled loop indexes them
  // statically), its next load issued as soon as it is staged: the loads of the following
  // kAccumTrip tiles are in flight while these accumulate
  u32x4 buf[kAccumTrip];
#pragma unroll
  for (int d = 0; d < kAccumTrip; ++d) buf[d] = load_tile(d);
  for (uint64_t tile = 0; tile < n_tiles; tile += kAccumTrip) {
#pragma unroll
    for (int d = 0; d < kAccumTrip; ++d) {
      if (tile + d < n_tiles) {  // block-uniform
        const u32x4 c = buf[d];
        buf[d] = load_tile(tile + d + kAccumTrip);
        run_tile(tile + d, c);
      }
    }
  }
}

// The final gradient g of table parameter i: stored into d_table, or (a.adam.p set) Adam's update of
// parameter i with it, the arithmetic of optim.hip's adam_range term for term (-ffp-contract=off in
// both files), so the parameters, moments and fp16 shadow are bitwise those of lnr_adam_step.
// ADAM is a template flag (the kernels are instantiated twice) so the plain kernels carry none of the
// epilogue's registers: with a runtime branch the accumulate spilled 20 VGPRs at its 64-VGPR cap.
template <bool ADAM>
__device__ __forceinline__ void put_grad(const GridArgs& a, float* __restrict__ d_table, int64_t i, float g) {
  const AdamEpi& e = a.adam;
  if (!ADAM) {
    d_table[i] = g;
    return;
  }
  const float step_size = e.dev_step ? e.dev_step->adam_step_size : e.step_size;
  const float bc2_sqrt = e.dev_step ? e.dev_step->adam_bc2_sqrt : e.bc2_sqrt;
  float m = e.m[i], v = e.v[i], p = e.p[i];
  m = m + e.one_minus_b1 * (g - m);
  v = v * e.b2 + e.one_minus_b2 * g * g;
  const float denom = sqrtf(v) / bc2_sqrt + e.eps;
  p = p + (-step_size) * (m / denom);
  e.m[i] = m;
  e.v[i] = v;
  e.p[i] = p;
  e.shadow[i] = f2h(p);
}

// Eight consecutive final gradients g[0..7] of table parameters i0 .. i0 + 7 (i0 a multiple of 8, the
// table's slice 16-B aligned), the first `cnt` of them valid: with the Adam epilogue every load of the
// eight is issued before any arithmetic (16-B loads of p, m, v, one 16-B shadow store), so a thread
// waits for memory once per eight parameters, not once per parameter.
template <bool ADAM>
__device__ __forceinline__ void put_grad8(const GridArgs& a, float* __restrict__ d_table, int64_t i0, const float (&g)[8],
                                          uint32_t cnt) {
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const AdamEpi& e = a.adam;
  if (cnt < 8) {
    for (uint32_t k = 0; k < cnt; ++k) put_grad<ADAM>(a, d_table, i0 + k, g[k]);
    return;
  }
  if (!ADAM) {
    f32x4v* d = reinterpret_cast<f32x4v*>(d_table + i0);
    d[0] = f32x4v{g[0], g[1], g[2], g[3]};
    d[1] = f32x4v{g[4], g[5], g[6], g[7]};
    return;
  }
  const float step_size = e.dev_step ? e.dev_step->adam_step_size : e.step_size;
  const float bc2_sqrt = e.dev_step ? e.dev_step->adam_bc2_sqrt : e.bc2_sqrt;
  f32x4v* pp = reinterpret_cast<f32x4v*>(e.p + i0);
  f32x4v* mp = reinterpret_cast<f32x4v*>(e.m + i0);
  f32x4v* vp = reinterpret_cast<f32x4v*>(e.v + i0);
  const f32x4v p4[2] = {pp[0], pp[1]}, m4[2] = {mp[0], mp[1]}, v4[2] = {vp[0], vp[1]};
  float po[8], mo[8], vo[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float m = m4[k >> 2][k & 3], v = v4[k >> 2][k & 3], p = p4[k >> 2][k & 3];
    m = m + e.one_minus_b1 * (g[k] - m);
    v = v * e.b2 + e.one_minus_b2 * g[k] * g[k];
    const float denom = sqrtf(v) / bc2_sqrt + e.eps;
    p = p + (-step_size) * (m / denom);
    po[k] = p;
    mo[k] = m;
    vo[k] = v;
  }
  pp[0] = f32x4v{po[0], po[1], po[2], po[3]};
  pp[1] = f32x4v{po[4], po[5], po[6], po[7]};
  mp[0] = f32x4v{mo[0], mo[1], mo[2], mo[3]};
  mp[1] = f32x4v{mo[4], mo[5], mo[6], mo[7]};
  vp[0] = f32x4v{vo[0], vo[1], vo[2], vo[3]};
  vp[1] = f32x4v{vo[4], vo[5], vo[6], vo[7]};
  uint4 h;
  h.x = (uint32_t)f2h(po[0]) | ((uint32_t)f2h(po[1]) << 16);
  h.y = (uint32_t)f2h(po[2]) | ((uint32_t)f2h(po[3]) << 16);
  h.z = (uint32_t)f2h(po[4]) | ((uint32_t)f2h(po[5]) << 16);
  h.w = (uint32_t)f2h(po[6]) | ((uint32_t)f2h(po[7]) << 16);
  *reinterpret_cast<uint4*>(e.shadow + i0) = h;
}

// A whole bucket's final fp32 values from its LDS chunk.
template <bool ADAM>
__device__ __forceinline__ void store_bucket(const unsigned long long* acc, const GridArgs& a, const BwdWorkspace& ws,
                                             float* __restrict__ d_table, uint32_t l, uint32_t ent0, uint32_t nent,
                                             int k2) {
  const double inv = unit_back(a, ws, l, k2);
  const int64_t base = 2 * ((int64_t)a.lv[l].offset + ent0);
  if (ADAM) {  // eight consecutive parameters per thread per pass (put_grad8)
    for (uint32_t t0 = 8 * threadIdx.x; t0 < 2 * nent; t0 += 8 * blockDim.x) {
      float g[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t t = t0 + k;
        g[k] = (float)((double)(long long)acc[(t & 1) * kChunk + (t >> 1)] * inv);
      }
      put_grad8<true>(a, d_table, base + t0, g, 2 * nent - t0 < 8 ? 2 * nent - t0 : 8);
    }
    return;
  }
  for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x)
    put_grad<false>(a, d_table, base + t, (float)((double)(long long)acc[(t & 1) * kChunk + (t >> 1)] * inv));
}

// One workgroup per kAccumGroups-th of the records of buckets [b_begin, b_end).  Per bucket piece:
// int64 fixed-point sums in a 64 KB LDS chunk with ds_add_u64, then the fp32 gradient (a whole
// bucket) or the piece's int64 partial chunk (a bucket the range boundaries cut; partial slot 2i for
// a piece cut at its start, 2i + 1 for one cut only at its end).
// FINISH: a cut bucket is finished inside this kernel by the last of its pieces' workgroups to get
// there (a per-bucket arrival counter, ws.bucket_done): it adds the other pieces' partial chunks into
// its own LDS sums (int64: exact, so the arrival order does not matter) and stores the fp32 values;
// the workgroup whose range holds an empty bucket's position stores its zeros.  Without FINISH,
// k_bwd_finalize does both in a second launch.
template <bool ADAM>
__device__ __forceinline__ void store_zero_bucket(const GridArgs& a, float* __restrict__ d_table, uint32_t b) {
  const uint32_t l = level_of_bucket(a, b);
  const uint32_t ent0 = (b - a.bucket_base[l]) * kChunk;
  const uint32_t nent = (a.lv[l].size - ent0) < (uint32_t)kChunk ? (a.lv[l].size - ent0) : (uint32_t)kChunk;
  const int64_t base = 2 * ((int64_t)a.lv[l].offset + ent0);
  if (ADAM) {
    const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (uint32_t t0 = 8 * threadIdx.x; t0 < 2 * nent; t0 += 8 * blockDim.x)
      put_grad8<true>(a, d_table, base + t0, z, 2 * nent - t0 < 8 ? 2 * nent - t0 : 8);
    return;
  }
  for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x) put_grad<false>(a, d_table, base + t, 0.f);
}

template <bool FINISH, bool ADAM>
__global__ void __launch_bounds__(kAccumThreads, LNR_ACCUM_WAVES_PER_EU) k_bwd_accum(GridArgs a, BwdWorkspace ws, float* __restrict__ d_table,
                                                                                        uint32_t b_begin, uint32_t b_end) {
  __shared__ unsigned long long acc[2 * kChunk];  // int64 fixed point, one array per feature (8-B atomics
                                                  // on random entries spread over twice the bank pairs)
  __shared__ __attribute__((aligned(16))) uint2 stage[kTile];  // the tile's records, swizzled
  const uint64_t r0 = ws.seg_start[b_begin], rtot = ws.seg_start[b_end], R = rtot - r0;
  const uint32_t gi = blockIdx.x;
  if (FINISH && R == 0) {  // no records at all: workgroup 0 stores every bucket's zeros
    if (gi == 0)
      for (uint32_t b = b_begin; b < b_end; ++b) store_zero_bucket<ADAM>(a, d_table, b);
    return;
  }
  const uint64_t rbeg = range_at(r0, R, gi), rend = range_at(r0, R, gi + 1);
  if (rbeg >= rend) return;
  // first bucket to visit: the one holding record rbeg, or (FINISH) the first empty one sitting at rbeg
  uint32_t lo = b_begin, hi = b_end;  // FINISH: first b with seg_start[b] >= rbeg; else last with <= rbeg
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (FINISH ? ws.seg_start[mid] < rbeg : ws.seg_start[mid + 1] <= rbeg) lo = mid + 1;
    else hi = mid;
  }
  if (FINISH && lo > b_begin && ws.seg_start[lo] > rbeg) --lo;  // rbeg strictly inside bucket lo - 1
  for (uint32_t b = lo; b < b_end; ++b) {
    const uint64_t s0 = ws.seg_start[b], s1 = ws.seg_start[b + 1];
    if (s0 >= rend && !(FINISH && s0 == rend && rend == rtot)) break;  // (the last range owns trailing empties)
    if (s0 == s1) {  // empty bucket
      if (FINISH) store_zero_bucket<ADAM>(a, d_table, b);  // owned: rbeg <= s0 < rend, or trailing
      continue;
    }
    const uint64_t beg = s0 > rbeg ? s0 : rbeg, end = s1 < rend ? s1 : rend;
    if (beg >= end) continue;
    const uint32_t l = level_of_bucket(a, b);
    const uint32_t ent0 = (b - a.bucket_base[l]) * kChunk;
    const uint32_t nent = (a.lv[l].size - ent0) < (uint32_t)kChunk ? (a.lv[l].size - ent0) : (uint32_t)kChunk;
    for (int t = threadIdx.x; t < 2 * kChunk; t += blockDim.x) acc[t] = 0ull;
    lds_barrier();
    // one scale per bucket (the pieces' partials add exactly)
    const int k2 = bucket_k2(ws, b);
    accum_records(acc, stage, ws, beg, end, ldexpf(1.f, k2));
    lds_barrier();
    if (beg == s0 && end == s1) {  // the whole bucket: the final values
      store_bucket<ADAM>(acc, a, ws, d_table, l, ent0, nent, k2);
      lds_barrier();
      continue;
    }
    // this piece's int64 partial chunk
    long long* dst = ws.partial + (int64_t)(2 * gi + (beg > s0 ? 0 : 1)) * (2 * kChunk);
    for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x) dst[t] = (long long)acc[(t & 1) * kChunk + (t >> 1)];
    if (FINISH) {
      // in-launch hand-off (cdna_hip_programming.md, split-K reduction recipe): every storing wave
      // drains its stores, the workgroup meets, ONE lane releases at agent scope and takes a ticket;
      // the last arriver's lane acquires at agent scope before its workgroup reads the other chunks
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const uint32_t g0 = group_of(r0, R, s0), g1 = group_of(r0, R, s1 - 1);
      if (threadIdx.x == 0) {
        uint32_t pieces = 0;  // groups with a non-empty range inside the bucket
        for (uint32_t g = g0; g <= g1; ++g) pieces += range_at(r0, R, g) < range_at(r0, R, g + 1) ? 1u : 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t old = __hip_atomic_fetch_add(&ws.bucket_done[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = old + 1 == pieces;
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        stage[0].x = last ? 1u : 0u;  // (the tile stage is idle here: no second LDS object, which would
                                      // push the workgroup past 80 KB and halve the residency)
      }
      __syncthreads();
      if (stage[0].x) {  // the last piece: add the others' partial chunks, store the fp32 values
        for (uint32_t g = g0; g <= g1; ++g) {
          const uint64_t gb = range_at(r0, R, g);
          if (g == gi || gb >= range_at(r0, R, g + 1)) continue;
          const long long* src = ws.partial + (int64_t)(2 * g + (gb > s0 ? 0 : 1)) * (2 * kChunk);
          for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x)
            acc[(t & 1) * kChunk + (t >> 1)] += (unsigned long long)src[t];
        }
        lds_barrier();
        store_bucket<ADAM>(acc, a, ws, d_table, l, ent0, nent, k2);
      }
    }
    lds_barrier();
  }
}

// Small batches (few records per bucket): one workgroup per whole bucket, the finest level's
// first (the dispatcher hands workgroups out in launch order as slots free, so the large fine-level
// buckets start first and the small coherent ones fill in).  No bucket is cut, so there are no
// partial chunks and no k_bwd_finalize; an empty bucket stores its zeros.  The same per-bucket
// fixed-point unit as k_bwd_accum: bitwise the same gradient.  The record-balanced k_bwd_accum
// instead pays two 64 KB partial chunks per workgroup and a finalize pass over every cut bucket,
// which dominates when a bucket holds a tile or two of records.
template <bool ADAM>
__global__ void __launch_bounds__(kAccumThreads, LNR_ACCUM_WAVES_PER_EU) k_bwd_accum_buckets(GridArgs a, BwdWorkspace ws,
                                                                                                float* __restrict__ d_table,
                                                                                                uint32_t b_begin, uint32_t b_end) {
  __shared__ unsigned long long acc[2 * kChunk];
  __shared__ __attribute__((aligned(16))) uint2 stage[kTile];
  const uint32_t b = b_end - 1 - blockIdx.x;
  const uint64_t s0 = ws.seg_start[b], s1 = ws.seg_start[b + 1];
  const uint32_t l = level_of_bucket(a, b);
  const uint32_t ent0 = (b - a.bucket_base[l]) * kChunk;
  const uint32_t nent = (a.lv[l].size - ent0) < (uint32_t)kChunk ? (a.lv[l].size - ent0) : (uint32_t)kChunk;
  if (s0 == s1) {
    store_zero_bucket<ADAM>(a, d_table, b);
    return;
  }
  for (int t = threadIdx.x; t < 2 * kChunk; t += blockDim.x) acc[t] = 0ull;
  lds_barrier();
  const int k2 = bucket_k2(ws, b);
  accum_records(acc, stage, ws, s0, s1, ldexpf(1.f, k2));
  lds_barrier();
  store_bucket<ADAM>(acc, a, ws, d_table, l, ent0, nent, k2);
}

// One workgroup per unit of the work list (UnitTable): a whole bucket (its fp32 values, or its zeros
// when empty) or one of the equal pieces of a large bucket (its int64 partial chunk, added by
// k_bwd_finalize_units).  The grid is the list's bound; workgroups past n_units return at once.
// FINISH: the last of a cut bucket's pieces to arrive adds the others' partial chunks and stores the
// bucket (the split-K hand-off of k_bwd_accum<true>; counters zeroed by k_bwd_scan_buckets), so no
// k_bwd_finalize_units launch.  The cut buckets are the coarse levels', first in the list, so their
// finishing overlaps the fine levels' units.
static_assert(kUnitMinRecords == (uint64_t)kTile, "pieces of at least one tile");
template <bool FINISH, bool ADAM>
__global__ void __launch_bounds__(kAccumThreads, LNR_ACCUM_WAVES_PER_EU) k_bwd_accum_units(GridArgs a, BwdWorkspace ws,
                                                                                              float* __restrict__ d_table) {
  __shared__ unsigned long long acc[2 * kChunk];
  __shared__ __attribute__((aligned(16))) uint2 stage[kTile];
  const UnitTable* ut = ws.units;
  if (blockIdx.x >= ut->n_units) return;
  const uint2 e = ut->unit[blockIdx.x];
  const uint32_t b = e.x, k = e.y >> 16, P = e.y & 0xFFFFu;
  const uint64_t s0 = ws.seg_start[b], s1 = ws.seg_start[b + 1];
  const uint32_t l = level_of_bucket(a, b);
  const uint32_t ent0 = (b - a.bucket_base[l]) * kChunk;
  const uint32_t nent = (a.lv[l].size - ent0) < (uint32_t)kChunk ? (a.lv[l].size - ent0) : (uint32_t)kChunk;
  if (s0 == s1) {
    store_zero_bucket<ADAM>(a, d_table, b);
    return;
  }
  const uint64_t n = s1 - s0, beg = s0 + n * k / P, end = s0 + n * (k + 1) / P;
  for (int t = threadIdx.x; t < 2 * kChunk; t += blockDim.x) acc[t] = 0ull;
  lds_barrier();
  const int k2 = bucket_k2(ws, b);
  accum_records(acc, stage, ws, beg, end, ldexpf(1.f, k2));
  lds_barrier();
  if (P == 1) {
    store_bucket<ADAM>(acc, a, ws, d_table, l, ent0, nent, k2);
    return;
  }
  const uint32_t slot0 = ut->slot[b];
  long long* dst = ws.partial + (int64_t)(slot0 + k) * (2 * kChunk);
  for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x) dst[t] = (long long)acc[(t & 1) * kChunk + (t >> 1)];
  if (!FINISH) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's partial stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(&ws.bucket_done[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old + 1 == P;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    stage[0].x = last ? 1u : 0u;  // (the tile stage is idle here)
  }
  __syncthreads();
  if (!stage[0].x) return;
  for (uint32_t q = 0; q < P; ++q) {  // the other pieces' partial chunks (int64: exact in any order)
    if (q == k) continue;
    const long long* src = ws.partial + (int64_t)(slot0 + q) * (2 * kChunk);
    for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x)
      acc[(t & 1) * kChunk + (t >> 1)] += (unsigned long long)src[t];
  }
  lds_barrier();
  store_bucket<ADAM>(acc, a, ws, d_table, l, ent0, nent, k2);
}

// Buckets the accumulation did not finish: cut buckets = the sum of their pieces' partial chunks in
// workgroup order (deterministic), empty buckets = 0.  One workgroup per bucket of [b_begin, b_end).
constexpr int kFinalizeThreads = 1024;  // 8 consecutive values per thread: 2 kChunk in one pass
template <bool ADAM>
__global__ void __launch_bounds__(kFinalizeThreads) k_bwd_finalize(GridArgs a, BwdWorkspace ws, float* __restrict__ d_table,
                                                                   uint32_t b_begin, uint32_t b_end) {
  static_assert(2 * kChunk == 8 * kFinalizeThreads, "one pass");
  typedef long long i64x2 __attribute__((ext_vector_type(2)));
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const uint32_t b = b_begin + blockIdx.x;
  const uint64_t r0 = ws.seg_start[b_begin], R = ws.seg_start[b_end] - r0;
  const uint64_t s0 = ws.seg_start[b], s1 = ws.seg_start[b + 1];
  uint32_t g0 = 1, g1 = 0;  // pieces g0..g1 (none for an empty bucket)
  if (s1 > s0) {
    g0 = group_of(r0, R, s0);
    g1 = group_of(r0, R, s1 - 1);
    if (g0 == g1) return;  // one workgroup held the whole bucket
  }
  const uint32_t l = level_of_bucket(a, b);
  const uint32_t ent0 = (b - a.bucket_base[l]) * kChunk;
  const uint32_t nent = (a.lv[l].size - ent0) < (uint32_t)kChunk ? (a.lv[l].size - ent0) : (uint32_t)kChunk;
  const double inv = unit_back(a, ws, l, bucket_k2(ws, b));  // the accumulate kernel's per-bucket unit
  const uint32_t t0 = 8 * threadIdx.x;
  if (t0 >= 2 * nent) return;
  long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t g = g0; g <= g1; ++g) {  // pieces in workgroup order: deterministic (and exact anyway)
    const uint64_t gb = range_at(r0, R, g);
    if (gb >= range_at(r0, R, g + 1)) continue;  // an empty range holds no piece
    const i64x2* src = reinterpret_cast<const i64x2*>(ws.partial + (int64_t)(2 * g + (gb > s0 ? 0 : 1)) * (2 * kChunk) + t0);
    i64x2 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = src[k];  // 4 loads in flight
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] += q[k].x;
      v[2 * k + 1] += q[k].y;
    }
  }
  float o[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = (float)((double)v[k] * inv);
  const int64_t base = 2 * ((int64_t)a.lv[l].offset + ent0) + t0;
  if (ADAM) {
    put_grad8<true>(a, d_table, base, o, 2 * nent - t0 < 8 ? 2 * nent - t0 : 8);
    return;
  }
  float* dst = d_table + base;
  if (t0 + 8 <= 2 * nent && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0)) {
    reinterpret_cast<f32x4v*>(dst)[0] = f32x4v{o[0], o[1], o[2], o[3]};
    reinterpret_cast<f32x4v*>(dst)[1] = f32x4v{o[4], o[5], o[6], o[7]};
  } else {
    for (int k = 0; k < 8; ++k)
      if (t0 + k < 2 * nent) dst[k] = o[k];
  }
}

// The cut buckets of the unit accumulation: the sum of their pieces' partial chunks in piece order.
// One workgroup per cut bucket (the grid is the bound kAccumGroups; the rest return at once).
template <bool ADAM>
__global__ void __launch_bounds__(kFinalizeThreads) k_bwd_finalize_units(GridArgs a, BwdWorkspace ws,
                                                                         float* __restrict__ d_table) {
  typedef long long i64x2 __attribute__((ext_vector_type(2)));
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const UnitTable* ut = ws.units;
  if (blockIdx.x >= ut->n_cut) return;
  const uint2 cb = ut->cut[blockIdx.x];
  const uint32_t b = cb.x, P = cb.y, slot0 = ut->slot[b];
  const uint32_t l = level_of_bucket(a, b);
  const uint32_t ent0 = (b - a.bucket_base[l]) * kChunk;
  const uint32_t nent = (a.lv[l].size - ent0) < (uint32_t)kChunk ? (a.lv[l].size - ent0) : (uint32_t)kChunk;
  const double inv = unit_back(a, ws, l, bucket_k2(ws, b));
  const uint32_t t0 = 8 * threadIdx.x;
  if (t0 >= 2 * nent) return;
  long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t k = 0; k < P; ++k) {
    const i64x2* src = reinterpret_cast<const i64x2*>(ws.partial + (int64_t)(slot0 + k) * (2 * kChunk) + t0);
    i64x2 q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = src[j];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] += q[j].x;
      v[2 * j + 1] += q[j].y;
    }
  }
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (float)((double)v[j] * inv);
  const int64_t base = 2 * ((int64_t)a.lv[l].offset + ent0) + t0;
  if (ADAM) {
    put_grad8<true>(a, d_table, base, o, 2 * nent - t0 < 8 ? 2 * nent - t0 : 8);
    return;
  }
  float* dst = d_table + base;
  if (t0 + 8 <= 2 * nent && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0)) {
    reinterpret_cast<f32x4v*>(dst)[0] = f32x4v{o[0], o[1], o[2], o[3]};
    reinterpret_cast<f32x4v*>(dst)[1] = f32x4v{o[4], o[5], o[6], o[7]};
  } else {
    for (int j = 0; j < 8; ++j)
      if (t0 + j < 2 * nent) dst[j] = o[j];
  }
}

// Samples up to which the accumulation takes whole buckets (k_bwd_accum_buckets) instead of the
// record-balanced split; LONER_ACCUM_BUCKETS_MAX_N overrides it (measurements: DESIGN.md section 4).
// (read at every launch, so a process can switch between the two: tests/test_gpu_fullsize.py)
static int64_t accum_buckets_max_n() {
  const char* e = getenv("LONER_ACCUM_BUCKETS_MAX_N");
  return e ? (int64_t)atoll(e) : (int64_t)LNR_ACCUM_BUCKETS_MAX_N;
}

// Rows (512-sample histogram rows) from which the scatter takes the level-looped kernel;
// LONER_SCATTER_ROWS_MIN overrides it (read at every launch).
static int64_t scatter_rows_min() {
  const char* e = getenv("LONER_SCATTER_ROWS_MIN");
  return e ? (int64_t)atoll(e) : (int64_t)LNR_SCATTER_ROWS_MIN;
}

// The unit accumulation (k_bwd_accum_units + k_bwd_finalize_units) for mid-size batches: above the
// whole-bucket kernel's range, up to LNR_ACCUM_UNITS_MAX_N samples.  Measured (r03, backward stage):
// C4 shard 1/8 (0.59 M samples) 214 -> 188 us and shard 1/4 321 -> 312 us (the record-balanced split's
// ~1000 partial chunks and its finalize pass are a fixed ~35 us); C2 (4.7 M) 964 -> 984 us (equal
// record ranges balance the chip better than whole buckets there).  LONER_ACCUM_UNITS=1 / 0 forces
// it on / off (read at every launch).
// The unit accumulation's cut buckets finished by their last piece (1, default) or by
// k_bwd_finalize_units (0): LONER_UNITS_FINISH, read at every launch.
static bool units_finish() {
  const char* e = getenv("LONER_UNITS_FINISH");
  return e ? atoi(e) != 0 : true;
}
#ifndef LNR_ACCUM_UNITS_MAX_N
#define LNR_ACCUM_UNITS_MAX_N (int64_t(1) << 21)
#endif
// live: the live backward's records (a trained field's: ~20 % of every sample's at C2), for which the unit list
// balances better at any batch size (C2 trained: backward 0.307 -> 0.268 ms)
static bool accum_units(int64_t n, bool live = false) {
  const char* e = getenv("LONER_ACCUM_UNITS");
  if (e) return atoi(e) != 0;
  return n > accum_buckets_max_n() && (live || n <= LNR_ACCUM_UNITS_MAX_N);
}

// 1: cut buckets are finished inside k_bwd_accum by their last piece's workgroup; 0 (default): by
// k_bwd_finalize, one workgroup per bucket (LONER_ACCUM_FINISH).  Measured (r03): the in-kernel
// finishing serialises a workgroup's cut buckets behind its own accumulation, the finalize launch
// spreads them over the chip: C4 shard 1/8 backward 280 against 213 us, C2 972 against 966 us.
static bool accum_finish() {
  const char* e = getenv("LONER_ACCUM_FINISH");
  return e ? atoi(e) != 0 : false;
}

// Accumulate + finalize the buckets of levels [l0, l1): their slice of d_table becomes final.
static void launch_accum(const GridArgs& a, const BwdWorkspace& w, const lnr_grid_desc* d, int64_t n, uint32_t l0,
                         uint32_t l1, float* d_table, hipStream_t st, bool live = false) {
  const uint32_t b0 = a.bucket_base[l0], b1 = a.bucket_base[l1];
  if (b1 <= b0) return;
  const bool adam = a.adam.p != nullptr;
  if (accum_units(n, live)) {  // the work list: whole buckets and equal pieces of the large ones
    if (b0 != 0 || b1 != a.n_buckets)  // (a level range: its own list; the whole range's is the scan's)
      hipLaunchKernelGGL(k_bwd_units, dim3(1), dim3(1024), 0, st, w, b0, b1);
    if (units_finish()) {
      hipLaunchKernelGGL((adam ? k_bwd_accum_units<true, true> : k_bwd_accum_units<true, false>), dim3(b1 - b0 + kAccumGroups), dim3(kAccumThreads), 0, st, a, w,
                         d_table);
      return;
    }
    hipLaunchKernelGGL((adam ? k_bwd_accum_units<false, true> : k_bwd_accum_units<false, false>), dim3(b1 - b0 + kAccumGroups), dim3(kAccumThreads), 0, st, a, w,
                       d_table);
    hipLaunchKernelGGL((adam ? k_bwd_finalize_units<true> : k_bwd_finalize_units<false>), dim3(std::min<uint32_t>(b1 - b0, kAccumGroups)), dim3(kFinalizeThreads), 0,
                       st, a, w, d_table);
    return;
  }
  if (n <= accum_buckets_max_n()) {  // small batches: whole buckets, no partials, no finalize
    hipLaunchKernelGGL((adam ? k_bwd_accum_buckets<true> : k_bwd_accum_buckets<false>), dim3(b1 - b0), dim3(kAccumThreads), 0, st, a, w, d_table, b0, b1);
    return;
  }
  if (accum_finish()) {  // cut buckets finished by their last piece's workgroup: no finalize launch
    hipLaunchKernelGGL((adam ? k_bwd_accum<true, true> : k_bwd_accum<true, false>), dim3(kAccumGroups), dim3(kAccumThreads), 0, st, a, w, d_table, b0, b1);
    return;
  }
  hipLaunchKernelGGL((adam ? k_bwd_accum<false, true> : k_bwd_accum<false, false>), dim3(kAccumGroups), dim3(kAccumThreads), 0, st, a, w, d_table, b0, b1);
  hipLaunchKernelGGL((adam ? k_bwd_finalize<true> : k_bwd_finalize<false>), dim3(b1 - b0), dim3(kFinalizeThreads), 0, st, a, w, d_table, b0, b1);
}

template <class PosFn, class GradFn>
static int launch_bwd_bucketed(const lnr_grid_desc* d, PosFn pos, int64_t n, GradFn grad, float* d_table,
                               void* workspace, int64_t ws_bytes, int32_t flags, hipStream_t st, const char* who,
                               const AdamEpi* adam = nullptr) {
  GridArgs a = make_args(d, pos.samples_per_ray());
  if (adam) a.adam = *adam;
  LNR_REQUIRE(a.n_buckets <= (uint32_t)kMaxBuckets, "%s: too many table chunks (%u)", who, a.n_buckets);
  for (uint32_t l = 0; l < d->n_levels; ++l)
    LNR_REQUIRE(a.bucket_base[l + 1] - a.bucket_base[l] <= (uint32_t)kMaxChunksPerLevel,
                "%s: level %u has more than %d table chunks", who, l, kMaxChunksPerLevel);
  LNR_REQUIRE(workspace != nullptr && ws_bytes >= bwd_workspace_bytes(d, n),
              "%s: workspace too small (%lld < %lld bytes)", who, (long long)ws_bytes,
              (long long)bwd_workspace_bytes(d, n));
  LNR_REQUIRE(n < (int64_t(1) << 31), "%s: n=%lld samples exceeds 2^31", who, (long long)n);
  BwdWorkspace w = carve_workspace(workspace, a, d, n);
  const bool skip_zero = !(flags & LNR_BWD_COUNTS_READY);
  const uint32_t m = a.merge_levels, L = d->n_levels;
  bool all_fine = true, pow2 = true;
  uint32_t maxnb = 0;
  for (uint32_t l = 0; l < L; ++l) {
    if (l >= m) all_fine = all_fine && a.lv[l].fine;
    pow2 = pow2 && a.lv[l].size_mask != 0;
    maxnb = std::max(maxnb, a.bucket_base[l + 1] - a.bucket_base[l]);
  }
  // the reference's sigma grid (16 levels, base 16, scale 2, 2^18 entries): the level-looped scatter
  // plus the pass over the rows it could not stage; other grids (the colour grid's 2^19 levels have
  // 128 chunks): one workgroup per (row, level)
  // A small batch has too few rows for the level-looped kernel to fill the chip (C1: 64 rows, one
  // workgroup each walking 16 levels in sequence): one workgroup per (row, level) instead.
  const bool rows = L == 16 && all_fine && pow2 && 8 * n * (int64_t)L + 2 < (int64_t(1) << 32) &&
                    w.n_sb >= scatter_rows_min();
  const bool rows64 = rows && m >= 3 && m <= 7 && maxnb <= 64;
  // the live backward (LNR_BWD_LIVE): dL/dsigma-scaled gradients, the level-looped scatter, its own histogram of
  // the live records (a forward histogram, if any, is not read); otherwise the flag is ignored (the full backward:
  // bitwise the same gradient)
  const bool live = (flags & LNR_BWD_LIVE) && GradFn::kScaled && rows64;
  const bool prepare_only = (flags & LNR_BWD_PREPARE_ONLY) != 0, prepared = (flags & LNR_BWD_PREPARED) != 0;
  LNR_REQUIRE(!(prepare_only && prepared), "%s: PREPARE_ONLY and PREPARED together", who);
  LNR_REQUIRE(!(prepare_only || prepared) || live || (flags & LNR_BWD_COUNTS_READY),
              "%s: a split backward needs LNR_BWD_LIVE or LNR_BWD_COUNTS_READY (its counts must not read J)", who);
  if (prepared) {
    w.use_live = live;  // (the prepare call's scans cover the live rows)
  } else {
  if (!(flags & LNR_BWD_COUNTS_READY) && !live)
    hipLaunchKernelGGL((k_bwd_count<PosFn, GradFn>), dim3((unsigned)w.n_sb, d->n_levels), dim3(kSB), 0, st, a, pos, n,
                       grad, w);
  if (w.n_chunks > 1 && !live)
    hipLaunchKernelGGL(k_bwd_chunk_sums, dim3((unsigned)w.n_chunks, d->n_levels), dim3(kMaxChunksPerLevel), 0, st, a, w);
  if (live) {
    if constexpr (GradFn::kScaled) {
      const int64_t n_waves = (n + 63) / 64;
      hipLaunchKernelGGL(k_bwd_live_flags, dim3((unsigned)((n_waves * 16 + 255) / 256)), dim3(256), 0, st, grad.dsig, n, w);
      hipLaunchKernelGGL(k_bwd_live_list, dim3(1), dim3(1024), 0, st, n_waves, w);
      auto cnt = m == 3   ? k_bwd_count_live<PosFn, 16, 3, 64>
                 : m == 4 ? k_bwd_count_live<PosFn, 16, 4, 64>
                 : m == 5 ? k_bwd_count_live<PosFn, 16, 5, 64>
                 : m == 6 ? k_bwd_count_live<PosFn, 16, 6, 64>
                          : k_bwd_count_live<PosFn, 16, 7, 64>;
      hipLaunchKernelGGL(cnt, dim3((unsigned)w.n_sb), dim3(kSB), 0, st, a, pos, n, grad.dsig, w);
      w.use_live = true;  // the scans and the scatter below: the live rows
      if (w.n_chunks > 1)
        hipLaunchKernelGGL(k_bwd_chunk_sums, dim3((unsigned)w.n_chunks, d->n_levels), dim3(kMaxChunksPerLevel), 0, st, a,
                           w);
    }
  }
  hipLaunchKernelGGL(k_bwd_scan_rows, dim3((unsigned)w.n_chunks, d->n_levels), dim3(kMaxChunksPerLevel), 0, st, a, w);
  hipLaunchKernelGGL(k_bwd_scan_buckets, dim3(1), dim3(1024), 0, st, w, a.n_buckets);
  if (prepare_only) LNR_RETURN_LAUNCH(who);
  }
  if (!(flags & LNR_BWD_LEVEL_MAX_READY)) {  // (the record scales: after the MLP backward, which writes d_enc / J)
    LNR_REQUIRE(hipMemsetAsync(w.level_max, 0, LNR_MAX_LEVELS * sizeof(float), st) == hipSuccess, "%s: memset failed",
                who);
    hipLaunchKernelGGL(k_denc_level_max<GradFn>, dim3(kMaxBlocks, d->n_levels), dim3(256), 0, st, grad, n, w);
  }
  if (live) {
    if constexpr (GradFn::kScaled) {
      auto kern = m == 3   ? k_bwd_scatter_rows<PosFn, GradFn, 16, 3, 64, true>
                  : m == 4 ? k_bwd_scatter_rows<PosFn, GradFn, 16, 4, 64, true>
                  : m == 5 ? k_bwd_scatter_rows<PosFn, GradFn, 16, 5, 64, true>
                  : m == 6 ? k_bwd_scatter_rows<PosFn, GradFn, 16, 6, 64, true>
                           : k_bwd_scatter_rows<PosFn, GradFn, 16, 7, 64, true>;
      hipLaunchKernelGGL(kern, dim3((unsigned)w.n_sb), dim3(kSB), 0, st, a, pos, n, grad, w, skip_zero);
    }
  } else if (rows64) {
    auto kern = m == 3   ? k_bwd_scatter_rows<PosFn, GradFn, 16, 3, 64>
                : m == 4 ? k_bwd_scatter_rows<PosFn, GradFn, 16, 4, 64>
                : m == 5 ? k_bwd_scatter_rows<PosFn, GradFn, 16, 5, 64>
                : m == 6 ? k_bwd_scatter_rows<PosFn, GradFn, 16, 6, 64>
                         : k_bwd_scatter_rows<PosFn, GradFn, 16, 7, 64>;
    hipLaunchKernelGGL(kern, dim3((unsigned)w.n_sb), dim3(kSB), 0, st, a, pos, n, grad, w, skip_zero);
#if LNR_ROWS_NB128
  } else if (rows && m >= 5 && m <= 7 && maxnb <= 128) {  // the colour grid (2^19 entries: 128 chunks per level)
    auto kern = m == 5   ? k_bwd_scatter_rows<PosFn, GradFn, 16, 5, 128>
                : m == 6 ? k_bwd_scatter_rows<PosFn, GradFn, 16, 6, 128>
                         : k_bwd_scatter_rows<PosFn, GradFn, 16, 7, 128>;
    hipLaunchKernelGGL(kern, dim3((unsigned)w.n_sb), dim3(kSB), 0, st, a, pos, n, grad, w, skip_zero);
#endif
  } else {
    hipLaunchKernelGGL((k_bwd_scatter<PosFn, GradFn, kLevelsAny>), dim3((unsigned)(w.n_sb * L)), dim3(kSB), kScatterLds,
                       st, a, pos, n, grad, w, 0u, skip_zero);
  }
  if (flags & LNR_BWD_NO_ACCUM) LNR_RETURN_LAUNCH(who);  // accumulate later, by level range
  launch_accum(a, w, d, n, 0, d->n_levels, d_table, st, live);
  LNR_RETURN_LAUNCH(who);
}

static int check_desc_bwd(const lnr_grid_desc* d, const char* who) {
  LNR_REQUIRE(d != nullptr && d->n_levels >= 1 && d->n_levels <= LNR_MAX_LEVELS && d->n_features == 2,
              "%s: invalid grid descriptor", who);
  return LNR_OK;
}

// ---------------------------------------------------------------- input gradient (K3)
// dL/dpos01 of the encoding, tcnn v1.7 grid.h: kernel_grid's dy_dx branch (per level and feature the
// derivative of the trilinear blend along each axis: over the 4 cell edges along that axis, the
// product of the other two axes' weights times scale_l times (value at the edge's upper corner -
// value at its lower corner), the other axes in increasing order) followed by
// kernel_grid_backward_input (dL/dx[dim] = sum over (level, feature) in output order of
// dL/dy * dy/dx[dim]).  Table values are the fp16 forward operand; the arithmetic is fp32.
// One thread per sample walks every level, so each sample's gradient is one fixed-order sum (no
// atomics): deterministic.  The 8 corner gathers of a level are issued before any arithmetic.
// Only launched when the caller asks for d_pos: the map-only step (poses fixed) never pays for it; the
// joint pose + map step (loner_amd/pose.py) does, over its live samples only (dL/dsigma != 0).
constexpr int kDposThreads = 256;
#ifndef LNR_DPOS_LEVELS_PER_PASS
#define LNR_DPOS_LEVELS_PER_PASS 2  // C2 (tools/k3_metrics.py): 1.47 ms at 16, 1.35 at 8, 1.23 at 4, 1.13 at 2, 1.25 at 1
#endif
#ifndef LNR_DPOS_SPT
#define LNR_DPOS_SPT 0  // samples per thread of the one-launch, level-outer kernel (k_hashgrid_dpos_k: 2, 4, 8); 0: passes
#endif
#ifndef LNR_DPOS_SPT_SPARSE
#define LNR_DPOS_SPT_SPARSE 2  // the same for the compact (d_sigma J) gradient, whose dead waves leave at once
#endif
// Levels [l0, l1) per launch, added to the running sums d_pos holds (l0 > 0) in level order: the same
// fp32 additions in the same order as one pass over every level, so the result does not depend on the
// split, while each launch's gathers stay within a few levels' table slices (L2-resident: the whole
// 14.8 MB table is not).
// One level's term of sample i, added to its running sums (r0, r1, r2).
template <class GradFn>
__device__ __forceinline__ void dpos_level(const LevelParams& p, uint32_t l, int64_t i, float x, float y, float z,
                                           const uint32_t* __restrict__ table, const GradFn& grad, float& r0,
                                           float& r1, float& r2) {
  {
    Corners c;
    level_corners(p, x, y, z, c);
    uint32_t raw[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) raw[k] = table[c.idx[k]];
    const float2 g = grad.load(l, i);
    float2 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = half2_to_float2(raw[k]);
    const float t[3] = {c.tx, c.ty, c.tz};
    float dy[2][3];
#pragma unroll
    for (int dim = 0; dim < 3; ++dim) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float w = p.scale;
        int k = 0, nd = 0;
#pragma unroll
        for (int od = 0; od < 3; ++od) {
          if (od == dim) continue;
          const int bit = (e >> nd) & 1;
          w *= bit ? t[od] : 1.0f - t[od];
          k |= bit << od;
          ++nd;
        }
        const float2 lo = v[k], hi = v[k | (1 << dim)];
        s0 += w * (hi.x - lo.x);
        s1 += w * (hi.y - lo.y);
      }
      dy[0][dim] = s0;
      dy[1][dim] = s1;
    }
    r0 += g.x * dy[0][0];
    r1 += g.x * dy[0][1];
    r2 += g.x * dy[0][2];
    r0 += g.y * dy[1][0];
    r1 += g.y * dy[1][1];
    r2 += g.y * dy[1][2];
  }
}

template <class PosFn, class GradFn>
__global__ void __launch_bounds__(kDposThreads) k_hashgrid_dpos(GridArgs a, PosFn pos, int64_t n,
                                                                const uint32_t* __restrict__ table, GradFn grad,
                                                                float* __restrict__ d_pos, uint32_t l0, uint32_t l1) {
  const int64_t i = (int64_t)blockIdx.x * kDposThreads + threadIdx.x;
  if (i >= n) return;
  if constexpr (GradFn::kScaled) {
    // a sample with dL/dsigma = 0 has d_enc = 0 at every level, so d_pos = 0 (every term is +-0 * a finite
    // difference of fp16 values): skip its gathers (most samples of a trained field: the live backward's
    // dead samples, hashgrid.hpp) -- bitwise the full sum
    if (grad.scale(i) == 0.f) {
      if (l0 == 0) d_pos[3 * i + 0] = d_pos[3 * i + 1] = d_pos[3 * i + 2] = 0.f;
      return;
    }
  }
  float x, y, z;
  pos(i, x, y, z);
  float r0 = 0.f, r1 = 0.f, r2 = 0.f;
  if (l0 > 0) {
    r0 = d_pos[3 * i + 0];
    r1 = d_pos[3 * i + 1];
    r2 = d_pos[3 * i + 2];
  }
  for (uint32_t l = l0; l < l1; ++l) dpos_level(a.lv[l], l, i, x, y, z, table, grad, r0, r1, r2);
  d_pos[3 * i + 0] = r0;
  d_pos[3 * i + 1] = r1;
  d_pos[3 * i + 2] = r2;
}

// The same sums with K samples per thread (samples blockIdx.x K kDposThreads + k kDposThreads + t) and
// the levels as the OUTER loop, running sums in registers: the whole grid walks the levels roughly
// together (every workgroup starts at level 0), so the live table slices stay few without the passes'
// re-reads and re-writes of the running sums.  Same additions per sample in the same order: bitwise
// the result of k_hashgrid_dpos.
template <class PosFn, class GradFn, int K>
__global__ void __launch_bounds__(kDposThreads) k_hashgrid_dpos_k(GridArgs a, PosFn pos, int64_t n,
                                                                  const uint32_t* __restrict__ table, GradFn grad,
                                                                  float* __restrict__ d_pos) {
  const int64_t base = (int64_t)blockIdx.x * K * kDposThreads + threadIdx.x;
  float r[K][3];
#pragma unroll
  for (int k = 0; k < K; ++k) r[k][0] = r[k][1] = r[k][2] = 0.f;
  if constexpr (GradFn::kScaled) {  // a wave with no live sample (dL/dsigma = 0 throughout): zeros, no work
    bool any = false;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = base + (int64_t)k * kDposThreads;
      any |= i < n && grad.scale(i) != 0.f;
    }
    if (!__any(any)) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int64_t i = base + (int64_t)k * kDposThreads;
        if (i < n) d_pos[3 * i + 0] = d_pos[3 * i + 1] = d_pos[3 * i + 2] = 0.f;
      }
      return;
    }
  }
  for (uint32_t l = 0; l < a.n_levels; ++l) {
    const LevelParams& p = a.lv[l];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = base + (int64_t)k * kDposThreads;
      const bool in = i < n;
      float x = 0.f, y = 0.f, z = 0.f;
      pos.wave(i, n, in, x, y, z);
      bool live = in;
      if constexpr (GradFn::kScaled) live = live && grad.scale(i) != 0.f;  // (as k_hashgrid_dpos)
      if (live) dpos_level(p, l, i, x, y, z, table, grad, r[k][0], r[k][1], r[k][2]);
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int64_t i = base + (int64_t)k * kDposThreads;
    if (i < n) {
      d_pos[3 * i + 0] = r[k][0];
      d_pos[3 * i + 1] = r[k][1];
      d_pos[3 * i + 2] = r[k][2];
    }
  }
}

template <class PosFn, class GradFn>
static int launch_dpos(const lnr_grid_desc* d, PosFn pos, int64_t n, const uint16_t* table, GradFn grad,
                       float* d_pos, hipStream_t st, const char* who) {
  LNR_REQUIRE(table != nullptr, "%s: d_pos needs the fp16 table", who);
  LNR_REQUIRE((reinterpret_cast<uintptr_t>(table) & 3) == 0, "%s: table must be 4-byte aligned", who);
  const GridArgs a = make_args(d, pos.samples_per_ray());
  const int64_t nb = (n + kDposThreads - 1) / kDposThreads;
  LNR_REQUIRE(nb < (int64_t(1) << 31), "%s: n=%lld too large", who, (long long)n);
  // the compact encoding gradient (GradJac) is sparse on a trained field (most samples' dL/dsigma = 0): one
  // level-outer launch whose dead waves leave at once (LNR_DPOS_SPT_SPARSE samples per thread) instead of the
  // passes, which re-read every sample per pass (C2 joint pose + map: tools/experiments/r06_ert.sh)
  const char* ek = getenv("LONER_DPOS_SPT");
  const int spt = ek ? atoi(ek) : (GradFn::kScaled ? LNR_DPOS_SPT_SPARSE : LNR_DPOS_SPT);
  if (spt == 2 || spt == 4 || spt == 8) {
    const unsigned g = (unsigned)((n + (int64_t)spt * kDposThreads - 1) / ((int64_t)spt * kDposThreads));
    const uint32_t* tb = reinterpret_cast<const uint32_t*>(table);
    if (spt == 2)
      hipLaunchKernelGGL((k_hashgrid_dpos_k<PosFn, GradFn, 2>), dim3(g), dim3(kDposThreads), 0, st, a, pos, n, tb, grad, d_pos);
    else if (spt == 4)
      hipLaunchKernelGGL((k_hashgrid_dpos_k<PosFn, GradFn, 4>), dim3(g), dim3(kDposThreads), 0, st, a, pos, n, tb, grad, d_pos);
    else
      hipLaunchKernelGGL((k_hashgrid_dpos_k<PosFn, GradFn, 8>), dim3(g), dim3(kDposThreads), 0, st, a, pos, n, tb, grad, d_pos);
    LNR_RETURN_LAUNCH(who);
  }
  const char* e = getenv("LONER_DPOS_LEVELS_PER_PASS");
  const uint32_t per = e ? (uint32_t)std::max(1, atoi(e)) : (uint32_t)LNR_DPOS_LEVELS_PER_PASS;
  for (uint32_t l0 = 0; l0 < d->n_levels; l0 += per)
    hipLaunchKernelGGL((k_hashgrid_dpos<PosFn, GradFn>), dim3((unsigned)nb), dim3(kDposThreads), 0, st, a, pos, n,
                       reinterpret_cast<const uint32_t*>(table), grad, d_pos, l0, std::min(l0 + per, d->n_levels));
  LNR_RETURN_LAUNCH(who);
}

// An empty batch still overwrites its outputs: the table gradient (or the level range's slice of it)
// is zero.
static int zero_table_levels(const lnr_grid_desc* d, float* d_table, uint32_t l0, uint32_t l1, hipStream_t st,
                             const char* who) {
  if (!d_table || l1 <= l0) return LNR_OK;
  const size_t e0 = d->offset[l0], e1 = d->offset[l1];
  LNR_REQUIRE(hipMemsetAsync(d_table + 2 * e0, 0, (e1 - e0) * 2 * sizeof(float), st) == hipSuccess,
              "%s: memset failed", who);
  return LNR_OK;
}

}  // namespace lnr

using namespace lnr;

extern "C" int64_t lnr_hashgrid_bwd_workspace_bytes(const lnr_grid_desc* d, int64_t n) {
  if (d == nullptr || n < 0) return -1;
  return bwd_workspace_bytes(d, n);
}

extern "C" float* lnr_hashgrid_bwd_level_max(const lnr_grid_desc* d, int64_t n, void* workspace) {
  if (d == nullptr || n < 0 || workspace == nullptr || check_desc_bwd(d, "lnr_hashgrid_bwd_level_max")) return nullptr;
  return carve_workspace(workspace, make_args(d), d, n).level_max;
}

extern "C" const uint64_t* lnr_hashgrid_bwd_seg_start(const lnr_grid_desc* d, int64_t n, void* workspace) {
  if (d == nullptr || n < 0 || workspace == nullptr || check_desc_bwd(d, "lnr_hashgrid_bwd_seg_start")) return nullptr;
  return carve_workspace(workspace, make_args(d), d, n).seg_start;
}

// The three backward entry points: d_table (optional: NULL = no table gradient) through the binned
// scatter, d_pos (optional: NULL = no input gradient) through k_hashgrid_dpos.
template <class PosFn, class GradFn>
static int bwd_entry(const lnr_grid_desc* d, PosFn pos, int64_t n, GradFn grad, float* d_table, const uint16_t* table,
                     float* d_pos, void* workspace, int64_t workspace_bytes, int32_t flags, hipStream_t st,
                     const char* who) {
  if (n == 0) {
    if (flags & LNR_BWD_NO_ACCUM) return LNR_OK;  // lnr_hashgrid_bwd_accum zeroes each range
    if (int e = zero_table_levels(d, d_table, 0, d->n_levels, st, who)) return e;
    LNR_RETURN_LAUNCH(who);
  }
  if (d_pos)
    if (int e = launch_dpos(d, pos, n, table, grad, d_pos, st, who)) return e;
  if (!d_table) return LNR_OK;
  return launch_bwd_bucketed(d, pos, n, grad, d_table, workspace, workspace_bytes, flags, st, who);
}

extern "C" int lnr_hashgrid_bwd(const lnr_grid_desc* d, const float* pos01, int64_t n, const float* d_enc,
                                int64_t enc_stride, float* d_table, const uint16_t* table, float* d_pos,
                                void* workspace, int64_t workspace_bytes, int32_t flags, void* stream) {
  if (int e = check_desc_bwd(d, "lnr_hashgrid_bwd")) return e;
  LNR_REQUIRE(n >= 0 && enc_stride >= n, "lnr_hashgrid_bwd: bad sizes");
  LNR_REQUIRE(n == 0 || (pos01 && d_enc && (d_table || d_pos)), "lnr_hashgrid_bwd: null pointer");
  return bwd_entry(d, PosFromArray{pos01}, n, GradF32{reinterpret_cast<const float2*>(d_enc), enc_stride}, d_table,
                   table, d_pos, workspace, workspace_bytes, flags, as_stream(stream), "lnr_hashgrid_bwd");
}

extern "C" int lnr_hashgrid_bwd_accum(const lnr_grid_desc* d, int64_t n, void* workspace, int64_t workspace_bytes,
                                      uint32_t level_begin, uint32_t level_end, float* d_table, void* stream) {
  return lnr_hashgrid_bwd_accum_flags(d, n, workspace, workspace_bytes, level_begin, level_end, d_table, 0, stream);
}

extern "C" int lnr_hashgrid_bwd_accum_flags(const lnr_grid_desc* d, int64_t n, void* workspace, int64_t workspace_bytes,
                                            uint32_t level_begin, uint32_t level_end, float* d_table, int32_t flags,
                                            void* stream) {
  if (int e = check_desc_bwd(d, "lnr_hashgrid_bwd_accum")) return e;
  LNR_REQUIRE(level_begin <= level_end && level_end <= d->n_levels, "lnr_hashgrid_bwd_accum: bad level range");
  LNR_REQUIRE(n >= 0 && workspace && workspace_bytes >= bwd_workspace_bytes(d, n) && d_table,
              "lnr_hashgrid_bwd_accum: bad workspace / pointers");
  if (n == 0) {
    if (int e = zero_table_levels(d, d_table, level_begin, level_end, as_stream(stream), "lnr_hashgrid_bwd_accum"))
      return e;
    LNR_RETURN_LAUNCH("lnr_hashgrid_bwd_accum");
  }
  const GridArgs a = make_args(d);
  launch_accum(a, carve_workspace(workspace, a, d, n), d, n, level_begin, level_end, d_table, as_stream(stream),
               (flags & LNR_BWD_LIVE) != 0);
  LNR_RETURN_LAUNCH("lnr_hashgrid_bwd_accum");
}

extern "C" int lnr_hashgrid_bwd_rays(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                     int32_t n_samples, const float* d_enc, int64_t enc_stride, float* d_table,
                                     const uint16_t* table, float* d_pos, void* workspace, int64_t workspace_bytes,
                                     int32_t flags, void* stream) {
  if (int e = check_desc_bwd(d, "lnr_hashgrid_bwd_rays")) return e;
  const int64_t n = n_rays * (int64_t)n_samples;
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && enc_stride >= n, "lnr_hashgrid_bwd_rays: bad sizes");
  LNR_REQUIRE(n == 0 || (rays && z && d_enc && (d_table || d_pos)), "lnr_hashgrid_bwd_rays: null pointer");
  return bwd_entry(d, PosFromRays{rays, z, n_samples}, n, GradF32{reinterpret_cast<const float2*>(d_enc), enc_stride},
                   d_table, table, d_pos, workspace, workspace_bytes, flags, as_stream(stream),
                   "lnr_hashgrid_bwd_rays");
}

extern "C" int lnr_hashgrid_bwd_rays_live(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                          int32_t n_samples, const float* d_enc, int64_t enc_stride, const float* live,
                                          float* d_table, void* workspace, int64_t workspace_bytes, int32_t flags,
                                          void* stream) {
  if (int e = check_desc_bwd(d, "lnr_hashgrid_bwd_rays_live")) return e;
  const int64_t n = n_rays * (int64_t)n_samples;
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && enc_stride >= n, "lnr_hashgrid_bwd_rays_live: bad sizes");
  LNR_REQUIRE(n == 0 || (rays && z && d_enc && live && d_table), "lnr_hashgrid_bwd_rays_live: null pointer");
  return bwd_entry(d, PosFromRays{rays, z, n_samples}, n,
                   GradF32{reinterpret_cast<const float2*>(d_enc), enc_stride, live}, d_table, nullptr, nullptr,
                   workspace, workspace_bytes, flags, as_stream(stream), "lnr_hashgrid_bwd_rays_live");
}

// Adam with a zero gradient on every table parameter (the fused entry's empty batch)
__global__ void __launch_bounds__(256) k_adam_zero_grad(GridArgs a, int64_t n) {
  const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t i = 8 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x); i < n; i += 8 * (int64_t)gridDim.x * blockDim.x)
    put_grad8<true>(a, nullptr, i, z, n - i < 8 ? (uint32_t)(n - i) : 8u);
}

extern "C" int lnr_hashgrid_bwd_rays_jac_adam(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                              int32_t n_samples, const uint32_t* d_jac, const float* d_sigma,
                                              int64_t jac_stride, const lnr_adam_epilogue* adam, void* workspace,
                                              int64_t workspace_bytes, int32_t flags, void* stream) {
  const char* who = "lnr_hashgrid_bwd_rays_jac_adam";
  if (int e = check_desc_bwd(d, who)) return e;
  const int64_t n = n_rays * (int64_t)n_samples;
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && jac_stride >= n, "%s: bad sizes", who);
  LNR_REQUIRE(adam && adam->param && adam->shadow && adam->m && adam->v && adam->step >= 1, "%s: bad Adam epilogue", who);
  LNR_REQUIRE(((uintptr_t)adam->param | (uintptr_t)adam->shadow | (uintptr_t)adam->m | (uintptr_t)adam->v) % 16 == 0,
              "%s: the Adam epilogue's buffers must be 16-byte aligned", who);
  LNR_REQUIRE(!(flags & LNR_BWD_NO_ACCUM), "%s: LNR_BWD_NO_ACCUM has no place with the Adam epilogue", who);
  LNR_REQUIRE(n == 0 || (rays && z && d_jac && d_sigma), "%s: null pointer", who);
  AdamEpi e{};
  e.p = adam->param;
  e.shadow = adam->shadow;
  e.m = adam->m;
  e.v = adam->v;
  e.dev_step = adam->dev_step;
  if (int r = lnr_adam_coefficients(adam->step, adam->lr, adam->beta1, adam->beta2, &e.step_size, &e.bc2_sqrt)) return r;
  e.one_minus_b1 = (float)(1.0 - adam->beta1);  // as lnr_adam_step forms them
  e.b2 = (float)adam->beta2;
  e.one_minus_b2 = (float)(1.0 - adam->beta2);
  e.eps = (float)adam->eps;
  hipStream_t st = as_stream(stream);
  if (n == 0) {
    GridArgs a = make_args(d);
    a.adam = e;
    const int64_t np = 2 * (int64_t)d->n_entries;
    hipLaunchKernelGGL(k_adam_zero_grad, dim3((unsigned)std::min<int64_t>((np + 255) / 256, 8192)), dim3(256), 0, st, a, np);
    LNR_RETURN_LAUNCH(who);
  }
  return launch_bwd_bucketed(d, PosFromRays{rays, z, n_samples}, n, GradJac{d_jac, d_sigma, jac_stride}, nullptr,
                             workspace, workspace_bytes, flags, st, who, &e);
}

extern "C" int lnr_hashgrid_bwd_rays_jac(const lnr_grid_desc* d, const float* rays, const float* z, int64_t n_rays,
                                         int32_t n_samples, const uint32_t* d_jac, const float* d_sigma,
                                         int64_t jac_stride, float* d_table, const uint16_t* table, float* d_pos,
                                         void* workspace, int64_t workspace_bytes, int32_t flags, void* stream) {
  if (int e = check_desc_bwd(d, "lnr_hashgrid_bwd_rays_jac")) return e;
  const int64_t n = n_rays * (int64_t)n_samples;
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && jac_stride >= n, "lnr_hashgrid_bwd_rays_jac: bad sizes");
  LNR_REQUIRE(n == 0 || (rays && z && d_jac && d_sigma && (d_table || d_pos)),
              "lnr_hashgrid_bwd_rays_jac: null pointer");
  return bwd_entry(d, PosFromRays{rays, z, n_samples}, n, GradJac{d_jac, d_sigma, jac_stride}, d_table, table, d_pos,
                   workspace, workspace_bytes, flags, as_stream(stream), "lnr_hashgrid_bwd_rays_jac");
}

LNR_PHASE_EXPORT(hashgrid_bwd)
