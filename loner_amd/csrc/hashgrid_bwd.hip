// Hash-grid backward (tcnn kernel_grid_backward semantics) as an atomic-free binned scatter.
//
// Measured on MI355X: scattered fp32 global atomics run at ~20 G lane-ops/s (memory-side
// execution) and LDS ds_add_f32 at only 0.33 lanes/clk/CU whatever the address pattern, while
// ds_add_u64 runs at 4.8 lanes/clk/CU.  So the backward is
//   count   per (kSB-sample row, level) record histogram per 4096-entry table chunk
//           (emitted by the training forward, or by k_bwd_count)
//   scan    column prefix over rows -> exact record offsets (no global atomics, no capacity guess)
//   scatter 12-byte records (hashgrid.hpp: one per x-pair of corners at fine levels, one per
//           merged corner at coherent levels) staged in LDS in bucket order and written as
//           coalesced runs; per-row max |value| for the fixed-point scale
//   accum   one workgroup per (bucket, slice): int64 fixed-point sums in a 64 KB LDS chunk with
//           ds_add_u64, converted back to fp32 and stored; a bucket split over several slices
//           stores per-slice int64 partial chunks that k_bwd_finalize adds exactly
// No float atomics anywhere: the result is bitwise reproducible, and d_table is overwritten.
#include "hashgrid.hpp"

namespace lnr {

// Histogram after the MLP backward: samples whose d_enc is zero at a non-coherent level (ReLU'd
// sigma: relu(sigma + noise) = 0 gives dL/dsigma = 0 exactly, typically half the samples) emit no
// records there; the scatter skips them the same way (skip_zero).
template <class PosFn>
__global__ void __launch_bounds__(kSB) k_bwd_count(GridArgs a, PosFn pos, int64_t n, const float2* __restrict__ d_enc,
                                                   int64_t stride, BwdWorkspace ws) {
  __shared__ uint32_t hist[kMaxChunksPerLevel];
  const uint32_t l = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * kSB + threadIdx.x;
  const bool in = i < n;
  for (int b = threadIdx.x; b < kMaxChunksPerLevel; b += blockDim.x) hist[b] = 0;
  float x = 0.f, y = 0.f, z = 0.f;
  bool act = false;
  if (in) {
    pos(i, x, y, z);
    const float2 g = d_enc[(int64_t)l * stride + i];
    act = g.x != 0.f || g.y != 0.f;
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
  const int64_t r0 = (int64_t)ch * kRowsPerChunk;
  const int64_t r1 = r0 + kRowsPerChunk < ws.n_sb ? r0 + kRowsPerChunk : ws.n_sb;
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
__global__ void __launch_bounds__(1024) k_bwd_scan_buckets(BwdWorkspace ws, uint32_t n_buckets, uint32_t coarse_end) {
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
    const int64_t slr = b < coarse_end ? kSliceRecordsCoarse : kSliceRecords;
    const uint32_t k = (uint32_t)((c + slr - 1) / slr);
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
  lds_barrier();
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
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// KIND: the levels one launch covers, so each gets only its own code and registers.
// kLevelsAny: one launch over every level, grid.x = rows x levels with the level fastest, so each CU
// interleaves VALU-heavy coherent-level rows with store-heavy fine-level rows; consecutive rows of
// one level are L blocks apart, i.e. on the same XCD when L is a multiple of 8 (see xcd_row).
enum : int { kLevelsCoherent = 0, kLevelsFine = 1, kLevelsGeneric = 2, kLevelsAny = 3 };

#ifndef LNR_SCATTER_WAVES_PER_EU
#define LNR_SCATTER_WAVES_PER_EU 1
#endif
// One (histogram row sb, level l) of the scatter; KIND as below, kLevelsAny meaning "any level".
template <class PosFn, int KIND>
__device__ __forceinline__ void scatter_row_level(const GridArgs& a, const PosFn& pos, int64_t n,
                                                  const float2* __restrict__ d_enc, int64_t stride,
                                                  const BwdWorkspace& ws, uint32_t l, int64_t sb, bool skip_zero,
                                                  char* smem) {
  RecVal* stage_v = reinterpret_cast<RecVal*>(smem);                         // [kCap]
  uint64_t* gbase = reinterpret_cast<uint64_t*>(stage_v + kCap);             // [kMaxChunksPerLevel]
  uint32_t* stage_w = reinterpret_cast<uint32_t*>(gbase + kMaxChunksPerLevel);  // [kCap]
  uint32_t* rank_ctr = stage_w + kCap;                                       // [kMaxChunksPerLevel]
  uint32_t* start = rank_ctr + kMaxChunksPerLevel;                           // [kMaxChunksPerLevel + 1]
  float* wmax = reinterpret_cast<float*>(start + kMaxChunksPerLevel + 1);    // [kSB / 64]
  uint8_t* sbk = reinterpret_cast<uint8_t*>(wmax + kSB / 64);                // [kCap] bucket of each staged record
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
  static_assert(kMaxChunksPerLevel <= 128, "two buckets per lane of wave 0");
  LNR_STAMP(t0);
  // 1. Global loads, all unconditional (clamped indices) so nothing waits for them before it must:
  //    the sample's position inputs and d_enc, and (wave 0) the row's offsets.
  const int64_t ic = in ? i : n - 1;
  const typename PosFn::Raw raw = pos.load(ic);
  // d_enc is read once: a nontemporal load keeps it from displacing the L2 lines in which adjacent
  // rows' bucket runs combine (scatter -1.5 % at C2)
  const f32x2 g_nt = __builtin_nontemporal_load(reinterpret_cast<const f32x2*>(&d_enc[(int64_t)l * stride + ic]));
  const float2 g_raw = make_float2(g_nt.x, g_nt.y);
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
  const bool act = in && (!skip_zero || g.x != 0.f || g.y != 0.f);
  float m = 0.f;
  bool staged = true;
  auto place = [&](bool valid, uint32_t bk, uint32_t rank, uint32_t word, float2 val) {
    if (!valid) return;
    m = fmaxf(m, fmaxf(fabsf(val.x), fabsf(val.y)));
    if (staged) {
      const uint32_t t = start[bk] + rank;
      stage_w[t] = word;
      stage_v[t] = pack_rec(val.x, val.y);
      sbk[t] = (uint8_t)bk;
    } else {
      const uint64_t dst = gbase[bk] + rank;
      ws.rec_w[dst] = word;
      ws.rec_v[dst] = pack_rec(val.x, val.y);
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
  m = wave_max(m);
  if (lane == 0) wmax[wid] = m;
  LNR_STAMP(t2);
  lds_barrier();
  LNR_STAMP(t3);
  if (wid == 0) {
    float mm = lane < kSB / 64 ? wmax[lane] : 0.f;
    mm = wave_max(mm);
    if (lane == 0) ws.blockmax[(int64_t)l * ws.n_sb + sb] = mm;
  }
  // 3. copy the staged row out in bucket order (consecutive lanes -> consecutive slots of a run)
  if (staged) {
    const uint32_t total = start[nb];
    for (uint32_t t = threadIdx.x; t < total; t += kSB) {
      const uint32_t bk = sbk[t];
      const uint64_t dst = gbase[bk] + (t - start[bk]);
#ifndef LNR_EXP_SKIP_STORE
      ws.rec_w[dst] = stage_w[t];
      ws.rec_v[dst] = stage_v[t];
#else
      if (stage_w[t] == 0x12345678u) ws.rec_w[dst] = 0;
#endif
    }
  }
  LNR_STAMP(t4);
  LNR_PHASE_BY(sb, 5 * kind + 0, t1, t0);
  LNR_PHASE_BY(sb, 5 * kind + 1, t2, t1);
  LNR_PHASE_BY(sb, 5 * kind + 2, t3, t2);
  LNR_PHASE_BY(sb, 5 * kind + 3, t4, t3);
}

template <class PosFn, int KIND>
__global__ void __launch_bounds__(kSB, LNR_SCATTER_WAVES_PER_EU) k_bwd_scatter(GridArgs a, PosFn pos, int64_t n,
                                                                             const float2* __restrict__ d_enc,
                                                                             int64_t stride, BwdWorkspace ws, uint32_t l0,
                                                                             bool skip_zero) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t l = KIND == kLevelsAny ? blockIdx.x % a.n_levels : l0 + blockIdx.y;
  const int64_t sb = KIND == kLevelsAny ? (int64_t)(blockIdx.x / a.n_levels) : xcd_row(blockIdx.x, gridDim.x);
  scatter_row_level<PosFn, KIND>(a, pos, n, d_enc, stride, ws, l, sb, skip_zero, smem);
}

// The (row, level) items the level-looped scatter could not stage (more than kCap records: rows of
// coherent levels whose runs did not merge, or pathological split pairs), each as above.
template <class PosFn>
__global__ void __launch_bounds__(kSB, LNR_SCATTER_WAVES_PER_EU) k_bwd_scatter_overflow(GridArgs a, PosFn pos, int64_t n,
                                                                                      const float2* __restrict__ d_enc,
                                                                                      int64_t stride, BwdWorkspace ws,
                                                                                      bool skip_zero) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ unsigned long long masks[kSB / 64];
  // workgroup b checks the flags of items [b kSB, (b + 1) kSB), item = level * n_sb + row
  const int64_t items = ws.n_sb * a.n_levels;
  const int64_t it = (int64_t)blockIdx.x * kSB + threadIdx.x;
  const unsigned long long m = __ballot(it < items && ws.ovf[it] != 0);
  if ((threadIdx.x & 63) == 0) masks[threadIdx.x >> 6] = m;
  __syncthreads();
  for (int w = 0; w < kSB / 64; ++w) {
    for (unsigned long long mm = masks[w]; mm; mm &= mm - 1) {
      const int64_t q = (int64_t)blockIdx.x * kSB + 64 * w + __ffsll((long long)mm) - 1;
      scatter_row_level<PosFn, kLevelsAny>(a, pos, n, d_enc, stride, ws, (uint32_t)(q / ws.n_sb), q % ws.n_sb,
                                           skip_zero, smem);
      lds_barrier();
    }
  }
}

// Level-looped scatter: one workgroup per histogram row walks every level, so a sample's position is
// loaded and decoded once (not once per level), the next level's d_enc and histogram row are in
// flight while this level ranks and places, and the copy-out of level l - 1 overlaps the ranking of
// level l (double-buffered staging, one barrier per level).  A level's bucket starts come from the
// forward's histogram alone, so wave 0 computes them one level ahead and every record is placed the
// moment its rank returns.  Same records, counts and blockmax as k_bwd_scatter.
// ---------------------------------------------------------------------------------------------
// Level-looped scatter: one workgroup per histogram row walks every level.
//  * All global loads happen in the prologue: the sample's position, its d_enc at every level (32
//    registers) and, wave w, the histogram rows of levels 2w and 2w + 1, turned at once into every
//    level's bucket starts.  The level loop then issues only LDS operations and the copy-out
//    stores, so nothing in it ever waits on global memory.
//  * Each record is ranked (returning LDS atomic) and placed at once, 16 B {word, global slot, v0,
//    v1} in bucket order; the copy-out of level l - 1 overlaps level l (double-buffered stage, one
//    barrier per level).
//  * A (row, level) with more than kRowsCap records is flagged and left to k_bwd_scatter_overflow.
// Same records, counts and blockmax as k_bwd_scatter.
constexpr int kRowsCap = 2176;  // 4.25 records per sample: fine rows hold 4 + the rare split pairs
template <int NL, int NB>
struct RowsLds {  // the small tables first: their addresses fit the 16-bit LDS instruction offset
  uint2 sg[NL][NB];           // per level and bucket: {start in the stage, global slot of the run}
  uint32_t total[NL];         // records of the row at each level
  uint32_t ctr[2][NB];        // rank counters
  float wmax[2][kSB / 64];
  LevelParams lv[NL];         // the level table (kernel arguments indexed per level would be loads)
  uint4 stage[2][kRowsCap];   // staged records {word, global slot, v0, v1}, bucket order
};
static_assert(sizeof(RecVal) == 8, "the level-looped scatter stages fp32 record values");

// NL levels, the first NM coherent (run-merging) and the rest fine, at most NB buckets per level:
// compile-time, so the level loop unrolls into straight-line code.  Record slots are 32-bit (the
// launcher checks 8 N L < 2^32).
template <class PosFn, int NL, int NM, int NB>
__global__ void __launch_bounds__(kSB) __attribute__((amdgpu_waves_per_eu(4, 4)))
k_bwd_scatter_rows(GridArgs a, PosFn pos, int64_t n, const float2* __restrict__ d_enc, int64_t stride, BwdWorkspace ws,
                   bool skip_zero) {
  static_assert(NL <= 2 * (kSB / 64), "wave w prepares levels 2w and 2w + 1");
  static_assert(NB <= 128, "two buckets per lane");
  __shared__ RowsLds<NL, NB> sm;
  const int64_t sb = xcd_row(blockIdx.x, gridDim.x);
  const int64_t i = sb * kSB + threadIdx.x;
  const bool in = i < n;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool last = sb + 1 >= ws.n_sb;
  const int64_t ic = in ? i : n - 1;
  uint32_t* rec_v32 = reinterpret_cast<uint32_t*>(ws.rec_v);
  const uint32_t spare = (uint32_t)(8 * n * (int64_t)NL);  // one of the 2 slack records past the last slot

  // prologue 1: the level table and zero rank counters
  if (threadIdx.x < NL * (sizeof(LevelParams) / 4))
    reinterpret_cast<uint32_t*>(sm.lv)[threadIdx.x] = reinterpret_cast<const uint32_t*>(a.lv)[threadIdx.x];
  if (threadIdx.x < 2 * NB) (&sm.ctr[0][0])[threadIdx.x] = 0u;
  // prologue 2: every global load of the kernel
  const typename PosFn::Raw raw = pos.load(ic);
  f32x2 g[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l)  // read once: nontemporal, so they do not displace the runs' L2 lines
    g[l] = __builtin_nontemporal_load(reinterpret_cast<const f32x2*>(&d_enc[(int64_t)l * stride + ic]));
  uint32_t h0[2][2], h1[2][2];
  uint64_t seg[2][2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const uint32_t l = 2 * wid + p;
    if (l < (uint32_t)NL) {
      const uint32_t b0 = a.bucket_base[l], nb = a.bucket_base[l + 1] - b0;
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
  float x = 0.f, y = 0.f, z = 0.f;
  pos.eval(raw, x, y, z);
  // prologue 3: wave w's levels' bucket starts (a wave prefix over the buckets, two per lane)
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const uint32_t l = 2 * wid + p;
    if (l < (uint32_t)NL) {
      const uint32_t nb = a.bucket_base[l + 1] - a.bucket_base[l];
      const uint32_t c0 = 2 * lane < nb ? h1[p][0] - h0[p][0] : 0u;
      const uint32_t c1 = 2 * lane + 1 < nb ? h1[p][1] - h0[p][1] : 0u;
      const uint32_t inc = wave_incl_scan_u32(c0 + c1);
      const uint32_t ex = inc - c0 - c1;
      if (2 * lane < nb) sm.sg[l][2 * lane] = make_uint2(ex, (uint32_t)(seg[p][0] + h0[p][0]));
      if (2 * lane + 1 < nb) sm.sg[l][2 * lane + 1] = make_uint2(ex + c0, (uint32_t)(seg[p][1] + h0[p][1]));
      if (lane == 63) {
        sm.total[l] = inc;
        ws.ovf[(int64_t)l * ws.n_sb + sb] = inc > (uint32_t)kRowsCap;  // unstaged: k_bwd_scatter_overflow's item
      }
    }
  }
  lds_barrier();

  // copy level l's staged row out (consecutive threads -> consecutive slots of a run); a second wave
  // publishes the row's max |value|.  Every lane stores on every trip (lanes past the row's records
  // into the spare slot), so the trip count is fixed
  auto copy_out = [&](uint32_t l) {
    const int sbuf = l & 1;
    const uint32_t total = sm.total[l];
    const uint32_t lim = total <= (uint32_t)kRowsCap ? total : 0u;
#pragma unroll
    for (int u = 0; u < (kRowsCap + kSB - 1) / kSB; ++u) {
      const uint32_t t = threadIdx.x + u * kSB;
      const uint4 q = sm.stage[sbuf][t < (uint32_t)kRowsCap ? t : kRowsCap - 1];
      const uint32_t d = t < lim ? q.y : spare;
      ws.rec_w[d] = q.x;
      *reinterpret_cast<u32x2*>(rec_v32 + 2 * (uint64_t)d) = u32x2{q.z, q.w};
    }
    if (wid == 1) {
      const float mm = wave_max_nonneg(lane < kSB / 64 ? sm.wmax[sbuf][lane] : 0.f);
      if (lane == 0) ws.blockmax[(int64_t)l * ws.n_sb + sb] = mm;
    }
  };

#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const int sbuf = l & 1;
    const LevelParams lv = sm.lv[l];
    const bool staged = sm.total[l] <= (uint32_t)kRowsCap;  // block-uniform
    uint32_t* ctr = sm.ctr[sbuf];
    const uint2* sgl = sm.sg[l];
    const float2 gv = in ? make_float2(g[l].x, g[l].y) : make_float2(0.f, 0.f);
    const bool inr = staged && in;  // an unstaged row emits nothing here: k_bwd_scatter_overflow redoes it
    const bool act = inr && (!skip_zero || gv.x != 0.f || gv.y != 0.f);
    float m = 0.f;
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
          m = fmaxf(m, fmaxf(fabsf(val[k].x), fabsf(val[k].y)));
          sm.stage[sbuf][s4[k].x + rank[k]] = make_uint4(word[k], s4[k].y + rank[k], __float_as_uint(val[k].x),
                                                         __float_as_uint(val[k].y));
        }
      }
    };
    uint32_t bk4[4], w4[4];
    float2 val4[4];
    if (l >= NM) {  // fine: one record per x-pair (hashgrid.hpp "Backward records")
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
      const bool valid = inr && ri.tail;
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
    m = wave_max_nonneg(m);
    if (lane == 0) sm.wmax[sbuf][wid] = m;
    if (threadIdx.x < NB) sm.ctr[sbuf ^ 1][threadIdx.x] = 0u;  // level l + 1's counters (last used by l - 1)
    if (l >= 1) copy_out(l - 1);
    lds_barrier();
  }
  copy_out(NL - 1);
}

constexpr size_t kScatterLds = (size_t)kCap * sizeof(RecVal) + kMaxChunksPerLevel * 8 + (size_t)kCap * 4 + kMaxChunksPerLevel * 4 +
                               (kMaxChunksPerLevel + 1) * 4 + (kSB / 64) * 4 + kCap;
static_assert(kScatterLds <= 65536, "scatter LDS within the default dynamic limit");

__global__ void __launch_bounds__(256) k_bwd_level_max(BwdWorkspace ws) {
  __shared__ float red[4];
  const float* col = ws.blockmax + (int64_t)blockIdx.x * ws.n_sb;
  float m = 0.f;
  for (int64_t j = threadIdx.x; j < ws.n_sb; j += 256) m = fmaxf(m, col[j]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  lds_barrier();
  if (threadIdx.x == 0) ws.level_max[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

constexpr int kAccumThreads = 1024;

// Fixed-point exponent of bucket b: |record| < 2^E (the level's max) and at most cnt records in the
// bucket, so every value, and every partial or total sum, stays below 2^50 in magnitude: inside the
// exact-integer range of the double-precision conversion below.  The unit is 2^(lg cnt + E - 50),
// about 2^-32 of the level maximum at C2's bucket sizes.
__device__ __forceinline__ int bucket_k2(const BwdWorkspace& ws, uint32_t l, uint32_t b) {
  int E;
  frexpf(ws.level_max[l], &E);
  const uint64_t bcnt = ws.seg_start[b + 1] - ws.seg_start[b];
  const int lg = 64 - __clzll((long long)(bcnt > 0 ? bcnt : 1));  // ceil-ish log2(cnt + 1)
  const int k2 = 50 - lg - E;
  return k2 > 120 ? 120 : (k2 < -120 ? -120 : k2);
}

// round(x) as int64 for |x| < 2^51: x + 1.5 2^52 in double places the rounded integer in the low
// mantissa bits, and the constant's low word is 0, so only the high word needs the subtraction.
__device__ __forceinline__ unsigned long long fixed_i64(float x) {
  const double d = (double)x + 6755399441055744.0;
  const unsigned long long b = (unsigned long long)__double_as_longlong(d);
  return b - 0x4338000000000000ull;
}

#ifndef LNR_ACCUM_WAVES_PER_EU
#define LNR_ACCUM_WAVES_PER_EU 8
#endif
#ifndef LNR_ACCUM_LOADS
#define LNR_ACCUM_LOADS 2
#endif
__global__ void __launch_bounds__(kAccumThreads, LNR_ACCUM_WAVES_PER_EU) k_bwd_accum(GridArgs a, BwdWorkspace ws, float* __restrict__ d_table,
                                                                                        uint32_t b_begin, uint32_t b_end) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem);  // [2][kChunk] int64 fixed point
  // (one array per feature: 8-B atomics on random entries spread over twice the bank pairs)
  const uint32_t nbk = a.n_buckets;
  const uint32_t s_end = ws.slice_pre[b_end];  // work items of buckets [b_begin, b_end)
  const int lane = threadIdx.x & 63;
  for (uint32_t s = ws.slice_pre[b_begin] + blockIdx.x; s < s_end; s += gridDim.x) {
    uint32_t lo = 0, hi = nbk;  // bucket b with slice_pre[b] <= s < slice_pre[b+1]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (ws.slice_pre[mid] <= s) lo = mid;
      else hi = mid;
    }
    const uint32_t b = lo;
    const uint32_t nsl = ws.slice_pre[b + 1] - ws.slice_pre[b];
    const uint32_t j = s - ws.slice_pre[b];
    const uint64_t slr = b < a.bucket_base[a.merge_levels] ? kSliceRecordsCoarse : kSliceRecords;
    const uint64_t beg = ws.seg_start[b] + (uint64_t)j * slr;
    uint64_t end = ws.seg_start[b + 1];
    if (beg + slr < end) end = beg + slr;
    uint32_t l = 0;
    while (l + 1 < a.n_levels && a.bucket_base[l + 1] <= b) ++l;
    const uint32_t chunk = b - a.bucket_base[l];
    const uint32_t ent0 = chunk * kChunk;
    const uint32_t nent = (a.lv[l].size - ent0) < (uint32_t)kChunk ? (a.lv[l].size - ent0) : (uint32_t)kChunk;
    const int k2 = bucket_k2(ws, l, b);  // one scale per bucket: split buckets' partials add exactly
    const float scale = ldexpf(1.f, k2);
    LNR_STAMP(t0);
    for (int t = threadIdx.x; t < 2 * kChunk; t += blockDim.x) acc[t] = 0ull;
    lds_barrier();
    LNR_STAMP(t1);
    // 2 records per lane per load (8-B words, 16-B fp32 value pairs), LNR_ACCUM_LOADS loads in flight;
    // a pair record (p > 0) adds (1 - tx) v to corner e0 and tx v to e1 = e0 ^ (2^p - 1), a single
    // record (p = 0, tx = 0) adds v to e0.  int64 sums: the result does not depend on the order.
    const uint64_t beg2 = beg & ~1ull;
    for (uint64_t rb = beg2 + 2 * (threadIdx.x & ~63u); rb < end; rb += 2 * LNR_ACCUM_LOADS * kAccumThreads) {
      uint2 qw[LNR_ACCUM_LOADS];
      float4 qv[LNR_ACCUM_LOADS];
#pragma unroll
      for (int u = 0; u < LNR_ACCUM_LOADS; ++u) {
        const uint64_t rr = rb + 2 * lane + (uint64_t)u * 2 * kAccumThreads;
        const uint64_t rc = rr < end ? rr : beg2;  // unconditional loads: no branch to wait at
        const u32x2 w2 = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(&ws.rec_w[rc]));
        const f32x4 v4 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(&ws.rec_v[rc]));
        qv[u] = make_float4(v4.x, v4.y, v4.z, v4.w);
        qw[u] = make_uint2(rr < beg || rr >= end ? kRecNone : w2.x, rr + 1 >= end ? kRecNone : w2.y);
      }
#pragma unroll
      for (int u = 0; u < 2 * LNR_ACCUM_LOADS; ++u) {
        const uint32_t w = (u & 1) ? qw[u >> 1].y : qw[u >> 1].x;
        if (w != kRecNone) {
          const float v0 = ((u & 1) ? qv[u >> 1].z : qv[u >> 1].x) * scale;
          const float v1 = ((u & 1) ? qv[u >> 1].w : qv[u >> 1].y) * scale;
          const uint32_t e0 = w & (kChunk - 1);
          const uint32_t p = (w >> kChunkLog2) & 15u;
          const float tx = (float)(w >> 16) * kInvU16;  // 0 for single-corner records
          const float s0 = 1.0f - tx;
          atomicAdd(&acc[e0], fixed_i64(s0 * v0));
          atomicAdd(&acc[kChunk + e0], fixed_i64(s0 * v1));
          if (p) {
            const uint32_t e1 = e0 ^ ((1u << p) - 1u);
            atomicAdd(&acc[e1], fixed_i64(tx * v0));
            atomicAdd(&acc[kChunk + e1], fixed_i64(tx * v1));
          }
        }
      }
    }
    LNR_STAMP(t2);
    lds_barrier();
    LNR_STAMP(t3);
    if (nsl == 1) {  // the final values
      const float inv = ldexpf(1.f, -k2);
      float* dst = d_table + 2 * ((int64_t)a.lv[l].offset + ent0);
      for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x)
        dst[t] = (float)(long long)acc[(t & 1) * kChunk + (t >> 1)] * inv;
    } else {  // this slice's int64 partial chunk
      long long* dst = ws.partial + (int64_t)(ws.part_pre[b] + j) * (2 * kChunk);
      for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x) dst[t] = (long long)acc[(t & 1) * kChunk + (t >> 1)];
    }
    lds_barrier();
    LNR_STAMP(t4);
    LNR_PHASE(16, t1, t0);
    LNR_PHASE(17, t2, t1);
    LNR_PHASE(18, t3, t2);
    LNR_PHASE(19, t4, t3);
    LNR_PHASE(20, 1ull, 0ull);
    LNR_PHASE(21, end - beg, 0ull);
  }
}

// Split buckets: d_table = sum of the slices' partial chunks, in slice order (deterministic).
__global__ void __launch_bounds__(256) k_bwd_finalize(GridArgs a, BwdWorkspace ws, float* __restrict__ d_table,
                                                      uint32_t b_begin) {
  const uint32_t b = b_begin + blockIdx.x;
  const uint32_t nsl = ws.part_pre[b + 1] - ws.part_pre[b];
  if (nsl == 0) return;
  uint32_t l = 0;
  while (l + 1 < a.n_levels && a.bucket_base[l + 1] <= b) ++l;
  const uint32_t ent0 = (b - a.bucket_base[l]) * kChunk;
  const uint32_t nent = (a.lv[l].size - ent0) < (uint32_t)kChunk ? (a.lv[l].size - ent0) : (uint32_t)kChunk;
  const float inv = ldexpf(1.f, -bucket_k2(ws, l, b));  // the accumulate kernel's per-bucket scale
  const long long* src = ws.partial + (int64_t)ws.part_pre[b] * (2 * kChunk);
  float* dst = d_table + 2 * ((int64_t)a.lv[l].offset + ent0);
  for (uint32_t t = threadIdx.x; t < 2 * nent; t += blockDim.x) {
    long long v = 0;
    for (uint32_t k = 0; k < nsl; ++k) v += src[(int64_t)k * (2 * kChunk) + t];
    dst[t] = (float)v * inv;
  }
}

// Accumulate + finalize the buckets of levels [l0, l1): their slice of d_table becomes final.
static void launch_accum(const GridArgs& a, const BwdWorkspace& w, const lnr_grid_desc* d, int64_t n, uint32_t l0,
                         uint32_t l1, float* d_table, hipStream_t st) {
  const uint32_t b0 = a.bucket_base[l0], b1 = a.bucket_base[l1];
  if (b1 <= b0) return;
  const int64_t max_slices = (b1 - b0) + (8 * n * (int64_t)(l1 - l0)) / kSliceRecordsCoarse + 1;
  const unsigned g = (unsigned)(max_slices < 4096 ? max_slices : 4096);
  hipLaunchKernelGGL(k_bwd_accum, dim3(g), dim3(kAccumThreads), 2 * kChunk * sizeof(unsigned long long), st, a, w,
                     d_table, b0, b1);
  hipLaunchKernelGGL(k_bwd_finalize, dim3(b1 - b0), dim3(256), 0, st, a, w, d_table, b0);
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
  dim3 grid((unsigned)w.n_sb, d->n_levels);
  const bool skip_zero = !(flags & LNR_BWD_COUNTS_READY);
  if (!(flags & LNR_BWD_COUNTS_READY)) {
    hipLaunchKernelGGL(k_bwd_count<PosFn>, grid, dim3(kSB), 0, st, a, pos, n, reinterpret_cast<const float2*>(d_enc),
                       stride, w);
  }
  hipLaunchKernelGGL(k_bwd_chunk_sums, dim3((unsigned)w.n_chunks, d->n_levels), dim3(kMaxChunksPerLevel), 0, st, a, w);
  hipLaunchKernelGGL(k_bwd_scan_rows, dim3((unsigned)w.n_chunks, d->n_levels), dim3(kMaxChunksPerLevel), 0, st, a, w);
  hipLaunchKernelGGL(k_bwd_scan_buckets, dim3(1), dim3(1024), 0, st, w, a.n_buckets, a.bucket_base[a.merge_levels]);
  {
    const float2* de = reinterpret_cast<const float2*>(d_enc);
    const uint32_t m = a.merge_levels, L = d->n_levels;
    bool all_fine = true;
    for (uint32_t l = m; l < L; ++l) all_fine = all_fine && a.lv[l].fine;
#if !defined(LNR_EXP_SPLIT_SCATTER) && !defined(LNR_EXP_SCATTER_PER_LEVEL)
    uint32_t maxnb = 0;
    for (uint32_t l = 0; l < L; ++l) maxnb = std::max(maxnb, a.bucket_base[l + 1] - a.bucket_base[l]);
    // the reference's grids: 16 levels (base 16, scale 2), 2^18 (sigma) or 2^19 (colour) entries
    bool pow2 = true;
    for (uint32_t l = 0; l < L; ++l) pow2 = pow2 && a.lv[l].size_mask != 0;
    const bool rows = L == 16 && all_fine && pow2 && 8 * n * (int64_t)L + 2 < (int64_t(1) << 32);
    if (rows && m == 5 && maxnb <= 64) {
      hipLaunchKernelGGL((k_bwd_scatter_rows<PosFn, 16, 5, 64>), dim3((unsigned)w.n_sb), dim3(kSB), 0, st, a, pos, n,
                         de, stride, w, skip_zero);
      hipLaunchKernelGGL((k_bwd_scatter_overflow<PosFn>), dim3((unsigned)((w.n_sb * L + kSB - 1) / kSB)), dim3(kSB),
                         kScatterLds, st, a, pos, n, de, stride, w, skip_zero);
    } else
      hipLaunchKernelGGL((k_bwd_scatter<PosFn, kLevelsAny>), dim3((unsigned)(w.n_sb * L)), dim3(kSB), kScatterLds, st,
                         a, pos, n, de, stride, w, 0u, skip_zero);
#elif defined(LNR_EXP_SCATTER_PER_LEVEL)
    (void)m;
    (void)all_fine;
    hipLaunchKernelGGL((k_bwd_scatter<PosFn, kLevelsAny>), dim3((unsigned)(w.n_sb * L)), dim3(kSB), kScatterLds, st, a,
                       pos, n, de, stride, w, 0u, skip_zero);
#else
    if (m > 0)
      hipLaunchKernelGGL((k_bwd_scatter<PosFn, kLevelsCoherent>), dim3((unsigned)w.n_sb, m), dim3(kSB), kScatterLds, st,
                         a, pos, n, de, stride, w, 0u, skip_zero);
    if (L > m) {
      if (all_fine)
        hipLaunchKernelGGL((k_bwd_scatter<PosFn, kLevelsFine>), dim3((unsigned)w.n_sb, L - m), dim3(kSB), kScatterLds,
                           st, a, pos, n, de, stride, w, m, skip_zero);
      else
        hipLaunchKernelGGL((k_bwd_scatter<PosFn, kLevelsGeneric>), dim3((unsigned)w.n_sb, L - m), dim3(kSB),
                           kScatterLds, st, a, pos, n, de, stride, w, m, skip_zero);
    }
#endif
  }
  hipLaunchKernelGGL(k_bwd_level_max, dim3(d->n_levels), dim3(256), 0, st, w);
  if (flags & LNR_BWD_NO_ACCUM) LNR_RETURN_LAUNCH(who);  // accumulate later, by level range
  launch_accum(a, w, d, n, 0, d->n_levels, d_table, st);
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

extern "C" int lnr_hashgrid_bwd_accum(const lnr_grid_desc* d, int64_t n, void* workspace, int64_t workspace_bytes,
                                      uint32_t level_begin, uint32_t level_end, float* d_table, void* stream) {
  if (int e = check_desc_bwd(d, "lnr_hashgrid_bwd_accum")) return e;
  LNR_REQUIRE(level_begin <= level_end && level_end <= d->n_levels, "lnr_hashgrid_bwd_accum: bad level range");
  LNR_REQUIRE(n >= 0 && workspace && workspace_bytes >= bwd_workspace_bytes(d, n) && d_table,
              "lnr_hashgrid_bwd_accum: bad workspace / pointers");
  if (n == 0) return LNR_OK;
  const GridArgs a = make_args(d);
  launch_accum(a, carve_workspace(workspace, a, d, n), d, n, level_begin, level_end, d_table, as_stream(stream));
  LNR_RETURN_LAUNCH("lnr_hashgrid_bwd_accum");
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

LNR_PHASE_EXPORT(hashgrid_bwd)
