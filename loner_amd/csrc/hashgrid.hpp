// Shared definitions of the multi-resolution hash grid (tiny-cuda-nn v1.7 HashGrid semantics):
// level layout, corner indexing, sample positions, and the backward's bucket geometry.
#pragma once
#include "common.hpp"
#include <cstdlib>

namespace lnr {

struct LevelParams {
  float scale;
  uint32_t res;
  uint32_t size;
  uint32_t size_mask;  // size - 1 when size is a power of two, else 0
  uint32_t offset;
  uint32_t hashed;     // stride walk exceeded size -> coherent prime hash
  uint32_t fine;       // hashed, power-of-two size, not coherent: FineCell fast path
};

// Backward buckets: each level's table slice is cut into chunks of 2^kChunkLog2 entries; one
// chunk is one LDS accumulator of 4096 entries x 2 features x int64 fixed point = 64 KB.
constexpr int kChunkLog2 = 12;
constexpr int kChunk = 1 << kChunkLog2;
constexpr int kMaxChunksPerLevel = 128;
constexpr int kMaxBuckets = 2048;
// The accumulation splits the records of a bucket range evenly over kAccumGroups workgroups (two
// 64 KB-LDS workgroups per CU of the 256): each walks its own record range bucket by bucket, so
// every CU does the same work whatever the bucket sizes.  A bucket cut by a range boundary leaves an
// int64 partial chunk per piece (at most two per workgroup), added exactly by the last piece's
// workgroup to arrive (or by k_bwd_finalize).
constexpr int kAccumGroups = 512;
// Unit accumulation (k_bwd_accum_units, mid-size batches): each bucket is one work unit when it holds at
// most T = max(R / kAccumGroups, one tile) records, else ceil(n / T) equal pieces.  Only the large
// buckets (the coarse levels' few chunks) leave partial chunks, and a finalize workgroup per such
// bucket adds them.  Sum of the pieces <= kMaxBuckets + kAccumGroups; cut buckets < kAccumGroups;
// their pieces <= 2 kAccumGroups (the partial chunks).
constexpr int kMaxUnits = kMaxBuckets + kAccumGroups;
struct UnitTable {
  uint32_t n_units, n_cut, pad0, pad1;
  uint2 unit[kMaxUnits];       // {bucket, piece << 16 | pieces}, bucket order
  uint32_t slot[kMaxBuckets];  // a cut bucket's first partial chunk
  uint2 cut[kAccumGroups];     // {bucket, pieces} of the cut buckets, bucket order
};

// Adam applied where the backward finishes a table entry's gradient (lnr_hashgrid_bwd_rays_jac_adam):
// the same arithmetic as k_adam on the table's slice of the flat parameters, so the gradient never
// goes to memory.  p == nullptr: the backward stores the gradient into d_table instead.
struct AdamEpi {
  float* p;
  uint16_t* shadow;
  float* m;
  float* v;
  const lnr_step_scalars* dev_step;  // graph replay: step_size and bc2_sqrt from device memory
  float one_minus_b1, b2, one_minus_b2, step_size, bc2_sqrt, eps;
};

struct GridArgs {
  AdamEpi adam;
  LevelParams lv[LNR_MAX_LEVELS];
  uint32_t bucket_base[LNR_MAX_LEVELS + 1];
  uint32_t n_levels;
  uint32_t n_buckets;
  uint32_t merge_levels;  // levels [0, merge_levels) merge equal corner indices across lanes
};

// Levels whose cell edge spans several consecutive samples of a ray produce runs of equal corner
// indices.  At the reference's 512 samples per ray (after the OGM has concentrated them) that holds
// up to resolution 512; the sample density along a ray scales with the samples
// per ray, so the bound does too (C1's 64 samples: resolution <= 64).  Positions not from rays: 512.
#ifndef LNR_MERGE_MAX_RES
#define LNR_MERGE_MAX_RES 512
#endif
inline uint32_t merge_levels_for(const lnr_grid_desc* d, int32_t samples_per_ray = 0) {
  const int64_t max_res = samples_per_ray > 0 ? (int64_t)LNR_MERGE_MAX_RES * samples_per_ray / 512 : LNR_MERGE_MAX_RES;
  uint32_t m = 0;
  for (uint32_t l = 0; l < d->n_levels; ++l)
    if ((int64_t)d->resolution[l] <= max_res) m = l + 1;
  return m;
}

inline GridArgs make_args(const lnr_grid_desc* d, int32_t samples_per_ray = 0) {
  GridArgs a{};
  a.n_levels = d->n_levels;
  for (uint32_t l = 0; l < d->n_levels; ++l) {
    LevelParams& p = a.lv[l];
    p.scale = d->scale[l];
    p.res = d->resolution[l];
    p.size = d->size[l];
    p.size_mask = (p.size & (p.size - 1)) == 0 ? p.size - 1 : 0;
    p.offset = d->offset[l];
    // grid_index: dense stride walk while stride <= size; hashed iff final stride > size
    uint64_t stride = 1;
    for (int dim = 0; dim < 3 && stride <= p.size; ++dim) stride *= p.res;
    p.hashed = stride > p.size ? 1u : 0u;
  }
  uint32_t b = 0;
  for (uint32_t l = 0; l < d->n_levels; ++l) {
    a.bucket_base[l] = b;
    b += (d->size[l] + kChunk - 1) / kChunk;
  }
  a.bucket_base[d->n_levels] = b;
  a.n_buckets = b;
  a.merge_levels = merge_levels_for(d, samples_per_ray);
  for (uint32_t l = 0; l < d->n_levels; ++l)
    a.lv[l].fine = (a.lv[l].hashed && a.lv[l].size_mask && l >= a.merge_levels) ? 1u : 0u;
  return a;
}

__device__ __forceinline__ uint32_t grid_index(const LevelParams& p, uint32_t x, uint32_t y, uint32_t z) {
  uint32_t idx;
  if (p.hashed) {
    idx = x ^ (y * 2654435761u) ^ (z * 805459861u);
  } else {
    idx = x + y * p.res + z * p.res * p.res;
  }
  return p.size_mask ? (idx & p.size_mask) : (idx % p.size);
}

// Sample position in [0,1]^3.  From rays: xyz = o + d*z (rendering_tcnn.py:390), pos = (xyz+1)/2
// (nerf_tcnn.py:63); compiled with -ffp-contract=off so the op order matches torch.
// load() issues the global loads, eval() does the arithmetic: kernels that must not wait for the
// loads before a barrier call them on either side of it.
struct PosFromArray {
  const float* pos;
  int32_t samples_per_ray() const { return 0; }  // not from rays
  struct Raw {
    float x, y, z;
  };
  __device__ __forceinline__ Raw load(int64_t n) const { return {pos[3 * n + 0], pos[3 * n + 1], pos[3 * n + 2]}; }
  __device__ __forceinline__ void eval(const Raw& r, float& x, float& y, float& z) const {
    x = r.x;
    y = r.y;
    z = r.z;
  }
  __device__ __forceinline__ void operator()(int64_t n, float& x, float& y, float& z) const { eval(load(n), x, y, z); }
  // (the same for a wave's 64 consecutive samples; see PosFromRays)
  __device__ __forceinline__ void wave(int64_t n, int64_t n_total, bool in, float& x, float& y, float& z) const {
    if (in) (*this)(n, x, y, z);
  }
};
struct PosFromRays {
  const float* rays;
  const float* zs;
  int32_t n_samples;
  int32_t samples_per_ray() const { return n_samples; }
  struct Raw {
    float ox, oy, oz, dx, dy, dz, t;
  };
  __device__ __forceinline__ Raw load(int64_t n) const {
    const uint32_t r = (uint32_t)n / (uint32_t)n_samples;  // N < 2^31 (checked at the C ABI)
    const float* ry = rays + 13 * r;
    return {ry[0], ry[1], ry[2], ry[3], ry[4], ry[5], zs[n]};
  }
  __device__ __forceinline__ void eval(const Raw& r, float& x, float& y, float& z) const {
    x = (r.ox + r.dx * r.t + 1.0f) * 0.5f;
    y = (r.oy + r.dy * r.t + 1.0f) * 0.5f;
    z = (r.oz + r.dz * r.t + 1.0f) * 0.5f;
  }
  __device__ __forceinline__ void operator()(int64_t n, float& x, float& y, float& z) const { eval(load(n), x, y, z); }
  // A wave's 64 consecutive samples (wave-aligned, n_samples % 64 == 0) all lie on one ray: its origin
  // and direction are wave-uniform, loaded once through the scalar cache instead of by every lane
  // through the vector memory path (two fewer VMEM instructions per wave and level in the encode).
  // Lanes past n_total evaluate the last ray's (the wave's first lane may be past it too).
  __device__ __forceinline__ void wave(int64_t n, int64_t n_total, bool in, float& x, float& y, float& z) const {
    if ((n_samples & 63) != 0) {
      if (in) (*this)(n, x, y, z);
      return;
    }
    const int64_t first = n < n_total ? n : n_total - 1;
    const uint32_t r = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)first / (uint32_t)n_samples));
    const float* ry = rays + 13 * (int64_t)r;
    Raw q{ry[0], ry[1], ry[2], ry[3], ry[4], ry[5], in ? zs[n] : 0.f};
    eval(q, x, y, z);
    if (!in) x = y = z = 0.f;
  }
};

// Encoding gradient sources of the backward.  GradF32: d_enc itself, level-major float2.  GradJac:
// d_enc = d_sigma * J with J = d sigma / d enc, the sigma MLP's input Jacobian, level-major fp16
// pairs (lnr_field_train's compact output: 4 B per sample and level instead of 8, and d_sigma 4 B
// per sample).  load_nt: read once (nontemporal).
typedef float gf32x2 __attribute__((ext_vector_type(2)));
// live_at(i): whether sample i may emit records at the fine levels.  GradF32's optional ``live`` mask (the
// colour grid's compositing weights: a sample of weight exactly 0 has d_enc = 0) makes the scatter skip by
// the mask, the criterion of a forward that counted the histogram with it (lnr_hashgrid_fwd_rays_live_ws);
// without one every sample may.
struct GradF32 {
  static constexpr bool kScaled = false;  // no per-sample scale: scale() is not dL/dsigma
  const float2* g;
  int64_t stride;
  const float* live = nullptr;
  __device__ __forceinline__ bool live_at(int64_t i) const { return live == nullptr || live[i] != 0.f; }
  __device__ __forceinline__ float2 load(uint32_t l, int64_t i) const { return g[(int64_t)l * stride + i]; }
  __device__ __forceinline__ float2 load_nt(uint32_t l, int64_t i) const {
    const gf32x2 v = __builtin_nontemporal_load(reinterpret_cast<const gf32x2*>(&g[(int64_t)l * stride + i]));
    return make_float2(v.x, v.y);
  }
  // the split form (GradJac holds half the registers this way): per-level raw value + per-sample scale
  typedef float2 Raw;
  __device__ __forceinline__ Raw load_raw_nt(uint32_t l, int64_t i) const { return load_nt(l, i); }
  __device__ __forceinline__ float scale(int64_t) const { return 0.f; }
  __device__ __forceinline__ static float2 finish(const Raw& r, float) { return r; }
};
// A sample with dL/dsigma = 0 (relu(sigma + noise) = 0: alpha = 1 - exp(-delta relu(sigma + n)),
// rendering_tcnn.py:252,260) has d_enc = 0 exactly, and its J is not written: the MLP backward skips the
// 32-sample tile pairs whose d sigma are all 0 (k_mlp_bwd_tiles), so apply() returns 0 for s = 0 instead of
// reading a stale J.
struct GradJac {
  static constexpr bool kScaled = true;  // scale(i) = dL/dsigma of sample i
  const uint32_t* jac;
  const float* dsig;
  int64_t stride;
  __device__ __forceinline__ static constexpr bool live_at(int64_t) { return true; }
  __device__ __forceinline__ static float2 apply(uint32_t h, float s) {
    if (s == 0.f) return make_float2(0.f, 0.f);
    return make_float2((float)__builtin_bit_cast(_Float16, (uint16_t)(h & 0xFFFFu)) * s,
                       (float)__builtin_bit_cast(_Float16, (uint16_t)(h >> 16)) * s);
  }
  __device__ __forceinline__ float2 load(uint32_t l, int64_t i) const { return apply(jac[(int64_t)l * stride + i], dsig[i]); }
  __device__ __forceinline__ float2 load_nt(uint32_t l, int64_t i) const {
    return apply(__builtin_nontemporal_load(&jac[(int64_t)l * stride + i]), dsig[i]);
  }
  typedef uint32_t Raw;
  __device__ __forceinline__ Raw load_raw_nt(uint32_t l, int64_t i) const {
    return __builtin_nontemporal_load(&jac[(int64_t)l * stride + i]);
  }
  __device__ __forceinline__ float scale(int64_t i) const { return dsig[i]; }
  __device__ __forceinline__ static float2 finish(const Raw& r, float s) { return apply(r, s); }
};

struct Corners {
  uint32_t idx[8];
  float w[8];
  float tx, ty, tz;     // cell fractions (the backward's x-pair records split by tx)
  uint32_t cx, cy, cz;  // the cell (coherent levels merge runs of lanes in one cell)
};

// POW2: the caller guarantees a power-of-two table size (size_mask != 0), so no modulo path.
template <bool POW2 = false>
__device__ __forceinline__ void level_corners(const LevelParams& p, float x, float y, float z, Corners& c) {
  // tcnn pos_fract: pos = fmaf(scale, x, 0.5); cell = floor(pos); frac = pos - cell
  float px = fmaf(p.scale, x, 0.5f), py = fmaf(p.scale, y, 0.5f), pz = fmaf(p.scale, z, 0.5f);
  float fx = floorf(px), fy = floorf(py), fz = floorf(pz);
  uint32_t cx = (uint32_t)(int)fx, cy = (uint32_t)(int)fy, cz = (uint32_t)(int)fz;
  float tx = px - fx, ty = py - fy, tz = pz - fz;
  c.cx = cx;
  c.cy = cy;
  c.cz = cz;
  c.tx = tx;
  c.ty = ty;
  c.tz = tz;
  // grid_index per corner from per-axis terms formed once: the hash XORs x with y*P1 and z*P2, the
  // dense walk adds x, y*res and z*res^2 (same values as grid_index, fewer multiplies)
  uint32_t ty0, ty1, tz0, tz1;
  if (p.hashed) {
    ty0 = cy * 2654435761u;
    tz0 = cz * 805459861u;
    ty1 = ty0 + 2654435761u;
    tz1 = tz0 + 805459861u;
  } else {
    const uint32_t r2 = p.res * p.res;
    ty0 = cy * p.res;
    tz0 = cz * r2;
    ty1 = ty0 + p.res;
    tz1 = tz0 + r2;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int bx = k & 1, by = (k >> 1) & 1, bz = (k >> 2) & 1;
    float w = bx ? tx : 1.0f - tx;
    w *= by ? ty : 1.0f - ty;
    w *= bz ? tz : 1.0f - tz;
    c.w[k] = w;
    const uint32_t xx = cx + bx, yy = by ? ty1 : ty0, zz = bz ? tz1 : tz0;
    const uint32_t idx = p.hashed ? (xx ^ yy ^ zz) : (xx + yy + zz);
    c.idx[k] = p.offset + ((POW2 || p.size_mask) ? (idx & p.size_mask) : (idx % p.size));
  }
}

// Hashed levels with a power-of-two table (every level finer than 256^3 cells when log2 T <= 24).
// The cell's four y/z edges share the x-neighbour mask: corner 2j+1 = corner 2j ^ d with
// d = (x ^ (x + 1)) & (size - 1), a mask of the form 2^p - 1.  Entries are relative to the level
// offset; the y/z prime products are formed once per cell.
struct FineCell {
  uint32_t e[4];  // entry of corner 2j (bx = 0, by = j & 1, bz = j >> 1)
  uint32_t d;     // x-pair mask
  float tx, ty, tz;
};
__device__ __forceinline__ void fine_cell(const LevelParams& p, float x, float y, float z, FineCell& c) {
  const float px = fmaf(p.scale, x, 0.5f), py = fmaf(p.scale, y, 0.5f), pz = fmaf(p.scale, z, 0.5f);
  const float fx = floorf(px), fy = floorf(py), fz = floorf(pz);
  const uint32_t cx = (uint32_t)(int)fx, cy = (uint32_t)(int)fy, cz = (uint32_t)(int)fz;
  c.tx = px - fx;
  c.ty = py - fy;
  c.tz = pz - fz;
  const uint32_t hy0 = cy * 2654435761u, hy1 = (cy + 1u) * 2654435761u;
  const uint32_t hz0 = cz * 805459861u, hz1 = (cz + 1u) * 805459861u;
  const uint32_t m = p.size_mask;
  c.e[0] = (cx ^ hy0 ^ hz0) & m;
  c.e[1] = (cx ^ hy1 ^ hz0) & m;
  c.e[2] = (cx ^ hy0 ^ hz1) & m;
  c.e[3] = (cx ^ hy1 ^ hz1) & m;
  c.d = (cx ^ (cx + 1u)) & m;
}
// level_corners' weight of corner k = 2j + bx: ((wx * wy) * wz), same rounding
__device__ __forceinline__ float fine_weight(const FineCell& c, int j, int bx) {
  float w = bx ? c.tx : 1.0f - c.tx;
  w *= (j & 1) ? c.ty : 1.0f - c.ty;
  w *= (j & 2) ? c.tz : 1.0f - c.tz;
  return w;
}

// Runs of equal keys across consecutive lanes: head/tail flags and the lane of the run head.
struct RunInfo {
  unsigned long long heads;
  int head_lane;
  bool tail;
};
__device__ __forceinline__ RunInfo lane_runs(uint32_t key) {
  const int lane = threadIdx.x & 63;
  const uint32_t prev = __shfl_up(key, 1, 64);
  const bool head = (lane == 0) || (prev != key);
  RunInfo ri;
  ri.heads = __ballot(head);
  ri.head_lane = 63 - __clzll(ri.heads & ((2ull << lane) - 1ull));
  ri.tail = (lane == 63) || ((ri.heads >> (lane + 1)) & 1ull);
  return ri;
}
// Segmented inclusive sum: the tail lane of each run ends with the run total.
__device__ __forceinline__ void run_sum(const RunInfo& ri, float& v0, float& v1) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float q0 = __shfl_up(v0, o, 64), q1 = __shfl_up(v1, o, 64);
    if (lane - o >= ri.head_lane) {
      v0 += q0;
      v1 += q1;
    }
  }
}

// DPP forms of the above (gfx9 DPP: row_shr within 16-lane rows, row_bcast across rows): VALU
// data movement instead of ds_bpermute round trips through the LDS unit.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}
__device__ __forceinline__ RunInfo lane_runs_dpp(uint32_t key) {
  const int lane = threadIdx.x & 63;
  // wave_shr:1 (0x138): lane i reads lane i - 1; lane 0 keeps the "old" operand (~key: a head)
  const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)~key, (int)key, 0x138, 0xF, 0xF, false);
  const bool head = (lane == 0) || (prev != key);
  RunInfo ri;
  ri.heads = __ballot(head);
  ri.head_lane = 63 - __clzll(ri.heads & ((2ull << lane) - 1ull));
  ri.tail = (lane == 63) || ((ri.heads >> (lane + 1)) & 1ull);
  return ri;
}
// Segmented inclusive sum over runs (head_lane per lane): within-row shifts, then row 15 / 31
// broadcasts, each added only where the run reaches back that far.
__device__ __forceinline__ void run_sum_dpp(const RunInfo& ri, float& v0, float& v1) {
  const int lane = threadIdx.x & 63;
  const int h = ri.head_lane;
#define LNR_SEG_STEP(CTRL, RMASK, COND)        \
  {                                           \
    const float q0 = dpp_f32<CTRL, RMASK>(v0); \
    const float q1 = dpp_f32<CTRL, RMASK>(v1); \
    if (COND) {                               \
      v0 += q0;                               \
      v1 += q1;                               \
    }                                         \
  }
  LNR_SEG_STEP(0x111, 0xF, lane - 1 >= h)                        // row_shr:1
  LNR_SEG_STEP(0x112, 0xF, lane - 2 >= h)                        // row_shr:2
  LNR_SEG_STEP(0x114, 0xF, lane - 4 >= h)                        // row_shr:4
  LNR_SEG_STEP(0x118, 0xF, lane - 8 >= h)                        // row_shr:8
  LNR_SEG_STEP(0x142, 0xA, (lane & 16) && h < (lane & ~15))      // row_bcast:15 -> rows 1, 3
  LNR_SEG_STEP(0x143, 0xC, lane >= 32 && h < 32)                 // row_bcast:31 -> rows 2, 3
#undef LNR_SEG_STEP
}

// Runs of consecutive lanes in one cell (coherent levels: consecutive samples of a ray): every
// corner index of such lanes is equal, so one run detection serves all 8 corners.  Lanes without a
// sample (in = false) are runs of their own.
__device__ __forceinline__ RunInfo cell_runs_dpp(bool in, uint32_t cx, uint32_t cy, uint32_t cz) {
  const int lane = threadIdx.x & 63;
  // wave_shr:1 (0x138): lane i reads lane i - 1 (lane 0 keeps "old", and is a head anyway)
  const uint32_t px = (uint32_t)__builtin_amdgcn_update_dpp((int)~cx, (int)cx, 0x138, 0xF, 0xF, false);
  const uint32_t py = (uint32_t)__builtin_amdgcn_update_dpp((int)~cy, (int)cy, 0x138, 0xF, 0xF, false);
  const uint32_t pz = (uint32_t)__builtin_amdgcn_update_dpp((int)~cz, (int)cz, 0x138, 0xF, 0xF, false);
  const int pin = __builtin_amdgcn_update_dpp(0, in ? 1 : 0, 0x138, 0xF, 0xF, false);
  const bool head = (lane == 0) || !in || !pin || px != cx || py != cy || pz != cz;
  RunInfo ri;
  ri.heads = __ballot(head);
  ri.head_lane = 63 - __clzll(ri.heads & ((2ull << lane) - 1ull));
  ri.tail = (lane == 63) || ((ri.heads >> (lane + 1)) & 1ull);
  return ri;
}

// One step of a segmented sum as ONE instruction per value: v += dpp(v) * f, with f = 1.0 where this
// lane's run reaches back over the shift and 0.0 elsewhere (v_fmac_f32 with a DPP source operand;
// the compiler does not fold a DPP move into fmac, so it is written out).  x * 1.0 is exact, so each
// add rounds exactly as the conditional add it replaces; where f = 0 the value is unchanged (up to
// the sign of a zero).  Every row enabled and bound_ctrl: a source lane outside the shift reads 0.
// The leading s_nop 1 covers the DPP source hazard (2 wait states after a VALU write of the source,
// e.g. a copy the compiler places before the block); inside the block value k is last written 16
// instructions back.
#define LNR_FMAC_DPP_16(DPP, v, f)                                                                        \
  asm volatile(                                                                                          \
      "s_nop 1\n\t"                                                                                      \
      "v_fmac_f32_dpp %0, %0, %16 " DPP "\n\tv_fmac_f32_dpp %1, %1, %16 " DPP "\n\t"                    \
      "v_fmac_f32_dpp %2, %2, %16 " DPP "\n\tv_fmac_f32_dpp %3, %3, %16 " DPP "\n\t"                    \
      "v_fmac_f32_dpp %4, %4, %16 " DPP "\n\tv_fmac_f32_dpp %5, %5, %16 " DPP "\n\t"                    \
      "v_fmac_f32_dpp %6, %6, %16 " DPP "\n\tv_fmac_f32_dpp %7, %7, %16 " DPP "\n\t"                    \
      "v_fmac_f32_dpp %8, %8, %16 " DPP "\n\tv_fmac_f32_dpp %9, %9, %16 " DPP "\n\t"                    \
      "v_fmac_f32_dpp %10, %10, %16 " DPP "\n\tv_fmac_f32_dpp %11, %11, %16 " DPP "\n\t"                \
      "v_fmac_f32_dpp %12, %12, %16 " DPP "\n\tv_fmac_f32_dpp %13, %13, %16 " DPP "\n\t"                \
      "v_fmac_f32_dpp %14, %14, %16 " DPP "\n\tv_fmac_f32_dpp %15, %15, %16 " DPP                       \
      : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]), \
        "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]),        \
        "+v"(v[15])                                                                                      \
      : "v"(f))
#ifndef LNR_SEG_FMAC
#define LNR_SEG_FMAC 1  // the segmented sums as v_fmac_f32_dpp (1) or DPP move + masked add (0)
#endif

// Segmented inclusive sum of N values over runs sharing one RunInfo: the run's tail lane ends with
// the run totals.  Each step's lane condition is computed once for all N values.  Fixed order:
// deterministic.  N = 16 (the coherent levels' 8 corners x 2 features) takes every step as one
// v_fmac_f32_dpp per value; otherwise each step is a DPP move and a masked add per value, and only
// the steps the wave's runs need are taken: row shifts up to the longest within-row run prefix, the
// row broadcasts only when a run crosses a 16-lane row boundary.
template <int N>
__device__ __forceinline__ void run_sum_dpp_n(const RunInfo& ri, float (&v)[N]) {
  const int lane = threadIdx.x & 63;
  const int h = ri.head_lane;
  const int rs = lane & ~15;
  if constexpr (LNR_SEG_FMAC && N == 16) {
    // (branching around a step would cost the register copies the compiler places at the joins; a
    // step no run needs multiplies by 0 everywhere)
    LNR_FMAC_DPP_16("row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1", v, (lane - 1 >= h) ? 1.f : 0.f);
    LNR_FMAC_DPP_16("row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1", v, (lane - 2 >= h) ? 1.f : 0.f);
    LNR_FMAC_DPP_16("row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1", v, (lane - 4 >= h) ? 1.f : 0.f);
    LNR_FMAC_DPP_16("row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1", v, (lane - 8 >= h) ? 1.f : 0.f);
    LNR_FMAC_DPP_16("row_bcast:15 row_mask:0xf bank_mask:0xf bound_ctrl:1", v, ((lane & 16) && h < rs) ? 1.f : 0.f);
    LNR_FMAC_DPP_16("row_bcast:31 row_mask:0xf bank_mask:0xf bound_ctrl:1", v, (lane >= 32 && h < 32) ? 1.f : 0.f);
    return;
  }
  // longest distance from a lane back to its run's first lane in the same row (0..15), wave-uniform
  int d = lane - (h > rs ? h : rs);
  d = max(d, __builtin_amdgcn_update_dpp(0, d, 0x111, 0xF, 0xF, true));
  d = max(d, __builtin_amdgcn_update_dpp(0, d, 0x112, 0xF, 0xF, true));
  d = max(d, __builtin_amdgcn_update_dpp(0, d, 0x114, 0xF, 0xF, true));
  d = max(d, __builtin_amdgcn_update_dpp(0, d, 0x118, 0xF, 0xF, true));
  d = max(d, __builtin_amdgcn_update_dpp(0, d, 0x142, 0xA, 0xF, false));
  d = max(d, __builtin_amdgcn_update_dpp(0, d, 0x143, 0xC, 0xF, false));
  const int dmax = __builtin_amdgcn_readlane(d, 63);
  const bool cross = (ri.heads & 0x0001000100010000ull) != 0x0001000100010000ull;
  // every row enabled and bound_ctrl: a source lane outside the shift reads 0 (no "old" operand to
  // initialise); the lane conditions exclude the rows a broadcast does not address
#define LNR_SEG_STEP_N(CTRL, RMASK, COND)                                                  \
  {                                                                                        \
    float q[N];                                                                            \
    _Pragma("unroll") for (int k = 0; k < N; ++k) q[k] =                                   \
        __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[k]), CTRL, 0xF, 0xF, true)); \
    if (COND) {                                                                            \
      _Pragma("unroll") for (int k = 0; k < N; ++k) v[k] += q[k];                          \
    }                                                                                      \
  }
  if (dmax >= 1) LNR_SEG_STEP_N(0x111, 0xF, lane - 1 >= h)
  if (dmax >= 2) LNR_SEG_STEP_N(0x112, 0xF, lane - 2 >= h)
  if (dmax >= 4) LNR_SEG_STEP_N(0x114, 0xF, lane - 4 >= h)
  if (dmax >= 8) LNR_SEG_STEP_N(0x118, 0xF, lane - 8 >= h)
  if (cross) {
    LNR_SEG_STEP_N(0x142, 0xA, (lane & 16) && h < rs)  // row_bcast:15 -> rows 1, 3
    LNR_SEG_STEP_N(0x143, 0xC, lane >= 32 && h < 32)   // row_bcast:31 -> rows 2, 3
  }
#undef LNR_SEG_STEP_N
}

// Coherent-level records of one lane: corner k's (g0, g1) contributions summed over the lane's run;
// valid at the run's tail lanes (in).  The forward's histogram, the scatters and the count kernel
// all merge this way, so their record counts agree.
__device__ __forceinline__ void coherent_run_values(const Corners& c, bool in, float g0, float g1, RunInfo& ri,
                                                    float (&v)[16]) {
  ri = cell_runs_dpp(in, c.cx, c.cy, c.cz);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[2 * k] = c.w[k] * g0;
    v[2 * k + 1] = c.w[k] * g1;
  }
  run_sum_dpp_n<16>(ri, v);
}

// The same in int64 (exact and associative: the result does not depend on the record order).
__device__ __forceinline__ void run_sum_i64(const RunInfo& ri, long long& v0, long long& v1) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long q0 = __shfl_up(v0, o, 64), q1 = __shfl_up(v1, o, 64);
    if (lane - o >= ri.head_lane) {
      v0 += q0;
      v1 += q1;
    }
  }
}

// Backward workspace (device), carved from one caller-provided buffer.
// Records are binned per "super-block" of kSB consecutive samples (one histogram row per
// (level, super-block), one scatter workgroup per row): rows are written and read coalesced, and
// each block's run of records in a bucket averages kSB * 8 / buckets-per-level entries.
#ifndef LNR_KSB
#define LNR_KSB 512
#endif
constexpr int kSB = LNR_KSB;        // samples per histogram row / count / scatter workgroup
#ifndef LNR_ROWS_PER_CHUNK
#define LNR_ROWS_PER_CHUNK 64  // 38 -> 25 us for the two scan kernels at C2 against 256 (128: 26 us)
#endif
constexpr int kRowsPerChunk = LNR_ROWS_PER_CHUNK;  // histogram rows per scan chunk

// Record values: two fp16 of v 2^k_l (8-B records {word, half2}), at a per-level power-of-two scale
// 2^k_l from the level's max |d_enc| (ws.level_max, known before the scatter): every fine or generic
// record is w * g with w <= 1, and a coherent record sums at most one wave's run of 64 lanes, so
// |v| 2^k_l < 2^15 (2^k_l = 2^9 / 2^E, level max < 2^E) and no record overflows.  Each record rounds to 11 significant bits (relative
// 2^-12), where tcnn's own fp16 gradient rounds every partial sum; the accumulation adds the
// records exactly (int64 fixed point), so that rounding is the only one.  (fp32 values, 12-B
// records, were measured: the scatter 0.85 against 0.69 ms and the accumulation 0.56 against 0.45
// ms at C2.)
// Every level keeps the coherent levels' 2^6 headroom, so a level's scale does not depend on which
// levels merge runs (that follows the samples per ray); fine-level records then sit below 2^9, still
// normal fp16 down to 2^-23 of the level's largest.
__device__ __forceinline__ int rec_exp_for(float level_max) {
  int E;
  frexpf(level_max, &E);  // level_max < 2^E (E = 0 for 0)
  const int k = 9 - E;
  return k > 100 ? 100 : (k < -60 ? -60 : k);
}
__device__ __forceinline__ uint32_t rec_half2(float v0, float v1, float s) {
  const _Float16 a = (_Float16)(v0 * s), b = (_Float16)(v1 * s);
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}
__device__ __forceinline__ float rec_v0(uint32_t h) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(h & 0xFFFFu)); }
__device__ __forceinline__ float rec_v1(uint32_t h) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(h >> 16)); }

struct BwdWorkspace {
  uint32_t* hist;        // per level l: [n_sb][nb_l] record counts -> exclusive offsets within bucket
  uint32_t* chunk_sum;   // [L][n_chunks][kMaxChunksPerLevel] per-chunk column sums (k_bwd_chunk_sums)
  float* level_max;      // [LNR_MAX_LEVELS] max |d_enc| per level (as uint bits: k_denc_level_max's atomicMax)
  uint32_t* counts;      // [kMaxBuckets] records per bucket (the scatter's: placement, work split)
  uint64_t* seg_start;   // [kMaxBuckets + 1]
  long long* partial;    // [2 kAccumGroups][2 * kChunk] int64 fixed-point partial sums of cut buckets
  uint32_t* bucket_done; // [kMaxBuckets] pieces of a cut bucket accumulated so far (k_bwd_accum<true>)
  UnitTable* units;      // the unit accumulation's work list (k_bwd_scan_buckets / k_bwd_units)
  uint2* rec;            // [8 * N * L] records {word, half2} (see "Backward records")
  // the live backward (LNR_BWD_LIVE): its histogram rows are groups of 8 live waves (64-sample groups holding a
  // sample with dL/dsigma != 0), listed in sample order
  uint8_t* wflags;       // [ceil(N / 64)] wave w holds a live sample
  uint32_t* wlist;       // [ceil(N / 64)] the live waves, ascending
  uint32_t* live;        // [2] live waves, live rows (= ceil(live waves / 8))
  int64_t n_sb;
  int64_t n_chunks;
  int32_t k2;            // the fixed-point exponent of every bucket (bwd_fixed_k2: from N alone)
  bool use_live;         // the scans cover live[1] rows instead of n_sb (the live histogram)
};

inline int64_t bwd_n_sb(int64_t n) { return (n + kSB - 1) / kSB; }
inline int64_t bwd_n_chunks(int64_t n) { return (bwd_n_sb(n) + kRowsPerChunk - 1) / kRowsPerChunk; }

inline int64_t align256(int64_t b) { return (b + 255) / 256 * 256; }

struct WsLayout {
  int64_t hist, chunk_sum, level_max, counts, seg_start, partial, bucket_done, units, wflags, wlist, live, rec,
      total;
};

inline WsLayout ws_layout(const lnr_grid_desc* d, const GridArgs& a, int64_t n) {
  const int64_t nsb = bwd_n_sb(n), nch = bwd_n_chunks(n);
  WsLayout w{};
  int64_t b = 0;
  w.level_max = b; b += align256(LNR_MAX_LEVELS * 4);  // first: its address does not depend on n
  w.hist = b;      b += align256((int64_t)a.n_buckets * nsb * 4);
  w.chunk_sum = b; b += align256((int64_t)d->n_levels * nch * kMaxChunksPerLevel * 4);
  w.counts = b;    b += align256(kMaxBuckets * 4);
  w.seg_start = b; b += align256((kMaxBuckets + 1) * 8);
  w.partial = b;   b += align256((int64_t)2 * kAccumGroups * 2 * kChunk * 8);
  w.bucket_done = b; b += align256(kMaxBuckets * 4);
  w.units = b;     b += align256(sizeof(UnitTable));
  w.wflags = b;    b += align256((n + 63) / 64);
  w.wlist = b;     b += align256((n + 63) / 64 * 4);
  w.live = b;      b += align256(2 * 4);
  // +2 records: the accumulate loads records in pairs
  w.rec = b;       b += align256((8 * n * (int64_t)d->n_levels + 2) * 8);
  w.total = b;
  return w;
}

inline int64_t bwd_workspace_bytes(const lnr_grid_desc* d, int64_t n) { return ws_layout(d, make_args(d), n).total; }

// The backward's fixed-point exponent (records scaled by 2^k2, in the level's record units): the records of one
// level and feature, |w g| 2^k < 2^9 per sample (2^k = 2^9 / 2^E, level max |d_enc| < 2^E) with corner weights
// summing to 1 per sample, add up to less than N 2^9 in any bucket, so 2^(53 - lg N) keeps every int64 sum below
// 2^62 whatever the counts; one record converted stays below 2^51 (|record| < 2^15, k2 <= 36).  C2 (N = 2^22):
// k2 = 30, finer than a per-bucket count gives (47 - lg cnt: 27 for a fine bucket of every sample's records).  It
// depends on N alone: the full backward, the live backward and the skip-zero count all round alike.
inline int32_t bwd_fixed_k2(int64_t n) {
  const int lg = n > 0 ? 64 - __builtin_clzll((unsigned long long)n) : 1;  // bits of n (>= log2 n)
  return 53 - lg < 36 ? 53 - lg : 36;
}
inline BwdWorkspace carve_workspace(void* base, const GridArgs& a, const lnr_grid_desc* d, int64_t n) {
  const WsLayout L = ws_layout(d, a, n);
  char* p = reinterpret_cast<char*>(base);
  BwdWorkspace w{};
  w.hist = reinterpret_cast<uint32_t*>(p + L.hist);
  w.chunk_sum = reinterpret_cast<uint32_t*>(p + L.chunk_sum);
  w.level_max = reinterpret_cast<float*>(p + L.level_max);
  w.counts = reinterpret_cast<uint32_t*>(p + L.counts);
  w.seg_start = reinterpret_cast<uint64_t*>(p + L.seg_start);
  w.partial = reinterpret_cast<long long*>(p + L.partial);
  w.bucket_done = reinterpret_cast<uint32_t*>(p + L.bucket_done);
  w.units = reinterpret_cast<UnitTable*>(p + L.units);
  w.wflags = reinterpret_cast<uint8_t*>(p + L.wflags);
  w.wlist = reinterpret_cast<uint32_t*>(p + L.wlist);
  w.live = reinterpret_cast<uint32_t*>(p + L.live);
  w.rec = reinterpret_cast<uint2*>(p + L.rec);
  w.n_sb = bwd_n_sb(n);
  w.n_chunks = bwd_n_chunks(n);
  w.k2 = bwd_fixed_k2(n);
  return w;
}


__device__ __forceinline__ uint32_t* hist_row(const GridArgs& a, const BwdWorkspace& ws, uint32_t l, int64_t sb) {
  const uint32_t nb = a.bucket_base[l + 1] - a.bucket_base[l];
  return ws.hist + (int64_t)a.bucket_base[l] * ws.n_sb + sb * nb;
}

// Backward records.  A word w = entry within its 4096-entry chunk (bits 0-11) | pair code p (bits
// 12-15) | tx as unorm16 (bits 16-31), and two values (see "Record values").
//   p = 0  one corner; the values are its (g0, g1) contribution (coherent levels: summed over the
//          run of lanes that share the corner).
//   p > 0  the two x-adjacent corners e0 and e1 = e0 ^ (2^p - 1) of one y/z edge, in one chunk; the
//          values are wy*wz*(g0, g1), split (1 - tx, tx) when accumulated.  The x-neighbour of a
//          hashed corner, (x + 1) ^ h against x ^ h, flips the trailing ones of x and one more bit;
//          a dense level's neighbour is idx + 1: both are an XOR with 2^p - 1.
// Slots per (sample, level): coherent levels: slot k = corner k after the lane-run merge.  Other
// levels: slot j < 4 = the x-pair (2j, 2j+1), or corner 2j when the pair spans two chunks; slot
// 4 + j = corner 2j+1 of such a split pair.  So fine levels emit 4 records per sample, not 8.
constexpr uint32_t kRecNone = 0xFFFFFFFFu;  // never a valid word (p <= 12)

__device__ __forceinline__ bool pairable(uint32_t e0, uint32_t e1) {
  const uint32_t d = e0 ^ e1;
  return d != 0u && (d >> kChunkLog2) == 0u && (d & (d + 1u)) == 0u;
}
__device__ __forceinline__ uint32_t pair_word(uint32_t e0, uint32_t e1, uint32_t txq) {
  return (e0 & (kChunk - 1)) | ((uint32_t)__popc(e0 ^ e1) << kChunkLog2) | (txq << 16);
}
__device__ __forceinline__ uint32_t tx_unorm16(float tx) {
  const float q = fminf(fmaxf(tx, 0.f), 1.f) * 65535.f + 0.5f;
  return (uint32_t)q;
}
constexpr float kInvU16 = 1.0f / 65535.0f;

// Per-(super-block, level) record histogram: one kSB-thread workgroup, one sample per thread.
// Shared by the forward (training mode) and the standalone count kernel: identical corners, merge
// and pairing decisions as the scatter kernel, so counts and ranks agree exactly.  Writes the
// histogram row (k_bwd_chunk_sums then sums rows per scan chunk: no global atomics).
__device__ __forceinline__ void publish_block_counts(const GridArgs& a, uint32_t l, const uint32_t* hist,
                                                     const BwdWorkspace& ws) {
  const uint32_t nb = a.bucket_base[l + 1] - a.bucket_base[l];
  uint32_t* row = hist_row(a, ws, l, blockIdx.x);
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) row[b] = hist[b];
}

// Fine levels: one record per x-pair, two when the pair spans two chunks (d >= kChunk).  The _add
// forms only count (LDS atomics): the forward counts two samples per thread before publishing.
__device__ __forceinline__ void count_fine_add(const FineCell& c, bool in, uint32_t* hist) {
  if (in) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      atomicAdd(&hist[c.e[j] >> kChunkLog2], 1u);
      if (c.d >= (uint32_t)kChunk) atomicAdd(&hist[(c.e[j] ^ c.d) >> kChunkLog2], 1u);
    }
  }
}
__device__ __forceinline__ void count_block_records_fine(const GridArgs& a, uint32_t l, const FineCell& c, bool in,
                                                         uint32_t* hist, const BwdWorkspace& ws) {
  count_fine_add(c, in, hist);
  lds_barrier();
  publish_block_counts(a, l, hist, ws);
}

// ``in``: the sample exists; ``act``: it has a non-zero gradient at this level (only the count
// after the MLP backward knows; = in otherwise).  Coherent levels count every sample (zero lanes
// merge into the runs harmlessly), the others only active ones: the scatter decides the same way.
// Every lane of the wave must call it (the run ballot).
__device__ __forceinline__ void count_add(const GridArgs& a, uint32_t l, const Corners& c, bool in, bool act,
                                          uint32_t* hist) {
  const uint32_t off = a.lv[l].offset;
  if (l < a.merge_levels) {
    const RunInfo ri = cell_runs_dpp(in, c.cx, c.cy, c.cz);  // every lane must take part in the ballot
    if (in && ri.tail) {  // run tails only: few lanes
#pragma unroll
      for (int k = 0; k < 8; ++k) atomicAdd(&hist[(c.idx[k] - off) >> kChunkLog2], 1u);
    }
  } else if (act) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t e0 = c.idx[2 * j] - off, e1 = c.idx[2 * j + 1] - off;
      atomicAdd(&hist[e0 >> kChunkLog2], 1u);
      if (!pairable(e0, e1)) atomicAdd(&hist[e1 >> kChunkLog2], 1u);
    }
  }
}
__device__ __forceinline__ void count_block_records(const GridArgs& a, uint32_t l, const Corners& c, bool in,
                                                    bool act, uint32_t* hist, const BwdWorkspace& ws) {
  count_add(a, l, c, in, act, hist);
  lds_barrier();
  publish_block_counts(a, l, hist, ws);
}

}  // namespace lnr
