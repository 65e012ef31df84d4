// Shared device/host helpers for the LONER MI355X path (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdint>
#include <cstdio>
#include <cstdarg>
#include <cmath>

#include "../../include/loner_amd.h"

namespace lnr {

// ------------------------------------------------------------------ errors (host)
void set_error(const char* fmt, ...);
#define LNR_REQUIRE(cond, ...)                     \
  do {                                             \
    if (!(cond)) {                                 \
      ::lnr::set_error(__VA_ARGS__);               \
      return LNR_ERR_ARG;                          \
    }                                              \
  } while (0)
#define LNR_RETURN_LAUNCH(what)                                                   \
  do {                                                                            \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess) {                                                       \
      ::lnr::set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e_)); \
      return LNR_ERR_HIP;                                                         \
    }                                                                             \
    return LNR_OK;                                                                \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

// ------------------------------------------------------------------ RNG (oracle/rng.py)
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__host__ __device__ __forceinline__ uint32_t rand_u32(uint32_t key, uint32_t stream, uint32_t a, uint32_t b) {
  uint32_t h = mix32(key ^ (stream * 0x9E3779B9u));
  h = mix32(h ^ a);
  h = mix32(h ^ (b * 0x85EBCA6Bu + 0x632BE5ABu));
  return h;
}
__device__ __forceinline__ float rand_uniform(uint32_t key, uint32_t stream, uint32_t a, uint32_t b) {
  return (float)(rand_u32(key, stream, a, b) >> 8) * 5.9604644775390625e-08f;  // 2^-24
}
__device__ __forceinline__ float rand_normal(uint32_t key, uint32_t stream, uint32_t a, uint32_t b) {
  float u1 = ((float)(rand_u32(key, stream, a, b) >> 8) + 1.0f) * 5.9604644775390625e-08f;
  float u2 = (float)(rand_u32(key, stream + 1, a, b) >> 8) * 5.9604644775390625e-08f;
  return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}
enum : uint32_t { kStreamJitter = 1, kStreamPdf = 2, kStreamNoise = 3 };

// ------------------------------------------------------------------ fp16
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef _Float16 half2v_t __attribute__((ext_vector_type(2)));
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef short v4i16_t __attribute__((__vector_size__(8)));
typedef uint16_t u16x2v_t __attribute__((ext_vector_type(2)));
typedef int16_t i16x2v_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
__device__ __forceinline__ float round_f16(float f) { return (float)(_Float16)f; }
__device__ __forceinline__ float2 half2_to_float2(uint32_t v) {
  return make_float2(h2f((uint16_t)(v & 0xFFFFu)), h2f((uint16_t)(v >> 16)));
}

__device__ __forceinline__ float pk_lo(uint32_t v) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(v & 0xFFFFu)); }
__device__ __forceinline__ float pk_hi(uint32_t v) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(v >> 16)); }
// fp32 pair -> packed fp16 (round to nearest even), ReLU on the halves (the ReLU of the rounded value is the
// rounding of the ReLU; a negative value may give -0, which every consumer treats as 0)
__device__ __forceinline__ uint32_t pk_relu(float x, float y) {
  half2v_t h = {(_Float16)x, (_Float16)y};
  const half2v_t z = {(_Float16)0.f, (_Float16)0.f};
  h = __builtin_elementwise_max(h, z);
  return __builtin_bit_cast(uint32_t, h);
}
// 0xFFFF in each half whose value is not +-0: bit 15 of (|h| + 0x7FFF) per half, spread by an arithmetic shift
// (v_and, v_pk_add_u16, v_pk_ashrrev_i16: no carries between the halves, |h| <= 0x7FFF)
__device__ __forceinline__ uint32_t pk_nonzero_mask(uint32_t h) {
  const u16x2v_t t = __builtin_bit_cast(u16x2v_t, h & 0x7FFF7FFFu) + (u16x2v_t){0x7FFF, 0x7FFF};
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(i16x2v_t, t) >> (i16x2v_t){15, 15});
}
// ds_read_b64_tr_b16: in each 16-lane group, lane 4q + p gives the address of 4 halves (columns 4p .. 4p + 3 of
// row q); lane i receives column i of the 4 rows
__device__ __forceinline__ half4_t lds_tr16(const uint32_t* p) {
  return __builtin_bit_cast(half4_t, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                         (__attribute__((address_space(3))) v4i16_t*)(p)));
}

// ------------------------------------------------------------------ barriers
// Workgroup barrier that orders LDS only: waits for this wave's LDS operations (lgkmcnt), not for
// its global loads and stores (vmcnt), which __syncthreads' full fence would drain.  For barriers
// that only publish LDS data, so global loads issued before them stay in flight across them.
// The scheduling barriers keep register copies of in-flight loads from being hoisted above it
// (such a copy waits for its load).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  __builtin_amdgcn_sched_barrier(0);
}

// ------------------------------------------------------------------ wave / block reductions
// The butterfly over lane distances 32, 16, 8, 4, 2, 1 (every lane ends with the total).  LNR_WAVE_RED_DPP: the
// exchanges without LDS permutes: v_permlane32_swap / v_permlane16_swap (gfx950) for 32 and 16, DPP row_ror:8
// for 8 (within a row, lane p + 8 mod 16 = p ^ 8), row_ror:4 for 4 (lane p + 4 mod 16 holds the same value as
// p ^ 4 once the 8-apart lanes are equal), quad_perm for 2 and 1.  Each lane adds the same two values as the
// __shfl_xor butterfly (operands at most swapped): bitwise the same sums (tools/ubench/ubench_permlane.hip; C2 loss
// bit-identical, field stage 0.244-0.246 -> 0.242 ms).
#ifndef LNR_WAVE_RED_DPP
#define LNR_WAVE_RED_DPP 1
#endif
template <class Op>
__device__ __forceinline__ float wave_butterfly(float v, Op op) {
  if (LNR_WAVE_RED_DPP) {
    const uint32_t b = __float_as_uint(v);
    const auto r32 = __builtin_amdgcn_permlane32_swap(b, b, false, false);  // {lanes 0-31, lanes 32-63} in both halves
    v = op(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
    const uint32_t c = __float_as_uint(v);
    const auto r16 = __builtin_amdgcn_permlane16_swap(c, c, false, false);  // {even row, odd row} of each row pair
    v = op(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false)));  // row_ror:8
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false)));  // row_ror:4
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));   // quad [2,3,0,1]
    v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));   // quad [1,0,3,2]
    return v;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  return wave_butterfly(v, [](float x, float y) { return x + y; });
}
__device__ __forceinline__ float wave_max(float v) {
  return wave_butterfly(v, [](float x, float y) { return fmaxf(x, y); });
}

// Max of a NON-NEGATIVE float over the wave on DPP (row shifts, row_bcast15/31: no LDS permutes),
// read back from lane 63 so the result is wave-uniform.
__device__ __forceinline__ float wave_max_nonneg(float v) {
  int x = __float_as_int(v);  // non-negative floats order like their bit patterns; 0 is the identity
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true));  // row_shr:1
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true));  // row_shr:2
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true));  // row_shr:4
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true));  // row_shr:8 -> lane 15 of each row
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false));  // row_bcast:15 into rows 1, 3
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false));  // row_bcast:31 into rows 2, 3
  return __int_as_float(__builtin_amdgcn_readlane(x, 63));
}

// Inclusive prefix sum of a u32 over the wave on DPP (row shifts, then row_bcast15/31), no LDS.
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  int x = (int)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);   // row_shr:1 (row edge reads 0)
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 into rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 into rows 2, 3
  return (uint32_t)x;
}

// Block-wide sum of K values for a block of NT threads (NT/64 waves).  `scratch` needs
// K * (NT/64) floats; all threads receive the totals.  Contains two barriers.
template <int NT, int K>
__device__ __forceinline__ void block_sum(float (&v)[K], float* scratch) {
  constexpr int NW = NT / kWave;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_sum(v[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) scratch[k * NW + wid] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += scratch[k * NW + w];
    v[k] = s;
  }
  __syncthreads();
}

// ------------------------------------------------------------------ diagnostic phase stamps
// Experiment builds only (-DLNR_EXP_STAMPS, tools/exp_variants.py): thread 0 of each workgroup adds
// the s_memtime cycles of phase k to this translation unit's g_phase[k];
// LNR_PHASE_EXPORT(tu) defines lnr_debug_phases_<tu>() to read and clear them.
#ifdef LNR_EXP_STAMPS
static __device__ unsigned long long g_phase[32];
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define LNR_STAMP(var) unsigned long long var = (threadIdx.x == 0) ? ::lnr::stamp() : 0ull
#define LNR_PHASE(k, t1, t0) \
  if (threadIdx.x == 0 && (blockIdx.x & 63) == 0) atomicAdd(&::lnr::g_phase[k], (t1) - (t0))  // 1/64 sampled
// sampled by an explicit key (e.g. the row, so every level of a level-fastest grid is sampled)
#define LNR_PHASE_BY(key, k, t1, t0) \
  if (threadIdx.x == 0 && ((key) & 63) == 0) atomicAdd(&::lnr::g_phase[k], (t1) - (t0))
#define LNR_PHASE_EXPORT(tu)                                                                      \
  extern "C" int lnr_debug_phases_##tu(unsigned long long* out32) {                              \
    if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(::lnr::g_phase), 32 * 8) != hipSuccess) return -1; \
    unsigned long long z[32] = {};                                                                \
    return hipMemcpyToSymbol(HIP_SYMBOL(::lnr::g_phase), z, sizeof(z)) == hipSuccess ? 0 : -1;    \
  }
#else
#define LNR_STAMP(var)
#define LNR_PHASE(k, t1, t0)
#define LNR_PHASE_BY(key, k, t1, t0)
#define LNR_PHASE_EXPORT(tu)
#endif

// OccupancyGridModel.interpolate (src/models/model_tcnn.py:126-134): grid_sample of the (R, R, R) grid
// at (x, y, z) in [-1, 1] (x the fastest axis), trilinear, align_corners=False, zeros padding.  Its
// corner order and weights are those of the grid-gradient splat (optim.hip).
#ifndef LNR_OCC_PAIR
#define LNR_OCC_PAIR 1
#endif
__device__ __forceinline__ float occ_grid_sample(const float* __restrict__ occ, int R, float x, float y, float z) {
  const float ix = ((x + 1.f) * (float)R - 1.f) / 2.f;
  const float iy = ((y + 1.f) * (float)R - 1.f) / 2.f;
  const float iz = ((z + 1.f) * (float)R - 1.f) / 2.f;
  const float fx = floorf(ix), fy = floorf(iy), fz = floorf(iz);
  const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
  const float wx[2] = {(float)(x0 + 1) - ix, ix - (float)x0};
  const float wy[2] = {(float)(y0 + 1) - iy, iy - (float)y0};
  const float wz[2] = {(float)(z0 + 1) - iz, iz - (float)z0};
  float acc = 0.f;
#if LNR_OCC_PAIR
  // The two x-corners of each y/z edge are adjacent floats: one 8-B load per edge (4 gathers, not 8), from
  // x0 clamped to [0, R - 2] so that a pair with one corner outside the grid reads the other one.  The same
  // products added in the same order (a corner outside adds nothing, as before): bitwise the 8-load form.
  if (R >= 2) {
    typedef float f32x2u __attribute__((ext_vector_type(2), aligned(4)));
    const bool in0 = x0 >= 0 && x0 < R, in1 = x0 + 1 >= 0 && x0 + 1 < R;
    const int xb = min(max(x0, 0), R - 2);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int by = e & 1, bz = e >> 1;
      const int cy = y0 + by, cz = z0 + bz;
      const bool yz = cy >= 0 && cy < R && cz >= 0 && cz < R;
      f32x2u v = {0.f, 0.f};
      if (yz && (in0 || in1)) v = *(const f32x2u*)(occ + ((int64_t)cz * R + cy) * R + xb);
      const float v0 = xb == x0 ? v.x : v.y, v1 = xb == x0 ? v.y : v.x;
      const float w0 = wx[0] * wy[by] * wz[bz], w1 = wx[1] * wy[by] * wz[bz];
      if (yz && in0) acc += v0 * w0;
      if (yz && in1) acc += v1 * w1;
    }
    return acc;
  }
#endif
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int bx = c & 1, by = (c >> 1) & 1, bz = (c >> 2) & 1;
    const int cx = x0 + bx, cy = y0 + by, cz = z0 + bz;
    const float w = wx[bx] * wy[by] * wz[bz];
    if (cx >= 0 && cx < R && cy >= 0 && cy < R && cz >= 0 && cz < R) acc += occ[((int64_t)cz * R + cy) * R + cx] * w;
  }
  return acc;
}

}  // namespace lnr
