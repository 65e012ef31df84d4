// Colour head (tcnn FullyFusedMLP 48 -> 64 x (NH+1) -> 3, padded 16) operand layouts on gfx950 MFMA,
// shared by the render kernel (rgb.hip) and the training kernels (rgb_train.hip).  See rgb.hip.
#pragma once
#include "mlp.hpp"
#include "sh.hpp"

namespace lnr {


constexpr int kRgbWaves = 4;

constexpr int kRgbIn = 48, kRgbWidth = 64, kRgbOutPad = 16;

struct RgbArgs {
  const uint16_t* w;      // tcnn flat params of the colour network
  const uint32_t* enc;    // colour hash-grid encodings, level-major half2
  int64_t enc_stride;
  const float* rays;
  const float* weights;   // (R, S) compositing weights of the sigma pass
  int64_t n_rays;
  int32_t S;
  float* rgb;             // (R, 3)
  // training (lnr_rgb_train): L1 loss against the pixel intensities, mean over 3 x n_rays_global
  const float* gt;        // (R, 3)
  float* g;               // (R, 3) dL/drgb = sign(rgb - gt) * inv_count
  float* ray_loss;        // (R) sum_k |rgb_k - gt_k|
  float inv_count;
  float* denc_max;        // optional [16]: max |d_enc| per level (float bits, atomicMax; zeroed by the render)
  // training: the 16-sample tiles with a non-zero weight.  The render flags them (tile_live) and writes d_enc = 0
  // for the others (d_enc); k_rgb_tile_list lists them (tile_list, tile_count) for k_rgb_bwd2, which visits
  // only those
  float* d_enc;
  uint8_t* tile_live;     // (R * S / 16)
  uint32_t* tile_list;    // (R * S / 16)
  uint32_t* tile_count;   // [1]
};

template <int NH>
constexpr int rgb_mlp_params() { return 64 * kRgbIn + NH * 64 * 64 + kRgbOutPad * 64; }

template <int NH>
__device__ __forceinline__ int rgb_layer_offset(int l) {  // tcnn flat offset of matrix l (l = NH + 1: output)
  return l == 0 ? 0 : 64 * kRgbIn + (l - 1) * 64 * 64;
}

// The colour-head training backward, k_rgb_bwd2 (rgb_train.hip: compiled with MFMA results in VGPRs), for
// NH hidden-to-hidden layers on nb workgroups of kRgbBwd2Waves waves
constexpr int kRgbBwd2Waves = 8;
void launch_rgb_bwd2(int NH, const RgbArgs& a, float* d_enc, float* slab, int nb, hipStream_t st);

template <int NH>
struct RgbWeights {
  half8_t a0[4];          // layer 0, enc columns: W0[16t + c][8g + j]
  half8_t as[4];          // layer 0, SH columns (k-step zero-padded to 32): W0[16t + c][32 + 8g + j], g < 2
  half8_t ah[NH > 0 ? NH : 1][4][2];  // hidden layer h, row tile t, k-step s: Wh[16t + c][hid_perm(s, g, j)]
  half8_t ao[2];          // output: Wout[c][hid_perm(s, g, j)]
};

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

// 8 halves = 4 packed dwords: 16 contiguous bytes, or two 8-byte runs (hid_perm: 4g..4g+3 and
// 16+4g..16+4g+3 of a 32-wide k-step).
__device__ __forceinline__ half8_t ld_half8(const uint16_t* p) {
  return __builtin_bit_cast(half8_t, *reinterpret_cast<const u32x4_t*>(p));
}
__device__ __forceinline__ half8_t ld_half8_perm(const uint16_t* row, int s, int g) {
  const u32x2_t lo = *reinterpret_cast<const u32x2_t*>(row + 32 * s + 4 * g);
  const u32x2_t hi = *reinterpret_cast<const u32x2_t*>(row + 32 * s + 16 + 4 * g);
  const u32x4_t v = {lo.x, lo.y, hi.x, hi.y};
  return __builtin_bit_cast(half8_t, v);
}

template <int NH>
__device__ __forceinline__ void load_rgb_weights(const uint16_t* __restrict__ w, RgbWeights<NH>& rw) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const uint16_t* w0 = w;  // (64, 48)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    rw.a0[t] = ld_half8(w0 + (16 * t + c) * kRgbIn + 8 * g);
    const half8_t z = {};
    rw.as[t] = g < 2 ? ld_half8(w0 + (16 * t + c) * kRgbIn + 32 + 8 * g) : z;
  }
  const uint16_t* wh = w0 + kRgbWidth * kRgbIn;
#pragma unroll
  for (int h = 0; h < NH; ++h) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) rw.ah[h][t][s] = ld_half8_perm(wh + (16 * t + c) * kRgbWidth, s, g);
    wh += kRgbWidth * kRgbWidth;
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) rw.ao[s] = ld_half8_perm(wh + c * kRgbWidth, s, g);
}

// B operand (k-step s) from a layer's fp16-valued activations h[4t + r] = hid 16t + 4g + r.
__device__ __forceinline__ half8_t hid_operand(const float (&h)[16], int s) {
  half8_t b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (_Float16)h[4 * (2 * s + (j >> 2)) + (j & 3)];
  return b;
}

}  // namespace lnr
