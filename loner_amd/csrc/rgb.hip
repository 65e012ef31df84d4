// Colour head forward + colour compositing, fused (inference, C3 shape).
//
// Reference: DecoupledNeRF.forward with sigma_only=False (src/models/nerf_tcnn.py:80-95):
//   h_x   = colour HashGrid(pos01)                           (L=16, F=2, T=2^19: 32 features)
//   h_d   = SphericalHarmonics(deg 4)((viewdir + 1) / 2)     (16 features)
//   h_c   = FullyFusedMLP([h_x, h_d])  48 -> 64 (ReLU) -> ... -> 3 (padded 16), fp16, no bias
//   color = sigmoid(h_c)                                      (fp16)
// and raw2outputs' colour map (src/models/rendering_tcnn.py:283-289):
//   rgb = sum_i w_i * color_i + (1 - sum_i w_i)   (white background, rendering_tcnn.py:288-289)
// with the weights of the sigma pass (lnr_field_render), the direction repeated per sample
// (rendering_tcnn.py:319-320: the view direction, rays[:, 6:9]).
//
// One wave per ray, 16-sample tiles on v_mfma_f32_16x16x32_f16.  The first layer's 48 inputs are two
// k-steps: the 32 colour-grid features, and the 16 SH values (constant along the ray, one B operand
// per ray) zero-padded to 32.  Hidden activations are rounded to fp16 (tcnn keeps
// them in fp16) and stay in registers between layers: a layer's accumulator (hid on rows, sample on
// the lane) is the next layer's B operand when the next layer's weights are read with the k index
// permuted by hid_perm (mlp.hpp).  Weights of every layer live in registers (NH hidden-to-hidden
// layers, template).  The colour encodings are read once (64 B per sample): the kernel is bound by
// the MFMA chain (8 + 8 * NH + 2 MFMAs per 16 samples) and that read.
#include "mlp.hpp"
#include "sh.hpp"

namespace lnr {

constexpr int kRgbWaves = 4;
constexpr int kRgbIn = 48, kRgbWidth = 64, kRgbOutPad = 16;

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

struct RgbArgs {
  const uint16_t* w;      // tcnn flat params of the colour network
  const uint32_t* enc;    // colour hash-grid encodings, level-major half2
  int64_t enc_stride;
  const float* rays;
  const float* weights;   // (R, S) compositing weights of the sigma pass
  int64_t n_rays;
  int32_t S;
  float* rgb;             // (R, 3)
};

template <int NH>
__global__ void __launch_bounds__(64 * kRgbWaves) k_rgb_render(RgbArgs a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  RgbWeights<NH> rw;
  load_rgb_weights<NH>(a.w, rw);
  for (int64_t r = (int64_t)blockIdx.x * kRgbWaves + wid; r < a.n_rays; r += (int64_t)gridDim.x * kRgbWaves) {
    const float* ry = a.rays + 13 * r;
    // dir = (viewdir + 1) / 2 (nerf_tcnn.py:83), SH degree 4 rounded to fp16 (tcnn encodings are fp16)
    float sh[16];
    sh_eval<4>((ry[6] + 1.0f) / 2.0f, (ry[7] + 1.0f) / 2.0f, (ry[8] + 1.0f) / 2.0f, sh);
    // B operand of the SH k-step: the same 16 fp16 values for every sample column, zero padding
    half8_t bsh = {};
    if (g < 2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) bsh[j] = (_Float16)sh[8 * g + j];
    }
    float acc_c[3] = {0.f, 0.f, 0.f}, acc_w = 0.f;
    const int64_t base = r * a.S;
    for (int tb = 0; tb < a.S; tb += 16) {
      const half8_t benc = load_enc_operand(a.enc, a.enc_stride, base + tb + c, true);
      float h[16];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float4_t acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.a0[t], benc, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.as[t], bsh, acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) h[4 * t + q] = round_f16(fmaxf(acc[q], 0.f));
      }
#pragma unroll
      for (int l = 0; l < NH; ++l) {
        const half8_t b0 = hid_operand(h, 0), b1 = hid_operand(h, 1);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          float4_t acc = {0.f, 0.f, 0.f, 0.f};
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.ah[l][t][0], b0, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.ah[l][t][1], b1, acc, 0, 0, 0);
#pragma unroll
          for (int q = 0; q < 4; ++q) h[4 * t + q] = round_f16(fmaxf(acc[q], 0.f));
        }
      }
      float4_t o = {0.f, 0.f, 0.f, 0.f};
      o = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.ao[0], hid_operand(h, 0), o, 0, 0, 0);
      o = __builtin_amdgcn_mfma_f32_16x16x32_f16(rw.ao[1], hid_operand(h, 1), o, 0, 0, 0);
      if (g == 0) {  // rows 0..2 = the three colour channels of sample tb + c
        const float w = a.weights[base + tb + c];
        acc_w += w;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float hc = round_f16(o[k]);                             // tcnn fp16 output
          const float col = round_f16(1.0f / (1.0f + expf(-hc)));       // torch.sigmoid on fp16
          acc_c[k] = fmaf(w, col, acc_c[k]);
        }
      }
    }
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) {  // lanes 0..15 hold the partial sums
      acc_w += __shfl_xor(acc_w, off, 64);
#pragma unroll
      for (int k = 0; k < 3; ++k) acc_c[k] += __shfl_xor(acc_c[k], off, 64);
    }
    if (lane < 3) a.rgb[3 * r + lane] = (lane == 0 ? acc_c[0] : lane == 1 ? acc_c[1] : acc_c[2]) + (1.0f - acc_w);
  }
}

}  // namespace lnr

using namespace lnr;

extern "C" int lnr_rgb_render(const uint16_t* w_rgb, int32_t n_hidden_layers, const uint32_t* enc_rgb,
                              int64_t enc_stride, const float* rays, const float* weights, int64_t n_rays,
                              int32_t n_samples, float* rgb, void* stream) {
  LNR_REQUIRE(n_hidden_layers >= 1 && n_hidden_layers <= 4,
              "lnr_rgb_render: n_hidden_layers=%d not supported (1..4, 64 neurons)", n_hidden_layers);
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && n_samples % 16 == 0,
              "lnr_rgb_render: n_samples=%d must be a positive multiple of 16", n_samples);
  LNR_REQUIRE(enc_stride >= n_rays * (int64_t)n_samples, "lnr_rgb_render: enc_stride too small");
  if (n_rays == 0) return LNR_OK;
  LNR_REQUIRE(w_rgb && enc_rgb && rays && weights && rgb, "lnr_rgb_render: null pointer");
  RgbArgs a{w_rgb, enc_rgb, enc_stride, rays, weights, n_rays, n_samples, rgb};
  const int64_t nb = (n_rays + kRgbWaves - 1) / kRgbWaves;
  const dim3 grid((unsigned)(nb < 4096 ? nb : 4096)), block(64 * kRgbWaves);
  hipStream_t st = as_stream(stream);
  switch (n_hidden_layers - 1) {
    case 0: hipLaunchKernelGGL(k_rgb_render<0>, grid, block, 0, st, a); break;
    case 1: hipLaunchKernelGGL(k_rgb_render<1>, grid, block, 0, st, a); break;
    case 2: hipLaunchKernelGGL(k_rgb_render<2>, grid, block, 0, st, a); break;
    default: hipLaunchKernelGGL(k_rgb_render<3>, grid, block, 0, st, a); break;
  }
  LNR_RETURN_LAUNCH("lnr_rgb_render");
}
