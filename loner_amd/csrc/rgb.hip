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
#include "rgb.hpp"

namespace lnr {



template <int NH, bool TRAIN>
__global__ void __launch_bounds__(64 * kRgbWaves) k_rgb_render(RgbArgs a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  if (TRAIN && a.denc_max && blockIdx.x == 0 && threadIdx.x < 16) a.denc_max[threadIdx.x] = 0.f;  // before k_rgb_bwd2
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
      const float w = a.weights[base + tb + c];
      // a tile whose 16 weights are all exactly 0 adds nothing to rgb (w * colour = 0): skipped
      // (its encodings may be the zeros of lnr_hashgrid_fwd_rays_live)
      const bool live = __ballot(w != 0.f) != 0ull;
      if (TRAIN) {  // the tile list of k_rgb_bwd2, and the dead tile's encoding gradient (16 levels x 16 samples)
        const int64_t tile = (base + tb) / 16;
        if (lane == 0) a.tile_live[tile] = live ? 1 : 0;
        if (!live) {
          float2* de = reinterpret_cast<float2*>(a.d_enc);
#pragma unroll
          for (int k = 0; k < 4; ++k) de[(int64_t)(4 * k + g) * a.enc_stride + base + tb + c] = make_float2(0.f, 0.f);
        }
      }
      if (!live) continue;
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
    if (TRAIN && lane == 0) {  // nn.functional.l1_loss(rgb.reshape(-1, 1), gt.reshape(-1, 1)) (optimizer.py:883-884)
      float l = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float d = acc_c[k] + (1.0f - acc_w) - a.gt[3 * r + k];
        a.g[3 * r + k] = (d > 0.f ? a.inv_count : (d < 0.f ? -a.inv_count : 0.f));  // torch.sign
        l += fabsf(d);
      }
      a.ray_loss[r] = l;
    }
  }
}


// ------------------------------------------------------------------ colour-head training backward
// The camera phase's backward (optimizer.py:541-688, compute_loss_camera :861-894) is k_rgb_bwd2
// (rgb_train.hip); round 4's k_rgb_bwd_tiles, kept for A/B in round 5 (LONER_RGB_BWD=1), was removed in round 6
// (history before commit e32a0b7; its numbers in DESIGN.md section 7c).

// d_w[i] = sum over the nb slabs, fixed order (as reduce_slabs_fixed, any parameter count)
__global__ void __launch_bounds__(64 * kSlabWaves) k_rgb_reduce_slabs(const float* __restrict__ slab, int nb, int P,
                                                                      float* __restrict__ dw) {
  __shared__ float part[kSlabWaves][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const int per = (nb + kSlabWaves - 1) / kSlabWaves;
  const int b0 = wid * per, b1 = b0 + per < nb ? b0 + per : nb;
  float s = 0.f;
  if (i < P) {
    int b = b0;
    for (; b + 16 <= b1; b += 16) {  // 16 rows in flight, added in order
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = slab[(int64_t)(b + u) * P + i];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; b < b1; ++b) s += slab[(int64_t)b * P + i];
  }
  part[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && i < P) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kSlabWaves; ++w) t += part[w][lane];
    dw[i] = t;
  }
}

// loss = inv_count * sum_r ray_loss[r], one workgroup, fixed order
__global__ void __launch_bounds__(1024) k_rgb_loss_sum(const float* __restrict__ ray_loss, int64_t n, float inv,
                                                       float* out) {
  __shared__ float red[16];
  float v = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) v += ray_loss[i];
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += red[w];
    out[0] = t * inv;
  }
}

constexpr int kRgbBwdMaxBlocks = 256;

// The live tiles (tile_live, k_rgb_render<NH, true>) in order: one workgroup, 16 consecutive tiles per thread per
// chunk of 16 K, a block-wide exclusive scan per chunk.
constexpr int kTileListThreads = 1024, kTileListPer = 16;
__global__ void __launch_bounds__(kTileListThreads) k_rgb_tile_list(const uint8_t* __restrict__ live, int64_t n_tiles,
                                                                   uint32_t* __restrict__ list,
                                                                   uint32_t* __restrict__ count) {
  __shared__ uint32_t wsum[kTileListThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  uint32_t base = 0;
  for (int64_t c0 = 0; c0 < n_tiles; c0 += (int64_t)kTileListThreads * kTileListPer) {
    const int64_t e0 = c0 + (int64_t)t * kTileListPer;
    uint8_t f[kTileListPer];
    if (e0 + kTileListPer <= n_tiles) {
      const uint4 v = *reinterpret_cast<const uint4*>(live + e0);  // (n_tiles padded to 16 in the workspace)
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < kTileListPer; ++j) f[j] = (uint8_t)((w4[j >> 2] >> (8 * (j & 3))) & 0xFFu);
    } else {
#pragma unroll
      for (int j = 0; j < kTileListPer; ++j) f[j] = e0 + j < n_tiles ? live[e0 + j] : 0;
    }
    uint32_t mine = 0;
#pragma unroll
    for (int j = 0; j < kTileListPer; ++j) mine += f[j] ? 1u : 0u;
    uint32_t inc = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t off = base + inc - mine, tot = 0;
    for (int w = 0; w < kTileListThreads / 64; ++w) {
      const uint32_t v = wsum[w];
      if (w < wid) off += v;
      tot += v;
    }
#pragma unroll
    for (int j = 0; j < kTileListPer; ++j)
      if (f[j]) list[off++] = (uint32_t)(e0 + j);
    base += tot;
    __syncthreads();
  }
  if (t == 0) count[0] = base;
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
  RgbArgs a{};
  a.w = w_rgb; a.enc = enc_rgb; a.enc_stride = enc_stride; a.rays = rays; a.weights = weights; a.n_rays = n_rays;
  a.S = n_samples; a.rgb = rgb;
  const int64_t nb = (n_rays + kRgbWaves - 1) / kRgbWaves;
  const dim3 grid((unsigned)(nb < 4096 ? nb : 4096)), block(64 * kRgbWaves);
  hipStream_t st = as_stream(stream);
  switch (n_hidden_layers - 1) {
    case 0: hipLaunchKernelGGL((k_rgb_render<0, false>), grid, block, 0, st, a); break;
    case 1: hipLaunchKernelGGL((k_rgb_render<1, false>), grid, block, 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_rgb_render<2, false>), grid, block, 0, st, a); break;
    default: hipLaunchKernelGGL((k_rgb_render<3, false>), grid, block, 0, st, a); break;
  }
  LNR_RETURN_LAUNCH("lnr_rgb_render");
}

extern "C" int64_t lnr_rgb_mlp_params(int32_t n_hidden_layers) {
  return 64 * kRgbIn + (int64_t)(n_hidden_layers - 1) * 64 * 64 + kRgbOutPad * 64;
}

// slabs | g (3R) | ray_loss (R) | the live-tile flags, list and count (tiles = R x S / 16; n_samples <= 2048)
static int64_t rgb_tiles_cap(int64_t n_rays) { return ((n_rays * 128 + 63) / 64) * 64; }
extern "C" int64_t lnr_rgb_train_workspace_bytes(int32_t n_hidden_layers, int64_t n_rays) {
  const int64_t P = lnr_rgb_mlp_params(n_hidden_layers);
  const int64_t tc = rgb_tiles_cap(n_rays);
  return (int64_t)kRgbBwdMaxBlocks * P * 4 + ((3 * n_rays + 63) / 64) * 64 * 4 + ((n_rays + 63) / 64) * 64 * 4 +
         tc + tc * 4 + 64;
}

template <int NH>
static int rgb_train_launch(RgbArgs a, float* d_enc, float* d_w, float* slab, float* loss, hipStream_t st) {
  const int64_t nb_r = (a.n_rays + kRgbWaves - 1) / kRgbWaves;
  hipLaunchKernelGGL((k_rgb_render<NH, true>), dim3((unsigned)(nb_r < 4096 ? nb_r : 4096)), dim3(64 * kRgbWaves), 0,
                     st, a);
  const int64_t tiles = a.n_rays * (int64_t)(a.S / 16);
  hipLaunchKernelGGL(k_rgb_tile_list, dim3(1), dim3(kTileListThreads), 0, st, a.tile_live, tiles, a.tile_list,
                     a.tile_count);
  const int64_t want = (tiles + kRgbBwd2Waves - 1) / kRgbBwd2Waves;  // a tile per wave per iteration
  const int nb = (int)(want < kRgbBwdMaxBlocks ? want : kRgbBwdMaxBlocks);
  launch_rgb_bwd2(NH, a, d_enc, slab, nb, st);
  const int P = rgb_mlp_params<NH>();
  hipLaunchKernelGGL(k_rgb_reduce_slabs, dim3((P + 63) / 64), dim3(64 * kSlabWaves), 0, st, slab, nb, P, d_w);
  if (loss) hipLaunchKernelGGL(k_rgb_loss_sum, dim3(1), dim3(1024), 0, st, a.ray_loss, a.n_rays, a.inv_count, loss);
  return LNR_OK;
}

extern "C" int lnr_rgb_train(const uint16_t* w_rgb, int32_t n_hidden_layers, const uint32_t* enc_rgb,
                             int64_t enc_stride, const float* rays, const float* weights, const float* intensities,
                             int64_t n_rays, int32_t n_samples, float inv_count, float* rgb, float* loss,
                             float* d_enc, float* d_w, void* workspace, int64_t workspace_bytes,
                             float* d_enc_level_max, void* stream) {
  LNR_REQUIRE(n_hidden_layers >= 1 && n_hidden_layers <= 4,
              "lnr_rgb_train: n_hidden_layers=%d not supported (1..4, 64 neurons)", n_hidden_layers);
  LNR_REQUIRE(n_rays >= 0 && n_samples > 0 && n_samples % 16 == 0 && n_samples <= 2048,
              "lnr_rgb_train: n_samples=%d must be a positive multiple of 16, at most 2048", n_samples);
  LNR_REQUIRE(n_rays * (int64_t)n_samples < (int64_t(1) << 35), "lnr_rgb_train: too many samples");
  LNR_REQUIRE(enc_stride >= n_rays * (int64_t)n_samples, "lnr_rgb_train: enc_stride too small");
  LNR_REQUIRE(workspace_bytes >= lnr_rgb_train_workspace_bytes(n_hidden_layers, n_rays),
              "lnr_rgb_train: workspace too small (%lld < %lld bytes)", (long long)workspace_bytes,
              (long long)lnr_rgb_train_workspace_bytes(n_hidden_layers, n_rays));
  if (n_rays == 0) return LNR_OK;
  LNR_REQUIRE(w_rgb && enc_rgb && rays && weights && intensities && rgb && d_enc && d_w && workspace,
              "lnr_rgb_train: null pointer");
  const int64_t P = lnr_rgb_mlp_params(n_hidden_layers);
  float* slab = reinterpret_cast<float*>(workspace);
  float* g = slab + (int64_t)kRgbBwdMaxBlocks * P;
  float* ray_loss = g + ((3 * n_rays + 63) / 64) * 64;
  uint8_t* tile_live = reinterpret_cast<uint8_t*>(ray_loss + ((n_rays + 63) / 64) * 64);
  uint32_t* tile_list = reinterpret_cast<uint32_t*>(tile_live + rgb_tiles_cap(n_rays));
  uint32_t* tile_count = tile_list + rgb_tiles_cap(n_rays);
  RgbArgs a{};
  a.w = w_rgb; a.enc = enc_rgb; a.enc_stride = enc_stride; a.rays = rays; a.weights = weights; a.n_rays = n_rays;
  a.S = n_samples; a.rgb = rgb; a.gt = intensities; a.g = g; a.ray_loss = ray_loss; a.inv_count = inv_count;
  a.denc_max = d_enc_level_max;
  a.d_enc = d_enc; a.tile_live = tile_live; a.tile_list = tile_list; a.tile_count = tile_count;
  hipStream_t st = as_stream(stream);
  switch (n_hidden_layers - 1) {
    case 0: rgb_train_launch<0>(a, d_enc, d_w, slab, loss, st); break;
    case 1: rgb_train_launch<1>(a, d_enc, d_w, slab, loss, st); break;
    case 2: rgb_train_launch<2>(a, d_enc, d_w, slab, loss, st); break;
    default: rgb_train_launch<3>(a, d_enc, d_w, slab, loss, st); break;
  }
  LNR_RETURN_LAUNCH("lnr_rgb_train");
}
