// Sample-wise sigma MLP kernels behind the tcnn-compatible module path
// (tcnn.NetworkWithInputEncoding forward/backward, src/models/nerf_tcnn.py:35-38,71).
// The fused per-ray path (field.hip) uses the same device functions from mlp.hpp.
#include "mlp.hpp"

namespace lnr {

__global__ void __launch_bounds__(256) k_sigma_mlp_fwd(const uint16_t* __restrict__ w, const uint32_t* __restrict__ enc,
                                                       int64_t stride, int64_t n, uint16_t* __restrict__ sigma) {
  SigmaWeights sw;
  load_sigma_weights(w, sw);
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int64_t n_tiles = (n + 15) / 16;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t tile = wave; tile < n_tiles; tile += n_waves) {
    const int64_t s = tile * 16 + c;
    const bool valid = s < n;
    half8_t b = load_enc_operand(enc, stride, s, valid);
    SigmaHidden h;
    const float sg = sigma_tile_fwd(sw, b, h);
    if (g == 0 && valid) sigma[s] = f2h(sigma_to_f16(sg));
  }
}

__global__ void __launch_bounds__(256) k_sigma_mlp_bwd(const uint16_t* __restrict__ w, const uint32_t* __restrict__ enc,
                                                       int64_t stride, int64_t n, const float* __restrict__ dsig,
                                                       float* __restrict__ d_enc, float* __restrict__ slab) {
  // 4 waves x 6 KB dW0 transposes; reused as the 12 KB dW slab reduction buffer at the end
  __shared__ __attribute__((aligned(16))) char smem[4 * (64 * 32 + 32 * 32) * 2];
  SigmaWeights sw;
  load_sigma_weights(w, sw);
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4, wid = threadIdx.x >> 6;
  _Float16* lds = reinterpret_cast<_Float16*>(smem) + wid * (64 * 32 + 32 * 32);
  DW0Acc acc;
  float dw1[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) dw1[k] = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc.v[t][m][q] = 0.f;
  float2* de = reinterpret_cast<float2*>(d_enc);
  const int64_t n_pairs = (n + 31) / 32;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t pr = wave; pr < n_pairs; pr += n_waves) {
    const int64_t s0 = pr * 32 + c, s1 = pr * 32 + 16 + c;
    const bool v0 = s0 < n, v1 = s1 < n;
    half8_t e0 = load_enc_operand(enc, stride, s0, v0);
    half8_t e1 = load_enc_operand(enc, stride, s1, v1);
    SigmaHidden h0, h1;
    (void)sigma_tile_fwd(sw, e0, h0);
    (void)sigma_tile_fwd(sw, e1, h1);
    const float ds0 = v0 ? dsig[s0] : 0.f, ds1 = v1 ? dsig[s1] : 0.f;
    float mx = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      dw1[k] = fmaf(ds0, h0[k], dw1[k]);
      dw1[k] = fmaf(ds1, h1[k], dw1[k]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fmaxf(fabsf((float)e0[j] * ds0), fabsf((float)e1[j] * ds1)));
    const float scale = grad_scale(wave_max(mx));
    float d[2][4];
    sigma_tile_bwd_denc(sw, h0, d);
    if (v0) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int lvl = 8 * m + 2 * g;
        de[(int64_t)lvl * stride + s0] = make_float2(d[m][0] * ds0, d[m][1] * ds0);
        de[(int64_t)(lvl + 1) * stride + s0] = make_float2(d[m][2] * ds0, d[m][3] * ds0);
      }
    }
    sigma_tile_bwd_denc(sw, h1, d);
    if (v1) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int lvl = 8 * m + 2 * g;
        de[(int64_t)lvl * stride + s1] = make_float2(d[m][0] * ds1, d[m][1] * ds1);
        de[(int64_t)(lvl + 1) * stride + s1] = make_float2(d[m][2] * ds1, d[m][3] * ds1);
      }
    }
    dw0_pair(lds, sw, h0, h1, e0, e1, ds0, ds1, scale, acc);
  }
  __syncthreads();
  write_dw_slab<256>(reinterpret_cast<float*>(smem), acc, dw1, slab + (int64_t)blockIdx.x * LNR_SIGMA_MLP_PARAMS);
}

// dW += the per-workgroup slabs, fixed summation order (mlp.hpp reduce_slabs_fixed)
__global__ void __launch_bounds__(64 * kSlabWaves) k_reduce_slabs_mlp(const float* __restrict__ slab, int nb, float* __restrict__ dw) {
  reduce_slabs_fixed(slab, nb, dw);
}

static int mlp_blocks(int64_t n_rows) {
  int64_t nb = n_rows < 1024 ? n_rows : 1024;
  return (int)(nb < 1 ? 1 : nb);
}

}  // namespace lnr

using namespace lnr;

extern "C" int lnr_sigma_mlp_fwd(const uint16_t* w, const uint32_t* enc, int64_t enc_stride, int64_t n, uint16_t* sigma,
                                 void* stream) {
  LNR_REQUIRE(n >= 0 && enc_stride >= n, "lnr_sigma_mlp_fwd: bad sizes");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(w && enc && sigma, "lnr_sigma_mlp_fwd: null pointer");
  const int64_t tiles = (n + 15) / 16;
  int64_t nb = (tiles + 3) / 4;
  if (nb > 8192) nb = 8192;
  hipLaunchKernelGGL(k_sigma_mlp_fwd, dim3((unsigned)nb), dim3(256), 0, as_stream(stream), w, enc, enc_stride, n, sigma);
  LNR_RETURN_LAUNCH("lnr_sigma_mlp_fwd");
}

extern "C" int lnr_sigma_mlp_bwd(const uint16_t* w, const uint32_t* enc, int64_t enc_stride, int64_t n,
                                 const float* d_sigma, float* d_enc, float* d_w, float* workspace, void* stream) {
  LNR_REQUIRE(n >= 0 && enc_stride >= n, "lnr_sigma_mlp_bwd: bad sizes");
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(w && enc && d_sigma && d_enc && d_w && workspace, "lnr_sigma_mlp_bwd: null pointer");
  const int64_t pairs = (n + 31) / 32;
  const int nb = mlp_blocks((pairs + 3) / 4);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(k_sigma_mlp_bwd, dim3(nb), dim3(256), 0, st, w, enc, enc_stride, n, d_sigma, d_enc, workspace);
  hipLaunchKernelGGL(k_reduce_slabs_mlp, dim3((LNR_SIGMA_MLP_PARAMS + 63) / 64), dim3(64 * kSlabWaves), 0, st, workspace, nb, d_w);
  LNR_RETURN_LAUNCH("lnr_sigma_mlp_bwd");
}
