// Direction encoding of the colour head: real spherical harmonics up to degree 4 (16 outputs),
// the tiny-cuda-nn "SphericalHarmonics" encoding used by DecoupledNeRF._dir_encoding
// (src/models/nerf_tcnn.py:43,86; cfg/nerf_config/default_nerf_hash.yaml:5-7).  tcnn takes the
// direction in [0,1]^3 and maps it back with 2x-1 (nerf_tcnn.py:83 does the (d+1)/2).
// Elementwise and HBM-bound: 12 B in, 2*degree^2 B out per direction.
#include "sh.hpp"

namespace lnr {

template <int DEG>
__global__ void __launch_bounds__(256) k_sh_encode(const float* __restrict__ dir01, int64_t n, uint16_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float o[16];
  sh_eval<DEG>(dir01[3 * i + 0], dir01[3 * i + 1], dir01[3 * i + 2], o);
  uint16_t* dst = out + i * (DEG * DEG);
#pragma unroll
  for (int k = 0; k < DEG * DEG; ++k) dst[k] = f2h(o[k]);
}

}  // namespace lnr

using namespace lnr;

extern "C" int lnr_sh_encode(const float* dir01, int64_t n, int32_t degree, uint16_t* out, void* stream) {
  LNR_REQUIRE(degree >= 1 && degree <= 4, "SphericalHarmonics: degree=%d not supported (1..4)", degree);
  LNR_REQUIRE(n >= 0, "lnr_sh_encode: n=%lld", (long long)n);
  if (n == 0) return LNR_OK;
  LNR_REQUIRE(dir01 && out, "lnr_sh_encode: null pointer");
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  hipStream_t st = as_stream(stream);
  switch (degree) {
    case 1: hipLaunchKernelGGL(k_sh_encode<1>, grid, block, 0, st, dir01, n, out); break;
    case 2: hipLaunchKernelGGL(k_sh_encode<2>, grid, block, 0, st, dir01, n, out); break;
    case 3: hipLaunchKernelGGL(k_sh_encode<3>, grid, block, 0, st, dir01, n, out); break;
    default: hipLaunchKernelGGL(k_sh_encode<4>, grid, block, 0, st, dir01, n, out); break;
  }
  LNR_RETURN_LAUNCH("lnr_sh_encode");
}
