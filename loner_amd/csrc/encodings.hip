// Direction encoding of the colour head: real spherical harmonics up to degree 4 (16 outputs),
// the tiny-cuda-nn "SphericalHarmonics" encoding used by DecoupledNeRF._dir_encoding
// (src/models/nerf_tcnn.py:43,86; cfg/nerf_config/default_nerf_hash.yaml:5-7).  tcnn takes the
// direction in [0,1]^3 and maps it back with 2x-1 (nerf_tcnn.py:83 does the (d+1)/2).
// Elementwise and HBM-bound: 12 B in, 2*degree^2 B out per direction.
#include "common.hpp"

namespace lnr {

template <int DEG>
__global__ void __launch_bounds__(256) k_sh_encode(const float* __restrict__ dir01, int64_t n, uint16_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = dir01[3 * i + 0] * 2.0f - 1.0f;
  const float y = dir01[3 * i + 1] * 2.0f - 1.0f;
  const float z = dir01[3 * i + 2] * 2.0f - 1.0f;
  float o[16];
  const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
  o[0] = 0.28209479177387814f;
  if (DEG > 1) {
    o[1] = -0.48860251190291987f * y;
    o[2] = 0.48860251190291987f * z;
    o[3] = -0.48860251190291987f * x;
  }
  if (DEG > 2) {
    o[4] = 1.0925484305920792f * xy;
    o[5] = -1.0925484305920792f * yz;
    o[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
    o[7] = -1.0925484305920792f * xz;
    o[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
  }
  if (DEG > 3) {
    o[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
    o[10] = 2.8906114426405538f * xy * z;
    o[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
    o[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
    o[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
    o[14] = 1.4453057213202769f * z * (x2 - y2);
    o[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
  }
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
