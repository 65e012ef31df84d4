// Lane patterns of v_permlane16_swap / v_permlane32_swap and the DPP row mirrors on gfx950 (one wave, lane ids):
//   hipcc --offload-arch=gfx950 -O2 -w tools/ubench/ubench_permlane.hip -o /tmp/pl && /tmp/pl
#include <hip/hip_runtime.h>
__global__ void k(float* o) {
  float v = (float)threadIdx.x;
  auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  o[threadIdx.x] = __uint_as_float(r16[0]);
  o[64 + threadIdx.x] = __uint_as_float(r16[1]);
  o[128 + threadIdx.x] = __uint_as_float(r32[0]);
  o[192 + threadIdx.x] = __uint_as_float(r32[1]);
  o[256 + threadIdx.x] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
  o[320 + threadIdx.x] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));  // row_mirror
}
int main() {
  float* d; hipMalloc(&d, 384 * 4); hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
  float h[384]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[6] = {"pl16[0]", "pl16[1]", "pl32[0]", "pl32[1]", "half_mirror", "mirror"};
  for (int k = 0; k < 6; ++k) { printf("%s:", nm[k]); for (int i = 0; i < 64; ++i) printf(" %d", (int)h[64 * k + i]); printf("\n"); }
  return 0;
}
