#include <hip/hip_runtime.h>
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((__vector_size__(8)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
__global__ void k(float* out, const _Float16* in) {
  __shared__ _Float16 img[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) img[i] = in[i];
  __syncthreads();
  const int lane = threadIdx.x, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  // transposed read of rows 4g+q, cols 4p..4p+3
  lds_v4i16* a = (lds_v4i16*)((__attribute__((address_space(3))) char*)img + ((4 * g + q) * 64 + 4 * p) * 2);
  half4_t v = __builtin_bit_cast(half4_t, __builtin_amdgcn_ds_read_tr16_b64_v4i16(a));
  float4_t acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f32_16x16x16f16(v, v, acc, 0, 0, 0);
  for (int j = 0; j < 4; ++j) out[lane * 4 + j] = (float)v[j] + acc[j] * 0.f;
}
int main() {
  _Float16 h[64 * 64];
  for (int r = 0; r < 64; ++r) for (int c = 0; c < 64; ++c) h[r * 64 + c] = (_Float16)(r * 100 + c);
  _Float16* din; float* dout; hipMalloc(&din, sizeof(h)); hipMalloc(&dout, 256 * 4);
  hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
  k<<<1, 64>>>(dout, din);
  float o[256]; hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 1) printf("lane %d: %g %g %g %g\n", l, o[4*l], o[4*l+1], o[4*l+2], o[4*l+3]);
  return 0;
}
