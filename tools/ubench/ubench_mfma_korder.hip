// Does v_mfma_f32_16x16x32_f16's result depend on the order of k?  D = A B with random fp16 operands, once
// with k in natural order and once with k permuted (the same permutation on A's columns and B's rows: the
// same products); prints how many of the 256 outputs differ in their bits.
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/ubench_mfma_korder.hip -o /tmp/korder && /tmp/korder
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float float4_t __attribute__((ext_vector_type(4)));

// A [16][32], B [32][16] fp16, perm[32]: k -> source k; out [2][256] (natural, permuted)
__global__ void k_korder(const _Float16* A, const _Float16* B, const int* perm, float* out) {
  const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
  half8_t a, b, ap, bp;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * g + j;
    a[j] = A[c * 32 + k];
    b[j] = B[k * 16 + c];
    ap[j] = A[c * 32 + perm[k]];
    bp[j] = B[perm[k] * 16 + c];
  }
  float4_t z = {0.f, 0.f, 0.f, 0.f};
  const float4_t d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, z, 0, 0, 0);
  const float4_t dp = __builtin_amdgcn_mfma_f32_16x16x32_f16(ap, bp, z, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    out[(4 * g + r) * 16 + c] = d[r];
    out[256 + (4 * g + r) * 16 + c] = dp[r];
  }
}

int main() {
  srand(7);
  _Float16 A[512], B[512];
  int perm[32];
  float out[512];
  _Float16 *dA, *dB;
  int* dP;
  float* dO;
  hipMalloc(&dA, sizeof(A));
  hipMalloc(&dB, sizeof(B));
  hipMalloc(&dP, sizeof(perm));
  hipMalloc(&dO, sizeof(out));
  const char* names[3] = {"reverse", "swap halves of 8", "rows 8g+q -> interleaved"};
  for (int trial = 0; trial < 3; ++trial) {
    for (int i = 0; i < 512; ++i) {
      // wide dynamic range, so that rounding order shows
      const float m = (float)(rand() % 2000 - 1000) / 1000.f;
      const int e = rand() % 12 - 6;
      A[i] = (_Float16)(m * (float)(1 << (e + 6)) / 64.f);
      B[i] = (_Float16)((float)(rand() % 2000 - 1000) / 1000.f);
    }
    for (int k = 0; k < 32; ++k)
      perm[k] = trial == 0 ? 31 - k : trial == 1 ? (k ^ 4) : (8 * (k & 3) + (k >> 2));
    hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
    hipMemcpy(dB, B, sizeof(B), hipMemcpyHostToDevice);
    hipMemcpy(dP, perm, sizeof(perm), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_korder, dim3(1), dim3(64), 0, 0, dA, dB, dP, dO);
    hipMemcpy(out, dO, sizeof(out), hipMemcpyDeviceToHost);
    int diff = 0;
    for (int i = 0; i < 256; ++i) diff += memcmp(&out[i], &out[256 + i], 4) != 0;
    printf("permutation %-26s: %d of 256 outputs differ in their bits\n", names[trial], diff);
  }
  return 0;
}
