// Write a buffer of B bytes (streaming, 16 B/lane) then read it back (sum), same buffer reused:
// does the Infinity Cache absorb a write->read round trip when B < 256 MiB?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void kw(float4* p, size_t n, float s) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_float4(s, s + 1, s + 2, (float)i);
}
__global__ void kr(const float4* p, size_t n, float* out) {
  float a = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float4 v = p[i]; a += v.x + v.w;
  }
  if (a == 12345.f) out[0] = a;
}
int main() {
  const size_t sizes_mb[] = {64, 128, 192, 224, 256, 320, 512, 2048};
  size_t maxb = 2048ull << 20;
  float4* buf; float* out;
  hipMalloc(&buf, maxb); hipMalloc(&out, 4);
  hipEvent_t e0, e1, e2; hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2);
  for (size_t mb : sizes_mb) {
    size_t n = (mb << 20) / 16;
    float tw = 0, tr = 0; int reps = 20;
    for (int r = 0; r < reps + 3; ++r) {
      hipEventRecord(e0);
      kw<<<4096, 256>>>(buf, n, (float)r);
      hipEventRecord(e1);
      kr<<<4096, 256>>>(buf, n, out);
      hipEventRecord(e2);
      hipEventSynchronize(e2);
      float a, b; hipEventElapsedTime(&a, e0, e1); hipEventElapsedTime(&b, e1, e2);
      if (r >= 3) { tw += a; tr += b; }
    }
    tw /= reps; tr /= reps;
    printf("%5zu MB: write %.1f us (%.2f TB/s)  read %.1f us (%.2f TB/s)\n", mb, tw * 1e3, (mb << 20) / (tw * 1e-3) / 1e12,
           tr * 1e3, (mb << 20) / (tr * 1e-3) / 1e12);
  }
  return 0;
}
