// LDS ds_add_u64 throughput on one CU's 64 KB chunk (the hash-grid backward's accumulation): what
// the bank pattern of one wave-instruction costs.  Each wave issues K atomics per loop trip; lanes
// address entries of a 2 x 4096 u64 array by pattern:
//   RANDOM  hashed entries (the accumulate today: records of random entries)
//   BANKED  lane l of a 32-lane half: an entry with (entry mod 32) == l, otherwise random (bank-sorted)
//   LINEAR  entry = base + lane (consecutive entries: every lane its own bank pair)
//   SAME2   pairs of lanes share an entry (runs of equal corners), otherwise random
// 2 workgroups of 1024 threads per CU (the accumulate's shape), 80 KB LDS each.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/ubench_lds_atomic.hip -o tools/ubench/ubench_lds_atomic
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ uint32_t mix(uint32_t x) { x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x; }
template <int MODE>
__global__ void __launch_bounds__(1024, 8) ka(int trips, unsigned long long* out) {
  __shared__ unsigned long long acc[2 * 4096];
  __shared__ uint2 pad[2048];  // the accumulate's tile stage (same LDS footprint: 2 workgroups per CU)
  for (int t = threadIdx.x; t < 2 * 4096; t += 1024) acc[t] = 0;
  if (threadIdx.x < 2048 / 2) pad[threadIdx.x] = make_uint2(0, 0);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  uint32_t s = mix(blockIdx.x * 1024 + threadIdx.x);
  for (int it = 0; it < trips; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s = mix(s + k);
      uint32_t e;
      if (MODE == 0) e = s & 4095u;
      else if (MODE == 1) e = ((s & 4095u) & ~31u) | (lane & 31);
      else if (MODE == 2) e = ((s & 127u) << 5) | (lane & 31);  // (same as BANKED but row fixed per lane)
      else e = __shfl(s, lane & ~1, 64) & 4095u;
      atomicAdd(&acc[e], (unsigned long long)(k + 1));
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = acc[7] + pad[5].x;
}
int main() {
  int dev;
  hipGetDevice(&dev);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount, blocks = 2 * cus, trips = 2000;
  unsigned long long* out;
  hipMalloc(&out, blocks * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"RANDOM", "BANKED", "LINEAR", "SAME2"};
  for (int m = 0; m < 4; ++m) {
    float best = 1e9f;
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(a);
      switch (m) {
        case 0: ka<0><<<blocks, 1024>>>(trips, out); break;
        case 1: ka<1><<<blocks, 1024>>>(trips, out); break;
        case 2: ka<2><<<blocks, 1024>>>(trips, out); break;
        default: ka<3><<<blocks, 1024>>>(trips, out); break;
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep > 0 && ms < best) best = ms;
    }
    const double lanes = (double)blocks * 1024 * trips * 8;
    const double clk = p.clockRate * 1e3;  // Hz
    printf("%-7s %.3f ms  %.2f lane-atomics/clk/CU (at %.0f MHz)\n", names[m], best, lanes / (best * 1e-3) / clk / cus,
           clk / 1e6);
  }
  return 0;
}
