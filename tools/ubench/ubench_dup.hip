// Duplicate-lane gathers from an L2-resident 1 MB table (the hash-grid forward at levels where
// consecutive samples of a ray share a cell): does the texture-addresser charge a wave's gather by
// lanes, by distinct addresses or by distinct lines?  Each thread does K dword gathers; in mode DUP,
// groups of G consecutive lanes read the SAME address; in mode LINE, groups of G consecutive lanes
// read consecutive dwords of one 128-B line (G <= 32).  Time per wave-instruction against G answers it.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/ubench_dup.hip -o /tmp/ubench_dup && /tmp/ubench_dup
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ uint32_t mix(uint32_t x) { x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x; }
template <int MODE>
__global__ void __launch_bounds__(256) kd(const uint32_t* __restrict__ t, uint32_t mask, int K, int G, uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const uint32_t grp = i / G, sub = i % G;
  uint32_t acc = 0;
  for (int k = 0; k < K; ++k) {
    uint32_t e;
    if (MODE == 0) e = mix(grp * 8 + k) & mask;                          // DUP: one address per group
    else e = ((mix(grp * 8 + k) & mask) & ~31u) + (sub & 31u);            // LINE: one line per group
    acc += t[e];
  }
  if (acc == 0x12345678u) out[0] = acc;
}
int main() {
  const uint32_t n = 1u << 18;  // 1 MB of 4-B entries
  uint32_t *t, *out;
  hipMalloc(&t, n * 4);
  hipMalloc(&out, 4);
  hipMemset(t, 1, n * 4);
  const int blocks = 65536, K = 8;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int gs[] = {1, 2, 4, 8, 16, 32, 64};
  for (int mode = 0; mode < 2; ++mode) {
    for (int gi = 0; gi < 7; ++gi) {
      const int G = gs[gi];
      if (mode == 1 && G > 32) continue;
      float best = 1e9f;
      for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(a);
        if (mode == 0) kd<0><<<blocks, 256>>>(t, n - 1, K, G, out);
        else kd<1><<<blocks, 256>>>(t, n - 1, K, G, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (rep > 0 && ms < best) best = ms;
      }
      const double lanes = (double)blocks * 256 * K;
      const double insts = lanes / 64;
      printf("%-4s G=%2d  %.3f ms  %.1f G lane-gathers/s  %.2f ns per wave-instruction per CU (x256)\n",
             mode == 0 ? "DUP" : "LINE", G, best, lanes / best / 1e6, best * 1e6 / insts * 256);
    }
  }
  return 0;
}
