// Gather throughput from an L2-resident 1 MB table: cost model of the hash-grid forward's loads.
// Each thread: K gathers at random (hashed) positions; variants differ in width / pairing and in the
// cache-policy bits of the load (does an L1-bypassing gather move less than a 128-B line from L2?).
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ uint32_t mix(uint32_t x) { x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x; }
template <int MODE, int AUX = 0>
__global__ void __launch_bounds__(256) kg(const uint32_t* __restrict__ t, uint32_t mask, int K, uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (int k = 0; k < K; ++k) {
    uint32_t e = mix(i * 8 + k) & mask;  // entry index (4-B entries)
    if (MODE == 0) {  // 2 dword gathers, partner e^1 (same 8 B)
      acc += t[e] + t[e ^ 1u];
    } else if (MODE == 1) {  // 1 dwordx2 gather covering both
      const uint2 v = *reinterpret_cast<const uint2*>(t + (e & ~1u));
      acc += v.x + v.y;
    } else if (MODE == 2) {  // 1 dwordx4 gather
      const uint4 v = *reinterpret_cast<const uint4*>(t + (e & ~3u));
      acc += v.x + v.w;
    } else if (MODE == 3) {  // 1 dword gather only
      acc += t[e];
    } else if (MODE == 4) {  // 2 dword gathers, partner in a different line
      acc += t[e] + t[(e + 4096u) & mask];
    } else if (MODE == 5) {  // 1 dword, nontemporal
      acc += __builtin_nontemporal_load(t + e);
    } else {  // 1 dword buffer load with cache-policy bits MODE - 6 (gfx950: 1 sc0, 2 nt, 8? sc1)
      __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)t, 0, (int)((mask + 1) * 4), 0x00020000);
      acc += __builtin_amdgcn_raw_buffer_load_b32(r, (int)(e * 4), 0, AUX);
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}
int main() {
  const uint32_t n = 1u << 18;  // 1 MB of 4-B entries
  uint32_t *t, *out;
  hipMalloc(&t, n * 4); hipMalloc(&out, 4); hipMemset(t, 1, n * 4);
  const int blocks = 65536, K = 8;
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const char* names[] = {"2x dword (pair)", "1x dwordx2", "1x dwordx4", "1x dword", "2x dword (far)", "1x dword nt",
                         "buf aux0", "buf aux1 sc0", "buf aux2 nt", "buf aux3", "buf aux16", "buf aux17"};
  for (int m = 0; m < 12; ++m) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      switch (m) {
        case 0: kg<0><<<blocks, 256>>>(t, n - 1, K, out); break;
        case 1: kg<1><<<blocks, 256>>>(t, n - 1, K, out); break;
        case 2: kg<2><<<blocks, 256>>>(t, n - 1, K, out); break;
        case 3: kg<3><<<blocks, 256>>>(t, n - 1, K, out); break;
        case 4: kg<4><<<blocks, 256>>>(t, n - 1, K, out); break;
        case 5: kg<5><<<blocks, 256>>>(t, n - 1, K, out); break;
        case 6: kg<6, 0><<<blocks, 256>>>(t, n - 1, K, out); break;
        case 7: kg<6, 1><<<blocks, 256>>>(t, n - 1, K, out); break;
        case 8: kg<6, 2><<<blocks, 256>>>(t, n - 1, K, out); break;
        case 9: kg<6, 3><<<blocks, 256>>>(t, n - 1, K, out); break;
        case 10: kg<6, 16><<<blocks, 256>>>(t, n - 1, K, out); break;
        case 11: kg<6, 17><<<blocks, 256>>>(t, n - 1, K, out); break;
      }
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (rep == 2) {
        const double lanes = (double)blocks * 256 * K;
        printf("%-18s %.3f ms  %.1f G pair-lookups/s\n", names[m], ms, lanes / ms / 1e6);
      }
    }
  }
  return 0;
}
