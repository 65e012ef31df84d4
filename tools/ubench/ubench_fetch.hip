// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns of this build's
// kernels (MI355X_MICROARCH.md: FETCH_SIZE reports half of a wide streaming read; other widths are
// uncalibrated).  Every kernel touches a known number of bytes of an HBM-resident buffer (2 GiB, far
// past the 256 MiB Infinity Cache), once, so the counter per launch divided by the known bytes is the
// factor to apply.  Run each counter in its own pass:
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/ubench_fetch.hip -o /tmp/ubf
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d out -o run -- /tmp/ubf
//   rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d out -o run -- /tmp/ubf
// The program prints, per kernel, the bytes it moves (the denominators).
//   kr16   coalesced 16 B/lane loads (the accumulate's record reads, the streaming rule's case)
//   kr4    coalesced 4 B/lane loads (the scatter's / MLP's J, d_sigma and encoding reads)
//   kg4    random 4 B gathers, one per distinct 128-B line (the encode's table misses)
//   kg4p   lane pairs gathering the two dwords of one 8-B pair (the lane-paired encode)
//   kw8    coalesced 8 B/lane stores (record runs copied out whole)
//   kw8r   8-record runs (64 B) of 8-B stores at random 64-B aligned places (short record runs)
//   kw4    coalesced 4 B/lane stores (the encoding and J stores)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) kr16(const u32x4* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void __launch_bounds__(256) kr4(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    acc += __builtin_nontemporal_load(p + i);
  if (acc == 0x12345678u) out[0] = acc;
}
// one gather per thread into line (i * odd) mod lines (lines a power of two: a permutation, so every
// gather touches a line of its own)
__global__ void __launch_bounds__(256) kg4(const uint32_t* __restrict__ p, uint32_t lines, uint32_t g, uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= g) return;
  const uint32_t line = (i * 2654435761u) & (lines - 1u);
  const uint32_t v = p[(size_t)line * 32 + (i & 31)];
  if (v == 0x12345678u) out[0] = v;
}
__global__ void __launch_bounds__(256) kg4p(const uint32_t* __restrict__ p, uint32_t lines, uint32_t g, uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;  // pairs of lanes share one gather's 8-B pair
  if (i >= 2 * g) return;
  const uint32_t line = ((i >> 1) * 2654435761u) & (lines - 1u);
  const uint32_t v = p[(size_t)line * 32 + (((i >> 1) & 15) << 1) + (i & 1)];
  if (v == 0x12345678u) out[0] = v;
}
__global__ void __launch_bounds__(256) kw8(uint2* __restrict__ p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    p[i] = make_uint2((uint32_t)i, (uint32_t)(i >> 32));
}
__global__ void __launch_bounds__(256) kw8r(uint2* __restrict__ p, uint32_t slots, uint32_t runs) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;  // 8 lanes per 64-B run
  if (i >= 8 * runs) return;
  const uint32_t slot = ((i >> 3) * 2654435761u) & (slots - 1u);
  p[(size_t)slot * 8 + (i & 7)] = make_uint2(i, slot);
}
__global__ void __launch_bounds__(256) kw4(uint32_t* __restrict__ p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = (uint32_t)i;
}

int main() {
  const size_t bytes = size_t(2) << 30;  // 2 GiB
  void* buf;
  uint32_t* out;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  if (hipMemset(buf, 1, bytes) != hipSuccess) return 1;
  // a 1 GiB region per kernel, the other half written in between so no read starts L2/MALL-resident
  char* a = (char*)buf;
  char* b = a + (bytes / 2);
  const size_t half = bytes / 2;
  const uint32_t lines = (uint32_t)(half / 128);
  const uint32_t g = 1u << 22;  // 4 M gathers (512 MB of lines if 128 B each) out of 8 M lines
  auto flush = [&]() { hipLaunchKernelGGL(kw4, dim3(8192), dim3(256), 0, 0, (uint32_t*)b, half / 4); };
  for (int rep = 0; rep < 2; ++rep) {
    flush();
    hipLaunchKernelGGL(kr16, dim3(8192), dim3(256), 0, 0, (const u32x4*)a, half / 16, out);
    flush();
    hipLaunchKernelGGL(kr4, dim3(8192), dim3(256), 0, 0, (const uint32_t*)a, half / 4, out);
    flush();
    hipLaunchKernelGGL(kg4, dim3(g / 256), dim3(256), 0, 0, (const uint32_t*)a, lines, g, out);
    flush();
    hipLaunchKernelGGL(kg4p, dim3(2 * g / 256), dim3(256), 0, 0, (const uint32_t*)a, lines, g, out);
    flush();
    hipLaunchKernelGGL(kw8, dim3(8192), dim3(256), 0, 0, (uint2*)a, half / 8);
    flush();
    hipLaunchKernelGGL(kw8r, dim3(8 * g / 256), dim3(256), 0, 0, (uint2*)a, (uint32_t)(half / 64), g);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"kr16_read_bytes\": %zu, \"kr4_read_bytes\": %zu, \"kg4_gathers\": %u, \"kg4p_gathers\": %u, "
         "\"kw8_write_bytes\": %zu, \"kw8r_runs_64B\": %u, \"kw4_write_bytes\": %zu}\n",
         half, half, g, g, half, g, half);
  return (hipFree(buf) == hipSuccess && hipFree(out) == hipSuccess) ? 0 : 3;
}
