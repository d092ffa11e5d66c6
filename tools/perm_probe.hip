// perm_probe.hip — is a random permutation of 100-B records cheaper as a gather (read random,
// write in order: today's reduce-sort gather) or as a scatter (read in order, write random)?
// 5 M records (500 MB, the bench's reduce partition), a random permutation; each record is
// moved by a 32-lane half-wave, 25 dwords (records are 4-byte aligned at 100-B strides).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/perm_probe tools/perm_probe.hip
// Prints one JSON line per kernel: mean ms over 10 launches after 2 warm-ups.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr uint32_t kRecWords = 25;  // 100 B

// out[o] = in[src[o]]
__global__ __launch_bounds__(256) void k_gather(const uint32_t* __restrict__ in,
                                                uint32_t* __restrict__ out,
                                                const uint32_t* __restrict__ src, uint32_t n) {
  const uint32_t half = (blockIdx.x * 256u + threadIdx.x) / 32u, l = threadIdx.x % 32u;
  const uint32_t halves = gridDim.x * 8u;
  for (uint32_t o = half; o < n; o += halves) {
    const uint32_t s = src[o];
    if (l < kRecWords) out[(uint64_t)o * kRecWords + l] = in[(uint64_t)s * kRecWords + l];
  }
}

// out[dst[i]] = in[i]
__global__ __launch_bounds__(256) void k_scatter(const uint32_t* __restrict__ in,
                                                 uint32_t* __restrict__ out,
                                                 const uint32_t* __restrict__ dst, uint32_t n) {
  const uint32_t half = (blockIdx.x * 256u + threadIdx.x) / 32u, l = threadIdx.x % 32u;
  const uint32_t halves = gridDim.x * 8u;
  for (uint32_t i = half; i < n; i += halves) {
    const uint32_t d = dst[i];
    if (l < kRecWords) out[(uint64_t)d * kRecWords + l] = in[(uint64_t)i * kRecWords + l];
  }
}

// out[i] = in[i] (the copy ceiling of the same shape)
__global__ __launch_bounds__(256) void k_copy(const uint32_t* __restrict__ in,
                                              uint32_t* __restrict__ out, uint32_t n) {
  const uint32_t half = (blockIdx.x * 256u + threadIdx.x) / 32u, l = threadIdx.x % 32u;
  const uint32_t halves = gridDim.x * 8u;
  for (uint32_t i = half; i < n; i += halves)
    if (l < kRecWords) out[(uint64_t)i * kRecWords + l] = in[(uint64_t)i * kRecWords + l];
}

int main() {
  const uint32_t n = 5000000;
  std::vector<uint32_t> perm(n), inv(n);
  std::iota(perm.begin(), perm.end(), 0u);
  std::mt19937_64 rng(7);
  std::shuffle(perm.begin(), perm.end(), rng);
  for (uint32_t o = 0; o < n; ++o) inv[perm[o]] = o;
  uint32_t *in, *out, *src, *dst;
  CK(hipMalloc(&in, (size_t)n * 100));
  CK(hipMalloc(&out, (size_t)n * 100));
  CK(hipMalloc(&src, (size_t)n * 4));
  CK(hipMalloc(&dst, (size_t)n * 4));
  CK(hipMemset(in, 0x5a, (size_t)n * 100));
  CK(hipMemcpy(src, perm.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dst, inv.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (uint32_t wpc : {8u, 16u, 32u}) {  // workgroups per CU
    const dim3 grid(ncu * wpc);
    auto time = [&](const char* name, auto&& launch) {
      for (int w = 0; w < 2; ++w) launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < 10; ++r) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipDeviceSynchronize());
      CK(hipGetLastError());
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 10;
      printf("{\"kernel\": \"%s\", \"wg_per_cu\": %u, \"records\": %u, \"ms\": %.4f, "
             "\"GBps_of_2x500MB\": %.1f}\n", name, wpc, n, ms, 2.0 * n * 100 / ms / 1e6);
      fflush(stdout);
    };
    time("copy", [&] { hipLaunchKernelGGL(k_copy, grid, dim3(256), 0, 0, in, out, n); });
    time("gather", [&] { hipLaunchKernelGGL(k_gather, grid, dim3(256), 0, 0, in, out, src, n); });
    time("scatter", [&] { hipLaunchKernelGGL(k_scatter, grid, dim3(256), 0, 0, in, out, dst, n); });
  }
  return 0;
}
