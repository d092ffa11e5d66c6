// scatter_probe.hip — what scattered 16-byte record writes cost on MI355X (gfx950), to tell a
// ranking-bound small-record scatter from a write-bound one.  Reads 16-byte units in order and
// writes them permuted inside a window of W units (a map's output: 2^20 records = 16 MB): the
// window's units are cut into runs of L consecutive units and the runs are permuted by an affine
// bijection, so L = 1 is a record-by-record scatter (C5 at R = 10000 writes runs of ~0.4 record
// per 4096-record chunk) and larger L is what a coalescing pass would write.  Prints GB/s of
// read + write bytes (1e9 B/s), the same accounting as the kernels' roofline.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/scatter_probe tools/scatter_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void k_scatter(const u32x4* __restrict__ a, u32x4* __restrict__ b,
                                                 size_t n, uint32_t wbits, uint32_t lbits) {
  const uint64_t wmask = (1ull << wbits) - 1, runs = 1ull << (wbits - lbits);
  for (size_t blk = blockIdx.x; blk * 256 * U < n; blk += gridDim.x) {
    const size_t base = blk * (size_t)(256 * U) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = a[base + (size_t)k * 256];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t i = base + (uint64_t)k * 256;
      const uint64_t w = i & ~wmask, o = i & wmask;
      const uint64_t run = o >> lbits, in = o & ((1ull << lbits) - 1);
      const uint64_t prun = (run * 0x9E3779B1ull + 12345) & (runs - 1);  // odd multiplier: bijection
      b[w + (prun << lbits) + in] = v[k];
    }
  }
}

int main() {
  const size_t n = (size_t)1 << 30;  // 2^30 units = 17.2 GB each way (C5's bytes per step)
  u32x4 *a, *b;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, n * 16));
  CK(hipMemset(a, 1, n * 16));
  CK(hipMemset(b, 0, n * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t wbits = 20;
  for (uint32_t lbits : {0u, 1u, 2u, 3u, 4u, 5u, 6u, 8u, 12u, 20u}) {
    for (int grid : {2048, 8192}) {
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_scatter<4>), dim3(grid), dim3(256), 0, 0, a, b, n, wbits, lbits);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep && ms < best) best = ms;
      }
      printf("window 2^%u units, runs of %5u units (%6u B), grid %5d: %7.3f ms  %7.1f GB/s\n",
             wbits, 1u << lbits, 16u << lbits, grid, best, 2.0 * n * 16 / (best * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
