// hbm_probe.hip — HBM ceilings for the access patterns of the shuffle kernels (MI355X, gfx950).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.hip
// Prints GB/s (1e9 B/s) for: streaming read (x4), streaming write (x4), copy (x4 load + x4
// store), copy with dword stores, copy of 100-B records to permuted record slots (dword stores,
// record-coalesced), and strided key-dword reads at a 100-B stride.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_read(const u32x4* __restrict__ a, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    u32x4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void k_write(u32x4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    a[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}
__global__ void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}
__global__ void k_copy_dw(const uint32_t* __restrict__ a, uint32_t* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}
// record permutation: dword d of record r goes to record perm[r]; lanes walk dwords in order
__global__ void k_perm_dw(const uint32_t* __restrict__ a, uint32_t* __restrict__ b,
                          const uint32_t* __restrict__ perm, size_t nrec) {
  const size_t n = nrec * 25;
  for (size_t d = blockIdx.x * 256ull + threadIdx.x; d < n; d += (size_t)gridDim.x * 256) {
    size_t r = d / 25, w = d - r * 25;
    b[(size_t)perm[r] * 25 + w] = a[d];
  }
}
// strided key reads: 3 dwords at the start of every 100-B record
__global__ void k_keys(const uint32_t* __restrict__ a, size_t nrec, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t r = blockIdx.x * 256ull + threadIdx.x; r < nrec; r += (size_t)gridDim.x * 256) {
    const uint32_t* p = a + r * 25;
    acc ^= p[0] ^ p[1] ^ p[2];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// the scatter's write pattern: a 1024-thread workgroup copies 100 KB chunks (coalesced reads)
// and writes each as `runs` runs of 100KB/runs bytes, run r of chunk c at region r, offset c*len:
// consecutive chunks extend every region sequentially (as partition p's output does)
__global__ __launch_bounds__(1024) void k_runcopy(const u32x4* __restrict__ a, u32x4* __restrict__ b,
                                                  size_t n, uint32_t runs, uint32_t shift) {
  const uint32_t chunk_units = 6400, per_run = chunk_units / runs;  // 16-B units
  const size_t chunks = n / chunk_units, region = chunks * per_run;
  for (size_t c = blockIdx.x; c < chunks; c += gridDim.x) {
    for (uint32_t u = threadIdx.x; u < chunk_units; u += 1024) {
      const uint32_t r = u / per_run, k = u - r * per_run;
      if (r < runs) b[r * region + c * per_run + k + shift] = a[c * chunk_units + u];
    }
  }
}

template <class F>
static float time_it(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  size_t bytes = (argc > 1 ? atoll(argv[1]) : 4000) * 1000000ull;  // default 4 GB
  bytes = bytes / 1600 * 1600;
  const size_t n4 = bytes / 16, nrec = bytes / 100;
  uint8_t *a, *b;
  uint32_t *perm, *sink;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&perm, nrec * 4));
  CK(hipMemset(a, 1, bytes));
  // block-local permutation: records shuffled among 200 "partitions" of a 1024-record tile
  std::vector<uint32_t> hp(nrec);
  for (size_t t0 = 0; t0 < nrec; t0 += 1024) {
    size_t m = (nrec - t0 < 1024) ? nrec - t0 : 1024;
    for (size_t j = 0; j < m; ++j) hp[t0 + j] = (uint32_t)(t0 + (j * 797) % m);
  }
  CK(hipMemcpy(perm, hp.data(), nrec * 4, hipMemcpyHostToDevice));
  const int G = 256 * 16, reps = 10;
  auto gbs = [&](double moved, float ms) { return moved / (ms * 1e-3) / 1e9; };
  float t;
  t = time_it([&] { hipLaunchKernelGGL(k_read, dim3(G), dim3(256), 0, 0, (const u32x4*)a, n4, sink); }, reps);
  printf("read_x4        %8.1f GB/s\n", gbs(bytes, t));
  t = time_it([&] { hipLaunchKernelGGL(k_write, dim3(G), dim3(256), 0, 0, (u32x4*)b, n4); }, reps);
  printf("write_x4       %8.1f GB/s\n", gbs(bytes, t));
  t = time_it([&] { hipLaunchKernelGGL(k_copy, dim3(G), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, n4); }, reps);
  printf("copy_x4        %8.1f GB/s (read+write)\n", gbs(2.0 * bytes, t));
  t = time_it([&] { hipLaunchKernelGGL(k_copy_dw, dim3(G), dim3(256), 0, 0, (const uint32_t*)a, (uint32_t*)b, bytes / 4); }, reps);
  printf("copy_dword     %8.1f GB/s (read+write)\n", gbs(2.0 * bytes, t));
  t = time_it([&] { hipLaunchKernelGGL(k_perm_dw, dim3(G), dim3(256), 0, 0, (const uint32_t*)a, (uint32_t*)b, perm, nrec); }, reps);
  printf("perm100_dword  %8.1f GB/s (read+write)\n", gbs(2.0 * bytes, t));
  t = time_it([&] { hipLaunchKernelGGL(k_keys, dim3(G), dim3(256), 0, 0, (const uint32_t*)a, nrec, sink); }, reps);
  printf("keys100_read   %8.1f GB/s (record bytes / time)\n", gbs(bytes, t));
  for (uint32_t shift : {0u, 3u})
    for (uint32_t runs : {1u, 50u, 200u, 800u}) {
      t = time_it([&] { hipLaunchKernelGGL(k_runcopy, dim3(256 * 2), dim3(1024), 0, 0, (const u32x4*)a, (u32x4*)b, n4 - 8, runs, shift); }, reps);
      printf("runcopy %4u runs/100KB (%5u B runs) start+%2u B %8.1f GB/s (read+write)\n", runs, 102400 / runs, 16 * shift, gbs(2.0 * bytes, t));
    }
  return 0;
}
