// mall_probe.hip — does a map batch read by the histogram pass stay in the 256 MiB Infinity
// Cache (MALL) for the scatter pass that follows it?  (MI355X, gfx950)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mall_probe tools/mall_probe.hip
// For slice sizes of 32 MB .. 1 GB walked through a 16 GB buffer (every slice fresh, so no
// repetition hits the cache by accident) it times, per slice:
//   read        one streaming read of the slice (the histogram pass alone)
//   copy        a streaming copy slice -> out (the scatter pass alone, cold input)
//   read+copy   read of the slice, then its copy (the two-pass map side)
// If the copy after the read runs faster than the cold copy, the MALL served the re-read.
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

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    u32x4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
// per-wave contiguous ranges of `per` units (the hist kernel's tile walk), 8 loads in flight
__global__ __launch_bounds__(256) void k_read_tiles(const u32x4* __restrict__ a, size_t n,
                                                    size_t per, uint32_t* sink) {
  const size_t w = (blockIdx.x * 256ull + threadIdx.x) / 64, lane = threadIdx.x % 64;
  uint32_t acc = 0;
  const size_t b = w * per, e = b + per < n ? b + per : n;
  for (size_t i = b + lane; i < e; i += 64 * 8) {
    u32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = a[i + 64 * k < e ? i + 64 * k : i];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

int main(int argc, char** argv) {
  const size_t total = (argc > 1 ? atoll(argv[1]) : 16000) * 1000000ull;
  uint8_t *a, *b;
  uint32_t* sink;
  CK(hipMalloc(&a, total));
  CK(hipMalloc(&b, total));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(a, 1, total));
  CK(hipMemset(b, 2, total));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int G = 256 * 8;
  const size_t sizes[] = {32u << 20, 64u << 20, 100000000, 128u << 20, 200000000, 256u << 20,
                          400000000, 838860800, 1u << 30};
  printf("%10s %9s %9s %9s %9s %9s %9s %9s | %s\n", "slice_MB", "read", "tiles", "copy", "rd+copy",
         "copy|rd", "rd+rd", "rd|rd", "GB/s: read=S/t copy=2S/t rd+copy=3S/t copy|rd=2S/(t_rd+copy - t_read) rd|rd=S/(t_rd+rd - t_read)");
  for (size_t S : sizes) {
    const size_t n4 = S / 16, slices = total / S;
    float t_read = 0, t_tiles = 0, t_copy = 0, t_both = 0, t_rr = 0;
    for (int mode = 0; mode < 5; ++mode) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (size_t s = 0; s < slices; ++s) {
        const u32x4* src = reinterpret_cast<const u32x4*>(a + s * S);
        u32x4* dst = reinterpret_cast<u32x4*>(b + s * S);
        if (mode == 0 || mode == 3 || mode == 4)
          hipLaunchKernelGGL(k_read, dim3(G), dim3(256), 0, 0, src, n4, sink);
        if (mode == 4) hipLaunchKernelGGL(k_read, dim3(G), dim3(256), 0, 0, src, n4, sink);
        if (mode == 1) {
          const size_t per = 6400;  // 100 KB per wave
          const size_t waves = (n4 + per - 1) / per;
          hipLaunchKernelGGL(k_read_tiles, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, 0, src,
                             n4, per, sink);
        }
        if (mode == 2 || mode == 3) hipLaunchKernelGGL(k_copy, dim3(G), dim3(256), 0, 0, src, dst, n4);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= slices;
      (mode == 0 ? t_read : mode == 1 ? t_tiles : mode == 2 ? t_copy : mode == 3 ? t_both : t_rr) = ms;
    }
    auto g = [](double bytes, float ms) { return bytes / (ms * 1e-3) / 1e9; };
    printf("%10.1f %9.1f %9.1f %9.1f %9.1f %9.1f %9.1f %9.1f\n", S / 1e6, g(S, t_read), g(S, t_tiles),
           g(2.0 * S, t_copy), g(3.0 * S, t_both), g(2.0 * S, t_both - t_read), g(2.0 * S, t_rr),
           g(S, t_rr - t_read));
  }
  return 0;
}
