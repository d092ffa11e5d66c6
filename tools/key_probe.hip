// key_probe.hip — can K1 fetch less than the whole 100-byte record to read its 10-byte key?
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/key_probe tools/key_probe.hip
//
// K1 (k_hist4) streams every byte of a TeraSort record (100 B) to get the 10-byte key at its
// start, so the map side moves 100 B in K1 + 200 B in K3 per record.  The key of record i lies at
// [100i, 100i + 10): one or two 32-byte sectors (or one/two 64-byte halves) of its 128-byte line.
// If the L2 -> fabric path fetches sectors, not whole lines, a key-only pass reads ~40 B (32-B
// sectors) or ~68 B (64-B halves) per record.  This probe times, over the same 3.36 GB buffer:
//   read_all  — the whole buffer, 16-B units, 8 per lane in flight (the streaming ceiling);
//   key3      — the 3 key dwords of every record (lane l of a wave: record base + 64k + l);
//   key1      — the first key dword only;
//   key3_nt   — key3 with non-temporal loads.
// and prints the time and the "record bytes per second" (records x 100 B / t).  Run it once
// plain and once per PMC pass (FETCH_SIZE; TCC_EA0_RDREQ_32B_sum / TCC_EA0_RDREQ_sum) to read
// the bytes each variant actually fetches.
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
__global__ __launch_bounds__(256) void k_read_all(const u32x4* __restrict__ a, size_t nblk,
                                                  uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const size_t base = blk * (size_t)(256 * U) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = a[base + (size_t)k * 256];
#pragma unroll
    for (int k = 0; k < U; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// KW key dwords of every record; a workgroup block = 256 * U records, wave w / lane l / step k
// -> record blk * 256U + w * 64U + 64k + l (each wave instruction spans 64 consecutive records).
template <int U, int KW, bool NT>
__global__ __launch_bounds__(256) void k_keys(const uint8_t* __restrict__ recs, size_t nrec,
                                              uint32_t* sink) {
  uint32_t acc = 0;
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const size_t nblk = nrec / (256 * U);
  for (size_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const size_t r0 = blk * (size_t)(256 * U) + (size_t)wave * 64 * U + lane;
    uint32_t v[U][KW];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(recs + (r0 + (size_t)k * 64) * 100);
#pragma unroll
      for (int q = 0; q < KW; ++q) v[k][q] = NT ? __builtin_nontemporal_load(p + q) : p[q];
    }
#pragma unroll
    for (int k = 0; k < U; ++k)
#pragma unroll
      for (int q = 0; q < KW; ++q) acc ^= v[k][q];
  }
  if (acc == 0x12345678u) sink[0] = acc;
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
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const size_t nrec = (argc > 1 ? atoll(argv[1]) : 32ll << 20);  // one 32-map launch group
  const size_t bytes = nrec * 100;
  uint8_t* A;
  uint32_t* sink;
  CK(hipMalloc(&A, bytes + 4096));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(A, 1, bytes));
  printf("records %zu (%.2f GB)\n", nrec, bytes / 1e9);
  auto report = [&](const char* name, float ms) {
    printf("%-22s %8.3f ms  %8.1f GB/s of record bytes\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  for (int pc : {2, 4, 8}) {
    const size_t nblk = bytes / (16ull * 256 * 8);
    char nm[64];
    snprintf(nm, sizeof nm, "read_all U8 x%d", pc);
    report(nm, time_it([&] { hipLaunchKernelGGL((k_read_all<8>), dim3(256 * pc), dim3(256), 0, 0,
                                                reinterpret_cast<const u32x4*>(A), nblk, sink); }, 10));
  }
  for (int pc : {2, 4, 8}) {
    char nm[64];
    snprintf(nm, sizeof nm, "key3 U8 x%d", pc);
    report(nm, time_it([&] { hipLaunchKernelGGL((k_keys<8, 3, false>), dim3(256 * pc), dim3(256), 0, 0,
                                                A, nrec, sink); }, 10));
    snprintf(nm, sizeof nm, "key3 U16 x%d", pc);
    report(nm, time_it([&] { hipLaunchKernelGGL((k_keys<16, 3, false>), dim3(256 * pc), dim3(256), 0, 0,
                                                A, nrec, sink); }, 10));
    snprintf(nm, sizeof nm, "key1 U16 x%d", pc);
    report(nm, time_it([&] { hipLaunchKernelGGL((k_keys<16, 1, false>), dim3(256 * pc), dim3(256), 0, 0,
                                                A, nrec, sink); }, 10));
    snprintf(nm, sizeof nm, "key3_nt U16 x%d", pc);
    report(nm, time_it([&] { hipLaunchKernelGGL((k_keys<16, 3, true>), dim3(256 * pc), dim3(256), 0, 0,
                                                A, nrec, sink); }, 10));
  }
  return 0;
}
