// copy_probe.hip — the HBM copy ceiling the map-side kernels are judged against (MI355X, gfx950).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/copy_probe tools/copy_probe.hip
//
// Round 1's probe (tools/hbm_probe.hip) issued ONE 16-byte load per lane per loop trip and read
// 5.0 TB/s for a copy; MI355X_MICROARCH.md quotes 6.29 TB/s for a float4 copy.  This probe sweeps
// the loads a lane keeps in flight (U = 1..16 units of 16 B, all issued before the first store),
// the workgroup shape and the grid, plus non-temporal stores, and prints GB/s of read+write bytes
// (1e9 B/s) so the scatter's roofline fraction can be read against a measured copy ceiling.
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

// Each workgroup copies blocks of NT*U units: thread t loads units t, t+NT, ..., t+(U-1)NT of the
// block (one coalesced 1 KiB wave-instruction each), then stores them.  Grid-stride over blocks.
template <int NT, int U, bool NTS>
__global__ __launch_bounds__(NT) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b,
                                             size_t nblk) {
  for (size_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const size_t base = blk * (size_t)(NT * U) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = a[base + (size_t)k * NT];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if constexpr (NTS) __builtin_nontemporal_store(v[k], &b[base + (size_t)k * NT]);
      else b[base + (size_t)k * NT] = v[k];
    }
  }
}

template <int NT, int U>
__global__ __launch_bounds__(NT) void k_read(const u32x4* __restrict__ a, size_t nblk,
                                             uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const size_t base = blk * (size_t)(NT * U) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = a[base + (size_t)k * NT];
#pragma unroll
    for (int k = 0; k < U; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int NT, int U>
__global__ __launch_bounds__(NT) void k_write(u32x4* __restrict__ b, size_t nblk) {
  for (size_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const size_t base = blk * (size_t)(NT * U) + threadIdx.x;
#pragma unroll
    for (int k = 0; k < U; ++k) b[base + (size_t)k * NT] = u32x4{(uint32_t)base, 1u, 2u, (uint32_t)k};
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
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

static u32x4 *A, *B;
static uint32_t* SINK;
static size_t BYTES;

template <int NT, int U, bool NTS>
static void copy_case(int per_cu) {
  const size_t nblk = BYTES / (16ull * NT * U);
  const unsigned grid = 256u * per_cu;
  const float t = time_it([&] { hipLaunchKernelGGL((k_copy<NT, U, NTS>), dim3(grid), dim3(NT), 0, 0,
                                                     A, B, nblk); }, 10);
  const double moved = 2.0 * nblk * NT * U * 16;
  printf("copy  NT=%4d U=%2d grid=256x%-2d %s %8.1f GB/s\n", NT, U, per_cu, NTS ? "nt " : "   ",
         moved / (t * 1e-3) / 1e9);
}

template <int NT, int U>
static void read_case(int per_cu) {
  const size_t nblk = BYTES / (16ull * NT * U);
  const float t = time_it([&] { hipLaunchKernelGGL((k_read<NT, U>), dim3(256 * per_cu), dim3(NT), 0, 0,
                                                     A, nblk, SINK); }, 10);
  printf("read  NT=%4d U=%2d grid=256x%-2d    %8.1f GB/s\n", NT, U, per_cu,
         (double)nblk * NT * U * 16 / (t * 1e-3) / 1e9);
}

template <int NT, int U>
static void write_case(int per_cu) {
  const size_t nblk = BYTES / (16ull * NT * U);
  const float t = time_it([&] { hipLaunchKernelGGL((k_write<NT, U>), dim3(256 * per_cu), dim3(NT), 0, 0,
                                                     B, nblk); }, 10);
  printf("write NT=%4d U=%2d grid=256x%-2d    %8.1f GB/s\n", NT, U, per_cu,
         (double)nblk * NT * U * 16 / (t * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
  BYTES = (argc > 1 ? atoll(argv[1]) : 3355) * 1000000ull;  // default: one 32-map launch group
  BYTES = BYTES / (1u << 20) * (1u << 20);
  CK(hipMalloc(&A, BYTES));
  CK(hipMalloc(&B, BYTES));
  CK(hipMalloc(&SINK, 4));
  CK(hipMemset(A, 1, BYTES));
  CK(hipMemset(B, 2, BYTES));
  printf("buffer %.2f GB\n", BYTES / 1e9);
  for (int pc : {1, 2, 4, 8}) {
    read_case<256, 4>(pc);
    read_case<256, 8>(pc);
  }
  for (int pc : {2, 4, 8}) {
    write_case<256, 4>(pc);
    write_case<256, 8>(pc);
  }
  for (int pc : {1, 2, 4, 8}) {
    copy_case<256, 1, false>(pc);
    copy_case<256, 4, false>(pc);
    copy_case<256, 8, false>(pc);
    copy_case<256, 16, false>(pc);
    copy_case<256, 8, true>(pc);
  }
  for (int pc : {1, 2}) {
    copy_case<1024, 4, false>(pc);
    copy_case<1024, 8, false>(pc);
    copy_case<512, 8, false>(pc);
  }
  return 0;
}
