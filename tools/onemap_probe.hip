// onemap_probe — the ceiling of a ONE-READ map side at the headline's map size.
//
// The two-kernel map side reads every 100-byte record twice (K1 for the histogram, K3 to place
// it).  A one-read design must hold a whole map on chip while its histogram forms: a 2^20-record
// TeraSort map is 100 MB = 400 KB per CU on 256 CUs, which fits only in the register file
// (512 KB per CU).  This probe runs that design's memory skeleton and nothing else:
//   1. load: each CU's 512 threads load the CU's 4096 records (409,600 B, 50 16-byte units per
//      thread, coalesced): 34 units per thread into registers, 16 through registers into LDS
//      (128 KB) — all 50 in registers leave no room to work (256 VGPRs, scratch spills);
//   2. place: a partition per record (a hash, uniform over R = 200: the key lookup is left out),
//      its rank among the CU's records of that partition (LDS atomics), the CU's 200 counts
//      published write-through (sc1) -> grid barrier -> CU p < R scans column p over the 256 CUs
//      -> grid barrier -> each CU reads its 200 offsets and the 200 totals;
//   3. write: every unit stored from registers to its final place (runs of ~20 records = 2 KB
//      per (CU, partition), 4-byte phases, 16-byte stores; the one or two units that straddle two
//      records go as dwords).
// Modes: 0 = all of it; 1 = no grid barriers (each CU places its records in its own 400 KB
// output window, partition-sorted: the same write pattern without the synchronisation) — the
// difference is the price of the two barriers and the count exchange per map.
// A sum of every 4-byte word in and out checks the output is a permutation.
//
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/onemap_probe.hip -o tools/onemap_probe
// run:   tools/onemap_probe [maps=32]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

// REC records per CU: 4096 = a 2^20-record map on 256 CUs (the headline's maps); 2048 = 2^19.
#ifndef ONEMAP_REC
#define ONEMAP_REC 2048
#endif
constexpr uint32_t S = 100, R = 200, REC = ONEMAP_REC, NT = 256, UNITS = REC * S / 16,
                   PER = UNITS / NT;
constexpr uint32_t PL = 32, PR = PER - PL;  // units per thread held in LDS / in registers
static_assert(UNITS % NT == 0, "units per thread");

__device__ __forceinline__ uint32_t hash_pid(uint64_t g) {
  uint64_t z = g * 0x9E3779B97F4A7C15ull;
  z ^= z >> 31;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 29;
  return (uint32_t)((z >> 32) % R);
}

// Grid barrier on a monotonic counter, MI355X_MICROARCH.md's hand-off row 1: the payload was
// stored write-through (sc1) and every storing wave drained its stores (vmcnt(0)) before the
// workgroup barrier; one lane adds (agent scope) and polls with sc1 loads; the payload is read
// with sc1 loads after the closing workgroup barrier.  Bounded: err set, wait abandoned after ~1 s.
__device__ bool grid_sync(unsigned* ctr, unsigned target, unsigned* err) {
  __shared__ unsigned failed;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    failed = 0;
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        failed = 1;
        break;
      }
    }
  }
  __syncthreads();
  return failed == 0;  // a timed-out barrier ends the workgroup (every one leaves in ~1 s)
}

template <int MODE>
__global__ __launch_bounds__(NT, 1) void k_onemap(const u32x4* __restrict__ in,
                                                  uint8_t* __restrict__ out, uint32_t maps,
                                                  uint32_t* counts, uint32_t* pre,
                                                  unsigned* sync, unsigned* err) {
  __shared__ uint32_t cnt[R], off[R], tot[R];
  __shared__ uint32_t dst[REC];  // the byte offset of each record in the map's output
  __shared__ uint32_t ssum[NT / 64 + 1];
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_stage[];  // [PL][NT] u32x4
  u32x4* stage = reinterpret_cast<u32x4*>(lds_stage);
  const uint32_t tid = threadIdx.x, w = blockIdx.x, G = gridDim.x;
  for (uint32_t m = 0; m < maps; ++m) {
    // 1. the CU's records of map m into registers
    const u32x4* src = in + ((uint64_t)m * G + w) * UNITS;
    u32x4 v[PR];
#pragma unroll
    for (uint32_t k = 0; k < PL; ++k) stage[tid + k * NT] = src[tid + (PR + k) * NT];
#pragma unroll
    for (uint32_t k = 0; k < PR; ++k) v[k] = src[tid + k * NT];
    // 2. partition + rank per record (8 records per thread)
    for (uint32_t p = tid; p < R; p += NT) cnt[p] = 0;
    __syncthreads();
    uint32_t rp[REC / NT], rr[REC / NT];
#pragma unroll
    for (uint32_t j = 0; j < REC / NT; ++j) {
      const uint32_t r = tid + j * NT;
      rp[j] = hash_pid(((uint64_t)m * G + w) * REC + r);
      rr[j] = atomicAdd(&cnt[rp[j]], 1u);
    }
    __syncthreads();
    if (MODE == 0) {
      for (uint32_t p = tid; p < R; p += NT)
        __hip_atomic_store(&counts[(uint64_t)w * R + p], cnt[p], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      if (!grid_sync(&sync[2 * m], G, err)) return;
      // column scan: CU p < R owns partition p
      if (w < R) {
        uint32_t acc = 0;
        for (uint32_t b0 = 0; b0 < G; b0 += NT) {
          const uint32_t b = b0 + tid;
          const uint32_t c = b < G ? __hip_atomic_load(&counts[(uint64_t)b * R + w], __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : 0u;
          // block exclusive scan of c
          uint32_t x = c;
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d);
            if ((tid & 63) >= (uint32_t)d) x += y;
          }
          if ((tid & 63) == 63) ssum[tid / 64] = x;
          __syncthreads();
          uint32_t before = acc, all = 0;
          for (uint32_t q = 0; q < NT / 64; ++q) {
            before += q < tid / 64 ? ssum[q] : 0u;
            all += ssum[q];
          }
          if (b < G)
            __hip_atomic_store(&pre[(uint64_t)b * (R + 1) + w], before + x - c, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          acc += all;
          __syncthreads();
        }
        if (tid == 0)
          __hip_atomic_store(&pre[(uint64_t)G * (R + 1) + w], acc, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      if (!grid_sync(&sync[2 * m + 1], G, err)) return;
      for (uint32_t p = tid; p < R; p += NT) {
        off[p] = __hip_atomic_load(&pre[(uint64_t)w * (R + 1) + p], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        tot[p] = __hip_atomic_load(&pre[(uint64_t)G * (R + 1) + p], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (tid == 0) {  // exclusive scan of the totals (200 entries, one lane: cheap at this size)
        uint32_t a = 0;
        for (uint32_t p = 0; p < R; ++p) {
          const uint32_t t = tot[p];
          tot[p] = a;
          a += t;
        }
      }
      __syncthreads();
#pragma unroll
      for (uint32_t j = 0; j < REC / NT; ++j)
        dst[tid + j * NT] = (tot[rp[j]] + off[rp[j]] + rr[j]) * S;
    } else {
      // the CU's own window, partition-sorted (same run structure, no cross-CU exchange)
      if (tid == 0) {
        uint32_t a = 0;
        for (uint32_t p = 0; p < R; ++p) {
          off[p] = a;
          a += cnt[p];
        }
      }
      __syncthreads();
#pragma unroll
      for (uint32_t j = 0; j < REC / NT; ++j)
        dst[tid + j * NT] = ((uint32_t)w * REC + off[rp[j]] + rr[j]) * S;
    }
    __syncthreads();
    // 3. every unit from registers to its place
    uint8_t* mo = out + (uint64_t)m * G * REC * S;
    auto put = [&](uint32_t u, const u32x4& x) {
      const uint32_t b = 16 * u, r = b / S, o = b - r * S;
      if (o + 16 <= S) {
        *reinterpret_cast<u32x4a4*>(mo + dst[r] + o) = x;  // 4-byte aligned 16-byte store
      } else {
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
          const uint32_t bb = b + 4 * q, rq = bb / S, oq = bb - rq * S;
          *reinterpret_cast<uint32_t*>(mo + dst[rq] + oq) = x[q];
        }
      }
    };
#pragma unroll
    for (uint32_t k = 0; k < PR; ++k) put(tid + k * NT, v[k]);
#pragma unroll 4
    for (uint32_t k = 0; k < PL; ++k) put(tid + (PR + k) * NT, stage[tid + k * NT]);
    __syncthreads();
  }
}

__global__ void k_sum(const uint32_t* p, uint64_t n, unsigned long long* acc) {
  uint64_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    s += p[i];
  atomicAdd(acc, (unsigned long long)s);
}

int main(int argc, char** argv) {
  const uint32_t maps = argc > 1 ? (uint32_t)atoi(argv[1]) : 32;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t G = (uint32_t)ncu;  // one workgroup per CU: every one resident (barriers)
  const uint64_t per_map = (uint64_t)G * REC * S, bytes = per_map * maps;
  printf("onemap_probe: %u CUs, %u maps of %u records (%.1f MB each), %.2f GB\n", G, maps, G * REC,
         per_map / 1e6, bytes / 1e9);
  uint8_t *in = nullptr, *out = nullptr;
  uint32_t *counts = nullptr, *pre = nullptr;
  unsigned *sync = nullptr, *err = nullptr;
  unsigned long long* acc = nullptr;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&counts, (size_t)G * R * 4));
  CK(hipMalloc(&pre, (size_t)(G + 1) * (R + 1) * 4));
  CK(hipMalloc(&sync, (size_t)2 * maps * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&acc, 16));
  {
    std::vector<uint32_t> h(1 << 24);
    uint64_t z = 12345;
    for (auto& x : h) {
      z = z * 6364136223846793005ull + 1442695040888963407ull;
      x = (uint32_t)(z >> 33);
    }
    for (uint64_t o = 0; o < bytes; o += h.size() * 4)
      CK(hipMemcpy(in + o, h.data(), std::min<uint64_t>(h.size() * 4, bytes - o),
                   hipMemcpyHostToDevice));
  }
  CK(hipMemset(err, 0, 4));
  constexpr size_t kStage = (size_t)PL * NT * 16;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_onemap<0>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStage));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_onemap<1>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStage));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemset(sync, 0, (size_t)2 * maps * 4));
      CK(hipMemset(out, 0, bytes));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      if (mode == 0)
        hipLaunchKernelGGL(k_onemap<0>, dim3(G), dim3(NT), kStage, 0, reinterpret_cast<const u32x4*>(in),
                           out, maps, counts, pre, sync, err);
      else
        hipLaunchKernelGGL(k_onemap<1>, dim3(G), dim3(NT), kStage, 0, reinterpret_cast<const u32x4*>(in),
                           out, maps, counts, pre, sync, err);
      CK(hipGetLastError());
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned herr = 0;
      CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      CK(hipMemset(acc, 0, 16));
      hipLaunchKernelGGL(k_sum, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const uint32_t*>(in),
                         bytes / 4, acc);
      hipLaunchKernelGGL(k_sum, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const uint32_t*>(out),
                         bytes / 4, acc + 1);
      unsigned long long sums[2];
      CK(hipMemcpy(sums, acc, 16, hipMemcpyDeviceToHost));
      printf("mode %d (%s) rep %d: %.3f ms = %.2f us per map, %.2f TB/s of read+write, %s%s\n",
             mode, mode == 0 ? "load, 2 grid barriers + count scan, write" : "load, write (no barriers)",
             rep, ms, 1e3 * ms / maps, 2.0 * bytes / (ms * 1e-3) / 1e12,
             sums[0] == sums[1] ? "permutation ok" : "SUM MISMATCH", herr ? " BARRIER TIMEOUT" : "");
      if (herr) return 2;
    }
  }
  return 0;
}
