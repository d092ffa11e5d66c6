// msd_split_probe.hip — could C5's two passes overlap on disjoint CUs?  (The 100-B path's split
// mode runs K1 on a few CUs beside K3 on the rest because K1 holds its rate on few CUs.)
// Times the product's pass A (k_msd16a) and pass B (k_msd16b, msd_direct 24: 32-partition
// buckets, element map) of one C5 launch group — 200 maps x 2^20 random 16-byte records, Spark
// SQL murmur3 of the int64 key, R = 10 000 — alone on CU-masked streams of C CUs, and both at
// once: pass A of one buffer set on C CUs while pass B of another set runs on the other 256 - C.
// Every launch is the product's kernel on the product's data; pass B reads a pass A output made
// by the product's own sequence (pass A, scan) first.
// Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I sparkucx_amd/csrc \
//         -o tools/msd_split_probe tools/msd_split_probe.hip
// Prints one JSON line per measurement.
#include "../sparkucx_amd/csrc/sux_small.hip"

#include <hip/hip_ext.h>

#include <cstdio>
#include <vector>

namespace sux {
int stream_cus(hipStream_t) { return 256; }
void timer_note(Timer*, int, const char*) {}
void timer_begin(Timer*, int, hipStream_t) {}
void timer_end(Timer*, int, hipStream_t) {}
}  // namespace sux

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void k_fill(uint64_t* p, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x1234567ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

using namespace sux;
constexpr uint32_t R = 10000, S = 16, DB = 9, NWA = 8, NWB = 8, PTB = 8;
using MB = M16b<NWB, PTB, kM16LoWide, kM16MaxChunks>;

// the CU mask of the library's create_cu_stream: bits 0..C-1 (round robin over XCD / SE)
static hipStream_t cu_stream(uint32_t C, bool complement, uint32_t P) {
  hipStream_t st;
  if (C == 0 || C == P) {
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    return st;
  }
  std::vector<uint32_t> mask((P + 31) / 32, 0u);
  for (uint32_t i = 0; i < P; ++i)
    if ((i < C) != complement) mask[i / 32] |= 1u << (i % 32);
  CK(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
  return st;
}

struct Set {
  uint8_t *tmp, *out, *ibe;
  int64_t* idx;
  uint16_t* offs;
  uint64_t* segbase;
};

int main() {
  const uint64_t rpm = 1 << 20, maps = 200, n = rpm * maps;
  const uint32_t cpm = (uint32_t)(rpm / kM16Chunk), nbk = (R + 31) / 32;
  uint8_t* recs;
  CK(hipMalloc(&recs, n * S));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(recs), n * S / 8);
  Set set[2];
  for (Set& x : set) {
    CK(hipMalloc(&x.tmp, n * S));
    CK(hipMalloc(&x.out, n * S));
    CK(hipMalloc(&x.idx, maps * (R + 1) * 8));
    CK(hipMalloc(&x.ibe, maps * (R + 1) * 8));
    CK(hipMalloc(&x.offs, maps * cpm * nbk * 2));
    CK(hipMalloc(&x.segbase, maps * nbk * 8));
  }
  PartDev pd{};
  pd.kind = 2;
  pd.R = R;
  pd.key_offset = 0;
  pd.key_len = 8;
  pd.seed = 42;
  pd.ascending = 1;
  pd.rmagic = part_magic(pd.R);
  MapGroup g{};
  g.recs = recs;
  g.records_per_map = rpm;
  g.num_records = n;
  g.num_maps = (uint32_t)maps;
  g.rec_size = S;
  int P = 0;
  CK(hipDeviceGetAttribute(&P, hipDeviceAttributeMultiprocessorCount, 0));
  constexpr size_t lda = M16a<NWA, DB>::lds_bytes(), ldb = MB::lds_bytes();
  auto* ka = &k_msd16a<2, NWA, DB, kM16LoWide, false>;
  auto* kb = &k_msd16b<2, NWB, PTB, kM16LoWide, kM16MaxChunks, false, true, false>;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(ka), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lda));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kb), hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldb));
  auto pass_a = [&](Set& x, uint32_t C, hipStream_t s) {
    hipLaunchKernelGGL(ka, dim3(std::min<uint32_t>(maps * cpm, C * 2)), dim3(NWA * kWave), lda, s,
                       pd, g, cpm, nbk, x.offs, (uint16_t*)nullptr, x.tmp);
  };
  auto scan = [&](Set& x, hipStream_t s) {
    hipLaunchKernelGGL(k_msd16_scan, dim3(maps), dim3(kScanThreads), 0, s, g, cpm, nbk, x.offs,
                       x.segbase, x.idx, x.ibe, (uint64_t*)nullptr, (int)R);
  };
  auto pass_b = [&](Set& x, uint32_t C, hipStream_t s) {
    hipLaunchKernelGGL(kb, dim3(std::min<uint32_t>(maps * nbk, C * 2)), dim3(NWB * kWave), ldb, s,
                       pd, g, cpm, nbk, x.offs, x.segbase, x.tmp, x.out, x.idx, x.ibe);
  };
  // both sets hold a complete pass A + scan output (pass B's input)
  for (Set& x : set) {
    pass_a(x, P, 0);
    scan(x, 0);
    pass_b(x, P, 0);
  }
  CK(hipDeviceSynchronize());
  CK(hipGetLastError());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  constexpr int reps = 4;
  auto time_on = [&](hipStream_t s, auto&& fn) {
    fn();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) fn();
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
  };
  const double gb = 32.0 * n / 1e9;  // algorithmic bytes of one pass
  for (uint32_t C : {64u, 96u, 128u, 160u, 192u, 256u}) {
    hipStream_t s = cu_stream(C, false, (uint32_t)P);
    const float ta = time_on(s, [&] { pass_a(set[0], C, s); });
    const float tb = time_on(s, [&] { pass_b(set[1], C, s); });
    CK(hipGetLastError());
    printf("{\"what\": \"alone\", \"cus\": %u, \"pass_a_ms\": %.4f, \"pass_a_TBps\": %.3f, "
           "\"pass_b_ms\": %.4f, \"pass_b_TBps\": %.3f}\n",
           C, ta, gb / ta, tb, gb / tb);
    fflush(stdout);
    CK(hipStreamDestroy(s));
  }
  // pass A (set 0) on C CUs and pass B (set 1) on the other CUs at once; `reps` of each, each
  // stream back to back; the wall time of both
  for (uint32_t C : {64u, 96u, 128u, 160u}) {
    hipStream_t sa = cu_stream(C, false, (uint32_t)P), sb = cu_stream(C, true, (uint32_t)P);
    CK(hipDeviceSynchronize());
    hipEvent_t a0, a1, b1;
    CK(hipEventCreate(&a0));
    CK(hipEventCreate(&a1));
    CK(hipEventCreate(&b1));
    CK(hipEventRecord(a0, sa));
    CK(hipStreamWaitEvent(sb, a0, 0));
    for (int r = 0; r < reps; ++r) {
      pass_a(set[0], C, sa);
      pass_b(set[1], (uint32_t)P - C, sb);
    }
    CK(hipEventRecord(a1, sa));
    CK(hipEventRecord(b1, sb));
    CK(hipDeviceSynchronize());
    CK(hipGetLastError());
    float ta = 0, tb = 0;
    CK(hipEventElapsedTime(&ta, a0, a1));
    CK(hipEventElapsedTime(&tb, a0, b1));
    printf("{\"what\": \"together\", \"pass_a_cus\": %u, \"pass_b_cus\": %u, \"pass_a_ms\": %.4f, "
           "\"pass_b_ms\": %.4f, \"wall_ms_per_pair\": %.4f}\n",
           C, (uint32_t)P - C, ta / reps, tb / reps, std::max(ta, tb) / reps);
    fflush(stdout);
    CK(hipStreamDestroy(sa));
    CK(hipStreamDestroy(sb));
  }
  return 0;
}
