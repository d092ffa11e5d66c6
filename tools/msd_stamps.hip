// msd_stamps.hip — per-phase cycle profile of the two-level small-record pass B (k_msd16b),
// diagnostic build of sux_small.hip.  Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I sparkucx_amd/csrc \
//         -o tools/msd_stamps tools/msd_stamps.hip
// Runs pass A + scan + pass B over 200 maps x 2^20 16-byte random records (Spark SQL murmur3 of
// the int64 key, R = 10000, 16-partition buckets: 10-bit pass A digits) and prints the mean cycles per segment of each phase of pass B,
// over every workgroup:
//   0 load issue (run search)  1 rank + scan + stage (waits for the loads)  2 cursors + index
//   3 place (LDS -> HBM)       4 run table of the next segment
#define SUX_MSD_STAMPS 1
#include "../sparkucx_amd/csrc/sux_small.hip"

#include <cstdio>
#include <vector>

// host symbols sux_small.hip's launchers refer to (never called by this tool)
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

int main(int argc, char** argv) {
  using namespace sux;
  const uint32_t R = argc > 2 ? atoi(argv[2]) : 10000, S = 16;
  const uint64_t rpm = 1 << 20, maps = argc > 1 ? atoi(argv[1]) : 200, n = rpm * maps;
  uint8_t *recs, *out, *tmp, *ibe;
  int64_t* idx;
  uint16_t* offs;
  uint64_t* segbase;
  const uint32_t cpm = (uint32_t)(rpm / kM16Chunk), nbk = (R + 15) / 16;
  CK(hipMalloc(&recs, n * S));
  CK(hipMalloc(&out, n * S));
  CK(hipMalloc(&tmp, n * S));
  CK(hipMalloc(&idx, maps * (R + 1) * 8));
  CK(hipMalloc(&ibe, maps * (R + 1) * 8));
  CK(hipMalloc(&offs, maps * cpm * nbk * 2));
  CK(hipMalloc(&segbase, maps * nbk * 8));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(recs), n * S / 8);
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
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t gb = std::min<uint32_t>(maps * nbk, ncu * 4);
  unsigned long long* st;
  CK(hipMalloc(&st, gb * 8 * 8));
  CK(hipMemset(st, 0, gb * 8 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_msd_stamps), &st, sizeof st));
  constexpr size_t lda = M16a<8, 10>::lds_bytes(), ldb = M16b<4, 8>::lds_bytes();
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_msd16a<2, 8, 10, kM16Lo>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lda));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_msd16b<2, 4, 8, kM16Lo, kM16MaxChunks>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldb));
  hipEvent_t e0, e1, e2, e3;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  CK(hipEventCreate(&e3));
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((k_msd16a<2, 8, 10, kM16Lo>), dim3(std::min<uint32_t>(maps * cpm, ncu * 2)), dim3(512), lda, 0, pd, g, cpm, nbk, offs, (uint16_t*)nullptr, tmp);
    CK(hipEventRecord(e1, 0));
    hipLaunchKernelGGL(k_msd16_scan, dim3(maps), dim3(kScanThreads), 0, 0, g, cpm, nbk, offs, segbase, idx, ibe, (uint64_t*)nullptr, (int)R);
    CK(hipEventRecord(e2, 0));
    hipLaunchKernelGGL((k_msd16b<2, 4, 8, kM16Lo, kM16MaxChunks>), dim3(gb), dim3(256), ldb, 0, pd, g, cpm, nbk, offs, segbase, tmp, out, idx, ibe);
    CK(hipEventRecord(e3, 0));
    CK(hipDeviceSynchronize());
  }
  float ta, ts, tb;
  CK(hipEventElapsedTime(&ta, e0, e1));
  CK(hipEventElapsedTime(&ts, e1, e2));
  CK(hipEventElapsedTime(&tb, e2, e3));
  std::vector<unsigned long long> h(gb * 8);
  CK(hipMemcpy(h.data(), st, gb * 64, hipMemcpyDeviceToHost));
  const double segs = (double)maps * nbk / gb;
  printf("maps %llu R %u: pass A %.3f ms (%.2f TB/s), scan %.3f ms, pass B %.3f ms (%.2f TB/s), %u workgroups, %.1f segments each\n",
         (unsigned long long)maps, R, ta, 2.0 * n * S / ta / 1e9, ts, tb, 2.0 * n * S / tb / 1e9, gb, segs);
  const char* names[5] = {"load issue", "rank+stage (load wait)", "cursors+index", "place", "next run table"};
  double tot = 0;
  for (int k = 0; k < 5; ++k) {
    double s = 0;
    for (uint32_t b = 0; b < gb; ++b) s += (double)h[b * 8 + k];
    tot += s;
  }
  for (int k = 0; k < 5; ++k) {
    double s = 0;
    for (uint32_t b = 0; b < gb; ++b) s += (double)h[b * 8 + k];
    printf("  %-24s %9.0f s_memtime ticks per segment (%4.1f %%)\n", names[k], s / gb / segs, 100.0 * s / tot);
  }
  return 0;
}
