// msd_whatif.hip — what do k_msd16a's LDS bank conflicts cost?  Times pass A of
// the two-level small-record path ALONE (no scan, no pass B: the what-if builds' output is not
// bucket-sorted, and pass B must never read it) on C5's shape: 200 maps x 2^20 16-byte random
// records, Spark SQL murmur3 of the int64 key, R = 10 000, 32-partition buckets (9-bit digit),
// two 512-thread workgroups per CU — the product launch.  Build (from the repo root), one binary
// per level:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I sparkucx_amd/csrc \
//         [-DSUX_MSD_WHATIF=1|2|3] -o tools/msd_whatif[1|2|3] tools/msd_whatif.hip
// Level 0 (no define): the product kernel; -DMSD_TOOL_ATOM (reported as level 64): the product's
// msd_direct bit-6 kernel (atomic ranking).  1: the stage store at the record's own conflict-free
// slot, no bucket-start read.  2: 1 + the wave ranking's counters at conflict-free digits (and,
// as compiled, three fewer match ballots per record).  3: 1 + digits unique in the wave (lane
// in the low 6 bits: counters <= 2-way conflicted) with all nine ballots.
// Prints one JSON line: pass A's mean ms over 5 launches after 2 warm-ups and its rate at the
// algorithmic 32 B per record.
#include "../sparkucx_amd/csrc/sux_small.hip"

#include <cstdio>

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

#ifndef SUX_MSD_WHATIF
#define SUX_MSD_WHATIF 0
#endif

int main() {
  using namespace sux;
  constexpr uint32_t R = 10000, S = 16, DB = 9, NWA = 8;
  const uint64_t rpm = 1 << 20, maps = 200, n = rpm * maps;
  const uint32_t cpm = (uint32_t)(rpm / kM16Chunk), nbk = (R + 31) / 32;
  static_assert(((R + 31) / 32) > 256 && ((R + 31) / 32) <= 512, "9-bit digit");
  uint8_t *recs, *tmp;
  uint16_t* offs;
  CK(hipMalloc(&recs, n * S));
  CK(hipMalloc(&tmp, n * S));
  CK(hipMalloc(&offs, maps * cpm * nbk * 2));  // [map][chunk][bucket], every item's nbk entries
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
#ifdef MSD_TOOL_ATOM  // the product's msd_direct bit 6 (atomic ranking), for comparison
  constexpr size_t lda = M16a<NWA, DB, 4>::lds_bytes();
  auto* kern = &k_msd16a<2, NWA, DB, kM16LoWide, false, true>;
  const int level = 64;
#elif defined(MSD_TOOL_TAG)  // msd_direct bit 7 (the 6-bit tag match)
  constexpr size_t lda = M16a<NWA, DB, 2, true>::lds_bytes();
  auto* kern = &k_msd16a<2, NWA, DB, kM16LoWide, false, false, true>;
  const int level = 128;
#else
  constexpr size_t lda = M16a<NWA, DB>::lds_bytes();
  auto* kern = &k_msd16a<2, NWA, DB, kM16LoWide, false>;
  const int level = SUX_MSD_WHATIF;
#endif
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lda));
  const dim3 ga(std::min<uint32_t>(maps * cpm, ncu * 2));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL(kern, ga, dim3(NWA * kWave), lda, 0, pd, g, cpm, nbk, offs,
                       (uint16_t*)nullptr, tmp);
  CK(hipDeviceSynchronize());
  constexpr int reps = 5;
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(kern, ga, dim3(NWA * kWave), lda, 0, pd, g, cpm, nbk, offs,
                       (uint16_t*)nullptr, tmp);
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  CK(hipGetLastError());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  printf("{\"what\": \"k_msd16a alone\", \"whatif\": %d, \"maps\": %llu, \"records\": %llu, "
         "\"R\": %u, \"workgroups\": %u, \"ms\": %.4f, \"TB/s_at_32B_per_record\": %.3f}\n",
         level, (unsigned long long)maps, (unsigned long long)n, R, ga.x, ms,
         32.0 * n / ms / 1e9);
  return 0;
}
