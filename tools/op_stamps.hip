// op_stamps.hip — per-phase cycle timeline of the one-pass map side (diagnostic build, gfx950).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I sparkucx_amd/csrc \
//          -o tools/op_stamps tools/op_stamps.hip
// Runs k_onepass on 64 maps x 131072 x 100-B random records (Spark SQL murmur3 of the int64
// key, R=200), then prints, over workgroups 0..63 and maps 4..59, the mean s_memtime cycles of
// each phase of the map loop:
//   0-1 poll (wait for map m's counts)   1-2 offsets (sc1 loads + scan)   2-3 image build
//   3-4 count map m+2 + publish/arrive   4-5 issue map m+3   5-6 write-out   6-0' loop
#define SUX_OP_STAMPS 1
#include "../sparkucx_amd/csrc/sux_onepass.hip"

#include <cstdio>
#include <vector>

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
  const uint32_t R = 200, S = 100;
  const uint64_t rpm = 131072, maps = argc > 1 ? atoi(argv[1]) : 64, n = rpm * maps;
  uint8_t *recs, *out, *ws, *ibe;
  int64_t* idx;
  CK(hipMalloc(&recs, n * S));
  CK(hipMalloc(&out, n * S));
  CK(hipMalloc(&idx, maps * (R + 1) * 8));
  CK(hipMalloc(&ibe, maps * (R + 1) * 8));
  const uint64_t wsb = onepass_sync_bytes(R);
  CK(hipMalloc(&ws, wsb));
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
  uint32_t grid = 0, cs = 0;
  if (!onepass_eligible(pd, g, 1, out, nullptr, 0, &grid, &cs)) {
    fprintf(stderr, "not eligible\n");
    return 1;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0, 0));
    CK(launch_onepass(pd, g, out, idx, ibe, nullptr, ws, grid, cs, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("launch %d: %.3f ms for %llu maps (%.2f us/map, %.0f GB/s of 2*N*S)\n", rep, ms,
           (unsigned long long)maps, ms * 1e3 / maps, 2.0 * n * S / (ms * 1e-3) / 1e9);
  }
  std::vector<uint64_t> st(64 * 64 * 16);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(onepass::g_op_stamps), st.size() * 8));
  const int m0 = 4, m1 = (int)std::min<uint64_t>(60, maps - 3);
  // timeline order of the stamps inside one map, with the next map's 0 as the end
  const int order[] = {0, 1, 2, 3, 4, 5, 6, 7, 8};
  const char* names[] = {"S1 unit scan", "S2 recoff", "S3 image", "S4 poll+loads", "S5 count+2",
                         "S6 offsets", "S7 write-out", "S8 issue", "loop"};
  const int np = 9;
  double ph[16] = {0};
  int cnt = 0;
  for (int w = 0; w < (int)std::min<uint32_t>(64, grid); ++w)
    for (int m = m0; m < m1; ++m) {
      const uint64_t* t = &st[(w * 64 + m) * 16];
      for (int p = 0; p + 1 < np; ++p) ph[p] += (double)(t[order[p + 1]] - t[order[p]]);
      ph[np - 1] += (double)(st[(w * 64 + m + 1) * 16] - t[8]);
      ++cnt;
    }
  double tot = 0;
  for (int p = 0; p < np; ++p) tot += ph[p] / cnt;
  printf("mean cycles per map (WG 0..63, maps %d..%d): total %.0f\n", m0, m1 - 1, tot);
  for (int p = 0; p < np; ++p) printf("  %-14s %8.0f  (%4.1f%%)\n", names[p], ph[p] / cnt, 100 * ph[p] / cnt / tot);
  return 0;
}
