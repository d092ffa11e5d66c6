// stamps.hip — per-phase cycle timeline of the default scatter (v8 since round 2; diagnostic
// build, gfx950).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I sparkucx_amd/csrc \
//          -o tools/stamps tools/stamps.hip
// Runs the map side (hist + scans + scatter) on 32 maps x 1 Mi x 100-B random records with the
// Spark SQL murmur3 partitioner (R=200), then prints, for the first 64 scatter workgroups and
// their chunks 1..15, the mean s_memtime cycles of each phase of the chunk loop:
//   v8: 0-1 rank   1-2 prefix+region scan   2-3 region table   3-4 carries in + offsets + unit
//   tags   4-5 image fill+issue   5-6 write-out (whole lines)   6-7 carries out   7-0' loop back
#define SUX_STAMPS 1
#include "../sparkucx_amd/csrc/sux_partition.hip"

#include <cstdio>
#include <vector>

namespace sux {
struct Timer {};
void timer_begin(Timer*, int, hipStream_t) {}
void timer_end(Timer*, int, hipStream_t) {}
void timer_note(Timer*, int, const char*) {}
int stream_cus(hipStream_t) { return 256; }
uint64_t onepass_sync_bytes(uint32_t) { return 0; }  // the one-pass path is not built here
bool onepass_eligible(const PartDev&, const MapGroup&, int, const void*, const uint64_t*,
                      hipStream_t, uint32_t*, uint32_t*) { return false; }
hipError_t launch_onepass(const PartDev&, const MapGroup&, uint8_t*, int64_t*, uint8_t*,
                          uint16_t*, uint8_t*, uint32_t, uint32_t, hipStream_t) {
  return hipSuccess;
}
// the small-record path (sux_small.hip) is not built here
bool msd16_eligible(const PartDev&, const MapGroup&, const LayoutDesc&, const uint8_t*,
                    const Workspace&, const Tuning&) { return false; }
hipError_t launch_msd16(const PartDev&, const MapGroup&, uint8_t*, int64_t*, uint8_t*, uint16_t*,
                        uint8_t*, const Workspace&, uint64_t*, const Tuning&, Timer*, hipStream_t) {
  return hipErrorInvalidValue;
}
hipError_t launch_hist16(const PartDev&, const MapGroup&, uint16_t*, uint32_t*, hipStream_t) {
  return hipErrorInvalidValue;
}
hipError_t launch_scatter16(const MapGroup&, int, int, const uint16_t*, const uint32_t*,
                            const uint64_t*, uint8_t*, const Tuning&, Timer*, hipStream_t) {
  return hipErrorInvalidValue;
}
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

int main() {
  using namespace sux;
  const uint32_t R = 200, S = 100;
  const uint64_t rpm = 1u << 20, maps = 32, n = rpm * maps;
  uint8_t *recs, *out, *ws, *ibe;
  int64_t* idx;
  CK(hipMalloc(&recs, n * S));
  CK(hipMalloc(&out, n * S));
  CK(hipMalloc(&idx, maps * (R + 1) * 8));
  CK(hipMalloc(&ibe, maps * (R + 1) * 8));
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
  g.num_maps = maps;
  g.rec_size = S;
  const Tuning tn{};
  g.tile_recs = choose_tile_recs(R, S, rpm, tn);
  g.tiles_per_map = (uint32_t)((rpm + g.tile_recs - 1) / g.tile_recs);
  Workspace w = workspace_layout(R, S, rpm, n, g.tile_recs, true);
  CK(hipMalloc(&ws, w.total));
  LayoutDesc lay{1, S};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipEventRecord(e0, 0));
    CK(launch_partition_group(pd, g, lay, out, idx, ibe, nullptr, ws, w, nullptr, tn, nullptr, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("map side %.3f ms  (%.1f GB/s of 2*N*S)\n", ms, 2.0 * n * S / (ms * 1e-3) / 1e9);
  }
  std::vector<uint64_t> st(64 * 16 * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8));
  double acc[8] = {0};
  int cnt = 0;
  for (int b = 0; b < 64; ++b)
    for (int c = 1; c < 15; ++c) {
      const uint64_t* t = &st[(b * 16 + c) * 8];
      const uint64_t* tn = &st[(b * 16 + c + 1) * 8];
      if (!t[0] || !t[7] || !tn[0]) continue;
      for (int k = 0; k < 7; ++k) acc[k] += (double)(t[k + 1] - t[k]);
      acc[7] += (double)(tn[0] - t[7]);
      ++cnt;
    }
  const char* names[8] = {"rank", "prefix+scan", "region tbl", "tags+offs", "fill+issue",
                          "write-out", "carries", "loop"};
  double tot = 0;
  for (int k = 0; k < 8; ++k) tot += acc[k] / cnt;
  printf("chunks sampled: %d, mean cycles per chunk %.0f\n", cnt, tot);
  for (int k = 0; k < 8; ++k)
    printf("  %-11s %8.0f cycles  %5.1f %%\n", names[k], acc[k] / cnt, 100.0 * acc[k] / cnt / tot);
  return 0;
}
