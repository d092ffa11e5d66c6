// vstamps.hip — per-phase cycle timeline of the variable-length line-image scatter (k_vscatter3;
// diagnostic build, gfx950).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I sparkucx_amd/csrc \
//          -o tools/vstamps tools/vstamps.hip
// Runs the variable-length map side (hist + scans + scatter) on 32 maps x 1 Mi rows of
// 20 + 8k bytes (k in [0, 12], the bench's varlen leg) with the Spark SQL murmur3 long
// partitioner (R = 200), then prints, for the first 64 scatter workgroups and their chunks
// 1..14, the mean s_memtime cycles of each phase of the chunk loop:
//   0-1 offsets + fit   1-2 byte ranks   2-3 regions   3-4 carries in + row offsets + unit tags
//   4-5 window fill + next loads   5-6 write-out   6-7 carries out + seams   7-0' loop back
#define SUX_STAMPS 1
#include "../sparkucx_amd/csrc/sux_varlen.hip"

#include <cstdio>
#include <vector>

namespace sux {
struct Timer {};
void timer_begin(Timer*, int, hipStream_t) {}
void timer_end(Timer*, int, hipStream_t) {}
void timer_note(Timer*, int, const char*) {}
int stream_cus(hipStream_t) { return 256; }

// map bases: base[m][p] = map m's first byte + the bytes of partitions < p (one thread per map)
__global__ void k_bases(const uint64_t* offs, const uint64_t* totals, uint64_t* base, uint32_t maps,
                        int R, uint64_t rpm) {
  const uint32_t m = blockIdx.x * 64 + threadIdx.x;
  if (m >= maps) return;
  uint64_t b = offs[m * rpm] - offs[0];
  for (int p = 0; p < R; ++p) {
    base[(uint64_t)m * R + p] = b;
    b += totals[(uint64_t)m * R + p];
  }
}
hipError_t launch_varlen_map_scan(const VarGroup& g, int R, const uint64_t* totals, uint64_t* base,
                                  int64_t*, uint8_t*, hipStream_t s) {
  hipLaunchKernelGGL(k_bases, dim3((g.num_maps + 63) / 64), dim3(64), 0, s, g.offs, totals, base,
                     g.num_maps, R, g.records_per_map);
  return hipGetLastError();
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

int main(int argc, char** argv) {
  using namespace sux;
  const int R = argc > 1 ? atoi(argv[1]) : 200;
  const int ver = argc > 2 ? atoi(argv[2]) : 3;
  const uint64_t rpm = 1u << 20, maps = 32, n = rpm * maps;
  std::vector<uint64_t> offs(n + 1);
  offs[0] = 0;
  uint64_t z = 88172645463325252ull;
  for (uint64_t i = 0; i < n; ++i) {
    z ^= z << 13;
    z ^= z >> 7;
    z ^= z << 17;
    offs[i + 1] = offs[i] + 4 + 8 * (2 + z % 13);
  }
  const uint64_t tot = offs[n];
  uint8_t *data, *out, *ws, *ibe;
  uint64_t* d_offs;
  int64_t* idx;
  CK(hipMalloc(&data, tot + 64));
  CK(hipMalloc(&out, tot + 64));
  CK(hipMalloc(&d_offs, (n + 1) * 8));
  CK(hipMalloc(&idx, maps * (R + 1) * 8));
  CK(hipMalloc(&ibe, maps * (R + 1) * 8));
  CK(hipMemcpy(d_offs, offs.data(), (n + 1) * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(data), tot / 8);
  PartDev pd{};
  pd.kind = 2;
  pd.R = R;
  pd.key_offset = 12;
  pd.key_len = 8;
  pd.seed = 42;
  pd.ascending = 1;
  pd.rmagic = part_magic(pd.R);
  Tuning tn{};
  tn.varlen_kernel = ver;
  VarGroup g{};
  g.data = data;
  g.offs = d_offs;
  g.records_per_map = rpm;
  g.num_records = n;
  g.num_maps = maps;
  g.tile_recs = choose_varlen_tile(R, n, tn);
  g.tiles_per_map = (uint32_t)((rpm + g.tile_recs - 1) / g.tile_recs);
  VarWorkspace w = varlen_workspace_layout(R, rpm, n, g.tile_recs);
  CK(hipMalloc(&ws, w.total));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipEventRecord(e0, 0));
    CK(launch_varlen_group(pd, g, out, idx, ibe, nullptr, nullptr, ws, w, tn, nullptr, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("v%d map side %.3f ms  (%.1f GB/s of row bytes)\n", ver, ms, tot / (ms * 1e-3) / 1e9);
  }
  if (ver != 3) return 0;
  std::vector<uint64_t> st(64 * 16 * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_vstamps), st.size() * 8));
  double acc[8] = {0};
  int cnt = 0;
  for (int b = 0; b < 64; ++b)
    for (int c = 1; c < 15; ++c) {
      const uint64_t* t = &st[(b * 16 + c) * 8];
      const uint64_t* tn2 = &st[(b * 16 + c + 1) * 8];
      if (!t[0] || !t[7] || !tn2[0]) continue;
      for (int k = 0; k < 7; ++k) acc[k] += (double)(t[k + 1] - t[k]);
      acc[7] += (double)(tn2[0] - t[7]);
      ++cnt;
    }
  const char* names[8] = {"offs+fit", "ranks", "regions", "tags+offs", "fill+issue",
                          "write-out", "carries", "loop"};
  double sum = 0;
  for (int k = 0; k < 8; ++k) sum += acc[k] / cnt;
  printf("chunks sampled: %d, mean cycles per chunk %.0f\n", cnt, sum);
  for (int k = 0; k < 8; ++k)
    printf("  %-11s %8.0f cycles  %5.1f %%\n", names[k], acc[k] / cnt, 100.0 * acc[k] / cnt / sum);
  return 0;
}
