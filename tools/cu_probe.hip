// cu_probe.hip — where do the workgroups of a CU-masked stream land?  (MI355X, gfx950)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/cu_probe tools/cu_probe.hip
// For each mask (none; sux_stream_create's "reserve C" set and its complement) it launches 8192
// short workgroups and records HW_REG_XCC_ID and HW_REG_HW_ID of each; prints, per XCD, the
// number of distinct CUs that ran work, and for the reserve sets the mask bit -> (XCD, SE, CU).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void k_where(uint32_t* out, int spin) {
  if (threadIdx.x == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < spin) __builtin_amdgcn_s_sleep(1);
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
}

static uint32_t reserved_cu(uint32_t k) { return k; }  // same pick as sux_api.cpp

int main() {
  const int NB = 8192;
  uint32_t* d;
  CK(hipMalloc(&d, NB * 8));
  std::vector<uint32_t> h(NB * 2);
  struct Mode {
    const char* name;
    int C;
    bool comp;
  } modes[] = {{"none", 0, false}, {"res32", 32, false}, {"comp32", 32, true},
               {"res64", 64, false}, {"comp64", 64, true}};
  for (const Mode& m : modes) {
    hipStream_t st;
    if (m.C == 0) {
      CK(hipStreamCreate(&st));
    } else {
      std::vector<uint32_t> mask(8, 0);
      std::vector<int> pick(256, 0);
      for (int k = 0; k < m.C; ++k) pick[reserved_cu(k)] = 1;
      for (int i = 0; i < 256; ++i)
        if (pick[i] != (m.comp ? 1 : 0)) mask[i / 32] |= 1u << (i % 32);
      CK(hipExtStreamCreateWithCUMask(&st, 8, mask.data()));
    }
    CK(hipMemset(d, 0xFF, NB * 8));
    hipLaunchKernelGGL(k_where, dim3(NB), dim3(64), 0, st, d, 2000);  // 20 us per block
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(h.data(), d, NB * 8, hipMemcpyDeviceToHost));
    std::map<uint32_t, std::set<uint32_t>> cus;  // xcc -> (se, sh, cu)
    std::map<uint32_t, int> blocks;
    for (int b = 0; b < NB; ++b) {
      const uint32_t xcc = h[2 * b] & 0xF, hw = h[2 * b + 1];
      const uint32_t cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      cus[xcc].insert(se << 8 | sh << 4 | cu);
      blocks[xcc]++;
    }
    printf("%-7s", m.name);
    for (auto& kv : cus) printf(" xcc%u:%zu cus/%d blk", kv.first, kv.second.size(), blocks[kv.first]);
    printf("\n");
    if (m.name[0] == 'n') {
      // the unmasked (se, sh, cu) universe of each XCD
      for (auto& kv : cus) {
        printf("  xcc%u ids:", kv.first);
        for (uint32_t v : kv.second) printf(" %x", v);
        printf("\n");
      }
    }
    if (m.C && !m.comp) {
      for (auto& kv : cus) {
        printf("  xcc%u ids:", kv.first);
        for (uint32_t v : kv.second) printf(" %x", v);
        printf("\n");
      }
    }
    CK(hipStreamDestroy(st));
  }
  return 0;
}
