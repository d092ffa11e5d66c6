// sux_sort.hip — reduce-side consumer: a stable sort of fixed-size
// records by key, the step Spark's reader runs after the fetch when the dependency has a key
// ordering (ExternalSorter, compat/spark_3_0/UcxShuffleReader.scala:138-154; TeraSort's reducer).
//
// LSD radix sort over 16-byte (key, index) pairs, then one gather of the whole records:
//   k_sort_pairs    record i -> pair {key as big-endian bytes [0, 12), i as u32 LE at [12, 16)};
//                   signed keys get their sign bit flipped so unsigned order = signed order
//   digit passes    stable partitions of the pairs by a 12-bit digit of the big-endian 128-bit
//                   pair value (least significant key digit first) — the map-side kernels with
//                   the internal radix partitioner (kind 7, R = 4096: k_hist16 + k_scatter16)
//   k_gather_records out record j = in record pairs[j].index (coalesced dword writes)
// Equal keys keep their input order (every pass is stable and the index is never a digit).
// Segmented (sux_sort_segments): the record's segment id, big-endian, sits above the key bytes,
// so one sort orders every segment (a reducer's partitions) in place.
#include <hip/hip_runtime.h>

#include "sux_internal.h"

namespace sux {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_sort_pairs(const uint8_t* __restrict__ in, uint64_t n,
                                                    uint32_t rs, int kind, int key_offset,
                                                    int key_len, const int64_t* __restrict__ seg,
                                                    int nseg, int sbytes,
                                                    u32x4* __restrict__ pairs) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint8_t* r = in + i * rs + key_offset;
  uint8_t kb[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (kind == 1 && (key_offset & 3) == 0) {  // unsigned bytes, dword-aligned: dword loads
    const uint32_t* r4 = reinterpret_cast<const uint32_t*>(r);
    for (int q = 0; q < (key_len + 3) / 4; ++q) {
      const uint32_t w = r4[q];
      for (int k = 0; k < 4 && 4 * q + k < key_len; ++k) kb[4 * q + k] = (uint8_t)(w >> (8 * k));
    }
  } else if (kind == 1) {  // unsigned lexicographic bytes
    for (int k = 0; k < key_len; ++k) kb[k] = r[k];
  } else {          // signed little-endian int64 (2) / int32 (3): big-endian, sign bit flipped
    const int w = kind == 2 ? 8 : 4;
    for (int k = 0; k < w; ++k) kb[k] = r[w - 1 - k];
    kb[0] ^= 0x80u;
  }
  if (sbytes) {  // segmented: the segment id (big-endian) above the key
    int lo = 0, hi = nseg;  // last segment whose start is <= i
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if ((uint64_t)seg[mid] <= i) lo = mid; else hi = mid;
    }
    for (int k = 11; k >= sbytes; --k) kb[k] = kb[k - sbytes];
    for (int k = 0; k < sbytes; ++k) kb[k] = (uint8_t)((uint32_t)lo >> (8 * (sbytes - 1 - k)));
  }
  u32x4 p;
  p[0] = (uint32_t)kb[0] | ((uint32_t)kb[1] << 8) | ((uint32_t)kb[2] << 16) | ((uint32_t)kb[3] << 24);
  p[1] = (uint32_t)kb[4] | ((uint32_t)kb[5] << 8) | ((uint32_t)kb[6] << 16) | ((uint32_t)kb[7] << 24);
  p[2] = (uint32_t)kb[8] | ((uint32_t)kb[9] << 8) | ((uint32_t)kb[10] << 16) | ((uint32_t)kb[11] << 24);
  p[3] = (uint32_t)i;
  pairs[i] = p;
}

__global__ __launch_bounds__(256) void k_gather_records(const uint32_t* __restrict__ in,
                                                        const u32x4* __restrict__ pairs,
                                                        uint64_t n, uint32_t W,
                                                        uint32_t* __restrict__ out) {
  const uint64_t total = n * W;
  for (uint64_t d = (uint64_t)blockIdx.x * 256 + threadIdx.x; d < total;
       d += (uint64_t)gridDim.x * 256) {
    const uint64_t j = d / W, w = d - j * W;
    const uint32_t src = pairs[j][3];
    out[d] = in[(uint64_t)src * W + w];
  }
}

hipError_t launch_sort_pairs(const uint8_t* in, uint64_t n, uint32_t rs, int kind, int key_offset,
                             int key_len, const int64_t* seg, int nseg, int sbytes, void* pairs,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sort_pairs, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, in, n, rs,
                     kind, key_offset, key_len, seg, nseg, sbytes, static_cast<u32x4*>(pairs));
  return hipGetLastError();
}

hipError_t launch_gather_records(const void* in, const void* pairs, uint64_t n, uint32_t rs,
                                 void* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t total = n * (rs / 4);
  const uint64_t blocks = std::min<uint64_t>((total + 255) / 256, 256ull * 32);
  hipLaunchKernelGGL(k_gather_records, dim3((uint32_t)blocks), dim3(256), 0, s,
                     static_cast<const uint32_t*>(in), static_cast<const u32x4*>(pairs), n,
                     rs / 4, static_cast<uint32_t*>(out));
  return hipGetLastError();
}

}  // namespace sux
