// sux_copy.hip — batched device gather copy for sux_fetch_blocks: the phase-2 GETs of
// OnOffsetsFetchCallback.java:80-87 (block i -> contiguous destination at a running offset)
// as one launch.  Blocks are cut into fixed chunks, one workgroup per chunk, so skewed block
// sizes (Zipf) still spread over the whole chip.
#include <hip/hip_runtime.h>

#include "sux_internal.h"

namespace sux {

constexpr uint32_t kCopyChunk = 64 * 1024;
constexpr int kCopyThreads = 256;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kCopyThreads) void k_gather_copy(const CopyDesc* __restrict__ desc,
                                                              uint32_t n,
                                                              const uint32_t* __restrict__ first) {
  // descriptor owning this chunk: largest d with first[d] <= blockIdx.x
  uint32_t lo = 0, hi = n - 1, c = blockIdx.x;
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if (first[mid] <= c) lo = mid; else hi = mid - 1;
  }
  const CopyDesc d = desc[lo];
  const uint64_t beg = (uint64_t)(c - first[lo]) * kCopyChunk;
  if (beg >= d.bytes) return;
  uint64_t len = d.bytes - beg;
  if (len > kCopyChunk) len = kCopyChunk;
  const uint8_t* src = d.src + beg;
  uint8_t* dst = d.dst + beg;
  const uintptr_t mis = ((uintptr_t)src | (uintptr_t)dst | (uintptr_t)len);
  if ((mis & 15) == 0) {
    const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
    u32x4* d4 = reinterpret_cast<u32x4*>(dst);
    for (uint64_t k = threadIdx.x; k < len / 16; k += kCopyThreads) d4[k] = s4[k];
  } else if ((mis & 3) == 0) {
    const uint32_t* s1 = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d1 = reinterpret_cast<uint32_t*>(dst);
    for (uint64_t k = threadIdx.x; k < len / 4; k += kCopyThreads) d1[k] = s1[k];
  } else {
    for (uint64_t k = threadIdx.x; k < len; k += kCopyThreads) dst[k] = src[k];
  }
}

hipError_t launch_gather_copy(const CopyDesc* d_desc, uint32_t n, uint32_t chunks_total,
                              const uint32_t* d_chunk_first, Timer* timer, hipStream_t s) {
  if (n == 0 || chunks_total == 0) return hipSuccess;
  timer_begin(timer, kCopy, s);
  hipLaunchKernelGGL(k_gather_copy, dim3(chunks_total), dim3(kCopyThreads), 0, s, d_desc, n,
                     d_chunk_first);
  timer_end(timer, kCopy, s);
  return hipGetLastError();
}

}  // namespace sux
