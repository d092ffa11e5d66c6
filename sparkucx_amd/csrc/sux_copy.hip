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
    // four 16-byte loads in flight per lane before their stores (one at a time leaves the copy
    // latency-bound: a load, a wait, a store, per 4 KiB of the chunk)
    const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
    u32x4* d4 = reinterpret_cast<u32x4*>(dst);
    const uint64_t n16 = len / 16;
    uint64_t k = threadIdx.x;
    for (; k + 3 * kCopyThreads < n16; k += 4 * kCopyThreads) {
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = s4[k + u * kCopyThreads];
#pragma unroll
      for (int u = 0; u < 4; ++u) d4[k + u * kCopyThreads] = v[u];
    }
    for (; k < n16; k += kCopyThreads) d4[k] = s4[k];
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

namespace sux {

// ---------------------------------------------------------------------------------------------
// One-sided pull of a peer-major launch group (sux_pull_group).  Workgroup b serves source
// g = b / per_src and strides over that source's range.  Every workgroup first derives, from the
// all-gathered index tables, where this rank's share sits in g's send buffer and where it goes
// in the receive buffer (the arithmetic of sux_plan_group, done on the device).
// ---------------------------------------------------------------------------------------------
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ int32_t owner_lo_d(int32_t h, int32_t R, int32_t W,
                                              const int32_t* own) {
  return own ? own[h] : (int32_t)(((int64_t)h * R) / W);
}

__global__ __launch_bounds__(256) void k_pull(int32_t W, int32_t me, const uint64_t* __restrict__ srcs,
                                              const int64_t* __restrict__ gi, int32_t M, int32_t R,
                                              uint8_t* __restrict__ recv, uint64_t cap,
                                              uint64_t* recv_bytes, uint32_t per_src,
                                              const int32_t* __restrict__ own) {
  __shared__ uint64_t red[3][256];
  const int32_t g = blockIdx.x / per_src;
  const uint32_t slot = blockIdx.x - g * per_src;
  const int64_t stride = (int64_t)R + 1;
  const int32_t lo = owner_lo_d(me, R, W, own), hi = owner_lo_d(me + 1, R, W, own);
  // per thread partial sums: [0] offset of my share in g's buffer, [1] its size,
  // [2] bytes from sources before g (my receive offset), [3] everything (total received)
  uint64_t a = 0, b = 0, c = 0, tot = 0;
  for (int32_t t = threadIdx.x; t < W * M; t += 256) {
    const int32_t gg = t / M, m = t - gg * M;
    const int64_t* ix = gi + ((int64_t)gg * M + m) * stride;
    const uint64_t mine = (uint64_t)(ix[hi] - ix[lo]);
    tot += mine;
    if (gg < g) c += mine;
    if (gg == g) {
      b += mine;
      a += (uint64_t)(ix[lo] - ix[0]);  // shares of peers < me in g's peer-major buffer
    }
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  red[2][threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
      for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + s];
    __syncthreads();
  }
  const uint64_t src_off = red[0][0], size = red[1][0], dst_off = red[2][0];
  __syncthreads();
  red[0][threadIdx.x] = tot;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[0][threadIdx.x] += red[0][threadIdx.x + s];
    __syncthreads();
  }
  const uint64_t total = red[0][0];
  if (blockIdx.x == 0 && threadIdx.x == 0 && recv_bytes) *recv_bytes = total > cap ? ~0ull : total;
  if (total > cap) return;
  // g's buffer is [peer h][map m][partitions of h]: my share starts after every peer h < me,
  // i.e. at sum_m sum_{h<me} (ix[hi_h] - ix[lo_h]) = sum_m (ix[lo_me] - ix[0]), and holds my
  // ranges of maps 0..M-1 in order — exactly the [source][map][partition] receive layout.
  const uint8_t* src = reinterpret_cast<const uint8_t*>(srcs[g]) + src_off;
  uint8_t* dst = recv + dst_off;
  // 16-byte pieces when both sides are 4-byte aligned, then whole dwords, then single bytes:
  // never a byte past `size` (compressed map outputs are byte-granular)
  const bool al4 = (((uintptr_t)src | (uintptr_t)dst) & 3) == 0;
  const uint64_t n16 = al4 ? size / 16 : 0, n4 = al4 ? size / 4 : 0;
  const uint64_t t0 = (uint64_t)slot * 256 + threadIdx.x, step = (uint64_t)per_src * 256;
  uint64_t i = t0;
  for (; i + 3 * step < n16; i += 4 * step) {  // four loads in flight per lane (xGMI latency)
    u32x4a4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const u32x4a4*>(src + 16 * (i + u * step));
#pragma unroll
    for (int u = 0; u < 4; ++u) *reinterpret_cast<u32x4a4*>(dst + 16 * (i + u * step)) = v[u];
  }
  for (; i < n16; i += step)
    *reinterpret_cast<u32x4a4*>(dst + 16 * i) = *reinterpret_cast<const u32x4a4*>(src + 16 * i);
  for (uint64_t i = n16 * 4 + t0; i < n4; i += step)
    *reinterpret_cast<uint32_t*>(dst + 4 * i) = *reinterpret_cast<const uint32_t*>(src + 4 * i);
  for (uint64_t i = n4 * 4 + t0; i < size; i += step) dst[i] = src[i];
}

// out[i] = *ptrs[i]: the index entries a batch of block resolves needs from device-resident index
// tables (adopted map outputs), 16 bytes per block each way instead of every table.
__global__ __launch_bounds__(256) void k_gather_i64(const int64_t* const* __restrict__ ptrs,
                                                    uint32_t n, int64_t* __restrict__ out) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) out[i] = *ptrs[i];
}

hipError_t launch_gather_i64(const int64_t* const* d_ptrs, uint32_t n, int64_t* d_out,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t g = (n + 255) / 256;
  hipLaunchKernelGGL(k_gather_i64, dim3(g < 2048 ? g : 2048), dim3(256), 0, s, d_ptrs, n, d_out);
  return hipGetLastError();
}

// Zero-copy resolve of world-1 local blocks on the device (sux_resolve_blocks): block i =
// {map, start, end, 0} -> addrs[i] = data base of the map + index[start], sizes[i] = index[end] -
// index[start], from the per-map table {index table, data base} (index = nullptr: the map is not
// resolvable here).  A malformed id or such a map gets sizes[i] = -1 and is resolved again on the
// host, which raises the reference's error for it.
__global__ __launch_bounds__(256) void k_resolve_blocks(const int4* __restrict__ blocks, uint32_t n,
                                                        const ResolveMap* __restrict__ maps,
                                                        int32_t num_maps, int32_t R,
                                                        uint64_t* __restrict__ addrs,
                                                        int64_t* __restrict__ sizes) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int4 b = blocks[i];
    uint64_t a = 0;
    int64_t sz = -1;
    if (b.x >= 0 && b.x < num_maps && b.y >= 0 && b.z > b.y && b.z <= R) {
      const ResolveMap mp = maps[b.x];
      if (mp.index) {
        const int64_t lo = mp.index[b.y], hi = mp.index[b.z];
        a = mp.base + (uint64_t)lo;
        sz = hi - lo;
      }
    }
    addrs[i] = a;
    sizes[i] = sz;
  }
}

hipError_t launch_resolve_blocks(const void* d_blocks, uint32_t n, const ResolveMap* d_maps,
                                 int32_t num_maps, int32_t R, uint64_t* d_addrs, int64_t* d_sizes,
                                 hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t g = (n + 255) / 256;
  hipLaunchKernelGGL(k_resolve_blocks, dim3(g < 4096 ? g : 4096), dim3(256), 0, s,
                     static_cast<const int4*>(d_blocks), n, d_maps, num_maps, R, d_addrs, d_sizes);
  return hipGetLastError();
}

hipError_t launch_pull(int32_t W, int32_t me, const uint64_t* srcs, const int64_t* gi, int32_t M,
                       int32_t R, uint8_t* recv, uint64_t cap, uint64_t* recv_bytes,
                       hipStream_t s, const int32_t* own) {
  const uint32_t per_src = 1024 / (uint32_t)(W > 0 ? W : 1) + 1;
  hipLaunchKernelGGL(k_pull, dim3(per_src * W), dim3(256), 0, s, W, me, srcs, gi, M, R, recv, cap,
                     recv_bytes, per_src, own);
  return hipGetLastError();
}

}  // namespace sux
