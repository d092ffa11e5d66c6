// sux_sort.hip — reduce-side consumer: a stable sort of fixed-size
// records by key, the step Spark's reader runs after the fetch when the dependency has a key
// ordering (ExternalSorter, compat/spark_3_0/UcxShuffleReader.scala:138-154; TeraSort's reducer).
//
// Default path (planned on the device, no host wait, graph-capturable):
//   k_sort_pairs    record i -> 16-byte pair {order key big-endian in [0, 12), i as u32 LE at
//                   [12, 16)} (or, for records of <= 16 bytes with the segment id, the record
//                   itself re-laid so its key leads: inline mode); signed keys get their sign bit
//                   flipped so unsigned order = signed order; per-block AND / OR of the key words
//   k_span_reduce (+ make_sort_plan) the key span -> the top digit (the tb highest varying bits)
//                   and the 8-bit LDS digits below it that vary (SortPlanDev)
//   top pass        one stable partition of the pairs by the top digit (the map-side small-record
//                   kernels with the internal radix partitioner, digit shift read on the device)
//   k_sort_local    every bucket of <= 4096 pairs sorted inside LDS by the lower digits; in
//                   gather mode it then gathers the bucket's records straight into the output
//                   (k_sort_bucket_global sorts larger buckets through global memory,
//                   k_gather_rest gathers them); inline mode ends in k_unpair_records
// LSD path (sort_msd = 2, sort_all_passes, or more pairs than 2^14 LDS buckets hold): 12-bit
// digit passes with the constant ones skipped after a host read of the span, then the gather.
// Equal keys keep their input order (every pass is stable and the index is never a digit).
// Segmented (sux_sort_segments): the record's segment id, big-endian, sits above the key bytes,
// so one sort orders every segment (a reducer's partitions) in place.
#include "sux_part.h"

namespace sux {

// Pair bytes: [0, kbytes) the order key (segment id big-endian, then the key big-endian, sign
// flipped for signed kinds); then either the record index as u32 LE at [12, 16) (gather mode) or,
// when record_size + segment bytes <= 16 (inline mode), the record's other bytes in record order
// at [kbytes, kbytes + rs - key_len): the pair IS the record, and k_unpair_records rebuilds it in
// one streaming pass instead of the random-access gather.  Digits only ever cover the key bytes.
__device__ inline u32x4 make_pair(const uint8_t* __restrict__ in, uint64_t i, uint32_t rs, int kind,
                                  int key_offset, int key_len, const int64_t* __restrict__ seg,
                                  int nseg, int sbytes) {
  const uint8_t* r = in + i * rs + key_offset;
  uint8_t kb[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (kind == 1 && (key_offset & 3) == 0 && key_offset + 16 <= (int)rs) {
    // unsigned bytes, dword-aligned, 16 bytes inside the record: ONE 16-byte load per record
    // (a wave instruction brings 64 keys; three dword loads made three passes over the same
    // lines), streamed (the records are read again only by the final gather, long after)
    const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4a4*>(r));
#pragma unroll
    for (int k = 0; k < 12; ++k) kb[k] = k < key_len ? (uint8_t)(w[k / 4] >> (8 * (k % 4))) : 0u;
  } else if (kind == 1 && (key_offset & 3) == 0) {  // unsigned bytes, dword-aligned: dword loads
    // all three loads issued unconditionally (the key's last dword repeated when shorter), then
    // bytes picked with constant indices: a load per loop trip made every record wait for its
    // previous key dword
    const uint32_t* r4 = reinterpret_cast<const uint32_t*>(r);
    const int nd = (key_len + 3) / 4;
    uint32_t w[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) w[q] = r4[q < nd ? q : nd - 1];
#pragma unroll
    for (int k = 0; k < 12; ++k) kb[k] = k < key_len ? (uint8_t)(w[k / 4] >> (8 * (k % 4))) : 0u;
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
  p[3] = (uint32_t)i;
  p[0] = (uint32_t)kb[0] | ((uint32_t)kb[1] << 8) | ((uint32_t)kb[2] << 16) | ((uint32_t)kb[3] << 24);
  p[1] = (uint32_t)kb[4] | ((uint32_t)kb[5] << 8) | ((uint32_t)kb[6] << 16) | ((uint32_t)kb[7] << 24);
  p[2] = (uint32_t)kb[8] | ((uint32_t)kb[9] << 8) | ((uint32_t)kb[10] << 16) | ((uint32_t)kb[11] << 24);
  return p;
}

// Inline mode, at 128-bit word level (a byte loop with run-time indices costs ~3x the bandwidth
// time): rec = the record as a little-endian u128; the pair's memory bytes, also a LE u128, are
// seg (big-endian, sbytes) | order key (klen bytes) | the record's other bytes in record order.
typedef unsigned __int128 u128;
__device__ inline u128 shl(u128 x, int b) { return b >= 128 ? (u128)0 : x << b; }
__device__ inline u128 shr(u128 x, int b) { return b >= 128 ? (u128)0 : x >> b; }
__device__ inline u128 lowmask(int nbytes) { return nbytes >= 16 ? ~(u128)0 : shl(1, 8 * nbytes) - 1; }

__device__ inline u128 load_rec(const uint8_t* rec, uint32_t rs) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(rec);
  u128 v = w[0];
  if (rs > 4) v |= (u128)w[1] << 32;
  if (rs > 8) v |= (u128)w[2] << 64;
  if (rs > 12) v |= (u128)w[3] << 96;
  return v;
}

__device__ inline u128 inline_pair(u128 rec, int kind, int off, int klen, uint32_t seg_be,
                                   int sbytes, uint32_t rs) {
  u128 key = shr(rec, 8 * off) & lowmask(klen);
  if (kind == 2) key = (u128)(__builtin_bswap64((uint64_t)key) ^ 0x80ull);
  else if (kind == 3) key = (u128)(__builtin_bswap32((uint32_t)key) ^ 0x80u);
  const u128 rest = (rec & lowmask(off)) | shl(shr(rec, 8 * (off + klen)) & lowmask((int)rs - off - klen), 8 * off);
  return (u128)seg_be | shl(key, 8 * sbytes) | shl(rest, 8 * (sbytes + klen));
}

__device__ inline u128 inline_unpair(u128 pr, int kind, int off, int klen, int sbytes, uint32_t rs) {
  u128 key = shr(pr, 8 * sbytes) & lowmask(klen);
  if (kind == 2) key = (u128)__builtin_bswap64((uint64_t)key ^ 0x80ull);
  else if (kind == 3) key = (u128)__builtin_bswap32((uint32_t)key ^ 0x80u);
  const u128 rest = shr(pr, 8 * (sbytes + klen)) & lowmask((int)rs - klen);
  return (rest & lowmask(off)) | shl(key, 8 * off) | shl(shr(rest, 8 * off), 8 * (off + klen));
}

// Inline mode's final pass: sorted pair j -> output record j.  Streaming: 16 B read, rs B written.
// sel (device-planned sort): *sel != 0 takes the pairs from pairs_b.
__global__ __launch_bounds__(256) void k_unpair_records(const u32x4* __restrict__ pairs, uint64_t n,
                                                        uint32_t rs, int kind, int key_offset,
                                                        int key_len, int sbytes,
                                                        uint32_t* __restrict__ out,
                                                        const u32x4* __restrict__ pairs_b,
                                                        const uint32_t* __restrict__ sel) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  if (sel && *sel) pairs = pairs_b;
  const u32x4 p = pairs[j];
  const u128 pr = (u128)p[0] | ((u128)p[1] << 32) | ((u128)p[2] << 64) | ((u128)p[3] << 96);
  const u128 rec = inline_unpair(pr, kind, key_offset, key_len, sbytes, rs);
  uint32_t* dst = out + j * (rs / 4);
  if (rs == 16 && ((uintptr_t)out & 15) == 0) {
    u32x4 v;
    v[0] = (uint32_t)rec; v[1] = (uint32_t)(rec >> 32); v[2] = (uint32_t)(rec >> 64);
    v[3] = (uint32_t)(rec >> 96);
    *reinterpret_cast<u32x4*>(dst) = v;
    return;
  }
  dst[0] = (uint32_t)rec;
  if (rs > 4) dst[1] = (uint32_t)(rec >> 32);
  if (rs > 8) dst[2] = (uint32_t)(rec >> 64);
  if (rs > 12) dst[3] = (uint32_t)(rec >> 96);
}

// The pair as one big-endian 128-bit value (the order key in its top bits).
__device__ __forceinline__ u128 pair_be128(const u32x4& w) {
  return ((u128)__builtin_bswap32(w[0]) << 96) | ((u128)__builtin_bswap32(w[1]) << 64) |
         ((u128)__builtin_bswap32(w[2]) << 32) | (u128)__builtin_bswap32(w[3]);
}
__device__ __forceinline__ u128 shfl_xor128(u128 v, int m) {
  const unsigned long long lo = __shfl_xor((unsigned long long)(uint64_t)v, m);
  const unsigned long long hi = __shfl_xor((unsigned long long)(uint64_t)(v >> 64), m);
  return ((u128)hi << 64) | (u128)lo;
}
__device__ __forceinline__ void put128(uint32_t* d, u128 v) {
  for (int k = 0; k < 4; ++k) d[k] = (uint32_t)(v >> (96 - 32 * k));
}
__device__ __forceinline__ u128 get128(const uint32_t* d) {
  return ((u128)d[0] << 96) | ((u128)d[1] << 64) | ((u128)d[2] << 32) | (u128)d[3];
}

// Grid-stride pair build that also records which key bits vary: each workgroup writes the AND and
// the OR of its pairs' key words to part[block][0..5] and its smallest and largest pair to
// part[block][8..15]; k_span_reduce folds them.  A digit whose bits are equal in AND and OR is the
// same for every record, so its pass is the identity and the host skips it (Spark long / int keys
// of small magnitude leave the top digits constant); the key range places the top digit's
// buckets over [min, max] only (a reducer's keys are one range partition's: round 4's bit span
// left a third of the 4096 buckets of such a partition empty and the rest ~1.5x fuller).
__global__ __launch_bounds__(256) void k_sort_pairs(const uint8_t* __restrict__ in, uint64_t n,
                                                    uint32_t rs, int kind, int key_offset,
                                                    int key_len, const int64_t* __restrict__ seg,
                                                    int nseg, int sbytes,
                                                    u32x4* __restrict__ pairs,
                                                    uint32_t* __restrict__ part, int inline_rec) {
  uint32_t a0 = ~0u, a1 = ~0u, a2 = ~0u, o0 = 0, o1 = 0, o2 = 0;
  u128 mn = ~(u128)0, mx = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * 256) {
    u32x4 p;
    if (inline_rec) {
      uint32_t seg_be = 0;
      if (sbytes) {  // last segment whose start is <= i, big-endian in sbytes bytes
        int lo = 0, hi = nseg;
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if ((uint64_t)seg[mid] <= i) lo = mid; else hi = mid;
        }
        seg_be = __builtin_bswap32((uint32_t)lo) >> (8 * (4 - sbytes));
      }
      const u128 pr = inline_pair(load_rec(in + i * rs, rs), kind, key_offset, key_len, seg_be,
                                  sbytes, rs);
      p[0] = (uint32_t)pr; p[1] = (uint32_t)(pr >> 32); p[2] = (uint32_t)(pr >> 64);
      p[3] = (uint32_t)(pr >> 96);
    } else {
      p = make_pair(in, i, rs, kind, key_offset, key_len, seg, nseg, sbytes);
    }
    pairs[i] = p;
    a0 &= p[0]; a1 &= p[1]; a2 &= p[2];
    o0 |= p[0]; o1 |= p[1]; o2 |= p[2];
    const u128 v = pair_be128(p);
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
  for (int m = 32; m >= 1; m >>= 1) {
    a0 &= __shfl_xor(a0, m); a1 &= __shfl_xor(a1, m); a2 &= __shfl_xor(a2, m);
    o0 |= __shfl_xor(o0, m); o1 |= __shfl_xor(o1, m); o2 |= __shfl_xor(o2, m);
    const u128 vn = shfl_xor128(mn, m), vx = shfl_xor128(mx, m);
    mn = vn < mn ? vn : mn;
    mx = vx > mx ? vx : mx;
  }
  __shared__ uint32_t red[4][6];
  __shared__ u128 rmm[4][2];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[wv][0] = a0; red[wv][1] = a1; red[wv][2] = a2;
    red[wv][3] = o0; red[wv][4] = o1; red[wv][5] = o2;
    rmm[wv][0] = mn;
    rmm[wv][1] = mx;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    uint32_t v = red[0][threadIdx.x];
    for (int w = 1; w < 4; ++w)
      v = threadIdx.x < 3 ? (v & red[w][threadIdx.x]) : (v | red[w][threadIdx.x]);
    part[blockIdx.x * 16 + threadIdx.x] = v;
  } else if (threadIdx.x == 8) {
    u128 a = rmm[0][0], b = rmm[0][1];
    for (int w = 1; w < 4; ++w) {
      a = rmm[w][0] < a ? rmm[w][0] : a;
      b = rmm[w][1] > b ? rmm[w][1] : b;
    }
    put128(part + blockIdx.x * 16 + 8, a);
    put128(part + blockIdx.x * 16 + 12, b);
  }
}

__device__ void make_sort_plan(const uint32_t* span, int bits, int tb, SortPlanDev* plan,
                               const u128* range, bool rebase_ok);

// The key span; with `plan`, thread 0 then plans the sort from it (the device-planned MSD path:
// one launch fewer than a separate planning kernel); `ranged` plans the top digit over the key
// range [min, max] instead of the varying bits.
__global__ __launch_bounds__(1024) void k_span_reduce(const uint32_t* __restrict__ part,
                                                      uint32_t blocks, uint32_t* __restrict__ span,
                                                      int bits, int tb, SortPlanDev* __restrict__ plan,
                                                      int ranged) {
  // wave folds by shuffles, one barrier, then thread 0 folds the 16 waves' results and plans
  // (round 4's 256-thread LDS tree took 8 barriers: 14 us of the 0.6 ms sort)
  constexpr int NW = 1024 / kWave;
  __shared__ uint32_t red[NW][6];
  __shared__ u128 rmm[NW][2];
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  uint32_t v[6] = {~0u, ~0u, ~0u, 0, 0, 0};
  u128 mn = ~(u128)0, mx = 0;
  for (uint32_t b = tid; b < blocks; b += 1024) {
    for (int k = 0; k < 6; ++k)
      v[k] = k < 3 ? (v[k] & part[b * 16 + k]) : (v[k] | part[b * 16 + k]);
    const u128 a = get128(part + b * 16 + 8), c = get128(part + b * 16 + 12);
    mn = a < mn ? a : mn;
    mx = c > mx ? c : mx;
  }
  for (int m = kWave / 2; m >= 1; m >>= 1) {
    for (int k = 0; k < 6; ++k) {
      const uint32_t o = __shfl_xor(v[k], m, kWave);
      v[k] = k < 3 ? (v[k] & o) : (v[k] | o);
    }
    const u128 vn = shfl_xor128(mn, m), vx = shfl_xor128(mx, m);
    mn = vn < mn ? vn : mn;
    mx = vx > mx ? vx : mx;
  }
  if (lane == 0) {
    for (int k = 0; k < 6; ++k) red[wave][k] = v[k];
    rmm[wave][0] = mn;
    rmm[wave][1] = mx;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < NW; ++w) {
      for (int k = 0; k < 6; ++k)
        red[0][k] = k < 3 ? (red[0][k] & red[w][k]) : (red[0][k] | red[w][k]);
      if (rmm[w][0] < rmm[0][0]) rmm[0][0] = rmm[w][0];
      if (rmm[w][1] > rmm[0][1]) rmm[0][1] = rmm[w][1];
    }
    for (int k = 0; k < 6; ++k) span[k] = red[0][k];
    if (plan) make_sort_plan(&red[0][0], bits, tb, plan, ranged ? rmm[0] : nullptr, ranged == 2);
  }
}

// One output dword per thread and step: record j = d / W, dword w of it, read from the record
// the pair names.  When n * W < 2^32 the division is a 32-bit multiply-high by ceil(2^32 / W)
// plus one correction (the quotient is exact or one too big), not a 64-bit division; only the
// pair's index word is loaded.
__global__ __launch_bounds__(256) void k_gather_records(const uint32_t* __restrict__ in,
                                                        const u32x4* __restrict__ pairs,
                                                        uint64_t n, uint32_t W, uint32_t magic,
                                                        uint32_t* __restrict__ out,
                                                        const u32x4* __restrict__ pairs_b,
                                                        const uint32_t* __restrict__ sel) {
  if (sel && *sel) pairs = pairs_b;
  const uint64_t total = n * W;
  const uint32_t* idx = reinterpret_cast<const uint32_t*>(pairs) + 3;  // pairs[j][3]
  if (magic) {
    const uint32_t t32 = (uint32_t)total;
    for (uint32_t d = blockIdx.x * 256u + threadIdx.x; d < t32; d += gridDim.x * 256u) {
      uint32_t j = __umulhi(d, magic);
      if (j * W > d) --j;
      const uint32_t w = d - j * W;
      const uint32_t src = idx[4ull * j];
      out[d] = in[(uint64_t)src * W + w];
    }
    return;
  }
  for (uint64_t d = (uint64_t)blockIdx.x * 256 + threadIdx.x; d < total;
       d += (uint64_t)gridDim.x * 256) {
    const uint64_t j = d / W, w = d - j * W;
    const uint32_t src = idx[4 * j];
    out[d] = in[(uint64_t)src * W + w];
  }
}

// Record gather with whole 16-byte units: L lanes per record (L = the power of two covering its
// units, <= 64), 64 / L records per wave and step; lane l moves units l, l + L, ... of its record
// (a record starts at a 4-byte phase: dword-aligned 16-byte accesses; the last unit's tail as
// dwords).  One load instruction carries 64 x 16 B instead of k_gather_records' 64 x 4 B.
__global__ __launch_bounds__(256) void k_gather_records16(const uint8_t* __restrict__ in,
                                                          const u32x4* __restrict__ pairs,
                                                          uint64_t n, uint32_t rs, uint32_t L,
                                                          uint8_t* __restrict__ out,
                                                          const u32x4* __restrict__ pairs_b,
                                                          const uint32_t* __restrict__ sel) {
  if (sel && *sel) pairs = pairs_b;
  const uint32_t* idx = reinterpret_cast<const uint32_t*>(pairs) + 3;  // pairs[j][3]
  const uint32_t lane = threadIdx.x % kWave, l = lane % L, per_wave = kWave / L;
  const uint32_t full = rs / 16, tail = (rs % 16) / 4;  // whole units, dwords after them
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / kWave);
  const uint64_t w0 = (uint64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  for (uint64_t j = w0 * per_wave + lane / L; j < n; j += waves * per_wave) {
    const uint32_t src = idx[4 * j];
    const uint8_t* s = in + (uint64_t)src * rs;
    uint8_t* d = out + j * rs;
    for (uint32_t u = l; u < full; u += L)
      *reinterpret_cast<u32x4a4*>(d + 16 * u) = *reinterpret_cast<const u32x4a4*>(s + 16 * u);
    if (tail && l == full % L) {
      const uint32_t* s4 = reinterpret_cast<const uint32_t*>(s + 16 * full);
      uint32_t* d4 = reinterpret_cast<uint32_t*>(d + 16 * full);
      for (uint32_t t = 0; t < tail; ++t) d4[t] = s4[t];
    }
  }
}

hipError_t launch_sort_pairs(const uint8_t* in, uint64_t n, uint32_t rs, int kind, int key_offset,
                             int key_len, const int64_t* seg, int nseg, int sbytes, void* pairs,
                             void* span_ws, bool inline_rec, hipStream_t s, int bits, int tb,
                             SortPlanDev* plan, int ranged) {
  if (n == 0) return hipSuccess;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, kSortSpanBlocks);
  uint32_t* part = static_cast<uint32_t*>(span_ws) + 8;
  hipLaunchKernelGGL(k_sort_pairs, dim3(blocks), dim3(256), 0, s, in, n, rs, kind, key_offset,
                     key_len, seg, nseg, sbytes, static_cast<u32x4*>(pairs), part,
                     inline_rec ? 1 : 0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_span_reduce, dim3(1), dim3(1024), 0, s, part, blocks,
                     static_cast<uint32_t*>(span_ws), bits, tb, plan, ranged);
  return hipGetLastError();
}

hipError_t launch_unpair_records_sel(const void* pairs_a, const void* pairs_b, const uint32_t* sel,
                                     uint64_t n, uint32_t rs, int kind, int key_offset,
                                     int key_len, int sbytes, void* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpair_records, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                     static_cast<const u32x4*>(pairs_a), n, rs, kind, key_offset, key_len, sbytes,
                     static_cast<uint32_t*>(out), static_cast<const u32x4*>(pairs_b), sel);
  return hipGetLastError();
}

hipError_t launch_unpair_records(const void* pairs, uint64_t n, uint32_t rs, int kind,
                                 int key_offset, int key_len, int sbytes, void* out, hipStream_t s) {
  return launch_unpair_records_sel(pairs, nullptr, nullptr, n, rs, kind, key_offset, key_len,
                                   sbytes, out, s);
}

hipError_t launch_gather_records(const void* in, const void* pairs, uint64_t n, uint32_t rs,
                                 void* out, hipStream_t s) {
  return launch_gather_records_sel(in, pairs, nullptr, nullptr, n, rs, out, s, true);
}

hipError_t launch_gather_records_sel(const void* in, const void* pairs, const void* pairs_b,
                                     const uint32_t* sel, uint64_t n, uint32_t rs, void* out,
                                     hipStream_t s, bool gather16) {
  if (n == 0) return hipSuccess;
  if (rs >= 16 && rs % 4 == 0 && gather16) {
    uint32_t L = 1;
    while (L < 64 && 16 * L < rs) L <<= 1;
    const uint64_t blocks = std::min<uint64_t>((n * L + 255) / 256, 256ull * 16);
    hipLaunchKernelGGL(k_gather_records16, dim3((uint32_t)blocks), dim3(256), 0, s,
                       static_cast<const uint8_t*>(in), static_cast<const u32x4*>(pairs), n, rs, L,
                       static_cast<uint8_t*>(out), static_cast<const u32x4*>(pairs_b), sel);
    return hipGetLastError();
  }
  const uint64_t total = n * (rs / 4);
  const uint64_t blocks = std::min<uint64_t>((total + 255) / 256, 256ull * 32);
  const uint32_t W = rs / 4;
  // ceil(2^32 / W): the 32-bit quotient path when every output dword index fits 32 bits
  const uint32_t magic = total + W < (1ull << 32) && W > 1
                             ? (uint32_t)(((1ull << 32) + W - 1) / W) : 0u;
  hipLaunchKernelGGL(k_gather_records, dim3((uint32_t)blocks), dim3(256), 0, s,
                     static_cast<const uint32_t*>(in), static_cast<const u32x4*>(pairs), n, W,
                     magic, static_cast<uint32_t*>(out), static_cast<const u32x4*>(pairs_b), sel);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// MSD finish (sux_sort_records / sux_sort_segments): one stable digit pass
// over the top bits of the keys' varying range leaves R buckets of <= kSortLocalCap pairs
// (k_sort_local; larger ones k_sort_bucket_global); k_sort_local then sorts every bucket inside LDS by a stable LSD radix
// over the lower key digits that vary (8-bit digits: wave-ballot ranks + one block scan per
// digit; the pairs live in registers, one LDS buffer takes each digit's permutation) and writes
// it back.  Each pair crosses HBM twice
// after the top pass instead of twice per digit.  Stable: the top pass keeps input order inside
// a bucket and every LDS pass is stable.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pair_digit8(const u32x4& w, uint32_t sh) {
  const uint64_t hi = ((uint64_t)__builtin_bswap32(w[0]) << 32) | __builtin_bswap32(w[1]);
  const uint64_t lo = ((uint64_t)__builtin_bswap32(w[2]) << 32) | __builtin_bswap32(w[3]);
  const uint64_t v = sh >= 64 ? (hi >> (sh - 64)) : ((lo >> sh) | (sh ? (hi << (64 - sh)) : 0));
  return (uint32_t)v & 255u;
}

// key(a) > key(b): the top kbits bits of the big-endian 128-bit pairs (the order key; in
// inline mode the bits below are record payload, which must not order equal keys)
__device__ __forceinline__ bool key_greater(const u32x4& a, const u32x4& b, int kbits) {
  const uint64_t ah = ((uint64_t)__builtin_bswap32(a[0]) << 32) | __builtin_bswap32(a[1]);
  const uint64_t bh = ((uint64_t)__builtin_bswap32(b[0]) << 32) | __builtin_bswap32(b[1]);
  if (kbits <= 64) return (ah >> (64 - kbits)) > (bh >> (64 - kbits));
  if (ah != bh) return ah > bh;
  const uint64_t al = ((uint64_t)__builtin_bswap32(a[2]) << 32) | __builtin_bswap32(a[3]);
  const uint64_t bl = ((uint64_t)__builtin_bswap32(b[2]) << 32) | __builtin_bswap32(b[3]);
  return (al >> (128 - kbits)) > (bl >> (128 - kbits));
}
constexpr int kTopDigits = 2;          // LDS digit passes before the tie fix-up
constexpr uint32_t kMaxTieRun = 16;    // longer tie runs: every digit pass instead

// Bits [sh, sh + nb) of the big-endian 128-bit pair (nb <= 32).
__device__ __forceinline__ uint32_t pair_bits(const u32x4& w, uint32_t sh, uint32_t nb) {
  const uint64_t hi = ((uint64_t)__builtin_bswap32(w[0]) << 32) | __builtin_bswap32(w[1]);
  const uint64_t lo = ((uint64_t)__builtin_bswap32(w[2]) << 32) | __builtin_bswap32(w[3]);
  const uint64_t v = sh >= 64 ? (hi >> (sh - 64)) : ((lo >> sh) | (sh ? (hi << (64 - sh)) : 0));
  return (uint32_t)v & (uint32_t)((1ull << nb) - 1);
}

// The top digit of a pair: ((key >> sh) - base) & (2^nb - 1) — bits [sh, sh + nb) when base is
// 0; with a ranged plan (base = min >> sh) the bucket of the key's aligned 2^sh block counted from
// the smallest key's (the difference is exact in 64 bits: it is < 2^nb).
__device__ __forceinline__ uint32_t top_digit(const u32x4& w, uint32_t sh, uint64_t base,
                                              uint32_t nb) {
  const uint64_t hi = ((uint64_t)__builtin_bswap32(w[0]) << 32) | __builtin_bswap32(w[1]);
  const uint64_t lo = ((uint64_t)__builtin_bswap32(w[2]) << 32) | __builtin_bswap32(w[3]);
  const uint64_t v = sh >= 64 ? (hi >> (sh - 64)) : ((lo >> sh) | (sh ? (hi << (64 - sh)) : 0));
  return (uint32_t)(v - base) & (uint32_t)((1ull << nb) - 1);
}

// The key of a pair (its top kbits bits) as a right-aligned 128-bit value.
__device__ __forceinline__ u128 pair_key(const u32x4& w, int kbits) {
  return pair_be128(w) >> (128 - kbits);
}
// Rebased plan's top digit: the key's slice of [kmin, kmax] (monotone in the key, < 2^tb).
__device__ __forceinline__ uint32_t rebased_digit(const u32x4& w, const SortPlanDev* plan) {
  const u128 kmin = ((u128)plan->kmin_hi << 64) | plan->kmin_lo;
  const uint64_t v = (uint64_t)((pair_key(w, plan->kbits) - kmin) >> plan->rq);  // < 2^32
  return (uint32_t)((v * plan->rm) >> 32);
}

// ------------------------------------------------------------------------------------------
// Chunked top pass (round 4; the default when the top digit has <= 12 bits and the pairs fit
// kTopMaxChunks chunks).  The one-pass top-digit partition (k_hist16 + scans + k_scatter16s)
// puts ~1 pair per bucket per 4096-pair chunk: every pair leaves as a lone 16-byte store (2x
// write amplification, 131 us of the 0.64 ms sort).  Here every pass streams whole lines:
//   k_top_chunks   each 4096-pair chunk stable-sorted by the top digit in LDS and written back to
//                  ITS OWN place in the chunked copy, with the chunk's bucket starts (u16,
//                  offs[chunk][0..R], the last = the chunk's pairs);
//   k_top_colsum + k_top_scan   bucket sizes summed over the chunks -> the bucket index (bytes);
//   k_sort_local   gathers its bucket's run from every chunk (run table in LDS: the adjacent
//                  buckets a CU's neighbours sort read the same lines, so they come from L2);
//   k_top_materialize   only the buckets the LDS shapes do not take (above kSortLocalCap), or
//                  every bucket when no lower digit varies, are copied contiguously into b.
// Stable: chunks keep input order between them and the LDS passes keep it inside a chunk.
// ------------------------------------------------------------------------------------------
template <uint32_t NT, uint32_t DB>  // DB: bits per LSD pass (6: top digits of <= 12 bits)
__global__ __launch_bounds__(NT, 3 * NT / 256) void k_top_chunks(const u32x4* __restrict__ pairs,
                                                                uint64_t n, int tb,
                                                                const SortPlanDev* __restrict__ plan,
                                                                u32x4* __restrict__ outp,
                                                                uint16_t* __restrict__ offs,
                                                                uint32_t* __restrict__ tot) {
  if (!plan->msd_ok) return;  // every key equal: nothing reads the chunked copy
  if (blockIdx.x == 0)         // k_top_colsum's bucket totals (atomic adds), after this launch
    for (uint32_t b = threadIdx.x; b < (1u << tb); b += NT) tot[b] = 0;
  constexpr uint32_t NW = NT / kWave, PT = kTopChunk / NT, CH = kTopChunk, IDX = 12, ND = 1u << DB;
  constexpr uint32_t SE = ND * NW / NT;  // scan entries per thread
  static_assert(CH == 1u << IDX && SE >= 1 && ND * NW == SE * NT, "chunk index bits, scan shape");
  __shared__ uint32_t keys0[CH], keys1[CH];
  __shared__ uint32_t wc0[2 * NW * ND];  // [pass parity][wave][digit]
  __shared__ uint32_t wsum[NW];
  __shared__ uint16_t rs[1u << kTopMaxBits];  // bucket -> its first sorted position (~0: empty)
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const uint32_t R = 1u << tb, top_lo = (uint32_t)plan->top_lo;
  const uint64_t top_base = plan->top_base;
  const bool rebase = plan->rebase != 0;
  const int passes = tb <= (int)DB ? 1 : 2;
  const uint32_t D = passes == 1 ? (uint32_t)tb : (uint32_t)(tb + 1) / 2;  // <= DB bits a pass
  const uint32_t nch = (uint32_t)((n + CH - 1) / CH);
  for (uint32_t i = tid; i < 2 * NW * ND; i += NT) wc0[i] = 0;
  for (uint32_t i = tid; i < (1u << kTopMaxBits); i += NT) rs[i] = 0xFFFFu;
  // Two workgroups per CU within 64 VGPRs: the pairs are not held across the ranking — only
  // their keys (LDS); the sorted write reads each pair again, from the chunk just read (L2 /
  // Infinity Cache), in sorted order, and stores it coalesced
  for (uint32_t c = xcd_map(blockIdx.x, gridDim.x); c < nch; c += gridDim.x) {
    const uint64_t c0 = (uint64_t)c * CH;
    const uint32_t nc = (uint32_t)min<uint64_t>(CH, n - c0);
    uint32_t* kin = keys0;
    uint32_t* kout = keys1;
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {  // clamped, unconditional loads
      const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
      const u32x4 p = pairs[c0 + min(e, nc - 1)];
      if (e < nc)
        kin[e] = ((rebase ? rebased_digit(p, plan) : top_digit(p, top_lo, top_base, (uint32_t)tb))
                  << IDX) | e;
    }
    __syncthreads();
    // 1. LSD passes over (bucket << 12 | position), D bits each: wave-ballot ranks against the
    //    wave's own digit counters, one block scan over (digit, wave)
    for (int d = 0; d < passes; ++d) {
      uint32_t* wc = wc0 + (d & 1) * NW * ND;
      const uint32_t sh = IDX + d * D;
      uint32_t key[PT], dig[PT], rank[PT];
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
        const bool valid = e < nc;
        key[j] = valid ? kin[e] : 0u;
        dig[j] = valid ? (key[j] >> sh) & ((1u << D) - 1) : 0u;
        rank[j] = wave_rank<DB>(dig[j], valid, wc + wave * ND, lt_mask);
      }
      __syncthreads();
      {  // exclusive scan in (digit, wave) order: thread t owns entries [t SE, (t + 1) SE)
        uint32_t a[SE], sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < SE; ++k) {
          const uint32_t idx = (uint32_t)tid * SE + k;
          a[k] = wc[(idx % NW) * ND + idx / NW];
          sum += a[k];
        }
        const uint32_t incl = wave_incl_scan(sum, lane);
        if (lane == kWave - 1) wsum[wave] = incl;
        __syncthreads();
        uint32_t run = incl - sum;
#pragma unroll
        for (uint32_t q = 0; q < NW; ++q) run += q < (uint32_t)wave ? wsum[q] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < SE; ++k) {
          const uint32_t idx = (uint32_t)tid * SE + k;
          wc[(idx % NW) * ND + idx / NW] = run;
          run += a[k];
        }
      }
      __syncthreads();
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j)
        if (rank[j] != ~0u) kout[wc[wave * ND + dig[j]] + rank[j]] = key[j];
      __syncthreads();
      for (uint32_t i = tid; i < NW * ND; i += NT) wc[i] = 0;  // next used a barrier later
      uint32_t* t = kin;
      kin = kout;
      kout = t;
    }
    // 2. the chunk back to its own place in bucket order: sorted position s takes pair
    //    kin[s] & 4095, coalesced 16-byte stores; a bucket's first position (its bucket differs
    //    from the previous position's) is noted in rs
#pragma unroll
    for (uint32_t k = 0; k < PT; ++k) {
      const uint32_t s = tid + k * NT;
      if (s < nc) {
        const uint32_t ks = kin[s];
        outp[c0 + s] = pairs[c0 + (ks & (CH - 1))];
        if (s == 0 || (kin[s - 1] >> IDX) != (ks >> IDX)) rs[ks >> IDX] = (uint16_t)s;
      }
    }
    __syncthreads();
    // 3. the chunk's bucket starts, row[q] = the pairs of buckets below q = the first position of
    //    the first non-empty bucket >= q (nc past the last): a suffix minimum over rs.  Thread t
    //    owns buckets [t E, (t + 1) E); rs is reset behind the reads for the next chunk.  (Round 4
    //    ran a 13-step lower-bound search per bucket here: 117 dependent LDS reads per thread.)
    {
      constexpr uint32_t EQ = (1u << kTopMaxBits) / NT;
      const uint32_t E = (R + NT - 1) / NT;
      uint32_t m = 0xFFFFu;
#pragma unroll
      for (uint32_t k = 0; k < EQ; ++k) {
        const uint32_t q = (uint32_t)tid * E + k;
        if (k < E && q < R) m = min(m, (uint32_t)rs[q]);
      }
      uint32_t suf = m;  // min over this lane and the lanes above it
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t t = __shfl_down(suf, d, kWave);
        if (lane + d < kWave) suf = min(suf, t);
      }
      if (lane == 0) wsum[wave] = suf;
      __syncthreads();
      uint32_t run = nc;
#pragma unroll
      for (uint32_t q = 0; q < NW; ++q) run = q > (uint32_t)wave ? min(run, wsum[q]) : run;
      const uint32_t above = __shfl_down(suf, 1, kWave);
      if (lane + 1 < kWave) run = min(run, above);
      uint16_t* row = offs + (uint64_t)c * (R + 1);
#pragma unroll
      for (int k = (int)EQ - 1; k >= 0; --k) {
        const uint32_t q = (uint32_t)tid * E + (uint32_t)k;
        if ((uint32_t)k < E && q < R) {
          run = min(run, (uint32_t)rs[q]);
          row[q] = (uint16_t)run;
          rs[q] = 0xFFFFu;
        }
      }
      if (tid == 0) row[R] = (uint16_t)nc;
    }
    __syncthreads();  // kin / kout / wsum are rewritten by the next chunk
  }
}

// Bucket sizes: each workgroup sums one of kTopSegs chunk segments for 256 buckets and adds it
// to the bucket's total (32 atomic adds per bucket; tot zeroed by k_top_chunks).
__global__ __launch_bounds__(256) void k_top_colsum(const uint16_t* __restrict__ offs, uint32_t nch,
                                                    uint32_t R, const SortPlanDev* __restrict__ plan,
                                                    uint32_t* __restrict__ tot) {
  if (!plan->msd_ok) return;
  const uint32_t b = blockIdx.x * 256 + threadIdx.x, sg = blockIdx.y;
  if (b >= R) return;
  const uint32_t c0 = (uint32_t)((uint64_t)nch * sg / kTopSegs);
  const uint32_t c1 = (uint32_t)((uint64_t)nch * (sg + 1) / kTopSegs);
  uint32_t sum = 0, c = c0;
  for (; c + 8 <= c1; c += 8) {
    uint32_t v[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      const uint16_t* row = offs + (uint64_t)(c + k) * (R + 1) + b;
      v[k] = (uint32_t)row[1] - row[0];
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) sum += v[k];
  }
  for (; c < c1; ++c) {
    const uint16_t* row = offs + (uint64_t)c * (R + 1) + b;
    sum += (uint32_t)row[1] - row[0];
  }
  if (sum) atomicAdd(&tot[b], sum);
}

// The bucket index (bytes, R + 1 entries) from the bucket totals; every key equal: one bucket.
__global__ __launch_bounds__(1024) void k_top_scan(const uint32_t* __restrict__ tot, uint32_t R,
                                                   uint64_t n, SortPlanDev* __restrict__ plan,
                                                   int64_t* __restrict__ index) {
  __shared__ uint64_t sh[2 * kWave + 1];
  const uint32_t tid = threadIdx.x;
  if (!plan->msd_ok) {
    for (uint32_t b = tid; b <= R; b += 1024) index[b] = b == 0 ? 0 : (int64_t)(16 * n);
    return;
  }
  const uint32_t E = (R + 1023) / 1024;  // <= 8 (R <= 8192)
  uint32_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t v = 0;
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) {
    const uint32_t b = tid * E + k;
    t[k] = k < E && b < R ? tot[b] : 0u;
    v += t[k];
  }
  uint64_t all;
  uint64_t ex = block_excl_scan(v, sh, &all);
  bool big = false;
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) big = big || t[k] > kSortLocalCap;
  // k_gather_rest has work only for a bucket above the LDS shapes
  if (!__syncthreads_or(big) && tid == 0) plan->big = 0u;
  for (uint32_t k = 0; k < E; ++k) {
    const uint32_t b = tid * E + k;
    if (b >= R) break;
    index[b] = (int64_t)(16 * ex);
    ex += t[k];
  }
  if (tid == 0) index[R] = (int64_t)(16 * n);
}

// The buckets k_sort_local leaves (above kSortLocalCap; every bucket when no lower digit varies,
// whose final order is then this one) copied from their runs into b at their index range.
__global__ __launch_bounds__(256) void k_top_materialize(const u32x4* __restrict__ runs,
                                                         const uint16_t* __restrict__ offs,
                                                         uint32_t nch, uint32_t R,
                                                         const int64_t* __restrict__ index,
                                                         const SortPlanDev* __restrict__ plan,
                                                         u32x4* __restrict__ outb) {
  if (!plan->msd_ok) return;
  const bool all = plan->dg.n == 0;
  __shared__ uint32_t st[256], pre[256], wsum[4];
  const uint32_t tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  for (uint32_t b = blockIdx.x; b < R; b += gridDim.x) {
    const uint64_t s0 = (uint64_t)index[b] / 16, s1 = (uint64_t)index[b + 1] / 16;
    if (s1 == s0 || (!all && s1 - s0 <= kSortLocalCap)) continue;
    uint64_t done = 0;
    for (uint32_t t0 = 0; t0 < nch; t0 += 256) {
      const uint32_t c = t0 + tid;
      uint32_t len = 0, start = 0;
      if (c < nch) {
        const uint16_t* row = offs + (uint64_t)c * (R + 1);
        len = (uint32_t)row[b + 1] - row[b];
        start = c * kTopChunk + row[b];
      }
      const uint32_t incl = wave_incl_scan(len, (int)lane);
      if (lane == kWave - 1) wsum[wave] = incl;
      __syncthreads();
      uint32_t before = 0, total = 0;
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) {
        before += q < wave ? wsum[q] : 0u;
        total += wsum[q];
      }
      pre[tid] = before + incl - len;
      st[tid] = start;
      __syncthreads();
      const uint32_t m = min(256u, nch - t0);
      for (uint32_t e = tid; e < total; e += 256) {
        uint32_t lo = 0, hi = m;  // the last run starting at or before e
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (pre[mid] <= e) lo = mid; else hi = mid;
        }
        outb[s0 + done + e] = runs[st[lo] + (e - pre[lo])];
      }
      done += total;
      __syncthreads();
    }
  }
}

hipError_t launch_top_chunks(const void* pairs, uint64_t n, int tb, SortPlanDev* plan,
                             void* chunked, uint16_t* offs, uint32_t* tot, int64_t* index,
                             hipStream_t s) {
  const uint32_t ncu = (uint32_t)std::max(1, stream_cus(s));
  const uint32_t nch = (uint32_t)((n + kTopChunk - 1) / kTopChunk), R = 1u << tb;
  static_assert(kTopMaxBits <= 12, "two 6-bit LDS passes");
  hipLaunchKernelGGL((k_top_chunks<512, 6>), dim3(std::min(nch, 3 * ncu)), dim3(512), 0, s,
                     static_cast<const u32x4*>(pairs), n, tb, plan, static_cast<u32x4*>(chunked),
                     offs, tot);
  hipLaunchKernelGGL(k_top_colsum, dim3((R + 255) / 256, kTopSegs), dim3(256), 0, s, offs, nch, R,
                     plan, tot);
  hipLaunchKernelGGL(k_top_scan, dim3(1), dim3(1024), 0, s, tot, R, n, plan, index);
  return hipGetLastError();
}

// Gather of records [0, n) of one bucket (fused sort): output record e = input record sidx[e].
// L = 2^lsh lanes per record, each moving at most one 16-byte unit (lane l < rs / 16) or the
// record's tail dwords (lane rs / 16) — so rs <= 1024 (L <= 64); NT / L records per step, U steps'
// loads issued before their stores (clamped, unconditional: no per-load wait).  Records start at a
// 4-byte phase (dword-aligned 16-byte accesses).
#ifndef SUX_SORT_GATHER_U
#define SUX_SORT_GATHER_U 8  // records per lane group in flight in the fused sort's gather
#endif
#ifndef SUX_SORT_GATHER_NT
#define SUX_SORT_GATHER_NT 0
#endif
template <uint32_t NT, uint32_t U>
__device__ __forceinline__ void gather_run(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                           const uint32_t* sidx, uint32_t n, uint32_t rs,
                                           uint32_t lsh, uint32_t tid) {
  const uint32_t L = 1u << lsh, l = tid & (L - 1), G = NT >> lsh;
  const uint32_t full = rs / 16, tail = (rs % 16) / 4;
  const bool unit = l < full, tl = tail != 0 && l == full;
  if (!unit && !tl) return;
  for (uint32_t r0 = tid >> lsh; r0 < n; r0 += U * G) {
    u32x4 v[U];
#pragma unroll
    for (uint32_t k = 0; k < U; ++k) {
      const uint32_t e = min(r0 + k * G, n - 1);
      const uint8_t* s = in + (uint64_t)sidx[e] * rs + 16 * l;
      if (unit) {
#if SUX_SORT_GATHER_NT
        v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4a4*>(s));
#else
        v[k] = *reinterpret_cast<const u32x4a4*>(s);
#endif
      } else {
        const uint32_t* s4 = reinterpret_cast<const uint32_t*>(s);
        v[k][0] = s4[0];
        v[k][1] = tail > 1 ? s4[1] : 0u;
        v[k][2] = tail > 2 ? s4[2] : 0u;
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < U; ++k) {
      const uint32_t e = r0 + k * G;
      if (e >= n) break;
      uint8_t* d = out + (uint64_t)e * rs + 16 * l;
      if (unit) {
        *reinterpret_cast<u32x4a4*>(d) = v[k];
      } else {
        uint32_t* d4 = reinterpret_cast<uint32_t*>(d);
        d4[0] = v[k][0];
        if (tail > 1) d4[1] = v[k][1];
        if (tail > 2) d4[2] = v[k][2];
      }
    }
  }
}

// Where the fused sort gathers records (k_sort_local with GATHER): the input records, the output
// records, the record size and log2 of the lanes per record.
struct SortGather {
  const uint8_t* in;
  uint8_t* out;
  uint32_t rs, lsh;
};

template <uint32_t NW, uint32_t CAP>  // buf[CAP] u32x4 | wc[NW][256] u32 | wsum[NW]
struct SortLocal {
  static constexpr uint32_t NT = NW * kWave, PT = CAP / NT, NB = 256;
  static constexpr uint32_t lds_bytes() { return CAP * 16 + NW * NB * 4 + NW * 4; }
};

// <8 waves, 4096 pairs>: two workgroups per CU; <4 waves, 1024 pairs>: six per CU, for the
// ~600-pair buckets of a 5 M-record reduce partition.  A launch sorts the buckets of
// lo_cap < n <= CAP (one launch per size class) when the plan says the MSD path finishes the sort.
// GATHER (the fused sort, tuning gather_kernel 3): a sorted bucket is not written back as pairs —
// its record indices go to LDS and the workgroup gathers the bucket's records straight into the
// output (gather_run).  The random record reads of one workgroup then overlap the LDS digit
// passes of the others on the CU, and the pairs' last write + read (2 x 16 B per record) and the
// separate gather launch are gone.
template <uint32_t NW, uint32_t CAP, bool GATHER = false>
__global__ __launch_bounds__(NW * 64, NW == 8 ? 4 : CAP == 1024 ? 6 : 4) void k_sort_local(const u32x4* __restrict__ in,
                                                        u32x4* __restrict__ out,
                                                        const int64_t* __restrict__ index,
                                                        uint32_t R, uint32_t lo_cap,
                                                        const SortPlanDev* __restrict__ plan,
                                                        SortGather gth, SortRuns runs) {
  if (!plan->msd_ok || plan->dg.n == 0) return;  // the LSD fallback, or the top digit was all
  const SortDigits dg = plan->dg;
  const int kbits = plan->kbits;
  // the tie fix-up compares keys: a rebased bucket's keys are u, in the pair's top rbits bits
  const int tkbits = GATHER && plan->rebase ? plan->rbits : kbits;
  __shared__ uint32_t tie_redo;
  __shared__ u128 rmin[NW];
  if (threadIdx.x == 0) tie_redo = 0;
  using K = SortLocal<NW, CAP>;
  constexpr uint32_t NT = K::NT, PT = K::PT, NB = K::NB;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  u32x4* buf = reinterpret_cast<u32x4*>(lds8);
  uint32_t* wc = reinterpret_cast<uint32_t*>(buf + CAP);  // [NW][NB]
  uint32_t* wsum = wc + NW * NB;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
  __syncthreads();
  for (uint32_t b = xcd_map(blockIdx.x, gridDim.x); b < R; b += gridDim.x) {
    const uint64_t s0 = (uint64_t)index[b] / 16, s1 = (uint64_t)index[b + 1] / 16;
    const uint32_t n = (uint32_t)(s1 - s0);
    if (n <= lo_cap || n > CAP) continue;  // another size class (n = 0: nothing to do)
    u32x4 v[PT];
    if (runs.pairs) {
      __syncthreads();  // the previous bucket's gather has read its record indices out of buf
      // chunked top pass: the bucket is one run per chunk.  Its run table goes to buf (free until
      // the first digit pass): the run's first pair and its offset in the bucket, per chunk;
      // thread t owns chunks [t K, (t + 1) K)
      uint32_t* rstart = reinterpret_cast<uint32_t*>(buf);
      uint32_t* rpre = rstart + runs.nch;
      const uint32_t K = (runs.nch + NT - 1) / NT;
      uint32_t sum = 0;
      for (uint32_t k = 0; k < K; ++k) {
        const uint32_t c = tid * K + k;
        if (c >= runs.nch) break;
        const uint16_t* row = runs.offs + (uint64_t)c * (R + 1) + b;
        const uint32_t o = row[0];
        rstart[c] = c * kTopChunk + o;
        rpre[c] = sum;
        sum += (uint32_t)row[1] - o;
      }
      const uint32_t incl = wave_incl_scan(sum, lane);
      if (lane == kWave - 1) wsum[wave] = incl;
      __syncthreads();
      uint32_t ex = incl - sum;
#pragma unroll
      for (uint32_t q = 0; q < NW; ++q) ex += q < (uint32_t)wave ? wsum[q] : 0u;
      for (uint32_t k = 0; k < K; ++k) {
        const uint32_t c = tid * K + k;
        if (c >= runs.nch) break;
        rpre[c] += ex;
      }
      __syncthreads();
      // the last run starting at or before e: a branch-free search of fixed depth (kTopMaxChunks
      // = 2^11 runs), so the PT searches interleave
      static_assert(kTopMaxChunks == 2048, "search depth");
      uint32_t e[PT], lo[PT];
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        e[j] = min(wave * (PT * kWave) + j * kWave + lane, n - 1);
        lo[j] = 0;
      }
#pragma unroll
      for (uint32_t step = kTopMaxChunks / 2; step > 0; step >>= 1) {
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j) {
          const uint32_t t = lo[j] + step;
          if (t < runs.nch && rpre[t] <= e[j]) lo[j] = t;
        }
      }
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j)  // unconditional (clamped) loads
        v[j] = static_cast<const u32x4*>(runs.pairs)[rstart[lo[j]] + (e[j] - rpre[lo[j]])];
      __syncthreads();  // every run-table read is done before a digit pass rewrites buf
    } else {
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {  // unconditional (clamped) loads: no per-load wait
        const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
        v[j] = in[s0 + min(e, n - 1)];
      }
    }
    if constexpr (GATHER) {
      if (plan->rebase) {
        // u = K - (the bucket's smallest key), in the pair's top rbits bits; the record index
        // (word 3) stays.  u < 2^rbits: the plan bounds every bucket's key width
        u128 m = ~(u128)0;
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j) {
          const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
          const u128 k = pair_key(v[j], kbits);
          if (e < n && k < m) m = k;
        }
        for (int sft = 32; sft >= 1; sft >>= 1) {
          const u128 o = shfl_xor128(m, sft);
          m = o < m ? o : m;
        }
        if (lane == 0) rmin[wave] = m;
        __syncthreads();
        m = rmin[0];
#pragma unroll
        for (uint32_t q = 1; q < NW; ++q) m = rmin[q] < m ? rmin[q] : m;
        const int rb = plan->rbits;
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j) {
          const u128 u = pair_key(v[j], kbits) - m;
          const u128 nv = (u << (128 - rb)) | (u128)__builtin_bswap32(v[j][3]);
          v[j][0] = __builtin_bswap32((uint32_t)(nv >> 96));
          v[j][1] = __builtin_bswap32((uint32_t)(nv >> 64));
          v[j][2] = __builtin_bswap32((uint32_t)(nv >> 32));
        }
        __syncthreads();  // rmin is rewritten by the next bucket only after this
      }
    }
    // one stable 8-bit digit pass in LDS (digit d of dg): ranks, block scan, permutation into
    // buf, the pairs back into registers in the new order
    auto digit_pass = [&](int d) {
      const uint64_t w = d < 8 ? dg.lo : dg.hi;  // shifts packed 8 bits apiece
      const uint32_t sh = (uint32_t)(w >> (8 * (d & 7))) & 255u;
      uint32_t dig[PT], rank[PT];
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
        const bool valid = e < n;
        dig[j] = valid ? pair_digit8(v[j], sh) : 0u;
        rank[j] = wave_rank<8>(dig[j], valid, wc + wave * NB, lt_mask);
      }
      __syncthreads();
      scan_digit_wave<NB, NW>(wc, wsum, tid, lane, wave);
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j)
        if (rank[j] != ~0u) buf[wc[wave * NB + dig[j]] + rank[j]] = v[j];
      __syncthreads();
      for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
      // the next digit ranks the pairs in this digit's order: reload them, wave-contiguous
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
        if (e < n) v[j] = buf[e];
      }
      __syncthreads();  // every pair is back in registers before the next digit rewrites buf
    };
    // The top kTopDigits digits below the bucket's digit first (LSD among them): after them the
    // pairs are in order but for runs whose top digits tie — with random keys a few runs of 2
    // per bucket.  Each run is then finished in place by one thread (a stable insertion sort on
    // the key bits); a run longer than kMaxTieRun (duplicate-heavy keys) sends the bucket through
    // every digit pass instead, from this order (equal keys are still in input order, so the
    // LSD result stays stable).  With random TeraSort keys: 2 LDS passes instead of 9.
    const int nd = n > 1 ? dg.n : 0;
    const int K = nd < kTopDigits ? nd : kTopDigits;
    for (int d = nd - K; d < nd; ++d) digit_pass(d);
    if (nd > K) {
      const uint64_t wt = (nd - 1) < 8 ? dg.lo : dg.hi, wt2 = (nd - 2) < 8 ? dg.lo : dg.hi;
      const uint32_t sh1 = (uint32_t)(wt >> (8 * ((nd - 1) & 7))) & 255u;
      const uint32_t sh0 = (uint32_t)(wt2 >> (8 * ((nd - 2) & 7))) & 255u;
      auto top = [&](const u32x4& x) { return (pair_digit8(x, sh1) << 8) | pair_digit8(x, sh0); };
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
        if (e >= n) continue;
        const uint32_t t = top(v[j]);
        if ((e > 0 && top(buf[e - 1]) == t) || e + 1 >= n || top(buf[e + 1]) != t) continue;
        uint32_t L = 2;  // a run of >= 2 starts at e
        while (e + L < n && L <= kMaxTieRun && top(buf[e + L]) == t) ++L;
        if (L > kMaxTieRun) {
          atomicOr(&tie_redo, 1u);
          continue;
        }
        for (uint32_t i = 1; i < L; ++i) {  // stable: only strictly greater keys move up
          const u32x4 x = buf[e + i];
          uint32_t k = i;
          while (k > 0 && key_greater(buf[e + k - 1], x, tkbits)) {
            buf[e + k] = buf[e + k - 1];
            --k;
          }
          buf[e + k] = x;
        }
      }
      __syncthreads();
      const bool redo = tie_redo != 0;
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
        if (e < n) v[j] = buf[e];
      }
      __syncthreads();  // every thread read the flag and its pairs before anyone moves on
      if (tid == 0) tie_redo = 0;  // (read again only after the next bucket's first barrier)
      if (redo)
        for (int d = 0; d < nd; ++d) digit_pass(d);
    }
    if constexpr (GATHER) {
      // every thread passed a barrier after its last read of buf (each digit pass and the tie
      // fix-up end in one), so buf's first CAP dwords can take the record indices; the next
      // bucket writes buf only after a barrier, so the gather's reads of them are safe too
      uint32_t* sidx = reinterpret_cast<uint32_t*>(buf);
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
        if (e < n) sidx[e] = v[j][3];
      }
      __syncthreads();
      gather_run<NT, SUX_SORT_GATHER_U>(gth.in, gth.out + s0 * gth.rs, sidx, n, gth.rs, gth.lsh,
                                        (uint32_t)tid);
    } else {
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
        if (e < n) out[s0 + e] = v[j];
      }
    }
  }
}

// The fused sort's other records: a workgroup per 4096-record chunk of the output gathers the
// parts of the buckets overlapping it that k_sort_local<GATHER> did not — every bucket when the
// plan finished without it (no lower digit varies: the top pass's order; every key equal: the
// input order), else the buckets above kSortLocalCap (sorted as pairs by k_sort_bucket_global).
// Chunks of done buckets cost a binary search over the bucket index and nothing else.
constexpr uint32_t kGatherRestChunk = 4096;
__global__ __launch_bounds__(256) void k_gather_rest(const u32x4* __restrict__ pairs_a,
                                                     const u32x4* __restrict__ pairs_b,
                                                     const int64_t* __restrict__ index, uint32_t R,
                                                     uint64_t n, const SortPlanDev* __restrict__ plan,
                                                     SortGather gth) {
  __shared__ uint32_t sidx[kGatherRestChunk];
  __shared__ uint32_t b_first;
  const bool all = !plan->msd_ok || plan->dg.n == 0;
  if (!all && !plan->big) return;  // every bucket fit the LDS shapes, which gathered it
  const u32x4* pairs = plan->final_b ? pairs_b : pairs_a;
  const uint32_t tid = threadIdx.x;
  for (uint64_t c0 = (uint64_t)blockIdx.x * kGatherRestChunk; c0 < n;
       c0 += (uint64_t)gridDim.x * kGatherRestChunk) {
    const uint64_t c1 = min<uint64_t>(c0 + kGatherRestChunk, n);
    if (tid == 0) {  // the last bucket starting at or before c0
      uint32_t lo = 0, hi = R;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((uint64_t)index[mid] / 16 <= c0) lo = mid; else hi = mid;
      }
      b_first = lo;
    }
    __syncthreads();
    for (uint32_t b = b_first; b < R; ++b) {
      const uint64_t s0 = (uint64_t)index[b] / 16, s1 = (uint64_t)index[b + 1] / 16;
      if (s0 >= c1) break;
      const uint64_t r0 = max(s0, c0), r1 = min(s1, c1);
      if (r0 >= r1 || (!all && s1 - s0 <= kSortLocalCap)) continue;
      const uint32_t m = (uint32_t)(r1 - r0);
      for (uint32_t e = tid; e < m; e += 256) sidx[e] = pairs[r0 + e][3];
      __syncthreads();
      gather_run<256, 4>(gth.in, gth.out + r0 * gth.rs, sidx, m, gth.rs, gth.lsh, tid);
      __syncthreads();
    }
    __syncthreads();  // b_first is rewritten for the next chunk
  }
}

// Buckets above kSortLocalCap (skewed keys: heavy hitters, long duplicate runs): one
// 1024-thread workgroup per bucket runs a stable LSD over the plan's digits through global
// memory — one counting sweep for every digit, then per varying digit a ranked scatter sweep in
// 4096-element chunks (wave-ballot
// ranks + one (digit, wave) scan per chunk, per-digit cursors carried across chunks), ping-ponging
// between the bucket's range of the top pass's output (`in`) and of the final buffer (`out`), and
// ends in `out` (one copy when the digit count is even).  Slow per bucket (one CU), but only a
// skewed key set has such buckets, and it replaces round 2's fallback to the whole LSD sort.
template <uint32_t NW>
__global__ __launch_bounds__(NW * 64) void k_sort_bucket_global(u32x4* __restrict__ in,
                                                                u32x4* __restrict__ out,
                                                                const int64_t* __restrict__ index,
                                                                uint32_t R,
                                                                const SortPlanDev* __restrict__ plan) {
  if (!plan->msd_ok || plan->dg.n == 0) return;
  const SortDigits dg = plan->rebase ? plan->dg_raw : plan->dg;  // its pairs are not rebased
  constexpr uint32_t NT = NW * kWave, NB = 256, PT = 4, CH = NT * PT;
  __shared__ uint32_t wc[NW * NB];
  __shared__ uint32_t wsum[NW];
  __shared__ uint32_t cur[NB];
  __shared__ uint32_t hist[16 * NB];  // [digit][value] counts of the bucket (SortDigits: <= 16)
  __shared__ uint32_t one_bin;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
  __syncthreads();
  for (uint32_t b = blockIdx.x; b < R; b += gridDim.x) {
    const uint64_t s0 = (uint64_t)index[b] / 16, s1 = (uint64_t)index[b + 1] / 16;
    const uint32_t n = (uint32_t)(s1 - s0);
    if (n <= kSortLocalCap) continue;  // k_sort_local's
    u32x4* src = in + s0;
    u32x4* dst = out + s0;
    // ONE counting sweep for every digit (the per-digit count sweeps read the bucket once more
    // per digit): each wave's equal digits are matched by ballots and added by their first lane
    // (one LDS atomic per distinct digit value per wave, so a heavy hitter's equal keys do not
    // serialise on one counter).  A digit whose histogram is one bin is constant inside the
    // bucket — an identity pass, skipped (a bucket of equal keys skips them all).
    for (uint32_t i = tid; i < 16 * NB; i += NT) hist[i] = 0;
    __syncthreads();
    for (uint32_t c0 = 0; c0 < n; c0 += CH) {
      u32x4 v[PT];
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t e = c0 + wave * (PT * kWave) + j * kWave + lane;
        v[j] = src[e < n ? e : n - 1];
      }
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t e = c0 + wave * (PT * kWave) + j * kWave + lane;
        const bool valid = e < n;
        for (int d = 0; d < dg.n; ++d) {
          const uint64_t w = d < 8 ? dg.lo : dg.hi;
          const uint32_t dig = pair_digit8(v[j], (uint32_t)(w >> (8 * (d & 7))) & 255u);
          uint64_t peers = __ballot(valid);
#pragma unroll
          for (uint32_t bb = 0; bb < 8; ++bb) {
            const bool bit = (dig >> bb) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
          }
          if (valid && (peers & lt_mask) == 0) atomicAdd(&hist[d * NB + dig], (uint32_t)__popcll(peers));
        }
      }
    }
    __syncthreads();
    for (int d = 0; d < dg.n; ++d) {
      const uint64_t w = d < 8 ? dg.lo : dg.hi;
      const uint32_t sh = (uint32_t)(w >> (8 * (d & 7))) & 255u;
      // exclusive digit starts in cur; one bin holding every pair: the digit is constant
      if (tid == 0) one_bin = 0;
      __syncthreads();
      uint32_t x = 0, incl = 0;
      if (tid < (int)NB) {
        x = hist[d * NB + tid];
        if (x == n) one_bin = 1;
        incl = wave_incl_scan(x, lane);
        if (lane == kWave - 1) wsum[wave] = incl;
      }
      __syncthreads();
      const bool constant = one_bin != 0;
      __syncthreads();  // every thread has read one_bin before the next digit resets it
      if (constant) continue;
      if (tid < (int)NB) {
        uint32_t base = 0;
        for (int q = 0; q < wave; ++q) base += wsum[q];
        cur[tid] = base + incl - x;
      }
      __syncthreads();
      // ranked scatter, chunk by chunk in element order (stable).  The next chunk's pairs are
      // loaded while this one is ranked and scattered (src and dst are different buffers inside
      // a digit pass): one workgroup's sweep otherwise waited a full memory round trip per chunk
      u32x4 vn[PT];
      auto load_chunk = [&](uint32_t c0, u32x4 (&x)[PT]) {
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j) {
          const uint32_t e = c0 + wave * (PT * kWave) + j * kWave + lane;
          x[j] = src[e < n ? e : n - 1];
        }
      };
      load_chunk(0, vn);
      for (uint32_t c0 = 0; c0 < n; c0 += CH) {
        u32x4 v[PT];
        uint32_t dig[PT], rank[PT];
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j) v[j] = vn[j];
        if (c0 + CH < n) load_chunk(c0 + CH, vn);  // uniform
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j) {
          const uint32_t e = c0 + wave * (PT * kWave) + j * kWave + lane;
          const bool valid = e < n;
          dig[j] = valid ? pair_digit8(v[j], sh) : 0u;
          rank[j] = wave_rank<8>(dig[j], valid, wc + wave * NB, lt_mask);
        }
        __syncthreads();
        scan_digit_wave<NB, NW>(wc, wsum, tid, lane, wave);
        // wc[w][t] is the chunk-wide (digit, wave) prefix; wc[0][t] = where digit t starts in
        // the chunk, so wc[w][t] - wc[0][t] is wave w's offset inside the chunk's digit-t run
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j)
          if (rank[j] != ~0u)
            dst[cur[dig[j]] + (wc[wave * NB + dig[j]] - wc[dig[j]]) + rank[j]] = v[j];
        __syncthreads();
        // the chunk's digit counts advance the cursors: start of digit t+1 minus start of t
        const uint32_t cn = min(CH, n - c0);
        uint32_t adv = 0;
        if (tid < (int)NB) adv = ((uint32_t)tid + 1 < NB ? wc[tid + 1] : cn) - wc[tid];
        __syncthreads();
        if (tid < (int)NB) cur[tid] += adv;
        for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
        __syncthreads();
      }
      u32x4* t = src;
      src = dst;
      dst = t;
      __threadfence_block();
      __syncthreads();
    }
    if (src != out + s0) {  // an even number of digits: the result sits in `in`
      for (uint32_t e = tid; e < n; e += NT) out[s0 + e] = src[e];
      __syncthreads();
    }
  }
}

// True when bits [lo, hi) of the big-endian 128-bit pair differ between some records (span: the
// AND of key words 0..2, then their OR) — sux_api.cpp's span_varies, on the device.
// The key bits that vary, as the big-endian 128-bit pair value (bit b = pair bit b; the index word's
// bits, below 32, are 0): AND ^ OR of the key words, byte-swapped like pair_be128.  Held in
// registers: testing the span bit by bit from LDS cost ~10 us of single-thread latency per sort.
__device__ __forceinline__ u128 span_vary_mask(const uint32_t* span) {
  u32x4 d;
  d[0] = span[0] ^ span[3];
  d[1] = span[1] ^ span[4];
  d[2] = span[2] ^ span[5];
  d[3] = 0u;
  return pair_be128(d);
}
// some bit in [lo, hi) varies (lo < hi <= 128)
__device__ __forceinline__ bool vary_in(u128 v, int lo, int hi) {
  const u128 m = (hi - lo >= 128) ? ~(u128)0 : ((((u128)1) << (hi - lo)) - 1);
  return ((v >> lo) & m) != 0;
}

// The plan from the key span (AND of key words 0..2, then their OR): the highest varying key
// bit, the top digit (its tb bits end there) and the LDS sort's 8-bit digits below it that vary.
// One thread (k_span_reduce's thread 0).
__device__ void make_sort_plan(const uint32_t* span, int bits, int tb, SortPlanDev* plan,
                               const u128* range, bool rebase_ok) {
  const u128 vary = span_vary_mask(span) & (~(u128)0 << (128 - bits));
  const uint64_t vh = (uint64_t)(vary >> 64), vl = (uint64_t)vary;
  const int hb = vh ? 127 - __builtin_clzll(vh) : vl ? 63 - __builtin_clzll(vl) : -1;
  int top_lo = hb >= 0 ? max(hb + 1 - tb, 128 - bits) : 128 - bits;
  uint64_t top_base = 0;
  plan->rebase = 0;
  if (range && hb >= 0) {
    // the lowest shift at which the aligned blocks the keys [min, max] touch number <= 2^tb (the
    // bit-span shift above always qualifies: every key shares the bits above hb)
    const u128 mn = range[0], mx = range[1];
    int sh = 128 - bits;
    const u128 d = mx - mn;
    const int dl = 128 - (int)(d >> 64 ? __builtin_clzll((uint64_t)(d >> 64))
                                       : 64 + ((uint64_t)d ? __builtin_clzll((uint64_t)d) : 64));
    sh = max(sh, dl - tb);  // below it the span alone needs more than 2^tb blocks
    // the lowest sh in [sh, top_lo] with (mx >> sh) - (mn >> sh) < 2^tb (non-increasing in sh,
    // and true at top_lo): a binary search, not a step per bit (one thread plans the sort)
    if (sh < top_lo && ((mx >> sh) - (mn >> sh)) >= ((u128)1 << tb)) {
      int lo = sh, hi = top_lo;  // f(lo) fails, f(hi) holds
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (((mx >> mid) - (mn >> mid)) >= ((u128)1 << tb)) lo = mid; else hi = mid;
      }
      sh = hi;
    }
    top_lo = min(sh, top_lo);
    top_base = (uint64_t)(mn >> top_lo);
    // Rebase (fused-gather sorts only) when the aligned blocks leave more than a third of the
    // 2^tb buckets empty — a range partition's keys, whose width is no power of two: equal
    // slices of [kmin, kmax] instead, each bucket sorted by its keys' offset from its smallest
    const u128 blocks = (mx >> top_lo) - (mn >> top_lo) + 1;
    if (rebase_ok && blocks * 3 < ((u128)2 << tb)) {
      const u128 kmin = mn >> (128 - bits), kd = (mx >> (128 - bits)) - kmin;
      const int kl = kd >> 64 ? 128 - __builtin_clzll((uint64_t)(kd >> 64))
                              : ((uint64_t)kd ? 64 - __builtin_clzll((uint64_t)kd) : 0);
      const uint32_t q = kl > 32 ? (uint32_t)(kl - 32) : 0u;
      const uint64_t dd = (uint64_t)(kd >> q) + 1;  // <= 2^32
      const uint64_t rm = (((uint64_t)1 << tb) << 32) / dd;
      // a bucket's key width: < (ceil(2^32 / rm) + 1) << q
      const u128 w = ((u128)(((uint64_t)1 << 32) / rm + 2)) << q;
      const int rb = w >> 64 ? 128 - __builtin_clzll((uint64_t)(w >> 64))
                             : 64 - __builtin_clzll((uint64_t)w);
      if (rb <= 96 && rm > 0) {
        plan->rebase = 1;
        plan->rbits = rb;
        plan->rq = q;
        plan->rm = rm;
        plan->kmin_hi = (uint64_t)(kmin >> 64);
        plan->kmin_lo = (uint64_t)kmin;
      }
    }
  }
  // The LDS digits hang down from the top digit — [top_lo - 8, top_lo), [top_lo - 16, top_lo -
  // 8), ... — so the two the bucket sort runs first (and whose ties its insertion sort finishes)
  // hold 16 bits that vary inside a bucket.  Counted up from the key's lowest bit instead, the
  // highest digit straddled the top digit's constant bits: int64 keys below 2^31 kept 9 varying
  // bits in those two digits (tie runs of ~4 in 2048-pair buckets, the 32 Mi-row sort 2.1 -> 3.8
  // ms).  The lowest digit is clamped to the key's first bit (it may overlap the digit above it:
  // LSD over overlapping digits still orders by the whole key, and no bit below the key — record
  // payload in inline mode — is ever a digit); a digit whose new bits never vary is skipped.
  SortDigits dg{};
  uint32_t shs[16];
  int m = 0;
  for (int hi = top_lo; hi > 128 - bits && m < 16; hi -= 8) {
    const int sh = max(hi - 8, 128 - bits);
    if (vary_in(vary, sh, hi)) shs[m++] = (uint32_t)sh;
  }
  for (int i = m - 1; i >= 0; --i) dg.push(shs[i]);  // least significant first
  if (plan->rebase) {
    // the global sort of oversized buckets orders raw pairs by every key digit; the LDS sort
    // orders rebased pairs by u's digits, hanging down from bit 128 to 128 - rbits
    SortDigits raw{};
    uint32_t rsh[16];
    int rn = 0;
    for (int hi = 128; hi > 128 - bits && rn < 16; hi -= 8) rsh[rn++] = (uint32_t)max(hi - 8, 128 - bits);
    for (int i = rn - 1; i >= 0; --i) raw.push(rsh[i]);
    plan->dg_raw = raw;
    SortDigits ud{};
    rn = 0;
    for (int hi = 128; hi > 128 - plan->rbits && rn < 16; hi -= 8)
      rsh[rn++] = (uint32_t)max(hi - 8, 128 - plan->rbits);
    for (int i = rn - 1; i >= 0; --i) ud.push(rsh[i]);
    dg = ud;
  }
  plan->top_lo = top_lo;
  plan->top_base = top_base;
  plan->hb = hb;
  plan->kbits = bits;
  plan->dg = dg;
  // buckets up to kSortLocalCap sort in LDS (k_sort_local), larger ones through global memory
  // (k_sort_bucket_global): the MSD path always finishes once some key bit varies.  The pairs
  // go a -> top pass -> b -> bucket sorts -> a; with no lower digit varying they end in the top
  // pass's b; with every key equal, in a (the input order)
  plan->msd_ok = hb >= 0 ? 1u : 0u;
  plan->big = 1u;  // until k_top_scan has seen every bucket fit
  plan->final_b = hb < 0 ? 0u : (dg.n ? 0u : 1u);
}

template <bool GATHER>
static void launch_sort_local_classes(const u32x4* in, u32x4* out, const int64_t* d_index,
                                      uint32_t R, const SortPlanDev* plan, const SortGather& gth,
                                      const SortRuns& runs, uint32_t ncu, uint64_t avg,
                                      hipStream_t s) {
  // size classes (0, 1024], (1024, 2048] (the third, (2048, kSortLocalCap], is launched by the
  // caller on the side stream): each bucket on the smallest shape that holds it — unless the
  // buckets average above 1024 pairs: then the few small ones (the key range's edge buckets) go to
  // the 2048-pair launch too, instead of a launch of their own whose one or two buckets cost a
  // bucket's whole latency chain (~30 us: run table, digit passes, gather) ahead of it
  const bool small_class = avg <= 1024;
  if (small_class) {
    constexpr size_t l1 = SortLocal<4, 1024>::lds_bytes();
    hipLaunchKernelGGL((k_sort_local<4, 1024, GATHER>), dim3(std::min<uint32_t>(R, 6 * ncu)),
                       dim3(4 * kWave), l1, s, in, out, d_index, R, 0u, plan, gth, runs);
  }
  constexpr size_t l2 = SortLocal<4, 2048>::lds_bytes();
  static_assert(4 * l2 <= 160 * 1024, "four workgroups per CU");
  hipLaunchKernelGGL((k_sort_local<4, 2048, GATHER>), dim3(std::min<uint32_t>(R, 4 * ncu)),
                     dim3(4 * kWave), l2, s, in, out, d_index, R, small_class ? 1024u : 0u, plan,
                     gth, runs);
}

hipError_t launch_sort_local_planned(const void* in_pairs, void* out_pairs, const int64_t* d_index,
                                     uint32_t R, const SortPlanDev* plan, hipStream_t s,
                                     const void* recs_in, void* recs_out, uint32_t rs,
                                     const SortRuns& runs, const SortSide& side, uint64_t avg) {
  const uint32_t ncu = (uint32_t)std::max(1, stream_cus(s));
  const u32x4* in = static_cast<const u32x4*>(in_pairs);
  u32x4* out = static_cast<u32x4*>(out_pairs);
  SortGather gth{static_cast<const uint8_t*>(recs_in), static_cast<uint8_t*>(recs_out), rs, 0};
  while (gth.lsh < 6 && (16u << gth.lsh) < rs) ++gth.lsh;
  // The buckets above the common 2048-pair shape (a few of them when the buckets average close
  // to 2048 pairs: a range partition's keys fill only part of the top digit) and those for the
  // global sort go on a side stream, launched first, so they overlap the main LDS launch instead
  // of trailing it one bucket per workgroup.  Every launch writes only its own buckets' ranges.
  hipStream_t sb = s;
  if (side.s) {
    hipError_t e = hipEventRecord(side.fork, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(side.s, side.fork, 0);
    if (e != hipSuccess) return e;
    sb = side.s;
  }
  constexpr size_t l3 = SortLocal<8, kSortLocalCap>::lds_bytes();
  static_assert(2 * l3 <= 160 * 1024, "two workgroups per CU");
  if (recs_out) {
    allow_lds(reinterpret_cast<const void*>(&k_sort_local<8, kSortLocalCap, true>), l3);
    hipLaunchKernelGGL((k_sort_local<8, kSortLocalCap, true>), dim3(std::min<uint32_t>(R, 2 * ncu)),
                       dim3(8 * kWave), l3, sb, in, out, d_index, R, 2048u, plan, gth, runs);
  } else {
    allow_lds(reinterpret_cast<const void*>(&k_sort_local<8, kSortLocalCap, false>), l3);
    hipLaunchKernelGGL((k_sort_local<8, kSortLocalCap, false>), dim3(std::min<uint32_t>(R, 2 * ncu)),
                       dim3(8 * kWave), l3, sb, in, out, d_index, R, 2048u, plan, gth, runs);
  }
  if (runs.pairs)  // the buckets left to the global sort (or the whole order) into `in` = b
    hipLaunchKernelGGL(k_top_materialize, dim3(std::min<uint32_t>(R, 4 * ncu)), dim3(256), 0, sb,
                       static_cast<const u32x4*>(runs.pairs), runs.offs, runs.nch, R, d_index, plan,
                       const_cast<u32x4*>(in));
  hipLaunchKernelGGL((k_sort_bucket_global<16>), dim3(std::min<uint32_t>(R, ncu)), dim3(16 * kWave),
                     0, sb, const_cast<u32x4*>(in), out, d_index, R, plan);
  if (recs_out)
    launch_sort_local_classes<true>(in, out, d_index, R, plan, gth, runs, ncu, avg, s);
  else
    launch_sort_local_classes<false>(in, out, d_index, R, plan, gth, runs, ncu, avg, s);
  if (side.s) {
    hipError_t e = hipEventRecord(side.join, side.s);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, side.join, 0);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

bool sort_gather_fusable(uint32_t rs) { return rs >= 16 && rs % 4 == 0 && rs <= 1024; }

hipError_t launch_gather_rest(const void* recs_in, const void* pairs_a, const void* pairs_b,
                              const int64_t* d_index, uint32_t R, uint64_t n,
                              const SortPlanDev* plan, uint32_t rs, void* recs_out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  SortGather gth{static_cast<const uint8_t*>(recs_in), static_cast<uint8_t*>(recs_out), rs, 0};
  while (gth.lsh < 6 && (16u << gth.lsh) < rs) ++gth.lsh;
  const uint64_t chunks = (n + kGatherRestChunk - 1) / kGatherRestChunk;
  hipLaunchKernelGGL(k_gather_rest, dim3((uint32_t)std::min<uint64_t>(chunks, 8192)), dim3(256), 0,
                     s, static_cast<const u32x4*>(pairs_a), static_cast<const u32x4*>(pairs_b),
                     d_index, R, n, plan, gth);
  return hipGetLastError();
}

}  // namespace sux
