// sux_partition.hip — map-side hot path for gfx950.
//
// One launch group = M consecutive map batches (default 32 x 100 MB).  Four kernels:
//   K1 hist      key -> partition id (P1), pid store, LDS histograms, counts[m][p][tile]
//                (partition-major).  Default k_hist4: persistent; a workgroup's 4 waves split a
//                4096-record tile, read it as coalesced 16-byte units through a wave LDS stage
//                with two chunks in flight, and look keys up in an LDS range table.
//   K2a k_tile_scan one wave per (map, partition): exclusive scan of counts over tiles in place,
//                totals[m][p].
//   K2b k_group_scan one workgroup per group: per-map index tables (P3, native + big-endian) and
//                the destination base of every (map, partition) for the chosen layout.
//   K3 scatter   stable regroup of the records by pid (P2).  Default k_scatter7: persistent, one
//                1024-thread workgroup per CU, 1024-record chunks staged straight into a
//                partition-sorted LDS image in destination-unit space, written out as aligned
//                16-byte stores; the next chunk's loads fly during the write-out.
// Older shapes (other record sizes, R beyond the LDS image) use the v1/v2/v3/v6 kernels below.
//
// Stability: records are visited in input order (waves in order inside a chunk, chunks in order
// inside a tile range, tile ranges ordered by the partition-major tile prefix); equal pids inside
// 64 lanes are ranked by a ballot match.  So records keep input order inside a partition, as
// Spark's writers do (P2).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "sux_internal.h"

namespace sux {

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

constexpr int kWave = 64;

// P1: partition functions — sux_p1.h
#include "sux_p1.h"

// ------------------------------------------------------------------------------------------
// geometry helpers
// ------------------------------------------------------------------------------------------
struct TileRange {
  uint32_t map, tile;
  uint64_t begin, end;  // record indices within the group
};

__device__ __forceinline__ TileRange tile_range(const MapGroup& g, uint32_t gtile) {
  TileRange tr;
  tr.map = gtile / g.tiles_per_map;
  tr.tile = gtile - tr.map * g.tiles_per_map;
  uint64_t map_begin = (uint64_t)tr.map * g.records_per_map;
  uint64_t map_end = map_begin + g.records_per_map;
  if (map_end > g.num_records) map_end = g.num_records;
  tr.begin = map_begin + (uint64_t)tr.tile * g.tile_recs;
  tr.end = tr.begin + g.tile_recs;
  if (tr.end > map_end) tr.end = map_end;
  if (tr.begin > tr.end) tr.begin = tr.end;
  return tr;
}

// xcd_map: sux_p1.h

// ------------------------------------------------------------------------------------------
// K1: partition ids + per-tile histogram
// ------------------------------------------------------------------------------------------
template <int WPG>
__global__ __launch_bounds__(WPG * kWave) void k_hist(PartDev pd, MapGroup g, uint16_t* pids,
                                                      uint32_t* counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const uint32_t gtile = blockIdx.x * WPG + wave;
  const uint32_t total_tiles = g.num_maps * g.tiles_per_map;
  const int R = pd.R;
  uint32_t* hist = lds + wave * R;
  for (int p = lane; p < R; p += kWave) hist[p] = 0;
  __builtin_amdgcn_wave_barrier();
  if (gtile >= total_tiles) return;
  const TileRange tr = tile_range(g, gtile);
  for (uint64_t i = tr.begin + lane; i < tr.end; i += kWave) {
    int p = get_partition(pd, g.recs + i * g.rec_size);
    pids[i] = (uint16_t)p;
    atomicAdd(&hist[p], 1u);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint32_t* dst = counts + ((uint64_t)tr.map * R) * g.tiles_per_map + tr.tile;
  for (int p = lane; p < R; p += kWave) dst[(uint64_t)p * g.tiles_per_map] = hist[p];
}

// ------------------------------------------------------------------------------------------
// K2a: exclusive scan over tiles of each (map, partition) row; row totals
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    uint32_t t = __shfl_up(v, d, kWave);
    if (lane >= d) v += t;
  }
  return v;
}

__global__ __launch_bounds__(256) void k_tile_scan(uint32_t* counts, uint64_t* totals,
                                                   uint32_t rows, uint32_t tiles) {
  const int lane = threadIdx.x % kWave;
  const uint32_t row = blockIdx.x * 4 + threadIdx.x / kWave;
  if (row >= rows) return;
  uint32_t* c = counts + (uint64_t)row * tiles;
  uint32_t carry = 0;
  constexpr int U = 8;  // all loads of 8 x 64 tiles in flight before the first scan
  for (uint32_t t0 = 0; t0 < tiles; t0 += kWave * U) {
    uint32_t v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t t = t0 + k * kWave + lane;
      v[k] = t < tiles ? c[t] : 0u;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t t = t0 + k * kWave + lane;
      const uint32_t inc = wave_incl_scan(v[k], lane);
      if (t < tiles) c[t] = carry + inc - v[k];
      carry += __shfl(inc, kWave - 1, kWave);
    }
  }
  if (lane == 0) totals[row] = carry;
}

// Few tiles per map (large R: 10,000 partitions x 16 tiles): one thread per row, so a row of
// T <= 64 counters is not a whole (mostly idle) wave.
__global__ __launch_bounds__(256) void k_tile_scan_rows(uint32_t* counts, uint64_t* totals,
                                                        uint32_t rows, uint32_t tiles) {
  const uint32_t row = blockIdx.x * 256 + threadIdx.x;
  if (row >= rows) return;
  uint32_t* c = counts + (uint64_t)row * tiles;
  uint32_t carry = 0;
  uint32_t t = 0;
  for (; t + 8 <= tiles; t += 8) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = c[t + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      c[t + k] = carry;
      carry += v[k];
    }
  }
  for (; t < tiles; ++t) {
    const uint32_t v = c[t];
    c[t] = carry;
    carry += v;
  }
  totals[row] = carry;
}

// Tile-major counts [map][tile][p] (the small-record path and the sort's digit passes).  A
// workgroup owns 16 partitions of one map; its 16 x 16 threads each sum one of 16 segments of
// the tile column (reads: 16 consecutive counters of one tile row per wave quarter), the 16
// segment sums of a partition are scanned in LDS, and every thread rewrites its segment.
__global__ __launch_bounds__(256) void k_tile_scan_tm(uint32_t* counts, uint64_t* totals,
                                                      uint32_t maps, uint32_t R, uint32_t tiles) {
  __shared__ uint32_t seg[16][17];
  const uint32_t pl = threadIdx.x % 16, sg = threadIdx.x / 16;
  const uint32_t pgroups = (R + 15) / 16;
  const uint32_t m = blockIdx.x / pgroups, p = (blockIdx.x - m * pgroups) * 16 + pl;
  const uint32_t per = (tiles + 15) / 16, t0 = min(sg * per, tiles), t1 = min(t0 + per, tiles);
  uint32_t* c = counts + (uint64_t)m * tiles * R + p;
  uint32_t sum = 0;
  if (p < R)
    for (uint32_t t = t0; t < t1; ++t) sum += c[(uint64_t)t * R];
  seg[pl][sg] = sum;
  __syncthreads();
  if (sg == 0) {
    uint32_t run = 0;
    for (int k = 0; k < 16; ++k) {
      const uint32_t x = seg[pl][k];
      seg[pl][k] = run;
      run += x;
    }
    if (p < R) totals[(uint64_t)m * R + p] = run;
  }
  __syncthreads();
  if (p < R) {
    uint32_t carry = seg[pl][sg];
    for (uint32_t t = t0; t < t1; ++t) {
      const uint32_t v = c[(uint64_t)t * R];
      c[(uint64_t)t * R] = carry;
      carry += v;
    }
  }
}

// ------------------------------------------------------------------------------------------
// K2b: per-group scans -> index tables and destination bases
// ------------------------------------------------------------------------------------------
constexpr int kScanThreads = 1024;

// Block-wide exclusive scan of one u64 per thread; returns the exclusive prefix, *total = sum.
__device__ uint64_t block_excl_scan(uint64_t v, uint64_t* sh, uint64_t* total) {
  const int lane = threadIdx.x % kWave, wave = threadIdx.x / kWave;
  constexpr int nw = kScanThreads / kWave;
  uint64_t inc = v;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    uint64_t t = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += t;
  }
  if (lane == kWave - 1) sh[wave] = inc;
  __syncthreads();
  if (wave == 0) {
    uint64_t w = lane < nw ? sh[lane] : 0;
    uint64_t wi = w;
#pragma unroll
    for (int d = 1; d < nw; d <<= 1) {
      uint64_t t = __shfl_up(wi, d, kWave);
      if (lane >= d) wi += t;
    }
    if (lane < nw) sh[kWave + lane] = wi - w;
    if (lane == nw - 1) sh[2 * kWave] = wi;
  }
  __syncthreads();
  uint64_t r = sh[kWave + wave] + inc - v;
  *total = sh[2 * kWave];
  __syncthreads();
  return r;
}

__device__ __forceinline__ uint64_t bswap64(uint64_t v) {
  return ((uint64_t)__builtin_bswap32((uint32_t)v) << 32) | __builtin_bswap32((uint32_t)(v >> 32));
}

__device__ __forceinline__ uint32_t owner_of(uint32_t p, int R, int G) {
  // largest h with floor(h*R/G) <= p
  return (uint32_t)((((uint64_t)p + 1) * G + R - 1) / R) - 1;
}

// K2b: one workgroup per map.  In-map exclusive scan of the partition totals -> the map's index
// file (P3: native and big-endian), and
//   G == 1 (map-major data files): base[m][p] = m * records_per_map + prefix (all maps but the
//          last are full, so map m's data file starts at record m * records_per_map);
//   G > 1  (peer-major send layout): prefix -> pre[m][p], per-peer sums -> mh[m][h].
// Maps are independent, so the launch has M workgroups (was one workgroup over M x R).
__global__ __launch_bounds__(kScanThreads) void k_map_scan(const uint64_t* __restrict__ totals,
                                                           uint64_t* __restrict__ base,
                                                           uint64_t* __restrict__ pre,
                                                           uint64_t* __restrict__ mh,
                                                           int64_t* __restrict__ index,
                                                           uint8_t* __restrict__ index_be,
                                                           uint64_t* __restrict__ peer_bytes,
                                                           int R, int G, uint32_t rec_size,
                                                           uint64_t records_per_map,
                                                           uint64_t num_records,
                                                           const uint64_t* __restrict__ map_offs) {
  __shared__ uint64_t sh[2 * kWave + 1];
  __shared__ unsigned long long hs[1024];
  const uint32_t m = blockIdx.x;
  const uint64_t* tm = totals + (uint64_t)m * R;
  int64_t* im = index + (uint64_t)m * (R + 1);
  uint64_t* ibe = index_be ? reinterpret_cast<uint64_t*>(index_be) + (uint64_t)m * (R + 1) : nullptr;
  if (G > 1)
    for (int h = threadIdx.x; h < G; h += kScanThreads) hs[h] = 0;
  uint64_t carry = 0;
  for (int p0 = 0; p0 < R; p0 += kScanThreads) {
    const int p = p0 + threadIdx.x;
    const uint64_t v = p < R ? tm[p] : 0;
    uint64_t tot;
    const uint64_t ex = carry + block_excl_scan(v, sh, &tot);  // barriers inside
    if (p < R) {
      const int64_t off = (int64_t)(ex * rec_size);
      im[p] = off;
      if (ibe) ibe[p] = bswap64((uint64_t)off);
      if (map_offs) {  // variable-length records: bases and offsets in bytes
        base[(uint64_t)m * R + p] = (map_offs[(uint64_t)m * records_per_map] - map_offs[0]) + ex;
      } else if (G == 1) {
        base[(uint64_t)m * R + p] = (uint64_t)m * records_per_map + ex;
      } else {
        pre[(uint64_t)m * R + p] = ex;
        atomicAdd(&hs[owner_of((uint32_t)p, R, G)], (unsigned long long)v);
      }
    }
    carry += tot;
  }
  if (threadIdx.x == 0) {
    const int64_t off = (int64_t)(carry * rec_size);
    im[R] = off;
    if (ibe) ibe[R] = bswap64((uint64_t)off);
    if (G == 1 && m == 0 && peer_bytes) peer_bytes[0] = num_records * rec_size;
  }
  if (G > 1) {
    __syncthreads();
    for (int h = threadIdx.x; h < G; h += kScanThreads) mh[(uint64_t)m * G + h] = hs[h];
  }
}

// G > 1: per-peer byte counts, then an exclusive scan of mh in peer-major (h, m) order, in place:
// mh[m][h] becomes the send-buffer record offset of (peer h, map m).
__global__ __launch_bounds__(kScanThreads) void k_peer_off(uint64_t* __restrict__ mh,
                                                           uint64_t* __restrict__ peer_bytes,
                                                           uint32_t M, int G, uint32_t rec_size) {
  __shared__ uint64_t sh[2 * kWave + 1];
  if (peer_bytes)
    for (int h = threadIdx.x; h < G; h += kScanThreads) {
      uint64_t t = 0;
      for (uint32_t m = 0; m < M; ++m) t += mh[(uint64_t)m * G + h];
      peer_bytes[h] = t * rec_size;
    }
  __syncthreads();
  const uint64_t L = (uint64_t)M * G;
  uint64_t carry = 0;
  for (uint64_t j0 = 0; j0 < L; j0 += kScanThreads) {
    const uint64_t j = j0 + threadIdx.x;  // j = h * M + m
    uint64_t v = 0, idx = 0;
    if (j < L) {
      const uint64_t h = j / M, m = j - h * M;
      idx = m * G + h;
      v = mh[idx];
    }
    uint64_t tot;
    const uint64_t ex = carry + block_excl_scan(v, sh, &tot);
    if (j < L) mh[idx] = ex;
    carry += tot;
  }
}

// G > 1: base[m][p] = offset of (owner(p), m) + prefix of p inside its owner's range of map m.
__global__ __launch_bounds__(256) void k_peer_base(const uint64_t* __restrict__ pre,
                                                   const uint64_t* __restrict__ mh,
                                                   uint64_t* __restrict__ base, uint32_t M, int R,
                                                   int G) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= (uint64_t)M * R) return;
  const uint64_t m = j / R;
  const uint32_t p = (uint32_t)(j - m * R);
  const uint32_t h = owner_of(p, R, G);
  const uint32_t lo = (uint32_t)(((int64_t)h * R) / G);
  base[j] = mh[m * G + h] + pre[j] - pre[m * R + lo];
}

// ------------------------------------------------------------------------------------------
// K3: stable scatter
// ------------------------------------------------------------------------------------------
template <uint32_t S>
__device__ __forceinline__ void copy_record(const uint8_t* __restrict__ src,
                                           uint8_t* __restrict__ dst, uint32_t rs) {
  if constexpr (S != 0) {
#pragma unroll
    for (uint32_t k = 0; k + 16 <= S; k += 16)
      *reinterpret_cast<u32x4a4*>(dst + k) = *reinterpret_cast<const u32x4a4*>(src + k);
#pragma unroll
    for (uint32_t k = S - S % 16; k < S; k += 4)
      *reinterpret_cast<uint32_t*>(dst + k) = *reinterpret_cast<const uint32_t*>(src + k);
  } else {
    uint32_t k = 0;
    for (; k + 16 <= rs; k += 16)
      *reinterpret_cast<u32x4a4*>(dst + k) = *reinterpret_cast<const u32x4a4*>(src + k);
    for (; k < rs; k += 4)
      *reinterpret_cast<uint32_t*>(dst + k) = *reinterpret_cast<const uint32_t*>(src + k);
  }
}

template <int WPG, uint32_t S>
__global__ __launch_bounds__(WPG * kWave) void k_scatter(MapGroup g, int R, int pid_bits,
                                                         const uint16_t* __restrict__ pids,
                                                         const uint32_t* __restrict__ prefix,
                                                         const uint64_t* __restrict__ base,
                                                         uint8_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const uint32_t gtile = blockIdx.x * WPG + wave;
  if (gtile >= g.num_maps * g.tiles_per_map) return;
  const TileRange tr = tile_range(g, gtile);
  if (tr.begin >= tr.end) return;
  const uint32_t rs = S ? S : g.rec_size;
  // running destination (in records, relative to the group output) of every partition
  uint32_t* run = lds + wave * R;
  const uint64_t* bm = base + (uint64_t)tr.map * R;
  const uint32_t* pm = prefix + (uint64_t)tr.map * R * g.tiles_per_map + tr.tile;
  for (int p = lane; p < R; p += kWave)
    run[p] = (uint32_t)(bm[p] + pm[(uint64_t)p * g.tiles_per_map]);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  for (uint64_t i0 = tr.begin; i0 < tr.end; i0 += kWave) {
    const uint64_t i = i0 + lane;
    const bool valid = i < tr.end;
    const uint32_t pid = valid ? pids[i] : 0u;
    uint64_t peers = __ballot(valid);
    for (int b = 0; b < pid_bits; ++b) {
      const bool bit = (pid >> b) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    uint32_t r0 = 0;
    if (valid) r0 = run[pid];
    __builtin_amdgcn_wave_barrier();
    if (valid && (peers & lt_mask) == 0) run[pid] = r0 + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      const uint32_t dst = r0 + (uint32_t)__popcll(peers & lt_mask);
      copy_record<S>(g.recs + i * rs, out + (uint64_t)dst * rs, rs);
    }
  }
}

// ------------------------------------------------------------------------------------------
// v2 kernels: a wave stages CH records of its tile in LDS with fully coalesced 16-byte loads
// (1 KiB per wave instruction), works on them there, and (scatter) writes them out record-
// coalesced: consecutive lanes store consecutive dwords, so a wave instruction covers ~2.5
// whole records instead of touching 64 cache lines.
// ------------------------------------------------------------------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <uint32_t S, uint32_t CH>
struct Stage {
  static constexpr uint32_t kUnits = (CH * S + 12 + 15) / 16;  // 16-B units incl. a <=12 B head
  static constexpr uint32_t kPer = (kUnits + kWave - 1) / kWave;
  static constexpr uint32_t kBufBytes = kUnits * 16;
};

// Load the 16-byte units covering [a, a + len) into `dst` (a is 4-byte aligned); returns the
// offset of `a` in dst.  Every unit holds a requested byte, so no load leaves the buffer's pages.
template <uint32_t PER>
__device__ __forceinline__ uint32_t stage_units(const uint8_t* a, uint32_t len, u32x4* dst,
                                                int lane) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(a);
  const uint32_t head = (uint32_t)(p & 15u);
  const u32x4* src = reinterpret_cast<const u32x4*>(p - head);
  const uint32_t units = (head + len + 15) >> 4;
  u32x4 v[PER];
#pragma unroll
  for (uint32_t k = 0; k < PER; ++k) {
    const uint32_t u = lane + k * kWave;
    if (u < units) v[k] = src[u];
  }
#pragma unroll
  for (uint32_t k = 0; k < PER; ++k) {
    const uint32_t u = lane + k * kWave;
    if (u < units) dst[u] = v[k];
  }
  return head;
}

template <uint32_t S, uint32_t CH>
__host__ __device__ constexpr uint32_t hist2_wave_bytes(int R) {
  return Stage<S, CH>::kBufBytes + (((uint32_t)R * 4 + 15) / 16) * 16;
}
template <uint32_t S, uint32_t CH>
__host__ __device__ constexpr uint32_t scatter2_wave_bytes(int R) {
  return Stage<S, CH>::kBufBytes + CH * 4 + (((uint32_t)R * 4 + 15) / 16) * 16;
}

template <uint32_t S, uint32_t CH>
__global__ __launch_bounds__(256) void k_hist2(PartDev pd, MapGroup g, uint16_t* __restrict__ pids,
                                               uint32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  using St = Stage<S, CH>;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int R = pd.R;
  uint8_t* wb = lds8 + wave * hist2_wave_bytes<S, CH>(R);
  u32x4* buf = reinterpret_cast<u32x4*>(wb);
  uint32_t* hist = reinterpret_cast<uint32_t*>(wb + St::kBufBytes);
  for (int p = lane; p < R; p += kWave) hist[p] = 0;
  const uint32_t gtile = blockIdx.x * 4 + wave;
  if (gtile >= g.num_maps * g.tiles_per_map) return;
  const TileRange tr = tile_range(g, gtile);
  for (uint64_t c0 = tr.begin; c0 < tr.end; c0 += CH) {
    const uint32_t nrec = (uint32_t)min<uint64_t>(CH, tr.end - c0);
    const uint32_t head = stage_units<St::kPer>(g.recs + c0 * S, nrec * S, buf, lane);
    __builtin_amdgcn_wave_barrier();
    const uint8_t* b = reinterpret_cast<const uint8_t*>(buf) + head;
#pragma unroll
    for (uint32_t j = 0; j < CH / kWave; ++j) {
      const uint32_t r = j * kWave + lane;
      if (r < nrec) {
        const int p = get_partition(pd, b + r * S);
        pids[c0 + r] = (uint16_t)p;
        atomicAdd(&hist[p], 1u);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint32_t* dst = counts + ((uint64_t)tr.map * R) * g.tiles_per_map + tr.tile;
  for (int p = lane; p < R; p += kWave) dst[(uint64_t)p * g.tiles_per_map] = hist[p];
}

template <uint32_t S, uint32_t CH>
__global__ __launch_bounds__(256) void k_scatter2(MapGroup g, int R, int pid_bits,
                                                  const uint16_t* __restrict__ pids,
                                                  const uint32_t* __restrict__ prefix,
                                                  const uint64_t* __restrict__ base,
                                                  uint8_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  using St = Stage<S, CH>;
  constexpr uint32_t W = S / 4;  // dwords per record
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const uint32_t gtile = xcd_map(blockIdx.x, gridDim.x) * 4 + wave;
  if (gtile >= g.num_maps * g.tiles_per_map) return;
  const TileRange tr = tile_range(g, gtile);
  if (tr.begin >= tr.end) return;
  uint8_t* wb = lds8 + wave * scatter2_wave_bytes<S, CH>(R);
  u32x4* buf = reinterpret_cast<u32x4*>(wb);
  uint32_t* dest = reinterpret_cast<uint32_t*>(wb + St::kBufBytes);
  uint32_t* run = dest + CH;
  const uint64_t* bm = base + (uint64_t)tr.map * R;
  const uint32_t* pm = prefix + (uint64_t)tr.map * R * g.tiles_per_map + tr.tile;
  for (int p = lane; p < R; p += kWave)
    run[p] = (uint32_t)(bm[p] + pm[(uint64_t)p * g.tiles_per_map]);
  __builtin_amdgcn_wave_barrier();
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out);
  for (uint64_t c0 = tr.begin; c0 < tr.end; c0 += CH) {
    const uint32_t nrec = (uint32_t)min<uint64_t>(CH, tr.end - c0);
    const uint32_t head = stage_units<St::kPer>(g.recs + c0 * S, nrec * S, buf, lane);
    // destinations, in input order (stable: lane order inside 64, chunk order across)
#pragma unroll
    for (uint32_t j = 0; j < CH / kWave; ++j) {
      const uint32_t r = j * kWave + lane;
      const bool valid = r < nrec;
      const uint32_t pid = valid ? pids[c0 + r] : 0u;
      uint64_t peers = __ballot(valid);
      for (int bb = 0; bb < pid_bits; ++bb) {
        const bool bit = (pid >> bb) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
      }
      uint32_t r0 = 0;
      if (valid) r0 = run[pid];
      __builtin_amdgcn_wave_barrier();
      if (valid && (peers & lt_mask) == 0) run[pid] = r0 + (uint32_t)__popcll(peers);
      if (valid) dest[r] = r0 + (uint32_t)__popcll(peers & lt_mask);
      __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // record-coalesced write-out: lane -> dword d of the chunk, in input order
    const uint32_t* bw = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(buf) + head);
    const uint32_t total = nrec * W;
#pragma unroll 4
    for (uint32_t d = lane; d < total; d += kWave) {
      const uint32_t r = d / W, w = d - r * W;
      out32[(uint64_t)dest[r] * W + w] = bw[d];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------------------------------
// v3 hist: register streaming.  Each lane loads the key dwords of RPL records straight to
// registers (all loads issued before the first use), the range table (bounds + 10-bit prefix
// LUT) lives in LDS so no dependent global load stalls the stream, and workgroups are mapped
// XCD-contiguously (T1) so neighbouring tiles share an L2.
// ------------------------------------------------------------------------------------------

// range_search_t, partition_words, KeyVec: sux_p1.h

template <int KW, int RPL, bool TAB>
__global__ __launch_bounds__(256) void k_hist3(PartDev pd, MapGroup g, uint16_t* __restrict__ pids,
                                               uint32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint64_t ldsq[];
  const int R = pd.R;
  const int nb = TAB ? 2 * (R - 1) : 0;
  uint64_t* sb = ldsq;
  uint32_t* slut = reinterpret_cast<uint32_t*>(ldsq + nb);
  uint16_t* pbuf_all = reinterpret_cast<uint16_t*>(slut + (TAB ? (1 << kLutBits) : 0));
  uint32_t* hist_all = reinterpret_cast<uint32_t*>(pbuf_all + 4 * kWave * RPL);
  if constexpr (TAB) {
    for (int i = threadIdx.x; i < nb; i += 256) sb[i] = pd.bounds[i];
    for (int i = threadIdx.x; i < (1 << kLutBits); i += 256) slut[i] = pd.lut[i];
  }
  for (int i = threadIdx.x; i < 4 * R; i += 256) hist_all[i] = 0;
  __syncthreads();
  const uint64_t* bounds = TAB ? sb : pd.bounds;
  const uint32_t* lut = TAB ? slut : pd.lut;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  uint32_t* hist = hist_all + wave * R;
  uint16_t* pbuf = pbuf_all + wave * kWave * RPL;
  const uint32_t gtile = xcd_map(blockIdx.x, gridDim.x) * 4 + wave;
  if (gtile >= g.num_maps * g.tiles_per_map) return;
  const TileRange tr = tile_range(g, gtile);
  const uint8_t* keys = g.recs + pd.key_offset;
  typedef typename KeyVec<KW>::T KV;
  for (uint64_t i0 = tr.begin; i0 < tr.end; i0 += kWave * RPL) {
    KV kv[RPL];
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      const uint64_t i = i0 + k * kWave + lane;
      kv[k] = *reinterpret_cast<const KV*>(keys + (i < tr.end ? i : tr.begin) * g.rec_size);
    }
    // whole 8-record groups of this block go out as 16-byte pid stores via LDS
    const bool packed = (tr.end - i0 >= (uint64_t)kWave * RPL) &&
                        ((reinterpret_cast<uintptr_t>(pids + i0) & 15) == 0);
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      const uint64_t i = i0 + k * kWave + lane;
      if (i < tr.end) {
        uint32_t w[KW];
        KeyVec<KW>::get(kv[k], w);
        const int p = partition_words<KW, TAB>(pd, w, bounds, lut);
        atomicAdd(&hist[p], 1u);
        if (packed) pbuf[k * kWave + lane] = (uint16_t)p;
        else pids[i] = (uint16_t)p;
      }
    }
    if (packed) {
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if (lane < kWave * RPL / 8)
        reinterpret_cast<u32x4*>(pids + i0)[lane] = reinterpret_cast<const u32x4*>(pbuf)[lane];
      __builtin_amdgcn_wave_barrier();
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint32_t* dst = counts + ((uint64_t)tr.map * R) * g.tiles_per_map + tr.tile;
  for (int p = lane; p < R; p += kWave) dst[(uint64_t)p * g.tiles_per_map] = hist[p];
}

// ------------------------------------------------------------------------------------------
// v4 hist: coalesced streaming.  v3's per-lane key loads (one 12-byte access per record, 64
// lines per wave-instruction) kept the texture addresser stalled on the L1 (PMC:
// TA_ADDR_STALLED_BY_TC ~72 % of TA busy) at ~4 TB/s.  Here every wave reads its tile as
// contiguous 16-byte units (1 KiB per wave-instruction), drops each CH-record chunk into a
// wave-private LDS stage, and reads the keys back from LDS (stride S/4 dwords: S/4 odd for
// S=100, so the 32 lanes of a ds_read_b32 hit 32 different banks).  The next chunk's loads are
// issued right after the stage is written, so they fly during the key math.
// ------------------------------------------------------------------------------------------
template <uint32_t S, uint32_t CH>
struct Hs4 {
  // a step reads CH records with CH / 64 record slots per lane: CH < 64 would read none
  static_assert(CH % kWave == 0 && CH >= kWave, "k_hist4 stages whole waves of records");
  static constexpr uint32_t kUnits = (CH * S + 12 + 15) / 16;
  static constexpr uint32_t kPer = (kUnits + kWave - 1) / kWave;
  static constexpr uint32_t kStage = kPer * kWave * 16;  // bytes per wave
  // stage[4] | bounds 2(R-1) u64 | lut | hist[4][R] u32
  static __host__ __device__ constexpr uint32_t lds_bytes(int R, bool tab) {
    return 4 * kStage + (tab ? (uint32_t)(R - 1) * 16 + (4u << kLutBits) : 0u) + 16u * R;
  }
};

template <uint32_t S, uint32_t CH, int KW, bool TAB, bool NTL>
__global__ __launch_bounds__(256) void k_hist4(PartDev pd, MapGroup g, uint16_t* __restrict__ pids,
                                               uint32_t* __restrict__ counts) {
  using H = Hs4<S, CH>;
  constexpr uint32_t PER = H::kPer;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const int R = pd.R;
  const int nb = TAB ? 2 * (R - 1) : 0;
  u32x4* stage_all = reinterpret_cast<u32x4*>(lds8);
  uint64_t* sb = reinterpret_cast<uint64_t*>(lds8 + 4 * H::kStage);
  uint32_t* slut = reinterpret_cast<uint32_t*>(sb + nb);
  uint32_t* hist_all = slut + (TAB ? (1 << kLutBits) : 0);
  if constexpr (TAB) {
    for (int i = threadIdx.x; i < nb; i += 256) sb[i] = pd.bounds[i];
    for (int i = threadIdx.x; i < (1 << kLutBits); i += 256) slut[i] = pd.lut[i];
  }
  for (int i = threadIdx.x; i < 4 * R; i += 256) hist_all[i] = 0;
  __syncthreads();
  const uint64_t* bounds = TAB ? sb : pd.bounds;
  const uint32_t* lut = TAB ? slut : pd.lut;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  uint32_t* hist = hist_all + wave * R;
  u32x4* stage = stage_all + wave * (H::kStage / 16);
  const uint32_t* st32 = reinterpret_cast<const uint32_t*>(stage);
  const uint32_t ntiles = g.num_maps * g.tiles_per_map;
  const uint32_t Q = (g.tile_recs + 3) / 4;  // records per wave per tile
  uint64_t wb = 0, we = 0;                    // this wave's range of the current tile

  auto issue = [&](uint64_t c0, u32x4 (&v)[PER]) {
    const uint32_t n = (uint32_t)min<uint64_t>(CH, we - c0);
    const uint8_t* a = g.recs + c0 * S;
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 15u);
    const u32x4* src = reinterpret_cast<const u32x4*>(a - head);
    const uint32_t units = (head + n * S + 15) >> 4;
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
      const u32x4* a4 = src + min(lane + k * kWave, units - 1);
      // NTL: the records are streamed once here (K3 reads them again long after they left L2)
      v[k] = NTL ? __builtin_nontemporal_load(a4) : *a4;
    }
  };
  // chunk c0 (held in v) -> stage -> keys -> pids + histogram; if `next` v is refilled with
  // the chunk at c0 + 2CH.  Every lane stores a pid (lanes past the chunk's end repeat the last
  // record's), so a step issues a fixed set of memory instructions.
  auto step = [&](uint64_t c0, u32x4 (&v)[PER], bool next) {
    const uint32_t n = (uint32_t)min<uint64_t>(CH, we - c0);
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(g.recs + c0 * S) & 15u);
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) stage[lane + k * kWave] = v[k];
    if (next) issue(c0 + 2 * CH, v);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (uint32_t j = 0; j < CH / kWave; ++j) {
      const uint32_t r = j * kWave + lane;
      const uint32_t rr = r < n ? r : n - 1;
      const uint32_t o = (head + rr * S + (uint32_t)pd.key_offset) >> 2;
      uint32_t w[KW];
#pragma unroll
      for (int q = 0; q < KW; ++q) w[q] = st32[o + q];
      const int p = partition_words<KW, TAB>(pd, w, bounds, lut);
      if (r < n) atomicAdd(&hist[p], 1u);
      pids[c0 + rr] = (uint16_t)p;
    }
    __builtin_amdgcn_wave_barrier();
  };

  // Persistent: the workgroup walks tiles gridDim.x apart (the table above is loaded once);
  // the 4 waves split a tile, so a tile takes a quarter of a wave's time and the launch's tail
  // is short.  Two chunks in flight per wave (register double buffer): HBM wants ~200 KB in
  // flight per CU.  The steady-state loop has no conditional memory instruction, so the
  // compiler's wait for the older buffer is a counted vmcnt that leaves the younger in flight.
  for (uint32_t gt = blockIdx.x; gt < ntiles; gt += gridDim.x) {
    const TileRange tr = tile_range(g, gt);
    wb = min(tr.begin + (uint64_t)wave * Q, tr.end);
    we = min(wb + Q, tr.end);
    u32x4 va[PER], vb[PER];
    const uint32_t nch = (uint32_t)((we - wb + CH - 1) / CH);
    if (nch >= 4) {
      issue(wb, va);
      issue(wb + CH, vb);
      uint32_t i = 0;
      for (; i + 3 < nch; i += 2) {
        step(wb + (uint64_t)i * CH, va, true);
        step(wb + (uint64_t)(i + 1) * CH, vb, true);
      }
      // tail: 2 or 3 chunks left (the third is loaded into va by the first tail step)
      step(wb + (uint64_t)i * CH, va, i + 2 < nch);
      step(wb + (uint64_t)(i + 1) * CH, vb, false);
      if (i + 2 < nch) step(wb + (uint64_t)(i + 2) * CH, va, false);
    } else if (nch > 0) {
      issue(wb, va);
      if (nch > 1) issue(wb + CH, vb);
      step(wb, va, nch > 2);
      if (nch > 1) step(wb + CH, vb, false);
      if (nch > 2) step(wb + 2 * CH, va, false);
    }
    // an empty tile (the tail of a short last map) still publishes its zero counts; tile-major
    // counts are one contiguous 4R-byte store per tile, partition-major ones R strided dwords
    __syncthreads();
    const bool tm = g.counts_tm != 0;
    uint32_t* dst = tm ? counts + ((uint64_t)tr.map * g.tiles_per_map + tr.tile) * R
                       : counts + ((uint64_t)tr.map * R) * g.tiles_per_map + tr.tile;
    const uint64_t stride = tm ? 1 : g.tiles_per_map;
    for (int p = threadIdx.x; p < R; p += 256) {
      dst[(uint64_t)p * stride] =
          hist_all[p] + hist_all[R + p] + hist_all[2 * R + p] + hist_all[3 * R + p];
      hist_all[p] = hist_all[R + p] = hist_all[2 * R + p] = hist_all[3 * R + p] = 0;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// v6 scatter: v5's destination-unit image, re-shaped for one big workgroup per CU.
//   - NW waves (NW*64 threads) and C-record chunks (C*S bytes, ~100 KB at C=1024): a partition's
//     run per chunk is ~C/R records long, so a chunk writes R runs of ~C*S/R bytes and the
//     partial 128-B lines at run ends are few and stay in L2 until the next chunk completes them
//     (one workgroup per CU keeps <= R open lines per CU).
//   - Software pipelined: the next chunk's pids and records are loaded into registers right
//     after this chunk's records were moved into the LDS image, so the loads fly while this
//     chunk's image is written out and its carries are folded.
//   - Each workgroup walks `tpw` consecutive tiles of one map (a longer range amortises the
//     per-range setup: R prefix reads and R tail flushes).
//   - Record dwords enter the image with a per-lane dword rotation ((lane>>3)&3) so that the
//     8 lanes sharing a bank row in one ds_write_b32 write 4 different banks of it.
// ------------------------------------------------------------------------------------------
// destination-unit words of the v6/v7 image: unit index (30 bits: a launch group's output
// up to 16 GiB) | foreign head dwords (0..3) << 30
constexpr uint32_t kSkipShift = 30;
constexpr uint32_t kNoUnit = 0xFFFFFFFFu;       // tail unit still partial: becomes the carry
constexpr uint32_t kUnitMask = (1u << kSkipShift) - 1;
constexpr uint64_t kImageMaxBytes = (1ull << (kSkipShift + 4)) - 64;  // kNoUnit never a real unit

// Diagnostic build only (-DSUX_STAMPS, tools/stamps.hip): thread 0 of workgroups < 64 records
// s_memtime at the phase boundaries of its first 16 chunks.  No stamp executes otherwise.
#ifdef SUX_STAMPS
__device__ uint64_t g_stamps[64][16][8];
#define SUX_STAMP(ci, ph)                                                        \
  do {                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < 64 && (ci) < 16)                        \
      g_stamps[blockIdx.x][(ci)][(ph)] = __builtin_amdgcn_s_memtime();          \
  } while (0)
#else
#define SUX_STAMP(ci, ph) \
  do {                    \
  } while (0)
#endif

template <uint32_t S, uint32_t C, uint32_t NW>
struct Sc6 {
  static constexpr uint32_t NT = NW * kWave;
  static constexpr uint32_t W = S / 4;
  static constexpr uint32_t RPW = C / NW;  // records per wave per chunk
  static constexpr uint32_t NG = (RPW + kWave - 1) / kWave;
  static constexpr uint32_t kUnits = (C * S + 12 + 15) / 16;
  static constexpr uint32_t kPer = (kUnits + NT - 1) / NT;
  static_assert(C % NW == 0 && RPW % kWave == 0, "whole 64-record groups per wave");
  static __host__ __device__ constexpr uint32_t space(int R) {
    return (C * S) / 16 + (3u * R + 1) / 2 + 1;
  }
  // img[SP] u32x4 | carry[R] u32x4 | pos[R] u64 | dstu[SP] | recoff[C] | wcnt[NW][R] | cnt[R]
  // | first[R] | lbase[R] | scan tmp[NW + 1]   (all u32 past pos)
  static __host__ __device__ constexpr uint32_t lds_bytes(int R) {
    return space(R) * 16 + (uint32_t)R * 24 + space(R) * 4 + C * 4 + NW * (uint32_t)R * 4 +
           3u * R * 4 + (NW + 1) * 4;
  }
};

// Exclusive scan of R u32 in LDS (in place) by NT threads; returns the total (all threads).
template <uint32_t NT>
__device__ __forceinline__ uint32_t block_scan_u32(uint32_t* v, int R, uint32_t* tmp) {
  constexpr uint32_t NW = NT / kWave;
  const int t = threadIdx.x, lane = t % kWave, wave = t / kWave;
  const int per = (R + NT - 1) / NT;
  const int lo = t * per, hi = min(R, lo + per);
  uint32_t s = 0;
  for (int i = lo; i < hi; ++i) s += v[i];
  const uint32_t inc = wave_incl_scan(s, lane);
  if (lane == kWave - 1) tmp[wave] = inc;
  __syncthreads();
  if (wave == 0) {
    const uint32_t x = lane < (int)NW ? tmp[lane] : 0u;
    const uint32_t xi = wave_incl_scan(x, lane);
    if (lane < (int)NW) tmp[lane] = xi - x;
    if (lane == (int)NW - 1) tmp[NW] = xi;
  }
  __syncthreads();
  uint32_t run = tmp[wave] + inc - s;
  for (int i = lo; i < hi; ++i) {
    const uint32_t x = v[i];
    v[i] = run;
    run += x;
  }
  const uint32_t total = tmp[NW];
  __syncthreads();
  return total;
}

template <uint32_t S, uint32_t C, uint32_t NW>
__global__ __launch_bounds__(NW * 64) void k_scatter6(MapGroup g, int R, int pid_bits,
                                                     const uint16_t* __restrict__ pids,
                                                     const uint32_t* __restrict__ prefix,
                                                     const uint64_t* __restrict__ base,
                                                     uint8_t* __restrict__ out, uint32_t tpw,
                                                     uint32_t wg_per_map) {
  using K = Sc6<S, C, NW>;
  constexpr uint32_t NT = K::NT, W = K::W, RPW = K::RPW, NG = K::NG, PER = K::kPer;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const uint32_t SP = K::space(R);
  u32x4* img = reinterpret_cast<u32x4*>(lds8);
  uint32_t* img32 = reinterpret_cast<uint32_t*>(lds8);
  u32x4* carry = img + SP;
  uint64_t* pos = reinterpret_cast<uint64_t*>(carry + R);
  uint32_t* dstu = reinterpret_cast<uint32_t*>(pos + R);
  uint32_t* recoff = dstu + SP;
  uint32_t* wcnt = recoff + C;
  uint32_t* cnt = wcnt + NW * R;
  uint32_t* first = cnt + R;
  uint32_t* lbase = first + R;
  uint32_t* tmp = lbase + R;

  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint32_t wg = xcd_map(blockIdx.x, gridDim.x);
  const uint32_t map = wg / wg_per_map, t0 = (wg - map * wg_per_map) * tpw;
  const uint64_t map_begin = (uint64_t)map * g.records_per_map;
  const uint64_t map_end = min(map_begin + g.records_per_map, g.num_records);
  const uint64_t begin = min(map_begin + (uint64_t)t0 * g.tile_recs, map_end);
  const uint64_t end = min(begin + (uint64_t)tpw * g.tile_recs, map_end);
  if (begin >= end) return;  // uniform for the workgroup

  const uint64_t* bm = base + (uint64_t)map * R;
  const uint32_t* pm = prefix + (uint64_t)map * R * g.tiles_per_map + t0;
  for (int p = tid; p < R; p += NT) {
    const uint64_t d = (bm[p] + pm[(uint64_t)p * g.tiles_per_map]) * S;
    pos[p] = d;
    first[p] = (uint32_t)(d & 15) >> 2;
    carry[p] = u32x4{0, 0, 0, 0};
  }
  for (int i = tid; i < (int)NW * R; i += NT) wcnt[i] = 0;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out);
  const uint32_t rot = (uint32_t)(lane >> 3) & 3u;

  // prologue: loads of chunk 0
  uint32_t pidv[NG];
  u32x4 v[PER];
  auto issue = [&](uint64_t c0) {
    const uint32_t n = (uint32_t)min<uint64_t>(C, end - c0);
#pragma unroll
    for (uint32_t j = 0; j < NG; ++j) {
      const uint32_t r = wave * RPW + j * kWave + lane;
      pidv[j] = pids[c0 + min(r, n - 1)];
    }
    const uint8_t* a = g.recs + c0 * S;
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 15u);
    const u32x4* src = reinterpret_cast<const u32x4*>(a - head);
    const uint32_t units = (head + n * S + 15) >> 4;
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) v[k] = src[min(tid + k * NT, units - 1)];
  };
  issue(begin);
  __syncthreads();

  uint32_t ci = 0;
  for (uint64_t c0 = begin; c0 < end; c0 += C, ++ci) {
    SUX_STAMP(ci, 0);
    const uint32_t n = (uint32_t)min<uint64_t>(C, end - c0);
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(g.recs + c0 * S) & 15u);
    const uint32_t units = (head + n * S + 15) >> 4;
    // 1. stable per-wave ranks (ballot match over the pid bits)
    uint32_t my_pid[NG], my_rank[NG];
    uint32_t* wc = wcnt + wave * R;
#pragma unroll
    for (uint32_t j = 0; j < NG; ++j) {
      const uint32_t r = wave * RPW + j * kWave + lane;
      const bool valid = r < n;
      const uint32_t pid = valid ? pidv[j] : 0u;
      uint64_t peers = __ballot(valid);
      for (int bb = 0; bb < pid_bits; ++bb) {
        const bool bit = (pid >> bb) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
      }
      uint32_t r0 = 0;
      if (valid) r0 = wc[pid];
      __builtin_amdgcn_wave_barrier();
      if (valid && (peers & lt_mask) == 0) wc[pid] = r0 + (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
      my_pid[j] = valid ? pid : kNoUnit;
      my_rank[j] = r0 + (uint32_t)__popcll(peers & lt_mask);
    }
    __syncthreads();
    SUX_STAMP(ci, 1);
    // 2. per partition: cross-wave prefix, count, image units (carry + run, rounded up)
    for (int p = tid; p < R; p += NT) {
      uint32_t s = 0;
#pragma unroll
      for (uint32_t w = 0; w < NW; ++w) {
        const uint32_t x = wcnt[w * R + p];
        wcnt[w * R + p] = s;
        s += x;
      }
      cnt[p] = s;
      const uint32_t cd = (uint32_t)(pos[p] & 15) >> 2;
      lbase[p] = (cd + s * W + 3) >> 2;
    }
    __syncthreads();
    const uint32_t U = block_scan_u32<NT>(lbase, R, tmp);  // ends with a barrier
    SUX_STAMP(ci, 2);
    // 3. carries in front of the runs, record image offsets, destination units
    for (int p = tid; p < R; p += NT) {
      const uint32_t c = cnt[p], cd = (uint32_t)(pos[p] & 15) >> 2, lb = lbase[p];
      const uint32_t full = (cd + c * W) >> 2, sp = (cd + c * W + 3) >> 2;
      const u32x4 cv = carry[p];
      for (uint32_t i = 0; i < cd; ++i) img32[4 * lb + i] = cv[i];
      if (sp) dstu[lb] = full ? ((uint32_t)(pos[p] >> 4) | (first[p] << kSkipShift)) : kNoUnit;
    }
#pragma unroll
    for (uint32_t j = 0; j < NG; ++j) {
      const uint32_t p = my_pid[j];
      if (p == kNoUnit) continue;
      const uint32_t jr = wcnt[wave * R + p] + my_rank[j];
      const uint32_t c = cnt[p], cd = (uint32_t)(pos[p] & 15) >> 2, lb = lbase[p];
      const uint32_t o = 4 * cd + jr * S;
      recoff[wave * RPW + j * kWave + lane] = 16 * lb + o;
      const uint32_t full = (cd + c * W) >> 2, sp = (cd + c * W + 3) >> 2;
      const uint32_t u0 = (uint32_t)(pos[p] >> 4);
      for (uint32_t k = (o + 15) >> 4; k * 16 < o + S && k < sp; ++k)
        if (k) dstu[lb + k] = k < full ? (u0 + k) : kNoUnit;
    }
    __syncthreads();
    SUX_STAMP(ci, 3);
    // 4. records -> image (dword granular, rotated per lane octet against bank conflicts)
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
      const uint32_t u = tid + k * NT;
      if (u < units) {
#pragma unroll
        for (uint32_t cc = 0; cc < 4; ++cc) {
          const uint32_t c = (cc + rot) & 3u;
          const int32_t b = (int32_t)(16 * u + 4 * c) - (int32_t)head;
          if (b >= 0 && (uint32_t)b < n * S) {
            const uint32_t r = (uint32_t)b / S, off = (uint32_t)b - r * S;
            const uint32_t x = c == 0 ? v[k][0] : c == 1 ? v[k][1] : c == 2 ? v[k][2] : v[k][3];
            img32[(recoff[r] + off) >> 2] = x;
          }
        }
      }
    }
    SUX_STAMP(ci, 4);
    // 5. the registers are free: start the next chunk's loads
    if (c0 + C < end) issue(c0 + C);
    __syncthreads();
    SUX_STAMP(ci, 5);
    // 6. writer: one aligned 16-byte store per completed destination unit
    for (uint32_t q = tid; q < U; q += NT) {
      const uint32_t d = dstu[q];
      if (d == kNoUnit) continue;
      const u32x4 x = img[q];
      const uint32_t skip = d >> kSkipShift;
      const uint64_t A = (uint64_t)(d & kUnitMask) * 16;
      if (skip == 0) {
        *reinterpret_cast<u32x4*>(out + A) = x;
      } else {
#pragma unroll
        for (uint32_t c = 0; c < 4; ++c)
          if (c >= skip) out32[(A >> 2) + c] = x[c];
      }
    }
    __syncthreads();
    SUX_STAMP(ci, 6);
    // 7. new carries and positions
    for (int p = tid; p < R; p += NT) {
      const uint32_t c = cnt[p];
      if (c == 0) continue;
      const uint32_t cd = (uint32_t)(pos[p] & 15) >> 2, lb = lbase[p];
      const uint32_t full = (cd + c * W) >> 2, rest = (cd + c * W) & 3;
      if (rest) carry[p] = img[lb + full];
      if (full) first[p] = 0;
      pos[p] += (uint64_t)c * S;
    }
    for (int i = tid; i < (int)NW * R; i += NT) wcnt[i] = 0;
    __syncthreads();
    SUX_STAMP(ci, 7);
  }
  // 8. flush the tails (the next range's workgroup writes the rest of these units)
  for (int p = tid; p < R; p += NT) {
    const uint64_t ps = pos[p];
    const uint32_t cd = (uint32_t)(ps & 15) >> 2;
    const u32x4 cv = carry[p];
    for (uint32_t c = first[p]; c < cd; ++c) out32[((ps & ~15ull) >> 2) + c] = cv[c];
  }
}

// ------------------------------------------------------------------------------------------
// v7 scatter: v6 with the per-chunk bookkeeping cut down (tools/stamps: v6 spent 57 % of a
// chunk's cycles in rank/prefix/scan/offsets/carries, none of it overlapping memory at one
// workgroup per CU).  R <= NW*64, so thread p owns partition p for the whole range and keeps
// its output cursor in registers; per-wave counters are stored partition-major (NW contiguous
// u32 = NW/4 ds_read_b128); prefix over waves and the scan of image units are one fused phase
// (wave scan + NW wave totals); records read one packed {lb, cd, full, sp} per partition; the
// destination-unit loop of a record is a fixed, predicated trip count.
// ------------------------------------------------------------------------------------------
template <uint32_t S, uint32_t C, uint32_t NW>
struct Sc7 {
  static constexpr uint32_t NT = NW * kWave;
  static constexpr uint32_t W = S / 4;
  static constexpr uint32_t RPW = C / NW;
  static constexpr uint32_t NG = (RPW + kWave - 1) / kWave;
  static constexpr uint32_t kUnits = (C * S + 12 + 15) / 16;
  static constexpr uint32_t kPer = (kUnits + NT - 1) / NT;
  static constexpr uint32_t kRecUnits = (S + 15) / 16 + 1;  // units that can start in a record
  static_assert(C % NW == 0 && RPW % kWave == 0 && NW % 4 == 0, "shape");
  static __host__ __device__ constexpr uint32_t space(int R) {
    return (C * S) / 16 + (3u * R + 1) / 2 + 1;
  }
  // img[SP] u32x4 | pinfo[R] u32x4 | carry[R] u32x4 | dstu[SP] | recoff[C] | wcnt[R][NW]
  // | u0[R] | tmp[NW + 1]
  static __host__ __device__ constexpr uint32_t lds_bytes(int R) {
    return space(R) * 16 + (uint32_t)R * 32 + space(R) * 4 + C * 4 + NW * (uint32_t)R * 4 +
           (uint32_t)R * 4 + (NW + 1) * 4;
  }
};

template <uint32_t S, uint32_t C, uint32_t NW, uint32_t DEPTH>
__global__ __launch_bounds__(NW * 64) void k_scatter7(MapGroup g, int R, int pid_bits,
                                                     const uint16_t* __restrict__ pids,
                                                     const uint32_t* __restrict__ prefix,
                                                     const uint64_t* __restrict__ base,
                                                     uint8_t* __restrict__ out, uint32_t tpw,
                                                     uint32_t wg_per_map) {
  using K = Sc7<S, C, NW>;
  constexpr uint32_t NT = K::NT, W = K::W, RPW = K::RPW, NG = K::NG, PER = K::kPer;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const uint32_t SP = K::space(R);
  u32x4* img = reinterpret_cast<u32x4*>(lds8);
  uint32_t* img32 = reinterpret_cast<uint32_t*>(lds8);
  u32x4* pinfo = img + SP;   // {lb, cd, full, sp}
  u32x4* carry = pinfo + R;  // pending tail dwords of p
  uint32_t* dstu = reinterpret_cast<uint32_t*>(carry + R);
  uint32_t* recoff = dstu + SP;
  uint32_t* wcnt = recoff + C;  // [R][NW]
  uint32_t* u0s = wcnt + NW * R;
  uint32_t* tmp = u0s + R;

  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const bool owner = tid < R;  // thread p owns partition p: cursor and head state in registers
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out);
  const uint32_t rot = (uint32_t)(lane >> 3) & 3u;

  // Persistent: workgroup b walks work items slot(b), slot(b) + G, ... where an item is `tpw`
  // tiles of one map and slot() keeps the items an XCD works on at one time adjacent.  The chunk
  // stream runs across item seams: the first chunk of the next item is loaded while the last
  // chunk of this one is written out.
  const uint32_t nitems = g.num_maps * wg_per_map;
  const uint32_t G = gridDim.x;
  struct Item {
    uint32_t map, t0;
    uint64_t begin, end;
  };
  auto item_of = [&](uint32_t it) {
    Item x;
    x.map = it / wg_per_map;
    x.t0 = (it - x.map * wg_per_map) * tpw;
    const uint64_t map_begin = (uint64_t)x.map * g.records_per_map;
    const uint64_t map_end = min(map_begin + g.records_per_map, g.num_records);
    x.begin = min(map_begin + (uint64_t)x.t0 * g.tile_recs, map_end);
    x.end = min(x.begin + (uint64_t)tpw * g.tile_recs, map_end);
    return x;
  };
  const uint32_t it = xcd_map(blockIdx.x, G);
  if (it >= nitems) return;
  const Item cur = item_of(it);

  uint64_t pos = 0;
  uint32_t first = 0;
  auto begin_item = [&](const Item& x) {
    if (owner) {
      pos = (base[(uint64_t)x.map * R + tid] +
             prefix[g.counts_tm ? ((uint64_t)x.map * g.tiles_per_map + x.t0) * R + tid
                                : (uint64_t)x.map * R * g.tiles_per_map + (uint64_t)tid * g.tiles_per_map + x.t0]) * S;
      first = (uint32_t)(pos & 15) >> 2;
      carry[tid] = u32x4{0, 0, 0, 0};
    }
  };
  // the tails of this item's runs: the next range's workgroup writes the rest of these units
  auto end_item = [&]() {
    if (owner) {
      const uint32_t cd = (uint32_t)(pos & 15) >> 2;
      const u32x4 cv = carry[tid];
      for (uint32_t cc = first; cc < cd; ++cc) out32[((pos & ~15ull) >> 2) + cc] = cv[cc];
    }
  };

  // Chunk stream: a cursor walks (item, chunk) pairs; `issue` always emits the same loads
  // (a finished stream loads one unit of the input again) so that the compiler's waits for the
  // older of two register buffers are counted and leave the younger one in flight.
  struct Cur {
    uint32_t it;
    uint64_t c0, end;
    bool valid;
  };
  auto first_cur = [&](uint32_t it0) {
    Cur k;
    k.it = it0;
    k.valid = it0 < nitems;
    const Item x = item_of(k.valid ? it0 : 0);
    k.c0 = x.begin;
    k.end = x.end;
    return k;
  };
  auto next_cur = [&](const Cur& k) {
    Cur nk = k;
    nk.c0 = k.c0 + C;
    if (nk.c0 >= k.end) nk = first_cur(k.it + G);
    return nk;
  };
  auto issue = [&](const Cur& k, uint32_t (&pidv)[NG], u32x4 (&v)[PER]) {
    const uint32_t n = k.valid ? (uint32_t)min<uint64_t>(C, k.end - k.c0) : 1u;
    const uint64_t c0 = k.valid ? k.c0 : 0;
#pragma unroll
    for (uint32_t j = 0; j < NG; ++j) {
      const uint32_t r = wave * RPW + j * kWave + lane;
      pidv[j] = pids[c0 + min(r, n - 1)];
    }
    const uint8_t* a = g.recs + c0 * S;
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 15u);
    const u32x4* src = reinterpret_cast<const u32x4*>(a - head);
    const uint32_t units = (head + n * S + 15) >> 4;
#pragma unroll
    for (uint32_t k2 = 0; k2 < PER; ++k2) v[k2] = src[min(tid + k2 * NT, units - 1)];
  };

  if (owner) {
#pragma unroll
    for (uint32_t w = 0; w < NW; w += 4)
      reinterpret_cast<u32x4*>(wcnt + tid * NW)[w / 4] = u32x4{0, 0, 0, 0};
  }
  begin_item(cur);
  [[maybe_unused]] uint32_t ci = 0;  // chunk counter for the diagnostic stamps
  // one chunk: pids and records in (pidv, v); `ahead` is the chunk DEPTH positions later, loaded
  // into the same registers once they are free.  Returns false after the stream's last chunk.
  auto process = [&](const Cur& k, const Cur& ahead, uint32_t (&pidv)[NG], u32x4 (&v)[PER]) {
    SUX_STAMP(ci, 0);
    const uint64_t c0 = k.c0;
    const uint32_t n = (uint32_t)min<uint64_t>(C, k.end - c0);
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(g.recs + c0 * S) & 15u);
    const uint32_t units = (head + n * S + 15) >> 4;
    const Cur nk = next_cur(k);
    const bool seam = nk.it != k.it, more = nk.valid;
    // 1. stable per-wave ranks (ballot match over the pid bits)
    uint32_t my_pid[NG], my_rank[NG];
#pragma unroll
    for (uint32_t j = 0; j < NG; ++j) {
      const uint32_t r = wave * RPW + j * kWave + lane;
      const bool valid = r < n;
      const uint32_t pid = valid ? pidv[j] : 0u;
      uint64_t peers = __ballot(valid);
      for (int bb = 0; bb < pid_bits; ++bb) {
        const bool bit = (pid >> bb) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
      }
      uint32_t* wc = wcnt + pid * NW + wave;
      uint32_t r0 = 0;
      if (valid) r0 = *wc;
      __builtin_amdgcn_wave_barrier();
      if (valid && (peers & lt_mask) == 0) *wc = r0 + (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
      my_pid[j] = valid ? pid : kNoUnit;
      my_rank[j] = r0 + (uint32_t)__popcll(peers & lt_mask);
    }
    __syncthreads();
    SUX_STAMP(ci, 1);
    // 2. fused: prefix over waves (registers), count, image units, scan of units over R
    uint32_t c = 0, cd = 0, sp = 0, full = 0;
    if (owner) {
      u32x4* row = reinterpret_cast<u32x4*>(wcnt + tid * NW);
      u32x4 x[NW / 4];
#pragma unroll
      for (uint32_t q = 0; q < NW / 4; ++q) x[q] = row[q];
#pragma unroll
      for (uint32_t q = 0; q < NW / 4; ++q) {
        u32x4 y;
        y[0] = c;
        y[1] = c + x[q][0];
        y[2] = y[1] + x[q][1];
        y[3] = y[2] + x[q][2];
        c = y[3] + x[q][3];
        row[q] = y;
      }
      cd = (uint32_t)(pos & 15) >> 2;
      full = (cd + c * W) >> 2;
      sp = (cd + c * W + 3) >> 2;
    }
    const uint32_t incl = wave_incl_scan(sp, lane);
    if (lane == kWave - 1) tmp[wave] = incl;
    __syncthreads();
    SUX_STAMP(ci, 2);
    uint32_t lb = incl - sp, U = 0;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) {
      const uint32_t t = tmp[w];
      lb += (w < (uint32_t)wave) ? t : 0u;
      U += t;
    }
    if (owner) {
      pinfo[tid] = u32x4{lb, cd, full, sp};
      u0s[tid] = (uint32_t)(pos >> 4);
      const u32x4 cv = carry[tid];
#pragma unroll
      for (uint32_t i = 0; i < 3; ++i)
        if (i < cd) img32[4 * lb + i] = cv[i];
      if (sp) dstu[lb] = full ? ((uint32_t)(pos >> 4) | (first << kSkipShift)) : kNoUnit;
    }
    __syncthreads();
    SUX_STAMP(ci, 3);
    // 3. record image offsets and the destination units that start inside each record
#pragma unroll
    for (uint32_t j = 0; j < NG; ++j) {
      const uint32_t p = my_pid[j];
      if (p == kNoUnit) continue;
      const u32x4 pi = pinfo[p];
      const uint32_t jr = wcnt[p * NW + wave] + my_rank[j];
      const uint32_t o = 4 * pi[1] + jr * S;
      recoff[wave * RPW + j * kWave + lane] = 16 * pi[0] + o;
      const uint32_t u0 = u0s[p];
      const uint32_t k0 = (o + 15) >> 4;
#pragma unroll
      for (uint32_t t = 0; t < K::kRecUnits; ++t) {
        const uint32_t k = k0 + t;
        if (k > 0 && k * 16 < o + S && k < pi[3]) dstu[pi[0] + k] = k < pi[2] ? (u0 + k) : kNoUnit;
      }
    }
    __syncthreads();
    SUX_STAMP(ci, 4);
    // 4. records -> image.  A staged unit whose 16 bytes lie inside one record goes in as ONE
    //    4-byte-aligned ds_write_b128 (the record's image offset is only 4-byte aligned); a unit
    //    that straddles two records goes dword by dword, rotated per lane octet against bank
    //    conflicts.
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
      const uint32_t u = tid + k * NT;
      const int32_t b0 = (int32_t)(16 * u) - (int32_t)head;
      const uint32_t r0 = b0 >= 0 ? (uint32_t)b0 / S : 0u, off0 = (uint32_t)b0 - r0 * S;
      if (u < units && b0 >= 0 && (uint32_t)b0 + 16 <= n * S && off0 + 16 <= S) {
        *reinterpret_cast<u32x4a4*>(img32 + ((recoff[r0] + off0) >> 2)) = v[k];
      } else if (u < units) {
#pragma unroll
        for (uint32_t cc = 0; cc < 4; ++cc) {
          const uint32_t q = (cc + rot) & 3u;
          const int32_t b = (int32_t)(16 * u + 4 * q) - (int32_t)head;
          if (b >= 0 && (uint32_t)b < n * S) {
            const uint32_t r = (uint32_t)b / S, off = (uint32_t)b - r * S;
            const uint32_t x = q == 0 ? v[k][0] : q == 1 ? v[k][1] : q == 2 ? v[k][2] : v[k][3];
            img32[(recoff[r] + off) >> 2] = x;
          }
        }
      }
    }
    // 5. the registers are free: start the loads of the chunk DEPTH ahead
    issue(ahead, pidv, v);
    __syncthreads();
    SUX_STAMP(ci, 5);
    // 6. writer: one aligned 16-byte store per completed destination unit
    for (uint32_t q = tid; q < U; q += NT) {
      const uint32_t d = dstu[q];
      if (d == kNoUnit) continue;
      const u32x4 x = img[q];
      const uint32_t skip = d >> kSkipShift;
      const uint64_t A = (uint64_t)(d & kUnitMask) * 16;
      if (skip == 0) {
        *reinterpret_cast<u32x4*>(out + A) = x;
      } else {
#pragma unroll
        for (uint32_t cc = 0; cc < 4; ++cc)
          if (cc >= skip) out32[(A >> 2) + cc] = x[cc];
      }
    }
    __syncthreads();
    SUX_STAMP(ci, 6);
    // 7. new carries and cursors (owner threads), counters cleared for the next chunk; at an
    //    item seam the tails are flushed and the next item's cursors loaded (owner-local state)
    if (owner) {
      if (c) {
        if ((cd + c * W) & 3) carry[tid] = img[lb + full];
        if (full) first = 0;
        pos += (uint64_t)c * S;
      }
#pragma unroll
      for (uint32_t w = 0; w < NW; w += 4)
        reinterpret_cast<u32x4*>(wcnt + tid * NW)[w / 4] = u32x4{0, 0, 0, 0};
    }
    if (seam) {
      end_item();
      if (more) begin_item(item_of(nk.it));
    }
    __syncthreads();
    SUX_STAMP(ci, 7);
    ++ci;
    return more;
  };

  uint32_t pa[NG];
  u32x4 va[PER];
  Cur k = first_cur(it);
  if constexpr (DEPTH == 1) {
    issue(k, pa, va);
    __syncthreads();
    while (true) {
      const Cur k1 = next_cur(k);
      if (!process(k, k1, pa, va)) break;
      k = k1;
    }
  } else {
    uint32_t pb[NG];
    u32x4 vb[PER];
    Cur k1 = next_cur(k);
    issue(k, pa, va);
    issue(k1, pb, vb);
    __syncthreads();
    while (true) {
      const Cur k2 = next_cur(k1);
      if (!process(k, k2, pa, va)) break;
      const Cur k3 = next_cur(k2);
      if (!process(k1, k3, pb, vb)) break;
      k = k2;
      k1 = k3;
    }
  }
}

// ------------------------------------------------------------------------------------------
// v8 scatter: v7 writing whole 128-byte lines.  v7 writes every completed 16-byte unit, so each
// partition run of a chunk (~5 records at R = 200) starts and ends inside a line — the copy
// pattern measured at 3.7 TB/s against 5.2+ for line-aligned runs (round-1 hbm_probe).  Here a
// partition's region in the chunk image starts at the LINE that holds its cursor: the line's
// earlier dwords (this workgroup's from the previous chunk, or another range's at an item start)
// come first, the writer stores only the region's complete lines, and the rest of the last line
// is carried to the next chunk in the registers of four "carry" threads per partition (2 units
// each) instead of LDS.  A line holding another range's dwords (item start) is stored dword by
// dword without them; an item's last partial line is flushed dword by dword.  The per-record
// loop that tagged destination units (v7 phase 3) becomes one partition byte per image unit.
// R <= 215 at C = 1024 (LDS) and 4R <= NT (carry threads).
// ------------------------------------------------------------------------------------------
template <uint32_t S, uint32_t C, uint32_t NW, uint32_t RMAX = 208>
struct Sc8 {
  static constexpr uint32_t NT = NW * kWave;
  static constexpr uint32_t W = S / 4;
  static constexpr uint32_t RPW = C / NW;
  static constexpr uint32_t NG = (RPW + kWave - 1) / kWave;
  static constexpr uint32_t kUnits = (C * S + 12 + 15) / 16;
  static constexpr uint32_t kPer = (kUnits + NT - 1) / NT;
  static_assert(C % NW == 0 && RPW % kWave == 0 && NW % 4 == 0 && S % 4 == 0, "shape");
  // a region: <= 31 dwords of the cursor's line + W*c dwords, in units
  static __host__ __device__ constexpr uint32_t space(int R) {
    return (C * S) / 16 + (17u * R + 1) / 2 + 1;
  }
  // pinfo[RMAX] u32x4 | recoff[C] | wcnt[NW][RMAX] | lunit[RMAX] | fhead[RMAX] | lpos[RMAX]
  // | tmp[NW + 1] (16-B padded) | img[SP] u32x4 | upid[SP] u8.  Every per-partition table sits at a
  // compile-time offset sized for RMAX partitions: with R-dependent offsets each thread kept one
  // VGPR of LDS address per table (and per wave row of wcnt) across the chunk loop, the kernel
  // ran out of its 128 VGPRs and spilled to scratch — and every scratch reload is a vmcnt(0)
  // that also waits for the next chunk's in-flight loads and the line stores
  static constexpr uint32_t kPinfo = 0;
  static constexpr uint32_t kRecoff = kPinfo + RMAX * 16;
  static constexpr uint32_t kWcnt = kRecoff + C * 4;
  static constexpr uint32_t kLunit = kWcnt + NW * RMAX * 4;
  static constexpr uint32_t kFhead = kLunit + RMAX * 4;
  static constexpr uint32_t kLpos = kFhead + RMAX * 4;
  static constexpr uint32_t kTmp = kLpos + RMAX * 4;
  static constexpr uint32_t kImg = (kTmp + (NW + 1) * 4 + 15) / 16 * 16;
  static __host__ __device__ constexpr uint32_t lds_bytes(int R) {
    return kImg + space(R) * 16 + space(R);
  }
  static __host__ __device__ constexpr bool fits(int R) {
    return R >= 1 && (uint32_t)R <= RMAX && 4u * (uint32_t)R <= NT && lds_bytes(R) <= 160u * 1024;
  }
};

template <uint32_t S, uint32_t C, uint32_t NW, bool WM>
__global__ __launch_bounds__(NW * 64) void k_scatter8(MapGroup g, int R, int pid_bits,
                                                     const uint16_t* __restrict__ pids,
                                                     const uint32_t* __restrict__ prefix,
                                                     const uint64_t* __restrict__ base,
                                                     uint8_t* __restrict__ out, uint32_t cyc,
                                                     uint32_t tw0, uint32_t tw1) {
  using K = Sc8<S, C, NW>;
  constexpr uint32_t NT = K::NT, W = K::W, RPW = K::RPW, NG = K::NG, PER = K::kPer;
  constexpr uint32_t RM = 208;  // K's RMAX: the tables' compile-time stride
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const uint32_t SP = K::space(R);
  u32x4* img = reinterpret_cast<u32x4*>(lds8 + K::kImg);
  uint32_t* img32 = reinterpret_cast<uint32_t*>(lds8 + K::kImg);
  u32x4* pinfo = reinterpret_cast<u32x4*>(lds8 + K::kPinfo);  // {lb, cd, full lines, sp}
  uint32_t* recoff = reinterpret_cast<uint32_t*>(lds8 + K::kRecoff);
  // per-wave counters, wave-major [NW][RM]: a wave's lanes touch different words of one row
  // (partition-major [R][NW] put every pid of a wave on 64 / NW banks: 41 % of the LDS cycles
  // were bank conflicts, profiles/pmc_r02.json)
  uint32_t* wcnt = reinterpret_cast<uint32_t*>(lds8 + K::kWcnt);
  // counter of (partition p, wave w): wave-major (WM) or round 2's partition-major [R][NW]
  auto WC = [&](uint32_t p, uint32_t w) -> uint32_t& { return WM ? wcnt[w * RM + p] : wcnt[p * NW + w]; };
  uint32_t* lunit = reinterpret_cast<uint32_t*>(lds8 + K::kLunit);  // unit of the cursor's line
  uint32_t* fhead = reinterpret_cast<uint32_t*>(lds8 + K::kFhead);  // its dwords of another range
  uint32_t* lpos = reinterpret_cast<uint32_t*>(lds8 + K::kLpos);    // cursor in dwords (item end)
  uint32_t* tmp = reinterpret_cast<uint32_t*>(lds8 + K::kTmp);
  uint8_t* upid = lds8 + K::kImg + (size_t)SP * 16;

  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const bool owner = tid < R;
  const uint32_t cp = (uint32_t)tid >> 2, cj = (uint32_t)tid & 3u;  // carry thread: (p, quarter)
  const bool carrier = cp < (uint32_t)R;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out);
  u32x4* out4 = reinterpret_cast<u32x4*>(out);
  const uint32_t rot = (uint32_t)(lane >> 3) & 3u;

  // Workgroup b walks ONE contiguous range of the launch's tiles, [T r / G, T (r+1) / G) with
  // r = xcd_map(b) (an XCD's workgroups get neighbouring ranges): balanced to one tile whatever
  // the grid (a CU-masked stream's 224 CUs as well as 256), cut into items at map boundaries.
  // cyc > 0 (block-cyclic): the tiles of the `cyc` workgroups sharing an XCD are cut into
  // 16 * cyc near-equal blocks dealt round robin, so at any time they write close to each other
  // (a launch of one huge map otherwise spreads an XCD's writes over its whole span).
  const uint32_t T = g.num_maps * g.tiles_per_map, G = gridDim.x;
  const uint32_t rr = xcd_map(blockIdx.x, G);
  constexpr uint32_t kBlocks = 16;
  uint32_t blk = 0, nblk = 1, gstride = 1, span_lo = 0, span_n = 0;
  uint32_t t_lo, t_hi;
  auto block_range = [&](uint32_t j, uint32_t& lo, uint32_t& hi) {
    const uint32_t k = blk + j * gstride;
    lo = span_lo + (uint32_t)((uint64_t)span_n * k / (nblk));
    hi = span_lo + (uint32_t)((uint64_t)span_n * (k + 1) / (nblk));
  };
  if (cyc == 0) {  // the launch's tile window [tw0, tw1) (the whole group unless windowed)
    const uint32_t TW = tw1 - tw0;
    t_lo = tw0 + (uint32_t)((uint64_t)TW * rr / G);
    t_hi = tw0 + (uint32_t)((uint64_t)TW * (rr + 1) / G);
  } else {
    const uint32_t grp = rr / cyc, members = min(cyc, G - grp * cyc);
    span_lo = (uint32_t)((uint64_t)T * (grp * cyc) / G);
    span_n = (uint32_t)((uint64_t)T * (grp * cyc + members) / G) - span_lo;
    nblk = kBlocks * members;
    gstride = members;
    blk = rr - grp * cyc;
    block_range(0, t_lo, t_hi);
  }
  if (t_lo >= t_hi && cyc == 0) return;
  struct Item {
    uint32_t map, t0;
    uint64_t begin, end;
  };
  auto item_of = [&](uint32_t t, uint32_t hi) {  // the item starting at tile t of a range ending at hi
    Item x;
    x.map = t / g.tiles_per_map;
    x.t0 = t - x.map * g.tiles_per_map;
    const uint32_t t_end = min(hi, (x.map + 1) * g.tiles_per_map);
    const uint64_t map_begin = (uint64_t)x.map * g.records_per_map;
    const uint64_t map_end = min(map_begin + g.records_per_map, g.num_records);
    x.begin = min(map_begin + (uint64_t)x.t0 * g.tile_recs, map_end);
    x.end = min(map_begin + (uint64_t)(t_end - x.map * g.tiles_per_map) * g.tile_recs, map_end);
    return x;
  };

  uint64_t pos = 0;  // owner: p's output cursor (bytes)
  auto begin_item = [&](const Item& x) {
    if (owner) {
      pos = (base[(uint64_t)x.map * R + tid] +
             prefix[g.counts_tm ? ((uint64_t)x.map * g.tiles_per_map + x.t0) * R + tid
                                : (uint64_t)x.map * R * g.tiles_per_map + (uint64_t)tid * g.tiles_per_map + x.t0]) * S;
      fhead[tid] = (uint32_t)(pos & 127) >> 2;  // the line's earlier dwords: another range's
    }
  };
  struct Cur {
    uint32_t it;  // global tile the chunk's item starts at
    uint32_t bj, hi;  // the range (block) it belongs to and that range's end
    uint64_t c0, end;
    bool valid;
  };
  auto first_cur = [&](uint32_t t, uint32_t bj, uint32_t hi) {
    Cur k;
    k.it = t;
    k.bj = bj;
    k.hi = hi;
    k.valid = t < hi;
    const Item x = item_of(k.valid ? t : t_lo, k.valid ? hi : t_hi);
    k.c0 = x.begin;
    k.end = x.end;
    return k;
  };
  auto next_cur = [&](const Cur& k) {  // pure: called ahead (prefetch) and again (seams)
    Cur nk = k;
    nk.c0 = k.c0 + C;
    if (nk.c0 >= k.end) {  // the item ends at its map's end or at the range's end
      const uint32_t m = k.it / g.tiles_per_map;
      const uint32_t nt = min(k.hi, (m + 1) * g.tiles_per_map);
      if (nt < k.hi || cyc == 0) {
        nk = first_cur(nt, k.bj, k.hi);
      } else {  // block-cyclic: the next non-empty block of this workgroup, if any
        uint32_t lo = k.hi, hi = k.hi, b = k.bj;
        while (b + 1 < kBlocks) {
          ++b;
          block_range(b, lo, hi);
          if (lo < hi) break;
        }
        nk = lo < hi ? first_cur(lo, b, hi) : first_cur(k.hi, k.bj, k.hi);  // else: invalid, ends
      }
    }
    return nk;
  };
  auto issue = [&](const Cur& k, uint32_t (&pidv)[NG], u32x4 (&v)[PER]) {
    const uint32_t n = k.valid && k.end > k.c0 ? (uint32_t)min<uint64_t>(C, k.end - k.c0) : 1u;
    const uint64_t c0 = k.valid && k.end > k.c0 ? k.c0 : 0;
#pragma unroll
    for (uint32_t j = 0; j < NG; ++j) {
      const uint32_t r = wave * RPW + j * kWave + lane;
      pidv[j] = pids[c0 + min(r, n - 1)];
    }
    const uint8_t* a = g.recs + c0 * S;
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 15u);
    const u32x4* src = reinterpret_cast<const u32x4*>(a - head);
    const uint32_t units = (head + n * S + 15) >> 4;
#pragma unroll
    for (uint32_t k2 = 0; k2 < PER; ++k2) v[k2] = src[min(tid + k2 * NT, units - 1)];
  };

  if (owner) {
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) WC(tid, w) = 0;
  }
  u32x4 cu0{0, 0, 0, 0}, cu1{0, 0, 0, 0};  // carrier: units 2cj, 2cj+1 of p's carried line
  // (block-cyclic) the first non-empty block
  uint32_t b0 = 0;
  if (cyc) {
    while (t_lo >= t_hi && b0 + 1 < kBlocks) block_range(++b0, t_lo, t_hi);
    if (t_lo >= t_hi) return;
  }
  begin_item(item_of(t_lo, t_hi));
  __syncthreads();
  [[maybe_unused]] uint32_t ci = 0;  // chunk counter for the diagnostic stamps
  auto process = [&](const Cur& k, const Cur& ahead, uint32_t (&pidv)[NG], u32x4 (&v)[PER]) {
    SUX_STAMP(ci, 0);
    const uint64_t c0 = k.c0;
    const uint32_t n = (uint32_t)min<uint64_t>(C, k.end - c0);
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(g.recs + c0 * S) & 15u);
    const uint32_t units = (head + n * S + 15) >> 4;
    const Cur nk = next_cur(k);
    const bool seam = nk.it != k.it, more = nk.valid;
    // 1. stable per-wave ranks (ballot match over the pid bits)
    uint32_t my_pid[NG], my_rank[NG];
#pragma unroll
    for (uint32_t j = 0; j < NG; ++j) {
      const uint32_t r = wave * RPW + j * kWave + lane;
      const bool valid = r < n;
      const uint32_t pid = valid ? pidv[j] : 0u;
      uint64_t peers = __ballot(valid);
      for (int bb = 0; bb < pid_bits; ++bb) {
        const bool bit = (pid >> bb) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
      }
      uint32_t* wc = &WC(pid, wave);
      uint32_t r0 = 0;
      if (valid) r0 = *wc;
      __builtin_amdgcn_wave_barrier();
      if (valid && (peers & lt_mask) == 0) *wc = r0 + (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
      my_pid[j] = valid ? pid : 0xFFFFFFFFu;
      my_rank[j] = r0 + (uint32_t)__popcll(peers & lt_mask);
    }
    __syncthreads();
    SUX_STAMP(ci, 1);
    // 2. owners: prefix over waves, region = the cursor's line from its start + c records
    uint32_t c = 0, full = 0, sp = 0;
    if (owner) {
      uint32_t x[NW];
#pragma unroll
      for (uint32_t w = 0; w < NW; ++w) x[w] = WC(tid, w);
#pragma unroll
      for (uint32_t w = 0; w < NW; ++w) {
        WC(tid, w) = c;
        c += x[w];
      }
      const uint32_t cd = (uint32_t)(pos & 127) >> 2;
      const uint32_t tot = cd + c * W;
      full = tot >> 5;
      sp = (tot + 3) >> 2;
    }
    const uint32_t incl = wave_incl_scan(sp, lane);
    if (lane == kWave - 1) tmp[wave] = incl;
    __syncthreads();
    SUX_STAMP(ci, 2);
    uint32_t lb = incl - sp, U = 0;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) {
      const uint32_t t = tmp[w];
      lb += (w < (uint32_t)wave) ? t : 0u;
      U += t;
    }
    if (owner) {
      pinfo[tid] = u32x4{lb, (uint32_t)(pos & 127) >> 2, full, sp};
      lunit[tid] = (uint32_t)(pos >> 4) & ~7u;
    }
    __syncthreads();
    SUX_STAMP(ci, 3);
    // 3. carried units into the region heads, record offsets, and the partition byte of every
    //    image unit — written by whoever holds the unit's first dword (a carrier for the
    //    carried head, else the record it starts in), so a hot partition's thousands of units
    //    are tagged by its records, not by its four carriers
    if (carrier) {
      const u32x4 pi = pinfo[cp];
      const uint32_t cdu = (pi[1] + 3) >> 2;  // units starting in carried dwords
      if (2 * cj < cdu) {
        img[pi[0] + 2 * cj] = cu0;
        upid[pi[0] + 2 * cj] = (uint8_t)cp;
      }
      if (2 * cj + 1 < cdu) {
        img[pi[0] + 2 * cj + 1] = cu1;
        upid[pi[0] + 2 * cj + 1] = (uint8_t)cp;
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < NG; ++j) {
      const uint32_t p = my_pid[j];
      if (p == 0xFFFFFFFFu) continue;
      const u32x4 pi = pinfo[p];
      const uint32_t jr = WC(p, wave) + my_rank[j];
      recoff[wave * RPW + j * kWave + lane] = 16 * pi[0] + 4 * pi[1] + jr * S;
      const uint32_t d0 = pi[1] + jr * W;  // the record's first dword in the region
      const uint32_t k0 = (d0 + 3) >> 2, k1 = (d0 + W + 3) >> 2;
#pragma unroll
      for (uint32_t t = 0; t < (W + 3) / 4 + 1; ++t)
        if (k0 + t < k1) upid[pi[0] + k0 + t] = (uint8_t)p;
    }
    __syncthreads();
    SUX_STAMP(ci, 4);
    // 4. records -> image (as v7: whole 16-byte units inside a record as one ds_write_b128)
#pragma unroll
    for (uint32_t k2 = 0; k2 < PER; ++k2) {
      const uint32_t u = tid + k2 * NT;
      const int32_t b0 = (int32_t)(16 * u) - (int32_t)head;
      const uint32_t r0 = b0 >= 0 ? (uint32_t)b0 / S : 0u, off0 = (uint32_t)b0 - r0 * S;
      if (u < units && b0 >= 0 && (uint32_t)b0 + 16 <= n * S && off0 + 16 <= S) {
        *reinterpret_cast<u32x4a4*>(img32 + ((recoff[r0] + off0) >> 2)) = v[k2];
      } else if (u < units) {
#pragma unroll
        for (uint32_t cc = 0; cc < 4; ++cc) {
          const uint32_t q = (cc + rot) & 3u;
          const int32_t b = (int32_t)(16 * u + 4 * q) - (int32_t)head;
          if (b >= 0 && (uint32_t)b < n * S) {
            const uint32_t r = (uint32_t)b / S, off = (uint32_t)b - r * S;
            const uint32_t x = q == 0 ? v[k2][0] : q == 1 ? v[k2][1] : q == 2 ? v[k2][2] : v[k2][3];
            img32[(recoff[r] + off) >> 2] = x;
          }
        }
      }
    }
    // 5. the registers are free: start the loads of the next chunk
    issue(ahead, pidv, v);
    __syncthreads();
    SUX_STAMP(ci, 5);
    // 6. writer: the complete lines of every region, line-aligned 16-byte stores; the dwords of
    //    another range at the head of an item's first line are skipped
    for (uint32_t q = tid; q < U; q += NT) {
      const uint32_t p = upid[q];
      const u32x4 pi = pinfo[p];
      const uint32_t kq = q - pi[0];
      if (kq >= 8 * pi[2]) continue;
      const uint64_t A = (uint64_t)lunit[p] + kq;
      const u32x4 x = img[q];
      const uint32_t f = kq < 8 ? fhead[p] : 0u;
      if (f <= 4 * kq) {
        out4[A] = x;
      } else if (f < 4 * kq + 4) {
#pragma unroll
        for (uint32_t cc = 0; cc < 4; ++cc)
          if (4 * kq + cc >= f) out32[4 * A + cc] = x[cc];
      }
    }
    __syncthreads();
    SUX_STAMP(ci, 6);
    // 7. carries into the carrier registers, cursors advance; an item's last line is flushed
    if (carrier) {
      const u32x4 pi = pinfo[cp];
      const uint32_t b = pi[0] + 8 * pi[2] + 2 * cj;
      if (2 * cj < pi[3] - 8 * pi[2]) cu0 = img[b];
      if (2 * cj + 1 < pi[3] - 8 * pi[2]) cu1 = img[b + 1];
    }
    if (owner) {
      if (full) fhead[tid] = 0;
      pos += (uint64_t)c * S;
      lpos[tid] = (uint32_t)(pos >> 2);
#pragma unroll
      for (uint32_t w = 0; w < NW; ++w) WC(tid, w) = 0;
    }
    if (seam) {
      __syncthreads();
      if (carrier) {  // dwords [fhead, cursor) of the cursor's line: this range's, not yet stored
        const uint32_t dp = lpos[cp], cdn = dp & 31u, f = fhead[cp];
        const uint64_t L = ((uint64_t)dp & ~31ull);
#pragma unroll
        for (uint32_t cc = 0; cc < 8; ++cc) {
          const uint32_t d = 8 * cj + cc;
          const uint32_t x = cc < 4 ? cu0[cc] : cu1[cc - 4];
          if (d >= f && d < cdn) out32[L + d] = x;
        }
      }
      __syncthreads();
      if (more) begin_item(item_of(nk.it, nk.hi));
    }
    __syncthreads();
    SUX_STAMP(ci, 7);
    ++ci;
    return more;
  };

  uint32_t pa[NG];
  u32x4 va[PER];
  Cur k = first_cur(t_lo, b0, t_hi);
  issue(k, pa, va);
  while (true) {
    const Cur k1 = next_cur(k);
    if (!process(k, k1, pa, va)) break;
    k = k1;
  }
}

// ------------------------------------------------------------------------------------------
// Small records (S = 16, SURVEY.md config C5: 16-byte key/value rows, 10,000 partitions).
// A record is one aligned 16-byte unit and R is far too large for per-wave counters, so:
//   k_hist16   persistent workgroups of 1024 threads, one tile at a time; every lane loads whole
//              records (coalesced 16-byte units, 8 in flight per lane), hashes the key from its
//              registers and counts into ONE per-workgroup LDS histogram of R counters.
//   k_scatter16 persistent 1024-thread workgroups, one tile range at a time with an LDS cursor
//              per partition.  The tile is cut into 64-record groups dealt to the waves in order;
//              a group ranks its equal pids with a ballot match, then, when the LDS turn counter
//              reaches it, reads and advances the cursors of its pids and hands the turn on.  Only
//              that short step is serialised; loads and the 16-byte stores are not.
// ------------------------------------------------------------------------------------------
template <int KW>
__global__ __launch_bounds__(1024) void k_hist16(PartDev pd, MapGroup g, uint16_t* __restrict__ pids,
                                                uint32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];  // [R]
  const int R = pd.R;
  const uint32_t ntiles = g.num_maps * g.tiles_per_map;
  const u32x4* recs = reinterpret_cast<const u32x4*>(g.recs);
  const int kw0 = pd.key_offset / 4;
  for (int p = threadIdx.x; p < R; p += 1024) hist[p] = 0;
  __syncthreads();
  for (uint32_t gt = blockIdx.x; gt < ntiles; gt += gridDim.x) {
    const TileRange tr = tile_range(g, gt);
    for (uint64_t i0 = tr.begin; i0 < tr.end; i0 += 8 * 1024) {
      u32x4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint64_t i = i0 + k * 1024 + threadIdx.x;
        v[k] = recs[i < tr.end ? i : tr.begin];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint64_t i = i0 + k * 1024 + threadIdx.x;
        if (i < tr.end) {
          uint32_t w[KW];
#pragma unroll
          for (int q = 0; q < KW; ++q) {
            const int d = kw0 + q;
            w[q] = d == 0 ? v[k][0] : d == 1 ? v[k][1] : d == 2 ? v[k][2] : v[k][3];
          }
          const int p = partition_words<KW, false>(pd, w, pd.bounds, pd.lut);
          atomicAdd(&hist[p], 1u);
          pids[i] = (uint16_t)p;
        }
      }
    }
    __syncthreads();
    // tile-major counts [map][tile][p]: one contiguous row per tile (a partition-major column
    // would touch R lines at a 4*tiles stride for R 4-byte counters)
    uint32_t* dst = counts + ((uint64_t)tr.map * g.tiles_per_map + tr.tile) * R;
    for (int p = threadIdx.x; p < R; p += 1024) {
      dst[p] = hist[p];
      hist[p] = 0;
    }
    __syncthreads();
  }
}

// Wait until the LDS turn counter reaches `want`.  Bounded: after 2^22 sleeps (far beyond any
// legitimate wait) the wave sets the node's device error word (sux_node_check reports it) and
// the workgroup's stop flag, and every wave of the workgroup leaves without touching the
// cursors again; a wave that sees the stop flag while it waits leaves too.  Returns false then.
__device__ __forceinline__ bool wait_turn(uint32_t* turn, uint32_t want, uint32_t* stop,
                                          uint32_t* err) {
  for (uint32_t spin = 0;; ++spin) {
    if (__hip_atomic_load(turn, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == want) return true;
    if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
    if (spin > (1u << 22)) {
      if (__lane_id() == 0) {
        if (err) atomicOr(err, kErrTurnTimeout);
        __hip_atomic_store(stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

template <uint32_t NW>
__global__ __launch_bounds__(NW * 64) void k_scatter16(MapGroup g, int R, int pid_bits,
                                                       const uint16_t* __restrict__ pids,
                                                       const uint32_t* __restrict__ prefix,
                                                       const uint64_t* __restrict__ base,
                                                       uint8_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cur[];  // [R] next output record of p
  __shared__ uint32_t turn, stop;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint32_t ntiles = g.num_maps * g.tiles_per_map;
  const u32x4* recs = reinterpret_cast<const u32x4*>(g.recs);
  u32x4* out4 = reinterpret_cast<u32x4*>(out);
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  if (tid == 0) stop = 0;
  for (uint32_t gt = xcd_map(blockIdx.x, gridDim.x); gt < ntiles; gt += gridDim.x) {
    const TileRange tr = tile_range(g, gt);
    const uint64_t* bm = base + (uint64_t)tr.map * R;
    const uint32_t* pm = prefix + ((uint64_t)tr.map * g.tiles_per_map + tr.tile) * R;  // tile-major
    for (int p = tid; p < R; p += NW * kWave) cur[p] = (uint32_t)(bm[p] + pm[p]);
    if (tid == 0) turn = 0;
    __syncthreads();
    const uint32_t ngroups = (uint32_t)((tr.end - tr.begin + kWave - 1) / kWave);
    // group q = wave + k * NW; the loads of the next two groups of this wave are in flight
    // during this group's turn (clamped, unconditional: the compiler's waits stay counted)
    auto load = [&](uint32_t qq, uint32_t& pv, u32x4& rv) {
      const uint64_t i = tr.begin + (uint64_t)qq * kWave + lane;
      const uint64_t ii = i < tr.end ? i : tr.end - 1;
      pv = pids[ii];
      rv = recs[ii];
    };
    uint32_t q = wave;
    uint32_t pid0, pid1;
    u32x4 rec0, rec1;
    load(q, pid0, rec0);
    load(q + NW, pid1, rec1);
    while (q < ngroups) {
      const uint64_t i = tr.begin + (uint64_t)q * kWave + lane;
      const bool valid = i < tr.end;
      uint32_t pid2;
      u32x4 rec2;
      load(q + 2 * NW, pid2, rec2);
      const uint32_t p = valid ? pid0 : 0u;
      uint64_t peers = __ballot(valid);
      for (int bb = 0; bb < pid_bits; ++bb) {
        const bool bit = (p >> bb) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
      }
      // this group's turn: groups update the cursors in input order (stability)
      if (!wait_turn(&turn, q, &stop, g.err)) break;
      uint32_t r0 = 0;
      if (valid) r0 = cur[p];
      __builtin_amdgcn_wave_barrier();
      if (valid && (peers & lt_mask) == 0) cur[p] = r0 + (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&turn, q + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (valid) out4[(uint64_t)r0 + (uint32_t)__popcll(peers & lt_mask)] = rec0;
      pid0 = pid1;
      rec0 = rec1;
      pid1 = pid2;
      rec1 = rec2;
      q += NW;
    }
    __syncthreads();
    if (stop) return;  // a turn timed out: the error word is set, nothing more is written
  }
}

// k_scatter16 with the turn handed on once per batch of GB consecutive 64-record groups instead of
// once per group: a wave ranks GB groups, then in its turn walks their cursor updates back to
// back (LDS ops of one wave stay in order), so the cross-wave hand-off (acquire spin, release
// fence) is paid GB x less often.  Same output bytes as k_scatter16 (input order kept).
template <uint32_t NW, int GB>
__global__ __launch_bounds__(NW * 64) void k_scatter16b(MapGroup g, int R, int pid_bits,
                                                        const uint16_t* __restrict__ pids,
                                                        const uint32_t* __restrict__ prefix,
                                                        const uint64_t* __restrict__ base,
                                                        uint8_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cur[];  // [R] next output record of p
  __shared__ uint32_t turn, stop;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint32_t ntiles = g.num_maps * g.tiles_per_map;
  const u32x4* recs = reinterpret_cast<const u32x4*>(g.recs);
  u32x4* out4 = reinterpret_cast<u32x4*>(out);
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  if (tid == 0) stop = 0;
  for (uint32_t gt = xcd_map(blockIdx.x, gridDim.x); gt < ntiles; gt += gridDim.x) {
    const TileRange tr = tile_range(g, gt);
    const uint64_t* bm = base + (uint64_t)tr.map * R;
    const uint32_t* pm = prefix + ((uint64_t)tr.map * g.tiles_per_map + tr.tile) * R;  // tile-major
    for (int p = tid; p < R; p += NW * kWave) cur[p] = (uint32_t)(bm[p] + pm[p]);
    if (tid == 0) turn = 0;
    __syncthreads();
    const uint32_t ngroups = (uint32_t)((tr.end - tr.begin + kWave - 1) / kWave);
    const uint32_t nbatch = (ngroups + GB - 1) / GB;
    uint32_t pa[GB], pb[GB];
    u32x4 ra[GB], rb[GB];
    auto load = [&](uint32_t bb, uint32_t (&pv)[GB], u32x4 (&rv)[GB]) {
#pragma unroll
      for (int k = 0; k < GB; ++k) {
        const uint64_t i = tr.begin + ((uint64_t)bb * GB + k) * kWave + lane;
        const uint64_t ii = i < tr.end ? i : tr.end - 1;  // clamped, unconditional
        pv[k] = pids[ii];
        rv[k] = recs[ii];
      }
    };
    uint32_t b = wave;
    load(b, pa, ra);
    while (b < nbatch) {
      load(b + NW, pb, rb);  // next batch in flight during this one's turn
      uint64_t peers[GB];
      uint32_t pp[GB];
      bool valid[GB];
#pragma unroll
      for (int k = 0; k < GB; ++k) {
        const uint64_t i = tr.begin + ((uint64_t)b * GB + k) * kWave + lane;
        valid[k] = i < tr.end;
        pp[k] = valid[k] ? pa[k] : 0u;
        uint64_t pe = __ballot(valid[k]);
        for (int bb = 0; bb < pid_bits; ++bb) {
          const bool bit = (pp[k] >> bb) & 1u;
          const uint64_t m = __ballot(bit);
          pe &= bit ? m : ~m;
        }
        peers[k] = pe;
      }
      if (!wait_turn(&turn, b, &stop, g.err)) break;
      uint32_t dst[GB];
#pragma unroll
      for (int k = 0; k < GB; ++k) {
        uint32_t r0 = 0;
        if (valid[k]) r0 = cur[pp[k]];
        __builtin_amdgcn_wave_barrier();
        if (valid[k] && (peers[k] & lt_mask) == 0) cur[pp[k]] = r0 + (uint32_t)__popcll(peers[k]);
        __builtin_amdgcn_wave_barrier();
        dst[k] = r0 + (uint32_t)__popcll(peers[k] & lt_mask);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&turn, b + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
      for (int k = 0; k < GB; ++k)
        if (valid[k]) out4[dst[k]] = ra[k];
#pragma unroll
      for (int k = 0; k < GB; ++k) {
        pa[k] = pb[k];
        ra[k] = rb[k];
      }
      b += NW;
    }
    __syncthreads();
    if (stop) return;  // a turn timed out: the error word is set, nothing more is written
  }
}

// ------------------------------------------------------------------------------------------
// k_scatter16s: the small-record scatter without turns (R <= kS16sMaxR).  A persistent
// 1024-thread workgroup walks tile ranges in 4096-record chunks; a chunk's stable rank of every
// record among the chunk's records of its partition comes from sorting the chunk's
// (pid, position) keys in LDS, not from waves taking turns on the cursors:
//   1. LSD radix passes of 7 pid bits over the 4096 keys (two for R <= 16384): a wave owns 256
//      consecutive positions and ranks them group by group with a ballot match against its own
//      per-digit counters; one block scan over (digit, wave) gives every wave's digit offsets, so
//      each pass is stable and needs no atomics;
//   2. run starts of the sorted keys (rs[p] = first sorted position of p), then every record's
//      destination cursor[p] + (sorted position - rs[p]); run ends advance the cursors;
//   3. every thread stores the records it loaded, in input order (16-byte stores).
// Three barriers per pass and three for the rest; the next chunk's pids and records are in
// flight the whole time.  Same bytes as k_scatter16 / k_scatter16b.
// ------------------------------------------------------------------------------------------
constexpr uint32_t kS16sChunk = 4096;    // records per chunk: 4 per thread of 1024
constexpr uint32_t kS16sIdxBits = 12;    // log2(kS16sChunk)
constexpr uint32_t kS16sDigit = 7;       // pid bits per LDS radix pass
constexpr int kS16sMaxR = 16384;         // two passes; cursors + run starts fit the LDS

struct Sc16s {
  static constexpr uint32_t NT = 1024, NW = 16, PT = kS16sChunk / NT, NB = 1u << kS16sDigit;
  // cur[R] u32 | rs[R] u16 (padded) | keys[2][chunk] u32 | wc[2][NW][NB] u32 | wsum[NW] u32
  static __host__ __device__ constexpr uint32_t lds_bytes(int R) {
    return (uint32_t)R * 4 + ((uint32_t)R * 2 + 15) / 16 * 16 + 2 * kS16sChunk * 4 +
           2 * NW * NB * 4 + NW * 4;
  }
};

__global__ __launch_bounds__(1024) void k_scatter16s(MapGroup g, int R, int pid_bits,
                                                     const uint16_t* __restrict__ pids,
                                                     const uint32_t* __restrict__ prefix,
                                                     const uint64_t* __restrict__ base,
                                                     uint8_t* __restrict__ out) {
  using K = Sc16s;
  constexpr uint32_t NT = K::NT, NW = K::NW, PT = K::PT, NB = K::NB, CH = kS16sChunk;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  uint32_t* cur = reinterpret_cast<uint32_t*>(lds8);
  uint16_t* rs = reinterpret_cast<uint16_t*>(cur + R);
  uint32_t* keys0 = reinterpret_cast<uint32_t*>(lds8 + (uint32_t)R * 4 + ((uint32_t)R * 2 + 15) / 16 * 16);
  uint32_t* keys1 = keys0 + CH;
  uint32_t* wc0 = keys1 + CH;  // [2][NW][NB]
  uint32_t* wsum = wc0 + 2 * NW * NB;

  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const uint32_t ntiles = g.num_maps * g.tiles_per_map;
  const u32x4* recs = reinterpret_cast<const u32x4*>(g.recs);
  u32x4* out4 = reinterpret_cast<u32x4*>(out);
  const int passes = pid_bits <= (int)kS16sDigit ? 1 : 2;

  for (uint32_t i = tid; i < 2 * NW * NB; i += NT) wc0[i] = 0;
  for (uint32_t gt = xcd_map(blockIdx.x, gridDim.x); gt < ntiles; gt += gridDim.x) {
    const TileRange tr = tile_range(g, gt);
    const uint64_t* bm = base + (uint64_t)tr.map * R;
    const uint32_t* pm = prefix + ((uint64_t)tr.map * g.tiles_per_map + tr.tile) * R;  // tile-major
    for (int p = tid; p < R; p += NT) cur[p] = (uint32_t)(bm[p] + pm[p]);
    const uint32_t nchunks = (uint32_t)((tr.end - tr.begin + CH - 1) / CH);
    // element e = wave * 256 + j * 64 + lane: a wave's positions are contiguous and visited in
    // order, which is what keeps every radix pass stable
    uint32_t pv[PT];
    u32x4 rv[PT];
    auto load = [&](uint32_t c, uint32_t (&p)[PT], u32x4 (&r)[PT]) {
      const uint64_t c0 = tr.begin + (uint64_t)(c < nchunks ? c : 0) * CH;
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint64_t i = c0 + wave * (PT * kWave) + j * kWave + lane;
        const uint64_t ii = i < tr.end ? i : tr.end - 1;  // clamped, unconditional
        p[j] = pids[ii];
        r[j] = recs[ii];
      }
    };
    if (nchunks) load(0, pv, rv);
    __syncthreads();  // cursors ready
    for (uint32_t c = 0; c < nchunks; ++c) {
      const uint32_t n = (uint32_t)min<uint64_t>(CH, tr.end - tr.begin - (uint64_t)c * CH);
      uint32_t pn[PT];
      u32x4 rn[PT];
      load(c + 1, pn, rn);  // the next chunk flies during this one
      // 1. LSD radix passes over (pid << 12 | position)
      uint32_t* kin = keys0;
      uint32_t* kout = keys1;
      for (int d = 0; d < passes; ++d) {
        uint32_t* wc = wc0 + (d & 1) * NW * NB;
        const uint32_t sh = kS16sIdxBits + d * kS16sDigit;
        uint32_t key[PT], dig[PT], rank[PT];
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j) {
          const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
          const bool valid = e < n;
          key[j] = d == 0 ? ((pv[j] << kS16sIdxBits) | e) : (valid ? kin[e] : 0u);
          dig[j] = valid ? (key[j] >> sh) & (NB - 1) : 0u;
          uint64_t peers = __ballot(valid);
#pragma unroll
          for (uint32_t bb = 0; bb < kS16sDigit; ++bb) {
            const bool bit = (dig[j] >> bb) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
          }
          uint32_t* w = wc + wave * NB + dig[j];
          uint32_t r0 = 0;
          if (valid) r0 = *w;
          __builtin_amdgcn_wave_barrier();
          if (valid && (peers & lt_mask) == 0) *w = r0 + (uint32_t)__popcll(peers);
          __builtin_amdgcn_wave_barrier();
          rank[j] = valid ? r0 + (uint32_t)__popcll(peers & lt_mask) : ~0u;
        }
        __syncthreads();
        // block exclusive scan of the counters in (digit, wave) order: thread t owns digit
        // t / 8 and waves 2(t % 8), 2(t % 8) + 1
        {
          const uint32_t dg = tid / (NW / 2), w0 = 2 * (tid % (NW / 2));
          const uint32_t a = wc[w0 * NB + dg], b = wc[(w0 + 1) * NB + dg];
          const uint32_t incl = wave_incl_scan(a + b, lane);
          if (lane == kWave - 1) wsum[wave] = incl;
          __syncthreads();
          uint32_t before = 0;
#pragma unroll
          for (uint32_t w = 0; w < NW; ++w) before += w < (uint32_t)wave ? wsum[w] : 0u;
          const uint32_t ex = before + incl - (a + b);
          wc[w0 * NB + dg] = ex;
          wc[(w0 + 1) * NB + dg] = ex + a;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j)
          if (rank[j] != ~0u) kout[wc[wave * NB + dig[j]] + rank[j]] = key[j];
        __syncthreads();
        // this counter set is next used at least one barrier later (next chunk or pass)
        for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
        uint32_t* t = kin;
        kin = kout;
        kout = t;
      }
      // 2. run starts, destinations (into the free key buffer, by position), cursor advances
      uint32_t* dsta = kout;
      uint32_t endp[PT], endv[PT];
#pragma unroll
      for (uint32_t k = 0; k < PT; ++k) {
        const uint32_t s = tid + k * NT;
        endp[k] = ~0u;
        if (s < n) {
          const uint32_t p = kin[s] >> kS16sIdxBits;
          if (s == 0 || (kin[s - 1] >> kS16sIdxBits) != p) rs[p] = (uint16_t)s;
        }
      }
      __syncthreads();
#pragma unroll
      for (uint32_t k = 0; k < PT; ++k) {
        const uint32_t s = tid + k * NT;
        if (s < n) {
          const uint32_t key = kin[s], p = key >> kS16sIdxBits;
          const uint32_t dst = cur[p] + (s - rs[p]);
          dsta[key & (CH - 1)] = dst;
          if (s + 1 == n || (kin[s + 1] >> kS16sIdxBits) != p) {
            endp[k] = p;
            endv[k] = dst + 1;
          }
        }
      }
      __syncthreads();
      // 3. stores in input order; the cursors move on (every read of them is behind the barrier)
#pragma unroll
      for (uint32_t k = 0; k < PT; ++k)
        if (endp[k] != ~0u) cur[endp[k]] = endv[k];
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
        if (e < n) out4[dsta[e]] = rv[j];
      }
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        pv[j] = pn[j];
        rv[j] = rn[j];
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------------------------
// Two-pass small-record scatter (16-byte records, R > 1024): C5 writes ~0.4 record per
// partition per 4096-record chunk, so a one-pass scatter stores every record alone — a partial
// 128-B line each (PMC: 32 B written per 16-B record) at a random address.  Instead:
//   pass A (k_bucket16a) regroups every tile by bucket = pid >> 6 (<= 256 buckets) into the
//          workspace's temp buffer, at the bucket's final position: bucket h of map m starts at
//          base[m][64h], the tile's share after the earlier tiles' (the K2 tile prefix summed
//          over the bucket's 64 partitions).  A chunk is stable-sorted by bucket in LDS and
//          written in sorted order: runs of ~26 records per bucket instead of ~0.4;
//   pass B (k_bucket16b) takes one (map, bucket) segment — its output range is the same
//          range of the output, [base[m][64h], base[m][64h+64]) — recomputes each record's pid
//          from its key, stable-sorts by the low 6 bits in LDS and writes the segment back in
//          order: one contiguous, fully coalesced range per segment.
// 16 + 2 + 16 (A) and 16 + 16 (B) bytes per record, every write a long run.  Stable: pass A
// keeps input order inside a bucket, pass B inside a partition.
// ------------------------------------------------------------------------------------------
constexpr uint32_t kB16Lo = 6;         // partitions per bucket: 64
constexpr uint32_t kB16PT = 4;         // records per thread per LDS chunk (chunk = 256 x waves)

template <uint32_t NW>  // stage[chunk] u32x4 | wc[NW][256] u32 | cb[256] u32 | wsum[NW] | hs[chunk] u8
struct B16a {
  static constexpr uint32_t NB = 256, CH = NW * kWave * kB16PT;
  static constexpr uint32_t lds_bytes() { return CH * 16 + NW * NB * 4 + NB * 4 + NW * 4 + CH; }
};
template <uint32_t NW>  // stage[chunk] u32x4 | wc[NW][64] u32 | cur[64] u32 | wsum[NW] | los[chunk] u8
struct B16b {
  static constexpr uint32_t NB = 1u << kB16Lo, CH = NW * kWave * kB16PT;
  static constexpr uint32_t lds_bytes() { return CH * 16 + NW * NB * 4 + NB * 4 + NW * 4 + CH; }
};

// Stable in-wave rank of `dig` (DB bits) against the wave's running per-digit counters wcw[]:
// lanes of the group in lane order after the wave's earlier groups.  ~0 for invalid lanes.
template <uint32_t DB, typename CT = uint32_t>
__device__ __forceinline__ uint32_t wave_rank(uint32_t dig, bool valid, CT* wcw, uint64_t lt_mask) {
  uint64_t peers = __ballot(valid);
#pragma unroll
  for (uint32_t bb = 0; bb < DB; ++bb) {
    const bool bit = (dig >> bb) & 1u;
    const uint64_t m = __ballot(bit);
    peers &= bit ? m : ~m;
  }
  uint32_t r0 = 0;
  if (valid) r0 = wcw[dig];
  __builtin_amdgcn_wave_barrier();
  if (valid && (peers & lt_mask) == 0) wcw[dig] = (CT)(r0 + (uint32_t)__popcll(peers));
  __builtin_amdgcn_wave_barrier();
  return valid ? r0 + (uint32_t)__popcll(peers & lt_mask) : ~0u;
}

// Block exclusive scan of wc[NW][NB] in (digit, wave) order, in place (NW*64 threads, NB*NW
// entries, E = NB/64 consecutive entries per thread).  Two barriers.
template <uint32_t NB, uint32_t NW>
__device__ __forceinline__ void scan_digit_wave(uint32_t* wc, uint32_t* wsum, int tid, int lane, int wave) {
  constexpr uint32_t E = NB / kWave;
  static_assert(E >= 1 && NW % E == 0, "entries per thread");
  const uint32_t dg = (uint32_t)tid * E / NW, w0 = ((uint32_t)tid * E) % NW;
  uint32_t v[E], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < E; ++k) {
    v[k] = wc[(w0 + k) * NB + dg];
    sum += v[k];
  }
  const uint32_t incl = wave_incl_scan(sum, lane);
  if (lane == kWave - 1) wsum[wave] = incl;
  __syncthreads();
  uint32_t run = incl - sum;
#pragma unroll
  for (uint32_t w = 0; w < NW; ++w) run += w < (uint32_t)wave ? wsum[w] : 0u;
#pragma unroll
  for (uint32_t k = 0; k < E; ++k) {
    wc[(w0 + k) * NB + dg] = run;
    run += v[k];
  }
  __syncthreads();
}

template <uint32_t NW>
__global__ __launch_bounds__(NW * 64) void k_bucket16a(MapGroup g, int R,
                                                    const uint16_t* __restrict__ pids,
                                                    const uint32_t* __restrict__ prefix,
                                                    const uint64_t* __restrict__ base,
                                                    uint8_t* __restrict__ tmp) {
  constexpr uint32_t NB = B16a<NW>::NB, CH = B16a<NW>::CH, PT = kB16PT, NT = NW * kWave;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  u32x4* stage = reinterpret_cast<u32x4*>(lds8);
  uint32_t* wc = reinterpret_cast<uint32_t*>(stage + CH);  // [NW][NB]
  uint32_t* cb = wc + NW * NB;
  uint32_t* wsum = cb + NB;
  uint8_t* hs = reinterpret_cast<uint8_t*>(wsum + NW);
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const uint32_t ntiles = g.num_maps * g.tiles_per_map;
  const uint32_t nbk = ((uint32_t)R + (1u << kB16Lo) - 1) >> kB16Lo;
  const u32x4* recs = reinterpret_cast<const u32x4*>(g.recs);
  u32x4* t4 = reinterpret_cast<u32x4*>(tmp);
  for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
  for (uint32_t gt = xcd_map(blockIdx.x, gridDim.x); gt < ntiles; gt += gridDim.x) {
    const TileRange tr = tile_range(g, gt);
    if (tid < (int)nbk) {  // bucket cursor: its base + the earlier tiles' records of its partitions
      const uint32_t p0 = (uint32_t)tid << kB16Lo, p1 = min(p0 + (1u << kB16Lo), (uint32_t)R);
      const uint32_t* pm = prefix + ((uint64_t)tr.map * g.tiles_per_map + tr.tile) * R;
      uint32_t s = 0;
      for (uint32_t p = p0; p < p1; ++p) s += pm[p];
      cb[tid] = (uint32_t)base[(uint64_t)tr.map * R + p0] + s;
    }
    const uint32_t nchunks = (uint32_t)((tr.end - tr.begin + CH - 1) / CH);
    uint32_t pv[PT];
    u32x4 rv[PT];
    auto load = [&](uint32_t c, uint32_t (&p)[PT], u32x4 (&r)[PT]) {
      const uint64_t c0 = tr.begin + (uint64_t)(c < nchunks ? c : 0) * CH;
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint64_t i = c0 + wave * (PT * kWave) + j * kWave + lane;
        const uint64_t ii = i < tr.end ? i : tr.end - 1;
        p[j] = pids[ii];
        r[j] = recs[ii];
      }
    };
    if (nchunks) load(0, pv, rv);
    __syncthreads();
    for (uint32_t c = 0; c < nchunks; ++c) {
      const uint32_t n = (uint32_t)min<uint64_t>(CH, tr.end - tr.begin - (uint64_t)c * CH);
      uint32_t pn[PT];
      u32x4 rn[PT];
      load(c + 1, pn, rn);
      uint32_t h[PT], rank[PT];
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
        h[j] = (pv[j] >> kB16Lo) & (NB - 1);
        rank[j] = wave_rank<8>(h[j], e < n, wc + wave * NB, lt_mask);
      }
      __syncthreads();
      scan_digit_wave<NB, NW>(wc, wsum, tid, lane, wave);
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j)
        if (rank[j] != ~0u) {
          const uint32_t pos = wc[wave * NB + h[j]] + rank[j];
          stage[pos] = rv[j];
          hs[pos] = (uint8_t)h[j];
        }
      __syncthreads();
      // sorted order: consecutive positions of a bucket go to consecutive temp records
#pragma unroll
      for (uint32_t k = 0; k < PT; ++k) {
        const uint32_t i = tid + k * NT;
        if (i < n) {
          const uint32_t b = hs[i];
          const uint64_t dst = (uint64_t)cb[b] + (i - wc[b]);  // wc[0 * NB + b]: bucket start
          if (dst < g.num_records) t4[dst] = stage[i];         // (a bad pid cannot fault)
        }
      }
      uint32_t ncb = 0;
      if (tid < (int)nbk) {
        const uint32_t end = (uint32_t)tid + 1 < NB ? wc[tid + 1] : n;
        ncb = cb[tid] + (end - wc[tid]);
      }
      __syncthreads();
      if (tid < (int)nbk) cb[tid] = ncb;
      for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        pv[j] = pn[j];
        rv[j] = rn[j];
      }
      __syncthreads();
    }
  }
}

// Pass B walks a stream of (segment, chunk) pairs: the next chunk's records — across a segment
// seam too, with the next segment's 64 cursors — are loaded while this chunk is sorted and
// written, so no chunk waits for its loads.
template <int KW, uint32_t NW>
__global__ __launch_bounds__(NW * 64) void k_bucket16b(PartDev pd, MapGroup g,
                                                    const uint64_t* __restrict__ base,
                                                    const uint64_t* __restrict__ totals,
                                                    const uint8_t* __restrict__ tmp,
                                                    uint8_t* __restrict__ out) {
  constexpr uint32_t NB = B16b<NW>::NB, CH = B16b<NW>::CH, PT = kB16PT, NT = NW * kWave;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  u32x4* stage = reinterpret_cast<u32x4*>(lds8);
  uint32_t* wc = reinterpret_cast<uint32_t*>(stage + CH);  // [NW][NB]
  uint32_t* cur = wc + NW * NB;
  uint32_t* wsum = cur + NB;
  uint8_t* los = reinterpret_cast<uint8_t*>(wsum + NW);
  const int R = pd.R;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const uint32_t nbk = ((uint32_t)R + NB - 1) / NB;
  const uint32_t nitems = g.num_maps * nbk, G = gridDim.x;
  const int kw0 = pd.key_offset / 4;
  const u32x4* t4 = reinterpret_cast<const u32x4*>(tmp);
  u32x4* out4 = reinterpret_cast<u32x4*>(out);

  struct Cur {
    uint32_t it, p0;
    uint64_t c0, b1;
    bool valid, first;
  };
  auto seg = [&](uint32_t it) {  // first chunk of segment `it` (an empty segment: c0 == b1)
    Cur k;
    k.it = it;
    k.valid = it < nitems;
    k.first = true;
    const uint32_t m = k.valid ? it / nbk : 0, hb = k.valid ? it - m * nbk : 0;
    k.p0 = hb * NB;
    const uint32_t p1 = min(k.p0 + NB, (uint32_t)R);
    const uint64_t* bm = base + (uint64_t)m * R;
    k.c0 = bm[k.p0];
    k.b1 = bm[p1 - 1] + totals[(uint64_t)m * R + p1 - 1];
    return k;
  };
  auto next = [&](const Cur& k) {
    Cur nk = k;
    nk.first = false;
    nk.c0 = k.c0 + CH;
    if (nk.c0 >= k.b1) nk = seg(k.it + G);
    return nk;
  };
  // loads of chunk k (clamped, unconditional) and, at a segment's first chunk, its cursors
  auto issue = [&](const Cur& k, u32x4 (&r)[PT], uint32_t& cv) {
    const uint32_t n = k.valid && k.b1 > k.c0 ? (uint32_t)min<uint64_t>(CH, k.b1 - k.c0) : 1u;
    const uint64_t c0 = k.valid && k.b1 > k.c0 ? k.c0 : 0;
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
      const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
      r[j] = t4[c0 + (e < n ? e : n - 1)];
    }
    if (k.valid && k.first && tid < (int)NB) {
      const uint32_t m = k.it / nbk;
      const uint32_t p = min(k.p0 + (uint32_t)tid, (uint32_t)R - 1);
      cv = (uint32_t)base[(uint64_t)m * R + p];
    }
  };

  for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
  Cur k = seg(xcd_map(blockIdx.x, G));
  u32x4 rv[PT];
  uint32_t cv = 0;
  issue(k, rv, cv);
  while (k.valid) {
    if (k.first && tid < (int)NB) cur[tid] = cv;  // nothing reads cur until the write phase
    const Cur nk = next(k);
    u32x4 rn[PT];
    uint32_t cn = cv;
    issue(nk, rn, cn);
    const uint32_t n = k.b1 > k.c0 ? (uint32_t)min<uint64_t>(CH, k.b1 - k.c0) : 0u;
    uint32_t lo[PT], rank[PT];
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
      const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
      uint32_t w[KW];
#pragma unroll
      for (int q = 0; q < KW; ++q) {
        const int d = kw0 + q;
        w[q] = d == 0 ? rv[j][0] : d == 1 ? rv[j][1] : d == 2 ? rv[j][2] : rv[j][3];
      }
      lo[j] = ((uint32_t)partition_words<KW, false>(pd, w, pd.bounds, pd.lut) - k.p0) & (NB - 1);
      rank[j] = wave_rank<kB16Lo>(lo[j], e < n, wc + wave * NB, lt_mask);
    }
    __syncthreads();
    scan_digit_wave<NB, NW>(wc, wsum, tid, lane, wave);
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j)
      if (rank[j] != ~0u) {
        const uint32_t pos = wc[wave * NB + lo[j]] + rank[j];
        stage[pos] = rv[j];
        los[pos] = (uint8_t)lo[j];
      }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < PT; ++q) {
      const uint32_t i = tid + q * NT;
      if (i < n) {
        const uint32_t l = los[i];
        const uint64_t dst = (uint64_t)cur[l] + (i - wc[l]);
        if (dst < g.num_records) out4[dst] = stage[i];  // (a bad pid cannot fault)
      }
    }
    uint32_t ncur = 0;
    if (tid < (int)NB) {
      const uint32_t end = (uint32_t)tid + 1 < NB ? wc[tid + 1] : n;
      ncur = cur[tid] + (end - wc[tid]);
    }
    __syncthreads();
    if (tid < (int)NB) cur[tid] = ncur;
    for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) rv[j] = rn[j];
    cv = cn;
    k = nk;
  }
}

// ------------------------------------------------------------------------------------------
// Two-level (MSD) small-record map side without K1 (16-byte records, 1024 < R <= 16384,
// map-major layout; tuning small_kernel = 4).  Every pass streams whole lines:
//   pass A (k_msd16a) reads each 4096-record chunk once, computes every record's pid from its
//          key, stable-sorts the chunk by bucket = pid >> 5 in LDS and writes it back to the
//          temp copy AT THE CHUNK'S OWN POSITION (a contiguous write), with the chunk's bucket
//          starts (u16) in offs[map][chunk][bucket];
//   K2     (k_msd16_scan) one workgroup per map: bucket totals over the map's chunks ->
//          segment bases segbase[map][bucket] and the index table's last entry;
//   pass B (k_msd16b) one (map, bucket) segment at a time: the segment's runs (one ~13-record
//          run per chunk at R = 10 000) are gathered into LDS, stable-sorted by pid & 31,
//          written as ONE contiguous output range, and the bucket's 32 index entries (native +
//          big-endian) are written.  A segment larger than the LDS (skewed keys) is counted
//          first and then placed piece by piece through per-partition cursors.
// 16 + 16 (A) and 16 + 16 (B) bytes per record, no pid array, no R-wide histogram: the
// sorted-chunk scatter (k_hist16 + k_scatter16s) moves 19 + 54 bytes per record, 32 of them as
// lone 16-byte stores.  Both passes run two 512-thread workgroups per CU, whose load, rank and
// store phases interleave.  Stable: pass A keeps input order inside a bucket (chunks in order,
// ranks in order inside a chunk), pass B keeps segment order inside a partition.
// ------------------------------------------------------------------------------------------
// Diagnostic build only (tools/msd_stamps.hip defines SUX_MSD_STAMPS): per-phase s_memtime
// cycles of k_msd16b, summed per workgroup into g_msd_stamps[block][phase].
#ifdef SUX_MSD_STAMPS
__device__ unsigned long long* g_msd_stamps;
#define SUX_MSD_STAMP_INIT()                 \
  unsigned long long st_acc[5] = {0, 0, 0, 0, 0}; \
  unsigned long long st_t = __builtin_amdgcn_s_memtime()
#define SUX_MSD_STAMP(k)                                   \
  do {                                                     \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t_ - st_t;                                \
    st_t = t_;                                             \
  } while (0)
#define SUX_MSD_STAMP_END()                                              \
  do {                                                                   \
    if (threadIdx.x == 0 && g_msd_stamps)                                \
      for (int k_ = 0; k_ < 5; ++k_) g_msd_stamps[blockIdx.x * 8 + k_] = st_acc[k_]; \
  } while (0)
#else
#define SUX_MSD_STAMP_INIT() do {} while (0)
#define SUX_MSD_STAMP(k) do {} while (0)
#define SUX_MSD_STAMP_END() do {} while (0)
#endif
constexpr uint32_t kM16Chunk = 4096;      // pass A records per chunk (the run table's unit)
constexpr uint32_t kM16Lo = 4;            // partitions per bucket: 16
constexpr uint32_t kM16MaxChunks = 512;   // chunks per map pass B's run table holds (2 Mi records)

// Block exclusive scan, in (digit, wave) order, of u16 per-wave digit counters wc[NW][NB]
// (NW*64 threads; each thread owns E = NB/64 consecutive (digit, wave) entries).  Counts and
// prefixes fit u16: a chunk holds kM16Chunk records.  Two barriers; wsum[NW] scratch.
template <uint32_t NB, uint32_t NW>
__device__ __forceinline__ void scan_digit_wave16(uint16_t* wc, uint32_t* wsum, int tid, int lane,
                                                  int wave) {
  constexpr uint32_t E = NB / kWave;
  uint32_t sum = 0;  // the entries are read twice instead of held (registers are the limit)
#pragma unroll
  for (uint32_t k = 0; k < E; ++k) {
    const uint32_t idx = (uint32_t)tid * E + k, d = idx / NW, w = idx % NW;
    sum += wc[w * NB + d];
  }
  const uint32_t incl = wave_incl_scan(sum, lane);
  if (lane == kWave - 1) wsum[wave] = incl;
  __syncthreads();
  uint32_t run = incl - sum;
#pragma unroll
  for (uint32_t w = 0; w < NW; ++w) run += w < (uint32_t)wave ? wsum[w] : 0u;
#pragma unroll
  for (uint32_t k = 0; k < E; ++k) {
    const uint32_t idx = (uint32_t)tid * E + k, d = idx / NW, w = idx % NW;
    const uint32_t v = wc[w * NB + d];
    wc[w * NB + d] = (uint16_t)run;
    run += v;
  }
  __syncthreads();
}

template <uint32_t NW, uint32_t DB>  // stage[CH] u32x4 (its first NW words double as wsum) | wc[NW][2^DB] u16
struct M16a {
  static constexpr uint32_t NB = 1u << DB, NT = NW * kWave, PT = kM16Chunk / NT;
  static constexpr uint32_t lds_bytes() { return kM16Chunk * 16 + NW * NB * 2; }
};
template <uint32_t NW, uint32_t PT>  // stage[CAP] u32x4 | wc[NW][64] | cur[64] | wsum[NW] | los[CAP] u8 | rp[MAXCH+1] u32 | ro[MAXCH] u16
struct M16b {
  static constexpr uint32_t NB = 64, NT = NW * kWave, CAP = NT * PT;
  static constexpr uint32_t lds_bytes() {
    return CAP * 16 + NW * NB * 4 + NB * 4 + NW * 4 + CAP + (kM16MaxChunks + 1) * 4 +
           kM16MaxChunks * 2;
  }
};

// records of map m in the group, and of its chunk c
__device__ __forceinline__ uint32_t m16_map_len(const MapGroup& g, uint32_t m) {
  const uint64_t b = (uint64_t)m * g.records_per_map;
  const uint64_t e = min(b + g.records_per_map, g.num_records);
  return (uint32_t)(e > b ? e - b : 0);
}
__device__ __forceinline__ uint32_t m16_chunk_len(uint32_t map_len, uint32_t c) {
  const uint32_t b = c * kM16Chunk;
  return map_len > b ? min(kM16Chunk, map_len - b) : 0u;
}

template <int KW>
__device__ __forceinline__ uint32_t m16_pid(const PartDev& pd, const u32x4& r, int kw0) {
  uint32_t w[KW];
#pragma unroll
  for (int q = 0; q < KW; ++q) {
    const int d = kw0 + q;
    w[q] = d == 0 ? r[0] : d == 1 ? r[1] : d == 2 ? r[2] : r[3];
  }
  return (uint32_t)partition_words<KW, false>(pd, w, pd.bounds, pd.lut);
}

template <int KW, uint32_t NW, uint32_t DB>
__global__ __launch_bounds__(NW * 64, 4) void k_msd16a(PartDev pd, MapGroup g, uint32_t cpm,
                                                 uint32_t nbk, uint16_t* __restrict__ offs,
                                                 uint16_t* __restrict__ pids_out,
                                                 uint8_t* __restrict__ tmp) {
  using K = M16a<NW, DB>;
  constexpr uint32_t NB = K::NB, NT = K::NT, PT = K::PT, CH = kM16Chunk;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  u32x4* stage = reinterpret_cast<u32x4*>(lds8);
  uint16_t* wc = reinterpret_cast<uint16_t*>(stage + CH);  // [NW][NB]
  uint32_t* wsum = reinterpret_cast<uint32_t*>(lds8);       // only inside the scan: stage is idle
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const int kw0 = pd.key_offset / 4;
  const u32x4* recs = reinterpret_cast<const u32x4*>(g.recs);
  u32x4* t4 = reinterpret_cast<u32x4*>(tmp);
  // one contiguous, balanced range of (map, chunk) items per workgroup
  const uint32_t items = g.num_maps * cpm, G = gridDim.x, b = xcd_map(blockIdx.x, G);
  const uint32_t it0 = (uint32_t)((uint64_t)items * b / G), it1 = (uint32_t)((uint64_t)items * (b + 1) / G);
  struct Item {
    uint64_t c0;  // first record of the chunk (group index)
    uint32_t n;   // its records (0 past the range)
  };
  auto item = [&](uint32_t it) {
    const uint32_t m = it / cpm, c = it - m * cpm;
    Item k;
    k.c0 = (uint64_t)m * g.records_per_map + (uint64_t)c * CH;
    k.n = it < it1 ? m16_chunk_len(m16_map_len(g, m), c) : 0u;
    return k;
  };
  auto load = [&](const Item& k, u32x4 (&r)[PT]) {
    if (k.n == 0) return;
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {  // unconditional (clamped) loads: no per-load wait
      const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
      r[j] = recs[k.c0 + min(e, k.n - 1)];
    }
  };
  for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
  __syncthreads();
  u32x4 rv[PT];
  for (uint32_t it = it0; it < it1; ++it) {
    const Item k = item(it);
    load(k, rv);
    uint32_t h[PT], rank[PT];
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
      const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
      const bool valid = e < k.n;
      uint32_t p = 0;
      if (valid) {
        p = m16_pid<KW>(pd, rv[j], kw0);
        if (pids_out) pids_out[k.c0 + e] = (uint16_t)p;
      }
      h[j] = (p >> kM16Lo) & (NB - 1);
      rank[j] = wave_rank<DB, uint16_t>(h[j], valid, wc + wave * NB, lt_mask);
    }
    __syncthreads();
    scan_digit_wave16<NB, NW>(wc, wsum, tid, lane, wave);
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j)
      if (rank[j] != ~0u) stage[wc[wave * NB + h[j]] + rank[j]] = rv[j];
    __syncthreads();
    // the chunk goes back to its own place, in bucket order: one contiguous write
#pragma unroll
    for (uint32_t q = 0; q < PT; ++q) {
      const uint32_t i = tid + q * NT;
      if (i < k.n) t4[k.c0 + i] = stage[i];
    }
    for (uint32_t hb = tid; hb < nbk; hb += NT)
      offs[(uint64_t)it * nbk + hb] = (uint16_t)wc[hb];  // wc[0][hb]: bucket start in the chunk
    __syncthreads();
    for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
    __syncthreads();
  }
}

// K2 of the MSD path: one workgroup (kScanThreads) per map.  Bucket totals over the map's chunks
// (one thread per bucket), exclusive scan over buckets ->
// segbase[m][h] (record index in the group's output), the index table's last entry and, at
// world 1, the peer byte count.
__global__ __launch_bounds__(kScanThreads) void k_msd16_scan(MapGroup g, uint32_t cpm, uint32_t nbk,
                                                             const uint16_t* __restrict__ offs,
                                                             uint64_t* __restrict__ segbase,
                                                             int64_t* __restrict__ index,
                                                             uint8_t* __restrict__ index_be,
                                                             uint64_t* __restrict__ peer_bytes,
                                                             int R) {
  constexpr uint32_t HG = 1024, NG = kScanThreads / HG;  // one thread per bucket (nbk <= 1024)
  __shared__ uint64_t sh[2 * kWave + 1];
  __shared__ uint32_t part[kScanThreads];
  const uint32_t m = blockIdx.x, tid = threadIdx.x;
  const uint32_t len = m16_map_len(g, m), nch = (len + kM16Chunk - 1) / kM16Chunk;
  const uint32_t h = tid % HG, cg = tid / HG;
  uint32_t t = 0;
  if (h < nbk) {
    const uint16_t* om = offs + (uint64_t)m * cpm * nbk;
    for (uint32_t c = cg; c < nch; c += NG) {
      const uint32_t o = om[(uint64_t)c * nbk + h];
      const uint32_t e = h + 1 < nbk ? om[(uint64_t)c * nbk + h + 1] : m16_chunk_len(len, c);
      t += e - o;
    }
  }
  part[tid] = t;
  __syncthreads();
  uint64_t v = 0;
  if (tid < HG)
    for (uint32_t q = 0; q < NG; ++q) v += part[tid + q * HG];
  uint64_t tot;
  const uint64_t ex = block_excl_scan(tid < nbk ? v : 0, sh, &tot);
  if (tid < nbk) segbase[(uint64_t)m * nbk + tid] = (uint64_t)m * g.records_per_map + ex;
  if (tid == 0) {
    const int64_t off = (int64_t)len * g.rec_size;
    index[(uint64_t)m * (R + 1) + R] = off;
    if (index_be) reinterpret_cast<uint64_t*>(index_be)[(uint64_t)m * (R + 1) + R] = bswap64((uint64_t)off);
    if (m == 0 && peer_bytes) peer_bytes[0] = g.num_records * g.rec_size;
  }
}

template <int KW, uint32_t NW, uint32_t PT>
__global__ __launch_bounds__(NW * 64, 4) void k_msd16b(PartDev pd, MapGroup g, uint32_t cpm,
                                                 uint32_t nbk, const uint16_t* __restrict__ offs,
                                                 const uint64_t* __restrict__ segbase,
                                                 const uint8_t* __restrict__ tmp,
                                                 uint8_t* __restrict__ out,
                                                 int64_t* __restrict__ index,
                                                 uint8_t* __restrict__ index_be) {
  using K = M16b<NW, PT>;
  constexpr uint32_t NB = K::NB, NT = K::NT, CAP = K::CAP, MC = kM16MaxChunks, PB = 1u << kM16Lo;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  u32x4* stage = reinterpret_cast<u32x4*>(lds8);
  uint32_t* wc = reinterpret_cast<uint32_t*>(stage + CAP);  // [NW][NB]
  uint32_t* cur = wc + NW * NB;
  uint32_t* wsum = cur + NB;
  uint8_t* los = reinterpret_cast<uint8_t*>(wsum + NW);
  uint32_t* rp = reinterpret_cast<uint32_t*>(los + CAP);   // [MC + 1] run starts in the segment
  uint16_t* ro = reinterpret_cast<uint16_t*>(rp + MC + 1);  // [MC] run starts in their chunk
  const int R = pd.R;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const int kw0 = pd.key_offset / 4;
  const u32x4* t4 = reinterpret_cast<const u32x4*>(tmp);
  u32x4* out4 = reinterpret_cast<u32x4*>(out);
  uint64_t* ibe = reinterpret_cast<uint64_t*>(index_be);
  const uint32_t items = g.num_maps * nbk, G = gridDim.x, b = xcd_map(blockIdx.x, G);
  // segments dealt round robin (segment it to workgroup it % G, an XCD's workgroups taking
  // consecutive segments): at any moment the grid works on ~G consecutive segments, i.e. on
  // every bucket of a map or two, so the runs it gathers cover whole chunks of the temp copy
  // (DRAM rows and L2 lines shared by neighbouring runs are read together), and the outputs it
  // writes are adjacent.  (One contiguous range of segments per workgroup: 2.45 TB/s.)
  const uint32_t it0 = b, it1 = items;

  struct Seg {
    uint32_t m, h, nch, T, len;
    uint64_t mbase, out;  // first record of map m, first output record of the segment
  };
  // the global reads a segment's run table starts from (offs pair of chunk tid, segment base),
  // issued one segment ahead so that build() does not wait for them
  struct Pre {
    uint32_t o, e;
    uint64_t sb;
  };
  auto seg = [&](uint32_t it) {
    Seg s;
    s.m = it / nbk;
    s.h = it - s.m * nbk;
    s.len = m16_map_len(g, s.m);
    s.nch = (s.len + kM16Chunk - 1) / kM16Chunk;
    s.mbase = (uint64_t)s.m * g.records_per_map;
    return s;
  };
  auto run_ends = [&](const Seg& s, uint32_t c, uint32_t& o, uint32_t& e) {
    const uint16_t* oc = offs + ((uint64_t)s.m * cpm + c) * nbk;
    o = oc[s.h];
    e = s.h + 1 < nbk ? oc[s.h + 1] : m16_chunk_len(s.len, c);
  };
  auto prefetch = [&](uint32_t it) {
    Pre p{0, 0, 0};
    if (it < it1) {
      const Seg s = seg(it);
      if ((uint32_t)tid < s.nch) run_ends(s, tid, p.o, p.e);
      p.sb = segbase[it];
    }
    return p;
  };
  // run table of segment `it` (run c = the bucket's records of chunk c; rp = exclusive prefix
  // over chunks); all threads, barriers inside
  auto build = [&](uint32_t it, const Pre& pre) {
    Seg s = seg(it);
    s.out = pre.sb;
    uint32_t carry = 0;
    // the last batch's thread 0 also writes rp[nch] = T, the search's sentinel (no extra batch
    // when nch is a multiple of the workgroup: 2^20-record maps have exactly 256 chunks)
    for (uint32_t c0 = 0; c0 < s.nch; c0 += NT) {
      const uint32_t c = c0 + (uint32_t)tid;
      uint32_t o = pre.o, e = pre.e;
      if (c0 && c < s.nch) run_ends(s, c, o, e);
      const uint32_t cnt = c < s.nch ? e - o : 0u;
      const uint32_t incl = wave_incl_scan(cnt, lane);
      if (lane == kWave - 1) wsum[wave] = incl;
      __syncthreads();
      uint32_t run = carry + incl - cnt, blk = 0;
#pragma unroll
      for (uint32_t w = 0; w < NW; ++w) {
        run += w < (uint32_t)wave ? wsum[w] : 0u;
        blk += wsum[w];
      }
      if (c < s.nch) {
        ro[c] = (uint16_t)o;
        rp[c] = run;
      }
      if (tid == 0 && c0 + NT >= s.nch) rp[s.nch] = carry + blk;
      carry += blk;
      __syncthreads();
    }
    s.T = carry;
    return s;
  };
  // loads of segment elements [e0, min(T, e0 + CAP)) in wave-contiguous order
  auto load = [&](const Seg& s, uint32_t e0, u32x4 (&r)[PT]) {
    const uint32_t lim = min(s.T, e0 + CAP);
    if (lim <= e0) return;
    // element e's run = the largest c with rp[c] <= e: a branch-free search whose PT lookups
    // interleave step by step (rp[nch] = T > e stops every search inside the segment).  Lanes
    // past the piece re-read its last element: the loads are unconditional — a load under a
    // branch made the compiler wait for every earlier load before the next one's address
    // (s_waitcnt vmcnt(0) per element), serialising the gather.
    uint32_t lo[PT], ev[PT];
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
      lo[j] = 0;
      ev[j] = min(e0 + wave * (PT * kWave) + j * kWave + lane, lim - 1);
    }
#pragma unroll
    for (uint32_t step = MC / 2; step; step >>= 1) {
      uint32_t v[PT];
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) v[j] = rp[min(lo[j] + step, s.nch)];
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) lo[j] = v[j] <= ev[j] ? min(lo[j] + step, s.nch) : lo[j];
    }
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
#ifdef SUX_MSD_LINEAR  // diagnostic (tools/msd_stamps): contiguous in-map reads, wrong data
      r[j] = t4[s.mbase + ((uint64_t)s.h * 3350 + ev[j]) % s.len];
#else
      r[j] = t4[s.mbase + (uint64_t)lo[j] * kM16Chunk + ro[lo[j]] + (ev[j] - rp[lo[j]])];
#endif
    }
  };
  auto digit = [&](const Seg& s, const u32x4& r) {
    return (m16_pid<KW>(pd, r, kw0) - (s.h << kM16Lo)) & (NB - 1);
  };
  // stable rank by pid & 31 -> stage/los in sorted order; wc[0][l] = digit starts afterwards
  auto rank_stage = [&](const Seg& s, uint32_t n, const u32x4 (&r)[PT]) {
    uint32_t lo[PT], rk[PT];
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
      const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
      const bool valid = e < n;
      lo[j] = valid ? digit(s, r[j]) : 0u;
      rk[j] = wave_rank<kM16Lo>(lo[j], valid, wc + wave * NB, lt_mask);
    }
    __syncthreads();
    scan_digit_wave<NB, NW>(wc, wsum, tid, lane, wave);
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j)
      if (rk[j] != ~0u) {
        const uint32_t pos = wc[wave * NB + lo[j]] + rk[j];
        stage[pos] = r[j];
        los[pos] = (uint8_t)lo[j];
      }
  };
  auto write_index = [&](const Seg& s, uint32_t start_l) {
    const uint64_t seg_out = s.out;
    const uint32_t p = (s.h << kM16Lo) + (uint32_t)tid;  // in-segment record offset of partition p
    if (tid < (int)PB && p < (uint32_t)R) {
      const int64_t off = (int64_t)((seg_out - s.mbase + start_l) * g.rec_size);
      index[(uint64_t)s.m * (R + 1) + p] = off;
      if (ibe) ibe[(uint64_t)s.m * (R + 1) + p] = bswap64((uint64_t)off);
    }
  };
  // sorted stage -> output through the per-partition cursors; cursors advance; wc cleared
  auto place = [&](const Seg& s, uint32_t n) {
#pragma unroll
    for (uint32_t q = 0; q < PT; ++q) {
      const uint32_t i = tid + q * NT;
      if (i < n) {
        const uint32_t l = los[i];
        out4[s.mbase + cur[l] + (i - wc[l])] = stage[i];
      }
    }
    uint32_t ncur = 0;
    if (tid < (int)NB) ncur = cur[tid] + ((uint32_t)tid + 1 < NB ? wc[tid + 1] : n) - wc[tid];
    __syncthreads();
    if (tid < (int)NB) cur[tid] = ncur;
    for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
    __syncthreads();
  };

  for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
  __syncthreads();
  if (it0 >= it1) return;
  Seg s = build(it0, prefetch(it0));
  u32x4 rv[PT];
  SUX_MSD_STAMP_INIT();
  for (uint32_t it = it0; it < it1; it += G) {
    const uint32_t seg_rel = (uint32_t)(s.out - s.mbase);  // in-map record offset of the segment
    const bool multi = s.T > CAP;
    if (multi) {
      // larger than the LDS (skewed keys): count the digits first, then place piece by piece
      for (uint32_t e0 = 0; e0 < s.T; e0 += CAP) {
        load(s, e0, rv);
        const uint32_t n = min(CAP, s.T - e0);
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j) {
          const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
          if (e < n) atomicAdd(&wc[wave * NB + digit(s, rv[j])], 1u);
        }
      }
      __syncthreads();
      scan_digit_wave<NB, NW>(wc, wsum, tid, lane, wave);
      if (tid < (int)NB) cur[tid] = seg_rel + wc[tid];
      write_index(s, tid < (int)NB ? wc[tid] : 0u);
      __syncthreads();
      for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
      __syncthreads();
    }
    // one piece (the whole segment) unless multi; an empty segment still writes its index
    for (uint32_t e0 = 0; e0 == 0 || e0 < s.T; e0 += CAP) {
      load(s, e0, rv);
      SUX_MSD_STAMP(0);
      const uint32_t n = min(CAP, s.T - e0);
      rank_stage(s, n, rv);
      __syncthreads();
      SUX_MSD_STAMP(1);
      if (!multi) {
        if (tid < (int)NB) cur[tid] = seg_rel + wc[tid];
        write_index(s, tid < (int)NB ? wc[tid] : 0u);
      }
      __syncthreads();
      SUX_MSD_STAMP(2);
      place(s, n);
      SUX_MSD_STAMP(3);
    }
    if (it + G < it1) s = build(it + G, prefetch(it + G));
    SUX_MSD_STAMP(4);
  }
  SUX_MSD_STAMP_END();
}

// ------------------------------------------------------------------------------------------
// Reduce-side sort, MSD finish (sux_sort_records / sux_sort_segments): one stable digit pass
// over the top bits of the keys' varying range leaves R buckets of <= kSortLocalCap pairs
// (checked on the host); k_sort_local then sorts every bucket inside LDS by a stable LSD radix
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

template <uint32_t NW, uint32_t CAP>  // buf[CAP] u32x4 | wc[NW][256] u32 | wsum[NW]
struct SortLocal {
  static constexpr uint32_t NT = NW * kWave, PT = CAP / NT, NB = 256;
  static constexpr uint32_t lds_bytes() { return CAP * 16 + NW * NB * 4 + NW * 4; }
};

// <8 waves, 4096 pairs>: two workgroups per CU; <4 waves, 1024 pairs>: six per CU, for the
// ~600-pair buckets of a 5 M-record reduce partition
template <uint32_t NW, uint32_t CAP>
__global__ __launch_bounds__(NW * 64, NW == 8 ? 4 : CAP == 1024 ? 6 : 4) void k_sort_local(const u32x4* __restrict__ in,
                                                        u32x4* __restrict__ out,
                                                        const int64_t* __restrict__ index,
                                                        uint32_t R, SortDigits dg) {
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
    if (n == 0 || n > CAP) continue;  // (the host never passes a bucket above CAP)
    u32x4 v[PT];
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {  // unconditional (clamped) loads: no per-load wait
      const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
      v[j] = in[s0 + min(e, n - 1)];
    }
#pragma unroll 1
    for (int d = 0; d < (n > 1 ? dg.n : 0); ++d) {
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
    }
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
      const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
      if (e < n) out[s0 + e] = v[j];
    }
  }
}

// Largest bucket of an index table, in records of 16 bytes: one workgroup.
__global__ __launch_bounds__(1024) void k_index_maxdiff(const int64_t* __restrict__ index,
                                                        uint32_t R, uint64_t* __restrict__ out) {
  __shared__ unsigned long long m;
  if (threadIdx.x == 0) m = 0;
  __syncthreads();
  unsigned long long local = 0;
  for (uint32_t p = threadIdx.x; p < R; p += 1024)
    local = max(local, (unsigned long long)((index[p + 1] - index[p]) / 16));
  atomicMax(&m, local);
  __syncthreads();
  if (threadIdx.x == 0) *out = m;
}

hipError_t launch_sort_local(const void* in_pairs, void* out_pairs, const int64_t* d_index,
                             uint32_t R, const SortDigits& dg, uint64_t* d_maxbucket, bool max_only,
                             hipStream_t s) {
  if (max_only) {
    hipLaunchKernelGGL(k_index_maxdiff, dim3(1), dim3(1024), 0, s, d_index, R, d_maxbucket);
    return hipGetLastError();
  }
  const uint32_t ncu = (uint32_t)std::max(1, stream_cus(s));
  // the smallest shape holding the largest bucket (d_maxbucket carries it, host-read, in
  // SortDigits::pad)
  if (dg.pad <= 1024) {
    constexpr size_t lds = SortLocal<4, 1024>::lds_bytes();
    hipLaunchKernelGGL((k_sort_local<4, 1024>), dim3(std::min<uint32_t>(R, 6 * ncu)), dim3(4 * kWave),
                       lds, s, static_cast<const u32x4*>(in_pairs), static_cast<u32x4*>(out_pairs),
                       d_index, R, dg);
  } else if (dg.pad <= 2048) {
    constexpr size_t lds = SortLocal<4, 2048>::lds_bytes();
    static_assert(4 * lds <= 160 * 1024, "four workgroups per CU");
    hipLaunchKernelGGL((k_sort_local<4, 2048>), dim3(std::min<uint32_t>(R, 4 * ncu)), dim3(4 * kWave),
                       lds, s, static_cast<const u32x4*>(in_pairs), static_cast<u32x4*>(out_pairs),
                       d_index, R, dg);
  } else {
    constexpr size_t lds = SortLocal<8, kSortLocalCap>::lds_bytes();
    static_assert(2 * lds <= 160 * 1024, "two workgroups per CU");
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sort_local<8, kSortLocalCap>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((k_sort_local<8, kSortLocalCap>), dim3(std::min<uint32_t>(R, 2 * ncu)),
                       dim3(8 * kWave), lds, s, static_cast<const u32x4*>(in_pairs),
                       static_cast<u32x4*>(out_pairs), d_index, R, dg);
  }
  return hipGetLastError();
}

template <int KW, bool TAB>
static void launch_hist3_kw(dim3 grid, size_t lds, hipStream_t s, const PartDev& pd,
                            const MapGroup& g, uint16_t* pids, uint32_t* counts) {
  constexpr int RPL = 4;
  hipLaunchKernelGGL((k_hist3<KW, RPL, TAB>), grid, dim3(256), lds, s, pd, g, pids, counts);
}

// ------------------------------------------------------------------------------------------
// pid-only kernel (sux_partition_ids)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pids(PartDev pd, const uint8_t* recs, uint32_t rs,
                                              uint64_t n, uint16_t* pids) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * 256)
    pids[i] = (uint16_t)get_partition(pd, recs + i * rs);
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
uint32_t choose_tile_recs(uint32_t R, uint32_t rec_size, uint64_t records_per_map,
                          const Tuning& tn) {
  // 4096 records (400 KB at S=100) per tile: fewer counters to scan, and the partial 128-B
  // lines at tile seams are rarer (measured: 1024 -> 4096 takes ~1 ms off a 100 GB step)
  uint32_t t = 4096;
  while (t < 4u * R && t < (1u << 22)) t <<= 1;
  // small records, many partitions: the sorted-chunk scatter re-reads R cursors per tile
  // (32 Ki records measured best at R = 10000, profiles/r02_small_b); the two-pass scatter's
  // pass A walks whole tiles too (one tile per persistent workgroup at a time: a launch group
  // needs >> 256 tiles)
  if (small_two_pass_shape(R, rec_size) && tn.small_kernel == 2) t = 32768;
  if (small_two_pass_shape(R, rec_size) && tn.small_kernel == 3) t = 32768;
  // very long maps: longer tiles, so that a map has <= 2048 of them — k_tile_scan gives one wave
  // to each (map, partition) row of tile counts, and a 2^27-record map at 4096-record tiles has
  // 32768 per row (3.9 ms of scan per 13.4 GB launch group, profiles/r02_configs)
  while (t < (1u << 16) && (records_per_map + t - 1) / t > 2048) t <<= 1;
  const uint32_t v = (uint32_t)tn.tile_records;  // tuning override (power of two, >= 64)
  if (v >= 64 && (v & (v - 1)) == 0) t = v;
  // no point in tiles longer than a map
  uint64_t cap = ((records_per_map + kWave - 1) / kWave) * kWave;
  if (cap < t) t = (uint32_t)(cap < kWave ? kWave : cap);
  return t;
}

static uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

Workspace workspace_layout(uint32_t R, uint32_t rec_size, uint64_t records_per_map,
                           uint64_t num_records, uint32_t tile_recs, bool need_pids,
                           bool small_tmp) {
  Workspace w{};
  uint64_t maps = records_per_map ? (num_records + records_per_map - 1) / records_per_map : 0;
  if (maps == 0) maps = 1;
  uint64_t tiles = (records_per_map + tile_recs - 1) / tile_recs;
  if (tiles == 0) tiles = 1;
  uint64_t off = 0;
  w.counts_off = off;
  w.counts_bytes = align_up(maps * R * tiles * 4, 256);
  off += w.counts_bytes;
  w.totals_off = off;
  w.totals_bytes = align_up(maps * R * 8, 256);
  off += w.totals_bytes;
  w.base_off = off;
  // base [M][R] | in-map prefix [M][R] | per-(map, peer) sums [M][min(R, 1024)] (peer-major)
  w.base_bytes = align_up((2 * maps * R + maps * (R < 1024 ? R : 1024)) * 8, 256);
  off += w.base_bytes;
  w.pids_off = off;
  w.pids_bytes = need_pids ? align_up(num_records * 2, 256) : 0;
  off += w.pids_bytes;
  w.op_off = off;
  w.op_bytes = (rec_size == 100 && R <= 1024) ? onepass_sync_bytes(R) : 0;
  off += w.op_bytes;
  w.tmp_off = off;  // the two-pass small-record scatter's bucketed copy of the records
  w.tmp_bytes = small_tmp ? align_up(num_records * rec_size, 256) : 0;
  off += w.tmp_bytes;
  w.total = off;
  return w;
}

static int waves_per_group(int R) { return (R * 4 * 4 <= 64 * 1024) ? 4 : 1; }

// Dynamic LDS above 64 KiB must be opted into per kernel (gfx950 allows 160 KiB per workgroup).
static void allow_lds(const void* fn, size_t lds) {
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

template <int WPG>
static hipError_t launch_scatter(uint32_t S, dim3 grid, size_t lds, hipStream_t s, const MapGroup& g,
                                 int R, int bits, const uint16_t* pids, const uint32_t* prefix,
                                 const uint64_t* base, uint8_t* out) {
  allow_lds(reinterpret_cast<const void*>(&k_scatter<WPG, 100>), lds);
  allow_lds(reinterpret_cast<const void*>(&k_scatter<WPG, 16>), lds);
  allow_lds(reinterpret_cast<const void*>(&k_scatter<WPG, 0>), lds);
  switch (S) {
    case 100:
      hipLaunchKernelGGL((k_scatter<WPG, 100>), grid, dim3(WPG * kWave), lds, s, g, R, bits, pids,
                         prefix, base, out);
      break;
    case 16:
      hipLaunchKernelGGL((k_scatter<WPG, 16>), grid, dim3(WPG * kWave), lds, s, g, R, bits, pids,
                         prefix, base, out);
      break;
    default:
      hipLaunchKernelGGL((k_scatter<WPG, 0>), grid, dim3(WPG * kWave), lds, s, g, R, bits, pids,
                         prefix, base, out);
  }
  return hipGetLastError();
}

// The MSD small-record path (k_msd16a / k_msd16_scan / k_msd16b) applies: tuning small_kernel 4,
// 16-byte records with a fixed-width key in the first 16 bytes, 1024 < R <= 16384, 16-byte
// aligned input and output, map-major layout, maps of <= kM16MaxChunks chunks, and a workspace
// with the temp copy (its chunk-offset table lives in the counts region, the segment bases in
// the totals region).
static bool msd16_eligible(const PartDev& pd, const MapGroup& g, const LayoutDesc& lay,
                           const uint8_t* d_out, const Workspace& ws, const Tuning& tn) {
  if (tn.small_kernel != 4 || g.rec_size != 16 || lay.world != 1) return false;
  if (pd.R <= 1024 || pd.R > 16384 || pd.kind == 4 || pd.key_offset % 4 != 0 ||
      pd.key_offset + pd.key_len > 16)
    return false;
  if (((reinterpret_cast<uintptr_t>(g.recs) | reinterpret_cast<uintptr_t>(d_out)) & 15) != 0)
    return false;
  const uint64_t cpm = (g.records_per_map + kM16Chunk - 1) / kM16Chunk;
  const uint64_t nbk = ((uint64_t)pd.R + (1u << kM16Lo) - 1) >> kM16Lo;
  // by default only when a (map, bucket) segment holds >= 1024 records on average: a segment
  // costs ~6 us of run table, search and barriers whatever its size, so short maps run the
  // sorted-chunk scatter instead (64 Ki-record maps at R = 10 000: 105-record segments, 194 vs
  // 507 GB/s; 2^20-record maps: 1677-record segments, 1027 vs 750 GB/s)
  if (tn.small_auto && g.records_per_map < 1024 * nbk) return false;
  return cpm >= 1 && cpm <= kM16MaxChunks && ws.tmp_bytes >= g.num_records * 16 &&
         (uint64_t)g.num_maps * cpm * nbk * 2 <= ws.counts_bytes &&
         (uint64_t)g.num_maps * nbk * 8 <= ws.totals_bytes;
}

hipError_t launch_partition_group(const PartDev& pd, const MapGroup& g_in, const LayoutDesc& lay,
                                  uint8_t* d_out, int64_t* d_index, uint8_t* d_index_be,
                                  uint16_t* d_pids, uint8_t* d_ws, const Workspace& ws,
                                  uint64_t* d_peer_bytes, const Tuning& tn, Timer* timer,
                                  hipStream_t s) {
  MapGroup g = g_in;  // counts_tm is decided below, with the K1 / K3 pair
  g.counts_tm = 0;
  const int R = pd.R;
  const uint32_t S = g.rec_size;
  // persistent grids are sized to the CUs the stream may use (a CU-masked stream at N > 1):
  // with static work items, workgroups beyond the resident ones would start only after a
  // resident one finished ALL its items
  const uint32_t ncu = (uint32_t)std::max(1, stream_cus(s));
  // one pass (sux_onepass.hip) whenever a map batch fits on chip: every record read once
  uint32_t op_grid = 0, op_cs = 0;
  if (tn.onepass && ws.op_bytes && onepass_eligible(pd, g, lay.world, d_out, d_peer_bytes, s, &op_grid, &op_cs)) {
    timer_note(timer, kScatter, "k_onepass");
    timer_begin(timer, kScatter, s);
    const hipError_t eo = launch_onepass(pd, g, d_out, d_index, d_index_be, d_pids,
                                         d_ws + ws.op_off, op_grid, op_cs, s);
    timer_end(timer, kScatter, s);
    return eo;
  }
  const uint32_t total_tiles = g.num_maps * g.tiles_per_map;
  uint32_t* counts = reinterpret_cast<uint32_t*>(d_ws + ws.counts_off);
  uint64_t* totals = reinterpret_cast<uint64_t*>(d_ws + ws.totals_off);
  uint64_t* base = reinterpret_cast<uint64_t*>(d_ws + ws.base_off);
  uint16_t* pids = d_pids ? d_pids : reinterpret_cast<uint16_t*>(d_ws + ws.pids_off);

  // ---- small records, many partitions, map-major: the two-level path without K1 (k_msd16*)
  if (msd16_eligible(pd, g, lay, d_out, ws, tn)) {
    const uint32_t cpm = (uint32_t)((g.records_per_map + kM16Chunk - 1) / kM16Chunk);
    const uint32_t nbk = ((uint32_t)R + (1u << kM16Lo) - 1) >> kM16Lo;
    uint16_t* offs = reinterpret_cast<uint16_t*>(counts);  // [map][chunk][bucket]
    uint64_t* segbase = totals;                              // [map][bucket]
    uint8_t* tmp = d_ws + ws.tmp_off;
    const int kw = (pd.key_len + 3) / 4;
    // two 512-thread workgroups per CU in both passes: their load / rank / store phases
    // interleave (one prefetching 1024-thread workgroup measured slower: 9.4 vs 8.4 ms of
    // pass A per 17 GB step, and pass B spills; profiles/r02_sweeps/msd)
    constexpr uint32_t NWA = 8, NWB = 4, PTB = 8;
    timer_note(timer, kHist, "k_msd16a");
    timer_begin(timer, kHist, s);
    const uint32_t wpc = (uint32_t)tn.small_wgs_per_cu;
    const dim3 ga(std::min<uint32_t>(g.num_maps * cpm, ncu * wpc));
#define SUX_M16A(KW, DB)                                                                           \
  do {                                                                                             \
    constexpr size_t ldsa = M16a<NWA, DB>::lds_bytes();                                            \
    allow_lds(reinterpret_cast<const void*>(&k_msd16a<KW, NWA, DB>), ldsa);                        \
    hipLaunchKernelGGL((k_msd16a<KW, NWA, DB>), ga, dim3(NWA * kWave), ldsa, s, pd, g, cpm, nbk,   \
                       offs, d_pids, tmp);                                                         \
  } while (0)
#define SUX_M16AK(DB)                   \
  do {                                  \
    if (kw <= 1) SUX_M16A(1, DB);       \
    else if (kw == 2) SUX_M16A(2, DB);  \
    else if (kw == 3) SUX_M16A(3, DB);  \
    else SUX_M16A(4, DB);               \
  } while (0)
    if (nbk > 512) SUX_M16AK(10);
    else if (nbk > 256) SUX_M16AK(9);
    else SUX_M16AK(8);
#undef SUX_M16AK
#undef SUX_M16A
    timer_end(timer, kHist, s);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    timer_note(timer, kScan, "k_msd16_scan");
    timer_begin(timer, kScan, s);
    hipLaunchKernelGGL(k_msd16_scan, dim3(g.num_maps), dim3(kScanThreads), 0, s, g, cpm, nbk, offs,
                       segbase, d_index, d_index_be, d_peer_bytes, R);
    timer_end(timer, kScan, s);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    timer_note(timer, kScatter, "k_msd16b");
    timer_begin(timer, kScatter, s);
    // pass B's 256-thread workgroups are half the size of pass A's: twice as many per CU
    const dim3 gb(std::min<uint32_t>(g.num_maps * nbk, ncu * 2 * wpc));
    constexpr size_t ldsb = M16b<NWB, PTB>::lds_bytes();
    static_assert(4 * ldsb <= 160 * 1024, "pass B: four workgroups per CU");
    static_assert(2 * M16a<NWA, 10>::lds_bytes() <= 160 * 1024, "pass A: two workgroups per CU");
#define SUX_M16B(KW)                                                                               \
  do {                                                                                             \
    allow_lds(reinterpret_cast<const void*>(&k_msd16b<KW, NWB, PTB>), ldsb);                      \
    hipLaunchKernelGGL((k_msd16b<KW, NWB, PTB>), gb, dim3(NWB * kWave), ldsb, s, pd, g, cpm, nbk,  \
                       offs, segbase, tmp, d_out, d_index, d_index_be);                            \
  } while (0)
    if (kw <= 1) SUX_M16B(1);
    else if (kw == 2) SUX_M16B(2);
    else if (kw == 3) SUX_M16B(3);
    else SUX_M16B(4);
#undef SUX_M16B
    timer_end(timer, kScatter, s);
    return hipGetLastError();
  }
  int bits = 0;
  while ((1 << bits) < R) ++bits;
  const int wpg = waves_per_group(R);
  const dim3 grid1((total_tiles + wpg - 1) / wpg), grid4((total_tiles + 3) / 4);
  const size_t lds1 = (size_t)wpg * R * 4;

  const int sv = tn.scatter_kernel;
  const int s6c = tn.s6_chunk;
  const int s6tpw = tn.tiles_per_item;
  size_t lds6 = 0;
  int c6 = 0;
  if (sv >= 6 && S == 100 && (reinterpret_cast<uintptr_t>(d_out) & 15) == 0 &&
      g.num_records * S < kImageMaxBytes) {
    for (int c : {1024, 512, 384, 256}) {
      if (c > s6c) continue;
      const size_t b = c == 1024 ? Sc6<100, 1024, 16>::lds_bytes(R)
                     : c == 512  ? Sc6<100, 512, 8>::lds_bytes(R)
                     : c == 384  ? Sc6<100, 384, 6>::lds_bytes(R)
                                 : Sc6<100, 256, 4>::lds_bytes(R);
      if (b <= 160 * 1024) {
        c6 = c;
        lds6 = b;
        break;
      }
    }
  }
  const bool v8 = c6 == 1024 && sv >= 8 && tn.scatter_chunk == 1024 &&
                  Sc8<100, 1024, 16>::fits(R);
  const bool v7 = !v8 && c6 == 1024 && sv >= 7 && R <= 512 &&
                  Sc7<100, 1024, 16>::lds_bytes(R) <= 160 * 1024;
  // ---- K1: pids + tile histograms
  const int hv = tn.hist_kernel;
  const bool shaped = (S == 100 || S == 16) && R <= 4096;  // v2 instantiations
  const bool words = pd.kind != 4 && pd.key_offset % 4 == 0 && pd.key_len <= 16;
  // small records with many partitions: k_hist16 + tile-major counts + k_scatter16, together
  const bool s16 = hv >= 4 && sv >= 7 && words && S == 16 && R > 1024 &&
                   (reinterpret_cast<uintptr_t>(g.recs) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(d_out) & 15) == 0;
  int hist = 1;
  if (s16) hist = 16;
  else if (hv >= 4 && words && R <= 4096 && S == 100 && (pd.key_offset + pd.key_len) <= (int)S) hist = 4;
  else if (hv >= 3 && words && R <= 4096) hist = 3;
  else if (hv >= 2 && shaped) hist = 2;
  // k_hist4 feeding k_scatter7/8: tile-major counts (one contiguous store per tile; k_hist4 with
  // strided counts wrote ~2 B per record in partial-line dword stores, profiles/pmc_r02.json)
  g.counts_tm = (hist == 4 && (v8 || v7) && tn.counts_tm) ? 1u : 0u;
  timer_note(timer, kHist, hist == 16 ? "k_hist16" : hist == 4 ? "k_hist4" : hist == 3 ? "k_hist3"
                          : hist == 2 ? "k_hist2" : "k_hist");
  timer_begin(timer, kHist, s);
  if (hist == 16) {
    const size_t lds = (size_t)R * 4;
    const int kw = (pd.key_len + 3) / 4;
    const dim3 gridp(std::min<uint32_t>(total_tiles, ncu * std::max<uint32_t>(1, (160u * 1024) / (uint32_t)lds)));
#define SUX_H16(KW)                                                                        \
  do {                                                                                     \
    allow_lds(reinterpret_cast<const void*>(&k_hist16<KW>), lds);                          \
    hipLaunchKernelGGL((k_hist16<KW>), gridp, dim3(1024), lds, s, pd, g, pids, counts);     \
  } while (0)
    if (kw <= 1) SUX_H16(1);
    else if (kw == 2) SUX_H16(2);
    else if (kw == 3) SUX_H16(3);
    else SUX_H16(4);
#undef SUX_H16
  } else if (hist == 4) {
    const int hch = tn.hist_stage;
    const bool tab = pd.kind == 1 && R > 1 &&
                     Hs4<100, 128>::lds_bytes(R, true) <= 160 * 1024;
    const int kw = (pd.key_len + 3) / 4;
    (void)tab;
#define SUX_H4(CHV, KW)                                                                            \
  do {                                                                                             \
    const size_t lds = Hs4<100, CHV>::lds_bytes(R, tab);                                           \
    uint32_t per_cu = std::max<uint32_t>(1, (160u * 1024) / (uint32_t)lds);                        \
    if (tn.hist_wgs_per_cu > 0) per_cu = std::min<uint32_t>(per_cu, (uint32_t)tn.hist_wgs_per_cu); \
    const dim3 gridp(std::min<uint32_t>(total_tiles, ncu * per_cu));                              \
    if (tab && tn.hist_nt) {                                                                       \
      allow_lds(reinterpret_cast<const void*>(&k_hist4<100, CHV, KW, true, true>), lds);          \
      hipLaunchKernelGGL((k_hist4<100, CHV, KW, true, true>), gridp, dim3(256), lds, s, pd, g,     \
                         pids, counts);                                                            \
    } else if (tab) {                                                                              \
      allow_lds(reinterpret_cast<const void*>(&k_hist4<100, CHV, KW, true, false>), lds);         \
      hipLaunchKernelGGL((k_hist4<100, CHV, KW, true, false>), gridp, dim3(256), lds, s, pd, g,    \
                         pids, counts);                                                            \
    } else {                                                                                       \
      allow_lds(reinterpret_cast<const void*>(&k_hist4<100, CHV, KW, false, false>), lds);        \
      hipLaunchKernelGGL((k_hist4<100, CHV, KW, false, false>), gridp, dim3(256), lds, s, pd, g,   \
                         pids, counts);                                                            \
    }                                                                                              \
  } while (0)
#define SUX_H4K(CHV)                 \
  do {                               \
    if (kw <= 1) SUX_H4(CHV, 1);     \
    else if (kw == 2) SUX_H4(CHV, 2); \
    else if (kw == 3) SUX_H4(CHV, 3); \
    else SUX_H4(CHV, 4);             \
  } while (0)
    if (hch == 128) SUX_H4K(128);
    else SUX_H4K(64);
#undef SUX_H4K
#undef SUX_H4
  } else if (hist == 3) {
    const bool tab = pd.kind == 1 && R > 1 &&
                     (size_t)(R - 1) * 16 + (4u << kLutBits) + 2048 + 16u * R <= 64 * 1024;
    const size_t lds = (tab ? (size_t)(R - 1) * 16 + (4u << kLutBits) : 0) + 2048 + 16u * R;
    const int kw = (pd.key_len + 3) / 4;
#define SUX_H3(KW)                                                              \
  (tab ? launch_hist3_kw<KW, true>(grid4, lds, s, pd, g, pids, counts)           \
       : launch_hist3_kw<KW, false>(grid4, lds, s, pd, g, pids, counts))
    if (kw <= 1) SUX_H3(1);
    else if (kw == 2) SUX_H3(2);
    else if (kw == 3) SUX_H3(3);
    else SUX_H3(4);
#undef SUX_H3
  } else if (hist == 2) {
    const size_t lds = 4 * (size_t)(S == 100 ? hist2_wave_bytes<100, 128>(R) : hist2_wave_bytes<16, 512>(R));
    allow_lds(reinterpret_cast<const void*>(&k_hist2<100, 128>), lds);
    allow_lds(reinterpret_cast<const void*>(&k_hist2<16, 512>), lds);
    if (S == 100)
      hipLaunchKernelGGL((k_hist2<100, 128>), grid4, dim3(256), lds, s, pd, g, pids, counts);
    else
      hipLaunchKernelGGL((k_hist2<16, 512>), grid4, dim3(256), lds, s, pd, g, pids, counts);
  } else {
    allow_lds(reinterpret_cast<const void*>(&k_hist<1>), lds1);
    if (wpg == 4)
      hipLaunchKernelGGL((k_hist<4>), grid1, dim3(4 * kWave), lds1, s, pd, g, pids, counts);
    else
      hipLaunchKernelGGL((k_hist<1>), grid1, dim3(kWave), lds1, s, pd, g, pids, counts);
  }
  timer_end(timer, kHist, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;

  // ---- K2: scans -> index tables + destination bases
  timer_begin(timer, kScan, s);
  const uint32_t rows = g.num_maps * (uint32_t)R;
  if (s16 || g.counts_tm)
    hipLaunchKernelGGL(k_tile_scan_tm, dim3(g.num_maps * ((R + 15) / 16)), dim3(256), 0, s, counts,
                       totals, g.num_maps, (uint32_t)R, g.tiles_per_map);
  else if (g.tiles_per_map <= 64)
    hipLaunchKernelGGL(k_tile_scan_rows, dim3((rows + 255) / 256), dim3(256), 0, s, counts, totals,
                       rows, g.tiles_per_map);
  else
    hipLaunchKernelGGL(k_tile_scan, dim3((rows + 3) / 4), dim3(256), 0, s, counts, totals, rows,
                       g.tiles_per_map);
  const uint64_t L = (uint64_t)g.num_maps * R;
  uint64_t* pre = base + L;
  uint64_t* mh = base + 2 * L;
  hipLaunchKernelGGL(k_map_scan, dim3(g.num_maps), dim3(kScanThreads), 0, s, totals, base, pre, mh,
                     d_index, d_index_be, lay.world == 1 ? d_peer_bytes : nullptr, R, lay.world,
                     g.rec_size, g.records_per_map, g.num_records, nullptr);
  if (lay.world > 1) {
    hipLaunchKernelGGL(k_peer_off, dim3(1), dim3(kScanThreads), 0, s, mh, d_peer_bytes,
                       g.num_maps, lay.world, g.rec_size);
    hipLaunchKernelGGL(k_peer_base, dim3((uint32_t)((L + 255) / 256)), dim3(256), 0, s, pre, mh,
                       base, g.num_maps, R, lay.world);
  }
  timer_end(timer, kScan, s);
  e = hipGetLastError();
  if (e != hipSuccess) return e;

  // ---- K3: stable scatter.  S = 100 (TeraSort rows): v7 for R <= 512, v6 for the R whose
  // LDS image still fits; any other shape: the v2 (R <= 4096, S in {16, 100}) or v1 kernels.
  // tuning (Tuning): s6_chunk caps the v6 chunk, tiles_per_item sets the v6/v7 work item,
  // scatter_chunk/scatter_depth pick the v7 shape (768-record chunks leave room for a K1
  // workgroup on the CU: the co-resident pipeline)
  timer_begin(timer, kScatter, s);
  const bool two16 = s16 && small_two_pass_shape((uint32_t)R, S) && tn.small_kernel == 3 &&
                     ws.tmp_bytes >= g.num_records * 16;
  const bool sorted16 = s16 && R <= kS16sMaxR && tn.small_kernel != 1;
  if (two16) {
    timer_note(timer, kScatter, "k_bucket16a+k_bucket16b");
    uint8_t* tmp = d_ws + ws.tmp_off;
    const uint32_t items = g.num_maps * (((uint32_t)R + B16b<8>::NB - 1) / B16b<8>::NB);
    const int kw = (pd.key_len + 3) / 4;
    // wave count per workgroup: 8 = two 512-thread workgroups per CU (their phases interleave),
    // 16 = one 1024-thread workgroup (tuning small_waves; default 8)
    const bool w16 = tn.small_waves == 16;
#define SUX_B16(NWV)                                                                             \
  do {                                                                                           \
    allow_lds(reinterpret_cast<const void*>(&k_bucket16a<NWV>), B16a<NWV>::lds_bytes());         \
    hipLaunchKernelGGL((k_bucket16a<NWV>), dim3(std::min<uint32_t>(total_tiles, ncu * (16 / NWV))), \
                       dim3(NWV * kWave), B16a<NWV>::lds_bytes(), s, g, R, pids, counts, base, tmp); \
    const dim3 gridb(std::min<uint32_t>(items, ncu * (16 / NWV)));                              \
    if (kw <= 1) SUX_B16B(1, NWV);                                                               \
    else if (kw == 2) SUX_B16B(2, NWV);                                                          \
    else if (kw == 3) SUX_B16B(3, NWV);                                                          \
    else SUX_B16B(4, NWV);                                                                       \
  } while (0)
#define SUX_B16B(KW, NWV)                                                                        \
  do {                                                                                           \
    allow_lds(reinterpret_cast<const void*>(&k_bucket16b<KW, NWV>), B16b<NWV>::lds_bytes());     \
    hipLaunchKernelGGL((k_bucket16b<KW, NWV>), gridb, dim3(NWV * kWave), B16b<NWV>::lds_bytes(), \
                       s, pd, g, base, totals, tmp, d_out);                                      \
  } while (0)
    if (w16) SUX_B16(16);
    else SUX_B16(8);
#undef SUX_B16
#undef SUX_B16B
    e = hipGetLastError();
  } else if (sorted16) {
    timer_note(timer, kScatter, "k_scatter16s");
    const size_t lds = Sc16s::lds_bytes(R);
    allow_lds(reinterpret_cast<const void*>(&k_scatter16s), lds);
    const dim3 grid(std::min<uint32_t>(total_tiles, ncu));  // one LDS-bound workgroup per CU
    hipLaunchKernelGGL(k_scatter16s, grid, dim3(1024), lds, s, g, R, bits, pids, counts, base,
                       d_out);
    e = hipGetLastError();
  } else if (s16) {
    timer_note(timer, kScatter, "k_scatter16b");
    const size_t lds = (size_t)R * 4;
    const uint32_t per_cu = std::max<uint32_t>(1, std::min<uint32_t>(2, (160u * 1024) / (uint32_t)lds));
    const dim3 grid(std::min<uint32_t>(total_tiles, ncu * per_cu));
    const int gb = tn.small_groups;  // groups per turn (1 = k_scatter16)
    if (gb == 2 || gb == 4) {
      const void* kf = gb == 2 ? reinterpret_cast<const void*>(&k_scatter16b<16, 2>)
                               : reinterpret_cast<const void*>(&k_scatter16b<16, 4>);
      allow_lds(kf, lds);
      if (gb == 2)
        hipLaunchKernelGGL((k_scatter16b<16, 2>), grid, dim3(1024), lds, s, g, R, bits, pids,
                           counts, base, d_out);
      else
        hipLaunchKernelGGL((k_scatter16b<16, 4>), grid, dim3(1024), lds, s, g, R, bits, pids,
                           counts, base, d_out);
    } else {
      allow_lds(reinterpret_cast<const void*>(&k_scatter16<16>), lds);
      hipLaunchKernelGGL((k_scatter16<16>), grid, dim3(1024), lds, s, g, R, bits, pids, counts,
                         base, d_out);
    }
    e = hipGetLastError();
  } else if (v8) {
    timer_note(timer, kScatter, "k_scatter8");
    // one contiguous, balanced tile range per workgroup (k_scatter8), one workgroup per CU
    const dim3 grid(std::min<uint32_t>(g.num_maps * g.tiles_per_map, ncu));
    const size_t lds8b = Sc8<100, 1024, 16>::lds_bytes(R);
    const bool wm = tn.scatter_counters != 1;
    allow_lds(reinterpret_cast<const void*>(&k_scatter8<100, 1024, 16, true>), lds8b);
    allow_lds(reinterpret_cast<const void*>(&k_scatter8<100, 1024, 16, false>), lds8b);
    // tile order: contiguous ranges (default; scatter_order 1) or block-cyclic inside an XCD's
    // workgroups (2: 2^27-record maps 49.7 -> 50.3 ms, 2^20 42.9 -> 46.3, profiles/r02_m27_b)
    const uint32_t tiles_per_wg = (g.num_maps * g.tiles_per_map + grid.x - 1) / grid.x;
    (void)tiles_per_wg;  // block-cyclic measured slower for 2^20 and 2^27-record maps alike
    const bool cyc = tn.scatter_order == 2;
    const uint32_t per_xcd = std::max<uint32_t>(1, grid.x / 8);
    // a launch group whose output passes ~4 GB (one 2^27-record map is 13.4 GB) is scattered in
    // tile windows, one launch each: at any time the grid then writes into a quarter of every
    // partition's region instead of spreading its 256 x R write streams over the whole output
    const uint32_t T = g.num_maps * g.tiles_per_map;
    const uint64_t out_bytes = g.num_records * (uint64_t)S;
    const uint32_t nwin = cyc ? 1u : (uint32_t)std::min<uint64_t>(
                                        std::max<uint64_t>(1, (out_bytes + (4ull << 30) - 1) >> 32), T);
    for (uint32_t w = 0; w < nwin; ++w) {
      const uint32_t tw0 = (uint32_t)((uint64_t)T * w / nwin), tw1 = (uint32_t)((uint64_t)T * (w + 1) / nwin);
      const dim3 gw(std::min<uint32_t>(tw1 - tw0, ncu));
      if (wm)
        hipLaunchKernelGGL((k_scatter8<100, 1024, 16, true>), gw, dim3(1024), lds8b, s, g, R, bits,
                           pids, counts, base, d_out, cyc ? per_xcd : 0u, tw0, tw1);
      else
        hipLaunchKernelGGL((k_scatter8<100, 1024, 16, false>), gw, dim3(1024), lds8b, s, g, R, bits,
                           pids, counts, base, d_out, cyc ? per_xcd : 0u, tw0, tw1);
    }
    e = hipGetLastError();
  } else if (v7) {
    timer_note(timer, kScatter, "k_scatter7");
    uint32_t tpw = s6tpw > 0 ? (uint32_t)s6tpw
                             : (uint32_t)std::max<uint64_t>(1, (8ull * 1024 + g.tile_recs - 1) / g.tile_recs);
    if (tpw > g.tiles_per_map) tpw = g.tiles_per_map;
    const uint32_t wpm = (g.tiles_per_map + tpw - 1) / tpw;
    // persistent: the workgroups the LDS allows per CU (one 1024-thread workgroup at 1024-record
    // chunks; 512-record chunks of 512 threads fit twice at small R) walk the items
    const uint32_t per_cu = tn.scatter_chunk == 512
        ? std::max<uint32_t>(1, std::min<uint32_t>(2, (160u * 1024) / (uint32_t)Sc7<100, 512, 8>::lds_bytes(R)))
        : 1u;
    const dim3 grid((uint32_t)std::min<uint64_t>((uint64_t)g.num_maps * wpm, ncu * per_cu));
#define SUX_S7L(CC, NWV, DV)                                                                     \
  do {                                                                                          \
    const size_t lds7 = Sc7<100, CC, NWV>::lds_bytes(R);                                        \
    allow_lds(reinterpret_cast<const void*>(&k_scatter7<100, CC, NWV, DV>), lds7);              \
    hipLaunchKernelGGL((k_scatter7<100, CC, NWV, DV>), grid, dim3(NWV * kWave), lds7, s, g, R,   \
                       bits, pids, counts, base, d_out, tpw, wpm);                               \
  } while (0)
    if (tn.scatter_chunk == 512) SUX_S7L(512, 8, 1);
    else if (tn.scatter_chunk == 768 && tn.scatter_depth == 2) SUX_S7L(768, 12, 2);
    else if (tn.scatter_chunk == 768) SUX_S7L(768, 12, 1);
    else SUX_S7L(1024, 16, 1);
#undef SUX_S7L
    e = hipGetLastError();
  } else if (c6) {
    timer_note(timer, kScatter, "k_scatter6");
    uint32_t tpw = s6tpw > 0 ? (uint32_t)s6tpw
                             : (uint32_t)std::max<uint64_t>(1, (8ull * c6 + g.tile_recs - 1) / g.tile_recs);
    if (tpw > g.tiles_per_map) tpw = g.tiles_per_map;
    const uint32_t wpm = (g.tiles_per_map + tpw - 1) / tpw;
    const dim3 grid((uint32_t)(g.num_maps * wpm));
#define SUX_S6L(CC, NWV)                                                                         \
  do {                                                                                          \
    allow_lds(reinterpret_cast<const void*>(&k_scatter6<100, CC, NWV>), lds6);                  \
    hipLaunchKernelGGL((k_scatter6<100, CC, NWV>), grid, dim3(NWV * kWave), lds6, s, g, R, bits, \
                       pids, counts, base, d_out, tpw, wpm);                                     \
  } while (0)
    if (c6 == 1024) SUX_S6L(1024, 16);
    else if (c6 == 512) SUX_S6L(512, 8);
    else if (c6 == 384) SUX_S6L(384, 6);
    else SUX_S6L(256, 4);
#undef SUX_S6L
    e = hipGetLastError();
  } else if (sv >= 2 && shaped) {
    timer_note(timer, kScatter, "k_scatter2");
    const size_t lds = 4 * (size_t)(S == 100 ? scatter2_wave_bytes<100, 128>(R)
                                             : scatter2_wave_bytes<16, 512>(R));
    allow_lds(reinterpret_cast<const void*>(&k_scatter2<100, 128>), lds);
    allow_lds(reinterpret_cast<const void*>(&k_scatter2<16, 512>), lds);
    if (S == 100)
      hipLaunchKernelGGL((k_scatter2<100, 128>), grid4, dim3(256), lds, s, g, R, bits, pids,
                         counts, base, d_out);
    else
      hipLaunchKernelGGL((k_scatter2<16, 512>), grid4, dim3(256), lds, s, g, R, bits, pids,
                         counts, base, d_out);
    e = hipGetLastError();
  } else if (wpg == 4) {
    timer_note(timer, kScatter, "k_scatter");
    e = launch_scatter<4>(S, grid1, lds1, s, g, R, bits, pids, counts, base, d_out);
  } else {
    timer_note(timer, kScatter, "k_scatter");
    e = launch_scatter<1>(S, grid1, lds1, s, g, R, bits, pids, counts, base, d_out);
  }
  timer_end(timer, kScatter, s);
  return e;
}

hipError_t launch_partition_ids(const PartDev& pd, const uint8_t* recs, uint32_t rec_size,
                                uint64_t n, uint16_t* d_pids, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_pids, dim3((uint32_t)blocks), dim3(256), 0, s, pd, recs, rec_size, n,
                     d_pids);
  return hipGetLastError();
}

hipError_t launch_varlen_map_scan(const VarGroup& g, int R, const uint64_t* totals, uint64_t* base,
                                  int64_t* d_index, uint8_t* d_index_be, hipStream_t s) {
  const uint64_t L = (uint64_t)g.num_maps * R;
  hipLaunchKernelGGL(k_map_scan, dim3(g.num_maps), dim3(kScanThreads), 0, s, totals, base,
                     base + L, base + 2 * L, d_index, d_index_be, nullptr, R, 1, 1u,
                     g.records_per_map, g.num_records, g.offs);
  return hipGetLastError();
}

// Index tables from per-(map, partition) byte sizes (sux_lz4.hip's compressed runs).
hipError_t launch_rows_index(const uint64_t* sizes, uint32_t maps, uint32_t R, uint64_t* base,
                             int64_t* d_index, uint8_t* d_index_be, hipStream_t s) {
  const uint64_t L = (uint64_t)maps * R;
  hipLaunchKernelGGL(k_map_scan, dim3(maps), dim3(kScanThreads), 0, s, sizes, base, base + L,
                     base + 2 * L, d_index, d_index_be, nullptr, (int)R, 1, 1u, 0ull, 0ull,
                     nullptr);
  return hipGetLastError();
}

}  // namespace sux
