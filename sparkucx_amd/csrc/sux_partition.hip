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
// Other shapes: k_scatter7 (R <= 512) and k_scatter6 (R up to the LDS image) for 100-byte
// records; k_hist3 / k_hist + k_scatter (v1) for any record size; 16-byte records with R > 1024
// go to sux_small.hip.
//
// Stability: records are visited in input order (waves in order inside a chunk, chunks in order
// inside a tile range, tile ranges ordered by the partition-major tile prefix); equal pids inside
// 64 lanes are ranked by a ballot match.  So records keep input order inside a partition, as
// Spark's writers do (P2).
#include "sux_part.h"

namespace sux {

// geometry (TileRange, tile_range), scans (wave_incl_scan, block_excl_scan) and the P1
// partition functions: sux_part.h / sux_p1.h

// ------------------------------------------------------------------------------------------
// K1: partition ids + per-tile histogram
// ------------------------------------------------------------------------------------------
template <int WPG>
__global__ __launch_bounds__(WPG * kWave) void k_hist(PartDev pd, MapGroup g, uint16_t* pids,
                                                      uint32_t* counts) {
  resolve_seed(pd);
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
                                                           const uint64_t* __restrict__ map_offs,
                                                           const int32_t* __restrict__ own) {
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
        atomicAdd(&hs[owner_of((uint32_t)p, R, G, own)], (unsigned long long)v);
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
                                                   int G, const int32_t* __restrict__ own) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= (uint64_t)M * R) return;
  const uint64_t m = j / R;
  const uint32_t p = (uint32_t)(j - m * R);
  const uint32_t h = owner_of(p, R, G, own);
  const uint32_t lo = owner_lo_of(h, R, G, own);
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
// v3 hist: register streaming.  Each lane loads the key dwords of RPL records straight to
// registers (all loads issued before the first use), the range table (bounds + 10-bit prefix
// LUT) lives in LDS so no dependent global load stalls the stream, and workgroups are mapped
// XCD-contiguously (T1) so neighbouring tiles share an L2.
// ------------------------------------------------------------------------------------------

// range_search_t, partition_words, KeyVec: sux_p1.h

template <int KW, int RPL, bool TAB>
__global__ __launch_bounds__(256) void k_hist3(PartDev pd, MapGroup g, uint16_t* __restrict__ pids,
                                               uint32_t* __restrict__ counts) {
  resolve_seed(pd);
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
  // stage[4] | bounds 2(R-1) u64 | lut | hist[4][R] u32 | pid line[4][CH] u16
  static __host__ __device__ constexpr uint32_t lds_bytes(int R, bool tab) {
    return 4 * kStage + (tab ? (uint32_t)(R - 1) * 16 + (4u << kLutBits) : 0u) + 16u * R + 8 * CH;
  }
};

// PK: the pids of a full chunk leave as 16-byte stores of 8 pids (through a wave LDS line),
// chosen by the host when every chunk a wave's steady-state loop handles starts 16-B aligned
// (aligned pid array, maps and tiles multiples of 8 records).  Lane-wise 2-byte stores wrote
// 4.1 B per record (PMC, profiles/pmc_r02.json), the packed ones the 2 B of the pids.
template <uint32_t S, uint32_t CH, int KW, bool TAB, bool NTL, bool PK>
__global__ __launch_bounds__(256) void k_hist4(PartDev pd, MapGroup g, uint16_t* __restrict__ pids,
                                               uint32_t* __restrict__ counts) {
  resolve_seed(pd);
  using H = Hs4<S, CH>;
  constexpr uint32_t PER = H::kPer;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const int R = pd.R;
  const int nb = TAB ? 2 * (R - 1) : 0;
  u32x4* stage_all = reinterpret_cast<u32x4*>(lds8);
  uint64_t* sb = reinterpret_cast<uint64_t*>(lds8 + 4 * H::kStage);
  uint32_t* slut = reinterpret_cast<uint32_t*>(sb + nb);
  uint32_t* hist_all = slut + (TAB ? (1 << kLutBits) : 0);
  uint16_t* pline_all = reinterpret_cast<uint16_t*>(hist_all + 4 * R);  // 16-B aligned
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
  uint16_t* pline = pline_all + wave * CH;
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
  // record's), so a step issues a fixed set of memory instructions.  pk (compile-time): the
  // chunk is full and 16-B aligned, its pids leave packed.
  auto step = [&](uint64_t c0, u32x4 (&v)[PER], bool next, auto pk) {
    constexpr bool packed = decltype(pk)::value;
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
      if constexpr (packed) pline[r] = (uint16_t)p;
      else pids[c0 + rr] = (uint16_t)p;
    }
    __builtin_amdgcn_wave_barrier();
    if constexpr (packed) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      // every lane stores (lanes past CH / 8 repeat a lower lane's unit: same bytes, same
      // address), so no branch makes the compiler's vmcnt for the prefetched chunk conservative
      const uint32_t u = (uint32_t)lane % (CH / 8);
      reinterpret_cast<u32x4*>(pids + c0)[u] = reinterpret_cast<const u32x4*>(pline)[u];
      __builtin_amdgcn_wave_barrier();
    }
  };
  using Packed = std::integral_constant<bool, PK>;
  using Lanes = std::integral_constant<bool, false>;

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
      for (; i + 3 < nch; i += 2) {  // full chunks
        step(wb + (uint64_t)i * CH, va, true, Packed{});
        step(wb + (uint64_t)(i + 1) * CH, vb, true, Packed{});
      }
      // tail: 2 or 3 chunks left (the third is loaded into va by the first tail step); the
      // first is full
      step(wb + (uint64_t)i * CH, va, i + 2 < nch, Packed{});
      step(wb + (uint64_t)(i + 1) * CH, vb, false, Lanes{});
      if (i + 2 < nch) step(wb + (uint64_t)(i + 2) * CH, va, false, Lanes{});
    } else if (nch > 0) {
      issue(wb, va);
      if (nch > 1) issue(wb + CH, vb);
      step(wb, va, nch > 2, Lanes{});
      if (nch > 1) step(wb + CH, vb, false, Lanes{});
      if (nch > 2) step(wb + 2 * CH, va, false, Lanes{});
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

template <uint32_t S, uint32_t C, uint32_t NW, bool WM, int NTMODE = 0>
__global__ __launch_bounds__(NW * 64) void k_scatter8(MapGroup g, int R, int pid_bits,
                                                     const uint16_t* __restrict__ pids,
                                                     const uint32_t* __restrict__ prefix,
                                                     const uint64_t* __restrict__ base,
                                                     uint8_t* __restrict__ out, uint32_t cyc,
                                                     uint32_t tw0, uint32_t tw1) {
  using K = Sc8<S, C, NW>;
  constexpr uint32_t NT = K::NT, W = K::W, RPW = K::RPW, NG = K::NG, PER = K::kPer;
  constexpr uint32_t RM = 208;  // K's RMAX: the tables' compile-time stride
  constexpr int NTM = NTMODE;   // non-temporal: bit 0 record loads, bit 1 line stores
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
    for (uint32_t k2 = 0; k2 < PER; ++k2) {
      const u32x4* a4 = &src[min(tid + k2 * NT, units - 1)];
      v[k2] = (NTM & 1) ? __builtin_nontemporal_load(a4) : *a4;  // streamed once
    }
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
        // two ds_write2_b32 (4-byte-aligned units); four lane-rotated ds_write_b32 that cover
        // all 64 banks measured slower (round 4)
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
        if (NTM & 2)
          __builtin_nontemporal_store(x, &out4[A]);  // whole lines, never read back here
        else
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
  // (32 Ki records measured best at R = 10000, profiles/r02_small_b)
  if (small_two_pass_shape(R, rec_size) && tn.small_kernel == 2) t = 32768;
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
  w.tmp_off = off;  // the two-level small-record path's chunk-sorted copy of the records
  w.tmp_bytes = small_tmp ? align_up(num_records * rec_size, 256) : 0;
  off += w.tmp_bytes;
  w.total = off;
  return w;
}

static int waves_per_group(int R) { return (R * 4 * 4 <= 64 * 1024) ? 4 : 1; }

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

hipError_t launch_partition_group(const PartDev& pd, const MapGroup& g_in, const LayoutDesc& lay,
                                  uint8_t* d_out, int64_t* d_index, uint8_t* d_index_be,
                                  uint16_t* d_pids, uint8_t* d_ws, const Workspace& ws,
                                  uint64_t* d_peer_bytes, const Tuning& tn, Timer* timer,
                                  hipStream_t s, hipStream_t s_k1, hipEvent_t k1_done) {
  MapGroup g = g_in;  // counts_tm is decided below, with the K1 / K3 pair
  g.counts_tm = 0;
  const int R = pd.R;
  const uint32_t S = g.rec_size;
  // persistent grids are sized to the CUs the stream may use (a CU-masked stream at N > 1):
  // with static work items, workgroups beyond the resident ones would start only after a
  // resident one finished ALL its items
  const uint32_t ncu = (uint32_t)std::max(1, stream_cus(s));
  const hipStream_t s_main = s;
  const uint32_t ncu_main = ncu;
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
  if (msd16_eligible(pd, g, lay, d_out, ws, tn))
    return launch_msd16(pd, g, d_out, d_index, d_index_be, d_pids, d_ws, ws, d_peer_bytes, tn,
                        timer, s);
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
  const bool words = pd.kind != 4 && pd.key_offset % 4 == 0 && pd.key_len <= 16;
  // 16-byte records, R >= 256: k_hist16 + tile-major counts + k_scatter16s / k_scatter16b (sux_small.hip)
  const bool s16 = hv >= 4 && sv >= 7 && words && S == 16 && R >= 256 &&
                   (reinterpret_cast<uintptr_t>(g.recs) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(d_out) & 15) == 0;
  int hist = 1;
  if (s16) hist = 16;
  else if (hv >= 4 && words && R <= 4096 && S == 100 && (pd.key_offset + pd.key_len) <= (int)S) hist = 4;
  else if (hv >= 3 && words && R <= 4096) hist = 3;
  // k_hist4 feeding k_scatter7/8: tile-major counts (one contiguous store per tile; k_hist4 with
  // strided counts wrote ~2 B per record in partial-line dword stores, profiles/pmc_r02.json)
  g.counts_tm = (hist == 4 && (v8 || v7) && tn.counts_tm) ? 1u : 0u;
  timer_note(timer, kHist, hist == 16 ? "k_hist16" : hist == 4 ? "k_hist4" : hist == 3 ? "k_hist3"
                                                                               : "k_hist");
  hipError_t e = hipSuccess;
  {
  // K1 on its own stream when given one (sux_partition_maps_pipelined's split mode: K1 of group
  // g on a few CUs beside group g - 1's K3 on the others); K2 and K3 wait for it on s
  hipStream_t s = s_k1 ? s_k1 : s_main;
  const uint32_t ncu = s_k1 ? (uint32_t)std::max(1, stream_cus(s_k1)) : ncu_main;
  timer_begin(timer, kHist, s);
  if (hist == 16) {
    e = launch_hist16(pd, g, pids, counts, s);
  } else if (hist == 4) {
    const int hch = tn.hist_stage;
    const bool tab = pd.kind == 1 && R > 1 &&
                     Hs4<100, 128>::lds_bytes(R, true) <= 160 * 1024;
    const int kw = (pd.key_len + 3) / 4;
    // packed pid stores: every full chunk of a wave's loop starts 16-B aligned in the pid array
    const bool pk = (reinterpret_cast<uintptr_t>(pids) & 15) == 0 && g.records_per_map % 8 == 0 &&
                    g.tile_recs % 32 == 0;
#define SUX_H4V(CHV, KW, TV, NV, PV)                                                               \
  do {                                                                                             \
    allow_lds(reinterpret_cast<const void*>(&k_hist4<100, CHV, KW, TV, NV, PV>), lds);             \
    hipLaunchKernelGGL((k_hist4<100, CHV, KW, TV, NV, PV>), gridp, dim3(256), lds, s, pd, g, pids,  \
                       counts);                                                                    \
  } while (0)
#define SUX_H4(CHV, KW)                                                                            \
  do {                                                                                             \
    const size_t lds = Hs4<100, CHV>::lds_bytes(R, tab);                                           \
    uint32_t per_cu = std::max<uint32_t>(1, (160u * 1024) / (uint32_t)lds);                        \
    if (tn.hist_wgs_per_cu > 0) per_cu = std::min<uint32_t>(per_cu, (uint32_t)tn.hist_wgs_per_cu); \
    const dim3 gridp(std::min<uint32_t>(total_tiles, ncu * per_cu));                              \
    if (tab && tn.hist_nt) {                                                                       \
      if (pk) SUX_H4V(CHV, KW, true, true, true);                                                  \
      else SUX_H4V(CHV, KW, true, true, false);                                                    \
    } else if (tab) {                                                                              \
      if (pk) SUX_H4V(CHV, KW, true, false, true);                                                 \
      else SUX_H4V(CHV, KW, true, false, false);                                                   \
    } else {                                                                                       \
      if (pk) SUX_H4V(CHV, KW, false, false, true);                                                \
      else SUX_H4V(CHV, KW, false, false, false);                                                  \
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
#undef SUX_H4V
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
  } else {
    allow_lds(reinterpret_cast<const void*>(&k_hist<1>), lds1);
    if (wpg == 4)
      hipLaunchKernelGGL((k_hist<4>), grid1, dim3(4 * kWave), lds1, s, pd, g, pids, counts);
    else
      hipLaunchKernelGGL((k_hist<1>), grid1, dim3(kWave), lds1, s, pd, g, pids, counts);
  }
  timer_end(timer, kHist, s);
  }
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (s_k1) {
    e = hipEventRecord(k1_done, s_k1);
    if (e == hipSuccess) e = hipStreamWaitEvent(s_main, k1_done, 0);
    if (e != hipSuccess) return e;
  }

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
                     g.rec_size, g.records_per_map, g.num_records, nullptr, lay.own);
  if (lay.world > 1) {
    hipLaunchKernelGGL(k_peer_off, dim3(1), dim3(kScanThreads), 0, s, mh, d_peer_bytes,
                       g.num_maps, lay.world, g.rec_size);
    hipLaunchKernelGGL(k_peer_base, dim3((uint32_t)((L + 255) / 256)), dim3(256), 0, s, pre, mh,
                       base, g.num_maps, R, lay.world, lay.own);
  }
  timer_end(timer, kScan, s);
  e = hipGetLastError();
  if (e != hipSuccess) return e;

  // ---- K3: stable scatter.  S = 100 (TeraSort rows): v8 for R <= 208, v7 for R <= 512, v6 for
  // the R whose LDS image still fits; 16-byte rows with R > 1024: sux_small.hip; any other
  // shape: the v1 kernel.
  // tuning (Tuning): s6_chunk caps the v6 chunk, tiles_per_item sets the v6/v7 work item,
  // scatter_chunk/scatter_depth pick the v7 shape (768-record chunks leave room for a K1
  // workgroup on the CU: the co-resident pipeline)
  timer_begin(timer, kScatter, s);
  if (s16) {
    e = launch_scatter16(g, R, bits, pids, counts, base, d_out, tn, timer, s);
  } else if (v8) {
    timer_note(timer, kScatter, "k_scatter8");
    // one contiguous, balanced tile range per workgroup (k_scatter8), one workgroup per CU
    const dim3 grid(std::min<uint32_t>(g.num_maps * g.tiles_per_map, ncu));
    const size_t lds8b = Sc8<100, 1024, 16>::lds_bytes(R);
    const bool wm = tn.scatter_counters != 1;
    allow_lds(reinterpret_cast<const void*>(&k_scatter8<100, 1024, 16, true>), lds8b);
    allow_lds(reinterpret_cast<const void*>(&k_scatter8<100, 1024, 16, false>), lds8b);
    allow_lds(reinterpret_cast<const void*>(&k_scatter8<100, 1024, 16, true, 1>), lds8b);
    allow_lds(reinterpret_cast<const void*>(&k_scatter8<100, 1024, 16, true, 2>), lds8b);
    allow_lds(reinterpret_cast<const void*>(&k_scatter8<100, 1024, 16, true, 3>), lds8b);
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
      const uint32_t cy = cyc ? per_xcd : 0u;
      if (wm && tn.scatter_nt == 1)
        hipLaunchKernelGGL((k_scatter8<100, 1024, 16, true, 1>), gw, dim3(1024), lds8b, s, g, R,
                           bits, pids, counts, base, d_out, cy, tw0, tw1);
      else if (wm && tn.scatter_nt == 2)
        hipLaunchKernelGGL((k_scatter8<100, 1024, 16, true, 2>), gw, dim3(1024), lds8b, s, g, R,
                           bits, pids, counts, base, d_out, cy, tw0, tw1);
      else if (wm && tn.scatter_nt == 3)
        hipLaunchKernelGGL((k_scatter8<100, 1024, 16, true, 3>), gw, dim3(1024), lds8b, s, g, R,
                           bits, pids, counts, base, d_out, cy, tw0, tw1);
      else if (wm)
        hipLaunchKernelGGL((k_scatter8<100, 1024, 16, true>), gw, dim3(1024), lds8b, s, g, R, bits,
                           pids, counts, base, d_out, cy, tw0, tw1);
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
                     g.records_per_map, g.num_records, g.offs, nullptr);
  return hipGetLastError();
}

// Index tables from per-(map, partition) byte sizes (sux_lz4.hip's compressed runs).
hipError_t launch_rows_index(const uint64_t* sizes, uint32_t maps, uint32_t R, uint64_t* base,
                             int64_t* d_index, uint8_t* d_index_be, hipStream_t s) {
  const uint64_t L = (uint64_t)maps * R;
  hipLaunchKernelGGL(k_map_scan, dim3(maps), dim3(kScanThreads), 0, s, sizes, base, base + L,
                     base + 2 * L, d_index, d_index_be, nullptr, (int)R, 1, 1u, 0ull, 0ull,
                     nullptr, nullptr);
  return hipGetLastError();
}

}  // namespace sux
