// sux_varlen.hip — variable-length records on the map side: Spark SQL's
// UnsafeRowSerializer writes every row as a 4-byte big-endian length L and the L bytes of the
// UnsafeRow [ext]; rows differ in size, so partitions are measured in BYTES, not records.
// Record i = data[offs[i] - offs[0], offs[i+1] - offs[0]); maps are runs of records_per_map
// records and map m's data file occupies the same byte range of the output as its input.
//   k_vhist     one wave per tile of records: pid (P1) from the key inside the row, pid store,
//               per-wave LDS byte histogram -> counts[m][p][t] (bytes, partition-major)
//   (k_tile_scan + k_map_scan with the map byte starts: index = byte offsets, bases in bytes)
//   k_vscatter  one wave per tile, records in input order 64 at a time: ballot-match ranks,
//               each record's byte offset = its partition's cursor + the sizes of its lower
//               peers; every lane then copies its own row (16-byte pieces, 4-byte aligned).
// Stable like the fixed-size path: tiles in order, records in order inside a tile.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "sux_internal.h"

namespace sux {

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
constexpr int kVWave = 64;

#include "sux_p1.h"

template <int WPG>
__global__ __launch_bounds__(WPG * kVWave) void k_vhist(PartDev pd, VarGroup g,
                                                       const uint16_t* __restrict__ pids_in,
                                                       uint16_t* __restrict__ pids,
                                                       uint64_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int wave = threadIdx.x / kVWave, lane = threadIdx.x % kVWave;
  const uint32_t gtile = blockIdx.x * WPG + wave;
  const int R = pd.R;
  uint32_t* hist = lds + wave * R;
  for (int p = lane; p < R; p += kVWave) hist[p] = 0;
  __builtin_amdgcn_wave_barrier();
  if (gtile >= g.num_maps * g.tiles_per_map) return;
  const uint32_t map = gtile / g.tiles_per_map, tile = gtile - map * g.tiles_per_map;
  const uint64_t mb = (uint64_t)map * g.records_per_map;
  const uint64_t me = min(mb + g.records_per_map, g.num_records);
  const uint64_t tb = min(mb + (uint64_t)tile * g.tile_recs, me);
  const uint64_t te = min(tb + g.tile_recs, me);
  const uint64_t o0 = g.offs[0];
  for (uint64_t i = tb + lane; i < te; i += kVWave) {
    const uint64_t a = g.offs[i] - o0, b = g.offs[i + 1] - o0;
    int p;
    if (pids_in) {
      p = min((int)pids_in[i], R - 1);  // caller's ids (Spark SQL's projected partition ids)
    } else {
      p = get_partition(pd, g.data + a);
      pids[i] = (uint16_t)p;
    }
    atomicAdd(&hist[p], (uint32_t)(b - a));
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint64_t* dst = counts + ((uint64_t)map * R) * g.tiles_per_map + tile;
  for (int p = lane; p < R; p += kVWave) dst[(uint64_t)p * g.tiles_per_map] = hist[p];
}

template <int WPG>
__global__ __launch_bounds__(WPG * kVWave) void k_vscatter(VarGroup g, int R, int pid_bits,
                                                          const uint16_t* __restrict__ pids,
                                                          const uint64_t* __restrict__ prefix,
                                                          const uint64_t* __restrict__ base,
                                                          uint8_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint64_t curs[];
  const int wave = threadIdx.x / kVWave, lane = threadIdx.x % kVWave;
  const uint32_t gtile = blockIdx.x * WPG + wave;
  if (gtile >= g.num_maps * g.tiles_per_map) return;
  uint64_t* cur = curs + (uint64_t)wave * R;
  const uint32_t map = gtile / g.tiles_per_map, tile = gtile - map * g.tiles_per_map;
  const uint64_t mb = (uint64_t)map * g.records_per_map;
  const uint64_t me = min(mb + g.records_per_map, g.num_records);
  const uint64_t tb = min(mb + (uint64_t)tile * g.tile_recs, me);
  const uint64_t te = min(tb + g.tile_recs, me);
  const uint64_t* bm = base + (uint64_t)map * R;
  const uint64_t* pm = prefix + (uint64_t)map * R * g.tiles_per_map + tile;
  for (int p = lane; p < R; p += kVWave) cur[p] = bm[p] + pm[(uint64_t)p * g.tiles_per_map];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const uint64_t o0 = g.offs[0];
  for (uint64_t i0 = tb; i0 < te; i0 += kVWave) {
    const uint64_t i = i0 + lane;
    const bool valid = i < te;
    uint64_t a = 0, len = 0;
    uint32_t pid = 0;
    if (valid) {
      a = g.offs[i] - o0;
      len = g.offs[i + 1] - o0 - a;
      pid = min((int)pids[i], R - 1);
    }
    uint64_t peers = __ballot(valid);
    for (int bb = 0; bb < pid_bits; ++bb) {
      const bool bit = (pid >> bb) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    if (!valid) peers = 0;
    // bytes of the lower peers (this record's offset in its partition's run of this group) and
    // of all peers (the leader advances the cursor by it)
    uint64_t below = 0, all = 0;
    for (int j = 0; j < kVWave; ++j) {
      const uint64_t lj = __shfl(len, j, kVWave);
      const bool pj = (peers >> j) & 1ull;
      all += pj ? lj : 0;
      below += (pj && j < lane) ? lj : 0;
    }
    uint64_t c0 = 0;
    if (valid) c0 = cur[pid];
    __builtin_amdgcn_wave_barrier();
    if (valid && (peers & lt_mask) == 0) cur[pid] = c0 + all;
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(g.data + a);
      uint32_t* dst = reinterpret_cast<uint32_t*>(out + c0 + below);
      const uint32_t nd = (uint32_t)(len >> 2);
      uint32_t k = 0;
      for (; k + 4 <= nd; k += 4)
        *reinterpret_cast<u32x4a4*>(dst + k) = *reinterpret_cast<const u32x4a4*>(src + k);
      for (; k < nd; ++k) dst[k] = src[k];
    }
  }
}

// ---- v2: register-streamed hist, wave-cooperative row copy ------------------------------------
// k_vhist2: U = 4 steps of 64 rows per round: every offset load, then every key load, issued
// before the first use (no dependent global load inside a step); pid stores unconditional at a
// clamped index (duplicates rewrite the same value).  Keys at a 4-aligned key_offset, KW words.
template <int WPG, int KW>
__global__ __launch_bounds__(WPG * kVWave) void k_vhist2(PartDev pd, VarGroup g,
                                                        uint16_t* __restrict__ pids,
                                                        uint64_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  constexpr int U = 4;
  const int wave = threadIdx.x / kVWave, lane = threadIdx.x % kVWave;
  const uint32_t total = g.num_maps * g.tiles_per_map;
  const uint32_t gtile = xcd_map(blockIdx.x, gridDim.x) * WPG + wave;
  const int R = pd.R;
  uint32_t* hist = lds + wave * R;
  for (int p = lane; p < R; p += kVWave) hist[p] = 0;
  __builtin_amdgcn_wave_barrier();
  if (gtile >= total) return;
  const uint32_t map = gtile / g.tiles_per_map, tile = gtile - map * g.tiles_per_map;
  const uint64_t mb = (uint64_t)map * g.records_per_map;
  const uint64_t me = min(mb + g.records_per_map, g.num_records);
  const uint64_t tb = min(mb + (uint64_t)tile * g.tile_recs, me);
  const uint64_t te = min(tb + g.tile_recs, me);
  const uint64_t o0 = g.offs[0];
  using KV = KeyVec<KW>;
  for (uint64_t i0 = tb; i0 < te; i0 += kVWave * U) {
    uint64_t a[U], e[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t ic = min(i0 + k * kVWave + lane, te - 1);
      a[k] = g.offs[ic];
      e[k] = g.offs[ic + 1];
    }
    typename KV::T kv[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      kv[k] = *reinterpret_cast<const typename KV::T*>(g.data + (a[k] - o0) + pd.key_offset);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t i = i0 + k * kVWave + lane;
      uint32_t w[KW];
      KV::get(kv[k], w);
      const int p = partition_words<KW, false>(pd, w, pd.bounds, pd.lut);
      pids[min(i, te - 1)] = (uint16_t)p;
      if (i < te) atomicAdd(&hist[p], (uint32_t)(e[k] - a[k]));
    }
  }
  __builtin_amdgcn_wave_barrier();
  uint64_t* dst = counts + ((uint64_t)map * R) * g.tiles_per_map + tile;
  for (int p = lane; p < R; p += kVWave) dst[(uint64_t)p * g.tiles_per_map] = hist[p];
}

// k_vscatter2: one wave per tile, 64 rows per step.
//   rank: ballot-match peers; the DWORDS of the lower peers / of all peers from one ballot per
//         length bit (popc of peers & lower & bit-mask), no cross-lane shuffles;
//   copy: 8 lanes per row, 8 rows per round, the first 128 bytes of all 64 rows loaded (8 x 16 B
//         per lane) before the first store; a row's last piece overlaps its previous one instead
//         of a partial store; the rest of longer rows by the whole wave, rows under 16 bytes by
//         their own lane in dwords.
template <int WPG>
__global__ __launch_bounds__(WPG * kVWave) void k_vscatter2(VarGroup g, int R, int pid_bits,
                                                           const uint16_t* __restrict__ pids,
                                                           const uint64_t* __restrict__ prefix,
                                                           const uint64_t* __restrict__ base,
                                                           uint8_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint64_t curs[];
  const int wave = threadIdx.x / kVWave, lane = threadIdx.x % kVWave;
  const uint32_t total = g.num_maps * g.tiles_per_map;
  const uint32_t gtile = xcd_map(blockIdx.x, gridDim.x) * WPG + wave;
  uint64_t* cur = curs + (uint64_t)wave * (R + 2 * kVWave);
  uint64_t* info = cur + R;  // [64] x {src byte offset | dwords << 44, dst byte offset}
  if (gtile >= total) return;
  const uint32_t map = gtile / g.tiles_per_map, tile = gtile - map * g.tiles_per_map;
  const uint64_t mb = (uint64_t)map * g.records_per_map;
  const uint64_t me = min(mb + g.records_per_map, g.num_records);
  const uint64_t tb = min(mb + (uint64_t)tile * g.tile_recs, me);
  const uint64_t te = min(tb + g.tile_recs, me);
  const uint64_t* bm = base + (uint64_t)map * R;
  const uint64_t* pm = prefix + (uint64_t)map * R * g.tiles_per_map + tile;
  for (int p = lane; p < R; p += kVWave) cur[p] = bm[p] + pm[(uint64_t)p * g.tiles_per_map];
  __builtin_amdgcn_wave_barrier();
  if (tb >= te) return;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const uint64_t o0 = g.offs[0];
  // every 16-byte load stays inside the rows: addresses clamp to tot - 16; under 16 bytes of
  // rows in all, every row takes the dword path
  const uint64_t tot = g.offs[g.num_records] - o0;
  const bool tiny = tot < 16;
  // next step's row (clamped: always a real row)
  uint64_t na = g.offs[min(tb + lane, te - 1)], ne = g.offs[min(tb + lane, te - 1) + 1];
  uint32_t npid = pids[min(tb + lane, te - 1)];
  for (uint64_t i0 = tb; i0 < te; i0 += kVWave) {
    const uint32_t nvalid = (uint32_t)min((uint64_t)kVWave, te - i0);
    const bool valid = (uint32_t)lane < nvalid;
    const uint64_t a = na - o0;
    const uint32_t dw = (uint32_t)((ne - na) >> 2);
    const uint32_t pid = min(npid, (uint32_t)(R - 1));
    {
      const uint64_t inext = min(i0 + kVWave + lane, te - 1);
      na = g.offs[inext];
      ne = g.offs[inext + 1];
      npid = pids[inext];
    }
    uint64_t peers = __ballot(valid);
    for (int bb = 0; bb < pid_bits; ++bb) {
      const bool bit = (pid >> bb) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    if (!valid) peers = 0;
    uint32_t below = 0, all = 0;
    const uint64_t pl = peers & lt_mask;
    for (int bb = 0; bb < 18; ++bb) {
      const uint64_t m = __ballot(valid && ((dw >> bb) & 1u));
      if (m == 0) continue;  // uniform
      below += (uint32_t)__popcll(pl & m) << bb;
      all += (uint32_t)__popcll(peers & m) << bb;
    }
    uint64_t c0 = 0;
    if (valid) c0 = cur[pid];
    __builtin_amdgcn_wave_barrier();
    if (valid && pl == 0) cur[pid] = c0 + 4ull * all;
    const uint64_t d = c0 + 4ull * below;
    info[2 * lane] = a | ((uint64_t)dw << 44);
    info[2 * lane + 1] = d;
    __builtin_amdgcn_wave_barrier();
    if (!tiny) {
    // first 128 bytes of every row, 8 lanes per row
    const uint32_t pc = (uint32_t)lane & 7u;
    u32x4a4 v[8];
    uint64_t dd[8];
    uint32_t ok = 0;
#pragma unroll
    for (int rnd = 0; rnd < 8; ++rnd) {
      const uint32_t r = min((uint32_t)rnd * 8u + ((uint32_t)lane >> 3), nvalid - 1);
      const uint64_t s0 = info[2 * r], d0 = info[2 * r + 1];
      const uint32_t L = (uint32_t)(s0 >> 44) * 4u;
      const uint64_t src = s0 & ((1ull << 44) - 1);
      uint32_t off = 16u * pc;
      if (L <= 128) off = min(off, L >= 16 ? L - 16 : 0u);
      v[rnd] = *reinterpret_cast<const u32x4a4*>(g.data + min(src + off, tot - 16));
      dd[rnd] = d0 + off;
      const bool use = (rnd * 8u + ((uint32_t)lane >> 3)) < nvalid && L >= 16 && 16u * pc < L;
      ok |= (uint32_t)use << rnd;
    }
#pragma unroll
    for (int rnd = 0; rnd < 8; ++rnd)
      if ((ok >> rnd) & 1u) *reinterpret_cast<u32x4a4*>(out + dd[rnd]) = v[rnd];
    // rows past 128 bytes: the whole wave, 16 bytes per lane per round
    uint64_t longm = __ballot(valid && dw > 32);
    while (longm) {
      const int j = __builtin_ctzll(longm);
      longm &= longm - 1;
      const uint64_t s0 = info[2 * j], d0 = info[2 * j + 1];
      const uint32_t L = (uint32_t)(s0 >> 44) * 4u;
      const uint64_t src = s0 & ((1ull << 44) - 1);
      for (uint32_t b0 = 128; b0 < L; b0 += 16 * kVWave * 4) {
        u32x4a4 w[4];
        uint32_t offs[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          offs[k] = min(b0 + 16u * (lane + kVWave * k), L - 16);
          w[k] = *reinterpret_cast<const u32x4a4*>(g.data + src + offs[k]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (b0 + 16u * (lane + kVWave * k) < L)
            *reinterpret_cast<u32x4a4*>(out + d0 + offs[k]) = w[k];
      }
    }
    }
    // rows under 16 bytes: their own lane, in dwords
    const bool small = valid && (dw < 4 || tiny);
    if (__ballot(small)) {
      if (small) {
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(g.data + a);
        uint32_t* d32 = reinterpret_cast<uint32_t*>(out + d);
        for (uint32_t k = 0; k < dw; ++k) d32[k] = s32[k];
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------------------------------
// k_vscatter3: variable-length rows through a partition-sorted LDS image written as whole 128-B
// lines (k_scatter8's scheme, sux_partition.hip, with byte ranks).  k_vscatter2 copies every row
// straight to its destination: ~0.3 row per partition per 64-row step, so nearly every row is a
// short write inside a line (PMC: 3.18 GB written for 2.28 GB of rows).  Here a 1024-thread
// workgroup walks one balanced range of tiles in chunks of <= 1024 rows and <= kV3Bytes bytes
// (a row is < 64 KiB, so a chunk holds at least one):
//   0. the chunk's row offsets into LDS, the rows that fit (their bytes were loaded as one window
//      of 16-byte units during the previous chunk), the next chunk's byte bound loaded;
//   1. per-wave byte ranks: ballot match over the pid bits, one ballot per size bit;
//   2. owners: p's dwords in the chunk; p's region = the line holding its cursor + those dwords;
//   3. carried units into region heads, each row's image offset, the partition byte of every
//      image unit (by the row it starts in; a long row by its whole wave);
//   4. the window's units into the image (the row holding a unit: binary search of the offsets);
//   5. the next chunk's loads;  6. complete lines out;  7. carries, cursors, item seams.
// Rows stay in input order inside a partition (waves in order, lanes in order), as k_vscatter.
// ------------------------------------------------------------------------------------------
typedef uint32_t vu32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kV3Rows = 1024;        // rows per chunk at most (one per thread)
constexpr uint32_t kV3Bytes = 88 * 1024;  // bytes per chunk at most (> the 64 KiB row limit)

struct Vs3 {
  static constexpr uint32_t NW = 16, NT = NW * kVWave, C = kV3Rows;
  static constexpr uint32_t PER = (kV3Bytes / 16 + 1 + NT - 1) / NT;  // window units per thread
  static constexpr uint32_t NB = (kV3Bytes / 128 + 8) & ~7u;  // 128-byte buckets of a chunk
  // a region: <= 31 dwords of the cursor's line + the partition's dwords, in units
  static __host__ __device__ constexpr uint32_t space(int R) {
    return kV3Bytes / 16 + (17u * R + 1) / 2 + 1;
  }
  // img[SP] u32x4 | pinfo[R] u32x4 | rowimg[C] | rofs[C + 4] | wcnt[NW][R] | lunit, fhead,
  // lpos [R] | tmp[NW + 1] | misc[4] | brow[NB] u16 | upid[SP] u8
  static __host__ __device__ constexpr uint32_t lds_bytes(int R) {
    return space(R) * 16 + (uint32_t)R * 16 + C * 4 + (C + 4) * 4 + NW * (uint32_t)R * 4 +
           3u * R * 4 + (NW + 1) * 4 + 16 + NB * 2 + space(R);
  }
  static __host__ __device__ constexpr bool fits(int R) {
    return R >= 1 && 4u * (uint32_t)R <= NT && lds_bytes(R) <= 160u * 1024;
  }
};

__device__ __forceinline__ uint32_t v3_wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int d = 1; d < kVWave; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, kVWave);
    if (lane >= d) v += t;
  }
  return v;
}

// Diagnostic build only (-DSUX_STAMPS, tools/vstamps.hip): thread 0 of workgroups < 64 records
// s_memtime at the phase boundaries of its first 16 chunks.  No stamp executes otherwise.
#ifdef SUX_STAMPS
__device__ uint64_t g_vstamps[64][16][8];
#define SUX_VSTAMP(ci, ph)                                                       \
  do {                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < 64 && (ci) < 16)                        \
      g_vstamps[blockIdx.x][(ci)][(ph)] = __builtin_amdgcn_s_memtime();         \
  } while (0)
#else
#define SUX_VSTAMP(ci, ph) \
  do {                     \
  } while (0)
#endif

__global__ __launch_bounds__(1024) void k_vscatter3(VarGroup g, int R, int pid_bits,
                                                    const uint16_t* __restrict__ pids,
                                                    const uint64_t* __restrict__ prefix,
                                                    const uint64_t* __restrict__ base,
                                                    uint8_t* __restrict__ out) {
  using K = Vs3;
  constexpr uint32_t NW = K::NW, NT = K::NT, C = K::C, PER = K::PER;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const uint32_t SP = K::space(R);
  vu32x4* img = reinterpret_cast<vu32x4*>(lds8);
  uint32_t* img32 = reinterpret_cast<uint32_t*>(lds8);
  vu32x4* pinfo = img + SP;  // {lb, cd, full lines, sp}
  uint32_t* rowimg = reinterpret_cast<uint32_t*>(pinfo + R);  // row t's image byte offset
  uint32_t* rofs = rowimg + C;      // row t's first byte from the chunk start; rofs[n] = bytes
  uint32_t* wcnt = rofs + C + 4;    // [NW][R]: dwords of p in wave w's rows
  uint32_t* lunit = wcnt + NW * R;  // the line holding p's cursor (128-byte line index)
  uint32_t* fhead = lunit + R;      // dwords of that line that belong to another range
  uint32_t* lpos = fhead + R;       // p's cursor's dword inside its line (flush at an item end)
  uint32_t* tmp = lpos + R;
  uint32_t* misc = tmp + NW + 1;  // [0] rows of the chunk that fit
  uint16_t* brow = reinterpret_cast<uint16_t*>(misc + 4);  // the row holding bucket j's first byte
  uint8_t* upid = reinterpret_cast<uint8_t*>(brow + K::NB);

  const int tid = threadIdx.x, wave = tid / kVWave, lane = tid % kVWave;
  const bool owner = tid < R;
  const uint32_t cp = (uint32_t)tid >> 2, cj = (uint32_t)tid & 3u;  // carry thread: (p, quarter)
  const bool carrier = cp < (uint32_t)R;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out);
  vu32x4* out4 = reinterpret_cast<vu32x4*>(out);
  const uint64_t o0 = g.offs[0];

  // one contiguous balanced range of the launch's tiles per workgroup, cut into items at map
  // boundaries (k_scatter8)
  const uint32_t T = g.num_maps * g.tiles_per_map, G = gridDim.x;
  const uint32_t rr = xcd_map(blockIdx.x, G);
  const uint32_t t_lo = (uint32_t)((uint64_t)T * rr / G), t_hi = (uint32_t)((uint64_t)T * (rr + 1) / G);
  if (t_lo >= t_hi) return;
  struct Cur {
    uint32_t it;      // the item's first tile
    uint64_t c0, ie;  // the chunk's first row, the item's end row
    uint64_t w;       // byte offset (from offs[0]) of row c0
    bool valid;
  };
  auto item_cur = [&](uint32_t t, uint64_t w) {  // the first chunk of the item at tile t
    Cur k;
    k.it = t;
    k.valid = t < t_hi;
    k.c0 = k.ie = 0;
    k.w = w;
    if (k.valid) {
      const uint32_t m = t / g.tiles_per_map, t0 = t - m * g.tiles_per_map;
      const uint32_t te = min(t_hi, (m + 1) * g.tiles_per_map) - m * g.tiles_per_map;
      const uint64_t mb = (uint64_t)m * g.records_per_map;
      const uint64_t me = min(mb + g.records_per_map, g.num_records);
      k.c0 = min(mb + (uint64_t)t0 * g.tile_recs, me);
      k.ie = min(mb + (uint64_t)te * g.tile_recs, me);
    }
    return k;
  };
  // the chunk after one of n rows and `bytes` bytes: an item ends at its map's end (the next map's
  // rows follow in the input) or at the range's end
  auto next_cur = [&](const Cur& k, uint32_t n, uint32_t bytes) {
    Cur nk = k;
    nk.c0 = k.c0 + n;
    nk.w = k.w + bytes;
    if (nk.c0 >= k.ie) nk = item_cur(min(t_hi, (k.it / g.tiles_per_map + 1) * g.tiles_per_map), nk.w);
    return nk;
  };
  // a chunk's loads: the offset and pid of row c0 + tid, the window [w, min(kend, w + kV3Bytes))
  auto issue = [&](const Cur& k, uint64_t kend, uint64_t& offv, uint32_t& pidv, vu32x4 (&v)[PER]) {
    const bool any = k.valid && k.ie > k.c0;
    const uint64_t r = any ? min(k.c0 + (uint64_t)tid, k.ie - 1) : 0;
    offv = g.offs[r];
    pidv = min((uint32_t)pids[r], (uint32_t)(R - 1));
    const uint8_t* a = g.data + k.w;
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 15u);
    const vu32x4* src = reinterpret_cast<const vu32x4*>(a - head);
    const uint32_t ext = any ? (uint32_t)min(kend - o0 - k.w, (uint64_t)kV3Bytes) : 0u;
    const uint32_t units = ext ? (head + ext + 15) >> 4 : 0u;
    // unconditional (clamped) loads: a load under a per-lane branch makes the compiler wait for
    // the earlier ones before the next (k_msd16b measured: 2.5x the issue time)
    if (units == 0) return;
#pragma unroll
    for (uint32_t k2 = 0; k2 < PER; ++k2) v[k2] = src[min(tid + k2 * NT, units - 1)];
  };

  uint64_t pos = 0;  // owner: p's output cursor (bytes)
  auto begin_item = [&](uint32_t t) {
    if (owner) {
      const uint32_t m = t / g.tiles_per_map, t0 = t - m * g.tiles_per_map;
      pos = base[(uint64_t)m * R + tid] + prefix[((uint64_t)m * R + tid) * g.tiles_per_map + t0];
      fhead[tid] = (uint32_t)(pos & 127) >> 2;  // the line's earlier dwords: another range's
    }
  };
  if (owner)
    for (uint32_t w = 0; w < NW; ++w) wcnt[w * R + tid] = 0;
  vu32x4 cu0{0, 0, 0, 0}, cu1{0, 0, 0, 0};  // carrier: units 2cj, 2cj+1 of p's carried line
  begin_item(t_lo);
  Cur k = item_cur(t_lo, 0);
  k.w = g.offs[k.c0] - o0;
  uint64_t kend = g.offs[min(k.c0 + (uint64_t)C, k.ie)];
  uint64_t offv;
  uint32_t pidv;
  vu32x4 v[PER];
  issue(k, kend, offv, pidv, v);
  __syncthreads();
  [[maybe_unused]] uint32_t ci = 0;  // chunk counter for the diagnostic stamps
  while (true) {
    SUX_VSTAMP(ci, 0);
    // 0. row offsets, the rows that fit, the next chunk's bound
    const uint64_t cstart = k.w + o0;
    const uint64_t avail = k.valid && k.ie > k.c0 ? min((uint64_t)C, k.ie - k.c0) : 0;
    rofs[tid] = (uint32_t)min(offv - cstart, (uint64_t)0xFFFFFFFFu);
    if (tid == 0) {
      rofs[C] = (uint32_t)min(kend - cstart, (uint64_t)0xFFFFFFFFu);
      misc[0] = 0;
    }
    __syncthreads();
    {
      const uint32_t nxt = (uint64_t)tid + 1 < avail ? rofs[tid + 1] : rofs[C];
      const bool fit = (uint64_t)tid < avail && nxt <= kV3Bytes;
      const uint64_t bm = __ballot(fit);
      if (lane == 0 && bm) atomicAdd(&misc[0], (uint32_t)__popcll(bm));
    }
    __syncthreads();
    const uint32_t n = misc[0];
    if (n == 0 && avail > 0) break;  // a row over kV3Bytes: outside the contract (rows < 64 KiB)
    const uint32_t nb = n ? (n < avail ? rofs[n] : rofs[C]) : 0u;
    const Cur nk = next_cur(k, n, nb);
    const bool seam = nk.it != k.it, more = nk.valid;
    const uint64_t nend = more ? g.offs[min(nk.c0 + (uint64_t)C, nk.ie)] : 0;
    if (tid == 0 && n == avail && n < C) rofs[n] = nb;  // the last row's end (else already there)
    __syncthreads();
    SUX_VSTAMP(ci, 1);
    // 1. per-wave byte ranks (dwords)
    const bool valid = (uint32_t)tid < n;
    const uint32_t pid = valid ? pidv : 0u;
    const uint32_t dw = valid ? (rofs[tid + 1] - rofs[tid]) >> 2 : 0u;
    uint64_t peers = __ballot(valid);
    for (int bb = 0; bb < pid_bits; ++bb) {
      const bool bit = (pid >> bb) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    if (!valid) peers = 0;
    const uint64_t pl = peers & lt_mask;
    uint32_t below = 0, all = 0;
    uint32_t mx = dw;  // the wave's longest row bounds the size bits
#pragma unroll
    for (int d = 1; d < kVWave; d <<= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, d, kVWave));
    const int nbits = 32 - __builtin_clz(mx | 1u);  // rows < 64 KiB: <= 14
    for (int bb = 0; bb < nbits; ++bb) {
      const uint64_t m = __ballot(valid && ((dw >> bb) & 1u));
      if (m == 0) continue;  // uniform
      below += (uint32_t)__popcll(pl & m) << bb;
      all += (uint32_t)__popcll(peers & m) << bb;
    }
    if (valid && pl == 0) wcnt[wave * R + pid] = all;
    __syncthreads();
    SUX_VSTAMP(ci, 2);
    // 2. owners: prefix over waves, region = the cursor's line from its start + c dwords
    uint32_t c = 0, full = 0, sp = 0;
    if (owner) {
      uint32_t x[NW];
#pragma unroll
      for (uint32_t w = 0; w < NW; ++w) x[w] = wcnt[w * R + tid];
#pragma unroll
      for (uint32_t w = 0; w < NW; ++w) {
        wcnt[w * R + tid] = c;
        c += x[w];
      }
      const uint32_t totd = ((uint32_t)(pos & 127) >> 2) + c;
      full = totd >> 5;
      sp = (totd + 3) >> 2;
    }
    const uint32_t incl = v3_wave_incl_scan(sp, lane);
    if (lane == kVWave - 1) tmp[wave] = incl;
    __syncthreads();
    uint32_t lb = incl - sp, U = 0;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) {
      const uint32_t t = tmp[w];
      lb += (w < (uint32_t)wave) ? t : 0u;
      U += t;
    }
    if (owner) {
      pinfo[tid] = vu32x4{lb, (uint32_t)(pos & 127) >> 2, full, sp};
      lunit[tid] = (uint32_t)(pos >> 7);
    }
    __syncthreads();
    SUX_VSTAMP(ci, 3);
    // 3. carried units, row image offsets, the partition byte of every image unit (written by
    //    whoever holds the unit's first dword: a carrier for the carried head, else its row)
    if (carrier) {
      const vu32x4 pi = pinfo[cp];
      const uint32_t cdu = (pi[1] + 3) >> 2;
      if (2 * cj < cdu) {
        img[pi[0] + 2 * cj] = cu0;
        upid[pi[0] + 2 * cj] = (uint8_t)cp;
      }
      if (2 * cj + 1 < cdu) {
        img[pi[0] + 2 * cj + 1] = cu1;
        upid[pi[0] + 2 * cj + 1] = (uint8_t)cp;
      }
    }
    //    and brow: the row holding the first byte of every 128-byte bucket of the chunk
    {
      uint32_t q0 = 0, q1 = 0, j0 = 0, j1 = 0;
      if (valid) {
        const vu32x4 pi = pinfo[pid];
        const uint32_t d0 = pi[1] + wcnt[wave * R + pid] + below;  // the row's first dword
        rowimg[tid] = 16 * pi[0] + 4 * d0;
        q0 = pi[0] + ((d0 + 3) >> 2);
        q1 = pi[0] + ((d0 + dw + 3) >> 2);
        j0 = (rofs[tid] + 127) >> 7;
        j1 = (rofs[tid + 1] + 127) >> 7;
        if (q1 - q0 <= 8 && j1 - j0 <= 2) {
          for (uint32_t q = q0; q < q1; ++q) upid[q] = (uint8_t)pid;
          for (uint32_t j = j0; j < j1; ++j) brow[j] = (uint16_t)tid;
        }
      }
      uint64_t lm = __ballot(valid && (q1 - q0 > 8 || j1 - j0 > 2));
      while (lm) {  // long rows: the whole wave
        const int j = __builtin_ctzll(lm);
        lm &= lm - 1;
        const uint32_t a = __shfl(q0, j, kVWave), b = __shfl(q1, j, kVWave);
        const uint8_t p = (uint8_t)__shfl(pid, j, kVWave);
        for (uint32_t q = a + lane; q < b; q += kVWave) upid[q] = p;
        const uint32_t ja = __shfl(j0, j, kVWave), jb = __shfl(j1, j, kVWave);
        const uint16_t row = (uint16_t)(wave * kVWave + j);
        for (uint32_t q = ja + lane; q < jb; q += kVWave) brow[q] = row;
      }
    }
    __syncthreads();
    SUX_VSTAMP(ci, 4);
    // 4. the window's units -> image (a unit inside one row as one ds_write_b128, else dwords)
    {
      const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(g.data + k.w) & 15u);
#pragma unroll
      for (uint32_t k2 = 0; k2 < PER; ++k2) {
        const int32_t b0 = (int32_t)(16 * (tid + k2 * NT)) - (int32_t)head;
        if (b0 + 16 <= 0 || b0 >= (int32_t)nb) continue;
        const uint32_t b = b0 < 0 ? 0u : (uint32_t)b0;
        uint32_t lo = brow[b >> 7];  // rofs[lo] <= b: then the few rows up to b (rows >= 4 B)
        while (rofs[lo + 1] <= b) ++lo;
        if (b0 >= 0 && b + 16 <= rofs[lo + 1]) {
          *reinterpret_cast<u32x4a4*>(img32 + ((rowimg[lo] + b - rofs[lo]) >> 2)) = v[k2];
        } else {
          uint32_t r = lo;
#pragma unroll
          for (uint32_t q = 0; q < 4; ++q) {
            const int32_t bq = b0 + 4 * (int32_t)q;
            if (bq < 0 || bq >= (int32_t)nb) continue;
            while ((uint32_t)bq >= rofs[r + 1]) ++r;
            const uint32_t x = q == 0 ? v[k2][0] : q == 1 ? v[k2][1] : q == 2 ? v[k2][2] : v[k2][3];
            img32[(rowimg[r] + (uint32_t)bq - rofs[r]) >> 2] = x;
          }
        }
      }
    }
    // 5. the registers are free: the next chunk's loads
    issue(nk, nend, offv, pidv, v);
    __syncthreads();
    SUX_VSTAMP(ci, 5);
    // 6. complete lines of every region out (the dwords of another range skipped)
    for (uint32_t q = tid; q < U; q += NT) {
      const uint32_t p = upid[q];
      const vu32x4 pi = pinfo[p];
      const uint32_t kq = q - pi[0];
      if (kq >= 8 * pi[2]) continue;
      const uint64_t A = 8ull * lunit[p] + kq;
      const vu32x4 x = img[q];
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
    SUX_VSTAMP(ci, 6);
    // 7. carries into the carrier registers, cursors advance; an item's last line is flushed
    if (carrier) {
      const vu32x4 pi = pinfo[cp];
      const uint32_t b = pi[0] + 8 * pi[2] + 2 * cj;
      if (2 * cj < pi[3] - 8 * pi[2]) cu0 = img[b];
      if (2 * cj + 1 < pi[3] - 8 * pi[2]) cu1 = img[b + 1];
    }
    if (owner) {
      if (full) fhead[tid] = 0;
      pos += 4ull * c;
      lunit[tid] = (uint32_t)(pos >> 7);
      lpos[tid] = (uint32_t)(pos >> 2) & 31u;
      for (uint32_t w = 0; w < NW; ++w) wcnt[w * R + tid] = 0;
    }
    if (seam) {
      __syncthreads();
      if (carrier) {  // dwords [fhead, cursor) of the cursor's line: this range's, not yet stored
        const uint32_t cdn = lpos[cp], f = fhead[cp];
        const uint64_t L = 32ull * lunit[cp];
#pragma unroll
        for (uint32_t cc = 0; cc < 8; ++cc) {
          const uint32_t d = 8 * cj + cc;
          const uint32_t x = cc < 4 ? cu0[cc] : cu1[cc - 4];
          if (d >= f && d < cdn) out32[L + d] = x;
        }
      }
      __syncthreads();
      if (more) begin_item(nk.it);
    }
    __syncthreads();
    SUX_VSTAMP(ci, 7);
    ++ci;
    if (!more) break;
    k = nk;
    kend = nend;
  }
}

// K2a: exclusive scan of one (map, partition) row of byte counts over its tiles, in place, one
// wave per row (u64: a map's partition may pass 4 GiB); totals[m][p] = the row's sum.
__global__ __launch_bounds__(256) void k_vtile_scan(uint64_t* __restrict__ counts,
                                                    uint64_t* __restrict__ totals, uint32_t rows,
                                                    uint32_t tiles) {
  const int lane = threadIdx.x % kVWave;
  const uint32_t row = blockIdx.x * 4 + threadIdx.x / kVWave;
  if (row >= rows) return;
  uint64_t* c = counts + (uint64_t)row * tiles;
  uint64_t carry = 0;
  for (uint32_t t0 = 0; t0 < tiles; t0 += kVWave) {
    const uint32_t t = t0 + lane;
    const uint64_t v = t < tiles ? c[t] : 0;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < kVWave; d <<= 1) {
      const uint64_t y = __shfl_up(x, d, kVWave);
      if (lane >= d) x += y;
    }
    if (t < tiles) c[t] = carry + x - v;
    carry += __shfl(x, kVWave - 1, kVWave);
  }
  if (lane == 0) totals[row] = carry;
}

VarWorkspace varlen_workspace_layout(uint32_t R, uint64_t records_per_map, uint64_t num_records,
                                     uint32_t tile_recs) {
  VarWorkspace w{};
  uint64_t maps = records_per_map ? (num_records + records_per_map - 1) / records_per_map : 0;
  if (maps == 0) maps = 1;
  uint64_t tiles = (records_per_map + tile_recs - 1) / tile_recs;
  if (tiles == 0) tiles = 1;
  auto up = [](uint64_t x) { return (x + 255) & ~255ull; };
  uint64_t off = 0;
  w.counts_off = off;
  off += up(maps * R * tiles * 8);
  w.totals_off = off;
  off += up(maps * R * 8);
  w.base_off = off;  // base | (unused by G == 1) in-map prefix | per-peer sums, as k_map_scan wants
  off += up(3 * maps * R * 8);
  w.pids_off = off;
  off += up(num_records * 2);
  w.total = off;
  return w;
}

uint32_t choose_varlen_tile(uint32_t R, uint64_t rows, const Tuning& tn) {
  if (tn.varlen_tile >= 64 && tn.varlen_tile % 64 == 0) return (uint32_t)tn.varlen_tile;
  uint32_t t = 512;
  while (t < 2 * R && t < 65536) t <<= 1;  // counts stay <= 4 B per record
  // longer tiles (longer per-partition runs per wave) while >= 16 Ki tiles keep every CU busy
  while (t < 2048 && rows / (2ull * t) >= 16384) t <<= 1;
  return t;
}

hipError_t launch_varlen_group(const PartDev& pd, const VarGroup& g, uint8_t* d_out,
                               int64_t* d_index, uint8_t* d_index_be, const uint16_t* d_pids_in,
                               uint16_t* d_pids, uint8_t* d_ws, const VarWorkspace& ws,
                               const Tuning& tn, Timer* timer, hipStream_t s) {
  const int R = pd.R;
  uint64_t* counts = reinterpret_cast<uint64_t*>(d_ws + ws.counts_off);
  uint64_t* totals = reinterpret_cast<uint64_t*>(d_ws + ws.totals_off);
  uint64_t* base = reinterpret_cast<uint64_t*>(d_ws + ws.base_off);
  uint16_t* pids = d_pids ? d_pids : reinterpret_cast<uint16_t*>(d_ws + ws.pids_off);
  int bits = 0;
  while ((1 << bits) < R) ++bits;
  const uint32_t total_tiles = g.num_maps * g.tiles_per_map;
  const bool four = (size_t)(R + 2 * kVWave) * 8 * 4 <= 64 * 1024;  // 4 waves per workgroup while LDS allows
  const uint32_t wpg = four ? 4 : 1;
  const dim3 grid((total_tiles + wpg - 1) / wpg);
  const int ver = tn.varlen_kernel;
  // v2 needs: a fixed-width key at a 4-aligned offset (or caller ids) and >= 16 bytes of rows
  int kw = 0;
  if (pd.key_offset % 4 == 0) {
    if (pd.kind == 2 || pd.kind == 5) kw = 2;
    else if (pd.kind == 3 || pd.kind == 6) kw = 1;
    else if (pd.kind == 1) kw = (pd.key_len + 3) / 4;
  }
  const bool v2 = ver >= 2;
  const bool hist2 = v2 && kw > 0 && !d_pids_in;
  timer_note(timer, kHist, "k_vhist");
  timer_begin(timer, kHist, s);
  if (hist2) {
    const size_t lds = (size_t)wpg * R * 4;
    if (lds > 64 * 1024) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vhist2<1, 1>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vhist2<1, 2>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vhist2<1, 3>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vhist2<1, 4>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
#define SUX_VH2(W, K) \
  hipLaunchKernelGGL((k_vhist2<W, K>), grid, dim3(W * kVWave), lds, s, pd, g, pids, counts)
    if (four) {
      if (kw == 1) SUX_VH2(4, 1); else if (kw == 2) SUX_VH2(4, 2); else if (kw == 3) SUX_VH2(4, 3); else SUX_VH2(4, 4);
    } else {
      if (kw == 1) SUX_VH2(1, 1); else if (kw == 2) SUX_VH2(1, 2); else if (kw == 3) SUX_VH2(1, 3); else SUX_VH2(1, 4);
    }
#undef SUX_VH2
  } else {
    const size_t lds = (size_t)wpg * R * 4;
    if (lds > 64 * 1024) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vhist<1>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (four)
      hipLaunchKernelGGL((k_vhist<4>), grid, dim3(4 * kVWave), lds, s, pd, g, d_pids_in, pids,
                         counts);
    else
      hipLaunchKernelGGL((k_vhist<1>), grid, dim3(kVWave), lds, s, pd, g, d_pids_in, pids, counts);
  }
  timer_end(timer, kHist, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  timer_begin(timer, kScan, s);
  {
    const uint32_t rows = g.num_maps * (uint32_t)R;
    hipLaunchKernelGGL(k_vtile_scan, dim3((rows + 3) / 4), dim3(256), 0, s, counts, totals, rows,
                       g.tiles_per_map);
  }
  e = launch_varlen_map_scan(g, R, totals, base, d_index, d_index_be, s);
  timer_end(timer, kScan, s);
  if (e != hipSuccess) return e;
  if (d_pids_in) pids = const_cast<uint16_t*>(d_pids_in);
  timer_note(timer, kScatter, "k_vscatter");
  timer_begin(timer, kScatter, s);
  if (ver == 3 && Vs3::fits(R)) {
    // one workgroup per CU of the stream, each one balanced range of tiles
    const uint32_t lds = Vs3::lds_bytes(R);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vscatter3),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const uint32_t g3 = std::min<uint32_t>(total_tiles, (uint32_t)stream_cus(s));
    hipLaunchKernelGGL(k_vscatter3, dim3(g3), dim3(Vs3::NT), lds, s, g, R, bits, pids, counts,
                       base, d_out);
  } else if (v2) {
    const size_t lds = (size_t)wpg * (R + 2 * kVWave) * 8;
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vscatter2<1>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (four)
      hipLaunchKernelGGL((k_vscatter2<4>), grid, dim3(4 * kVWave), lds, s, g, R, bits, pids,
                         counts, base, d_out);
    else
      hipLaunchKernelGGL((k_vscatter2<1>), grid, dim3(kVWave), lds, s, g, R, bits, pids, counts,
                         base, d_out);
  } else {
    const size_t lds = (size_t)wpg * R * 8;
    if (lds > 64 * 1024) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vscatter<1>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (four)
      hipLaunchKernelGGL((k_vscatter<4>), grid, dim3(4 * kVWave), lds, s, g, R, bits, pids, counts,
                         base, d_out);
    else
      hipLaunchKernelGGL((k_vscatter<1>), grid, dim3(kVWave), lds, s, g, R, bits, pids, counts,
                         base, d_out);
  }
  timer_end(timer, kScatter, s);
  return hipGetLastError();
}

}  // namespace sux
