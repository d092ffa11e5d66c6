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
  if (v2) {
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
