// sux_part.h — device pieces shared by the map-side kernels (sux_partition.hip, sux_small.hip)
// and the reduce-side LDS sort (sux_sort.hip): wave shape, tile geometry, wave / block scans, the
// stable in-wave rank, and the small-record launchers sux_partition.hip dispatches to.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "sux_internal.h"

namespace sux {

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    uint32_t t = __shfl_up(v, d, kWave);
    if (lane >= d) v += t;
  }
  return v;
}

constexpr int kScanThreads = 1024;

// Block-wide exclusive scan of one u64 per thread; returns the exclusive prefix, *total = sum.
__device__ inline uint64_t block_excl_scan(uint64_t v, uint64_t* sh, uint64_t* total) {
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

__device__ __forceinline__ uint32_t owner_of(uint32_t p, int R, int G,
                                             const int32_t* own = nullptr) {
  if (own) {  // largest h with own[h] <= p (an empty range's owner is never the answer)
    uint32_t lo = 0, hi = (uint32_t)G;  // own[lo] <= p < own[hi]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if ((uint32_t)own[mid] <= p) lo = mid; else hi = mid;
    }
    return lo;
  }
  // largest h with floor(h*R/G) <= p
  return (uint32_t)((((uint64_t)p + 1) * G + R - 1) / R) - 1;
}
// First partition peer h owns (h = G: R).
__device__ __forceinline__ uint32_t owner_lo_of(uint32_t h, int R, int G, const int32_t* own) {
  return own ? (uint32_t)own[h] : (uint32_t)(((int64_t)h * R) / G);
}

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

// wave_rank with the digit match on a 6-bit group tag instead of the DB digit bits: every valid
// lane stores its lane index at tag[dig] (one byte per digit, the wave's own array) and reads it
// back.  Whichever lane's store landed, all lanes of one digit read the same lane index and
// lanes of different digits read different ones (a digit's slot only ever holds a lane of that
// digit this round), so matching the 6 tag bits finds exactly the lanes of the same digit.
// Same ranks as wave_rank; 6 ballots instead of DB.
template <uint32_t DB, typename CT = uint32_t>
__device__ __forceinline__ uint32_t wave_rank_tag(uint32_t dig, bool valid, CT* wcw, uint8_t* tag,
                                                  int lane, uint64_t lt_mask) {
  if (valid) tag[dig] = (uint8_t)lane;
  // the read below must reload the byte (other lanes' stores), never forward this lane's own
  // store: a compiler memory barrier; the wave's LDS operations complete in order
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  const uint32_t t = valid ? (uint32_t)tag[dig] : 0u;
  uint64_t peers = __ballot(valid);
#pragma unroll
  for (uint32_t bb = 0; bb < 6; ++bb) {
    const bool bit = (t >> bb) & 1u;
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

// PartDev::dseed: the digit shift of a sort pass decided on the device (make_sort_plan).
__device__ __forceinline__ void resolve_seed(PartDev& pd) {
  if (pd.dseed) pd.seed = *pd.dseed;
}

// Dynamic LDS above 64 KiB must be opted into per kernel (gfx950 allows 160 KiB per workgroup).
static inline void allow_lds(const void* fn, size_t lds) {
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

// ---- small records (16-byte rows, R > 1024; sux_small.hip) ----------------------------------
// The two-level MSD path without K1 applies (tuning small_kernel 4, map-major, ...).
bool msd16_eligible(const PartDev& pd, const MapGroup& g, const LayoutDesc& lay,
                    const uint8_t* d_out, const Workspace& ws, const Tuning& tn);
// k_msd16a -> k_msd16_scan -> k_msd16b: the whole map side of the group (index tables included).
hipError_t launch_msd16(const PartDev& pd, const MapGroup& g, uint8_t* d_out, int64_t* d_index,
                        uint8_t* d_index_be, uint16_t* d_pids, uint8_t* d_ws, const Workspace& ws,
                        uint64_t* d_peer_bytes, const Tuning& tn, Timer* timer, hipStream_t s);
// K1 of the small-record path: pids + tile-major counts [map][tile][p].
hipError_t launch_hist16(const PartDev& pd, const MapGroup& g, uint16_t* pids, uint32_t* counts,
                         hipStream_t s);
// K3 of the small-record path: k_scatter16s (sorted chunks, R <= 16384, small_kernel != 1) or the
// turn-taking k_scatter16b; notes the variant in the timer's scatter slot.
hipError_t launch_scatter16(const MapGroup& g, int R, int pid_bits, const uint16_t* pids,
                            const uint32_t* prefix, const uint64_t* base, uint8_t* d_out,
                            const Tuning& tn, Timer* timer, hipStream_t s);

}  // namespace sux
