// sux_small.hip — the map side for small records (16-byte rows, R > 1024: SURVEY.md §8 C5).
// Called from sux_partition.hip's launch_partition_group when the group's records are 16-byte
// units with a word-aligned key of <= 16 bytes; the 100-byte TeraSort path lives there.  Output
// contract identical to the large-record kernels: stable per-partition regroup (P2), index tables
// native + big-endian (P3).
#include <type_traits>

#include "sux_part.h"

namespace sux {

// ------------------------------------------------------------------------------------------
// Small records (S = 16, SURVEY.md config C5: 16-byte key/value rows, 10,000 partitions).
// A record is one aligned 16-byte unit and R is far too large for per-wave counters, so:
//   k_hist16    persistent workgroups of 1024 threads, one tile at a time; every lane loads whole
//               records (coalesced 16-byte units, 8 in flight per lane), hashes the key from its
//               registers and counts into ONE per-workgroup LDS histogram of R counters.
//   k_scatter16b persistent 1024-thread workgroups, one tile range at a time with an LDS cursor
//               per partition.  The tile is cut into 64-record groups dealt to the waves in
//               order; a wave ranks GB groups' equal pids with ballot matches, then, when the LDS
//               turn counter reaches it, reads and advances the cursors of its pids and hands the
//               turn on.  Only that short step is serialised; loads and 16-byte stores are not.
//   k_scatter16s the same without turns: chunks sorted by pid in LDS (below).
//   k_msd16a/b  the two-level path without K1 (below; the default for long maps).
// ------------------------------------------------------------------------------------------
template <int KW>
__global__ __launch_bounds__(1024) void k_hist16(PartDev pd, MapGroup g, uint16_t* __restrict__ pids,
                                                uint32_t* __restrict__ counts) {
  resolve_seed(pd);
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

// The turn is handed on once per batch of GB consecutive 64-record groups: a wave ranks GB groups,
// then in its turn walks their cursor updates back to back (LDS ops of one wave stay in order), so
// the cross-wave hand-off (acquire spin, release fence) is paid GB x less often (GB = 1: once per
// group, round 1's k_scatter16).  The next batch's loads fly during this batch's turn.
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
// Partitions per bucket, 2^LO: 16 (LO 4) for long maps; 256 (LO 8) for short maps, whose 16-
// partition segments would be too short to pay a segment's fixed cost (64 Ki-record maps at
// R = 10 000: 105 records at LO 4, 1677 at LO 8 — the 2^20-record maps' segment at LO 4).
constexpr uint32_t kM16Lo = 4;
constexpr uint32_t kM16LoShort = 8;
// msd_direct bit 3: 32-partition buckets (runs of ~13 records = ~210 B per (chunk, bucket) at
// R = 10 000 instead of ~6.5 = ~105 B) with 512-thread, 4096-record pass-B workgroups
constexpr uint32_t kM16LoWide = 5;
constexpr uint32_t kM16MaxChunks = 512;   // chunks per map pass B's run table holds (2 Mi records)
constexpr uint32_t kM16MaxChunksShort = 64;  // LO 8: maps of <= 256 Ki records

// A workgroup barrier that leaves LDS-DMA prefetches in flight: this wave's LDS accesses are
// complete (lgkmcnt(0)) and every wave arrived — no vmcnt wait, which __syncthreads' fence would
// emit while a global_load_lds is outstanding (cdna_hip_programming.md, "Pipelining across
// barriers").  The "memory" clobber keeps the compiler from moving memory accesses across it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Block exclusive scan, in (digit, wave) order, of u16 per-wave digit counters wc[NW][NB]
// (NW*64 threads; each thread owns E = NB/64 consecutive (digit, wave) entries).  Counts and
// prefixes fit u16: a chunk holds kM16Chunk records.  Two barriers (RAW: lds_barrier); wsum[NW]
// scratch.
template <uint32_t NB, uint32_t NW, bool RAW = false, typename CT = uint16_t>
__device__ __forceinline__ void scan_digit_wave16(CT* wc, uint32_t* wsum, int tid, int lane,
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
  if constexpr (RAW) lds_barrier(); else __syncthreads();
  uint32_t run = incl - sum;
#pragma unroll
  for (uint32_t w = 0; w < NW; ++w) run += w < (uint32_t)wave ? wsum[w] : 0u;
#pragma unroll
  for (uint32_t k = 0; k < E; ++k) {
    const uint32_t idx = (uint32_t)tid * E + k, d = idx / NW, w = idx % NW;
    const uint32_t v = wc[w * NB + d];
    wc[w * NB + d] = (CT)run;
    run += v;
  }
  if constexpr (RAW) lds_barrier(); else __syncthreads();
}

// stage[CH] u32x4 (its first NW words double as wsum) | wc[NW][2^DB] u16 (u32: atomic ranking)
// (| tag[NW][2^DB] u8 with the tag match, TAG)
template <uint32_t NW, uint32_t DB, uint32_t CB = 2, bool TAG = false>
struct M16a {
  static constexpr uint32_t NB = 1u << DB, NT = NW * kWave, PT = kM16Chunk / NT;
  static constexpr uint32_t lds_bytes() { return kM16Chunk * 16 + NW * NB * CB + (TAG ? NW * NB : 0u); }
};
// stage[CAP] u32x4 | wc[NW][NB] | cur[NB] | wsum[NW] | los[CAP] u8 | rp[MC+1] u32 | ro[MC] u16
template <uint32_t NW, uint32_t PT, uint32_t LO = kM16Lo, uint32_t MC = kM16MaxChunks>
struct M16b {
  static constexpr uint32_t NB = (1u << LO) > 64 ? (1u << LO) : 64, NT = NW * kWave, CAP = NT * PT;
  static constexpr uint32_t lds_bytes() {
    return CAP * 16 + NW * NB * 4 + NB * 4 + NW * 4 + CAP + (MC + 1) * 4 + MC * 2;
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

// ATOM (msd_direct bit 6): the ranking's counters are u32 and each digit group's leader updates
// its counter with one returning atomic, all PT rounds issued before any result is used — the
// u16 read-by-every-lane + leader-write round trip of wave_rank, once per round, is pass A's
// costliest bank-conflicted LDS traffic (tools/msd_whatif.hip: with conflict-free counters pass A
// would be 14 % faster).
// TAG (msd_direct bit 7): the ranking matches digits on a 6-bit lane tag (wave_rank_tag).
template <int KW, uint32_t NW, uint32_t DB, uint32_t LO, bool DIRECT = false, bool ATOM = false,
          bool TAG = false>
__global__ __launch_bounds__(NW * 64, 4) void k_msd16a(PartDev pd, MapGroup g, uint32_t cpm,
                                                 uint32_t nbk, uint16_t* __restrict__ offs,
                                                 uint16_t* __restrict__ pids_out,
                                                 uint8_t* __restrict__ tmp) {
  static_assert(!(TAG && ATOM), "one ranking");
  resolve_seed(pd);
  using CT = typename std::conditional<ATOM, uint32_t, uint16_t>::type;
  using K = M16a<NW, DB, sizeof(CT), TAG>;
  constexpr uint32_t NB = K::NB, NT = K::NT, PT = K::PT, CH = kM16Chunk;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  u32x4* stage = reinterpret_cast<u32x4*>(lds8);
  CT* wc = reinterpret_cast<CT*>(stage + CH);  // [NW][NB]
  uint8_t* tag8 = reinterpret_cast<uint8_t*>(wc + NW * NB);  // TAG: [NW][NB]
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
      h[j] = (p >> LO) & (NB - 1);
#if defined(SUX_MSD_WHATIF) && SUX_MSD_WHATIF == 2
      // diagnostic (level 2): the ranking's counter read / update at a conflict-free digit (the
      // lane's own), the pid kept alive through the digit's top bit (the compiler proves that
      // bit and bits 6..8 of the digit zero, so three of the nine match ballots fold away too)
      h[j] = ((uint32_t)lane | (p >> 31)) & (NB - 1);
#elif defined(SUX_MSD_WHATIF) && SUX_MSD_WHATIF == 3
      // diagnostic (level 3): the digit's low 6 bits replaced by the lane — no two lanes of a
      // wave share a digit and the counter accesses are at most 2-way conflicted — with every
      // bit still data-dependent, so all nine match ballots stay
      // (the lane XORed with a run-time zero the compiler cannot see through)
      h[j] = (((uint32_t)lane ^ (uint32_t)(g.num_records >> 56)) & 63u) | (h[j] & ~63u);
#endif
      if constexpr (ATOM) {
        // the group's leader (its lowest lane) adds the group's size with a returning atomic;
        // nothing waits for it here: the PT atomics of a wave queue back to back (one wave's LDS
        // operations complete in order, so each returns the count before its own round) and
        // the lanes fetch their leader's old count after the loop.  Meanwhile the record's
        // digit, rank inside its group and leader lane are packed into h[j].
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (uint32_t bb = 0; bb < DB; ++bb) {
          const bool bit = (h[j] >> bb) & 1u;
          const uint64_t m = __ballot(bit);
          peers &= bit ? m : ~m;
        }
        uint32_t o = 0;
        if (valid && (peers & lt_mask) == 0)
          o = atomicAdd(wc + wave * NB + h[j], (uint32_t)__popcll(peers));
        rank[j] = o;
        h[j] = valid ? h[j] | ((uint32_t)__popcll(peers & lt_mask) << 9) |
                           ((uint32_t)__builtin_ctzll(peers) << 16)
                     : ~0u;
      } else if constexpr (TAG) {
        rank[j] = wave_rank_tag<DB, uint16_t>(h[j], valid, wc + wave * NB, tag8 + wave * NB, lane,
                                              lt_mask);
      } else {
        rank[j] = wave_rank<DB, uint16_t>(h[j], valid, wc + wave * NB, lt_mask);
      }
    }
    if constexpr (ATOM) {
      static_assert(DB <= 9, "digit, group rank and leader packed into 9 + 7 + 6 bits");
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t pk = h[j];
        const int ldr = pk == ~0u ? 0 : (int)((pk >> 16) & 63u);
        const uint32_t o = (uint32_t)__builtin_amdgcn_ds_bpermute(ldr << 2, (int)rank[j]);
        rank[j] = pk == ~0u ? ~0u : o + ((pk >> 9) & 127u);
        h[j] = pk & (NB - 1);
      }
    }
    __syncthreads();
    scan_digit_wave16<NB, NW, false, CT>(wc, wsum, tid, lane, wave);
    if constexpr (DIRECT) {
      // each record straight from its registers to its bucket-sorted place in the chunk's own
      // 64 KB window (the window is written whole, so its lines merge in the L2)
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j)
        if (rank[j] != ~0u) t4[k.c0 + wc[wave * NB + h[j]] + rank[j]] = rv[j];
    } else {
#ifdef SUX_MSD_WHATIF
      // diagnostic build only (tools/msd_whatif.sh; the output is NOT bucket-sorted): the stage
      // store at the record's own, conflict-free slot, without the bucket-start read — what pass A
      // would cost if its two random LDS accesses per record had no bank conflicts
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j)
        if (rank[j] != ~0u) stage[wave * (PT * kWave) + j * kWave + lane] = rv[j];
#else
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j)
        if (rank[j] != ~0u) stage[wc[wave * NB + h[j]] + rank[j]] = rv[j];
#endif
      __syncthreads();
      // the chunk goes back to its own place, in bucket order: one contiguous write
#pragma unroll
      for (uint32_t q = 0; q < PT; ++q) {
        const uint32_t i = tid + q * NT;
        if (i < k.n) t4[k.c0 + i] = stage[i];
      }
    }
    for (uint32_t hb = tid; hb < nbk; hb += NT)
      offs[(uint64_t)it * nbk + hb] = (uint16_t)wc[hb];  // wc[0][hb]: bucket start in the chunk
    __syncthreads();
    for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
    __syncthreads();
  }
}

// Pass A with its next chunk prefetched by LDS-DMA (msd_direct bit 2, round 4): one 512-thread
// workgroup per CU and two 64 KB chunk buffers in LDS.  While chunk k is ranked, bucket-sorted
// in place in its buffer and written back, chunk k + 1 streams into the other buffer through
// global_load_lds_dwordx4 (no VGPRs: the two-workgroup k_msd16a has no registers for a second
// chunk and no prefetch at all).  Barriers inside the loop are raw (lds_barrier), so the
// prefetch stays in flight across them; the only vmcnt(0) is at the top of an iteration, where
// the chunk about to be read must have landed.  Same bytes as k_msd16a.
template <int KW, uint32_t DB, uint32_t LO>
__global__ __launch_bounds__(512, 1) void k_msd16a_dma(PartDev pd, MapGroup g, uint32_t cpm,
                                                      uint32_t nbk, uint16_t* __restrict__ offs,
                                                      uint16_t* __restrict__ pids_out,
                                                      uint8_t* __restrict__ tmp) {
  resolve_seed(pd);
  constexpr uint32_t NW = 8, NB = 1u << DB, NT = NW * kWave, CH = kM16Chunk, PT = CH / NT;
  __shared__ __attribute__((aligned(16))) u32x4 buf0[CH];
  __shared__ __attribute__((aligned(16))) u32x4 buf1[CH];
  __shared__ uint16_t wc[NW * NB];
  __shared__ uint32_t wsum[NW];
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const int kw0 = pd.key_offset / 4;
  const u32x4* recs = reinterpret_cast<const u32x4*>(g.recs);
  u32x4* t4 = reinterpret_cast<u32x4*>(tmp);
  const uint32_t items = g.num_maps * cpm, G = gridDim.x, b = xcd_map(blockIdx.x, G);
  const uint32_t it0 = (uint32_t)((uint64_t)items * b / G), it1 = (uint32_t)((uint64_t)items * (b + 1) / G);
  struct Item {
    uint64_t c0;
    uint32_t n;
  };
  auto item = [&](uint32_t it) {
    const uint32_t m = it / cpm, c = it - m * cpm;
    Item k;
    k.c0 = (uint64_t)m * g.records_per_map + (uint64_t)c * CH;
    k.n = it < it1 ? m16_chunk_len(m16_map_len(g, m), c) : 0u;
    return k;
  };
  // the chunk's records, in order, land linearly in `dst` (a wave-instruction writes 1 KB: the
  // LDS address is wave-uniform + 16 x lane); records past a short chunk re-read its last one
  auto prefetch = [&](const Item& k, u32x4* dst) {
    if (k.n == 0) return;
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
      const uint32_t e0 = wave * (PT * kWave) + j * kWave;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(recs + k.c0 + min(e0 + (uint32_t)lane, k.n - 1)),
          (__attribute__((address_space(3))) void*)(dst + e0), 16, 0, 0);
    }
  };
  for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
  if (it0 < it1) prefetch(item(it0), buf0);
  for (uint32_t it = it0; it < it1; ++it) {
    u32x4* cur = ((it - it0) & 1) ? buf1 : buf0;
    u32x4* nxt = ((it - it0) & 1) ? buf0 : buf1;
    const Item k = item(it);
    __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA of chunk `it` (and earlier stores) done
    lds_barrier();                  // ... and every other wave's; nxt was last read before here
    if (it + 1 < it1) prefetch(item(it + 1), nxt);
    u32x4 rv[PT];
    uint32_t h[PT], rank[PT];
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) rv[j] = cur[wave * (PT * kWave) + j * kWave + lane];
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
      const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
      const bool valid = e < k.n;
      uint32_t p = 0;
      if (valid) {
        p = m16_pid<KW>(pd, rv[j], kw0);
        if (pids_out) pids_out[k.c0 + e] = (uint16_t)p;
      }
      h[j] = (p >> LO) & (NB - 1);
      rank[j] = wave_rank<DB, uint16_t>(h[j], valid, wc + wave * NB, lt_mask);
    }
    lds_barrier();
    scan_digit_wave16<NB, NW, true>(wc, wsum, tid, lane, wave);
    // every wave read its records of `cur` before the first barrier above: sort them into it
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j)
      if (rank[j] != ~0u) cur[wc[wave * NB + h[j]] + rank[j]] = rv[j];
    lds_barrier();
    // the chunk goes back to its own place, in bucket order: one contiguous write
#pragma unroll
    for (uint32_t q = 0; q < PT; ++q) {
      const uint32_t i = tid + q * NT;
      if (i < k.n) t4[k.c0 + i] = cur[i];
    }
    for (uint32_t hb = tid; hb < nbk; hb += NT)
      offs[(uint64_t)it * nbk + hb] = (uint16_t)wc[hb];  // wc[0][hb]: bucket start in the chunk
    lds_barrier();
    for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
  }
}

// K2 of the MSD path: one workgroup (kScanThreads) per map.  Bucket totals over the map's chunks,
// exclusive scan over buckets -> segbase[m][h] (record index in the group's output), the index
// table's last entry and, at world 1, the peer byte count.  A bucket's total is S[h+1] - S[h]
// with S[h] = the sum over chunks of the bucket's start in the chunk (offs) and S[nbk] = the map's
// records: one u16 read per (chunk, bucket), a thread per bucket with 16 reads in flight (round
// 3's two dependent reads per chunk kept each launch ~0.76 ms: 256 chunks of latency in a row).
__global__ __launch_bounds__(kScanThreads) void k_msd16_scan(MapGroup g, uint32_t cpm, uint32_t nbk,
                                                             const uint16_t* __restrict__ offs,
                                                             uint64_t* __restrict__ segbase,
                                                             int64_t* __restrict__ index,
                                                             uint8_t* __restrict__ index_be,
                                                             uint64_t* __restrict__ peer_bytes,
                                                             int R) {
  constexpr uint32_t HG = kScanThreads;  // one thread per bucket (nbk <= 1024)
  constexpr uint32_t U = 16;             // chunk reads in flight per thread
  __shared__ uint64_t sh[2 * kWave + 1];
  __shared__ uint32_t colsum[HG + 1];
  const uint32_t m = blockIdx.x, tid = threadIdx.x;
  const uint32_t len = m16_map_len(g, m), nch = (len + kM16Chunk - 1) / kM16Chunk;
  uint32_t S = 0;
  if (tid < nbk) {
    const uint16_t* om = offs + (uint64_t)m * cpm * nbk + tid;
    uint32_t c = 0;
    for (; c + U <= nch; c += U) {
      uint32_t v[U];
#pragma unroll
      for (uint32_t k = 0; k < U; ++k) v[k] = om[(uint64_t)(c + k) * nbk];
#pragma unroll
      for (uint32_t k = 0; k < U; ++k) S += v[k];
    }
    for (; c < nch; ++c) S += om[(uint64_t)c * nbk];
  }
  // S[nbk] = every chunk's records: written by thread nbk (or thread 0 when nbk == HG)
  colsum[tid] = tid == nbk ? len : S;
  if (tid == 0 && nbk == HG) colsum[HG] = len;
  __syncthreads();
  const uint64_t v = tid < nbk ? (uint64_t)(colsum[tid + 1] - colsum[tid]) : 0u;
  uint64_t tot;
  const uint64_t ex = block_excl_scan(v, sh, &tot);
  if (tid < nbk) segbase[(uint64_t)m * nbk + tid] = (uint64_t)m * g.records_per_map + ex;
  if (tid == 0) {
    const int64_t off = (int64_t)len * g.rec_size;
    index[(uint64_t)m * (R + 1) + R] = off;
    if (index_be) reinterpret_cast<uint64_t*>(index_be)[(uint64_t)m * (R + 1) + R] = bswap64((uint64_t)off);
    if (m == 0 && peer_bytes) peer_bytes[0] = g.num_records * g.rec_size;
  }
}

template <int KW, uint32_t NW, uint32_t PT, uint32_t LO, uint32_t MCH, bool DIRECT = false,
          bool ERUN = false, bool PIPE = false>
__global__ __launch_bounds__(NW * 64, 4) void k_msd16b(PartDev pd, MapGroup g, uint32_t cpm,
                                                 uint32_t nbk, const uint16_t* __restrict__ offs,
                                                 const uint64_t* __restrict__ segbase,
                                                 const uint8_t* __restrict__ tmp,
                                                 uint8_t* __restrict__ out,
                                                 int64_t* __restrict__ index,
                                                 uint8_t* __restrict__ index_be) {
  resolve_seed(pd);
  using K = M16b<NW, PT, LO, MCH>;
  constexpr uint32_t NB = K::NB, NT = K::NT, CAP = K::CAP, MC = MCH, PB = 1u << LO;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  u32x4* stage = reinterpret_cast<u32x4*>(lds8);
  uint32_t* wc = reinterpret_cast<uint32_t*>(stage + CAP);  // [NW][NB]
  uint32_t* cur = wc + NW * NB;
  uint32_t* wsum = cur + NB;
  uint8_t* los = reinterpret_cast<uint8_t*>(wsum + NW);
  uint32_t* rp = reinterpret_cast<uint32_t*>(los + CAP);   // [MC + 1] run starts in the segment
  uint16_t* ro = reinterpret_cast<uint16_t*>(rp + MC + 1);  // [MC] run starts in their chunk
  // ERUN (msd_direct bit 4): element -> run map of a segment that fits the stage, over the
  // stage's first 2 CAP bytes (idle between place() and the next rank_stage): one LDS read per
  // element instead of the run table's log2(MC)-step search
  uint16_t* erun = reinterpret_cast<uint16_t*>(lds8);
  // PIPE (msd_direct bit 5, round 6): the next segment's records are gathered into registers
  // while this one's sorted stage is written out, so the element map cannot share the stage: it
  // gets its own u8 region after the kernel's LDS (maps of <= 256 chunks)
  uint8_t* erun8 = lds8 + K::lds_bytes();
  static_assert(!PIPE || (ERUN && !DIRECT), "PIPE runs on the element map, stage path");
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
    if constexpr (ERUN) {
      if (s.T <= CAP) {
        for (uint32_t c = tid; c < s.nch; c += NT)
          for (uint32_t k = rp[c], e = rp[c + 1]; k < e; ++k) {
            if constexpr (PIPE) erun8[k] = (uint8_t)c;
            else erun[k] = (uint16_t)c;
          }
        __syncthreads();
      }
    }
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
    if constexpr (ERUN) {
      if (s.T <= CAP) {
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j) lo[j] = PIPE ? (uint32_t)erun8[ev[j]] : (uint32_t)erun[ev[j]];
#pragma unroll
        for (uint32_t j = 0; j < PT; ++j)
          r[j] = t4[s.mbase + (uint64_t)lo[j] * kM16Chunk + ro[lo[j]] + (ev[j] - rp[lo[j]])];
        return;
      }
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
      r[j] = t4[s.mbase + (uint64_t)lo[j] * kM16Chunk + ro[lo[j]] + (ev[j] - rp[lo[j]])];
    }
  };
  auto digit = [&](const Seg& s, const u32x4& r) {
    return (m16_pid<KW>(pd, r, kw0) - (s.h << LO)) & (NB - 1);
  };
  // stable rank by pid & 31 -> stage/los in sorted order; wc[0][l] = digit starts afterwards.
  // DIRECT: the sorted positions stay in registers (pos[j], ~0u for none) for place_direct
  uint32_t dl[PT], dp[PT];
  auto rank_stage = [&](const Seg& s, uint32_t n, const u32x4 (&r)[PT]) {
    uint32_t lo[PT], rk[PT];
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
      const uint32_t e = wave * (PT * kWave) + j * kWave + lane;
      const bool valid = e < n;
      lo[j] = valid ? digit(s, r[j]) : 0u;
      rk[j] = wave_rank<LO>(lo[j], valid, wc + wave * NB, lt_mask);
    }
    __syncthreads();
    scan_digit_wave<NB, NW>(wc, wsum, tid, lane, wave);
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j)
      if (rk[j] != ~0u) {
        const uint32_t pos = wc[wave * NB + lo[j]] + rk[j];
        if constexpr (DIRECT) {
          dl[j] = lo[j];
          dp[j] = pos;
        } else {
          stage[pos] = r[j];
          los[pos] = (uint8_t)lo[j];
        }
      } else if constexpr (DIRECT) {
        dp[j] = ~0u;
      }
  };
  auto write_index = [&](const Seg& s, uint32_t start_l) {
    const uint64_t seg_out = s.out;
    const uint32_t p = (s.h << LO) + (uint32_t)tid;  // in-segment record offset of partition p
    if (tid < (int)PB && p < (uint32_t)R) {
      const int64_t off = (int64_t)((seg_out - s.mbase + start_l) * g.rec_size);
      index[(uint64_t)s.m * (R + 1) + p] = off;
      if (ibe) ibe[(uint64_t)s.m * (R + 1) + p] = bswap64((uint64_t)off);
    }
  };
  // sorted stage -> output through the per-partition cursors; cursors advance; wc cleared.
  // DIRECT: every record from its registers to cur[l] + its rank among the piece's digit l
  auto place = [&](const Seg& s, uint32_t n, const u32x4 (&r)[PT]) {
    if constexpr (DIRECT) {
#pragma unroll
      for (uint32_t j = 0; j < PT; ++j)
        if (dp[j] != ~0u) out4[s.mbase + cur[dl[j]] + (dp[j] - wc[dl[j]])] = r[j];
    } else {
#pragma unroll
      for (uint32_t q = 0; q < PT; ++q) {
        const uint32_t i = tid + q * NT;
        if (i < n) {
          const uint32_t l = los[i];
          out4[s.mbase + cur[l] + (i - wc[l])] = stage[i];
        }
      }
    }
    uint32_t ncur = 0;
    if (tid < (int)NB) ncur = cur[tid] + ((uint32_t)tid + 1 < NB ? wc[tid + 1] : n) - wc[tid];
    // PIPE: the next segment's gather is in flight here — a __syncthreads() fence would wait for
    // it (vmcnt(0)); these barriers only order LDS accesses, so a raw one keeps it flying
    if constexpr (PIPE) lds_barrier(); else __syncthreads();
    if (tid < (int)NB) cur[tid] = ncur;
    for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
    if constexpr (PIPE) lds_barrier(); else __syncthreads();
  };

  for (uint32_t i = tid; i < NW * NB; i += NT) wc[i] = 0;
  __syncthreads();
  if (it0 >= it1) return;
  Seg s = build(it0, prefetch(it0));
  u32x4 rv[PT];
  // a segment larger than the stage (skewed keys): count the digits, then place piece by piece
  auto multi_segment = [&](const Seg& s) {
    const uint32_t seg_rel = (uint32_t)(s.out - s.mbase);
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
    for (uint32_t e0 = 0; e0 < s.T; e0 += CAP) {
      load(s, e0, rv);
      const uint32_t n = min(CAP, s.T - e0);
      rank_stage(s, n, rv);
      __syncthreads();
      __syncthreads();
      place(s, n, rv);
    }
  };
  if constexpr (PIPE) {
    // segment s's records are in rv when its iteration starts; after s is ranked into the
    // stage, the next segment's run table is built and its records are gathered into rv while
    // s's stage goes out (place) — the gather's latency hides behind the stores instead of
    // stalling every segment (round 2 stamps: ~half a segment waited on its loads)
    if (s.T <= CAP) load(s, 0, rv);
    for (uint32_t it = it0; it < it1; it += G) {
      const bool have = it + G < it1;
      const Pre pre = prefetch(it + G);  // the next run table's reads fly during this segment
      if (s.T > CAP) {
        multi_segment(s);
        if (have) {
          s = build(it + G, pre);
          if (s.T <= CAP) load(s, 0, rv);
        }
        continue;
      }
      const uint32_t seg_rel = (uint32_t)(s.out - s.mbase);
      const uint32_t n = s.T;
      rank_stage(s, n, rv);
      __syncthreads();
      if (tid < (int)NB) cur[tid] = seg_rel + wc[tid];
      write_index(s, tid < (int)NB ? wc[tid] : 0u);
      __syncthreads();
      Seg nx = s;
      if (have) {
        nx = build(it + G, pre);  // rp / ro / erun8: place() reads none of them
        if (nx.T <= CAP) load(nx, 0, rv);
      }
      place(s, n, rv);  // the stage path: reads stage / los / cur / wc, not rv
      s = nx;
    }
    return;
  }
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
      place(s, n, rv);
      SUX_MSD_STAMP(3);
    }
    if (it + G < it1) s = build(it + G, prefetch(it + G));
    SUX_MSD_STAMP(4);
  }
  SUX_MSD_STAMP_END();
}
// ------------------------------------------------------------------------------------------
// host launchers (called by launch_partition_group, sux_partition.hip)
// ------------------------------------------------------------------------------------------
// The MSD small-record path (k_msd16a / k_msd16_scan / k_msd16b) applies: tuning small_kernel 4,
// 16-byte records with a fixed-width key in the first 16 bytes, 1024 < R <= 16384, 16-byte
// aligned input and output, map-major layout, maps of <= MC chunks, and a workspace with the
// temp copy (its chunk-offset table lives in the counts region, the segment bases in the totals
// region).  Returns the bucket width LO it runs with (16 partitions per bucket; 256 for maps too
// short for 16), 0 when it does not apply.
static uint32_t msd16_lo(const PartDev& pd, const MapGroup& g, const LayoutDesc& lay,
                         const uint8_t* d_out, const Workspace& ws, const Tuning& tn) {
  if (tn.small_kernel != 4 || g.rec_size != 16 || lay.world != 1) return 0;
  if (pd.R <= 1024 || pd.R > 16384 || pd.kind == 4 || pd.key_offset % 4 != 0 ||
      pd.key_offset + pd.key_len > 16)
    return 0;
  if (((reinterpret_cast<uintptr_t>(g.recs) | reinterpret_cast<uintptr_t>(d_out)) & 15) != 0)
    return 0;
  const uint64_t cpm = (g.records_per_map + kM16Chunk - 1) / kM16Chunk;
  if (cpm < 1 || ws.tmp_bytes < g.num_records * 16) return 0;
  for (const uint32_t lo : {(tn.msd_direct & 8) ? kM16LoWide : kM16Lo, kM16LoShort}) {
    const uint64_t nbk = ((uint64_t)pd.R + (1u << lo) - 1) >> lo;
    if (cpm > (lo == kM16LoShort ? kM16MaxChunksShort : kM16MaxChunks)) continue;
    // by default only when a (map, bucket) segment holds >= 1024 records on average: a segment
    // costs ~6 us of run table, search and barriers whatever its size (64 Ki-record maps at
    // R = 10 000 and 16 partitions per bucket: 105-record segments, 194 GB/s vs 553 for the
    // sorted-chunk scatter; 2^20-record maps: 1677-record segments, 1027 vs 750 GB/s) — short
    // maps take 256-partition buckets, longer segments again
    if (tn.small_auto && g.records_per_map < 1024 * nbk) continue;
    if ((uint64_t)g.num_maps * cpm * nbk * 2 <= ws.counts_bytes &&
        (uint64_t)g.num_maps * nbk * 8 <= ws.totals_bytes)
      return lo;
  }
  return 0;
}

bool msd16_eligible(const PartDev& pd, const MapGroup& g, const LayoutDesc& lay,
                    const uint8_t* d_out, const Workspace& ws, const Tuning& tn) {
  return msd16_lo(pd, g, lay, d_out, ws, tn) != 0;
}

hipError_t launch_msd16(const PartDev& pd, const MapGroup& g, uint8_t* d_out, int64_t* d_index,
                        uint8_t* d_index_be, uint16_t* d_pids, uint8_t* d_ws, const Workspace& ws,
                        uint64_t* d_peer_bytes, const Tuning& tn, Timer* timer, hipStream_t s) {
  const int R = pd.R;
  const uint32_t ncu = (uint32_t)std::max(1, stream_cus(s));
  const uint32_t cpm = (uint32_t)((g.records_per_map + kM16Chunk - 1) / kM16Chunk);
  const LayoutDesc lay1{1, 16};
  const uint32_t LO = msd16_lo(pd, g, lay1, d_out, ws, tn);
  if (LO == 0) return hipErrorInvalidValue;  // (the caller checked msd16_eligible)
  const uint32_t nbk = ((uint32_t)R + (1u << LO) - 1) >> LO;
  uint16_t* offs = reinterpret_cast<uint16_t*>(d_ws + ws.counts_off);  // [map][chunk][bucket]
  uint64_t* segbase = reinterpret_cast<uint64_t*>(d_ws + ws.totals_off);  // [map][bucket]
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
#define SUX_M16A_D(KW, DB, LOV, D, A, T)                                                           \
  do {                                                                                             \
    constexpr size_t ldsa = M16a<NWA, DB, A ? 4 : 2, T>::lds_bytes();                              \
    static_assert(2 * ldsa <= 160 * 1024, "pass A: two workgroups per CU");                       \
    allow_lds(reinterpret_cast<const void*>(&k_msd16a<KW, NWA, DB, LOV, D, A, T>), ldsa);          \
    hipLaunchKernelGGL((k_msd16a<KW, NWA, DB, LOV, D, A, T>), ga, dim3(NWA * kWave), ldsa, s, pd,  \
                       g, cpm, nbk, offs, d_pids, tmp);                                            \
  } while (0)
  // msd_direct bit 6: the atomic ranking (u32 counters: 32-partition buckets, digits <= 9 bits);
  // bit 7: the tag match (same shapes)
  const bool atom_a = (tn.msd_direct & 64) && !(tn.msd_direct & 5) && LO == kM16LoWide;
  const bool tag_a = (tn.msd_direct & 128) && !(tn.msd_direct & 69) && LO == kM16LoWide;
#define SUX_M16A_X(KW, DB, LOV, ATOM_OK)                                                   \
  do {                                                                                     \
    if (tn.msd_direct & 4) {                                                               \
      const dim3 gd(std::min<uint32_t>(g.num_maps * cpm, ncu));                            \
      hipLaunchKernelGGL((k_msd16a_dma<KW, DB, LOV>), gd, dim3(512), 0, s, pd, g, cpm, nbk, \
                         offs, d_pids, tmp);                                               \
    } else if (tn.msd_direct & 1) {                                                        \
      SUX_M16A_D(KW, DB, LOV, true, false, false);                                         \
    } else if (ATOM_OK && atom_a) {                                                        \
      SUX_M16A_D(KW, DB, LOV, false, ATOM_OK, false);                                      \
    } else if (ATOM_OK && tag_a) {                                                         \
      SUX_M16A_D(KW, DB, LOV, false, false, ATOM_OK);                                      \
    } else {                                                                               \
      SUX_M16A_D(KW, DB, LOV, false, false, false);                                        \
    }                                                                                      \
  } while (0)
#define SUX_M16A(KW, DB, LOV) SUX_M16A_X(KW, DB, LOV, (LOV == kM16LoWide && DB <= 9))
#define SUX_M16AK(DB, LOV)                   \
  do {                                       \
    if (kw <= 1) SUX_M16A(1, DB, LOV);       \
    else if (kw == 2) SUX_M16A(2, DB, LOV);  \
    else if (kw == 3) SUX_M16A(3, DB, LOV);  \
    else SUX_M16A(4, DB, LOV);               \
  } while (0)
  // pass A's digit is the bucket pid >> LO: the template's LO must be the LO chosen above
  if (LO == kM16LoShort) SUX_M16AK(6, kM16LoShort);  // R <= 16384: <= 64 buckets
  else if (LO == kM16LoWide && nbk > 256) SUX_M16AK(9, kM16LoWide);  // R <= 16384: <= 512
  else if (LO == kM16LoWide) SUX_M16AK(8, kM16LoWide);
  else if (nbk > 512) SUX_M16AK(10, kM16Lo);
  else if (nbk > 256) SUX_M16AK(9, kM16Lo);
  else SUX_M16AK(8, kM16Lo);
#undef SUX_M16AK
#undef SUX_M16A
#undef SUX_M16A_X
#undef SUX_M16A_D
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
  const dim3 gb(std::min<uint32_t>(g.num_maps * nbk, ncu * (LO == kM16LoWide ? 1 : 2) * wpc));
  using MB4 = M16b<NWB, PTB, kM16Lo, kM16MaxChunks>;
  using MB5 = M16b<8, PTB, kM16LoWide, kM16MaxChunks>;
  static_assert(2 * MB5::lds_bytes() <= 160 * 1024, "pass B (32-partition buckets): two per CU");
  using MB8 = M16b<NWB, PTB, kM16LoShort, kM16MaxChunksShort>;
  static_assert(4 * MB4::lds_bytes() <= 160 * 1024, "pass B: four workgroups per CU");
  static_assert(4 * MB8::lds_bytes() <= 160 * 1024, "pass B (256-partition buckets): four per CU");
  static_assert(2 * M16a<NWA, 10>::lds_bytes() <= 160 * 1024, "pass A: two workgroups per CU");
#define SUX_M16B_P(KW, LOV, MCV, D, ER, P)                                                         \
  do {                                                                                             \
    constexpr uint32_t nwb = LOV == kM16LoWide ? 8 : NWB;                                          \
    using MBK = M16b<nwb, PTB, LOV, MCV>;                                                          \
    constexpr size_t ldsb = MBK::lds_bytes() + (P ? MBK::CAP : 0);                                 \
    static_assert(!P || 2 * ldsb <= 160 * 1024, "pipelined pass B: two workgroups per CU");      \
    allow_lds(reinterpret_cast<const void*>(&k_msd16b<KW, nwb, PTB, LOV, MCV, D, ER, P>), ldsb);  \
    hipLaunchKernelGGL((k_msd16b<KW, nwb, PTB, LOV, MCV, D, ER, P>), gb, dim3(nwb * kWave), ldsb, \
                       s, pd, g, cpm, nbk, offs, segbase, tmp, d_out, d_index, d_index_be);        \
  } while (0)
#define SUX_M16B_D(KW, LOV, MCV, D, ER) SUX_M16B_P(KW, LOV, MCV, D, ER, false)
  // msd_direct bit 5: pass B gathers the next segment while the current one is written out
  // (32-partition buckets, element map, maps of <= 256 chunks)
  const bool pipe_b = (tn.msd_direct & 32) && (tn.msd_direct & 16) && !(tn.msd_direct & 2) &&
                      LO == kM16LoWide && cpm <= 256;
#define SUX_M16B(KW, LOV, MCV)                                      \
  do {                                                              \
    if (tn.msd_direct & 2) SUX_M16B_D(KW, LOV, MCV, true, false);   \
    else if (pipe_b && LOV == kM16LoWide) SUX_M16B_P(KW, kM16LoWide, kM16MaxChunks, false, true, true); \
    else if (tn.msd_direct & 16) SUX_M16B_D(KW, LOV, MCV, false, true); \
    else SUX_M16B_D(KW, LOV, MCV, false, false);                    \
  } while (0)
#define SUX_M16BK(LOV, MCV)                   \
  do {                                        \
    if (kw <= 1) SUX_M16B(1, LOV, MCV);       \
    else if (kw == 2) SUX_M16B(2, LOV, MCV);  \
    else if (kw == 3) SUX_M16B(3, LOV, MCV);  \
    else SUX_M16B(4, LOV, MCV);               \
  } while (0)
  if (LO == kM16LoShort) SUX_M16BK(kM16LoShort, kM16MaxChunksShort);
  else if (LO == kM16LoWide) SUX_M16BK(kM16LoWide, kM16MaxChunks);
  else SUX_M16BK(kM16Lo, kM16MaxChunks);
#undef SUX_M16BK
#undef SUX_M16B
#undef SUX_M16B_D
#undef SUX_M16B_P
  timer_end(timer, kScatter, s);
  return hipGetLastError();
}

hipError_t launch_hist16(const PartDev& pd, const MapGroup& g, uint16_t* pids, uint32_t* counts,
                         hipStream_t s) {
  const uint32_t ncu = (uint32_t)std::max(1, stream_cus(s));
  const size_t lds = (size_t)pd.R * 4;
  const int kw = (pd.key_len + 3) / 4;
  const dim3 gridp(std::min<uint32_t>(g.num_maps * g.tiles_per_map,
                                      ncu * std::max<uint32_t>(1, (160u * 1024) / (uint32_t)lds)));
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
  return hipGetLastError();
}

hipError_t launch_scatter16(const MapGroup& g, int R, int pid_bits, const uint16_t* pids,
                            const uint32_t* prefix, const uint64_t* base, uint8_t* d_out,
                            const Tuning& tn, Timer* timer, hipStream_t s) {
  const uint32_t ncu = (uint32_t)std::max(1, stream_cus(s));
  const uint32_t total_tiles = g.num_maps * g.tiles_per_map;
  if (R <= kS16sMaxR && tn.small_kernel != 1) {
    timer_note(timer, kScatter, "k_scatter16s");
    const size_t lds = Sc16s::lds_bytes(R);
    allow_lds(reinterpret_cast<const void*>(&k_scatter16s), lds);
    const dim3 grid(std::min<uint32_t>(total_tiles, ncu));  // one LDS-bound workgroup per CU
    hipLaunchKernelGGL(k_scatter16s, grid, dim3(1024), lds, s, g, R, pid_bits, pids, prefix, base,
                       d_out);
    return hipGetLastError();
  }
  timer_note(timer, kScatter, "k_scatter16b");
  const size_t lds = (size_t)R * 4;
  const uint32_t per_cu = std::max<uint32_t>(1, std::min<uint32_t>(2, (160u * 1024) / (uint32_t)lds));
  const dim3 grid(std::min<uint32_t>(total_tiles, ncu * per_cu));
  const int gb = tn.small_groups;  // 64-record groups per turn
#define SUX_S16B(GB)                                                                               \
  do {                                                                                             \
    allow_lds(reinterpret_cast<const void*>(&k_scatter16b<16, GB>), lds);                          \
    hipLaunchKernelGGL((k_scatter16b<16, GB>), grid, dim3(1024), lds, s, g, R, pid_bits, pids,     \
                       prefix, base, d_out);                                                       \
  } while (0)
  if (gb == 1) SUX_S16B(1);
  else if (gb == 2) SUX_S16B(2);
  else SUX_S16B(4);
#undef SUX_S16B
  return hipGetLastError();
}

}  // namespace sux
