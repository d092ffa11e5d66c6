// sux_onepass.hip — one-pass map side for fixed-size records, gfx950.
//
// The three-kernel path (sux_partition.hip: K1 hist, K2 scans, K3 scatter) needs a map batch's
// whole histogram before its first record can be placed, so every record crosses the fabric
// three times (K1 reads it for its key, K3 reads and writes it): 3·N·S bytes of HBM traffic for
// the 2·N·S algorithmic bytes, and the XCD↔IOD fabric, not HBM, is what bounds both kernels.
//
// Here a map batch is held ON CHIP while its histogram forms.  One persistent launch, one
// 1024-thread workgroup per CU (LDS-bound).  For every map batch each workgroup takes one slice
// of ≤ 1024 records (≤ 100 KB at S = 100; one record per thread) into registers:
//   count   key → partition id (P1, as K1), stable per-wave ranks by ballot match (as K3), the
//           slice's per-partition counts published write-through (sc1) to the sync workspace;
//   scan    two levels, each run by the LAST arriver of its level (agent-scope atomic counter,
//           the value its add returned tells it so): a group of 32 consecutive slices (the
//           workgroups one XCD gets under xcd_map) → exclusive prefix of every slice per
//           partition + group totals; then the last group → partition totals, the map's index
//           file (P3, native + big-endian) and every group's offsets, published through one
//           done-flag per group;
//   place   the slice goes registers → partition-sorted LDS image in destination-unit space →
//           aligned 16-byte stores (K3 v7's image), each run's head/tail unit partial (dword
//           stores of only this slice's dwords; the neighbouring slice writes the rest).
// Pipelined one map deep: map m+1 is counted and its scan is in flight while map m is placed,
// and map m+2's loads fly during map m's write-out.  A map batch therefore holds at most
// gridDim × 1024 records (2^18 = 26 MB at 256 CUs); every record is read once and written once.
//
// Visibility (MI355X_MICROARCH.md, inter-workgroup hand-offs): every handed-off word is stored
// sc1 and loaded sc1, each storing wave drains with s_waitcnt vmcnt(0) before its workgroup's
// one lane signals (agent-scope add or sc1 flag store), consumers poll with sc1 loads and read
// behind a workgroup barrier.  Every spin is bounded (s_memrealtime): a grid that is not fully
// resident sets the abort word and the launch drains instead of hanging.
//
// Stability: slices are consecutive record ranges in slice order, records inside a slice in
// order (waves in order, ballot ranks inside a wave), so a partition keeps input order — the
// byte layout of the three-kernel path and of Spark's writers (P2), bit for bit.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "sux_internal.h"

namespace sux {

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

namespace onepass {
constexpr int kWave = 64;
}
using onepass::kWave;

// P1: partition functions — sux_p1.h
#include "sux_p1.h"

namespace onepass {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kGroup = 32;           // slices per scan group
constexpr uint32_t kMaxGroups = 16;
constexpr uint64_t kSpinTicks = 200000000;  // s_memrealtime runs at 100 MHz: 2 s

// sync words (u32), one 256-byte line each: per-map arrival counters in a ring of kSlots,
// kMaxGroups replicas each (every slice adds to all replicas of its map; a slice polls its
// group's), then the abort word
constexpr uint32_t kLine = 64;
constexpr uint32_t kSlots = 4;
constexpr uint32_t kAbort = kSlots * kMaxGroups * kLine;
constexpr uint32_t kSyncWords = kAbort + kLine;
// ring depths: counts of maps m..m+2 are live at once (4 buffers); the group totals of map m
// are cleared by slice 0 at map m+2 and refilled for map m+6 (6 buffers)
constexpr uint32_t kCntBufs = 4;
constexpr uint32_t kGtBufs = 6;

__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t add_agent(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    uint32_t t = __shfl_up(v, d, kWave);
    if (lane >= d) v += t;
  }
  return v;
}

__device__ __forceinline__ uint64_t bswap64(uint64_t v) {
  return ((uint64_t)__builtin_bswap32((uint32_t)v) << 32) | __builtin_bswap32((uint32_t)(v >> 32));
}

template <uint32_t S, uint32_t NW>
struct Shape {
  static constexpr uint32_t NT = NW * kWave;
  static constexpr uint32_t C = NT;  // records per slice: one per thread
  static constexpr uint32_t W = S / 4;
  static constexpr uint32_t kUnits = (C * S + 12 + 15) / 16;
  static constexpr uint32_t kPer = (kUnits + NT - 1) / NT;
  static constexpr uint32_t kRecUnits = (S + 15) / 16 + 1;
  static_assert(S % 4 == 0 && NW % 4 == 0, "shape");
  // image units: the slice's bytes + per-run head padding (<= 3 dwords) and tail slack,
  // rounded to 4 so that the u32x4 arrays behind dstu[SP] stay 16-byte aligned
  static __host__ __device__ constexpr uint32_t space(int R) {
    return ((C * S) / 16 + (3u * R + 1) / 2 + 1 + 3) & ~3u;
  }
  // img[SP] u32x4 | dstu[SP] | pinfo[R] u32x4 | recoff[C] | wcnt[R][NW] | u0s[R] | tmp[NW] | flags[4]
  static __host__ __device__ constexpr uint32_t lds_bytes(int R) {
    return space(R) * 16 + space(R) * 4 + (uint32_t)R * 16 + C * 4 + NW * (uint32_t)R * 4 +
           (uint32_t)R * 4 + NW * 4 + 16;
  }
};

// Diagnostic build only (-DSUX_OP_STAMPS, tools/op_stamps.hip): thread 0 of workgroups < 64
// records s_memtime at the phase boundaries of maps < 64.  No stamp executes otherwise.
#ifdef SUX_OP_STAMPS
__device__ uint64_t g_op_stamps[64][64][16];
#define SUX_OP_STAMP(m, ph)                                                      \
  do {                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < 64 && (m) < 64)                         \
      g_op_stamps[blockIdx.x][(m)][(ph)] = __builtin_amdgcn_s_memtime();        \
  } while (0)
#else
#define SUX_OP_STAMP(m, ph) \
  do {                      \
  } while (0)
#endif

struct SyncWs {
  uint32_t* sync;  // kSyncWords: arrival counters [kSlots][kMaxGroups replicas], abort word
  uint32_t* cnt;   // [kCntBufs][nwg][R]   slice counts, stored sc1
  uint32_t* gt;    // [kGtBufs][kMaxGroups][R]  group totals, agent-scope atomic adds
};

// Per-map state a workgroup carries in registers: the slice's 16-byte units, its records' keys,
// and once counted, each record's partition and rank inside (slice, partition) + the owner
// thread's count.
template <uint32_t PER, int KW>
struct Set {
  u32x4 v[PER];
  uint32_t k[KW];
  uint32_t pid, jr, c, off;
};

// MINW: waves per SIMD the launch needs resident (workgroups per CU x NW / 4) — caps the VGPRs
template <uint32_t S, uint32_t NW, int KW, int MINW>
__global__ __launch_bounds__(NW * 64, MINW) void k_onepass(PartDev pd, MapGroup g,
                                                     uint8_t* __restrict__ out,
                                                     int64_t* __restrict__ index,
                                                     uint8_t* __restrict__ index_be,
                                                     uint16_t* __restrict__ pids, SyncWs sw,
                                                     uint32_t cs) {
  using K = Shape<S, NW>;
  using St = Set<K::kPer, KW>;
  constexpr uint32_t NT = K::NT, W = K::W, PER = K::kPer;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const int R = pd.R;
  const uint32_t SP = K::space(R);
  u32x4* img = reinterpret_cast<u32x4*>(lds8);
  uint32_t* img32 = reinterpret_cast<uint32_t*>(lds8);
  uint32_t* dstu = reinterpret_cast<uint32_t*>(img + SP);
  u32x4* pinfo = reinterpret_cast<u32x4*>(dstu + SP);  // {lb, cd | keep << 8, full, sp}
  uint32_t* recoff = reinterpret_cast<uint32_t*>(pinfo + R);
  uint32_t* wcnt = recoff + K::C;  // [R][NW]
  uint32_t* u0s = wcnt + NW * R;
  uint32_t* tmp = u0s + R;
  int* flags = reinterpret_cast<int*>(tmp + NW);

  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const bool owner = tid < R;  // thread p owns partition p
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const uint32_t nwg = gridDim.x;
  const uint32_t s = xcd_map(blockIdx.x, nwg);  // this workgroup's slice of every map
  const uint32_t grp = s / kGroup, ngr = (nwg + kGroup - 1) / kGroup;
  const uint32_t g0 = grp * kGroup;  // first slice of my group
  const uint32_t M = g.num_maps;
  const int n_owner_waves = (R + kWave - 1) / kWave;
  int pid_bits = 0;
  while ((1 << pid_bits) < R) ++pid_bits;
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out);
  const uint32_t rot = (uint32_t)(lane >> 3) & 3u;

  auto slice_of = [&](uint32_t m, uint64_t& c0, uint32_t& n) {
    const uint64_t mb = (uint64_t)m * g.records_per_map;
    const uint64_t me = min(mb + g.records_per_map, g.num_records);
    const uint64_t a = min(mb + (uint64_t)s * cs, me);
    c0 = a;
    n = (uint32_t)(min(a + cs, me) - a);
  };
  // loads of map m's slice: coalesced 16-byte units + this thread's record key.  A map past
  // the last (or an empty slice) loads record 0 of the group instead, so that every issue is
  // the same instruction sequence (the compiler's counted waits then leave younger sets in
  // flight).
  auto issue = [&](uint32_t m, St& x) {
    uint64_t c0 = 0;
    uint32_t n = 0;
    if (m < M) slice_of(m, c0, n);
    if (n == 0) {
      c0 = 0;
      n = 1;
    }
    const uint8_t* a = g.recs + c0 * S;
    const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 15u);
    const u32x4* src = reinterpret_cast<const u32x4*>(a - head);
    const uint32_t units = (head + n * S + 15) >> 4;
    // the key first: the count waits for it alone (vmcnt counts in issue order)
    const uint32_t r = min((uint32_t)tid, n - 1);
    const uint32_t* kp = reinterpret_cast<const uint32_t*>(a + (size_t)r * S + pd.key_offset);
    typename KeyVec<KW>::T kvv = *reinterpret_cast<const typename KeyVec<KW>::T*>(kp);
    KeyVec<KW>::get(kvv, x.k);
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) x.v[k] = src[min(tid + k * NT, units - 1)];
  };

  // ---- count map m (keys in z), in three barrier-separated parts -------------------------
  // a: key -> pid, stable ballot ranks inside each wave, per-wave counts into wcnt
  auto count_a = [&](uint32_t m, St& z, uint64_t& peers_out) {
    uint64_t c0;
    uint32_t n;
    slice_of(m, c0, n);
    const bool valid = (uint32_t)tid < n;
    const uint32_t pid = valid ? (uint32_t)partition_words<KW, false>(pd, z.k, pd.bounds, pd.lut) : 0u;
    uint64_t peers = __ballot(valid);
    for (int bb = 0; bb < pid_bits; ++bb) {
      const bool bit = (pid >> bb) & 1u;
      const uint64_t mk = __ballot(bit);
      peers &= bit ? mk : ~mk;
    }
    if (valid && (peers & lt_mask) == 0) wcnt[pid * NW + wave] = (uint32_t)__popcll(peers);
    if (pids && valid) pids[c0 + tid] = (uint16_t)pid;
    z.pid = valid ? pid : kNone;
    peers_out = peers;
  };
  // b (after a barrier): owner p -> exclusive prefix over waves in place, the slice's count of
  // p; published at once (sc1 store for the later slices of my group, agent-scope add to my
  // group's total) so the stores travel while part c and other work run
  auto count_b = [&](uint32_t m, St& z) {
    uint32_t c = 0;
    if (owner) {
      u32x4* row = reinterpret_cast<u32x4*>(wcnt + tid * NW);
      u32x4 xr[NW / 4];
#pragma unroll
      for (uint32_t q = 0; q < NW / 4; ++q) xr[q] = row[q];
#pragma unroll
      for (uint32_t q = 0; q < NW / 4; ++q) {
        u32x4 y;
        y[0] = c;
        y[1] = c + xr[q][0];
        y[2] = y[1] + xr[q][1];
        y[3] = y[2] + xr[q][2];
        c = y[3] + xr[q][3];
        row[q] = y;
      }
      st_sc1(sw.cnt + ((uint64_t)(m % kCntBufs) * nwg + s) * R + tid, c);
      (void)add_agent(sw.gt + ((uint64_t)(m % kGtBufs) * kMaxGroups + grp) * R + tid, c);
    }
    z.c = c;
  };
  // c (after a barrier): each record's rank inside (slice, partition); the owner waves drain
  // their publishing stores and count themselves off in LDS; the last one arrives for map m
  // (one wave instruction, +1 on every replica of map m's counter)
  auto count_c = [&](uint32_t m, St& z, uint64_t peers) {
    z.jr = z.pid != kNone ? wcnt[z.pid * NW + wave] + (uint32_t)__popcll(peers & lt_mask) : 0u;
    if (wave < n_owner_waves) {
      drain();
      uint32_t last = 0;
      if (lane == 0) last = atomicAdd(reinterpret_cast<uint32_t*>(flags + 3), 1u) % n_owner_waves ==
                            (uint32_t)n_owner_waves - 1;
      last = __shfl(last, 0, kWave);
      if (last && lane < (int)ngr)
        (void)add_agent(sw.sync + (m % kSlots) * kMaxGroups * kLine + lane * kLine, 1u);
    }
  };
  auto zero_wcnt = [&]() {
    if (owner) {
#pragma unroll
      for (uint32_t q = 0; q < NW / 4; ++q) reinterpret_cast<u32x4*>(wcnt + tid * NW)[q] = u32x4{0, 0, 0, 0};
    }
  };

  // ---- map m's offsets: poll its arrival counter, then (owner p) the map-level offset of p
  // (scan of the partition totals) + the groups before mine + the slices before mine in my
  // group; slice 0 also writes the map's index file and clears the group totals of map m-2
  auto poll = [&](uint32_t m) -> bool {
    if (tid == 0) {
      flags[2] = 0;
      const uint32_t want = (m / kSlots + 1) * nwg;
      const uint32_t* ctr = sw.sync + (m % kSlots) * kMaxGroups * kLine + grp * kLine;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (ld_sc1(ctr) < want) {
        if (ld_sc1(sw.sync + kAbort)) {
          flags[2] = 1;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
          st_sc1(sw.sync + kAbort, 1u);
          index[(uint64_t)(M - 1) * (R + 1)] = -1;  // the host sees a broken index table
          flags[2] = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
    }
    __syncthreads();
    return !flags[2];
  };
  struct OffLoads {
    uint32_t gv[kMaxGroups], cv[kGroup];
  };
  auto offsets_issue = [&](uint32_t m, OffLoads& L) {
    if (owner) {
      const uint32_t* gtm = sw.gt + (uint64_t)(m % kGtBufs) * kMaxGroups * R + tid;
#pragma unroll
      for (uint32_t q = 0; q < kMaxGroups; ++q) L.gv[q] = q < ngr ? ld_sc1(gtm + q * R) : 0u;
      const uint32_t* cm = sw.cnt + (uint64_t)(m % kCntBufs) * nwg * R + tid;
#pragma unroll
      for (uint32_t j = 0; j < kGroup; ++j) L.cv[j] = (g0 + j < s) ? ld_sc1(cm + (uint64_t)(g0 + j) * R) : 0u;
    }
  };
  auto offsets_finish = [&](uint32_t m, const OffLoads& L, St& y) {
    uint32_t T = 0, before = 0;
    if (owner) {
#pragma unroll
      for (uint32_t j = 0; j < kGroup; ++j) before += L.cv[j];
#pragma unroll
      for (uint32_t q = 0; q < kMaxGroups; ++q) {
        T += L.gv[q];
        before += q < grp ? L.gv[q] : 0u;
      }
    }
    const uint32_t tincl = wave_incl_scan(T, lane);
    if (lane == kWave - 1) tmp[wave] = tincl;
    __syncthreads();
    uint32_t ex = tincl - T, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) {
      const uint32_t t = tmp[w];
      ex += (w < (uint32_t)wave) ? t : 0u;
      tot += t;
    }
    y.off = ex + before;
    if (s == 0) {
      int64_t* im = index + (uint64_t)m * (R + 1);
      uint64_t* ibe = index_be ? reinterpret_cast<uint64_t*>(index_be) + (uint64_t)m * (R + 1) : nullptr;
      if (owner) {
        const int64_t off = (int64_t)ex * S;
        im[tid] = off;
        if (ibe) ibe[tid] = bswap64((uint64_t)off);
        if (m >= 2) {
          uint32_t* gz = sw.gt + (uint64_t)((m - 2) % kGtBufs) * kMaxGroups * R + tid;
#pragma unroll
          for (uint32_t q = 0; q < kMaxGroups; ++q)
            if (q < ngr) st_sc1(gz + q * R, 0u);
        }
      }
      if (tid == 0) {
        const int64_t off = (int64_t)tot * S;
        im[R] = off;
        if (ibe) ibe[R] = bswap64((uint64_t)off);
      }
    }
  };

  // ---- one map: place m (x), offsets of m+1 (y), count m+2 (z), load m+3 into x ----------
  // Order matters for the compiler's vmcnt waits (one in-order counter for loads and stores):
  // map m+3's loads are issued AFTER map m's stores, so that re-using a store's data registers
  // waits for the stores only, never for the prefetch.
  auto process = [&](uint32_t m, St& x, St& y, St& z) -> bool {
    SUX_OP_STAMP(m, 0);
    const bool next = m + 1 < M, cnt2 = m + 2 < M;
    // S1: run geometry of this slice's runs, scan of image units over p
    uint64_t c0;
    uint32_t n;
    slice_of(m, c0, n);
    const uint64_t mbase = (uint64_t)m * g.records_per_map * S;  // map m's data file
    const uint64_t mal = mbase & ~15ull;
    uint32_t sp = 0, u0 = 0, cd = 0, full = 0, keep = 0;
    if (owner) {
      const uint64_t pos = mbase + (uint64_t)x.off * S;
      u0 = (uint32_t)((pos - mal) >> 4);
      cd = (uint32_t)(pos & 15) >> 2;
      if (x.c) {
        const uint32_t dw = cd + x.c * W;
        full = dw >> 2;
        sp = (dw + 3) >> 2;
        keep = dw & 3u;
      }
    }
    const uint32_t incl = wave_incl_scan(sp, lane);
    if (lane == kWave - 1) tmp[wave] = incl;
    __syncthreads();
    uint32_t lb = incl - sp, U = 0;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) {
      const uint32_t t = tmp[w];
      lb += (w < (uint32_t)wave) ? t : 0u;
      U += t;
    }
    if (owner) {
      pinfo[tid] = u32x4{lb, cd | (keep << 8), full, sp};
      u0s[tid] = u0;
      if (sp) dstu[lb] = u0 | (cd << 28);  // head unit: its first cd dwords are the previous slice's
    }
    __syncthreads();
    SUX_OP_STAMP(m, 1);
    // S2: record image offsets, destination units that start inside each record
    if (x.pid != kNone) {
      const u32x4 pi = pinfo[x.pid];
      const uint32_t pcd = pi[1] & 0xFFu, pkeep = pi[1] >> 8;
      const uint32_t o = 4 * pcd + x.jr * S;
      recoff[tid] = 16 * pi[0] + o;
      const uint32_t pu0 = u0s[x.pid];
      const uint32_t k0 = (o + 15) >> 4;
#pragma unroll
      for (uint32_t t = 0; t < K::kRecUnits; ++t) {
        const uint32_t k = k0 + t;
        if (k > 0 && k * 16 < o + S && k < pi[3])
          dstu[pi[0] + k] = (pu0 + k) | (k == pi[2] ? (pkeep << 30) : 0u);
      }
    }
    __syncthreads();
    SUX_OP_STAMP(m, 2);
    // S3: records -> image (K3 v7 step 4)
    {
      const uint32_t head = (uint32_t)(reinterpret_cast<uintptr_t>(g.recs + c0 * S) & 15u);
      const uint32_t units = n ? (head + n * S + 15) >> 4 : 0u;
#pragma unroll
      for (uint32_t k = 0; k < PER; ++k) {
        const uint32_t u = tid + k * NT;
        const int32_t b0 = (int32_t)(16 * u) - (int32_t)head;
        const uint32_t r0 = b0 >= 0 ? (uint32_t)b0 / S : 0u, off0 = (uint32_t)b0 - r0 * S;
        if (u < units && b0 >= 0 && (uint32_t)b0 + 16 <= n * S && off0 + 16 <= S) {
          *reinterpret_cast<u32x4a4*>(img32 + ((recoff[r0] + off0) >> 2)) = x.v[k];
        } else if (u < units) {
#pragma unroll
          for (uint32_t cc = 0; cc < 4; ++cc) {
            const uint32_t q = (cc + rot) & 3u;
            const int32_t b = (int32_t)(16 * u + 4 * q) - (int32_t)head;
            if (b >= 0 && (uint32_t)b < n * S) {
              const uint32_t r = (uint32_t)b / S, off = (uint32_t)b - r * S;
              const uint32_t xv = q == 0 ? x.v[k][0] : q == 1 ? x.v[k][1] : q == 2 ? x.v[k][2] : x.v[k][3];
              img32[(recoff[r] + off) >> 2] = xv;
            }
          }
        }
      }
    }
    SUX_OP_STAMP(m, 3);
    // S4: map m+1's offsets: every slice arrived for it a map ago; the sc1 loads fly while
    //     map m+2 is counted
    OffLoads L;
    if (next) {
      if (!poll(m + 1)) return false;
      offsets_issue(m + 1, L);
    }
    SUX_OP_STAMP(m, 4);
    // S5: count map m+2 (loaded at the end of the previous map), publish, arrive
    if (cnt2) {
      uint64_t peers = 0;
      count_a(m + 2, z, peers);
      __syncthreads();
      count_b(m + 2, z);
      __syncthreads();
      count_c(m + 2, z, peers);
    }
    SUX_OP_STAMP(m, 5);
    // S6: finish map m+1's offsets (scan of the partition totals; barriers inside)
    if (next) offsets_finish(m + 1, L, y);
    __syncthreads();
    zero_wcnt();
    SUX_OP_STAMP(m, 6);
    // S7: write map m's image: aligned 16-byte units, partial head/tail units as dwords
#pragma unroll 4
    for (uint32_t q = tid; q < U; q += NT) {
      const uint32_t d = dstu[q];
      const u32x4 xv = img[q];
      const uint64_t A = mal + (uint64_t)(d & 0x0FFFFFFFu) * 16;
      const uint32_t skip = (d >> 28) & 3u, keep2 = d >> 30;
      if (skip == 0 && keep2 == 0) {
        *reinterpret_cast<u32x4*>(out + A) = xv;
      } else {
        const uint32_t e = keep2 ? keep2 : 4u;
#pragma unroll
        for (uint32_t cc = 0; cc < 4; ++cc)
          if (cc >= skip && cc < e) out32[(A >> 2) + cc] = xv[cc];
      }
    }
    SUX_OP_STAMP(m, 7);
    // S8: x's registers are free: load map m+3 (counted in two maps' time)
    issue(m + 3, x);
    __syncthreads();
    SUX_OP_STAMP(m, 8);
    return true;
  };

  if (M == 0) return;
  if (tid == 0) flags[3] = 0;
  zero_wcnt();
  __syncthreads();
  // three maps in registers, roles rotating by unrolling (no register moves: a move of a set
  // whose loads are in flight would wait for them)
  St a, b, c;
  a.pid = b.pid = c.pid = kNone;
  a.jr = b.jr = c.jr = a.c = b.c = c.c = a.off = b.off = c.off = 0;
  issue(0, a);
  issue(1, b);
  issue(2, c);
  for (uint32_t m = 0; m < 2 && m < M; ++m) {
    St& z = m == 0 ? a : b;
    uint64_t peers = 0;
    count_a(m, z, peers);
    __syncthreads();
    count_b(m, z);
    __syncthreads();
    count_c(m, z, peers);
    __syncthreads();
    zero_wcnt();
    __syncthreads();
  }
  if (!poll(0)) return;
  {
    OffLoads L;
    offsets_issue(0, L);
    offsets_finish(0, L, a);
    __syncthreads();
  }
  for (uint32_t m = 0; m < M; m += 3) {
    if (!process(m, a, b, c)) return;
    if (m + 1 >= M) break;
    if (!process(m + 1, b, c, a)) return;
    if (m + 2 >= M) break;
    if (!process(m + 2, c, a, b)) return;
  }
}

}  // namespace onepass

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
namespace {
using onepass::Shape;
// 256-thread workgroups, KOPWG per CU: while one workgroup counts or builds its image the other's
// loads and stores are in flight.  Three register sets need ~220 VGPRs: 2 waves per SIMD.
constexpr uint32_t kOpS = 100, kOpNW = 4, kOpWgPerCu = 2, kOpMaxWg = 512;
constexpr int kOpMinW = (int)(kOpWgPerCu * kOpNW / 4);

}  // namespace

int stream_cus(hipStream_t s) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  uint32_t mask[32] = {0};
  const uint32_t words = (uint32_t)std::min(32, (cus + 31) / 32);
  if (s && hipExtStreamGetCUMask(s, words, mask) == hipSuccess) {
    int n = 0;
    for (uint32_t i = 0; i < words; ++i) n += __builtin_popcount(mask[i]);
    if (n > 0 && n < cus) return n;
  }
  return cus;
}

uint64_t onepass_sync_bytes(uint32_t R) {
  const uint64_t words = onepass::kSyncWords + (uint64_t)onepass::kCntBufs * kOpMaxWg * R +
                         (uint64_t)onepass::kGtBufs * onepass::kMaxGroups * R;
  return (words * 4 + 255) / 256 * 256;
}

bool onepass_eligible(const PartDev& pd, const MapGroup& g, int world, const void* d_out,
                      const uint64_t* d_peer_bytes, hipStream_t s, uint32_t* grid_out,
                      uint32_t* cs_out) {
  // opt-in (sux_tuning.onepass; the launcher checks it).  Measured on MI355X at R = 200 it is
  // slower than the three-kernel path: a slice's run of one partition is only
  // ~C/R records, so its writes are short misaligned runs.
  if (world != 1 || d_peer_bytes || g.rec_size != kOpS) return false;
  if (pd.kind == 4 || pd.key_offset % 4 || pd.key_len < 1 || pd.key_len > 16 ||
      pd.key_offset + pd.key_len > (int)kOpS)
    return false;
  if (pd.R < 1 || pd.R > (int)Shape<kOpS, kOpNW>::NT ||
      Shape<kOpS, kOpNW>::lds_bytes(pd.R) > 160 * 1024)
    return false;
  if ((reinterpret_cast<uintptr_t>(d_out) & 15) || g.records_per_map * kOpS >= (1ull << 32))
    return false;
  const int cus = stream_cus(s);
  if (cus < 1 || cus > 256) return false;
  const uint32_t wgs = (uint32_t)cus * kOpWgPerCu;
  const uint64_t cs = (g.records_per_map + wgs - 1) / wgs;
  if (cs > Shape<kOpS, kOpNW>::C) return false;
  if (grid_out) *grid_out = wgs;
  if (cs_out) *cs_out = (uint32_t)cs;
  return true;
}

hipError_t launch_onepass(const PartDev& pd, const MapGroup& g, uint8_t* d_out, int64_t* d_index,
                          uint8_t* d_index_be, uint16_t* d_pids, uint8_t* d_sync, uint32_t grid,
                          uint32_t cs, hipStream_t s) {
  const int R = pd.R;
  onepass::SyncWs sw;
  uint32_t* w = reinterpret_cast<uint32_t*>(d_sync);
  sw.sync = w;
  sw.cnt = w + onepass::kSyncWords;
  sw.gt = sw.cnt + (uint64_t)onepass::kCntBufs * kOpMaxWg * R;
  // counters and the group-total accumulators start at zero in every launch
  hipError_t e = hipMemsetAsync(sw.sync, 0, onepass::kSyncWords * 4, s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(sw.gt, 0, (size_t)onepass::kGtBufs * onepass::kMaxGroups * R * 4, s);
  if (e != hipSuccess) return e;
  const size_t lds = Shape<kOpS, kOpNW>::lds_bytes(R);
  const int kw = (pd.key_len + 3) / 4;
#define SUX_OP(KW)                                                                              \
  do {                                                                                          \
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&onepass::k_onepass<kOpS, kOpNW, KW, kOpMinW>), \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);            \
    hipLaunchKernelGGL((onepass::k_onepass<kOpS, kOpNW, KW, kOpMinW>), dim3(grid), dim3(kOpNW * kWave),   \
                       lds, s, pd, g, d_out, d_index, d_index_be, d_pids, sw, cs);              \
  } while (0)
  if (kw <= 1) SUX_OP(1);
  else if (kw == 2) SUX_OP(2);
  else if (kw == 3) SUX_OP(3);
  else SUX_OP(4);
#undef SUX_OP
  return hipGetLastError();
}

}  // namespace sux
