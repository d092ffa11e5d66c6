// sux_lz4.hip — compressed map outputs (spark.shuffle.compress=true with
// Spark's default lz4 codec): every non-empty (map, partition) run of a map output becomes its own
// lz4-java LZ4BlockOutputStream stream, as Spark's writers wrap each partition segment in a fresh
// compressed stream [ext: Spark 3.0 LZ4CompressionCodec.compressedOutputStream =
// new LZ4BlockOutputStream(s, spark.io.compression.lz4.blockSize)].  Stream layout (lz4-java
// 1.7.1 [ext]): per chunk of <= blockSize bytes a 21-byte header
//   "LZ4Block" | token = method | level | compressed length LE32 | original length LE32 |
//   XXH32(original, 0x9747b28c) & 0x0FFFFFFF LE32
// then the LZ4 block (method 0x20) or the raw bytes (method 0x10, when compressing does not
// shrink the chunk); close() appends an end mark (method 0x10, all lengths and checksum 0).
// level = max(0, ceil(log2(blockSize)) - 10).  An empty run writes nothing (streams open lazily).
//
// Kernels (one launch each, sizes bounded on the host so nothing waits on the device):
//   k_lz4_map_base  map data starts (maps are consecutive: prefix of index[m][R])
//   k_lz4_runs      chunks per run -> (rocprim scan) -> k_lz4_fill: chunk table, map-major
//   k_lz4_default   one wave per chunk: liblz4's LZ4_compress_default, exactly (below)
//   k_xxh32         4 lanes per chunk (XXH32's four accumulators), 16 chunks per wave
//   k_lz4_sizes     framed size of every chunk (+ the end mark on a run's last chunk)
//                   -> (rocprim scan) -> output offsets; run sizes -> k_map_scan -> index
//   k_lz4_emit      one wave per chunk: header + payload (compressed or raw) + end mark
//
// The parse is liblz4 1.9.3's LZ4_compress_default, byte for byte (k_lz4_default below).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "sux_internal.h"

namespace sux {

namespace {
constexpr int kLWave = 64;
constexpr int kLz4Hdr = 21;
constexpr uint32_t kXxhSeed = 0x9747b28cu;
constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                   P5 = 374761393u;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// 4 bytes at any byte address: two aligned dword loads (the second only when the bytes straddle),
// funnel-shifted.  Never reads outside the aligned dwords holding the 4 bytes.
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) {
  const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3u);
  // pointer arithmetic (not an integer round trip) keeps the global address space: global_load,
  // not flat_load (whose lgkmcnt share would make every LDS wait drain the loads in flight)
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p - mis);
  uint32_t k = mis ? 1u : 0u;
  asm volatile("" : "+v"(k));  // opaque: both loads stay unconditional (no branch, counted vmcnt)
  const uint32_t lo = q[0];
  const uint32_t hi = q[k];
  return __builtin_amdgcn_alignbyte(hi, lo, mis);  // ({hi, lo} >> 8 * mis), = lo when aligned
}

// Wave-cooperative copy of n bytes, any alignment on either side: byte stores up to dst's first
// dword boundary, dword stores for the body (source funnel-shifted), byte stores for the tail.
// The head and tail bytes are loaded up front (clamped, unconditional), so their loads share the
// body's first round trip instead of taking one each.
__device__ __forceinline__ void wave_copy(uint8_t* dst, const uint8_t* src, uint32_t n, int lane) {
  if (n == 0) return;
  const uint32_t head = min(n, (uint32_t)((4u - (reinterpret_cast<uintptr_t>(dst) & 3u)) & 3u));
  const uint32_t nd = (n - head) / 4u;
  const uint32_t done = head + 4u * nd;
  const uint8_t hb = src[min((uint32_t)lane, n - 1u)];
  const uint8_t tb = src[min(done + (uint32_t)lane, n - 1u)];
  uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + head);
  const uint8_t* s = src + head;
  uint32_t k = lane;
  for (; k + 3u * kLWave < nd; k += 4u * kLWave) {
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld32u(s + 4u * (k + u * kLWave));
#pragma unroll
    for (int u = 0; u < 4; ++u) d32[k + u * kLWave] = v[u];
  }
  for (; k < nd; k += kLWave) d32[k] = ld32u(s + 4u * k);
  if ((uint32_t)lane < head) dst[lane] = hb;
  if ((uint32_t)lane < n - done) dst[done + lane] = tb;
}

__device__ __forceinline__ uint32_t ext_bytes(uint32_t v) { return v >= 15u ? (v - 15u) / 255u + 1u : 0u; }


__host__ __device__ __forceinline__ int lz4_level(uint32_t bs) {
  const int l = 32 - __builtin_clz(bs - 1u);
  return l > 10 ? l - 10 : 0;
}
}  // namespace

__global__ __launch_bounds__(256) void k_lz4_map_base(const int64_t* __restrict__ index, int maps,
                                                      int R, uint64_t* __restrict__ map_base) {
  __shared__ uint64_t part[256];
  // one workgroup: per-thread serial sums over a slice of maps, then a block scan of the slices
  const int t = threadIdx.x, per = (maps + 255) / 256;
  const int m0 = min(maps, t * per), m1 = min(maps, m0 + per);
  uint64_t s = 0;
  for (int m = m0; m < m1; ++m) s += (uint64_t)index[(uint64_t)m * (R + 1) + R];
  part[t] = s;
  __syncthreads();
  if (t == 0) {
    uint64_t c = 0;
    for (int i = 0; i < 256; ++i) { const uint64_t v = part[i]; part[i] = c; c += v; }
    map_base[maps] = c;
  }
  __syncthreads();
  uint64_t c = part[t];
  for (int m = m0; m < m1; ++m) {
    map_base[m] = c;
    c += (uint64_t)index[(uint64_t)m * (R + 1) + R];
  }
}

__global__ __launch_bounds__(256) void k_lz4_runs(const int64_t* __restrict__ index, int maps,
                                                  int R, uint32_t bs, uint32_t* __restrict__ nb) {
  const uint64_t r = blockIdx.x * 256ull + threadIdx.x;
  if (r >= (uint64_t)maps * R) return;
  const uint64_t m = r / R, p = r - m * R;
  const int64_t* im = index + m * (R + 1);
  const uint64_t L = (uint64_t)(im[p + 1] - im[p]);
  nb[r] = (uint32_t)((L + bs - 1) / bs);
}

__global__ __launch_bounds__(256) void k_lz4_fill(const int64_t* __restrict__ index, int maps,
                                                  int R, uint32_t bs,
                                                  const uint64_t* __restrict__ map_base,
                                                  const uint32_t* __restrict__ b0,
                                                  Lz4Chunk* __restrict__ chunks,
                                                  uint32_t* __restrict__ nchunks) {
  const uint64_t r = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t runs = (uint64_t)maps * R;
  if (r >= runs) return;
  const uint64_t m = r / R, p = r - m * R;
  const int64_t* im = index + m * (R + 1);
  const uint64_t start = map_base[m] + (uint64_t)im[p];
  const uint64_t L = (uint64_t)(im[p + 1] - im[p]);
  const uint32_t n = (uint32_t)((L + bs - 1) / bs);
  for (uint32_t k = 0; k < n; ++k) {
    Lz4Chunk c;
    c.src = start + (uint64_t)k * bs;
    c.len = (uint32_t)min((uint64_t)bs, L - (uint64_t)k * bs);
    c.run = (uint32_t)r;
    c.last = (k + 1 == n) ? 1u : 0u;
    c.clen = 0;
    c.csum = 0;
    c.pad = 0;
    chunks[b0[r] + k] = c;
  }
  if (r + 1 == runs) *nchunks = b0[r] + n;
}

// One wave per chunk: liblz4 1.9.3's LZ4_compress_default (oracle/lz4.c o_lz4_compress_default
// restates it; tests pin both to the system liblz4), the compressor lz4-java's JNI instance runs
// for every chunk of Spark's LZ4BlockOutputStream.  The hash table is liblz4's: 8192 u16
// positions (byU16, 13-bit hash of the 4 bytes at a position), zeroed per chunk — a never
// written entry reads as position 0 and is a real candidate.  The parse is sequential by
// definition; the wave runs it exactly, parallelising what can be:
//   - the match search probes positions q_i = q_0 + sum(step) (step 1 for 64 probes, then 2,
//     3, ...: liblz4's acceleration schedule), 64 probes per round, one per lane.  Probe i sees
//     the table as liblz4 would: the entry of the latest earlier probe of this round with the
//     same hash (13-ballot match), else the table as it stood before the round.  The first
//     probe whose candidate's 4 bytes agree ends the search; only the probes up to it are
//     inserted (later lanes never happened).  A probe whose successor would pass len - 11 ends
//     the parse (last literals) before its own insertion, as in liblz4;
//   - the backward catch-up, the forward match count (LZ4_count up to len - 5) and the literal
//     copies are wave-wide compares / copies;
//   - the table updates after a match (ip - 2, then the probe of ip itself) are single-lane.
// A chunk whose block would not be shorter than the chunk is stored raw (lz4-java's rule); the
// parse stops as soon as that is certain, so the scratch never needs more than the chunk's bytes.
// Chunk deal: Q = false, the fixed grid-stride deal; Q = true, a device work queue (tuning
// lz4_queue) — lane 0 claims the next chunk with one vector atomic on a counter the launcher
// zeroes on the same stream, and the index reaches the wave through readfirstlane, so the loop
// exit is wave-uniform by construction (a scalar register) and the counter only grows: every wave
// leaves after at most one claim past the last chunk.
constexpr int kLz4TabBits = 13;          // liblz4: LZ4_HASHLOG + 1 for byU16 tables
constexpr int kLz4Waves = 2;             // waves per workgroup: 2 x 16 KiB of tables

__device__ __forceinline__ uint32_t lz4_hash(uint32_t seq) { return (seq * P1) >> (32 - kLz4TabBits); }

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// bytes of an LZ4 length field beyond its 4-bit token nibble: (v - 15) as 255s then the rest
__device__ __forceinline__ void put_len(uint8_t* d, uint32_t v, int lane) {
  const uint32_t nb = ext_bytes(v);
  for (uint32_t k = lane; k < nb; k += kLWave) d[k] = (k + 1 < nb) ? 255u : (uint8_t)((v - 15u) % 255u);
}

__device__ __forceinline__ uint32_t lz4_claim(uint32_t* q, int lane) {
  uint32_t t = 0;
  if (lane == 0) t = atomicAdd(q, 1u);
  return (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)t, 0, kLWave));
}

template <bool Q>
__global__ __launch_bounds__(kLz4Waves * kLWave) void k_lz4_default(
    const uint8_t* __restrict__ data, Lz4Chunk* __restrict__ chunks,
    const uint32_t* __restrict__ nchunks, uint8_t* __restrict__ scratch, uint32_t* __restrict__ qctr) {
  __shared__ __attribute__((aligned(16))) uint16_t ltab[kLz4Waves][1u << kLz4TabBits];
  const int wave = threadIdx.x / kLWave, lane = threadIdx.x % kLWave;
  uint16_t* tab = ltab[wave];
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t n = *nchunks;
  for (uint32_t b = Q ? lz4_claim(qctr, lane) : blockIdx.x * kLz4Waves + wave; b < n;
       b = Q ? lz4_claim(qctr, lane) : b + gridDim.x * kLz4Waves) {
    const Lz4Chunk C = chunks[b];
    const uint8_t* src = data + C.src;
    const uint32_t len = C.len;
    uint8_t* dst = scratch + ((C.src + 16ull * b) & ~3ull);
    bool raw = len < 13;  // LZ4_minLength: one literal run, never shorter than the chunk
    if (!raw) {
      // LZ4_initStream: a zeroed table
      typedef uint32_t u4 __attribute__((ext_vector_type(4)));
      for (uint32_t i = lane; i < (1u << kLz4TabBits) / 8; i += kLWave)
        reinterpret_cast<u4*>(tab)[i] = u4{0u, 0u, 0u, 0u};
      wave_lds_sync();
      const uint32_t mflimit1 = len - 11, matchlimit = len - 5;
      uint32_t anchor = 0, op = 0, ip = 1, match = 0;
      bool last = false;  // go to the last literals
      // ---- find a match from ip (liblz4's do-while search), 64 probes per round
      // The words at a round's probes are loaded one round early (probe positions do not depend
      // on the table); pre holds round 0's, the words at ip + lane.
      auto search = [&](uint32_t pre) -> bool {  // true: (ip, match) is a match; false: last literals
        uint32_t q0 = ip, r = 0, seq = pre;
        while (true) {
          // probe i = 64 r + lane steps by (i == 0 ? 1 : (63 + i) >> 6): r + 1 on lanes >= 1 and
          // s0 = max(r, 1) on lane 0, so the prefix of the steps has a closed form
          const uint32_t s0 = r ? r : 1u;
          const uint32_t s = lane ? r + 1u : s0;
          const uint32_t q = lane ? q0 + s0 + ((uint32_t)lane - 1u) * (r + 1u) : q0, nxt = q + s;
          const bool live = nxt <= mflimit1;  // monotone over the lanes
          const uint32_t q0n = q0 + s0 + 63u * (r + 1u);  // the next round's first probe
          const uint32_t qn = lane ? q0n + (r + 1u) + ((uint32_t)lane - 1u) * (r + 2u) : q0n;
          // clamped: a live probe of the next round lies below mflimit1, so it reads its own word
          const uint32_t seqn = ld32u(src + min(qn, len - 4u));
          const uint32_t h = lz4_hash(seq);
          uint64_t peers = __ballot(live);
#pragma unroll
          for (int bb = 0; bb < kLz4TabBits; ++bb) {
            const bool bit = (h >> bb) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
          }
          const uint64_t prev = peers & lt;
          const uint32_t from_tab = tab[h];
          const uint32_t pl = prev ? 63u - (uint32_t)__builtin_clzll(prev) : 0u;
          const uint32_t qprev = (uint32_t)__shfl((int)q, (int)pl, kLWave);
          const uint32_t m = prev ? qprev : from_tab;
          const bool hit = live && ld32u(src + m) == seq;
          const uint64_t hits = __ballot(hit), lives = __ballot(live);
          const uint64_t commit = hits ? (lives & ((2ull << __builtin_ctzll(hits)) - 1ull)) : lives;
          wave_lds_sync();  // every lane read the table before any insertion of this round
          const uint64_t later = peers & ~lt & ~(1ull << lane) & commit;
          if (((commit >> lane) & 1ull) && !later) tab[h] = (uint16_t)q;
          wave_lds_sync();
          if (hits) {
            const int f = __builtin_ctzll(hits);
            ip = (uint32_t)__shfl((int)q, f, kLWave);
            match = (uint32_t)__shfl((int)m, f, kLWave);
            return true;
          }
          if (~lives) return false;  // a probe's successor passed mflimitPlusOne
          q0 = q0n;
          ++r;
          seq = seqn;
        }
      };
      // LZ4_count: equal bytes from p + 4 / mt + 4 up to matchlimit, 4 per lane per round.  The
      // first round's loads come from cnt_load, issued by the caller next to other loads (one
      // memory round trip for both); the addresses stay in the chunk (a round starts at or before
      // matchlimit), so the loads are unconditional.
      auto cnt_load = [&](uint32_t p, uint32_t mt, uint32_t mc) -> uint32_t {
        const uint32_t a = p + 4u + mc;
        const uint32_t lim = matchlimit > a ? matchlimit - a : 0u;
        const uint32_t o = 4u * (uint32_t)lane < lim ? 4u * (uint32_t)lane : 0u;
        return ld32u(src + a + o) ^ ld32u(src + mt + 4u + mc + o);
      };
      auto count = [&](uint32_t p, uint32_t mt, uint32_t x) -> uint32_t {
        uint32_t mc = 0;
        while (true) {
          const uint32_t a = p + 4u + mc;
          const uint32_t lim = matchlimit > a ? matchlimit - a : 0u;
          const uint32_t o = 4u * (uint32_t)lane;
          uint32_t eq = 0;
          if (o < lim) eq = min(x ? (uint32_t)(__builtin_ctz(x) >> 3) : 4u, lim - o);
          const uint64_t stop = __ballot(eq < 4u);
          if (stop) {
            const int sl = __builtin_ctzll(stop);
            return mc + 4u * (uint32_t)sl + (uint32_t)__shfl((int)eq, sl, kLWave);
          }
          mc += 4u * kLWave;
          x = cnt_load(p, mt, mc);
        }
      };
      // emits one sequence (literals [anchor, ip) + the match at ip, mc bytes past its first 4);
      // false = the block cannot be shorter than the chunk (stored raw).  The 4-byte words the
      // re-probe at the match end hashes are loaded before the sequence's stores (gfx950's vmcnt
      // counts stores: loads issued after them would wait for them too).
      uint32_t w2 = 0, w0 = 0, pw = ld32u(src + min(1u + (uint32_t)lane, len - 4u));
      auto sequence = [&](uint32_t mc) -> bool {
        const uint32_t ll = ip - anchor;
        const uint32_t need = 1u + ext_bytes(ll) + ll + 2u + ext_bytes(mc);
        if (op + need >= len) return false;
        const uint32_t end = ip + mc + 4u;  // <= matchlimit: both words lie inside the chunk
        w2 = ld32u(src + end - 2u);
        w0 = ld32u(src + end);
        pw = ld32u(src + min(end + 1u + (uint32_t)lane, len - 4u));  // a failed re-probe's search
        uint8_t* d = dst + op;
        if (lane == 0) d[0] = (uint8_t)((min(ll, 15u) << 4) | min(mc, 15u));
        put_len(d + 1, ll, lane);
        const uint32_t lo = 1u + ext_bytes(ll);
        wave_copy(d + lo, src + anchor, ll, lane);
        const uint32_t off = ip - match;
        if (lane == 0) {
          d[lo + ll] = (uint8_t)off;
          d[lo + ll + 1] = (uint8_t)(off >> 8);
        }
        put_len(d + lo + ll + 2, mc, lane);
        op += need;
        ip = end;
        anchor = ip;
        return true;
      };
      while (!last && !raw) {
        if (!search(pw)) {
          last = true;
          break;
        }
        // the backward catch-up (extend while ip > anchor, match > 0 and the bytes before agree)
        // and the forward count from the hit, their first rounds' loads together.  Counting from
        // the hit is exact: the caught-up bytes and the hit's 4 agree, so the match ends where it
        // would counting from the caught-up ip, back bytes further on.
        uint32_t back = 0;
        uint32_t room = min(ip - anchor, match);
        const uint32_t k1 = (uint32_t)lane + 1u;
        uint32_t kc = k1 <= room ? k1 : 0u;  // clamped: the loads are unconditional
        uint8_t bi = src[ip - kc], bm = src[match - kc];
        uint32_t mc = count(ip, match, cnt_load(ip, match, 0u));
        while (room) {
          const bool eq = k1 <= room && bi == bm;
          const uint64_t ne = __ballot(!eq);
          const uint32_t bk = ne ? (uint32_t)__builtin_ctzll(ne) : (uint32_t)kLWave;
          ip -= bk;
          match -= bk;
          back += bk;
          if (bk < (uint32_t)kLWave) break;
          room = min(ip - anchor, match);
          kc = k1 <= room ? k1 : 0u;
          bi = src[ip - kc];
          bm = src[match - kc];
        }
        mc += back;
        // the match, then liblz4's immediate re-probes at the match end
        while (true) {
          if (!sequence(mc)) {
            raw = true;
            break;
          }
          if (ip >= mflimit1) {
            last = true;
            break;
          }
          const uint32_t h2 = lz4_hash(w2);
          const uint32_t h = lz4_hash(w0);
          if (lane == 0) tab[h2] = (uint16_t)(ip - 2u);
          wave_lds_sync();
          const uint32_t mi = tab[h];
          wave_lds_sync();
          if (lane == 0) tab[h] = (uint16_t)ip;
          wave_lds_sync();
          // the candidate's word and the first count round from it, one round trip
          const uint32_t cand = ld32u(src + mi);
          const uint32_t x = cnt_load(ip, mi, 0u);
          if (cand == w0) {  // a new sequence with no literals
            match = mi;
            mc = count(ip, mi, x);
            continue;
          }
          ip += 1u;  // the search restarts after the probed position
          break;
        }
      }
      if (!raw) {
        const uint32_t ll = len - anchor;
        const uint32_t need = 1u + ext_bytes(ll) + ll;
        if (op + need >= len) {
          raw = true;
        } else {
          uint8_t* d = dst + op;
          if (lane == 0) d[0] = (uint8_t)(min(ll, 15u) << 4);
          put_len(d + 1, ll, lane);
          wave_copy(d + 1 + ext_bytes(ll), src + anchor, ll, lane);
          op += need;
        }
      }
      if (lane == 0) chunks[b].clen = raw ? 0u : op;
    } else if (lane == 0) {
      chunks[b].clen = 0u;
    }
  }
}

// XXH32 (seed 0x9747b28c) of every chunk's original bytes, masked to 28 bits as lz4-java's
// StreamingXXHash32.asChecksum() does.  Lanes 4g..4g+3 run the four stripe accumulators of
// chunk 16 * wave + g; the tail and avalanche on the group's first lane.
__global__ __launch_bounds__(256) void k_xxh32(const uint8_t* __restrict__ data,
                                               Lz4Chunk* __restrict__ chunks,
                                               const uint32_t* __restrict__ nchunks) {
  const uint32_t n = *nchunks;
  const int lane = threadIdx.x % kLWave, sub = lane & 3;
  const uint32_t gw = (blockIdx.x * 256u + threadIdx.x) / kLWave;
  const uint32_t waves = gridDim.x * 4u;
  for (uint32_t b0 = gw * 16u; b0 < n; b0 += waves * 16u) {
    const uint32_t b = min(b0 + (uint32_t)(lane >> 2), n - 1);
    const Lz4Chunk C = chunks[b];
    const uint8_t* s = data + C.src;
    const uint32_t len = C.len, stripes = len / 16u;
    uint32_t v = sub == 0 ? kXxhSeed + P1 + P2 : sub == 1 ? kXxhSeed + P2 : sub == 2 ? kXxhSeed : kXxhSeed - P1;
    uint32_t k = 0;
    for (; k + 8 <= stripes; k += 8) {
      uint32_t x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = ld32u(s + 16u * (k + u) + 4u * sub);
#pragma unroll
      for (int u = 0; u < 8; ++u) v = rotl(v + x[u] * P2, 13) * P1;
    }
    for (; k < stripes; ++k) v = rotl(v + ld32u(s + 16u * k + 4u * sub) * P2, 13) * P1;
    const int base = lane & ~3;
    const uint32_t v1 = __shfl((int)v, base, kLWave), v2 = __shfl((int)v, base + 1, kLWave);
    const uint32_t v3 = __shfl((int)v, base + 2, kLWave), v4 = __shfl((int)v, base + 3, kLWave);
    if (sub == 0 && b0 + (uint32_t)(lane >> 2) < n) {
      uint32_t h = len >= 16 ? rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18) : kXxhSeed + P5;
      h += len;
      uint32_t i = stripes * 16u;
      for (; i + 4 <= len; i += 4) h = rotl(h + ld32u(s + i) * P3, 17) * P4;
      for (; i < len; ++i) h = rotl(h + (uint32_t)s[i] * P5, 11) * P1;
      h ^= h >> 15;
      h *= P2;
      h ^= h >> 13;
      h *= P3;
      h ^= h >> 16;
      chunks[b].csum = h & 0x0FFFFFFFu;
    }
  }
}

// framed bytes of chunk b (0 past the chunk count: the scan runs over the host-side bound)
__global__ __launch_bounds__(256) void k_lz4_sizes(const Lz4Chunk* __restrict__ chunks,
                                                   const uint32_t* __restrict__ nchunks,
                                                   uint64_t bound, uint64_t* __restrict__ sz) {
  const uint64_t b = blockIdx.x * 256ull + threadIdx.x;
  if (b >= bound) return;
  uint64_t v = 0;
  if (b < *nchunks) {
    const Lz4Chunk C = chunks[b];
    v = kLz4Hdr + (C.clen ? C.clen : C.len) + (C.last ? kLz4Hdr : 0);
  }
  sz[b] = v;
}

// per-run framed bytes: first chunk's offset to the last chunk's end (0 for an empty run)
__global__ __launch_bounds__(256) void k_lz4_run_sizes(const uint32_t* __restrict__ b0,
                                                       const uint64_t* __restrict__ off,
                                                       const uint64_t* __restrict__ sz,
                                                       uint64_t runs,
                                                       const uint32_t* __restrict__ nchunks,
                                                       uint64_t* __restrict__ rs,
                                                       uint64_t* __restrict__ total) {
  const uint64_t r = blockIdx.x * 256ull + threadIdx.x;
  if (r >= runs) return;
  const uint32_t first = b0[r];
  const uint32_t end = (r + 1 < runs) ? b0[r + 1] : *nchunks;
  rs[r] = end > first ? (off[end - 1] + sz[end - 1] - off[first]) : 0ull;
  if (r + 1 == runs && total) *total = end > 0 ? off[end - 1] + sz[end - 1] : 0ull;
}

__global__ __launch_bounds__(256) void k_lz4_emit(const uint8_t* __restrict__ data,
                                                  const Lz4Chunk* __restrict__ chunks,
                                                  const uint32_t* __restrict__ nchunks,
                                                  const uint8_t* __restrict__ scratch,
                                                  const uint64_t* __restrict__ off, int level,
                                                  uint8_t* __restrict__ out) {
  const int wave = threadIdx.x / kLWave, lane = threadIdx.x % kLWave;
  const uint32_t n = *nchunks;
  for (uint32_t b = blockIdx.x * 4u + wave; b < n; b += gridDim.x * 4u) {
    const Lz4Chunk C = chunks[b];
    uint8_t* d = out + off[b];
    const bool raw = C.clen == 0;
    const uint32_t plen = raw ? C.len : C.clen;
    if (lane < kLz4Hdr) {
      const char* magic = "LZ4Block";
      uint8_t v;
      if (lane < 8) v = (uint8_t)magic[lane];
      else if (lane == 8) v = (uint8_t)((raw ? 0x10 : 0x20) | level);
      else {
        const int f = (lane - 9) / 4, sh = 8 * ((lane - 9) % 4);
        const uint32_t x = f == 0 ? plen : f == 1 ? C.len : C.csum;
        v = (uint8_t)(x >> sh);
      }
      d[lane] = v;
    }
    const uint8_t* s = raw ? data + C.src : scratch + ((C.src + 16ull * b) & ~3ull);
    wave_copy(d + kLz4Hdr, s, plen, lane);
    if (C.last && lane < kLz4Hdr) {
      const char* magic = "LZ4Block";
      d[kLz4Hdr + plen + lane] =
          lane < 8 ? (uint8_t)magic[lane] : lane == 8 ? (uint8_t)(0x10 | level) : (uint8_t)0;
    }
  }
}

// ---- host-side launcher -----------------------------------------------------------------------
uint64_t lz4_chunk_bound(uint64_t data_bytes, uint64_t runs, uint32_t bs) {
  return data_bytes / bs + runs + 1;
}

uint64_t lz4_output_bound(uint64_t data_bytes, uint64_t runs, uint32_t bs) {
  return data_bytes + lz4_chunk_bound(data_bytes, runs, bs) * kLz4Hdr + runs * kLz4Hdr;
}

static size_t scan_temp_bytes(uint64_t n32, uint64_t n64) {
  size_t a = 0, b = 0;
  (void)rocprim::exclusive_scan(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u,
                                (size_t)n32, rocprim::plus<uint32_t>());
  (void)rocprim::exclusive_scan(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr, 0ull,
                                (size_t)n64, rocprim::plus<uint64_t>());
  return std::max(a, b);
}

static uint64_t up256(uint64_t x) { return (x + 255) & ~255ull; }

Lz4Workspace lz4_workspace_layout(uint64_t data_bytes, uint32_t maps, uint32_t R, uint32_t bs) {
  Lz4Workspace w{};
  const uint64_t runs = (uint64_t)maps * R;
  const uint64_t cb = lz4_chunk_bound(data_bytes, runs, bs);
  uint64_t o = 0;
  w.map_base_off = o;  o += up256((maps + 1) * 8ull);
  w.nb_off = o;        o += up256(runs * 4);
  w.b0_off = o;        o += up256(runs * 4);
  w.nchunks_off = o;   o += 256;
  w.chunks_off = o;    o += up256(cb * sizeof(Lz4Chunk));
  w.sz_off = o;        o += up256(cb * 8);
  w.off_off = o;       o += up256(cb * 8);
  w.rs_off = o;        o += up256(runs * 8);
  w.base_off = o;      o += up256(3 * runs * 8);
  w.temp_off = o;
  w.temp_bytes = up256(scan_temp_bytes(runs, cb));
  o += w.temp_bytes;
  w.scratch_off = o;   o += up256(data_bytes + 16 * cb + 64);
  w.chunk_bound = cb;
  w.total = o;
  return w;
}

hipError_t launch_lz4_compress(const uint8_t* d_data, const int64_t* d_index, uint32_t maps,
                               uint32_t R, uint32_t bs, uint8_t* d_out, int64_t* d_out_index,
                               uint8_t* d_out_index_be, uint64_t* d_out_bytes, uint8_t* d_ws,
                               const Lz4Workspace& w, bool queue, hipStream_t s) {
  const uint64_t runs = (uint64_t)maps * R;
  uint64_t* map_base = reinterpret_cast<uint64_t*>(d_ws + w.map_base_off);
  uint32_t* nb = reinterpret_cast<uint32_t*>(d_ws + w.nb_off);
  uint32_t* b0 = reinterpret_cast<uint32_t*>(d_ws + w.b0_off);
  uint32_t* nchunks = reinterpret_cast<uint32_t*>(d_ws + w.nchunks_off);
  Lz4Chunk* chunks = reinterpret_cast<Lz4Chunk*>(d_ws + w.chunks_off);
  uint64_t* sz = reinterpret_cast<uint64_t*>(d_ws + w.sz_off);
  uint64_t* off = reinterpret_cast<uint64_t*>(d_ws + w.off_off);
  uint64_t* rs = reinterpret_cast<uint64_t*>(d_ws + w.rs_off);
  uint64_t* base = reinterpret_cast<uint64_t*>(d_ws + w.base_off);
  void* temp = d_ws + w.temp_off;
  uint8_t* scratch = d_ws + w.scratch_off;
  const uint32_t rg = (uint32_t)((runs + 255) / 256);
  hipLaunchKernelGGL(k_lz4_map_base, dim3(1), dim3(256), 0, s, d_index, (int)maps, (int)R, map_base);
  hipLaunchKernelGGL(k_lz4_runs, dim3(rg), dim3(256), 0, s, d_index, (int)maps, (int)R, bs, nb);
  size_t tb = w.temp_bytes;
  hipError_t e = rocprim::exclusive_scan(temp, tb, nb, b0, 0u, (size_t)runs,
                                         rocprim::plus<uint32_t>(), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_lz4_fill, dim3(rg), dim3(256), 0, s, d_index, (int)maps, (int)R, bs, map_base,
                     b0, chunks, nchunks);
  const uint32_t cg = (uint32_t)std::min<uint64_t>((w.chunk_bound + 3) / 4, 8192);
  const uint32_t zg = (uint32_t)std::min<uint64_t>((w.chunk_bound + kLz4Waves - 1) / kLz4Waves,
                                                   256u * 16u);
  uint32_t* qctr = nchunks + 1;  // the work queue's counter (nchunks_off holds 256 bytes)
  if (queue) {
    e = hipMemsetAsync(qctr, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lz4_default<true>, dim3(zg), dim3(kLz4Waves * kLWave), 0, s, d_data,
                       chunks, nchunks, scratch, qctr);
  } else {
    hipLaunchKernelGGL(k_lz4_default<false>, dim3(zg), dim3(kLz4Waves * kLWave), 0, s, d_data,
                       chunks, nchunks, scratch, qctr);
  }
  const uint32_t xg = (uint32_t)std::min<uint64_t>((w.chunk_bound + 63) / 64, 4096);
  hipLaunchKernelGGL(k_xxh32, dim3(xg), dim3(256), 0, s, d_data, chunks, nchunks);
  const uint32_t bg = (uint32_t)((w.chunk_bound + 255) / 256);
  hipLaunchKernelGGL(k_lz4_sizes, dim3(bg), dim3(256), 0, s, chunks, nchunks, w.chunk_bound, sz);
  tb = w.temp_bytes;
  e = rocprim::exclusive_scan(temp, tb, sz, off, 0ull, (size_t)w.chunk_bound,
                              rocprim::plus<uint64_t>(), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_lz4_run_sizes, dim3(rg), dim3(256), 0, s, b0, off, sz, runs, nchunks, rs,
                     d_out_bytes);
  e = launch_rows_index(rs, maps, R, base, d_out_index, d_out_index_be, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_lz4_emit, dim3(cg), dim3(256), 0, s, d_data, chunks, nchunks, scratch, off,
                     lz4_level(bs), d_out);
  return hipGetLastError();
}


// ---- the reader's side: LZ4BlockInputStream over fetched blocks (sux_decompress_blocks) ----------
// lz4-java 1.7.1 [ext] LZ4BlockInputStream.refill, as Spark's LZ4CompressionCodec opens it (stream
// concatenation on: after an end mark the next stream's header may follow, and the input may end
// at any header boundary): per chunk a 21-byte header — magic, token (method | level), compressed
// and original LE32 lengths, XXH32 & 0x0FFFFFFF — then the payload; a chunk is corrupted when the
// original length exceeds 1 << (10 + level) (or our max_block_size), a length is negative, exactly
// one of them is 0, a raw chunk's lengths differ, the LZ4 block does not decode to exactly the
// original length from exactly the compressed bytes, or the checksum differs.  An end mark
// (original length 0) must carry compressed length 0 and checksum 0.
//   k_lz4d_walk<false>  one thread per block: validate every header, count chunks + decoded bytes
//   (rocPRIM scans)     -> chunk bases, decoded block offsets (the caller's d_out_offsets)
//   k_lz4d_total        the totals; output past the capacity: error, nothing decoded
//   k_lz4d_walk<true>   the chunk table (payload offset, output offset, lengths, method, checksum)
//   k_lz4d_decode       one wave per chunk: raw -> copy; LZ4 -> payload staged in LDS, decoded
//                       in LDS, written out as one contiguous range
//   k_xxh32 + k_lz4d_verify   the checksum of every decoded chunk
__device__ __forceinline__ uint32_t rd_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__host__ __device__ __forceinline__ uint32_t lz4d_in_cap(uint32_t max_bs) {
  return max_bs + max_bs / 255u + 16u;  // LZ4_compressBound: the largest block for max_bs bytes
}
// The decoder's one buffer per wave: LZ4 in-place decompression (lz4.h, LZ4_DECOMPRESS_INPLACE_
// MARGIN): the payload staged at the END of a buffer of the decoded size + (clen >> 8) + 32, the
// output written from its start — the output never overtakes the unread input — then the parse
// window's 256-byte overhang; the byte-store sink after it.
__host__ __device__ __forceinline__ uint32_t lz4d_buf_bytes(uint32_t max_bs, uint32_t in_cap) {
  const uint32_t a = max_bs + (in_cap >> 8) + 32u + 16u, b = in_cap + 16u;
  return ((a > b ? a : b) + 15u) & ~15u;
}
__host__ __device__ __forceinline__ uint32_t lz4d_lds_bytes(uint32_t max_bs, uint32_t in_cap) {
  return lz4d_buf_bytes(max_bs, in_cap) + 4u * 64u + 4u * 64u;
}

template <bool FILL>
__global__ __launch_bounds__(256) void k_lz4d_walk(const uint8_t* __restrict__ in,
                                                   const int64_t* __restrict__ in_off, uint32_t nb,
                                                   uint64_t in_bytes, uint32_t max_bs, uint32_t* __restrict__ counts,
                                                   uint64_t* __restrict__ obytes,
                                                   const uint32_t* __restrict__ cbase,
                                                   const int64_t* __restrict__ out_off,
                                                   const uint32_t* __restrict__ ok,
                                                   Lz4DChunk* __restrict__ chunks,
                                                   Lz4Chunk* __restrict__ xc,
                                                   unsigned long long* __restrict__ total,
                                                   uint32_t* __restrict__ err) {
  const uint32_t k = blockIdx.x * 256u + threadIdx.x;
  if (k >= nb) return;
  if (FILL && (!*ok || counts[k] == 0)) return;  // capacity error, or an empty / corrupted block
  const uint64_t b = (uint64_t)in_off[k], e = (uint64_t)in_off[k + 1];
  uint64_t p = b, o = FILL ? (uint64_t)out_off[k] : 0ull;
  uint32_t c = 0;
  bool bad = in_off[k] < 0 || e < b || e > in_bytes;  // a range outside the input
  while (!bad && p < e) {
    if (e - p < (uint64_t)kLz4Hdr) { bad = true; break; }  // "Stream ended prematurely"
    const uint8_t* h = in + p;
    const char* magic = "LZ4Block";
    for (int i = 0; i < 8; ++i) bad = bad || h[i] != (uint8_t)magic[i];
    const uint32_t method = h[8] & 0xF0u, level = h[8] & 0x0Fu;
    const uint32_t clen = rd_le32(h + 9), olen = rd_le32(h + 13), chk = rd_le32(h + 17);
    p += kLz4Hdr;
    if (bad) break;
    if (olen == 0) {  // an end mark; concatenated streams may follow
      bad = clen != 0 || chk != 0 || (method != 0x10u && method != 0x20u);
      continue;
    }
    const uint64_t blk = 1ull << (10u + level);
    bad = (method != 0x10u && method != 0x20u) || (int32_t)clen <= 0 || (int32_t)olen < 0 ||
          olen > blk || olen > max_bs || (method == 0x10u && clen != olen) ||
          (method == 0x20u && clen > lz4d_in_cap(max_bs)) || e - p < clen;
    if (bad) break;
    if (FILL) {
      const uint32_t i = cbase[k] + c;
      chunks[i] = Lz4DChunk{p, o, clen, olen, method, chk};
      Lz4Chunk x;
      x.src = o;
      x.len = olen;
      x.run = k;
      x.last = 0;
      x.clen = 0;
      x.csum = 0;
      x.pad = 0;
      xc[i] = x;
    }
    ++c;
    o += olen;
    p += clen;
  }
  if (FILL) return;
  if (bad) {
    atomicOr(err, kErrLz4Stream);
    c = 0;
    o = 0;
  }
  counts[k] = c;
  obytes[k] = o;
  // the chunk total in 64 bits: blocks whose ranges overlap (non-monotone
  // in_offsets) can hold more headers than the input, and the u32 scan of counts would wrap
  if (c) atomicAdd(total, (unsigned long long)c);
}

// The totals after the scans: chunk count (0 when the decoded bytes exceed the capacity, which
// sets the error word instead), and the decoded total at out_off[nb].
__global__ void k_lz4d_total(const uint32_t* __restrict__ counts, const uint32_t* __restrict__ cbase,
                             const uint64_t* __restrict__ obytes, int64_t* __restrict__ out_off,
                             uint32_t nb, uint64_t cap, uint64_t chunk_bound,
                             const unsigned long long* __restrict__ chunk_total,
                             uint32_t* __restrict__ nchunks, uint32_t* __restrict__ ok,
                             uint32_t* __restrict__ err) {
  if (threadIdx.x != 0) return;
  const uint64_t total = nb ? (uint64_t)out_off[nb - 1] + obytes[nb - 1] : 0ull;
  // counted in 64 bits by the walk: the u32 chunk bases are valid only when this fits the table
  const uint64_t chunks = nb ? (uint64_t)*chunk_total : 0ull;
  out_off[nb] = (int64_t)total;
  const bool fits = total <= cap;
  // the ranges overlap (more headers than the input holds): a caller error, nothing decoded
  const bool table = chunks <= chunk_bound;
  if (!fits) atomicOr(err, kErrLz4Capacity);
  if (!table) atomicOr(err, kErrLz4Stream);
  *ok = fits && table ? 1u : 0u;
  *nchunks = fits && table ? (uint32_t)chunks : 0u;
  nchunks[2] = 0u;  // k_lz4d_decode's work-queue counter
}

// One wave per chunk (one wave per workgroup, its LDS = one in-place buffer: four per CU at
// 32 KiB blocks, where separate payload and output buffers allowed two).  The
// parse is LZ4's, sequence by sequence, on every lane at once (uniform control flow, the values
// made scalar with readfirstlane): a 64-byte window at the token serves the token, its length
// bytes and the offset in one LDS round trip (bytes past the window: one uniform read each); the
// literal and match copies are wave-wide, one byte per lane and step.  A match byte j is
// out[op - off + j % off] — inside what was decoded before this match even when the match
// overlaps itself — so a step's 64 bytes never depend on each other.  The decoded chunk sits in
// LDS at the output's dword phase, so it leaves as aligned dword stores (bytes at the ends).
__device__ __forceinline__ uint32_t sgpr(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

__global__ __launch_bounds__(kLWave) void k_lz4d_decode(const uint8_t* __restrict__ in,
                                                        const Lz4DChunk* __restrict__ chunks,
                                                        const uint32_t* __restrict__ nchunks,
                                                        uint32_t in_cap, uint32_t max_bs,
                                                        uint8_t* __restrict__ out,
                                                        uint32_t* __restrict__ qctr,
                                                        uint32_t* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x;
  const uint32_t n = *nchunks;
  uint8_t* ob = lds;  // decoded chunk, at its output's dword phase
  uint8_t* sink = lds + lz4d_buf_bytes(max_bs, in_cap) + 4u * kLWave + 4u * lane;
  // chunks from a work queue (k_lz4d_total zeroed its counter on this stream): a chunk's cost
  // varies with its sequences, so a fixed deal left the launch's tail to the unlucky waves; the
  // counter only grows, the index reaches the wave through readfirstlane (a wave-uniform exit)
  for (uint32_t c = lz4_claim(qctr, lane); c < n; c = lz4_claim(qctr, lane)) {
    const Lz4DChunk C = chunks[c];
    uint8_t* dst = out + C.dst;
    if (C.method == 0x10u) {  // stored raw
      wave_copy(dst, in + C.src, C.olen, lane);
      continue;
    }
    // stage the payload: every aligned dword holding a payload byte (such a dword lies in
    // mapped memory), so the copy is aligned both sides
    const uint8_t* src = in + C.src;
    const uint32_t ia = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 3u);
    const uint32_t oa = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 3u);
    // in place: the payload ends >= the in-place margin past the decoded bytes (a payload longer
    // than that — no LZ4 encoder makes one — starts at 0 and decodes to a checksum error at worst)
    const uint32_t pend = oa + C.olen + (C.clen >> 8) + 32u;
    uint8_t* ib = lds + (pend > C.clen ? ((pend - C.clen + 3u) & ~3u) : 0u);
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src - ia);
    const uint32_t nd = (ia + C.clen + 3u) / 4u;
    uint32_t* i4 = reinterpret_cast<uint32_t*>(ib);
    // 32 loads in flight per lane: a 32 KiB payload in 4 memory round trips (4 at a time took
    // 32 — the staging, not the parse, bounded the decoder)
    constexpr uint32_t SU = 32;
    for (uint32_t t = lane; t < nd; t += SU * kLWave) {
      uint32_t v[SU];
#pragma unroll
      for (uint32_t u = 0; u < SU; ++u) v[u] = s4[min(t + u * kLWave, nd - 1u)];
#pragma unroll
      for (uint32_t u = 0; u < SU; ++u)
        if (t + u * kLWave < nd) i4[t + u * kLWave] = v[u];
    }
    wave_lds_sync();
    const uint8_t* ip8 = ib + ia;
    uint8_t* op8 = ob + oa;
    const uint32_t iend = C.clen, oend = C.olen;
    uint32_t ip = 0, op = 0;
    bool bad = false;
    const uint32_t* ib32 = reinterpret_cast<const uint32_t*>(ib);
    while (true) {
      // a block ends with a literal-only sequence (the LZ4 format; liblz4's safe decoder rejects
      // a block ending in a match)
      if (ip >= iend) { bad = true; break; }
      // a 256-byte window at the token: lane l holds the dword at payload position wp + 4 l
      // (wp = the token's dword boundary; up to 3 bytes before the token, the LDS padding after
      // the payload keeps the read in bounds); the token, the length bytes, the offset and the
      // literals inside it need no LDS read of their own
      const uint32_t wq = (ia + ip) & ~3u;  // LDS offset of the window in ib
      const int wp = (int)wq - (int)ia;       // payload position of the window's first byte
      const uint32_t wv = ib32[(wq >> 2) + (uint32_t)lane];
      auto byte_at = [&](uint32_t x) -> uint32_t {  // payload byte x (< iend: checked)
        const uint32_t q = (uint32_t)((int)x - wp);
        return q < 4u * kLWave
                   ? ((uint32_t)__builtin_amdgcn_readlane((int)wv, (int)(q >> 2)) >> (8u * (q & 3u))) &
                         255u
                   : sgpr(ip8[x]);
      };
      const uint32_t tok = byte_at(ip);
      uint32_t x = ip + 1u, lit = tok >> 4;
      if (lit == 15u) {
        uint32_t b;
        do {
          if (x >= iend) { bad = true; break; }
          b = byte_at(x++);
          lit += b;
        } while (b == 255u);
        if (bad) break;
      }
      if (iend - x < lit || oend - op < lit) { bad = true; break; }
      // literals [x, x + lit) -> out[op, ...): the window's bytes by byte stores from this lane's
      // dword, the rest (a literal run past the window) LDS to LDS
      const int wend = wp + 4 * kLWave;
      {
        // unconditional byte stores (a byte outside the literal goes to this lane's slot past the
        // buffers): no branch per byte, so no wait between them
        const int p0 = wp + 4 * lane;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int pj = p0 + j;
          const bool in = pj >= (int)x && pj < (int)(x + lit);
          uint8_t* d = in ? op8 + op + (uint32_t)(pj - (int)x) : sink + j;
          *d = (uint8_t)(wv >> (8 * j));
        }
        const uint32_t from = (int)(x + lit) > wend ? (uint32_t)max(wend, (int)x) : x + lit;
        for (uint32_t k = from + lane; k < x + lit; k += kLWave) op8[op + (k - x)] = ip8[k];
      }
      op += lit;
      x += lit;
      if (x == iend) break;  // the last sequence: literals only
      if (iend - x < 2u) { bad = true; break; }
      const uint32_t off = byte_at(x) | (byte_at(x + 1u) << 8);
      x += 2u;
      uint32_t ml = (tok & 15u) + 4u;
      if ((tok & 15u) == 15u) {
        uint32_t b;
        do {
          if (x >= iend) { bad = true; break; }
          b = byte_at(x++);
          ml += b;
        } while (b == 255u);
        if (bad) break;
      }
      if (off == 0u || off > op || oend - op < ml) { bad = true; break; }
      // The literals just written may be the match's source: a wave's LDS operations execute
      // in issue order, so only the compiler must keep them in order (no wait for the writes)
      asm volatile("" ::: "memory");
      const uint32_t from = op - off;
      if (off >= ml) {
        for (uint32_t k = lane; k < ml; k += kLWave) op8[op + k] = op8[from + k];
      } else {
        for (uint32_t k = lane; k < ml; k += kLWave) op8[op + k] = op8[from + k % off];
      }
      asm volatile("" ::: "memory");
      op += ml;
      ip = x;
    }
    if (bad || op != oend) {
      if (lane == 0) atomicOr(err, kErrLz4Stream);
      continue;
    }
    wave_lds_sync();
    // out: head bytes up to dst's dword boundary, aligned dwords, tail bytes
    const uint32_t head = min(oend, (4u - oa) & 3u);
    if ((uint32_t)lane < head) dst[lane] = op8[lane];
    const uint32_t body = (oend - head) / 4u;
    const uint32_t* o4 = reinterpret_cast<const uint32_t*>(op8 + head);  // = ob + 4 (or ob)
    uint32_t* d4 = reinterpret_cast<uint32_t*>(dst + head);
    for (uint32_t t = lane; t < body; t += kLWave) d4[t] = o4[t];
    const uint32_t done = head + 4u * body;
    if ((uint32_t)lane < oend - done) dst[done + lane] = op8[done + lane];
    wave_lds_sync();  // the next chunk overwrites the buffers only after every lane read them
  }
}

__global__ __launch_bounds__(256) void k_lz4d_verify(const Lz4DChunk* __restrict__ chunks,
                                                     const Lz4Chunk* __restrict__ xc,
                                                     const uint32_t* __restrict__ nchunks,
                                                     uint32_t* __restrict__ err) {
  const uint32_t n = *nchunks;
  for (uint32_t c = blockIdx.x * 256u + threadIdx.x; c < n; c += gridDim.x * 256u)
    if (xc[c].csum != chunks[c].csum) atomicOr(err, kErrLz4Checksum);
}

uint64_t lz4d_chunk_bound(uint64_t in_bytes) { return in_bytes / kLz4Hdr + 1; }

Lz4DWorkspace lz4d_workspace_layout(uint64_t in_bytes, uint32_t nb) {
  Lz4DWorkspace w{};
  const uint64_t cb = lz4d_chunk_bound(in_bytes);
  uint64_t o = 0;
  w.counts_off = o;  o += up256((nb + 1) * 4ull);
  w.cbase_off = o;   o += up256((nb + 1) * 4ull);
  w.obytes_off = o;  o += up256((nb + 1) * 8ull);
  w.misc_off = o;    o += 256;  // nchunks, ok, the decode queue counter; u64 chunk total at +16
  w.chunks_off = o;  o += up256(cb * sizeof(Lz4DChunk));
  w.xc_off = o;      o += up256(cb * sizeof(Lz4Chunk));
  w.temp_off = o;
  w.temp_bytes = up256(scan_temp_bytes(nb, nb));
  o += w.temp_bytes;
  w.chunk_bound = cb;
  w.total = o;
  return w;
}

hipError_t launch_lz4_decompress(const uint8_t* d_in, uint64_t in_bytes, const int64_t* d_in_off,
                                 uint32_t nb, uint32_t max_bs, uint8_t* d_out, uint64_t cap,
                                 int64_t* d_out_off, uint8_t* d_ws, const Lz4DWorkspace& w,
                                 uint32_t* d_err, hipStream_t s) {
  uint32_t* counts = reinterpret_cast<uint32_t*>(d_ws + w.counts_off);
  uint32_t* cbase = reinterpret_cast<uint32_t*>(d_ws + w.cbase_off);
  uint64_t* obytes = reinterpret_cast<uint64_t*>(d_ws + w.obytes_off);
  uint32_t* nchunks = reinterpret_cast<uint32_t*>(d_ws + w.misc_off);
  uint32_t* ok = nchunks + 1;
  unsigned long long* ctotal = reinterpret_cast<unsigned long long*>(d_ws + w.misc_off + 16);
  Lz4DChunk* chunks = reinterpret_cast<Lz4DChunk*>(d_ws + w.chunks_off);
  Lz4Chunk* xc = reinterpret_cast<Lz4Chunk*>(d_ws + w.xc_off);
  void* temp = d_ws + w.temp_off;
  const uint32_t g = (nb + 255) / 256;
  if (nb) {
    hipError_t z = hipMemsetAsync(ctotal, 0, sizeof *ctotal, s);
    if (z != hipSuccess) return z;
    hipLaunchKernelGGL(k_lz4d_walk<false>, dim3(g), dim3(256), 0, s, d_in, d_in_off, nb, in_bytes,
                       max_bs, counts, obytes, nullptr, nullptr, nullptr, nullptr, nullptr, ctotal,
                       d_err);
    size_t tb = w.temp_bytes;
    hipError_t e = rocprim::exclusive_scan(temp, tb, counts, cbase, 0u, (size_t)nb,
                                           rocprim::plus<uint32_t>(), s);
    if (e != hipSuccess) return e;
    tb = w.temp_bytes;
    e = rocprim::exclusive_scan(temp, tb, obytes, reinterpret_cast<uint64_t*>(d_out_off), 0ull,
                                (size_t)nb, rocprim::plus<uint64_t>(), s);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_lz4d_total, dim3(1), dim3(64), 0, s, counts, cbase, obytes, d_out_off, nb,
                     d_out ? cap : ~0ull, w.chunk_bound, ctotal, nchunks, ok, d_err);
  if (nb == 0 || !d_out) return hipGetLastError();  // no output: the decoded sizes only
  hipLaunchKernelGGL(k_lz4d_walk<true>, dim3(g), dim3(256), 0, s, d_in, d_in_off, nb, in_bytes,
                     max_bs, counts, obytes, cbase, d_out_off, ok, chunks, xc, nullptr, d_err);
  const uint32_t in_cap = lz4d_in_cap(max_bs);
  const size_t lds = lz4d_lds_bytes(max_bs, in_cap);
  const uint32_t ncu = (uint32_t)std::max(1, stream_cus(s));
  const uint32_t per_cu = std::max<uint32_t>(1u, (uint32_t)((160u * 1024u) / lds));
  const uint32_t dg = (uint32_t)std::min<uint64_t>(w.chunk_bound, (uint64_t)ncu * per_cu);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_lz4d_decode),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k_lz4d_decode, dim3(dg), dim3(kLWave), lds, s, d_in, chunks, nchunks, in_cap,
                     max_bs, d_out, nchunks + 2, d_err);
  const uint32_t xg = (uint32_t)std::min<uint64_t>((w.chunk_bound + 63) / 64, 4096);
  hipLaunchKernelGGL(k_xxh32, dim3(xg), dim3(256), 0, s, d_out, xc, nchunks);
  const uint32_t vg = (uint32_t)std::min<uint64_t>((w.chunk_bound + 255) / 256, 1024);
  hipLaunchKernelGGL(k_lz4d_verify, dim3(vg), dim3(256), 0, s, chunks, xc, nchunks, d_err);
  return hipGetLastError();
}

}  // namespace sux
