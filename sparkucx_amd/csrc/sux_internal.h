// sux_internal.h — internal declarations shared by the C-ABI (sux_api.cpp) and the gfx950
// kernels (sux_partition.hip, sux_gen.hip, sux_copy.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>

namespace sux {

constexpr int kMaxPartitions = 32768;
constexpr int kMaxVarPartitions = 16384;  // k_vscatter: one u64 LDS cursor per partition  // LDS histogram: 128 KiB of u32 counters at the limit
constexpr int kMaxRecordSize = 4096;
constexpr int kLutBits = 10;  // range-partitioner prefix lookup: 1024 u32 entries

// Device-side partitioner (P1).  Range bounds are pre-packed as (hi, lo) big-endian words so a
// key compare is two unsigned 64-bit compares.
struct PartDev {
  int32_t kind;
  int32_t R;
  int32_t key_offset;
  int32_t key_len;
  int32_t seed;
  int32_t ascending;
  const uint64_t* bounds;  // 2*(R-1) words: bounds[2i] = hi, bounds[2i+1] = lo (RANGE only)
  // top-bits lookup: for key prefix v = hi >> (64 - lut_bits), the answer lies in
  // [lut[v] & 0xFFFF, lut[v] >> 16]; 0 bits = no table (RANGE only)
  const uint32_t* lut;
  int32_t lut_bits;
  int32_t pad;
  // a sort pass's digit shift decided on the device (make_sort_plan): when set, K1 replaces `seed`
  // with *dseed before computing any pid
  const int32_t* dseed;
  // floor((2^64 - 1) / R) + 1 (part_magic): the hash partitioners' modulo by R as two multiplies
  // (Lemire's fastmod) instead of a 32-bit division sequence per record
  uint64_t rmagic;
};
// PartDev::rmagic for R >= 1 (R = 1 wraps to 0, which the fastmod maps to remainder 0).
inline uint64_t part_magic(int32_t R) { return ~0ull / (uint64_t)R + 1ull; }

// Kernel tuning of one launch: the node's sux_tuning with every default filled in (sux_api.cpp,
// resolve_tuning).  Replaces round 1's process-wide environment overrides.
struct Tuning {
  int hist_kernel = 4;      // newest K1 variant allowed
  int scatter_kernel = 8;   // newest K3 variant allowed
  bool coresident = false;  // K1/K3 shapes that share a CU (two launch groups in flight)
  int scatter_chunk = 1024; // k_scatter7 records per chunk: 1024 | 768
  int scatter_depth = 1;    // k_scatter7 chunks loaded ahead (768-record chunks: 1 | 2)
  int hist_stage = 64;      // k_hist4 records per LDS stage: 64 | 128
  int hist_wgs_per_cu = 0;  // k_hist4 workgroups per CU (0: as many as LDS allows)
  int small_kernel = 0;     // 16-byte records, R > 1024: 1 turn-taking k_scatter16b, 2 sorted
                            // chunks, 4 two-level MSD passes (needs the temp copy)
  int scatter_order = 0;    // k_scatter8 tile order: 1 contiguous ranges, 2 block-cyclic per XCD
  int small_wgs_per_cu = 2; // k_msd16a / k_msd16b workgroups per CU (1: two groups share a CU)
  bool small_auto = true;   // small_kernel left to the default: the MSD path only when its
                            // segments are long enough to pay for their fixed cost
  int s6_chunk = 1024;      // k_scatter6 largest chunk
  int tiles_per_item = 0;   // k_scatter6/7 tiles per work item (0: 8 chunks' worth)
  int small_groups = 4;     // k_scatter16b record groups per turn: 1 | 2 | 4
  int tile_records = 0;     // K1 tile override (0: choose_tile_recs's rule)
  bool onepass = false;     // the one-pass kernel when a map batch fits on chip
  int varlen_kernel = 3;    // variable-length rows: 1 | 2 | 3 (line image; default: 1055 vs 840 GB/s)
  int varlen_tile = 0;      // variable-length K1 tile override
  bool hist_nt = false;     // k_hist4: non-temporal (streaming) record loads
  bool counts_tm = true;    // k_hist4 + k_scatter7/8: tile-major counts (MapGroup::counts_tm)
  int scatter_counters = 2; // k_scatter8 per-wave counters: 1 partition-major, 2 wave-major
  bool lz4_queue = true;    // k_lz4_default: chunks from a device work queue (else grid-stride)
  int scatter_nt = 0;       // k_scatter8 non-temporal record loads (bit 0) / line stores (bit 1)
  int gather_kernel = 3;    // the sort's record gather: 1 its own launch in 16-byte units, 2 its
                            // own launch, one dword per lane, 3 fused into the bucket sort
  bool gather16 = true;     // (1 and 3) 16-byte units
  int split_cus = 0;        // sux_partition_maps_pipelined: K1 on this many CUs beside the
                            // previous group's K3 on the others (0: one stream per group)
  int msd_direct = 0;       // k_msd16a (bit 0) / k_msd16b (bit 1): records stored from registers
                            // to their sorted place, no LDS stage
};

// Per-launch geometry of a group of consecutive map batches.
struct MapGroup {
  const uint8_t* recs;       // first record of map 0 of the group
  uint64_t records_per_map;  // records of every map but possibly the last
  uint64_t num_records;      // records in the whole group
  uint32_t num_maps;
  uint32_t rec_size;
  uint32_t tile_recs;      // records per tile (one wave's work in hist/scatter)
  uint32_t tiles_per_map;  // ceil(records_per_map / tile_recs)
  uint32_t* err;           // the node's device error word (kErr* bits), or nullptr
  // K1 -> K2 -> K3 tile counts layout: 0 partition-major [map][p][tile] (a row per (map, p) for
  // the scan), 1 tile-major [map][tile][p] (k_hist4 with k_scatter7/8: each tile's R counters
  // are one contiguous store instead of R scattered 4-byte writes)
  uint32_t counts_tm;
};
// Device error word bits (sux_node_check turns a set word into SUX_EHIP).
constexpr uint32_t kErrTurnTimeout = 1u;  // k_scatter16b: a wave waited 2^22 sleeps for its turn
constexpr uint32_t kErrLz4Stream = 2u;    // sux_decompress_blocks: a corrupted block
constexpr uint32_t kErrLz4Capacity = 4u;  // sux_decompress_blocks: output past the capacity
constexpr uint32_t kErrLz4Checksum = 8u;  // sux_decompress_blocks: a chunk's XXH32 differs

// Per-launch geometry of a group of variable-length record maps (sux_varlen.hip): record i is
// data[offs[i] - offs[0], offs[i+1] - offs[0]).
struct VarGroup {
  const uint8_t* data;
  const uint64_t* offs;      // num_records + 1 offsets (device)
  uint64_t records_per_map;
  uint64_t num_records;
  uint32_t num_maps;
  uint32_t tile_recs;
  uint32_t tiles_per_map;
  uint32_t pad;
};

// Workspace of the variable-length path: u64 tile counts [M][R][T] | totals [M][R] | bases | pids
struct VarWorkspace {
  uint64_t counts_off, totals_off, base_off, pids_off, total;
};

// Workspace carve-up (sizes in bytes), computed by workspace_layout().
struct Workspace {
  uint64_t counts_off, counts_bytes;  // u32 [map][R][tiles]  -> exclusive tile prefix in place
  uint64_t totals_off, totals_bytes;  // u64 [map][R] partition record counts
  uint64_t base_off, base_bytes;      // u64 [map][R] destination record offset of (map, p)
  uint64_t pids_off, pids_bytes;      // u16 [records] when the caller passes no pid buffer
  uint64_t op_off, op_bytes;          // one-pass kernel's sync words + scan tables (S = 100)
  uint64_t tmp_off, tmp_bytes;        // two-level small-record path: pass A's chunk-sorted copy
  uint64_t total;
};
// Small records whose map side may take the two-level MSD path (it needs the temp copy).
inline bool small_two_pass_shape(uint32_t R, uint32_t rec_size) {
  return rec_size == 16 && R > 1024 && R <= 16384;
}
Workspace workspace_layout(uint32_t R, uint32_t rec_size, uint64_t records_per_map,
                           uint64_t num_records, uint32_t tile_recs, bool need_pids,
                           bool small_tmp = false);
uint32_t choose_tile_recs(uint32_t R, uint32_t rec_size, uint64_t records_per_map,
                          const Tuning& tn);

// Destination layout of a group (K2b): map-major (Spark data files side by side), or
// peer-major for the exchange ([peer][map][partitions owned by peer]).
struct LayoutDesc {
  int32_t world;  // 1 = map-major
  uint32_t rec_size;
  // peer h owns partitions [own[h], own[h + 1]) (device, world + 1 int32; sux_node_set_ownership);
  // nullptr = the equal split [h R / world, (h + 1) R / world)
  const int32_t* own = nullptr;
};

// CUs a stream may use: its CU mask's population, or every CU of the device (sux_onepass.hip).
int stream_cus(hipStream_t s);

// One-pass map side (sux_onepass.hip): fixed 100-byte records, map batch held on chip.
uint64_t onepass_sync_bytes(uint32_t R);
bool onepass_eligible(const PartDev& pd, const MapGroup& g, int world, const void* d_out,
                      const uint64_t* d_peer_bytes, hipStream_t s, uint32_t* grid_out,
                      uint32_t* cs_out);
hipError_t launch_onepass(const PartDev& pd, const MapGroup& g, uint8_t* d_out, int64_t* d_index,
                          uint8_t* d_index_be, uint16_t* d_pids, uint8_t* d_sync, uint32_t grid,
                          uint32_t cs, hipStream_t s);

// Kernel timing slots (sux_kernel_times order).
enum KernelSlot { kHist = 0, kScan = 1, kScatter = 2, kCopy = 3, kNumSlots = 4 };
struct Timer;  // owned by the node; nullptr = no timing
void timer_begin(Timer* t, int slot, hipStream_t s);
void timer_end(Timer* t, int slot, hipStream_t s);
// Name of the kernel variant last launched in `slot` (a string literal), for sux_kernel_variant.
void timer_note(Timer* t, int slot, const char* kernel);

// Launchers (sux_partition.hip).  All enqueue on `s` and return the hipError_t of the launch.
hipError_t launch_partition_group(const PartDev& pd, const MapGroup& g, const LayoutDesc& lay,
                                  uint8_t* d_out, int64_t* d_index, uint8_t* d_index_be,
                                  uint16_t* d_pids, uint8_t* d_ws, const Workspace& ws,
                                  uint64_t* d_peer_bytes, const Tuning& tn, Timer* timer,
                                  hipStream_t s, hipStream_t s_k1 = nullptr,
                                  hipEvent_t k1_done = nullptr);
hipError_t launch_varlen_group(const PartDev& pd, const VarGroup& g, uint8_t* d_out,
                               int64_t* d_index, uint8_t* d_index_be, const uint16_t* d_pids_in,
                               uint16_t* d_pids, uint8_t* d_ws, const VarWorkspace& ws,
                               const Tuning& tn, Timer* timer, hipStream_t s);
VarWorkspace varlen_workspace_layout(uint32_t R, uint64_t records_per_map, uint64_t num_records,
                                     uint32_t tile_recs);
uint32_t choose_varlen_tile(uint32_t R, uint64_t rows, const Tuning& tn);
// K2b of the variable-length path (sux_partition.hip, k_map_scan): per-(map, partition) byte
// totals -> index tables in bytes + byte bases of every (map, partition) run
hipError_t launch_varlen_map_scan(const VarGroup& g, int R, const uint64_t* totals, uint64_t* base,
                                  int64_t* d_index, uint8_t* d_index_be, hipStream_t s);
// ---- compressed map outputs (sux_lz4.hip) ----
struct Lz4Chunk {            // one <= blockSize piece of a (map, partition) run
  uint64_t src;              // byte offset in the map-output buffer
  uint32_t len, run, last;   // bytes, run id (map * R + partition), last piece of its run
  uint32_t clen, csum, pad;  // LZ4 block bytes (0: stored raw), XXH32 & 0x0FFFFFFF
};
struct Lz4Workspace {
  uint64_t map_base_off, nb_off, b0_off, nchunks_off, chunks_off, sz_off, off_off, rs_off,
      base_off, temp_off, temp_bytes, scratch_off, chunk_bound, total;
};
uint64_t lz4_chunk_bound(uint64_t data_bytes, uint64_t runs, uint32_t bs);
uint64_t lz4_output_bound(uint64_t data_bytes, uint64_t runs, uint32_t bs);
Lz4Workspace lz4_workspace_layout(uint64_t data_bytes, uint32_t maps, uint32_t R, uint32_t bs);
hipError_t launch_lz4_compress(const uint8_t* d_data, const int64_t* d_index, uint32_t maps,
                               uint32_t R, uint32_t bs, uint8_t* d_out, int64_t* d_out_index,
                               uint8_t* d_out_index_be, uint64_t* d_out_bytes, uint8_t* d_ws,
                               const Lz4Workspace& w, bool queue, hipStream_t s);
// The reader's side (sux_decompress_blocks): one LZ4Block chunk of a fetched block.
struct Lz4DChunk {
  uint64_t src, dst;                  // payload offset in the input, decoded offset in the output
  uint32_t clen, olen, method, csum;  // header fields (method 0x10 raw / 0x20 LZ4)
};
struct Lz4DWorkspace {
  uint64_t counts_off, cbase_off, obytes_off, misc_off, chunks_off, xc_off, temp_off, temp_bytes,
      chunk_bound, total;
};
uint64_t lz4d_chunk_bound(uint64_t in_bytes);
Lz4DWorkspace lz4d_workspace_layout(uint64_t in_bytes, uint32_t num_blocks);
hipError_t launch_lz4_decompress(const uint8_t* d_in, uint64_t in_bytes, const int64_t* d_in_off,
                                 uint32_t nb, uint32_t max_bs, uint8_t* d_out, uint64_t cap,
                                 int64_t* d_out_off, uint8_t* d_ws, const Lz4DWorkspace& w,
                                 uint32_t* d_err, hipStream_t s);
hipError_t launch_rows_index(const uint64_t* sizes, uint32_t maps, uint32_t R, uint64_t* base,
                             int64_t* d_index, uint8_t* d_index_be, hipStream_t s);
hipError_t launch_partition_ids(const PartDev& pd, const uint8_t* recs, uint32_t rec_size,
                                uint64_t n, uint16_t* d_pids, hipStream_t s);

// Batched device copy (sux_copy.hip): n descriptors {src, dst, bytes}.
struct CopyDesc {
  const uint8_t* src;
  uint8_t* dst;
  uint64_t bytes;
};
hipError_t launch_gather_copy(const CopyDesc* d_desc, uint32_t n, uint32_t chunks_total,
                              const uint32_t* d_chunk_first, Timer* timer, hipStream_t s);

// out[i] = *ptrs[i] (device pointers to int64 index entries; sux_copy.hip).
// one map of a device resolve: its index table (nullptr: not resolvable on the device) and the
// device address of its data file
struct ResolveMap {
  const int64_t* index;
  uint64_t base;
};
hipError_t launch_resolve_blocks(const void* d_blocks, uint32_t n, const ResolveMap* d_maps,
                                 int32_t num_maps, int32_t R, uint64_t* d_addrs, int64_t* d_sizes,
                                 hipStream_t s);
hipError_t launch_gather_i64(const int64_t* const* d_ptrs, uint32_t n, int64_t* d_out,
                             hipStream_t s);

// One-sided pull of a peer-major group from mapped peer buffers (sux_copy.hip).
hipError_t launch_pull(int32_t W, int32_t me, const uint64_t* srcs, const int64_t* gi, int32_t M,
                       int32_t R, uint8_t* recv, uint64_t cap, uint64_t* recv_bytes,
                       hipStream_t s, const int32_t* own = nullptr);

// Reduce-side sort (sux_sort.hip): (key, index) pairs, and the final gather of whole records.
constexpr int kPartRadix = 7;  // internal partitioner: 12-bit digit (shift in PartDev::seed)
constexpr int kRadixBits = 12;
struct SortPlanDev;
// k_sort_pairs + the key span; with `plan`, the span's reduction also plans the MSD sort (bits:
// key bits with the segment id, tb: top-digit bits).
hipError_t launch_sort_pairs(const uint8_t* in, uint64_t n, uint32_t rs, int kind, int key_offset,
                             int key_len, const int64_t* seg, int nseg, int sbytes, void* pairs,
                             void* span_ws, bool inline_rec, hipStream_t s, int bits = 0,
                             int tb = 0, SortPlanDev* plan = nullptr, int ranged = 0);
hipError_t launch_unpair_records(const void* pairs, uint64_t n, uint32_t rs, int kind,
                                 int key_offset, int key_len, int sbytes, void* out, hipStream_t s);
// span_ws: 8 u32 (AND of key words 0..2, OR of key words 0..2) + kSortSpanBlocks x 8 u32 partials
constexpr uint32_t kSortSpanBlocks = 2048;
// header (8 u32) + per block 16 u32: AND of key words 0..2, OR of them, 2 spare, then the
// smallest and the largest pair as big-endian 128-bit values (4 u32 each)
constexpr uint64_t kSortSpanBytes = 4ull * (8 + 16ull * kSortSpanBlocks);
hipError_t launch_gather_records_sel(const void* in, const void* pairs_a, const void* pairs_b,
                                     const uint32_t* sel, uint64_t n, uint32_t rs, void* out,
                                     hipStream_t s, bool gather16 = true);
hipError_t launch_unpair_records_sel(const void* pairs_a, const void* pairs_b, const uint32_t* sel,
                                     uint64_t n, uint32_t rs, int kind, int key_offset,
                                     int key_len, int sbytes, void* out, hipStream_t s);
hipError_t launch_gather_records(const void* in, const void* pairs, uint64_t n, uint32_t rs,
                                 void* out, hipStream_t s);
// MSD finish of the sort (sux_sort.hip): buckets of <= kSortLocalCap pairs sorted in LDS by
// the listed 8-bit digits (shifts into the big-endian pair, least significant first).
constexpr uint32_t kSortLocalCap = 4096;
struct SortDigits {
  uint64_t lo, hi;  // shift of digit d in byte d (lo: digits 0..7, hi: 8..15)
  int32_t n;
  int32_t pad;
  __host__ __device__ void push(uint32_t sh) {
    if (n < 8) lo |= (uint64_t)sh << (8 * n);
    else hi |= (uint64_t)sh << (8 * (n - 8));
    ++n;
  }
};
// The device-planned sort (sux_sort_records with no host wait): make_sort_plan (in k_span_reduce) fills the first
// fields from the key span (before the top-digit pass); every later
// kernel of the sort reads its decision from here.
struct SortPlanDev {
  int32_t top_lo;    // shift of the top digit (the tb highest varying key bits)
  int32_t hb;        // highest varying key bit; -1: every key is equal (the sort is the identity)
  uint32_t msd_ok;   // 1: the bucket sorts finish the sort (0: every key is equal)
  uint32_t big;      // 1: some bucket may exceed kSortLocalCap (k_gather_rest has work); set by
                     // make_sort_plan, cleared by k_top_scan when every bucket fits
  uint32_t final_b;  // 1: the sorted pairs end in buffer b, 0: in buffer a
  int32_t kbits;     // key bits (with the segment id): the top kbits of the big-endian pair
  uint64_t top_base; // the top digit is ((key >> top_lo) - top_base) & (2^tb - 1): with the key
                     // range (min, max) of a ranged plan, top_lo is the lowest shift whose
                     // aligned blocks [min, max] spans fit 2^tb buckets and top_base = min >>
                     // top_lo, so every bucket is used; 0 = the bits [top_lo, top_lo + tb)
  SortDigits dg;     // the LDS sort's digits: 8-bit, below top_lo, only those that vary
  // Rebased plan (fused-gather sorts whose key range fills too few aligned buckets, e.g. one
  // range partition's keys): the top digit is ((K - kmin) >> rq) * rm >> 32 over the key K (the
  // pair's top kbits), every bucket an equal slice of [kmin, kmax]; k_sort_local then sorts a
  // bucket by u = K - (the bucket's smallest K) < 2^rbits, placed in the pair's top rbits (the
  // record index stays), with `dg` hanging down from bit 128; dg_raw = the whole key's digits,
  // for the global-memory sort of oversized buckets (their pairs are not rebased).
  int32_t rebase;
  int32_t rbits;
  uint32_t rq;
  uint32_t pad2;
  uint64_t rm;
  uint64_t kmin_hi, kmin_lo;  // kmin (the key, right-aligned) as a 128-bit value
  SortDigits dg_raw;
};
constexpr uint64_t kSortPlanBytes = 256;
static_assert(sizeof(SortPlanDev) <= kSortPlanBytes, "plan slot");
// The sort of every top-digit bucket, driven by the plan (a no-op unless plan->msd_ok): one LDS
// launch per bucket-size class (each bucket on the smallest shape that holds it), then buckets
// above kSortLocalCap through global memory.
// recs_out != nullptr (the fused sort): the LDS launches gather their buckets' records from
// recs_in straight into recs_out instead of writing sorted pairs; launch_gather_rest then gathers
// every record they did not (needs sort_gather_fusable(rs)).  avg: the pairs per bucket on
// average (n >> tb): above 1024 the (0, 1024] class is left to the 2048-pair shape.
// Chunked top pass (round 4): each 4096-pair chunk of the pairs sorted by the top digit in place
// into `chunked`, offs[chunk][0..R] its bucket starts (u16), then the bucket index (bytes).  A
// sort with R = 2^tb <= 4096 buckets and at most kTopMaxChunks chunks takes it.
constexpr uint32_t kTopChunk = 4096;
constexpr uint32_t kTopSegs = 32;        // chunk segments of the bucket-size column sums
constexpr uint32_t kTopMaxChunks = 2048; // run table of the 1024-pair LDS shape (2 u32 per chunk)
constexpr int kTopMaxBits = 12;
hipError_t launch_top_chunks(const void* pairs, uint64_t n, int tb, SortPlanDev* plan,
                             void* chunked, uint16_t* offs, uint32_t* tot, int64_t* index,
                             hipStream_t s);
// Where k_sort_local finds its buckets after the chunked top pass (pairs == nullptr: contiguous
// at their index range of in_pairs, the one-pass top pass's output).
struct SortRuns {
  const void* pairs = nullptr;
  const uint16_t* offs = nullptr;
  uint32_t nch = 0;
};
// A side stream (with its fork / join events) for the large-bucket launches; s == nullptr: all on
// the caller's stream (under graph capture).
struct SortSide {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
hipError_t launch_sort_local_planned(const void* in_pairs, void* out_pairs, const int64_t* d_index,
                                     uint32_t R, const SortPlanDev* plan, hipStream_t s,
                                     const void* recs_in = nullptr, void* recs_out = nullptr,
                                     uint32_t rs = 0, const SortRuns& runs = SortRuns{},
                                     const SortSide& side = SortSide{}, uint64_t avg = 0);
bool sort_gather_fusable(uint32_t rs);
hipError_t launch_gather_rest(const void* recs_in, const void* pairs_a, const void* pairs_b,
                              const int64_t* d_index, uint32_t R, uint64_t n,
                              const SortPlanDev* plan, uint32_t rs, void* recs_out, hipStream_t s);


// Generators (sux_gen.hip).
hipError_t launch_generate(int kind, uint64_t seed, uint64_t first, uint64_t n,
                           const uint64_t* d_zipf_bounds, const uint64_t* d_zipf_thresh,
                           int zipf_nb, uint8_t* d_out, hipStream_t s);

// Host-side Zipf table (bit-identical construction to oracle/oracle.c).
int zipf_table_size(uint64_t zipf_n);
void zipf_table(double s, uint64_t zipf_n, uint64_t* bounds, uint64_t* thresh);

}  // namespace sux
