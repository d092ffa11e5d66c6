/*
 * sparkucx_amd.h — C-ABI of the MI355X shuffle data path (libsparkucx_amd.so).
 *
 * This is the drop-in boundary under SparkUCX's Spark-3.0 plugin surface.  Every entry point
 * names the reference interface it replaces (paths relative to the reference checkout,
 * src/main/{scala,java}/org/apache/spark/shuffle/...).  A JNI shim binds these
 * symbols 1:1; nothing in this header uses C++ or torch types.
 *
 * Conventions:
 *   - every function returns SUX_OK (0) or a negative SUX_E* code; sux_last_error() gives the
 *     message of the last failure on the calling thread; no C++ exception crosses the boundary;
 *   - handles are opaque; device pointers are plain `void*` in the node's HIP device space;
 *   - `stream` arguments are hipStream_t passed as `void*`; NULL = the HIP null stream.  A task
 *     thread that wants its own ordering domain (the analog of UcxNode.getThreadLocalWorker,
 *     UcxNode.java:147-176) passes its own stream or hipStreamPerThread;
 *   - all integers are fixed-width; byte counts are uint64_t.
 */
#ifndef SPARKUCX_AMD_H_
#define SPARKUCX_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SUX_ABI_VERSION 6

/* ---- status codes ---------------------------------------------------------------------- */
#define SUX_OK 0
#define SUX_EINVAL -1  /* bad argument (IllegalArgumentException / assume() failure)         */
#define SUX_ENOMEM -2  /* device or host allocation failed                                    */
#define SUX_EHIP -3    /* HIP runtime error                                                   */
#define SUX_ECOMM -4   /* RCCL error (UcxException on the transport in the reference)        */
#define SUX_ENOENT -5  /* unknown shuffle / map output / block (SparkException "Unknown block") */
#define SUX_ESTATE -6  /* wrong lifecycle state (IllegalStateException "must be initialized") */
#define SUX_ERANGE -7  /* size limit exceeded (SparkException "Metadata block size ...")      */
#define SUX_EIO -8     /* file I/O error (IOException "fail to rename file ...")              */

/* ---- partitioners ---------------------------------------------------- */
/* Spark RangePartitioner over an unsigned lexicographic byte key (TeraSort's 10-byte key):
 * pid = #{ i : bounds[i] < key }  (RangePartitioner.getPartition [ext], bounds strictly rising). */
#define SUX_PART_RANGE_BYTES 1
/* Spark SQL HashPartitioning of one LongType column: pmod(Murmur3_x86_32.hashLong(key, seed), R),
 * key = little-endian int64 at key_offset (UnsafeRow word order).                              */
#define SUX_PART_MURMUR3_LONG 2
/* Spark SQL HashPartitioning of one IntegerType column: pmod(hashInt(key, seed), R).           */
#define SUX_PART_MURMUR3_INT 3
/* Spark SQL HashPartitioning of one BinaryType column: pmod(hashUnsafeBytes(key, seed), R)
 * (legacy tail-byte mixing, see oracle/oracle.c).                                              */
#define SUX_PART_MURMUR3_BYTES 4
/* RDD HashPartitioner on a java.lang.Long key: nonNegativeMod(Long.hashCode(key), R).          */
#define SUX_PART_HASH_LONG 5
/* RDD HashPartitioner on a java.lang.Integer key: nonNegativeMod(key, R).                      */
#define SUX_PART_HASH_INT 6

typedef struct sux_partitioner_desc {
  int32_t kind;           /* SUX_PART_*                                                        */
  int32_t num_partitions; /* R, 1 .. 32768 (LDS-resident counters)                            */
  int32_t key_offset;     /* byte offset of the key inside a record                            */
  int32_t key_len;        /* key bytes: RANGE 1..16, MURMUR3_BYTES 1..64, LONG 8, INT 4        */
  int32_t seed;           /* Murmur3 seed (Spark SQL uses 42)                                  */
  int32_t ascending;      /* RANGE only: 1 = ascending (Spark default), 0 = descending         */
  const uint8_t* range_bounds; /* RANGE only: host array of (R-1)*key_len bytes, strictly rising */
} sux_partitioner_desc;

/* ---- node (UcxNode, UcxNode.java:60-96 / close :194-221) -------------------------------- */
typedef struct sux_node sux_node;
typedef struct sux_partitioner sux_partitioner;
typedef struct sux_buffer sux_buffer;

typedef struct sux_conf {
  int32_t device;     /* HIP device ordinal this executor owns                                 */
  int32_t rank;       /* rank of this executor in the node's exchange group                    */
  int32_t world_size; /* executors (GPUs) in the exchange group; 1 = local resolve only        */
  int32_t num_streams;/* internal streams (compute + comm); 0 = default (2)                    */
  uint8_t comm_id[128];         /* RCCL unique id from sux_comm_unique_id(); all-zero = no comm at world_size 1 */
  uint64_t min_buffer_size;     /* spark.shuffle.ucx.memory.minBufferSize (UcxShuffleConf.scala:66-72) */
  uint64_t min_allocation_size; /* spark.shuffle.ucx.memory.minAllocationSize (:74-81)         */
  uint64_t metadata_block_size; /* 2*spark.shuffle.ucx.rkeySize (:32-40): directory slot bytes */
  /* spark.shuffle.ucx.memory.preAllocateBuffers (UcxShuffleConf.scala:52-64): num_prealloc
   * (size, count) pairs preallocated in the device pool when an executor node starts
   * (MemoryPool.preAlocate, MemoryPool.java:170-176, called for executors only at UcxNode.java:81-83). */
  uint32_t num_prealloc;
  /* spark.shuffle.ucx.gpu.poolLimitMiB: cap on the device pool's allocations in MiB (0 = none).
   * Past it an allocation fails like a failed hipMalloc; with a spill directory the node then
   * spills committed map outputs to Spark's files (sux_node_set_spill_dir) and retries. */
  uint32_t pool_limit_mib;
  uint64_t prealloc_size[16];
  uint64_t prealloc_count[16];
} sux_conf;
#define SUX_MAX_PREALLOC 16

/* Fill defaults (UcxShuffleConf.scala:17-90): 1 KiB min buffer, 4 MiB min allocation, 300 B slot,
 * nothing preallocated. */
void sux_conf_init(sux_conf* conf);
/* Parse Spark's preAllocateBuffers string ("4k:1000,16k:500": Utils.byteStringAsBytes sizes,
 * decimal counts; "" = none) into conf->prealloc_*.  SUX_EINVAL on a malformed entry. */
int sux_conf_set_prealloc(sux_conf* conf, const char* spec);

int sux_abi_version(void);
/* Message of the last failed call on this thread; returns the full length. */
int sux_last_error(char* buf, size_t len);

/* Bootstrap of the exchange group.  Replaces the executor->driver tag-send of worker addresses
 * (UcxNode.startExecutor, UcxNode.java:130-145; RpcConnectionCallback.java:47-89): rank 0 makes
 * the id and any side channel (Spark RPC, torch.distributed store) carries the 128 bytes. */
int sux_comm_unique_id(uint8_t out[128]);

int sux_node_create(const sux_conf* conf, int is_driver, sux_node** out);
int sux_node_destroy(sux_node* node);

/* Host all-gather supplied by the embedding runtime (Spark RPC through the driver in a JVM; a
 * torch.distributed store or gloo group in tests): every rank of the node's group passes `bytes`
 * bytes in `send`; on return `recv` holds world_size * bytes, rank r's bytes at r * bytes.  `tag`
 * names the collective: (shuffle id << 32) | the shuffle's all-gather sequence number — equal on
 * every rank for the same call, so a control plane keys its rounds by it (not by arrival).  It is
 * the control plane the reference builds from UCX tag messages (UcxNode.startExecutor,
 * UcxNode.java:130-145; RpcConnectionCallback.java:47-89).  Return 0 on success.  With a
 * bootstrap and no RCCL communicator, sux_exchange moves the blocks by one-sided pulls from the
 * owners' device memory over HIP IPC (xGMI peer reads) — the GET model of the reference — so the
 * exchange also runs where RCCL cannot (several ranks on one GPU). */
typedef int (*sux_allgather_fn)(void* ctx, uint64_t tag, const void* send, uint64_t bytes,
                                void* recv);
int sux_node_set_bootstrap(sux_node* node, sux_allgather_fn fn, void* ctx);

/* Join the group's RCCL communicator now, after the node exists: rank 0 makes the unique id,
 * the node's bootstrap all-gathers it (tag SUX_TAG_COMM_ID), and every rank calls
 * ncclCommInitRank — a collective over the whole group, so a runtime calls it where every rank
 * gets to it without depending on its tasks: the JVM's exchange thread, before the first
 * exchange window the driver relays to every executor.  A node then starts without blocking on
 * its peers (hello -> rank -> node), the way the reference's executors connect to a peer only
 * when they first fetch from it (UcxWorkerWrapper.getConnection, UcxWorkerWrapper.scala:129-152).
 * Idempotent (a node that has a communicator returns SUX_OK); needs the bootstrap
 * (SUX_ESTATE without one); at world size 1 it makes a one-rank communicator.  Not concurrent
 * with the node's own exchange calls. */
#define SUX_TAG_COMM_ID 0xFFFFFFFF00000000ull
int sux_node_connect(sux_node* node);

/* ---- executor group membership (driver side) --------------------------------------------- *
 * The reference's executors introduce themselves to the driver with their BlockManagerId
 * (UcxNode.startExecutor, UcxNode.java:111-145) and the driver fans every address out to every
 * peer (RpcConnectionCallback.java:47-89).  The executors of a GPU group all start from the SAME
 * SparkConf, so nothing in it can tell an executor its rank: the driver keeps one sux_group per
 * application and answers each executor's hello with its rank, in order of first arrival, keyed
 * by executor id (a repeated hello — a lost reply, a retried RPC — gets the same answer), and its
 * local index = how many executors of the same host joined before it: the GPU an executor takes
 * when Spark assigned it none.  Host-only (no HIP call, usable on a driver without a GPU) and
 * thread-safe.  An executor that joins a complete group is SUX_ERANGE (the group is formed once:
 * an RCCL communicator cannot take a replacement rank). */
typedef struct sux_group sux_group;
int sux_group_create(int32_t world_size, sux_group** out);
int sux_group_destroy(sux_group* group);
int sux_group_join(sux_group* group, const char* executor_id, const char* host, int32_t* rank,
                   int32_t* local_index);
/* Executors joined so far. */
int sux_group_size(sux_group* group, int32_t* joined);

/* HBM-capacity fallback (the reference serves every block from Spark's disk files,
 * CommonUcxShuffleBlockResolver.scala:45-58; here map outputs live in HBM): when the device pool
 * cannot hold a new map output, the node writes committed map outputs of its shuffles to
 * Spark's data + index files under `dir` (spark.local.dir), frees their device memory and
 * retries.  Spilling runs at world size 1 only (a node of a larger group never spills: its peers
 * may read its slabs).  A shuffle any of whose blocks sux_resolve_blocks returned is never
 * spilled before sux_unregister_shuffle (its addresses are read without a reference).  Spilled
 * blocks are served by sux_fetch_blocks from the files; sux_resolve_blocks reports them as not
 * device-resident.  `dir` should be private to this executor and application (two nodes spilling
 * into one directory would overwrite each other's files) and must exist.  NULL or ""
 * disables spilling (allocation failures then return SUX_ENOMEM). */
int sux_node_set_spill_dir(sux_node* node, const char* dir);
/* Map outputs spilled so far by this node. */
int sux_node_spills(sux_node* node, uint64_t* spilled_maps);

/* Device pool counters (MemoryPool's close-time stats, MemoryPool.java:30-39): bytes held in
 * device allocations, get() requests, allocations made, preallocated slabs. */
int sux_pool_stats(sux_node* node, uint64_t* allocated_bytes, uint64_t* requests, uint64_t* allocs,
                   uint64_t* preallocs);

/* Kernel tuning table of one node.  Every field 0 = the measured default (DESIGN.md §4 records
 * the sweeps behind each); a value outside a field's listed set is SUX_EINVAL.  Set it between
 * calls (not while another thread is inside a call on the same node); workspace sizes follow
 * it (tile_records), so query sux_partition_workspace_size after a change.  No knob changes a
 * byte of any output: every variant is parity-tested against the CPU oracle. */
typedef struct sux_tuning {
  int32_t hist_kernel;      /* newest K1 variant allowed: 1, 3, 4 (2 was retired in round 3)    */
  int32_t scatter_kernel;   /* newest K3 variant allowed: 1, 6, 7, 8 (2 was retired in round 3) */
  int32_t coresident;       /* 1: in calls that keep two launch groups in flight, K3 shapes that
                               leave a K1 workgroup room on the CU (measured slower: opt-in);
                               0 or -1: not                                                     */
  int32_t scatter_chunk;    /* k_scatter7 records per chunk: 1024, 768, 512 (0: 768 co-resident,
                               else 1024); 512 = 512-thread workgroups, two per CU at small R   */
  int32_t scatter_depth;    /* k_scatter7 chunks loaded ahead: 1, 2 (768-record chunks only)     */
  int32_t hist_stage;       /* k_hist4 records per LDS stage: 64, 128 (0: 64)                   */
  int32_t s6_chunk;         /* k_scatter6 largest records per chunk: 1024, 512, 384, 256         */
  int32_t tiles_per_item;   /* k_scatter6/7 tiles per work item (0: 8 chunks' worth), 1 .. 4096  */
  int32_t small_groups;     /* k_scatter16b record groups per turn: 1, 2, 4                       */
  int32_t tile_records;     /* K1 tile: power of two in [64, 2^22] (0: 4096, or more for big R)  */
  int32_t onepass;          /* 1: the one-pass kernel whenever a map batch fits on chip          */
  int32_t varlen_kernel;    /* variable-length rows: 1, 2, 3 (128-B line image; 0: 3)            */
  int32_t varlen_tile;      /* variable-length K1 tile: multiple of 64 in [64, 65536]            */
  int32_t sort_max_digit_bits; /* widest radix digit of sux_sort_records: 8 .. 16                */
  int32_t sort_gather;      /* 1: records gathered after the sort instead of riding in the pairs */
  int32_t sort_all_passes;  /* 1: every digit pass runs (no key-span read-back)                  */
  int32_t hist_wgs_per_cu;  /* k_hist4 workgroups per CU: 1 .. 8 (0: as many as LDS allows)     */
  int32_t small_kernel;     /* 16-byte records, R > 1024: 1 turn-taking scatter, 2 sorted chunks,
                               4 two-level MSD passes without K1 (map-major, R <= 16384);
                               3 (two passes through bucket order) was retired in round 3    */
  int32_t small_waves;      /* 8 or 16; no effect since round 3 (it shaped the retired
                               small_kernel 3), kept so the table's layout does not move      */
  int32_t scatter_order;    /* k_scatter8 tiles: 1 one contiguous range per workgroup (0), 2
                               blocks dealt round robin among an XCD's workgroups (slower)     */
  int32_t small_wgs_per_cu; /* two-level small-record kernels (small_kernel 4): workgroups per CU
                               of each pass, 1 or 2 (0: 2); 1 lets two launch groups' passes
                               share every CU                                                  */
  int32_t sort_msd;         /* reduce-side sort: 1 (0) top digit + per-bucket LDS sort, the top
                               digit chunked (chunks sorted in place, buckets read as runs) when
                               it has <= 12 bits and n <= 2048 x 4096; 3 the same with the one-
                               pass top-digit partition; 2 LSD digit passes only               */
  int32_t exchange_self;    /* 1: the exchange also moves this rank's own maps' owned ranges
                               through its transport into the receive buffer (loopback; at
                               world 1 it runs the whole RCCL / IPC path on one GPU); 0 or -1: no */
  int32_t hist_nt;          /* k_hist4 record loads: 1 or 0 non-temporal (streaming), -1 plain  */
  int32_t counts_layout;    /* k_hist4 + k_scatter7/8 tile counts: 1 partition-major, 2 (0)
                               tile-major (one contiguous store of a tile's R counters)        */
  int32_t scatter_counters; /* k_scatter8 per-wave rank counters in LDS: 1 partition-major
                               [R][waves] (round 2), 2 (0) wave-major [waves][R]               */
  int32_t lz4_queue;        /* LZ4 compressor chunk deal: 1 (0) a device work queue (one atomic
                               per chunk), 2 the fixed grid-stride deal                        */
  int32_t scatter_nt;       /* k_scatter8 non-temporal accesses: 1 loads, 2 stores, 3 both,
                               -1 or 0 none                                                    */
  int32_t gather_kernel;    /* sort's record gather: 3 (0) fused into the LDS bucket sort (each
                               sorted bucket gathers its own records; records <= 1024 B), 1 its
                               own launch in 16-byte units, L lanes per record, 2 its own
                               launch, one dword per lane                                      */
  int32_t split_cus;        /* sux_partition_maps_pipelined: 32..224 (multiple of 32) K1 of
                               group g runs on that many CUs beside group g-1's K2 + K3 on the
                               others (K1 holds its rate on few CUs, K3 scales with them);
                               -1 or 0 every group's K1 -> K2 -> K3 on one of two streams    */
  int32_t msd_direct;       /* two-level small-record passes (small_kernel 4): bit 0 pass A, bit 1
                               pass B store each record from its registers straight to its
                               sorted place instead of through the LDS stage (measured slower);
                               bit 2: pass A prefetches its next chunk into LDS by DMA
                               (global_load_lds), one workgroup per CU; bit 3: 32-partition
                               buckets, 512-thread pass-B workgroups; bit 4: pass B finds each
                               element's run in an LDS map instead of a binary search; bit 5
                               (with 3 + 4): pass B gathers the next segment while the current
                               one is written out (maps of <= 256 chunks); bit 6 (with 3):
                               pass A ranks with one returning LDS atomic per digit group on
                               u32 counters; bit 7 (with 3): pass A matches digits on a 6-bit
                               lane tag instead of the digit bits; 0: bits 3 + 4 + 7 (the
                               measured default), -1: none (round 4's shape)                  */
  int32_t reserved[1];
} sux_tuning;
int sux_node_set_tuning(sux_node* node, const sux_tuning* tuning);
/* Waits for the device, then reports (and clears) failures the kernels recorded in the node's
 * device error word: a bounded in-kernel wait that timed out (the kernel stopped without
 * writing through it).  SUX_EHIP names the failure; SUX_OK when none.  The asynchronous calls
 * cannot return such a failure themselves; call this after synchronising on their stream. */
int sux_node_check(sux_node* node);
int sux_node_get_tuning(sux_node* node, sux_tuning* tuning);

/* ---- partitioner object: P1 (UcxShuffleManager.getWriter picks the writer, :36-50) ---------- */
int sux_partitioner_create(sux_node* node, const sux_partitioner_desc* desc, sux_partitioner** out);
int sux_partitioner_destroy(sux_partitioner* part);

/* ---- map side, stateless: P1+P2+P3 over device-resident map batches ------------------------ *
 * Partition `num_records` fixed-size records (record_size % 4 == 0, 4 .. 4096) laid out as
 * consecutive map batches of `records_per_map` records (the last one may be shorter).  For each
 * map batch m the output is Spark's sort-shuffle data file restated on the GPU: its records
 * regrouped by partition id 0..R-1, stable within a partition, written to
 * d_out + m*records_per_map*record_size, and its index file: R+1 cumulative
 * byte offsets starting at 0, native int64 into d_index[m*(R+1) ..] and, if d_index_be is not
 * NULL, big-endian bytes into d_index_be[m*(R+1)*8 ..] — the exact bytes of IndexShuffleBlockResolver.
 * d_pids (nullable) receives each record's partition id as uint16 in input order.
 * Workspace: sux_partition_workspace_size().  Everything is enqueued on `stream`; no host sync. */
int sux_partition_workspace_size(const sux_partitioner* part, uint32_t record_size,
                                 uint64_t records_per_map, uint64_t num_records, uint64_t* bytes);
int sux_partition_maps(sux_node* node, const sux_partitioner* part, const void* d_records,
                       uint32_t record_size, uint64_t records_per_map, uint64_t num_records,
                       void* d_out, int64_t* d_index, uint8_t* d_index_be, uint16_t* d_pids,
                       void* d_workspace, uint64_t workspace_bytes, void* stream);

/* sux_partition_maps over many map batches at once, the way Spark runs map tasks: several in
 * flight.  The records are cut into launch groups of `group_records` (a multiple of
 * records_per_map; 0 = 2^27 records' worth of whole maps) and the groups are dealt to two
 * node-owned streams, so that while group g scatters (K3, one LDS-bound workgroup per CU) group
 * g+1 histograms (K1's launch gaps and tail fill with the other group's work).  Output, index tables and
 * d_index_be exactly as ONE sux_partition_maps call over all num_records would write them.  The
 * node owns the two group workspaces (pool memory, kept for the next call).  Ordered after the
 * work already on `stream`; the work it enqueues is joined back into `stream` (no host sync). */
int sux_partition_maps_pipelined(sux_node* node, const sux_partitioner* part,
                                 const void* d_records, uint32_t record_size,
                                 uint64_t records_per_map, uint64_t num_records,
                                 uint64_t group_records, void* d_out, int64_t* d_index,
                                 uint8_t* d_index_be, void* stream);

/* Same as sux_partition_maps, but the output is laid out for the exchange: peer-major
 * [peer h][map m][partitions owned by h (floor(hR/W) .. floor((h+1)R/W))], so that every peer's
 * share of the whole group is ONE contiguous byte range and the all-to-all needs no repacking.
 * The index tables are still each map's logical data-file offsets (Spark's index file bytes).
 * d_peer_bytes (device, `world` u64) receives the bytes destined to each peer. */
int sux_partition_maps_peer_major(sux_node* node, const sux_partitioner* part,
                                  const void* d_records, uint32_t record_size,
                                  uint64_t records_per_map, uint64_t num_records, int32_t world,
                                  void* d_send, int64_t* d_index, uint8_t* d_index_be,
                                  uint64_t* d_peer_bytes, void* d_workspace,
                                  uint64_t workspace_bytes, void* stream);

/* Exchange plan of one peer-major group (host arithmetic, no device access; usable on CPU):
 * from the all-gathered index tables gathered[g][m][0..R] (world*num_maps*(R+1) int64) compute,
 * for `rank`, the per-peer byte counts/displacements of the all-to-all.  Received layout on rank h:
 * [source g][map m of g][partitions owned by h]. */
int sux_plan_group(int32_t world, int32_t rank, int32_t num_maps, int32_t num_partitions,
                   const int64_t* gathered_index, uint64_t* sendcounts, uint64_t* sdispls,
                   uint64_t* recvcounts, uint64_t* rdispls);
/* Byte offset, inside rank `rank`'s receive buffer, of block (source g, map m, partition p);
 * p must be owned by `rank`.  Returns -1 if not. */
int64_t sux_plan_block_offset(int32_t world, int32_t rank, int32_t num_maps,
                              int32_t num_partitions, const int64_t* gathered_index, int32_t g,
                              int32_t m, int32_t p);

/* Partition ownership (round 5).  Reduce partitions are owned in contiguous ranges: peer h owns
 * [owner_bounds[h], owner_bounds[h + 1]) (world + 1 rising int32 from 0 to R).  The default is
 * the equal split [h R / world, (h + 1) R / world); with skewed keys (Zipf: one partition can
 * hold ~12 % of a shuffle) an equal count of partitions per owner leaves one owner with far more
 * bytes than the others, and the exchange runs at that owner's ingress.  The reference fetches
 * per block (OnOffsetsFetchCallback.java:53-87), so any partition-aligned ownership is legal.
 * sux_plan_ownership: the contiguous split of R partitions of `partition_bytes` into `world`
 * non-empty ranges whose largest range holds the fewest bytes (exact: binary search on that
 * bound with a greedy fill).  Host arithmetic; usable on CPU. */
int sux_plan_ownership(int32_t world, int32_t num_partitions, const int64_t* partition_bytes,
                       int32_t* owner_bounds);
/* The node's ownership for the stateless group calls with `world` peers and R partitions —
 * sux_partition_maps_peer_major (the send layout), sux_exchange_group / _post / _issue (the
 * plan) and sux_pull_group — until set again; NULL owner_bounds restores the equal split.
 * Every rank must set the same table before its next group call (the plugin path's
 * sux_exchange_maps keeps the equal split). */
int sux_node_set_ownership(sux_node* node, int32_t world, int32_t num_partitions,
                           const int32_t* owner_bounds);
/* sux_plan_group / sux_plan_block_offset under an ownership table (NULL = the equal split). */
int sux_plan_group_owned(int32_t world, int32_t rank, int32_t num_maps, int32_t num_partitions,
                         const int64_t* gathered_index, const int32_t* owner_bounds,
                         uint64_t* sendcounts, uint64_t* sdispls, uint64_t* recvcounts,
                         uint64_t* rdispls);
int64_t sux_plan_block_offset_owned(int32_t world, int32_t rank, int32_t num_maps,
                                    int32_t num_partitions, const int64_t* gathered_index,
                                    const int32_t* owner_bounds, int32_t g, int32_t m, int32_t p);

/* One pipelined exchange step over the node's RCCL communicator: all-gather this rank's
 * num_maps index tables into d_gathered_index (device, world*num_maps*(R+1) int64), bring them
 * to the host (the only host sync), plan (sux_plan_group) and all-to-all d_send -> d_recv.
 * Every all-to-all of the library is grouped ncclSend/ncclRecv pieces of <= 256 MiB per peer:
 * the RCCL that torch ships (2.26.6) drops the second half of an ncclAllToAllv count past 1 GiB.
 * recv_bytes (host, world u64, nullable) receives the per-source byte counts. */
int sux_exchange_group(sux_node* node, const void* d_send, const int64_t* d_index,
                       int32_t num_maps, int32_t num_partitions, int64_t* d_gathered_index,
                       void* d_recv, uint64_t recv_capacity, uint64_t* recv_bytes, void* stream);
/* sux_exchange_group in two halves, so that the stream carrying the all-to-alls never waits on
 * the host between an all-gather and the all-to-all it plans.  _post enqueues
 * the all-gather of this launch group's index tables into d_gathered and their asynchronous
 * read-back into pinned staging on `stream` and returns a ticket; _issue (any thread) waits on
 * the host for that read-back, plans the counts (sux_plan_group) and enqueues the
 * partition-aligned all-to-all on ITS stream, over a second communicator split from the
 * node's (made by the first _post of every rank, a collective).  The bench posts group k right
 * after enqueueing its partition and then issues group k - 1: the all-gather of k overlaps the
 * all-to-all of k - 1 and the all-to-all stream is fed before its previous transfer drains.
 * _issue consumes the ticket (also on failure).  Every rank posts and issues the same groups in
 * the same order. */
typedef struct sux_xticket sux_xticket;
int sux_exchange_group_post(sux_node* node, const int64_t* d_index, int32_t num_maps,
                            int32_t num_partitions, int64_t* d_gathered, void* stream,
                            sux_xticket** out);
int sux_exchange_group_issue(sux_node* node, sux_xticket* ticket, const void* d_send,
                             void* d_recv, uint64_t recv_capacity, uint64_t* recv_bytes,
                             void* stream);
/* A posted ticket that will not be issued (another rank failed, teardown): waits for its
 * read-back and frees it.  Tickets never outlive their node: sux_node_destroy frees any left. */
int sux_exchange_group_discard(sux_node* node, sux_xticket* ticket);

/* ---- one-sided exchange over HIP IPC (xGMI peer access) ----------------------------------- *
 * The GET model of UcxShuffleClient (UcxShuffleClient.java:50-127, OnOffsetsFetchCallback.java
 * :80-87) with the peers' send buffers mapped into this process instead of registered with UCX
 * (ucp_mem_map/rkey, CommonUcxShuffleBlockResolver.scala:45-66): export a device buffer's IPC
 * descriptor (handle of its allocation + the buffer's offset in it, carried by any side channel
 * like the reference's address + rkey descriptor, :80-87), open the peers' descriptors, then
 * pull.  sux_pull_group reads, from every source g's peer-major send buffer, the
 * range holding this rank's partitions and writes it to d_recv at the sux_plan_group layout.
 * Offsets are computed on the device from the all-gathered index tables (d_gathered_index,
 * world*num_maps*(R+1) int64), so no host synchronisation is needed; the caller orders the pull
 * after every source's partition step (e.g. after the index all-gather completes).
 * d_recv_bytes (device u64, nullable) receives the bytes pulled; a capacity overflow pulls
 * nothing and stores UINT64_MAX there. */
#define SUX_IPC_DESC_BYTES 72 /* 64-byte hipIpcMemHandle of the allocation + u64 offset in it */
int sux_ipc_export(sux_node* node, const void* d_ptr, uint8_t out[SUX_IPC_DESC_BYTES]);
int sux_ipc_open(sux_node* node, const uint8_t desc[SUX_IPC_DESC_BYTES], void** d_ptr);
int sux_ipc_close(sux_node* node, void* d_ptr);
int sux_pull_group(sux_node* node, int32_t world, int32_t rank, const uint64_t* d_src_ptrs,
                   const int64_t* d_gathered_index, int32_t num_maps, int32_t num_partitions,
                   void* d_recv, uint64_t recv_capacity, uint64_t* d_recv_bytes, void* stream);

/* Partition ids only (P1), uint16 per record; used by tests and by the exchange planner. */
int sux_partition_ids(sux_node* node, const sux_partitioner* part, const void* d_records,
                      uint32_t record_size, uint64_t num_records, uint16_t* d_pids, void* stream);

/* ---- variable-length records: Spark SQL's UnsafeRowSerializer framing ----------------------
 * Replaces the same P1-P3 step as sux_partition_maps (the UnsafeShuffleWriter chosen at
 * compat/spark_3_0/UcxShuffleManager.scala:37-46 and the index write at
 * compat/spark_3_0/UcxShuffleBlockResolver.scala:35) for rows of differing size: Spark SQL's
 * UnsafeRowSerializer frames each row as a 4-byte big-endian length + the UnsafeRow, so a row is
 * 4 + 8k bytes.  Record i = d_data[d_offsets[i] - d_offsets[0], d_offsets[i+1] - d_offsets[0])
 * (num_records + 1 device u64 offsets, every one a multiple of 4, rows < 64 KiB).  The key the
 * partitioner reads lies at key_offset inside each row (e.g. 12: the frame length, the 8-byte null
 * bitset, then the first fixed-width field); rows must hold it.  d_pids_in (optional, device u16
 * per record, each < R) replaces the partitioner with ids the caller projected itself (Spark SQL
 * computes them from the partitioning expressions); then d_pids is not written.
 * Map m's data file occupies the same byte range of d_out as its rows occupy in d_data; its index
 * (R + 1 int64, native and optionally big-endian) holds byte offsets.  R <= 16384. */
int sux_partition_varlen_workspace_size(const sux_partitioner* part, uint64_t records_per_map,
                                        uint64_t num_records, uint64_t* bytes);
int sux_partition_varlen(sux_node* node, const sux_partitioner* part, const void* d_data,
                         const uint64_t* d_offsets, uint64_t records_per_map,
                         uint64_t num_records, const uint16_t* d_pids_in, void* d_out,
                         int64_t* d_index, uint8_t* d_index_be, uint16_t* d_pids,
                         void* d_workspace, uint64_t workspace_bytes, void* stream);

/* ---- compressed map outputs: spark.shuffle.compress=true, lz4 codec ------------------------
 * Replaces the per-partition compression stream Spark's writers open around each partition
 * segment ([ext] SerializerManager.wrapStream -> LZ4CompressionCodec.compressedOutputStream =
 * lz4-java LZ4BlockOutputStream(out, spark.io.compression.lz4.blockSize), inside the writer
 * chosen at compat/spark_3_0/UcxShuffleManager.scala:36-50).  Input: num_maps consecutive map
 * outputs in d_data (data_bytes in all) with their native index tables d_index
 * (num_maps * (R + 1) int64, as sux_partition_maps / sux_partition_varlen write them).  Output:
 * every non-empty (map, partition) run as its own LZ4Block stream (21-byte chunk headers with
 * XXH32 checksums, raw chunks where LZ4 does not shrink them, an end mark), maps consecutive in
 * d_out, their index tables (native + optional big-endian) and the total in *d_out_bytes
 * (device u64).  d_out must hold sux_compress_bound bytes.  block_size: multiple of 4 in
 * [64, 65536] (Spark's default 32768). */
int sux_compress_bound(uint64_t data_bytes, int32_t num_maps, int32_t num_partitions,
                       int32_t block_size, uint64_t* bytes);
int sux_compress_workspace_size(uint64_t data_bytes, int32_t num_maps, int32_t num_partitions,
                                int32_t block_size, uint64_t* bytes);
int sux_compress_map_outputs(sux_node* node, const void* d_data, uint64_t data_bytes,
                             const int64_t* d_index, int32_t num_maps, int32_t num_partitions,
                             int32_t block_size, void* d_out, uint64_t out_capacity,
                             int64_t* d_out_index, uint8_t* d_out_index_be,
                             uint64_t* d_out_bytes, void* d_workspace, uint64_t workspace_bytes,
                             void* stream);

/* ---- reading compressed blocks: the reducer's side of spark.shuffle.compress=true ----------
 * Replaces the decompression stream Spark's reader wraps around every fetched block ([ext]
 * BlockStoreShuffleReader -> SerializerManager.wrapStream -> LZ4CompressionCodec.
 * compressedInputStream = lz4-java LZ4BlockInputStream, stream concatenation on), for the blocks
 * one fetch delivered (compat/spark_3_0/UcxShuffleReader.scala:39-61 wraps them, sux_fetch_blocks): num_blocks
 * byte ranges of d_in (in_bytes in all), block k = [d_in_offsets[k], d_in_offsets[k + 1])
 * (num_blocks + 1 int64 on the device; an empty range is an empty block).  Each range is a
 * sequence of LZ4Block chunks and end marks checked as LZ4BlockInputStream checks them (magic,
 * method raw / LZ4, lengths against the block size the token declares and max_block_size, the
 * LZ4 block decoding to exactly its original length, the XXH32 & 0x0FFFFFFF checksum of the
 * decoded bytes) and decoded into d_out, blocks consecutive; d_out_offsets (num_blocks + 1 int64,
 * device) receives each block's decoded start and the total.  d_out == NULL: only d_out_offsets
 * (the decoded sizes; read the total, then call again with an output that holds it).  A malformed
 * block, or decoded bytes past out_capacity, sets the node's device error word (sux_node_check
 * reports it) and nothing is written outside d_out.  max_block_size: the largest chunk the blocks
 * may carry (spark.io.compression.lz4.blockSize, 64..65536); workspace: 256-byte aligned,
 * sux_decompress_workspace_size bytes.  Asynchronous on `stream`, no host wait. */
int sux_decompress_workspace_size(uint64_t in_bytes, int32_t num_blocks, int32_t max_block_size,
                                  uint64_t* bytes);
int sux_decompress_blocks(sux_node* node, const void* d_in, uint64_t in_bytes,
                          const int64_t* d_in_offsets, int32_t num_blocks, int32_t max_block_size,
                          void* d_out, uint64_t out_capacity, int64_t* d_out_offsets,
                          void* d_workspace, uint64_t workspace_bytes, void* stream);

/* ---- Spark's on-disk shuffle files (local-disk fallback / external shuffle service) ---------
 * sux_index_file_commit: IndexShuffleBlockResolver.writeIndexFileAndCommit [ext] (the super call
 * at compat/spark_3_0/UcxShuffleBlockResolver.scala:35), host-only: if index_path + data_path
 * already hold a consistent committed pair (index = R+1 BE offsets from 0, data length = their
 * sum) its lengths are returned (*reused = 1) and data_tmp is deleted; otherwise the index is
 * written to a temp file and both files are replaced by rename (data_tmp may be NULL).
 * sux_write_map_files: num_maps consecutive device map outputs + their native index tables ->
 * one data + index file pair per map (pinned double-buffered D2H, temp file, commit as above);
 * lengths_out (num_maps * R, optional) receives the committed lengths.
 * sux_read_file_blocks: the bytes of partitions [start, end) of one map's files
 * (IndexShuffleBlockResolver.getBlockData [ext] for a ShuffleBlockBatchId) into device memory. */
int sux_index_file_commit(const char* index_path, const char* data_path, const char* data_tmp,
                          const int64_t* lengths, int32_t num_partitions, int64_t* lengths_out,
                          int32_t* reused);
int sux_write_map_files(sux_node* node, const void* d_data, const int64_t* d_index,
                        int32_t num_maps, int32_t num_partitions, const char* const* data_paths,
                        const char* const* index_paths, int64_t* lengths_out, void* stream);
int sux_read_file_blocks(sux_node* node, const char* data_path, const char* index_path,
                         int32_t num_partitions, int32_t start_partition, int32_t end_partition,
                         void* d_dst, uint64_t capacity, uint64_t* bytes, void* stream);

/* ---- shuffle lifecycle: CommonUcxShuffleManager.registerShuffleCommon :39-56 ---------------- */
typedef struct sux_handle_desc {
  int32_t shuffle_id;
  int32_t num_maps;       /* directory slots: sized by MAP count (fixes quirk Q1, :27)          */
  int32_t num_partitions;
  int32_t record_size;
  uint64_t directory_bytes; /* num_maps * metadata_block_size                                  */
} sux_handle_desc;

int sux_register_shuffle(sux_node* node, int32_t shuffle_id, int32_t num_maps,
                         int32_t num_partitions, int32_t record_size, sux_handle_desc* out);
/* CommonUcxShuffleManager.unregisterShuffle :73-77 + CommonUcxShuffleBlockResolver.removeShuffle :116-121 */
int sux_unregister_shuffle(sux_node* node, int32_t shuffle_id);

/* getWriter(...).write(records) + UcxShuffleBlockResolver.writeIndexFileAndCommit
 * (compat/spark_3_0/UcxShuffleBlockResolver.scala:33-51 -> CommonUcxShuffleBlockResolver.scala:33-107):
 * partition one map batch held in device memory into a pooled device buffer owned by the node,
 * build its index, and publish the map's directory slot (the 300-byte driver descriptor analog).
 * An empty map output publishes nothing (UcxShuffleBlockResolver.scala:42-45). */
int sux_write_map_output(sux_node* node, int32_t shuffle_id, int32_t map_index,
                         const sux_partitioner* part, const void* d_records, uint64_t num_records,
                         void* stream);
/* The same for `num_records` records forming consecutive map tasks first_map_index,
 * first_map_index + 1, ... of `records_per_map` records each (the last may be shorter): one
 * launch group, no host wait.  Each map's index is published in its directory slot when the
 * node next makes progress after the kernels completed (any later call on the shuffle, or
 * sux_wait_map_outputs), the analog of the reference's completion callbacks running inside
 * worker.progress() on the calling thread (UcxWorkerWrapper.scala:100-120).  A map already
 * committed or being written is skipped (first commit wins); d_records must stay valid until
 * the stream reaches the work.  sux_write_map_output is this call for one map plus the wait
 * for it (CommonUcxShuffleBlockResolver.scala:101-103 blocks until the map is published). */
int sux_write_map_outputs(sux_node* node, int32_t shuffle_id, int32_t first_map_index,
                          const sux_partitioner* part, const void* d_records,
                          uint64_t records_per_map, uint64_t num_records, void* stream);
/* spark.shuffle.compress for the maps this node writes (sux_write_map_output(s) / _host):
 * SUX_CODEC_LZ4 = every non-empty (map, partition) run committed as its own lz4-java
 * LZ4BlockOutputStream stream of block_size-byte chunks (spark.io.compression.lz4.blockSize,
 * Spark's default 32768), byte-equal to what Spark's writers produce through
 * SerializerManager.wrapStream -> LZ4CompressionCodec.compressedOutputStream [ext] around each
 * partition segment (the writers chosen at compat/spark_3_0/UcxShuffleManager.scala:36-50); the
 * committed index file and the MapStatus lengths are then the compressed ones, and a reducer's
 * wrapStream decodes the fetched blocks exactly as it decodes Spark-written ones
 * (compat/spark_3_0/UcxShuffleReader.scala:61).  SUX_CODEC_NONE (the default) = raw data files
 * (spark.shuffle.compress=false).  Only before the shuffle's first map output (SUX_ESTATE after).
 * Map outputs committed by sux_commit_map_output / _adopt_ are taken as they are: Spark's own
 * writers already applied the codec. */
#define SUX_CODEC_NONE 0
#define SUX_CODEC_LZ4 1
int sux_shuffle_set_codec(sux_node* node, int32_t shuffle_id, int32_t codec, int32_t block_size);
/* Block until every map output enqueued for the shuffle (by any thread) is published. */
int sux_wait_map_outputs(sux_node* node, int32_t shuffle_id);
/* sux_write_map_output for records the JVM serialized into host memory (Spark's serializer
 * output): the bytes are staged into a pooled device buffer on `stream`, then partitioned as
 * above; blocks until the map is published. */
int sux_write_map_output_host(sux_node* node, int32_t shuffle_id, int32_t map_index,
                              const sux_partitioner* part, const void* host_records,
                              uint64_t num_records, void* stream);
/* writeIndexFileAndCommit for a map output produced elsewhere: `d_data` (data_bytes, device or
 * host memory — a data file Spark's own writer produced) is adopted by copy; `lengths` are R host
 * int64 partition lengths (Spark's lengths[]). */
int sux_commit_map_output(sux_node* node, int32_t shuffle_id, int32_t map_index,
                          const void* d_data, uint64_t data_bytes, const int64_t* lengths,
                          void* stream);
/* writeIndexFileAndCommit for map outputs a stateless call (sux_partition_maps*) already wrote
 * into the caller's device memory: maps first_map_index .. of records_per_map records each, map m
 * at d_out + m*records_per_map*record_size (the shuffle's record size), native index tables in
 * d_index (num_maps*(R+1) int64, device).  Nothing is copied: the node keeps BOTH pointers —
 * d_out and d_index must stay allocated and unchanged until sux_unregister_shuffle (at world 1
 * the index tables are read from d_index when blocks are resolved; at world > 1 they are also
 * read back on `stream` for the directory).  The maps are published like sux_write_map_outputs
 * (first commit wins).  The Spark analog is a writer whose output Spark did not copy. */
int sux_adopt_map_outputs(sux_node* node, int32_t shuffle_id, int32_t first_map_index,
                          const void* d_out, uint64_t records_per_map, uint64_t num_records,
                          const int64_t* d_index, void* stream);
/* Read back a committed map's index file bytes ((R+1)*8 big-endian, host buffer). */
int sux_map_output_index(sux_node* node, int32_t shuffle_id, int32_t map_index,
                         uint8_t* out_index_be, uint64_t out_len);

/* ---- exchange: the reduce-side fetch as a partition-aligned all-to-all -------- *
 * Collective over the node's group: every rank calls it after committing its map outputs.
 * Rank h receives partitions [floor(h*R/G), floor((h+1)*R/G)) of every map of every rank.
 * Replaces the driver-table GET (UcxWorkerWrapper.fetchDriverMetadataBuffer :176-196) by an
 * all-gather of the committed maps' directory entries, and the phase-1/phase-2 GETs
 * (UcxShuffleClient.java:50-127, OnOffsetsFetchCallback.java:44-92) by one partition-aligned
 * all-to-all per round of map batches over xGMI (RCCL communicator) or, with a bootstrap and
 * no communicator, by the same plan as one-sided pulls from the owners' IPC-mapped batch slabs.
 * The receive buffer is sized exactly from the gathered index tables.  sux_exchange is
 * sux_exchange_maps over every map + sux_exchange_wait: it returns when this rank's blocks are
 * in place and every rank has finished reading (so owners may unregister afterwards). */
int sux_exchange(sux_node* node, int32_t shuffle_id, void* stream);
/* The exchange of one window of map tasks, asynchronous: every rank calls it with the same
 * [first_map_index, first_map_index + num_maps) once the maps it writes there are enqueued.  It
 * waits only for this rank's writes of that window (later batches keep running), all-gathers
 * their directory entries, and enqueues on `stream` one partition-aligned all-to-all per round
 * of batches (round k = every rank's k-th batch of the window; counts/displacements straight from
 * the index tables; a batch's peer-major slab is the send buffer as it stands), or the same plan
 * as one-sided IPC pulls.  Maps already exchanged are skipped.  Returns without a host wait on
 * the data: fetches of the window's blocks on another stream are ordered after it by the node,
 * and sux_exchange_wait completes it.  Receive memory in flight = the window's owned bytes (the
 * reader's maxBytesInFlight, UcxShuffleReader.scala:56-70, chooses the window). */
int sux_exchange_maps(sux_node* node, int32_t shuffle_id, int32_t first_map_index,
                      int32_t num_maps, void* stream);
/* Collective: blocks until every exchange enqueued for the shuffle on this rank has completed
 * and (IPC transport) every rank has finished its pulls, so owners may unregister. */
int sux_exchange_wait(sux_node* node, int32_t shuffle_id);
/* The plan of one sux_exchange_maps call for rank `rank` (host arithmetic, no device; the call
 * runs exactly this on the gathered directory, so every rank's counts agree).  Input: the n
 * directory entries of the window, per entry its map, owner and batch, and per (entry, peer h)
 * seg = offset of the map's range for h in its batch slab and len = that range's bytes.
 * Pieces = the maps of one (owner, batch); round k = every owner's k-th piece, one all-to-all.
 * Output per round k (counts[k][0..3][h]): sendcounts, sdispls (offsets in this rank's batch
 * slab), recvcounts, rdispls (offsets in the round's part of the receive buffer) for peer h;
 * piece_entry[k][g] = the lowest-map entry of owner g's k-th piece (-1: none);
 * round_base[k] (rounds + 1) = where round k starts in the receive buffer (the last = total);
 * recv_off[i] = receive-buffer offset of entry i's owned range (UINT64_MAX: not received). */
typedef struct sux_xplan_entry {
  int32_t map, owner, batch, reserved;
} sux_xplan_entry;
int sux_plan_exchange(int32_t world, int32_t rank, int32_t loopback, int32_t n,
                      const sux_xplan_entry* entries, const uint64_t* seg, const uint64_t* len,
                      int32_t max_rounds, int32_t* rounds, uint64_t* counts, int32_t* piece_entry,
                      uint64_t* round_base, uint64_t* recv_off);
/* Reduce-partition ownership of a rank: [*start, *end). */
int sux_owned_partitions(sux_node* node, int32_t shuffle_id, int32_t rank, int32_t* start,
                         int32_t* end);

/* ---- fetch: UcxShuffleClient.fetchBlocks (reducer/compat/spark_3_0/UcxShuffleClient.java:94-127) */
typedef struct sux_block_id {
  int32_t map_index;    /* mapIdToBlockIndex(mapTaskId) (compat/spark_3_0/UcxShuffleReader.scala:42-50) */
  int32_t start_reduce; /* ShuffleBlockId.reduceId, or ShuffleBlockBatchId.startReduceId         */
  int32_t end_reduce;   /* start+1 for ShuffleBlockId, ShuffleBlockBatchId.endReduceId          */
  int32_t reserved;
} sux_block_id;

/* Fetch `n` blocks into one contiguous pooled device buffer, in request order (the layout of
 * OnOffsetsFetchCallback.java:75-87); sizes[i] = off[end]-off[start] (:53-72); block i starts at
 * sum(sizes[0..i)).  The buffer is refcounted: one reference per block, like the slices of
 * OnBlocksFetchCallback.java:33-57; sux_buffer_release() drops one, the last returns it to the
 * pool.  Blocks must be local to this rank (own maps at G=1, owned partitions after exchange).
 * Unlike the reference (which never calls onBlockFetchFailure), a missing block fails the call
 * with SUX_ENOENT and names it in sux_last_error(). */
int sux_fetch_blocks(sux_node* node, int32_t shuffle_id, const sux_block_id* blocks, int32_t n,
                     int64_t* sizes, sux_buffer** out, void* stream);
/* Zero-copy resolve: device address and size of each block (no copy; local blocks only).  No
 * reference is taken: the addresses stay valid until sux_unregister_shuffle of this shuffle —
 * from this call on, the node never spills the shuffle's map outputs (sux_node_set_spill_dir). */
int sux_resolve_blocks(sux_node* node, int32_t shuffle_id, const sux_block_id* blocks, int32_t n,
                       uint64_t* dev_addrs, int64_t* sizes);
int sux_buffer_info(sux_buffer* buf, void** dev_ptr, uint64_t* size, uint64_t* capacity);
/* A pooled device buffer of `bytes` with one reference (MemoryPool.get, MemoryPool.java:153-162):
 * the reducer's own scratch, e.g. the output and workspace of sux_sort_records over a fetched
 * buffer in the JVM reader, released with sux_buffer_release. */
int sux_buffer_alloc(sux_node* node, uint64_t bytes, sux_buffer** out);
/* Copy bytes [offset, offset + len) of a fetched buffer to host memory (the reducer's
 * deserialization side, NioManagedBuffer.nioByteBuffer); waits for the copy. */
int sux_buffer_read(sux_buffer* buf, uint64_t offset, void* host_dst, uint64_t len, void* stream);
int sux_buffer_retain(sux_buffer* buf, int32_t count);
int sux_buffer_release(sux_buffer* buf);
/* The reducer's decode of fetched LZ4Block streams (spark.shuffle.compress=true, lz4 codec) on
 * the device, for a consumer that needs the rows themselves on the GPU (the JVM reader's GPU key
 * sort, which replaces ExternalSorter at compat/spark_3_0/UcxShuffleReader.scala:138-154, after
 * the wrapStream of :61): num_blocks consecutive blocks of `in` starting at in_offset (host
 * block_sizes) are decoded as sux_decompress_blocks decodes them into a new pooled buffer (one
 * reference), blocks consecutive; out_sizes (optional, num_blocks) receives each block's decoded
 * size.  Waits for the decoded sizes and for the decode; a corrupted stream is SUX_EIO (Spark's
 * "Stream is corrupted"), and then no buffer is returned. */
int sux_buffer_decompress(sux_node* node, sux_buffer* in, uint64_t in_offset,
                          const int64_t* block_sizes, int32_t num_blocks, int32_t max_block_size,
                          sux_buffer** out, int64_t* out_sizes, void* stream);

/* ---- reduce side: sort by key ------------------------------------- *
 * After the fetch, Spark's reader sorts the partition's records when the dependency has a key
 * ordering (ExternalSorter, compat/spark_3_0/UcxShuffleReader.scala:138-154; TeraSort's reduce).
 * sux_sort_records is that sort on the GPU: `n` fixed-size records (record_size % 4 == 0) from
 * d_in are written to d_out (out of place) in ascending key order; records with equal keys keep
 * their input order, so sorting the canonical map-ordered concatenation of a partition's blocks
 * (sux_fetch_blocks) gives one deterministic answer where Spark's depends on fetch order (Q4).
 * Keys: SUX_SORT_BYTES = key_len (1..12) bytes compared unsigned lexicographically (TeraSort's
 * 10-byte keys); SUX_SORT_LONG / SUX_SORT_INT = signed little-endian int64 / int32 (Spark's
 * LongType / IntegerType orderings).  Workspace: sux_sort_workspace_size (about 32 B/record;
 * about 50 B/record up to 2048 x 4096 records, where the top digit is chunked).
 * The default path (tuning sort_msd 0 / 1 / 3) is planned on the device from the key span and
 * never waits on the host, so it can be captured into a HIP graph.  The LSD path (sort_msd 2,
 * sort_all_passes, or more than about 2^14 x 2048 records) waits on `stream` once, after the key pass,
 * to read back which key bits vary (24 bytes) and skips the digit passes over bits that never
 * vary; under graph capture it does not wait and runs every pass (same bytes).  The output is
 * complete when the stream's later work runs. */
#define SUX_SORT_BYTES 1
#define SUX_SORT_LONG 2
#define SUX_SORT_INT 3
int sux_sort_workspace_size(uint64_t n, uint32_t record_size, uint64_t* bytes);
int sux_sort_records(sux_node* node, int32_t key_kind, const void* d_in, uint64_t n,
                     uint32_t record_size, int32_t key_offset, int32_t key_len, void* d_out,
                     void* d_ws, uint64_t ws_bytes, void* stream);
/* Segmented: the records are num_segments consecutive runs (a reducer's partitions, e.g. the
 * canonical per-partition concatenations from sux_fetch_blocks), run k = records
 * [d_segment_offsets[k], d_segment_offsets[k+1]) (num_segments + 1 device int64, from 0 to n);
 * every run is sorted in place of itself, all in one call.  Key bytes + segment-id bytes (1 for
 * <= 256 segments, 2 for <= 65536, else 3) must fit 12.  Same workspace as sux_sort_records. */
int sux_sort_segments(sux_node* node, int32_t key_kind, const void* d_in, uint64_t n,
                      uint32_t record_size, int32_t key_offset, int32_t key_len,
                      const int64_t* d_segment_offsets, int32_t num_segments, void* d_out,
                      void* d_ws, uint64_t ws_bytes, void* stream);

/* ---- CU-partitioned streams (exchange/compute overlap) ---------------------------------- *
 * A non-blocking HIP stream (returned as void*) whose kernels run on `num_cus` of the device's
 * CUs, spread evenly over all 8 XCDs x 4 shader engines (use a multiple of 32: an SE with fewer
 * CUs than its peers becomes the straggler), or on the other CUs when `complement` is non-zero
 * (hipExtStreamCreateWithCUMask).  The map-side kernels fill every CU they are given (LDS-bound
 * occupancy), so a pipeline that overlaps the all-to-all of launch group k with the partition
 * of group k+1 runs the partition on a complement stream and leaves `num_cus` CUs to the
 * collective.  No reference counterpart: UCX moves bytes with the NIC, not with cores. */
int sux_stream_create(sux_node* node, int32_t num_cus, int32_t complement, void** out_stream);
int sux_stream_destroy(sux_node* node, void* stream);

/* ---- measurement hooks ------------------------------------------------------------------ */
/* When enabled, the node brackets each partition-kernel launch with HIP events on the launch
 * stream; sux_kernel_times() returns per-kernel {launches, total_ms} for kernels
 * 0=hist 1=scan 2=scatter 3=gather-copy (order fixed), and resets them. */
int sux_set_kernel_timing(sux_node* node, int enable);
int sux_kernel_times(sux_node* node, int64_t* launches, double* total_ms, int32_t nkernels);
/* Name of the kernel variant the node last launched for slot 0..3 (e.g. "k_scatter7"), so that a
 * measurement can be matched with the PMC profile of the kernel that actually ran; "" if none. */
int sux_kernel_variant(sux_node* node, int32_t slot, char* buf, size_t len);

/* ---- synthetic inputs (counter-based; identical bytes to oracle/oracle.c) --------------- */
#define SUX_GEN_TERASORT 1 /* 100-byte records: 10-byte key + row id + filler                  */
#define SUX_GEN_SMALL 2    /* 16-byte records: int64 uniform key + int64 value                  */
#define SUX_GEN_ZIPF 3     /* 100-byte records: int64 Zipf(s) key over `zipf_n` keys + filler   */
int sux_generate(sux_node* node, int32_t kind, uint64_t seed, uint64_t first_record,
                 uint64_t num_records, double zipf_s, uint64_t zipf_n, void* d_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SPARKUCX_AMD_H_ */
