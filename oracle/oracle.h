/*
 * oracle.h — CPU restatement of the SparkUCX shuffle data path (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code, and
 * only as the checker / the timed CPU baseline — never as a product path.  See oracle.c.
 */
#ifndef SUX_ORACLE_H_
#define SUX_ORACLE_H_
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* generators (bit-identical to sparkucx_amd/csrc/sux_gen.hip) */
uint64_t o_mix64(uint64_t z);
void o_gen_terasort(uint64_t seed, uint64_t first, uint64_t n, uint8_t* out);
void o_gen_small(uint64_t seed, uint64_t first, uint64_t n, uint8_t* out);
/* Zipf table: nb buckets, bounds[nb+1] (key ranges), thresh[nb+1] (u64 CDF thresholds). */
int o_zipf_table_size(uint64_t zipf_n);
void o_zipf_table(double s, uint64_t zipf_n, uint64_t* bounds, uint64_t* thresh);
void o_gen_zipf(uint64_t seed, uint64_t first, uint64_t n, double s, uint64_t zipf_n, uint8_t* out);

/* Spark hashing primitives */
int32_t o_murmur3_hash_int(int32_t v, int32_t seed);
int32_t o_murmur3_hash_long(int64_t v, int32_t seed);
int32_t o_murmur3_hash_unsafe_bytes(const uint8_t* p, int32_t len, int32_t seed);
int32_t o_pmod(int32_t a, int32_t n);
int32_t o_non_negative_mod(int32_t a, int32_t n);

/* partitioner (same field meaning as sux_partitioner_desc in include/sparkucx_amd.h) */
typedef struct o_part {
  int32_t kind, num_partitions, key_offset, key_len, seed, ascending;
  const uint8_t* range_bounds;
} o_part;
void o_range_bounds_uniform(int32_t R, int32_t key_len, uint8_t* out);
int32_t o_get_partition(const o_part* p, const uint8_t* record);
void o_partition_ids(const o_part* p, const uint8_t* recs, uint64_t n, uint32_t rec_size,
                     uint16_t* pids);

/* Spark sort-shuffle write of ONE map batch: stable group-by-pid; lengths[R]; index (R+1) i64
 * native + big-endian bytes. */
void o_write_map(const o_part* p, const uint8_t* recs, uint64_t n, uint32_t rec_size,
                 uint8_t* out, int64_t* lengths, int64_t* index, uint8_t* index_be);
void o_index_from_lengths(const int64_t* lengths, int32_t R, int64_t* index, uint8_t* index_be);

/* UcxShuffleClient.fetchBlocks + OnOffsetsFetchCallback: n blocks {map,start,end}; index_be of
 * every map ((R+1)*8 bytes each, map-major), data base pointers per map.  Writes sizes[n] and the
 * contiguous destination; returns total bytes, or -1 on an invalid block. */
int64_t o_fetch_blocks(const uint8_t* const* map_data, const uint8_t* const* map_index_be,
                       int32_t num_maps, int32_t R, const int32_t* blocks /* n*3 */, int32_t n,
                       int64_t* sizes, uint8_t* dst);

/* Exchange restatement: rank h owns [floor(h*R/G), floor((h+1)*R/G)). */
int32_t o_owner_start(int32_t h, int32_t R, int32_t G);

/* CPU baseline: Spark-style map write to files + UCX-style two-phase fetch. */
typedef struct o_cpu_result {
  double map_s, fetch_s, total_s;
  uint64_t bytes_in, bytes_fetched;
  uint64_t checksum;
} o_cpu_result;
int o_cpu_shuffle(const o_part* p, const uint8_t* recs, uint64_t n, uint32_t rec_size,
                  int32_t num_maps, int32_t threads, const char* dir, o_cpu_result* res,
                  int64_t* index_out /* nullable: num_maps * (R+1) */);

/* order-independent checksum helpers */
uint64_t o_checksum(const uint8_t* p, uint64_t n);

/* compressed map outputs (lz4.c) */
uint32_t o_xxh32(const uint8_t* p, uint64_t len, uint32_t seed);
int32_t o_lz4_compress_default(const uint8_t* src, int32_t len, uint8_t* dst);
int32_t o_lz4_compress_block(const uint8_t* src, int32_t len, uint8_t* dst);
int32_t o_lz4_decompress_block(const uint8_t* src, int32_t slen, uint8_t* dst, int32_t cap);
uint64_t o_lz4_stream(const uint8_t* src, uint64_t n, uint32_t bs, uint8_t* dst);
uint64_t o_lz4_map_outputs(const uint8_t* data, const int64_t* index, int32_t maps, int32_t R,
                           uint32_t bs, uint8_t* out, int64_t* out_index);
int64_t o_lz4_unframe(const uint8_t* s, uint64_t n, uint8_t* dst, uint64_t cap);

#ifdef __cplusplus
}
#endif

#endif
