/*
 * oracle.c — CPU restatement of SparkUCX's shuffle data path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load or run this file, and only as the checker or the reported CPU baseline.  The
 * product path (libsparkucx_amd.so) never links, loads or falls back to it.
 *
 * What it restates (file:line relative to /root/reference, [ext] = Apache Spark 3.0 semantics
 * the reference delegates to and which is not vendored — see SURVEY.md §8c):
 *   P1  partitioners            [ext] RangePartitioner.getPartition, HashPartitioner,
 *                               Spark SQL HashPartitioning = Pmod(Murmur3Hash(cols, 42), R);
 *                               writer chosen at compat/spark_3_0/UcxShuffleManager.scala:36-50
 *   P2  sort-shuffle write      [ext] SortShuffleWriter / UnsafeShuffleWriter: records grouped by
 *                               partition id 0..R-1, stable (input order) inside a partition
 *   P3  index file              [ext] IndexShuffleBlockResolver.writeIndexFileAndCommit, called at
 *                               compat/spark_3_0/UcxShuffleBlockResolver.scala:35; (R+1) BE int64,
 *                               size asserted at CommonUcxShuffleBlockResolver.scala:53
 *   P8-P10 fetch                reducer/compat/spark_3_0/UcxShuffleClient.java:50-127 (phase 1:
 *                               16-byte offset pairs, or (end-start) pairs for a batch block),
 *                               OnOffsetsFetchCallback.java:44-92 (size = off[end]-off[start],
 *                               blocks packed contiguously in request order), OnBlocksFetchCallback
 *                               .java:33-57 (one slice per block)
 *   §8e exchange ownership      rank h owns partitions [floor(hR/G), floor((h+1)R/G))
 *
 * Pinning.  The reference has no unit tests, fixtures or golden vectors and is
 * JVM-only (no JDK here), so it cannot be run.  The Murmur3 primitive is pinned by the known
 * answers of Spark's Murmur3_x86_32Suite (tests/test_oracle.py) and by an independent
 * implementation, scikit-learn's MurmurHash3_x86_32 (tests/test_oracle_pins.py, which also checks
 * the partitioners, the map write, the index bytes and the key sort against plain-Python/numpy
 * restatements that share no code with this file).  Everything else (partition
 * grouping, index bytes, fetch packing) is a restatement of the cited code and is therefore
 * "parity unpinned" against the reference itself; tests/golden/ freezes the restatement's
 * outputs so that later rounds cannot drift.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <errno.h>
#include <fcntl.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

/* ------------------------------------------------------------------------------------------ */
/* generators: counter-based, bit-identical to sparkucx_amd/csrc/sux_gen.hip                   */
/* ------------------------------------------------------------------------------------------ */
uint64_t o_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline void rec_words(uint64_t seed, uint64_t i, uint64_t* a, uint64_t* b) {
  *a = o_mix64((seed * 0x2545F4914F6CDD1Dull) ^ i);
  *b = o_mix64(*a ^ 0xA0761D6478BD642Full);
}

static inline void st32(uint8_t* p, uint32_t v) { memcpy(p, &v, 4); }

static void fill_tail100(uint8_t* r, uint64_t i, uint64_t b) {
  /* dword 2 = low 32 bits of b, dwords 3-4 = row id, dwords 5..24 = filler */
  st32(r + 8, (uint32_t)b);
  st32(r + 12, (uint32_t)i);
  st32(r + 16, (uint32_t)(i >> 32));
  uint32_t f = (uint32_t)(b >> 32);
  for (int k = 0; k < 20; ++k) st32(r + 20 + 4 * k, f + (uint32_t)k * 0x01010101u);
}

void o_gen_terasort(uint64_t seed, uint64_t first, uint64_t n, uint8_t* out) {
  for (uint64_t j = 0; j < n; ++j) {
    uint64_t i = first + j, a, b;
    rec_words(seed, i, &a, &b);
    uint8_t* r = out + j * 100;
    st32(r, (uint32_t)a);
    st32(r + 4, (uint32_t)(a >> 32));
    fill_tail100(r, i, b);
  }
}

void o_gen_small(uint64_t seed, uint64_t first, uint64_t n, uint8_t* out) {
  for (uint64_t j = 0; j < n; ++j) {
    uint64_t i = first + j, a, b;
    rec_words(seed, i, &a, &b);
    uint8_t* r = out + j * 16;
    st32(r, (uint32_t)a);
    st32(r + 4, (uint32_t)(a >> 32));
    st32(r + 8, (uint32_t)i);
    st32(r + 12, (uint32_t)(i >> 32));
  }
}

/* Zipf(s) over keys 1..n as a bucketed inverse CDF: keys 1..256 exactly, then 1024 geometric
 * buckets sampled uniformly inside.  The table is plain double arithmetic (no FMA contraction);
 * sampling is integer-only so CPU and GPU draw the same keys from the same table. */
#define ZIPF_EXACT 256
#define ZIPF_GEO 1024
static int zipf_bounds(uint64_t n, uint64_t* bounds) {
  int nb = 0;
  uint64_t e = n < ZIPF_EXACT ? n : ZIPF_EXACT;
  for (uint64_t k = 1; k <= e; ++k) {
    if (bounds) bounds[nb] = k;
    nb++;
  }
  uint64_t prev = e + 1;
  if (n > e) {
    double base = (double)(e + 1), ratio = (double)(n + 1) / base;
    for (int j = 1; j <= ZIPF_GEO; ++j) {
      uint64_t b = (j == ZIPF_GEO) ? n + 1 : (uint64_t)llround(base * pow(ratio, (double)j / ZIPF_GEO));
      if (b <= prev) continue;
      if (b > n + 1) b = n + 1;
      if (bounds) bounds[nb] = prev;
      nb++;
      prev = b;
      if (b == n + 1) break;
    }
  }
  if (bounds) bounds[nb] = prev; /* == n + 1 */
  return nb;
}

int o_zipf_table_size(uint64_t zipf_n) { return zipf_bounds(zipf_n, NULL); }

static double zipf_mass(uint64_t lo, uint64_t hi, double s) { /* sum_{k=lo}^{hi-1} k^-s */
  if (hi - lo <= 4) {
    double m = 0;
    for (uint64_t k = lo; k < hi; ++k) m += pow((double)k, -s);
    return m;
  }
  double a = (double)lo - 0.5, b = (double)hi - 0.5;
  if (fabs(s - 1.0) < 1e-12) return log(b) - log(a);
  return (pow(a, 1.0 - s) - pow(b, 1.0 - s)) / (s - 1.0);
}

void o_zipf_table(double s, uint64_t zipf_n, uint64_t* bounds, uint64_t* thresh) {
  int nb = zipf_bounds(zipf_n, bounds);
  double* w = (double*)malloc(sizeof(double) * (size_t)nb);
  double total = 0;
  for (int j = 0; j < nb; ++j) {
    w[j] = zipf_mass(bounds[j], bounds[j + 1], s);
    total += w[j];
  }
  double cum = 0;
  for (int j = 0; j < nb; ++j) {
    double f = ldexp(cum / total, 64);
    thresh[j] = (j == 0) ? 0 : (f >= 18446744073709551615.0 ? UINT64_MAX : (uint64_t)f);
    cum += w[j];
  }
  thresh[nb] = UINT64_MAX;
  free(w);
}

static inline uint64_t mulhi64(uint64_t a, uint64_t b) {
  return (uint64_t)(((__uint128_t)a * (__uint128_t)b) >> 64);
}

static uint64_t zipf_draw(const uint64_t* bounds, const uint64_t* thresh, int nb, uint64_t u1,
                          uint64_t u2) {
  int lo = 0, hi = nb - 1; /* largest j with thresh[j] <= u1 */
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (thresh[mid] <= u1) lo = mid; else hi = mid - 1;
  }
  return bounds[lo] + mulhi64(u2, bounds[lo + 1] - bounds[lo]);
}

void o_gen_zipf(uint64_t seed, uint64_t first, uint64_t n, double s, uint64_t zipf_n,
                uint8_t* out) {
  int nb = o_zipf_table_size(zipf_n);
  uint64_t* bounds = (uint64_t*)malloc(8 * (size_t)(nb + 1));
  uint64_t* thresh = (uint64_t*)malloc(8 * (size_t)(nb + 1));
  o_zipf_table(s, zipf_n, bounds, thresh);
  for (uint64_t j = 0; j < n; ++j) {
    uint64_t i = first + j, a, b;
    rec_words(seed, i, &a, &b);
    uint64_t key = zipf_draw(bounds, thresh, nb, a, b);
    uint8_t* r = out + j * 100;
    st32(r, (uint32_t)key);
    st32(r + 4, (uint32_t)(key >> 32));
    fill_tail100(r, i, b);
  }
  free(bounds);
  free(thresh);
}

/* ------------------------------------------------------------------------------------------ */
/* Spark Murmur3_x86_32 [ext] (org.apache.spark.unsafe.hash.Murmur3_x86_32)                   */
/* ------------------------------------------------------------------------------------------ */
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t mix_k1(uint32_t k1) {
  k1 *= 0xcc9e2d51u;
  k1 = rotl32(k1, 15);
  return k1 * 0x1b873593u;
}
static inline uint32_t mix_h1(uint32_t h1, uint32_t k1) {
  h1 ^= k1;
  h1 = rotl32(h1, 13);
  return h1 * 5u + 0xe6546b64u;
}
static inline uint32_t fmix32(uint32_t h1, uint32_t len) {
  h1 ^= len;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  return h1 ^ (h1 >> 16);
}

int32_t o_murmur3_hash_int(int32_t v, int32_t seed) {
  return (int32_t)fmix32(mix_h1((uint32_t)seed, mix_k1((uint32_t)v)), 4);
}

int32_t o_murmur3_hash_long(int64_t v, int32_t seed) {
  uint64_t u = (uint64_t)v;
  uint32_t h1 = mix_h1((uint32_t)seed, mix_k1((uint32_t)u));
  h1 = mix_h1(h1, mix_k1((uint32_t)(u >> 32)));
  return (int32_t)fmix32(h1, 8);
}

/* Legacy hashUnsafeBytes: 4-byte little-endian words, then EACH tail byte, sign-extended, as
 * its own mixing round (not standard murmur3 tail handling), fmix with the byte length. */
int32_t o_murmur3_hash_unsafe_bytes(const uint8_t* p, int32_t len, int32_t seed) {
  int32_t aligned = len - len % 4;
  uint32_t h1 = (uint32_t)seed;
  for (int32_t i = 0; i < aligned; i += 4) {
    uint32_t w;
    memcpy(&w, p + i, 4);
    h1 = mix_h1(h1, mix_k1(w));
  }
  for (int32_t i = aligned; i < len; ++i) {
    int32_t half = (int32_t)(int8_t)p[i];
    h1 = mix_h1(h1, mix_k1((uint32_t)half));
  }
  return (int32_t)fmix32(h1, (uint32_t)len);
}

int32_t o_pmod(int32_t a, int32_t n) { /* Spark SQL Pmod for ints */
  int32_t r = a % n;
  return r < 0 ? (r + n) % n : r;
}

int32_t o_non_negative_mod(int32_t a, int32_t n) { /* Utils.nonNegativeMod */
  int32_t r = a % n;
  return r + (r < 0 ? n : 0);
}

/* ------------------------------------------------------------------------------------------ */
/* partitioners                                                                               */
/* ------------------------------------------------------------------------------------------ */
void o_range_bounds_uniform(int32_t R, int32_t key_len, uint8_t* out) {
  /* bound i = floor((i+1) * 2^64 / R) as the big-endian first min(8,key_len) bytes, rest 0 */
  for (int32_t i = 0; i + 1 < R; ++i) {
    uint64_t v = (uint64_t)((((__uint128_t)(uint64_t)(i + 1)) << 64) / (uint64_t)R);
    uint8_t* b = out + (size_t)i * key_len;
    memset(b, 0, (size_t)key_len);
    for (int k = 0; k < 8 && k < key_len; ++k) b[k] = (uint8_t)(v >> (56 - 8 * k));
  }
}

static inline int64_t ld64(const uint8_t* p) { int64_t v; memcpy(&v, p, 8); return v; }
static inline int32_t ld32(const uint8_t* p) { int32_t v; memcpy(&v, p, 4); return v; }

int32_t o_get_partition(const o_part* p, const uint8_t* rec) {
  const uint8_t* key = rec + p->key_offset;
  int32_t R = p->num_partitions;
  switch (p->kind) {
    case 1: { /* RANGE: count bounds strictly below the key (linear form of getPartition) */
      int32_t part = 0;
      while (part < R - 1 &&
             memcmp(key, p->range_bounds + (size_t)part * p->key_len, (size_t)p->key_len) > 0)
        part++;
      return p->ascending ? part : (R - 1) - part;
    }
    case 2: return o_pmod(o_murmur3_hash_long(ld64(key), p->seed), R);
    case 3: return o_pmod(o_murmur3_hash_int(ld32(key), p->seed), R);
    case 4: return o_pmod(o_murmur3_hash_unsafe_bytes(key, p->key_len, p->seed), R);
    case 5: {
      uint64_t v = (uint64_t)ld64(key);
      return o_non_negative_mod((int32_t)(uint32_t)(v ^ (v >> 32)), R);
    }
    case 6: return o_non_negative_mod(ld32(key), R);
  }
  return -1;
}

void o_partition_ids(const o_part* p, const uint8_t* recs, uint64_t n, uint32_t rec_size,
                     uint16_t* pids) {
  for (uint64_t i = 0; i < n; ++i) pids[i] = (uint16_t)o_get_partition(p, recs + i * rec_size);
}

/* ------------------------------------------------------------------------------------------ */
/* map write: P2 + P3                                                                          */
/* ------------------------------------------------------------------------------------------ */
static void store_be64(uint8_t* p, int64_t v) {
  for (int k = 0; k < 8; ++k) p[k] = (uint8_t)((uint64_t)v >> (56 - 8 * k));
}
static int64_t load_be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int k = 0; k < 8; ++k) v = (v << 8) | p[k];
  return (int64_t)v;
}

void o_index_from_lengths(const int64_t* lengths, int32_t R, int64_t* index, uint8_t* index_be) {
  int64_t off = 0;
  for (int32_t r = 0; r <= R; ++r) {
    if (index) index[r] = off;
    if (index_be) store_be64(index_be + 8 * r, off);
    if (r < R) off += lengths[r];
  }
}

void o_write_map(const o_part* p, const uint8_t* recs, uint64_t n, uint32_t rec_size,
                 uint8_t* out, int64_t* lengths, int64_t* index, uint8_t* index_be) {
  int32_t R = p->num_partitions;
  uint16_t* pids = (uint16_t*)malloc(sizeof(uint16_t) * (n ? n : 1));
  uint64_t* cur = (uint64_t*)calloc((size_t)R, sizeof(uint64_t));
  o_partition_ids(p, recs, n, rec_size, pids);
  for (uint64_t i = 0; i < n; ++i) cur[pids[i]]++;
  uint64_t acc = 0;
  for (int32_t r = 0; r < R; ++r) {
    lengths[r] = (int64_t)(cur[r] * rec_size);
    uint64_t c = cur[r];
    cur[r] = acc;
    acc += c;
  }
  for (uint64_t i = 0; i < n; ++i)
    memcpy(out + (cur[pids[i]]++) * rec_size, recs + i * rec_size, rec_size);
  o_index_from_lengths(lengths, R, index, index_be);
  free(cur);
  free(pids);
}

/* ------------------------------------------------------------------------------------------ */
/* fetch: P8-P10                                                                               */
/* ------------------------------------------------------------------------------------------ */
int64_t o_fetch_blocks(const uint8_t* const* map_data, const uint8_t* const* map_index_be,
                       int32_t num_maps, int32_t R, const int32_t* blocks, int32_t n,
                       int64_t* sizes, uint8_t* dst) {
  int64_t pos = 0;
  for (int32_t i = 0; i < n; ++i) {
    int32_t m = blocks[3 * i], s = blocks[3 * i + 1], e = blocks[3 * i + 2];
    if (m < 0 || m >= num_maps || s < 0 || e <= s || e > R) return -1;
    /* phase 1: offset pair(s) from the map's index file; a batch block reads end-start+1 longs
     * (the reference reads 2*(end-start), quirk Q2 — only the first and last matter) */
    int64_t start = load_be64(map_index_be[m] + 8 * (size_t)s);
    int64_t end = load_be64(map_index_be[m] + 8 * (size_t)e);
    sizes[i] = end - start;
    /* phase 2: block bytes into the contiguous destination at a running offset */
    if (dst && sizes[i] > 0) memcpy(dst + pos, map_data[m] + start, (size_t)sizes[i]);
    pos += sizes[i];
  }
  return pos;
}

int32_t o_owner_start(int32_t h, int32_t R, int32_t G) {
  return (int32_t)(((int64_t)h * R) / G);
}

uint64_t o_checksum(const uint8_t* p, uint64_t n) {
  uint64_t h = 0, i = 0;
  for (; i + 8 <= n; i += 8) h += o_mix64((uint64_t)ld64(p + i) ^ (i >> 3));
  uint64_t t = 0;
  for (uint64_t k = 0; i + k < n; ++k) t |= (uint64_t)p[i + k] << (8 * k);
  if (i < n) h += o_mix64(t ^ (i >> 3) ^ 0xFFull << 56);
  return h;
}

/* ------------------------------------------------------------------------------------------ */
/* CPU baseline: Spark sort-shuffle write to files + UCX-style two-phase fetch   */
/* ------------------------------------------------------------------------------------------ */
typedef struct cpu_ctx {
  const o_part* p;
  const uint8_t* recs;
  uint64_t n, per_map;
  uint32_t rec_size;
  int32_t num_maps, R;
  const char* dir;
  int next; /* work counter */
  pthread_mutex_t mu;
  uint8_t** data_map;  /* mmapped data files */
  uint8_t** index_map; /* mmapped index files */
  uint64_t* data_len;
  uint64_t checksum, fetched;
  int err;
} cpu_ctx;

static int take(cpu_ctx* c, int limit) {
  pthread_mutex_lock(&c->mu);
  int v = c->next < limit ? c->next++ : -1;
  pthread_mutex_unlock(&c->mu);
  return v;
}

static int write_all(int fd, const uint8_t* p, uint64_t n) {
  while (n) {
    ssize_t w = write(fd, p, n > (1u << 30) ? (1u << 30) : n);
    if (w <= 0) return -1;
    p += w;
    n -= (uint64_t)w;
  }
  return 0;
}

static void* map_worker(void* arg) {
  cpu_ctx* c = (cpu_ctx*)arg;
  int32_t R = c->R;
  uint8_t* out = (uint8_t*)malloc(c->per_map * c->rec_size + 1);
  int64_t* lengths = (int64_t*)malloc(sizeof(int64_t) * (size_t)R);
  uint8_t* index_be = (uint8_t*)malloc(8 * (size_t)(R + 1));
  char path[4096];
  for (int m; (m = take(c, c->num_maps)) >= 0;) {
    uint64_t first = (uint64_t)m * c->per_map;
    uint64_t cnt = first >= c->n ? 0 : (c->n - first < c->per_map ? c->n - first : c->per_map);
    o_write_map(c->p, c->recs + first * c->rec_size, cnt, c->rec_size, out, lengths, NULL,
                index_be);
    snprintf(path, sizeof path, "%s/shuffle_0_%d_0.data", c->dir, m);
    int fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0600);
    if (fd < 0 || write_all(fd, out, cnt * c->rec_size)) c->err = 1;
    if (fd >= 0) close(fd);
    snprintf(path, sizeof path, "%s/shuffle_0_%d_0.index", c->dir, m);
    fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0600);
    if (fd < 0 || write_all(fd, index_be, 8 * (uint64_t)(R + 1))) c->err = 1;
    if (fd >= 0) close(fd);
  }
  free(out);
  free(lengths);
  free(index_be);
  return NULL;
}

static void* fetch_worker(void* arg) {
  cpu_ctx* c = (cpu_ctx*)arg;
  int32_t R = c->R;
  uint64_t cap = 0;
  uint8_t* buf = NULL;
  uint64_t sum = 0, bytes = 0;
  for (int r; (r = take(c, R)) >= 0;) {
    /* phase 1: 16-byte offset pair of block (m, r) from every map's index file */
    uint64_t total = 0;
    for (int m = 0; m < c->num_maps; ++m)
      total += (uint64_t)(load_be64(c->index_map[m] + 8 * (size_t)(r + 1)) -
                          load_be64(c->index_map[m] + 8 * (size_t)r));
    if (total > cap) {
      free(buf);
      cap = total;
      buf = (uint8_t*)malloc(cap);
    }
    /* phase 2: block bytes into one contiguous buffer in request order */
    uint64_t pos = 0;
    for (int m = 0; m < c->num_maps; ++m) {
      int64_t s = load_be64(c->index_map[m] + 8 * (size_t)r);
      int64_t e = load_be64(c->index_map[m] + 8 * (size_t)(r + 1));
      if (e > s) memcpy(buf + pos, c->data_map[m] + s, (size_t)(e - s));
      pos += (uint64_t)(e - s);
    }
    sum += o_checksum(buf, pos);
    bytes += pos;
  }
  free(buf);
  pthread_mutex_lock(&c->mu);
  c->checksum += sum;
  c->fetched += bytes;
  pthread_mutex_unlock(&c->mu);
  return NULL;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void* map_file(const char* path, uint64_t* len) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return NULL;
  struct stat st;
  fstat(fd, &st);
  *len = (uint64_t)st.st_size;
  void* p = *len ? mmap(NULL, *len, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0) : NULL;
  close(fd);
  return p == MAP_FAILED ? NULL : p;
}

int o_cpu_shuffle(const o_part* p, const uint8_t* recs, uint64_t n, uint32_t rec_size,
                  int32_t num_maps, int32_t threads, const char* dir, o_cpu_result* res,
                  int64_t* index_out) {
  cpu_ctx c;
  memset(&c, 0, sizeof c);
  c.p = p;
  c.recs = recs;
  c.n = n;
  c.rec_size = rec_size;
  c.num_maps = num_maps;
  c.R = p->num_partitions;
  c.per_map = (n + (uint64_t)num_maps - 1) / (uint64_t)num_maps;
  c.dir = dir;
  pthread_mutex_init(&c.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);

  double t0 = now_s();
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, map_worker, &c);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  double t1 = now_s();

  /* register (mmap) every committed map output, like CommonUcxShuffleBlockResolver :45-58 */
  c.data_map = (uint8_t**)calloc((size_t)num_maps, sizeof(void*));
  c.index_map = (uint8_t**)calloc((size_t)num_maps, sizeof(void*));
  c.data_len = (uint64_t*)calloc((size_t)num_maps, sizeof(uint64_t));
  char path[4096];
  uint64_t ilen;
  for (int m = 0; m < num_maps && !c.err; ++m) {
    snprintf(path, sizeof path, "%s/shuffle_0_%d_0.data", dir, m);
    c.data_map[m] = (uint8_t*)map_file(path, &c.data_len[m]);
    snprintf(path, sizeof path, "%s/shuffle_0_%d_0.index", dir, m);
    c.index_map[m] = (uint8_t*)map_file(path, &ilen);
    if (!c.index_map[m] || ilen != 8 * (uint64_t)(c.R + 1)) c.err = 1;
  }
  c.next = 0;
  if (!c.err) {
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, fetch_worker, &c);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  }
  double t2 = now_s();
  /* (untimed) the committed index files, native order, for a parity check against the GPU */
  if (index_out && !c.err)
    for (int m = 0; m < num_maps; ++m)
      for (int r = 0; r <= c.R; ++r)
        index_out[(size_t)m * (c.R + 1) + r] = load_be64(c.index_map[m] + 8 * (size_t)r);
  for (int m = 0; m < num_maps; ++m) {
    if (c.data_map[m]) munmap(c.data_map[m], c.data_len[m]);
    if (c.index_map[m]) munmap(c.index_map[m], 8 * (uint64_t)(c.R + 1));
    snprintf(path, sizeof path, "%s/shuffle_0_%d_0.data", dir, m);
    unlink(path);
    snprintf(path, sizeof path, "%s/shuffle_0_%d_0.index", dir, m);
    unlink(path);
  }
  free(c.data_map);
  free(c.index_map);
  free(c.data_len);
  free(th);
  pthread_mutex_destroy(&c.mu);
  res->map_s = t1 - t0;
  res->fetch_s = t2 - t1;
  res->total_s = t2 - t0;
  res->bytes_in = n * rec_size;
  res->bytes_fetched = c.fetched;
  res->checksum = c.checksum;
  return c.err ? -1 : 0;
}
