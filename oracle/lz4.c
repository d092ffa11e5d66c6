/*
 * lz4.c — CPU restatement of compressed map outputs.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.c's header): the checker of sux_compress_map_outputs.
 *
 * What it restates ([ext] = not vendored under /root/reference):
 *   - Spark 3.0 spark.shuffle.compress=true with the default codec: each partition segment of a
 *     map output is written through its own LZ4CompressionCodec.compressedOutputStream =
 *     lz4-java 1.7.1 LZ4BlockOutputStream(out, spark.io.compression.lz4.blockSize) [ext];
 *     streams open lazily, so an empty segment is zero bytes.
 *   - LZ4BlockOutputStream framing [ext]: per chunk of <= blockSize bytes a 21-byte header
 *     "LZ4Block" | method|level | compressed len LE32 | original len LE32 | checksum LE32, then
 *     the payload; method 0x20 = LZ4 block, 0x10 = raw (used when compression does not shrink the
 *     chunk); level = max(0, ceil(log2(blockSize)) - 10); checksum = XXH32(original, seed
 *     0x9747b28c) & 0x0FFFFFFF (StreamingXXHash32.asChecksum); close() appends an end mark
 *     (method 0x10|level, lengths and checksum 0).
 *   - XXH32 [ext: xxHash spec]; pinned by the python xxhash module (tests/test_oracle_lz4.py).
 *   - The LZ4 block format [ext: lz4 block format spec]: sequences of token, literal-length
 *     extension, literals, LE16 offset, match-length extension; min match 4; the last 5 bytes
 *     are literals; the last match starts >= 12 bytes before the end.  The decoder below is
 *     cross-checked against the system liblz4 (LZ4_decompress_safe / LZ4_compress_default) in
 *     tests/test_oracle_lz4.py.
 *   - o_lz4_compress_default restates liblz4's LZ4_compress_default (the compressor lz4-java's
 *     JNI instance calls for every chunk), so a GPU stream is compared byte for byte with what
 *     Spark's writer emits; tests/test_oracle_lz4.py pins the restatement to the system
 *     liblz4.so.1.9.3 on every input it tries.
 */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

#define XP1 2654435761u
#define XP2 2246822519u
#define XP3 3266489917u
#define XP4 668265263u
#define XP5 374761393u

static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
static void wr32(uint8_t* p, uint32_t v) { memcpy(p, &v, 4); }

uint32_t o_xxh32(const uint8_t* p, uint64_t len, uint32_t seed) {
  const uint8_t* e = p + len;
  uint32_t h;
  if (len >= 16) {
    uint32_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    const uint8_t* lim = e - 16;
    do {
      v1 = rotl32(v1 + rd32(p) * XP2, 13) * XP1;
      v2 = rotl32(v2 + rd32(p + 4) * XP2, 13) * XP1;
      v3 = rotl32(v3 + rd32(p + 8) * XP2, 13) * XP1;
      v4 = rotl32(v4 + rd32(p + 12) * XP2, 13) * XP1;
      p += 16;
    } while (p <= lim);
    h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
  } else {
    h = seed + XP5;
  }
  h += (uint32_t)len;
  for (; p + 4 <= e; p += 4) h = rotl32(h + rd32(p) * XP3, 17) * XP4;
  for (; p < e; ++p) h = rotl32(h + (uint32_t)(*p) * XP5, 11) * XP1;
  h ^= h >> 15;
  h *= XP2;
  h ^= h >> 13;
  h *= XP3;
  h ^= h >> 16;
  return h;
}

/* LZ4_compress_default of liblz4 1.9.3 [ext, not vendored; the system liblz4.so.1.9.3 is the
 * pin, tests/test_oracle_lz4.py], as lz4-java's JNI compressor calls it for every chunk of an
 * LZ4BlockOutputStream (maxDestLen = LZ4_compressBound, so the output is never limited):
 * LZ4_compress_fast(acceleration 1) -> LZ4_compress_fast_extState on a freshly zeroed state ->
 * LZ4_compress_generic(byU16 table for inputs below LZ4_64Klimit, noDict, noDictIssue).
 *   - hash = (read32(p) * 2654435761) >> (32 - 13), 8192 u16 entries holding positions; an entry
 *     never written reads 0 — position 0 — and is a real candidate;
 *   - inputs below LZ4_minLength (13) are one literal run;
 *   - position 0 goes into the table, the search starts at 1; the search visits forwardIp with
 *     step 1 for 64 probes, then 2, 3, ... (step = searchMatchNb++ >> 6, searchMatchNb from 64);
 *     a probe is abandoned — last literals — when the NEXT forwardIp passes len - 11
 *     (mflimitPlusOne), before the probe's own insertion; every other probe is inserted, then
 *     compared (4 bytes);
 *   - a match is extended backwards while ip > anchor, match > 0 and the previous bytes agree,
 *     then forwards (LZ4_count) up to len - 5 (matchlimit);
 *   - after a match: stop if ip >= len - 11; insert ip - 2; probe ip itself (insert, compare):
 *     a hit is a new sequence with no literals; otherwise the search restarts at ip + 1.
 * Returns the LZ4 block size (always > 0). */
int32_t o_lz4_compress_default(const uint8_t* src, int32_t len, uint8_t* dst) {
  static const uint32_t kMinLength = 13, kMfLimit = 12, kLastLiterals = 5, kSkip = 6;
  uint16_t tab[1u << 13];
  memset(tab, 0, sizeof tab);
  const uint32_t n = (uint32_t)len;
  uint8_t* op = dst;
  uint8_t* token = NULL;
  uint32_t anchor = 0, ip = 0, match = 0;
#define O_H(p) ((rd32(src + (p)) * XP1) >> 19)
  if (n >= kMinLength) {
    const uint32_t mflimit1 = n - kMfLimit + 1, matchlimit = n - kLastLiterals;
    tab[O_H(0)] = 0;
    ip = 1;
    uint32_t fh = O_H(ip);
    for (;;) {
      /* find a match */
      {
        uint32_t fip = ip, step = 1, nb = 1u << kSkip;
        for (;;) {
          const uint32_t h = fh, cur = fip;
          const uint32_t mi = tab[h];
          ip = fip;
          fip += step;
          step = nb++ >> kSkip;
          if (fip > mflimit1) goto last_literals;
          match = mi;
          fh = O_H(fip);
          tab[h] = (uint16_t)cur;
          if (rd32(src + match) == rd32(src + ip)) break;
        }
      }
      /* catch up */
      while (ip > anchor && match > 0 && src[ip - 1] == src[match - 1]) {
        --ip;
        --match;
      }
      /* literals */
      {
        const uint32_t ll = ip - anchor;
        token = op++;
        if (ll >= 15) {
          *token = 15 << 4;
          uint32_t r = ll - 15;
          for (; r >= 255; r -= 255) *op++ = 255;
          *op++ = (uint8_t)r;
        } else {
          *token = (uint8_t)(ll << 4);
        }
        memcpy(op, src + anchor, ll);
        op += ll;
      }
      for (;;) { /* _next_match */
        const uint32_t off = ip - match;
        *op++ = (uint8_t)off;
        *op++ = (uint8_t)(off >> 8);
        uint32_t mc = 0;
        while (ip + 4 + mc < matchlimit && src[ip + 4 + mc] == src[match + 4 + mc]) ++mc;
        ip += mc + 4;
        if (mc >= 15) {
          *token += 15;
          mc -= 15;
          for (; mc >= 255; mc -= 255) *op++ = 255;
          *op++ = (uint8_t)mc;
        } else {
          *token += (uint8_t)mc;
        }
        anchor = ip;
        if (ip >= mflimit1) goto last_literals;
        tab[O_H(ip - 2)] = (uint16_t)(ip - 2);
        /* test next position */
        const uint32_t h = O_H(ip), mi = tab[h];
        tab[h] = (uint16_t)ip;
        if (rd32(src + mi) == rd32(src + ip)) {
          token = op++;
          *token = 0;
          match = mi;
          continue;
        }
        break;
      }
      fh = O_H(++ip);
    }
  }
last_literals: {
    const uint32_t ll = n - anchor;
    if (ll >= 15) {
      *op++ = 15 << 4;
      uint32_t r = ll - 15;
      for (; r >= 255; r -= 255) *op++ = 255;
      *op++ = (uint8_t)r;
    } else {
      *op++ = (uint8_t)(ll << 4);
    }
    memcpy(op, src + anchor, ll);
    op += ll;
  }
#undef O_H
  return (int32_t)(op - dst);
}

/* lz4-java's LZ4BlockOutputStream.flushBufferedData: the chunk is stored raw when the LZ4 block
 * is not shorter.  Returns the LZ4 block size, or 0 for a raw chunk. */
int32_t o_lz4_compress_block(const uint8_t* src, int32_t len, uint8_t* dst) {
  uint8_t tmp[65536 + 65536 / 255 + 16 + 64];
  if (len <= 0 || len > 65536) return 0;
  const int32_t c = o_lz4_compress_default(src, len, tmp);
  if (c >= len) return 0;
  memcpy(dst, tmp, (size_t)c);
  return c;
}

/* LZ4 block decoder (spec restatement).  Returns the decoded size, or -1 on malformed input. */
int32_t o_lz4_decompress_block(const uint8_t* src, int32_t slen, uint8_t* dst, int32_t cap) {
  const uint8_t *ip = src, *ie = src + slen;
  int32_t op = 0;
  while (ip < ie) {
    const uint32_t tok = *ip++;
    uint32_t LL = tok >> 4;
    if (LL == 15) {
      uint32_t b;
      do {
        if (ip >= ie) return -1;
        b = *ip++;
        LL += b;
      } while (b == 255);
    }
    if ((int64_t)(ie - ip) < LL || op + (int64_t)LL > cap) return -1;
    memcpy(dst + op, ip, LL);
    ip += LL;
    op += (int32_t)LL;
    if (ip == ie) break; /* last sequence: literals only */
    if (ie - ip < 2) return -1;
    const uint32_t off = ip[0] | ((uint32_t)ip[1] << 8);
    ip += 2;
    if (off == 0 || (int32_t)off > op) return -1;
    uint32_t ml = (tok & 15) + 4;
    if ((tok & 15) == 15) {
      uint32_t b;
      do {
        if (ip >= ie) return -1;
        b = *ip++;
        ml += b;
      } while (b == 255);
    }
    if (op + (int64_t)ml > cap) return -1;
    for (uint32_t k = 0; k < ml; ++k) dst[op + k] = dst[op - off + k];
    op += (int32_t)ml;
  }
  return op;
}

static int lz4_level(uint32_t bs) {
  int l = 32 - __builtin_clz(bs - 1u);
  return l > 10 ? l - 10 : 0;
}

/* One LZ4BlockOutputStream stream of src[0, n) (n > 0); returns its size.  dst must hold
 * n + (n / bs + 1) * 21 + 21 bytes. */
uint64_t o_lz4_stream(const uint8_t* src, uint64_t n, uint32_t bs, uint8_t* dst) {
  const int level = lz4_level(bs);
  uint64_t o = 0;
  for (uint64_t a = 0; a < n; a += bs) {
    const uint32_t len = (uint32_t)(n - a < bs ? n - a : bs);
    uint8_t* h = dst + o;
    memcpy(h, "LZ4Block", 8);
    const int32_t c = o_lz4_compress_block(src + a, (int32_t)len, h + 21);
    if (c == 0) memcpy(h + 21, src + a, len);
    h[8] = (uint8_t)((c ? 0x20 : 0x10) | level);
    wr32(h + 9, c ? (uint32_t)c : len);
    wr32(h + 13, len);
    wr32(h + 17, o_xxh32(src + a, len, 0x9747b28cu) & 0x0FFFFFFFu);
    o += 21 + (c ? (uint32_t)c : len);
  }
  uint8_t* h = dst + o;
  memcpy(h, "LZ4Block", 8);
  h[8] = (uint8_t)(0x10 | level);
  memset(h + 9, 0, 12);
  return o + 21;
}

/* Every (map, partition) run of consecutive map outputs -> its stream (empty runs: nothing),
 * and the per-map index of the compressed output (R + 1 int64 per map, native). */
uint64_t o_lz4_map_outputs(const uint8_t* data, const int64_t* index, int32_t maps, int32_t R,
                           uint32_t bs, uint8_t* out, int64_t* out_index) {
  uint64_t in = 0, o = 0;
  for (int32_t m = 0; m < maps; ++m) {
    const int64_t* im = index + (int64_t)m * (R + 1);
    int64_t* om = out_index + (int64_t)m * (R + 1);
    const uint64_t mo = o;
    for (int32_t p = 0; p < R; ++p) {
      om[p] = (int64_t)(o - mo);
      const uint64_t L = (uint64_t)(im[p + 1] - im[p]);
      if (L) o += o_lz4_stream(data + in + im[p], L, bs, out + o);
    }
    om[R] = (int64_t)(o - mo);
    in += (uint64_t)im[R];
  }
  return o;
}

/* Decode one concatenation of LZ4BlockOutputStream streams (what a reader fetches for a block
 * range); verifies magic, lengths and checksums.  Returns the decoded size, or -1. */
int64_t o_lz4_unframe(const uint8_t* s, uint64_t n, uint8_t* dst, uint64_t cap) {
  uint64_t i = 0, o = 0;
  while (i < n) {
    if (n - i < 21 || memcmp(s + i, "LZ4Block", 8) != 0) return -1;
    const uint32_t method = s[i + 8] & 0xF0;
    const uint32_t clen = rd32(s + i + 9), olen = rd32(s + i + 13), chk = rd32(s + i + 17);
    i += 21;
    if (olen == 0) { /* end mark */
      if (clen != 0 || chk != 0 || method != 0x10) return -1;
      continue;
    }
    if (n - i < clen || o + olen > cap) return -1;
    if (method == 0x10) {
      if (clen != olen) return -1;
      memcpy(dst + o, s + i, olen);
    } else if (method == 0x20) {
      if (o_lz4_decompress_block(s + i, (int32_t)clen, dst + o, (int32_t)olen) != (int32_t)olen)
        return -1;
    } else {
      return -1;
    }
    if ((o_xxh32(dst + o, olen, 0x9747b28cu) & 0x0FFFFFFFu) != chk) return -1;
    i += clen;
    o += olen;
  }
  return (int64_t)o;
}
