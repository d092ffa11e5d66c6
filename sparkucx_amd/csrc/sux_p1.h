// sux_p1.h — device-side partition functions, shared by the map-side kernel
// files (sux_partition.hip, sux_varlen.hip).  Spark semantics, restated in oracle/oracle.c
// (o_get_partition).  Device code only; included inside namespace sux.
#pragma once

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t mix_k1(uint32_t k1) {
  k1 *= 0xcc9e2d51u;
  k1 = rotl32(k1, 15);
  return k1 * 0x1b873593u;
}
__device__ __forceinline__ uint32_t mix_h1(uint32_t h1, uint32_t k1) {
  h1 ^= k1;
  h1 = rotl32(h1, 13);
  return h1 * 5u + 0xe6546b64u;
}
__device__ __forceinline__ uint32_t fmix32(uint32_t h1, uint32_t len) {
  h1 ^= len;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  return h1 ^ (h1 >> 16);
}
__device__ __forceinline__ int32_t pmod(int32_t a, int32_t n) {
  int32_t r = a % n;
  return r < 0 ? (r + n) % n : r;
}

__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p, int off) {
  if ((off & 3) == 0) return *reinterpret_cast<const uint32_t*>(p + off);
  return (uint32_t)p[off] | ((uint32_t)p[off + 1] << 8) | ((uint32_t)p[off + 2] << 16) |
         ((uint32_t)p[off + 3] << 24);
}

// Big-endian (hi, lo) words of a key of `len` (1..16) bytes, bytes past len zeroed.
__device__ __forceinline__ void load_key_be(const uint8_t* rec, int off, int len, uint64_t& hi,
                                            uint64_t& lo) {
  uint32_t w0 = ld_u32(rec, off);
  uint32_t w1 = len > 4 ? ld_u32(rec, off + 4) : 0u;
  uint32_t w2 = len > 8 ? ld_u32(rec, off + 8) : 0u;
  uint32_t w3 = len > 12 ? ld_u32(rec, off + 12) : 0u;
  hi = ((uint64_t)__builtin_bswap32(w0) << 32) | __builtin_bswap32(w1);
  lo = ((uint64_t)__builtin_bswap32(w2) << 32) | __builtin_bswap32(w3);
  if (len < 8) {
    hi &= ~0ull << (8 * (8 - len));
    lo = 0;
  } else if (len < 16) {
    lo = (len == 8) ? 0 : (lo & (~0ull << (8 * (16 - len))));
  }
}

__device__ __forceinline__ int range_search(const PartDev& pd, uint64_t hi, uint64_t lo) {
  int a = 0, b = pd.R - 1;  // answer = #{bounds < key} in [a, b]
  if (pd.lut_bits) {
    uint32_t e = pd.lut[hi >> (64 - pd.lut_bits)];
    a = e & 0xFFFFu;
    b = e >> 16;
  }
  while (a < b) {
    int mid = (a + b) >> 1;
    uint64_t bh = pd.bounds[2 * mid], bl = pd.bounds[2 * mid + 1];
    bool less = (bh < hi) || (bh == hi && bl < lo);  // bound < key
    if (less) a = mid + 1; else b = mid;
  }
  return a;
}

__device__ __forceinline__ int get_partition(const PartDev& pd, const uint8_t* rec) {
  switch (pd.kind) {
    case 1: {  // SUX_PART_RANGE_BYTES
      uint64_t hi, lo;
      load_key_be(rec, pd.key_offset, pd.key_len, hi, lo);
      int p = range_search(pd, hi, lo);
      return pd.ascending ? p : (pd.R - 1) - p;
    }
    case 2: {  // SUX_PART_MURMUR3_LONG
      uint32_t lo32 = ld_u32(rec, pd.key_offset), hi32 = ld_u32(rec, pd.key_offset + 4);
      uint32_t h1 = mix_h1((uint32_t)pd.seed, mix_k1(lo32));
      h1 = mix_h1(h1, mix_k1(hi32));
      return pmod((int32_t)fmix32(h1, 8), pd.R);
    }
    case 3: {  // SUX_PART_MURMUR3_INT
      uint32_t v = ld_u32(rec, pd.key_offset);
      return pmod((int32_t)fmix32(mix_h1((uint32_t)pd.seed, mix_k1(v)), 4), pd.R);
    }
    case 4: {  // SUX_PART_MURMUR3_BYTES (legacy hashUnsafeBytes)
      const int off = pd.key_offset, len = pd.key_len, aligned = len - len % 4;
      uint32_t h1 = (uint32_t)pd.seed;
      for (int i = 0; i < aligned; i += 4) h1 = mix_h1(h1, mix_k1(ld_u32(rec, off + i)));
      for (int i = aligned; i < len; ++i)
        h1 = mix_h1(h1, mix_k1((uint32_t)(int32_t)(int8_t)rec[off + i]));
      return pmod((int32_t)fmix32(h1, (uint32_t)len), pd.R);
    }
    case 5: {  // SUX_PART_HASH_LONG: nonNegativeMod(Long.hashCode)
      uint32_t h = ld_u32(rec, pd.key_offset) ^ ld_u32(rec, pd.key_offset + 4);
      int32_t r = (int32_t)h % pd.R;
      return r + (r < 0 ? pd.R : 0);
    }
    case 6: {  // SUX_PART_HASH_INT
      int32_t r = (int32_t)ld_u32(rec, pd.key_offset) % pd.R;
      return r + (r < 0 ? pd.R : 0);
    }
    case kPartRadix: {  // internal: digit of the big-endian 128-bit (key, index) pair
      const uint64_t hi = ((uint64_t)__builtin_bswap32(ld_u32(rec, 0)) << 32) |
                          __builtin_bswap32(ld_u32(rec, 4));
      const uint64_t lo = ((uint64_t)__builtin_bswap32(ld_u32(rec, 8)) << 32) |
                          __builtin_bswap32(ld_u32(rec, 12));
      const int sh = pd.seed;
      const uint64_t v = sh >= 64 ? (hi >> (sh - 64)) : ((lo >> sh) | (sh ? (hi << (64 - sh)) : 0));
      return (int)(v & (uint64_t)(pd.R - 1));
    }
  }
  return 0;
}

