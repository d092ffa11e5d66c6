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
// a mod n in [0, n) for n >= 1 — Spark's pmod (Pmod of HashPartitioning) and nonNegativeMod
// (HashPartitioner) agree with it for a positive modulus.  The remainder of |a| comes from
// Lemire's fastmod with M = part_magic(n): ((M * u mod 2^64) * n) >> 64, exact for every 32-bit u
// and n; a negative a with a non-zero remainder m maps to n - m.  (Checked against the C `%`
// definition on 4.7e8 cases, every R the tests use among them; the GPU tests check it against
// oracle.c.)
__device__ __forceinline__ int32_t mod_pos(int32_t a, int32_t n, uint64_t M) {
  const uint32_t u = a < 0 ? 0u - (uint32_t)a : (uint32_t)a;
  const uint32_t m = (uint32_t)__umul64hi(M * (uint64_t)u, (uint64_t)(uint32_t)n);
  return (a < 0 && m) ? n - (int32_t)m : (int32_t)m;
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
      return mod_pos((int32_t)fmix32(h1, 8), pd.R, pd.rmagic);
    }
    case 3: {  // SUX_PART_MURMUR3_INT
      uint32_t v = ld_u32(rec, pd.key_offset);
      return mod_pos((int32_t)fmix32(mix_h1((uint32_t)pd.seed, mix_k1(v)), 4), pd.R, pd.rmagic);
    }
    case 4: {  // SUX_PART_MURMUR3_BYTES (legacy hashUnsafeBytes)
      const int off = pd.key_offset, len = pd.key_len, aligned = len - len % 4;
      uint32_t h1 = (uint32_t)pd.seed;
      for (int i = 0; i < aligned; i += 4) h1 = mix_h1(h1, mix_k1(ld_u32(rec, off + i)));
      for (int i = aligned; i < len; ++i)
        h1 = mix_h1(h1, mix_k1((uint32_t)(int32_t)(int8_t)rec[off + i]));
      return mod_pos((int32_t)fmix32(h1, (uint32_t)len), pd.R, pd.rmagic);
    }
    case 5: {  // SUX_PART_HASH_LONG: nonNegativeMod(Long.hashCode)
      uint32_t h = ld_u32(rec, pd.key_offset) ^ ld_u32(rec, pd.key_offset + 4);
      return mod_pos((int32_t)h, pd.R, pd.rmagic);
    }
    case 6: {  // SUX_PART_HASH_INT
      return mod_pos((int32_t)ld_u32(rec, pd.key_offset), pd.R, pd.rmagic);
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

// Range search with the bounds + 10-bit prefix LUT (LDS-resident when TAB).
template <bool TAB>
__device__ __forceinline__ int range_search_t(int R, const uint64_t* bounds, const uint32_t* lut,
                                              uint64_t hi, uint64_t lo) {
  const uint32_t e = lut[hi >> (64 - kLutBits)];
  int a = e & 0xFFFFu, b = e >> 16;
  while (a < b) {
    const int mid = (a + b) >> 1;
    const uint64_t bh = bounds[2 * mid], bl = bounds[2 * mid + 1];
    if ((bh < hi) || (bh == hi && bl < lo)) a = mid + 1; else b = mid;
  }
  return a;
}

// P1 from preloaded little-endian key dwords (key at a 4-byte aligned record offset).
template <int KW, bool TAB>
__device__ __forceinline__ int partition_words(const PartDev& pd, const uint32_t (&w)[KW],
                                               const uint64_t* bounds, const uint32_t* lut) {
  const int R = pd.R;
  switch (pd.kind) {
    case 1: {
      if (R == 1) return 0;
      uint64_t hi = (uint64_t)__builtin_bswap32(w[0]) << 32, lo = 0;
      if constexpr (KW > 1) hi |= __builtin_bswap32(w[1]);
      if constexpr (KW > 2) lo = (uint64_t)__builtin_bswap32(w[2]) << 32;
      if constexpr (KW > 3) lo |= __builtin_bswap32(w[3]);
      const int len = pd.key_len;
      if (len < 8) {
        hi &= ~0ull << (8 * (8 - len));
        lo = 0;
      } else if (len < 16) {
        lo = (len == 8) ? 0 : (lo & (~0ull << (8 * (16 - len))));
      }
      const int p = range_search_t<TAB>(R, bounds, lut, hi, lo);
      return pd.ascending ? p : (R - 1) - p;
    }
    case 2: {
      uint32_t h1 = mix_h1((uint32_t)pd.seed, mix_k1(w[0]));
      if constexpr (KW > 1) h1 = mix_h1(h1, mix_k1(w[1]));
      return mod_pos((int32_t)fmix32(h1, 8), R, pd.rmagic);
    }
    case 3:
      return mod_pos((int32_t)fmix32(mix_h1((uint32_t)pd.seed, mix_k1(w[0])), 4), R, pd.rmagic);
    case 5: {
      uint32_t h = w[0];
      if constexpr (KW > 1) h ^= w[1];
      return mod_pos((int32_t)h, R, pd.rmagic);
    }
    case 6: {
      return mod_pos((int32_t)w[0], R, pd.rmagic);
    }
    case kPartRadix:  // internal (sux_sort_records): digit of the big-endian 128-bit pair
      if constexpr (KW == 4) {
        const uint64_t hi = ((uint64_t)__builtin_bswap32(w[0]) << 32) | __builtin_bswap32(w[1]);
        const uint64_t lo = ((uint64_t)__builtin_bswap32(w[2]) << 32) | __builtin_bswap32(w[3]);
        const int sh = pd.seed;
        const uint64_t v = sh >= 64 ? (hi >> (sh - 64)) : ((lo >> sh) | (sh ? (hi << (64 - sh)) : 0));
        return (int)(v & (uint64_t)(R - 1));
      }
      return 0;
  }
  return 0;
}

template <int KW>
struct KeyVec;
template <>
struct KeyVec<1> {
  typedef uint32_t T;
  static __device__ __forceinline__ void get(T v, uint32_t (&w)[1]) { w[0] = v; }
};
template <>
struct KeyVec<2> {
  typedef uint32_t T __attribute__((ext_vector_type(2), aligned(4)));
  static __device__ __forceinline__ void get(T v, uint32_t (&w)[2]) { w[0] = v.x; w[1] = v.y; }
};
template <>
struct KeyVec<3> {
  typedef uint32_t T __attribute__((ext_vector_type(3), aligned(4)));
  static __device__ __forceinline__ void get(T v, uint32_t (&w)[3]) {
    w[0] = v.x; w[1] = v.y; w[2] = v.z;
  }
};
template <>
struct KeyVec<4> {
  typedef uint32_t T __attribute__((ext_vector_type(4), aligned(4)));
  static __device__ __forceinline__ void get(T v, uint32_t (&w)[4]) {
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  }
};

// Workgroup b -> work index, so that the ~gridDim/8 workgroups the dispatcher deals to one XCD
// (b, b+8, b+16, ...) get one contiguous range of tiles.  A bijection on [0, n); placement is a
// speed hint only, never a correctness assumption.
__device__ __forceinline__ uint32_t xcd_map(uint32_t b, uint32_t n) {
  const uint32_t per = (n + 7) / 8, rem = n % 8, x = b % 8, k = b / 8;
  if (rem == 0 || x < rem) return x * per + k;
  return rem * per + (x - rem) * (per - 1) + k;
}
