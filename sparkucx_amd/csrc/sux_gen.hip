// sux_gen.hip — synthetic shuffle inputs, generated on the device (not part of the timed path).
// Counter-based: record i depends only on (seed, i), bit-identical to oracle/oracle.c, so a CPU
// checker can regenerate any slice without a transfer.  One thread per output dword keeps the
// stores fully coalesced.
#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

#include "sux_internal.h"

namespace sux {

__device__ __host__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ void rec_words(uint64_t seed, uint64_t i, uint64_t& a, uint64_t& b) {
  a = mix64((seed * 0x2545F4914F6CDD1Dull) ^ i);
  b = mix64(a ^ 0xA0761D6478BD642Full);
}

__device__ __forceinline__ uint64_t zipf_draw(const uint64_t* bounds, const uint64_t* thresh,
                                              int nb, uint64_t u1, uint64_t u2) {
  int lo = 0, hi = nb - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (thresh[mid] <= u1) lo = mid; else hi = mid - 1;
  }
  return bounds[lo] + __umul64hi(u2, bounds[lo + 1] - bounds[lo]);
}

// dword w (0..24) of a 100-byte record whose key words are (k_lo, k_hi)
__device__ __forceinline__ uint32_t word100(uint32_t w, uint64_t i, uint64_t keyw, uint64_t b) {
  switch (w) {
    case 0: return (uint32_t)keyw;
    case 1: return (uint32_t)(keyw >> 32);
    case 2: return (uint32_t)b;
    case 3: return (uint32_t)i;
    case 4: return (uint32_t)(i >> 32);
    default: return (uint32_t)(b >> 32) + (w - 5) * 0x01010101u;
  }
}

__global__ __launch_bounds__(256) void k_gen(int kind, uint64_t seed, uint64_t first, uint64_t n,
                                             const uint64_t* zb, const uint64_t* zt, int znb,
                                             uint32_t* out) {
  const uint32_t words = (kind == 2) ? 4u : 25u;
  const uint64_t total = n * words;
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * 256) {
    uint64_t j = t / words;
    uint32_t w = (uint32_t)(t - j * words);
    uint64_t i = first + j, a, b;
    rec_words(seed, i, a, b);
    uint32_t v;
    if (kind == 2) {
      v = (w == 0) ? (uint32_t)a : (w == 1) ? (uint32_t)(a >> 32) : (w == 2) ? (uint32_t)i
                                                                               : (uint32_t)(i >> 32);
    } else {
      uint64_t keyw = a;
      if (kind == 3 && w < 2) keyw = zipf_draw(zb, zt, znb, a, b);
      v = word100(w, i, keyw, b);
    }
    out[t] = v;
  }
}

hipError_t launch_generate(int kind, uint64_t seed, uint64_t first, uint64_t n,
                           const uint64_t* d_zipf_bounds, const uint64_t* d_zipf_thresh,
                           int zipf_nb, uint8_t* d_out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t words = n * ((kind == 2) ? 4 : 25);
  uint64_t blocks = (words + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(k_gen, dim3((uint32_t)blocks), dim3(256), 0, s, kind, seed, first, n,
                     d_zipf_bounds, d_zipf_thresh, zipf_nb, reinterpret_cast<uint32_t*>(d_out));
  return hipGetLastError();
}

// ---- host Zipf table: same construction as oracle/oracle.c (o_zipf_table) -----------------
constexpr uint64_t kZipfExact = 256;
constexpr int kZipfGeo = 1024;

static int zipf_bounds(uint64_t n, uint64_t* bounds) {
  int nb = 0;
  uint64_t e = n < kZipfExact ? n : kZipfExact;
  for (uint64_t k = 1; k <= e; ++k) {
    if (bounds) bounds[nb] = k;
    nb++;
  }
  uint64_t prev = e + 1;
  if (n > e) {
    double base = (double)(e + 1), ratio = (double)(n + 1) / base;
    for (int j = 1; j <= kZipfGeo; ++j) {
      uint64_t b = (j == kZipfGeo) ? n + 1
                                   : (uint64_t)std::llround(base * std::pow(ratio, (double)j / kZipfGeo));
      if (b <= prev) continue;
      if (b > n + 1) b = n + 1;
      if (bounds) bounds[nb] = prev;
      nb++;
      prev = b;
      if (b == n + 1) break;
    }
  }
  if (bounds) bounds[nb] = prev;
  return nb;
}

int zipf_table_size(uint64_t zipf_n) { return zipf_bounds(zipf_n, nullptr); }

static double zipf_mass(uint64_t lo, uint64_t hi, double s) {
  if (hi - lo <= 4) {
    double m = 0;
    for (uint64_t k = lo; k < hi; ++k) m += std::pow((double)k, -s);
    return m;
  }
  double a = (double)lo - 0.5, b = (double)hi - 0.5;
  if (std::fabs(s - 1.0) < 1e-12) return std::log(b) - std::log(a);
  return (std::pow(a, 1.0 - s) - std::pow(b, 1.0 - s)) / (s - 1.0);
}

void zipf_table(double s, uint64_t zipf_n, uint64_t* bounds, uint64_t* thresh) {
  int nb = zipf_bounds(zipf_n, bounds);
  std::vector<double> w((size_t)nb);
  double total = 0;
  for (int j = 0; j < nb; ++j) {
    w[j] = zipf_mass(bounds[j], bounds[j + 1], s);
    total += w[j];
  }
  double cum = 0;
  for (int j = 0; j < nb; ++j) {
    double f = std::ldexp(cum / total, 64);
    thresh[j] = (j == 0) ? 0 : (f >= 18446744073709551615.0 ? UINT64_MAX : (uint64_t)f);
    cum += w[j];
  }
  thresh[nb] = UINT64_MAX;
}

}  // namespace sux
