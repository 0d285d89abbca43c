// Seeded initialisation replay: torch's CPU generator (mt19937) and
// uniform_real_distribution<float>, reproduced draw for draw on the host so a
// sweep's ~10^8 init draws cost the generator's time rather than ~6 ns each
// through Tensor.uniform_ (see include/nerfhip.h).  The reference draws them
// through nn.Linear + Tensor.uniform_ (nerf_attention/siren.py:17-67); the
// result is checked bit for bit against torch in tests/test_host.py.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "nerfhip.h"

namespace {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

inline uint32_t twist(uint32_t u, uint32_t v) {
  return (((u & kUpper) | (v & kLower)) >> 1) ^ ((v & 1u) ? kMatrixA : 0u);
}

// The generator's whole-state refresh (the standard mt19937 recurrence).
__attribute__((always_inline)) inline void regenerate(uint32_t* s) {
  int i = 0;
  for (; i < kN - kM; ++i) s[i] = s[i + kM] ^ twist(s[i], s[i + 1]);
  for (; i < kN - 1; ++i) s[i] = s[i + kM - kN] ^ twist(s[i], s[i + 1]);
  s[kN - 1] = s[kM - 1] ^ twist(s[kN - 1], s[0]);
}

inline uint32_t temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// One draw in torch's terms: `if (--left == 0) refresh; y = state[next++]`.
// Equivalently, left - 1 words (state[next ..]) remain before the next
// refresh, after which left = 625, next = 0.  Blocks of words are consumed at
// a time between refreshes.  The transform is x = (y & 2^24-1) * 2^-24, then
// fma(x, hi - lo, lo): torch's AVX2 / AVX-512 CPU kernels contract x*(hi-lo)+lo
// into one rounding, and half the values differ in the last bit without it.
__attribute__((always_inline)) inline void consume_body(uint32_t* s, int32_t& left,
                                                        uint32_t& next, int64_t n, float lo,
                                                        float hi, float* out) {
  const float span = hi - lo;
  const float scale = 1.0f / 16777216.0f;
  while (n > 0) {
    if (left <= 1) {
      regenerate(s);
      left = kN + 1;
      next = 0;
    }
    int64_t take = left - 1;
    if (take > n) take = n;
    if (out) {
      const uint32_t* w = s + next;
      for (int64_t i = 0; i < take; ++i) {
        const float x = static_cast<float>(temper(w[i]) & 0xffffffu) * scale;
        out[i] = __builtin_fmaf(x, span, lo);
      }
      out += take;
    }
    next += static_cast<uint32_t>(take);
    left -= static_cast<int32_t>(take);
    n -= take;
  }
}

// Hardware FMA + AVX2 where the host has them (the MI355X hosts do); the
// portable build calls libm's fmaf, same bits, ~2x slower.
__attribute__((target("avx2,fma"))) void consume_fma(uint32_t* s, int32_t& left, uint32_t& next,
                                                     int64_t n, float lo, float hi, float* out) {
  consume_body(s, left, next, n, lo, hi, out);
}

void consume_portable(uint32_t* s, int32_t& left, uint32_t& next, int64_t n, float lo, float hi,
                      float* out) {
  consume_body(s, left, next, n, lo, hi, out);
}

}  // namespace

extern "C" int nerfhip_rng_uniform_segments(uint32_t* state, int32_t* left, uint32_t* next,
                                            int32_t n_segments, const int64_t* counts,
                                            const double* lo, const double* hi,
                                            const int64_t* out_off, float* out) {
  if (!state || !left || !next || (n_segments > 0 && (!counts || !lo || !hi || !out_off)))
    return NERFHIP_ERR_NULL;
  if (n_segments < 0 || *left < 1 || *left > kN || *next > static_cast<uint32_t>(kN))
    return NERFHIP_ERR_BAD_SHAPE;
  for (int32_t k = 0; k < n_segments; ++k) {      // validate first: the state moves all or not at all
    if (counts[k] < 0) return NERFHIP_ERR_BAD_SHAPE;
    if (out_off[k] >= 0 && !out) return NERFHIP_ERR_NULL;
  }
  int32_t l = *left;
  uint32_t nx = *next;
  const bool fma = __builtin_cpu_supports("fma") && __builtin_cpu_supports("avx2");
  for (int32_t k = 0; k < n_segments; ++k) {
    const float a = static_cast<float>(lo[k]), b = static_cast<float>(hi[k]);
    float* dst = out_off[k] >= 0 ? out + out_off[k] : nullptr;
    if (fma)
      consume_fma(state, l, nx, counts[k], a, b, dst);
    else
      consume_portable(state, l, nx, counts[k], a, b, dst);
  }
  *left = l;
  *next = nx;
  return NERFHIP_OK;
}
