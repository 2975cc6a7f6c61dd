/* TEST INFRASTRUCTURE (oracle side) -- the counter-based synthetic weight generator of
 * oracle/weightgen.py in plain C, for the CPU oracle's Qwen3-8B / 32B runs (numpy takes minutes
 * for the 8 G values of a whole Qwen3-8B).  Same integer and fp32 arithmetic as the module
 * docstring there, so the two are bit-identical (tests/test_oracle_golden.py checks it):
 *     u24(i) = splitmix64(key + i) >> 40
 *     t      = u24 * 2^-23 - 1            (exact in fp32)
 *     w      = fl(fl(t * scale) + center)  (two roundings: built with -ffp-contract=off)
 *     out    = bf16_rne(w)
 * Not product code: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it
 * (through oracle/weightgen.py). */
#include <stdint.h>

static inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline uint16_t bf16_rne(float f) {
  union { float f; uint32_t u; } v = {f};
  return (uint16_t)((v.u + 0x7FFFu + ((v.u >> 16) & 1u)) >> 16);
}

/* out[i] = bf16 bits of w(offset + i), i < n */
void wg_bf16(uint64_t key, float scale, float center, int64_t offset, int64_t n, uint16_t* out) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t z = splitmix64(key + (uint64_t)(offset + i));
    const float t = (float)(uint32_t)(z >> 40) * 1.1920928955078125e-07f - 1.0f;
    const float w = t * scale;
    out[i] = bf16_rne(w + center);
  }
}
