// Host check (test infrastructure): the packed Box-Muller pair (noise_block_pk) against the scalar
// noise_block, bit for bit, over random Philox blocks and the edge uniforms.  Built and run by
// tests/test_noise_pack.py with -ffp-contract=off, as the library.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "mppi_detmath.h"

using namespace mppi;

static uint64_t sm(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static int cmp4(const float* a, const float* b) { return std::memcmp(a, b, 4 * sizeof(float)) != 0; }

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  uint64_t st = 12345;
  long bad = 0;
  for (long i = 0; i < n; ++i) {
    const uint64_t seed = sm(st), nn = sm(st) >> (i & 31), k = sm(st) >> (i & 63 ? 20 : 0);
    float a[4], b[4];
    noise_block(seed, nn, k, a, a + 1, a + 2, a + 3);
    noise_block_pk(seed, nn, k, b, b + 1, b + 2, b + 3);
    if (cmp4(a, b) && bad++ < 5)
      printf("mismatch seed %llu n %llu k %llu: %a %a %a %a vs %a %a %a %a\n", (unsigned long long)seed,
             (unsigned long long)nn, (unsigned long long)k, a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]);
  }
  // every edge of the 24-bit uniforms through the Box-Muller pair directly (u = 2^-24 .. 1, v = 0 ..)
  const uint32_t edges[] = {0u, 0xFFu, 0x100u, 0x1FFu, 0x7FFFFF00u, 0x80000000u, 0xFFFFFEFFu, 0xFFFFFF00u, 0xFFFFFFFFu};
  for (uint32_t ra : edges)
    for (uint32_t rb : edges) {
      float a[4], b[4];
      dm_box_muller(ra, rb, a, a + 1);
      dm_box_muller(rb, ra, a + 2, a + 3);
      const mf2 u = (mf2{(float)(ra >> 8), (float)(rb >> 8)} + 1.0f) * 5.9604644775390625e-8f;
      const mf2 v = mf2{(float)(rb >> 8), (float)(ra >> 8)} * 5.9604644775390625e-8f;
      const mf2 l = -2.0f * dm_logf2(u);
      const mf2 rad = mf2{sqrtf(l.x), sqrtf(l.y)};
      mf2 s, c;
      dm_sincosf2_pos(6.2831853071795864769f * v, &s, &c);
      const mf2 zc = rad * c, zs = rad * s;
      b[0] = zc.x; b[1] = zs.x; b[2] = zc.y; b[3] = zs.y;
      if (cmp4(a, b) && bad++ < 10) printf("edge mismatch ra %08x rb %08x\n", ra, rb);
    }
  // the sincos quadrants: every 24-bit v near the octant boundaries
  for (int q = 0; q <= 8; ++q)
    for (int d = -300; d <= 300; ++d) {
      const double vv = q / 8.0 + d * 5.9604644775390625e-8;
      if (vv < 0 || vv >= 1) continue;
      const uint32_t rb = ((uint32_t)(vv * 16777216.0)) << 8;
      float a[2];
      dm_box_muller(0x12345600u, rb, a, a + 1);
      const mf2 u = (mf2{(float)(0x12345600u >> 8), (float)(0x12345600u >> 8)} + 1.0f) * 5.9604644775390625e-8f;
      const mf2 v = mf2{(float)(rb >> 8), (float)(rb >> 8)} * 5.9604644775390625e-8f;
      const mf2 l = -2.0f * dm_logf2(u);
      const mf2 rad = mf2{sqrtf(l.x), sqrtf(l.y)};
      mf2 s, c;
      dm_sincosf2_pos(6.2831853071795864769f * v, &s, &c);
      const mf2 zc = rad * c, zs = rad * s;
      const float g0 = zc.x, g1 = zs.x;
      if ((std::memcmp(&a[0], &g0, 4) || std::memcmp(&a[1], &g1, 4)) && bad++ < 15) printf("quadrant mismatch rb %08x\n", rb);
    }
  printf("checked %ld blocks: %ld mismatches\n", n, bad);
  return bad != 0;
}
