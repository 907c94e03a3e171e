// Deterministic float32 math + Philox4x32-10 for the MPPI engine (gfx950).
//
// The reference evaluates wp.sin/wp.cos/wp.exp/wp.randn with CUDA libdevice
// (projection_warp.py:236-237, critics_warp.py:347, sampling_warp.py:73-91).
// This engine DEFINES each transcendental as a fixed sequence of IEEE float32
// + - * / operations (Cephes minimax polynomials).  The file must be compiled
// with -ffp-contract=off so that no a*b+c is fused: the numpy restatement in
// oracle/dmath.py runs the identical sequence and matches bit for bit.
//
// Noise: Philox4x32-10, the generator of rocrand_philox4x32_10.h
// (ten_rounds / single_round), keyed by the 64-bit seed, counter
// (n_lo, n_hi, k_lo, k_hi)  ==  rocrand_init(seed, subsequence = k,
// offset = 4 n).  One block feeds two rollout-steps of one trajectory.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define MPPI_HD __host__ __device__ __forceinline__

namespace mppi {

MPPI_HD float bits_f(uint32_t u) { return __builtin_bit_cast(float, u); }
MPPI_HD uint32_t f_bits(float f) { return __builtin_bit_cast(uint32_t, f); }

// ------------------------------------------------------------------ log
// Cephes logf; x must be a positive normal float (Box-Muller: x in [2^-24, 1]).
MPPI_HD float dm_logf(float x) {
  const uint32_t b = f_bits(x);
  int e = (int)((b >> 23) & 0xFFu) - 126;
  float m = bits_f((b & 0x807FFFFFu) | 0x3F000000u);  // [0.5, 1)
  if (m < 0.707106781186547524f) {
    e -= 1;
    m = (m + m) - 1.0f;
  } else {
    m = m - 1.0f;
  }
  const float z = m * m;
  float y = 7.0376836292e-2f;
  y = y * m + -1.1514610310e-1f;
  y = y * m + 1.1676998740e-1f;
  y = y * m + -1.2420140846e-1f;
  y = y * m + 1.4249322787e-1f;
  y = y * m + -1.6668057665e-1f;
  y = y * m + 2.0000714765e-1f;
  y = y * m + -2.4999993993e-1f;
  y = y * m + 3.3333331174e-1f;
  y = y * m;
  y = y * z;
  const float fe = (float)e;
  y = y + -2.12194440e-4f * fe;
  y = y + -0.5f * z;
  float r = m + y;
  r = r + 0.693359375f * fe;
  return r;
}

// ------------------------------------------------------------------ exp
// Cephes expf; DEFINED as 0 for x < -87 (keeps the 2^n scale a normal float).
MPPI_HD float dm_expf(float x) {
  if (x < -87.0f) return 0.0f;
  float t = 1.44269504088896341f * x;
  t = t + 0.5f;
  const float z = floorf(t);
  float r = x - z * 0.693359375f;
  r = r - z * -2.12194440e-4f;
  const int n = (int)z;
  const float zz = r * r;
  float p = 1.9875691500e-4f;
  p = p * r + 1.3981999507e-3f;
  p = p * r + 8.3334519073e-3f;
  p = p * r + 4.1665795894e-2f;
  p = p * r + 1.6666665459e-1f;
  p = p * r + 5.0000001201e-1f;
  float y = p * zz;
  y = y + r;
  y = y + 1.0f;
  return y * bits_f((uint32_t)(n + 127) << 23);
}

// ------------------------------------------------------------------ sincos
// Cephes sinf/cosf with a shared Cody-Waite reduction (accurate for |x| < 8192).
MPPI_HD void dm_sincosf(float x, float* s_out, float* c_out) {
  const float ax = fabsf(x);
  int j = (int)(ax * 1.27323954473516f);
  float y = (float)j;
  const bool odd = (j & 1) != 0;  // branch-free: selects, no divergent blocks
  j = odd ? j + 1 : j;
  y = odd ? y + 1.0f : y;
  j &= 7;
  float r = ax - y * 0.78515625f;
  r = r - y * 2.4187564849853515625e-4f;
  r = r - y * 3.77489497744594108e-8f;
  const float z = r * r;
  float ps = -1.9515295891e-4f * z;
  ps = ps + 8.3321608736e-3f;
  ps = ps * z;
  ps = ps + -1.6666654611e-1f;
  ps = ps * z;
  ps = ps * r;
  ps = ps + r;
  float pc = 2.443315711809948e-5f * z;
  pc = pc + -1.388731625493765e-3f;
  pc = pc * z;
  pc = pc + 4.166664568298827e-2f;
  pc = pc * z;
  pc = pc * z;
  pc = pc - 0.5f * z;
  pc = pc + 1.0f;
  // quadrant q = j/2: (sin, cos) = (ps, pc), (pc, -ps), (-ps, -pc), (-pc, ps)
  const bool swap = (j & 2) != 0;
  const float s0 = swap ? pc : ps;
  const float c0 = swap ? ps : pc;
  const bool sneg = (j & 4) != 0;
  const bool cneg = ((j >> 1) ^ (j >> 2)) & 1;
  const float s = sneg ? -s0 : s0;
  *s_out = (x < 0.0f) ? -s : s;
  *c_out = cneg ? -c0 : c0;
}

// dm_sincosf for |x| * 4/pi < 1 (quadrant 0), the same bits: there j = 0, the reduction subtracts
// exact zeros (r = |x|), no swap and no sign flips but sin's, and (poly * z) * x + x = -((poly * z)
// * |x| + |x|) for x < 0 (IEEE negation is exact): the Rodrigues angle w * dt of the rollout, with
// |w| <= max(|w_min|, |w_max|) and that bound times dt under pi/4 (RolloutArgs::small_angle).
MPPI_HD void dm_sincosf_small(float x, float* s_out, float* c_out) {
  const float z = x * x;
  float ps = -1.9515295891e-4f * z;
  ps = ps + 8.3321608736e-3f;
  ps = ps * z;
  ps = ps + -1.6666654611e-1f;
  ps = ps * z;
  ps = ps * x;
  ps = ps + x;
  float pc = 2.443315711809948e-5f * z;
  pc = pc + -1.388731625493765e-3f;
  pc = pc * z;
  pc = pc + 4.166664568298827e-2f;
  pc = pc * z;
  pc = pc * z;
  pc = pc - 0.5f * z;
  pc = pc + 1.0f;
  *s_out = ps;
  *c_out = pc;
}

// ------------------------------------------------------------------ Philox4x32-10
struct U4 {
  uint32_t x, y, z, w;
};

// a ^ b ^ c: one v_bitop3_b32 (truth table 0x96) on gfx950, which the compiler does not form itself
MPPI_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

MPPI_HD U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = U4{xor3(hi1, c.y, k0), lo1, xor3(hi0, c.w, k1), lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Two uint32 -> two N(0,1) float32 (Box-Muller, DEFINED op sequence).
MPPI_HD void dm_box_muller(uint32_t ra, uint32_t rb, float* z0, float* z1) {
  const float u = ((float)(ra >> 8) + 1.0f) * 5.9604644775390625e-8f;  // (0, 1]
  const float v = (float)(rb >> 8) * 5.9604644775390625e-8f;           // [0, 1)
  const float rad = sqrtf(-2.0f * dm_logf(u));
  float s, c;
  dm_sincosf(6.2831853071795864769f * v, &s, &c);
  *z0 = rad * c;
  *z1 = rad * s;
}

// ------------------------------------------------------------------ the two Box-Mullers of a block, packed
// The same op sequences as dm_logf / dm_sincosf / dm_box_muller on (ra, rb) and (rc, rd) side by side:
// every float product and sum of the pair is one packed FP32 instruction (v_pk_mul_f32 / v_pk_add_f32,
// IEEE per half, so each half's bits are the scalar sequence's); integer parts, square roots and the
// quadrant selects stay per half.  sincos: the argument 2 pi v is >= +0, where dm_sincosf's |x| and
// final sign flip are identities.  Bit-identical to noise_block (tests/test_noise_pack.py, host).
typedef float mf2 __attribute__((ext_vector_type(2)));

MPPI_HD mf2 dm_logf2(mf2 x) {
  const uint32_t b0 = f_bits(x.x), b1 = f_bits(x.y);
  int e0 = (int)((b0 >> 23) & 0xFFu) - 126, e1 = (int)((b1 >> 23) & 0xFFu) - 126;
  const mf2 m0 = mf2{bits_f((b0 & 0x807FFFFFu) | 0x3F000000u), bits_f((b1 & 0x807FFFFFu) | 0x3F000000u)};
  const mf2 lo = (m0 + m0) - 1.0f;
  const mf2 hi = m0 - 1.0f;
  const bool s0 = m0.x < 0.707106781186547524f, s1 = m0.y < 0.707106781186547524f;
  e0 -= s0 ? 1 : 0;
  e1 -= s1 ? 1 : 0;
  const mf2 m = mf2{s0 ? lo.x : hi.x, s1 ? lo.y : hi.y};
  const mf2 z = m * m;
  mf2 y = mf2{7.0376836292e-2f, 7.0376836292e-2f};
  y = y * m + -1.1514610310e-1f;
  y = y * m + 1.1676998740e-1f;
  y = y * m + -1.2420140846e-1f;
  y = y * m + 1.4249322787e-1f;
  y = y * m + -1.6668057665e-1f;
  y = y * m + 2.0000714765e-1f;
  y = y * m + -2.4999993993e-1f;
  y = y * m + 3.3333331174e-1f;
  y = y * m;
  y = y * z;
  const mf2 fe = mf2{(float)e0, (float)e1};
  y = y + -2.12194440e-4f * fe;
  y = y + -0.5f * z;
  mf2 r = m + y;
  r = r + 0.693359375f * fe;
  return r;
}

// dm_sincosf of x >= +0 in both halves
MPPI_HD void dm_sincosf2_pos(mf2 x, mf2* s_out, mf2* c_out) {
  const mf2 t = x * 1.27323954473516f;
  int j0 = (int)t.x, j1 = (int)t.y;
  j0 += j0 & 1;  // odd j up, and y = (float)j exactly as dm_sincosf's y + 1 (j < 2^24)
  j1 += j1 & 1;
  const mf2 y = mf2{(float)j0, (float)j1};
  mf2 r = x - y * 0.78515625f;
  r = r - y * 2.4187564849853515625e-4f;
  r = r - y * 3.77489497744594108e-8f;
  const mf2 z = r * r;
  mf2 ps = -1.9515295891e-4f * z;
  ps = ps + 8.3321608736e-3f;
  ps = ps * z;
  ps = ps + -1.6666654611e-1f;
  ps = ps * z;
  ps = ps * r;
  ps = ps + r;
  mf2 pc = 2.443315711809948e-5f * z;
  pc = pc + -1.388731625493765e-3f;
  pc = pc * z;
  pc = pc + 4.166664568298827e-2f;
  pc = pc * z;
  pc = pc * z;
  pc = pc - 0.5f * z;
  pc = pc + 1.0f;
  // the sign flips as sign-bit xors (IEEE negation): bit 2 of j for sin; for cos (j >> 1 ^ j >> 2) & 1,
  // which for even j is bit 2 of j + 2
  auto quad = [](int j, float ps_, float pc_, float* so, float* co) {
    const bool swap = (j & 2) != 0;
    const float s0 = swap ? pc_ : ps_;
    const float c0 = swap ? ps_ : pc_;
    *so = bits_f(f_bits(s0) ^ (((uint32_t)j << 29) & 0x80000000u));
    *co = bits_f(f_bits(c0) ^ (((uint32_t)j + 2u) << 29 & 0x80000000u));
  };
  float sa, ca, sb, cb;
  quad(j0, ps.x, pc.x, &sa, &ca);
  quad(j1, ps.y, pc.y, &sb, &cb);
  *s_out = mf2{sa, sb};
  *c_out = mf2{ca, cb};
}

// sqrtf of the Box-Muller radius argument -2 log(u), in {-0, +0} U [2^-24, 34]: on the device
// v_sqrt_f32 (within 1 ulp) and the neighbour residual test, correctly rounded there without
// hipcc's denormal scaling and class tests (-0: the down-neighbour is a NaN, whose compare is
// false, so -0 stays -0 as IEEE sqrt gives it)
MPPI_HD float sqrt_bm(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float s = __builtin_amdgcn_sqrtf(x);
  const uint32_t si = f_bits(s);
  const float sdn = bits_f(si - 1u), sup = bits_f(si + 1u);
  const float out = (__builtin_fmaf(-sdn, s, x) <= 0.0f) ? sdn : s;
  return (__builtin_fmaf(-sup, s, x) > 0.0f) ? sup : out;
#else
  return sqrtf(x);
#endif
}

MPPI_HD void noise_block_pk(uint64_t seed, uint64_t n, uint64_t k, float* a1, float* a2, float* b1, float* b2) {
  const U4 r = philox4x32_10(U4{(uint32_t)n, (uint32_t)(n >> 32), (uint32_t)k, (uint32_t)(k >> 32)},
                             (uint32_t)seed, (uint32_t)(seed >> 32));
  const mf2 u = (mf2{(float)(r.x >> 8), (float)(r.z >> 8)} + 1.0f) * 5.9604644775390625e-8f;
  const mf2 v = mf2{(float)(r.y >> 8), (float)(r.w >> 8)} * 5.9604644775390625e-8f;
  const mf2 l = -2.0f * dm_logf2(u);
  const mf2 rad = mf2{sqrt_bm(l.x), sqrt_bm(l.y)};
  mf2 s, c;
  dm_sincosf2_pos(6.2831853071795864769f * v, &s, &c);
  const mf2 zc = rad * c, zs = rad * s;
  *a1 = zc.x;
  *a2 = zs.x;
  *b1 = zc.y;
  *b2 = zs.y;
}

// Noise block n of trajectory k: e1[t], e2[t], e1[t+1], e2[t+1] (t = 2(n mod ceil(H/2))).
MPPI_HD void noise_block(uint64_t seed, uint64_t n, uint64_t k, float* a1, float* a2, float* b1,
                         float* b2) {
  const U4 r = philox4x32_10(U4{(uint32_t)n, (uint32_t)(n >> 32), (uint32_t)k, (uint32_t)(k >> 32)},
                             (uint32_t)seed, (uint32_t)(seed >> 32));
  dm_box_muller(r.x, r.y, a1, a2);
  dm_box_muller(r.z, r.w, b1, b2);
}

}  // namespace mppi
