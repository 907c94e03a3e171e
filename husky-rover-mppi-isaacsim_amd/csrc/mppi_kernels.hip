// MI355X (gfx950) MPPI rollout-and-cost engine: kernels.
//
// One MPPI step (reference: thesis_master/warp_implementation/MPPI_isaac.py:505-720,
// nine Warp launches) runs here as:
//
//   mppi_rollout_pair_kernel (#1-#7 fused)  256 trajectories per workgroup: chain waves
//       run the serial 2.5D projection, side waves the sampling, wheel filter, wheel
//       contacts and the four critics, paired through LDS rings; then the workgroup's
//       softmax leaf record (min, sum w, sum w*u[t]) in float64.
//   mppi_colfin_kernel (#7-#9)  column-split tree over the records, u_opt = V/S, the
//       optimal-sequence filter and the first optimal-rollout step; outputs to host memory.
//   mppi_tail_kernel  the rest of the optimal rollout, on a side stream.
//   mppi_noise_kernel the Philox sampling normals, two steps ahead, on a side stream.
// mppi_finish_kernel (the record tree) is the finish where the column split does not fit
// (mppi_set_option "record_tree_finish" selects it everywhere).
//
// Numerics: compile with -ffp-contract=off.  Every float op is one IEEE f32
// operation in the reference's source order; transcendentals come from
// mppi_detmath.h.  oracle/mppi_ref.py restates the same sequence in numpy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <stdint.h>

#include "mppi_detmath.h"
#include "mppi_kernels.h"

namespace mppi {

// =====================================================================  exact f32 division / sqrt
// Every division and square root of a rollout-step is correctly rounded (IEEE
// binary32, round to nearest even).  Two implementations, selected by the
// template flag F:
//   F = false  the IEEE operators `/` and sqrtf (hipcc's generic expansions);
//   F = true   fast paths that are bit-identical on a checked operand range:
//     division: v_rcp_f32, one Newton step on the reciprocal (y), q0 = a y and ONE
//       fma residual correction q1 = q0 + (a - b q0) y (Markstein); LLVM's fdiv
//       expansion applies a second correction and the v_div_scale / v_div_fixup
//       steps, which are the identity when |a|, |b| lie in [2^-40, 2^40] (a = +-0
//       handled by a select).  q1 equals the IEEE quotient for EVERY pair of
//       significands (2^46 pairs, exhaustive, on MI355X: profiles/ubench/div1_check.hip,
//       profiles/r04_div1_check.txt), and exponents scale all of it exactly in that
//       range.  The refined reciprocal is shared by all quotients with one divisor
//       and needs no VCC;
//     sqrt: LLVM's expansion (v_sqrt_f32 + one-ulp fma correction) without the
//       small-input scaling, valid for x = 0 or x in [2^-96, 2^128).
// A fast-path rollout-step ORs "operand outside its range" into a per-lane
// flag; a flagged lane recomputes the whole step with F = false, so results
// never depend on the path.  mppi_selftest() checks the fast paths bitwise.
// kFastMath selects the fast paths in the rollout-steps.  Measured on MI355X
// (C3, profiles/r01_*): the range guards cost about what the shorter sequences
// save (rollout kernel 287 us fast vs 250 us IEEE), so the IEEE path is the default.
constexpr bool kFastMath = false;
// The serial chain (chain3d) of the warp-specialised rollout and of the optimal
// rollout is latency-bound: there the VCC-free fast division (three quotients of
// a normalisation in parallel instead of serialised through VCC) shortens the
// dependency chain, and its range guards are off the critical path.
constexpr bool kChainFast = true;

struct Recip {
  float b, y;
};
__device__ __forceinline__ bool div_ok(float v) {
  const float a = fabsf(v);
  return a >= 9.094947017729282e-13f && a <= 1.099511627776e12f;  // 2^-40 .. 2^40
}
template <bool F>
__device__ __forceinline__ Recip rc(float b, bool& bad) {
  Recip r;
  r.b = b;
  r.y = 0.0f;
  if constexpr (F) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    r.y = __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
    bad |= !div_ok(b);
  }
  return r;
}
template <bool F>
__device__ __forceinline__ float dv(float a, const Recip& r, bool& bad) {
  if constexpr (!F) {
    return a / r.b;
  } else {
    const float q0 = a * r.y;
    const float e0 = __builtin_fmaf(-r.b, q0, a);
    const float q1 = __builtin_fmaf(e0, r.y, q0);
    const bool zero = (a == 0.0f);
    bad |= !(zero || div_ok(a));
    return zero ? q0 : q1;  // q0 = a*y carries the IEEE sign of a zero quotient
  }
}
template <bool F>
__device__ __forceinline__ float dv1(float a, float b, bool& bad) {
  return dv<F>(a, rc<F>(b, bad), bad);
}
// Measured on MI355X (profiles/ubench/lat.hip): the IEEE sqrt expansion has the
// shorter dependent latency (144 vs 158 cycles), so sq() uses it on both paths.
constexpr bool kFastSqrt = false;
template <bool F>
__device__ __forceinline__ float sq(float x, bool& bad) {
  if constexpr (!F || !kFastSqrt) {
    return sqrtf(x);
  } else {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __builtin_bit_cast(float, __builtin_bit_cast(int, s) - 1);
    const float sup = __builtin_bit_cast(float, __builtin_bit_cast(int, s) + 1);
    const float rdn = __builtin_fmaf(-sdn, s, x);
    const float rup = __builtin_fmaf(-sup, s, x);
    float out = (rdn <= 0.0f) ? sdn : s;
    out = (rup > 0.0f) ? sup : out;
    bad |= !(x == 0.0f || (x >= 1.2621774483536189e-29f && x <= 3.4e38f));  // 2^-96
    return out;
  }
}

// Division by a launch constant b for quotients that are only truncated to a grid
// index: y = 1/b rounded, q = q0 + (a - q0*b)*y (Markstein's correction).  The
// host accepts y only after launch_cdiv_verify found the result equal to the IEEE
// quotient for every significand a in [1, 2); by scaling that covers every a
// whose quotient has magnitude in [2^-100, 2^126], and a smaller quotient
// truncates to 0 on both paths.  3 VALU ops instead of the ~10-op IEEE expansion.
__device__ __forceinline__ float cdiv_f(float a, float b, float y) {
  const float q0 = a * y;
  const float r = __builtin_fmaf(-q0, b, a);
  return __builtin_fmaf(r, y, q0);
}

// =====================================================================  grid lookups
// projection_warp.py:39-40 / :338-339 — C-style truncation; clamping is DEFINED
// here (the reference reads out of bounds).
__device__ __forceinline__ int trunc_clamped(float f, float lo, float hi) {
  return (int)fminf(fmaxf(f, lo), hi);
}
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

struct Dem {
  const float* Z;    // global DEM (row-major rows x grid)
  int rows, grid;
  float x_min, y_min, res;
  Recip rres;  // fast-path reciprocal of res (res is validated on the host)
  float rinv;  // verified reciprocal for cdiv_f (cdiv != 0)
  int cdiv;
  const float4* N = nullptr;  // per-cell normals (normal_cell), global path only

  __device__ __forceinline__ void init(const float* Z_, int rows_, int grid_, float x_min_, float y_min_,
                                       float res_, float rinv_ = 0.0f, int cdiv_ = 0) {
    rinv = rinv_;
    cdiv = cdiv_;
    Z = Z_;
    rows = rows_;
    grid = grid_;
    x_min = x_min_;
    y_min = y_min_;
    res = res_;
    bool unused = false;
    rres = rc<true>(res_, unused);
  }
  template <bool F>
  __device__ __forceinline__ Recip rr() const {
    Recip r = rres;
    if constexpr (!F) r.b = res;
    return r;
  }
  template <bool F>
  __device__ __forceinline__ void cell(float x, float y, int& i, int& j, bool& bad) const {
    float fi, fj;
    if (cdiv) {  // uniform branch
      fi = cdiv_f(x - x_min, res, rinv);
      fj = cdiv_f(y + y_min, res, rinv);
    } else {
      fi = dv<F>(x - x_min, rr<F>(), bad);
      fj = dv<F>(y + y_min, rr<F>(), bad);
    }
    i = trunc_clamped(fi, -1.0f, (float)grid);
    j = -trunc_clamped(fj, -(float)rows, 1.0f);
  }
  __device__ __forceinline__ float at(int row, int col) const {
    row = clampi(row, 0, rows - 1);
    col = clampi(col, 0, grid - 1);
    return Z[(size_t)row * grid + col];
  }
  // projection_warp.py:8-48
  template <bool F>
  __device__ __forceinline__ void corners(float x, float y, float (&q)[4], bool& bad) const {
    int i, j;
    cell<F>(x, y, i, j, bad);
    const int r0 = clampi(j, 0, rows - 1), r1 = clampi(j + 1, 0, rows - 1);
    const int c0 = clampi(i, 0, grid - 1), c1 = clampi(i + 1, 0, grid - 1);
    q[0] = Z[(size_t)r0 * grid + c0];
    q[1] = Z[(size_t)r0 * grid + c1];
    q[2] = Z[(size_t)r1 * grid + c0];
    q[3] = Z[(size_t)r1 * grid + c1];
  }
  // normal of the cell (i, j) from the table: i in [-1, grid], j in [-1, rows] as cell()
  // returns them; i = grid selects the same corners as i = grid - 1 (both clamp to the last
  // column), so the table has (rows + 1) x (grid + 1) entries
  __device__ __forceinline__ float4 normal_cell(int i, int j) const {
    const int ii = min(i, grid - 1) + 1, jj = min(j, rows - 1) + 1;
    return N[(uint32_t)(jj * (grid + 1) + ii)];
  }
  // cell() + at() in two instructions per index: clamp(trunc(clamp(f, -1, grid)), 0, grid - 1)
  // == trunc(med3(f, 0, grid - 1)) and clamp(-trunc(clamp(f, -rows, 1)), 0, rows - 1)
  // == -trunc(med3(f, 1 - rows, 0)); a NaN lands on the same bound (v_med3_f32 with a NaN
  // operand returns the min3 of the others)
  template <bool F>
  __device__ __forceinline__ float point(float x, float y, bool& bad) const {
    float fi, fj;
    if (cdiv) {  // uniform branch
      fi = cdiv_f(x - x_min, res, rinv);
      fj = cdiv_f(y + y_min, res, rinv);
    } else {
      fi = dv<F>(x - x_min, rr<F>(), bad);
      fj = dv<F>(y + y_min, rr<F>(), bad);
    }
    const int col = (int)__builtin_amdgcn_fmed3f(fi, 0.0f, (float)(grid - 1));
    const int row = -(int)__builtin_amdgcn_fmed3f(fj, (float)(1 - rows), 0.0f);
    return Z[(size_t)row * grid + col];
  }
};

// projection_warp.py:70-100 (trunc; x-fraction paired with the row neighbour q10)
template <bool F>
__device__ __forceinline__ float bilinear(float x, float y, const float (&q)[4], const Recip& rres,
                                          bool& bad) {
  const float xn = dv<F>(x, rres, bad), yn = dv<F>(y, rres, bad);
  const float x2 = xn - truncf(xn), y2 = yn - truncf(yn);
  const float a = ((1.0f - x2) * (1.0f - y2)) * q[0];
  const float b = (x2 * (1.0f - y2)) * q[2];
  const float c = ((1.0f - x2) * y2) * q[1];
  const float d = (x2 * y2) * q[3];
  return ((a + b) + c) + d;
}

__device__ __forceinline__ float clampf(float x, float lo, float hi) {
  return fminf(fmaxf(x, lo), hi);
}

// =====================================================================  one rollout-step
struct Traj {                 // state of one trajectory between steps
  float x, y;                 // position[tid]
  float hx, hy, hz;           // `previous` heading
};

struct StepOut {
  float z;                         // trajectory height
  float lx, ly, lz, rx, ry, rz;    // wheel points
};

// Serial part of one 3D rollout-step (projection_warp.py:314-326): position
// update, corner lookup, normal, tangent projection, Rodrigues yaw.  (sn, cs)
// = dm_sincosf(w*dt).  Leaves the new heading in s and the quad / normal in q, n.
template <bool F>
__device__ __forceinline__ void chain3d(const Dem& dem, float res_half_neg, float res_sq,
                                        float dt, float v, float sn, float cs, Traj& s,
                                        float (&q)[4], float& nx, float& ny, float& nz, bool& bad) {
  {  // _update_position :207-223
    const Recip r = rc<F>(sq<F>((s.hx * s.hx + s.hy * s.hy) + s.hz * s.hz, bad), bad);
    const float ux = dv<F>(s.hx, r, bad), uy = dv<F>(s.hy, r, bad);
    s.x = s.x + (ux * v) * dt;
    s.y = s.y + (uy * v) * dt;
  }
  dem.template corners<F>(s.x, s.y, q, bad);
  {  // _normal_on_grid :129-151
    const float vx = res_half_neg * (((q[1] - q[0]) - q[2]) + q[3]);
    const float vy = res_half_neg * (((q[2] - q[0]) - q[1]) + q[3]);
    const Recip r = rc<F>(sq<F>((vx * vx + vy * vy) + res_sq * res_sq, bad), bad);
    nx = dv<F>(vx, r, bad);
    ny = dv<F>(vy, r, bad);
    nz = dv<F>(res_sq, r, bad);
  }
  float tx, ty, tz;
  {  // _get_heading_tangent_vector :168-190
    const float d = (s.hx * nx + s.hy * ny) + s.hz * nz;
    tx = s.hx - d * nx;
    ty = s.hy - d * ny;
    tz = s.hz - d * nz;
    const Recip r = rc<F>(sq<F>((tx * tx + ty * ty) + tz * tz, bad), bad);
    tx = dv<F>(tx, r, bad);
    ty = dv<F>(ty, r, bad);
    tz = dv<F>(tz, r, bad);
  }
  {  // _update_orientation :225-248 (Rodrigues about n)
    const Recip ro = rc<F>(sq<F>((tx * tx + ty * ty) + tz * tz, bad), bad);
    const float ox = dv<F>(tx, ro, bad), oy = dv<F>(ty, ro, bad), oz = dv<F>(tz, ro, bad);
    const float crx = ny * oz - nz * oy, cry = nz * ox - nx * oz, crz = nx * oy - ny * ox;
    const float dn = (nx * ox + ny * oy) + nz * oz;
    const float omc = 1.0f - cs;
    const float rx = (ox * cs + crx * sn) + (nx * dn) * omc;
    const float ry = (oy * cs + cry * sn) + (ny * dn) * omc;
    const float rz = (oz * cs + crz * sn) + (nz * dn) * omc;
    const Recip r = rc<F>(sq<F>((rx * rx + ry * ry) + rz * rz, bad), bad);
    s.hx = dv<F>(rx, r, bad);
    s.hy = dv<F>(ry, r, bad);
    s.hz = dv<F>(rz, r, bad);
  }
}

// ---------------------------------------------------------------------  lean guards
// A chain wave issues about one instruction per ~5 cycles on its own, so its step time is mostly
// instruction count.  The chains (chain_wave_3d, tail_chain_3d) compute the values of chain3d<true>
// with fewer instructions:
//  * range guards folded into running extrema instead of a compare-and-OR per
//    operand: the smallest frexp exponent over the numerators (a zero numerator
//    has exponent 0 and passes) and the min / max bit pattern of the squared
//    norms (non-negative floats order like ints; +NaN and inf land above the
//    upper bound, -NaN below the lower one);
//  * divisor = a norm, so the quotient's sign is the numerator's: copysign
//    replaces the zero-numerator select;
//  * sqrt of a norm in [2^-80, 2^80] needs no denormal scaling or class fix-up:
//    hardware sqrt (1 ulp) + the neighbour residual test (correctly rounded).
// In range: numerators zero or |a| >= 2^-80, squared norms in [2^-80, 2^80] (so
// divisors in [2^-40, 2^40] and every quotient / residual normal).  A lane out
// of range redoes the step with chain3d<false> (IEEE), so results never depend
// on the path; mppi_selftest (what 2, 3) checks the primitives bitwise.
struct Lean {
  int emin;      // min frexp exponent of the numerators
  int nlo, nhi;  // min / max bit pattern of the squared norms
  int n1lo = 0x3F800000, n1hi = 0x3F800000;  // ... of the squared norms of unit vectors (sqrt_near1)
  int emin40 = 0;  // min frexp exponent of the numerators guarded at 2^-40 (orient_step, see there)
};
constexpr int kLeanEmin = -79;          // |a| >= 2^-80 <=> frexp exponent >= -79
constexpr int kLeanNlo = 0x17800000;    // 2^-80
constexpr int kLeanNhi = 0x67800000;    // 2^80
__device__ __forceinline__ void lean_init(Lean& l) {
  l.emin = 0;
  l.nlo = kLeanNhi;
  l.nhi = kLeanNlo;
}
constexpr int kNear1 = 4095;  // sqrt_near1: squared norms within 4095 ulps of 1
constexpr int kLeanEmin40 = -39;  // |a| >= 2^-40 <=> frexp exponent >= -39
__device__ __forceinline__ bool lean_bad(const Lean& l) {
  return (l.emin < kLeanEmin) | (l.nlo < kLeanNlo) | (l.nhi > kLeanNhi) | (l.n1lo < 0x3F800000 - kNear1) |
         (l.n1hi > 0x3F800000 + kNear1) | (l.emin40 < kLeanEmin40);
}
// correctly rounded sqrt of a normal positive n (neighbour residual test)
__device__ __forceinline__ float sqrt_cr(float n) {
  const float s = __builtin_amdgcn_sqrtf(n);
  const int si = __builtin_bit_cast(int, s);
  const float sdn = __builtin_bit_cast(float, si - 1), sup = __builtin_bit_cast(float, si + 1);
  const float rdn = __builtin_fmaf(-sdn, s, n);
  const float rup = __builtin_fmaf(-sup, s, n);
  float out = (rdn <= 0.0f) ? sdn : s;
  return (rup > 0.0f) ? sup : out;
}
// 1 / sqrt(n) setup for the quotients a / sqrt(n) (IEEE: sqrt rounded, then each division)
__device__ __forceinline__ Recip lean_norm(float n, Lean& l) {
  const int nb = __builtin_bit_cast(int, n);
  l.nlo = min(l.nlo, nb);
  l.nhi = max(l.nhi, nb);
  Recip r;
  r.b = sqrt_cr(n);
  const float y0 = __builtin_amdgcn_rcpf(r.b);
  r.y = __builtin_fmaf(__builtin_fmaf(-r.b, y0, 1.0f), y0, y0);
  return r;
}
__device__ __forceinline__ float lean_div(float a, const Recip& r, Lean& l) {
  l.emin = min(l.emin, __builtin_amdgcn_frexp_expf(a));
  const float q0 = a * r.y;
  const float e0 = __builtin_fmaf(-r.b, q0, a);
  return __builtin_copysignf(__builtin_fmaf(e0, r.y, q0), a);
}

// ---------------------------------------------------------------------  packed chain (roles kernel)
// The role-split kernel's chain wave is bound by its own instruction issue (one wave issues
// about one instruction per 5 cycles, whatever its type), so the serial step is written with
// packed-FP32 instructions (v_pk_mul / v_pk_add / v_pk_fma: the x and y components in one
// instruction, each lane an ordinary IEEE f32 operation, results unchanged) wherever the
// reference computes the same operation on x and y.  Range guards (Lean) and the IEEE redo as
// above.
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 bc2(float s) { return f2{s, s}; }
// [x > 0] for an int x in one v_med3_i32 (written out: the compiler rewrites min(max(x, 0), 1)
// into a compare + select pair, which also costs VCC wait states)
__device__ __forceinline__ int pos01(int x) {
  int r;
  asm("v_med3_i32 %0, %1, 0, 1" : "=v"(r) : "v"(x));
  return r;
}

// sqrt_cr without compares: sqrt_cr = sdn + [rdn > 0] + [rup > 0] (rdn <= 0 < rup is
// impossible: sdn < sup), and a residual n - x*s is exactly zero only as +0, so [r > 0] is
// med3(bits(r), 0, 1) on its bit pattern as an integer (pos01: one instruction, no VCC, no
// wait states).  The residuals stay two scalar fmas: with the lanes of a packed fma bit-cast to
// integers this compiler (ROCm 7.2 LLVM) folded lane 1's test onto lane 0's.
__device__ __forceinline__ float sqrt_cr2(float n) {
  const float s = __builtin_amdgcn_sqrtf(n);
  const int si = __builtin_bit_cast(int, s);
  const float sdn = __builtin_bit_cast(float, si - 1), sup = __builtin_bit_cast(float, si + 1);
  const float rdn = __builtin_fmaf(-sdn, s, n);
  const float rup = __builtin_fmaf(-sup, s, n);
  return __builtin_bit_cast(float, (si - 1) + pos01(__builtin_bit_cast(int, rdn)) +
                                       pos01(__builtin_bit_cast(int, rup)));
}
// Correctly rounded sqrt of the squared norm of a vector that is already unit up to rounding
// (the reference normalises the tangent and the rotated heading twice).  With n = 1 + k 2^-23
// (k >= 0) sqrt(n) = 1 + k 2^-24 - k^2 2^-49 + ..., with n = 1 - k 2^-24 it is 1 - k 2^-25 -
// k^2 2^-51 - ...: for |k| < 5792 the quadratic term never crosses a rounding boundary (even k:
// it stays within half an ulp of the grid point, odd k: it moves the midpoint down), so
// RN(sqrt(n)) = 1 + floor(k / 2) ulp above 1, 1 - ceil(k / 2) ulp below: in bits,
// C + ((bits(n) - C) >> 1) = (bits(n) + C) >> 1 with C = bits(1.0f).  Guarded to |k| <= 4095.
__device__ __forceinline__ Recip lean_norm_near1(float n, Lean& l) {
  const int nb = __builtin_bit_cast(int, n);
  l.n1lo = min(l.n1lo, nb);
  l.n1hi = max(l.n1hi, nb);
  Recip r;
  r.b = __builtin_bit_cast(float, (int)((unsigned)(nb + 0x3F800000) >> 1));
  const float y0 = __builtin_amdgcn_rcpf(r.b);
  r.y = __builtin_fmaf(__builtin_fmaf(-r.b, y0, 1.0f), y0, y0);
  return r;
}
// lean_norm_near1 for a squared norm PROVEN within 4095 ulps of 1 (no guard; see orient_step)
__device__ __forceinline__ Recip norm_near1_trusted(float n) {
  const int nb = __builtin_bit_cast(int, n);
  Recip r;
  r.b = __builtin_bit_cast(float, (int)((unsigned)(nb + 0x3F800000) >> 1));
  const float y0 = __builtin_amdgcn_rcpf(r.b);
  r.y = __builtin_fmaf(__builtin_fmaf(-r.b, y0, 1.0f), y0, y0);
  return r;
}
__device__ __forceinline__ Recip lean_norm2(float n, Lean& l) {
  const int nb = __builtin_bit_cast(int, n);
  l.nlo = min(l.nlo, nb);
  l.nhi = max(l.nhi, nb);
  Recip r;
  r.b = sqrt_cr2(n);
  const float y0 = __builtin_amdgcn_rcpf(r.b);
  r.y = __builtin_fmaf(__builtin_fmaf(-r.b, y0, 1.0f), y0, y0);
  return r;
}
// a / r.b without the sign fix-up: the residuals are formed negated, E = b q - a (= -(a - b q)
// exactly, round-to-nearest is symmetric), and subtracted, q' = q - E y.  For a != 0 that is
// lean_div's sequence; for a = +-0 every intermediate is a zero and q0 = a y, q' = (-E) y + q
// keep the sign of a (lean_div needed a copysign there).
__device__ __forceinline__ float lean_div_s(float a, const Recip& r, Lean& l) {
  l.emin = min(l.emin, __builtin_amdgcn_frexp_expf(a));
  const float q0 = a * r.y;
  const float e0 = __builtin_fmaf(r.b, q0, -a);
  return __builtin_fmaf(-e0, r.y, q0);
}
// (a.x, a.y) / r.b, each lane lean_div_s (G = 0: numerators proven in range, no guard)
template <int G = 1>
__device__ __forceinline__ f2 lean_div2(f2 a, const Recip& r, Lean& l) {
  if constexpr (G == 1) l.emin = min(l.emin, min(__builtin_amdgcn_frexp_expf(a.x), __builtin_amdgcn_frexp_expf(a.y)));
  const f2 b = bc2(r.b), y = bc2(r.y);
  const f2 q0 = a * y;
  const f2 e0 = pk_fma(b, q0, -a);
  return pk_fma(-e0, y, q0);
}
// (a.x, a.y, az) / r.b: lean_div2 and lean_div_s with their dependent steps interleaved, so the
// scalar chain's instructions fill the wait states between the packed chain's dependent steps
// (same operations, same results).  G: 0 = numerators proven in range (no guard), 1 = guarded at
// 2^-80 (emin), 2 = guarded at 2^-40 (emin40).
template <int G = 1>
__device__ __forceinline__ void lean_div3(f2 a, float az, const Recip& r, Lean& l, f2& qxy, float& qz) {
  if constexpr (G == 1)
    l.emin = min(l.emin, min(min(__builtin_amdgcn_frexp_expf(a.x), __builtin_amdgcn_frexp_expf(a.y)),
                             __builtin_amdgcn_frexp_expf(az)));
  if constexpr (G == 2)
    l.emin40 = min(l.emin40, min(min(__builtin_amdgcn_frexp_expf(a.x), __builtin_amdgcn_frexp_expf(a.y)),
                                 __builtin_amdgcn_frexp_expf(az)));
  const f2 b = bc2(r.b), y = bc2(r.y);
  const f2 q0 = a * y;
  const float q0z = az * r.y;
  const f2 e0 = pk_fma(b, q0, -a);
  const float e0z = __builtin_fmaf(r.b, q0z, -az);
  qxy = pk_fma(-e0, y, q0);
  qz = __builtin_fmaf(-e0z, r.y, q0z);
}
// cross(n, o).xy = (ny oz - nz oy, nz ox - nx oz), as (ny oz, -nx oz) + (-nz oy, nz ox)
__device__ __forceinline__ f2 cross_xy(f2 nxy, float nz, f2 oxy, float oz) {
  const f2 p1 = nxy.yx * f2{oz, -oz};
  const f2 p2 = f2{-nz, nz} * oxy.yx;
  return p1 + p2;
}

struct Head {  // heading vector (x, y packed)
  f2 xy;
  float z;
};

// _get_heading_tangent_vector + _update_orientation (projection_warp.py:168-248): the new heading
// from the previous one, the surface normal n and sin / cos / (1 - cos) of w dt.
// Guards of the fast path (F): only the two vectors that can come out arbitrary are checked,
//   p = h - (h.n) n: every component 0 or |.| >= 2^-40, |p|^2 in [2^-80, 2^80];
//   r (the Rodrigues rotation): every component 0 or |.| >= 2^-40, |r|^2 within 4095 ulps of 1.
// The rest follows.  t = p / |p| has components 0 or >= 2^-40 / 2^40 = 2^-80 (the quotient guard),
// and with p's quotients exact |t|^2 = 1 + e, |e| <= ~14 ulps (3-term sum of squares of correctly
// rounded quotients by a correctly rounded square root of a 3-term sum: ~5u + 2u + 3u + 2u), so
// the second normalisation needs no guard.  Likewise the new heading h' = r / |r| has components
// 0 or >= 2^-41 and |h'|^2 within ~14 ulps of 1: the next position update (advance_step<true,
// false>) needs no guard either.  Out of range -> the caller redoes the step with IEEE operators.
template <bool F>
__device__ __forceinline__ Head orient_step(f2 nxy, float nz, const Head& h, float sn, float cs, float omc,
                                           Lean& l) {
  const f2 hn = h.xy * nxy;
  const float d = (hn.x + hn.y) + h.z * nz;
  const f2 pxy = h.xy - bc2(d) * nxy;
  const float pz = h.z - d * nz;
  f2 txy, oxy;
  float tz, oz;
  if constexpr (F) {
    const f2 p2 = pxy * pxy;
    const Recip r = lean_norm2((p2.x + p2.y) + pz * pz, l);
    lean_div3<2>(pxy, pz, r, l, txy, tz);
    const f2 t2 = txy * txy;
    const Recip ro = norm_near1_trusted((t2.x + t2.y) + tz * tz);
    lean_div3<0>(txy, tz, ro, l, oxy, oz);
  } else {
    const float pn = sqrtf((pxy.x * pxy.x + pxy.y * pxy.y) + pz * pz);
    txy = f2{pxy.x / pn, pxy.y / pn};
    tz = pz / pn;
    const float tn = sqrtf((txy.x * txy.x + txy.y * txy.y) + tz * tz);
    oxy = f2{txy.x / tn, txy.y / tn};
    oz = tz / tn;
  }
  const f2 cxy = cross_xy(nxy, nz, oxy, oz);
  const f2 cz2 = nxy * oxy.yx;
  const float crz = cz2.x - cz2.y;
  const f2 no = nxy * oxy;
  const float dn = (no.x + no.y) + nz * oz;
  const f2 rxy = (oxy * bc2(cs) + cxy * bc2(sn)) + (nxy * bc2(dn)) * bc2(omc);
  const float rz = (oz * cs + crz * sn) + (nz * dn) * omc;
  Head o;
  if constexpr (F) {
    const f2 r2 = rxy * rxy;
    const Recip r = lean_norm_near1((r2.x + r2.y) + rz * rz, l);
    lean_div3<2>(rxy, rz, r, l, o.xy, o.z);
  } else {
    const float rn = sqrtf((rxy.x * rxy.x + rxy.y * rxy.y) + rz * rz);
    o.xy = f2{rxy.x / rn, rxy.y / rn};
    o.z = rz / rn;
  }
  return o;
}
// _update_position (projection_warp.py:207-223): pos + normalize(h).xy * v * dt
// GUARD = false: h is the heading a fast-path orient_step just produced (its guards cover this
// normalisation, see orient_step).
template <bool F, bool GUARD = true>
__device__ __forceinline__ f2 advance_step(const Head& h, float v, float dt, f2 pos, Lean& l) {
  f2 u;
  if constexpr (F) {
    const f2 h2 = h.xy * h.xy;
    if constexpr (GUARD) {
      const Recip r = lean_norm_near1((h2.x + h2.y) + h.z * h.z, l);
      u = lean_div2(h.xy, r, l);
    } else {
      const Recip r = norm_near1_trusted((h2.x + h2.y) + h.z * h.z);
      u = lean_div2<0>(h.xy, r, l);
    }
  } else {
    const float hn = sqrtf((h.xy.x * h.xy.x + h.xy.y * h.xy.y) + h.z * h.z);
    u = f2{h.xy.x / hn, h.xy.y / hn};
  }
  return pos + (u * bc2(v)) * bc2(dt);
}

// Height and wheel contacts of a rollout-step (projection_warp.py:318, :333-348),
// right = offset * cross(normal, current_hv).
template <bool F>
__device__ __forceinline__ void wheels3d(const Dem& dem, float off, float x, float y,
                                         const float (&q)[4], float nx, float ny, float nz,
                                         float hx, float hy, float hz, StepOut& o, bool& bad) {
  o.z = bilinear<F>(x, y, q, dem.template rr<F>(), bad);
  const float cx = off * (ny * hz - nz * hy);
  const float cy = off * (nz * hx - nx * hz);
  o.lx = x + cx;
  o.ly = y + cy;
  o.lz = dem.template point<F>(o.lx, o.ly, bad);
  o.rx = x - cx;
  o.ry = y - cy;
  o.rz = dem.template point<F>(o.rx, o.ry, bad);
}

// 2D step: projection_warp.py:373-382 (wheels DEFINED as zero).
template <bool F>
__device__ __forceinline__ void step2d(const Dem& dem, float dt, float v, float sn, float cs,
                                       Traj& s, StepOut& o, bool& bad) {
  {
    const Recip r = rc<F>(sq<F>((s.hx * s.hx + s.hy * s.hy) + s.hz * s.hz, bad), bad);
    const float ux = dv<F>(s.hx, r, bad), uy = dv<F>(s.hy, r, bad);
    s.x = s.x + (ux * v) * dt;
    s.y = s.y + (uy * v) * dt;
  }
  {  // _update_orientation_2D :251-275
    float nx = cs * s.hx - sn * s.hy;
    float ny = sn * s.hx + cs * s.hy;
    const float nrm = sq<F>(nx * nx + ny * ny, bad);
    if (nrm > 0.0f) {
      const Recip r = rc<F>(nrm, bad);
      nx = dv<F>(nx, r, bad);
      ny = dv<F>(ny, r, bad);
    }
    s.hx = nx;
    s.hy = ny;
    s.hz = 0.0f;
  }
  float q[4];
  dem.template corners<F>(s.x, s.y, q, bad);
  o.z = bilinear<F>(s.x, s.y, q, dem.template rr<F>(), bad);
  o.lx = o.ly = o.lz = o.rx = o.ry = o.rz = 0.0f;
}

// critics_warp.py:190-218, term for points (t, t+2) of both wheels.
template <bool F>
__device__ __forceinline__ float slope_term(float plx, float ply, float plz, float clx, float cly,
                                            float clz, float prx, float pry, float prz, float crx,
                                            float cry, float crz, bool& bad) {
  const float eps = 1e-6f;
  const float dzl = clz - plz;
  const float dxl = clx - plx, dyl = cly - ply;
  const float dl = sq<F>(dxl * dxl + dyl * dyl, bad);
  const float dzr = crz - prz;
  const float dxr = crx - prx, dyr = cry - pry;
  const float dr = sq<F>(dxr * dxr + dyr * dyr, bad);
  const float ratl = fabsf(dv1<F>(dzl, dl + eps, bad));
  const float ratr = fabsf(dv1<F>(dzr, dr + eps, bad));
  const float al = 1.0f + 5.0f * ratl;
  const float ar = 1.0f + 5.0f * ratr;
  const float ls = al * al, rs = ar * ar;
  return (ls > rs) ? ls : rs;
}

// critics_warp.py:244-248 costmap index (clamped, DEFINED)
template <bool F>
__device__ __forceinline__ int costmap_index(int size, float hw, const Recip& rres_c, float x,
                                             float y, bool& bad, float rinv = 0.0f, int cdiv = 0) {
  float fx, fy;
  if (cdiv) {  // uniform branch
    fx = cdiv_f(x + hw, rres_c.b, rinv);
    fy = cdiv_f((-y) + hw, rres_c.b, rinv);
  } else {
    fx = dv<F>(x + hw, rres_c, bad);
    fy = dv<F>((-y) + hw, rres_c, bad);
  }
  // clamp(trunc(clamp(f, -1, size)), 0, size - 1) == trunc(med3(f, 0, size - 1)) (as Dem::point)
  const int ix = (int)__builtin_amdgcn_fmed3f(fx, 0.0f, (float)(size - 1));
  const int iy = (int)__builtin_amdgcn_fmed3f(fy, 0.0f, (float)(size - 1));
  return ix + size * iy;
}


// =====================================================================  reductions
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}

// Record combine a (+) b for element j (oracle/mppi_ref.py combine).
struct __attribute__((aligned(16))) PairScale {  // one 16-byte LDS read
  float m;
  float ea, eb;
  int mode;  // 0 normal, 1 take a, 2 take b
};
__device__ __forceinline__ PairScale pair_scale(float ma, float mb, float T) {
  PairScale p;
  const bool ae = !(ma < INFINITY);  // empty (+inf) — NaN treated as empty too
  const bool be = !(mb < INFINITY);
  p.m = fminf(ma, mb);
  p.ea = p.eb = 0.0f;
  if (ae) {
    p.mode = 2;
  } else if (be) {
    p.mode = 1;
  } else {
    p.mode = 0;
    p.ea = dm_expf(-((ma - p.m) / T));
    p.eb = dm_expf(-((mb - p.m) / T));
  }
  return p;
}
__device__ __forceinline__ double pair_apply(const PairScale& p, double a, double b, int j) {
  if (p.mode == 1) return a;
  if (p.mode == 2) return b;
  if (j == 0) return (double)p.m;
  return (double)p.ea * a + (double)p.eb * b;
}
// The same value without branches (selects after the arithmetic; what a discarded product of an
// empty side holds does not matter): a wave's pair applies then issue their LDS reads together
// instead of a dependent read of `mode`, a branch, then a read of the scales, per pair.
// (The empty asm statement pins the products ahead of the selects: without it the compiler turns
// the selects back into branches around the loads.)
__device__ __forceinline__ PairScale ld_scale(const PairScale* ps) { return *ps; }
__device__ __forceinline__ double pair_apply_raw(const PairScale p, double a, double b, int j) {
  double r = (double)p.ea * a + (double)p.eb * b;
  asm volatile("" : "+v"(r));
  const double n = j == 0 ? (double)p.m : r;
  return p.mode == 1 ? a : (p.mode == 2 ? b : n);
}
__device__ __forceinline__ double pair_apply_sel(const PairScale& ps, double a, double b, int j) {
  return pair_apply_raw(ps, a, b, j);
}

// Subtree over an aligned group of G records (log2 G levels of the binary tree):
// scales of its G-1 pairs, level by level (ps[0 .. G/2) first), from the members' m.
template <int G>
__device__ __forceinline__ void group_scales(const float (&m)[G], float T, PairScale (&ps)[G - 1]) {
  float cur[G];
#pragma unroll
  for (int i = 0; i < G; ++i) cur[i] = m[i];
  int base = 0;
#pragma unroll
  for (int w = G / 2; w >= 1; w >>= 1) {
#pragma unroll
    for (int i = 0; i < w; ++i) {
      ps[base + i] = pair_scale(cur[2 * i], cur[2 * i + 1], T);
      cur[i] = ps[base + i].m;
    }
    base += w;
  }
}
template <int G>
__device__ __forceinline__ double group_apply(const PairScale* ps, const double (&v)[G], int j) {
  double cur[G];
#pragma unroll
  for (int i = 0; i < G; ++i) cur[i] = v[i];
  int base = 0;
#pragma unroll
  for (int w = G / 2; w >= 1; w >>= 1) {
#pragma unroll
    for (int i = 0; i < w; ++i) cur[i] = pair_apply(ps[base + i], cur[2 * i], cur[2 * i + 1], j);
    base += w;
  }
  return cur[0];
}

// threadIdx.x, and for the resident server (FRESH) laundered through an empty asm once per step: the
// thread-derived addresses of a step then cannot be hoisted out of the server's step loop and stay
// live across the whole loop (they raised it from ~96 to ~125 VGPRs); the range stays known.
template <bool FRESH, int NT = 1024>
__device__ __forceinline__ int thread_id() {
  int t = threadIdx.x;
  if constexpr (FRESH) asm volatile("" : "+v"(t));
  __builtin_assume(t >= 0 && t < NT);
  return t;
}

// =====================================================================  sampling normals
// The step's sampling normals (sampling_warp.py:54-92 with the Philox noise of DEFINED D1),
// precomputed so the rollout's producer waves only load them.  Unit g = (block g / NB, Philox block
// n = g % NB) for the trajectory tj of that block: eps1 / eps2 of steps t = 2n, 2n + 1, stored
// write-through (agent scope, sc1): the rows do not sit dirty in the XCD's L2 (a later kernel
// boundary would write them back) and other CUs read them after an L1 invalidate only.
struct NoiseVals {
  float a1, a2, b1, b2;
};
__device__ __forceinline__ NoiseVals noise_gen(uint64_t seed, uint64_t n_base, int64_t k_offset, int blk, int n, int tj) {
  const uint64_t kg = (uint64_t)(k_offset + (int64_t)blk * 256 + tj);
  NoiseVals v;
  noise_block_pk(seed, n_base + (uint64_t)n, kg, &v.a1, &v.a2, &v.b1, &v.b2);
  return v;
}
__device__ __forceinline__ void noise_store(float* __restrict__ eps, int H, int blk, int n, int tj, const NoiseVals& v) {
  const int t = 2 * n;
  float* e1 = eps + ((size_t)blk * 2 * H + t) * 256 + tj;
  float* e2 = e1 + (size_t)H * 256;
  __hip_atomic_store(e1, v.a1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(e2, v.a2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t + 1 < H) {
    __hip_atomic_store(e1 + 256, v.b1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(e2 + 256, v.b2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void noise_unit(uint64_t seed, uint64_t n_base, int64_t k_offset, int H, int blk, int n,
                                           float* __restrict__ eps, int tj) {
  noise_store(eps, H, blk, n, tj, noise_gen(seed, n_base, k_offset, blk, n, tj));
}
// units g0, g0 + gstride, ... below `end` (unit g = block g / NB, Philox block g % NB), the block and
// Philox index carried from unit to unit (wave-uniform: no 64-bit division per unit; g < 2^31,
// mppi_create bounds K)
__device__ __forceinline__ void noise_rows(uint64_t seed, uint64_t n_base, int64_t k_offset, int H, int end,
                                           float* __restrict__ eps, int g0, int gstride, int tj) {
  const int NB = (H + 1) >> 1;
  if (g0 >= end) return;
  int blk = g0 / NB, n = g0 - blk * NB;
  const int sq = gstride / NB, sr = gstride - sq * NB;
  for (int g = g0; g < end; g += gstride) {
    noise_unit(seed, n_base, k_offset, H, blk, n, eps, tj);
    blk += sq;
    n += sr;
    if (n >= NB) {
      n -= NB;
      ++blk;
    }
  }
}
// wave-units q0, q0 + stride, ... below q1 (wave-unit q = trajectories 64 (q % 4) .. + 63 of unit
// q / 4), two per iteration (independent Philox blocks: each one's dependent packed steps fill the
// other's wait states), the units' block and Philox index carried (all wave-uniform)
struct NoisePos {
  int q, g, blk, n;
};
__device__ __forceinline__ void noise_pos_step(NoisePos& p, int stride, int NB) {
  p.q += stride;
  p.n += (p.q >> 2) - p.g;
  p.g = p.q >> 2;
  while (p.n >= NB) {
    p.n -= NB;
    ++p.blk;
  }
}
__device__ __forceinline__ void noise_waves(uint64_t seed, uint64_t n_base, int64_t k_offset, int H, int q, int q1,
                                            int stride, float* __restrict__ eps, int lane) {
  const int NB = (H + 1) >> 1;
  if (q >= q1) return;
  NoisePos a;
  a.q = q;
  a.g = q >> 2;
  a.blk = a.g / NB;
  a.n = a.g - a.blk * NB;
  for (;;) {
    NoisePos b = a;
    noise_pos_step(b, stride, NB);
    const bool has_b = b.q < q1;
    if (!has_b) b = a;  // (computed, not stored)
    const NoiseVals va = noise_gen(seed, n_base, k_offset, a.blk, a.n, ((a.q & 3) << 6) + lane);
    const NoiseVals vb = noise_gen(seed, n_base, k_offset, b.blk, b.n, ((b.q & 3) << 6) + lane);
    noise_store(eps, H, a.blk, a.n, ((a.q & 3) << 6) + lane, va);
    if (!has_b) break;
    noise_store(eps, H, b.blk, b.n, ((b.q & 3) << 6) + lane, vb);
    a = b;
    noise_pos_step(a, stride, NB);
    if (a.q >= q1) break;
  }
}

// LDS row stride (floats) of the pair kernel's control cache: 256 trajectories + one float4 of
// skew, so the leaf's lanes (one row each) hit different banks
constexpr int UCACHE_ROW = 256 + 4;
template <int TB, int NT, bool EPS = false, bool WT = false>
__device__ __forceinline__ void leaf_records(const RolloutArgs& a, const float* cost_lds,
                                             unsigned char* scratch, const float* ub_block,
                                             const float* unom = nullptr, const float* ucache = nullptr,
                                             int uc_steps = 0, int blk = -1);

// =====================================================================  leaf records (shared)
// Softmax leaf records (DEFINED replacement of critics_warp.py:338-376) for the
// TB trajectories of a workgroup, whose costs are in cost_lds[TB] and sampled
// controls in ustore rows [2H][TB] (EPS: the normals rows, with the nominal sequence at `unom`
// [2H] in LDS and the first uc_steps steps' sampled controls at `ucache`).  Leaf = 256 trajectories.
//   m = leaf min, w = dm_expf(-(c - m)/T),
//   record [m, S, V1[H], V2[H]], each sum over the leaf's 256 trajectories the
//   pairwise tree in index order ((x0+x1)+(x2+x3)) + ... (float64);
// then the workgroup's subtree over its TB/256 leaves (tree_reduce order).
// Called by all NT threads; `scratch` is LDS of at least
// TB*4 + TB/64*4 (rounded to 16) + TB/256*(2H+2)*8 bytes.  WT: the record is stored
// write-through (agent-scope atomic stores) for the finish workgroups of the resident server.
template <int TB, int NT, bool EPS, bool WT>
__device__ __forceinline__ void leaf_records(const RolloutArgs& a, const float* cost_lds,
                                             unsigned char* scratch, const float* ub_block,
                                             const float* unom, const float* ucache, int uc_steps, int blk) {
  if (blk < 0) blk = blockIdx.x;  // the block whose record this is (a workgroup may run several)
  constexpr int NL = TB / 256;
  constexpr int NWL = TB / 64;   // waves' worth of trajectories
  const int tid = thread_id<WT, NT>(), lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, E = 2 * H + 2;
  float* wbuf = reinterpret_cast<float*>(scratch);                           // [TB]
  float* wave_m = wbuf + TB;                                                 // [NWL]
  double* red = reinterpret_cast<double*>(scratch + ((TB + NWL) * 4 + 15) / 16 * 16);  // [NL][E]
  // rows (leaf, j), j in [1, E): the pairwise tree over the leaf's 256 trajectories in index
  // order = (half 0) + (half 1), half = ((line 0 + line 1) + (line 2 + line 3)), line = 32
  // trajectories (8 float4 groups, a pairwise tree of its own).  One LINE per thread and round, its
  // loads issued before any is used: the re-read normals rows come from HBM / MALL (all workgroups'
  // leaves at once), and the first round's loads are issued before the weights are formed, so their
  // latency overlaps the weight phase (round 6).  A wave holds 8 rows x 8 lines: lane = 8 k + (row & 7)
  // for line k of the row, so the eight units of a row sit 8 lanes apart and combine by lane shuffles
  // (xor 8, 16, 32) in the same order, and the lanes that an LDS read serves together (8 consecutive)
  // read 8 different rows of the control cache (row stride UCACHE_ROW: 4 banks apart, conflict-free)
  // or the same weights (a broadcast); with the eight lines of one row in 8 consecutive lanes every
  // 16-byte read hit the same 4 banks 8 times.
  const int NR = NL * (E - 1);
  const int NU = ((NR + 7) >> 3) << 6;       // unit slots: 8 rows per wave (the last wave partly empty)
  struct Unit {
    float4 uq[8];
    int j;
    bool cached;
    float nom, sg, lo, hi;
    const float4* w4;
  };
  auto load = [&](int it, Unit& U) __attribute__((always_inline)) {  // unit slot: row 8 (it >> 6) + (it & 7), line (it >> 3) & 7
    const int k = (it >> 3) & 7;
    const int r = min(((it >> 6) << 3) + (it & 7), NR - 1);
    const int half = k >> 2, line = k & 3;
    const int leaf = r / (E - 1), j = 1 + r - leaf * (E - 1);
    U.j = j;
    const int tr0 = 256 * leaf + 128 * half + 32 * line;  // first trajectory of the line
    U.w4 = reinterpret_cast<const float4*>(wbuf + tr0);
    const float4* u4 = reinterpret_cast<const float4*>(ub_block + (size_t)(j >= 2 ? j - 2 : 0) * TB + tr0);
    U.cached = false;  // the sampled controls of this row are in LDS (no normals re-read)
    U.nom = U.sg = U.lo = U.hi = 0.f;
    if constexpr (EPS) {  // rows hold the normals: u = clamp(u_nom[t+1] + sigma*eps) as sampled
      const int c = (j - 2) >= H ? 1 : 0;
      const int t = max(j - 2, 0) - c * H;
      const int ti = min(t + 1, H - 1);
      U.nom = unom[c * H + ti];
      U.sg = c ? a.s2 : a.s1;
      U.lo = c ? a.min_u2 : a.min_u1;
      U.hi = c ? a.max_u2 : a.max_u1;
      if (j >= 2 && t < uc_steps) {
        U.cached = true;
        u4 = reinterpret_cast<const float4*>(ucache + (size_t)(c * uc_steps + t) * UCACHE_ROW + tr0);
      }
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) U.uq[g] = (j >= 2) ? u4[g] : make_float4(1.f, 1.f, 1.f, 1.f);
  };
  auto reduce = [&](int it, const Unit& U) __attribute__((always_inline)) {
    const int j = U.j;
    double gs[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const float4 w = U.w4[g];
      float4 u = U.uq[g];
      if (EPS && !U.cached) {
        u.x = clampf(U.nom + U.sg * u.x, U.lo, U.hi);
        u.y = clampf(U.nom + U.sg * u.y, U.lo, U.hi);
        u.z = clampf(U.nom + U.sg * u.z, U.lo, U.hi);
        u.w = clampf(U.nom + U.sg * u.w, U.lo, U.hi);
      }
      if (j < 2) u = make_float4(1.f, 1.f, 1.f, 1.f);  // j == 1: S, the weights alone
      // (w0 u0 + w1 u1) + (w2 u2 + w3 u3) in float64: a product of two floats is exact in a
      // double, so fma(w0, u0, w1 u1) is the rounded sum of the exact products (one product and
      // one fma instead of two products and an add per pair; same bits)
      const double x = __builtin_fma((double)w.x, (double)u.x, (double)w.y * (double)u.y);
      const double y = __builtin_fma((double)w.z, (double)u.z, (double)w.w * (double)u.w);
      gs[g] = x + y;
    }
    const double ls = ((gs[0] + gs[1]) + (gs[2] + gs[3])) + ((gs[4] + gs[5]) + (gs[6] + gs[7]));
    // (line 0 + line 1), (line 2 + line 3): left + right; then the half; then the row
    const double s2 = ls + __shfl_xor(ls, 8, 64);
    const double hs = s2 + __shfl_xor(s2, 16, 64);
    const double rs = hs + __shfl_xor(hs, 32, 64);
    const int r = ((it >> 6) << 3) + (it & 7);
    if (r < NR && ((it >> 3) & 7) == 0) {
      const int leaf = r / (E - 1);
      red[leaf * E + j] = rs;
    }
  };
  Unit first;
  if (tid < NU) load(tid, first);
  if (wave < NWL) {
    const float wm = wave_min(cost_lds[tid]);
    if (lane == 0) wave_m[wave] = wm;
  }
  __syncthreads();
  for (int j = tid; j < TB; j += NT) {
    const int leaf = j >> 8;
    const float m = fminf(fminf(wave_m[4 * leaf], wave_m[4 * leaf + 1]),
                          fminf(wave_m[4 * leaf + 2], wave_m[4 * leaf + 3]));
    const float c = cost_lds[j];
    wbuf[j] = (c < INFINITY) ? dm_expf(-((c - m) / a.T)) : 0.0f;
  }
  __syncthreads();
  if (tid < NU) reduce(tid, first);
  for (int it = NT + tid; it < NU; it += NT) {
    Unit U;
    load(it, U);
    reduce(it, U);
  }
  __syncthreads();
  for (int j = tid; j < E; j += NT) {
    double val[NL];
    float lm[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      lm[q] = fminf(fminf(wave_m[4 * q], wave_m[4 * q + 1]), fminf(wave_m[4 * q + 2], wave_m[4 * q + 3]));
      val[q] = (j == 0) ? (double)lm[q] : red[q * E + j];
    }
#pragma unroll
    for (int width = NL; width > 1; width >>= 1) {
#pragma unroll
      for (int q = 0; q < width / 2; ++q) {
        const PairScale ps = pair_scale(lm[2 * q], lm[2 * q + 1], a.T);
        val[q] = pair_apply(ps, val[2 * q], val[2 * q + 1], j);
        lm[q] = ps.m;
      }
    }
    if constexpr (WT)
      __hip_atomic_store(a.nodes + (size_t)blk * E + j, val[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      a.nodes[(size_t)blk * E + j] = val[0];
    if (j == 0 && a.rec_m) {  // m again in the contiguous array (one line per 32 records to read)
      if constexpr (WT)
        __hip_atomic_store(a.rec_m + blk, lm[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        a.rec_m[blk] = lm[0];
    }
  }
}

// =====================================================================  pair-synchronised rollout kernel
// Chain wave c and side wave c serve the trajectories 64c..64c+63 (lane = trajectory).
// Each chain/side PAIR synchronises only with itself, through LDS progress
// counters, never at a workgroup barrier.  Rings PAIR_D steps deep let a pair
// absorb step-to-step jitter (DEM gather latency):
//   chain step s : needs produced > s and consumed > s - D        -> chained = s + 1
//   side  iter p : produce p   (needs chained > p - D)           -> produced = p + 1
//                  consume p-L (needs chained > p - L)           -> consumed = p - L + 1
// with L = PAIR_LAG; deadlock-free for 0 < L < D (the chain's waits are always
// satisfied by side iterations that do not wait on it).  Bitwise identical results.
constexpr int PAIR_D = PAIR_RING;
constexpr int PAIR_LAG = 4;  // the largest even lag below D = 6 (at D = 8, 6 beat 2 and 4: profiles/r01_notes.md)
static_assert(PAIR_LAG > 0 && PAIR_LAG < PAIR_D, "ring depth must exceed the consume lag");
static_assert(PAIR_LAG % 2 == 0, "the side loop pairs even and odd steps");

// The flags and the rings are LDS, so the acquire / release fences are restricted to
// the local address space: a plain workgroup-scope release also orders the wave's
// global loads (s_waitcnt vmcnt(0) before every flag store), which would drain the
// side wave's prefetches (normals, costmap, wheel heights) at every publication.
__device__ __forceinline__ int lds_load_acquire(const int* f) {
  const int v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  return v;
}
__device__ __forceinline__ void lds_store_release(int* f, int v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ---------------------------------------------------------------------  the chain wave (3D)
// The serial 3D projection of 64 trajectories (projection_warp.py:306-348), shared by both
// rollout kernels.  Reads (v, sin, cos, 1 - cos) of each step from ring_in [D][4][TB] once
// f_prod covers it, writes (x, y, cx, cy) to ring_out [D][4][TB] and releases f_chain; a ring
// slot is rewritten once every consumer counter f_cons[0..NC) has passed it.
// Software-pipelined: iteration t orients step t (its normal gathered during iteration t - 1),
// then advances the position of step t + 1 and issues that step's normal gather, which stays in
// flight while step t's outputs are published.  Arithmetic: packed x / y FP32 (orient_step,
// advance_step), every quotient and square root correctly rounded; an out-of-range lane redoes
// its step with the IEEE operators.
__device__ __forceinline__ void lds_wait_ge(const int* f, int target, int& seen) {
  if (seen >= target) return;
  int v;
  // (the chain waves: no s_sleep between reads, a woken chain lost up to ~64 cycles per wait; C3
  // +0.7 % at 200 steps, chain waits 131 -> 120 cycles per step)
  while ((v = lds_load_acquire(f)) < target) {
  }
  seen = v;
}

template <int TB, int NC, bool DUMP, int DO = PAIR_D>
__device__ __forceinline__ void chain_wave_3d(const RolloutArgs& a, const Dem& dem, const Traj& s, int tj,
                                              bool valid, int64_t kl, const float* ring_in, float* ring_out,
                                              const int* f_prod, int* f_chain, const int* const (&f_cons)[NC],
                                              int& seen_prod, int (&seen_cons)[NC]) {
  constexpr int D = PAIR_D;
  constexpr int RI = 4;
  using T_ = std::true_type;
  using F_ = std::false_type;
  const int H = a.H;
  bool nobad = false;
  const bool clk = a.clk != nullptr && blockIdx.x == 0 && tj < 64;  // wave-uniform
  uint64_t clk_t0 = 0, clk_r0 = 0;
  if (clk) {
    clk_t0 = __builtin_amdgcn_s_memtime();
    clk_r0 = __builtin_amdgcn_s_memrealtime();
  }
  // dem.cdiv (uniform) as a compile-time tag: one copy of the loop per cell-division path, so
  // no branch inside a step separates the gather from the work around it
  auto body = [&](auto cd_tag) __attribute__((always_inline)) {
      constexpr bool CD = decltype(cd_tag)::value;
      // Software-pipelined: iteration t orients step t (its normal gathered during iteration
      // t - 1), then advances the position of step t + 1 and issues that step's normal gather,
      // which stays in flight while step t's outputs are published.  Register sets A / B
      // alternate between steps (no loop-carried copy of a load in flight).
      Head hd{f2{s.hx, s.hy}, s.hz};
      f2 posA = f2{s.x, s.y}, posB = posA;
      float4 nvA = make_float4(0.f, 0.f, 0.f, 0.f), nvB = nvA;
      float snA = 0.f, csA = 0.f, omA = 0.f, snB = 0.f, csB = 0.f, omB = 0.f;
      const f2 cell_off = f2{-a.x_min, a.y_min};
      const float fi_hi = (float)(a.grid - 1), fj_lo = (float)(1 - a.rows);
      // entry (jj, ii) = (1 - tjj, ti + 1) of the table: element (ti + grid + 2) - tjj * (grid + 1) >= 0 from
      // dem.N, addressed as the uniform base plus a 32-bit byte offset (table < 4 GiB, check_grid):
      // one v_mad_i32_i24 (|tjj|, grid + 1 < 2^23) instead of a quarter-rate 32-bit multiply and 64-bit adds
      const char* nbase = reinterpret_cast<const char*>(dem.N);
      const int nrow = a.grid + 1;
      const int ncol0 = a.grid + 2;
      // normal-table entry of the cell holding pos (Dem::cell + Dem::normal_cell)
      auto gather = [&](f2 pos, float4& nv) __attribute__((always_inline)) {
        f2 f;
        if constexpr (CD) {  // division by the verified reciprocal (cdiv_f), both axes at once
          const f2 aa = pos + cell_off;
          const f2 q0 = aa * bc2(dem.rinv);
          const f2 r = pk_fma(-q0, bc2(dem.res), aa);
          f = pk_fma(r, bc2(dem.rinv), q0);
        } else {
          f = f2{(pos.x - a.x_min) / a.res, (pos.y + a.y_min) / a.res};
        }
        const int ti = (int)__builtin_amdgcn_fmed3f(f.x, -1.0f, fi_hi);  // min(i, grid - 1)
        const int tjj = (int)__builtin_amdgcn_fmed3f(f.y, fj_lo, 1.0f);  // -min(j, rows - 1)
        const int idx = __mul24(tjj, -nrow) + (ti + ncol0);
        nv = *reinterpret_cast<const float4*>(nbase + (uint32_t)(idx << 4));
      };
      auto read_in = [&](int t, float& v, float& sn, float& cs, float& om, int need) __attribute__((always_inline)) {
        if (need) lds_wait_ge(f_prod, need, seen_prod);
        const float* ri = ring_in + (t % D) * RI * TB + tj;
        v = ri[0];
        sn = ri[TB];
        cs = ri[2 * TB];
        om = ri[3 * TB];
      };
      {  // step 0's position and normal
        float v0;
        read_in(0, v0, snA, csA, omA, 1);
        Lean l;
        lean_init(l);
        f2 p = advance_step<true>(hd, v0, a.dt, posA, l);
        if (__builtin_expect(lean_bad(l), 0)) p = advance_step<false>(hd, v0, a.dt, posA, l);
        posA = p;
        gather(posA, nvA);
      }
      // step t in set X (pos, normal in flight, sin / cos / 1 - cos); step t + 1 into set Y.
      // Even steps wait for two steps' worth of progress (the producer's steps t + 1, t + 2 and
      // the consumers' ring slots of t, t + 1), odd steps are covered by them.
      // more = t + 1 < H as a compile-time tag: the loop body has no branch around the next
      // step's advance and gather, so the scheduler can interleave them with step t's outputs
      auto it = [&](auto even_tag, auto more_tag, int t, f2& pX, float4& nX, float& snX, float& csX, float& omX,
                    f2& pY, float4& nY, float& snY, float& csY, float& omY) __attribute__((always_inline)) {
        constexpr bool EVEN = decltype(even_tag)::value;
        constexpr bool more = decltype(more_tag)::value;
        float v1 = 0.f;
        if constexpr (more) read_in(t + 1, v1, snY, csY, omY, EVEN ? min(t + 3, H) : 0);
        const f2 nxy = f2{nX.x, nX.y};
        const float nz = nX.z;
        Lean l;
        lean_init(l);
        Head ho = orient_step<true>(nxy, nz, hd, snX, csX, omX, l);
        f2 p1 = pX;
        if constexpr (more) p1 = advance_step<true, false>(ho, v1, a.dt, pX, l);
        if (__builtin_expect(lean_bad(l), 0)) {  // operand outside the fast range: IEEE redo
          ho = orient_step<false>(nxy, nz, hd, snX, csX, omX, l);
          if constexpr (more) p1 = advance_step<false>(ho, v1, a.dt, pX, l);
        }
        // wheel offset right = 0.2 * cross(normal, current_hv) (projection_warp.py:333)
        const f2 cxy = bc2(a.off) * cross_xy(nxy, nz, ho.xy, ho.z);
        if constexpr (more) {
          pY = p1;
          gather(pY, nY);
        }
        if constexpr (EVEN) {
#pragma unroll
          for (int c = 0; c < NC; ++c) lds_wait_ge(f_cons[c], t - DO + 2, seen_cons[c]);
        }
        float* ro = ring_out + (t % DO) * 4 * TB + tj;
        ro[0] = pX.x;
        ro[TB] = pX.y;
        ro[2 * TB] = cxy.x;
        ro[3 * TB] = cxy.y;
        if constexpr (DUMP) {
          if (valid) {
            float q[4];
            dem.template corners<false>(pX.x, pX.y, q, nobad);
            const float z = bilinear<false>(pX.x, pX.y, q, dem.template rr<false>(), nobad);
            const size_t o3 = ((size_t)kl * H + t) * 3;
            if (a.d_traj) { a.d_traj[o3] = pX.x; a.d_traj[o3 + 1] = pX.y; a.d_traj[o3 + 2] = z; }
            if (a.d_hv) { a.d_hv[o3] = ho.xy.x; a.d_hv[o3 + 1] = ho.xy.y; a.d_hv[o3 + 2] = ho.z; }
          }
        }
        lds_store_release(f_chain, t + 1);
        hd = ho;
      };
      int t = 0;
      for (; t + 2 < H; t += 2) {
        it(T_{}, T_{}, t, posA, nvA, snA, csA, omA, posB, nvB, snB, csB, omB);
        it(F_{}, T_{}, t + 1, posB, nvB, snB, csB, omB, posA, nvA, snA, csA, omA);
      }
      if (t + 1 < H) {  // the last two steps
        it(T_{}, T_{}, t, posA, nvA, snA, csA, omA, posB, nvB, snB, csB, omB);
        it(F_{}, F_{}, t + 1, posB, nvB, snB, csB, omB, posA, nvA, snA, csA, omA);
      } else {  // the last step (H odd)
        it(T_{}, F_{}, t, posA, nvA, snA, csA, omA, posB, nvB, snB, csB, omB);
      }
  };
  if (dem.cdiv)
    body(T_{});
  else
    body(F_{});
  if (clk) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (tj == 0) {
      a.clk[0] = clk_t0;
      a.clk[1] = clk_r0;
      a.clk[2] = t1;
      a.clk[3] = r1;
    }
  }
}

template <int TB, int PROJ, int MODE, bool DUMP>
__global__ __launch_bounds__(2 * TB) void mppi_rollout_pair_kernel(const RolloutArgs a_in) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  RolloutArgs a = a_in;
  constexpr int NT = 2 * TB;
  constexpr int NWC = TB / 64;
  constexpr int D = PAIR_D;
  constexpr int RI = PAIR_RING_IN;
  float* ring_in = reinterpret_cast<float*>(smem_raw);   // [D][RI][TB]: v, w or v, sin, cos
  float* ring_out = ring_in + D * RI * TB;               // [D][4][TB]: x, y, cx, cy
  float* cost_lds = ring_out + D * 4 * TB;               // [TB]
  int* flags = reinterpret_cast<int*>(cost_lds + TB);    // [4][NWC]: produced, chained, consumed, -
  float* unom_lds = reinterpret_cast<float*>(flags + 4 * NWC);  // [2H] u_nom1 | u_nom2 (padded to 4)
  unsigned char* scratch = reinterpret_cast<unsigned char*>(unom_lds + ((2 * a.H + 3) & ~3));
  static_assert(TB == 256, "UCACHE_ROW assumes 256 trajectories per workgroup");
  // sampled controls of steps [0, ucache_steps) for leaf_records: [2][ucache_steps][UCACHE_ROW] after
  // the leaf scratch (layout of make_plan in mppi_capi.cpp)
  float* ucache = reinterpret_cast<float*>(
      smem_raw + ((size_t)(scratch - smem_raw) + ((TB + TB / 64) * 4 + 15) / 16 * 16 +
                  (size_t)(TB / 256) * (2 * a.H + 2) * sizeof(double) + 15) / 16 * 16);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool side = wave >= NWC;
  const int tj = side ? tid - TB : tid;  // trajectory within the workgroup
  const int pair = side ? wave - NWC : wave;
  // issue priority over the deferred optimal rollout of the previous step (mppi_tail_kernel,
  // priority 0), which shares one CU with a rollout workgroup: it has a whole step of slack
  if (a.wave_prio) __builtin_amdgcn_s_setprio(2);
  int* f_prod = flags + pair;
  int* f_chain = flags + NWC + pair;
  int* f_cons = flags + 2 * NWC + pair;
  const int64_t kl = (int64_t)blockIdx.x * TB + tj;
  const bool valid = kl < a.K;
  const int H = a.H;
  Dem dem;
  dem.init(a.Z, a.rows, a.grid, a.x_min, a.y_min, a.res, a.rinv_res, a.cdiv_res);
  dem.N = a.ntab;
  const float res_half_neg = (-a.res) / 2.0f;
  const float res_sq = a.res * a.res;
  bool nobad = false;
  if (tid < 4 * NWC) flags[tid] = 0;
  // the nominal sequence in LDS: the side wave reads one element per step, and a vector
  // load there would make every wait for it (vmcnt is in order) also wait for the normals
  // prefetched just before it
  if constexpr (MODE == 0)
    for (int i = tid; i < 2 * H; i += NT)  // agent-scope: written through by the resident server's finish
      unom_lds[i] = __hip_atomic_load(i < H ? a.u_nom1 + i : a.u_nom2 + (i - H), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);

  // ---------------- per-role state
  Traj s;                       // chain
  float L = a.wl, R = a.wr;     // side: filter
  // side, MODE 0: this trajectory's normals, rows [2][H] of 256 (mppi_noise_kernel)
  const float* eps_row = (MODE == 0) ? a.eps + (size_t)blockIdx.x * (2 * H) * TB + tj : nullptr;
  float en1 = 0.f, en2 = 0.f;
  if constexpr (MODE == 0) {
    if (side) {
      en1 = eps_row[0];
      en2 = eps_row[(size_t)H * TB];
    }
  }
  float pf_sum = 0.f, sw = 0.f, sp = 0.f, ob = 0.f, last_x = a.x0, last_y = a.y0;
  float lwx = 0.f, lwy = 0.f, lwz = 0.f, rwx = 0.f, rwy = 0.f, rwz = 0.f;
  float* ust = a.ustore + (size_t)blockIdx.x * (2 * H) * TB + tj;

  if (!side) {  // initial projection at the robot pose (projection_warp.py:306-310)
    s.x = a.x0;
    s.y = a.y0;
    float q[4];
    dem.template corners<false>(s.x, s.y, q, nobad);
    const float vx = res_half_neg * (((q[1] - q[0]) - q[2]) + q[3]);
    const float vy = res_half_neg * (((q[2] - q[0]) - q[1]) + q[3]);
    const float nn = sqrtf((vx * vx + vy * vy) + res_sq * res_sq);
    const float nx = vx / nn, ny = vy / nn, nz = res_sq / nn;
    if constexpr (PROJ == 3) {
      const float d = (a.h0x * nx + a.h0y * ny) + a.h0z * nz;
      const float tx = a.h0x - d * nx, ty = a.h0y - d * ny, tz = a.h0z - d * nz;
      const float tn = sqrtf((tx * tx + ty * ty) + tz * tz);
      s.hx = tx / tn;
      s.hy = ty / tn;
      s.hz = tz / tn;
    } else {
      s.hx = a.h0x;
      s.hy = a.h0y;
      s.hz = a.h0z;
    }
  }
  __syncthreads();  // flags initialised

  // Wait until *f >= target; `seen` caches the last value this wave acquired from f.  The
  // counters only grow, and everything published before a value is visible to the wave
  // once it has acquired that value, so a cached value that already covers the target
  // needs no LDS read and no fence (the partner usually runs several steps ahead).
  auto wait_ge = [&](const int* f, int target, int& seen) __attribute__((always_inline)) {
    if (seen >= target) return;
    int v;
    while ((v = lds_load_acquire(f)) < target) __builtin_amdgcn_s_sleep(1);
    seen = v;
  };

  if (!side) {
    // ---------------- chain wave: the serial projection, one step per iteration
    int seen_prod = 0, seen_cons = 0;
    if constexpr (PROJ == 3) {
      const int* cons[1] = {f_cons};
      int seen_c[1] = {0};
      chain_wave_3d<TB, 1, DUMP>(a, dem, s, tj, valid, kl, ring_in, ring_out, f_prod, f_chain, cons, seen_prod,
                                 seen_c);
    } else
    for (int sc = 0; sc < H; ++sc) {  // 2D: the planar step (projection_warp.py:353-382)
      wait_ge(f_prod, sc + 1, seen_prod);
      wait_ge(f_cons, sc - D + 1, seen_cons);
      const float* ri = ring_in + (sc % D) * RI * TB + tj;
      const float v = ri[0];
      const float sn = ri[TB], cs = ri[2 * TB];  // sin/cos of the Rodrigues angle (side wave)
      const float cx = 0.f, cy = 0.f;
      StepOut o;
      step2d<false>(dem, a.dt, v, sn, cs, s, o, nobad);
      const float z = o.z;
      (void)z;
      float* ro = ring_out + (sc % D) * 4 * TB + tj;
      ro[0] = s.x;
      ro[TB] = s.y;
      ro[2 * TB] = cx;
      ro[3 * TB] = cy;
      if constexpr (DUMP) {
        if (valid) {
          const size_t o3 = ((size_t)kl * H + sc) * 3;
          if (a.d_traj) { a.d_traj[o3] = s.x; a.d_traj[o3 + 1] = s.y; a.d_traj[o3 + 2] = z; }
          if (a.d_hv) { a.d_hv[o3] = s.hx; a.d_hv[o3 + 1] = s.hy; a.d_hv[o3 + 2] = s.hz; }
        }
      }
      lds_store_release(f_chain, sc + 1);
    }
  } else {
    // ---------------- side wave: produce step p, consume step p - PAIR_LAG
    // Unrolled by two (even / odd steps, PAIR_LAG even so both have the same parity)
    // so that every value loaded for a later half stays in its own registers: a
    // loop-carried copy of a load in flight makes the compiler wait for it (vmcnt(0))
    // at the back edge, and vmcnt is in order, so the normals prefetched for the next
    // step would also be waited for at the first wheel-height wait.  Loads:
    //  * normals of step p + 2 into the registers that served step p, after its consume;
    //  * costmap value of step sc, used (obstacle critic) in the other half;
    //  * wheel heights of the EVEN steps only (the slope critic, critics_warp.py:220-267,
    //    reads lw/rw at i, i+2 for even i; odd-step contacts are computed only for
    //    DUMP), used one half later.
    int seen_chain = 0;                                 // last acquired value of f_chain
    float eA1 = en1, eA2 = en2, eB1 = 0.f, eB2 = 0.f;  // normals of the even / odd step
    if constexpr (MODE == 0) {
      const int t1 = min(1, H - 1);
      eB1 = eps_row[(size_t)t1 * TB];
      eB2 = eps_row[(size_t)(H + t1) * TB];
    }
    float cmA = 0.f, cmB = 0.f;                        // costmap value of the even / odd step
    float elx = 0.f, ely = 0.f, elz = 0.f, erx = 0.f, ery = 0.f, erz = 0.f;  // even step's contacts
    // PROD / CONS: the half produces step p / consumes step sc = p - PAIR_LAG for sure
    // (no runtime test: branch-free loads let the compiler count vmcnt exactly); with
    // neither set, both are tested at run time (the few halves at the ends).
    auto half = [&](auto odd_tag, auto prod_tag, auto cons_tag, int p, float& e1r, float& e2r,
                    float& cm_mine, float& cm_prev) __attribute__((always_inline)) {
      constexpr bool ODD = decltype(odd_tag)::value;
      constexpr bool PROD = decltype(prod_tag)::value, CONS = decltype(cons_tag)::value;
      constexpr bool GUARD = !PROD && !CONS;
      if (PROD || (GUARD && p < H)) {  // sampling, filter (sampling_warp.py:54-138); normals precomputed
        float u1, u2;
        if constexpr (MODE == 0) {
          const int ti = min(p + 1, H - 1);
          u1 = clampf(unom_lds[ti] + a.s1 * e1r, a.min_u1, a.max_u1);
          u2 = clampf(unom_lds[H + ti] + a.s2 * e2r, a.min_u2, a.max_u2);
          if (p < a.ucache_steps) {  // kept for the leaf reduction (uniform branch)
            ucache[(size_t)p * UCACHE_ROW + tj] = u1;
            ucache[(size_t)(a.ucache_steps + p) * UCACHE_ROW + tj] = u2;
          }
        } else {
          const size_t o = (size_t)(valid ? kl : 0) * H + p;
          u1 = a.inj_u1[o];
          u2 = a.inj_u2[o];
          ust[(size_t)p * TB] = u1;   // MODE 1: the leaf records read the injected controls back
          ust[(size_t)(H + p) * TB] = u2;
        }
        wait_ge(f_chain, p - D + 1, seen_chain);
        L = L * a.fa + (u1 * a.fk) * (1.0f - a.fa);
        R = R * a.fa + (u2 * a.fk) * (1.0f - a.fa);
        const float vp = clampf((L + R) / 2.0f, a.vmin, a.vmax);
        const float wp = clampf(((-L) + R) / a.rwheel, a.wmin, a.wmax);
        float* ri = ring_in + (p % D) * RI * TB + tj;
        ri[0] = vp;
        {
          float sn, cs;
          if (a.small_angle) dm_sincosf_small(wp * a.dt, &sn, &cs);
          else dm_sincosf(wp * a.dt, &sn, &cs);
          ri[TB] = sn;
          ri[2 * TB] = cs;
          ri[3 * TB] = 1.0f - cs;
        }
        if constexpr (DUMP) {
          if (valid) {
            const size_t o1 = (size_t)kl * H + p;
            if (a.d_u1) a.d_u1[o1] = u1;
            if (a.d_u2) a.d_u2[o1] = u2;
            if (a.d_w) a.d_w[o1] = wp;
          }
        }
        lds_store_release(f_prod, p + 1);
      }
      const int sc = p - PAIR_LAG;
      if (CONS || (GUARD && sc >= 0 && sc < H)) {  // contacts + critics of step sc (projection_warp.py:333-348)
        wait_ge(f_chain, sc + 1, seen_chain);
        const float* ro = ring_out + (sc % D) * 4 * TB + tj;
        const float x = ro[0], y = ro[TB], cx = ro[2 * TB], cy = ro[3 * TB];
        const float vq = ring_in[(sc % D) * RI * TB + tj];  // v of step sc (slot not reused yet)
        if constexpr (!ODD) {  // contacts of an even step: heights in flight until the odd half
          if constexpr (PROJ == 3) {
            elx = x + cx;
            ely = y + cy;
            elz = dem.template point<false>(elx, ely, nobad);
            erx = x - cx;
            ery = y - cy;
            erz = dem.template point<false>(erx, ery, nobad);
          }
        }
        Recip rcm;
        rcm.b = a.res_c;
        cm_mine = a.cm[costmap_index<false>(a.cm_size, a.hw, rcm, x, y, nobad, a.rinv_res_c, a.cdiv_res_c)];
        const float pft = pf_sum + 10.0f * (fabsf(x - a.gx) + fabsf(y - a.gy));
        pf_sum = (sc < H - 1) ? pft : pf_sum;   // _path_follow_critic sum over t < H-1
        last_x = x;
        last_y = y;
        if constexpr (ODD) {  // _avoid_slope_wheels term (i, i+2) of the even step i = sc - 1 < H-3
          const int se = sc - 1;
          const float term = slope_term<false>(lwx, lwy, lwz, elx, ely, elz, rwx, rwy, rwz, erx, ery, erz, nobad);
          sw = (se >= 2 && se - 2 < H - 3) ? sw + term : sw;
          lwx = elx; lwy = ely; lwz = elz;
          rwx = erx; rwy = ery; rwz = erz;
        }
        const float spt = sp + (a.vmax - vq) / (vq + 0.0001f);  // _maximise_speed
        sp = a.speed_on ? spt : sp;
        // _avoid_obstacle: the costmap value gathered in the other half (step sc - 1)
        const float ob1 = (cm_prev > a.thr) ? ob + a.pen : ob;
        ob = (sc > 0) ? ob1 + cm_prev : ob;
        if constexpr (DUMP) {
          if (valid) {
            float lx = elx, ly = ely, lz = elz, rx = erx, ry = ery, rz = erz;
            if (ODD) {
              lx = ly = lz = rx = ry = rz = 0.f;
              if constexpr (PROJ == 3) {
                lx = x + cx;
                ly = y + cy;
                lz = dem.template point<false>(lx, ly, nobad);
                rx = x - cx;
                ry = y - cy;
                rz = dem.template point<false>(rx, ry, nobad);
              }
            }
            const size_t o3 = ((size_t)kl * H + sc) * 3;
            if (a.d_lw) { a.d_lw[o3] = lx; a.d_lw[o3 + 1] = ly; a.d_lw[o3 + 2] = lz; }
            if (a.d_rw) { a.d_rw[o3] = rx; a.d_rw[o3 + 1] = ry; a.d_rw[o3 + 2] = rz; }
            const size_t o1 = (size_t)kl * H + sc;
            if (a.d_v) a.d_v[o1] = vq;
          }
        }
        lds_store_release(f_cons, sc + 1);
      }
      if constexpr (MODE == 0) {  // prefetch the normals of step p + 2 into the registers just freed
        const int tn = min(p + 2, H - 1);
        e1r = eps_row[(size_t)tn * TB];
        e2r = eps_row[(size_t)(H + tn) * TB];
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    int p = 0;
    for (const int p1 = min(H, PAIR_LAG) & ~1; p < p1; p += 2) {  // produce only
      half(F_{}, T_{}, F_{}, p, eA1, eA2, cmA, cmB);
      half(T_{}, T_{}, F_{}, p + 1, eB1, eB2, cmB, cmA);
    }
    if (p == PAIR_LAG) {  // steady state: produce p, consume p - PAIR_LAG
      for (; p + 1 < H; p += 2) {
        half(F_{}, T_{}, T_{}, p, eA1, eA2, cmA, cmB);
        half(T_{}, T_{}, T_{}, p + 1, eB1, eB2, cmB, cmA);
      }
    }
    for (; p < H + PAIR_LAG; p += 2) {  // the ends, tested per half
      half(F_{}, F_{}, F_{}, p, eA1, eA2, cmA, cmB);
      if (p + 1 < H + PAIR_LAG) half(T_{}, F_{}, F_{}, p + 1, eB1, eB2, cmB, cmA);
    }
    const float cm_last = ((H - 1) & 1) ? cmB : cmA;
    if (cm_last > a.thr) ob = ob + a.pen;  // last step's obstacle term
    ob = ob + cm_last;
    // _evaluate_trajectories_kernel (critics_warp.py:325-329)
    float pf;
    if (a.pf_far) {
      const float dx = last_x - a.igx, dy = last_y - a.igy;
      pf = (dx * dx + dy * dy) * a.pf_scale;
    } else {
      pf = pf_sum;
    }
    float cost = a.w_path * pf;
    cost = cost + a.w_slope * sw;
    cost = cost + a.w_speed * sp;
    cost = cost + a.w_obs * ob;
    if (valid) a.cost_out[kl] = cost;
    cost_lds[tj] = valid ? cost : INFINITY;
  }
  __syncthreads();
  if constexpr (MODE == 0)  // rows hold the normals; the leaf recomputes the sampled controls
    leaf_records<TB, NT, true>(a, cost_lds, scratch, a.eps + (size_t)blockIdx.x * (2 * H) * TB, unom_lds, ucache,
                               a.ucache_steps);
  else
    leaf_records<TB, NT>(a, cost_lds, scratch, a.ustore + (size_t)blockIdx.x * (2 * H) * TB);
}

// =====================================================================  role-split rollout kernel
// Four waves per 64 trajectories (lane = trajectory), one per role, wave = role * NG + group,
// so the four roles of a group share one SIMD:
//   CHAIN  the serial projection (projection_warp.py:314-326), as the pair kernel's chain wave;
//   PROD   sampling, wheel filter (sampling_warp.py:54-138) and sin / cos of the Rodrigues angle
//          -> ring_in (v, sin, cos);
//   WHEEL  wheel contacts and heights of the even steps and the slope critic
//          (projection_warp.py:333-348, critics_warp.py:220-267);
//   COST   costmap gather, obstacle, path-follow and speed critics (critics_warp.py:85-300).
// One wave issues at most one instruction per ~4 cycles whatever its type, and the SIMD takes
// up to ~2 waves' worth of VALU issue (profiles/ubench/issue.hip): the chain wave's
// instruction count per step bounds the kernel, so everything off its recurrence runs in the
// other three waves, whose own streams are then shorter than the chain's.
// Progress counters per group (LDS), each wave caching the last value it acquired:
//   CHAIN step s : produced > s, wheel > s - D, cost > s - D   (ring_out slot s % D free)
//   PROD  step p : chained > p - D   (ring_in slot p % D is read by CHAIN only: the speed critic, the
//                  one consumer of v, runs in PROD itself since round 6, so the producer runs up to D
//                  steps ahead of the chain instead of the cost wave, which trails the chain)
//   WHEEL / COST step s : chained > s
// Deadlock-free: no wave waits on a later step of a wave that waits on it.
// Issue priorities: the chain 3; the producer 1 (the chain waits on it each step: +1.3 % C3 steps/s
// with 6-deep rings, profiles/r04_notes.md); the wheel and cost waves 0, level with the deferred
// optimal rollout of the previous step (mppi_tail_kernel) on the CU they share: at 2 the tail,
// starved, ran ~105 us and into the next finish, and pipelined C3 steps alternated between ~98 and
// ~120 us (profiles/r02_notes.md; 0: ~9900 against ~9200 steps/s).
constexpr int kProdPrio = 1, kSidePrio = 0;
// steps ahead the producer loads each step's normals (round 6: 4 and 8 measured within noise of 2 on
// the server and in separate launches, profiles/r06_notes.md)
constexpr int kProdPrefetch = 2;
constexpr int ROLE_CHAIN = 0, ROLE_PROD = 1, ROLE_WHEEL = 2, ROLE_COST = 3, NROLES = 4;

// FUSED: returns the workgroup's ticket (its rank among the workgroups that have completed their
// records, from the record counter rec_cnt); otherwise -1.
template <int TB, int PROJ, int MODE, bool DUMP, bool FUSED>
__device__ __forceinline__ int roles_body(const RolloutArgs& a, int blk, unsigned* rec_cnt, int* ticket_lds = nullptr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  constexpr int NT = NROLES * TB;
  constexpr int NG = TB / 64;  // trajectory groups (waves per role)
  constexpr int D = PAIR_D;
  constexpr int DO = ROLES_RING_OUT;  // ring_out's depth (the consumers' slack behind the chain)
  constexpr int RI = 4;
  static_assert(TB == 256, "UCACHE_ROW assumes 256 trajectories per workgroup");
  float* ring_in = reinterpret_cast<float*>(smem_raw);   // [D][4][TB]: v, sin, cos, 1 - cos
  float* ring_out = ring_in + D * RI * TB;               // [DO][4][TB]: x, y, cx, cy
  float* cost_lds = ring_out + DO * 4 * TB;              // [TB]
  float* sw_lds = cost_lds + TB;                         // [TB] slope critic (WHEEL -> COST)
  int* flags = reinterpret_cast<int*>(sw_lds + TB);      // [4][NG]: produced, chained, wheel, cost
  float* unom_lds = reinterpret_cast<float*>(flags + 4 * NG);  // [2H] u_nom1 | u_nom2 (padded to 4)
  unsigned char* scratch = reinterpret_cast<unsigned char*>(unom_lds + ((2 * a.H + 3) & ~3));
  float* ucache = reinterpret_cast<float*>(
      smem_raw + ((size_t)(scratch - smem_raw) + ((TB + TB / 64) * 4 + 15) / 16 * 16 +
                  (size_t)(TB / 256) * (2 * a.H + 2) * sizeof(double) + 15) / 16 * 16);
  const int tid = thread_id<FUSED, NT>();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int role = wave / NG;
  const int grp = wave - role * NG;
  const int tj = grp * 64 + (tid & 63);  // trajectory within the workgroup
  if (a.wave_prio) {  // above the deferred optimal rollout (priority 0); the chain above all
    if (role == ROLE_CHAIN) __builtin_amdgcn_s_setprio(3);
    else if (role == ROLE_PROD) __builtin_amdgcn_s_setprio(kProdPrio);
    else __builtin_amdgcn_s_setprio(kSidePrio);
  }
  int* f_prod = flags + grp;
  int* f_chain = flags + NG + grp;
  int* f_wheel = flags + 2 * NG + grp;
  int* f_cost = flags + 3 * NG + grp;
  const int64_t kl = (int64_t)blk * TB + tj;
  const bool valid = kl < a.K;
  const int H = a.H;
  Dem dem;
  dem.init(a.Z, a.rows, a.grid, a.x_min, a.y_min, a.res, a.rinv_res, a.cdiv_res);
  dem.N = a.ntab;
  const float res_half_neg = (-a.res) / 2.0f;
  const float res_sq = a.res * a.res;
  bool nobad = false;
  const bool clk_wg = a.clk != nullptr && blockIdx.x == 0 && tid == 0;
  if (clk_wg) a.clk[4] = __builtin_amdgcn_s_memrealtime();  // workgroup 0 starts
  const bool clk_any = a.clk != nullptr && tid == 0 && blockIdx.x < kClkBlocks;
  if (clk_any) a.clk[kClkBase + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();  // every workgroup
  if (tid < 4 * NG) flags[tid] = 0;
  if constexpr (MODE == 0)
    for (int i = tid; i < 2 * H; i += NT)  // agent-scope: written through by the resident server's finish
      unom_lds[i] = __hip_atomic_load(i < H ? a.u_nom1 + i : a.u_nom2 + (i - H), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();  // flags and nominal sequence initialised

  auto wait_ge = [&](const int* f, int target, int& seen) __attribute__((always_inline)) {
    if (seen >= target) return;
    int v;
    while ((v = lds_load_acquire(f)) < target) __builtin_amdgcn_s_sleep(1);
    seen = v;
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  float c_pf = 0.f, c_ob = 0.f;  // COST: the critic sums, kept across the barrier

  if (role == ROLE_CHAIN) {
    // ---------------- the serial projection, one step per iteration
    Traj s;
    s.x = a.x0;
    s.y = a.y0;
    {  // initial projection at the robot pose (projection_warp.py:306-310)
      float q[4];
      dem.template corners<false>(s.x, s.y, q, nobad);
      const float vx = res_half_neg * (((q[1] - q[0]) - q[2]) + q[3]);
      const float vy = res_half_neg * (((q[2] - q[0]) - q[1]) + q[3]);
      const float nn = sqrtf((vx * vx + vy * vy) + res_sq * res_sq);
      const float nx = vx / nn, ny = vy / nn, nz = res_sq / nn;
      if constexpr (PROJ == 3) {
        const float d = (a.h0x * nx + a.h0y * ny) + a.h0z * nz;
        const float tx = a.h0x - d * nx, ty = a.h0y - d * ny, tz = a.h0z - d * nz;
        const float tn = sqrtf((tx * tx + ty * ty) + tz * tz);
        s.hx = tx / tn;
        s.hy = ty / tn;
        s.hz = tz / tn;
      } else {
        s.hx = a.h0x;
        s.hy = a.h0y;
        s.hz = a.h0z;
      }
    }
    int seen_prod = 0, seen_wheel = 0, seen_cost = 0;
    if constexpr (PROJ == 3) {
      const int* cons[2] = {f_wheel, f_cost};
      int seen_cons[2] = {0, 0};
      chain_wave_3d<TB, 2, DUMP, DO>(a, dem, s, tj, valid, kl, ring_in, ring_out, f_prod, f_chain, cons, seen_prod,
                                 seen_cons);
    } else
    for (int sc = 0; sc < H; ++sc) {  // 2D (projection_warp.py:373-382): no normal, wheels zero
      wait_ge(f_prod, sc + 1, seen_prod);
      wait_ge(f_wheel, sc - DO + 1, seen_wheel);
      wait_ge(f_cost, sc - DO + 1, seen_cost);
      const float* ri = ring_in + (sc % D) * RI * TB + tj;
      const float v = ri[0], sn = ri[TB], cs = ri[2 * TB];
      const float cx = 0.f, cy = 0.f;
      StepOut o;
      step2d<false>(dem, a.dt, v, sn, cs, s, o, nobad);
      const float z = o.z;
      float* ro = ring_out + (sc % DO) * 4 * TB + tj;
      ro[0] = s.x;
      ro[TB] = s.y;
      ro[2 * TB] = cx;
      ro[3 * TB] = cy;
      if constexpr (DUMP) {
        if (valid) {
          const size_t o3 = ((size_t)kl * H + sc) * 3;
          if (a.d_traj) { a.d_traj[o3] = s.x; a.d_traj[o3 + 1] = s.y; a.d_traj[o3 + 2] = z; }
          if (a.d_hv) { a.d_hv[o3] = s.hx; a.d_hv[o3 + 1] = s.hy; a.d_hv[o3 + 2] = s.hz; }
        }
      }
      lds_store_release(f_chain, sc + 1);
    }
  }
  else if (role == ROLE_PROD) {
    // ---------------- sampling + wheel filter + sin/cos, normals prefetched PF steps ahead (step p in
    // register set p % PF: no loop-carried copy of a load in flight)
    const float* eps_row = (MODE == 0) ? a.eps + (size_t)blk * (2 * H) * TB + tj : nullptr;
    float* ust = a.ustore + (size_t)blk * (2 * H) * TB + tj;
    float L = a.wl, R = a.wr;
    float sp = 0.f;  // _maximise_speed (critics_warp.py:281-300) over the v it produces
    int seen_chain = 0;
    constexpr int PF = kProdPrefetch;
    float e[PF][2] = {};
    if constexpr (MODE == 0) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int t = min(q, H - 1);
        e[q][0] = eps_row[(size_t)t * TB];
        e[q][1] = eps_row[(size_t)(H + t) * TB];
      }
    }
    auto prod = [&](int p, float& e1r, float& e2r) __attribute__((always_inline)) {
      float u1, u2;
      if constexpr (MODE == 0) {
        const int ti = min(p + 1, H - 1);
        u1 = clampf(unom_lds[ti] + a.s1 * e1r, a.min_u1, a.max_u1);
        u2 = clampf(unom_lds[H + ti] + a.s2 * e2r, a.min_u2, a.max_u2);
        if (p < a.ucache_steps) {  // kept for the leaf reduction (uniform branch)
          ucache[(size_t)p * UCACHE_ROW + tj] = u1;
          ucache[(size_t)(a.ucache_steps + p) * UCACHE_ROW + tj] = u2;
        }
      } else {
        const size_t o = (size_t)(valid ? kl : 0) * H + p;
        u1 = a.inj_u1[o];
        u2 = a.inj_u2[o];
        ust[(size_t)p * TB] = u1;  // MODE 1: the leaf records read the injected controls back
        ust[(size_t)(H + p) * TB] = u2;
      }
      L = L * a.fa + (u1 * a.fk) * (1.0f - a.fa);
      R = R * a.fa + (u2 * a.fk) * (1.0f - a.fa);
      const float vp = clampf((L + R) / 2.0f, a.vmin, a.vmax);
      const float wp = clampf(((-L) + R) / a.rwheel, a.wmin, a.wmax);
      float sn, cs;
      if (a.small_angle) dm_sincosf_small(wp * a.dt, &sn, &cs);
      else dm_sincosf(wp * a.dt, &sn, &cs);
      const float spt = sp + (a.vmax - vp) / (vp + 0.0001f);
      sp = a.speed_on ? spt : sp;
      // ring_in slot p % D held step p - D, which only the chain reads (at the latest by its
      // iteration p - D, so chained >= p - D + 1 covers it; step 0 before its first iteration)
      wait_ge(f_chain, p - D + 1, seen_chain);
      float* ri = ring_in + (p % D) * RI * TB + tj;
      ri[0] = vp;
      ri[TB] = sn;
      ri[2 * TB] = cs;
      ri[3 * TB] = 1.0f - cs;
      if constexpr (DUMP) {
        if (valid) {
          const size_t o1 = (size_t)kl * H + p;
          if (a.d_u1) a.d_u1[o1] = u1;
          if (a.d_u2) a.d_u2[o1] = u2;
          if (a.d_w) a.d_w[o1] = wp;
          if (a.d_v) a.d_v[o1] = vp;
        }
      }
      lds_store_release(f_prod, p + 1);
      if constexpr (MODE == 0) {  // the normals of step p + PF into the registers just freed
        const int tn = min(p + PF, H - 1);
        e1r = eps_row[(size_t)tn * TB];
        e2r = eps_row[(size_t)(H + tn) * TB];
      }
    };
    int p = 0;
    for (; p + PF <= H; p += PF) {
#pragma unroll
      for (int q = 0; q < PF; ++q) prod(p + q, e[q][0], e[q][1]);
    }
#pragma unroll
    for (int q = 0; q < PF - 1; ++q)
      if (p + q < H) prod(p + q, e[q][0], e[q][1]);
    cost_lds[tj] = sp;  // (to the cost wave, which reads it after the barrier and then stores the cost)
  } else if (role == ROLE_WHEEL) {
    // ---------------- wheel contacts of the even steps (the slope critic reads lw / rw at i,
    // i + 2 for even i, critics_warp.py:220-267) and the slope critic.  Contact sets A / B
    // alternate (steps 0, 4, 8, ... / 2, 6, 10, ...); the term of (i, i + 2) = (sc - 4, sc - 2)
    // is added at even step sc, before sc's contacts replace those of sc - 4, so every height
    // gathered has two chain steps to arrive and no register holding a load in flight is copied.
    int seen_chain = 0;
    float sw = 0.f;
    float Alx = 0.f, Aly = 0.f, Alz = 0.f, Arx = 0.f, Ary = 0.f, Arz = 0.f;
    float Blx = 0.f, Bly = 0.f, Blz = 0.f, Brx = 0.f, Bry = 0.f, Brz = 0.f;
    auto contacts = [&](int sc, float& lx, float& ly, float& lz, float& rx, float& ry, float& rz)
        __attribute__((always_inline)) {
      wait_ge(f_chain, sc + 1, seen_chain);
      const float* ro = ring_out + (sc % DO) * 4 * TB + tj;
      const float x = ro[0], y = ro[TB], cx = ro[2 * TB], cy = ro[3 * TB];
      lx = ly = lz = rx = ry = rz = 0.f;
      if constexpr (PROJ == 3) {
        lx = x + cx;
        ly = y + cy;
        lz = dem.template point<false>(lx, ly, nobad);
        rx = x - cx;
        ry = y - cy;
        rz = dem.template point<false>(rx, ry, nobad);
      }
      if constexpr (DUMP) {
        if (valid) {
          const size_t o3 = ((size_t)kl * H + sc) * 3;
          if (a.d_lw) { a.d_lw[o3] = lx; a.d_lw[o3 + 1] = ly; a.d_lw[o3 + 2] = lz; }
          if (a.d_rw) { a.d_rw[o3] = rx; a.d_rw[o3 + 1] = ry; a.d_rw[o3 + 2] = rz; }
        }
      }
    };
    // even step sc in set X (other set Y): the term of (sc - 4, sc - 2) = (X, Y), then X = sc
    auto wstep = [&](auto x_is_a, int sc) __attribute__((always_inline)) {
      constexpr bool XA = decltype(x_is_a)::value;
      float& Xlx = XA ? Alx : Blx; float& Xly = XA ? Aly : Bly; float& Xlz = XA ? Alz : Blz;
      float& Xrx = XA ? Arx : Brx; float& Xry = XA ? Ary : Bry; float& Xrz = XA ? Arz : Brz;
      const float& Ylx = XA ? Blx : Alx; const float& Yly = XA ? Bly : Aly; const float& Ylz = XA ? Blz : Alz;
      const float& Yrx = XA ? Brx : Arx; const float& Yry = XA ? Bry : Ary; const float& Yrz = XA ? Brz : Arz;
      const int i = sc - 4;
      if (i >= 0 && i < H - 3) {
        const float term = slope_term<false>(Xlx, Xly, Xlz, Ylx, Yly, Ylz, Xrx, Xry, Xrz, Yrx, Yry, Yrz, nobad);
        sw = sw + term;
      }
      contacts(sc, Xlx, Xly, Xlz, Xrx, Xry, Xrz);
      if constexpr (DUMP) {  // odd-step contacts are written for the dump only
        if (sc + 1 < H) {
          float lx, ly, lz, rx, ry, rz;
          contacts(sc + 1, lx, ly, lz, rx, ry, rz);
        }
        lds_store_release(f_wheel, min(sc + 2, H));
      } else {
        // the odd step's slot is not read here: release it with the even one
        lds_store_release(f_wheel, min(sc + 2, H));
      }
    };
    int sc = 0;
    for (; sc + 2 < H; sc += 4) {
      wstep(T_{}, sc);
      wstep(F_{}, sc + 2);
    }
    if (sc < H) {
      wstep(T_{}, sc);
      sc += 2;
    }
    // sc - 2 = the last even step processed; its set is A if (sc - 2) % 4 == 0
    const int last = sc - 2;
    const int i = last - 2;  // the term (last - 2, last)
    if (i >= 0 && i < H - 3) {
      const float term = (last % 4 == 0)
          ? slope_term<false>(Blx, Bly, Blz, Alx, Aly, Alz, Brx, Bry, Brz, Arx, Ary, Arz, nobad)
          : slope_term<false>(Alx, Aly, Alz, Blx, Bly, Blz, Arx, Ary, Arz, Brx, Bry, Brz, nobad);
      sw = sw + term;
    }
    sw_lds[tj] = sw;
  } else {
    // ---------------- costmap gather (used one step later), path-follow, speed, obstacle
    int seen_chain = 0;
    float pf_sum = 0.f, ob = 0.f, last_x = a.x0, last_y = a.y0;
    float cmA = 0.f, cmB = 0.f;  // costmap value of the even / odd step
    Recip rcm;
    rcm.b = a.res_c;
    auto cstep = [&](int sc, float& cm_mine, float& cm_prev) __attribute__((always_inline)) {
      wait_ge(f_chain, sc + 1, seen_chain);
      const float* ro = ring_out + (sc % DO) * 4 * TB + tj;
      const float x = ro[0], y = ro[TB];
      cm_mine = a.cm[costmap_index<false>(a.cm_size, a.hw, rcm, x, y, nobad, a.rinv_res_c, a.cdiv_res_c)];
      const float pft = pf_sum + 10.0f * (fabsf(x - a.gx) + fabsf(y - a.gy));
      pf_sum = (sc < H - 1) ? pft : pf_sum;  // _path_follow_critic sum over t < H-1
      last_x = x;
      last_y = y;
      // _avoid_obstacle: the costmap value gathered one step earlier (step sc - 1)
      const float ob1 = (cm_prev > a.thr) ? ob + a.pen : ob;
      ob = (sc > 0) ? ob1 + cm_prev : ob;
      if constexpr (DUMP) {
      }
      lds_store_release(f_cost, sc + 1);
    };
    int sc = 0;
    for (; sc + 1 < H; sc += 2) {
      cstep(sc, cmA, cmB);
      cstep(sc + 1, cmB, cmA);
    }
    if (sc < H) cstep(sc, cmA, cmB);
    const float cm_last = ((H - 1) & 1) ? cmB : cmA;
    if (cm_last > a.thr) ob = ob + a.pen;  // last step's obstacle term
    ob = ob + cm_last;
    float pf;  // _evaluate_trajectories_kernel (critics_warp.py:325-329)
    if (a.pf_far) {
      const float dx = last_x - a.igx, dy = last_y - a.igy;
      pf = (dx * dx + dy * dy) * a.pf_scale;
    } else {
      pf = pf_sum;
    }
    c_pf = pf;
    c_ob = ob;
  }
  __syncthreads();  // WHEEL's slope sums are in sw_lds
  if (clk_wg) a.clk[5] = __builtin_amdgcn_s_memrealtime();  // every role of workgroup 0 done
  if (role == ROLE_COST) {  // critics_warp.py:325-329, this f32 add order
    float cost = a.w_path * c_pf;
    cost = cost + a.w_slope * sw_lds[tj];
    cost = cost + a.w_speed * cost_lds[tj];  // (the producer's speed critic sum)
    cost = cost + a.w_obs * c_ob;
    if (valid) a.cost_out[kl] = cost;
    cost_lds[tj] = valid ? cost : INFINITY;
  }
  __syncthreads();
  if constexpr (MODE == 0)  // rows hold the normals; the leaf recomputes the sampled controls
    leaf_records<TB, NT, true, FUSED>(a, cost_lds, scratch, a.eps + (size_t)blk * (2 * H) * TB, unom_lds,
                                      ucache, a.ucache_steps, blk);
  else
    leaf_records<TB, NT, false, FUSED>(a, cost_lds, scratch, a.ustore + (size_t)blk * (2 * H) * TB, nullptr, nullptr,
                                       0, blk);
  if (clk_wg) a.clk[6] = __builtin_amdgcn_s_memrealtime();  // workgroup 0's leaf record written
  if (clk_any) a.clk[kClkBase + 2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  if constexpr (FUSED) {  // the record is written through: count it (D8: complete, then a relaxed count)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      *ticket_lds = (int)__hip_atomic_fetch_add(rec_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return *ticket_lds;
  }
  return -1;
}

// One workgroup per CU at most: a grid smaller than the blocks runs them in turn (block blockIdx.x,
// + gridDim.x, ...), each a whole role-split rollout and leaf record.
template <int TB, int PROJ, int MODE, bool DUMP>
__global__ __launch_bounds__(NROLES * TB) void mppi_rollout_roles_kernel(const RolloutArgs a_in) {
  RolloutArgs a = a_in;
  const int nblk = (int)((a.K + TB - 1) / TB);
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    roles_body<TB, PROJ, MODE, DUMP, false>(a, blk, nullptr);
    if (blk + (int)gridDim.x < nblk) __syncthreads();  // (the next block reuses the LDS)
  }
}

// =====================================================================  finish kernel
// One workgroup.  (1) Binary tree over n records (padded to a power of two with
// empty records): passes combining aligned groups of 8 (three tree levels) while
// more than 32 nodes remain, then the last levels in LDS.  (2) MODE 0 writes the
// root (rank record); MODE 1 computes u_opt = V/S, the optimal filter
// (MPPI_isaac.py:672-692) and the 3D rollout of the optimal sequence (:696-720):
// only the serial chain (chain3d) runs on one lane, sin/cos, heights and wheel
// contacts are computed by all lanes around it.
constexpr int FIN_THREADS = 1024;
constexpr int FIN_LDS_NODES = 16;
constexpr int FIN_GROUP_CHUNK = 64;    // groups per scale-table fill (15 PairScale + 16 m each)

__device__ __forceinline__ void group8_scales(const float (&m)[8], float T, PairScale (&ps)[7]) {
  group_scales<8>(m, T, ps);
}
__device__ __forceinline__ double group8_apply(const PairScale* ps, const double (&v)[8], int j) {
  return group_apply<8>(ps, v, j);
}

// Robot pose with the heading projected on the DEM (projection_warp.py:306-310).
__device__ __forceinline__ Traj initial_pose(const FinishArgs& f, const Dem& dem, const float* qpre = nullptr) {
  const float res_half_neg = (-f.res) / 2.0f;
  const float res_sq = f.res * f.res;
  Traj s;
  s.x = f.x0;
  s.y = f.y0;
  bool unused = false;
  float q[4];
  if (qpre) {  // the corners, loaded when the finish started (same cell: corners<false> of (x0, y0))
    q[0] = qpre[0];
    q[1] = qpre[1];
    q[2] = qpre[2];
    q[3] = qpre[3];
  } else {
    dem.template corners<false>(s.x, s.y, q, unused);
  }
  const float vx = res_half_neg * (((q[1] - q[0]) - q[2]) + q[3]);
  const float vy = res_half_neg * (((q[2] - q[0]) - q[1]) + q[3]);
  const float nn = sqrtf((vx * vx + vy * vy) + res_sq * res_sq);
  const float nx = vx / nn, ny = vy / nn, nz = res_sq / nn;
  const float h0x = f.h0x, h0y = f.h0y, h0z = f.h0z;
  const float d = (h0x * nx + h0y * ny) + h0z * nz;
  const float tx = h0x - d * nx, ty = h0y - d * ny, tz = h0z - d * nz;
  const float tn = sqrtf((tx * tx + ty * ty) + tz * tz);
  s.hx = tx / tn;
  s.hy = ty / tn;
  s.hz = tz / tn;
  return s;
}

// The optimal rollout's serial chain (projection_warp.py:306-326 on one trajectory) on one
// whole wave, every lane computing the same values: a lone lane waits out each step's
// normal-table load (L2 / MALL latency, about half of a step).  Instead each step's normal comes
// from the 8 x 8-cell neighbourhood of the position two steps earlier, loaded one cell per lane
// while those two steps run, and is read from the lane holding it (v_readlane); a position more
// than 3 cells from that centre loads its entry directly.  Arithmetic as the rollout chain
// (advance_step / orient_step, correctly rounded, IEEE redo out of range), so every value is
// the rollout chain's.  Inputs: in4[t] = (v[t + 1], sin, cos, 1 - cos of step t) (v[H - 1] in the last
// row) and in4[H].x = v[0], one LDS read per step.  Writes x, y, n, the new heading of each step into
// chain[8 t ..].
constexpr int TAIL_WIN = 8, TAIL_WIN_LO = 3;  // neighbourhood cells [c - 3, c + 4] per axis
// Every lane computes the same values, so the lane holding a step's cell is found by comparing each
// lane's table offset with the cell's (one compare, a ballot, the first set bit): the control flow is
// uniform (a scalar branch on the ballot), and a lane whose clamped neighbour repeats another's holds
// the same entry (the offset ti - tjj (grid + 1) is one-to-one on the clamped cells).  The rest of the
// step is the rollout chain's (orient_step, then advance_step<true, false> of the next position, both
// redone with IEEE operators if the guards fail).  Each step's v / sin / cos are read one step ahead.
// Every lane stores the step's record (same values, same LDS words).
__device__ __forceinline__ void tail_chain_3d(const FinishArgs& f, const Dem& dem, const float4* in4, float* chain,
                                              int H, int lane, const float* qpre) {
  const f2 cell_off = f2{-f.x_min, f.y_min};
  const float fi_hi = (float)(f.grid - 1), fj_lo = (float)(1 - f.rows);
  const float4* ntab0 = dem.N + (f.grid + 2);  // entry (jj, ii) = (1 - tjj, ti + 1): offset ti - tjj * (grid + 1)
  const int nrow = f.grid + 1;
  const int ldx = (lane % TAIL_WIN) - TAIL_WIN_LO, ldy = (lane / TAIL_WIN) - TAIL_WIN_LO;
  // (ti, tjj) of the cell holding pos: min(i, grid - 1), -min(j, rows - 1) (Dem::cell)
  auto cell_of = [&](f2 pos, int& ti, int& tjj) __attribute__((always_inline)) {
    f2 q;
    if (dem.cdiv) {
      const f2 aa = pos + cell_off;
      const f2 q0 = aa * bc2(dem.rinv);
      const f2 r = pk_fma(-q0, bc2(dem.res), aa);
      q = pk_fma(r, bc2(dem.rinv), q0);
    } else {
      q = f2{(pos.x - f.x_min) / f.res, (pos.y + f.y_min) / f.res};
    }
    ti = (int)__builtin_amdgcn_fmed3f(q.x, -1.0f, fi_hi);
    tjj = (int)__builtin_amdgcn_fmed3f(q.y, fj_lo, 1.0f);
  };
  // this lane's cell of the neighbourhood centred on (ti, tjj): its table offset, load issued
  // (|tjj|, nrow < 2^23 and the table < 4 GiB: 24-bit multiplies, as the rollout chain)
  auto issue = [&](int ti, int tjj, int& lo, float4& w) __attribute__((always_inline)) {
    const int ci = min(max(ti + ldx, -1), f.grid - 1);
    const int cj = min(max(tjj + ldy, 1 - f.rows), 1);
    lo = ci - __mul24(cj, nrow);
    w = ntab0[lo];
  };
  // the normal of (ti, tjj): from the lane holding it, else loaded
  auto pick = [&](int ti, int tjj, int lo, const float4& w) __attribute__((always_inline)) {
    const int to = ti - __mul24(tjj, nrow);
    const uint64_t hit = __builtin_amdgcn_ballot_w64(lo == to);
    float3 n;
    if (hit) {
      const int src = __builtin_ctzll(hit);
      n.x = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, w.x), src));
      n.y = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, w.y), src));
      n.z = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, w.z), src));
    } else {  // outside the neighbourhood: a load of the entry
      const float4 d = ntab0[to];
      n = make_float3(d.x, d.y, d.z);
    }
    return n;
  };
  const Traj s0 = initial_pose(f, dem, qpre);
  Head hd{f2{s0.hx, s0.hy}, s0.hz};
  f2 pos = f2{s0.x, s0.y};
  {  // step 0's position (guarded: the heading comes from the IEEE initial pose)
    Lean la;
    lean_init(la);
    const float v0 = in4[H].x;
    f2 p = advance_step<true>(hd, v0, f.dt, pos, la);
    if (__builtin_expect(lean_bad(la), 0)) p = advance_step<false>(hd, v0, f.dt, pos, la);
    pos = p;
  }
  int ti, tjj;
  cell_of(pos, ti, tjj);
  int loA, loB;  // neighbourhoods of steps 0 and 1: around step 0
  float4 wA, wB;
  issue(ti, tjj, loA, wA);
  loB = loA;
  wB = wA;
  float4 inn = in4[0];
  // step t (position known, its cell (ti, tjj)): normal from neighbourhood X (centred two steps
  // back), refill X around this cell for step t + 2, orientation, record, next position and cell
  auto step = [&](auto more_tag, int t, int& loX, float4& wX) __attribute__((always_inline)) {
    constexpr bool more = decltype(more_tag)::value;
    const float v1 = inn.x, sn = inn.y, cs = inn.z, omc = inn.w;
    if constexpr (more) inn = in4[t + 1];  // the next step's inputs, one step ahead
    const float3 n = pick(ti, tjj, loX, wX);
    issue(ti, tjj, loX, wX);
    const f2 nxy = f2{n.x, n.y};
    Lean l;
    lean_init(l);
    Head ho = orient_step<true>(nxy, n.z, hd, sn, cs, omc, l);
    f2 p1 = pos;
    if constexpr (more) p1 = advance_step<true, false>(ho, v1, f.dt, pos, l);
    if (__builtin_expect(lean_bad(l), 0)) {
      ho = orient_step<false>(nxy, n.z, hd, sn, cs, omc, l);
      if constexpr (more) p1 = advance_step<false>(ho, v1, f.dt, pos, l);
    }
    float* ch = chain + 8 * t;
    ch[0] = pos.x; ch[1] = pos.y;
    ch[2] = n.x; ch[3] = n.y; ch[4] = n.z;
    ch[5] = ho.xy.x; ch[6] = ho.xy.y; ch[7] = ho.z;
    hd = ho;
    if constexpr (more) {
      pos = p1;
      cell_of(pos, ti, tjj);
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  int t = 0;
  for (; t + 2 < H; t += 2) {
    step(T_{}, t, loA, wA);
    step(T_{}, t + 1, loB, wB);
  }
  if (t + 1 < H) {
    step(T_{}, t, loA, wA);
    step(F_{}, t + 1, loB, wB);
  } else {
    step(F_{}, t, loA, wA);
  }
}

// Step 0 of the optimal rollout on one lane (no barrier): traj | hv | lw | rw of the
// first step into out[0..12), the layout optimal_rollout uses for nsteps = 1.
__device__ __forceinline__ void first_step(const FinishArgs& f, const Dem& dem, float v, float sn, float cs,
                                           float* out, const float* qpre) {
  const float res_half_neg = (-f.res) / 2.0f;
  const float res_sq = f.res * f.res;
  Traj s = initial_pose(f, dem, qpre);
  const Traj saved = s;
  float q[4], nx, ny, nz;
  bool bad = false;
  chain3d<kChainFast>(dem, res_half_neg, res_sq, f.dt, v, sn, cs, s, q, nx, ny, nz, bad);
  if (kChainFast && __builtin_expect(bad, 0)) {
    s = saved;
    chain3d<false>(dem, res_half_neg, res_sq, f.dt, v, sn, cs, s, q, nx, ny, nz, bad);
  }
  StepOut o;
  bool bad2 = false;
  wheels3d<false>(dem, f.off, s.x, s.y, q, nx, ny, nz, s.hx, s.hy, s.hz, o, bad2);
  out[0] = s.x; out[1] = s.y; out[2] = o.z;
  out[3] = s.hx; out[4] = s.hy; out[5] = s.hz;
  out[6] = o.lx; out[7] = o.ly; out[8] = o.lz;
  out[9] = o.rx; out[10] = o.ry; out[11] = o.rz;
}

// The 3D rollout of the optimal sequence for `nsteps` steps from the robot pose
// (projection_warp.py:306-348 on one trajectory): the serial chain on wave 0 (8 floats per step
// into LDS `chain`, 16-byte aligned), then heights and wheel contacts on all lanes.  Writes
// traj[3n] | hv[3n] | lw[3n] | rw[3n] at `out`.
__device__ __forceinline__ void optimal_rollout(const FinishArgs& f, const Dem& dem, const float4* in4, float* chain,
                                                int nsteps, float* out, int tid, int nthreads,
                                                const float* qpre = nullptr) {
  if (tid < 64) tail_chain_3d(f, dem, in4, chain, nsteps, tid, qpre);  // the serial chain, wave 0
  __syncthreads();
  for (int t = tid; t < nsteps; t += nthreads) {  // heights + wheel contacts, all lanes
    const float4 ca = reinterpret_cast<const float4*>(chain)[2 * t], cb = reinterpret_cast<const float4*>(chain)[2 * t + 1];
    const float ch[8] = {ca.x, ca.y, ca.z, ca.w, cb.x, cb.y, cb.z, cb.w};  // x, y, n, heading
    float q[4];
    {  // the chain read the normal table: corners here
      bool unused = false;
      dem.template corners<false>(ch[0], ch[1], q, unused);
    }
    StepOut o;
    bool bad = false;
    wheels3d<kFastMath>(dem, f.off, ch[0], ch[1], q, ch[2], ch[3], ch[4], ch[5], ch[6], ch[7], o, bad);
    if (kFastMath && bad)
      wheels3d<false>(dem, f.off, ch[0], ch[1], q, ch[2], ch[3], ch[4], ch[5], ch[6], ch[7], o, bad);
    float* o_traj = out + 3 * t;
    float* o_hv = out + 3 * nsteps + 3 * t;
    float* o_lw = out + 6 * nsteps + 3 * t;
    float* o_rw = out + 9 * nsteps + 3 * t;
    o_traj[0] = ch[0]; o_traj[1] = ch[1]; o_traj[2] = o.z;
    o_hv[0] = ch[5]; o_hv[1] = ch[6]; o_hv[2] = ch[7];
    o_lw[0] = o.lx; o_lw[1] = o.ly; o_lw[2] = o.lz;
    o_rw[0] = o.rx; o_rw[1] = o.ry; o_rw[2] = o.rz;
  }
}

// Publish f.seq once every output is in host memory.  The outputs were stored with
// system-scope (write-through) atomic stores, so completing them (vmcnt) is enough:
// no cache write-back, whose cost grows with whatever else is dirty in L2 (e.g. the
// next step's normals being generated on other CUs).
__device__ __forceinline__ void store_out(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Every wave's stores (outputs, nominal sequence, tail inputs; all write-through) complete, then the
// completion word (the host launches a resident server's deferred tail after seeing it).
__device__ __forceinline__ void signal_done(const FinishArgs& f) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && f.done) __hip_atomic_store(f.done, f.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Phase 2 of the finish (MPPI_isaac.py:655-720): `ures` = u_opt[tid] for tid < 2H
// (V/S of the root record); the optimal-sequence filter, the outputs, and the
// optimal rollout (whole, or step 0 with the rest deferred, f.mode 2), then the
// completion word.  Called by all `nthreads` threads of one workgroup; smem holds
// uo[2][PS] in4[4(H + 1)] chain[8H] out[16H] lr[2][PS] floats (<= fin_phase2_floats).
// qpre: the DEM corners of the robot's cell, loaded at the start of the finish by waves 0 and
// nthreads / 64 - 1 (the waves that use them here), or nullptr.
__device__ __forceinline__ void finish_phase2(const FinishArgs& f, float ures, unsigned char* smem, int tid,
                                              int nthreads, const float* qpre = nullptr) {
  const int H = f.H;
  const int PS = fin_plane_stride(H);
  float* uo = reinterpret_cast<float*>(smem);  // [2][PS]: the L inputs, then the R inputs
  float4* in4 = reinterpret_cast<float4*>(uo + 2 * PS);  // [H + 1]: the optimal rollout's inputs
  float* chain = reinterpret_cast<float*>(in4 + H + 1);  // [H][8]: x, y, nx, ny, nz, hx, hy, hz
  // outputs are staged here and stored to f.out (pinned host memory) in one burst at the
  // end: a workgroup barrier after host stores would wait for their PCIe round trip
  float* ostage = chain + 8 * H;  // [16H]
  float* lrp = ostage + 16 * H;    // [2][PS]: the filtered L, then R (16-byte aligned)
  const int nout = f.mode == 2 ? 4 * H + 12 : 16 * H;
  const float one_m_a = 1.0f - f.oa;
  if (tid < 2 * H) {
    // written through (agent scope): the resident server's next step reads it in the same launch
    __hip_atomic_store(f.u_nom_next + tid, ures, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ostage[tid] = ures;
    // optimal-sequence wheel filter (sampling_warp.py:120-138, k=3.0, a=0.92): the
    // inputs (u*k)*(1-a) in parallel, only the recurrences L = L*a + in on two lanes
    uo[tid < H ? tid : PS + (tid - H)] = (ures * f.ok) * one_m_a;
  }
  __syncthreads();
  Dem dem;
  dem.init(f.Z, f.rows, f.grid, f.x_min, f.y_min, f.res, f.rinv_res, f.cdiv_res);
  dem.N = f.ntab;
  const int lane = tid & 63, wave = tid >> 6;
  if (wave == 0) {
    if (lane < 2) {
      // The two recurrences L = L a + in_L (lane 0) and R = R a + in_R (lane 1), one v_mul and one
      // v_add per step (the reference's two IEEE roundings), each lane over its own planar row.
      // A lone wave's LDS instructions cost far more issue time than its VALU ones (one lane
      // packing (L, R) with a read and a write per two steps: ~44 cycles per step against ~23
      // here, profiles/ubench/filt.hip), so every LDS access moves 4 steps (ds_read/write_b128):
      // two blocks of 16 steps per iteration, each block's inputs read one block before it runs
      // (the read-ahead stays inside the row's PS >= H + 32 floats), results written after it
      const f4* p = reinterpret_cast<const f4*>(uo + lane * PS);
      f4* q = reinterpret_cast<f4*>(lrp + lane * PS);
      const float a = f.oa;
      float x = lane ? f.wr : f.wl;
      f4 A[4], B[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) A[k] = p[k];
      int t = 0;
      for (; t + 32 <= H; t += 32, p += 8, q += 8) {
#pragma unroll
        for (int k = 0; k < 4; ++k) B[k] = p[4 + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          x = x * a + A[k].x;
          A[k].x = x;
          x = x * a + A[k].y;
          A[k].y = x;
          x = x * a + A[k].z;
          A[k].z = x;
          x = x * a + A[k].w;
          A[k].w = x;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = A[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) A[k] = p[8 + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          x = x * a + B[k].x;
          B[k].x = x;
          x = x * a + B[k].y;
          B[k].y = x;
          x = x * a + B[k].z;
          B[k].z = x;
          x = x * a + B[k].w;
          B[k].w = x;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) q[4 + k] = B[k];
      }
      const float* pf = reinterpret_cast<const float*>(p);
      float* qf = reinterpret_cast<float*>(q);
      for (int k = 0; t < H; ++t, ++k) {
        x = x * a + pf[k];
        qf[k] = x;
      }
    }
  } else if (wave == nthreads / 64 - 1 && f.mode == 2) {
    if (lane == 0) {  // step 0 of the optimal rollout needs only the first filter step
      const float L0 = f.wl * f.oa + uo[0], R0 = f.wr * f.oa + uo[PS];
      const float v0 = clampf((L0 + R0) / 2.0f, f.vmin, f.vmax);
      const float w0 = clampf(((-L0) + R0) / f.rwheel, f.wmin, f.wmax);
      float sn0, cs0;
      dm_sincosf(w0 * f.dt, &sn0, &cs0);
      first_step(f, dem, v0, sn0, cs0, ostage + 4 * H, qpre);
    }
  }
  __syncthreads();
  for (int t = tid; t < H; t += nthreads) {
    const float L = lrp[t], R = lrp[PS + t];
    const float v = clampf((L + R) / 2.0f, f.vmin, f.vmax);
    const float w = clampf(((-L) + R) / f.rwheel, f.wmin, f.wmax);
    float sn, cs;
    dm_sincosf(w * f.dt, &sn, &cs);
    in4[t].y = sn;
    in4[t].z = cs;
    in4[t].w = 1.0f - cs;
    in4[t > 0 ? t - 1 : H].x = v;  // v of step t in the row before (v[0]: row H)
    if (t == H - 1) in4[t].x = v;
    ostage[2 * H + t] = v;
    ostage[3 * H + t] = w;
    if (f.mode == 2) {  // inputs of the deferred optimal rollout (mppi_tail_kernel), written through
      __hip_atomic_store(f.tail_in + t, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(f.tail_in + H + t, sn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(f.tail_in + 2 * H + t, cs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  // mode 1: the whole optimal rollout; mode 2: its first step only (the pose the
  // closed loop needs now), the rest runs in mppi_tail_kernel on a side stream
  if (f.mode != 2) optimal_rollout(f, dem, in4, chain, H, ostage + 4 * H, tid, nthreads, qpre);
  __syncthreads();
  for (int i = tid; i < nout; i += nthreads) store_out(f.out + i, ostage[i]);
  signal_done(f);
}

__global__ __launch_bounds__(FIN_THREADS) void mppi_finish_kernel(const FinishArgs f) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int tid = threadIdx.x;
  const int H = f.H;
  const int E = 2 * H + 2;
  // ---------------- (1) tree
  // LDS during the tree: [FIN_LDS_NODES][E] doubles, then PairScale table
  double* lnode = reinterpret_cast<double*>(smem_raw);
  PairScale* lps = reinterpret_cast<PairScale*>(smem_raw + (size_t)FIN_LDS_NODES * E * sizeof(double));
  const double* cur = f.recs;
  int n = f.n_recs;
  double* bufs[2] = {f.scratch0, f.scratch1};
  int flip = 0;
  if (gridDim.x > 1) {
    // first level on gridDim.x workgroups: workgroup b combines records [16b, 16b+16) into
    // f.level1[b]; the last to finish (device-scope counter) carries on with the rest
    const int b = blockIdx.x;
    const int gsize = min(16, n - 16 * b);
    float* lm = reinterpret_cast<float*>(lps + 15);
    if (tid < 16) lm[tid] = (tid < gsize) ? (float)cur[(size_t)(16 * b + tid) * E] : INFINITY;
    __syncthreads();
    int base = 0;
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1) {
      PairScale p;
      if (tid < w) {
        p = pair_scale(lm[2 * tid], lm[2 * tid + 1], f.T);
        lps[base + tid] = p;
      }
      __syncthreads();
      if (tid < w) lm[tid] = p.m;
      __syncthreads();
      base += w;
    }
    // device-scope stores write through the XCD's L2, so no fence has to write the whole
    // (rollout-dirty) L2 back: completion of these stores (vmcnt) orders them before the count
    for (int j = tid; j < E; j += FIN_THREADS) {
      double v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = cur[(size_t)(16 * b + min(i, gsize - 1)) * E + j];
      __hip_atomic_store(f.level1 + (size_t)b * E + j, group_apply<16>(lps, v, j), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lm + 16);
    if (tid == 0) {
      const unsigned prev = __hip_atomic_fetch_add(f.level1_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == gridDim.x - 1;
      if (last) __hip_atomic_store(f.level1_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    // the level-1 records, read at device scope (past any stale copy in this XCD's L2)
    n = gridDim.x;
    if (tid < 16) lm[tid] = (tid < n) ? (float)__hip_atomic_load(f.level1 + (size_t)tid * E, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT)
                                      : INFINITY;
    __syncthreads();
    if (n <= 16) {
      int base2 = 0;
#pragma unroll
      for (int w = 8; w >= 1; w >>= 1) {
        PairScale p;
        if (tid < w) {
          p = pair_scale(lm[2 * tid], lm[2 * tid + 1], f.T);
          lps[base2 + tid] = p;
        }
        __syncthreads();
        if (tid < w) lm[tid] = p.m;
        __syncthreads();
        base2 += w;
      }
      for (int j = tid; j < E; j += FIN_THREADS) {
        double v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i)
          v[i] = __hip_atomic_load(f.level1 + (size_t)min(i, n - 1) * E + j, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        lnode[j] = group_apply<16>(lps, v, j);
      }
      n = 1;
      __syncthreads();
      goto root_ready;
    }
    __threadfence();  // more than 256 level-1 records: the general passes below read them plainly
    cur = f.level1;
  }
  while (n > FIN_LDS_NODES) {  // global -> global, aligned groups of 16 (4 tree levels)
    const int groups = (n + 15) >> 4;
    double* out = bufs[flip];
    for (int g0 = 0; g0 < groups; g0 += FIN_GROUP_CHUNK) {
      const int ng = min(FIN_GROUP_CHUNK, groups - g0);
      // pair scales of the chunk's groups, level by level: lm[ng][16] -> lps[ng][15]
      float* lm = reinterpret_cast<float*>(lps + FIN_GROUP_CHUNK * 15);
      for (int i = tid; i < ng * 16; i += FIN_THREADS) {
        const int r = 16 * g0 + i;
        lm[i] = (r < n) ? (float)cur[(size_t)r * E] : INFINITY;
      }
      __syncthreads();
      int base = 0;
#pragma unroll
      for (int w = 8; w >= 1; w >>= 1) {
        PairScale p;
        const int gl = tid / w, pi = tid - gl * w;
        const bool act = tid < ng * w;
        if (act) {
          p = pair_scale(lm[gl * 16 + 2 * pi], lm[gl * 16 + 2 * pi + 1], f.T);
          lps[gl * 15 + base + pi] = p;
        }
        __syncthreads();
        if (act) lm[gl * 16 + pi] = p.m;
        __syncthreads();
        base += w;
      }
      // every element of every group, two items per thread with all 32 loads in flight
      for (int it0 = tid; it0 < ng * E; it0 += 2 * FIN_THREADS) {
        double v[2][16];
#pragma unroll
        for (int q = 0; q < 2; ++q) {  // clamped, unconditional loads (empty members are skipped
          const int it = min(it0 + q * FIN_THREADS, ng * E - 1);  // by their pair scales)
          const int gl = it / E, j = it - gl * E;
          const int r0 = 16 * (g0 + gl);
#pragma unroll
          for (int i = 0; i < 16; ++i) v[q][i] = cur[(size_t)min(r0 + i, n - 1) * E + j];
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int it = it0 + q * FIN_THREADS;
          if (it < ng * E) {
            const int gl = it / E, j = it - gl * E;
            out[(size_t)(g0 + gl) * E + j] = group_apply<16>(lps + gl * 15, v[q], j);
          }
        }
      }
      __syncthreads();
    }
    cur = out;
    n = groups;
    flip ^= 1;
  }
  // the last <= 16 records: one aligned group of 16 (empty members padded) -> root in lnode[0..E)
  if (n > 1) {
    float* lm = reinterpret_cast<float*>(lps + 15);
    if (tid < 16) lm[tid] = (tid < n) ? (float)cur[(size_t)tid * E] : INFINITY;
    __syncthreads();
    int base = 0;
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1) {
      PairScale p;
      if (tid < w) {
        p = pair_scale(lm[2 * tid], lm[2 * tid + 1], f.T);
        lps[base + tid] = p;
      }
      __syncthreads();
      if (tid < w) lm[tid] = p.m;
      __syncthreads();
      base += w;
    }
    for (int j = tid; j < E; j += FIN_THREADS) {
      double v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = cur[(size_t)min(i, n - 1) * E + j];
      lnode[j] = group_apply<16>(lps, v, j);
    }
    n = 1;
  } else {
    for (int j = tid; j < n * E; j += FIN_THREADS) lnode[j] = cur[j];
  }
  __syncthreads();
root_ready:
  // root = lnode[0..E) (n == 1) or empty (n == 0)
  if (f.mode == 0) {
    for (int j = tid; j < E; j += FIN_THREADS)
      f.record_out[j] = (n == 1) ? lnode[j] : (j == 0 ? (double)INFINITY : 0.0);
    return;
  }
  // ---------------- (2) optimal sequence
  const double S = (n == 1) ? lnode[1] : 0.0;
  // u_opt = V / S (DEFINED; zero when no trajectory has a finite cost)
  const float ures = (tid < 2 * H && S > 0.0) ? (float)(lnode[2 + tid] / S) : 0.0f;
  __syncthreads();  // lnode is dead from here on
  finish_phase2(f, ures, smem_raw, tid, FIN_THREADS);
}

// ---------------------------------------------------------------------  column-split finish
// The same tree as mppi_finish_kernel (D2: binary, adjacent pairs, leaves padded with
// empty records to a power of two P >= 16; an empty member passes its partner through,
// so the padding does not change the root), split by COLUMN instead of by record: every
// workgroup builds the whole pair-scale table from the n leaf minima (it depends on
// nothing else) and reduces its own slice of the 2H+2 columns over all n records.  No
// workgroup waits for another's partial tree; the only handoff is the u_opt slice each
// stores before the device-scope counter, and the last workgroup to arrive runs phase 2.
// One round trip through global memory instead of two (level 1, then the last group) or
// more (n > 256), and every level but the 4 in registers is an LDS pass.
// LDS: PairScale[P - 1] | node minima m[2P] (all levels) | partial[ncol + 1][P / 16] doubles.
constexpr int COLFIN_PMAX = 4096;
constexpr uint64_t kColfinPollTicks = 200000000ull;  // the last workgroup's u_opt wait bound (2 s)  // leaf records (K <= 1,048,576 per context)
__device__ __forceinline__ int colfin_level_base(int P, int l) { return P - (P >> l); }

// Records written by this launch's own rollout blocks (resident server, RECS_WT) are read with
// agent-scope atomic loads: they bypass a stale line of the previous step's records in this XCD's
// L2 (the rollout blocks store them write-through).
template <bool RECS_WT, typename V>
__device__ __forceinline__ V rec_load(const V* p) {
  if constexpr (RECS_WT) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

// The column-split finish of workgroup `blk` of `nblk` (mppi_colfin_kernel, or the finish
// workgroups of the resident server, which also re-arm its record counter).  false: the last
// workgroup gave up waiting for a slice and published nothing.
template <bool RECS_WT>
__device__ __forceinline__ bool colfin_body(const FinishArgs& f, int P, int ncol, int blk, int nblk,
                                            unsigned* rec_cnt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  // the separate-launch finish (mppi_colfin_kernel: C4, C5, the K-sharded group step) outranks the
  // noise kernel of step + 2 that runs beside it: the sharded C4 step 0.1915 -> 0.179-0.180 ms
  // (profiles/r04_notes.md).  Not in the resident server (RECS_WT), whose noise runs in its own
  // workgroups after their records (there the priority measured no gain, r02_notes.md).
  if constexpr (!RECS_WT) __builtin_amdgcn_s_setprio(3);
  const int tid = thread_id<RECS_WT, FIN_THREADS>();
  const int H = f.H;
  const int E = 2 * H + 2;
  const int n = f.n_recs;
  const double* recs = f.recs;
  float qpre[4] = {0.f, 0.f, 0.f, 0.f};
  PairScale* lps = reinterpret_cast<PairScale*>(smem_raw);
  float* mlev = reinterpret_cast<float*>(lps + (P - 1));  // node minima, level l at 2P - (2P >> l)
  double* part = reinterpret_cast<double*>(mlev + 2 * P);  // [ncol + 1][P / 16], 8-byte aligned (P >= 16)
  // this workgroup's columns: [c0, c1) plus column 1 (S) as slot ncol when c0 > 1
  const int c0 = blk * ncol;
  const int c1 = min(E, c0 + ncol);
  const int nc = c1 - c0;
  const bool extra_s = c0 > 1;
  const int ncols = nc + (extra_s ? 1 : 0);
  const int NG = P >> 4;  // register groups of 16 leaves per column
  // (1) the records' minima (the scale table waits on them; thread t < T owns the L consecutive
  //     records [t L, t L + L)), then the leaf values of the (column, group) items on other waves,
  //     whose latency overlaps the table
  const int L = P > FIN_THREADS ? P / FIN_THREADS : 1;  // 1, 2 or 4 (P <= COLFIN_PMAX)
  const int T = P / L;
  float lm[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
  // (2) pair scales: first the node minima (the m pair_scale forms; level l of the minima at
  //     mlev + 2P - (2P >> l), level 0 the records): a thread's own records, then lane shuffles
  //     inside the wave, then the waves' minima on wave 0 (two barriers, not log2 P); then every
  //     node's pair scale in one pass, so the exponentials of all levels run side by side
  auto lev = [&](int l) __attribute__((always_inline)) { return mlev + (2 * P - ((2 * P) >> l)); };
  float mm = INFINITY;
  int ml = 0;  // the level mm belongs to
  if (tid < T) {  // (loads and their use in one branch: no load of it is pending past the join)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = tid * L + k;
      if (k < L && r < n)
        lm[k] = f.rec_m ? rec_load<RECS_WT>(f.rec_m + r) : (float)rec_load<RECS_WT>(recs + (size_t)r * E);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < L) lev(0)[tid * L + k] = lm[k];
    if (L == 1) {
      mm = lm[0];
    } else if (L == 2) {
      mm = fminf(lm[0], lm[1]);
      lev(1)[tid] = mm;
    } else {
      const float m01 = fminf(lm[0], lm[1]), m23 = fminf(lm[2], lm[3]);
      lev(1)[2 * tid] = m01;
      lev(1)[2 * tid + 1] = m23;
      mm = fminf(m01, m23);
      lev(2)[tid] = mm;
    }
  }
  ml = L == 1 ? 0 : (L == 2 ? 1 : 2);
  // the robot cell's DEM corners for phase 2's initial pose, loaded now by the two waves that use
  // them there (only the last workgroup does), so that load is off phase 2's serial path; after the
  // minima (a wave's loads complete in order: wave 0's minima no longer wait behind them)
  {
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (f.mode != 0 && (w == 0 || w == FIN_THREADS / 64 - 1)) {
      Dem d0;
      d0.init(f.Z, f.rows, f.grid, f.x_min, f.y_min, f.res, f.rinv_res, f.cdiv_res);
      bool unused = false;
      d0.template corners<false>(f.x0, f.y0, qpre, unused);
    }
  }
  // the items on the LAST waves (a column's groups in consecutive lanes), clear of the waves
  // that load the minima where they fit: a wave's loads complete in order, and behind a branch
  // the compiler waits for all of them (vmcnt(0)) before using the minima
  const int items = ncols * NG;  // <= FIN_THREADS (colfin_shape)
  const int item_base = FIN_THREADS - ((items + 63) & ~63);
  const int it = max(tid - item_base, 0);
  const int it_g = it % NG, it_c = it / NG;
  const bool has_item = tid >= item_base && tid - item_base < items;
  const int col = (it_c < nc) ? c0 + it_c : 1;
  double v[16];
  if (has_item) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = min(16 * it_g + i, n - 1);
      v[i] = rec_load<RECS_WT>(recs + (size_t)r * E + col);
    }
  }
  const int TW = min(T, 64);
  for (int k = 1; k < TW; k *= 2) {  // (left child first in every fminf, as pair_scale forms m)
    const float o = __shfl_xor(mm, k, 64);
    mm = (tid & k) ? fminf(o, mm) : fminf(mm, o);
    ++ml;
    if (tid < T && (tid & (2 * k - 1)) == 0) lev(ml)[tid / (2 * k)] = mm;
  }
  if (T > 64) {
    __syncthreads();  // the waves' minima (level ml, T / 64 of them)
    if (tid < 64) {
      const int NW = T >> 6;
      float x = tid < NW ? lev(ml)[tid] : INFINITY;
      int l2 = ml;
      for (int k = 1; k < NW; k *= 2) {
        const float o = __shfl_xor(x, k, 64);
        x = (tid & k) ? fminf(o, x) : fminf(x, o);
        ++l2;
        if (tid < NW && (tid & (2 * k - 1)) == 0) lev(l2)[tid / (2 * k)] = x;
      }
    }
  }
  __syncthreads();
  const int log2P = 31 - __clz(P);
  for (int g = tid; g < P - 1; g += FIN_THREADS) {
    const int r = P - g;  // level l holds nodes g with P >> (l + 1) < P - g <= P >> l
    const int l = log2P - (r <= 1 ? 0 : 32 - __clz(r - 1));
    const int i = g - colfin_level_base(P, l);
    const float* s = mlev + (2 * P - ((2 * P) >> l));
    // the register levels (l < 4, w = 8 >> l nodes per group) transposed: node k of group gi at
    // k * NG + gi, so the lanes of one column (consecutive groups) read consecutive entries
    // (group-major, their 16-byte reads hit the same banks: an up to 32-way conflict)
    const int lc = min(l, 3);  // (no division by 8 >> l = 0 above level 3)
    const int dst = l < 4 ? colfin_level_base(P, l) + (i & ((8 >> lc) - 1)) * NG + (i >> (3 - lc)) : g;
    lps[dst] = pair_scale(s[2 * i], s[2 * i + 1], f.T);
  }
  __syncthreads();
  // (3) the 4 lowest levels of every item in registers, each level's pair scales read together
  //     ahead of its arithmetic (one LDS round trip per level, not two per pair), then the
  //     scales of the shuffle levels, all at once.  (Deeper prefetch raised the fused step
  //     launch, which shares this code, from 89 to 117 VGPRs.)
  double v0 = 0.0;
  const int NGW = min(NG, 64);
  PairScale sh[6];  // the shuffle levels' scales (k = 1, 2, 4, .. < NGW)
  if (has_item) {
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int w = 8 >> l;
      PairScale cur[8];
#pragma unroll
      for (int i = 0; i < w; ++i) cur[i] = ld_scale(lps + colfin_level_base(P, l) + it_g + i * NG);
#pragma unroll
      for (int i = 0; i < w; ++i) v[i] = pair_apply_raw(cur[i], v[2 * i], v[2 * i + 1], col);
    }
    v0 = v[0];
#pragma unroll
    for (int q = 0; q < 6; ++q)
      if ((1 << q) < NGW) sh[q] = ld_scale(lps + colfin_level_base(P, 4 + q) + (it_g >> (q + 1)));
  }
  // (4a) the next levels inside a wave: a column's NG (<= 64 at a time) consecutive lanes
  //      combine by lane shuffles, left child = the lane with the bit clear (no barrier)
  int lvl = 4;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int k = 1 << q;
    if (k < NGW) {
      const double o = __shfl_xor(v0, k, 64);  // every lane: item groups are NG-aligned
      if (has_item && (it_g & (2 * k - 1)) == 0) v0 = pair_apply_raw(sh[q], v0, o, col);
      ++lvl;
    }
  }
  if (has_item && (it_g & (NGW - 1)) == 0) part[it_c * NG + it_g] = v0;
  __syncthreads();
  // (4b) levels above a wave (NG > 64) in LDS, in place (stride doubling)
  for (int stride = NGW; stride < NG; stride *= 2, ++lvl) {
    const int w = NG / (2 * stride);
    const PairScale* ps = lps + colfin_level_base(P, lvl);
    for (int it = tid; it < ncols * w; it += FIN_THREADS) {
      const int c = it % ncols, i = it / ncols;
      const int cc = (c < nc) ? c0 + c : 1;
      double* pc = part + c * NG;
      pc[2 * stride * i] = pair_apply_sel(ps[i], pc[2 * stride * i], pc[2 * stride * i + stride], cc);
    }
    __syncthreads();
  }
  // root of slot c: part[c * NG]
  if (f.mode == 0) {
    for (int c = tid; c < nc; c += FIN_THREADS) f.record_out[c0 + c] = part[c * NG];
    return true;
  }
  const double S = extra_s ? part[nc * NG] : part[(1 - c0) * NG];
  // u_opt of this slice (columns 2 + t).  One workgroup: straight from its LDS.  Several: each
  // stores its slice as tagged words {u, seq} (agent-scope atomic stores) and only the LAST
  // workgroup (blk nblk - 1: in the server the one with the last ticket) goes on: it polls the
  // 2H words until each carries this step's seq.  Value and tag travel in one 64-bit word, so
  // the handoff orders nothing across locations, and no workgroup waits for its stores to
  // complete or counts itself in (round 2-3's store, vmcnt(0), barrier, counter add, barrier).
  float ures = 0.0f;
  if (nblk == 1) {
    if (tid < 2 * H) ures = (S > 0.0) ? (float)(part[(tid + 2) * NG] / S) : 0.0f;
    __syncthreads();
    if (RECS_WT && tid == 0) __hip_atomic_store(rec_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    const unsigned long long tag = (unsigned long long)f.seq << 32;
    for (int c = tid; c < nc; c += FIN_THREADS) {
      const int j = c0 + c;
      if (j >= 2) {
        const float u = (S > 0.0) ? (float)(part[c * NG] / S) : 0.0f;
        __hip_atomic_store(f.uopt + (j - 2), tag | __builtin_bit_cast(unsigned, u), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (blk != nblk - 1) return true;
    int late = 0;
    if (tid < 2 * H) {  // bounded (2 s of the 100 MHz clock): a lost slice cannot hang the device
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      unsigned long long w = __hip_atomic_load(f.uopt + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while ((unsigned)(w >> 32) != f.seq) {
        if (__builtin_amdgcn_s_memrealtime() - t0 >= kColfinPollTicks ||
            (f.abort && __hip_atomic_load(f.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == f.seq)) {
          late = 1;  // (or another finish workgroup of the server gave up: its slice never comes)
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        w = __hip_atomic_load(f.uopt + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      ures = __builtin_bit_cast(float, (unsigned)w);
    }
    // a slice that never came: publish nothing (the host's wait reports the step as failed)
    if (__syncthreads_or(late)) return false;
    // every finish workgroup has passed its record wait (resident server): re-arm the count
    if (RECS_WT && tid == 0) __hip_atomic_store(rec_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();  // the tree's LDS is dead from here on
  finish_phase2(f, ures, smem_raw, tid, FIN_THREADS, qpre);
  return true;
}

__global__ __launch_bounds__(FIN_THREADS) void mppi_colfin_kernel(const FinishArgs f, int P, int ncol) {
  (void)colfin_body<false>(f, P, ncol, (int)blockIdx.x, (int)gridDim.x, nullptr);
}

// Deferred optimal rollout (MPPI_isaac.py:696-720) of the sequence a mode-2
// finish left in f.tail_in; launched on a side stream so that it overlaps the
// next step's rollout kernel.  Bitwise identical to the mode-1 finish.
__global__ __launch_bounds__(TAIL_THREADS) void mppi_tail_kernel(const FinishArgs f) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int tid = threadIdx.x;
  const int H = f.H;
  float4* in4 = reinterpret_cast<float4*>(smem_raw);  // [H + 1] (finish_phase2's layout)
  float* chain = reinterpret_cast<float*>(in4 + H + 1);
  if (tid == 0 && f.clk) f.clk[kClkServer + 8 * (f.seq & 7) + 4] = __builtin_amdgcn_s_memrealtime();
  // (agent-scope loads: written through by the finish; an L1 line of an earlier tail could be stale)
  auto ld = [&](int i) { return __hip_atomic_load(f.tail_in + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  for (int t = tid; t <= H; t += TAIL_THREADS) {
    if (t == H) {
      in4[H] = make_float4(ld(0), 0.f, 0.f, 0.f);
    } else {
      const float cs = ld(2 * H + t);
      in4[t] = make_float4(ld(min(t + 1, H - 1)), ld(H + t), cs, 1.0f - cs);
    }
  }
  __syncthreads();
  Dem dem;
  dem.init(f.Z, f.rows, f.grid, f.x_min, f.y_min, f.res, f.rinv_res, f.cdiv_res);
  dem.N = f.ntab;
  optimal_rollout(f, dem, in4, chain, H, f.tail_out, tid, TAIL_THREADS);
  if (tid == 0 && f.clk) f.clk[kClkServer + 8 * (f.seq & 7) + 5] = __builtin_amdgcn_s_memrealtime();
}

// =====================================================================  standalone bilinear
// Scattered-query corner lookup + bilinear (projection_warp.py:8-100) over the
// full DEM in HBM: one lane per query.
__global__ __launch_bounds__(256) void mppi_bilinear_kernel(const float* __restrict__ Z, int rows,
                                                            int grid, float x_min, float y_min,
                                                            float res, const float* __restrict__ xs,
                                                            const float* __restrict__ ys,
                                                            float* __restrict__ hs, int64_t n) {
  Dem dem;
  dem.init(Z, rows, grid, x_min, y_min, res);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float x = xs[i], y = ys[i];
    float q[4];
    bool bad = false;
    dem.template corners<true>(x, y, q, bad);
    float h = bilinear<true>(x, y, q, dem.template rr<true>(), bad);
    if (bad) {
      dem.template corners<false>(x, y, q, bad);
      h = bilinear<false>(x, y, q, dem.template rr<false>(), bad);
    }
    hs[i] = h;
  }
}

// =====================================================================  tiled bilinear (§8(d))
// Queries binned by DEM tile (BIL_TS x BIL_TS cells; launch_bin_queries): the
// workgroup of tile b stages the tile's (TS+1)^2 window (the +1 row/col holds the
// corners of the tile's last cells, clamped to the map) in LDS with row-coalesced
// loads, then streams the tile's queries: x, y in, h out, all coalesced.  Every
// DEM byte is read once and each query moves 12 bytes, the kernel's algorithmic
// traffic.  Cell index and corners follow projection_warp.py:8-48 exactly as
// Dem::corners (the same clamping), the height projection_warp.py:70-100.
constexpr int BIL_TS = BIL_TILE;
constexpr int BIL_W = BIL_TS + 1;
constexpr int BIL_T = 1024;  // threads of the lookup and binning workgroups

// corner rows (r0, r1) and columns (c0, c1) of a query, clamped as Dem::corners
__device__ __forceinline__ void query_cell(float x, float y, float x_min, float y_min, float res,
                                           float rinv, int cdiv, int rows, int grid, int& r0, int& c0,
                                           int& r1, int& c1) {
  float fi, fj;
  if (cdiv) {
    fi = cdiv_f(x - x_min, res, rinv);
    fj = cdiv_f(y + y_min, res, rinv);
  } else {
    fi = (x - x_min) / res;
    fj = (y + y_min) / res;
  }
  const int i = trunc_clamped(fi, -1.0f, (float)grid);
  const int j = -trunc_clamped(fj, -(float)rows, 1.0f);
  r0 = clampi(j, 0, rows - 1);
  c0 = clampi(i, 0, grid - 1);
  r1 = clampi(j + 1, 0, rows - 1);
  c1 = clampi(i + 1, 0, grid - 1);
}

// x / res for the bilinear fraction: the verified reciprocal where it is exact
// (|quotient| >= 2^-90, see cdiv_f), IEEE otherwise.
__device__ __forceinline__ float frac_div(float x, float res, float rinv, int cdiv) {
  if (cdiv) {
    const float q = cdiv_f(x, res, rinv);
    if (__builtin_expect(fabsf(q) >= 8.077935669463161e-28f, 1)) return q;  // 2^-90
  }
  return x / res;
}

__global__ __launch_bounds__(BIL_T) void mppi_bilinear_tiled_kernel(
    const float* __restrict__ Z, int rows, int grid, float x_min, float y_min, float res, float rinv,
    int cdiv, const float* __restrict__ xs, const float* __restrict__ ys, float* __restrict__ hs,
    const int* __restrict__ tile_off, int ntx) {
  extern __shared__ float win[];  // [BIL_W * BIL_W]
  const int tile = blockIdx.x;
  const int q0 = tile_off[tile], q1 = tile_off[tile + 1];
  if (q0 == q1) return;
  const int r0 = (tile / ntx) * BIL_TS, c0 = (tile % ntx) * BIL_TS;
  {  // stage the window: every load of a round issued before its LDS stores
    constexpr int NLD = (BIL_W * BIL_W + BIL_T - 1) / BIL_T;
    float tmp[NLD];
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = threadIdx.x + BIL_T * k;
      const int wr = idx / BIL_W, wc = idx - wr * BIL_W;
      tmp[k] = (idx < BIL_W * BIL_W) ? Z[(size_t)min(r0 + wr, rows - 1) * grid + min(c0 + wc, grid - 1)] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int idx = threadIdx.x + BIL_T * k;
      if (idx < BIL_W * BIL_W) win[idx] = tmp[k];
    }
  }
  __syncthreads();
  // BIL_UNROLL queries per thread per pass, loads issued before any is used
  constexpr int BIL_UNROLL = 4;
  for (int qb = q0 + threadIdx.x; qb < q1; qb += BIL_T * BIL_UNROLL) {
    float xv[BIL_UNROLL], yv[BIL_UNROLL];
#pragma unroll
    for (int u = 0; u < BIL_UNROLL; ++u) {
      const int q = qb + BIL_T * u;
      xv[u] = (q < q1) ? xs[q] : 0.0f;
      yv[u] = (q < q1) ? ys[q] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < BIL_UNROLL; ++u) {
      const int q = qb + BIL_T * u;
      if (q < q1) {
        const float x = xv[u], y = yv[u];
        int ra, ca, rb, cb;
        query_cell(x, y, x_min, y_min, res, rinv, cdiv, rows, grid, ra, ca, rb, cb);
        const int wa = (ra - r0) * BIL_W, wb = (rb - r0) * BIL_W;
        const float qa0 = win[wa + (ca - c0)], qa1 = win[wa + (cb - c0)];
        const float qb0 = win[wb + (ca - c0)], qb1 = win[wb + (cb - c0)];
        const float xn = frac_div(x, res, rinv, cdiv), yn = frac_div(y, res, rinv, cdiv);
        const float x2 = xn - truncf(xn), y2 = yn - truncf(yn);
        const float a0 = ((1.0f - x2) * (1.0f - y2)) * qa0;
        const float b0 = (x2 * (1.0f - y2)) * qb0;
        const float c2 = ((1.0f - x2) * y2) * qa1;
        const float d0 = (x2 * y2) * qb1;
        hs[q] = ((a0 + b0) + c2) + d0;
      }
    }
  }
}

// Binning: the tile of each query (the tile holding its first corner cell).  G chunks of the
// queries (bin_chunks), one workgroup each: an LDS histogram over the tiles, written to
// hist[g][ntiles] and added to the tile counts (one global atomic per non-empty bin per chunk
// instead of one per query); then the exclusive scan of the counts; then each chunk claims its
// run of every tile from the tile cursors (one atomic per non-empty bin) and scatters its queries
// with LDS ranks.  Order inside a tile is arbitrary; perm maps sorted position -> input index.
__device__ __forceinline__ int query_tile(float x, float y, float x_min, float y_min, float res, float rinv, int cdiv,
                                          int rows, int grid, int ntx) {
  int ra, ca, rb, cb;
  query_cell(x, y, x_min, y_min, res, rinv, cdiv, rows, grid, ra, ca, rb, cb);
  return (ra / BIL_TS) * ntx + ca / BIL_TS;
}

int bin_chunks(int64_t n, int ntiles) {
  // ~16 queries per tile and chunk (runs of 64 B in the scatter), 64 .. 2048 chunks
  const int64_t g = n / (16 * (int64_t)std::max(ntiles, 1));
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(g, std::min<int64_t>(64, (n + 1023) / 1024)), 2048));
}

__global__ __launch_bounds__(BIL_T) void mppi_bin_hist_kernel(const float* __restrict__ xs, const float* __restrict__ ys,
                                                              int64_t n, int64_t chunk, float x_min, float y_min,
                                                              float res, float rinv, int cdiv, int rows, int grid,
                                                              int ntx, int ntiles, int* __restrict__ hist,
                                                              int* __restrict__ counts) {
  extern __shared__ int lh[];  // [ntiles]
  for (int t = threadIdx.x; t < ntiles; t += BIL_T) lh[t] = 0;
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * chunk, e = min(n, b + chunk);
  for (int64_t q = b + threadIdx.x; q < e; q += BIL_T)
    atomicAdd(&lh[query_tile(xs[q], ys[q], x_min, y_min, res, rinv, cdiv, rows, grid, ntx)], 1);
  __syncthreads();
  int* gh = hist + (size_t)blockIdx.x * ntiles;
  for (int t = threadIdx.x; t < ntiles; t += BIL_T) {
    const int h = lh[t];
    gh[t] = h;
    if (h) atomicAdd(&counts[t], h);
  }
}

// exclusive scan of counts[ntiles] into off[ntiles+1]; one workgroup of 1024 threads
__global__ __launch_bounds__(1024) void mppi_bin_scan_kernel(const int* counts, int ntiles, int* off,
                                                             int* cursor) {
  __shared__ int part[1024];
  const int per = (ntiles + 1023) / 1024;
  const int b = threadIdx.x * per, e = min(b + per, ntiles);
  int sum = 0;
  for (int t = b; t < e; ++t) sum += counts[t];
  part[threadIdx.x] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan of the partial sums
    const int v = (threadIdx.x >= o) ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int run = (threadIdx.x == 0) ? 0 : part[threadIdx.x - 1];
  for (int t = b; t < e; ++t) {
    off[t] = run;
    cursor[t] = run;
    run += counts[t];
  }
  if (threadIdx.x == 1023) off[ntiles] = part[1023];
}

__global__ __launch_bounds__(BIL_T) void mppi_bin_scatter_kernel(const float* __restrict__ xs,
                                                                 const float* __restrict__ ys, int64_t n,
                                                                 int64_t chunk, float x_min, float y_min, float res,
                                                                 float rinv, int cdiv, int rows, int grid, int ntx,
                                                                 int ntiles, const int* __restrict__ hist,
                                                                 int* __restrict__ cursor, float* __restrict__ xs_out,
                                                                 float* __restrict__ ys_out, int32_t* __restrict__ perm) {
  extern __shared__ int lb[];  // [ntiles] this chunk's next position in each tile
  const int* gh = hist + (size_t)blockIdx.x * ntiles;
  for (int t = threadIdx.x; t < ntiles; t += BIL_T) {
    const int h = gh[t];
    lb[t] = h ? atomicAdd(&cursor[t], h) : 0;
  }
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * chunk, e = min(n, b + chunk);
  for (int64_t q = b + threadIdx.x; q < e; q += BIL_T) {
    const float x = xs[q], y = ys[q];
    const int pos = atomicAdd(&lb[query_tile(x, y, x_min, y_min, res, rinv, cdiv, rows, grid, ntx)], 1);
    xs_out[pos] = x;
    ys_out[pos] = y;
    perm[pos] = (int32_t)q;
  }
}

// Two-level scatter (ntiles <= BIN2_MAX_TILES).  The one-level scatter above writes every query to
// a random one of the ~4096 open tile runs of its chunk (~16 queries per run), so each store
// instruction touches 64 cache lines and every line is completed by several workgroups (1.34 ms of
// the 1.5 ms binning at C5).  Here both levels sort a block of BIN2_S queries in LDS first and store
// it as runs: (1) by bucket = tile row (<= 64 buckets at C5: runs of ~64 queries) into the bucket
// regions of an intermediate array, (2) blocks of that array by tile (a block spans one or two
// buckets, <= 2 x 64 tiles: runs of ~32-64) into the final tile runs.  Positions come from the
// same tile counts and offsets (off) as the one-level path; the order inside a tile is arbitrary.
constexpr int BIN2_S = 4096;            // queries per LDS-sorted block
constexpr int BIN2_MAX_TILES = 4096;    // LDS bins of the fine level
constexpr int BIN2_PER = BIN2_S / BIL_T;

// exclusive scan of cnt[0..nb) into off[0..nb) by one 1024-thread workgroup (tmp: 1024 + 16 ints)
__device__ inline void block_excl_scan(const int* cnt, int* off, int nb, int* tmp) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int per = (nb + BIL_T - 1) / BIL_T;
  const int b0 = tid * per;
  int s = 0;
  for (int i = 0; i < per; ++i)
    if (b0 + i < nb) s += cnt[b0 + i];
  int x = s;  // inclusive scan inside the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) tmp[wv] = x;
  __syncthreads();
  int wbase = 0;
  for (int w = 0; w < wv; ++w) wbase += tmp[w];
  int run = wbase + x - s;
  for (int i = 0; i < per; ++i)
    if (b0 + i < nb) {
      off[b0 + i] = run;
      run += cnt[b0 + i];
    }
  __syncthreads();
}

// Sort up to BIN2_S (x, y, index) entries of this workgroup by key in LDS and store them as runs:
// entry of key k at sorted position j goes to base[k] + (j - koff[k]).  kcnt/koff/base: [nk] LDS.
struct Bin2Lds {
  float* sx;
  float* sy;
  int* si;
  unsigned short* sk;
  int* kcnt;
  int* koff;
  int* base;
  int* tmp;
};

__device__ inline Bin2Lds bin2_lds(unsigned char* sm, int nk) {
  Bin2Lds L;
  L.sx = reinterpret_cast<float*>(sm);
  L.sy = L.sx + BIN2_S;
  L.si = reinterpret_cast<int*>(L.sy + BIN2_S);
  L.kcnt = L.si + BIN2_S;
  L.koff = L.kcnt + nk;
  L.base = L.koff + nk;
  L.tmp = L.base + nk;
  L.sk = reinterpret_cast<unsigned short*>(L.tmp + 16);
  return L;
}
size_t bin2_lds_bytes(int nk) { return (size_t)BIN2_S * (3 * 4 + 2) + (size_t)(3 * nk + 16) * 4; }

// place this thread's entries (key, rank inside the key) at their sorted LDS slots, then write
// every slot to global memory at base[key] + (slot - koff[key]); kcnt must hold the block's counts
__device__ inline void bin2_store(const Bin2Lds& L, int m, const int (&key)[BIN2_PER], const int (&rank)[BIN2_PER],
                                  const float (&x)[BIN2_PER], const float (&y)[BIN2_PER],
                                  const int (&idx)[BIN2_PER], float* __restrict__ ox, float* __restrict__ oy,
                                  int32_t* __restrict__ oi) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < BIN2_PER; ++k) {
    const int q = tid + k * BIL_T;
    if (q < m) {
      const int p = L.koff[key[k]] + rank[k];
      L.sx[p] = x[k];
      L.sy[p] = y[k];
      L.si[p] = idx[k];
      L.sk[p] = (unsigned short)key[k];
    }
  }
  __syncthreads();
  for (int j = tid; j < m; j += BIL_T) {
    const int kk = L.sk[j];
    const int pos = L.base[kk] + (j - L.koff[kk]);
    ox[pos] = L.sx[j];
    oy[pos] = L.sy[j];
    oi[pos] = L.si[j];
  }
  __syncthreads();
}

// level 1: chunk g of the queries (the histogram kernel's chunking), blocks of BIN2_S sorted by
// tile row into bucket regions [off[r ntx], off[(r + 1) ntx]) of (cx, cy, ci); the chunk claims its
// share of every bucket once from bcur (initialised to the bucket starts).  The next block's loads
// are issued before the current block is sorted.
__global__ __launch_bounds__(BIL_T) void mppi_bin2_coarse_kernel(const float* __restrict__ xs,
                                                                 const float* __restrict__ ys, int64_t n,
                                                                 int64_t chunk, float x_min, float y_min, float res,
                                                                 float rinv, int cdiv, int rows, int grid, int ntx,
                                                                 int nty, int ntiles, const int* __restrict__ hist,
                                                                 int* __restrict__ bcur, float* __restrict__ cx,
                                                                 float* __restrict__ cy, int32_t* __restrict__ ci) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const Bin2Lds L = bin2_lds(sm, nty);
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * chunk, e = min(n, b0 + chunk);
  float xn[BIN2_PER], yn[BIN2_PER];
  auto load = [&](int64_t s0) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < BIN2_PER; ++k) {
      const int64_t q = s0 + tid + k * BIL_T;
      xn[k] = q < e ? xs[q] : 0.0f;
      yn[k] = q < e ? ys[q] : 0.0f;
    }
  };
  load(b0);
  for (int r = tid; r < nty; r += BIL_T) {
    const int* gh = hist + (size_t)blockIdx.x * ntiles + (size_t)r * ntx;
    int s = 0;
    for (int i = 0; i < ntx; ++i) s += gh[i];
    L.base[r] = s ? atomicAdd(&bcur[r], s) : 0;
  }
  for (int64_t s0 = b0; s0 < e; s0 += BIN2_S) {
    const int m = (int)min((int64_t)BIN2_S, e - s0);
    for (int r = tid; r < nty; r += BIL_T) L.kcnt[r] = 0;
    int key[BIN2_PER], rank[BIN2_PER], idx[BIN2_PER];
    float x[BIN2_PER], y[BIN2_PER];
#pragma unroll
    for (int k = 0; k < BIN2_PER; ++k) {
      x[k] = xn[k];
      y[k] = yn[k];
    }
    load(s0 + BIN2_S);  // in flight while this block is sorted and stored
    __syncthreads();
#pragma unroll
    for (int k = 0; k < BIN2_PER; ++k) {
      const int q = tid + k * BIL_T;
      idx[k] = (int)(s0 + q);
      key[k] = 0;
      rank[k] = 0;
      if (q < m) {
        key[k] = query_tile(x[k], y[k], x_min, y_min, res, rinv, cdiv, rows, grid, ntx) / ntx;
        rank[k] = atomicAdd(&L.kcnt[key[k]], 1);
      }
    }
    __syncthreads();
    block_excl_scan(L.kcnt, L.koff, nty, L.tmp);
    bin2_store(L, m, key, rank, x, y, idx, cx, cy, ci);
    for (int r = tid; r < nty; r += BIL_T) L.base[r] += L.kcnt[r];
    __syncthreads();
  }
}

// level 2: blocks b = blockIdx.x, blockIdx.x + gridDim.x, ... of the bucket-sorted array, each
// sorted by tile and stored into the tile runs, each tile's share claimed from the tile cursors
// (initialised to off); the next block's loads issued before the current block is sorted
__global__ __launch_bounds__(BIL_T) void mppi_bin2_fine_kernel(const float* __restrict__ cx, const float* __restrict__ cy,
                                                               const int32_t* __restrict__ ci, int64_t n, float x_min,
                                                               float y_min, float res, float rinv, int cdiv, int rows,
                                                               int grid, int ntx, int ntiles, int* __restrict__ cursor,
                                                               float* __restrict__ xs_out, float* __restrict__ ys_out,
                                                               int32_t* __restrict__ perm) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const Bin2Lds L = bin2_lds(sm, ntiles);
  const int tid = threadIdx.x;
  const int64_t nblk = (n + BIN2_S - 1) / BIN2_S;
  float xn[BIN2_PER], yn[BIN2_PER];
  int in_[BIN2_PER];
  auto load = [&](int64_t blk) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < BIN2_PER; ++k) {
      const int64_t q = blk * BIN2_S + tid + k * BIL_T;
      const bool ok = blk < nblk && q < n;
      xn[k] = ok ? cx[q] : 0.0f;
      yn[k] = ok ? cy[q] : 0.0f;
      in_[k] = ok ? ci[q] : 0;
    }
  };
  load(blockIdx.x);
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t s0 = blk * BIN2_S;
    const int m = (int)min((int64_t)BIN2_S, n - s0);
    for (int t = tid; t < ntiles; t += BIL_T) L.kcnt[t] = 0;
    int key[BIN2_PER], rank[BIN2_PER], idx[BIN2_PER];
    float x[BIN2_PER], y[BIN2_PER];
#pragma unroll
    for (int k = 0; k < BIN2_PER; ++k) {
      x[k] = xn[k];
      y[k] = yn[k];
      idx[k] = in_[k];
    }
    load(blk + gridDim.x);  // in flight while this block is sorted and stored
    __syncthreads();
#pragma unroll
    for (int k = 0; k < BIN2_PER; ++k) {
      const int q = tid + k * BIL_T;
      key[k] = 0;
      rank[k] = 0;
      if (q < m) {
        key[k] = query_tile(x[k], y[k], x_min, y_min, res, rinv, cdiv, rows, grid, ntx);
        rank[k] = atomicAdd(&L.kcnt[key[k]], 1);
      }
    }
    __syncthreads();
    block_excl_scan(L.kcnt, L.koff, ntiles, L.tmp);
    for (int t = tid; t < ntiles; t += BIL_T) {
      const int c = L.kcnt[t];
      L.base[t] = c ? atomicAdd(&cursor[t], c) : 0;
    }
    __syncthreads();
    bin2_store(L, m, key, rank, x, y, idx, xs_out, ys_out, perm);
  }
}

// bucket starts: bcur[r] = off[r ntx] (after the scan)
__global__ void mppi_bin2_bucket_start_kernel(const int* __restrict__ off, int ntx, int nty, int* __restrict__ bcur) {
  for (int r = threadIdx.x; r < nty; r += blockDim.x) bcur[r] = off[r * ntx];
}

hipError_t launch_bin_queries(const float* xs, const float* ys, int64_t n, float x_min, float y_min, float res,
                              float rinv, int cdiv, int rows, int grid, int* hist, int* counts, int* cursor,
                              int* off, float* xs_out, float* ys_out, int32_t* perm, hipStream_t st,
                              float* cx, float* cy, int32_t* ci, int* bcur) {
  const int ntx = (grid + BIL_TS - 1) / BIL_TS, nty = (rows + BIL_TS - 1) / BIL_TS;
  const int ntiles = ntx * nty;
  hipError_t e = hipMemsetAsync(counts, 0, (size_t)ntiles * sizeof(int), st);
  if (e != hipSuccess) return e;
  const int G = bin_chunks(n, ntiles);
  const int64_t chunk = (n + G - 1) / G;
  const size_t lds = (size_t)ntiles * sizeof(int);
  if (n > 0)
    hipLaunchKernelGGL(mppi_bin_hist_kernel, dim3(G), dim3(BIL_T), lds, st, xs, ys, n, chunk, x_min, y_min, res, rinv,
                       cdiv, rows, grid, ntx, ntiles, hist, counts);
  hipLaunchKernelGGL(mppi_bin_scan_kernel, dim3(1), dim3(1024), 0, st, counts, ntiles, off, cursor);
  if (n > 0 && cx && ntiles <= BIN2_MAX_TILES) {  // two levels of LDS-sorted runs
    hipLaunchKernelGGL(mppi_bin2_bucket_start_kernel, dim3(1), dim3(256), 0, st, off, ntx, nty, bcur);
    hipLaunchKernelGGL(mppi_bin2_coarse_kernel, dim3(G), dim3(BIL_T), bin2_lds_bytes(nty), st, xs, ys, n, chunk, x_min,
                       y_min, res, rinv, cdiv, rows, grid, ntx, nty, ntiles, hist, bcur, cx, cy, ci);
    // persistent: one workgroup per CU (its LDS), each looping over blocks
    const unsigned nb = (unsigned)std::min<int64_t>((n + BIN2_S - 1) / BIN2_S, 256);
    hipLaunchKernelGGL(mppi_bin2_fine_kernel, dim3(nb), dim3(BIL_T), bin2_lds_bytes(ntiles), st, cx, cy, ci, n, x_min,
                       y_min, res, rinv, cdiv, rows, grid, ntx, ntiles, cursor, xs_out, ys_out, perm);
  } else if (n > 0) {
    hipLaunchKernelGGL(mppi_bin_scatter_kernel, dim3(G), dim3(BIL_T), lds, st, xs, ys, n, chunk, x_min, y_min, res,
                       rinv, cdiv, rows, grid, ntx, ntiles, hist, cursor, xs_out, ys_out, perm);
  }
  return hipGetLastError();
}

hipError_t launch_bilinear_tiled(const float* Z, int rows, int grid, float x_min, float y_min, float res,
                                 float rinv, int cdiv, const float* xs, const float* ys, float* hs,
                                 const int* tile_off, hipStream_t st) {
  const int ntx = (grid + BIL_TS - 1) / BIL_TS, nty = (rows + BIL_TS - 1) / BIL_TS;
  hipLaunchKernelGGL(mppi_bilinear_tiled_kernel, dim3(ntx * nty), dim3(BIL_T), (size_t)BIL_W * BIL_W * sizeof(float),
                     st, Z, rows, grid, x_min, y_min, res, rinv, cdiv, xs, ys, hs, tile_off, ntx);
  return hipGetLastError();
}

// =====================================================================  self-test
// Bitwise check of the fast division / sqrt paths against the IEEE operators
// on random operands spanning the fast-path range and beyond; an operand
// flagged out of range counts as checked (the engine would recompute it).
__global__ __launch_bounds__(256) void mppi_selftest_kernel(int what, int64_t n, uint64_t seed,
                                                            unsigned long long* bad_count) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned long long local = 0;
  if (what == 4) {  // the chain's quotient (refined reciprocal, ONE correction: lean_div_s) against a / b
    // for every significand of a and the divisor significands (seed + 8191 k) mod 2^23, k = i >> 23
    // (profiles/ubench/div1_check.hip ran all 2^46 pairs); b in [1, 2), exponents scale exactly
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const float a = bits_f(0x3F800000u | (uint32_t)(i & 0x7FFFFF));
      const float b = bits_f(0x3F800000u | (uint32_t)(((uint64_t)(i >> 23) * 8191u + seed) & 0x7FFFFFu));
      Lean l;
      lean_init(l);
      Recip r;
      r.b = b;
      const float y0 = __builtin_amdgcn_rcpf(b);
      r.y = __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
      if (f_bits(lean_div_s(a, r, l)) != f_bits(a / b)) ++local;
    }
    if (local) atomicAdd(bad_count, local);
    return;
  }
  if (what == 5) {  // the noise radius' sqrt_bm against sqrtf: -0, +0, then every float from 2^-24 on
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const float x = i < 2 ? (i == 0 ? -0.0f : 0.0f) : bits_f(0x33800000u + (uint32_t)(i - 2));
      if (f_bits(sqrt_bm(x)) != f_bits(sqrtf(x))) ++local;
    }
    if (local) atomicAdd(bad_count, local);
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const U4 r = philox4x32_10(U4{(uint32_t)i, (uint32_t)(i >> 32), 0x5e1fu, 0x7e57u}, (uint32_t)seed,
                               (uint32_t)(seed >> 32));
    // random sign/mantissa; exponent uniform over [-50, 50] (beyond the fast-path bounds)
    auto mk = [](uint32_t bits, uint32_t eb) {
      const int e = (int)(eb % 101u) - 50 + 127;
      return bits_f((bits & 0x807FFFFFu) | ((uint32_t)e << 23));
    };
    float a = mk(r.x, r.z), b = mk(r.y, r.w);
    if ((i & 1023) == 7) a = 0.0f;
    if ((i & 1023) == 9) a = -0.0f;
    if ((i & 4095) == 11) a = bits_f(r.x & 0x807FFFFFu);  // subnormal
    bool flagged = false;
    if (what == 0) {
      const float want = a / b;
      const float got = dv1<true>(a, b, flagged);
      if (!flagged && f_bits(want) != f_bits(got)) ++local;
    } else if (what == 1) {
      const float x = fabsf(a);
      const float want = sqrtf(x);
      const float got = sq<true>(x, flagged);
      if (!flagged && f_bits(want) != f_bits(got)) ++local;
    } else {  // 2, 3: lean normalisation (a, b, c) / sqrt(a^2 + b^2 + c^2) (lean_norm / lean_div)
      const U4 r2 = philox4x32_10(U4{(uint32_t)i, (uint32_t)(i >> 32), 0x5e1fu, 0x1ea4u}, (uint32_t)seed,
                                  (uint32_t)(seed >> 32));
      // what 3: c dominant (exponent in [-30, 30)), a and b anywhere in [-50, 50]
      const float c = (what == 3) ? bits_f((r2.x & 0x807FFFFFu) | ((127u - 30u + r2.y % 60u) << 23))
                                  : mk(r2.x, r2.y);
      const float n = (a * a + b * b) + c * c;
      const float sr = sqrtf(n);
      Lean l;
      lean_init(l);
      const Recip rr = lean_norm(n, l);
      const float g0 = lean_div(a, rr, l), g1 = lean_div(b, rr, l), g2 = lean_div(c, rr, l);
      if (!lean_bad(l) && (f_bits(rr.b) != f_bits(sr) || f_bits(g0) != f_bits(a / sr) ||
                           f_bits(g1) != f_bits(b / sr) || f_bits(g2) != f_bits(c / sr)))
        ++local;
    }
  }
  if (local) atomicAdd(bad_count, local);
}

// =====================================================================  launchers
template <int TB, int PROJ>
static hipError_t launch_pair_m(const RolloutArgs& a, int blocks, size_t lds, hipStream_t st, int mode,
                                bool dump) {
  if (mode == 0) {
    if (dump)
      hipLaunchKernelGGL((mppi_rollout_pair_kernel<TB, PROJ, 0, true>), dim3(blocks), dim3(2 * TB), lds, st, a);
    else
      hipLaunchKernelGGL((mppi_rollout_pair_kernel<TB, PROJ, 0, false>), dim3(blocks), dim3(2 * TB), lds, st, a);
  } else {
    if (dump)
      hipLaunchKernelGGL((mppi_rollout_pair_kernel<TB, PROJ, 1, true>), dim3(blocks), dim3(2 * TB), lds, st, a);
    else
      hipLaunchKernelGGL((mppi_rollout_pair_kernel<TB, PROJ, 1, false>), dim3(blocks), dim3(2 * TB), lds, st, a);
  }
  return hipGetLastError();
}

template <int TB, int PROJ>
static hipError_t launch_roles_m(const RolloutArgs& a, int blocks, size_t lds, hipStream_t st, int mode,
                                 bool dump) {
  const dim3 g(blocks), b(NROLES * TB);
  if (mode == 0) {
    if (dump)
      hipLaunchKernelGGL((mppi_rollout_roles_kernel<TB, PROJ, 0, true>), g, b, lds, st, a);
    else
      hipLaunchKernelGGL((mppi_rollout_roles_kernel<TB, PROJ, 0, false>), g, b, lds, st, a);
  } else {
    if (dump)
      hipLaunchKernelGGL((mppi_rollout_roles_kernel<TB, PROJ, 1, true>), g, b, lds, st, a);
    else
      hipLaunchKernelGGL((mppi_rollout_roles_kernel<TB, PROJ, 1, false>), g, b, lds, st, a);
  }
  return hipGetLastError();
}

hipError_t launch_rollout_pair(const RolloutArgs& a, int blocks, size_t lds, hipStream_t st, int proj,
                               int mode, bool dump, bool roles) {
  if (roles) {
    if (proj == 3) return launch_roles_m<256, 3>(a, blocks, lds, st, mode, dump);
    return launch_roles_m<256, 2>(a, blocks, lds, st, mode, dump);
  }
  if (proj == 3) return launch_pair_m<256, 3>(a, blocks, lds, st, mode, dump);
  return launch_pair_m<256, 2>(a, blocks, lds, st, mode, dump);
}

hipError_t launch_finish(const FinishArgs& f, size_t lds, hipStream_t st, int groups) {
  hipLaunchKernelGGL(mppi_finish_kernel, dim3(groups), dim3(FIN_THREADS), lds, st, f);
  return hipGetLastError();
}

// Column-split finish (mppi_colfin_kernel): P = leaves padded to a power of two >= 16,
// ncol columns per workgroup; returns the LDS bytes the tree needs in *lds_tree.
int colfin_shape(int n, int H, int* P_out, int* ncol_out, int* groups_out, size_t* lds_tree, int max_groups) {
  if (n < 1 || n > COLFIN_PMAX || max_groups < 1) return 0;
  int P = 16;
  while (P < n) P *= 2;
  const int E = 2 * H + 2;
  // about 64 workgroups, at least 2 columns each (at most max_groups workgroups)
  const int ncol = std::max({2, (E + 63) / 64, (E + max_groups - 1) / max_groups});
  if ((ncol + 1) * (P / 16) > FIN_THREADS) return 0;  // one (column, group) item per thread
  const int groups = (E + ncol - 1) / ncol;
  *P_out = P;
  *ncol_out = ncol;
  *groups_out = groups;
  *lds_tree = (size_t)(P - 1) * sizeof(PairScale) + (size_t)(2 * P) * sizeof(float) +
              (size_t)(ncol + 1) * (P / 16) * sizeof(double);
  return 1;
}

hipError_t launch_colfin(const FinishArgs& f, size_t lds, hipStream_t st, int P, int ncol, int groups) {
  hipLaunchKernelGGL(mppi_colfin_kernel, dim3(groups), dim3(FIN_THREADS), lds, st, f, P, ncol);
  return hipGetLastError();
}

hipError_t launch_tail(const FinishArgs& f, hipStream_t st) {
  const size_t lds = (size_t)(12 * f.H + 4) * sizeof(float);  // in4[H + 1], chain[8H]
  hipLaunchKernelGGL(mppi_tail_kernel, dim3(1), dim3(TAIL_THREADS), lds, st, f);
  return hipGetLastError();
}

// Per-cell surface normals (projection_warp.py:129-151 `_normal_on_grid` on the four
// corners that projection_warp.py:8-48 selects for a cell), built once per DEM: entry
// (j + 1, i + 1) for the cell indices i in [-1, grid - 1], j in [-1, rows - 1] that
// Dem::cell produces (i = grid and j = rows select the same clamped corners as grid - 1
// and rows - 1).  IEEE float operations in the reference order, i.e. exactly the normal
// the rollout chain computed per step before (chain3d<false> / the lean chains agree on
// it bit for bit), so reading it from the table changes no result.
__global__ __launch_bounds__(256) void mppi_normal_table_kernel(const float* __restrict__ Z, int rows, int grid,
                                                                float res, float4* __restrict__ out) {
  const int64_t cols = (int64_t)grid + 1;
  const int64_t n = ((int64_t)rows + 1) * cols;
  const float res_half_neg = (-res) / 2.0f;
  const float res_sq = res * res;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < n; g += (int64_t)gridDim.x * 256) {
    const int j = (int)(g / cols) - 1, i = (int)(g % cols) - 1;
    const int r0 = clampi(j, 0, rows - 1), r1 = clampi(j + 1, 0, rows - 1);
    const int c0 = clampi(i, 0, grid - 1), c1 = clampi(i + 1, 0, grid - 1);
    const float q0 = Z[(size_t)r0 * grid + c0], q1 = Z[(size_t)r0 * grid + c1];
    const float q2 = Z[(size_t)r1 * grid + c0], q3 = Z[(size_t)r1 * grid + c1];
    bool unused = false;
    const float vx = res_half_neg * (((q1 - q0) - q2) + q3);
    const float vy = res_half_neg * (((q2 - q0) - q1) + q3);
    const Recip r = rc<false>(sq<false>((vx * vx + vy * vy) + res_sq * res_sq, unused), unused);
    out[g] = make_float4(dv<false>(vx, r, unused), dv<false>(vy, r, unused), dv<false>(res_sq, r, unused), 0.0f);
  }
}

hipError_t launch_normal_table(const float* Z, int rows, int grid, float res, float4* out, hipStream_t st) {
  const int64_t n = ((int64_t)rows + 1) * ((int64_t)grid + 1);
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(mppi_normal_table_kernel, dim3(blocks), dim3(256), 0, st, Z, rows, grid, res, out);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void mppi_noise_kernel(uint64_t seed, uint64_t n_base, int64_t k_offset,
                                                         int H, int n_blocks, float* __restrict__ eps) {
  noise_rows(seed, n_base, k_offset, H, n_blocks * ((H + 1) >> 1), eps, blockIdx.x, gridDim.x, threadIdx.x);
}

// =====================================================================  resident step server
// One launch serves a sequence of sampled steps (mppi_capi.cpp "resident step server"): workgroup b
// is rollout block b of every step.  Per step: the head's wave 0 polls cmd->seq (one lane, system
// scope) until it reaches `expect` (or cmd->stop, or idle_ticks without a command: it relays a stop
// and every workgroup exits), the others poll its relay; each reads the command words into LDS, and the workgroup runs the role-split rollout with
// the command's state, normals slot and nominal buffer.  Its record is written through and counted
// (rec_cnt); the workgroups holding the last fin_groups tickets run the column-split finish, each
// after rec_cnt reaches nroll (bounded by wait_ticks: a finish without every record publishes
// done = seq | kDoneFail); the others generate the normals of step + 2 meanwhile (noise phase:
// the chip is otherwise idle while the finish reduces and the host turns the step around).  No assumption on dispatch order or co-residency: a workgroup waits only
// for records of workgroups that run or get a slot as others reach their wait.
// Cross-step data: the nominal sequence, the tail inputs and the records are
// written through and read with agent-scope loads; the normals rows (another kernel's write-through
// stores) are read with plain loads after this CU's L1 was invalidated at the end of the previous step.
// Kernel arguments re-read every step: a pointer laundered through an empty asm, so the compiler
// cannot hoist the (invariant) argument loads out of the step loop and keep them live across it
// (that raised the kernel from 88 to 128 VGPRs with spills); scalar loads once per step instead.
struct ServerLaunch {
  RolloutArgs a;
  ServerArgs z;
};
__device__ __forceinline__ const ServerLaunch* fresh_args() {
#if __HIP_DEVICE_COMPILE__
  uint64_t v = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
  asm volatile("" : "+s"(v));
  // (constant address space, then generic: the loads through it stay scalar kernarg loads)
  return (const ServerLaunch*)reinterpret_cast<const __attribute__((address_space(4))) ServerLaunch*>(v);
#else
  return nullptr;
#endif
}

template <int TB, int PROJ>
__global__ __launch_bounds__(NROLES * TB) void mppi_step_server_kernel(const ServerLaunch args) {
  __shared__ unsigned cmd_lds[32];
  __shared__ int sh[2];
  const int tid = threadIdx.x;
  unsigned expect = args.z.first_seq;
  // the head polls the pinned command and relays it: workgroup 0 for the first step of the launch,
  // then the workgroup that took the previous step's last ticket (it ran the finish's phase 2 and
  // published the completion word, so it is the first to be free)
  bool head = blockIdx.x == 0;
  for (;;) {
    const auto* L = fresh_args();
    const ServerArgs& z = L->z;
    if (tid < 64) {
      // the head polls the pinned command (seq and stop in one 8-byte read) and relays it: the
      // command words to relay[16..], then (after they completed) seq / stop to relay[0..1]; the
      // others poll relay[0..1] in device memory.  An idle head relays a stop.  Stop words are this
      // launch's launch_id (a stale one from an earlier launch never matches), so the host launches
      // without resetting the relay or the command's stop word.
      const unsigned long long* src = head ? reinterpret_cast<const unsigned long long*>(z.cmd)
                                           : reinterpret_cast<const unsigned long long*>(z.relay);
      // Only the head leaves on its own (idle limit, or the exit_after test hook); the others leave
      // on the stop it relays.  So an exit is all-or-nothing: either every workgroup serves a command
      // or none does, and a command the head never relayed leaves no trace of the step (the host sees
      // the launch retire without a completion word and relaunches the server with that command).
      // The host's stop is read before seq (a stop posted before a later launch's command ends this
      // launch first), and the others also read it themselves every ~100 us: after a finish that gave
      // up no workgroup holds the last ticket, so there is no head to relay it.
      unsigned ok = 0;
      if (tid == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint64_t t_stop = t0;
        if (head && z.clk) z.clk[kClkServer + 8 * (expect & 7) + 6] = t0;
        const bool forced = head && z.exit_after != 0 && expect - z.first_seq >= z.exit_after;
        while (!forced) {
          const unsigned long long w = head ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                            : __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((unsigned)(w >> 32) == z.launch_id) break;
          if ((int)((unsigned)w - expect) >= 0) {
            ok = 1;
            break;
          }
          const uint64_t now = __builtin_amdgcn_s_memrealtime();
          if (head) {
            if (now - t0 >= z.idle_ticks) break;
          } else {
            if (now - t_stop >= 10000) {
              t_stop = now;
              if (__hip_atomic_load(&z.cmd->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == z.launch_id) break;
            }
            __builtin_amdgcn_s_sleep(2);  // (~0.06 us; 8: server rollout +0.4 us, its start spread)
          }
        }
      }
      ok = __builtin_amdgcn_readfirstlane(ok);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler only: the words below after the poll)
      if (ok && tid < kCmdWords) {
        unsigned wv;
        if (head) {
          wv = __hip_atomic_load(reinterpret_cast<const unsigned*>(z.cmd) + tid, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(z.relay + 16 + tid, wv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          wv = __hip_atomic_load(z.relay + 16 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        cmd_lds[tid] = wv;
      }
      if (head) {  // the words are written through and complete, then seq (or stop: every workgroup exits)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0) {
          if (ok)
            __hip_atomic_store(z.relay, cmd_lds[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else
            __hip_atomic_store(z.relay + 1, z.launch_id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (tid == 0) cmd_lds[31] = ok;
      if (tid == 0 && head && z.clk && ok)  // (write-through: the last ticket and the finish read it)
        __hip_atomic_store(z.clk + kClkServer + 8 * (cmd_lds[0] & 7), (uint64_t)__builtin_amdgcn_s_memrealtime(),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!cmd_lds[31]) return;  // stop, or idle: the host relaunches
    const ServerCmd& c = *reinterpret_cast<const ServerCmd*>(cmd_lds);
    auto rd = [&](const float& x) __attribute__((always_inline)) {
      return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, x)));
    };
    const unsigned seq = __builtin_amdgcn_readfirstlane(c.seq);
    const int eps_slot = __builtin_amdgcn_readfirstlane(c.eps_slot);
    const int cur = __builtin_amdgcn_readfirstlane(c.cur);
    RolloutArgs a = L->a;
    a.eps = z.eps[eps_slot];
    a.u_nom1 = z.u_nom[cur];
    a.u_nom2 = z.u_nom[cur] + a.H;
    a.x0 = rd(c.x0);
    a.y0 = rd(c.y0);
    a.h0x = rd(c.h0x);
    a.h0y = rd(c.h0y);
    a.h0z = rd(c.h0z);
    a.wl = rd(c.wl);
    a.wr = rd(c.wr);
    a.gx = rd(c.gx);
    a.gy = rd(c.gy);
    a.s1 = rd(c.s1);
    a.s2 = rd(c.s2);
    a.igx = rd(c.igx);
    a.igy = rd(c.igy);
    a.pf_scale = rd(c.pf_scale);
    a.pf_far = __builtin_amdgcn_readfirstlane(c.pf_far);
    a.speed_on = __builtin_amdgcn_readfirstlane(c.speed_on);
    const int nslot = __builtin_amdgcn_readfirstlane(c.noise_slot);
    const uint64_t nbase = ((uint64_t)__builtin_amdgcn_readfirstlane(c.noise_n_base_hi) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane(c.noise_n_base_lo);
    // the normals of step + 2 (when commanded): W wave-units (one Philox block of 64 trajectories
    // each) in S static shares, two per workgroup outside the finish (ticket t: shares 2t, 2t + 1,
    // from its record on) and one per finish workgroup but the last (blk: share 2 nn + blk, after
    // its columns, ~10 us later); the last finish workgroup runs phase 2 and heads the next poll
    const int64_t W = 4 * (int64_t)z.nroll * ((a.H + 1) >> 1);
    const int nn = z.nroll - z.fin_groups;
    const int64_t S = 2 * (int64_t)nn + z.fin_groups - 1;
    const int ticket = roles_body<TB, PROJ, 0, false, true>(a, (int)blockIdx.x, z.rec_cnt, sh);
    if (ticket == z.nroll - 1 && tid == 0 && z.clk) {  // the rollout's time on the server, summed
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      z.clk[kClkServer + 8 * (seq & 7) + 1] = now;
      const uint64_t t0 = __hip_atomic_load(z.clk + kClkServer + 8 * (seq & 7), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(z.clk + kClkSums, now - t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(z.clk + kClkSums + 1, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const int blk = ticket - (z.nroll - z.fin_groups);
    if (blk < 0 && nslot >= 0) {
      // shares 2t, 2t + 1 of the normals of step + 2 while the finish workgroups reduce the records
      // and the host turns the step around (static: no claims)
      __builtin_amdgcn_s_setprio(0);
      const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
      const int q0 = (int)(W * (2 * ticket) / S), q1 = (int)(W * (2 * ticket + 2) / S);
      noise_waves(a.seed, nbase, a.k_offset, a.H, q0 + wave, q1, NROLES * TB / 64, z.eps[nslot], tid & 63);
    }
    if (blk >= 0) {
      __builtin_amdgcn_s_setprio(0);  // the rollout waves' priorities do not carry into the finish
      if (tid == 0) {  // bounded (z.wait_ticks of the 100 MHz clock): a lost count cannot hang the device
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int late = z.wait_ticks == 0;  // 0: give up at once (the test hook of mppi_set_option)
        while (!late && __hip_atomic_load(z.rec_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)z.nroll) {
          // (another finish workgroup gave up on this step: the step has failed, stop waiting)
          if (__builtin_amdgcn_s_memrealtime() - t0 >= z.wait_ticks ||
              __hip_atomic_load(z.f.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == seq) {
            late = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        // the step fails: the last finish workgroup's u_opt poll and the other finish workgroups still
        // waiting stop on this word instead of their own bounds
        if (late) __hip_atomic_store(z.f.abort, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sh[1] = late;
      }
      __syncthreads();
      bool ok = !sh[1];
      if (ok) {
        FinishArgs f = z.f;
        const int mode = __builtin_amdgcn_readfirstlane(c.mode);
        const int slot = __builtin_amdgcn_readfirstlane(c.tail_slot);
        f.mode = mode;
        f.seq = seq;
        f.u_nom_next = z.u_nom[cur ^ 1];
        f.tail_in = z.tail_in[slot];
        f.tail_out = z.tail_out[slot];
        f.x0 = a.x0;
        f.y0 = a.y0;
        f.h0x = a.h0x;
        f.h0y = a.h0y;
        f.h0z = a.h0z;
        f.wl = a.wl;
        f.wr = a.wr;
        ok = colfin_body<true>(f, z.fin_P, z.fin_ncol, blk, z.fin_groups, z.rec_cnt);
        if (ok && blk == z.fin_groups - 1 && tid == 0 && z.clk) {  // and the whole step's
          const uint64_t now = __builtin_amdgcn_s_memrealtime();
          z.clk[kClkServer + 8 * (seq & 7) + 2] = now;
          const uint64_t t0 = __hip_atomic_load(z.clk + kClkServer + 8 * (seq & 7), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add(z.clk + kClkSums + 2, now - t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add(z.clk + kClkSums + 3, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      // a finish that gave up publishes the failure (the host stops the server and re-arms the count)
      if (!ok && tid == 0)
        __hip_atomic_store(z.f.done, seq | kDoneFail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (nslot >= 0 && blk < z.fin_groups - 1) {  // its share of the normals of step + 2 (see above)
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int q0 = (int)(W * (2 * nn + blk) / S), q1 = (int)(W * (2 * nn + blk + 1) / S);
        noise_waves(a.seed, nbase, a.k_offset, a.H, q0 + wave, q1, NROLES * TB / 64, z.eps[nslot], tid & 63);
      }
    }
    // this CU's L1 forgets the step's normals rows before a later step reads rewritten ones
    // (asynchronous: the next poll's wait covers it)
    if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    expect = seq + 1;
    head = ticket == z.nroll - 1;
    __syncthreads();  // every wave is done with this step's LDS and command words
    if (tid == 0 && z.clk) {  // the latest end of a noise share (3) and of any workgroup's step (7)
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (blk < 0) __hip_atomic_fetch_max(z.clk + kClkServer + 8 * (seq & 7) + 3, now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_max(z.clk + kClkServer + 8 * (seq & 7) + 7, now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

hipError_t launch_step_server(const RolloutArgs& a, const ServerArgs& z, size_t lds, hipStream_t st, int proj) {
  const dim3 g((unsigned)z.nroll), b(NROLES * 256);
  if (proj == 3)
    hipLaunchKernelGGL((mppi_step_server_kernel<256, 3>), g, b, lds, st, ServerLaunch{a, z});
  else
    hipLaunchKernelGGL((mppi_step_server_kernel<256, 2>), g, b, lds, st, ServerLaunch{a, z});
  return hipGetLastError();
}

hipError_t launch_noise(uint64_t seed, uint64_t n_base, int64_t k_offset, int blocks, int H, float* eps,
                        hipStream_t st, int max_groups) {
  // Grid capped (max_groups, a few workgroups per CU): the noise of step i+2 is generated
  // while the finish of step i runs and the next rollout starts; a full-size grid fills every
  // wave slot ahead of their 16-wave workgroups, which then wait for the whole noise kernel.
  const int NB = (H + 1) >> 1;
  const int64_t total = (int64_t)blocks * NB;
  const unsigned grid = (unsigned)std::min<int64_t>(total, std::max(max_groups, 1));
  hipLaunchKernelGGL(mppi_noise_kernel, dim3(grid), dim3(256), 0, st, seed, n_base, k_offset, H, blocks, eps);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void mppi_cdiv_verify_kernel(float b, float y, unsigned* bad) {
  const unsigned i = blockIdx.x * 256u + threadIdx.x;  // significand bits, 2^23 threads
  const float a = __builtin_bit_cast(float, 0x3f800000u | i);
  const float q = cdiv_f(a, b, y);
  const float ref = a / b;
  if (__builtin_bit_cast(unsigned, q) != __builtin_bit_cast(unsigned, ref)) atomicAdd(bad, 1u);
}

// Test hook (mppi_debug_hold): workgroups that each hold `lds` bytes of a CU's LDS for `ticks` of the
// 100 MHz clock, i.e. another stream's kernels occupying CUs when a step is posted.  Time-bounded.
__global__ __launch_bounds__(64) void mppi_hold_kernel(uint64_t ticks) {
  extern __shared__ unsigned char hold_lds[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  hold_lds[threadIdx.x] = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}

hipError_t launch_hold(int groups, size_t lds, uint64_t ticks, hipStream_t st) {
  hipLaunchKernelGGL(mppi_hold_kernel, dim3((unsigned)groups), dim3(64), lds, st, ticks);
  return hipGetLastError();
}

hipError_t launch_cdiv_verify(float b, float y, unsigned* bad, hipStream_t st) {
  hipLaunchKernelGGL(mppi_cdiv_verify_kernel, dim3(1u << 15), dim3(256), 0, st, b, y, bad);
  return hipGetLastError();
}

hipError_t launch_selftest(int what, int64_t n, uint64_t seed, unsigned long long* bad, hipStream_t st) {
  hipLaunchKernelGGL(mppi_selftest_kernel, dim3(2048), dim3(256), 0, st, what, n, seed, bad);
  return hipGetLastError();
}

hipError_t launch_bilinear(const float* Z, int rows, int grid, float x_min, float y_min, float res,
                           const float* xs, const float* ys, float* hs, int64_t n, hipStream_t st) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(mppi_bilinear_kernel, dim3((unsigned)blocks), dim3(256), 0, st, Z, rows, grid,
                     x_min, y_min, res, xs, ys, hs, n);
  return hipGetLastError();
}

}  // namespace mppi
