// MI355X (gfx950) MPPI rollout-and-cost engine: kernels.
//
// One MPPI step (reference: thesis_master/warp_implementation/MPPI_isaac.py:505-720,
// nine Warp launches) runs here as two kernels:
//
//   mppi_rollout_kernel  (#1-#7 fused)  one lane per sampled trajectory; Philox
//       noise, wheel filter, 2.5D rollout on the DEM (staged once per workgroup
//       into LDS), the four critics accumulated online, then the workgroup's
//       softmax leaf records (min, sum w, sum w*u[t]) -> one float64 record per
//       workgroup.  Nothing per (k, t) touches HBM.
//   mppi_finish_kernel   (#7-#9)  one workgroup; binary tree over the records,
//       u_opt = V/S, optimal-sequence filter and the 3D rollout of it.
//
// Numerics: compile with -ffp-contract=off.  Every float op is one IEEE f32
// operation in the reference's source order; transcendentals come from
// mppi_detmath.h.  oracle/mppi_ref.py restates the same sequence in numpy.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mppi_detmath.h"
#include "mppi_kernels.h"

namespace mppi {

// =====================================================================  grid lookups
// projection_warp.py:39-40 / :338-339 — C-style truncation; clamping is DEFINED
// here (the reference reads out of bounds).
__device__ __forceinline__ int trunc_clamped(float f, float lo, float hi) {
  return (int)fminf(fmaxf(f, lo), hi);
}
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

template <bool LDS>
struct Dem {
  const float* Z;    // global DEM (row-major rows x grid)
  const float* win;  // LDS window (Wr x W), LDS only
  int rows, grid, wx0, wy0, W, Wr;
  float x_min, y_min, res;

  __device__ __forceinline__ void cell(float x, float y, int& i, int& j) const {
    i = trunc_clamped((x - x_min) / res, -1.0f, (float)grid);
    j = -trunc_clamped((y + y_min) / res, -(float)rows, 1.0f);
  }
  __device__ __forceinline__ float at(int row, int col) const {
    row = clampi(row, 0, rows - 1);
    col = clampi(col, 0, grid - 1);
    if constexpr (LDS) {
      const int r = clampi(row - wy0, 0, Wr - 1);
      const int c = clampi(col - wx0, 0, W - 1);
      return win[r * W + c];
    } else {
      return Z[(size_t)row * grid + col];
    }
  }
  // projection_warp.py:8-48
  __device__ __forceinline__ void corners(float x, float y, float& q00, float& q01, float& q10,
                                          float& q11) const {
    int i, j;
    cell(x, y, i, j);
    const int r0 = clampi(j, 0, rows - 1), r1 = clampi(j + 1, 0, rows - 1);
    const int c0 = clampi(i, 0, grid - 1), c1 = clampi(i + 1, 0, grid - 1);
    if constexpr (LDS) {
      const int a0 = clampi(r0 - wy0, 0, Wr - 1) * W, a1 = clampi(r1 - wy0, 0, Wr - 1) * W;
      const int b0 = clampi(c0 - wx0, 0, W - 1), b1 = clampi(c1 - wx0, 0, W - 1);
      q00 = win[a0 + b0];
      q01 = win[a0 + b1];
      q10 = win[a1 + b0];
      q11 = win[a1 + b1];
    } else {
      q00 = Z[(size_t)r0 * grid + c0];
      q01 = Z[(size_t)r0 * grid + c1];
      q10 = Z[(size_t)r1 * grid + c0];
      q11 = Z[(size_t)r1 * grid + c1];
    }
  }
  __device__ __forceinline__ float point(float x, float y) const {
    int i, j;
    cell(x, y, i, j);
    return at(j, i);
  }
};

// projection_warp.py:70-100 (trunc; x-fraction paired with the row neighbour q10)
__device__ __forceinline__ float bilinear(float x, float y, float q00, float q01, float q10,
                                          float q11, float res) {
  const float xn = x / res, yn = y / res;
  const float x2 = xn - truncf(xn), y2 = yn - truncf(yn);
  const float a = ((1.0f - x2) * (1.0f - y2)) * q00;
  const float b = (x2 * (1.0f - y2)) * q10;
  const float c = ((1.0f - x2) * y2) * q01;
  const float d = (x2 * y2) * q11;
  return ((a + b) + c) + d;
}

struct Cost {  // critics_warp.py accumulators
  float pf_sum, sw, sp, ob, last_x, last_y;
};

// =====================================================================  one rollout-step
// State of one trajectory between steps.
struct Traj {
  float x, y;         // position[tid]
  float hx, hy, hz;   // `previous` heading
  float lwx, lwy, lwz, rwx, rwy, rwz;   // wheel points of the last even step (slope critic)
};

struct StepOut {
  float z;                              // trajectory height
  float lx, ly, lz, rx, ry, rz;         // wheel points
};

// 3D step: projection_warp.py:312-350 (loop body of _generate_trajectories_kernel).
template <bool LDS>
__device__ __forceinline__ void step3d(const Dem<LDS>& dem, float res_half_neg, float res_sq,
                                       float dt, float off, float v, float w, Traj& s,
                                       StepOut& o) {
  // _update_position :207-223
  {
    const float nrm = sqrtf((s.hx * s.hx + s.hy * s.hy) + s.hz * s.hz);
    const float ux = s.hx / nrm, uy = s.hy / nrm;
    s.x = s.x + (ux * v) * dt;
    s.y = s.y + (uy * v) * dt;
  }
  float q00, q01, q10, q11;
  dem.corners(s.x, s.y, q00, q01, q10, q11);
  o.z = bilinear(s.x, s.y, q00, q01, q10, q11, dem.res);
  // _normal_on_grid :129-151
  const float vx = res_half_neg * (((q01 - q00) - q10) + q11);
  const float vy = res_half_neg * (((q10 - q00) - q01) + q11);
  const float nn = sqrtf((vx * vx + vy * vy) + res_sq * res_sq);
  const float nx = vx / nn, ny = vy / nn, nz = res_sq / nn;
  // _get_heading_tangent_vector :168-190
  float tx, ty, tz;
  {
    const float d = (s.hx * nx + s.hy * ny) + s.hz * nz;
    tx = s.hx - d * nx;
    ty = s.hy - d * ny;
    tz = s.hz - d * nz;
    const float tn = sqrtf((tx * tx + ty * ty) + tz * tz);
    tx = tx / tn;
    ty = ty / tn;
    tz = tz / tn;
  }
  // _update_orientation :225-248 (Rodrigues about n)
  {
    const float on = sqrtf((tx * tx + ty * ty) + tz * tz);
    const float ox = tx / on, oy = ty / on, oz = tz / on;
    float sn, cs;
    dm_sincosf(w * dt, &sn, &cs);
    const float crx = ny * oz - nz * oy, cry = nz * ox - nx * oz, crz = nx * oy - ny * ox;
    const float dn = (nx * ox + ny * oy) + nz * oz;
    const float omc = 1.0f - cs;
    const float rx = (ox * cs + crx * sn) + (nx * dn) * omc;
    const float ry = (oy * cs + cry * sn) + (ny * dn) * omc;
    const float rz = (oz * cs + crz * sn) + (nz * dn) * omc;
    const float rn = sqrtf((rx * rx + ry * ry) + rz * rz);
    s.hx = rx / rn;
    s.hy = ry / rn;
    s.hz = rz / rn;
  }
  // wheels :333-348, right = offset * cross(normal, current_hv)
  const float cx = off * (ny * s.hz - nz * s.hy);
  const float cy = off * (nz * s.hx - nx * s.hz);
  o.lx = s.x + cx;
  o.ly = s.y + cy;
  o.lz = dem.point(o.lx, o.ly);
  o.rx = s.x - cx;
  o.ry = s.y - cy;
  o.rz = dem.point(o.rx, o.ry);
}

// 2D step: projection_warp.py:373-382 (wheels DEFINED as zero).
template <bool LDS>
__device__ __forceinline__ void step2d(const Dem<LDS>& dem, float dt, float v, float w, Traj& s,
                                       StepOut& o) {
  {
    const float nrm = sqrtf((s.hx * s.hx + s.hy * s.hy) + s.hz * s.hz);
    const float ux = s.hx / nrm, uy = s.hy / nrm;
    s.x = s.x + (ux * v) * dt;
    s.y = s.y + (uy * v) * dt;
  }
  {  // _update_orientation_2D :251-275
    float sn, cs;
    dm_sincosf(w * dt, &sn, &cs);
    float nx = cs * s.hx - sn * s.hy;
    float ny = sn * s.hx + cs * s.hy;
    const float nrm = sqrtf(nx * nx + ny * ny);
    if (nrm > 0.0f) {
      nx = nx / nrm;
      ny = ny / nrm;
    }
    s.hx = nx;
    s.hy = ny;
    s.hz = 0.0f;
  }
  float q00, q01, q10, q11;
  dem.corners(s.x, s.y, q00, q01, q10, q11);
  o.z = bilinear(s.x, s.y, q00, q01, q10, q11, dem.res);
  o.lx = o.ly = o.lz = o.rx = o.ry = o.rz = 0.0f;
}

// critics_warp.py:190-218, term for points (t, t+2) of both wheels.
__device__ __forceinline__ float slope_term(float plx, float ply, float plz, float clx, float cly,
                                            float clz, float prx, float pry, float prz, float crx,
                                            float cry, float crz) {
  const float eps = 1e-6f;
  const float dzl = clz - plz;
  const float dxl = clx - plx, dyl = cly - ply;
  const float dl = sqrtf(dxl * dxl + dyl * dyl);
  const float dzr = crz - prz;
  const float dxr = crx - prx, dyr = cry - pry;
  const float dr = sqrtf(dxr * dxr + dyr * dyr);
  const float ratl = fabsf(dzl / (dl + eps));
  const float ratr = fabsf(dzr / (dr + eps));
  const float al = 1.0f + 5.0f * ratl;
  const float ar = 1.0f + 5.0f * ratr;
  const float ls = al * al, rs = ar * ar;
  return (ls > rs) ? ls : rs;
}

// critics_warp.py:244-253
__device__ __forceinline__ float costmap_at(const float* cm, int size, float hw, float res_c,
                                            float x, float y) {
  const int ix = clampi(trunc_clamped((x + hw) / res_c, -1.0f, (float)size), 0, size - 1);
  const int iy = clampi(trunc_clamped(((-y) + hw) / res_c, -1.0f, (float)size), 0, size - 1);
  return cm[ix + size * iy];
}

__device__ __forceinline__ float clampf(float x, float lo, float hi) {
  return fminf(fmaxf(x, lo), hi);
}

// =====================================================================  reductions
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
// xor-butterfly order (pairs l, l^32 first) — oracle/mppi_ref.py _wave_tree
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = v + __shfl_xor(v, o, 64);
  return v;
}

// Record combine a (+) b for element j (oracle/mppi_ref.py combine).
struct PairScale {
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

// =====================================================================  rollout kernel
template <int BLOCK, bool LDS, int PROJ, int MODE, bool DUMP>
__global__ __launch_bounds__(BLOCK) void mppi_rollout_kernel(const RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  float* win = reinterpret_cast<float*>(smem_raw);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  constexpr int NW = BLOCK / 64;

  // ---- stage the DEM window [wy0, wy0+Wr) x [wx0, wx0+W) into LDS (coalesced rows)
  if constexpr (LDS) {
    for (int r = wave; r < a.Wr; r += NW) {
      const float* src = a.Z + (size_t)(a.wy0 + r) * a.grid + a.wx0;
      float* dst = win + r * a.W;
      for (int c = lane; c < a.W; c += 64) dst[c] = src[c];
    }
    __syncthreads();
  }
  Dem<LDS> dem;
  dem.Z = a.Z;
  dem.win = win;
  dem.rows = a.rows;
  dem.grid = a.grid;
  dem.wx0 = a.wx0;
  dem.wy0 = a.wy0;
  dem.W = a.W;
  dem.Wr = a.Wr;
  dem.x_min = a.x_min;
  dem.y_min = a.y_min;
  dem.res = a.res;

  const int64_t kl = (int64_t)blockIdx.x * BLOCK + tid;  // shard-local trajectory
  const bool valid = kl < a.K;
  const uint64_t kg = (uint64_t)(a.k_offset + kl);         // global trajectory (Philox subsequence)
  const int H = a.H;
  const float res_half_neg = (-a.res) / 2.0f;
  const float res_sq = a.res * a.res;
  const float one_m_fa = 1.0f - a.fa;

  // ---- initial projection at the robot pose (projection_warp.py:306-310)
  Traj s;
  s.x = a.x0;
  s.y = a.y0;
  {
    float q00, q01, q10, q11;
    dem.corners(s.x, s.y, q00, q01, q10, q11);
    const float vx = res_half_neg * (((q01 - q00) - q10) + q11);
    const float vy = res_half_neg * (((q10 - q00) - q01) + q11);
    const float nn = sqrtf((vx * vx + vy * vy) + res_sq * res_sq);
    const float nx = vx / nn, ny = vy / nn, nz = res_sq / nn;
    if constexpr (PROJ == 3) {
      const float d = (a.h0x * nx + a.h0y * ny) + a.h0z * nz;
      float tx = a.h0x - d * nx, ty = a.h0y - d * ny, tz = a.h0z - d * nz;
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
  s.lwx = s.lwy = s.lwz = s.rwx = s.rwy = s.rwz = 0.0f;

  Cost c;
  c.pf_sum = c.sw = c.sp = c.ob = 0.0f;
  c.last_x = s.x;
  c.last_y = s.y;
  float L = a.wl, R = a.wr;

  auto one_step = [&](int t, float u1, float u2) {
    // _convert_inputs_to_velocities (sampling_warp.py:120-138)
    L = L * a.fa + (u1 * a.fk) * one_m_fa;
    R = R * a.fa + (u2 * a.fk) * one_m_fa;
    const float v = clampf((L + R) / 2.0f, a.vmin, a.vmax);
    const float w = clampf(((-L) + R) / a.rwheel, a.wmin, a.wmax);
    StepOut o;
    if constexpr (PROJ == 3)
      step3d<LDS>(dem, res_half_neg, res_sq, a.dt, a.off, v, w, s, o);
    else
      step2d<LDS>(dem, a.dt, v, w, s, o);
    // _path_follow_critic sum branch (:125-126) over t < H-1; last point (:116)
    if (t < H - 1) c.pf_sum = c.pf_sum + 10.0f * (fabsf(s.x - a.gx) + fabsf(s.y - a.gy));
    c.last_x = s.x;
    c.last_y = s.y;
    // _avoid_slope_wheels (:190-216): terms (i, i+2) for even i < H-3
    if ((t & 1) == 0) {
      if (t >= 2 && t - 2 < H - 3)
        c.sw = c.sw + slope_term(s.lwx, s.lwy, s.lwz, o.lx, o.ly, o.lz, s.rwx, s.rwy, s.rwz, o.rx,
                                 o.ry, o.rz);
      s.lwx = o.lx; s.lwy = o.ly; s.lwz = o.lz;
      s.rwx = o.rx; s.rwy = o.ry; s.rwz = o.rz;
    }
    // _maximise_speed (:296-297)
    if (a.speed_on) c.sp = c.sp + (a.vmax - v) / (v + 0.0001f);
    // _avoid_obstacle (:244-253)
    const float cm = costmap_at(a.cm, a.cm_size, a.hw, a.res_c, s.x, s.y);
    if (cm > a.thr) c.ob = c.ob + a.pen;
    c.ob = c.ob + cm;
    if constexpr (DUMP) {
      if (valid) {
        const size_t o3 = ((size_t)kl * H + t) * 3;
        if (a.d_traj) { a.d_traj[o3] = s.x; a.d_traj[o3 + 1] = s.y; a.d_traj[o3 + 2] = o.z; }
        if (a.d_hv) { a.d_hv[o3] = s.hx; a.d_hv[o3 + 1] = s.hy; a.d_hv[o3 + 2] = s.hz; }
        if (a.d_lw) { a.d_lw[o3] = o.lx; a.d_lw[o3 + 1] = o.ly; a.d_lw[o3 + 2] = o.lz; }
        if (a.d_rw) { a.d_rw[o3] = o.rx; a.d_rw[o3 + 1] = o.ry; a.d_rw[o3 + 2] = o.rz; }
        const size_t o1 = (size_t)kl * H + t;
        if (a.d_v) a.d_v[o1] = v;
        if (a.d_w) a.d_w[o1] = w;
        if (a.d_u1) a.d_u1[o1] = u1;
        if (a.d_u2) a.d_u2[o1] = u2;
      }
    }
  };

  // sampled control u[k,t] (sampling_warp.py:71-92, noise DEFINED as Philox + Box-Muller)
  auto sample = [&](int t, float e1, float e2, float& u1, float& u2) {
    const int ti = min(t + 1, H - 1);
    u1 = clampf(a.u_nom1[ti] + a.s1 * e1, a.min_u1, a.max_u1);
    u2 = clampf(a.u_nom2[ti] + a.s2 * e2, a.min_u2, a.max_u2);
  };

  for (int t = 0; t < H; t += 2) {
    float u1a, u2a, u1b, u2b;
    if constexpr (MODE == 0) {
      float e1a, e2a, e1b, e2b;
      noise_block(a.seed, a.n_base + (uint64_t)(t >> 1), kg, &e1a, &e2a, &e1b, &e2b);
      sample(t, e1a, e2a, u1a, u2a);
      sample(t + 1, e1b, e2b, u1b, u2b);
    } else {
      const size_t o = (size_t)(valid ? kl : 0) * H + t;
      u1a = a.inj_u1[o];
      u2a = a.inj_u2[o];
      u1b = (t + 1 < H) ? a.inj_u1[o + 1] : 0.0f;
      u2b = (t + 1 < H) ? a.inj_u2[o + 1] : 0.0f;
    }
    one_step(t, u1a, u2a);
    if (t + 1 < H) one_step(t + 1, u1b, u2b);
  }

  // ---- _evaluate_trajectories_kernel (critics_warp.py:325-329), costs[] zeroed by reset
  float pf;
  if (a.pf_far) {
    const float dx = c.last_x - a.igx, dy = c.last_y - a.igy;
    pf = (dx * dx + dy * dy) * a.pf_scale;
  } else {
    pf = c.pf_sum;
  }
  float cost = a.w_path * pf;
  cost = cost + a.w_slope * c.sw;
  cost = cost + a.w_speed * c.sp;
  cost = cost + a.w_obs * c.ob;
  if (valid) a.cost_out[kl] = cost;

  // ---- softmax leaf records (DEFINED replacement of critics_warp.py:338-376)
  __syncthreads();  // LDS window no longer needed: reuse it as reduction scratch
  const int E = 2 * H + 2;
  double* red = reinterpret_cast<double*>(smem_raw);     // [NW][2H+1]
  float* leaf_m = reinterpret_cast<float*>(red + NW * (2 * H + 1));  // [NW/4]
  const float cval = valid ? cost : INFINITY;
  float wm = wave_min(cval);
  if (lane == 0) leaf_m[wave] = wm;  // temporarily per wave
  __syncthreads();
  const int leaf = wave >> 2;
  const float m_leaf =
      fminf(fminf(leaf_m[4 * leaf], leaf_m[4 * leaf + 1]), fminf(leaf_m[4 * leaf + 2], leaf_m[4 * leaf + 3]));
  const bool finite = cval < INFINITY;
  const float wgt = finite ? dm_expf(-((cval - m_leaf) / a.T)) : 0.0f;
  const double wd = (double)wgt;
  {
    const double sw = wave_sum(wd);
    if (lane == 0) red[wave * (2 * H + 1) + 2 * H] = sw;
  }
  // regenerate u[k,t] (bitwise identical to the rollout) and reduce w*u per t
  for (int t = 0; t < H; t += 2) {
    float u1a, u2a, u1b, u2b;
    if constexpr (MODE == 0) {
      float e1a, e2a, e1b, e2b;
      noise_block(a.seed, a.n_base + (uint64_t)(t >> 1), kg, &e1a, &e2a, &e1b, &e2b);
      sample(t, e1a, e2a, u1a, u2a);
      sample(t + 1, e1b, e2b, u1b, u2b);
    } else {
      const size_t o = (size_t)(valid ? kl : 0) * H + t;
      u1a = a.inj_u1[o];
      u2a = a.inj_u2[o];
      u1b = (t + 1 < H) ? a.inj_u1[o + 1] : 0.0f;
      u2b = (t + 1 < H) ? a.inj_u2[o + 1] : 0.0f;
    }
    const double p1a = wave_sum(wd * (double)u1a);
    const double p2a = wave_sum(wd * (double)u2a);
    if (lane == 0) {
      red[wave * (2 * H + 1) + t] = p1a;
      red[wave * (2 * H + 1) + H + t] = p2a;
    }
    if (t + 1 < H) {
      const double p1b = wave_sum(wd * (double)u1b);
      const double p2b = wave_sum(wd * (double)u2b);
      if (lane == 0) {
        red[wave * (2 * H + 1) + t + 1] = p1b;
        red[wave * (2 * H + 1) + H + t + 1] = p2b;
      }
    }
  }
  __syncthreads();
  // leaf records: ((W0 + W1) + (W2 + W3)); then the block's subtree over its leaves
  constexpr int NL = NW / 4;
  for (int j = tid; j < E; j += BLOCK) {
    double val[NL];
    float lm[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      lm[l] = fminf(fminf(leaf_m[4 * l], leaf_m[4 * l + 1]), fminf(leaf_m[4 * l + 2], leaf_m[4 * l + 3]));
      if (j == 0) {
        val[l] = (double)lm[l];
      } else {
        const int jj = (j == 1) ? 2 * H : j - 2;  // record [m, S, V1, V2] <- red [V1, V2, S]
        const double* rr = red + (4 * l) * (2 * H + 1) + jj;
        const int st = 2 * H + 1;
        val[l] = (rr[0] + rr[st]) + (rr[2 * st] + rr[3 * st]);
      }
    }
#pragma unroll
    for (int width = NL; width > 1; width >>= 1) {
#pragma unroll
      for (int l = 0; l < width / 2; ++l) {
        const PairScale ps = pair_scale(lm[2 * l], lm[2 * l + 1], a.T);
        val[l] = pair_apply(ps, val[2 * l], val[2 * l + 1], j);
        lm[l] = ps.m;  // fminf(m, +inf) = m covers the empty-child modes
      }
    }
    a.nodes[(size_t)blockIdx.x * E + j] = val[0];
  }
}

// =====================================================================  finish kernel
// Tree over n records (padded to a power of two with empty records), then
// (MODE_RECORD) write the root, or (MODE_FINISH) u_opt = V/S, optimal filter
// (MPPI_isaac.py:672-692) and the 3D rollout of the optimal sequence (:696-720).
template <bool LDS>
__global__ __launch_bounds__(1024) void mppi_finish_kernel(const FinishArgs f) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int tid = threadIdx.x;
  const int H = f.H;
  const int E = 2 * H + 2;
  PairScale* scales = reinterpret_cast<PairScale*>(smem_raw);  // [1024]

  const double* cur = f.recs;
  int n = f.n_recs;
  double* bufs[2] = {f.scratch0, f.scratch1};
  int flip = 0;
  while (n > 1) {
    const int pairs = (n + 1) >> 1;
    double* out = bufs[flip];
    for (int p0 = 0; p0 < pairs; p0 += 1024) {
      const int np = min(1024, pairs - p0);
      if (tid < np) {
        const int p = p0 + tid;
        const float ma = (float)cur[(size_t)(2 * p) * E];
        const float mb = (2 * p + 1 < n) ? (float)cur[(size_t)(2 * p + 1) * E] : INFINITY;
        scales[tid] = pair_scale(ma, mb, f.T);
      }
      __syncthreads();
      for (int it = tid; it < np * E; it += 1024) {
        const int pl = it / E, j = it - pl * E;
        const int p = p0 + pl;
        const double va = cur[(size_t)(2 * p) * E + j];
        const double vb = (2 * p + 1 < n) ? cur[(size_t)(2 * p + 1) * E + j] : 0.0;
        out[(size_t)p * E + j] = pair_apply(scales[pl], va, vb, j);
      }
      __syncthreads();
    }
    cur = out;
    n = pairs;
    flip ^= 1;
  }
  if (f.mode == 0) {  // rank record
    for (int j = tid; j < E; j += 1024) f.record_out[j] = (n == 1) ? cur[j] : (j == 0 ? INFINITY : 0.0);
    return;
  }
  // ---- u_opt = V / S (DEFINED; zero if no finite cost)
  float* uo = reinterpret_cast<float*>(smem_raw);  // [2H] (scales no longer needed)
  __syncthreads();
  const double S = (n == 1) ? cur[1] : 0.0;
  for (int j = tid; j < 2 * H; j += 1024) {
    const float u = (S > 0.0) ? (float)(cur[2 + j] / S) : 0.0f;
    uo[j] = u;
    f.u_nom_next[j] = u;
    f.out[j] = u;
  }
  float* win = reinterpret_cast<float*>(smem_raw + f.win_offset);
  if constexpr (LDS) {
    const int lane = tid & 63, wave = tid >> 6;
    for (int r = wave; r < f.Wr; r += 16) {
      const float* src = f.Z + (size_t)(f.wy0 + r) * f.grid + f.wx0;
      float* dst = win + r * f.W;
      for (int c2 = lane; c2 < f.W; c2 += 64) dst[c2] = src[c2];
    }
  }
  __syncthreads();
  if (tid != 0) return;
  Dem<LDS> dem;
  dem.Z = f.Z;
  dem.win = win;
  dem.rows = f.rows;
  dem.grid = f.grid;
  dem.wx0 = f.wx0;
  dem.wy0 = f.wy0;
  dem.W = f.W;
  dem.Wr = f.Wr;
  dem.x_min = f.x_min;
  dem.y_min = f.y_min;
  dem.res = f.res;
  const float res_half_neg = (-f.res) / 2.0f;
  const float res_sq = f.res * f.res;
  float* o_v = f.out + 2 * H;
  float* o_w = f.out + 3 * H;
  float* o_traj = f.out + 4 * H;
  float* o_hv = f.out + 7 * H;
  float* o_lw = f.out + 10 * H;
  float* o_rw = f.out + 13 * H;
  Traj s;
  s.x = f.x0;
  s.y = f.y0;
  {
    float q00, q01, q10, q11;
    dem.corners(s.x, s.y, q00, q01, q10, q11);
    const float vx = res_half_neg * (((q01 - q00) - q10) + q11);
    const float vy = res_half_neg * (((q10 - q00) - q01) + q11);
    const float nn = sqrtf((vx * vx + vy * vy) + res_sq * res_sq);
    const float nx = vx / nn, ny = vy / nn, nz = res_sq / nn;
    const float d = (f.h0x * nx + f.h0y * ny) + f.h0z * nz;
    float tx = f.h0x - d * nx, ty = f.h0y - d * ny, tz = f.h0z - d * nz;
    const float tn = sqrtf((tx * tx + ty * ty) + tz * tz);
    s.hx = tx / tn;
    s.hy = ty / tn;
    s.hz = tz / tn;
  }
  float L = f.wl, R = f.wr;
  const float one_m_a = 1.0f - f.oa;
  for (int t = 0; t < H; ++t) {
    L = L * f.oa + (uo[t] * f.ok) * one_m_a;
    R = R * f.oa + (uo[H + t] * f.ok) * one_m_a;
    const float v = clampf((L + R) / 2.0f, f.vmin, f.vmax);
    const float w = clampf(((-L) + R) / f.rwheel, f.wmin, f.wmax);
    o_v[t] = v;
    o_w[t] = w;
    StepOut o;
    step3d<LDS>(dem, res_half_neg, res_sq, f.dt, f.off, v, w, s, o);
    o_traj[3 * t] = s.x; o_traj[3 * t + 1] = s.y; o_traj[3 * t + 2] = o.z;
    o_hv[3 * t] = s.hx; o_hv[3 * t + 1] = s.hy; o_hv[3 * t + 2] = s.hz;
    o_lw[3 * t] = o.lx; o_lw[3 * t + 1] = o.ly; o_lw[3 * t + 2] = o.lz;
    o_rw[3 * t] = o.rx; o_rw[3 * t + 1] = o.ry; o_rw[3 * t + 2] = o.rz;
  }
}

// =====================================================================  standalone bilinear
// Scattered-query corner lookup + bilinear (projection_warp.py:8-100) over the
// full DEM in HBM: one lane per query, float4 query loads.
__global__ __launch_bounds__(256) void mppi_bilinear_kernel(const float* __restrict__ Z, int rows,
                                                            int grid, float x_min, float y_min,
                                                            float res, const float* __restrict__ xs,
                                                            const float* __restrict__ ys,
                                                            float* __restrict__ hs, int64_t n) {
  Dem<false> dem;
  dem.Z = Z;
  dem.win = nullptr;
  dem.rows = rows;
  dem.grid = grid;
  dem.wx0 = dem.wy0 = 0;
  dem.W = dem.Wr = 0;
  dem.x_min = x_min;
  dem.y_min = y_min;
  dem.res = res;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float x = xs[i], y = ys[i];
    float q00, q01, q10, q11;
    dem.corners(x, y, q00, q01, q10, q11);
    hs[i] = bilinear(x, y, q00, q01, q10, q11, res);
  }
}

// =====================================================================  launchers
template <int BLOCK, bool LDS, int PROJ, int MODE, bool DUMP>
static hipError_t launch_rollout_t(const RolloutArgs& a, int blocks, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((mppi_rollout_kernel<BLOCK, LDS, PROJ, MODE, DUMP>), dim3(blocks), dim3(BLOCK),
                     lds, st, a);
  return hipGetLastError();
}

template <int BLOCK, bool LDS, int PROJ>
static hipError_t launch_rollout_m(const RolloutArgs& a, int blocks, size_t lds, hipStream_t st,
                                   int mode, bool dump) {
  if (mode == 0) {
    if (dump) return launch_rollout_t<BLOCK, LDS, PROJ, 0, true>(a, blocks, lds, st);
    return launch_rollout_t<BLOCK, LDS, PROJ, 0, false>(a, blocks, lds, st);
  }
  if (dump) return launch_rollout_t<BLOCK, LDS, PROJ, 1, true>(a, blocks, lds, st);
  return launch_rollout_t<BLOCK, LDS, PROJ, 1, false>(a, blocks, lds, st);
}

template <int BLOCK>
static hipError_t launch_rollout_b(const RolloutArgs& a, int blocks, size_t lds, hipStream_t st,
                                   bool use_lds, int proj, int mode, bool dump) {
  if (use_lds) {
    if (proj == 3) return launch_rollout_m<BLOCK, true, 3>(a, blocks, lds, st, mode, dump);
    return launch_rollout_m<BLOCK, true, 2>(a, blocks, lds, st, mode, dump);
  }
  if (proj == 3) return launch_rollout_m<BLOCK, false, 3>(a, blocks, lds, st, mode, dump);
  return launch_rollout_m<BLOCK, false, 2>(a, blocks, lds, st, mode, dump);
}

hipError_t launch_rollout(const RolloutArgs& a, int block, int blocks, size_t lds, hipStream_t st,
                          bool use_lds, int proj, int mode, bool dump) {
  switch (block) {
    case 256: return launch_rollout_b<256>(a, blocks, lds, st, use_lds, proj, mode, dump);
    case 512: return launch_rollout_b<512>(a, blocks, lds, st, use_lds, proj, mode, dump);
    case 1024: return launch_rollout_b<1024>(a, blocks, lds, st, use_lds, proj, mode, dump);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_finish(const FinishArgs& f, size_t lds, hipStream_t st, bool use_lds) {
  if (use_lds)
    hipLaunchKernelGGL(mppi_finish_kernel<true>, dim3(1), dim3(1024), lds, st, f);
  else
    hipLaunchKernelGGL(mppi_finish_kernel<false>, dim3(1), dim3(1024), lds, st, f);
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
