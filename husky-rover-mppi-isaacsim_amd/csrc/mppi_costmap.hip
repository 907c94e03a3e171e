// On-device obstacle costmap builder: the work of
// Surface.create_obstacles_costmap (thesis_master/warp_implementation/MPPI_isaac.py:361-378),
// which the Isaac loop re-runs on every high-resolution block change
// (visual_terrain_stack_full_terrain.py:561-563) before re-uploading the result.
//
//   raster   disc mask (X - x_local)^2 + (Y - y_local)^2 <= r_total^2 per obstacle  (:365-372)
//   EDT      distance of every free cell to the nearest occupied one               (:374)
//   scale    min-max normalise to [0, 1]                                           (:375)
//   cost     (1 - d)^power                                                         (:376)
//
// DEFINED (oracle/costmap_ref.py): the distance is the exact Euclidean one (scipy's EDT), not
// cv2's 5x5 chamfer approximation (cv2 is not available to pin it), the normalisation and
// the power run in float64 and the result is rounded once to float32.  Squared distances are
// integers, computed exactly: a column pass (vertical distance to the nearest obstacle, from
// per-segment first/last occupied rows) and a row pass (min over x' of (x - x')^2 + g(x')^2,
// searched outwards from x only while o^2 can still improve the best).  The arithmetic is
// HBM/latency-light: ~22 B per cell in six short launches; see DESIGN.md §3.4.
#include <climits>

#include "mppi_costmap.h"

namespace mppi {

namespace {

constexpr int CM_THREADS = 256;

// One workgroup per obstacle: mark the cells of its (conservative) bounding box that pass the
// reference's float64 disc test.  Workgroup 0 also re-arms the min/max cell.
__global__ __launch_bounds__(CM_THREADS) void costmap_raster_kernel(const double* __restrict__ obs, int n_obs,
                                                                    const double* __restrict__ xs, int size,
                                                                    uint8_t* __restrict__ occ,
                                                                    int32_t* __restrict__ range) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    range[0] = INT_MAX;
    range[1] = -1;
  }
  if ((int)blockIdx.x >= n_obs) return;
  const double xl = obs[3 * blockIdx.x + 0];
  const double yl = obs[3 * blockIdx.x + 1];
  const double r2 = obs[3 * blockIdx.x + 2];  // total_radius**2 (host pow, as CPython's float **)
  const double r = sqrt(r2);
  const double lo = xs[0], step = (xs[size - 1] - xs[0]) / (double)(size - 1);
  // cell index range of [c - r, c + r], widened by two cells on each side (the exact test decides)
  auto span = [&](double c, int& a, int& b) {
    double fa = (c - r - lo) / step - 2.0, fb = (c + r - lo) / step + 2.0;
    fa = fmax(fa, 0.0);
    fb = fmin(fb, (double)(size - 1));
    if (!(fa <= fb)) {  // outside the map (or NaN)
      a = 1;
      b = 0;
      return;
    }
    a = (int)fa;
    b = (int)fb;
  };
  int i0, i1, j0, j1;
  span(xl, i0, i1);
  span(yl, j0, j1);
  if (i0 > i1 || j0 > j1) return;
  const int bw = i1 - i0 + 1;
  const int cells = bw * (j1 - j0 + 1);
  for (int c = threadIdx.x; c < cells; c += CM_THREADS) {
    const int i = i0 + c % bw, j = j0 + c / bw;
    const double dx = xs[i] - xl;  // X_costmap[j, i] = xs[i]
    const double dy = xs[j] - yl;  // Y_costmap[j, i] = xs[j]
    if (dx * dx + dy * dy <= r2) occ[(size_t)j * size + i] = 1;
  }
}

// Column pass, part 1: first / last occupied row of each COSTMAP_SEG-row segment of a column.
__global__ __launch_bounds__(CM_THREADS) void costmap_colseg_kernel(const uint8_t* __restrict__ occ, int size,
                                                                    int32_t* __restrict__ first,
                                                                    int32_t* __restrict__ last) {
  const int col = blockIdx.x * CM_THREADS + threadIdx.x;
  const int seg = blockIdx.y;
  if (col >= size) return;
  const int r0 = seg * COSTMAP_SEG, r1 = min(size, r0 + COSTMAP_SEG);
  uint8_t v[COSTMAP_SEG];
#pragma unroll
  for (int k = 0; k < COSTMAP_SEG; ++k) v[k] = (r0 + k < r1) ? occ[(size_t)(r0 + k) * size + col] : 0;
  int f = -1, l = -1;
#pragma unroll
  for (int k = COSTMAP_SEG - 1; k >= 0; --k)
    if (v[k]) f = r0 + k;
#pragma unroll
  for (int k = 0; k < COSTMAP_SEG; ++k)
    if (v[k]) l = r0 + k;
  first[(size_t)seg * size + col] = f;
  last[(size_t)seg * size + col] = l;
}

// Column pass, part 2: g(col, row) = distance to the nearest occupied row of the column (INF if
// none), stored squared.  INF = 2*size+1 so INF^2 loses against every real candidate.
__global__ __launch_bounds__(CM_THREADS) void costmap_colg_kernel(const uint8_t* __restrict__ occ, int size,
                                                                  int nseg, const int32_t* __restrict__ first,
                                                                  const int32_t* __restrict__ last,
                                                                  int32_t* __restrict__ g2) {
  const int col = blockIdx.x * CM_THREADS + threadIdx.x;
  const int seg = blockIdx.y;
  if (col >= size) return;
  const int INF = 2 * size + 1;
  int above = -1, below = -1;
  for (int s = seg - 1; s >= 0; --s) {
    const int l = last[(size_t)s * size + col];
    if (l >= 0) {
      above = l;
      break;
    }
  }
  for (int s = seg + 1; s < nseg; ++s) {
    const int f = first[(size_t)s * size + col];
    if (f >= 0) {
      below = f;
      break;
    }
  }
  const int r0 = seg * COSTMAP_SEG, r1 = min(size, r0 + COSTMAP_SEG);
  uint8_t v[COSTMAP_SEG];
#pragma unroll
  for (int k = 0; k < COSTMAP_SEG; ++k) v[k] = (r0 + k < r1) ? occ[(size_t)(r0 + k) * size + col] : 0;
  int up[COSTMAP_SEG];
  int prev = above;
#pragma unroll
  for (int k = 0; k < COSTMAP_SEG; ++k) {
    if (v[k]) prev = r0 + k;
    up[k] = prev >= 0 ? r0 + k - prev : INF;
  }
  int nxt = below;
#pragma unroll
  for (int k = COSTMAP_SEG - 1; k >= 0; --k) {
    if (v[k]) nxt = r0 + k;
    const int dn = nxt >= 0 ? nxt - (r0 + k) : INF;
    const int g = min(up[k], dn);
    if (r0 + k < r1) g2[(size_t)(r0 + k) * size + col] = g * g;
  }
}

__device__ inline int wave_min(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ inline int wave_max(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// Row pass: one workgroup per row, the row's g^2 in LDS.  d2(x) = min_x' (x - x')^2 + g2(x'),
// searched from o = 0 outwards while o^2 < best (no farther column can win).
__global__ __launch_bounds__(CM_THREADS) void costmap_row_kernel(const int32_t* __restrict__ g2, int size,
                                                                 int32_t* __restrict__ d2,
                                                                 int32_t* __restrict__ range) {
  extern __shared__ int32_t srow[];
  __shared__ int red[2][CM_THREADS / 64];
  const size_t base = (size_t)blockIdx.x * size;
  for (int x = threadIdx.x; x < size; x += CM_THREADS) srow[x] = g2[base + x];
  __syncthreads();
  int mn = INT_MAX, mx = -1;
  for (int x = threadIdx.x; x < size; x += CM_THREADS) {
    int best = srow[x];
    for (int o = 1; o * o < best; ++o) {
      const bool l = x - o >= 0, r = x + o < size;
      if (!l && !r) break;
      const int oo = o * o;
      if (l) best = min(best, oo + srow[x - o]);
      if (r) best = min(best, oo + srow[x + o]);
    }
    d2[base + x] = best;
    mn = min(mn, best);
    mx = max(mx, best);
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = mn;
    red[1][w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < CM_THREADS / 64; ++k) {
      mn = min(mn, red[0][k]);
      mx = max(mx, red[1][k]);
    }
    atomicMin(&range[0], mn);
    atomicMax(&range[1], mx);
  }
}

// x^n in double-double (exponentiation by squaring with exact fma products), rounded once to
// double: the correctly rounded power barring a 2^-99-relative tie, i.e. what numpy's
// float64 `**` (libm pow) returns.
__device__ inline double pow_int_dd(double x, int n) {
  double rh = 1.0, rl = 0.0, bh = x, bl = 0.0;
  auto mul = [](double ah, double al, double ch, double cl, double& oh, double& ol) {
    const double p = ah * ch;
    double e = fma(ah, ch, -p);
    e += ah * cl + al * ch;
    const double s = p + e;
    ol = e - (s - p);
    oh = s;
  };
  while (n > 0) {
    if (n & 1) mul(rh, rl, bh, bl, rh, rl);
    n >>= 1;
    if (n) mul(bh, bl, bh, bl, bh, bl);
  }
  return rh;
}

// d = sqrt(d2); dn = (d - lo) / (hi - lo) (0 when hi == lo); out = float((1 - dn)^power).
__global__ __launch_bounds__(CM_THREADS) void costmap_scale_kernel(const int32_t* __restrict__ d2, int64_t n,
                                                                   const int32_t* __restrict__ range, int power,
                                                                   float* __restrict__ out) {
  const double lo = sqrt((double)range[0]);
  const double hi = sqrt((double)range[1]);
  const double span = hi - lo;
  for (int64_t i = (int64_t)blockIdx.x * CM_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * CM_THREADS) {
    const double d = sqrt((double)d2[i]);
    const double dn = hi > lo ? (d - lo) / span : 0.0;
    out[i] = (float)pow_int_dd(1.0 - dn, power);
  }
}

// ---------------------------------------------------------------------  cv2 DIST_L2 mask-5 chamfer
// cv2.distanceTransform(obs_costmap, DIST_L2, 5) (MPPI_isaac.py:374), restated from OpenCV's
// published distanceTransform_5x5 (imgproc/src/distransform.cpp; oracle/costmap_ref.py
// chamfer_l2_5x5): metrics {1, 1.4, 2.1969} in 16.16 fixed point, INIT_DIST0 = INT_MAX on a
// 2-pixel border, a forward raster pass over the upper half-mask, a backward one over the lower
// half, d = float(t) / 65536.  Rows depend on the two previous rows, so both passes walk the rows
// in order on ONE wave (no workgroup barrier; LDS holds the last three rows); inside a row the
// left-to-right chain t[j] = min(a[j], t[j-1] + 1.0) is a min-plus scan: each lane runs it over
// its contiguous chunk, a 64-lane exclusive min-scan of (chunk end - column * 1.0) carries the
// chain across chunks, exact in integers (the sequential sums never exceed 2^32 at size <= 8192).
constexpr uint32_t CV_HV = 65536u, CV_DIAG = 91750u, CV_LONG = 143976u, CV_INIT = 0x7FFFFFFFu;
constexpr int CH_B = 2;  // border columns each side

// Exclusive min-scans over the 64 lanes of a wave with DPP row shifts / broadcasts (no LDS):
// up = min over lanes < lane, down = min over lanes > lane (the lane order reversed around an
// upward scan); UINT_MAX for none.
__device__ inline uint32_t dpp_min(uint32_t x, uint32_t y) { return x < y ? x : y; }
__device__ inline uint32_t wave_incl_min_scan(uint32_t x) {
  x = dpp_min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x111, 0xF, 0xF, false));  // row_shr:1
  x = dpp_min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x112, 0xF, 0xF, false));  // row_shr:2
  x = dpp_min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x114, 0xF, 0xF, false));  // row_shr:4
  x = dpp_min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x118, 0xF, 0xF, false));  // row_shr:8
  x = dpp_min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x142, 0xA, 0xF, false));  // row_bcast:15
  x = dpp_min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return x;
}
__device__ inline uint32_t wave_excl_min_scan_up(uint32_t v) {
  const uint32_t x = wave_incl_min_scan(v);
  return (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x138, 0xF, 0xF, false);  // wave_shr:1
}
__device__ inline uint32_t wave_excl_min_scan_down(uint32_t v, int lane) {
  const uint32_t r = (uint32_t)__shfl((int)v, 63 - lane, 64);
  const uint32_t x = wave_excl_min_scan_up(r);
  return (uint32_t)__shfl((int)x, 63 - lane, 64);
}

// One workgroup of CH_T threads walks the rows of both passes; thread t owns the contiguous
// columns [t C, t C + C) (C = ceil(W / CH_T) <= CM), so a 1024^2 map has one column per thread.
// Per row: the thread's chunk from the three LDS rows (7 mask taps per column), its in-chunk
// chain, then the carry of the row chain across chunks as an exclusive min-scan over the
// workgroup (a 64-lane DPP scan inside each wave, the waves' totals through LDS), the row written
// to LDS and global memory; two barriers per row (totals visible / row visible).  Round 2 ran the
// same arithmetic on one wave (C = W / 64 columns per lane): 3.96 ms per 1024^2 map.
constexpr int CH_T = 1024;
constexpr int CH_W = CH_T / 64;  // waves

// min over the waves strictly before (UP) / after (!UP) wave w of their totals tot[0..CH_W)
template <bool UP>
__device__ inline uint32_t waves_prefix_min(const uint32_t* tot, int w, int lane) {
  uint32_t x = 0xFFFFFFFFu;
  if (lane < CH_W && (UP ? lane < w : lane > w)) x = tot[lane];
  // min over lanes 0..15 (row 0 of the wave): row_shr 1, 2, 4, 8, then lane 15 holds it
  x = dpp_min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x111, 0xF, 0xF, false));
  x = dpp_min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x112, 0xF, 0xF, false));
  x = dpp_min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x114, 0xF, 0xF, false));
  x = dpp_min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x118, 0xF, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
}

// Global reads of later rows (occupancy forward, the forward result backward) are issued CH_PF
// rows ahead into a register ring: a row takes well under the HBM latency.
constexpr int CH_PF = 4;

template <int CM>
__global__ __launch_bounds__(CH_T) void costmap_chamfer_kernel(const uint8_t* __restrict__ occ, int H, int W,
                                                               uint32_t* __restrict__ tmp, float* __restrict__ dist,
                                                               int32_t* __restrict__ range) {
  extern __shared__ uint32_t srows[];  // [3][W + 4] rows, then [2][CH_W] wave totals
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int S = W + 2 * CH_B;
  uint32_t* tot = srows + 3 * S;
  const int C = (W + CH_T - 1) / CH_T;
  const int j0 = min(W, tid * C), j1 = min(W, j0 + C);
  for (int k = tid; k < 3 * S; k += CH_T) srows[k] = CV_INIT;
  __syncthreads();
  uint32_t loc[CM];
  uint32_t pre[CH_PF][CM];  // rows i .. i + CH_PF - 1 of the pass's global input, slot r % CH_PF
  auto load_occ = [&](int r, uint32_t (&dst)[CM]) __attribute__((always_inline)) {
    const uint8_t* row = occ + (size_t)min(r, H - 1) * W;
#pragma unroll
    for (int k = 0; k < CM; ++k) dst[k] = j0 + k < j1 ? row[j0 + k] : 0u;
  };
  auto load_tmp = [&](int r, uint32_t (&dst)[CM]) __attribute__((always_inline)) {
    const uint32_t* row = tmp + (size_t)max(r, 0) * W;
#pragma unroll
    for (int k = 0; k < CM; ++k) dst[k] = j0 + k < j1 ? row[j0 + k] : 0u;
  };
  // ---- forward pass: rows top to bottom, columns left to right
  auto frow = [&](int i, uint32_t (&oc)[CM]) __attribute__((always_inline)) {
    const uint32_t* up2 = srows + ((i + 1) % 3) * S + CH_B;  // row i - 2 (INIT above the map)
    const uint32_t* up1 = srows + ((i + 2) % 3) * S + CH_B;  // row i - 1
    uint32_t* cur = srows + (i % 3) * S + CH_B;
    uint64_t run = 0xFFFFFFFFull;  // the chain inside the chunk, no left input yet
#pragma unroll
    for (int k = 0; k < CM; ++k) {
      const int j = j0 + k;
      const int jc = min(j, W - 1);  // (columns past the chunk end are computed, not kept)
      uint32_t t = min(up2[jc - 1] + CV_LONG, up2[jc + 1] + CV_LONG);
      t = min(t, up1[jc - 2] + CV_LONG);
      t = min(t, up1[jc - 1] + CV_DIAG);
      t = min(t, up1[jc] + CV_HV);
      t = min(t, up1[jc + 1] + CV_DIAG);
      t = min(t, up1[jc + 2] + CV_LONG);
      const uint64_t nr = oc[k] ? 0ull : min((uint64_t)t, run + CV_HV);
      run = j < j1 ? nr : run;
      loc[k] = (uint32_t)nr;
    }
    load_occ(i + CH_PF, oc);  // this slot's next row
    // value at column j0 - 1: a source at column js holding v contributes v + (j - js) HV, the
    // border (INIT at column -1) INIT + (j + 1) HV; carried as v + (W - js) HV, which stays below
    // 2^32 (v < 3.3e9, W HV < 5.4e8 at W <= 8192), and the minimum exceeds (W - j) HV
    const uint32_t mine = j0 < j1 ? (uint32_t)run + (uint32_t)(W - (j1 - 1)) * CV_HV : 0xFFFFFFFFu;
    const uint32_t incl = wave_incl_min_scan(mine);
    const uint32_t excl = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)incl, 0x138, 0xF, 0xF, false);
    uint32_t* tt = tot + (i & 1) * CH_W;
    if (lane == 63) tt[wv] = incl;
    __syncthreads();  // wave totals visible; every thread has read the rows it needs (cur written below)
    const uint32_t carry = min(min(excl, waves_prefix_min<true>(tt, wv, lane)), CV_INIT + (uint32_t)(W + 1) * CV_HV);
#pragma unroll
    for (int k = 0; k < CM; ++k) {
      const int j = j0 + k;
      if (j < j1) {
        const uint32_t v = min(loc[k], carry - (uint32_t)(W - j) * CV_HV);
        cur[j] = v;
        tmp[(size_t)i * W + j] = v;
      }
    }
    __syncthreads();  // row i visible
  };
#pragma unroll
  for (int q = 0; q < CH_PF; ++q) load_occ(q, pre[q]);
  int i = 0;
  for (; i + CH_PF <= H; i += CH_PF) {
#pragma unroll
    for (int q = 0; q < CH_PF; ++q) frow(i + q, pre[q]);
  }
#pragma unroll
  for (int q = 0; q < CH_PF; ++q)
    if (i + q < H) frow(i + q, pre[q]);
  __threadfence_block();  // the forward rows in tmp are re-read below by the same threads only
  // ---- backward pass: rows bottom to top, columns right to left
  for (int k = tid; k < 3 * S; k += CH_T) srows[k] = CV_INIT;
  __syncthreads();
  float dmin = INFINITY, dmax = -INFINITY;
  auto brow = [&](int i, uint32_t (&fc)[CM]) __attribute__((always_inline)) {
    const int r = H - 1 - i;                                  // rows done so far
    const uint32_t* dn2 = srows + ((r + 1) % 3) * S + CH_B;  // row i + 2 (INIT below the map)
    const uint32_t* dn1 = srows + ((r + 2) % 3) * S + CH_B;  // row i + 1
    uint32_t* cur = srows + (r % 3) * S + CH_B;
    uint64_t run = 0xFFFFFFFFull;
#pragma unroll
    for (int k = CM - 1; k >= 0; --k) {  // right to left
      const int j = j0 + k;
      const int jc = min(j, W - 1);
      uint32_t t = fc[k];
      t = min(t, dn2[jc + 1] + CV_LONG);
      t = min(t, dn2[jc - 1] + CV_LONG);
      t = min(t, dn1[jc + 2] + CV_LONG);
      t = min(t, dn1[jc + 1] + CV_DIAG);
      t = min(t, dn1[jc] + CV_HV);
      t = min(t, dn1[jc - 1] + CV_DIAG);
      t = min(t, dn1[jc - 2] + CV_LONG);
      const uint64_t nr = min((uint64_t)t, run + CV_HV);
      run = j < j1 ? nr : run;
      loc[k] = (uint32_t)nr;
    }
    load_tmp(i - CH_PF, fc);
    // value at column j1: a source at column js holding v contributes v + (js - j) HV, the border
    // (INIT at column W) INIT + (W - j) HV; carried as v + js HV (< 2^32 as above)
    const uint32_t mine = j0 < j1 ? (uint32_t)run + (uint32_t)j0 * CV_HV : 0xFFFFFFFFu;
    const uint32_t down = wave_excl_min_scan_down(mine, lane);
    // this wave's total: the inclusive scan from the top lane down, read at lane 0
    const uint32_t wtot = min(down, mine);
    uint32_t* tt = tot + (i & 1) * CH_W;
    if (lane == 0) tt[wv] = wtot;
    __syncthreads();
    const uint32_t carry = min(min(down, waves_prefix_min<false>(tt, wv, lane)), CV_INIT + (uint32_t)W * CV_HV);
#pragma unroll
    for (int k = 0; k < CM; ++k) {
      const int j = j0 + k;
      if (j < j1) {
        const uint32_t v = min(loc[k], carry - (uint32_t)j * CV_HV);
        cur[j] = v;
        const float d = (float)v * (1.0f / 65536.0f);
        dist[(size_t)i * W + j] = d;
        dmin = fminf(dmin, d);
        dmax = fmaxf(dmax, d);
      }
    }
    __syncthreads();
  };
#pragma unroll
  for (int q = 0; q < CH_PF; ++q) load_tmp(H - 1 - q, pre[q]);
  i = H - 1;
  for (; i - CH_PF + 1 >= 0; i -= CH_PF) {
#pragma unroll
    for (int q = 0; q < CH_PF; ++q) brow(i - q, pre[q]);
  }
#pragma unroll
  for (int q = 0; q < CH_PF; ++q)
    if (i - q >= 0) brow(i - q, pre[q]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    dmin = fminf(dmin, __shfl_xor(dmin, o, 64));
    dmax = fmaxf(dmax, __shfl_xor(dmax, o, 64));
  }
  float* red = reinterpret_cast<float*>(srows);  // the rows are dead now
  if (lane == 0) {
    red[wv] = dmin;
    red[CH_W + wv] = dmax;
  }
  __syncthreads();
  if (tid == 0) {
    for (int k = 1; k < CH_W; ++k) {
      dmin = fminf(dmin, red[k]);
      dmax = fmaxf(dmax, red[CH_W + k]);
    }
    range[0] = __builtin_bit_cast(int32_t, dmin);
    range[1] = __builtin_bit_cast(int32_t, dmax);
  }
}

// cv2.normalize(NORM_MINMAX, 0, 1) (:375) as OpenCV 4.x's cv::normalize / convertTo write it for a
// CV_32F destination: scale = 1 / (smax - smin) (0 if smax - smin <= DBL_EPSILON) rounded to
// float, shift = -(float)(smin * scale), dst = fma(src, scale, shift) in float32 (cvt_32f's v_fma);
// then (1 - d)**power (:376): 1 - d in float32, the power correctly rounded to float32.
__global__ __launch_bounds__(CM_THREADS) void costmap_cv_scale_kernel(const float* __restrict__ dist, int64_t n,
                                                                      const int32_t* __restrict__ range, int power,
                                                                      float* __restrict__ out) {
  const double smin = (double)__builtin_bit_cast(float, range[0]);
  const double smax = (double)__builtin_bit_cast(float, range[1]);
  const double scale = 1.0 * ((smax - smin > 2.220446049250313e-16) ? 1.0 / (smax - smin) : 0.0);
  const float a = (float)scale;
  const float b = 0.0f - (float)(smin * (double)a);
  for (int64_t i = (int64_t)blockIdx.x * CM_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * CM_THREADS) {
    const float dn = __builtin_fmaf(dist[i], a, b);
    const float bb = 1.0f - dn;
    out[i] = (float)pow_int_dd((double)bb, power);
  }
}

}  // namespace

hipError_t launch_costmap_build(const CostmapScratch& sc, int n_obs, int size, int power, float* out,
                                hipStream_t st, int metric) {
  const size_t cells = (size_t)size * size;
  hipError_t e = hipMemsetAsync(sc.occ, 0, cells, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(costmap_raster_kernel, dim3(n_obs > 0 ? n_obs : 1), dim3(CM_THREADS), 0, st, sc.obs, n_obs,
                     sc.xs, size, sc.occ, sc.range);
  if (metric == COSTMAP_CHAMFER5) {
    float* dist = reinterpret_cast<float*>(sc.d2);
    const size_t lds = ((size_t)3 * (size + 2 * CH_B) + 2 * CH_W) * sizeof(uint32_t);
    uint32_t* t32 = reinterpret_cast<uint32_t*>(sc.g2);
    const int per = (size + CH_T - 1) / CH_T;  // columns per thread
    if (per <= 1)
      hipLaunchKernelGGL(costmap_chamfer_kernel<1>, dim3(1), dim3(CH_T), lds, st, sc.occ, size, size, t32, dist, sc.range);
    else if (per <= 2)
      hipLaunchKernelGGL(costmap_chamfer_kernel<2>, dim3(1), dim3(CH_T), lds, st, sc.occ, size, size, t32, dist, sc.range);
    else if (per <= 4)
      hipLaunchKernelGGL(costmap_chamfer_kernel<4>, dim3(1), dim3(CH_T), lds, st, sc.occ, size, size, t32, dist, sc.range);
    else
      hipLaunchKernelGGL(costmap_chamfer_kernel<8>, dim3(1), dim3(CH_T), lds, st, sc.occ, size, size, t32, dist, sc.range);
    const unsigned blocks = (unsigned)std::min<size_t>((cells + CM_THREADS - 1) / CM_THREADS, 256 * 8);
    hipLaunchKernelGGL(costmap_cv_scale_kernel, dim3(blocks), dim3(CM_THREADS), 0, st, dist, (int64_t)cells,
                       sc.range, power, out);
    return hipGetLastError();
  }
  const int nseg = (size + COSTMAP_SEG - 1) / COSTMAP_SEG;
  const dim3 cgrid((size + CM_THREADS - 1) / CM_THREADS, nseg);
  hipLaunchKernelGGL(costmap_colseg_kernel, cgrid, dim3(CM_THREADS), 0, st, sc.occ, size, sc.first, sc.last);
  hipLaunchKernelGGL(costmap_colg_kernel, cgrid, dim3(CM_THREADS), 0, st, sc.occ, size, nseg, sc.first, sc.last,
                     sc.g2);
  hipLaunchKernelGGL(costmap_row_kernel, dim3(size), dim3(CM_THREADS), (size_t)size * sizeof(int32_t), st, sc.g2,
                     size, sc.d2, sc.range);
  const unsigned blocks = (unsigned)std::min<size_t>((cells + CM_THREADS - 1) / CM_THREADS, 256 * 8);
  hipLaunchKernelGGL(costmap_scale_kernel, dim3(blocks), dim3(CM_THREADS), 0, st, sc.d2, (int64_t)cells, sc.range,
                     power, out);
  return hipGetLastError();
}

}  // namespace mppi
