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
// Two distance metrics (oracle/costmap_ref.py):
//   chamfer (default, the reference's cv2.distanceTransform(DIST_L2, 5)): OpenCV's published
//     distanceTransform_5x5 in 16.16 fixed point, computed as 16 independent line scans (below;
//     the row-serial raster passes remain for a map without obstacle cells), then cv2.normalize
//     as OpenCV 4.x's float32 path and (1 - d)^power; parity unpinned (no cv2 here).
//   exact: the exact Euclidean distance from integer squared distances: a column
//     pass (vertical distance to the nearest obstacle, from per-segment first/last occupied rows)
//     and a row pass (min over x' of (x - x')^2 + g(x')^2, searched outwards from x only while o^2
//     can still improve the best), normalise and power in float64, one rounding to float32.
// Both are integer-exact up to the normalisation; see DESIGN.md §3.6.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "mppi_costmap.h"

namespace mppi {

namespace {

constexpr int CM_THREADS = 256;

// One workgroup per obstacle: mark the cells of its (conservative) bounding box that pass the
// reference's float64 disc test.
__global__ __launch_bounds__(CM_THREADS) void costmap_raster_kernel(const double* __restrict__ obs, int n_obs,
                                                                    const double* __restrict__ xs, int size,
                                                                    uint8_t* __restrict__ occ) {
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
    // the row's min / max in its own slot (no contended atomics; costmap_scale_kernel reduces them)
    range[2 + blockIdx.x] = mn;
    range[2 + COSTMAP_MAX_SIZE + blockIdx.x] = mx;
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

// d = sqrt(d2); dn = (d - lo) / (hi - lo) (0 when hi == lo); out = float((1 - dn)^power); lo / hi
// from the `rows` per-row partials of costmap_row_kernel.
__global__ __launch_bounds__(CM_THREADS) void costmap_scale_kernel(const int32_t* __restrict__ d2, int64_t n,
                                                                   const int32_t* __restrict__ range, int rows, int power,
                                                                   float* __restrict__ out) {
  __shared__ int red[2][CM_THREADS / 64];
  int mn = INT_MAX, mx = -1;
  for (int k = threadIdx.x; k < rows; k += CM_THREADS) {
    mn = min(mn, range[2 + k]);
    mx = max(mx, range[2 + COSTMAP_MAX_SIZE + k]);
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = mn;
    red[1][threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  for (int k = 0; k < CM_THREADS / 64; ++k) {
    mn = min(mn, red[0][k]);
    mx = max(mx, red[1][k]);
  }
  const double lo = sqrt((double)mn);
  const double hi = sqrt((double)mx);
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
// min / max partials of the chamfer map (range[2 ..]), reduced by costmap_cv_scale_kernel
constexpr int CL_PART = COSTMAP_PARTIALS;

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
                                                               int32_t* __restrict__ range, int only_if_empty) {
  extern __shared__ uint32_t srows[];  // [3][W + 4] rows, then [2][CH_W] wave totals
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // after the line scans: they already produced the map unless it has no obstacle cell (min 0)
  if (only_if_empty) {
    const int any0 = __syncthreads_or(tid < CL_PART && range[2 + tid] == 0);  // float bits of 0.0f
    if (any0) return;
  }
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
  for (int k = 1; k < CH_W; ++k) {
    dmin = fminf(dmin, red[k]);
    dmax = fmaxf(dmax, red[CH_W + k]);
  }
  // every partial slot the normalisation reduces holds the map's min / max
  if (tid < CL_PART) {
    range[2 + tid] = __builtin_bit_cast(int32_t, dmin);
    range[2 + CL_PART + tid] = __builtin_bit_cast(int32_t, dmax);
  }
}

// ------------------------------------------------- the same chamfer as independent line scans
// The two raster passes are min-plus linear in the initial map (0 on obstacles, INIT elsewhere),
// so with at least one obstacle cell their result is min over obstacle cells q of the cost of a
// cheapest path q -> p built from the 16 mask moves (the 2-pixel INIT border never wins: a real
// distance is < 2^30).  The mask's moves in angular order, axial / diagonal (even) and knight
// (odd), form a unimodular fan and the weights {65536, 91750, 143976} a convex chamfer norm, so a
// cheapest path uses only the two moves bounding its sector: n1 knight moves k then n2 moves e of
// a neighbouring axial/diagonal direction, in any order.  Hence
//   d = min over the 8 axial/diagonal e of scan_e(min(scan_k(g), scan_k'(g)))
// with k, k' the knight moves on either side of e and scan_m(h)(p) = min_n h(p - n m) + n w(m)
// (a running minimum along the lines of direction m).  Every scan is integer min / add, so the
// result is the raster passes' bit for bit (checked on random, single-cell-at-the-corner and
// 1024^2 maps against oracle/costmap_ref.py chamfer_l2_5x5 and by the GPU costmap tests), and
// every line of a scan is independent (below: 64 lines per workgroup, each split into 32-step
// segments over the waves and stitched by the carry).  Two launches of
// 8 scans each (knight scans of the occupancy, then the axial/diagonal scans of their pairwise
// minima) replace 2 x H serial rows on one workgroup.  A map without any obstacle cell (all
// distances measured from the INIT border) keeps the raster kernel above, which then runs alone.
constexpr uint32_t CL_INF = 1u << 30;  // "no obstacle yet"; real distances < 1.4 * 8192 * 65536 < 2^30
constexpr int CL_L = 32;               // steps per wave segment
constexpr int CL_SEGS = 8;             // segments (waves) per workgroup: 256-step chunks, 2 workgroups per CU
constexpr int CL_T = 64 * CL_SEGS;

struct ClScan {
  int8_t ax, ay;      // direction in the virtual frame (ax, ay >= 0; (1,0) (0,1) (1,1) (2,1) (1,2))
  int8_t fx, fy;      // virtual -> physical mirror of x / y
  uint32_t w;         // move weight
  int32_t in_a, in_b; // phase 2: the two knight scans whose minimum is scanned (buffer indices)
  int32_t nlines;     // lines of this scan
};
struct ClJobs {
  ClScan s[8];
};

// Lines of direction (ax, ay) in an H x W map: ay == 0 -> the H rows; otherwise lines (u, phi),
// phi in [0, ay), points (u + ax n, phi + ay n), n in [0, N_phi), N_phi = ceil((H - phi) / ay),
// u in [-ax (N_phi - 1), W - 1] so that some point lies inside.
__host__ __device__ inline int cl_nsteps(int H, int ay, int phi) { return (H - phi + ay - 1) / ay; }
__host__ __device__ inline int cl_lines_phi(int H, int W, int ax, int ay, int phi) {
  return W + ax * (cl_nsteps(H, ay, phi) - 1);
}
inline int cl_lines(int H, int W, int ax, int ay) {
  if (ay == 0) return H;
  int n = 0;
  for (int phi = 0; phi < ay; ++phi) n += cl_lines_phi(H, W, ax, ay, phi);
  return n;
}

// PHASE 1: h = occ ? 0 : INF, out = buf[job].  PHASE 2: h = min(buf[in_a], buf[in_b], INF), out =
// buf[8 + job].  buf holds 16 planes of H x W words.
//
// One workgroup scans 64 consecutive lines (a wave's lanes, so every step of a wave reads one
// contiguous run of a row) in chunks of CL_SEGS * CL_L steps; wave s takes steps [s CL_L, (s+1) CL_L)
// of the chunk: all its loads issued at once, the running minimum over its segment with no input
// (carry INF), the segment's last value to LDS, then the value entering the segment,
//   C_0 = the chunk's carry, C_{s+1} = min(T_s, C_s + CL_L w)
// (T_s the last local value of segment s), and v = min(local, C_seg + (k+1) w), which is the
// serial recurrence's value exactly (integer min / add are associative).  Cells outside the map
// read INF and are not stored; every value stays <= INF, so no sum overflows.
__device__ inline __amdgpu_buffer_rsrc_t cl_rsrc(const void* p, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// Horizontal scans (virtual (1, 0)): one wave per row, lane l holding 16 consecutive columns of a
// 1024-column chunk (the row is contiguous, so lanes read it in order); the in-lane chain runs
// serially and the chain across lanes as an exclusive min-scan of keys (value at the lane's last
// column + (W - that column) w: a later column p then reads key - (W - p) w; keys < 2^32 as
// INF + (W + 1) w < 1.9e9).  Backward (fx) mirrors it: right to left, keys v + column w.
template <bool BACK>
__device__ inline void cl_row_scan(__amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, __amdgpu_buffer_rsrc_t ro,
                                   int y, int W, uint32_t w, int lane) {
  constexpr int C = 16;
  uint32_t carry = CL_INF;  // value at the column just before (after, BACK) the chunk
  const int nch = (W + 64 * C - 1) / (64 * C);
  for (int q = 0; q < nch; ++q) {
    const int cb = (BACK ? nch - 1 - q : q) * 64 * C;
    const int j0 = cb + lane * C;
    uint32_t v[C];
#pragma unroll
    for (int k = 0; k < C; ++k) {
      const int j = j0 + k;
      const int off = (y * W + j) * 4;
      v[k] = j < W ? min(min(__builtin_amdgcn_raw_buffer_load_b32(ra, off, 0, 0),
                             __builtin_amdgcn_raw_buffer_load_b32(rb, off, 0, 0)), CL_INF)
                   : CL_INF;
    }
    uint32_t run = CL_INF;
    if (!BACK) {
#pragma unroll
      for (int k = 0; k < C; ++k) {
        run = min(v[k], run + w);
        v[k] = run;
      }
      // (a lane whose chunk passes column W - 1 may wrap its key; only later lanes, all past the
      // map and never stored, read it)
      const uint32_t key = run + (uint32_t)(W - (j0 + C - 1)) * w;
      const uint32_t kin = carry + (uint32_t)(W - (cb - 1)) * w;
      const uint32_t kc = min(wave_excl_min_scan_up(key), kin);
#pragma unroll
      for (int k = 0; k < C; ++k) {
        const int j = j0 + k;
        v[k] = min(v[k], kc - (uint32_t)(W - j) * w);
        if (j < W) __builtin_amdgcn_raw_buffer_store_b32(v[k], ro, (y * W + j) * 4, 0, 0);
      }
      carry = (uint32_t)__builtin_amdgcn_readlane((int)v[C - 1], 63);
    } else {
#pragma unroll
      for (int k = C - 1; k >= 0; --k) {
        run = min(v[k], run + w);
        v[k] = run;
      }
      const uint32_t key = run + (uint32_t)j0 * w;
      const uint32_t kin = carry + (uint32_t)(cb + 64 * C) * w;
      const uint32_t kc = min(wave_excl_min_scan_down(key, lane), kin);
#pragma unroll
      for (int k = 0; k < C; ++k) {
        const int j = j0 + k;
        v[k] = min(v[k], kc - (uint32_t)j * w);
        if (j < W) __builtin_amdgcn_raw_buffer_store_b32(v[k], ro, (y * W + j) * 4, 0, 0);
      }
      carry = (uint32_t)__builtin_amdgcn_readlane((int)v[0], 0);
    }
  }
}

template <int PHASE>
__global__ __launch_bounds__(CL_T, 4) void costmap_line_scan_kernel(const uint8_t* __restrict__ occ, int H, int W,
                                                                 uint32_t* __restrict__ buf, ClJobs jobs) {
  __shared__ uint32_t tails[CL_SEGS][64];
  const ClScan sc = jobs.s[blockIdx.y];
  const int lane = threadIdx.x & 63, seg = threadIdx.x >> 6;
  const size_t plane = (size_t)H * W;
  const auto ro = cl_rsrc(buf + (size_t)(PHASE == 1 ? blockIdx.y : 8 + blockIdx.y) * plane, plane * 4);
  const auto ra = cl_rsrc(buf + (size_t)sc.in_a * plane, plane * 4);
  const auto rb = cl_rsrc(buf + (size_t)sc.in_b * plane, plane * 4);
  const auto rocc = cl_rsrc(occ, plane);
  const int ax = sc.ax, ay = sc.ay;
  if (ay == 0) {  // rows (PHASE 2 only): one wave per row
    const int y = blockIdx.x * CL_SEGS + seg;
    if (y >= H) return;
    if (sc.fx)
      cl_row_scan<true>(ra, rb, ro, y, W, sc.w, lane);
    else
      cl_row_scan<false>(ra, rb, ro, y, W, sc.w, lane);
    return;
  }
  const int line0 = blockIdx.x * 64;
  if (line0 >= sc.nlines) return;  // uniform over the workgroup
  const int t = line0 + lane;
  // this lane's line: start (x0, y0) in the virtual frame, step (ax, ay), valid n in [nlo, nhi]
  int x0, y0, nlo, nhi;
  auto line_of = [&](int tt, int& lx0, int& ly0, int& lo, int& hi) {
    int phi = 0, u = tt;
    const int l0 = cl_lines_phi(H, W, ax, ay, 0);
    if (ay == 2 && u >= l0) {
      phi = 1;
      u -= l0;
    }
    const int N = cl_nsteps(H, ay, phi);
    u -= ax * (N - 1);  // u in [-ax (N - 1), W - 1]
    lx0 = u;
    ly0 = phi;
    lo = 0;
    hi = N - 1;
    if (ax > 0) {
      if (u < 0) lo = (-u + ax - 1) / ax;  // first n with u + ax n >= 0
      hi = min(N - 1, (W - 1 - u) / ax);   // last n with u + ax n <= W - 1 (W - 1 - u >= 0)
    }
  };
  const bool live = t < sc.nlines;
  line_of(live ? t : line0, x0, y0, nlo, nhi);
  if (!live) {
    nlo = 0;
    nhi = -1;
  }
  // step range of the 64 lines (the same in every wave of the workgroup)
  int wlo = live ? nlo : INT_MAX, whi = live ? nhi : -1;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    wlo = min(wlo, __shfl_xor(wlo, o, 64));
    whi = max(whi, __shfl_xor(whi, o, 64));
  }
  // physical cell of step n: x' = x0 + ax n, y' = y0 + ay n, mirrored; 32-bit cell index (< 2^26)
  const int sx = sc.fx ? -ax : ax, sy = sc.fy ? -ay : ay;
  const int px0 = sc.fx ? W - 1 - x0 : x0, py0 = sc.fy ? H - 1 - y0 : y0;
  const int ibase = py0 * W + px0;
  const int istep = sy * W + sx;
  const uint32_t w = sc.w, wl = (uint32_t)CL_L * sc.w;
  uint32_t carry = CL_INF;  // the value at the step before the chunk
  for (int c0 = wlo; c0 <= whi; c0 += CL_SEGS * CL_L) {
    const int n0 = c0 + seg * CL_L;
    uint32_t v[CL_L];
#pragma unroll
    for (int k = 0; k < CL_L; ++k) {
      const int nn = n0 + k;
      const bool in = nn >= nlo && nn <= nhi;
      const int idx = ibase + istep * nn;
      if (PHASE == 1) {
        v[k] = in ? (__builtin_amdgcn_raw_buffer_load_b8(rocc, idx, 0, 0) ? 0u : CL_INF) : CL_INF;
      } else {
        v[k] = in ? min(min(__builtin_amdgcn_raw_buffer_load_b32(ra, idx * 4, 0, 0),
                            __builtin_amdgcn_raw_buffer_load_b32(rb, idx * 4, 0, 0)), CL_INF)
                  : CL_INF;
      }
    }
    uint32_t run = CL_INF;
#pragma unroll
    for (int k = 0; k < CL_L; ++k) {
      run = min(v[k], run + w);
      v[k] = run;
    }
    tails[seg][lane] = run;
    __syncthreads();
    uint32_t cin = carry, cout = carry;
#pragma unroll
    for (int s = 0; s < CL_SEGS; ++s) {
      if (s == seg) cin = cout;
      cout = min(tails[s][lane], cout + wl);
    }
    __syncthreads();  // tails read before the next chunk writes them
#pragma unroll
    for (int k = 0; k < CL_L; ++k) {
      const int nn = n0 + k;
      if (nn >= nlo && nn <= nhi)
        __builtin_amdgcn_raw_buffer_store_b32(min(v[k], cin + (uint32_t)(k + 1) * w), ro, (ibase + istep * nn) * 4, 0, 0);
    }
    carry = cout;
  }
}

// dist = float(min over the 8 axial/diagonal scans) / 65536; workgroup b (of exactly CL_PART)
// stores its min / max (float bits) in range[2 + b] / range[2 + CL_PART + b].
__global__ __launch_bounds__(CM_THREADS) void costmap_line_min_kernel(const uint32_t* __restrict__ buf, int64_t n,
                                                                      float* __restrict__ dist,
                                                                      int32_t* __restrict__ range) {
  __shared__ float red[2][CM_THREADS / 64];
  const uint32_t* r = buf + 8 * n;
  float dmin = INFINITY, dmax = -INFINITY;
  auto one = [&](uint32_t v, int64_t i) __attribute__((always_inline)) {
    const float d = (float)v * (1.0f / 65536.0f);
    dist[i] = d;
    dmin = fminf(dmin, d);
    dmax = fmaxf(dmax, d);
  };
  const int64_t gsz = (int64_t)gridDim.x * CM_THREADS, tid = (int64_t)blockIdx.x * CM_THREADS + threadIdx.x;
  if ((n & 3) == 0) {  // planes 16-byte aligned: four cells per load
    const int64_t n4 = n >> 2;
    for (int64_t i = tid; i < n4; i += gsz) {
      uint4 v = reinterpret_cast<const uint4*>(r)[i];
#pragma unroll
      for (int k = 1; k < 8; ++k) {
        const uint4 u = reinterpret_cast<const uint4*>(r + k * n)[i];
        v.x = min(v.x, u.x);
        v.y = min(v.y, u.y);
        v.z = min(v.z, u.z);
        v.w = min(v.w, u.w);
      }
      one(v.x, 4 * i);
      one(v.y, 4 * i + 1);
      one(v.z, 4 * i + 2);
      one(v.w, 4 * i + 3);
    }
  } else {
    for (int64_t i = tid; i < n; i += gsz) {
      uint32_t v = r[i];
#pragma unroll
      for (int k = 1; k < 8; ++k) v = min(v, r[k * n + i]);
      one(v, i);
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    dmin = fminf(dmin, __shfl_xor(dmin, o, 64));
    dmax = fmaxf(dmax, __shfl_xor(dmax, o, 64));
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wv] = dmin;
    red[1][wv] = dmax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < CM_THREADS / 64; ++k) {
      dmin = fminf(dmin, red[0][k]);
      dmax = fmaxf(dmax, red[1][k]);
    }
    range[2 + blockIdx.x] = __builtin_bit_cast(int32_t, dmin);  // no contended atomics: one slot per workgroup
    range[2 + CL_PART + blockIdx.x] = __builtin_bit_cast(int32_t, dmax);
  }
}

// cv2.normalize(NORM_MINMAX, 0, 1) (:375) as OpenCV 4.x's cv::normalize / convertTo write it for a
// CV_32F destination: scale = 1 / (smax - smin) (0 if smax - smin <= DBL_EPSILON) rounded to
// float, shift = -(float)(smin * scale), dst = fma(src, scale, shift) in float32 (cvt_32f's v_fma);
// then (1 - d)**power (:376): 1 - d in float32, the power correctly rounded to float32.
__global__ __launch_bounds__(CM_THREADS) void costmap_cv_scale_kernel(const float* __restrict__ dist, int64_t n,
                                                                      const int32_t* __restrict__ range, int power,
                                                                      float* __restrict__ out) {
  __shared__ float red[2][CM_THREADS / 64];
  float pmin = INFINITY, pmax = -INFINITY;  // the CL_PART partials (chamfer line / raster kernels)
  for (int k = threadIdx.x; k < CL_PART; k += CM_THREADS) {
    pmin = fminf(pmin, __builtin_bit_cast(float, range[2 + k]));
    pmax = fmaxf(pmax, __builtin_bit_cast(float, range[2 + CL_PART + k]));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    pmin = fminf(pmin, __shfl_xor(pmin, o, 64));
    pmax = fmaxf(pmax, __shfl_xor(pmax, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = pmin;
    red[1][threadIdx.x >> 6] = pmax;
  }
  __syncthreads();
  for (int k = 0; k < CM_THREADS / 64; ++k) {
    pmin = fminf(pmin, red[0][k]);
    pmax = fmaxf(pmax, red[1][k]);
  }
  const double smin = (double)pmin;
  const double smax = (double)pmax;
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
                     sc.xs, size, sc.occ);
  if (metric == COSTMAP_CHAMFER5 || metric == COSTMAP_CHAMFER5_RASTER) {
    float* dist = reinterpret_cast<float*>(sc.d2);
    const int lines = metric == COSTMAP_CHAMFER5;
    if (lines) {
      // phase 1: the 8 knight scans of the occupancy -> planes 0..7
      const int H = size, W = size;
      ClJobs j1{}, j2{};
      const int kn[8][2] = {{2, 1}, {-2, 1}, {2, -1}, {-2, -1}, {1, 2}, {-1, 2}, {1, -2}, {-1, -2}};
      auto knight = [&](int mx, int my) {
        for (int k = 0; k < 8; ++k)
          if (kn[k][0] == mx && kn[k][1] == my) return k;
        return -1;
      };
      auto fill = [&](ClScan& s, int mx, int my, uint32_t w) {
        s.ax = (int8_t)std::abs(mx);
        s.ay = (int8_t)std::abs(my);
        s.fx = (int8_t)(mx < 0);
        s.fy = (int8_t)(my < 0);
        s.w = w;
        s.nlines = cl_lines(H, W, s.ax, s.ay);
      };
      int most = 0;
      for (int k = 0; k < 8; ++k) {
        fill(j1.s[k], kn[k][0], kn[k][1], CV_LONG);
        most = std::max(most, j1.s[k].nlines);
      }
      hipLaunchKernelGGL(costmap_line_scan_kernel<1>, dim3((most + 63) / 64, 8), dim3(CL_T), 0, st, sc.occ,
                         H, W, sc.lines, j1);
      // phase 2: each axial / diagonal direction e scans min of the knight scans on either side
      const int ad[8][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}, {-1, 0}, {-1, -1}, {0, -1}, {1, -1}};
      most = 0;
      for (int k = 0; k < 8; ++k) {
        const int mx = ad[k][0], my = ad[k][1];
        fill(j2.s[k], mx, my, (mx != 0 && my != 0) ? CV_DIAG : CV_HV);
        // the two knight moves angularly adjacent to e (the sectors on either side of e)
        int a, b;
        if (my == 0) {
          a = knight(2 * mx, 1);
          b = knight(2 * mx, -1);
        } else if (mx == 0) {
          a = knight(1, 2 * my);
          b = knight(-1, 2 * my);
        } else {
          a = knight(2 * mx, my);
          b = knight(mx, 2 * my);
        }
        j2.s[k].in_a = a;
        j2.s[k].in_b = b;
        most = std::max(most, my == 0 ? (H + CL_SEGS - 1) / CL_SEGS * 64 : j2.s[k].nlines);
      }
      hipLaunchKernelGGL(costmap_line_scan_kernel<2>, dim3((most + 63) / 64, 8), dim3(CL_T), 0, st, sc.occ,
                         H, W, sc.lines, j2);
      hipLaunchKernelGGL(costmap_line_min_kernel, dim3(CL_PART), dim3(CM_THREADS), 0, st, sc.lines, (int64_t)cells,
                         dist, sc.range);
    }
    const size_t lds = ((size_t)3 * (size + 2 * CH_B) + 2 * CH_W) * sizeof(uint32_t);
    uint32_t* t32 = reinterpret_cast<uint32_t*>(sc.g2);
    const int per = (size + CH_T - 1) / CH_T;  // columns per thread
    if (per <= 1)
      hipLaunchKernelGGL(costmap_chamfer_kernel<1>, dim3(1), dim3(CH_T), lds, st, sc.occ, size, size, t32, dist, sc.range,
                         lines);
    else if (per <= 2)
      hipLaunchKernelGGL(costmap_chamfer_kernel<2>, dim3(1), dim3(CH_T), lds, st, sc.occ, size, size, t32, dist, sc.range,
                         lines);
    else if (per <= 4)
      hipLaunchKernelGGL(costmap_chamfer_kernel<4>, dim3(1), dim3(CH_T), lds, st, sc.occ, size, size, t32, dist, sc.range,
                         lines);
    else
      hipLaunchKernelGGL(costmap_chamfer_kernel<8>, dim3(1), dim3(CH_T), lds, st, sc.occ, size, size, t32, dist, sc.range,
                         lines);
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
                     size, power, out);
  return hipGetLastError();
}

}  // namespace mppi
