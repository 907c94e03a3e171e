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

}  // namespace

hipError_t launch_costmap_build(const CostmapScratch& sc, int n_obs, int size, int power, float* out,
                                hipStream_t st) {
  const size_t cells = (size_t)size * size;
  hipError_t e = hipMemsetAsync(sc.occ, 0, cells, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(costmap_raster_kernel, dim3(n_obs > 0 ? n_obs : 1), dim3(CM_THREADS), 0, st, sc.obs, n_obs,
                     sc.xs, size, sc.occ, sc.range);
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
