// Reference-integrator mode "python25d" (SURVEY.md §8(f)4): the numpy 2.5D integrator of
// thesis_master/python_mppi_projection/debug.py:170-364 (generate_trajectory_25D), batched one
// trajectory per lane, in float64 like numpy.  It differs from the Warp rollout the MPPI step
// uses (projection_warp.py:284-350) in ordering (the heading is rotated about the previous
// normal before the lookup), indexing (searchsorted on the linspace grid, rows ascending in y)
// and rounding (floor, not trunc); it exists so whole trajectories can be compared with the
// reference's own numpy function.  Not on the MPPI step path.
#include "mppi_python25d.h"

namespace mppi {

namespace {

// np.linspace(-hw, hw, n)[k]: k*step + start, the last element = stop.
__device__ inline double grid_at(int k, int n, double start, double stop, double step) {
  return k == n - 1 ? stop : (double)k * step + start;
}

// np.searchsorted(grid, v) (side='left'): the number of grid values < v.
__device__ inline int searchsorted(double v, int n, double start, double stop, double step) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (grid_at(mid, n, start, stop, step) < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

struct Quad {
  double q00, q01, q10, q11;
};

// find_corners_heights (debug.py:186-198); i, j clamped to [0, n-2] (DEFINED, the reference
// raises IndexError there).
__device__ inline Quad corners(const P25Args& a, double x, double y) {
  const double x0 = floor(x / a.res) * a.res;
  const double y0 = floor(y / a.res) * a.res;
  int i = searchsorted(x0, a.cols, -a.hw, a.hw, a.xstep);
  int j = searchsorted(y0, a.rows, -a.hw, a.hw, a.ystep);
  i = min(max(i, 0), a.cols - 2);
  j = min(max(j, 0), a.rows - 2);
  const float* r0 = a.Z + (size_t)j * a.cols + i;
  const float* r1 = r0 + a.cols;
  return Quad{(double)r0[0], (double)r0[1], (double)r1[0], (double)r1[1]};
}

// bilinear_interpolator (debug.py:246-257)
__device__ inline double bilinear(double x, double y, const Quad& q, double res) {
  const double xn = x / res, yn = y / res;
  const double x2 = xn - floor(xn), y2 = yn - floor(yn);
  return (1.0 - x2) * (1.0 - y2) * q.q00 + x2 * (1.0 - y2) * q.q10 + (1.0 - x2) * y2 * q.q01 + x2 * y2 * q.q11;
}

__device__ inline double norm3(double x, double y, double z) { return sqrt(x * x + y * y + z * z); }

// normal_on_grid (debug.py:211-216)
__device__ inline void normal(const Quad& q, double g, double& nx, double& ny, double& nz) {
  const double vx = -g / 2.0 * (q.q01 - q.q00 - q.q10 + q.q11);
  const double vy = -g / 2.0 * (q.q10 - q.q00 - q.q01 + q.q11);
  const double vz = g * g;
  const double l = norm3(vx, vy, vz);
  nx = vx / l;
  ny = vy / l;
  nz = vz / l;
}

// get_heading_tangent_vector (debug.py:230-232)
__device__ inline void tangent(double nx, double ny, double nz, double& hx, double& hy, double& hz) {
  const double d = hx * nx + hy * ny + hz * nz;
  const double px = hx - d * nx, py = hy - d * ny, pz = hz - d * nz;
  const double l = norm3(px, py, pz);
  hx = px / l;
  hy = py / l;
  hz = pz / l;
}

// scipy Rotation.from_rotvec(rv).apply(v) (debug.py:286-287): quaternion with the small-angle
// Taylor scale below 1e-3 rad, rotation matrix, M v.
__device__ inline void rotvec_apply(double rx, double ry, double rz, double& vx, double& vy, double& vz) {
  const double ang = norm3(rx, ry, rz);
  const double a2 = ang * ang;
  const double scale = ang <= 1e-3 ? 0.5 - a2 / 48 + a2 * a2 / 3840 : sin(ang / 2) / ang;
  const double x = scale * rx, y = scale * ry, z = scale * rz, w = cos(ang / 2);
  const double x2 = x * x, y2 = y * y, z2 = z * z, w2 = w * w;
  const double xy = x * y, zw = z * w, xz = x * z, yw = y * w, yz = y * z, xw = x * w;
  const double m00 = x2 - y2 - z2 + w2, m01 = 2 * (xy - zw), m02 = 2 * (xz + yw);
  const double m10 = 2 * (xy + zw), m11 = -x2 + y2 - z2 + w2, m12 = 2 * (yz - xw);
  const double m20 = 2 * (xz - yw), m21 = 2 * (yz + xw), m22 = -x2 - y2 + z2 + w2;
  const double ox = m00 * vx + m01 * vy + m02 * vz;
  const double oy = m10 * vx + m11 * vy + m12 * vz;
  const double oz = m20 * vx + m21 * vy + m22 * vz;
  vx = ox;
  vy = oy;
  vz = oz;
}

__global__ __launch_bounds__(256) void mppi_python25d_kernel(P25Args a) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.n) return;
  double x = a.x0[k], y = a.y0[k];
  double hx = a.hd[3 * k], hy = a.hd[3 * k + 1], hz = a.hd[3 * k + 2];
  double nx, ny, nz;
  Quad q = corners(a, x, y);  // generate_trajectory_25D initial conditions :341-344
  normal(q, a.res, nx, ny, nz);
  tangent(nx, ny, nz, hx, hy, hz);
  const double* vk = a.v + (size_t)k * a.H;
  const double* wk = a.w + (size_t)k * a.H;
  double* out = a.traj + (size_t)k * a.H * 3;
  int valid = 1;
  for (int t = 0; t < a.H; ++t) {
    // update_position (debug.py:278-290) about the previous normal
    double l = norm3(hx, hy, hz);
    hx /= l;
    hy /= l;
    hz /= l;
    x = x + hx * vk[t] * a.dt;
    y = y + hy * vk[t] * a.dt;
    const double ang = wk[t] * a.dt;
    rotvec_apply(ang * nx, ang * ny, ang * nz, hx, hy, hz);
    l = norm3(hx, hy, hz);
    hx /= l;
    hy /= l;
    hz /= l;
    // lookup at the new position (:354-357)
    q = corners(a, x, y);
    const double height = bilinear(x, y, q, a.res);
    normal(q, a.res, nx, ny, nz);
    tangent(nx, ny, nz, hx, hy, hz);
    if (x >= a.bound || x <= -a.bound || y >= a.bound || y <= -a.bound) {  // :359-360
      valid = 0;
      for (int s = t; s < a.H; ++s) out[3 * s] = out[3 * s + 1] = out[3 * s + 2] = 0.0;
      break;
    }
    out[3 * t] = x;
    out[3 * t + 1] = y;
    out[3 * t + 2] = height;
  }
  a.valid[k] = valid;
}

}  // namespace

hipError_t launch_python25d(const P25Args& a, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((a.n + 255) / 256);
  hipLaunchKernelGGL(mppi_python25d_kernel, dim3(blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace mppi
