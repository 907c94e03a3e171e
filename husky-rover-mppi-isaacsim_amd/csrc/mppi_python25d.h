// Reference-integrator mode "python25d" (debug.py:312-364), see mppi_python25d.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mppi {

struct P25Args {
  const float* Z;     // DEM [rows][cols], row j at y = linspace(-hw, hw, rows)[j] (ascending)
  int rows, cols;
  double hw, res;     // half width; `resolution` = 2 hw / grid (floor / bilinear step)
  double xstep, ystep;  // linspace spacings 2 hw / (cols - 1), 2 hw / (rows - 1)
  double dt, bound;
  int64_t n;          // trajectories
  int H;
  const double *x0, *y0, *hd;  // [n], [n], [n][3]
  const double *v, *w;         // [n][H] trajectory-major
  double* traj;                // [n][H][3]
  int32_t* valid;              // [n]
};

hipError_t launch_python25d(const P25Args& a, hipStream_t st);

}  // namespace mppi
