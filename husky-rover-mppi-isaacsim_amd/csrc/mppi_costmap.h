// On-device obstacle costmap builder:
// Surface.create_obstacles_costmap, thesis_master/warp_implementation/MPPI_isaac.py:361-378.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mppi {

// Device scratch for one build of a size x size costmap (grown on demand by the caller).
struct CostmapScratch {
  uint8_t* occ = nullptr;    // [size*size] 1 = inside an inflated obstacle disc
  int32_t* first = nullptr;  // [segments*size] first occupied row of each column segment (-1: none)
  int32_t* last = nullptr;   // [segments*size] last occupied row of each column segment (-1: none)
  int32_t* g2 = nullptr;     // [size*size] squared vertical distance to the nearest obstacle (column pass)
  int32_t* d2 = nullptr;     // [size*size] squared Euclidean distance (row pass)
  int32_t* range = nullptr;  // [2] min / max of d2 (exact), then [2][COSTMAP_PARTIALS] chamfer min / max partials
  uint32_t* lines = nullptr; // [16*size*size] chamfer line scans: 8 knight planes, 8 axial/diagonal planes
  double* obs = nullptr;     // [n*3] (x_local, y_local, total_radius) per obstacle
  double* xs = nullptr;      // [size] np.linspace(-hw, hw, size)
  size_t cells_cap = 0, obs_cap = 0, xs_cap = 0;
};

constexpr int COSTMAP_PARTIALS = 1024;  // = CL_PART in mppi_costmap.hip
constexpr int COSTMAP_SEG = 32;         // rows per column segment of the column pass
constexpr int COSTMAP_MAX_SIZE = 8192;  // (2*size+1)^2 must fit int32 (the no-obstacle marker)

// distance metric of the build
constexpr int COSTMAP_CHAMFER5 = 0;  // cv2.distanceTransform(DIST_L2, 5), the reference (default)
constexpr int COSTMAP_EXACT = 1;     // exact Euclidean distance
constexpr int COSTMAP_CHAMFER5_RASTER = 2;  // the chamfer by the row-serial raster kernel (same result)

// Enqueue the whole build on `st`: raster -> distance (chamfer: 16 independent line scans, or the
// two raster passes on one workgroup for a map without obstacle cells / COSTMAP_CHAMFER5_RASTER;
// exact: column pass, row pass) -> min/max -> min-max normalise -> (1 - d)^power, written to
// out[size*size] (device, float32, row-major).  sc.obs / sc.xs must already hold the n obstacle
// triples and the size grid coordinates.
hipError_t launch_costmap_build(const CostmapScratch& sc, int n_obs, int size, int power, float* out,
                                hipStream_t st, int metric);

}  // namespace mppi
