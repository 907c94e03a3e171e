// Calibration of rocprofv3's WRITE_SIZE for the store widths the engine uses (MI355X_MICROARCH.md:
// only 16 B/lane streaming stores are calibrated).  Each kernel writes exactly 64 MiB once per launch.
//   st4      4 B/lane plain stores, one contiguous 256 B run per wave instruction
//   st4_wt   4 B/lane agent-scope relaxed atomic stores (sc1 write-through: mppi noise_store)
//   st16     16 B/lane float4 stores
//   noise    mppi noise_store's pattern: 4 write-through 4 B/lane stores to 4 rows 1 KB apart... of
//            [blk][2][H][256] rows (H = 100), 64 MiB of rows in total
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr size_t N = (64u << 20) / 4;  // floats
__global__ void st4(float* p) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < N; i += (size_t)gridDim.x * 256) p[i] = 1.0f;
}
__global__ void st4_wt(float* p) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < N; i += (size_t)gridDim.x * 256)
    __hip_atomic_store(p + i, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void st16(float4* p) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < N / 4; i += (size_t)gridDim.x * 256) p[i] = make_float4(1, 1, 1, 1);
}
__global__ void noise(float* eps, int blocks) {  // unit g = (block g / 50, Philox block g % 50), 256 trajectories
  const int H = 100, NB = 50;
  for (int g = blockIdx.x; g < blocks * NB; g += gridDim.x) {
    const int blk = g / NB, n = g % NB, t = 2 * n, tj = threadIdx.x;
    float* e1 = eps + ((size_t)blk * 2 * H + t) * 256 + tj;
    float* e2 = e1 + (size_t)H * 256;
    __hip_atomic_store(e1, 1.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(e2, 2.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(e1 + 256, 3.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(e2 + 256, 4.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
int main() {
  float* p = nullptr;
  if (hipMalloc(&p, N * 4) != hipSuccess) return 1;
  const int blocks = (int)(N / (2 * 100 * 256));  // 327 blocks of rows = 64 MiB (minus a remainder)
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(st4, dim3(2048), dim3(256), 0, 0, p);
    hipLaunchKernelGGL(st4_wt, dim3(2048), dim3(256), 0, 0, p);
    hipLaunchKernelGGL(st16, dim3(2048), dim3(256), 0, 0, (float4*)p);
    hipLaunchKernelGGL(noise, dim3(1024), dim3(256), 0, 0, p, blocks);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("wcal: 64 MiB per st4/st4_wt/st16 launch; noise %zu bytes per launch\n", (size_t)blocks * 2 * 100 * 256 * 4);
  return 0;
}
