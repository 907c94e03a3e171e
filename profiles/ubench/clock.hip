// Diagnostic (not product): in-kernel shader clock = d(s_memtime) / d(s_memrealtime) * 100 MHz
// for a dependent-ALU loop at different grid sizes (waves per SIMD), after a sustained warmup.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void spin(int iters, float* sink, unsigned long long* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float x = threadIdx.x * 1e-3f, y = 1.0001f;
  for (int i = 0; i < iters; ++i) {
    x = x * y + 0.5f;
    y = y * 0.99999f + 1e-6f;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (x == 12345.f) sink[0] = x + y;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = r1 - r0;
  }
}

int main() {
  float* sink;
  unsigned long long* out;
  hipMalloc(&sink, 4);
  hipMalloc(&out, 16);
  int grids[] = {256, 1024, 2048, 4096, 8192};
  for (int g : grids) {
    for (int rep = 0; rep < 20; ++rep) hipLaunchKernelGGL(spin, dim3(g), dim3(256), 0, 0, 200000, sink, out);
    hipDeviceSynchronize();
    unsigned long long h[2];
    hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
    printf("grid %5d x 256 (%.1f waves/SIMD): %llu cyc / %llu ticks -> %.2f GHz\n", g,
           g * 4.0 / 1024.0, h[0], h[1], (double)h[0] / (double)h[1] * 0.1);
  }
  return 0;
}
