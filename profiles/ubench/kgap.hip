// Diagnostic microbenchmark (not part of the product): the gap between two dependent kernels on
// one stream (B starts after A ends), read from rocprofv3 --kernel-trace, with nothing, an event
// record, or an event another stream waits on between them, and with A storing to pinned memory.
// Build: hipcc --offload-arch=gfx950 -O3 kgap.hip -o kgap
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void ka(float* p, unsigned* host, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    p[0] += 1.0f;
    if (host) __hip_atomic_store(host, (unsigned)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
__global__ void kb(float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[1] += 1.0f;
}
__global__ void kc(float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[2] += 1.0f;
}

int main() {
  float* d;
  unsigned* h;
  hipMalloc(&d, 64);
  hipHostMalloc(&h, 64, hipHostMallocDefault);
  hipStream_t s, s2;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e;
  hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (int mode = 0; mode < 4; ++mode) {
    for (int i = 0; i < 200; ++i) {
      // A (256 workgroups, like a finish) then B; mode 1: event record between; mode 2: + another
      // stream waits on it and runs C; mode 3: A stores to pinned memory
      hipLaunchKernelGGL(ka, dim3(256), dim3(256), 0, s, d, mode == 3 ? h : nullptr, i);
      if (mode == 1 || mode == 2) hipEventRecord(e, s);
      if (mode == 2) {
        hipStreamWaitEvent(s2, e, 0);
        hipLaunchKernelGGL(kc, dim3(1), dim3(64), 0, s2, d);
      }
      hipLaunchKernelGGL(kb, dim3(256), dim3(256), 0, s, d);
    }
    hipDeviceSynchronize();
    // mark the end of a mode with a distinct kernel
    hipLaunchKernelGGL(kc, dim3(1), dim3(64), 0, s, d);
    hipDeviceSynchronize();
  }
  printf("done\n");
  return 0;
}
