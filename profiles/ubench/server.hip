// Diagnostic microbenchmark (not part of the product): per-step overhead of a host-driven step
// loop, one launch per step vs one resident (persistent) kernel that polls a go word in pinned host
// memory.  Each "step" is 256 workgroups x 1024 threads (150 KB LDS each: one per CU, as the
// role-split rollout) that spin W us, then take a ticket; the last one stores `done` (pinned).
// Build: hipcc --offload-arch=gfx950 -O3 server.hip -o server ; run: ./server [W_us] [steps]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

struct Box {
  unsigned go;
  unsigned stop;
  unsigned pad[14];
  float state[16];
};

__device__ __forceinline__ void spin_us(unsigned us) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)us * 100) __builtin_amdgcn_s_sleep(4);
}

__device__ __forceinline__ void ticket_done(unsigned* cnt, unsigned* done, unsigned seq, unsigned nwg) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == nwg - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ __launch_bounds__(1024) void k_step(unsigned* cnt, unsigned* done, unsigned seq, unsigned w_us,
                                               float* sink) {
  extern __shared__ float lds[];
  lds[threadIdx.x] = (float)seq;
  spin_us(w_us);
  if (threadIdx.x == 0 && lds[5] < 0.f) sink[0] = lds[7];
  ticket_done(cnt, done, seq, gridDim.x);
}

// resident: poll box->go, run the step, repeat; exits on stop or 200 ms idle.  poll: 0 every
// workgroup polls host memory back to back, 1 with s_sleep(1), 2 with s_sleep(8), 3 workgroup 0
// relays (it polls host memory and stores a device word every other workgroup polls), 4 every
// workgroup polls host memory with s_sleep(127)
__global__ __launch_bounds__(1024) void k_server(const Box* box, unsigned* cnt, unsigned* done, unsigned w_us,
                                                 float* sink, int poll, unsigned first, unsigned* relay) {
  extern __shared__ float lds[];
  __shared__ unsigned cmd;
  unsigned expect = first;
  for (;;) {
    if (threadIdx.x == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      unsigned v;
      const bool host = poll != 3 || blockIdx.x == 0;
      for (;;) {
        if (host) {
          const unsigned long long w = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(box),
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          v = (unsigned)w;
          if ((int)(v - expect) >= 0) {
            if (poll == 3) __hip_atomic_store(relay, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          if (w >> 32) { v = 0; if (poll == 3) __hip_atomic_store(relay, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
        } else {
          v = __hip_atomic_load(relay, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (v == 0xFFFFFFFFu) { v = 0; break; }
          if ((int)(v - expect) >= 0) break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) { v = 0; break; }
        if (poll == 1 || (poll == 3 && !host)) __builtin_amdgcn_s_sleep(1);
        if (poll == 2) __builtin_amdgcn_s_sleep(8);
        if (poll == 4) __builtin_amdgcn_s_sleep(127);
      }
      cmd = v;
    }
    __syncthreads();
    const unsigned v = cmd;
    if (v == 0) return;
    lds[threadIdx.x & 511] = (float)v;
    spin_us(w_us);
    if (threadIdx.x == 0 && lds[5] < 0.f) sink[0] = lds[7];
    ticket_done(cnt, done, v, gridDim.x);
    expect = v + 1;
    __syncthreads();
  }
}

// a noise-like side kernel (4-wave workgroups, few VGPRs, no LDS) on another stream
__global__ __launch_bounds__(256) void k_side(float* out, int iters) {
  float x = (float)threadIdx.x;
  for (int i = 0; i < iters; ++i) x = x * 1.0001f + 0.5f;
  out[(blockIdx.x * 256 + threadIdx.x) & 4095] = x;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const unsigned w_us = argc > 1 ? atoi(argv[1]) : 70;
  const int steps = argc > 2 ? atoi(argv[2]) : 2000;
  const size_t lds = 150 * 1024;
  hipFuncSetAttribute((const void*)k_step, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipFuncSetAttribute((const void*)k_server, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  unsigned *cnt, *done;
  float* sink;
  Box* box;
  hipMalloc(&cnt, 64);
  hipMemset(cnt, 0, 64);
  hipMalloc(&sink, 64);
  hipHostMalloc(&done, 64, hipHostMallocDefault);
  hipHostMalloc(&box, sizeof(Box), hipHostMallocDefault);
  *done = 0;
  box->go = 0;
  box->stop = 0;
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  unsigned seq = 0;
  auto wait = [&](unsigned v) {
    const double t0 = now_us();
    while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != v) {
      __builtin_ia32_pause();
      if (now_us() - t0 > 2e6) {
        printf("timeout waiting for step %u\n", v);
        box->stop = 1;
        hipDeviceSynchronize();
        exit(2);
      }
    }
  };
  // launch per step
  for (int rep = 0; rep < 2; ++rep) {
    const double t0 = now_us();
    for (int i = 0; i < steps; ++i) {
      ++seq;
      hipLaunchKernelGGL(k_step, dim3(256), dim3(1024), lds, s, cnt, done, seq, w_us, sink);
      wait(seq);
    }
    const double t1 = now_us();
    hipStreamSynchronize(s);
    printf("launch-per-step  W=%u us: %.2f us/step (overhead %.2f)\n", w_us, (t1 - t0) / steps, (t1 - t0) / steps - w_us);
  }
  unsigned* relay;
  hipMalloc(&relay, 64);
  hipMemset(relay, 0, 64);
  for (int ps = 0; ps < 6; ++ps) {
    const int grid = ps == 5 ? 1 : 256;
    const int poll = ps == 5 ? 0 : ps;
    for (int rep = 0; rep < 2; ++rep) {
      box->stop = 0;
      hipMemset(relay, 0, 64);
      hipDeviceSynchronize();
      hipLaunchKernelGGL(k_server, dim3(grid), dim3(1024), lds, s, (const Box*)box, cnt, done, w_us, sink, poll, seq + 1,
                         relay);
      const double t0 = now_us();
      for (int i = 0; i < steps; ++i) {
        ++seq;
        box->state[3] = (float)i;
        __atomic_store_n(&box->go, seq, __ATOMIC_RELEASE);
        wait(seq);
      }
      const double t1 = now_us();
      __atomic_store_n(&box->stop, 1u, __ATOMIC_RELEASE);
      hipStreamSynchronize(s);
      printf("resident grid=%d poll=%d W=%u us: %.2f us/step (overhead %.2f)\n", grid, poll, w_us, (t1 - t0) / steps,
             (t1 - t0) / steps - w_us);
    }
  }
  // co-residency: a side kernel (1024 x 256 threads) on a low-priority stream per step while the
  // resident kernel (relay polling) serves the steps; time the host waits for the side kernel
  {
    hipStream_t s2;
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, lo);
    hipEvent_t e2;
    hipEventCreateWithFlags(&e2, hipEventDisableTiming);
    float* side;
    hipMalloc(&side, 4096 * sizeof(float));
    box->stop = 0;
    hipMemset(relay, 0, 64);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k_server, dim3(256), dim3(1024), lds, s, (const Box*)box, cnt, done, w_us, sink, 3, seq + 1, relay);
    double side_wait = 0, t0 = now_us();
    const int n = 200;
    for (int i = 0; i < n; ++i) {
      ++seq;
      __atomic_store_n(&box->go, seq, __ATOMIC_RELEASE);
      hipLaunchKernelGGL(k_side, dim3(1024), dim3(256), 0, s2, side, 2000);
      hipEventRecord(e2, s2);
      wait(seq);
      const double a = now_us();
      hipEventSynchronize(e2);
      side_wait += now_us() - a;
    }
    const double t1 = now_us();
    __atomic_store_n(&box->stop, 1u, __ATOMIC_RELEASE);
    hipStreamSynchronize(s);
    printf("resident + side kernel per step: %.2f us/step, host wait for the side kernel %.2f us/step\n",
           (t1 - t0) / n, side_wait / n);
  }
  return 0;
}
