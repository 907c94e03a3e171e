// Diagnostic (not part of the product): the cost of hipDeviceSynchronize / hipStreamSynchronize after N
// small kernels on side streams whose completion the host already saw (a flag each kernel writes to
// pinned memory), with and without an event recorded after each kernel.  Times in us.
// Build: hipcc --offload-arch=gfx950 -O2 devsync.hip -o devsync
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void touch(volatile unsigned* flag, unsigned v) {
  if (threadIdx.x == 0) __hip_atomic_store(const_cast<unsigned*>(flag), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t s[2];
  for (auto& x : s) hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
  hipEvent_t ev[2];
  for (auto& e : ev) hipEventCreateWithFlags(&e, hipEventDisableTiming);
  unsigned* flag = nullptr;
  hipHostMalloc(&flag, 64, hipHostMallocDefault);
  *flag = 0;
  unsigned seq = 0;
  for (int events = 0; events < 5; ++events) {
    for (int n : {1, 5, 20, 60}) {
      for (int rep = 0; rep < 3; ++rep) {
        hipDeviceSynchronize();
        for (int i = 0; i < n; ++i) {
          hipStream_t st = s[i & 1];
          ++seq;
          touch<<<1, 64, 0, st>>>(flag, seq);
          if (events == 1) hipEventRecord(ev[i & 1], st);
          // the host waits for this kernel by its flag (as the engine waits for a step's done word)
          // or, events == 2, by spinning on the event
          if (events == 2) {
            hipEventRecord(ev[i & 1], st);
            while (hipEventQuery(ev[i & 1]) == hipErrorNotReady) {
            }
          } else {
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
            }
          }
          // 3: a stream query once the kernel is seen done; 4: a stream synchronize then (timed)
          if (events == 3) (void)hipStreamQuery(st);
          if (events == 4) {
            const double a = now_us();
            hipStreamSynchronize(st);
            if (i == n - 1) printf("   (last incremental sync %.1f us)\n", now_us() - a);
          }
        }
        const double t0 = now_us();
        hipStreamSynchronize(s[0]);
        const double t1 = now_us();
        hipStreamSynchronize(s[1]);
        const double t2 = now_us();
        hipDeviceSynchronize();
        const double t3 = now_us();
        printf("events %d n %2d: stream sync %6.1f %6.1f  device sync %6.1f\n", events, n, t1 - t0, t2 - t1, t3 - t2);
      }
    }
  }
  return 0;
}
