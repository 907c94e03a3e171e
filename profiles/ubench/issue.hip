// VALU issue rate and dependent latency on one SIMD with 1, 2 or 4 co-resident waves (MI355X).
// One workgroup per CU (LDS-forced), each wave runs a 64-instruction inline-asm block per loop
// iteration: NACC independent chains (NACC = 1: dependent latency); s_memtime around the loop.
// Build: hipcc --offload-arch=gfx950 -O3 issue.hip -o issue
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

#define REP8(X) X X X X X X X X

template <int OP>
__global__ void issue_kernel(float* out, int iters, unsigned long long* cyc) {
  extern __shared__ float lds[];
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
        a6 = a0 + 6, a7 = a0 + 7;
  f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
  const float c = 0.99991f;
  unsigned si = blockIdx.x;
  if (threadIdx.x == 0) lds[0] = 0.f;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (OP == 0) {  // 8 independent v_fma_f32, x8
      REP8(asm volatile(
          "v_fma_f32 %0, %0, %8, 0.5\n v_fma_f32 %1, %1, %8, 0.5\n v_fma_f32 %2, %2, %8, 0.5\n"
          " v_fma_f32 %3, %3, %8, 0.5\n v_fma_f32 %4, %4, %8, 0.5\n v_fma_f32 %5, %5, %8, 0.5\n"
          " v_fma_f32 %6, %6, %8, 0.5\n v_fma_f32 %7, %7, %8, 0.5"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(c));)
    } else if constexpr (OP == 1) {  // one dependent chain of v_fma_f32, 64 long
      REP8(asm volatile(
          "v_fma_f32 %0, %0, %1, 0.5\n v_fma_f32 %0, %0, %1, 0.5\n v_fma_f32 %0, %0, %1, 0.5\n"
          " v_fma_f32 %0, %0, %1, 0.5\n v_fma_f32 %0, %0, %1, 0.5\n v_fma_f32 %0, %0, %1, 0.5\n"
          " v_fma_f32 %0, %0, %1, 0.5\n v_fma_f32 %0, %0, %1, 0.5"
          : "+v"(a0)
          : "v"(c));)
    } else if constexpr (OP == 2) {  // 4 independent v_pk_fma_f32 (8 FMAs), x16
      REP8(asm volatile(
          "v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n v_pk_fma_f32 %2, %2, %4, %4\n"
          " v_pk_fma_f32 %3, %3, %4, %4\n v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n"
          " v_pk_fma_f32 %2, %2, %4, %4\n v_pk_fma_f32 %3, %3, %4, %4"
          : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)
          : "v"(f2{c, c}));)
    } else if constexpr (OP == 3) {  // 8 independent v_sqrt_f32
      REP8(asm volatile(
          "v_sqrt_f32 %0, %0\n v_sqrt_f32 %1, %1\n v_sqrt_f32 %2, %2\n v_sqrt_f32 %3, %3\n"
          " v_sqrt_f32 %4, %4\n v_sqrt_f32 %5, %5\n v_sqrt_f32 %6, %6\n v_sqrt_f32 %7, %7"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    } else if constexpr (OP == 4) {  // dependent v_pk_fma_f32 chain
      REP8(asm volatile(
          "v_pk_fma_f32 %0, %0, %1, %1\n v_pk_fma_f32 %0, %0, %1, %1\n v_pk_fma_f32 %0, %0, %1, %1\n"
          " v_pk_fma_f32 %0, %0, %1, %1\n v_pk_fma_f32 %0, %0, %1, %1\n v_pk_fma_f32 %0, %0, %1, %1\n"
          " v_pk_fma_f32 %0, %0, %1, %1\n v_pk_fma_f32 %0, %0, %1, %1"
          : "+v"(p0)
          : "v"(f2{c, c}));)
    } else if constexpr (OP == 6) {  // 4 independent v_fma_f32 interleaved with 4 s_add_u32, x8
      REP8(asm volatile(
          "v_fma_f32 %0, %0, %5, 0.5\n s_add_u32 %4, %4, 3\n v_fma_f32 %1, %1, %5, 0.5\n s_add_u32 %4, %4, 5\n"
          " v_fma_f32 %2, %2, %5, 0.5\n s_add_u32 %4, %4, 7\n v_fma_f32 %3, %3, %5, 0.5\n s_add_u32 %4, %4, 9"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+s"(si)
          : "v"(c) : "scc");)
    } else if constexpr (OP == 7) {  // 8 v_mov_b32 from SGPR, x8
      REP8(asm volatile(
          "v_mov_b32 %0, %8\n v_mov_b32 %1, %8\n v_mov_b32 %2, %8\n v_mov_b32 %3, %8\n"
          " v_mov_b32 %4, %8\n v_mov_b32 %5, %8\n v_mov_b32 %6, %8\n v_mov_b32 %7, %8"
          : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7)
          : "s"(si));)
    } else if constexpr (OP == 8) {  // 7 independent v_fma_f32 + 1 v_sqrt_f32, x8
      REP8(asm volatile(
          "v_fma_f32 %0, %0, %8, 0.5\n v_fma_f32 %1, %1, %8, 0.5\n v_fma_f32 %2, %2, %8, 0.5\n"
          " v_sqrt_f32 %3, %3\n v_fma_f32 %4, %4, %8, 0.5\n v_fma_f32 %5, %5, %8, 0.5\n"
          " v_fma_f32 %6, %6, %8, 0.5\n v_fma_f32 %7, %7, %8, 0.5"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(c));)
    } else {  // dependent v_sqrt_f32 chain
      REP8(asm volatile(
          "v_sqrt_f32 %0, %0\n v_sqrt_f32 %0, %0\n v_sqrt_f32 %0, %0\n v_sqrt_f32 %0, %0\n"
          " v_sqrt_f32 %0, %0\n v_sqrt_f32 %0, %0\n v_sqrt_f32 %0, %0\n v_sqrt_f32 %0, %0"
          : "+v"(a0));)
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const float s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p0.y + p1.x + p1.y + p2.x + p2.y + p3.x + p3.y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s + lds[0] + (float)si;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
static void run(const char* name, int threads) {
  const int blocks = 256, iters = 2048;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * threads * sizeof(float));
  hipMalloc(&cyc, blocks * (threads / 64) * sizeof(unsigned long long));
  const size_t lds = 96 * 1024;
  hipFuncSetAttribute((const void*)issue_kernel<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  for (int r = 0; r < 2; ++r) issue_kernel<OP><<<blocks, threads, lds>>>(out, iters, cyc);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * (threads / 64));
  hipMemcpy(h.data(), cyc, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double sum = 0;
  for (auto v : h) sum += (double)v;
  const double per_wave = sum / h.size();
  const double ins = (double)iters * 64;
  printf("%-12s waves/SIMD=%d  cycles/instr per wave=%6.2f  SIMD aggregate=%6.2f\n", name, threads / 256,
         per_wave / ins, per_wave / ins / (threads / 256));
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  for (int t : {256, 512, 768, 1024}) {
    run<0>("fma x8", t);
    run<1>("fma dep", t);
    run<2>("pk_fma x4", t);
    run<4>("pk_fma dep", t);
    run<3>("sqrt x8", t);
    run<5>("sqrt dep", t);
    run<6>("fma+salu", t);
    run<7>("vmov x8", t);
    run<8>("fma7+sqrt", t);
  }
  return 0;
}
