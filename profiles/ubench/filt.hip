// Diagnostic microbenchmark (not part of the product): the finish's serial wheel filter
// (L = L a + in, R = R a + in on one lane) in isolation, packed (v_pk_mul/v_pk_add on (L, R)) or
// as two scalar chains, with 64 or 1024 threads in the workgroup (the other waves at a barrier).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize filt.hip -o filt
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ void filt_kernel(int H, float a, float wl, float wr, unsigned long long* cyc, float* sink) {
  __shared__ __attribute__((aligned(16))) float uo[2 * 256 + 128];
  __shared__ __attribute__((aligned(16))) f2 lr[256 + 64];
  for (int i = threadIdx.x; i < 2 * 256 + 128; i += blockDim.x) uo[i] = 1e-3f * (float)(i % 17);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (MODE == 0) {  // the product loop: two blocks of 8 packed steps per iteration
      const f2* p = reinterpret_cast<const f2*>(uo);
      f2* q = lr;
      const f2 a2 = f2{a, a};
      f2 LR = f2{wl, wr};
      f2 A[8], B[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) A[k] = p[k];
      int t = 0;
      for (; t + 16 <= H; t += 16, p += 16, q += 16) {
#pragma unroll
        for (int k = 0; k < 8; ++k) B[k] = p[8 + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          LR = LR * a2 + A[k];
          A[k] = LR;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = A[k];
#pragma unroll
        for (int k = 0; k < 8; ++k) A[k] = p[16 + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          LR = LR * a2 + B[k];
          B[k] = LR;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) q[8 + k] = B[k];
      }
      for (int k = 0; t < H; ++t, ++k) {
        LR = LR * a2 + p[k];
        q[k] = LR;
      }
    } else if constexpr (MODE == 1) {  // the same on two scalar chains
      const f2* p = reinterpret_cast<const f2*>(uo);
      f2* q = lr;
      float L = wl, R = wr;
      f2 A[8], B[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) A[k] = p[k];
      int t = 0;
      for (; t + 16 <= H; t += 16, p += 16, q += 16) {
#pragma unroll
        for (int k = 0; k < 8; ++k) B[k] = p[8 + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          L = L * a + A[k].x;
          R = R * a + A[k].y;
          A[k] = f2{L, R};
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = A[k];
#pragma unroll
        for (int k = 0; k < 8; ++k) A[k] = p[16 + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          L = L * a + B[k].x;
          R = R * a + B[k].y;
          B[k] = f2{L, R};
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) q[8 + k] = B[k];
      }
      for (int k = 0; t < H; ++t, ++k) {
        L = L * a + p[k].x;
        R = R * a + p[k].y;
        q[k] = f2{L, R};
      }
    } else if constexpr (MODE == 3) {
      // (handled below by lanes 0 and 1)
    } else {  // registers only: 96 steps, no LDS in the loop
      f2 LR = f2{wl, wr};
      const f2 a2 = f2{a, a};
      const f2 in = f2{uo[3], uo[5]};
#pragma unroll
      for (int k = 0; k < 96; ++k) LR = LR * a2 + in;
      lr[0] = LR;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (MODE != 3) cyc[0] = t1 - t0;
  }
  if (MODE == 3 && threadIdx.x < 2) {
    // lanes 0 and 1 each run one wheel's scalar chain over a planar row (L then R, stride PS):
    // one ds_read_b128 / ds_write_b128 per lane per 4 steps
    const int PS = ((H + 3) & ~3) + 32;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4* p = reinterpret_cast<const f4*>(uo + threadIdx.x * PS);
    f4* q = reinterpret_cast<f4*>(reinterpret_cast<float*>(lr) + threadIdx.x * PS);
    float x = threadIdx.x ? wr : wl;
    f4 A[4], B[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) A[k] = p[k];
    int t = 0;
    for (; t + 32 <= H; t += 32, p += 8, q += 8) {
#pragma unroll
      for (int k = 0; k < 4; ++k) B[k] = p[4 + k];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x = x * a + A[k].x; A[k].x = x;
        x = x * a + A[k].y; A[k].y = x;
        x = x * a + A[k].z; A[k].z = x;
        x = x * a + A[k].w; A[k].w = x;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = A[k];
#pragma unroll
      for (int k = 0; k < 4; ++k) A[k] = p[8 + k];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x = x * a + B[k].x; B[k].x = x;
        x = x * a + B[k].y; B[k].y = x;
        x = x * a + B[k].z; B[k].z = x;
        x = x * a + B[k].w; B[k].w = x;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) q[4 + k] = B[k];
    }
    const float* pf = reinterpret_cast<const float*>(p);
    float* qf = reinterpret_cast<float*>(q);
    for (int k = 0; t < H; ++t, ++k) {
      x = x * a + pf[k];
      qf[k] = x;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
  }
  __syncthreads();
  if (threadIdx.x == 0) sink[0] = lr[H - 1].x + lr[0].y;
}

int main() {
  unsigned long long* d;
  float* s;
  hipMalloc(&d, 64);
  hipMalloc(&s, 64);
  unsigned long long h = 0;
  const char* names[] = {"packed (product loop)", "two scalar chains", "packed, registers only (96)", "lanes 0/1 planar b128"};
  for (int nt : {64, 1024}) {
    for (int rep = 0; rep < 3; ++rep) {
#define RUN(M)                                                                                  \
  hipLaunchKernelGGL(filt_kernel<M>, dim3(1), dim3(nt), 0, 0, 100, 0.92f, 0.1f, 0.2f, d, s);   \
  hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);                                                  \
  if (rep == 2) printf("threads %4d  %-28s %7llu cycles / 100 steps\n", nt, names[M], h);
      RUN(0) RUN(1) RUN(2) RUN(3)
    }
  }
  return 0;
}
