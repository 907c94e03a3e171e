// Exhaustive checks (GPU) of the hardware reciprocal and square root against the correctly rounded
// results, for the chain's fast paths:
//   (1) v_rcp_f32(b) == RN(1/b) (the refined y0 + y0 (1 - b y0), itself checked against 1.0f / b)
//       for every significand of b in [1, 2);
//   (2) the quotient with the UNREFINED reciprocal and one residual correction against a / b for
//       every pair of significands (only if (1) fails somewhere: else Markstein applies as it is);
//   (3) v_sqrt_f32(x) == sqrtf(x) (IEEE) for every x in [2^-80, 2^80] (both binade parities).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off rcp_sqrt_check.hip -o rcp_sqrt_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void rcp_all(unsigned long long* bad, uint32_t* ex) {
  const uint32_t mb = blockIdx.x * blockDim.x + threadIdx.x;
  if (mb >= (1u << 23)) return;
  const float b = __builtin_bit_cast(float, 0x3F800000u | mb);
  const float y0 = __builtin_amdgcn_rcpf(b);
  const float r = 1.0f / b;
  if (__builtin_bit_cast(uint32_t, y0) != __builtin_bit_cast(uint32_t, r)) {
    const unsigned long long k = atomicAdd(bad, 1ull);
    if (k < 8) ex[k] = __builtin_bit_cast(uint32_t, b);
  }
}
__global__ void div_raw(uint32_t b0, uint32_t a0, uint32_t na, unsigned long long* bad, uint32_t* ex) {
  const uint32_t mb = b0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (mb >= (1u << 23)) return;
  const float b = __builtin_bit_cast(float, 0x3F800000u | mb);
  const float y = __builtin_amdgcn_rcpf(b);
  for (uint32_t i = 0; i < na; ++i) {
    const float a = __builtin_bit_cast(float, 0x3F800000u | (a0 + i));
    const float q0 = a * y;
    const float e0 = __builtin_fmaf(b, q0, -a);
    const float q = __builtin_fmaf(-e0, y, q0);
    if (__builtin_bit_cast(uint32_t, q) != __builtin_bit_cast(uint32_t, a / b)) {
      const unsigned long long k = atomicAdd(bad, 1ull);
      if (k < 8) { ex[2 * k] = __builtin_bit_cast(uint32_t, a); ex[2 * k + 1] = __builtin_bit_cast(uint32_t, b); }
    }
  }
}
__global__ void sqrt_all(uint32_t lo, uint32_t n, unsigned long long* bad, uint32_t* ex) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = __builtin_bit_cast(float, lo + i);
  const float s = __builtin_amdgcn_sqrtf(x);
  if (__builtin_bit_cast(uint32_t, s) != __builtin_bit_cast(uint32_t, sqrtf(x))) {
    const unsigned long long k = atomicAdd(bad, 1ull);
    if (k < 8) ex[k] = lo + i;
  }
}

int main() {
  unsigned long long* bad;
  uint32_t* ex;
  unsigned long long h = 0;
  uint32_t hx[16];
  (void)hipMalloc(&bad, 8);
  (void)hipMalloc(&ex, 64);
  (void)hipMemset(bad, 0, 8);
  rcp_all<<<(1u << 23) / 256, 256>>>(bad, ex);
  (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hx, ex, 64, hipMemcpyDeviceToHost);
  printf("(1) v_rcp_f32 != RN(1/b): %llu of 2^23 significands", h);
  for (unsigned k = 0; k < 8 && k < h; ++k) printf(" 0x%08x", hx[k]);
  printf("\n");
  fflush(stdout);
  if (h) {
    (void)hipMemset(bad, 0, 8);
    for (uint32_t b0 = 0; b0 < (1u << 23); b0 += (1u << 20)) {
      for (uint32_t a0 = 0; a0 < (1u << 23); a0 += (1u << 20)) div_raw<<<(1u << 20) / 256, 256>>>(b0, a0, 1u << 20, bad, ex);
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
      printf("  (2) raw-reciprocal quotients, b significands < %u: %llu mismatches\n", b0 + (1u << 20), h);
      fflush(stdout);
    }
    (void)hipMemcpy(hx, ex, 64, hipMemcpyDeviceToHost);
    for (unsigned k = 0; k < 4 && k < h; ++k) printf("    a=0x%08x b=0x%08x\n", hx[2 * k], hx[2 * k + 1]);
  }
  (void)hipMemset(bad, 0, 8);
  const uint32_t lo = 0x17800000u, hi = 0x67800000u;  // 2^-80 .. 2^80
  for (uint32_t s = lo; s < hi; s += (1u << 26)) {
    const uint32_t n = (hi - s) < (1u << 26) ? (hi - s) : (1u << 26);
    sqrt_all<<<(n + 255) / 256, 256>>>(s, n, bad, ex);
  }
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hx, ex, 64, hipMemcpyDeviceToHost);
  printf("(3) v_sqrt_f32 != sqrtf over [2^-80, 2^80]: %llu", h);
  for (unsigned k = 0; k < 8 && k < h; ++k) printf(" 0x%08x", hx[k]);
  printf("\n");
  return 0;
}
