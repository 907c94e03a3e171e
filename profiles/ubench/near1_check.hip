// Exhaustive check (GPU): for divisors b within 4096 ulps of 1 (the chain's re-normalisations of
// vectors that are unit up to rounding), is the quotient with the UNREFINED v_rcp_f32 and one residual
// correction equal to the IEEE quotient, for every significand of a (and both signs of the binade of b)?
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off near1_check.hip -o near1_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void near1(uint32_t a0, uint32_t na, unsigned long long* bad, uint32_t* ex) {
  const uint32_t bb = 0x3F800000u - 4096u + blockIdx.x * blockDim.x + threadIdx.x;  // 8192 divisors
  const float b = __builtin_bit_cast(float, bb);
  const float y = __builtin_amdgcn_rcpf(b);
  for (uint32_t i = 0; i < na; ++i) {
    const float a = __builtin_bit_cast(float, 0x3F800000u | (a0 + i));
    const float q0 = a * y;
    const float e0 = __builtin_fmaf(b, q0, -a);
    const float q = __builtin_fmaf(-e0, y, q0);
    if (__builtin_bit_cast(uint32_t, q) != __builtin_bit_cast(uint32_t, a / b)) {
      const unsigned long long k = atomicAdd(bad, 1ull);
      if (k < 8) { ex[2 * k] = __builtin_bit_cast(uint32_t, a); ex[2 * k + 1] = bb; }
    }
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
  for (uint32_t a0 = 0; a0 < (1u << 23); a0 += (1u << 18)) near1<<<8192 / 256, 256>>>(a0, 1u << 18, bad, ex);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hx, ex, 64, hipMemcpyDeviceToHost);
  printf("unrefined-reciprocal quotients, b in [1 - 4096 ulp, 1 + 4096 ulp) x all a significands: %llu mismatches\n", h);
  for (unsigned k = 0; k < 8 && k < h; ++k) printf("  a=0x%08x b=0x%08x\n", hx[2 * k], hx[2 * k + 1]);
  return 0;
}
