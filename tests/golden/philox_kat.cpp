// Known-answer vectors for the engine's noise counter mapping, produced by
// rocRAND's own Philox4x32-10 (rocrand_philox4x32_10.h, ROCm 7.2 headers),
// evaluated on the host.  For each (seed, subsequence k, block n) prints
//   rocrand4(rocrand_init(seed, k, 4*n))
// which the engine restates as philox4x32_10(counter=(n, k), key=seed)
// (csrc/mppi_detmath.h, oracle/dmath.py).  Built and run by make_golden.py.
#include <rocrand/rocrand_kernel.h>

#include <cstdio>

int main() {
  const unsigned long long seeds[] = {0ull, 42ull, 0xFFFFFFFFull, 0x123456789ABCDEF0ull};
  const unsigned long long ks[] = {0ull, 1ull, 5ull, 65535ull, (1ull << 32) + 3ull};
  const unsigned long long ns[] = {0ull, 1ull, 7ull, 50ull, (1ull << 32) + 1ull};
  for (unsigned long long s : seeds)
    for (unsigned long long k : ks)
      for (unsigned long long n : ns) {
        rocrand_state_philox4x32_10 st;
        rocrand_init(s, k, 4ull * n, &st);
        uint4 r = rocrand4(&st);
        std::printf("%llu %llu %llu %u %u %u %u\n", s, k, n, r.x, r.y, r.z, r.w);
      }
  return 0;
}
