// Phase timeline of sumcheck_group_kernel (one launch = the 3 rounds of an
// eq-factored head group): builds sumcheck.hip with MLH_TAIL_PROF so thread 0
// stamps wall_clock64() at each phase.  Dev tool, not product code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/group_bench.hip -o tools/group_bench
#define MLH_TAIL_PROF 1
#include "../multilinear_amd/csrc/sumcheck.hip"

#include <stdio.h>

#include <vector>

#define CHECK(x)                                                       \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main() {
  using namespace mlh;
  const uint32_t J = 3, J2 = 3, nb = 64, NP = nb << (J + J2);
  std::vector<fe> hp(NP + 8);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  auto next = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (uint32_t)x; };
  for (auto& v : hp) v = fe{{next(), next(), next(), next() >> 1}};
  fe *parts, *pts, *c, *prev, *polys, *rs;
  DevSha* t;
  CHECK(hipMalloc(&parts, NP * sizeof(fe)));
  CHECK(hipMalloc(&pts, 8 * sizeof(fe)));
  CHECK(hipMalloc(&c, sizeof(fe)));
  CHECK(hipMalloc(&prev, sizeof(fe)));
  CHECK(hipMalloc(&polys, 12 * sizeof(fe)));
  CHECK(hipMalloc(&rs, 6 * sizeof(fe)));
  CHECK(hipMalloc(&t, sizeof(DevSha)));
  CHECK(hipMemcpy(parts, hp.data(), NP * sizeof(fe), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(pts, hp.data() + NP, 8 * sizeof(fe), hipMemcpyHostToDevice));
  int wrate_khz = 0;
  CHECK(hipDeviceGetAttribute(&wrate_khz, hipDeviceAttributeWallClockRate, 0));
  const double us = 1e3 / wrate_khz;
  for (int len0 = 0; len0 < 2; ++len0) {  // transcript len 0 / 32 mod 64: which rounds compress
    for (int rep = 0; rep < 3; ++rep) {
      DevSha hs{};
      hs.len = 32 * len0;
      const fe one{{1, 0, 0, 0}};
      CHECK(hipMemcpy(t, &hs, sizeof hs, hipMemcpyHostToDevice));
      CHECK(hipMemcpy(c, &one, sizeof one, hipMemcpyHostToDevice));
      CHECK(hipMemset(prev, 0, sizeof(fe)));
      CHECK(launch_sumcheck_group(parts, nb, J, J2, 0, J, prev, t, polys, rs, pts, c, nullptr, CoopCtl{}, nullptr));
      CHECK(hipDeviceSynchronize());
    }
    uint64_t ts[64];
    CHECK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(g_tail_ts), sizeof ts));
    uint64_t cy[64];
    CHECK(hipMemcpyFromSymbol(cy, HIP_SYMBOL(g_tail_cyc), sizeof cy));
    printf("shader clock %.3f GHz (s_memtime / wall over the launch); challenge cycles:",
           (cy[63] - cy[0]) / ((ts[63] - ts[0]) * us * 1e3));
    for (uint32_t k = 0; k < J; ++k) printf(" %llu", (unsigned long long)(cy[3 + 8 * k + 5] - cy[3 + 8 * k + 4]));
    printf("\n");
    printf("len0 %d: total %.2f us; partial loads %.2f; block reduce %.2f\n", 32 * len0,
           (ts[63] - ts[0]) * us, (ts[1] - ts[0]) * us, (ts[2] - ts[1]) * us);
    printf(" round  stepA  E-shfl  stepB  interp  absorb  challenge  bcast\n");
    for (uint32_t k = 0; k < J; ++k) {
      const int b = 3 + 8 * k;
      const uint64_t a = k == 0 ? ts[2] : ts[b - 8 + 7];
      printf(" %5u  %5.2f  %6.2f  %5.2f  %6.2f  %6.2f  %9.2f  %5.2f\n", k, (ts[b] - a) * us,
             (ts[b + 1] - ts[b]) * us, (ts[b + 2] - ts[b + 1]) * us, (ts[b + 3] - ts[b + 2]) * us,
             (ts[b + 4] - ts[b + 3]) * us, (ts[b + 5] - ts[b + 4]) * us,
             (ts[b + 7] - ts[b + 5]) * us);
    }
  }
  return 0;
}
