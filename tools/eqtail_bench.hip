// Phase timeline of sumcheck_eq_tail_kernel (the last 12 rounds of the
// eq-factored sumcheck in one LDS workgroup, after a 3-level load fold):
// sumcheck.hip built with MLH_TAIL_PROF, thread 0 stamps wall_clock64().
// Dev tool:  hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/eqtail_bench.hip -o tools/eqtail_bench
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
  const uint32_t a = 12, Jin = 0, NT = 1u << (a + Jin);
  std::vector<fe> h(NT + (1u << a) + 16);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  auto next = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (uint32_t)x; };
  for (auto& v : h) v = fe{{next(), next(), next(), next() >> 1}};
  fe *tin, *ets, *pts, *c, *prev, *polys, *rs, *mo, *dout;
  DevSha* t;
  CHECK(hipMalloc(&tin, NT * sizeof(fe)));
  CHECK(hipMalloc(&ets, (1u << a) * sizeof(fe)));
  CHECK(hipMalloc(&pts, 16 * sizeof(fe)));
  CHECK(hipMalloc(&c, sizeof(fe)));
  CHECK(hipMalloc(&prev, sizeof(fe)));
  CHECK(hipMalloc(&polys, 2 * a * sizeof(fe)));
  CHECK(hipMalloc(&rs, (a + 3) * sizeof(fe)));
  CHECK(hipMalloc(&mo, sizeof(fe)));
  CHECK(hipMalloc(&dout, sizeof(fe)));
  CHECK(hipMalloc(&t, sizeof(DevSha)));
  CHECK(hipMemcpy(tin, h.data(), NT * sizeof(fe), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(ets, h.data() + NT, (1u << a) * sizeof(fe), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(pts, h.data() + NT + (1u << a), 16 * sizeof(fe), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(rs, h.data(), 3 * sizeof(fe), hipMemcpyHostToDevice));
  int khz = 0;
  CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const double us = 1e3 / khz;
  for (int rep = 0; rep < 3; ++rep) {
    DevSha hs{};
    const fe one{{1, 0, 0, 0}};
    CHECK(hipMemcpy(t, &hs, sizeof hs, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(c, &one, sizeof one, hipMemcpyHostToDevice));
    CHECK(hipMemset(prev, 0, sizeof(fe)));
    CHECK(launch_sumcheck_eq_tail(tin, Jin, rs, a, ets, pts, c, prev, t, polys, rs + 3, mo, dout,
                                  nullptr, CoopCtl{}));
    CHECK(hipDeviceSynchronize());
  }
  uint64_t ts[64];
  CHECK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(g_tail_ts), sizeof ts));
  printf("eq tail: total %.2f us, load+fold %.2f us\n", (ts[42 + 12] - ts[38]) * us,
         (ts[39] - ts[38]) * us);
  for (int g = 0; g < 4; ++g) {
    const uint64_t a0 = g == 0 ? ts[39] : ts[42 + 4 * (g - 1)];
    printf(" group %d: corner sums %.2f  rounds %.2f  fold %.2f\n", g, (ts[40 + 4 * g] - a0) * us,
           (ts[41 + 4 * g] - ts[40 + 4 * g]) * us, (ts[42 + 4 * g] - ts[41 + 4 * g]) * us);
  }
  printf(" last group rounds: stepA E-shfl stepB interp absorb challenge bcast\n");
  for (int k = 0; k < 3; ++k) {
    const int b = 3 + 8 * k;
    const uint64_t a0 = k == 0 ? ts[40 + 12] : ts[b - 8 + 7];
    printf("  %d: %5.2f %5.2f %5.2f %5.2f %5.2f %5.2f %5.2f\n", k, (ts[b] - a0) * us,
           (ts[b + 1] - ts[b]) * us, (ts[b + 2] - ts[b + 1]) * us, (ts[b + 3] - ts[b + 2]) * us,
           (ts[b + 4] - ts[b + 3]) * us, (ts[b + 5] - ts[b + 4]) * us, (ts[b + 7] - ts[b + 5]) * us);
  }
  return 0;
}
