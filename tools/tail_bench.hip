// Phase timeline of sumcheck_tail_kernel (the last 12 sumcheck rounds in one
// LDS-resident workgroup): builds sumcheck.hip with MLH_TAIL_PROF so thread 0
// stamps wall_clock64() at each phase, then prints per-round durations of
// reduce / absorb / challenge / barrier / fold.  Dev tool, not product code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/tail_bench.hip -o tools/tail_bench
#define MLH_TAIL_PROF 1
#include "../multilinear_amd/csrc/sumcheck.hip"

#include <stdio.h>
#include <string.h>

#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

int main() {
  using namespace mlh;
  const uint32_t log_s = 12, S = 1u << log_s;
  std::vector<fe> hm(S), hd(S);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  auto next = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (uint32_t)x; };
  for (uint32_t i = 0; i < S; ++i) {  // top limb < 2^31: canonical
    hm[i] = fe{{next(), next(), next(), next() >> 1}};
    hd[i] = fe{{next(), next(), next(), next() >> 1}};
  }
  fe *m, *d, *prev, *polys, *rs;
  DevSha* t;
  CHECK(hipMalloc(&m, S * sizeof(fe)));
  CHECK(hipMalloc(&d, S * sizeof(fe)));
  CHECK(hipMalloc(&prev, sizeof(fe)));
  CHECK(hipMalloc(&polys, 2 * log_s * sizeof(fe)));
  CHECK(hipMalloc(&rs, log_s * sizeof(fe)));
  CHECK(hipMalloc(&t, sizeof(DevSha)));
  int wrate_khz = 0;
  CHECK(hipDeviceGetAttribute(&wrate_khz, hipDeviceAttributeWallClockRate, 0));
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipMemcpy(m, hm.data(), S * sizeof(fe), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d, hd.data(), S * sizeof(fe), hipMemcpyHostToDevice));
    CHECK(hipMemset(prev, 0, sizeof(fe)));
    CHECK(hipMemset(t, 0, sizeof(DevSha)));
    CHECK(launch_sumcheck_tail(m, d, log_s, prev, t, polys, rs, nullptr, nullptr));
    CHECK(hipDeviceSynchronize());
  }
  uint64_t ts[64];
  CHECK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(g_tail_ts), sizeof ts));
  const double us = 1e3 / wrate_khz;  // one wall-clock tick in us
  printf("wall clock %d kHz; total %.1f us; load %.1f us; first sums %.1f us\n", wrate_khz,
         (ts[63] - ts[0]) * us, (ts[1] - ts[0]) * us, (ts[2] - ts[1]) * us);
  printf("round  fold+sums  block_reduce  absorb  challenge+p  barrier\n");
  for (uint32_t k = 0; k < log_s; ++k) {
    const uint64_t a = k == 0 ? ts[2] : ts[6 + 4 * (k - 1)];
    printf("%5u  %9.2f  %12.2f  %6.2f  %11.2f  %7.2f\n", k, (ts[51 + k] - a) * us,
           (ts[3 + 4 * k] - ts[51 + k]) * us, (ts[4 + 4 * k] - ts[3 + 4 * k]) * us,
           (ts[5 + 4 * k] - ts[4 + 4 * k]) * us, (ts[6 + 4 * k] - ts[5 + 4 * k]) * us);
  }
  printf("(fold+sums: the previous round's fold with this round's sums; round 0: none)\n");
  return 0;
}
