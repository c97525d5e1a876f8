// Round timeline of the cooperative serial-round kernels (sumcheck_group_kernel
// with 6 rounds from 64 corners, sumcheck_eq_tail_kernel with 12 rounds):
// builds sumcheck.hip with MLH_COOP_PROF, so wave 0 and the coefficient helper
// stamp s_memtime per round.  Prints per round: wave 0's wait for its slot,
// evaluation + absorb, challenge; and when the helper published the slot.
// Synthetic inputs; dev tool, not product code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/coop_bench.hip -o tools/coop_bench
#ifdef MLH_COOP_OLD  // an older sumcheck.hip for A/B launch timing (no per-round stamps)
#include MLH_COOP_OLD
#else
#define MLH_COOP_PROF 1
#include "../multilinear_amd/csrc/sumcheck.hip"
#endif

#include <stdio.h>
#include <stdlib.h>
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

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t next32() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)rng;
}
static mlh::fe rand_fe() { return mlh::fe{{next32(), next32(), next32(), next32() >> 1}}; }

static uint32_t hrotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
// K + W of the padding-only block of a message of len bytes (len % 64 == 0)
static void pad_kw(uint64_t len, uint32_t* kw) {
  static const uint32_t K[64] = MLH_SHA_K;
  uint32_t w[64] = {};
  w[0] = 0x80000000u;
  w[14] = (uint32_t)((len * 8) >> 32);
  w[15] = (uint32_t)(len * 8);
  for (int t = 16; t < 64; ++t) {
    const uint32_t a = w[t - 15], b = w[t - 2];
    w[t] = w[t - 16] + (hrotr(a, 7) ^ hrotr(a, 18) ^ (a >> 3)) + w[t - 7] +
           (hrotr(b, 17) ^ hrotr(b, 19) ^ (b >> 10));
  }
  for (int t = 0; t < 64; ++t) kw[t] = K[t] + w[t];
}

static int report(const char* what, uint32_t R) {
#ifdef MLH_COOP_OLD
  (void)what;
  (void)R;
  return 0;
#else
  uint64_t ts[10][64];
  CHECK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(mlh::g_coop_ts), sizeof ts));
  const double cyc_us = 1.0 / 2400.0;  // s_memtime ticks at the shader clock (~2.4 GHz)
  uint64_t ed[4];
  CHECK(hipMemcpyFromSymbol(ed, HIP_SYMBOL(mlh::g_coop_edge), sizeof ed));
  int wrate_khz = 0;
  CHECK(hipDeviceGetAttribute(&wrate_khz, hipDeviceAttributeWallClockRate, 0));
  printf("%s: total %.1f us (first wait start -> last r); entry -> roles %.2f us (wall %.2f us, "
         "clock %.2f GHz)\n", what, (ts[3][R - 1] - ts[0][0]) * cyc_us, (ed[2] - ed[0]) * cyc_us,
         (ed[3] - ed[1]) * 1e3 / wrate_khz, (double)(ed[2] - ed[0]) / ((ed[3] - ed[1]) * 1e6 / wrate_khz) / 1e3);
  printf("round   wait  eval+absorb  challenge   slot_ready(vs r_{k-2})\n");
  for (uint32_t k = 0; k < R; ++k) {
    const double lag = k >= 2 ? ((double)ts[4][k] - (double)ts[3][k - 2]) * cyc_us : 0.0;
    printf("%5u %6.2f %12.2f %10.2f %12.2f\n", k, (ts[1][k] - ts[0][k]) * cyc_us,
           (ts[2][k] - ts[1][k]) * cyc_us, (ts[3][k] - ts[2][k]) * cyc_us, lag);
  }
  printf("helper: round  eval+LW  bucket  ps_next  to_slot\n");
  for (uint32_t k = 1; k < R; ++k)
    printf("       %5u %8.2f %7.2f %8.2f %8.2f\n", k, (ts[6][k] - ts[5][k]) * cyc_us,
           (ts[7][k] - ts[6][k]) * cyc_us, (ts[8][k] - ts[7][k]) * cyc_us,
           (ts[4][k] - ts[8][k]) * cyc_us);
  return 0;
#endif
}

int main() {
  using namespace mlh;
  // ---- group kernel: J = 3 + J2 = 3, 64 corners, nb = 64 partials per corner (as config 4)
  {
    const uint32_t nb = 64, JT = 6;
    fe *big, *bigH;
    CHECK(hipMalloc(&big, (1ull << 24) * sizeof(fe)));
    CHECK(hipMalloc(&bigH, 4096 * sizeof(fe)));
    CHECK(hipMemset(big, 0x11, (1ull << 24) * sizeof(fe)));
    CHECK(hipMemset(bigH, 0x01, 4096 * sizeof(fe)));
    std::vector<fe> hp(64 * nb), hpts(JT);
    for (auto& v : hp) v = rand_fe();
    for (auto& v : hpts) v = rand_fe();
    fe *partials, *prev, *polys, *rs, *pts, *cdev, *wout;
    DevSha* t;
    uint32_t* kw;
    CHECK(hipMalloc(&partials, hp.size() * sizeof(fe)));
    CHECK(hipMalloc(&prev, sizeof(fe)));
    CHECK(hipMalloc(&polys, 2 * JT * sizeof(fe)));
    CHECK(hipMalloc(&rs, JT * sizeof(fe)));
    CHECK(hipMalloc(&pts, JT * sizeof(fe)));
    CHECK(hipMalloc(&cdev, sizeof(fe)));
    CHECK(hipMalloc(&wout, 64 * sizeof(fe)));
    CHECK(hipMalloc(&t, sizeof(DevSha)));
    CHECK(hipMalloc(&kw, 64 * JT * 4));
    std::vector<uint32_t> hkw(64 * JT, 0);
    for (uint32_t k = 0; k < JT; ++k)
      if ((32 * (k + 1)) % 64 == 0) pad_kw(32 * (k + 1), hkw.data() + 64 * k);
    CHECK(hipMemcpy(kw, hkw.data(), hkw.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(partials, hp.data(), hp.size() * sizeof(fe), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(pts, hpts.data(), JT * sizeof(fe), hipMemcpyHostToDevice));
    // FLUSH=1: stream 1 GiB through the L2s before each launch (as the folds
    // before the tail launch of a prove do), so the kernel's code comes from HBM
    const char* fl = getenv("FLUSH");
    void* junk = nullptr;
    if (fl && *fl == '1') CHECK(hipMalloc(&junk, 1ull << 30));
    for (int rep = 0; rep < 5; ++rep) {
      if (junk) CHECK(hipMemsetAsync(junk, rep, 1ull << 30, 0));
      const fe one{{1, 0, 0, 0}}, cl = rand_fe();
      CHECK(hipMemcpy(cdev, &one, sizeof(fe), hipMemcpyHostToDevice));
      CHECK(hipMemcpy(prev, &cl, sizeof(fe), hipMemcpyHostToDevice));
      DevSha s0{};
      for (int i = 0; i < 8; ++i) s0.h[i] = 0x6a09e667u + i;
      CHECK(hipMemcpy(t, &s0, sizeof s0, hipMemcpyHostToDevice));
      hipEvent_t e0, e1;
      CHECK(hipEventCreate(&e0));
      CHECK(hipEventCreate(&e1));
      if (rep >= 3) {  // as in the prove: right after the 2^24-entry streaming pass
        uint32_t nbx = 0;
        CHECK(launch_group_sums_eq(big, 1ull << 24, 6, bigH, bigH, 12, partials, 0, &nbx));
      }
      CHECK(hipEventRecord(e0, 0));
      CHECK(launch_sumcheck_group(partials, nb, 3, 3, 0, 3, prev, t, polys, rs, pts, cdev, 0, CoopCtl{}, kw,
                                  wout));
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipDeviceSynchronize());
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("group kernel launch%s, HIP events: %.1f us\n", rep >= 3 ? " after the streaming pass" : "",
             ms * 1e3);
    }
    if (report("sumcheck_group_kernel (6 rounds)", JT)) return 1;
  }
  // ---- eq tail: a = 12
  {
    const uint32_t a = 12, S0 = 1u << a;
    std::vector<fe> hm(S0), he(S0 - 1), hpts(a);
    for (auto& v : hm) v = rand_fe();
    for (auto& v : he) v = rand_fe();
    for (auto& v : hpts) v = rand_fe();
    fe *m, *e, *pts, *cdev, *prev, *polys, *rs, *mout, *dout;
    DevSha* t;
    uint32_t* kw;
    CHECK(hipMalloc(&m, S0 * sizeof(fe)));
    CHECK(hipMalloc(&e, S0 * sizeof(fe)));
    CHECK(hipMalloc(&pts, a * sizeof(fe)));
    CHECK(hipMalloc(&cdev, sizeof(fe)));
    CHECK(hipMalloc(&prev, sizeof(fe)));
    CHECK(hipMalloc(&polys, 2 * a * sizeof(fe)));
    CHECK(hipMalloc(&rs, a * sizeof(fe)));
    CHECK(hipMalloc(&mout, sizeof(fe)));
    CHECK(hipMalloc(&dout, sizeof(fe)));
    CHECK(hipMalloc(&t, sizeof(DevSha)));
    CHECK(hipMalloc(&kw, 64 * a * 4));
    std::vector<uint32_t> hkw(64 * a, 0);
    for (uint32_t k = 0; k < a; ++k)
      if ((32 * (k + 1)) % 64 == 0) pad_kw(32 * (k + 1), hkw.data() + 64 * k);
    CHECK(hipMemcpy(kw, hkw.data(), hkw.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(m, hm.data(), S0 * sizeof(fe), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(e, he.data(), (S0 - 1) * sizeof(fe), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(pts, hpts.data(), a * sizeof(fe), hipMemcpyHostToDevice));
    // FLUSH=1: stream 1 GiB through the L2s before each launch (as the folds
    // before the tail launch of a prove do), so the kernel's code comes from HBM
    const char* fl = getenv("FLUSH");
    void* junk = nullptr;
    if (fl && *fl == '1') CHECK(hipMalloc(&junk, 1ull << 30));
    for (int rep = 0; rep < 5; ++rep) {
      if (junk) CHECK(hipMemsetAsync(junk, rep, 1ull << 30, 0));
      const fe one{{1, 0, 0, 0}}, cl = rand_fe();
      CHECK(hipMemcpy(cdev, &one, sizeof(fe), hipMemcpyHostToDevice));
      CHECK(hipMemcpy(prev, &cl, sizeof(fe), hipMemcpyHostToDevice));
      DevSha s0{};
      for (int i = 0; i < 8; ++i) s0.h[i] = 0x6a09e667u + i;
      CHECK(hipMemcpy(t, &s0, sizeof s0, hipMemcpyHostToDevice));
      hipEvent_t e0, e1;
      CHECK(hipEventCreate(&e0));
      CHECK(hipEventCreate(&e1));
      CHECK(hipEventRecord(e0, 0));
      CHECK(launch_sumcheck_eq_tail(m, 0, nullptr, a, e, pts, cdev, prev, t, polys, rs, mout, dout, 0, CoopCtl{},
                                    kw));
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipDeviceSynchronize());
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 4) printf("eq tail launch, HIP events: %.1f us\n", ms * 1e3);
    }
    if (report("sumcheck_eq_tail_kernel (12 rounds)", a)) return 1;
  }
  return 0;
}
