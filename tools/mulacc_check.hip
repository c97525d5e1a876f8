// Dev check: lazy multiply-accumulate (sumcheck.hip mulacc / acc_reduce) vs
// reduced products summed with fe_add, on random and extreme operands.
#include "../multilinear_amd/csrc/sumcheck.hip"
#include <stdio.h>
#include <vector>
using namespace mlh;
__global__ void chk(const fe* a, const fe* b, int n, uint32_t* bad) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  acc9 s;
  acc_zero(s);
  acccol sc;
  acccol_zero(sc);
  fe ref = fe_zero();
  for (int k = 0; k < n; ++k) {
    const fe x = a[t * n + k], y = b[t * n + k];
    mulacc(s, x, y);
    mulacc_col(sc, x, y);
    ref = fe_add(ref, fe_mul(x, y));
  }
  const fe got = acc_reduce(s);
  if (!fe_eq(got, ref)) atomicAdd(bad, 1u);
  if (!fe_eq(acc_reduce(acccol_limbs(sc)), ref)) atomicAdd(bad + 1, 1u);
}
int main() {
  const uint64_t M0 = 1, M1 = 0xFFFFD300ull;
  for (int n : {1, 2, 3, 16, 64, 300}) {
    const int T = 4096;
    std::vector<fe> ha(T * n), hb(T * n);
    uint64_t x = 0x9E3779B97F4A7C15ull + n;
    auto next = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (uint32_t)x; };
    for (int i = 0; i < T * n; ++i) {
      const int mode = i % 4;
      if (mode == 0) ha[i] = fe{{(uint32_t)M0 - 1 + 0xFFFFFFFFu, (uint32_t)M1, 0xFFFFFFFFu, 0xFFFFFFFFu}};  // M - 1 - ...
      else ha[i] = fe{{next(), next(), next(), next() >> 1}};
      if (i % 7 == 0) ha[i] = fe{{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}};  // relaxed 2^128-1
      hb[i] = (i % 5 == 0) ? fe{{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}} : (i % 3 == 0) ? fe{{0u, (uint32_t)M1, 0xFFFFFFFFu, 0xFFFFFFFFu}} : fe{{next(), next(), next(), next() >> 1}};
    }
    fe *da, *db; uint32_t* bad;
    hipMalloc(&da, sizeof(fe) * T * n); hipMalloc(&db, sizeof(fe) * T * n); hipMalloc(&bad, 8);
    hipMemcpy(da, ha.data(), sizeof(fe) * T * n, hipMemcpyHostToDevice);
    hipMemcpy(db, hb.data(), sizeof(fe) * T * n, hipMemcpyHostToDevice);
    hipMemset(bad, 0, 8);
    hipLaunchKernelGGL(chk, dim3(T / 256), dim3(256), 0, 0, da, db, n, bad);
    uint32_t hbad[2] = {0, 0};
    hipMemcpy(hbad, bad, 8, hipMemcpyDeviceToHost);
    printf("n=%d mismatches acc9 %u acccol %u / %d\n", n, hbad[0], hbad[1], T);
  }
  return 0;
}
