// Dev tool: throughput of the generated relaxed butterflies (bfly_asm.hpp) vs
// the canonical C++ butterfly (fe_mul_pre_r + fe_add + fe_sub), register-
// resident, no memory traffic in the loop; plus a per-lane equality check of
// the two on random data (results compared after canonicalisation).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../multilinear_amd/csrc/bfly_asm.hpp"
using namespace mlh;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);             \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

__global__ void __launch_bounds__(256) k_old(const fe* __restrict__ in, const fe* __restrict__ tw,
                                             fe* __restrict__ out, int iters) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  fe x[8];
  for (int e = 0; e < 8; ++e) x[e] = fe_load(in + ((g * 8 + e) & 4095));
  const fe* B = tw + 8 * (threadIdx.x & 7);
  const fe b0 = fe_load(B), b1 = fe_load(B + 1), b2 = fe_load(B + 2), b3 = fe_load(B + 3);
  const fe c0 = fe_load(B + 4), c1 = fe_load(B + 5), c2 = fe_load(B + 6), c3 = fe_load(B + 7);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const fe v = (e & 2) ? fe_mul_pre_r(x[e + 1], c0, c1, c2, c3) : fe_mul_pre_r(x[e + 1], b0, b1, b2, b3);
      const fe u = x[e];
      x[e] = fe_add(u, v);
      x[e + 1] = fe_sub(u, v);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const fe t = x[e];
      x[e] = x[e + 4];
      x[e + 4] = t;
    }
  }
  for (int e = 0; e < 8; ++e) fe_store(out + g * 8 + e, x[e]);
}

__global__ void __launch_bounds__(256) k_new(const fe* __restrict__ in, const fe* __restrict__ tw,
                                             fe* __restrict__ out, int iters) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  fe x[8];
  for (int e = 0; e < 8; ++e) x[e] = fe_load(in + ((g * 8 + e) & 4095));
  const fe* B = tw + 8 * (threadIdx.x & 7);
  const fe b0 = fe_load(B), b1 = fe_load(B + 1), b2 = fe_load(B + 2), b3 = fe_load(B + 3);
  const fe c0 = fe_load(B + 4), c1 = fe_load(B + 5), c2 = fe_load(B + 6), c3 = fe_load(B + 7);
  for (int it = 0; it < iters; ++it) {
    uint64_t r0, r1;
    bfly_mm_v(x[0], x[1], b0, b1, b2, b3, x[2], x[3], c0, c1, c2, c3, r0);
    bfly_mm_v(x[4], x[5], b0, b1, b2, b3, x[6], x[7], c0, c1, c2, c3, r1);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const fe t = x[e];
      x[e] = x[e + 4];
      x[e + 4] = t;
    }
  }
  for (int e = 0; e < 8; ++e) fe_store(out + g * 8 + e, relaxed_canon(x[e]));
}

// one butterfly per lane, arbitrary (u, v, w) with w's expanded multiples given
__global__ void k_check(const fe* __restrict__ u, const fe* __restrict__ v, const fe* __restrict__ Bx,
                        uint32_t* __restrict__ bad, uint64_t n, int variant) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe a = u[i], d = v[i];
  const fe B0 = Bx[4 * i], B1 = Bx[4 * i + 1], B2 = Bx[4 * i + 2], B3 = Bx[4 * i + 3];
  const fe p = fe_mul_pre_r(canon_with_carry(d, 0u), B0, B1, B2, B3);
  const fe uc = canon_with_carry(a, 0u);
  const fe wa = fe_add(uc, p), wd = fe_sub(uc, p);
  uint64_t rare;
  if (variant == 0) {
    bfly_m_v(a, d, B0, B1, B2, B3, rare);
  } else {
    fe a2 = a, d2 = d;
    bfly_mm_v(a, d, B0, B1, B2, B3, a2, d2, B0, B1, B2, B3, rare);
    if (!fe_eq(relaxed_canon(a2), wa) || !fe_eq(relaxed_canon(d2), wd)) atomicAdd(bad, 1u);
  }
  if (!fe_eq(relaxed_canon(a), wa) || !fe_eq(relaxed_canon(d), wd)) atomicAdd(bad, 1u);
}

__global__ void k_expand(fe* bx, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe w = bx[4 * i];
  for (int k = 1; k < 4; ++k) {
    w = fe_mul(w, fe{{0u, 1u, 0u, 0u}});
    bx[4 * i + k] = w;
  }
}

static uint64_t sm = 0x5EED;
static uint64_t next() {
  uint64_t z = (sm += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main() {
  // --- correctness on random relaxed inputs, twiddles = powers of a 2^9 root
  const uint64_t n = 1 << 22;
  fe* u = (fe*)malloc(n * sizeof(fe));
  fe* v = (fe*)malloc(n * sizeof(fe));
  fe* bx = (fe*)malloc(4 * n * sizeof(fe));
  fe *du, *dv, *dbx;
  uint32_t* dbad;
  CHECK(hipMalloc(&du, n * sizeof(fe)));
  CHECK(hipMalloc(&dv, n * sizeof(fe)));
  CHECK(hipMalloc(&dbx, 4 * n * sizeof(fe)));
  CHECK(hipMalloc(&dbad, 4));
  // expanded twiddles: host computes nothing modular -- use the device's fe ops
  // on a small table built from random canonical w < 2^127 (limbs ok)
  for (uint64_t i = 0; i < n; ++i) {
    for (int k = 0; k < 4; ++k) {
      u[i].w[k] = (uint32_t)next();
      v[i].w[k] = (uint32_t)next();
    }
    if ((i & 15) == 0) for (int k = 0; k < 4; ++k) u[i].w[k] = 0xFFFFFFFFu;
    if ((i & 15) == 1) for (int k = 0; k < 4; ++k) v[i].w[k] = 0xFFFFFFFFu;
    if ((i & 15) == 2) for (int k = 0; k < 4; ++k) u[i].w[k] = 0u;
    // w < 2^96 with small top limbs: B_k computed on the device below
    fe w{{(uint32_t)next(), (uint32_t)next() & 0xFFFFFFF0u, (uint32_t)(next() & 0x7FFFFFFF), 0u}};
    if ((i & 15) == 3) w = fe{{2u, 0u, 0u, 0u}};  // with v = 2^128-1 below: product wraps (flag K)
    if ((i & 15) == 3) for (int k = 0; k < 4; ++k) v[i].w[k] = 0xFFFFFFFFu;
    bx[4 * i] = w;
  }
  // B_k = w * 2^(32k) mod M on the host via 128-bit shifts by hand: do it on device
  // with a tiny kernel-free trick: fe_mul is __device__ only, so launch a lambda kernel
  CHECK(hipMemcpy(du, u, n * sizeof(fe), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dv, v, n * sizeof(fe), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dbx, bx, 4 * n * sizeof(fe), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_expand, dim3((unsigned)(n / 256)), dim3(256), 0, 0, dbx, n);
  for (int variant = 0; variant < 2; ++variant) {
    uint32_t bad = 0;
    CHECK(hipMemcpy(dbad, &bad, 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_check, dim3((unsigned)(n / 256)), dim3(256), 0, 0, du, dv, dbx, dbad, n, variant);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
    printf("check variant %d: %u mismatches of %llu\n", variant, bad, (unsigned long long)n);
  }

  // --- throughput
  const int blocks = 256 * 8 * 4, threads = 256, iters = 256;
  fe *in, *tw, *out;
  CHECK(hipMalloc(&in, 4096 * sizeof(fe)));
  CHECK(hipMalloc(&tw, 64 * sizeof(fe)));
  CHECK(hipMalloc(&out, (size_t)blocks * threads * 8 * sizeof(fe)));
  CHECK(hipMemcpy(in, du, 4096 * sizeof(fe), hipMemcpyDefault));
  CHECK(hipMemcpy(tw, dbx, 64 * sizeof(fe), hipMemcpyDefault));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    for (int which = 0; which < 2; ++which) {
      CHECK(hipEventRecord(e0));
      if (which == 0)
        hipLaunchKernelGGL(k_old, dim3(blocks), dim3(threads), 0, 0, in, tw, out, iters);
      else
        hipLaunchKernelGGL(k_new, dim3(blocks), dim3(threads), 0, 0, in, tw, out, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double bfly = (double)blocks * threads * iters * 4;
      printf("%s: %.3f ms  %.3e butterflies/s\n", which ? "new (asm relaxed)" : "old (C canonical)", ms,
             bfly / (ms * 1e-3));
    }
  }
  return 0;
}
