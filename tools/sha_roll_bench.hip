// SHA-256 code size vs speed (dev tool): the Merkle level kernels with the
// 64 rounds fully unrolled (merkle.hip, ~7k-13k instructions per kernel)
// against the same kernels with the rounds rolled in blocks of 16 (round
// constants from a scalar-loaded table): instruction-cache misses or not.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "../multilinear_amd/csrc/field.hpp"
#include "../multilinear_amd/csrc/sha256.hpp"
using namespace mlh;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__constant__ uint32_t cK[64] = MLH_SHA_K;
__constant__ uint32_t cKW[64];

#define SHA_ROUND(kw)                                               \
  do {                                                              \
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); \
    const uint32_t ch = (e & f) ^ (~e & g);                         \
    const uint32_t t1 = h + S1 + ch + (kw);                         \
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); \
    const uint32_t mj = maj3(a, b, c);                              \
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a;           \
    a = t1 + S0 + mj;                                               \
  } while (0)

template <int BLK>
__device__ __forceinline__ void compress_r(Sha256State& st, uint32_t w[16]) {
  constexpr uint32_t K[64] = MLH_SHA_K;
  uint32_t a = st.h[0], b = st.h[1], c = st.h[2], d = st.h[3];
  uint32_t e = st.h[4], f = st.h[5], g = st.h[6], h = st.h[7];
#pragma unroll
  for (int t = 0; t < 16; ++t) SHA_ROUND(K[t] + w[t]);
#pragma unroll 1
  for (int blk = 1; blk < 4; ++blk) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      w[i] = w[i] + s0 + w[(i + 9) & 15] + s1;
      SHA_ROUND(cK[blk * 16 + i] + w[i]);
    }
  }
  st.h[0] += a; st.h[1] += b; st.h[2] += c; st.h[3] += d;
  st.h[4] += e; st.h[5] += f; st.h[6] += g; st.h[7] += h;
}
__device__ __forceinline__ void pad_r(Sha256State& st) {
  uint32_t a = st.h[0], b = st.h[1], c = st.h[2], d = st.h[3];
  uint32_t e = st.h[4], f = st.h[5], g = st.h[6], h = st.h[7];
#pragma unroll 1
  for (int blk = 0; blk < 4; ++blk) {
#pragma unroll
    for (int i = 0; i < 16; ++i) SHA_ROUND(cKW[blk * 16 + i]);
  }
  st.h[0] += a; st.h[1] += b; st.h[2] += c; st.h[3] += d;
  st.h[4] += e; st.h[5] += f; st.h[6] += g; st.h[7] += h;
}
__device__ __forceinline__ Sha256State node_r(const Sha256State& l, const Sha256State& r) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { w[i] = l.h[i]; w[8 + i] = r.h[i]; }
  Sha256State st = sha256_iv();
  compress_r<16>(st, w);
  pad_r(st);
  return st;
}
__device__ __forceinline__ Sha256State msg32_r(const uint32_t m[8]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = m[i];
  w[8] = 0x80000000u;
#pragma unroll
  for (int i = 9; i < 15; ++i) w[i] = 0;
  w[15] = 256u;
  Sha256State st = sha256_iv();
  compress_r<16>(st, w);
  return st;
}

template <bool ROLL>
__global__ void __launch_bounds__(256) lvl2(const uint8_t* __restrict__ child, uint8_t* __restrict__ parent,
                                            uint8_t* __restrict__ grand, uint64_t ngrand) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ngrand) return;
  const uint8_t* c = child + j * 128;
  const Sha256State c0 = digest_load(c), c1 = digest_load(c + 32);
  const Sha256State p0 = ROLL ? node_r(c0, c1) : sha256_node(c0, c1);
  digest_store(parent + (2 * j) * 32, p0);
  const Sha256State c2 = digest_load(c + 64), c3 = digest_load(c + 96);
  const Sha256State p1 = ROLL ? node_r(c2, c3) : sha256_node(c2, c3);
  digest_store(parent + (2 * j + 1) * 32, p1);
  digest_store(grand + j * 32, ROLL ? node_r(p0, p1) : sha256_node(p0, p1));
}

template <bool ROLL>
__global__ void __launch_bounds__(256) leaves2(const fe* __restrict__ code, uint64_t half, uint8_t* __restrict__ layers) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= half / 4) return;
  Sha256State lf[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint64_t i = 4 * j + q;
    const fe a = fe_load(code + i), b = fe_load(code + i + half);
    uint32_t m[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) { m[k] = bswap32(a.w[k]); m[4 + k] = bswap32(b.w[k]); }
    lf[q] = ROLL ? msg32_r(m) : sha256_msg32(m);
    digest_store(layers + i * 32, lf[q]);
  }
  const Sha256State p0 = ROLL ? node_r(lf[0], lf[1]) : sha256_node(lf[0], lf[1]);
  const Sha256State p1 = ROLL ? node_r(lf[2], lf[3]) : sha256_node(lf[2], lf[3]);
  digest_store(layers + (half + 2 * j) * 32, p0);
  digest_store(layers + (half + 2 * j + 1) * 32, p1);
  digest_store(layers + (half + half / 2 + j) * 32, ROLL ? node_r(p0, p1) : sha256_node(p0, p1));
}

template <class F>
float timeit(F f, hipEvent_t a, hipEvent_t b) {
  float best = 1e30f;
  for (int r = 0; r < 7; ++r) {
    (void)hipEventRecord(a, 0);
    f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (r && ms < best) best = ms;
  }
  return best;
}

int main() {
  {
    Pad64KW kw;
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(cKW), kw.v, sizeof(kw.v)));
  }
  hipEvent_t ea, eb;
  CHECK(hipEventCreate(&ea));
  CHECK(hipEventCreate(&eb));
  // level2 over 2^22 child digests
  const uint64_t nch = 1ull << 22, ng = nch / 4;
  uint8_t *child, *par[2], *gr[2];
  CHECK(hipMalloc(&child, nch * 32));
  std::vector<uint8_t> h(nch * 32);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)((i * 2654435761u) >> 11);
  CHECK(hipMemcpy(child, h.data(), h.size(), hipMemcpyHostToDevice));
  for (int v = 0; v < 2; ++v) {
    CHECK(hipMalloc(&par[v], nch / 2 * 32));
    CHECK(hipMalloc(&gr[v], ng * 32));
  }
  const unsigned blocks = (unsigned)(ng / 256);
  float t0 = timeit([&] { hipLaunchKernelGGL(lvl2<false>, dim3(blocks), dim3(256), 0, 0, child, par[0], gr[0], ng); }, ea, eb);
  float t1 = timeit([&] { hipLaunchKernelGGL(lvl2<true>, dim3(blocks), dim3(256), 0, 0, child, par[1], gr[1], ng); }, ea, eb);
  std::vector<uint8_t> g0(ng * 32), g1(ng * 32);
  CHECK(hipMemcpy(g0.data(), gr[0], g0.size(), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(g1.data(), gr[1], g1.size(), hipMemcpyDeviceToHost));
  printf("{\"kernel\": \"level2 (2^22 digests)\", \"unrolled_ms\": %.4f, \"rolled_ms\": %.4f, \"equal\": %d}\n", t0, t1,
         (int)(g0 == g1));
  // leaf_pairs_level2 over a code of 2^23 (2^22 leaves)
  const uint64_t half = 1ull << 22;
  fe* code;
  uint8_t* lay[2];
  CHECK(hipMalloc(&code, 2 * half * sizeof(fe)));
  CHECK(hipMemcpy(code, h.data(), 2 * half * sizeof(fe) <= h.size() ? 2 * half * sizeof(fe) : h.size(), hipMemcpyHostToDevice));
  for (int v = 0; v < 2; ++v) CHECK(hipMalloc(&lay[v], 2 * half * 32));
  const unsigned lb = (unsigned)(half / 4 / 256);
  float t2 = timeit([&] { hipLaunchKernelGGL(leaves2<false>, dim3(lb), dim3(256), 0, 0, code, half, lay[0]); }, ea, eb);
  float t3 = timeit([&] { hipLaunchKernelGGL(leaves2<true>, dim3(lb), dim3(256), 0, 0, code, half, lay[1]); }, ea, eb);
  std::vector<uint8_t> l0(2 * half * 32), l1(2 * half * 32);
  CHECK(hipMemcpy(l0.data(), lay[0], (half + half / 2 + half / 4) * 32, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(l1.data(), lay[1], (half + half / 2 + half / 4) * 32, hipMemcpyDeviceToHost));
  printf("{\"kernel\": \"leaf_pairs_level2 (2^22 leaves)\", \"unrolled_ms\": %.4f, \"rolled_ms\": %.4f, \"equal\": %d}\n",
         t2, t3, (int)(memcmp(l0.data(), l1.data(), (half + half / 2 + half / 4) * 32) == 0));
  return 0;
}
