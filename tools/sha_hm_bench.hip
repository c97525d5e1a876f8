// Tree-tail node hash on ONE wave (dev tool): the lane-pair SHA-256
// (sha2l_node: lanes 2i / 2i+1, quad_perm swap, the new-e/new-a select on the
// round's dependency chain) against a half-mirror layout (lanes j and 7 - j of
// each 8-lane half row, row_half_mirror DPP):
//   e-side lanes (banks 0, 2) hold e f g h, a-side lanes (banks 1, 3) a b c d;
//   x = h + K + W + d on the e side, -d on the a side, so that
//   u = Sigma + Ch|Maj + x is e' = T1 + d on the e side and T2 - d on the a
//   side, and ONE bank-masked DPP add writes a' = u_e + u_a on the a side
//   while the e side keeps u: the chain per round is alignbit, xor3, add3,
//   dpp-add (the lane-pair form also has the select).  The next round's x
//   is off the chain: n = -r2 (all lanes), then a bank-masked DPP add writes
//   r2(partner) + r2 + KW on the e side.
// Checks that both layouts give the same digests, then times a dependent
// chain of node hashes (s_memtime cycles).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/sha_hm_bench.hip -o tools/bin/sha_hm_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../multilinear_amd/csrc/sha256.hpp"
#include "../multilinear_amd/csrc/transcript_dev.hpp"
using namespace mlh;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kHalfMirror = 0x141;

struct ShaH {
  uint32_t r0, r1, r2, r3;  // e side: e f g h; a side: a b c d
  uint32_t m;               // a side ~0, e side 0
  uint32_t s1, s2, s3;
};
__device__ __forceinline__ bool hm_aside() { return (__lane_id() >> 2) & 1u; }
__device__ __forceinline__ void shah_init(ShaH& q, const uint32_t (&v)[8]) {
  const bool a = hm_aside();
  q.m = a ? ~0u : 0u;
  asm("" : "+v"(q.m));
  q.r0 = a ? v[0] : v[4];
  q.r1 = a ? v[1] : v[5];
  q.r2 = a ? v[2] : v[6];
  q.r3 = a ? v[3] : v[7];
  q.s1 = a ? 2u : 6u;
  q.s2 = a ? 13u : 11u;
  q.s3 = a ? 22u : 25u;
}
// e side: partner's value + y; a side: keeps old.  (old = y's register)
__device__ __forceinline__ uint32_t dpp_add_eside(uint32_t old_y, uint32_t src, uint32_t y) {
  uint32_t r = old_y;
  asm("v_add_u32_dpp %0, %1, %2 row_half_mirror row_mask:0xf bank_mask:0x5"
               : "+v"(r) : "v"(src), "v"(y));
  return r;
}
template <int T0, int T1, class KWF>
__device__ __forceinline__ void shah_rounds(ShaH& q, KWF&& kwf) {
  // x for round T0: e side h + KW + d (d = the partner's r3), a side -d
  uint32_t x;
  {
    const uint32_t n = 0u - q.r3;
    const uint32_t hk = q.r3 + kwf(T0);
    const uint32_t dp = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r3, kHalfMirror, 0xF, 0xF, false);
    x = q.m ? n : hk + dp;
  }
#pragma unroll
  for (int t = T0; t < T1; ++t) {
    const uint32_t sg = xor3(__builtin_amdgcn_alignbit(q.r0, q.r0, q.s1),
                             __builtin_amdgcn_alignbit(q.r0, q.r0, q.s2),
                             __builtin_amdgcn_alignbit(q.r0, q.r0, q.s3));
    const uint32_t p = q.r0 ^ (q.r2 & q.m);       // e | a ^ c
    const uint32_t f = (p & q.r1) | (~p & q.r2);  // Ch | Maj
    const uint32_t u = sg + f + x;                // e' | T2 - d
    uint32_t xn = 0;
    if (t + 1 < T1) {  // the next round's x (r2 becomes r3)
      const uint32_t hk = q.r2 + kwf(t + 1);
      xn = dpp_add_eside(0u - q.r2, q.r2, hk);
    }
    q.r3 = q.r2;
    q.r2 = q.r1;
    q.r1 = q.r0;
    // a side: u_e (partner) + u_a; e side keeps u (bank mask, old = 0 identity)
    q.r0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, kHalfMirror, 0xF, 0xA, false) + u;
    x = xn;
  }
}
__device__ __forceinline__ uint32_t shah_sched(uint32_t* w, int t, const Sched2L& c) {
  const uint32_t x = (w[(t - 2) & 15] & c.m) | (w[(t - 15) & 15] & ~c.m);
  const uint32_t sg = xor3(__builtin_amdgcn_alignbit(x, x, c.c1), __builtin_amdgcn_alignbit(x, x, c.c2),
                           x >> c.c3);
  uint32_t both = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sg, kHalfMirror, 0xF, 0xF, true) + sg;
  asm("" : "+v"(both));
  return w[t & 15] = both + w[(t - 7) & 15] + w[t & 15];
}
__device__ __forceinline__ Sched2L schedh_init() {
  const bool a = hm_aside();
  Sched2L c;
  c.m = a ? ~0u : 0u;
  asm("" : "+v"(c.m));
  c.c1 = a ? 17u : 7u;
  c.c2 = a ? 19u : 18u;
  c.c3 = a ? 10u : 3u;
  return c;
}
__device__ __forceinline__ void shah_state_pair(const ShaH& q, uint32_t (&v)[8]) {
  const bool a = q.m != 0u;
  const uint32_t o0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r0, kHalfMirror, 0xF, 0xF, true);
  const uint32_t o1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r1, kHalfMirror, 0xF, 0xF, true);
  const uint32_t o2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r2, kHalfMirror, 0xF, 0xF, true);
  const uint32_t o3 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r3, kHalfMirror, 0xF, 0xF, true);
  v[0] = a ? q.r0 : o0;
  v[1] = a ? q.r1 : o1;
  v[2] = a ? q.r2 : o2;
  v[3] = a ? q.r3 : o3;
  v[4] = a ? o0 : q.r0;
  v[5] = a ? o1 : q.r1;
  v[6] = a ? o2 : q.r2;
  v[7] = a ? o3 : q.r3;
}
__device__ __forceinline__ Sha256State shah_node(const Sha256State& l, const Sha256State& r) {
  constexpr uint32_t K[64] = MLH_SHA_K;
  constexpr Pad64KW KW;
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    w[i] = l.h[i];
    w[8 + i] = r.h[i];
  }
  const Sha256State iv = sha256_iv();
  ShaH q;
  shah_init(q, iv.h);
  const Sched2L sc = schedh_init();
  shah_rounds<0, 64>(q, [&](int t) -> uint32_t {
    if (t >= 16) shah_sched(w, t, sc);
    return K[t] + w[t & 15];
  });
  uint32_t v[8], h1[8];
  shah_state_pair(q, v);
#pragma unroll
  for (int i = 0; i < 8; ++i) h1[i] = iv.h[i] + v[i];
  shah_init(q, h1);
  shah_rounds<0, 64>(q, [&](int t) -> uint32_t { return KW.v[t]; });
  shah_state_pair(q, v);
  Sha256State o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o.h[i] = h1[i] + v[i];
  return o;
}

// MODE 1: lane pairs (node = lane >> 1), MODE 3: half mirror (node = lane & 3 | (lane >> 3) << 2)
template <int MODE>
__global__ void __launch_bounds__(64) chain(int iters, uint32_t* out, unsigned long long* clk) {
  const uint32_t lane = threadIdx.x;
  const uint32_t id = MODE == 1 ? lane >> 1 : ((lane & 3) | ((lane >> 3) << 2));
  const bool lead = MODE == 1 ? (lane & 1) == 0 : ((lane >> 2) & 1) == 0;
  Sha256State a = sha256_iv(), b = sha256_iv();
  a.h[0] ^= id * 977 + 1;
  b.h[3] ^= id * 131 + 7;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    const Sha256State c = MODE == 1 ? sha2l_node(a, b) : shah_node(a, b);
    b = a;
    a = c;
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) clk[0] = c1 - c0;
  if (lead)
    for (int i = 0; i < 8; ++i) out[id * 8 + i] = a.h[i];
}

template <int MODE>
int run(const char* name, int iters, uint32_t* d, unsigned long long* clk, uint32_t* host) {
  hipLaunchKernelGGL(chain<MODE>, dim3(1), dim3(64), 0, 0, iters, d, clk);
  CHECK(hipDeviceSynchronize());
  unsigned long long best = ~0ull;
  for (int r = 0; r < 7; ++r) {
    hipLaunchKernelGGL(chain<MODE>, dim3(1), dim3(64), 0, 0, iters, d, clk);
    CHECK(hipDeviceSynchronize());
    unsigned long long h;
    CHECK(hipMemcpy(&h, clk, 8, hipMemcpyDeviceToHost));
    if (h < best) best = h;
  }
  CHECK(hipMemcpy(host, d, 32 * 8 * 4, hipMemcpyDeviceToHost));
  printf("{\"layout\": \"%s\", \"cycles_per_node\": %.0f}\n", name, (double)best / iters);
  return 0;
}

int main() {
  uint32_t* d;
  unsigned long long* clk;
  CHECK(hipMalloc(&d, 4096));
  CHECK(hipMalloc(&clk, 64));
  static uint32_t h1[256], h3[256];
  const int it = 256;
  if (run<1>("lane pair (quad_perm swap, select on the chain)", it, d, clk, h1)) return 1;
  if (run<3>("half mirror (bank-masked DPP adds)", it, d, clk, h3)) return 1;
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += h1[i] != h3[i];
  printf("{\"digests_equal\": %s, \"mismatched_words\": %d}\n", bad ? "false" : "true", bad);
  return bad ? 2 : 0;
}
