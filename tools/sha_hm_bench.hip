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

// The earlier adjacent-lane layout (lanes 2i / 2i+1, quad_perm swap; the
// library's sha2l_* before the half-mirror layout), kept for the comparison.
namespace adj {
struct Sha2L {
  uint32_t r0, r1, r2, r3;  // even lane: e f g h; odd lane: a b c d
  uint32_t m;               // odd lane ~0, even lane 0
  uint32_t s1, s2, s3;      // the lane's Sigma rotation counts
};
__device__ __forceinline__ void sha2l_init(Sha2L& q, const uint32_t (&v)[8]) {
  const bool odd = __lane_id() & 1u;
  q.m = odd ? ~0u : 0u;
  // opaque to the compiler: p = r0 ^ (r2 & m) stays one v_bitop3 (as a select
  // of constants it lowers to v_cndmask + v_xor)
  asm("" : "+v"(q.m));
  q.r0 = odd ? v[0] : v[4];
  q.r1 = odd ? v[1] : v[5];
  q.r2 = odd ? v[2] : v[6];
  q.r3 = odd ? v[3] : v[7];
  q.s1 = odd ? 2u : 6u;
  q.s2 = odd ? 13u : 11u;
  q.s3 = odd ? 22u : 25u;
}
// The working state a..h, wave-uniform (read from lanes 1 and 0).
__device__ __forceinline__ void sha2l_state(const Sha2L& q, uint32_t (&v)[8]) {
  v[0] = __builtin_amdgcn_readlane(q.r0, 1);
  v[1] = __builtin_amdgcn_readlane(q.r1, 1);
  v[2] = __builtin_amdgcn_readlane(q.r2, 1);
  v[3] = __builtin_amdgcn_readlane(q.r3, 1);
  v[4] = __builtin_amdgcn_readlane(q.r0, 0);
  v[5] = __builtin_amdgcn_readlane(q.r1, 0);
  v[6] = __builtin_amdgcn_readlane(q.r2, 0);
  v[7] = __builtin_amdgcn_readlane(q.r3, 0);
}
// Rounds T0..T1-1; kwf(t) returns K[t] + W[t] (wave-uniform) and is called
// once per t in increasing order (so it may extend the message schedule).
template <int T0, int T1, class KWF>
__device__ __forceinline__ void sha2l_rounds(Sha2L& q, KWF&& kwf) {
  uint32_t x = (q.r3 + kwf(T0)) & ~q.m;  // even lane: h + K + W; odd lane: 0
#pragma unroll
  for (int t = T0; t < T1; ++t) {
    const uint32_t sg = xor3(__builtin_amdgcn_alignbit(q.r0, q.r0, q.s1),
                             __builtin_amdgcn_alignbit(q.r0, q.r0, q.s2),
                             __builtin_amdgcn_alignbit(q.r0, q.r0, q.s3));
    const uint32_t p = q.r0 ^ (q.r2 & q.m);       // e | a ^ c
    const uint32_t f = (p & q.r1) | (~p & q.r2);  // Ch | Maj
    const uint32_t u = sg + f + x;                // T1 | T2
    const uint32_t y = (q.m & q.r3) | (~q.m & u); // T1 | d
    if (t + 1 < T1) x = (q.r2 + kwf(t + 1)) & ~q.m;  // the next round's h + K + W
    q.r3 = q.r2;
    q.r2 = q.r1;
    q.r1 = q.r0;
    // pair swap (quad_perm [1,0,3,2]) folded into the add: d + T1 | T1 + T2
    q.r0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)y, 0xB1, 0xF, 0xF, true) + u;
  }
}
// Message-schedule word t (t >= 16) in place in w[16].
__device__ __forceinline__ uint32_t sha_sched(uint32_t* w, int t) {
  const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
  const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
  const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
  return w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
}

// Message-schedule word t (t >= 16) in place in w[16] on a lane pair whose two
// lanes hold the same w: the even lane computes sigma0(w[t-15]) and the odd
// lane sigma1(w[t-2]) in one instruction stream (per-lane v_alignbit and
// v_lshrrev counts) and one quad_perm DPP add sums them: 7 VALU per word
// instead of the one-lane 10.
struct Sched2L {
  uint32_t m;           // odd lane ~0, even lane 0
  uint32_t c1, c2, c3;  // even: 7, 18, 3 (sigma0); odd: 17, 19, 10 (sigma1)
};
__device__ __forceinline__ Sched2L sched2l_init() {
  const bool odd = __lane_id() & 1u;
  Sched2L c;
  c.m = odd ? ~0u : 0u;
  asm("" : "+v"(c.m));
  c.c1 = odd ? 17u : 7u;
  c.c2 = odd ? 19u : 18u;
  c.c3 = odd ? 10u : 3u;
  return c;
}
__device__ __forceinline__ uint32_t sha2l_sched(uint32_t* w, int t, const Sched2L& c) {
  const uint32_t x = (w[(t - 2) & 15] & c.m) | (w[(t - 15) & 15] & ~c.m);
  const uint32_t sg = xor3(__builtin_amdgcn_alignbit(x, x, c.c1), __builtin_amdgcn_alignbit(x, x, c.c2),
                           x >> c.c3);
  uint32_t both = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sg, 0xB1, 0xF, 0xF, true) + sg;
  asm("" : "+v"(both));  // one v_add_u32_dpp (else: v_mov_dpp + a reassociated add)
  return w[t & 15] = both + w[(t - 7) & 15] + w[t & 15];
}

// The working state a..h of each lane pair, on both lanes of the pair (one
// DPP swap per word), for lane pairs that hash different messages.
__device__ __forceinline__ void sha2l_state_pair(const Sha2L& q, uint32_t (&v)[8]) {
  const bool odd = q.m != 0u;
  const uint32_t o0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r0, 0xB1, 0xF, 0xF, true);
  const uint32_t o1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r1, 0xB1, 0xF, 0xF, true);
  const uint32_t o2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r2, 0xB1, 0xF, 0xF, true);
  const uint32_t o3 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r3, 0xB1, 0xF, 0xF, true);
  v[0] = odd ? q.r0 : o0;
  v[1] = odd ? q.r1 : o1;
  v[2] = odd ? q.r2 : o2;
  v[3] = odd ? q.r3 : o3;
  v[4] = odd ? o0 : q.r0;
  v[5] = odd ? o1 : q.r1;
  v[6] = odd ? o2 : q.r2;
  v[7] = odd ? o3 : q.r3;
}
// sha256_node (SHA-256 of the 64 bytes left || right) on a lane pair: both
// lanes of the pair pass the same children and get the digest (~20 % less
// latency than one lane: the latency-bound tree levels, where lanes idle).
__device__ __forceinline__ Sha256State sha2l_node(const Sha256State& l, const Sha256State& r) {
  constexpr uint32_t K[64] = MLH_SHA_K;
  constexpr Pad64KW KW;
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    w[i] = l.h[i];
    w[8 + i] = r.h[i];
  }
  const Sha256State iv = sha256_iv();
  Sha2L q;
  sha2l_init(q, iv.h);
  const Sched2L sc = sched2l_init();
  sha2l_rounds<0, 64>(q, [&](int t) -> uint32_t {
    if (t >= 16) sha2l_sched(w, t, sc);
    return K[t] + w[t & 15];
  });
  uint32_t v[8], h1[8];
  sha2l_state_pair(q, v);
#pragma unroll
  for (int i = 0; i < 8; ++i) h1[i] = iv.h[i] + v[i];
  sha2l_init(q, h1);
  sha2l_rounds<0, 64>(q, [&](int t) -> uint32_t { return KW.v[t]; });
  sha2l_state_pair(q, v);
  Sha256State o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o.h[i] = h1[i] + v[i];
  return o;
}
}  // namespace adj

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
template <int T0, int T1, bool BT0 = false, class KWF>
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
      if (BT0 && t == T0) {
        const uint32_t c = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r2, kHalfMirror, 0xF, 0xF, false);
        xn = q.m ? 0u - q.r2 : hk + c;
      } else {
        xn = dpp_add_eside(0u - q.r2, q.r2, hk);
      }
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
template <bool BT0 = false>
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
  shah_rounds<0, 64, BT0>(q, [&](int t) -> uint32_t {
    if (t >= 16) shah_sched(w, t, sc);
    return K[t] + w[t & 15];
  });
  uint32_t v[8], h1[8];
  shah_state_pair(q, v);
#pragma unroll
  for (int i = 0; i < 8; ++i) h1[i] = iv.h[i] + v[i];
  shah_init(q, h1);
  shah_rounds<0, 64, BT0>(q, [&](int t) -> uint32_t { return KW.v[t]; });
  shah_state_pair(q, v);
  Sha256State o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o.h[i] = h1[i] + v[i];
  return o;
}

// MODE 1: lane pairs (node = lane >> 1), MODE 3: half mirror (node = 4 (lane >> 3) + min(k, 7 - k), k = lane & 7)
template <int MODE, int ACTIVE = 64>
__global__ void __launch_bounds__(64) chain(int iters, uint32_t* out, unsigned long long* clk) {
  const uint32_t lane = threadIdx.x;
  if (lane >= (uint32_t)ACTIVE) return;  // a partly active wave (the tree tail's small levels)
  const uint32_t hk = lane & 7;  // half mirror: lanes k and 7 - k of a half row share a node
  const uint32_t id = MODE == 1 ? lane >> 1 : (((lane >> 3) << 2) | (hk < 4 ? hk : 7 - hk));
  const bool lead = MODE == 1 ? (lane & 1) == 0 : ((lane >> 2) & 1) == 0;  // MODE 2: the library's (half mirror)
  Sha256State a = sha256_iv(), b = sha256_iv();
  a.h[0] ^= id * 977 + 1;
  b.h[3] ^= id * 131 + 7;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    const Sha256State c = MODE == 1 ? adj::sha2l_node(a, b) : MODE == 2 ? sha2l_node(a, b) : MODE == 4 ? shah_node<true>(a, b) : shah_node(a, b);
    b = a;
    a = c;
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) clk[0] = c1 - c0;
  if (lead)
    for (int i = 0; i < 8; ++i) out[id * 8 + i] = a.h[i];
}

template <int MODE, int ACTIVE = 64>
int run(const char* name, int iters, uint32_t* d, unsigned long long* clk, uint32_t* host) {
  hipLaunchKernelGGL((chain<MODE, ACTIVE>), dim3(1), dim3(64), 0, 0, iters, d, clk);
  CHECK(hipDeviceSynchronize());
  unsigned long long best = ~0ull;
  for (int r = 0; r < 7; ++r) {
    hipLaunchKernelGGL((chain<MODE, ACTIVE>), dim3(1), dim3(64), 0, 0, iters, d, clk);
    CHECK(hipDeviceSynchronize());
    unsigned long long h;
    CHECK(hipMemcpy(&h, clk, 8, hipMemcpyDeviceToHost));
    if (h < best) best = h;
  }
  CHECK(hipMemcpy(host, d, 32 * 8 * 4, hipMemcpyDeviceToHost));
  printf("{\"layout\": \"%s\", \"active_lanes\": %d, \"cycles_per_node\": %.0f}\n", name, ACTIVE,
         (double)best / iters);
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
  static uint32_t h2[256], h4[256];
  if (run<2>("library sha2l_node", it, d, clk, h2)) return 1;
  if (run<4>("half mirror, first round's x through the compiler's DPP", it, d, clk, h4)) return 1;
  static uint32_t hx[256];
  for (int a = 0; a < 3; ++a) {  // partly active waves: 32, 16, 8 lanes
    if (a == 0 && (run<1, 32>("lane pair", it, d, clk, hx) || run<2, 32>("library sha2l_node", it, d, clk, hx))) return 1;
    if (a == 1 && (run<1, 16>("lane pair", it, d, clk, hx) || run<2, 16>("library sha2l_node", it, d, clk, hx))) return 1;
    if (a == 2 && (run<1, 8>("lane pair", it, d, clk, hx) || run<2, 8>("library sha2l_node", it, d, clk, hx))) return 1;
  }
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += (h1[i] != h3[i]) + (h2[i] != h3[i]) + (h4[i] != h3[i]);
  printf("{\"digests_equal\": %s, \"mismatched_words\": %d}\n", bad ? "false" : "true", bad);
  return bad ? 2 : 0;
}
