// Device-side Fiat-Shamir transcript (one lane): the same SHA-256 state
// machine as HostSha256 (src/transcript.rs semantics: absorb = update,
// random = digest of a clone, next_challenge = F::from(u128_le(random[..16]))).
// Lets the FRI / PCS commit loops derive each round's challenge on the GPU
// from the root just written to HBM, so the loop never waits on the host; the
// host transcript is brought to the same state afterwards by replaying the
// same absorbs (it is a pure function of the absorbed bytes).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.hpp"
#include "sha256.hpp"

namespace mlh {

// Byte-identical layout to HostSha256 {h[8], buf[64], len}.
struct DevSha {
  uint32_t h[8];
  uint8_t buf[64];
  uint64_t len;
};

// The transcript runs on one lane with wave-uniform data; left to itself the
// compiler splits each round between the SALU (adds) and the VALU (v_alignbit,
// v_bitop3: no scalar forms) with a v_readfirstlane per crossing, which halves
// the speed of this latency-bound chain (tools/dsha_bench.hip: 8.1 vs 4.3 us
// per node hash).  Pinning the compression's inputs to VGPRs keeps it on the
// VALU.
__device__ __forceinline__ void pin_vgpr(uint32_t& x) { asm volatile("" : "+v"(x)); }

__device__ __forceinline__ void sha256_compress_valu(Sha256State& st, uint32_t w[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) pin_vgpr(w[i]);
#pragma unroll
  for (int i = 0; i < 8; ++i) pin_vgpr(st.h[i]);
  sha256_compress(st, w);
}

__device__ inline void dsha_compress_buf(DevSha& s) {
  uint32_t w[16];
  const uint32_t* bw = reinterpret_cast<const uint32_t*>(s.buf);
  for (int i = 0; i < 16; ++i) w[i] = bswap32(bw[i]);  // big-endian words
  Sha256State st;
  for (int i = 0; i < 8; ++i) st.h[i] = s.h[i];
  sha256_compress_valu(st, w);
  for (int i = 0; i < 8; ++i) s.h[i] = st.h[i];
}

// Word path when the fill and the length are multiples of 4 and p is
// 4-byte aligned (every device absorb: roots, field elements); bytes
// otherwise.  buf keeps memory byte order, exactly as HostSha256.  Out of
// line: the one-lane transcript kernels are instruction-fetch bound, and
// unrolled copies of this rare path would evict the compression code.
__device__ __noinline__ void dsha_update(DevSha& s, const uint8_t* p, uint32_t n) {
  if (((s.len | n | reinterpret_cast<uintptr_t>(p)) & 3) == 0) {
    uint32_t* bw = reinterpret_cast<uint32_t*>(s.buf);
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(p);
    for (uint32_t i = 0; i < n / 4; ++i) {
      bw[(s.len % 64) / 4] = pw[i];
      s.len += 4;
      if (s.len % 64 == 0) dsha_compress_buf(s);
    }
    return;
  }
  for (uint32_t i = 0; i < n; ++i) {
    s.buf[s.len % 64] = p[i];
    s.len += 1;
    if (s.len % 64 == 0) dsha_compress_buf(s);
  }
}

// Absorb N words held in registers (memory byte order: the bytes as stored),
// for a state with len % 4 == 0: at most one compression (N <= 16), no
// loads from the source.  dsha_update on a global source costs a dependent
// global load per word; on a register array with a byte fallback the array
// lands in scratch.
template <int N>
__device__ inline void dsha_absorb_words(DevSha& s, const uint32_t (&w)[N]) {
  static_assert(N >= 1 && N <= 16, "at most one block per call");
  uint32_t* bw = reinterpret_cast<uint32_t*>(s.buf);
  const uint32_t pos = (uint32_t)(s.len % 64) / 4;
  const uint32_t first = 16 - pos < (uint32_t)N ? 16 - pos : (uint32_t)N;
#pragma unroll
  for (int i = 0; i < N; ++i)
    if ((uint32_t)i < first) bw[pos + i] = w[i];
  if (pos + N >= 16) {
    dsha_compress_buf(s);
#pragma unroll
    for (int i = 0; i < N; ++i)
      if ((uint32_t)i >= first) bw[i - first] = w[i];
  }
  s.len += 4 * N;
}

// absorb N words (registers); a state whose length is not a multiple of 4
// (bytes absorbed on the host before the device loop) goes bytewise through
// the LDS staging area `stage` (>= N words)
template <int N>
__device__ inline void dsha_absorb(DevSha& s, const uint32_t (&w)[N], uint32_t* stage) {
  if ((s.len & 3) == 0) {
    dsha_absorb_words<N>(s, w);
    return;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) stage[i] = w[i];
  dsha_update(s, reinterpret_cast<const uint8_t*>(stage), 4 * N);
}

// Final state words of a clone (the state itself is unchanged; at most two
// compressions).  Digest byte 4i+j is byte (3 - j) of h[i] (big-endian words).
__device__ inline void dsha_final(const DevSha& s0, uint32_t h[8]) {
  const uint64_t bits = s0.len * 8;
  if ((s0.len & 3) == 0) {
    // word fill (every device absorb): the padded block(s) are built in
    // registers straight from the buffer words -- no copy of the state
    const uint32_t* bw = reinterpret_cast<const uint32_t*>(s0.buf);
    const uint32_t pos = (uint32_t)(s0.len % 64) / 4;
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t b = bw[i];
      w[i] = (uint32_t)i < pos ? bswap32(b) : ((uint32_t)i == pos ? 0x80000000u : 0u);
    }
    Sha256State st;
#pragma unroll
    for (int i = 0; i < 8; ++i) st.h[i] = s0.h[i];
    if (pos >= 14) {  // no room for the length: 0x80 block, then a zero block
      sha256_compress_valu(st, w);
#pragma unroll
      for (int i = 0; i < 14; ++i) w[i] = 0;
    }
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
    sha256_compress_valu(st, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = st.h[i];
    return;
  }
  __shared__ DevSha c;
  c = s0;
  {
    const uint8_t one = 0x80, z = 0;
    dsha_update(c, &one, 1);
    while (c.len % 64 != 56) dsha_update(c, &z, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
    dsha_update(c, lb, 8);
  }
  for (int i = 0; i < 8; ++i) h[i] = c.h[i];
}

__device__ inline void dsha_digest(const DevSha& s0, uint8_t out[32]) {
  uint32_t h[8];
  dsha_final(s0, h);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(h[i] >> 8);
    out[4 * i + 3] = (uint8_t)h[i];
  }
}

// K[t] + W[t] of the padding-only final block of a message of `len` bytes
// (len % 64 == 0: 0x80, zeros, the bit length): the schedule depends on len
// alone, so the transcript's challenge after a block-completing absorb can run
// the round function only (sha256_compress_kw).
__device__ inline void sha256_pad_kw(uint64_t len, uint32_t* kw) {
  constexpr uint32_t K[64] = MLH_SHA_K;
  uint32_t w[16] = {};
  w[0] = 0x80000000u;
  w[14] = (uint32_t)((len * 8) >> 32);
  w[15] = (uint32_t)(len * 8);
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    uint32_t x;
    if (t < 16) {
      x = w[t];
    } else {
      const uint32_t a = w[(t - 15) & 15], b = w[(t - 2) & 15];
      const uint32_t s0 = rotr(a, 7) ^ rotr(a, 18) ^ (a >> 3);
      const uint32_t s1 = rotr(b, 17) ^ rotr(b, 19) ^ (b >> 10);
      x = w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
    }
    kw[t] = K[t] + x;
  }
}

// One compression whose K[t] + W[t] come precomputed (a constant block).
__device__ __forceinline__ void sha256_compress_kw(Sha256State& st, const uint32_t* __restrict__ kw) {
  uint32_t k[64];
#pragma unroll
  for (int t = 0; t < 64; t += 4) {
    const uint4 q = *reinterpret_cast<const uint4*>(kw + t);
    k[t] = q.x;
    k[t + 1] = q.y;
    k[t + 2] = q.z;
    k[t + 3] = q.w;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) pin_vgpr(st.h[i]);
  uint32_t a = st.h[0], b = st.h[1], c = st.h[2], d = st.h[3];
  uint32_t e = st.h[4], f = st.h[5], g = st.h[6], h = st.h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + k[t];
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t maj = maj3(a, b, c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + maj;
  }
  st.h[0] += a;
  st.h[1] += b;
  st.h[2] += c;
  st.h[3] += d;
  st.h[4] += e;
  st.h[5] += f;
  st.h[6] += g;
  st.h[7] += h;
}

// Rounds T0..T1-1 of one compression on the working state v = (a..h), block w
// (big-endian words; the schedule is extended in place); mid (T0 == 0,
// optional) receives (a..h) after round 7.  Two compressions from the same
// chaining value whose blocks share words 0..7 share rounds 0..7 exactly: the
// transcript's challenge after a half-block absorb (block = the 32 absorbed
// bytes || padding) and the next absorb's block-completing compression (block
// = the same 32 bytes || the next 32) -- the second starts at round 8 from mid.
template <int T0, int T1 = 64>
__device__ __forceinline__ void sha256_rounds_from(uint32_t (&v)[8], uint32_t w[16], uint32_t* mid) {
  constexpr uint32_t K[64] = MLH_SHA_K;
#pragma unroll
  for (int i = 0; i < 16; ++i) pin_vgpr(w[i]);
#pragma unroll
  for (int i = 0; i < 8; ++i) pin_vgpr(v[i]);
  uint32_t a = v[0], b = v[1], c = v[2], d = v[3], e = v[4], f = v[5], g = v[6], h = v[7];
#pragma unroll
  for (int t = T0; t < T1; ++t) {
    if (t >= 16) {
      const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
    }
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + K[t] + w[t & 15];
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t t2 = S0 + maj3(a, b, c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
    if (t == 7 && mid) {
      mid[0] = a;
      mid[1] = b;
      mid[2] = c;
      mid[3] = d;
      mid[4] = e;
      mid[5] = f;
      mid[6] = g;
      mid[7] = h;
    }
  }
  v[0] = a;
  v[1] = b;
  v[2] = c;
  v[3] = d;
  v[4] = e;
  v[5] = f;
  v[6] = g;
  v[7] = h;
}

// ---- two-lane SHA-256 rounds ------------------------------------------------
// A one-lane compression issues ~14 VALU per round (6 v_alignbit, 4 v_bitop3,
// 4 adds).  Two lanes share a round in SIMT form: lanes k and 7 - k of each
// 8-lane half row (k < 4; the row_half_mirror DPP swaps them), the "e side"
// (banks 0 and 2 of a row) holding (e, f, g, h) and the "a side" (banks 1 and
// 3) (a, b, c, d).  One instruction stream computes Sigma1(e) | Sigma0(a)
// (v_alignbit with per-lane counts), Ch(e, f, g) | Maj(a, b, c) (= bfi(e, f,
// g) | bfi(a ^ c, b, c)) and u = Sigma + Ch|Maj + x with x = h + K + W + d on
// the e side and -d on the a side: u is the new e (T1 + d) on the e side and
// T2 - d on the a side, and ONE bank-masked DPP add (a side only) forms the
// new a = u_e + u_a = T1 + T2 while the e side keeps u.  The dependency chain
// of a round is v_alignbit, xor3, add3, DPP add; the next round's x (n = -c on
// every lane, then c(partner) + g + K + W on the e side through a second
// bank-masked DPP add) is off it.  11 VALU per round; a dependent node hash
// on one wave 7.5k cycles against 8.5k with the earlier adjacent-lane pairs,
// whose select of (T1 | d) sat on the chain (tools/sha_hm_bench.hip).  Every
// lane pair computes the same compression; inputs are wave-uniform.
constexpr int kSha2lDpp = 0x141;  // row_half_mirror
__device__ __forceinline__ bool sha2l_aside(uint32_t lane) { return (lane >> 2) & 1u; }
// node of thread t when the nodes of a workgroup are hashed on lane pairs
// (32 per wave), and whether t is its e-side lane (the one that stores it)
__device__ __forceinline__ uint32_t sha2l_pair(uint32_t t) {
  const uint32_t k = t & 7;
  return ((t >> 3) << 2) | (k < 4 ? k : 7 - k);
}
__device__ __forceinline__ bool sha2l_lead(uint32_t t) { return !sha2l_aside(t); }
struct Sha2L {
  uint32_t r0, r1, r2, r3;  // e side: e f g h; a side: a b c d
  uint32_t m;               // a side ~0, e side 0
  uint32_t s1, s2, s3;      // the lane's Sigma rotation counts
};
__device__ __forceinline__ void sha2l_init(Sha2L& q, const uint32_t (&v)[8]) {
  const bool a = sha2l_aside(__lane_id());
  q.m = a ? ~0u : 0u;
  // opaque to the compiler: p = r0 ^ (r2 & m) stays one v_bitop3 (as a select
  // of constants it lowers to v_cndmask + v_xor)
  asm("" : "+v"(q.m));
  q.r0 = a ? v[0] : v[4];
  q.r1 = a ? v[1] : v[5];
  q.r2 = a ? v[2] : v[6];
  q.r3 = a ? v[3] : v[7];
  q.s1 = a ? 2u : 6u;
  q.s2 = a ? 13u : 11u;
  q.s3 = a ? 22u : 25u;
}
// The working state a..h, wave-uniform (read from an a-side and an e-side lane).
__device__ __forceinline__ void sha2l_state(const Sha2L& q, uint32_t (&v)[8]) {
  v[0] = __builtin_amdgcn_readlane(q.r0, 4);
  v[1] = __builtin_amdgcn_readlane(q.r1, 4);
  v[2] = __builtin_amdgcn_readlane(q.r2, 4);
  v[3] = __builtin_amdgcn_readlane(q.r3, 4);
  v[4] = __builtin_amdgcn_readlane(q.r0, 0);
  v[5] = __builtin_amdgcn_readlane(q.r1, 0);
  v[6] = __builtin_amdgcn_readlane(q.r2, 0);
  v[7] = __builtin_amdgcn_readlane(q.r3, 0);
}
// e side: src(partner) + y; a side keeps old.  The DPP source must not be
// written by either of the two instructions before (gfx950 DPP hazard, not
// seen through inline asm): the rounds pass r2, written two rounds earlier (or
// by sha2l_init before round T0's 11 instructions), and tools/
// dpp_hazard_check.py, run by build(), verifies every DPP of the built
// library.  (Round T0 through the compiler's own DPP instead reschedules the
// whole block: 8.0k instead of 7.5k cycles per node hash.)
__device__ __forceinline__ uint32_t sha2l_dpp_add_eside(uint32_t old, uint32_t src, uint32_t y) {
  asm("v_add_u32_dpp %0, %1, %2 row_half_mirror row_mask:0xf bank_mask:0x5" : "+v"(old) : "v"(src), "v"(y));
  return old;
}
// Rounds T0..T1-1; kwf(t) returns K[t] + W[t] (wave-uniform) and is called
// once per t in increasing order (so it may extend the message schedule).
template <int T0, int T1, class KWF>
__device__ __forceinline__ void sha2l_rounds(Sha2L& q, KWF&& kwf) {
  uint32_t x;  // e side: h + K + W + d (d from the partner); a side: -d
  {
    const uint32_t hk = q.r3 + kwf(T0);
    const uint32_t d = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r3, kSha2lDpp, 0xF, 0xF, false);
    x = q.m ? 0u - q.r3 : hk + d;
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
    if (t + 1 < T1) {  // the next round's x: r2 becomes r3 (g -> h, c -> d)
      const uint32_t hk = q.r2 + kwf(t + 1);
      xn = sha2l_dpp_add_eside(0u - q.r2, q.r2, hk);
    }
    q.r3 = q.r2;
    q.r2 = q.r1;
    q.r1 = q.r0;
    // a side: u_e (partner) + u_a; the e side keeps u (bank mask; old 0 is
    // the add's identity, so this is one v_add_u32_dpp)
    q.r0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, kSha2lDpp, 0xF, 0xA, false) + u;
    x = xn;
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
// lanes hold the same w: the e side computes sigma0(w[t-15]) and the a side
// sigma1(w[t-2]) in one instruction stream (per-lane v_alignbit and
// v_lshrrev counts) and one DPP add sums them: 7 VALU per word instead of the
// one-lane 10.
struct Sched2L {
  uint32_t m;           // a side ~0, e side 0
  uint32_t c1, c2, c3;  // e side: 7, 18, 3 (sigma0); a side: 17, 19, 10 (sigma1)
};
__device__ __forceinline__ Sched2L sched2l_init() {
  const bool a = sha2l_aside(__lane_id());
  Sched2L c;
  c.m = a ? ~0u : 0u;
  asm("" : "+v"(c.m));
  c.c1 = a ? 17u : 7u;
  c.c2 = a ? 19u : 18u;
  c.c3 = a ? 10u : 3u;
  return c;
}
__device__ __forceinline__ uint32_t sha2l_sched(uint32_t* w, int t, const Sched2L& c) {
  const uint32_t x = (w[(t - 2) & 15] & c.m) | (w[(t - 15) & 15] & ~c.m);
  const uint32_t sg = xor3(__builtin_amdgcn_alignbit(x, x, c.c1), __builtin_amdgcn_alignbit(x, x, c.c2),
                           x >> c.c3);
  uint32_t both = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sg, kSha2lDpp, 0xF, 0xF, true) + sg;
  asm("" : "+v"(both));  // one v_add_u32_dpp (else: v_mov_dpp + a reassociated add)
  return w[t & 15] = both + w[(t - 7) & 15] + w[t & 15];
}

// The working state a..h of each lane pair, on both lanes of the pair (one
// DPP swap per word), for lane pairs that hash different messages.
__device__ __forceinline__ void sha2l_state_pair(const Sha2L& q, uint32_t (&v)[8]) {
  const bool a = q.m != 0u;
  const uint32_t o0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r0, kSha2lDpp, 0xF, 0xF, true);
  const uint32_t o1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r1, kSha2lDpp, 0xF, 0xF, true);
  const uint32_t o2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r2, kSha2lDpp, 0xF, 0xF, true);
  const uint32_t o3 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.r3, kSha2lDpp, 0xF, 0xF, true);
  v[0] = a ? q.r0 : o0;
  v[1] = a ? q.r1 : o1;
  v[2] = a ? q.r2 : o2;
  v[3] = a ? q.r3 : o3;
  v[4] = a ? o0 : q.r0;
  v[5] = a ? o1 : q.r1;
  v[6] = a ? o2 : q.r2;
  v[7] = a ? o3 : q.r3;
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

// next_challenge() after an absorb that ended on a block boundary (chaining
// value h0..h7, wave-uniform): the padding-only block from its precomputed
// K + W table, on two lanes; Field128::from of the digest's first 16 bytes.
// Out of line, so a rehearsal of it warms the code the rounds run.
__device__ __noinline__ fe sha2l_pad_challenge(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3,
                                               uint32_t h4, uint32_t h5, uint32_t h6, uint32_t h7,
                                               const uint32_t* kw) {
  const uint32_t h[8] = {h0, h1, h2, h3, h4, h5, h6, h7};
  uint32_t k[64];
#pragma unroll
  for (int t = 0; t < 64; t += 4) {
    const uint4 x = *reinterpret_cast<const uint4*>(kw + t);
    k[t] = x.x;
    k[t + 1] = x.y;
    k[t + 2] = x.z;
    k[t + 3] = x.w;
  }
  Sha2L q;
  sha2l_init(q, h);
  sha2l_rounds<0, 64>(q, [&](int t) -> uint32_t { return k[t]; });
  uint32_t v[8];
  sha2l_state(q, v);
  fe o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o.w[i] = bswap32(h[i] + v[i]);
  return canon_with_carry(o, 0u);
}

// Field128::from(u128) (field.rs:138-142): one conditional subtraction of M.
// The u128 is LE over digest bytes 0..15, i.e. limb i = bswap(h[i]).
__device__ inline fe dsha_challenge(const DevSha& s) {
  uint32_t h[8];
  dsha_final(s, h);
  fe v;
  for (int i = 0; i < 4; ++i) v.w[i] = bswap32(h[i]);
  return canon_with_carry(v, 0u);
}

// dsha_challenge with the padding-only block's K + W table for this length
// (kw, or nullptr): used when the buffer is empty (len % 64 == 0).
__device__ inline fe dsha_challenge_kw(const DevSha& s, const uint32_t* kw) {
  if (!kw || (s.len & 63) != 0) return dsha_challenge(s);
  Sha256State st;
  for (int i = 0; i < 8; ++i) st.h[i] = s.h[i];
  sha256_compress_kw(st, kw);
  fe v;
  for (int i = 0; i < 4; ++i) v.w[i] = bswap32(st.h[i]);
  return canon_with_carry(v, 0u);
}

// One compression of the 16 block words w0..w15 (big-endian, wave-uniform)
// into the chaining value h0..h7 (wave-uniform) on a lane pair: sha2l rounds
// with the two-lane message schedule; returns the new chaining value.  Out of
// line with everything passed in registers: a transcript step calls it up to
// three times, and one copy stays in the instruction cache.
__device__ __noinline__ Sha256State sha2l_compress(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3,
                                                   uint32_t h4, uint32_t h5, uint32_t h6, uint32_t h7,
                                                   uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                                   uint32_t w4, uint32_t w5, uint32_t w6, uint32_t w7,
                                                   uint32_t w8, uint32_t w9, uint32_t w10, uint32_t w11,
                                                   uint32_t w12, uint32_t w13, uint32_t w14,
                                                   uint32_t w15) {
  constexpr uint32_t K[64] = MLH_SHA_K;
  const uint32_t h[8] = {h0, h1, h2, h3, h4, h5, h6, h7};
  uint32_t blk[16] = {w0, w1, w2, w3, w4, w5, w6, w7, w8, w9, w10, w11, w12, w13, w14, w15};
  const Sched2L sc = sched2l_init();
  Sha2L q;
  sha2l_init(q, h);
  sha2l_rounds<0, 64>(q, [&](int t) -> uint32_t {
    if (t >= 16) sha2l_sched(blk, t, sc);
    return K[t] + blk[t & 15];
  });
  uint32_t v[8];
  sha2l_state(q, v);
  Sha256State o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o.h[i] = h[i] + v[i];
  return o;
}
__device__ __forceinline__ void sha2l_compress_into(uint32_t (&h)[8], const uint32_t (&b)[16]) {
  const Sha256State o = sha2l_compress(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], b[0], b[1], b[2],
                                       b[3], b[4], b[5], b[6], b[7], b[8], b[9], b[10], b[11], b[12],
                                       b[13], b[14], b[15]);
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = o.h[i];
}

// Transcript step on a lane pair, for a caller whose whole wave runs it
// (uniform control flow; every lane pair carries the two-lane SHA-256 of the
// same words): absorb the NW words w (memory byte order, wave-uniform) into s
// (shared memory; lane 0 writes it), then (r_out) write next_challenge() to
// r_out and return it (wave-uniform; lane 0's on the one-lane path).  Same
// state and challenge as dsha_absorb +
// dsha_challenge, with the compressions at ~2.5 instead of ~4.3 us.  A
// length not a multiple of 4 (bytes absorbed on the host) takes the one-lane
// path.
template <int NW>
__device__ fe dsha2l_step(DevSha& s, const uint32_t (&w)[NW], uint32_t* stage, fe* r_out) {
  const uint32_t lane = __lane_id();
  const uint64_t len0 = s.len;
  if (len0 & 3) {
    fe r = fe_zero();
    if (lane == 0) {
      dsha_absorb<NW>(s, w, stage);
      if (r_out) fe_store(r_out, r = dsha_challenge(s));
    }
    return r;  // (lane 0's)
  }
  uint32_t* bw = reinterpret_cast<uint32_t*>(s.buf);
  uint32_t h[8], blk[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = s.h[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) blk[i] = bswap32(bw[i]);
  const uint32_t pos0 = (uint32_t)(len0 & 63) / 4;
  // the words that fit the buffer, then (if it fills) one compression and the
  // rest into the next block -- selects over constant indices, no dynamic
  // register indexing
  uint32_t nxt[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) nxt[j] = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint32_t x = bswap32(w[i]);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if ((uint32_t)j == pos0 + i) blk[j] = x;
      if ((uint32_t)j + 16 == pos0 + i) nxt[j] = x;
    }
  }
  uint32_t pos = pos0 + NW;
  if (pos >= 16) {
    sha2l_compress_into(h, blk);
#pragma unroll
    for (int j = 0; j < 16; ++j) blk[j] = nxt[j];
    pos -= 16;
  }
  const uint64_t len = len0 + 4 * NW;
  if (lane == 0) {  // the state: chaining value, buffer (memory byte order), length
#pragma unroll
    for (int i = 0; i < 8; ++i) s.h[i] = h[i];
#pragma unroll
    for (int i = 0; i < 16; ++i) bw[i] = bswap32(blk[i]);
    s.len = len;
  }
  if (!r_out) return fe_zero();
  // next_challenge(): finalize a copy -- 0x80, zeros, the bit length
  const uint64_t bits = len * 8;
#pragma unroll
  for (int j = 0; j < 16; ++j)
    blk[j] = (uint32_t)j < pos ? blk[j] : ((uint32_t)j == pos ? 0x80000000u : 0u);
  if (pos >= 14) {
    sha2l_compress_into(h, blk);
#pragma unroll
    for (int j = 0; j < 14; ++j) blk[j] = 0;
  }
  blk[14] = (uint32_t)(bits >> 32);
  blk[15] = (uint32_t)bits;
  sha2l_compress_into(h, blk);
  fe v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v.w[i] = bswap32(h[i]);
  const fe r = canon_with_carry(v, 0u);
  if (lane == 0) fe_store(r_out, r);
  return r;
}

// absorb n bytes from device memory, then (if r_out) write next_challenge();
// copy_out (optional) receives a copy of the absorbed bytes
hipError_t launch_transcript_absorb(DevSha* t, const uint8_t* src, uint32_t n, fe* r_out,
                                    hipStream_t st, uint8_t* copy_out = nullptr);
// final FRI layer (2 values): flag = (v0 != v1) ("not an RS code"),
// absorb LE16(v0), copy v0 to last_out
hipError_t launch_fri_last(const fe* vals, DevSha* t, uint32_t* flag, fe* last_out,
                           hipStream_t st);

}  // namespace mlh
