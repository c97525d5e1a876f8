// SHA-256 compression on gfx950 VALU (FIPS 180-4), one message per lane.
//
// Sigma/sigma 3-way XORs are single v_bitop3_b32 (gfx950).
// Reference: the sha2 0.10.8 crate (Cargo.lock:261-269) used by
// src/merkle_tree/mod.rs:178-189 (hash_leaf / hash_node) and
// src/transcript.rs.  Rotations are v_alignbit_b32, Ch and Maj one
// v_bitop3_b32 each, the 3-input adds fold to v_add3_u32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mlh {

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
// a ^ b ^ c in one full-rate v_bitop3_b32 (truth table 0x96); hipcc emits two
// v_xor_b32 for the Sigma/sigma functions otherwise.
// Operands that are compile-time constants after unrolling (the constant words
// of a 32-byte message's padded block, the IV in the first rounds) take the
// plain expression instead, which folds (the bitop3 intrinsic does not), so
// no instruction is spent on them.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  if (__builtin_constant_p(a) && __builtin_constant_p(b) && __builtin_constant_p(c)) return a ^ b ^ c;
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// Maj(a, b, c) in one v_bitop3_b32 (table 0xE8: set where >= 2 inputs are);
// left to itself hipcc emits xor + and + bitop3 per round.
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
  if (__builtin_constant_p(a) && __builtin_constant_p(b) && __builtin_constant_p(c))
    return (a & b) | (c & (a | b));
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

#define MLH_SHA_K                                                                               \
  {0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,   \
   0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,   \
   0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,   \
   0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,   \
   0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,   \
   0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,   \
   0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,   \
   0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,   \
   0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,   \
   0xc67178f2u}

struct Sha256State {
  uint32_t h[8];
};

__device__ __forceinline__ Sha256State sha256_iv() {
  return Sha256State{{0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu,
                      0x1f83d9abu, 0x5be0cd19u}};
}

// One compression of a 16-word (big-endian-interpreted) block.
__device__ __forceinline__ void sha256_compress(Sha256State& st, uint32_t w[16]) {
  constexpr uint32_t K[64] = MLH_SHA_K;
  uint32_t a = st.h[0], b = st.h[1], c = st.h[2], d = st.h[3];
  uint32_t e = st.h[4], f = st.h[5], g = st.h[6], h = st.h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
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
    const uint32_t maj = maj3(a, b, c);
    const uint32_t t2 = S0 + maj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
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

// K[t] + W[t] of the constant padding block of a 64-byte message (0x80,
// zeros, bit length 512): its message schedule is a compile-time constant.
struct Pad64KW {
  uint32_t v[64];
  constexpr Pad64KW() : v() {
    constexpr uint32_t K[64] = MLH_SHA_K;
    uint32_t w[64] = {};
    w[0] = 0x80000000u;
    w[15] = 512u;
    for (int t = 16; t < 64; ++t) {
      const uint32_t a = w[t - 15], b = w[t - 2];
      const uint32_t s0 = ((a >> 7) | (a << 25)) ^ ((a >> 18) | (a << 14)) ^ (a >> 3);
      const uint32_t s1 = ((b >> 17) | (b << 15)) ^ ((b >> 19) | (b << 13)) ^ (b >> 10);
      w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    for (int t = 0; t < 64; ++t) v[t] = K[t] + w[t];
  }
};

// Compression of that padding block: only the round function runs.
__device__ __forceinline__ void sha256_compress_pad64(Sha256State& st) {
  constexpr Pad64KW KW;
  uint32_t a = st.h[0], b = st.h[1], c = st.h[2], d = st.h[3];
  uint32_t e = st.h[4], f = st.h[5], g = st.h[6], h = st.h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + KW.v[t];
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

// SHA256(32-byte message), words given big-endian-interpreted.
__device__ __forceinline__ Sha256State sha256_msg32(const uint32_t m[8]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = m[i];
  w[8] = 0x80000000u;
#pragma unroll
  for (int i = 9; i < 15; ++i) w[i] = 0;
  w[15] = 256u;
  Sha256State st = sha256_iv();
  sha256_compress(st, w);
  return st;
}

// SHA256(left32 ‖ right32) with digests in word form (h[i] = BE word i).
__device__ __forceinline__ Sha256State sha256_node(const Sha256State& l, const Sha256State& r) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    w[i] = l.h[i];
    w[8 + i] = r.h[i];
  }
  Sha256State st = sha256_iv();
  sha256_compress(st, w);
  sha256_compress_pad64(st);
  return st;
}

// Digest <-> HBM: the stored bytes are the standard digest bytes
// (GenericArray<u8, 32>), i.e. each word big-endian.
__device__ __forceinline__ void digest_store(uint8_t* p, const Sha256State& s) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(bswap32(s.h[0]), bswap32(s.h[1]), bswap32(s.h[2]), bswap32(s.h[3]));
  q[1] = make_uint4(bswap32(s.h[4]), bswap32(s.h[5]), bswap32(s.h[6]), bswap32(s.h[7]));
}
__device__ __forceinline__ Sha256State digest_load(const uint8_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 a = q[0], b = q[1];
  return Sha256State{{bswap32(a.x), bswap32(a.y), bswap32(a.z), bswap32(a.w), bswap32(b.x),
                      bswap32(b.y), bswap32(b.z), bswap32(b.w)}};
}

}  // namespace mlh
