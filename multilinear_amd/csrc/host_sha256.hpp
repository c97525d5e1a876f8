// Host SHA-256 (FIPS 180-4) for the Fiat-Shamir transcript.
// Reference: src/transcript.rs (sha2 0.10.8 Sha256: update / finalize of a
// clone).  Incremental, copyable state.
#pragma once
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

namespace mlh {

static const uint32_t kHostShaK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

// One compression with the x86 SHA extensions (sha256rnds2 does two rounds on
// the ABEF/CDGH state halves; sha256msg1/msg2 extend the schedule).  The host
// transcript replays every device absorb and derives the 128 query indices,
// so its speed is on the prove's critical path.
__attribute__((target("sha,sse4.1,ssse3"))) static inline void host_sha256_compress_ni(
    uint32_t h[8], const uint8_t* blk) {
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i tmp = _mm_loadu_si128(reinterpret_cast<const __m128i*>(h));      // a b c d
  __m128i st1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(h + 4));  // e f g h
  tmp = _mm_shuffle_epi32(tmp, 0xB1);
  st1 = _mm_shuffle_epi32(st1, 0x1B);
  __m128i st0 = _mm_alignr_epi8(tmp, st1, 8);   // ABEF
  st1 = _mm_blend_epi16(st1, tmp, 0xF0);        // CDGH
  const __m128i abef = st0, cdgh = st1;
  __m128i m[4];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (j < 4)
      m[j] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(blk + 16 * j)), bswap);
    const __m128i cur = m[j & 3];
    __m128i msg = _mm_add_epi32(cur, _mm_loadu_si128(reinterpret_cast<const __m128i*>(kHostShaK + 4 * j)));
    st1 = _mm_sha256rnds2_epu32(st1, st0, msg);
    if (j >= 3 && j <= 14) {
      const __m128i t = _mm_alignr_epi8(cur, m[(j - 1) & 3], 4);
      m[(j + 1) & 3] = _mm_sha256msg2_epu32(_mm_add_epi32(m[(j + 1) & 3], t), cur);
    }
    msg = _mm_shuffle_epi32(msg, 0x0E);
    st0 = _mm_sha256rnds2_epu32(st0, st1, msg);
    if (j >= 1 && j <= 12) m[(j - 1) & 3] = _mm_sha256msg1_epu32(m[(j - 1) & 3], cur);
  }
  st0 = _mm_add_epi32(st0, abef);
  st1 = _mm_add_epi32(st1, cdgh);
  tmp = _mm_shuffle_epi32(st0, 0x1B);           // FEBA
  st1 = _mm_shuffle_epi32(st1, 0xB1);           // DCHG
  st0 = _mm_blend_epi16(tmp, st1, 0xF0);        // DCBA
  st1 = _mm_alignr_epi8(st1, tmp, 8);           // HGFE
  _mm_storeu_si128(reinterpret_cast<__m128i*>(h), st0);
  _mm_storeu_si128(reinterpret_cast<__m128i*>(h + 4), st1);
}

// SHA extensions present and not disabled (MLH_NO_SHANI=1 forces the portable
// compression; tests run both)
static inline bool host_sha_ni() {
  static const int ok = __builtin_cpu_supports("sha") && !getenv("MLH_NO_SHANI") ? 1 : 0;
  return ok != 0;
}

struct HostSha256 {
  uint32_t h[8];
  uint8_t buf[64];
  uint64_t len = 0;  // bytes absorbed

  HostSha256() { reset(); }
  void reset() {
    static const uint32_t iv[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    memcpy(h, iv, sizeof(h));
    len = 0;
  }
  static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
  void compress(const uint8_t* blk) {
    if (host_sha_ni()) {
      host_sha256_compress_ni(h, blk);
      return;
    }
    const uint32_t* K = kHostShaK;
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
      w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
             ((uint32_t)blk[4 * i + 2] << 8) | (uint32_t)blk[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
      const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = hh + S1 + ch + K[i] + w[i];
      const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
      const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
      const uint32_t t2 = S0 + mj;
      hh = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + t2;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
    h[5] += f;
    h[6] += g;
    h[7] += hh;
  }
  void update(const uint8_t* p, size_t n) {
    size_t fill = (size_t)(len % 64);
    len += n;
    if (fill) {
      const size_t take = n < 64 - fill ? n : 64 - fill;
      memcpy(buf + fill, p, take);
      p += take;
      n -= take;
      fill += take;
      if (fill < 64) return;
      compress(buf);
    }
    while (n >= 64) {
      compress(p);
      p += 64;
      n -= 64;
    }
    if (n) memcpy(buf, p, n);
  }
  // finalize a copy; this state is unchanged
  void digest(uint8_t out[32]) const {
    HostSha256 c = *this;
    const uint64_t bits = c.len * 8;
    uint8_t pad[72] = {0x80};  // 0x80, zeros up to 56 mod 64, then the bit length
    const size_t fill = (size_t)(c.len % 64);
    const size_t np = (fill < 56 ? 56 - fill : 120 - fill);
    for (int i = 0; i < 8; ++i) pad[np + i] = (uint8_t)(bits >> (56 - 8 * i));
    c.update(pad, np + 8);
    for (int i = 0; i < 8; ++i) {
      out[4 * i] = (uint8_t)(c.h[i] >> 24);
      out[4 * i + 1] = (uint8_t)(c.h[i] >> 16);
      out[4 * i + 2] = (uint8_t)(c.h[i] >> 8);
      out[4 * i + 3] = (uint8_t)c.h[i];
    }
  }
};

}  // namespace mlh
