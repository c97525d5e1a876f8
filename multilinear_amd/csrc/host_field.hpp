// Host-side F_M arithmetic (generators, inverses, scalars shipped to kernels).
// Same canonical u128 representation as the device (field.hpp).
// Reference: src/field.rs, src/ntt/mod.rs:34-58.
#pragma once
#include <stdint.h>
#include <string.h>

namespace mlh {

typedef unsigned __int128 u128;

static const u128 kModulus = (((u128)0xFFFFFFFFFFFFFFFFull) << 64) | (u128)0xFFFFD30000000001ull;
static const u128 kCfold = (u128)0x2CFFFFFFFFFFull;  // 2^128 mod M

inline u128 h_reduce_once(u128 v) { return v >= kModulus ? v - kModulus : v; }

inline u128 h_add(u128 a, u128 b) {
  u128 s = a + b;
  if (s < a) return s + kCfold;  // wrapped: s + 2^128 - M = s + C
  return h_reduce_once(s);
}

inline u128 h_sub(u128 a, u128 b) { return a >= b ? a - b : a - b + kModulus; }

inline u128 h_mul(u128 a, u128 b) {
  const uint64_t a0 = (uint64_t)a, a1 = (uint64_t)(a >> 64);
  const uint64_t b0 = (uint64_t)b, b1 = (uint64_t)(b >> 64);
  const u128 p00 = (u128)a0 * b0, p01 = (u128)a0 * b1, p10 = (u128)a1 * b0, p11 = (u128)a1 * b1;
  // 256-bit product hi:lo
  u128 lo = p00;
  u128 mid = p01 + p10;
  u128 mid_carry = (mid < p01) ? ((u128)1 << 64) : 0;  // carry of mid into bit 192
  u128 lo2 = lo + (mid << 64);
  u128 hi = p11 + (mid >> 64) + mid_carry + (lo2 < lo ? 1 : 0);
  lo = lo2;
  // P = hi*2^128 + lo == lo + hi*C (mod M); hi*C < 2^174: fold twice.
  while (hi != 0) {
    const uint64_t h0 = (uint64_t)hi, h1 = (uint64_t)(hi >> 64);
    // hi*C = h0*C + h1*C*2^64 ; C < 2^46 so h0*C < 2^110, h1*C < 2^110
    const u128 t0 = (u128)h0 * (uint64_t)kCfold;
    const u128 t1 = (u128)h1 * (uint64_t)kCfold;
    u128 nhi = 0;
    u128 s = lo + t0;
    if (s < lo) nhi += 1;
    u128 t1lo = t1 << 64;
    u128 s2 = s + t1lo;
    if (s2 < s) nhi += 1;
    nhi += t1 >> 64;
    lo = s2;
    hi = nhi;
  }
  return h_reduce_once(lo);
}

inline u128 h_pow(u128 b, u128 e) {
  u128 acc = 1;
  while (e) {
    if (e & 1) acc = h_mul(acc, b);
    b = h_mul(b, b);
    e >>= 1;
  }
  return acc;
}

inline u128 h_inv(u128 a) { return h_pow(a, kModulus - 2); }

// NttField::pow_2_generator (src/ntt/mod.rs:42-54); 0 when log_size > 40.
inline u128 h_pow2_generator(unsigned log_size) {
  if (log_size > 40) return 0;
  return h_pow(3, (kModulus - 1) >> log_size);
}

inline u128 h_load(const uint8_t* p) {
  u128 v;
  memcpy(&v, p, 16);  // little-endian host (x86_64)
  return v;
}
inline void h_store(uint8_t* p, u128 v) { memcpy(p, &v, 16); }

}  // namespace mlh
