// Device arithmetic over F_M, M = 2^128 - 45*2^40 + 1 (the `field.rs` modulus).
//
// Reference: src/field.rs:31 (Field128 wraps winter-math f128 BaseElement),
// src/ntt/mod.rs:34-36 (modulus).  winter-math keeps elements canonical
// (value < M) and Field128::as_ref exposes the raw little-endian u128, so the
// device keeps exactly that representation in HBM: 16 bytes per element, four
// little-endian u32 limbs, always canonical.  Any mathematically correct
// arithmetic is then bit-identical to the reference's.
//
// gfx950 notes: there is no 64x64 multiplier; the 128x128 product is 16
// v_mad_u64_u32 (32x32+64 -> 64) and the reduction uses the special form
//   2^128 = C (mod M),  C = 45*2^40 - 1 = 0x2CFF_FFFFFFFF
// so H*C = H*0x2D00*2^32 - H  (four small-constant mads, no second wide product).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mlh {

struct __attribute__((aligned(16))) fe {
  uint32_t w[4];
};

// 0x2D00 * 2^32 - 1 = C
constexpr uint32_t kC0 = 0xFFFFFFFFu;
constexpr uint32_t kC1 = 0x00002CFFu;
constexpr uint32_t kCmul = 0x2D00u;  // C = kCmul*2^32 - 1
// M = 0xFFFFFFFF_FFFFFFFF_FFFFD300_00000001
constexpr uint32_t kM0 = 0x00000001u;
constexpr uint32_t kM1 = 0xFFFFD300u;
constexpr uint32_t kM2 = 0xFFFFFFFFu;
constexpr uint32_t kM3 = 0xFFFFFFFFu;

__device__ __forceinline__ fe fe_zero() { return fe{{0u, 0u, 0u, 0u}}; }
__device__ __forceinline__ fe fe_one() { return fe{{1u, 0u, 0u, 0u}}; }

__device__ __forceinline__ bool fe_eq(const fe& a, const fe& b) {
  return ((a.w[0] ^ b.w[0]) | (a.w[1] ^ b.w[1]) | (a.w[2] ^ b.w[2]) | (a.w[3] ^ b.w[3])) == 0u;
}

__device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  return __builtin_addc(a, b, cin, cout);
}
__device__ __forceinline__ uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  return __builtin_subc(a, b, bin, bout);
}

// x + C, returning the carry out of bit 128.
__device__ __forceinline__ fe add_c(const fe& x, uint32_t* carry) {
  fe t;
  uint32_t k;
  t.w[0] = addc(x.w[0], kC0, 0u, &k);
  t.w[1] = addc(x.w[1], kC1, k, &k);
  t.w[2] = addc(x.w[2], 0u, k, &k);
  t.w[3] = addc(x.w[3], 0u, k, &k);
  *carry = k;
  return t;
}

// s in [0, 2^128) plus an extra carry bit k (value s + k*2^128 < 2M):
// canonical representative.  s + k*2^128 >= M  <=>  k | carry(s + C).
__device__ __forceinline__ fe canon_with_carry(const fe& s, uint32_t k) {
  uint32_t k2;
  fe t = add_c(s, &k2);
  const bool take = (k | k2) != 0u;
  fe r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.w[i] = take ? t.w[i] : s.w[i];
  return r;
}

__device__ __forceinline__ fe fe_add(const fe& a, const fe& b) {
  fe s;
  uint32_t k;
  s.w[0] = addc(a.w[0], b.w[0], 0u, &k);
  s.w[1] = addc(a.w[1], b.w[1], k, &k);
  s.w[2] = addc(a.w[2], b.w[2], k, &k);
  s.w[3] = addc(a.w[3], b.w[3], k, &k);
  return canon_with_carry(s, k);
}

__device__ __forceinline__ fe fe_sub(const fe& a, const fe& b) {
  fe d;
  uint32_t br;
  d.w[0] = subb(a.w[0], b.w[0], 0u, &br);
  d.w[1] = subb(a.w[1], b.w[1], br, &br);
  d.w[2] = subb(a.w[2], b.w[2], br, &br);
  d.w[3] = subb(a.w[3], b.w[3], br, &br);
  // borrow: d + M = d - C (mod 2^128); d >= C+1 here so no further borrow.
  const uint32_t m0 = br ? kC0 : 0u;
  const uint32_t m1 = br ? kC1 : 0u;
  uint32_t b2;
  fe r;
  r.w[0] = subb(d.w[0], m0, 0u, &b2);
  r.w[1] = subb(d.w[1], m1, b2, &b2);
  r.w[2] = subb(d.w[2], 0u, b2, &b2);
  r.w[3] = subb(d.w[3], 0u, b2, &b2);
  return r;
}

__device__ __forceinline__ fe fe_neg(const fe& a) { return fe_sub(fe_zero(), a); }

__device__ __forceinline__ fe fe_dbl(const fe& a) { return fe_add(a, a); }

// x / 2 mod M: even -> x >> 1, odd -> (x + M) >> 1 (x + M < 2^129).
__device__ __forceinline__ fe fe_half(const fe& x) {
  const uint32_t odd = x.w[0] & 1u;
  fe s;
  uint32_t k;
  s.w[0] = addc(x.w[0], odd ? kM0 : 0u, 0u, &k);
  s.w[1] = addc(x.w[1], odd ? kM1 : 0u, k, &k);
  s.w[2] = addc(x.w[2], odd ? kM2 : 0u, k, &k);
  s.w[3] = addc(x.w[3], odd ? kM3 : 0u, k, &k);
  fe r;
  r.w[0] = __builtin_amdgcn_alignbit(s.w[1], s.w[0], 1);
  r.w[1] = __builtin_amdgcn_alignbit(s.w[2], s.w[1], 1);
  r.w[2] = __builtin_amdgcn_alignbit(s.w[3], s.w[2], 1);
  r.w[3] = __builtin_amdgcn_alignbit(k, s.w[3], 1);
  return r;
}

// 16-byte vector load/store of one element (global_load_dwordx4).
__device__ __forceinline__ fe fe_load(const fe* p) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  return fe{{v.x, v.y, v.z, v.w}};
}
__device__ __forceinline__ void fe_store(fe* p, const fe& x) {
  *reinterpret_cast<uint4*>(p) = make_uint4(x.w[0], x.w[1], x.w[2], x.w[3]);
}

// acc += a*b with the 64-bit carry-out of v_mad_u64_u32 (an SGPR lane mask)
// counted into c2 by v_addc.  hipcc never uses that carry-out on its own and
// instead shuffles {x, 0} register pairs (~37 v_mov per product).
__device__ __forceinline__ void mac_carry(uint64_t& acc, uint32_t a, uint32_t b, uint32_t& c2) {
  uint64_t out, cy, cy2;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(out), "=s"(cy) : "v"(a), "v"(b), "v"(acc));
  asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(c2), "=s"(cy2) : "v"(c2), "s"(cy));
  acc = out;
}

// Full 256-bit product, product scanning (Comba) over 64-bit column
// accumulators {lo, hi}.  Column 1's first MAC adds to hi(a0*b0) < 2^32 and
// column 6 holds the top 64 bits of a < 2^256 product, so neither can
// overflow; every other MAC counts its carry (13 in total: a first MAC of
// columns 2..5 adds to {hi(prev), carries} < 2^34 and CAN overflow).
__device__ __forceinline__ void mul_wide(const fe& a, const fe& b, uint32_t r[8]) {
  uint64_t acc;
  uint32_t c2;
  acc = (uint64_t)a.w[0] * b.w[0];
  r[0] = (uint32_t)acc;
  acc >>= 32;
  acc = (uint64_t)a.w[0] * b.w[1] + acc;
  c2 = 0;
  mac_carry(acc, a.w[1], b.w[0], c2);
  r[1] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)c2 << 32);
  c2 = 0;
  mac_carry(acc, a.w[0], b.w[2], c2);
  mac_carry(acc, a.w[1], b.w[1], c2);
  mac_carry(acc, a.w[2], b.w[0], c2);
  r[2] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)c2 << 32);
  c2 = 0;
  mac_carry(acc, a.w[0], b.w[3], c2);
  mac_carry(acc, a.w[1], b.w[2], c2);
  mac_carry(acc, a.w[2], b.w[1], c2);
  mac_carry(acc, a.w[3], b.w[0], c2);
  r[3] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)c2 << 32);
  c2 = 0;
  mac_carry(acc, a.w[1], b.w[3], c2);
  mac_carry(acc, a.w[2], b.w[2], c2);
  mac_carry(acc, a.w[3], b.w[1], c2);
  r[4] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)c2 << 32);
  c2 = 0;
  mac_carry(acc, a.w[2], b.w[3], c2);
  mac_carry(acc, a.w[3], b.w[2], c2);
  r[5] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)c2 << 32);
  acc = (uint64_t)a.w[3] * b.w[3] + acc;
  r[6] = (uint32_t)acc;
  r[7] = (uint32_t)(acc >> 32);
}

// Reduce a 256-bit value r (little-endian limbs) to canonical form.
__device__ __forceinline__ fe reduce_wide(const uint32_t r[8]) {
  // U = H * 0x2D00 (5 limbs), T = L + U*2^32 - H  (6 limbs, T >= 0)
  uint32_t u[5];
  uint64_t t;
  t = (uint64_t)r[4] * kCmul;
  u[0] = (uint32_t)t;
  t = (uint64_t)r[5] * kCmul + (t >> 32);
  u[1] = (uint32_t)t;
  t = (uint64_t)r[6] * kCmul + (t >> 32);
  u[2] = (uint32_t)t;
  t = (uint64_t)r[7] * kCmul + (t >> 32);
  u[3] = (uint32_t)t;
  u[4] = (uint32_t)(t >> 32);
  // A = L + (U << 32)
  uint32_t a[6], k;
  a[0] = r[0];
  a[1] = addc(r[1], u[0], 0u, &k);
  a[2] = addc(r[2], u[1], k, &k);
  a[3] = addc(r[3], u[2], k, &k);
  a[4] = addc(u[3], 0u, k, &k);
  a[5] = u[4] + k;
  // A -= H
  uint32_t b;
  a[0] = subb(a[0], r[4], 0u, &b);
  a[1] = subb(a[1], r[5], b, &b);
  a[2] = subb(a[2], r[6], b, &b);
  a[3] = subb(a[3], r[7], b, &b);
  a[4] = subb(a[4], 0u, b, &b);
  a[5] = a[5] - b;
  // Second fold: Th = a[4] + a[5]*2^32 (< 2^47).  X = Th*C = Th*0x2D00*2^32 - Th
  // (>= 0, < 2^93: three limbs); value = a[0..3] + X < 2^128 + 2^93 < 2M.
  const uint64_t th = (uint64_t)a[4] | ((uint64_t)a[5] << 32);
  const uint64_t v = th * (uint64_t)kCmul;  // < 2^61
  const uint32_t x0 = subb(0u, (uint32_t)th, 0u, &b);
  const uint32_t x1 = subb((uint32_t)v, (uint32_t)(th >> 32), b, &b);
  const uint32_t x2 = (uint32_t)(v >> 32) - b;
  fe s;
  s.w[0] = addc(a[0], x0, 0u, &k);
  s.w[1] = addc(a[1], x1, k, &k);
  s.w[2] = addc(a[2], x2, k, &k);
  s.w[3] = addc(a[3], 0u, k, &k);
  return canon_with_carry(s, k);
}

__device__ __forceinline__ fe fe_mul(const fe& a, const fe& b) {
  uint32_t r[8];
  mul_wide(a, b, r);
  return reduce_wide(r);
}

// a * w for a twiddle w supplied as its limb-shifted multiples
// B_k = w * 2^(32k) mod M (k = 0..3, canonical; "expanded" tables):
//   a * w = sum_k a_k * B_k   (< 2^162: four 32x128 rows summed column-wise)
// then one fold of the top T < 2^35: T * 2^128 = T * 0x2D00 * 2^32 - T.
// Every MAC after a column's first product counts its carry; the first MAC
// of columns 1..3 adds to {hi(prev), carries} < 2^35, which can exceed 2^64
// together with a product of two limbs >= 2^32 - 8, so it counts too.  (The
// NTT's hot path uses the generated asm of bfly_asm.hpp instead; this is the
// C reference it was checked against, tools/bfly2_bench.hip.)
__device__ __forceinline__ fe fe_mul_pre_r(const fe& a, const fe& B0, const fe& B1, const fe& B2,
                                           const fe& B3) {
  uint64_t acc;
  uint32_t c2, r0, r1, r2, r3;
  acc = (uint64_t)a.w[0] * B0.w[0];
  c2 = 0;
  mac_carry(acc, a.w[1], B1.w[0], c2);
  mac_carry(acc, a.w[2], B2.w[0], c2);
  mac_carry(acc, a.w[3], B3.w[0], c2);
  r0 = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)c2 << 32);
  c2 = 0;
  mac_carry(acc, a.w[0], B0.w[1], c2);
  mac_carry(acc, a.w[1], B1.w[1], c2);
  mac_carry(acc, a.w[2], B2.w[1], c2);
  mac_carry(acc, a.w[3], B3.w[1], c2);
  r1 = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)c2 << 32);
  c2 = 0;
  mac_carry(acc, a.w[0], B0.w[2], c2);
  mac_carry(acc, a.w[1], B1.w[2], c2);
  mac_carry(acc, a.w[2], B2.w[2], c2);
  mac_carry(acc, a.w[3], B3.w[2], c2);
  r2 = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)c2 << 32);
  c2 = 0;
  mac_carry(acc, a.w[0], B0.w[3], c2);
  mac_carry(acc, a.w[1], B1.w[3], c2);
  mac_carry(acc, a.w[2], B2.w[3], c2);
  mac_carry(acc, a.w[3], B3.w[3], c2);
  r3 = (uint32_t)acc;
  const uint32_t t_lo = (uint32_t)(acc >> 32), t_hi = c2;  // T = t_lo + t_hi 2^32 < 2^35
  // X = T*C = T*0x2D00*2^32 - T (>= 0, < 2^81: three limbs), value = r + X < 2^128 + 2^81
  const uint64_t v = (uint64_t)t_lo * kCmul;
  const uint32_t vh = (uint32_t)(v >> 32) + __umul24(t_hi, kCmul);
  uint32_t b, k;
  const uint32_t x0 = subb(0u, t_lo, 0u, &b);
  const uint32_t x1 = subb((uint32_t)v, t_hi, b, &b);
  const uint32_t x2 = vh - b;
  fe s;
  s.w[0] = addc(r0, x0, 0u, &k);
  s.w[1] = addc(r1, x1, k, &k);
  s.w[2] = addc(r2, x2, k, &k);
  s.w[3] = addc(r3, 0u, k, &k);
  return canon_with_carry(s, k);
}

__device__ __forceinline__ fe fe_mul_pre(const fe& a, const fe* B) {
  return fe_mul_pre_r(a, fe_load(B), fe_load(B + 1), fe_load(B + 2), fe_load(B + 3));
}

__device__ __forceinline__ fe fe_sqr(const fe& a) { return fe_mul(a, a); }

__device__ __forceinline__ fe fe_pow(fe base, uint64_t e) {
  fe acc = fe_one();
  while (e) {
    if (e & 1) acc = fe_mul(acc, base);
    base = fe_mul(base, base);
    e >>= 1;
  }
  return acc;
}

}  // namespace mlh
