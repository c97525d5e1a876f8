// Device helpers shared by the sumcheck kernels (sumcheck.hip) and the FRI
// fold kernel's PCS round workgroup (fri.hip): 64-lane / block reductions of
// field sums, the streaming product, and the PCS round body.  Internal.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bfly_asm.hpp"
#include "field.hpp"
#include "sumcheck.hpp"

namespace mlh {

constexpr int kRedThreads = 256;

__device__ __forceinline__ fe shfl_xor_fe(const fe& x, int mask) {
  fe r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.w[i] = (uint32_t)__shfl_xor((int)x.w[i], mask, 64);
  return r;
}

// Block reduction of two field sums; thread 0 ends with the totals.
__device__ __forceinline__ void block_reduce2(fe& a, fe& b) {
  __shared__ fe sa[16], sb[16];  // up to 1024 threads
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    a = fe_add(a, shfl_xor_fe(a, m));
    b = fe_add(b, shfl_xor_fe(b, m));
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sa[wid] = a;
    sb[wid] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      a = fe_add(a, sa[w]);
      b = fe_add(b, sb[w]);
    }
  }
}

// Throughput form of the product for the HBM-streaming kernels: the
// generated hand-scheduled 128x128 product + special-form fold (bfly_asm.hpp,
// kind "f": any a < 2^128, canonical b; 62 VALU, no per-MAC pads) and one
// conditional subtraction back to canonical form.
#ifndef MLH_SC_ASM_MUL
#define MLH_SC_ASM_MUL 1
#endif
__device__ __forceinline__ fe fe_mul_s(const fe& a, const fe& b) {
#if MLH_SC_ASM_MUL
  fe x = a;
  uint64_t rare;
  bfly_f_v(x, b, rare);
  return relaxed_canon(x);
#else
  return fe_mul(a, b);
#endif
}
// A wave-uniform field element kept in VGPRs.  Left in SGPRs, the compiler
// runs the uniform arithmetic on the one scalar unit of the CU: 128-bit adds
// as s_add/s_addc with the carry moved through s_cselect / s_cmp per limb
// (three to four instructions per limb instead of one v_addc), which was most
// of a helper wave's time per round.
__device__ __forceinline__ fe fe_vgpr(fe x) {
  asm volatile("" : "+v"(x.w[0]), "+v"(x.w[1]), "+v"(x.w[2]), "+v"(x.w[3]));
  return x;
}
__device__ __forceinline__ fe lerp_s(const fe& lo, const fe& hi, const fe& r) {
  return fe_add(lo, fe_mul_s(fe_sub(hi, lo), r));
}

// PCSProverData::fold (multilinear_pcs.rs:43-76): round k's polynomial
// (sumcheck.rs:174-202) depends on r_{k-1} but not on the FRI root absorbed
// between the two challenges, so it is computed here -- one small workgroup on
// the eq-factored table -- and absorbed, with root k, by the launch that writes
// root k (top_kernel, RootAbsorb::poly_in), which then draws r_k.  Nothing of
// the sumcheck but those 32 bytes sits on the transcript chain.
//
// The table of round k (MSB = variable k) is, in the head (k < B), the B
// corner sums Y[c] = sum_i T[c 2^a + i] lo[i] folded over the variables
// already challenged, with e = H_k = eq(p_{k+1}..p_{B-1}); in the tail it is T
// folded over the B head variables (fold_group_eq passes) and then over the
// tail variables challenged so far, with e = eq(p_{k+1}..p_{L-1}) (Hs).  With
// delta_k = c_k eq(p_k..) (never materialised):
//   E_b = sum_{i<h/2} tab[b h/2 + i] e[i],  s1 = c_k p_k E1,
//   s2 = c_k (3 p_k - 1)(2 E1 - E0),  e0 = claim - s1,
//   c2 = (s2 - 2 s1 + e0) / 2,  c1 = s1 - e0 - c2        (x = 0, 1, 2)
// and after r: claim' = e0 + c1 r + c2 r^2, c' = c ((1 - r)(1 - p) + r p).
__device__ __forceinline__ void pcs_round_body(const PcsJob& J) {
  const fe* src = J.src;
  fe* dst = J.dst;
  const uint32_t log_h = J.log_h;
  const bool fold = J.fold != 0;
  const fe *r_prev = J.r_prev, *p_prev = J.p_prev, *p_k = J.p_k, *e = J.e;
  PcsRoundState* st = J.st;
  fe* poly_out = J.poly_out;
  const uint64_t h = 1ull << log_h, q = h / 2;
  fe r = fe_zero();
  if (r_prev) r = fe_load(r_prev);
  fe E0 = fe_zero(), E1 = fe_zero();
  for (uint64_t i = threadIdx.x; i < q; i += blockDim.x) {
    fe lo, hi;
    if (fold) {  // tab = src folded over its MSB with r (sumcheck.rs:234-247)
      lo = lerp_s(fe_load(src + i), fe_load(src + i + h), r);
      hi = lerp_s(fe_load(src + i + q), fe_load(src + i + q + h), r);
      fe_store(dst + i, lo);
      fe_store(dst + i + q, hi);
    } else {
      lo = fe_load(src + i);
      hi = fe_load(src + i + q);
    }
    const fe ei = fe_load(e + i);
    E0 = fe_add(E0, fe_mul_s(lo, ei));
    E1 = fe_add(E1, fe_mul_s(hi, ei));
  }
  block_reduce2(E0, E1);
  if (threadIdx.x != 0) return;
  // (one lane's serial chain: its operands in VGPRs, fe_vgpr)
  const fe one = fe_one();
  fe claim = fe_vgpr(fe_load(&st->claim)), c = fe_vgpr(fe_load(&st->c));
  if (r_prev) {  // the previous round's claim p(r) and eq scale
    const fe pp = fe_vgpr(fe_load(p_prev)), rv = fe_vgpr(r);
    claim = fe_add(fe_vgpr(fe_load(&st->e0)),
                   fe_mul_s(fe_add(fe_vgpr(fe_load(&st->c1)), fe_mul_s(fe_vgpr(fe_load(&st->c2)), rv)), rv));
    c = fe_mul_s(c, fe_add(fe_mul_s(fe_sub(one, rv), fe_sub(one, pp)), fe_mul_s(rv, pp)));
  }
  const fe p = fe_vgpr(fe_load(p_k));
  const fe s1 = fe_mul_s(c, fe_mul_s(p, E1));
  const fe s2 = fe_mul_s(fe_mul_s(c, fe_sub(fe_add(fe_dbl(p), p), one)), fe_sub(fe_dbl(E1), E0));
  const fe e0 = fe_sub(claim, s1);
  const fe c2 = fe_half(fe_add(fe_sub(s2, fe_dbl(s1)), e0));
  const fe c1 = fe_sub(fe_sub(s1, e0), c2);
  fe_store(poly_out, c1);
  fe_store(poly_out + 1, c2);
  fe_store(&st->claim, claim);
  fe_store(&st->c, c);
  fe_store(&st->e0, e0);
  fe_store(&st->c1, c1);
  fe_store(&st->c2, c2);
}


}  // namespace mlh
