// MLE / sumcheck kernels on gfx950.
//
// Reference:
//   * eq ("delta") table: src/constraint_system/sumcheck.rs:128-145 with
//     Mask::evaluate (evaluation.rs:51-73): delta[idx] = prod_i (bit_i(idx) ?
//     p[n-1-i] : 1 - p[n-1-i]) (big-endian point order);
//   * round sums: SumcheckTables::partial_sum (sumcheck.rs:204-232), PCS
//     composition x[0] (multilinear_pcs.rs:56), evaluated at X = 1 and X = 2:
//       s1 = sum_{i<h} m[i+h] d[i+h],
//       s2 = sum_{i<h} (2 m[i+h] - m[i]) (2 d[i+h] - d[i]);
//   * fold: SumcheckTables::fold (sumcheck.rs:234-247): t[i] = (1-r) t[i] + r t[i+h],
//     computed as t[i] + r (t[i+h] - t[i]) (same field value, one modmul);
//   * Moebius transform: MultilinearPolynomialEvals::to_coefficient
//     (polynomials.rs:150-163), and its zeta inverse (:111-124);
//   * MLE evaluate (polynomials.rs:165-187) = dot(evals, eq(args)).
//
// The round kernels are HBM-streaming: 16 B per lane dwordx4 loads, sums
// reduced with 64-lane shuffles, then LDS, then one partial per workgroup
// (reduced by a second single-workgroup launch; no float-style atomics exist
// for F_M).  fold_sums fuses round k's fold with round k+1's sums: lane i reads
// t[i], t[i+h/2], t[i+h], t[i+3h/2] and writes the two folded values, so each
// round moves 2*S*16 B in and S*16 B out (the survey's 48 S bytes).
#include "bfly_asm.hpp"
#include "field.hpp"
#include "sumcheck.hpp"
#include "sc_dev.hpp"
#include "transcript_dev.hpp"

namespace mlh {

// The 2^24-table sweeps of the eq-factored prove (corner_sums_lo_kernel and
// the 6-level fold_group_eq_kernel) read through a raw buffer load with the
// nontemporal policy (`nt`): the sweep then does not flush the L2 of the code
// and tables of the one-workgroup eq-tail launches between sweeps, which
// otherwise start cold (their instruction fetches from HBM).  Measured per
// prove: eq-tail launches 76 -> 67 us each, the 6-level fold +2 us, the corner
// sums +5 us (a plain global load with the same hint: fold +8 us; the sc0 /
// sc1 policies: no effect on the eq tail).  base: uniform; idx < 2^28.
#ifndef MLH_SWEEP_AUX
#define MLH_SWEEP_AUX 2  // cache-policy word of the buffer load (gfx950: sc0 1, nt 2, sc1 16); < 0: plain load
#endif
__device__ __forceinline__ fe sweep_load(const fe* base, uint32_t idx) {
#if MLH_SWEEP_AUX < 0
  return fe_load(base + idx);
#else
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<fe*>(base), 0, (int)0xFFFFFFFFu, 0x00020000);
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, idx * 16u, 0, MLH_SWEEP_AUX);
  return fe{{v.x, v.y, v.z, v.w}};
#endif
}
constexpr uint32_t kTailLogMax = 12;  // sumcheck_tail_kernel: 2 x 2^12 x 16 B = 128 KiB LDS

// Phase timestamps of sumcheck_tail_kernel (tools/tail_bench.hip builds this
// file with -DMLH_TAIL_PROF; compiled out otherwise).
#ifdef MLH_TAIL_PROF
__device__ uint64_t g_tail_ts[64], g_tail_cyc[64];
#define MLH_TAIL_TS(i)                                \
  do {                                                \
    if (threadIdx.x == 0 && (i) < 64) {               \
      g_tail_ts[i] = wall_clock64();                  \
      g_tail_cyc[i] = __builtin_amdgcn_s_memtime();   \
    }                                                 \
  } while (0)
#else
#define MLH_TAIL_TS(i) \
  do {                 \
  } while (0)
#endif

__global__ void __launch_bounds__(kRedThreads)
sums_kernel(const fe* __restrict__ m, const fe* __restrict__ d, uint64_t h,
            fe* __restrict__ partials) {
  fe s1 = fe_zero(), s2 = fe_zero();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < h; i += stride) {
    const fe m0 = fe_load(m + i), m1 = fe_load(m + i + h);
    const fe d0 = fe_load(d + i), d1 = fe_load(d + i + h);
    s1 = fe_add(s1, fe_mul(m1, d1));
    const fe mm = fe_sub(fe_dbl(m1), m0), dd = fe_sub(fe_dbl(d1), d0);
    s2 = fe_add(s2, fe_mul(mm, dd));
  }
  block_reduce2(s1, s2);
  if (threadIdx.x == 0) {
    fe_store(partials + 2 * blockIdx.x, s1);
    fe_store(partials + 2 * blockIdx.x + 1, s2);
  }
}

__device__ __forceinline__ fe lerp(const fe& lo, const fe& hi, const fe& r) {
  return fe_add(lo, fe_mul(r, fe_sub(hi, lo)));
}

// Lazy accumulation for the streaming sums: acc (9 limbs) += a b unreduced.
// Operand scanning: row i's product a_i b_j takes acc[i+j] + carry as its
// 64-bit addend, which cannot overflow ((2^32-1)^2 + 2 (2^32-1) = 2^64 - 1),
// so no carry-out is needed inside a row (16 mads, ~52 VALU per product
// against ~85 for a reduced product plus a modular add).
struct acc9 {
  uint32_t w[9];
};
__device__ __forceinline__ void acc_zero(acc9& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) a.w[i] = 0;
}
__device__ __forceinline__ void mulacc(acc9& acc, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t carry = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t t = (uint64_t)a.w[i] * b.w[j] + ((uint64_t)acc.w[i + j] + carry);
      acc.w[i + j] = (uint32_t)t;
      carry = (uint32_t)(t >> 32);
    }
    uint32_t k;
    acc.w[i + 4] = __builtin_addc(acc.w[i + 4], carry, 0u, &k);
#pragma unroll
    for (int j = i + 5; j < 9; ++j) acc.w[j] = __builtin_addc(acc.w[j], 0u, k, &k);
  }
}
// Canonical value of an accumulator (< 2^288): the low 256 bits reduced, plus
// the top limb times 2^256 mod M = C^2 (< 2^91).
__device__ __forceinline__ fe acc_reduce(const acc9& a) {
  const fe lo = reduce_wide(a.w);
  const fe k256{{0x00000001u, 0xFFFFA600u, 0x07E8FFFFu, 0u}};
  return fe_add(lo, fe_mul_s(fe{{a.w[8], 0u, 0u, 0u}}, k256));
}

// Column accumulator for the HBM-streaming sums: column k (weight 2^(32k))
// holds a 64-bit sum c[k] of the products a_i b_j with i + j = k plus a count
// h[k] of its wraps (weight 2^(32k+64)).  One product is v_mad_u64_u32 into
// its column (carry-out to an SGPR pair) and one v_addc into the column's
// count: 32 VALU per mulacc and no register moves, against ~52 VALU plus ~25
// moves for acc9's carry-chained rows.  The 16 (mad, addc) pairs are issued
// with the addc three slots behind its mad through 4 rotating SGPR pairs,
// which covers gfx950's VALU-SGPR-write -> VALU-read wait states.
// Value = sum_k (c[k] + h[k] 2^64) 2^(32k) < 2^288.  Bound: column 3 takes
// four mads per product and each can wrap once into h[3], so the 32-bit counts
// stay exact for < 2^30 products per accumulator (launch_group_sums_eq checks
// a thread's trip count against kAcccolMaxProducts).
constexpr uint64_t kAcccolMaxProducts = 1ull << 30;
struct acccol {
  uint64_t c[7];  // columns 0..6 (a_3 b_3's high word sits in c[6]'s top half)
  uint32_t h[7];
};
__device__ __forceinline__ void acccol_zero(acccol& a) {
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    a.c[k] = 0;
    a.h[k] = 0;
  }
}
__device__ __forceinline__ void mulacc_col(acccol& s, const fe& x, const fe& y) {
  uint64_t cc0, cc1, cc2, cc3;  // carry-out pairs, rotated (product n uses pair n % 4)
  // one statement for all 16 products (columns 0..6 each get 1..4 products)
  asm volatile(
      "v_mad_u64_u32 %[C0], %[q0], %[x0], %[y0], %[C0]\n\t"  // n0  (0,0) col 0
      "v_mad_u64_u32 %[C1], %[q1], %[x0], %[y1], %[C1]\n\t"  // n1  (0,1) col 1
      "v_mad_u64_u32 %[C2], %[q2], %[x0], %[y2], %[C2]\n\t"  // n2  (0,2) col 2
      "v_addc_co_u32_e64 %[H0], %[q0], %[H0], 0, %[q0]\n\t"
      "v_mad_u64_u32 %[C3], %[q3], %[x0], %[y3], %[C3]\n\t"  // n3  (0,3) col 3
      "v_addc_co_u32_e64 %[H1], %[q1], %[H1], 0, %[q1]\n\t"
      "v_mad_u64_u32 %[C1], %[q0], %[x1], %[y0], %[C1]\n\t"  // n4  (1,0) col 1
      "v_addc_co_u32_e64 %[H2], %[q2], %[H2], 0, %[q2]\n\t"
      "v_mad_u64_u32 %[C2], %[q1], %[x1], %[y1], %[C2]\n\t"  // n5  (1,1) col 2
      "v_addc_co_u32_e64 %[H3], %[q3], %[H3], 0, %[q3]\n\t"
      "v_mad_u64_u32 %[C3], %[q2], %[x1], %[y2], %[C3]\n\t"  // n6  (1,2) col 3
      "v_addc_co_u32_e64 %[H1], %[q0], %[H1], 0, %[q0]\n\t"
      "v_mad_u64_u32 %[C4], %[q3], %[x1], %[y3], %[C4]\n\t"  // n7  (1,3) col 4
      "v_addc_co_u32_e64 %[H2], %[q1], %[H2], 0, %[q1]\n\t"
      "v_mad_u64_u32 %[C2], %[q0], %[x2], %[y0], %[C2]\n\t"  // n8  (2,0) col 2
      "v_addc_co_u32_e64 %[H3], %[q2], %[H3], 0, %[q2]\n\t"
      "v_mad_u64_u32 %[C3], %[q1], %[x2], %[y1], %[C3]\n\t"  // n9  (2,1) col 3
      "v_addc_co_u32_e64 %[H4], %[q3], %[H4], 0, %[q3]\n\t"
      "v_mad_u64_u32 %[C4], %[q2], %[x2], %[y2], %[C4]\n\t"  // n10 (2,2) col 4
      "v_addc_co_u32_e64 %[H2], %[q0], %[H2], 0, %[q0]\n\t"
      "v_mad_u64_u32 %[C5], %[q3], %[x2], %[y3], %[C5]\n\t"  // n11 (2,3) col 5
      "v_addc_co_u32_e64 %[H3], %[q1], %[H3], 0, %[q1]\n\t"
      "v_mad_u64_u32 %[C3], %[q0], %[x3], %[y0], %[C3]\n\t"  // n12 (3,0) col 3
      "v_addc_co_u32_e64 %[H4], %[q2], %[H4], 0, %[q2]\n\t"
      "v_mad_u64_u32 %[C4], %[q1], %[x3], %[y1], %[C4]\n\t"  // n13 (3,1) col 4
      "v_addc_co_u32_e64 %[H5], %[q3], %[H5], 0, %[q3]\n\t"
      "v_mad_u64_u32 %[C5], %[q2], %[x3], %[y2], %[C5]\n\t"  // n14 (3,2) col 5
      "v_addc_co_u32_e64 %[H3], %[q0], %[H3], 0, %[q0]\n\t"
      "v_mad_u64_u32 %[C6], %[q3], %[x3], %[y3], %[C6]\n\t"  // n15 (3,3) col 6
      "v_addc_co_u32_e64 %[H4], %[q1], %[H4], 0, %[q1]\n\t"
      "v_addc_co_u32_e64 %[H5], %[q2], %[H5], 0, %[q2]\n\t"
      "v_addc_co_u32_e64 %[H6], %[q3], %[H6], 0, %[q3]"
      : [C0] "+v"(s.c[0]), [C1] "+v"(s.c[1]), [C2] "+v"(s.c[2]), [C3] "+v"(s.c[3]),
        [C4] "+v"(s.c[4]), [C5] "+v"(s.c[5]), [C6] "+v"(s.c[6]), [H0] "+v"(s.h[0]),
        [H1] "+v"(s.h[1]), [H2] "+v"(s.h[2]), [H3] "+v"(s.h[3]), [H4] "+v"(s.h[4]),
        [H5] "+v"(s.h[5]), [H6] "+v"(s.h[6]), [q0] "=&s"(cc0), [q1] "=&s"(cc1), [q2] "=&s"(cc2),
        [q3] "=&s"(cc3)
      : [x0] "v"(x.w[0]), [x1] "v"(x.w[1]), [x2] "v"(x.w[2]), [x3] "v"(x.w[3]), [y0] "v"(y.w[0]),
        [y1] "v"(y.w[1]), [y2] "v"(y.w[2]), [y3] "v"(y.w[3]));
}
// Limbs of a column accumulator (< 2^288 by the bound above).
__device__ __forceinline__ acc9 acccol_limbs(const acccol& s) {
  acc9 r;
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    uint64_t t = carry;
    if (k < 7) t += (uint32_t)s.c[k];
    if (k >= 1 && k <= 7) t += s.c[k - 1] >> 32;
    if (k >= 2) t += s.h[k - 2];
    r.w[k] = (uint32_t)t;
    carry = t >> 32;
  }
  return r;
}

// Accumulator of the HBM-streaming corner-sum kernels.
#ifndef MLH_ACCCOL
#define MLH_ACCCOL 1
#endif
#if MLH_ACCCOL
using sacc = acccol;
__device__ __forceinline__ void sacc_zero(sacc& a) { acccol_zero(a); }
__device__ __forceinline__ void sacc_mac(sacc& a, const fe& x, const fe& y) { mulacc_col(a, x, y); }
__device__ __forceinline__ fe sacc_reduce(const sacc& a) { return acc_reduce(acccol_limbs(a)); }
#else
using sacc = acc9;
__device__ __forceinline__ void sacc_zero(sacc& a) { acc_zero(a); }
__device__ __forceinline__ void sacc_mac(sacc& a, const fe& x, const fe& y) { mulacc(a, x, y); }
__device__ __forceinline__ fe sacc_reduce(const sacc& a) { return acc_reduce(a); }
#endif

// Fold of 2^J values in registers (index MSB = the first variable) with
// r[0..J-1]; v[0] ends with the folded value.
template <int J>
__device__ __forceinline__ void fold_regs(fe (&v)[1 << J], const fe* r) {
#pragma unroll
  for (int u = 0; u < J; ++u) {
    const int half = (1 << J) >> (u + 1);
#pragma unroll
    for (int c = 0; c < half; ++c) v[c] = lerp_s(v[c], v[c + half], r[u]);
  }
}
// Fold of the 2^J corners src[c * stride] (c's MSB = the first variable) with
// r[0..J-1]: the folded table's entry.  J > 3: the top 3 variables per group
// of 8 loads first (8 values in flight, not 2^J), then the rest in registers.
template <int J>
__device__ __forceinline__ fe fold_corners(const fe* src, uint64_t stride, const fe* r) {
  if constexpr (J <= 3) {
    fe v[1 << J];
#pragma unroll
    for (int c = 0; c < (1 << J); ++c) v[c] = src[(uint64_t)c * stride];
    fold_regs<J>(v, r);
    return v[0];
  } else {
    constexpr int J2 = J - 3;
    fe part[1 << J2];
#pragma unroll
    for (int cl = 0; cl < (1 << J2); ++cl)
      part[cl] = fold_corners<3>(src + (uint64_t)cl * stride, stride << J2, r);
    fold_regs<J2>(part, r + 3);
    return part[0];
  }
}
__device__ __forceinline__ fe fold_corners_n(uint32_t J, const fe* src, uint64_t stride,
                                             const fe* r) {
  switch (J) {
    case 0: return src[0];
    case 1: return fold_corners<1>(src, stride, r);
    case 2: return fold_corners<2>(src, stride, r);
    default: return fold_corners<3>(src, stride, r);
  }
}

// Fold tables of size S with r (in place, first half) and emit the next
// round's sums over the folded tables (h' = S/4).
__global__ void __launch_bounds__(kRedThreads)
fold_sums_kernel(fe* m, fe* __restrict__ d, uint64_t S, fe r, fe* __restrict__ partials,
                 const fe* __restrict__ rp, const fe* msrc) {
  if (rp) r = fe_load(rp);
  const uint64_t h = S / 2, q = S / 4;
  fe s1 = fe_zero(), s2 = fe_zero();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < q; i += stride) {
    const fe ma = fe_load(msrc + i), mb = fe_load(msrc + i + q);
    const fe mc = fe_load(msrc + i + h), md = fe_load(msrc + i + h + q);
    const fe da = fe_load(d + i), db = fe_load(d + i + q);
    const fe dc = fe_load(d + i + h), dd = fe_load(d + i + h + q);
    const fe m0 = lerp(ma, mc, r), m1 = lerp(mb, md, r);
    const fe d0 = lerp(da, dc, r), d1 = lerp(db, dd, r);
    fe_store(m + i, m0);
    fe_store(m + i + q, m1);
    fe_store(d + i, d0);
    fe_store(d + i + q, d1);
    s1 = fe_add(s1, fe_mul(m1, d1));
    s2 = fe_add(s2, fe_mul(fe_sub(fe_dbl(m1), m0), fe_sub(fe_dbl(d1), d0)));
  }
  block_reduce2(s1, s2);
  if (threadIdx.x == 0) {
    fe_store(partials + 2 * blockIdx.x, s1);
    fe_store(partials + 2 * blockIdx.x + 1, s2);
  }
}

__global__ void __launch_bounds__(256)
fold_kernel(fe* m, fe* __restrict__ d, uint64_t S, fe r, const fe* __restrict__ rp,
            const fe* msrc) {
  if (rp) r = fe_load(rp);
  const uint64_t h = S / 2;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= h) return;
  fe_store(m + i, lerp(fe_load(msrc + i), fe_load(msrc + i + h), r));
  if (d) fe_store(d + i, lerp(fe_load(d + i), fe_load(d + i + h), r));  // d == null: m only
}

// ---- eq-factored rounds (delta never materialised) ---------------------------
// For the PCS tables delta = eq(p) (big-endian, sumcheck.rs:128-145) the fold
// keeps delta an eq table: folding the MSB variable (point p_k) with r gives
//   delta_{k+1}[i] = ((1-r)(1-p_k) + r p_k) * eq(p_{k+1..})[i],
// so round k's delta is c_k * eq(p_k, ..., p_{L-1}) with a running scalar c_k.
// Its halves are d[i] = c_k (1-p_k) e(i), d[i+h] = c_k p_k e(i) with
// e = eq(p_{k+1..}) over h entries, hence (composition x[0])
//   s1 = c_k p_k E1,  s2 = c_k (3 p_k - 1)(2 E1 - E0),
//   E0 = sum_{i<h} m[i] e(i),  E1 = sum_{i<h} m[i+h] e(i),
// and e(i) = H_k[i >> a] * lo[i mod 2^a] (lo = eq of the last a points, H_k =
// eq(p_{k+1}..p_{L-a-1}), eq_setup_kernel).  The kernels stream only m: half
// the HBM traffic of the two-table rounds, and no 2^L eq table is ever written.

// ---- grouped eq-factored rounds ------------------------------------------------
// A group of J consecutive head rounds k..k+J-1 is served by ONE read of
// its table T (S entries): with Q = S / 2^J and the corner sums
//   X_c = sum_{i<Q} T[c Q + i] e(i),  e = eq(p_{k+J}, ..., p_{L-1}) = H_{k+J-1}[i >> a] lo[..],
// round k+t's eq-factored sums are the contraction
//   E_b = sum_{c: c_t = b} prod_{u<t} (c_u ? r_{k+u} : 1 - r_{k+u})
//                          prod_{t<u<J} (c_u ? p_{k+u} : 1 - p_{k+u}) X_c
// (c_u = bit J-1-u of c: the group's first variable is the table's MSB).  The
// weights fold the t variables already challenged with their r's (the tables
// the per-round kernels would have folded) and expand eq over the rest, so the
// E0/E1 equal the per-round kernels' exactly.  One 16-B read and one modmul per
// element serve J rounds; the J folds are applied in one pass afterwards
// (fold_group_eq_kernel), which also emits the next group's corner sums.
// mlh_sumcheck_prove_eq takes 6 rounds per pass (64 corners, contracted as two
// chained 3-round groups in sumcheck_group_kernel); the PCS 3-round groups.

// corner sums X_c of a group of J rounds over T (S entries).  The grid is
// 2^J corners x nbc blocks (block = c * nbc + bb, so partials[block] is
// corner-major); a corner's nbc * 256 threads (a power of two >= 2^a) stride
// over its Q entries, so a thread's i mod 2^a is fixed and lo is applied once.
constexpr uint32_t kGroupHLds = 1024;
#ifndef MLH_GS_UNROLL
#define MLH_GS_UNROLL 8  // group_sums_eq_kernel: table entries in flight per thread
#endif
#ifndef MLH_GS_NBC_CAP
#define MLH_GS_NBC_CAP 16  // cap on group_sums_eq blocks per corner (fewer, longer blocks: measured faster)
#endif  // group_sums_eq_kernel: H entries staged in LDS (16 KiB)
__global__ void __launch_bounds__(kRedThreads)
group_sums_eq_kernel(const fe* __restrict__ T, uint64_t S, uint32_t J, const fe* H,
                     const fe* __restrict__ lo, uint32_t a, uint32_t nbc,
                     fe* __restrict__ partials) {
  const uint64_t Q = S >> J;
  const uint32_t c = blockIdx.x / nbc, bb = blockIdx.x % nbc;
  const fe* Tc = T + (uint64_t)c * Q;
  // H (Q >> a entries) from LDS when it fits: one vector-memory instruction
  // per element instead of two (the H reads are wave-uniform broadcasts)
  __shared__ fe hs[kGroupHLds];
  const uint64_t nh = Q >> a;
  if (nh <= kGroupHLds) {
    for (uint32_t k = threadIdx.x; k < nh; k += blockDim.x) hs[k] = fe_load(H + k);
    __syncthreads();
    H = hs;
  }
  sacc s0, s1;  // unreduced (two for ILP); < 2^288 for < 2^32 products each
  sacc_zero(s0);
  sacc_zero(s1);
  const uint64_t stride = (uint64_t)nbc * blockDim.x;
  const uint64_t i0 = (uint64_t)bb * blockDim.x + threadIdx.x;
  uint64_t i = i0;
  // MLH_GS_UNROLL entries in flight per thread (loads first, then the products)
  for (; i + (MLH_GS_UNROLL - 1) * stride < Q; i += MLH_GS_UNROLL * stride) {
    fe v[MLH_GS_UNROLL];
#pragma unroll
    for (int u = 0; u < MLH_GS_UNROLL; ++u) v[u] = fe_load(Tc + i + u * stride);
#pragma unroll
    for (int u = 0; u < MLH_GS_UNROLL; ++u) sacc_mac((u & 1) ? s1 : s0, v[u], fe_load(H + ((i + u * stride) >> a)));
  }
  for (; i < Q; i += stride) sacc_mac(s0, fe_load(Tc + i), fe_load(H + (i >> a)));
  fe acc = fe_add(sacc_reduce(s0), sacc_reduce(s1));
  if (i0 < Q) acc = fe_mul_s(acc, fe_load(lo + (i0 & ((1ull << a) - 1))));
  fe z = fe_zero();
  block_reduce2(acc, z);
  if (threadIdx.x == 0) fe_store(partials + blockIdx.x, acc);
}

// Fold T (S entries) over its J top variables with rs[0..J-1] into Tout
// (S / 2^J entries; Tout == T allowed: each output slot is read, as corner 0,
// only by the thread that writes it), and (JN > 0) the corner sums of the next
// group of JN rounds over the folded table (grid: 2^JN corners x nbc blocks,
// as group_sums_eq_kernel, but the eq weight applied per output: any stride).
template <int J, bool SPLIT>
__global__ void __launch_bounds__(kRedThreads)
fold_group_eq_kernel(const fe* Tin, uint64_t S, uint32_t JN, const fe* __restrict__ rs,
                     const fe* __restrict__ w, fe* Tout, const fe* __restrict__ H,
                     const fe* __restrict__ lo, uint32_t a, uint32_t nbc,
                     fe* __restrict__ partials) {
  // !SPLIT: the folded entry is the eq-weighted sum of its 2^J corners,
  //   Tout[x] = sum_c w_c Tin[c Sp + x],  w_c = prod_u (c_u ? r_u : 1 - r_u)
  // (the same field value as J rounds of lerps), accumulated unreduced with the
  // weights (sumcheck_group_kernel's output) broadcast from LDS.
  // SPLIT (J > 3, few outputs): 2^(J-3) lanes per output, lane l folds the 8
  // corners (c_hi, l) over the top 3 variables by lerps, then shuffle-lerps
  // combine the lanes over the rest (more loads in flight per output).
  constexpr int J2 = SPLIT && J > 3 ? J - 3 : 0, JH = J - J2;
  const uint64_t Sp = S >> J, Qp = Sp >> JN;
  const uint32_t co = blockIdx.x / nbc, bb = blockIdx.x % nbc;
  const uint32_t l = threadIdx.x & ((1u << J2) - 1);
  __shared__ fe wsh[SPLIT ? 1 : 1 << J];
  fe r[SPLIT ? J : 1];
  if constexpr (SPLIT) {
#pragma unroll
    for (int u = 0; u < J; ++u) r[u] = fe_load(rs + u);
  } else {
    if (threadIdx.x < (1u << J)) wsh[threadIdx.x] = fe_load(w + threadIdx.x);
    __syncthreads();
  }
  fe acc = fe_zero();
  const uint64_t stride = ((uint64_t)nbc * blockDim.x) >> J2;
  const uint64_t i0 = ((uint64_t)bb * blockDim.x + threadIdx.x) >> J2;
  // BUF: the !SPLIT loads through sweep_load (32-bit byte offsets: S <= 2^28)
  auto run = [&](auto BUF_) {
    constexpr bool BUF = decltype(BUF_)::value;
    for (uint64_t i = i0; i < Qp; i += stride) {
      const uint64_t x = (uint64_t)co * Qp + i;
      fe v;
      if constexpr (SPLIT) {
        v = fold_corners<JH>(Tin + (uint64_t)l * Sp + x, Sp << J2, r);
#pragma unroll
        for (int u = 0; u < J2; ++u) {
          const uint32_t m = 1u << (J2 - 1 - u);
          const fe o = shfl_xor_fe(v, m);
          const bool hi = l & m;
          v = lerp_s(hi ? o : v, hi ? v : o, r[JH + u]);
        }
      } else {
        acc9 t;  // (the column accumulator measured slower here: 24 registers per output)
        acc_zero(t);
#pragma unroll
        for (int c0 = 0; c0 < (1 << J); c0 += 8) {  // 8 loads in flight at a time
          fe tv[8];
#pragma unroll
          for (int c = 0; c < 8; ++c)
            if (c0 + c < (1 << J)) {
              const uint64_t ix = (uint64_t)(c0 + c) * Sp + x;
              tv[c] = BUF ? sweep_load(Tin, (uint32_t)ix) : fe_load(Tin + ix);
            }
#pragma unroll
          for (int c = 0; c < 8; ++c)
            if (c0 + c < (1 << J)) mulacc(t, tv[c], wsh[c0 + c]);
        }
        v = acc_reduce(t);
      }
      if (l == 0) {
        fe_store(Tout + x, v);
        // e(i) = H[i >> a] lo[i mod 2^a] in full: one output per 2^J inputs
        if (JN)
          acc = fe_add(acc, fe_mul_s(v, fe_mul_s(fe_load(H + (i >> a)),
                                                 fe_load(lo + (i & ((1ull << a) - 1))))));
      }
    }
  };
  if (!SPLIT && S <= (1ull << 28))
    run(std::true_type{});
  else
    run(std::false_type{});
  if (JN) {
    fe z = fe_zero();
    block_reduce2(acc, z);
    if (threadIdx.x == 0) fe_store(partials + blockIdx.x, acc);
  }
}

// out[i] = c * src[i], c read from HBM (the running eq scale c_k)
__global__ void scale_dev_kernel(const fe* __restrict__ src, const fe* __restrict__ c, uint64_t n,
                                 fe* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) fe_store(out + i, fe_mul(fe_load(c), fe_load(src + i)));
}

__global__ void __launch_bounds__(kRedThreads)
reduce_partials_kernel(const fe* __restrict__ partials, uint32_t nblocks, fe* __restrict__ out) {
  fe a = fe_zero(), b = fe_zero();
  for (uint32_t i = threadIdx.x; i < nblocks; i += blockDim.x) {
    a = fe_add(a, fe_load(partials + 2 * i));
    b = fe_add(b, fe_load(partials + 2 * i + 1));
  }
  block_reduce2(a, b);
  if (threadIdx.x == 0) {
    fe_store(out, a);
    fe_store(out + 1, b);
  }
}

// dot(a, b) partials (second slot unused = 0).
__global__ void __launch_bounds__(kRedThreads)
dot_kernel(const fe* __restrict__ a, const fe* __restrict__ b, uint64_t n,
           fe* __restrict__ partials) {
  fe s = fe_zero(), z = fe_zero();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    s = fe_add(s, fe_mul(fe_load(a + i), fe_load(b + i)));
  block_reduce2(s, z);
  if (threadIdx.x == 0) {
    fe_store(partials + 2 * blockIdx.x, s);
    fe_store(partials + 2 * blockIdx.x + 1, z);
  }
}

// Trace::evaluate (evaluation.rs:31-48) partials: columns [col0, col0 + ncols)
// of a row-major height x width trace dotted with the eq table.  256 threads
// = G = 256 / ncols row groups x ncols columns, so a group reads ncols
// consecutive elements of one row and the block a contiguous run of G rows.
__global__ void __launch_bounds__(kRedThreads)
trace_eval_kernel(const fe* __restrict__ m, const fe* __restrict__ eq, uint64_t height,
                  uint32_t width, uint32_t col0, uint32_t ncols, fe* __restrict__ partials) {
  __shared__ fe acc[kRedThreads];
  const uint32_t G = kRedThreads / ncols;
  const uint32_t g = threadIdx.x / ncols, j = threadIdx.x % ncols;
  fe s = fe_zero();
  if (g < G) {
    const uint64_t step = (uint64_t)gridDim.x * G;
    for (uint64_t i = (uint64_t)blockIdx.x * G + g; i < height; i += step)
      s = fe_add(s, fe_mul(fe_load(eq + i), fe_load(m + i * width + col0 + j)));
  }
  acc[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < ncols) {
    fe t = fe_zero();
    for (uint32_t q = 0; q < G; ++q) t = fe_add(t, acc[q * ncols + threadIdx.x]);
    fe_store(partials + (uint64_t)blockIdx.x * ncols + threadIdx.x, t);
  }
}

__global__ void trace_eval_finish_kernel(const fe* __restrict__ partials, uint32_t nblocks,
                                         uint32_t ncols, fe* __restrict__ out) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ncols) return;
  fe t = fe_zero();
  for (uint32_t b = 0; b < nblocks; ++b) t = fe_add(t, fe_load(partials + (uint64_t)b * ncols + j));
  fe_store(out + j, t);
}

// eq table of `cnt` points (big-endian): out[x] = prod_{i<cnt} (bit_i(x) ?
// p[cnt-1-i] : 1 - p[cnt-1-i]).
// mono: the monomial table instead, bit_i(x) ? p[cnt-1-i] : 1
// (MultilinearPolynomial::evaluate, polynomials.rs:126-146).
__global__ void eq_small_kernel(const fe* __restrict__ pts, uint32_t cnt, fe* __restrict__ out,
                                int mono) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= (1u << cnt)) return;
  fe acc = fe_one();
  for (uint32_t i = 0; i < cnt; ++i) {
    const fe p = pts[cnt - 1 - i];
    if ((x >> i) & 1u)
      acc = fe_mul(acc, p);
    else if (!mono)
      acc = fe_mul(acc, fe_sub(fe_one(), p));
  }
  fe_store(out + x, acc);
}

// Polynomial::evaluate (ntt/mod.rs:61-67, Horner) as sum_i c_i x^i with
// x^i = tlo[i mod 4096] * thi[i / 4096]: per-block partial sums.
__global__ void __launch_bounds__(kRedThreads)
poly_eval_kernel(const fe* __restrict__ c, uint64_t n, const fe* __restrict__ tlo,
                 const fe* __restrict__ thi, fe* __restrict__ partials) {
  fe s = fe_zero(), z = fe_zero();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    s = fe_add(s, fe_mul(fe_load(c + i), fe_mul(tlo[i & 4095], thi[i >> 12])));
  block_reduce2(s, z);
  if (threadIdx.x == 0) {
    fe_store(partials + 2 * blockIdx.x, s);
    fe_store(partials + 2 * blockIdx.x + 1, z);
  }
}

// delta[idx] = lo[idx & (2^a - 1)] * hi[idx >> a]
__global__ void __launch_bounds__(256)
eq_expand_kernel(const fe* __restrict__ lo, const fe* __restrict__ hi, uint32_t a, uint64_t n,
                 fe* __restrict__ out) {
  const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  fe_store(out + idx, fe_mul(lo[idx & ((1ull << a) - 1)], hi[idx >> a]));
}

// Moebius (sign = -1) / zeta (sign = +1) transform over `nbits` consecutive
// index bits [b0, b0 + nbits) of a 2^log_n table, src -> c (src may equal c:
// a tile is read whole before it is written).  A workgroup owns
// a tile of 8 adjacent low-index columns (or 8 consecutive elements of each
// row when b0 == 0) x 2^nbits rows staged in LDS.
template <int SIGN>
__global__ void __launch_bounds__(256)
mobius_pass_kernel(const fe* src, fe* c, uint32_t log_n, uint32_t b0, uint32_t nbits) {
  __shared__ fe lds[2048];
  const uint64_t W = 1ull << b0;  // row stride
  // columns = index bits below b0 (contiguous); tile = up to 8 of them
  const uint32_t lc = b0 < 3 ? b0 : 3;  // log2(cols)
  const uint32_t cmask = (1u << lc) - 1;
  const uint64_t lowcount = W >> lc;
  const uint64_t tile = blockIdx.x;
  const uint64_t hi = tile / lowcount, lo = tile % lowcount;
  const uint64_t base = (hi << (nbits + b0)) + (lo << lc);
  const uint32_t E = 1u << (nbits + lc);  // <= 2048
  for (uint32_t e = threadIdx.x; e < E; e += blockDim.x)
    lds[e] = fe_load(src + base + ((uint64_t)(e >> lc) << b0) + (e & cmask));
  __syncthreads();
  for (uint32_t b = 0; b < nbits; ++b) {
    const uint32_t bit = 1u << b;
    for (uint32_t e = threadIdx.x; e < E / 2; e += blockDim.x) {
      const uint32_t pr = e >> lc, col = e & cmask;  // pair index over rows
      const uint32_t r0 = (pr & (bit - 1)) | ((pr >> b) << (b + 1));
      const uint32_t i0 = (r0 << lc) + col, i1 = ((r0 | bit) << lc) + col;
      lds[i1] = SIGN < 0 ? fe_sub(lds[i1], lds[i0]) : fe_add(lds[i1], lds[i0]);
    }
    __syncthreads();
  }
  for (uint32_t e = threadIdx.x; e < E; e += blockDim.x)
    fe_store(c + base + ((uint64_t)(e >> lc) << b0) + (e & cmask), lds[e]);
  (void)log_n;
}

// The same transform over 8 index bits [b0, b0 + 8) with the butterflies in
// registers: a tile is 2^8 positions (the 8 bits) x 8 others (index bits 0..2
// when b0 >= 3: 128-byte runs; bits 8..10 when b0 = 0: consecutive blocks),
// 2048 elements; each thread holds 8 elements and applies 3 of the bits in
// registers, 3 more after one LDS exchange and the last 2 after a second --
// two exchanges instead of one LDS read-modify-write sweep per bit.  (Moebius
// steps for different bits commute, so any order of the bits is the same map.)
template <int SIGN>
__device__ __forceinline__ void mobius_reg(fe (&v)[8], uint32_t jbits) {
#pragma unroll
  for (uint32_t b = 0; b < 3; ++b) {
    if (!((jbits >> b) & 1u)) continue;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j)
      if (j & (1u << b)) v[j] = SIGN < 0 ? fe_sub(v[j], v[j ^ (1u << b)]) : fe_add(v[j], v[j ^ (1u << b)]);
  }
}
template <int SIGN>
__global__ void __launch_bounds__(256)
mobius_pass8_kernel(const fe* src, fe* c, uint32_t b0) {
  __shared__ fe lds[2048];
  const uint32_t t = threadIdx.x;
  const bool lowb = b0 == 0;
  // thread -> (o, g): lanes along the contiguous index direction
  const uint32_t o = lowb ? t >> 5 : t & 7, g = lowb ? t & 31 : t >> 3;
  const uint64_t W = 1ull << b0;
  uint64_t base;  // index of (p = 0, o = 0)
  if (lowb) {
    base = (uint64_t)blockIdx.x << 11;
  } else {
    const uint64_t lowcount = W >> 3, tile = blockIdx.x;
    base = ((tile / lowcount) << (b0 + 8)) + ((tile % lowcount) << 3);
  }
  auto gidx = [&](uint32_t p) -> uint64_t { return lowb ? base + (o << 8) + p : base + p * W + o; };
  auto lidx = [&](uint32_t p) -> uint32_t { return lowb ? (o << 8) + p : (p << 3) + o; };
  fe v[8];
  // round 1: positions g + 32 j (bits 5, 6, 7 in registers)
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) v[j] = fe_load(src + gidx(g + 32 * j));
  mobius_reg<SIGN>(v, 7);
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) lds[lidx(g + 32 * j)] = v[j];
  __syncthreads();
  // round 2: positions (g & 3) + 4 j + 32 (g >> 2) (bits 2, 3, 4)
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) v[j] = lds[lidx((g & 3) + 4 * j + 32 * (g >> 2))];
  mobius_reg<SIGN>(v, 7);
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) lds[lidx((g & 3) + 4 * j + 32 * (g >> 2))] = v[j];
  __syncthreads();
  // round 3: positions (j & 3) + 4 (j >> 2) + 8 g (bits 0, 1)
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) v[j] = lds[lidx((j & 3) + 4 * (j >> 2) + 8 * g)];
  mobius_reg<SIGN>(v, 3);
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) fe_store(c + gidx((j & 3) + 4 * (j >> 2) + 8 * g), v[j]);
}

// out[i] = in[bitrev(i)] (bit_reverse_permutation, src/ntt/mod.rs:113-123).
__global__ void __launch_bounds__(256)
bitrev_kernel(const fe* __restrict__ in, fe* __restrict__ out, uint32_t log_n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (1ull << log_n)) return;
  const uint64_t j = log_n ? (__builtin_bitreverse64(i) >> (64 - log_n)) : 0;
  fe_store(out + i, fe_load(in + j));
}

// ---- PCS rounds off the transcript kernel ----------------------------------
// (the round body: sc_dev.hpp pcs_round_body; also run by an extra workgroup
// of the FRI fold kernel, fri.hip)
__global__ void __launch_bounds__(kRedThreads) pcs_round_kernel(PcsJob job) { pcs_round_body(job); }

// wf[c] = prod_{u<JA} (c_u ? r_u : 1 - r_u), wf[64 + c] the same over
// r_{JA..JA+JB-1} (c_u = bit J-1-u of c): fold_group_eq's weights of two groups.
__global__ void eq_weights_kernel(const fe* __restrict__ rs, uint32_t JA, uint32_t JB,
                                  fe* __restrict__ wf) {
  const uint32_t t = threadIdx.x;
  const bool B = t >= 64;
  const uint32_t c = t & 63, J = B ? JB : JA;
  if (c >= (1u << J)) return;
  const fe one = fe_one();
  fe w = one;
  for (uint32_t u = 0; u < J; ++u) {
    const fe r = fe_load(rs + (B ? JA : 0) + u);
    w = fe_mul_s(w, (c >> (J - 1 - u)) & 1u ? r : fe_sub(one, r));
  }
  fe_store(wf + t, w);
}

// ---- launchers -------------------------------------------------------------

static inline unsigned red_blocks(uint64_t work) {
  uint64_t b = (work + kRedThreads - 1) / kRedThreads;
  if (b > kMaxRedBlocks) b = kMaxRedBlocks;
  if (b == 0) b = 1;
  return (unsigned)b;
}

hipError_t launch_sums(const fe* m, const fe* d, uint64_t h, fe* partials, fe* out,
                       hipStream_t st, uint32_t* nparts) {
  const unsigned nb = red_blocks(h);
  hipLaunchKernelGGL(sums_kernel, dim3(nb), dim3(kRedThreads), 0, st, m, d, h, partials);
  if (nparts)
    *nparts = nb;  // the caller reduces (sumcheck_round_kernel)
  else
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(kRedThreads), 0, st, partials, nb,
                       out);
  return hipGetLastError();
}

hipError_t launch_fold_sums(fe* m, fe* d, uint64_t S, fe r, fe* partials, fe* out,
                            hipStream_t st, const fe* r_dev, uint32_t* nparts, const fe* m_src) {
  const unsigned nb = red_blocks(S / 4);
  hipLaunchKernelGGL(fold_sums_kernel, dim3(nb), dim3(kRedThreads), 0, st, m, d, S, r, partials,
                     r_dev, m_src ? m_src : m);
  if (nparts)
    *nparts = nb;
  else
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(kRedThreads), 0, st, partials, nb,
                       out);
  return hipGetLastError();
}

hipError_t launch_fold(fe* m, fe* d, uint64_t S, fe r, hipStream_t st, const fe* r_dev,
                       const fe* m_src) {
  const uint64_t h = S / 2;
  hipLaunchKernelGGL(fold_kernel, dim3((unsigned)((h + 255) / 256)), dim3(256), 0, st, m, d, S, r,
                     r_dev, m_src ? m_src : m);
  return hipGetLastError();
}

// One launch for the eq-factored sumcheck's setup (EqSetupArgs by value, so no
// host-to-device copies): lo = eq(p_B..p_{L-1}) (2^a), the head suffix tables
// H (2^B - 1, as eq_suffix_kernel over p_0..p_{B-1}), the tail suffix tables
// Hs (2^a - 1, over p_B..p_{L-1}; optional); thread 0 also writes the points,
// c_0 = 1 and (optional) the transcript state and the claim.
#ifndef MLH_SETUP_TREE
#define MLH_SETUP_TREE 1
#endif
#ifndef MLH_TAIL_DMA
#define MLH_TAIL_DMA 1  // sumcheck_eq_tail_kernel: wave 3 copies the table by LDS-DMA (xc_part launches)
#endif
__global__ void __launch_bounds__(256)
eq_setup_kernel(const EqSetupArgs args, fe* __restrict__ pts_out, fe* __restrict__ c_out,
                fe* __restrict__ lo, fe* __restrict__ H, fe* __restrict__ Hs, DevSha* dt_out,
                fe* prev_out, uint32_t* __restrict__ kw, fe* __restrict__ rsuf) {
  const uint32_t L = args.L, B = args.B, a = L - B;
  const uint64_t NL = 1ull << a, NH = (1ull << B) - 1, NS = Hs ? NL - 1 : 0;
  uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // after the tables, from a wave boundary (so no table wave also runs these
  // paths): one wave of copies -- lane i < L point i, lane 40 c_0, lane 41 the
  // claim, lanes 48.. the transcript state's words -- then kw: per round k
  // whose absorb of (c1, c2) empties the buffer, the padding block's K + W
  // table (the transcript then grows 32 bytes per round)
  const uint64_t NT = (NL + NH + NS + 63) & ~63ull;
  if (x >= NT) {
    const uint32_t y = (uint32_t)(x - NT);
    if (y < 64) {
      if (y < L) pts_out[y] = args.pts[y];
      if (y == 40) *c_out = fe_one();
      if (y == 41 && prev_out) *prev_out = args.sum;
      constexpr uint32_t SW = sizeof(DevSha) / 8;
      static_assert(sizeof(DevSha) % 8 == 0 && SW <= 16, "DevSha copy");
      if (dt_out && y >= 48 && y < 48 + SW)
        reinterpret_cast<uint2*>(dt_out)[y - 48] = reinterpret_cast<const uint2*>(&args.sha)[y - 48];
    } else if (y < 128) {
      if (kw && y - 64 < L) {
        const uint32_t k = y - 64;
        const uint64_t len = args.sha.len + 32ull * (k + 1);
        if ((len & 63) == 0) sha256_pad_kw(len, kw + 64 * k);
      }
    } else if (rsuf && y - 128 < 2 * kEqTailRsuf) {
      // the suffix products of the eq tail's (h = 0: points p_B..) and the
      // eq head's (h = 1: p_0..p_{B-1}, when B <= 12) corner groups, moved
      // off those launches' critical paths (their prologue's
      // suffix_products): group g = 0 over the first JA = min(n, 6) points,
      // g = 1 over the next n - JA; rs[u][c] = prod_{u<v<J} (bit J-1-v of c
      // ? p_v : 1 - p_v)
      const uint32_t h = (y - 128) / kEqTailRsuf, z = (y - 128) % kEqTailRsuf;
      const uint32_t g = z / 384, u = (z % 384) / 64, c = z % 64;
      const uint32_t n = h ? (B <= 12 ? B : 0) : a;
      const uint32_t JA = n < 6 ? n : 6, J = g ? n - JA : JA;
      if (u < J) {
        const fe* pv = args.pts + (h ? 0 : B) + (g ? JA : 0);
        const fe one = fe_one();
        fe acc = one;
        for (uint32_t v = J - 1; v > u; --v) {
          const fe p = fe_vgpr(pv[v]);
          acc = fe_mul_s(acc, ((c >> (J - 1 - v)) & 1u) ? p : fe_sub(one, p));
        }
        fe_store(rsuf + (y - 128), acc);
      }
    }
    return;
  }
  // entry j of an eq suffix family over points q[0..n): the table of index k
  // (2^(n-1-k) entries at offset 2^n - 2^(n-k)) = prod_{i < n-1-k} (bit_i(j) ?
  // q[n-1-i] : 1 - q[n-1-i]); lo = the family's "k = -1" table (n factors)
  const fe* q;
  uint32_t n, cnt;
  uint64_t j;
  fe* out;
  if (x < NL) {
    q = args.pts + B; n = a; cnt = a; j = x; out = lo + x;
  } else if ((x -= NL) < NH) {
    const uint64_t y = (1ull << B) - x;
    const uint32_t k = B - (64 - __builtin_clzll(y - 1));
    q = args.pts; n = B; cnt = B - 1 - k; j = x - ((1ull << B) - (1ull << (B - k))); out = H + x;
  } else if ((x -= NH) < NS) {
    const uint64_t y = NL - x;
    const uint32_t k = a - (64 - __builtin_clzll(y - 1));
    q = args.pts + B; n = a; cnt = a - 1 - k; j = x - (NL - (NL >> k)); out = Hs + x;
  } else {
    return;
  }
  // (the chain of products is the launch's critical path, one thread per
  // entry: the generated asm multiply, operands in VGPRs)
#if MLH_SETUP_TREE
  // the first 12 factors as a product tree (depth 4 instead of a chain of up
  // to 12: one wave per SIMD here, so the products' latency is the launch's
  // time), the rest (cnt > 12: heads of more than 13 variables) chained on
  const fe one = fe_one();
  fe f[12];
#pragma unroll
  for (uint32_t i = 0; i < 12; ++i) {
    f[i] = one;
    if (i < cnt) {
      const fe p = fe_vgpr(q[n - 1 - i]);
      f[i] = ((j >> i) & 1) ? p : fe_sub(one, p);
    }
  }
#pragma unroll
  for (uint32_t i = 0; i < 6; ++i) f[i] = fe_mul_s(f[2 * i], f[2 * i + 1]);
#pragma unroll
  for (uint32_t i = 0; i < 3; ++i) f[i] = fe_mul_s(f[2 * i], f[2 * i + 1]);
  fe acc = fe_mul_s(fe_mul_s(f[0], f[1]), f[2]);
  for (uint32_t i = 12; i < cnt; ++i) {
    const fe p = fe_vgpr(q[n - 1 - i]);
    acc = fe_mul_s(acc, ((j >> i) & 1) ? p : fe_sub(one, p));
  }
#else
  fe acc = fe_one();
  for (uint32_t i = 0; i < cnt; ++i) {
    const fe p = fe_vgpr(q[n - 1 - i]);
    acc = fe_mul_s(acc, ((j >> i) & 1) ? p : fe_sub(fe_one(), p));
  }
#endif
  fe_store(out, acc);
}

hipError_t launch_eq_setup(const EqSetupArgs& args, fe* pts_out, fe* c_out, fe* lo, fe* H, fe* Hs,
                           DevSha* dt_out, fe* prev_out, hipStream_t st, uint32_t* kw,
                           fe* rsuf_out) {
  if (args.L == 0 || args.L > 40 || args.B > args.L || args.L - args.B > kTailLogMax)
    return hipErrorInvalidValue;
  const uint64_t NL = 1ull << (args.L - args.B);
  const uint64_t total = ((NL + (1ull << args.B) - 1 + (Hs ? NL - 1 : 0) + 63) & ~63ull) + 128 +
                         (rsuf_out ? 2 * kEqTailRsuf : 0);
  hipLaunchKernelGGL(eq_setup_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, args,
                     pts_out, c_out, lo, H, Hs, dt_out, prev_out, kw, rsuf_out);
  return hipGetLastError();
}

// grouped kernels: per corner nbc blocks (a power of two), the corners x nbc
// partials within the 2 * kMaxRedBlocks buffer; work >= 2^a keeps a corner's
// stride a multiple of 2^a
static inline unsigned group_blocks(uint64_t work, uint32_t corners) {
  uint64_t b = work / (4 * kRedThreads);  // >= 4 entries per thread
  const uint64_t cap = 2ull * kMaxRedBlocks / corners;
  if (b > cap) b = cap;
  return (unsigned)(b ? b : 1);
}

hipError_t launch_group_sums_eq(const fe* T, uint64_t S, uint32_t J, const fe* H, const fe* lo,
                                uint32_t a, fe* partials, hipStream_t st, uint32_t* nb) {
  if (J < 1 || J > kMaxGroup || a < 8 || (S >> J) < (1ull << a)) return hipErrorInvalidValue;
  uint32_t nbc = group_blocks(S >> J, 1u << J);
  if (MLH_GS_NBC_CAP && nbc > MLH_GS_NBC_CAP) nbc = MLH_GS_NBC_CAP;
  while ((uint64_t)nbc * kRedThreads < (1ull << a)) nbc *= 2;  // stride >= 2^a
  if ((nbc << J) > 2 * kMaxRedBlocks) return hipErrorInvalidValue;
  // products per thread accumulator: Q / (nbc * threads) entries of its corner
  if (((S >> J) + (uint64_t)nbc * kRedThreads - 1) / ((uint64_t)nbc * kRedThreads) >= kAcccolMaxProducts)
    return hipErrorInvalidValue;
  *nb = nbc;
  hipLaunchKernelGGL(group_sums_eq_kernel, dim3(nbc << J), dim3(kRedThreads), 0, st, T, S, J, H, lo,
                     a, nbc, partials);
  return hipGetLastError();
}

hipError_t launch_fold_group_eq(const fe* Tin, uint64_t S, uint32_t J, uint32_t JN, const fe* rs,
                                const fe* w, fe* Tout, const fe* H, const fe* lo, uint32_t a,
                                fe* partials, hipStream_t st, uint32_t* nb) {
  // (a < 8 only in the tail form: 2^a outputs per corner, e = lo, H = [1])
  if (J < 1 || J > kMaxGroup || JN > kMaxGroup || (S >> (J + JN)) < (1ull << a) || !w ||
      (a < 8 && !(JN && (S >> (J + JN)) == (1ull << a))))
    return hipErrorInvalidValue;
#ifndef MLH_FOLD_SPLIT
#define MLH_FOLD_SPLIT (1u << 16)  // outputs below which a J > 3 fold splits across lanes
#endif
  const bool split = J > 3 && (S >> J) < MLH_FOLD_SPLIT;
  const uint32_t lanes = split ? 1u << (J - 3) : 1u;  // threads per output
  const uint64_t work = (S >> (J + JN)) * lanes;      // threads per output corner
  uint32_t nbc = (uint32_t)(work / kRedThreads < 1 ? 1 : work / kRedThreads);
  const uint32_t cap = (2 * kMaxRedBlocks) >> JN;
  if (nbc > cap) nbc = cap;
  *nb = nbc;
  const dim3 g(nbc << JN), b(kRedThreads);
#define MLH_FOLD_J(j, sp)                                                                   \
  if (J == j && split == sp)                                                                \
    hipLaunchKernelGGL((fold_group_eq_kernel<j, sp>), g, b, 0, st, Tin, S, JN, rs, w, Tout, H, lo, \
                       a, nbc, partials);
  MLH_FOLD_J(1, false) MLH_FOLD_J(2, false) MLH_FOLD_J(3, false)
  MLH_FOLD_J(4, false) MLH_FOLD_J(5, false) MLH_FOLD_J(6, false)
  MLH_FOLD_J(4, true) MLH_FOLD_J(5, true) MLH_FOLD_J(6, true)
#undef MLH_FOLD_J
  return hipGetLastError();
}

hipError_t launch_scale_dev(const fe* src, const fe* c, uint64_t n, fe* out, hipStream_t st) {
  hipLaunchKernelGGL(scale_dev_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, c,
                     n, out);
  return hipGetLastError();
}

hipError_t launch_poly_eval(const fe* c, uint64_t n, const fe* tlo, const fe* thi, fe* partials,
                            fe* out, hipStream_t st) {
  const unsigned nb = red_blocks(n);
  hipLaunchKernelGGL(poly_eval_kernel, dim3(nb), dim3(kRedThreads), 0, st, c, n, tlo, thi,
                     partials);
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(kRedThreads), 0, st, partials, nb, out);
  return hipGetLastError();
}

hipError_t launch_dot(const fe* a, const fe* b, uint64_t n, fe* partials, fe* out,
                      hipStream_t st) {
  const unsigned nb = red_blocks(n);
  hipLaunchKernelGGL(dot_kernel, dim3(nb), dim3(kRedThreads), 0, st, a, b, n, partials);
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(kRedThreads), 0, st, partials, nb, out);
  return hipGetLastError();
}

uint32_t trace_eval_blocks(uint64_t height, uint32_t ncols) {
  const uint64_t G = kRedThreads / ncols;
  uint64_t b = (height + G - 1) / G;
  if (b > 1024) b = 1024;
  return (uint32_t)(b ? b : 1);
}

hipError_t launch_trace_eval(const fe* m, const fe* eq, uint64_t height, uint32_t width,
                             fe* partials, fe* out, hipStream_t st) {
  for (uint32_t col0 = 0; col0 < width; col0 += kRedThreads) {
    const uint32_t nc = width - col0 < (uint32_t)kRedThreads ? width - col0 : kRedThreads;
    const uint32_t nb = trace_eval_blocks(height, nc);
    hipLaunchKernelGGL(trace_eval_kernel, dim3(nb), dim3(kRedThreads), 0, st, m, eq, height, width,
                       col0, nc, partials);
    hipLaunchKernelGGL(trace_eval_finish_kernel, dim3((nc + 63) / 64), dim3(64), 0, st, partials,
                       nb, nc, out + col0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// pts: n device points; scratch: 2^(n-a) + 2^a elements.
hipError_t launch_eq_table(const fe* pts, uint32_t n, fe* scratch, fe* out, hipStream_t st,
                           bool mono) {
  const uint32_t a = n / 2, b = n - a;
  fe* lo = scratch;
  fe* hi = scratch + (1u << a);
  // lo: last a points (bits 0..a-1), hi: first b points (bits a..n-1)
  hipLaunchKernelGGL(eq_small_kernel, dim3(((1u << a) + 255) / 256), dim3(256), 0, st, pts + b, a,
                     lo, mono ? 1 : 0);
  hipLaunchKernelGGL(eq_small_kernel, dim3(((1u << b) + 255) / 256), dim3(256), 0, st, pts, b, hi,
                     mono ? 1 : 0);
  const uint64_t N = 1ull << n;
  hipLaunchKernelGGL(eq_expand_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, lo, hi,
                     a, N, out);
  return hipGetLastError();
}

hipError_t launch_mobius(fe* c, uint32_t log_n, bool inverse_zeta, hipStream_t st,
                         const fe* src) {
  if (!src) src = c;
  if (log_n == 0 && src != c) {
    hipError_t e = hipMemcpyAsync(c, src, sizeof(fe), hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return e;
  }
  uint32_t b0 = 0;
  while (b0 < log_n) {
    const uint32_t nb = (log_n - b0) < 8 ? (log_n - b0) : 8;
#ifndef MLH_MOBIUS_REG
#define MLH_MOBIUS_REG 1
#endif
    if (MLH_MOBIUS_REG && nb == 8 && log_n >= 11 && (b0 == 0 || b0 >= 3)) {
      const unsigned tiles = (unsigned)((1ull << log_n) >> 11);
      if (inverse_zeta)
        hipLaunchKernelGGL(mobius_pass8_kernel<1>, dim3(tiles), dim3(256), 0, st, src, c, b0);
      else
        hipLaunchKernelGGL(mobius_pass8_kernel<-1>, dim3(tiles), dim3(256), 0, st, src, c, b0);
      src = c;
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      b0 += 8;
      continue;
    }
    const uint64_t W = 1ull << b0;
    const uint64_t cols = W < 8 ? W : 8;
    // tile: 2^nb rows x cols elements must fit 2048 LDS slots
    uint32_t bits = nb;
    while ((1ull << bits) * cols > 2048) --bits;
    const uint64_t tiles = (1ull << log_n) / ((1ull << bits) * cols);
    if (inverse_zeta)
      hipLaunchKernelGGL(mobius_pass_kernel<1>, dim3((unsigned)tiles), dim3(256), 0, st, src, c,
                         log_n, b0, bits);
    else
      hipLaunchKernelGGL(mobius_pass_kernel<-1>, dim3((unsigned)tiles), dim3(256), 0, st, src, c,
                         log_n, b0, bits);
    src = c;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    b0 += bits;
  }
  return hipSuccess;
}

hipError_t launch_bitrev(const fe* in, fe* out, uint32_t log_n, hipStream_t st) {
  const uint64_t N = 1ull << log_n;
  hipLaunchKernelGGL(bitrev_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, in, out,
                     log_n);
  return hipGetLastError();
}

}  // namespace mlh

// ---- one sumcheck round with the transcript on the device -------------------
namespace mlh {

// Lane-0 round step: (s1, s2) = p(1), p(2) and the claim p(0) + p(1) ->
// interpolate (closed form on x = 0,1,2), store (c1, c2), absorb them, draw
// r (stored to r_out) and advance the claim to p(r).
// round_step on wave 0 (s1, s2, claim: thread 0's, made wave-uniform): the
// closed-form interpolation, the absorb and the challenge on the lane pair
// (dsha2l_step); thread 0 writes the polynomial and returns with the claim p(r).
__device__ __forceinline__ uint32_t lane0_u32(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ fe lane0_fe(const fe& x) {
  fe y;
#pragma unroll
  for (int i = 0; i < 4; ++i) y.w[i] = lane0_u32(x.w[i]);
  return y;
}
__device__ __forceinline__ fe round_step_wave(fe s1, fe s2, fe& claim, DevSha& s, uint32_t* stage,
                                              fe* poly_out, fe* r_out) {
  s1 = lane0_fe(s1);
  s2 = lane0_fe(s2);
  claim = lane0_fe(claim);
  const fe e0 = fe_sub(claim, s1);
  const fe c2 = fe_half(fe_add(fe_sub(s2, fe_add(s1, s1)), e0));
  const fe c1 = fe_sub(fe_sub(s1, e0), c2);
  if (threadIdx.x == 0) {
    fe_store(poly_out, c1);
    fe_store(poly_out + 1, c2);
  }
  const uint32_t w[8] = {c1.w[0], c1.w[1], c1.w[2], c1.w[3], c2.w[0], c2.w[1], c2.w[2], c2.w[3]};
  const fe r = dsha2l_step<8>(s, w, stage, r_out);  // LE16(c1) || LE16(c2), next_challenge()
  claim = fe_add(e0, fe_mul(r, fe_add(c1, fe_mul(c2, r))));
  return r;
}
// One two-table round (mlh_sumcheck_prove's per-round path, the PCS's rounds
// after the eq-factored head, mlh_device_sumcheck_round): reduce the
// per-workgroup partial (s1, s2) = p(1), p(2) pairs, then wave 0 runs
// round_step_wave (the closed-form interpolation on x = 0,1,2 of
// polynomials.rs:51-87, absorb LE16(c1) || LE16(c2) as sumcheck.rs:188-199,
// r = next_challenge() on the lane pair, claim = p(r)).
__global__ void __launch_bounds__(kRedThreads)
sumcheck_round_kernel(const fe* __restrict__ partials, uint32_t nparts, fe* prev, DevSha* t,
                      fe* poly_out, fe* r_out) {
  __shared__ DevSha s;
  __shared__ uint32_t stage[8];
  // the transcript state (one word per lane) and the claim are loaded first, so
  // their latency overlaps the partial-sum reduction
  if (threadIdx.x < sizeof(DevSha) / 4)
    reinterpret_cast<uint32_t*>(&s)[threadIdx.x] = reinterpret_cast<const uint32_t*>(t)[threadIdx.x];
  fe p = fe_zero();
  if (threadIdx.x == 0) p = fe_load(prev);
  // loads unrolled so a lane's few loads are in flight together
  fe s1 = fe_zero(), s2 = fe_zero();
#pragma unroll 4
  for (uint32_t i = threadIdx.x; i < nparts; i += kRedThreads) {
    s1 = fe_add(s1, fe_load(partials + 2 * i));
    s2 = fe_add(s2, fe_load(partials + 2 * i + 1));
  }
  block_reduce2(s1, s2);  // (its barriers also publish the staged state)
  if (threadIdx.x >= 64) return;
  round_step_wave(s1, s2, p, s, stage, poly_out, r_out);
  if (threadIdx.x == 0) {
    *t = s;
    fe_store(prev, p);
  }
}

// out = P + Q (R + S T): the one two-modmul form every lane-parallel step of
// sumcheck_group_kernel is cast in, so independent chains (corner weights,
// the claim p(r), the eq scale) run side by side on different lanes.
__device__ __forceinline__ fe pqrst(const fe& P, const fe& Q, const fe& R, const fe& S,
                                    const fe& T) {
  return fe_add(P, fe_mul_s(fe_add(R, fe_mul_s(S, T)), Q));
}
// (fe_vgpr: sc_dev.hpp)
// An LDS entry every lane reads (a uniform address) into VGPRs.
__device__ __forceinline__ fe lds_fe(const fe& x) { return fe_vgpr(x); }
// The same lane's value as a wave-uniform (v_readlane): no LDS round trip.
__device__ __forceinline__ fe bcast_fe(const fe& x, int src) {
  fe r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.w[i] = (uint32_t)__builtin_amdgcn_readlane((int)x.w[i], src);
  return fe_vgpr(r);
}
__device__ __forceinline__ fe shfl_fe(const fe& x, int src) {
  fe r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.w[i] = (uint32_t)__shfl((int)x.w[i], src, 64);
  return r;
}

// ---- serial rounds: a transcript wave and helper waves ----------------------
// A round's Fiat-Shamir step is one lane's SHA-256 work (1.5 compressions per
// round on average) and cannot be shortened; everything else is taken off
// that chain.  Round t's polynomial (c1, c2) depends on the previous challenge
// r_{t-1} only through quadratics: E_b(t) = A_b + r B_b (the only weight
// factor or fold involving r_{t-1} is linear in it), the eq scale c_t = U + V r
// and the claim p_{t-1}(r) = e0 + c1 r + c2 r^2, hence with
//   X(r) = p_t c_t E1 = s1,  Y(r) = c_t ((3 p_t - 1)(2 E1 - E0) - 3 p_t E1) = s2 - 3 s1,
//   c2 = (Y + claim) / 2,  c1 = 2 X - claim - c2,  e0' = claim - X
// they are quadratics in r_{t-1} whose coefficients need r_{t-2} but not
// r_{t-1}.  A helper wave (the "lead") builds round t's coefficients while
// wave 0 runs the SHA-256 of round t-1; wave 0 only evaluates two quadratics
// (two dependent products on two lanes), absorbs (c1, c2) and draws r_t.
// Exchange through LDS: per round parity the four quadratics (c1, c2, e0', c),
// the published challenges, and sequence counters (release / acquire at
// workgroup scope).  A wait longer than the spin limit sets `fail` and gives
// up instead of hanging the device; the kernel then reports it (CoopCtl) and
// the prove returns MLH_ERR_DEVICE.
//
// The lead works on corner sums (see "grouped eq-factored rounds"): lane c of
// its wave is corner c of a group of J <= 6 variables (c_u = bit J-1-u), with
// L_c = X_c prod_{challenged u} (c_u ? r_u : 1 - r_u) and the suffix products
// Rs_u = prod_{u<v<J} (c_v ? p_v : 1 - p_v); round u's E_b sums L_c Rs_u over
// c_u = b, split by c_{u-1} (whose factor is the one linear in r_{u-1}).
struct CoopSync {
  fe poly[2][12];    // round parity -> c1 | c2 | e0' | eq scale (k0, k1, k2) in r_{t-1}
  fe rsh[64];        // r of each round of the launch (relative index)
  fe red[4][2];      // per-wave partial sums
  fe pg[16];         // the launch's points, by variable
  fe xc[64];         // corner sums of the first group
  fe rsuf[6][64];    // Rs of the first group (per corner lane; runtime-indexed: LDS)
  fe rsufB[6][64];   // ... of the eq tail's second group
  fe ab[2][4];       // round parity -> A0, B0, A1, B1 (corner wave -> coefficient wave)
  uint32_t coef_seq, r_seq, hbar, mseq, fail, ab_seq, spin_limit;
  // transcript wave: working state after round 7 of the last half-block
  // challenge and the transcript length it belongs to (sha256_rounds_from)
  uint32_t mid[8];
  uint64_t mid_len;
};

// Per-round timestamps of the cooperative kernels (tools/coop_bench.hip builds
// this file with -DMLH_COOP_PROF; compiled out otherwise): [0][k] wave 0
// starts waiting for round k's slot, [1][k] has it, [2][k] has absorbed,
// [3][k] published r_k, [4][k] the lead published round k's slot, [5..8][k]
// the lead's phases.
#ifdef MLH_COOP_PROF
__device__ uint64_t g_coop_ts[10][64];
__device__ uint64_t g_coop_edge[4];  // kernel entry / roles start: s_memtime, wall_clock64
#define MLH_COOP_EDGE(i)                                         \
  do {                                                           \
    if (threadIdx.x == 0) {                                      \
      g_coop_edge[2 * (i)] = __builtin_amdgcn_s_memtime();       \
      g_coop_edge[2 * (i) + 1] = wall_clock64();                 \
    }                                                            \
  } while (0)
#define MLH_COOP_TS(e, k)                                                                    \
  do {                                                                                       \
    if ((threadIdx.x & 63) == 0 && (k) < 64) g_coop_ts[e][k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define MLH_COOP_TS(e, k) \
  do {                    \
  } while (0)
#define MLH_COOP_EDGE(i) \
  do {                   \
  } while (0)
#endif

__device__ __forceinline__ void lds_publish(uint32_t* f, uint32_t v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Waits for *f >= v.  Gives up (sets S.fail) after S.spin_limit sleeps, or at
// once when another wave already gave up, so one stalled wave costs one limit,
// not one per remaining wait.
__device__ __forceinline__ void lds_wait_ge(CoopSync& S, uint32_t* f, uint32_t v) {
  const uint32_t lim = S.spin_limit;
  for (uint32_t n = 0; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < v;) {
    __builtin_amdgcn_s_sleep(1);
    if (++n >= lim || __hip_atomic_load(&S.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
      __hip_atomic_store(&S.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// At the end of a cooperative kernel: every wave that finishes after a
// timeout (the wave that timed out among them) reports it to the host.
__device__ __forceinline__ void coop_report(CoopSync& S, const CoopCtl& ctl) {
  if ((threadIdx.x & 63) == 0 && ctl.status &&
      __hip_atomic_load(&S.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
    __hip_atomic_store(ctl.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// barrier of nw helper waves only (wave 0 never joins): a monotonic count
__device__ __forceinline__ void helper_barrier(CoopSync& S, uint32_t nw, uint32_t& target) {
  target += nw;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(&S.hbar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  lds_wait_ge(S, &S.hbar, target);
}

// The launch's padding-block K + W tables (64 words per round, <= 12 rounds)
// copied to LDS in the prologue: the challenge after a block-completing absorb
// reads round k's table as its first operand, and from HBM that read's latency
// (~0.5 us) sat on the serial chain every other round.
// The loads are issued with the prologue's other HBM reads, the LDS stores
// after them (a store of a loaded value waits for the load).
constexpr uint32_t kPadKwLds = 12 * 64, kPadKwPer = kPadKwLds / kRedThreads;
struct PadKw {
  uint32_t v[kPadKwPer];
};
__device__ __forceinline__ PadKw pad_kw_load(const uint32_t* __restrict__ kw, uint32_t n) {
  PadKw p;
#pragma unroll
  for (uint32_t u = 0; u < kPadKwPer; ++u) {
    const uint32_t i = u * kRedThreads + threadIdx.x;
    p.v[u] = kw && i < n ? kw[i] : 0u;
  }
  return p;
}
__device__ __forceinline__ void pad_kw_store(const PadKw& p, uint32_t* kwl) {
#pragma unroll
  for (uint32_t u = 0; u < kPadKwPer; ++u) kwl[u * kRedThreads + threadIdx.x] = p.v[u];
}

// Wave 0: rounds 0..R-1 of the launch.  polys: round 0's (c1, c2) slot, rs:
// round 0's r slot, kw (or nullptr): round 0's padding-block K + W table.
//
// dry: a rehearsal on a scratch state (s, mid, mid_len its own; nothing
// published or stored) that runs the half-block and block-completing paths
// once, so that another wave of the workgroup has their code in the
// instruction cache when the real rounds start.
__device__ void transcript_rounds(CoopSync& S, uint32_t R, DevSha& s, uint32_t* stage, fe* polys,
                                  fe* rs, const uint32_t* kw, bool dry, uint32_t* mid,
                                  uint64_t* mid_len) {
  const uint32_t lane = threadIdx.x & 63;
  fe r = fe_zero();
  for (uint32_t k = 0; k < R; ++k) {
    if (!dry) MLH_COOP_TS(0, k);
    if (!dry) lds_wait_ge(S, &S.coef_seq, k + 1);
    if (!dry) MLH_COOP_TS(1, k);
    const fe* sl = S.poly[k & 1] + (lane == 1 ? 3 : 0);
    const fe v = pqrst(sl[0], r, sl[1], sl[2], r);  // lane 0: c1, lane 1: c2
    const fe c2 = bcast_fe(v, 1);
    fe rr = fe_zero();
    // wave-uniform from here (lanes 0 and 1 run the compressions together,
    // two-lane SHA-256: transcript_dev.hpp sha2l_*); LDS state written by lane 0
    const fe c1 = bcast_fe(v, 0);
    if (!dry && lane == 0) {
      fe_store(polys + 2 * k, c1);
      fe_store(polys + 2 * k + 1, c2);
    }
    const uint32_t w[8] = {c1.w[0], c1.w[1], c1.w[2], c1.w[3], c2.w[0], c2.w[1], c2.w[2], c2.w[3]};
    // absorb LE16(c1) || LE16(c2) (sumcheck.rs:188-199), then r = next_challenge()
    uint32_t* bw = reinterpret_cast<uint32_t*>(s.buf);
    const uint64_t len0 = s.len;
    const uint32_t pos = (uint32_t)(len0 & 63);
    const bool half = (len0 & 3) == 0 && pos == 0;
    if (half || ((len0 & 3) == 0 && pos == 32 && *mid_len == len0)) {
      // half: the challenge compresses the 32 bytes + padding, and its rounds
      // 0..7 are kept for the next absorb's compression; else the block
      // completes and its first 8 rounds were run by the last challenge.
      // Both continue in ONE copy of rounds 8..63 (the rehearsal of one path
      // brings the other's code into the instruction cache).
      constexpr uint32_t K[64] = MLH_SHA_K;
      uint32_t blk[16], st[8];
      if (half) {
        const uint64_t bits = (len0 + 32) * 8;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          blk[i] = bswap32(w[i]);
          blk[8 + i] = 0;
          st[i] = s.h[i];
        }
        blk[8] = 0x80000000u;
        blk[14] = (uint32_t)(bits >> 32);
        blk[15] = (uint32_t)bits;
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          blk[i] = bswap32(bw[i]);
          blk[8 + i] = bswap32(w[i]);
          st[i] = mid[i];
        }
      }
      const Sched2L sc = sched2l_init();
      auto kwf = [&](int t) -> uint32_t {
        if (t >= 16) sha2l_sched(blk, t, sc);
        return K[t] + blk[t & 15];
      };
      Sha2L q;
      if (half) {
        if (!dry) MLH_COOP_TS(2, k);
        sha2l_init(q, st);
        sha2l_rounds<0, 8>(q, kwf);
        sha2l_state(q, st);
        if (lane == 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            bw[i] = w[i];
            mid[i] = st[i];
          }
          s.len = len0 + 32;
          *mid_len = len0 + 32;
        }
      }
      sha2l_init(q, st);
      sha2l_rounds<8, 64>(q, kwf);
      uint32_t vv[8];
      sha2l_state(q, vv);
      if (half) {
        fe o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o.w[i] = bswap32(s.h[i] + vv[i]);
        rr = canon_with_carry(o, 0u);
      } else {
        uint32_t nh[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) nh[i] = s.h[i] + vv[i];
        if (lane == 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) s.h[i] = nh[i];
          s.len = len0 + 32;
        }
        if (!dry) MLH_COOP_TS(2, k);
        rr = kw ? sha2l_pad_challenge(nh[0], nh[1], nh[2], nh[3], nh[4], nh[5], nh[6], nh[7], kw + 64 * k)
                : dsha_challenge(s);
      }
    } else {
      if (lane == 0) dsha_absorb<8>(s, w, stage);
      if (!dry) MLH_COOP_TS(2, k);
      if (lane == 0) rr = dsha_challenge_kw(s, kw ? kw + 64 * k : nullptr);
    }
    if (lane == 0) {
      if (!dry) {
        fe_store(rs + k, rr);
        S.rsh[k] = rr;
      } else {
        s.h[0] ^= rr.w[0];  // (keeps the rehearsal's result live; s is its scratch state)
      }
    }
    r = bcast_fe(rr, 0);
    if (dry) continue;
    lds_publish(&S.r_seq, k + 1);
    if (!dry) MLH_COOP_TS(3, k);
  }
}

// Rehearsals that bring the transcript's code into the instruction cache
// before the real rounds run it (on a cold CU the first pass through a
// compression costs ~3 us more): round = one half-block round on a scratch
// state (see `dry`; its compression body is shared with the block-completing
// path), run by wave 0 itself while round 0's coefficients are being built;
// otherwise the padding-block challenge, run by an idle wave.
#ifndef MLH_REH
#define MLH_REH 2  // 0: none; 1: wave 3 a round + the pad challenge; 2: wave 0 a round, wave 3 the pad;
                   // 3: as 2, the eq tail's wave-0 round during its prologue loads
#endif
__device__ void transcript_rehearsal(CoopSync& S, const DevSha& s, const uint32_t* kw, bool round) {
  if (round) {  // one half-block round on a scratch state
    __shared__ DevSha sdry;
    __shared__ uint32_t dmid[8];
    __shared__ uint64_t dmid_len;
    if ((threadIdx.x & 63) == 0) {
      sdry = s;
      sdry.len = 0;
      dmid_len = ~0ull;
    }
    transcript_rounds(S, 1, sdry, nullptr, nullptr, nullptr, kw, true, dmid, &dmid_len);
  } else if (kw) {  // the padding-block challenge (out of line, two lanes; result discarded)
    __shared__ volatile uint32_t sink;  // (keeps the call: its result is discarded)
    (void)sink;
    const fe o = sha2l_pad_challenge(s.h[0], s.h[1], s.h[2], s.h[3], s.h[4], s.h[5], s.h[6], s.h[7], kw);
    if ((threadIdx.x & 63) == 0) sink = o.w[0];
  }
}

// Lane-keyed choices among wave-uniform values.  Written as one chain of
// ternaries on the lane index, the compiler turns them into a lookup table in
// scratch memory (stores of the candidates, a lane-indexed scratch load: an L2
// round trip on the serial chain, ~1 us per choice).  Each comparison here
// reads its own opaque copy of the lane index, so every choice stays a
// v_cndmask.
__device__ __forceinline__ bool lane_is(uint32_t k) {
  uint32_t l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l == k;
}
__device__ __forceinline__ bool lane_below(uint32_t k) {
  uint32_t l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l < k;
}
__device__ __forceinline__ fe fe_if(bool c, const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.w[i] = c ? a.w[i] : b.w[i];
  return r;
}

// Values of round t's four quadratics at r (lane j < 4 evaluates quadratic j).
// (Cross-lane values move by v_readlane: an LDS round trip measured slower.)
__device__ __forceinline__ void quad_eval(const fe* q, const fe& r, fe& c1, fe& c2, fe& e0, fe& cs) {
  const uint32_t lane = threadIdx.x & 63;
  const fe* k = q + 3 * (lane < 4 ? lane : 0);
  const fe v = pqrst(k[0], r, k[1], k[2], r);
  c1 = bcast_fe(v, 0);
  c2 = bcast_fe(v, 1);
  e0 = bcast_fe(v, 2);
  cs = bcast_fe(v, 3);
}
// Round t's four quadratics in r_{t-1} into q (12 entries) from E_b = A_b +
// r B_b, the claim quadratic (cl0, cl1, cl2) = (e0', c1, c2) of round t-1 and
// its eq scale cs; p = p_t, pp = p_{t-1}.  first: round t is the launch's first
// (cl0, cs constants; cl1 = cl2 = 0, B_b = 0).  Products on lanes, two deep.
__device__ __forceinline__ void quad_next(bool first, const fe& cl0, const fe& cl1, const fe& cl2, const fe& cs,
                          const fe& A0, const fe& B0, const fe& A1, const fe& B1, const fe& p,
                          const fe& pp, fe* q, uint32_t tq = 0) {
  const uint32_t lane = threadIdx.x & 63;
  (void)tq;
  MLH_COOP_TS(9, 32 + 2 * tq);
  const fe one = fe_one();
  const fe p3 = fe_add(fe_dbl(p), p), qq = fe_sub(p3, one);
  const fe D0 = fe_sub(fe_dbl(A1), A0), D1 = fe_sub(fe_dbl(B1), B0);
  // lanes 0..5: U = c (1 - pp), V = c (2 pp - 1), q D0, p A1, q D1, p B1
  const fe a1 = fe_if(lane_below(2), cs, fe_if((lane & 1) != 0, p, qq));
  const fe b1 = fe_if(lane_is(0), fe_sub(one, pp),
                      fe_if(lane_is(1), fe_sub(fe_dbl(pp), one),
                            fe_if(lane_is(2), D0, fe_if(lane_is(3), A1, fe_if(lane_is(4), D1, B1)))));
  fe y = fe_mul_s(a1, b1);
  if (first) y = fe_if(lane_is(0), cs, fe_if(lane_is(1), fe_zero(), y));
  const fe U = bcast_fe(y, 0), V = bcast_fe(y, 1), pA1 = bcast_fe(y, 3), pB1 = bcast_fe(y, 5);
  MLH_COOP_TS(9, 33 + 2 * tq);
  const fe f0 = fe_sub(bcast_fe(y, 2), fe_add(fe_dbl(pA1), pA1));
  const fe f1 = fe_sub(bcast_fe(y, 4), fe_add(fe_dbl(pB1), pB1));
  // lanes 0..7: U f0, V f0, U f1, V f1, U h0, V h0, U h1, V h1 (h = p A1, p B1)
  const fe b2 = fe_if(lane_below(2), f0, fe_if(lane_below(4), f1, fe_if(lane_below(6), pA1, pB1)));
  const fe z = fe_mul_s(fe_if((lane & 1) != 0, V, U), b2);
  const fe Uf0 = bcast_fe(z, 0), Vf0 = bcast_fe(z, 1), Uf1 = bcast_fe(z, 2), Vf1 = bcast_fe(z, 3);
  const fe Uh0 = bcast_fe(z, 4), Vh0 = bcast_fe(z, 5), Uh1 = bcast_fe(z, 6), Vh1 = bcast_fe(z, 7);
  // lane k < 3: coefficient k of Y = (U+Vr)(f0+f1 r), X = (U+Vr)(h0+h1 r), the claim
  const fe Yk = fe_if(lane_is(0), Uf0, fe_if(lane_is(1), fe_add(Uf1, Vf0), Vf1));
  const fe Xk = fe_if(lane_is(0), Uh0, fe_if(lane_is(1), fe_add(Uh1, Vh0), Vh1));
  const fe Ck = fe_if(lane_is(0), cl0, fe_if(lane_is(1), cl1, cl2));
  const fe c2 = fe_half(fe_add(Yk, Ck));
  const fe c1 = fe_sub(fe_sub(fe_dbl(Xk), Ck), c2);
  const fe e0 = fe_sub(Ck, Xk);
  if (lane < 3) {
    q[lane] = c1;
    q[3 + lane] = c2;
    q[6 + lane] = e0;
    q[9 + lane] = fe_if(lane_is(0), U, fe_if(lane_is(1), V, fe_zero()));
  }
}

// E_b split by the corner bit at position mt (and, me != 0, the bit at me):
// returns the sums over lanes of x with (bit mt, bit me) = (b, e) as
// S[2 b + e] (me = 0: S[0], S[2] only).
__device__ __forceinline__ void bucket_sums(fe x, uint32_t mt, uint32_t me, fe (&Sb)[4]) {
  for (uint32_t m = 1; m < 64; m <<= 1)
    if (m != mt && m != me) x = fe_add(x, shfl_xor_fe(x, (int)m));
  Sb[0] = bcast_fe(x, 0);
  Sb[2] = bcast_fe(x, (int)mt);
  if (me) {
    Sb[1] = bcast_fe(x, (int)me);
    Sb[3] = bcast_fe(x, (int)(mt | me));
  }
}

// K = 2 or 4 values per lane, summed over the lanes that agree on the bits
// in `excl` (the bucket bits), with ONE value per lane left: the first
// log2 K of the other bits halve the set (the lane with that bit clear keeps
// the lower half and sends the upper), the rest are plain butterfly levels --
// log2 K + (6 - |excl| - log2 K) exchanges instead of K x (6 - |excl|).
// Value k of bucket pattern e is then on lane e | hb(k): bit hb[0] set iff
// k >> (log2 K - 1), bit hb[1] (K = 4) iff k & 1.
template <int K>
__device__ __forceinline__ fe bucket_halve(const fe (&v)[K], uint32_t excl, uint32_t (&hb)[2]) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t m1 = ~excl & (excl + 1u);                 // lowest bit not in excl
  const uint32_t m2 = ~(excl | m1) & ((excl | m1) + 1u);  // the next one
  fe z;
  uint32_t done = excl | m1;
  if constexpr (K == 4) {
    const bool b1 = (lane & m1) != 0;
    fe k0 = fe_add(fe_if(b1, v[2], v[0]), shfl_xor_fe(fe_if(b1, v[0], v[2]), (int)m1));
    fe k1 = fe_add(fe_if(b1, v[3], v[1]), shfl_xor_fe(fe_if(b1, v[1], v[3]), (int)m1));
    const bool b2 = (lane & m2) != 0;
    z = fe_add(fe_if(b2, k1, k0), shfl_xor_fe(fe_if(b2, k0, k1), (int)m2));
    hb[0] = m1;
    hb[1] = m2;
    done |= m2;
  } else {
    const bool b1 = (lane & m1) != 0;
    z = fe_add(fe_if(b1, v[1], v[0]), shfl_xor_fe(fe_if(b1, v[0], v[1]), (int)m1));
    hb[0] = m1;
    hb[1] = 0;
  }
  for (uint32_t m = 1; m < 64; m <<= 1)
    if (!(m & done)) z = fe_add(z, shfl_xor_fe(z, (int)m));
  return z;
}

// Suffix products Rs of a group (J <= 6 variables, points pv in HBM) into
// rs[u][c].  The J point loads are all issued before the product chain (a
// load per link of the chain cost one HBM latency each: ~9 us of prologue).
__device__ __forceinline__ void suffix_products(uint32_t J, const fe* pv, fe (*rs)[64]) {
  const uint32_t c = threadIdx.x & 63;
  const fe one = fe_one();
  fe p[6];
#pragma unroll
  for (int u = 0; u < 6; ++u) p[u] = u < (int)J ? fe_vgpr(fe_load(pv + u)) : one;
  fe acc = one;
#pragma unroll
  for (int u = 5; u >= 0; --u) {
    if (u < (int)J) {
      rs[u][c] = acc;
      acc = fe_mul_s(acc, (c >> (J - 1 - (uint32_t)u)) & 1u ? p[u] : fe_sub(one, p[u]));
    }
  }
}

// The helpers of rounds (variables) u0..vend-1 of the launch's corner groups
// -- group A = variables [0, JA) with corner sums X = S.xc[c] (and Rs in
// S.rsuf), group B = [JA, JA + JB) (eq tail with JB > 0: its corner sums come
// from S.msplit folded with r_3, r_4 and split by r_5, Rs in S.rsufB).
// Variable v is launch round v - u0; r_v for v < u0 are in rs_known.  Two
// waves per round, in parallel once r_{t-2} is out: the corner wave updates
// the corner weights and sums E_b = A_b + r B_b (S.ab), the coefficient wave
// evaluates round t-1's quadratics at r_{t-2} and then builds round t's.
//
// Corner wave: writes (wout) group A's fold weights or (m_out) the fully
// folded table entry sum_c W_c X_c.
__device__ void corner_rounds(CoopSync& S, uint32_t JA, uint32_t JB, uint32_t u0, uint32_t vend,
                              const fe* rs_known, fe* wout, fe* m_out, fe* wfold,
                              const fe* msp = nullptr) {
  const uint32_t c = threadIdx.x & 63;
  const fe one = fe_one();
  fe X = S.xc[c];
  if (c >= (1u << JA)) X = fe_zero();
  fe L = X, W = one, Xa = fe_zero(), Xb = fe_zero(), Xact = X;
  auto gsel = [&](uint32_t v, const fe& x) -> fe {  // corner c's factor of variable v
    const uint32_t J = v < JA ? JA : JB, u = v < JA ? v : v - JA;
    return (c >> (J - 1 - u)) & 1u ? x : fe_sub(one, x);
  };
  {  // the r's of earlier launches (u0 <= 5): loads first, then the products
    fe rk[6];
#pragma unroll
    for (uint32_t v = 0; v < 6; ++v) rk[v] = v < u0 ? fe_vgpr(fe_load(rs_known + v)) : one;
#pragma unroll
    for (uint32_t v = 0; v < 6; ++v)
      if (v < u0) {
        const fe g = gsel(v, rk[v]);
        L = fe_mul_s(L, g);
        W = fe_mul_s(W, g);
      }
  }
  for (uint32_t v = u0; v < vend; ++v) {
    const bool inB = v >= JA;
    const uint32_t J = inB ? JB : JA, u = inB ? v - JA : v, t = v - u0;
    const bool first = t == 0;
    const uint32_t mt = 1u << (J - 1 - u);
    // A regular round (variable v - 2 in the same group, its challenge r_{t-2}
    // the one awaited) is linear in that challenge: with P_c = L_c Rs_u[c]
    // (L without v - 2's factor), E_b = sum_c P_c g_c(r), g_c = r or 1 - r by
    // the corner's bit md of v - 2.  So the products and the shuffle levels
    // over the bits other than (md, me, mt) run BEFORE r_{t-2} is out; after
    // it, one product, one level and the four broadcasts (the weights' update
    // follows the publish).
    const bool regular = u >= 2 && v - 2 >= u0;
    const uint32_t me_r = 1u << (J - u), md = 1u << (J + 1 - u);
    fe Pr = fe_zero();
    if (regular) {
      fe x = fe_mul_s(L, inB ? S.rsufB[u][c] : S.rsuf[u][c]);
      for (uint32_t m = 1; m < 64; m <<= 1)
        if (m != mt && m != me_r && m != md) x = fe_add(x, shfl_xor_fe(x, (int)m));
      Pr = x;
    }
    // Group B's first two rounds are linear in their awaited challenge too.
    // Round u = 0 (r_4 awaited): the corner sums fold the split table with r_3
    // (known) and r_4, n_b5 = lo_b5 + r_4 (hi_b5 - lo_b5), so X_a = n_0 and
    // X_b = n_1 - n_0 are a + r_4 a' and b + r_4 b', and their bucket sums
    // (split by mt) are taken before r_4.  Round u = 1 (r_5 awaited): L = X_a +
    // r_5 X_b, the bucket sums of X_a Rs_1 and X_b Rs_1 (split by mt, me) before
    // r_5.  After the challenge: one product on four lanes.
    const bool b0r = inB && u == 0, b1r = inB && u == 1;
    fe Tz = fe_zero(), la = fe_zero(), lb = fe_zero(), ma = fe_zero(), mb = fe_zero();
    uint32_t hb[2] = {0, 0};
    if (b0r) {
      lds_wait_ge(S, &S.r_seq, 4 - u0);  // r_3
      lds_wait_ge(S, &S.mseq, 1);
      const fe r3 = lds_fe(S.rsh[3 - u0]);
      const uint32_t qb = 1u << JB;  // split table: msp[d qb + x], d = bits of variables 3, 4, 5
      const fe* M = msp + (c < qb ? c : 0);
      const fe lo0 = lerp_s(M[qb * 0], M[qb * 4], r3), hi0 = lerp_s(M[qb * 2], M[qb * 6], r3);
      const fe lo1 = lerp_s(M[qb * 1], M[qb * 5], r3), hi1 = lerp_s(M[qb * 3], M[qb * 7], r3);
      const bool live = c < qb;
      la = live ? lo0 : fe_zero();
      ma = live ? fe_sub(hi0, lo0) : fe_zero();
      lb = live ? fe_sub(lo1, lo0) : fe_zero();
      mb = live ? fe_sub(fe_sub(hi1, lo1), fe_sub(hi0, lo0)) : fe_zero();
      const fe R0 = S.rsufB[0][c];
      const fe vv[4] = {fe_mul_s(la, R0), fe_mul_s(ma, R0), fe_mul_s(lb, R0), fe_mul_s(mb, R0)};
      Tz = bucket_halve<4>(vv, mt, hb);
    } else if (b1r) {
      const fe R1 = S.rsufB[1][c];
      const fe vv[2] = {fe_mul_s(Xa, R1), fe_mul_s(Xb, R1)};
      Tz = bucket_halve<2>(vv, mt | me_r, hb);
    }
    fe rv = fe_zero();
    if (t >= 2) {
      lds_wait_ge(S, &S.r_seq, t - 1);
      rv = lds_fe(S.rsh[t - 2]);
    }
    MLH_COOP_TS(6, t);
    fe Sb[4];
    fe A0, B0 = fe_zero(), A1, B1 = fe_zero();
    fe greg = one;
    if (regular) {
      greg = (c & md) ? rv : fe_sub(one, rv);  // gsel(v - 2, rv)
      fe y = fe_mul_s(Pr, greg);
      y = fe_add(y, shfl_xor_fe(y, (int)md));
      A0 = bcast_fe(y, 0);
      A1 = bcast_fe(y, (int)mt);
      B0 = fe_sub(bcast_fe(y, (int)me_r), A0);
      B1 = fe_sub(bcast_fe(y, (int)(mt | me_r)), A1);
    } else if (b0r || b1r) {
      // lane j < 4: output j = base + r slope, base / slope = bucket sums
      // (value k, bucket e) on lane e | hb(k)
      const uint32_t j = c & 3;
      uint32_t e, kb, ks;  // bucket, base value, slope value
      if (b0r) {  // A0, A1 from (a, a'), B0, B1 from (b, b'); buckets 0, mt
        e = (j & 1) ? mt : 0u;
        kb = (j >> 1) ? 2u : 0u;
        ks = kb + 1;
      } else {  // Sb[0..3] over buckets 0, me, mt, mt | me; values X_a (0), X_b (1)
        e = ((j & 2) ? mt : 0u) | ((j & 1) ? me_r : 0u);
        kb = 0;
        ks = 1;
      }
      auto at = [&](uint32_t k) -> int {
        return (int)(e | (b0r ? (((k >> 1) ? hb[0] : 0u) | ((k & 1) ? hb[1] : 0u)) : (k ? hb[0] : 0u)));
      };
      const fe o = fe_add(shfl_fe(Tz, at(kb)), fe_mul_s(rv, shfl_fe(Tz, at(ks))));
      if (b0r) {
        A0 = bcast_fe(o, 0);
        A1 = bcast_fe(o, 1);
        B0 = bcast_fe(o, 2);
        B1 = bcast_fe(o, 3);
      } else {
        Sb[0] = bcast_fe(o, 0);
        Sb[1] = bcast_fe(o, 1);
        Sb[2] = bcast_fe(o, 2);
        Sb[3] = bcast_fe(o, 3);
        A0 = Sb[0];
        A1 = Sb[2];
        B0 = fe_sub(Sb[1], Sb[0]);
        B1 = fe_sub(Sb[3], Sb[2]);
      }
    } else {
      const fe x = fe_mul_s(L, inB ? S.rsufB[u][c] : S.rsuf[u][c]);
      const uint32_t me = (first || u == 0) ? 0u : 1u << (J - u);
      bucket_sums(x, mt, me, Sb);
      A0 = Sb[0];
      A1 = Sb[2];
      if (me) {
        B0 = fe_sub(Sb[1], Sb[0]);
        B1 = fe_sub(Sb[3], Sb[2]);
      }
    }
    if (c == 0) {
      fe* ab = S.ab[t & 1];
      ab[0] = A0;
      ab[1] = B0;
      ab[2] = A1;
      ab[3] = B1;
    }
    lds_publish(&S.ab_seq, t + 1);
    MLH_COOP_TS(7, t);
    if (regular) {  // the weights take v - 2's factor (used from the next round on)
      L = fe_mul_s(L, greg);
      W = fe_mul_s(W, greg);
    } else if (b0r) {  // group B's corner sums at r_4
      Xa = fe_add(la, fe_mul_s(rv, ma));
      Xb = fe_add(lb, fe_mul_s(rv, mb));
      W = one;
    } else if (b1r) {  // ... and at r_5
      L = fe_add(Xa, fe_mul_s(rv, Xb));
      Xact = L;
    }
  }
  if (!wout && !m_out && !wfold) return;
  // the last round's variables: r of the one before it, then its own.  All
  // but one product per lane happen before the last challenge is out: group
  // A's fold weights need only r_0..r_{JA-1}, and the folded entry sum_c W_c
  // X_c is linear in the last challenge (bucket sums by its bit first).
  const uint32_t vl = vend - 1, tl = vl - u0, ul = vl >= JA ? vl - JA : vl;
  const uint32_t Jl = vl >= JA ? JB : JA, mb = 1u << (Jl - 1 - ul);
  fe WA = one;
  if (wfold && JB) {
    lds_wait_ge(S, &S.r_seq, JA - u0);
    for (uint32_t v = 0; v < JA; ++v) WA = fe_mul_s(WA, gsel(v, lds_fe(S.rsh[v - u0])));
  }
  fe rv = fe_zero();
  if (tl >= 1) {
    lds_wait_ge(S, &S.r_seq, tl);
    rv = lds_fe(S.rsh[tl - 1]);
  }
  if (vl >= JA && ul == 0)
    Xact = fe_add(Xa, fe_mul_s(rv, Xb));  // a one-variable group B: m_6 at r_5
  else if (ul >= 1 && vl - 1 >= u0)
    W = fe_mul_s(W, gsel(vl - 1, rv));    // (the loop took the variables before)
  fe T = fe_zero();
  if (m_out) {
    T = c < (1u << Jl) ? fe_mul_s(W, Xact) : fe_zero();
    for (uint32_t m = 1; m < 64; m <<= 1)
      if (m != mb) T = fe_add(T, shfl_xor_fe(T, (int)m));
  }
  lds_wait_ge(S, &S.r_seq, tl + 1);
  const fe rl = lds_fe(S.rsh[tl]);
  if (m_out) {  // sum over the last group's corners of W_c X_c
    const fe T0 = bcast_fe(T, 0);
    const fe x = fe_add(T0, fe_mul_s(rl, fe_sub(bcast_fe(T, (int)mb), T0)));
    if (c == 0) fe_store(m_out, x);
  }
  if (wout || wfold) W = fe_mul_s(W, gsel(vl, rl));
  if (wout && c < (1u << JA)) fe_store(wout + c, W);
  if (wfold) {  // the fold weights of both groups: W_A at wfold[0..64), W_B at wfold[64..)
    if (JB) {
      if (c < (1u << JB)) fe_store(wfold + 64 + c, W);
    } else {
      WA = W;
    }
    if (c < (1u << JA)) fe_store(wfold + c, WA);
  }
}

// Coefficient wave: publishes round t's quadratics (S.poly, coef_seq); writes
// the claim and eq scale after the last round (prev, cdev; d_out too).
// claim0, cs0: *prev and *cdev, loaded by the caller at kernel entry (their
// HBM latency then overlaps the table loads instead of round 0's slot).
__device__ void coef_rounds(CoopSync& S, uint32_t u0, uint32_t vend, fe* prev, fe* cdev, fe* d_out,
                            const fe& claim0, const fe& cs0) {
  const uint32_t c = threadIdx.x & 63;
  const fe one = fe_one();
  fe c1v = fe_zero(), c2v = fe_zero(), e0v = fe_zero(), csv = fe_zero();
  for (uint32_t v = u0; v < vend; ++v) {
    const uint32_t t = v - u0;
    const bool first = t == 0;
    fe rv = fe_zero();
    if (t >= 2) {
      lds_wait_ge(S, &S.r_seq, t - 1);
      rv = lds_fe(S.rsh[t - 2]);
    }
    MLH_COOP_TS(5, t);
    if (!first) quad_eval(S.poly[(t - 1) & 1], rv, c1v, c2v, e0v, csv);  // round t-1's values
    lds_wait_ge(S, &S.ab_seq, t + 1);
    const fe* abp = S.ab[t & 1];
    const fe ab[4] = {lds_fe(abp[0]), lds_fe(abp[1]), lds_fe(abp[2]), lds_fe(abp[3])};
    MLH_COOP_TS(8, t);
    // (values, not `first ? claim0 : e0v` bound to a reference: a choice
    // between two lvalues is a choice of addresses, which puts both in scratch)
    const fe cl0 = fe_if(first, claim0, e0v), csx = fe_if(first, cs0, csv);
    const fe pv = lds_fe(S.pg[v]), ppv = v ? lds_fe(S.pg[v - 1]) : fe_zero();
    quad_next(first, cl0, c1v, c2v, csx, ab[0], ab[1], ab[2], ab[3], pv, ppv, S.poly[t & 1], t);
    lds_publish(&S.coef_seq, t + 1);
    MLH_COOP_TS(4, t);
  }
  // the last round's values (at r of the variable before it), its challenge
  const uint32_t vl = vend - 1, tl = vl - u0;
  fe rv = fe_zero();
  if (tl >= 1) {
    lds_wait_ge(S, &S.r_seq, tl);
    rv = lds_fe(S.rsh[tl - 1]);
  }
  quad_eval(S.poly[tl & 1], rv, c1v, c2v, e0v, csv);
  // before the last challenge: scale = cs ((1 - r)(1 - p) + r p) = al + r be
  const fe p = lds_fe(S.pg[vl]);
  const fe al = fe_mul_s(csv, fe_sub(one, p)), be = fe_mul_s(csv, fe_sub(fe_dbl(p), one));
  lds_wait_ge(S, &S.r_seq, tl + 1);
  const fe r = lds_fe(S.rsh[tl]);
  // lane 1: the scale; lane 0: c1 + c2 r, then claim = e0 + r (c1 + c2 r)
  const bool l1 = lane_is(1);
  const fe z = fe_add(fe_if(l1, al, c1v), fe_mul_s(fe_if(l1, be, c2v), r));
  const fe scale = bcast_fe(z, 1);
  const fe claim = fe_add(e0v, fe_mul_s(z, r));
  if (c == 0) {
    fe_store(prev, claim);
    fe_store(cdev, scale);
    if (d_out) fe_store(d_out, scale);
  }
}

// Rounds t0..t1-1 of a group of J (+ J2) eq-factored head rounds k.. from the
// corner sums (see "grouped eq-factored rounds"): the NC x nb partials are
// summed into the NC = 2^(J+J2) corner sums, then wave 0 runs the transcript
// and wave 1 the coefficients (J2 > 0: all J + J2 rounds, t0 = 0).  pts, rs:
// p_k.., r_k.. (rs[u] for u < t0 were written by earlier launches of this
// group); polys: round t0's slot; kw: round 0's padding table (or nullptr);
// wout (when the launch ends the group): the fold weights of its challenges.
__global__ void __launch_bounds__(kRedThreads)
sumcheck_group_kernel(const fe* __restrict__ partials, uint32_t nb, uint32_t J, uint32_t J2,
                      uint32_t t0, uint32_t t1, fe* prev, DevSha* t, fe* polys, fe* rs,
                      const fe* __restrict__ pts, fe* cdev, const uint32_t* __restrict__ kw,
                      fe* wout, CoopCtl ctl) {
  MLH_COOP_EDGE(0);
  fe claim0 = fe_zero(), cs0 = fe_zero();
  if ((threadIdx.x >> 6) == 1) {  // the coefficient wave's inputs, early
    claim0 = fe_load(prev);
    cs0 = fe_load(cdev);
  }
  __shared__ DevSha s;
  __shared__ uint32_t stage[8];
  __shared__ fe slotY[64];
  __shared__ CoopSync S;
  __shared__ uint32_t kwl[kPadKwLds];
  const uint32_t tend = J2 ? J + J2 : t1;
  const uint32_t* kwx = kw ? kwl : nullptr;  // the launch's pad K + W tables, in LDS
  const PadKw pkw = pad_kw_load(kw ? kw + 64 * t0 : nullptr, 64 * (tend - t0));
  if (threadIdx.x < sizeof(DevSha) / 4)
    reinterpret_cast<uint32_t*>(&s)[threadIdx.x] = reinterpret_cast<const uint32_t*>(t)[threadIdx.x];
  if (threadIdx.x == 0) {
    S.coef_seq = S.r_seq = S.hbar = S.mseq = S.fail = S.ab_seq = 0;
    S.spin_limit = ctl.spin_limit ? ctl.spin_limit : kSpinLimit;
    S.mid_len = ~0ull;
  }
  const uint32_t JT = J + J2, NC = 1u << JT, G = kRedThreads >> JT;  // threads per corner
  const uint32_t GW = G < 64 ? G : 64;                                // ... within one wave
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave == 1 && lane < JT) S.pg[lane] = fe_load(pts + lane);
  if (wave == 2) suffix_products(JT, pts, S.rsuf);  // the corner wave's, independent of the partials
  {
    const uint32_t c = threadIdx.x / G, j = threadIdx.x % G;
    fe acc = fe_zero();
#pragma unroll 4
    for (uint32_t b = j; b < nb; b += G) acc = fe_add(acc, fe_load(partials + (uint64_t)c * nb + b));
    for (uint32_t m = GW / 2; m >= 1; m >>= 1) acc = fe_add(acc, shfl_xor_fe(acc, (int)m));
    if (threadIdx.x % GW == 0) slotY[threadIdx.x / GW] = acc;
  }
  pad_kw_store(pkw, kwl);
  __syncthreads();
  MLH_COOP_EDGE(1);
  if (wave == 0) {
    if (MLH_REH >= 2) transcript_rehearsal(S, s, kwx, true);
    transcript_rounds(S, tend - t0, s, stage, polys, rs + t0, kwx, false, S.mid, &S.mid_len);
    if (lane == 0) *t = s;
  } else if (wave == 1) {
    coef_rounds(S, t0, tend, prev, cdev, nullptr, claim0, cs0);
  } else if (wave == 3) {
    if (MLH_REH == 1) transcript_rehearsal(S, s, kwx, true);
    if (MLH_REH != 0) transcript_rehearsal(S, s, kwx, false);
  } else if (wave == 2) {
    fe X = fe_zero();
    const uint32_t per = G / GW;  // slots per corner
    if (lane < NC)
      for (uint32_t q = 0; q < per; ++q) X = fe_add(X, slotY[lane * per + q]);
    S.xc[lane] = X;
    corner_rounds(S, JT, 0, t0, tend, rs, (wout && (J2 || t1 == J)) ? wout : nullptr, nullptr,
                  nullptr);
  }
  coop_report(S, ctl);
}

// The last a rounds of an eq-factored sumcheck (mlh_sumcheck_prove_eq) in ONE
// workgroup: the 2^a-entry matrix table m and the suffix tables e_j =
// eq(p_{B+j+1}..p_{L-1}) (2^(a-1-j) entries at offset 2^a - 2^(a-j), as H_k)
// staged in LDS, delta = c eq(p_B..) never materialised.  The rounds go in
// corner groups as the head's: group A = the first JA = min(a, 6) variables,
// corner sums X_c = sum_{i<Q} m[c Q + i] e_{JA-1}[i] (Q = 2^(a-JA)); group B
// = the rest (a > 6), whose table m_6 (Q entries, its own corner sums) is m
// folded over group A.  Wave 0 runs the transcript, wave 1 the coefficients,
// waves 2-3 fold m over group A's first 3 variables once r_0..r_2 are out,
// keeping the next 3 split (S.msplit); the lead folds those with r_3, r_4 and
// takes m_6 = N_0 + r_5 (N_1 - N_0) as linear in r_5.  On load, m is Tin
// folded over Jin <= 3 pending variables with rs_in.  Writes the folded
// matrix m_out[0], the final delta c_L (eq of no points = 1) to d_out[0], the
// claim and the transcript.
__global__ void __launch_bounds__(kRedThreads)
sumcheck_eq_tail_kernel(const fe* Tin, uint32_t Jin, const fe* __restrict__ rs_in, uint32_t a,
                        const fe* __restrict__ e_grp, const fe* __restrict__ pts, fe* cdev, fe* prev,
                        DevSha* t, fe* polys, fe* rs, fe* m_out, fe* d_out,
                        const uint32_t* __restrict__ kw, fe* wfold, CoopCtl ctl, HostOut ho,
                        const fe* __restrict__ xc_part, uint32_t xc_nb, const fe* __restrict__ rsuf) {
  MLH_COOP_EDGE(0);
  extern __shared__ fe eq_tail_lds[];
  const uint32_t JA = a < 6 ? a : 6, JB = a - JA, QA = 1u << (a - JA);
  // tdma: with the corner sums from xc_part, the table is read only by wave
  // 3's fold levels (and, after them, the corner wave's group B): wave 3
  // copies it HBM -> LDS itself (LDS-DMA, no registers) once the roles start,
  // so the prologue waits for neither the table nor e
  const bool tdma = MLH_TAIL_DMA && xc_part && JB && Jin == 0;
  fe claim0 = fe_zero(), cs0 = fe_zero();
  if ((threadIdx.x >> 6) == 1) {  // the coefficient wave's inputs, early
    claim0 = fe_load(prev);
    cs0 = fe_load(cdev);
  }
  fe* lm = eq_tail_lds;                    // 2^a
  fe* le = eq_tail_lds + (1u << a);        // e_{JA-1}: QA entries
  __shared__ DevSha s;
  __shared__ uint32_t stage[8];
  __shared__ CoopSync S;
  __shared__ uint32_t kwl[kPadKwLds];
  const uint32_t* kwx = kw ? kwl : nullptr;  // the launch's pad K + W tables, in LDS
  const uint32_t S0 = 1u << a;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // every HBM read of the prologue is issued before the first LDS store (a
  // store of a loaded value waits for it): transcript state, points, and for
  // plain copies the table (2^a / 256 <= 16 per thread) and e
  const uint32_t sw = threadIdx.x < sizeof(DevSha) / 4 ? reinterpret_cast<const uint32_t*>(t)[threadIdx.x] : 0u;
  const fe pgv = threadIdx.x < a ? fe_load(pts + threadIdx.x) : fe_zero();
  const PadKw pkw = pad_kw_load(kw, 64 * a);
  constexpr uint32_t PER = (1u << kTailLogMax) / kRedThreads;
  fe v[PER];
  if (Jin == 0 && !tdma) {
#pragma unroll
    for (uint32_t u = 0; u < PER; ++u) {
      const uint32_t x = u * kRedThreads + threadIdx.x;
      v[u] = x < S0 ? fe_load(Tin + x) : fe_zero();
    }
  }
  // xc_part (optional, the tail launch): group A's corner sums as xc_nb (a
  // few) partials per corner, written by the fold that produced Tin
  // (fold_group_eq_kernel's JN path with e = e_grp): the corner-sum phase
  // below is skipped.  (The head's terms -- 64 per corner from the corner-sum
  // pass -- summed here measured slower than that phase.)
  fe xcv = fe_zero();
  if (xc_part && threadIdx.x < (1u << JA))
    for (uint32_t bb = 0; bb < xc_nb; ++bb) xcv = fe_add(xcv, fe_load(xc_part + threadIdx.x * xc_nb + bb));
  // wave 0 rehearses a half-block transcript round NOW, while the loads above
  // are in flight (its inputs are not loaded yet: garbage in, result
  // discarded -- it only brings the code into the instruction cache), instead
  // of at the start of the rounds, where it sat before round 0
  if (MLH_REH == 3 && (threadIdx.x >> 6) == 0) transcript_rehearsal(S, s, kwx, true);
  if (threadIdx.x < sizeof(DevSha) / 4) reinterpret_cast<uint32_t*>(&s)[threadIdx.x] = sw;
  if (threadIdx.x == 0) {
    S.coef_seq = S.r_seq = S.hbar = S.mseq = S.fail = S.ab_seq = 0;
    S.spin_limit = ctl.spin_limit ? ctl.spin_limit : kSpinLimit;
    S.mid_len = ~0ull;
  }
  if (threadIdx.x < a) S.pg[threadIdx.x] = pgv;
  pad_kw_store(pkw, kwl);
  if (Jin == 0) {
    // plain copies: the groups' suffix products (their points' loads too, or
    // the precomputed products), then the LDS stores
    const fe ev = !xc_part && threadIdx.x < QA ? fe_load(e_grp + threadIdx.x) : fe_zero();
    if (rsuf) {
      const uint32_t J = wave == 2 ? JA : JB;
      if (wave == 2 || wave == 3) {
        fe (*dst)[64] = wave == 2 ? S.rsuf : S.rsufB;
        fe t[6];
#pragma unroll
        for (uint32_t u = 0; u < 6; ++u)
          if (u < J) t[u] = fe_load(rsuf + (wave - 2) * 384 + u * 64 + lane);
#pragma unroll
        for (uint32_t u = 0; u < 6; ++u)
          if (u < J) dst[u][lane] = t[u];
      }
    } else {
      if (wave == 2) suffix_products(JA, pts, S.rsuf);
      if (wave == 3 && JB) suffix_products(JB, pts + JA, S.rsufB);
    }
    if (!tdma) {
#pragma unroll
      for (uint32_t u = 0; u < PER; ++u) {
        const uint32_t x = u * kRedThreads + threadIdx.x;
        if (x < S0) lm[x] = v[u];
      }
    }
    if (!xc_part && threadIdx.x < QA) le[threadIdx.x] = ev;
    MLH_COOP_TS(9, 10);
  } else {
    // the groups' suffix products (from the points in HBM) while the tables load
    if (wave == 2) suffix_products(JA, pts, S.rsuf);
    if (wave == 3 && JB) suffix_products(JB, pts + JA, S.rsufB);
    for (uint32_t x = threadIdx.x; x < QA; x += blockDim.x) le[x] = fe_load(e_grp + x);
    fe rin[3];
#pragma unroll
    for (uint32_t u = 0; u < 3; ++u) rin[u] = u < Jin ? fe_load(rs_in + u) : fe_zero();
    for (uint32_t x = threadIdx.x; x < S0; x += blockDim.x) lm[x] = fold_corners_n(Jin, Tin + x, S0, rin);
  }
  if (xc_part && threadIdx.x < (1u << JA)) S.xc[threadIdx.x] = xcv;
  __syncthreads();
  MLH_COOP_TS(9, 11);
  // group A's corner sums: 2^JA corners x QA entries, G = 256 / 2^JA threads per corner
  if (!xc_part) {
    const uint32_t G = kRedThreads >> JA, c = threadIdx.x / G, j = threadIdx.x % G;
    const fe* e = le;  // e_{JA-1}: QA entries
    sacc q;
    sacc_zero(q);
    for (uint32_t i = j; i < QA; i += G) sacc_mac(q, lm[c * QA + i], e[i]);
    fe x = sacc_reduce(q);
    for (uint32_t m = (G < 64 ? G : 64) / 2; m >= 1; m >>= 1) x = fe_add(x, shfl_xor_fe(x, (int)m));
    if (G <= 64) {
      if (j == 0) S.xc[c] = x;
    } else {  // G = 128 or 256 (JA <= 1): 2 or 4 waves per corner
      if (lane == 0) S.red[wave][0] = x;
    }
    __syncthreads();
    if ((kRedThreads >> JA) > 64 && threadIdx.x < (1u << JA)) {
      const uint32_t per = (kRedThreads >> JA) / 64;
      fe y = fe_zero();
      for (uint32_t w = 0; w < per; ++w) y = fe_add(y, S.red[threadIdx.x * per + w][0]);
      S.xc[threadIdx.x] = y;
    }
    __syncthreads();
  }
  MLH_COOP_EDGE(1);
#ifdef MLH_COOP_PROF
  if (lane == 0) g_coop_ts[9][20 + wave] = __builtin_amdgcn_s_getreg(4 | (31 << 11));  // HW_ID: SIMD in bits 5:4
#endif
  if (wave == 0) {
    if (MLH_REH == 2) transcript_rehearsal(S, s, kwx, true);
    transcript_rounds(S, a, s, stage, polys, rs, kwx, false, S.mid, &S.mid_len);
    if (lane == 0) *t = s;
  } else if (wave == 1) {
    coef_rounds(S, 0, a, prev, cdev, d_out, claim0, cs0);
  } else if (wave == 2) {
    corner_rounds(S, JA, JB, 0, a, nullptr, nullptr, m_out, wfold, lm);
  } else {
    // wave 3: first rehearse the transcript's two round paths on a scratch
    // state (instruction cache; rounds 0-1 otherwise run cold), then (JB > 0)
    // fold m in place over variables 0, 1, 2 as r_0, r_1, r_2 come out, so
    // that lm[d QA + x] (d: the bits of variables 3, 4, 5) is group B's split
    // table well before the corner wave's round-6 transition needs it.
    if (tdma) {  // the table, HBM -> LDS (1 KiB per instruction; waited for below)
      for (uint32_t i = 0; i < S0; i += 64)
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(Tin + i + lane),
                                         (__attribute__((address_space(3))) void*)(lm + i),
                                         16, 0, 0);
    }
    if (MLH_REH == 1) transcript_rehearsal(S, s, kwx, true);
    if (MLH_REH != 0) transcript_rehearsal(S, s, kwx, false);
    MLH_COOP_TS(9, 1);
    if (tdma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (JB) {
      uint32_t n = 1u << a;
      for (uint32_t u = 0; u < 3; ++u) {
        lds_wait_ge(S, &S.r_seq, u + 1);
        MLH_COOP_TS(9, 2 + 2 * u);
        const fe r = lds_fe(S.rsh[u]);
        n >>= 1;
        if (n % 256 == 0) {
          // four lerps per lane per step, loads first (their LDS latency
          // overlaps), the products as generated butterflies with r expanded
          // (u + r d, d = hi - lo: 60 VALU per pair half instead of ~100)
          const fe two32 = fe{{0u, 1u, 0u, 0u}};
          const fe R1 = fe_mul_s(r, two32), R2 = fe_mul_s(R1, two32), R3 = fe_mul_s(R2, two32);
          for (uint32_t i0 = lane; i0 < n; i0 += 256) {
            fe a[4], d[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
              a[k] = lm[i0 + 64 * k];
              d[k] = lm[i0 + 64 * k + n];
            }
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) d[k] = fe_sub(d[k], a[k]);
            uint64_t rare;
            bfly_mm_v(a[0], d[0], r, R1, R2, R3, a[1], d[1], r, R1, R2, R3, rare);
            bfly_mm_v(a[2], d[2], r, R1, R2, R3, a[3], d[3], r, R1, R2, R3, rare);
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) lm[i0 + 64 * k] = relaxed_canon(a[k]);
          }
        } else {
          for (uint32_t i = lane; i < n; i += 64) lm[i] = lerp_s(lm[i], lm[i + n], r);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // the next level reads other lanes' entries
        MLH_COOP_TS(9, 3 + 2 * u);
      }
      lds_publish(&S.mseq, 1);
      MLH_COOP_TS(9, 0);
    }
  }
  coop_report(S, ctl);
  if (ho.dst) {  // the prove's results straight into pinned host memory (no copy launch)
    __syncthreads();  // every role's writes done
    const uint32_t* src = reinterpret_cast<const uint32_t*>(ho.src);
    uint32_t* dst = reinterpret_cast<uint32_t*>(ho.dst);
    for (uint32_t i = threadIdx.x; i < ho.bytes / 4; i += blockDim.x) dst[i] = src[i];
  }
}

// The last rounds of a device-resident sumcheck (tables of S <= kTailMax
// entries) in ONE workgroup with m and d staged in LDS: per round the round
// polynomial + Fiat-Shamir step (lane 0, as sumcheck_round_kernel), then one
// phase that folds with r AND accumulates the next round's sums over the
// folded values (as fold_sums_kernel: lane i owns pairs i, i + q of the
// folded table, so no other lane touches its entries), then the reduction.
// The tables are folded in place exactly as fold_kernel does; the folded half
// is written back at the end.
#ifndef MLH_TAIL_THREADS
#define MLH_TAIL_THREADS 256
#endif
__device__ __forceinline__ void tail_sums(const fe* lm, const fe* ld, uint32_t h, fe& s1, fe& s2) {
  for (uint32_t i = threadIdx.x; i < h; i += blockDim.x) {
    const fe m0 = lm[i], m1 = lm[i + h], d0 = ld[i], d1 = ld[i + h];
    s1 = fe_add(s1, fe_mul(m1, d1));
    s2 = fe_add(s2, fe_mul(fe_sub(fe_dbl(m1), m0), fe_sub(fe_dbl(d1), d0)));
  }
}

__global__ void __launch_bounds__(MLH_TAIL_THREADS)
sumcheck_tail_kernel(fe* m, fe* __restrict__ d, uint32_t S, fe* prev, DevSha* t, fe* polys,
                     fe* rs, const fe* msrc) {
  extern __shared__ fe tail_lds[];
  fe* lm = tail_lds;
  fe* ld = tail_lds + S;
  __shared__ DevSha sh;
  __shared__ fe r_sh;
  __shared__ uint32_t stage[8];
  if (threadIdx.x < sizeof(DevSha) / 4)
    reinterpret_cast<uint32_t*>(&sh)[threadIdx.x] = reinterpret_cast<const uint32_t*>(t)[threadIdx.x];
  MLH_TAIL_TS(0);
  fe p = fe_zero();
  if (threadIdx.x == 0) p = fe_load(prev);
  for (uint32_t i = threadIdx.x; i < S; i += blockDim.x) {
    lm[i] = fe_load(msrc + i);
    ld[i] = fe_load(d + i);
  }
  __syncthreads();
  MLH_TAIL_TS(1);
  const uint32_t S0 = S;
  fe s1 = fe_zero(), s2 = fe_zero();
  tail_sums(lm, ld, S / 2, s1, s2);
  MLH_TAIL_TS(2);
  for (uint32_t k = 0; S > 1; ++k, S /= 2) {
    const uint32_t h = S / 2;
    MLH_TAIL_TS(51 + k);
    block_reduce2(s1, s2);
    MLH_TAIL_TS(3 + 4 * k);
    if (threadIdx.x == 0) {
      const fe e0 = fe_sub(p, s1);
      const fe c2 = fe_half(fe_add(fe_sub(s2, fe_add(s1, s1)), e0));
      const fe c1 = fe_sub(fe_sub(s1, e0), c2);
      fe_store(polys + 2 * k, c1);
      fe_store(polys + 2 * k + 1, c2);
      const uint32_t w[8] = {c1.w[0], c1.w[1], c1.w[2], c1.w[3], c2.w[0], c2.w[1], c2.w[2], c2.w[3]};
      dsha_absorb<8>(sh, w, stage);  // LE16(c1) || LE16(c2)
      MLH_TAIL_TS(4 + 4 * k);
      const fe r = dsha_challenge(sh);
      MLH_TAIL_TS(5 + 4 * k);
      fe_store(rs + k, r);
      p = fe_add(e0, fe_mul(r, fe_add(c1, fe_mul(c2, r))));
      r_sh = r;
    }
    __syncthreads();
    MLH_TAIL_TS(6 + 4 * k);
    const fe r = r_sh;
    s1 = fe_zero();
    s2 = fe_zero();
    if (h >= 2) {  // fold S -> h, next round's sums over pairs (i, i + q) of the folded table
      const uint32_t q = h / 2;
      for (uint32_t i = threadIdx.x; i < q; i += blockDim.x) {
        const fe m0 = lerp(lm[i], lm[i + h], r), m1 = lerp(lm[i + q], lm[i + q + h], r);
        const fe d0 = lerp(ld[i], ld[i + h], r), d1 = lerp(ld[i + q], ld[i + q + h], r);
        lm[i] = m0;
        lm[i + q] = m1;
        ld[i] = d0;
        ld[i + q] = d1;
        s1 = fe_add(s1, fe_mul(m1, d1));
        s2 = fe_add(s2, fe_mul(fe_sub(fe_dbl(m1), m0), fe_sub(fe_dbl(d1), d0)));
      }
    } else if (threadIdx.x == 0) {  // last round: fold the final pair
      lm[0] = lerp(lm[0], lm[1], r);
      ld[0] = lerp(ld[0], ld[1], r);
    }
    // (block_reduce2 at the top of the next round orders these LDS writes
    // before any other lane reads them)
  }
  __syncthreads();
  // the folds only ever write the first half (entries >= S0/2 keep their
  // input values), so that half is all there is to write back
  for (uint32_t i = threadIdx.x; i < S0 / 2; i += blockDim.x) {
    fe_store(m + i, lm[i]);
    fe_store(d + i, ld[i]);
  }
  if (threadIdx.x == 0) {
    *t = sh;
    fe_store(prev, p);
  }
  MLH_TAIL_TS(63);
}

uint32_t sumcheck_tail_rounds(uint32_t log_height) {
  return log_height < kTailLogMax ? log_height : kTailLogMax;
}

hipError_t launch_sumcheck_tail(fe* m, fe* d, uint32_t log_s, fe* prev, DevSha* t, fe* polys,
                                fe* rs, hipStream_t st, const fe* m_src) {
  if (log_s == 0 || log_s > kTailLogMax) return hipErrorInvalidValue;
  const uint32_t S = 1u << log_s;
  // 256 threads: 1024 measured slower (150 vs 127 us for 12 rounds) -- a
  // round is dominated by lane 0's SHA-256 work, the rest by barriers
  hipLaunchKernelGGL(sumcheck_tail_kernel, dim3(1), dim3(MLH_TAIL_THREADS), 2 * S * sizeof(fe), st,
                     m, d, S, prev, t, polys, rs, m_src ? m_src : m);
  return hipGetLastError();
}

hipError_t launch_sumcheck_round(const fe* partials, uint32_t nparts, fe* prev, DevSha* t,
                                 fe* poly_out, fe* r_out, hipStream_t st) {
  hipLaunchKernelGGL(sumcheck_round_kernel, dim3(1), dim3(kRedThreads), 0, st, partials, nparts,
                     prev, t, poly_out, r_out);
  return hipGetLastError();
}

hipError_t launch_sumcheck_eq_tail(const fe* Tin, uint32_t Jin, const fe* rs_in, uint32_t a,
                                   const fe* ets, const fe* pts, fe* c, fe* prev, DevSha* t,
                                   fe* polys, fe* rs, fe* m_out, fe* d_out, hipStream_t st,
                                   CoopCtl ctl, const uint32_t* kw, HostOut ho, const fe* xc_part,
                                   uint32_t xc_nb, const fe* rsuf) {
  if (a == 0 || a > kTailLogMax || Jin > 3 || (xc_part && (Jin || a < 6 || xc_nb == 0)) ||
      (rsuf && Jin))
    return hipErrorInvalidValue;
  const uint32_t JA = a < 6 ? a : 6, S0 = 1u << a;
  const size_t lds = ((1ull << a) + (1ull << (a - JA))) * sizeof(fe);  // m + e_{JA-1}
  hipLaunchKernelGGL(sumcheck_eq_tail_kernel, dim3(1), dim3(kRedThreads), lds, st, Tin, Jin, rs_in,
                     a, ets + (S0 - (S0 >> (JA - 1))), pts, c, prev, t, polys, rs, m_out, d_out, kw,
                     (fe*)nullptr, ctl, ho, xc_part, xc_nb, rsuf);
  return hipGetLastError();
}

// Y[c] = sum_{i < 2^a} T[c 2^a + i] lo[i], c < 2^B: a workgroup takes
// MLH_CS_CPB consecutive corners (CPB * 2^a contiguous entries); a thread's
// lo entries stay in registers across them, its table loads are issued 8 at a
// time, and the CPB sums leave through one block reduction.
#ifndef MLH_CS_CPB
#define MLH_CS_CPB 1
#endif
__global__ void __launch_bounds__(kRedThreads)
corner_sums_lo_kernel(const fe* __restrict__ T, uint32_t a, const fe* __restrict__ lo,
                      fe* __restrict__ Y) {
  constexpr int CPB = MLH_CS_CPB, PER = 16;  // 2^a = 4096 entries: 16 per thread
  const uint64_t Q = 1ull << a;
  const uint32_t c0 = blockIdx.x * CPB;
  fe lv[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) lv[k] = fe_load(lo + threadIdx.x + k * kRedThreads);
  fe acc[CPB];
#pragma unroll
  for (int q = 0; q < CPB; ++q) {
    const fe* Tc = T + (uint64_t)(c0 + q) * Q;
    sacc s0;
    sacc_zero(s0);
#pragma unroll
    for (int k0 = 0; k0 < PER; k0 += 8) {
      fe v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = sweep_load(Tc, threadIdx.x + (k0 + k) * kRedThreads);
#pragma unroll
      for (int k = 0; k < 8; ++k) sacc_mac(s0, v[k], lv[k0 + k]);
    }
    acc[q] = sacc_reduce(s0);
  }
  // one block reduction of the CPB sums
  __shared__ fe part[kRedThreads / 64][CPB];
#pragma unroll
  for (int q = 0; q < CPB; ++q) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) acc[q] = fe_add(acc[q], shfl_xor_fe(acc[q], m));
  }
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < CPB; ++q) part[threadIdx.x >> 6][q] = acc[q];
  __syncthreads();
  if (threadIdx.x < CPB) {
    fe x = part[0][threadIdx.x];
    for (int w = 1; w < kRedThreads / 64; ++w) x = fe_add(x, part[w][threadIdx.x]);
    fe_store(Y + c0 + threadIdx.x, x);
  }
}

hipError_t launch_corner_sums_lo(const fe* T, uint32_t B, uint32_t a, const fe* lo, fe* Y,
                                 hipStream_t st) {
  if (B > 12 || a != 12 || (1u << B) % MLH_CS_CPB) return hipErrorInvalidValue;
  hipLaunchKernelGGL(corner_sums_lo_kernel, dim3((1u << B) / MLH_CS_CPB), dim3(kRedThreads), 0, st, T,
                     a, lo, Y);
  return hipGetLastError();
}

hipError_t launch_sumcheck_eq_head(const fe* Y, uint32_t B, const fe* e_grp, const fe* pts, fe* c,
                                   fe* prev, DevSha* t, fe* polys, fe* rs, fe* wfold,
                                   hipStream_t st, CoopCtl ctl, const uint32_t* kw, const fe* rsuf) {
  if (B == 0 || B > kTailLogMax || !wfold) return hipErrorInvalidValue;
  const uint32_t JA = B < 6 ? B : 6;
  const size_t lds = ((1ull << B) + (1ull << (B - JA))) * sizeof(fe);
  hipLaunchKernelGGL(sumcheck_eq_tail_kernel, dim3(1), dim3(kRedThreads), lds, st, Y, 0u,
                     (const fe*)nullptr, B, e_grp, pts, c, prev, t, polys, rs, (fe*)nullptr,
                     (fe*)nullptr, kw, wfold, ctl, HostOut{}, (const fe*)nullptr, 0u, rsuf);
  return hipGetLastError();
}

hipError_t launch_sumcheck_group(const fe* partials, uint32_t nb, uint32_t J, uint32_t J2,
                                 uint32_t t0, uint32_t t1, fe* prev, DevSha* t, fe* polys, fe* rs,
                                 const fe* pts, fe* c, hipStream_t st, CoopCtl ctl,
                                 const uint32_t* kw, fe* wout) {
  if (J < 1 || J > 3 || J2 > 3 || t0 >= t1 || t1 > J || (J2 && (t0 != 0 || t1 != J)) || nb == 0 ||
      (nb << (J + J2)) > 2 * kMaxRedBlocks)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(sumcheck_group_kernel, dim3(1), dim3(kRedThreads), 0, st, partials, nb, J, J2,
                     t0, t1, prev, t, polys, rs, pts, c, kw, wout, ctl);
  return hipGetLastError();
}

hipError_t launch_pcs_round(const fe* src, fe* dst, uint32_t log_h, bool fold, const fe* r_prev,
                            const fe* p_prev, const fe* p_k, const fe* e, PcsRoundState* st,
                            fe* poly_out, hipStream_t stream) {
  if (log_h < 1 || log_h > kTailLogMax || (fold && !r_prev) || (r_prev && !p_prev))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(pcs_round_kernel, dim3(1), dim3(kRedThreads), 0, stream,
                     PcsJob{src, dst, log_h, fold ? 1u : 0u, r_prev, p_prev, p_k, e, st, poly_out});
  return hipGetLastError();
}

hipError_t launch_eq_weights(const fe* rs, uint32_t JA, uint32_t JB, fe* wf, hipStream_t st) {
  if (JA > 6 || JB > 6) return hipErrorInvalidValue;
  hipLaunchKernelGGL(eq_weights_kernel, dim3(1), dim3(128), 0, st, rs, JA, JB, wf);
  return hipGetLastError();
}

}  // namespace mlh

#ifdef MLH_COOP_PROF
// Dev builds only (tools/coop_pipeline.py): the last cooperative launch's
// per-round stamps (g_coop_ts, 10 x 64) and edges (g_coop_edge, 4).
extern "C" int mlh_debug_coop_stamps(uint64_t* ts_out, uint64_t* edge_out) {
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(ts_out, HIP_SYMBOL(mlh::g_coop_ts), sizeof(uint64_t) * 640) != hipSuccess)
    return 1;
  return hipMemcpyFromSymbol(edge_out, HIP_SYMBOL(mlh::g_coop_edge), sizeof(uint64_t) * 4) != hipSuccess;
}
#endif
