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
#include "transcript_dev.hpp"

namespace mlh {

constexpr int kRedThreads = 256;
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
__device__ __forceinline__ fe lerp_s(const fe& lo, const fe& hi, const fe& r) {
  return fe_add(lo, fe_mul_s(fe_sub(hi, lo), r));
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
constexpr uint32_t kGroupHLds = 1024;  // group_sums_eq_kernel: H entries staged in LDS (16 KiB)
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
  acc9 s0, s1;  // unreduced (two for ILP); < 2^288 for < 2^32 products each
  acc_zero(s0);
  acc_zero(s1);
  const uint64_t stride = (uint64_t)nbc * blockDim.x;
  const uint64_t i0 = (uint64_t)bb * blockDim.x + threadIdx.x;
  uint64_t i = i0;
  for (; i + stride < Q; i += 2 * stride) {  // two entries in flight per thread
    const fe h0 = fe_load(H + (i >> a)), h1 = fe_load(H + ((i + stride) >> a));
    const fe v0 = fe_load(Tc + i), v1 = fe_load(Tc + i + stride);
    mulacc(s0, v0, h0);
    mulacc(s1, v1, h1);
  }
  if (i < Q) mulacc(s0, fe_load(Tc + i), fe_load(H + (i >> a)));
  fe acc = fe_add(acc_reduce(s0), acc_reduce(s1));
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
      acc9 t;
      acc_zero(t);
#pragma unroll
      for (int c0 = 0; c0 < (1 << J); c0 += 8) {  // 8 loads in flight at a time
        fe tv[8];
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (c0 + c < (1 << J)) tv[c] = fe_load(Tin + (uint64_t)(c0 + c) * Sp + x);
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

// out[i] = in[bitrev(i)] (bit_reverse_permutation, src/ntt/mod.rs:113-123).
__global__ void __launch_bounds__(256)
bitrev_kernel(const fe* __restrict__ in, fe* __restrict__ out, uint32_t log_n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (1ull << log_n)) return;
  const uint64_t j = log_n ? (__builtin_bitreverse64(i) >> (64 - log_n)) : 0;
  fe_store(out + i, fe_load(in + j));
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
__global__ void __launch_bounds__(256)
eq_setup_kernel(const EqSetupArgs args, fe* __restrict__ pts_out, fe* __restrict__ c_out,
                fe* __restrict__ lo, fe* __restrict__ H, fe* __restrict__ Hs, DevSha* dt_out,
                fe* prev_out, uint32_t* __restrict__ kw) {
  const uint32_t L = args.L, B = args.B, a = L - B;
  const uint64_t NL = 1ull << a, NH = (1ull << B) - 1, NS = Hs ? NL - 1 : 0;
  uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // kw: per round k whose absorb of (c1, c2) empties the buffer, the padding
  // block's K + W table (the transcript then grows 32 bytes per round)
  if (kw && x >= NL + NH + NS && x < NL + NH + NS + L) {
    const uint32_t k = (uint32_t)(x - (NL + NH + NS));
    const uint64_t len = args.sha.len + 32ull * (k + 1);
    if ((len & 63) == 0) sha256_pad_kw(len, kw + 64 * k);
    return;
  }
  if (x == 0) {
    for (uint32_t i = 0; i < L; ++i) pts_out[i] = args.pts[i];
    *c_out = fe_one();
    if (dt_out) *dt_out = args.sha;
    if (prev_out) *prev_out = args.sum;
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
  fe acc = fe_one();
  for (uint32_t i = 0; i < cnt; ++i) {
    const fe p = q[n - 1 - i];
    acc = fe_mul(acc, ((j >> i) & 1) ? p : fe_sub(fe_one(), p));
  }
  fe_store(out, acc);
}

hipError_t launch_eq_setup(const EqSetupArgs& args, fe* pts_out, fe* c_out, fe* lo, fe* H, fe* Hs,
                           DevSha* dt_out, fe* prev_out, hipStream_t st, uint32_t* kw) {
  if (args.L == 0 || args.L > 40 || args.B > args.L || args.L - args.B > kTailLogMax)
    return hipErrorInvalidValue;
  const uint64_t NL = 1ull << (args.L - args.B);
  const uint64_t total = NL + (1ull << args.B) - 1 + (Hs ? NL - 1 : 0) + (kw ? args.L : 0);
  hipLaunchKernelGGL(eq_setup_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, args,
                     pts_out, c_out, lo, H, Hs, dt_out, prev_out, kw);
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
  while ((uint64_t)nbc * kRedThreads < (1ull << a)) nbc *= 2;  // stride >= 2^a
  if ((nbc << J) > 2 * kMaxRedBlocks) return hipErrorInvalidValue;
  *nb = nbc;
  hipLaunchKernelGGL(group_sums_eq_kernel, dim3(nbc << J), dim3(kRedThreads), 0, st, T, S, J, H, lo,
                     a, nbc, partials);
  return hipGetLastError();
}

hipError_t launch_fold_group_eq(const fe* Tin, uint64_t S, uint32_t J, uint32_t JN, const fe* rs,
                                const fe* w, fe* Tout, const fe* H, const fe* lo, uint32_t a,
                                fe* partials, hipStream_t st, uint32_t* nb) {
  if (J < 1 || J > kMaxGroup || JN > kMaxGroup || a < 8 || (S >> (J + JN)) < (1ull << a) || !w)
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
__device__ __forceinline__ fe round_step(const fe& s1, const fe& s2, fe& claim, DevSha& s,
                                         uint32_t* stage, fe* poly_out, fe* r_out) {
  const fe e0 = fe_sub(claim, s1);
  const fe c2 = fe_half(fe_add(fe_sub(s2, fe_add(s1, s1)), e0));
  const fe c1 = fe_sub(fe_sub(s1, e0), c2);
  fe_store(poly_out, c1);
  fe_store(poly_out + 1, c2);
  const uint32_t w[8] = {c1.w[0], c1.w[1], c1.w[2], c1.w[3], c2.w[0], c2.w[1], c2.w[2], c2.w[3]};
  dsha_absorb<8>(s, w, stage);  // LE16(c1) || LE16(c2)
  const fe r = dsha_challenge(s);
  fe_store(r_out, r);
  claim = fe_add(e0, fe_mul(r, fe_add(c1, fe_mul(c2, r))));
  return r;
}
// One two-table round (mlh_sumcheck_prove's per-round path, the PCS's rounds
// after the eq-factored head, mlh_device_sumcheck_round): reduce the
// per-workgroup partial (s1, s2) = p(1), p(2) pairs, then lane 0 runs
// round_step (the closed-form interpolation on x = 0,1,2 of polynomials.rs:51-87,
// absorb LE16(c1) || LE16(c2) as sumcheck.rs:188-199, r = next_challenge(),
// claim = p(r)).
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
  if (threadIdx.x != 0) return;
  round_step(s1, s2, p, s, stage, poly_out, r_out);
  *t = s;
  fe_store(prev, p);
}

// out = P + Q (R + S T): the one two-modmul form every lane-parallel step of
// sumcheck_group_kernel is cast in, so independent chains (corner weights,
// the claim p(r), the eq scale) run side by side on different lanes.
__device__ __forceinline__ fe pqrst(const fe& P, const fe& Q, const fe& R, const fe& S,
                                    const fe& T) {
  return fe_add(P, fe_mul_s(fe_add(R, fe_mul_s(S, T)), Q));
}
// The same lane's value as a wave-uniform (v_readlane): no LDS round trip.
__device__ __forceinline__ fe bcast_fe(const fe& x, int src) {
  fe r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.w[i] = (uint32_t)__builtin_amdgcn_readlane((int)x.w[i], src);
  return r;
}
// x from the lane at the given DPP pattern (quad_perm / row_half_mirror).
template <int CTRL>
__device__ __forceinline__ fe dpp_fe(const fe& x) {
  fe r;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    r.w[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)x.w[i], CTRL, 0xF, 0xF, true);
  return r;
}
// Sum over each aligned group of n (2, 4 or 8) lanes, every lane of the group
// ending with it: DPP butterflies (xor 1, xor 2 quad_perms, then the mirror
// within 8 lanes, which pairs the two summed quads), no LDS crossbar.
__device__ __forceinline__ fe group_sum_dpp(fe x, uint32_t n) {
  if (n > 1) x = fe_add(x, dpp_fe<0xB1>(x));   // quad_perm [1,0,3,2]
  if (n > 2) x = fe_add(x, dpp_fe<0x4E>(x));   // quad_perm [2,3,0,1]
  if (n > 4) x = fe_add(x, dpp_fe<0x141>(x));  // row_half_mirror
  return x;
}
__device__ __forceinline__ fe shfl_fe(const fe& x, int src) {
  fe r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.w[i] = (uint32_t)__shfl((int)x.w[i], src, 64);
  return r;
}

// Wave 0 (all 64 lanes) runs rounds t0..t1-1 of a group of J eq-factored
// rounds from its corner sums, lanes split by role: lanes 8..15 hold the
// corner sums (lane 8 + c: X_c), lane 0 the claim and the round's
// interpolation / transcript, lane 1 the eq scale c (v: lane 0 the claim,
// lane 1 c, on entry and on exit).  Per round: step A (pqrst on every lane) =
// corner weights + the previous round's claim p(r) (lane 0) and scale
// c <- c (1 - p - r + 2 r p) (lane 1); a 3-level shuffle sum gives E0/E1;
// step B (pqrst) = s1 = (c p) E1 on lane 0 and s2 = (c (3p - 1)) (2 E1 - E0) on
// lane 1; lane 0 interpolates, absorbs and draws r.  p / r: the group's
// points / challenges (r[u] for u < t0 known on entry; the rest filled in);
// polys: round t0's slot; rs: round 0's r slot (lane 0 stores r_t at rs + t);
// kw (or nullptr): per round t the padding-block K + W table at kw + 64 t
// (eq_setup_kernel; used when round t's absorb leaves the buffer empty).
__device__ __forceinline__ void eq_group_rounds(const fe& X, uint32_t J, uint32_t t0, uint32_t t1,
                                                const fe (&p)[3], fe (&r)[3], fe& v, DevSha& s,
                                                uint32_t* stage, fe* polys, fe* rs,
                                                const uint32_t* kw) {
  const uint32_t NC = 1u << J;
  const uint32_t lane = threadIdx.x & 63;
  const bool is0 = lane == 0, is1 = lane == 1;
  const bool wl = lane >= 8 && lane < 8 + NC;  // corner-weight lane
  const uint32_t cl = lane - 8;                // its corner
  const fe one = fe_one();
  // A corner lane's weight in round t is X_c times the J - 1 factors
  // (c_u ? x_u : 1 - x_u), u != t, x_u = r_u (u < t) or p_u (u > t), kept in
  // increasing u in F0, F1 (one when absent).  Going from round t to t + 1
  // only slot t changes (p_{t+1}'s factor becomes r_t's), so after each
  // challenge one factor is replaced instead of all being re-selected.
  fe F0 = one, F1 = one;
  {
    uint32_t k = 0;
#pragma unroll
    for (uint32_t u = 0; u < 3; ++u) {
      if (u >= J || u == t0) continue;
      const fe x = u < t0 ? r[u] : p[u];
      const fe f = (cl >> (J - 1 - u)) & 1u ? x : fe_sub(one, x);
      if (k == 0) F0 = f; else F1 = f;
      ++k;
    }
  }
  // step A operands, v = P + Q (R + S T): round t0 keeps the claim (lane 0)
  // and the eq scale (lane 1) as given; corner lanes X F0 F1
  fe P = is0 || is1 ? v : fe_zero(), Q = wl ? X : fe_zero(), R = fe_zero(), S = F0, T = F1;
  for (uint32_t tt = t0;; ++tt) {
    const int tb = 3 + 8 * (int)tt;
    (void)tb;
    v = pqrst(P, Q, R, S, T);
    if (tt == t1) break;
    MLH_TAIL_TS(tb);
    const fe pv = tt == 0 ? p[0] : (tt == 1 ? p[1] : p[2]);  // wave-uniform
    const bool bt = (cl >> (J - 1 - tt)) & 1u;
    fe E0 = wl && !bt ? v : fe_zero(), E1 = wl && bt ? v : fe_zero();
    E0 = group_sum_dpp(E0, NC);  // corner lanes 8..8+NC: an aligned group
    E1 = group_sum_dpp(E1, NC);
    MLH_TAIL_TS(tb + 1);
    // step B: lane 0 s1 = E1 (c p), the others s2 = (2 E1 - E0)(c (3p - 1))
    E0 = bcast_fe(E0, 8);
    E1 = bcast_fe(E1, 8);
    const fe cs = bcast_fe(v, 1);
    const fe sB = fe_mul_s(fe_mul_s(cs, is0 ? pv : fe_sub(fe_add(fe_dbl(pv), pv), one)),
                           is0 ? E1 : fe_sub(fe_dbl(E1), E0));
    const fe s2 = bcast_fe(sB, 1);
    MLH_TAIL_TS(tb + 2);
    fe rr = fe_zero(), e0 = fe_zero(), c1 = fe_zero(), c2 = fe_zero();
    if (is0) {
      const fe s1 = sB;
      e0 = fe_sub(v, s1);
      c2 = fe_half(fe_add(fe_sub(s2, fe_add(s1, s1)), e0));
      c1 = fe_sub(fe_sub(s1, e0), c2);
      fe* po = polys + 2 * (tt - t0);
      fe_store(po, c1);
      fe_store(po + 1, c2);
      const uint32_t w[8] = {c1.w[0], c1.w[1], c1.w[2], c1.w[3], c2.w[0], c2.w[1], c2.w[2], c2.w[3]};
      MLH_TAIL_TS(tb + 3);
      dsha_absorb<8>(s, w, stage);  // LE16(c1) || LE16(c2)
      MLH_TAIL_TS(tb + 4);
      rr = dsha_challenge_kw(s, kw ? kw + 64 * tt : nullptr);
      MLH_TAIL_TS(tb + 5);
      fe_store(rs + tt, rr);
    }
    rr = bcast_fe(rr, 0);
    if (tt == 0) r[0] = rr; else if (tt == 1) r[1] = rr; else r[2] = rr;
    // the next round's factor slot tt: r_t's in place of p_{t+1}'s
    const fe f = bt ? rr : fe_sub(one, rr);
    if (tt == 0) F0 = f; else if (tt == 1) F1 = f;
    // step A of the next round: lane 0 the claim e0 + r (c1 + c2 r), lane 1
    // the scale c ((1 - p) + r (2p - 1)), corner lanes X F0 F1
    P = e0;  // zero off lane 0
    Q = is0 ? rr : (is1 ? v : Q);
    R = is0 ? c1 : (is1 ? fe_sub(one, pv) : fe_zero());
    S = is0 ? c2 : (is1 ? rr : F0);
    T = is0 ? rr : (is1 ? fe_sub(fe_dbl(pv), one) : F1);
    MLH_TAIL_TS(tb + 7);
  }
}

// Rounds t0..t1-1 of a group of J eq-factored head rounds k..k+J-1 from the
// corner sums (see "grouped eq-factored rounds"): the NC x nb partials are
// summed 32 lanes per corner, then wave 0 runs eq_group_rounds.  pts, rs:
// p_k.., r_k.. (rs[u] for u < t0 were written by earlier launches of this
// group).
__global__ void __launch_bounds__(kRedThreads)
sumcheck_group_kernel(const fe* __restrict__ partials, uint32_t nb, uint32_t J, uint32_t J2,
                      uint32_t t0, uint32_t t1, fe* prev, DevSha* t, fe* polys, fe* rs,
                      const fe* __restrict__ pts, fe* cdev, const uint32_t* __restrict__ kw,
                      fe* wout) {
  __shared__ DevSha s;
  __shared__ uint32_t stage[8];
  __shared__ fe slot[64];
  MLH_TAIL_TS(0);
  if (threadIdx.x < sizeof(DevSha) / 4)
    reinterpret_cast<uint32_t*>(&s)[threadIdx.x] = reinterpret_cast<const uint32_t*>(t)[threadIdx.x];
  const uint32_t JT = J + J2, NC = 1u << JT, G = kRedThreads >> JT;  // threads per corner
  const uint32_t GW = G < 64 ? G : 64;                                // ... within one wave
  {
    const uint32_t c = threadIdx.x / G, j = threadIdx.x % G;
    fe acc = fe_zero();
#pragma unroll 4
    for (uint32_t b = j; b < nb; b += G) acc = fe_add(acc, fe_load(partials + (uint64_t)c * nb + b));
    MLH_TAIL_TS(1);
    for (uint32_t m = GW / 2; m >= 1; m >>= 1) acc = fe_add(acc, shfl_xor_fe(acc, m));
    if (threadIdx.x % GW == 0) slot[threadIdx.x / GW] = acc;
  }
  __syncthreads();
  MLH_TAIL_TS(2);
  if (threadIdx.x >= 64) return;
  const uint32_t lane = threadIdx.x, per = G / GW;  // slots per corner
  // lane c < NC: the corner sum Y_c
  fe Y = fe_zero();
  if (lane < NC)
    for (uint32_t q = 0; q < per; ++q) Y = fe_add(Y, slot[lane * per + q]);
  fe p[3], r[3];
#pragma unroll
  for (uint32_t u = 0; u < 3; ++u) {
    p[u] = u < J ? fe_load(pts + u) : fe_zero();
    r[u] = u < t0 ? fe_load(rs + u) : fe_zero();
  }
  // lane 0: the claim; lane 1: the eq scale
  fe v = lane == 0 ? fe_load(prev) : (lane == 1 ? fe_load(cdev) : fe_zero());
  const fe one = fe_one();
  // one group (J2 == 0): its corner sums; two chained groups over the corners
  // c = (c_hi: J bits, c_lo: J2 bits): group 1's corner sums sum out c_lo with
  // its eq weights, group 2's fold c_hi with group 1's challenges (see
  // "grouped eq-factored rounds").  One loop body for both (code size: the
  // one-lane transcript is instruction-fetch bound).
  const uint32_t chi = lane >> J2, clo = lane & ((1u << J2) - 1);
  fe w1 = fe_one();  // two groups: group 1's factor of the fold weight (lane = corner)
  for (uint32_t g = 0; g < (J2 ? 2u : 1u); ++g) {
    const uint32_t Jg = g ? J2 : J;
    fe x = Y;
    if (J2) {
      fe pr[3];  // the summed-out variables' factors: group 2's points / group 1's challenges
      if (g == 0) {
#pragma unroll
        for (uint32_t u = 0; u < 3; ++u) pr[u] = u < J2 ? fe_load(pts + J + u) : fe_zero();
      } else {
#pragma unroll
        for (uint32_t u = 0; u < 3; ++u) pr[u] = r[u];
      }
      const uint32_t nb_ = g ? J : J2, bits = g ? chi : clo;
#pragma unroll
      for (uint32_t u = 0; u < 3; ++u)
        if (u < nb_) x = fe_mul_s(x, (bits >> (nb_ - 1 - u)) & 1u ? pr[u] : fe_sub(one, pr[u]));
      const uint32_t m0 = g ? 1u << J2 : 1u, m1 = g ? NC : 1u << J2;
      for (uint32_t m = m0; m < m1; m <<= 1) x = fe_add(x, shfl_xor_fe(x, m));
      if (g == 1) {
        // group 1's factor of this lane's fold weight, while its r's are at hand
#pragma unroll
        for (uint32_t u = 0; u < 3; ++u)
          if (u < J) w1 = fe_mul_s(w1, (chi >> (J - 1 - u)) & 1u ? r[u] : fe_sub(one, r[u]));
#pragma unroll
        for (uint32_t u = 0; u < 3; ++u) {
          p[u] = u < J2 ? fe_load(pts + J + u) : fe_zero();
          r[u] = fe_zero();
        }
      }
    }
    // group g's corner sum X_c to lane 8 + c (group 1 of two: from lane c << J2)
    const uint32_t src = (g == 0 && J2) ? ((lane - 8) << J2) : (lane - 8);
    const fe X = shfl_fe(x, src & 63);
    eq_group_rounds(lane >= 8 && lane < 8 + (1u << Jg) ? X : fe_zero(), Jg, g ? 0 : t0,
                    g ? Jg : t1, p, r, v, s, stage, g ? polys + 2 * J : polys, g ? rs + J : rs,
                    kw ? (g ? kw + 64 * J : kw) : nullptr);
  }
  if (lane == 0) {
    *t = s;
    fe_store(prev, v);
  }
  if (lane == 1) fe_store(cdev, v);
  // the eq weights of the finished group's challenges for the fold pass:
  // w_c = prod_u (c_u ? r_u : 1 - r_u) over the J (+ J2) variables, lane c
  if (wout && t1 == J && lane < NC) {
    fe wc = w1;  // J2 == 0: r holds the group's challenges; else group 2's
    const uint32_t nbits = J2 ? J2 : J, bits = J2 ? clo : chi;
#pragma unroll
    for (uint32_t u = 0; u < 3; ++u)
      if (u < nbits) wc = fe_mul_s(wc, (bits >> (nbits - 1 - u)) & 1u ? r[u] : fe_sub(one, r[u]));
    fe_store(wout + lane, wc);
  }
  MLH_TAIL_TS(63);
}

// The last a rounds of an eq-factored sumcheck (mlh_sumcheck_prove_eq) in ONE
// workgroup: the 2^a-entry matrix table m and the suffix tables e_j =
// eq(p_{B+j+1}..p_{L-1}) (2^(a-1-j) entries at offset 2^a - 2^(a-j), as H_k)
// staged in LDS, delta = c eq(p_B..) never materialised.  The rounds go in
// groups of up to 3 exactly as the HBM head groups: corner sums of the group
// over m (all waves), the group's rounds on wave 0 (eq_group_rounds), a
// J-level fold of m in LDS.  On load, m is Tin folded over Jin <= 3 pending
// variables with rs_in (the last head group's fold, fused here).  Writes the
// folded matrix m_out[0], the final delta c_L (eq of no points = 1) to
// d_out[0], the claim and the transcript.
__global__ void __launch_bounds__(kRedThreads)
sumcheck_eq_tail_kernel(const fe* Tin, uint32_t Jin, const fe* __restrict__ rs_in, uint32_t a,
                        const fe* __restrict__ ets, const fe* __restrict__ pts, fe* cdev, fe* prev,
                        DevSha* t, fe* polys, fe* rs, fe* m_out, fe* d_out,
                        const uint32_t* __restrict__ kw) {
  extern __shared__ fe eq_tail_lds[];
  fe* lm = eq_tail_lds;                 // 2^a
  fe* le = eq_tail_lds + (1u << a);     // 2^a - 1
  __shared__ DevSha s;
  __shared__ uint32_t stage[8];
  __shared__ fe slot[kRedThreads / 32];
  __shared__ fe r_sh[3];
  if (threadIdx.x < sizeof(DevSha) / 4)
    reinterpret_cast<uint32_t*>(&s)[threadIdx.x] = reinterpret_cast<const uint32_t*>(t)[threadIdx.x];
  const uint32_t S0 = 1u << a;
  MLH_TAIL_TS(38);
  {
    fe rin[3];
#pragma unroll
    for (uint32_t u = 0; u < 3; ++u) rin[u] = u < Jin ? fe_load(rs_in + u) : fe_zero();
    if (Jin == 0) {  // plain copies, 8 per thread in flight at a time
      for (uint32_t x0 = 0; x0 < S0; x0 += 8 * kRedThreads) {
        fe v[8], w[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
          const uint32_t x = x0 + u * kRedThreads + threadIdx.x;
          v[u] = x < S0 ? fe_load(Tin + x) : fe_zero();
          w[u] = x + 1 < S0 ? fe_load(ets + x) : fe_zero();
        }
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
          const uint32_t x = x0 + u * kRedThreads + threadIdx.x;
          if (x < S0) lm[x] = v[u];
          if (x + 1 < S0) le[x] = w[u];
        }
      }
    } else {
      for (uint32_t x = threadIdx.x; x < S0; x += blockDim.x) {
        lm[x] = fold_corners_n(Jin, Tin + x, S0, rin);
        if (x + 1 < S0) le[x] = fe_load(ets + x);
      }
    }
  }
  MLH_TAIL_TS(39);
  const uint32_t lane = threadIdx.x & 63;
  fe v = fe_zero();  // wave 0: lane 0 the claim, lane 1 the eq scale
  if (threadIdx.x == 0) v = fe_load(prev);
  if (threadIdx.x == 1) v = fe_load(cdev);
  __syncthreads();
  for (uint32_t j = 0; j < a;) {
    const uint32_t J = a - j < 3 ? a - j : 3, NC = 1u << J, G = kRedThreads >> J;
    const uint32_t S = S0 >> j, Q = S >> J;
    const fe* e = le + (S0 - (S0 >> (j + J - 1)));  // e_{j+J-1}: Q entries
    {  // corner sums of the group: 2^J corners x G threads
      const uint32_t c = threadIdx.x / G, jj = threadIdx.x % G;
      fe acc = fe_zero();
      for (uint32_t i = jj; i < Q; i += G) acc = fe_add(acc, fe_mul_s(lm[c * Q + i], e[i]));
#pragma unroll
      for (int m = 16; m >= 1; m >>= 1) acc = fe_add(acc, shfl_xor_fe(acc, m));
      if ((threadIdx.x & 31) == 0) slot[threadIdx.x >> 5] = acc;
    }
    __syncthreads();
    MLH_TAIL_TS(40 + 4 * (j / 3));
    if (threadIdx.x < 64) {
      fe X = fe_zero();
      if (lane >= 8 && lane < 8 + NC)
        for (uint32_t q = 0; q < G / 32; ++q) X = fe_add(X, slot[(lane - 8) * (G / 32) + q]);
      fe p[3], r[3];
#pragma unroll
      for (uint32_t u = 0; u < 3; ++u) {
        p[u] = u < J ? fe_load(pts + j + u) : fe_zero();
        r[u] = fe_zero();
      }
      eq_group_rounds(X, J, 0, J, p, r, v, s, stage, polys + 2 * j, rs + j,
                      kw ? kw + 64 * j : nullptr);
      if (lane == 0) {
        r_sh[0] = r[0];
        r_sh[1] = r[1];
        r_sh[2] = r[2];
      }
    }
    __syncthreads();
    MLH_TAIL_TS(41 + 4 * (j / 3));
    // fold m over the group's J variables (in place: output x reads corner 0 at x)
    const fe rr[3] = {r_sh[0], r_sh[1], r_sh[2]};
    for (uint32_t x = threadIdx.x; x < Q; x += blockDim.x) lm[x] = fold_corners_n(J, lm + x, Q, rr);
    __syncthreads();
    MLH_TAIL_TS(42 + 4 * (j / 3));
    j += J;
  }
  if (threadIdx.x == 0) {
    *t = s;
    fe_store(prev, v);
    fe_store(m_out, lm[0]);
  }
  if (threadIdx.x == 1) {
    fe_store(cdev, v);
    fe_store(d_out, v);
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
                                   const uint32_t* kw) {
  if (a == 0 || a > kTailLogMax || Jin > 3) return hipErrorInvalidValue;
  const size_t lds = (2ull << a) * sizeof(fe);
  hipLaunchKernelGGL(sumcheck_eq_tail_kernel, dim3(1), dim3(kRedThreads), lds, st, Tin, Jin, rs_in,
                     a, ets, pts, c, prev, t, polys, rs, m_out, d_out, kw);
  return hipGetLastError();
}

hipError_t launch_sumcheck_group(const fe* partials, uint32_t nb, uint32_t J, uint32_t J2,
                                 uint32_t t0, uint32_t t1, fe* prev, DevSha* t, fe* polys, fe* rs,
                                 const fe* pts, fe* c, hipStream_t st, const uint32_t* kw,
                                 fe* wout) {
  if (J < 1 || J > 3 || J2 > 3 || t0 >= t1 || t1 > J || (J2 && (t0 != 0 || t1 != J)) || nb == 0 ||
      (nb << (J + J2)) > 2 * kMaxRedBlocks)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(sumcheck_group_kernel, dim3(1), dim3(kRedThreads), 0, st, partials, nb, J, J2,
                     t0, t1, prev, t, polys, rs, pts, c, kw, wout);
  return hipGetLastError();
}

}  // namespace mlh
