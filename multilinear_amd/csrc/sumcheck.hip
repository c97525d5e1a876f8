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
#include "field.hpp"
#include "sumcheck.hpp"
#include "transcript_dev.hpp"

namespace mlh {

constexpr int kRedThreads = 256;
constexpr uint32_t kTailLogMax = 12;  // sumcheck_tail_kernel: 2 x 2^12 x 16 B = 128 KiB LDS

// Phase timestamps of sumcheck_tail_kernel (tools/tail_bench.hip builds this
// file with -DMLH_TAIL_PROF; compiled out otherwise).
#ifdef MLH_TAIL_PROF
__device__ uint64_t g_tail_ts[64];
#define MLH_TAIL_TS(i)                                        \
  do {                                                        \
    if (threadIdx.x == 0 && (i) < 64) g_tail_ts[i] = wall_clock64(); \
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
// eq(p_{k+1}..p_{L-a-1})).  The kernels stream only m: half the HBM traffic of
// the two-table rounds, and no 2^L eq table is ever written.  Thread counts are
// powers of two >= 2^a, so a thread's i mod 2^a is fixed: it accumulates
// m[i] * H[i >> a] and multiplies by lo once at the end (2 modmuls per pair).

// H_k for k = 0..B-1 concatenated: H_k = eq(p_{k+1}, ..., p_{B-1}) has
// 2^(B-1-k) entries at offset 2^B - 2^(B-k); entry j = prod_{i < B-1-k}
// (bit_i(j) ? p[B-1-i] : 1 - p[B-1-i]).
__global__ void eq_suffix_kernel(const fe* __restrict__ pts, uint32_t B, fe* __restrict__ out) {
  const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t total = (1ull << B) - 1;
  if (x >= total) return;
  const uint64_t y = (1ull << B) - x;                  // >= 2
  const uint32_t clog = 64 - __builtin_clzll(y - 1);   // ceil(log2 y)
  const uint32_t k = B - clog;
  const uint64_t j = x - ((1ull << B) - (1ull << (B - k)));
  const uint32_t cnt = B - 1 - k;
  fe acc = fe_one();
  for (uint32_t i = 0; i < cnt; ++i) {
    const fe p = pts[B - 1 - i];
    acc = fe_mul(acc, ((j >> i) & 1) ? p : fe_sub(fe_one(), p));
  }
  fe_store(out + x, acc);
}

__global__ void __launch_bounds__(kRedThreads)
sums_eq_kernel(const fe* __restrict__ m, uint64_t h, const fe* __restrict__ H,
               const fe* __restrict__ lo, uint32_t a, fe* __restrict__ partials) {
  fe e0 = fe_zero(), e1 = fe_zero();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;  // power of two >= 2^a
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t i = i0; i < h; i += stride) {
    const fe hv = fe_load(H + (i >> a));
    e0 = fe_add(e0, fe_mul(fe_load(m + i), hv));
    e1 = fe_add(e1, fe_mul(fe_load(m + i + h), hv));
  }
  const fe l = fe_load(lo + (i0 & ((1ull << a) - 1)));
  e0 = fe_mul(e0, l);
  e1 = fe_mul(e1, l);
  block_reduce2(e0, e1);
  if (threadIdx.x == 0) {
    fe_store(partials + 2 * blockIdx.x, e0);
    fe_store(partials + 2 * blockIdx.x + 1, e1);
  }
}

// fold m (size S) with r, then the eq-factored sums of the folded table
// (h' = S/4, next round's H table).  msrc: the table folded (== m in place; a
// separate source lets the first fold read the caller's evaluations without
// the build_tables_for_pcs clone).
__global__ void __launch_bounds__(kRedThreads)
fold_sums_eq_kernel(fe* m, uint64_t S, const fe* __restrict__ rp, const fe* __restrict__ H,
                    const fe* __restrict__ lo, uint32_t a, fe* __restrict__ partials,
                    const fe* msrc) {
  const fe r = fe_load(rp);
  const uint64_t h = S / 2, q = S / 4;
  fe e0 = fe_zero(), e1 = fe_zero();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t i = i0; i < q; i += stride) {
    const fe ma = fe_load(msrc + i), mb = fe_load(msrc + i + q);
    const fe mc = fe_load(msrc + i + h), md = fe_load(msrc + i + h + q);
    const fe hv = fe_load(H + (i >> a));
    const fe m0 = lerp(ma, mc, r), m1 = lerp(mb, md, r);
    fe_store(m + i, m0);
    fe_store(m + i + q, m1);
    e0 = fe_add(e0, fe_mul(m0, hv));
    e1 = fe_add(e1, fe_mul(m1, hv));
  }
  const fe l = fe_load(lo + (i0 & ((1ull << a) - 1)));
  e0 = fe_mul(e0, l);
  e1 = fe_mul(e1, l);
  block_reduce2(e0, e1);
  if (threadIdx.x == 0) {
    fe_store(partials + 2 * blockIdx.x, e0);
    fe_store(partials + 2 * blockIdx.x + 1, e1);
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

// thread count for the eq-factored kernels: a power of two >= 2^a (work >= 2^a)
#ifndef MLH_EQ_BLOCKS
#define MLH_EQ_BLOCKS 1024  // 2048 and 512 measured 1-2 % slower (tools/sumcheck_ab.py)
#endif
static inline unsigned eq_blocks(uint64_t work) {
  const unsigned b = red_blocks(work);
  return b < MLH_EQ_BLOCKS ? b : MLH_EQ_BLOCKS;
}

hipError_t launch_eq_suffix(const fe* pts, uint32_t B, fe* H, hipStream_t st) {
  const uint64_t total = (1ull << B) - 1;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(eq_suffix_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, pts,
                     B, H);
  return hipGetLastError();
}

hipError_t launch_sums_eq(const fe* m, uint64_t h, const fe* H, const fe* lo, uint32_t a,
                          fe* partials, hipStream_t st, uint32_t* nparts) {
  if (h < (1ull << a) || a < 8) return hipErrorInvalidValue;  // stride must be a multiple of 2^a
  const unsigned nb = eq_blocks(h);
  hipLaunchKernelGGL(sums_eq_kernel, dim3(nb), dim3(kRedThreads), 0, st, m, h, H, lo, a, partials);
  *nparts = nb;
  return hipGetLastError();
}

hipError_t launch_fold_sums_eq(fe* m, uint64_t S, const fe* r_dev, const fe* H, const fe* lo,
                               uint32_t a, fe* partials, hipStream_t st, uint32_t* nparts,
                               const fe* m_src) {
  if (S / 4 < (1ull << a) || a < 8) return hipErrorInvalidValue;
  const unsigned nb = eq_blocks(S / 4);
  hipLaunchKernelGGL(fold_sums_eq_kernel, dim3(nb), dim3(kRedThreads), 0, st, m, S, r_dev, H, lo, a,
                     partials, m_src ? m_src : m);
  *nparts = nb;
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

// sums = (s1, s2) = p(1), p(2); prev = claimed sum = p(0) + p(1).  Closed-form
// interpolation on x = 0,1,2 (polynomials.rs:51-87): e0 = prev - s1,
// c2 = (s2 - 2 s1 + e0) / 2, c1 = s1 - e0 - c2; absorb LE16(c1), LE16(c2)
// (sumcheck.rs:188-199), r = next_challenge(), prev = e0 + r (c1 + c2 r).
// pk != null: eq-factored round (partials hold (E0, E1); s1 = c p_k E1,
// s2 = c (3 p_k - 1)(2 E1 - E0)), and the scale advances to
// c <- c ((1 - r)(1 - p_k) + r p_k) once r is known.
__global__ void __launch_bounds__(kRedThreads)
sumcheck_round_kernel(const fe* __restrict__ partials, uint32_t nparts, fe* prev, DevSha* t,
                      fe* poly_out, fe* r_out, const fe* __restrict__ pk, fe* cdev) {
  __shared__ DevSha s;
  __shared__ uint32_t stage[8];
  // the transcript state (one word per lane) and lane 0's scalars are loaded
  // first, so their latency overlaps the partial-sum reduction
  if (threadIdx.x < sizeof(DevSha) / 4)
    reinterpret_cast<uint32_t*>(&s)[threadIdx.x] = reinterpret_cast<const uint32_t*>(t)[threadIdx.x];
  fe p = fe_zero(), c = fe_zero(), pv = fe_zero();
  if (threadIdx.x == 0) {
    p = fe_load(prev);
    if (pk) {
      c = fe_load(cdev);
      pv = fe_load(pk);
    }
  }
  // the round sums: reduce the per-workgroup partials (loads unrolled so a
  // lane's few loads are in flight together), then one lane runs the round
  fe s1 = fe_zero(), s2 = fe_zero();
#pragma unroll 4
  for (uint32_t i = threadIdx.x; i < nparts; i += kRedThreads) {
    s1 = fe_add(s1, fe_load(partials + 2 * i));
    s2 = fe_add(s2, fe_load(partials + 2 * i + 1));
  }
  block_reduce2(s1, s2);  // (its barriers also publish the staged state)
  if (threadIdx.x != 0) return;
  if (pk) {
    const fe E0 = s1, E1 = s2;
    const fe three_p_1 = fe_sub(fe_add(fe_dbl(pv), pv), fe_one());
    s1 = fe_mul(fe_mul(c, pv), E1);
    s2 = fe_mul(fe_mul(c, three_p_1), fe_sub(fe_dbl(E1), E0));
  }
  const fe e0 = fe_sub(p, s1);
  const fe c2 = fe_half(fe_add(fe_sub(s2, fe_add(s1, s1)), e0));
  const fe c1 = fe_sub(fe_sub(s1, e0), c2);
  fe_store(poly_out, c1);
  fe_store(poly_out + 1, c2);
  const uint32_t w[8] = {c1.w[0], c1.w[1], c1.w[2], c1.w[3], c2.w[0], c2.w[1], c2.w[2], c2.w[3]};
  dsha_absorb<8>(s, w, stage);  // LE16(c1) || LE16(c2)
  *t = s;
  const fe r = dsha_challenge(s);
  fe_store(r_out, r);
  fe_store(prev, fe_add(e0, fe_mul(r, fe_add(c1, fe_mul(c2, r)))));
  if (pk) {  // (1 - r)(1 - p) + r p = 1 - p - r + 2 r p
    const fe f = fe_add(fe_sub(fe_sub(fe_one(), pv), r), fe_dbl(fe_mul(r, pv)));
    fe_store(cdev, fe_mul(c, f));
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
                                 fe* poly_out, fe* r_out, hipStream_t st, const fe* pk, fe* c) {
  hipLaunchKernelGGL(sumcheck_round_kernel, dim3(1), dim3(kRedThreads), 0, st, partials, nparts,
                     prev, t, poly_out, r_out, pk, c);
  return hipGetLastError();
}

}  // namespace mlh
