// Radix-2 NTT over F_M for gfx950.
//
// Reference semantics: src/ntt/mod.rs:69-110 (Polynomial::ntt) and :132-173
// (LagrangePolynomial::intt): natural-order coefficients in, natural-order
// evaluations out, evals[i] = sum_j c_j * gen^(i*j); the inverse uses gen^-1
// and scales by n^-1.  The reference's bit-reverse + serial-twiddle DIT is an
// implementation detail; any exact algorithm gives identical field values.
//
// MI355X design (DESIGN.md "NTT"): N = R_1 * ... * R_P with R_p = 2^6..2^9.
// Pass p transforms digit p of the index in place (a generalised four-step):
//   * a workgroup owns C = 8 adjacent "columns" x R rows, so every global
//     access is 8 elements x 16 B = 128 contiguous bytes (dwordx4 per lane);
//   * each thread holds 8 elements in VGPRs and runs radix-2 DIT stages in
//     register phases of <= 3 stages; phases exchange through LDS
//     (C*R*16 B, 32 KiB at R = 256);
//   * the sub-transform input is read in bit-reversed row order straight from
//     HBM (the permutation is on the per-lane global address, free), so the
//     DIT output is in natural order;
//   * passes p < P multiply by the inter-pass twiddle w^(j_rest*k*S_p), read
//     from one table TA[k][j_rest] or, when that would exceed 2^22 entries,
//     TA[k][j_lo] * TB[k][j_hi] (TB expanded, staged through LDS: one j_hi
//     per tile);
//     for the inverse, pass 0's TA carries the n^-1 scale (no extra pass);
//   * stage twiddles: expanded tables (fe_mul_pre), the lane-dependent ones
//     read from a per-workgroup LDS copy;
//   * the last pass tiles 8 consecutive k_1 values so its scattered natural-
//     order stores are still 128-byte runs.
// Sizes N <= 2^10 use one LDS-resident workgroup (ntt_small).
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#include "bfly_asm.hpp"
#include "field.hpp"
#include "ntt.hpp"

namespace mlh {

constexpr int kCols = 8;  // columns per tile (8 x 16 B = 128 B runs)
constexpr int kLogCols = 3;
constexpr int kEPT = 8;   // elements per thread

__device__ __forceinline__ uint32_t bitrev(uint32_t x, int bits) {
  return __builtin_bitreverse32(x) >> (32 - bits);
}

struct PassGeom {
  uint32_t log_n;
  uint32_t nradix;      // P
  uint32_t p;           // 0-based pass index
  uint32_t logr[kMaxPasses];
  // every stride and count is a power of two: log2 of each, so that the
  // kernels index by shifts (no 64-bit multiplies or divisions per address)
  uint32_t lstride;     // W_p = 2^lstride (elements between consecutive rows of this digit)
  uint32_t loga;        // inter-pass twiddle split jrest = jh * 2^loga + jl
  uint32_t ltpv;        // tiles per vector (batched transforms: blockIdx.x = b*2^ltpv + tile)
  uint32_t lin_v;       // elements between consecutive input vectors
  uint32_t lout_v;      // elements between consecutive output vectors
  // TW 4 (the sharded NTT's fused last pass, mlh_sharded_ntt_fused_batch):
  // log2 P, this rank, log2 of the per-source chunk of the receive buffer
  uint32_t sh_p = 0, sh_rank = 0, sh_lchunk = 0;
};

// Last pass: natural output index is K = k_1 + R_1*rev(mid) + (N/R_P)*k_P,
// where mid holds digits 2..P-1 in storage order (digit 2 most significant)
// and rev() re-weights them in natural order (digit 2 least significant).
__device__ __forceinline__ uint64_t reverse_mid_digits(const PassGeom& g, uint64_t mid) {
  uint64_t rev = 0;
  // storage: lowest digit of mid is digit P-1 (0-based index nradix-2)
  for (int q = (int)g.nradix - 2; q >= 1; --q) {
    uint32_t shift = 0;  // natural weight of digit q: R_2*...*R_{q}
    for (int i = 1; i < q; ++i) shift += g.logr[i];
    rev += (mid & ((1ull << g.logr[q]) - 1)) << shift;
    mid >>= g.logr[q];
  }
  return rev;
}

// TW: 0 = two-table twiddle (TA * TB), 1 = one table (TA), 2 = none (last pass),
// 5 = pass 0's twiddle as a progression (ta = P[k0][j] = w_S^(k0 j), k0 < 64;
// tb = C[j] = w_S^(64 j), expanded): a thread's rows after its last register
// phase are k0 + 64 i, so w_S^(j (k0 + 64 i)) = P[k0][j] C[j]^i -- one product
// per step instead of TA * TB per element, no TB staging through LDS, 2 + 4
// twiddle loads per thread instead of 8 + TB's (LOGR 7 and 8);
// 3 = one table on pass 0 (same code as 1; its own kernel so that rocprof and
// the kernel timer tell the first pass from the middle ones), 4 = the last
// pass of a sharded transform (as 2, over this rank's share of the global
// tiles, reading the all-to-all's receive buffer: global storage index V lives
// at ((V mod P) << sh_lchunk) | ((V >> p) mod 2^sh_lchunk); writing the
// block-cyclic local output, K with bits [logr0 - p, logr0) removed)
// waves per SIMD the LDS tile allows (160 KiB/CU): caps VGPRs to match
#ifndef MLH_WPS8
#define MLH_WPS8 4  // R = 2^8: 32 KiB tile + 8 KiB twiddle copy -> 4 workgroups per CU
#endif
#ifndef MLH_LAST_STAGED
#define MLH_LAST_STAGED 1  // last pass loads through LDS (coalesced runs): pass -3..6 %
#endif
#ifndef MLH_LAST_DIRECT
// last pass (not sharded, full input): phase 1 runs with the lanes of a
// column on consecutive rows (coalesced 16 B x TPC runs straight from HBM),
// the first exchange switches to the 8-columns-per-row lane map the later
// phases and the natural-order stores use: no staged tile, one LDS round trip
// and one barrier fewer
#define MLH_LAST_DIRECT 1
#endif
#ifndef MLH_LDS_PAD
#define MLH_LDS_PAD 0  // extra dynamic LDS per pass workgroup (occupancy experiments)
#endif
#ifndef MLH_DIAG_TW  // diagnostics only (WRONG results): 1 = no TB, 2 = no TB and no TA loads
#define MLH_DIAG_TW 0
#endif
#ifndef MLH_LDS_TW
#define MLH_LDS_TW 1  // stage twiddles of the lane-dependent phases read from an LDS copy
#endif
constexpr int pass_waves_per_simd(int logr, int ept) {
  return ept == 16 ? 2 : (logr == 8 ? MLH_WPS8 : (logr == 9 ? 4 : (logr == 7 ? 4 : 2)));
}

// ZT: 0 = full input; 1 = input has N/2 elements, upper half implicit zeros
// (Reed-Solomon); 2 = as 1, with the N/2 inputs stored bit-reversed, i.e.
// coefficient j is in[bitrev_{log_n - 1}(j)] (the PCS's bit_reverse_permutation
// folded into pass 0's loads; pass 0 only, never the last pass).
// EPT: elements per thread (8: register phases of 3 stages; 16: of 4 stages,
// one LDS exchange fewer at R = 2^8, twice the VGPRs).
template <int LOGR, int TW, int ZT, int EPT = kEPT>
__global__ void __launch_bounds__(kCols * (1 << LOGR) / EPT,
                                  (TW == 2 || TW == 4) ? 1 : pass_waves_per_simd(LOGR, EPT))
ntt_pass_kernel(const fe* in, fe* out, const fe* __restrict__ tw,
                const fe* __restrict__ ta, const fe* __restrict__ tb, PassGeom g) {
  constexpr int R = 1 << LOGR;
  constexpr int LQ = EPT == 16 ? 4 : 3;  // stages per register phase
  constexpr int TPC = R / EPT;  // threads per column
  constexpr bool LAST = TW == 2 || TW == 4;
  constexpr bool SH = TW == 4;
  // sharded last pass: global storage index -> receive-buffer position
  auto phys = [&](uint64_t v) -> uint64_t {
    if constexpr (SH)
      return ((v & ((1ull << g.sh_p) - 1)) << g.sh_lchunk) |
             ((v >> g.sh_p) & ((1ull << g.sh_lchunk) - 1));
    else
      return v;
  };
  __shared__ fe lds[R * kCols];
#if MLH_LDS_TW
  // The expanded stage twiddles (R/2 entries x 4 limb-shifted multiples, 2R
  // fe).  Phase 1 indexes them by compile-time j (scalar loads); the later
  // phases by a lane-dependent j, where 4 global dwordx4 loads per twiddle per
  // lane were 3/4 of the pass's vector loads: those read this broadcast copy.
  // Written here; read only after the first exchange's barriers.
  __shared__ fe lds_tw[LOGR > LQ ? 2 * R : 1];
  if constexpr (LOGR > LQ) {
    constexpr int NT = kCols * R / EPT;  // threads per workgroup
    static_assert((2 * R) % NT == 0, "twiddle copy: whole rounds");
#pragma unroll
    for (int e = 0; e < 2 * R / NT; ++e)
      lds_tw[e * NT + threadIdx.x] = fe_load(tw + e * NT + threadIdx.x);
  }
#endif

  const int tid = threadIdx.x;
  // kDirect: phase 1 with column cA = tid / TPC and t = bitrev(tid mod TPC),
  // so lane l of a column loads row rev(8t + e) = rev3(e) TPC + l (consecutive
  // across lanes); the first exchange switches to c = tid mod 8, t = tid / 8
  constexpr bool kDirect = MLH_LAST_DIRECT && LAST && !SH && ZT == 0 && EPT == 8 && LOGR >= 6;
  constexpr int kLTPC = LOGR - 3;  // log2 threads per column (EPT = 8)
  const int cB = tid % kCols;
  int c = cB;
  int t = tid / kCols;
  if constexpr (kDirect) {
    c = tid >> kLTPC;
    t = (int)bitrev((uint32_t)tid & ((1u << kLTPC) - 1), kLTPC);
  }
  const uint64_t vec = (uint64_t)blockIdx.x >> g.ltpv;
  uint64_t tile = blockIdx.x & ((1ull << g.ltpv) - 1);
  if constexpr (SH) {  // this rank's tiles: first-digit columns whose top p bits are the rank
    const uint32_t lmid = g.log_n - g.logr[0] - LOGR;
    const uint32_t ld1 = g.logr[0] - kLogCols - g.sh_p;  // local first-digit column groups
    tile = ((((uint64_t)g.sh_rank << ld1) | (tile >> lmid)) << lmid) | (tile & ((1ull << lmid) - 1));
  }
  in += vec << g.lin_v;
  out += vec << g.lout_v;

  // ---- tile geometry -----------------------------------------------------
  uint64_t base, jrest = 0, k1 = 0, mid = 0;
  uint32_t rshift;  // log2 element stride between rows of this digit
  uint32_t cshift;  // log2 element stride between the 8 columns
  if (!LAST) {
    const uint32_t lw = g.lstride;  // W >= kCols
    const uint64_t hi = tile >> (lw - kLogCols), lo = tile & ((1ull << (lw - kLogCols)) - 1);
    base = (hi << (LOGR + lw)) + (lo << kLogCols);
    jrest = (lo << kLogCols) + cB;
    rshift = lw;
    cshift = 0;
  } else {
    const uint32_t lw1 = g.log_n - g.logr[0];  // W1 = N / R1
    const uint32_t lmid = lw1 - LOGR;          // MID = N / (R1 R_P)
    const uint64_t d1hi = tile >> lmid;
    mid = tile & ((1ull << lmid) - 1);
    base = (d1hi << (kLogCols + lw1)) + (mid << LOGR);
    k1 = (d1hi << kLogCols) + cB;
    rshift = 0;
    cshift = lw1;
  }
  const fe* src = in + base + ((uint64_t)c << cshift);  // phase 1's column
  fe* dst = out + base + ((uint64_t)cB << cshift);


  // ---- phase 1: load bit-reversed rows, stages 0..2 in registers ---------
  fe x[EPT];
#if MLH_LAST_STAGED
  // last pass: its rows are consecutive elements, so a lane's bit-reversed
  // rows scatter one wave's loads over 64 separate 16-B pieces.  Load the tile
  // as 8 x 128-B runs per wave instruction (8 consecutive rows x 8 columns)
  // into LDS, then read the bit-reversed rows from there.
  if constexpr (LAST && ZT == 0 && !kDirect) {
    constexpr int NT = kCols * R / EPT;
    // (the staged tile's columns are XOR-swizzled by row: lanes 0..7 write 8
    // consecutive rows of one column, which unswizzled sit 128 B apart on the
    // same LDS banks; the reads take one row's 8 columns, a permutation either way)
    // SH: a row's low p bits are its source rank, so the 8 lanes of a column
    // take rows P apart (consecutive in that source's chunk), and the swizzle
    // mixes in the bits above the rank bits.
    auto swz = [&](uint32_t row) -> uint32_t {
      if constexpr (SH) return (row ^ (row >> g.sh_p)) & (kCols - 1);
      else return row & (kCols - 1);
    };
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const uint32_t idx = (uint32_t)(e * NT + tid);
      const uint32_t l = idx & 63, grp = idx >> 6;
      uint32_t row = grp * 8 + (l & 7);
      if constexpr (SH) {
        const uint32_t lq = LOGR - g.sh_p - 3;  // groups of 8 rows per source rank: 2^lq
        const uint32_t src = grp >> lq, q0 = grp & ((1u << lq) - 1);
        row = ((((q0 << 3) + (l & 7)) << g.sh_p)) | src;
      }
      const uint32_t col = l >> 3;
      lds[row * kCols + (col ^ swz(row))] = fe_load(in + phys(base + ((uint64_t)col << cshift) + row));
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const uint32_t row = bitrev((uint32_t)(t * EPT + e), LOGR);
      x[e] = lds[row * kCols + (c ^ swz(row))];
    }
  } else
#endif
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const uint32_t row = bitrev((uint32_t)(t * EPT + e), LOGR);
    // rows >= R/2 are the implicit zero half; bitrev puts them exactly at odd e
    if (ZT != 0 && (e & 1)) {
      x[e] = fe_zero();
    } else if (ZT == 2) {
      // coefficient row*W + col, row < R/2, lives at bitrev(col)*(R/2) +
      // bitrev_{LOGR-1}(row) = bitrev(col)*(R/2) + (t*EPT + e)/2: each lane
      // reads 4 consecutive elements
      const uint32_t logw = g.log_n - LOGR;
      const uint64_t colr = __builtin_bitreverse64(jrest) >> (64 - logw);
      x[e] = fe_load(in + (colr << (LOGR - 1)) + ((uint32_t)(t * EPT + e) >> 1));
    } else if constexpr (SH) {
      x[e] = fe_load(in + phys(base + ((uint64_t)c << cshift) + ((uint64_t)row << rshift)));
    } else {
      x[e] = fe_load(src + ((uint64_t)row << rshift));
    }
  }

  // Generic register phase: stages [s0, s0+q) on groups of 2^q elements.
  // Butterflies run two at a time through the generated asm (bfly_asm.hpp) in
  // the relaxed representation; phase 1's twiddles are wave-uniform (SGPR
  // operands), the later phases' come from the LDS copy (VGPR operands).
  auto run_phase = [&](auto S0_, auto Q_) {
    constexpr int s0 = decltype(S0_)::value;
    constexpr int q = decltype(Q_)::value;
    constexpr int G = EPT >> q;
    constexpr int NB = EPT / 2;            // butterflies per stage
    constexpr int BPG = 1 << (q - 1);      // per group
#pragma unroll
    for (int s = s0; s < s0 + q; ++s) {
      const int d = 1 << (s - s0);  // element distance inside a group
      int be0[NB], be1[NB];
      uint32_t bj[NB];
      bool btriv[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int gi = b / BPG, m = b % BPG;
        const int i = ((m >> (s - s0)) << (s - s0 + 1)) | (m & (d - 1));
        be0[b] = gi * (1 << q) + i;
        be1[b] = be0[b] + d;
        const uint32_t gamma = (uint32_t)(t * G + gi);
        const uint32_t bpos = (gamma & ((1u << s0) - 1u)) | ((gamma >> s0) << (s0 + q));
        const uint32_t pos = bpos + ((uint32_t)i << s0);
        bj[b] = pos & ((1u << s) - 1u);
        // phase 1: j is a compile-time function of i (s == 0 or j == 0: w = 1)
        btriv[b] = s0 == 0 && (s == 0 || (i & ((1 << s) - 1)) == 0);
      }
      if (ZT != 0 && s0 == 0 && s == 0) {  // (u, 0) -> (u, u)
#pragma unroll
        for (int b = 0; b < NB; ++b) x[be1[b]] = x[be0[b]];
        continue;
      }
      uint64_t rare;
#pragma unroll
      for (int b = 0; b < NB; b += 2) {
        fe& u0 = x[be0[b]];
        fe& v0 = x[be1[b]];
        fe& u1 = x[be0[b + 1]];
        fe& v1 = x[be1[b + 1]];
        if (s0 == 0) {
          const fe* w0 = tw + 4 * (bj[b] << (LOGR - 1 - s));
          const fe* w1 = tw + 4 * (bj[b + 1] << (LOGR - 1 - s));
          if (!btriv[b] && !btriv[b + 1])
            bfly_mm_s(u0, v0, w0[0], w0[1], w0[2], w0[3], u1, v1, w1[0], w1[1], w1[2], w1[3], rare);
          else if (!btriv[b])
            bfly_mt_s(u0, v0, w0[0], w0[1], w0[2], w0[3], u1, v1, rare);
          else if (!btriv[b + 1])
            bfly_mt_s(u1, v1, w1[0], w1[1], w1[2], w1[3], u0, v0, rare);
          else
            bfly_tt_v(u0, v0, u1, v1, rare);
        } else {
#if MLH_LDS_TW
          const fe* w0 = lds_tw + 4 * (bj[b] << (LOGR - 1 - s));
          const fe* w1 = lds_tw + 4 * (bj[b + 1] << (LOGR - 1 - s));
#else
          const fe* w0 = tw + 4 * (bj[b] << (LOGR - 1 - s));
          const fe* w1 = tw + 4 * (bj[b + 1] << (LOGR - 1 - s));
#endif
          bfly_mm_v(u0, v0, w0[0], w0[1], w0[2], w0[3], u1, v1, w1[0], w1[1], w1[2], w1[3], rare);
        }
      }
    }
  };
  auto positions = [&](auto S0_, auto Q_, uint32_t (&pos)[EPT]) {
    constexpr int s0 = decltype(S0_)::value;
    constexpr int q = decltype(Q_)::value;
    constexpr int G = EPT >> q;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const uint32_t gamma = (uint32_t)(t * G + gi);
      const uint32_t bpos = (gamma & ((1u << s0) - 1u)) | ((gamma >> s0) << (s0 + q));
#pragma unroll
      for (int i = 0; i < (1 << q); ++i) pos[gi * (1 << q) + i] = bpos + ((uint32_t)i << s0);
    }
  };

  using I0 = std::integral_constant<int, 0>;
  constexpr int Q1 = LOGR < LQ ? LOGR : LQ;
  run_phase(I0{}, std::integral_constant<int, Q1>{});
  uint32_t pos[EPT];
  positions(I0{}, std::integral_constant<int, Q1>{}, pos);

  // ---- remaining phases through LDS -------------------------------------
  auto exchange_and_run = [&](auto S0_, auto Q_) {
    __syncthreads();  // previous phase's reads of lds are done
#pragma unroll
    for (int e = 0; e < EPT; ++e) fe_store(&lds[pos[e] * kCols + c], x[e]);
    __syncthreads();
    positions(S0_, Q_, pos);
#pragma unroll
    for (int e = 0; e < EPT; ++e) x[e] = fe_load(&lds[pos[e] * kCols + c]);
    run_phase(S0_, Q_);
  };
  // Two-table twiddle: TB[k][jh] has one jh for the tile's 8 columns (loga >=
  // 3), so the 8 lanes of a row read the same entry: one row per thread is
  // loaded and shared through the idle exchange tile.  TB is stored EXPANDED
  // (the 4 limb-shifted multiples, as the stage twiddles), so its product is
  // the 43-VALU expanded one (bfly_pp_v) instead of the 62-VALU full product.
  // MLH_P0_EARLY_TB: its loads (and the first TA pair's) are issued before the
  // last register phase, whose butterflies cover their latency; otherwise
  // just before the epilogue's barriers.
  constexpr int NTt = kCols * R / EPT;
  constexpr int kTbPerThread = TW == 0 ? R / NTt : 1;
  fe tbv[kTbPerThread][4];
  const uint64_t jl = jrest & ((1ull << g.loga) - 1);
  fe ta_c0, ta_c1;
  // MLH_TB_COALESCED: the 4R dwordx4 pieces of the tile's TB column are dealt
  // to the threads in order (piece i = part i mod 4 of row i / 4), so 4
  // adjacent lanes read one row's 64-B entry and a wave instruction touches 16
  // entries instead of 64 (each row's entry sits 2^ltcols x 64 B from the
  // next).  Round 5 counters (profiles/r05_ntt_pass_attrib.json): the
  // one-row-per-lane form made 256 of pass 0's 672 L1 requests per wave and
  // kept TA 62 % busy against 27 % in pass 1.  The LDS image is the same.
#ifndef MLH_TB_COALESCED
#define MLH_TB_COALESCED 1
#endif
  auto load_tb = [&]() {
    if constexpr (TW == 0 && MLH_DIAG_TW == 0) {
      const uint64_t jh = jrest >> g.loga;  // the same for the whole tile (loga >= 3)
      const uint32_t ltcols = g.lstride - g.loga;
#pragma unroll
      for (int e = 0; e < kTbPerThread; ++e) {
#if MLH_TB_COALESCED
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t i = (uint32_t)((e * 4 + k) * NTt + tid);
          tbv[e][k] = fe_load(tb + ((((uint64_t)(i >> 2) << ltcols) + jh) << 2) + (i & 3));
        }
#else
        const fe* q = tb + ((((uint64_t)(e * NTt + tid) << ltcols) + jh) << 2);
#pragma unroll
        for (int k = 0; k < 4; ++k) tbv[e][k] = fe_load(q + k);
#endif
      }
    }
  };
  // the first pair's inter-pass twiddles (the asm products below keep later
  // loads from being hoisted, so each pair's are issued one pair ahead)
  auto load_ta0 = [&](const uint32_t (&pf)[EPT]) {
    if constexpr (TW == 5) {
      (void)pf;
    } else if constexpr (!LAST && MLH_DIAG_TW == 2) {
      ta_c0 = fe{{(uint32_t)jl | 1u, 7u, 9u, 3u}};
      ta_c1 = fe{{(uint32_t)pf[1] | 1u, 5u, 9u, 3u}};
    } else if constexpr (!LAST) {
      ta_c0 = fe_load(ta + ((uint64_t)pf[0] << g.loga) + jl);
      ta_c1 = fe_load(ta + ((uint64_t)pf[1] << g.loga) + jl);
    }
  };
#ifndef MLH_P0_EARLY_TB
#define MLH_P0_EARLY_TB 0
#endif

  constexpr bool kEarly = MLH_P0_EARLY_TB && TW == 0 && LOGR > 2 * LQ;
  if constexpr (LOGR > LQ) {
    constexpr int Q2 = (LOGR - LQ) < LQ ? (LOGR - LQ) : LQ;
    if constexpr (kDirect) {
      // written in the phase-1 map, read in the 8-columns-per-row map; the
      // column slot is XORed with the row's top 3 bits, so the 8 lanes of a
      // write group (consecutive l: distinct top bits of t) and of a read
      // group (8 columns of one row) each hit 8 distinct 16-B slots
      auto slot = [&](uint32_t row, int col) -> uint32_t {
        return row * kCols + ((uint32_t)col ^ ((row >> (LOGR - 3)) & (kCols - 1)));
      };
      __syncthreads();  // (the twiddle copy's writes, before the phase-2 reads of lds_tw)
#pragma unroll
      for (int e = 0; e < EPT; ++e) fe_store(&lds[slot(pos[e], c)], x[e]);
      __syncthreads();
      c = cB;
      t = tid / kCols;
      positions(std::integral_constant<int, LQ>{}, std::integral_constant<int, Q2>{}, pos);
#pragma unroll
      for (int e = 0; e < EPT; ++e) x[e] = fe_load(&lds[slot(pos[e], c)]);
      run_phase(std::integral_constant<int, LQ>{}, std::integral_constant<int, Q2>{});
    } else {
      exchange_and_run(std::integral_constant<int, LQ>{}, std::integral_constant<int, Q2>{});
    }
    if constexpr (LOGR > 2 * LQ) {
      constexpr int Q3 = LOGR - 2 * LQ;
      static_assert(Q3 <= LQ, "LOGR <= 3 * LQ");
      if constexpr (kEarly) {
        uint32_t pf[EPT];
        positions(std::integral_constant<int, 2 * LQ>{}, std::integral_constant<int, Q3>{}, pf);
        load_tb();
        if (MLH_P0_EARLY_TB == 1) load_ta0(pf);  // 2: TB only
      }
      exchange_and_run(std::integral_constant<int, 2 * LQ>{}, std::integral_constant<int, Q3>{});
    }
  }

  // ---- epilogue: inter-pass twiddle, store --------------------------------
  if constexpr (!kEarly) {
    load_ta0(pos);
    load_tb();
  } else if (MLH_P0_EARLY_TB == 2) {
    load_ta0(pos);
  }
  if constexpr (TW == 0) {
    static_assert(4 * R <= R * kCols, "the expanded TB column fits the exchange tile");
    constexpr int NT = NTt;
    __syncthreads();  // every lane's reads of the exchange tile are done
#pragma unroll
    for (int e = 0; e < kTbPerThread; ++e)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        lds[MLH_TB_COALESCED ? (e * 4 + k) * NT + tid : 4 * (e * NT + tid) + k] = tbv[e][k];
    __syncthreads();
  }
  uint64_t kbase = 0;
  uint32_t kshift = 0;
  if (LAST) {
    kbase = k1 + (reverse_mid_digits(g, mid) << g.logr[0]);
    kshift = g.log_n - LOGR;
  }
  if constexpr (TW == 5) {
    constexpr int Q3 = LOGR - 2 * LQ, NI = 1 << Q3, G = EPT / NI;
    static_assert(LOGR > 2 * LQ && G % 2 == 0, "progression twiddle: groups in pairs");
    // (loaded here: issued before the last register phase instead -- P alone,
    // or P and C with 6 spilled registers -- measured no faster / 8 % slower)
    fe tv[G];  // P[k0][j] of each group (k0 = pos[g NI]: the group's first row)
#pragma unroll
    for (int gq = 0; gq < G; ++gq) tv[gq] = fe_load(ta + ((uint64_t)pos[gq * NI] << g.lstride) + jrest);
    const fe* cp = tb + 4 * jrest;
    const fe c0 = fe_load(cp), c1 = fe_load(cp + 1), c2 = fe_load(cp + 2), c3 = fe_load(cp + 3);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      uint64_t rare;
#pragma unroll
      for (int gq = 0; gq < G; gq += 2) {
        const int e0 = gq * NI + i, e1 = (gq + 1) * NI + i;
        bfly_ff_v(x[e0], tv[gq], x[e1], tv[gq + 1], rare);
        fe_store(dst + ((uint64_t)pos[e0] << rshift), x[e0]);
        fe_store(dst + ((uint64_t)pos[e1] << rshift), x[e1]);
      }
      if (i + 1 < NI) {
#pragma unroll
        for (int gq = 0; gq < G; gq += 2) bfly_pp_v(tv[gq], c0, c1, c2, c3, tv[gq + 1], c0, c1, c2, c3, rare);
      }
    }
  } else if constexpr (!LAST) {
    // w_S^(jrest k) = TA[k][jl] * TB[k][jh]: the 8 columns of a tile are 8
    // consecutive jl, so a wave's lanes read 8 runs of 128 B per table.  The
    // products run two elements per generated asm statement (relaxed result;
    // bfly_asm.hpp), and the next pass takes relaxed input.
#pragma unroll
    for (int e = 0; e < EPT; e += 2) {
      uint64_t rare;
      const fe a0 = ta_c0, a1 = ta_c1;
      if (e + 2 < EPT && MLH_DIAG_TW < 2) {  // the next pair's, in flight during this pair's products
        ta_c0 = fe_load(ta + ((uint64_t)pos[e + 2] << g.loga) + jl);
        ta_c1 = fe_load(ta + ((uint64_t)pos[e + 3] << g.loga) + jl);
      }
      bfly_ff_v(x[e], a0, x[e + 1], a1, rare);
      if constexpr (TW == 0 && MLH_DIAG_TW == 0) {
        const fe* b0 = lds + 4 * pos[e];
        const fe* b1 = lds + 4 * pos[e + 1];
        bfly_pp_v(x[e], b0[0], b0[1], b0[2], b0[3], x[e + 1], b1[0], b1[1], b1[2], b1[3], rare);
      }
      fe_store(dst + ((uint64_t)pos[e] << rshift), x[e]);
      fe_store(dst + ((uint64_t)pos[e + 1] << rshift), x[e + 1]);
    }
  } else {
    // canonical output, four elements per asm statement
    static_assert(EPT % 4 == 0, "canonicalisation in fours");
#pragma unroll
    for (int e = 0; e < EPT; e += 4) bfly_cccc_v(x[e], x[e + 1], x[e + 2], x[e + 3]);
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      uint64_t K = kbase + ((uint64_t)pos[e] << kshift);
      if constexpr (SH) {  // drop the rank bits [logr0 - p, logr0) of K
        const uint32_t lo = g.logr[0] - g.sh_p;
        K = ((K >> g.logr[0]) << lo) | (K & ((1ull << lo) - 1));
      }
      fe_store(out + K, x[e]);
    }
  }
  (void)TPC;
}

// Single-workgroup NTT for N <= 2^10: LDS-resident radix-2 DIT.
__global__ void __launch_bounds__(512)
ntt_small_kernel(const fe* __restrict__ in, fe* __restrict__ out, const fe* __restrict__ tw,
                 uint32_t log_n, uint32_t in_len, fe scale, int apply_scale, int brev_in) {
  __shared__ fe lds[1024];
  const uint32_t N = 1u << log_n;
  in += (uint64_t)blockIdx.x * in_len;
  out += (uint64_t)blockIdx.x * N;
  for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
    const uint32_t src = bitrev(i, (int)log_n);
    // brev_in: coefficient src is stored at bitrev_{log2 in_len}(src) (ZT == 2)
    const uint32_t at = (brev_in && in_len > 1) ? bitrev(src, 31 - __builtin_clz(in_len)) : src;
    lds[i] = src < in_len ? fe_load(in + at) : fe_zero();
  }
  __syncthreads();
  for (uint32_t s = 0; s < log_n; ++s) {
    const uint32_t h = 1u << s;
    for (uint32_t b = threadIdx.x; b < N / 2; b += blockDim.x) {
      const uint32_t j = b & (h - 1);
      const uint32_t p0 = j + ((b >> s) << (s + 1));
      const fe u = lds[p0];
      fe v = lds[p0 + h];
      if (j) v = fe_mul(v, tw[j << (log_n - 1 - s)]);
      lds[p0] = fe_add(u, v);
      lds[p0 + h] = fe_sub(u, v);
    }
    __syncthreads();
  }
  for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
    fe v = lds[i];
    if (apply_scale) v = fe_mul(v, scale);
    fe_store(out + i, v);
  }
}

// table[t] = base^t * scale, t < count (twiddle tables; one-time per context).
// expand: entry t is the 4 limb-shifted multiples v * 2^(32k) (fe_mul_pre).
__global__ void pow_table_kernel(fe* __restrict__ out, fe base, fe scale, uint64_t count,
                                 int expand) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= count) return;
  fe v = fe_pow(base, t);
  v = fe_mul(v, scale);
  if (!expand) {
    fe_store(out + t, v);
    return;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    fe_store(out + 4 * t + k, v);
    v = fe_mul(v, fe{{0u, 1u, 0u, 0u}});  // * 2^32
  }
}

// 2D table out[k * cols + j] = base^(k * j * mult) * scale (inter-pass twiddles).
// expand: entry t is the 4 limb-shifted multiples (fe_mul_pre), as pow_table.
__global__ void pow_table2d_kernel(fe* __restrict__ out, fe base, fe scale, uint64_t rows,
                                   uint64_t cols, uint64_t mult, int expand) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * cols) return;
  const uint64_t k = t / cols, j = t % cols;
  fe v = fe_mul(fe_pow(base, k * j * mult), scale);
  if (!expand) {
    fe_store(out + t, v);
    return;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    fe_store(out + 4 * t + q, v);
    v = fe_mul(v, fe{{0u, 1u, 0u, 0u}});  // * 2^32
  }
}

hipError_t launch_pow_table2d(fe* out, fe base, fe scale, uint64_t rows, uint64_t cols,
                              uint64_t mult, hipStream_t st, bool expand) {
  const uint64_t n = rows * cols;
  hipLaunchKernelGGL(pow_table2d_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out,
                     base, scale, rows, cols, mult, expand ? 1 : 0);
  return hipGetLastError();
}

// gen_pows[i] = g^i for i < count (NttField::pow_2_generator_powers,
// src/ntt/mod.rs:18-28): block-base x in-block power, no serial chain.
__global__ void pow_series_kernel(fe* __restrict__ out, const fe* __restrict__ tlo,
                                  const fe* __restrict__ thi, uint64_t count) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= count) return;
  fe_store(out + t, fe_mul(tlo[t & 4095], thi[t >> 12]));
}

// mlh_gen_pows_verify: gp[t] (t < count, table index base + t) against
// g^(base + t); the smallest mismatching index to *bad (initialised ~0).
__global__ void pow_series_check_kernel(const fe* __restrict__ gp, uint64_t base, uint64_t count,
                                        const fe* __restrict__ tlo, const fe* __restrict__ thi,
                                        unsigned long long* bad) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= count) return;
  const uint64_t i = base + t;
  const fe want = fe_mul(tlo[i & 4095], thi[i >> 12]);
  const fe got = fe_load(gp + t);
  if ((want.w[0] ^ got.w[0]) | (want.w[1] ^ got.w[1]) | (want.w[2] ^ got.w[2]) | (want.w[3] ^ got.w[3]))
    atomicMin(bad, (unsigned long long)i);
}

// ---- general-generator network --------------------------------------------
// Polynomial::ntt / LagrangePolynomial::intt (src/ntt/mod.rs:69-110, :132-173)
// for a generator whose order is not exactly N.  The reference's loop --
// bit-reverse, then stage len = 4..N with butterflies u +- v * g_len^j,
// g_len = gen^(N/len) -- is then a well-defined linear map but no DFT: with
// gen^(N/2) != -1, "u - w v" is not "u + w' v" for any power w', so the
// four-step passes above (which rely on that) cannot reproduce it.  These
// kernels run the same butterfly network stage by stage: the first kNetLB
// stages per LDS-resident block of 2^kNetLB positions, the rest up to 4 per
// launch in registers.  w^t (t < N/2) = tlo[t mod 2^12] * thi[t >> 12] (two
// small tables instead of one of N/2 entries, which would be 32 GiB at 2^32);
// stage s (len = 2^(s+1)) uses w^(j << (log_n - 1 - s)) = g_len^j, the
// reference's gen_pows[j] (exact: the field is exact, however the power is
// formed).  Correctness path, not tuned.
constexpr uint32_t kNetLB = 11;  // 2^11 entries = 32 KiB of LDS

__device__ __forceinline__ fe net_tw(const fe* __restrict__ tlo, const fe* __restrict__ thi,
                                     uint64_t t) {
  const uint64_t lo = t & 4095, hi = t >> 12;
  if (!hi) return fe_load(tlo + lo);
  if (!lo) return fe_load(thi + hi);
  return fe_mul(fe_load(tlo + lo), fe_load(thi + hi));
}

__device__ __forceinline__ uint64_t bitrev64(uint64_t x, uint32_t bits) {
  return bits ? __builtin_bitreverse64(x) >> (64 - bits) : 0;
}

// zero_top: 0 = N inputs; 1 = N/2 inputs, the rest zero (reed_solomon's
// resize, fri/mod.rs:19-28); 2 = as 1, coefficient c stored at
// in[bitrev_{log_n - 1}(c)].
__global__ void __launch_bounds__(1024)
ntt_net_block_kernel(const fe* __restrict__ in, fe* __restrict__ out, const fe* __restrict__ tlo,
                     const fe* __restrict__ thi, uint32_t log_n, uint32_t lb, int zero_top, fe scale, int apply_scale) {
  __shared__ fe lds[1u << kNetLB];
  const uint32_t B = 1u << lb;
  const uint64_t N = 1ull << log_n, base = (uint64_t)blockIdx.x << lb;
  for (uint32_t i = threadIdx.x; i < B; i += blockDim.x) {
    const uint64_t src = bitrev64(base + i, log_n);  // bit_reverse_permutation (ntt/mod.rs:113-123)
    fe v;
    if (zero_top == 0) v = fe_load(in + src);
    else if (src >= N / 2) v = fe_zero();
    else v = fe_load(in + (zero_top == 2 ? bitrev64(src, log_n - 1) : src));
    lds[i] = v;
  }
  __syncthreads();
  for (uint32_t s = 0; s < lb; ++s) {
    const uint32_t h = 1u << s;
    for (uint32_t b = threadIdx.x; b < B / 2; b += blockDim.x) {
      const uint32_t j = b & (h - 1);
      const uint32_t p0 = j + ((b >> s) << (s + 1));
      const fe u = lds[p0];
      fe v = lds[p0 + h];
      if (j) v = fe_mul(v, net_tw(tlo, thi, (uint64_t)j << (log_n - 1 - s)));  // gen_pows[0] = 1
      lds[p0] = fe_add(u, v);
      lds[p0 + h] = fe_sub(u, v);
    }
    __syncthreads();
  }
  for (uint32_t i = threadIdx.x; i < B; i += blockDim.x) {
    fe v = lds[i];
    if (apply_scale) v = fe_mul(v, scale);
    fe_store(out + base + i, v);
  }
}

// Stages s0 .. s0 + Q - 1 (s0 >= kNetLB): each thread owns the 2^Q positions
// base + m 2^s0 (m < 2^Q) that these stages couple; consecutive threads take
// consecutive low bits, so every load and store is a contiguous wave run.
// Runs in place (in == out) or out of place.
template <int Q>
__global__ void __launch_bounds__(256)
ntt_net_stage_kernel(const fe* in, fe* out, const fe* __restrict__ tlo, const fe* __restrict__ thi,
                     uint32_t log_n,
                     uint32_t s0, fe scale, int apply_scale) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (1ull << (log_n - Q))) return;
  const uint64_t low = g & ((1ull << s0) - 1);
  const uint64_t base = ((g >> s0) << (s0 + Q)) | low;
  fe x[1 << Q];
#pragma unroll
  for (int m = 0; m < (1 << Q); ++m) x[m] = fe_load(in + base + ((uint64_t)m << s0));
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const uint32_t s = s0 + q;
    const int d = 1 << q;
#pragma unroll
    for (int b = 0; b < (1 << (Q - 1)); ++b) {
      const int m = ((b >> q) << (q + 1)) | (b & (d - 1));  // pairs (m, m + d)
      const uint64_t j = (base + ((uint64_t)m << s0)) & ((1ull << s) - 1);
      const fe v = j ? fe_mul(x[m + d], net_tw(tlo, thi, j << (log_n - 1 - s))) : x[m + d];
      const fe u = x[m];
      x[m] = fe_add(u, v);
      x[m + d] = fe_sub(u, v);
    }
  }
#pragma unroll
  for (int m = 0; m < (1 << Q); ++m) {
    fe v = x[m];
    if (apply_scale) v = fe_mul(v, scale);
    fe_store(out + base + ((uint64_t)m << s0), v);
  }
}

hipError_t launch_ntt_network(const fe* in, fe* out, fe* scratch, const fe* tlo, const fe* thi,
                              uint32_t log_n,
                              int zero_top, fe scale, bool apply_scale, hipStream_t st) {
  if (log_n < 1 || log_n > 40 || (zero_top && in == out)) return hipErrorInvalidValue;
  const uint32_t lb = log_n < kNetLB ? log_n : kNetLB;
  const uint64_t blocks = 1ull << (log_n - lb);
  // the block pass gathers bit-reversed positions from all of `in`: out of
  // place whenever it has more than one block
  fe* first = (in == out && blocks > 1) ? scratch : out;
  const bool only = lb == log_n;
  const uint32_t threads = lb >= 11 ? 1024 : (1u << lb) / 2 < 64 ? 64 : (1u << lb) / 2;
  hipLaunchKernelGGL(ntt_net_block_kernel, dim3((unsigned)blocks), dim3(threads), 0, st, in, first,
                     tlo, thi, log_n, lb, zero_top, scale, (only && apply_scale) ? 1 : 0);
  hipError_t e = hipGetLastError();
  for (uint32_t s0 = lb; e == hipSuccess && s0 < log_n;) {
    const uint32_t q = log_n - s0 < 4 ? log_n - s0 : 4;
    const bool last = s0 + q == log_n;
    fe* dst = last ? out : first;
    const int sc = (last && apply_scale) ? 1 : 0;
    const dim3 grid((unsigned)(((1ull << (log_n - q)) + 255) / 256)), blk(256);
    switch (q) {
      case 1: hipLaunchKernelGGL(ntt_net_stage_kernel<1>, grid, blk, 0, st, first, dst, tlo, thi, log_n, s0, scale, sc); break;
      case 2: hipLaunchKernelGGL(ntt_net_stage_kernel<2>, grid, blk, 0, st, first, dst, tlo, thi, log_n, s0, scale, sc); break;
      case 3: hipLaunchKernelGGL(ntt_net_stage_kernel<3>, grid, blk, 0, st, first, dst, tlo, thi, log_n, s0, scale, sc); break;
      default: hipLaunchKernelGGL(ntt_net_stage_kernel<4>, grid, blk, 0, st, first, dst, tlo, thi, log_n, s0, scale, sc); break;
    }
    e = hipGetLastError();
    s0 += q;
  }
  return e;
}

// ---- host-side launchers ---------------------------------------------------

template <int LOGR, int EPT>
static hipError_t launch_pass_ept(bool last, int zero_top, const fe* in, fe* out, const fe* tw,
                                  const fe* ta, const fe* tb, const PassGeom& g, uint64_t tiles,
                                  hipStream_t st, bool geo = false) {
  constexpr int threads = kCols * (1 << LOGR) / EPT;
  const dim3 grid((unsigned)tiles), blk(threads);
#define MLH_PASS(TWV, ZTV)                                                                  \
  hipLaunchKernelGGL((ntt_pass_kernel<LOGR, TWV, ZTV, EPT>), grid, blk, MLH_LDS_PAD, st, in, out, \
                     tw, ta, tb, g)
  if (last) {
    if (zero_top) return hipErrorInvalidValue;  // pass 0 is never the last pass here
    MLH_PASS(2, 0);
  } else if (geo) {  // TW 5 (pass 0, LOGR 7 / 8; ta = P, tb = C)
    if constexpr ((LOGR == 7 || LOGR == 8) && EPT == 8) {
      if (zero_top == 2) MLH_PASS(5, 2);
      else if (zero_top == 1) MLH_PASS(5, 1);
      else MLH_PASS(5, 0);
    } else {
      return hipErrorInvalidValue;
    }
  } else if (!tb && g.p == 0) {  // TW 3: as 1, a distinct kernel for the first pass
    if (zero_top == 2) MLH_PASS(3, 2);
    else if (zero_top == 1) MLH_PASS(3, 1);
    else MLH_PASS(3, 0);
  } else if (!tb) {
    if (zero_top) return hipErrorInvalidValue;  // only pass 0 has an implicit zero half
    MLH_PASS(1, 0);
  } else {
    if (zero_top == 2) MLH_PASS(0, 2);
    else if (zero_top == 1) MLH_PASS(0, 1);
    else MLH_PASS(0, 0);
  }
#undef MLH_PASS
  return hipGetLastError();
}

// EPT = 8 throughout: 16 elements per thread (4-stage register phases, one
// LDS exchange fewer at R = 2^8) measured 23 % slower for a 2^24 NTT -- 190
// VGPRs leave 2 waves per SIMD against 5, and the extra ILP does not cover it.
template <int LOGR>
static hipError_t launch_pass(bool last, int zero_top, const fe* in, fe* out, const fe* tw,
                              const fe* ta, const fe* tb, const PassGeom& g, uint64_t tiles,
                              hipStream_t st, bool geo = false) {
  return launch_pass_ept<LOGR, kEPT>(last, zero_top, in, out, tw, ta, tb, g, tiles, st, geo);
}

void ntt_plan_radices(uint32_t log_n, uint32_t* nradix, uint32_t* logr, const uint32_t* forced,
                      uint32_t nforced) {
  // A forced plan (mlh_set_ntt_plan: digits 4..9 summing to log_n) lets the
  // tests check every pass shape at oracle-sized N; otherwise the default.
  if (forced && nforced >= 2 && nforced <= (uint32_t)kMaxPasses) {
    uint32_t sum = 0;
    bool ok = true;
    for (uint32_t i = 0; i < nforced; ++i) {
      ok = ok && forced[i] >= 4 && forced[i] <= 9;
      sum += forced[i];
    }
    if (ok && sum == log_n) {
      *nradix = nforced;
      for (uint32_t i = 0; i < nforced; ++i) logr[i] = forced[i];
      return;
    }
  }
  const uint32_t P = (log_n + 8) / 9;  // ceil(log_n / 9)
  *nradix = P;
  uint32_t rem = log_n;
  for (uint32_t p = 0; p < P; ++p) {
    const uint32_t left = P - p;
    const uint32_t r = (rem + left - 1) / left;  // larger digits first
    logr[p] = r;
    rem -= r;
  }
}

hipError_t launch_ntt_small(const fe* in, fe* out, const fe* tw, uint32_t log_n, uint64_t in_len,
                            fe scale, bool apply_scale, hipStream_t st, uint64_t batch,
                            bool brev_in) {
  const uint32_t N = 1u << log_n;
  const uint32_t threads = N / 2 < 64 ? 64 : (N / 2 > 512 ? 512 : N / 2);
  hipLaunchKernelGGL(ntt_small_kernel, dim3((unsigned)batch), dim3(threads), 0, st, in, out, tw, log_n,
                     (uint32_t)in_len, scale, apply_scale ? 1 : 0, brev_in ? 1 : 0);
  return hipGetLastError();
}

void ntt_pass_label(const NttTables& tb, uint32_t p, int zero_top, char* buf, size_t n) {
  const bool last = p + 1 == tb.nradix;
  const int tw = last ? 2 : (tb.gp[p] ? 5 : (tb.tb[p] ? 0 : (p == 0 ? 3 : 1)));
  snprintf(buf, n, "ntt_pass<%u,%d,%d>", tb.logr[p], tw, p == 0 ? zero_top : 0);
}

hipError_t launch_ntt_passes(const fe* in, fe* out, fe* scratch, const NttTables& tb,
                             uint32_t log_n, int zero_top, hipStream_t st, hipEvent_t* ev,
                             uint64_t batch) {
  PassGeom g;
  g.log_n = log_n;
  g.nradix = tb.nradix;
  for (uint32_t p = 0; p < tb.nradix; ++p) g.logr[p] = tb.logr[p];
  const uint64_t N = 1ull << log_n;
  uint64_t W = N;
  for (uint32_t p = 0; p < tb.nradix; ++p) {
    const uint32_t lr = tb.logr[p];
    W >>= lr;
    g.p = p;
    g.lstride = (uint32_t)__builtin_ctzll(W);
    g.loga = tb.loga[p];
    const bool last = (p + 1 == tb.nradix);
    g.ltpv = log_n - kLogCols - lr;
    const uint64_t tiles = (N >> (kLogCols + lr)) * batch;
    g.lin_v = (p == 0 && zero_top) ? log_n - 1 : log_n;
    g.lout_v = log_n;
    // pass 0: in -> scratch; middle passes in place on scratch; the last pass
    // (a digit-reversal permutation of its tiles) scratch -> out.  The last
    // pass can never run in place: a block would overwrite tiles that other,
    // not yet resident, blocks still have to read.
    const fe* src = (p == 0) ? in : scratch;
    fe* dst = last ? out : scratch;
    const int zt = p == 0 ? zero_top : 0;
    if (ev) (void)hipEventRecord(ev[p], st);
    hipError_t e;
    const bool geo = tb.gp[p] != nullptr;  // TW 5: the progression tables instead of TA, TB
    const fe* ta = geo ? tb.gp[p] : tb.ta[p];
    const fe* tbb = geo ? tb.gc[p] : tb.tb[p];
    switch (lr) {
      case 4: e = launch_pass<4>(last, zt, src, dst, tb.tw[p], ta, tbb, g, tiles, st, geo); break;
      case 5: e = launch_pass<5>(last, zt, src, dst, tb.tw[p], ta, tbb, g, tiles, st, geo); break;
      case 6: e = launch_pass<6>(last, zt, src, dst, tb.tw[p], ta, tbb, g, tiles, st, geo); break;
      case 7: e = launch_pass<7>(last, zt, src, dst, tb.tw[p], ta, tbb, g, tiles, st, geo); break;
      case 8: e = launch_pass<8>(last, zt, src, dst, tb.tw[p], ta, tbb, g, tiles, st, geo); break;
      case 9: e = launch_pass<9>(last, zt, src, dst, tb.tw[p], ta, tbb, g, tiles, st, geo); break;
      default: return hipErrorInvalidValue;
    }
    if (e != hipSuccess) return e;
    if (tb.debug_sync) {
      e = hipStreamSynchronize(st);
      if (e != hipSuccess) return e;
    }
  }
  if (ev) (void)hipEventRecord(ev[tb.nradix], st);
  return hipSuccess;
}

// out[k][j] = in[k][j] * rowbase^k (k < rows, j < 2^lcols): an inter-pass
// twiddle table with a per-row factor (the sharded fused NTT's rank twist)
__global__ void __launch_bounds__(256)
scale_rows_kernel(const fe* __restrict__ in, fe* __restrict__ out, uint64_t n, uint32_t lcols, fe rowbase) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t k = i >> lcols;
  fe f = fe_one(), b = rowbase;
  while (k) {
    if (k & 1) f = fe_mul(f, b);
    b = fe_mul(b, b);
    k >>= 1;
  }
  fe_store(out + i, fe_mul(fe_load(in + i), f));
}

hipError_t launch_scale_rows(const fe* in, fe* out, uint64_t rows, uint32_t lcols, fe rowbase,
                             hipStream_t st) {
  const uint64_t n = rows << lcols;
  hipLaunchKernelGGL(scale_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, out, n,
                     lcols, rowbase);
  return hipGetLastError();
}

hipError_t launch_ntt_passes_pre(const fe* in, fe* out, const NttTables& tb, uint32_t log_n,
                                 uint32_t npasses, hipStream_t st) {
  if (npasses == 0 || npasses >= tb.nradix) return hipErrorInvalidValue;
  PassGeom g;
  g.log_n = log_n;
  g.nradix = tb.nradix;
  for (uint32_t p = 0; p < tb.nradix; ++p) g.logr[p] = tb.logr[p];
  const uint64_t N = 1ull << log_n;
  uint64_t W = N;
  for (uint32_t p = 0; p < npasses; ++p) {
    const uint32_t lr = tb.logr[p];
    W >>= lr;
    g.p = p;
    g.lstride = (uint32_t)__builtin_ctzll(W);
    g.loga = tb.loga[p];
    g.ltpv = log_n - kLogCols - lr;
    g.lin_v = g.lout_v = log_n;
    const uint64_t tiles = N >> (kLogCols + lr);
    const fe* src = p == 0 ? in : out;  // pass 0: in -> out; then in place on out
    hipError_t e;
    switch (lr) {
      case 4: e = launch_pass<4>(false, 0, src, out, tb.tw[p], tb.ta[p], tb.tb[p], g, tiles, st); break;
      case 5: e = launch_pass<5>(false, 0, src, out, tb.tw[p], tb.ta[p], tb.tb[p], g, tiles, st); break;
      case 6: e = launch_pass<6>(false, 0, src, out, tb.tw[p], tb.ta[p], tb.tb[p], g, tiles, st); break;
      case 7: e = launch_pass<7>(false, 0, src, out, tb.tw[p], tb.ta[p], tb.tb[p], g, tiles, st); break;
      case 8: e = launch_pass<8>(false, 0, src, out, tb.tw[p], tb.ta[p], tb.tb[p], g, tiles, st); break;
      case 9: e = launch_pass<9>(false, 0, src, out, tb.tw[p], tb.ta[p], tb.tb[p], g, tiles, st); break;
      default: return hipErrorInvalidValue;
    }
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_ntt_shard_last(const fe* recv, fe* out, const fe* tw, const uint32_t* logr,
                                 uint32_t nradix, uint32_t log_n, uint32_t log_p, uint32_t rank,
                                 hipStream_t st) {
  if (nradix < 2 || nradix > (uint32_t)kMaxPasses) return hipErrorInvalidValue;
  const uint32_t lr = logr[nradix - 1];
  if (lr < log_p + 3 || logr[0] < kLogCols + log_p) return hipErrorInvalidValue;
  PassGeom g;
  g.log_n = log_n;
  g.nradix = nradix;
  for (uint32_t p = 0; p < nradix; ++p) g.logr[p] = logr[p];
  g.p = nradix - 1;
  g.lstride = 0;
  g.loga = 0;
  g.ltpv = log_n - kLogCols - lr - log_p;  // this rank's tiles
  g.lin_v = g.lout_v = log_n;
  g.sh_p = log_p;
  g.sh_rank = rank;
  g.sh_lchunk = log_n - 2 * log_p;
  const dim3 grid((unsigned)(1ull << g.ltpv));
#define MLH_SHL(LR)                                                                                 \
  hipLaunchKernelGGL((ntt_pass_kernel<LR, 4, 0, kEPT>), grid, dim3(kCols * (1 << LR) / kEPT), MLH_LDS_PAD, \
                     st, recv, out, tw, nullptr, nullptr, g)
  switch (lr) {
    case 6: MLH_SHL(6); break;
    case 7: MLH_SHL(7); break;
    case 8: MLH_SHL(8); break;
    case 9: MLH_SHL(9); break;
    default: return hipErrorInvalidValue;
  }
#undef MLH_SHL
  return hipGetLastError();
}

hipError_t launch_pow_table(fe* out, fe base, fe scale, uint64_t count, hipStream_t st,
                            bool expand) {
  const unsigned blocks = (unsigned)((count + 255) / 256);
  hipLaunchKernelGGL(pow_table_kernel, dim3(blocks), dim3(256), 0, st, out, base, scale, count,
                     expand ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_pow_series(fe* out, const fe* tlo, const fe* thi, uint64_t count,
                             hipStream_t st) {
  const unsigned blocks = (unsigned)((count + 255) / 256);
  hipLaunchKernelGGL(pow_series_kernel, dim3(blocks), dim3(256), 0, st, out, tlo, thi, count);
  return hipGetLastError();
}

hipError_t launch_pow_series_check(const fe* gp, uint64_t base, uint64_t count, const fe* tlo,
                                   const fe* thi, unsigned long long* bad, hipStream_t st) {
  if (count == 0) return hipSuccess;
  const unsigned blocks = (unsigned)((count + 255) / 256);
  hipLaunchKernelGGL(pow_series_check_kernel, dim3(blocks), dim3(256), 0, st, gp, base, count, tlo,
                     thi, bad);
  return hipGetLastError();
}

}  // namespace mlh
