// NTT launch interface (internal to libmlhip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.hpp"

namespace mlh {

constexpr int kMaxPasses = 6;
// Inter-pass twiddles w_S^(jrest k) of a pass with W columns, R rows: one
// table TA[k][jrest] (one modmul per element) while R * W <= 2^kFullTwLog
// entries (64 MiB), else split TA[k][jl] * TB[k][jh] with 2^kTwLogA columns
// in TA (two modmuls).  The full table measured -6 % per transform at 2^22
// and -11 % at 2^20 (it stays in the MALL); at 2^24 (256 MiB read at 16 B per
// element beside the 32 B of data) pass 0 was no faster, so there the split
// tables stay.  Re-measured with the LDS twiddle copies (MLH_FULL_TW_LOG=24):
// pass 0 -2..6 %, the transform -1..2 %, for +48 % HBM bytes on pass 0 --
// kept at 22 (the split tables' traffic stays at the algorithmic bytes).
// Expanded inter-pass tables through the generated asm product (round 2:
// 43 instead of ~66 VALU per multiply) measured slower -- pass 0 0.201 ->
// 0.211-0.223 ms: the 4 expanded loads per twiddle cannot be hoisted across
// the asm statements, so every pair of elements waits on its L2 loads.
constexpr uint32_t kTwLogA = 8;
#ifndef MLH_FULL_TW_LOG
#define MLH_FULL_TW_LOG 22
#endif
constexpr uint32_t kFullTwLog = MLH_FULL_TW_LOG;

// Device twiddle tables for one (log_n, generator, direction).
struct NttTables {
  uint32_t log_n = 0;
  uint32_t nradix = 0;
  uint32_t logr[kMaxPasses] = {0};
  // stage twiddles, EXPANDED (4 fe per entry: the limb-shifted multiples
  // consumed by fe_mul_pre): per pass w_R^t, t < R/2
  const fe* tw[kMaxPasses] = {nullptr};
  // inter-pass twiddle of pass p (not last): w_S^(jrest k), jrest < W, k < R,
  // jrest = jh 2^loga + jl: TA[k][jl] = w_S^(k jl) (x n^-1 on pass 0 of the
  // inverse), TB[k][jh] = w_S^(k jh 2^loga); TB = null when W <= 2^loga.
  const fe* ta[kMaxPasses] = {nullptr};
  const fe* tb[kMaxPasses] = {nullptr};
  uint32_t loga[kMaxPasses] = {0};
  // pass 0's twiddle as a progression (ntt_pass_kernel TW 5; single-GPU
  // launch_ntt_passes only, when set): gp = P[k0][j] = w_S^(k0 j) (x n^-1 on
  // the inverse), k0 < 64, j < W; gc = C[j] = w_S^(64 j), expanded
  const fe* gp[kMaxPasses] = {nullptr};
  const fe* gc[kMaxPasses] = {nullptr};
  const fe* tw_small = nullptr;          // N <= 2^10: w^t, t < N/2
  fe scale;                              // n^-1 (inverse) or 1
  bool inverse = false;
  bool debug_sync = false;               // sync after every pass (MLH_DEBUG_SYNC at context creation)
};

// Radix plan of a 2^log_n transform: the default, or `forced` (nforced
// digits 4..9 summing to log_n; ignored otherwise).
void ntt_plan_radices(uint32_t log_n, uint32_t* nradix, uint32_t* logr,
                      const uint32_t* forced = nullptr, uint32_t nforced = 0);

// batch: vectors of in_len inputs / N outputs, contiguous
hipError_t launch_ntt_small(const fe* in, fe* out, const fe* tw, uint32_t log_n, uint64_t in_len,
                            fe scale, bool apply_scale, hipStream_t st, uint64_t batch = 1,
                            bool brev_in = false);
// in: N elements, or N/2 when zero_top != 0 (the upper half is implicit
// zeros); zero_top == 2: those N/2 are stored in bit-reversed order.
// in may equal out; scratch: N elements, distinct from in and out.
// ev (optional, nradix + 1 events): ev[p] is recorded before pass p, ev[P]
// after the last pass (kernel timing on the launch stream).
hipError_t launch_ntt_passes(const fe* in, fe* out, fe* scratch, const NttTables& tb,
                             uint32_t log_n, int zero_top, hipStream_t st,
                             hipEvent_t* ev = nullptr, uint64_t batch = 1);
// out[k][j] = in[k][j] * rowbase^k for a rows x 2^lcols table
hipError_t launch_scale_rows(const fe* in, fe* out, uint64_t rows, uint32_t lcols, fe rowbase,
                             hipStream_t st);
// Passes 0 .. npasses-1 of tb's plan (npasses < nradix): pass 0 in -> out, the
// others in place on out (the sharded fused NTT's local part).
hipError_t launch_ntt_passes_pre(const fe* in, fe* out, const NttTables& tb, uint32_t log_n,
                                 uint32_t npasses, hipStream_t st);
// The last pass of a 2^log_n transform with plan logr[0..nradix) sharded over
// 2^log_p ranks (ntt_pass_kernel TW 4): this rank's tiles, reading the
// all-to-all receive buffer (2^log_p chunks of 2^(log_n - 2 log_p)), writing
// the block-cyclic output (block 2^(logr[0] - log_p)); tw: the pass's stage
// twiddles (expanded).  Needs logr[last] >= log_p + 3, logr[0] >= log_p + 3.
hipError_t launch_ntt_shard_last(const fe* recv, fe* out, const fe* tw, const uint32_t* logr,
                                 uint32_t nradix, uint32_t log_n, uint32_t log_p, uint32_t rank,
                                 hipStream_t st);
// rocprof-style kernel label of pass p ("ntt_pass<8,0,0>")
void ntt_pass_label(const NttTables& tb, uint32_t p, int zero_top, char* buf, size_t n);
// The reference's radix-2 network for any generator (ntt.hip "general-generator
// network"): w^t = tlo[t mod 4096] * thi[t >> 12] for t < N/2; zero_top as
// launch_ntt_passes; scratch (N elements) is used when in == out; apply_scale
// multiplies the outputs by scale (the inverse's n^-1).
hipError_t launch_ntt_network(const fe* in, fe* out, fe* scratch, const fe* tlo, const fe* thi,
                              uint32_t log_n,
                              int zero_top, fe scale, bool apply_scale, hipStream_t st);
hipError_t launch_pow_table(fe* out, fe base, fe scale, uint64_t count, hipStream_t st,
                            bool expand = false);
hipError_t launch_pow_table2d(fe* out, fe base, fe scale, uint64_t rows, uint64_t cols,
                              uint64_t mult, hipStream_t st, bool expand = false);
hipError_t launch_pow_series(fe* out, const fe* tlo, const fe* thi, uint64_t count,
                             hipStream_t st);
// *bad = min(*bad, first t with gp[t] != tlo[(base+t) mod 4096] thi[(base+t) >> 12], as base + t)
hipError_t launch_pow_series_check(const fe* gp, uint64_t base, uint64_t count, const fe* tlo,
                                   const fe* thi, unsigned long long* bad, hipStream_t st);

}  // namespace mlh
