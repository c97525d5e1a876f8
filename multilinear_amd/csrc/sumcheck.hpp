// Sumcheck / MLE launch interface (internal to libmlhip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.hpp"
#include "transcript_dev.hpp"

namespace mlh {

constexpr uint32_t kMaxRedBlocks = 2048;  // partials buffer: 2 * kMaxRedBlocks elements
#ifndef MLH_MAX_GROUP
#define MLH_MAX_GROUP 6
#endif
constexpr uint32_t kMaxGroup = MLH_MAX_GROUP;  // eq-factored head rounds per HBM pass (3 + 3)

// Failure reporting of the cooperative (single-workgroup, role-split) sumcheck
// kernels: a wait on another wave longer than spin_limit sleeps abandons the
// launch's rounds, and a wave that saw it writes 1 to *status (pinned host
// memory, ctx->dev_status), which the prove reads after its sync.
constexpr uint32_t kSpinLimit = 1u << 22;
struct CoopCtl {
  uint32_t* status;     // may be null (no report)
  uint32_t spin_limit;  // sleeps per wait; 0 = kSpinLimit
};

// out[0] = s1, out[1] = s2 over tables of size 2h (device).
hipError_t launch_sums(const fe* m, const fe* d, uint64_t h, fe* partials, fe* out,
                       hipStream_t st, uint32_t* nparts = nullptr);
// fold size-S tables with r, then sums of the folded (size S/2) tables.
// nparts != null: skip the partials reduction and report the partial count
// m_src (optional): fold from m_src into m (out of place; m needs S/2 entries)
hipError_t launch_fold_sums(fe* m, fe* d, uint64_t S, fe r, fe* partials, fe* out,
                            hipStream_t st, const fe* r_dev = nullptr, uint32_t* nparts = nullptr,
                            const fe* m_src = nullptr);
hipError_t launch_fold(fe* m, fe* d, uint64_t S, fe r, hipStream_t st, const fe* r_dev = nullptr,
                       const fe* m_src = nullptr);
// one two-table sumcheck round on the device: reduce the nparts partial sum
// pairs, interpolate, absorb, challenge, new claim
hipError_t launch_sumcheck_round(const fe* partials, uint32_t nparts, fe* prev, DevSha* t,
                                 fe* poly_out, fe* r_out, hipStream_t st);
// Grouped eq-factored head rounds (sumcheck.hip, "grouped eq-factored
// rounds"): corner sums of a group of J <= 6 rounds over T (S entries, e from
// H = H_{k+J-1}) into partials[corner * nb + block]; a J-level fold of T with
// rs[0..J-1] into Tout (S / 2^J entries, may alias T) plus the corner sums of
// the next group of JN rounds (JN = 0: fold only; H = that group's
// H_{k+J+JN-1}); rounds t0..t1-1 of the group from the partials (polys =
// round k+t0's slot, rs / pts = round k's r / p).
hipError_t launch_group_sums_eq(const fe* T, uint64_t S, uint32_t J, const fe* H, const fe* lo,
                                uint32_t a, fe* partials, hipStream_t st, uint32_t* nb);
// (w: the 2^J eq weights of rs, sumcheck_group_kernel's wout)
hipError_t launch_fold_group_eq(const fe* Tin, uint64_t S, uint32_t J, uint32_t JN, const fe* rs,
                                const fe* w, fe* Tout, const fe* H, const fe* lo, uint32_t a,
                                fe* partials, hipStream_t st, uint32_t* nb);
// J2 > 0: two chained groups (J then J2 rounds, all of them) from the
// 2^(J+J2) corner sums of one pass.
// kw (optional): the padding-block K + W tables of eq_setup (round t0's at kw);
// wout (optional): a launch that finishes the group writes the 2^(J+J2) eq
// weights of its challenges there (corner c's MSB = the first variable).
hipError_t launch_sumcheck_group(const fe* partials, uint32_t nb, uint32_t J, uint32_t J2,
                                 uint32_t t0, uint32_t t1, fe* prev, DevSha* t, fe* polys, fe* rs,
                                 const fe* pts, fe* c, hipStream_t st, CoopCtl ctl,
                                 const uint32_t* kw = nullptr, fe* wout = nullptr);
// The last a <= 12 rounds of an eq-factored sumcheck in one LDS-resident
// workgroup (sumcheck_eq_tail_kernel): table = Tin folded over Jin <= 3
// pending variables with rs_in (2^a entries after it), ets = eq suffix tables
// of pts (eq_setup_kernel's Hs), c = the running eq scale; round j's
// outputs at polys + 2j, rs + j; m_out[0] / d_out[0] = the folded tables.
// A device region the last kernel of a prove copies into pinned host memory
// at its end (bytes a multiple of 4; dst == nullptr: none).
struct HostOut {
  const uint8_t* src = nullptr;
  uint8_t* dst = nullptr;
  uint32_t bytes = 0;
};
// xc_part (a >= 6, Jin = 0, optional): group A's corner sums sum_i Tin[c 2^(a-6) + i] e_{5}[i]
// as xc_nb partials per corner (c xc_nb + b), from the fold that wrote Tin.
// rsuf (Jin = 0, optional): the two groups' suffix products of pts as
// eq_setup_kernel writes them (rsuf_out) instead of computed in the prologue.
hipError_t launch_sumcheck_eq_tail(const fe* Tin, uint32_t Jin, const fe* rs_in, uint32_t a,
                                   const fe* ets, const fe* pts, fe* c, fe* prev, DevSha* t,
                                   fe* polys, fe* rs, fe* m_out, fe* d_out, hipStream_t st,
                                   CoopCtl ctl, const uint32_t* kw = nullptr, HostOut ho = {},
                                   const fe* xc_part = nullptr, uint32_t xc_nb = 0,
                                   const fe* rsuf = nullptr);
// The first B <= 12 rounds of an eq-factored sumcheck of 2^(B + a) entries in
// one launch each for their corner sums and their rounds: Y[c] = sum_i T[c 2^a
// + i] lo[i] (the B-variable corner sums, lo = eq of the last a points), then
// the tail kernel's rounds on Y (e_grp = eq of the points after its first
// group of min(B, 6), i.e. H_{min(B,6)-1}); wfold receives the fold weights
// of the two groups (64 + 64), for two fold_group_eq passes over T.
hipError_t launch_corner_sums_lo(const fe* T, uint32_t B, uint32_t a, const fe* lo, fe* Y,
                                 hipStream_t st);
hipError_t launch_sumcheck_eq_head(const fe* Y, uint32_t B, const fe* e_grp, const fe* pts, fe* c,
                                   fe* prev, DevSha* t, fe* polys, fe* rs, fe* wfold,
                                   hipStream_t st, CoopCtl ctl, const uint32_t* kw = nullptr,
                                   const fe* rsuf = nullptr);
// Setup of the eq-factored sumcheck in one launch (arguments by value): the
// points, c_0 = 1, lo = eq(p_B..p_{L-1}), head suffix tables H (over
// p_0..p_{B-1}), tail suffix tables Hs (optional), transcript state and claim
// (optional).  Requires L <= 40, L - B <= 12.
struct EqSetupArgs {
  fe pts[40];
  fe sum;
  DevSha sha;
  uint32_t L, B;
};
// kw (optional, 64 L words): per round k whose (c1, c2) absorb leaves the
// transcript buffer empty (len + 32 (k + 1) = 0 mod 64), the padding block's
// K + W table at kw + 64 k.  rsuf_out (optional, 2 kEqTailRsuf entries): the
// eq tail's two corner groups' suffix products over p_B.. (group g, variable
// u, corner c at g 384 + u 64 + c; sumcheck_eq_tail_kernel's S.rsuf /
// S.rsufB), then the eq head's over p_0..p_{B-1} (B <= 12).
constexpr uint32_t kEqTailRsuf = 2 * 6 * 64;
hipError_t launch_eq_setup(const EqSetupArgs& args, fe* pts_out, fe* c_out, fe* lo, fe* H, fe* Hs,
                           DevSha* dt_out, fe* prev_out, hipStream_t st, uint32_t* kw = nullptr,
                           fe* rsuf_out = nullptr);
// PCS rounds (sumcheck.hip "PCS rounds off the transcript kernel"): the
// running claim, eq scale and last polynomial (e0, c1, c2) in HBM.
struct PcsRoundState {
  fe claim, c, e0, c1, c2;
};
// One PCS round's inputs (launch_pcs_round's arguments): src / dst / log_h /
// fold: the table and its optional fold with *r_prev; p_prev, p_k: points of
// the previous and this round; e: eq suffix; st: state; poly_out: (c1, c2).
struct PcsJob {
  const fe* src;
  fe* dst;
  uint32_t log_h, fold;
  const fe* r_prev;
  const fe* p_prev;
  const fe* p_k;
  const fe* e;
  PcsRoundState* st;
  fe* poly_out;
};
// Round k's (c1, c2) into poly_out from the table src (2^log_h entries after
// the optional fold of src's 2^(log_h+1) entries with *r_prev into dst) and
// e = eq suffix (2^(log_h-1) entries); r_prev non-null: first the previous
// round's claim / eq scale update (p_prev = its point).  One workgroup.
hipError_t launch_pcs_round(const fe* src, fe* dst, uint32_t log_h, bool fold, const fe* r_prev,
                            const fe* p_prev, const fe* p_k, const fe* e, PcsRoundState* st,
                            fe* poly_out, hipStream_t stream);
// fold_group_eq weights of rs[0..JA) at wf[0..2^JA) and rs[JA..JA+JB) at wf[64..64+2^JB)
hipError_t launch_eq_weights(const fe* rs, uint32_t JA, uint32_t JB, fe* wf, hipStream_t st);
// out[i] = (*c) * src[i]
hipError_t launch_scale_dev(const fe* src, const fe* c, uint64_t n, fe* out, hipStream_t st);
// Trace::evaluate: out[j] = sum_i eq[i] * m[i * width + j], j < width;
// partials: trace_eval_blocks(height, min(width, 256)) * min(width, 256) elements.
uint32_t trace_eval_blocks(uint64_t height, uint32_t ncols);
hipError_t launch_trace_eval(const fe* m, const fe* eq, uint64_t height, uint32_t width,
                             fe* partials, fe* out, hipStream_t st);
// Device-resident sumcheck tail: the last sumcheck_tail_rounds(L) rounds on
// tables of 2^log_s entries in one workgroup (LDS); polys/rs/prev/t as for
// sumcheck_round_kernel, round k's outputs at polys + 2k, rs + k.
uint32_t sumcheck_tail_rounds(uint32_t log_height);
// m_src (optional): read the tables' m from m_src, write the folded half to m
hipError_t launch_sumcheck_tail(fe* m, fe* d, uint32_t log_s, fe* prev, DevSha* t, fe* polys,
                                fe* rs, hipStream_t st, const fe* m_src = nullptr);
hipError_t launch_dot(const fe* a, const fe* b, uint64_t n, fe* partials, fe* out,
                      hipStream_t st);
// mono: monomial table prod_{bit_i set} p[n-1-i] (coefficient-form MLE evaluation)
hipError_t launch_eq_table(const fe* pts, uint32_t n, fe* scratch, fe* out, hipStream_t st,
                           bool mono = false);
// out[0] = sum_i c[i] * tlo[i mod 4096] * thi[i / 4096] (partials: kMaxRedBlocks pairs)
hipError_t launch_poly_eval(const fe* c, uint64_t n, const fe* tlo, const fe* thi, fe* partials,
                            fe* out, hipStream_t st);
// src (optional): the first pass reads src instead of c (out-of-place transform)
hipError_t launch_mobius(fe* c, uint32_t log_n, bool inverse_zeta, hipStream_t st,
                         const fe* src = nullptr);
hipError_t launch_bitrev(const fe* in, fe* out, uint32_t log_n, hipStream_t st);

}  // namespace mlh
