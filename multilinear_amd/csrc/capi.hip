// C ABI (include/mlhip.h) and the C++ host layer above the gfx950 kernels.
//
// This file mirrors the reference's prover-side orchestration:
//   FriProverData::{init, fold_step, fold, open_query_at}  src/fri/mod.rs:57-175
//   FriProof::{prove, verify, verify_queries}               src/fri/mod.rs:260-341
//   SumcheckTables::compute_sumcheck_polynomial(s)          sumcheck.rs:77-202
//   PCSProof::{prove, verify}                               multilinear_pcs.rs:90-190
// with every large vector device resident; only roots (32 B), round sums
// (32 B), the last element and the opened query paths cross PCIe.  The
// Fiat-Shamir transcript runs on the host (it is a strict sequence of small
// SHA-256 updates; one host round trip per round).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/mlhip.h"
#include "field.hpp"
#include "batched.hpp"
#include "dist.hpp"
#include "fieldops.hpp"
#include "host_field.hpp"
#include "host_sha256.hpp"
#include "host_transcript.hpp"
#include "context.hpp"
#include "fused_ntt.hpp"
#include "merkle.hpp"
#include "ntt.hpp"
#include "sha256.hpp"
#include "sumcheck.hpp"
#include "transcript_dev.hpp"

using namespace mlh;


// Table cache bound: when a new table would take the cache past its limit,
// least-recently-used tables are freed (after the stream drains, since queued
// kernels may still read them).  The tables one operation fetches are stamped
// consecutively and fewer than kTablePin (an NTT of 2^40: 5 stage + 4 + 4
// inter-pass tables; a PCS prove: those + 2 fold tables), so the newest
// kTablePin stamps -- every table the running operation holds a pointer to --
// are never evicted.
constexpr uint64_t kTablePin = 24;

static mlh_status table_make_room(mlh_ctx* ctx, size_t need) {
  if (ctx->table_bytes + need <= ctx->table_limit) return MLH_OK;
  std::vector<std::pair<uint64_t, TableKey>> order;
  for (auto& kv : ctx->tables)
    if (kv.second.stamp + kTablePin <= ctx->table_stamp) order.push_back({kv.second.stamp, kv.first});
  std::sort(order.begin(), order.end(),
            [](const std::pair<uint64_t, TableKey>& a, const std::pair<uint64_t, TableKey>& b) {
              return a.first < b.first;
            });
  bool synced = false;
  for (auto& o : order) {
    if (ctx->table_bytes + need <= ctx->table_limit) break;
    if (!synced) {
      HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
      synced = true;
    }
    auto it = ctx->tables.find(o.second);
    HIP_TRY(ctx, hipFree(it->second.d));
    ctx->table_bytes -= it->second.bytes;
    ctx->tables.erase(it);
  }
  return MLH_OK;
}

static bool table_hit(mlh_ctx* ctx, const TableKey& k, const fe** out) {
  auto it = ctx->tables.find(k);
  if (it == ctx->tables.end()) return false;
  it->second.stamp = ++ctx->table_stamp;
  *out = it->second.d;
  return true;
}

static mlh_status table_alloc(mlh_ctx* ctx, const TableKey& k, size_t bytes, fe** d) {
  MLH_TRY(table_make_room(ctx, bytes));
  HIP_TRY(ctx, hipMalloc(d, bytes));
  ctx->tables[k] = CachedTable{*d, bytes, ++ctx->table_stamp};
  ctx->table_bytes += bytes;
  return MLH_OK;
}

// table[t] = base^t * scale, t < count, cached per context.  expand: 4 fe per
// entry (t * 2^(32k), k < 4) for fe_mul_pre.
static mlh_status get_table(mlh_ctx* ctx, u128 base, uint64_t count, u128 scale, const fe** out,
                            bool expand = false) {
  TableKey k{base, count, scale, expand ? 1 : 0};
  if (table_hit(ctx, k, out)) return MLH_OK;
  fe* d = nullptr;
  MLH_TRY(table_alloc(ctx, k, count * sizeof(fe) * (expand ? 4 : 1), &d));
  HIP_TRY(ctx, launch_pow_table(d, to_fe(base), to_fe(scale), count, ctx->stream, expand));
  *out = d;
  return MLH_OK;
}

// 2D table[k * cols + j] = base^(k j mult) * scale, k < rows, cached per context
static mlh_status get_table2d(mlh_ctx* ctx, u128 base, uint64_t rows, uint64_t cols,
                              uint64_t mult, u128 scale, const fe** out, bool expand = false) {
  TableKey k{base, rows, scale, expand ? 1 : 0, cols, mult};
  if (table_hit(ctx, k, out)) return MLH_OK;
  fe* d = nullptr;
  MLH_TRY(table_alloc(ctx, k, rows * cols * sizeof(fe) * (expand ? 4 : 1), &d));
  HIP_TRY(ctx, launch_pow_table2d(d, to_fe(base), to_fe(scale), rows, cols, mult, ctx->stream,
                                  expand));
  *out = d;
  return MLH_OK;
}

static CoopCtl coop_ctl(mlh_ctx* ctx) {
  return CoopCtl{const_cast<uint32_t*>(ctx->dev_status), ctx->coop_spin};
}

static uint64_t hi_count(uint32_t log_n) {
  const uint64_t N = 1ull << log_n;
  return N <= 4096 ? 1 : N / 4096;
}

#ifndef MLH_P0_GEO
#define MLH_P0_GEO 1  // 0: pass 0 always multiplies TA * TB
#endif
#ifndef MLH_P0_GEO_MAXLOGW
#define MLH_P0_GEO_MAXLOGW 16  // largest W (columns) of the progression table: 64 W entries
#endif
static mlh_status get_ntt_tables(mlh_ctx* ctx, u128 gen, uint32_t log_n, bool inverse,
                                 NttTables* tb, const uint32_t* plan = nullptr, uint32_t nplan = 0) {
  const uint64_t N = 1ull << log_n;
  const u128 w = inverse ? h_inv(gen) : gen;
  const u128 scale = inverse ? h_inv((u128)N) : (u128)1;
  tb->log_n = log_n;
  tb->inverse = inverse;
  tb->scale = to_fe(scale);
  if (log_n <= 10) {
    MLH_TRY(get_table(ctx, w, N / 2 ? N / 2 : 1, 1, &tb->tw_small));
    return MLH_OK;
  }
  tb->debug_sync = ctx->debug_sync;
  if (plan)
    ntt_plan_radices(log_n, &tb->nradix, tb->logr, plan, nplan);
  else
    ntt_plan_radices(log_n, &tb->nradix, tb->logr, ctx->forced_plan, ctx->forced_plan_len);
  for (uint32_t p = 0; p < tb->nradix; ++p) {
    const uint64_t R = 1ull << tb->logr[p];
    MLH_TRY(get_table(ctx, h_pow(w, N / R), R / 2, 1, &tb->tw[p], true));
  }
  uint64_t S = 1;
  for (uint32_t p = 0; p + 1 < tb->nradix; ++p) {  // the last pass has no twiddle
    const uint64_t R = 1ull << tb->logr[p];
    const uint32_t logw = log_n - (uint32_t)__builtin_ctzll(S) - tb->logr[p];
    const uint32_t loga =
        tb->logr[p] + logw <= kFullTwLog ? logw : (logw < kTwLogA ? logw : kTwLogA);
    const u128 ws = h_pow(w, S);
    tb->loga[p] = loga;
    MLH_TRY(get_table2d(ctx, ws, R, 1ull << loga, 1, p == 0 ? scale : (u128)1, &tb->ta[p]));
    tb->tb[p] = nullptr;
    if (logw > loga)  // expanded: the kernel multiplies by it with the expanded product
      MLH_TRY(get_table2d(ctx, ws, R, 1ull << (logw - loga), 1ull << loga, 1, &tb->tb[p], true));
    // pass 0 with two tables, R = 2^7 / 2^8, W <= 2^16: the progression form
    // (64 W + 4 W entries: 68 MiB at 2^24)
    if (MLH_P0_GEO && p == 0 && logw > loga && (tb->logr[0] == 7 || tb->logr[0] == 8) &&
        logw <= MLH_P0_GEO_MAXLOGW) {
      MLH_TRY(get_table2d(ctx, ws, 64, 1ull << logw, 1, scale, &tb->gp[0]));
      MLH_TRY(get_table(ctx, h_pow(ws, 64), 1ull << logw, 1, &tb->gc[0], true));
    }
    S <<= tb->logr[p];
  }
  return MLH_OK;
}

// gen must have order exactly 2^log_n
static bool check_generator(u128 gen, uint32_t log_n) {
  if (gen >= kModulus) return false;
  if (log_n == 0) return gen == 1;
  const u128 half = h_pow(gen, (u128)1 << (log_n - 1));
  return half == kModulus - 1;  // gen^(N/2) = -1  <=>  order exactly N
}

static mlh_status ensure_ntt_scratch(mlh_ctx* ctx, uint32_t log_n) {
  const size_t need = (size_t)16 << log_n;
  if (ctx->ntt_scratch_bytes < need) {
    if (ctx->ntt_scratch) {
      HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
      HIP_TRY(ctx, hipFree(ctx->ntt_scratch));
      ctx->ntt_scratch = nullptr;
      ctx->ntt_scratch_bytes = 0;
    }
    HIP_TRY(ctx, hipMalloc(&ctx->ntt_scratch, need));
    ctx->ntt_scratch_bytes = need;
  }
  return MLH_OK;
}

// Generator of any other order (gen < M; 0 included): the reference's radix-2
// network stage by stage (ntt.hip "general-generator network"), w = gen or,
// for the inverse, gen^-1 (winter-math inverts 0 to 0, as h_inv does).
static mlh_status ntt_network_core(mlh_ctx* ctx, const fe* in, fe* out, uint32_t log_n, u128 gen,
                                   bool inverse, int zero_top) {
  const u128 w = inverse ? h_inv(gen) : gen;
  const fe *tlo, *thi;  // w^t = tlo[t mod 4096] thi[t >> 12], t < N/2
  MLH_TRY(get_table(ctx, w, 4096, 1, &tlo));
  MLH_TRY(get_table(ctx, h_pow(w, 4096), hi_count(log_n - 1), 1, &thi));
  fe* scratch = nullptr;
  if (in == out && log_n > 11) {
    MLH_TRY(ensure_ntt_scratch(ctx, log_n));
    scratch = ctx->ntt_scratch;
  }
  const u128 scale = inverse ? h_inv((u128)1 << log_n) : (u128)1;
  HIP_TRY(ctx, launch_ntt_network(in, out, scratch, tlo, thi, log_n, zero_top, to_fe(scale), inverse,
                                  ctx->stream));
  return MLH_OK;
}

// ---------------------------------------------------------------------------
// Sharded NTT with the rank digit fused into the last pass (fused_ntt.hpp):
// the global 2^L transform runs the plan (local digits..., c + p) where the
// local 2^(L-p) array of rank g (cyclic: global index P m + g) takes the
// passes before the last one exactly as a local NTT with plan (local digits...,
// c) would, except that each inter-pass table row k carries the extra factor
// (w_N^S)^(k g) (the global column index is P j + g); the last pass transforms
// the low (c + p) bits of the global index -- c local bits and the p rank bits
// -- on the all-to-all's receive buffer.  Three HBM passes instead of the
// local NTT's three plus the cross-shard DFT's one.
FusedNtt::~FusedNtt() {
  for (void* q : scaled) pool_free(ctx, q);
}

mlh_status FusedNtt::prepare(mlh_ctx* c, u128 gen, uint32_t log_n, uint32_t log_p, uint32_t rank_) {
  ctx = c;
  L = log_n;
  p = log_p;
  rank = rank_;
  const uint32_t Lloc = L - p;
  const uint32_t cl = 9 - p;  // local bits of the last digit: the fused radix is 2^9
  if (p < 1 || p > 4 || cl < 4 || Lloc < cl + 4 || Lloc > 40) return fail(ctx, MLH_ERR_INVALID, "fused plan");
  uint32_t npre = 0, pre[kMaxPasses];
  ntt_plan_radices(Lloc - cl, &npre, pre);
  if (npre + 1 > (uint32_t)kMaxPasses || pre[0] < p + 3) return fail(ctx, MLH_ERR_INVALID, "fused plan");
  uint32_t plan[kMaxPasses];
  for (uint32_t i = 0; i < npre; ++i) plan[i] = pre[i];
  plan[npre] = cl;
  // the local plan as a forced plan needs digits 4..9 (ntt_plan_radices)
  for (uint32_t i = 0; i <= npre; ++i)
    if (plan[i] < 4 || plan[i] > 9) return fail(ctx, MLH_ERR_INVALID, "fused plan");
  const u128 gl = h_pow(gen, (u128)1 << p);  // the local generator w_N^P
  MLH_TRY(get_ntt_tables(ctx, gl, Lloc, false, &loc, plan, npre + 1));
  if (loc.nradix != npre + 1) return fail(ctx, MLH_ERR_INVALID, "fused plan");
  nglob = npre + 1;
  for (uint32_t i = 0; i < npre; ++i) logr[i] = plan[i];
  logr[npre] = cl + p;
  // rank twist of the pre-exchange passes' TA rows: (w_N^S)^(k rank)
  uint64_t S = 1;
  for (uint32_t i = 0; i < npre; ++i) {
    const uint64_t R = 1ull << plan[i];
    void* q;
    MLH_TRY(pool_alloc(ctx, (R << loc.loga[i]) * sizeof(fe), &q));
    scaled.push_back(q);
    const u128 rb = h_pow(gen, (u128)S * rank);
    HIP_TRY(ctx, launch_scale_rows(loc.ta[i], reinterpret_cast<fe*>(q), R, loc.loga[i], to_fe(rb), ctx->stream));
    loc.ta[i] = reinterpret_cast<const fe*>(q);
    S <<= plan[i];
  }
  // the fused last pass's stage twiddles: w_N^(N / 2^9), expanded
  const uint64_t Rl = 1ull << logr[npre];
  MLH_TRY(get_table(ctx, h_pow(gen, (u128)(1ull << (L - logr[npre]))), Rl / 2, 1, &tw_last, true));
  return MLH_OK;
}

mlh_status FusedNtt::run_pre(const void* in, void* out) {
  ProfScope ps(ctx, "ntt_fused_pre");
  HIP_TRY(ctx, launch_ntt_passes_pre(reinterpret_cast<const fe*>(in), reinterpret_cast<fe*>(out), loc, L - p,
                                     nglob - 1, ctx->stream));
  ps.end();
  return MLH_OK;
}

mlh_status FusedNtt::run_last(const void* recv, void* out) {
  ProfScope ps(ctx, "ntt_fused_last");
  HIP_TRY(ctx, launch_ntt_shard_last(reinterpret_cast<const fe*>(recv), reinterpret_cast<fe*>(out), tw_last,
                                     logr, nglob, L, p, rank, ctx->stream));
  ps.end();
  return MLH_OK;
}

// Core NTT on device (in may equal out; zero_top 1: input has N/2 elements,
// 2: N/2 elements stored bit-reversed -- then in must not equal out).
static mlh_status ntt_core(mlh_ctx* ctx, const fe* in, fe* out, uint32_t log_n, u128 gen,
                           bool inverse, int zero_top) {
  NttTables tb;
  MLH_TRY(get_ntt_tables(ctx, gen, log_n, inverse, &tb));
  if (log_n <= 10) {
    const uint64_t N = 1ull << log_n;
    // (in-place is safe: the small kernel reads everything into LDS before writing)
    HIP_TRY(ctx, launch_ntt_small(in, out, tb.tw_small, log_n, zero_top ? N / 2 : N, tb.scale,
                                  inverse, ctx->stream, 1, zero_top == 2));
    return MLH_OK;
  }
  MLH_TRY(ensure_ntt_scratch(ctx, log_n));
  char lab0[64];
  if (ctx->prof_on) ntt_pass_label(tb, 0, zero_top, lab0, sizeof lab0);
  if (ctx->prof_on && prof_sample(ctx, lab0)) {
    std::vector<hipEvent_t> ev(tb.nradix + 1);
    for (auto& e : ev) e = take_event(ctx);
    HIP_TRY(ctx, launch_ntt_passes(in, out, ctx->ntt_scratch, tb, log_n, zero_top, ctx->stream,
                                   ev.data()));
    for (uint32_t p = 0; p < tb.nradix; ++p) {
      char lab[64];
      ntt_pass_label(tb, p, zero_top, lab, sizeof lab);
      ctx->pending.push_back(mlh_ctx::Pending{lab, ev[p], ev[p + 1]});
    }
    return MLH_OK;
  }
  HIP_TRY(ctx, launch_ntt_passes(in, out, ctx->ntt_scratch, tb, log_n, zero_top, ctx->stream));
  return MLH_OK;
}

// ---------------------------------------------------------------------------
// context / memory API
// ---------------------------------------------------------------------------
extern "C" {

const char* mlh_version(void) { return "mlhip 0.1 (gfx950)"; }

// why the last mlh_context_create of this thread failed (no context to hold it):
// mlh_last_error(NULL) returns it
static thread_local char g_create_err[160] = "null context";

mlh_status mlh_context_create(int device, void* hip_stream, mlh_ctx** out) {
  if (!out) return MLH_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= device || device < 0) {
    snprintf(g_create_err, sizeof g_create_err, "mlh_context_create: hipGetDeviceCount -> %s, %d devices, device %d",
             hipGetErrorString(e), n, device);
    return MLH_ERR_HIP;
  }
  e = hipSetDevice(device);
  if (e != hipSuccess) {
    snprintf(g_create_err, sizeof g_create_err, "mlh_context_create: hipSetDevice(%d) -> %s", device,
             hipGetErrorString(e));
    return MLH_ERR_HIP;
  }
  std::unique_ptr<mlh_ctx> c(new mlh_ctx());
  c->device = device;
  c->stream = reinterpret_cast<hipStream_t>(hip_stream);
  const char* dbg = getenv("MLH_DEBUG_SYNC");
  c->debug_sync = dbg && *dbg && strcmp(dbg, "0") != 0;
  void* st = nullptr;
  const bool ok = hipMalloc(&c->partials, 2 * kMaxRedBlocks * sizeof(fe)) == hipSuccess &&
                  hipMalloc(&c->small, 64 * sizeof(fe)) == hipSuccess &&
                  hipHostMalloc(&c->pinned, kPinnedBytes, 0) == hipSuccess &&
                  hipHostMalloc(&st, 64, hipHostMallocCoherent) == hipSuccess;
  if (!ok) {  // (hipFree / hipHostFree of a null pointer are no-ops)
    snprintf(g_create_err, sizeof g_create_err, "mlh_context_create: allocation failed (%s)",
             hipGetErrorString(hipGetLastError()));
    (void)hipFree(c->partials);
    (void)hipFree(c->small);
    (void)hipHostFree(c->pinned);
    (void)hipHostFree(st);
    return MLH_ERR_OOM;
  }
  c->dev_status = reinterpret_cast<volatile uint32_t*>(st);
  *c->dev_status = 0;
  *out = c.release();
  return MLH_OK;
}

void mlh_context_destroy(mlh_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->side) (void)hipStreamSynchronize(ctx->side);  // before anything it may use is freed
  if (ctx->side2) (void)hipStreamSynchronize(ctx->side2);
  resolve_profile(ctx);
  for (auto e : ctx->ev_free) (void)hipEventDestroy(e);
  for (auto& kv : ctx->tables) (void)hipFree(kv.second.d);
  for (auto& kv : ctx->pool) (void)hipFree(kv.second);
  for (auto& kv : ctx->live) (void)hipFree(kv.first);
  (void)hipFree(ctx->ntt_scratch);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  if (ctx->side2) (void)hipStreamDestroy(ctx->side2);
  (void)hipFree(ctx->partials);
  (void)hipFree(ctx->small);
  (void)hipHostFree(ctx->pinned);
  (void)hipHostFree(const_cast<uint32_t*>(ctx->dev_status));
  if (ctx->qstage) (void)hipHostFree(ctx->qstage);
  delete ctx;
}

mlh_status mlh_set_table_cache_limit(mlh_ctx* ctx, uint64_t bytes) {
  if (!ctx) return MLH_ERR_INVALID;
  ctx->table_limit = (size_t)bytes;
  return table_make_room(ctx, 0);
}

uint64_t mlh_table_cache_bytes(const mlh_ctx* ctx) { return ctx ? ctx->table_bytes : 0; }

mlh_status mlh_set_ntt_plan(mlh_ctx* ctx, const uint32_t* logr, uint32_t count) {
  if (!ctx || (count && !logr) || count > (uint32_t)kMaxPasses)
    return fail(ctx, MLH_ERR_INVALID, "plan: at most kMaxPasses digits");
  for (uint32_t i = 0; i < count; ++i)
    if (logr[i] < 4 || logr[i] > 9) return fail(ctx, MLH_ERR_INVALID, "plan digits must be 4..9");
  ctx->forced_plan_len = count;
  for (uint32_t i = 0; i < count; ++i) ctx->forced_plan[i] = logr[i];
  return MLH_OK;
}

mlh_status mlh_set_coop_spin_limit(mlh_ctx* ctx, uint32_t sleeps) {
  if (!ctx) return MLH_ERR_INVALID;
  ctx->coop_spin = sleeps;
  return MLH_OK;
}

mlh_status mlh_set_pcs_fused_max(mlh_ctx* ctx, uint32_t max_vars) {
  if (!ctx) return MLH_ERR_INVALID;
  ctx->pcs_fused_max = max_vars < 24 ? max_vars : 24;
  return MLH_OK;
}

mlh_status mlh_set_stream(mlh_ctx* ctx, void* hip_stream) {
  if (!ctx) return MLH_ERR_INVALID;
  ctx->stream = reinterpret_cast<hipStream_t>(hip_stream);
  return MLH_OK;
}

mlh_status mlh_synchronize(mlh_ctx* ctx) {
  if (!ctx) return MLH_ERR_INVALID;
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MLH_OK;
}

const char* mlh_last_error(const mlh_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err; }

mlh_status mlh_malloc(mlh_ctx* ctx, size_t bytes, void** dev) {
  if (!ctx || !dev) return MLH_ERR_INVALID;
  HIP_TRY(ctx, hipMalloc(dev, bytes ? bytes : 16));
  return MLH_OK;
}
mlh_status mlh_free(mlh_ctx* ctx, void* dev) {
  if (!ctx) return MLH_ERR_INVALID;
  HIP_TRY(ctx, hipFree(dev));
  return MLH_OK;
}
mlh_status mlh_memcpy_h2d(mlh_ctx* ctx, void* dev, const void* host, size_t bytes) {
  if (!ctx) return MLH_ERR_INVALID;
  HIP_TRY(ctx, hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MLH_OK;
}
mlh_status mlh_memcpy_d2h(mlh_ctx* ctx, void* host, const void* dev, size_t bytes) {
  if (!ctx) return MLH_ERR_INVALID;
  HIP_TRY(ctx, hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MLH_OK;
}
mlh_status mlh_memcpy_d2d(mlh_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return MLH_ERR_INVALID;
  HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  return MLH_OK;
}

// ---------------------------------------------------------------------------
// field helpers / NTT
// ---------------------------------------------------------------------------
mlh_status mlh_pow_2_generator(uint32_t log_size, uint8_t gen_out[16]) {
  if (!gen_out || log_size > 40) return MLH_ERR_INVALID;
  h_store(gen_out, h_pow2_generator(log_size));
  return MLH_OK;
}

mlh_status mlh_gen_pows_params(const uint8_t* gen_pows, uint64_t len, uint8_t gen_out[16],
                               uint32_t* log_len_out) {
  if (!gen_pows || !gen_out || !log_len_out) return MLH_ERR_INVALID;
  if (len < 2 || (len & (len - 1)) || len > (1ull << 40)) return MLH_ERR_INVALID;
  const uint32_t lg = 63 - __builtin_clzll(len);
  auto at = [&](uint64_t i) { return h_load(gen_pows + 16 * i); };
  const u128 g = at(1);
  if (at(0) != 1 || !check_generator(g, lg)) return MLH_ERR_INVALID;  // order exactly len
  u128 p = g;
  for (uint32_t j = 0; j < lg; ++j, p = h_mul(p, p))
    if (at(1ull << j) != p) return MLH_ERR_INVALID;  // gen_pows[2^j] = g^(2^j)
  if (at(len / 2) != kModulus - 1 || h_mul(at(len - 1), g) != 1) return MLH_ERR_INVALID;
  // every index below 4096, and 16 pseudo-random ones (SplitMix64 of len)
  p = 1;
  for (uint64_t i = 0; i < len && i < 4096; ++i, p = h_mul(p, g))
    if (at(i) != p) return MLH_ERR_INVALID;
  uint64_t x = len ^ 0x9E3779B97F4A7C15ull;
  for (int q = 0; q < 16; ++q) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const uint64_t i = z & (len - 1);
    if (at(i) != h_pow(g, (u128)i)) return MLH_ERR_INVALID;
  }
  h_store(gen_out, g);
  *log_len_out = lg;
  return MLH_OK;
}

mlh_status mlh_gen_pows_verify(mlh_ctx* ctx, const uint8_t* gen_pows, uint64_t len,
                               uint8_t gen_out[16], uint32_t* log_len_out) {
  if (!ctx || !gen_pows) return fail(ctx, MLH_ERR_INVALID, "null argument");
  uint8_t gb[16];
  uint32_t lg = 0;
  if (mlh_gen_pows_params(gen_pows, len, gb, &lg) != MLH_OK)
    return fail(ctx, MLH_ERR_INVALID, "gen_pows is not the power series of an element of order len");
  const u128 g = h_load(gb);
  const fe *tlo, *thi;
  MLH_TRY(get_table(ctx, g, 4096, 1, &tlo));
  MLH_TRY(get_table(ctx, h_pow(g, 4096), hi_count(lg), 1, &thi));
  const uint64_t chunk = len < (1ull << 20) ? len : (1ull << 20);
  PoolBuf buf(ctx), badb(ctx);
  MLH_TRY(buf.alloc(chunk * 16));
  MLH_TRY(badb.alloc(8));
  unsigned long long* bad = badb.as<unsigned long long>();
  HIP_TRY(ctx, hipMemsetAsync(bad, 0xFF, 8, ctx->stream));
  for (uint64_t base = 0; base < len; base += chunk) {  // stream order keeps buf's reuse safe
    const uint64_t cnt = len - base < chunk ? len - base : chunk;
    HIP_TRY(ctx, hipMemcpyAsync(buf.p, gen_pows + 16 * base, cnt * 16, hipMemcpyHostToDevice,
                                ctx->stream));
    HIP_TRY(ctx, launch_pow_series_check(buf.as<fe>(), base, cnt, tlo, thi, bad, ctx->stream));
  }
  HIP_TRY(ctx, hipMemcpyAsync(ctx->pinned + kPinSlotB, bad, 8, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  uint64_t first;
  memcpy(&first, ctx->pinned + kPinSlotB, 8);
  if (first != ~0ull)
    return fail(ctx, MLH_ERR_INVALID,
                "gen_pows[" + std::to_string(first) + "] is not gen_pows[1]^" + std::to_string(first));
  if (gen_out) memcpy(gen_out, gb, 16);
  if (log_len_out) *log_len_out = lg;
  return MLH_OK;
}

mlh_status mlh_pow_2_generator_powers(mlh_ctx* ctx, uint32_t log_size, void* dev_out) {
  if (!ctx || !dev_out || log_size > 40) return fail(ctx, MLH_ERR_INVALID, "bad argument");
  const u128 g = h_pow2_generator(log_size);
  const fe *tlo, *thi;
  MLH_TRY(get_table(ctx, g, 4096, 1, &tlo));
  MLH_TRY(get_table(ctx, h_pow(g, 4096), hi_count(log_size), 1, &thi));
  HIP_TRY(ctx, launch_pow_series(reinterpret_cast<fe*>(dev_out), tlo, thi, 1ull << log_size,
                                 ctx->stream));
  return MLH_OK;
}

static mlh_status ntt_entry(mlh_ctx* ctx, const void* in, void* out, uint32_t log_n,
                            const uint8_t gen[16], bool inverse) {
  if (!ctx || !in || !out || !gen) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_n < 1 || log_n > 32) return fail(ctx, MLH_ERR_NOT_POW2, "The number of coeffs must be a power of 2 (n >= 2)");
  const u128 g = h_load(gen);
  if (g >= kModulus) return fail(ctx, MLH_ERR_BAD_GENERATOR, "generator not canonical");
  if (!check_generator(g, log_n))  // not of order n: the reference's network, not a DFT
    return ntt_network_core(ctx, reinterpret_cast<const fe*>(in), reinterpret_cast<fe*>(out),
                            log_n, g, inverse, 0);
  return ntt_core(ctx, reinterpret_cast<const fe*>(in), reinterpret_cast<fe*>(out), log_n, g,
                  inverse, false);
}

mlh_status mlh_ntt(mlh_ctx* ctx, const void* dev_coeffs, void* dev_evals, uint32_t log_n,
                   const uint8_t gen[16]) {
  return ntt_entry(ctx, dev_coeffs, dev_evals, log_n, gen, false);
}

mlh_status mlh_intt(mlh_ctx* ctx, const void* dev_evals, void* dev_coeffs, uint32_t log_n,
                    const uint8_t gen[16]) {
  return ntt_entry(ctx, dev_evals, dev_coeffs, log_n, gen, true);
}

static mlh_status vec_op(mlh_ctx* ctx, int op, const void* a, const void* b, void* out, uint64_t n) {
  if (!ctx || !a || !out || (op < 3 && !b)) return fail(ctx, MLH_ERR_INVALID, "null argument");
  HIP_TRY(ctx, launch_vec_op(op, reinterpret_cast<const fe*>(a), reinterpret_cast<const fe*>(b),
                             reinterpret_cast<fe*>(out), n, ctx->stream));
  return MLH_OK;
}
mlh_status mlh_field_add(mlh_ctx* ctx, const void* a, const void* b, void* out, uint64_t n) {
  return vec_op(ctx, 0, a, b, out, n);
}
mlh_status mlh_field_sub(mlh_ctx* ctx, const void* a, const void* b, void* out, uint64_t n) {
  return vec_op(ctx, 1, a, b, out, n);
}
mlh_status mlh_field_mul(mlh_ctx* ctx, const void* a, const void* b, void* out, uint64_t n) {
  return vec_op(ctx, 2, a, b, out, n);
}
mlh_status mlh_field_neg(mlh_ctx* ctx, const void* a, void* out, uint64_t n) {
  return vec_op(ctx, 3, a, nullptr, out, n);
}
mlh_status mlh_field_scale(mlh_ctx* ctx, const void* a, const uint8_t c[16], void* out,
                           uint64_t n) {
  if (!ctx || !a || !out || !c) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (h_load(c) >= kModulus) return fail(ctx, MLH_ERR_INVALID, "scalar not canonical");
  HIP_TRY(ctx, launch_vec_op(4, reinterpret_cast<const fe*>(a), nullptr, reinterpret_cast<fe*>(out),
                             n, ctx->stream, to_fe(h_load(c))));
  return MLH_OK;
}

mlh_status mlh_bit_reverse_permutation(mlh_ctx* ctx, const void* dev_in, void* dev_out,
                                       uint32_t log_n) {
  if (!ctx || !dev_in || !dev_out || dev_in == dev_out)
    return fail(ctx, MLH_ERR_INVALID, "bit_reverse_permutation is out of place");
  if (log_n > 40) return fail(ctx, MLH_ERR_INVALID, "log_n too large");
  // n = 1 has no bit reversal in the reference (a usize shifted by 64: a
  // panic); n >= 2 as there
  if (log_n == 0) return fail(ctx, MLH_ERR_NOT_POW2, "bit_reverse_permutation needs n >= 2");
  HIP_TRY(ctx, launch_bitrev(reinterpret_cast<const fe*>(dev_in), reinterpret_cast<fe*>(dev_out),
                             log_n, ctx->stream));
  return MLH_OK;
}

mlh_status mlh_ntt_host(mlh_ctx* ctx, const uint8_t* host_in, uint8_t* host_out, uint32_t log_n,
                        const uint8_t gen[16], int inverse) {
  if (!ctx || !host_in || !host_out) return fail(ctx, MLH_ERR_INVALID, "null argument");
  const size_t bytes = (size_t)16 << log_n;
  PoolBuf buf(ctx);
  MLH_TRY(buf.alloc(bytes));
  HIP_TRY(ctx, hipMemcpyAsync(buf.p, host_in, bytes, hipMemcpyHostToDevice, ctx->stream));
  MLH_TRY(ntt_entry(ctx, buf.p, buf.p, log_n, gen, inverse != 0));
  HIP_TRY(ctx, hipMemcpyAsync(host_out, buf.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MLH_OK;
}

// ---------------------------------------------------------------------------
// Reed-Solomon / Merkle / fold
// ---------------------------------------------------------------------------
mlh_status mlh_reed_solomon(mlh_ctx* ctx, const void* dev_coeffs, uint32_t log_n,
                            const uint8_t gen[16], void* dev_code) {
  if (!ctx || !dev_coeffs || !dev_code || !gen) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_n > 31) return fail(ctx, MLH_ERR_INVALID, "log_n too large");
  if (dev_coeffs == dev_code) return fail(ctx, MLH_ERR_INVALID, "reed_solomon is out of place");
  const uint32_t lc = log_n + MLH_LOG_BLOWUP;
  const u128 g = h_load(gen);
  if (g >= kModulus) return fail(ctx, MLH_ERR_BAD_GENERATOR, "generator not canonical");
  if (!check_generator(g, lc))  // not of order 2n: the reference's network, not a DFT
    return ntt_network_core(ctx, reinterpret_cast<const fe*>(dev_coeffs),
                            reinterpret_cast<fe*>(dev_code), lc, g, false, 1);
  return ntt_core(ctx, reinterpret_cast<const fe*>(dev_coeffs), reinterpret_cast<fe*>(dev_code),
                  lc, g, false, 1);
}

mlh_status mlh_reed_solomon_brev(mlh_ctx* ctx, const void* dev_coeffs, uint32_t log_n,
                                 const uint8_t gen[16], void* dev_code) {
  if (!ctx || !dev_coeffs || !dev_code || !gen) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_n > 31) return fail(ctx, MLH_ERR_INVALID, "log_n too large");
  if (dev_coeffs == dev_code) return fail(ctx, MLH_ERR_INVALID, "reed_solomon is out of place");
  const uint32_t lc = log_n + MLH_LOG_BLOWUP;
  const u128 g = h_load(gen);
  if (g >= kModulus) return fail(ctx, MLH_ERR_BAD_GENERATOR, "generator not canonical");
  if (!check_generator(g, lc))  // not of order 2n: the reference's network, not a DFT
    return ntt_network_core(ctx, reinterpret_cast<const fe*>(dev_coeffs),
                            reinterpret_cast<fe*>(dev_code), lc, g, false, 2);
  return ntt_core(ctx, reinterpret_cast<const fe*>(dev_coeffs), reinterpret_cast<fe*>(dev_code),
                  lc, g, false, 2);
}

uint64_t mlh_merkle_layers_bytes(uint64_t leaves) { return leaves ? (2 * leaves - 1) * 32 : 0; }

static mlh_status read_root(mlh_ctx* ctx, const uint8_t* layers, uint64_t leaves, uint8_t out[32]) {
  if (!out) return MLH_OK;
  HIP_TRY(ctx, hipMemcpyAsync(ctx->pinned, layers + (2 * leaves - 2) * 32, 32,
                              hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  memcpy(out, ctx->pinned, 32);
  return MLH_OK;
}

static bool is_pow2(uint64_t x) { return x && !(x & (x - 1)); }

mlh_status mlh_merkle_commit_pairs(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                                   void* dev_layers, uint8_t root_out[32]) {
  if (!ctx || !dev_code || !dev_layers) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_code < 1 || log_code > 40)
    return fail(ctx, MLH_ERR_NOT_POW2, "Data length must be a power of two");
  const uint64_t L = 1ull << (log_code - 1);
  uint8_t* layers = reinterpret_cast<uint8_t*>(dev_layers);
  HIP_TRY(ctx, launch_commit_pairs(reinterpret_cast<const fe*>(dev_code), L, layers, ctx->stream));
  return read_root(ctx, layers, L, root_out);
}

mlh_status mlh_merkle_commit(mlh_ctx* ctx, const void* dev_items, uint64_t item_len,
                             uint64_t count, void* dev_layers, uint8_t root_out[32]) {
  if (!ctx || !dev_items || !dev_layers) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (!is_pow2(count)) return fail(ctx, MLH_ERR_NOT_POW2, "Data length must be a power of two");
  uint8_t* layers = reinterpret_cast<uint8_t*>(dev_layers);
  HIP_TRY(ctx, launch_leaf_bytes(reinterpret_cast<const uint8_t*>(dev_items), item_len, count,
                                 layers, ctx->stream));
  HIP_TRY(ctx, launch_merkle_levels(layers, count, ctx->stream));
  return read_root(ctx, layers, count, root_out);
}

mlh_status mlh_merkle_batch_commit(mlh_ctx* ctx, const void* dev_items, uint64_t item_len,
                                   uint32_t m, uint64_t count, void* dev_layers,
                                   uint8_t root_out[32]) {
  if (!ctx || !dev_items || !dev_layers) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (m == 0) return fail(ctx, MLH_ERR_INVALID, "Data must not be empty");
  if (!is_pow2(count))
    return fail(ctx, MLH_ERR_NOT_POW2, "Each batch length must be a power of two");
  uint8_t* layers = reinterpret_cast<uint8_t*>(dev_layers);
  HIP_TRY(ctx, launch_leaf_batch(reinterpret_cast<const uint8_t*>(dev_items), item_len,
                                 item_len * count, m, count, layers, ctx->stream));
  HIP_TRY(ctx, launch_merkle_levels(layers, count, ctx->stream));
  return read_root(ctx, layers, count, root_out);
}

// Fold twiddles gen_pows[len - e] = g^(-e), e < len = 2^log_len (fri/mod.rs:106-110),
// as T_lo[e mod 4096] * T_hi[e / 4096] of g^-1.
static mlh_status fold_tables_g(mlh_ctx* ctx, u128 g, uint32_t log_len, const fe** tlo,
                                const fe** thi) {
  const u128 ginv = h_inv(g);
  MLH_TRY(get_table(ctx, ginv, 4096, 1, tlo));
  MLH_TRY(get_table(ctx, h_pow(ginv, 4096), hi_count(log_len), 1, thi));
  return MLH_OK;
}
static mlh_status fold_tables(mlh_ctx* ctx, uint32_t log_domain, const fe** tlo, const fe** thi) {
  return fold_tables_g(ctx, h_pow2_generator(log_domain), log_domain, tlo, thi);
}

// Every fold layer's twiddles of the domain of g (order 2^L) in one cached
// table (fri.hip fold_layer_table): a pair's twiddle is one 16-B load instead
// of a product of two table entries.  Domains up to 2^25 (512 MiB, the size of
// the reference's own gen_pows table there); *out = nullptr above that.
#ifndef MLH_FOLD_TABLE_MAX_LOG
#define MLH_FOLD_TABLE_MAX_LOG 25
#endif
static mlh_status fold_layer_table(mlh_ctx* ctx, u128 g, uint32_t L, const fe** out) {
  *out = nullptr;
  if (L < 2 || L > MLH_FOLD_TABLE_MAX_LOG) return MLH_OK;
  const TableKey key{h_inv(g), (1ull << L) - 1, 0, 2};
  if (table_hit(ctx, key, out)) return MLH_OK;
  fe* d = nullptr;
  MLH_TRY(table_alloc(ctx, key, ((1ull << L) - 1) * sizeof(fe), &d));
  const fe *tlo, *thi;  // (after the big allocation: it cannot evict these)
  MLH_TRY(fold_tables_g(ctx, g, L, &tlo, &thi));
  HIP_TRY(ctx, launch_fold_layer_table(d, tlo, thi, L, ctx->stream));
  *out = d;
  return MLH_OK;
}

mlh_status mlh_fri_fold(mlh_ctx* ctx, const void* dev_layer, uint32_t log_layer, uint32_t k,
                        uint32_t log_domain, const uint8_t r[16], void* dev_next) {
  if (!ctx || !dev_layer || !dev_next || !r) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_layer < 1 || log_domain > 40 || log_layer + k != log_domain)
    return fail(ctx, MLH_ERR_INVALID, "layer size must be 2^(log_domain - k)");
  const fe *tlo, *thi;
  MLH_TRY(fold_tables(ctx, log_domain, &tlo, &thi));
  HIP_TRY(ctx, launch_fri_fold(reinterpret_cast<const fe*>(dev_layer), 1ull << log_layer,
                               reinterpret_cast<fe*>(dev_next), to_fe(h_load(r)), tlo, thi, k,
                               1ull << log_domain, ctx->stream));
  return MLH_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// FRI prover (FriProverData)
// ---------------------------------------------------------------------------
struct FriLayer {
  const fe* values = nullptr;  // 2^log_n values (pairs i, i + n/2)
  void* owned_values = nullptr;
  uint8_t* tree = nullptr;  // 2L-1 digests, L = n/2
  uint32_t log_n = 0;
  uint8_t root[32];
};

struct mlh_fri_prover {
  mlh_ctx* ctx;
  uint32_t log_code;
  // gen_pows of the reference's FriProverData calls (fri/mod.rs:58,79,136,261):
  // a geometric table of 2^log_gp powers of gp_gen; fold twiddle
  // gen_pows[len - i 2^k] = gp_gen^(-i 2^k).  Default: the code's domain.
  u128 gp_gen = 0;
  uint32_t log_gp = 0;
  std::vector<FriLayer> layers;
  bool has_last = false;
  uint8_t last[16];
  ~mlh_fri_prover() {
    for (auto& l : layers) {
      pool_free(ctx, l.owned_values);
      pool_free(ctx, l.tree);
    }
  }
};

// gen_pows = [g^0 .. g^(2^log_gp - 1)] (NttField::pow_2_generator_powers,
// ntt/mod.rs:18-28, or any generator of order exactly 2^log_gp).  The
// reference indexes gen_pows[len - i 2^k] with i 2^k < 2^(log_code - 1), so a
// table shorter than half the code underflows its index (a panic there).
static mlh_status set_gen_pows(mlh_ctx* ctx, mlh_fri_prover* p, const uint8_t* gen,
                               uint32_t log_gp) {
  if (!gen) {
    p->gp_gen = h_pow2_generator(p->log_code);
    p->log_gp = p->log_code;
    return MLH_OK;
  }
  if (log_gp > 40 || log_gp + 1 < p->log_code)
    return fail(ctx, MLH_ERR_INVALID, "gen_pows shorter than half the code");
  const u128 g = h_load(gen);
  if (!check_generator(g, log_gp))
    return fail(ctx, MLH_ERR_BAD_GENERATOR, "gen_pows[1] must have order exactly gen_pows.len()");
  p->gp_gen = g;
  p->log_gp = log_gp;
  return MLH_OK;
}

extern "C" {

mlh_status mlh_fri_prover_init(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                               mlh_transcript* tr, mlh_fri_prover** out) {
  return mlh_fri_prover_init_gp(ctx, dev_code, log_code, nullptr, 0, tr, out);
}

mlh_status mlh_fri_prover_init_gp(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                                  const uint8_t gen_pows_1[16], uint32_t log_gen_pows,
                                  mlh_transcript* tr, mlh_fri_prover** out) {
  if (!ctx || !dev_code || !tr || !out) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_code < 1 || log_code > 40)
    return fail(ctx, MLH_ERR_NOT_POW2, "Input size must be a power of two");
  std::unique_ptr<mlh_fri_prover> p(new mlh_fri_prover());
  p->ctx = ctx;
  p->log_code = log_code;
  MLH_TRY(set_gen_pows(ctx, p.get(), gen_pows_1, log_gen_pows));
  FriLayer l0;
  l0.values = reinterpret_cast<const fe*>(dev_code);
  l0.log_n = log_code;
  const uint64_t L = 1ull << (log_code - 1);
  void* tree;
  MLH_TRY(pool_alloc(ctx, mlh_merkle_layers_bytes(L), &tree));
  l0.tree = reinterpret_cast<uint8_t*>(tree);
  p->layers.push_back(l0);
  MLH_TRY(mlh_merkle_commit_pairs(ctx, dev_code, log_code, tree, p->layers[0].root));
  mlh_transcript_absorb(tr, p->layers[0].root, 32);
  *out = p.release();
  return MLH_OK;
}

}  // extern "C"

// fold_step (fri/mod.rs:79-134) with the table (gen, log_gp): twiddle
// gen_pows[len - i 2^k] = gen^(-(i 2^k) mod len).  The reference accepts any k
// whose indices stay in the table -- (n/2 - 1) 2^k <= len, else its usize index
// underflows (a panic, MLH_ERR_INVALID here); its callers pass k in sequence.
static mlh_status fold_step_impl(mlh_ctx* ctx, mlh_fri_prover* p, u128 gen, uint32_t log_gp,
                                 uint32_t k, const uint8_t r[16], mlh_transcript* tr) {
  // a batched prover's inner view has no tree before batched_fold_step, nor
  // after a step that produced the last element directly (log_code 2); the
  // reference panics on merkle_trees.last().unwrap() there
  if (p->layers.empty())
    return fail(ctx, MLH_ERR_INVALID, "fold_step before any tree (batched_fold_step not applied)");
  const FriLayer& cur = p->layers.back();
  const uint32_t log_n = cur.log_n;  // n = 2 * pairs
  const uint64_t blowup = 1ull << MLH_LOG_BLOWUP;
  if ((1ull << log_n) <= blowup) return MLH_OK;  // fri/mod.rs:83-85
  // (after the last element, the reference folds its last tree again and
  // re-absorbs the element: layers.back() is still that tree here, too)
  const uint64_t half_n = 1ull << (log_n - 1);
  // (log space first: half_n - 1 < 2^(log_n - 1), so with (log_n - 1) + k <= 62
  // the shift cannot wrap 64 bits; beyond it the product exceeds any table)
  if (k > 40 || (log_n - 1) + k > 62 || ((half_n - 1) << k) > (1ull << log_gp))
    return fail(ctx, MLH_ERR_INVALID, "gen_pows index len - i*2^k underflows (fri/mod.rs:106-110)");
  const fe *tlo, *thi;
  MLH_TRY(fold_tables_g(ctx, gen, log_gp, &tlo, &thi));
  const fe rr = to_fe(h_load(r));
  FriLayer nx;
  nx.log_n = log_n - 1;
  PoolBuf vb(ctx), tb(ctx);  // released into the new layer on success only
  MLH_TRY(vb.alloc(half_n * sizeof(fe)));
  void* vals = vb.p;
  nx.values = reinterpret_cast<const fe*>(vals);
  if (half_n == blowup) {  // fri/mod.rs:116-126
    HIP_TRY(ctx, launch_fri_fold(cur.values, 1ull << log_n, reinterpret_cast<fe*>(vals), rr, tlo,
                                 thi, k, 1ull << log_gp, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->pinned, vals, 32, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (memcmp(ctx->pinned, ctx->pinned + 16, 16) != 0)
      return fail(ctx, MLH_ERR_NOT_RS_CODE, "not an RS code");
    memcpy(p->last, ctx->pinned, 16);
    p->has_last = true;
    mlh_transcript_absorb(tr, p->last, 16);
    return MLH_OK;
  }
  const uint64_t L = half_n / 2;
  MLH_TRY(tb.alloc(mlh_merkle_layers_bytes(L)));
  nx.tree = tb.as<uint8_t>();
  HIP_TRY(ctx, launch_fri_fold_commit(cur.values, 1ull << log_n, reinterpret_cast<fe*>(vals),
                                      nx.tree, rr, tlo, thi, k, 1ull << log_gp,
                                      ctx->stream));
  MLH_TRY(read_root(ctx, nx.tree, L, nx.root));
  nx.owned_values = vb.release();
  tb.release();
  p->layers.push_back(nx);
  mlh_transcript_absorb(tr, p->layers.back().root, 32);
  return MLH_OK;
}

extern "C" {

mlh_status mlh_fri_prover_fold_step(mlh_ctx* ctx, mlh_fri_prover* p, uint32_t k,
                                    const uint8_t r[16], mlh_transcript* tr) {
  if (!ctx || !p || !r || !tr) return fail(ctx, MLH_ERR_INVALID, "null argument");
  return fold_step_impl(ctx, p, p->gp_gen, p->log_gp, k, r, tr);
}

mlh_status mlh_fri_prover_fold_step_gp(mlh_ctx* ctx, mlh_fri_prover* p, const uint8_t gen_pows_1[16],
                                       uint32_t log_gen_pows, uint32_t k, const uint8_t r[16],
                                       mlh_transcript* tr) {
  if (!ctx || !p || !gen_pows_1 || !r || !tr) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_gen_pows < 1 || log_gen_pows > 40) return fail(ctx, MLH_ERR_INVALID, "gen_pows length");
  const u128 g = h_load(gen_pows_1);
  if (!check_generator(g, log_gen_pows))
    return fail(ctx, MLH_ERR_BAD_GENERATOR, "gen_pows[1] must have order exactly gen_pows.len()");
  return fold_step_impl(ctx, p, g, log_gen_pows, k, r, tr);
}

}  // extern "C"

// FriProverData::fold (fri/mod.rs:136-145) with the transcript on the device:
// every round's challenge is derived on the GPU from the root just written,
// so the whole commit phase is one stream of kernels with a single sync at
// the end; the host transcript then replays the same absorbs (root_0,
// root_1, ..., last element) and ends in the identical state.
static_assert(sizeof(DevSha) == sizeof(HostSha256), "transcript layouts differ");

// Device-side commit loop state: [transcript | r_0..r_steps | last (16) |
// flag (16) | batch root (32) | fingerprint r (16) | roots 32 x (steps + 1) |
// polys 32 x steps | prev (16) | extra (16 x n_extra)].
struct FriDevLoop {
  mlh_ctx* ctx;
  mlh_fri_prover* p;
  const fe *tlo = nullptr, *thi = nullptr;
  const fe* twt = nullptr;  // every fold layer's twiddles (fold_layer_table), or nullptr
  PoolBuf scratch;
  size_t off_r = 128, off_last = 0, off_flag = 0, off_broot = 0, off_fr = 0, off_roots = 0,
         off_polys = 0, off_prev = 0, off_extra = 0;
  bool done = false;
  // batched mode: the m codes ([m][N]) and the batch-layer tree
  const fe* codes = nullptr;
  uint32_t m = 0;
  PoolBuf btree;
  explicit FriDevLoop(mlh_ctx* c, mlh_fri_prover* pr) : ctx(c), p(pr), scratch(c), btree(c) {}
  uint8_t* sb() const { return scratch.as<uint8_t>(); }
  DevSha* dt() const { return reinterpret_cast<DevSha*>(sb()); }
  fe* r(uint32_t k) const { return reinterpret_cast<fe*>(sb() + off_r) + k; }
  uint8_t* root(uint32_t t) const { return sb() + off_roots + 32 * t; }
  fe* poly(uint32_t k) const { return reinterpret_cast<fe*>(sb() + off_polys) + 2 * k; }
  fe* prev() const { return reinterpret_cast<fe*>(sb() + off_prev); }
  fe* fr() const { return reinterpret_cast<fe*>(sb() + off_fr); }
  fe* extra() const { return reinterpret_cast<fe*>(sb() + off_extra); }

  mlh_status layout(uint32_t log_code, const mlh_transcript* tr, size_t n_extra = 0) {
    const uint32_t steps = log_code - MLH_LOG_BLOWUP;
    off_last = off_r + 16 * (steps + 1);
    off_flag = off_last + 16;
    off_broot = off_flag + 16;
    off_fr = off_broot + 32;
    off_roots = off_fr + 16;
    off_polys = off_roots + 32 * (steps + 1);
    off_prev = off_polys + 32 * steps;
    off_extra = off_prev + 16;
    MLH_TRY(scratch.alloc(off_extra + 16 * (n_extra ? n_extra : 1)));
    if (!p->log_gp) {
      p->gp_gen = h_pow2_generator(log_code);
      p->log_gp = log_code;
    }
    if (p->log_gp == log_code) MLH_TRY(fold_layer_table(ctx, p->gp_gen, log_code, &twt));
    MLH_TRY(fold_tables_g(ctx, p->gp_gen, p->log_gp, &tlo, &thi));
    memcpy(ctx->pinned, &tr->sha, sizeof(DevSha));
    HIP_TRY(ctx, hipMemcpyAsync(dt(), ctx->pinned, sizeof(DevSha), hipMemcpyHostToDevice,
                                ctx->stream));
    return MLH_OK;
  }

  // BatchedFriProverData::init (batched_fri.rs:41-98): batch layer over the
  // m codes' RS pairs, absorb its root, fingerprint_r = next_challenge(),
  // absorb LE16(fingerprint_r); r_0 = next_challenge() if challenge_r0.
  mlh_status init_batched(const fe* dev_codes, uint32_t num_codes, uint32_t log_code,
                          const mlh_transcript* tr, bool challenge_r0, size_t n_extra = 0) {
    MLH_TRY(layout(log_code, tr, n_extra));
    codes = dev_codes;
    m = num_codes;
    const uint64_t N = 1ull << log_code, L = N / 2;
    MLH_TRY(btree.alloc(mlh_merkle_layers_bytes(L)));
    uint8_t* bt = btree.as<uint8_t>();
    HIP_TRY(ctx, launch_batch_pairs_leaves(codes, m, N, bt, ctx->stream));
    HIP_TRY(ctx, launch_merkle_levels(bt, L, ctx->stream, RootAbsorb{dt(), fr(), sb() + off_broot}));
    HIP_TRY(ctx, launch_transcript_absorb(dt(), reinterpret_cast<const uint8_t*>(fr()), 16,
                                          challenge_r0 ? r(0) : nullptr, ctx->stream));
    return MLH_OK;
  }

  // batched_fold_step (batched_fri.rs:100-176): fold the fingerprinted pairs
  // with r at rp into the inner prover's first layer (or the last element).
  mlh_status step_batched(const fe* rp, bool challenge_next, const fe* poly_next = nullptr) {
    const uint32_t L = p->log_code;
    const uint64_t N = 1ull << L, half_n = N / 2;
    void* vals;
    MLH_TRY(pool_alloc(ctx, half_n * sizeof(fe), &vals));
    if (half_n == (1ull << MLH_LOG_BLOWUP)) {
      HIP_TRY(ctx, launch_batched_fold_leaves(codes, m, N, fr(), rp, tlo, thi,
                                              reinterpret_cast<fe*>(vals), nullptr, ctx->stream));
      HIP_TRY(ctx, launch_fri_last(reinterpret_cast<const fe*>(vals), dt(),
                                   reinterpret_cast<uint32_t*>(sb() + off_flag),
                                   reinterpret_cast<fe*>(sb() + off_last), ctx->stream));
      pool_free(ctx, vals);
      done = true;
      return MLH_OK;
    }
    FriLayer nx;
    nx.log_n = L - 1;
    nx.owned_values = vals;
    nx.values = reinterpret_cast<const fe*>(vals);
    const uint64_t leaves = half_n / 2;
    void* tree;
    MLH_TRY(pool_alloc(ctx, mlh_merkle_layers_bytes(leaves), &tree));
    nx.tree = reinterpret_cast<uint8_t*>(tree);
    p->layers.push_back(nx);
    HIP_TRY(ctx, launch_batched_fold_leaves(codes, m, N, fr(), rp, tlo, thi,
                                            reinterpret_cast<fe*>(vals), nx.tree, ctx->stream));
    HIP_TRY(ctx, launch_merkle_levels(nx.tree, leaves, ctx->stream,
                                      RootAbsorb{dt(), challenge_next ? r(1) : nullptr, root(0), poly_next}));
    return MLH_OK;
  }

  // poly0 (optional): 32 bytes absorbed after root 0, before its challenge;
  // n_extra: 16-byte slots at extra()
  mlh_status init(const void* dev_code, uint32_t log_code, const mlh_transcript* tr,
                  bool challenge_after_root0, const fe* poly0 = nullptr, size_t n_extra = 0) {
    MLH_TRY(layout(log_code, tr, n_extra));
    return init_after_layout(dev_code, log_code, challenge_after_root0, poly0);
  }
  // init's commit of layer 0, after layout() (whose extra() slots the caller
  // may fill first)
  mlh_status init_after_layout(const void* dev_code, uint32_t log_code, bool challenge_after_root0,
                               const fe* poly0) {
    FriLayer l0;
    l0.values = reinterpret_cast<const fe*>(dev_code);
    l0.log_n = log_code;
    const uint64_t L = 1ull << (log_code - 1);
    void* tree;
    MLH_TRY(pool_alloc(ctx, mlh_merkle_layers_bytes(L), &tree));
    l0.tree = reinterpret_cast<uint8_t*>(tree);
    p->layers.push_back(l0);
    HIP_TRY(ctx, launch_commit_pairs(
                     l0.values, L, l0.tree, ctx->stream,
                     RootAbsorb{dt(), challenge_after_root0 ? r(0) : nullptr, root(0), poly0}));
    return MLH_OK;
  }

  // fold_step k with the challenge at rp (device); absorbs the new root (or
  // the last element) and (poly_next) 32 more bytes; writes next_challenge()
  // to r(k + 1) if challenge_next.
  // job (optional): a PCS round run by an extra workgroup of the fold launch
  mlh_status step(uint32_t k, const fe* rp, bool challenge_next, const fe* poly_next = nullptr,
                  const PcsJob* job = nullptr) {
    if (done) return MLH_OK;
    const FriLayer cur = p->layers.back();
    const uint32_t log_n = cur.log_n;
    if ((1ull << log_n) <= (1ull << MLH_LOG_BLOWUP)) return MLH_OK;
    const uint64_t half_n = 1ull << (log_n - 1);
    void* vals;
    MLH_TRY(pool_alloc(ctx, half_n * sizeof(fe), &vals));
    if (half_n == (1ull << MLH_LOG_BLOWUP)) {  // fri/mod.rs:116-126
      if (job || poly_next) {
        pool_free(ctx, vals);
        return fail(ctx, MLH_ERR_INVALID, "no PCS round after the last FRI fold");
      }
      HIP_TRY(ctx, launch_fri_fold(cur.values, 1ull << log_n, reinterpret_cast<fe*>(vals), fe{},
                                   tlo, thi, k, 1ull << p->log_gp, ctx->stream, ShardMap(), rp));
      HIP_TRY(ctx, launch_fri_last(reinterpret_cast<const fe*>(vals), dt(),
                                   reinterpret_cast<uint32_t*>(sb() + off_flag),
                                   reinterpret_cast<fe*>(sb() + off_last), ctx->stream));
      pool_free(ctx, vals);
      done = true;
      return MLH_OK;
    }
    FriLayer nx;
    nx.log_n = log_n - 1;
    nx.owned_values = vals;
    nx.values = reinterpret_cast<const fe*>(vals);
    const uint64_t L = half_n / 2;
    void* tree;
    MLH_TRY(pool_alloc(ctx, mlh_merkle_layers_bytes(L), &tree));
    nx.tree = reinterpret_cast<uint8_t*>(tree);
    p->layers.push_back(nx);
    const uint32_t t = (uint32_t)p->layers.size() - 1;
    const uint32_t Lg = p->log_gp;  // the layer table's part for fold k (pairs of a 2^(Lg - k) layer)
    const fe* twl = twt && log_n + k == Lg ? twt + ((1ull << Lg) - (1ull << (Lg - k))) : nullptr;
    HIP_TRY(ctx, launch_fri_fold_commit(
                     cur.values, 1ull << log_n, reinterpret_cast<fe*>(vals), nx.tree, fe{}, tlo,
                     thi, k, 1ull << p->log_gp, ctx->stream, ShardMap(), rp,
                     RootAbsorb{dt(), challenge_next ? r(k + 1) : nullptr, root(t), poly_next}, job,
                     twl));
    return MLH_OK;
  }

  // one sync: challenges, last element, RS flag, roots (+ polys_bytes of
  // sumcheck polys); then the cooperative kernels' failure word
  mlh_status finish(size_t polys_bytes) {
    if (!done) return fail(ctx, MLH_ERR_INVALID, "fold produced no last element");
    const size_t nt = p->layers.size();
    const size_t bytes = off_polys - off_r + polys_bytes;
    if (bytes > kPinStage) return fail(ctx, MLH_ERR_INVALID, "proof staging too large");
    HIP_TRY(ctx, hipMemcpyAsync(ctx->pinned, sb() + off_r, bytes, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    MLH_TRY(device_check(ctx));
    const uint8_t* h = ctx->pinned;
    for (size_t t = 0; t < nt; ++t)
      memcpy(p->layers[t].root, h + (off_roots - off_r) + 32 * t, 32);
    uint32_t flag;
    memcpy(&flag, h + (off_flag - off_r), 4);
    if (flag) return fail(ctx, MLH_ERR_NOT_RS_CODE, "not an RS code");
    memcpy(p->last, h + (off_last - off_r), 16);
    p->has_last = true;
    return MLH_OK;
  }
  // the device's challenge slot k, as copied back by finish()
  const uint8_t* host_r(uint32_t k) const { return ctx->pinned + 16 * k; }
  const uint8_t* host_polys() const { return ctx->pinned + (off_polys - off_r); }
  const uint8_t* host_broot() const { return ctx->pinned + (off_broot - off_r); }
  const uint8_t* host_fr() const { return ctx->pinned + (off_fr - off_r); }
};

// FriProverData::fold (fri/mod.rs:136-145) with the transcript on the device:
// every round's challenge is derived on the GPU from the root just written,
// so the whole commit phase is one stream of kernels with a single sync at
// the end; the host transcript then replays the same absorbs (root_0,
// root_1, ..., last element) and ends in the identical state.
static mlh_status fri_fold_device(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                                  const uint8_t* gen, uint32_t log_gp, mlh_transcript* tr,
                                  mlh_fri_prover** out) {
  if (!ctx || !dev_code || !tr || !out) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_code < 2 || log_code > 40)
    return fail(ctx, log_code < 2 ? MLH_ERR_INVALID : MLH_ERR_NOT_POW2,
                "fold needs 4 <= code length <= 2^40");
  std::unique_ptr<mlh_fri_prover> p(new mlh_fri_prover());
  p->ctx = ctx;
  p->log_code = log_code;
  MLH_TRY(set_gen_pows(ctx, p.get(), gen, log_gp));
  FriDevLoop lp(ctx, p.get());
  device_arm(ctx);
  MLH_TRY(lp.init(dev_code, log_code, tr, true));
  const uint32_t steps = log_code - MLH_LOG_BLOWUP;
  for (uint32_t k = 0; k < steps; ++k) MLH_TRY(lp.step(k, lp.r(k), true));
  MLH_TRY(lp.finish(0));
  // host replay: root_t, then the challenge r_t the device drew from it
  ReplayCheck rc(ctx, tr);
  for (size_t t = 0; t < p->layers.size(); ++t) {
    rc.absorb(p->layers[t].root, 32);
    rc.expect(lp.host_r((uint32_t)t));
  }
  rc.absorb(p->last, 16);
  MLH_TRY(rc.status());
  *out = p.release();
  return MLH_OK;
}

extern "C" {

mlh_status mlh_fri_prover_fold(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                               mlh_transcript* tr, mlh_fri_prover** out) {
  return fri_fold_device(ctx, dev_code, log_code, nullptr, 0, tr, out);
}

mlh_status mlh_fri_prover_fold_gp(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                                  const uint8_t gen_pows_1[16], uint32_t log_gen_pows,
                                  mlh_transcript* tr, mlh_fri_prover** out) {
  if (!gen_pows_1) return fail(ctx, MLH_ERR_INVALID, "null argument");
  return fri_fold_device(ctx, dev_code, log_code, gen_pows_1, log_gen_pows, tr, out);
}

uint32_t mlh_fri_prover_num_trees(const mlh_fri_prover* p) {
  return p ? (uint32_t)p->layers.size() : 0;
}

mlh_status mlh_fri_prover_roots(const mlh_fri_prover* p, uint8_t* roots_out) {
  if (!p || !roots_out) return MLH_ERR_INVALID;
  for (size_t i = 0; i < p->layers.size(); ++i) memcpy(roots_out + 32 * i, p->layers[i].root, 32);
  return MLH_OK;
}

mlh_status mlh_fri_prover_last_element(const mlh_fri_prover* p, uint8_t out[16]) {
  if (!p || !out || !p->has_last) return MLH_ERR_INVALID;
  memcpy(out, p->last, 16);
  return MLH_OK;
}

void mlh_fri_prover_destroy(mlh_fri_prover* p) { delete p; }

}  // extern "C"

// Gather opened query records from the device-resident layers/trees.
struct QueryTree {
  const fe* values;
  const uint8_t* tree;
  uint32_t log_n;  // layer values
};
// The layer table travels in the kernel arguments (up to 40 layers, ~1 KB)
// with, for a proof's 128 queries, the indices (1 KB): the query phase is then
// one launch and one D2H copy, no host-to-device copies.
constexpr uint32_t kMaxQueryTrees = 40;
struct QueryTrees {
  QueryTree t[kMaxQueryTrees];
  uint32_t n;
};
static_assert(MLH_NUM_QUERIES == 128, "QueryIdx holds 128 indices");
static_assert(sizeof(QueryTrees) + sizeof(mlh::QueryIdx) + 64 <= 4096, "kernel argument budget");

// d_idx: device indices (openings of more than 128 queries), else idx.v
__global__ void gather_queries_kernel(const QueryTrees trees, const mlh::QueryIdx idx,
                                      const uint64_t* __restrict__ d_idx, uint32_t nq,
                                      uint64_t qbytes, uint64_t base, uint8_t* __restrict__ out) {
  const uint32_t q = blockIdx.x;
  if (q >= nq) return;
  const uint64_t iq = d_idx ? d_idx[q] : idx.v[q];
  // record offsets per tree
  uint64_t off = base;
  for (uint32_t t = 0; t < trees.n; ++t) {
    const QueryTree T = trees.t[t];
    const uint64_t half = 1ull << (T.log_n - 1);  // leaves
    const uint64_t i = iq % half;                   // fri/mod.rs:169-170
    const uint32_t depth = T.log_n - 1;
    uint8_t* rec = out + q * qbytes + off;
    if (threadIdx.x == 0) {
      fe_store(reinterpret_cast<fe*>(rec), fe_load(T.values + i));
      fe_store(reinterpret_cast<fe*>(rec + 16), fe_load(T.values + i + half));
    }
    // siblings: level l node (i >> l) ^ 1, level l starts at sum_{j<l} half>>j
    for (uint32_t l = threadIdx.x; l < depth; l += blockDim.x) {
      const uint64_t lvl_off = 2 * half - (2 * half >> l);
      const uint64_t sib = ((i >> l) ^ 1ull);
      const uint4* src = reinterpret_cast<const uint4*>(T.tree + (lvl_off + sib) * 32);
      uint4* dst = reinterpret_cast<uint4*>(rec + 32 + (uint64_t)l * 32);
      dst[0] = src[0];
      dst[1] = src[1];
    }
    off += 32ull * (1 + depth);
  }
}

// Pinned host staging for a query phase: the gather kernels write the
// records straight into it (zero-copy over PCIe, ~1.3 MB for a 2^25 code: no
// device buffer, no copy launch), and it holds indices beyond 128.  Grow-only;
// a caller's stream sync ends every use before the next one.  Allocated
// non-coherent (explicitly; what flags 0 gives under the default
// HIP_HOST_COHERENT=0): the kernels' writes become visible to the host only
// at the end of the kernel, so EVERY host read of records a kernel wrote here
// must follow a sync of the stream that ran it (each caller syncs ctx->stream
// before copying records out).
static mlh_status query_stage(mlh_ctx* ctx, size_t bytes, uint8_t** out) {
  if (bytes > ctx->qstage_bytes) {
    if (ctx->qstage) HIP_TRY(ctx, hipHostFree(ctx->qstage));
    ctx->qstage = nullptr;
    ctx->qstage_bytes = 0;
    void* h = nullptr;
    HIP_TRY(ctx, hipHostMalloc(&h, bytes, hipHostMallocNonCoherent));
    ctx->qstage = reinterpret_cast<uint8_t*>(h);
    ctx->qstage_bytes = bytes;
  }
  *out = ctx->qstage;
  return MLH_OK;
}

// Launch the per-tree gathers of p's layers into records at d_out (qbytes
// each, this part starting at byte `base` of a record; device or pinned host
// memory); indices in idx.v, or
// at d_idx (device) when nq > 128.
static mlh_status gather_queries_dev(mlh_ctx* ctx, const mlh_fri_prover* p, const mlh::QueryIdx& idx,
                                     const uint64_t* d_idx, uint32_t nq, uint64_t qbytes,
                                     uint64_t base, uint8_t* d_out) {
  const uint32_t nt = (uint32_t)p->layers.size();
  if (nt == 0 || nq == 0) return MLH_OK;
  if (nt > kMaxQueryTrees) return fail(ctx, MLH_ERR_INVALID, "more than 40 FRI layers");
  if (nq > MLH_NUM_QUERIES && !d_idx) return fail(ctx, MLH_ERR_INVALID, "query indices not on the device");
  QueryTrees qt;
  qt.n = nt;
  for (uint32_t t = 0; t < nt; ++t)
    qt.t[t] = QueryTree{p->layers[t].values, p->layers[t].tree, p->layers[t].log_n};
  hipLaunchKernelGGL(gather_queries_kernel, dim3(nq), dim3(64), 0, ctx->stream, qt, idx,
                     nq > MLH_NUM_QUERIES ? d_idx : nullptr, nq, qbytes, base, d_out);
  HIP_TRY(ctx, hipGetLastError());
  return MLH_OK;
}

static mlh_status gather_queries(mlh_ctx* ctx, const mlh_fri_prover* p, const uint64_t* idx,
                                 uint32_t nq, uint8_t* host_out) {
  const uint64_t qbytes = mlh_fri_query_bytes(p->log_code);
  const size_t off_out = nq > MLH_NUM_QUERIES ? 8ull * nq : 0;
  uint8_t* h;
  MLH_TRY(query_stage(ctx, off_out + nq * qbytes, &h));
  mlh::QueryIdx qi;
  memset(&qi, 0, sizeof(qi));
  PoolBuf didx(ctx);
  if (nq > MLH_NUM_QUERIES) {
    memcpy(h, idx, 8ull * nq);
    MLH_TRY(didx.alloc(nq * sizeof(uint64_t)));
    HIP_TRY(ctx, hipMemcpyAsync(didx.p, h, nq * sizeof(uint64_t), hipMemcpyHostToDevice,
                                ctx->stream));
  } else {
    memcpy(qi.v, idx, 8ull * nq);
  }
  MLH_TRY(gather_queries_dev(ctx, p, qi, didx.as<uint64_t>(), nq, qbytes, 0, h + off_out));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  memcpy(host_out, h + off_out, nq * qbytes);
  return MLH_OK;
}

// FriProof::prove tail (fri/mod.rs:266-284): query indices from the
// transcript, openings, last_random.
static mlh_status fri_queries(mlh_ctx* ctx, mlh_fri_prover* p, mlh_transcript* tr,
                              mlh_fri_proof* proof) {
  const uint64_t domain = 1ull << p->log_code;
  proof->log_code = p->log_code;
  proof->num_trees = (uint32_t)p->layers.size();
  proof->num_queries = MLH_NUM_QUERIES;
  std::vector<uint64_t> idx(MLH_NUM_QUERIES);
  for (int q = 0; q < MLH_NUM_QUERIES; ++q) {
    uint8_t rnd[32];
    mlh_transcript_random(tr, rnd);
    uint64_t u;
    memcpy(&u, rnd, 8);
    idx[q] = u % (domain / 2);
    uint8_t le[8];
    memcpy(le, &idx[q], 8);
    mlh_transcript_absorb(tr, le, 8);
  }
  if (proof->query_indices) memcpy(proof->query_indices, idx.data(), idx.size() * 8);
  if (proof->commitments) mlh_fri_prover_roots(p, proof->commitments);
  memcpy(proof->last_elem, p->last, 16);
  mlh_transcript_random(tr, proof->last_random);
  if (proof->queries) MLH_TRY(gather_queries(ctx, p, idx.data(), MLH_NUM_QUERIES, proof->queries));
  return MLH_OK;
}

extern "C" {

mlh_status mlh_fri_prover_open_query(mlh_ctx* ctx, const mlh_fri_prover* p, uint64_t index,
                                     uint8_t* out) {
  if (!ctx || !p || !out) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (index >= (1ull << (p->log_code - 1))) return fail(ctx, MLH_ERR_INVALID, "index out of bounds");
  return gather_queries(ctx, p, &index, 1, out);
}

mlh_status mlh_fri_prover_open_queries(mlh_ctx* ctx, const mlh_fri_prover* p,
                                       const uint64_t* idx, uint32_t nq, uint8_t* out) {
  if (!ctx || !p || !idx || !out) return fail(ctx, MLH_ERR_INVALID, "null argument");
  for (uint32_t q = 0; q < nq; ++q)
    if (idx[q] >= (1ull << (p->log_code - 1))) return fail(ctx, MLH_ERR_INVALID, "index out of bounds");
  if (nq == 0) return MLH_OK;
  return gather_queries(ctx, p, idx, nq, out);
}

// ---------------------------------------------------------------------------
// sharded building blocks (dist.hip; orchestration in tests/dist_spec.py)
// ---------------------------------------------------------------------------
mlh_status mlh_shard_ntt_cross(mlh_ctx* ctx, const void* dev_in, void* dev_out, uint32_t log_n,
                               uint32_t log_p, uint32_t rank, const uint8_t gen[16], int inverse) {
  if (!ctx || !dev_in || !dev_out || !gen) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_p < 1 || log_p > 4 || log_n < 2 * log_p || log_n > 40)
    return fail(ctx, MLH_ERR_INVALID, "need 1 <= log_p <= 4 and log_n >= 2 log_p");
  if (rank >> log_p) return fail(ctx, MLH_ERR_INVALID, "rank out of range");
  if (dev_in == dev_out) return fail(ctx, MLH_ERR_INVALID, "shard_ntt_cross is out of place");
  const u128 g = h_load(gen);
  if (!check_generator(g, log_n)) return fail(ctx, MLH_ERR_BAD_GENERATOR, "generator order != n");
  const uint64_t P = 1ull << log_p, S = 1ull << (log_n - 2 * log_p);
  const u128 w = inverse ? h_inv(g) : g;
  const fe *tlo, *thi, *wp;
  MLH_TRY(get_table(ctx, w, 4096, 1, &tlo));
  MLH_TRY(get_table(ctx, h_pow(w, 4096), hi_count(log_n - log_p), 1, &thi));
  MLH_TRY(get_table(ctx, h_pow(w, 1ull << (log_n - log_p)), P / 2, 1, &wp));
  const u128 scale = inverse ? h_inv((u128)P) : (u128)1;
  static const char* labs[2][5] = {{"", "shard_dft<1,0>", "shard_dft<2,0>", "shard_dft<3,0>", "shard_dft<4,0>"},
                                   {"", "shard_dft<1,1>", "shard_dft<2,1>", "shard_dft<3,1>", "shard_dft<4,1>"}};
  ProfScope ps(ctx, labs[inverse ? 1 : 0][log_p]);
  HIP_TRY(ctx, launch_shard_dft(reinterpret_cast<const fe*>(dev_in), reinterpret_cast<fe*>(dev_out),
                                S, (uint64_t)rank * S, log_p, inverse != 0, tlo, thi, wp,
                                to_fe(scale), ctx->stream));
  ps.end();
  return MLH_OK;
}

static mlh_status shard_fold_args(mlh_ctx* ctx, const void* a, const void* b, const uint8_t* r,
                                  uint32_t log_local, uint32_t k, uint32_t log_domain,
                                  uint32_t log_s, uint32_t log_p, uint32_t rank, ShardMap* m) {
  if (!ctx || !a || !b || !r) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_domain > 40 || log_p > 4 || (rank >> log_p) || log_local < 1 ||
      log_local + log_p + k != log_domain)
    return fail(ctx, MLH_ERR_INVALID, "local layer must be 2^(log_domain - k - log_p)");
  if (log_s + 1 > log_local && log_p > 0)
    return fail(ctx, MLH_ERR_INVALID, "pairs not local: layer spans < 2 blocks per rank");
  m->log_s = log_p ? log_s : 40;
  m->log_p = log_p;
  m->rank = rank;
  return MLH_OK;
}

mlh_status mlh_shard_fri_fold(mlh_ctx* ctx, const void* dev_layer, uint32_t log_local, uint32_t k,
                              uint32_t log_domain, const uint8_t r[16], void* dev_next,
                              uint32_t log_s, uint32_t log_p, uint32_t rank) {
  ShardMap m;
  MLH_TRY(shard_fold_args(ctx, dev_layer, dev_next, r, log_local, k, log_domain, log_s, log_p,
                          rank, &m));
  const fe *tlo, *thi;
  MLH_TRY(fold_tables(ctx, log_domain, &tlo, &thi));
  HIP_TRY(ctx, launch_fri_fold(reinterpret_cast<const fe*>(dev_layer), 1ull << log_local,
                               reinterpret_cast<fe*>(dev_next), to_fe(h_load(r)), tlo, thi, k,
                               1ull << log_domain, ctx->stream, m));
  return MLH_OK;
}

mlh_status mlh_shard_fri_fold_commit(mlh_ctx* ctx, const void* dev_layer, uint32_t log_local,
                                     uint32_t k, uint32_t log_domain, const uint8_t r[16],
                                     void* dev_next, void* dev_tree, uint32_t log_s,
                                     uint32_t log_p, uint32_t rank) {
  ShardMap m;
  MLH_TRY(shard_fold_args(ctx, dev_layer, dev_next, r, log_local, k, log_domain, log_s, log_p,
                          rank, &m));
  if (!dev_tree) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_local < 2 || (log_p && log_s + 2 > log_local))
    return fail(ctx, MLH_ERR_INVALID, "folded layer's pairs are not local");
  const fe *tlo, *thi;
  MLH_TRY(fold_tables(ctx, log_domain, &tlo, &thi));
  uint8_t* tree = reinterpret_cast<uint8_t*>(dev_tree);
  HIP_TRY(ctx, launch_fri_fold_commit(reinterpret_cast<const fe*>(dev_layer), 1ull << log_local,
                                      reinterpret_cast<fe*>(dev_next), tree, to_fe(h_load(r)),
                                      tlo, thi, k, 1ull << log_domain, ctx->stream, m));
  return MLH_OK;
}

mlh_status mlh_merkle_open_pairs(mlh_ctx* ctx, const void* dev_values, uint32_t log_n,
                                 const void* dev_tree, uint32_t levels, const uint64_t* idx,
                                 uint32_t nq, uint8_t* out) {
  if (!ctx || !dev_values || !dev_tree || (nq && (!idx || !out)))
    return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_n < 1 || log_n > 40 || levels > log_n - 1)
    return fail(ctx, MLH_ERR_INVALID, "levels must be <= log_n - 1");
  const uint64_t half = 1ull << (log_n - 1);
  for (uint32_t q = 0; q < nq; ++q)
    if (idx[q] >= half) return fail(ctx, MLH_ERR_INVALID, "index out of bounds");
  if (nq == 0) return MLH_OK;
  const uint64_t rec = 32ull * (1 + levels);
  PoolBuf didx(ctx), dout(ctx);
  MLH_TRY(didx.alloc(nq * sizeof(uint64_t)));
  MLH_TRY(dout.alloc(nq * rec));
  HIP_TRY(ctx, hipMemcpyAsync(didx.p, idx, nq * sizeof(uint64_t), hipMemcpyHostToDevice,
                              ctx->stream));
  HIP_TRY(ctx, launch_open_pairs(reinterpret_cast<const fe*>(dev_values), half,
                                 reinterpret_cast<const uint8_t*>(dev_tree), levels,
                                 didx.as<uint64_t>(), nq, dout.as<uint8_t>(), ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(out, dout.p, nq * rec, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MLH_OK;
}

mlh_status mlh_fri_prove(mlh_ctx* ctx, const void* dev_code, uint32_t log_code, mlh_transcript* tr,
                         mlh_fri_proof* proof) {
  if (!ctx || !dev_code || !tr || !proof) return fail(ctx, MLH_ERR_INVALID, "null argument");
  mlh_fri_prover* p = nullptr;
  MLH_TRY(mlh_fri_prover_fold(ctx, dev_code, log_code, tr, &p));
  mlh_status s = fri_queries(ctx, p, tr, proof);
  mlh_fri_prover_destroy(p);
  return s;
}

mlh_status mlh_fri_prove_gp(mlh_ctx* ctx, const void* dev_code, uint32_t log_code,
                            const uint8_t gen_pows_1[16], uint32_t log_gen_pows, mlh_transcript* tr,
                            mlh_fri_proof* proof) {
  if (!ctx || !dev_code || !tr || !proof || !gen_pows_1)
    return fail(ctx, MLH_ERR_INVALID, "null argument");
  mlh_fri_prover* p = nullptr;
  MLH_TRY(mlh_fri_prover_fold_gp(ctx, dev_code, log_code, gen_pows_1, log_gen_pows, tr, &p));
  mlh_status s = fri_queries(ctx, p, tr, proof);
  mlh_fri_prover_destroy(p);
  return s;
}

// ---------------------------------------------------------------------------
// multilinear / sumcheck
// ---------------------------------------------------------------------------
mlh_status mlh_mle_to_coefficient(mlh_ctx* ctx, void* dev_evals, uint32_t log_n) {
  if (!ctx || !dev_evals || log_n > 40) return fail(ctx, MLH_ERR_INVALID, "bad argument");
  HIP_TRY(ctx, launch_mobius(reinterpret_cast<fe*>(dev_evals), log_n, false, ctx->stream));
  return MLH_OK;
}

mlh_status mlh_mle_to_evaluation(mlh_ctx* ctx, void* dev_coeffs, uint32_t log_n) {
  if (!ctx || !dev_coeffs || log_n > 40) return fail(ctx, MLH_ERR_INVALID, "bad argument");
  HIP_TRY(ctx, launch_mobius(reinterpret_cast<fe*>(dev_coeffs), log_n, true, ctx->stream));
  return MLH_OK;
}

static mlh_status eq_table_impl(mlh_ctx* ctx, const uint8_t* host_points, uint32_t n,
                                void* dev_out, bool mono);

mlh_status mlh_eq_table(mlh_ctx* ctx, const uint8_t* host_points, uint32_t n, void* dev_out) {
  return eq_table_impl(ctx, host_points, n, dev_out, false);
}

static mlh_status eq_table_impl(mlh_ctx* ctx, const uint8_t* host_points, uint32_t n,
                                void* dev_out, bool mono) {
  if (!ctx || !dev_out || (n && !host_points) || n > 40)
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  PoolBuf pts(ctx), scratch(ctx);
  MLH_TRY(pts.alloc((n ? n : 1) * sizeof(fe)));
  const uint32_t a = n / 2, b = n - a;
  MLH_TRY(scratch.alloc(((1ull << a) + (1ull << b)) * sizeof(fe)));
  if (n) HIP_TRY(ctx, hipMemcpyAsync(pts.p, host_points, n * 16ull, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(ctx, launch_eq_table(pts.as<fe>(), n, scratch.as<fe>(), reinterpret_cast<fe*>(dev_out),
                               ctx->stream, mono));
  // pts/scratch go back to the pool now: a later user of those blocks is
  // ordered after these kernels on the same stream (and the pageable H2D
  // above has consumed host_points before returning)
  return MLH_OK;
}

static mlh_status read_pair(mlh_ctx* ctx, const fe* dev2, uint8_t out[32]) {
  HIP_TRY(ctx, hipMemcpyAsync(ctx->pinned, dev2, 32, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  memcpy(out, ctx->pinned, 32);
  return MLH_OK;
}

mlh_status mlh_mle_evaluate(mlh_ctx* ctx, const void* dev_evals, uint32_t n,
                            const uint8_t* host_args, uint8_t out[16]) {
  if (!ctx || !dev_evals || !out || n > 40) return fail(ctx, MLH_ERR_INVALID, "bad argument");
  PoolBuf eq(ctx);
  MLH_TRY(eq.alloc((16ull << n)));
  MLH_TRY(mlh_eq_table(ctx, host_args, n, eq.p));
  HIP_TRY(ctx, launch_dot(reinterpret_cast<const fe*>(dev_evals), eq.as<fe>(), 1ull << n,
                          ctx->partials, ctx->small, ctx->stream));
  uint8_t pair[32];
  MLH_TRY(read_pair(ctx, ctx->small, pair));
  memcpy(out, pair, 16);
  return MLH_OK;
}

mlh_status mlh_mle_coeffs_evaluate(mlh_ctx* ctx, const void* dev_coeffs, uint32_t n,
                                   const uint8_t* host_args, uint8_t out[16]) {
  if (!ctx || !dev_coeffs || !out || n > 40) return fail(ctx, MLH_ERR_INVALID, "bad argument");
  PoolBuf mono(ctx);
  MLH_TRY(mono.alloc((16ull << n)));
  MLH_TRY(eq_table_impl(ctx, host_args, n, mono.p, true));
  HIP_TRY(ctx, launch_dot(reinterpret_cast<const fe*>(dev_coeffs), mono.as<fe>(), 1ull << n,
                          ctx->partials, ctx->small, ctx->stream));
  uint8_t pair[32];
  MLH_TRY(read_pair(ctx, ctx->small, pair));
  memcpy(out, pair, 16);
  return MLH_OK;
}

mlh_status mlh_poly_evaluate(mlh_ctx* ctx, const void* dev_coeffs, uint64_t n, const uint8_t x[16],
                             uint8_t out[16]) {
  if (!ctx || (n && !dev_coeffs) || !x || !out || n > (1ull << 40))
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  if (n == 0) {  // fold over nothing: F::from(0)
    memset(out, 0, 16);
    return MLH_OK;
  }
  const u128 xv = h_load(x);
  if (xv >= kModulus) return fail(ctx, MLH_ERR_INVALID, "x not canonical");
  const uint64_t nlo = n < 4096 ? n : 4096, nhi = (n + 4095) / 4096;
  PoolBuf tlo(ctx), thi(ctx);
  MLH_TRY(tlo.alloc(16 * nlo));
  MLH_TRY(thi.alloc(16 * nhi));
  HIP_TRY(ctx, launch_pow_table(tlo.as<fe>(), to_fe(xv), to_fe(1), nlo, ctx->stream));
  HIP_TRY(ctx, launch_pow_table(thi.as<fe>(), to_fe(h_pow(xv, 4096)), to_fe(1), nhi, ctx->stream));
  HIP_TRY(ctx, launch_poly_eval(reinterpret_cast<const fe*>(dev_coeffs), n, tlo.as<fe>(),
                                thi.as<fe>(), ctx->partials, ctx->small, ctx->stream));
  uint8_t pair[32];
  MLH_TRY(read_pair(ctx, ctx->small, pair));
  memcpy(out, pair, 16);
  return MLH_OK;
}

mlh_status mlh_trace_evaluate(mlh_ctx* ctx, const void* dev_matrix, uint32_t log_height,
                             uint32_t width, const uint8_t* host_points, uint8_t* out) {
  if (!ctx || !dev_matrix || !out || log_height > 40 || width == 0 || width > (1u << 20) ||
      (log_height && !host_points))
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  const uint64_t height = 1ull << log_height;
  const uint32_t nc = width < 256 ? width : 256;
  PoolBuf eq(ctx), partials(ctx), res(ctx);
  MLH_TRY(eq.alloc(16ull << log_height));
  MLH_TRY(partials.alloc(16ull * trace_eval_blocks(height, nc) * nc));
  MLH_TRY(res.alloc(16ull * width));
  MLH_TRY(mlh_eq_table(ctx, host_points, log_height, eq.p));
  HIP_TRY(ctx, launch_trace_eval(reinterpret_cast<const fe*>(dev_matrix), eq.as<fe>(), height, width,
                                 partials.as<fe>(), res.as<fe>(), ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(out, res.p, 16ull * width, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MLH_OK;
}

mlh_status mlh_sumcheck_partial_sums(mlh_ctx* ctx, const void* dev_matrix, const void* dev_delta,
                                     uint32_t log_height, uint8_t out[32]) {
  if (!ctx || !dev_matrix || !dev_delta || !out || log_height < 1 || log_height > 40)
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  HIP_TRY(ctx, launch_sums(reinterpret_cast<const fe*>(dev_matrix),
                           reinterpret_cast<const fe*>(dev_delta), 1ull << (log_height - 1),
                           ctx->partials, ctx->small, ctx->stream));
  return read_pair(ctx, ctx->small, out);
}

mlh_status mlh_sumcheck_fold(mlh_ctx* ctx, void* dev_matrix, void* dev_delta, uint32_t log_height,
                             const uint8_t r[16]) {
  if (!ctx || !dev_matrix || !dev_delta || !r || log_height < 1 || log_height > 40)
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  HIP_TRY(ctx, launch_fold(reinterpret_cast<fe*>(dev_matrix), reinterpret_cast<fe*>(dev_delta),
                           1ull << log_height, to_fe(h_load(r)), ctx->stream));
  return MLH_OK;
}

mlh_status mlh_sumcheck_fold_and_sums(mlh_ctx* ctx, void* dev_matrix, void* dev_delta,
                                      uint32_t log_height, const uint8_t r[16], uint8_t out[32]) {
  if (!ctx || !dev_matrix || !dev_delta || !r || !out || log_height < 2 || log_height > 40)
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  HIP_TRY(ctx, launch_fold_sums(reinterpret_cast<fe*>(dev_matrix), reinterpret_cast<fe*>(dev_delta),
                                1ull << log_height, to_fe(h_load(r)), ctx->partials, ctx->small,
                                ctx->stream));
  return read_pair(ctx, ctx->small, out);
}

}  // extern "C"

extern "C" {

mlh_status mlh_sumcheck_prove(mlh_ctx* ctx, void* dev_matrix, void* dev_delta, uint32_t log_height,
                              const uint8_t sum[16], mlh_transcript* tr, uint8_t* polys_out,
                              uint8_t* rs_out) {
  if (!ctx || !dev_matrix || !dev_delta || !sum || !tr || log_height < 1 || log_height > 40)
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  // transcript on the device (one sync): [DevSha | prev | polys 32 x L | rs 16 x L]
  const uint32_t L = log_height;
  PoolBuf sc(ctx);
  MLH_TRY(sc.alloc(128 + 16 + 48ull * L));
  uint8_t* sb = sc.as<uint8_t>();
  DevSha* dt = reinterpret_cast<DevSha*>(sb);
  fe* prev = reinterpret_cast<fe*>(sb + 128);
  fe* polys = reinterpret_cast<fe*>(sb + 144);
  fe* rs = reinterpret_cast<fe*>(sb + 144 + 32ull * L);
  memcpy(ctx->pinned, &tr->sha, sizeof(DevSha));
  memcpy(ctx->pinned + 128, sum, 16);
  HIP_TRY(ctx, hipMemcpyAsync(sb, ctx->pinned, 144, hipMemcpyHostToDevice, ctx->stream));
  fe* m = reinterpret_cast<fe*>(dev_matrix);
  fe* d = reinterpret_cast<fe*>(dev_delta);
  // rounds on tables > 2^tail entries: partial-sum kernels over HBM + the
  // one-lane round kernel; the last `tail` rounds in one LDS-resident launch
  const uint32_t tail = sumcheck_tail_rounds(L);
  uint32_t np = 0;
  if (L > tail)
    HIP_TRY(ctx, launch_sums(m, d, 1ull << (L - 1), ctx->partials, ctx->small, ctx->stream, &np));
  for (uint32_t k = 0; k + tail < L; ++k) {
    HIP_TRY(ctx, launch_sumcheck_round(ctx->partials, np, prev, dt, polys + 2 * k, rs + k,
                                       ctx->stream));
    const uint64_t S = 1ull << (L - k);
    if (k + 1 + tail < L)  // the next round is not a tail round: fold + its sums
      HIP_TRY(ctx, launch_fold_sums(m, d, S, fe{}, ctx->partials, ctx->small, ctx->stream, rs + k,
                                    &np));
    else
      HIP_TRY(ctx, launch_fold(m, d, S, fe{}, ctx->stream, rs + k));
  }
  HIP_TRY(ctx, launch_sumcheck_tail(m, d, tail, prev, dt, polys + 2 * (L - tail),
                                    rs + (L - tail), ctx->stream));
  std::vector<uint8_t> host(48ull * L);
  HIP_TRY(ctx, hipMemcpyAsync(ctx->pinned, polys, 48ull * L, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  memcpy(host.data(), ctx->pinned, 48ull * L);
  ReplayCheck rc(ctx, tr);
  for (uint32_t k = 0; k < L; ++k) {  // host transcript replay (sumcheck.rs:188-199)
    rc.absorb(host.data() + 32 * k, 16);
    rc.absorb(host.data() + 32 * k + 16, 16);
    rc.expect(host.data() + 32ull * L + 16 * k);
  }
  MLH_TRY(rc.status());
  if (polys_out) memcpy(polys_out, host.data(), 32ull * L);
  if (rs_out) memcpy(rs_out, host.data() + 32ull * L, 16ull * L);
  return MLH_OK;
}

// ---------------------------------------------------------------------------
// multilinear PCS
// ---------------------------------------------------------------------------
// Sumcheck fold (+ the next round's partial sums) of a device-resident round,
// r read from HBM.  (Running it on a second stream beside the FRI fold_step,
// which needs the same r, measured no faster: the tree tail it would fill is
// a handful of waves, and the cross-stream events cost about what it saved.)
static mlh_status sumcheck_fold_dr(mlh_ctx* ctx, fe* m, fe* d, uint64_t S, const fe* r_dev,
                                   uint32_t* np, const fe* m_src = nullptr) {
  if (S >= 4)
    HIP_TRY(ctx, launch_fold_sums(m, d, S, fe{}, ctx->partials, ctx->small, ctx->stream, r_dev, np,
                                  m_src));
  else
    HIP_TRY(ctx, launch_fold(m, d, S, fe{}, ctx->stream, r_dev, m_src));
  return MLH_OK;
}

// Sumcheck over SumcheckTables::build_tables_for_pcs (sumcheck.rs:128-145:
// matrix, delta = eq(points)) with delta kept factored while the tables are
// larger than 2^a entries (sumcheck.hip, "eq-factored rounds"): rounds
// k < B = L - a stream only the matrix and carry delta as c_k * eq(p_k..);
// folding round B-1 writes delta_B = c_B * eq(p_B..p_{L-1}) (2^a entries) and
// the remaining rounds run the two-table kernels on it.  Round polynomials,
// challenges and the folded matrix equal those of the materialised tables.
#ifndef MLH_TAIL_XC
#define MLH_TAIL_XC 1  // 0: the tail launch sums its group-A corners itself
#endif
#ifndef MLH_TAIL_RSUF
#define MLH_TAIL_RSUF 1  // 0: the tail launch computes its suffix products itself
#endif
struct EqSumcheck {
  static constexpr uint32_t kEqLo = 12;  // = sumcheck_tail_rounds' LDS limit
  mlh_ctx* ctx;
  const fe* src = nullptr;  // round 0's matrix (read only)
  fe* m = nullptr;          // the folded matrix (== src: folded in place)
  uint32_t L = 0, a = 0, B = 0;
  PoolBuf buf;
  fe *pts = nullptr, *c = nullptr, *lo = nullptr, *d = nullptr, *H = nullptr;
  fe* Hs = nullptr;  // eq suffix tables of the last a points (sumcheck_eq_tail_kernel)
  uint32_t* kw = nullptr;  // padding-block K + W tables per round (init with a transcript)
  fe* wts = nullptr;       // eq weights of the last finished group's challenges (its fold)
  uint32_t tail_xc_nb = 0; // head_rounds: the tail's group-A corner sums are in ctx->partials
  bool tail_tables = false; // Hs filled (init's want_tail)
  fe* rsuf = nullptr;       // the tail's suffix products (want_tail; eq_setup_kernel)
  explicit EqSumcheck(mlh_ctx* c_) : ctx(c_), buf(c_) {}

  // matrix: round 0's table; work (2^(L-1) entries, optional) receives the
  // folded table -- the first fold reads `matrix` and writes `work`, so the
  // caller's evaluations are never copied (build_tables_for_pcs's clone)
  // sha / sum / dt_out / prev_out (optional): also place the transcript state
  // and the claimed sum on the device in the same launch
  mlh_status init(const fe* matrix, fe* work, uint32_t L_, const uint8_t* host_points,
                  bool want_tail = false, const void* sha = nullptr, const uint8_t* sum = nullptr,
                  DevSha* dt_out = nullptr, fe* prev_out = nullptr) {
    src = matrix;
    m = work ? work : const_cast<fe*>(matrix);
    L = L_;
    tail_tables = want_tail;
    a = L < kEqLo ? L : kEqLo;
    B = L - a;
    // c | lo[2^a] | d[2^a] | H[2^B - 1] | Hs[2^a - 1] | pts[L] | kw[64 L words] | wts[64] |
    // rsuf[2 kEqTailRsuf] (tail, head)
    MLH_TRY(buf.alloc(16 * (1 + 3 * (1ull << a) + (1ull << B) + L + 16ull * L + 64 + 2 * kEqTailRsuf)));
    c = buf.as<fe>();
    lo = c + 1;
    d = B ? lo + (1ull << a) : lo;  // B == 0: delta is the whole eq table
    H = lo + 2 * (1ull << a);
    Hs = H + (1ull << B);
    pts = Hs + (1ull << a);
    kw = sha ? reinterpret_cast<uint32_t*>(pts + L) : nullptr;
    wts = pts + L + 16ull * L;
    rsuf = MLH_TAIL_RSUF && want_tail ? wts + 64 : nullptr;
    EqSetupArgs args{};
    if (L) memcpy(args.pts, host_points, 16ull * L);
    if (sha) memcpy(&args.sha, sha, sizeof(DevSha));
    if (sum) memcpy(&args.sum, sum, 16);
    args.L = L;
    args.B = B;
    HIP_TRY(ctx, launch_eq_setup(args, pts, c, lo, H, want_tail ? Hs : nullptr, dt_out, prev_out,
                                 ctx->stream, kw, rsuf));
    return MLH_OK;
  }
  const fe* Hk(uint32_t k) const { return H + ((1ull << B) - (1ull << (B - k))); }

  // Head rounds k < B go in groups of up to kGroup (sumcheck.hip, "grouped
  // eq-factored rounds"): one HBM pass yields the corner sums of a whole
  // group, the group's rounds run from them, and one pass folds the group's
  // variables and yields the next group's corner sums.  gk / gJ / gnb: the
  // current group's first round, size and partial block count.
  static constexpr uint32_t kGroup = 3;
  uint32_t gk = 0, gJ = 0, gnb = 0;
  uint32_t group_len(uint32_t k) const { return B - k < kGroup ? B - k : kGroup; }

  // round 0's sums (B > 0: the first group's corner sums) into ctx->partials
  mlh_status first_sums(uint32_t* np) {
    if (B) {
      gk = 0;
      gJ = group_len(0);
      HIP_TRY(ctx, launch_group_sums_eq(src, 1ull << L, gJ, Hk(gJ - 1), lo, a, ctx->partials,
                                        ctx->stream, &gnb));
      *np = gnb;
    } else {
      HIP_TRY(ctx, launch_sums(src, d, 1ull << (L - 1), ctx->partials, ctx->small, ctx->stream, np));
    }
    return MLH_OK;
  }
  // round k (r: its challenge slot; the slots of one group are contiguous)
  mlh_status round(uint32_t k, uint32_t np, fe* prev, DevSha* dt, fe* poly, fe* r) {
    if (k < B) {
      const uint32_t t = k - gk;
      HIP_TRY(ctx, launch_sumcheck_group(ctx->partials, gnb, gJ, 0, t, t + 1, prev, dt, poly, r - t,
                                         pts + gk, c, ctx->stream, coop_ctl(ctx), nullptr, wts));
    } else {
      HIP_TRY(ctx, launch_sumcheck_round(ctx->partials, np, prev, dt, poly, r, ctx->stream));
    }
    return MLH_OK;
  }
  // The head of a prove with no work between rounds (mlh_sumcheck_prove_eq):
  // passes of up to 6 rounds (two chained groups of <= 3 from one set of
  // corner sums), each folded in one HBM pass that also sums the next; the
  // last pass's fold leaves T_B (2^a entries) in m for the tail.
  mlh_status head_rounds(fe* prev, DevSha* dt, fe* polys, fe* rs) {
    if (!B) return MLH_OK;
    if (B <= kEqLo && a == kEqLo && B >= 2) {
      // B <= 12: one pass for the B-variable corner sums Y, all B rounds in one
      // launch on Y (two corner groups), then the B-variable fold of the table
      // as two eq-weighted passes (sumcheck.hip "grouped eq-factored rounds")
      PoolBuf yb(ctx);
      MLH_TRY(yb.alloc(16 * ((1ull << B) + 128)));
      fe* Y = yb.as<fe>();
      fe* wf = Y + (1ull << B);
      const uint32_t JA = B < 6 ? B : 6, JB = B - JA;
      HIP_TRY(ctx, launch_corner_sums_lo(src, B, a, lo, Y, ctx->stream));
      HIP_TRY(ctx, launch_sumcheck_eq_head(Y, B, Hk(JA - 1), pts, c, prev, dt, polys, rs, wf,
                                           ctx->stream, coop_ctl(ctx), kw,
                                           rsuf ? rsuf + kEqTailRsuf : nullptr));
      // the last fold also sums the tail's group-A corners (JN = 6 over its
      // 2^12 outputs, e = Hs_5, H = H_{B-1} = [1]): the tail launch then skips
      // that phase of its prologue (tail_xc_nb partials per corner in
      // ctx->partials; tail launch 59.3 -> 56.5 us, the fold +1 us)
      const bool xc = MLH_TAIL_XC && tail_tables;
      const fe* e5 = Hs + ((1ull << a) - (1ull << (a - 5)));
      uint32_t nb = 0;
      HIP_TRY(ctx, launch_fold_group_eq(src, 1ull << L, JA, xc && !JB ? 6 : 0, rs, wf, m,
                                        xc && !JB ? Hk(B - 1) : nullptr, xc && !JB ? e5 : lo,
                                        xc && !JB ? 6 : a, ctx->partials, ctx->stream, &nb));
      if (JB)
        HIP_TRY(ctx, launch_fold_group_eq(m, 1ull << (L - JA), JB, xc ? 6 : 0, rs + JA, wf + 64, m,
                                          xc ? Hk(B - 1) : nullptr, xc ? e5 : lo, xc ? 6 : a, ctx->partials,
                                          ctx->stream, &nb));
      tail_xc_nb = xc ? nb : 0;
      return MLH_OK;
    }
    uint32_t nb = 0, k = 0, JT = B < kMaxGroup ? B : kMaxGroup;
    HIP_TRY(ctx, launch_group_sums_eq(src, 1ull << L, JT, Hk(JT - 1), lo, a, ctx->partials,
                                      ctx->stream, &nb));
    for (;;) {
      const uint32_t J1 = JT < 3 ? JT : 3;
      HIP_TRY(ctx, launch_sumcheck_group(ctx->partials, nb, J1, JT - J1, 0, J1, prev, dt,
                                         polys + 2 * k, rs + k, pts + k, c, ctx->stream,
                                         coop_ctl(ctx), kw ? kw + 64 * k : nullptr, wts));
      const fe* in = k == 0 ? src : m;
      const uint64_t S = 1ull << (L - k);
      k += JT;
      const uint32_t JN = B - k < kMaxGroup ? B - k : kMaxGroup;
      HIP_TRY(ctx, launch_fold_group_eq(in, S, JT, JN, rs + k - JT, wts, m,
                                        JN ? Hk(k + JN - 1) : nullptr, lo, a, ctx->partials,
                                        ctx->stream, &nb));
      if (!JN) return MLH_OK;
      JT = JN;
    }
  }
  // after round k's challenge (r_dev): fold what is due (HBM); want_sums: also
  // round k+1's sums.  A head group folds once, after its last round.
  mlh_status fold(uint32_t k, const fe* r_dev, uint32_t* np, bool want_sums = true) {
    const uint64_t S = 1ull << (L - k);
    if (k < B) {
      if (k + 1 < gk + gJ) return MLH_OK;  // mid-group: nothing to fold yet
      const fe* in = gk == 0 ? src : m;
      const uint32_t JN = group_len(k + 1);
      HIP_TRY(ctx, launch_fold_group_eq(in, 1ull << (L - gk), gJ, JN, r_dev - (gJ - 1), wts, m,
                                        JN ? Hk(k + JN) : nullptr, lo, a, ctx->partials,
                                        ctx->stream, &gnb));
      if (JN) {
        gk = k + 1;
        gJ = JN;
        *np = gnb;
        return MLH_OK;
      }
      HIP_TRY(ctx, launch_scale_dev(lo, c, 1ull << a, d, ctx->stream));
      if (want_sums)
        HIP_TRY(ctx, launch_sums(m, d, 1ull << (a - 1), ctx->partials, ctx->small, ctx->stream, np));
    } else {
      MLH_TRY(sumcheck_fold_dr(ctx, m, d, S, r_dev, np, k == 0 ? src : m));
    }
    return MLH_OK;
  }
};

mlh_status mlh_sumcheck_prove_eq(mlh_ctx* ctx, const void* dev_evals, void* dev_work,
                                 uint32_t log_height, const uint8_t* host_points,
                                 const uint8_t sum[16], mlh_transcript* tr, uint8_t* polys_out,
                                 uint8_t* rs_out, uint8_t* delta_out) {
  if (!ctx || !dev_evals || !host_points || !sum || !tr || log_height < 1 || log_height > 40)
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  const uint32_t L = log_height;
  PoolBuf sc(ctx);
  MLH_TRY(sc.alloc(128 + 16 + 48ull * L + 16));
  uint8_t* sb = sc.as<uint8_t>();
  DevSha* dt = reinterpret_cast<DevSha*>(sb);
  fe* prev = reinterpret_cast<fe*>(sb + 128);
  fe* polys = reinterpret_cast<fe*>(sb + 144);
  fe* rs = reinterpret_cast<fe*>(sb + 144 + 32ull * L);
  fe* dfin = reinterpret_cast<fe*>(sb + 144 + 48ull * L);  // the final delta
  EqSumcheck es(ctx);  // its setup launch also places the transcript state and the claim
  device_arm(ctx);
  MLH_TRY(es.init(reinterpret_cast<const fe*>(dev_evals), reinterpret_cast<fe*>(dev_work), L,
                  host_points, true, &tr->sha, sum, dt, prev));
  // head rounds stream only the matrix (passes of up to 6 rounds); the last a
  // rounds run in the LDS-resident eq tail on the 2^a-entry folded table
  MLH_TRY(es.head_rounds(prev, dt, polys, rs));
  HIP_TRY(ctx, launch_sumcheck_eq_tail(es.B ? es.m : es.src, 0, nullptr, es.a, es.Hs,
                                       es.pts + es.B, es.c, prev, dt, polys + 2 * es.B, rs + es.B,
                                       es.m, dfin, ctx->stream, coop_ctl(ctx),
                                       es.kw ? es.kw + 64 * es.B : nullptr,
                                       HostOut{reinterpret_cast<const uint8_t*>(polys), ctx->pinned,
                                               (uint32_t)(48ull * L + 16)},
                                       es.tail_xc_nb ? ctx->partials : nullptr, es.tail_xc_nb,
                                       es.rsuf));
  HIP_TRY(ctx, prove_wait(ctx));
  MLH_TRY(device_check(ctx));
  std::vector<uint8_t> host(ctx->pinned, ctx->pinned + 48ull * L + 16);
  ReplayCheck rc(ctx, tr);
  for (uint32_t k = 0; k < L; ++k) {  // host transcript replay (sumcheck.rs:188-199)
    rc.absorb(host.data() + 32 * k, 16);
    rc.absorb(host.data() + 32 * k + 16, 16);
    rc.expect(host.data() + 32ull * L + 16 * k);
  }
  MLH_TRY(rc.status());
  if (polys_out) memcpy(polys_out, host.data(), 32ull * L);
  if (rs_out) memcpy(rs_out, host.data() + 32ull * L, 16ull * L);
  if (delta_out) memcpy(delta_out, host.data() + 48ull * L, 16);
  return MLH_OK;
}

// PCSProverData::fold (multilinear_pcs.rs:43-76) for n_vars <= 24, with the
// sumcheck off the transcript chain (sumcheck.hip "PCS rounds off the
// transcript kernel"): round k's (c1, c2) come from a one-workgroup job on
// the eq-factored table once r_{k-1} exists -- an extra workgroup of FRI step
// k-1's fold launch -- and the launch that writes FRI root k absorbs root k,
// then (c1, c2)_k, and draws r_k: the transcript order of the reference
// (root_k | c1_k | c2_k -> r_k), with no sumcheck launch between challenges.
// Head (the first B = n - 12 variables): the 2^B corner sums of the 2^n table
// in one pass; after r_{B-1} two fold_group_eq passes fold the table to the
// 2^12 entries the tail rounds use.  Shared by the PCS and the batched PCS.
struct PcsRounds {
  static constexpr uint32_t kMaxVars = 2 * EqSumcheck::kEqLo;
  mlh_ctx* ctx;
  FriDevLoop& lp;
  EqSumcheck es;
  PoolBuf yb;
  const fe* evals = nullptr;
  fe* work = nullptr;
  fe* Y = nullptr;   // head table: the 2^B corner sums, folded in place
  fe* wf = nullptr;  // the two fold_group_eq passes' weights
  PcsRoundState* st = nullptr;
  uint32_t n = 0, B = 0, a = 0;
  PcsRounds(mlh_ctx* c, FriDevLoop& l) : ctx(c), lp(l), es(c), yb(c) {}

  // after lp.layout(.., >= 5 extra slots): tables, round state (claim =
  // claim_host, or claim_dev copied on the device), round 0's polynomial
  mlh_status init(const fe* evals_, fe* work_, uint32_t n_, const uint8_t* host_inputs,
                  const uint8_t* claim_host, const fe* claim_dev) {
    evals = evals_;
    work = work_;
    n = n_;
    MLH_TRY(es.init(evals, work, n, host_inputs, /*want_tail=*/true));
    B = es.B;
    a = es.a;
    if (B) {
      MLH_TRY(yb.alloc(16 * ((1ull << B) + 128)));
      Y = yb.as<fe>();
      wf = Y + (1ull << B);
    }
    uint8_t init_state[80] = {};  // (claim, c = 1, e0 = c1 = c2 = 0)
    if (claim_host) memcpy(init_state, claim_host, 16);
    init_state[16] = 1;
    memcpy(ctx->pinned + kPinSlotA, init_state, 80);
    st = reinterpret_cast<PcsRoundState*>(lp.extra());
    HIP_TRY(ctx, hipMemcpyAsync(st, ctx->pinned + kPinSlotA, 80, hipMemcpyHostToDevice, ctx->stream));
    if (claim_dev)
      HIP_TRY(ctx, hipMemcpyAsync(&st->claim, claim_dev, 16, hipMemcpyDeviceToDevice, ctx->stream));
    if (B) {
      HIP_TRY(ctx, launch_corner_sums_lo(evals, B, a, es.lo, Y, ctx->stream));
      HIP_TRY(ctx, launch_pcs_round(Y, Y, B, false, nullptr, nullptr, es.pts, e_of(0), st, lp.poly(0),
                                    ctx->stream));
    } else {
      HIP_TRY(ctx, launch_pcs_round(evals, work, n, false, nullptr, nullptr, es.pts, e_of(0), st,
                                    lp.poly(0), ctx->stream));
    }
    return MLH_OK;
  }
  // e of round k: H_k (head) or Hs_{k-B} (tail); 2^(h-1) entries for a table of 2^h
  const fe* e_of(uint32_t k) const {
    return k < B ? es.Hk(k) : es.Hs + ((1ull << a) - (1ull << (a - (k - B))));
  }
  // round kn (>= 1) as a job; at kn == B the table fold over the head
  // variables is enqueued first (it needs r_0..r_{B-1})
  mlh_status job(uint32_t kn, PcsJob* out) {
    const uint32_t k = kn - 1;
    PcsJob j{nullptr, work, 0, 1, lp.r(k), es.pts + k, es.pts + kn, e_of(kn), st, lp.poly(kn)};
    if (kn < B) {  // head: fold Y with r_k
      j.src = Y;
      j.dst = Y;
      j.log_h = B - kn;
    } else if (kn == B) {  // fold the table over the B head variables; round B on it
      const uint32_t JA = B < 6 ? B : 6, JB = B - JA;
      uint32_t nb = 0;
      HIP_TRY(ctx, launch_eq_weights(lp.r(0), JA, JB, wf, ctx->stream));
      HIP_TRY(ctx, launch_fold_group_eq(evals, 1ull << n, JA, 0, lp.r(0), wf, work, nullptr, es.lo, a,
                                        ctx->partials, ctx->stream, &nb));
      if (JB)
        HIP_TRY(ctx, launch_fold_group_eq(work, 1ull << (n - JA), JB, 0, lp.r(JA), wf + 64, work,
                                          nullptr, es.lo, a, ctx->partials, ctx->stream, &nb));
      j.src = work;
      j.log_h = a;
      j.fold = 0;
    } else {  // tail: fold with r_k (the first tail fold of B = 0 reads the evaluations)
      j.src = (B == 0 && kn == 1) ? evals : work;
      j.log_h = n - kn;
    }
    *out = j;
    return MLH_OK;
  }
};

static mlh_status pcs_rounds_fused(mlh_ctx* ctx, FriDevLoop& lp, const fe* evals, fe* work,
                                   uint32_t n, const uint8_t* host_inputs, const uint8_t output[16],
                                   const void* code, uint32_t log_domain, mlh_transcript* tr) {
  MLH_TRY(lp.layout(log_domain, tr, 5));
  PcsRounds pr(ctx, lp);
  MLH_TRY(pr.init(evals, work, n, host_inputs, output, nullptr));
  // FRI init: root 0 | (c1, c2)_0 -> r_0
  MLH_TRY(lp.init_after_layout(code, log_domain, true, lp.poly(0)));
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t kn = k + 1;  // the round whose polynomial follows r_k
    PcsJob job{};
    if (kn < n) MLH_TRY(pr.job(kn, &job));
    MLH_TRY(lp.step(k, lp.r(k), kn < n, kn < n ? lp.poly(kn) : nullptr, kn < n ? &job : nullptr));
  }
  return MLH_OK;
}

mlh_status mlh_pcs_prove(mlh_ctx* ctx, const void* dev_evals, uint32_t n_vars,
                         const uint8_t* host_inputs, const uint8_t output[16], mlh_transcript* tr,
                         mlh_pcs_proof* proof) {
  if (!ctx || !dev_evals || !output || !tr || !proof || (n_vars && !host_inputs))
    return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (n_vars < 1 || n_vars > 36) return fail(ctx, MLH_ERR_INVALID, "n_vars out of range");
  const uint32_t log_domain = n_vars + MLH_LOG_BLOWUP;
  const uint64_t n = 1ull << n_vars;
  const u128 gen = h_pow2_generator(log_domain);  // gen_pows[1] (multilinear_pcs.rs:103-104)
  uint8_t genb[16];
  h_store(genb, gen);
  PoolBuf coeffs(ctx), code(ctx), matrix(ctx);
  MLH_TRY(coeffs.alloc(n * 16));
  MLH_TRY(code.alloc(2 * n * 16));
  MLH_TRY(matrix.alloc(n / 2 * 16));  // the folded table (the first fold reads dev_evals)
  // to_coefficient (:102), bit reverse (:104), reed_solomon (:107); the copy
  // and the permutation are folded into the Moebius and first NTT passes
  HIP_TRY(ctx, launch_mobius(coeffs.as<fe>(), n_vars, false, ctx->stream,
                             reinterpret_cast<const fe*>(dev_evals)));
  MLH_TRY(mlh_reed_solomon_brev(ctx, coeffs.p, n_vars, genb, code.p));  // bitrev fused
  // PCSProverData::init (:28-42) + fold loop (:57-75), transcript on the
  // device: per round the sumcheck round kernel absorbs (c1, c2) and derives
  // r, which the sumcheck fold and the FRI fold_step read from HBM.
  std::unique_ptr<mlh_fri_prover> fp(new mlh_fri_prover());
  fp->ctx = ctx;
  fp->log_code = log_domain;
  FriDevLoop lp(ctx, fp.get());
  device_arm(ctx);
  if (n_vars <= ctx->pcs_fused_max) {
    MLH_TRY(pcs_rounds_fused(ctx, lp, reinterpret_cast<const fe*>(dev_evals), matrix.as<fe>(),
                             n_vars, host_inputs, output, code.p, log_domain, tr));
  } else {
    MLH_TRY(lp.init(code.p, log_domain, tr, false));
    EqSumcheck es(ctx);  // delta = eq(inputs), factored (build_tables_for_pcs)
    MLH_TRY(es.init(reinterpret_cast<const fe*>(dev_evals), matrix.as<fe>(), n_vars, host_inputs));
    memcpy(ctx->pinned + kPinSlotA, output, 16);
    HIP_TRY(ctx, hipMemcpyAsync(lp.prev(), ctx->pinned + kPinSlotA, 16, hipMemcpyHostToDevice,
                                ctx->stream));
    uint32_t np = 0;
    MLH_TRY(es.first_sums(&np));
    for (uint32_t k = 0; k < n_vars; ++k) {
      MLH_TRY(es.round(k, np, lp.prev(), lp.dt(), lp.poly(k), lp.r(k)));
      MLH_TRY(es.fold(k, lp.r(k), &np));
      MLH_TRY(lp.step(k, lp.r(k), false));
    }
  }
  MLH_TRY(lp.finish(32ull * n_vars));
  // host transcript replay: root_0, then per round (c1, c2), root_{k+1} / last
  const uint8_t* polys = lp.host_polys();
  if (proof->sumcheck_polys) memcpy(proof->sumcheck_polys, polys, 32ull * n_vars);
  ReplayCheck rc(ctx, tr);
  rc.absorb(fp->layers[0].root, 32);
  for (uint32_t k = 0; k < n_vars; ++k) {
    rc.absorb(polys + 32 * k, 16);
    rc.absorb(polys + 32 * k + 16, 16);
    rc.expect(lp.host_r(k));
    if (k + 1 < fp->layers.size())
      rc.absorb(fp->layers[k + 1].root, 32);
    else
      rc.absorb(fp->last, 16);
  }
  MLH_TRY(rc.status());
  mlh_fri_prover* fpp = fp.get();
  MLH_TRY(fri_queries(ctx, fpp, tr, &proof->fri));
  return MLH_OK;
}

}  // extern "C"

extern "C" {

mlh_status mlh_merkle_open(mlh_ctx* ctx, const void* dev_layers, uint64_t leaves,
                           const uint64_t* host_idx, uint32_t nq, uint8_t* out) {
  if (!ctx || !dev_layers || (nq && (!host_idx || !out)))
    return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (!is_pow2(leaves)) return fail(ctx, MLH_ERR_NOT_POW2, "Data length must be a power of two");
  for (uint32_t q = 0; q < nq; ++q)
    if (host_idx[q] >= leaves) return fail(ctx, MLH_ERR_INVALID, "index out of bounds");
  const uint32_t depth = 63 - __builtin_clzll(leaves);
  if (nq == 0 || depth == 0) return MLH_OK;
  const uint64_t rec = 32ull * depth;
  PoolBuf didx(ctx), dout(ctx);
  MLH_TRY(didx.alloc(nq * sizeof(uint64_t)));
  MLH_TRY(dout.alloc(nq * rec));
  HIP_TRY(ctx, hipMemcpyAsync(didx.p, host_idx, nq * sizeof(uint64_t), hipMemcpyHostToDevice,
                              ctx->stream));
  HIP_TRY(ctx, launch_merkle_paths(reinterpret_cast<const uint8_t*>(dev_layers), leaves,
                                   didx.as<uint64_t>(), nq, dout.as<uint8_t>(), ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(out, dout.p, nq * rec, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MLH_OK;
}

}  // extern "C"

extern "C" {

// ---------------------------------------------------------------------------
// kernel timer
// ---------------------------------------------------------------------------
mlh_status mlh_profile_enable(mlh_ctx* ctx, int on) {
  if (!ctx || on < 0) return MLH_ERR_INVALID;
  ctx->prof_on = on != 0;
  ctx->prof_every = on > 1 ? (uint32_t)on : 1u;
  ctx->prof_ticks.clear();
  return MLH_OK;
}

mlh_status mlh_profile_reset(mlh_ctx* ctx) {
  if (!ctx) return MLH_ERR_INVALID;
  resolve_profile(ctx);
  ctx->prof.clear();
  return MLH_OK;
}

mlh_status mlh_profile_get(mlh_ctx* ctx, const char* label, uint64_t* count, double* total_ms) {
  if (!ctx || !label || !count || !total_ms) return MLH_ERR_INVALID;
  resolve_profile(ctx);
  auto it = ctx->prof.find(label);
  *count = it == ctx->prof.end() ? 0 : it->second.first;
  *total_ms = it == ctx->prof.end() ? 0.0 : it->second.second;
  return MLH_OK;
}

// ---------------------------------------------------------------------------
// bench helper
// ---------------------------------------------------------------------------
mlh_status mlh_bench_ntt(mlh_ctx* ctx, void* dev_buf, uint32_t log_n, uint32_t iters,
                         float* ms_out) {
  if (!ctx || !dev_buf || !ms_out || iters == 0) return fail(ctx, MLH_ERR_INVALID, "bad argument");
  uint8_t gen[16];
  h_store(gen, h_pow2_generator(log_n));
  MLH_TRY(mlh_ntt(ctx, dev_buf, dev_buf, log_n, gen));  // warm the table cache
  hipEvent_t a, b;
  HIP_TRY(ctx, hipEventCreate(&a));
  HIP_TRY(ctx, hipEventCreate(&b));
  HIP_TRY(ctx, hipEventRecord(a, ctx->stream));
  for (uint32_t i = 0; i < iters; ++i) MLH_TRY(mlh_ntt(ctx, dev_buf, dev_buf, log_n, gen));
  HIP_TRY(ctx, hipEventRecord(b, ctx->stream));
  HIP_TRY(ctx, hipEventSynchronize(b));
  float ms = 0;
  HIP_TRY(ctx, hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *ms_out = ms / iters;
  return MLH_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// batched FRI / batched PCS (src/fri/batched_fri.rs, batched_pcs.rs)
// ---------------------------------------------------------------------------
// Queries of a batched proof (batched_fri.rs:287-300): the transcript draws
// the indices, the batch column + batch siblings and the inner paths are
// gathered into one device buffer, one D2H.
static mlh_status batched_queries(mlh_ctx* ctx, FriDevLoop& lp, mlh_transcript* tr,
                                  mlh_batched_fri_proof* pf) {
  const uint32_t L = lp.p->log_code, m = lp.m;
  const uint64_t N = 1ull << L;
  std::vector<uint64_t> idx(MLH_NUM_QUERIES);
  for (int q = 0; q < MLH_NUM_QUERIES; ++q) {
    idx[q] = transcript_query_index(tr, N / 2);
    uint8_t le[8];
    memcpy(le, &idx[q], 8);
    mlh_transcript_absorb(tr, le, 8);
  }
  pf->log_code = L;
  pf->num_codes = m;
  pf->num_trees = (uint32_t)lp.p->layers.size();
  pf->num_queries = MLH_NUM_QUERIES;
  if (pf->query_indices) memcpy(pf->query_indices, idx.data(), idx.size() * 8);
  memcpy(pf->last_elem, lp.p->last, 16);
  mlh_transcript_random(tr, pf->last_random);
  if (pf->commitments) mlh_fri_prover_roots(lp.p, pf->commitments);
  if (!pf->queries) return MLH_OK;
  const uint64_t qbytes = mlh_batched_fri_query_bytes(L, m);
  uint8_t* h;
  MLH_TRY(query_stage(ctx, MLH_NUM_QUERIES * qbytes, &h));
  mlh::QueryIdx qi;
  memcpy(qi.v, idx.data(), 8ull * MLH_NUM_QUERIES);
  HIP_TRY(ctx, launch_batch_queries(lp.codes, m, N, lp.btree.as<uint8_t>(), qi, MLH_NUM_QUERIES,
                                    qbytes, h, ctx->stream));
  MLH_TRY(gather_queries_dev(ctx, lp.p, qi, nullptr, MLH_NUM_QUERIES, qbytes,
                             32ull * m + 32ull * (L - 1), h));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  memcpy(pf->queries, h, MLH_NUM_QUERIES * qbytes);
  return MLH_OK;
}

extern "C" {

mlh_status mlh_batched_fri_prove(mlh_ctx* ctx, const void* dev_codes, uint32_t num_codes,
                                 uint32_t log_code, mlh_transcript* tr,
                                 mlh_batched_fri_proof* proof) {
  if (!ctx || !dev_codes || !tr || !proof) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (num_codes == 0) return fail(ctx, MLH_ERR_INVALID, "Codes must not be empty");
  if (log_code < 2 || log_code > 40)
    return fail(ctx, MLH_ERR_NOT_POW2, "Code size must be a power of two (>= 4)");
  std::unique_ptr<mlh_fri_prover> p(new mlh_fri_prover());
  p->ctx = ctx;
  p->log_code = log_code;
  FriDevLoop lp(ctx, p.get());
  device_arm(ctx);
  MLH_TRY(lp.init_batched(reinterpret_cast<const fe*>(dev_codes), num_codes, log_code, tr, true));
  // fold (batched_fri.rs:178-205): the batched step, then ordinary steps
  MLH_TRY(lp.step_batched(lp.r(0), true));
  const uint32_t steps = log_code - MLH_LOG_BLOWUP;
  for (uint32_t k = 1; k < steps; ++k) MLH_TRY(lp.step(k, lp.r(k), true));
  MLH_TRY(lp.finish(0));
  // host transcript replay: batch root, fingerprint_r, inner roots, last
  ReplayCheck rc(ctx, tr);
  rc.absorb(lp.host_broot(), 32);
  rc.expect(lp.host_fr());
  rc.absorb(lp.host_fr(), 16);
  rc.expect(lp.host_r(0));
  for (size_t t = 0; t < p->layers.size(); ++t) {
    rc.absorb(p->layers[t].root, 32);
    rc.expect(lp.host_r((uint32_t)t + 1));
  }
  rc.absorb(p->last, 16);
  MLH_TRY(rc.status());
  memcpy(proof->batch_commitment, lp.host_broot(), 32);
  return batched_queries(ctx, lp, tr, proof);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// BatchedFriProverData step by step (batched_fri.rs:9-224), host transcript:
// init -> batched_fold_step(gen_pows, r, tr) -> the inner fri_data's
// fold_step(gen_pows, k, r, tr) for k >= 1 (mlh_fri_prover_fold_step(_gp) on
// the handle mlh_batched_fri_prover_inner returns) -> open_query_at.  The
// whole-proof path (mlh_batched_fri_prove) keeps the transcript on the device.
// ---------------------------------------------------------------------------
struct mlh_batched_fri_prover {
  mlh_ctx* ctx;
  const fe* codes = nullptr;  // caller's [m][N], must outlive the prover
  uint32_t m = 0, log_code = 0;
  void* btree = nullptr;      // batch layer: N/2 leaves + levels
  void* scal = nullptr;       // device [fingerprint_r | r]
  uint8_t broot[32];
  uint8_t fr[16];
  mlh_fri_prover inner;       // fri_data: merkle_trees start at the folded layer
  ~mlh_batched_fri_prover() {
    pool_free(ctx, btree);
    pool_free(ctx, scal);
  }
};

extern "C" {

mlh_status mlh_batched_fri_prover_init(mlh_ctx* ctx, const void* dev_codes, uint32_t num_codes,
                                       uint32_t log_code, mlh_transcript* tr, mlh_batched_fri_prover** out) {
  if (!ctx || !dev_codes || !tr || !out) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (num_codes == 0) return fail(ctx, MLH_ERR_INVALID, "Codes must not be empty");
  if (log_code < 2 || log_code > 40)
    return fail(ctx, MLH_ERR_NOT_POW2, "Code size must be a power of two (>= 4)");
  std::unique_ptr<mlh_batched_fri_prover> bp(new mlh_batched_fri_prover());
  bp->ctx = ctx;
  bp->codes = reinterpret_cast<const fe*>(dev_codes);
  bp->m = num_codes;
  bp->log_code = log_code;
  bp->inner.ctx = ctx;
  bp->inner.log_code = log_code - 1;  // its first tree is the folded layer's
  bp->inner.gp_gen = h_pow2_generator(log_code);  // the batched code's domain
  bp->inner.log_gp = log_code;
  const uint64_t N = 1ull << log_code, L = N / 2;
  MLH_TRY(pool_alloc(ctx, mlh_merkle_layers_bytes(L), &bp->btree));
  MLH_TRY(pool_alloc(ctx, 32, &bp->scal));
  uint8_t* bt = reinterpret_cast<uint8_t*>(bp->btree);
  HIP_TRY(ctx, launch_batch_pairs_leaves(bp->codes, num_codes, N, bt, ctx->stream));
  HIP_TRY(ctx, launch_merkle_levels(bt, L, ctx->stream));
  MLH_TRY(read_root(ctx, bt, L, bp->broot));
  // batched_fri.rs:82-89: absorb the root, fingerprint_r = next_challenge(),
  // absorb LE16(fingerprint_r)
  mlh_transcript_absorb(tr, bp->broot, 32);
  mlh_transcript_next_challenge(tr, bp->fr);
  mlh_transcript_absorb(tr, bp->fr, 16);
  *out = bp.release();
  return MLH_OK;
}

mlh_status mlh_batched_fri_prover_fold_step_gp(mlh_ctx* ctx, mlh_batched_fri_prover* bp,
                                               const uint8_t gen_pows_1[16], uint32_t log_gen_pows,
                                               const uint8_t r[16], mlh_transcript* tr) {
  if (!ctx || !bp || !gen_pows_1 || !r || !tr) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_gen_pows < 1 || log_gen_pows > 40) return fail(ctx, MLH_ERR_INVALID, "gen_pows length");
  const u128 g = h_load(gen_pows_1);
  if (!check_generator(g, log_gen_pows))
    return fail(ctx, MLH_ERR_BAD_GENERATOR, "gen_pows[1] must have order exactly gen_pows.len()");
  const uint64_t N = 1ull << bp->log_code, half_n = N / 2;
  if (N <= (1ull << MLH_LOG_BLOWUP)) return MLH_OK;  // batched_fri.rs:104-106
  if (half_n - 1 > (1ull << log_gen_pows))
    return fail(ctx, MLH_ERR_INVALID, "gen_pows index len - i underflows (batched_fri.rs:131-136)");
  // (called again, the reference folds the batch layer again and pushes a
  // second tree onto fri_data; this binding folds it once)
  if (!bp->inner.layers.empty() || bp->inner.has_last)
    return fail(ctx, MLH_ERR_INVALID, "batched_fold_step already applied");
  const fe *tlo, *thi;
  MLH_TRY(fold_tables_g(ctx, g, log_gen_pows, &tlo, &thi));
  memcpy(ctx->pinned, bp->fr, 16);
  memcpy(ctx->pinned + 16, r, 16);
  fe* sc = reinterpret_cast<fe*>(bp->scal);
  HIP_TRY(ctx, hipMemcpyAsync(sc, ctx->pinned, 32, hipMemcpyHostToDevice, ctx->stream));
  PoolBuf vb(ctx), tb(ctx);  // released into fri_data on success only
  MLH_TRY(vb.alloc(half_n * sizeof(fe)));
  void* vals = vb.p;
  if (half_n == (1ull << MLH_LOG_BLOWUP)) {  // batched_fri.rs:152-162
    HIP_TRY(ctx, launch_batched_fold_leaves(bp->codes, bp->m, N, sc, sc + 1, tlo, thi,
                                            reinterpret_cast<fe*>(vals), nullptr, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->pinned, vals, 32, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (memcmp(ctx->pinned, ctx->pinned + 16, 16) != 0)
      return fail(ctx, MLH_ERR_NOT_RS_CODE, "not an RS code");
    memcpy(bp->inner.last, ctx->pinned, 16);
    bp->inner.has_last = true;
    mlh_transcript_absorb(tr, bp->inner.last, 16);
    return MLH_OK;
  }
  FriLayer nx;
  nx.log_n = bp->log_code - 1;
  nx.values = reinterpret_cast<const fe*>(vals);
  const uint64_t leaves = half_n / 2;
  MLH_TRY(tb.alloc(mlh_merkle_layers_bytes(leaves)));
  nx.tree = tb.as<uint8_t>();
  HIP_TRY(ctx, launch_batched_fold_leaves(bp->codes, bp->m, N, sc, sc + 1, tlo, thi,
                                          reinterpret_cast<fe*>(vals), nx.tree, ctx->stream));
  HIP_TRY(ctx, launch_merkle_levels(nx.tree, leaves, ctx->stream));
  MLH_TRY(read_root(ctx, nx.tree, leaves, nx.root));
  nx.owned_values = vb.release();  // owned by fri_data from here on (its destructor frees them)
  tb.release();
  bp->inner.layers.push_back(nx);
  mlh_transcript_absorb(tr, bp->inner.layers.back().root, 32);
  return MLH_OK;
}

mlh_fri_prover* mlh_batched_fri_prover_inner(mlh_batched_fri_prover* bp) {
  return bp ? &bp->inner : nullptr;
}

mlh_status mlh_batched_fri_prover_batch_root(const mlh_batched_fri_prover* bp, uint8_t out[32]) {
  if (!bp || !out) return MLH_ERR_INVALID;
  memcpy(out, bp->broot, 32);
  return MLH_OK;
}

mlh_status mlh_batched_fri_prover_fingerprint_r(const mlh_batched_fri_prover* bp, uint8_t out[16]) {
  if (!bp || !out) return MLH_ERR_INVALID;
  memcpy(out, bp->fr, 16);
  return MLH_OK;
}

mlh_status mlh_batched_fri_prover_open_query(mlh_ctx* ctx, const mlh_batched_fri_prover* bp,
                                             uint64_t index, uint8_t* out) {
  if (!ctx || !bp || !out) return fail(ctx, MLH_ERR_INVALID, "null argument");
  const uint32_t L = bp->log_code;
  if (index >= (1ull << (L - 1))) return fail(ctx, MLH_ERR_INVALID, "index out of bounds");
  const uint64_t qbytes = mlh_batched_fri_query_bytes(L, bp->m);
  uint8_t* h;
  MLH_TRY(query_stage(ctx, qbytes, &h));
  mlh::QueryIdx qi;
  memset(&qi, 0, sizeof(qi));
  qi.v[0] = index;
  HIP_TRY(ctx, launch_batch_queries(bp->codes, bp->m, 1ull << L, reinterpret_cast<const uint8_t*>(bp->btree),
                                    qi, 1, qbytes, h, ctx->stream));
  // the inner paths at index mod N/4 (batched_fri.rs:215-221; the gather
  // reduces the index per tree); zero where the inner prover has fewer trees
  const uint64_t base = 32ull * bp->m + 32ull * (L - 1);
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  memset(h + base, 0, qbytes - base);
  MLH_TRY(gather_queries_dev(ctx, &bp->inner, qi, nullptr, 1, qbytes, base, h));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  memcpy(out, h, qbytes);
  return MLH_OK;
}

void mlh_batched_fri_prover_destroy(mlh_batched_fri_prover* bp) {
  if (bp) {
    (void)hipStreamSynchronize(bp->ctx->stream);
    delete bp;
  }
}

mlh_status mlh_batched_pcs_prove(mlh_ctx* ctx, const void* dev_evals, uint32_t num_polys,
                                 uint32_t n_vars, const uint8_t* inputs, const uint8_t* outputs,
                                 mlh_transcript* tr, mlh_batched_pcs_proof* proof) {
  if (!ctx || !dev_evals || !inputs || !outputs || !tr || !proof)
    return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (num_polys == 0) return fail(ctx, MLH_ERR_INVALID, "no polynomials");
  if (n_vars < 1 || n_vars > 36) return fail(ctx, MLH_ERR_INVALID, "n_vars out of range");
  const uint32_t log_domain = n_vars + MLH_LOG_BLOWUP;
  const uint64_t n = 1ull << n_vars, N = 2 * n;
  uint8_t genb[16];
  h_store(genb, h_pow2_generator(log_domain));
  // codes: to_coefficient, bit reverse, RS per polynomial (batched_pcs.rs:137-146)
  PoolBuf coeffs(ctx), codes(ctx), matrix(ctx), outs(ctx);
  MLH_TRY(coeffs.alloc(n * 16));
  MLH_TRY(codes.alloc((uint64_t)num_polys * N * 16));
  MLH_TRY(matrix.alloc(n * 16));
  MLH_TRY(outs.alloc(16ull * num_polys));
  const uint8_t* ev = reinterpret_cast<const uint8_t*>(dev_evals);
  for (uint32_t j = 0; j < num_polys; ++j) {
    HIP_TRY(ctx, launch_mobius(coeffs.as<fe>(), n_vars, false, ctx->stream,
                               reinterpret_cast<const fe*>(ev + (uint64_t)j * n * 16)));
    MLH_TRY(mlh_reed_solomon_brev(ctx, coeffs.p, n_vars, genb,
                                  codes.as<uint8_t>() + (uint64_t)j * N * 16));
  }
  // init (batched_pcs.rs:36-78): absorb the claim, batched FRI init.  The
  // replay check is armed first: any failure from here on restores the
  // caller's transcript to its state at entry.
  ReplayCheck rc(ctx, tr);
  for (uint32_t i = 0; i < n_vars; ++i) rc.absorb(inputs + 16 * i, 16);
  for (uint32_t j = 0; j < num_polys; ++j) rc.absorb(outputs + 16 * j, 16);
  std::unique_ptr<mlh_fri_prover> fp(new mlh_fri_prover());
  fp->ctx = ctx;
  fp->log_code = log_domain;
  FriDevLoop lp(ctx, fp.get());
  device_arm(ctx);
  const bool fused = n_vars <= ctx->pcs_fused_max;
  MLH_TRY(lp.init_batched(codes.as<fe>(), num_polys, log_domain, tr, false, fused ? 5 : 0));
  // fingerprinted MLE + eq table; previous_sum = fingerprint(fr, outputs)
  HIP_TRY(ctx, launch_fingerprint(reinterpret_cast<const fe*>(dev_evals), num_polys, n, lp.fr(),
                                  matrix.as<fe>(), ctx->stream));
  {
    std::vector<uint8_t> ob(outputs, outputs + 16ull * num_polys);
    HIP_TRY(ctx, hipMemcpyAsync(outs.p, ob.data(), ob.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // ob is pageable and goes out of scope
  }
  HIP_TRY(ctx, launch_fingerprint_scalar(outs.as<fe>(), num_polys, lp.fr(), lp.prev(), ctx->stream));
  if (fused) {  // (batched_pcs.rs:80-125) the PCS rounds off the transcript chain (PcsRounds)
    PcsRounds pr(ctx, lp);
    fe* mt = matrix.as<fe>();  // the fingerprinted table is ours: its folds run in place
    MLH_TRY(pr.init(mt, mt, n_vars, inputs, nullptr, lp.prev()));
    HIP_TRY(ctx, launch_transcript_absorb(lp.dt(), reinterpret_cast<const uint8_t*>(lp.poly(0)), 32,
                                          lp.r(0), ctx->stream));  // (c1, c2)_0 -> r_0
    for (uint32_t k = 0; k < n_vars; ++k) {
      const uint32_t kn = k + 1;
      PcsJob job{};
      if (kn < n_vars) MLH_TRY(pr.job(kn, &job));
      if (k == 0) {  // the batched step: round 1 as its own launch before its tree's root absorb
        if (kn < n_vars)
          HIP_TRY(ctx, launch_pcs_round(job.src, job.dst, job.log_h, job.fold != 0, job.r_prev, job.p_prev,
                                        job.p_k, job.e, job.st, job.poly_out, ctx->stream));
        MLH_TRY(lp.step_batched(lp.r(0), kn < n_vars, kn < n_vars ? lp.poly(1) : nullptr));
      } else {
        MLH_TRY(lp.step(k, lp.r(k), kn < n_vars, kn < n_vars ? lp.poly(kn) : nullptr,
                        kn < n_vars ? &job : nullptr));
      }
    }
  } else {
    EqSumcheck es(ctx);  // delta = eq(inputs), factored
    MLH_TRY(es.init(matrix.as<fe>(), nullptr, n_vars, inputs));
    uint32_t np = 0;
    MLH_TRY(es.first_sums(&np));
    for (uint32_t k = 0; k < n_vars; ++k) {  // fold (batched_pcs.rs:80-125)
      MLH_TRY(es.round(k, np, lp.prev(), lp.dt(), lp.poly(k), lp.r(k)));
      MLH_TRY(es.fold(k, lp.r(k), &np));
      if (k == 0)
        MLH_TRY(lp.step_batched(lp.r(0), false));
      else
        MLH_TRY(lp.step(k, lp.r(k), false));
    }
  }
  MLH_TRY(lp.finish(32ull * n_vars));
  // host transcript replay
  const uint8_t* polys = lp.host_polys();
  if (proof->sumcheck_polys) memcpy(proof->sumcheck_polys, polys, 32ull * n_vars);
  rc.absorb(lp.host_broot(), 32);
  rc.expect(lp.host_fr());
  rc.absorb(lp.host_fr(), 16);
  for (uint32_t k = 0; k < n_vars; ++k) {
    rc.absorb(polys + 32 * k, 16);
    rc.absorb(polys + 32 * k + 16, 16);
    rc.expect(lp.host_r(k));
    if (k < fp->layers.size())
      rc.absorb(fp->layers[k].root, 32);
    else
      rc.absorb(fp->last, 16);
  }
  MLH_TRY(rc.status());
  memcpy(proof->fri.batch_commitment, lp.host_broot(), 32);
  return batched_queries(ctx, lp, tr, &proof->fri);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// device-resident transcript + sharded steps that read the challenge from HBM
// (tests/dist_spec.py fri_prove: no host round trip inside the fold loop)
// ---------------------------------------------------------------------------
extern "C" {

uint64_t mlh_device_transcript_bytes(void) { return 128; }

mlh_status mlh_transcript_to_device(mlh_ctx* ctx, const mlh_transcript* tr, void* dev_state) {
  if (!ctx || !tr || !dev_state) return fail(ctx, MLH_ERR_INVALID, "null argument");
  std::vector<uint8_t> b(sizeof(DevSha));
  memcpy(b.data(), &tr->sha, sizeof(DevSha));
  HIP_TRY(ctx, hipMemcpyAsync(dev_state, b.data(), sizeof(DevSha), hipMemcpyHostToDevice,
                              ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MLH_OK;
}

mlh_status mlh_transcript_from_device(mlh_ctx* ctx, const void* dev_state, mlh_transcript* tr) {
  if (!ctx || !tr || !dev_state) return fail(ctx, MLH_ERR_INVALID, "null argument");
  HIP_TRY(ctx, hipMemcpyAsync(ctx->pinned, dev_state, sizeof(DevSha), hipMemcpyDeviceToHost,
                              ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  memcpy(&tr->sha, ctx->pinned, sizeof(DevSha));
  return MLH_OK;
}

mlh_status mlh_device_transcript_absorb(mlh_ctx* ctx, void* dev_state, const void* dev_src,
                                        uint32_t n, void* dev_challenge) {
  if (!ctx || !dev_state || (n && !dev_src)) return fail(ctx, MLH_ERR_INVALID, "null argument");
  HIP_TRY(ctx, launch_transcript_absorb(reinterpret_cast<DevSha*>(dev_state),
                                        reinterpret_cast<const uint8_t*>(dev_src), n,
                                        reinterpret_cast<fe*>(dev_challenge), ctx->stream));
  return MLH_OK;
}

mlh_status mlh_device_fri_last(mlh_ctx* ctx, const void* dev_vals2, void* dev_state,
                               void* dev_flag, void* dev_last) {
  if (!ctx || !dev_vals2 || !dev_state || !dev_flag || !dev_last)
    return fail(ctx, MLH_ERR_INVALID, "null argument");
  HIP_TRY(ctx, launch_fri_last(reinterpret_cast<const fe*>(dev_vals2),
                               reinterpret_cast<DevSha*>(dev_state),
                               reinterpret_cast<uint32_t*>(dev_flag),
                               reinterpret_cast<fe*>(dev_last), ctx->stream));
  return MLH_OK;
}

mlh_status mlh_shard_fri_fold_dr(mlh_ctx* ctx, const void* dev_layer, uint32_t log_local,
                                 uint32_t k, uint32_t log_domain, const void* dev_r,
                                 void* dev_next, uint32_t log_s, uint32_t log_p, uint32_t rank) {
  ShardMap m;
  const uint8_t dummy[16] = {0};
  MLH_TRY(shard_fold_args(ctx, dev_layer, dev_next, dummy, log_local, k, log_domain, log_s, log_p,
                          rank, &m));
  if (!dev_r) return fail(ctx, MLH_ERR_INVALID, "null argument");
  const fe *tlo, *thi;
  MLH_TRY(fold_tables(ctx, log_domain, &tlo, &thi));
  HIP_TRY(ctx, launch_fri_fold(reinterpret_cast<const fe*>(dev_layer), 1ull << log_local,
                               reinterpret_cast<fe*>(dev_next), fe{}, tlo, thi, k,
                               1ull << log_domain, ctx->stream, m,
                               reinterpret_cast<const fe*>(dev_r)));
  return MLH_OK;
}

mlh_status mlh_shard_fri_fold_commit_dr(mlh_ctx* ctx, const void* dev_layer, uint32_t log_local,
                                        uint32_t k, uint32_t log_domain, const void* dev_r,
                                        void* dev_next, void* dev_tree, uint32_t log_s,
                                        uint32_t log_p, uint32_t rank) {
  ShardMap m;
  const uint8_t dummy[16] = {0};
  MLH_TRY(shard_fold_args(ctx, dev_layer, dev_next, dummy, log_local, k, log_domain, log_s, log_p,
                          rank, &m));
  if (!dev_tree || !dev_r) return fail(ctx, MLH_ERR_INVALID, "null argument");
  if (log_local < 2 || (log_p && log_s + 2 > log_local))
    return fail(ctx, MLH_ERR_INVALID, "folded layer's pairs are not local");
  const fe *tlo, *thi;
  MLH_TRY(fold_tables(ctx, log_domain, &tlo, &thi));
  uint8_t* tree = reinterpret_cast<uint8_t*>(dev_tree);
  HIP_TRY(ctx, launch_fri_fold_commit(reinterpret_cast<const fe*>(dev_layer), 1ull << log_local,
                                      reinterpret_cast<fe*>(dev_next), tree, fe{}, tlo, thi, k,
                                      1ull << log_domain, ctx->stream, m,
                                      reinterpret_cast<const fe*>(dev_r)));
  return MLH_OK;
}

mlh_status mlh_merkle_top(mlh_ctx* ctx, const void* dev_gathered, uint32_t P, uint64_t per_rank,
                          void* dev_levels) {
  if (!ctx || !dev_gathered || !dev_levels) return fail(ctx, MLH_ERR_INVALID, "null argument");
  const uint64_t n = (uint64_t)P * per_rank;
  if (!is_pow2(n)) return fail(ctx, MLH_ERR_NOT_POW2, "top tree size must be a power of two");
  uint8_t* lv = reinterpret_cast<uint8_t*>(dev_levels);
  HIP_TRY(ctx, launch_top_reorder(reinterpret_cast<const uint8_t*>(dev_gathered), P, per_rank, lv,
                                  ctx->stream));
  HIP_TRY(ctx, launch_merkle_levels(lv, n, ctx->stream));
  return MLH_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// device-resident sumcheck steps (sharded sumcheck in tests/dist_spec.py)
// ---------------------------------------------------------------------------
extern "C" {

mlh_status mlh_sumcheck_sums_dev(mlh_ctx* ctx, const void* dev_matrix, const void* dev_delta,
                                 uint32_t log_height, void* dev_sums) {
  if (!ctx || !dev_matrix || !dev_delta || !dev_sums || log_height < 1 || log_height > 40)
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  HIP_TRY(ctx, launch_sums(reinterpret_cast<const fe*>(dev_matrix),
                           reinterpret_cast<const fe*>(dev_delta), 1ull << (log_height - 1),
                           ctx->partials, reinterpret_cast<fe*>(dev_sums), ctx->stream));
  return MLH_OK;
}

mlh_status mlh_sumcheck_fold_sums_dr(mlh_ctx* ctx, void* dev_matrix, void* dev_delta,
                                     uint32_t log_height, const void* dev_r, void* dev_sums) {
  if (!ctx || !dev_matrix || !dev_delta || !dev_r || !dev_sums || log_height < 2 ||
      log_height > 40)
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  HIP_TRY(ctx, launch_fold_sums(reinterpret_cast<fe*>(dev_matrix), reinterpret_cast<fe*>(dev_delta),
                                1ull << log_height, fe{}, ctx->partials,
                                reinterpret_cast<fe*>(dev_sums), ctx->stream,
                                reinterpret_cast<const fe*>(dev_r)));
  return MLH_OK;
}

mlh_status mlh_sumcheck_fold_dr(mlh_ctx* ctx, void* dev_matrix, void* dev_delta,
                                uint32_t log_height, const void* dev_r) {
  if (!ctx || !dev_matrix || !dev_delta || !dev_r || log_height < 1 || log_height > 40)
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  HIP_TRY(ctx, launch_fold(reinterpret_cast<fe*>(dev_matrix), reinterpret_cast<fe*>(dev_delta),
                           1ull << log_height, fe{}, ctx->stream,
                           reinterpret_cast<const fe*>(dev_r)));
  return MLH_OK;
}

mlh_status mlh_device_sumcheck_round(mlh_ctx* ctx, const void* dev_sum_pairs, uint32_t npairs,
                                     void* dev_prev, void* dev_state, void* dev_poly_out,
                                     void* dev_r_out) {
  if (!ctx || !dev_sum_pairs || !dev_prev || !dev_state || !dev_poly_out || !dev_r_out ||
      npairs == 0)
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  HIP_TRY(ctx, launch_sumcheck_round(reinterpret_cast<const fe*>(dev_sum_pairs), npairs,
                                     reinterpret_cast<fe*>(dev_prev),
                                     reinterpret_cast<DevSha*>(dev_state),
                                     reinterpret_cast<fe*>(dev_poly_out),
                                     reinterpret_cast<fe*>(dev_r_out), ctx->stream));
  return MLH_OK;
}

}  // extern "C"
