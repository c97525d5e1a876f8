// Multi-GPU orchestration behind the C ABI: one process per GPU, the exchange
// steps through a pluggable transport (mlh_transport) whose built-in
// implementation is RCCL over xGMI (mlh_comm, librccl).  The reference has no
// distributed API (its prover is single-threaded: src/ntt/mod.rs:69-173,
// src/fri/mod.rs:19-145 and :261-285, sumcheck.rs:77-247); SURVEY.md 8(e)
// prescribes the sharding, DESIGN.md §6 describes the layouts.  This is the
// one product implementation of the schedules (a Rust caller binds it
// directly); tests/dist_spec.py restates them in Python as the executable spec
// the CPU gloo tests run with oracle rank-local steps.
//
// Layout: a sharded vector of 2^log_n elements over P = 2^log_p ranks is
// block-cyclic with block S = 2^log_s: local l of rank r is global
// ((l >> log_s) << (log_s + log_p)) | (r << log_s) | (l mod S).
//   * NTT / RS: cyclic in (S = 1), block 2^log_n / P^2 out, ONE all-to-all.
//   * FRI prove: block layout; every pair (i, i + n/2) and every aligned run of
//     S leaves is local; per layer one all-gather of the subtree roots; a layer
//     whose local part becomes one block is re-dealt by one all-to-all (or
//     gathered below gather_log and finished replicated); transcript
//     replicated in HBM; queries opened by the owner, combined by one gather.
//   * Sumcheck: cyclic (rank r holds index l P + r); folds are local while the
//     local table has >= 2 entries; the per-rank round sums are all-gathered
//     and a device kernel adds them; the last log P rounds run replicated.
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "context.hpp"
#include "fused_ntt.hpp"
#include "host_sha256.hpp"
#include "host_transcript.hpp"

using namespace mlh;

// ---------------------------------------------------------------------------
// RCCL communicator and the transport wrapper
// ---------------------------------------------------------------------------
struct mlh_comm {
  ncclComm_t comm = nullptr;
  int device = 0;
  uint32_t world = 1, rank = 0;
};

static int rccl_all_to_all(void* user, const void* send, void* recv, uint64_t bytes_per_rank,
                           void* stream) {
  mlh_comm* c = static_cast<mlh_comm*>(user);
  return ncclAllToAll(send, recv, (size_t)bytes_per_rank, ncclUint8, c->comm,
                      static_cast<hipStream_t>(stream)) == ncclSuccess
             ? 0
             : 1;
}

static int rccl_all_gather(void* user, const void* send, void* recv, uint64_t bytes, void* stream) {
  mlh_comm* c = static_cast<mlh_comm*>(user);
  return ncclAllGather(send, recv, (size_t)bytes, ncclUint8, c->comm,
                       static_cast<hipStream_t>(stream)) == ncclSuccess
             ? 0
             : 1;
}

namespace {

uint32_t log2u(uint64_t v) { return 63 - __builtin_clzll(v); }

// Collectives of one sharded call on the context's stream.
struct Tp {
  mlh_ctx* ctx;
  const mlh_transport* t;
  uint32_t P, p, rank;
  Tp(mlh_ctx* c, const mlh_transport* tr)
      : ctx(c), t(tr), P(tr->world), p(log2u(tr->world)), rank(tr->rank) {}
  mlh_status prep() {
    if (t->host_side) HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return MLH_OK;
  }
  // chunk i (bytes_per_rank) of send goes to rank i; chunk i of recv came from rank i
  // lab (optional): a kernel-timer label (mlh_profile_*) for the exchange
  mlh_status all_to_all(const void* send, void* recv, uint64_t bytes_per_rank,
                        const char* lab = nullptr) {
    MLH_TRY(prep());
    auto go = [&]() { return t->all_to_all(t->user, send, recv, bytes_per_rank, ctx->stream); };
    int rc;
    if (lab) {
      ProfScope ps(ctx, lab);
      rc = go();
      ps.end();
    } else {
      rc = go();
    }
    if (rc != 0) return fail(ctx, MLH_ERR_COMM, "transport all_to_all failed");
    return MLH_OK;
  }
  // recv = concatenation over ranks (rank order) of every rank's `bytes`
  mlh_status all_gather(const void* send, void* recv, uint64_t bytes) {
    MLH_TRY(prep());
    if (t->all_gather(t->user, send, recv, bytes, ctx->stream) != 0)
      return fail(ctx, MLH_ERR_COMM, "transport all_gather failed");
    return MLH_OK;
  }
};

mlh_status check_transport(mlh_ctx* ctx, const mlh_transport* t) {
  if (!t || !t->all_to_all || !t->all_gather) return fail(ctx, MLH_ERR_INVALID, "null transport");
  if (t->world == 0 || t->world > 16 || (t->world & (t->world - 1)) || t->rank >= t->world)
    return fail(ctx, MLH_ERR_INVALID, "world must be a power of two <= 16, rank < world");
  return MLH_OK;
}

// Device buffers owned by one sharded call, released to the context pool.
struct Bufs {
  mlh_ctx* ctx;
  std::vector<void*> held;
  explicit Bufs(mlh_ctx* c) : ctx(c) {}
  ~Bufs() {
    for (void* p : held) pool_free(ctx, p);
  }
  template <class T>
  mlh_status get(size_t bytes, T** out) {
    void* p = nullptr;
    MLH_TRY(pool_alloc(ctx, bytes ? bytes : 16, &p));
    held.push_back(p);
    *out = static_cast<T*>(p);
    return MLH_OK;
  }
};

void store_fe(uint8_t out[16], u128 v) { h_store(out, v); }

// gen has order exactly 2^log_n (the cross-shard DFT needs a DFT generator)
// The side streams of the pipelined sharded calls (lazy).  (Giving the
// exchange stream the device's highest priority measured no change in
// tools/shard_step_emul.py: 0.766-0.769 vs 0.763 ms a step; not kept.)
mlh_status ensure_side_streams(mlh_ctx* ctx) {
  if (!ctx->side) HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
  if (!ctx->side2) HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->side2, hipStreamNonBlocking));
  return MLH_OK;
}

bool gen_has_order(u128 gen, uint32_t log_n) {
  if (gen >= kModulus) return false;
  if (log_n == 0) return gen == 1;
  return h_pow(gen, (u128)1 << (log_n - 1)) == kModulus - 1;
}

}  // namespace

extern "C" {

mlh_status mlh_comm_unique_id(uint8_t out[128]) {
  if (!out) return MLH_ERR_INVALID;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return MLH_ERR_COMM;
  static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
  memcpy(out, &id, 128);
  return MLH_OK;
}

mlh_status mlh_comm_create(mlh_ctx* ctx, uint32_t world, uint32_t rank, const uint8_t id[128],
                           mlh_comm** out) {
  if (!ctx || !id || !out || world == 0 || rank >= world) return MLH_ERR_INVALID;
  *out = nullptr;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  ncclUniqueId uid;
  memcpy(&uid, id, 128);
  std::unique_ptr<mlh_comm> c(new mlh_comm());
  c->device = ctx->device;
  c->world = world;
  c->rank = rank;
  const ncclResult_t r = ncclCommInitRank(&c->comm, (int)world, uid, (int)rank);
  if (r != ncclSuccess) return fail(ctx, MLH_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  *out = c.release();
  return MLH_OK;
}

void mlh_comm_destroy(mlh_comm* c) {
  if (!c) return;
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
}

mlh_status mlh_comm_info(mlh_comm* c, uint32_t* count, uint32_t* rank, int* device) {
  if (!c || !c->comm) return MLH_ERR_INVALID;
  int n = 0, r = 0, d = -1;
  if (ncclCommCount(c->comm, &n) != ncclSuccess || ncclCommUserRank(c->comm, &r) != ncclSuccess ||
      ncclCommCuDevice(c->comm, &d) != ncclSuccess)
    return MLH_ERR_COMM;
  if (count) *count = (uint32_t)n;
  if (rank) *rank = (uint32_t)r;
  if (device) *device = d;
  return MLH_OK;
}

mlh_status mlh_comm_transport(mlh_comm* c, mlh_transport* out) {
  if (!c || !out) return MLH_ERR_INVALID;
  out->world = c->world;
  out->rank = c->rank;
  out->host_side = 0;
  out->user = c;
  out->all_to_all = rccl_all_to_all;
  out->all_gather = rccl_all_gather;
  return MLH_OK;
}

// ---------------------------------------------------------------------------
// Transport pre-flight: one all-to-all and one all-gather of a rank-tagged
// pattern, checked on the device.  A multi-GPU caller runs it before its first
// data-path collective, so a miswired or stalled transport shows up as a
// named failure (and a watchdog can say which phase hung) instead of a wrong
// proof.  Word i of the chunk rank s sends to rank d is pf_word(s, d, i); the
// all-gather sends pf_word(s, kPfGather, i).
// ---------------------------------------------------------------------------
namespace {

constexpr uint32_t kPfGather = 0xA5u;

__device__ __forceinline__ uint32_t pf_word(uint32_t src, uint32_t dst, uint32_t i) {
  uint32_t x = src * 0x9E3779B1u ^ (dst + 0x7F4A7C15u) * 0x85EBCA77u ^ i * 0xC2B2AE3Du;
  x ^= x >> 15;
  x *= 0x2C1B3C6Du;
  x ^= x >> 12;
  return x;
}

__global__ void __launch_bounds__(256)
pf_fill_kernel(uint32_t* a2a_send, uint32_t* ag_send, uint32_t words, uint32_t P, uint32_t rank) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= words) return;
  for (uint32_t d = 0; d < P; ++d) a2a_send[(uint64_t)d * words + i] = pf_word(rank, d, i);
  ag_send[i] = pf_word(rank, kPfGather, i);
}

__global__ void __launch_bounds__(256)
pf_check_kernel(const uint32_t* a2a_recv, const uint32_t* ag_recv, uint32_t words, uint32_t P,
                uint32_t rank, unsigned long long* bad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= words) return;
  unsigned long long n = 0;
  for (uint32_t s = 0; s < P; ++s) {
    n += a2a_recv[(uint64_t)s * words + i] != pf_word(s, rank, i);
    n += ag_recv[(uint64_t)s * words + i] != pf_word(s, kPfGather, i);
  }
  if (n) atomicAdd(bad, n);
}

}  // namespace

extern "C" mlh_status mlh_comm_preflight(mlh_ctx* ctx, const mlh_transport* tp, uint64_t bytes_per_rank,
                                         uint64_t* mismatches, float* ms) {
  if (!ctx || !mismatches) return fail(ctx, MLH_ERR_INVALID, "null argument");
  MLH_TRY(check_transport(ctx, tp));
  if (bytes_per_rank == 0 || bytes_per_rank % 4 || bytes_per_rank > (1ull << 30))
    return fail(ctx, MLH_ERR_INVALID, "preflight chunk must be a non-zero multiple of 4 B, <= 1 GiB");
  Tp T(ctx, tp);
  const uint32_t P = T.P, words = (uint32_t)(bytes_per_rank / 4);
  Bufs B(ctx);
  uint32_t *send, *recv, *ags, *agr;
  unsigned long long* bad;
  MLH_TRY(B.get(bytes_per_rank * P, &send));
  MLH_TRY(B.get(bytes_per_rank * P, &recv));
  MLH_TRY(B.get(bytes_per_rank, &ags));
  MLH_TRY(B.get(bytes_per_rank * P, &agr));
  MLH_TRY(B.get(16, &bad));
  HIP_TRY(ctx, hipMemsetAsync(bad, 0, 8, ctx->stream));
  HIP_TRY(ctx, hipMemsetAsync(recv, 0, bytes_per_rank * P, ctx->stream));
  HIP_TRY(ctx, hipMemsetAsync(agr, 0, bytes_per_rank * P, ctx->stream));
  const unsigned grid = (words + 255) / 256;
  hipLaunchKernelGGL(pf_fill_kernel, dim3(grid), dim3(256), 0, ctx->stream, send, ags, words, P, T.rank);
  HIP_TRY(ctx, hipGetLastError());
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ms) {
    HIP_TRY(ctx, hipEventCreate(&e0));
    HIP_TRY(ctx, hipEventCreate(&e1));
    HIP_TRY(ctx, hipEventRecord(e0, ctx->stream));
  }
  mlh_status st = T.all_to_all(send, recv, bytes_per_rank);
  if (st == MLH_OK) st = T.all_gather(ags, agr, bytes_per_rank);
  if (st == MLH_OK && ms) {
    if (T.t->host_side) (void)hipStreamSynchronize(ctx->stream);
    (void)hipEventRecord(e1, ctx->stream);
  }
  if (st == MLH_OK) {
    hipLaunchKernelGGL(pf_check_kernel, dim3(grid), dim3(256), 0, ctx->stream, recv, agr, words, P, T.rank,
                       bad);
    if (hipGetLastError() != hipSuccess) st = fail(ctx, MLH_ERR_HIP, "preflight check launch");
  }
  unsigned long long h = 0;
  if (st == MLH_OK && hipMemcpyAsync(ctx->pinned, bad, 8, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
    st = fail(ctx, MLH_ERR_HIP, "preflight copy");
  if (hipStreamSynchronize(ctx->stream) != hipSuccess && st == MLH_OK) st = fail(ctx, MLH_ERR_HIP, "preflight sync");
  if (st == MLH_OK) {
    memcpy(&h, ctx->pinned, 8);
    *mismatches = h;
    if (ms) (void)hipEventElapsedTime(ms, e0, e1);
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  return st;
}

// ---------------------------------------------------------------------------
// NTT / INTT / Reed-Solomon (ntt/mod.rs:69-173, fri/mod.rs:19-28)
// ---------------------------------------------------------------------------
// X[j + M t] = sum_g wP^(g t) w^(g j) Z_g[j], Z_g = NTT_M(x[g + P .]) with
// generator w^P, M = N / P: local NTT, all-to-all of the M/P-element chunks,
// cross-shard DFT (mlh_shard_ntt_cross).
mlh_status mlh_sharded_ntt(mlh_ctx* ctx, const mlh_transport* t, const void* dev_in, void* dev_out,
                           uint32_t log_n, const uint8_t gen[16], int inverse) {
  if (!ctx || !dev_in || !dev_out || !gen) return fail(ctx, MLH_ERR_INVALID, "null argument");
  MLH_TRY(check_transport(ctx, t));
  Tp tp(ctx, t);
  if (tp.P == 1)
    return inverse ? mlh_intt(ctx, dev_in, dev_out, log_n, gen) : mlh_ntt(ctx, dev_in, dev_out, log_n, gen);
  if (log_n < 2 * tp.p + 1 || log_n > 40)
    return fail(ctx, MLH_ERR_INVALID, "sharded NTT needs 2^log_n >= 2 P^2");
  if (!gen_has_order(h_load(gen), log_n))  // before any local work or collective
    return fail(ctx, MLH_ERR_BAD_GENERATOR, "generator order != n");
  const uint64_t M = 1ull << (log_n - tp.p);
  uint8_t gp[16];
  store_fe(gp, h_pow(h_load(gen), (u128)tp.P));
  Bufs b(ctx);
  fe *z, *recv;
  MLH_TRY(b.get(M * 16, &z));
  MLH_TRY(b.get(M * 16, &recv));
  if (!inverse) {
    MLH_TRY(mlh_ntt(ctx, dev_in, z, log_n - tp.p, gp));
    MLH_TRY(tp.all_to_all(z, recv, M / tp.P * 16, "ntt_all_to_all"));
    MLH_TRY(mlh_shard_ntt_cross(ctx, recv, dev_out, log_n, tp.p, tp.rank, gen, 0));
  } else {
    MLH_TRY(mlh_shard_ntt_cross(ctx, dev_in, z, log_n, tp.p, tp.rank, gen, 1));
    MLH_TRY(tp.all_to_all(z, recv, M / tp.P * 16));
    MLH_TRY(mlh_intt(ctx, recv, dev_out, log_n - tp.p, gp));
  }
  return MLH_OK;
}

// `count` transforms, pipelined over three streams: the first local step A
// (forward: the local NTT; inverse: the cross-shard DFT) on the context
// stream, the exchange on the side stream, the second local step C
// (forward: the cross-shard DFT; inverse: the local INTT) on a third stream.
// So A(i+1), the exchange of i and C(i-1) run at once, and a step costs about
// max(A || C, exchange): the VALU-bound NTT and the HBM-bound cross-shard DFT
// share the chip better side by side than in turn (0.566 ms
// against 0.584 ms for the 2^24 NTT + the P = 8 cross step on one MI355X), and
// C no longer sits behind the exchange on its stream (0.58-0.74 ms a step at
// P = 8 for the xGMI rates assumed there).  Buffers: z[k] (A's output, sent)
// and recv[k] (received, C's input), k = i mod 2; A(i+2) reuses z[k] after
// the exchange of i sent it; the exchange of i+2 fills recv[k] after C(i) has
// read it.  On return the context stream is ordered after every transform.
// With a host-side transport the transforms run one after another.
mlh_status mlh_sharded_ntt_batch(mlh_ctx* ctx, const mlh_transport* t, const void* const* dev_in,
                                 void* const* dev_out, uint32_t count, uint32_t log_n,
                                 const uint8_t gen[16], int inverse) {
  if (!ctx || (count && (!dev_in || !dev_out)) || !gen) return fail(ctx, MLH_ERR_INVALID, "null argument");
  MLH_TRY(check_transport(ctx, t));
  for (uint32_t i = 0; i < count; ++i)
    if (!dev_in[i] || !dev_out[i]) return fail(ctx, MLH_ERR_INVALID, "null argument");
  Tp tp(ctx, t);
  if (tp.P == 1 || t->host_side) {
    for (uint32_t i = 0; i < count; ++i)
      MLH_TRY(mlh_sharded_ntt(ctx, t, dev_in[i], dev_out[i], log_n, gen, inverse));
    return MLH_OK;
  }
  if (log_n < 2 * tp.p + 1 || log_n > 40)
    return fail(ctx, MLH_ERR_INVALID, "sharded NTT needs 2^log_n >= 2 P^2");
  if (!gen_has_order(h_load(gen), log_n)) return fail(ctx, MLH_ERR_BAD_GENERATOR, "generator order != n");
  if (!count) return MLH_OK;
  MLH_TRY(ensure_side_streams(ctx));
  const uint64_t M = 1ull << (log_n - tp.p);
  uint8_t gp[16];
  store_fe(gp, h_pow(h_load(gen), (u128)tp.P));
  Bufs b(ctx);
  fe *z[2], *recv[2];
  for (int k = 0; k < 2; ++k) {
    MLH_TRY(b.get(M * 16, &z[k]));
    MLH_TRY(b.get(M * 16, &recv[k]));
  }
  hipEvent_t a_done[2], x_done[2], c_done[2];
  for (int k = 0; k < 2; ++k) {
    a_done[k] = take_event(ctx);
    x_done[k] = take_event(ctx);
    c_done[k] = take_event(ctx);
  }
  struct Recycle {  // the events go back to the context's free list
    mlh_ctx* c;
    hipEvent_t* e;
    ~Recycle() {
      for (int k = 0; k < 9; ++k) c->ev_free.push_back(e[k]);
    }
  };
  hipEvent_t evs[9] = {a_done[0], a_done[1], x_done[0], x_done[1], c_done[0], c_done[1],
                       take_event(ctx), take_event(ctx), take_event(ctx)};
  Recycle rec{ctx, evs};
  hipStream_t main = ctx->stream, side = ctx->side, third = ctx->side2;
  // the third stream starts after the caller's work (the side stream's first
  // wait is on a_done, recorded on the context stream)
  HIP_TRY(ctx, hipEventRecord(evs[8], main));
  HIP_TRY(ctx, hipStreamWaitEvent(third, evs[8], 0));
  // On every exit, error paths included, the context stream waits for all the
  // side streams' work: the pooled buffers (Bufs, released after this guard)
  // and the events are reused only behind it.
  struct JoinSide {
    hipStream_t main, s1, s2;
    hipEvent_t e1, e2;
    ~JoinSide() {
      (void)hipEventRecord(e1, s1);
      (void)hipStreamWaitEvent(main, e1, 0);
      (void)hipEventRecord(e2, s2);
      (void)hipStreamWaitEvent(main, e2, 0);
    }
  } join{main, side, third, evs[6], evs[7]};
  for (uint32_t i = 0; i < count; ++i) {
    const int k = i & 1;
    if (i >= 2) HIP_TRY(ctx, hipStreamWaitEvent(main, x_done[k], 0));  // z[k] was sent
    if (!inverse) MLH_TRY(mlh_ntt(ctx, dev_in[i], z[k], log_n - tp.p, gp));
    else MLH_TRY(mlh_shard_ntt_cross(ctx, dev_in[i], z[k], log_n, tp.p, tp.rank, gen, 1));
    HIP_TRY(ctx, hipEventRecord(a_done[k], main));
    HIP_TRY(ctx, hipStreamWaitEvent(side, a_done[k], 0));
    if (i >= 2) HIP_TRY(ctx, hipStreamWaitEvent(side, c_done[k], 0));  // C(i - 2) read recv[k]
    {
      StreamSwap sw(ctx, side);
      MLH_TRY(tp.all_to_all(z[k], recv[k], M / tp.P * 16, "ntt_all_to_all"));
    }
    HIP_TRY(ctx, hipEventRecord(x_done[k], side));
    HIP_TRY(ctx, hipStreamWaitEvent(third, x_done[k], 0));
    {
      StreamSwap sw(ctx, third);
      if (!inverse) MLH_TRY(mlh_shard_ntt_cross(ctx, recv[k], dev_out[i], log_n, tp.p, tp.rank, gen, 0));
      else MLH_TRY(mlh_intt(ctx, recv[k], dev_out[i], log_n - tp.p, gp));
    }
    HIP_TRY(ctx, hipEventRecord(c_done[k], third));
  }
  return MLH_OK;  // (join: main waits for both side streams)
}

// `count` forward transforms with the rank digit fused into the last pass
// (FusedNtt, capi.hip): per transform the local passes but the last (context
// stream), ONE all-to-all of their output (side stream), and one fused last
// pass over the received chunks (third stream) -- three HBM passes per element
// against four for mlh_sharded_ntt_batch's local NTT + cross-shard DFT.  Input:
// the cyclic layout (rank g holds x[g + P m]); output: block-cyclic with block
// 2^out_log_s (*log_s_out), out_log_s = the plan's first digit - log2 P, e.g. 6
// for 2^27 over 8 ranks.  Pipelined like mlh_sharded_ntt_batch.  Needs
// 2 <= P <= 8 and 2^(log_n - log P) >= 2^(13 - log P) local elements, else
// MLH_ERR_INVALID (use mlh_sharded_ntt_batch).
mlh_status mlh_sharded_ntt_fused_batch(mlh_ctx* ctx, const mlh_transport* t, const void* const* dev_in,
                                       void* const* dev_out, uint32_t count, uint32_t log_n,
                                       const uint8_t gen[16], uint32_t* log_s_out) {
  if (!ctx || (count && (!dev_in || !dev_out)) || !gen) return fail(ctx, MLH_ERR_INVALID, "null argument");
  MLH_TRY(check_transport(ctx, t));
  for (uint32_t i = 0; i < count; ++i)
    if (!dev_in[i] || !dev_out[i]) return fail(ctx, MLH_ERR_INVALID, "null argument");
  Tp tp(ctx, t);
  if (tp.P < 2 || tp.P > 8) return fail(ctx, MLH_ERR_INVALID, "fused sharded NTT: 2 <= P <= 8");
  if (log_n > 40) return fail(ctx, MLH_ERR_INVALID, "log_n");
  if (!gen_has_order(h_load(gen), log_n)) return fail(ctx, MLH_ERR_BAD_GENERATOR, "generator order != n");
  FusedNtt fz;
  MLH_TRY(fz.prepare(ctx, h_load(gen), log_n, tp.p, tp.rank));
  if (log_s_out) *log_s_out = fz.out_log_s();
  if (!count) return MLH_OK;
  const uint64_t M = 1ull << (log_n - tp.p);
  if (t->host_side) {  // transforms in turn
    Bufs b(ctx);
    fe *z, *recv;
    MLH_TRY(b.get(M * 16, &z));
    MLH_TRY(b.get(M * 16, &recv));
    for (uint32_t i = 0; i < count; ++i) {
      MLH_TRY(fz.run_pre(dev_in[i], z));
      MLH_TRY(tp.all_to_all(z, recv, M / tp.P * 16, "ntt_all_to_all"));
      MLH_TRY(fz.run_last(recv, dev_out[i]));
    }
    return MLH_OK;
  }
  MLH_TRY(ensure_side_streams(ctx));
  Bufs b(ctx);
  fe *z[2], *recv[2];
  for (int k = 0; k < 2; ++k) {
    MLH_TRY(b.get(M * 16, &z[k]));
    MLH_TRY(b.get(M * 16, &recv[k]));
  }
  hipEvent_t evs[9];
  for (auto& e : evs) e = take_event(ctx);
  struct Recycle {
    mlh_ctx* c;
    hipEvent_t* e;
    ~Recycle() {
      for (int k = 0; k < 9; ++k) c->ev_free.push_back(e[k]);
    }
  } rec{ctx, evs};
  hipEvent_t *a_done = evs, *x_done = evs + 2, *c_done = evs + 4;
  hipStream_t main = ctx->stream, side = ctx->side, third = ctx->side2;
  HIP_TRY(ctx, hipEventRecord(evs[8], main));  // the third stream starts after the caller's work
  HIP_TRY(ctx, hipStreamWaitEvent(third, evs[8], 0));
  struct JoinSide {  // every exit: the context stream waits for both side streams
    hipStream_t main, s1, s2;
    hipEvent_t e1, e2;
    ~JoinSide() {
      (void)hipEventRecord(e1, s1);
      (void)hipStreamWaitEvent(main, e1, 0);
      (void)hipEventRecord(e2, s2);
      (void)hipStreamWaitEvent(main, e2, 0);
    }
  } join{main, side, third, evs[6], evs[7]};
  for (uint32_t i = 0; i < count; ++i) {
    const int k = i & 1;
    if (i >= 2) HIP_TRY(ctx, hipStreamWaitEvent(main, x_done[k], 0));  // z[k] was sent
    MLH_TRY(fz.run_pre(dev_in[i], z[k]));
    HIP_TRY(ctx, hipEventRecord(a_done[k], main));
    HIP_TRY(ctx, hipStreamWaitEvent(side, a_done[k], 0));
    if (i >= 2) HIP_TRY(ctx, hipStreamWaitEvent(side, c_done[k], 0));  // recv[k] was read
    {
      StreamSwap sw(ctx, side);
      MLH_TRY(tp.all_to_all(z[k], recv[k], M / tp.P * 16, "ntt_all_to_all"));
    }
    HIP_TRY(ctx, hipEventRecord(x_done[k], side));
    HIP_TRY(ctx, hipStreamWaitEvent(third, x_done[k], 0));
    {
      StreamSwap sw(ctx, third);
      MLH_TRY(fz.run_last(recv[k], dev_out[i]));
    }
    HIP_TRY(ctx, hipEventRecord(c_done[k], third));
  }
  return MLH_OK;
}

mlh_status mlh_sharded_reed_solomon(mlh_ctx* ctx, const mlh_transport* t, const void* dev_coeffs,
                                    uint32_t log_n, const uint8_t gen[16], void* dev_code) {
  if (!ctx || !dev_coeffs || !dev_code || !gen) return fail(ctx, MLH_ERR_INVALID, "null argument");
  MLH_TRY(check_transport(ctx, t));
  Tp tp(ctx, t);
  if (tp.P == 1) return mlh_reed_solomon(ctx, dev_coeffs, log_n, gen, dev_code);
  const uint32_t log_c = log_n + MLH_LOG_BLOWUP;
  if (log_c < 2 * tp.p + 1 || log_c > 40)
    return fail(ctx, MLH_ERR_INVALID, "sharded RS needs 2^(log_n+1) >= 2 P^2");
  if (!gen_has_order(h_load(gen), log_c))
    return fail(ctx, MLH_ERR_BAD_GENERATOR, "generator order != 2n");
  const uint64_t M2 = 1ull << (log_c - tp.p);  // local code length
  uint8_t gp[16];
  store_fe(gp, h_pow(h_load(gen), (u128)tp.P));
  Bufs b(ctx);
  fe *z, *recv;
  MLH_TRY(b.get(M2 * 16, &z));
  MLH_TRY(b.get(M2 * 16, &recv));
  MLH_TRY(mlh_reed_solomon(ctx, dev_coeffs, log_n - tp.p, gp, z));
  MLH_TRY(tp.all_to_all(z, recv, M2 / tp.P * 16));
  return mlh_shard_ntt_cross(ctx, recv, dev_code, log_c, tp.p, tp.rank, gen, 0);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// FRI prove (fri/mod.rs:57-175, 261-285) of a block-layout codeword
// ---------------------------------------------------------------------------
namespace {

struct SLayer {
  const fe* values = nullptr;
  uint8_t* tree = nullptr;
  uint32_t log_n = 0, log_p = 0, log_s = 0;
  uint32_t sub_levels = 0;        // tree levels held locally
  uint8_t* top = nullptr;         // device tree over the gathered level-log_s nodes
  const uint8_t* root = nullptr;  // 32-byte device view of the root
  std::vector<uint8_t> top_host;  // host copy of `top` (query phase)
  uint64_t local_leaves() const { return 1ull << (log_n - 1 - log_p); }
};

uint64_t level_offset(uint64_t leaves, uint32_t level) {
  uint64_t off = 0;
  for (uint32_t i = 0; i < level; ++i) off += leaves >> i;
  return off;
}

struct ShardedFri {
  mlh_ctx* ctx;
  Tp& tp;
  Bufs& b;
  std::vector<SLayer> layers;
  ShardedFri(mlh_ctx* c, Tp& t, Bufs& bb) : ctx(c), tp(t), b(bb) {}

  mlh_status make_layer(const fe* values, uint32_t log_n, bool sharded, SLayer* out) {
    SLayer L;
    L.values = values;
    L.log_n = log_n;
    L.log_p = sharded ? tp.p : 0;
    L.log_s = sharded ? log_n - 2 * tp.p : 0;
    L.sub_levels = sharded ? L.log_s : log_n - 1;
    *out = L;
    return MLH_OK;
  }
  mlh_status commit(SLayer& L) {  // local tree, then the top over all ranks
    MLH_TRY(b.get(mlh_merkle_layers_bytes(L.local_leaves()), &L.tree));
    MLH_TRY(mlh_merkle_commit_pairs(ctx, L.values, L.log_n - L.log_p, L.tree, nullptr));
    return commit_top(L);
  }
  mlh_status commit_top(SLayer& L) {
    const uint64_t tree_bytes = mlh_merkle_layers_bytes(L.local_leaves());
    if (L.log_p == 0) {
      L.root = L.tree + tree_bytes - 32;
      return MLH_OK;
    }
    const uint64_t half_t = L.local_leaves() >> L.sub_levels;
    const uint8_t* nodes = L.tree + 32 * level_offset(L.local_leaves(), L.sub_levels);
    uint8_t* gathered;
    MLH_TRY(b.get(32 * half_t * tp.P, &gathered));
    MLH_TRY(tp.all_gather(nodes, gathered, 32 * half_t));
    MLH_TRY(b.get(mlh_merkle_layers_bytes(half_t * tp.P), &L.top));
    MLH_TRY(mlh_merkle_top(ctx, gathered, tp.P, half_t, L.top));
    L.root = L.top + mlh_merkle_layers_bytes(half_t * tp.P) - 32;
    return MLH_OK;
  }
  // block layout -> natural order on every rank (all-gather + one 2D copy per rank)
  mlh_status to_natural(const fe* values, uint32_t log_n, fe** out) {
    const uint64_t local = 1ull << (log_n - tp.p), S = 1ull << (log_n - 2 * tp.p), T = local / S;
    fe *g, *nat;
    MLH_TRY(b.get(local * tp.P * 16, &g));
    MLH_TRY(b.get(local * tp.P * 16, &nat));
    MLH_TRY(tp.all_gather(values, g, local * 16));
    for (uint32_t r = 0; r < tp.P; ++r)
      HIP_TRY(ctx, hipMemcpy2DAsync(nat + r * S, tp.P * S * 16, g + r * local, S * 16, S * 16, T,
                                    hipMemcpyDeviceToDevice, ctx->stream));
    *out = nat;
    return MLH_OK;
  }
};

}  // namespace

extern "C" {

mlh_status mlh_sharded_fri_prove(mlh_ctx* ctx, const mlh_transport* t, const void* dev_code,
                                 uint32_t log_code, uint32_t gather_log, mlh_transcript* tr,
                                 mlh_fri_proof* proof) {
  if (!ctx || !dev_code || !tr || !proof || !proof->commitments || !proof->queries)
    return fail(ctx, MLH_ERR_INVALID, "null argument");
  MLH_TRY(check_transport(ctx, t));
  Tp tp(ctx, t);
  if (log_code < 2 || log_code > 40) return fail(ctx, MLH_ERR_INVALID, "log_code out of range");
  if (tp.p && log_code < 2 * tp.p) return fail(ctx, MLH_ERR_INVALID, "codeword too small for the world");
  if (tp.P == 1) return mlh_fri_prove(ctx, dev_code, log_code, tr, proof);
  if (gather_log < 2 * tp.p + 2) gather_log = 2 * tp.p + 2;
  const uint32_t n0 = log_code, steps = log_code - MLH_LOG_BLOWUP;
  Bufs b(ctx);
  ShardedFri F(ctx, tp, b);
  uint8_t* state;
  fe *rbuf, *lastbuf;
  uint32_t* flagbuf;
  MLH_TRY(b.get(mlh_device_transcript_bytes(), &state));
  MLH_TRY(b.get(16 * (steps + 1), &rbuf));
  MLH_TRY(b.get(16, &lastbuf));
  MLH_TRY(b.get(16, &flagbuf));
  HIP_TRY(ctx, hipMemsetAsync(flagbuf, 0, 16, ctx->stream));
  MLH_TRY(mlh_transcript_to_device(ctx, tr, state));
  SLayer L0;
  if (log_code > gather_log) {
    MLH_TRY(F.make_layer(static_cast<const fe*>(dev_code), log_code, true, &L0));
  } else {
    fe* nat;
    MLH_TRY(F.to_natural(static_cast<const fe*>(dev_code), log_code, &nat));
    MLH_TRY(F.make_layer(nat, log_code, false, &L0));
  }
  MLH_TRY(F.commit(L0));
  F.layers.push_back(L0);
  MLH_TRY(mlh_device_transcript_absorb(ctx, state, F.layers.back().root, 32, rbuf));
  bool done = false;
  for (uint32_t k = 0; k < steps; ++k) {
    const SLayer cur = F.layers.back();
    if ((1ull << cur.log_n) <= (1ull << MLH_LOG_BLOWUP)) break;
    const fe* r = rbuf + k;
    const uint32_t log_next = cur.log_n - 1;
    const uint64_t next_local = 1ull << (log_next - cur.log_p);
    fe* nv;
    MLH_TRY(b.get(next_local * 16, &nv));
    if ((1ull << log_next) == (1ull << MLH_LOG_BLOWUP)) {  // fri/mod.rs:116-126
      MLH_TRY(mlh_shard_fri_fold_dr(ctx, cur.values, cur.log_n, k, n0, r, nv, 40, 0, 0));
      MLH_TRY(mlh_device_fri_last(ctx, nv, state, flagbuf, lastbuf));
      done = true;
      break;
    }
    SLayer nx;
    if (cur.log_p == 0) {
      MLH_TRY(F.make_layer(nv, log_next, false, &nx));
      MLH_TRY(b.get(mlh_merkle_layers_bytes(nx.local_leaves()), &nx.tree));
      MLH_TRY(mlh_shard_fri_fold_commit_dr(ctx, cur.values, cur.log_n, k, n0, r, nv, nx.tree, 40, 0, 0));
    } else if (log_next >= cur.log_p + cur.log_s + 1) {  // >= 2 local blocks: pairs stay local
      nx.values = nv;
      nx.log_n = log_next;
      nx.log_p = cur.log_p;
      nx.log_s = cur.log_s;
      nx.sub_levels = cur.log_s;
      MLH_TRY(b.get(mlh_merkle_layers_bytes(nx.local_leaves()), &nx.tree));
      MLH_TRY(mlh_shard_fri_fold_commit_dr(ctx, cur.values, cur.log_n - cur.log_p, k, n0, r, nv,
                                           nx.tree, cur.log_s, cur.log_p, tp.rank));
    } else {  // the folded layer is in natural block order: re-deal or gather
      MLH_TRY(mlh_shard_fri_fold_dr(ctx, cur.values, cur.log_n - cur.log_p, k, n0, r, nv, cur.log_s,
                                    cur.log_p, tp.rank));
      fe* dealt;
      if (log_next > gather_log) {
        MLH_TRY(b.get(next_local * 16, &dealt));
        MLH_TRY(tp.all_to_all(nv, dealt, next_local / tp.P * 16));
        MLH_TRY(F.make_layer(dealt, log_next, true, &nx));
      } else {
        MLH_TRY(b.get(next_local * tp.P * 16, &dealt));
        MLH_TRY(tp.all_gather(nv, dealt, next_local * 16));
        MLH_TRY(F.make_layer(dealt, log_next, false, &nx));
      }
      MLH_TRY(b.get(mlh_merkle_layers_bytes(nx.local_leaves()), &nx.tree));
      MLH_TRY(mlh_merkle_commit_pairs(ctx, nx.values, nx.log_n - nx.log_p, nx.tree, nullptr));
    }
    MLH_TRY(F.commit_top(nx));
    F.layers.push_back(nx);
    MLH_TRY(mlh_device_transcript_absorb(ctx, state, F.layers.back().root, 32, rbuf + k + 1));
  }
  if (!done) return fail(ctx, MLH_ERR_INVALID, "fold produced no last element");

  // one wait: roots, last element, RS flag; the host transcript replays them
  const size_t nt = F.layers.size();
  std::vector<uint8_t> roots(32 * nt);
  for (size_t i = 0; i < nt; ++i)
    HIP_TRY(ctx, hipMemcpyAsync(roots.data() + 32 * i, F.layers[i].root, 32, hipMemcpyDeviceToHost,
                                ctx->stream));
  uint8_t last[16];
  uint32_t flag = 0;
  std::vector<uint8_t> rhost(16 * nt);
  HIP_TRY(ctx, hipMemcpyAsync(rhost.data(), rbuf, 16 * nt, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(last, lastbuf, 16, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(&flag, flagbuf, 4, hipMemcpyDeviceToHost, ctx->stream));
  for (auto& L : F.layers)
    if (L.top) {
      const uint64_t nb = mlh_merkle_layers_bytes(L.local_leaves() >> L.sub_levels << tp.p);
      L.top_host.resize(nb);
      HIP_TRY(ctx, hipMemcpyAsync(L.top_host.data(), L.top, nb, hipMemcpyDeviceToHost, ctx->stream));
    }
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (flag) return fail(ctx, MLH_ERR_NOT_RS_CODE, "not an RS code");
  {  // host replay: root_i, then the challenge r_i the device drew from it
    ReplayCheck rc(ctx, tr);
    for (size_t i = 0; i < nt; ++i) {
      rc.absorb(roots.data() + 32 * i, 32);
      rc.expect(rhost.data() + 16 * i);
    }
    rc.absorb(last, 16);
    MLH_TRY(rc.status());
  }

  // queries (fri/mod.rs:266-277): the owner opens, records combined by a gather
  const uint64_t half = 1ull << (log_code - 1);
  std::vector<uint64_t> idx(MLH_NUM_QUERIES);
  for (uint32_t q = 0; q < MLH_NUM_QUERIES; ++q) {
    idx[q] = transcript_query_index(tr, half);
    uint8_t le[8];
    memcpy(le, &idx[q], 8);
    mlh_transcript_absorb(tr, le, 8);
  }
  const uint64_t qbytes = mlh_fri_query_bytes(log_code);
  std::vector<uint8_t> mine(qbytes * MLH_NUM_QUERIES, 0);
  uint64_t layer_off = 0;
  for (const SLayer& L : F.layers) {
    const uint64_t leaves = 1ull << (L.log_n - 1);
    const uint64_t rec_len = 32ull * L.log_n;  // pair + (log_n - 1) siblings
    std::vector<uint32_t> who;
    std::vector<uint64_t> loc;
    for (uint32_t q = 0; q < MLH_NUM_QUERIES; ++q) {
      const uint64_t i = idx[q] % leaves;
      if (L.log_p) {
        const uint64_t r = (i >> L.log_s) & ((1ull << L.log_p) - 1);
        if (r != tp.rank) continue;
        loc.push_back(((i >> (L.log_s + L.log_p)) << L.log_s) | (i & ((1ull << L.log_s) - 1)));
      } else {
        loc.push_back(i);
      }
      who.push_back(q);
    }
    const uint64_t sub_rec = 32ull * (1 + L.sub_levels);
    std::vector<uint8_t> recs(sub_rec * (loc.size() ? loc.size() : 1));
    if (!loc.empty())
      MLH_TRY(mlh_merkle_open_pairs(ctx, L.values, L.log_n - L.log_p, L.tree, L.sub_levels, loc.data(),
                                    (uint32_t)loc.size(), recs.data()));
    // host top levels of a sharded layer: leaves = P * half_t nodes
    const uint64_t top_leaves = L.top ? (L.local_leaves() >> L.sub_levels) << tp.p : 0;
    for (size_t w = 0; w < who.size(); ++w) {
      const uint32_t q = who[w];
      const uint64_t i = idx[q] % leaves;
      uint8_t* dst = mine.data() + q * qbytes + layer_off;
      memcpy(dst, recs.data() + w * sub_rec, sub_rec);
      uint64_t off = 0, cnt = top_leaves;
      for (uint32_t lv = 0; L.top && cnt > 1; ++lv, off += cnt, cnt >>= 1) {
        const uint64_t node = (i >> (L.sub_levels + lv)) ^ 1;
        memcpy(dst + sub_rec + 32 * lv, L.top_host.data() + 32 * (off + node), 32);
      }
    }
    layer_off += rec_len;
  }
  // every record is written by exactly one rank: OR of the gathered copies
  uint8_t *dmine, *dall;
  MLH_TRY(b.get(mine.size(), &dmine));
  MLH_TRY(b.get(mine.size() * tp.P, &dall));
  HIP_TRY(ctx, hipMemcpyAsync(dmine, mine.data(), mine.size(), hipMemcpyHostToDevice, ctx->stream));
  MLH_TRY(tp.all_gather(dmine, dall, mine.size()));
  std::vector<uint8_t> all(mine.size() * tp.P);
  HIP_TRY(ctx, hipMemcpyAsync(all.data(), dall, all.size(), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  for (uint32_t r = 1; r < tp.P; ++r)
    for (size_t i = 0; i < mine.size(); ++i) all[i] |= all[r * mine.size() + i];
  proof->log_code = log_code;
  proof->num_trees = (uint32_t)nt;
  proof->num_queries = MLH_NUM_QUERIES;
  memcpy(proof->commitments, roots.data(), 32 * nt);
  memcpy(proof->queries, all.data(), mine.size());
  if (proof->query_indices) memcpy(proof->query_indices, idx.data(), 8 * MLH_NUM_QUERIES);
  memcpy(proof->last_elem, last, 16);
  mlh_transcript_random(tr, proof->last_random);
  return MLH_OK;
}

// commit_rs_code of a block-layout codeword: local leaves and subtrees, one
// all-gather of the subtree roots, the top levels on every rank.
mlh_status mlh_sharded_commit_rs_code(mlh_ctx* ctx, const mlh_transport* t, const void* dev_code,
                                      uint32_t log_code, uint8_t root_out[32]) {
  if (!ctx || !dev_code || !root_out) return fail(ctx, MLH_ERR_INVALID, "null argument");
  MLH_TRY(check_transport(ctx, t));
  Tp tp(ctx, t);
  if (log_code < 1 || log_code > 40) return fail(ctx, MLH_ERR_INVALID, "log_code out of range");
  if (tp.P == 1) {
    const uint64_t bytes = mlh_merkle_layers_bytes(1ull << (log_code - 1));
    PoolBuf tree(ctx);
    MLH_TRY(tree.alloc(bytes));
    return mlh_merkle_commit_pairs(ctx, dev_code, log_code, tree.p, root_out);
  }
  if (log_code < 2 * tp.p + 1) return fail(ctx, MLH_ERR_INVALID, "codeword too small for the world");
  Bufs b(ctx);
  ShardedFri F(ctx, tp, b);
  SLayer L;
  MLH_TRY(F.make_layer(static_cast<const fe*>(dev_code), log_code, true, &L));
  MLH_TRY(F.commit(L));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->pinned + kPinSlotB, L.root, 32, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  memcpy(root_out, ctx->pinned + kPinSlotB, 32);
  return MLH_OK;
}

// ---------------------------------------------------------------------------
// Sumcheck (sumcheck.rs:77-247) of cyclic-layout tables
// ---------------------------------------------------------------------------
// delta of build_tables_for_pcs (sumcheck.rs:128-145) in the cyclic layout:
// rank r holds delta[l P + r] = eq(points[:n-p], l) * c_r, where
// c_r = prod_{b<p} (bit_b(r) ? points[n-1-b] : 1 - points[n-1-b]).
mlh_status mlh_sharded_eq_table(mlh_ctx* ctx, const mlh_transport* t, const uint8_t* points,
                                uint32_t n, void* dev_out) {
  if (!ctx || !dev_out || (n && !points)) return fail(ctx, MLH_ERR_INVALID, "null argument");
  MLH_TRY(check_transport(ctx, t));
  Tp tp(ctx, t);
  if (n < tp.p) return fail(ctx, MLH_ERR_INVALID, "fewer variables than log2(world)");
  u128 c = 1;
  for (uint32_t bit = 0; bit < tp.p; ++bit) {
    const u128 pt = h_load(points + 16 * (n - 1 - bit));
    c = h_mul(c, ((tp.rank >> bit) & 1) ? pt : h_sub(1, pt));
  }
  MLH_TRY(mlh_eq_table(ctx, points, n - tp.p, dev_out));
  if (c == 1) return MLH_OK;
  uint8_t cb[16];
  store_fe(cb, c);
  return mlh_field_scale(ctx, dev_out, cb, dev_out, 1ull << (n - tp.p));
}

mlh_status mlh_sharded_sumcheck_prove(mlh_ctx* ctx, const mlh_transport* t, void* dev_m, void* dev_d,
                                      uint32_t n, const uint8_t sum[16], mlh_transcript* tr,
                                      uint8_t* polys_out, uint8_t* rs_out) {
  if (!ctx || !dev_m || !dev_d || !sum || !tr || n < 1 || n > 40)
    return fail(ctx, MLH_ERR_INVALID, "bad argument");
  MLH_TRY(check_transport(ctx, t));
  Tp tp(ctx, t);
  if (n < tp.p) return fail(ctx, MLH_ERR_INVALID, "fewer variables than log2(world)");
  if (tp.P == 1) return mlh_sumcheck_prove(ctx, dev_m, dev_d, n, sum, tr, polys_out, rs_out);
  Bufs b(ctx);
  uint8_t* state;
  fe *prev, *polys, *rs, *sums, *pairs;
  MLH_TRY(b.get(mlh_device_transcript_bytes(), &state));
  MLH_TRY(b.get(16, &prev));
  MLH_TRY(b.get(32ull * n, &polys));
  MLH_TRY(b.get(16ull * n, &rs));
  MLH_TRY(b.get(32, &sums));
  MLH_TRY(b.get(32ull * tp.P, &pairs));
  MLH_TRY(mlh_transcript_to_device(ctx, tr, state));
  memcpy(ctx->pinned + kPinSlotA, sum, 16);
  HIP_TRY(ctx, hipMemcpyAsync(prev, ctx->pinned + kPinSlotA, 16, hipMemcpyHostToDevice, ctx->stream));
  fe* m = static_cast<fe*>(dev_m);
  fe* d = static_cast<fe*>(dev_d);
  bool sharded = true;
  uint32_t log_local = n - tp.p;
  auto go_replicated = [&](uint64_t cnt) -> mlh_status {  // gather cnt entries per rank
    fe *gm, *gd;
    MLH_TRY(b.get(16 * cnt * tp.P, &gm));
    MLH_TRY(b.get(16 * cnt * tp.P, &gd));
    MLH_TRY(tp.all_gather(m, gm, 16 * cnt));
    MLH_TRY(tp.all_gather(d, gd, 16 * cnt));
    m = gm;
    d = gd;
    sharded = false;
    return MLH_OK;
  };
  if (log_local == 0) {
    MLH_TRY(go_replicated(1));
    log_local = n;
  }
  MLH_TRY(mlh_sumcheck_sums_dev(ctx, m, d, log_local, sums));
  for (uint32_t k = 0; k < n; ++k) {
    const fe* pr = sums;
    if (sharded) {
      MLH_TRY(tp.all_gather(sums, pairs, 32));
      pr = pairs;
    }
    MLH_TRY(mlh_device_sumcheck_round(ctx, pr, sharded ? tp.P : 1, prev, state, polys + 2 * k, rs + k));
    if (k + 1 == n) {
      MLH_TRY(mlh_sumcheck_fold_dr(ctx, m, d, log_local, rs + k));
      break;
    }
    if (log_local >= 2) {
      MLH_TRY(mlh_sumcheck_fold_sums_dr(ctx, m, d, log_local, rs + k, sums));
      --log_local;
    } else {  // sharded, local 2 -> 1 entries: gather the P-entry tables, go replicated
      MLH_TRY(mlh_sumcheck_fold_dr(ctx, m, d, log_local, rs + k));
      MLH_TRY(go_replicated(1));
      log_local = tp.p;
      MLH_TRY(mlh_sumcheck_sums_dev(ctx, m, d, log_local, sums));
    }
  }
  // the last rounds folded pool copies: hand the fully folded m(r), d(r) back
  // to entry 0 of the caller's tables (the reference's tables end at length 1)
  if (m != dev_m) {
    HIP_TRY(ctx, hipMemcpyAsync(dev_m, m, 16, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dev_d, d, 16, hipMemcpyDeviceToDevice, ctx->stream));
  }
  std::vector<uint8_t> host(48ull * n);
  HIP_TRY(ctx, hipMemcpyAsync(host.data(), polys, 32ull * n, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(host.data() + 32ull * n, rs, 16ull * n, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  ReplayCheck rc(ctx, tr);
  for (uint32_t k = 0; k < n; ++k) {
    rc.absorb(host.data() + 32 * k, 32);
    rc.expect(host.data() + 32ull * n + 16 * k);
  }
  MLH_TRY(rc.status());
  if (polys_out) memcpy(polys_out, host.data(), 32ull * n);
  if (rs_out) memcpy(rs_out, host.data() + 32ull * n, 16ull * n);
  return MLH_OK;
}

}  // extern "C"
