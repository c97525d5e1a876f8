// Internal state of an mlh_ctx and the helpers every host-side translation
// unit of libmlhip shares (capi.hip: the single-GPU C ABI; sharded.hip: the
// multi-GPU orchestration): the device memory pool, the table cache record,
// error reporting.  Not part of the public C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <tuple>
#include <vector>

#include "../../include/mlhip.h"
#include "host_transcript.hpp"
#include "field.hpp"
#include "host_field.hpp"
#include "ntt.hpp"

using mlh::fe;
using mlh::kMaxPasses;
using mlh::u128;

// ctx->pinned: [0, kPinStage) staging of a prove's one D2H copy; two 512-B
// slots after it for small copies that may be in flight beside it.
constexpr size_t kPinnedBytes = 16384, kPinStage = 12288, kPinSlotA = 12288, kPinSlotB = 12800;

struct TableKey {
  u128 base;
  uint64_t count;
  u128 scale;
  int expand;
  uint64_t cols = 0;  // 2D tables: count = rows, entry (k, j) = base^(k j mult)
  uint64_t mult = 0;
  bool operator<(const TableKey& o) const {
    return std::tie(base, count, scale, expand, cols, mult) <
           std::tie(o.base, o.count, o.scale, o.expand, o.cols, o.mult);
  }
};

// A cached twiddle table: device buffer, size, LRU stamp.
struct CachedTable {
  fe* d = nullptr;
  size_t bytes = 0;
  uint64_t stamp = 0;
};

struct mlh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  // twiddle / fold tables, bounded LRU (mlh_set_table_cache_limit)
  std::map<TableKey, CachedTable> tables;
  size_t table_bytes = 0;
  size_t table_limit = (size_t)1 << 30;
  uint64_t table_stamp = 0;
  std::multimap<size_t, void*> pool;  // cached free device blocks
  std::map<void*, size_t> live;       // pool-owned live blocks
  fe* partials = nullptr;             // 2 * kMaxRedBlocks
  fe* small = nullptr;                // 64 elements scratch (sums, points)
  uint8_t* pinned = nullptr;          // kPinnedBytes pinned host staging
  // Device-side failure word, in pinned host memory the kernels write
  // directly (only on failure: a cooperative kernel's LDS wait that timed
  // out).  Cleared before, read after each prove's final sync (device_check).
  volatile uint32_t* dev_status = nullptr;
  uint32_t coop_spin = 0;  // cooperative kernels' wait limit in sleeps (0: default)
  uint32_t pcs_fused_max = 24;  // PCS provers: rounds off the transcript chain up to this many vars
  uint8_t* qstage = nullptr;          // pinned staging of query phases (grow-only)
  size_t qstage_bytes = 0;
  fe* ntt_scratch = nullptr;          // NTT ping-pong buffer (grow-only)
  size_t ntt_scratch_bytes = 0;
  hipStream_t side = nullptr;         // second stream of pipelined calls (lazy)
  hipStream_t side2 = nullptr;        // third stream (sharded NTT batch: the cross-shard step)
  // debug / test hooks, fixed at creation (MLH_DEBUG_SYNC) or set through the
  // API (mlh_set_ntt_plan): never read from the environment on a hot path
  bool debug_sync = false;
  uint32_t forced_plan[kMaxPasses] = {0};
  uint32_t forced_plan_len = 0;
  // kernel timer (mlh_profile_*): HIP events on the launch stream
  bool prof_on = false;
  uint32_t prof_every = 1;  // bracket every prof_every-th transform / launch of each label
  std::unordered_map<std::string, uint64_t> prof_ticks;
  std::vector<hipEvent_t> ev_free;
  struct Pending {
    std::string label;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::map<std::string, std::pair<uint64_t, double>> prof;  // label -> (count, total ms)
};

inline hipEvent_t take_event(mlh_ctx* ctx) {
  if (!ctx->ev_free.empty()) {
    hipEvent_t e = ctx->ev_free.back();
    ctx->ev_free.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

inline void resolve_profile(mlh_ctx* ctx) {
  for (auto& p : ctx->pending) {
    (void)hipEventSynchronize(p.b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, p.a, p.b);
    auto& slot = ctx->prof[p.label];
    slot.first += 1;
    slot.second += ms;
  }
  // events are shared between consecutive pairs: collect unique ones
  std::vector<hipEvent_t> evs;
  for (auto& p : ctx->pending) {
    evs.push_back(p.a);
    evs.push_back(p.b);
  }
  std::sort(evs.begin(), evs.end());
  evs.erase(std::unique(evs.begin(), evs.end()), evs.end());
  for (auto e : evs) ctx->ev_free.push_back(e);
  ctx->pending.clear();
}

// Whether the kernel timer brackets this transform / launch: every
// prof_every-th one of its label while enabled (the events cost the stream a
// few us each; counting per label keeps interleaved kinds all sampled).
inline bool prof_sample(mlh_ctx* ctx, const char* label) {
  if (!ctx->prof_on) return false;
  if (ctx->prof_every <= 1) return true;
  return ctx->prof_ticks[label]++ % ctx->prof_every == 0;
}

// Kernel-timer bracket around one launch (no-op unless mlh_profile_enable).
struct ProfScope {
  mlh_ctx* ctx;
  const char* label;
  hipEvent_t a = nullptr;
  ProfScope(mlh_ctx* c, const char* lab) : ctx(c), label(lab) {
    if (prof_sample(ctx, label)) {
      a = take_event(ctx);
      (void)hipEventRecord(a, ctx->stream);
    }
  }
  void end() {
    if (!a) return;
    hipEvent_t b = take_event(ctx);
    (void)hipEventRecord(b, ctx->stream);
    ctx->pending.push_back(mlh_ctx::Pending{label, a, b});
    a = nullptr;
  }
  // an early error return skipped end(): recycle the start event
  ~ProfScope() {
    if (a) ctx->ev_free.push_back(a);
  }
};


inline mlh_status fail(mlh_ctx* ctx, mlh_status st, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return st;
}

// The one wait of a prove: poll the stream instead of blocking in
// hipStreamSynchronize (whose wake-up after the last kernel is several
// microseconds of a ~0.24 ms prove).  MLH_SYNC_SPIN selects it at build time.
#ifndef MLH_SYNC_SPIN
#define MLH_SYNC_SPIN 0
#endif
inline hipError_t prove_wait(mlh_ctx* ctx) {
  if (!MLH_SYNC_SPIN) return hipStreamSynchronize(ctx->stream);
  hipError_t e;
  while ((e = hipStreamQuery(ctx->stream)) == hipErrorNotReady) {
  }
  return e;
}

// Device-side failures (MLH_ERR_DEVICE).  device_arm before a prove enqueues
// its cooperative kernels, device_check after its final sync.
// The clear is enqueued on ctx->stream (not a host store), so a kernel of an
// earlier call still running on the stream cannot set the word after it is
// cleared, nor have a real report wiped.
inline void device_arm(mlh_ctx* ctx) {
  (void)hipMemsetAsync(const_cast<uint32_t*>(ctx->dev_status), 0, sizeof(uint32_t), ctx->stream);
}
inline mlh_status device_check(mlh_ctx* ctx) {
  const uint32_t s = *ctx->dev_status;
  if (!s) return MLH_OK;
  *ctx->dev_status = 0;
  return fail(ctx, MLH_ERR_DEVICE,
              "a cooperative sumcheck kernel gave up waiting (spin limit): its outputs are invalid");
}

// Host replay of a prove's transcript (transcript.rs:23-38): absorbs the bytes
// the device absorbed and, at each point where the device drew a challenge,
// compares next_challenge() with the device's value.  Any difference -- a
// device SHA-256 or synchronisation fault -- fails the prove (MLH_ERR_DEVICE)
// instead of returning a proof whose challenges do not follow from it.  The
// caller's transcript is restored to its state at construction unless
// status() succeeded, so a rejected prove leaves it as a device_check failure
// does: untouched (mlhip.h).
struct ReplayCheck {
  mlh_ctx* ctx;
  mlh_transcript* tr;
  mlh::HostSha256 saved;
  bool committed = false;
  uint32_t bad = 0, first_bad = ~0u, n = 0;
  ReplayCheck(mlh_ctx* c, mlh_transcript* t) : ctx(c), tr(t), saved(t->sha) {}
  ReplayCheck(const ReplayCheck&) = delete;
  ReplayCheck& operator=(const ReplayCheck&) = delete;
  ~ReplayCheck() {
    if (!committed) tr->sha = saved;
  }
  void absorb(const uint8_t* p, uint64_t len) { mlh_transcript_absorb(tr, p, len); }
  void expect(const uint8_t* dev_r) {
    uint8_t h[16];
    mlh_transcript_next_challenge(tr, h);
    if (memcmp(h, dev_r, 16) != 0) {
      if (!bad) first_bad = n;
      ++bad;
    }
    ++n;
  }
  mlh_status status() {
    if (!bad) {
      committed = true;
      return MLH_OK;
    }
    return fail(ctx, MLH_ERR_DEVICE,
                "device transcript diverged from the host replay at challenge " +
                    std::to_string(first_bad) + " (" + std::to_string(bad) + " of " +
                    std::to_string(n) + " differ)");
  }
};

// Runs the enclosed entry-point calls on another stream: every launch and
// copy of the library goes to ctx->stream, which is swapped for the scope.
struct StreamSwap {
  mlh_ctx* ctx;
  hipStream_t saved;
  StreamSwap(mlh_ctx* c, hipStream_t s) : ctx(c), saved(c->stream) { c->stream = s; }
  ~StreamSwap() { ctx->stream = saved; }
};

#define HIP_TRY(ctx, expr)                                                                \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail((ctx), MLH_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_));  \
  } while (0)

#define MLH_TRY(expr)              \
  do {                             \
    mlh_status s_ = (expr);        \
    if (s_ != MLH_OK) return s_;   \
  } while (0)

inline mlh::fe to_fe(u128 v) {
  fe r;
  memcpy(r.w, &v, 16);
  return r;
}
inline mlh::u128 from_fe(const mlh::fe& x) {
  u128 v;
  memcpy(&v, x.w, 16);
  return v;
}

// pooled device allocation: large per-call buffers are reused across calls
inline mlh_status pool_alloc(mlh_ctx* ctx, size_t bytes, void** out) {
  bytes = (bytes + 255) & ~(size_t)255;
  auto it = ctx->pool.lower_bound(bytes);
  if (it != ctx->pool.end() && it->first <= bytes + bytes / 4) {
    *out = it->second;
    ctx->live[it->second] = it->first;
    ctx->pool.erase(it);
    return MLH_OK;
  }
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, bytes);
  if (e != hipSuccess) {
    // release cached blocks and retry once
    for (auto& kv : ctx->pool) (void)hipFree(kv.second);
    ctx->pool.clear();
    e = hipMalloc(&p, bytes);
    if (e != hipSuccess) return fail(ctx, MLH_ERR_OOM, "hipMalloc failed");
  }
  ctx->live[p] = bytes;
  *out = p;
  return MLH_OK;
}
inline void pool_free(mlh_ctx* ctx, void* p) {
  if (!p) return;
  auto it = ctx->live.find(p);
  if (it == ctx->live.end()) return;
  ctx->pool.emplace(it->second, p);
  ctx->live.erase(it);
}

// RAII helper for pooled buffers
struct PoolBuf {
  mlh_ctx* ctx;
  void* p = nullptr;
  explicit PoolBuf(mlh_ctx* c) : ctx(c) {}
  ~PoolBuf() { pool_free(ctx, p); }
  mlh_status alloc(size_t bytes) { return pool_alloc(ctx, bytes, &p); }
  void* release() {  // ownership passes to the caller
    void* q = p;
    p = nullptr;
    return q;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

