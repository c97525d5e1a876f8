// Sharded NTT with the rank digit fused into the last pass: the rank-local
// parts (capi.hip; orchestration in sharded.hip mlh_sharded_ntt_fused_batch).
#pragma once
#include <vector>

#include "context.hpp"
#include "ntt.hpp"

struct FusedNtt {
  mlh_ctx* ctx = nullptr;
  uint32_t L = 0, p = 0, rank = 0;
  mlh::NttTables loc;                 // local plan, TA rows twisted by the rank
  uint32_t nglob = 0;
  uint32_t logr[mlh::kMaxPasses] = {0};  // global plan (the last digit includes the rank bits)
  const mlh::fe* tw_last = nullptr;
  std::vector<void*> scaled;
  ~FusedNtt();
  // gen: order exactly 2^log_n (global); this rank of 2^log_p
  mlh_status prepare(mlh_ctx* ctx, mlh::u128 gen, uint32_t log_n, uint32_t log_p, uint32_t rank);
  // local passes: the rank's 2^(log_n - log_p) cyclic shard -> out (sent by the all-to-all)
  mlh_status run_pre(const void* in, void* out);
  // the fused last pass: the receive buffer -> the block-cyclic output
  // (block 2^(logr[0] - log_p))
  mlh_status run_last(const void* recv, void* out);
  uint32_t out_log_s() const { return logr[0] - p; }
};
