// Device parts of a tree's latency-bound finish, shared by top_kernel
// (merkle.hip) and the fused small FRI step (fri.hip).  Internal.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "merkle.hpp"
#include "sha256.hpp"
#include "transcript_dev.hpp"

namespace mlh {

// Per-level s_memtime stamps of a tree tail's workgroup 0 (tools/
// tree_tail_bench.hip builds merkle.hip with MLH_TREE_TS; off otherwise).
#ifdef MLH_TREE_TS
extern __device__ uint64_t g_tree_ts[4][64];
#define MLH_TREE_STAMP(k, i)                                                  \
  do {                                                                         \
    if (blockIdx.x == 0 && threadIdx.x == 0 && (i) < 64) {                  \
      g_tree_ts[k][i] = __builtin_amdgcn_s_memtime();                          \
      g_tree_ts[(k) + 2][i] = __builtin_amdgcn_s_memrealtime();                \
    }                                                                          \
  } while (0)
#else
#define MLH_TREE_STAMP(k, i) \
  do {                       \
  } while (0)
#endif

#ifndef MLH_PAIR_LEVELS_MAX
// a level is hashed on lane pairs only while its 2 np lanes are at most one
// wave per SIMD of the CU (4 x 64): beyond that the pairs' 22 lane-instructions
// per round-node lose to the single lane's 14 (the level is issue-bound)
#define MLH_PAIR_LEVELS_MAX 256
#endif
__device__ __forceinline__ bool pair_level(uint64_t np) {
  return 2 * np <= blockDim.x && 2 * np <= MLH_PAIR_LEVELS_MAX;
}
// The levels above the n digests in s (shared memory, n a power of two) up to
// the root s[0], each level written to out consecutively (level order); a
// level of few nodes (pair_level) hashes each node on a lane pair
// (sha2l_node).  Every thread of the workgroup calls it.
__device__ __forceinline__ void lds_tree_levels(Sha256State* s, uint64_t n, uint8_t* __restrict__ out,
                                                int ts_k = 1) {
  uint64_t off = 0;
  [[maybe_unused]] int lvl = 0;
  while (n > 1) {
    const uint64_t np = n / 2;
    Sha256State r;
    const bool two = pair_level(np);
    const uint32_t node = two ? sha2l_pair(threadIdx.x) : threadIdx.x;
    const bool active = node < np;
    if (active) r = two ? sha2l_node(s[2 * node], s[2 * node + 1]) : sha256_node(s[2 * node], s[2 * node + 1]);
    __syncthreads();
    if (active && (!two || sha2l_lead(threadIdx.x))) {
      s[node] = r;
      digest_store(out + (off + node) * 32, r);
    }
    __syncthreads();
    MLH_TREE_STAMP(ts_k, 2 + lvl);
    ++lvl;
    off += np;
    n = np;
  }
}

// RootAbsorb's transcript step after the root is known (every thread calls;
// wave 0 runs it on a lane pair): absorb the 32 root bytes, then pw (8 words,
// optional: RootAbsorb::poly_in staged in shared memory), write the state to
// ra.t, the root bytes to ra.copy_out and next_challenge() to ra.r_out.
// ts: the transcript state in shared memory.
__device__ __forceinline__ void root_transcript(const Sha256State& root, DevSha& ts, uint32_t* stage,
                                                const uint32_t* pw, const RootAbsorb& ra) {
  if (!ra.t || threadIdx.x >= 64) return;
  uint32_t w[8];  // the digest's memory bytes (big-endian words)
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = bswap32(root.h[i]);
  if (pw) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      v[i] = w[i];
      v[8 + i] = pw[i];
    }
    dsha2l_step<16>(ts, v, stage, ra.r_out);
  } else {
    dsha2l_step<8>(ts, w, stage, ra.r_out);
  }
  if (threadIdx.x == 0) {
    *ra.t = ts;
    if (ra.copy_out) {
      uint4* q = reinterpret_cast<uint4*>(ra.copy_out);
      q[0] = make_uint4(w[0], w[1], w[2], w[3]);
      q[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
  }
}

}  // namespace mlh
