// FRI layer folding on gfx950.
//
// Reference: src/fri/mod.rs:79-134 (FriProverData::fold_step).  A layer of n
// values is read as pairs (a, b) = (layer[i], layer[i + n/2]) and folded to
//   next[i] = ((a + b) + r * (a - b) * gen_pows[len - i*2^k]) * 1/2,
// gen_pows[len - i*2^k] = g^(-i*2^k) with g the generator of the original
// domain (order n0).  The device keeps the layer as a flat value array (the
// pair layout of ReedSolomonPair is a view: pair i = (layer[i], layer[i+n/2])).
//
// * the twiddle comes from a two-level table of g^-1 (T_lo[e & 4095] *
//   T_hi[e >> 12]), no 2^25-entry gen_pows array in HBM;
// * a sharded layer (ShardMap, block-cyclic over ranks) folds with the same
//   kernels: the pair partner is local, only the twiddle exponent needs the
//   global index;
// * `* 1/2` is a shift (x even: x >> 1, odd: (x + M) >> 1), not a modmul;
// * fold_leaves fuses the fold with the next layer's Merkle leaf hash: lane j
//   produces next[j] and next[j + n/4] (from pairs j and j + n/4), stores
//   both and the digest of the pair (next[j], next[j + n/4]) -- the next
//   layer is written once and never re-read for hashing.
#include "field.hpp"
#include "merkle.hpp"
#include "merkle_dev.hpp"
#include "sc_dev.hpp"
#include "sha256.hpp"
#include "transcript_dev.hpp"

namespace mlh {

// ASM: the products through the generated asm multiply (sc_dev.hpp fe_mul_s,
// 72 VALU against ~85 for the C++ fe_mul): faster in the latency-bound
// one-workgroup tail steps, slower in the streaming fold + leaves kernel
// (measured: 39.6 -> 38.7 us and 71.2 -> 74.0 us per launch)
#ifndef MLH_FOLD_ASM
#define MLH_FOLD_ASM 2  // 0: C++ products everywhere, 1: asm everywhere, 2: asm in the tail steps only
#endif
template <bool ASM>
__device__ __forceinline__ fe fold_one(const fe& a, const fe& b, const fe& r, const fe& tw) {
  const fe even = fe_add(a, b);
  const fe odd = ASM ? fe_mul_s(fe_sub(a, b), tw) : fe_mul(fe_sub(a, b), tw);
  return fe_half(fe_add(even, ASM ? fe_mul_s(r, odd) : fe_mul(r, odd)));
}

template <bool ASM = false>
__device__ __forceinline__ fe twiddle(const fe* tlo, const fe* thi, uint64_t e) {
  return ASM ? fe_mul_s(tlo[e & 4095], thi[e >> 12]) : fe_mul(tlo[e & 4095], thi[e >> 12]);
}
constexpr bool kFoldAsmStream = MLH_FOLD_ASM == 1, kFoldAsmTail = MLH_FOLD_ASM >= 1;

__global__ void __launch_bounds__(256)
fold_layer_table_kernel(fe* __restrict__ out, const fe* __restrict__ tlo, const fe* __restrict__ thi,
                        uint32_t L) {
  const uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= (1ull << L) - 1) return;
  const uint64_t y = (1ull << L) - o;  // in [2, 2^L]: layer k has y in (2^(L-1-k), 2^(L-k)]
  const uint32_t k = L - (64 - __builtin_clzll(y - 1));
  const uint64_t j = o - ((1ull << L) - (1ull << (L - k)));
  fe_store(out + o, twiddle(tlo, thi, j << k));
}

hipError_t launch_fold_layer_table(fe* out, const fe* tlo_inv, const fe* thi_inv, uint32_t L,
                                   hipStream_t st) {
  if (L < 2 || L > 40) return hipErrorInvalidValue;
  const uint64_t n = (1ull << L) - 1;
  hipLaunchKernelGGL(fold_layer_table_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out,
                     tlo_inv, thi_inv, L);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256)
fri_fold_kernel(const fe* __restrict__ layer, uint64_t n, fe* __restrict__ next, fe r,
                const fe* __restrict__ tlo, const fe* __restrict__ thi, uint32_t k, uint64_t n0,
                ShardMap map, const fe* __restrict__ rp) {
  if (rp) r = fe_load(rp);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t h = n / 2;
  if (i >= h) return;
  const fe a = fe_load(layer + i), b = fe_load(layer + i + h);
  const fe tw = twiddle<kFoldAsmStream>(tlo, thi, (map.global(i) << k) & (n0 - 1));
  fe_store(next + i, fold_one<kFoldAsmStream>(a, b, r, tw));
}

// job.st non-null: the grid's last workgroup runs that PCS round instead
// (sc_dev.hpp pcs_round_body; it reads the same challenge, so it overlaps the
// fold and the tree instead of sitting between them).
__global__ void __launch_bounds__(256)
fri_fold_leaves_kernel(const fe* __restrict__ layer, uint64_t n, fe* __restrict__ next,
                       uint8_t* __restrict__ leaves, fe r, const fe* __restrict__ tlo,
                       const fe* __restrict__ thi, uint32_t k, uint64_t n0, ShardMap map,
                       const fe* __restrict__ rp, PcsJob job, const fe* __restrict__ twl) {
  if (job.st && blockIdx.x == gridDim.x - 1) {
    pcs_round_body(job);
    return;
  }
  if (rp) r = fe_load(rp);
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t h = n / 2, q = n / 4;
  if (j >= q) return;
  const fe a0 = fe_load(layer + j), b0 = fe_load(layer + j + h);
  const fe a1 = fe_load(layer + j + q), b1 = fe_load(layer + j + q + h);
  fe tw0, tw1;
  if (twl) {
    tw0 = fe_load(twl + j);
    tw1 = fe_load(twl + j + q);
  } else {
    tw0 = twiddle<kFoldAsmStream>(tlo, thi, (map.global(j) << k) & (n0 - 1));
    tw1 = twiddle<kFoldAsmStream>(tlo, thi, (map.global(j + q) << k) & (n0 - 1));
  }
  const fe x0 = fold_one<kFoldAsmStream>(a0, b0, r, tw0);
  const fe x1 = fold_one<kFoldAsmStream>(a1, b1, r, tw1);
  fe_store(next + j, x0);
  fe_store(next + j + q, x1);
  uint32_t m[8];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    m[t] = bswap32(x0.w[t]);
    m[4 + t] = bswap32(x1.w[t]);
  }
  digest_store(leaves + j * 32, sha256_msg32(m));
}

// fold_step + commit of a next layer whose tree has L = n/4 <= 1024 leaves,
// in ONE workgroup of max(64, L) threads (the latency-bound tail rounds of a
// prove): lane j folds pairs j and j + L, hashes leaf j into shared memory,
// the levels run in shared memory (lds_tree_levels), wave 0 absorbs the root
// (+ poly) and draws the next challenge (root_transcript); job.st: the PCS
// round whose polynomial that absorb takes runs in between (sc_dev.hpp).
// One launch per round instead of fold + top (+ the PCS round's): each launch
// boundary drains the chain for several microseconds.
__global__ void __launch_bounds__(1024)
fri_fold_commit_small_kernel(const fe* __restrict__ layer, uint64_t n, fe* __restrict__ next,
                             uint8_t* __restrict__ tree, fe r, const fe* __restrict__ tlo,
                             const fe* __restrict__ thi, uint32_t k, uint64_t n0, ShardMap map,
                             const fe* __restrict__ rp, RootAbsorb ra, PcsJob job,
                             const fe* __restrict__ twl) {
  __shared__ Sha256State s[1024];
  __shared__ DevSha ts;
  __shared__ uint32_t stage[8], pw[8];
  if (ra.t && threadIdx.x < sizeof(DevSha) / 4)
    reinterpret_cast<uint32_t*>(&ts)[threadIdx.x] = reinterpret_cast<const uint32_t*>(ra.t)[threadIdx.x];
  if (rp) r = fe_load(rp);
  const uint64_t h = n / 2, q = n / 4;
  const uint32_t j = threadIdx.x;
  if (j < q) {
    const fe a0 = fe_load(layer + j), b0 = fe_load(layer + j + h);
    const fe a1 = fe_load(layer + j + q), b1 = fe_load(layer + j + q + h);
    const fe tw0 = twl ? fe_load(twl + j) : twiddle<kFoldAsmTail>(tlo, thi, (map.global(j) << k) & (n0 - 1));
    const fe tw1 = twl ? fe_load(twl + j + q)
                       : twiddle<kFoldAsmTail>(tlo, thi, (map.global(j + q) << k) & (n0 - 1));
    const fe x0 = fold_one<kFoldAsmTail>(a0, b0, r, tw0);
    const fe x1 = fold_one<kFoldAsmTail>(a1, b1, r, tw1);
    fe_store(next + j, x0);
    fe_store(next + j + q, x1);
    uint32_t m[8];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      m[t] = bswap32(x0.w[t]);
      m[4 + t] = bswap32(x1.w[t]);
    }
    const Sha256State leaf = sha256_msg32(m);
    s[j] = leaf;
    digest_store(tree + (uint64_t)j * 32, leaf);
  }
  if (job.st) pcs_round_body(job);  // (every thread: it reduces over the workgroup)
  __syncthreads();
  if (ra.poly_in && threadIdx.x < 8)  // written just above when job.st (same workgroup)
    pw[threadIdx.x] = reinterpret_cast<const uint32_t*>(ra.poly_in)[threadIdx.x];
  __syncthreads();
  lds_tree_levels(s, q, tree + q * 32);
  root_transcript(s[0], ts, stage, ra.poly_in ? pw : nullptr, ra);
}

// fold_step + commit of the next layer.  (A variant that also hashed the
// tree's first two levels in the fold lanes, like leaf_pairs_level2_kernel,
// measured 10 % slower over a FRI prove: 8 folds + 7 hashes per lane need
// 129 VGPRs, 3 waves per SIMD, against the fold's 4 memory streams.)
hipError_t launch_fri_fold_commit(const fe* layer, uint64_t n, fe* next, uint8_t* tree, fe r,
                                  const fe* tlo_inv, const fe* thi_inv, uint32_t k, uint64_t n0,
                                  hipStream_t st, ShardMap map, const fe* r_dev, RootAbsorb ra,
                                  const PcsJob* job, const fe* twl) {
#ifndef MLH_FRI_SMALL_LEAVES
#define MLH_FRI_SMALL_LEAVES 1024  // trees of at most this many leaves: one fused launch (0: off)
#endif
  if (n / 4 <= MLH_FRI_SMALL_LEAVES && n >= 8) {
    PcsJob pj{};
    if (job) {
      if (job->log_h < 1 || job->log_h > 12 || (job->fold && !job->r_prev) || (job->r_prev && !job->p_prev))
        return hipErrorInvalidValue;
      pj = *job;
    }
    const unsigned threads = n / 4 < 64 ? 64 : (unsigned)(n / 4);
    hipLaunchKernelGGL(fri_fold_commit_small_kernel, dim3(1), dim3(threads), 0, st, layer, n, next, tree,
                       r, tlo_inv, thi_inv, k, n0, map, r_dev, ra, pj, twl);
    return hipGetLastError();
  }
  hipError_t e = launch_fri_fold_leaves(layer, n, next, tree, r, tlo_inv, thi_inv, k, n0, st, map,
                                        r_dev, job, twl);
  if (e != hipSuccess) return e;
  return launch_merkle_levels(tree, n / 4, st, ra);
}

hipError_t launch_fri_fold(const fe* layer, uint64_t n, fe* next, fe r, const fe* tlo_inv,
                           const fe* thi_inv, uint32_t k, uint64_t n0, hipStream_t st,
                           ShardMap map, const fe* r_dev) {
  const uint64_t h = n / 2;
  hipLaunchKernelGGL(fri_fold_kernel, dim3((unsigned)((h + 255) / 256)), dim3(256), 0, st, layer,
                     n, next, r, tlo_inv, thi_inv, k, n0, map, r_dev);
  return hipGetLastError();
}

hipError_t launch_fri_fold_leaves(const fe* layer, uint64_t n, fe* next, uint8_t* leaves, fe r,
                                  const fe* tlo_inv, const fe* thi_inv, uint32_t k, uint64_t n0,
                                  hipStream_t st, ShardMap map, const fe* r_dev, const PcsJob* job,
                                  const fe* twl) {
  const uint64_t q = n / 4;
  PcsJob pj{};
  if (job) {
    if (job->log_h < 1 || job->log_h > 12 || (job->fold && !job->r_prev) || (job->r_prev && !job->p_prev))
      return hipErrorInvalidValue;
    pj = *job;
  }
  const unsigned blocks = (unsigned)((q + 255) / 256) + (job ? 1u : 0u);
  hipLaunchKernelGGL(fri_fold_leaves_kernel, dim3(blocks), dim3(256), 0, st, layer, n, next, leaves,
                     r, tlo_inv, thi_inv, k, n0, map, r_dev, pj, twl);
  return hipGetLastError();
}

}  // namespace mlh

// ---- device transcript steps (transcript_dev.hpp) ---------------------------
namespace mlh {

__global__ void transcript_absorb_kernel(DevSha* t, const uint8_t* src, uint32_t n, fe* r_out,
                                         uint8_t* copy_out) {
  // the state lives in LDS while a single lane updates it (the byte buffer is
  // indexed dynamically; in VGPRs it would spill to scratch).  State and
  // source are loaded by parallel lanes (one word each); lane 0 then absorbs
  // from registers (a global source costs a dependent load per word).
  __shared__ DevSha s;
  __shared__ uint32_t stage[8], stage2[8];
  const uint32_t tid = threadIdx.x;
  const bool words = (n == 32 || n == 16) &&
                     (((uintptr_t)src | (uintptr_t)copy_out) & 3) == 0;
  if (tid < sizeof(DevSha) / 4)
    reinterpret_cast<uint32_t*>(&s)[tid] = reinterpret_cast<const uint32_t*>(t)[tid];
  if (words && tid < n / 4) {
    const uint32_t v = reinterpret_cast<const uint32_t*>(src)[tid];
    stage[tid] = v;
    if (copy_out) reinterpret_cast<uint32_t*>(copy_out)[tid] = v;
  }
  __syncthreads();
  // (one wave: the word paths on a lane pair, dsha2l_step)
  if (words && n == 32) {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = stage[i];
    dsha2l_step<8>(s, w, stage2, r_out);
  } else if (words) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = stage[i];
    dsha2l_step<4>(s, w, stage2, r_out);
  } else if (tid == 0) {
    dsha_update(s, src, n);
    if (copy_out)
      for (uint32_t i = 0; i < n; ++i) copy_out[i] = src[i];
    if (r_out) fe_store(r_out, dsha_challenge(s));
  }
  if (tid == 0) *t = s;
}

hipError_t launch_transcript_absorb(DevSha* t, const uint8_t* src, uint32_t n, fe* r_out,
                                    hipStream_t st, uint8_t* copy_out) {
  hipLaunchKernelGGL(transcript_absorb_kernel, dim3(1), dim3(64), 0, st, t, src, n, r_out,
                     copy_out);
  return hipGetLastError();
}

__global__ void fri_last_kernel(const fe* vals, DevSha* t, uint32_t* flag, fe* last_out) {
  __shared__ DevSha s;
  __shared__ uint32_t stage[4];
  if (threadIdx.x < sizeof(DevSha) / 4)
    reinterpret_cast<uint32_t*>(&s)[threadIdx.x] = reinterpret_cast<const uint32_t*>(t)[threadIdx.x];
  __syncthreads();
  const fe a = fe_load(vals), b = fe_load(vals + 1);
  if (threadIdx.x == 0) {
    *flag = fe_eq(a, b) ? 0u : 1u;
    fe_store(last_out, a);
  }
  const uint32_t w[4] = {a.w[0], a.w[1], a.w[2], a.w[3]};
  dsha2l_step<4>(s, w, stage, nullptr);  // LE16(last) (one wave, lane pair)
  if (threadIdx.x == 0) *t = s;
}

hipError_t launch_fri_last(const fe* vals, DevSha* t, uint32_t* flag, fe* last_out,
                           hipStream_t st) {
  hipLaunchKernelGGL(fri_last_kernel, dim3(1), dim3(64), 0, st, vals, t, flag, last_out);
  return hipGetLastError();
}

}  // namespace mlh
