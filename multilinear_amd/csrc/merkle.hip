// SHA-256 Merkle tree build on gfx950.
//
// Reference: src/merkle_tree/mod.rs:65-85 (Merkle::commit: leaf digests, then
// `chunks(2)` levels until one digest is left, every layer kept), :92-131
// (batch_commit), :178-189 (hash_leaf / hash_node), and src/fri/mod.rs:45-55
// (commit_rs_code: leaf i = LE16(code[i]) ‖ LE16(code[i + n/2])).
//
// HBM layout of a tree with L = 2^l leaves: one buffer of 2L-1 digests in
// level order (leaves at [0, L), level 1 at [L, L + L/2), ..., root last),
// each digest the standard 32 SHA-256 output bytes.
//
// Kernels (one lane = one message; SHA-256 is VALU-bound, ~2k ops per
// compression, so the design goal is full lanes, not bandwidth):
//   * leaf_pairs   : leaf i from the RS pair (code[i], code[i + half]);
//   * leaf_bytes   : generic fixed-length items (Merkle::commit over any T);
//   * level2       : one lane builds a 2-level subtree (4 children -> 2 -> 1),
//                    halving the launch count;
//   * top          : one workgroup finishes the last <= 1024 nodes in LDS.
#include "field.hpp"
#include "merkle.hpp"
#include "merkle_dev.hpp"
#include "sha256.hpp"
#include "transcript_dev.hpp"

namespace mlh {

#ifdef MLH_TREE_TS
__device__ uint64_t g_tree_ts[4][64];
// host access for the bench (out: 4 x 64 stamps; clear before a stamped call)
hipError_t tree_ts_read(uint64_t* out, bool clear) {
  if (clear) {
    static const uint64_t zero[4][64] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_tree_ts), zero, sizeof(zero));
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tree_ts), sizeof(g_tree_ts));
}
#endif

__global__ void __launch_bounds__(256)
leaf_pairs_kernel(const fe* __restrict__ code, uint64_t half, uint8_t* __restrict__ leaves) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= half) return;
  const fe a = fe_load(code + i), b = fe_load(code + i + half);
  uint32_t m[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    m[k] = bswap32(a.w[k]);
    m[4 + k] = bswap32(b.w[k]);
  }
  digest_store(leaves + i * 32, sha256_msg32(m));
}

// Leaves 4j..4j+3 of commit_rs_code plus their two parents and grandparent
// in one lane: the leaf hashes never make a round trip through HBM before the
// first two levels, and the leaf level costs no launch of its own.
__global__ void __launch_bounds__(256)
leaf_pairs_level2_kernel(const fe* __restrict__ code, uint64_t half, uint8_t* __restrict__ layers) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= half / 4) return;
  Sha256State lf[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint64_t i = 4 * j + q;
    const fe a = fe_load(code + i), b = fe_load(code + i + half);
    uint32_t m[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      m[k] = bswap32(a.w[k]);
      m[4 + k] = bswap32(b.w[k]);
    }
    lf[q] = sha256_msg32(m);
    digest_store(layers + i * 32, lf[q]);
  }
  const Sha256State p0 = sha256_node(lf[0], lf[1]), p1 = sha256_node(lf[2], lf[3]);
  digest_store(layers + (half + 2 * j) * 32, p0);
  digest_store(layers + (half + 2 * j + 1) * 32, p1);
  digest_store(layers + (half + half / 2 + j) * 32, sha256_node(p0, p1));
}

// Generic leaf: SHA256 of `item_len` bytes at items + i*item_len (any length).
__global__ void leaf_bytes_kernel(const uint8_t* __restrict__ items, uint64_t item_len,
                                  uint64_t count, uint8_t* __restrict__ leaves) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint8_t* p = items + i * item_len;
  Sha256State st = sha256_iv();
  uint32_t w[16];
  const uint64_t total = item_len + 9;  // + 0x80 + 8-byte length
  const uint64_t nblocks = (total + 63) / 64;
  for (uint64_t blk = 0; blk < nblocks; ++blk) {
    for (int wi = 0; wi < 16; ++wi) {
      uint32_t word = 0;
      for (int bi = 0; bi < 4; ++bi) {
        const uint64_t pos = blk * 64 + wi * 4 + bi;
        uint32_t byte;
        if (pos < item_len) {
          byte = p[pos];
        } else if (pos == item_len) {
          byte = 0x80u;
        } else if (pos >= nblocks * 64 - 8) {
          const uint64_t bits = item_len * 8;
          const int sh = (int)(nblocks * 64 - 1 - pos) * 8;
          byte = (uint32_t)((bits >> sh) & 0xFF);
        } else {
          byte = 0;
        }
        word = (word << 8) | byte;
      }
      w[wi] = word;
    }
    sha256_compress(st, w);
  }
  digest_store(leaves + i * 32, st);
}

// Batch leaf (merkle_tree/mod.rs:109-116): SHA256 of the m items data[j][i]
// (j < m) concatenated; items are item_len bytes, batch j at items + j*stride.
__global__ void leaf_batch_kernel(const uint8_t* __restrict__ items, uint64_t item_len,
                                  uint64_t batch_stride, uint32_t m, uint64_t count,
                                  uint8_t* __restrict__ leaves) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint64_t msg_len = item_len * m;
  Sha256State st = sha256_iv();
  uint32_t w[16];
  const uint64_t total = msg_len + 9;
  const uint64_t nblocks = (total + 63) / 64;
  for (uint64_t blk = 0; blk < nblocks; ++blk) {
    for (int wi = 0; wi < 16; ++wi) {
      uint32_t word = 0;
      for (int bi = 0; bi < 4; ++bi) {
        const uint64_t pos = blk * 64 + wi * 4 + bi;
        uint32_t byte;
        if (pos < msg_len) {
          const uint64_t j = pos / item_len, o = pos % item_len;
          byte = items[j * batch_stride + i * item_len + o];
        } else if (pos == msg_len) {
          byte = 0x80u;
        } else if (pos >= nblocks * 64 - 8) {
          const uint64_t bits = msg_len * 8;
          const int sh = (int)(nblocks * 64 - 1 - pos) * 8;
          byte = (uint32_t)((bits >> sh) & 0xFF);
        } else {
          byte = 0;
        }
        word = (word << 8) | byte;
      }
      w[wi] = word;
    }
    sha256_compress(st, w);
  }
  digest_store(leaves + i * 32, st);
}

// One lane: children 4j..4j+3 -> parents 2j, 2j+1 -> grandparent j.
__global__ void __launch_bounds__(256)
level2_kernel(const uint8_t* __restrict__ child, uint8_t* __restrict__ parent,
              uint8_t* __restrict__ grand, uint64_t ngrand) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ngrand) return;
  const uint8_t* c = child + j * 128;
  const Sha256State c0 = digest_load(c), c1 = digest_load(c + 32);
  const Sha256State p0 = sha256_node(c0, c1);
  digest_store(parent + (2 * j) * 32, p0);
  const Sha256State c2 = digest_load(c + 64), c3 = digest_load(c + 96);
  const Sha256State p1 = sha256_node(c2, c3);
  digest_store(parent + (2 * j + 1) * 32, p1);
  digest_store(grand + j * 32, sha256_node(p0, p1));
}

__global__ void __launch_bounds__(256)
level1_kernel(const uint8_t* __restrict__ child, uint8_t* __restrict__ parent, uint64_t nparent) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nparent) return;
  const Sha256State a = digest_load(child + j * 64), b = digest_load(child + j * 64 + 32);
  digest_store(parent + j * 32, sha256_node(a, b));
}

// Finish a level of n <= 1024 digests (n a power of two >= 2) to the root in
// one workgroup; writes every level into `out` consecutively.  ra.t: wave 0
// then absorbs the root (and ra.poly_in) into the device transcript
// (RootAbsorb, merkle_dev.hpp); the state is staged into LDS by parallel lanes
// while the levels run.
__global__ void __launch_bounds__(512)
top_kernel(const uint8_t* __restrict__ level, uint64_t n, uint8_t* __restrict__ out,
           RootAbsorb ra) {
  __shared__ Sha256State s[1024];
  __shared__ DevSha ts;
  __shared__ uint32_t stage[8], pw[8];
  MLH_TREE_STAMP(1, 0);
  if (ra.t && threadIdx.x < sizeof(DevSha) / 4)
    reinterpret_cast<uint32_t*>(&ts)[threadIdx.x] = reinterpret_cast<const uint32_t*>(ra.t)[threadIdx.x];
  if (ra.poly_in && threadIdx.x < 8)  // (loaded with the level, not on lane 0's chain)
    pw[threadIdx.x] = reinterpret_cast<const uint32_t*>(ra.poly_in)[threadIdx.x];
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) s[i] = digest_load(level + i * 32);
  __syncthreads();
  MLH_TREE_STAMP(1, 1);
  lds_tree_levels(s, n, out);
  root_transcript(s[0], ts, stage, ra.poly_in ? pw : nullptr, ra);
  MLH_TREE_STAMP(1, 63);
}

// The latency-bound tail of a tree (levels of <= kTailLevel digests, ~one
// wave per SIMD or less): each workgroup reduces a chunk of C = 2*blockDim.x
// digests to its subtree root through LDS, all log2(C) levels in one launch
// (a level costs one SHA-256 latency, ~4.1 us, not a launch); top_kernel then
// finishes the subtree roots.  Level i >= 1 below `level` is written at
// out + (n/2 + ... + n/2^(i-1)) digests, i.e. the tree's level order.
// (A last-arriving-workgroup finish in the same launch measured slower: its
// device-scope fences write back and invalidate L2 in every workgroup.)
__global__ void __launch_bounds__(512)
subtree_kernel(const uint8_t* __restrict__ level, uint64_t n, uint8_t* __restrict__ out) {
  __shared__ Sha256State s[512];
  const uint32_t t = threadIdx.x;
  const uint64_t b = blockIdx.x;
  uint32_t m = blockDim.x;  // nodes of this chunk at the current level
  const uint8_t* c = level + (b * 2 * m + 2 * t) * 32;
  MLH_TREE_STAMP(0, 0);
  const Sha256State c0 = digest_load(c), c1 = digest_load(c + 32);
  MLH_TREE_STAMP(0, 1);
  Sha256State r = sha256_node(c0, c1);
  uint64_t off = 0, lvl = n / 2;  // offset and size of the current level in out
  digest_store(out + (off + b * m + t) * 32, r);
  s[t] = r;
  MLH_TREE_STAMP(0, 2);
  while (m > 1) {
    off += lvl;
    lvl /= 2;
    const uint32_t mp = m / 2;
    __syncthreads();
    // levels after the first have at most half a node per thread: a lane
    // pair per node (two-lane SHA-256, ~20 % less latency per level) once the
    // pairs fit one wave per SIMD (pair_level), one lane per node before
    const bool two = pair_level(mp);
    const uint32_t node = two ? sha2l_pair(t) : t;
    const bool active = node < mp;
    if (active) r = two ? sha2l_node(s[2 * node], s[2 * node + 1]) : sha256_node(s[2 * node], s[2 * node + 1]);
    __syncthreads();
    if (active && (!two || sha2l_lead(t))) {
      s[node] = r;
      digest_store(out + (off + b * mp + node) * 32, r);
    }
    MLH_TREE_STAMP(0, 2 + __builtin_ctz(blockDim.x / mp));
    m = mp;
  }
}

static inline unsigned blocks_for(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

hipError_t launch_leaf_pairs(const fe* code, uint64_t half, uint8_t* leaves, hipStream_t st) {
  hipLaunchKernelGGL(leaf_pairs_kernel, dim3(blocks_for(half, 256)), dim3(256), 0, st, code, half,
                     leaves);
  return hipGetLastError();
}

hipError_t launch_leaf_bytes(const uint8_t* items, uint64_t item_len, uint64_t count,
                             uint8_t* leaves, hipStream_t st) {
  hipLaunchKernelGGL(leaf_bytes_kernel, dim3(blocks_for(count, 128)), dim3(128), 0, st, items,
                     item_len, count, leaves);
  return hipGetLastError();
}

hipError_t launch_leaf_batch(const uint8_t* items, uint64_t item_len, uint64_t batch_stride,
                             uint32_t m, uint64_t count, uint8_t* leaves, hipStream_t st) {
  hipLaunchKernelGGL(leaf_batch_kernel, dim3(blocks_for(count, 128)), dim3(128), 0, st, items,
                     item_len, batch_stride, m, count, leaves);
  return hipGetLastError();
}

// Levels above the level of n digests at layers + off digests (level order).
hipError_t launch_merkle_levels_from(uint8_t* layers, uint64_t off, uint64_t n, hipStream_t st,
                                     RootAbsorb ra) {
  constexpr uint64_t kTailLevel = 1ull << 18;  // 256 workgroups of 1024-digest chunks
  constexpr uint64_t kChunk = 1024;
  constexpr unsigned kSpreadLds = 96 * 1024;
  while (n > kTailLevel) {
    uint8_t* child = layers + off * 32;
    uint8_t* parent = child + n * 32;
    if (n >= 4 * 1024) {
      uint8_t* grand = parent + (n / 2) * 32;
      hipLaunchKernelGGL(level2_kernel, dim3(blocks_for(n / 4, 256)), dim3(256), 0, st, child,
                         parent, grand, n / 4);
      off += n + n / 2;
      n /= 4;
    } else {
      hipLaunchKernelGGL(level1_kernel, dim3(blocks_for(n / 2, 256)), dim3(256), 0, st, child,
                         parent, n / 2);
      off += n;
      n /= 2;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (n > 1024) {
    // Chunks of 1024 at 2^18 digests (2^17 hashes = 2 waves per SIMD however
    // they are cut), 512 below it, so that the first level is one wave per
    // SIMD.  The (unused) dynamic LDS keeps it to one workgroup per CU: two on
    // a CU would double every level's latency while other CUs idle.
    const uint64_t chunk = n >= kTailLevel ? kChunk : kChunk / 2;
    hipLaunchKernelGGL(subtree_kernel, dim3((unsigned)(n / chunk)), dim3((unsigned)(chunk / 2)),
                       kSpreadLds, st, layers + off * 32, n, layers + (off + n) * 32);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    for (uint64_t c = chunk; c > 1; c /= 2) {  // input level + log2(chunk) - 1 levels
      off += n;
      n /= 2;
    }
  }
  if (n > 1) {
    // n <= the pair limit: a thread per digest, so that the first level runs
    // on lane pairs too
    const unsigned threads = n <= MLH_PAIR_LEVELS_MAX ? (n < 64 ? 64 : (unsigned)n)
                                                       : (n / 2 < 64 ? 64 : (unsigned)(n / 2));
    hipLaunchKernelGGL(top_kernel, dim3(1), dim3(threads), 0, st, layers + off * 32, n,
                       layers + (off + n) * 32, ra);
  } else if (ra.t) {  // the level is the root already (one leaf)
    hipError_t e = launch_transcript_absorb(ra.t, layers + off * 32, 32, ra.poly_in ? nullptr : ra.r_out,
                                            st, ra.copy_out);
    if (e == hipSuccess && ra.poly_in)
      e = launch_transcript_absorb(ra.t, reinterpret_cast<const uint8_t*>(ra.poly_in), 32, ra.r_out, st,
                                   nullptr);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

// layers: 2L-1 digests, leaves already at [0, L).
hipError_t launch_merkle_levels(uint8_t* layers, uint64_t L, hipStream_t st, RootAbsorb ra) {
  return launch_merkle_levels_from(layers, 0, L, st, ra);
}

hipError_t launch_commit_pairs(const fe* code, uint64_t L, uint8_t* layers, hipStream_t st,
                               RootAbsorb ra) {
  if (L < 4) {
    hipError_t e = launch_leaf_pairs(code, L, layers, st);
    if (e != hipSuccess) return e;
    return launch_merkle_levels_from(layers, 0, L, st, ra);
  }
  hipLaunchKernelGGL(leaf_pairs_level2_kernel, dim3(blocks_for(L / 4, 256)), dim3(256), 0, st,
                     code, L, layers);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_merkle_levels_from(layers, L + L / 2, L / 4, st, ra);
}

// Merkle::open (merkle_tree/mod.rs:31-58): for query q (one workgroup) the
// sibling of idx[q] on every level below the root, bottom-up.
__global__ void merkle_path_kernel(const uint8_t* __restrict__ layers, uint64_t L,
                                   const uint64_t* __restrict__ idx, uint8_t* __restrict__ out) {
  const uint32_t depth = 63 - __builtin_clzll(L);
  const uint64_t i = idx[blockIdx.x];
  uint8_t* rec = out + (uint64_t)blockIdx.x * 32 * depth;
  for (uint32_t l = threadIdx.x; l < depth; l += blockDim.x) {
    uint64_t off = 0;
    for (uint32_t t = 0; t < l; ++t) off += L >> t;
    const uint4* src = reinterpret_cast<const uint4*>(layers + (off + ((i >> l) ^ 1ull)) * 32);
    uint4* dst = reinterpret_cast<uint4*>(rec + 32ull * l);
    dst[0] = src[0];
    dst[1] = src[1];
  }
}

hipError_t launch_merkle_paths(const uint8_t* layers, uint64_t L, const uint64_t* idx, uint32_t nq,
                               uint8_t* out, hipStream_t st) {
  if (nq == 0 || L < 2) return hipSuccess;
  hipLaunchKernelGGL(merkle_path_kernel, dim3(nq), dim3(64), 0, st, layers, L, idx, out);
  return hipGetLastError();
}

}  // namespace mlh
