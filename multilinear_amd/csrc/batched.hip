// Batched FRI / batched PCS kernels (src/fri/batched_fri.rs, batched_pcs.rs).
//
// m codes of N elements are stored back to back ([m][N], code j at j*N).
// * batch_pairs_leaf_kernel: leaf i = SHA256(pair_0[i] || ... || pair_{m-1}[i]),
//   pair_j[i] = LE16(code_j[i]) || LE16(code_j[i + N/2]) -- Merkle::batch_commit
//   of the RS pairs (merkle_tree/mod.rs:92-131); two pairs per 64-byte block;
// * fingerprint(r, c_0..c_{m-1}) is Horner, sum_j c_j r^(m-1-j)
//   (batched_fri.rs:30-38);
// * batched_fold_leaves_kernel: batched_fold_step (batched_fri.rs:100-176) --
//   fingerprints of the values and of the minus-values, the k = 0 fold, and
//   the next layer's leaf hash, as fri_fold_leaves_kernel does for one code;
// * fingerprint_kernel: the fingerprinted MLE of batched_pcs.rs:57-65.
// Every challenge is read from device memory (device transcript).
#include "batched.hpp"
#include "sha256.hpp"

namespace mlh {

__device__ __forceinline__ fe horner(const fe* __restrict__ base, uint64_t stride, uint32_t m,
                                     uint64_t i, const fe& r) {
  fe acc = fe_load(base + i);
  for (uint32_t j = 1; j < m; ++j) acc = fe_add(fe_mul(acc, r), fe_load(base + j * stride + i));
  return acc;
}

__global__ void __launch_bounds__(256)
batch_pairs_leaf_kernel(const fe* __restrict__ codes, uint32_t m, uint64_t N,
                        uint8_t* __restrict__ leaves) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t h = N / 2;
  if (i >= h) return;
  Sha256State st = sha256_iv();
  uint32_t w[16];
  auto put_pair = [&](uint32_t j, int at) {
    const fe a = fe_load(codes + (uint64_t)j * N + i), b = fe_load(codes + (uint64_t)j * N + i + h);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      w[at + k] = bswap32(a.w[k]);
      w[at + 4 + k] = bswap32(b.w[k]);
    }
  };
  uint32_t j = 0;
  for (; j + 2 <= m; j += 2) {
    put_pair(j, 0);
    put_pair(j + 1, 8);
    sha256_compress(st, w);
  }
  const uint32_t bits = 256u * m;  // message length in bits (m < 2^24)
  if (j < m) {  // one pair + padding fit the last block (32 + 1 + 8 <= 64)
    put_pair(j, 0);
    w[8] = 0x80000000u;
#pragma unroll
    for (int k = 9; k < 15; ++k) w[k] = 0;
    w[15] = bits;
  } else {
    w[0] = 0x80000000u;
#pragma unroll
    for (int k = 1; k < 15; ++k) w[k] = 0;
    w[15] = bits;
  }
  sha256_compress(st, w);
  digest_store(leaves + i * 32, st);
}

__device__ __forceinline__ fe bfold(const fe& a, const fe& b, const fe& r, const fe& tw) {
  const fe even = fe_add(a, b);
  const fe odd = fe_mul(fe_sub(a, b), tw);
  return fe_half(fe_add(even, fe_mul(r, odd)));
}

// lane j < N/4 (or the single lane of N = 4): next[j], next[j + N/4] and, if
// leaves, the digest of the next layer's pair j.
__global__ void __launch_bounds__(256)
batched_fold_leaves_kernel(const fe* __restrict__ codes, uint32_t m, uint64_t N,
                           const fe* __restrict__ frp, const fe* __restrict__ rp,
                           const fe* __restrict__ tlo, const fe* __restrict__ thi,
                           fe* __restrict__ next, uint8_t* __restrict__ leaves) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t h = N / 2, q = N / 4;
  if (j >= q) return;
  const fe fr = fe_load(frp), r = fe_load(rp);
  const fe a0 = horner(codes, N, m, j, fr), b0 = horner(codes, N, m, j + h, fr);
  const fe a1 = horner(codes, N, m, j + q, fr), b1 = horner(codes, N, m, j + q + h, fr);
  const fe x0 = bfold(a0, b0, r, fe_mul(tlo[j & 4095], thi[j >> 12]));
  const uint64_t e1 = j + q;
  const fe x1 = bfold(a1, b1, r, fe_mul(tlo[e1 & 4095], thi[e1 >> 12]));
  fe_store(next + j, x0);
  fe_store(next + j + q, x1);
  if (!leaves) return;
  uint32_t msg[8];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    msg[t] = bswap32(x0.w[t]);
    msg[4 + t] = bswap32(x1.w[t]);
  }
  digest_store(leaves + j * 32, sha256_msg32(msg));
}

__global__ void __launch_bounds__(256)
fingerprint_kernel(const fe* __restrict__ polys, uint32_t m, uint64_t n,
                   const fe* __restrict__ frp, fe* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe_store(out + i, horner(polys, n, m, i, fe_load(frp)));
}

// Opened batch column + batch-tree siblings for each query (batched_fri.rs:
// 207-224, Merkle::batch_open): record q at out + q * qbytes.
__global__ void batch_query_kernel(const fe* __restrict__ codes, uint32_t m, uint64_t N,
                                   const uint8_t* __restrict__ tree,
                                   const QueryIdx idx, uint64_t qbytes,
                                   uint8_t* __restrict__ out) {
  const uint32_t qi = blockIdx.x;
  const uint64_t h = N / 2, i = idx.v[qi];
  uint8_t* rec = out + qi * qbytes;
  for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
    fe_store(reinterpret_cast<fe*>(rec + 32ull * j), fe_load(codes + (uint64_t)j * N + i));
    fe_store(reinterpret_cast<fe*>(rec + 32ull * j + 16), fe_load(codes + (uint64_t)j * N + i + h));
  }
  const uint32_t depth = 63 - __builtin_clzll(h);  // leaves = N/2
  uint8_t* sib = rec + 32ull * m;
  for (uint32_t l = threadIdx.x; l < depth; l += blockDim.x) {
    uint64_t off = 0;
    for (uint32_t t = 0; t < l; ++t) off += h >> t;
    const uint4* src = reinterpret_cast<const uint4*>(tree + (off + ((i >> l) ^ 1ull)) * 32);
    uint4* dst = reinterpret_cast<uint4*>(sib + 32ull * l);
    dst[0] = src[0];
    dst[1] = src[1];
  }
}

// prev = fingerprint(fr, outputs) (batched_pcs.rs:90-91), one lane
__global__ void fingerprint_scalar_kernel(const fe* __restrict__ vals, uint32_t m,
                                          const fe* __restrict__ frp, fe* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  fe_store(out, horner(vals, 1, m, 0, fe_load(frp)));
}

static inline unsigned nblocks(uint64_t n) { return (unsigned)((n + 255) / 256); }

hipError_t launch_batch_pairs_leaves(const fe* codes, uint32_t m, uint64_t N, uint8_t* leaves,
                                     hipStream_t st) {
  hipLaunchKernelGGL(batch_pairs_leaf_kernel, dim3(nblocks(N / 2)), dim3(256), 0, st, codes, m, N,
                     leaves);
  return hipGetLastError();
}

hipError_t launch_batched_fold_leaves(const fe* codes, uint32_t m, uint64_t N, const fe* fr,
                                      const fe* r, const fe* tlo, const fe* thi, fe* next,
                                      uint8_t* leaves, hipStream_t st) {
  hipLaunchKernelGGL(batched_fold_leaves_kernel, dim3(nblocks(N / 4)), dim3(256), 0, st, codes, m,
                     N, fr, r, tlo, thi, next, leaves);
  return hipGetLastError();
}

hipError_t launch_fingerprint(const fe* polys, uint32_t m, uint64_t n, const fe* fr, fe* out,
                              hipStream_t st) {
  hipLaunchKernelGGL(fingerprint_kernel, dim3(nblocks(n)), dim3(256), 0, st, polys, m, n, fr, out);
  return hipGetLastError();
}

hipError_t launch_fingerprint_scalar(const fe* vals, uint32_t m, const fe* fr, fe* out,
                                     hipStream_t st) {
  hipLaunchKernelGGL(fingerprint_scalar_kernel, dim3(1), dim3(64), 0, st, vals, m, fr, out);
  return hipGetLastError();
}

hipError_t launch_batch_queries(const fe* codes, uint32_t m, uint64_t N, const uint8_t* tree,
                                const QueryIdx& idx, uint32_t nq, uint64_t qbytes, uint8_t* out,
                                hipStream_t st) {
  if (nq == 0) return hipSuccess;
  if (nq > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(batch_query_kernel, dim3(nq), dim3(64), 0, st, codes, m, N, tree, idx, qbytes,
                     out);
  return hipGetLastError();
}

}  // namespace mlh
