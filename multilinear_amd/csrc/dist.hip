// Sharded building blocks: the cross-shard stage of the distributed NTT and
// leaf openings of a shard's local Merkle subtrees.
//
// Distributed NTT over P = 2^p ranks ("Multi-GPU"): N = P * M,
// rank g holds x[g + P m] (cyclic shard layout).  Then
//   X[j + M t] = sum_g wP^(g t) * w^(g j) * Z_g[j],   Z_g = NTT_M(x[g + P .])
// so each rank runs a plain length-M NTT with generator w^P, one all-to-all
// moves chunk h = Z_g[h S .. (h+1) S) (S = M / P) to rank h, and the kernel
// below finishes with a length-P DFT per column j: it reads the P received
// rows [g][jl], multiplies by w^(g j) and writes the rows [t][jl].  Rank h
// ends up with X[t M + h S + jl] -- a block-cyclic layout with block S, in
// which every FRI pair (i, i + N/2) and every aligned S-leaf Merkle subtree
// is local.  HBM traffic: one read + one write of the shard (32 B/element),
// ~2.3 field multiplications per element (P = 8).
#include "dist.hpp"
#include "sha256.hpp"

namespace mlh {

template <int LOGP>
__device__ __forceinline__ int brev(int p) {
  int r = 0;
#pragma unroll
  for (int b = 0; b < LOGP; ++b) r |= ((p >> b) & 1) << (LOGP - 1 - b);
  return r;
}

template <int LOGP, bool INV>
__global__ void __launch_bounds__(256)
shard_dft_kernel(const fe* __restrict__ in, fe* __restrict__ out, uint64_t S, uint64_t j0,
                 const fe* __restrict__ tlo, const fe* __restrict__ thi,
                 const fe* __restrict__ wp, fe scale) {
  constexpr int P = 1 << LOGP;
  const uint64_t jl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (jl >= S) return;
  const uint64_t j = j0 + jl;
  const fe w1 = fe_mul(tlo[j & 4095], thi[j >> 12]);
  fe y[P];
#pragma unroll
  for (int g = 0; g < P; ++g) y[g] = fe_load(in + (uint64_t)g * S + jl);
  if (!INV) {  // y_g *= w^(g j)
    fe tw = w1;
#pragma unroll
    for (int g = 1; g < P; ++g) {
      y[g] = fe_mul(y[g], tw);
      if (g + 1 < P) tw = fe_mul(tw, w1);
    }
  }
  // radix-2 DIF, natural in, bit-reversed out: y[p] = DFT[brev(p)]
#pragma unroll
  for (int st = 0; st < LOGP; ++st) {
    const int span = P >> (st + 1);
#pragma unroll
    for (int b = 0; b < P; b += 2 * span) {
#pragma unroll
      for (int i = 0; i < span; ++i) {
        const fe u = y[b + i], v = y[b + i + span];
        y[b + i] = fe_add(u, v);
        const fe d = fe_sub(u, v);
        const int e = i * (P / (2 * span));
        y[b + i + span] = e ? fe_mul(d, wp[e]) : d;
      }
    }
  }
  if (!INV) {
#pragma unroll
    for (int p = 0; p < P; ++p) fe_store(out + (uint64_t)brev<LOGP>(p) * S + jl, y[p]);
  } else {  // row g *= scale * w^(-g j)
    fe tw = scale;
#pragma unroll
    for (int g = 0; g < P; ++g) {
      fe_store(out + (uint64_t)g * S + jl, fe_mul(y[brev<LOGP>(g)], tw));
      if (g + 1 < P) tw = fe_mul(tw, w1);
    }
  }
}

template <int LOGP>
static void launch_dft_p(const fe* in, fe* out, uint64_t S, uint64_t j0, bool inverse,
                         const fe* tlo, const fe* thi, const fe* wp, fe scale, hipStream_t st) {
  const dim3 grid((unsigned)((S + 255) / 256)), blk(256);
  if (inverse)
    hipLaunchKernelGGL((shard_dft_kernel<LOGP, true>), grid, blk, 0, st, in, out, S, j0, tlo, thi,
                       wp, scale);
  else
    hipLaunchKernelGGL((shard_dft_kernel<LOGP, false>), grid, blk, 0, st, in, out, S, j0, tlo, thi,
                       wp, scale);
}

hipError_t launch_shard_dft(const fe* in, fe* out, uint64_t S, uint64_t j0, uint32_t log_p,
                            bool inverse, const fe* tlo, const fe* thi, const fe* wp, fe scale,
                            hipStream_t st) {
  switch (log_p) {
    case 1: launch_dft_p<1>(in, out, S, j0, inverse, tlo, thi, wp, scale, st); break;
    case 2: launch_dft_p<2>(in, out, S, j0, inverse, tlo, thi, wp, scale, st); break;
    case 3: launch_dft_p<3>(in, out, S, j0, inverse, tlo, thi, wp, scale, st); break;
    case 4: launch_dft_p<4>(in, out, S, j0, inverse, tlo, thi, wp, scale, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// One workgroup per opened leaf: lane 0 copies the pair, lanes copy siblings.
__global__ void open_pairs_kernel(const fe* __restrict__ values, uint64_t half,
                                  const uint8_t* __restrict__ tree, uint32_t levels,
                                  const uint64_t* __restrict__ idx, uint8_t* __restrict__ out) {
  const uint32_t q = blockIdx.x;
  const uint64_t i = idx[q];
  uint8_t* rec = out + (uint64_t)q * 32 * (1 + levels);
  if (threadIdx.x == 0) {
    fe_store(reinterpret_cast<fe*>(rec), fe_load(values + i));
    fe_store(reinterpret_cast<fe*>(rec + 16), fe_load(values + i + half));
  }
  for (uint32_t l = threadIdx.x; l < levels; l += blockDim.x) {
    uint64_t off = 0;  // level l starts at sum_{m<l} half >> m
    for (uint32_t m = 0; m < l; ++m) off += half >> m;
    const uint4* src = reinterpret_cast<const uint4*>(tree + (off + ((i >> l) ^ 1ull)) * 32);
    uint4* dst = reinterpret_cast<uint4*>(rec + 32 + (uint64_t)l * 32);
    dst[0] = src[0];
    dst[1] = src[1];
  }
}

hipError_t launch_open_pairs(const fe* values, uint64_t half, const uint8_t* tree,
                             uint32_t levels, const uint64_t* idx, uint32_t nq, uint8_t* out,
                             hipStream_t st) {
  if (nq == 0) return hipSuccess;
  hipLaunchKernelGGL(open_pairs_kernel, dim3(nq), dim3(64), 0, st, values, half, tree, levels,
                     idx, out);
  return hipGetLastError();
}

}  // namespace mlh

namespace mlh {

// level-0 of the cross-rank top tree: gathered[h][t] (P ranks x per-rank
// subtree roots) -> out[t * P + h], the global order of the level-log_s nodes.
__global__ void top_reorder_kernel(const uint8_t* __restrict__ gathered, uint32_t P,
                                   uint64_t per_rank, uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * per_rank) return;
  const uint64_t t = i / P, h = i % P;
  const uint4* src = reinterpret_cast<const uint4*>(gathered + (h * per_rank + t) * 32);
  uint4* dst = reinterpret_cast<uint4*>(out + i * 32);
  dst[0] = src[0];
  dst[1] = src[1];
}

hipError_t launch_top_reorder(const uint8_t* gathered, uint32_t P, uint64_t per_rank,
                              uint8_t* out, hipStream_t st) {
  const uint64_t n = P * per_rank;
  hipLaunchKernelGGL(top_reorder_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     gathered, P, per_rank, out);
  return hipGetLastError();
}

}  // namespace mlh
