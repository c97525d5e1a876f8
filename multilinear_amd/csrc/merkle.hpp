// Merkle launch interface (internal to libmlhip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.hpp"

namespace mlh {

hipError_t launch_leaf_pairs(const fe* code, uint64_t half, uint8_t* leaves, hipStream_t st);
hipError_t launch_leaf_bytes(const uint8_t* items, uint64_t item_len, uint64_t count,
                             uint8_t* leaves, hipStream_t st);
hipError_t launch_leaf_batch(const uint8_t* items, uint64_t item_len, uint64_t batch_stride,
                             uint32_t m, uint64_t count, uint8_t* leaves, hipStream_t st);
struct DevSha;
// Optional Fiat-Shamir step fused into the launch that writes a tree's root:
// absorb the 32 root bytes into the device transcript t, copy them to
// copy_out, and write next_challenge() to r_out (each pointer optional; t
// null = no transcript step).  Same effect as launch_transcript_absorb(t,
// root, 32, r_out, st, copy_out) after the tree, without its launch.
// poly_in (optional): 32 more bytes absorbed after the root and before the
// challenge -- a PCS round's LE16(c1) || LE16(c2) (multilinear_pcs.rs:57-75).
struct RootAbsorb {
  DevSha* t = nullptr;
  fe* r_out = nullptr;
  uint8_t* copy_out = nullptr;
  const fe* poly_in = nullptr;
};
hipError_t launch_merkle_levels(uint8_t* layers, uint64_t L, hipStream_t st,
                                RootAbsorb ra = RootAbsorb());
// the levels above the level of n digests stored at layers + off digests
hipError_t launch_merkle_levels_from(uint8_t* layers, uint64_t off, uint64_t n, hipStream_t st,
                                     RootAbsorb ra = RootAbsorb());
// sibling paths (depth = log2 L digests, bottom-up) of leaves idx[0..nq) (device array)
hipError_t launch_merkle_paths(const uint8_t* layers, uint64_t L, const uint64_t* idx, uint32_t nq,
                               uint8_t* out, hipStream_t st);
// commit_rs_code tree of the L = n/2 pairs (code[i], code[i + L]): leaves and
// every level up to the root into layers (2L-1 digests, level order).
hipError_t launch_commit_pairs(const fe* code, uint64_t L, uint8_t* layers, hipStream_t st,
                               RootAbsorb ra = RootAbsorb());

// Block-cyclic shard layout of a layer spread over 2^log_p ranks: local
// index l of rank `rank` holds global index
//   ((l >> log_s) << (log_s + log_p)) | (rank << log_s) | (l & (2^log_s - 1))
// (blocks of 2^log_s consecutive elements dealt round-robin to the ranks).
// log_p = 0, log_s >= 40 is the identity (single GPU).
struct ShardMap {
  uint32_t log_s = 40;
  uint32_t log_p = 0;
  uint64_t rank = 0;
  __host__ __device__ uint64_t global(uint64_t l) const {
    return ((l >> log_s) << (log_s + log_p)) | (rank << log_s) | (l & ((1ull << log_s) - 1));
  }
};

// FRI fold (fri.hip).  tables: two-level powers of g^-1 (g of order n0).
// r_dev (optional): read the challenge from device memory instead of r.
// n is the LOCAL layer length; the twiddle exponent uses map.global(i).
hipError_t launch_fri_fold(const fe* layer, uint64_t n, fe* next, fe r, const fe* tlo_inv,
                           const fe* thi_inv, uint32_t k, uint64_t n0, hipStream_t st,
                           ShardMap map = ShardMap(), const fe* r_dev = nullptr);
// Fold and hash the next layer's leaves (pairs (next[j], next[j + n/4])).
struct PcsJob;
// job (optional): one PCS round (sumcheck.hpp PcsJob) run by an extra
// workgroup of the same launch
// twl (optional): this layer's twiddles, twl[j] = g^(-j 2^k) for its n/2 pairs
// (fold_layer_table: every layer of a domain in one table), instead of the
// product T_lo[e & 4095] * T_hi[e >> 12] per pair
hipError_t launch_fri_fold_leaves(const fe* layer, uint64_t n, fe* next, uint8_t* leaves, fe r,
                                  const fe* tlo_inv, const fe* thi_inv, uint32_t k, uint64_t n0,
                                  hipStream_t st, ShardMap map = ShardMap(),
                                  const fe* r_dev = nullptr, const PcsJob* job = nullptr,
                                  const fe* twl = nullptr);
// Fold and commit the next layer: its whole tree (L = n/4 leaves, 2L-1
// digests) into `tree` (leaves hashed by the fold lanes).
hipError_t launch_fri_fold_commit(const fe* layer, uint64_t n, fe* next, uint8_t* tree, fe r,
                                  const fe* tlo_inv, const fe* thi_inv, uint32_t k, uint64_t n0,
                                  hipStream_t st, ShardMap map = ShardMap(),
                                  const fe* r_dev = nullptr, RootAbsorb ra = RootAbsorb(),
                                  const PcsJob* job = nullptr, const fe* twl = nullptr);
// All layers' twiddles of a domain of 2^L (L >= 2) in one table of 2^L - 1
// entries: layer k (2^(L-1-k) pairs) at offset 2^L - 2^(L-k), entry j =
// g^(-j 2^k) = T_lo[e & 4095] * T_hi[e >> 12], e = j 2^k.
hipError_t launch_fold_layer_table(fe* out, const fe* tlo_inv, const fe* thi_inv, uint32_t L,
                                   hipStream_t st);

}  // namespace mlh
