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
hipError_t launch_merkle_levels(uint8_t* layers, uint64_t L, hipStream_t st);

// FRI fold (fri.hip).  tables: two-level powers of g^-1 (g of order n0).
hipError_t launch_fri_fold(const fe* layer, uint64_t n, fe* next, fe r, const fe* tlo_inv,
                           const fe* thi_inv, uint32_t k, uint64_t n0, hipStream_t st);
// Fold and hash the next layer's leaves (pairs (next[j], next[j + n/4])).
hipError_t launch_fri_fold_leaves(const fe* layer, uint64_t n, fe* next, uint8_t* leaves, fe r,
                                  const fe* tlo_inv, const fe* thi_inv, uint32_t k, uint64_t n0,
                                  hipStream_t st);

}  // namespace mlh
