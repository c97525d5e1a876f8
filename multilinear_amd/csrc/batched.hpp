// Batched FRI / PCS launchers (batched.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.hpp"

namespace mlh {

// A query phase's indices, passed by value in the kernel arguments (no
// host-to-device copy on the proof's critical path).
struct QueryIdx {
  uint64_t v[128];  // MLH_NUM_QUERIES
};

hipError_t launch_batch_pairs_leaves(const fe* codes, uint32_t m, uint64_t N, uint8_t* leaves,
                                     hipStream_t st);
// fr, r: device pointers; leaves may be null (final fold to two values)
hipError_t launch_batched_fold_leaves(const fe* codes, uint32_t m, uint64_t N, const fe* fr,
                                      const fe* r, const fe* tlo, const fe* thi, fe* next,
                                      uint8_t* leaves, hipStream_t st);
hipError_t launch_fingerprint(const fe* polys, uint32_t m, uint64_t n, const fe* fr, fe* out,
                              hipStream_t st);
hipError_t launch_fingerprint_scalar(const fe* vals, uint32_t m, const fe* fr, fe* out,
                                     hipStream_t st);
hipError_t launch_batch_queries(const fe* codes, uint32_t m, uint64_t N, const uint8_t* tree,
                                const QueryIdx& idx, uint32_t nq, uint64_t qbytes, uint8_t* out,
                                hipStream_t st);

}  // namespace mlh
