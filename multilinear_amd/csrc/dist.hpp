// Launchers for the sharded (one process per GPU) building blocks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.hpp"

namespace mlh {

// Cross-shard stage of the distributed NTT over P = 2^log_p ranks (dist.hip).
// in/out: [P][S] row-major.  Forward: out[t][jl] = sum_g wP^(g t) w^(g j) in[g][jl],
// j = j0 + jl.  Inverse: out[g][jl] = scale * w^(-g j) sum_t wP^(-g t) in[t][jl].
// tlo/thi: two-level powers of w (forward) or w^-1 (inverse); wp: wP^e (or wP^-e), e < P/2.
hipError_t launch_shard_dft(const fe* in, fe* out, uint64_t S, uint64_t j0, uint32_t log_p,
                            bool inverse, const fe* tlo, const fe* thi, const fe* wp, fe scale,
                            hipStream_t st);

// Open `nq` leaves of a (local) pair tree: record q = values[idx], values[idx + half],
// then the siblings of levels 0..levels-1 (tree = leaves-first flattened levels).
hipError_t launch_open_pairs(const fe* values, uint64_t half, const uint8_t* tree,
                             uint32_t levels, const uint64_t* idx, uint32_t nq, uint8_t* out,
                             hipStream_t st);

// gathered [P][per_rank] digests -> out [per_rank][P] (global node order)
hipError_t launch_top_reorder(const uint8_t* gathered, uint32_t P, uint64_t per_rank,
                              uint8_t* out, hipStream_t st);

}  // namespace mlh
