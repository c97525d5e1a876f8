#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.hpp"

namespace mlh {
// op: 0 add, 1 sub, 2 mul, 3 neg (b unused)
// op: 0 add, 1 sub, 2 mul, 3 neg, 4 scale by c
hipError_t launch_vec_op(int op, const fe* a, const fe* b, fe* out, uint64_t n, hipStream_t st,
                         fe c = fe{});
}  // namespace mlh
