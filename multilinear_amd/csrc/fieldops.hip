// Elementwise Field128 ops on device vectors (src/field.rs:66-136: Add, Sub,
// Mul, Neg of winter-math f128 BaseElement), streaming dwordx4 per lane.
#include "field.hpp"
#include "fieldops.hpp"

namespace mlh {

template <int OP>
__global__ void __launch_bounds__(256)
vec_op_kernel(const fe* a, const fe* b, fe* out, uint64_t n, fe c) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const fe x = fe_load(a + i);
    fe r;
    if (OP == 0) r = fe_add(x, fe_load(b + i));
    if (OP == 1) r = fe_sub(x, fe_load(b + i));
    if (OP == 2) r = fe_mul(x, fe_load(b + i));
    if (OP == 3) r = fe_neg(x);
    if (OP == 4) r = fe_mul(x, c);
    fe_store(out + i, r);
  }
}

hipError_t launch_vec_op(int op, const fe* a, const fe* b, fe* out, uint64_t n, hipStream_t st,
                         fe c) {
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) return hipSuccess;
  switch (op) {
    case 0: hipLaunchKernelGGL(vec_op_kernel<0>, dim3((unsigned)blocks), dim3(256), 0, st, a, b, out, n, c); break;
    case 1: hipLaunchKernelGGL(vec_op_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, st, a, b, out, n, c); break;
    case 2: hipLaunchKernelGGL(vec_op_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, st, a, b, out, n, c); break;
    case 3: hipLaunchKernelGGL(vec_op_kernel<3>, dim3((unsigned)blocks), dim3(256), 0, st, a, b, out, n, c); break;
    case 4: hipLaunchKernelGGL(vec_op_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, st, a, b, out, n, c); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace mlh
