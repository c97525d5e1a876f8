// Practical VALU issue peak for the NTT's instruction mix (dev tool): radix-2
// butterflies with fe_mul_pre on register-resident values, no memory traffic
// in the loop.  Prints butterflies/s and (with the static VALU count of one
// iteration, from tools/kstat.py) lane-instructions/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../multilinear_amd/csrc/field.hpp"
using namespace mlh;

__global__ void __launch_bounds__(256) bfly_loop(const fe* __restrict__ in, const fe* __restrict__ tw,
                                                 fe* __restrict__ out, int iters) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  fe x[8];
  for (int e = 0; e < 8; ++e) x[e] = fe_load(in + ((g * 8 + e) & 4095));
  const fe* B = tw + 4 * (threadIdx.x & 7);
  const fe b0 = fe_load(B), b1 = fe_load(B + 1), b2 = fe_load(B + 2), b3 = fe_load(B + 3);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const fe v = fe_mul_pre_r(x[e + 1], b0, b1, b2, b3);
      const fe u = x[e];
      x[e] = fe_add(u, v);
      x[e + 1] = fe_sub(u, v);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {  // mix lanes of the register file
      const fe t = x[e];
      x[e] = x[e + 4];
      x[e + 4] = t;
    }
  }
  for (int e = 0; e < 8; ++e) fe_store(out + g * 8 + e, x[e]);
}

int main() {
  const int blocks = 256 * 8 * 4, threads = 256, iters = 256;
  fe *in, *tw, *out;
  hipMalloc(&in, 4096 * sizeof(fe));
  hipMalloc(&tw, 64 * sizeof(fe));
  hipMalloc(&out, (size_t)blocks * threads * 8 * sizeof(fe));
  hipMemset(in, 7, 4096 * sizeof(fe));
  hipMemset(tw, 3, 64 * sizeof(fe));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(bfly_loop, dim3(blocks), dim3(threads), 0, 0, in, tw, out, iters);
  hipEventRecord(a);
  hipLaunchKernelGGL(bfly_loop, dim3(blocks), dim3(threads), 0, 0, in, tw, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double bf = (double)blocks * threads * iters * 4;
  printf("butterflies/s %.3e  (%.3f ms)\n", bf / (ms * 1e-3), ms);
  return 0;
}
