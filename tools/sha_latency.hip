// SHA-256 node-hash latency microbenchmark (dev tool): each lane runs a chain
// of `iters` dependent sha256_node calls; reports us per hash per chain for a
// few launch shapes, and the shader clock from clock64 / wall_clock64.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../multilinear_amd/csrc/sha256.hpp"
using namespace mlh;

__global__ void chain_kernel(int iters, uint32_t* out, unsigned long long* clk) {
  Sha256State a = sha256_iv(), b = sha256_iv();
  a.h[0] ^= threadIdx.x + blockIdx.x * 977;
  const unsigned long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
    Sha256State c = sha256_node(a, b);
    b = a;
    a = c;
  }
  const unsigned long long c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = c1 - c0;
    clk[1] = w1 - w0;
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.h[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// three node hashes per iteration, unrolled (level2_kernel's code footprint)
__global__ void chain3_kernel(int iters, uint32_t* out) {
  Sha256State a = sha256_iv(), b = sha256_iv();
  a.h[0] ^= threadIdx.x + blockIdx.x * 977;
  for (int i = 0; i < iters; ++i) {
    Sha256State c = sha256_node(a, b);
    Sha256State d = sha256_node(b, a);
    a = sha256_node(c, d);
    b = c;
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.h[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// same work, one node-hash body in a rolled loop
__global__ void chain3r_kernel(int iters, uint32_t* out) {
  Sha256State a = sha256_iv(), b = sha256_iv();
  a.h[0] ^= threadIdx.x + blockIdx.x * 977;
  for (int i = 0; i < iters; ++i) {
    Sha256State c, d;
#pragma unroll 1
    for (int k = 0; k < 3; ++k) {
      const Sha256State x = k == 0 ? a : (k == 1 ? b : c);
      const Sha256State y = k == 0 ? b : (k == 1 ? a : d);
      const Sha256State r = sha256_node(x, y);
      if (k == 0) c = r; else if (k == 1) d = r; else { b = c; a = r; }
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.h[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
  uint32_t* out;
  unsigned long long* clk;
  hipMalloc(&out, 64 << 20);  // >= 8192 x 256 lanes x 4 B
  hipMalloc(&clk, 16);
  int wrate = 0;
  hipDeviceGetAttribute(&wrate, hipDeviceAttributeWallClockRate, 0);  // kHz
  const int shapes[][2] = {{1, 64}, {1, 256}, {1, 512}, {256, 64}, {256, 128}, {256, 256},
                           {256, 512}, {1024, 256}, {2048, 256}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 200;
  for (auto& s : shapes) {
    hipLaunchKernelGGL(chain_kernel, dim3(s[0]), dim3(s[1]), 0, 0, 10, out, clk);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(chain_kernel, dim3(s[0]), dim3(s[1]), 0, 0, iters, out, clk);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[2];
    hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    const double wall_us = (double)h[1] / (wrate * 1e-3);
    printf("grid %5d x %4d: %.3f us/hash (event), %.0f cycles/hash, shader clock %.0f MHz, "
           "%.3e hashes/s\n",
           s[0], s[1], ms * 1e3 / iters, (double)h[0] / iters, h[0] / wall_us,
           (double)s[0] * s[1] * iters / (ms * 1e-3));
  }
  for (int v = 0; v < 2; ++v) {
    for (int grid : {256, 2048, 8192}) {
      auto k = v ? chain3r_kernel : chain3_kernel;
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, 2, out);
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, 40, out);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s grid %5d x 256: %.3e hashes/s\n", v ? "rolled  " : "unrolled", grid,
             3.0 * grid * 256 * 40 / (ms * 1e-3));
    }
  }
  return 0;
}
