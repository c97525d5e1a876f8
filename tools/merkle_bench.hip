// Merkle level-kernel throughput on a 2^log_l-leaf tree (dev tool): times
// launch_merkle_levels and each level2 launch with HIP events.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../multilinear_amd/csrc/merkle.hip"
using namespace mlh;

int main(int argc, char** argv) {
  const int log_l = argc > 1 ? atoi(argv[1]) : 24;
  const uint64_t L = 1ull << log_l;
  uint8_t* layers;
  if (hipMalloc(&layers, (2 * L - 1) * 32) != hipSuccess) return 1;
  hipMemset(layers, 0x5a, L * 32);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(e0, 0);
    launch_merkle_levels(layers, L, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("levels of 2^%d leaves: %.3f ms, %.3e node hashes/s\n", log_l, ms, (L - 1) / (ms * 1e-3));
  }
  // first level2 launch alone
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(level2_kernel, dim3((unsigned)(L / 4 / 256)), dim3(256), 0, 0, layers,
                       layers + L * 32, layers + (L + L / 2) * 32, L / 4);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("level2 (2^%d -> 2^%d): %.3f ms, %.3e hashes/s\n", log_l, log_l - 2, ms,
           (L / 2 + L / 4) / (ms * 1e-3));
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
