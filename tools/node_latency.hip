// Tree-tail node-hash latency on ONE wave (dev tool): cycles per dependent
// SHA-256 node hash, one-lane (sha256_node) vs lane pair (sha2l_node), and the
// lane pair with two independent chains interleaved (does ILP hide the
// dependent-issue latency?).  s_memtime cycles and wall_clock64 per launch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../multilinear_amd/csrc/sha256.hpp"
#include "../multilinear_amd/csrc/transcript_dev.hpp"
using namespace mlh;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int MODE>
__global__ void __launch_bounds__(64) chain(int iters, uint32_t* out, unsigned long long* clk) {
  const uint32_t id = MODE == 0 ? threadIdx.x : threadIdx.x >> 1;  // lane pairs share data
  Sha256State a = sha256_iv(), b = sha256_iv(), a2 = sha256_iv(), b2 = sha256_iv();
  a.h[0] ^= id * 977 + 1;
  a2.h[1] ^= id * 131 + 7;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), w0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {
      const Sha256State c = sha256_node(a, b);
      b = a;
      a = c;
    } else if (MODE == 1) {
      const Sha256State c = sha2l_node(a, b);
      b = a;
      a = c;
    } else {
      const Sha256State c = sha2l_node(a, b);
      const Sha256State c2 = sha2l_node(a2, b2);
      b = a;
      a = c;
      b2 = a2;
      a2 = c2;
    }
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), w1 = wall_clock64();
  if (threadIdx.x == 0) {
    clk[0] = c1 - c0;
    clk[1] = w1 - w0;
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= a.h[i] ^ a2.h[i];
  out[threadIdx.x] = x;
}

template <int MODE>
int run(const char* name, int iters, uint32_t* d, unsigned long long* clk) {
  hipLaunchKernelGGL(chain<MODE>, dim3(1), dim3(64), 0, 0, iters, d, clk);
  CHECK(hipDeviceSynchronize());
  unsigned long long best_c = ~0ull, best_w = ~0ull;
  for (int r = 0; r < 5; ++r) {
    hipLaunchKernelGGL(chain<MODE>, dim3(1), dim3(64), 0, 0, iters, d, clk);
    CHECK(hipDeviceSynchronize());
    unsigned long long h[2];
    CHECK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
    if (h[0] < best_c) best_c = h[0];
    if (h[1] < best_w) best_w = h[1];
  }
  // wall_clock64 ticks at 100 MHz on gfx950
  printf("{\"chain\": \"%s\", \"cycles_per_node\": %.0f, \"us_per_node\": %.3f}\n", name,
         (double)best_c / iters, (double)best_w / iters / 100.0);
  return 0;
}

int main() {
  uint32_t* d;
  unsigned long long* clk;
  CHECK(hipMalloc(&d, 4096));
  CHECK(hipMalloc(&clk, 64));
  const int it = 256;
  run<0>("one-lane sha256_node", it, d, clk);
  run<1>("lane-pair sha2l_node", it, d, clk);
  run<2>("lane-pair, two chains interleaved (per node of one chain)", it, d, clk);
  return 0;
}
