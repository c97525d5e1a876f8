// Dev probe: does straight-line VALU code slow down when the waves of one
// workgroup run more distinct code than the instruction cache holds?  Each of
// the 4 waves runs its own copy (template instance) of an unrolled SHA-like
// round chain, `reps` times; the per-wave shader-clock count over the loop is
// printed per instruction, for 1, 2 and 4 active waves and several copy sizes.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/icache_probe.hip -o tools/icache_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <stdint.h>

template <int S, int N>
__device__ __noinline__ uint32_t body(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    uint32_t t = __builtin_amdgcn_alignbit(a, a, 6) ^ __builtin_amdgcn_alignbit(a, a, 11) ^
                 __builtin_amdgcn_alignbit(a, a, 25);
    uint32_t ch = (a & b) ^ (~a & c);
    uint32_t n = d + t + ch + (uint32_t)(S * 7919 + i * 104729 + 12345);
    d = c;
    c = b;
    b = a;
    a = n;
  }
  return a ^ b ^ c ^ d;
}

template <int N>
__global__ void __launch_bounds__(256) probe(uint32_t* out, long long* cyc, int reps, int active) {
  const int w = threadIdx.x >> 6;
  uint32_t a = threadIdx.x, b = 1, c = 2, d = 3;
  if (!((active >> w) & 1)) return;
  __builtin_amdgcn_s_waitcnt(0);
  const long long t0 = clock64();
  for (int r = 0; r < reps; ++r) {
    switch (w) {
      case 0: a = body<0, N>(a, b, c, d); break;
      case 1: a = body<1, N>(a, b, c, d); break;
      case 2: a = body<2, N>(a, b, c, d); break;
      default: a = body<3, N>(a, b, c, d); break;
    }
    b += r;
  }
  const long long t1 = clock64();
  out[threadIdx.x] = a;
  if ((threadIdx.x & 63) == 0) cyc[w] = t1 - t0;
}

template <int N>
static void run(uint32_t* dout, long long* dcyc, int reps) {
  const int masks[4] = {1, 3, 15, 5};
  for (int m : masks) {
    long long h[4] = {0, 0, 0, 0};
    hipMemset(dcyc, 0, sizeof h);
    // warm (first touch of the code), then timed
    hipLaunchKernelGGL(probe<N>, dim3(1), dim3(256), 0, 0, dout, dcyc, 1, m);
    hipLaunchKernelGGL(probe<N>, dim3(1), dim3(256), 0, 0, dout, dcyc, reps, m);
    if (hipMemcpy(h, dcyc, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) {
      printf("HIP error\n");
      return;
    }
    // 8 VALU + 1 SALU, 64 bytes of code per unrolled step
    printf("N=%4d (~%5.1f KB/copy) waves=0x%x  cycles/step:", N, N * 64 / 1024.0, m);
    for (int w = 0; w < 4; ++w)
      if ((m >> w) & 1) printf(" w%d %.2f", w, (double)h[w] / reps / N);
    printf("\n");
  }
}

int main() {
  uint32_t* dout;
  long long* dcyc;
  hipMalloc(&dout, 256 * 4);
  hipMalloc(&dcyc, 4 * sizeof(long long));
  run<64>(dout, dcyc, 400);
  run<256>(dout, dcyc, 100);
  run<512>(dout, dcyc, 50);
  run<1024>(dout, dcyc, 25);
  return 0;
}
