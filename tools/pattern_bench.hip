// Memory-pattern microbenchmark (dev tool): time pure load/store kernels that
// use the NTT pass access patterns, to separate HBM-pattern cost from VALU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void copy_contig(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) out[i] = in[i];
}

// tile = COLS adjacent columns x R rows (row stride W); thread holds EPT rows of one column
template <int COLS, int R, int EPT>
__global__ void __launch_bounds__(COLS * R / EPT) copy_tile(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t W, int bitrev_rows) {
  const int tid = threadIdx.x;
  const int c = tid % COLS, t = tid / COLS;
  const uint64_t lowcount = W / COLS;
  const uint64_t tile = blockIdx.x;
  const uint64_t hi = tile / lowcount, lo = tile % lowcount;
  const uint64_t base = hi * (uint64_t)R * W + lo * COLS + c;
  uint4 x[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    uint32_t row = t * EPT + e;
    if (bitrev_rows) row = __builtin_bitreverse32(row) >> (32 - __builtin_ctz(R));
    x[e] = in[base + (uint64_t)row * W];
  }
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    // store rows t + e*R/EPT (like the phase-3 layout)
    const uint32_t row = t + e * (R / EPT);
    out[base + (uint64_t)row * W] = x[e];
  }
}

template <int COLS, int R, int EPT>
static float run_tile(const uint4* in, uint4* out, uint64_t N, uint64_t W, int br) {
  const uint64_t tiles = N / ((uint64_t)COLS * R);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((copy_tile<COLS, R, EPT>), dim3(tiles), dim3(COLS * R / EPT), 0, 0, in, out, W, br);
  hipEventRecord(a);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((copy_tile<COLS, R, EPT>), dim3(tiles), dim3(COLS * R / EPT), 0, 0, in, out, W, br);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const uint64_t N = 1ull << 24;
  uint4 *in, *out;
  CK(hipMalloc(&in, N * 16)); CK(hipMalloc(&out, N * 16));
  CK(hipMemset(in, 1, N * 16));
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(copy_contig, dim3(4096), dim3(256), 0, 0, in, out, N);
  hipEventRecord(a);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(copy_contig, dim3(4096), dim3(256), 0, 0, in, out, N);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= 20;
  printf("contig copy 2^24 x16B: %.4f ms  %.0f GB/s\n", ms, 32.0 * N / ms / 1e6);
  const uint64_t Ws[] = {1ull << 16, 1ull << 8, 8, 16, 32, 64};
  for (uint64_t W : Ws) {
    for (int br = 0; br < 2; ++br) {
      float t8 = run_tile<8, 256, 8>(in, out, N, W, br);
      float t16 = W >= 16 ? run_tile<16, 128, 8>(in, out, N, W, br) : 0;
      float t32 = W >= 32 ? run_tile<32, 64, 8>(in, out, N, W, br) : 0;
      printf("W=2^%2d bitrev=%d  cols8xR256: %.4f ms (%.0f GB/s)  cols16xR128: %.4f  cols32xR64: %.4f\n",
             __builtin_ctzll(W), br, t8, 32.0 * N / t8 / 1e6, t16, t32);
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
