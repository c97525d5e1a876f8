// Microbenchmark: VALU throughput of the integer primitives the F_M arithmetic
// is built from on gfx950 (v_mad_u64_u32, v_mul_lo/hi_u32, 24-bit muls, carry
// chains, f64 fma) and of the full field multiply.  Not product code: it
// decides the modmul design (DESIGN.md "Field arithmetic").
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../multilinear_amd/csrc/field.hpp"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;
constexpr int CH = 8;

__global__ void k_mad64(uint64_t* out, uint32_t b) {
  uint64_t acc[CH];
  for (int k = 0; k < CH; ++k) acc[k] = threadIdx.x * 7 + k;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = (uint64_t)(uint32_t)acc[k] * b + acc[k];
  uint64_t s = 0;
  for (int k = 0; k < CH; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mullo(uint64_t* out, uint32_t b) {
  uint32_t acc[CH];
  for (int k = 0; k < CH; ++k) acc[k] = threadIdx.x * 7 + k;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = acc[k] * b;
  uint32_t s = 0;
  for (int k = 0; k < CH; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mulhi(uint64_t* out, uint32_t b) {
  uint32_t acc[CH];
  for (int k = 0; k < CH; ++k) acc[k] = threadIdx.x * 7 + k;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = __umulhi(acc[k], b) | b;
  uint32_t s = 0;
  for (int k = 0; k < CH; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad24(uint64_t* out, uint32_t b) {
  uint32_t acc[CH];
  for (int k = 0; k < CH; ++k) acc[k] = threadIdx.x * 7 + k;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = __umul24(acc[k], b) + acc[k];
  uint32_t s = 0;
  for (int k = 0; k < CH; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add32(uint64_t* out, uint32_t b) {
  uint32_t acc[CH];
  for (int k = 0; k < CH; ++k) acc[k] = threadIdx.x * 7 + k;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = (acc[k] + b) ^ k;
  uint32_t s = 0;
  for (int k = 0; k < CH; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma64(uint64_t* out, uint32_t b) {
  double acc[CH];
  const double m = 1.0000001 + b * 1e-12, c = 1e-9;
  for (int k = 0; k < CH; ++k) acc[k] = threadIdx.x * 7 + k;
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = __fma_rn(acc[k], m, c);
  double s = 0;
  for (int k = 0; k < CH; ++k) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

constexpr int FITERS = 256;
__global__ void k_fmul(uint64_t* out, uint32_t b) {
  mlh::fe x[4], y;
  y = mlh::fe{{b, b * 3u, b * 5u, 0x7fffffffu}};
  for (int k = 0; k < 4; ++k) x[k] = mlh::fe{{threadIdx.x + k, blockIdx.x, 7u, 9u}};
  for (int it = 0; it < FITERS; ++it)
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = mlh::fe_mul(x[k], y);
  uint32_t s = 0;
  for (int k = 0; k < 4; ++k) s ^= x[k].w[0] ^ x[k].w[1] ^ x[k].w[2] ^ x[k].w[3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fadd(uint64_t* out, uint32_t b) {
  mlh::fe x[4], y;
  y = mlh::fe{{b, b * 3u, b * 5u, 0x7fffffffu}};
  for (int k = 0; k < 4; ++k) x[k] = mlh::fe{{threadIdx.x + k, blockIdx.x, 7u, 9u}};
  for (int it = 0; it < FITERS; ++it)
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = mlh::fe_add(x[k], y);
  uint32_t s = 0;
  for (int k = 0; k < 4; ++k) s ^= x[k].w[0] ^ x[k].w[1] ^ x[k].w[2] ^ x[k].w[3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t*, uint32_t);

int run(const char* name, kfn f, double ops_per_thread, uint64_t* d, int grid, int block) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(f, dim3(grid), dim3(block), 0, 0, d, 12345u);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(f, dim3(grid), dim3(block), 0, 0, d, 12345u + r);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double lane_ops = ops_per_thread * (double)grid * block;
  const double rate = lane_ops / (best * 1e-3);
  // 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz = 7.86e13 full-rate lane-ops/s
  printf("%-8s %8.3f ms  %.3e ops/s  = %.3f of full-rate VALU peak (7.86e13)\n", name, best, rate,
         rate / 7.864e13);
  return 0;
}

int main() {
  const int grid = 256 * 16, block = 256;
  uint64_t* d;
  CHECK(hipMalloc(&d, sizeof(uint64_t) * grid * block));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  run("mad64", k_mad64, (double)ITERS * CH, d, grid, block);
  run("mullo", k_mullo, (double)ITERS * CH, d, grid, block);
  run("mulhi+or", k_mulhi, (double)ITERS * CH * 2, d, grid, block);
  run("mad24", k_mad24, (double)ITERS * CH, d, grid, block);
  run("add+xor", k_add32, (double)ITERS * CH * 2, d, grid, block);
  run("fma64", k_fma64, (double)ITERS * CH, d, grid, block);
  run("fe_mul", k_fmul, (double)FITERS * 4, d, grid, block);
  run("fe_add", k_fadd, (double)FITERS * 4, d, grid, block);
  return 0;
}
