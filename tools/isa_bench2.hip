// Microbenchmark of the 32-bit ops SHA-256 uses on gfx950 (not product code).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s\n", hipGetErrorString(e)); return 1; } } while (0)
constexpr int IT = 2048, CH = 8;
#define KERNEL(NAME, EXPR) \
__global__ void NAME(uint32_t* out, uint32_t b) { \
  uint32_t a[CH]; for (int k = 0; k < CH; ++k) a[k] = threadIdx.x * 7 + k + blockIdx.x; \
  uint32_t c = b * 3 + 1; \
  for (int it = 0; it < IT; ++it) { _Pragma("unroll") for (int k = 0; k < CH; ++k) { uint32_t x = a[k]; a[k] = EXPR; } \
    asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])); } \
  uint32_t s = 0; for (int k = 0; k < CH; ++k) s ^= a[k]; out[blockIdx.x * blockDim.x + threadIdx.x] = s; }
KERNEL(k_alignbit, __builtin_amdgcn_alignbit(x, x, 7))
KERNEL(k_xor, x ^ c)
KERNEL(k_add3, x + c + b)
KERNEL(k_xor3, x ^ c ^ b)
KERNEL(k_shr, x >> 7)
KERNEL(k_rot2, (x >> 7) | (x << 25))
KERNEL(k_bfi, (x & c) ^ (~x & b))
KERNEL(k_perm, __builtin_bswap32(x))
typedef void (*kfn)(uint32_t*, uint32_t);
int run(const char* n, kfn f, uint32_t* d) {
  const int grid = 256 * 16, block = 256;
  hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(f, dim3(grid), dim3(block), 0, 0, d, 5u); CHECK(hipDeviceSynchronize());
  float best = 1e9;
  for (int r = 0; r < 5; ++r) { CHECK(hipEventRecord(a)); hipLaunchKernelGGL(f, dim3(grid), dim3(block), 0, 0, d, 5u + r);
    CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); float ms; CHECK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms; }
  double ops = (double)IT * CH * grid * block;
  printf("%-10s %.3f ms  %.3e expr/s = %.3f of 7.86e13\n", n, best, ops / (best * 1e-3), ops / (best * 1e-3) / 7.864e13);
  return 0;
}
int main() { uint32_t* d; CHECK(hipMalloc(&d, 4 * 256 * 16 * 256));
  run("alignbit", k_alignbit, d); run("xor", k_xor, d); run("add3", k_add3, d); run("xor3", k_xor3, d);
  run("shr", k_shr, d); run("rot2", k_rot2, d); run("bfi", k_bfi, d); run("perm", k_perm, d); return 0; }
