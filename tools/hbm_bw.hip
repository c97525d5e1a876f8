// Achievable HBM bandwidth on the box (dev tool): streaming read (xor-reduce)
// and copy of large buffers with 16-B lane accesses, grid-stride, HIP events.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void read_kernel(const uint4* __restrict__ a, uint64_t n, uint32_t* out) {
  uint32_t x = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint4 v = a[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) out[0] = x;  // keeps the loads
}

__global__ void copy_kernel(const uint4* __restrict__ a, uint4* __restrict__ b, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) b[i] = a[i];
}

int main() {
  const uint64_t bytes = 1ull << 30, n = bytes / 16;
  uint4 *a, *b;
  uint32_t* o;
  if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&o, 4)) return 1;
  hipMemset(a, 1, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (unsigned blocks : {1024u, 2048u, 4096u, 8192u, 16384u}) {
    float best_r = 1e9, best_c = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      float ms;
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(read_kernel, dim3(blocks), dim3(256), 0, 0, a, n, o);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best_r) best_r = ms;
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(copy_kernel, dim3(blocks), dim3(256), 0, 0, a, b, n / 2);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best_c) best_c = ms;
    }
    printf("blocks %5u: read 1 GiB %.3f ms = %.2f TB/s; copy 512 MiB %.3f ms = %.2f TB/s (R+W)\n",
           blocks, best_r, bytes / (best_r * 1e-3) / 1e12, best_c, bytes / (best_c * 1e-3) / 1e12);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
