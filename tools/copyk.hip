// Copy kernels for the all-to-all contention experiment (tools/a2a_contention.py):
// a CU-resident copy with a fixed number of workgroups, the way RCCL's
// all-to-all kernels occupy a few CUs per channel while they move data.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) copyk_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                    uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

extern "C" int copyk_launch(void* dst, const void* src, uint64_t bytes, int wgs, void* stream) {
  if (bytes % 16 || wgs <= 0) return 1;
  hipLaunchKernelGGL(copyk_kernel, dim3(wgs), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<uint4*>(dst), static_cast<const uint4*>(src), bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
