// Probe of the stream wait-value path (dev tool): attribute, signal memory,
// memset, a wait released by a kernel's store.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
__global__ void setk(uint32_t* p, uint32_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void spin(volatile uint32_t* p) {
  for (int i = 0; i < 100000 && *p == 0; ++i) __builtin_amdgcn_s_sleep(8);
}
int main() {
  int can = -1;
  hipError_t e = hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0);
  printf("attr %d can %d\n", (int)e, can);
  void* p = nullptr;
  e = hipExtMallocWithFlags(&p, 64, hipMallocSignalMemory);
  printf("signal malloc %d %s ptr %p\n", (int)e, hipGetErrorString(e), p);
  if (!p) { e = hipMalloc(&p, 64); printf("plain malloc %d\n", (int)e); }
  e = hipMemset(p, 0, 64);
  printf("memset %d %s\n", (int)e, hipGetErrorString(e));
  hipStream_t a, b;
  hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
  uint32_t* q = nullptr;
  hipMalloc(&q, 4);
  hipMemset(q, 0, 4);
  e = hipStreamWaitValue32(b, p, 7, hipStreamWaitValueEq, 0xFFFFFFFFu);
  printf("waitvalue %d %s\n", (int)e, hipGetErrorString(e));
  hipLaunchKernelGGL(setk, dim3(1), dim3(64), 0, b, q, 1u);  // runs after the wait
  hipLaunchKernelGGL(setk, dim3(1), dim3(64), 0, a, (uint32_t*)p, 7u);
  e = hipStreamSynchronize(b);
  uint32_t h = 0;
  hipMemcpy(&h, q, 4, hipMemcpyDeviceToHost);
  printf("sync b %d, after-wait kernel ran: %u\n", (int)e, h);
  return 0;
}
