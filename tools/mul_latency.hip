// Single-lane latency of the field primitives (one wave, one active lane, a
// dependent chain), timed with wall_clock64 inside the kernel: what the
// latency-bound sumcheck round / tail kernels pay per fe_mul / fe_add.
// Dev tool:  hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/mul_latency.hip -o tools/mul_latency
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../multilinear_amd/csrc/field.hpp"

using namespace mlh;
constexpr int kIters = 2000;

template <int OP>
__global__ void chain(fe* io, uint64_t* ticks) {
  if (threadIdx.x != 0) return;
  fe x = io[0];
  const fe y = io[1];
  const uint64_t t0 = wall_clock64();
  for (int i = 0; i < kIters; ++i) {
    if (OP == 0) x = fe_mul(x, y);
    if (OP == 1) x = fe_add(x, y);
    if (OP == 2) x = fe_sub(x, y);
  }
  const uint64_t t1 = wall_clock64();
  io[2] = x;
  ticks[0] = t1 - t0;
}

int main() {
  fe h[3] = {fe{{1u, 2u, 3u, 4u}}, fe{{0x12345678u, 0x9abcdef0u, 0x0fedcba9u, 0x7654321u}}, fe{}};
  fe* io;
  uint64_t* tk;
  hipMalloc(&io, sizeof h);
  hipMalloc(&tk, 8);
  hipMemcpy(io, h, sizeof h, hipMemcpyHostToDevice);
  int khz = 0;
  hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  const char* names[3] = {"fe_mul", "fe_add", "fe_sub"};
  for (int op = 0; op < 3; ++op) {
    for (int rep = 0; rep < 3; ++rep) {
      if (op == 0) hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, io, tk);
      if (op == 1) hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, io, tk);
      if (op == 2) hipLaunchKernelGGL(chain<2>, dim3(1), dim3(64), 0, 0, io, tk);
      hipDeviceSynchronize();
    }
    uint64_t t = 0;
    hipMemcpy(&t, tk, 8, hipMemcpyDeviceToHost);
    printf("%-7s %.1f ns per dependent op (one lane)\n", names[op], t * 1e6 / khz / kIters);
  }
  return 0;
}
