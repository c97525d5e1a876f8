// One-wave VALU issue vs dependent-issue cost on gfx950 (dev tool): cycles per
// instruction of 1, 2, 4 interleaved dependent chains of v_xor / v_alignbit /
// v_bitop3 / v_add3 / v_mad_u64_u32, timed with s_memtime around 256 instrs.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/dep_latency.hip -o tools/dep_latency
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define R4(x) x x x x
#define R16(x) R4(R4(x))
#define R64(x) R4(R16(x))
#define R2X "v_xor_b32 %0, %0, %4\nv_xor_b32 %1, %1, %4\nv_xor_b32 %0, %0, %4\nv_xor_b32 %1, %1, %4\n"

template <int K>
__global__ void k(uint64_t* out, uint32_t seed) {
  uint32_t a = seed, b = seed * 3, c = seed * 5, d = seed * 7, e = seed ^ 0x55;
  uint64_t t0 = 0, t1 = 0;
  for (int pass = 0; pass < 2; ++pass) {  // the second pass runs from a warm instruction cache
  t0 = __builtin_amdgcn_s_memtime();
  if (K == 0) asm volatile(R64(R4("v_xor_b32 %0, %0, %4\n")) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e));
  if (K == 1) asm volatile(R64(R2X) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e));
  if (K == 2) asm volatile(R64("v_xor_b32 %0, %0, %4\nv_xor_b32 %1, %1, %4\nv_xor_b32 %2, %2, %4\nv_xor_b32 %3, %3, %4\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e));
  if (K == 3) asm volatile(R64(R4("v_alignbit_b32 %0, %0, %0, 7\n")) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e));
  if (K == 4) asm volatile(R64("v_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e));
  if (K == 5) asm volatile(R64(R4("v_add3_u32 %0, %0, %4, %4\n")) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e));
  if (K == 6) asm volatile(R64("v_add3_u32 %0, %0, %4, %4\nv_add3_u32 %1, %1, %4, %4\nv_add3_u32 %2, %2, %4, %4\nv_add3_u32 %3, %3, %4, %4\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e));
  if (K == 7) asm volatile(R64(R4("v_bitop3_b32 %0, %0, %4, %4 bitop3:0x96\n")) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e));
  if (K == 8) asm volatile(R64("v_bitop3_b32 %0, %0, %4, %4 bitop3:0x96\nv_bitop3_b32 %1, %1, %4, %4 bitop3:0x96\nv_bitop3_b32 %2, %2, %4, %4 bitop3:0x96\nv_bitop3_b32 %3, %3, %4, %4 bitop3:0x96\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e));
  if (K == 9) asm volatile(R64("v_add_u32_e32 %0, 0x428a2f98, %0\nv_add_u32_e32 %1, 0x428a2f98, %1\nv_add_u32_e32 %2, 0x428a2f98, %2\nv_add_u32_e32 %3, 0x428a2f98, %3\n") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e));
  if (K == 10) {
    uint32_t s0 = seed, s1 = seed * 9;
    asm volatile(R64("v_xor_b32 %0, %0, %6\ns_xor_b32 %4, %4, %5\nv_xor_b32 %1, %1, %6\ns_xor_b32 %5, %5, %4\n")
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "+s"(s1) : "v"(e));
    a += s0 + s1;
  }
  if (K == 11) {
    uint32_t s0 = seed, s1 = seed * 9;
    asm volatile(R64("s_xor_b32 %4, %4, %5\ns_xor_b32 %5, %5, %4\ns_xor_b32 %4, %4, %5\ns_xor_b32 %5, %5, %4\n")
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "+s"(s1) : "v"(e));
    a += s0 + s1;
  }
  if (K == 12) {
    uint32_t s0 = seed, s1 = seed * 9, s2 = seed * 11, s3 = seed * 13;
    asm volatile(R64("s_xor_b32 %4, %4, %8\ns_xor_b32 %5, %5, %8\ns_xor_b32 %6, %6, %8\ns_xor_b32 %7, %7, %8\n")
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3) : "s"(e));
    a += s0 + s1 + s2 + s3;
  }
  if (K == 13) {  // VALU reading an SGPR written by the SALU just before
    uint32_t s0 = seed, s1 = seed * 9;
    asm volatile(R64("s_xor_b32 %4, %4, %5\nv_xor_b32 %0, %0, %4\ns_xor_b32 %5, %5, %4\nv_xor_b32 %1, %1, %5\n")
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "+s"(s1) : "v"(e));
    a += s0 + s1;
  }
  t1 = __builtin_amdgcn_s_memtime();
  }
  if (threadIdx.x == 0) out[K] = t1 - t0;
  if (a + b + c + d == 12345) out[15] = 1;
}

int main() {
  uint64_t* d;
  hipMalloc(&d, 16 * 8);
  const char* names[14] = {"xor 1 chain", "xor 2 chains", "xor 4 chains", "alignbit 1 chain",
                           "alignbit 4 chains", "add3 1 chain", "add3 4 chains", "bitop3 1 chain",
                           "bitop3 4 chains", "add_lit 4 chains", "v/s xor interleaved", "s_xor chain",
                           "s_xor 4 indep", "s->v dependent mix"};
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k<0>, 1, 64, 0, 0, d, 1); hipLaunchKernelGGL(k<1>, 1, 64, 0, 0, d, 1);
    hipLaunchKernelGGL(k<2>, 1, 64, 0, 0, d, 1); hipLaunchKernelGGL(k<3>, 1, 64, 0, 0, d, 1);
    hipLaunchKernelGGL(k<4>, 1, 64, 0, 0, d, 1); hipLaunchKernelGGL(k<5>, 1, 64, 0, 0, d, 1);
    hipLaunchKernelGGL(k<6>, 1, 64, 0, 0, d, 1); hipLaunchKernelGGL(k<7>, 1, 64, 0, 0, d, 1);
    hipLaunchKernelGGL(k<8>, 1, 64, 0, 0, d, 1); hipLaunchKernelGGL(k<9>, 1, 64, 0, 0, d, 1);
    hipLaunchKernelGGL(k<10>, 1, 64, 0, 0, d, 1); hipLaunchKernelGGL(k<11>, 1, 64, 0, 0, d, 1);
    hipLaunchKernelGGL(k<12>, 1, 64, 0, 0, d, 1); hipLaunchKernelGGL(k<13>, 1, 64, 0, 0, d, 1);
    hipDeviceSynchronize();
  }
  uint64_t h[16];
  hipMemcpy(h, d, 16 * 8, hipMemcpyDeviceToHost);
  for (int i = 0; i < 14; ++i) printf("%-18s %.2f cycles/instr\n", names[i], h[i] / 256.0);
  return 0;
}
