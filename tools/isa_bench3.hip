// Microbenchmark (dev tool, not product code): issue rate of the single
// integer VALU instructions the field / SHA-256 code is made of, many waves
// per SIMD, 8 independent chains per lane.  Evidence for the VALU ceiling
// bench.py divides by (one wave64 VOP3 integer instruction per 4 cycles per
// SIMD) -- and for which encodings issue faster than that.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;
constexpr int CH = 8;

#define KERNEL(NAME, BODY)                                                     \
  __global__ void NAME(uint32_t* out, uint32_t b) {                           \
    uint32_t acc[CH];                                                          \
    for (int k = 0; k < CH; ++k) acc[k] = threadIdx.x * 7 + k;                 \
    for (int it = 0; it < ITERS; ++it) {                                       \
      _Pragma("unroll") for (int k = 0; k < CH; ++k) { uint32_t x = acc[k]; BODY; acc[k] = x; } \
    }                                                                          \
    uint32_t s = 0;                                                            \
    for (int k = 0; k < CH; ++k) s ^= acc[k];                                  \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                            \
  }

// one instruction per chain step each (checked in the ISA: tools/isa_bench3.s)
KERNEL(k_add_vop2, asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(x) : "v"(b)))
KERNEL(k_xor_vop2, asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(x) : "v"(b)))
KERNEL(k_add3_vop3, asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(b)))
KERNEL(k_alignbit, asm volatile("v_alignbit_b32 %0, %0, %0, %1" : "+v"(x) : "v"(b)))
KERNEL(k_bitop3, asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(x) : "v"(b)))
KERNEL(k_addco, asm volatile("v_add_co_u32_e32 %0, vcc, %1, %0" : "+v"(x) : "v"(b) : "vcc"))
KERNEL(k_mad64, { uint64_t y; asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, 0" : "=v"(y) : "v"(x), "v"(b) : "s0", "s1"); x = (uint32_t)y ^ (uint32_t)(y >> 32); })
KERNEL(k_mullo, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b)))
KERNEL(k_mulhi, asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b)))
KERNEL(k_cndmask, asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[2:3]" : "+v"(x) : "v"(b) : "s2", "s3"))

typedef void (*kfn)(uint32_t*, uint32_t);

static double run(const char* name, kfn f, double instr_per_step, uint32_t* d, int grid, int block) {
  hipEvent_t a, e;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&e);
  hipLaunchKernelGGL(f, dim3(grid), dim3(block), 0, 0, d, 12345u);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(f, dim3(grid), dim3(block), 0, 0, d, 12345u + r);
    (void)hipEventRecord(e);
    (void)hipEventSynchronize(e);
    float ms;
    (void)hipEventElapsedTime(&ms, a, e);
    if (ms < best) best = ms;
  }
  const double waves = (double)grid * block / 64.0;
  const double wave_instr = waves * ITERS * CH * instr_per_step;
  // cycles per wave64 instruction per SIMD at 2.4 GHz nominal
  const double cyc = 256.0 * 4 * 2.4e9 * (best * 1e-3) / wave_instr;
  printf("{\"instr\": \"%s\", \"ms\": %.4f, \"lane_instr_per_s\": %.4e, \"cycles_per_wave_instr_per_simd_at_2p4\": %.3f}\n",
         name, best, wave_instr * 64 / (best * 1e-3), cyc);
  return cyc;
}

int main() {
  const int grid = 256 * 32, block = 256;  // 8 waves per SIMD
  uint32_t* d;
  CHECK(hipMalloc(&d, sizeof(uint32_t) * grid * block));
  run("v_add_u32_e32 (VOP2)", k_add_vop2, 1, d, grid, block);
  run("v_xor_b32_e32 (VOP2)", k_xor_vop2, 1, d, grid, block);
  run("v_add3_u32 (VOP3)", k_add3_vop3, 1, d, grid, block);
  run("v_alignbit_b32 (VOP3)", k_alignbit, 1, d, grid, block);
  run("v_bitop3_b32 (VOP3)", k_bitop3, 1, d, grid, block);
  run("v_add_co_u32_e32 (VOP2, vcc)", k_addco, 1, d, grid, block);
  run("v_mad_u64_u32 + v_xor (VOP3 + VOP3)", k_mad64, 2, d, grid, block);
  run("v_mul_lo_u32 (VOP3)", k_mullo, 1, d, grid, block);
  run("v_mul_hi_u32 (VOP3)", k_mulhi, 1, d, grid, block);
  run("v_cndmask_b32_e64 (VOP3)", k_cndmask, 1, d, grid, block);
  return 0;
}
