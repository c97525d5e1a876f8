// NTT launch interface (internal to libmlhip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.hpp"

namespace mlh {

constexpr int kMaxPasses = 6;
constexpr uint64_t kDirectMax = 1ull << 16;  // 1 MiB direct twiddle tables

// Device twiddle tables for one (log_n, generator, direction).
struct NttTables {
  uint32_t log_n = 0;
  uint32_t nradix = 0;
  uint32_t logr[kMaxPasses] = {0};
  const fe* tw[kMaxPasses] = {nullptr};  // per pass: w_R^t, t < R/2
  const fe* tlo0 = nullptr;              // pass 0: w^t * scale, t < 4096
  const fe* tlo = nullptr;               // passes > 0: w^t, t < 4096
  const fe* thi = nullptr;               // w^(4096 t), t < ceil(N/4096)
  const fe* tw_small = nullptr;          // N <= 2^10: w^t, t < N/2
  // per pass with N/S <= kDirectMax: w^(S t) (x scale on pass 0), t < N/S --
  // the inter-pass twiddle becomes one lookup instead of lookup*lookup
  const fe* tdir[kMaxPasses] = {nullptr};
  fe scale;                              // n^-1 (inverse) or 1
  bool inverse = false;
};

void ntt_plan_radices(uint32_t log_n, uint32_t* nradix, uint32_t* logr);

// batch: vectors of in_len inputs / N outputs, contiguous
hipError_t launch_ntt_small(const fe* in, fe* out, const fe* tw, uint32_t log_n, uint64_t in_len,
                            fe scale, bool apply_scale, hipStream_t st, uint64_t batch = 1);
// in: N elements (or N/2 when zero_top: the upper half is implicit zeros).
// in may equal out; scratch: N elements, distinct from in and out.
// ev (optional, nradix + 1 events): ev[p] is recorded before pass p, ev[P]
// after the last pass (kernel timing on the launch stream).
hipError_t launch_ntt_passes(const fe* in, fe* out, fe* scratch, const NttTables& tb,
                             uint32_t log_n, bool zero_top, hipStream_t st,
                             hipEvent_t* ev = nullptr, uint64_t batch = 1);
// rocprof-style kernel label of pass p ("ntt_pass<8,0,0>")
void ntt_pass_label(const NttTables& tb, uint32_t p, bool zero_top, char* buf, size_t n);
hipError_t launch_pow_table(fe* out, fe base, fe scale, uint64_t count, hipStream_t st);
hipError_t launch_pow_series(fe* out, const fe* tlo, const fe* thi, uint64_t count,
                             hipStream_t st);

}  // namespace mlh
