// Tree-tail timing (dev tool): launch_merkle_levels_from over a level of n
// random digests, n = 2^10..2^18 (subtree_kernel + top_kernel, with and
// without the root's transcript step): HIP-event time per call, and per-level
// s_memtime stamps of workgroup 0 ([level, cycles, us (s_memrealtime)]) (merkle.hip built with -DMLH_TREE_TS).
// Build: tools/build_tree_tail_bench.sh
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "../multilinear_amd/csrc/host_sha256.hpp"
#include "../multilinear_amd/csrc/merkle.hpp"
#include "../multilinear_amd/csrc/transcript_dev.hpp"

namespace mlh {
hipError_t tree_ts_read(uint64_t* out, bool clear);
}
using namespace mlh;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  const uint64_t maxn = 1ull << 18;
  uint8_t* layers;
  CHECK(hipMalloc(&layers, 2 * maxn * 32));
  std::vector<uint8_t> h(maxn * 32);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)(i * 2654435761u >> 13);
  CHECK(hipMemcpy(layers, h.data(), h.size(), hipMemcpyHostToDevice));
  DevSha* dt;
  fe* r;
  CHECK(hipMalloc(&dt, sizeof(DevSha)));
  CHECK(hipMalloc(&r, 64));
  HostSha256 hs;
  CHECK(hipMemcpy(dt, &hs, sizeof(DevSha), hipMemcpyHostToDevice));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int with_t = 0; with_t < 2; ++with_t) {
    for (uint32_t ln = 10; ln <= 18; ln += 2) {
      const uint64_t n = 1ull << ln;
      RootAbsorb ra;
      if (with_t) {
        ra.t = dt;
        ra.r_out = r;
      }
      for (int w = 0; w < 3; ++w) CHECK(launch_merkle_levels_from(layers, 0, n, st, ra));
      const int reps = 50;
      CHECK(hipEventRecord(a, st));
      for (int i = 0; i < reps; ++i) CHECK(launch_merkle_levels_from(layers, 0, n, st, ra));
      CHECK(hipEventRecord(b, st));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      // one stamped call
      CHECK(tree_ts_read(nullptr, true));
      CHECK(launch_merkle_levels_from(layers, 0, n, st, ra));
      CHECK(hipStreamSynchronize(st));
      uint64_t ts[4][64];
      CHECK(tree_ts_read(&ts[0][0], false));
      printf("{\"log_n\": %u, \"transcript\": %d, \"us_per_call\": %.2f", ln, with_t, ms * 1e3 / reps);
      for (int k = 0; k < 2; ++k) {
        printf(", \"%s_cycles\": [", k ? "top" : "subtree");
        bool first = true;
        for (int i = 1; i < 64; ++i) {
          if (!ts[k][i] || !ts[k][0]) continue;
          printf("%s[%d, %llu, %.2f]", first ? "" : ", ", i, (unsigned long long)(ts[k][i] - ts[k][0]),
                 (ts[k + 2][i] - ts[k + 2][0]) * 0.01);
          first = false;
        }
        printf("]");
      }
      printf("}\n");
    }
  }
  return 0;
}
