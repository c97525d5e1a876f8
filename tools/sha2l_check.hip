// Dev check: two-lane SHA-256 rounds and message schedule (transcript_dev.hpp
// sha2l_*, sha2l_sched) against the
// one-lane sha256_rounds_from / sha256_compress_kw on random states and blocks:
// a full compression, the 0..8 + 8..64 split with the mid-state, and a
// padding-only block from a precomputed K + W table.  One wave per test case.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/sha2l_check.hip -o tools/sha2l_check
#include "../multilinear_amd/csrc/transcript_dev.hpp"

#include <stdio.h>

#include <vector>

using namespace mlh;

__global__ void chk(const uint32_t* states, const uint32_t* blocks, const uint32_t* kwt, int n,
                    uint32_t* bad) {
  const int c = blockIdx.x;
  if (c >= n) return;
  const uint32_t lane = threadIdx.x;
  uint32_t v0[8], blk[16], w[16];
  for (int i = 0; i < 8; ++i) v0[i] = states[8 * c + i];
  for (int i = 0; i < 16; ++i) blk[i] = w[i] = blocks[16 * c + i];
  constexpr uint32_t K[64] = MLH_SHA_K;
  // reference: one lane
  uint32_t ref[8], refmid[8], refkw[8];
  {
    uint32_t v[8], b[16];
    for (int i = 0; i < 8; ++i) v[i] = v0[i];
    for (int i = 0; i < 16; ++i) b[i] = blk[i];
    sha256_rounds_from<0>(v, b, refmid);
    for (int i = 0; i < 8; ++i) ref[i] = v[i];
    Sha256State st;
    for (int i = 0; i < 8; ++i) st.h[i] = v0[i];
    sha256_compress_kw(st, kwt);
    for (int i = 0; i < 8; ++i) refkw[i] = st.h[i] - v0[i];  // the working state
  }
  // two lanes: 0..8, mid, 8..64
  Sha2L q;
  sha2l_init(q, v0);
  const Sched2L sc = sched2l_init();
  auto kwf = [&](int t) -> uint32_t {
    if (t >= 16) sha2l_sched(w, t, sc);
    return K[t] + w[t & 15];
  };
  sha2l_rounds<0, 8>(q, kwf);
  uint32_t mid[8];
  sha2l_state(q, mid);
  sha2l_init(q, mid);
  sha2l_rounds<8, 64>(q, kwf);
  uint32_t got[8];
  sha2l_state(q, got);
  Sha2L q2;
  sha2l_init(q2, v0);
  sha2l_rounds<0, 64>(q2, [&](int t) -> uint32_t { return kwt[t]; });
  uint32_t gotkw[8];
  sha2l_state(q2, gotkw);
  if (lane == 0) {
    uint32_t e = 0;
    for (int i = 0; i < 8; ++i) e |= (got[i] != ref[i]) | ((mid[i] != refmid[i]) << 1) | ((gotkw[i] != refkw[i]) << 2);
    if (e) atomicOr(bad, e);
  }
}

int main() {
  const int n = 512;
  std::vector<uint32_t> st(8 * n), bl(16 * n), kw(64);
  uint64_t x = 0x243F6A8885A308D3ull;
  auto next = [&]() {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return (uint32_t)x;
  };
  for (auto& v : st) v = next();
  for (auto& v : bl) v = next();
  for (auto& v : kw) v = next();
  uint32_t *ds, *db, *dk, *bad;
  hipMalloc(&ds, 4 * st.size());
  hipMalloc(&db, 4 * bl.size());
  hipMalloc(&dk, 4 * kw.size());
  hipMalloc(&bad, 4);
  hipMemcpy(ds, st.data(), 4 * st.size(), hipMemcpyHostToDevice);
  hipMemcpy(db, bl.data(), 4 * bl.size(), hipMemcpyHostToDevice);
  hipMemcpy(dk, kw.data(), 4 * kw.size(), hipMemcpyHostToDevice);
  hipMemset(bad, 0, 4);
  hipLaunchKernelGGL(chk, dim3(n), dim3(64), 0, 0, ds, db, dk, n, bad);
  uint32_t hb = 0;
  if (hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost) != hipSuccess) {
    printf("HIP error\n");
    return 1;
  }
  printf("two-lane SHA-256 vs one-lane over %d cases: %s (flags %u: 1 full, 2 mid, 4 kw)\n", n,
         hb ? "MISMATCH" : "match", hb);
  return hb ? 1 : 0;
}
