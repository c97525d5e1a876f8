// Host fuzz driver for the untrusted-input paths of the C ABI: the FriProof
// wire decoder (wire.hip) and the FRI / PCS / batched verifiers (verify.cpp).
// Built with -fsanitize=address,undefined by tests/test_host_sanitized.py and
// run on CPU.  Input: a valid encoded FriProof (the oracle's proof of a small
// RS codeword).  It checks the seed decodes and verifies, then decodes and
// verifies thousands of mutations (byte flips, truncations, extensions,
// forged lengths, non-canonical field elements, forged directions) and calls
// the PCS / batched verifiers with inconsistent headers.  Any out-of-bounds
// access or UB aborts through the sanitizers; a mutated proof that verifies is
// reported and fails the run.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/mlhip.h"

static uint64_t rng_state = 0x5EEDull;
static uint64_t rnd() {
  uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Buf {
  std::vector<uint8_t> commit, queries, last_random;
  std::vector<uint64_t> idx;
  mlh_fri_proof pf{};
  bool alloc(uint32_t L, uint32_t nq) {
    if (L < 2 || L > 24 || nq > 4096) return false;
    commit.assign(32ull * (L - 1), 0);
    queries.assign(mlh_fri_query_bytes(L) * nq, 0);
    idx.assign(nq ? nq : 1, 0);
    pf = mlh_fri_proof{};
    pf.log_code = L;
    pf.num_queries = nq;
    pf.commitments = commit.data();
    pf.queries = queries.data();
    pf.query_indices = idx.data();
    return true;
  }
};

// decode (and verify when it decodes); returns the verify status or the decode error
static mlh_status decode_verify(const std::vector<uint8_t>& w, Buf& b) {
  uint32_t L = 0, nq = 0;
  mlh_status s = mlh_fri_proof_decode_header(w.data(), w.size(), &L, &nq);
  if (s != MLH_OK) return s;
  if (!b.alloc(L, nq)) return MLH_ERR_INVALID;
  s = mlh_fri_proof_decode(w.data(), w.size(), &b.pf);
  if (s != MLH_OK) return s;
  return mlh_fri_verify(&b.pf);
}

static void put_u64(std::vector<uint8_t>& w, size_t at, uint64_t v) {
  if (at + 8 > w.size()) return;
  for (int i = 0; i < 8; ++i) w[at + i] = (uint8_t)(v >> (8 * i));
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: fuzz_verify <proof.bin> <iterations>\n");
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> seed;
  uint8_t tmp[4096];
  size_t k;
  while ((k = fread(tmp, 1, sizeof tmp, f)) > 0) seed.insert(seed.end(), tmp, tmp + k);
  fclose(f);
  const long iters = atol(argv[2]);

  Buf b;
  if (decode_verify(seed, b) != MLH_OK) {
    fprintf(stderr, "seed proof does not verify\n");
    return 1;
  }
  // re-encode round trip
  std::vector<uint8_t> enc(mlh_fri_proof_encoded_size(&b.pf));
  if (mlh_fri_proof_encode(&b.pf, enc.data(), enc.size()) != MLH_OK || enc != seed) {
    fprintf(stderr, "encode(decode(seed)) != seed\n");
    return 1;
  }
  const uint32_t L = b.pf.log_code;

  long accepted = 0, rejected = 0;
  for (long it = 0; it < iters; ++it) {
    std::vector<uint8_t> w = seed;
    const int kind = (int)(rnd() % 8);
    switch (kind) {
      case 0:  // flip 1..8 random bytes
        for (int j = 0, n = 1 + (int)(rnd() % 8); j < n; ++j) w[rnd() % w.size()] ^= (uint8_t)(1 + rnd() % 255);
        break;
      case 1:  // truncate
        w.resize(rnd() % w.size());
        break;
      case 2:  // extend with garbage
        for (int j = 0, n = 1 + (int)(rnd() % 64); j < n; ++j) w.push_back((uint8_t)rnd());
        break;
      case 3:  // forged commitment count / query count
        put_u64(w, 0, rnd() % 3 == 0 ? rnd() : rnd() % 64);
        break;
      case 4:
        put_u64(w, 8 + 32ull * (L - 1), rnd() % 3 == 0 ? rnd() : rnd() % 300);
        break;
      case 5: {  // non-canonical field element (>= M) somewhere: 16 bytes of 0xFF
        size_t at = rnd() % w.size();
        for (size_t j = at; j < at + 16 && j < w.size(); ++j) w[j] = 0xFF;
        break;
      }
      case 6: {  // forged u64 length at a random 8-aligned offset
        put_u64(w, (rnd() % (w.size() / 8)) * 8, rnd() % 2 ? rnd() : rnd() % 100);
        break;
      }
      default: {  // flip a direction word (u32 0/1 -> other values)
        size_t at = rnd() % w.size();
        if (at + 4 <= w.size()) {
          uint32_t v = (uint32_t)(rnd() % 4);
          memcpy(&w[at], &v, 4);
        }
        break;
      }
    }
    Buf m;
    const mlh_status s = decode_verify(w, m);
    if (s == MLH_OK) {
      // only a mutation that left the proof's meaning intact may verify:
      // the decoded proof must re-encode to exactly the seed's bytes
      std::vector<uint8_t> re(mlh_fri_proof_encoded_size(&m.pf));
      mlh_fri_proof_encode(&m.pf, re.data(), re.size());
      if (re != seed) {
        fprintf(stderr, "mutation %ld (kind %d) verified but differs from the seed\n", it, kind);
        return 1;
      }
      ++accepted;
    } else {
      ++rejected;
    }
  }

  // PCS / batched verifiers: inconsistent headers must be rejected before any
  // index or shift is derived from them (n_vars = 0, log_code mismatch, huge
  // log_code, tree counts off by one)
  std::vector<uint8_t> polys(32 * 64, 0), inputs(16 * 64, 0), out16(16, 0), outs(16 * 4, 0);
  mlh_transcript* tr = nullptr;
  mlh_transcript_create(&tr);
  const uint32_t bad_nvars[] = {0, L - 2, L, L + 1, 63, 0xFFFFFFFFu};
  for (uint32_t nv : bad_nvars) {
    mlh_pcs_proof pp{};
    pp.sumcheck_polys = polys.data();
    pp.fri = b.pf;
    if (nv == L - 1) continue;
    mlh_status s = mlh_pcs_verify(&pp, nv, inputs.data(), out16.data(), tr);
    if (s == MLH_OK) {
      fprintf(stderr, "pcs_verify accepted n_vars=%u\n", nv);
      return 1;
    }
  }
  for (uint32_t lc : {0u, 1u, 42u, 64u, 200u}) {
    mlh_pcs_proof pp{};
    pp.sumcheck_polys = polys.data();
    pp.fri = b.pf;
    pp.fri.log_code = lc;
    if (mlh_pcs_verify(&pp, L - 1, inputs.data(), out16.data(), tr) == MLH_OK) return 1;
    mlh_fri_proof fp = b.pf;
    fp.log_code = lc;
    fp.num_trees = lc ? lc - 1 : 0;
    if (mlh_fri_verify(&fp) == MLH_OK) return 1;
  }
  {
    mlh_batched_fri_proof bp{};
    std::vector<uint8_t> bq(1 << 20, 0);
    bp.commitments = b.commit.data();
    bp.queries = bq.data();
    bp.num_queries = MLH_NUM_QUERIES;
    bp.num_codes = 2;
    for (uint32_t lc : {0u, 1u, 2u, 42u, 64u}) {
      for (uint32_t nt : {0u, 1u, 0xFFFFFFFFu}) {
        bp.log_code = lc;
        bp.num_trees = nt;
        if (mlh_batched_fri_verify(&bp) == MLH_OK) return 1;
        mlh_batched_pcs_proof bpp{};
        bpp.sumcheck_polys = polys.data();
        bpp.fri = bp;
        for (uint32_t nv : {0u, 1u, 2u, 40u}) {
          if (mlh_batched_pcs_verify(&bpp, nv, inputs.data(), outs.data(), tr) == MLH_OK) return 1;
        }
      }
    }
  }
  mlh_transcript_destroy(tr);
  printf("fuzz ok: %ld mutations (%ld decoded+verified identical, %ld rejected)\n", iters, accepted,
         rejected);
  return 0;
}
