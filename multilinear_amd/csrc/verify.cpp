// Host-only half of the C ABI: the Fiat-Shamir transcript, Merkle path
// verification and the FRI / PCS / batched verifiers (fri/mod.rs:184-340,
// multilinear_pcs.rs:138-190, batched_fri.rs:226-388, batched_pcs.rs:186-250,
// merkle_tree/mod.rs:216-293, transcript.rs).  Plain C++ with no HIP
// dependency, so the untrusted-input paths (these verifiers and the wire
// decoder, wire.hip) also build with host ASan/UBSan for the fuzz tests
// (tests/test_host_sanitized.py).
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/mlhip.h"
#include "host_field.hpp"
#include "host_sha256.hpp"
#include "host_transcript.hpp"

using namespace mlh;

extern "C" {

mlh_status mlh_transcript_create(mlh_transcript** out) {
  if (!out) return MLH_ERR_INVALID;
  *out = new mlh_transcript();
  return MLH_OK;
}
mlh_status mlh_transcript_clone(const mlh_transcript* t, mlh_transcript** out) {
  if (!t || !out) return MLH_ERR_INVALID;
  *out = new mlh_transcript(*t);
  return MLH_OK;
}
void mlh_transcript_destroy(mlh_transcript* t) { delete t; }
mlh_status mlh_transcript_absorb(mlh_transcript* t, const uint8_t* bytes, uint64_t len) {
  if (!t || (!bytes && len)) return MLH_ERR_INVALID;
  t->sha.update(bytes, (size_t)len);
  return MLH_OK;
}
mlh_status mlh_transcript_random(const mlh_transcript* t, uint8_t out[32]) {
  if (!t || !out) return MLH_ERR_INVALID;
  t->sha.digest(out);
  return MLH_OK;
}
mlh_status mlh_transcript_next_challenge(mlh_transcript* t, uint8_t out[16]) {
  if (!t || !out) return MLH_ERR_INVALID;
  uint8_t d[32];
  t->sha.digest(d);
  h_store(out, h_reduce_once(h_load(d)));  // Field128::from(u128), field.rs:138-142
  return MLH_OK;
}

uint64_t mlh_fri_query_bytes(uint32_t log_code) {
  if (log_code < 2) return 0;
  uint64_t items = 0;
  for (uint32_t t = 0; t + 1 < log_code; ++t) items += 1 + (log_code - 1 - t);
  return items * 32;
}


uint64_t mlh_batched_fri_query_bytes(uint32_t log_code, uint32_t num_codes) {
  if (log_code < 2 || num_codes == 0) return 0;
  uint64_t b = 32ull * num_codes + 32ull * (log_code - 1);
  for (uint32_t t = 0; t + 2 < log_code; ++t) b += 32ull * (1 + (log_code - 2 - t));
  return b;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// host verifiers (fri/mod.rs:184-340, multilinear_pcs.rs:138-190)
// ---------------------------------------------------------------------------
static void sha_pair(const uint8_t* a, const uint8_t* b, uint8_t out[32]) {
  HostSha256 s;
  s.update(a, 32);
  s.update(b, 32);
  s.digest(out);
}

// MerkleInclusionPath::verify (merkle_tree/mod.rs:216-253); directions from index bits.
static bool verify_path_len(const uint8_t* value, uint64_t len, const uint8_t* sibs,
                            uint32_t depth, const uint8_t root[32], uint64_t index) {
  uint8_t h[32];
  HostSha256 s;
  s.update(value, len);
  s.digest(h);
  for (uint32_t l = 0; l < depth; ++l) {
    uint8_t nh[32];
    if ((index >> l) & 1)
      sha_pair(sibs + 32 * l, h, nh);  // Direction::Left
    else
      sha_pair(h, sibs + 32 * l, nh);  // Direction::Right
    memcpy(h, nh, 32);
  }
  return memcmp(h, root, 32) == 0;
}

static bool verify_path(const uint8_t* value32, const uint8_t* sibs, uint32_t depth,
                        const uint8_t root[32], uint64_t index) {
  return verify_path_len(value32, 32, sibs, depth, root, index);
}

extern "C" {

mlh_status mlh_merkle_verify(const uint8_t* value, uint64_t value_len, const uint8_t* sibs,
                             uint32_t depth, uint64_t dirs, const uint8_t root[32],
                             uint64_t index) {
  if ((value_len && !value) || (depth && !sibs) || !root || depth > 63) return MLH_ERR_INVALID;
  uint8_t h[32];
  HostSha256 s;
  s.update(value, value_len);
  s.digest(h);
  uint64_t computed = 0;
  for (uint32_t l = 0; l < depth; ++l) {
    uint8_t nh[32];
    if ((dirs >> l) & 1) {  // Direction::Left
      computed += 1ull << l;
      sha_pair(sibs + 32 * l, h, nh);
    } else {
      sha_pair(h, sibs + 32 * l, nh);
    }
    memcpy(h, nh, 32);
  }
  if (memcmp(h, root, 32) != 0) return MLH_ERR_VERIFY;
  if (computed != index) return MLH_ERR_VERIFY_INDEX;
  return MLH_OK;
}

}  // extern "C"

// QueryProof::verify (fri/mod.rs:184-236) over flat records: ntrees paths,
// tree t has leaves n/2^t (depth log2(n) - t), gen of order 2n.
static bool query_chain(const uint8_t* rec, const uint8_t* commitments, uint32_t ntrees,
                        uint64_t n, uint64_t index, u128 gen, const u128* rs, u128 last) {
  const u128 inv2 = h_inv(2);
  uint64_t cur_n = n, cur_idx = index, off = 0;
  u128 cur_gen = gen;
  const uint32_t depth0 = 63 - __builtin_clzll(n);
  for (uint32_t t = 0; t < ntrees; ++t) {
    const uint32_t depth = depth0 - t;
    const uint8_t* val = rec + off;
    if (!verify_path(val, val + 32, depth, commitments + 32 * t, cur_idx)) return false;
    const u128 v = h_load(val), mv = h_load(val + 16);
    const u128 gp = h_pow(cur_gen, cur_idx);
    const u128 even = h_mul(h_add(v, mv), inv2);
    const u128 odd = h_mul(h_sub(v, mv), h_inv(h_mul(2, gp)));
    const u128 folded = h_add(even, h_mul(rs[t], odd));
    if (t + 1 == ntrees) return folded == last;
    const uint64_t nidx = cur_idx % (cur_n / 2);
    const uint8_t* nval = rec + off + 32ull * (1 + depth);
    const u128 nv = nidx == cur_idx ? h_load(nval) : h_load(nval + 16);
    if (nv != folded) return false;
    cur_gen = h_mul(cur_gen, cur_gen);
    cur_n /= 2;
    cur_idx = nidx;
    off += 32ull * (1 + depth);
  }
  return true;
}

static mlh_status fri_verify_queries(const mlh_fri_proof* pf, mlh_transcript* tr,
                                     const std::vector<u128>& rs) {
  const uint32_t L = pf->log_code;
  const uint64_t domain = 1ull << L;
  const u128 gen = h_pow2_generator(L);
  const uint64_t qbytes = mlh_fri_query_bytes(L);
  const u128 last = h_load(pf->last_elem);
  for (uint32_t q = 0; q < pf->num_queries; ++q) {
    const uint64_t index = transcript_query_index(tr, domain / 2);
    uint8_t le[8];
    memcpy(le, &index, 8);
    mlh_transcript_absorb(tr, le, 8);
    if (pf->query_indices && pf->query_indices[q] != index) return MLH_ERR_VERIFY;
    if (!query_chain(pf->queries + q * qbytes, pf->commitments, pf->num_trees, domain / 2, index,
                     gen, rs.data(), last))
      return MLH_ERR_VERIFY;
  }
  uint8_t lr[32];
  mlh_transcript_random(tr, lr);
  return memcmp(lr, pf->last_random, 32) == 0 ? MLH_OK : MLH_ERR_VERIFY;
}

// BatchedFriProof::verify_queries (batched_fri.rs:226-278, 345-388).
static mlh_status batched_verify_queries(const mlh_batched_fri_proof* pf, mlh_transcript* tr,
                                         const std::vector<u128>& rs, u128 fr) {
  const uint32_t L = pf->log_code, m = pf->num_codes;
  const uint64_t domain = 1ull << L, n = domain / 2;
  const u128 gen = h_pow2_generator(L);
  const uint64_t qbytes = mlh_batched_fri_query_bytes(L, m);
  const u128 inv2 = h_inv(2), last = h_load(pf->last_elem);
  for (uint32_t q = 0; q < pf->num_queries; ++q) {
    const uint64_t index = transcript_query_index(tr, n);
    if (pf->query_indices && pf->query_indices[q] != index) return MLH_ERR_VERIFY;
    const uint8_t* rec = pf->queries + q * qbytes;
    if (!verify_path_len(rec, 32ull * m, rec + 32ull * m, L - 1, pf->batch_commitment, index))
      return MLH_ERR_VERIFY;
    u128 v = 0, mv = 0;  // fingerprints (Horner over the codes)
    for (uint32_t j = 0; j < m; ++j) {
      v = h_add(h_mul(v, fr), h_load(rec + 32ull * j));
      mv = h_add(h_mul(mv, fr), h_load(rec + 32ull * j + 16));
    }
    const u128 gp = h_pow(gen, index);
    const u128 even = h_mul(h_add(v, mv), inv2);
    const u128 odd = h_mul(h_sub(v, mv), h_inv(h_mul(2, gp)));
    const u128 folded = h_add(even, h_mul(rs[0], odd));
    const uint8_t* inner = rec + 32ull * m + 32ull * (L - 1);
    if (pf->num_trees == 0) {
      if (folded != last) return MLH_ERR_VERIFY;
    } else {
      const uint64_t nidx = index % (n / 2);
      const u128 nv = nidx == index ? h_load(inner) : h_load(inner + 16);
      if (nv != folded) return MLH_ERR_VERIFY;
      if (!query_chain(inner, pf->commitments, pf->num_trees, n / 2, nidx, h_mul(gen, gen),
                       rs.data() + 1, last))
        return MLH_ERR_VERIFY;
    }
    uint8_t le[8];
    memcpy(le, &index, 8);
    mlh_transcript_absorb(tr, le, 8);
  }
  uint8_t lr[32];
  mlh_transcript_random(tr, lr);
  return memcmp(lr, pf->last_random, 32) == 0 ? MLH_OK : MLH_ERR_VERIFY;
}

extern "C" {

// Header checks of an untrusted proof before any shift or index is derived
// from it: the reference's verifiers index Vecs whose lengths the proof
// fixes and panic on an inconsistent proof; here that is MLH_ERR_VERIFY.
static bool fri_header_ok(uint32_t log_code, uint32_t num_trees, uint32_t want_trees) {
  return log_code >= 2 && log_code <= 41 && num_trees == want_trees;
}

mlh_status mlh_fri_verify(const mlh_fri_proof* pf) {
  if (!pf || !pf->commitments || !pf->queries) return MLH_ERR_INVALID;
  if (pf->num_queries != MLH_NUM_QUERIES) return MLH_ERR_VERIFY;
  if (pf->log_code < 2 || pf->log_code > 41) return MLH_ERR_VERIFY;
  if (pf->num_trees + MLH_LOG_BLOWUP != pf->log_code) return MLH_ERR_VERIFY;
  mlh_transcript tr;
  std::vector<u128> rs;
  for (uint32_t t = 0; t < pf->num_trees; ++t) {
    mlh_transcript_absorb(&tr, pf->commitments + 32 * t, 32);
    uint8_t r[16];
    mlh_transcript_next_challenge(&tr, r);
    rs.push_back(h_load(r));
  }
  mlh_transcript_absorb(&tr, pf->last_elem, 16);
  return fri_verify_queries(pf, &tr, rs);
}

mlh_status mlh_pcs_verify(const mlh_pcs_proof* pf, uint32_t n_vars, const uint8_t* inputs,
                          const uint8_t output[16], mlh_transcript* tr) {
  if (!pf || !tr || !output || !pf->sumcheck_polys || (n_vars && !inputs)) return MLH_ERR_INVALID;
  const mlh_fri_proof* fp = &pf->fri;
  if (fp->num_queries != MLH_NUM_QUERIES) return MLH_ERR_VERIFY;
  // n_vars >= 1: rs[n_vars - 1] below; the code of an n-variate MLE has
  // 2^(n + LOG_BLOWUP) elements (multilinear_pcs.rs:103-107)
  if (n_vars == 0 || !fri_header_ok(fp->log_code, fp->num_trees, n_vars) ||
      fp->log_code != n_vars + MLH_LOG_BLOWUP)
    return MLH_ERR_VERIFY;
  std::vector<u128> rs;
  for (uint32_t k = 0; k < n_vars; ++k) {
    mlh_transcript_absorb(tr, fp->commitments + 32 * k, 32);
    mlh_transcript_absorb(tr, pf->sumcheck_polys + 32 * k, 32);
    uint8_t r[16];
    mlh_transcript_next_challenge(tr, r);
    rs.push_back(h_load(r));
  }
  mlh_transcript_absorb(tr, fp->last_elem, 16);
  // SumcheckPolynomial::to_polynomial chain (sumcheck.rs:269-276)
  const u128 inv2 = h_inv(2);
  auto to_poly = [&](uint32_t k, u128 s, u128 c[3]) {
    c[1] = h_load(pf->sumcheck_polys + 32 * k);
    c[2] = h_load(pf->sumcheck_polys + 32 * k + 16);
    c[0] = h_mul(h_sub(s, h_add(c[1], c[2])), inv2);
  };
  auto eval = [&](const u128 c[3], u128 x) { return h_add(c[0], h_mul(x, h_add(c[1], h_mul(c[2], x)))); };
  u128 c[3];
  to_poly(0, h_load(output), c);
  for (uint32_t k = 1; k < n_vars; ++k) {
    const u128 v = eval(c, rs[k - 1]);
    to_poly(k, v, c);
  }
  const u128 r = rs[n_vars - 1];
  // Delta::evaluate (evaluation.rs:75-91)
  u128 delta = 1;
  for (uint32_t i = 0; i < n_vars; ++i) {
    const u128 a = h_load(inputs + 16 * i), b = rs[i];
    delta = h_mul(delta, h_add(h_mul(a, b), h_mul(h_sub(1, a), h_sub(1, b))));
  }
  if (h_mul(delta, h_load(fp->last_elem)) != eval(c, r)) return MLH_ERR_VERIFY;
  return fri_verify_queries(fp, tr, rs);
}

mlh_status mlh_batched_fri_verify(const mlh_batched_fri_proof* pf) {
  if (!pf || !pf->queries || (pf->num_trees && !pf->commitments) || pf->num_codes == 0)
    return MLH_ERR_INVALID;
  if (pf->num_queries != MLH_NUM_QUERIES) return MLH_ERR_VERIFY;
  if (pf->log_code < 2 || pf->log_code > 41) return MLH_ERR_VERIFY;
  if (pf->num_trees + 1 + MLH_LOG_BLOWUP != pf->log_code) return MLH_ERR_VERIFY;
  mlh_transcript tr;
  mlh_transcript_absorb(&tr, pf->batch_commitment, 32);
  uint8_t frb[16];
  mlh_transcript_next_challenge(&tr, frb);
  mlh_transcript_absorb(&tr, frb, 16);
  std::vector<u128> rs;
  uint8_t r[16];
  mlh_transcript_next_challenge(&tr, r);
  rs.push_back(h_load(r));
  for (uint32_t t = 0; t < pf->num_trees; ++t) {
    mlh_transcript_absorb(&tr, pf->commitments + 32 * t, 32);
    mlh_transcript_next_challenge(&tr, r);
    rs.push_back(h_load(r));
  }
  mlh_transcript_absorb(&tr, pf->last_elem, 16);
  return batched_verify_queries(pf, &tr, rs, h_load(frb));
}

mlh_status mlh_batched_pcs_verify(const mlh_batched_pcs_proof* pf, uint32_t n_vars,
                                  const uint8_t* inputs, const uint8_t* outputs,
                                  mlh_transcript* tr) {
  if (!pf || !tr || !inputs || !outputs || !pf->sumcheck_polys) return MLH_ERR_INVALID;
  const mlh_batched_fri_proof* fp = &pf->fri;
  if (fp->num_queries != MLH_NUM_QUERIES) return MLH_ERR_VERIFY;
  // n_vars >= 1 (the first round is the batch layer), num_trees = n_vars - 1,
  // code length 2^(n_vars + LOG_BLOWUP) (batched_pcs.rs:137-147, 186-250)
  if (n_vars == 0 || fp->num_codes == 0 || !fri_header_ok(fp->log_code, fp->num_trees, n_vars - 1) ||
      fp->log_code != n_vars + MLH_LOG_BLOWUP)
    return MLH_ERR_VERIFY;
  const uint32_t m = fp->num_codes;
  for (uint32_t i = 0; i < n_vars; ++i) mlh_transcript_absorb(tr, inputs + 16 * i, 16);
  for (uint32_t j = 0; j < m; ++j) mlh_transcript_absorb(tr, outputs + 16 * j, 16);
  std::vector<u128> rs;
  u128 fr = 0;
  for (uint32_t i = 0; i < n_vars; ++i) {
    if (i == 0) {
      mlh_transcript_absorb(tr, fp->batch_commitment, 32);
      uint8_t b[16];
      mlh_transcript_next_challenge(tr, b);
      fr = h_load(b);
      mlh_transcript_absorb(tr, b, 16);
    } else {
      mlh_transcript_absorb(tr, fp->commitments + 32 * (i - 1), 32);
    }
    mlh_transcript_absorb(tr, pf->sumcheck_polys + 32 * i, 32);
    uint8_t r[16];
    mlh_transcript_next_challenge(tr, r);
    rs.push_back(h_load(r));
  }
  mlh_transcript_absorb(tr, fp->last_elem, 16);
  // sumcheck chain from fingerprint(fr, outputs) (batched_pcs.rs:221-240)
  u128 sum = 0;
  for (uint32_t j = 0; j < m; ++j) sum = h_add(h_mul(sum, fr), h_load(outputs + 16 * j));
  const u128 inv2 = h_inv(2);
  u128 cur = sum, val = 0;
  for (uint32_t k = 0; k < n_vars; ++k) {
    const u128 c1 = h_load(pf->sumcheck_polys + 32 * k), c2 = h_load(pf->sumcheck_polys + 32 * k + 16);
    const u128 c0 = h_mul(h_sub(cur, h_add(c1, c2)), inv2);
    val = h_add(c0, h_mul(rs[k], h_add(c1, h_mul(c2, rs[k]))));
    cur = val;
  }
  // Delta::evaluate(inputs, rs) (evaluation.rs:75-91)
  u128 delta = 1;
  for (uint32_t i = 0; i < n_vars; ++i) {
    const u128 a = h_load(inputs + 16 * i), b = rs[i];
    delta = h_mul(delta, h_add(h_mul(a, b), h_mul(h_sub(1, a), h_sub(1, b))));
  }
  if (h_mul(delta, h_load(fp->last_elem)) != val) return MLH_ERR_VERIFY;
  return batched_verify_queries(fp, tr, rs, fr);
}

}  // extern "C"
