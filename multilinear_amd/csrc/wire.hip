// FriProof wire format (host only): the reference serialises FriProof<Field128>
// with serde + bincode 2, config standard().with_little_endian()
// .with_fixed_int_encoding() (src/fri/mod.rs:239-249, 367-397):
//   Vec<T>            u64 LE length, then the items
//   HashDigest        GenericArray<u8, 32>: serde tuple -> 32 raw bytes
//   [u8; 32]          serde tuple -> 32 raw bytes
//   Field128          serialize_bytes(as_ref()) (field.rs:40-47): u64 length 16 + LE16
//   Direction         unit variant: u32 LE variant index (Left = 0, Right = 1)
//   structs / tuples  fields in declaration order, no framing
// FriProof = {commitments: Vec<HashDigest>, queries: Vec<QueryProof>,
//             last_elem: F, last_random: [u8; 32]};
// QueryProof = {paths: Vec<MerkleInclusionPath<ReedSolomonPair>>};
// MerkleInclusionPath = {value: ReedSolomonPair{value, minus_value},
//                        path: Vec<(HashDigest, Direction)>}.
// The flat mlh_fri_proof record omits the Direction (bit i of the opened
// index: Left iff set, merkle_tree/mod.rs:43-47); encode derives it from
// query_indices, decode recovers the indices from tree 0's directions and
// rejects paths whose directions disagree with index % leaves (the reference
// verifier would fail them with IncompatibleIndex, merkle_tree/mod.rs:243-248).
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/mlhip.h"
#include "host_field.hpp"

using namespace mlh;

namespace {

struct Writer {
  uint8_t* out;
  uint64_t cap, n = 0;
  void bytes(const uint8_t* p, uint64_t k) {
    if (out && n + k <= cap) memcpy(out + n, p, k);
    n += k;
  }
  void u64(uint64_t v) {
    uint8_t b[8];
    for (int i = 0; i < 8; ++i) b[i] = (uint8_t)(v >> (8 * i));
    bytes(b, 8);
  }
  void u32(uint32_t v) {
    uint8_t b[4];
    for (int i = 0; i < 4; ++i) b[i] = (uint8_t)(v >> (8 * i));
    bytes(b, 4);
  }
  void field(const uint8_t* le16) {
    u64(16);
    bytes(le16, 16);
  }
};

struct Reader {
  const uint8_t* in;
  uint64_t len, n = 0;
  bool ok = true;
  const uint8_t* take(uint64_t k) {
    if (!ok || n + k > len) {
      ok = false;
      return nullptr;
    }
    const uint8_t* p = in + n;
    n += k;
    return p;
  }
  uint64_t u64() {
    const uint8_t* p = take(8);
    uint64_t v = 0;
    if (p)
      for (int i = 0; i < 8; ++i) v |= (uint64_t)p[i] << (8 * i);
    return v;
  }
  uint32_t u32() {
    const uint8_t* p = take(4);
    uint32_t v = 0;
    if (p)
      for (int i = 0; i < 4; ++i) v |= (uint32_t)p[i] << (8 * i);
    return v;
  }
  // Field128 deserialize: 16 bytes, BaseElement::new reduces mod M
  bool field(uint8_t out[16]) {
    if (u64() != 16) ok = false;
    const uint8_t* p = take(16);
    if (!p) return false;
    h_store(out, h_reduce_once(h_load(p)));
    return ok;
  }
};

mlh_status encode(const mlh_fri_proof* pf, Writer& w) {
  const uint32_t L = pf->log_code, T = pf->num_trees;
  if (T + MLH_LOG_BLOWUP != L || L < 2 || L > 40) return MLH_ERR_INVALID;
  w.u64(T);
  for (uint32_t t = 0; t < T; ++t) w.bytes(pf->commitments + 32 * t, 32);
  const uint64_t qb = mlh_fri_query_bytes(L);
  w.u64(pf->num_queries);
  for (uint32_t q = 0; q < pf->num_queries; ++q) {
    const uint8_t* rec = pf->queries + q * qb;
    const uint64_t index = pf->query_indices[q];
    w.u64(T);
    for (uint32_t t = 0; t < T; ++t) {
      const uint32_t depth = L - 1 - t;
      const uint64_t idx = index & ((1ull << depth) - 1);  // index % leaves of tree t
      w.field(rec);
      w.field(rec + 16);
      w.u64(depth);
      for (uint32_t i = 0; i < depth; ++i) {
        w.bytes(rec + 32 + 32 * i, 32);
        w.u32((idx >> i) & 1 ? 0u : 1u);  // Left = 0 iff bit set
      }
      rec += 32 * (1 + depth);
    }
  }
  w.field(pf->last_elem);
  w.bytes(pf->last_random, 32);
  return MLH_OK;
}

}  // namespace

extern "C" {

uint64_t mlh_fri_proof_encoded_size(const mlh_fri_proof* pf) {
  if (!pf) return 0;
  const uint32_t L = pf->log_code, T = pf->num_trees;
  uint64_t per_query = 8;
  for (uint32_t t = 0; t < T; ++t) per_query += 48 + 8 + 36ull * (L - 1 - t);
  return 8 + 32ull * T + 8 + per_query * pf->num_queries + 24 + 32;
}

mlh_status mlh_fri_proof_encode(const mlh_fri_proof* pf, uint8_t* out, uint64_t cap) {
  if (!pf || !out || !pf->commitments || !pf->queries || !pf->query_indices) return MLH_ERR_INVALID;
  if (cap < mlh_fri_proof_encoded_size(pf)) return MLH_ERR_INVALID;
  Writer w{out, cap};
  return encode(pf, w);
}

mlh_status mlh_fri_proof_decode_header(const uint8_t* in, uint64_t len, uint32_t* log_code,
                                       uint32_t* num_queries) {
  if (!in || !log_code || !num_queries) return MLH_ERR_INVALID;
  Reader r{in, len};
  const uint64_t T = r.u64();
  if (!r.ok || T < 1 || T > 39) return MLH_ERR_INVALID;
  r.take(32 * T);
  const uint64_t nq = r.u64();
  if (!r.ok || nq > (1u << 20)) return MLH_ERR_INVALID;
  *log_code = (uint32_t)T + MLH_LOG_BLOWUP;
  *num_queries = (uint32_t)nq;
  return MLH_OK;
}

mlh_status mlh_fri_proof_decode(const uint8_t* in, uint64_t len, mlh_fri_proof* pf) {
  if (!in || !pf || !pf->commitments || !pf->queries) return MLH_ERR_INVALID;
  uint32_t L, nq;
  if (mlh_fri_proof_decode_header(in, len, &L, &nq) != MLH_OK) return MLH_ERR_INVALID;
  if (L != pf->log_code || nq != pf->num_queries) return MLH_ERR_INVALID;
  const uint32_t T = L - MLH_LOG_BLOWUP;
  pf->num_trees = T;
  Reader r{in, len};
  r.u64();
  memcpy(pf->commitments, r.take(32ull * T), 32ull * T);
  r.u64();
  const uint64_t qb = mlh_fri_query_bytes(L);
  bool consistent = true;
  for (uint32_t q = 0; q < nq && r.ok; ++q) {
    uint8_t* rec = pf->queries + q * qb;
    if (r.u64() != T) return MLH_ERR_INVALID;
    uint64_t index = 0;
    for (uint32_t t = 0; t < T && r.ok; ++t) {
      const uint32_t depth = L - 1 - t;
      r.field(rec);
      r.field(rec + 16);
      if (r.u64() != depth) return MLH_ERR_INVALID;
      for (uint32_t i = 0; i < depth && r.ok; ++i) {
        const uint8_t* sib = r.take(32);
        if (!sib) break;
        memcpy(rec + 32 + 32 * i, sib, 32);
        const uint32_t dir = r.u32();
        if (dir > 1) return MLH_ERR_INVALID;
        const uint64_t bit = dir == 0 ? 1 : 0;
        if (t == 0)
          index |= bit << i;
        else if (((index >> i) & 1) != bit)
          consistent = false;
      }
      rec += 32 * (1 + depth);
    }
    if (pf->query_indices) pf->query_indices[q] = index;
  }
  r.field(pf->last_elem);
  const uint8_t* lr = r.take(32);
  if (!r.ok || r.n != len) return MLH_ERR_INVALID;
  memcpy(pf->last_random, lr, 32);
  return consistent ? MLH_OK : MLH_ERR_VERIFY;
}

}  // extern "C"
