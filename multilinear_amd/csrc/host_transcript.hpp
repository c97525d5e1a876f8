// The host Fiat-Shamir transcript object behind mlh_transcript* (transcript.rs:5-55):
// a running SHA-256; random() = digest of a clone; next_challenge() =
// Field128::from(u128_le(random()[..16])) without absorbing.
#pragma once
#include <stdint.h>
#include <string.h>

#include "host_sha256.hpp"

struct mlh_transcript {
  mlh::HostSha256 sha;
};

// FriProof::prove / verify query index (fri/mod.rs:268-277):
// u64_le(random()[..8]) % half.
static inline uint64_t transcript_query_index(const mlh_transcript* tr, uint64_t half) {
  uint8_t rnd[32];
  tr->sha.digest(rnd);
  uint64_t u;
  memcpy(&u, rnd, 8);
  return u % half;
}
