"""bincode 2 wire format of FriProof<Field128> (oracle).  Test infrastructure only.

Restates what the reference's `bincode::serde::encode_to_vec(&proof,
standard().with_little_endian().with_fixed_int_encoding())` produces for
src/fri/mod.rs:239-249 (FriProof), :177-181 (QueryProof), :31-35
(ReedSolomonPair), src/merkle_tree/mod.rs:13-24 (Direction,
MerkleInclusionPath) and src/field.rs:40-47 (Field128 -> serialize_bytes):
bincode 2 + serde, fixed-int: sequence and byte-slice lengths are u64 LE,
unit enum variants are their u32 LE index, tuples / arrays / GenericArray are
their elements back to back.  (bincode 2.0.1 and serde 1.0.219 are not
vendored in /root/reference: these rules are their published encoding,
recalled; no reference-produced proof bytes exist -- parity unpinned.)
"""
import struct

from . import field as F


def _u64(v):
    return struct.pack("<Q", v)


def _field(v):
    return _u64(16) + F.to_bytes(v)


def encode_fri_proof(proof):
    """proof: oracle.fri.FriProof (commitments, queries = [[(pair32, [(sib, dir)])]],
    last_elem, last_random); dir 0 = Left, 1 = Right."""
    out = [_u64(len(proof.commitments))] + list(proof.commitments)
    out.append(_u64(len(proof.queries)))
    for q in proof.queries:
        out.append(_u64(len(q)))
        for pair, path in q:
            out.append(_field(F.from_bytes(pair[:16])) + _field(F.from_bytes(pair[16:])))
            out.append(_u64(len(path)))
            for sib, d in path:
                out.append(sib + struct.pack("<I", d))
    out.append(_field(proof.last_elem))
    out.append(proof.last_random)
    return b"".join(out)
