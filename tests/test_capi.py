"""CPU tests of the drop-in boundary: libmlhip.so loads, exports every symbol
include/mlhip.h declares, the ctypes table covers them, and the host-only
entry points (generators, transcript, proof sizes, the host-side FRI / PCS
verifiers) behave like the reference -- no GPU compute is called here."""
import ctypes
import os
import re

import pytest

from multilinear_amd import _lib
from oracle import field as F
from oracle import fri as OF
from oracle import pcs as OP
from oracle import polynomials as OPL
from oracle import transcript as OT

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "mlhip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mlh_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 50
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_no_gpu_means_loud_failure():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.mlh_context_create(0, None, ctypes.byref(h)) == 4  # MLH_ERR_HIP, no fallback
    assert b"hipGetDeviceCount" in lib.mlh_last_error(None)  # the reason, without a context


def test_generators_match_oracle():
    lib = _lib.load()
    for k in (0, 1, 12, 24, 25, 40):
        out = (ctypes.c_uint8 * 16)()
        assert lib.mlh_pow_2_generator(k, out) == 0
        assert int.from_bytes(bytes(out), "little") == F.pow_2_generator(k)
    assert lib.mlh_pow_2_generator(41, (ctypes.c_uint8 * 16)()) == 1


def _gp_call(lib, table):
    raw = b"".join(int(v).to_bytes(16, "little") for v in table)
    buf = (ctypes.c_uint8 * max(16, len(raw))).from_buffer_copy(raw.ljust(16, b"\0"))
    g, lg = (ctypes.c_uint8 * 16)(), ctypes.c_uint32()
    st = lib.mlh_gen_pows_params(buf, len(table), g, ctypes.byref(lg))
    return st, int.from_bytes(bytes(g), "little"), lg.value


def test_gen_pows_shim_accepts_power_series_rejects_others():
    """The Rust shim's mapping gen_pows: &[F] -> (gen_pows[1], log2 len) of the
    _gp entry points (fri/mod.rs:79-114, :261): the reference's own table
    (pow_2_generator_powers) maps to (g, log2 len); a table that differs from
    that power series at an index the spot check covers (every index < 4096,
    every 2^j, len/2, len-1) is rejected with MLH_ERR_INVALID.  What it does
    not cover is mlh_gen_pows_verify's (test_gpu_parity.py)."""
    lib = _lib.load()
    for lg in (1, 2, 5, 10, 13):
        tab = F.pow_2_generator_powers(lg)
        assert _gp_call(lib, tab) == (0, tab[1], lg)
    tab = F.pow_2_generator_powers(10)
    bad = [list(tab) for _ in range(8)]
    bad[0][0] = 2                                # gen_pows[0] != 1
    bad[1][len(tab) - 1] = (tab[-1] + 1) % F.M   # last entry not g^-1
    bad[2][512] = 1                              # gen_pows[len/2] != -1
    bad[3][64] = (tab[64] * 3) % F.M             # gen_pows[2^j] != g^(2^j)
    bad[4] = F.pow_2_generator_powers(11)[:1024]  # g of order 2^11, table of 2^10
    bad[5][1] = F.M + 1                          # non-canonical g
    bad[6][3] = (tab[3] + 1) % F.M               # an interior entry
    bad[7][1000] = tab[999]                      # a late interior entry (< 4096: checked)
    for b in bad:
        assert _gp_call(lib, b)[0] == 1, b[:3]
    assert _gp_call(lib, tab[:768])[0] == 1      # not a power of two
    assert _gp_call(lib, tab[:1])[0] == 1
    # beyond index 4096 only the structural and sampled indices are checked:
    # the documented limit of the spot check (mlh_gen_pows_verify is the full one)
    big = F.pow_2_generator_powers(13)
    assert _gp_call(lib, big) == (0, big[1], 13)
    alt = list(big)
    alt[4097] = (alt[4097] + 1) % F.M
    assert _gp_call(lib, alt)[0] == 0  # 4097 is not among the sampled indices at len 2^13


def test_transcript_matches_reference_semantics():
    from multilinear_amd.transcript import Transcript

    t, o = Transcript(), OT.Transcript()
    for chunk in (b"", b"root" * 8, bytes(range(100)), b"x" * 64, b"y" * 63):
        t.absorb(chunk)
        o.absorb(chunk)
        assert t.random() == o.random()
        assert t.next_challenge() == o.next_challenge()
        assert t.next_challenge() == t.next_challenge()  # no absorb between calls
    c = t.clone()
    c.absorb(b"z")
    assert c.random() != t.random()


_SHA_STREAM = r"""
import hashlib, random, sys
sys.path.insert(0, %r)
from multilinear_amd.transcript import Transcript
rr = random.Random(11)
t, h = Transcript(), hashlib.sha256()
for _ in range(300):
    b = bytes(rr.randrange(256) for _ in range(rr.choice([0, 1, 3, 8, 16, 32, 55, 56, 63, 64, 65, 200])))
    t.absorb(b)
    h.update(b)
    assert t.random() == h.digest()
print("ok")
"""


@pytest.mark.parametrize("no_shani", [False, True])
def test_host_sha256_both_compressions(no_shani):
    """The host transcript's SHA-256 (x86 SHA extensions when present, else
    portable) against hashlib over random absorb chunk sizes; the portable
    path forced with MLH_NO_SHANI=1 in a fresh process."""
    import os
    import subprocess
    import sys

    env = dict(os.environ)
    env.pop("MLH_NO_SHANI", None)
    if no_shani:
        env["MLH_NO_SHANI"] = "1"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _SHA_STREAM % root], env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr


def test_proof_sizes():
    lib = _lib.load()
    assert lib.mlh_merkle_layers_bytes(1 << 10) == (2 * 1024 - 1) * 32
    L = 11
    assert lib.mlh_fri_query_bytes(L) == 32 * sum(1 + (L - 1 - t) for t in range(L - 1))


def _fill_fri_struct(proof, log_code):
    """Pack an oracle FriProof into the C struct layout of mlhip.h."""
    from multilinear_amd import _lib as L

    T = log_code - 1
    commit = (ctypes.c_uint8 * (32 * T)).from_buffer_copy(b"".join(proof.commitments))
    qb = L.load().mlh_fri_query_bytes(log_code)
    raw = b""
    for q in proof.queries:
        for value, path in q:
            raw += value + b"".join(s for s, _ in path)
    assert len(raw) == qb * 128
    qbuf = (ctypes.c_uint8 * len(raw)).from_buffer_copy(raw)
    c = L.FriProofC()
    c.log_code = log_code
    c.num_trees = T
    c.num_queries = 128
    c.commitments = ctypes.cast(commit, ctypes.c_void_p)
    c.last_elem[:] = list(F.to_bytes(proof.last_elem))
    c.last_random[:] = list(proof.last_random)
    c.query_indices = None
    c.queries = ctypes.cast(qbuf, ctypes.c_void_p)
    return c, (commit, qbuf)


def test_host_fri_verifier_accepts_oracle_proof():
    """mlh_fri_verify (FriProof::verify, fri/mod.rs:287-340) on an oracle proof."""
    lib = _lib.load()
    ln = 8
    vals = [F.from_i64(7 * i + 3) for i in range(1 << ln)]
    gp = F.pow_2_generator_powers(ln + 1)
    code = OF.reed_solomon(vals, gp[1])
    proof = OF.FriProof.prove(code, gp, OT.Transcript())
    c, keep = _fill_fri_struct(proof, ln + 1)
    assert lib.mlh_fri_verify(ctypes.byref(c)) == 0
    c.last_random[0] ^= 1
    assert lib.mlh_fri_verify(ctypes.byref(c)) == 7
    c.last_random[0] ^= 1
    keep[1][100] ^= 1
    assert lib.mlh_fri_verify(ctypes.byref(c)) == 7


def test_host_pcs_verifier_accepts_oracle_proof():
    """mlh_pcs_verify (PCSProof::verify, multilinear_pcs.rs:138-190)."""
    from multilinear_amd.device import fe_bytes
    from multilinear_amd.polynomials import _points
    from multilinear_amd.transcript import Transcript

    lib = _lib.load()
    n = 7
    ev = [F.from_i64(7 * i + 3) for i in range(1 << n)]
    pts = [F.from_i64(i) for i in range(n)]
    out = OPL.mle_evaluate(ev, pts)
    p = OP.PCSProof.prove(pts, out, ev, OT.Transcript())
    c, keep = _fill_fri_struct(p.fri_proof, n + 1)
    polys = (ctypes.c_uint8 * (32 * n)).from_buffer_copy(
        b"".join(F.to_bytes(a) + F.to_bytes(b) for a, b in p.sumcheck_polynomials))
    pc = _lib.PcsProofC()
    pc.fri = c
    pc.sumcheck_polys = ctypes.cast(polys, ctypes.c_void_p)
    t1, t2 = Transcript(), Transcript()  # (alive across the calls: the C side takes their pointers)
    assert lib.mlh_pcs_verify(ctypes.byref(pc), n, _points(pts), fe_bytes(out), t1.h) == 0
    assert lib.mlh_pcs_verify(ctypes.byref(pc), n, _points(pts), fe_bytes(out + 1), t2.h) == 7


def test_fri_proof_wire_format_matches_oracle_encoding():
    """mlh_fri_proof_{encode,decode} vs oracle/wire.py (bincode 2 fixed-int
    serde layout of FriProof<Field128>, fri/mod.rs:239-249, 367-397)."""
    from multilinear_amd.fri import FriProof
    from oracle import wire as OW

    ln = 7
    vals = [F.from_i64(7 * i + 3) for i in range(1 << ln)]
    gp = F.pow_2_generator_powers(ln + 1)
    proof = OF.FriProof.prove(OF.reed_solomon(vals, gp[1]), gp, OT.Transcript())
    want = OW.encode_fri_proof(proof)
    L = ln + 1
    per_query = 8 + sum(48 + 8 + 36 * (L - 1 - t) for t in range(L - 1))
    assert len(want) == 8 + 32 * (L - 1) + 8 + 128 * per_query + 24 + 32
    dec = FriProof.from_bytes(want)  # indices recovered from the directions
    assert dec.verify()
    assert dec.commitments == proof.commitments and dec.last_elem == proof.last_elem
    tr = OT.Transcript()
    for c in proof.commitments:
        tr.absorb(c)
    tr.absorb(F.to_bytes(proof.last_elem))
    for q in range(128):
        i = OF.query_index(tr, 1 << L)
        tr.absorb(i.to_bytes(8, "little"))
        assert dec.query_indices[q] == i
    assert dec.to_bytes() == want
    # malformed: truncated, trailing byte, wrong field length, bad / inconsistent direction
    with pytest.raises(_lib.MlhError):
        FriProof.from_bytes(want[:-1])
    with pytest.raises(_lib.MlhError):
        FriProof.from_bytes(want + b"\0")
    off = 8 + 32 * (L - 1) + 8 + 8  # first query's first path: value field length
    bad = bytearray(want)
    bad[off] = 15
    with pytest.raises(_lib.MlhError):
        FriProof.from_bytes(bytes(bad))
    # direction of tree 1, level 0 (inconsistent with tree 0's index bit)
    d_off = off + 48 + 8 + 36 * (L - 1) + 48 + 8 + 32
    bad = bytearray(want)
    bad[d_off] ^= 1
    with pytest.raises(_lib.MlhError) as e:
        FriProof.from_bytes(bytes(bad))
    assert e.value.status == 7
    bad[d_off] = 2
    with pytest.raises(_lib.MlhError):
        FriProof.from_bytes(bytes(bad))


def _fill_batched(proof, log_code, m):
    """oracle BatchedFriProof -> C layout (mlh_batched_fri_proof)."""
    from multilinear_amd.batched import BatchedFriProof

    p = BatchedFriProof(log_code, m)
    raw = b""
    for (col, bpath), inner in proof.queries:
        raw += b"".join(col) + b"".join(s for s, _ in bpath)
        for value, path in inner:
            raw += value + b"".join(s for s, _ in path)
    assert len(raw) == p.qbytes * 128
    ctypes.memmove(p._q, raw, len(raw))
    if proof.commitments:
        ctypes.memmove(p._commit, b"".join(proof.commitments), 32 * len(proof.commitments))
    p.c.num_trees = len(proof.commitments)
    p.c.num_queries = 128
    p.c.query_indices = None
    p.c.batch_commitment[:] = list(proof.batch_commitment)
    p.c.last_elem[:] = list(F.to_bytes(proof.last_elem))
    p.c.last_random[:] = list(proof.last_random)
    return p


@pytest.mark.parametrize("m,log_n", [(1, 4), (3, 5), (2, 1)])
def test_host_batched_fri_verifier_accepts_oracle_proof(m, log_n):
    """mlh_batched_fri_verify (batched_fri.rs:313-388) on oracle proofs."""
    from oracle import batched as OB

    gp = F.pow_2_generator_powers(log_n + 1)
    codes = [OF.reed_solomon([F.from_i64(7 * i + 3 + 100 * j) for i in range(1 << log_n)], gp[1])
             for j in range(m)]
    proof = OB.BatchedFriProof.prove(codes, gp, OT.Transcript())
    assert proof.verify()
    p = _fill_batched(proof, log_n + 1, m)
    assert p.verify()
    p.c.batch_commitment[3] ^= 1
    assert not p.verify()
    p.c.batch_commitment[3] ^= 1
    p._q[5] ^= 1  # an opened batch value
    assert not p.verify()


def test_host_batched_pcs_verifier_accepts_oracle_proof():
    """mlh_batched_pcs_verify (batched_pcs.rs:182-250) on an oracle proof."""
    from multilinear_amd.batched import BatchedPCSProof
    from oracle import batched as OB

    n, m = 5, 3
    pts = [F.from_i64(i) for i in range(n)]
    polys = [[F.from_i64((j * 3 + i * 5) % 100) for j in range(1 << n)] for i in range(m)]
    outs = [OPL.mle_evaluate(p, pts) for p in polys]
    pr = OB.BatchedPCSProof.prove(pts, outs, polys, OT.Transcript())
    assert pr.verify(OT.Transcript())
    bp = BatchedPCSProof(n, m)
    fp = _fill_batched(pr.fri_proof, n + 1, m)
    bp.fri_proof = fp
    raw = b"".join(F.to_bytes(a) + F.to_bytes(b) for a, b in pr.sumcheck_polynomials)
    ctypes.memmove(bp._polys, raw, len(raw))
    bp.inputs, bp.outputs = pts, outs
    from multilinear_amd.transcript import Transcript

    assert bp.verify(Transcript())
    bp.outputs = [outs[0] + 1] + outs[1:]
    assert not bp.verify(Transcript())


def test_host_merkle_verify_matches_reference_semantics():
    """MerkleInclusionPath::verify / batch_verify (merkle_tree/mod.rs:216-293)
    through mlh_merkle_verify on oracle-built paths: Ok, IncompatibleHash for a
    wrong value, IncompatibleIndex for directions that do not spell the index."""
    from multilinear_amd import _lib
    from multilinear_amd import merkle_tree as MM
    from oracle import merkle as OM

    data = [bytes([v]) for v in [0, 8, 4, 1, 5, 7, 6, 1]]
    t = OM.Merkle.commit(data)
    for i in range(8):
        value, path = t.open(i)
        assert MM.verify_status(value, path, t.root(), i) == _lib.MLH_OK
    value, path = t.open(5)
    assert MM.verify_status(value, path, t.root(), 4) == _lib.STATUS_CODES["MLH_ERR_VERIFY_INDEX"]
    assert MM.verify_status(b"\x00", path, t.root(), 5) == _lib.STATUS_CODES["MLH_ERR_VERIFY"]
    bt = OM.Merkle.batch_commit([data, [bytes([v]) for v in [1, 3, 2, 3, 2, 1, 2, 3]]])
    col, path = OM.batch_open(bt, 2)
    assert MM.batch_verify(col, path, bt.root(), 2)
    assert not MM.batch_verify(col, path, bt.root(), 1)
