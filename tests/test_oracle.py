"""CPU tests of the oracle (the checker): known answers of the algorithms the
reference depends on, the reference's own tests restated, golden fixtures,
and agreement of the two independent restatements (Python and C)."""
import hashlib
import json
import os
import random

import pytest

from oracle import field as F
from oracle import fri as OF
from oracle import merkle as OM
from oracle import ntt as ON
from oracle import pcs as OP
from oracle import polynomials as OPL
from oracle import sumcheck as OS
from oracle import transcript as OT

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def h(v):
    return "%032x" % v


# ---- published known answers --------------------------------------------------

def test_sha256_fips180_vectors():
    """FIPS 180-4 / NIST CAVS examples (sha2 0.10.8 implements this)."""
    kat = {
        b"": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
        b"abc": "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad",
        b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq":
            "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1",
    }
    for msg, want in kat.items():
        assert hashlib.sha256(msg).hexdigest() == want
        assert OM.hash_leaf(msg).hex() == want


def test_field_constants():
    """src/ntt/mod.rs:34-54 and winter-math f128's published constants."""
    assert F.M == 340282366920938463463374557953744961537 == 2**128 - 45 * 2**40 + 1
    assert (F.M - 1) & -(F.M - 1) == 2**40  # two-adicity 40
    g40 = F.pow_2_generator(40)
    assert g40 == F.WINTER_TWO_ADIC_ROOT
    assert F.fpow(g40, 2**40) == 1 and F.fpow(g40, 2**39) == F.M - 1
    assert F.pow_2_generator(41) is None
    # From<i64> of a negative value is NOT -v mod M (field.rs:150-154)
    assert F.from_i64(-1) == 49478023249918 == int(GOLDEN["from_i64_minus1"])
    assert F.from_u128(F.M) == 0 and F.from_u128(2**128 - 1) == 2**128 - 1 - F.M


# ---- the reference's own tests, restated on the oracle ---------------------------

def test_intt_roundtrip_oracle():
    """intt_test (ntt/mod.rs:191-201) at 2^10 (2^18 in the C oracle test)."""
    ln = 10
    coeffs = [F.from_i64(i) for i in range(1 << ln)]
    g = F.pow_2_generator(ln)
    assert ON.intt(ON.ntt(coeffs, g), g) == coeffs


def test_ntt_equals_definition():
    for ln in range(1, 8):
        g = F.pow_2_generator(ln)
        x = [random.Random(ln).randrange(F.M) for _ in range(1 << ln)]
        assert ON.ntt(x, g) == ON.ntt_direct(x, g)


def test_merkle_open_verify():
    """merkle_test (merkle_tree/mod.rs:300-309)."""
    data = [bytes([v]) for v in [0, 8, 4, 1, 5, 7, 6, 1]]
    t = OM.Merkle.commit(data)
    value, path = t.open(5)
    assert OM.verify(value, path, t.root(), 5)
    assert not OM.verify(value, path, t.root(), 4)


def test_batched_merkle():
    """batched_merkle_test (merkle_tree/mod.rs:311-351)."""
    data = [[bytes([v]) for v in [0, 8, 4, 1, 5, 7, 6, 1]],
            [bytes([v]) for v in [1, 3, 2, 3, 2, 1, 2, 3]]]
    t = OM.Merkle.batch_commit(data)
    value, path = OM.batch_open(t, 5)
    assert value == [bytes([7]), bytes([1])]
    assert OM.batch_verify(value, path, t.root(), 5)
    value, path = OM.batch_open(t, 2)
    assert value == [bytes([4]), bytes([2])]
    assert OM.batch_verify(value, path, t.root(), 2)
    assert not OM.batch_verify(value, path, t.root(), 1)


def test_fri_prove_and_verify_oracle():
    """prove_and_verify_test (fri/mod.rs:349-363): log_n 10, values 7i+3."""
    ln = 10
    vals = [F.from_i64(7 * i + 3) for i in range(1 << ln)]
    gp = F.pow_2_generator_powers(ln + 1)
    code = OF.reed_solomon(vals, gp[1])
    proof = OF.FriProof.prove(code, gp, OT.Transcript())
    assert proof.verify()
    proof.last_elem = (proof.last_elem + 1) % F.M
    assert not proof.verify()


def test_pcs_prove_and_verify_oracle():
    """multilinear_pcs_bench_test (multilinear_pcs.rs:210-228) at n = 10."""
    n = 10
    ev = [F.from_i64(7 * i + 3) for i in range(1 << n)]
    pts = [F.from_i64(i) for i in range(n)]
    out = OPL.mle_evaluate(ev, pts)
    p = OP.PCSProof.prove(pts, out, ev, OT.Transcript())
    assert p.verify(OT.Transcript())


def test_interpolation_and_multilinear_conversion():
    """interpolation_test / multilinear_conversion_test (polynomials.rs:196-214)."""
    e = [F.from_i64(v) for v in [0, 1, 4, 8, 9, 3]]
    pol = OPL.interpolate(e)
    assert [OPL.uni_evaluate(pol, i) for i in range(6)] == e
    assert OPL.to_evaluation(OPL.to_coefficient(e)) == e


def test_sumcheck_rounds_consistent():
    """Each round polynomial p satisfies p(0) + p(1) = previous sum, the last
    equals delta(r) * m(r) -- the debug verifier's checks (sumcheck.rs:270-304)."""
    n = 6
    r = random.Random(3)
    ev = [r.randrange(F.M) for _ in range(1 << n)]
    pts = [r.randrange(F.M) for _ in range(n)]
    total = OPL.mle_evaluate(ev, pts)
    t = OS.SumcheckTables.build_tables_for_pcs(pts, ev)
    tr = OT.Transcript()
    prev = total
    rs = []
    for _ in range(n):
        before = prev
        nz, rr, prev = t.compute_sumcheck_polynomial(prev, tr)
        pol = OS.to_polynomial(nz, before)
        assert (OPL.uni_evaluate(pol, 0) + OPL.uni_evaluate(pol, 1)) % F.M == before
        rs.append(rr)
    assert prev == OS.delta_evaluate(pts, rs) * OPL.mle_evaluate(ev, rs) % F.M
    assert OS.eq_table(pts) == [OS.mask_evaluate(i, n, pts) for i in range(1 << n)]


# ---- golden fixtures ---------------------------------------------------------------

def _digest(values):
    return hashlib.sha256(b"".join(F.to_bytes(v) for v in values)).hexdigest()


def test_golden_field_and_ntt():
    for k, v in GOLDEN["pow_2_generator"].items():
        assert h(F.pow_2_generator(int(k))) == v
    for a, b, c in GOLDEN["mul_kat"]:
        assert h(F.mul(int(a, 16), int(b, 16))) == c
    for ln, rec in GOLDEN["ntt_coeffs_0_to_n"].items():
        ln = int(ln)
        ev = ON.ntt([F.from_i64(i) for i in range(1 << ln)], F.pow_2_generator(ln))
        assert _digest(ev) == rec["sha256"]
        assert [h(v) for v in ev[:4]] == rec["head"]


def test_golden_fri_and_pcs():
    rec = GOLDEN["fri_7i3_log10"]
    ln = 10
    vals = [F.from_i64(7 * i + 3) for i in range(1 << ln)]
    gp = F.pow_2_generator_powers(ln + 1)
    code = OF.reed_solomon(vals, gp[1])
    assert _digest(code) == rec["code_sha256"]
    proof = OF.FriProof.prove(code, gp, OT.Transcript())
    assert [c.hex() for c in proof.commitments] == rec["commitments"]
    assert h(proof.last_elem) == rec["last_elem"]
    assert proof.last_random.hex() == rec["last_random"]
    n = 10
    ev = [F.from_i64(7 * i + 3) for i in range(1 << n)]
    pts = [F.from_i64(i) for i in range(n)]
    out = OPL.mle_evaluate(ev, pts)
    assert h(out) == GOLDEN["mle_eval_7i3_point_0_to_9"]
    p = OP.PCSProof.prove(pts, out, ev, OT.Transcript())
    pr = GOLDEN["pcs_7i3_n10"]
    assert [[h(c) for c in q] for q in p.sumcheck_polynomials] == pr["sumcheck_polys"]
    assert p.fri_proof.last_random.hex() == pr["last_random"]


# ---- two independent restatements agree (Python vs C) -------------------------------

@pytest.fixture(scope="module")
def C():
    from oracle import coracle

    try:
        coracle.lib()
    except ImportError:
        pytest.skip("oracle/liboracle.so not built")
    return coracle


def test_c_oracle_matches_python(C):
    from multilinear_amd.device import ints_to_limbs, limbs_to_ints

    rnd = random.Random(11)
    for msg in (b"", b"abc", bytes(range(200))):
        assert C.sha256(msg) == hashlib.sha256(msg).digest()
    for _ in range(200):
        a, b = rnd.randrange(F.M), rnd.randrange(F.M)
        assert C.mul(a, b) == a * b % F.M
    for ln in (1, 2, 5, 9):
        x = [rnd.randrange(F.M) for _ in range(1 << ln)]
        g = F.pow_2_generator(ln)
        assert limbs_to_ints(C.ntt(ints_to_limbs(x), ln, g)) == ON.ntt(x, g)
        assert limbs_to_ints(C.ntt(ints_to_limbs(x), ln, g, True)) == ON.intt(x, g)
    ln = 8
    vals = [F.from_i64(7 * i + 3) for i in range(1 << ln)]
    gp = F.pow_2_generator_powers(ln + 1)
    code = OF.reed_solomon(vals, gp[1])
    assert limbs_to_ints(C.reed_solomon(ints_to_limbs(vals), ln, gp[1])) == code
    pd = OF.FriProverData.fold(gp, code, OT.Transcript())
    roots, last, _, rc = C.fri_commit(ints_to_limbs(code), ln + 1)
    assert rc == 0 and roots == pd.fold_roots() and last == pd.last_element
    ev = [rnd.randrange(F.M) for _ in range(1 << 7)]
    assert limbs_to_ints(C.to_coefficient(ints_to_limbs(ev), 7)) == OPL.to_coefficient(ev)
    pts = [rnd.randrange(F.M) for _ in range(7)]
    assert limbs_to_ints(C.eq_table(pts)) == OS.eq_table(pts)
    t = OS.SumcheckTables.build_tables_for_pcs(pts, ev)
    assert C.partial_sums(ints_to_limbs(ev), C.eq_table(pts), 7) == (t.partial_sum(1), t.partial_sum(2))


def test_c_oracle_intt_roundtrip_2_18(C):
    """intt_test (ntt/mod.rs:191-201) at its own size 2^18, coeffs = i."""
    import numpy as np

    from multilinear_amd.device import ints_to_limbs

    ln = 18
    x = ints_to_limbs(list(range(1 << ln)))
    g = F.pow_2_generator(ln)
    back = C.ntt(C.ntt(x, ln, g), ln, g, inverse=True)
    assert np.array_equal(back, x)


def test_trace_evaluate_oracle():
    """Trace::evaluate (evaluation.rs:31-48): each column is the MLE of that
    column (MultilinearPolynomialEvals::evaluate, polynomials.rs:165-187 uses
    the same big-endian point order); n = 1 by hand."""
    rr = random.Random(77)
    n, w = 4, 3
    mat = [rr.randrange(F.M) for _ in range(w << n)]
    pts = [rr.randrange(F.M) for _ in range(n)]
    got = OS.trace_evaluate(mat, w, pts)
    for j in range(w):
        assert got[j] == OPL.mle_evaluate(mat[j::w], pts)
    a, b, c, d, p = 3, 5, 7, 11, 13
    assert OS.trace_evaluate([a, b, c, d], 2, [p]) == [((1 - p) * a + p * c) % F.M,
                                                       ((1 - p) * b + p * d) % F.M]
    assert OS.trace_evaluate([9, 8], 2, []) == [9, 8]


def _flat_fri_queries(queries):
    return b"".join(v + b"".join(s for s, _ in path) for q in queries for v, path in q)


def _flat_batched_queries(queries):
    raw = b""
    for (col, bpath), inner in queries:
        raw += b"".join(col) + b"".join(s for s, _ in bpath)
        for value, path in inner:
            raw += value + b"".join(s for s, _ in path)
    return raw


@pytest.mark.parametrize("n,prefix", [(1, b""), (2, b""), (5, b"abc"), (8, b""), (10, b"")])
def test_c_pcs_prove_matches_python(C, n, prefix):
    """The C end-to-end PCSProof::prove (multilinear_pcs.rs:90-136) -- the
    full-size checker of the GPU prove -- against the Python restatement:
    every round polynomial, root, query record, last element and the final
    transcript digest.  n = 10 is also the golden fixture."""
    from multilinear_amd.device import ints_to_limbs

    ev = [F.from_i64(7 * i + 3) for i in range(1 << n)]
    pts = [F.from_i64(i) for i in range(n)]
    out = OPL.mle_evaluate(ev, pts)
    assert C.mle_evaluate_par(ints_to_limbs(ev), n, pts) == out
    tr = OT.Transcript()
    tr.absorb(prefix)
    want = OP.PCSProof.prove(pts, out, ev, tr)
    got = C.pcs_prove_par(ints_to_limbs(ev), n, pts, [out], prefix=prefix)
    assert got["rc"] == 0
    assert got["polys"] == [tuple(p) for p in want.sumcheck_polynomials]
    assert got["roots"] == want.fri_proof.commitments
    assert got["last_elem"] == want.fri_proof.last_elem
    assert got["last_random"] == want.fri_proof.last_random
    assert got["queries"] == _flat_fri_queries(want.fri_proof.queries)
    if n == 10 and not prefix:
        pr = GOLDEN["pcs_7i3_n10"]
        assert [[h(c) for c in q] for q in got["polys"]] == pr["sumcheck_polys"]
        assert got["last_random"].hex() == pr["last_random"]


@pytest.mark.parametrize("m,n", [(1, 1), (2, 1), (3, 5), (10, 6), (2, 8)])
def test_c_batched_pcs_prove_matches_python(C, m, n):
    """The C end-to-end BatchedPCSProof::prove (batched_pcs.rs:127-180) against
    the Python restatement, with batched_pcs_verify_test's inputs
    (batched_pcs.rs:261-306) at a small size."""
    from multilinear_amd.device import ints_to_limbs
    from oracle import batched as OB

    pts = [F.from_i64(i) for i in range(n)]
    polys = [[F.from_i64((j * 3 + i * 5) % 100) for j in range(1 << n)] for i in range(m)]
    outs = [OPL.mle_evaluate(p, pts) for p in polys]
    want = OB.BatchedPCSProof.prove(pts, outs, polys, OT.Transcript())
    got = C.pcs_prove_par(ints_to_limbs([v for p in polys for v in p]), n, pts, outs, batched=True)
    assert got["rc"] == 0
    assert got["polys"] == [tuple(p) for p in want.sumcheck_polynomials]
    assert got["batch_root"] == want.fri_proof.batch_commitment
    assert got["roots"] == want.fri_proof.commitments
    assert got["last_elem"] == want.fri_proof.last_elem
    assert got["last_random"] == want.fri_proof.last_random
    assert got["queries"] == _flat_batched_queries(want.fri_proof.queries)
