"""GPU parity: libmlhip (HIP kernels through the C ABI) vs the CPU oracle.

Bit-exact comparisons (integer field work) on seeded inputs at sizes the
Python oracle finishes in seconds, plus the reference's own test patterns
(coeffs 0..N, ntt/mod.rs:185; values 7i+3, fri/mod.rs:352 and
multilinear_pcs.rs:218) and edge cases (n = 2, non-generators, bad sizes).
"""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import field as F  # noqa: E402  (checker only)
from oracle import fri as OF  # noqa: E402
from oracle import merkle as OM  # noqa: E402
from oracle import ntt as ON  # noqa: E402
from oracle import pcs as OP  # noqa: E402
from oracle import polynomials as OPL  # noqa: E402
from oracle import sumcheck as OS  # noqa: E402
from oracle import transcript as OT  # noqa: E402

from multilinear_amd import _lib  # noqa: E402
from multilinear_amd import device as D  # noqa: E402
from multilinear_amd import fri as MF  # noqa: E402
from multilinear_amd import merkle_tree as MM  # noqa: E402
from multilinear_amd import multilinear_pcs as MP  # noqa: E402
from multilinear_amd import ntt as MN  # noqa: E402
from multilinear_amd import polynomials as MPL  # noqa: E402
from multilinear_amd import sumcheck as MS  # noqa: E402
from multilinear_amd.transcript import Transcript  # noqa: E402


def dev(values):
    return D.to_device(D.ints_to_limbs(values))


def host(t):
    return D.limbs_to_ints(D.from_device(t))


def rand_vals(n, seed):
    r = random.Random(seed)
    return [r.randrange(F.M) for _ in range(n)]


# ---- NTT -------------------------------------------------------------------

@pytest.mark.parametrize("log_n", list(range(1, 15)) + [16])
def test_ntt_matches_oracle(log_n):
    n = 1 << log_n
    g = F.pow_2_generator(log_n)
    for coeffs in ([F.from_i64(i) for i in range(n)], rand_vals(n, log_n)):
        want = ON.ntt(coeffs, g)
        got = host(MN.Polynomial(dev(coeffs)).ntt(g).evals)
        assert got == want


@pytest.mark.parametrize("log_n", [1, 2, 5, 10, 11, 12, 13, 17, 18, 19, 20])
def test_intt_roundtrip(log_n):
    """intt_test (ntt/mod.rs:191-201): INTT(NTT(x)) == x."""
    n = 1 << log_n
    g = F.pow_2_generator(log_n)
    x = D.random_device(n, 1234 + log_n)
    lag = MN.Polynomial(x).ntt(g)
    back = lag.intt().coeffs
    assert bool((back == x).all())


@pytest.mark.parametrize("log_n", [3, 11, 14])
def test_intt_matches_oracle(log_n):
    n = 1 << log_n
    g = F.pow_2_generator(log_n)
    ev = rand_vals(n, 99 + log_n)
    got = host(MN.LagrangePolynomial(g, dev(ev)).intt().coeffs)
    assert got == ON.intt(ev, g)


def test_ntt_in_place_and_host_path():
    import ctypes

    log_n = 12
    n = 1 << log_n
    g = F.pow_2_generator(log_n)
    vals = rand_vals(n, 5)
    x = dev(vals)
    ctx = D.context()
    D.check(D.lib().mlh_ntt(ctx, D.ptr(x), D.ptr(x), log_n, D.fe_bytes(g)), ctx)
    want = ON.ntt(vals, g)
    assert host(x) == want
    src = D.ints_to_limbs(vals).tobytes()
    inb = (ctypes.c_uint8 * len(src)).from_buffer_copy(src)
    outb = (ctypes.c_uint8 * len(src))()
    D.check(D.lib().mlh_ntt_host(ctx, inb, outb, log_n, D.fe_bytes(g), 0), ctx)
    assert D.limbs_to_ints(np.frombuffer(bytes(outb), dtype=np.uint32)) == want


def test_ntt_rejects_bad_inputs():
    ctx = D.context()
    x = dev(list(range(16)))
    # not a canonical field element (a generator of any order is accepted)
    st = D.lib().mlh_ntt(ctx, D.ptr(x), D.ptr(x), 4, D.fe_bytes(F.M))
    assert st == 3
    st = D.lib().mlh_ntt(ctx, D.ptr(x), D.ptr(x), 0, D.fe_bytes(1))
    assert st == 2


def _other_order_generators(log_n, seed):
    """Generators whose order is not 2^log_n (order 2N, N/2, 1; zero; -1; a
    random element): Polynomial::ntt still runs its bit-reverse + radix-2 loop
    (ntt/mod.rs:69-110), a linear map that is not a DFT, and the device's
    stage-by-stage network must give the same values."""
    return [F.pow_2_generator(log_n + 1), F.pow_2_generator(max(log_n - 1, 0)), 1, 0, F.M - 1,
            rand_vals(1, seed)[0]]


@pytest.mark.parametrize("log_n", [1, 2, 3, 6, 10, 11, 12, 13])
def test_ntt_intt_any_generator_match_oracle(log_n):
    n = 1 << log_n
    vals = rand_vals(n, 31 + log_n)
    for g in _other_order_generators(log_n, 700 + log_n):
        assert host(MN.Polynomial(dev(vals)).ntt(g).evals) == ON.ntt(vals, g), g
        assert host(MN.LagrangePolynomial(g, dev(vals)).intt().coeffs) == ON.intt(vals, g), g
        x = dev(vals)  # in place (the network's block pass goes through scratch)
        ctx = D.context()
        D.check(D.lib().mlh_ntt(ctx, D.ptr(x), D.ptr(x), log_n, D.fe_bytes(g)), ctx)
        assert host(x) == ON.ntt(vals, g), g


@pytest.mark.parametrize("log_n", [0, 1, 5, 11, 12])
def test_reed_solomon_any_generator_matches_oracle(log_n):
    n = 1 << log_n
    vals = rand_vals(n, 55 + log_n)
    perm = [int(format(i, "0%db" % log_n)[::-1], 2) if log_n else 0 for i in range(n)]
    for g in _other_order_generators(log_n + 1, 800 + log_n):
        want = OF.reed_solomon(vals, g)
        assert host(MF.reed_solomon(dev(vals), g)) == want, g
        # reed_solomon_brev(x) = reed_solomon(bit_reverse_permutation(x))
        assert host(MF.reed_solomon_brev(dev([vals[perm[i]] for i in range(n)]), g)) == want, g


@pytest.mark.parametrize("log_n", [15, 16, 20, 22])
def test_ntt_any_generator_vs_c_oracle(log_n):
    """Past the LDS block (2^11): the register stage launches (4 + 4 + 1 stages
    at 2^20), in and out of place, forward and inverse, RS with an order-N
    generator (half the 2N the code needs)."""
    C = _c_oracle()
    g = rand_vals(1, 4000 + log_n)[0]
    x = D.random_limbs(1 << log_n, 600 + log_n)
    want = C.ntt(x, log_n, g)
    assert (D.from_device(MN.Polynomial(D.to_device(x)).ntt(g).evals) == want).all()
    d = D.to_device(x)
    ctx = D.context()
    D.check(D.lib().mlh_ntt(ctx, D.ptr(d), D.ptr(d), log_n, D.fe_bytes(g)), ctx)
    assert (D.from_device(d) == want).all()
    want_i = C.ntt(x, log_n, g, inverse=True)
    assert (D.from_device(MN.LagrangePolynomial(g, D.to_device(x)).intt().coeffs) == want_i).all()
    h = F.pow_2_generator(log_n - 1)
    half = np.ascontiguousarray(x[: 1 << (log_n - 2)])
    want_rs = C.reed_solomon(half, log_n - 2, h)
    assert (D.from_device(MF.reed_solomon(D.to_device(half), h)) == want_rs).all()


def test_bit_reverse_and_generator_powers():
    for ln in (1, 2, 10):
        vals = rand_vals(1 << ln, 7 + ln)
        got = host(MN.bit_reverse_permutation(dev(vals)))
        want = list(vals)
        ON.bit_reverse_permutation(want)
        assert got == want
    with pytest.raises(_lib.MlhError) as e:  # n = 1: a panic in the reference
        MN.bit_reverse_permutation(dev([5]))
    assert e.value.status == _lib.MLH_ERR_NOT_POW2
    for ls in (3, 12, 13):
        assert host(MN.pow_2_generator_powers(ls)) == F.pow_2_generator_powers(ls)
    assert MN.pow_2_generator(40) == F.WINTER_TWO_ADIC_ROOT
    assert MN.pow_2_generator(41) is None


# ---- Reed-Solomon / Merkle ---------------------------------------------------

@pytest.mark.parametrize("log_n", [1, 4, 10, 12])
def test_reed_solomon_matches_oracle(log_n):
    n = 1 << log_n
    vals = [F.from_i64(7 * i + 3) for i in range(n)]
    g = F.pow_2_generator(log_n + 1)
    assert host(MF.reed_solomon(dev(vals), g)) == OF.reed_solomon(vals, g)


@pytest.mark.parametrize("log_code", [1, 2, 3, 9, 10, 11, 12, 13, 15, 19])
def test_merkle_commit_pairs_matches_oracle(log_code):
    """Every layer against the oracle; the sizes walk the tree tails' level
    policy: top_kernel with 64..1024 digests (pairs for n <= 256, single lanes
    above), subtree_kernel chunks below and at 2^16 digests."""
    code = rand_vals(1 << log_code, 31 + log_code)
    want = OF.commit_rs_code(code)
    got = MM.Merkle.commit_pairs(dev(code))
    assert got.root() == want.root()
    gl = got.layers()
    assert len(gl) == len(want.layers)
    for a, b in zip(gl, want.layers):
        assert [bytes(x) for x in a] == b


def test_merkle_commit_generic_items():
    """merkle_test (merkle_tree/mod.rs:300-309) data, 1-byte items."""
    data = [bytes([v]) for v in [0, 8, 4, 1, 5, 7, 6, 1]]
    got = MM.Merkle.commit(data)
    want = OM.Merkle.commit(data)
    assert got.root() == want.root()
    value, path = want.open(5)
    assert OM.verify(value, path, got.root(), 5)
    # longer items cross SHA-256 block boundaries
    items = [bytes(random.Random(i).randrange(256) for _ in range(100)) for i in range(16)]
    assert MM.Merkle.commit(items).root() == OM.Merkle.commit(items).root()


def test_merkle_open_verify_device():
    """merkle_test (merkle_tree/mod.rs:300-309): open(5) from the device tree
    equals the oracle's opening and verifies; the wrong index is an
    IncompatibleIndex, a wrong value an IncompatibleHash; past the end: None."""
    data = [bytes([v]) for v in [0, 8, 4, 1, 5, 7, 6, 1]]
    t = MM.Merkle.commit(data)
    ot = OM.Merkle.commit(data)
    for i in range(8):
        assert t.open(i) == ot.open(i)
    value, path = t.open(5)
    assert MM.verify(value, path, t.root(), 5)
    assert MM.verify_status(value, path, t.root(), 4) == _lib.STATUS_CODES["MLH_ERR_VERIFY_INDEX"]
    assert MM.verify_status(b"\x09", path, t.root(), 5) == _lib.STATUS_CODES["MLH_ERR_VERIFY"]
    assert t.open(8) is None


def test_merkle_batch_open_verify_device():
    """batched_merkle_test (merkle_tree/mod.rs:311-351)."""
    data = [[bytes([v]) for v in [0, 8, 4, 1, 5, 7, 6, 1]],
            [bytes([v]) for v in [1, 3, 2, 3, 2, 1, 2, 3]]]
    t = MM.Merkle.batch_commit(data)
    value, path = t.batch_open(5)
    assert value == [bytes([7]), bytes([1])]
    assert MM.batch_verify(value, path, t.root(), 5)
    value, path = t.batch_open(2)
    assert value == [bytes([4]), bytes([2])]
    assert MM.batch_verify(value, path, t.root(), 2)
    assert not MM.batch_verify(value, path, t.root(), 1)
    assert (value, path) == OM.batch_open(OM.Merkle.batch_commit(data), 2)


@pytest.mark.parametrize("log_code", [2, 9, 14])
def test_merkle_open_pairs_tree(log_code):
    """Merkle::open on a commit_rs_code tree vs the oracle's (fri/mod.rs:45-55)."""
    code = rand_vals(1 << log_code, 70 + log_code)
    t = MM.Merkle.commit_pairs(dev(code))
    ot = OF.commit_rs_code(code)
    for i in (0, 1, (1 << (log_code - 1)) - 1, (1 << (log_code - 2)) + 1 if log_code > 2 else 0):
        value, path = t.open(i)
        assert value == OF.pair_bytes(code[i], code[i + (1 << (log_code - 1))])
        assert [bytes(p) for p, _ in path] == [bytes(p) for p, _ in ot.open(i)[1]]
        assert MM.verify(value, path, t.root(), i)


def test_merkle_batch_commit():
    """batched_merkle_test (merkle_tree/mod.rs:311-351)."""
    data = [[bytes([v]) for v in [0, 8, 4, 1, 5, 7, 6, 1]],
            [bytes([v]) for v in [1, 3, 2, 3, 2, 1, 2, 3]]]
    assert MM.Merkle.batch_commit(data).root() == OM.Merkle.batch_commit(data).root()


# ---- FRI ---------------------------------------------------------------------

@pytest.mark.parametrize("log_domain,k", [(11, 0), (11, 3), (13, 0), (13, 11), (14, 5)])
def test_fri_fold_matches_oracle(log_domain, k):
    n = 1 << (log_domain - k)
    layer = rand_vals(n, 1000 + k)
    r = rand_vals(1, 77)[0]
    gp = F.pow_2_generator_powers(log_domain)
    pairs = [(layer[i], layer[i + n // 2]) for i in range(n // 2)]
    want = OF.fold_layer(pairs, gp, k, r)
    assert host(MF.fold_layer(dev(layer), k, log_domain, r)) == want


def _fri_oracle(log_n, vals):
    gp = F.pow_2_generator_powers(log_n + 1)
    code = OF.reed_solomon(vals, gp[1])
    return code, OF.FriProof.prove(code, gp, OT.Transcript())


@pytest.mark.parametrize("log_n", [1, 2, 5, 10])
def test_fri_prove_matches_oracle(log_n):
    """prove_and_verify_test (fri/mod.rs:349-363): values 7i+3."""
    vals = [F.from_i64(7 * i + 3) for i in range(1 << log_n)]
    code, want = _fri_oracle(log_n, vals)
    dcode = dev(code)
    got = MF.FriProof.prove(dcode, Transcript())
    assert got.commitments == want.commitments
    assert got.last_elem == want.last_elem
    assert got.last_random == want.last_random
    for q in range(_lib.NUM_QUERIES):
        gq = got.query(q)
        wq = want.queries[q]
        assert len(gq) == len(wq)
        for (gv, gs), (wv, wpath) in zip(gq, wq):
            assert gv == wv
            assert gs == [s for s, _ in wpath]
    assert got.verify()
    assert want.verify()


def test_fri_verify_rejects_tampering():
    vals = [F.from_i64(7 * i + 3) for i in range(1 << 6)]
    code, _ = _fri_oracle(6, vals)
    p = MF.FriProof.prove(dev(code), Transcript())
    assert p.verify()
    p._q[40] ^= 1
    assert not p.verify()


def test_fri_prover_step_api():
    """FriProverData::init / fold_step / open_query_at used step by step."""
    log_n = 8
    vals = rand_vals(1 << log_n, 3)
    gp = F.pow_2_generator_powers(log_n + 1)
    code = OF.reed_solomon(vals, gp[1])
    otr = OT.Transcript()
    opd = OF.FriProverData.fold(gp, code, otr)
    tr = Transcript()
    dcode = dev(code)
    pd = MF.FriProverData.init(dcode, tr)
    for k in range(log_n):
        r = tr.next_challenge()
        pd.fold_step(k, r, tr)
    assert pd.fold_roots() == opd.fold_roots()
    assert pd.last_element == opd.last_element
    assert tr.random() == otr.random()
    q = pd.open_query_at(37, log_n + 1)
    wq = opd.open_query_at(37)
    assert [v for v, _ in q] == [v for v, _ in wq]


def _step_both(opd, otr, pd, tr, gp_list, gp_arg, steps):
    """Run fold_step(gen_pows, k, r, tr) on the oracle and through
    mlh_fri_prover_fold_step_gp with the same table; compare after each step.
    Returns the step at which the oracle panicked ("not an RS code"), else None."""
    for k in range(steps):
        r = tr.next_challenge()
        assert r == otr.next_challenge()
        try:
            opd.fold_step(gp_list, k, r, otr)
        except AssertionError:
            with pytest.raises(RuntimeError, match="not an RS code"):
                pd.fold_step(k, r, tr, gen_pows=gp_arg)
            return k
        pd.fold_step(k, r, tr, gen_pows=gp_arg)
        assert pd.fold_roots() == opd.fold_roots(), k
        assert tr.random() == otr.random(), k
    return None


@pytest.mark.parametrize("log_n", [3, 8, 11])
def test_fri_prover_fold_step_gp_reference_signature(log_n):
    """The reference's step API shape: FriProverData::init(code, tr) with no
    table, then fold_step(gen_pows, k, r, tr) with one (multilinear_pcs.rs:72,
    batched_fri.rs:200, fri/mod.rs:141).  (1) the canonical table
    pow_2_generator_powers(L); (2) the table of another generator h = g^3 of
    the same order with a code built with h; (3) a 2x-length table, which the
    reference folds with g_2N^(-i 2^k) and rejects at the last layer ("not an
    RS code") -- the same step returns MLH_ERR_NOT_RS_CODE here; (4) a table
    shorter than half the code (the reference's index underflows) and a
    generator of the wrong order are rejected; (5) a step after the last
    element re-absorbs it, as the reference does."""
    L = log_n + 1
    vals = rand_vals(1 << log_n, 40 + log_n)
    g = F.pow_2_generator(L)
    for h in (g, pow(g, 3, F.M)):
        code = OF.reed_solomon(vals, h)
        gp = [pow(h, j, F.M) for j in range(1 << L)]
        otr, tr = OT.Transcript(), Transcript()
        opd = OF.FriProverData.init(code, otr)
        pd = MF.FriProverData.init(dev(code), tr)
        assert _step_both(opd, otr, pd, tr, gp, (h, L), log_n) is None
        assert pd.last_element == opd.last_element
        assert [v for v, _ in pd.open_query_at(5, L)] == [v for v, _ in opd.open_query_at(5)]
        # (5) one more step: the reference folds its last tree again
        r = tr.next_challenge()
        opd.fold_step(gp, log_n - 1, r, otr)
        pd.fold_step(log_n - 1, r, tr, gen_pows=(h, L))
        assert tr.random() == otr.random() and pd.last_element == opd.last_element
    # (3) gen_pows twice the code's length
    code = OF.reed_solomon(vals, g)
    gp2 = F.pow_2_generator_powers(L + 1)
    otr, tr = OT.Transcript(), Transcript()
    opd = OF.FriProverData.init(code, otr)
    pd = MF.FriProverData.init(dev(code), tr)
    assert _step_both(opd, otr, pd, tr, gp2, (gp2[1], L + 1), log_n) == log_n - 1
    # (4) shorter than half the code; wrong order
    lib, ctx = D.lib(), D.context()
    tr = Transcript()
    pd = MF.FriProverData.init(dev(code), tr)
    r = D.fe_bytes(tr.next_challenge())
    st = lib.mlh_fri_prover_fold_step_gp(ctx, pd.h, D.fe_bytes(F.pow_2_generator(L - 2)), L - 2, 0, r,
                                         tr.h)
    assert st == _lib.MLH_ERR_INVALID and b"underflow" in lib.mlh_last_error(ctx)
    st = lib.mlh_fri_prover_fold_step_gp(ctx, pd.h, D.fe_bytes(g * g % F.M), L, 0, r, tr.h)
    assert st == _lib.MLH_ERR_BAD_GENERATOR
    assert pd.fold_roots() == [OF.commit_rs_code(code).root()]  # rejected steps left no layer


@pytest.mark.parametrize("nq", [1, 5, 128, 129, 300])
def test_fri_prover_open_queries_many(nq):
    """mlh_fri_prover_open_queries: indices in the kernel arguments (<= 128)
    or in device memory (> 128); duplicates and both ends of the range."""
    log_n = 9
    vals = rand_vals(1 << log_n, 5)
    gp = F.pow_2_generator_powers(log_n + 1)
    code = OF.reed_solomon(vals, gp[1])
    opd = OF.FriProverData.fold(gp, code, OT.Transcript())
    pd = MF.FriProverData.fold(dev(code), Transcript())
    rng = random.Random(nq)
    half = 1 << log_n
    idx = [rng.randrange(half) for _ in range(nq)]
    idx[0] = half - 1
    if nq > 2:
        idx[1] = 0
        idx[2] = idx[0]
    got = pd.open_queries(idx, log_n + 1)
    for i, q in zip(idx, got):
        want = opd.open_query_at(i)
        assert [v for v, _ in q] == [v for v, _ in want]
        assert [s for _, s in q] == [[s for s, _ in path] for _, path in want]
    with pytest.raises(_lib.MlhError):
        pd.open_queries(idx[:-1] + [half], log_n + 1)


def test_fri_not_rs_code():
    """fold of a non-codeword hits the reference's "not an RS code" assert."""
    log_code = 6
    code = rand_vals(1 << log_code, 11)
    with pytest.raises(_lib.MlhError) as e:
        MF.FriProof.prove(dev(code), Transcript())
    assert e.value.status == 6


# ---- multilinear / sumcheck / PCS -------------------------------------------

@pytest.mark.parametrize("log_n", [1, 3, 8, 11, 17])
def test_mobius_and_zeta(log_n):
    ev = rand_vals(1 << log_n, 50 + log_n)
    dv = dev(ev)
    c = MPL.to_coefficient(dv)
    if log_n <= 11:
        assert host(c) == OPL.to_coefficient(ev)
    assert bool((MPL.to_evaluation(c) == dv).all())


@pytest.mark.parametrize("vals", [[0, 1, 4, 8, 9, 3], [5], [2, 7, 1, 8, 2, 8, 1, 8, 2, 8, 4, 5]])
def test_mle_conversion_any_length(vals):
    """multilinear_conversion_test (polynomials.rs:206-214): 6 evals, not 2^k --
    only the low trailing_zeros(len) index bits are transformed."""
    ev = [F.from_i64(v) for v in vals]
    c = MPL.to_coefficient(dev(ev))
    assert host(c) == OPL.to_coefficient(ev)
    assert host(MPL.to_evaluation(c)) == ev


@pytest.mark.parametrize("n", [0, 1, 5, 4096, 4097, 12345, 1 << 18])
def test_poly_evaluate_matches_horner(n):
    """Polynomial::evaluate (ntt/mod.rs:61-67): sum c_i x^i on the GPU equals
    the oracle's Horner fold."""
    c = rand_vals(n, 80 + n % 97)
    x = rand_vals(1, 81)[0]
    t = dev(c) if n else D.empty(0)
    assert MN.Polynomial(t).evaluate(x) == OPL.uni_evaluate(c, x)


@pytest.mark.parametrize("m,n", [(1, 0), (2, 1), (6, 3), (8, 3), (1 << 10, 10), (1000, 10)])
def test_mle_evaluations_any_length(m, n):
    """MultilinearPolynomial::evaluate (coefficient form, polynomials.rs:126-146)
    and MultilinearPolynomialEvals::evaluate (:165-187) for len <= 2^n with
    len.next_power_of_two() == 2^n."""
    v = rand_vals(m, 90 + m)
    args = rand_vals(n, 91 + n)
    assert MPL.coeffs_evaluate(dev(v), args) == OPL.mle_coeffs_evaluate(v, args)
    assert MPL.evaluate(dev(v), args) == OPL.mle_evaluate(v, args)
    with pytest.raises(ValueError):
        MPL.evaluate(dev(v), args + [1])


def test_mle_coefficient_and_evaluation_forms_agree():
    """2^16: evaluate(evals) == coeffs_evaluate(to_coefficient(evals)) on the GPU."""
    n = 16
    ev = D.random_device(1 << n, 92)
    args = rand_vals(n, 93)
    assert MPL.coeffs_evaluate(MPL.to_coefficient(ev), args) == MPL.evaluate(ev, args)


def test_eq_table_and_evaluate():
    for n in (1, 2, 5, 9, 12):
        pts = rand_vals(n, 600 + n)
        assert host(MPL.eq_table(pts)) == OS.eq_table(pts)
        assert OS.eq_table(pts)[: 1 << min(n, 4)] == [OS.mask_evaluate(i, n, pts) for i in range(1 << min(n, 4))]
    n = 10
    ev = rand_vals(1 << n, 4)
    args = rand_vals(n, 5)
    assert MPL.evaluate(dev(ev), args) == OPL.mle_evaluate(ev, args)


@pytest.mark.parametrize("n,w", [(0, 1), (0, 5), (3, 1), (5, 3), (10, 7), (6, 300), (4, 513)])
def test_trace_evaluate_matches_oracle(n, w):
    """Trace::evaluate (evaluation.rs:31-48); w > 256 runs several column chunks."""
    mat = rand_vals(w << n, 40 + w)
    pts = rand_vals(n, 41)
    assert MPL.trace_evaluate(dev(mat), w, pts) == OS.trace_evaluate(mat, w, pts)


def test_trace_evaluate_large_vs_column_mles():
    """2^20 x 4 trace: each column equals the device MLE evaluate of it."""
    n, w = 20, 4
    m = D.random_device(w << n, 42)
    pts = rand_vals(n, 43)
    got = MPL.trace_evaluate(m, w, pts)
    cols = m.view(-1, w, 4)
    for j in range(w):
        assert got[j] == MPL.evaluate(cols[:, j, :].contiguous(), pts)
    with pytest.raises(ValueError):
        MPL.trace_evaluate(m, w, pts[:-1])


def test_sumcheck_rounds_match_oracle():
    n = 10
    ev = rand_vals(1 << n, 8)
    pts = rand_vals(n, 9)
    ot = OS.SumcheckTables.build_tables_for_pcs(pts, ev)
    mt = MS.SumcheckTables.build_tables_for_pcs(pts, dev(ev))
    assert mt.partial_sums() == (ot.partial_sum(1), ot.partial_sum(2))
    r = rand_vals(1, 10)[0]
    ot.fold(r)
    mt.fold(r)
    assert host(mt.matrix)[: 1 << (n - 1)] == ot.matrix
    assert host(mt.delta)[: 1 << (n - 1)] == ot.delta
    assert mt.partial_sums() == (ot.partial_sum(1), ot.partial_sum(2))
    # full prove against the oracle's round loop
    total = OPL.mle_evaluate(ev, pts)
    ot2 = OS.SumcheckTables.build_tables_for_pcs(pts, ev)
    otr = OT.Transcript()
    prev = total
    want_polys, want_rs = [], []
    for _ in range(n):
        nz, r2, prev = ot2.compute_sumcheck_polynomial(prev, otr)
        want_polys.append(tuple(nz))
        want_rs.append(r2)
    mt2 = MS.SumcheckTables.build_tables_for_pcs(pts, dev(ev))
    tr = Transcript()
    polys, rs = mt2.compute_sumcheck_polynomials(total, tr)
    assert polys == want_polys
    assert rs == want_rs
    assert tr.random() == otr.random()


@pytest.mark.parametrize("factored", [True, "inplace", False])
@pytest.mark.parametrize("n", [1, 2, 12, 13, 15, 16])
def test_sumcheck_prove_matches_oracle(n, factored):
    """Device-resident prove around the LDS tail (sumcheck_tail_kernel takes the
    last min(n, 12) rounds): polys, challenges, transcript and the folded
    tables (in place, as SumcheckTables::fold leaves them) vs the oracle.
    factored: fresh build_tables_for_pcs tables (mlh_sumcheck_prove_eq: delta
    kept as c_k * eq(p_k..) for the first n - 12 rounds; the first fold reads
    the evaluations, which stay unmodified); "inplace": the same with the
    matrix clone made first and folded in place; False: the delta table is
    materialised first (mlh_sumcheck_prove, two-table rounds)."""
    ev = rand_vals(1 << n, 60 + n)
    pts = rand_vals(n, 61 + n)
    total = OPL.mle_evaluate(ev, pts)
    ot = OS.SumcheckTables.build_tables_for_pcs(pts, ev)
    otr = OT.Transcript()
    otr.absorb(b"tail")
    prev, want_polys, want_rs = total, [], []
    for _ in range(n):
        nz, r2, prev = ot.compute_sumcheck_polynomial(prev, otr)
        want_polys.append(tuple(nz))
        want_rs.append(r2)
    evd = dev(ev)
    mt = MS.SumcheckTables.build_tables_for_pcs(pts, evd)
    if not factored:
        mt.delta  # noqa: B018 -- materialise the eq table
    if factored == "inplace":
        mt.matrix  # noqa: B018 -- materialise the matrix clone
    tr = Transcript()
    tr.absorb(b"tail")
    polys, rs = mt.compute_sumcheck_polynomials(total, tr)
    assert polys == want_polys and rs == want_rs
    assert tr.random() == otr.random()
    assert host(mt.matrix)[0] == ot.matrix[0] and host(mt.delta)[0] == ot.delta[0]
    assert host(evd) == ev  # build_tables_for_pcs clones: the evaluations are untouched


@pytest.mark.parametrize("label", [b"abc", b"x" * 33, b""])
@pytest.mark.parametrize("n", [3, 14, 18])
def test_sumcheck_prove_eq_transcript_alignments(n, label):
    """The device transcript's word path needs len % 4 == 0; a 3- or 33-byte
    prefix sends every absorb of the prove (head groups, eq tail) through the
    byte path, and an empty one makes every other challenge a padding-only
    block (the precomputed K + W tables).  Round polynomials, challenges and the
    final transcript state vs the oracle."""
    ev = rand_vals(1 << n, 90 + n)
    pts = rand_vals(n, 91 + n)
    total = OPL.mle_evaluate(ev, pts)
    ot = OS.SumcheckTables.build_tables_for_pcs(pts, ev)
    otr = OT.Transcript()
    otr.absorb(label)
    prev, want_polys, want_rs = total, [], []
    for _ in range(n):
        nz, r2, prev = ot.compute_sumcheck_polynomial(prev, otr)
        want_polys.append(tuple(nz))
        want_rs.append(r2)
    mt = MS.SumcheckTables.build_tables_for_pcs(pts, dev(ev))
    tr = Transcript()
    tr.absorb(label)
    polys, rs = mt.compute_sumcheck_polynomials(total, tr)
    assert polys == want_polys and rs == want_rs
    assert tr.random() == otr.random()


@pytest.mark.parametrize("n", [1, 2, 8, 10, 13, 14, 16, 17])
def test_pcs_prove_matches_oracle(n):
    """multilinear_pcs_bench_test pattern: evals 7i+3, point (0..n)."""
    ev = [F.from_i64(7 * i + 3) for i in range(1 << n)]
    inputs = [F.from_i64(i) for i in range(n)]
    out = OPL.mle_evaluate(ev, inputs)
    want = OP.PCSProof.prove(inputs, out, ev, OT.Transcript())
    got = MP.PCSProof.prove(inputs, out, dev(ev), Transcript())
    assert got.sumcheck_polynomials == [tuple(p) for p in want.sumcheck_polynomials]
    assert got.fri_proof.commitments == want.fri_proof.commitments
    assert got.fri_proof.last_elem == want.fri_proof.last_elem
    assert got.fri_proof.last_random == want.fri_proof.last_random
    assert got.verify(Transcript())
    assert want.verify(OT.Transcript())


def test_pcs_random_point():
    n = 9
    ev = rand_vals(1 << n, 21)
    inputs = rand_vals(n, 22)
    out = OPL.mle_evaluate(ev, inputs)
    got = MP.PCSProof.prove(inputs, out, dev(ev), Transcript())
    want = OP.PCSProof.prove(inputs, out, ev, OT.Transcript())
    assert got.fri_proof.last_random == want.fri_proof.last_random
    assert got.verify(Transcript())
    # wrong claimed output -> verifier rejects
    bad = MP.PCSProof.prove(inputs, (out + 1) % F.M, dev(ev), Transcript())
    assert not bad.verify(Transcript())


def test_pcs_random_point_factored_rounds():
    """n = 15: three eq-factored sumcheck rounds before delta is materialised."""
    n = 15
    ev = rand_vals(1 << n, 23)
    inputs = rand_vals(n, 24)
    out = OPL.mle_evaluate(ev, inputs)
    got = MP.PCSProof.prove(inputs, out, dev(ev), Transcript())
    want = OP.PCSProof.prove(inputs, out, ev, OT.Transcript())
    assert got.sumcheck_polynomials == [tuple(p) for p in want.sumcheck_polynomials]
    assert got.fri_proof.last_random == want.fri_proof.last_random
    assert got.verify(Transcript())


# ---- full-size properties (BASELINE configs) ----------------------------------

def test_sumcheck_factored_equals_two_table_full_size():
    """Config 4 size class (2^22 here): the eq-factored prove and the two-table
    prove over the materialised eq table give the same round polynomials,
    challenges, transcript, folded matrix and folded delta."""
    n = 22
    x = D.random_device(1 << n, 77)
    pts = rand_vals(n, 78)
    total = MPL.evaluate(x, pts)
    a = MS.SumcheckTables.build_tables_for_pcs(pts, x)
    b = MS.SumcheckTables.build_tables_for_pcs(pts, x)
    b.delta  # noqa: B018
    ta, tb = Transcript(), Transcript()
    pa, ra = a.compute_sumcheck_polynomials(total, ta)
    pb, rb = b.compute_sumcheck_polynomials(total, tb)
    assert pa == pb and ra == rb
    assert ta.random() == tb.random()
    assert host(a.matrix)[0] == host(b.matrix)[0]
    assert host(a.delta)[0] == host(b.delta)[0]
    import torch

    assert torch.equal(x, D.random_device(1 << n, 77))  # the evaluations are untouched
    # the round chain closes: p_k(0) + p_k(1) = previous claim (c0 = e0 here)
    prev = total
    for (c1, c2), r in zip(pa, ra):
        e0 = (prev - (c1 + c2)) * pow(2, -1, F.M) % F.M
        prev = (e0 + r * (c1 + c2 * r)) % F.M
    assert prev == host(a.matrix)[0] * host(a.delta)[0] % F.M


def _sum_mod(t):
    a = D.from_device(t).astype(np.uint64)
    s = [int(a[:, i].sum()) for i in range(4)]
    return (s[0] + (s[1] << 32) + (s[2] << 64) + (s[3] << 96)) % F.M


def _alt_sum_mod(t):
    a = D.from_device(t).astype(np.uint64)
    ev, od = a[0::2], a[1::2]
    s = [int(ev[:, i].sum()) - int(od[:, i].sum()) for i in range(4)]
    return (s[0] + (s[1] << 32) + (s[2] << 64) + (s[3] << 96)) % F.M


@pytest.mark.slow
def test_ntt_2_24_properties():
    """Config 2: 2^24 forward + inverse, bit-exact round trip; evals[0] =
    sum(c), evals[N/2] = alternating sum (size-independent identities)."""
    log_n = 24
    g = F.pow_2_generator(log_n)
    x = D.random_device(1 << log_n, 2024)
    ev = MN.Polynomial(x).ntt(g).evals
    e = D.from_device(ev[[0, 1 << (log_n - 1)]])
    vals = D.limbs_to_ints(e)
    assert vals[0] == _sum_mod(x)
    assert vals[1] == _alt_sum_mod(x)
    back = MN.LagrangePolynomial(g, ev).intt().coeffs
    assert bool((back == x).all())


def _const_device(v, n):
    import torch

    row = D.ints_to_limbs([v])
    return D.to_device(np.tile(row, (n, 1))) if n else torch.empty((0, 4), dtype=torch.int32)


@pytest.mark.parametrize("log_n", [11, 20, 24])
def test_ntt_extreme_values(log_n):
    """Operands at the top of the canonical range, which the uniform generator
    (top limb <= 0xFFFFFFFE) never produces and random intermediates reach with
    probability ~2^-32: all coefficients M-1 -> (N(M-1), 0, ..., 0); a single
    M-1 at index 1 -> -g^i; both round-trip through the INTT; Reed-Solomon of
    a single M-1 at index 0 is the constant codeword, at index 1 it is -g2^i."""
    import torch

    lib = _lib.load()
    ctx = D.context(0)
    n = 1 << log_n
    top = F.M - 1
    g = F.pow_2_generator(log_n)
    x = _const_device(top, n)
    ev = MN.Polynomial(x).ntt(g).evals
    assert D.limbs_to_ints(D.from_device(ev[:1]))[0] == n * top % F.M
    assert bool((ev[1:] == 0).all())
    assert bool((MN.LagrangePolynomial(g, ev).intt().coeffs == x).all())
    # single M-1 at index 1: evals[i] = -g^i
    d = torch.zeros_like(x)
    d[1] = x[0]
    ev = MN.Polynomial(d).ntt(g).evals
    gp = MN.pow_2_generator_powers(log_n)
    want = torch.empty_like(gp)
    D.check(lib.mlh_field_neg(ctx, D.ptr(gp), D.ptr(want), n), ctx)
    assert bool((ev == want).all())
    assert bool((MN.LagrangePolynomial(g, ev).intt().coeffs == d).all())
    # Reed-Solomon (implicit zero upper half in pass 0)
    g2 = F.pow_2_generator(log_n + 1)
    e0 = torch.zeros_like(x)
    e0[0] = x[0]
    assert bool((MF.reed_solomon(e0, g2) == _const_device(top, 2 * n)).all())
    code = MF.reed_solomon(d, g2)
    gp2 = MN.pow_2_generator_powers(log_n + 1)
    want2 = torch.empty_like(gp2)
    D.check(lib.mlh_field_neg(ctx, D.ptr(gp2), D.ptr(want2), 2 * n), ctx)
    assert bool((code == want2).all())


@pytest.mark.parametrize("log_n", [12, 16])
def test_ntt_near_modulus_inputs_match_oracle(log_n):
    """Random inputs drawn from the top of the range, M - 1 - u with u < 2^64
    (mixed with zeros and small values), vs the oracle: forward, inverse, RS."""
    rr = random.Random(900 + log_n)
    n = 1 << log_n
    vals = [rr.choice([F.M - 1 - rr.randrange(1 << 64), F.M - 1, 0, 1, rr.randrange(1 << 64)])
            for _ in range(n)]
    g = F.pow_2_generator(log_n)
    got = host(MN.Polynomial(dev(vals)).ntt(g).evals)
    want = ON.ntt(vals, g)
    assert got == want
    assert host(MN.LagrangePolynomial(g, dev(want)).intt().coeffs) == vals
    g2 = F.pow_2_generator(log_n + 1)
    assert host(MF.reed_solomon(dev(vals), g2)) == OF.reed_solomon(vals, g2)


def test_fri_and_sumcheck_extreme_values_match_oracle():
    """FRI prove of the RS codeword of the all-(M-1) coefficient vector and of
    near-modulus random coefficients, and an eq-factored sumcheck with M-1
    evaluations and points, vs the oracle (roots, last element, transcript,
    round polynomials)."""
    top = F.M - 1
    ln = 10
    g = F.pow_2_generator(ln + 1)
    rr = random.Random(77)
    for coeffs in ([top] * (1 << ln),
                   [F.M - 1 - rr.randrange(1 << 64) for _ in range(1 << ln)]):
        code = OF.reed_solomon(coeffs, g)
        want = OF.FriProof.prove(code, F.pow_2_generator_powers(ln + 1), OT.Transcript())
        got = MF.FriProof.prove(dev(code), Transcript())
        assert got.commitments == want.commitments
        assert got.last_elem == want.last_elem and got.last_random == want.last_random
        assert got.verify()
    n = 13
    ev = [top] * (1 << n)
    pts = [top] * n
    total = OPL.mle_evaluate(ev, pts)
    ot = OS.SumcheckTables.build_tables_for_pcs(pts, ev)
    otr = OT.Transcript()
    prev, want_polys = total, []
    for _ in range(n):
        nz, _r, prev = ot.compute_sumcheck_polynomial(prev, otr)
        want_polys.append(tuple(nz))
    polys, _rs = MS.SumcheckTables.build_tables_for_pcs(pts, dev(ev)).compute_sumcheck_polynomials(
        total, Transcript())
    assert polys == want_polys


@pytest.mark.slow
def test_fri_commit_2_24_verifies():
    """Config 3 shape: 2^24 coefficients -> RS code 2^25 -> full FRI prove,
    accepted by the verifier; code[0] == sum(coeffs)."""
    log_n = 24
    x = D.random_device(1 << log_n, 77)
    g = F.pow_2_generator(log_n + 1)
    code = MF.reed_solomon(x, g)
    assert D.limbs_to_ints(D.from_device(code[:1]))[0] == _sum_mod(x)
    p = MF.FriProof.prove(code, Transcript())
    assert p.verify()


@pytest.mark.parametrize("plan", ["4,4,4", "4,8,4", "8,4,4", "4,4,8", "5,5,5", "4,9,4",
                                  "4,4,4,4", "6,5,4"])
def test_ntt_forced_radix_plans(plan):
    """Every pass shape (first / middle / last, radix 2^4..2^9, 3-4 passes) at
    oracle-sized N via the mlh_set_ntt_plan test hook."""
    with D.ntt_plan(plan):
        _forced_plan_vs_python_oracle(plan)


def _forced_plan_vs_python_oracle(plan):
    log_n = sum(int(v) for v in plan.split(","))
    n = 1 << log_n
    g = F.pow_2_generator(log_n)
    vals = rand_vals(n, 4242 + log_n)
    got = MN.Polynomial(dev(vals)).ntt(g)
    assert host(got.evals) == ON.ntt(vals, g)
    assert host(got.intt().coeffs) == vals
    # RS LDE (zero-padded first pass) with the same plan on 2^log_n outputs
    half = vals[: n // 2]
    assert host(MF.reed_solomon(dev(half), g)) == OF.reed_solomon(half, g)


# ---- full-size parity against the C restatement of the reference loops ---------

def _c_oracle():
    from oracle import coracle

    coracle.lib()
    return coracle


@pytest.mark.parametrize("log_n", [15, 17, 19, 20, 21, 22, 23,
                                   pytest.param(24, marks=pytest.mark.slow)])
def test_ntt_vs_c_oracle(log_n):
    C = _c_oracle()
    g = F.pow_2_generator(log_n)
    x = D.random_limbs(1 << log_n, 900 + log_n)
    want = C.ntt(x, log_n, g)
    got = D.from_device(MN.Polynomial(D.to_device(x)).ntt(g).evals)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, "first mismatches at %s of %d" % (bad[:8].tolist(), bad.size)


@pytest.mark.parametrize("log_n", [18, 21])
def test_intt_vs_c_oracle(log_n):
    C = _c_oracle()
    g = F.pow_2_generator(log_n)
    x = D.random_limbs(1 << log_n, 300 + log_n)
    want = C.ntt(x, log_n, g, inverse=True)
    got = D.from_device(MN.LagrangePolynomial(g, D.to_device(x)).intt().coeffs)
    assert (got == want).all()


@pytest.mark.parametrize("log_n", [17, 20])
def test_reed_solomon_and_fri_commit_vs_c_oracle(log_n):
    C = _c_oracle()
    g = F.pow_2_generator(log_n + 1)
    x = D.random_limbs(1 << log_n, 500 + log_n)
    want = C.reed_solomon(x, log_n, g)
    dcode = MF.reed_solomon(D.to_device(x), g)
    assert (D.from_device(dcode) == want).all()
    roots, last, lr, rc = C.fri_commit(want, log_n + 1)
    assert rc == 0
    pd = MF.FriProverData.fold(dcode, Transcript())
    assert pd.fold_roots() == roots
    assert pd.last_element == last


@pytest.mark.parametrize("plan", ["9,4,4", "9,5,4", "4,4,9", "9,9,4", "7,7,7", "9,8,4", "5,5,5,5"])
def test_forced_plans_vs_c_oracle(plan):
    """Radix-2^9 first passes (the default 2^25 plan 9,8,8 starts with one) and
    every zero-top mode against the C oracle: NTT (pass 0 <9,3,0>), INTT, RS
    (<9,3,1>: implicit zero half) and RS of bit-reversed coefficients (<9,3,2>,
    the PCS path), at the plan's size."""
    with D.ntt_plan(plan):
        _forced_plan_vs_c_oracle(plan)


def _forced_plan_vs_c_oracle(plan):
    C = _c_oracle()
    log_n = sum(int(v) for v in plan.split(","))
    g = F.pow_2_generator(log_n)
    x = D.random_limbs(1 << log_n, 1700 + log_n)
    assert (D.from_device(MN.Polynomial(D.to_device(x)).ntt(g).evals) == C.ntt(x, log_n, g)).all()
    assert (D.from_device(MN.LagrangePolynomial(g, D.to_device(x)).intt().coeffs)
            == C.ntt(x, log_n, g, inverse=True)).all()
    half = np.ascontiguousarray(x[: 1 << (log_n - 1)])
    want = C.reed_solomon(half, log_n - 1, g)
    assert (D.from_device(MF.reed_solomon(D.to_device(half), g)) == want).all()
    perm = np.array([int(format(i, "0%db" % (log_n - 1))[::-1], 2) for i in range(1 << (log_n - 1))])
    brev = np.ascontiguousarray(half[perm])
    assert (D.from_device(MF.reed_solomon_brev(D.to_device(brev), g)) == want).all()


def _bitrev_perm(bits):
    i = np.arange(1 << bits, dtype=np.uint64)
    r = np.zeros_like(i)
    for b in range(bits):
        r |= ((i >> np.uint64(b)) & np.uint64(1)) << np.uint64(bits - 1 - b)
    return r.astype(np.int64)


@pytest.mark.parametrize("log_n", [23, pytest.param(24, marks=pytest.mark.slow)])
def test_default_plan_pass0_progression_vs_c_oracle(log_n):
    """2^23 and 2^24 (default plans 8,8,7 and 8,8,8): pass 0's inter-pass
    twiddle, too big for one table, runs as the progression P[k0][j] C[j]^i
    (ntt_pass_kernel TW 5) in every zero-top mode -- NTT, INTT (the n^-1 scale
    in P), RS of 2^(n-1) coefficients (implicit zero half) and RS of the
    bit-reversed coefficients (the PCS path) -- against the C oracle."""
    C = _c_oracle()
    g = F.pow_2_generator(log_n)
    x = D.random_limbs(1 << log_n, 2300 + log_n)
    assert (D.from_device(MN.Polynomial(D.to_device(x)).ntt(g).evals) == C.ntt(x, log_n, g)).all()
    assert (D.from_device(MN.LagrangePolynomial(g, D.to_device(x)).intt().coeffs)
            == C.ntt(x, log_n, g, inverse=True)).all()
    half = np.ascontiguousarray(x[: 1 << (log_n - 1)])
    want = C.reed_solomon(half, log_n - 1, g)
    assert (D.from_device(MF.reed_solomon(D.to_device(half), g)) == want).all()
    brev = np.ascontiguousarray(half[_bitrev_perm(log_n - 1)])
    assert (D.from_device(MF.reed_solomon_brev(D.to_device(brev), g)) == want).all()


@pytest.mark.parametrize("log_n", [0, 1, 4, 9, 10, 11, 13, 17, 20])
def test_reed_solomon_brev_vs_c_oracle(log_n):
    """Fused bit reversal (ZT == 2 pass-0 loads / small-kernel path) against
    the C oracle's reed_solomon of the explicitly permuted coefficients."""
    C = _c_oracle()
    n = 1 << log_n
    g = F.pow_2_generator(log_n + 1)
    x = D.random_limbs(n, 900 + log_n)
    perm = np.array([int(format(i, "0%db" % log_n)[::-1], 2) if log_n else 0 for i in range(n)])
    want = C.reed_solomon(np.ascontiguousarray(x[perm]), log_n, g)
    got = D.from_device(MF.reed_solomon_brev(D.to_device(x), g))
    assert (got == want).all()


# ---- GPU against the committed golden fixtures ---------------------------------

def _golden():
    import json
    import os

    return json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def _digest(values):
    import hashlib

    return hashlib.sha256(b"".join(F.to_bytes(v) for v in values)).hexdigest()


def test_gpu_matches_golden_fixtures():
    G = _golden()
    for ln, rec in G["ntt_coeffs_0_to_n"].items():
        ln = int(ln)
        ev = host(MN.Polynomial(dev([F.from_i64(i) for i in range(1 << ln)])).ntt(F.pow_2_generator(ln)).evals)
        assert _digest(ev) == rec["sha256"]
    rec = G["fri_7i3_log10"]
    vals = [F.from_i64(7 * i + 3) for i in range(1 << 10)]
    code = MF.reed_solomon(dev(vals), F.pow_2_generator(11))
    assert _digest(host(code)) == rec["code_sha256"]
    p = MF.FriProof.prove(code, Transcript())
    assert [c.hex() for c in p.commitments] == rec["commitments"]
    assert "%032x" % p.last_elem == rec["last_elem"]
    assert p.last_random.hex() == rec["last_random"]
    n = 10
    ev = [F.from_i64(7 * i + 3) for i in range(1 << n)]
    pts = [F.from_i64(i) for i in range(n)]
    out = MPL.evaluate(dev(ev), pts)
    assert "%032x" % out == G["mle_eval_7i3_point_0_to_9"]
    pc = MP.PCSProof.prove(pts, out, dev(ev), Transcript())
    pr = G["pcs_7i3_n10"]
    assert [["%032x" % c for c in q] for q in pc.sumcheck_polynomials] == pr["sumcheck_polys"]
    assert [c.hex() for c in pc.fri_proof.commitments] == pr["commitments"]
    assert pc.fri_proof.last_random.hex() == pr["last_random"]


# ---- field arithmetic on adversarial operands ------------------------------------

def _edge_values():
    """Limb patterns that stress every carry path of the 128x128 product and
    the 2^128 = C folds: all-ones limbs, values just below M, powers of two."""
    vals = [0, 1, 2, F.M - 1, F.M - 2, (F.M - 1) // 2, (F.M + 1) // 2, 2**127, 2**96, 2**64 - 1,
            2**96 - 1, 2**128 - 2**96 - 1, F.M - 2**64, F.M - 2**32, 0x2CFFFFFFFFFF, 0x2D0000000000]
    for top in (0xFFFFFFFE, 0xFFFFFFFF):
        for mid in (0xFFFFFFFF, 0xFFFFD2FF, 0xFFFFD300, 0):
            v = (top << 96) | (mid << 64) | (0xFFFFFFFF << 32) | 0xFFFFFFFF
            if v < F.M:
                vals.append(v)
    r = random.Random(77)
    for _ in range(64):  # near-M and dense-ones randoms
        vals.append(F.M - 1 - r.randrange(2**48))
        v = sum((0xFFFFFFFF if r.random() < 0.8 else r.randrange(2**32)) << (32 * i) for i in range(4))
        vals.append(v % F.M)
    return [v % F.M for v in vals]


def test_field_ops_adversarial():
    ev = _edge_values()
    a = [x for x in ev for _ in ev]
    b = [y for _ in ev for y in ev]
    da, db = dev(a), dev(b)
    out = D.empty(len(a))
    ctx = D.context()
    lib = D.lib()
    for fn, py in ((lib.mlh_field_mul, lambda x, y: x * y % F.M),
                   (lib.mlh_field_add, lambda x, y: (x + y) % F.M),
                   (lib.mlh_field_sub, lambda x, y: (x - y) % F.M)):
        D.check(fn(ctx, D.ptr(da), D.ptr(db), D.ptr(out), len(a)), ctx)
        got = host(out)
        want = [py(x, y) for x, y in zip(a, b)]
        bad = [i for i in range(len(a)) if got[i] != want[i]]
        assert not bad, (fn.__name__, len(bad), hex(a[bad[0]]), hex(b[bad[0]]))
    D.check(lib.mlh_field_neg(ctx, D.ptr(da), D.ptr(out), len(a)), ctx)
    assert host(out) == [(-x) % F.M for x in a]


def test_field_mul_random_bulk():
    n = 1 << 20
    x = D.random_limbs(n, 5)
    y = D.random_limbs(n, 6)
    out = D.empty(n)
    ctx = D.context()
    dx, dy = D.to_device(x), D.to_device(y)  # keep the tensors alive across the call
    D.check(D.lib().mlh_field_mul(ctx, D.ptr(dx), D.ptr(dy), D.ptr(out), n), ctx)
    got = D.from_device(out)
    xi, yi, gi = D.limbs_to_ints(x[:4096]), D.limbs_to_ints(y[:4096]), D.limbs_to_ints(got[:4096])
    assert gi == [p * q % F.M for p, q in zip(xi, yi)]
    from oracle import coracle

    coracle.lib()
    for i in range(0, n, 997):
        assert D.limbs_to_ints(got[i:i + 1])[0] == coracle.mul(D.limbs_to_ints(x[i:i + 1])[0],
                                                                 D.limbs_to_ints(y[i:i + 1])[0])


@pytest.mark.parametrize("log_n", [5, 9])
def test_fri_proof_wire_bytes_match_oracle(log_n):
    """GPU proof -> bincode bytes (mlh_fri_proof_encode) == the oracle's
    encoding of its own proof of the same code; decode round-trips."""
    from oracle import wire as OW

    vals = [F.from_i64(7 * i + 3) for i in range(1 << log_n)]
    gp = F.pow_2_generator_powers(log_n + 1)
    code = OF.reed_solomon(vals, gp[1])
    want = OW.encode_fri_proof(OF.FriProof.prove(code, gp, OT.Transcript()))
    p = MF.FriProof.prove(dev(code), Transcript())
    got = p.to_bytes()
    assert got == want
    q = MF.FriProof.from_bytes(got)
    assert q.verify() and q.to_bytes() == got and q.query_indices == p.query_indices


# ---- batched FRI / batched PCS (src/fri/batched_fri.rs, batched_pcs.rs) ------

def _flat_batched_queries(proof):
    raw = b""
    for (col, bpath), inner in proof.queries:
        raw += b"".join(col) + b"".join(s for s, _ in bpath)
        for value, path in inner:
            raw += value + b"".join(s for s, _ in path)
    return raw


@pytest.mark.parametrize("m,log_n", [(1, 4), (4, 6), (3, 9), (2, 1), (5, 2)])
def test_batched_fri_prove_matches_oracle(m, log_n):
    from multilinear_amd.batched import BatchedFriProof
    from oracle import batched as OB

    gp = F.pow_2_generator_powers(log_n + 1)
    codes = [OF.reed_solomon([F.from_i64(7 * i + 3 + 100 * j) for i in range(1 << log_n)], gp[1])
             for j in range(m)]
    want = OB.BatchedFriProof.prove(codes, gp, OT.Transcript())
    got = BatchedFriProof.prove(dev([v for c in codes for v in c]), m, Transcript())
    assert got.batch_commitment == want.batch_commitment
    assert got.commitments == want.commitments
    assert got.last_elem == want.last_elem and got.last_random == want.last_random
    assert bytes(got._q) == _flat_batched_queries(want)
    assert got.verify()


@pytest.mark.parametrize("m,log_n", [(3, 6), (1, 3), (2, 1), (4, 10), (10, 2)])
def test_batched_fri_prover_step_api_reference_shape(m, log_n):
    """BatchedFriProverData::fold (batched_fri.rs:178-205) written as the
    reference writes it, through the step API: init; r = next_challenge;
    batched_fold_step(gen_pows, r, tr); then fri_data.fold_step(gen_pows, k, r,
    tr) for k >= 1 (:200) on the inner FriProverData -- against oracle/batched.py
    after every step (batch root, fingerprint_r, inner roots, last element,
    transcript) and open_query_at records at both ends and a middle index."""
    from multilinear_amd.batched import BatchedFriProverData
    from oracle import batched as OB

    L = log_n + 1
    gp = F.pow_2_generator_powers(L)
    codes = [OF.reed_solomon([F.from_i64(7 * i + 3 + 100 * j) for i in range(1 << log_n)], gp[1])
             for j in range(m)]
    otr, tr = OT.Transcript(), Transcript()
    opd = OB.BatchedFriProverData.init(codes, otr)
    bp = BatchedFriProverData.init(dev([v for c in codes for v in c]), m, tr)
    assert bp.batch_root == opd.batch_layer.root() and bp.fingerprint_r == opd.fingerprint_r
    assert tr.random() == otr.random()
    r = tr.next_challenge()
    assert r == otr.next_challenge()
    opd.batched_fold_step(gp, r, otr)
    bp.batched_fold_step((gp[1], L), r, tr)
    fd = bp.fri_data
    assert fd.fold_roots() == opd.fri_data.fold_roots() and tr.random() == otr.random()
    for k in range(1, L - 1):
        r = tr.next_challenge()
        opd.fri_data.fold_step(gp, k, r, otr)
        fd.fold_step(k, r, tr, gen_pows=(gp[1], L))
        assert fd.fold_roots() == opd.fri_data.fold_roots(), k
        assert tr.random() == otr.random(), k
    assert fd.last_element == opd.fri_data.last_element is not None
    for idx in sorted({0, (1 << log_n) - 1, (1 << log_n) // 3}):
        want = _flat_batched_queries(type("P", (), {"queries": [opd.open_query_at(idx)]})())
        assert bp.open_query_at(idx) == want, idx
    with pytest.raises(_lib.MlhError):  # a second batched step: rejected, not re-folded
        bp.batched_fold_step((gp[1], L), r, tr)


def test_batched_inner_fold_step_without_tree_rejected():
    """fri_data.fold_step on a batched prover whose inner FriProverData holds no
    tree -- before batched_fold_step, and at log_code 2 where that step wrote
    the last element directly -- is MLH_ERR_INVALID (the reference panics on
    merkle_trees.last().unwrap()); a fri_data view keeps its parent alive."""
    import gc

    from multilinear_amd.batched import BatchedFriProverData

    for log_n in (1, 3):
        L = log_n + 1
        gp = F.pow_2_generator_powers(L)
        codes = [OF.reed_solomon([F.from_i64(5 * i + j) for i in range(1 << log_n)], gp[1])
                 for j in range(2)]
        tr = Transcript()
        bp = BatchedFriProverData.init(dev([v for c in codes for v in c]), 2, tr)
        fd = bp.fri_data
        with pytest.raises(_lib.MlhError) as e:
            fd.fold_step(1, 5, tr, gen_pows=(gp[1], L))
        assert e.value.status == _lib.MLH_ERR_INVALID
        bp.batched_fold_step((gp[1], L), tr.next_challenge(), tr)
        if log_n == 1:  # last element written, still no tree
            assert fd.last_element is not None
            with pytest.raises(_lib.MlhError) as e:
                fd.fold_step(1, 5, tr, gen_pows=(gp[1], L))
            assert e.value.status == _lib.MLH_ERR_INVALID
        else:
            del bp
            gc.collect()
            before = fd.fold_roots()
            fd.fold_step(1, tr.next_challenge(), tr, gen_pows=(gp[1], L))
            assert fd.fold_roots()[:len(before)] == before and len(fd.fold_roots()) == len(before) + 1


def test_fri_fold_step_huge_k_rejected():
    """k large enough that (n/2 - 1) 2^k wraps 64 bits is still rejected
    (MLH_ERR_INVALID, the reference's usize index underflow), not folded."""
    L = 12
    g = F.pow_2_generator(L)
    code = OF.reed_solomon([F.from_i64(7 * i + 3) for i in range(1 << (L - 1))], g)
    tr = Transcript()
    pd = MF.FriProverData.init(dev(code), tr)
    n0 = len(pd.fold_roots())
    for k in (2, 40, 41):
        with pytest.raises(_lib.MlhError) as e:
            pd.fold_step(k, 3, tr)
        assert e.value.status == _lib.MLH_ERR_INVALID
    assert len(pd.fold_roots()) == n0


def test_batched_fri_large_verifies():
    from multilinear_amd.batched import BatchedFriProof

    m, log_n = 4, 18
    g = F.pow_2_generator(log_n + 1)
    codes = [MF.reed_solomon(D.random_device(1 << log_n, 40 + j), g) for j in range(m)]
    import torch

    p = BatchedFriProof.prove(torch.cat(codes, 0), m, Transcript())
    assert p.verify()


@pytest.mark.parametrize("m,n", [(3, 5), (1, 4), (2, 1), (10, 7), (2, 13)])
def test_batched_pcs_prove_matches_oracle(m, n):
    from multilinear_amd.batched import BatchedPCSProof
    from oracle import batched as OB

    pts = [F.from_i64(i) for i in range(n)]
    polys = [[F.from_i64((j * 3 + i * 5) % 100) for j in range(1 << n)] for i in range(m)]
    outs = [OPL.mle_evaluate(p, pts) for p in polys]
    want = OB.BatchedPCSProof.prove(pts, outs, polys, OT.Transcript())
    got = BatchedPCSProof.prove(pts, outs, dev([v for p in polys for v in p]), Transcript())
    assert [tuple(x) for x in got.sumcheck_polynomials] == [tuple(x) for x in want.sumcheck_polynomials]
    fp = got.fri_proof
    assert fp.batch_commitment == want.fri_proof.batch_commitment
    assert fp.commitments == want.fri_proof.commitments
    assert fp.last_elem == want.fri_proof.last_elem
    assert fp.last_random == want.fri_proof.last_random
    assert bytes(fp._q) == _flat_batched_queries(want.fri_proof)
    assert got.verify(Transcript())
    got.outputs = [outs[0] + 1] + outs[1:]
    assert not got.verify(Transcript())


def test_table_cache_is_bounded_and_results_stay_exact():
    """The per-context twiddle cache is an LRU bounded by
    mlh_set_table_cache_limit: with a 2 MiB limit, transforms of many sizes
    (each needing its own tables, the 2^22 ones several MiB) still match the C
    oracle, and afterwards the cache holds no more than the last operation's
    tables."""
    C = _c_oracle()
    lib, ctx = D.lib(), D.context()
    D.check(lib.mlh_set_table_cache_limit(ctx, 2 << 20), ctx)
    try:
        for log_n in (12, 16, 20, 22, 13, 21, 22, 15):
            g = F.pow_2_generator(log_n)
            x = D.random_limbs(1 << log_n, 4000 + log_n)
            got = D.from_device(MN.Polynomial(D.to_device(x)).ntt(g).evals)
            assert (got == C.ntt(x, log_n, g)).all(), log_n
        # small transforms with distinct generators: their tables push the big
        # ones out of the pinned window; the cache then fits the limit
        x = D.random_limbs(1 << 12, 77)
        g12 = F.pow_2_generator(12)
        for e in range(1, 40, 2):
            g = pow(g12, e, F.M)
            got = D.from_device(MN.Polynomial(D.to_device(x)).ntt(g).evals)
            assert (got == C.ntt(x, 12, g)).all(), e
        assert lib.mlh_table_cache_bytes(ctx) <= 2 << 20
    finally:
        D.check(lib.mlh_set_table_cache_limit(ctx, 1 << 30), ctx)


def test_kernel_timer_sampling():
    """mlh_profile_enable(ctx, k): HIP events around every k-th transform only
    (bench.py --prof-every); k = 1 brackets every launch."""
    import ctypes

    ctx = D.context()
    lib = D.lib()
    x = D.random_device(1 << 16, 77)
    g = D.fe_bytes(F.pow_2_generator(16))
    for k, want in ((1, 8), (4, 2), (3, 3)):
        lib.mlh_profile_reset(ctx)
        D.check(lib.mlh_profile_enable(ctx, k), ctx)
        for _ in range(8):
            D.check(lib.mlh_ntt(ctx, D.ptr(x), D.ptr(x), 16, g), ctx)
        lib.mlh_profile_enable(ctx, 0)
        for lab in (b"ntt_pass<8,3,0>", b"ntt_pass<8,2,0>"):
            cnt, tot = ctypes.c_uint64(), ctypes.c_double()
            D.check(lib.mlh_profile_get(ctx, lab, ctypes.byref(cnt), ctypes.byref(tot)), ctx)
            assert cnt.value == want and tot.value > 0, (k, lab, cnt.value)
    assert lib.mlh_profile_enable(ctx, -1) == _lib.MLH_ERR_INVALID
