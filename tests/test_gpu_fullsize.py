"""Full-size parity at the BASELINE.json configurations, and the gen_pows
argument of the FRI prover, against the oracle.

Config 3 (2^24 coefficients -> 2^25 RS code -> FRI commit), config 4 (24
variable eq-factored sumcheck) and config 5 at one GPU (2^27 coefficients ->
2^28 code -> FRI commit) are compared bit for bit with the C restatement of the
reference loops (oracle/c/oracle.c), run with OpenMP over the box's host cores
(the *_par checkers: the same arithmetic, parallel over independent work).
The checker is test infrastructure only; the product path is libmlhip.so.
"""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)

from oracle import coracle as C  # noqa: E402  (checker only)
from oracle import field as F  # noqa: E402
from oracle import fri as OF  # noqa: E402
from oracle import polynomials as OPL  # noqa: E402
from oracle import transcript as OT  # noqa: E402

from multilinear_amd import _lib  # noqa: E402
from multilinear_amd import device as D  # noqa: E402
from multilinear_amd import fri as MF  # noqa: E402
from multilinear_amd import sumcheck as MS  # noqa: E402
from multilinear_amd.transcript import Transcript  # noqa: E402


def _c():
    C.lib()
    return C


def _rand(n, seed):
    r = random.Random(seed)
    return [r.randrange(F.M) for _ in range(n)]


# ---- gen_pows (fri/mod.rs:58-145, 261: FriProof::prove(code, gen_pows, tr)) ----

def test_fri_prove_with_caller_gen_pows_table():
    """A code built with a non-canonical generator h (order 2N) and the table of
    h's powers: the reference folds with gen_pows[len - i 2^k] = h^(-i 2^k); the
    _gp entry points reproduce the proof byte for byte (roots, last element,
    transcript, every query path)."""
    L = 10
    g = F.pow_2_generator(L)
    h = pow(g, 3, F.M)  # another generator of order 2^L
    coeffs = _rand(1 << (L - 1), 31)
    code = OF.reed_solomon(coeffs, h)
    gp = [pow(h, j, F.M) for j in range(1 << L)]
    want = OF.FriProof.prove(code, gp, OT.Transcript())
    got = MF.FriProof.prove(D.to_device(D.ints_to_limbs(code)), Transcript(), gen_pows=(h, L))
    assert got.commitments == want.commitments
    assert got.last_elem == want.last_elem and got.last_random == want.last_random
    for q in range(_lib.NUM_QUERIES):
        for (gv, gs), (wv, wpath) in zip(got.query(q), want.queries[q]):
            assert gv == wv and gs == [sib for sib, _ in wpath]
    # the step-by-step API with the same table
    otr, tr = OT.Transcript(), Transcript()
    opd = OF.FriProverData.fold(gp, code, otr)
    pd = MF.FriProverData.init(D.to_device(D.ints_to_limbs(code)), tr, gen_pows=(h, L))
    for k in range(L - 1):
        pd.fold_step(k, tr.next_challenge(), tr)
    assert pd.fold_roots() == opd.fold_roots()
    assert pd.last_element == opd.last_element and tr.random() == otr.random()


def test_fri_prove_longer_gen_pows_table_matches_reference_panic():
    """gen_pows of 2N entries for a code of N: the reference folds with
    g_{2N}^(-i 2^k), which is not the code's domain, and panics "not an RS code"
    (fri/mod.rs:119-122); the drop-in returns MLH_ERR_NOT_RS_CODE on the same
    input.  Tables shorter than N/2 (index underflow in the reference) and
    generators of the wrong order are rejected."""
    L = 9
    g = F.pow_2_generator(L)
    code = OF.reed_solomon(_rand(1 << (L - 1), 5), g)
    gp_long = F.pow_2_generator_powers(L + 1)
    with pytest.raises(AssertionError):
        OF.FriProof.prove(code, gp_long, OT.Transcript())
    dcode = D.to_device(D.ints_to_limbs(code))
    with pytest.raises(_lib.MlhError) as e:
        MF.FriProof.prove(dcode, Transcript(), gen_pows=(gp_long[1], L + 1))
    assert e.value.status == _lib.MLH_ERR_NOT_RS_CODE
    with pytest.raises(_lib.MlhError) as e:
        MF.FriProof.prove(dcode, Transcript(), gen_pows=(F.pow_2_generator(L - 2), L - 2))
    assert e.value.status == _lib.MLH_ERR_INVALID
    with pytest.raises(_lib.MlhError) as e:
        MF.FriProof.prove(dcode, Transcript(), gen_pows=(F.pow_2_generator(L - 1), L))
    assert e.value.status == _lib.MLH_ERR_BAD_GENERATOR
    # the canonical table through the _gp path equals the plain entry point
    a = MF.FriProof.prove(dcode, Transcript(), gen_pows=(g, L))
    b = MF.FriProof.prove(dcode, Transcript())
    assert a.commitments == b.commitments and a.last_random == b.last_random


# ---- config 3: 2^24 coefficients -> RS 2^25 -> FRI commit (fri/mod.rs:19-145) ----

@pytest.mark.slow
def test_config3_rs_2_25_and_fri_commit_vs_c_oracle():
    """Bit-exact RS LDE through the default 2^25 plan (pass 0 ntt_pass<9,3,1>)
    and the 2^24-leaf tree plus all 24 fold layers: roots, last element and the
    final transcript state against the C oracle."""
    Cq = _c()
    log_n = 24
    x = D.random_limbs(1 << log_n, 3333)
    g = F.pow_2_generator(log_n + 1)
    want = Cq.reed_solomon_par(x, log_n, g)
    dcode = MF.reed_solomon(D.to_device(x), g)
    got = D.from_device(dcode)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, "RS mismatches at %s of %d" % (bad[:8].tolist(), bad.size)
    roots, last, lr, rc = Cq.fri_commit_par(want, log_n + 1)
    assert rc == 0
    tr = Transcript()
    pd = MF.FriProverData.fold(dcode, tr)
    assert pd.fold_roots() == roots
    assert pd.last_element == last
    assert tr.random() == lr


# ---- config 4: 24-variable sumcheck rounds (sumcheck.rs:77-247) ----

@pytest.mark.slow
@pytest.mark.parametrize("n,label", [(17, b""), (19, b""), (20, b"abc"), (21, b""), (22, b"x" * 33), (23, b"abc"), (24, b"")])
def test_config4_sumcheck_24_vars_vs_c_oracle(n, label):
    """build_tables_for_pcs + compute_sumcheck_polynomials at 24 variables
    (the GPU keeps delta = eq(point) factored) against the reference round loop
    driven by the C oracle's eq table, partial sums and folds and the Python
    transcript: every round polynomial, every challenge, the final transcript.
    n = 17..24 has B = n - 12 = 5..12 head rounds: one corner-sum pass, ONE
    serial launch on the 2^B corner sums (a group of min(B, 6) variables, then
    B - 6 = 1..6 more for n >= 19) and the fold passes; the 3- and 33-byte
    transcript prefixes send every absorb through the device transcript's
    byte path."""
    Cq = _c()
    ev = D.random_limbs(1 << n, 2424)
    pts = _rand(n, 24)
    m = ev.copy()
    d = Cq.eq_table_par(pts)
    total = Cq.dot_par(m, d, n)
    tr = OT.Transcript()
    tr.absorb(label)
    prev = total
    want_polys, want_rs = [], []
    for k in range(n):
        lh = n - k
        s1, s2 = Cq.partial_sums_par(m, d, lh)
        pol = OPL.interpolate([(prev - s1) % F.M, s1, s2])
        for c in pol[1:]:
            tr.absorb(F.to_bytes(c))
        r = tr.next_challenge()
        prev = OPL.uni_evaluate(pol, r)
        want_polys.append(tuple(pol[1:]))
        want_rs.append(r)
        Cq.fold_par(m, d, lh, r)
        m, d = m[: 1 << (lh - 1)], d[: 1 << (lh - 1)]
    gtr = Transcript()
    gtr.absorb(label)
    polys, rs = MS.SumcheckTables.build_tables_for_pcs(pts, D.to_device(ev)).compute_sumcheck_polynomials(
        total, gtr)
    assert rs == want_rs
    assert polys == want_polys
    assert gtr.random() == tr.random()


# ---- config 5 on one GPU: 2^27 coefficients -> RS 2^28 -> FRI commit ----

@pytest.mark.slow
@pytest.mark.timeout(900)
def test_config5_rs_2_28_and_fri_commit_vs_c_oracle():
    """The single-GPU form of config 5 (the 8-GPU run shards the same code):
    RS through the 4-pass plan 7,7,7,7, 2^27-leaf tree, 27 fold layers."""
    Cq = _c()
    log_n = 27
    x = D.random_limbs(1 << log_n, 2828)
    g = F.pow_2_generator(log_n + 1)
    dcode = MF.reed_solomon(D.to_device(x), g)
    want = Cq.reed_solomon_par(x, log_n, g)
    del x
    got = D.from_device(dcode)
    assert (got == want).all()
    del got
    tr = Transcript()
    pd = MF.FriProverData.fold(dcode, tr)
    roots, last, lr, rc = Cq.fri_commit_par(want, log_n + 1)
    assert rc == 0
    assert pd.fold_roots() == roots
    assert pd.last_element == last
    assert tr.random() == lr
