"""The PCS provers' rounds off the transcript chain (sumcheck.hip "PCS rounds
off the transcript kernel"; capi.hip PcsRounds) against the cooperative
one-round-per-launch path, which the oracle pins at n <= 17
(test_gpu_parity.py::test_pcs_prove_matches_oracle, round 3 on): at the
sizes whose head / tail splits the oracle tests do not reach -- n = 12 (no
head), 18 (a 6-variable head: one fold pass), 19 and 20 (two fold passes),
24 (config 4's size, B = 12) -- the two give byte-identical proofs (round
polynomials, commitments, last element, final transcript output, every query
record), and the proof verifies.  Reference: multilinear_pcs.rs:43-136,
batched_pcs.rs:36-180."""
import ctypes
import random

import pytest

pytestmark = pytest.mark.gpu

from oracle import field as F  # noqa: E402  (checker only)
from oracle import polynomials as OPL  # noqa: E402

from multilinear_amd import device as D  # noqa: E402
from multilinear_amd import multilinear_pcs as MP  # noqa: E402
from multilinear_amd import polynomials as MPL  # noqa: E402
from multilinear_amd.transcript import Transcript  # noqa: E402


class fused_max:
    def __init__(self, v):
        self.v = v

    def __enter__(self):
        ctx = D.context()
        D.check(D.lib().mlh_set_pcs_fused_max(ctx, self.v), ctx)

    def __exit__(self, *exc):
        ctx = D.context()
        D.check(D.lib().mlh_set_pcs_fused_max(ctx, 24), ctx)
        return False


def _proof_bytes(p):
    fp = p.fri_proof
    return (p.sumcheck_polynomials, fp.commitments, fp.last_elem, fp.last_random,
            fp.query_indices, bytes(fp._q))


@pytest.mark.parametrize("n", [12, 18, 19, 20, 24])
def test_pcs_fused_equals_cooperative_path(n):
    r = random.Random(900 + n)
    x = D.random_device(1 << n, 900 + n)
    pts = [r.randrange(F.M) for _ in range(n)]
    out = MPL.evaluate(x, pts)
    got = MP.PCSProof.prove(pts, out, x, Transcript())
    with fused_max(0):
        want = MP.PCSProof.prove(pts, out, x, Transcript())
    assert _proof_bytes(got) == _proof_bytes(want)
    assert got.verify(Transcript())


@pytest.mark.parametrize("m,n", [(2, 12), (3, 19)])
def test_batched_pcs_fused_equals_cooperative_path(m, n):
    from multilinear_amd.batched import BatchedPCSProof

    r = random.Random(950 + n)
    x = D.random_device(m << n, 950 + n)
    pts = [r.randrange(F.M) for _ in range(n)]
    outs = [MPL.evaluate(x[i << n:(i + 1) << n], pts) for i in range(m)]
    got = BatchedPCSProof.prove(pts, outs, x, Transcript())
    with fused_max(0):
        want = BatchedPCSProof.prove(pts, outs, x, Transcript())
    assert [tuple(v) for v in got.sumcheck_polynomials] == [tuple(v) for v in want.sumcheck_polynomials]
    assert got.fri_proof.commitments == want.fri_proof.commitments
    assert got.fri_proof.last_random == want.fri_proof.last_random
    assert bytes(got.fri_proof._q) == bytes(want.fri_proof._q)
    assert got.verify(Transcript())
