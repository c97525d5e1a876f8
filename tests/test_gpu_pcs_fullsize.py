"""Production-shape PCS proves against the C oracle, byte for byte.

`mlh_pcs_prove` has three head shapes (capi.hip `PcsRounds`): n <= 12 no head,
n = 13..18 one `fold_group_eq` pass, n >= 19 two passes; the batched PCS adds
the fingerprinted batch layer.  These tests run the shapes the bench and the
reference's own tests use -- n = 19, 20 (multilinear_pcs_bench_test's evals
7i + 3 at the point 0..19, multilinear_pcs.rs:210-228) and 24, and the batched
PCS at (m, n) = (10, 20) with batched_pcs_verify_test's inputs
(batched_pcs.rs:261-306) and (3, 19) -- and compare every round polynomial,
the batch root, every fold root, the last element, the final transcript
digest, the 128 query indices and every query record with
`orc_pcs_prove_par` (oracle/c/oracle.c: PCSProof::prove / BatchedPCSProof::
prove restated end to end, OpenMP over independent loops).  The checker is
test infrastructure only; the product path is libmlhip.so.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs an MI355X", allow_module_level=True)

from oracle import coracle as C  # noqa: E402  (checker only)
from oracle import field as F  # noqa: E402

from multilinear_amd import device as D  # noqa: E402
from multilinear_amd.batched import BatchedPCSProof  # noqa: E402
from multilinear_amd.multilinear_pcs import PCSProof  # noqa: E402
from multilinear_amd.transcript import Transcript  # noqa: E402


def _small_limbs(vals):
    """non-negative integers < 2^64 -> (n, 4) uint32 limbs (Field128::from)."""
    v = np.asarray(vals, dtype=np.uint64)
    out = np.zeros((v.shape[0], 4), dtype=np.uint32)
    out[:, 0] = (v & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    out[:, 1] = (v >> np.uint64(32)).astype(np.uint32)
    return out


def _rand_points(n, seed):
    return D.limbs_to_ints(D.random_limbs(n, seed))


def _check(got_polys, fp, want, batched):
    assert want["rc"] == 0
    assert got_polys == want["polys"]
    if batched:
        assert fp.batch_commitment == want["batch_root"]
    assert fp.commitments == want["roots"]
    assert fp.last_elem == want["last_elem"]
    assert fp.last_random == want["last_random"]
    assert fp.query_indices == want["indices"]
    assert fp.qbytes == want["query_bytes"]
    q = bytes(fp._q)
    assert len(q) == len(want["queries"])
    if q != want["queries"]:
        qb = fp.qbytes
        bad = [i for i in range(128) if q[i * qb:(i + 1) * qb] != want["queries"][i * qb:(i + 1) * qb]]
        raise AssertionError("query records differ at queries %s" % bad[:8])


@pytest.mark.slow
@pytest.mark.parametrize("n,kind,prefix", [(19, "random", b"abc"), (20, "reference", b""),
                                           (24, "random", b"")])
def test_pcs_prove_production_shape_vs_c_oracle(n, kind, prefix):
    if kind == "reference":  # multilinear_pcs_bench_test: evals 7i + 3, point 0..n-1
        ev = _small_limbs(np.arange(1 << n, dtype=np.uint64) * 7 + 3)
        pts = [F.from_i64(i) for i in range(n)]
    else:
        ev = D.random_limbs(1 << n, 500 + n)
        pts = _rand_points(n, 600 + n)
    out = C.mle_evaluate_par(ev, n, pts)
    want = C.pcs_prove_par(ev, n, pts, [out], prefix=prefix)
    tr = Transcript()
    tr.absorb(prefix)
    dev = D.to_device(ev)
    got = PCSProof.prove(pts, out, dev, tr)
    _check(got.sumcheck_polynomials, got.fri_proof, want, batched=False)
    assert tr.random() == want["last_random"]
    # the evaluations are the caller's: PCSProof::prove takes them by value, the
    # drop-in must leave the device copy untouched
    assert np.array_equal(D.from_device(dev), ev)
    assert got.verify(Transcript() if not prefix else _prefixed(prefix))


def _prefixed(prefix):
    t = Transcript()
    t.absorb(prefix)
    return t


@pytest.mark.slow
@pytest.mark.parametrize("m,n,kind", [(10, 20, "reference"), (3, 19, "random")])
def test_batched_pcs_prove_production_shape_vs_c_oracle(m, n, kind):
    if kind == "reference":  # batched_pcs_verify_test: evals (3j + 5i) % 100
        j = np.arange(1 << n, dtype=np.uint64)
        ev = np.concatenate([_small_limbs((j * 3 + i * 5) % 100) for i in range(m)])
        pts = [F.from_i64(i) for i in range(n)]
    else:
        ev = D.random_limbs(m << n, 700 + n)
        pts = _rand_points(n, 800 + n)
    outs = [C.mle_evaluate_par(ev[i << n:(i + 1) << n], n, pts) for i in range(m)]
    want = C.pcs_prove_par(ev, n, pts, outs, batched=True)
    got = BatchedPCSProof.prove(pts, outs, D.to_device(ev), Transcript())
    _check(got.sumcheck_polynomials, got.fri_proof, want, batched=True)
    assert got.verify(Transcript())
