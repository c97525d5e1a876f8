"""Device-side failures are loud, and the gen_pows boundary checks what it says.

* A cooperative sumcheck kernel whose LDS wait times out (forced here with a
  spin limit of one sleep, mlh_set_coop_spin_limit) makes the prove return
  MLH_ERR_DEVICE instead of MLH_OK with wrong round polynomials; the next
  prove on the same context, at the default limit, is bit-exact again.  (The
  PCS provers no longer run a cooperative kernel at n <= 24.)
  (reference: sumcheck.rs:188-199, transcript.rs:23-38.)
* mlh_gen_pows_verify compares every entry of a host gen_pows table with
  gen_pows[1]^i on the device: the reference's pow_2_generator_powers passes,
  a table altered at any one index -- gen_pows[3], or one the host spot check
  of mlh_gen_pows_params does not sample -- is MLH_ERR_INVALID naming that
  index.  (reference: fri/mod.rs:79-114, :261.)
"""
import ctypes
import random

import pytest

pytestmark = pytest.mark.gpu

from oracle import field as F  # noqa: E402  (checker only)
from oracle import polynomials as OPL  # noqa: E402
from oracle import sumcheck as OS  # noqa: E402
from oracle import transcript as OT  # noqa: E402

from multilinear_amd import _lib  # noqa: E402
from multilinear_amd import device as D  # noqa: E402
from multilinear_amd import multilinear_pcs as MP  # noqa: E402
from multilinear_amd import sumcheck as MS  # noqa: E402
from multilinear_amd.transcript import Transcript  # noqa: E402


class spin_limit:
    def __init__(self, sleeps):
        self.sleeps = sleeps

    def __enter__(self):
        ctx = D.context()
        D.check(D.lib().mlh_set_coop_spin_limit(ctx, self.sleeps), ctx)

    def __exit__(self, *exc):
        ctx = D.context()
        D.check(D.lib().mlh_set_coop_spin_limit(ctx, 0), ctx)
        return False


def _sumcheck_case(n, seed):
    r = random.Random(seed)
    ev = [r.randrange(F.M) for _ in range(1 << n)]
    pts = [r.randrange(F.M) for _ in range(n)]
    return ev, pts, OPL.mle_evaluate(ev, pts)


def _oracle_rounds(ev, pts, total):
    ot, otr = OS.SumcheckTables.build_tables_for_pcs(pts, ev), OT.Transcript()
    prev, polys, rs = total, [], []
    for _ in range(len(pts)):
        nz, rr, prev = ot.compute_sumcheck_polynomial(prev, otr)
        polys.append(tuple(nz))
        rs.append(rr)
    return polys, rs, otr


@pytest.mark.parametrize("n", [13, 20])
def test_sumcheck_spin_timeout_is_an_error(n):
    """n = 13: the LDS eq tail (12 rounds) + one head round; n = 20: the
    corner-sum head launch as well."""
    ev, pts, total = _sumcheck_case(n, 700 + n)
    with spin_limit(1):
        t = MS.SumcheckTables.build_tables_for_pcs(pts, D.to_device(D.ints_to_limbs(ev)))
        bad_tr = Transcript()
        bad_tr.absorb(b"prefix")
        before = bad_tr.random()
        with pytest.raises(_lib.MlhError) as ei:
            t.compute_sumcheck_polynomials(total, bad_tr)
        assert ei.value.status == _lib.MLH_ERR_DEVICE
        assert bad_tr.random() == before  # a rejected prove leaves the transcript untouched
    # the same context at the default limit: bit-exact, and no stale error
    want_polys, want_rs, otr = _oracle_rounds(ev, pts, total)
    t = MS.SumcheckTables.build_tables_for_pcs(pts, D.to_device(D.ints_to_limbs(ev)))
    tr = Transcript()
    polys, rs = t.compute_sumcheck_polynomials(total, tr)
    assert polys == want_polys and rs == want_rs and tr.random() == otr.random()


def test_pcs_provers_run_no_cooperative_kernel():
    """The PCS and batched PCS provers (n <= 24) compute their rounds off the
    transcript chain with no cooperative kernel, so a spin limit of one sleep
    does not touch them: both proofs verify (the cooperative sumcheck above
    reports it)."""
    from multilinear_amd.batched import BatchedPCSProof

    n, m = 13, 2
    r = random.Random(78)
    polys = [[r.randrange(F.M) for _ in range(1 << n)] for _ in range(m)]
    pts = [r.randrange(F.M) for _ in range(n)]
    outs = [OPL.mle_evaluate(p, pts) for p in polys]
    evd = D.to_device(D.ints_to_limbs([v for p in polys for v in p]))
    with spin_limit(1):
        got = BatchedPCSProof.prove(pts, outs, evd, Transcript())
        assert got.verify(Transcript())
        pf = MP.PCSProof.prove(pts, outs[0], evd[: 1 << n], Transcript())
        assert pf.verify(Transcript())


def _verify(table):
    lib = D.lib()
    ctx = D.context()
    raw = b"".join(int(v).to_bytes(16, "little") for v in table) if isinstance(table, list) else table
    buf = (ctypes.c_uint8 * len(raw)).from_buffer_copy(raw)
    g, lg = (ctypes.c_uint8 * 16)(), ctypes.c_uint32()
    n = len(raw) // 16
    st = lib.mlh_gen_pows_verify(ctx, buf, n, g, ctypes.byref(lg))
    msg = (lib.mlh_last_error(ctx) or b"").decode()
    return st, int.from_bytes(bytes(g), "little"), lg.value, msg


def test_gen_pows_verify_full_table():
    tab = F.pow_2_generator_powers(13)
    assert _verify(tab)[:3] == (0, tab[1], 13)
    for i in (3, 4097, 5000, len(tab) - 2):
        alt = list(tab)
        alt[i] = (alt[i] + 1) % F.M
        st, _, _, msg = _verify(alt)
        assert st == _lib.MLH_ERR_INVALID, i
        # the host spot check (mlh_gen_pows_params) rejects it first, or
        # the device pass names the index
        assert msg.startswith("gen_pows is not the power series") or "gen_pows[%d]" % i in msg, msg
        if i in (4097, 5000):  # not among the spot check's indices: only the device pass sees it
            assert "gen_pows[%d]" % i in msg, msg
    alt = list(tab)
    alt[3] = tab[5]
    assert _verify(alt)[0] == _lib.MLH_ERR_INVALID


def test_gen_pows_verify_large_table_from_device():
    """A 2^21-entry table as the reference builds it (pow_2_generator_powers,
    here from mlh_pow_2_generator_powers) passes; one entry past the chunk
    boundary (2^20) altered is found."""
    import torch

    lg = 21
    out = D.empty(1 << lg)
    ctx = D.context()
    D.check(D.lib().mlh_pow_2_generator_powers(ctx, lg, D.ptr(out)), ctx)
    torch.cuda.synchronize()
    raw = bytearray(D.from_device(out).tobytes())
    g = F.pow_2_generator(lg)
    st, g_out, lg_out, _ = _verify(bytes(raw))
    assert (st, g_out, lg_out) == (0, g, lg)
    i = (1 << 20) + 12345
    raw[16 * i] ^= 1
    st, _, _, msg = _verify(bytes(raw))
    assert st == _lib.MLH_ERR_INVALID and "gen_pows[%d]" % i in msg, msg


def test_batched_pcs_device_failure_restores_transcript():
    """The batched PCS absorbs its claim on the host before the device rounds;
    when those rounds fail (cooperative path forced, spin limit of one sleep)
    the caller's transcript is restored to its state at entry (mlhip.h), and
    the next prove at the default limit equals the oracle-checked one."""
    from multilinear_amd.batched import BatchedPCSProof

    n, m = 13, 2
    r = random.Random(79)
    polys = [[r.randrange(F.M) for _ in range(1 << n)] for _ in range(m)]
    pts = [r.randrange(F.M) for _ in range(n)]
    outs = [OPL.mle_evaluate(p, pts) for p in polys]
    evd = D.to_device(D.ints_to_limbs([v for p in polys for v in p]))
    ctx = D.context()
    D.check(D.lib().mlh_set_pcs_fused_max(ctx, 0), ctx)
    try:
        with spin_limit(1):
            tr = Transcript()
            tr.absorb(b"abc")
            before = tr.random()
            with pytest.raises(_lib.MlhError) as ei:
                BatchedPCSProof.prove(pts, outs, evd, tr)
            assert ei.value.status == _lib.MLH_ERR_DEVICE
            assert tr.random() == before
            with pytest.raises(_lib.MlhError) as ei:
                MP.PCSProof.prove(pts, outs[0], evd[: 1 << n], tr)
            assert ei.value.status == _lib.MLH_ERR_DEVICE
            assert tr.random() == before
        good = BatchedPCSProof.prove(pts, outs, evd, Transcript())
        assert good.verify(Transcript())
    finally:
        D.check(D.lib().mlh_set_pcs_fused_max(ctx, 24), ctx)
