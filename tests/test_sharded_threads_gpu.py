"""The C++ multi-GPU schedules (csrc/sharded.hip: mlh_sharded_*) at P = 2..16
ranks in ONE process on the one GPU, with collectives ordered on the device
the way RCCL orders them -- no host drain (host_side = 0).

Each rank is a thread with its own mlh_ctx and HIP stream.  The transport
(``ThreadDeviceTransport``) enqueues the exchange on the stream the library
passes, like ncclAllToAll / ncclAllGather: every rank records an event after
the producer of its send buffer, each rank's stream waits for all senders'
events and copies its chunks device to device, records a second event, and
waits for every rank's second event before anything later on its stream may
overwrite its send buffer.  The library never synchronises around these calls,
so this runs the stream ordering of the RCCL path at P > 1 -- including the
two-stream pipeline of mlh_sharded_ntt_batch -- which a host-side transport
cannot.  Every result is compared with the oracle (C restatement
oracle/c/oracle.c, and oracle/fri.py for whole proofs at small sizes).
"""
import ctypes
import os
import random
import threading
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from multilinear_amd import _lib  # noqa: E402
from multilinear_amd import device as DV  # noqa: E402
from multilinear_amd import sharded as S  # noqa: E402
from multilinear_amd.fri import FriProof  # noqa: E402
from multilinear_amd.transcript import Transcript  # noqa: E402
from oracle import coracle as C  # noqa: E402  (checker only)
from oracle import field as F  # noqa: E402
from oracle import fri as OF  # noqa: E402
from oracle import polynomials as OPL  # noqa: E402
from oracle import transcript as OT  # noqa: E402

_D2D = 3  # hipMemcpyDeviceToDevice


def _hip():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    h.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
    h.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                 ctypes.c_void_p]
    h.hipEventDestroy.argtypes = [ctypes.c_void_p]
    return h


class ThreadDeviceTransport:
    """P in-process ranks; collectives enqueued on the caller's stream."""

    def __init__(self, P, a2a_shift=0):
        self.P = P
        self.hip = _hip()
        self.bar = threading.Barrier(P, timeout=120)
        self.ready = [self._event() for _ in range(P)]
        self.done = [self._event() for _ in range(P)]
        self.send = [None] * P
        self.error = []
        self.calls = []  # rank 0's collectives in order: ("a2a", bytes per peer) / ("ag", bytes)

        def a2a(user, send, recv, per, stream):  # (void* arguments arrive as int or None)
            me = user or 0
            if me == 0:
                self.calls.append(("a2a", per))
                _progress("a2a %d" % per)
            return self._run(me, send, stream, lambda s, src: self._copy(
                (recv or 0) + s * per, (src or 0) + ((me + a2a_shift) % P) * per, per, stream))

        def ag(user, send, recv, nbytes, stream):
            if (user or 0) == 0:
                self.calls.append(("ag", nbytes))
                _progress("ag %d" % nbytes)
            return self._run(user or 0, send, stream, lambda s, src: self._copy(
                (recv or 0) + s * nbytes, src, nbytes, stream))

        self._a2a = _lib.ALL_TO_ALL_FN(a2a)
        self._ag = _lib.ALL_GATHER_FN(ag)
        self.transports = [_Tp(_lib.TransportC(P, r, 0, ctypes.c_void_p(r), self._a2a, self._ag))
                           for r in range(P)]

    def _event(self):
        e = ctypes.c_void_p()
        assert self.hip.hipEventCreateWithFlags(ctypes.byref(e), 2) == 0  # hipEventDisableTiming
        return e

    def _copy(self, dst, src, n, stream):
        if n:
            assert self.hip.hipMemcpyAsync(dst, src, n, _D2D, stream) == 0

    def _run(self, rank, send, stream, copy_from):
        try:
            self.send[rank] = send
            assert self.hip.hipEventRecord(self.ready[rank], stream) == 0
            self.bar.wait()
            for s in range(self.P):
                assert self.hip.hipStreamWaitEvent(stream, self.ready[s], 0) == 0
                copy_from(s, self.send[s])
            assert self.hip.hipEventRecord(self.done[rank], stream) == 0
            self.bar.wait()
            for s in range(self.P):  # senders' buffers stay untouched until all copied
                assert self.hip.hipStreamWaitEvent(stream, self.done[s], 0) == 0
            self.bar.wait()
            return 0
        except Exception as e:  # pragma: no cover - reported as MLH_ERR_COMM
            self.error.append(repr(e))
            self.bar.abort()
            return 1


class _Tp:
    def __init__(self, c):
        self.transport = c


def _run_ranks(P, body, tr=None):
    """body(rank, ctx, stream_ptr, transport) in P threads; returns the results."""
    tr = tr or ThreadDeviceTransport(P)
    out, errs = [None] * P, []
    streams = [torch.cuda.Stream() for _ in range(P)]
    ctxs = []
    for r in range(P):
        h = ctypes.c_void_p()
        DV.check(DV.lib().mlh_context_create(0, ctypes.c_void_p(streams[r].cuda_stream), ctypes.byref(h)))
        ctxs.append(h.value)

    def run(r):
        try:
            with torch.cuda.stream(streams[r]):
                out[r] = body(r, ctxs[r], streams[r], tr.transports[r])
                streams[r].synchronize()
        except Exception:
            import traceback

            errs.append(traceback.format_exc())
            tr.bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    torch.cuda.synchronize()
    for c in ctxs:
        DV.lib().mlh_context_destroy(c)
    assert not tr.error, tr.error
    assert not errs, errs[0]
    return out


def _tp(t):
    return ctypes.byref(t.transport)


def _gen(log_n):
    return F.pow_2_generator(log_n)


@pytest.mark.parametrize("P,log_n,count", [(2, 14, 3), (4, 16, 4), (8, 18, 3), (16, 12, 2)])
def test_ntt_batch_pipelined_vs_c_oracle(P, log_n, count):
    """mlh_sharded_ntt_batch (two streams, device-ordered exchanges): every
    transform equals the C oracle's NTT; the inverse batch gives the inputs back."""
    L = DV.lib()
    xs = [DV.random_limbs(1 << log_n, seed=100 + i) for i in range(count)]
    g = _gen(log_n)

    def body(r, ctx, st, t):
        ins = [DV.to_device(S.shard_cyclic(x, P, r)) for x in xs]
        outs = [DV.empty(ins[0].shape[0]) for _ in range(count)]
        back = [DV.empty(ins[0].shape[0]) for _ in range(count)]
        pi = (ctypes.c_void_p * count)(*[i.data_ptr() for i in ins])
        po = (ctypes.c_void_p * count)(*[o.data_ptr() for o in outs])
        pb = (ctypes.c_void_p * count)(*[b.data_ptr() for b in back])
        torch.cuda.current_stream().synchronize()
        DV.check(L.mlh_sharded_ntt_batch(ctx, _tp(t), pi, po, count, log_n, DV.fe_bytes(g), 0), ctx)
        DV.check(L.mlh_sharded_ntt_batch(ctx, _tp(t), po, pb, count, log_n, DV.fe_bytes(g), 1), ctx)
        DV.check(L.mlh_synchronize(ctx), ctx)
        return ([DV.from_device(o) for o in outs], [DV.from_device(b) for b in back],
                [DV.from_device(i) for i in ins])

    res = _run_ranks(P, body)
    log_s = log_n - 2 * (P.bit_length() - 1)
    for i, x in enumerate(xs):
        want = C.ntt(x, log_n, g)
        got = S.unshard_blocks([res[r][0][i] for r in range(P)], log_s)
        assert np.array_equal(got, want), "transform %d" % i
        for r in range(P):
            assert np.array_equal(res[r][1][i], res[r][2][i]), "inverse of transform %d, rank %d" % (i, r)


@pytest.mark.parametrize("P,log_n,count", [(2, 15, 3), (4, 16, 3), (8, 18, 3), (8, 21, 2), (2, 25, 2),
                                           pytest.param(4, 26, 1, marks=pytest.mark.slow),
                                           pytest.param(8, 27, 2, marks=pytest.mark.slow)])
def test_ntt_fused_batch_vs_c_oracle(P, log_n, count):
    """mlh_sharded_ntt_fused_batch (the rank digit fused into the last pass;
    local passes, one all-to-all, one pass over the received chunks; three
    streams, device-ordered exchanges): every transform equals the C oracle's
    NTT once the block-cyclic outputs (block 2^log_s, log_s reported by the
    call) are put back in order.  (8, 27) is the bench's N = 8 shape: 2^24 per
    rank; (4, 26) its N = 4 shape."""
    L = DV.lib()
    xs = [DV.random_limbs(1 << log_n, seed=300 + i) for i in range(count)]
    g = _gen(log_n)

    def body(r, ctx, st, t):
        ins = [DV.to_device(S.shard_cyclic(x, P, r)) for x in xs]
        outs = [DV.empty(ins[0].shape[0]) for _ in range(count)]
        pi = (ctypes.c_void_p * count)(*[i.data_ptr() for i in ins])
        po = (ctypes.c_void_p * count)(*[o.data_ptr() for o in outs])
        ls = ctypes.c_uint32()
        torch.cuda.current_stream().synchronize()
        DV.check(L.mlh_sharded_ntt_fused_batch(ctx, _tp(t), pi, po, count, log_n, DV.fe_bytes(g),
                                               ctypes.byref(ls)), ctx)
        DV.check(L.mlh_synchronize(ctx), ctx)
        return [DV.from_device(o) for o in outs], ls.value

    res = _run_ranks(P, body)
    log_s = res[0][1]
    assert all(res[r][1] == log_s for r in range(P)) and 3 <= log_s < log_n
    for i, x in enumerate(xs):
        want = C.ntt_par(x, log_n, g) if log_n > 22 else C.ntt(x, log_n, g)
        got = S.unshard_blocks([res[r][0][i] for r in range(P)], log_s)
        assert np.array_equal(got, want), "transform %d" % i


def test_ntt_fused_batch_rejects_unsupported():
    """P = 16 and local sizes below the fused plan's minimum are refused
    (mlh_sharded_ntt_batch covers them); a generator of the wrong order too."""
    L = DV.lib()

    def body(r, ctx, st, t):
        x = DV.empty(1 << 8)
        pi = (ctypes.c_void_p * 1)(x.data_ptr())
        st1 = L.mlh_sharded_ntt_fused_batch(ctx, _tp(t), pi, pi, 1, 12, DV.fe_bytes(_gen(12)), None)
        st2 = L.mlh_sharded_ntt_fused_batch(ctx, _tp(t), pi, pi, 1, 12, DV.fe_bytes(_gen(11)), None)
        return st1, st2

    for P, want2 in ((16, _lib.MLH_ERR_INVALID), (8, _lib.MLH_ERR_BAD_GENERATOR)):
        for st1, st2 in _run_ranks(P, body):
            assert st1 == _lib.MLH_ERR_INVALID and st2 == want2


def test_ntt_spot_check_logic_vs_c_oracle_p8():
    """The bench's in-run check of the sharded headline (bench.py
    sharded_ntt_check) at P = 8 device-ordered ranks: the per-rank terms
    gen^(jg) poly_g(gen^(jP)) (mlh_poly_evaluate on the cyclic shard) summed
    over ranks equal the C oracle's X[j], and equal the sharded output at the
    rank / local index ntt_block_owner names; an output altered at one
    sampled index is caught."""
    P, log_n = 8, 18
    L = DV.lib()
    x = DV.random_limbs(1 << log_n, seed=4242)
    g = _gen(log_n)
    rr = random.Random(0xC0FFEE)
    js = [0, (1 << log_n) - 1] + [rr.randrange(1 << log_n) for _ in range(8)]

    def body(r, ctx, st, t):
        xin = DV.to_device(S.shard_cyclic(x, P, r))
        out = DV.empty(xin.shape[0])
        pi = (ctypes.c_void_p * 1)(xin.data_ptr())
        po = (ctypes.c_void_p * 1)(out.data_ptr())
        torch.cuda.current_stream().synchronize()
        DV.check(L.mlh_sharded_ntt_batch(ctx, _tp(t), pi, po, 1, log_n, DV.fe_bytes(g), 0), ctx)
        DV.check(L.mlh_synchronize(ctx), ctx)
        terms = S.ntt_spot_terms(xin, log_n, g, r, P, js, ctx=ctx)
        return DV.from_device(out), terms

    res = _run_ranks(P, body)
    want = C.ntt(x, log_n, g)
    want_ints = DV.limbs_to_ints(want)
    outs = [DV.limbs_to_ints(res[r][0]) for r in range(P)]
    for i, j in enumerate(js):
        X = sum(res[r][1][i] for r in range(P)) % F.M
        assert X == want_ints[j], j
        owner, loc = S.ntt_block_owner(j, log_n, 3)
        assert outs[owner][loc] == X, j
    # an altered output element is seen by the same comparison
    j = js[5]
    owner, loc = S.ntt_block_owner(j, log_n, 3)
    outs[owner][loc] = (outs[owner][loc] + 1) % F.M
    assert outs[owner][loc] != sum(res[r][1][5] for r in range(P)) % F.M


@pytest.mark.parametrize("P", [2, 8])
def test_comm_preflight_pattern_p8(P):
    """mlh_comm_preflight (bench.py runs it before the first data-path
    collective): a 1 MiB all-to-all + all-gather of rank-tagged words through
    a device-ordered transport -- 0 mismatches on every rank; a transport that
    delivers each all-to-all chunk from the wrong offset (a miswired exchange)
    is caught on every rank, with exactly the all-to-all's words counted."""
    per = (1 << 20) // P

    def body(r, ctx, st, t):
        return S.preflight(t, per, ctx=ctx)

    for shift, want in ((0, 0), (1, per // 4 * P)):
        res = _run_ranks(P, body, ThreadDeviceTransport(P, a2a_shift=shift))
        for r in range(P):
            bad, ms = res[r]
            assert bad == want, (shift, r, bad)
            assert ms >= 0.0
    L = DV.lib()
    ctx = DV.context()
    t = ThreadDeviceTransport(1).transports[0]
    bad = ctypes.c_uint64()
    assert L.mlh_comm_preflight(ctx, _tp(t), 6, ctypes.byref(bad), None) == _lib.MLH_ERR_INVALID


def _sumcheck_oracle(ev, pts, claim):
    m, d = ev.copy(), C.eq_table_par(pts)
    n = len(pts)
    tr = OT.Transcript()
    prev, polys, rs = claim, [], []
    for k in range(n):
        lh = n - k
        s1, s2 = C.partial_sums_par(m, d, lh)
        pol = OPL.interpolate([(prev - s1) % F.M, s1, s2])
        for c in pol[1:]:
            tr.absorb(F.to_bytes(c))
        rch = tr.next_challenge()
        prev = OPL.uni_evaluate(pol, rch)
        polys.append(tuple(pol[1:]))
        rs.append(rch)
        C.fold_par(m, d, lh, rch)
        m, d = m[: 1 << (lh - 1)], d[: 1 << (lh - 1)]
    return polys, rs, tr.random(), m[0].tobytes(), d[0].tobytes()


@pytest.mark.parametrize("P,log_code,gather_log,n_sc", [(2, 14, 8, 9), (4, 18, 12, 12),
                                                         (8, 16, 10, 11), (16, 12, 16, 4)])
def test_fri_and_sumcheck_device_ordered_vs_oracle(P, log_code, gather_log, n_sc):
    """Sharded RS -> commit root -> FRI prove, and the sharded eq table +
    sumcheck, through device-ordered collectives, against the oracle: RS code
    and FRI commitments / last element from the C oracle, whole proof (every
    query path) from oracle/fri.py at log_code <= 14, sumcheck round
    polynomials, challenges, transcript and folded m(r), d(r) from the
    reference round loop on the C oracle."""
    L = DV.lib()
    coeffs = DV.random_limbs(1 << (log_code - 1), seed=7)
    gc = _gen(log_code)
    ev = DV.random_limbs(1 << n_sc, seed=8)
    rr = random.Random(9)
    pts = [rr.randrange(F.M) for _ in range(n_sc)]
    claim = 1234567

    def body(r, ctx, st, t):
        c_loc = DV.to_device(S.shard_cyclic(coeffs, P, r))
        code = DV.empty(2 * c_loc.shape[0])
        torch.cuda.current_stream().synchronize()
        DV.check(L.mlh_sharded_reed_solomon(ctx, _tp(t), DV.ptr(c_loc), log_code - 1, DV.fe_bytes(gc),
                                            DV.ptr(code)), ctx)
        root = (ctypes.c_uint8 * 32)()
        DV.check(L.mlh_sharded_commit_rs_code(ctx, _tp(t), DV.ptr(code), log_code, root), ctx)
        pf = FriProof(log_code)
        tr = Transcript()
        DV.check(L.mlh_sharded_fri_prove(ctx, _tp(t), DV.ptr(code), log_code, gather_log, tr.h,
                                         ctypes.byref(pf.c)), ctx)
        m = DV.to_device(S.shard_cyclic(ev, P, r))
        pb = b"".join(int(v).to_bytes(16, "little") for v in pts)
        d = DV.empty(m.shape[0])
        DV.check(L.mlh_sharded_eq_table(ctx, _tp(t), (ctypes.c_uint8 * len(pb)).from_buffer_copy(pb),
                                        n_sc, DV.ptr(d)), ctx)
        str_ = Transcript()
        polys = (ctypes.c_uint8 * (32 * n_sc))()
        rsb = (ctypes.c_uint8 * (16 * n_sc))()
        DV.check(L.mlh_sharded_sumcheck_prove(ctx, _tp(t), DV.ptr(m), DV.ptr(d), n_sc,
                                              DV.fe_bytes(claim), str_.h, polys, rsb), ctx)
        DV.check(L.mlh_synchronize(ctx), ctx)
        P_, R_ = bytes(polys), bytes(rsb)
        sc = ([(int.from_bytes(P_[32 * k:32 * k + 16], "little"),
                int.from_bytes(P_[32 * k + 16:32 * k + 32], "little")) for k in range(n_sc)],
              [int.from_bytes(R_[16 * k:16 * k + 16], "little") for k in range(n_sc)],
              str_.random(), DV.from_device(m[:1]).tobytes(), DV.from_device(d[:1]).tobytes())
        return (DV.from_device(code), bytes(root), bytes(pf._commit), bytes(pf.c.last_elem),
                bytes(pf.c.last_random), [pf.query(q) for q in range(_lib.NUM_QUERIES)],
                pf.verify(), sc)

    res = _run_ranks(P, body)
    code_want = C.reed_solomon(coeffs, log_code - 1, gc)
    log_s = log_code - 2 * (P.bit_length() - 1)
    assert np.array_equal(S.unshard_blocks([res[r][0] for r in range(P)], log_s), code_want)
    roots, last, _, rc = C.fri_commit_par(code_want, log_code)
    assert rc == 0
    want_sc = _sumcheck_oracle(ev, pts, claim)
    for r in range(P):
        _, root, commit, last_b, _, _, ok, sc = res[r]
        assert root == roots[0], "rank %d: commit_rs_code root" % r
        assert [commit[32 * i:32 * i + 32] for i in range(len(roots))] == roots, "rank %d" % r
        assert int.from_bytes(last_b, "little") == last
        assert ok, "rank %d: proof rejected by the verifier" % r
        assert sc[0] == want_sc[0] and sc[1] == want_sc[1], "rank %d: sumcheck rounds" % r
        assert sc[2:] == want_sc[2:], "rank %d: transcript / folded tables" % r
        assert res[r][2:6] == res[0][2:6], "rank %d: proof differs from rank 0" % r
    if log_code <= 14:
        ints = [int.from_bytes(code_want[i].tobytes(), "little") for i in range(1 << log_code)]
        want = OF.FriProof.prove(ints, F.pow_2_generator_powers(log_code), OT.Transcript())
        assert res[0][2] == b"".join(want.commitments)
        assert res[0][4] == want.last_random
        for q, gq in enumerate(res[0][5]):
            for (gv, gs), (wv, wpath) in zip(gq, want.queries[q]):
                assert gv == wv and gs == [s for s, _ in wpath]


# ---- config 5 at its production shape (bench.config5 at N = 8 / 4 / 2) ----

_C5 = {}


def _progress(msg):
    """Progress lines for a long GPU test (MLH_TEST_PROGRESS=<file>): the
    long phases of the config-5 test leave a trace even if it is killed."""
    path = os.environ.get("MLH_TEST_PROGRESS")
    if path:
        with open(path, "a") as f:
            f.write("%.1f %s\n" % (time.time(), msg))


def _config5_reference():
    """The 2^27 coefficients, the C oracle's RS code and FRI commit, and the
    single-GPU proof (mlh_reed_solomon + mlh_fri_prove) of the same code --
    computed once for the three world sizes."""
    if not _C5:
        import gc

        from multilinear_amd import fri as MF

        log_c = 27
        _progress("config5 reference: start")
        coeffs = DV.random_limbs(1 << log_c, seed=5151)
        g = _gen(log_c + 1)
        dcode = MF.reed_solomon(DV.to_device(coeffs), g)
        single = MF.FriProof.prove(dcode, Transcript())
        code1 = DV.from_device(dcode)
        del dcode
        gc.collect()
        torch.cuda.empty_cache()
        _progress("config5 reference: single-GPU prove done")
        want = C.reed_solomon_par(coeffs, log_c, g)
        _progress("config5 reference: oracle RS done")
        assert np.array_equal(code1, want), "single-GPU RS 2^27 -> 2^28 differs from the C oracle"
        del code1
        roots, last, lr, rc = C.fri_commit_par(want, log_c + 1)
        _progress("config5 reference: oracle commit done")
        assert rc == 0
        _C5.update(coeffs=coeffs, g=g, want=want, roots=roots, last=last, single=single,
                   single_bytes=single.to_bytes())
        # the single-GPU proof against the oracle commit: every root, the last element
        assert single.commitments == roots and single.last_elem == last
        assert single.verify()
    return _C5


@pytest.mark.slow
@pytest.mark.timeout(900)
@pytest.mark.parametrize("P", [2, 4, 8])
def test_config5_sharded_prove_production_shape(P):
    """bench.config5's exact calls at N = P: mlh_sharded_reed_solomon of the
    2^27 cyclic coefficients, then mlh_sharded_fri_prove(log_code 28,
    gather_log 16) through device-ordered collectives.  The unsharded code
    equals the C oracle's RS code; every rank's proof equals, byte for byte
    (bincode wire form: all 27 commitments, the 128 query records, the last
    element, the final digest), the single-GPU mlh_fri_prove of the same
    natural-order code, whose commitments and last element equal the C
    oracle's fri_commit.  At P = 8 the path runs the re-deal all-to-alls of
    the 2^25, 2^22 and 2^19 layers and the all-gather of the 2^16 layer
    (fri/mod.rs:261-285)."""
    ref = _config5_reference()
    L = DV.lib()
    log_code, gather_log = 28, 16
    coeffs, g = ref["coeffs"], ref["g"]
    tr = ThreadDeviceTransport(P)

    def body(r, ctx, st, t):
        c_loc = DV.to_device(S.shard_cyclic(coeffs, P, r))
        code = DV.empty(2 * c_loc.shape[0])
        torch.cuda.current_stream().synchronize()
        DV.check(L.mlh_sharded_reed_solomon(ctx, _tp(t), DV.ptr(c_loc), log_code - 1, DV.fe_bytes(g),
                                            DV.ptr(code)), ctx)
        DV.check(L.mlh_synchronize(ctx), ctx)
        _progress("P=%d rank %d: sharded RS done" % (P, r))
        del c_loc
        pf = FriProof(log_code)
        trx = Transcript()  # (kept alive across the call: the C side holds its pointer)
        DV.check(L.mlh_sharded_fri_prove(ctx, _tp(t), DV.ptr(code), log_code, gather_log,
                                         trx.h, ctypes.byref(pf.c)), ctx)
        DV.check(L.mlh_synchronize(ctx), ctx)
        _progress("P=%d rank %d: sharded prove done" % (P, r))
        host = DV.from_device(code)
        _progress("P=%d rank %d: code copied out" % (P, r))
        wire = pf.to_bytes()
        ok = pf.verify()
        _progress("P=%d rank %d: proof encoded and verified" % (P, r))
        return host, wire, ok

    res = _run_ranks(P, body, tr)
    _progress("P=%d: ranks joined" % P)
    p = P.bit_length() - 1
    got = S.unshard_blocks([res[r][0] for r in range(P)], log_code - 2 * p)
    for r in range(P):
        res[r] = (None,) + tuple(res[r][1:])
    bad = np.nonzero((got != ref["want"]).any(axis=1))[0]
    assert bad.size == 0, "sharded RS mismatches at %s of %d" % (bad[:8].tolist(), bad.size)
    del got
    _progress("P=%d: code compared" % P)
    for r in range(P):
        assert res[r][1] == ref["single_bytes"], "rank %d: proof differs from the single-GPU proof" % r
        assert res[r][2], "rank %d: proof rejected by the verifier" % r
    # the schedule ran what bench.config5 runs: re-deals of the folded layers
    # above gather_log (bytes per peer = 16 * 2^log_next / P^2), then one
    # all-gather of the first layer at or below it (16 * 2^log / P per rank)
    redeals = sorted({(per // 16).bit_length() - 1 + 2 * p for kind, per in tr.calls if kind == "a2a"})
    gathers = {(nb // 16).bit_length() - 1 + p for kind, nb in tr.calls if kind == "ag" and nb % 16 == 0}
    if P == 8:
        assert {19, 22, 25} <= set(redeals), redeals
    assert gather_log in gathers, sorted(gathers)
    assert max(lg for lg in redeals if lg < log_code) > gather_log
