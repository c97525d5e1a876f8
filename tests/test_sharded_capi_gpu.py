"""The multi-GPU C ABI (csrc/sharded.hip: mlh_sharded_*, mlh_comm_*).

* 2 and 4 real processes sharing the one GPU, exchanges through
  sharded.HostTransport (torch.distributed gloo as C callbacks), every result
  compared with the ORACLE on the same inputs: the sharded NTT / INTT / RS
  outputs reassemble to the C oracle's (oracle/c/oracle.c: ntt /
  reed_solomon); the sharded FRI proof's commitments and last element equal
  the C oracle's FriProverData::fold (orc_fri_commit_par) and, at codewords
  the Python oracle proves in seconds, every query path equals
  oracle/fri.py's FriProof::prove; the sharded eq table + sumcheck give the
  round polynomials, challenges, final transcript and fully folded m(r), d(r)
  of the reference round loop run on the C oracle (eq_table_par,
  partial_sums_par, fold_par).  The single-GPU entry points are compared as
  well (same bytes).
* RCCL at world 1: an mlh_comm is created from a unique id and its transport
  callbacks (ncclAllToAll / ncclAllGather) move device buffers.
The C++ schedules follow the executable CPU spec tests/dist_spec.py, which
tests/test_dist_cpu.py checks against the oracle over gloo.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

from multilinear_amd import device as DV  # noqa: E402
from tests import dist_spec as D  # noqa: E402
from multilinear_amd import sharded as S  # noqa: E402
from oracle import coracle as C  # noqa: E402  (checker only)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, q):
    import random

    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from multilinear_amd import fri as MF
        from multilinear_amd import ntt as MN
        from multilinear_amd import polynomials as MPL
        from multilinear_amd import sumcheck as MS
        from multilinear_amd.fri import FriProof
        from multilinear_amd.transcript import Transcript

        torch.cuda.set_device(0)
        ht = S.HostTransport(D.Transport(host_staged=True))
        res = {}
        # NTT / INTT
        ln = cfg["log_ntt"]
        x = DV.random_limbs(1 << ln, seed=31)
        g = MN.pow_2_generator(ln)
        xl = DV.to_device(D.shard_cyclic(x, world, rank))
        X = S.ntt(xl, ln, g, ht)
        res["ntt"] = DV.from_device(X).tobytes()
        res["intt_ok"] = bool(torch.equal(S.ntt(X, ln, g, ht, inverse=True), xl))
        # RS + FRI prove
        lc = cfg["log_code"]
        coeffs = DV.random_limbs(1 << (lc - 1), seed=11)
        gc = MN.pow_2_generator(lc)
        code = S.reed_solomon(DV.to_device(D.shard_cyclic(coeffs, world, rank)), lc - 1, gc, ht)
        res["code"] = DV.from_device(code).tobytes()
        pf = S.fri_prove(code, lc, Transcript(), ht, gather_log=cfg["gather_log"])
        res["proof"] = (bytes(pf._commit), bytes(pf._q), list(pf._idx), bytes(pf.c.last_elem),
                        bytes(pf.c.last_random), pf.verify())
        # sumcheck
        n = cfg["n_sc"]
        ev = DV.random_limbs(1 << n, seed=21)
        rr = random.Random(4)
        pts = [rr.randrange(D.M) for _ in range(n)]
        d = S.eq_table(pts, ht)
        tr = Transcript()
        m_loc = DV.to_device(D.shard_cyclic(ev, world, rank))
        polys, rs = S.sumcheck_prove(m_loc, d, n, 777, tr, ht)
        res["sc"] = (polys, rs, tr.random())
        res["folded"] = (DV.from_device(m_loc[:1]).tobytes(), DV.from_device(d[:1]).tobytes())
        res["queries"] = [pf.query(q) for q in range(MF.NUM_QUERIES)] if rank == 0 else None
        if rank == 0:  # single-GPU references
            ref = {"ntt": DV.from_device(MN.Polynomial(DV.to_device(x)).ntt(g).evals),
                   "code": DV.from_device(MF.reed_solomon(DV.to_device(coeffs), gc))}
            rp = FriProof.prove(MF.reed_solomon(DV.to_device(coeffs), gc), Transcript())
            ref["proof"] = (bytes(rp._commit), bytes(rp._q), list(rp._idx), bytes(rp.c.last_elem),
                            bytes(rp.c.last_random))
            tab = MS.SumcheckTables(DV.to_device(ev), MPL.eq_table(pts))
            t2 = Transcript()
            p2, r2 = tab.compute_sumcheck_polynomials(777, t2)
            ref["sc"] = (p2, r2, t2.random())
            res["ref"] = ref
        torch.cuda.synchronize()
        q.put((rank, res))
    except Exception:
        import traceback

        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("world,cfg", [
    (2, dict(log_ntt=14, log_code=16, gather_log=8, n_sc=10)),
    (4, dict(log_ntt=16, log_code=20, gather_log=12, n_sc=12)),
    (4, dict(log_ntt=12, log_code=12, gather_log=16, n_sc=3)),
])
def test_sharded_capi_multiprocess(world, cfg):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=300) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
    for r in range(world):
        assert "error" not in res[r], res[r].get("error")
    ref = res[0].pop("ref")
    ln, lc = cfg["log_ntt"], cfg["log_code"]
    # the single-GPU references are themselves checked against the C oracle on
    # the same inputs (worker seeds 31 / 11)
    from multilinear_amd import ntt as MN

    x = DV.random_limbs(1 << ln, seed=31)
    assert (C.ntt(x, ln, MN.pow_2_generator(ln)) == ref["ntt"]).all()
    coeffs = DV.random_limbs(1 << (lc - 1), seed=11)
    assert (C.reed_solomon(coeffs, lc - 1, MN.pow_2_generator(lc)) == ref["code"]).all()
    parts = [np.frombuffer(res[r]["ntt"], dtype=np.uint32).reshape(-1, 4) for r in range(world)]
    assert (D.unshard_blocks(parts, ln - 2 * (world.bit_length() - 1)) == ref["ntt"]).all()
    parts = [np.frombuffer(res[r]["code"], dtype=np.uint32).reshape(-1, 4) for r in range(world)]
    assert (D.unshard_blocks(parts, lc - 2 * (world.bit_length() - 1)) == ref["code"]).all()
    for r in range(world):
        assert res[r]["intt_ok"], "rank %d: INTT(NTT(x)) != x" % r
        assert res[r]["proof"][5], "rank %d proof rejected" % r
        assert res[r]["proof"][:5] == ref["proof"], "rank %d: proof differs from single GPU" % r
        assert res[r]["sc"] == ref["sc"], "rank %d: sumcheck differs from single GPU" % r
    _check_against_oracle(res, world, cfg)


def _check_against_oracle(res, world, cfg):
    """The sharded results against the oracle (not only against single GPU)."""
    import random

    from oracle import field as F
    from oracle import fri as OF
    from oracle import polynomials as OPL
    from oracle import transcript as OT

    lc, n = cfg["log_code"], cfg["n_sc"]
    coeffs = DV.random_limbs(1 << (lc - 1), seed=11)
    code = C.reed_solomon(coeffs, lc - 1, F.pow_2_generator(lc))
    roots, last, _, rc = C.fri_commit_par(code, lc)
    assert rc == 0
    for r in range(world):
        commit, _, _, last_b, _, _ = res[r]["proof"]
        assert [commit[32 * i:32 * i + 32] for i in range(len(roots))] == roots, \
            "rank %d: FRI commitments differ from the C oracle" % r
        assert int.from_bytes(last_b, "little") == last, "rank %d: last element differs" % r
    if lc <= 16:  # the Python oracle's whole proof, query paths included
        ints = [int.from_bytes(code[i].tobytes(), "little") for i in range(1 << lc)]
        want = OF.FriProof.prove(ints, F.pow_2_generator_powers(lc), OT.Transcript())
        commit, _, _, last_b, last_r, _ = res[0]["proof"]
        assert commit == b"".join(want.commitments)
        assert last_r == want.last_random
        for q, gq in enumerate(res[0]["queries"]):
            wq = want.queries[q]
            assert len(gq) == len(wq)
            for (gv, gs), (wv, wpath) in zip(gq, wq):
                assert gv == wv
                assert gs == [s for s, _ in wpath]
    # sumcheck: the reference round loop on the C oracle, claim 777
    ev = DV.random_limbs(1 << n, seed=21)
    rr = random.Random(4)
    pts = [rr.randrange(D.M) for _ in range(n)]
    m = ev.copy()
    d = C.eq_table_par(pts)
    tr = OT.Transcript()
    prev = 777
    want_polys, want_rs = [], []
    for k in range(n):
        lh = n - k
        s1, s2 = C.partial_sums_par(m, d, lh)
        pol = OPL.interpolate([(prev - s1) % F.M, s1, s2])
        for c in pol[1:]:
            tr.absorb(F.to_bytes(c))
        rch = tr.next_challenge()
        prev = OPL.uni_evaluate(pol, rch)
        want_polys.append(tuple(pol[1:]))
        want_rs.append(rch)
        C.fold_par(m, d, lh, rch)
        m, d = m[: 1 << (lh - 1)], d[: 1 << (lh - 1)]
    for r in range(world):
        polys, rs, rnd = res[r]["sc"]
        assert [tuple(p) for p in polys] == want_polys, "rank %d: round polynomials" % r
        assert list(rs) == want_rs, "rank %d: challenges" % r
        assert rnd == tr.random(), "rank %d: final transcript" % r
        assert res[r]["folded"] == (m[0].tobytes(), d[0].tobytes()), \
            "rank %d: the folded tables' m(r), d(r)" % r


def _rccl_worker(port, q):
    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    tdist.init_process_group("gloo", rank=0, world_size=1)
    try:
        from multilinear_amd import ntt as MN

        comm = S.RcclComm.from_torch()
        t = comm.transport
        assert (t.world, t.rank) == (1, 0)
        x = DV.random_device(1 << 20, 5)
        y = torch.empty_like(x)
        st = torch.cuda.current_stream().cuda_stream
        ok_a2a = t.all_to_all(t.user, DV.ptr(x), DV.ptr(y), x.numel() * 4, st) == 0
        torch.cuda.synchronize()
        same_a2a = bool(torch.equal(x, y))
        z = torch.empty_like(x[:4096])
        ok_ag = t.all_gather(t.user, DV.ptr(x), DV.ptr(z), z.numel() * 4, st) == 0
        torch.cuda.synchronize()
        same_ag = bool(torch.equal(z, x[:4096]))
        g = MN.pow_2_generator(16)
        xs = DV.random_device(1 << 16, 6)
        same_ntt = bool(torch.equal(S.ntt(xs, 16, g, comm), MN.Polynomial(xs).ntt(g).evals))
        comm.close()
        q.put(dict(ok_a2a=ok_a2a, same_a2a=same_a2a, ok_ag=ok_ag, same_ag=same_ag, same_ntt=same_ntt))
    except Exception:
        import traceback

        q.put({"error": traceback.format_exc()})
    finally:
        tdist.destroy_process_group()


def test_rccl_comm_world1_transport():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    try:
        res = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert "error" not in res, res.get("error")
    assert all(res.values()), res


def _rccl_nccl_worker(port, q):
    """As the driver's N > 1 bench: torch.distributed on its nccl (RCCL)
    backend, eagerly initialised on the device, and libmlhip's own RCCL
    communicator beside it (one librccl.so.1 in the process)."""
    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        comm = S.RcclComm.from_torch()
        info = comm.info()
        bad, ms = S.preflight(comm, 1 << 20)
        v = torch.ones(1024, device="cuda")
        tdist.all_reduce(v)  # torch's communicator still works after ours ran
        torch.cuda.synchronize()
        comm.close()
        q.put(dict(info=info, bad=bad, ms=ms, torch_ok=bool(torch.all(v == 1.0))))
    except Exception:
        import traceback

        q.put({"error": traceback.format_exc()})
    finally:
        tdist.destroy_process_group()


def test_rccl_comm_beside_torch_nccl_backend():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_nccl_worker, args=(_free_port(), q))
    p.start()
    try:
        res = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert "error" not in res, res.get("error")
    assert res["info"]["ranks"] == 1 and res["info"]["transport"] == "rccl"
    assert res["bad"] == 0 and res["ms"] >= 0.0 and res["torch_ok"]
