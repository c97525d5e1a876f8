"""GPU tests of the sharded path (multilinear_amd/dist.py, libmlhip mlh_shard_*).

* In-process emulation of P ranks on one GPU: every rank-local HIP step runs
  through the C ABI, the all-to-all is done by slicing -- the sharded NTT /
  INTT / RS must equal the single-GPU transform bit for bit.
* Real multi-process runs (2 and 4 processes sharing the one GPU, gloo with
  host-staged buffers standing in for RCCL): the sharded FRI proof must equal
  the single-GPU mlh_fri_prove proof byte for byte and pass the verifier.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

from multilinear_amd import device as DV  # noqa: E402
from multilinear_amd import dist as D  # noqa: E402
from multilinear_amd import ntt as MN  # noqa: E402
from multilinear_amd.fri import FriProof  # noqa: E402
from multilinear_amd.transcript import Transcript  # noqa: E402

M = D.M


class _Emu:
    """P ranks in one process: all_to_all by slicing (list of tensors)."""

    def __init__(self, P):
        self.world = P

    def all_to_all(self, parts):
        P = self.world
        chunks = [p.chunk(P, 0) for p in parts]
        return [torch.cat([chunks[s][d] for s in range(P)], 0) for d in range(P)]


def _emu_ntt(xs, log_n, gen, ops, P):
    zs = [ops.ntt(x, pow(gen, P, M)) for x in xs]
    recv = _Emu(P).all_to_all(zs)
    return [ops.cross(recv[r], log_n, P.bit_length() - 1, r, gen, False) for r in range(P)]


def _emu_intt(Xs, log_n, gen, ops, P):
    ys = [ops.cross(Xs[r], log_n, P.bit_length() - 1, r, gen, True) for r in range(P)]
    zs = _Emu(P).all_to_all(ys)
    return [ops.ntt(z, pow(gen, P, M), inverse=True) for z in zs]


@pytest.mark.parametrize("P,log_n", [(2, 4), (2, 12), (4, 8), (4, 20), (8, 6), (8, 21), (16, 8),
                                     (16, 18)])
def test_sharded_ntt_emulated(P, log_n):
    ops = D.HipOps(0)
    x = DV.random_limbs(1 << log_n, seed=log_n * 31 + P)
    gen = MN.pow_2_generator(log_n)
    want = DV.from_device(MN.Polynomial(DV.to_device(x)).ntt(gen).evals)
    xs = [DV.to_device(D.shard_cyclic(x, P, r)) for r in range(P)]
    Xs = _emu_ntt(xs, log_n, gen, ops, P)
    log_s = D.cross_log_s(log_n, P.bit_length() - 1)
    got = D.unshard_blocks([DV.from_device(t) for t in Xs], log_s)
    assert np.array_equal(got, want)
    back = _emu_intt(Xs, log_n, gen, ops, P)
    for r in range(P):
        assert np.array_equal(DV.from_device(back[r]), D.shard_cyclic(x, P, r))


@pytest.mark.parametrize("P,log_n", [(2, 11), (8, 19)])
def test_sharded_rs_emulated(P, log_n):
    ops = D.HipOps(0)
    c = DV.random_limbs(1 << log_n, seed=5)
    gen = MN.pow_2_generator(log_n + 1)
    from multilinear_amd import fri as MF

    want = DV.from_device(MF.reed_solomon(DV.to_device(c), gen))
    g2 = pow(gen, P, M)
    zs = [ops.reed_solomon(DV.to_device(D.shard_cyclic(c, P, r)), g2) for r in range(P)]
    recv = _Emu(P).all_to_all(zs)
    lp = P.bit_length() - 1
    outs = [DV.from_device(ops.cross(recv[r], log_n + 1, lp, r, gen, False)) for r in range(P)]
    assert np.array_equal(D.unshard_blocks(outs, D.cross_log_s(log_n + 1, lp)), want)


def test_shard_cross_rejects_bad_args():
    from multilinear_amd import _lib

    ops = D.HipOps(0)
    x = DV.to_device(DV.random_limbs(16, 1))
    gen = MN.pow_2_generator(4)
    with pytest.raises(_lib.MlhError):
        ops.cross(x, 4, 3, 0, gen, False)  # log_n < 2 log_p
    with pytest.raises(_lib.MlhError):
        ops.cross(x, 4, 2, 0, MN.pow_2_generator(5), False)  # wrong order
    with pytest.raises(_lib.MlhError):
        ops.cross(x, 4, 2, 4, gen, False)  # rank out of range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, log_c, gather_log, q):
    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        tp, ops = D.Transport(host_staged=True), D.HipOps(0)
        log_n = log_c - 1
        coeffs = DV.random_limbs(1 << log_n, seed=11)
        gen = MN.pow_2_generator(log_c)
        local = DV.to_device(D.shard_cyclic(coeffs, world, rank))
        enc = D.reed_solomon(local, log_n, gen, tp, ops)
        proof = D.fri_prove(enc, log_c, Transcript(), tp, ops, gather_log=gather_log)
        torch.cuda.synchronize()
        res = {"commit": bytes(proof._commit), "q": bytes(proof._q), "idx": list(proof._idx),
               "last": bytes(proof.c.last_elem), "lr": bytes(proof.c.last_random),
               "ok": proof.verify()}
        if rank == 0:  # the single-GPU proof of the natural-order codeword
            from multilinear_amd import fri as MF

            code = MF.reed_solomon(DV.to_device(coeffs), gen)
            ref = FriProof.prove(code, Transcript())
            res["ref"] = {"commit": bytes(ref._commit), "q": bytes(ref._q),
                          "idx": list(ref._idx), "last": bytes(ref.c.last_elem),
                          "lr": bytes(ref.c.last_random)}
        q.put((rank, res))
    except Exception:
        import traceback

        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("world,log_c,gather_log", [(2, 16, 8), (4, 20, 12), (4, 12, 16)])
def test_sharded_fri_prove_multiprocess(world, log_c, gather_log):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, log_c, gather_log, q))
             for r in range(world)]
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
    for r in range(world):
        assert res[r]["ok"], "rank %d proof rejected" % r
        for key in ("commit", "q", "idx", "last", "lr"):
            assert res[r][key] == ref[key], "rank %d: %s differs from single-GPU proof" % (r, key)


def _sc_worker(rank, world, port, n, q):
    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import random

        from multilinear_amd import polynomials as MPL
        from multilinear_amd import sumcheck as MS

        torch.cuda.set_device(0)
        tp, ops = D.Transport(host_staged=True), D.HipOps(0)
        ev = DV.random_limbs(1 << n, seed=21)
        rr = random.Random(4)
        pts = [rr.randrange(M) for _ in range(n)]
        m = DV.to_device(D.shard_cyclic(ev, world, rank))
        d = D.eq_table(pts, tp, ops)
        tr = Transcript()
        polys, rs = D.sumcheck_prove(m, d, n, 777, tr, tp, ops)
        res = {"polys": polys, "rs": rs, "lr": tr.random()}
        if rank == 0:
            x = DV.to_device(ev)
            tab = MS.SumcheckTables(x.clone(), MPL.eq_table(pts))
            t2 = Transcript()
            rp, rr2 = tab.compute_sumcheck_polynomials(777, t2)
            res["ref"] = {"polys": rp, "rs": rr2, "lr": t2.random()}
        q.put((rank, res))
    except Exception:
        import traceback

        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 18), (4, 20)])
def test_sharded_sumcheck_multiprocess(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sc_worker, args=(r, world, port, n, q)) for r in range(world)]
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
    for r in range(world):
        assert [tuple(p) for p in res[r]["polys"]] == [tuple(p) for p in ref["polys"]]
        assert res[r]["rs"] == ref["rs"] and res[r]["lr"] == ref["lr"]


def _pipe_worker(rank, world, port, log_n, q):
    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        tp, ops = D.Transport(host_staged=True), D.HipOps(0)
        gen = MN.pow_2_generator(log_n)
        xs = [DV.to_device(D.shard_cyclic(DV.random_limbs(1 << log_n, seed=s), world, rank))
              for s in range(4)]
        pipe = D.NttPipeline(log_n, gen, tp, ops)
        outs = []
        for x in xs:
            outs += pipe.submit(x)
        outs += pipe.drain()
        ref = [D.ntt(x, log_n, gen, tp, ops) for x in xs]
        torch.cuda.synchronize()
        q.put((rank, {"ok": all(torch.equal(a, b) for a, b in zip(outs, ref)) and len(outs) == 4}))
    except Exception:
        import traceback

        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        tdist.destroy_process_group()


def test_ntt_pipeline_matches_sharded_ntt():
    world, log_n = 2, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, log_n, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=300) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
    for r in range(world):
        assert "error" not in res[r], res[r].get("error")
        assert res[r]["ok"]


def _rccl_worker(port, q):
    """World-1 RCCL communicator: the device-to-device collectives the sharded
    path issues at N > 1 (Transport(host_staged=False)), on HBM tensors."""
    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert tdist.get_backend() == "nccl"
        tp = D.Transport(host_staged=False)
        x = DV.random_device(1 << 24, 99)  # 256 MiB: the per-GPU shard the bench exchanges
        y = tp.all_to_all(x)
        g = tp.all_gather(x[: 1 << 12])
        nb = tp.gather_bytes(b"\x01\x02roots")
        torch.cuda.synchronize()
        res = {"a2a_same": bool(torch.equal(x, y)), "a2a_dev": y.device.type,
               "ag_same": bool(torch.equal(g, x[: 1 << 12])), "ag_dev": g.device.type,
               "bytes": nb}
        q.put(res)
    except Exception:
        import traceback

        q.put({"error": traceback.format_exc()})
    finally:
        tdist.destroy_process_group()


def test_rccl_world1_device_collectives():
    """The nccl (= RCCL) backend runs here before the driver's 8-GPU node: an
    all_to_all_single of a 256 MiB shard, all_gather_into_tensor and the byte
    gather, all on device tensors, through the same Transport the sharded NTT /
    FRI / sumcheck use."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    try:
        res = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert "error" not in res, res.get("error")
    assert res["a2a_same"] and res["a2a_dev"] == "cuda"
    assert res["ag_same"] and res["ag_dev"] == "cuda"
    assert res["bytes"] == [b"\x01\x02roots"]
