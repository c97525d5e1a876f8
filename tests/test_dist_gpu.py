"""GPU tests of the sharded building blocks (libmlhip mlh_shard_*).

* In-process emulation of P ranks on one GPU: every rank-local HIP step runs
  through the C ABI, the all-to-all is done by slicing -- the sharded NTT /
  INTT / RS must equal the single-GPU transform bit for bit.
* The nccl (RCCL) backend at world 1 through the spec's Transport.
The whole C++ schedules (mlh_sharded_*) are tested in test_sharded_capi_gpu.py
(processes over gloo) and test_sharded_threads_gpu.py (P ranks as threads with
device-ordered collectives, as RCCL orders them).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

from multilinear_amd import device as DV  # noqa: E402
from tests import dist_spec as D  # noqa: E402
from multilinear_amd import ntt as MN  # noqa: E402

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
