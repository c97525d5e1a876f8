"""Multi-GPU prover entry points of the C ABI (libmlhip ``mlh_sharded_*``):
thin callers of the C++ schedules in csrc/sharded.hip, one process per GPU.

Transports (``mlh_transport``):
  * ``RcclComm`` -- the library's RCCL communicator (device-to-device over
    xGMI); the 128-byte ncclUniqueId travels over the caller's existing
    torch.distributed group.
  * ``HostTransport`` -- collectives of a ``multilinear_amd.dist.Transport``
    (torch.distributed, e.g. gloo) run as C callbacks on host copies; used by
    the multi-process tests that share one GPU.

Layouts are those of ``multilinear_amd.dist`` (its Python schedule is the
executable spec the CPU tests check against the oracle): cyclic in for
NTT / RS / sumcheck, block 2^log_n / P^2 out of NTT / RS and into FRI.
"""
import ctypes

import numpy as np

from . import _lib
from .device import check, context, empty, fe_bytes, fe_from_bytes, lib, ptr
from .fri import FriProof

M = 340282366920938463463374557953744961537


def _log2(n):
    if n < 1 or n & (n - 1):
        raise ValueError("size must be a power of two")
    return n.bit_length() - 1


class RcclComm:
    """An RCCL communicator owned by libmlhip (mlh_comm_create)."""

    def __init__(self, world, rank, unique_id: bytes, device=0):
        ctx = context(device)
        h = ctypes.c_void_p()
        idb = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        check(lib().mlh_comm_create(ctx, world, rank, idb, ctypes.byref(h)), ctx)
        self.h = h.value
        self.world, self.rank = world, rank
        self.c = _lib.TransportC()
        check(lib().mlh_comm_transport(self.h, ctypes.byref(self.c)))

    @staticmethod
    def from_torch(group=None, device=0):
        """Rank 0 makes the unique id; it is broadcast over ``group``."""
        import torch
        import torch.distributed as dist

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        buf = (ctypes.c_uint8 * 128)()
        if rank == 0:
            check(lib().mlh_comm_unique_id(buf))
        dev = "cuda:%d" % device if dist.get_backend(group) == "nccl" else "cpu"
        t = torch.tensor(list(bytes(buf)), dtype=torch.uint8, device=dev)
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        return RcclComm(world, rank, bytes(t.cpu().numpy().tobytes()), device)

    @property
    def transport(self):
        return self.c

    def close(self):
        if self.h:
            lib().mlh_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostTransport:
    """mlh_transport over a multilinear_amd.dist.Transport (torch.distributed):
    device buffers are copied to the host, exchanged, copied back."""

    def __init__(self, tp, device=0):
        import torch

        self.tp, self.device = tp, device
        ctx = context(device)

        def to_host(src, nbytes):
            a = np.empty(nbytes, dtype=np.uint8)
            if nbytes:
                check(lib().mlh_memcpy_d2h(ctx, a.ctypes.data_as(ctypes.c_void_p), src, nbytes), ctx)
            return torch.from_numpy(a)

        def to_dev(dst, t):
            a = np.ascontiguousarray(t.numpy())
            if a.nbytes:
                check(lib().mlh_memcpy_h2d(ctx, dst, a.ctypes.data_as(ctypes.c_void_p), a.nbytes), ctx)

        def a2a(user, send, recv, per, stream):
            try:
                src = to_host(send, per * tp.world)
                out = torch.empty_like(src)
                tp.dist.all_to_all_single(out, src, group=tp.group)
                to_dev(recv, out)
                return 0
            except Exception:  # pragma: no cover - reported as MLH_ERR_COMM
                return 1

        def ag(user, send, recv, nbytes, stream):
            try:
                src = to_host(send, nbytes)
                out = torch.empty(nbytes * tp.world, dtype=torch.uint8)
                tp.dist.all_gather_into_tensor(out, src, group=tp.group)
                to_dev(recv, out)
                return 0
            except Exception:  # pragma: no cover
                return 1

        self._a2a = _lib.ALL_TO_ALL_FN(a2a)  # keep the callbacks alive
        self._ag = _lib.ALL_GATHER_FN(ag)
        self.c = _lib.TransportC(tp.world, tp.rank, 1, None, self._a2a, self._ag)

    @property
    def transport(self):
        return self.c


def _tp(transport):
    return ctypes.byref(transport.transport)


def ntt(x_local, log_n, gen, transport, inverse=False, device=0):
    """Sharded Polynomial::ntt (cyclic in, block 2^log_n / P^2 out) or, with
    inverse, LagrangePolynomial::intt (block in, cyclic out)."""
    ctx = context(device)
    out = empty(x_local.shape[0], device)
    check(lib().mlh_sharded_ntt(ctx, _tp(transport), ptr(x_local), ptr(out), log_n, fe_bytes(gen),
                                1 if inverse else 0), ctx)
    return out


def reed_solomon(coeffs_local, log_n, gen, transport, device=0):
    """Sharded reed_solomon of 2^log_n coefficients (cyclic) -> block-layout code."""
    ctx = context(device)
    out = empty(2 * coeffs_local.shape[0], device)
    check(lib().mlh_sharded_reed_solomon(ctx, _tp(transport), ptr(coeffs_local), log_n, fe_bytes(gen),
                                         ptr(out)), ctx)
    return out


def fri_prove(code_local, log_code, transcript, transport, gather_log=16, device=0):
    """Sharded FriProof::prove; every rank returns the same proof."""
    ctx = context(device)
    p = FriProof(log_code)
    check(lib().mlh_sharded_fri_prove(ctx, _tp(transport), ptr(code_local), log_code, gather_log,
                                      transcript.h, ctypes.byref(p.c)), ctx)
    return p


def eq_table(points, transport, device=0):
    """build_tables_for_pcs's delta in the cyclic layout (this rank's part)."""
    ctx = context(device)
    n = len(points)
    P = transport.transport.world
    out = empty(1 << (n - _log2(P)), device)
    pts = (ctypes.c_uint8 * max(16, 16 * n)).from_buffer_copy(
        b"".join(int(v).to_bytes(16, "little") for v in points) or bytes(16))
    check(lib().mlh_sharded_eq_table(ctx, _tp(transport), pts, n, ptr(out)), ctx)
    return out


def sumcheck_prove(m, d, n, total_sum, transcript, transport, device=0):
    """Sharded compute_sumcheck_polynomials -> ([(c1, c2)], [r]); m, d folded in place."""
    ctx = context(device)
    polys = (ctypes.c_uint8 * (32 * n))()
    rs = (ctypes.c_uint8 * (16 * n))()
    check(lib().mlh_sharded_sumcheck_prove(ctx, _tp(transport), ptr(m), ptr(d), n, fe_bytes(total_sum),
                                           transcript.h, polys, rs), ctx)
    P, R = bytes(polys), bytes(rs)
    return ([(fe_from_bytes(P[32 * k:32 * k + 16]), fe_from_bytes(P[32 * k + 16:32 * k + 32]))
             for k in range(n)],
            [fe_from_bytes(R[16 * k:16 * k + 16]) for k in range(n)])
