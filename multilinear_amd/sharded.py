"""Multi-GPU prover entry points of the C ABI (libmlhip ``mlh_sharded_*``):
thin callers of the C++ schedules in csrc/sharded.hip, one process per GPU.

Transports (``mlh_transport``):
  * ``RcclComm`` -- the library's RCCL communicator (device-to-device over
    xGMI); the 128-byte ncclUniqueId travels over the caller's existing
    torch.distributed group.
  * ``HostTransport`` -- collectives of a ``Transport`` (torch.distributed,
    e.g. gloo) run as C callbacks on host copies; used by the multi-process
    tests that share one GPU and by the bench's gloo rehearsal.

Layouts: a vector of n = 2^log_n elements over P = 2^p ranks is
block-cyclic with block S = 2^log_s: local index l of rank r holds global index
((l >> log_s) << (log_s + p)) | (r << log_s) | (l mod S).  Cyclic (S = 1) in
for NTT / RS / sumcheck, block 2^log_n / P^2 out of NTT / RS and into FRI.
The host helpers below shard / reassemble natural-order arrays in them.  The
same schedules restated in Python (tests/dist_spec.py) are the executable
spec the CPU gloo tests check against the oracle.
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


# ---------------------------------------------------------------------------
# transport
# ---------------------------------------------------------------------------

class Transport:
    """The collectives of the sharded path, on torch.distributed.

    ``host_staged`` copies device tensors through host memory around each
    collective (gloo with GPU buffers, e.g. several ranks sharing one GPU in
    the tests); with ``nccl`` (RCCL) tensors go device to device over xGMI."""

    def __init__(self, group=None, host_staged=False):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.host_staged = host_staged
        if self.world & (self.world - 1) or self.world > 16:
            raise ValueError("world size must be a power of two <= 16")

    def _stage(self, t):
        return t.cpu() if self.host_staged else t

    def all_to_all(self, t):
        """Chunk i of ``t`` (dim 0 split in world equal parts) goes to rank i;
        chunk i of the result came from rank i."""
        import torch

        src = self._stage(t)
        out = torch.empty_like(src)
        self.dist.all_to_all_single(out, src.contiguous(), group=self.group)
        return out.to(t.device) if self.host_staged else out

    def all_gather(self, t):
        """Concatenation over ranks (rank order) along dim 0."""
        import torch

        src = self._stage(t).contiguous()
        out = torch.empty((self.world * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype,
                          device=src.device)
        self.dist.all_gather_into_tensor(out, src, group=self.group)
        return out.to(t.device) if self.host_staged else out

    def gather_bytes(self, data: bytes):
        """All-gather equal-length host byte strings -> list per rank."""
        import torch

        dev = "cpu" if self.host_staged or self.dist.get_backend(self.group) == "gloo" else \
            "cuda:%d" % torch.cuda.current_device()
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev) if data else \
            torch.zeros(0, dtype=torch.uint8, device=dev)
        g = self.all_gather(t).cpu().numpy().tobytes()
        n = len(data)
        return [g[i * n:(i + 1) * n] for i in range(self.world)]


# ---------------------------------------------------------------------------
# layouts
# ---------------------------------------------------------------------------

def block_owner(i, log_s, log_p):
    """(rank, local index) of global index i in the block-(2^log_s) layout."""
    r = (i >> log_s) & ((1 << log_p) - 1)
    l = ((i >> (log_s + log_p)) << log_s) | (i & ((1 << log_s) - 1))
    return r, l


def shard_cyclic(x, world, rank):
    """Host helper: rank's part of a natural-order array in the cyclic layout."""
    return np.ascontiguousarray(x[rank::world])


def shard_blocks(x, world, rank, log_s):
    """Host helper: rank's part of a natural-order array in the block layout."""
    S = 1 << log_s
    return np.ascontiguousarray(x.reshape(-1, world, S, *x.shape[1:])[:, rank].reshape(
        -1, *x.shape[1:]))


def unshard_blocks(parts, log_s):
    """Host helper: natural order from all ranks' block-layout parts."""
    S = 1 << log_s
    P = len(parts)
    st = np.stack([p.reshape(-1, S, *p.shape[1:]) for p in parts], axis=1)
    return st.reshape(-1, *parts[0].shape[1:])


def cross_log_s(log_n, log_p):
    return log_n - 2 * log_p


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

    def info(self):
        """What RCCL reports for this communicator: {"ranks", "rank", "device"}
        (ncclCommCount / ncclCommUserRank / ncclCommCuDevice)."""
        n, r, d = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int()
        check(lib().mlh_comm_info(self.h, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d)))
        return {"ranks": n.value, "rank": r.value, "device": d.value, "transport": "rccl"}

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
    """mlh_transport over a Transport (torch.distributed, host-staged):
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

    def info(self):
        return {"ranks": self.tp.world, "rank": self.tp.rank, "device": self.device,
                "transport": "host-staged torch.distributed (%s)" % self.tp.dist.get_backend(self.tp.group)}


def preflight(transport, bytes_per_rank, device=0, ctx=None):
    """mlh_comm_preflight: one all-to-all and one all-gather of a rank-tagged
    pattern through the transport, checked on the device -> (mismatched words
    on this rank, ms of the two collectives).  ctx: the rank's own context when
    several ranks share a process (a context is not thread-safe)."""
    ctx = ctx or context(device)
    bad, ms = ctypes.c_uint64(), ctypes.c_float()
    check(lib().mlh_comm_preflight(ctx, _tp(transport), bytes_per_rank, ctypes.byref(bad),
                                   ctypes.byref(ms)), ctx)
    return bad.value, ms.value


def ntt_block_owner(j, log_total, log_p, log_s=None):
    """(rank, local index) holding X[j] of a sharded forward NTT: block
    2^(log_total - 2 log_p) output layout (mlh_sharded_ntt(_batch), DESIGN.md
    section 6), or block 2^log_s (mlh_sharded_ntt_fused_batch reports it)."""
    if log_s is None:
        log_s = log_total - 2 * log_p
    r = (j >> log_s) & ((1 << log_p) - 1)
    return r, ((j >> (log_s + log_p)) << log_s) | (j & ((1 << log_s) - 1))


def ntt_spot_terms(x_local, log_total, gen, rank, world, js, device=0, ctx=None):
    """This rank's share of X[j] = NTT(x)[j] = sum_i x_i gen^(i j) for each j
    in ``js``, x cyclic over the ranks (rank g holds x[g + P m]): X[j] =
    sum_g gen^(j g) poly_g(gen^(j P)), poly_g the rank's local coefficients as
    a polynomial (Polynomial::evaluate, ntt/mod.rs:61-67, on the device:
    mlh_poly_evaluate).  The sum over ranks mod M of these terms is X[j] -- an
    independent check of a sharded transform's output at a few points.
    ctx: an explicit mlh context (default: the device's)."""
    ctx = ctx if ctx is not None else context(device)
    n = x_local.shape[0]
    out = (ctypes.c_uint8 * 16)()
    terms = []
    for j in js:
        pt = pow(gen, j * world, M)
        check(lib().mlh_poly_evaluate(ctx, ptr(x_local), n, fe_bytes(pt), out), ctx)
        terms.append(fe_from_bytes(out) * pow(gen, j * rank, M) % M)
    return terms


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


def ntt_batch(xs_local, outs_local, log_n, gen, transport, inverse=False, device=0):
    """mlh_sharded_ntt_batch: len(xs_local) sharded transforms, xs[i] -> outs[i],
    the exchange of transform i overlapping the local step of i + 1 (enqueued;
    the context stream is ordered after all of them on return)."""
    ctx = context(device)
    n = len(xs_local)
    if len(outs_local) != n:
        raise ValueError("one output per input")
    ins = (ctypes.c_void_p * max(1, n))(*[ptr(x) for x in xs_local])
    outs = (ctypes.c_void_p * max(1, n))(*[ptr(y) for y in outs_local])
    check(lib().mlh_sharded_ntt_batch(ctx, _tp(transport), ins, outs, n, log_n, fe_bytes(gen),
                                      1 if inverse else 0), ctx)
    return outs_local


def reed_solomon(coeffs_local, log_n, gen, transport, device=0):
    """Sharded reed_solomon of 2^log_n coefficients (cyclic) -> block-layout code."""
    ctx = context(device)
    out = empty(2 * coeffs_local.shape[0], device)
    check(lib().mlh_sharded_reed_solomon(ctx, _tp(transport), ptr(coeffs_local), log_n, fe_bytes(gen),
                                         ptr(out)), ctx)
    return out


def commit_rs_code(code_local, log_code, transport, device=0):
    """commit_rs_code + Merkle::commit of a block-layout codeword -> the root
    (32 bytes, the same on every rank)."""
    ctx = context(device)
    root = (ctypes.c_uint8 * 32)()
    check(lib().mlh_sharded_commit_rs_code(ctx, _tp(transport), ptr(code_local), log_code, root), ctx)
    return bytes(root)


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
