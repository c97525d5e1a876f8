"""Executable specification of the multi-GPU schedules (TEST INFRASTRUCTURE).

The product implementation is C++ behind the C ABI (multilinear_amd/csrc/
sharded.hip: mlh_sharded_*), which a Rust caller binds; this module states the
same schedules in Python so that the CPU tests (tests/test_dist_cpu.py) can run
them over gloo with world sizes 2/4/8 and oracle rank-local steps
(tests/dist_cpu_ops.py), and the GPU tests with the C ABI's rank-local steps.
Nothing in multilinear_amd/ or bench.py imports it.

The reference (fr34za/multilinear) is single-node CPU code; its prover API is
``Polynomial::ntt`` / ``reed_solomon`` (src/ntt/mod.rs:69-108, src/fri/mod.rs:19-28)
and ``FriProof::prove`` (src/fri/mod.rs:261-285).  This module runs the same
computations on P = 2^p GPUs with rank-local HIP kernels (libmlhip
``mlh_shard_*``) between torch.distributed collectives (RCCL over xGMI for
``nccl``; ``gloo`` for the CPU tests).  The proof it returns is byte-for-byte the
single-GPU / reference proof of the same (natural order) codeword.

Shard layouts ("Multi-GPU").  A vector of n = 2^log_n elements is
spread block-cyclically with block S = 2^log_s: local index l of rank r holds
global index ``((l >> log_s) << (log_s + p)) | (r << log_s) | (l mod S)``.

* ``ntt`` / ``reed_solomon`` take the cyclic layout (S = 1: rank g holds
  x[g], x[g+P], ...) and return block S = n / P^2 after ONE all-to-all:
  local NTT of length n/P with generator w^P, all-to-all of contiguous
  chunks, then a length-P DFT per column with twiddle w^(g j)
  (``mlh_shard_ntt_cross``).
* In the block-(n/P^2) layout every FRI pair (i, i + n/2) is local and every
  aligned run of S leaves is a local Merkle subtree, so each FRI layer folds
  and hashes locally; only the level-log_s subtree roots (P * T/2 digests,
  T = local blocks) are all-gathered and the few top levels hashed on the host
  (SURVEY.md 8(e) "the host hashes the top log2 P levels").
* Each fold halves the number of local blocks T.  When T reaches 1 the layer is
  in natural block order (rank r holds [r n/P, (r+1) n/P)); one all-to-all of
  that (P times smaller) layer re-deals it with block n/P^2 and the local
  folding continues.  Below ``gather_log`` the layer is all-gathered and the
  remaining layers run replicated on every rank.
* Query openings: the owning rank reads the pair and the subtree siblings from
  HBM (``mlh_merkle_open_pairs``), the top siblings come from the host top
  levels; the records are combined with one all-gather.
"""
import ctypes
import hashlib

import numpy as np

from multilinear_amd import _lib
from multilinear_amd.device import check, context, fe_bytes, lib, ptr
from multilinear_amd.sharded import (Transport, block_owner, cross_log_s, shard_blocks,  # noqa: F401
                                     shard_cyclic, unshard_blocks)

M = 340282366920938463463374557953744961537
LOG_BLOWUP = _lib.LOG_BLOWUP
NUM_QUERIES = _lib.NUM_QUERIES


def _log2(n):
    if n < 1 or n & (n - 1):
        raise ValueError("size must be a power of two")
    return n.bit_length() - 1


# ---------------------------------------------------------------------------
# rank-local HIP operations (libmlhip)
# ---------------------------------------------------------------------------

class HipOps:
    """Rank-local steps on device tensors: field vectors (n, 4) int32, trees
    uint8 ((2L - 1) * 32,).  Every call is a libmlhip kernel launch."""

    def __init__(self, device=0):
        self.device = device

    def _ctx(self):
        return context(self.device)

    def empty(self, n):
        import torch

        return torch.empty((n, 4), dtype=torch.int32, device="cuda:%d" % self.device)

    def empty_tree(self, leaves):
        import torch

        return torch.empty(int(lib().mlh_merkle_layers_bytes(leaves)), dtype=torch.uint8,
                           device="cuda:%d" % self.device)

    def ntt(self, x, gen, inverse=False):
        c = self._ctx()
        out = self.empty(x.shape[0])
        fn = lib().mlh_intt if inverse else lib().mlh_ntt
        check(fn(c, ptr(x), ptr(out), _log2(x.shape[0]), fe_bytes(gen)), c)
        return out

    def reed_solomon(self, coeffs, gen):
        c = self._ctx()
        out = self.empty(2 * coeffs.shape[0])
        check(lib().mlh_reed_solomon(c, ptr(coeffs), _log2(coeffs.shape[0]), fe_bytes(gen),
                                     ptr(out)), c)
        return out

    def cross(self, x, log_n, log_p, rank, gen, inverse):
        c = self._ctx()
        out = self.empty(x.shape[0])
        check(lib().mlh_shard_ntt_cross(c, ptr(x), ptr(out), log_n, log_p, rank, fe_bytes(gen),
                                        1 if inverse else 0), c)
        return out

    def commit_pairs(self, values):
        c = self._ctx()
        n = values.shape[0]
        tree = self.empty_tree(n // 2)
        check(lib().mlh_merkle_commit_pairs(c, ptr(values), _log2(n), ptr(tree), None), c)
        return tree

    def fold(self, values, k, log_domain, r, log_s, log_p, rank):
        c = self._ctx()
        n = values.shape[0]
        out = self.empty(n // 2)
        check(lib().mlh_shard_fri_fold(c, ptr(values), _log2(n), k, log_domain, fe_bytes(r),
                                       ptr(out), log_s, log_p, rank), c)
        return out

    def fold_commit(self, values, k, log_domain, r, log_s, log_p, rank):
        c = self._ctx()
        n = values.shape[0]
        out = self.empty(n // 2)
        tree = self.empty_tree(n // 4)
        check(lib().mlh_shard_fri_fold_commit(c, ptr(values), _log2(n), k, log_domain,
                                              fe_bytes(r), ptr(out), ptr(tree), log_s, log_p,
                                              rank), c)
        return out, tree

    # -- device-resident transcript and roots --
    def dev_transcript(self, transcript):
        import torch

        st = torch.empty(int(lib().mlh_device_transcript_bytes()), dtype=torch.uint8,
                         device="cuda:%d" % self.device)
        c = self._ctx()
        check(lib().mlh_transcript_to_device(c, transcript.h, ptr(st)), c)
        return st

    def absorb(self, state, src, challenge_out=None):
        """absorb the bytes of device tensor ``src``; next_challenge() -> challenge_out."""
        c = self._ctx()
        check(lib().mlh_device_transcript_absorb(
            c, ptr(state), ptr(src), src.numel() * src.element_size(),
            ptr(challenge_out) if challenge_out is not None else None), c)

    def fri_last(self, vals2, state, flag_out, last_out):
        c = self._ctx()
        check(lib().mlh_device_fri_last(c, ptr(vals2), ptr(state), ptr(flag_out), ptr(last_out)), c)

    def fold_dr(self, values, k, log_domain, r_dev, log_s, log_p, rank):
        c = self._ctx()
        n = values.shape[0]
        out = self.empty(n // 2)
        check(lib().mlh_shard_fri_fold_dr(c, ptr(values), _log2(n), k, log_domain, ptr(r_dev),
                                          ptr(out), log_s, log_p, rank), c)
        return out

    def fold_commit_dr(self, values, k, log_domain, r_dev, log_s, log_p, rank):
        c = self._ctx()
        n = values.shape[0]
        out = self.empty(n // 2)
        tree = self.empty_tree(n // 4)
        check(lib().mlh_shard_fri_fold_commit_dr(c, ptr(values), _log2(n), k, log_domain,
                                                 ptr(r_dev), ptr(out), ptr(tree), log_s, log_p,
                                                 rank), c)
        return out, tree

    def merkle_top(self, gathered, P, per_rank):
        c = self._ctx()
        levels = self.empty_tree(P * per_rank)
        check(lib().mlh_merkle_top(c, ptr(gathered), P, per_rank, ptr(levels)), c)
        return levels

    @staticmethod
    def tree_root(tree):
        return tree[-32:]

    @staticmethod
    def tree_level_dev(tree, leaves, level):
        off = sum(leaves >> i for i in range(level))
        return tree[32 * off:32 * (off + (leaves >> level))]

    @staticmethod
    def concat_bytes(parts):
        import torch

        return torch.cat(parts).cpu().numpy().tobytes()

    def tree_level(self, tree, leaves, level):
        """Digests of one level of a flattened tree (leaves first) -> bytes."""
        off = sum(leaves >> i for i in range(level))
        cnt = leaves >> level
        return tree[32 * off:32 * (off + cnt)].cpu().numpy().tobytes()

    def open_pairs(self, values, tree, levels, idx):
        c = self._ctx()
        nq = len(idx)
        rec = 32 * (1 + levels)
        out = (ctypes.c_uint8 * max(1, nq * rec))()
        ia = (ctypes.c_uint64 * max(1, nq))(*idx)
        check(lib().mlh_merkle_open_pairs(c, ptr(values), _log2(values.shape[0]), ptr(tree),
                                          levels, ia, nq, out), c)
        raw = bytes(out)
        return [raw[q * rec:(q + 1) * rec] for q in range(nq)]

    def to_host(self, values):
        return values.cpu().contiguous().numpy().view(np.uint32).reshape(-1, 4)

    # -- sumcheck (tables folded in place) --
    def eq_table(self, points):
        from multilinear_amd.polynomials import eq_table

        return eq_table(points, self.device)

    def scale(self, x, c):
        ctx = self._ctx()
        out = self.empty(x.shape[0])
        check(lib().mlh_field_scale(ctx, ptr(x), fe_bytes(c), ptr(out), x.shape[0]), ctx)
        return out

    def _pair(self, raw):
        b = bytes(raw)
        return int.from_bytes(b[:16], "little"), int.from_bytes(b[16:], "little")

    def const(self, v):
        from multilinear_amd.device import ints_to_limbs, to_device

        return to_device(ints_to_limbs([v]), self.device)

    def sc_sums_dev(self, m, d, log_h, out):
        c = self._ctx()
        check(lib().mlh_sumcheck_sums_dev(c, ptr(m), ptr(d), log_h, ptr(out)), c)

    def sc_fold_sums_dr(self, m, d, log_h, r_dev, out):
        c = self._ctx()
        check(lib().mlh_sumcheck_fold_sums_dr(c, ptr(m), ptr(d), log_h, ptr(r_dev), ptr(out)), c)

    def sc_fold_dr(self, m, d, log_h, r_dev):
        c = self._ctx()
        check(lib().mlh_sumcheck_fold_dr(c, ptr(m), ptr(d), log_h, ptr(r_dev)), c)

    def sc_round(self, pairs, npairs, prev, state, poly_out, r_out):
        c = self._ctx()
        check(lib().mlh_device_sumcheck_round(c, ptr(pairs), npairs, ptr(prev), ptr(state),
                                              ptr(poly_out), ptr(r_out)), c)

    def sc_sums(self, m, d):
        ctx = self._ctx()
        out = (ctypes.c_uint8 * 32)()
        check(lib().mlh_sumcheck_partial_sums(ctx, ptr(m), ptr(d), _log2(m.shape[0]), out), ctx)
        return self._pair(out)

    def sc_fold_and_sums(self, m, d, log_h, r):
        ctx = self._ctx()
        out = (ctypes.c_uint8 * 32)()
        check(lib().mlh_sumcheck_fold_and_sums(ctx, ptr(m), ptr(d), log_h, fe_bytes(r), out), ctx)
        return self._pair(out)

    def sc_fold(self, m, d, log_h, r):
        ctx = self._ctx()
        check(lib().mlh_sumcheck_fold(ctx, ptr(m), ptr(d), log_h, fe_bytes(r)), ctx)

    def sync(self):
        import torch

        torch.cuda.synchronize(self.device)


# ---------------------------------------------------------------------------
# sharded NTT / RS
# ---------------------------------------------------------------------------

def ntt(x_local, log_n, gen, tp, ops):
    """Polynomial::ntt (ntt/mod.rs:69-110) of a 2^log_n vector in the cyclic
    layout -> evaluations in the block-(2^log_n / P^2) layout."""
    P = tp.world
    if P == 1:
        return ops.ntt(x_local, gen)
    z = ops.ntt(x_local, pow(gen, P, M))
    recv = tp.all_to_all(z)
    return ops.cross(recv, log_n, _log2(P), tp.rank, gen, False)


def intt(X_local, log_n, gen, tp, ops):
    """LagrangePolynomial::intt (ntt/mod.rs:132-173): block-(n/P^2) layout in,
    cyclic layout out."""
    P = tp.world
    if P == 1:
        return ops.ntt(X_local, gen, inverse=True)
    y = ops.cross(X_local, log_n, _log2(P), tp.rank, gen, True)
    z = tp.all_to_all(y)
    return ops.ntt(z, pow(gen, P, M), inverse=True)


def reed_solomon(coeffs_local, log_n, gen, tp, ops):
    """reed_solomon (fri/mod.rs:19-28) of 2^log_n coefficients in the cyclic
    layout -> the 2^(log_n+1) codeword in the block-(2^(log_n+1) / P^2) layout."""
    P = tp.world
    if P == 1:
        return ops.reed_solomon(coeffs_local, gen)
    z = ops.reed_solomon(coeffs_local, pow(gen, P, M))
    recv = tp.all_to_all(z)
    return ops.cross(recv, log_n + LOG_BLOWUP, _log2(P), tp.rank, gen, False)


# ---------------------------------------------------------------------------
# sharded FRI prove
# ---------------------------------------------------------------------------

def _hash_node(a, b):
    return hashlib.sha256(a + b).digest()


class _Layer:
    """One FRI layer: local values + local tree; ``log_p == 0`` = replicated."""

    def __init__(self, values, tree, log_n, log_p, log_s, rank):
        self.values, self.tree = values, tree
        self.log_n, self.log_p, self.log_s, self.rank = log_n, log_p, log_s, rank
        # tree levels held locally (siblings below this come from HBM)
        self.sub_levels = log_s if log_p else log_n - 1
        self.top_dev = None  # device tree over the all-gathered level-log_s nodes
        self.root_dev = None  # 32-byte device view of the root
        self.top = []  # host copy of top_dev's levels (query phase)

    @property
    def local_leaves(self):
        return 1 << (self.log_n - 1 - self.log_p)


def _commit_top(layer, tp, ops):
    """Root of the layer's tree, on the device: a replicated layer's own root;
    a sharded layer all-gathers its level-log_s subtree roots (T/2 per rank)
    and hashes the top levels (mlh_merkle_top).  No host round trip."""
    if layer.log_p == 0:
        layer.root_dev = ops.tree_root(layer.tree)
        return
    half_t = layer.local_leaves >> layer.sub_levels
    nodes = ops.tree_level_dev(layer.tree, layer.local_leaves, layer.sub_levels)
    gathered = tp.all_gather(nodes)
    layer.top_dev = ops.merkle_top(gathered, tp.world, half_t)
    layer.root_dev = ops.tree_root(layer.top_dev)


def _host_top(layer):
    """Host levels of a sharded layer's top tree (for the query phase)."""
    if layer.top_dev is None:
        return
    raw = ops_bytes(layer.top_dev)
    n = len(raw) // 32
    leaves = (n + 1) // 2
    levels, off = [], 0
    while leaves >= 1:
        levels.append([raw[32 * (off + i):32 * (off + i + 1)] for i in range(leaves)])
        off += leaves
        leaves //= 2
    layer.top = levels


def ops_bytes(t):
    return t.cpu().contiguous().numpy().tobytes()


def _open(layer, idx, tp, ops):
    """Query records of one layer for the global leaf indices idx: this rank's
    part (owned sharded leaves; all of them when replicated), others zero."""
    leaves = 1 << (layer.log_n - 1)
    rec_len = 32 * (1 + layer.log_n - 1)
    out = [None] * len(idx)
    mine, loc = [], []
    for q, i in enumerate(idx):
        i %= leaves
        if layer.log_p:
            r, l = block_owner(i, layer.log_s, layer.log_p)
            if r != layer.rank:
                continue
        else:
            l = i
        mine.append(q)
        loc.append(l)
    recs = ops.open_pairs(layer.values, layer.tree, layer.sub_levels, loc) if loc else []
    for q, rec in zip(mine, recs):
        i = idx[q] % leaves
        sibs = []
        for lv in range(len(layer.top) - 1):
            node = (i >> (layer.sub_levels + lv)) ^ 1
            sibs.append(layer.top[lv][node])
        out[q] = rec + b"".join(sibs)
        assert len(out[q]) == rec_len
    return [o if o is not None else bytes(rec_len) for o in out]


def commit_rs_code(code_local, log_code, tp, ops):
    """commit_rs_code + Merkle::commit (fri/mod.rs:45-55, merkle_tree/mod.rs:
    65-85) of a 2^log_code codeword in the block-(2^log_code / P^2) layout:
    local leaves and subtrees, one all-gather of the subtree roots, the top
    levels on the device.  Returns the root (32 bytes, host)."""
    P = tp.world
    log_p = _log2(P)
    if log_p:
        lay = _Layer(code_local, None, log_code, log_p, cross_log_s(log_code, log_p), tp.rank)
    else:
        lay = _Layer(code_local, None, log_code, 0, 0, tp.rank)
    lay.tree = ops.commit_pairs(lay.values)
    _commit_top(lay, tp, ops)
    return ops.concat_bytes([lay.root_dev])


def fri_prove(code_local, log_code, transcript, tp, ops, gather_log=16):
    """FriProof::prove (fri/mod.rs:261-285) of a 2^log_code codeword held in
    the block-(2^log_code / P^2) layout (``reed_solomon``'s output).

    The commit loop is device resident on every rank: the transcript state is
    replicated in HBM (mlh_transcript_to_device), each layer's root is built
    on the device (local subtrees, an all-gather of the subtree roots, the
    top levels) and absorbed by a device kernel that writes the next
    challenge to HBM, where the next fold reads it.  The host waits once,
    replays the absorbs into ``transcript`` and runs the query phase.
    Every rank returns the same proof; it equals the single-GPU proof of the
    natural-order codeword byte for byte."""
    from multilinear_amd.fri import FriProof

    P, rank = tp.world, tp.rank
    log_p = _log2(P)
    if log_code < 2:
        raise ValueError("log_code must be >= 2")
    if log_p and log_code - 2 * log_p < 0:
        raise ValueError("codeword too small for the world size")
    gather_log = max(gather_log, 2 * log_p + 2)
    n0 = log_code
    steps = log_code - LOG_BLOWUP
    state = ops.dev_transcript(transcript)
    rbuf = ops.empty(steps + 1)
    lastbuf, flagbuf = ops.empty(1), ops.empty(1)
    if log_p and log_code > gather_log:
        lay = _Layer(code_local, None, log_code, log_p, cross_log_s(log_code, log_p), rank)
    else:
        if log_p:
            code_local = _to_natural(code_local, log_code, log_p, cross_log_s(log_code, log_p),
                                     tp, ops)
        lay = _Layer(code_local, None, log_code, 0, 0, rank)
    lay.tree = ops.commit_pairs(lay.values)
    _commit_top(lay, tp, ops)
    layers = [lay]
    ops.absorb(state, lay.root_dev, rbuf[0])
    done = False
    for k in range(steps):
        cur = layers[-1]
        if (1 << cur.log_n) <= (1 << LOG_BLOWUP):
            break
        r = rbuf[k]
        log_next = cur.log_n - 1
        if (1 << log_next) == (1 << LOG_BLOWUP):  # fri/mod.rs:116-126
            nx = ops.fold_dr(cur.values, k, n0, r, 40, 0, 0)
            ops.fri_last(nx, state, flagbuf, lastbuf)
            done = True
            break
        if cur.log_p == 0:
            nv, tree = ops.fold_commit_dr(cur.values, k, n0, r, 40, 0, 0)
            lay = _Layer(nv, tree, log_next, 0, 0, rank)
        elif log_next - cur.log_p - cur.log_s >= 1:  # >= 2 local blocks: pairs local
            nv, tree = ops.fold_commit_dr(cur.values, k, n0, r, cur.log_s, cur.log_p, rank)
            lay = _Layer(nv, tree, log_next, cur.log_p, cur.log_s, rank)
        else:  # folded layer is in natural block order: re-deal or gather
            nv = ops.fold_dr(cur.values, k, n0, r, cur.log_s, cur.log_p, rank)
            if log_next > gather_log:
                nv = tp.all_to_all(nv)
                lay = _Layer(nv, None, log_next, log_p, cross_log_s(log_next, log_p), rank)
            else:
                nv = tp.all_gather(nv)
                lay = _Layer(nv, None, log_next, 0, 0, rank)
            lay.tree = ops.commit_pairs(lay.values)
        _commit_top(lay, tp, ops)
        layers.append(lay)
        ops.absorb(state, lay.root_dev, rbuf[k + 1])
    if not done:
        raise _lib.MlhError(_lib.MLH_ERR_INVALID, "fold produced no last element")

    # one wait: roots, last element, RS flag; the host transcript replays them
    roots = ops.concat_bytes([l.root_dev for l in layers])
    last = ops_bytes(lastbuf)[:16]
    if int.from_bytes(ops_bytes(flagbuf)[:4], "little"):
        raise _lib.MlhError(_lib.MLH_ERR_NOT_RS_CODE, "not an RS code")
    for t in range(len(layers)):
        transcript.absorb(roots[32 * t:32 * t + 32])
    transcript.absorb(last)
    for l in layers:
        _host_top(l)

    idx = []
    for _ in range(NUM_QUERIES):  # fri/mod.rs:266-277
        i = int.from_bytes(transcript.random()[:8], "little") % (1 << (log_code - 1))
        idx.append(i)
        transcript.absorb(i.to_bytes(8, "little"))
    per_layer = [_open(l, idx, tp, ops) for l in layers]
    mine = b"".join(per_layer[t][q] for q in range(NUM_QUERIES) for t in range(len(layers)))
    if P > 1:
        parts = tp.gather_bytes(mine)
        acc = np.zeros(len(mine), dtype=np.uint8)
        for p in parts:
            acc |= np.frombuffer(p, dtype=np.uint8)
        qraw = acc.tobytes()
    else:
        qraw = mine

    proof = FriProof(log_code)
    assert len(qraw) == proof.qbytes * NUM_QUERIES
    proof.c.log_code = log_code
    proof.c.num_trees = len(layers)
    proof.c.num_queries = NUM_QUERIES
    ctypes.memmove(proof._commit, roots, 32 * len(layers))
    ctypes.memmove(proof._q, qraw, len(qraw))
    for q, i in enumerate(idx):
        proof._idx[q] = i
    proof.c.last_elem[:] = list(last)
    proof.c.last_random[:] = list(transcript.random())
    return proof


def _to_natural(values, log_n, log_p, log_s, tp, ops):
    """Gather a block-layout vector to natural order on every rank."""
    g = tp.all_gather(values)  # [rank][T][S]
    S = 1 << log_s
    P = 1 << log_p
    return g.reshape(P, -1, S, 4).transpose(0, 1).reshape(-1, 4).contiguous()


# ---------------------------------------------------------------------------
# sharded sumcheck ("shard by low index bits")
# ---------------------------------------------------------------------------

def eq_table(points, tp, ops):
    """delta of build_tables_for_pcs (sumcheck.rs:128-145) in the cyclic
    layout: rank r holds delta[l P + r] = eq(points[:n-p], l) * c_r, where
    c_r = prod_{b<p} (bit_b(r) ? points[n-1-b] : 1 - points[n-1-b]) -- the low
    index bits pair with the LAST points (big-endian order)."""
    P, rank = tp.world, tp.rank
    p = _log2(P)
    n = len(points)
    if n < p:
        raise ValueError("fewer variables than log2(world)")
    c = 1
    for b in range(p):
        pt = points[n - 1 - b]
        c = c * (pt if (rank >> b) & 1 else (1 - pt) % M) % M
    local = ops.eq_table(points[:n - p]) if n > p else None
    if local is None:
        local = ops.eq_table([])
    return ops.scale(local, c) if c != 1 else local


def sumcheck_prove(m, d, n, total_sum, transcript, tp, ops):
    """SumcheckTables::compute_sumcheck_polynomials (sumcheck.rs:77-102) for
    the PCS composition x[0], tables of 2^n entries in the cyclic layout
    (``m``, ``d`` local, folded in place).  The MSB-first fold pairs (i, i+h)
    share their low bits, so they stay on one rank while the local table has
    >= 2 entries; each round all-gathers the ranks' (s1, s2) sums straight
    from HBM and a device kernel adds them, interpolates, absorbs (c1, c2)
    into the replicated device transcript and writes r to HBM for the folds;
    the last p rounds run replicated on the gathered P-entry tables.  The host
    waits once and replays the absorbs into ``transcript``.
    Returns ([(c1, c2)], [r]) -- identical to the single-GPU prover."""
    P = tp.world
    p = _log2(P)
    sharded = P > 1
    log_local = n - p
    state = ops.dev_transcript(transcript)
    prev = ops.const(total_sum % M)
    polys = ops.empty(2 * n)
    rs = ops.empty(n)
    sums = ops.empty(2)
    if sharded and log_local == 0:
        m, d, sharded, log_local = tp.all_gather(m), tp.all_gather(d), False, n
    ops.sc_sums_dev(m, d, log_local, sums)
    for k in range(n):
        pairs = tp.all_gather(sums) if sharded else sums
        ops.sc_round(pairs, P if sharded else 1, prev, state, polys[2 * k:2 * k + 2], rs[k])
        if k + 1 == n:
            ops.sc_fold_dr(m, d, log_local, rs[k])
            break
        if log_local >= 2:
            ops.sc_fold_sums_dr(m, d, log_local, rs[k], sums)
            log_local -= 1
        else:  # sharded, local 2 -> 1: gather the P-entry tables, go replicated
            ops.sc_fold_dr(m, d, log_local, rs[k])
            m, d = tp.all_gather(m[:1]), tp.all_gather(d[:1])
            sharded, log_local = False, p
            ops.sc_sums_dev(m, d, log_local, sums)
    raw_p, raw_r = ops_bytes(polys), ops_bytes(rs)
    out_p, out_r = [], []
    for k in range(n):
        c1, c2 = raw_p[32 * k:32 * k + 16], raw_p[32 * k + 16:32 * k + 32]
        transcript.absorb(c1)
        transcript.absorb(c2)
        out_p.append((int.from_bytes(c1, "little"), int.from_bytes(c2, "little")))
        out_r.append(int.from_bytes(raw_r[16 * k:16 * k + 16], "little"))
    return out_p, out_r


# ---------------------------------------------------------------------------
# fused sharded NTT (mlh_sharded_ntt_fused_batch): the rank digit in the last pass
# ---------------------------------------------------------------------------

def plan_radices(log_n):
    """ntt.hip ntt_plan_radices: ceil(log_n / 9) digits, larger first."""
    P = (log_n + 8) // 9
    out, rem = [], log_n
    for p in range(P):
        r = (rem + (P - p) - 1) // (P - p)
        out.append(r)
        rem -= r
    return out


def fused_plan(log_n, log_p):
    """(c, pre digits, output log_s) of the fused plan (capi.hip FusedNtt::prepare):
    the last global digit is c + p = 9 bits, c of them local."""
    c = 9 - log_p
    pre = plan_radices(log_n - log_p - c)
    return c, pre, pre[0] - log_p


def ntt_fused(x_local, log_n, gen, tp):
    """The fused sharded forward NTT on Python ints (the executable spec of
    mlh_sharded_ntt_fused_batch, at oracle sizes).  N = Mhi * Q with
    Q = 2^(c + p) (the last pass) and Mhi = 2^(log_n - c - p):
      X[kA + Mhi kB] = sum_{nB < Q} wQ^(nB kB) w^(nB kA) sum_{nA} x[nA Q + nB] wMhi^(nA kA).
    Rank g holds x[g + P m] (cyclic), i.e. nB = g + P mc, m = nA 2^c + mc, so the
    inner DFTs and the twiddle are local.  ONE all-to-all: (mc, kA) goes to the
    rank named by bits [a - p, a) of kA (a = the first local digit: the top
    bits of the first output digit, as the local passes store it).  The last
    stage: a Q-point DFT over nB for each received kA; X[K] lands at local index
    K with bits [a - p, a) removed (block-cyclic, block 2^(a - p)).
    x_local: list of ints; returns (list of ints, log_s)."""
    from oracle import ntt as ON

    P, g = tp.world, tp.rank
    p = _log2(P)
    N = 1 << log_n
    c, pre, log_s = fused_plan(log_n, p)
    a = pre[0]
    Q = 1 << (c + p)
    Mhi = N // Q
    C2 = 1 << c
    wM = pow(gen, Q, M)
    # local stage: for every mc, the Mhi-point DFT over nA, times w^(nB kA)
    Z = {}
    for mc in range(C2):
        nB = g + P * mc
        Y = ON.ntt([x_local[nA * C2 + mc] for nA in range(Mhi)], wM) if Mhi > 1 else [x_local[mc]]
        for kA in range(Mhi):
            Z[(mc, kA)] = Y[kA] * pow(gen, nB * kA, M) % M
    # all-to-all: destination h = bits [a - p, a) of kA; a fixed (mc, kA) order per chunk
    dest = lambda kA: (kA >> (a - p)) & (P - 1)  # noqa: E731
    chunks = [[] for _ in range(P)]
    for kA in range(Mhi):
        for mc in range(C2):
            chunks[dest(kA)].append(Z[(mc, kA)])
    per = len(chunks[0])
    assert all(len(ch) == per for ch in chunks)
    import torch

    send = torch.tensor([[v & 0xFFFFFFFF, (v >> 32) & 0xFFFFFFFF, (v >> 64) & 0xFFFFFFFF, v >> 96]
                         for ch in chunks for v in ch], dtype=torch.int64).to(torch.int32)
    recv = tp.all_to_all(send).to(torch.int64) & 0xFFFFFFFF
    vals = [int(r[0]) | int(r[1]) << 32 | int(r[2]) << 64 | int(r[3]) << 96 for r in recv.tolist()]
    mine = [kA for kA in range(Mhi) if dest(kA) == g]  # this rank's kA, in the senders' order
    wQ = pow(gen, Mhi, M)
    out = [0] * (N // P)
    for i, kA in enumerate(mine):
        col = [0] * Q
        for src in range(P):
            for mc in range(C2):
                col[src + P * mc] = vals[src * per + i * C2 + mc]  # nB = src + P mc
        XB = ON.ntt(col, wQ)
        for kB in range(Q):
            K = kA + Mhi * kB
            lo = a - p
            out[((K >> a) << lo) | (K & ((1 << lo) - 1))] = XB[kB]
    return out, log_s
