"""world_size 2 and 4 gloo tests of the sharded path (tests/dist_spec.py)
on CPU: the real orchestration (layouts, all-to-all, all-gather, subtree-root
combination, query ownership) with rank-local steps from the oracle
(tests/dist_cpu_ops.py).  Outputs must equal the single-process oracle's:
the sharded RS codeword / NTT, and the FRI proof byte for byte."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, log_c, gather_log, q):
    import torch
    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests import dist_spec as D
        from multilinear_amd.transcript import Transcript
        from oracle import coracle as C
        from oracle import field as F
        from tests.dist_cpu_ops import CpuOps

        tp, ops = D.Transport(), CpuOps()
        log_n = log_c - 1
        rng = np.random.default_rng(7)
        coeffs = rng.integers(0, 2**32, size=(1 << log_n, 4), dtype=np.uint64).astype(np.uint32)
        coeffs[:, 3] = np.minimum(coeffs[:, 3], 0xFFFFFFFE)
        gen = F.pow_2_generator(log_c)
        code = C.reed_solomon(coeffs, log_n, gen)
        log_s = D.cross_log_s(log_c, world.bit_length() - 1)

        local = torch.from_numpy(D.shard_cyclic(coeffs, world, rank).view(np.int32))
        enc = D.reed_solomon(local, log_n, gen, tp, ops)
        ok_rs = np.array_equal(enc.numpy().view(np.uint32), D.shard_blocks(code, world, rank, log_s))

        x = torch.from_numpy(D.shard_cyclic(code, world, rank).view(np.int32))
        X = D.ntt(x, log_c, gen, tp, ops)
        ref = C.ntt(code, log_c, gen)
        ok_ntt = np.array_equal(X.numpy().view(np.uint32), D.shard_blocks(ref, world, rank, log_s))
        back = D.intt(X, log_c, gen, tp, ops)
        ok_intt = np.array_equal(back.numpy(), x.numpy())

        proof = D.fri_prove(enc, log_c, Transcript(), tp, ops, gather_log=gather_log)
        blob = (bytes(proof._commit), bytes(proof._q), list(proof._idx), bytes(proof.c.last_elem),
                bytes(proof.c.last_random), proof.verify())
        q.put((rank, ok_rs, ok_ntt, ok_intt, blob))
    except Exception as e:  # surface the failure in the parent
        import traceback

        q.put((rank, "error", traceback.format_exc(), None, None))
    finally:
        tdist.destroy_process_group()


def _run(world, log_c, gather_log):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, log_c, gather_log, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda t: t[0])
    for r in res:
        assert r[1] != "error", r[2]
    return res


def _single_proof(log_c):
    from multilinear_amd.fri import FriProof
    from oracle import coracle as C
    from oracle import field as F
    from oracle import fri as OF
    from oracle.transcript import Transcript as OT

    log_n = log_c - 1
    rng = np.random.default_rng(7)
    coeffs = rng.integers(0, 2**32, size=(1 << log_n, 4), dtype=np.uint64).astype(np.uint32)
    coeffs[:, 3] = np.minimum(coeffs[:, 3], 0xFFFFFFFE)
    code = F.from_limbs(C.reed_solomon(coeffs, log_n, F.pow_2_generator(log_c)))
    gp = F.pow_2_generator_powers(log_c)
    return OF.FriProof.prove(code, gp, OT())


@pytest.mark.parametrize("world,log_c,gather_log", [(2, 10, 4), (4, 10, 4), (2, 9, 16), (4, 12, 6), (8, 13, 8)])
def test_sharded_rs_ntt_fri_match_single(world, log_c, gather_log):
    res = _run(world, log_c, gather_log)
    for r in res:
        assert r[1], "sharded reed_solomon != oracle (rank %d)" % r[0]
        assert r[2], "sharded ntt != oracle (rank %d)" % r[0]
        assert r[3], "sharded intt round trip failed (rank %d)" % r[0]
    blobs = [r[4] for r in res]
    assert all(b == blobs[0] for b in blobs), "ranks disagree on the proof"
    commit, qraw, idx, last, last_random, verified = blobs[0]
    assert verified
    ref = _single_proof(log_c)
    assert commit == b"".join(ref.commitments)
    assert int.from_bytes(last, "little") == ref.last_elem
    assert last_random == ref.last_random
    raw = b""
    for q in ref.queries:
        for value, path in q:
            raw += value + b"".join(s for s, _ in path)
    assert qraw == raw


def _sc_worker(rank, world, port, n, q):
    import torch
    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests import dist_spec as D
        from multilinear_amd.transcript import Transcript
        from tests.dist_cpu_ops import CpuOps

        tp, ops = D.Transport(), CpuOps()
        rng = np.random.default_rng(3)
        ev = rng.integers(0, 2**32, size=(1 << n, 4), dtype=np.uint64).astype(np.uint32)
        ev[:, 3] = np.minimum(ev[:, 3], 0xFFFFFFFE)
        pts = [int(x) for x in rng.integers(0, 2**62, size=n)]
        m = torch.from_numpy(D.shard_cyclic(ev, world, rank).view(np.int32).copy())
        d = D.eq_table(pts, tp, ops)
        tr = Transcript()
        tr.absorb(b"sumcheck")
        polys, rs = D.sumcheck_prove(m, d, n, 12345, tr, tp, ops)
        q.put((rank, polys, rs, tr.random()))
    except Exception:
        import traceback

        q.put((rank, "error", traceback.format_exc(), None))
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 6), (4, 7), (4, 2), (2, 1), (8, 5)])
def test_sharded_sumcheck_matches_oracle(world, n):
    """dist.eq_table + dist.sumcheck_prove vs the oracle's
    compute_sumcheck_polynomial loop (sumcheck.rs:77-102, 174-202)."""
    from oracle import field as F
    from oracle import sumcheck as OS
    from oracle.transcript import Transcript as OT

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sc_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r[2]
    rng = np.random.default_rng(3)
    ev = rng.integers(0, 2**32, size=(1 << n, 4), dtype=np.uint64).astype(np.uint32)
    ev[:, 3] = np.minimum(ev[:, 3], 0xFFFFFFFE)
    pts = [int(x) for x in rng.integers(0, 2**62, size=n)]
    tab = OS.SumcheckTables(F.from_limbs(ev), OS.eq_table(pts))
    tr = OT()
    tr.absorb(b"sumcheck")
    prev, polys, rs = 12345, [], []
    for _ in range(n):
        nz, r, prev = tab.compute_sumcheck_polynomial(prev, tr)
        polys.append(tuple(nz))
        rs.append(r)
    for r in res:
        assert [tuple(p) for p in r[1]] == polys, "rank %d polys" % r[0]
        assert r[2] == rs
        assert r[3] == tr.random()


def _commit_worker(rank, world, port, log_c, q):
    import torch
    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests import dist_spec as D
        from oracle import coracle as C
        from oracle import field as F
        from tests.dist_cpu_ops import CpuOps

        tp, ops = D.Transport(), CpuOps()
        rng = np.random.default_rng(9)
        code = rng.integers(0, 2**32, size=(1 << log_c, 4), dtype=np.uint64).astype(np.uint32)
        code[:, 3] = np.minimum(code[:, 3], 0xFFFFFFFE)
        log_s = D.cross_log_s(log_c, world.bit_length() - 1)
        local = torch.from_numpy(D.shard_blocks(code, world, rank, log_s).view(np.int32))
        root = D.commit_rs_code(local, log_c, tp, ops)
        want = bytes(C.merkle_commit_pairs(code, log_c)[-1])
        q.put((rank, root == want, None))
    except Exception:
        import traceback

        q.put((rank, "error", traceback.format_exc()))
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("world,log_c", [(2, 8), (4, 10), (8, 9)])
def test_sharded_merkle_commit_root(world, log_c):
    """dist.commit_rs_code (local subtrees + all-gathered roots + top) == the
    single Merkle root of the natural-order code (merkle_tree/mod.rs:65-85)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_commit_worker, args=(r, world, port, log_c, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] is True, r


def _fused_worker(rank, world, port, log_n, q):
    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import random

        from oracle import field as F
        from oracle import ntt as ON
        from tests import dist_spec as D

        rr = random.Random(log_n)
        x = [rr.randrange(F.M) for _ in range(1 << log_n)]
        gen = F.pow_2_generator(log_n)
        out, log_s = D.ntt_fused(x[rank::world], log_n, gen, D.Transport())
        q.put((rank, out, log_s, ON.ntt(x, gen) if rank == 0 else None))
    except Exception:
        import traceback

        q.put((rank, "error", traceback.format_exc(), None))
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("world,log_n", [(2, 14), (4, 14), (8, 15)])
def test_fused_sharded_ntt_spec_matches_oracle(world, log_n):
    """The fused sharded NTT's schedule (tests/dist_spec.py ntt_fused: local
    DFTs + twiddle, ONE gloo all-to-all by the first output digit's top bits,
    the last Q-point stage on the received columns) at world 2/4/8: the
    block-cyclic outputs (block 2^(a - p), the layout mlh_sharded_ntt_fused_batch
    reports) put back in order equal the oracle NTT."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fused_worker, args=(r, world, port, log_n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r[2]
    log_s = res[0][2]
    from tests import dist_spec as D

    assert log_s == D.fused_plan(log_n, world.bit_length() - 1)[2]
    S = 1 << log_s
    got = []
    n_local = len(res[0][1])
    for blk in range(n_local // S):
        for r in range(world):
            got.extend(res[r][1][blk * S:(blk + 1) * S])
    assert got == res[0][3]
