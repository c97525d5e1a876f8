"""bench.py's extras watchdog (CPU): the headline line survives a stalled
secondary timing, and is printed exactly once."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_watchdog_claim_once():
    import bench

    w = bench._ExtrasWatchdog({"value": 1.0}, 0, 30.0)
    assert w.claim() is True
    assert w.claim() is False


def test_watchdog_fires_with_headline_snapshot():
    code = ("import bench, time\n"
            "r = {'metric': 'm', 'value': 2.5}\n"
            "bench._ExtrasWatchdog(r, 0, 0.2)\n"
            "r['late_extra'] = 1\n"  # added after arming: not in the snapshot
            "time.sleep(20)\n"
            "print('not reached')\n")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 0
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and "not reached" not in p.stdout
    d = json.loads(lines[0])
    assert d["value"] == 2.5 and "extras_error" in d and "late_extra" not in d


def test_watchdog_silent_on_other_ranks():
    code = "import bench, time\nbench._ExtrasWatchdog({'value': 1}, 3, 0.2)\ntime.sleep(20)\n"
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 0 and p.stdout.strip() == ""


def test_sharded_phases_split_and_bandwidth():
    """The N > 1 line's phase split (bench.sharded_phases): local NTT = its
    passes summed, all-to-all GB/s = (P-1)/P of the 16 x 2^log_n-byte shard
    per all-to-all duration."""
    import bench

    k = {"ntt_pass<8,0,0>": {"avg_ms": 0.2, "launches": 3},
         "ntt_pass<8,1,0>": {"avg_ms": 0.15, "launches": 3},
         "ntt_pass<8,2,0>": {"avg_ms": 0.1, "launches": 3},
         "ntt_all_to_all": {"avg_ms": 0.5, "launches": 3},
         "shard_dft<3,0>": {"avg_ms": 0.05, "launches": 3}}
    ph = bench.sharded_phases(k, 24, 3, 3)
    assert abs(ph["local_ntt_ms"] - 0.45) < 1e-12
    assert ph["shard_dft_ms"] == 0.05 and ph["all_to_all_ms"] == 0.5
    sent = 16.0 * (1 << 24) * 7 / 8
    assert ph["all_to_all_bytes_sent_per_rank"] == sent
    assert abs(ph["all_to_all_gbs"] - sent / 0.5e-3 / 1e9) < 1e-6
    assert bench.sharded_phases({}, 24, 1, 3)["all_to_all_gbs"] is None


def test_sharded_ntt_spot_check_formula_vs_oracle():
    """The identity bench.sharded_ntt_check relies on, in exact integers: for
    x cyclic over P ranks (rank g holds x[g + P m]), X[j] = NTT(x)[j] =
    sum_g gen^(j g) poly_g(gen^(j P)); and ntt_block_owner names the rank /
    local index holding X[j] in the sharded NTT's block output layout (the
    layout of tests/dist_spec.py, checked against the oracle there)."""
    import random

    from multilinear_amd.sharded import M, ntt_block_owner
    from oracle import field as F
    from oracle import ntt as ON

    for log_n, log_p in ((6, 1), (8, 2), (9, 3)):
        n, P = 1 << log_n, 1 << log_p
        r = random.Random(log_n)
        x = [r.randrange(M) for _ in range(n)]
        g = F.pow_2_generator(log_n)
        X = ON.ntt(x, g)
        shards = [x[q::P] for q in range(P)]

        def poly(c, t):
            acc = 0
            for v in reversed(c):
                acc = (acc * t + v) % M
            return acc

        for j in [0, n - 1] + [r.randrange(n) for _ in range(6)]:
            got = sum(pow(g, j * q, M) * poly(shards[q], pow(g, j * P, M)) for q in range(P)) % M
            assert got == X[j]
        # block layout: local l of rank q <-> global ((l >> s) << (s + p)) | (q << s) | (l mod 2^s)
        s_ = log_n - 2 * log_p
        for j in range(n):
            q, l = ntt_block_owner(j, log_n, log_p)
            assert ((l >> s_) << (s_ + log_p)) | (q << s_) | (l & ((1 << s_) - 1)) == j
            assert 0 <= q < P and 0 <= l < n // P


def test_headline_watchdog_fires_with_phase_and_exits_nonzero():
    code = ("import bench, time\n"
            "w = bench._HeadlineWatchdog(0, 8, 0.3)\n"
            "w.info = {'ranks': 8, 'rank': 0, 'device': 0, 'transport': 'rccl'}\n"
            "w.phase('comm_create'); w.phase('preflight')\n"
            "time.sleep(20)\n"
            "print('not reached')\n")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 3
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and "not reached" not in p.stdout
    d = json.loads(lines[0])
    assert d["value"] is None and d["phase"] == "preflight" and d["rccl_ranks"] == 8
    assert "preflight" in d["headline_error"] and d["n_gpus"] == 8
    assert list(d["phases_started_s"]) == ["comm_create", "preflight"]


def test_headline_watchdog_disarm_and_fail():
    code = ("import bench, time\n"
            "w = bench._HeadlineWatchdog(0, 2, 0.3)\n"
            "w.disarm(); time.sleep(1.0)\n"
            "w2 = bench._HeadlineWatchdog(0, 2, 30)\n"
            "w2.phase('preflight'); w2.fail('pre-flight mismatch')\n")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 4
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["headline_error"] == "pre-flight mismatch"


_STALL_SCRIPT = r'''
import os, sys, time
sys.path.insert(0, os.environ["MLH_ROOT"])
import torch.distributed as dist
import torch
import bench
dist.init_process_group("gloo")
rank = dist.get_rank()
w = bench._HeadlineWatchdog(rank, 2, 5.0)
w.info = {"ranks": 2, "rank": rank, "device": 0, "transport": "host-staged gloo"}
w.phase("preflight")
if rank == 1:
    time.sleep(120)          # a dead peer: never joins the collective
t = torch.zeros(8)
dist.all_reduce(t)           # rank 0 waits here
print("not reached", flush=True)
'''


def test_headline_watchdog_ends_a_stalled_gloo_collective_world2(tmp_path):
    """world 2 over gloo on the CPU: rank 1 never joins, rank 0 blocks inside a
    real collective; within the budget rank 0 prints the diagnostic line (the
    phase reached) and both ranks exit non-zero."""
    import socket

    script = tmp_path / "stall.py"
    script.write_text(_STALL_SCRIPT)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MLH_ROOT=ROOT)
    t0 = __import__("time").time()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
                        "2", "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)],
                       cwd=ROOT, capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode != 0
    assert __import__("time").time() - t0 < 90
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout + p.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["phase"] == "preflight" and "did not finish" in d["headline_error"]
    assert "not reached" not in p.stdout
