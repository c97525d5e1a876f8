"""bench.py's N > 1 script rehearsed with two ranks sharing the box's one GPU
(gloo, host-staged transport; never a result): the line certifies itself
(pre-flight pattern check, in-run output check, a transport label that does
not claim xGMI), and a rank whose all-to-all never returns -- a dead RCCL peer
on the 8-GPU node -- ends the run within the headline budget with a
diagnostic line naming the phase, instead of a silent kill."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra_env, args, timeout, nproc=2):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MLH_BENCH_BACKEND="gloo", **extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc)] + args
    t0 = time.time()
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p, lines, time.time() - t0


def test_rehearsal_n2_line_certifies_itself():
    p, lines, _ = _run({}, ["--log-n", "20", "--steps", "3", "--warmup", "1", "--no-extras",
                            "--spinup-s", "0"], 110)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout + p.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["preflight"]["ok"] and d["preflight"]["mismatches_max"] == 0
    assert d["sharded_ntt_verified"] is True
    assert "xGMI" not in d["config"]["parallelism"] and "rehearsal" in d["config"]["parallelism"]
    assert d["rccl_ranks"] is None


def test_rehearsal_n2_stalled_all_to_all_reports_phase():
    p, lines, dt = _run({"MLH_BENCH_TEST_STALL_A2A": "1"},
                        ["--log-n", "20", "--steps", "3", "--warmup", "1", "--no-extras",
                         "--headline-budget-s", "20"], 110)
    assert p.returncode != 0
    assert len(lines) == 1, p.stdout + p.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["value"] is None and d["phase"] == "preflight"
    assert "did not finish within 20 s" in d["headline_error"]
    assert d["comm"]["ranks"] == 2 and d["rccl_ranks"] is None
    assert dt < 100


_CHECKS = ("config5_matches_single_gpu", "config3_sharded_matches_single_gpu",
           "config4_sharded_matches_single_gpu")


@pytest.mark.timeout(320)
@pytest.mark.parametrize("nproc,corrupt", [(2, None), (4, None), (2, "1")])
def test_rehearsal_extras_certify_against_single_gpu(nproc, corrupt):
    """Every N > 1 extra carries an in-run parity bit against a single-GPU
    recompute on rank 0 (config 5: the sharded proof's wire bytes vs
    reed_solomon + FriProof::prove of the gathered coefficients; config 3
    sharded: the root vs commit_rs_code of the gathered code; config 4 sharded:
    every round polynomial and challenge vs the single-GPU prove; strong NTT:
    the headline's spot check).  With one rank's shard altered after the timed
    loops (MLH_BENCH_TEST_CORRUPT_SHARD) every bit is false and the line is
    still printed."""
    env = {} if corrupt is None else {"MLH_BENCH_TEST_CORRUPT_SHARD": corrupt}
    p, lines, _ = _run(env, ["--log-n", "16", "--steps", "3", "--warmup", "1", "--spinup-s", "0",
                             "--no-cpu", "--fri-log", "20", "--strong-log", "20", "--extra-reps", "1"],
                       300, nproc)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout + p.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == nproc and d["sharded_ntt_verified"] is True
    want = corrupt is None
    for k in _CHECKS:
        assert d.get(k) is want, (k, d.get(k), {x: d.get(x) for x in d if x.endswith("_error")})
    assert d["strong_ntt"]["verified"] is want
    assert d["config5_verified"] is True  # the host verifier accepts either proof
