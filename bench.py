"""bench.py -- headline benchmark (BASELINE.json metric) on 1..8 MI355X.

Metric: "NTT 2^24 field-elems/sec + FRI commit ms; % HBM roofline".
  * N = 1: step = one forward 2^24-point NTT (config 2, src/ntt/mod.rs:69-110)
            over a device-resident synthetic vector (seeded uniform elements);
  * N > 1 (default --mode sharded): one forward NTT of N * 2^24 points per
            step, 2^24 per GPU: local NTT, one RCCL all-to-all over xGMI,
            cross-shard DFT kernel; the K steps are one
            mlh_sharded_ntt_batch call of the C ABI (csrc/sharded.hip), whose
            two streams overlap the exchange of step i with the local NTT of
            step i+1 (every exchange and cross kernel completes inside the
            timed region); weak scaling (2^24 per GPU);
  * N > 1, --mode replicas: every rank transforms its own 2^24-point
            polynomial per step (no data-path collective; reported as the
            extra "replicas_ntt" in the default mode);
  * strong scaling at every N (N = 1 included): "strong_ntt" = one 2^28-point
            NTT (single GPU at N = 1, sharded over the N ranks otherwise) and
            config 5 (RS + FRI prove of a 2^28 codeword), fixed total size;
  * value = 2^24 * N * steps / max-over-ranks(time of the K steps);
  * extras in the same JSON line: inverse NTT, FRI commit (config 3: 2^24
    coeffs -> RS LDE 2^25 -> Merkle root), full FRI prove, the 24-round
    sumcheck (config 4) [N = 1], and config 5: RS encode + FRI prove of a
    2^28-element codeword, single GPU at N = 1, sharded over the N ranks at
    N > 1 (strong scaling), each timed after the headline loop;
  * roofline: the dominant kernel (an ntt_pass) timed live with HIP events on
    its launch stream over the headline loop; algorithmic bytes per launch =
    that pass's share of the transform's 32 B x 2^24 (one read
    and one write of every element for the WHOLE NTT, never the multi-pass
    traffic), i.e. 32 B x 2^24 / passes; `bound` is the larger of that HBM
    fraction and the pass's VALU issue fraction (SQ_INSTS_VALU of the newest
    committed VALU pass x 64 lanes / live time, against one wave64 VALU
    instruction per 4 cycles per SIMD at 2.4 GHz);
  * cpu_baseline: the oracle's C restatement of the reference NTT
    (oracle/liboracle.so, 1 thread) on one 2^24 NTT, rank 0 at N = 1 only.

Run:  python bench.py [--gpus N --steps K --warmup W]
      torchrun --nproc-per-node N bench.py --gpus N ...  (one rank per GPU)
"""
import argparse
import ctypes
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# RCCL in production; MLH_BENCH_BACKEND=gloo rehearses the multi-rank logic with
# host-staged exchanges (e.g. 2 ranks sharing one GPU).  Never used for a result.
BACKEND = os.environ.get("MLH_BENCH_BACKEND", "nccl")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU issue ceiling of the integer VOP3 mix these kernels are made of
# (v_mad_u64_u32, v_add/sub with carry, v_cndmask, v_alignbit, v_bitop3): one
# wave64 instruction per 4 cycles per SIMD = 256 CU x 4 SIMD x 16 lanes x
# 2.4 GHz.  Measured: the generated asm butterflies (tools/bfly2_bench.hip)
# 6.45e11 butterflies/s x 60 VALU = 3.87e13 (98.5 %); SHA-256 node hashes
# (tools/sha_latency.hip) 1.65-1.75e10/s x 2272 VALU = 3.75-4.0e13.
VALU_PEAK = 256 * 4 * 16 * 2.4e9
CHIP_MAX_GHZ = 2.4


def _allreduce_max(x):
    """max over ranks of a host float (device tensor for RCCL, host for gloo)."""
    import torch
    import torch.distributed as tdist

    dev = "cuda" if BACKEND == "nccl" else "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())


def _agree_ok(ok):
    """True iff `ok` holds on every rank (rank 0 decides for rank-0-only checks)."""
    return _allreduce_max(0.0 if ok else 1.0) == 0.0


def _gather_shards(t_local, world):
    """Every rank's equal-size device shard, concatenated in rank order, on
    this rank's device (RCCL all-gather; host-staged in a gloo rehearsal)."""
    import torch
    import torch.distributed as tdist

    if BACKEND == "nccl":
        out = torch.empty((world * t_local.shape[0],) + tuple(t_local.shape[1:]), dtype=t_local.dtype,
                          device=t_local.device)
        tdist.all_gather_into_tensor(out, t_local.contiguous())
        return out
    parts = [torch.empty_like(t_local, device="cpu") for _ in range(world)]
    tdist.all_gather(parts, t_local.cpu())
    return torch.cat(parts, 0).to(t_local.device)


def _cyclic_to_natural(g, world):
    """[rank][m] gathered cyclic shards (rank r holds x[r + world m]) -> x."""
    n = g.shape[0] // world
    return g.reshape(world, n, *g.shape[1:]).transpose(0, 1).reshape(g.shape).contiguous()


def _blocks_to_natural(g, world, log_s):
    """[rank][T][2^log_s] gathered block-layout shards -> natural order."""
    S = 1 << log_s
    T = g.shape[0] // world // S
    return g.reshape(world, T, S, *g.shape[1:]).transpose(0, 1).reshape(g.shape).contiguous()


def _test_corrupt(t, rank):
    """Rehearsal hook (MLH_BENCH_TEST_CORRUPT_SHARD=<rank>): that rank alters
    element 0 of its shard after a timed loop, so the in-run check that
    follows must report false.  Never set in a measurement."""
    want = os.environ.get("MLH_BENCH_TEST_CORRUPT_SHARD")
    if want is not None and int(want) == rank:
        if bool((t[0] != 0).any()):
            t[0].zero_()
        else:
            t[0, 0] = 1


def _spot_check_sharded_ntt(x_local, y_local, log_total, gen, log_p, log_s, rank, world, local,
                            samples=8):
    """In-run check of a sharded forward NTT's output: for `samples` seeded
    indices j (plus 0 and N - 1), every rank evaluates its cyclic input shard
    at w^(jP) (mlh_poly_evaluate) and scales it by w^(jg); the ranks' terms
    are all-gathered and summed mod M, giving X[j] independently of the
    all-to-all; the rank holding X[j] (block 2^log_s output layout) compares
    it with its output.  True iff every sampled X[j] matches on every rank."""
    import random

    import torch
    import torch.distributed as tdist

    from multilinear_amd import device as D
    from multilinear_amd import sharded as SH

    rr = random.Random(0xC0FFEE)
    js = [0, (1 << log_total) - 1] + [rr.randrange(1 << log_total) for _ in range(samples)]
    torch.cuda.synchronize()
    terms = SH.ntt_spot_terms(x_local, log_total, gen, rank, world, js, local)
    allt = [None] * world
    tdist.all_gather_object(allt, terms)
    bad = 0
    for i, j in enumerate(js):
        want = sum(t[i] for t in allt) % D.M
        owner, l = SH.ntt_block_owner(j, log_total, log_p, log_s)
        if owner == rank:
            got = D.limbs_to_ints(D.from_device(y_local[l:l + 1]))[0]
            bad += int(got != want)
    return _allreduce_max(bad) == 0


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_baseline(log_n):
    """Oracle C restatement of the reference CPU NTT, 1 thread (bench leg only)."""
    from multilinear_amd import device as D
    from oracle import coracle
    from oracle import field as F

    x = D.random_limbs(1 << log_n, 1)
    g = F.pow_2_generator(log_n)
    # a bounded sample of ~10 s of single-core work: whole 2^log_n transforms
    # until 10 s have passed (at most 4)
    reps, t0 = 0, time.perf_counter()
    while reps < 4 and (reps == 0 or time.perf_counter() - t0 < 10.0):
        coracle.ntt(x, log_n, g)
        reps += 1
    dt = time.perf_counter() - t0
    return {
        "value": reps * (1 << log_n) / dt,
        "unit": "field-elems/s",
        "cores": 1,
        "kind": "port",
        "sample": "%d x 2^%d-point forward NTT, C restatement of src/ntt/mod.rs:69-110 "
                  "(bit-reverse + serial-twiddle DIT), %.2f s in all; host %s, nproc %d"
                  % (reps, log_n, dt, cpu_model(), os.cpu_count() or 0),
    }


def cpu_baseline_fri_commit(log_n, sample_log=None):
    """Config 3 (the metric's "FRI commit ms") on one host core: the oracle's C
    restatement of reed_solomon (fri/mod.rs:19-28, NTT of the zero-padded
    coefficients) and commit_rs_code + Merkle::commit (fri/mod.rs:30-55,
    merkle_tree/mod.rs:65-85: SHA-256 per leaf and node, every layer kept).
    Default: ONE commit at the config's own size, 2^log_n coefficients (~21 s
    of one core at 2^24) -- measured, not extrapolated; a smaller sample_log is
    scaled to 2^log_n (RS by N log N, Merkle by N) and labelled so (bench leg only)."""
    from multilinear_amd import device as D
    from oracle import coracle
    from oracle import field as F

    sl = log_n if sample_log is None else min(sample_log, log_n)
    x = D.random_limbs(1 << sl, 3)
    g2 = F.pow_2_generator(sl + 1)
    t0 = time.perf_counter()
    code = coracle.reed_solomon(x, sl, g2)
    t1 = time.perf_counter()
    layers = coracle.merkle_commit_pairs(code, sl + 1)
    t2 = time.perf_counter()
    del code, layers
    k = float(1 << (log_n - sl))
    rs_ms = (t1 - t0) * 1e3 * k * (log_n + 1) / (sl + 1)
    mk_ms = (t2 - t1) * 1e3 * k
    return {"ms": rs_ms + mk_ms, "rs_ms": rs_ms, "merkle_ms": mk_ms, "cores": 1, "kind": "port",
            "measured_at_config_size": sl == log_n,
            "sample": ("one commit of 2^%d coefficients (2^%d code, 2^%d leaves) in %.2f s, C "
                       "restatement of the reference loops" % (sl, sl + 1, sl, t2 - t0))
                      + ("" if sl == log_n else "; scaled to 2^%d (RS x N log N, Merkle x N)" % log_n)}


def cpu_baseline_all_cores(log_n):
    """OpenMP variant of the same C restatement on the host cores the box
    grants (OMP_NUM_THREADS, else os.cpu_count()); SURVEY.md 8(d)."""
    from multilinear_amd import device as D
    from oracle import coracle
    from oracle import field as F

    threads = int(os.environ.get("OMP_NUM_THREADS") or (os.cpu_count() or 1))
    x = D.random_limbs(1 << log_n, 1)
    g = F.pow_2_generator(log_n)
    coracle.ntt_omp(x[: 1 << 12], 12, F.pow_2_generator(12), threads)  # thread pool warm-up
    reps, t0 = 0, time.perf_counter()
    while reps < 20 and (reps == 0 or time.perf_counter() - t0 < 5.0):
        coracle.ntt_omp(x, log_n, g, threads)
        reps += 1
    dt = time.perf_counter() - t0
    return {
        "value": reps * (1 << log_n) / dt,
        "unit": "field-elems/s",
        "cores": threads,
        "kind": "port",
        "sample": "%d x 2^%d-point forward NTT, OpenMP restatement (stages split over %d threads), "
                  "%.2f s in all" % (reps, log_n, threads, dt),
    }


def load_valu(kernel):
    """SQ_INSTS_VALU per launch of `kernel` from the committed VALU summary
    (tools/valu_summary.py), or None."""
    import glob

    r, tw, z = kernel[len("ntt_pass<"):-1].split(",")
    name = "void mlh::ntt_pass_kernel<%s, %s, %s>" % (r, tw, z)  # ZT: int template argument
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_valu.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        ks = d.get("kernels", {})
        k = ks.get(name) or ks.get(name[:-1] + ", 8>")  # EPT template argument (r01e on)
        if k and d.get("log_n", 24) == 24:
            return k["SQ_INSTS_VALU"], os.path.basename(path)
    return None


def load_sumcheck_pmc():
    """(bytes per config-4 prove, source) from the newest committed
    profiles/*_sumcheck_pmc.json (tools/sumcheck_pmc.py), or None."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_sumcheck_pmc.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("bytes_per_prove"):
            return d["bytes_per_prove"], os.path.basename(path)
    return None


def load_valu_profile():
    """Per-kernel VALU issue reading of every config's dominant kernels from the
    newest committed rocprofv3 VALU pass (profile-derived, not live): lane
    instructions/s against one wave64 instruction per 4 cycles per SIMD at
    the clock the chip held during that kernel (GRBM_GUI_ACTIVE)."""
    import glob

    picks = {"ntt_pass_kernel<8, 0, 0, 8>": "config 2 NTT pass 0",
             "ntt_pass_kernel<8, 1, 0, 8>": "config 2 NTT pass 1",
             "ntt_pass_kernel<8, 2, 0, 8>": "config 2 NTT last pass",
             "ntt_pass_kernel<9, 0, 1, 8>": "config 3 RS LDE pass 0",
             "leaf_pairs_level2_kernel": "config 3 Merkle leaves + 2 levels",
             "fri_fold_leaves_kernel": "FRI fold + next-tree leaves",
             "corner_sums_lo_kernel": "config 4 sumcheck: corner sums of rounds 0-11 (HBM-streaming)",
             "fold_group_eq_kernel<6, false>": "config 4 sumcheck: 6-level fold of the 2^24 table (HBM-streaming)",
             "sumcheck_eq_tail_kernel": "config 4 sumcheck: 12 serial rounds (transcript wave + helper waves), "
                                        "twice (head on the corner sums, tail on the folded table)"}
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_valu.json")), reverse=True)
    if not paths:
        return None
    try:
        d = json.load(open(paths[0]))
    except (OSError, ValueError):
        return None
    out = {"source": os.path.basename(paths[0]),
           "clock": "GRBM_GUI_ACTIVE / 8 XCDs / wall, capped at the chip's %.1f GHz; kernels "
                    "under 50 us get the cap (the derivation breaks for short dispatches)"
                    % CHIP_MAX_GHZ,
           "issue_frac": "lane-instr/s over one wave64 VALU instruction per 4 cycles per SIMD at "
                         "that clock; the clock derivation is good to ~2 %, so issue_frac_raw "
                         "slightly above 1 means at the ceiling (issue_frac caps it at 1)",
           "kernels": {}}
    mix = {}
    mpaths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_isa_mix.json")), reverse=True)
    if mpaths:  # tools/isa_mix.py: the instruction-mix ceiling of each kernel
        try:
            mix = json.load(open(mpaths[0])).get("kernels", {})
            out["mix_source"] = os.path.basename(mpaths[0])
            out["mix_ceiling"] = ("one wave's static VALU mix weighted by the measured per-instruction "
                                  "issue rates (profiles/r04_isa.json): issue_frac_vs_mix = issue over "
                                  "that mix's ceiling at the same clock")
        except (OSError, ValueError):
            mix = {}
    for name, k in d.get("kernels", {}).items():
        for key, what in picks.items():
            if name.endswith("mlh::" + key) and k.get("eff_clock_ghz"):
                clk = k["eff_clock_ghz"] if k["avg_ms"] >= 0.05 else CHIP_MAX_GHZ
                clk = min(clk, CHIP_MAX_GHZ)
                ceiling = 256 * 4 * 64 / 4 * clk * 1e9
                rec = {"what": what, "avg_ms": k["avg_ms"],
                       "lane_instr_per_s": k["lane_instr_per_s"],
                       "clock_ghz": clk,
                       "issue_frac": min(1.0, k["lane_instr_per_s"] / ceiling),
                       "issue_frac_raw": k["lane_instr_per_s"] / ceiling}
                m = mix.get(key)
                if m and m.get("cycles_per_instr"):
                    mc = 256 * 4 * 64 * clk * 1e9 / m["cycles_per_instr"]
                    rec["mix_cycles_per_instr"] = m["cycles_per_instr"]
                    rec["mix_ceiling_lane_instr_per_s"] = mc
                    rec["issue_frac_vs_mix"] = k["lane_instr_per_s"] / mc
                out["kernels"][key] = rec
    return out


def load_pmc(kernel, log_n):
    """HBM traffic per launch from the committed rocprofv3 PMC summary, if it
    matches this kernel/size (tools/pmc_summary.py writes it)."""
    path = os.path.join(ROOT, "profiles", "pmc_ntt.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("log_n") == log_n and kernel in d.get("kernels", {}):
        return d["kernels"][kernel].get("traffic_bytes_per_launch")
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--spinup-s", type=float, default=0.3,
                    help="untimed setup: run the step this long first so clocks settle")
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--prof-every", type=int, default=8,
                    help="HIP-event kernel timer on every k-th step of the timed region (each "
                         "timing event costs the stream a few us; 1 = every step)")
    ap.add_argument("--extra-reps", type=int, default=3, help="reps of the secondary timings")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--extras-budget-s", type=float, default=240.0,
                    help="watchdog on the secondary timings (0: off)")
    ap.add_argument("--headline-budget-s", type=float, default=180.0,
                    help="N > 1: watchdog from before the first collective to the headline "
                         "line (0: off); on expiry rank 0 prints a diagnostic line and every "
                         "rank exits non-zero")
    ap.add_argument("--preflight-bytes", type=int, default=1 << 20,
                    help="N > 1: total bytes of the pre-flight all-to-all (checked pattern)")
    ap.add_argument("--fri-log", type=int, default=28, help="config 5 codeword size (log2)")
    ap.add_argument("--mode", choices=["replicas", "sharded"], default="sharded",
                    help="N > 1 headline step: one N*2^24 transform sharded with an all-to-all "
                         "(default) or each GPU transforms its own 2^24 polynomial (replicas)")
    ap.add_argument("--strong-log", type=int, default=28,
                    help="strong-scaling NTT size (log2), fixed over N; 0: off")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if BACKEND != "nccl":  # rehearsal: ranks may share the box's GPU(s)
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    hw = None
    if world > 1:
        import torch.distributed as dist

        # armed before the first collective (init_process_group with device_id
        # connects eagerly): a stalled exchange ends the run with a line that
        # names the phase instead of a silent kill at the driver's limit
        hw = _HeadlineWatchdog(rank, world, args.headline_budget_s)
        hw.phase("init_process_group")
        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:  # rehearsal of the N > 1 path with several ranks on one GPU
            dist.init_process_group(BACKEND)

    from multilinear_amd import device as D
    from multilinear_amd import fri as MF
    from multilinear_amd.transcript import Transcript

    log_n = args.log_n
    N = 1 << log_n
    lib = D.lib()
    ctx = D.context(local)
    gen = D.fe_bytes(int.from_bytes(bytes(_gen(lib, log_n)), "little"))
    x = D.random_device(N, 1000 + rank, local)
    out = D.empty(N, local)

    if world & (world - 1):
        raise SystemExit("world size must be a power of two")
    log_p = world.bit_length() - 1
    sharded = world > 1 and args.mode == "sharded"

    def ntt_local():
        D.check(lib.mlh_ntt(ctx, D.ptr(x), D.ptr(out), log_n, gen), ctx)

    batch = None
    preflight = None
    if world > 1:  # the C ABI's pipelined sharded NTT over libmlhip's RCCL communicator
        hw.phase("comm_create")
        tp = _transport(local)
        hw.info = tp.info()
        hw.phase("preflight")
        preflight = run_preflight(tp, world, args.preflight_bytes, local)
        hw.preflight = preflight
        if not preflight["ok"]:
            hw.fail("pre-flight all-to-all/all-gather pattern mismatch: %d words on the worst rank"
                    % preflight["mismatches_max"])
        batch = _ShardedBatch(lib, ctx, tp, x, out, log_n + log_p, local)

    def run_steps(k):
        """k headline steps, enqueued (x: this rank's shard / polynomial)."""
        if sharded:
            batch.run(k)  # one mlh_sharded_ntt_batch call: k pipelined transforms
        else:
            for _ in range(k):
                ntt_local()

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # setup (not a step): tables, allocator, clock ramp.  The iteration count
    # is agreed over ranks so the sharded step's collectives stay matched.
    if hw:
        hw.phase("first_step")
    run_steps(1)
    barrier()
    t_one = time.perf_counter()
    run_steps(1)
    torch.cuda.synchronize()
    iters = int(args.spinup_s / max(time.perf_counter() - t_one, 1e-5)) + 1
    if dist is not None:
        iters = int(_allreduce_max(iters))
    if hw:
        hw.phase("spinup")
    run_steps(min(iters, 5000))
    barrier()
    if hw:
        hw.phase("warmup")
    run_steps(args.warmup)
    barrier()
    if hw:
        hw.phase("timed_steps")
    lib.mlh_profile_reset(ctx)
    lib.mlh_profile_enable(ctx, max(1, args.prof_every))
    t0 = time.perf_counter()
    run_steps(args.steps)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    lib.mlh_profile_enable(ctx, 0)
    elapsed = t1 - t0
    if dist is not None:
        elapsed = _allreduce_max(elapsed)
    barrier()

    if hw:
        hw.phase("headline_checks")
    # dominant kernel timing (HIP events on the launch stream, timed region)
    kernels = {}
    labels = ["ntt_pass<%d,%d,%d>" % (r, tw, z) for r in range(4, 10) for tw in (0, 1, 2, 3, 5)
              for z in range(3)] + ["shard_dft<%d,0>" % p for p in range(1, 5)] + ["ntt_all_to_all",
                                                                                     "ntt_fused_pre",
                                                                                     "ntt_fused_last"]
    for lab in labels:
        cnt = ctypes.c_uint64()
        tot = ctypes.c_double()
        lib.mlh_profile_get(ctx, lab.encode(), ctypes.byref(cnt), ctypes.byref(tot))
        if cnt.value:
            kernels[lab] = {"launches": cnt.value, "avg_ms": tot.value / cnt.value}
    fused = batch is not None and sharded and batch.fused
    pref = "ntt_fused" if fused else "ntt_pass"
    dom = max(((k, v) for k, v in kernels.items() if k.startswith(pref)),
              key=lambda kv: kv[1]["avg_ms"] * kv[1]["launches"])
    dom_name, dom_stat = dom
    # the NTT's algorithmic bytes are 2 x 16 x N for the whole
    # transform; a pass is credited with its share (passes = NTT launches per step)
    if fused:  # the fused pre launch runs npre passes, the last launch one
        npre = (log_n - (9 - log_p) + 8) // 9
        passes = npre + 1
        share = npre if dom_name == "ntt_fused_pre" else 1
    else:
        passes = max(1, round(sum(v["launches"] for k, v in kernels.items() if k.startswith("ntt_pass"))
                              / dom_stat["launches"]))
        share = 1
    alg_bytes = 32.0 * N * share / passes
    achieved_gbs = alg_bytes / (dom_stat["avg_ms"] * 1e-3) / 1e9
    traffic = load_pmc(dom_name, log_n)
    valu = load_valu(dom_name) if log_n == 24 and dom_name.startswith("ntt_pass") else None
    valu_frac = (valu[0] * 64 / (dom_stat["avg_ms"] * 1e-3) / VALU_PEAK) if valu else None

    ms_per_step = elapsed / args.steps * 1e3
    # the live timer's own cost: the sampled launches are bracketed by HIP
    # events, so the per-pass averages summed over one step exceed the
    # unsampled step time by the events' overhead; per launch
    pass_sum = sum(v["avg_ms"] for k, v in kernels.items() if k.startswith("ntt_pass"))
    timing_overhead_us = ((pass_sum - ms_per_step) * 1e3 / passes
                          if not sharded and pass_sum and world == 1 else None)
    value = N * args.steps * world / elapsed
    result = {
        "metric": "NTT 2^24 field-elems/sec + FRI commit ms; % HBM roofline at 1/2/4/8 GPUs",
        "value": value,
        "unit": "field-elems/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u128 mod M (F_M, M = 2^128 - 45*2^40 + 1)",
        "data": "synthetic: seeded uniform field elements generated on device",
        "config": {
            "workload": ("config 2: forward 2^%d-point NTT per step per GPU, natural order "
                         "in/out, device resident" % log_n) if not sharded else
                        ("sharded forward 2^%d-point NTT per step (2^%d per GPU): cyclic shards "
                         "in, block-cyclic out, one RCCL all-to-all" % (log_n + log_p, log_n)),
            "log_n": log_n + (log_p if sharded else 0),
            "parallelism": "single GPU" if world == 1 else
                           ("replicas x%d (independent 2^%d polynomial per GPU)" % (world, log_n)
                            if not sharded else
                            ("sharded x%d (four-step NTT, RCCL all-to-all over xGMI)" % world
                             if BACKEND == "nccl" else
                             "sharded x%d (four-step NTT, host-staged %s all-to-all: a rehearsal, "
                             "not a measurement)" % (world, BACKEND))),
        },
        "ntt_hbm_frac": (32.0 * N / (ms_per_step * 1e-3) / 1e9) / HBM_PEAK_GBS,
        "roofline": {
            "bound": ("valu" if valu_frac > achieved_gbs / HBM_PEAK_GBS else "hbm") if valu_frac is not None
                     else ("valu" if dom_name.startswith("ntt_") else "hbm"),
            "bound_source": "SQ_INSTS_VALU of this kernel (valu_frac)" if valu_frac is not None else
                            ("the ntt_pass kernels this phase launches, VALU-issue bound per their "
                             "N = 1 counters (valu_profile)" if dom_name.startswith("ntt_") else None),
            "kernel": dom_name,
            "achieved": achieved_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS,
            "traffic": traffic,
            "launch_avg_ms": dom_stat["avg_ms"],
            "launch_timing": "HIP events on the launch stream around %s of the timed region "
                             "(%d timed launches)" % (
                                 "every step" if args.prof_every <= 1
                                 else "every %dth step" % args.prof_every, dom_stat["launches"]),
            "launch_timing_overhead_us": timing_overhead_us,
            "launch_timing_overhead_rule": "(sum of the per-pass live averages - ms_per_step) / passes: "
                                           "what the HIP events add to a sampled launch; launch_avg_ms "
                                           "includes it, so `achieved` is a slight underestimate",
            "alg_bytes_per_launch": alg_bytes,
            "alg_bytes_rule": "32 B x 2^%d x %d / %d passes (SURVEY.md 8(d))" % (log_n, share, passes),
            "valu_frac": valu_frac,
        },
        "kernels": kernels,
    }
    if valu:
        rate = valu[0] * 64 / (dom_stat["avg_ms"] * 1e-3)
        result["valu_roofline"] = {
            "kernel": dom_name, "achieved": rate, "unit": "lane-instr/s",
            "peak": VALU_PEAK, "frac": rate / VALU_PEAK,
            "peak_rule": "one wave64 VALU instruction per 4 cycles per SIMD at 2.4 GHz",
            "source": "SQ_INSTS_VALU per launch (%s) x 64 lanes / live avg launch time" % valu[1],
        }
    vp = load_valu_profile() if log_n == 24 else None
    if vp:
        result["valu_profile"] = vp
    if world > 1:
        # self-certification of the N > 1 line: the ranks RCCL itself reports,
        # the sharded step's phases, and its output spot-checked in-run
        tinfo = _transport(local).info()
        result["comm"] = tinfo
        result["rccl_ranks"] = tinfo["ranks"] if tinfo["transport"] == "rccl" else None
        if sharded:
            result["sharded_phases"] = sharded_phases(kernels, log_n, log_p, passes)
            result["sharded_algorithm"] = batch.algorithm
            result["sharded_output_block_log"] = batch.log_s if batch.fused else log_n - log_p
            try:
                result["sharded_ntt_verified"] = sharded_ntt_check(batch, log_n, log_p, rank, world,
                                                                   local)
            except Exception as e:  # keep the headline line; report the failure
                result["sharded_ntt_verified"] = False
                result["sharded_ntt_check_error"] = "%s: %s" % (type(e).__name__, e)

    if preflight is not None:
        result["preflight"] = preflight
    if hw:
        hw.disarm()
    # The extras run collectives at N > 1; if one of them stalls (a rank raising
    # inside a sharded prove leaves the others waiting in RCCL), every rank's
    # watchdog prints the headline line measured above and ends the process, so
    # the driver still gets the K-step measurement.
    watchdog = _ExtrasWatchdog(result, rank, args.extras_budget_s)

    if not args.no_extras and world == 1:
        reps = args.extra_reps
        # inverse NTT (out = NTT(x), so x is rewritten with itself); one
        # untimed call builds the inverse twiddle tables
        D.check(lib.mlh_intt(ctx, D.ptr(out), D.ptr(x), log_n, gen), ctx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            D.check(lib.mlh_intt(ctx, D.ptr(out), D.ptr(x), log_n, gen), ctx)
        torch.cuda.synchronize()
        result["intt_ms"] = (time.perf_counter() - t0) / 10 * 1e3
        # Vec -> Vec through pageable host buffers (mlh_ntt_host: the reference's
        # Polynomial::ntt signature, PCIe copies included) -- reported, never `value`
        hin = (ctypes.c_uint8 * (16 * N)).from_buffer(bytearray(x.cpu().numpy().tobytes()))
        hout = (ctypes.c_uint8 * (16 * N))()
        D.check(lib.mlh_ntt_host(ctx, hin, hout, log_n, gen, 0), ctx)
        t0 = time.perf_counter()
        for _ in range(reps):
            D.check(lib.mlh_ntt_host(ctx, hin, hout, log_n, gen, 0), ctx)
        host_ms = (time.perf_counter() - t0) / reps * 1e3
        result["ntt_host_pcie_inclusive"] = {"ms": host_ms, "field_elems_per_s": N / (host_ms * 1e-3),
                                             "note": "host in -> H2D -> NTT -> D2H -> host out"}
        del hin, hout
        # FRI commit (config 3): coeffs (2^log_n) -> RS code -> Merkle root
        code = D.empty(2 * N, local)
        layers = torch.empty((N * 2 - 1, 32), dtype=torch.uint8, device="cuda:%d" % local)
        g2 = D.fe_bytes(int.from_bytes(bytes(_gen(lib, log_n + 1)), "little"))
        root = (ctypes.c_uint8 * 32)()

        def fri_commit():
            D.check(lib.mlh_reed_solomon(ctx, D.ptr(x), log_n, g2, D.ptr(code)), ctx)
            D.check(lib.mlh_merkle_commit_pairs(ctx, D.ptr(code), log_n + 1, D.ptr(layers), root), ctx)

        # untimed spin-up, as the headline's (--spinup-s): the first ~10 commits
        # after the NTT loop run ~7 % slower while the clocks settle
        t_spin = time.perf_counter()
        n_spin = 0
        while n_spin < 3 or time.perf_counter() - t_spin < args.spinup_s:
            fri_commit()
            n_spin += 1
            if n_spin % 8 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        creps = max(reps, 10)  # ~30 ms of commits: a steadier mean than 3
        t0 = time.perf_counter()
        for _ in range(creps):
            fri_commit()
        torch.cuda.synchronize()
        fc_ms = (time.perf_counter() - t0) / creps * 1e3
        fc_bytes = 16 * N + 32 * N + 32 * N + 32 * (2 * N - 1)
        result["fri_commit_ms"] = fc_ms
        result["fri_commit_hbm_frac"] = fc_bytes / (fc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
        # split: the RS LDE alone, the Merkle tree = the rest; the tree is
        # 2^24 one-block leaf hashes + (2^24 - 1) two-block node hashes
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(creps):
            D.check(lib.mlh_reed_solomon(ctx, D.ptr(x), log_n, g2, D.ptr(code)), ctx)
        torch.cuda.synchronize()
        rs_ms = (time.perf_counter() - t0) / creps * 1e3
        result["fri_commit_rs_ms"] = rs_ms
        result["fri_commit_merkle_ms"] = fc_ms - rs_ms
        result["merkle_sha256_compressions_per_s"] = (N + 2 * (N - 1)) / ((fc_ms - rs_ms) * 1e-3)
        # full FRI prove (fold, 24 trees, 128 queries) on the same code
        p = MF.FriProof.prove(code, Transcript(), local)  # warm-up: pool, tables
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            p = MF.FriProof.prove(code, Transcript(), local)
        torch.cuda.synchronize()
        result["fri_prove_ms"] = (time.perf_counter() - t0) / reps * 1e3
        result["fri_prove_verified"] = bool(p.verify())
        del layers
        # sumcheck (config 4): 24 rounds over evals (2^log_n) with a random point
        import random

        from multilinear_amd import polynomials as MPL
        from multilinear_amd import sumcheck as MS

        rr = random.Random(5)
        M = D.M
        pts = [rr.randrange(M) for _ in range(log_n)]
        delta = MPL.eq_table(pts, local)  # warm (allocation, first launch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            delta = MPL.eq_table(pts, local)
        torch.cuda.synchronize()
        result["eq_table_ms"] = (time.perf_counter() - t0) * 1e3 / 5
        # two-table rounds over the materialised delta (eq table timed above)
        # (the rounds fold both tables in place: fresh copies per rep, made
        # outside the timed region; the first rep is the warm-up)
        for _ in range(2):
            tabs = MS.SumcheckTables(x.clone(), delta.clone())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tabs.compute_sumcheck_polynomials(0, Transcript(), local)
            torch.cuda.synchronize()
            result["sumcheck_two_table_ms"] = (time.perf_counter() - t0) * 1e3
            del tabs
        # build_tables_for_pcs + 24 rounds with delta kept factored (the PCS
        # path): eq factor tables built inside, only the matrix streamed
        def sc_eq():
            t = MS.SumcheckTables.build_tables_for_pcs(pts, x, local)
            t.compute_sumcheck_polynomials(0, Transcript(), local)

        sc_eq()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            sc_eq()
        torch.cuda.synchronize()
        result["sumcheck_py_ms"] = (time.perf_counter() - t0) * 1e3 / 5
        # the same prove through the C ABI as a native caller makes it
        # (mlh_sumcheck_prove_eq: setup, 24 rounds, D2H of the round
        # polynomials, host transcript replay), arguments marshalled outside
        # the timed region; the Python mirror's int conversions are excluded
        from multilinear_amd.polynomials import _points

        work = D.empty(N // 2, local)
        cpts = _points(pts)
        csum = (ctypes.c_uint8 * 16)()
        cpol = (ctypes.c_uint8 * (32 * log_n))()
        crs = (ctypes.c_uint8 * (16 * log_n))()
        cdl = (ctypes.c_uint8 * 16)()
        trs = [Transcript() for _ in range(25)]
        torch.cuda.synchronize()
        sc_times = []
        for rep in range(25):
            t0 = time.perf_counter()
            D.check(lib.mlh_sumcheck_prove_eq(ctx, D.ptr(x), D.ptr(work), log_n, cpts, csum,
                                              trs[rep].h, cpol, crs, cdl), ctx)
            sc_times.append(time.perf_counter() - t0)
        sc_ms = sum(sc_times[5:]) / 20 * 1e3  # the call synchronises; first 5 = warm-up
        del work
        result["sumcheck_ms"] = sc_ms
        # HBM fraction of the prove: `frac` is the
        # measured one -- the bytes the grouped eq-factored path moves per
        # prove, from the newest committed FETCH_SIZE / WRITE_SIZE passes
        # (tools/sumcheck_pmc.py) -- or null without them.  The reference
        # schedule's bytes (per round read matrix + delta, write
        # both folded, plus the 2^24-entry eq table = 1.88 GB) are an
        # equivalence figure only: what the per-round two-table schedule would
        # have to stream at this prove time, not traffic this path moves.
        ref_bytes = sum(48 * (N >> k) for k in range(log_n)) + 16 * N
        pmc = load_sumcheck_pmc() if log_n == 24 else None
        hf = {"frac": None, "bytes": None,
              "what": "measured HBM bytes per prove (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE) / "
                      "prove time / 8 TB/s"}
        if pmc:
            hf.update({"frac": pmc[0] / (sc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "bytes": pmc[0],
                       "source": pmc[1]})
        hf["reference_schedule_equiv"] = {
            "bytes": ref_bytes, "frac": ref_bytes / (sc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "what": "NOT traffic of this path: SURVEY §8(d)'s bytes of the reference's per-round "
                    "two-table schedule (sum over rounds of 2 S 16 B read + S 16 B written, plus the "
                    "2^24-entry eq table) over this prove's time"}
        result["sumcheck_hbm_frac"] = hf

        # PCSProof::prove (multilinear_pcs.rs:90-136) on the 2^log_n evaluations:
        # Moebius + fused bit-reverse/RS (2^(log_n+1) code) + log_n interleaved
        # sumcheck/FRI rounds + 128 queries; one warm-up, then the mean of 3
        from multilinear_amd.multilinear_pcs import PCSProof

        out_claim = MPL.evaluate(x, pts, local)  # the true claim, so the proof verifies
        PCSProof.prove(pts, out_claim, x, Transcript(), local)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            pcs = PCSProof.prove(pts, out_claim, x, Transcript(), local)
        torch.cuda.synchronize()
        result["pcs_prove_ms"] = (time.perf_counter() - t0) * 1e3 / 3
        result["pcs_prove_n_vars"] = log_n
        result["pcs_verified"] = bool(pcs.verify(Transcript()))
        del pcs
        try:
            result["reference_test_points"] = reference_test_points(lib, ctx, local, reps)
        except Exception as e:  # keep the headline line; report the failure
            result["reference_test_points_error"] = "%s: %s" % (type(e).__name__, e)

    if not args.no_extras and args.fri_log:
        try:
            result.update(config5(args, lib, ctx, local, world, rank, barrier))
        except Exception as e:  # keep the headline line; report the failure
            result["config5_error"] = "%s: %s" % (type(e).__name__, e)
        if world > 1 and not sharded:
            try:
                result["sharded_ntt"] = sharded_ntt_extra(args, batch, world, barrier, log_n,
                                                          log_p, lib, ctx)
            except Exception as e:
                result["sharded_ntt_error"] = "%s: %s" % (type(e).__name__, e)
        if world > 1 and sharded:
            try:
                result["replicas_ntt"] = replicas_ntt_extra(args, ntt_local, world, barrier, log_n)
            except Exception as e:
                result["replicas_ntt_error"] = "%s: %s" % (type(e).__name__, e)
    if not args.no_extras and args.strong_log:
        try:
            result["strong_ntt"] = strong_ntt(args, lib, ctx, local, world, rank, barrier)
        except Exception as e:
            result["strong_ntt_error"] = "%s: %s" % (type(e).__name__, e)
        if world > 1:
            try:
                result.update(config4_sharded(args, local, world, rank, barrier))
            except Exception as e:
                result["config4_sharded_error"] = "%s: %s" % (type(e).__name__, e)

    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(log_n)
        try:
            result["cpu_baseline_all_cores"] = cpu_baseline_all_cores(log_n)
        except Exception as e:  # the 1-core baseline stays the reported one
            result["cpu_baseline_all_cores"] = {"error": str(e)}
        result["vs_cpu_1core"] = value / result["cpu_baseline"]["value"]
        if not args.no_extras and result.get("fri_commit_ms"):
            try:
                cf = cpu_baseline_fri_commit(log_n)
                result["cpu_baseline_fri_commit"] = cf
                result["fri_commit_vs_cpu_1core"] = cf["ms"] / result["fri_commit_ms"]
            except Exception as e:
                result["cpu_baseline_fri_commit"] = {"error": str(e)}

    if dist is not None:
        dist.barrier()
    if not watchdog.claim():
        return  # the watchdog has printed the line and is ending the process
    if dist is not None:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


def run_preflight(tp, world, total_bytes, local):
    """mlh_comm_preflight through the headline's transport: an all-to-all of
    total_bytes (total_bytes / world per rank pair) and an all-gather, each
    word tagged with (source, destination, position) and checked on the
    device; the worst rank's mismatch count is agreed over ranks."""
    from multilinear_amd import sharded as SH

    per = max(4, (total_bytes // world) // 4 * 4)
    bad, ms = SH.preflight(tp, per, local)
    worst = int(_allreduce_max(bad))
    return {"bytes_per_rank_pair": per, "all_to_all_bytes": per * world, "mismatches_max": worst,
            "ok": worst == 0, "ms_rank0": ms,
            "transport": "rccl" if BACKEND == "nccl" else "host-staged " + BACKEND}


class _HeadlineWatchdog:
    """N > 1 guard from before the first collective until the headline line is
    built.  phase() records how far this rank got; if budget_s passes first (a
    stalled init, pre-flight or exchange -- RCCL waits forever for a missing
    peer), rank 0 prints one JSON line with the metric, "value": null,
    "headline_error", the phase reached, the per-phase times and what RCCL
    reported (rccl_ranks), and every rank ends with os._exit(3).  fail() does
    the same at once for a detected error (pre-flight mismatch)."""

    def __init__(self, rank, world, budget_s):
        import threading

        self.rank, self.world = rank, world
        self.info, self.preflight = None, None
        self._t0 = time.perf_counter()
        self._phases = []
        self._lock = threading.Lock()
        self._done = False
        self._timer = threading.Timer(budget_s, self._fire)
        self._timer.daemon = True
        self.budget_s = budget_s
        if budget_s > 0:
            self._timer.start()

    def phase(self, name):
        self._phases.append((name, round(time.perf_counter() - self._t0, 3)))

    def disarm(self):
        self._timer.cancel()
        with self._lock:
            self._done = True

    def _line(self, error):
        info = self.info or {}
        return {
            "metric": "NTT 2^24 field-elems/sec + FRI commit ms; % HBM roofline at 1/2/4/8 GPUs",
            "value": None, "unit": "field-elems/s", "n_gpus": self.world, "higher_is_better": True,
            "headline_error": error,
            "phase": self._phases[-1][0] if self._phases else None,
            "phases_started_s": dict(self._phases),
            "comm": self.info,
            "rccl_ranks": info.get("ranks") if info.get("transport") == "rccl" else None,
            "preflight": self.preflight,
        }

    def _end(self, error, code):
        with self._lock:
            if self._done:
                return
            self._done = True
        if self.rank == 0:
            print(json.dumps(self._line(error)), flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(code)

    def _fire(self):
        self._end("watchdog: phase %r did not finish within %.0f s"
                  % (self._phases[-1][0] if self._phases else None, self.budget_s), 3)

    def fail(self, error):
        self._timer.cancel()
        self._end(error, 4)


class _ExtrasWatchdog:
    """After budget_s seconds: rank 0 prints the headline fields (snapshot taken
    when armed) plus "extras_error", then the process exits with status 0.
    claim() is called by the main thread when the extras finished in time; the
    first of the two to take the lock prints."""

    def __init__(self, result, rank, budget_s):
        import threading

        self._snap = json.loads(json.dumps(result))
        self._rank = rank
        self._lock = threading.Lock()
        self._done = False
        self._timer = threading.Timer(budget_s, self._fire)
        self._timer.daemon = True
        if budget_s > 0:
            self._timer.start()

    def _take(self):
        with self._lock:
            if self._done:
                return False
            self._done = True
            return True

    def claim(self):
        self._timer.cancel()
        return self._take()

    def _fire(self):
        if not self._take():
            return
        if self._rank == 0:
            self._snap["extras_error"] = "secondary timings exceeded the watchdog budget"
            print(json.dumps(self._snap), flush=True)
        sys.stdout.flush()
        os._exit(0)


class _ShardedBatch:
    """k sharded forward NTTs of the rank's shard as ONE mlh_sharded_ntt_batch
    call (C ABI, csrc/sharded.hip): outputs alternate between two buffers;
    the pointer arrays are built once per k, outside any timed region."""

    def __init__(self, lib, ctx, transport, x, out, log_total, local, fused=True):
        from multilinear_amd import device as D

        self.lib, self.ctx, self.tp, self.log_total = lib, ctx, transport, log_total
        self.x, self.outs = x, [out, D.empty(x.shape[0], local)]
        self.gen = D.fe_bytes(int.from_bytes(bytes(_gen(lib, log_total)), "little"))
        self.arrays = {}
        # the fused schedule (rank digit in the last pass) where it applies;
        # else the local NTT + all-to-all + cross-shard DFT batch
        self.fused, self.log_s = False, None
        if fused:
            ls = ctypes.c_uint32()
            st = lib.mlh_sharded_ntt_fused_batch(ctx, ctypes.byref(transport.transport), None, None, 0,
                                                 log_total, self.gen, ctypes.byref(ls))
            if st == 0:
                self.fused, self.log_s = True, ls.value
        self.algorithm = ("fused: local passes, one all-to-all, the last pass over the received chunks "
                          "(mlh_sharded_ntt_fused_batch)" if self.fused else
                          "local NTT, one all-to-all, cross-shard DFT (mlh_sharded_ntt_batch)")

    def prepare(self, k):
        if k not in self.arrays:
            ins = (ctypes.c_void_p * max(1, k))(*([self.x.data_ptr()] * k))
            outs = (ctypes.c_void_p * max(1, k))(*[self.outs[i & 1].data_ptr() for i in range(k)])
            self.arrays[k] = (ins, outs)
        return self.arrays[k]

    def run(self, k):
        from multilinear_amd import device as D

        if k <= 0:
            return
        ins, outs = self.prepare(k)
        if self.fused:
            D.check(self.lib.mlh_sharded_ntt_fused_batch(self.ctx, ctypes.byref(self.tp.transport), ins, outs,
                                                         k, self.log_total, self.gen, None), self.ctx)
        else:
            D.check(self.lib.mlh_sharded_ntt_batch(self.ctx, ctypes.byref(self.tp.transport), ins, outs, k,
                                                   self.log_total, self.gen, 0), self.ctx)


def sharded_phases(kernels, log_n, log_p, passes):
    """Per-launch durations (HIP events on each phase's own stream, the
    sampled steps of the timed region) of the sharded step's three phases:
    the local 2^log_n NTT (its passes summed), the all-to-all (side stream),
    and the cross-shard DFT.  The pipeline overlaps the all-to-all of step i
    with the local NTT of step i + 1, so the phases need not add up to the
    step time.  all_to_all_gbs: bytes this rank sends to the others
    ((P - 1) / P of its 16 x 2^log_n-byte shard) per all-to-all duration."""
    P = 1 << log_p
    loc = [v["avg_ms"] for k, v in kernels.items() if k.startswith("ntt_pass")]
    if not loc and "ntt_fused_pre" in kernels:  # fused: the local passes but the last, one launch set
        loc = [kernels["ntt_fused_pre"]["avg_ms"]]
    a2a = kernels.get("ntt_all_to_all")
    dft = kernels.get("shard_dft<%d,0>" % log_p) or kernels.get("ntt_fused_last")
    sent = 16.0 * (1 << log_n) * (P - 1) / P
    return {
        "local_ntt_ms": sum(loc) if loc else None,
        "local_ntt_passes": passes,
        "all_to_all_ms": a2a["avg_ms"] if a2a else None,
        "all_to_all_bytes_sent_per_rank": sent,
        "all_to_all_gbs": sent / (a2a["avg_ms"] * 1e-3) / 1e9 if a2a else None,
        "shard_dft_ms": dft["avg_ms"] if dft else None,
        "shard_dft_what": ("the fused last pass (rank digit + the last local digit, on the received "
                           "chunks)" if "ntt_fused_last" in kernels else "the cross-shard DFT"),
        "timing": "HIP events around every sampled launch (mlh_profile_*), per rank 0",
    }


def sharded_ntt_check(batch, log_n, log_p, rank, world, local, samples=8):
    """In-run check of the sharded headline's output (_spot_check_sharded_ntt
    on one more step of the batch: outs[0] = NTT(x))."""
    import torch

    LT = log_n + log_p
    gen = int.from_bytes(bytes(batch.gen), "little")
    batch.run(1)
    torch.cuda.synchronize()
    return _spot_check_sharded_ntt(batch.x, batch.outs[0], LT, gen, log_p,
                                   batch.log_s if batch.fused else LT - 2 * log_p, rank, world, local,
                                   samples)


def sharded_ntt_extra(args, batch, world, barrier, log_n, log_p, lib, ctx):
    """The all-to-all sharded NTT (north star: "the NTT shards across the GPUs
    via an RCCL all-to-all transpose"): N*2^24 points per step, 2^24 per GPU,
    the K steps one pipelined mlh_sharded_ntt_batch call; same K / W as the
    headline."""
    import torch

    batch.run(max(1, args.warmup))
    batch.prepare(args.steps)
    barrier()
    lib.mlh_profile_reset(ctx)
    lib.mlh_profile_enable(ctx, max(1, args.prof_every))
    t0 = time.perf_counter()
    batch.run(args.steps)
    torch.cuda.synchronize()
    dt = _allreduce_max(time.perf_counter() - t0)
    lib.mlh_profile_enable(ctx, 0)
    c, t = ctypes.c_uint64(), ctypes.c_double()
    lib.mlh_profile_get(ctx, ("shard_dft<%d,0>" % log_p).encode(), ctypes.byref(c), ctypes.byref(t))
    return {"metric": "sharded NTT field-elems/s", "value": (1 << (log_n + log_p)) * args.steps / dt,
            "ms_per_step": dt / args.steps * 1e3, "log_n": log_n + log_p,
            "scaling": "weak (2^%d per GPU)" % log_n,
            "shard_dft_avg_ms": (t.value / c.value) if c.value else None,
            "layout": "cyclic shards in, block-cyclic (2^%d) out" % (log_n - log_p)}


def replicas_ntt_extra(args, ntt_local, world, barrier, log_n):
    """Every GPU transforms its own 2^24-point polynomial (independent objects,
    no collective): the weak-scaling ceiling the sharded headline compares to."""
    import torch

    for _ in range(max(1, args.warmup)):
        ntt_local()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ntt_local()
    torch.cuda.synchronize()
    dt = _allreduce_max(time.perf_counter() - t0)
    return {"value": (1 << log_n) * world * args.steps / dt, "unit": "field-elems/s",
            "ms_per_step": dt / args.steps * 1e3, "scaling": "weak (independent 2^%d per GPU)" % log_n}


def strong_ntt(args, lib, ctx, local, world, rank, barrier):
    """Fixed-size strong scaling: one 2^L-point forward NTT (L = --strong-log,
    28 by default), on one GPU at N = 1 and sharded over the N ranks (cyclic
    shards in, one all-to-all) otherwise.  hbm_frac: 32 B x 2^L algorithmic
    bytes over the time, against N x 8 TB/s."""
    import torch

    from multilinear_amd import device as D

    L = args.strong_log
    g = int.from_bytes(bytes(_gen(lib, L)), "little")
    reps = max(1, min(args.extra_reps, 5))
    if world == 1:
        xs = D.random_device(1 << L, 4242, local)
        ys = D.empty(1 << L, local)
        gb = D.fe_bytes(g)

        def run():
            D.check(lib.mlh_ntt(ctx, D.ptr(xs), D.ptr(ys), L, gb), ctx)
    else:  # mlh_sharded_ntt over libmlhip's RCCL communicator
        from multilinear_amd import sharded as SH

        tr = _transport(local)
        log_p = world.bit_length() - 1
        xs = D.random_device(1 << (L - log_p), 4242 + rank, local)

        def run():
            return SH.ntt(xs, L, g, tr, device=local)

    run()
    barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        y = run()
    torch.cuda.synchronize()
    dt = _allreduce_max(time.perf_counter() - t0) / reps if world > 1 else \
        (time.perf_counter() - t0) / reps
    res = {"log_n": L, "ms": dt * 1e3, "value": (1 << L) / dt, "unit": "field-elems/s",
           "scaling": "strong (2^%d total, %s)" % (L, "single GPU" if world == 1 else
                                                  "2^%d per GPU" % (L - world.bit_length() + 1)),
           "hbm_frac": 32.0 * (1 << L) / dt / (world * HBM_PEAK_GBS * 1e9)}
    if world > 1:  # the last timed output, spot-checked as the headline is
        _test_corrupt(xs, rank)
        try:
            res["verified"] = _spot_check_sharded_ntt(xs, y, L, g, log_p, L - 2 * log_p, rank, world, local)
        except Exception as e:
            res["verified"] = False
            res["check_error"] = "%s: %s" % (type(e).__name__, e)
    return res


def config4_sharded(args, local, world, rank, barrier):
    """Config 4 over the N ranks (strong scaling): 2^24-entry MLE in the cyclic
    layout, sharded eq table + 24 sumcheck rounds; and config 3 sharded
    (RS LDE + commit root); all through the C ABI's mlh_sharded_*."""
    import random

    import torch

    from multilinear_amd import device as D
    from multilinear_amd import sharded as SH
    from multilinear_amd.transcript import Transcript

    n = args.log_n
    tr = _transport(local)
    rr = random.Random(5)
    pts = [rr.randrange(D.M) for _ in range(n)]
    base = D.random_device(1 << (n - world.bit_length() + 1), 500 + rank, local)

    def run():  # the C-ABI schedule over libmlhip's RCCL communicator
        m = base.clone()
        d = SH.eq_table(pts, tr, local)
        return SH.sumcheck_prove(m, d, n, 0, Transcript(), tr, local)

    # config 3 sharded: RS LDE of 2^n coefficients + Merkle root over the ranks
    coeffs = D.random_device(1 << (n - world.bit_length() + 1), 700 + rank, local)
    g2 = int.from_bytes(bytes(_gen(D.lib(), n + 1)), "little")

    def commit():
        code = SH.reed_solomon(coeffs, n, g2, tr, local)
        return SH.commit_rs_code(code, n + 1, tr, local)

    commit()
    barrier()
    t0 = time.perf_counter()
    for _ in range(max(1, min(args.extra_reps, 3))):
        root = commit()
    torch.cuda.synchronize()
    commit_ms = _allreduce_max((time.perf_counter() - t0) / max(1, min(args.extra_reps, 3))) * 1e3
    out = {"config3_sharded_fri_commit_ms": commit_ms}
    # in-run parity: rank 0 recomputes reed_solomon + commit_rs_code on ONE GPU
    # from the gathered coefficients; the root must equal the sharded one
    _test_corrupt(coeffs, rank)
    try:
        nat = _cyclic_to_natural(_gather_shards(coeffs, world), world)
        ok = True
        if rank == 0:
            from multilinear_amd import fri as MF
            from multilinear_amd import merkle_tree as MM

            code1 = MF.reed_solomon(nat, g2, local)
            ok = MM.Merkle.commit_pairs(code1, local).root() == root
            del code1
        del nat
        out["config3_sharded_matches_single_gpu"] = _agree_ok(ok)
    except Exception as e:
        out["config3_sharded_matches_single_gpu"] = False
        out["config3_sharded_check_error"] = "%s: %s" % (type(e).__name__, e)

    run()
    barrier()
    reps = max(1, min(args.extra_reps, 3))
    t0 = time.perf_counter()
    for _ in range(reps):
        polys, rs = run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    out.update({"config4_sharded_eq_sumcheck_ms": _allreduce_max(dt) * 1e3,
                "config4_layout": "sharded x%d (cyclic by low index bits)" % world})
    # in-run parity: every round polynomial and challenge against the
    # single-GPU prove (build_tables_for_pcs + compute_sumcheck_polynomials)
    # of the gathered table, on rank 0
    _test_corrupt(base, rank)
    try:
        nat = _cyclic_to_natural(_gather_shards(base, world), world)
        ok = True
        if rank == 0:
            from multilinear_amd import sumcheck as MS

            p1, r1 = MS.SumcheckTables.build_tables_for_pcs(pts, nat, local).compute_sumcheck_polynomials(
                0, Transcript(), local)
            ok = p1 == polys and r1 == rs
        del nat
        out["config4_sharded_matches_single_gpu"] = _agree_ok(ok)
    except Exception as e:
        out["config4_sharded_matches_single_gpu"] = False
        out["config4_sharded_check_error"] = "%s: %s" % (type(e).__name__, e)
    return out


def reference_test_points(lib, ctx, local, reps):
    """The reference's own benchmark!() points, same sizes and inputs, on the
    device (its numbers are printed, never published: BASELINE.md section 1):
    ntt/mod.rs:191-201 (2^18 NTT -> INTT, coeffs i), fri/mod.rs:365-398 (2^20
    values i: gen_pows(21), RS, FriProof::prove, verify, bincode size),
    multilinear_pcs.rs:210-228 (20 vars, evals 7i + 3, inputs 0..19: prove,
    verify), batched_pcs.rs:261-306 (20 vars x 10 polys, evals (3j + 5i) % 100:
    prove, verify).  Median of `reps` timed calls after one warm-up; device
    calls end synchronised (the provers sync inside; the transforms here)."""
    import numpy as np
    import torch

    from multilinear_amd import device as D
    from multilinear_amd import fri as MF
    from multilinear_amd import ntt as MN
    from multilinear_amd import polynomials as MPL
    from multilinear_amd.batched import BatchedPCSProof
    from multilinear_amd.multilinear_pcs import PCSProof
    from multilinear_amd.transcript import Transcript

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        out = None
        for _ in range(max(1, reps)):
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        return ts[len(ts) // 2], out

    def dev_ints(vals):
        a = np.zeros((len(vals), 4), dtype=np.uint32)
        a[:, 0] = vals
        return torch.from_numpy(a.view(np.int32)).to("cuda:%d" % local)

    res = {}
    # ntt/mod.rs:191-201
    n18 = 1 << 18
    c18 = dev_ints(np.arange(n18, dtype=np.uint32))
    ev18, back = D.empty(n18, local), D.empty(n18, local)
    g18 = _gen(lib, 18)
    t_ntt, _ = timed(lambda: D.check(lib.mlh_ntt(ctx, D.ptr(c18), D.ptr(ev18), 18, g18), ctx))
    t_intt, _ = timed(lambda: D.check(lib.mlh_intt(ctx, D.ptr(ev18), D.ptr(back), 18, g18), ctx))
    res["ntt_intt_2_18"] = {"ntt_ms": t_ntt, "intt_ms": t_intt,
                            "round_trip_equal": bool(torch.equal(back, c18)), "ref": "ntt/mod.rs:191-201"}
    # fri/mod.rs:365-398
    n20 = 1 << 20
    vals = dev_ints(np.arange(n20, dtype=np.uint32))
    t_gp, gp = timed(lambda: MN.pow_2_generator_powers(21, local))
    g1 = D.fe_from_bytes(gp[1].cpu().numpy().tobytes())
    t_rs, code = timed(lambda: MF.reed_solomon(vals, g1, local))
    t_pf, proof = timed(lambda: MF.FriProof.prove(code, Transcript(), local))
    t_vf, ok = timed(lambda: proof.verify())
    res["fri_2_20"] = {"gen_pows_ms": t_gp, "reed_solomon_ms": t_rs, "prove_ms": t_pf,
                       "verify_ms_host": t_vf, "verified": bool(ok),
                       "proof_bytes": len(proof.to_bytes()), "ref": "fri/mod.rs:365-398"}
    del gp, code, proof
    # multilinear_pcs.rs:210-228
    ev = dev_ints((7 * np.arange(n20, dtype=np.uint64) + 3).astype(np.uint32))
    inputs = list(range(20))
    output = MPL.evaluate(ev, inputs, local)
    t_pp, pcs = timed(lambda: PCSProof.prove(inputs, output, ev, Transcript(), local))
    t_pv, ok = timed(lambda: pcs.verify(Transcript()))
    res["pcs_20_vars"] = {"prove_ms": t_pp, "verify_ms_host": t_pv, "verified": bool(ok),
                          "ref": "multilinear_pcs.rs:210-228"}
    del pcs, ev
    # batched_pcs.rs:261-306
    m = 10
    j = np.arange(n20, dtype=np.uint64)
    evs = dev_ints(np.concatenate([((3 * j + 5 * i) % 100).astype(np.uint32) for i in range(m)]))
    outs = [MPL.evaluate(evs[i * n20:(i + 1) * n20], inputs, local) for i in range(m)]
    t_bp, bpf = timed(lambda: BatchedPCSProof.prove(inputs, outs, evs, Transcript(), local))
    t_bv, ok = timed(lambda: bpf.verify(Transcript()))
    res["batched_pcs_20_vars_x10"] = {"prove_ms": t_bp, "verify_ms_host": t_bv, "verified": bool(ok),
                                      "ref": "batched_pcs.rs:261-306"}
    return res


def config5(args, lib, ctx, local, world, rank, barrier):
    """Config 5: RS encode (2^(L-1) coeffs) + FRI prove of the 2^L codeword;
    single GPU at N = 1, sharded over the ranks at N > 1 (strong scaling)."""
    import torch

    from multilinear_amd import device as D
    from multilinear_amd import fri as MF
    from multilinear_amd.transcript import Transcript

    L = args.fri_log
    g = int.from_bytes(bytes(_gen(lib, L)), "little")
    reps = max(1, min(args.extra_reps, 3))
    if world == 1:
        coeffs = D.random_device(1 << (L - 1), 77, local)

        def run():
            code = MF.reed_solomon(coeffs, g, local)
            return MF.FriProof.prove(code, Transcript(), local)
    else:  # the C-ABI schedule (csrc/sharded.hip) over libmlhip's RCCL communicator
        from multilinear_amd import sharded as SH

        tr = _transport(local)
        coeffs = D.random_device(1 << (L - 1 - world.bit_length() + 1), 77 + rank, local)

        def run():
            code = SH.reed_solomon(coeffs, L - 1, g, tr, local)
            return SH.fri_prove(code, L, Transcript(), tr, device=local)

    p = run()  # warm-up (tables, allocator)
    barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        p = run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    if world > 1:
        dt = _allreduce_max(dt)
    out = {"config5_log_code": L, "config5_rs_fri_prove_ms": dt * 1e3,
           "config5_verified": bool(p.verify()),
           "config5_verified_is": "the host verifier (FriProof::verify) accepting the proof; "
                                  "self-consistency, not parity",
           "config5_layout": "single GPU" if world == 1 else
                             "sharded x%d (mlh_sharded_reed_solomon + mlh_sharded_fri_prove)" % world}
    if world > 1:
        # in-run parity: rank 0 gathers the 2^(L-1) coefficients, runs
        # reed_solomon + FriProof::prove on ONE GPU, and compares the proof's
        # wire bytes (every commitment, the 128 query records, last_elem,
        # last_random) with the sharded proof
        _test_corrupt(coeffs, rank)
        try:
            nat = _cyclic_to_natural(_gather_shards(coeffs, world), world)
            ok = True
            if rank == 0:
                code1 = MF.reed_solomon(nat, g, local)
                del nat
                ok = MF.FriProof.prove(code1, Transcript(), local).to_bytes() == p.to_bytes()
                del code1
            else:
                del nat
            out["config5_matches_single_gpu"] = _agree_ok(ok)
        except Exception as e:
            out["config5_matches_single_gpu"] = False
            out["config5_check_error"] = "%s: %s" % (type(e).__name__, e)
    return out


_TRANSPORT = []


def _transport(local):
    """The multi-GPU transport of the C-ABI schedules: libmlhip's own RCCL
    communicator (unique id broadcast over the torch.distributed group); in a
    gloo rehearsal, torch collectives as host callbacks."""
    if not _TRANSPORT:
        from multilinear_amd import sharded as SH

        if BACKEND == "nccl":
            _TRANSPORT.append(SH.RcclComm.from_torch(device=local))
        else:
            ht = SH.HostTransport(SH.Transport(host_staged=True), local)
            stall = os.environ.get("MLH_BENCH_TEST_STALL_A2A")
            if stall is not None and ht.tp.rank == int(stall):
                # test hook of the gloo rehearsal only (tests/test_bench_rehearsal_gpu.py):
                # this rank's all-to-all never returns, as a dead RCCL peer would
                from multilinear_amd import _lib

                def hang(user, send, recv, per, stream):
                    time.sleep(1e9)
                    return 1

                ht._hang = _lib.ALL_TO_ALL_FN(hang)
                ht.c.all_to_all = ht._hang
            _TRANSPORT.append(ht)
    return _TRANSPORT[0]


def _gen(lib, log_n):
    out = (ctypes.c_uint8 * 16)()
    lib.mlh_pow_2_generator(log_n, out)
    return out


if __name__ == "__main__":
    main()
