"""One-GPU experiment for the N = 8 projection: what the
sharded headline's exchange costs the local NTT when both run at once.

At P = 8 each rank of the sharded N*2^24 NTT step sends (P-1)/P of its 256 MiB
shard (235 MB) per step while the local compute of the neighbouring steps runs
(mlh_sharded_ntt_batch: local NTT and cross-shard DFT on the context stream,
the exchange alone on the side stream).  On one GPU the xGMI transfer itself cannot be
measured, but what it takes from the NTT can: the same 235 MB is moved on a
second stream, beside back-to-back 2^24 NTTs, by
  * copyk<W>   a CU copy kernel with W workgroups (RCCL's all-to-all runs on a
               few CUs per channel: W = 16, 32, 64);
  * blit       hipMemcpyAsync device-to-device (ROCm's blit kernel, all CUs);
  * sdma       hipMemcpyAsync with hipMemcpyDeviceToDeviceNoCU (copy engines,
               no compute units).
Per variant: the NTT step time and its passes (HIP events on the NTT stream,
mlh_profile), the copy time (HIP events on the side stream), each alone and
overlapped.  Output: one JSON object (stdout and --out).

Run on the GPU box:  python tools/a2a_contention.py --out gpurun_out/r05_a2a.json
(under rocprofv3 --kernel-trace --memory-copy-trace for the trace)."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

D2D, D2D_NOCU = 3, 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--world", type=int, default=8, help="P of the projected all-to-all")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--variants", default="copyk16,copyk32,copyk64,blit,sdma")
    ap.add_argument("--out", default=None)
    ap.add_argument("--with-cross", type=int, default=1,
                    help="1: main-stream step = local NTT + the P-point cross-shard DFT in turn; "
                         "2: the cross-shard DFT concurrently on a third stream (of another "
                         "buffer); 0: the NTT alone")
    ap.add_argument("--rounds", type=int, default=3, help="alternations of alone / variants")
    ap.add_argument("--warm-s", type=float, default=2.0, help="clock warm-up before measuring")
    args = ap.parse_args()

    import torch

    from multilinear_amd import device as D

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    ck = ctypes.CDLL(os.path.join(ROOT, "tools", "bin", "libcopyk.so"))
    ck.copyk_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                ctypes.c_void_p]

    N = 1 << args.log_n
    P = args.world
    nbytes = 16 * N * (P - 1) // P  # what one rank sends per step
    lib, ctx = D.lib(), D.context()
    sA = torch.cuda.current_stream()
    sB = torch.cuda.Stream()
    gen = (ctypes.c_uint8 * 16)()
    lib.mlh_pow_2_generator(args.log_n, gen)
    x = D.random_device(N, 7)
    out = D.empty(N)
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    src.fill_(1)

    lp = P.bit_length() - 1
    gen_tot = (ctypes.c_uint8 * 16)()
    lib.mlh_pow_2_generator(args.log_n + lp, gen_tot)
    crossed = D.empty(N)

    sC = torch.cuda.Stream()
    out2 = D.empty(N)

    def ntt():
        D.check(lib.mlh_ntt(ctx, D.ptr(x), D.ptr(out), args.log_n, gen), ctx)
        if args.with_cross == 1:  # main stream: local NTT + cross-shard DFT, in turn
            D.check(lib.mlh_shard_ntt_cross(ctx, D.ptr(out), D.ptr(crossed), args.log_n + lp, lp, 0, gen_tot, 0),
                    ctx)
        elif args.with_cross == 2:  # the cross-shard DFT on a stream of its own, concurrent
            lib.mlh_set_stream(ctx, ctypes.c_void_p(sC.cuda_stream))
            D.check(lib.mlh_shard_ntt_cross(ctx, D.ptr(out2), D.ptr(crossed), args.log_n + lp, lp, 0, gen_tot, 0),
                    ctx)
            lib.mlh_set_stream(ctx, ctypes.c_void_p(sA.cuda_stream))

    def copy(kind):
        st = ctypes.c_void_p(sB.cuda_stream)
        if kind.startswith("copyk"):
            rc = ck.copyk_launch(dst.data_ptr(), src.data_ptr(), nbytes, int(kind[5:]), st)
        else:
            rc = hip.hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), nbytes, D2D if kind == "blit" else D2D_NOCU,
                                    st)
        assert rc == 0, (kind, rc)

    def passes():
        res = {}
        for r in range(4, 10):
            for tw in range(4):
                lab = "ntt_pass<%d,%d,0>" % (r, tw)
                c, t = ctypes.c_uint64(), ctypes.c_double()
                lib.mlh_profile_get(ctx, lab.encode(), ctypes.byref(c), ctypes.byref(t))
                if c.value:
                    res[lab] = t.value / c.value
        for q in range(1, 5):
            lab = "shard_dft<%d,0>" % q
            c, t = ctypes.c_uint64(), ctypes.c_double()
            lib.mlh_profile_get(ctx, lab.encode(), ctypes.byref(c), ctypes.byref(t))
            if c.value:
                res[lab] = t.value / c.value
        return res

    def run(kind, with_ntt, with_copy):
        K = args.steps
        evA = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        evB = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        for _ in range(3):  # warm
            if with_ntt:
                ntt()
            if with_copy:
                copy(kind)
        torch.cuda.synchronize()
        lib.mlh_profile_reset(ctx)
        lib.mlh_profile_enable(ctx, 1)
        t0 = time.perf_counter()
        evA[0].record(sA)
        for i in range(K):
            if with_copy:
                evB[i][0].record(sB)
                copy(kind)
                evB[i][1].record(sB)
            if with_ntt:
                ntt()
        evA[1].record(sA)
        if args.with_cross == 2:
            sA.wait_stream(sC)
            evA[1].record(sA)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / K * 1e3
        lib.mlh_profile_enable(ctx, 0)
        rec = {"wall_ms_per_step": wall}
        if with_ntt:
            rec["ntt_ms_per_step"] = evA[0].elapsed_time(evA[1]) / K
            rec["ntt_passes_ms"] = passes()
        if with_copy:
            ms = sorted(a.elapsed_time(b) for a, b in evB)
            rec["copy_ms_median"] = ms[len(ms) // 2]
            rec["copy_GBps_median"] = nbytes / (rec["copy_ms_median"] * 1e-3) / 1e9
        return rec

    res = {"tool": "tools/a2a_contention.py", "log_n": args.log_n, "projected_world": P,
           "bytes_per_step": nbytes, "steps": args.steps, "rounds": args.rounds,
           "main_stream_step": {0: "local NTT 2^%d" % args.log_n,
                                1: "local NTT 2^%d + shard_dft<%d> in turn" % (args.log_n, lp),
                                2: "local NTT 2^%d || shard_dft<%d> on a third stream" % (args.log_n, lp)}
                               [args.with_cross],
           "device": torch.cuda.get_device_name(0), "variants": {}}
    t_end = time.perf_counter() + args.warm_s  # clock ramp: the first loops run slow
    while time.perf_counter() < t_end:
        for _ in range(20):
            ntt()
        torch.cuda.synchronize()
    kinds = args.variants.split(",")
    alone, per = [], {k: {"copy_alone": [], "overlapped": []} for k in kinds}
    for _ in range(args.rounds):  # alternate so clock drift spreads over every variant
        alone.append(run(None, True, False))
        for kind in kinds:
            per[kind]["copy_alone"].append(run(kind, False, True))
            per[kind]["overlapped"].append(run(kind, True, True))
    alone.append(run(None, True, False))

    def med(rows, key):
        v = sorted(r[key] for r in rows)
        return v[len(v) // 2]

    base = med(alone, "ntt_ms_per_step")
    res["main_alone"] = {"ms_per_step_median": base, "runs": [r["ntt_ms_per_step"] for r in alone],
                         "passes_last": alone[-1]["ntt_passes_ms"]}
    for kind in kinds:
        ca, ov = per[kind]["copy_alone"], per[kind]["overlapped"]
        res["variants"][kind] = {
            "copy_alone_ms": med(ca, "copy_ms_median"), "copy_alone_GBps": med(ca, "copy_GBps_median"),
            "overlapped_main_ms": med(ov, "ntt_ms_per_step"), "overlapped_copy_ms": med(ov, "copy_ms_median"),
            "overlapped_wall_ms": med(ov, "wall_ms_per_step"),
            "main_slowdown": med(ov, "ntt_ms_per_step") / base,
            "passes_overlapped_last": ov[-1]["ntt_passes_ms"],
        }
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
