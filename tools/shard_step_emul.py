"""One rank's view of the sharded N-GPU NTT step on one MI355X (N = 8 by
default): the real mlh_sharded_ntt_batch / mlh_sharded_ntt_fused_batch
schedules (their kernels, streams and events) run for rank 0 of an 8-rank
world whose all-to-all is emulated by a device copy of the same size on the
stream the library passes -- (P - 1)/P of the 256 MiB shard plus the local
chunk -- through a CU copy kernel of W workgroups (W = 32 and 64 move
~290 / ~540 GB/s alone, the range of an xGMI all-to-all: tools/a2a_contention.py)
or the blit kernel (~2.6 TB/s: no exchange cost).  The data is not a real
transform (the peers do not exist); the kernels' cost does not depend on it.
Output: ms per step of each schedule with each exchange, and the per-phase
HIP-event times.

Run on the GPU box:  python tools/shard_step_emul.py [--out file]"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-local", type=int, default=24)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--exchanges", default="copyk32,copyk64,blit")
    ap.add_argument("--out", default=None)
    ap.add_argument("--lib", default=None, help="a libmlhip build to load instead of the in-tree one")
    args = ap.parse_args()

    import torch

    from multilinear_amd import _lib
    from multilinear_amd import device as D

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    ck = ctypes.CDLL(os.path.join(ROOT, "tools", "bin", "libcopyk.so"))
    ck.copyk_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                ctypes.c_void_p]
    P, lp = args.world, args.world.bit_length() - 1
    L = args.log_local + lp
    M = 1 << args.log_local
    if args.lib:
        lib = ctypes.CDLL(args.lib)
        for name, (rt, at) in _lib.SIGNATURES.items():
            f = getattr(lib, name, None)
            if f is not None:
                f.restype, f.argtypes = rt, at
        h = ctypes.c_void_p()
        assert lib.mlh_context_create(0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
                                      ctypes.byref(h)) == 0
        ctx = h.value
    else:
        lib, ctx = D.lib(), D.context()

    class _C:  # status check against this library's context
        @staticmethod
        def check(st, c=None):
            if st != 0:
                raise RuntimeError("status %d: %s" % (st, lib.mlh_last_error(ctx)))
    D = type("D", (), {"check": _C.check, "ptr": staticmethod(D.ptr), "random_device": staticmethod(D.random_device),
                       "empty": staticmethod(D.empty)})
    mode = {"kind": "blit"}

    def a2a(user, send, recv, per, stream):
        n = per * P
        if mode["kind"].startswith("copyk"):
            return ck.copyk_launch(recv, send, n, int(mode["kind"][5:]), stream)
        return hip.hipMemcpyAsync(recv, send, n, 3, stream)

    def ag(user, send, recv, nbytes, stream):
        return hip.hipMemcpyAsync(recv, send, nbytes, 3, stream)

    fa2a, fag = _lib.ALL_TO_ALL_FN(a2a), _lib.ALL_GATHER_FN(ag)
    tp = _lib.TransportC(P, 0, 0, None, fa2a, fag)
    gen = (ctypes.c_uint8 * 16)()
    lib.mlh_pow_2_generator(L, gen)
    x = D.random_device(M, 5)
    outs = [D.empty(M), D.empty(M)]

    def arrays(k):
        return ((ctypes.c_void_p * k)(*([x.data_ptr()] * k)),
                (ctypes.c_void_p * k)(*[outs[i & 1].data_ptr() for i in range(k)]))

    arr = arrays(args.steps)
    warm = arrays(8)

    def run(sched, k_arr):
        ins, os_ = k_arr
        k = len(ins)
        if sched == "fused":
            st = lib.mlh_sharded_ntt_fused_batch(ctx, ctypes.byref(tp), ins, os_, k, L, gen, None)
        else:
            st = lib.mlh_sharded_ntt_batch(ctx, ctypes.byref(tp), ins, os_, k, L, gen, 0)
        D.check(st, ctx)

    labels = ["ntt_pass<%d,%d,0>" % (r, t) for r in range(4, 10) for t in range(4)] + [
        "shard_dft<%d,0>" % lp, "ntt_all_to_all", "ntt_fused_pre", "ntt_fused_last"]

    def measure(sched, kind):
        mode["kind"] = kind
        run(sched, warm)
        torch.cuda.synchronize()
        lib.mlh_profile_reset(ctx)
        lib.mlh_profile_enable(ctx, 4)
        t0 = time.perf_counter()
        run(sched, arr)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        lib.mlh_profile_enable(ctx, 0)
        ph = {}
        for lab in labels:
            c, t = ctypes.c_uint64(), ctypes.c_double()
            lib.mlh_profile_get(ctx, lab.encode(), ctypes.byref(c), ctypes.byref(t))
            if c.value:
                ph[lab] = t.value / c.value
        return ms, ph

    t_end = time.perf_counter() + 2.0  # clock warm-up
    while time.perf_counter() < t_end:
        for _ in range(20):
            D.check(lib.mlh_ntt(ctx, D.ptr(x), D.ptr(outs[0]), args.log_local, gen), ctx)
        torch.cuda.synchronize()
    g1 = (ctypes.c_uint8 * 16)()
    lib.mlh_pow_2_generator(args.log_local, g1)
    res = {"tool": "tools/shard_step_emul.py", "lib": args.lib or "multilinear_amd/libmlhip.so", "world": P, "log_local": args.log_local,
           "exchange_bytes_per_rank": 16 * M, "rounds": args.rounds, "steps": args.steps, "runs": {}}
    single = []
    for _ in range(args.rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            D.check(lib.mlh_ntt(ctx, D.ptr(x), D.ptr(outs[0]), args.log_local, g1), ctx)
        torch.cuda.synchronize()
        single.append((time.perf_counter() - t0) / args.steps * 1e3)
        for sched in ("batch", "fused"):
            for kind in args.exchanges.split(","):
                ms, ph = measure(sched, kind)
                res["runs"].setdefault("%s/%s" % (sched, kind), []).append({"ms_per_step": ms, "phases": ph})
    single.sort()
    res["single_gpu_ntt_ms"] = single[len(single) // 2]
    summary = {}
    for key, runs in res["runs"].items():
        v = sorted(r["ms_per_step"] for r in runs)
        med = v[len(v) // 2]
        summary[key] = {"ms_per_step": med,
                        "projected_speedup_at_%d" % P: P * res["single_gpu_ntt_ms"] / med}
    res["summary"] = summary
    print(json.dumps({"single_gpu_ntt_ms": res["single_gpu_ntt_ms"], "summary": summary}), flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
