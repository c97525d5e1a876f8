"""Time the 2^24 NTT and the 2^24 -> 2^25 RS LDE under forced radix plans
(mlh_set_ntt_plan, the radix-plan test hook) -- dev tool for choosing the
default plan.  Outputs are checked equal to the default plan's."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multilinear_amd import device as D


def gen(lib, log_n):
    g = (ctypes.c_uint8 * 16)()
    lib.mlh_pow_2_generator(log_n, g)
    return g


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / reps)
    return best


def main():
    lib = D.lib()
    ctx = D.context()
    x = D.random_device(1 << 24, 3)
    out = D.empty(1 << 24)
    code = D.empty(1 << 25)
    g24, g25 = gen(lib, 24), gen(lib, 25)
    cases = [("ntt", 24, ["", "8,8,8", "9,8,7", "7,8,9", "8,9,7", "9,9,6", "6,9,9"]),
             ("rs", 25, ["", "9,8,8", "8,9,8", "8,8,9", "9,9,7", "7,9,9"])]
    for kind, ln, plans in cases:
        ref = None
        for plan in plans:
            digits = [int(v) for v in plan.split(",")] if plan else []
            arr = (ctypes.c_uint32 * max(1, len(digits)))(*digits)
            D.check(lib.mlh_set_ntt_plan(ctx, arr, len(digits)), ctx)
            if kind == "ntt":
                fn = lambda: D.check(lib.mlh_ntt(ctx, D.ptr(x), D.ptr(out), 24, g24), ctx)
                res = out
            else:
                fn = lambda: D.check(lib.mlh_reed_solomon(ctx, D.ptr(x), 24, g25, D.ptr(code)), ctx)
                res = code
            ms = timed(fn)
            if ref is None:
                ref = res.clone()
            print("%-3s 2^%d plan %-7s %.4f ms  same %s" % (kind, ln, plan or "default", ms,
                                                         bool(torch.equal(res, ref))), flush=True)
        D.check(lib.mlh_set_ntt_plan(ctx, None, 0), ctx)


if __name__ == "__main__":
    main()
