"""Time the 2^28 NTT (bench.py's strong-scaling transform) under forced radix
plans (mlh_set_ntt_plan); outputs checked equal to the default plan's (dev tool)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multilinear_amd import device as D

LOG = 28
lib = D.lib()
ctx = D.context()
x = D.random_device(1 << LOG, 3)
out = D.empty(1 << LOG)
g = (ctypes.c_uint8 * 16)()
lib.mlh_pow_2_generator(LOG, g)


def run():
    D.check(lib.mlh_ntt(ctx, D.ptr(x), D.ptr(out), LOG, g), ctx)


def timed(reps=5):
    run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        a.record()
        for _ in range(reps):
            run()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / reps)
    return best


ref = None
for plan in ["", "7,7,7,7", "8,8,6,6", "6,6,8,8", "9,9,5,5", "9,7,6,6", "8,7,7,6", "9,8,6,5",
             "5,5,9,9", "8,6,6,8"]:
    digits = [int(v) for v in plan.split(",")] if plan else []
    arr = (ctypes.c_uint32 * max(1, len(digits)))(*digits)
    D.check(lib.mlh_set_ntt_plan(ctx, arr, len(digits)), ctx)
    ms = timed()
    chk = out.view(torch.int64)[:: 4096].sum().item()
    if ref is None:
        ref = chk
    print("plan %-9s %.3f ms  %s" % (plan or "default", ms, "ok" if chk == ref else "MISMATCH"),
          flush=True)
