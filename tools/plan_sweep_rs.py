"""Time the 2^24 -> 2^25 RS LDE (config 3's LDE) under forced radix plans of the
2^25 transform (mlh_set_ntt_plan); outputs checked equal to the default's (dev tool)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multilinear_amd import device as D

LOG = 24
lib = D.lib()
ctx = D.context()
x = D.random_device(1 << LOG, 3)
code = D.empty(2 << LOG)
g = (ctypes.c_uint8 * 16)()
lib.mlh_pow_2_generator(LOG + 1, g)


def run():
    D.check(lib.mlh_reed_solomon(ctx, D.ptr(x), LOG, g, D.ptr(code)), ctx)


def timed(reps=20):
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
for plan in ["", "9,8,8", "8,9,8", "8,8,9", "9,9,7", "9,7,9", "7,9,9", "9,8,8", "6,6,6,7"]:
    digits = [int(v) for v in plan.split(",")] if plan else []
    arr = (ctypes.c_uint32 * max(1, len(digits)))(*digits)
    D.check(lib.mlh_set_ntt_plan(ctx, arr, len(digits)), ctx)
    ms = timed()
    chk = code.view(torch.int64)[::4096].sum().item()
    if ref is None:
        ref = chk
    print("plan %-9s %.3f ms  %s" % (plan or "default", ms, "ok" if chk == ref else "MISMATCH"),
          flush=True)
