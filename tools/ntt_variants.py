"""Time mlh_bench_ntt for several libmlhip builds, with per-pass kernel-timer
averages at 2^24 (dev tool)."""
import ctypes, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import _lib
from multilinear_amd import device as D

LABELS = ["ntt_pass<%d,%d,%d>" % (r, tw, z) for r in range(4, 10) for tw in range(3) for z in range(2)]

for path in sys.argv[1:]:
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name, None)
        if f is None: continue
        f.restype = res; f.argtypes = args
    h = ctypes.c_void_p()
    assert lib.mlh_context_create(0, None, ctypes.byref(h)) == 0
    x = D.random_device(1 << 24, 1)
    res = []
    for ln in (20, 22, 24):
        ms = ctypes.c_float()
        assert lib.mlh_bench_ntt(h, D.ptr(x), ln, 20, ctypes.byref(ms)) == 0
        res.append("2^%d %.3f ms" % (ln, ms.value))
    lib.mlh_profile_reset(h); lib.mlh_profile_enable(h, 1)
    ms = ctypes.c_float()
    lib.mlh_bench_ntt(h, D.ptr(x), 24, 20, ctypes.byref(ms))
    lib.mlh_profile_enable(h, 0)
    per = []
    for lab in LABELS:
        c, t = ctypes.c_uint64(), ctypes.c_double()
        lib.mlh_profile_get(h, lab.encode(), ctypes.byref(c), ctypes.byref(t))
        if c.value:
            per.append("%s %.4f" % (lab, t.value / c.value))
    print(path.split("/")[-2], " | ".join(res), " || ", "  ".join(per), flush=True)
    lib.mlh_context_destroy(h)
