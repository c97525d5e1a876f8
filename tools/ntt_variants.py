"""Time mlh_bench_ntt for several libmlhip builds, with per-pass kernel-timer
averages at 2^24 (dev tool)."""
import ctypes, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import _lib
from multilinear_amd import device as D

LABELS = ["ntt_pass<%d,%d,%d>" % (r, tw, z) for r in range(4, 10) for tw in range(4) for z in range(2)]

REF = [None]
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
    g = (ctypes.c_uint8 * 16)()
    lib.mlh_pow_2_generator(24, g)
    out = D.empty(1 << 24)
    assert lib.mlh_ntt(h, D.ptr(x), D.ptr(out), 24, g) == 0
    inv = D.empty(1 << 24)
    assert lib.mlh_intt(h, D.ptr(out), D.ptr(inv), 24, g) == 0
    torch.cuda.synchronize()
    if REF[0] is None:
        REF[0] = out.clone()
    res.append("same-as-first %s roundtrip %s" % (bool(torch.equal(out, REF[0])), bool(torch.equal(inv, x))))
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
    print(os.path.basename(path), " | ".join(res), " || ", "  ".join(per), flush=True)
    lib.mlh_context_destroy(h)
