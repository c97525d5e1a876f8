"""Time mlh_bench_ntt for several libmlhip builds (dev tool)."""
import ctypes, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import _lib
from multilinear_amd import device as D
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
    print(os.path.basename(path), " | ".join(res), flush=True)
    lib.mlh_context_destroy(h)
