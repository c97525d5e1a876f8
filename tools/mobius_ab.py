"""A/B of mlh_mle_to_coefficient / mlh_mle_to_evaluation (2^24, Moebius / zeta
passes) between libmlhip builds in one process (dev tool):
python tools/mobius_ab.py a.so b.so ..."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import _lib
from multilinear_amd import device as D

LOG = 24
x0 = D.random_device(1 << LOG, 11)


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


for rep in range(2):
    for path in sys.argv[1:]:
        lib = load(path)
        h = ctypes.c_void_p()
        assert lib.mlh_context_create(0, None, ctypes.byref(h)) == 0
        x = x0.clone()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(2):
            lib.mlh_mle_to_coefficient(h, D.ptr(x), LOG)
            lib.mlh_mle_to_evaluation(h, D.ptr(x), LOG)
        torch.cuda.synchronize()
        a.record()
        for _ in range(10):
            lib.mlh_mle_to_coefficient(h, D.ptr(x), LOG)
            lib.mlh_mle_to_evaluation(h, D.ptr(x), LOG)
        b.record()
        torch.cuda.synchronize()
        ok = bool((x == x0).all())
        print("%-14s mobius+zeta %.3f ms  roundtrip %s" % (os.path.basename(path),
              a.elapsed_time(b) / 10, "ok" if ok else "MISMATCH"), flush=True)
        lib.mlh_context_destroy(h)
