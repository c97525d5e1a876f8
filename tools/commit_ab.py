"""FRI commit (config 3) split per libmlhip build, alternating builds on one box:
RS LDE alone, Merkle commit alone, RS + Merkle back to back, and the 2^24 NTT
(dev tool: python tools/commit_ab.py libA.so libB.so libA.so ...)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multilinear_amd import _lib
from multilinear_amd import device as D


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name, None)
        if f is None:
            continue
        f.restype = res
        f.argtypes = args
    return lib


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    x = D.random_device(1 << 24, 7)
    code = D.empty(1 << 25)
    out = D.empty(1 << 24)
    layers = torch.empty(((1 << 25) - 1, 32), dtype=torch.uint8, device="cuda")
    for path in sys.argv[1:]:
        lib = load(path)
        h = ctypes.c_void_p()
        assert lib.mlh_context_create(0, None, ctypes.byref(h)) == 0
        g24, g25 = (ctypes.c_uint8 * 16)(), (ctypes.c_uint8 * 16)()
        lib.mlh_pow_2_generator(24, g24)
        lib.mlh_pow_2_generator(25, g25)
        root = (ctypes.c_uint8 * 32)()
        rs = lambda: lib.mlh_reed_solomon(h, D.ptr(x), 24, g25, D.ptr(code))
        mk = lambda: lib.mlh_merkle_commit_pairs(h, D.ptr(code), 25, D.ptr(layers), root)
        both = lambda: (rs(), mk())
        ntt = lambda: lib.mlh_ntt(h, D.ptr(x), D.ptr(out), 24, g24)
        r = [timed(ntt, 50), timed(rs, 10), timed(mk, 10), timed(both, 10)]
        print("%-12s ntt %.3f  rs %.3f  merkle %.3f  rs+merkle %.3f ms  root %s" % (
            os.path.basename(path), *r, bytes(root)[:6].hex()), flush=True)
        lib.mlh_context_destroy(h)


if __name__ == "__main__":
    main()
