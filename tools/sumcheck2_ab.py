"""A/B timing of the two-table mlh_sumcheck_prove at 2^24 (fresh copies of
the random matrix and delta tables per prove, outside the timed region) for
several libmlhip builds in one process (dev tool):
python tools/sumcheck2_ab.py a.so b.so ..."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import _lib
from multilinear_amd import device as D

LOG = int(os.environ.get("LOG", "24"))
m0 = D.random_device(1 << LOG, 11)
d0 = D.random_device(1 << LOG, 12)
m, d = torch.empty_like(m0), torch.empty_like(d0)
claim = (ctypes.c_uint8 * 16)(*([5] * 8 + [0] * 8))


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


for rep in range(3):
    for path in sys.argv[1:]:
        lib = load(path)
        h = ctypes.c_void_p()
        assert lib.mlh_context_create(0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
                                      ctypes.byref(h)) == 0
        polys = (ctypes.c_uint8 * (32 * LOG))()
        ts = []
        for it in range(6):
            m.copy_(m0)
            d.copy_(d0)
            t = ctypes.c_void_p()
            lib.mlh_transcript_create(ctypes.byref(t))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st = lib.mlh_sumcheck_prove(h, D.ptr(m), D.ptr(d), LOG, ctypes.cast(claim, ctypes.c_void_p), t,
                                        ctypes.cast(polys, ctypes.c_void_p), None)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
            assert st == 0, st
            lib.mlh_transcript_destroy(t)
        ts.sort()
        print("%-18s sumcheck_two_table %.3f ms (median of 5 after 1)  polys[0..8] %s" % (
            os.path.basename(path), ts[len(ts) // 2], bytes(polys[:8]).hex()), flush=True)
        lib.mlh_context_destroy(h)
