"""A/B timing of mlh_sumcheck_prove_eq at 2^24 (evaluations -> half-size work
table) for several libmlhip builds in one process (dev tool)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import _lib
from multilinear_amd import device as D

LOG = int(os.environ.get("LOG", "24"))
x = D.random_device(1 << LOG, 5)
work = D.empty(1 << (LOG - 1))
pts = (ctypes.c_uint8 * (16 * LOG))(*([3] * 16 * LOG))
zero = (ctypes.c_uint8 * 16)()


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
        assert lib.mlh_context_create(0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
                                      ctypes.byref(h)) == 0
        polys = (ctypes.c_uint8 * (32 * LOG))()
        rs = (ctypes.c_uint8 * (16 * LOG))()

        def run():
            t = ctypes.c_void_p()
            lib.mlh_transcript_create(ctypes.byref(t))
            assert lib.mlh_sumcheck_prove_eq(h, D.ptr(x), D.ptr(work), LOG, pts, zero, t, polys, rs,
                                             None) == 0
            lib.mlh_transcript_destroy(t)

        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        print("%-12s sumcheck_eq %.3f ms  polys[0..8] %s" % (os.path.basename(path),
              (time.perf_counter() - t0) / 10 * 1e3, bytes(polys)[:8].hex()), flush=True)
        lib.mlh_context_destroy(h)
