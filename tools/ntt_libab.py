"""A/B of the NTT / RS between libmlhip builds in one process (dev tool):
per build, the 2^24 forward NTT and the 2^24 -> 2^25 RS, alternated twice,
with per-pass averages from the library's HIP-event profiler.
usage: python tools/ntt_libab.py lib_a.so lib_b.so ..."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import _lib
from multilinear_amd import device as D

N = 1 << 24
x = D.random_device(N, 1)
out = D.empty(N)
code = D.empty(2 * N)


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


labels = ["ntt_pass<%d,%d,%d>" % (r, tw, z) for r in range(7, 10) for tw in (0, 1, 2, 3, 5) for z in range(3)]
for rep in range(2):
    for path in sys.argv[1:]:
        lib = load(path)
        h = ctypes.c_void_p()
        assert lib.mlh_context_create(0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
                                      ctypes.byref(h)) == 0
        g = (ctypes.c_uint8 * 16)()
        g2 = (ctypes.c_uint8 * 16)()
        lib.mlh_pow_2_generator(24, g)
        lib.mlh_pow_2_generator(25, g2)
        for _ in range(200):  # spin-up (clock)
            lib.mlh_ntt(h, D.ptr(x), D.ptr(out), 24, g)
        torch.cuda.synchronize()
        lib.mlh_profile_reset(h)
        lib.mlh_profile_enable(h, 1)
        t0 = time.perf_counter()
        for _ in range(100):
            lib.mlh_ntt(h, D.ptr(x), D.ptr(out), 24, g)
        torch.cuda.synchronize()
        ntt_ms = (time.perf_counter() - t0) / 100 * 1e3
        for _ in range(5):
            lib.mlh_reed_solomon(h, D.ptr(x), 24, g2, D.ptr(code))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            lib.mlh_reed_solomon(h, D.ptr(x), 24, g2, D.ptr(code))
        torch.cuda.synchronize()
        rs_ms = (time.perf_counter() - t0) / 20 * 1e3
        lib.mlh_profile_enable(h, 0)
        per = []
        for lab in labels:
            cnt, tot = ctypes.c_uint64(), ctypes.c_double()
            lib.mlh_profile_get(h, lab.encode(), ctypes.byref(cnt), ctypes.byref(tot))
            if cnt.value:
                per.append("%s %.4f" % (lab, tot.value / cnt.value))
        print("%-14s ntt %.4f ms  rs %.4f ms | %s" % (os.path.basename(path), ntt_ms, rs_ms,
              ", ".join(per)), flush=True)
        lib.mlh_context_destroy(h)
