"""FRI prove 2^25 on the host clock (dev tool): mlh_fri_prover_fold (commit
loop + replay) vs mlh_fri_prove (the same + the query phase), for each
library given: python tools/fri_phases.py a.so [b.so ...]"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import _lib
from multilinear_amd import device as D

LOG = 24
x = D.random_device(1 << LOG, 5)
code = D.empty(2 << LOG)


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


for path in sys.argv[1:]:
    lib = load(path)
    ctx = ctypes.c_void_p()
    assert lib.mlh_context_create(0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
                                  ctypes.byref(ctx)) == 0
    g = (ctypes.c_uint8 * 16)()
    lib.mlh_pow_2_generator(LOG + 1, g)
    assert lib.mlh_reed_solomon(ctx, D.ptr(x), LOG, g, D.ptr(code)) == 0
    qb = lib.mlh_fri_query_bytes(LOG + 1)
    com = (ctypes.c_uint8 * (32 * LOG))()
    idx = (ctypes.c_uint64 * 128)()
    q = (ctypes.c_uint8 * (128 * qb))()

    def fold():
        t = ctypes.c_void_p()
        lib.mlh_transcript_create(ctypes.byref(t))
        p = ctypes.c_void_p()
        assert lib.mlh_fri_prover_fold(ctx, D.ptr(code), LOG + 1, t, ctypes.byref(p)) == 0
        lib.mlh_fri_prover_destroy(p)
        lib.mlh_transcript_destroy(t)

    def prove():
        t = ctypes.c_void_p()
        lib.mlh_transcript_create(ctypes.byref(t))
        f = _lib.FriProofC()
        f.log_code, f.num_trees, f.num_queries = LOG + 1, LOG, 128
        f.commitments = ctypes.addressof(com)
        f.query_indices = ctypes.addressof(idx)
        f.queries = ctypes.addressof(q)
        assert lib.mlh_fri_prove(ctx, D.ptr(code), LOG + 1, t, ctypes.byref(f)) == 0
        lib.mlh_transcript_destroy(t)

    for rep in range(2):
        for name, fn in (("fold", fold), ("prove", prove)):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(10):
                t0 = time.perf_counter()
                fn()
                ts.append((time.perf_counter() - t0) * 1e3)
            ts.sort()
            print("%s %-6s median %.3f ms  min %.3f ms" % (os.path.basename(path), name, ts[5], ts[0]),
                  flush=True)
    lib.mlh_context_destroy(ctx)
