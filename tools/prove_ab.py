"""A/B timing of mlh_fri_prove and mlh_pcs_prove (2^24) for several libmlhip
builds in one process (dev tool): python tools/prove_ab.py a.so b.so ..."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import _lib
from multilinear_amd import device as D

LOG = 24
x = D.random_device(1 << LOG, 5)
code = D.empty(2 << LOG)
pts = (ctypes.c_uint8 * (16 * LOG))(*([7] * 16 * LOG))


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


for rep in range(int(os.environ.get("AB_REPS", "3"))):
    for path in sys.argv[1:]:
        lib = load(path)
        h = ctypes.c_void_p()
        assert lib.mlh_context_create(0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
                                      ctypes.byref(h)) == 0
        g = (ctypes.c_uint8 * 16)()
        lib.mlh_pow_2_generator(LOG + 1, g)
        assert lib.mlh_reed_solomon(h, D.ptr(x), LOG, g, D.ptr(code)) == 0
        qb = lib.mlh_fri_query_bytes(LOG + 1)
        com = (ctypes.c_uint8 * (32 * LOG))()
        idx = (ctypes.c_uint64 * 128)()
        q = (ctypes.c_uint8 * (128 * qb))()
        polys = (ctypes.c_uint8 * (32 * LOG))()
        out = (ctypes.c_uint8 * 16)()

        def fri_struct():
            f = _lib.FriProofC()
            f.log_code, f.num_trees, f.num_queries = LOG + 1, LOG, 128
            f.commitments = ctypes.addressof(com)
            f.query_indices = ctypes.addressof(idx)
            f.queries = ctypes.addressof(q)
            return f

        def fri():
            t = ctypes.c_void_p()
            lib.mlh_transcript_create(ctypes.byref(t))
            p = fri_struct()
            assert lib.mlh_fri_prove(h, D.ptr(code), LOG + 1, t, ctypes.byref(p)) == 0
            lib.mlh_transcript_destroy(t)

        def pcs():
            t = ctypes.c_void_p()
            lib.mlh_transcript_create(ctypes.byref(t))
            p = _lib.PcsProofC()
            p.fri = fri_struct()
            p.sumcheck_polys = ctypes.addressof(polys)
            assert lib.mlh_pcs_prove(h, D.ptr(x), LOG, pts, out, t, ctypes.byref(p)) == 0
            lib.mlh_transcript_destroy(t)

        res = []
        for fn in (fri, pcs):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            res.append((time.perf_counter() - t0) / 5 * 1e3)
        print("%-10s fri_prove %.3f ms  pcs_prove %.3f ms" % (os.path.basename(path), *res), flush=True)
        lib.mlh_context_destroy(h)
