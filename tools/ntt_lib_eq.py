"""Output equality of the NTT paths between two libmlhip builds (dev tool):
forward / inverse 2^23 and 2^24, RS and bit-reversed RS into 2^24, byte-equal.
usage: python tools/ntt_lib_eq.py lib_a.so lib_b.so"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import _lib
from multilinear_amd import device as D


def load(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


outs = []
for path in sys.argv[1:3]:
    lib = load(path)
    h = ctypes.c_void_p()
    assert lib.mlh_context_create(0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), ctypes.byref(h)) == 0
    res = []
    for log in (23, 24):
        x = D.random_device(1 << log, 77 + log)
        y = D.empty(1 << log)
        g = (ctypes.c_uint8 * 16)()
        lib.mlh_pow_2_generator(log, g)
        assert lib.mlh_ntt(h, D.ptr(x), D.ptr(y), log, g) == 0
        res.append(y.clone())
        assert lib.mlh_intt(h, D.ptr(x), D.ptr(y), log, g) == 0
        res.append(y.clone())
        assert lib.mlh_reed_solomon(h, D.ptr(x), log - 1, g, D.ptr(y)) == 0
        res.append(y.clone())
        assert lib.mlh_reed_solomon_brev(h, D.ptr(x), log - 1, g, D.ptr(y)) == 0
        res.append(y.clone())
    torch.cuda.synchronize()
    outs.append(res)
    lib.mlh_context_destroy(h)
ok = all(torch.equal(a, b) for a, b in zip(*outs))
print("outputs equal:", ok, len(outs[0]), "arrays")
sys.exit(0 if ok else 1)
