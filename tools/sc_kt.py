"""Kernel-trace driver (dev tool): 20 config-4 sumcheck proves (2^24,
mlh_sumcheck_prove_eq) and 5 PCS proves at n = 24, for
  rocprofv3 --kernel-trace --stats -- python3 tools/sc_kt.py"""
import ctypes
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from multilinear_amd import device as D  # noqa: E402
from multilinear_amd import polynomials as MPL  # noqa: E402
from multilinear_amd.multilinear_pcs import PCSProof  # noqa: E402
from multilinear_amd.polynomials import _points  # noqa: E402
from multilinear_amd.transcript import Transcript  # noqa: E402

LOG = 24
lib = D.lib()
ctx = D.context(0)
x = D.random_device(1 << LOG, 5)
work = D.empty(1 << (LOG - 1))
rr = random.Random(5)
pts = [rr.randrange(D.M) for _ in range(LOG)]
cp = _points(pts)
zero = (ctypes.c_uint8 * 16)()
polys = (ctypes.c_uint8 * (32 * LOG))()
rs = (ctypes.c_uint8 * (16 * LOG))()
dl = (ctypes.c_uint8 * 16)()
ts = []
for rep in range(25):
    tr = Transcript()
    t0 = time.perf_counter()
    D.check(lib.mlh_sumcheck_prove_eq(ctx, D.ptr(x), D.ptr(work), LOG, cp, zero, tr.h, polys, rs, dl), ctx)
    ts.append(time.perf_counter() - t0)
print("sumcheck_ms %.4f" % (sum(ts[5:]) / 20 * 1e3))
claim = MPL.evaluate(x, pts)
PCSProof.prove(pts, claim, x, Transcript())
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    p = PCSProof.prove(pts, claim, x, Transcript())
torch.cuda.synchronize()
print("pcs_prove_ms %.3f verified %s" % ((time.perf_counter() - t0) / 5 * 1e3, p.verify(Transcript())))
