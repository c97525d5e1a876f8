import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import coracle as C, field as F
from multilinear_amd import device as D, ntt as MN
ln, plan = 22, "6,8,8"
os.environ["MLH_NTT_PLAN"] = plan
g = F.pow_2_generator(ln)
x = D.random_limbs(1 << ln, 11)
want = C.ntt(x, ln, g)
dx = D.to_device(x)
def run(tag):
    got = D.from_device(MN.Polynomial(dx).ntt(g).evals)
    bad = np.nonzero((got != want).any(axis=1))[0]
    print(tag, "bad=%d" % bad.size, bad[:4].tolist(), flush=True)
    return got
a = run("run1")
b = run("run2")
print("run1==run2", bool((a == b).all()))
os.environ["MLH_DEBUG_SYNC"] = "1"
run("sync")
del os.environ["MLH_DEBUG_SYNC"]
torch.cuda.synchronize()
# default stream instead of torch's
import ctypes
from multilinear_amd import _lib
ctx = D.context()
out = D.empty(1 << ln)
D.lib().mlh_set_stream(ctx, None)
D.check(D.lib().mlh_ntt(ctx, D.ptr(dx), D.ptr(out), ln, D.fe_bytes(g)), ctx)
D.lib().mlh_synchronize(ctx)
got = D.from_device(out)
print("nullstream bad=%d" % np.count_nonzero((got != want).any(axis=1)))
# check input unchanged
print("input intact", bool((D.from_device(dx) == x).all()))
