"""Diagnostic: NTT radix plans vs the C oracle at several sizes (debug tool)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import coracle as C, field as F
from multilinear_amd import device as D, ntt as MN

cases = [(18, "8,5,5"), (18, "5,5,8"), (18, "5,8,5"), (19, "8,6,5"), (20, "8,6,6"), (20, "6,6,8"),
         (20, "6,8,6"), (21, "8,8,5"), (22, "8,7,7"), (22, "7,8,7"), (22, "7,7,8"), (22, "4,9,9"),
         (22, "9,9,4"), (22, "6,8,8"), (21, "7,7,7"), (22, "8,8,6"), (20, "9,6,5"), (20, "5,6,9")]
refs = {}
for ln, plan in cases:
    os.environ["MLH_NTT_PLAN"] = plan
    g = F.pow_2_generator(ln)
    if ln not in refs:
        x = D.random_limbs(1 << ln, 7 + ln)
        refs[ln] = (x, C.ntt(x, ln, g))
    x, want = refs[ln]
    got = D.from_device(MN.Polynomial(D.to_device(x)).ntt(g).evals)
    bad = np.nonzero((got != want).any(axis=1))[0]
    info = ""
    if bad.size:
        r = [int(v) for v in plan.split(",")]
        K = bad
        k1 = K % (1 << r[0]); rest = K >> r[0]
        info = "first=%s k1set=%d distinct_k1=%s" % (bad[:4].tolist(), len(set(k1.tolist())), sorted(set(k1.tolist()))[:10])
    print("log_n=%d plan=%s bad=%d %s" % (ln, plan, bad.size, info), flush=True)
