"""Diagnostic: device pow tables (tlo*thi) vs the C oracle's serial powers."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes
import numpy as np
from oracle import coracle as C, field as F
from multilinear_amd import device as D, ntt as MN

for ls in (12, 13, 16, 18, 19, 20, 21, 22):
    want = np.empty((1 << ls, 4), dtype=np.uint32)
    C.lib().orc_pow_2_generator_powers(ls, want.ctypes.data_as(ctypes.c_void_p))
    got = D.from_device(MN.pow_2_generator_powers(ls))
    bad = np.nonzero((got != want).any(axis=1))[0]
    print("ls=%d bad=%d first=%s" % (ls, bad.size, bad[:6].tolist()), flush=True)
    if bad.size:
        i = int(bad[0])
        print("  t=%d got=%x want=%x" % (i, D.limbs_to_ints(got[i:i+1])[0], D.limbs_to_ints(want[i:i+1])[0]))
        hi = sorted(set((bad >> 12).tolist()))
        print("  bad hi indices: n=%d first=%s" % (len(hi), hi[:10]))
        lo = sorted(set((bad & 4095).tolist()))
        print("  bad lo indices: n=%d first=%s" % (len(lo), lo[:10]))
