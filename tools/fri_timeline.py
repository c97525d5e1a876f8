"""FRI prove on a 2^(log_n+1) codeword, timed; run under rocprofv3 --kernel-trace (dev tool)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import device as D, fri as MF
from multilinear_amd.transcript import Transcript
log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
x = D.random_device(1 << log_n, 3)
g = MF.reed_solomon  # warm
from oracle import field as F
code = MF.reed_solomon(x, F.pow_2_generator(log_n + 1))
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    p = MF.FriProof.prove(code, Transcript())
    torch.cuda.synchronize()
    print("fri prove %.3f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
