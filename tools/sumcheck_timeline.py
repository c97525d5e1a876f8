"""eq table + 24-round sumcheck prove + PCS prove at 2^n, timed; run under
rocprofv3 --kernel-trace for per-kernel times (dev tool)."""
import os, random, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import device as D, polynomials as MPL, sumcheck as MS
from multilinear_amd import multilinear_pcs as MP
from multilinear_amd.transcript import Transcript
n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
rr = random.Random(5)
pts = [rr.randrange(D.M) for _ in range(n)]
x = D.random_device(1 << n, 9)
for rep in range(3):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    delta = MPL.eq_table(pts)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    m = x.clone(); torch.cuda.synchronize()
    t2 = time.perf_counter()
    MS.SumcheckTables(m, delta).compute_sumcheck_polynomials(0, Transcript())
    torch.cuda.synchronize(); t3 = time.perf_counter()
    print("eq %.3f ms  sumcheck %.3f ms" % ((t1 - t0) * 1e3, (t3 - t2) * 1e3), flush=True)
    time.sleep(0.01)
    tabs = MS.SumcheckTables.build_tables_for_pcs(pts, x)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    tabs.compute_sumcheck_polynomials(0, Transcript())
    torch.cuda.synchronize(); t1 = time.perf_counter()
    print("factored sumcheck %.3f ms" % ((t1 - t0) * 1e3), flush=True)
    time.sleep(0.01)
if len(sys.argv) > 2:
    out = MPL.evaluate(x, pts)
    for rep in range(2):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        MP.PCSProof.prove(pts, out, x, Transcript())
        torch.cuda.synchronize()
        print("pcs prove %.3f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
        time.sleep(0.01)
