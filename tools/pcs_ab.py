"""PCS prove at 2^n (default 24), timed 6 times in one process (dev tool)."""
import random
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

from multilinear_amd import device as D  # noqa: E402
from multilinear_amd import multilinear_pcs as MP  # noqa: E402
from multilinear_amd import polynomials as MPL  # noqa: E402
from multilinear_amd.transcript import Transcript  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
rr = random.Random(5)
pts = [rr.randrange(D.M) for _ in range(n)]
x = D.random_device(1 << n, 9)
out = MPL.evaluate(x, pts)
for rep in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    MP.PCSProof.prove(pts, out, x, Transcript())
    torch.cuda.synchronize()
    print("pcs prove 2^%d: %.3f ms" % (n, (time.perf_counter() - t0) * 1e3), flush=True)
