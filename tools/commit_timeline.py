"""FRI commit (config 3: RS of 2^n coeffs + commit_rs_code Merkle root), timed
5 times; run under rocprofv3 --kernel-trace for per-kernel times (dev tool)."""
import ctypes
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

from multilinear_amd import device as D  # noqa: E402
from multilinear_amd import ntt as MN  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
lib, ctx = D.lib(), D.context(0)
x = D.random_device(1 << n, 1)
code = D.empty(2 << n, 0)
layers = torch.empty(((2 << n) - 1, 32), dtype=torch.uint8, device="cuda:0")
g2 = D.fe_bytes(MN.pow_2_generator(n + 1))
root = (ctypes.c_uint8 * 32)()
for rep in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    D.check(lib.mlh_reed_solomon(ctx, D.ptr(x), n, g2, D.ptr(code)), ctx)
    D.check(lib.mlh_merkle_commit_pairs(ctx, D.ptr(code), n + 1, D.ptr(layers), root), ctx)
    print("fri commit 2^%d: %.3f ms" % (n, (time.perf_counter() - t0) * 1e3), flush=True)
    time.sleep(0.005)
