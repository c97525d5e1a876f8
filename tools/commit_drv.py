"""Driver for counter passes over the FRI commit (config 3): RS 2^24 -> 2^25
and commit_rs_code / Merkle::commit, `reps` times (dev tool; no timing)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from multilinear_amd import device as D  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
log_n = 24
lib, ctx = D.lib(), D.context()
x = D.random_device(1 << log_n, 3)
code = D.empty(2 << log_n)
layers = torch.empty(((2 << log_n) - 1, 32), dtype=torch.uint8, device="cuda")
g2 = (ctypes.c_uint8 * 16)()
lib.mlh_pow_2_generator(log_n + 1, g2)
root = (ctypes.c_uint8 * 32)()
for _ in range(reps):
    D.check(lib.mlh_reed_solomon(ctx, D.ptr(x), log_n, g2, D.ptr(code)), ctx)
    D.check(lib.mlh_merkle_commit_pairs(ctx, D.ptr(code), log_n + 1, D.ptr(layers), root), ctx)
torch.cuda.synchronize()
print("root", bytes(root).hex())
