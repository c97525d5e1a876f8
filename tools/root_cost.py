"""FRI commit with and without the host root readback (dev tool)."""
import ctypes, sys, time, os
sys.path.insert(0, os.getcwd())
import torch
from multilinear_amd import device as D
from oracle import field as F  # generator only
lib = D.lib(); ctx = D.context()
log_n = 24; N = 1 << log_n
x = D.random_device(N, 3); code = D.empty(2 * N)
layers = torch.empty((2 * N - 1) * 32, dtype=torch.uint8, device="cuda")
g2 = D.fe_bytes(F.pow_2_generator(log_n + 1))
root = (ctypes.c_uint8 * 32)()
def run(with_root, reps=10):
    for _ in range(2):
        D.check(lib.mlh_reed_solomon(ctx, D.ptr(x), log_n, g2, D.ptr(code)), ctx)
        D.check(lib.mlh_merkle_commit_pairs(ctx, D.ptr(code), log_n + 1, D.ptr(layers), root if with_root else None), ctx)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(reps):
        D.check(lib.mlh_reed_solomon(ctx, D.ptr(x), log_n, g2, D.ptr(code)), ctx)
        D.check(lib.mlh_merkle_commit_pairs(ctx, D.ptr(code), log_n + 1, D.ptr(layers), root if with_root else None), ctx)
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / reps * 1e3
for i in range(3):
    print("root %.3f ms  no-root %.3f ms" % (run(True), run(False)))
