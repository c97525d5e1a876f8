"""A/B the 2^24 NTT timing paths in one process (dev tool): mlh_bench_ntt
(in place) vs a Python loop of mlh_ntt (x -> out), profiler on/off."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import device as D
lib = D.lib(); ctx = D.context(0)
N = 1 << 24
x = D.random_device(N, 1); out = D.empty(N)
g = (ctypes.c_uint8 * 16)(); lib.mlh_pow_2_generator(24, g)
def loop(steps=20, prof=False):
    for _ in range(3): lib.mlh_ntt(ctx, D.ptr(x), D.ptr(out), 24, g)
    torch.cuda.synchronize()
    if prof: lib.mlh_profile_reset(ctx); lib.mlh_profile_enable(ctx, 1)
    t0 = time.perf_counter()
    for _ in range(steps): lib.mlh_ntt(ctx, D.ptr(x), D.ptr(out), 24, g)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps * 1e3
    lib.mlh_profile_enable(ctx, 0)
    return dt
for rep in range(2):
    ms = ctypes.c_float()
    lib.mlh_bench_ntt(ctx, D.ptr(x), 24, 20, ctypes.byref(ms))
    print("bench_ntt in-place %.4f ms | loop x->out %.4f ms | loop+prof %.4f ms" % (ms.value, loop(), loop(prof=True)), flush=True)
y = torch.empty_like(x)
def loop2(steps=20):
    for _ in range(3): lib.mlh_ntt(ctx, D.ptr(y), D.ptr(y), 24, g)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(steps): lib.mlh_ntt(ctx, D.ptr(y), D.ptr(y), 24, g)
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / steps * 1e3
y.copy_(x)
print("loop in-place torch buffer %.4f ms" % loop2())
z = D.random_device(N, 1)
print("fresh random in-place %.4f" % (lambda: (lib.mlh_bench_ntt(ctx, D.ptr(z), 24, 20, ctypes.byref(ms)), ms.value)[1])())
