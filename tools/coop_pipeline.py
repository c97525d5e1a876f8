"""Per-round timeline of the LAST cooperative sumcheck launch of a 2^LOG
mlh_sumcheck_prove_eq (the eq tail), as it runs inside the prove (dev tool).
Needs a libmlhip built with -DMLH_COOP_PROF (exports mlh_debug_coop_stamps):
  python tools/coop_pipeline.py tools/variants/libPROF.so"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from multilinear_amd import _lib
from multilinear_amd import device as D

LOG = int(os.environ.get("LOG", "24"))
lib = ctypes.CDLL(sys.argv[1])
for name, (res, args) in _lib.SIGNATURES.items():
    f = getattr(lib, name, None)
    if f is not None:
        f.restype, f.argtypes = res, args
x = D.random_device(1 << LOG, 5)
work = D.empty(1 << (LOG - 1))
pts = (ctypes.c_uint8 * (16 * LOG))(*([3] * 16 * LOG))
zero = (ctypes.c_uint8 * 16)()
h = ctypes.c_void_p()
assert lib.mlh_context_create(0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), ctypes.byref(h)) == 0
polys = (ctypes.c_uint8 * (32 * LOG))()
rs = (ctypes.c_uint8 * (16 * LOG))()
for rep in range(3):
    t = ctypes.c_void_p()
    lib.mlh_transcript_create(ctypes.byref(t))
    assert lib.mlh_sumcheck_prove_eq(h, D.ptr(x), D.ptr(work), LOG, pts, zero, t, polys, rs, None) == 0
    lib.mlh_transcript_destroy(t)
ts = (ctypes.c_uint64 * 640)()
ed = (ctypes.c_uint64 * 4)()
assert lib.mlh_debug_coop_stamps(ts, ed) == 0
T = [[ts[64 * e + k] for k in range(64)] for e in range(10)]
ghz = (ed[2] - ed[0]) / ((ed[3] - ed[1]) / 100e6) / 1e9
us = lambda c: c / (ghz * 1e3)
R = int(os.environ.get("R", "12"))
print("clock %.2f GHz; entry -> roles %.2f us; roles -> last r %.2f us" %
      (ghz, us(ed[2] - ed[0]), us(T[3][R - 1] - ed[2])))
print("prologue (wave 0, vs entry): loads+stores %.2f, first barrier %.2f, roles %.2f us" % (
    us(T[9][10] - ed[0]), us(T[9][11] - ed[0]), us(ed[2] - ed[0])))
print("round 0 helpers vs roles: corner ts6 %.2f ts7 %.2f; coef start %.2f got-ab %.2f slot %.2f" % (
    us(T[6][0] - ed[2]), us(T[7][0] - ed[2]), us(T[5][0] - ed[2]), us(T[8][0] - ed[2]), us(T[4][0] - ed[2])))
print("HW_ID per wave: %s (SIMD = bits 5:4, CU = bits 11:8)" % " ".join(
    "w%d:simd%d/cu%d" % (w, (T[9][20 + w] >> 4) & 3, (T[9][20 + w] >> 8) & 15) for w in range(4)))
print("round   wait  eval+absorb  challenge  slot_ready(vs r_{k-2})")
for k in range(R):
    lag = us(T[4][k] - T[3][k - 2]) if k >= 2 else 0.0
    print("%5d %6.2f %12.2f %10.2f %12.2f" % (k, us(T[1][k] - T[0][k]), us(T[2][k] - T[1][k]),
                                             us(T[3][k] - T[2][k]), lag))
print("msplit published %.2f us after r_2; corner wave round-6 work done %.2f us after r_4" %
      (us(T[9][0] - T[3][2]), us(T[6][6] - T[3][4])))
print("wave 3: rehearsal done %.2f us after roles; fold levels (got r_u, done) vs roles: %s" % (
    us(T[9][1] - ed[2]), " ".join("%.2f/%.2f" % (us(T[9][2 + 2 * u] - ed[2]), us(T[9][3 + 2 * u] - ed[2])) for u in range(3))))
print("r_k published vs roles: %s" % " ".join("%.2f" % us(T[3][k] - ed[2]) for k in range(R)))
print("corner wave: round  start->ts6(after transition/weights)  ts6->ts7(bucket+publish)")
for k in range(2, R):
    print("       %5d %8.2f %8.2f" % (k, us(T[6][k] - T[3][k - 2]), us(T[7][k] - T[6][k])))
print("helper: round  eval  ->ab  ->slot")
for k in range(1, R):
    print("       %5d %6.2f %6.2f %6.2f" % (k, us(T[8][k] - T[5][k]), 0.0, us(T[4][k] - T[8][k])))
print("quad_next: round  start->y-bcast  y-bcast->published")
for k in range(R):
    print("       %5d %8.2f %8.2f" % (k, us(T[9][33 + 2 * k] - T[9][32 + 2 * k]), us(T[4][k] - T[9][33 + 2 * k])))
