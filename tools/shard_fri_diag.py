"""Diagnostic (dev tool): mlh_sharded_reed_solomon + mlh_sharded_fri_prove on
P device-ordered thread ranks (tests/test_sharded_threads_gpu.py transport)
against the single-GPU proof of the same code, over a grid of (P, log_code).
  python tools/shard_fri_diag.py "P:log_code:gather_log,..." (e.g. "2:14:8,8:24:16")"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from multilinear_amd import device as DV  # noqa: E402
from multilinear_amd import fri as MF  # noqa: E402
from multilinear_amd import sharded as S  # noqa: E402
from multilinear_amd.fri import FriProof  # noqa: E402
from multilinear_amd.transcript import Transcript  # noqa: E402
from oracle import field as F  # noqa: E402  (generator only)
import test_sharded_threads_gpu as T  # noqa: E402

grid = [tuple(int(v) for v in x.split(":")) for x in sys.argv[1].split(",")]
L = DV.lib()
for P, log_code, gather_log in grid:
    t0 = time.time()
    coeffs = DV.random_limbs(1 << (log_code - 1), seed=77 + log_code)
    g = F.pow_2_generator(log_code)
    def reference():
        code1 = MF.reed_solomon(DV.to_device(coeffs), g)
        sp = MF.FriProof.prove(code1, Transcript())
        single = sp.to_bytes()
        sparts = (bytes(sp._commit), bytes(sp.c.last_elem), bytes(sp.c.last_random), bytes(sp._idx), bytes(sp._q),
                  sp.c.num_trees, sp.c.num_queries)
        want = DV.from_device(code1)
        from oracle import coracle as C  # noqa: E402  (checker)
        oroots, olast, _, orc = C.fri_commit_par(want, log_code)
        single_vs_oracle = (sp.commitments == oroots, sp.last_elem == olast, sp.verify())
        del code1
        torch.cuda.empty_cache()
        return sp, single, sparts, want, oroots, olast, single_vs_oracle

    AFTER = os.environ.get('DIAG_ORDER') == 'after'
    NOCOPY = os.environ.get('DIAG_NOCOPY') == '1'
    if not AFTER:
        sp, single, sparts, want, oroots, olast, single_vs_oracle = reference()
    stage = {}

    def body(r, ctx, st, t):
        c_loc = DV.to_device(S.shard_cyclic(coeffs, P, r))
        code = DV.empty(2 * c_loc.shape[0])
        torch.cuda.current_stream().synchronize()
        DV.check(L.mlh_sharded_reed_solomon(ctx, T._tp(t), DV.ptr(c_loc), log_code - 1, DV.fe_bytes(g),
                                            DV.ptr(code)), ctx)
        DV.check(L.mlh_synchronize(ctx), ctx)
        host = None if NOCOPY else DV.from_device(code)
        pf = FriProof(log_code)
        trx = Transcript()  # (kept alive across the call: the C side holds its pointer)
        st_ = L.mlh_sharded_fri_prove(ctx, T._tp(t), DV.ptr(code), log_code, gather_log, trx.h,
                                      ctypes.byref(pf.c))
        DV.check(L.mlh_synchronize(ctx), ctx)
        parts = (bytes(pf._commit), bytes(pf.c.last_elem), bytes(pf.c.last_random), bytes(pf._idx),
                 bytes(pf._q), pf.c.num_trees, pf.c.num_queries)
        if NOCOPY:
            host = DV.from_device(code)
        return host, st_, (pf.to_bytes() if st_ == 0 else b""), parts, (pf.verify() if st_ == 0 else None)

    try:
        res = T._run_ranks(P, body, T.ThreadDeviceTransport(P))
        if AFTER:
            sp, single, sparts, want, oroots, olast, single_vs_oracle = reference()
        p = P.bit_length() - 1
        got = S.unshard_blocks([res[r][0] for r in range(P)], log_code - 2 * p)
        rs_ok = bool(np.array_equal(got, want))
        sts = [res[r][1] for r in range(P)]
        same = [res[r][2] == single for r in range(P)]
        names = ("commitments", "last_elem", "last_random", "indices", "queries", "num_trees", "num_queries")
        diff = [n for i, n in enumerate(names) if res[0][3][i] != sparts[i]]
        qd = ""
        if "queries" in diff:
            qb = sp.qbytes
            a, b = res[0][3][4], sparts[4]
            bad = [q for q in range(128) if a[q * qb:(q + 1) * qb] != b[q * qb:(q + 1) * qb]]
            q = bad[0]
            off = next(i for i in range(qb) if a[q * qb + i] != b[q * qb + i])
            qd = " (%d query records differ, first q=%d at byte %d of %d)" % (len(bad), q, off, qb)
        print("   single vs oracle (roots, last, verify) %s; rank 0 roots vs oracle %s, verify %s" % (
            single_vs_oracle, res[0][3][0] == b"".join(oroots), res[0][4]), flush=True)
        print("P=%d log_code=%d gather_log=%d: RS %s, prove status %s, proof==single %s, differing %s%s (%.1f s)" % (
            P, log_code, gather_log, "ok" if rs_ok else "MISMATCH", sts, same, diff, qd, time.time() - t0), flush=True)
    except Exception as e:  # keep going through the grid
        print("P=%d log_code=%d gather_log=%d: EXC %s" % (P, log_code, gather_log, repr(e)[:600]), flush=True)
