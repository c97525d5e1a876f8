"""SumcheckTables for the PCS (src/constraint_system/sumcheck.rs:10-277),
composition x[0], width 1, on the MI355X (tables folded in place)."""
import ctypes

from .device import (check, context, empty, fe_bytes, fe_from_bytes, ints_to_limbs, lib, ptr,
                     to_device)
from .polynomials import _points, eq_table
from .transcript import Transcript


class SumcheckTables:
    def __init__(self, matrix, delta):
        self._matrix = matrix
        self._delta = delta
        self._evals = None   # build_tables_for_pcs: matrix = clone of these, not yet made
        self._points = None  # build_tables_for_pcs: delta = eq(points), not yet built
        self._delta_final = None  # after the factored rounds: the 1-entry delta (bytes)
        self._device = 0
        self.height = matrix.shape[0] if matrix is not None else 0

    @staticmethod
    def build_tables_for_pcs(inputs, evals, device=0):
        """sumcheck.rs:128-145 (matrix = evals clone, delta = eq table).  Both
        tables are built on first access; compute_sumcheck_polynomials on fresh
        tables builds neither (mlh_sumcheck_prove_eq keeps delta factored and
        its first fold reads the evaluations, which are never modified)."""
        assert 1 << len(inputs) == evals.shape[0]
        t = SumcheckTables(None, None)
        t._evals = evals
        t._points = list(inputs)
        t._device = device
        t.height = evals.shape[0]
        return t

    @property
    def matrix(self):
        if self._matrix is None:
            self._matrix = self._evals.clone()
        return self._matrix

    @property
    def delta(self):
        if self._delta is None:
            if self._delta_final is not None:  # uploaded on first access only
                self._delta = to_device(ints_to_limbs([fe_from_bytes(self._delta_final)]),
                                        self._device)
            else:
                self._delta = eq_table(self._points, self._device)
        return self._delta

    def _lh(self):
        return self.height.bit_length() - 1

    def partial_sums(self, device=0):
        """partial_sum at X = 1 and X = 2 (sumcheck.rs:204-232)."""
        ctx = context(device)
        out = (ctypes.c_uint8 * 32)()
        check(lib().mlh_sumcheck_partial_sums(ctx, ptr(self.matrix), ptr(self.delta), self._lh(),
                                              out), ctx)
        raw = bytes(out)
        return fe_from_bytes(raw[:16]), fe_from_bytes(raw[16:])

    def fold(self, r, device=0):
        """sumcheck.rs:234-247."""
        ctx = context(device)
        check(lib().mlh_sumcheck_fold(ctx, ptr(self.matrix), ptr(self.delta), self._lh(),
                                      fe_bytes(r)), ctx)
        self.height //= 2

    def compute_sumcheck_polynomials(self, total_sum, transcript: Transcript, device=0):
        """sumcheck.rs:77-102 -> ([(c1, c2)] per round, [r])."""
        ctx = context(device)
        n = self._lh()
        polys = (ctypes.c_uint8 * (32 * n))()
        rs = (ctypes.c_uint8 * (16 * n))()
        if self._delta is None and self._delta_final is None:  # delta = eq(points), unbuilt
            dl = (ctypes.c_uint8 * 16)()
            if self._matrix is None:  # read the evaluations, fold into a half-size table
                src, work = self._evals, empty(self.height // 2, device)
            else:
                src, work = self._matrix, None
            check(lib().mlh_sumcheck_prove_eq(ctx, ptr(src), ptr(work) if work is not None else None,
                                              n, _points(self._points), fe_bytes(total_sum),
                                              transcript.h, polys, rs, dl), ctx)
            if work is not None:
                self._matrix = work
            self._delta_final = bytes(dl)
            self._device = device
        else:
            check(lib().mlh_sumcheck_prove(ctx, ptr(self.matrix), ptr(self._delta), n,
                                           fe_bytes(total_sum), transcript.h, polys, rs), ctx)
        self.height = 1
        P, R = bytes(polys), bytes(rs)
        return ([(fe_from_bytes(P[32 * k:32 * k + 16]), fe_from_bytes(P[32 * k + 16:32 * k + 32]))
                 for k in range(n)],
                [fe_from_bytes(R[16 * k:16 * k + 16]) for k in range(n)])
