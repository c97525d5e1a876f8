"""SumcheckTables for the PCS (src/constraint_system/sumcheck.rs:10-277),
composition x[0], width 1, on the MI355X (tables folded in place)."""
import ctypes

from .device import check, context, fe_bytes, fe_from_bytes, lib, ptr
from .polynomials import eq_table
from .transcript import Transcript


class SumcheckTables:
    def __init__(self, matrix, delta):
        self.matrix = matrix
        self.delta = delta
        self.height = matrix.shape[0]

    @staticmethod
    def build_tables_for_pcs(inputs, evals, device=0):
        """sumcheck.rs:128-145 (matrix = evals clone, delta = eq table)."""
        assert 1 << len(inputs) == evals.shape[0]
        return SumcheckTables(evals.clone(), eq_table(inputs, device))

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
        check(lib().mlh_sumcheck_prove(ctx, ptr(self.matrix), ptr(self.delta), n,
                                       fe_bytes(total_sum), transcript.h, polys, rs), ctx)
        self.height = 1
        P, R = bytes(polys), bytes(rs)
        return ([(fe_from_bytes(P[32 * k:32 * k + 16]), fe_from_bytes(P[32 * k + 16:32 * k + 32]))
                 for k in range(n)],
                [fe_from_bytes(R[16 * k:16 * k + 16]) for k in range(n)])
