"""Sumcheck tables for the PCS (oracle).  Test infrastructure only.

Reference: src/constraint_system/sumcheck.rs:128-277 and
src/constraint_system/evaluation.rs:51-91.  The fold variable is the MSB of
the table index (pairs i, i + height/2).
"""
from . import field as F
from .polynomials import interpolate, uni_evaluate


def mask_evaluate(index, n_vars, points):
    """Mask::evaluate (evaluation.rs:51-73): prod_i (bit_i ? p[n-1-i] : 1-p[n-1-i])."""
    acc = 1
    for i in range(n_vars):
        p = points[n_vars - 1 - i]
        acc = acc * (p if (index >> i) & 1 else (1 - p)) % F.M
    return acc


def eq_table(points):
    """delta table of build_tables_for_pcs (sumcheck.rs:133-138), by the
    doubling expansion (same values as mask_evaluate per index)."""
    n = len(points)
    tab = [1]
    # bit i of the index <-> points[n-1-i]: the first doubling creates bit 0,
    # so walk the points from the last one.
    for i in range(n - 1, -1, -1):
        p = points[i]
        tab = [t * (1 - p) % F.M for t in tab] + [t * p % F.M for t in tab]
    return tab


def trace_evaluate(matrix, width, points):
    """Trace::evaluate (evaluation.rs:31-48): res[j] = sum_row Mask(row)(points)
    * matrix[row * width + j] over the row-major height x width trace."""
    assert width >= 1 and len(matrix) % width == 0
    height = len(matrix) // width
    n = len(points)
    assert height == 1 << n
    res = [0] * width
    for row in range(height):
        c = mask_evaluate(row, n, points)
        for j in range(width):
            res[j] = (res[j] + c * matrix[row * width + j]) % F.M
    return res


def delta_evaluate(data, points):
    """Delta::evaluate (evaluation.rs:75-91): prod a*b + (1-a)(1-b)."""
    acc = 1
    for a, b in zip(data, points):
        acc = acc * ((a * b + (1 - a) * (1 - b)) % F.M) % F.M
    return acc


class SumcheckTables:
    def __init__(self, matrix, delta, width=1):
        self.matrix = list(matrix)
        self.delta = list(delta)
        self.width = width
        self.height = len(delta)

    @staticmethod
    def build_tables_for_pcs(inputs, evals):  # sumcheck.rs:128-145
        n = len(inputs)
        assert 1 << n == len(evals)
        return SumcheckTables(evals, eq_table(inputs), 1)

    def partial_sum(self, r):
        """sumcheck.rs:204-232 with composition x[0] (width 1)."""
        off = self.height >> 1
        m, d = self.matrix, self.delta
        if r == 1:
            return sum(m[i + off] * d[i + off] for i in range(off)) % F.M
        s = (1 - r) % F.M
        tot = 0
        for i in range(off):
            dd = (s * d[i] + r * d[i + off]) % F.M
            mm = (s * m[i] + r * m[i + off]) % F.M
            tot += mm * dd
        return tot % F.M

    def fold(self, r):  # sumcheck.rs:234-247
        self.height >>= 1
        off = self.height
        s = (1 - r) % F.M
        for i in range(off):
            self.delta[i] = (s * self.delta[i] + r * self.delta[i + off]) % F.M
            self.matrix[i] = (s * self.matrix[i] + r * self.matrix[i + off]) % F.M
        del self.delta[off:]
        del self.matrix[off:]

    def compute_sumcheck_polynomial(self, previous_sum, transcript, total_degree=2):
        """sumcheck.rs:174-202 -> (nonzero_coeffs, r, new_previous_sum)."""
        evals = [0] * (total_degree + 1)
        for i in range(1, total_degree + 1):
            evals[i] = self.partial_sum(F.from_i64(i))
        evals[0] = (previous_sum - evals[1]) % F.M
        pol = interpolate(evals)
        nonzero = pol[1:]
        for c in nonzero:
            transcript.absorb(F.to_bytes(c))
        r = transcript.next_challenge()
        new_prev = uni_evaluate(pol, r)
        self.fold(r)
        return nonzero, r, new_prev


def to_polynomial(nonzero_coeffs, s):
    """SumcheckPolynomial::to_polynomial (sumcheck.rs:269-276)."""
    a0 = F.div((s - sum(nonzero_coeffs)) % F.M, 2)
    return [a0] + list(nonzero_coeffs)


def round_coeffs_from_sums(previous_sum, s1, s2):
    """Closed form of interpolate() on x = 0,1,2 (same field values as
    polynomials.rs:51-87): c2 = (e2 - 2e1 + e0)/2, c1 = e1 - e0 - c2."""
    e0 = (previous_sum - s1) % F.M
    c2 = F.div((s2 - 2 * s1 + e0) % F.M, 2)
    c1 = (s1 - e0 - c2) % F.M
    return e0, c1, c2
