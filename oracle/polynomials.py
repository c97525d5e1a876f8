"""Multilinear / univariate polynomial helpers (oracle).  Test infrastructure only.

Reference: src/polynomials.rs.  Multilinear index convention: bit b of the
evaluation index pairs with args[n-1-b] (big endian), :126-146, :165-187.
"""
from . import field as F


def to_coefficient(evals):
    """MultilinearPolynomialEvals::to_coefficient (polynomials.rs:150-163):
    Moebius transform, for bit i (LSB first): c[j] -= c[j ^ 2^i] if bit set.
    Like the reference, len need not be a power of two (only the low
    trailing_zeros(len) bits are transformed)."""
    n = (len(evals) & -len(evals)).bit_length() - 1
    c = list(evals)
    for i in range(n):
        m = 1 << i
        for j in range(1 << n):
            if j & m:
                c[j] = (c[j] - c[j ^ m]) % F.M
    return c


def to_evaluation(coeffs):
    """MultilinearPolynomial::to_evaluation (polynomials.rs:111-124): zeta."""
    n = (len(coeffs) & -len(coeffs)).bit_length() - 1
    e = list(coeffs)
    for i in range(n):
        m = 1 << i
        for j in range(1 << n):
            if j & m:
                e[j] = (e[j] + e[j ^ m]) % F.M
    return e


def mle_evaluate(evals, args):
    """MultilinearPolynomialEvals::evaluate (polynomials.rs:165-187)."""
    n = len(args)
    assert 1 << n == _next_pow2(len(evals)), "Wrong number of arguments"
    total = 0
    for pos, e in enumerate(evals):
        term = e
        for bit_pos in range(n):
            a = args[n - 1 - bit_pos]
            term = term * (a if (pos >> bit_pos) & 1 else (1 - a)) % F.M
        total += term
    return total % F.M


def mle_coeffs_evaluate(coeffs, args):
    """MultilinearPolynomial::evaluate (polynomials.rs:126-146)."""
    n = len(args)
    total = 0
    for pos, c in enumerate(coeffs):
        term = c
        for bit_pos in range(n):
            if (pos >> bit_pos) & 1:
                term = term * args[n - 1 - bit_pos] % F.M
        total += term
    return total % F.M


def _next_pow2(x):
    p = 1
    while p < x:
        p <<= 1
    return p


def uni_evaluate(coeffs, x):
    """Polynomial::evaluate (polynomials.rs:9-14), Horner."""
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % F.M
    return acc


def interpolate(evals):
    """PolynomialEvals::interpolate (polynomials.rs:51-87): Lagrange on
    x = 0..n-1 (F::from(i as i64))."""
    n = len(evals)
    coeffs = [0] * n
    for j, yj in enumerate(evals):
        lj = [1]
        denom = 1
        for m in range(n):
            if m == j:
                continue
            # lj *= (x - m)
            nl = [0] * (len(lj) + 1)
            for i, a in enumerate(lj):
                nl[i] = (nl[i] - a * m) % F.M
                nl[i + 1] = (nl[i + 1] + a) % F.M
            lj = nl
            denom = denom * (j - m) % F.M
        scale = yj * F.inv(denom) % F.M
        for i in range(n):
            coeffs[i] = (coeffs[i] + scale * lj[i]) % F.M
    return coeffs
