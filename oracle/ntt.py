"""Radix-2 NTT / INTT (oracle).  Test infrastructure only.

Reference: src/ntt/mod.rs:60-173.  Natural-order input and output:
evals[i] = sum_j coeffs[j] * gen^(i*j).  The restatement keeps the
reference's algorithm (bit-reverse, unrolled len=2 stage, iterative DIT with a
per-stage serial twiddle vector) so that it doubles as the CPU-path model.
"""
from . import field as F


def bit_reverse_permutation(values):
    """src/ntt/mod.rs:113-123 (in place).  n must be a power of two >= 2
    (n = 1 would shift a usize by 64 in the reference)."""
    n = len(values)
    bits = n.bit_length() - 1
    for i in range(n):
        j = int(format(i, "0%db" % bits)[::-1], 2) if bits else 0
        if i < j:
            values[i], values[j] = values[j], values[i]


def _dit(values, gen):
    n = len(values)
    # unrolled first stage, src/ntt/mod.rs:80-86
    for i in range(0, n, 2):
        u, v = values[i], values[i + 1]
        values[i] = (u + v) % F.M
        values[i + 1] = (u - v) % F.M
    length = 4
    while length <= n:  # src/ntt/mod.rs:88-107
        cur = F.fpow(gen, n // length)
        half = length // 2
        pows = [1] * half
        for j in range(1, half):
            pows[j] = pows[j - 1] * cur % F.M
        for i in range(0, n, length):
            for j in range(half):
                v = values[i + j + half] * pows[j] % F.M
                u = values[i + j]
                values[i + j] = (u + v) % F.M
                values[i + j + half] = (u - v) % F.M
        length *= 2


def ntt(coeffs, gen):
    """Polynomial::ntt (src/ntt/mod.rs:69-110) -> evals (new list)."""
    n = len(coeffs)
    assert n & (n - 1) == 0 and n >= 2, "The number of coeffs must be a power of 2"
    values = list(coeffs)
    bit_reverse_permutation(values)
    _dit(values, gen)
    return values


def intt(evals, gen):
    """LagrangePolynomial::intt (src/ntt/mod.rs:132-173): ntt with gen^-1,
    then scale by 1/F::from(n as i64)."""
    n = len(evals)
    assert n & (n - 1) == 0 and n >= 2
    values = list(evals)
    bit_reverse_permutation(values)
    _dit(values, F.inv(gen))
    n_inv = F.inv(F.from_i64(n))
    return [v * n_inv % F.M for v in values]


def evaluate(coeffs, x):
    """Polynomial::evaluate (src/ntt/mod.rs:62-67), Horner."""
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % F.M
    return acc


def ntt_direct(coeffs, gen):
    """O(n^2) definition, used only to cross-check tiny cases."""
    n = len(coeffs)
    return [sum(c * F.fpow(gen, i * j) for j, c in enumerate(coeffs)) % F.M for i in range(n)]
