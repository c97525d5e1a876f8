"""src/ntt/mod.rs on the MI355X: Polynomial::ntt, LagrangePolynomial::intt,
bit_reverse_permutation, NttField::pow_2_generator(_powers).

Values are device tensors (n, 4) int32 (see device.py)."""
import ctypes

from .device import check, context, empty, fe_bytes, fe_from_bytes, lib, ptr


def _log2(n):
    if n < 1 or n & (n - 1):
        raise ValueError("The number of coeffs must be a power of 2")
    return n.bit_length() - 1


def pow_2_generator(log_size):
    """NttField::pow_2_generator (ntt/mod.rs:42-54); None beyond 2^40."""
    out = (ctypes.c_uint8 * 16)()
    if lib().mlh_pow_2_generator(log_size, out) != 0:
        return None
    return fe_from_bytes(out)


def pow_2_generator_powers(log_size, device=0):
    """ntt/mod.rs:18-28 -> device tensor [g^0 .. g^(2^log_size - 1)]."""
    ctx = context(device)
    out = empty(1 << log_size, device)
    check(lib().mlh_pow_2_generator_powers(ctx, log_size, ptr(out)), ctx)
    return out


def bit_reverse_permutation(values, device=0):
    """ntt/mod.rs:113-123 (returns a new tensor)."""
    ctx = context(device)
    out = empty(values.shape[0], device)
    check(lib().mlh_bit_reverse_permutation(ctx, ptr(values), ptr(out), _log2(values.shape[0])), ctx)
    return out


class LagrangePolynomial:
    def __init__(self, gen, evals):
        self.gen = gen
        self.evals = evals

    def intt(self, device=0):
        """ntt/mod.rs:132-173."""
        ctx = context(device)
        out = empty(self.evals.shape[0], device)
        check(lib().mlh_intt(ctx, ptr(self.evals), ptr(out), _log2(self.evals.shape[0]),
                             fe_bytes(self.gen)), ctx)
        return Polynomial(out)


class Polynomial:
    def __init__(self, coeffs):
        self.coeffs = coeffs

    def evaluate(self, x, device=0):
        """ntt/mod.rs:61-67 (Horner): sum_i coeffs[i] x^i, any length."""
        ctx = context(device)
        out = (ctypes.c_uint8 * 16)()
        n = self.coeffs.shape[0]
        check(lib().mlh_poly_evaluate(ctx, ptr(self.coeffs) if n else None, n, fe_bytes(x), out),
              ctx)
        return fe_from_bytes(out)

    def ntt(self, gen, device=0):
        """ntt/mod.rs:69-110: natural order in and out."""
        ctx = context(device)
        out = empty(self.coeffs.shape[0], device)
        check(lib().mlh_ntt(ctx, ptr(self.coeffs), ptr(out), _log2(self.coeffs.shape[0]),
                            fe_bytes(gen)), ctx)
        return LagrangePolynomial(gen, out)
