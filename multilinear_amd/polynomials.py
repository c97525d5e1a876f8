"""src/polynomials.rs multilinear parts on the MI355X."""
import ctypes

from .device import check, context, fe_from_bytes, lib, ptr


def _log2(n):
    if n < 1 or n & (n - 1):
        raise ValueError("length must be a power of two")
    return n.bit_length() - 1


def _low_bits(n):
    """trailing_zeros(len): the reference transforms the first 2^tz entries
    over tz index bits and leaves the rest (len need not be a power of two)."""
    if n < 1:
        raise ValueError("empty polynomial")
    return (n & -n).bit_length() - 1


def to_coefficient(evals, device=0):
    """MultilinearPolynomialEvals::to_coefficient (polynomials.rs:150-163); new tensor."""
    ctx = context(device)
    out = evals.clone()
    check(lib().mlh_mle_to_coefficient(ctx, ptr(out), _low_bits(evals.shape[0])), ctx)
    return out


def to_evaluation(coeffs, device=0):
    """MultilinearPolynomial::to_evaluation (polynomials.rs:111-124); new tensor."""
    ctx = context(device)
    out = coeffs.clone()
    check(lib().mlh_mle_to_evaluation(ctx, ptr(out), _low_bits(coeffs.shape[0])), ctx)
    return out


def _points(args):
    raw = b"".join(int(a).to_bytes(16, "little") for a in args)
    return (ctypes.c_uint8 * max(1, len(raw))).from_buffer_copy(raw or b"\0")


def _padded(t, n):
    """The reference asserts 1 << len(args) == len.next_power_of_two(): a
    shorter table sums over its own positions only, i.e. zero padding."""
    m = t.shape[0]
    if m < 1 or 1 << n != 1 << (m - 1).bit_length():
        raise ValueError("Wrong number of arguments")
    if m == 1 << n:
        return t
    import torch

    out = torch.zeros((1 << n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    out[:m] = t
    return out


def evaluate(evals, args, device=0):
    """MultilinearPolynomialEvals::evaluate (polynomials.rs:165-187)."""
    n = len(args)
    evals = _padded(evals, n)
    ctx = context(device)
    out = (ctypes.c_uint8 * 16)()
    check(lib().mlh_mle_evaluate(ctx, ptr(evals), n, _points(args), out), ctx)
    return fe_from_bytes(out)


def coeffs_evaluate(coeffs, args, device=0):
    """MultilinearPolynomial::evaluate (polynomials.rs:126-146), coefficient
    form: sum_pos coeffs[pos] * prod_{bit b of pos set} args[n-1-b]."""
    n = len(args)
    coeffs = _padded(coeffs, n)
    ctx = context(device)
    out = (ctypes.c_uint8 * 16)()
    check(lib().mlh_mle_coeffs_evaluate(ctx, ptr(coeffs), n, _points(args), out), ctx)
    return fe_from_bytes(out)


def trace_evaluate(matrix, width, points, device=0):
    """Trace::evaluate (constraint_system/evaluation.rs:31-48): the row-major
    height x width trace on the device, one MLE per column, at `points`."""
    n = len(points)
    if matrix.shape[0] != width << n:
        raise ValueError("trace height must be 2^len(points)")
    ctx = context(device)
    out = (ctypes.c_uint8 * (16 * width))()
    check(lib().mlh_trace_evaluate(ctx, ptr(matrix), n, width, _points(points), out), ctx)
    raw = bytes(out)
    return [fe_from_bytes(raw[16 * j:16 * j + 16]) for j in range(width)]


def eq_table(points, device=0):
    """delta table of build_tables_for_pcs (sumcheck.rs:133-138)."""
    from .device import empty

    ctx = context(device)
    out = empty(1 << len(points), device)
    check(lib().mlh_eq_table(ctx, _points(points), len(points), ptr(out)), ctx)
    return out
