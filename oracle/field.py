"""F_M arithmetic (oracle).  Test infrastructure only -- see oracle/__init__.py.

Reference: src/field.rs (Field128 = winter-math f128 BaseElement) and
src/ntt/mod.rs:34-58 (modulus, generator 3, pow_2_generator, pow).
Elements are Python ints in [0, M); the byte form is the canonical u128
little-endian (src/field.rs:33-38, AsRef<[u8]> returns the raw u128 bytes).
"""

M = 340282366920938463463374557953744961537  # src/ntt/mod.rs:35
assert M == 2**128 - 45 * 2**40 + 1
TWO_ADICITY = 40  # trailing_zeros(M - 1), src/ntt/mod.rs:44
GENERATOR = 3  # src/ntt/mod.rs:39
# winter-math f128 publishes this 2^40-th root of unity (G); 3^((M-1)/2^40).
WINTER_TWO_ADIC_ROOT = 23953097886125630542083529559205016746


def from_u128(v: int) -> int:
    """Field128::from(u128) (src/field.rs:138-142): BaseElement::new reduces
    once; 2M > 2^128 so a single conditional subtraction is complete."""
    assert 0 <= v < 2**128
    return v - M if v >= M else v


def from_i64(v: int) -> int:
    """Field128::from(i64) (src/field.rs:150-154): `val as u128` sign-extends,
    so negative inputs are NOT -v mod M (from(-1) = 2^128 - 1 - M)."""
    return from_u128(v % 2**128)


def add(a, b):
    return (a + b) % M


def sub(a, b):
    return (a - b) % M


def mul(a, b):
    return (a * b) % M


def neg(a):
    return (-a) % M


def inv(a):
    """Field128 Div (field.rs:113-124) -> winterfell 0.12's f128 BaseElement
    division, self * rhs.inv(); winter-math documents inv(ZERO) = ZERO, which
    a^(M-2) gives as well (LagrangePolynomial::intt with gen = 0)."""
    return pow(a % M, M - 2, M)


def div(a, b):
    return mul(a, inv(b))


def fpow(a, e):
    """FieldElement::exp (src/ntt/mod.rs:56-58)."""
    return pow(a, e, M)


def to_bytes(a: int) -> bytes:
    """src/field.rs:33-38: the canonical u128, little endian."""
    return a.to_bytes(16, "little")


def from_bytes(b: bytes) -> int:
    return int.from_bytes(b, "little")


def pow_2_generator(log_size: int):
    """NttField::pow_2_generator (src/ntt/mod.rs:42-54)."""
    if log_size > TWO_ADICITY:
        return None
    return fpow(GENERATOR, (M - 1) // (1 << log_size))


def pow_2_generator_powers(log_size: int):
    """NttField::pow_2_generator_powers (src/ntt/mod.rs:18-28): serial powers."""
    g = pow_2_generator(log_size)
    if g is None:
        return None
    out = []
    cur = 1
    for _ in range(1 << log_size):
        out.append(cur)
        cur = mul(cur, g)
    return out


# ---- bulk helpers: lists of ints <-> numpy (N, 4) uint32 limb arrays ----

def to_limbs(values):
    import numpy as np

    arr = np.empty((len(values), 4), dtype=np.uint32)
    for i, v in enumerate(values):
        arr[i, 0] = v & 0xFFFFFFFF
        arr[i, 1] = (v >> 32) & 0xFFFFFFFF
        arr[i, 2] = (v >> 64) & 0xFFFFFFFF
        arr[i, 3] = (v >> 96) & 0xFFFFFFFF
    return arr


def from_limbs(arr):
    a = arr.reshape(-1, 4).astype(object)
    return [int(r[0]) | (int(r[1]) << 32) | (int(r[2]) << 64) | (int(r[3]) << 96) for r in a]
