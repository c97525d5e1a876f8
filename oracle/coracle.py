"""ctypes binding of the C oracle (oracle/liboracle.so).  Test infrastructure only."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise ImportError("oracle/liboracle.so not built (make -C oracle)")
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        U = ctypes.c_uint32
        L.orc_ntt.argtypes = [P, P, U, P, ctypes.c_int]
        L.orc_reed_solomon.argtypes = [P, U, P, P]
        L.orc_merkle_commit_pairs.argtypes = [P, U, P]
        L.orc_fri_commit.argtypes = [P, U, P, P, P]
        L.orc_to_coefficient.argtypes = [P, U]
        L.orc_eq_table.argtypes = [P, U, P]
        L.orc_partial_sums.argtypes = [P, P, U, P]
        L.orc_fold.argtypes = [P, P, U, P]
        L.orc_sha256.argtypes = [P, ctypes.c_uint64, P]
        L.orc_mul.argtypes = [P, P, P]
        L.orc_ntt_omp.argtypes = [P, P, U, P, ctypes.c_int]
        L.orc_pow_2_generator.argtypes = [U, P]
        L.orc_pow_2_generator_powers.argtypes = [U, P]
        I = ctypes.c_int
        L.orc_ntt_par.argtypes = [P, P, U, P, I, I]
        L.orc_reed_solomon_par.argtypes = [P, U, P, P, I]
        L.orc_fri_commit_par.argtypes = [P, U, U, P, P, P, I]
        L.orc_eq_table_par.argtypes = [P, U, P, I]
        L.orc_partial_sums_par.argtypes = [P, P, U, P, I]
        L.orc_fold_par.argtypes = [P, P, U, P, I]
        L.orc_dot_par.argtypes = [P, P, U, P, I]
        L.orc_pcs_query_bytes.argtypes = [U, U, I]
        L.orc_pcs_query_bytes.restype = ctypes.c_uint64
        L.orc_pcs_prove_par.argtypes = [P, U, U, P, P, I, P, ctypes.c_uint64, P, P, P, P, P, P, P, I]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _fe(v):
    return np.frombuffer(int(v).to_bytes(16, "little"), dtype=np.uint8).copy()


def ntt(limbs, log_n, gen, inverse=False):
    """limbs: (n,4) uint32 array -> new array."""
    a = np.ascontiguousarray(limbs, dtype=np.uint32)
    out = np.empty_like(a)
    g = _fe(gen)
    rc = lib().orc_ntt(_p(a), _p(out), log_n, _p(g), 1 if inverse else 0)
    assert rc == 0
    return out


def ntt_omp(limbs, log_n, gen, threads):
    """OpenMP variant of ntt (cpu_baseline on all host cores)."""
    a = np.ascontiguousarray(limbs, dtype=np.uint32)
    out = np.empty_like(a)
    rc = lib().orc_ntt_omp(_p(a), _p(out), log_n, _p(_fe(gen)), threads)
    assert rc == 0
    return out


def reed_solomon(limbs, log_n, gen):
    a = np.ascontiguousarray(limbs, dtype=np.uint32)
    out = np.empty((2 * a.shape[0], 4), dtype=np.uint32)
    rc = lib().orc_reed_solomon(_p(a), log_n, _p(_fe(gen)), _p(out))
    assert rc == 0
    return out


def merkle_commit_pairs(limbs, log_code):
    a = np.ascontiguousarray(limbs, dtype=np.uint32)
    L = 1 << (log_code - 1)
    layers = np.empty((2 * L - 1, 32), dtype=np.uint8)
    lib().orc_merkle_commit_pairs(_p(a), log_code, _p(layers))
    return layers


def fri_commit(limbs, log_code):
    """-> (roots list, last_elem int, last_random bytes, rc)."""
    a = np.ascontiguousarray(limbs, dtype=np.uint32)
    roots = np.zeros((log_code - 1, 32), dtype=np.uint8)
    last = np.zeros(16, dtype=np.uint8)
    lr = np.zeros(32, dtype=np.uint8)
    rc = lib().orc_fri_commit(_p(a), log_code, _p(roots), _p(last), _p(lr))
    return [bytes(r) for r in roots], int.from_bytes(bytes(last), "little"), bytes(lr), rc


def to_coefficient(limbs, log_n):
    a = np.ascontiguousarray(limbs, dtype=np.uint32).copy()
    lib().orc_to_coefficient(_p(a), log_n)
    return a


def eq_table(points):
    pts = np.frombuffer(b"".join(int(p).to_bytes(16, "little") for p in points) or b"\0" * 16,
                        dtype=np.uint8).copy()
    out = np.empty((1 << len(points), 4), dtype=np.uint32)
    lib().orc_eq_table(_p(pts), len(points), _p(out))
    return out


def partial_sums(m, d, log_h):
    out = np.zeros(32, dtype=np.uint8)
    lib().orc_partial_sums(_p(np.ascontiguousarray(m)), _p(np.ascontiguousarray(d)), log_h, _p(out))
    b = bytes(out)
    return int.from_bytes(b[:16], "little"), int.from_bytes(b[16:], "little")


def sha256(msg: bytes) -> bytes:
    buf = np.frombuffer(msg, dtype=np.uint8).copy() if msg else np.zeros(1, dtype=np.uint8)
    out = np.zeros(32, dtype=np.uint8)
    lib().orc_sha256(_p(buf), len(msg), _p(out))
    return bytes(out)


def mul(a, b):
    out = np.zeros(16, dtype=np.uint8)
    lib().orc_mul(_p(_fe(a)), _p(_fe(b)), _p(out))
    return int.from_bytes(bytes(out), "little")


# ---- parallel checkers (same arithmetic, OpenMP; full-size parity tests) ----

def threads():
    return max(1, min(16, os.cpu_count() or 1))


def ntt_par(limbs, log_n, gen, inverse=False):
    a = np.ascontiguousarray(limbs, dtype=np.uint32)
    out = np.empty_like(a)
    rc = lib().orc_ntt_par(_p(a), _p(out), log_n, _p(_fe(gen)), 1 if inverse else 0, threads())
    assert rc == 0
    return out


def reed_solomon_par(limbs, log_n, gen):
    a = np.ascontiguousarray(limbs, dtype=np.uint32)
    out = np.empty((2 * a.shape[0], 4), dtype=np.uint32)
    rc = lib().orc_reed_solomon_par(_p(a), log_n, _p(_fe(gen)), _p(out), threads())
    assert rc == 0
    return out


def fri_commit_par(limbs, log_code, log_gp=None):
    """FriProverData::fold with gen_pows of 2^log_gp entries (default: the code
    length) -> (roots, last_elem, last_random, rc)."""
    a = np.ascontiguousarray(limbs, dtype=np.uint32)
    roots = np.zeros((log_code - 1, 32), dtype=np.uint8)
    last = np.zeros(16, dtype=np.uint8)
    lr = np.zeros(32, dtype=np.uint8)
    rc = lib().orc_fri_commit_par(_p(a), log_code, log_code if log_gp is None else log_gp, _p(roots),
                                  _p(last), _p(lr), threads())
    return [bytes(r) for r in roots], int.from_bytes(bytes(last), "little"), bytes(lr), rc


def eq_table_par(points):
    pts = np.frombuffer(b"".join(int(p).to_bytes(16, "little") for p in points) or b"\0" * 16,
                        dtype=np.uint8).copy()
    out = np.empty((1 << len(points), 4), dtype=np.uint32)
    lib().orc_eq_table_par(_p(pts), len(points), _p(out), threads())
    return out


def partial_sums_par(m, d, log_h):
    out = np.zeros(32, dtype=np.uint8)
    lib().orc_partial_sums_par(_p(np.ascontiguousarray(m)), _p(np.ascontiguousarray(d)), log_h, _p(out),
                               threads())
    b = bytes(out)
    return int.from_bytes(b[:16], "little"), int.from_bytes(b[16:], "little")


def fold_par(m, d, log_h, r):
    """In place on (contiguous uint32) m and d."""
    lib().orc_fold_par(_p(m), _p(d), log_h, _p(_fe(r)), threads())


def dot_par(m, d, log_n):
    out = np.zeros(16, dtype=np.uint8)
    lib().orc_dot_par(_p(np.ascontiguousarray(m)), _p(np.ascontiguousarray(d)), log_n, _p(out), threads())
    return int.from_bytes(bytes(out), "little")


def _fe_array(vals):
    return np.frombuffer(b"".join(int(v).to_bytes(16, "little") for v in vals) or b"\0" * 16,
                         dtype=np.uint8).copy()


def pcs_prove_par(evals, n, points, outputs, batched=False, prefix=b""):
    """PCSProof::prove (multilinear_pcs.rs:90-136) or, batched,
    BatchedPCSProof::prove (batched_pcs.rs:127-180) in C, end to end.
    evals: (m * 2^n, 4) uint32 limbs, polynomial-major.  Returns a dict with
    polys [(c1, c2)], batch_root, roots, last_elem, last_random, indices and
    the flat query records (bytes, the layout of libmlhip's query staging)."""
    ev = np.ascontiguousarray(evals, dtype=np.uint32)
    m = ev.shape[0] >> n
    assert ev.shape[0] == m << n and len(outputs) == m
    L = lib()
    qb = L.orc_pcs_query_bytes(m, n, 1 if batched else 0)
    polys = np.zeros(32 * n, dtype=np.uint8)
    broot = np.zeros(32, dtype=np.uint8)
    nroots = n - (1 if batched else 0)
    roots = np.zeros(32 * max(nroots, 1), dtype=np.uint8)
    last = np.zeros(16, dtype=np.uint8)
    lr = np.zeros(32, dtype=np.uint8)
    qidx = np.zeros(128, dtype=np.uint64)
    qrec = np.zeros(128 * qb, dtype=np.uint8)
    pre = np.frombuffer(prefix, dtype=np.uint8).copy() if prefix else np.zeros(1, dtype=np.uint8)
    rc = L.orc_pcs_prove_par(_p(ev), m, n, _p(_fe_array(points)), _p(_fe_array(outputs)),
                             1 if batched else 0, _p(pre), len(prefix), _p(polys), _p(broot), _p(roots),
                             _p(last), _p(lr), _p(qidx), _p(qrec), threads())
    raw = bytes(polys)
    rr = bytes(roots)
    return {
        "rc": rc,
        "polys": [(int.from_bytes(raw[32 * k:32 * k + 16], "little"),
                   int.from_bytes(raw[32 * k + 16:32 * k + 32], "little")) for k in range(n)],
        "batch_root": bytes(broot) if batched else None,
        "roots": [rr[32 * i:32 * i + 32] for i in range(nroots)],
        "last_elem": int.from_bytes(bytes(last), "little"),
        "last_random": bytes(lr),
        "indices": [int(x) for x in qidx],
        "queries": bytes(qrec),
        "query_bytes": qb,
    }


def mle_evaluate_par(evals, n, points):
    """MultilinearPolynomialEvals::evaluate (polynomials.rs:165-187) as
    sum_i evals[i] * eq(points)[i]."""
    return dot_par(np.ascontiguousarray(evals, dtype=np.uint32), eq_table_par(points), n)
