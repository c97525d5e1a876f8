"""src/fri/batched_fri.rs and src/fri/batched_pcs.rs on the MI355X.

Codes / MLEs are one device tensor of shape (m * size, 4): item j occupies
rows [j * size, (j + 1) * size).  Proofs are host buffers in the C layout of
include/mlhip.h (mlh_batched_fri_proof)."""
import ctypes

from . import _lib
from .device import check, context, fe_bytes, fe_from_bytes, lib, ptr

NUM_QUERIES = _lib.NUM_QUERIES


def _log2(n):
    if n < 1 or n & (n - 1):
        raise ValueError("size must be a power of two")
    return n.bit_length() - 1


class BatchedFriProof:
    """BatchedFriProof (batched_fri.rs:21-27) backed by the C struct."""

    def __init__(self, log_code, m):
        self.log_code, self.m = log_code, m
        t = max(0, log_code - 2)
        self._commit = (ctypes.c_uint8 * max(1, 32 * t))()
        self._idx = (ctypes.c_uint64 * NUM_QUERIES)()
        self.qbytes = lib().mlh_batched_fri_query_bytes(log_code, m)
        self._q = (ctypes.c_uint8 * (self.qbytes * NUM_QUERIES))()
        self.c = _lib.BatchedFriProofC()
        self.c.log_code, self.c.num_codes = log_code, m
        self.c.commitments = ctypes.cast(self._commit, ctypes.c_void_p)
        self.c.query_indices = ctypes.cast(self._idx, ctypes.c_void_p)
        self.c.queries = ctypes.cast(self._q, ctypes.c_void_p)

    @staticmethod
    def prove(codes, m, transcript, device=0):
        """BatchedFriProof::prove (batched_fri.rs:280-311)."""
        ctx = context(device)
        size = codes.shape[0] // m
        lc = _log2(size)
        p = BatchedFriProof(lc, m)
        check(lib().mlh_batched_fri_prove(ctx, ptr(codes), m, lc, transcript.h,
                                          ctypes.byref(p.c)), ctx)
        return p

    @property
    def batch_commitment(self):
        return bytes(self.c.batch_commitment)

    @property
    def commitments(self):
        raw = bytes(self._commit)
        return [raw[32 * i:32 * i + 32] for i in range(self.c.num_trees)]

    @property
    def last_elem(self):
        return fe_from_bytes(self.c.last_elem)

    @property
    def last_random(self):
        return bytes(self.c.last_random)

    @property
    def query_indices(self):
        return list(self._idx)

    def query(self, q):
        """-> ((m pair bytes32 list, batch siblings), [(pair32, siblings)] inner)."""
        raw = bytes(self._q)[q * self.qbytes:(q + 1) * self.qbytes]
        L, m = self.log_code, self.m
        col = [raw[32 * j:32 * j + 32] for j in range(m)]
        off = 32 * m
        bs = [raw[off + 32 * i:off + 32 * i + 32] for i in range(L - 1)]
        off += 32 * (L - 1)
        inner = []
        for t in range(L - 2):
            depth = L - 2 - t
            val = raw[off:off + 32]
            sibs = [raw[off + 32 * (1 + i):off + 32 * (2 + i)] for i in range(depth)]
            inner.append((val, sibs))
            off += 32 * (1 + depth)
        return (col, bs), inner

    def verify(self):
        """BatchedFriProof::verify (batched_fri.rs:313-343), host side."""
        return lib().mlh_batched_fri_verify(ctypes.byref(self.c)) == 0


def _fes(vals):
    raw = b"".join(int(v).to_bytes(16, "little") for v in vals)
    return (ctypes.c_uint8 * max(1, len(raw))).from_buffer_copy(raw or b"\0")


class BatchedPCSProof:
    """BatchedPCSProof (batched_pcs.rs:22-34)."""

    def __init__(self, n_vars, m):
        self.fri_proof = BatchedFriProof(n_vars + 1, m)
        self._polys = (ctypes.c_uint8 * (32 * n_vars))()
        self.c = _lib.BatchedPcsProofC()
        self.c.fri = self.fri_proof.c
        self.c.sumcheck_polys = ctypes.cast(self._polys, ctypes.c_void_p)
        self.n_vars, self.m = n_vars, m

    @staticmethod
    def prove(inputs, outputs, evals, transcript, device=0):
        """BatchedPCSProof::prove (batched_pcs.rs:127-180); evals: (m * 2^n, 4)."""
        n, m = len(inputs), len(outputs)
        assert evals.shape[0] == m << n
        ctx = context(device)
        p = BatchedPCSProof(n, m)
        check(lib().mlh_batched_pcs_prove(ctx, ptr(evals), m, n, _fes(inputs), _fes(outputs),
                                          transcript.h, ctypes.byref(p.c)), ctx)
        p.fri_proof.c = p.c.fri
        p.inputs, p.outputs = list(inputs), list(outputs)
        return p

    @property
    def sumcheck_polynomials(self):
        raw = bytes(self._polys)
        return [(fe_from_bytes(raw[32 * k:32 * k + 16]), fe_from_bytes(raw[32 * k + 16:32 * k + 32]))
                for k in range(self.n_vars)]

    def verify(self, transcript):
        """BatchedPCSProof::verify (batched_pcs.rs:182-250), host side."""
        c = _lib.BatchedPcsProofC()
        c.fri = self.fri_proof.c
        c.sumcheck_polys = ctypes.cast(self._polys, ctypes.c_void_p)
        return lib().mlh_batched_pcs_verify(ctypes.byref(c), self.n_vars, _fes(self.inputs),
                                            _fes(self.outputs), transcript.h) == 0


class BatchedFriProverData:
    """BatchedFriProverData (batched_fri.rs:9-224) step by step on the device,
    the transcript on the host.  codes: (m * 2^L, 4) device tensor (outlives it)."""

    def __init__(self, handle, codes, m, log_code):
        self.h, self._codes, self.m, self.log_code = handle, codes, m, log_code

    def __del__(self):
        try:
            lib().mlh_batched_fri_prover_destroy(self.h)
        except Exception:
            pass

    @staticmethod
    def init(codes, m, transcript, device=0):
        """batched_fri.rs:41-98."""
        ctx = context(device)
        n = codes.shape[0] // m
        assert n * m == codes.shape[0]
        h = ctypes.c_void_p()
        check(lib().mlh_batched_fri_prover_init(ctx, ptr(codes), m, _log2(n), transcript.h,
                                                ctypes.byref(h)), ctx)
        return BatchedFriProverData(h.value, codes, m, _log2(n))

    def batched_fold_step(self, gen_pows, r, transcript, device=0):
        """batched_fold_step(gen_pows, r, transcript) (batched_fri.rs:100-176);
        gen_pows = (gen_pows[1], log2(gen_pows.len()))."""
        ctx = context(device)
        check(lib().mlh_batched_fri_prover_fold_step_gp(ctx, self.h, fe_bytes(gen_pows[0]), gen_pows[1],
                                                        fe_bytes(r), transcript.h), ctx)

    @property
    def fri_data(self):
        """self.fri_data: the inner FriProverData (a view; this object owns it)."""
        from .fri import FriProverData

        return FriProverData(lib().mlh_batched_fri_prover_inner(self.h), self._codes, owned=False,
                             owner=self)

    @property
    def batch_root(self):
        out = (ctypes.c_uint8 * 32)()
        check(lib().mlh_batched_fri_prover_batch_root(self.h, out))
        return bytes(out)

    @property
    def fingerprint_r(self):
        out = (ctypes.c_uint8 * 16)()
        check(lib().mlh_batched_fri_prover_fingerprint_r(self.h, out))
        return fe_from_bytes(out)

    def open_query_at(self, index, device=0):
        """batched_fri.rs:207-224 -> the flat record (mlh_batched_fri_query_bytes)."""
        ctx = context(device)
        nb = lib().mlh_batched_fri_query_bytes(self.log_code, self.m)
        buf = (ctypes.c_uint8 * nb)()
        check(lib().mlh_batched_fri_prover_open_query(ctx, self.h, index, buf), ctx)
        return bytes(buf)
