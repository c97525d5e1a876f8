"""src/fri on the MI355X: reed_solomon, the fold loop, FriProverData,
FriProof::{prove, verify} (LOG_BLOWUP = 1, NUM_QUERIES = 128)."""
import ctypes

from . import _lib
from .device import check, context, empty, fe_bytes, fe_from_bytes, lib, ptr

LOG_BLOWUP = _lib.LOG_BLOWUP
NUM_QUERIES = _lib.NUM_QUERIES


def _log2(n):
    if n < 1 or n & (n - 1):
        raise ValueError("Input size must be a power of two")
    return n.bit_length() - 1


def reed_solomon(coeffs, gen, device=0):
    """fri/mod.rs:19-28: zero-pad to 2N, NTT with gen (order 2N)."""
    ctx = context(device)
    n = coeffs.shape[0]
    out = empty(2 * n, device)
    check(lib().mlh_reed_solomon(ctx, ptr(coeffs), _log2(n), fe_bytes(gen), ptr(out)), ctx)
    return out


def reed_solomon_brev(coeffs, gen, device=0):
    """reed_solomon(bit_reverse_permutation(coeffs)) in one transform
    (multilinear_pcs.rs:104-107): the permutation is folded into the loads."""
    ctx = context(device)
    n = coeffs.shape[0]
    out = empty(2 * n, device)
    check(lib().mlh_reed_solomon_brev(ctx, ptr(coeffs), _log2(n), fe_bytes(gen), ptr(out)), ctx)
    return out


def fold_layer(layer, k, log_domain, r, device=0):
    """The fold loop of FriProverData::fold_step (fri/mod.rs:89-114)."""
    ctx = context(device)
    n = layer.shape[0]
    out = empty(n // 2, device)
    check(lib().mlh_fri_fold(ctx, ptr(layer), _log2(n), k, log_domain, fe_bytes(r), ptr(out)), ctx)
    return out


class FriProverData:
    """fri/mod.rs:10-175, device resident.  The code tensor must outlive it."""

    def __init__(self, handle, code, owned=True, owner=None):
        self.h = handle
        self._code = code
        self._owned = owned  # False: a view of a handle another object owns
        self._owner = owner  # that object, kept alive as long as the view

    def __del__(self):
        if not getattr(self, "_owned", True):
            return
        try:
            lib().mlh_fri_prover_destroy(self.h)
        except Exception:
            pass

    @staticmethod
    def init(code, transcript, device=0, gen_pows=None):
        """gen_pows: None (canonical table of the code's length) or
        (gen_pows[1], log2(gen_pows.len())), used by the later fold steps."""
        ctx = context(device)
        h = ctypes.c_void_p()
        if gen_pows is None:
            check(lib().mlh_fri_prover_init(ctx, ptr(code), _log2(code.shape[0]), transcript.h,
                                            ctypes.byref(h)), ctx)
        else:
            check(lib().mlh_fri_prover_init_gp(ctx, ptr(code), _log2(code.shape[0]),
                                               fe_bytes(gen_pows[0]), gen_pows[1], transcript.h,
                                               ctypes.byref(h)), ctx)
        return FriProverData(h.value, code)

    def fold_step(self, k, r, transcript, device=0, gen_pows=None):
        """fold_step(gen_pows, k, r, transcript) (fri/mod.rs:79-134); gen_pows:
        None (the table given at init) or (gen_pows[1], log2(gen_pows.len()))."""
        ctx = context(device)
        if gen_pows is None:
            check(lib().mlh_fri_prover_fold_step(ctx, self.h, k, fe_bytes(r), transcript.h), ctx)
        else:
            check(lib().mlh_fri_prover_fold_step_gp(ctx, self.h, fe_bytes(gen_pows[0]), gen_pows[1], k,
                                                    fe_bytes(r), transcript.h), ctx)

    @staticmethod
    def fold(code, transcript, device=0, gen_pows=None):
        ctx = context(device)
        h = ctypes.c_void_p()
        if gen_pows is None:
            check(lib().mlh_fri_prover_fold(ctx, ptr(code), _log2(code.shape[0]), transcript.h,
                                            ctypes.byref(h)), ctx)
        else:
            check(lib().mlh_fri_prover_fold_gp(ctx, ptr(code), _log2(code.shape[0]),
                                               fe_bytes(gen_pows[0]), gen_pows[1], transcript.h,
                                               ctypes.byref(h)), ctx)
        return FriProverData(h.value, code)

    def fold_roots(self):
        t = lib().mlh_fri_prover_num_trees(self.h)
        buf = (ctypes.c_uint8 * (32 * t))()
        check(lib().mlh_fri_prover_roots(self.h, buf))
        raw = bytes(buf)
        return [raw[32 * i:32 * i + 32] for i in range(t)]

    @property
    def last_element(self):
        out = (ctypes.c_uint8 * 16)()
        if lib().mlh_fri_prover_last_element(self.h, out) != 0:
            return None
        return fe_from_bytes(out)

    def open_query_at(self, index, log_code, device=0):
        ctx = context(device)
        nb = lib().mlh_fri_query_bytes(log_code)
        buf = (ctypes.c_uint8 * nb)()
        check(lib().mlh_fri_prover_open_query(ctx, self.h, index, buf), ctx)
        return parse_query(bytes(buf), log_code)

    def open_queries(self, indices, log_code, device=0):
        """open_query_at for many indices in one gather (any count; up to 128
        travel in the kernel arguments, more through device memory)."""
        ctx = context(device)
        nb = lib().mlh_fri_query_bytes(log_code)
        n = len(indices)
        idx = (ctypes.c_uint64 * max(n, 1))(*indices)
        buf = (ctypes.c_uint8 * max(nb * n, 1))()
        check(lib().mlh_fri_prover_open_queries(ctx, self.h, idx, n, buf), ctx)
        raw = bytes(buf)
        return [parse_query(raw[q * nb:(q + 1) * nb], log_code) for q in range(n)]


def parse_query(raw, log_code):
    """-> [(pair_bytes32, [sibling digests])] per tree (QueryProof.paths)."""
    out, off = [], 0
    for t in range(log_code - 1):
        depth = log_code - 1 - t
        val = raw[off:off + 32]
        sibs = [raw[off + 32 * (1 + i):off + 32 * (2 + i)] for i in range(depth)]
        out.append((val, sibs))
        off += 32 * (1 + depth)
    return out


class FriProof:
    """fri/mod.rs:239-249 backed by the C struct."""

    def __init__(self, log_code):
        self.log_code = log_code
        t = log_code - LOG_BLOWUP
        self._commit = (ctypes.c_uint8 * (32 * t))()
        self._idx = (ctypes.c_uint64 * NUM_QUERIES)()
        qb = lib().mlh_fri_query_bytes(log_code)
        self._q = (ctypes.c_uint8 * (qb * NUM_QUERIES))()
        self.qbytes = qb
        self.c = _lib.FriProofC()
        self.c.commitments = ctypes.cast(self._commit, ctypes.c_void_p)
        self.c.query_indices = ctypes.cast(self._idx, ctypes.c_void_p)
        self.c.queries = ctypes.cast(self._q, ctypes.c_void_p)

    @staticmethod
    def prove(code, transcript, device=0, gen_pows=None):
        """FriProof::prove (fri/mod.rs:261-285).  gen_pows: None for the
        canonical table of the code's length, else (gen_pows[1], log2(len))."""
        ctx = context(device)
        lc = _log2(code.shape[0])
        p = FriProof(lc)
        if gen_pows is None:
            check(lib().mlh_fri_prove(ctx, ptr(code), lc, transcript.h, ctypes.byref(p.c)), ctx)
        else:
            g, lg = gen_pows
            check(lib().mlh_fri_prove_gp(ctx, ptr(code), lc, fe_bytes(g), lg, transcript.h,
                                         ctypes.byref(p.c)), ctx)
        return p

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
        raw = bytes(self._q)[q * self.qbytes:(q + 1) * self.qbytes]
        return parse_query(raw, self.log_code)

    def verify(self):
        """FriProof::verify (fri/mod.rs:287-309) in libmlhip (host)."""
        return lib().mlh_fri_verify(ctypes.byref(self.c)) == 0

    def to_bytes(self):
        """bincode 2 (standard, LE, fixed-int) serde encoding, as the reference's
        encode_to_vec (fri/mod.rs:367-392)."""
        n = lib().mlh_fri_proof_encoded_size(ctypes.byref(self.c))
        buf = (ctypes.c_uint8 * n)()
        check(lib().mlh_fri_proof_encode(ctypes.byref(self.c), buf, n))
        return bytes(buf)

    @staticmethod
    def from_bytes(data: bytes):
        """decode_from_slice (fri/mod.rs:394-397) into a host FriProof."""
        src = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
        lc, nq = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().mlh_fri_proof_decode_header(src, len(data), ctypes.byref(lc), ctypes.byref(nq)))
        if nq.value != NUM_QUERIES:
            raise _lib.MlhError(_lib.MLH_ERR_INVALID, "expected %d queries" % NUM_QUERIES)
        p = FriProof(lc.value)
        p.c.log_code = lc.value
        p.c.num_queries = nq.value
        check(lib().mlh_fri_proof_decode(src, len(data), ctypes.byref(p.c)))
        return p
