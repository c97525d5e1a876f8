"""ctypes binding of libmlhip.so (the C ABI declared in include/mlhip.h).

The library is built in-tree (``multilinear_amd/libmlhip.so``) by
``__graft_entry__.build()`` / ``make -C multilinear_amd/csrc``.  There is no
fallback: if the library is missing this module raises, and every compute
entry point returns MLH_ERR_HIP when no gfx950 device is usable.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmlhip.so")

MLH_OK = 0
STATUS_NAMES = {
    0: "MLH_OK",
    1: "MLH_ERR_INVALID",
    2: "MLH_ERR_NOT_POW2",
    3: "MLH_ERR_BAD_GENERATOR",
    4: "MLH_ERR_HIP",
    5: "MLH_ERR_OOM",
    6: "MLH_ERR_NOT_RS_CODE",
    7: "MLH_ERR_VERIFY",
    8: "MLH_ERR_VERIFY_INDEX",
    9: "MLH_ERR_COMM",
    10: "MLH_ERR_DEVICE",
}
STATUS_CODES = {v: k for k, v in STATUS_NAMES.items()}
globals().update(STATUS_CODES)  # MLH_ERR_INVALID, ... as module constants
LOG_BLOWUP = 1
NUM_QUERIES = 128


class MlhError(RuntimeError):
    def __init__(self, status, msg=""):
        self.status = status
        super().__init__("%s: %s" % (STATUS_NAMES.get(status, status), msg))


class FriProofC(ctypes.Structure):
    _fields_ = [
        ("log_code", ctypes.c_uint32),
        ("num_trees", ctypes.c_uint32),
        ("num_queries", ctypes.c_uint32),
        ("commitments", ctypes.c_void_p),
        ("last_elem", ctypes.c_uint8 * 16),
        ("last_random", ctypes.c_uint8 * 32),
        ("query_indices", ctypes.c_void_p),
        ("queries", ctypes.c_void_p),
    ]


class PcsProofC(ctypes.Structure):
    _fields_ = [("fri", FriProofC), ("sumcheck_polys", ctypes.c_void_p)]


class BatchedFriProofC(ctypes.Structure):
    _fields_ = [
        ("log_code", ctypes.c_uint32),
        ("num_codes", ctypes.c_uint32),
        ("num_trees", ctypes.c_uint32),
        ("num_queries", ctypes.c_uint32),
        ("batch_commitment", ctypes.c_uint8 * 32),
        ("commitments", ctypes.c_void_p),
        ("last_elem", ctypes.c_uint8 * 16),
        ("last_random", ctypes.c_uint8 * 32),
        ("query_indices", ctypes.c_void_p),
        ("queries", ctypes.c_void_p),
    ]


class BatchedPcsProofC(ctypes.Structure):
    _fields_ = [("fri", BatchedFriProofC), ("sumcheck_polys", ctypes.c_void_p)]


# mlh_transport (include/mlhip.h): collectives as C callbacks
ALL_TO_ALL_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_uint64, ctypes.c_void_p)
ALL_GATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_uint64, ctypes.c_void_p)


class TransportC(ctypes.Structure):
    _fields_ = [
        ("world", ctypes.c_uint32),
        ("rank", ctypes.c_uint32),
        ("host_side", ctypes.c_uint32),
        ("user", ctypes.c_void_p),
        ("all_to_all", ALL_TO_ALL_FN),
        ("all_gather", ALL_GATHER_FN),
    ]


_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I = ctypes.c_int
_S = ctypes.c_size_t

# name -> (restype, argtypes)
SIGNATURES = {
    "mlh_version": (ctypes.c_char_p, []),
    "mlh_context_create": (_I, [_I, _P, ctypes.POINTER(_P)]),
    "mlh_context_destroy": (None, [_P]),
    "mlh_set_stream": (_I, [_P, _P]),
    "mlh_set_ntt_plan": (_I, [_P, ctypes.POINTER(ctypes.c_uint32), _U32]),
    "mlh_set_coop_spin_limit": (_I, [_P, _U32]),
    "mlh_set_pcs_fused_max": (_I, [_P, _U32]),
    "mlh_set_table_cache_limit": (_I, [_P, ctypes.c_uint64]),
    "mlh_table_cache_bytes": (ctypes.c_uint64, [_P]),
    "mlh_synchronize": (_I, [_P]),
    "mlh_last_error": (ctypes.c_char_p, [_P]),
    "mlh_malloc": (_I, [_P, _S, ctypes.POINTER(_P)]),
    "mlh_free": (_I, [_P, _P]),
    "mlh_memcpy_h2d": (_I, [_P, _P, _P, _S]),
    "mlh_memcpy_d2h": (_I, [_P, _P, _P, _S]),
    "mlh_memcpy_d2d": (_I, [_P, _P, _P, _S]),
    "mlh_pow_2_generator": (_I, [_U32, _P]),
    "mlh_pow_2_generator_powers": (_I, [_P, _U32, _P]),
    "mlh_field_add": (_I, [_P, _P, _P, _P, _U64]),
    "mlh_field_sub": (_I, [_P, _P, _P, _P, _U64]),
    "mlh_field_mul": (_I, [_P, _P, _P, _P, _U64]),
    "mlh_field_neg": (_I, [_P, _P, _P, _U64]),
    "mlh_field_scale": (_I, [_P, _P, _P, _P, _U64]),
    "mlh_ntt": (_I, [_P, _P, _P, _U32, _P]),
    "mlh_intt": (_I, [_P, _P, _P, _U32, _P]),
    "mlh_bit_reverse_permutation": (_I, [_P, _P, _P, _U32]),
    "mlh_ntt_host": (_I, [_P, _P, _P, _U32, _P, _I]),
    "mlh_reed_solomon": (_I, [_P, _P, _U32, _P, _P]),
    "mlh_reed_solomon_brev": (_I, [_P, _P, _U32, _P, _P]),
    "mlh_merkle_layers_bytes": (_U64, [_U64]),
    "mlh_merkle_commit_pairs": (_I, [_P, _P, _U32, _P, _P]),
    "mlh_merkle_commit": (_I, [_P, _P, _U64, _U64, _P, _P]),
    "mlh_merkle_batch_commit": (_I, [_P, _P, _U64, _U32, _U64, _P, _P]),
    "mlh_fri_fold": (_I, [_P, _P, _U32, _U32, _U32, _P, _P]),
    "mlh_fri_prover_init": (_I, [_P, _P, _U32, _P, ctypes.POINTER(_P)]),
    "mlh_fri_prover_fold_step": (_I, [_P, _P, _U32, _P, _P]),
    "mlh_fri_prover_fold_step_gp": (_I, [_P, _P, _P, _U32, _U32, _P, _P]),
    "mlh_fri_prover_fold": (_I, [_P, _P, _U32, _P, ctypes.POINTER(_P)]),
    "mlh_fri_prover_init_gp": (_I, [_P, _P, _U32, _P, _U32, _P, ctypes.POINTER(_P)]),
    "mlh_fri_prover_fold_gp": (_I, [_P, _P, _U32, _P, _U32, _P, ctypes.POINTER(_P)]),
    "mlh_fri_prover_num_trees": (_U32, [_P]),
    "mlh_fri_prover_roots": (_I, [_P, _P]),
    "mlh_fri_prover_last_element": (_I, [_P, _P]),
    "mlh_fri_prover_open_query": (_I, [_P, _P, _U64, _P]),
    "mlh_fri_prover_open_queries": (_I, [_P, _P, _P, _U32, _P]),
    "mlh_fri_prover_destroy": (None, [_P]),
    "mlh_fri_query_bytes": (_U64, [_U32]),
    "mlh_fri_prove": (_I, [_P, _P, _U32, _P, ctypes.POINTER(FriProofC)]),
    "mlh_fri_prove_gp": (_I, [_P, _P, _U32, _P, _U32, _P, ctypes.POINTER(FriProofC)]),
    "mlh_fri_verify": (_I, [ctypes.POINTER(FriProofC)]),
    "mlh_fri_proof_encoded_size": (_U64, [ctypes.POINTER(FriProofC)]),
    "mlh_fri_proof_encode": (_I, [ctypes.POINTER(FriProofC), _P, _U64]),
    "mlh_fri_proof_decode_header": (_I, [_P, _U64, ctypes.POINTER(_U32), ctypes.POINTER(_U32)]),
    "mlh_fri_proof_decode": (_I, [_P, _U64, ctypes.POINTER(FriProofC)]),
    "mlh_shard_ntt_cross": (_I, [_P, _P, _P, _U32, _U32, _U32, _P, _I]),
    "mlh_shard_fri_fold": (_I, [_P, _P, _U32, _U32, _U32, _P, _P, _U32, _U32, _U32]),
    "mlh_shard_fri_fold_commit": (_I, [_P, _P, _U32, _U32, _U32, _P, _P, _P, _U32, _U32, _U32]),
    "mlh_merkle_open_pairs": (_I, [_P, _P, _U32, _P, _U32, _P, _U32, _P]),
    "mlh_merkle_open": (_I, [_P, _P, _U64, _P, _U32, _P]),
    "mlh_merkle_verify": (_I, [_P, _U64, _P, _U32, _U64, _P, _U64]),
    "mlh_batched_fri_query_bytes": (_U64, [_U32, _U32]),
    "mlh_batched_fri_prove": (_I, [_P, _P, _U32, _U32, _P, ctypes.POINTER(BatchedFriProofC)]),
    "mlh_batched_fri_prover_init": (_I, [_P, _P, _U32, _U32, _P, ctypes.POINTER(_P)]),
    "mlh_batched_fri_prover_fold_step_gp": (_I, [_P, _P, _P, _U32, _P, _P]),
    "mlh_batched_fri_prover_inner": (_P, [_P]),
    "mlh_batched_fri_prover_batch_root": (_I, [_P, _P]),
    "mlh_batched_fri_prover_fingerprint_r": (_I, [_P, _P]),
    "mlh_batched_fri_prover_open_query": (_I, [_P, _P, ctypes.c_uint64, _P]),
    "mlh_batched_fri_prover_destroy": (None, [_P]),
    "mlh_batched_fri_verify": (_I, [ctypes.POINTER(BatchedFriProofC)]),
    "mlh_batched_pcs_prove": (_I, [_P, _P, _U32, _U32, _P, _P, _P,
                                   ctypes.POINTER(BatchedPcsProofC)]),
    "mlh_batched_pcs_verify": (_I, [ctypes.POINTER(BatchedPcsProofC), _U32, _P, _P, _P]),
    "mlh_device_transcript_bytes": (_U64, []),
    "mlh_transcript_to_device": (_I, [_P, _P, _P]),
    "mlh_transcript_from_device": (_I, [_P, _P, _P]),
    "mlh_device_transcript_absorb": (_I, [_P, _P, _P, _U32, _P]),
    "mlh_device_fri_last": (_I, [_P, _P, _P, _P, _P]),
    "mlh_shard_fri_fold_dr": (_I, [_P, _P, _U32, _U32, _U32, _P, _P, _U32, _U32, _U32]),
    "mlh_shard_fri_fold_commit_dr": (_I, [_P, _P, _U32, _U32, _U32, _P, _P, _P, _U32, _U32, _U32]),
    "mlh_merkle_top": (_I, [_P, _P, _U32, _U64, _P]),
    "mlh_sumcheck_sums_dev": (_I, [_P, _P, _P, _U32, _P]),
    "mlh_sumcheck_fold_sums_dr": (_I, [_P, _P, _P, _U32, _P, _P]),
    "mlh_sumcheck_fold_dr": (_I, [_P, _P, _P, _U32, _P]),
    "mlh_device_sumcheck_round": (_I, [_P, _P, _U32, _P, _P, _P, _P]),
    "mlh_transcript_create": (_I, [ctypes.POINTER(_P)]),
    "mlh_transcript_clone": (_I, [_P, ctypes.POINTER(_P)]),
    "mlh_transcript_destroy": (None, [_P]),
    "mlh_transcript_absorb": (_I, [_P, _P, _U64]),
    "mlh_transcript_random": (_I, [_P, _P]),
    "mlh_transcript_next_challenge": (_I, [_P, _P]),
    "mlh_mle_to_coefficient": (_I, [_P, _P, _U32]),
    "mlh_mle_to_evaluation": (_I, [_P, _P, _U32]),
    "mlh_eq_table": (_I, [_P, _P, _U32, _P]),
    "mlh_mle_coeffs_evaluate": (_I, [_P, _P, _U32, _P, _P]),
    "mlh_poly_evaluate": (_I, [_P, _P, _U64, _P, _P]),
    "mlh_trace_evaluate": (_I, [_P, _P, _U32, _U32, _P, _P]),
    "mlh_mle_evaluate": (_I, [_P, _P, _U32, _P, _P]),
    "mlh_sumcheck_partial_sums": (_I, [_P, _P, _P, _U32, _P]),
    "mlh_sumcheck_fold": (_I, [_P, _P, _P, _U32, _P]),
    "mlh_sumcheck_fold_and_sums": (_I, [_P, _P, _P, _U32, _P, _P]),
    "mlh_sumcheck_prove": (_I, [_P, _P, _P, _U32, _P, _P, _P, _P]),
    "mlh_sumcheck_prove_eq": (_I, [_P, _P, _P, _U32, _P, _P, _P, _P, _P, _P]),
    "mlh_pcs_prove": (_I, [_P, _P, _U32, _P, _P, _P, ctypes.POINTER(PcsProofC)]),
    "mlh_pcs_verify": (_I, [ctypes.POINTER(PcsProofC), _U32, _P, _P, _P]),
    "mlh_bench_ntt": (_I, [_P, _P, _U32, _U32, ctypes.POINTER(ctypes.c_float)]),
    "mlh_profile_enable": (_I, [_P, _I]),
    "mlh_profile_reset": (_I, [_P]),
    "mlh_profile_get": (_I, [_P, ctypes.c_char_p, ctypes.POINTER(_U64), ctypes.POINTER(ctypes.c_double)]),
    "mlh_comm_unique_id": (_I, [_P]),
    "mlh_comm_create": (_I, [_P, _U32, _U32, _P, ctypes.POINTER(_P)]),
    "mlh_comm_destroy": (None, [_P]),
    "mlh_comm_transport": (_I, [_P, ctypes.POINTER(TransportC)]),
    "mlh_comm_info": (_I, [_P, ctypes.POINTER(_U32), ctypes.POINTER(_U32), ctypes.POINTER(ctypes.c_int)]),
    "mlh_comm_preflight": (_I, [_P, ctypes.POINTER(TransportC), ctypes.c_uint64,
                                ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_float)]),
    "mlh_sharded_ntt": (_I, [_P, ctypes.POINTER(TransportC), _P, _P, _U32, _P, _I]),
    "mlh_gen_pows_params": (_I, [_P, _U64, _P, ctypes.POINTER(_U32)]),
    "mlh_gen_pows_verify": (_I, [_P, _P, _U64, _P, ctypes.POINTER(_U32)]),
    "mlh_sharded_ntt_batch": (_I, [_P, ctypes.POINTER(TransportC), ctypes.POINTER(_P),
                                   ctypes.POINTER(_P), _U32, _U32, _P, _I]),
    "mlh_sharded_ntt_fused_batch": (_I, [_P, ctypes.POINTER(TransportC), ctypes.POINTER(_P),
                                         ctypes.POINTER(_P), _U32, _U32, _P, ctypes.POINTER(_U32)]),
    "mlh_sharded_reed_solomon": (_I, [_P, ctypes.POINTER(TransportC), _P, _U32, _P, _P]),
    "mlh_sharded_commit_rs_code": (_I, [_P, ctypes.POINTER(TransportC), _P, _U32, _P]),
    "mlh_sharded_fri_prove": (_I, [_P, ctypes.POINTER(TransportC), _P, _U32, _U32, _P,
                                   ctypes.POINTER(FriProofC)]),
    "mlh_sharded_eq_table": (_I, [_P, ctypes.POINTER(TransportC), _P, _U32, _P]),
    "mlh_sharded_sumcheck_prove": (_I, [_P, ctypes.POINTER(TransportC), _P, _P, _U32, _P, _P, _P, _P]),
}

_lib = None


def load():
    """Load libmlhip.so once; raises if it is missing (no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libmlhip.so not built at %s -- run `python -c 'import __graft_entry__ as g; g.build()'`"
            % LIB_PATH
        )
    # torch first: its wheel bundles its own HIP runtime (libamdhip64.so.7, the
    # same soname as /opt/rocm's), and a process must hold ONE of them.  Loaded
    # before torch, libmlhip would bind /opt/rocm's runtime while torch maps its
    # own beside it, and that second runtime sees no device.
    import torch  # noqa: F401

    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
