"""multilinear_amd -- MI355X-native (gfx950) backend for the proving hot path
of fr34za/multilinear: NTT/INTT, Reed-Solomon LDE, SHA-256 Merkle commit, FRI
folding and MLE/sumcheck rounds over the field.rs prime, behind the C ABI in
include/mlhip.h (libmlhip.so).

The Python modules mirror the reference's public API names (src/ntt,
src/fri, src/merkle_tree, src/polynomials.rs, sumcheck, multilinear_pcs) so
the parity tests read like the reference's own tests; they are thin ctypes
wrappers -- all compute runs in the HIP kernels of libmlhip.so.
"""
from . import _lib

__all__ = ["_lib"]
