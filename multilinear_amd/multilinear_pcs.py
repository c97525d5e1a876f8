"""PCSProof (src/fri/multilinear_pcs.rs:78-190) on the MI355X."""
import ctypes

from . import _lib
from .device import check, context, fe_bytes, fe_from_bytes, lib, ptr
from .fri import FriProof
from .polynomials import _points


class PCSProof:
    def __init__(self, n_vars):
        self.n_vars = n_vars
        self.fri_proof = FriProof(n_vars + _lib.LOG_BLOWUP)
        self._polys = (ctypes.c_uint8 * (32 * n_vars))()
        self.c = _lib.PcsProofC()
        self.c.fri = self.fri_proof.c
        self.c.sumcheck_polys = ctypes.cast(self._polys, ctypes.c_void_p)
        self.inputs = None
        self.output = None

    @staticmethod
    def prove(inputs, output, evals, transcript, device=0):
        """PCSProof::prove (multilinear_pcs.rs:90-136); evals: device tensor."""
        n = len(inputs)
        assert evals.shape[0] == 1 << n
        ctx = context(device)
        p = PCSProof(n)
        check(lib().mlh_pcs_prove(ctx, ptr(evals), n, _points(inputs), fe_bytes(output),
                                  transcript.h, ctypes.byref(p.c)), ctx)
        # the fri struct inside p.c was filled in place; mirror it
        p.fri_proof.c = p.c.fri
        p.inputs = list(inputs)
        p.output = output
        return p

    @property
    def sumcheck_polynomials(self):
        raw = bytes(self._polys)
        return [(fe_from_bytes(raw[32 * k:32 * k + 16]), fe_from_bytes(raw[32 * k + 16:32 * k + 32]))
                for k in range(self.n_vars)]

    def verify(self, transcript):
        """PCSProof::verify (multilinear_pcs.rs:138-190), host side in libmlhip."""
        st = lib().mlh_pcs_verify(ctypes.byref(self.c), self.n_vars, _points(self.inputs),
                                  fe_bytes(self.output), transcript.h)
        return st == 0
