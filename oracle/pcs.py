"""Multilinear PCS prove / verify (oracle).  Test infrastructure only.

Reference: src/fri/multilinear_pcs.rs:22-190.
"""
from . import field as F
from .fri import LOG_BLOWUP, NUM_QUERIES, FriProof, FriProverData, query_index, reed_solomon
from .ntt import bit_reverse_permutation
from .polynomials import to_coefficient, uni_evaluate
from .sumcheck import SumcheckTables, delta_evaluate, to_polynomial


class PCSProof:
    def __init__(self, fri_proof, sumcheck_polynomials, inputs, output):
        self.fri_proof = fri_proof
        self.sumcheck_polynomials = sumcheck_polynomials
        self.inputs = inputs
        self.output = output

    @staticmethod
    def prove(inputs, output, evals, transcript):
        """PCSProof::prove (multilinear_pcs.rs:90-136)."""
        log_domain = (len(evals).bit_length() - 1) + LOG_BLOWUP
        gen_pows = F.pow_2_generator_powers(log_domain)
        gen = gen_pows[1]
        coeffs = to_coefficient(evals)
        bit_reverse_permutation(coeffs)
        code = reed_solomon(coeffs, gen)
        # PCSProverData::fold (multilinear_pcs.rs:43-76)
        fri = FriProverData.init(code, transcript)
        tables = SumcheckTables.build_tables_for_pcs(inputs, evals)
        num_steps = (len(code).bit_length() - 1) - LOG_BLOWUP
        prev = output
        polys = []
        for k in range(num_steps):
            nz, r, prev = tables.compute_sumcheck_polynomial(prev, transcript, 2)
            polys.append(nz)
            fri.fold_step(gen_pows, k, r, transcript)
        assert fri.last_element is not None
        domain_size = 1 << log_domain
        queries = []
        for _ in range(NUM_QUERIES):
            idx = query_index(transcript, domain_size)
            queries.append(fri.open_query_at(idx))
            transcript.absorb(idx.to_bytes(8, "little"))
        fp = FriProof(fri.fold_roots(), queries, fri.last_element, transcript.random())
        return PCSProof(fp, polys, list(inputs), output)

    def verify(self, transcript):
        """PCSProof::verify (multilinear_pcs.rs:138-190)."""
        fp = self.fri_proof
        if len(fp.queries) != NUM_QUERIES:
            return False
        n = len(fp.commitments)
        assert n == len(self.sumcheck_polynomials) == len(self.inputs)
        rs = []
        for root, poly in zip(fp.commitments, self.sumcheck_polynomials):
            transcript.absorb(root)
            for c in poly:
                transcript.absorb(F.to_bytes(c))
            rs.append(transcript.next_challenge())
        transcript.absorb(F.to_bytes(fp.last_elem))
        pol = to_polynomial(self.sumcheck_polynomials[0], self.output)
        for sp, r in zip(self.sumcheck_polynomials[1:], rs):
            pol = to_polynomial(sp, uni_evaluate(pol, r))
        r = rs[-1]
        delta = delta_evaluate(self.inputs, rs)
        if delta * fp.last_elem % F.M != uni_evaluate(pol, r):
            return False
        return fp.verify_queries(transcript, rs)
