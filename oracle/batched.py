"""Batched FRI and batched multilinear PCS (oracle).  Test infrastructure only.

Reference: src/fri/batched_fri.rs:9-363 and src/fri/batched_pcs.rs:14-250.
* fingerprint(r, c_0..c_{m-1}) is Horner: ((c_0 r + c_1) r + ...) + c_{m-1}
  = sum_j c_j r^(m-1-j)  (batched_fri.rs:30-38; the comment there says
  c_0 + r c_1 + ..., which is NOT what the loop computes);
* the batch layer is Merkle::batch_commit of the per-code RS pairs: leaf i =
  SHA256(pair_0[i] || pair_1[i] || ...) (merkle_tree/mod.rs:92-131);
* after its root: fingerprint_r = next_challenge(), absorb LE16(fingerprint_r)
  (batched_fri.rs:82-89); the first fold runs on the fingerprinted pairs
  (batched_fold_step, :92-176), all later folds are ordinary fold_steps on the
  inner FriProverData, whose first tree is the folded layer.
"""
from . import field as F
from . import merkle as MK
from .fri import (LOG_BLOWUP, NUM_QUERIES, FriProverData, commit_rs_code, fold_layer, pair_bytes,
                  query_index, reed_solomon, verify_query)
from .ntt import bit_reverse_permutation
from .polynomials import to_coefficient
from .sumcheck import SumcheckTables, delta_evaluate, to_polynomial
from .transcript import Transcript

INV2 = F.inv(2)


def fingerprint(r, coeffs):
    """batched_fri.rs:30-38 (Horner)."""
    acc = 0
    for c in coeffs:
        acc = (acc * r + c) % F.M
    return acc


class BatchedFriProverData:
    def __init__(self, batch_layer, fingerprint_r, fri_data):
        self.batch_layer = batch_layer
        self.fingerprint_r = fingerprint_r
        self.fri_data = fri_data

    @staticmethod
    def init(codes, transcript):  # batched_fri.rs:41-98
        assert codes
        n = len(codes[0])
        assert n & (n - 1) == 0 and all(len(c) == n for c in codes)
        h = n // 2
        pairs = [[(c[i], c[i + h]) for i in range(h)] for c in codes]
        layer = MK.Merkle.batch_commit([[pair_bytes(a, b) for a, b in p] for p in pairs])
        layer.pairs = pairs
        transcript.absorb(layer.root())
        fr = transcript.next_challenge()
        transcript.absorb(F.to_bytes(fr))
        return BatchedFriProverData(layer, fr, FriProverData([], None))

    def batched_fold_step(self, gen_pows, r, transcript):  # batched_fri.rs:100-176
        pairs = self.batch_layer.pairs
        n = 2 * len(pairs[0])
        if n <= (1 << LOG_BLOWUP):
            return
        half_n = n // 2
        fp = [(fingerprint(self.fingerprint_r, [p[i][0] for p in pairs]),
               fingerprint(self.fingerprint_r, [p[i][1] for p in pairs])) for i in range(half_n)]
        nxt = fold_layer(fp, gen_pows, 0, r)
        if half_n == (1 << LOG_BLOWUP):
            assert all(x == nxt[0] for x in nxt), "not an RS code"
            self.fri_data.last_element = nxt[0]
            transcript.absorb(F.to_bytes(nxt[0]))
            return
        tree = commit_rs_code(nxt)
        self.fri_data.merkle_trees.append(tree)
        transcript.absorb(tree.root())

    @staticmethod
    def fold(gen_pows, codes, transcript):  # batched_fri.rs:178-205
        pd = BatchedFriProverData.init(codes, transcript)
        steps = (len(codes[0]).bit_length() - 1) - LOG_BLOWUP
        pd.batched_fold_step(gen_pows, transcript.next_challenge(), transcript)
        for k in range(1, steps):
            pd.fri_data.fold_step(gen_pows, k, transcript.next_challenge(), transcript)
        assert pd.fri_data.last_element is not None
        return pd

    def open_query_at(self, index):  # batched_fri.rs:207-224
        value, path = MK.batch_open(self.batch_layer, index)
        n = len(self.batch_layer.data[0]) // 2
        inner = self.fri_data.open_query_at(index % n) if self.fri_data.merkle_trees else []
        return (value, path), inner


class BatchedFriProof:
    def __init__(self, batch_commitment, commitments, queries, last_elem, last_random):
        self.batch_commitment = batch_commitment
        self.commitments = commitments
        self.queries = queries
        self.last_elem = last_elem
        self.last_random = last_random

    @staticmethod
    def prove(codes, gen_pows, transcript):  # batched_fri.rs:280-311
        domain = len(codes[0])
        pd = BatchedFriProverData.fold(gen_pows, codes, transcript)
        queries = []
        for _ in range(NUM_QUERIES):
            idx = query_index(transcript, domain)
            queries.append(pd.open_query_at(idx))
            transcript.absorb(idx.to_bytes(8, "little"))
        return BatchedFriProof(pd.batch_layer.root(), pd.fri_data.fold_roots(), queries,
                               pd.fri_data.last_element, transcript.random())

    def verify(self):  # batched_fri.rs:313-343
        tr = Transcript()
        tr.absorb(self.batch_commitment)
        fr = tr.next_challenge()
        tr.absorb(F.to_bytes(fr))
        rs = [tr.next_challenge()]
        for c in self.commitments:
            tr.absorb(c)
            rs.append(tr.next_challenge())
        tr.absorb(F.to_bytes(self.last_elem))
        return self.verify_queries(tr, rs, fr)

    def verify_queries(self, tr, rs, fr):  # batched_fri.rs:345-388
        if len(self.queries) != NUM_QUERIES:
            return False
        log_domain = len(self.commitments) + 1 + LOG_BLOWUP
        domain = 1 << log_domain
        gen = F.pow_2_generator(log_domain)
        for q in self.queries:
            n = domain // 2
            idx = query_index(tr, domain)
            if not verify_batched_query(q, self, n, idx, gen, rs, fr):
                return False
            tr.absorb(idx.to_bytes(8, "little"))
        return self.last_random == tr.random()


def verify_batched_query(q, proof, n, index, gen, rs, fr):  # batched_fri.rs:226-278
    (value, path), inner = q
    if len(inner) != len(proof.commitments):
        return False
    if not MK.batch_verify(value, path, proof.batch_commitment, index):
        return False
    v = fingerprint(fr, [F.from_bytes(p[:16]) for p in value])
    mv = fingerprint(fr, [F.from_bytes(p[16:32]) for p in value])
    gp = F.fpow(gen, index)
    even = F.div(v + mv, 2)
    odd = F.div(v - mv, F.mul(2, gp))
    folded = (even + rs[0] * odd) % F.M
    if not inner:
        return proof.last_elem == folded
    nxt_idx = index % (n // 2)
    nv, _ = inner[0]
    nxt_val = F.from_bytes(nv[:16]) if nxt_idx == index else F.from_bytes(nv[16:32])
    if nxt_val != folded:
        return False
    return verify_query(inner, proof.commitments, proof.last_elem, n // 2, nxt_idx,
                        F.mul(gen, gen), rs[1:])


class BatchedPCSProof:
    def __init__(self, fri_proof, sumcheck_polynomials, inputs, outputs):
        self.fri_proof = fri_proof
        self.sumcheck_polynomials = sumcheck_polynomials
        self.inputs = inputs
        self.outputs = outputs

    @staticmethod
    def prove(inputs, outputs, polys, transcript):  # batched_pcs.rs:127-180
        log_domain = (len(polys[0]).bit_length() - 1) + LOG_BLOWUP
        gen_pows = F.pow_2_generator_powers(log_domain)
        codes = []
        for p in polys:
            c = to_coefficient(p)
            bit_reverse_permutation(c)
            codes.append(reed_solomon(c, gen_pows[1]))
        # BatchedPCSProverData::init (:36-78)
        for x in inputs:
            transcript.absorb(F.to_bytes(x))
        for y in outputs:
            transcript.absorb(F.to_bytes(y))
        fri = BatchedFriProverData.init(codes, transcript)
        fr = fri.fingerprint_r
        fp = [fingerprint(fr, [p[i] for p in polys]) for i in range(len(polys[0]))]
        tables = SumcheckTables.build_tables_for_pcs(inputs, fp)
        # fold (:80-125)
        steps = (len(codes[0]).bit_length() - 1) - LOG_BLOWUP
        prev = fingerprint(fr, outputs)
        sc = []
        for k in range(steps):
            nz, r, prev = tables.compute_sumcheck_polynomial(prev, transcript, 2)
            sc.append(nz)
            if k == 0:
                fri.batched_fold_step(gen_pows, r, transcript)
            else:
                fri.fri_data.fold_step(gen_pows, k, r, transcript)
        assert fri.fri_data.last_element is not None
        domain = 1 << log_domain
        queries = []
        for _ in range(NUM_QUERIES):
            idx = query_index(transcript, domain)
            queries.append(fri.open_query_at(idx))
            transcript.absorb(idx.to_bytes(8, "little"))
        proof = BatchedFriProof(fri.batch_layer.root(), fri.fri_data.fold_roots(), queries,
                                fri.fri_data.last_element, transcript.random())
        return BatchedPCSProof(proof, sc, list(inputs), list(outputs))

    def verify(self, transcript):  # batched_pcs.rs:182-250
        fp = self.fri_proof
        if len(fp.queries) != NUM_QUERIES:
            return False
        n = len(fp.commitments) + 1
        assert n == len(self.sumcheck_polynomials) == len(self.inputs)
        for x in self.inputs:
            transcript.absorb(F.to_bytes(x))
        for y in self.outputs:
            transcript.absorb(F.to_bytes(y))
        fr, rs = 0, []
        for i, poly in enumerate(self.sumcheck_polynomials):
            if i == 0:
                transcript.absorb(fp.batch_commitment)
                fr = transcript.next_challenge()
                transcript.absorb(F.to_bytes(fr))
            else:
                transcript.absorb(fp.commitments[i - 1])
            for c in poly:
                transcript.absorb(F.to_bytes(c))
            rs.append(transcript.next_challenge())
        transcript.absorb(F.to_bytes(fp.last_elem))
        pol = to_polynomial(self.sumcheck_polynomials[0], fingerprint(fr, self.outputs))
        for sp, r in zip(self.sumcheck_polynomials[1:], rs):
            pol = to_polynomial(sp, uni(pol, r))
        delta = delta_evaluate(self.inputs, rs)
        if delta * fp.last_elem % F.M != uni(pol, rs[-1]):
            return False
        return fp.verify_queries(transcript, rs, fr)


def uni(coeffs, x):
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % F.M
    return acc
