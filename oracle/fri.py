"""FRI commit / fold / prove / verify (oracle).  Test infrastructure only.

Reference: src/fri/mod.rs.  LOG_BLOWUP = 1, NUM_QUERIES = 128 (:16-17).
"""
from . import field as F
from . import merkle as MK
from .ntt import ntt
from .transcript import Transcript

LOG_BLOWUP = 1
NUM_QUERIES = 128
INV2 = F.inv(2)


def reed_solomon(coeffs, gen):
    """fri/mod.rs:19-28: zero-pad to 2N, NTT with gen (order 2N)."""
    n = len(coeffs)
    return ntt(list(coeffs) + [0] * ((1 << LOG_BLOWUP) * n - n), gen)


def pair_bytes(value, minus_value) -> bytes:
    """ReedSolomonPair as_ref (fri/mod.rs:30-43): repr(C) {value, minus_value}."""
    return F.to_bytes(value) + F.to_bytes(minus_value)


def commit_rs_code(code):
    """fri/mod.rs:45-55: pairs (code[i], code[i + n/2]) -> Merkle."""
    h = len(code) // 2
    pairs = [(code[i], code[i + h]) for i in range(h)]
    tree = MK.Merkle.commit([pair_bytes(a, b) for a, b in pairs])
    tree.pairs = pairs
    return tree


def fold_layer(pairs, gen_pows, k, r):
    """The fold loop of FriProverData::fold_step (fri/mod.rs:89-114):
    next[i] = ((a+b) + r*(a-b)*gen_pows[len - i*2^k]) * 1/2, i=0 special."""
    L = len(gen_pows)
    out = []
    for i, (a, b) in enumerate(pairs):
        tw = 1 if i == 0 else gen_pows[L - i * (1 << k)]
        odd = (a - b) * tw % F.M
        out.append(((a + b) + r * odd) * INV2 % F.M)
    return out


class FriProverData:
    def __init__(self, trees, last_element):
        self.merkle_trees = trees
        self.last_element = last_element

    @staticmethod
    def init(code, transcript):  # fri/mod.rs:58-76
        n = len(code)
        assert n & (n - 1) == 0, "Input size must be a power of two"
        tree = commit_rs_code(code)
        transcript.absorb(tree.root())
        return FriProverData([tree], None)

    def fold_step(self, gen_pows, k, r, transcript):  # fri/mod.rs:79-134
        last = self.merkle_trees[-1].pairs
        n = 2 * len(last)
        blowup = 1 << LOG_BLOWUP
        if n <= blowup:
            return
        half_n = n >> 1
        nxt = fold_layer(last, gen_pows, k, r)
        if half_n == blowup:
            first = nxt[0]
            assert all(x == first for x in nxt), "not an RS code"
            self.last_element = first
            transcript.absorb(F.to_bytes(first))
            return
        tree = commit_rs_code(nxt)
        self.merkle_trees.append(tree)
        transcript.absorb(tree.root())

    @staticmethod
    def fold(gen_pows, code, transcript):  # fri/mod.rs:136-145
        pd = FriProverData.init(code, transcript)
        num_steps = (len(code).bit_length() - 1) - LOG_BLOWUP
        for k in range(num_steps):
            r = transcript.next_challenge()
            pd.fold_step(gen_pows, k, r, transcript)
        assert pd.last_element is not None
        return pd

    def fold_roots(self):  # fri/mod.rs:147-152
        return [t.root() for t in self.merkle_trees]

    def open_query_at(self, index):  # fri/mod.rs:154-175
        n = len(self.merkle_trees[0].data)
        assert index < n
        paths = []
        cur, cur_n = index, n
        for tree in self.merkle_trees:
            paths.append(tree.open(cur))
            cur_n //= 2
            cur %= cur_n
        return paths


def query_index(transcript, domain_size):
    """fri/mod.rs:268-277: u64_le(random()[..8]) % (domain_size/2), absorbed
    as usize LE (8 bytes)."""
    idx = int.from_bytes(transcript.random()[:8], "little") % (domain_size // 2)
    return idx


class FriProof:
    def __init__(self, commitments, queries, last_elem, last_random):
        self.commitments = commitments
        self.queries = queries
        self.last_elem = last_elem
        self.last_random = last_random

    @staticmethod
    def prove(code, gen_pows, transcript):  # fri/mod.rs:261-285
        domain_size = len(code)
        pd = FriProverData.fold(gen_pows, code, transcript)
        queries = []
        for _ in range(NUM_QUERIES):
            idx = query_index(transcript, domain_size)
            queries.append(pd.open_query_at(idx))
            transcript.absorb(idx.to_bytes(8, "little"))
        return FriProof(pd.fold_roots(), queries, pd.last_element, transcript.random())

    def verify(self):  # fri/mod.rs:287-309
        if len(self.queries) != NUM_QUERIES:
            return False
        tr = Transcript()
        rs = []
        for root in self.commitments:
            tr.absorb(root)
            rs.append(tr.next_challenge())
        tr.absorb(F.to_bytes(self.last_elem))
        return self.verify_queries(tr, rs)

    def verify_queries(self, tr, rs):  # fri/mod.rs:311-340
        log_domain = len(self.commitments) + LOG_BLOWUP
        domain_size = 1 << log_domain
        gen = F.pow_2_generator(log_domain)
        for q in self.queries:
            n = domain_size // 2
            idx = query_index(tr, domain_size)
            tr.absorb(idx.to_bytes(8, "little"))
            if not verify_query(q, self.commitments, self.last_elem, n, idx, gen, rs):
                return False
        return self.last_random == tr.random()


def verify_query(paths, commitments, last_element, n, index, gen, rs):
    """QueryProof::verify (fri/mod.rs:184-236)."""
    if len(paths) != len(commitments):
        return False
    cur_n, cur_idx, cur_gen = n, index, gen
    for i, (value, path) in enumerate(paths):
        if not MK.verify(value, path, commitments[i], cur_idx):
            return False
        v = F.from_bytes(value[:16])
        mv = F.from_bytes(value[16:32])
        gp = F.fpow(cur_gen, cur_idx)
        even = F.div(v + mv, 2)
        odd = F.div(v - mv, F.mul(2, gp))
        folded = (even + rs[i] * odd) % F.M
        if i == len(paths) - 1:
            return last_element == folded
        nxt_idx = cur_idx % (cur_n // 2)
        nv, _ = paths[i + 1]
        nxt_val = F.from_bytes(nv[:16]) if nxt_idx == cur_idx else F.from_bytes(nv[16:32])
        if nxt_val != folded:
            return False
        cur_gen = F.mul(cur_gen, cur_gen)
        cur_n //= 2
        cur_idx = nxt_idx
    return True
