"""CPU stand-in for tests/dist_spec.HipOps (test infrastructure only).

Lets the gloo world_size>1 CPU tests drive the real sharded orchestration
(tests/dist_spec.py: layouts, all-to-all / all-gather exchanges, subtree
root combination, query ownership) with every rank-local step computed by the
oracle: C-oracle NTT / RS / Merkle, and the defining formulas of the
cross-shard DFT and the index-mapped fold written out in Python ints."""
import numpy as np
import torch

from tests import dist_spec as D
from oracle import coracle as C
from oracle import field as F

INV2 = F.inv(2)


def _ints(t):
    a = t.contiguous().numpy().view(np.uint32).reshape(-1, 4)
    return F.from_limbs(a)


def _tensor(vals):
    return torch.from_numpy(F.to_limbs(vals).view(np.int32).reshape(-1, 4).copy())


def _limbs(t):
    return t.contiguous().numpy().view(np.uint32).reshape(-1, 4)


class CpuOps(D.HipOps):
    def __init__(self):
        super().__init__(device=None)

    def empty(self, n):
        return torch.zeros((n, 4), dtype=torch.int32)

    def ntt(self, x, gen, inverse=False):
        n = x.shape[0]
        return torch.from_numpy(C.ntt(_limbs(x), n.bit_length() - 1, gen, inverse).view(np.int32))

    def reed_solomon(self, coeffs, gen):
        n = coeffs.shape[0]
        return torch.from_numpy(C.reed_solomon(_limbs(coeffs), n.bit_length() - 1, gen).view(np.int32))

    def cross(self, x, log_n, log_p, rank, gen, inverse):
        P = 1 << log_p
        S = 1 << (log_n - 2 * log_p)
        rows = _ints(x)
        w = F.inv(gen) if inverse else gen
        wP = F.fpow(w, 1 << (log_n - log_p))
        out = [0] * (P * S)
        for jl in range(S):
            j = rank * S + jl
            col = [rows[a * S + jl] for a in range(P)]
            for b in range(P):
                if not inverse:  # X[t] = sum_g wP^(g t) w^(g j) R[g]
                    v = sum(F.fpow(wP, a * b) * F.fpow(w, a * j) * col[a] for a in range(P))
                else:  # Z[g] = 1/P w^(-g j) sum_t wP^(-g t) X[t]
                    v = F.inv(P) * F.fpow(w, b * j) * sum(F.fpow(wP, a * b) * col[a] for a in range(P))
                out[b * S + jl] = v % F.M
        return _tensor(out)

    def commit_pairs(self, values):
        n = values.shape[0]
        return torch.from_numpy(C.merkle_commit_pairs(_limbs(values), n.bit_length() - 1).reshape(-1))

    def fold(self, values, k, log_domain, r, log_s, log_p, rank):
        v = _ints(values)
        n = len(v)
        ginv = F.inv(F.pow_2_generator(log_domain))
        out = []
        for l in range(n // 2):
            if log_p:
                gi = ((l >> log_s) << (log_s + log_p)) | (rank << log_s) | (l & ((1 << log_s) - 1))
            else:
                gi = l
            a, b = v[l], v[l + n // 2]
            tw = F.fpow(ginv, (gi << k) % (1 << log_domain))
            out.append(((a + b) + r * ((a - b) * tw % F.M)) * INV2 % F.M)
        return _tensor(out)

    def fold_commit(self, values, k, log_domain, r, log_s, log_p, rank):
        nx = self.fold(values, k, log_domain, r, log_s, log_p, rank)
        return nx, self.commit_pairs(nx)

    def open_pairs(self, values, tree, levels, idx):
        v = _limbs(values)
        half = v.shape[0] // 2
        t = tree.numpy().reshape(-1, 32)
        recs = []
        for i in idx:
            rec = v[i].tobytes() + v[i + half].tobytes()
            off = 0
            for lv in range(levels):
                rec += t[off + ((i >> lv) ^ 1)].tobytes()
                off += half >> lv
            recs.append(rec)
        return recs

    def to_host(self, values):
        return _limbs(values)

    # -- device-resident transcript stand-ins (state = a host Transcript) ------
    def dev_transcript(self, transcript):
        return transcript.clone()

    def absorb(self, state, src, challenge_out=None):
        state.absorb(src.contiguous().numpy().tobytes())
        if challenge_out is not None:
            challenge_out[:] = _tensor([state.next_challenge()])[0]

    def fri_last(self, vals2, state, flag_out, last_out):
        v = _limbs(vals2)
        flag_out[:] = 0
        flag_out[0, 0] = 0 if (v[0] == v[1]).all() else 1
        last_out[:] = vals2[0]
        state.absorb(v[0].tobytes())

    @staticmethod
    def _r(r_dev):
        return _ints(r_dev.reshape(1, 4))[0]

    def fold_dr(self, values, k, log_domain, r_dev, log_s, log_p, rank):
        return self.fold(values, k, log_domain, self._r(r_dev), log_s, log_p, rank)

    def fold_commit_dr(self, values, k, log_domain, r_dev, log_s, log_p, rank):
        return self.fold_commit(values, k, log_domain, self._r(r_dev), log_s, log_p, rank)

    def merkle_top(self, gathered, P, per_rank):
        import hashlib

        g = gathered.numpy().tobytes()
        lvl = [g[32 * (h * per_rank + t):32 * (h * per_rank + t + 1)]
               for t in range(per_rank) for h in range(P)]
        out = list(lvl)
        while len(lvl) > 1:
            lvl = [hashlib.sha256(lvl[2 * i] + lvl[2 * i + 1]).digest() for i in range(len(lvl) // 2)]
            out += lvl
        return torch.frombuffer(bytearray(b"".join(out)), dtype=torch.uint8)

    # -- sumcheck: oracle formulas, tables mutated in place ---------------------
    def eq_table(self, points):
        from oracle import sumcheck as OS

        return _tensor(OS.eq_table(points))

    def scale(self, x, c):
        return _tensor([v * c % F.M for v in _ints(x)])

    @staticmethod
    def _sums(m, d):
        h = len(m) // 2
        s1 = sum(m[i + h] * d[i + h] for i in range(h)) % F.M
        s2 = sum((2 * m[i + h] - m[i]) * (2 * d[i + h] - d[i]) for i in range(h)) % F.M
        return s1, s2

    def sc_sums(self, m, d):
        return self._sums(_ints(m), _ints(d))

    def sc_fold(self, m, d, log_h, r):
        for t in (m, d):
            v = _ints(t)
            h = 1 << (log_h - 1)
            folded = [(v[i] + r * (v[i + h] - v[i])) % F.M for i in range(h)]
            t[:h] = _tensor(folded)

    def const(self, v):
        return _tensor([v])

    def sc_sums_dev(self, m, d, log_h, out):
        out[:] = _tensor(list(self._sums(_ints(m[:1 << log_h]), _ints(d[:1 << log_h]))))

    def sc_fold_sums_dr(self, m, d, log_h, r_dev, out):
        out[:] = _tensor(list(self.sc_fold_and_sums(m, d, log_h, self._r(r_dev))))

    def sc_fold_dr(self, m, d, log_h, r_dev):
        self.sc_fold(m, d, log_h, self._r(r_dev))

    def sc_round(self, pairs, npairs, prev, state, poly_out, r_out):
        v = _ints(pairs)
        s1 = sum(v[0::2]) % F.M
        s2 = sum(v[1::2]) % F.M
        e0 = (_ints(prev)[0] - s1) % F.M
        c2 = (s2 - 2 * s1 + e0) * INV2 % F.M
        c1 = (s1 - e0 - c2) % F.M
        poly_out[:] = _tensor([c1, c2])
        state.absorb(F.to_bytes(c1))
        state.absorb(F.to_bytes(c2))
        r = state.next_challenge()
        r_out[:] = _tensor([r])[0]
        prev[:] = _tensor([(e0 + r * (c1 + c2 * r)) % F.M])

    def sc_fold_and_sums(self, m, d, log_h, r):
        self.sc_fold(m, d, log_h, r)
        h = 1 << (log_h - 1)
        return self._sums(_ints(m[:h]), _ints(d[:h]))

    def sync(self):
        pass
