"""CPU restatement of the grouped eq-factored sumcheck schedule that
mlh_sumcheck_prove_eq runs on the GPU (csrc/sumcheck.hip
"grouped eq-factored rounds"), checked against the oracle's per-round loop
(sumcheck.rs:174-247 restated in oracle/sumcheck.py).

The device never materialises delta = eq(points): a pass over the table T of
round k yields the corner sums Y_c = sum_i T[c Q + i] e(i) of up to six
rounds (e = eq of the points after them), one wave contracts them into the
rounds' E0/E1 as two chained 3-round groups, and one pass folds all six
variables at once.  The last `a` rounds run the same grouping on a small
table.  This test restates exactly that arithmetic in Python integers, so the
identities the kernels rely on are pinned independently of the GPU (the GPU
tests compare the kernels with the same oracle at n up to 24)."""
import random

from oracle import field as F
from oracle import sumcheck as OS
from oracle import transcript as OT
from oracle.polynomials import mle_evaluate


def _bit(c, nbits, u):  # variable u of a corner index (u = 0: the MSB)
    return (c >> (nbits - 1 - u)) & 1


def _eq_factor(b, x):
    return x if b else (1 - x) % F.M


def _rounds_from_corners(X, J, pts, state, tr, polys, rs):
    """J rounds from the 2^J corner sums X (eq_group_rounds): round t's
    E_b = sum_{c: c_t = b} prod_{u<t} f(c_u, r_u) prod_{t<u<J} f(c_u, p_u) X_c,
    s1 = c p E1, s2 = c (3p - 1)(2 E1 - E0)."""
    r = []
    for t in range(J):
        E = [0, 0]
        for c, x in enumerate(X):
            w = x
            for u in range(J):
                if u != t:
                    w = w * _eq_factor(_bit(c, J, u), r[u] if u < t else pts[u]) % F.M
            E[_bit(c, J, t)] = (E[_bit(c, J, t)] + w) % F.M
        p, cs = pts[t], state["c"]
        s1 = cs * p % F.M * E[1] % F.M
        s2 = cs * ((3 * p - 1) % F.M) % F.M * ((2 * E[1] - E[0]) % F.M) % F.M
        e0, c1, c2 = OS.round_coeffs_from_sums(state["claim"], s1, s2)
        tr.absorb(F.to_bytes(c1))
        tr.absorb(F.to_bytes(c2))
        rr = tr.next_challenge()
        state["claim"] = (e0 + rr * (c1 + c2 * rr)) % F.M
        state["c"] = cs * (((1 - rr) * (1 - p) + rr * p) % F.M) % F.M
        polys.append((c1, c2))
        rs.append(rr)
        r.append(rr)
    return r


def _fold(T, r):
    """Fold the len(r) top variables of T (MSB first), all at once."""
    for rr in r:
        h = len(T) // 2
        T = [(T[i] + rr * (T[i + h] - T[i])) % F.M for i in range(h)]
    return T


def grouped_prove(ev, pts, total, tr, a, head_pass=6):
    L = len(pts)
    B = L - a
    state = {"claim": total, "c": 1}
    polys, rs = [], []
    T, k = list(ev), 0
    while k < L:
        JT = min(head_pass if k < B else 3, (B if k < B else L) - k)
        J1 = min(3, JT)
        J2 = JT - J1
        Q = len(T) >> JT
        e = OS.eq_table(pts[k + JT:]) if k + JT < L else [1]
        Y = [sum(T[c * Q + i] * e[i] for i in range(Q)) % F.M for c in range(1 << JT)]
        # group 1: sum out the low J2 bits with their eq weights
        X1 = [0] * (1 << J1)
        for c, y in enumerate(Y):
            w = y
            for u in range(J2):
                w = w * _eq_factor(_bit(c, JT, J1 + u), pts[k + J1 + u]) % F.M
            X1[c >> J2] = (X1[c >> J2] + w) % F.M
        r1 = _rounds_from_corners(X1, J1, pts[k:k + J1], state, tr, polys, rs)
        r2 = []
        if J2:  # group 2: fold the high J1 bits with group 1's challenges
            X2 = [0] * (1 << J2)
            for c, y in enumerate(Y):
                w = y
                for u in range(J1):
                    w = w * _eq_factor(_bit(c, JT, u), r1[u]) % F.M
                X2[c & ((1 << J2) - 1)] = (X2[c & ((1 << J2) - 1)] + w) % F.M
            r2 = _rounds_from_corners(X2, J2, pts[k + J1:k + JT], state, tr, polys, rs)
        T = _fold(T, r1 + r2)
        k += JT
    return polys, rs, T[0], state["c"]


def _oracle_prove(ev, pts, total, label):
    t = OS.SumcheckTables.build_tables_for_pcs(pts, ev)
    tr = OT.Transcript()
    tr.absorb(label)
    prev, polys, rs = total, [], []
    for _ in range(len(pts)):
        nz, r, prev = t.compute_sumcheck_polynomial(prev, tr)
        polys.append(tuple(nz))
        rs.append(r)
    return polys, rs, t.matrix[0], t.delta[0], tr.random()


def test_grouped_schedule_matches_per_round_oracle():
    rng = random.Random(2024)
    # (n, a): head rounds B = n - a in passes of <= 6 (3 + 3), tail of a rounds
    for n, a in [(1, 1), (3, 3), (4, 1), (7, 2), (9, 2), (10, 3), (13, 1)]:
        ev = [rng.randrange(F.M) for _ in range(1 << n)]
        pts = [rng.randrange(F.M) for _ in range(n)]
        total = mle_evaluate(ev, pts)
        want = _oracle_prove(ev, pts, total, b"grouped")
        tr = OT.Transcript()
        tr.absorb(b"grouped")
        polys, rs, m0, c = grouped_prove(ev, pts, total, tr, a)
        assert polys == want[0] and rs == want[1], (n, a)
        assert m0 == want[2] and c == want[3], (n, a)  # folded matrix, final delta = c_L
        assert tr.random() == want[4], (n, a)


def test_grouped_schedule_pass_lengths():
    """Any split of the head into passes gives the same proof (the device uses
    6; the PCS keeps 3-round groups)."""
    rng = random.Random(7)
    n, a = 11, 2
    ev = [rng.randrange(F.M) for _ in range(1 << n)]
    pts = [rng.randrange(F.M) for _ in range(n)]
    total = mle_evaluate(ev, pts)
    outs = []
    for hp in (1, 2, 3, 5, 6):
        tr = OT.Transcript()
        outs.append(grouped_prove(ev, pts, total, tr, a, head_pass=hp)[:2] + (tr.random(),))
    assert all(o == outs[0] for o in outs)
