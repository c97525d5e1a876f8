"""Generator for the hand-scheduled gfx950 radix-2 butterflies (multilinear_amd/csrc/bfly_asm.hpp).

Why: the NTT passes are VALU-issue bound.  hipcc cannot use the
carry-out of v_mad_u64_u32, so the field product was written as one small asm
statement per multiply-accumulate; every statement boundary then costs a pad
and every carry a 2-state SGPR hazard (gfx950: a VALU write of an SGPR/VCC must
be 2 wait states ahead of a VALU read of it), ~1.5 `s_nop` per mad.  This tool
emits whole butterflies (one or two per statement, interleaved) with the
hazards covered by independent work, in the RELAXED representation:

  values are any representative in [0, 2^128) (2M > 2^128, so every residue
  has one or two), canonicalised only where they leave the NTT.

Butterfly (DIT): (u, v) -> (u + w*v, u - w*v), w given as its four limb-shifted
multiples B_k = w * 2^(32k) mod M ("expanded" stage twiddles, fe_mul_pre):
  * product: 16 v_mad_u64_u32 column-scanned, carries counted by v_addc;
    T = top bits (< 2^34) folded once: r + T*C, C = 2^128 - M = 0x2D00*2^32 - 1.
    If r + T*C wraps 2^128 (probability ~2^-48) flag K (true t = s + C).
  * a = u + t: carry -> + C; a second carry (only when the first sum's
    remainder was >= 2^128 - C, probability ~2^-46) is flagged (C2).
  * d = u - t: borrow -> - C; a second borrow is flagged (B2).
  60 VALU per butterfly with a twiddle, 20 without, no s_nop in steady state.
The flags are SGPR lane masks; the C++ wrapper checks them with SALU ops and
fixes flagged lanes on a cold path (each fix is +-C in relaxed arithmetic).

Precondition of the product (checked by tests/test_bfly_asm.py over every
stage twiddle the NTT can use): the first mad of columns 1..3 adds
v0*B0[j] to a carry word < 2^35, which cannot overflow 64 bits when
B0[j] = w's limb j <= 2^32 - 8.  Every root of unity of order <= 2^9 except -1
satisfies it, and -1 is never a stage twiddle (j < len/2).

The same instruction list drives a one-lane emulator and a hazard checker
(`emulate`, `check_hazards`), so the asm is validated on the CPU before it
ever runs.  Run:  python tools/gen_bfly.py   (rewrites bfly_asm.hpp)
"""
import os
import random

M = (1 << 128) - 45 * (1 << 40) + 1
C = (1 << 128) - M
MASK32 = (1 << 32) - 1
KC1 = C >> 32  # 0x2CFF
K2D00 = 0x2D00

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "multilinear_amd", "csrc", "bfly_asm.hpp")

# VGPR temporaries live in physical registers (pairs must be even-aligned and
# their halves addressable, which an inline-asm operand cannot give).
VBASE = 0

# ---------------------------------------------------------------- program ---


class Ins:
    """One instruction.  dst/src name virtual registers (str) or immediates (int).
    A pair is ('pair', lo, hi).  sdst/cin name SGPR-pair virtual registers."""

    def __init__(self, op, dst, src, sdst=None, cin=None, tag=0, after=()):
        self.op, self.dst, self.src, self.sdst, self.cin, self.tag = op, dst, src, sdst, cin, tag
        # names whose every read must precede this instruction (it reuses
        # their register: the second hi partner of a pair's lo, see allocate)
        self.after = tuple(after)

    def vreads(self):
        out = []
        for s in self.src:
            if isinstance(s, tuple):
                out += [s[1], s[2]]
            elif isinstance(s, str):
                out.append(s)
        return out

    def vwrites(self):
        if isinstance(self.dst, tuple):
            return [self.dst[1], self.dst[2]]
        return [self.dst] if self.dst else []

    def sreads(self):
        return [self.cin] if self.cin else []

    def swrites(self):
        return [self.sdst] if self.sdst and self.sdst != "junk" else []


def product_prog(E, p, V, B, safe, kflag):
    """t = sum_k V_k * B_k (relaxed), appended through E.  safe: count the carry
    of every column's first mad too (any twiddle); otherwise columns 1..3 rely
    on the stage-twiddle precondition (module docstring).  Returns the four
    limb names of t; the wrap flag goes to SGPR kflag."""
    r = []
    acc = 0
    for j in range(4):
        cys = []
        for k in range(4):
            dst = ("pair", p + "P%d_%d.lo" % (j, k), p + "P%d_%d.hi" % (j, k))
            if k == 0 and (j == 0 or not safe):
                E("mad", dst, [V[k], B[k][j], acc], sdst="junk")
            else:
                cy = p + "cy%d%d" % (j, k)
                cys.append(cy)
                E("mad", dst, [V[k], B[k][j], acc], sdst=cy)
            acc = dst
        r.append(acc[1])
        # carry count -> hi half of the next column's addend pair
        nlo, nhi = p + "Q%d.lo" % (j + 1), p + "Q%d.hi" % (j + 1)
        c = 0
        for n, cy in enumerate(cys):
            d = nhi if n == len(cys) - 1 else p + "c%d_%d" % (j, n)
            E("addc", d, [c, 0], sdst="junk", cin=cy)
            c = d
        if j < 3:
            E("mov", nlo, [acc[2]])
            acc = ("pair", nlo, nhi)
        else:
            t_lo, t_hi = acc[2], nhi
    # fold T*2^128 = T*C = T*0x2D00*2^32 - T
    Y = ("pair", p + "Y.lo", p + "Y.hi")
    E("mad", Y, [t_lo, "k2d00", 0], sdst="junk")
    E("mad24", p + "Yh2", [t_hi, "k2d00", Y[2]])
    E("sub", p + "x0", [0, t_lo], sdst=p + "bb0")
    E("subb", p + "x1", [Y[1], t_hi], sdst=p + "bb1", cin=p + "bb0")
    E("subb", p + "x2", [p + "Yh2", 0], sdst="junk", cin=p + "bb1")
    return r, p


def fmul_prog(E, p, V, W):
    """Full product v * w of two plain 128-bit values (w: a table entry, any
    value < 2^128), relaxed result written to the tied output d.  Product
    scan over 7 columns (16 mads; the first mad of columns 0, 1 and the single
    mad of column 6 cannot overflow, every other carry is counted), then
    H*2^128 = H*C = H*0x2D00*2^32 - H: Z = L + (H*0x2D00 << 32) by 4 mads,
    Z - H, and the top T < 2^47 folded once more (T*0x2D00*2^32 - T).  A
    carry out of the last add (value >= 2^128, probability ~2^-35) is flagged
    in K: the true value is s + C."""
    acc = 0
    r = []
    col_hi = {}
    for j in range(7):
        terms = [(i, j - i) for i in range(4) if 0 <= j - i <= 3]
        cys = []
        for n, (i, jj) in enumerate(terms):
            dst = ("pair", p + "P%d_%d.lo" % (j, n), p + "P%d_%d.hi" % (j, n))
            if (n == 0 and j <= 1) or j == 6:
                E("mad", dst, [V[i], W[jj], acc], sdst="junk")
            else:
                cy = p + "cy%d%d" % (j, n)
                cys.append(cy)
                E("mad", dst, [V[i], W[jj], acc], sdst=cy)
            acc = dst
        r.append(acc[1])
        col_hi[j] = acc[2]
        if j == 6:
            r.append(acc[2])
            break
        nlo, nhi = p + "Q%d.lo" % (j + 1), p + "Q%d.hi" % (j + 1)
        if cys:
            c = 0
            for n, cy in enumerate(cys):
                d = nhi if n == len(cys) - 1 else p + "c%d_%d" % (j, n)
                E("addc", d, [c, 0], sdst="junk", cin=cy)
                c = d
        else:
            E("mov", nhi, [0])
        E("mov", nlo, [acc[2]])
        acc = ("pair", nlo, nhi)
    # Z = L + (H * 0x2D00) << 32.  Z_j = r_j + r_{j+3}*0x2D00 (j = 1..3) by a
    # mad onto the pair {r_j, 0}: r_j's own register pair, whose hi half
    # (the column's carry word, already moved on) is re-zeroed; Z_4 = r_7*0x2D00.
    Z = {}
    for j in (1, 2, 3):
        zr = p + "Zr%d" % j
        E("mov", zr, [0], after=[col_hi[j]])
        Z[j] = ("pair", p + "Z%d.lo" % j, p + "Z%d.hi" % j)
        E("mad", Z[j], [r[j + 3], "k2d00", ("pair", r[j], zr)], sdst="junk")
    Z[4] = ("pair", p + "Z4.lo", p + "Z4.hi")
    E("mad", Z[4], [r[7], "k2d00", 0], sdst="junk")
    # carry words (< 2^15) into the next limb
    E("add", p + "a2", [Z[2][1], Z[1][2]], sdst=p + "e3")
    E("addc", p + "a3", [Z[3][1], Z[2][2]], sdst=p + "e4", cin=p + "e3")
    E("addc", p + "a4", [Z[4][1], Z[3][2]], sdst=p + "e5", cin=p + "e4")
    E("addc", p + "a5", [Z[4][2], 0], sdst="junk", cin=p + "e5")
    # X = Z - H (>= 0): x0..x3, top T = (tl, th) < 2^47
    E("sub", p + "x0", [r[0], r[4]], sdst=p + "bb0")
    E("subb", p + "x1", [Z[1][1], r[5]], sdst=p + "bb1", cin=p + "bb0")
    E("subb", p + "x2", [p + "a2", r[6]], sdst=p + "bb2", cin=p + "bb1")
    E("subb", p + "x3", [p + "a3", r[7]], sdst=p + "bb3", cin=p + "bb2")
    E("subb", p + "tl", [p + "a4", 0], sdst=p + "bb4", cin=p + "bb3")
    E("subb", p + "th", [p + "a5", 0], sdst="junk", cin=p + "bb4")
    # fold T: T*C = (T*0x2D00) << 32 - T  (three limbs y0..y2, >= 0)
    Y = ("pair", p + "Y.lo", p + "Y.hi")
    E("mad", Y, [p + "tl", "k2d00", 0], sdst="junk")
    E("mad24", p + "Yh2", [p + "th", "k2d00", Y[2]])
    E("sub", p + "y0", [0, p + "tl"], sdst=p + "bb5")
    E("subb", p + "y1", [Y[1], p + "th"], sdst=p + "bb6", cin=p + "bb5")
    E("subb", p + "y2", [p + "Yh2", 0], sdst="junk", cin=p + "bb6")
    return [p + "x0", p + "x1", p + "x2", p + "x3"], [p + "y0", p + "y1", p + "y2"]


def canon_prog(E, p, b):
    """Relaxed -> canonical: x >= M iff x + C carries out of 2^128."""
    V = ["v%d_%d" % (b, i) for i in range(4)]
    T = [p + "T%d" % i for i in range(4)]
    E("add", T[0], [V[0], -1], sdst=p + "e0")
    E("addc", T[1], [V[1], "kc1"], sdst=p + "e1", cin=p + "e0")
    E("addc", T[2], [V[2], 0], sdst=p + "e2", cin=p + "e1")
    E("addc", T[3], [V[3], 0], sdst=p + "e3", cin=p + "e2")
    for i in range(4):
        E("cnd", "d%d_%d" % (b, i), [V[i], T[i]], cin=p + "e3")


def bfly_prog(b, kind):
    """Instruction list of butterfly b.  kind 'm': with a stage twiddle, 't':
    trivial (w = 1), 'p': product only v <- w v (safe first mads; any twiddle).
    Operand names: u{b}_{i} (in, tied to a), v{b}_{i} (in, tied to d),
    B{b}_{k}{j} (twiddle limbs), kc1 (VGPR 0x2CFF), k2d00 (SGPR 0x2D00).
    Flags K{b}, C2{b}, B2{b}."""
    p = "b%d." % b
    U = ["u%d_%d" % (b, i) for i in range(4)]
    V = ["v%d_%d" % (b, i) for i in range(4)]
    prog = []
    E = lambda *a, **k: prog.append(Ins(*a, tag=b, **k))
    if kind == "c":
        canon_prog(E, p, b)
        return prog
    if kind == "f":
        W = ["W%d_%d" % (b, j) for j in range(4)]
        X, Yl = fmul_prog(E, p, V, W)
        S = ["d%d_%d" % (b, i) for i in range(4)]
        E("add", S[0], [X[0], Yl[0]], sdst=p + "e0")
        E("addc", S[1], [X[1], Yl[1]], sdst=p + "e1", cin=p + "e0")
        E("addc", S[2], [X[2], Yl[2]], sdst=p + "e2", cin=p + "e1")
        E("addc", S[3], [X[3], 0], sdst="K%d" % b, cin=p + "e2")
        return prog
    if kind in ("m", "p"):
        B = [["B%d_%d%d" % (b, k, j) for j in range(4)] for k in range(4)]
        r, _ = product_prog(E, p, V, B, kind == "p", "K%d" % b)
        if kind == "p":  # s = r + X written straight into v (tied output d)
            S = ["d%d_%d" % (b, i) for i in range(4)]
        else:
            S = [p + "s%d" % i for i in range(4)]
        E("add", S[0], [r[0], p + "x0"], sdst=p + "e0")
        E("addc", S[1], [r[1], p + "x1"], sdst=p + "e1", cin=p + "e0")
        E("addc", S[2], [r[2], p + "x2"], sdst=p + "e2", cin=p + "e1")
        E("addc", S[3], [r[3], 0], sdst="K%d" % b, cin=p + "e2")
        if kind == "p":
            return prog
    else:
        S = V
    A = [p + "A%d" % i for i in range(4)]
    D = [p + "D%d" % i for i in range(4)]
    E("add", A[0], [U[0], S[0]], sdst=p + "f0")
    E("sub", D[0], [U[0], S[0]], sdst=p + "g0")
    for i in (1, 2, 3):
        E("addc", A[i], [U[i], S[i]], sdst=p + ("f%d" % i if i < 3 else "C1"), cin=p + "f%d" % (i - 1))
        E("subb", D[i], [U[i], S[i]], sdst=p + ("g%d" % i if i < 3 else "B1"), cin=p + "g%d" % (i - 1))
    # a + C1*C, d - B1*C   (C = 0x2CFF_FFFFFFFF)
    E("cnd", p + "ma0", [0, -1], cin=p + "C1")
    E("cnd", p + "ma1", [0, "kc1"], cin=p + "C1")
    E("cnd", p + "md0", [0, -1], cin=p + "B1")
    E("cnd", p + "md1", [0, "kc1"], cin=p + "B1")
    aout = ["a%d_%d" % (b, i) for i in range(4)]  # tied to U
    dout = ["d%d_%d" % (b, i) for i in range(4)]  # tied to V
    E("add", aout[0], [A[0], p + "ma0"], sdst=p + "h0")
    E("sub", dout[0], [D[0], p + "md0"], sdst=p + "i0")
    E("addc", aout[1], [A[1], p + "ma1"], sdst=p + "h1", cin=p + "h0")
    E("subb", dout[1], [D[1], p + "md1"], sdst=p + "i1", cin=p + "i0")
    E("addc", aout[2], [A[2], 0], sdst=p + "h2", cin=p + "h1")
    E("subb", dout[2], [D[2], 0], sdst=p + "i2", cin=p + "i1")
    E("addc", aout[3], [A[3], 0], sdst="C2%d" % b, cin=p + "h2")
    E("subb", dout[3], [D[3], 0], sdst="B2%d" % b, cin=p + "i2")
    return prog


# ------------------------------------------------------------- scheduling ---

SGPR_GAP = 3  # consumer index - producer index >= 3: two wait states between


def schedule(progs):
    """List-schedule the union of independent instruction lists.  Dependencies:
    true (RAW) on VGPRs (no gap) and SGPRs (SGPR_GAP), plus program order
    between writes/reads of tied output operands.  Priority: longest path."""
    ins = [i for p in progs for i in p]
    n = len(ins)
    writer = {}
    deps = [[] for _ in range(n)]  # (pred, gap)
    readers = {}
    for idx, it in enumerate(ins):
        for r in it.vreads():
            if r in writer:
                deps[idx].append((writer[r], 1))
            readers.setdefault(r, []).append(idx)
        for r in it.sreads():
            deps[idx].append((writer[r], SGPR_GAP))
        for w in it.vwrites() + it.swrites():
            writer[w] = idx
    # tied outputs: a{b}_i overwrites u{b}_i, d{b}_i overwrites v{b}_i -> after every read
    for idx, it in enumerate(ins):
        for w in it.vwrites():
            if w[0] in "ad" and "_" in w and not w.startswith("b"):
                src = ("u" if w[0] == "a" else "v") + w[1:]
                for rd in readers.get(src, []):
                    if rd != idx:
                        deps[idx].append((rd, 0))
    for idx, it in enumerate(ins):
        for nm in it.after:
            for rd in readers.get(nm, []):
                deps[idx].append((rd, 0))
            if nm in writer:
                deps[idx].append((writer[nm], 0))
    succ = [[] for _ in range(n)]
    for i in range(n):
        for (p, g) in deps[i]:
            succ[p].append((i, g))
    prio = [0] * n
    for i in reversed(range(n)):
        prio[i] = 1 + max([prio[s] + (g - 1 if g > 1 else 0) for s, g in succ[i]] + [0])
    done_at = {}
    order = []  # list of instruction indices or None (s_nop 0)
    remaining = set(range(n))
    t = 0
    while remaining:
        ready = [i for i in remaining if all(p in done_at and t - done_at[p] >= g for p, g in deps[i])]
        if not ready:
            order.append(None)
            t += 1
            continue
        # prefer mads slightly (long latency), then priority, then program order
        i = max(ready, key=lambda i: (prio[i], -i))
        order.append(i)
        done_at[i] = t
        remaining.discard(i)
        t += 1
    return ins, order


# -------------------------------------------------------- register alloc ---


def allocate(ins, order):
    """Physical VGPRs for temporaries (pairs even-aligned), SGPR-pair slots for
    carries.  Operand-backed names (inputs/outputs/constants) are not allocated."""
    seq = [ins[i] if i is not None else None for i in order]
    first, last = {}, {}
    pairs = []
    for t, it in enumerate(seq):
        if it is None:
            continue
        for r in it.vreads() + it.sreads():
            last[r] = t
        for w in it.vwrites() + it.swrites():
            first.setdefault(w, t)
            last.setdefault(w, t)
        if isinstance(it.dst, tuple):
            pairs.append((it.dst[1], it.dst[2]))
        for s in it.src:
            if isinstance(s, tuple):
                pairs.append((s[1], s[2]))
    is_temp = lambda r: r.startswith("b") and "." in r
    # pair groups (halves may be defined by different instructions); a lo may
    # have several hi partners with disjoint lifetimes (one odd register)
    lo_his, hi_lo = {}, {}
    for lo, hi in pairs:
        lo_his.setdefault(lo, [])
        if hi not in lo_his[lo]:
            lo_his[lo].append(hi)
        assert hi_lo.get(hi, lo) == lo, ("hi with two lo partners", hi)
        hi_lo[hi] = lo
    vtemps = [r for r in first if is_temp(r) and not is_sgpr_name(r)]
    stemps = [r for r in first if is_temp(r) and is_sgpr_name(r)]
    # half-step intervals: defined by instruction t -> occupied from 2t+1, last
    # read by t -> until 2t, so the reader of a dying value may write the same
    # register (reads precede writes); a dead write still occupies 2t+1
    busy = {}  # phys -> list of (a, b) inclusive

    def span(r):
        return (2 * first[r] + 1, max(2 * last[r], 2 * first[r] + 1))

    def free(phys, a, b):
        for (x, y) in busy.get(phys, []):
            if not (b < x or y < a):
                return False
        return True

    assign = {}
    for r in sorted(vtemps, key=lambda r: first[r]):
        if r in assign:
            continue
        if r in lo_his or r in hi_lo:
            lo = r if r in lo_his else hi_lo[r]
            his = lo_his[lo]
            ivs = [span(h) for h in his]
            for i in range(len(ivs)):
                for j in range(i):
                    a, b = ivs[i], ivs[j]
                    assert a[1] < b[0] or b[1] < a[0], ("hi partners overlap", lo, his)
            ia = span(lo)
            m = 0
            while not (free(VBASE + 2 * m, *ia) and all(free(VBASE + 2 * m + 1, *iv) for iv in ivs)):
                m += 1
            busy.setdefault(VBASE + 2 * m, []).append(ia)
            assign[lo] = "v%d" % (VBASE + 2 * m)
            for h, iv in zip(his, ivs):
                busy.setdefault(VBASE + 2 * m + 1, []).append(iv)
                assign[h] = "v%d" % (VBASE + 2 * m + 1)
        else:
            iv = span(r)
            m = VBASE
            while not free(m, *iv):
                m += 1
            busy.setdefault(m, []).append(iv)
            assign[r] = "v%d" % m
    sbusy = {}
    for r in sorted(stemps, key=lambda r: first[r]):
        iv = span(r)
        m = 0
        while any(not (iv[1] < x or y < iv[0]) for (x, y) in sbusy.get(m, [])):
            m += 1
        sbusy.setdefault(m, []).append(iv)
        assign[r] = ("sgpr", m)
    nv = 1 + max([int(v[1:]) for v in assign.values() if isinstance(v, str)] + [-1])
    ns = 1 + max([v[1] for v in assign.values() if isinstance(v, tuple)] + [-1])
    return seq, assign, nv, ns


def is_sgpr_name(r):
    base = r.split(".", 1)[1]
    return base.startswith(("cy", "bb", "e", "f", "g", "h", "i")) or base in ("C1", "B1")


# ----------------------------------------------------------------- emit ----


def emit(kinds, bsrc):
    """kinds: tuple of 'm' (with twiddle) / 't' (trivial, w = 1) per butterfly.
    bsrc: 's' (twiddle limbs in SGPRs) or 'v'.  Returns (asm lines, operand
    description, nvgpr, nsgpr-pairs)."""
    progs = [bfly_prog(b, k) for b, k in enumerate(kinds)]
    ins, order = schedule(progs)
    seq, assign, nv, ns = allocate(ins, order)
    # trailing pad: the C++ code may read the flag SGPRs with a VALU right away
    tail = 0
    for back, it in enumerate(reversed(seq)):
        if it is not None and any(s.startswith(("K", "C2", "B2")) for s in it.swrites()):
            tail = max(tail, SGPR_GAP - 1 - back)
    return seq, assign, nv, ns, max(tail, 0)


def has_u(k):
    return k in ("m", "t")


def operand_names(kinds):
    outs, ins = [], []
    for b, k in enumerate(kinds):
        if has_u(k):
            outs += ["u%d_%d" % (b, i) for i in range(4)]
        outs += ["v%d_%d" % (b, i) for i in range(4)]
    flags = []
    for b, k in enumerate(kinds):
        if k in ("m", "p", "f"):
            flags.append("K%d" % b)
        if has_u(k):
            flags += ["C2%d" % b, "B2%d" % b]
    for b, k in enumerate(kinds):
        if k in ("m", "p"):
            ins += ["B%d_%d%d" % (b, kk, j) for kk in range(4) for j in range(4)]
        if k == "f":
            ins += ["W%d_%d" % (b, j) for j in range(4)]
    if any(k in ("m", "t", "c") for k in kinds):
        ins += ["kc1"]
    if any(k in ("m", "p", "f") for k in kinds):
        ins += ["k2d00"]
    return outs, flags, ins


def render(kinds, bsrc):
    seq, assign, nv, ns, tail = emit(kinds, bsrc)
    outs, flags, ins = operand_names(kinds)
    # operand numbering: outputs (tied "+v"), flags "=&s", sgpr temps "=&s", junk "=&s", inputs
    opn = {}
    k = 0
    for o in outs:
        opn[o] = k
        k += 1
    for f in flags:
        opn[f] = k
        k += 1
    stmp = []
    for s in range(ns):
        opn[("sgpr", s)] = k
        stmp.append(k)
        k += 1
    opn["junk"] = k
    k += 1
    for i in ins:
        opn[i] = k
        k += 1

    def name(r):
        if isinstance(r, int):
            return str(r)
        if r in assign:
            a = assign[r]
            return "%%%d" % opn[a] if isinstance(a, tuple) else a
        if r[0] in "ad" and "_" in r and "." not in r:  # tied outputs
            return "%%%d" % opn[("u" if r[0] == "a" else "v") + r[1:]]
        return "%%%d" % opn[r]

    def pname(p):
        lo, hi = name(p[1]), name(p[2])
        assert lo.startswith("v") and hi == "v%d" % (int(lo[1:]) + 1) and int(lo[1:]) % 2 == 0, (p, lo, hi)
        return "v[%d:%d]" % (int(lo[1:]), int(hi[1:]))

    lines = []
    for it in seq:
        if it is None:
            lines.append("s_nop 0")
            continue
        sd = name(it.sdst) if it.sdst else None
        if it.op == "mad":
            s2 = pname(it.src[2]) if isinstance(it.src[2], tuple) else "0"
            lines.append("v_mad_u64_u32 %s, %s, %s, %s, %s" % (pname(it.dst), sd, name(it.src[0]),
                                                               name(it.src[1]), s2))
        elif it.op == "mad24":
            lines.append("v_mad_u32_u24 %s, %s, %s, %s" % (name(it.dst), name(it.src[0]), name(it.src[1]),
                                                          name(it.src[2])))
        elif it.op == "addc":
            lines.append("v_addc_co_u32_e64 %s, %s, %s, %s, %s" % (name(it.dst), sd, name(it.src[0]),
                                                                   name(it.src[1]), name(it.cin)))
        elif it.op == "subb":
            lines.append("v_subb_co_u32_e64 %s, %s, %s, %s, %s" % (name(it.dst), sd, name(it.src[0]),
                                                                   name(it.src[1]), name(it.cin)))
        elif it.op == "add":
            lines.append("v_add_co_u32_e64 %s, %s, %s, %s" % (name(it.dst), sd, name(it.src[0]),
                                                              name(it.src[1])))
        elif it.op == "sub":
            lines.append("v_sub_co_u32_e64 %s, %s, %s, %s" % (name(it.dst), sd, name(it.src[0]),
                                                              name(it.src[1])))
        elif it.op == "cnd":
            lines.append("v_cndmask_b32_e64 %s, %s, %s, %s" % (name(it.dst), name(it.src[0]),
                                                               name(it.src[1]), name(it.cin)))
        elif it.op == "mov":
            lines.append("v_mov_b32 %s, %s" % (name(it.dst), name(it.src[0])))
        else:
            raise ValueError(it.op)
    if tail:
        lines.append("s_nop %d" % (tail - 1))
    return lines, outs, flags, ins, ns, nv, opn


# ------------------------------------------------------------- emulation ---


def emulate(lines, env):
    """One-lane emulator of the rendered asm.  env maps '%N' operand refs and
    physical 'vN' to 32-bit ints; SGPR pairs to 0/1 carries."""
    regs = dict(env)

    def rd(x):
        if x.startswith("v[") or x.startswith("%") or x.startswith("v"):
            return regs[x]
        return int(x) & MASK32

    def rdp(x):
        if x == "0":
            return 0
        a, b = x[2:-1].split(":")
        return regs["v" + a] | (regs["v" + b] << 32)

    def wrp(x, val):
        a, b = x[2:-1].split(":")
        regs["v" + a] = val & MASK32
        regs["v" + b] = (val >> 32) & MASK32

    for ln in lines:
        op, _, rest = ln.partition(" ")
        a = [s.strip() for s in rest.split(",")] if rest else []
        if op == "s_nop":
            continue
        if op == "v_mad_u64_u32":
            v = rd(a[2]) * rd(a[3]) + rdp(a[4])
            wrp(a[0], v)
            regs[a[1]] = v >> 64
        elif op == "v_mad_u32_u24":
            regs[a[0]] = ((rd(a[1]) & 0xFFFFFF) * (rd(a[2]) & 0xFFFFFF) + rd(a[3])) & MASK32
        elif op in ("v_addc_co_u32_e64", "v_add_co_u32_e64"):
            cin = regs[a[4]] if op == "v_addc_co_u32_e64" else 0
            v = rd(a[2]) + rd(a[3]) + cin
            regs[a[0]] = v & MASK32
            regs[a[1]] = v >> 32
        elif op in ("v_subb_co_u32_e64", "v_sub_co_u32_e64"):
            bin_ = regs[a[4]] if op == "v_subb_co_u32_e64" else 0
            v = rd(a[2]) - rd(a[3]) - bin_
            regs[a[0]] = v & MASK32
            regs[a[1]] = 1 if v < 0 else 0
        elif op == "v_cndmask_b32_e64":
            regs[a[0]] = rd(a[2]) if regs[a[3]] else rd(a[1])
        elif op == "v_mov_b32":
            regs[a[0]] = rd(a[1])
        else:
            raise ValueError(op)
    return regs


def check_hazards(lines):
    """Every VALU read of an SGPR written by a VALU must be >= 2 wait states later."""
    last_w = {}
    t = 0
    for ln in lines:
        op, _, rest = ln.partition(" ")
        a = [s.strip() for s in rest.split(",")] if rest else []
        if op == "s_nop":
            t += int(a[0]) + 1
            continue
        reads, writes = [], []
        if op in ("v_addc_co_u32_e64", "v_subb_co_u32_e64"):
            reads.append(a[4])
        if op == "v_cndmask_b32_e64":
            reads.append(a[3])
        if op in ("v_mad_u64_u32", "v_addc_co_u32_e64", "v_add_co_u32_e64", "v_subb_co_u32_e64",
                  "v_sub_co_u32_e64"):
            writes.append(a[1])
        for r in reads:
            if r in last_w and t - last_w[r] < SGPR_GAP:
                raise AssertionError("SGPR hazard on %s at '%s' (distance %d)" % (r, ln, t - last_w[r]))
        for w in writes:
            last_w[w] = t
        t += 1


def limbs(x):
    return [(x >> (32 * i)) & MASK32 for i in range(4)]


def value(l):
    return sum(v << (32 * i) for i, v in enumerate(l))


def run_case(kinds, lines, opn, nv, uvals, vvals, wvals):
    """Emulate one lane; apply the flag fixes as the C++ cold path does;
    return [(a, d)] as integers (a = None for the one-operand kinds)."""
    env = {}
    for b in range(len(kinds)):
        for i in range(4):
            if has_u(kinds[b]):
                env["%%%d" % opn["u%d_%d" % (b, i)]] = limbs(uvals[b])[i]
            env["%%%d" % opn["v%d_%d" % (b, i)]] = limbs(vvals[b])[i]
        if kinds[b] in ("m", "p"):
            Bs = [wvals[b] * (1 << (32 * k)) % M for k in range(4)]
            for k in range(4):
                for j in range(4):
                    env["%%%d" % opn["B%d_%d%d" % (b, k, j)]] = limbs(Bs[k])[j]
        if kinds[b] == "f":
            for j in range(4):
                env["%%%d" % opn["W%d_%d" % (b, j)]] = limbs(wvals[b])[j]
    if "kc1" in opn:
        env["%%%d" % opn["kc1"]] = KC1
    if "k2d00" in opn:
        env["%%%d" % opn["k2d00"]] = K2D00
    regs = emulate(lines, env)
    res = []
    for b in range(len(kinds)):
        d = value([regs["%%%d" % opn["v%d_%d" % (b, i)]] for i in range(4)])
        if kinds[b] in ("p", "f"):  # v <- w v; flag K: true value s + C
            res.append((None, add_c(d) if regs["%%%d" % opn["K%d" % b]] else d))
            continue
        if kinds[b] == "c":
            res.append((None, d))
            continue
        a = value([regs["%%%d" % opn["u%d_%d" % (b, i)]] for i in range(4)])
        fk = regs.get("%%%d" % opn["K%d" % b], 0) if kinds[b] == "m" else 0
        fc = regs["%%%d" % opn["C2%d" % b]]
        fb = regs["%%%d" % opn["B2%d" % b]]
        a, d = fix(a, d, fk, fc, fb)
        res.append((a, d))
    return res


def add_c(x):
    x += C
    if x >> 128:
        x = (x & ((1 << 128) - 1)) + C
    return x


def sub_c(x):
    x -= C
    if x < 0:
        x = x + (1 << 128) - C
    return x


def fix(a, d, fk, fc, fb):
    """The cold path of the C++ wrapper (relaxed +-C fixes)."""
    if fk:
        a, d = add_c(a), sub_c(d)
    if fc:
        a = add_c(a)
    if fb:
        d = sub_c(d)
    return a, d


def selftest(kinds, lines, opn, nv, trials=3000, seed=1):
    rng = random.Random(seed)
    edge = [0, 1, M - 1, M, (1 << 128) - 1, C, C - 1, (1 << 128) - C, (1 << 128) - C - 1, M - C,
            (1 << 127), (1 << 96) - 1, 0xFFFFFFFF, ((1 << 128) - 1) ^ 0xFFFFFFFF]
    # twiddles: roots of unity of small order (what the NTT uses) and random
    roots = []
    g = pow(3, (M - 1) >> 9, M)
    for e in range(512):
        roots.append(pow(g, e, M))
    roots = [w for w in roots if w != M - 1]
    checked = 0
    for t in range(trials):
        nb = len(kinds)
        pick = lambda: rng.choice(edge) if rng.random() < 0.3 else rng.randrange(1 << 128)
        uv = [pick() for _ in range(nb)]
        vv = [pick() for _ in range(nb)]
        # products ('p') take any canonical twiddle, limbs of 0xFFFFFFFF included
        wv = [rng.choice(roots) if k not in ("p", "f") else
              (rng.choice([M - 1, M - 2, (1 << 127) | 0xFFFFFFFF_FFFFFFFF_FFFFFFFF, 1, 2])
               if rng.random() < 0.3 else rng.randrange(M)) for k in kinds]
        got = run_case(kinds, lines, opn, nv, uv, vv, wv)
        for b in range(nb):
            w = wv[b] if kinds[b] in ("m", "p", "f") else 1
            a, d = got[b]
            if kinds[b] in ("p", "f"):
                assert 0 <= d < (1 << 128) and d % M == (w * vv[b]) % M, (kinds, b, vv[b], w)
                checked += 1
                continue
            if kinds[b] == "c":
                assert d == vv[b] % M, (kinds, b, vv[b])
                checked += 1
                continue
            assert 0 <= a < (1 << 128) and 0 <= d < (1 << 128)
            assert a % M == (uv[b] + w * vv[b]) % M, (kinds, b, uv[b], vv[b], w)
            assert d % M == (uv[b] - w * vv[b]) % M, (kinds, b, uv[b], vv[b], w)
            checked += 1
    return checked


def twiddle_precondition():
    """Max of w's limbs 1..3 over all roots of order <= 2^9 except -1."""
    g = pow(3, (M - 1) >> 9, M)
    worst = 0
    for e in range(512):
        w = pow(g, e, M)
        if w == M - 1:
            continue
        worst = max(worst, max(limbs(w)[1:]))
    return worst


# ------------------------------------------------------------ C++ header ---

VARIANTS = [("m", "m"), ("m",), ("t", "t"), ("t",), ("m", "t"), ("p", "p"), ("p",), ("f", "f"), ("f",),
            ("c", "c", "c", "c"), ("c",)]


def cxx_function(kinds, bsrc):
    lines, outs, flags, ins, ns, nv, opn = render(kinds, bsrc)
    fname = "bfly_%s_%s" % ("".join(kinds), bsrc)
    nb = len(kinds)
    args = []
    for b in range(nb):
        args += (["fe& u%d" % b] if has_u(kinds[b]) else []) + ["fe& v%d" % b]
        if kinds[b] in ("m", "p"):
            args += ["const fe& B%d_%d" % (b, k) for k in range(4)]
        if kinds[b] == "f":
            args.append("const fe& W%d" % b)
    if flags:
        args += ["uint64_t& rare"]
    body = []
    for f in flags:
        body.append("  uint64_t %s;" % f)
    if ns:
        body.append("  uint64_t st[%d];" % ns)
    body.append("  uint64_t junk;")
    if "kc1" in ins:
        body.append("  const uint32_t kc1 = 0x2CFFu;")
    if "k2d00" in ins:
        body.append("  const uint32_t k2d00 = 0x2D00u;")
    asm = "\\n\\t".join(lines)
    ol = []
    for o in outs:
        b, i = o[1:].split("_")
        ol.append('"+v"(%s%s.w[%s])' % (o[0], b, i))
    for f in flags:
        ol.append('"=&s"(%s)' % f)
    for s in range(ns):
        ol.append('"=&s"(st[%d])' % s)
    ol.append('"=&s"(junk)')
    il = []
    for i in ins:
        if i == "kc1":
            il.append('"v"(kc1)')
        elif i == "k2d00":
            il.append('"s"(k2d00)')
        elif i[0] == "W":
            b, j = i[1:].split("_")
            il.append('"v"(W%s.w[%s])' % (b, j))
        else:
            b, kj = i[1:].split("_")
            il.append('"%s"(B%s_%s.w[%s])' % (bsrc, b, kj[0], kj[1]))
    clob = ", ".join('"v%d"' % (VBASE + r) for r in range(nv))
    body.append('  asm volatile(\n      "%s"\n      : %s\n      : %s\n      : %s);' % (
        asm, ",\n        ".join(ol), ",\n        ".join(il), clob))
    if flags:
        body.append("  rare = %s;" % " | ".join(flags))
        body.append("  if (__builtin_expect(rare != 0, 0)) {")
    for b in range(nb):
        if kinds[b] in ("p", "f"):
            body.append("    if ((K%d >> __lane_id()) & 1u) v%d = relaxed_add_c(v%d);" % (b, b, b))
        elif kinds[b] != "c":
            fk = "K%d" % b if kinds[b] == "m" else "0ull"
            body.append("    bfly_fix(u%d, v%d, %s, C2%d, B2%d);" % (b, b, fk, b, b))
    if flags:
        body.append("  }")
    stats = "%d VALU, %d s_nop, %d VGPR temps, %d SGPR-pair temps" % (
        sum(1 for l in lines if l.startswith("v_")), sum(1 for l in lines if l.startswith("s_nop")), nv, ns)
    return fname, "// %s\n__device__ __forceinline__ void %s(%s) {\n%s\n}\n" % (
        stats, fname, ", ".join(args), "\n".join(body)), lines


HEADER = """// GENERATED by tools/gen_bfly.py -- do not edit by hand.
//
// Hand-scheduled gfx950 radix-2 DIT butterflies over F_M in the relaxed
// representation (any residue in [0, 2^128)); see tools/gen_bfly.py for the
// algorithm, the hazard rule they are scheduled for and the emulator that
// checks them (tests/test_bfly_asm.py).  (u, v) -> (u + w v, u - w v), w given
// as its expanded multiples B_k = w 2^(32k) mod M (stage twiddle tables).
// Temporaries use physical VGPRs v0..; the statements clobber them.
#pragma once
#include "field.hpp"

namespace mlh {

// Relaxed x + C / x - C (one wrap corrected; the second cannot wrap).
__device__ __forceinline__ fe relaxed_add_c(const fe& x) {
  uint32_t k;
  fe t = add_c(x, &k);
  if (k) {
    uint32_t k2;
    t = add_c(t, &k2);
  }
  return t;
}
__device__ __forceinline__ fe relaxed_sub_c(const fe& x) {
  fe t;
  uint32_t b;
  t.w[0] = subb(x.w[0], kC0, 0u, &b);
  t.w[1] = subb(x.w[1], kC1, b, &b);
  t.w[2] = subb(x.w[2], 0u, b, &b);
  t.w[3] = subb(x.w[3], 0u, b, &b);
  if (b) {
    t.w[0] = subb(t.w[0], kC0, 0u, &b);
    t.w[1] = subb(t.w[1], kC1, b, &b);
    t.w[2] = subb(t.w[2], 0u, b, &b);
    t.w[3] = subb(t.w[3], 0u, b, &b);
  }
  return t;
}

// Cold path: this lane's flags (K: the product wrapped, true t = s + C;
// C2: a second carry in u + t; B2: a second borrow in u - t).
__device__ __forceinline__ void bfly_fix_lane(fe& a, fe& d, uint32_t fk, uint32_t fc, uint32_t fb) {
  if (fk) {
    a = relaxed_add_c(a);
    d = relaxed_sub_c(d);
  }
  if (fc) a = relaxed_add_c(a);
  if (fb) d = relaxed_sub_c(d);
}
__device__ __forceinline__ void bfly_fix(fe& a, fe& d, uint64_t fk, uint64_t fc, uint64_t fb) {
  const uint32_t lane = __lane_id();
  bfly_fix_lane(a, d, (uint32_t)(fk >> lane) & 1u, (uint32_t)(fc >> lane) & 1u, (uint32_t)(fb >> lane) & 1u);
}

// Canonical representative of a relaxed value (x < 2^128 < 2M).
__device__ __forceinline__ fe relaxed_canon(const fe& x) { return canon_with_carry(x, 0u); }

"""


def main():
    parts = [HEADER]
    total = 0
    for kinds in VARIANTS:
        for bsrc in ("s", "v"):
            if not any(k in ("m", "p") for k in kinds) and bsrc == "s":
                continue
            fname, code, lines = cxx_function(kinds, bsrc)
            _, _, _, _, _, nv, opn = render(kinds, bsrc)
            check_hazards(lines)
            total += selftest(kinds, lines, opn, nv, trials=400)
            parts.append(code)
    parts.append("}  // namespace mlh\n")
    open(OUT, "w").write("\n".join(parts))
    print("wrote", OUT, "emulated butterflies:", total, "twiddle max limb:", hex(twiddle_precondition()))


if __name__ == "__main__":
    main()
