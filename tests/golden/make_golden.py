"""Generate tests/golden/golden.json from the exact Python restatement of the
reference (oracle/).  The reference itself (Rust, winter-math, sha2) cannot be
built here and its own tests hold no absolute vectors, so
these fixtures pin the *oracle* against drift and give the GPU tests stored
known answers; their provenance is this script.

    python tests/golden/make_golden.py   # rewrites golden.json
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import field as F  # noqa: E402
from oracle import fri as OF  # noqa: E402
from oracle import ntt as ON  # noqa: E402
from oracle import pcs as OP  # noqa: E402
from oracle import polynomials as OPL  # noqa: E402
from oracle import sumcheck as OS  # noqa: E402
from oracle import transcript as OT  # noqa: E402


def h(v):
    return "%032x" % v


def digest(values):
    return hashlib.sha256(b"".join(F.to_bytes(v) for v in values)).hexdigest()


def main():
    g = {}
    g["modulus"] = str(F.M)
    g["pow_2_generator"] = {str(k): h(F.pow_2_generator(k)) for k in range(0, 41)}
    a, b = 0x0123456789ABCDEF0FEDCBA987654321, 0xFFFFFFFFFFFFFFFFFFFFD30000000000
    g["mul_kat"] = [[h(a), h(b), h(F.mul(a, b))], [h(F.M - 1), h(F.M - 1), h(F.mul(F.M - 1, F.M - 1))]]
    g["from_i64_minus1"] = str(F.from_i64(-1))
    # NTT: coeffs = 0..n-1 (ntt/mod.rs:185 pattern)
    ntt = {}
    for ln in range(1, 13):
        n = 1 << ln
        c = [F.from_i64(i) for i in range(n)]
        ev = ON.ntt(c, F.pow_2_generator(ln))
        ntt[str(ln)] = {"sha256": digest(ev), "head": [h(v) for v in ev[:4]]}
    g["ntt_coeffs_0_to_n"] = ntt
    g["ntt_full_2_4"] = [h(v) for v in ON.ntt([F.from_i64(i) for i in range(16)], F.pow_2_generator(4))]
    # RS + Merkle + FRI (fri/mod.rs:349-363: values 7i+3, log_n = 10)
    ln = 10
    vals = [F.from_i64(7 * i + 3) for i in range(1 << ln)]
    gp = F.pow_2_generator_powers(ln + 1)
    code = OF.reed_solomon(vals, gp[1])
    proof = OF.FriProof.prove(code, gp, OT.Transcript())
    qd = hashlib.sha256()
    for q in proof.queries:
        for value, path in q:
            qd.update(value)
            for sib, d in path:
                qd.update(sib + bytes([d]))
    g["fri_7i3_log10"] = {
        "code_sha256": digest(code),
        "rs_root": OF.commit_rs_code(code).root().hex(),
        "commitments": [c.hex() for c in proof.commitments],
        "last_elem": h(proof.last_elem),
        "last_random": proof.last_random.hex(),
        "queries_sha256": qd.hexdigest(),
    }
    # sumcheck + PCS (multilinear_pcs.rs:210-228 pattern at n = 10)
    n = 10
    ev = [F.from_i64(7 * i + 3) for i in range(1 << n)]
    pts = [F.from_i64(i) for i in range(n)]
    out = OPL.mle_evaluate(ev, pts)
    g["mle_eval_7i3_point_0_to_9"] = h(out)
    g["eq_table_point_0_to_9_sha256"] = digest(OS.eq_table(pts))
    g["to_coefficient_7i3_sha256"] = digest(OPL.to_coefficient(ev))
    pcs = OP.PCSProof.prove(pts, out, ev, OT.Transcript())
    g["pcs_7i3_n10"] = {
        "sumcheck_polys": [[h(c) for c in p] for p in pcs.sumcheck_polynomials],
        "commitments": [c.hex() for c in pcs.fri_proof.commitments],
        "last_elem": h(pcs.fri_proof.last_elem),
        "last_random": pcs.fri_proof.last_random.hex(),
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    with open(path, "w") as f:
        json.dump(g, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
