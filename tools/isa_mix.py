"""Instruction-mix VALU ceilings of the SHA-256 and NTT kernels (VERDICT r04
item 6).  Run on the build host (no GPU):  python tools/isa_mix.py

The "one wave64 VALU instruction per 4 cycles per SIMD" ceiling (bench.py
VALU_PEAK) is the rate of the VOP3 integer instructions; plain VOP2
instructions without a carry issue faster (profiles/r04_isa.json: v_add_u32_e32
2.41, v_xor_b32_e32 2.24 cycles) and v_mad_u64_u32 slower (~5.2).  A kernel's
true issue ceiling is therefore its instruction mix weighted by those measured
rates.  This tool compiles the kernels to gfx950 assembly, counts the VALU
instructions of the path every wave executes (the SHA kernels are straight
line; the NTT passes' out-of-line carry-fix blocks and fri_fold_leaves_kernel's
PCS-round branch are excluded), classifies them, and writes
profiles/r05_isa_mix.json:

  cycles_per_instr = sum(count_c * rate_c) / sum(count_c)
  mix_ceiling      = 256 CU x 4 SIMD x 64 lanes x clock / cycles_per_instr
  issue_frac_vs_mix = measured lane-instr/s / mix_ceiling

with the measured lane-instr/s and clock of the newest committed VALU pass
(profiles/*_valu.json, rocprofv3 SQ_INSTS_VALU and GRBM_GUI_ACTIVE).
Classes without a measured rate take the nearest measured one (named in
"rate_basis")."""
import collections
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "multilinear_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))

CARRY = {"v_add_co_u32_e32", "v_addc_co_u32_e32", "v_sub_co_u32_e32", "v_subb_co_u32_e32",
         "v_subrev_co_u32_e32", "v_subbrev_co_u32_e32", "v_cndmask_b32_e32"}


def rates():
    d = json.load(open(os.path.join(ROOT, "profiles", "r04_isa.json")))
    by = {e["instr"].split()[0]: e["cycles_per_wave_instr_per_simd_at_2p4"] for e in d["per_instruction"]}
    vop3 = [by[k] for k in ("v_add3_u32", "v_alignbit_b32", "v_mul_lo_u32", "v_mul_hi_u32",
                            "v_cndmask_b32_e64")]
    mad = [e for e in d["per_instruction"] if e["instr"].startswith("v_mad_u64_u32")][0]
    return {
        "vop2_plain": ((by["v_add_u32_e32"] + by["v_xor_b32_e32"]) / 2,
                       "mean of v_add_u32_e32 and v_xor_b32_e32 (other carry-free VOP1/VOP2 assumed alike)"),
        "vop2_carry": (by["v_add_co_u32_e32"], "v_add_co_u32_e32 (carry in/out through vcc)"),
        "bitop3": (by["v_bitop3_b32"], "v_bitop3_b32"),
        "mad_u64": (2 * mad["cycles_per_wave_instr_per_simd_at_2p4"] - by["v_xor_b32_e32"],
                    "v_mad_u64_u32 + v_xor pair minus the xor"),
        "vop3": (sum(vop3) / len(vop3), "mean of v_add3_u32, v_alignbit_b32, v_mul_lo/hi_u32, "
                                        "v_cndmask_b32_e64 (other VOP3/VOP3P/DPP/lane ops assumed alike)"),
    }


def klass(op):
    if op == "v_bitop3_b32":
        return "bitop3"
    if op == "v_mad_u64_u32":
        return "mad_u64"
    if op in CARRY:
        return "vop2_carry"
    if op.endswith("_e32") and not op.startswith("v_cmp"):
        return "vop2_plain"
    return "vop3"


def asm(src):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                               "--cuda-device-only", "-S", "-o", out, os.path.join(CSRC, src)], cwd=td,
                              stderr=subprocess.DEVNULL)
        return open(out).read()


def body(text, pattern):
    m = re.search(r"\n(" + pattern + r"):\s*;\s*@", text)
    end = text.index("s_endpgm", m.end())
    return m.group(1), text[m.end():end].split("\n")


def count(lines, skip=()):
    c = collections.Counter()
    for i, l in enumerate(lines):
        if i in skip:
            continue
        t = re.match(r"\s+(v_[a-z_0-9]+)", l)
        if t:
            c[t.group(1)] += 1
    return c


def after_first_branch(lines):
    """Lines before the target of the kernel's first conditional branch: the
    branch taken when the fold launch carries no PCS round (job.st == 0) skips
    them (fri.hip fri_fold_leaves_kernel: `if (job.st && last block)`)."""
    for l in lines:
        m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\w+)", l)
        if m:
            tgt = m.group(1)
            start = [i for i, x in enumerate(lines) if x.startswith(tgt + ":")][0]
            return set(range(0, start))
    return set()


def main():
    from isa_counts import cold_lines

    R = rates()
    kernels = []
    merkle = asm("merkle.hip")
    fri = asm("fri.hip")
    ntt = asm("ntt.hip")
    for name, text, pat, skip_fn, valu_key in (
            ("leaf_pairs_level2_kernel", merkle, r"_ZN3mlh24leaf_pairs_level2_kernel\w*", None,
             "mlh::leaf_pairs_level2_kernel"),
            ("level2_kernel", merkle, r"_ZN3mlh13level2_kernel\w*", None, "mlh::level2_kernel"),
            ("fri_fold_leaves_kernel", fri, r"_ZN3mlh22fri_fold_leaves_kernel\w*", after_first_branch,
             "mlh::fri_fold_leaves_kernel"),
            ("ntt_pass_kernel<8, 0, 0, 8>", ntt, r"_ZN3mlh15ntt_pass_kernelILi8ELi0ELi0ELi8\w*", cold_lines,
             "void mlh::ntt_pass_kernel<8, 0, 0, 8>"),
            ("ntt_pass_kernel<8, 1, 0, 8>", ntt, r"_ZN3mlh15ntt_pass_kernelILi8ELi1ELi0ELi8\w*", cold_lines,
             "void mlh::ntt_pass_kernel<8, 1, 0, 8>"),
            ("ntt_pass_kernel<8, 2, 0, 8>", ntt, r"_ZN3mlh15ntt_pass_kernelILi8ELi2ELi0ELi8\w*", cold_lines,
             "void mlh::ntt_pass_kernel<8, 2, 0, 8>"),
            ("ntt_pass_kernel<9, 0, 1, 8>", ntt, r"_ZN3mlh15ntt_pass_kernelILi9ELi0ELi1ELi8\w*", cold_lines,
             "void mlh::ntt_pass_kernel<9, 0, 1, 8>")):
        _, lines = body(text, pat)
        skip = skip_fn(lines) if skip_fn else set()
        c = count(lines, skip)
        by = collections.Counter()
        for op, n in c.items():
            by[klass(op)] += n
        total = sum(by.values())
        cyc = sum(n * R[k][0] for k, n in by.items())
        kernels.append((name, valu_key, {
            "valu_per_wave_static": total,
            "by_class": dict(by),
            "top_ops": dict(c.most_common(8)),
            "cycles_per_wave_at_mix": round(cyc, 1),
            "cycles_per_instr": round(cyc / total, 3),
            "mix_vs_4cycle": round(4.0 / (cyc / total), 4),
        }))
    vpaths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_valu.json")), reverse=True)
    vd = json.load(open(vpaths[0]))
    out = {"tool": "tools/isa_mix.py", "valu_source": os.path.basename(vpaths[0]),
           "rates_cycles_per_wave_instr": {k: round(v[0], 3) for k, v in R.items()},
           "rate_basis": {k: v[1] for k, v in R.items()},
           "rate_source": "profiles/r04_isa.json (tools/isa_bench3.hip, 8 independent chains per lane, "
                          "8 waves per SIMD)",
           "kernels": {}}
    for name, vk, rec in kernels:
        m = vd["kernels"].get(vk)
        if m and m.get("eff_clock_ghz"):
            clk = min(m["eff_clock_ghz"], 2.4)
            ceil = 256 * 4 * 64 * clk * 1e9 / rec["cycles_per_instr"]
            dyn = m["SQ_INSTS_VALU"]
            rec.update({
                "measured_lane_instr_per_s": m["lane_instr_per_s"], "clock_ghz": clk,
                "mix_ceiling_lane_instr_per_s": ceil,
                "issue_frac_vs_4cycle": m["lane_instr_per_s"] / (256 * 4 * 16 * clk * 1e9),
                "issue_frac_vs_mix": m["lane_instr_per_s"] / ceil,
                "avg_ms": m["avg_ms"], "SQ_INSTS_VALU_per_dispatch": dyn,
            })
        out["kernels"][name] = rec
    path = os.path.join(ROOT, "profiles", "r05_isa_mix.json")
    json.dump(out, open(path, "w"), indent=1)
    for k, v in out["kernels"].items():
        print("%-30s valu/wave %6d  cyc/instr %.3f  mix/4cyc %.3f  vs4 %.3f  vsmix %.3f" % (
            k, v["valu_per_wave_static"], v["cycles_per_instr"], v["mix_vs_4cycle"],
            v.get("issue_frac_vs_4cycle", float("nan")), v.get("issue_frac_vs_mix", float("nan"))))


if __name__ == "__main__":
    main()
