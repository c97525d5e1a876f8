"""Static per-wave instruction counts of the straight-line NTT pass kernels
(fully unrolled: static count = executed count per wave, except the
butterflies' out-of-line rare-correction blocks, counted apart as valu_cold /
s_nop_cold).  Compiles ntt.hip for gfx950 to assembly and writes
profiles/isa_counts.json:
  {"ntt_pass<8,0,0>": {"valu": .., "mad_u64": .., "salu": .., "lds": .., "vmem": ..,
                       "vgpr": .., "ept": 8}, ...}
Run on the build host (no GPU):  python tools/isa_counts.py"""
import collections
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "multilinear_amd", "csrc", "ntt.hip")


def cold_lines(lines):
    """Line numbers of the out-of-line blocks of the butterflies' rare-case
    branches (bfly_asm.hpp `rare`): a conditional branch whose target chain
    ends in an `s_branch` back to the branch's own fall-through label.  The
    hot path -- what every wave executes -- is everything else."""
    label_at = {}
    for i, l in enumerate(lines):
        m = re.match(r"(\.LBB\w+):", l)
        if m:
            label_at[m.group(1)] = i
    cold = set()
    for i, l in enumerate(lines):
        m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\w+)", l)
        if not m or m.group(1) not in label_at:
            continue
        j = i + 1  # fall-through label
        while j < len(lines) and not re.match(r"\.LBB\w+:", lines[j]):
            if re.match(r"\s+[vs]_", lines[j]):
                j = None
                break
            j += 1
        if j is None or j >= len(lines):
            continue
        fall = re.match(r"(\.LBB\w+):", lines[j]).group(1)
        t = label_at[m.group(1)]
        if t < i:
            continue
        for k in range(t, len(lines)):
            b = re.match(r"\s+s_branch\s+(\.LBB\w+)", lines[k])
            if b:
                if b.group(1) == fall:
                    cold.update(range(t, k + 1))
                break
    return cold


def main():
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "ntt.s")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                               "--cuda-device-only", "-S", "-o", asm, SRC], cwd=td)
        text = open(asm).read()
    out = {}
    # kernel bodies: "<mangled>:  ; @<mangled>" ... "s_endpgm"
    for m in re.finditer(r"\n(_ZN3mlh15ntt_pass_kernelILi(\d+)ELi(\d)ELi(\d)ELi(\d+)\w*):\s*;\s*@",
                         text):
        name, logr, tw, zt, ept = m.group(1), m.group(2), m.group(3), m.group(4), m.group(5)
        end = text.index("s_endpgm", m.end())
        body = text[m.end():end]
        lines = body.split("\n")
        cold = cold_lines(lines)
        c = collections.Counter()
        for ln, line in enumerate(lines):
            t = re.match(r"\s+([vsdgb][a-z_0-9]+)", line)
            if not t:
                continue
            op = t.group(1)
            if ln in cold:  # out-of-line rare-correction code (not executed in practice)
                if op.startswith("v_"):
                    c["valu_cold"] += 1
                elif op == "s_nop":
                    c["s_nop_cold"] += 1
                continue
            if op.startswith("v_"):
                c["valu"] += 1
                if op == "v_mad_u64_u32":
                    c["mad_u64"] += 1
            elif op.startswith("s_") and not op.startswith(("s_nop", "s_waitcnt", "s_barrier",
                                                            "s_endpgm", "s_cbranch", "s_branch")):
                c["salu"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith(("global_", "buffer_")):
                c["vmem"] += 1
            if op == "s_nop":
                c["s_nop"] += 1
        meta = re.search(r"\.name:\s+%s\s*\n(.*?)\.vgpr_count:\s+(\d+)" % re.escape(name), text, re.S)
        lab = "ntt_pass<%s,%s,%s>" % (logr, tw, zt)
        if int(ept) != 8:
            lab += "/ept%s" % ept
        out[lab] = dict(c, ept=int(ept), vgpr=int(meta.group(2)) if meta else None)
    dst = os.path.join(ROOT, "profiles", "isa_counts.json")
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print("wrote", dst, "kernels:", len(out))


if __name__ == "__main__":
    main()
