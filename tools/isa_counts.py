"""Static per-wave instruction counts of the straight-line NTT pass kernels
(fully unrolled: static count = executed count per wave), for the VALU issue
model in bench.py.  Compiles ntt.hip for gfx950 to assembly and writes
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


def main():
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "ntt.s")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                               "--cuda-device-only", "-S", "-o", asm, SRC], cwd=td)
        text = open(asm).read()
    out = {}
    # kernel bodies: "<mangled>:  ; @<mangled>" ... "s_endpgm"
    for m in re.finditer(r"\n(_ZN3mlh15ntt_pass_kernelILi(\d)ELi(\d)ELi(\d)ELi(\d+)\w*):\s*;\s*@",
                         text):
        name, logr, tw, zt, ept = m.group(1), m.group(2), m.group(3), m.group(4), m.group(5)
        end = text.index("s_endpgm", m.end())
        body = text[m.end():end]
        c = collections.Counter()
        for line in body.split("\n"):
            t = re.match(r"\s+([vsdgb][a-z_0-9]+)", line)
            if not t:
                continue
            op = t.group(1)
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
