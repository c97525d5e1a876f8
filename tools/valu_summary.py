"""VALU-boundedness summary from one rocprofv3 pass with
--pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
--kernel-trace (dev tool) -> profiles/<tag>_valu.json.

Per kernel (averaged over its dispatches):
  lane_instr_per_s = SQ_INSTS_VALU * 64 / kernel duration   (wave-instructions x 64 lanes)
  frac_nominal     = that / 7.864e13 (256 CU x 4 SIMD x 32 lanes x 2.4 GHz)
  valu_active_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   (share of wave lifetime issuing VALU;
                     both in quad-cycles)
usage: python tools/valu_summary.py <tag> <pmc_dir> [kernel substrings...]
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NOMINAL = 7.864e13


def main():
    tag, d = sys.argv[1], sys.argv[2]
    want = sys.argv[3:] or ["ntt_pass", "level2", "leaf_pairs", "fri_fold_leaves", "top_kernel",
                            "fold_sums", "shard_dft", "mobius", "group_sums", "fold_group", "sumcheck_", "subtree"]
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        ctr[r["Kernel_Name"]][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    dur = {}
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {"round": tag, "log_n": 24, "nominal_lane_instr_per_s": NOMINAL, "kernels": {}}
    for name, cs in ctr.items():
        if not any(w in name for w in want):
            continue
        # per dispatch: sum counter values (one row per dimension/XCD)
        per = collections.defaultdict(dict)
        for cname, vals in cs.items():
            acc = collections.defaultdict(float)
            for did, v in vals:
                acc[did] += v
            for did, v in acc.items():
                per[did][cname] = v
        rows = [(did, c) for did, c in per.items() if did in dur and "SQ_INSTS_VALU" in c]
        if not rows:
            continue
        t = sum(dur[did] for did, _ in rows) / len(rows)
        insts = sum(c["SQ_INSTS_VALU"] for _, c in rows) / len(rows)
        act = sum(c.get("SQ_ACTIVE_INST_VALU", 0) for _, c in rows) / len(rows)
        wav = sum(c.get("SQ_WAVE_CYCLES", 0) for _, c in rows) / len(rows)
        grbm = sum(c.get("GRBM_GUI_ACTIVE", 0) for _, c in rows) / len(rows)
        rate = insts * 64 / t if t else 0
        short = name.split("(")[0]
        out["kernels"][short] = {
            "dispatches": len(rows), "avg_ms": t * 1e3, "SQ_INSTS_VALU": insts,
            "lane_instr_per_s": rate, "frac_nominal": rate / NOMINAL,
            "valu_active_frac": act / wav if wav else None,
            # MI355X_MICROARCH.md "DVFS give-back": GRBM_GUI_ACTIVE summed over the
            # 8 XCDs / 8 / wall time (reads high on dispatches under ~0.3 ms)
            "eff_clock_ghz": grbm / 8 / t / 1e9 if (grbm and t) else None,
        }
    path = os.path.join(ROOT, "profiles", "%s_valu.json" % tag)
    json.dump(out, open(path, "w"), indent=1)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["avg_ms"]):
        print("%-45s %8.3f ms  %.2e lane-instr/s  %.0f%% nominal  VALU-active %s  clock %s" % (
            k[:45], v["avg_ms"], v["lane_instr_per_s"], 100 * v["frac_nominal"],
            "%.0f%%" % (100 * v["valu_active_frac"]) if v["valu_active_frac"] is not None else "-",
            "%.2f GHz" % v["eff_clock_ghz"] if v["eff_clock_ghz"] else "-"))


if __name__ == "__main__":
    main()
