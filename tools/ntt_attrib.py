"""Summarise tools/run_ntt_attrib.sh's three rocprofv3 --pmc passes into
profiles/<tag>_ntt_pass_attrib.json: per 2^24 NTT pass (pass 0, 1, last),
per-dispatch counter averages and the per-wave readings that attribute pass
0's and the last pass's lower VALU issue rate.

  per wave: VALU / LDS / SALU / SMEM / VMEM instructions (SQ_INSTS_* / SQ_WAVES)
  fractions of wave time (quad-cycles, MI355X_MICROARCH.md: WAIT_ANY +
  WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES): parked (SQ_WAIT_ANY),
  issue-stalled (SQ_WAIT_INST_ANY, of which LDS issue SQ_WAIT_INST_LDS),
  VALU / LDS / scalar active
  occupancy: SQ_LEVEL_WAVES / SQ_BUSY_CYCLES (mean resident waves per SQ)
  issue: SQ_INSTS_VALU x 64 / (duration x 256 CU x 4 SIMD x 16 lanes x clock),
  clock = GRBM_GUI_ACTIVE / 8 / duration

usage: python tools/ntt_attrib.py gpurun_out/r05_attrib [out.json]"""
import collections
import csv
import json
import os
import sys

PASSES = {"ntt_pass_kernel<8, 0, 0, 8>": "pass 0", "ntt_pass_kernel<8, 1, 0, 8>": "pass 1",
          "ntt_pass_kernel<8, 2, 0, 8>": "last pass"}
if os.environ.get("MLH_ATTRIB_KERNELS"):  # e.g. "leaf_pairs_level2_kernel,level2_kernel"
    PASSES = {k: k for k in os.environ["MLH_ATTRIB_KERNELS"].split(",")}


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        did = int(r["Dispatch_Id"])
        names[did] = r["Kernel_Name"]
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = {}
    p = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for key in PASSES:
        rows = [(did, cs) for did, cs in per.items()
                if ("mlh::" + key + "(") in names[did] or ("mlh::" + key + "<") in names[did]
                or names[did].endswith("mlh::" + key)]
        if not rows:
            continue
        avg = collections.defaultdict(float)
        for _, cs in rows:
            for k, v in cs.items():
                avg[k] += v / len(rows)
        ds = [dur[did] for did, _ in rows if did in dur]
        avg["_dispatches"] = len(rows)
        avg["_duration_s"] = sum(ds) / len(ds) if ds else float("nan")
        out[key] = dict(avg)
    return out


def main():
    base = sys.argv[1]
    tag = os.path.basename(base.rstrip("/"))
    outp = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "%s_ntt_pass_attrib.json" % tag.split("_")[0])
    merged = collections.defaultdict(dict)
    for sfx in "abc":
        d = base + "_" + sfx
        if not os.path.isdir(d):
            continue
        for k, v in load(d).items():
            for c, x in v.items():
                if c.startswith("_"):
                    merged[k].setdefault(c + "_" + sfx, x)
                else:
                    merged[k][c] = x
    res = {"tool": "tools/run_ntt_attrib.sh + tools/ntt_attrib.py", "passes": {}}
    for k, a in merged.items():
        w = a.get("SQ_WAVES") or float("nan")
        t = a.get("_duration_s_a", float("nan"))
        clk = a.get("GRBM_GUI_ACTIVE", float("nan")) / 8 / t
        wc = a.get("SQ_WAVE_CYCLES", float("nan"))
        rd = {
            "what": PASSES[k], "dispatches": a.get("_dispatches_a"), "avg_ms": t * 1e3,
            "clock_ghz": clk / 1e9,
            "per_wave": {n: a[c] / w for n, c in (("valu", "SQ_INSTS_VALU"), ("lds", "SQ_INSTS_LDS"),
                                                 ("salu", "SQ_INSTS_SALU"), ("smem", "SQ_INSTS_SMEM"),
                                                 ("vmem_rd", "SQ_INSTS_VMEM_RD"),
                                                 ("vmem_wr", "SQ_INSTS_VMEM_WR")) if c in a},
            "wave_cycles_per_wave": wc / w * 4,
            "frac_of_wave_time": {n: a[c] / wc for n, c in (("parked_WAIT_ANY", "SQ_WAIT_ANY"),
                                                            ("issue_stall_WAIT_INST_ANY", "SQ_WAIT_INST_ANY"),
                                                            ("lds_issue_stall_WAIT_INST_LDS", "SQ_WAIT_INST_LDS"),
                                                            ("valu_active", "SQ_ACTIVE_INST_VALU"),
                                                            ("lds_active", "SQ_ACTIVE_INST_LDS"),
                                                            ("scalar_active", "SQ_ACTIVE_INST_SCA"),
                                                            ("misc_active", "SQ_ACTIVE_INST_MISC"),
                                                            ("lds_bank_conflict", "SQ_LDS_BANK_CONFLICT"))
                                  if c in a},
            "mean_resident_waves_per_sq": a["SQ_LEVEL_WAVES"] / a["SQ_BUSY_CYCLES"]
            if a.get("SQ_LEVEL_WAVES") and a.get("SQ_BUSY_CYCLES") else None,  # (reads 0 on gfx950)
            "valu_issue_frac_4cycle": a["SQ_INSTS_VALU"] * 64 / (t * 256 * 4 * 16 * clk)
            if "SQ_INSTS_VALU" in a else None,
            "ta_busy_avr": a.get("TA_BUSY_avr"), "ta_busy_max": a.get("TA_BUSY_max"),
            "td_busy_avr": a.get("TD_BUSY_avr"),
            "tcp_accesses": a.get("TCP_TOTAL_CACHE_ACCESSES_sum"),
            "tcp_tcc_read_req": a.get("TCP_TCC_READ_REQ_sum"),
            "raw": {c: v for c, v in a.items()},
        }
        res["passes"][PASSES[k]] = rd
    json.dump(res, open(outp, "w"), indent=1)
    for n, r in res["passes"].items():
        print(n, json.dumps({k: r[k] for k in ("avg_ms", "clock_ghz", "per_wave", "frac_of_wave_time",
                                                 "mean_resident_waves_per_sq", "valu_issue_frac_4cycle",
                                                 "ta_busy_avr")}, indent=None))
    print("->", outp)


if __name__ == "__main__":
    main()
