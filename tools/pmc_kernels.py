"""Per-kernel averages of any rocprofv3 --pmc pass (dev tool).

usage: python tools/pmc_kernels.py <pmc_dir> [kernel substrings...]
Prints, per kernel: dispatches, avg duration (kernel trace) and every counter
summed over its dimensions and averaged over dispatches; with SQ_WAVE_CYCLES
present, the SQ_WAIT_* / SQ_ACTIVE_* counters also as fractions of it."""
import collections
import csv
import os
import sys


def main():
    d = sys.argv[1]
    want = sys.argv[2:]
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
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    agg = collections.defaultdict(list)
    for did, cs in per.items():
        agg[names[did]].append((did, cs))
    for name, rows in sorted(agg.items(), key=lambda kv: -len(kv[1])):
        if want and not any(w in name for w in want):
            continue
        n = len(rows)
        avg = collections.defaultdict(float)
        for _, cs in rows:
            for k, v in cs.items():
                avg[k] += v / n
        ms = [dur[did] for did, _ in rows if did in dur]
        print("%s  dispatches=%d  avg_ms=%s" % (name[:90], n, "%.4f" % (sum(ms) / len(ms)) if ms else "-"))
        wc = avg.get("SQ_WAVE_CYCLES")
        for k in sorted(avg):
            extra = ""
            if wc and k != "SQ_WAVE_CYCLES" and k.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_LDS")):
                extra = "  (%.3f of wave cycles)" % (avg[k] / wc)
            print("   %-28s %.4g%s" % (k, avg[k], extra))


if __name__ == "__main__":
    main()
