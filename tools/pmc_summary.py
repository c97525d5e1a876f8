"""Summarise rocprofv3 outputs into profiles/ (tracked).

usage: python tools/pmc_summary.py <round-tag> <ktrace_dir> <fetch_dir> <write_dir> [log_n]

* copies <ktrace_dir>/run_kernel_stats.csv -> profiles/<tag>_kernel_stats.csv
* writes profiles/pmc_ntt.json: HBM traffic per launch of the dominant NTT
  pass kernel, from separate FETCH_SIZE and WRITE_SIZE passes, corrected as
  MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE (KiB) reads half the bytes
  of a wide coalesced stream on gfx950 -> x2; WRITE_SIZE (KiB) is exact for
  16-B-per-lane stores.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LABELS = ["ntt_pass<%d,%d,%d>" % (r, tw, z) for r in range(4, 10) for tw in (0, 1, 2, 3, 5) for z in range(3)]


def prefix(label):
    """kernel-timer label "ntt_pass<8,0,0>" -> demangled rocprof kernel name prefix"""
    r, tw, z = label[len("ntt_pass<"):-1].split(",")
    return "void mlh::ntt_pass_kernel<%s, %s, %s>" % (r, tw, z)  # ZT is an int template arg


def norm(kernel_name):
    """rocprof kernel name -> prefix() form (drops the argument list and the
    EPT = 8 template argument: "ntt_pass_kernel<8, 0, 0, 8>" -> "<8, 0, 0>")"""
    k = kernel_name.split("(")[0]
    return k[:-len(", 8>")] + ">" if k.endswith(", 8>") else k


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    tag, kdir, fdir, wdir = sys.argv[1:5]
    log_n = int(sys.argv[5]) if len(sys.argv) > 5 else 24
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(kdir, "run_kernel_stats.csv"), os.path.join(prof, "%s_kernel_stats.csv" % tag))
    fetch = per_kernel(os.path.join(fdir, "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(wdir, "run_counter_collection.csv"), "WRITE_SIZE")
    out = {"log_n": log_n, "round": tag,
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE counts "
                         "half of a wide stream)",
           "alg_bytes_per_launch": 32 * (1 << log_n), "kernels": {}}
    for label in LABELS:
        pre = prefix(label)
        fk = [v for k, vs in fetch.items() if norm(k) == pre for v in vs]
        wk = [v for k, vs in write.items() if norm(k) == pre for v in vs]
        if not fk or not wk:
            continue
        f_kib = sum(fk) / len(fk)
        w_kib = sum(wk) / len(wk)
        out["kernels"][label] = {
            "launches_fetch_pass": len(fk),
            "launches_write_pass": len(wk),
            "FETCH_SIZE_KiB_avg": f_kib,
            "WRITE_SIZE_KiB_avg": w_kib,
            "traffic_bytes_per_launch": (2.0 * f_kib + w_kib) * 1024.0,
        }
    with open(os.path.join(prof, "pmc_ntt.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
