"""Print the kernels of the last trace window with start offset, duration and
the idle gap before each (rocprofv3 kernel_trace.csv; dev tool)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
idx = 0
for i in range(1, len(rows)):
    if int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) > 2e6:
        idx = i
w = rows[idx:]
t0 = int(w[0]["Start_Timestamp"])
end = int(w[0]["End_Timestamp"])
for k, r in enumerate(w):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - end) / 1e3
    if gap >= thr or thr == 0:
        prev = w[k - 1]["Kernel_Name"].split("(")[0][-30:] if k else ""
        print("%9.1f us dur %7.1f gap %7.1f  %-34s <- %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap,
                                                            r["Kernel_Name"].split("(")[0][-34:], prev))
    end = max(end, e)
