"""Print the kernel sequence of the last window of a rocprofv3 kernel trace
(windows split at gaps > 2 ms): per kernel its duration and the idle gap before
it, plus totals (dev tool).  usage: kernel_seq.py kernel_trace.csv [window_from_end]"""
import csv, sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
wins, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 2e6:
        wins.append(cur); cur = []
    cur.append(b)
wins.append(cur)
w = wins[-int(sys.argv[2]) if len(sys.argv) > 2 else -1]
busy = gap = 0.0
prev_end = None
for r in w:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (s - prev_end) / 1e3 if prev_end else 0.0
    prev_end = e
    busy += (e - s) / 1e3
    gap += g
    print("%8.2f us  gap %6.2f  %s" % ((e - s) / 1e3, g, r["Kernel_Name"].split("(")[0][-60:]))
print("span %.1f us = busy %.1f + gaps %.1f, %d kernels" % (busy + gap, busy, gap, len(w)))
