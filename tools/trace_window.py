"""Last window (split at idle gaps > 2 ms) of a rocprofv3 kernel trace with
start offsets, so overlapping kernels show (dev tool): trace_window.py csv"""
import csv, sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
wins, cur = [], [rows[0]]
end = int(rows[0]["End_Timestamp"])
for b in rows[1:]:
    if int(b["Start_Timestamp"]) - end > 2e6:
        wins.append(cur); cur = []
    cur.append(b)
    end = max(end, int(b["End_Timestamp"]))
wins.append(cur)
w = wins[-1]
t0 = int(w[0]["Start_Timestamp"])
for r in w:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("start %8.2f  end %8.2f  dur %7.2f us  q%s  %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3,
          r.get("Queue_Id", "?"), r["Kernel_Name"].split("(")[0][-50:]))
print("span %.2f us" % ((max(int(r["End_Timestamp"]) for r in w) - t0) / 1e3))
