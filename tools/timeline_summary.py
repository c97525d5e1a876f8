"""Summarise a rocprofv3 kernel trace: for the last N 'windows' separated by
gaps > 2 ms, print span, kernel busy time and the top kernels (dev tool)."""
import collections, csv, sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
wins, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 2e6:
        wins.append(cur); cur = []
    cur.append(b)
wins.append(cur)
for w in wins[-int(sys.argv[2]) if len(sys.argv) > 2 else -3:]:
    t0, t1 = int(w[0]["Start_Timestamp"]), int(w[-1]["End_Timestamp"])
    busy = collections.Counter(); cnt = collections.Counter()
    gaps = []
    for a, b in zip(w, w[1:]):
        gaps.append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
    for r in w:
        k = r["Kernel_Name"].split("(")[0][-44:]
        busy[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        cnt[k] += 1
    print("window span %.3f ms busy %.3f ms kernels %d, gaps>20us: %d (sum %.3f ms)" % (
        (t1 - t0) / 1e6, sum(busy.values()), len(w), sum(1 for g in gaps if g > 20),
        sum(g for g in gaps if g > 20) / 1e3))
    for k, v in busy.most_common(10):
        print("   %-46s %4d  %.3f ms" % (k, cnt[k], v))
