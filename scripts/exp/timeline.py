"""Busy time and gaps of the engine's kernels in a rocprofv3 kernel trace (the last N fg:: dispatches).
usage: python scripts/exp/timeline.py run_kernel_trace.csv [last_n]"""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "fg::" in r["Kernel_Name"] or "dict::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows)
rows = rows[-n:]
t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
busy = collections.Counter()
gaps = collections.Counter()
prev_end, prev_name = None, None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = r["Kernel_Name"].split("(")[0].replace("void ", "")
    busy[nm] += e - s
    if prev_end is not None and s > prev_end:
        gaps[prev_name + " -> " + nm] += s - prev_end
    prev_end, prev_name = max(e, prev_end or 0), nm
span = t1 - t0
print("span %.3f ms, busy %.3f ms, gaps %.3f ms" % (span / 1e6, sum(busy.values()) / 1e6, sum(gaps.values()) / 1e6))
for k, v in busy.most_common():
    print("  busy %-40s %8.3f ms" % (k[:40], v / 1e6))
for k, v in gaps.most_common(8):
    print("  gap  %-60s %8.3f ms" % (k[:60], v / 1e6))
