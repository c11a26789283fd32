"""Inter-kernel gaps of a rocprofv3 kernel trace over the last timed step, with the HIP API calls
made inside the largest gaps (a --hip-trace run). usage: python scripts/gap_report.py DIR [part1 launches per step]"""
import collections
import csv
import sys

d = sys.argv[1]
per = int(sys.argv[2]) if len(sys.argv) > 2 else 10
K = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[-34:])
           for r in csv.DictReader(open(d + "/run_kernel_trace.csv")))
A = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
           for r in csv.DictReader(open(d + "/run_hip_api_trace.csv")))
p1 = [i for i, k in enumerate(K) if k[2].endswith("k_tile_part1")]
a, b = p1[-2 * per], p1[-per]   # the last full step before the final one
sel = K[a:b]
span = (sel[-1][1] - sel[0][0]) / 1e6
busy = sum(k[1] - k[0] for k in sel) / 1e6
print("step span %.3f ms, busy %.3f, gaps %.3f" % (span, busy, span - busy))
tot, n = collections.defaultdict(float), collections.Counter()
for x, y in zip(sel, sel[1:]):
    tot[(x[2], y[2])] += (y[0] - x[1]) / 1e3
    n[(x[2], y[2])] += 1
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:8]:
    print("%9.1f us  n=%4d  %s -> %s" % (v, n[k], k[0], k[1]))
api = collections.defaultdict(float)
cnt = collections.Counter()
for s, e, f in A:
    if sel[0][0] <= s <= sel[-1][1]:
        api[f] += (e - s) / 1e3
        cnt[f] += 1
print("HIP API in the step (us, calls):", [(f, round(v), cnt[f]) for f, v in sorted(api.items(), key=lambda kv: -kv[1])[:10]])
