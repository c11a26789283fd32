"""Per-step kernel time and inter-kernel gaps of a rocprofv3 kernel trace of the default bench.
usage: python scripts/gaps.py run_kernel_trace.csv [step index] [pass-1 launches per step (10: 100M batches)]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[-28:])
            for r in rows)
p1 = [i for i, k in enumerate(ks) if k[2].endswith("k_part1")]
step = int(sys.argv[2]) if len(sys.argv) > 2 else 1
per = int(sys.argv[3]) if len(sys.argv) > 3 else 10
a, b = p1[per * step], p1[per * (step + 1)] if len(p1) > per * (step + 1) else len(ks)
sel = ks[a:b]
span = (sel[-1][0] - sel[0][0]) / 1e6
busy = sum(k[1] - k[0] for k in sel) / 1e6
print("step span ms %.3f busy %.3f gaps %.3f" % (span, busy, span - busy))
tot = collections.defaultdict(float)
c = collections.Counter()
for x, y in zip(sel, sel[1:]):
    tot[(x[2], y[2])] += y[0] - x[1]
    c[(x[2], y[2])] += 1
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:10]:
    print(f"{v / 1e3:9.1f} us  n={c[k]:4d}  {k}")
