"""Summarize rocprofv3 --pmc CSVs: mean counter value per dispatch for each fg:: kernel."""
import collections
import csv
import glob
import sys


def summarize(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if not k.startswith("fg::"):
                continue
            k = k.split("(")[0]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    out = {}
    for k, cs in agg.items():
        out[k] = {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()}
    return out


if __name__ == "__main__":
    res = summarize(glob.glob(sys.argv[1]))
    for k, cs in sorted(res.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {v:16.1f}")
