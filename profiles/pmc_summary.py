"""Summarize rocprofv3 --pmc CSVs: mean counter value per dispatch for each fg:: kernel.

usage: python profiles/pmc_summary.py "<glob of run_counter_collection.csv>" [out.json]

With an output path, also writes the per-launch HBM traffic of each engine kernel class
(the `roofline.traffic` field bench.py reports), corrected as MI355X_MICROARCH.md's
HBM/rocprofv3 section prescribes: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE counts half the bytes of wide (16 B/lane) coalesced streaming reads, which is
how every engine kernel reads, so it is doubled; WRITE_SIZE is taken as is.
"""
import collections
import csv
import glob
import json
import sys

# engine kernel -> fg_kernel_stats class names it is timed under
CLASSES = {
    "fg::k_part1": ["ingest_part1"],
    "fg::k_part2": ["ingest_part2"],
    "fg::k_ingest_count": ["ingest_count"],
    "fg::k_ingest_scatter_sorted": ["ingest_scatter"],
    "fg::k_ingest_scatter_direct": ["ingest_scatter"],
    "fg::k_merge": ["merge_flush_fire", "merge_flush", "merge_fire", "restore"],
    "fg::k_tile_part1": ["tile_part1"],
    "fg::k_tile_fire": ["tile_fire", "tile_flush"],
    # the key dictionary's lookup (timed as "dict_probe"): one random 64-B slot per row, a 128-B
    # line request, tallied at 64 B like the streaming reads -- doubled alike (calibrated: 100M
    # 32-B rows read 17.2 GB = row + line + id per row)
    "dict::k_dict_lookup": ["dict_probe"],
}


def summarize(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if k.startswith("void "):
                k = k[5:]
            if k.startswith("(anonymous namespace)::k_dict_"):   # fg_keydict.hip's kernels
                k = "dict::" + k[len("(anonymous namespace)::"):]
            if not k.startswith(("fg::", "dict::")):
                continue
            k = k.split("(")[0]
            if "<" in k:
                k = k.split("<")[0]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    out = {}
    for k, cs in agg.items():
        out[k] = {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()}
    return out


def traffic(res):
    t = {}
    for k, cs in res.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        fetch = 2.0 * cs["FETCH_SIZE"] * 1024.0
        write = cs["WRITE_SIZE"] * 1024.0
        for cls in CLASSES.get(k, []):
            t[cls] = {"kernel": k, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                      "hbm_bytes_per_launch": fetch + write}
    return t


if __name__ == "__main__":
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from flink_amd import buildinfo
    res = summarize(glob.glob(sys.argv[1]))
    for k, cs in sorted(res.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {v:16.1f}")
    if len(sys.argv) > 2:
        t = traffic(res)
        # provenance: bench.py reports these bytes only for the kernels they were counted on
        # (sha256 of libflinkgpu.so's device code objects), never for other kernels
        lib = sys.argv[3] if len(sys.argv) > 3 else None
        t["_provenance"] = {"lib_sha256": buildinfo.file_sha256(lib) if lib else None,
                            "kernels_sha256": buildinfo.kernels_sha256(lib) if lib else None,
                            "source": sys.argv[1],
                            # the bench workload counted (a kernel class's bytes differ by workload:
                            # the CUMULATE tile_fire reads and writes tables, the TUMBLE one does not)
                            "workload": sys.argv[4] if len(sys.argv) > 4 else os.environ.get("WL") or "tumble"}
        json.dump(t, open(sys.argv[2], "w"), indent=1)
        print("wrote", sys.argv[2])
