"""Debug: rows per step of a bench workload across op.reset() (device output, as bench.py)."""
import sys

import torch

sys.path.insert(0, ".")
import bench as B  # noqa: E402
import flink_amd as F  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "zipf"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000_000
aggs = tuple(sys.argv[3].split(",")) if len(sys.argv) > 3 else ("avg",)
bufrec = int(sys.argv[4]) if len(sys.argv) > 4 else 200_000_000
wl = B.WORKLOADS[w]
dev = torch.device("cuda", 0)
key, ts, val = B.gen_columns(n, wl["keys"], wl["rate"], 0, dev, jitter=wl["jitter"], zipf=wl["zipf"])
torch.cuda.synchronize()
wname, *wargs = wl["window"]
op = F.WindowAggOperator(getattr(F, wname)(*wargs), aggs=aggs, val_type="f64", expected_keys=int(wl["keys"] * 1.05) + 1,
                         buffer_records=bufrec, kernel_timing=True)
for step in range(3):
    op.reset()
    rows = 0
    for lo in range(0, n, 50_000_000):
        hi = min(n, lo + 50_000_000)
        op.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        for wm in B.watermarks_for(lo, hi, wl["rate"], 1_000_000, wl["delay"], wl["jitter"]):
            rows += op.process_watermark(wm, device_output=True).n
    rows += op.process_watermark(B.JMAX, device_output=True).n
    print("step", step, "rows", rows, "late", op.num_late_records_dropped, flush=True)
