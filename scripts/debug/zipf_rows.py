"""Debug: compare the engine's fired (window, key, COUNT(*)) on a bench workload with a
torch.unique count of the generated records (tumbling windows, no late records)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench as B  # noqa: E402
import flink_amd as F  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "zipf"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000_000
wl = B.WORKLOADS[w]
size = wl["window"][1]
dev = torch.device("cuda", 0)
key, ts, val = B.gen_columns(n, wl["keys"], wl["rate"], 0, dev, jitter=wl["jitter"], zipf=wl["zipf"])
op = F.WindowAggOperator(F.tumbling(size), aggs=("count_star",), val_type="f64", expected_keys=int(wl["keys"] * 1.05),
                         buffer_records=1 << 28, kernel_timing=True)
batch = 50_000_000
rows = []
for lo in range(0, n, batch):
    hi = min(n, lo + batch)
    op.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
    print("batch", lo, "late so far", op.num_late_records_dropped, "ts range", int(ts[lo:hi].min()) - B.T0,
          int(ts[lo:hi].max()) - B.T0, flush=True)
    for wm in B.watermarks_for(lo, hi, wl["rate"], 1_000_000, wl["delay"], wl["jitter"]):
        r = op.process_watermark(wm)
        if wm == B.watermarks_for(lo, hi, wl["rate"], 1_000_000, wl["delay"], wl["jitter"])[-1]:
            print("  last wm", wm - B.T0, flush=True)
        if len(r):
            rows.append(r)
rows.append(op.process_watermark(B.JMAX))
rows = np.concatenate(rows)
print("rows", len(rows), "late", op.num_late_records_dropped, {k: v["launches"] for k, v in op.kernel_stats().items()})
got = torch.from_numpy(((rows["window_end"] - B.T0 - size) // size) * (1 << 26) + rows["key"]).to(dev)
gcnt = torch.from_numpy(np.ascontiguousarray(rows["count_star"])).to(dev)
comp = torch.div(ts - B.T0, size, rounding_mode="floor") * (1 << 26) + key
u, c = torch.unique(comp, return_counts=True)
print("expected", u.numel(), "got", got.numel(), "dup rows", got.numel() - torch.unique(got).numel())
miss = u[~torch.isin(u, got)]
print("missing", miss.numel(), [(int(x) >> 26, int(x) & ((1 << 26) - 1)) for x in miss[:10].cpu()])
extra = got[~torch.isin(got, u)]
print("extra", extra.numel(), [(int(x) >> 26, int(x) & ((1 << 26) - 1)) for x in extra[:10].cpu()])
order = torch.argsort(got)
gs, gc = got[order], gcnt[order]
idx = torch.searchsorted(u, gs)
ok = (idx < u.numel())
idx = idx.clamp(max=u.numel() - 1)
bad = ok & (u[idx] == gs) & (c[idx] != gc)
print("count mismatches", int(bad.sum()), [(int(x) >> 26, int(x) & ((1 << 26) - 1)) for x in gs[bad][:10].cpu()],
      gc[bad][:10].tolist(), c[idx[bad]][:10].tolist())
