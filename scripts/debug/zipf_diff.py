"""Debug: fired (window, key, COUNT(*)) of a bench workload, device output + reset as
bench.py, against torch.unique of the generated records."""
import sys

import torch

sys.path.insert(0, ".")
import bench as B  # noqa: E402
import flink_amd as F  # noqa: E402
from flink_amd.exchange import device_columns  # noqa: E402

w = sys.argv[1]
n = int(sys.argv[2])
bufrec = int(sys.argv[3])
wl = B.WORKLOADS[w]
size = wl["window"][1]
dev = torch.device("cuda", 0)
key, ts, val = B.gen_columns(n, wl["keys"], wl["rate"], 0, dev, jitter=wl["jitter"], zipf=wl["zipf"])
torch.cuda.synchronize()
op = F.WindowAggOperator(F.tumbling(size), aggs=("count_star",), val_type="f64",
                         expected_keys=int(wl["keys"] * 1.05) + 1, buffer_records=bufrec, kernel_timing=True)
op.reset()
got, gc = [], []
log = []


def take(r, tag):
    if r.n:
        k, we, c = device_columns(r, names=("key", "window_end"), aggs=(0,), device=dev)
        got.append(((we - B.T0 - size) // size) * (1 << 26) + k)
        gc.append(c.clone())
        log.append((tag, int(r.n)))


for lo in range(0, n, 50_000_000):
    hi = min(n, lo + 50_000_000)
    op.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
    for wm in B.watermarks_for(lo, hi, wl["rate"], 1_000_000, wl["delay"], wl["jitter"]):
        take(op.process_watermark(wm, device_output=True), (lo, wm - B.T0))
take(op.process_watermark(B.JMAX, device_output=True), "final")
got = torch.cat(got)
gcnt = torch.cat(gc)
print("fires", log)
print("rows", got.numel(), {k: v["launches"] for k, v in op.kernel_stats().items()})
comp = torch.div(ts - B.T0, size, rounding_mode="floor") * (1 << 26) + key
u, c = torch.unique(comp, return_counts=True)
gu, ginv, gcount = torch.unique(got, return_inverse=True, return_counts=True)
print("expected", u.numel(), "got", got.numel(), "dup rows", got.numel() - gu.numel())
dups = gu[gcount > 1]
print("dup pairs", [(int(x) >> 26, int(x) & ((1 << 26) - 1)) for x in dups[:10].cpu()])
miss = u[~torch.isin(u, gu)]
print("missing", miss.numel(), [(int(x) >> 26, int(x) & ((1 << 26) - 1)) for x in miss[:10].cpu()])
tot = torch.zeros(gu.numel(), dtype=torch.int64, device=dev).index_add_(0, ginv, gcnt)
idx = torch.searchsorted(u, gu).clamp(max=u.numel() - 1)
bad = (u[idx] == gu) & (c[idx] != tot)
print("count mismatches", int(bad.sum()), [(int(x) >> 26, int(x) & ((1 << 26) - 1)) for x in gu[bad][:10].cpu()],
      tot[bad][:10].tolist(), c[idx[bad]][:10].tolist())
