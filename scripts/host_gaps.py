"""Host-side time per operator call in the bench loop (GPU box): where the gaps between
kernels go. Runs 2 steps of the configs[1] job on 400M records and prints the mean wall
time of process_batch / process_watermark (firing and non-firing) calls."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as B  # noqa: E402
import flink_amd as F  # noqa: E402

n, keys, rate, batch = 400_000_000, 10_000_000, 100_000_000, 50_000_000
dev = torch.device("cuda", 0)
key, ts, val = B.gen_columns(n, keys, rate, 0, dev)
torch.cuda.synchronize()
op = F.WindowAggOperator(F.tumbling(1000), aggs=("count_star", "sum", "avg"), val_type="f64",
                         expected_keys=int(keys * 1.05) + 1, buffer_records=4 * batch, device=0)
acc = {}


def tick(name, t0):
    d = acc.setdefault(name, [0, 0.0])
    d[0] += 1
    d[1] += time.perf_counter() - t0


for step in range(3):
    if step == 1:
        acc.clear()
        torch.cuda.synchronize()
        T0 = time.perf_counter()
    op.reset()
    for lo in range(0, n, batch):
        hi = lo + batch
        t0 = time.perf_counter()
        k, t, v = key[lo:hi], ts[lo:hi], val[lo:hi]
        wms = B.watermarks_for(lo, hi, rate, 1_000_000)
        tick("slice+wms", t0)
        t0 = time.perf_counter()
        op.process_batch(k, t, v)
        tick("process_batch", t0)
        for j, wm in enumerate(wms):
            t0 = time.perf_counter()
            op.process_watermark(wm, device_output=True, wait=False)
            tick("wm_first" if j == 0 else "wm_rest", t0)
    t0 = time.perf_counter()
    op.process_watermark(B.JMAX, device_output=True)
    tick("wm_final", t0)
op.synchronize()
el = time.perf_counter() - T0
for k, (c, s) in acc.items():
    print(f"{k:14s} calls {c:5d}  mean {s / c * 1e6:9.1f} us  total {s * 1e3:8.2f} ms")
print(f"2 steps x {n:,} records: {el * 1e3:.1f} ms")
op.close()
