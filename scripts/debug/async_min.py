"""Minimal async-advance scenario with progress prints (diagnostics)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import flink_amd as F
from tests.streams import make_stream
key, ts, val, _ = make_stream(300_000, 30_000, "f64")
op = F.WindowAggOperator(F.tumbling(1000), aggs=("count_star", "sum"), val_type="f64", expected_keys=30_000,
                         buffer_records=240_000)
print("open", flush=True)
for lo in range(0, 300_000, 60_000):
    op.process_batch(key[lo:lo + 60_000], ts[lo:lo + 60_000], val[lo:lo + 60_000])
    print("batch", lo, flush=True)
    for c in np.linspace(lo, lo + 60_000, 7)[1:].astype(np.int64):
        wm = int(ts[lo:c].max()) - 1
        print(" wm", wm, flush=True)
        op.process_watermark(wm, device_output=True, wait=False)
    r = op.collect_fired()
    print("collected", r.n, flush=True)
print("stats", op.stats(), flush=True)
op.close()
