# debug: hop snapshot/restore with many regions
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import flink_amd as F
from tests.streams import batches_with_watermarks, make_stream
from tests.gpu_adapter import GpuOperator
from oracle import oracle as O
O.build()
cfg = dict(mode="sql", kind="hop", size=4000, slide=1000, offset=0, tz_offset_ms=0, val_type="f64", count_star_index=0)
n, keys = 400_000, int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
key, ts, val, isnull = make_stream(n, keys, "f64", jitter_ms=500)
g = GpuOperator(cfg, expected_keys=keys, buffer_records=1 << 17)
print("stats0", g.op.stats())
step = 0
for lo, hi, wm in batches_with_watermarks(n, 20_000, ts, 100):
    g.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
    g.process_watermark(wm)
    r = g.take_rows()
    step += 1
    print("step", step, "wm", wm, "rows", len(r), g.op.stats())
    if step == 9:
        g.prepare_snapshot()
        img, twm = g.op.snapshot_state()
        print("snapshot rows", len(img["key"]) if hasattr(img, "__getitem__") else img, "twm", twm)
        g2 = g.restore_copy()
        print("restored", g2.op.stats())
        g.close(); g = g2
    if step == 12:
        break
