"""Debug probe (GPU): the first batch + watermark of tests/test_gpu_parity.py's tumble_i64_l600_zipf
case, rows of the HIP path against the oracle's; prints the missing / extra (key, window) rows
with each key's state region and its record count. Run with FG_MIN_REGION_BITS=10."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import oracle as O  # noqa: E402
from tests.streams import make_stream  # noqa: E402
from tests.test_gpu_parity import batches_with_watermarks, cfg_of, gpu_mk, oracle_mk  # noqa: E402


cfg = dict(cfg_of("tumble", 1000, vt="i64", mode="datastream"), allowed_lateness=600)
n, keys, batch, delay, jitter = 200_000, 5000, 20_000, 50, 1200
key, ts, val, _ = make_stream(n, keys, "i64", jitter_ms=jitter, zipf=1.3)
g = gpu_mk(cfg, expected_keys=keys, buffer_records=max(batch * 4, 1 << 16), kernel_timing=True)
o = oracle_mk(O, cfg)
for step, (lo, hi, wm) in enumerate(batches_with_watermarks(n, batch, ts, delay)):
    g.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi], None)
    o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi], None)
    g.process_watermark(wm)
    o.process_watermark(wm)
    a, b = g.take_rows(), o.take_rows()
    ga = {(int(k), int(w)) for k, w in zip(a["key"], a["window_end"])}
    ob = {(int(k), int(w)) for k, w in zip(b["key"], b["window_end"])}
    miss, extra = sorted(ob - ga), sorted(ga - ob)
    print(f"step {step}: got {len(a)} exp {len(b)} missing {len(miss)} extra {len(extra)}")
    if miss or extra:
        cnt = {}
        for k in key[lo:hi]:
            cnt[int(k)] = cnt.get(int(k), 0) + 1
        top = sorted(cnt.items(), key=lambda kv: -kv[1])[:5]
        print("  stats:", {k: v for k, v in g.op.stats().items() if "region" in k or "lane" in k or "grow" in k})
        print("  hottest keys of the batch:", top)
        for k, w in miss[:20]:
            print(f"  missing key {k} window_end {w} records_in_batch {cnt.get(k, 0)}")
        for k, w in extra[:10]:
            print(f"  extra key {k} window_end {w}")
        print("  kernels:", {k: v["launches"] for k, v in g.op.kernel_stats().items() if v["launches"]})
        break
