"""CUMULATE restore divergence (sync path): print the (key, window) rows that differ between GPU and oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from oracle import oracle as O
O.build()
from tests.streams import make_stream
from tests.test_gpu_parity import oracle_mk
from tests.test_gpu_async import _cfg
from tests.gpu_adapter import GpuOperator
cfg = _cfg("cumulate")
n, keys, batch, wpb, jitter, delay = 900_000, 30_000, 60_000, 6, 1500, 300
key, ts, val, _ = make_stream(n, keys, "f64", jitter_ms=jitter)
g = GpuOperator(cfg, expected_keys=keys, buffer_records=4 * batch)
o = oracle_mk(O, cfg)
mx = np.iinfo(np.int64).min
nb = 0
wmlog = []
for lo in range(0, n, batch):
    hi = lo + batch
    g.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi]); o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
    for c in np.linspace(lo, hi, wpb + 1)[1:].astype(np.int64):
        mx = max(mx, int(ts[lo:c].max())); wm = mx - delay - 1
        g.process_watermark(wm); o.process_watermark(wm)
        a, b = g.take_rows(), o.take_rows()
        ka = set(zip(a["key"].tolist(), a["window_start"].tolist(), a["window_end"].tolist()))
        kb = set(zip(b["key"].tolist(), b["window_start"].tolist(), b["window_end"].tolist()))
        if ka != kb:
            print("batch", nb + 1, "wm", wm, "gpu-only", sorted(ka - kb)[:5], "oracle-only", sorted(kb - ka)[:5], flush=True)
            for k, ws, we in sorted(kb - ka)[:3]:
                m = key == k
                print("   key", k, "records (rowtime, batch):", [(int(t), int(i) // batch + 1) for t, i in zip(ts[m], np.nonzero(m)[0])][:40])
    nb += 1
    if nb == 8:
        print("checkpoint after batch 8 at wm", wm, flush=True)
        g.prepare_snapshot(); o.prepare_snapshot()
        g2, o2 = g.restore_copy(), o.restore_copy()
        g.close(); o.close(); g, o = g2, o2
    if nb == 11:
        break
