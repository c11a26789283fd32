"""The shim's checkpoint, incremental (ABI 16: fg_snapshot_slices): at every barrier the keyed
state backend is brought up to date with the engine's image by rewriting only the slices whose
tables changed since the previous image (flink_amd.keyed_state, the mirror of
GpuSlicingWindowProcessor.writeKeyedState), and must then equal the backend round 5's full rewrite
leaves. A configs[4]-shaped stream (Zipf keys, jitter, bounded out-of-orderness) checkpoints often;
after the last checkpoint a failover restores a new operator from the BACKEND (restoreFromKeyedState,
not the engine's own image) and the rows that follow must equal the oracle's, restored from its own
snapshot."""
import numpy as np
import pytest

from tests.streams import batches_with_watermarks, make_stream
from tests.test_gpu_parity import assert_rows_equal, cfg_of, gpu_mk, oracle_mk

pytestmark = pytest.mark.gpu

CASES = [
    # (name, cfg, stream, checkpoint steps, restore)
    ("tumble_zipf", cfg_of("tumble", 1000),
     dict(n=1_200_000, keys=200_000, batch=60_000, rate_per_ms=300, delay=400, jitter=600, zipf=1.1), (3, 4, 9, 14), True),
    ("hop", cfg_of("hop", 3000, 1000),
     dict(n=600_000, keys=50_000, batch=30_000, rate_per_ms=100, delay=300, jitter=500), (4, 5, 11), False),
    ("cumulate", cfg_of("cumulate", 4000, 1000),
     dict(n=600_000, keys=50_000, batch=30_000, rate_per_ms=100, delay=300, jitter=500), (4, 5, 11, 16), False),
]
KIND = {"tumble": 0, "hop": 1, "cumulate": 2}


@pytest.mark.parametrize("name,cfg,kw,ckpts,restore", CASES, ids=[c[0] for c in CASES])
def test_incremental_checkpoints_equal_full_rewrite(oracle_mod, name, cfg, kw, ckpts, restore):
    from flink_amd.keyed_state import SliceSpec, WindowAggsState
    O = oracle_mod
    kw = dict(kw)
    n, keys, batch, delay, jitter = kw.pop("n"), kw.pop("keys"), kw.pop("batch"), kw.pop("delay"), kw.pop("jitter")
    key, ts, val, _ = make_stream(n, keys, cfg["val_type"], jitter_ms=jitter, **kw)
    spec = SliceSpec(KIND[cfg["kind"]], cfg["size"], cfg["slide"])
    inc, full = WindowAggsState(spec), WindowAggsState(spec)
    g = gpu_mk(cfg, expected_keys=keys, buffer_records=max(4 * batch, 1 << 16))
    o = oracle_mk(O, cfg)
    o_base = g_base = 0
    costs = []
    for step, (lo, hi, wm) in enumerate(batches_with_watermarks(n, batch, ts, delay)):
        g.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        g.process_watermark(wm)
        o.process_watermark(wm)
        assert_rows_equal(g.take_rows(), o.take_rows(), cfg["val_type"], f"{name} step {step}", sums=True)
        if step not in ckpts:
            continue
        # prepareSnapshotPreBarrier + snapshotState: the image, its slices, the backend write
        g.prepare_snapshot()
        o.prepare_snapshot()
        img, twm = g.op.snapshot_state()
        sl = g.op.snapshot_slices()
        assert sl["rows"].sum() == len(img["key"]) and (np.diff(sl["slice_end"]) > 0).all()
        for b in (inc, full):
            b.advance_watermark(twm)
        c = inc.write_image(img, sl, twm)
        costs.append((c, len(img["key"])))
        if cfg["kind"] != "cumulate":   # (one slice per namespace: exactly the changed slices' rows)
            assert c["put"] == int(sl["rows"][sl["changed"]].sum()), (step, c)
        assert c["timer_delete"] == 0 and c["put"] <= len(img["key"])
        full.write_image_full(img, sl, twm)
        assert inc.entries == full.entries, f"{name} checkpoint at step {step}: entries differ"
        assert inc.timers == full.timers, f"{name} checkpoint at step {step}: timers differ"
        if restore and step == max(ckpts):
            break   # (a failover right after the last checkpoint)
    # the second of two checkpoints one micro-batch apart: HOP rewrites only the slices that batch
    # touched, a part of the state (the older slices of the open windows stay as written); every kind
    # clears only the namespaces that left the image (round 5 cleared every entry and deleted every
    # timer, then put the whole image)
    (c0, rows0), (c1, rows1) = costs[0], costs[1]
    if cfg["kind"] == "hop":
        assert c1["put"] < rows1, costs
    assert c1["clear"] <= rows0 and c1["timer_delete"] == 0, costs
    if not restore:
        g.close()
        o.close()
        return
    # failover after the last checkpoint: the new operator restores from the backend
    cols, twm = inc.image()
    cols = {k: v for k, v in cols.items() if k not in ("min", "max")}   # (one value accumulator)
    g2 = gpu_mk(cfg, expected_keys=keys, buffer_records=max(4 * batch, 1 << 16))
    g2.op.restore_state(cols, twm)
    o2 = o.restore_copy()
    g_base, o_base = g.late_dropped, o.late_dropped
    g.close()
    o.close()
    last = max(ckpts)
    for step, (lo, hi, wm) in enumerate(batches_with_watermarks(n, batch, ts, delay)):
        if step <= last:
            continue
        g2.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        o2.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        g2.process_watermark(wm)
        o2.process_watermark(wm)
        assert_rows_equal(g2.take_rows(), o2.take_rows(), cfg["val_type"], f"{name} restored step {step}", sums=True)
    g2.process_watermark((1 << 63) - 1)
    o2.process_watermark((1 << 63) - 1)
    assert_rows_equal(g2.take_rows(), o2.take_rows(), cfg["val_type"], f"{name} final", sums=True)
    assert g_base + g2.late_dropped == o_base + o2.late_dropped
    g2.close()
    o2.close()
