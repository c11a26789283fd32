"""fg_snapshot_state_async / _wait (ABI 15): snapshotState split into its synchronous part (the
staged records flushed, every resident slice exported on the GPU, the image's copy to the host
queued on a stream of its own) and its asynchronous part (the host image), as a heap state
backend's AsyncSnapshotCallable runs it (SnapshotStrategyRunner.snapshot). Two identical
operators take the same stream: at the checkpoint one snapshots synchronously, the other
asynchronously and then keeps processing batches and watermarks (which fire windows, write
slice tables and flush lanes) before it collects the image -- which must equal the synchronous
image bit for bit, as must both operators' fired rows before and after."""
import numpy as np
import pytest

from tests.test_gpu_parity import assert_rows_equal, cfg_of, gpu_mk
from tests.streams import batches_with_watermarks, make_stream

pytestmark = pytest.mark.gpu
JMAX = (1 << 63) - 1

CASES = [
    # Zipf keys, out of order: the checkpoint flushes skewed lanes (split fire with tables)
    ("tumble_zipf_ooo", cfg_of("tumble", 1000), dict(n=6_000_000, keys=500_000, batch=1_000_000, rate_per_ms=2_000,
                                                      zipf=1.1, delay=400, jitter=700), 3, 2),
    ("hop_f64", cfg_of("hop", 3000, 1000), dict(n=600_000, keys=50_000, batch=40_000, rate_per_ms=100,
                                                 delay=200, jitter=800), 6, 4),
    ("cumulate_i64", cfg_of("cumulate", 4000, 500, vt="i64"), dict(n=400_000, keys=30_000, batch=20_000,
                                                                   rate_per_ms=100, delay=50, jitter=900), 8, 5),
]


def _sorted_image(img):
    o = np.lexsort((img["key"], img["slice_end"]))
    return {k: np.asarray(v)[o] for k, v in img.items()}


@pytest.mark.parametrize("name,cfg,kw,snap_at,after", CASES, ids=[c[0] for c in CASES])
def test_async_snapshot_equals_sync_snapshot(name, cfg, kw, snap_at, after):
    kw = dict(kw)
    n, keys, batch, delay, jitter = (kw.pop(k) for k in ("n", "keys", "batch", "delay", "jitter"))
    key, ts, val, isnull = make_stream(n, keys, cfg["val_type"], jitter_ms=jitter, **kw)
    a = gpu_mk(cfg, expected_keys=keys, buffer_records=batch * 4)
    b = gpu_mk(cfg, expected_keys=keys, buffer_records=batch * 4)
    img_a = wm_a = None
    pending = False
    for step, (lo, hi, wm) in enumerate(batches_with_watermarks(n, batch, ts, delay)):
        for g in (a, b):
            g.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi], None)
            g.process_watermark(wm)
        assert_rows_equal(b.take_rows(), a.take_rows(), cfg["val_type"], f"step {step}")
        if step == snap_at:
            a.prepare_snapshot()
            b.prepare_snapshot()
            img_a, wm_a = a.op.snapshot_state()
            b.op.snapshot_state_async()
            pending = True
            with pytest.raises(RuntimeError):   # one snapshot at a time
                b.op.snapshot_state_async()
            with pytest.raises(RuntimeError):
                b.op.snapshot_state()
        elif pending and step == snap_at + after:
            img_b, wm_b = b.op.snapshot_state_wait()
            pending = False
            assert wm_b == wm_a
            assert len(img_a["key"]) > 0 and set(img_b) == set(img_a)
            sa, sb = _sorted_image(img_a), _sorted_image(img_b)
            for k in sa:   # bit-exact, but DOUBLE sums: two operators add in different orders (LDS atomics)
                if k == "sum" and cfg["val_type"] == "f64":
                    x, y = sa[k].view(np.float64), sb[k].view(np.float64)
                    assert (np.abs(x - y) <= 1e-9 * np.maximum(np.abs(x), np.abs(y))).all(), k
                else:
                    assert np.array_equal(sa[k], sb[k]), k
    assert img_a is not None and not pending
    with pytest.raises(RuntimeError):   # nothing pending
        b.op.snapshot_state_wait()
    for g in (a, b):
        g.process_watermark(JMAX)
    assert_rows_equal(b.take_rows(), a.take_rows(), cfg["val_type"], "final")
    a.close()
    b.close()
