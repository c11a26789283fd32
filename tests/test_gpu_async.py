"""fg_advance_progress_async / fg_collect_fired (ABI 11) / fg_collect_fired_to (ABI 12) on the GPU.

The asynchronous advance queues a watermark's fires and returns at once; the fires' completion
(row count, region retries, overflow check) is taken by the next call that needs it, and the
watermarks in between -- which fire nothing -- only move the progress. Rows of async advances
accumulate until fg_collect_fired returns them. These tests deliver several watermarks per
micro-batch (the bench's cadence), most of them quiet, collect after one or two batches, and
require exactly the oracle's rows (SlicingWindowOperator / WindowOperator via oracle/).
"""
import numpy as np
import pytest

from tests.streams import make_stream
from tests.test_gpu_parity import assert_rows_equal, oracle_mk

pytestmark = pytest.mark.gpu

JMAX = (1 << 63) - 1


def _cfg(kind, mode="sql", vt="f64"):
    size, slide = {"tumble": (1000, 0), "hop": (4000, 1000), "cumulate": (4000, 1000)}[kind]
    return dict(mode=mode, kind=kind, size=size, slide=slide, offset=0, tz_offset_ms=0, val_type=vt,
                count_star_index=0)


def _run(O, cfg, n=900_000, keys=30_000, batch=60_000, wms_per_batch=6, jitter=0, delay=0, collect_every=1,
         regions_small=False, ckpt_every=0, zipf=0.0, sync=False, collect="device", batched=False):
    """collect: "device" (fg_collect_fired, rows copied out by torch), "host" (fg_collect_fired_to
    FG_HOST), or "sync_wm" (no collect: a synchronous watermark instead, whose rows must lead with
    every async row not collected yet)."""
    from tests.gpu_adapter import GpuOperator
    key, ts, val, _ = make_stream(n, keys, cfg["val_type"], jitter_ms=jitter, zipf=zipf)
    g = GpuOperator(cfg, expected_keys=1000 if regions_small else keys, buffer_records=4 * batch)
    o = oracle_mk(O, cfg)
    op = g.op
    exp = []
    fired_total = 0
    o_base = 0
    mx = np.iinfo(np.int64).min
    nb = 0
    for lo in range(0, n, batch):
        hi = min(n, lo + batch)
        op.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        # watermarks at sub-batch boundaries (max rowtime so far - delay - 1)
        held = []
        for c in np.linspace(lo, hi, wms_per_batch + 1)[1:].astype(np.int64):
            mx = max(mx, int(ts[lo:c].max()))
            wm = mx - delay - 1
            if sync:   # (the synchronous advance, host rows: the A/B reference of these tests)
                g.process_watermark(wm)
            elif batched:   # (the batch's watermarks in one call: fg_advance_progress_async_n)
                held.append(wm)
            else:
                assert op.process_watermark(wm, device_output=True, wait=False) is None
            o.process_watermark(wm)
            exp.append(o.take_rows())
        if held:
            op.process_watermarks(held)
        nb += 1
        ckpt = ckpt_every and nb % ckpt_every == 0
        if ckpt:   # checkpoint while the watermarks' fires are pending and their rows uncollected
            g.prepare_snapshot()
            o.prepare_snapshot()
        if nb % collect_every == 0 or ckpt:
            if sync:
                pass
            elif collect == "host":
                g._rows = [op.collect_fired(host=True)]
            elif collect == "sync_wm":   # the last watermark again, synchronously: fires nothing new
                g._rows = [op.process_watermark(wm)]
            else:
                g._rows = [op.rows_to_host(op.collect_fired())]
            got = g.take_rows()
            assert_rows_equal(got, np.concatenate(exp), cfg["val_type"], f"batch {nb}")
            fired_total += len(got)
            exp = []
            assert g.late_dropped == o_base + o.late_dropped
        if ckpt:   # restore both from their images and go on
            assert op.stats()["rows_fired"] == fired_total
            g2, o2 = g.restore_copy(), o.restore_copy()
            o_base += o.late_dropped
            g.close()
            o.close()
            g, o, op = g2, o2, g2.op
            fired_total = 0
    if sync:
        g.process_watermark(JMAX)
    else:
        op.process_watermark(JMAX, device_output=True, wait=False)
        g._rows.append(op.rows_to_host(op.collect_fired()))
    o.process_watermark(JMAX)
    exp.append(o.take_rows())
    got = g.take_rows()
    assert_rows_equal(got, np.concatenate(exp), cfg["val_type"], "final")
    fired_total += len(got)
    assert op.stats()["rows_fired"] == fired_total
    # a collect with nothing fired since the last one
    assert op.collect_fired().n == 0
    g.close()
    o.close()


@pytest.mark.parametrize("kind", ["tumble", "hop", "cumulate"])
@pytest.mark.parametrize("collect_every", [1, 2])
def test_async_watermarks_match_oracle(oracle_mod, kind, collect_every):
    _run(oracle_mod, _cfg(kind), collect_every=collect_every)


@pytest.mark.parametrize("kind", ["tumble", "hop", "cumulate"])
def test_batched_watermarks_match_oracle(oracle_mod, kind):
    """fg_advance_progress_async_n (ABI 13): each batch's six watermarks in one call, rows as the
    oracle's after every watermark"""
    _run(oracle_mod, _cfg(kind), batched=True, collect_every=2)


def test_batched_watermarks_datastream_out_of_order(oracle_mod):
    _run(oracle_mod, _cfg("tumble", mode="datastream", vt="i64"), batched=True, jitter=1500, delay=200)


@pytest.mark.parametrize("kind", ["tumble", "hop", "cumulate"])
@pytest.mark.parametrize("sync", [False, True], ids=["async", "sync"])
def test_async_watermarks_checkpoint_restore(oracle_mod, kind, sync):
    """prepareSnapshotPreBarrier + snapshotState with fires pending and rows uncollected, then
    initializeState of a new operator from the image; out of order, late data. (Also with the
    synchronous advance: CUMULATE once lost the rows of a key whose post-restore record landed in
    a slice fired before the checkpoint, when the first watermark after the restore passed the
    re-fire horizon and fired the next step window -- the fused flush+fire ran before the re-fire
    had folded that record into the cumulative window's first slice.)"""
    _run(oracle_mod, _cfg(kind), jitter=1500, delay=300, ckpt_every=4, collect_every=2, sync=sync)


@pytest.mark.parametrize("collect", ["host", "sync_wm"])
def test_async_rows_to_host_and_sync_watermark(oracle_mod, collect):
    """fg_collect_fired_to(FG_HOST) returns the async rows in library-owned host memory (what the
    JNI collectFired wraps in direct buffers); a synchronous watermark while async rows are
    uncollected returns them ahead of its own (none is dropped)."""
    _run(oracle_mod, _cfg("hop"), collect_every=2, collect=collect)


def test_async_watermarks_zipf(oracle_mod):
    """Hot keys (Zipf 1.1): the heavy-region pass behind deferred fires."""
    _run(oracle_mod, _cfg("tumble"), n=2_000_000, keys=200_000, batch=400_000, zipf=1.1, jitter=800, delay=500,
         collect_every=2)


@pytest.mark.parametrize("kind", ["tumble", "hop"])
def test_async_watermarks_out_of_order_late(oracle_mod, kind):
    """Jitter beyond the watermark delay: late records are dropped between async advances."""
    _run(oracle_mod, _cfg(kind), jitter=1500, delay=300, collect_every=2)


def test_async_watermarks_datastream(oracle_mod):
    _run(oracle_mod, _cfg("tumble", mode="datastream", vt="i64"), collect_every=2)


def test_async_watermarks_region_growth(oracle_mod):
    """Regions sized for 1,000 keys: the deferred fires' regions overflow and are split and redone
    when the fire completes (at the next call), every row still emitted once."""
    _run(oracle_mod, _cfg("tumble"), keys=60_000, regions_small=True, collect_every=2)


def test_async_advance_rejects_allowed_lateness():
    import flink_amd as F
    op = F.WindowAggOperator(F.tumbling(1000), aggs=("sum",), val_type="i64", mode="datastream",
                             expected_keys=1000, allowed_lateness=500)
    try:
        with pytest.raises(F.WindowSpecError):
            op.process_watermark(1000, device_output=True, wait=False)
    finally:
        op.close()
