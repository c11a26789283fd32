"""fg_advance_progress_async / fg_collect_fired (ABI 11) on the GPU.

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
         regions_small=False):
    from tests.gpu_adapter import GpuOperator
    key, ts, val, _ = make_stream(n, keys, cfg["val_type"], jitter_ms=jitter)
    g = GpuOperator(cfg, expected_keys=1000 if regions_small else keys, buffer_records=4 * batch)
    o = oracle_mk(O, cfg)
    op = g.op
    exp = []
    fired_total = 0
    mx = np.iinfo(np.int64).min
    nb = 0
    for lo in range(0, n, batch):
        hi = min(n, lo + batch)
        op.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        # watermarks at sub-batch boundaries (max rowtime so far - delay - 1)
        for c in np.linspace(lo, hi, wms_per_batch + 1)[1:].astype(np.int64):
            mx = max(mx, int(ts[lo:c].max()))
            wm = mx - delay - 1
            assert op.process_watermark(wm, device_output=True, wait=False) is None
            o.process_watermark(wm)
            exp.append(o.take_rows())
        nb += 1
        if nb % collect_every == 0:
            r = op.collect_fired()
            got = op.rows_to_host(r)
            g._rows = [got]
            assert_rows_equal(g.take_rows(), np.concatenate(exp), cfg["val_type"], f"batch {nb}")
            fired_total += len(got)
            exp = []
            assert op.num_late_records_dropped == o.late_dropped
    op.process_watermark(JMAX, device_output=True, wait=False)
    o.process_watermark(JMAX)
    exp.append(o.take_rows())
    got = op.rows_to_host(op.collect_fired())
    g._rows = [got]
    assert_rows_equal(g.take_rows(), np.concatenate(exp), cfg["val_type"], "final")
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
