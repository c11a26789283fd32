"""The level-C operator's watermark hold on a trickle stream (flink_amd.operator.HeldWatermarkOperator,
the Python mirror of GpuSlicingWindowAggOperator's policy).

Records arrive in 500-record chunks -- far below the 2^20-record micro-batch, so a micro-batch
never fills -- with a watermark after each chunk. The reference forwards every watermark with the
rows it fired (SlicingWindowOperator.java:207-210); the GPU operator holds a watermark while its
fires run and must release it no later than the next watermark: every window's rows come out
before the watermark that fired it is forwarded, and while the NEXT input watermark is processed at
the latest. A held watermark on an idle stream goes out at the processing-time bound. Rows equal
the oracle's (same schedule), and the synchronous path emits the same rows.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, KEYS, CHUNK = 300_000, 5_000, 500


def _run(async_wm, batch_records=1 << 20, idle_check=False):
    import flink_amd as F
    from flink_amd.operator import HeldWatermarkOperator
    from tests.streams import make_stream
    key, ts, val, _ = make_stream(N, KEYS, "f64", seed=91, jitter_ms=50)
    op = F.WindowAggOperator(F.tumbling(1000), aggs=("count_star", "count", "sum", "avg"), expected_keys=KEYS)
    clock = [0.0]
    h = HeldWatermarkOperator(op, batch_records=batch_records, async_watermarks=async_wm, max_hold_ms=200,
                              clock=lambda: clock[0])
    wms, out_len, mx = [], [], -(1 << 63)
    for lo in range(0, N, CHUNK):
        h.process_elements(key[lo:lo + CHUNK], ts[lo:lo + CHUNK], val[lo:lo + CHUNK])
        mx = max(mx, int(ts[lo:lo + CHUNK].max()))
        clock[0] += 0.001
        h.process_watermark(mx - 60)
        wms.append(mx - 60)
        out_len.append(len(h.output))   # output events after input watermark k was processed
    if idle_check and async_wm:
        assert h.held == wms[-1]
        h.on_processing_time(clock[0] + 0.1)      # within the bound: still held
        assert h.held == wms[-1]
        h.on_processing_time(clock[0] + 0.25)     # past it: released without further input
        assert h.held is None and h.output[-1] == ("watermark", wms[-1])
    h.end_input()
    rows = op.process_watermark((1 << 63) - 1)
    late = op.num_late_records_dropped
    op.close()
    return h.output, rows, wms, out_len, late


def _check_timing(output, wms, out_len):
    """window w's rows precede the forwarded watermark that fired it and were emitted while the
    input watermark after the firing one was processed, at the latest"""
    seen_wm = -(1 << 63)
    for i, (kind, x) in enumerate(output):
        if kind == "watermark":
            assert x >= seen_wm
            seen_wm = x
            continue
        # rows: their windows' triggers (end - 1) lie at or below the next forwarded watermark
        nxt = next(w for k2, w in output[i + 1:] if k2 == "watermark")
        assert int(x["window_end"].max()) - 1 <= nxt
        for we in np.unique(x["window_end"]):
            k = next(j for j, w in enumerate(wms) if w >= int(we) - 1)   # the input watermark that fired it
            if k + 1 < len(wms):   # (the last watermark's rows: released by the idle bound / end of input)
                assert i < out_len[k + 1], (int(we), k, i)


@pytest.mark.parametrize("batch_records", [1 << 20, 10_000])
def test_held_watermarks_trickle_stream(oracle_mod, batch_records):
    O = oracle_mod
    from tests.streams import make_stream
    output, tail, wms, out_len, late = _run(True, batch_records, idle_check=batch_records == 1 << 20)
    _check_timing(output, wms, out_len)
    got = np.concatenate([x for k, x in output if k == "rows"] + ([tail] if len(tail) else []))
    key, ts, val, _ = make_stream(N, KEYS, "f64", seed=91, jitter_ms=50)
    o = O.OracleOperator(kind=O.TUMBLE, size=1000, val_type=O.VAL_F64)
    exp = []
    for i, lo in enumerate(range(0, N, CHUNK)):
        o.process_batch(key[lo:lo + CHUNK], ts[lo:lo + CHUNK], val[lo:lo + CHUNK])
        o.process_watermark(wms[i])
        exp.append(o.take_rows())
    o.process_watermark((1 << 63) - 1)
    exp.append(o.take_rows())
    e = np.concatenate(exp)
    assert late == o.late_dropped
    o.close()
    g = got[np.lexsort((got["key"], got["window_end"]))]
    e = e[np.lexsort((e["key"], e["window_end"]))]
    assert len(g) == len(e)
    for f, fe in (("key", "key"), ("window_end", "window_end"), ("count_star", "cnt_star")):
        assert np.array_equal(g[f], e[fe]), f
    a, b = g["sum"], e["sum_d"]
    assert (np.abs(a - b) <= 1e-9 * np.maximum(np.abs(a), np.abs(b))).all()
    # the synchronous path (the reference's timing) emits the same rows
    so, stail, _, _, _ = _run(False, batch_records)
    s = np.concatenate([x for k, x in so if k == "rows"] + ([stail] if len(stail) else []))
    s = s[np.lexsort((s["key"], s["window_end"]))]
    assert np.array_equal(s["key"], g["key"]) and np.array_equal(s["count_star"], g["count_star"])
