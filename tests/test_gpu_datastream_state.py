"""DataStream WindowOperator state, both ways across a checkpoint (the Python mirror of the JVM
shim's GpuWindowOperator, flink_amd.datastream): the GPU operator's snapshot is the reference's
keyed-state image -- "window-contents" (one reduced Tuple2 value per (key, TimeWindow),
WindowOperatorBuilder.java:71,150-172) and "window-timers" (trigger at maxTimestamp, cleanup at
maxTimestamp + allowedLateness, WindowOperator.java:225,630-642) -- and it restores from one.

Per case, at the checkpoint:
  * the GPU image equals the oracle's heap image (the oracle restates WindowOperator with
    per-window state): the same (key, window) entries with the same values (bit-exact for BIGINT
    and MIN / MAX; DOUBLE sums within the north_star tolerance) and the same timers of every
    (key, window) holding state;
  * GPU -> CPU: an oracle restored from the GPU image continues exactly as the oracle restored
    from its own image;
  * CPU -> GPU: a GPU operator restored from the oracle's image continues exactly as that oracle.
"""
import numpy as np
import pytest

from tests.streams import batches_with_watermarks, make_stream

pytestmark = pytest.mark.gpu
REL = 1e-9
JMAX = (1 << 63) - 1

#      name                  kind      size  slide vt     agg    lateness purging jitter delay
CASES = [
    ("tumble_sum_i64",       "tumble", 1000, 0,    "i64", "sum", 0,       False,  600,   200),
    ("tumble_sum_f64_late",  "tumble", 1000, 0,    "f64", "sum", 700,     False,  1500,  100),
    ("tumble_min_f64_spec",  "tumble", 1000, 0,    "f64", "min", 0,       False,  600,   200),
    ("tumble_max_i64_late",  "tumble", 700,  0,    "i64", "max", 500,     False,  1200,  100),
    ("sliding_sum_i64",      "hop",    3000, 1000, "i64", "sum", 0,       False,  900,   300),
    ("sliding_sum_f64_late", "hop",    3000, 1000, "f64", "sum", 1200,    False,  2500,  100),
    ("sliding_min_i64",      "hop",    2000, 500,  "i64", "min", 0,       False,  700,   100),
    ("sliding_max_f64_late", "hop",    3000, 1000, "f64", "max", 800,     False,  2000,  200),
    ("sliding_sum_purging",  "hop",    3000, 1000, "i64", "sum", 1000,    True,   2500,  100),
]
# WindowedStream.aggregate(AggregateFunction) with the GPU's functions (GpuAggregateFunctions):
# "window-contents" is an AggregatingState of the accumulator (count; sum; (sum, count); extreme)
AGG_CASES = [
    ("agg_tumble_count",       "tumble", 1000, 0,    "i64", "count", 0,   False, 600,  200),
    ("agg_tumble_avg_f64",     "tumble", 1000, 0,    "f64", "avg",   700, False, 1500, 100),
    ("agg_tumble_sum_i64",     "tumble", 1000, 0,    "i64", "sum",   0,   False, 600,  200),
    ("agg_sliding_avg_i64",    "hop",    3000, 1000, "i64", "avg",   0,   False, 900,  300),
    ("agg_sliding_min_f64",    "hop",    3000, 1000, "f64", "min",   800, False, 2000, 200),
    ("agg_sliding_max_i64",    "hop",    2000, 500,  "i64", "max",   0,   False, 700,  100),
    ("agg_sliding_count_late", "hop",    3000, 1000, "f64", "count", 1200, False, 2500, 100),
]


def _oracle(O, kind, size, slide, vt, lateness, purging):
    return O.OracleOperator(mode=O.MODE_DATASTREAM, kind=O.TUMBLE if kind == "tumble" else O.HOP, size=size,
                            slide=slide, val_type=O.VAL_I64 if vt == "i64" else O.VAL_F64,
                            allowed_lateness=lateness, purging=purging)


def _oracle_field(agg, vt):
    return {"sum": "sum", "min": "min", "max": "max"}[agg] + ("_i" if vt == "i64" else "_d")


def _oracle_value(rows, agg, vt):
    """the emitted value's bits from oracle rows: the field, or the GPU aggregate function's
    getResult -- COUNT the count, AVG (double) sum / count"""
    if agg == "count":
        return rows["cnt_star"].astype(np.int64)
    if agg == "avg":
        s = rows["sum_d"] if vt == "f64" else rows["sum_i"].astype(np.float64)
        return (s / rows["cnt_star"].astype(np.float64)).view(np.int64)
    return np.ascontiguousarray(rows[_oracle_field(agg, vt)]).view(np.int64)


def _sorted(k, e, v):
    o = np.lexsort((e, k))
    return k[o], e[o], v[o]


def _assert_values(a, b, vt, agg, ctx):
    if (vt == "f64" and agg == "sum") or agg == "avg":
        x, y = a.view(np.float64), b.view(np.float64)
        ok = np.abs(x - y) <= REL * np.maximum(np.abs(x), np.abs(y)) + 1e-300
        assert ok.all(), f"{ctx}: f64 sums differ: {x[~ok][:5]} vs {y[~ok][:5]}"
    else:
        bad = np.flatnonzero(a != b)
        assert len(bad) == 0, f"{ctx}: values differ at {bad[:5]}: {a[bad[:5]]} vs {b[bad[:5]]}"


def _rows_equal(g, o_rows, vt, agg, ctx):
    ov = _oracle_value(o_rows, agg, vt)
    gk, ge, gv = _sorted(g["key"], g["window_end"], g["value"])
    ok_, oe, ov = _sorted(o_rows["key"].astype(np.int64), o_rows["window_end"].astype(np.int64), ov)
    assert len(gk) == len(ok_), f"{ctx}: {len(gk)} rows vs {len(ok_)}"
    assert np.array_equal(gk, ok_) and np.array_equal(ge, oe), f"{ctx}: (key, window) rows differ"
    assert np.array_equal(g["timestamp"], g["window_end"] - 1)
    _assert_values(gv, ov, vt, agg, ctx)


def _drive(g, o, key, ts, val, lo_hi_wm, vt, agg, tag):
    for step, (lo, hi, wm) in enumerate(lo_hi_wm):
        if g is not None:
            g.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        rows = g.process_watermark(wm) if g is not None else None
        o.process_watermark(wm)
        orow = o.take_rows()
        if g is not None:
            _rows_equal(rows, orow, vt, agg, f"{tag} step {step}")
        else:
            yield orow


@pytest.mark.parametrize("case", CASES + AGG_CASES, ids=[c[0] for c in CASES + AGG_CASES])
def test_datastream_window_contents_both_ways(oracle_mod, case):
    from flink_amd.datastream import DataStreamWindowOperator
    O = oracle_mod
    name, kind, size, slide, vt, agg, lateness, purging, jitter, delay = case
    api = "aggregate" if name.startswith("agg_") else "reduce"
    n, keys, batch = 240_000, 3000, 8_000
    key, ts, val, _ = make_stream(n, keys, vt, jitter_ms=jitter, rate_per_ms=20,
                                  specials=0.05 if "spec" in name else 0.0)
    val = np.ascontiguousarray(val)
    steps = list(batches_with_watermarks(n, batch, ts, delay))
    cut = len(steps) // 2
    mk = lambda: DataStreamWindowOperator(kind, size, slide, val_type=vt, agg=agg, allowed_lateness=lateness,
                                          purging=purging, api=api, expected_keys=keys, buffer_records=1 << 18)
    g = mk()
    o = _oracle(O, kind, size, slide, vt, lateness, purging)
    for _ in _drive(g, o, key, ts, val, steps[:cut], vt, agg, "before"):
        pass
    # -- the checkpoint: the GPU image is the reference's
    img_g = g.snapshot()
    o.prepare_snapshot()
    img_o = o.ds_state_image(agg)
    zeros_g = np.zeros(len(img_g["key"]), np.int64)
    gk, ge, gv = _sorted(img_g["key"], img_g["window_end"], img_g.get("value", zeros_g))
    ok_, oe, ov = _sorted(img_o["key"], img_o["window_end"], img_o["value"])
    assert len(gk) == len(ok_) and np.array_equal(gk, ok_) and np.array_equal(ge, oe), \
        f"window-contents entries differ: {len(gk)} vs {len(ok_)}"
    if "value" in img_g:   # (the accumulator's value part: SUM / AVG sum, MIN, MAX, the reduced field)
        _assert_values(gv, ov, vt, "sum" if agg == "avg" else agg, "window-contents")
    if "count" in img_g:   # (COUNT, AVG: the accumulator's count)
        _, _, gc = _sorted(img_g["key"], img_g["window_end"], img_g["count"])
        _, _, oc = _sorted(img_o["key"], img_o["window_end"], img_o["count"])
        assert np.array_equal(gc, oc), "window-contents counts differ"
    if api == "reduce":   # (a reduce's image carries no count: the reference's state is the Tuple2)
        img_o = {k: v for k, v in img_o.items() if k != "count"}
    elif agg not in ("count", "avg"):
        img_o = {k: v for k, v in img_o.items() if k != "count"}
    if agg == "count":
        img_o = {k: v for k, v in img_o.items() if k != "value"}
    assert np.array_equal(img_g["window_start"], img_g["window_end"] - size)
    live = set(zip(ok_.tolist(), oe.tolist()))
    t_o = {(k, e, t) for k, e, t in zip(img_o["timer_key"].tolist(), img_o["timer_window_end"].tolist(),
                                         img_o["timer_ts"].tolist()) if (k, e) in live}
    t_g = set(zip(img_g["timer_key"].tolist(), img_g["timer_window_end"].tolist(), img_g["timer_ts"].tolist()))
    assert t_g == t_o, f"window-timers differ: {len(t_g - t_o)} extra, {len(t_o - t_g)} missing"
    # -- GPU -> CPU: the oracle restored from the GPU image continues as from its own
    cfg = dict(kind=O.TUMBLE if kind == "tumble" else O.HOP, size=size, slide=slide,
               val_type=O.VAL_I64 if vt == "i64" else O.VAL_F64, allowed_lateness=lateness, purging=purging)
    o_self = O.OracleOperator.from_ds_state_image(img_o, **cfg)
    o_from_g = O.OracleOperator.from_ds_state_image(img_g, **cfg)
    exp = list(_drive(None, o_self, key, ts, val, steps[cut:], vt, agg, "self"))
    got = list(_drive(None, o_from_g, key, ts, val, steps[cut:], vt, agg, "from-gpu"))
    for i, (a, b) in enumerate(zip(got, exp)):
        ak, ae, av = _sorted(a["key"], a["window_end"], _oracle_value(a, agg, vt))
        bk, be, bv = _sorted(b["key"], b["window_end"], _oracle_value(b, agg, vt))
        assert np.array_equal(ak, bk) and np.array_equal(ae, be), f"GPU->CPU step {i}: rows differ"
        _assert_values(av, bv, vt, agg, f"GPU->CPU step {i}")
    # -- CPU -> GPU: the GPU restored from the oracle's image continues as that oracle
    g2 = mk()
    g2.restore(img_o)
    o2 = O.OracleOperator.from_ds_state_image(img_o, **cfg)
    for _ in _drive(g2, o2, key, ts, val, steps[cut:], vt, agg, "CPU->GPU"):
        pass
    rows = g2.process_watermark(JMAX)
    o2.process_watermark(JMAX)
    _rows_equal(rows, o2.take_rows(), vt, agg, "CPU->GPU end of input")
    g.close()
    g2.close()
