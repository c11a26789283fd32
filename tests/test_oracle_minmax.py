"""Oracle MIN / MAX (MinAggFunction.java:56-90, MaxAggFunction.java:56-96) on randomized
streams: the restatement against a direct numpy group-by of the same records. The literal
values are pinned by the reference's own vectors -- WindowAggregateITCase's MAX(`double`)
and MIN(`float`) per (name, window) for tumble / hop / cumulate (tests/golden,
itcase_*_max_double / itcase_*_min_float, run on the oracle in test_oracle_golden.py and on
the GPU in test_gpu_parity.py::test_golden_cases_on_gpu); this file adds coverage at scale."""
import numpy as np
import pytest

from tests.streams import make_stream

JMAX = (1 << 63) - 1


@pytest.mark.parametrize("vt", ["i64", "f64"])
@pytest.mark.parametrize("kind", ["tumble", "hop"])
def test_oracle_min_max_match_group_by(oracle_mod, vt, kind):
    O = oracle_mod
    n, keys, size, slide = 60_000, 500, 1000, 500
    key, ts, val, isnull = make_stream(n, keys, vt, rate_per_ms=20, null_frac=0.2)
    op = O.OracleOperator(kind=O.TUMBLE if kind == "tumble" else O.HOP, size=size,
                          slide=0 if kind == "tumble" else slide, val_type=O.VAL_I64 if vt == "i64" else O.VAL_F64)
    op.process_batch(key, ts, val, isnull)
    op.process_watermark(JMAX)
    rows = op.take_rows()
    op.close()
    ends = [(ts // size) * size + size] if kind == "tumble" else \
        [(ts // slide) * slide + slide + j * slide for j in range(size // slide)]
    sfx = "_i" if vt == "i64" else "_d"
    for r in rows[:2000]:
        m = (key == r["key"]) & np.any([e == r["window_end"] for e in ends], axis=0)
        assert m.sum() == r["cnt_star"]
        v = val[m & (isnull == 0)]
        assert len(v) == r["cnt_val"]
        if len(v) == 0:
            assert r["sum_null"] == 1
            continue
        assert r["min" + sfx] == v.min() and r["max" + sfx] == v.max()


def _java_double_key(x):
    """Double.compareTo's order as an integer key (doubleToLongBits: every NaN canonical)."""
    b = np.float64(x).view(np.int64)
    if np.isnan(x):
        b = np.int64(0x7FF8000000000000)
    return int(b) if b >= 0 else int(b ^ np.int64(0x7FFFFFFFFFFFFFFF))


def test_oracle_datastream_min_max_compare_to(oracle_mod):
    """DataStream WindowedStream.min / max over DOUBLE: ComparableAggregator.reduce
    (ComparableAggregator.java:83-104, Comparator.java:48-137) keeps the element whose field wins
    under Double.compareTo -- -0.0 below +0.0, NaN above +inf (MAX picks it, MIN avoids it),
    every NaN equal and returned canonical. A hand-written reduce over the arrival order is the
    check; SQL's Min/MaxAggFunction (primitive comparison) differs on exactly these values."""
    O = oracle_mod
    nan2 = np.int64(0x7FF0000000000001).view(np.float64)   # a signalling-payload NaN
    windows = [[1.0, np.nan, -0.0, 0.0], [0.0, -0.0], [np.inf, nan2, -np.inf], [-0.0, 0.0], [nan2]]
    key, ts, val = [], [], []
    for w, vs in enumerate(windows):
        for i, v in enumerate(vs):
            key.append(7)
            ts.append(w * 1000 + i)
            val.append(v)
    key, ts, val = np.array(key, np.int64), np.array(ts, np.int64), np.array(val, np.float64)
    op = O.OracleOperator(mode=O.MODE_DATASTREAM, kind=O.TUMBLE, size=1000, val_type=O.VAL_F64)
    op.process_batch(key, ts, val)
    op.process_watermark(JMAX)
    rows = op.take_rows()
    op.close()
    assert len(rows) == len(windows)
    rows = rows[np.argsort(rows["window_end"])]
    for r, vs in zip(rows, windows):
        mn = mx = vs[0]
        for v in vs[1:]:   # reduce(value1 = state, value2 = element)
            if not _java_double_key(mn) < _java_double_key(v):
                mn = v
            if not _java_double_key(mx) > _java_double_key(v):
                mx = v
        canon = lambda x: np.int64(0x7FF8000000000000) if np.isnan(x) else np.float64(x).view(np.int64)
        assert r["min_d"].view(np.int64) == canon(mn), (vs, r["min_d"])
        assert r["max_d"].view(np.int64) == canon(mx), (vs, r["max_d"])
    # where the orders part ways: MAX of [1.0, NaN, -0.0, 0.0] is NaN (the primitive `>` keeps 1.0)
    assert rows[0]["min_d"].view(np.int64) == np.float64(-0.0).view(np.int64)
    assert np.isnan(rows[0]["max_d"]) and np.isnan(rows[4]["min_d"])
