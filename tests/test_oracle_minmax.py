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
