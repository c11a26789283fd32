"""Pin the oracle (CPU restatement) against the reference's own known answers."""
import pytest

from tests.fixture_runner import KIND, MODE, VT, load_assigner_cases, load_operator_cases, run_case

OP_CASES = load_operator_cases()
AS = load_assigner_cases()


def make_oracle(O):
    def mk(cfg):
        return O.OracleOperator(mode=MODE[cfg["mode"]], kind=KIND[cfg["kind"]], size=cfg["size"],
                                slide=cfg["slide"], offset=cfg["offset"], tz_offset_ms=cfg["tz_offset_ms"],
                                val_type=VT[cfg["val_type"]], count_star_index=cfg["count_star_index"],
                                proctime=cfg.get("proctime", False), zone=cfg.get("zone"),
                                allowed_lateness=cfg.get("allowed_lateness", 0), purging=cfg.get("purging", False))
    return mk


@pytest.mark.parametrize("case", OP_CASES, ids=[c["name"] for c in OP_CASES])
def test_operator_golden(oracle_mod, case):
    results, late = run_case(case, make_oracle(oracle_mod))
    assert results, "fixture produced no checkpoints"
    for step, got, exp in results:
        assert got == exp, f"{case['name']} step {step}: got {got} expected {exp}"
    if case["expected_late_dropped"] is not None:
        assert late == case["expected_late_dropped"]


@pytest.mark.parametrize("case", AS["cases"], ids=[c["name"] for c in AS["cases"]])
def test_assigner_golden(oracle_mod, case):
    c = case["config"]
    cs = 0 if c["kind"] == "hop" else -1
    op = oracle_mod.OracleOperator(kind=KIND[c["kind"]], size=c["size"], slide=c["slide"], offset=c["offset"],
                                   tz_offset_ms=c["tz_offset_ms"], count_star_index=cs, zone=c.get("zone"),
                                   windowed=c.get("windowed", False))
    for ts, exp in case.get("assign", []):
        assert op.assign_slice_end(ts) == exp
    for w, exp in case.get("window_start", []):
        assert op.window_start(w) == exp
    for w, exp in case.get("expired", []):
        assert op.expired_slices(w) == exp
    for s, mr, lst in case.get("merge", []):
        got_mr, got_l = op.merge_slices(s)
        assert got_mr == mr and got_l == lst
    for w, empty, exp in case.get("next_trigger", []):
        assert op.next_trigger_window(w, empty) == exp


@pytest.mark.parametrize("case", AS["errors"], ids=[e["message"][:40] for e in AS["errors"]])
def test_assigner_errors(oracle_mod, case):
    c = case["config"]
    with pytest.raises(ValueError) as ei:
        oracle_mod.OracleOperator(kind=KIND[c["kind"]], size=c["size"], slide=c["slide"], offset=c["offset"],
                                  count_star_index=c.get("count_star_index", 0))
    assert str(ei.value) == case["message"]


def test_next_trigger_watermark(oracle_mod):
    # TimeWindowUtil.getNextTriggerWatermark (TimeWindowUtil.java:187-210); Long.MAX_VALUE passthrough
    O = oracle_mod
    assert O.next_trigger_watermark(999, 1000) == 1999
    assert O.next_trigger_watermark(1000, 1000) == 1999
    assert O.next_trigger_watermark(998, 1000) == 999
    assert O.next_trigger_watermark(-1, 1000) == 999
    assert O.next_trigger_watermark(-1001, 1000) == -1
    assert O.next_trigger_watermark(O.JMAX, 1000) == O.JMAX


def test_window_start_java_remainder(oracle_mod):
    # TimeWindow.getWindowStartWithOffset with Java's truncated % (TimeWindow.java:222-224)
    L = oracle_mod.lib()
    # ts < offset - size: (ts - offset + size) is negative, Java's % keeps the sign, so the
    # "start" lands ABOVE ts -- the reference quirk is kept bit for bit.
    assert L.or_window_start_with_offset(-2500, 0, 1000) == -2000
    assert L.or_window_start_with_offset(2500, 0, 1000) == 2000
    assert L.or_window_start_with_offset(-500, 0, 1000) == -1000
    assert L.or_window_start_with_offset(-1500, 0, 1000) == -1000
    assert L.or_window_start_with_offset(-2000, 0, 1000) == -2000


def test_sum0_known_answers(oracle_mod):
    """SUM0 (Sum0AggFunction.java:60-63,97-98,136-137): 0-initialised and never NULL, where
    SUM (SumAggFunction) is NULL for a window without non-null values; BIGINT wraps as long."""
    O = oracle_mod
    import numpy as np
    big = (1 << 63) - 1
    for vt, vals in ((O.VAL_I64, [0, 0, 5, 0, 7, big, 1]), (O.VAL_F64, [0.0, 0.0, 5.0, 0.0, 7.0, 1.5, 2.5])):
        o = O.OracleOperator(kind=O.TUMBLE, size=1000, val_type=vt)
        key = np.array([1, 1, 2, 2, 2, 3, 3], dtype=np.int64)
        ts = np.full(7, 10, dtype=np.int64)
        isnull = np.array([1, 1, 0, 1, 0, 0, 0], dtype=np.uint8)
        val = np.array(vals, dtype=np.int64 if vt == O.VAL_I64 else np.float64)
        o.process_batch(key, ts, val, isnull)
        o.process_watermark(big)
        r = o.take_rows()
        o.close()
        r = r[np.argsort(r["key"])]
        f = "sum0_i" if vt == O.VAL_I64 else "sum0_d"
        assert list(r["sum_null"]) == [1, 0, 0]
        if vt == O.VAL_I64:
            assert list(r[f]) == [0, 12, -(1 << 63)]   # Long.MAX_VALUE + 1 wraps
        else:
            assert list(r[f]) == [0.0, 12.0, 4.0]


@pytest.mark.parametrize("zone,fn,arg,exp", AS["timeutil"], ids=[f"{v[0]}-{v[1]}-{v[2]}" for v in AS["timeutil"]])
def test_time_window_util(oracle_mod, zone, fn, arg, exp):
    """TimeWindowUtilTest known answers (toUtcTimestampMills / toEpochMillsForTimer /
    toEpochMills in Asia/Shanghai and in America/Los_Angeles across its 2021 transitions)."""
    op = oracle_mod.OracleOperator(kind=oracle_mod.TUMBLE, size=1000, zone=zone)
    assert getattr(op, fn)(arg) == exp
    op.close()


def test_dst_next_trigger_watermark(oracle_mod):
    """getNextTriggerWatermark's daylight-saving branch (TimeWindowUtil.java:194-199): in
    America/Los_Angeles the next trigger after a watermark in the 2021-03-14 gap hour is the
    first skipped instant's hour, and zones without daylight saving take the plain branch."""
    H = 3600 * 1000
    la = oracle_mod.OracleOperator(kind=oracle_mod.TUMBLE, size=H, zone="America/Los_Angeles")
    # 09:30 UTC = 01:30 PST -> window [01:00, 02:00) local ends in the gap: trigger 09:59:59.999 UTC
    assert la.next_trigger(1615714200000) == 1615715999999
    # 10:00 UTC = 03:00 PDT -> next local hour end 04:00 -> 10:59:59.999 UTC
    assert la.next_trigger(1615716000000) == 1615719599999
    la.close()
    sh = oracle_mod.OracleOperator(kind=oracle_mod.TUMBLE, size=H, zone="Asia/Shanghai")
    assert sh.next_trigger(1615714200000) == oracle_mod.next_trigger_watermark(1615714200000, H)
    sh.close()
