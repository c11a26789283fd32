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
                                proctime=cfg.get("proctime", False))
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
                                   tz_offset_ms=c["tz_offset_ms"], count_star_index=cs)
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
