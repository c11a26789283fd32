"""Parity of the HIP engine (libflinkgpu.so via flink_amd) with the oracle and the
reference's golden vectors. Bit-exact for keys, windows, COUNT(*), COUNT, i64 SUM/AVG and
late-drop counts; |a - b| <= 1e-9 * max(|a|, |b|) for f64 SUM/AVG (north_star tolerance:
the GPU sums a (key, slice) in a different order than the Java combiner)."""
import numpy as np
import pytest

from tests.fixture_runner import KIND, MODE, VT, load_operator_cases, run_case
from tests.streams import batches_with_watermarks, make_stream

pytestmark = pytest.mark.gpu
REL_TOL = 1e-9
JMAX = (1 << 63) - 1

OP_CASES = load_operator_cases()


def gpu_mk(cfg, **kw):
    from tests.gpu_adapter import GpuOperator
    return GpuOperator(cfg, **kw)


def oracle_mk(O, cfg):
    return O.OracleOperator(mode=MODE[cfg["mode"]], kind=KIND[cfg["kind"]], size=cfg["size"], slide=cfg["slide"],
                            offset=cfg["offset"], tz_offset_ms=cfg["tz_offset_ms"], val_type=VT[cfg["val_type"]],
                            count_star_index=cfg["count_star_index"], proctime=cfg.get("proctime", False),
                            zone=cfg.get("zone"), windowed=cfg.get("windowed", False),
                            allowed_lateness=cfg.get("allowed_lateness", 0), purging=cfg.get("purging", False))


@pytest.mark.parametrize("case", OP_CASES, ids=[c["name"] for c in OP_CASES])
def test_golden_cases_on_gpu(case):
    results, late = run_case(case, gpu_mk)
    for step, got, exp in results:
        assert got == exp, f"{case['name']} step {step}: got {got} expected {exp}"
    if case["expected_late_dropped"] is not None:
        assert late == case["expected_late_dropped"]


TOLERANCE = {}   # test id -> {column: [rows checked, rows passing only on the summation-order bound]}


def tolerance_record(ctx, col, rows, relaxed):
    import os
    tid = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    d = TOLERANCE.setdefault(tid, {}).setdefault(col, [0, 0])
    d[0] += rows
    d[1] += relaxed


def sort_rows(r):
    # (window_end, key), then the accumulators: with allowed lateness one (key, window) may fire
    # several times in a step (every late element re-fires it, EventTimeTrigger.onElement)
    return r[np.lexsort((r["max_d"].view(np.int64), r["max_i"], r["min_d"].view(np.int64), r["min_i"], r["sum_d"],
                         r["sum_i"], r["cnt_star"], r["key"], r["window_end"]))]


F64_EPS = float(np.finfo(np.float64).eps)


def assert_rows_equal(got, exp, vt, ctx="", sum0=True, minmax=(), vmax=None, sums=None, aggs=None):
    """vmax (mixed-sign DOUBLE streams): besides the 1e-9 relative bar, a row passes when
    |a - b| <= 2 (n - 1) eps n vmax -- the worst-case difference of two summation orders of
    n values with |x| <= vmax (each within (n - 1) eps sum|x| of the exact sum); a near-
    cancelling sum has no meaningful relative error in any order, the reference's included."""
    assert len(got) == len(exp), f"{ctx}: {len(got)} rows vs {len(exp)} expected"
    if len(got) == 0:
        return
    g, e = sort_rows(got), sort_rows(exp)
    no_count = bool((g["cnt_val"] == -1).all())   # the operator's list has no COUNT(v)
    for f in ("key", "window_start", "window_end", "cnt_star", "cnt_val", "sum_null", "avg_null", "out_ts"):
        if f == "cnt_val" and no_count:
            continue
        bad = np.nonzero(g[f] != e[f])[0]
        assert len(bad) == 0, f"{ctx}: field {f} differs at {bad[:5]}: {g[f][bad[:5]]} vs {e[f][bad[:5]]}"
    if minmax:   # MIN / MAX operator: bit-exact (order-independent), NULL exactly when SUM is
        ok = e["sum_null"] == 0
        for m in minmax:
            f = m + ("_i" if vt == "i64" else "_d")
            a, b = g[f][ok].view(np.int64), e[f][ok].view(np.int64)
            bad = np.nonzero(a != b)[0]
            assert len(bad) == 0, f"{ctx}: {m.upper()} differs at {bad[:5]}: {g[f][ok][bad[:5]]} vs {e[f][ok][bad[:5]]}"
        if not sums:   # a MIN / MAX-only operator; several accumulators check the SUM family too
            return
    has = (lambda a: True) if aggs is None else (lambda a: a in aggs)   # aggregates the operator emits
    if vt == "i64":
        ok = e["sum_null"] == 0
        if has("sum"):
            assert np.array_equal(g["sum_i"][ok], e["sum_i"][ok]), f"{ctx}: i64 SUM differs"
        ok = e["avg_null"] == 0
        if has("avg"):
            assert np.array_equal(g["avg_i"][ok], e["avg_i"][ok]), f"{ctx}: i64 AVG differs"
        if sum0 and has("sum0"):
            assert np.array_equal(g["sum0_i"], e["sum0_i"]), f"{ctx}: i64 SUM0 differs"
    else:
        for f, nf in (("sum_d", "sum_null"), ("avg_d", "avg_null"), ("sum0_d", None)):
            if (f == "sum0_d" and not sum0) or not has(f[:-2]):
                continue
            ok = e[nf] == 0 if nf else np.ones(len(e), dtype=bool)
            a, b = g[f][ok], e[f][ok]
            rel = REL_TOL * np.maximum(np.abs(a), np.abs(b)) + 1e-300
            bound = rel
            if vmax is not None:
                cnt = e["cnt_val"][ok].astype(np.float64)
                order = 2.0 * np.maximum(cnt - 1, 0) * F64_EPS * cnt * vmax
                bound = np.maximum(bound, order / np.maximum(cnt, 1) if f == "avg_d" else order)
            err = np.abs(a - b) <= bound
            # rows that pass on the summation-order bound only (not on 1e-9 relative)
            tolerance_record(ctx, f, int(len(a)), int(((np.abs(a - b) > rel) & err).sum()))
            assert err.all(), f"{ctx}: f64 {f} beyond tolerance: {a[~err][:5]} vs {b[~err][:5]}"


def drive_both(O, cfg, n, keys, batch, delay, jitter, null_frac=0.0, snapshot_at=None, end_wm=JMAX,
               expected_keys=None, kstats=None, stats=None, buffer_records=None, **gen):
    key, ts, val, isnull = make_stream(n, keys, cfg["val_type"], jitter_ms=jitter, null_frac=null_frac, **gen)
    vmax = 1000.0 if gen.get("signed") and cfg["val_type"] == "f64" else None
    mm = tuple(a for a in cfg.get("aggs", ()) if a in ("min", "max"))
    aggs = cfg.get("aggs")
    chk = dict(minmax=mm, vmax=vmax, sums=aggs is None or any(a in ("sum", "avg", "sum0") for a in aggs),
               sum0=aggs is None or "sum0" in aggs, aggs=aggs)
    g = gpu_mk(cfg, expected_keys=keys if expected_keys is None else expected_keys,
               buffer_records=buffer_records or max(batch * 4, 1 << 16),
               kernel_timing=kstats is not None)
    o = oracle_mk(O, cfg)
    o_base = 0
    step = 0
    for lo, hi, wm in batches_with_watermarks(n, batch, ts, delay):
        nl = None if isnull is None else isnull[lo:hi]
        g.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi], nl)
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi], nl)
        g.process_watermark(wm)
        o.process_watermark(wm)
        assert_rows_equal(g.take_rows(), o.take_rows(), cfg["val_type"], f"step {step} wm {wm}", **chk)
        assert g.late_dropped == o_base + o.late_dropped, f"late drops differ at step {step}"
        step += 1
        if snapshot_at is not None and step == snapshot_at:
            g.prepare_snapshot()
            o.prepare_snapshot()
            g2, o2 = g.restore_copy(), o.restore_copy()
            o_base += o.late_dropped
            g.close()
            o.close()
            g, o = g2, o2
    g.process_watermark(end_wm)
    o.process_watermark(end_wm)
    assert_rows_equal(g.take_rows(), o.take_rows(), cfg["val_type"], "final", **chk)
    late = g.late_dropped
    if kstats is not None:
        kstats.update(g.op.kernel_stats())
    if stats is not None:
        stats.update(g.op.stats())
    g.close()
    o.close()
    return late


def cfg_of(kind, size, slide=0, vt="f64", mode="sql", tz=0, offset=0, zone=None):
    c = dict(mode=mode, kind=kind, size=size, slide=slide, offset=offset, tz_offset_ms=tz, val_type=vt,
             count_star_index=0)
    if zone:
        c["zone"] = zone
    return c


LA = "America/Los_Angeles"
SPRING, FALL = 1615708800000, 1636268400000   # 2021-03-14 / 2021-11-07 00:00 local, LA


STREAM_CASES = [
    ("tumble_f64_inorder", cfg_of("tumble", 1000), dict(n=200_000, keys=5000, batch=20_000, delay=0, jitter=0)),
    ("tumble_i64_ooo", cfg_of("tumble", 1000, vt="i64"), dict(n=200_000, keys=3000, batch=7_000, delay=300, jitter=900)),
    ("tumble_i64_wrap", cfg_of("tumble", 500, vt="i64"), dict(n=100_000, keys=100, batch=9_000, delay=0, jitter=200, big_ints=True)),
    ("tumble_f64_nulls_late", cfg_of("tumble", 700), dict(n=150_000, keys=2000, batch=5_000, delay=100, jitter=1500, null_frac=0.2)),
    ("tumble_spread_keys", cfg_of("tumble", 1000), dict(n=100_000, keys=4000, batch=10_000, delay=50, jitter=300, key_spread=True)),
    ("tumble_shanghai", cfg_of("tumble", 3000, tz=8 * 3600 * 1000), dict(n=100_000, keys=1000, batch=6_000, delay=0, jitter=400)),
    ("hop_f64", cfg_of("hop", 3000, 1000), dict(n=200_000, keys=4000, batch=10_000, delay=200, jitter=800)),
    ("hop_i64_late", cfg_of("hop", 5000, 1000, vt="i64"), dict(n=200_000, keys=2000, batch=4_000, delay=100, jitter=3000)),
    ("cumulate_f64", cfg_of("cumulate", 5000, 1000), dict(n=200_000, keys=3000, batch=10_000, delay=100, jitter=600)),
    ("cumulate_i64_late", cfg_of("cumulate", 4000, 500, vt="i64"), dict(n=150_000, keys=1500, batch=3_000, delay=50, jitter=2500)),
    ("ds_tumble_i64", cfg_of("tumble", 1000, vt="i64", mode="datastream"), dict(n=150_000, keys=2000, batch=8_000, delay=100, jitter=700)),
    ("ds_sliding_i64", cfg_of("hop", 3000, 1000, vt="i64", mode="datastream"), dict(n=150_000, keys=2000, batch=8_000, delay=100, jitter=1500)),
    ("tumble_many_regions", cfg_of("tumble", 1000), dict(n=1_000_000, keys=400_000, batch=100_000, delay=0, jitter=0)),
    # >= 64 state regions: two-pass partition + compact / wide merge paths
    ("regions_f64_nulls_late", cfg_of("tumble", 700), dict(n=600_000, keys=150_000, batch=60_000, delay=100, jitter=1500, null_frac=0.2)),
    ("regions_i64_ooo_lanes", cfg_of("tumble", 200, vt="i64"), dict(n=600_000, keys=120_000, batch=50_000, delay=150, jitter=450)),
    ("regions_i64_wrap", cfg_of("tumble", 500, vt="i64"), dict(n=400_000, keys=100_000, batch=40_000, delay=0, jitter=200, big_ints=True)),
    ("regions_hop_f64", cfg_of("hop", 3000, 1000), dict(n=600_000, keys=100_000, batch=40_000, delay=200, jitter=800)),
    ("regions_cumulate_i64_late", cfg_of("cumulate", 4000, 500, vt="i64"), dict(n=500_000, keys=100_000, batch=20_000, delay=50, jitter=2500)),
    ("regions_ds_sliding", cfg_of("hop", 3000, 1000, vt="i64", mode="datastream"), dict(n=400_000, keys=100_000, batch=30_000, delay=100, jitter=1500)),
    ("regions_spread_keys", cfg_of("tumble", 1000), dict(n=500_000, keys=200_000, batch=50_000, delay=50, jitter=300, key_spread=True)),
    # micro-batches of millions of records: pass-2 units span many sub-tiles, merge regions
    # stream many chunks
    ("big_units_f64", cfg_of("tumble", 1000), dict(n=40_000_000, keys=4_000_000, batch=20_000_000, delay=0, jitter=0,
                                                    rate_per_ms=20_000)),
    ("big_units_i64_nulls_ooo", cfg_of("tumble", 1000, vt="i64"), dict(n=16_000_000, keys=500_000, batch=8_000_000,
                                                                       delay=600, jitter=500, null_frac=0.1,
                                                                       rate_per_ms=10_000)),
    # processing-time windows (records carry their arrival time, nothing is late)
    ("proctime_hop_f64", dict(cfg_of("hop", 3000, 1000), proctime=True), dict(n=600_000, keys=100_000, batch=50_000,
                                                                              delay=0, jitter=0)),
    ("proctime_cumulate_i64", dict(cfg_of("cumulate", 4000, 1000, vt="i64"), proctime=True),
     dict(n=400_000, keys=20_000, batch=20_000, delay=0, jitter=0)),
    # Zipf(1.1) hot keys: regions over the skew threshold take the chunked heavy pass
    ("zipf_tumble_f64", cfg_of("tumble", 1000), dict(n=3_000_000, keys=100_000, batch=1_000_000, delay=0, jitter=0,
                                                      rate_per_ms=2_000, zipf=1.1)),
    ("zipf_tumble_i64_nulls_late", cfg_of("tumble", 1000, vt="i64"), dict(n=3_000_000, keys=100_000, batch=1_000_000,
                                                                          delay=200, jitter=600, null_frac=0.1,
                                                                          rate_per_ms=2_000, zipf=1.1)),
    ("zipf_hop_f64", cfg_of("hop", 3000, 1000), dict(n=3_000_000, keys=50_000, batch=1_000_000, delay=100, jitter=300,
                                                      rate_per_ms=1_000, zipf=1.1)),
    ("zipf_cumulate_i64", cfg_of("cumulate", 4000, 1000, vt="i64"), dict(n=3_000_000, keys=50_000, batch=1_000_000,
                                                                         delay=0, jitter=0, rate_per_ms=1_000,
                                                                         zipf=1.3)),
    ("zipf_ds_tumble_i64", cfg_of("tumble", 2000, vt="i64", mode="datastream"),
     dict(n=3_000_000, keys=100_000, batch=1_000_000, delay=0, jitter=0, rate_per_ms=1_000, zipf=1.1)),
    # mixed-sign DOUBLE values (SumAggFunction / AvgAggFunction over [-1000, 1000)), and pairs
    # of records whose values cancel within a (key, window): the summation-order bound applies
    ("signed_tumble_f64", cfg_of("tumble", 1000), dict(n=400_000, keys=20_000, batch=40_000, delay=100, jitter=300,
                                                        signed=True)),
    ("signed_hop_f64_regions", cfg_of("hop", 3000, 1000), dict(n=600_000, keys=100_000, batch=60_000, delay=200,
                                                                jitter=800, signed=True)),
    ("cancel_tumble_f64", cfg_of("tumble", 1000), dict(n=400_000, keys=5_000, batch=40_000, delay=0, jitter=0,
                                                        signed=True, cancel=True)),
    ("cancel_cumulate_f64_regions", cfg_of("cumulate", 4000, 1000), dict(n=600_000, keys=100_000, batch=50_000,
                                                                         delay=100, jitter=300, signed=True,
                                                                         cancel=True)),
    ("signed_zipf_tumble_f64", cfg_of("tumble", 1000), dict(n=3_000_000, keys=100_000, batch=1_000_000, delay=0,
                                                             jitter=0, rate_per_ms=2_000, zipf=1.1, signed=True)),
    # America/Los_Angeles zone rules across the 2021 gap (spring) and overlap (fall):
    # TIMESTAMP_LTZ windows in local time, DST trigger times, late records
    ("dst_tumble_spring_f64", cfg_of("tumble", 3600_000, zone=LA),
     dict(n=400_000, keys=3000, batch=20_000, delay=600_000, jitter=1_800_000, t0=SPRING, rate_per_ms=0.02)),
    ("dst_hop_fall_i64", cfg_of("hop", 4 * 3600_000, 3600_000, vt="i64", zone=LA),
     dict(n=400_000, keys=2000, batch=25_000, delay=300_000, jitter=2_400_000, t0=FALL, rate_per_ms=0.02)),
    ("dst_cumulate_spring_f64", cfg_of("cumulate", 4 * 3600_000, 3600_000, zone=LA),
     dict(n=300_000, keys=2000, batch=15_000, delay=900_000, jitter=3_000_000, t0=SPRING - 3600_000,
          rate_per_ms=0.02, null_frac=0.1)),
    ("dst_cumulate_fall_regions_i64", cfg_of("cumulate", 3 * 3600_000, 3600_000, vt="i64", zone=LA),
     dict(n=1_200_000, keys=150_000, batch=100_000, delay=300_000, jitter=1_200_000, t0=FALL - 1800_000,
          rate_per_ms=0.06)),
    ("dst_proctime_cumulate_fall", dict(cfg_of("cumulate", 3 * 3600_000, 3600_000, zone=LA), proctime=True),
     dict(n=300_000, keys=20_000, batch=20_000, delay=0, jitter=0, t0=FALL - 1800_000, rate_per_ms=0.02)),
]


MIN_AGGS = ("count_star", "count", "min")
MAX_AGGS = ("count_star", "count", "max")
# MIN / MAX (Min/MaxAggFunction): one operator per accumulator kind over the paths the SUM
# family takes -- small-table and two-pass partitions, compact and wide merges, NULLs, late
# records, hop/cumulate slice merges, Zipf heavy pass (wave pre-reduction by min/max),
# processing time, daylight-saving zones (DataStream: test_datastream_min_max_parity)
MINMAX_BASE = [c for c in STREAM_CASES if c[0] in (
    "tumble_f64_inorder", "tumble_i64_ooo", "tumble_i64_wrap", "tumble_f64_nulls_late", "tumble_spread_keys",
    "hop_f64", "hop_i64_late", "cumulate_f64", "cumulate_i64_late", "regions_f64_nulls_late",
    "regions_i64_ooo_lanes", "regions_hop_f64", "regions_cumulate_i64_late", "big_units_i64_nulls_ooo",
    "proctime_cumulate_i64", "zipf_tumble_f64", "zipf_tumble_i64_nulls_late", "zipf_hop_f64",
    "dst_hop_fall_i64")]
MINMAX_CASES = [(f"{m}_{name}", dict(cfg, aggs=aggs), kw) for name, cfg, kw in MINMAX_BASE
                for m, aggs in (("min", MIN_AGGS), ("max", MAX_AGGS))]


@pytest.mark.parametrize("name,cfg,kw", MINMAX_CASES, ids=[c[0] for c in MINMAX_CASES])
def test_min_max_parity(oracle_mod, name, cfg, kw):
    ks = {} if kw.get("zipf") else None
    drive_both(oracle_mod, cfg, kstats=ks, **kw)
    if ks is not None:
        assert ks.get("merge_heavy", {}).get("launches", 0) + ks.get("tile_split_fire", {}).get("launches", 0) > 0, ks


# DataStream WindowedStream.min / max (minBy / maxBy: the same value for a (key, value) tuple):
# ComparableAggregator (ComparableAggregator.java:83-104, Comparator.java:48-137); DOUBLE compares
# by Double.compareTo, so NaN / -0.0 / +0.0 / infinities are exact here (`specials`)
DS_MINMAX_BASE = [
    ("ds_tumble_i64", cfg_of("tumble", 1000, vt="i64", mode="datastream"),
     dict(n=150_000, keys=2000, batch=8_000, delay=100, jitter=700)),
    ("ds_tumble_f64_specials", cfg_of("tumble", 1000, mode="datastream"),
     dict(n=150_000, keys=2000, batch=8_000, delay=100, jitter=700, specials=0.05)),
    ("ds_sliding_f64_specials", cfg_of("hop", 3000, 1000, mode="datastream"),
     dict(n=150_000, keys=2000, batch=8_000, delay=100, jitter=1500, specials=0.05)),
    ("ds_regions_sliding_f64_specials", cfg_of("hop", 3000, 1000, mode="datastream"),
     dict(n=400_000, keys=100_000, batch=30_000, delay=100, jitter=1500, specials=0.02)),
    ("ds_zipf_tumble_f64_specials", cfg_of("tumble", 2000, mode="datastream"),
     dict(n=3_000_000, keys=100_000, batch=1_000_000, delay=0, jitter=0, rate_per_ms=1_000, zipf=1.1, specials=0.01)),
    ("ds_lateness_tumble_f64_specials", dict(cfg_of("tumble", 1000, mode="datastream"), allowed_lateness=800),
     dict(n=200_000, keys=3000, batch=10_000, delay=100, jitter=1500, specials=0.05)),
    ("ds_lateness_sliding_i64_purging", dict(cfg_of("hop", 3000, 1000, vt="i64", mode="datastream"),
                                             allowed_lateness=1500, purging=True),
     dict(n=200_000, keys=2000, batch=10_000, delay=100, jitter=4500)),
]
DS_MINMAX_CASES = [(f"{m}_{name}", dict(cfg, aggs=("count_star", m)), kw) for name, cfg, kw in DS_MINMAX_BASE
                   for m in ("min", "max")]


@pytest.mark.parametrize("name,cfg,kw", DS_MINMAX_CASES, ids=[c[0] for c in DS_MINMAX_CASES])
def test_datastream_min_max_parity(oracle_mod, name, cfg, kw):
    ks = {} if kw.get("zipf") else None
    drive_both(oracle_mod, cfg, kstats=ks, **kw)
    if ks is not None:
        assert ks.get("merge_heavy", {}).get("launches", 0) + ks.get("tile_split_fire", {}).get("launches", 0) > 0, ks


@pytest.mark.parametrize("kind", ["tumble", "hop", "cumulate"])
def test_min_max_snapshot_restore(oracle_mod, kind):
    for aggs in (MIN_AGGS, MAX_AGGS):
        cfg = dict(cfg_of(kind, 4000, 0 if kind == "tumble" else 1000, vt="i64"), aggs=aggs)
        drive_both(oracle_mod, cfg, n=120_000, keys=2000, batch=6_000, delay=100, jitter=500, snapshot_at=7,
                   null_frac=0.1)


ALL_AGGS = ("count_star", "count", "sum", "avg", "sum0", "min", "max")
# several value accumulators in one handle (value slots: SUM family, MIN, MAX): one staging
# pass feeds all of them, the row holds every aggregate as the reference's generated
# NamespaceAggsHandleFunction does (AggsHandlerCodeGenerator.scala:578-700)
MV_BASE = [c for c in STREAM_CASES if c[0] in (
    "tumble_f64_inorder", "tumble_i64_ooo", "tumble_i64_wrap", "tumble_f64_nulls_late", "hop_f64", "hop_i64_late",
    "cumulate_f64", "cumulate_i64_late", "regions_f64_nulls_late", "regions_i64_ooo_lanes", "regions_hop_f64",
    "regions_cumulate_i64_late", "big_units_i64_nulls_ooo", "proctime_hop_f64", "zipf_tumble_f64",
    "zipf_tumble_i64_nulls_late", "zipf_hop_f64", "signed_tumble_f64", "dst_cumulate_spring_f64")]
MV_CASES = [(f"mv_{name}", dict(cfg, aggs=ALL_AGGS), kw) for name, cfg, kw in MV_BASE] + [
    ("mv_avg_min_i64_ooo", dict(cfg_of("tumble", 1000, vt="i64"), aggs=("count_star", "avg", "min")),
     dict(n=200_000, keys=3000, batch=7_000, delay=300, jitter=900, null_frac=0.1)),
    ("mv_max_sum_hop_regions", dict(cfg_of("hop", 3000, 1000), aggs=("max", "count_star", "sum")),
     dict(n=600_000, keys=100_000, batch=40_000, delay=200, jitter=800, null_frac=0.1))]


@pytest.mark.parametrize("name,cfg,kw", MV_CASES, ids=[c[0] for c in MV_CASES])
def test_multi_accumulator_parity(oracle_mod, name, cfg, kw):
    ks = {} if kw.get("zipf") else None
    drive_both(oracle_mod, cfg, kstats=ks, **kw)
    if ks is not None:
        assert ks.get("merge_heavy", {}).get("launches", 0) + ks.get("tile_split_fire", {}).get("launches", 0) > 0, ks


@pytest.mark.parametrize("kind", ["tumble", "hop", "cumulate"])
def test_multi_accumulator_snapshot_restore(oracle_mod, kind):
    """The state image carries the MIN / MAX slots (fg_state_rows.min / max); late records
    after the restore re-fire old windows through the marked merges with every slot."""
    for vt in ("i64", "f64"):
        cfg = dict(cfg_of(kind, 4000, 0 if kind == "tumble" else 1000, vt=vt), aggs=ALL_AGGS)
        drive_both(oracle_mod, cfg, n=400_000, keys=100_000, batch=20_000, delay=100, jitter=1500, snapshot_at=9,
                   null_frac=0.1)


def test_multi_accumulator_grows(oracle_mod):
    """Far more keys than expected_keys: regions split with every value slot."""
    cfg = dict(cfg_of("hop", 3000, 1000, vt="i64"), aggs=ALL_AGGS)
    st = {}
    drive_both(oracle_mod, cfg, n=600_000, keys=200_000, batch=60_000, delay=100, jitter=300, expected_keys=1000,
               stats=st, null_frac=0.05)
    assert st["state_regions"] >= 8, st


@pytest.mark.parametrize("name,cfg,kw", STREAM_CASES, ids=[c[0] for c in STREAM_CASES])
def test_stream_parity(oracle_mod, name, cfg, kw):
    ks = {} if kw.get("zipf") else None
    drive_both(oracle_mod, cfg, kstats=ks, **kw)
    if ks is not None:   # the hot keys' regions did take the chunked heavy pass
        assert ks.get("merge_heavy", {}).get("launches", 0) + ks.get("tile_split_fire", {}).get("launches", 0) > 0, ks


@pytest.mark.parametrize("kind", ["tumble", "hop", "cumulate"])
def test_snapshot_restore_parity(oracle_mod, kind):
    cfg = cfg_of(kind, 4000, 0 if kind == "tumble" else 1000)
    drive_both(oracle_mod, cfg, n=120_000, keys=2000, batch=6_000, delay=100, jitter=500, snapshot_at=7)


def test_lane_conflict_slow_path(oracle_mod):
    """A batch spanning more slices than the staged lanes (filtered multi-pass ingest)."""
    cfg = cfg_of("tumble", 100)
    drive_both(oracle_mod, cfg, n=100_000, keys=500, batch=50_000, delay=0, jitter=0)


def test_lane_conflict_slow_path_two_pass(oracle_mod):
    """The same through the two-pass partition (>= 64 regions)."""
    cfg = cfg_of("tumble", 20)
    drive_both(oracle_mod, cfg, n=600_000, keys=100_000, batch=300_000, delay=0, jitter=0)


@pytest.mark.parametrize("kind", ["tumble", "hop", "cumulate"])
def test_snapshot_restore_many_regions(oracle_mod, kind):
    # jitter > watermark delay: records older than the checkpoint's watermark arrive after the
    # restore and re-fire their windows for their keys, as in the reference
    cfg = cfg_of(kind, 4000, 0 if kind == "tumble" else 1000)
    drive_both(oracle_mod, cfg, n=400_000, keys=100_000, batch=20_000, delay=100, jitter=1500, snapshot_at=9)


@pytest.mark.parametrize("mode,kind,wm1", [("sql", "tumble", 4999), ("datastream", "tumble", 4999),
                                           ("sql", "hop", 4999), ("sql", "cumulate", 4999),
                                           ("sql", "hop", 1999), ("sql", "cumulate", 1999),
                                           ("datastream", "hop", 4999), ("datastream", "hop", 1999)])
def test_restore_refires_old_windows(oracle_mod, mode, kind, wm1):
    """After initializeState the timer service restarts at Long.MIN_VALUE: rows older than the
    checkpoint's watermark are not late and fire their (already fired) window again on the next
    watermark -- HOP / CUMULATE for their keys only, chained on by nextTriggerWindow
    (SlicingWindowAggOperatorTest.java:173-184 restores mid-stream; the oracle replays the
    restored timer heap, oracle.c or_restore_copy). wm1 = 1999: the first watermark after the
    restore is below the checkpoint's, so the re-fire spans two watermarks."""
    cfg = cfg_of(kind, 1000 if kind == "tumble" else 2000, 0 if kind == "tumble" else 500, vt="i64", mode=mode)
    g = gpu_mk(cfg, expected_keys=300, buffer_records=1 << 16)
    o = oracle_mk(oracle_mod, cfg)
    rng = np.random.default_rng(7)
    k1 = rng.integers(0, 300, 5000).astype(np.int64)
    t1 = rng.integers(0, 5000, 5000).astype(np.int64)
    v1 = rng.integers(-50, 50, 5000).astype(np.int64)
    for op in (g, o):
        op.process_batch(k1, t1, v1)
        op.process_watermark(2999)
    assert_rows_equal(g.take_rows(), o.take_rows(), "i64", "before checkpoint")
    for op in (g, o):
        op.prepare_snapshot()
    g2, o2 = g.restore_copy(), o.restore_copy()
    g.close()
    o.close()
    # after the restore: rows of windows [0, 3000) that fired before the checkpoint, and newer ones
    k2 = rng.integers(0, 300, 4000).astype(np.int64)
    t2 = rng.integers(0, 7000, 4000).astype(np.int64)
    v2 = rng.integers(-50, 50, 4000).astype(np.int64)
    for op in (g2, o2):
        op.process_batch(k2, t2, v2)
        op.process_watermark(wm1)
    got, exp = g2.take_rows(), o2.take_rows()
    assert (exp["window_end"] <= 3000).any()   # the old windows did fire again
    assert_rows_equal(got, exp, "i64", "first watermark after restore")
    assert g2.late_dropped == o2.late_dropped
    k3 = rng.integers(0, 300, 3000).astype(np.int64)
    t3 = rng.integers(1000, 8000, 3000).astype(np.int64)
    v3 = rng.integers(-50, 50, 3000).astype(np.int64)
    for op in (g2, o2):
        op.process_batch(k3, t3, v3)
        op.process_watermark(5999)
    assert_rows_equal(g2.take_rows(), o2.take_rows(), "i64", "second watermark after restore")
    assert g2.late_dropped == o2.late_dropped
    for op in (g2, o2):
        op.process_watermark(JMAX)
    assert_rows_equal(g2.take_rows(), o2.take_rows(), "i64", "final")
    g2.close()
    o2.close()


def test_count_star_only_many_regions(oracle_mod):
    """COUNT(*) with no value column (8-byte staged records) vs the oracle's COUNT(*)."""
    import flink_amd as F
    n, keys = 500_000, 120_000
    key, ts, val, _ = make_stream(n, keys, "f64", jitter_ms=300)
    op = F.WindowAggOperator(F.tumbling(1000), aggs=("count_star",), val_type="none", expected_keys=keys,
                             buffer_records=1 << 18)
    o = oracle_mod.OracleOperator(kind=0, size=1000, val_type=2)
    got, exp = [], []
    for lo, hi, wm in batches_with_watermarks(n, 40_000, ts, 100):
        op.process_batch(key[lo:hi], ts[lo:hi])
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        got.append(op.process_watermark(wm))
        o.process_watermark(wm)
        exp.append(o.take_rows())
    got.append(op.process_watermark(JMAX))
    o.process_watermark(JMAX)
    exp.append(o.take_rows())
    g, e = np.concatenate(got), np.concatenate(exp)
    g = g[np.lexsort((g["key"], g["window_end"]))]
    e = e[np.lexsort((e["key"], e["window_end"]))]
    assert len(g) == len(e)
    assert np.array_equal(g["key"], e["key"]) and np.array_equal(g["window_end"], e["window_end"])
    assert np.array_equal(g["count_star"], e["cnt_star"])
    assert op.num_late_records_dropped == o.late_dropped
    op.close()


def test_empty_and_ragged_batches(oracle_mod):
    import flink_amd as F
    op = F.WindowAggOperator(F.tumbling(1000), expected_keys=100)
    op.process_batch(np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0))
    assert len(op.process_watermark(10_000)) == 0
    op.process_batch(np.array([7], np.int64), np.array([10_500], np.int64), np.array([2.5]))
    r = op.process_watermark(JMAX)
    assert len(r) == 1 and r["key"][0] == 7 and r["count_star"][0] == 1 and r["sum"][0] == 2.5
    op.close()


@pytest.mark.parametrize("kind", ["tumble", "hop", "cumulate"])
def test_regions_split_on_overflow(oracle_mod, kind):
    """An under-estimated key count no longer fails the job: a region that overflows its LDS
    table or its HBM capacity splits (BytesMap grows, BytesMap.java:229-290; the buffer flushes
    and retries, RecordsWindowBuffer.java:89-96) and its records are merged again. 400k keys
    into an operator sized for 1,000 (one region) give the oracle's rows."""
    cfg = cfg_of(kind, 1000 if kind == "tumble" else 3000, 0 if kind == "tumble" else 1000)
    st = {}
    drive_both(oracle_mod, cfg, n=800_000, keys=400_000, batch=100_000, delay=100, jitter=300, expected_keys=1000,
               stats=st)
    assert st["state_regions"] >= 32, st   # split from 1 region: ~88k distinct keys per 1-s slice


def test_regions_split_with_staged_lanes_and_restore(oracle_mod):
    """Splits while other slice lanes hold staged records (read through their parent buckets),
    a snapshot restored into a small operator (regions sized for the image), and the late
    rows that follow."""
    cfg = cfg_of("tumble", 200, vt="i64")
    drive_both(oracle_mod, cfg, n=900_000, keys=150_000, batch=60_000, delay=150, jitter=450, expected_keys=500,
               snapshot_at=6)


def test_capacity_limit_is_loud():
    """More distinct keys in one slice than 2^13 regions hold fails with FG_ECAPACITY."""
    import flink_amd as F
    op = F.WindowAggOperator(F.tumbling(1000), expected_keys=1)
    # 8,000 keys whose mix shares the top 13 bits and more: they land in one region at any split
    from tests.streams import keys_in_one_region
    keys = keys_in_one_region(8000)
    op.process_batch(keys, np.full(len(keys), 100, np.int64), np.ones(len(keys)))
    with pytest.raises(F.FlinkGpuError) as ei:
        op.process_watermark(JMAX)
    assert "regions" in str(ei.value)
    op.close()


def test_key_groups_bit_exact(oracle_mod):
    import flink_amd as F
    rng = np.random.default_rng(7)
    keys = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, 200_000, dtype=np.int64)
    keys[:4] = [0, -1, np.iinfo(np.int64).min, np.iinfo(np.int64).max]
    for maxp in (128, 256, 32768):
        got = F.key_groups(keys, maxp)
        exp = oracle_mod.key_groups_binaryrow(keys, maxp)
        assert np.array_equal(got, exp)
    got = F.key_groups(keys[:1000], 128, key_hash=1)
    L = oracle_mod.lib()
    exp = np.array([L.or_key_group(L.or_long_hash(int(k)), 128) for k in keys[:1000]])
    assert np.array_equal(got, exp)


def test_partition_by_owner():
    import torch

    from flink_amd.exchange import partition_by_owner
    n, par, maxp = 300_000, 8, 128
    key = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device="cuda")
    ts = torch.arange(n, dtype=torch.int64, device="cuda")
    val = torch.randn(n, dtype=torch.float64, device="cuda").view(torch.int64)
    ok, ot, ov, counts = partition_by_owner(key, ts, val, par, maxp)
    import flink_amd as F
    kg = F.key_groups(key.cpu().numpy(), maxp)
    owner = kg.astype(np.int64) * par // maxp
    exp_counts = np.bincount(owner, minlength=par)
    assert np.array_equal(counts.cpu().numpy(), exp_counts)
    okn, otn = ok.cpu().numpy(), ot.cpu().numpy()
    off = np.concatenate([[0], np.cumsum(exp_counts)])
    for d in range(par):
        seg = slice(off[d], off[d + 1])
        assert np.array_equal(np.sort(otn[seg]), np.sort(np.nonzero(owner == d)[0]))
        assert np.array_equal(np.sort(okn[seg]), np.sort(key.cpu().numpy()[owner == d]))


def test_conservation_large(oracle_mod):
    """Size-independent properties on a 20M-record stream: every non-dropped record is
    counted exactly once per tumbling window; SUM over all rows equals the sum of the
    accepted values (f64 within tolerance), and row counts match the oracle."""
    import flink_amd as F
    n, keys = 20_000_000, 2_000_000
    key, ts, val, _ = make_stream(n, keys, "f64", rate_per_ms=20_000, jitter_ms=30)
    op = F.WindowAggOperator(F.tumbling(100), expected_keys=keys, buffer_records=1 << 23)
    tot_cnt = 0
    tot_sum = 0.0
    rows = 0
    for lo, hi, wm in batches_with_watermarks(n, 2_000_000, ts, 20):
        op.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        r = op.process_watermark(wm)
        tot_cnt += int(r["count_star"].sum())
        tot_sum += float(r["sum"].sum())
        rows += len(r)
    r = op.process_watermark(JMAX)
    tot_cnt += int(r["count_star"].sum())
    tot_sum += float(r["sum"].sum())
    rows += len(r)
    late = op.num_late_records_dropped
    assert tot_cnt + late == n
    o = oracle_mod.OracleOperator(kind=0, size=100, val_type=2)
    exp_rows = 0
    for lo, hi, wm in batches_with_watermarks(n, 2_000_000, ts, 20):
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        o.process_watermark(wm)
        exp_rows += len(o.take_rows())
    o.process_watermark(JMAX)
    exp_rows += len(o.take_rows())
    assert rows == exp_rows and late == o.late_dropped
    accepted = float(val.sum())   # late-dropped values excluded below via the oracle's count
    assert abs(tot_sum - accepted) <= 1e-6 * accepted or late > 0
    op.close()


TWO_PHASE_CASES = [
    ("tumble_f64_regions", cfg_of("tumble", 1000), dict(n=600_000, keys=120_000, batch=60_000, delay=0, jitter=0)),
    ("tumble_i64_ooo_late", cfg_of("tumble", 300, vt="i64"), dict(n=300_000, keys=20_000, batch=20_000, delay=100, jitter=600)),
    ("hop_f64_late", cfg_of("hop", 3000, 1000), dict(n=300_000, keys=30_000, batch=20_000, delay=200, jitter=1500)),
    ("cumulate_i64_late", cfg_of("cumulate", 4000, 500, vt="i64"), dict(n=300_000, keys=30_000, batch=15_000, delay=50, jitter=2500)),
    # hot keys in the local phase: skewed regions take the heavy pass before the exchange
    ("zipf_tumble_f64", cfg_of("tumble", 1000), dict(n=6_000_000, keys=100_000, batch=3_000_000, delay=0, jitter=0,
                                                      rate_per_ms=3_000, zipf=1.1)),
    # MIN / MAX partial accumulators (LocalAggCombiner merges with Min/MaxAggFunction.merge)
    ("min_hop_f64_late", dict(cfg_of("hop", 3000, 1000), aggs=MIN_AGGS), dict(n=300_000, keys=30_000, batch=20_000,
                                                                             delay=200, jitter=1500)),
    ("max_cumulate_i64_late", dict(cfg_of("cumulate", 4000, 500, vt="i64"), aggs=MAX_AGGS),
     dict(n=300_000, keys=30_000, batch=15_000, delay=50, jitter=2500)),
    ("max_zipf_tumble_f64", dict(cfg_of("tumble", 1000), aggs=MAX_AGGS),
     dict(n=6_000_000, keys=100_000, batch=3_000_000, delay=0, jitter=0, rate_per_ms=3_000, zipf=1.1)),
    # America/Los_Angeles zone rules: partial rows carry local slice ends across the 2021
    # gap / overlap (the `sliced` assigner takes them as is)
    ("dst_hop_fall_i64", cfg_of("hop", 4 * 3600_000, 3600_000, vt="i64", zone=LA),
     dict(n=300_000, keys=2000, batch=25_000, delay=300_000, jitter=2_400_000, t0=FALL, rate_per_ms=0.02)),
    ("dst_cumulate_spring_f64", cfg_of("cumulate", 4 * 3600_000, 3600_000, zone=LA),
     dict(n=300_000, keys=2000, batch=15_000, delay=900_000, jitter=3_000_000, t0=SPRING - 3600_000,
          rate_per_ms=0.02)),
    ("dst_tumble_spring_f64", cfg_of("tumble", 3600_000, zone=LA),
     dict(n=300_000, keys=3000, batch=20_000, delay=600_000, jitter=1_800_000, t0=SPRING, rate_per_ms=0.02)),
    # several value accumulators (SUM family, MIN, MAX): the partial rows carry all three
    ("mv_hop_f64_late", dict(cfg_of("hop", 3000, 1000), aggs=ALL_AGGS), dict(n=300_000, keys=30_000, batch=20_000,
                                                                           delay=200, jitter=1500)),
    ("mv_cumulate_i64_late", dict(cfg_of("cumulate", 4000, 500, vt="i64"), aggs=ALL_AGGS),
     dict(n=300_000, keys=30_000, batch=15_000, delay=50, jitter=2500)),
    ("mv_zipf_tumble_f64", dict(cfg_of("tumble", 1000), aggs=("count_star", "avg", "min", "max")),
     dict(n=6_000_000, keys=100_000, batch=3_000_000, delay=0, jitter=0, rate_per_ms=3_000, zipf=1.1)),
]


@pytest.mark.parametrize("name", ["tumble_f64_regions", "tumble_i64_ooo_late", "hop_f64_late", "cumulate_i64_late"])
def test_two_phase_local_checkpoints(oracle_mod, name):
    """Checkpoint barriers at the local operators every other batch: each one's buffer flushes
    its partials to the output (LocalSlicingWindowAggOperator.prepareSnapshotPreBarrier ->
    WindowBuffer.flush; fg_flush_partials), so a slice's partials reach the global operators in
    several rows; the global result still equals the single-phase oracle."""
    case = {c[0]: c for c in TWO_PHASE_CASES}.get(name)
    if case is None:
        pytest.skip(f"no two-phase case {name}")
    test_two_phase_parity(oracle_mod, *case, local_ckpt=2)


@pytest.mark.parametrize("name,cfg,kw", TWO_PHASE_CASES, ids=[c[0] for c in TWO_PHASE_CASES])
def test_two_phase_parity(oracle_mod, name, cfg, kw, local_ckpt=0):
    """LocalAggCombiner -> key-group exchange -> GlobalAggCombiner: 3 source partitions with a
    local operator each, partial rows routed to 2 owners by KeyGroupRangeAssignment, global
    operators fire; the union of their rows equals the single-phase oracle over the whole
    stream (the exchange itself is tested under gloo in test_distributed.py). Late drops are
    counted per partial row in the global phase, as in the reference, so only rows compare."""
    import flink_amd as F
    from tests.gpu_adapter import window_of
    S, R, MAXP = 3, 2, 128
    n, keys, batch, delay, jitter = kw["n"], kw["keys"], kw["batch"], kw["delay"], kw["jitter"]
    key, ts, val, _ = make_stream(n, keys, cfg["val_type"], jitter_ms=jitter,
                                  **{k: kw[k] for k in ("rate_per_ms", "zipf", "t0") if k in kw})
    w = window_of(cfg)
    aggs = cfg.get("aggs", ("count_star", "count", "sum", "avg", "sum0"))
    mm = tuple(a for a in aggs if a in ("min", "max"))
    has_sum = any(a in ("sum", "avg", "sum0") for a in aggs)
    mv = len(mm) + int(has_sum) > 1   # several value accumulators: SUM, MIN, MAX travel together
    vcol = "sum" if mv or not mm else mm[0]   # the partial accumulator column
    zone = cfg.get("zone")
    local = [F.WindowAggOperator(w, aggs=aggs, val_type=cfg["val_type"], expected_keys=keys, buffer_records=1 << 18,
                                 local_partials=True, zone=zone) for _ in range(S)]
    glob = [F.WindowAggOperator(w, aggs=aggs, val_type=cfg["val_type"], expected_keys=keys // R + 1,
                                buffer_records=1 << 18, zone=zone) for _ in range(R)]
    o = oracle_mk(oracle_mod, cfg)
    src = np.arange(n) % S

    def route(rows_list):
        rows = np.concatenate(rows_list)
        if len(rows) == 0:
            return
        owner = F.key_groups(rows["key"], MAXP).astype(np.int64) * R // MAXP
        bits = lambda c: rows[c].view(np.int64) if rows[c].dtype == np.float64 else rows[c]
        sums = bits(vcol)
        for r in range(R):
            m = owner == r
            extra = (bits("min")[m], bits("max")[m]) if mv else ()
            glob[r].process_partials(rows["key"][m], rows["window_end"][m], rows["count_star"][m],
                                     rows["count"][m], sums[m], *extra)

    got, exp = [], []
    for bi, (lo, hi, wm) in enumerate(batches_with_watermarks(n, batch, ts, delay)):
        for s in range(S):
            m = src[lo:hi] == s
            local[s].process_batch(key[lo:hi][m], ts[lo:hi][m], val[lo:hi][m])
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        if local_ckpt and bi % local_ckpt == local_ckpt - 1:
            # a checkpoint barrier: each local operator's buffer flushes to the output (fg_flush_partials)
            route([local[s].prepare_snapshot_pre_barrier() for s in range(S)])
        route([local[s].process_watermark(wm) for s in range(S)])
        got += [g.process_watermark(wm) for g in glob]
        o.process_watermark(wm)
        exp.append(o.take_rows())
    route([local[s].process_watermark(JMAX) for s in range(S)])
    got += [g.process_watermark(JMAX) for g in glob]
    o.process_watermark(JMAX)
    exp.append(o.take_rows())
    g = np.concatenate([x for x in got if len(x)])
    from tests.gpu_adapter import GpuOperator
    adapter = GpuOperator.__new__(GpuOperator)
    adapter.cfg = cfg
    adapter._rows = [g]
    chk = dict(sums=True, aggs=aggs, sum0="sum0" in aggs) if mv else {}
    assert_rows_equal(adapter.take_rows(), np.concatenate(exp), cfg["val_type"], name, minmax=mm, **chk)
    for x in local + glob:
        x.close()
    o.close()


def windowed_rows(kind, size, slide, key, ts, val, isnull, zone=None):
    """A window TVF's output: every record once per window containing it (record-major),
    with the window's end as its `window_end` column (offset 0); with a zone, windows of
    the local (UTC-shifted) time toUtcTimestampMills gives (TimeWindowUtil.java:53-61)."""
    S = size if kind == "tumble" else (np.gcd(size, slide) if kind == "hop" else slide)
    if zone:
        from flink_amd.tz import zone_rules
        trans, offs, _ = zone_rules(zone)
        lt = ts + np.asarray(offs, dtype=np.int64)[np.searchsorted(np.asarray(trans, dtype=np.int64), ts, side="right")]
    else:
        lt = ts   # watermarks stay epoch times (the `ts` column below)
    se = (lt // S) * S + S
    if kind == "tumble":
        ends = [se]
    elif kind == "hop":
        ends = [se + j * S for j in range(size // S)]
    else:
        ws = (lt // size) * size
        ends = [np.where(se + j * S <= ws + size, se + j * S, -1) for j in range(size // S)]
    E = np.stack(ends, axis=1)
    rep = (E >= 0).sum(axis=1)
    keep = (E >= 0).ravel()
    out = dict(key=np.repeat(key, rep), wend=E.ravel()[keep], val=np.repeat(val, rep), ts=np.repeat(ts, rep))
    out["isnull"] = None if isnull is None else np.repeat(isnull, rep)
    return out


WINDOWED_CASES = [
    ("windowed_tumble_f64", cfg_of("tumble", 1000), dict(n=200_000, keys=3000, batch=10_000, delay=300, jitter=900)),
    ("windowed_hop_i64", cfg_of("hop", 3000, 1000, vt="i64"), dict(n=150_000, keys=2000, batch=12_000, delay=200, jitter=1500)),
    ("windowed_cumulate_f64_nulls", cfg_of("cumulate", 4000, 1000), dict(n=150_000, keys=2000, batch=9_000, delay=100,
                                                                        jitter=2500, null_frac=0.1)),
    ("windowed_hop_regions_f64", cfg_of("hop", 4000, 1000), dict(n=600_000, keys=100_000, batch=60_000, delay=200,
                                                                 jitter=800)),
    # zone rules: local window ends across the 2021 LA gap (spring) and overlap (fall)
    ("windowed_dst_tumble_spring_f64", cfg_of("tumble", 3600_000, zone=LA),
     dict(n=200_000, keys=2000, batch=10_000, delay=600_000, jitter=1_800_000, t0=SPRING, rate_per_ms=0.02)),
    ("windowed_dst_hop_fall_i64", cfg_of("hop", 4 * 3600_000, 3600_000, vt="i64", zone=LA),
     dict(n=150_000, keys=2000, batch=12_000, delay=300_000, jitter=2_400_000, t0=FALL, rate_per_ms=0.02)),
    ("windowed_dst_cumulate_fall_f64", cfg_of("cumulate", 3 * 3600_000, 3600_000, zone=LA),
     dict(n=150_000, keys=2000, batch=9_000, delay=900_000, jitter=3_000_000, t0=FALL - 1800_000, rate_per_ms=0.02,
          null_frac=0.1)),
]


@pytest.mark.parametrize("name,cfg,kw", WINDOWED_CASES, ids=[c[0] for c in WINDOWED_CASES])
def test_windowed_input_parity(oracle_mod, name, cfg, kw):
    """WindowedSliceAssigner (SliceAssigners.java:386-435): rows carrying their window_end;
    late rows of fired windows dropped; window_start from the inner assigner."""
    cfg = dict(cfg, windowed=True, count_star_index=-1 if cfg["kind"] == "hop" else 0)
    key, ts, val, isnull = make_stream(kw["n"], kw["keys"], cfg["val_type"], jitter_ms=kw["jitter"],
                                       null_frac=kw.get("null_frac", 0.0),
                                       **{k: kw[k] for k in ("rate_per_ms", "t0") if k in kw})
    r = windowed_rows(cfg["kind"], cfg["size"], cfg["slide"], key, ts, val, isnull, zone=cfg.get("zone"))
    g = gpu_mk(cfg, expected_keys=kw["keys"], buffer_records=max(4 * kw["batch"], 1 << 16))
    o = oracle_mk(oracle_mod, cfg)
    n = len(r["key"])
    mx = np.iinfo(np.int64).min
    for step, lo in enumerate(range(0, n, kw["batch"])):
        hi = min(n, lo + kw["batch"])
        nl = None if r["isnull"] is None else r["isnull"][lo:hi]
        for op in (g, o):
            op.process_batch(r["key"][lo:hi], r["wend"][lo:hi], r["val"][lo:hi], nl)
        mx = max(mx, int(r["ts"][lo:hi].max()))
        g.process_watermark(mx - kw["delay"] - 1)
        o.process_watermark(mx - kw["delay"] - 1)
        assert_rows_equal(g.take_rows(), o.take_rows(), cfg["val_type"], f"{name} step {step}")
        assert g.late_dropped == o.late_dropped, f"late drops differ at step {step}"
    g.process_watermark(JMAX)
    o.process_watermark(JMAX)
    assert_rows_equal(g.take_rows(), o.take_rows(), cfg["val_type"], f"{name} final")
    assert o.late_dropped > 0   # the jitter makes late rows of fired windows
    g.close()
    o.close()


def test_windowed_input_off_grid_is_loud():
    """A window_end off the window's slice grid is rejected, never silently re-sliced."""
    import flink_amd as F
    op = F.WindowAggOperator(F.tumbling(1000), windowed=True, expected_keys=100)
    with pytest.raises(F.WindowSpecError, match="off the slice grid"):
        op.process_batch(np.arange(4, dtype=np.int64), np.array([1000, 2000, 2500, 3000], dtype=np.int64),
                         np.ones(4))
    op.close()


@pytest.mark.parametrize("kind,vt,device_output", [("tumble", "f64", False), ("hop", "i64", False),
                                                   ("cumulate", "f64", True)])
def test_composite_sum_min_max(oracle_mod, kind, vt, device_output):
    """COUNT(*), COUNT, SUM, AVG, MIN, MAX of one column: one handle per accumulator kind,
    rows joined on (window_end, key) (flink_amd/composite.py) vs the oracle's one row."""
    import flink_amd as F
    from tests.gpu_adapter import window_of
    cfg = cfg_of(kind, 4000, 0 if kind == "tumble" else 1000, vt=vt)
    key, ts, val, isnull = make_stream(150_000, 3000, vt, jitter_ms=900, null_frac=0.1)
    aggs = ("count_star", "count", "sum", "avg", "min", "max")
    op = F.CompositeWindowAggOperator(window_of(cfg), aggs=aggs, val_type=vt, expected_keys=3000)
    assert len(op.ops) == 3
    o = oracle_mk(oracle_mod, cfg)
    sfx = "_i" if vt == "i64" else "_d"

    def check(got, exp, ctx):
        if device_output:
            got = {k: v.cpu().numpy() for k, v in got.items()}
        e = sort_rows(exp)
        assert len(got["key"]) == len(e), ctx
        for f, ef in (("key", "key"), ("window_start", "window_start"), ("window_end", "window_end"),
                      ("count_star", "cnt_star"), ("count", "cnt_val")):
            assert np.array_equal(got[f], e[ef]), (ctx, f)
        ok = e["sum_null"] == 0
        assert np.array_equal(got["sum_null"], ~ok) and np.array_equal(got["min_null"], ~ok), ctx
        for f in ("min", "max"):
            assert np.array_equal(got[f][ok], e[f + sfx][ok]), (ctx, f)
        for f in ("sum", "avg"):
            a, b = got[f][ok], e[f + sfx][ok]
            if vt == "i64":
                assert np.array_equal(a, b), (ctx, f)
            else:
                assert (np.abs(a - b) <= REL_TOL * np.maximum(np.abs(a), np.abs(b)) + 1e-300).all(), (ctx, f)

    for step, (lo, hi, wm) in enumerate(batches_with_watermarks(len(key), 9_000, ts, 300)):
        op.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi], isnull[lo:hi])
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi], isnull[lo:hi])
        got = op.process_watermark(wm, device_output=device_output)
        o.process_watermark(wm)
        check(got, o.take_rows(), f"step {step}")
    got = op.process_watermark(JMAX, device_output=device_output)
    o.process_watermark(JMAX)
    check(got, o.take_rows(), "final")
    assert op.num_late_records_dropped == o.late_dropped
    op.close()
    o.close()


def test_batch_limits_are_loud_and_recoverable(oracle_mod):
    """fg_add_batch rejects a batch over 2^31-1 records and missing columns with FG_EINVAL
    before touching any buffer; the operator keeps working afterwards."""
    import ctypes as C
    import flink_amd as F
    from flink_amd import _lib as L
    op = F.WindowAggOperator(F.tumbling(1000), aggs=("count_star", "sum"), val_type="i64", expected_keys=100)
    lib = L.load()
    b = L.FgBatch()
    b.location = L.DEVICE
    b.n = 1 << 31
    b.key, b.rowtime, b.val = 8, 8, 8    # never dereferenced: the size check comes first
    assert lib.fg_add_batch(op._h, C.byref(b)) == L.FG_EINVAL
    assert b"2^31" in lib.fg_last_error(op._h)
    b.n = 10
    b.key = 0
    assert lib.fg_add_batch(op._h, C.byref(b)) == L.FG_EINVAL
    key = np.arange(10, dtype=np.int64) % 3
    ts = np.full(10, 1_000_500, dtype=np.int64)
    op.process_batch(key, ts, np.arange(10, dtype=np.int64))
    r = op.process_watermark(JMAX)
    r = r[np.argsort(r["key"])]
    assert list(r["count_star"]) == [4, 3, 3] and list(r["sum"]) == [18, 12, 15]
    op.close()


def test_unknown_key_count_starts_small_and_grows(oracle_mod):
    """expected_keys = 0 (no key-count hint from the shim): 2^10 regions (117 MB per slice
    table instead of the largest table's 940 MB), split on demand: ~5.7M distinct keys in one
    slice grow it to 2^11."""
    cfg = cfg_of("tumble", 1000)
    st = {}
    drive_both(oracle_mod, cfg, n=10_000_000, keys=8_000_000, batch=2_500_000, delay=0, jitter=0, expected_keys=0,
               rate_per_ms=10_000, stats=st)
    assert st["state_regions"] >= 2048, st


@pytest.mark.parametrize("kind,outliers", [("tumble", "future"), ("tumble", "epoch0"), ("hop", "both"),
                                           ("cumulate", "future")])
def test_outlier_slices_cost_no_empty_passes(oracle_mod, kind, outliers):
    """A batch holding a record a day ahead (or at rowtime 0) spans ~86,400 (or ~1.6e9) empty
    1-s slices: the filtered ingest passes jump from occupied slice to occupied slice
    (each pass reports the next one), so the batch stages in a few passes and the rows and
    late drops still match the oracle. Watermarks follow the regular records (the outliers
    are held back by the source's watermark strategy)."""
    import time
    cfg = cfg_of(kind, 1000 if kind == "tumble" else 4000, 0 if kind == "tumble" else 1000)
    n, keys, batch = 200_000, 3000, 20_000
    key, ts, val, _ = make_stream(n, keys, "f64", jitter_ms=400)
    ts = ts.copy()
    if outliers in ("future", "both"):
        ts[5] = ts[5] + 86_400_000          # a day ahead
        ts[n // 2 + 7] = ts[n // 2 + 7] + 3 * 86_400_000
    if outliers in ("epoch0", "both"):
        ts[11] = 0                          # Long 0: an ancient record, before the first watermark
    g = gpu_mk(cfg, expected_keys=keys, buffer_records=1 << 17)
    o = oracle_mk(oracle_mod, cfg)
    regular = np.ones(n, dtype=bool)
    regular[[5, 11, n // 2 + 7]] = False
    mx = np.iinfo(np.int64).min
    t0 = time.time()
    for lo in range(0, n, batch):
        hi = min(n, lo + batch)
        g.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        mx = max(mx, int(ts[lo:hi][regular[lo:hi]].max()))
        g.process_watermark(mx - 300 - 1)
        o.process_watermark(mx - 300 - 1)
        assert_rows_equal(g.take_rows(), o.take_rows(), "f64", f"{kind} batch {lo}")
        assert g.late_dropped == o.late_dropped
    g.process_watermark(JMAX)
    o.process_watermark(JMAX)
    assert_rows_equal(g.take_rows(), o.take_rows(), "f64", "final")
    assert time.time() - t0 < 60, "empty slice stretches were walked pass by pass"
    g.close()
    o.close()


@pytest.mark.parametrize("case", ["tumble_f64_nulls", "hop_i64_padded", "cumulate_f64_device"])
def test_binary_rows_parity(oracle_mod, case):
    """fg_add_rows: the stream handed over as packed BinaryRowData rows (flink_amd.rows.pack_rows,
    BinaryRowData.java:68-76) gives the oracle's rows -- NULL values through the null bits, wider
    rows with the fields at other positions and padding, host and device rows."""
    import torch

    import flink_amd as F
    from flink_amd.rows import pack_rows
    kind, vt = {"tumble_f64_nulls": ("tumble", "f64"), "hop_i64_padded": ("hop", "i64"),
                "cumulate_f64_device": ("cumulate", "f64")}[case]
    cfg = cfg_of(kind, 1000 if kind == "tumble" else 3000, 0 if kind == "tumble" else 1000, vt=vt)
    n, keys, batch = 200_000, 20_000, 20_000
    key, ts, val, isnull = make_stream(n, keys, vt, jitter_ms=800, null_frac=0.15)
    g = gpu_mk(cfg, expected_keys=keys, buffer_records=1 << 18)
    o = oracle_mk(oracle_mod, cfg)
    for lo, hi, wm in batches_with_watermarks(n, batch, ts, 100):
        k, t, v, nl = key[lo:hi], ts[lo:hi], val[lo:hi], isnull[lo:hi]
        if case == "hop_i64_padded":   # (pad, value, pad, rowtime, key) + 16 bytes of padding
            z = np.zeros(hi - lo, dtype=np.int64)
            rows = pack_rows([z, v, z, t, k], [None, nl, None, None, None], stride=72)
            g.op.process_rows(rows, 72, 5, key_field=4, rowtime_field=3, val_field=1)
        else:
            rows = pack_rows([k, t, v], [None, None, nl])
            if case == "cumulate_f64_device":
                rows = torch.from_numpy(rows).cuda()
            g.op.process_rows(rows, 32, 3)
        o.process_batch(k, t, v, nl)
        g.process_watermark(wm)
        o.process_watermark(wm)
        assert_rows_equal(g.take_rows(), o.take_rows(), vt, f"wm {wm}")
        assert g.late_dropped == o.late_dropped
    g.process_watermark(JMAX)
    o.process_watermark(JMAX)
    assert_rows_equal(g.take_rows(), o.take_rows(), vt, "final")
    # a NULL key is refused before any record is staged
    bad = pack_rows([key[:10], ts[:10], val[:10]], [np.arange(10) == 3, None, None])
    with pytest.raises(F.WindowSpecError):
        g.op.process_rows(bad, 32, 3)
    g.close()
    o.close()


# DataStream allowed lateness (WindowOperator.java:608-681, EventTimeTrigger.java:37-51): the
# jitter exceeds the watermark delay, so elements reach windows that fired already; those within
# the lateness re-fire their window at once (with the whole state, or -- PurgingTrigger -- alone),
# the rest are dropped; fired windows keep their state until maxTimestamp + lateness.
LATENESS_CASES = [
    ("tumble_i64_l500", dict(cfg_of("tumble", 1000, vt="i64", mode="datastream"), allowed_lateness=500),
     dict(n=200_000, keys=3000, batch=10_000, delay=100, jitter=1500)),
    ("tumble_f64_l800", dict(cfg_of("tumble", 1000, mode="datastream"), allowed_lateness=800),
     dict(n=200_000, keys=3000, batch=10_000, delay=100, jitter=1500)),
    ("tumble_i64_l500_purging", dict(cfg_of("tumble", 1000, vt="i64", mode="datastream"), allowed_lateness=500,
                                     purging=True), dict(n=200_000, keys=3000, batch=10_000, delay=100, jitter=1500)),
    ("sliding_i64_l700", dict(cfg_of("hop", 3000, 1000, vt="i64", mode="datastream"), allowed_lateness=700),
     dict(n=200_000, keys=2000, batch=10_000, delay=100, jitter=3500)),   # drops need > 2,000 + 700
    ("sliding_f64_l1500_purging", dict(cfg_of("hop", 3000, 1000, mode="datastream"), allowed_lateness=1500,
                                       purging=True), dict(n=200_000, keys=2000, batch=10_000, delay=100, jitter=4500)),
    # hot keys: many late elements of one key in one batch (several rounds of the late path)
    ("tumble_i64_l600_zipf", dict(cfg_of("tumble", 1000, vt="i64", mode="datastream"), allowed_lateness=600),
     dict(n=200_000, keys=5000, batch=20_000, delay=50, jitter=1200, zipf=1.3)),
    # regions split while late elements append new keys (an operator sized for 100 keys)
    ("tumble_i64_l500_split", dict(cfg_of("tumble", 1000, vt="i64", mode="datastream"), allowed_lateness=500),
     dict(n=300_000, keys=60_000, batch=30_000, delay=100, jitter=1500, expected_keys=100)),
]


@pytest.mark.parametrize("name,cfg,kw", LATENESS_CASES, ids=[c[0] for c in LATENESS_CASES])
def test_datastream_allowed_lateness_parity(oracle_mod, name, cfg, kw):
    kw = dict(kw)
    ek = kw.pop("expected_keys", None)
    late = drive_both(oracle_mod, cfg, kw.pop("n"), kw.pop("keys"), kw.pop("batch"), kw.pop("delay"), kw.pop("jitter"),
                      expected_keys=ek, **kw)
    assert late > 0, "the stream should drop some elements beyond the lateness"


def test_datastream_lateness_wide_late_keys(oracle_mod):
    """Late-allowed elements enter the resident slice tables without pass 1's 32-bit key check
    (late_split): a late element whose key is k + 2^33 -- the same int32 as the staged key k --
    must not meet k in a sliding window's fire over those tables (the narrow LDS table keys
    entries by the int32 of their mix). Only late elements carry such keys."""
    cfg = dict(cfg_of("hop", 3000, 1000, vt="i64", mode="datastream"), allowed_lateness=1500)
    n, keys, batch, delay = 200_000, 2000, 10_000, 100
    key, ts, val, _ = make_stream(n, keys, "i64", jitter_ms=2500)
    prev = np.iinfo(np.int64).min
    for lo, hi, wm in batches_with_watermarks(n, batch, ts, delay):
        first_end = (ts[lo:hi] // 1000) * 1000 + 1000   # earliest window of the element
        late = np.nonzero(first_end - 1 <= prev)[0] + lo
        key[late[::2]] += 1 << 33
        prev = wm
    g = gpu_mk(cfg, expected_keys=keys, buffer_records=1 << 18)
    o = oracle_mk(oracle_mod, cfg)
    for step, (lo, hi, wm) in enumerate(batches_with_watermarks(n, batch, ts, delay)):
        g.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        g.process_watermark(wm)
        o.process_watermark(wm)
        assert_rows_equal(g.take_rows(), o.take_rows(), "i64", f"step {step}")
        assert g.late_dropped == o.late_dropped
    g.process_watermark(JMAX)
    o.process_watermark(JMAX)
    assert_rows_equal(g.take_rows(), o.take_rows(), "i64", "final")
    assert (key > (1 << 32)).any()
    g.close()
    o.close()


@pytest.mark.parametrize("kind", ["tumble", "hop"])
def test_narrow_staging_switches_to_wide_keys(oracle_mod, kind):
    """Narrow 12-B staging (keys within 32 bits, two-pass partition): batches of small keys are
    staged narrow; the first batch holding a key beyond 32 bits flushes the narrow lanes into
    their tables and the operator stages 16-B records from then on. Rows equal the oracle's
    throughout (incl. Long.MIN_VALUE and negative 32-bit keys)."""
    n, keys, batch = 1_200_000, 200_000, 100_000
    cfg = cfg_of(kind, 1000 if kind == "tumble" else 3000, 0 if kind == "tumble" else 1000)
    key, ts, val, _ = make_stream(n, keys, "f64", jitter_ms=800)
    key = key - keys // 2                                    # negative 32-bit keys too
    big = np.arange(n) >= n * 6 // 10                         # from 60 %: some keys beyond 32 bits
    wide = big & (np.arange(n) % 7 == 0)
    key[wide] = key[wide] * (1 << 33) + 12345
    key[np.nonzero(wide)[0][:3]] = np.iinfo(np.int64).min
    g = gpu_mk(cfg, expected_keys=keys, buffer_records=1 << 20)
    o = oracle_mk(oracle_mod, cfg)
    for step, (lo, hi, wm) in enumerate(batches_with_watermarks(n, batch, ts, 300)):
        g.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        g.process_watermark(wm)
        o.process_watermark(wm)
        assert_rows_equal(g.take_rows(), o.take_rows(), "f64", f"step {step}")
        assert g.late_dropped == o.late_dropped
    g.process_watermark(JMAX)
    o.process_watermark(JMAX)
    assert_rows_equal(g.take_rows(), o.take_rows(), "f64", "final")
    g.close()
    o.close()


# Tile staging (fg_kernels.h): TUMBLE batches of 32-bit keys stay in their pass-1 tiles, sorted by
# consumer bucket (4 state regions), and the window fires straight from them (k_tile_fire). The
# cases below take its other paths: the LDS table of a bucket overflowing (regions split, one
# region per retried item), and lanes whose tile passes must be materialized into regular staged
# passes (a batch with NULL values in the same slice; a checkpoint while tile passes are staged).
def test_tile_fire_bucket_overflow_splits(oracle_mod):
    """~1.3M distinct keys in one 30-s window of an operator sized for 60k keys (2^8 regions, 64
    buckets of ~20k keys against the 8,192-slot table): every bucket overflows, the regions split
    and each region is fired again on its own from the same six tile passes."""
    cfg = cfg_of("tumble", 30_000)
    st = {}
    drive_both(oracle_mod, cfg, n=3_000_000, keys=1_500_000, batch=500_000, delay=0, jitter=0, expected_keys=60_000,
               stats=st)
    assert st["state_regions"] >= 512, st


@pytest.mark.parametrize("vt", ["f64", "i64"])
def test_tile_passes_materialized(oracle_mod, vt):
    """A slice lane holding tile passes and a batch with NULL values (staged by pass 2): the tile
    passes are materialized and the lane merged as any staged lane; then a checkpoint while tile
    passes are staged (flushed into the slice table through the same conversion), a restore, and
    more batches. Rows and late drops equal the oracle's throughout."""
    cfg = cfg_of("tumble", 10_000, vt=vt)
    n, keys, batch = 1_200_000, 50_000, 100_000
    key, ts, val, isnull = make_stream(n, keys, vt, null_frac=0.05)
    g = gpu_mk(cfg, expected_keys=keys, buffer_records=1 << 21)
    o = oracle_mk(oracle_mod, cfg)
    o_base = 0
    for step, (lo, hi, wm) in enumerate(batches_with_watermarks(n, batch, ts, 200)):
        nl = isnull[lo:hi] if step in (2, 7) else None   # two batches with NULL values, the rest tile-staged
        g.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi], nl)
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi], nl)
        g.process_watermark(wm)
        o.process_watermark(wm)
        assert_rows_equal(g.take_rows(), o.take_rows(), vt, f"step {step}")
        assert g.late_dropped == o_base + o.late_dropped
        if step == 4:   # checkpoint with tile passes staged, failover, restore
            g.prepare_snapshot()
            o.prepare_snapshot()
            g2, o2 = g.restore_copy(), o.restore_copy()
            o_base += o.late_dropped
            g.close()
            o.close()
            g, o = g2, o2
    g.process_watermark(JMAX)
    o.process_watermark(JMAX)
    assert_rows_equal(g.take_rows(), o.take_rows(), vt, "final")
    g.close()
    o.close()


# ---- sparse regions ------------------------------------------------------------------------
# An operator whose regions far outnumber its keys (an expected-keys hint far too high, early
# slices, slices after a split) leaves most regions empty, so a merge workgroup walks runs of
# empty regions. Round 4 found the merge's staged-record cursor inserting a stale chunk in place
# of the first chunk of a region that followed an empty one (rows lost, rows with foreign keys):
# every case below failed at 2^10-2^12 regions before the fix (`settle` cold load, fg_kernels.hip).
SPARSE_CASES = (
    [("golden_" + c["name"], "golden", c) for c in OP_CASES
     if any(k in c["name"] for k in ("hop", "cumulate", "sliding", "cleanup"))]
    + [(n, "mv", (n, c, k)) for n, c, k in MV_CASES if "regions" in n]
    + [(n, "stream", (n, c, k)) for n, c, k in STREAM_CASES if n in ("regions_ds_sliding", "zipf_hop_f64")]
    + [(n, "two_phase", (n, c, k)) for n, c, k in TWO_PHASE_CASES if n.startswith("mv_")]
    + [(n, "lateness", (n, c, k)) for n, c, k in LATENESS_CASES if "zipf" in n]
    + [("restore_" + k, "restore", k) for k in ("tumble", "hop", "cumulate")])


@pytest.mark.parametrize("bits", [10, 12])
@pytest.mark.parametrize("name,kind,case", SPARSE_CASES, ids=[c[0] for c in SPARSE_CASES])
def test_sparse_regions_parity(oracle_mod, monkeypatch, bits, name, kind, case):
    """the same cases with 2^bits regions forced (FG_MIN_REGION_BITS, read at fg_open)"""
    monkeypatch.setenv("FG_MIN_REGION_BITS", str(bits))
    if kind == "golden":
        test_golden_cases_on_gpu(case)
    elif kind == "mv":
        test_multi_accumulator_parity(oracle_mod, *case)
    elif kind == "stream":
        test_stream_parity(oracle_mod, *case)
    elif kind == "two_phase":
        test_two_phase_parity(oracle_mod, *case)
    elif kind == "lateness":
        test_datastream_allowed_lateness_parity(oracle_mod, *case)
    else:
        test_snapshot_restore_many_regions(oracle_mod, case)


def test_tile_batches_with_a_short_last_segment(oracle_mod):
    """Tile staging with a pass-1 workgroup holding fewer tiles than the others: a batch of
    256 x 18,434 records (every workgroup 4 tiles, the last tile of each 2 records), then one of
    100 records fewer (the last workgroup 3 tiles). The missing tile's directory row must read as
    empty, not as the previous batch's row -- whose fragment would re-count the previous batch's
    last records (still in the reused tile buffer) into this batch's window. The batches fill
    windows 0 and 4: the same slice lane of 4, so the stale row's columns are the lane's own."""
    cfg = cfg_of("tumble", 1000)
    rng = np.random.default_rng(77)
    g = gpu_mk(cfg, expected_keys=100_000, buffer_records=1 << 23)
    o = oracle_mk(oracle_mod, cfg)
    for b, n in enumerate((256 * 18_434, 256 * 18_434 - 100)):
        key = rng.integers(0, 100_000, n).astype(np.int64)
        w0 = 4000 * b
        ts = (w0 + np.sort(rng.integers(0, 1000, n))).astype(np.int64)
        val = rng.random(n) * 100.0
        g.process_batch(key, ts, val)
        o.process_batch(key, ts, val)
        g.process_watermark(w0 + 999)
        o.process_watermark(w0 + 999)
        assert_rows_equal(g.take_rows(), o.take_rows(), "f64", f"batch {b} ({n} records)")
    g.close()
    o.close()
