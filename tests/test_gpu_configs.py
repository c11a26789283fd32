"""Parity at the BASELINE configurations' own key spaces (BASELINE.json configs[0..4]).

Each test generates the bench's synthetic stream for one config on the GPU (bench.gen_columns:
counter-based splitmix64, the same records `python bench.py --workload ...` times), feeds it
through the HIP engine in the bench's micro-batches and watermark cadence, and compares EVERY
fired row with the oracle (the C restatement of the reference operator) run over the same
records on the host cores, one operator instance per key-group range
(oracle.run_partitioned_rows; KeyGroupStreamPartitioner routing, maxParallelism 128).

Tolerance (north_star): keys, windows, COUNT(*), COUNT bit-exact, late drops equal, DOUBLE
SUM / AVG within 1e-9 relative (the GPU sums a (key, window) in another order than
AggCombiner's arrival order).

Each of configs[1..4] runs twice: with synchronous watermarks (host rows) and with the path the
bench times -- asynchronous watermarks held until the next micro-batch has been handed over, their
rows collected then (bench.one_step); rows returned equal the engine's rows_fired either way.

Sizes: configs[1] 200M records = 2 windows x 10M uniform keys; configs[2] 200M records = 6
event-minutes of HOP 5min/1min over 10M keys; configs[3] 70M records = 4+ steps of a
CUMULATE 1h/1min window over the 12.5M-key per-GPU share of 100M; configs[4] 300M records
of Zipf(1.1) keys with 2 s jitter, a bounded-out-of-orderness watermark and a checkpoint ->
failover -> restore mid-stream; configs[0] the whole 10M-record DataStream job.
"""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL_TOL = 1e-9
JMAX = (1 << 63) - 1
ORACLE_THREADS = int(os.environ.get("ORACLE_THREADS", "16"))


def _bench():
    import bench
    return bench


def log(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)   # progress (long cases; run with -s)


def gpu_rows_run(op, key, ts, val, n, batch, rate, wm_every, delay, jitter, snapshot_after_batch=None,
                 reopen=None, final_wm=JMAX, async_wm=False):
    """Drive the engine like bench.one_step; returns (rows, late drops, oracle watermark schedule,
    index of the snapshot watermark or -1).

    async_wm: the bench's (and a shim's) watermark path -- process_watermark(wm, device_output=True,
    wait=False) for every watermark of a batch, held until the NEXT batch has been handed over, then
    collect_fired() (bench.one_step); else the synchronous advance with host rows."""
    B = _bench()
    parts = []
    wm_at, wm_val = [], []
    snap_idx = -1
    late_base = 0
    held = False
    fired = 0   # rows returned, against the engine's own rows_fired

    def collect():
        r = op.collect_fired()
        parts.append(op.rows_to_host(r))
        return r.n
    for bi, lo in enumerate(range(0, n, batch)):
        hi = min(n, lo + batch)
        op.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        if held:   # the previous batch's watermarks: their rows now (fires completed behind this pass 1)
            fired += collect()
            held = False
        for wm in B.watermarks_for(lo, hi, rate, wm_every, delay, jitter):
            if async_wm:
                assert op.process_watermark(wm, device_output=True, wait=False) is None
                held = True
            else:
                parts.append(op.process_watermark(wm))
                fired += len(parts[-1])
            wm_at.append(hi)
            wm_val.append(wm)
        if snapshot_after_batch is not None and bi == snapshot_after_batch:
            if held:   # the rows go out before the checkpoint barrier
                fired += collect()
                held = False
            assert op.stats()["rows_fired"] == fired
            # prepareSnapshotPreBarrier + snapshotState, then a failover: a new operator
            # restored from the image (initializeState)
            op.prepare_snapshot_pre_barrier()
            img, twm = op.snapshot_state()
            late_base += op.num_late_records_dropped
            op.close()
            op = reopen()
            op.restore_state(img, twm)
            snap_idx = len(wm_at) - 1
            fired = 0
    if held:
        fired += collect()
    parts.append(op.process_watermark(final_wm))
    fired += len(parts[-1])
    wm_at.append(n)
    wm_val.append(final_wm)
    late = late_base + op.num_late_records_dropped
    assert op.stats()["rows_fired"] == fired, "rows returned vs the engine's rows_fired"
    op.close()
    parts = [p for p in parts if len(p)]
    rows = np.concatenate(parts) if parts else None
    return rows, late, np.array(wm_at, dtype=np.int64), np.array(wm_val, dtype=np.int64), snap_idx


def compare_rows(g, e, S, ctx, aggs):
    """Every row: sorted by (window_end, key) through one int64 sort key (keys < 2^32)."""
    assert len(g) == len(e), f"{ctx}: {len(g)} rows vs {len(e)} from the oracle"
    if len(g) == 0:
        return
    we0 = int(e["window_end"].min())
    assert int(g["key"].min()) >= 0 and int(g["key"].max()) < (1 << 32)
    sg = np.argsort(((g["window_end"] - we0) // S << 32) | g["key"], kind="stable")
    se = np.argsort(((e["window_end"] - we0) // S << 32) | e["key"], kind="stable")
    for gf, ef in (("key", "key"), ("window_start", "window_start"), ("window_end", "window_end"),
                   ("count_star", "cnt_star")):
        a, b = g[gf][sg], e[ef][se]
        bad = np.nonzero(a != b)[0]
        assert len(bad) == 0, f"{ctx}: {gf} differs at {bad[:5]}: {a[bad[:5]]} vs {b[bad[:5]]}"
    if "count" in aggs:
        assert np.array_equal(g["count"][sg], e["cnt_val"][se]), f"{ctx}: COUNT differs"
    for f, ef, nf in (("sum", "sum_d", "sum_null"), ("avg", "avg_d", "avg_null")):
        if f not in aggs:
            continue
        assert np.array_equal(g[f + "_null"][sg], e[nf][se] != 0), f"{ctx}: {f} NULLs differ"
        ok = e[nf][se] == 0
        a, b = g[f][sg][ok], e[ef][se][ok]
        err = np.abs(a - b) <= REL_TOL * np.maximum(np.abs(a), np.abs(b)) + 1e-300
        assert err.all(), f"{ctx}: {f} beyond 1e-9 relative: {a[~err][:5]} vs {b[~err][:5]}"


def run_config(workload, n, aggs, oracle_kind, size, slide, snapshot_after_batch=None, keys=None,
               final_wm_after=None, async_wm=False, batch=None):
    """final_wm_after: end with the watermark `final_wm_after` ms past the last regular one
    instead of Long.MAX_VALUE (CUMULATE: MAX_VALUE would fire every remaining step window of
    the hour for every key -- 60 x 12.5M rows)."""
    import torch

    import flink_amd as F
    from oracle import oracle as O
    B = _bench()
    wl = B.WORKLOADS[workload]
    keys = keys or wl["keys"]
    rate, batch = wl["rate"], batch or wl.get("batch", 50_000_000)
    wm_every = wl.get("wm_every", 1_000_000)
    dev = torch.device("cuda", 0)
    key, ts, val = B.gen_columns(n, keys, rate, 0, dev, jitter=wl["jitter"], zipf=wl["zipf"])
    datastream = wl.get("mode") == "datastream"
    if datastream:
        val = val.to(torch.int64)
    torch.cuda.synchronize()
    wname, *wargs = wl["window"]
    window = getattr(F, wname)(*wargs)
    if wl["zipf"] > 0:   # the bench's sizing hint: distinct keys in one slice's records, +10 %
        expected = int(1.1 * B.zipf_distinct_per_slice(keys, wl["zipf"], rate)) + 1
    else:
        expected = int(keys * 1.05) + 1

    def mk():
        return F.WindowAggOperator(window, aggs=aggs, val_type="i64" if datastream else "f64",
                                   mode="datastream" if datastream else "sql", expected_keys=expected,
                                   buffer_records=max(4 * batch, 1 << 26))
    final_wm = JMAX
    if final_wm_after is not None:
        final_wm = B.watermarks_for(0, n, rate, wm_every, wl["delay"], wl["jitter"])[-1] + final_wm_after
    log(f"{workload}: {n:,} records generated; GPU run ({'async' if async_wm else 'sync'} watermarks)")
    rows, late, wm_at, wm_val, snap = gpu_rows_run(mk(), key, ts, val, n, batch, rate, wm_every, wl["delay"],
                                                   wl["jitter"], snapshot_after_batch, reopen=mk, final_wm=final_wm,
                                                   async_wm=async_wm)
    log(f"{workload}: GPU fired {0 if rows is None else len(rows):,} rows; oracle run")
    kh, th, vh = key.cpu().numpy(), ts.cpu().numpy(), val.cpu().numpy()
    del key, ts, val
    torch.cuda.empty_cache()
    cfg = O.Config(O.MODE_DATASTREAM if datastream else O.MODE_SQL, oracle_kind, size, slide, 0, 0,
                   O.VAL_I64 if datastream else O.VAL_F64, 0)
    exp, olate, _ = O.run_partitioned_rows(cfg, ORACLE_THREADS, 128, kh, th, vh, wm_at, wm_val, snapshot_after=snap)
    log(f"{workload}: oracle fired {len(exp):,} rows; comparing")
    assert rows is not None and len(rows) > 0
    ctx = f"{workload} n={n}"
    if datastream:
        assert len(rows) == len(exp), f"{ctx}: rows"
        sg = np.lexsort((rows["key"], rows["window_end"]))
        se = np.lexsort((exp["key"], exp["window_end"]))
        for gf, ef in (("key", "key"), ("window_end", "window_end"), ("sum", "sum_i"), ("rowtime", "out_ts")):
            assert np.array_equal(rows[gf][sg], exp[ef][se]), f"{ctx}: {gf}"
    else:
        compare_rows(rows, exp, size if slide == 0 else slide, ctx, aggs)   # window ends lie on this grid
    assert late == olate, f"{ctx}: late drops {late} vs {olate}"
    return len(rows), late


def test_config0_datastream_tumble_10M_records():
    """configs[0]: DataStream keyBy().window(TumblingEventTimeWindows 1s).sum, 10M (long, long)
    records, 10k keys, watermark every 10k records (WindowOperator + SumAggregator)."""
    from oracle import oracle as O
    nrows, _ = run_config("datastream", 10_000_000, ("sum",), O.TUMBLE, 1000, 0)
    assert nrows == 10 * 10_000


@pytest.mark.parametrize("grid", ["-1", "3", "400"])
def test_config0_datastream_forced_tile_grid(monkeypatch, grid):
    """configs[0] with pass 1's grid of tile passes forced (FG_TILE_GRID, read at fg_open): the
    round-4 rule (one workgroup per 16,384 records), several tiles per workgroup, and more
    workgroups than a 1M-record batch's 163 tiles (empty segments). The default is one
    workgroup per tile; every consumer reads the segment split from the pass."""
    from oracle import oracle as O
    monkeypatch.setenv("FG_TILE_GRID", grid)
    nrows, _ = run_config("datastream", 4_000_000, ("sum",), O.TUMBLE, 1000, 0)
    assert nrows == 4 * 10_000


def test_config1_tumble_two_passes_per_window():
    """configs[1] in 50M-record micro-batches: every window fires from two tile passes of 8.1k tiles
    each, large enough that the fire's waves take their tile groups from the per-pass LDS counters
    (tile_walk_grab; one counter per pass, the second pass's groups taken while slower waves still
    walk the first)."""
    from oracle import oracle as O
    nrows, late = run_config("tumble", 200_000_000, ("count_star", "count", "sum", "avg"), O.TUMBLE, 1000, 0,
                             async_wm=True, batch=50_000_000)
    assert nrows > 19_000_000 and late == 0


@pytest.mark.parametrize("wm", ["sync", "async"])
def test_config1_tumble_10M_keys(wm):
    """configs[1]: SQL TUMBLE 1s COUNT(*)/COUNT/SUM/AVG(double), 10M uniform keys, 200M records =
    2 windows of 100M records (~10 records per (key, window))."""
    from oracle import oracle as O
    nrows, late = run_config("tumble", 200_000_000, ("count_star", "count", "sum", "avg"), O.TUMBLE, 1000, 0,
                             async_wm=wm == "async")
    assert nrows > 19_000_000 and late == 0


@pytest.mark.parametrize("wm", ["sync", "async"])
def test_config2_hop_5min_1min_10M_keys(wm):
    """configs[2]: SQL HOP 5min/1min, 10M keys, 200M records = 6 event-minutes: every window
    merges up to 5 one-minute slice tables on fire."""
    from oracle import oracle as O
    nrows, _ = run_config("hop", 200_000_000, ("count_star", "sum", "avg"), O.HOP, 300_000, 60_000,
                          async_wm=wm == "async")
    assert nrows > 50_000_000


@pytest.mark.parametrize("wm", ["sync", "async"])
def test_config3_cumulate_1h_1min_per_gpu_share(wm):
    """configs[3]: SQL CUMULATE 1h/1min over the 12.5M-key per-GPU share of 100M keys, 70M
    records = 4+ one-minute steps of the hour window (each step window folds its slice into
    the first slice's state and emits every key seen so far)."""
    from oracle import oracle as O
    nrows, _ = run_config("cumulate", 70_000_000, ("count_star", "sum", "avg"), O.CUMULATE, 3_600_000, 60_000,
                          final_wm_after=60_000, async_wm=wm == "async")
    assert nrows > 30_000_000


@pytest.mark.parametrize("wm", ["sync", "async"])
def test_config4_zipf_jitter_checkpoint_restore(wm):
    """configs[4]: TUMBLE 1s AVG(double) over Zipf(1.1) keys (10M ranks), rowtime jitter
    U[0, 2 s), watermark = max rowtime - 2 s - 1 (bounded out-of-orderness), and a checkpoint
    after the third micro-batch followed by a failover: the operator is closed and a new one
    restored from the snapshot image continues the stream."""
    from oracle import oracle as O
    nrows, _ = run_config("zipf", 300_000_000, ("count_star", "avg"), O.TUMBLE, 1000, 0, snapshot_after_batch=2,
                          async_wm=wm == "async")
    assert nrows > 5_000_000
