"""The shim's incremental checkpoint write (flink_amd.keyed_state, mirror of
GpuSlicingWindowProcessor.writeKeyedState) on synthetic engine images, without a GPU: after every
checkpoint the backend written incrementally equals the one round 5's full rewrite leaves (entries
and, once the timer service has passed the watermark, timers), and a checkpoint after which only
one slice changed costs that slice's entries, not the state's."""
import numpy as np
import pytest

from flink_amd.keyed_state import CUMULATE, HOP, TUMBLE, SliceSpec, WindowAggsState


def image_of(state):
    """an engine image + its fg_snapshot_slices view from {slice_end: {key: (cs, cv, sum)}} and
    {slice_end: changed}"""
    cols = {c: [] for c in ("key", "slice_end", "cnt_star", "cnt_val", "sum")}
    se_l, first, rows, changed = [], [], [], []
    for se in sorted(state):
        first.append(len(cols["key"]))
        for k, (cs, cv, s) in sorted(state[se]["rows"].items()):
            cols["key"].append(k)
            cols["slice_end"].append(se)
            cols["cnt_star"].append(cs)
            cols["cnt_val"].append(cv)
            cols["sum"].append(int(np.float64(s).view(np.int64)))
        se_l.append(se)
        rows.append(len(cols["key"]) - first[-1])
        changed.append(state[se]["changed"])
    img = {c: np.array(v, dtype=np.int64) for c, v in cols.items()}
    sl = dict(slice_end=np.array(se_l, dtype=np.int64), first_row=np.array(first, dtype=np.int64),
              rows=np.array(rows, dtype=np.int64), changed=np.array(changed, dtype=bool))
    return img, sl


def run_checkpoints(spec, images):
    inc, full = WindowAggsState(spec), WindowAggsState(spec)
    costs = []
    for state, progress in images:
        img, sl = image_of(state)
        for b in (inc, full):
            b.advance_watermark(progress)   # (the operator forwarded the watermark before the barrier)
        costs.append(inc.write_image(img, sl, progress))
        full.write_image_full(img, sl, progress)
        assert inc.entries == full.entries
        assert inc.timers == full.timers
    return inc, costs


def slice_rows(rng, keys, n):
    ks = rng.choice(keys, size=n, replace=False)
    return {int(k): (int(rng.integers(1, 9)), int(rng.integers(1, 9)), float(rng.random())) for k in ks}


@pytest.mark.parametrize("kind", ["tumble", "hop", "cumulate"])
def test_incremental_write_equals_full_rewrite(kind):
    rng = np.random.default_rng(5)
    keys = np.arange(2000)
    if kind == "tumble":
        spec = SliceSpec(TUMBLE, 1000)
    elif kind == "hop":
        spec = SliceSpec(HOP, 3000, 1000)
    else:
        spec = SliceSpec(CUMULATE, 4000, 1000)
    # checkpoint 1: slices 1000..4000; checkpoint 2: 1000 gone (expired), 3000 changed, 5000 new;
    # checkpoint 3: nothing changed but the progress moved past 3000
    s = {se: dict(rows=slice_rows(rng, keys, 300), changed=True) for se in (1000, 2000, 3000, 4000)}
    ck = [(s, 1500)]
    s2 = {se: dict(rows=dict(v["rows"]), changed=False) for se, v in s.items() if se != 1000}
    s2[3000]["rows"].update(slice_rows(rng, keys, 50))
    s2[3000]["changed"] = True
    s2[5000] = dict(rows=slice_rows(rng, keys, 200), changed=True)
    ck.append((s2, 2500))
    s3 = {se: dict(rows=v["rows"], changed=False) for se, v in s2.items()}
    ck.append((s3, 3200))
    inc, costs = run_checkpoints(spec, ck)
    total = sum(len(v["rows"]) for v in s2.values())
    if kind != "cumulate":   # (there a slice that fired moves into its window's namespace: rebuilt)
        assert costs[1]["put"] == len(s2[3000]["rows"]) + len(s2[5000]["rows"]) < total
        assert costs[2]["put"] == 0 and costs[2]["clear"] == 0


def test_second_checkpoint_writes_only_the_changed_slice():
    """two barriers close together (configs[4]: a checkpoint every 10 s of a 1 s TUMBLE): between
    them only the open slice took records -- the second write puts that slice's entries only"""
    rng = np.random.default_rng(9)
    keys = np.arange(100_000)
    spec = SliceSpec(TUMBLE, 1000)
    s = {se: dict(rows=slice_rows(rng, keys, 20_000), changed=True) for se in (10_000, 11_000, 12_000)}
    s2 = {se: dict(rows=dict(v["rows"]), changed=se == 12_000) for se, v in s.items()}
    s2[12_000]["rows"].update(slice_rows(rng, keys, 500))
    inc, costs = run_checkpoints(spec, [(s, 9_500), (s2, 9_600)])
    state = sum(len(v["rows"]) for v in s2.values())
    assert costs[1]["put"] == len(s2[12_000]["rows"]) <= state / 2
    assert costs[1]["clear"] == 0 and costs[1]["timer_delete"] == 0


def test_restore_image_roundtrip():
    """restoreFromKeyedState reads back what was written: every entry once, the timer watermark one
    below the smallest pending window timer"""
    rng = np.random.default_rng(3)
    spec = SliceSpec(TUMBLE, 1000)
    s = {se: dict(rows=slice_rows(rng, np.arange(500), 100), changed=True) for se in (3000, 4000)}
    inc, _ = run_checkpoints(spec, [(s, 2500)])
    cols, twm = inc.image()
    assert len(cols["key"]) == 200 and set(cols["slice_end"].tolist()) == {3000, 4000}
    assert twm == 3000 - 1 - 1   # (the timer of window end 3000 is at 2999)
