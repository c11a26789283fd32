"""GPU tests of the key dictionary (fg_key_dict_*): grouping keys of any type (STRING, several
key columns, NULL keys) interned as BinaryRowData key rows, with exact ids, Flink key groups
(BinarySection.hashCode -> KeyGroupRangeAssignment), and the reference's own operator tests run
with their literal STRING keys through the dictionary + the window engine."""

import numpy as np
import pytest

import flink_amd as F
from flink_amd import keys as K
from oracle import oracle as O
from tests.fixture_runner import load_operator_cases, run_case

pytestmark = pytest.mark.gpu

MAXP = 128
TYPES = ["string", "bigint"]


def random_keys(rng, n_distinct):
    out = set()
    while len(out) < n_distinct:
        n = int(rng.integers(0, 41))
        s = "".join(chr(c) for c in rng.integers(0x20, 0x7f, n))
        out.add((s if rng.random() > 0.02 else None, int(rng.integers(-5, 5))))
    return sorted(out, key=lambda t: (t[0] is None, t[0] or "", t[1]))


def check_interned(d, rows, ids, kgs):
    ids = np.asarray(ids)
    first = {}
    for r, i in zip(rows, ids.tolist()):
        assert first.setdefault(r, i) == i, "equal key rows got different ids"
    assert len(set(first.values())) == len(first), "distinct key rows share an id"
    exp_kg = np.array([O.key_group_of_row(r, MAXP) for r in rows], dtype=np.int32)
    assert np.array_equal(np.asarray(kgs), exp_kg)
    assert np.array_equal(K.key_group_of_id(ids, MAXP), exp_kg)
    assert d.lookup(ids) == list(rows)
    return first


def test_intern_exact_ids_key_groups_and_lookup():
    rng = np.random.default_rng(3)
    keys = random_keys(rng, 40_000)
    rows_all = [K.key_row(list(k), TYPES) for k in keys]
    d = F.KeyDictionary(max_parallelism=MAXP, expected_keys=1000)   # grows several times
    seen = {}
    for b in range(5):
        pick = rng.integers(0, len(rows_all), 60_000)
        rows = [rows_all[i] for i in pick]
        ids, kgs = d.intern(rows)
        m = check_interned(d, rows, ids, kgs)
        for r, i in m.items():
            assert seen.setdefault(r, i) == i, "an id changed across calls"
    assert len(d) == len(seen)
    # device input: the same rows as torch tensors on the GPU get the same ids
    import torch
    rows = [rows_all[i] for i in rng.integers(0, len(rows_all), 30_000)]
    buf, off, ln = K.pack_key_rows(rows)
    dev = torch.device("cuda", 0)
    ids_t, kg_t = d.intern(packed=(torch.from_numpy(buf.copy()).to(dev), torch.from_numpy(off).to(dev),
                                   torch.from_numpy(ln).to(dev)))
    ids = ids_t.cpu().numpy()
    for r, i in zip(rows, ids.tolist()):
        if r in seen:
            assert seen[r] == i
    check_interned(d, rows, ids, kg_t.cpu().numpy())
    d.close()


def test_intern_forced_hash_collisions_stay_exact(monkeypatch):
    """A 6-bit table tag (diagnostic knob): nearly every distinct row collides with another's
    tag; the byte comparison sends them to the host map and the ids stay exact."""
    monkeypatch.setenv("FG_DICT_TAG_BITS", "6")
    rng = np.random.default_rng(11)
    keys = random_keys(rng, 3000)
    rows_all = [K.key_row(list(k), TYPES) for k in keys]
    d = F.KeyDictionary(max_parallelism=MAXP, expected_keys=16)
    seen = {}
    for _ in range(3):
        rows = [rows_all[i] for i in rng.integers(0, len(rows_all), 8000)]
        ids, kgs = d.intern(rows)
        for r, i in check_interned(d, rows, ids, kgs).items():
            assert seen.setdefault(r, i) == i
    # the same from device buffers (the host resolves the colliding rows from one copy)
    import torch
    dev = torch.device("cuda", 0)
    for _ in range(2):
        rows = [rows_all[i] for i in rng.integers(0, len(rows_all), 8000)]
        buf, off, ln = K.pack_key_rows(rows)
        ids_t, kg_t = d.intern(packed=(torch.from_numpy(buf.copy()).to(dev), torch.from_numpy(off).to(dev),
                                       torch.from_numpy(ln).to(dev)))
        for r, i in check_interned(d, rows, ids_t.cpu().numpy(), kg_t.cpu().numpy()).items():
            assert seen.setdefault(r, i) == i
    assert len(d) == len(seen)
    d.close()


def test_intern_rejects_bad_rows_and_keeps_working():
    d = F.KeyDictionary(max_parallelism=MAXP)
    buf = np.zeros(64, dtype=np.uint8)
    with pytest.raises(F.WindowSpecError):
        d.intern(packed=(buf, np.array([0, 8], dtype=np.int64), np.array([16, 6], dtype=np.int32)))
    with pytest.raises(F.WindowSpecError):
        d.intern(packed=(buf, np.array([56], dtype=np.int64), np.array([16], dtype=np.int32)))
    import torch
    dev = torch.device("cuda", 0)
    with pytest.raises(F.WindowSpecError):
        d.intern(packed=(torch.zeros(64, dtype=torch.uint8, device=dev), torch.tensor([4, 60], device=dev),
                         torch.tensor([16, 8], dtype=torch.int32, device=dev)))
    rows = [K.key_row(["k%d" % i], ["string"]) for i in range(100)]
    ids, kgs = d.intern(rows)
    check_interned(d, rows, ids, kgs)
    assert len(d) == 100
    d.close()


# the reference's operator tests with their literal STRING keys (the fixtures number them)
SLICING_NAMES = {1: "key1", 2: "key2"}
ITCASE_NAMES = {1: "a", 2: "b", 3: None}   # TestData.windowDataWithTimestamp: a NULL name
STRING_CASES = [c for c in load_operator_cases() if c["config"]["mode"] == "sql"]


def names_of(case):
    if case["name"].startswith("itcase"):
        return ITCASE_NAMES
    if "dst" in case["name"]:
        return {1: "a"}
    return SLICING_NAMES


class StringKeyOperator:
    """GpuOperator whose keys enter as BinaryRowData STRING key rows interned by the dictionary
    (the shim's path for non-BIGINT keys) and leave as the rows' strings (back to the fixture's
    numbering for the comparison)."""

    def __init__(self, inner, d, names):
        self.inner, self.d, self.names = inner, d, names
        self.back = {v: k for k, v in names.items()}

    def process_batch(self, key, ts, val=None, isnull=None):
        rows = [K.key_row([self.names[int(k)]], ["string"]) for k in key]
        ids, _ = self.d.intern(rows)
        self.inner.process_batch(ids, ts, val, isnull)

    def process_watermark(self, wm):
        self.inner.process_watermark(wm)

    def prepare_snapshot(self):
        self.inner.prepare_snapshot()

    def restore_copy(self):
        return StringKeyOperator(self.inner.restore_copy(), self.d, self.names)

    @property
    def late_dropped(self):
        return self.inner.late_dropped

    def take_rows(self):
        r = self.inner.take_rows()
        if len(r):
            rows = self.d.lookup(r["key"])
            r["key"] = [self.back[K.decode_key_row(x, ["string"])[0]] for x in rows]
        return r

    def close(self):
        self.inner.close()


@pytest.mark.parametrize("case", STRING_CASES, ids=[c["name"] for c in STRING_CASES])
def test_golden_cases_with_string_keys(case):
    from tests.test_gpu_parity import gpu_mk
    d = F.KeyDictionary(max_parallelism=MAXP)
    results, late = run_case(case, lambda cfg: StringKeyOperator(gpu_mk(cfg), d, names_of(case)))
    for step, got, exp in results:
        assert got == exp, f"{case['name']} step {step}: got {got} expected {exp}"
    if case["expected_late_dropped"] is not None:
        assert late == case["expected_late_dropped"]
    d.close()


@pytest.mark.parametrize("kind", ["tumble", "hop"])
def test_string_keys_stream_vs_oracle(oracle_mod, kind):
    """A randomized out-of-order stream over 20k (STRING, BIGINT) keys: the GPU path (dictionary
    ids -> engine) against the oracle run on the same keys numbered by position."""
    from tests.test_gpu_parity import assert_rows_equal, cfg_of, gpu_mk, oracle_mk
    rng = np.random.default_rng(5)
    keys = random_keys(rng, 20_000)
    rows_all = [K.key_row(list(k), TYPES) for k in keys]
    index = {r: i for i, r in enumerate(rows_all)}
    n = 300_000
    pick = rng.integers(0, len(rows_all), n)
    ts = (1_000_000 + np.arange(n) // 100 + rng.integers(0, 300, n)).astype(np.int64)
    val = rng.random(n) * 1000.0
    cfg = cfg_of(kind, 3000 if kind == "hop" else 1000, 1000 if kind == "hop" else 0)
    d = F.KeyDictionary(max_parallelism=MAXP, expected_keys=len(rows_all))
    g = gpu_mk(cfg, expected_keys=len(rows_all))
    o = oracle_mk(oracle_mod, cfg)

    def check(ctx):
        r = g.take_rows()
        if len(r):
            r["key"] = [index[x] for x in d.lookup(r["key"])]
        assert_rows_equal(r, o.take_rows(), "f64", ctx)

    for lo in range(0, n, 50_000):
        hi = lo + 50_000
        ids, _ = d.intern([rows_all[i] for i in pick[lo:hi]])
        g.process_batch(ids, ts[lo:hi], val[lo:hi])
        o.process_batch(pick[lo:hi].astype(np.int64), ts[lo:hi], val[lo:hi])
        wm = int(ts[hi - 1]) - 400
        g.process_watermark(wm)
        o.process_watermark(wm)
        check(f"wm {wm}")
    assert g.late_dropped == o.late_dropped
    g.process_watermark((1 << 63) - 1)
    o.process_watermark((1 << 63) - 1)
    check("final")
    g.close()
    o.close()
    d.close()


def test_dictionary_ids_route_by_the_rows_key_group():
    """FG_KEYHASH_DICT_ID: owner partitioning of partial rows keyed by dictionary ids sends
    each row to the subtask of its key row's Flink key group (kg * P / maxP)."""
    import torch

    from flink_amd import _lib as L
    from flink_amd.exchange import partition_columns_by_owner
    rng = np.random.default_rng(9)
    keys = random_keys(rng, 5000)
    rows_all = [K.key_row(list(k), TYPES) for k in keys]
    d = F.KeyDictionary(max_parallelism=MAXP)
    pick = rng.integers(0, len(rows_all), 50_000)
    ids, kgs = d.intern([rows_all[i] for i in pick])
    assert np.array_equal(F.key_groups(ids, MAXP, key_hash=L.KEYHASH_DICT_ID), kgs)
    par = 8
    dev = torch.device("cuda", 0)
    cols = [torch.from_numpy(ids).to(dev), torch.arange(len(ids), dtype=torch.int64, device=dev)]
    outs, counts = partition_columns_by_owner(cols, par, MAXP, key_hash=L.KEYHASH_DICT_ID)
    owner = kgs.astype(np.int64) * par // MAXP
    assert np.array_equal(counts.cpu().numpy(), np.bincount(owner, minlength=par))
    pos = outs[1].cpu().numpy()
    off = np.concatenate([[0], np.cumsum(counts.cpu().numpy())])
    for r in range(par):
        assert (owner[pos[off[r]:off[r + 1]]] == r).all()
    d.close()


def test_intern_chunked_call_unaligned_rows_and_no_key_groups():
    """One call larger than a chunk (the table grows with the ids, the call is split into chunks
    of at most the table's headroom), BIGINT key rows read from 8-byte-aligned and from only
    4-byte-aligned offsets (register path, 8- and 4-byte loads), and the call without key groups:
    the same exact ids everywhere."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    distinct = rng.choice(np.arange(-(1 << 40), 1 << 40, 7919, dtype=np.int64), 50_000, replace=False)
    keys = distinct[rng.integers(0, len(distinct), 9_000_000)]
    n = len(keys)
    rows = np.zeros((n, 2), dtype=np.int64)   # BinaryRowData of one BIGINT field: null bits, value
    rows[:, 1] = keys
    buf = torch.from_numpy(rows.view(np.uint8).reshape(-1)).to(dev)
    off = torch.arange(n, dtype=torch.int64, device=dev) * 16
    ln = torch.full((n,), 16, dtype=torch.int32, device=dev)
    d = F.KeyDictionary(max_parallelism=MAXP, expected_keys=1000)
    ids_t, kg_t = d.intern(packed=(buf, off, ln))
    ids = ids_t.cpu().numpy()
    assert len(d) == len(distinct)
    pairs = np.unique(np.stack([keys, ids]), axis=1)
    assert pairs.shape[1] == len(distinct) and len(np.unique(ids)) == len(distinct)   # a bijection
    _, first, inv = np.unique(keys, return_index=True, return_inverse=True)
    kg_u = np.array([O.key_group_of_row(rows[i].tobytes(), MAXP) for i in first], dtype=np.int32)
    assert np.array_equal(kg_t.cpu().numpy(), kg_u[inv])
    assert np.array_equal(K.key_group_of_id(ids, MAXP), kg_t.cpu().numpy())
    # the same rows at 4-byte-aligned offsets (a 4-byte pad in front), without key groups
    buf4 = torch.cat([torch.zeros(4, dtype=torch.uint8, device=dev), buf])
    ids4, kg4 = d.intern(packed=(buf4, off + 4, ln), key_groups=False)
    assert kg4 is None
    assert np.array_equal(ids4.cpu().numpy(), ids)
    assert len(d) == len(distinct)
    d.close()


def test_intern_async_matches_sync_and_overlaps_the_engine():
    """fg_key_dict_intern_async + _wait: the same id partition as the one-call intern for new and known rows
    (misses interned in _wait), key groups when asked for, one call pending at a time (a second
    async call, a lookup or a copy of the arena in between fail with FG_ESTATE), bad device rows
    reported by _wait with nothing inserted -- and the window engine fed the awaited ids gives the
    oracle's rows while the next batch's lookup runs beside it."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(21)
    keys = random_keys(rng, 20_000)
    rows_all = [K.key_row(list(k), TYPES) for k in keys]
    d = F.KeyDictionary(max_parallelism=MAXP, expected_keys=1000)
    ref = F.KeyDictionary(max_parallelism=MAXP, expected_keys=1000)
    seen = {}

    def packed_dev(rows):
        buf, off, ln = K.pack_key_rows(rows)
        return torch.from_numpy(buf.copy()).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)

    for b in range(4):   # the first batches hold mostly new rows, the later ones mostly known
        rows = [rows_all[i] for i in rng.integers(0, len(rows_all) * (b + 1) // 4, 30_000)]
        p = packed_dev(rows)
        ids_t, kg_t = d.intern_async(p, key_groups=True)
        with pytest.raises(F.FlinkGpuError):
            d.intern_async(p)
        with pytest.raises(F.FlinkGpuError):
            d.lookup(np.zeros(1, dtype=np.int64))
        d.intern_wait()
        ids_r, kg_r = ref.intern(rows)   # ordinals are assigned in parallel: the same partition
        pairs = np.unique(np.stack([ids_t.cpu().numpy(), ids_r]), axis=1)
        assert len(np.unique(pairs[0])) == len(np.unique(pairs[1])) == pairs.shape[1]
        assert np.array_equal(kg_t.cpu().numpy(), kg_r)
        for r, i in check_interned(d, rows, ids_t.cpu().numpy(), kg_t.cpu().numpy()).items():
            assert seen.setdefault(r, i) == i, "an id changed across calls"
    n0 = len(d)
    bad = (torch.zeros(64, dtype=torch.uint8, device=dev), torch.tensor([4, 60], device=dev),
           torch.tensor([16, 8], dtype=torch.int32, device=dev))
    d.intern_async(bad)
    with pytest.raises(F.WindowSpecError):
        d.intern_wait()
    assert len(d) == n0
    d.intern_wait()   # nothing pending: a no-op
    # the pipeline of bench.py --keys string: batch k+1's lookup beside batch k's aggregation
    from tests.test_gpu_parity import assert_rows_equal, cfg_of, gpu_mk, oracle_mk
    index = {}
    n, batch = 240_000, 40_000
    pick = rng.integers(0, len(rows_all), n)
    ts = (1_000_000 + np.arange(n) // 100 + rng.integers(0, 300, n)).astype(np.int64)
    val = rng.random(n) * 1000.0
    cfg = cfg_of("tumble", 1000)
    g = gpu_mk(cfg, expected_keys=len(rows_all))
    o = oracle_mk(O, cfg)
    packs = [packed_dev([rows_all[i] for i in pick[lo:lo + batch]]) for lo in range(0, n, batch)]
    k_next, _ = d.intern_async(packs[0])
    d.intern_wait()
    for bi, lo in enumerate(range(0, n, batch)):
        hi = lo + batch
        k = k_next
        if bi + 1 < len(packs):
            k_next, _ = d.intern_async(packs[bi + 1])
        g.process_batch(k, torch.from_numpy(ts[lo:hi]).to(dev), torch.from_numpy(val[lo:hi]).to(dev))
        o.process_batch(pick[lo:hi].astype(np.int64), ts[lo:hi], val[lo:hi])
        wm = int(ts[hi - 1]) - 400
        g.process_watermark(wm)
        o.process_watermark(wm)
        if bi + 1 < len(packs):
            d.intern_wait()
    g.process_watermark((1 << 63) - 1)
    o.process_watermark((1 << 63) - 1)
    r = g.take_rows()
    index = {rows_all[i]: i for i in range(len(rows_all))}
    r["key"] = [index[x] for x in d.lookup(r["key"])]
    assert_rows_equal(r, o.take_rows(), "f64", "async intern pipeline")
    g.close()
    o.close()
    d.close()
    ref.close()
