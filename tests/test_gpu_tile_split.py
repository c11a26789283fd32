"""Skewed tile passes (Zipf hot keys) on the tile path: the split fire (k_tile_plan ->
k_tile_fire over chunk items -> k_tile_fire's merge launch over the split buckets' partial
entries; FG_TILE_HOT=1 adds the hot-key wave pre-combine) against the oracle, and the parallel materialize of a skewed lane (checkpoint). A hot key's bucket above
max(kTileChunk, 4x the lane's mean) records is cut into chunk items over its tiles
(fg_kernels.h TileSplit); results must equal the oracle's exactly as any other fire's
(bit-exact keys, counts, i64 sums, MIN / MAX; f64 sums within the north_star tolerance)."""
import pytest

from tests.test_gpu_parity import cfg_of, drive_both

pytestmark = pytest.mark.gpu

# slices of 4M records (rate 4000 / ms, 1 s windows): the top Zipf(1.1) key holds ~11 % of them,
# several kTileChunk chunks; jitter + delay leave a slice's records in 2-3 tile passes
BIG = dict(n=12_000_000, keys=1_000_000, batch=2_000_000, rate_per_ms=4_000, zipf=1.1)

CASES = [
    ("tumble_f64_inorder", cfg_of("tumble", 1000), dict(BIG, delay=0, jitter=0)),
    ("tumble_f64_ooo_passes", cfg_of("tumble", 1000), dict(BIG, delay=400, jitter=700)),
    ("tumble_i64_hot13", cfg_of("tumble", 1000, vt="i64"), dict(BIG, zipf=1.3, delay=200, jitter=300)),
    ("tumble_i64_min", dict(cfg_of("tumble", 1000, vt="i64"), aggs=("count_star", "count", "min")),
     dict(BIG, delay=200, jitter=300)),
    ("tumble_f64_max", dict(cfg_of("tumble", 1000), aggs=("count_star", "count", "max")),
     dict(BIG, delay=0, jitter=0)),
    ("ds_tumble_f64", cfg_of("tumble", 1000, mode="datastream"), dict(BIG, delay=100, jitter=200)),
    ("tumble_f64_snapshot", cfg_of("tumble", 1000), dict(BIG, delay=400, jitter=700, snapshot_at=3)),
]


@pytest.mark.parametrize("name,cfg,kw", CASES, ids=[c[0] for c in CASES])
def test_zipf_split_fire_parity(oracle_mod, name, cfg, kw):
    ks = {}
    drive_both(oracle_mod, cfg, kstats=ks, **kw)
    if "snapshot_at" in kw:   # (kstats: the restored copy's, which times nothing)
        return
    assert ks.get("tile_split_fire", {}).get("launches", 0) > 0, ks
    assert ks.get("merge_heavy", {}).get("launches", 0) == 0, ks   # (the skewed passes stayed on the tiles)


@pytest.mark.parametrize("name,cfg,kw", [CASES[1], CASES[2], CASES[4]], ids=[CASES[i][0] + "_hot" for i in (1, 2, 4)])
def test_zipf_split_fire_hot_precombine_parity(oracle_mod, name, cfg, kw, monkeypatch):
    """FG_TILE_HOT=1: chunk items pre-combine a wave's records of a hot key (off by default)."""
    monkeypatch.setenv("FG_TILE_HOT", "1")
    ks = {}
    drive_both(oracle_mod, cfg, kstats=ks, **kw)
    assert ks.get("tile_split_fire", {}).get("launches", 0) > 0, ks


def test_zipf_split_off_takes_heavy_path(oracle_mod, monkeypatch):
    """FG_TILE_SPLIT=0: a skewed tile pass is staged again by the two-pass partition (heavy path)."""
    monkeypatch.setenv("FG_TILE_SPLIT", "0")
    ks = {}
    drive_both(oracle_mod, cfg_of("tumble", 1000), kstats=ks, **dict(BIG, n=6_000_000, delay=0, jitter=0))
    assert ks.get("tile_split_fire", {}).get("launches", 0) == 0, ks
    assert ks.get("merge_heavy", {}).get("launches", 0) > 0, ks


# few buckets (a small key space, configs[0]-shaped): a lane of fewer buckets than CUs fires as
# ~2 chunk items per CU ("spread"), merged per bucket -- same rows as the one-workgroup fire
SPREAD = [
    ("ds_tumble_i64_10k_keys", cfg_of("tumble", 1000, vt="i64", mode="datastream"),
     dict(n=6_000_000, keys=10_000, batch=1_000_000, rate_per_ms=1_000, delay=0, jitter=0)),
    ("tumble_f64_6k_keys_ooo", cfg_of("tumble", 1000), dict(n=6_000_000, keys=6_000, batch=1_000_000,
                                                              rate_per_ms=2_000, delay=300, jitter=500)),
    ("ds_tumble_f64_min_specials", dict(cfg_of("tumble", 1000, mode="datastream"), aggs=("count_star", "min")),
     dict(n=4_000_000, keys=10_000, batch=1_000_000, rate_per_ms=1_000, delay=0, jitter=0, specials=0.02)),
    ("tumble_i64_max", dict(cfg_of("tumble", 1000, vt="i64"), aggs=("count_star", "count", "max")),
     dict(n=4_000_000, keys=8_000, batch=1_000_000, rate_per_ms=1_000, delay=0, jitter=0)),
]


@pytest.mark.parametrize("name,cfg,kw", SPREAD, ids=[c[0] for c in SPREAD])
def test_spread_fire_parity(oracle_mod, name, cfg, kw, monkeypatch):
    # 2^8 regions: 64 buckets per lane, fewer than the CUs (the default 2^10 from 4,096 expected
    # keys gives 256 buckets, one per CU, and needs no spread)
    monkeypatch.setenv("FG_MIN_REGION_BITS", "8")
    ks = {}
    drive_both(oracle_mod, cfg, kstats=ks, **kw)
    assert ks.get("tile_split_fire", {}).get("launches", 0) > 0, ks


def test_window_of_many_micro_batches_fires_from_the_tiles(oracle_mod):
    """A window spanning more micro-batches than the split fire walks (kMaxTilePasses = 8): 10
    uniform 100k-record batches per 1 s window (a shim with a small batchRecords). No pass is
    skewed, so the plain fire takes every pass from the tiles -- no lane is materialized (ADVICE
    round 5: the pass limit applied to unskewed lanes too)."""
    ks = {}
    drive_both(oracle_mod, cfg_of("tumble", 1000), kstats=ks,
               n=3_000_000, keys=1_000_000, batch=100_000, rate_per_ms=1_000, delay=0, jitter=0,
               buffer_records=4_000_000)
    assert ks.get("tile_fire", {}).get("launches", 0) > 0, ks
    assert ks.get("tile_materialize", {}).get("launches", 0) == 0, ks
