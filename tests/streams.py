"""Deterministic synthetic keyed streams (counter-based splitmix64, BASELINE.md seed)."""
from __future__ import annotations

import numpy as np

SEED = 0x5EEDF11C
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (x + np.uint64(0x9E3779B97F4A7C15)) & M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M64
        return z ^ (z >> np.uint64(31))


def zipf_keys(u, keys, s):
    """Zipf(s) ranks 0..keys-1 by inverse CDF of the uniform 53-bit fraction of u."""
    w = np.arange(1, keys + 1, dtype=np.float64) ** -s
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    q = (u >> np.uint64(11)).astype(np.float64) * (1.0 / float(1 << 53))
    return np.minimum(np.searchsorted(cdf, q), keys - 1).astype(np.int64)


def make_stream(n, keys, val_type="f64", t0=1_600_000_000_000, rate_per_ms=100, jitter_ms=0, null_frac=0.0,
                seed=SEED, key_spread=False, big_ints=False, zipf=0.0, signed=False, cancel=False, specials=0.0):
    """Returns (key, rowtime, val, isnull) numpy arrays.

    rowtime = t0 + i / rate_per_ms (+ uniform jitter in [0, jitter_ms) when out of order);
    keys uniform over [0, keys), or Zipf(zipf) ranks (hot keys) when zipf > 0.
    signed: DOUBLE values uniform in [-1000, 1000) instead of [0, 1000).
    cancel: every odd record repeats the previous record's key and rowtime with the negated
    value (plus a small perturbation), so (key, window) sums nearly cancel.
    specials (DOUBLE): that fraction of the values replaced by NaNs (several payloads and
    signs), -0.0, +0.0, +inf and -inf -- the cases where Double.compareTo and the primitive
    comparison part ways."""
    i = np.arange(n, dtype=np.uint64)
    u = splitmix64(np.uint64(seed) ^ i)
    u2 = splitmix64(np.uint64(seed * 3 + 1) ^ i)
    key = zipf_keys(u, keys, zipf) if zipf > 0 else (u % np.uint64(keys)).astype(np.int64)
    if key_spread:   # spread ids over the whole i64 range (incl. the sentinel Long.MIN_VALUE)
        key = splitmix64(key.astype(np.uint64) ^ np.uint64(77)).view(np.int64)
        key[key == key.min()] = np.iinfo(np.int64).min
    ts = (np.int64(t0) + (np.arange(n, dtype=np.int64) // rate_per_ms)).astype(np.int64)
    if jitter_ms:
        ts = ts + (u2 % np.uint64(jitter_ms)).astype(np.int64)
    if val_type == "f64":
        val = (u2 >> np.uint64(11)).astype(np.float64) * (1000.0 / float(1 << 53))
        if signed:
            val = val * 2.0 - 1000.0
    else:
        if big_ints:
            val = (u2 ^ (u << np.uint64(7))).view(np.int64)   # full-range: exercises Java wrap-around
        else:
            val = (u2 % np.uint64(1000)).astype(np.int64) - 300
    if cancel:
        odd = np.arange(1, n, 2)
        key[odd] = key[odd - 1]
        ts[odd] = ts[odd - 1]
        val[odd] = -val[odd - 1] + (val[odd] if val_type != "f64" else val[odd] * 1e-9)
    if specials > 0 and val_type == "f64":
        sp = np.array([0x7FF8000000000000, 0x7FF0000000000001, -0x0008000000000000, -0x0000000000000001,
                       -0x8000000000000000, 0, 0x7FF0000000000000, -0x0010000000000000], dtype=np.int64).view(np.float64)
        pick = (u2 >> np.uint64(20)) % np.uint64(1000) < np.uint64(int(specials * 1000))
        val[pick] = sp[((u >> np.uint64(50)) % np.uint64(len(sp))).astype(np.int64)[pick]]
    isnull = None
    if null_frac > 0:
        isnull = ((u2 >> np.uint64(40)) % np.uint64(1000) < np.uint64(int(null_frac * 1000))).astype(np.uint8)
    return key, ts, val, isnull


def batches_with_watermarks(n, batch, ts, delay_ms):
    """Yields (lo, hi, watermark) with watermark = max rowtime so far - delay - 1 (bounded
    out-of-orderness, BoundedOutOfOrdernessWatermarks.java:57,69)."""
    mx = np.iinfo(np.int64).min
    for lo in range(0, n, batch):
        hi = min(n, lo + batch)
        mx = max(mx, int(ts[lo:hi].max()))
        yield lo, hi, mx - delay_ms - 1


def fmix64_inv(h):
    """Inverse of the MurmurHash3 fmix64 finalizer (numpy uint64; fg_window.h fmix64_inv)."""
    h = np.asarray(h, dtype=np.uint64).copy()
    with np.errstate(over="ignore"):
        h ^= h >> np.uint64(33)
        h *= np.uint64(0x9cb4b2f8129337db)
        h ^= h >> np.uint64(33)
        h *= np.uint64(0x4f74430c22a54005)
        h ^= h >> np.uint64(33)
    return h


def keys_in_one_region(n, seed=SEED):
    """n distinct BIGINT keys whose fmix64 mix has its top 16 bits zero: they share a state
    region at every split the engine can make (at most 2^13 regions)."""
    h = np.unique(splitmix64(np.uint64(seed) ^ np.arange(2 * n, dtype=np.uint64)) >> np.uint64(16))[:n]
    return fmix64_inv(h).view(np.int64)
