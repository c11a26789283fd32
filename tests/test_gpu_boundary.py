"""Buffer-ownership contract of the C-ABI (include/flinkgpu.h, fg_location), on the GPU.

The reference's callers reuse their input objects as soon as addElement returns
(RecordsWindowBuffer.java:81-97 copies each row: `requiresCopy`), and a JNI shim recycles its
pinned staging ring the same way. These tests overwrite (or free and reallocate) every input
buffer immediately after the call that consumed it and require the fired rows to still equal
the oracle's on the original data:
  * FG_HOST from PINNED host memory (the DMA reads the caller's buffer directly), and from
    plain host memory page-locked by fg_host_register (a shim's managed-memory segments);
  * FG_DEVICE torch columns dropped right after process_batch (torch's caching allocator
    hands the blocks to the next allocation on the current stream);
  * device key rows interned through the key dictionary straight after a producer kernel on
    torch's stream (the dictionary reads them on its own stream).
"""
import numpy as np
import pytest

from tests.streams import batches_with_watermarks, make_stream
from tests.test_gpu_parity import assert_rows_equal, oracle_mk

pytestmark = pytest.mark.gpu

CFG = dict(mode="sql", kind="tumble", size=1000, slide=0, offset=0, tz_offset_ms=0, val_type="f64",
           count_star_index=0)


def _drive(O, feed, n=1_200_000, keys=20_000, batch=100_000, jitter=1500, delay=500, cfg=CFG):
    """feed(g, lo, hi, key, ts, val) hands one batch to the GPU operator g however the test
    wants; the oracle gets the plain arrays."""
    from tests.gpu_adapter import GpuOperator
    key, ts, val, _ = make_stream(n, keys, cfg["val_type"], jitter_ms=jitter)
    g = GpuOperator(cfg, expected_keys=keys, buffer_records=batch * 4)
    o = oracle_mk(O, cfg)
    for step, (lo, hi, wm) in enumerate(batches_with_watermarks(n, batch, ts, delay)):
        feed(g, lo, hi, key, ts, val)
        o.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi])
        g.process_watermark(wm)
        o.process_watermark(wm)
        assert_rows_equal(g.take_rows(), o.take_rows(), cfg["val_type"], f"step {step}")
        assert g.late_dropped == o.late_dropped
    g.process_watermark((1 << 63) - 1)
    o.process_watermark((1 << 63) - 1)
    assert_rows_equal(g.take_rows(), o.take_rows(), cfg["val_type"], "final")
    g.close()
    o.close()


@pytest.mark.parametrize("kind", ["tumble", "hop"])
def test_pinned_host_batches_overwritten_after_call(oracle_mod, kind):
    """One pinned buffer set reused for every batch and scribbled over the moment
    process_batch returns: FG_HOST buffers must have been read completely by then."""
    import torch
    cfg = dict(CFG, kind=kind, size=1000 if kind == "tumble" else 4000, slide=0 if kind == "tumble" else 1000)
    cap = 100_000
    pk = torch.empty(cap, dtype=torch.int64).pin_memory()
    pt = torch.empty(cap, dtype=torch.int64).pin_memory()
    pv = torch.empty(cap, dtype=torch.float64).pin_memory()
    nk, nt, nv = pk.numpy(), pt.numpy(), pv.numpy()
    garbage = np.random.default_rng(7)

    def feed(g, lo, hi, key, ts, val):
        m = hi - lo
        nk[:m], nt[:m], nv[:m] = key[lo:hi], ts[lo:hi], val[lo:hi]
        g.process_batch(nk[:m], nt[:m], nv[:m])          # FG_HOST from pinned memory
        nk[:m] = garbage.integers(0, 1 << 40, m)          # the shim refills its staging slot
        nt[:m] = garbage.integers(0, 1 << 42, m)
        nv[:m] = np.nan

    _drive(oracle_mod, feed, cfg=cfg)


def test_registered_host_segments_overwritten_after_call(oracle_mod):
    """The shim's managed-memory path (fg_host_register): plain host allocations -- numpy
    arrays standing in for off-heap MemorySegments -- page-locked once, reused for every batch
    and scribbled over as soon as process_batch returns; unregistered at the end."""
    import flink_amd as F
    from flink_amd import _lib as L
    cap = 100_000
    nk, nt, nv = np.empty(cap, np.int64), np.empty(cap, np.int64), np.empty(cap, np.float64)
    garbage = np.random.default_rng(11)
    reg = F.HostRegistration(nk, nt, nv)

    def feed(g, lo, hi, key, ts, val):
        m = hi - lo
        nk[:m], nt[:m], nv[:m] = key[lo:hi], ts[lo:hi], val[lo:hi]
        g.process_batch(nk[:m], nt[:m], nv[:m])          # FG_HOST from registered memory
        nk[:m] = garbage.integers(0, 1 << 40, m)
        nt[:m] = garbage.integers(0, 1 << 42, m)
        nv[:m] = np.nan

    try:
        _drive(oracle_mod, feed)
    finally:
        reg.close()
    with pytest.raises(F.WindowSpecError):       # null range
        L.check(L.load().fg_host_register(0, None, 8))


@pytest.mark.parametrize("vt", ["f64", "i64"])
def test_narrow_host_batches(oracle_mod, vt):
    """fg_batch.format: int32 keys (negative ones too), rowtime as uint32 offsets from a per-batch
    base, int32 BIGINT values -- widened on the device; rows equal the oracle's on the 8-byte
    columns. Buffers are overwritten after each call as a shim's staging ring would be."""
    cap = 100_000
    nk, nt = np.empty(cap, np.int32), np.empty(cap, np.uint32)
    nv = np.empty(cap, np.float64 if vt == "f64" else np.int32)

    def feed(g, lo, hi, key, ts, val):
        m = hi - lo
        base = int(ts[lo:hi].min()) - 7
        nk[:m] = key[lo:hi] - 10_000                       # (the oracle sees the same shift)
        nt[:m] = (ts[lo:hi] - base).astype(np.uint32)
        nv[:m] = val[lo:hi]
        g.op.process_batch(nk[:m], nt[:m], nv[:m], rowtime_base=base)
        nk[:m], nt[:m] = 12345, 0xFFFFFFFF
        nv[:m] = -1

    from tests.gpu_adapter import GpuOperator
    cfg = dict(CFG, val_type=vt)
    n, keys, batch = 1_200_000, 20_000, 100_000
    key, ts, val, _ = make_stream(n, keys, vt, jitter_ms=1500)
    g = GpuOperator(cfg, expected_keys=keys, buffer_records=batch * 4)
    o = oracle_mk(oracle_mod, cfg)
    for step, (lo, hi, wm) in enumerate(batches_with_watermarks(n, batch, ts, 500)):
        feed(g, lo, hi, key, ts, val)
        o.process_batch(key[lo:hi] - 10_000, ts[lo:hi], val[lo:hi])
        g.process_watermark(wm)
        o.process_watermark(wm)
        assert_rows_equal(g.take_rows(), o.take_rows(), vt, f"step {step}")
        assert g.late_dropped == o.late_dropped
    g.process_watermark((1 << 63) - 1)
    o.process_watermark((1 << 63) - 1)
    assert_rows_equal(g.take_rows(), o.take_rows(), vt, "final")
    g.close()
    o.close()


def test_narrow_batch_format_rules():
    """FG_BATCH_VAL32 needs a BIGINT value; narrow columns only from the host."""
    import ctypes as C

    import torch
    import flink_amd as F
    from flink_amd import _lib as L
    op = F.WindowAggOperator(F.tumbling(1000), val_type="f64", expected_keys=1000)
    z = np.zeros(4, np.int64)
    b = L.FgBatch(n=4, location=L.HOST, format=L.BATCH_VAL32, key=z.ctypes.data, rowtime=z.ctypes.data,
                  val=z.ctypes.data)
    with pytest.raises(F.WindowSpecError):   # a DOUBLE operator's value cannot be narrow
        L.check(L.load().fg_add_batch(op._h, C.byref(b)), op._h)
    b.format = 8
    with pytest.raises(F.WindowSpecError):   # unknown format bit
        L.check(L.load().fg_add_batch(op._h, C.byref(b)), op._h)
    with pytest.raises(F.WindowSpecError):   # device columns with a rowtime base
        op.process_batch(torch.zeros(4, dtype=torch.int64, device="cuda"), torch.zeros(4, dtype=torch.int64, device="cuda"),
                         torch.zeros(4, dtype=torch.float64, device="cuda"), rowtime_base=5)
    op.close()


def test_device_columns_freed_after_call(oracle_mod):
    """Device columns dropped right after process_batch; the next allocations on torch's
    stream (same sizes, so the caching allocator offers the same blocks) are filled with
    garbage at once. The operator holds the columns until an event on the engine's stream after
    the next call has completed (fg_add_batch finishes a batch's staging in the next call)."""
    import torch

    def feed(g, lo, hi, key, ts, val):
        k = torch.from_numpy(key[lo:hi]).cuda()
        t = torch.from_numpy(ts[lo:hi]).cuda()
        v = torch.from_numpy(val[lo:hi]).cuda()
        g.process_batch(k, t, v)
        del k, t, v
        junk = [torch.full((hi - lo,), -7, dtype=torch.int64, device="cuda") for _ in range(3)]
        del junk

    _drive(oracle_mod, feed)


def test_device_columns_outlive_the_operator():
    """The caller's columns freed after the operator closed (and the cache emptied): nothing may
    refer to the destroyed engine stream then (a record_stream on it did, and the allocator's
    free path crashed)."""
    import torch

    from flink_amd import WindowAggOperator, tumbling
    n = 200_000
    k = torch.randint(0, 1000, (n,), dtype=torch.int64, device="cuda")
    t = torch.arange(n, dtype=torch.int64, device="cuda")
    v = torch.ones(n, dtype=torch.float64, device="cuda")
    op = WindowAggOperator(tumbling(1000), aggs=("count", "sum"), expected_keys=1000, buffer_records=1 << 20)
    op.process_batch(k, t, v)
    op.process_batch(k[: n // 2], t[: n // 2] + n, v[: n // 2])
    rows = op.process_watermark((1 << 63) - 1)
    assert rows["count"].sum() == n + n // 2
    op.close()
    del k, t, v, op
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    torch.cuda.synchronize()


def test_dictionary_reads_device_rows_after_their_producer():
    """Key rows written by a torch kernel and interned at once: the dictionary's stream must
    wait for torch's stream (fg_key_dict_stream), or it hashes unwritten bytes."""
    import torch

    from flink_amd.keys import KeyDictionary, key_row, pack_key_rows
    rows = [key_row([f"user-{i:07d}"], ["string"]) for i in range(50_000)]
    buf, off, ln = pack_key_rows(rows)
    from oracle import oracle as O
    exp_kg = np.array([O.key_group_of_row(r, 128) for r in rows[:2000]], dtype=np.int32)
    d = KeyDictionary(expected_keys=1 << 16)
    first = None
    for rep in range(3):
        src = torch.from_numpy(buf.copy()).cuda()
        dst = torch.zeros_like(src)
        torch.cuda._sleep(20_000_000)   # keep torch's stream busy so an unordered read sees zeros
        dst.copy_(src)
        ids, kg = d.intern(packed=(dst, torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda()))
        ids, kg = ids.cpu().numpy(), kg.cpu().numpy()
        assert np.array_equal(kg[:2000], exp_kg), f"rep {rep}: key groups differ"
        assert len(np.unique(ids)) == len(rows), f"rep {rep}: distinct rows share ids"
        if first is None:
            first = ids
        assert np.array_equal(ids, first), f"rep {rep}: ids not stable"
    assert len(d) == len(rows)
    d.close()


def test_device_selfcheck_of_scans_and_tile_walk():
    """fg_selftest (ABI 16): the DPP wave scans (wave_incl_scan add / max, wave_shr1) and the tile
    walk's group setup, fragment map and record sources, as this library's code object compiled
    them, against host answers (round 5: a compiler fold of the walk's DPP scan produced a fragment
    base of -3). fg_open runs the same check once per process."""
    import ctypes as C

    from flink_amd import _lib as L
    lib = L.load()
    buf = C.create_string_buffer(160)
    rc = lib.fg_selftest(0, buf, 160)
    assert rc == 0 and buf.value == b"ok", buf.value
