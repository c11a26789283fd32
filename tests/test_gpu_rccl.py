"""RCCL itself on the MI355X: the two-phase exchange's collectives at world size 1.

The N > 1 tests (test_gpu_multiproc.py, test_distributed.py) run their collectives over gloo --
two ranks share one GPU, which RCCL refuses. Here one process initialises the `nccl` backend
(RCCL on ROCm) at world size 1 and drives the exchange's collective step on device tensors
(flink_amd.exchange.exchange_grouped_columns: the all-to-all of the counts with the watermark
in-band, the one host read, the all-to-all of the packed partial rows -- exchange_partials skips
the collectives at world size 1, so the test calls the collective step directly) between the
HIP local and global operators, and the fired rows are compared with the single-phase oracle.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, KEYS, BATCH = 400_000, 20_000, 100_000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rccl_child(port, q):
    try:
        import torch
        import torch.distributed as dist

        import flink_amd as F
        from flink_amd.exchange import device_columns, exchange_grouped_columns, partition_columns_by_owner
        from tests.streams import make_stream
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        assert dist.get_backend() == "nccl"
        key, ts, val, _ = make_stream(N, KEYS, "f64", seed=77, jitter_ms=300)
        aggs = ("count_star", "count", "sum", "avg")
        w = F.tumbling(1000)
        local = F.WindowAggOperator(w, aggs=aggs, expected_keys=KEYS, local_partials=True)
        glob = F.WindowAggOperator(w, aggs=aggs, expected_keys=KEYS)
        out, mx, checks = [], -(1 << 63), 0

        def round_(wm):
            nonlocal checks
            local.process_watermarks([wm])
            r = local.collect_fired()
            cols = device_columns(r, aggs=tuple(range(int(r.num_aggs))), device=dev)
            outs, counts = partition_columns_by_owner(cols, 1)
            recv, sent, gwm = exchange_grouped_columns(outs, counts, watermark=wm)   # RCCL on device tensors
            assert gwm == wm and sent == 0
            assert all(c.is_cuda for c in recv) and len(recv) == len(outs)
            for a, b in zip(recv, outs):   # world size 1: every row comes back to its owner unchanged
                assert torch.equal(a, b)
            checks += 1
            glob.process_partials(*recv)
            out.append(glob.process_watermark(gwm))

        for lo in range(0, N, BATCH):
            hi = lo + BATCH
            local.process_batch(torch.from_numpy(key[lo:hi]).to(dev), torch.from_numpy(ts[lo:hi]).to(dev),
                                torch.from_numpy(val[lo:hi]).to(dev))
            mx = max(mx, int(ts[lo:hi].max()))
            round_(mx - 100 - 1)
        round_((1 << 63) - 1)
        rows = np.concatenate([x for x in out if len(x)])
        late = glob.num_late_records_dropped
        local.close()
        glob.close()
        torch.cuda.synchronize()
        dist.destroy_process_group()
        q.put((rows.tobytes(), rows.dtype.descr, late, checks, None))
    except Exception as e:
        import traceback
        q.put((None, None, 0, 0, traceback.format_exc() + repr(e)))


def test_rccl_world1_exchange_between_hip_operators(oracle_mod):
    import torch.multiprocessing as mp

    from tests.streams import make_stream
    O = oracle_mod
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_child, args=(_free_port(), q))
    p.start()
    b, descr, late, checks, err = q.get(timeout=240)
    p.join(timeout=60)
    assert err is None, err
    assert p.exitcode == 0
    assert checks == N // BATCH + 1
    got = np.frombuffer(b, dtype=np.dtype([tuple(x) for x in descr]))
    key, ts, val, _ = make_stream(N, KEYS, "f64", seed=77, jitter_ms=300)
    # the two-phase plan at one subtask (local -> global, the global's late rules per partial row)
    loc = O.OracleOperator(kind=O.TUMBLE, size=1000, val_type=O.VAL_F64, phase=O.PHASE_LOCAL)
    glo = O.OracleOperator(kind=O.TUMBLE, size=1000, val_type=O.VAL_F64, phase=O.PHASE_GLOBAL)
    exp, mx = [], -(1 << 63)
    for lo in range(0, N, BATCH):
        loc.process_batch(key[lo:lo + BATCH], ts[lo:lo + BATCH], val[lo:lo + BATCH])
        mx = max(mx, int(ts[lo:lo + BATCH].max()))
        loc.process_watermark(mx - 101)
        glo.process_partials(loc.take_rows())
        glo.process_watermark(mx - 101)
        exp.append(glo.take_rows())
    loc.process_watermark((1 << 63) - 1)
    glo.process_partials(loc.take_rows())
    glo.process_watermark((1 << 63) - 1)
    exp.append(glo.take_rows())
    e = np.concatenate(exp)
    assert late == glo.late_dropped
    loc.close()
    glo.close()
    g = got[np.lexsort((got["key"], got["window_end"]))]
    e = e[np.lexsort((e["key"], e["window_end"]))]
    assert len(g) == len(e), (len(g), len(e))
    for f, fe in (("key", "key"), ("window_end", "window_end"), ("count_star", "cnt_star"), ("count", "cnt_val")):
        assert np.array_equal(g[f], e[fe]), f
    ok = e["sum_null"] == 0
    a, bb = g["sum"][ok], e["sum_d"][ok]
    assert (np.abs(a - bb) <= 1e-9 * np.maximum(np.abs(a), np.abs(bb))).all()


def _capi_child(q):
    """world size 1 through the C-ABI: fg_comm_unique_id -> fg_comm_open -> bench.TwoPhase with
    the communicator (fg_comm_exchange_fired / _flushed into the global operator)"""
    try:
        import torch

        import bench as B
        import flink_amd as F
        from flink_amd.comm import Communicator, unique_id
        from tests.streams import make_stream
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        comm = Communicator(0, 1, 0, unique_id())
        # the column exchange alone: at world size 1 every row comes back unchanged, watermark as given
        cols = [torch.arange(1000, dtype=torch.int64, device=dev) * 7 + j for j in range(5)]
        got, wm = comm.exchange_columns(cols, watermark=123)
        assert wm == 123 and all(torch.equal(a, b) for a, b in zip(got, cols)) and comm.bytes_sent == 0
        empty, wm = comm.exchange_columns([c[:0] for c in cols], watermark=5)
        assert wm == 5 and all(e.numel() == 0 for e in empty)
        key, ts, val, _ = make_stream(N, KEYS, "f64", seed=78, jitter_ms=1200)
        aggs = ("count_star", "count", "sum", "avg")
        w = F.tumbling(1000)
        local = F.WindowAggOperator(w, aggs=aggs, expected_keys=KEYS, local_partials=True)
        glob = F.WindowAggOperator(w, aggs=aggs, expected_keys=KEYS)
        tp = B.TwoPhase(local, glob, dev, comm=comm, host_rows=True)
        out, mx = [], -(1 << 63)
        for bi, lo in enumerate(range(0, N, BATCH)):
            hi = lo + BATCH
            local.process_batch(torch.from_numpy(key[lo:hi]).to(dev), torch.from_numpy(ts[lo:hi]).to(dev),
                                torch.from_numpy(val[lo:hi]).to(dev))
            m0 = mx
            mx = max(mx, int(ts[lo:hi].max()))
            got, _ = tp.round([m0 - 101 if m0 > -(1 << 62) else mx - 900, mx - 501, mx - 101])
            out.append(got)
            if bi == 1:
                got, _, (img, twm) = tp.checkpoint()
                out.append(got)
                assert len(img["key"]) > 0
        rest, _ = tp.finish()
        out += rest
        rows = np.concatenate([x for x in out if x is not None and len(x)])
        late = tp.glob.num_late_records_dropped
        local.close()
        glob.close()
        comm.close()
        q.put((rows.tobytes(), rows.dtype.descr, late, None))
    except Exception as e:
        import traceback
        q.put((None, None, 0, traceback.format_exc() + repr(e)))


def test_capi_comm_world1_two_phase(oracle_mod):
    """fg_comm_* (the C-ABI's RCCL edge) at world size 1: bench.TwoPhase through the
    communicator -- three watermarks per batch to the local operator, a checkpoint whose local
    flush crosses the edge -- against the two-phase oracle on the same schedule."""
    import torch.multiprocessing as mp

    from tests.streams import make_stream
    O = oracle_mod
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_capi_child, args=(q,))
    p.start()
    b, descr, late, err = q.get(timeout=240)
    p.join(timeout=60)
    assert err is None, err
    assert p.exitcode == 0
    got = np.frombuffer(b, dtype=np.dtype([tuple(x) for x in descr]))
    key, ts, val, _ = make_stream(N, KEYS, "f64", seed=78, jitter_ms=1200)
    loc = O.OracleOperator(kind=O.TUMBLE, size=1000, val_type=O.VAL_F64, phase=O.PHASE_LOCAL)
    glo = O.OracleOperator(kind=O.TUMBLE, size=1000, val_type=O.VAL_F64, phase=O.PHASE_GLOBAL)
    exp, mx = [], -(1 << 63)
    for bi, lo in enumerate(range(0, N, BATCH)):
        loc.process_batch(key[lo:lo + BATCH], ts[lo:lo + BATCH], val[lo:lo + BATCH])
        m0 = mx
        mx = max(mx, int(ts[lo:lo + BATCH].max()))
        for wm in (m0 - 101 if m0 > -(1 << 62) else mx - 900, mx - 501, mx - 101):
            loc.process_watermark(wm)
            glo.process_partials(loc.take_rows())
            glo.process_watermark(wm)
            exp.append(glo.take_rows())
        if bi == 1:
            loc.prepare_snapshot()
            glo.process_partials(loc.take_rows())
            glo.prepare_snapshot()
            exp.append(glo.take_rows())
    loc.process_watermark((1 << 63) - 1)
    glo.process_partials(loc.take_rows())
    glo.process_watermark((1 << 63) - 1)
    exp.append(glo.take_rows())
    e = np.concatenate(exp)
    assert late == glo.late_dropped and late > 0
    loc.close()
    glo.close()
    g = got[np.lexsort((got["key"], got["window_end"]))]
    e = e[np.lexsort((e["key"], e["window_end"]))]
    assert len(g) == len(e), (len(g), len(e))
    for f, fe in (("key", "key"), ("window_end", "window_end"), ("count_star", "cnt_star"), ("count", "cnt_val")):
        assert np.array_equal(g[f], e[fe]), f
    ok = e["sum_null"] == 0
    a, bb = g["sum"][ok], e["sum_d"][ok]
    assert (np.abs(a - bb) <= 1e-9 * np.maximum(np.abs(a), np.abs(bb))).all()


def _rounds_child(q):
    """the fused subtask (flink_amd.two_phase) over the C-ABI's RCCL rounds at world size 1
    (fg_comm_round_begin / _exchange / _end on the edge thread), with a checkpoint aligned through
    the rounds' epoch"""
    try:
        import torch

        import flink_amd as F
        from flink_amd.comm import Communicator, unique_id
        from flink_amd.two_phase import CapiRounds, GpuPair, TwoPhaseSubtask
        from tests.streams import make_stream
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        comm = Communicator(0, 1, 0, unique_id())
        key, ts, val, _ = make_stream(N, KEYS, "f64", seed=79, jitter_ms=300)
        aggs = ("count_star", "count", "sum", "avg")
        w = F.tumbling(1000)
        local = F.WindowAggOperator(w, aggs=aggs, expected_keys=KEYS, local_partials=True)
        glob = F.WindowAggOperator(w, aggs=aggs, expected_keys=KEYS)
        sub = TwoPhaseSubtask(GpuPair(local, glob, dev), CapiRounds(comm), device=dev)
        mx, img = -(1 << 63), None
        for bi, lo in enumerate(range(0, N, BATCH)):
            hi = lo + BATCH
            sub.process_batch(torch.from_numpy(key[lo:hi]).to(dev), torch.from_numpy(ts[lo:hi]).to(dev),
                              torch.from_numpy(val[lo:hi]).to(dev))
            mx = max(mx, int(ts[lo:hi].max()))
            sub.process_watermark(mx - 401)
            sub.drain()
            if bi == 1:
                img, _ = sub.prepare_snapshot_pre_barrier(1)
        sub.end_input()
        rows = np.concatenate([r for k, r in sub.output if k == "rows"])
        assert img is not None and len(img["key"]) > 0 and sub.rounds_run > 2
        local.close()
        glob.close()
        comm.close()
        q.put((rows.tobytes(), rows.dtype.descr, None))
    except Exception as e:
        import traceback
        q.put((None, None, traceback.format_exc() + repr(e)))


def test_capi_rounds_world1_fused_subtask(oracle_mod):
    """the fused two-phase subtask's edge thread over fg_comm_round_* (ABI 16) at world size 1:
    its rows equal the single-phase operator's (no late record: jitter < delay)"""
    import torch.multiprocessing as mp

    from tests.streams import make_stream
    O = oracle_mod
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rounds_child, args=(q,))
    p.start()
    b, descr, err = q.get(timeout=240)
    p.join(timeout=60)
    assert err is None, err
    got = np.frombuffer(b, dtype=np.dtype([tuple(x) for x in descr]))
    key, ts, val, _ = make_stream(N, KEYS, "f64", seed=79, jitter_ms=300)
    op = O.OracleOperator(kind=O.TUMBLE, size=1000, val_type=O.VAL_F64)
    op.process_batch(key, ts, val)
    op.process_watermark((1 << 63) - 1)
    e = op.take_rows()
    assert op.late_dropped == 0
    op.close()
    g = got[np.lexsort((got["key"], got["window_end"]))]
    e = e[np.lexsort((e["key"], e["window_end"]))]
    assert len(g) == len(e), (len(g), len(e))
    for f, fe in (("key", "key"), ("window_end", "window_end"), ("count_star", "cnt_star"), ("count", "cnt_val")):
        assert np.array_equal(g[f], e[fe]), f
