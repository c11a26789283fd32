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
