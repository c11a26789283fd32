"""Multi-rank path on CPU (gloo, world_size 2): key-group ownership, the all-to-all
exchange protocol of flink_amd.exchange, and the watermark min-combine. Every rank runs
the oracle operator on the records it owns; the union of the ranks' fired rows must
equal one operator over the whole stream (key-group sharding preserves per-key
semantics: KeyGroupRangeAssignment.java:63-77,124-127)."""
import os
import socket

import numpy as np
import pytest

WORLD = 2
MAXP = 128


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_q):
    import torch
    import torch.distributed as dist

    from flink_amd.exchange import exchange_partitioned, global_watermark
    from oracle import oracle as O
    from tests.streams import make_stream
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, keys, batch = 40_000, 3000, 5_000
    key, ts, val, _ = make_stream(n, keys, "i64", seed=1000 + rank, jitter_ms=50)
    op = O.OracleOperator(kind=O.TUMBLE, size=200, val_type=O.VAL_I64, count_star_index=0)
    rows = []
    received_kgs = set()
    mx = -(1 << 63)
    for lo in range(0, n, batch):
        hi = lo + batch
        k, t, v = key[lo:hi], ts[lo:hi], val[lo:hi]
        kg = O.key_groups_binaryrow(k, MAXP)
        owner = kg.astype(np.int64) * world // MAXP             # computeOperatorIndexForKeyGroup
        order = np.argsort(owner, kind="stable")
        counts = torch.from_numpy(np.bincount(owner, minlength=world).astype(np.int64))
        rk, rt, rv, _ = exchange_partitioned(torch.from_numpy(k[order]), torch.from_numpy(t[order]),
                                             torch.from_numpy(v[order]), counts)
        rk, rt, rv = rk.numpy(), rt.numpy(), rv.numpy()
        received_kgs.update(O.key_groups_binaryrow(rk, MAXP).tolist())
        op.process_batch(rk, rt, rv)
        mx = max(mx, int(t.max()))
        wm = global_watermark(mx - 60)
        op.process_watermark(wm)
        rows.append(op.take_rows())
    op.process_watermark((1 << 63) - 1)
    rows.append(op.take_rows())
    allrows = np.concatenate(rows)
    lo_kg, hi_kg = (rank * MAXP + world - 1) // world, ((rank + 1) * MAXP - 1) // world   # key-group range
    ok_range = all(lo_kg <= g <= hi_kg for g in received_kgs)
    out_q.put((rank, allrows.tobytes(), op.late_dropped, ok_range))
    dist.destroy_process_group()


def test_two_rank_exchange_matches_single_operator(oracle_mod):
    import torch.multiprocessing as mp

    from tests.streams import make_stream
    O = oracle_mod
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = np.concatenate([np.frombuffer(b, dtype=O.ROW_DTYPE) for _, b, _, _ in res])
    assert all(ok for *_, ok in res), "a rank received a key group it does not own"
    # reference: one operator over the interleaved stream (batch by batch, same watermarks)
    n, keys, batch = 40_000, 3000, 5_000
    streams = [make_stream(n, keys, "i64", seed=1000 + r, jitter_ms=50) for r in range(WORLD)]
    op = O.OracleOperator(kind=O.TUMBLE, size=200, val_type=O.VAL_I64, count_star_index=0)
    rows = []
    mxs = [-(1 << 63)] * WORLD
    for lo in range(0, n, batch):
        for r in range(WORLD):
            k, t, v, _ = streams[r]
            op.process_batch(k[lo:lo + batch], t[lo:lo + batch], v[lo:lo + batch])
            mxs[r] = max(mxs[r], int(t[lo:lo + batch].max()))
        op.process_watermark(min(mxs) - 60)     # StatusWatermarkValve: min over input channels
        rows.append(op.take_rows())
    op.process_watermark((1 << 63) - 1)
    rows.append(op.take_rows())
    exp = np.concatenate(rows)
    srt = lambda a: a[np.lexsort((a["key"], a["window_end"]))]
    g, e = srt(got), srt(exp)
    assert len(g) == len(e)
    for f in ("key", "window_end", "cnt_star", "sum_i"):
        assert np.array_equal(g[f], e[f]), f
    assert sum(l for _, _, l, _ in res) == op.late_dropped
