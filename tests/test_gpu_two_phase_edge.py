"""The fused two-phase subtask (flink_amd.two_phase.TwoPhaseSubtask, the mirror of
GpuTwoPhaseWindowAggOperator) on the HIP engine across PROCESSES: two ranks on device 0, each with
its HIP local (FG_FLAG_LOCAL_PARTIALS) and global operator and an edge thread exchanging rounds over
gloo (the same protocol fg_comm_round_* runs over RCCL on a multi-GPU node). The ranks' watermarks
arrive at different cadences, so only the rounds keep their collectives in step.

- TUMBLE and CUMULATE: the union of the global rows equals the single-phase oracle over both
  streams (no record is late: jitter < delay, so the rows do not depend on the rounds' timing);
- TUMBLE with a checkpoint (aligned across the edge) and a failover: the global images are union
  state -- each new subtask restores the entries of its key groups from BOTH images -- and the
  sources replay from the barrier: the rows emitted before the barrier plus the rows after the
  restore equal the oracle's, exactly once.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLD, MAXP = 2, 128
N, KEYS, BATCH, DELAY, JITTER, RATE = 600_000, 40_000, 50_000, 700, 500, 100
KINDS = {"tumble": ("tumble", 1000, 0), "cumulate": ("cumulate", 4000, 1000)}
CKPT_AFTER = 4
RANK_WAIT_S = 420


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stream(rank):
    from tests.streams import make_stream
    return make_stream(N, KEYS, "f64", seed=7000 + rank, jitter_ms=JITTER, rate_per_ms=RATE)[:3]


def _rank(rank, port, kind, ckpt, q):
    import faulthandler
    import sys
    faulthandler.enable(file=sys.stderr)
    faulthandler.dump_traceback_later(RANK_WAIT_S - 20, exit=True, file=sys.stderr)
    try:
        import datetime

        import torch
        import torch.distributed as dist

        import flink_amd as F
        from flink_amd.two_phase import GpuPair, TorchRounds, TwoPhaseSubtask, union_image_for
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD, timeout=datetime.timedelta(seconds=120))
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        k_, size, slide = KINDS[kind]
        w = F.tumbling(size) if k_ == "tumble" else F.cumulative(size, slide)
        kg = ((rank * MAXP + WORLD - 1) // WORLD, ((rank + 1) * MAXP - 1) // WORLD)
        aggs = ("count_star", "count", "sum", "avg")
        key, ts, val = _stream(rank)

        def subtask():
            local = F.WindowAggOperator(w, aggs=aggs, expected_keys=KEYS, buffer_records=1 << 20, local_partials=True)
            glob = F.WindowAggOperator(w, aggs=aggs, expected_keys=KEYS // WORLD + 1, buffer_records=1 << 20,
                                       key_group_range=kg)
            return TwoPhaseSubtask(GpuPair(local, glob, dev), TorchRounds(via_cpu=True), device=dev)

        def feed(sub, b0, b1, snap_at=None):
            """batches [b0, b1); rank 0 forwards a watermark after every batch, rank 1 after every
            other one; returns the image of the barrier after batch snap_at"""
            mx, image = -(1 << 63), None
            every = 1 if rank == 0 else 2
            for bi in range(b0, b1):
                lo, hi = bi * BATCH, (bi + 1) * BATCH
                sub.process_batch(torch.from_numpy(key[lo:hi]).to(dev), torch.from_numpy(ts[lo:hi]).to(dev),
                                  torch.from_numpy(val[lo:hi]).to(dev))
                mx = max(mx, int(ts[:hi].max()))
                if bi % every == every - 1:
                    sub.process_watermark(mx - DELAY - 1)
                sub.drain()
                if bi == snap_at:
                    image = sub.prepare_snapshot_pre_barrier(1)
                    before = sum(len(r) for kk, r in sub.output if kk == "rows")
            sub.end_input()
            rows = [r for kk, r in sub.output if kk == "rows"]
            rows = np.concatenate(rows) if rows else None
            wms = [x for kk, x in sub.output if kk == "watermark"]
            assert wms == sorted(wms) and wms[-1] == (1 << 63) - 1
            return rows, image, (before if image is not None else None)

        nb = N // BATCH
        sub = subtask()
        rows, image, before = feed(sub, 0, nb, CKPT_AFTER if ckpt else None)
        sub.pair.local.close()
        sub.pair.glob.close()
        rounds = sub.rounds_run
        after = None
        if ckpt:
            # failover: every subtask restarts from the checkpoint; its global restores the entries of
            # its key groups from the union of the images, the sources replay from the barrier
            imgs = [None] * WORLD
            dist.all_gather_object(imgs, image)
            restored, twm = union_image_for(imgs, kg, MAXP)
            sub2 = subtask()
            sub2.pair.glob.restore_state(restored, twm)
            after, _, _ = feed(sub2, CKPT_AFTER + 1, nb)
            sub2.pair.local.close()
            sub2.pair.glob.close()
        dist.barrier()
        dist.destroy_process_group()
        pack = lambda r: None if r is None else (r.tobytes(), r.dtype.descr)
        q.put((rank, pack(rows), before, pack(after), rounds, None))
    except Exception as e:   # reported to the parent
        import traceback
        q.put((rank, None, None, None, 0, traceback.format_exc() + repr(e)))


def _run(kind, ckpt):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, kind, ckpt, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(WORLD):
            res.append(q.get(timeout=RANK_WAIT_S))
            assert not res[-1][-1], res[-1][-1]
    finally:
        for p in procs:
            p.join(timeout=5 if len(res) < WORLD else 60)
            if p.is_alive():
                p.kill()
    return sorted(res)


def _oracle_rows(O, kind):
    k_, size, slide = KINDS[kind]
    op = O.OracleOperator(kind={"tumble": O.TUMBLE, "cumulate": O.CUMULATE}[k_], size=size, slide=slide,
                          val_type=O.VAL_F64)
    for r in range(WORLD):
        k, t, v = _stream(r)
        op.process_batch(k, t, v)
    op.process_watermark((1 << 63) - 1)
    e = op.take_rows()
    assert op.late_dropped == 0
    op.close()
    return e


def _unpack(p):
    b, descr = p
    return np.frombuffer(b, dtype=np.dtype([tuple(x) for x in descr]))


def _compare(g, e):
    g = g[np.lexsort((g["key"], g["window_end"]))]
    e = e[np.lexsort((e["key"], e["window_end"]))]
    assert len(g) == len(e), (len(g), len(e))
    for f, fe in (("key", "key"), ("window_start", "window_start"), ("window_end", "window_end"),
                  ("count_star", "cnt_star"), ("count", "cnt_val")):
        assert np.array_equal(g[f], e[fe]), f
    for f, fe in (("sum", "sum_d"), ("avg", "avg_d")):
        a, b = g[f], e[fe]
        assert (np.abs(a - b) <= 1e-9 * np.maximum(np.abs(a), np.abs(b))).all(), f


@pytest.mark.parametrize("kind", ["tumble", "cumulate"])
def test_fused_subtasks_with_unaligned_watermarks_match_oracle(oracle_mod, kind):
    res = _run(kind, ckpt=False)
    assert all(r[4] > 1 for r in res)
    got = np.concatenate([_unpack(r[1]) for r in res if r[1] is not None])
    _compare(got, _oracle_rows(oracle_mod, kind))


def test_fused_subtasks_checkpoint_failover_exactly_once(oracle_mod):
    res = _run("tumble", ckpt=True)
    full = np.concatenate([_unpack(r[1]) for r in res if r[1] is not None])
    e = _oracle_rows(oracle_mod, "tumble")
    _compare(full, e)   # the run without the failover
    # the committed output of the failover run: each subtask's rows before its barrier, then the
    # restored subtasks' rows
    parts = [_unpack(r[1])[:r[2]] for r in res] + [_unpack(r[3]) for r in res if r[3] is not None]
    _compare(np.concatenate(parts), e)
