"""The N > 1 path across PROCESSES on the HIP engine: two ranks (one process each, both on
device 0 -- the topology of scripts/rehearse_2rank.sh; the driver's 8-GPU node runs the same
code one rank per GPU over RCCL), collectives over gloo staged through host memory.

Each rank runs, exactly as bench.py's N > 1 path (partials_round) does: the HIP local operator
(LocalSlicingWindowAggOperator + LocalAggCombiner, FG_FLAG_LOCAL_PARTIALS) on its own source
partition, fg_partition_columns_by_owner + flink_amd.exchange.exchange_partials (one packed
all-to-all per watermark, the watermarks min-combined in-band with the counts:
StatusWatermarkValve) and the HIP global operator (GlobalAggCombiner) over the key groups it
owns, whose fire is asynchronous and collected in the next round before its partials merge.
The union of both ranks' fired rows must equal the single-phase oracle over both partitions,
late rows included, and the ranks' late-drop counts (per partial row, in the global phase)
must sum to the two-phase oracle's; the STRING-key variant interns key rows in per-rank GPU
dictionaries whose ids disagree, and ships the key rows with the partial rows
(exchange_partials key_rows).
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLD, MAXP = 2, 128
N, KEYS, BATCH, DELAY, JITTER = 1_000_000, 50_000, 100_000, 200, 1500
KINDS = {"tumble": ("tumble", 1000, 0), "hop": ("hop", 3000, 1000)}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _string_rows_u8(key):
    """32-B STRING key rows 'user%08x' as bench.py's string_key_rows writes them (host)."""
    import torch

    import bench
    return bench.string_key_rows(torch.from_numpy(key)).view(torch.uint8).reshape(-1)


def _rank(rank, port, kind, strings, q):
    try:
        import torch
        import torch.distributed as dist

        import flink_amd as F
        from flink_amd.exchange import device_columns, exchange_partials
        from tests.streams import make_stream
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        k_, size, slide = KINDS[kind]
        w = F.tumbling(size) if k_ == "tumble" else F.hopping(size, slide)
        key, ts, val, _ = make_stream(N, KEYS, "f64", seed=4000 + rank, jitter_ms=JITTER)
        kg_lo, kg_hi = (rank * MAXP + WORLD - 1) // WORLD, ((rank + 1) * MAXP - 1) // WORLD
        local = F.WindowAggOperator(w, aggs=("count_star", "count", "sum", "avg"), expected_keys=KEYS,
                                    buffer_records=1 << 20, local_partials=True)
        glob = F.WindowAggOperator(w, aggs=("count_star", "count", "sum", "avg"), expected_keys=KEYS // WORLD + 1,
                                   buffer_records=1 << 20, key_group_range=(kg_lo, kg_hi))
        from flink_amd import _lib as FL
        kd = ko = None
        key_hash = FL.KEYHASH_BINARYROW_BIGINT
        if strings:
            kd, ko = F.KeyDictionary(expected_keys=KEYS), F.KeyDictionary(expected_keys=KEYS)
            key_hash = FL.KEYHASH_DICT_ID
            if rank == 1:   # another first-seen order: this rank's ids differ from rank 0's
                warm = np.arange(KEYS - 1, -1, -3, dtype=np.int64)
                rows = _string_rows_u8(warm).to(dev)
                kd.intern(packed=(rows, torch.arange(len(warm), device=dev) * 32,
                                  torch.full((len(warm),), 32, dtype=torch.int32, device=dev)), key_groups=False)
        out, mx = [], -(1 << 63)
        held = [False]

        def collect():
            g = glob.collect_fired(host=True)
            held[0] = False
            if strings and len(g):   # owner ids -> the key rows' strings
                g = g.copy()
                names = [int(bytes(rw[16:28]).decode()[4:], 16) for rw in ko.lookup(g["key"])]
                g["key"] = np.array(names, dtype=np.int64)
            out.append(g)

        def round_(wm):
            r = local.process_watermark(wm, device_output=True)
            cols = device_columns(r, aggs=(0, 1, 2), device=dev)
            recv, _, gwm = exchange_partials(cols, max_parallelism=MAXP, key_hash=key_hash, via_cpu=True,
                                             key_rows=(kd, ko) if strings else None, watermark=wm)
            if held[0]:   # the previous round's global fires, before this round's partials merge
                collect()
            glob.process_partials(*recv)
            glob.process_watermark(gwm, device_output=True, wait=False)
            held[0] = True

        for lo in range(0, N, BATCH):
            hi = lo + BATCH
            if strings:
                rows = _string_rows_u8(key[lo:hi]).to(dev)
                k, _ = kd.intern(packed=(rows, torch.arange(hi - lo, device=dev) * 32,
                                         torch.full((hi - lo,), 32, dtype=torch.int32, device=dev)), key_groups=False)
            else:
                k = torch.from_numpy(key[lo:hi]).to(dev)
            local.process_batch(k, torch.from_numpy(ts[lo:hi]).to(dev), torch.from_numpy(val[lo:hi]).to(dev))
            mx = max(mx, int(ts[lo:hi].max()))
            round_(mx - DELAY - 1)
        round_((1 << 63) - 1)
        collect()
        rows = np.concatenate([x for x in out if len(x)]) if any(len(x) for x in out) else None
        late = glob.num_late_records_dropped
        for o in (local, glob, kd, ko):
            if o is not None:
                o.close()
        torch.cuda.synchronize()
        dist.destroy_process_group()
        q.put((rank, None if rows is None else rows.tobytes(), None if rows is None else rows.dtype.descr, late, None))
    except Exception as e:   # reported to the parent
        import traceback
        q.put((rank, None, None, 0, traceback.format_exc() + repr(e)))


@pytest.mark.parametrize("kind,strings", [("tumble", False), ("hop", False), ("tumble", True)])
def test_two_processes_two_phase_hip_path_matches_oracle(oracle_mod, kind, strings):
    import torch.multiprocessing as mp

    from tests.streams import make_stream
    O = oracle_mod
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, kind, strings, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
    errs = [e for *_, e in res if e]
    assert not errs, errs[0]
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    dt = np.dtype([tuple(x) for x in res[0][2]])
    got = np.concatenate([np.frombuffer(b, dtype=dt) for _, b, _, _, _ in res if b is not None])
    # the single-phase oracle over both partitions, batch by batch at the min watermark
    k_, size, slide = KINDS[kind]
    streams = [make_stream(N, KEYS, "f64", seed=4000 + r, jitter_ms=JITTER) for r in range(WORLD)]
    o = O.OracleOperator(kind=O.TUMBLE if k_ == "tumble" else O.HOP, size=size, slide=slide, val_type=O.VAL_F64)
    exp, mxs = [], [-(1 << 63)] * WORLD
    for lo in range(0, N, BATCH):
        for r in range(WORLD):
            k, t, v, _ = streams[r]
            o.process_batch(k[lo:lo + BATCH], t[lo:lo + BATCH], v[lo:lo + BATCH])
            mxs[r] = max(mxs[r], int(t[lo:lo + BATCH].max()))
        o.process_watermark(min(mxs) - DELAY - 1)
        exp.append(o.take_rows())
    o.process_watermark((1 << 63) - 1)
    exp.append(o.take_rows())
    e = np.concatenate(exp)
    # the two-phase oracle: each rank's local phase at its own watermark, its partial rows routed
    # by key group to the owners' global phase, which fires at the min over the ranks -- late
    # drops are counted there, per partial row (GlobalAggCombiner over the sliced assigner)
    okind = O.TUMBLE if k_ == "tumble" else O.HOP
    loc = [O.OracleOperator(kind=okind, size=size, slide=slide, val_type=O.VAL_F64, phase=O.PHASE_LOCAL)
           for _ in range(WORLD)]
    glo = [O.OracleOperator(kind=okind, size=size, slide=slide, val_type=O.VAL_F64, phase=O.PHASE_GLOBAL)
           for _ in range(WORLD)]
    mxs = [-(1 << 63)] * WORLD

    def route(wms):
        for r in range(WORLD):
            loc[r].process_watermark(wms[r])
            p = loc[r].take_rows()
            owner = O.key_groups_binaryrow(p["key"], MAXP).astype(np.int64) * WORLD // MAXP
            for d in range(WORLD):
                glo[d].process_partials(p[owner == d])
        for d in range(WORLD):
            glo[d].process_watermark(min(wms))

    for lo in range(0, N, BATCH):
        wms = []
        for r in range(WORLD):
            k, t, v, _ = streams[r]
            loc[r].process_batch(k[lo:lo + BATCH], t[lo:lo + BATCH], v[lo:lo + BATCH])
            mxs[r] = max(mxs[r], int(t[lo:lo + BATCH].max()))
            wms.append(mxs[r] - DELAY - 1)
        route(wms)
    route([(1 << 63) - 1] * WORLD)
    late_got = sum(x[3] for x in res)
    late_exp = sum(g.late_dropped for g in glo)
    assert late_got == late_exp, (late_got, late_exp)
    for x in loc + glo:
        x.close()
    if k_ == "tumble":
        # hop: a record is dropped only once its slice's LAST window fired (sliceEnd + size -
        # slide - 1 <= wm), i.e. ~2 s behind the watermark -- beyond this stream's 1.5 s jitter;
        # its late records are merged into fired-slice state instead (a2)
        assert o.late_dropped > 0, "the stream should hold late records"
    g = got[np.lexsort((got["key"], got["window_end"]))]
    e = e[np.lexsort((e["key"], e["window_end"]))]
    assert len(g) == len(e), (len(g), len(e))
    for f, fe in (("key", "key"), ("window_start", "window_start"), ("window_end", "window_end"),
                  ("count_star", "cnt_star"), ("count", "cnt_val")):
        assert np.array_equal(g[f], e[fe]), f
    ok = e["sum_null"] == 0
    assert np.array_equal(g["sum_null"], e["sum_null"] != 0)
    for f, fe in (("sum", "sum_d"), ("avg", "avg_d")):
        a, b = g[f][ok], e[fe][ok]
        assert (np.abs(a - b) <= 1e-9 * np.maximum(np.abs(a), np.abs(b))).all(), f
