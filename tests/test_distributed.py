"""Multi-rank path on CPU (gloo, world_size 2): key-group ownership, the all-to-all
exchange protocol of flink_amd.exchange, and the watermark min-combine. Every rank runs
the oracle operator on the records it owns; the union of the ranks' fired rows must
equal one operator over the whole stream (key-group sharding preserves per-key
semantics: KeyGroupRangeAssignment.java:63-77,124-127)."""
import os
import socket

import numpy as np
import pytest

from flink_amd.keys import dict_kg_bits, key_group_of_id

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


# ---- two-phase plan over the exchange (TwoStageOptimizedWindowAggregateRule) ---------------
TP_N, TP_KEYS, TP_BATCH, TP_DELAY, TP_RATE = 60_000, 4000, 6_000, 100, 10
# kind -> (oracle kind, size, slide, jitter): the jitter exceeds the window so rows are late
TP_KINDS = {"tumble": (0, 500, 0, 900), "hop": (1, 1500, 500, 2500), "cumulate": (2, 2000, 500, 3000)}


def _two_phase_rank(rank, world, port, kind, out_q, columns=False):
    import torch
    import torch.distributed as dist

    from flink_amd.exchange import exchange_columns, exchange_grouped, exchange_grouped_columns, global_watermark
    from oracle import oracle as O
    from tests.streams import make_stream
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    k_, size, slide, jitter = TP_KINDS[kind]
    key, ts, val, isnull = make_stream(TP_N, TP_KEYS, "f64", seed=2000 + rank, jitter_ms=jitter, null_frac=0.1,
                                       rate_per_ms=TP_RATE)
    local = O.OracleOperator(kind=k_, size=size, slide=slide, phase=O.PHASE_LOCAL)
    glob = O.OracleOperator(kind=k_, size=size, slide=slide, phase=O.PHASE_GLOBAL)
    rows, sent_total = [], 0
    mx = -(1 << 63)

    def round_(local_wm):
        nonlocal sent_total
        # LocalSlicingWindowAggOperator.processWatermark: its flush emits partial accumulators
        local.process_watermark(local_wm)
        part = local.take_rows()
        # key-group routing of the partial rows (KeyGroupStreamPartitioner.selectChannel)
        owner = O.key_groups_binaryrow(part["key"], MAXP).astype(np.int64) * world // MAXP
        part = part[np.argsort(owner, kind="stable")]
        counts = torch.from_numpy(np.bincount(owner, minlength=world).astype(np.int64))
        packed = torch.from_numpy(part.view(np.int64).reshape(len(part), O.ROW_DTYPE.itemsize // 8).copy())
        gwm = None
        if columns == "inband":   # bench.py's form: the watermark travels with the counts
            rc, sent, gwm = exchange_grouped_columns([packed[:, j].contiguous() for j in range(packed.shape[1])],
                                                     counts, watermark=local_wm)
            recv = torch.stack(rc, dim=1) if rc else packed[:0]
        elif columns:   # one all-to-all per column
            rc, sent = exchange_columns([packed[:, j].contiguous() for j in range(packed.shape[1])], counts)
            recv = torch.stack(rc, dim=1) if rc else packed[:0]
        else:
            recv, sent = exchange_grouped(packed, counts)
        sent_total += sent
        got = np.ascontiguousarray(recv.numpy()).view(O.ROW_DTYPE).reshape(-1)
        glob.process_partials(got)
        # StatusWatermarkValve: the global operator's watermark is the min over its inputs
        glob.process_watermark(global_watermark(local_wm) if gwm is None else gwm)
        rows.append(glob.take_rows())

    for lo in range(0, TP_N, TP_BATCH):
        hi = lo + TP_BATCH
        local.process_batch(key[lo:hi], ts[lo:hi], val[lo:hi], isnull[lo:hi])
        mx = max(mx, int(ts[lo:hi].max()))
        round_(mx - TP_DELAY)
    round_((1 << 63) - 1)
    out_q.put((rank, np.concatenate(rows).tobytes(), glob.late_dropped, sent_total))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,columns", [("tumble", False), ("hop", False), ("cumulate", False),
                                          ("tumble", True), ("hop", True), ("tumble", "inband"),
                                          ("cumulate", "inband")])
def test_two_phase_exchange_matches_single_operator(oracle_mod, kind, columns):
    """Two ranks run the local phase on their source partitions, exchange the partial
    accumulator rows by key-group owner (flink_amd.exchange.exchange_grouped, or exchange_columns:
    the collective step of exchange_partials, one all-to-all per column; gloo here, RCCL on
    GPUs) and merge them in the owners' global
    operators, which fire at the min-combined watermark. The union of the global rows equals
    one single-phase operator over both partitions (late rows included: the jitter exceeds
    the watermark delay); late partial rows are counted once each, as in the reference's
    two-phase plan (LocalSlicingWindowAggOperator.java:113-134, GlobalAggCombiner.java:77-110)."""
    import torch.multiprocessing as mp

    from tests.streams import make_stream
    O = oracle_mod
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_two_phase_rank, args=(r, WORLD, port, kind, q, columns)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = np.concatenate([np.frombuffer(b, dtype=O.ROW_DTYPE) for _, b, _, _ in res])
    assert all(sent > 0 for *_, sent in res)
    k_, size, slide, jitter = TP_KINDS[kind]
    streams = [make_stream(TP_N, TP_KEYS, "f64", seed=2000 + r, jitter_ms=jitter, null_frac=0.1, rate_per_ms=TP_RATE)
               for r in range(WORLD)]
    op = O.OracleOperator(kind=k_, size=size, slide=slide)
    rows = []
    mxs = [-(1 << 63)] * WORLD
    for lo in range(0, TP_N, TP_BATCH):
        for r in range(WORLD):
            k, t, v, nl = streams[r]
            op.process_batch(k[lo:lo + TP_BATCH], t[lo:lo + TP_BATCH], v[lo:lo + TP_BATCH], nl[lo:lo + TP_BATCH])
            mxs[r] = max(mxs[r], int(t[lo:lo + TP_BATCH].max()))
        op.process_watermark(min(mxs) - TP_DELAY)
        rows.append(op.take_rows())
    op.process_watermark((1 << 63) - 1)
    rows.append(op.take_rows())
    exp = np.concatenate(rows)
    assert op.late_dropped > 0
    srt = lambda a: a[np.lexsort((a["key"], a["window_end"]))]
    g, e = srt(got), srt(exp)
    assert len(g) == len(e)
    for f in ("key", "window_start", "window_end", "cnt_star", "cnt_val", "sum_null"):
        assert np.array_equal(g[f], e[f]), f
    ok = e["sum_null"] == 0
    assert np.allclose(g["sum_d"][ok], e["sum_d"][ok], rtol=1e-9, atol=0)
    assert sum(late for _, _, late, _ in res) > 0


# ---- STRING keys over the two-phase exchange -------------------------------------------------
class HostKeyDict:
    """A dictionary of key rows with the KeyDictionary interface exchange_partials uses
    (locate / intern_rows), on the host: ids = ordinal << kg_bits | key group in THIS dictionary's
    first-seen order, so two ranks' ids for one key differ, as the GPU dictionaries' do."""

    def __init__(self, max_parallelism=MAXP):
        self.maxp = max_parallelism
        self.rows, self.ids = [], {}

    def intern_bytes(self, row: bytes) -> int:
        from oracle import oracle as O
        i = self.ids.get(row)
        if i is None:
            i = len(self.rows) << dict_kg_bits(self.maxp) | O.key_group_of_row(row, self.maxp)
            self.ids[row] = i
            self.rows.append(row)
        return i

    def row_of(self, i: int) -> bytes:
        return self.rows[i >> dict_kg_bits(self.maxp)]

    def locate(self, ids):
        import torch
        blob = b"".join(self.rows)
        starts = np.cumsum([0] + [len(r) for r in self.rows])
        ords = ids.numpy() >> dict_kg_bits(self.maxp)
        woff = torch.from_numpy((starts[ords] // 4).astype(np.int64))
        nw = torch.from_numpy(np.array([len(self.rows[o]) // 4 for o in ords], dtype=np.int64))
        return woff, nw, torch.from_numpy(np.frombuffer(blob or b"\0" * 4, dtype=np.int32).copy())

    def intern_rows(self, data, offsets, lengths):
        import torch
        b = data.numpy().tobytes()
        return torch.from_numpy(np.array([self.intern_bytes(b[o:o + n]) for o, n in
                                          zip(offsets.tolist(), lengths.tolist())], dtype=np.int64))


def _string_rows(key):
    from flink_amd.keys import key_row
    return [key_row([f"name-{int(k):05d}" + "x" * (int(k) % 13)], ["string"]) for k in key]


def _two_phase_strings_rank(rank, world, port, out_q):
    import torch
    import torch.distributed as dist

    from flink_amd.exchange import exchange_grouped_columns, global_watermark
    from oracle import oracle as O
    from tests.streams import make_stream
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    k_, size, slide, jitter = TP_KINDS["hop"]
    n = TP_N // 3
    key, ts, val, isnull = make_stream(n, 1500, "f64", seed=3000 + rank, jitter_ms=jitter, null_frac=0.1,
                                       rate_per_ms=TP_RATE)
    local_d, owner_d = HostKeyDict(), HostKeyDict()
    if rank == 1:   # first-seen order differs between the ranks: their local ids disagree
        for r in _string_rows(np.arange(1499, -1, -7)):
            local_d.intern_bytes(r)
    ids = np.array([local_d.intern_bytes(r) for r in _string_rows(key)], dtype=np.int64)
    local = O.OracleOperator(kind=k_, size=size, slide=slide, phase=O.PHASE_LOCAL)
    glob = O.OracleOperator(kind=k_, size=size, slide=slide, phase=O.PHASE_GLOBAL)
    rows = []
    mx = -(1 << 63)

    def round_(local_wm):
        local.process_watermark(local_wm)
        part = local.take_rows()
        kg = key_group_of_id(part["key"], MAXP).astype(np.int64)   # FG_KEYHASH_DICT_ID
        owner = kg * world // MAXP
        part = part[np.argsort(owner, kind="stable")]
        counts = torch.from_numpy(np.bincount(owner, minlength=world).astype(np.int64))
        words = part.view(np.int64).reshape(len(part), O.ROW_DTYPE.itemsize // 8)
        cols = [torch.from_numpy(np.ascontiguousarray(words[:, j])) for j in range(words.shape[1])]
        recv, _ = exchange_grouped_columns(cols, counts, key_rows=(local_d, owner_d))
        got = np.ascontiguousarray(torch.stack(recv, dim=1).numpy()).view(O.ROW_DTYPE).reshape(-1)
        glob.process_partials(got)
        glob.process_watermark(global_watermark(local_wm))
        r = glob.take_rows()
        rows.append([(owner_d.row_of(int(x["key"])), int(x["window_end"]), int(x["cnt_star"]), int(x["cnt_val"]),
                      float(x["sum_d"]), int(x["sum_null"])) for x in r])

    for lo in range(0, n, TP_BATCH):
        hi = lo + TP_BATCH
        local.process_batch(ids[lo:hi], ts[lo:hi], val[lo:hi], isnull[lo:hi])
        mx = max(mx, int(ts[lo:hi].max()))
        round_(mx - TP_DELAY)
    round_((1 << 63) - 1)
    out_q.put((rank, [x for r in rows for x in r], glob.late_dropped))
    dist.destroy_process_group()


def test_two_phase_string_keys_travel_as_key_rows(oracle_mod):
    """STRING keys (BinaryRowData key rows) over the two-phase exchange: each rank's local
    dictionary ids are its own (different first-seen orders), so partial rows carry their key
    rows' bytes and the owner interns them (exchange_partials' key_rows). The owners' fired rows,
    mapped back to key rows, equal one single-phase operator over both partitions."""
    import torch.multiprocessing as mp

    from tests.streams import make_stream
    O = oracle_mod
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_two_phase_strings_rank, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = sorted(x for _, rows, _ in res for x in rows)
    k_, size, slide, jitter = TP_KINDS["hop"]
    n = TP_N // 3
    streams = [make_stream(n, 1500, "f64", seed=3000 + r, jitter_ms=jitter, null_frac=0.1, rate_per_ms=TP_RATE)
               for r in range(WORLD)]
    d = HostKeyDict()
    op = O.OracleOperator(kind=k_, size=size, slide=slide)
    rows, mxs = [], [-(1 << 63)] * WORLD
    for lo in range(0, n, TP_BATCH):
        for r in range(WORLD):
            k, t, v, nl = streams[r]
            ids = np.array([d.intern_bytes(x) for x in _string_rows(k[lo:lo + TP_BATCH])], dtype=np.int64)
            op.process_batch(ids, t[lo:lo + TP_BATCH], v[lo:lo + TP_BATCH], nl[lo:lo + TP_BATCH])
            mxs[r] = max(mxs[r], int(t[lo:lo + TP_BATCH].max()))
        op.process_watermark(min(mxs) - TP_DELAY)
        rows.append(op.take_rows())
    op.process_watermark((1 << 63) - 1)
    rows.append(op.take_rows())
    exp = sorted((d.row_of(int(x["key"])), int(x["window_end"]), int(x["cnt_star"]), int(x["cnt_val"]),
                  float(x["sum_d"]), int(x["sum_null"])) for x in np.concatenate(rows))
    assert len(got) == len(exp)
    for a, b in zip(got, exp):
        assert a[:4] == b[:4] and a[5] == b[5], (a, b)
        assert a[5] or abs(a[4] - b[4]) <= 1e-9 * max(abs(a[4]), abs(b[4])), (a, b)
    # the global phase counts late PARTIAL rows (one per key and slice), as the reference's
    # two-phase plan does; the single-phase operator counts records
    assert op.late_dropped > 0 and sum(late for *_, late in res) > 0
