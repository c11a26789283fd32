"""Key-group exchange between GPUs of one node (the keyBy shuffle).

Replaces the network edge KeyGroupStreamPartitioner.selectChannel
(SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:55-65) +
RecordWriter.emit (RT/io/network/api/writer/RecordWriter.java:101-128) for co-located
subtasks: every rank packs its source partition by owner subtask
(kg * parallelism / maxParallelism, KeyGroupRangeAssignment.java:124-127) on its GPU
(fg_partition_by_owner), then one RCCL all-to-all over xGMI delivers each owner its
records. The watermark is combined with an all-reduce(min), as StatusWatermarkValve
takes the minimum over input channels.

Two-phase form (TwoStageOptimizedWindowAggregateRule.java:81-104): what crosses the
exchange is the local phase's partial accumulator rows (LocalAggCombiner output: key,
slice_end, COUNT(*), COUNT(v), SUM) instead of raw records -- at most one row per (key,
slice) per source instead of one per record (exchange_partials).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L


def partition_by_owner(key: torch.Tensor, rowtime: torch.Tensor, val: torch.Tensor | None, parallelism: int,
                       max_parallelism: int = 128, key_hash: int = L.KEYHASH_BINARYROW_BIGINT, stream=None):
    """Reorder a device batch by destination subtask. Returns (key, rowtime, val, counts[parallelism])."""
    lib = L.load()
    n = key.numel()
    dev = key.device
    ok = torch.empty_like(key)
    ot = torch.empty_like(rowtime)
    ov = torch.empty_like(val) if val is not None else None
    counts = torch.empty(parallelism, dtype=torch.int64, device=dev)
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    rc = lib.fg_partition_by_owner(dev.index or 0, C.c_void_p(s), n, key.data_ptr(), rowtime.data_ptr(),
                                   val.data_ptr() if val is not None else None, key_hash, max_parallelism,
                                   parallelism, ok.data_ptr(), ot.data_ptr(),
                                   ov.data_ptr() if ov is not None else None, counts.data_ptr())
    L.check(rc)
    return ok, ot, ov, counts


def exchange(key, rowtime, val, group=None, max_parallelism: int = 128,
             key_hash: int = L.KEYHASH_BINARYROW_BIGINT):
    """All-to-all of a source partition to the key-group owners (one rank per subtask).

    Returns this rank's received (key, rowtime, val) and the bytes it sent to peers."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    ok, ot, ov, counts = partition_by_owner(key, rowtime, val, world, max_parallelism, key_hash)
    if world == 1:
        return ok, ot, ov, 0
    return exchange_partitioned(ok, ot, ov, counts, group)


def exchange_partitioned(ok, ot, ov, counts, group=None):
    """The collective step alone: columns already grouped by destination rank with
    `counts[d]` records for rank d. Works on any backend (RCCL on GPUs, gloo on CPU)."""
    import torch.distributed as dist
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    send = counts.cpu().tolist()
    recv = recv_counts.cpu().tolist()
    total = sum(recv)
    cols = [ok, ot] + ([ov] if ov is not None else [])
    # one all-to-all for all columns: pack [key | rowtime | val] per destination
    packed = torch.stack(cols, dim=1).contiguous()             # [n, ncol]
    out = torch.empty((total, len(cols)), dtype=packed.dtype, device=packed.device)
    dist.all_to_all_single(out, packed, output_split_sizes=recv, input_split_sizes=send, group=group)
    rk = out[:, 0].contiguous()
    rt = out[:, 1].contiguous()
    rv = out[:, 2].contiguous() if ov is not None else None
    rank = dist.get_rank(group)
    sent_bytes = 8 * len(cols) * (sum(send) - send[rank])
    return rk, rt, rv, sent_bytes


class _DeviceColumn:
    """Zero-copy view of an engine-owned device column (int64[n]) for torch.as_tensor."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i8", "data": (int(ptr or 0), False),
                                         "version": 2}


def device_columns(rows, names=("key", "window_end"), aggs=(0, 1, 2), device=None):
    """int64 tensor views of an FgRows returned with device_output=True (valid until the
    next call on the operator)."""
    n = int(rows.n)
    out = [torch.as_tensor(_DeviceColumn(getattr(rows, nm), n), device=device) for nm in names]
    out += [torch.as_tensor(_DeviceColumn(rows.agg[a], n), device=device) for a in aggs]
    return out


def partition_columns_by_owner(cols, parallelism: int, max_parallelism: int = 128,
                               key_hash: int = L.KEYHASH_BINARYROW_BIGINT, stream=None):
    """Reorder int64 device columns (cols[0] = key) by destination subtask.
    Returns (reordered columns, counts[parallelism])."""
    lib = L.load()
    n = cols[0].numel()
    dev = cols[0].device
    outs = [torch.empty_like(c) for c in cols]
    counts = torch.empty(parallelism, dtype=torch.int64, device=dev)
    if n == 0:
        counts.zero_()
        return outs, counts
    k = len(cols)
    ins = (C.c_void_p * k)(*[c.data_ptr() for c in cols])
    ous = (C.c_void_p * k)(*[o.data_ptr() for o in outs])
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    L.check(lib.fg_partition_columns_by_owner(dev.index or 0, C.c_void_p(s), n, k, ins, key_hash, max_parallelism,
                                              parallelism, ous, counts.data_ptr()))
    return outs, counts


def exchange_partials(cols, group=None, max_parallelism: int = 128, key_hash: int = L.KEYHASH_BINARYROW_BIGINT,
                      via_cpu: bool = False, key_rows=None, watermark=None):
    """Key-group exchange of partial accumulator rows (int64 device columns, key first).
    Returns the received columns and the bytes this rank sent to peers -- and, given this
    rank's `watermark`, the minimum over all ranks (StatusWatermarkValve) as a third value.

    Per call: the owner partition (a device counting sort), ONE all-to-all of the per-peer
    counts with the watermark in-band, ONE host read of them (the split sizes of the next
    collective, and the combined watermark: no separate all-reduce and no second host read),
    ONE all-to-all of the rows packed [n, c] (and, with key_rows, one of the key rows' words).
    The host read stays because the receiving fg_add_partials takes its row count on the host
    (and RCCL's all-to-all its split sizes); a fixed per-peer capacity would need a bound every
    rank agrees on beforehand -- world x the rows on the wire, or one more collective per round.

    key_rows = (local, owner) dictionaries (flink_amd.keys.KeyDictionary, or any objects with
    the same `locate` / `intern_rows` methods): the key column holds ids of this rank's `local`
    dictionary, which mean nothing on another rank, so each partial row travels with its key
    row's bytes -- as the reference's LocalAggCombiner emits the key BinaryRowData itself
    (LocalAggCombiner.java:100-106) -- and the owner interns them into its `owner` dictionary:
    the received key column holds owner ids. Routing is by the id's key group, which is the key
    row's (FG_KEYHASH_DICT_ID: computed from the bytes, the same on every rank).

    via_cpu stages the collectives through host memory (gloo; for rehearsing N > 1 on one
    device, and the CPU tests)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if key_rows is not None:
        key_hash = L.KEYHASH_DICT_ID
    outs, counts = partition_columns_by_owner(cols, world, max_parallelism, key_hash)
    if world == 1 and key_rows is None:
        return (outs, 0) if watermark is None else (outs, 0, int(watermark))
    return exchange_grouped_columns(outs, counts, group, via_cpu=via_cpu, key_rows=key_rows, watermark=watermark)


def exchange_grouped_columns(outs, counts, group=None, via_cpu: bool = False, key_rows=None, watermark=None):
    """The collective step of exchange_partials: int64 columns already grouped by destination
    rank (counts[d] rows for rank d; device tensors, or host tensors with gloo). With
    `watermark`, it travels in-band with the counts and the minimum over the ranks is returned
    as a third value."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    cols = outs
    words = None
    meta = [counts]
    if key_rows is not None:
        local, owner = key_rows
        woff, nw, arena = local.locate(outs[0])          # the key rows of the local ids
        ends = torch.cumsum(counts, 0)
        cw = torch.cumsum(nw, 0)
        at = torch.cat([torch.zeros(1, dtype=cw.dtype, device=cw.device), cw])
        wcounts = at[ends] - at[torch.cat([torch.zeros(1, dtype=ends.dtype, device=ends.device), ends[:-1]])]
        outs = outs + [nw]                                # row lengths (words) travel as a column
        meta.append(wcounts)
    if watermark is not None:                             # the same value to every peer
        meta.append(torch.full_like(counts, int(watermark)))
    counts_all = torch.stack(meta, dim=1)                 # [world, 1 + key_rows + watermark]
    packed = torch.stack(outs, dim=1)                     # [n, c]: one collective for every column
    if via_cpu:
        packed, counts_all = packed.cpu(), counts_all.cpu()
    recv_counts = torch.empty_like(counts_all)
    dist.all_to_all_single(recv_counts, counts_all, group=group)
    sc, rc = counts_all.cpu(), recv_counts.cpu()          # the one host read per exchange
    send, recv = sc[:, 0].tolist(), rc[:, 0].tolist()
    wm_min = int(rc[:, -1].min()) if watermark is not None else None
    out = torch.empty((sum(recv), packed.shape[1]), dtype=packed.dtype, device=packed.device)
    dist.all_to_all_single(out, packed, output_split_sizes=recv, input_split_sizes=send, group=group)
    rank = dist.get_rank(group)
    sent_bytes = 8 * packed.shape[1] * (sum(send) - send[rank])
    if key_rows is not None:
        wsend, wrecv = sc[:, 1].tolist(), rc[:, 1].tolist()
        total = sum(wsend)
        # word index of every row's bytes in the arena: row i's words woff[i] .. woff[i] + nw[i]
        rep = torch.repeat_interleave(torch.arange(len(nw), device=nw.device), nw, output_size=total)
        first = torch.cumsum(nw, 0) - nw
        idx = woff[rep] + (torch.arange(total, device=nw.device) - first[rep])
        words = arena[idx]
        if via_cpu:
            words = words.cpu()
        rwords = torch.empty(sum(wrecv), dtype=words.dtype, device=words.device)
        dist.all_to_all_single(rwords, words, output_split_sizes=wrecv, input_split_sizes=wsend, group=group)
        sent_bytes += 4 * (total - wsend[rank])
    cols_out = list(out.unbind(1))
    if via_cpu:
        dev = cols[0].device
        cols_out = [c.to(dev) for c in cols_out]
        if words is not None:
            rwords = rwords.to(dev)
    cols_out = [c.contiguous() for c in cols_out]
    if key_rows is not None:
        rlen = cols_out.pop() * 4                          # bytes per received row
        roff = torch.cumsum(rlen, 0) - rlen
        cols_out[0] = owner.intern_rows(rwords.view(torch.uint8), roff, rlen.to(torch.int32))
    return (cols_out, sent_bytes) if watermark is None else (cols_out, sent_bytes, wm_min)


def exchange_columns(cols, counts, group=None):
    """The collective step of the partial-row exchange on separate columns: `cols` (int64, the
    same length) grouped by destination rank, counts[d] rows for rank d. One all-to-all of the
    counts, then one per column. Returns the received columns and the bytes sent to peers."""
    import torch.distributed as dist
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    send = counts.cpu().tolist()
    recv = recv_counts.cpu().tolist()
    total = sum(recv)
    out = []
    for c in cols:
        r = torch.empty(total, dtype=c.dtype, device=c.device)
        dist.all_to_all_single(r, c, output_split_sizes=recv, input_split_sizes=send, group=group)
        out.append(r)
    rank = dist.get_rank(group)
    return out, 8 * len(cols) * (sum(send) - send[rank])


def exchange_grouped(packed, counts, group=None):
    """The collective step of the partial-row exchange: `packed` [n, c] int64 rows grouped
    by destination rank, counts[d] rows for rank d. One all-to-all of the counts, one of the
    rows (RCCL on device tensors, gloo on host tensors). Returns the received rows and the
    bytes sent to peers."""
    import torch.distributed as dist
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    send = counts.cpu().tolist()
    recv = recv_counts.cpu().tolist()
    out = torch.empty((sum(recv), packed.shape[1]), dtype=packed.dtype, device=packed.device)
    dist.all_to_all_single(out, packed, output_split_sizes=recv, input_split_sizes=send, group=group)
    rank = dist.get_rank(group)
    return out, 8 * packed.shape[1] * (sum(send) - send[rank])


def global_watermark(local_wm: int, group=None, device=None) -> int:
    """min over subtasks (StatusWatermarkValve)."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return int(local_wm)
    if dist.get_backend(group) == "gloo":
        device = "cpu"
    t = torch.tensor([int(local_wm)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item())
