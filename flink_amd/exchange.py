"""Key-group exchange between GPUs of one node (the keyBy shuffle).

Replaces the network edge KeyGroupStreamPartitioner.selectChannel
(SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:55-65) +
RecordWriter.emit (RT/io/network/api/writer/RecordWriter.java:101-128) for co-located
subtasks: every rank packs its source partition by owner subtask
(kg * parallelism / maxParallelism, KeyGroupRangeAssignment.java:124-127) on its GPU
(fg_partition_by_owner), then one RCCL all-to-all over xGMI delivers each owner its
records. The watermark is combined with an all-reduce(min), as StatusWatermarkValve
takes the minimum over input channels.
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


def global_watermark(local_wm: int, group=None, device=None) -> int:
    """min over subtasks (StatusWatermarkValve)."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return int(local_wm)
    t = torch.tensor([int(local_wm)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item())
