"""The fused two-phase subtask: local phase, keyBy edge and global phase in one operator, the edge
on a thread of its own (the Python mirror of java/.../gpu/GpuTwoPhaseWindowAggOperator.java).

The reference's two-phase plan (TwoStageOptimizedWindowAggregateRule.java:81-104) runs
LocalSlicingWindowAggOperator, a keyBy network edge (KeyGroupStreamPartitioner.selectChannel,
KeyGroupStreamPartitioner.java:55-65) and GlobalSlicingWindowAggOperator. On one node of GPUs the
edge is an RCCL all-to-all between the subtasks' GPUs (fg_comm), so one subtask holds the local and
the global operator of its GPU and the exchange is a collective every subtask must take part in --
the SAME number of times. Watermarks do not arrive in step at the subtasks (each source emits its
own), so the collective cannot be driven by them. Instead every subtask runs an edge thread that
exchanges in ROUNDS, forever, until every subtask has reached the end of its input:

  round (edge thread)     begin    [under the operator lock] the local operator's rows of the round --
                                   its uncollected async fires (FIRED), its whole buffer before a
                                   checkpoint barrier (FLUSHED), or nothing (IDLE) -- grouped by
                                   key-group owner, with this subtask's watermark and epoch
                          exchange [no lock: waits for the peers] one collective of (count, watermark,
                                   epoch, failure) per peer, then the rows
                          end      [under the lock] the received partial rows merged into the global
                                   operator (GlobalAggCombiner), the global advanced to the minimum
                                   watermark (StatusWatermarkValve) -- its fires are queued, and the
                                   task thread emits their rows (drain) before it forwards that
                                   watermark downstream

Checkpoints are aligned across the edge the way the reference aligns barriers on the global
operator's input channels: at its barrier a subtask flushes its local buffer into the next round
(LocalSlicingWindowAggOperator.prepareSnapshotPreBarrier :142-144) and advertises the checkpoint id as
its epoch; its task thread then waits until a round's minimum epoch reaches the id -- every subtask
has sent its pre-barrier rows -- and snapshots the global operator before the edge merges another
round. A subtask blocked at its barrier processes no post-barrier record, so no post-barrier row
reaches any image (the fast channels of an aligned checkpoint are blocked likewise).

Backends of a round: `CapiRounds` (fg_comm_round_begin / _exchange / _end, RCCL through the C-ABI) and
`TorchRounds` (torch.distributed: RCCL, or gloo through host memory for tests and rehearsals). The
subtask's operators are reached through a `pair` object (GpuPair for the HIP operators; tests plug
the oracle in the same way).
"""
from __future__ import annotations

import ctypes as C
import threading
import time

import numpy as np

from . import _lib as L

JMIN, JMAX = -(1 << 63), (1 << 63) - 1
FIRED, FLUSHED, IDLE = L.ROUND_FIRED, L.ROUND_FLUSHED, L.ROUND_IDLE


class RoundFailed(RuntimeError):
    """a round failed on some subtask: every subtask's edge stops with this error"""


class Round:
    __slots__ = ("min_watermark", "min_epoch", "rows_sent", "rows_received", "bytes_sent")

    def __init__(self, min_watermark, min_epoch, rows_sent, rows_received, bytes_sent):
        self.min_watermark, self.min_epoch = int(min_watermark), int(min_epoch)
        self.rows_sent, self.rows_received, self.bytes_sent = int(rows_sent), int(rows_received), int(bytes_sent)


class GpuPair:
    """The HIP local (FG_FLAG_LOCAL_PARTIALS) and global operators of one subtask."""

    def __init__(self, local, glob, device=None):
        import torch
        self.local, self.glob = local, glob
        self.device = device if device is not None else torch.device("cuda", 0)

    def local_batch(self, key, ts, val):
        self.local.process_batch(key, ts, val)

    def local_watermark(self, wm: int):
        self.local.process_watermarks([int(wm)])

    def local_rows(self, mode, world, max_parallelism, key_hash):
        """the round's local partial rows grouped by owner: (int64 device columns, counts[world])"""
        import torch

        from .exchange import device_columns, partition_columns_by_owner
        if mode == IDLE:
            return None, torch.zeros(world, dtype=torch.int64)
        r = self.local.collect_fired() if mode == FIRED else self.local.flush_partials(device_output=True)
        cols = device_columns(r, aggs=tuple(range(int(r.num_aggs))), device=self.device)
        outs, counts = partition_columns_by_owner(cols, world, max_parallelism, key_hash)
        torch.cuda.current_stream(self.device).synchronize()   # (the local's rows are read: it may fire again)
        return outs, counts

    def global_add(self, cols):
        if cols is not None and cols[0].numel():
            self.glob.process_partials(*cols)

    def global_advance(self, wm: int):
        self.glob.process_watermark(int(wm), device_output=True, wait=False)
        self._pending = True

    _pending = False

    def global_collect(self):
        """the rows of the global fires queued since the last collect (host), or None"""
        if not self._pending:
            return None
        self._pending = False
        return self.glob.collect_fired(host=True)

    def global_snapshot(self):
        self.glob.prepare_snapshot_pre_barrier()
        return self.glob.snapshot_state(copy=True)


class TorchRounds:
    """A round over torch.distributed (fg_comm_round semantics): ONE all-to-all of (count,
    watermark, epoch, columns << 1 | failed) per peer, one host read, ONE all-to-all of the rows
    packed [n, c]. via_cpu stages through host memory (gloo)."""

    def __init__(self, group=None, via_cpu=False, max_parallelism=128, key_hash=L.KEYHASH_BINARYROW_BIGINT):
        import torch.distributed as dist
        self.group, self.via_cpu = group, via_cpu
        self.maxp, self.key_hash = max_parallelism, key_hash
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._out = None
        self._recv = None
        self.bytes_sent = 0

    def begin(self, pair, mode, watermark, epoch):
        import torch
        self._err = None
        try:
            outs, counts = pair.local_rows(mode, self.world, self.maxp, self.key_hash)
        except Exception as e:   # (still takes part in the round: the peers learn of it)
            self._err = e
            outs, counts = None, torch.zeros(self.world, dtype=torch.int64)
        ncols = len(outs) if outs else 0
        n = int(outs[0].numel()) if outs else 0
        if outs and int(counts.sum()) != n:
            self._err, outs, counts = RoundFailed("owner partition lost rows"), None, torch.zeros(self.world, dtype=torch.int64)
        fail = 1 if self._err is not None else 0
        meta = torch.zeros((self.world, 4), dtype=torch.int64)
        meta[:, 0] = counts.cpu() if not fail else 0
        meta[:, 1] = int(watermark)
        meta[:, 2] = int(epoch)
        meta[:, 3] = ncols << 1 | fail
        self._meta = meta if self.via_cpu else meta.to(counts.device)
        self._out = None if fail or not outs else torch.stack(outs, dim=1).contiguous()

    def exchange(self) -> Round:
        import torch
        import torch.distributed as dist
        rmeta = torch.empty_like(self._meta)
        dist.all_to_all_single(rmeta, self._meta, group=self.group)
        ms, mr = self._meta.cpu(), rmeta.cpu()
        failed = [p for p in range(self.world) if int(mr[p, 3]) & 1]
        if failed:
            if self._err is not None:
                raise RoundFailed(f"this subtask's round failed: {self._err!r}")
            raise RoundFailed(f"subtask {failed[0]} failed its round (no rows moved on any subtask)")
        cols = {int(mr[p, 3]) >> 1 for p in range(self.world) if int(mr[p, 0]) > 0}
        if len(cols) > 1:
            raise RoundFailed("subtasks sent rows of different column counts")
        send, recv = ms[:, 0].tolist(), mr[:, 0].tolist()
        nc = cols.pop() if cols else 0
        self._recv = None
        if nc:
            packed = self._out if self._out is not None else torch.zeros((0, nc), dtype=torch.int64)
            if self.via_cpu:
                packed = packed.cpu()
            elif self._out is None:
                packed = packed.to(self._meta.device)
            out = torch.empty((sum(recv), nc), dtype=torch.int64, device=packed.device)
            dist.all_to_all_single(out, packed, output_split_sizes=recv, input_split_sizes=send, group=self.group)
            self._recv = out
        sent = 8 * nc * (sum(send) - send[self.rank])
        self.bytes_sent += sent
        return Round(int(mr[:, 1].min()), int(mr[:, 2].min()), sum(send), sum(recv), sent)

    def end(self, pair, device=None):
        if self._recv is None or self._recv.shape[0] == 0:
            return
        r = self._recv
        if device is not None and r.device != device:
            r = r.to(device)
        pair.global_add([c.contiguous() for c in r.unbind(1)])


class CapiRounds:
    """A round through the C-ABI (fg_comm_round_begin / _exchange / _end over RCCL): the pair's
    operators are HIP handles (GpuPair)."""

    def __init__(self, comm, max_parallelism=128, key_hash=L.KEYHASH_BINARYROW_BIGINT):
        self.comm, self.maxp, self.key_hash = comm, max_parallelism, key_hash
        self._lib = L.load()

    @property
    def bytes_sent(self):
        return self.comm.bytes_sent

    def begin(self, pair, mode, watermark, epoch):
        h = None if mode == IDLE else pair.local._h
        # (its failure is reported by exchange, on every rank)
        self._rc = self._lib.fg_comm_round_begin(self.comm._h, h, mode, self.key_hash, self.maxp, int(watermark),
                                                 int(epoch))

    def exchange(self) -> Round:
        r = L.FgRound()
        rc = self._lib.fg_comm_round_exchange(self.comm._h, C.byref(r))
        if rc:
            raise RoundFailed(self._lib.fg_comm_last_error(self.comm._h).decode(errors="replace"))
        return Round(r.min_watermark, r.min_epoch, r.rows_sent, r.rows_received, r.bytes_sent)

    def end(self, pair, device=None):
        rc = self._lib.fg_comm_round_end(self.comm._h, pair.glob._h)
        if rc:
            raise RoundFailed(self._lib.fg_comm_last_error(self.comm._h).decode(errors="replace"))


class TwoPhaseSubtask:
    """One subtask of the fused operator: the task thread's calls (records, watermarks, barriers,
    end of input, drain) and the edge thread's rounds, under one lock."""

    def __init__(self, pair, rounds, idle_sleep_s: float = 0.001, device=None):
        self.pair, self.rounds = pair, rounds
        self.idle_sleep_s, self.device = idle_sleep_s, device
        self.cv = threading.Condition()
        self.wm_local = JMIN       # the last watermark handed to the local operator
        self.dirty = False         # local fires since the last round
        self.flush_req = 0         # checkpoint id whose pre-barrier flush is requested
        self.sent_epoch = 0        # ... and the last one sent
        self.aligned = 0           # the last epoch every subtask has sent (a round's minimum)
        self.snap_done = 0         # the last aligned epoch this subtask has snapshotted
        self.glob_wm = JMIN        # the global operator's (combined) watermark
        self.forwarded = JMIN      # the watermark drain() last forwarded
        self.error = None
        self.rounds_run = 0
        self.output = []           # ("rows", numpy rows) and ("watermark", wm) in emission order
        self._thread = threading.Thread(target=self._edge, name="fg-edge", daemon=True)
        self._thread.start()

    # -- the task thread ---------------------------------------------------------------------------
    def _check(self):
        if self.error is not None:
            raise self.error

    def process_batch(self, key, ts, val):
        with self.cv:
            self._check()
            self.pair.local_batch(key, ts, val)

    def process_watermark(self, wm: int):
        with self.cv:
            self._check()
            if wm <= self.wm_local:
                return
            self.pair.local_watermark(wm)
            self.wm_local = int(wm)
            self.dirty = True

    def drain(self):
        """the mailbox action the edge posts: the global fires' rows emitted, then the combined
        watermark forwarded (rows always precede the watermark that fired them)"""
        with self.cv:
            self._check()
            self._drain_locked()

    def _drain_locked(self):
        rows = self.pair.global_collect()
        if rows is not None and len(rows):
            self.output.append(("rows", rows))
        if self.glob_wm > self.forwarded:
            self.forwarded = self.glob_wm
            self.output.append(("watermark", self.glob_wm))

    def prepare_snapshot_pre_barrier(self, checkpoint_id: int, timeout_s: float = 300.0):
        """the barrier of checkpoint `checkpoint_id` (ids increase): the local buffer goes out with
        the next round; once every subtask has sent its pre-barrier rows the global operator's rows
        are emitted and its image taken; returns (image, timer watermark)"""
        with self.cv:
            self._check()
            self.flush_req = int(checkpoint_id)
            self.cv.notify_all()
            if not self.cv.wait_for(lambda: self.aligned >= checkpoint_id or self.error is not None, timeout_s):
                raise TimeoutError(f"checkpoint {checkpoint_id} not aligned in {timeout_s} s")
            self._check()
            self._drain_locked()
            image = self.pair.global_snapshot()
            self.snap_done = int(checkpoint_id)
            self.cv.notify_all()
            return image

    def end_input(self, timeout_s: float = 300.0):
        """Long.MAX_VALUE: the edge runs until every subtask has ended; the last rows drained"""
        self.process_watermark(JMAX)
        self._thread.join(timeout_s)
        if self._thread.is_alive():
            raise TimeoutError("the edge did not finish")
        with self.cv:
            self._check()
            self._drain_locked()

    def close(self):
        with self.cv:
            if self.error is None and self._thread.is_alive():
                self.error = RuntimeError("closed")
            self.cv.notify_all()

    # -- the edge thread -----------------------------------------------------------------------------
    def _edge(self):
        try:
            while True:
                with self.cv:
                    if self.dirty:   # (fires before a flush: a barrier's flush follows in the next round)
                        mode, epoch = FIRED, self.sent_epoch
                    elif self.flush_req > self.sent_epoch:
                        mode, epoch = FLUSHED, self.flush_req
                    else:
                        mode, epoch = IDLE, self.sent_epoch
                    self.dirty = False
                    wm = self.wm_local
                    self.rounds.begin(self.pair, mode, wm, epoch)
                    if mode == FLUSHED:
                        self.sent_epoch = epoch
                r = self.rounds.exchange()   # (no lock: the task thread goes on meanwhile)
                with self.cv:
                    self.rounds_run += 1
                    self.rounds.end(self.pair, self.device)
                    if r.min_watermark > self.glob_wm:
                        self.pair.global_advance(r.min_watermark)
                        self.glob_wm = r.min_watermark
                    if r.min_epoch > self.aligned:
                        # every subtask has sent its pre-barrier rows: this subtask snapshots before
                        # another round merges (its task thread waits at the barrier)
                        self.aligned = r.min_epoch
                        self.cv.notify_all()
                        self.cv.wait_for(lambda: self.snap_done >= self.aligned or self.error is not None)
                        if self.error is not None:
                            return
                if r.min_watermark == JMAX:
                    return   # (every subtask has ended: the same round on all of them)
                if mode == IDLE and r.rows_received == 0:
                    time.sleep(self.idle_sleep_s)
        except BaseException as e:   # noqa: BLE001 (the task thread re-raises it)
            with self.cv:
                self.error = e if isinstance(e, Exception) else RuntimeError(repr(e))
                self.cv.notify_all()


def union_image_for(images, key_group_range, max_parallelism=128, key_groups=None):
    """Restore after a failover (or a rescale): the fused operator is not keyed, so its global
    images are union operator state -- every subtask reads all of them and keeps the entries of its
    own key groups (KeyGroupRangeAssignment). `key_groups(keys)` -> key groups (default: the device
    hash of BIGINT keys)."""
    cat = {c: np.concatenate([np.asarray(im[c]) for im, _ in images]) for c in images[0][0]}
    if key_groups is None:
        from .window_agg import key_groups as kg_dev
        kg = kg_dev(cat["key"], max_parallelism)
    else:
        kg = key_groups(cat["key"])
    lo, hi = key_group_range
    keep = (kg >= lo) & (kg <= hi)
    twm = min(w for _, w in images)
    return {c: v[keep] for c, v in cat.items()}, twm
