"""The level-C operator's host policy in Python: micro-batching of records and held watermarks.

Mirrors java/.../gpu/GpuSlicingWindowAggOperator.java + GpuSlicingWindowProcessor.java (the JVM
shim, not compiled in this image) over flink_amd.WindowAggOperator, so that the policy a Flink
job runs is the one the GPU tests exercise:

- process_elements: records are staged on the host and handed to the engine (fg_add_batch) in
  micro-batches of `batch_records` (GpuSlicingWindowProcessor.processElement -> flushBatch);
- process_watermark (async): a watermark still held is released first; then the staged records
  go with an asynchronous advance (fg_advance_progress_async) and the watermark is held;
- a held watermark is released -- its fired rows collected (fg_collect_fired) and emitted, then
  the watermark forwarded -- at the first of: the next micro-batch handed to the engine, the next
  watermark, `max_hold_ms` of processing time after the hold began (on_processing_time: a
  processing-time callback in the JVM), a checkpoint (prepare_snapshot_pre_barrier), end of input.

So rows always precede the watermark that fired them (SlicingWindowOperator.java:207-210 emits
them inside processWatermark), and a watermark reaches downstream at most one watermark interval
or max_hold_ms late, however slowly records arrive. async_watermarks=False: every watermark
advances synchronously and is forwarded at once (the reference's timing).

`output` collects ("rows", numpy rows) and ("watermark", wm) events in emission order.
"""
from __future__ import annotations

import time

import numpy as np


class HeldWatermarkOperator:
    def __init__(self, op, batch_records: int = 1 << 20, async_watermarks: bool = True, max_hold_ms: float = 200.0,
                 clock=time.monotonic):
        self.op = op
        self.batch_records = int(batch_records)
        self.async_watermarks = async_watermarks
        self.max_hold_ms = max_hold_ms
        self.clock = clock
        self._k = np.empty(self.batch_records, dtype=np.int64)
        self._t = np.empty(self.batch_records, dtype=np.int64)
        self._v = None
        self.count = 0
        self.held = None          # the held watermark
        self.held_at = 0.0        # processing time its hold began (seconds)
        self.output = []

    # -- records ---------------------------------------------------------------------------------
    def process_elements(self, key, ts, val):
        """processElement for each record in order (host arrays)."""
        key, ts, val = np.asarray(key, np.int64), np.asarray(ts, np.int64), np.asarray(val)
        if self._v is None:
            self._v = np.empty(self.batch_records, dtype=val.dtype)
        i = 0
        while i < len(key):
            m = min(len(key) - i, self.batch_records - self.count)
            self._k[self.count:self.count + m] = key[i:i + m]
            self._t[self.count:self.count + m] = ts[i:i + m]
            self._v[self.count:self.count + m] = val[i:i + m]
            self.count += m
            i += m
            if self.count == self.batch_records:
                self._flush_batch()
                if self.held is not None:   # a micro-batch handed over: the fires overlap it
                    self._release()

    def _flush_batch(self):
        if self.count:
            n = self.count
            self.op.process_batch(self._k[:n].copy(), self._t[:n].copy(), self._v[:n].copy())
            self.count = 0

    # -- watermarks ------------------------------------------------------------------------------
    def process_watermark(self, wm: int):
        if not self.async_watermarks:
            self._flush_batch()
            rows = self.op.process_watermark(int(wm))
            if len(rows):
                self.output.append(("rows", rows))
            self.output.append(("watermark", int(wm)))
            return
        if self.held is not None:   # a watermark waits at most one watermark interval
            self._release()
        self._flush_batch()
        self.op.process_watermark(int(wm), device_output=True, wait=False)
        self.held = int(wm)
        self.held_at = self.clock()

    def on_processing_time(self, now=None):
        """the processing-time callback registered at the hold (GpuSlicingWindowAggOperator)"""
        now = self.clock() if now is None else now
        if self.held is not None and (now - self.held_at) * 1e3 >= self.max_hold_ms:
            self._release()

    def _release(self):
        wm, self.held = self.held, None
        rows = self.op.collect_fired(host=True)
        if len(rows):
            self.output.append(("rows", rows))
        self.output.append(("watermark", wm))

    # -- checkpoint / end ------------------------------------------------------------------------
    def prepare_snapshot_pre_barrier(self):
        if self.held is not None:
            self._release()
        self._flush_batch()
        self.op.prepare_snapshot_pre_barrier()

    def end_input(self):
        if self.held is not None:
            self._release()
        self._flush_batch()
