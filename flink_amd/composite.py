"""Queries with several value accumulators (e.g. SUM, MIN and MAX of one column).

An engine handle keeps the SUM-family, MIN and MAX accumulators of one (key, slice) side by
side (value slots), so ``SELECT COUNT(*), SUM(v), MIN(v), MAX(v) ... GROUP BY TUMBLE(...)`` is
one handle and one staging pass (window_agg_operator). CompositeWindowAggOperator is the
split form: one handle per accumulator kind, each fed the same batches, the fired rows joined
on (window_end, key) -- what the local phase of a two-phase plan needs (one partial
accumulator per row), and a cross-check of the value slots in the tests. Every handle fires the same (key, window) set: emission is decided by
COUNT(*) / the presence of state, which all of them keep (the reference's generated
NamespaceAggsHandleFunction holds all accumulators of one (key, window) in one row,
AggsHandlerCodeGenerator.scala:578-700; the join restores that row). This is the
planner-side split INTEGRATION.md describes, mirrored here.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .window_agg import AGG_NAMES, AGGS, WindowAggOperator

_SUM_FAMILY = (L.AGG_SUM, L.AGG_AVG, L.AGG_SUM0)


def accumulator_groups(aggs):
    """Split an aggregate list into per-handle lists: the SUM family with the counts, then
    MIN and MAX each with COUNT(*) (HOP needs a COUNT(*) in every handle)."""
    codes = [AGGS[a] if isinstance(a, str) else int(a) for a in aggs]
    counts = [L.AGG_COUNT_STAR] + [c for c in codes if c == L.AGG_COUNT]
    groups = []
    fam = [c for c in codes if c in _SUM_FAMILY]
    if fam or not any(c in (L.AGG_MIN, L.AGG_MAX) for c in codes):
        groups.append(tuple(dict.fromkeys(counts + fam)))
    for op in (L.AGG_MIN, L.AGG_MAX):
        if op in codes:
            groups.append(tuple(dict.fromkeys(counts + [op])))
    return codes, groups


def window_agg_operator(window, aggs=("count_star", "count", "sum", "avg"), **kw):
    """One WindowAggOperator: a handle keeps the SUM-family, MIN and MAX accumulators side by
    side (value slots, include/flinkgpu.h fg_agg). Only the local phase of a two-phase plan,
    whose partial row holds one value accumulator, needs a handle per kind (open those with
    accumulator_groups)."""
    return WindowAggOperator(window, aggs=aggs, **kw)


class CompositeWindowAggOperator:
    """The WindowAggOperator surface over one engine handle per accumulator kind."""

    def __init__(self, window, aggs, **kw):
        if kw.get("local_partials"):
            raise ValueError("the local phase emits one partial accumulator: open one operator per kind")
        self.codes, groups = accumulator_groups(aggs)
        self.window = window
        self.ops = []
        try:
            for g in groups:
                self.ops.append(WindowAggOperator(window, aggs=g, **kw))
        except Exception:
            self.close()
            raise
        self.val_type = self.ops[0].val_type
        self.mode = self.ops[0].mode
        # output column -> the handle that computes it
        self._src = {}
        for c in self.codes:
            for op in self.ops:
                if c in op.aggs:
                    self._src[c] = op
                    break

    # -- processElement / processWatermark ------------------------------------------------------
    def process_batch(self, key, rowtime, val=None, val_null=None):
        for op in self.ops:
            op.process_batch(key, rowtime, val, val_null)

    def process_watermark(self, watermark: int, device_output: bool = False):
        """Rows fired by this watermark, joined over the handles and sorted by
        (window_end, key): a structured numpy array, or with device_output=True a dict of
        torch tensors (key, window_start, window_end, <agg>, <agg>_null)."""
        parts = [op.process_watermark(watermark, device_output=device_output) for op in self.ops]
        if device_output:
            return self._join_device(parts)
        return self._join_host(parts)

    def _join_host(self, parts):
        srt = []
        for p in parts:
            o = np.lexsort((p["key"], p["window_end"]))
            srt.append(p[o])
        base = srt[0]
        for p in srt[1:]:
            if len(p) != len(base) or not (np.array_equal(p["key"], base["key"]) and
                                           np.array_equal(p["window_end"], base["window_end"])):
                raise RuntimeError("accumulator handles fired different (key, window) sets")
        fields = [("key", "<i8"), ("window_start", "<i8"), ("window_end", "<i8")]
        for c in self.codes:
            nm = AGG_NAMES[c]
            fields += [(nm, srt[self.ops.index(self._src[c])].dtype.fields[nm][0]), (nm + "_null", "?")]
        if "rowtime" in base.dtype.names:
            fields.append(("rowtime", "<i8"))
        out = np.zeros(len(base), dtype=np.dtype(fields))
        for f in ("key", "window_start", "window_end") + (("rowtime",) if "rowtime" in base.dtype.names else ()):
            out[f] = base[f]
        for c in self.codes:
            nm = AGG_NAMES[c]
            src = srt[self.ops.index(self._src[c])]
            out[nm] = src[nm]
            out[nm + "_null"] = src[nm + "_null"]
        return out

    def _join_device(self, parts):
        import torch

        from .exchange import _DeviceColumn
        cols = []
        for op, r in zip(self.ops, parts):
            n = int(r.n)
            dev = torch.device("cuda", op.cfg.device_id)

            def col(ptr, dt=torch.int64):
                if n == 0:
                    return torch.empty(0, dtype=torch.int64, device=dev)
                return torch.as_tensor(_DeviceColumn(ptr, n), device=dev)
            torch.cuda.ExternalStream(op.stream, device=dev).synchronize()
            c = dict(key=col(r.key).clone(), window_start=col(r.window_start).clone(),
                     window_end=col(r.window_end).clone())
            nm_ = torch.as_tensor(_ByteColumn(r.null_mask, n), device=dev).clone() if n else \
                torch.zeros(0, dtype=torch.uint8, device=dev)
            for i, a in enumerate(op.aggs):
                v = col(r.agg[i]).clone()
                if self.val_type == L.VAL_F64 and a in (L.AGG_SUM, L.AGG_AVG, L.AGG_SUM0, L.AGG_MIN, L.AGG_MAX):
                    v = v.view(torch.float64)
                c[AGG_NAMES[a]] = v
                c[AGG_NAMES[a] + "_null"] = ((nm_ >> i) & 1).bool()
            # sort by (window_end, key): stable sort by key, then by window_end
            o = torch.argsort(c["key"], stable=True)
            o = o[torch.argsort(c["window_end"][o], stable=True)]
            cols.append({k: v[o] for k, v in c.items()})
        base = cols[0]
        for c in cols[1:]:
            if c["key"].numel() != base["key"].numel() or not (torch.equal(c["key"], base["key"]) and
                                                               torch.equal(c["window_end"], base["window_end"])):
                raise RuntimeError("accumulator handles fired different (key, window) sets")
        out = dict(key=base["key"], window_start=base["window_start"], window_end=base["window_end"])
        for c in self.codes:
            nm = AGG_NAMES[c]
            src = cols[self.ops.index(self._src[c])]
            out[nm] = src[nm]
            out[nm + "_null"] = src[nm + "_null"]
        return out

    # -- checkpointing -----------------------------------------------------------------------------
    def prepare_snapshot_pre_barrier(self):
        for op in self.ops:
            op.prepare_snapshot_pre_barrier()

    def snapshot_state(self):
        """(one window-aggs image per handle, timer watermark)."""
        snaps = [op.snapshot_state() for op in self.ops]
        return [s[0] for s in snaps], snaps[0][1]

    def restore_state(self, images, timer_watermark: int):
        for op, img in zip(self.ops, images):
            op.restore_state(img, timer_watermark)

    @property
    def num_late_records_dropped(self) -> int:
        return self.ops[0].num_late_records_dropped

    def reset(self):
        for op in self.ops:
            op.reset()

    def close(self):
        for op in getattr(self, "ops", []):
            op.close()
        self.ops = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class _ByteColumn:
    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (int(ptr or 0), False),
                                         "version": 2}
