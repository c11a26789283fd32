"""DataStream keyBy(f0).window(Tumbling|SlidingEventTimeWindows).sum / min / max(1) on
Tuple2<Long, Long | Double> -- the Python mirror of the JVM shim
java/.../streaming/runtime/operators/windowing/gpu/GpuWindowOperator.java, with the reference
WindowOperator's keyed-state layout on both sides of a checkpoint.

The reference (flink-streaming-java):
  WindowedStream.sum / min / max / minBy / maxBy (WindowedStream.java:671-850) -> aggregate ->
  reduce(SumAggregator | ComparableAggregator) -> WindowOperatorBuilder.reduce (:150-172): a
  ReducingStateDescriptor "window-contents" (:71) of the input type, namespace TimeWindow;
  WindowOperator (:225) keeps its timers in "window-timers": EventTimeTrigger's timer at
  window.maxTimestamp() (EventTimeTrigger.java:37-46) and the cleanup timer at
  maxTimestamp + allowedLateness (WindowOperator.java:630-642,669-673).

The engine (FG_MODE_DATASTREAM) keeps slices, not windows. At a checkpoint this operator writes
the reference's image -- one reduced value per (key, TimeWindow) and the timers the reference
would hold -- so that a CPU WindowOperator can restore a GPU savepoint:
  * a window's value is the reduce of its slices' values (a sliding window spans size / slide
    slices); windows past their cleanup time are gone (WindowOperator.clearAllState), and so are
    fired windows under a purging trigger;
  * a window not fired yet (maxTimestamp > watermark) holds its trigger timer; with allowed
    lateness every window holds its cleanup timer too (one timer when they coincide).
On restore (from a GPU or a CPU savepoint) the image's windows are kept on the host as restored
contents, and the engine starts empty at Long.MIN_VALUE (the restored timer service's watermark,
InternalTimerServiceImpl): a fired GPU row of a restored (key, window) carries the elements
since the restore and is reduced with the restored value; a restored (key, window) whose trigger
timer is pending and that has no GPU row fires its restored value alone when the watermark
passes its maxTimestamp; restored windows are dropped at their cleanup time (at their fire under
a purging trigger). This is the reference's behaviour for the restored windows -- its state is
the reduce of the restored value and every element accepted since -- without decomposing a
sliding window's value into slices, which the value does not determine.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .window_agg import WindowAggOperator, hopping, tumbling

JMIN = -(1 << 63)
JMAX = (1 << 63) - 1


def _ord(bits):
    """Double.compareTo's total order on canonical f64 bits (NaN above +inf, -0.0 below +0.0)."""
    b = bits.astype(np.int64)
    return np.where(b >= 0, b, b ^ np.int64(JMAX))


def _canon(bits):
    """Double.doubleToLongBits (every NaN -> the canonical NaN)."""
    b = bits.astype(np.int64)
    nan = (b & np.int64(JMAX)) > np.int64(0x7FF0000000000000)
    return np.where(nan, np.int64(0x7FF8000000000000), b)


def reduce_bits(agg: str, f64: bool, a, b):
    """The aggregator's reduce of two value-field bit arrays, a the earlier value (value1):
    SumAggregator (SumFunction: long +, double +), ComparableAggregator MIN / MAX (value2 wins
    unless value1 compares strictly smaller / greater, ComparableAggregator.java:83-104)."""
    a = np.asarray(a, dtype=np.int64)
    b = np.asarray(b, dtype=np.int64)
    if agg == "sum":
        if f64:
            return (a.view(np.float64) + b.view(np.float64)).view(np.int64)
        with np.errstate(over="ignore"):
            return a + b   # (two's complement wrap, Java long +)
    if f64:
        a, b = _canon(a), _canon(b)
        oa, ob = _ord(a), _ord(b)
    else:
        oa, ob = a, b
    keep_a = oa < ob if agg == "min" else oa > ob
    return np.where(keep_a, a, b)


def _group_reduce(agg: str, f64: bool, key, end, val):
    """(key, end) groups of (key, end, val) and the reduce of each group's values, in input order
    within a group (the f64 sum adds left to right)."""
    if len(key) == 0:
        z = np.zeros(0, dtype=np.int64)
        return z, z, z
    order = np.lexsort((end, key))
    k, e, v = key[order], end[order], val[order]
    start = np.ones(len(k), dtype=bool)
    start[1:] = (k[1:] != k[:-1]) | (e[1:] != e[:-1])
    idx = np.flatnonzero(start)
    if agg == "sum" and not f64:
        with np.errstate(over="ignore"):
            out = np.add.reduceat(v, idx)
    else:   # (f64 sums too: left to right, as the reduce adds; numpy's reduceat may pair them)
        out = v[idx].copy()
        nxt = np.append(idx[1:], len(k))   # (groups are short: a window's slices + its restored value)
        for j in range(1, int(np.max(nxt - idx))):
            pos = idx + j
            ok = pos < nxt
            out[ok] = reduce_bits(agg, f64, out[ok], v[pos[ok]])
    return k[idx], e[idx], out


class DataStreamWindowOperator:
    """keyBy(f0).window(...).{sum, min, max}(1) over Tuple2<Long, Long | Double> on the GPU."""

    def __init__(self, kind: str, size: int, slide: int = 0, offset: int = 0, val_type: str = "i64",
                 agg: str = "sum", allowed_lateness: int = 0, purging: bool = False, **engine):
        if agg not in ("sum", "min", "max"):
            raise ValueError(f"aggregation {agg!r}: sum, min or max (minBy / maxBy: min / max)")
        self.kind, self.size = kind, int(size)
        self.slide = int(size if kind == "tumble" else slide)
        self.offset = int(offset)
        self.agg, self.f64 = agg, val_type == "f64"
        self.lateness, self.purging = int(allowed_lateness), bool(purging)
        self._engine_kw = dict(engine)
        win = tumbling(size, offset) if kind == "tumble" else hopping(size, slide, offset)
        self.op = WindowAggOperator(win, aggs=("count_star", agg), val_type=val_type, mode="datastream",
                                    allowed_lateness=allowed_lateness, purging_trigger=purging, **engine)
        self.watermark = JMIN
        self.restored = {}   # window end -> dict(key, value, pending) of restored (key, window) entries

    def close(self):
        self.op.close()

    # -- processElement / processWatermark ----------------------------------------------------
    def process_batch(self, key, ts, val):
        self.op.process_batch(key, ts, val)

    def _cleanup_time(self, end):
        """WindowOperator.cleanupTime (:669-673): maxTimestamp + allowedLateness, Long.MAX_VALUE
        on overflow (scalar or array)."""
        with np.errstate(over="ignore"):
            max_ts = np.asarray(end, dtype=np.int64) - np.int64(1)
            c = max_ts + np.int64(self.lateness)
        c = np.where(c >= max_ts, c, np.int64(JMAX))
        return int(c) if c.ndim == 0 else c

    def process_watermark(self, wm: int) -> np.ndarray:
        """Rows fired by the watermark: (key, value bits, timestamp = window.maxTimestamp(),
        window_end) -- with restored windows reduced in (WindowOperator.emitWindowContents)."""
        r = self.op.process_watermark(wm)
        key = r["key"].astype(np.int64)
        end = r["window_end"].astype(np.int64)
        val = np.ascontiguousarray(r[self.agg]).view(np.int64).copy()
        extra_k, extra_e, extra_v = [], [], []
        if self.restored:
            for e in list(self.restored):
                R = self.restored[e]
                sel = np.flatnonzero(end == e)
                if len(sel):
                    pos = np.searchsorted(R["key"], key[sel])
                    pos_c = np.minimum(pos, len(R["key"]) - 1)
                    hit = (pos < len(R["key"])) & (R["key"][pos_c] == key[sel])
                    hit &= R["alive"][pos_c]   # (a purged (key, window) holds only the new elements)
                    hs = sel[hit]
                    val[hs] = reduce_bits(self.agg, self.f64, R["value"][pos_c[hit]], val[hs])
                    R["pending"][pos_c[hit]] = False
                    if self.purging:   # a fired (key, window) is purged
                        R["alive"][pos_c[hit]] = False
                if e - 1 <= wm:   # the window's trigger: restored entries without a GPU row fire alone
                    fire = R["pending"] & R["alive"]
                    extra_k.append(R["key"][fire])
                    extra_e.append(np.full(int(fire.sum()), e, dtype=np.int64))
                    extra_v.append(R["value"][fire])
                    R["pending"][:] = False
                    if self.purging:
                        R["alive"][fire] = False
                if self._cleanup_time(e) <= wm or not R["alive"].any():
                    del self.restored[e]
        self.watermark = max(self.watermark, int(wm))
        if extra_k:
            key = np.concatenate([key] + extra_k)
            end = np.concatenate([end] + extra_e)
            val = np.concatenate([val] + extra_v)
        out = np.zeros(len(key), dtype=[("key", "<i8"), ("value", "<i8"), ("timestamp", "<i8"), ("window_end", "<i8")])
        out["key"], out["value"], out["window_end"], out["timestamp"] = key, val, end, end - 1
        return out

    @property
    def late_dropped(self) -> int:
        return self.op.num_late_records_dropped

    # -- checkpoint ------------------------------------------------------------------------------
    def snapshot(self) -> dict:
        """prepareSnapshotPreBarrier + snapshotState: the reference WindowOperator's keyed state --
        "window-contents" (key, window_start, window_end, value bits) and "window-timers"
        (timer_key, timer_window_end, timer_ts)."""
        self.op.prepare_snapshot_pre_barrier()
        img, _ = self.op.snapshot_state()
        wm = self.watermark
        k, s, v = img["key"], img["slice_end"], img["sum"]
        n = self.size // self.slide
        ks = np.repeat(k, n)
        es = (np.repeat(s, n).reshape(-1, n) + np.arange(n, dtype=np.int64) * self.slide).reshape(-1)
        vs = np.repeat(v, n)
        live = self._cleanup_time(es) > wm
        if self.purging:   # a fired window's contents were purged
            live &= es - 1 > wm
        ks, es, vs = ks[live], es[live], vs[live]
        for e, R in self.restored.items():
            a = R["alive"]
            ks = np.concatenate([R["key"][a], ks])   # (restored value first: value1 of the reduce)
            es = np.concatenate([np.full(int(a.sum()), e, dtype=np.int64), es])
            vs = np.concatenate([R["value"][a], vs])
        key, end, val = _group_reduce(self.agg, self.f64, ks, es, vs)
        # timers: the trigger of a window not fired yet, the cleanup timer with allowed lateness
        trig = end - 1 > wm
        cl = self._cleanup_time(end)
        has_cl = (cl != JMAX) & (cl != end - 1)
        tk = np.concatenate([key[trig], key[has_cl]])
        te = np.concatenate([end[trig], end[has_cl]])
        tt = np.concatenate([end[trig] - 1, cl[has_cl]])
        return dict(key=key, window_start=end - self.size, window_end=end, value=val,
                    timer_key=tk, timer_window_end=te, timer_ts=tt)

    def restore(self, image: dict):
        """initializeState from a reference (or GPU) WindowOperator image: the engine restarts empty
        at Long.MIN_VALUE, the image's windows are held as restored contents."""
        self.op.reset()
        self.watermark = JMIN
        self.restored = {}
        key = np.asarray(image["key"], dtype=np.int64)
        end = np.asarray(image["window_end"], dtype=np.int64)
        val = np.asarray(image["value"], dtype=np.int64)
        tk = np.asarray(image["timer_key"], dtype=np.int64)
        te = np.asarray(image["timer_window_end"], dtype=np.int64)
        tt = np.asarray(image["timer_ts"], dtype=np.int64)
        trig = tt == te - 1
        pend = set(zip(tk[trig].tolist(), te[trig].tolist()))
        for e in np.unique(end):
            sel = np.flatnonzero(end == e)
            o = sel[np.argsort(key[sel], kind="stable")]
            kk = key[o]
            self.restored[int(e)] = dict(key=kk, value=val[o].copy(),
                                         pending=np.array([(int(x), int(e)) in pend for x in kk], dtype=bool),
                                         alive=np.ones(len(kk), dtype=bool))


__all__ = ["DataStreamWindowOperator", "reduce_bits"]
