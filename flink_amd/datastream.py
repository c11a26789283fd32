"""DataStream keyBy(f0).window(Tumbling|SlidingEventTimeWindows).sum / min / max(1), and
.aggregate(AggregateFunction) with the GPU's COUNT / SUM / AVG / MIN / MAX functions, on
Tuple2<Long, Long | Double> -- the Python mirror of the JVM shim
java/.../streaming/runtime/operators/windowing/gpu/GpuWindowOperator.java (and
GpuAggregateFunctions.java), with the reference WindowOperator's keyed-state layout on both sides
of a checkpoint.

aggregate (api="aggregate"): WindowedStream.aggregate (WindowedStream.java:283-349) ->
WindowOperatorBuilder.aggregate (:198-224): an AggregatingStateDescriptor "window-contents" of the
function's accumulator type. The accumulators of the GPU functions: COUNT a long count; SUM the
field's sum; AVG (sum, count); MIN / MAX the field's extreme under the field's compareTo (the
identity when empty: Long.MAX_VALUE / NaN for MIN, Long.MIN_VALUE / -inf for MAX); the result
(getResult): the count, the sum, sum / count as a double, the extreme. The engine keeps COUNT(*)
and the value accumulator per (key, slice); a window's accumulator is their merge.

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
    """keyBy(f0).window(...).{sum, min, max}(1) (api="reduce"), or .aggregate(f) for the GPU's
    f in {count, sum, avg, min, max} (api="aggregate"), over Tuple2<Long, Long | Double>.

    Internally every (key, window) holds an accumulator (a0, a1): a0 the value accumulator's bits
    (sum / min / max), a1 the record count."""

    def __init__(self, kind: str, size: int, slide: int = 0, offset: int = 0, val_type: str = "i64",
                 agg: str = "sum", allowed_lateness: int = 0, purging: bool = False, api: str = "reduce",
                 **engine):
        if api == "reduce" and agg not in ("sum", "min", "max"):
            raise ValueError(f"aggregation {agg!r}: sum, min or max (minBy / maxBy: min / max)")
        if api == "aggregate" and agg not in ("count", "sum", "avg", "min", "max"):
            raise ValueError(f"GPU aggregate function {agg!r}: count, sum, avg, min or max")
        if api not in ("reduce", "aggregate"):
            raise ValueError(f"api {api!r}: reduce or aggregate")
        self.kind, self.size = kind, int(size)
        self.slide = int(size if kind == "tumble" else slide)
        self.offset = int(offset)
        self.api, self.agg, self.f64 = api, agg, val_type == "f64"
        # the value accumulator's merge: sum (SUM, AVG) or the extreme; COUNT has none
        self.vkind = "sum" if agg in ("sum", "avg") else agg if agg in ("min", "max") else None
        self.lateness, self.purging = int(allowed_lateness), bool(purging)
        self._engine_kw = dict(engine)
        win = tumbling(size, offset) if kind == "tumble" else hopping(size, slide, offset)
        aggs = ("count_star",) + ((self.vkind,) if self.vkind else ())
        self.op = WindowAggOperator(win, aggs=aggs, val_type=val_type if self.vkind else "none",
                                    mode="datastream", allowed_lateness=allowed_lateness,
                                    purging_trigger=purging, **engine)
        self.watermark = JMIN
        self.restored = {}   # window end -> dict(key, value, pending) of restored (key, window) entries

    def close(self):
        self.op.close()

    # -- processElement / processWatermark ----------------------------------------------------
    def process_batch(self, key, ts, val):
        self.op.process_batch(key, ts, val if self.vkind else None)   # (COUNT reads no field)

    def _cleanup_time(self, end):
        """WindowOperator.cleanupTime (:669-673): maxTimestamp + allowedLateness, Long.MAX_VALUE
        on overflow (scalar or array)."""
        with np.errstate(over="ignore"):
            max_ts = np.asarray(end, dtype=np.int64) - np.int64(1)
            c = max_ts + np.int64(self.lateness)
        c = np.where(c >= max_ts, c, np.int64(JMAX))
        return int(c) if c.ndim == 0 else c

    # accumulators (a0 value bits, a1 count) -------------------------------------------------
    def _merge(self, a0, a1, b0, b1):
        """merge(acc a, acc b), a the earlier (restored) one: the value accumulator by its kind,
        the counts added"""
        v = reduce_bits(self.vkind, self.f64, a0, b0) if self.vkind else np.zeros(len(a0), np.int64)
        with np.errstate(over="ignore"):
            return v, np.asarray(a1, np.int64) + np.asarray(b1, np.int64)

    def _result(self, a0, a1):
        """the emitted value's bits: the reduced field (reduce), or getResult of the accumulator"""
        if self.api == "reduce" or self.agg in ("sum", "min", "max"):
            return a0
        if self.agg == "count":
            return a1.astype(np.int64)
        s = a0.view(np.float64) if self.f64 else a0.astype(np.float64)   # AVG: (double) sum / count
        return (s / a1.astype(np.float64)).view(np.int64)

    def _image_acc(self, image):
        """(a0, a1) of an image's entries: reduce keeps the value; aggregate's accumulators --
        COUNT its count, SUM / MIN / MAX the value, AVG (sum, count)"""
        n = len(image["key"])
        a0 = np.asarray(image["value"], np.int64) if "value" in image else np.zeros(n, np.int64)
        a1 = np.asarray(image["count"], np.int64) if "count" in image else np.ones(n, np.int64)
        return a0, a1

    def process_watermark(self, wm: int) -> np.ndarray:
        """Rows fired by the watermark: (key, value bits, timestamp = window.maxTimestamp(),
        window_end) -- with restored windows reduced in (WindowOperator.emitWindowContents)."""
        r = self.op.process_watermark(wm)
        key = r["key"].astype(np.int64)
        end = r["window_end"].astype(np.int64)
        a1 = r["count_star"].astype(np.int64).copy()
        a0 = (np.ascontiguousarray(r[self.vkind]).view(np.int64).copy() if self.vkind
              else np.zeros(len(key), np.int64))
        extra_k, extra_e, extra_0, extra_1 = [], [], [], []
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
                    a0[hs], a1[hs] = self._merge(R["a0"][pos_c[hit]], R["a1"][pos_c[hit]], a0[hs], a1[hs])
                    R["pending"][pos_c[hit]] = False
                    if self.purging:   # a fired (key, window) is purged
                        R["alive"][pos_c[hit]] = False
                if e - 1 <= wm:   # the window's trigger: restored entries without a GPU row fire alone
                    fire = R["pending"] & R["alive"]
                    extra_k.append(R["key"][fire])
                    extra_e.append(np.full(int(fire.sum()), e, dtype=np.int64))
                    extra_0.append(R["a0"][fire])
                    extra_1.append(R["a1"][fire])
                    R["pending"][:] = False
                    if self.purging:
                        R["alive"][fire] = False
                if self._cleanup_time(e) <= wm or not R["alive"].any():
                    del self.restored[e]
        self.watermark = max(self.watermark, int(wm))
        if extra_k:
            key = np.concatenate([key] + extra_k)
            end = np.concatenate([end] + extra_e)
            a0 = np.concatenate([a0] + extra_0)
            a1 = np.concatenate([a1] + extra_1)
        out = np.zeros(len(key), dtype=[("key", "<i8"), ("value", "<i8"), ("timestamp", "<i8"), ("window_end", "<i8")])
        out["key"], out["value"], out["window_end"], out["timestamp"] = key, self._result(a0, a1), end, end - 1
        return out

    @property
    def late_dropped(self) -> int:
        return self.op.num_late_records_dropped

    # -- checkpoint ------------------------------------------------------------------------------
    def snapshot(self) -> dict:
        """prepareSnapshotPreBarrier + snapshotState: the reference WindowOperator's keyed state --
        "window-contents" (key, window_start, window_end, and the state's value: the reduced
        field's bits for reduce; the accumulator for aggregate -- `value` (SUM / AVG sum, MIN,
        MAX bits) and `count` (COUNT, AVG)) and "window-timers" (timer_key, timer_window_end,
        timer_ts)."""
        self.op.prepare_snapshot_pre_barrier()
        img, _ = self.op.snapshot_state()
        wm = self.watermark
        k, s = img["key"], img["slice_end"]
        v0 = img["sum"] if self.vkind else np.zeros(len(k), np.int64)
        v1 = img["cnt_star"]
        n = self.size // self.slide
        ks = np.repeat(k, n)
        es = (np.repeat(s, n).reshape(-1, n) + np.arange(n, dtype=np.int64) * self.slide).reshape(-1)
        v0s, v1s = np.repeat(v0, n), np.repeat(v1, n)
        live = self._cleanup_time(es) > wm
        if self.purging:   # a fired window's contents were purged
            live &= es - 1 > wm
        ks, es, v0s, v1s = ks[live], es[live], v0s[live], v1s[live]
        for e, R in self.restored.items():
            a = R["alive"]   # (restored accumulator first: value1 of the reduce / merge)
            ks = np.concatenate([R["key"][a], ks])
            es = np.concatenate([np.full(int(a.sum()), e, dtype=np.int64), es])
            v0s = np.concatenate([R["a0"][a], v0s])
            v1s = np.concatenate([R["a1"][a], v1s])
        key, end, val = _group_reduce(self.vkind or "sum", self.f64 and self.vkind is not None, ks, es, v0s)
        _, _, cnt = _group_reduce("sum", False, ks, es, v1s)
        # timers: the trigger of a window not fired yet, the cleanup timer with allowed lateness
        trig = end - 1 > wm
        cl = self._cleanup_time(end)
        has_cl = (cl != JMAX) & (cl != end - 1)
        tk = np.concatenate([key[trig], key[has_cl]])
        te = np.concatenate([end[trig], end[has_cl]])
        tt = np.concatenate([end[trig] - 1, cl[has_cl]])
        out = dict(key=key, window_start=end - self.size, window_end=end,
                   timer_key=tk, timer_window_end=te, timer_ts=tt)
        if self.vkind:
            out["value"] = val
        if self.api == "aggregate" and self.agg in ("count", "avg"):
            out["count"] = cnt
        return out

    def restore(self, image: dict):
        """initializeState from a reference (or GPU) WindowOperator image: the engine restarts empty
        at Long.MIN_VALUE, the image's windows are held as restored contents."""
        self.op.reset()
        self.watermark = JMIN
        self.restored = {}
        key = np.asarray(image["key"], dtype=np.int64)
        end = np.asarray(image["window_end"], dtype=np.int64)
        a0, a1 = self._image_acc(image)
        tk = np.asarray(image["timer_key"], dtype=np.int64)
        te = np.asarray(image["timer_window_end"], dtype=np.int64)
        tt = np.asarray(image["timer_ts"], dtype=np.int64)
        trig = tt == te - 1
        pend = set(zip(tk[trig].tolist(), te[trig].tolist()))
        for e in np.unique(end):
            sel = np.flatnonzero(end == e)
            o = sel[np.argsort(key[sel], kind="stable")]
            kk = key[o]
            self.restored[int(e)] = dict(key=kk, a0=a0[o].copy(), a1=a1[o].copy(),
                                         pending=np.array([(int(x), int(e)) in pend for x in kk], dtype=bool),
                                         alive=np.ones(len(kk), dtype=bool))


__all__ = ["DataStreamWindowOperator", "reduce_bits"]
