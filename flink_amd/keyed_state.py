"""The SQL shim's checkpoint write into the keyed state backend, in Python.

Mirrors GpuSlicingWindowProcessor.writeKeyedState / restoreFromKeyedState
(java/.../window/gpu/GpuSlicingWindowProcessor.java; the JVM classes are not compiled in this
image) over a model of the heap backend's "window-aggs" ValueState (namespace = slice end, value =
the accumulator row) and its event-time timer service, so the GPU tests exercise the policy a Flink
job runs and count the backend operations a barrier costs.

The reference's prepareCheckpoint only flushes its buffer into state it already keeps in the
backend (AbstractWindowAggProcessor.java:195-197); AggCombiner.combine touches only the (key, slice)
pairs a flush saw (AggCombiner.java:76-115). The GPU engine keeps the state in HBM, so a checkpoint
must bring the backend up to date with the engine's image -- incrementally (`write_image`):

- the engine reports, per slice of the image, whether its table was written since the previous image
  (fg_snapshot_slices, include/flinkgpu.h ABI 16);
- every slice maps to a namespace: itself, or for a CUMULATE slice of a fired window the window's first
  slice + step, where CumulativeSliceAssigner.mergeSlices keeps the fired state (SliceAssigners.java:
  359-370); a namespace is rewritten iff one of its slices changed -- its entries put again, its
  window timer registered (AggCombiner.java:104-112; the timer service deduplicates);
- namespaces of the previous image that are gone (fired, expired), and namespaces whose slices changed
  (a CUMULATE slice that fired moves into its window's namespace) are cleared (their keys from
  getKeys(state, namespace)); their timers have fired already -- the operator forwards a watermark
  only after the engine fired its windows, so the timer service has passed them;
- a key holding state of fired slices only (HOP / CUMULATE) holds a timer at the next window end after
  the progress (SliceSharedWindowAggProcessor.fireWindow's nextTriggerWindow): registered for the keys
  of changed namespaces, and for every such key when the next window end moved.

`write_image_full` is round 5's rewrite (every entry cleared and put again, every timer deleted and
registered), kept as the cross-check: both leave the backend in the same state.
"""
from __future__ import annotations

import numpy as np

JMIN, JMAX = -(1 << 63), (1 << 63) - 1
TUMBLE, HOP, CUMULATE = 0, 1, 2


class SliceSpec:
    """The window spec the shim needs for namespaces and timers (GpuWindowAggSpec): kind, size,
    slide (HOP slide / CUMULATE step), offset, and a fixed shift-zone offset (TIMESTAMP_LTZ windows
    in a fixed-offset zone; 0 for UTC)."""

    def __init__(self, kind: int, size: int, slide: int = 0, offset: int = 0, tz_offset: int = 0):
        self.kind, self.size, self.slide, self.offset, self.tz = kind, size, slide, offset, tz_offset

    def window_start(self, ts: int, size: int) -> int:
        """TimeWindow.getWindowStartWithOffset"""
        r = (ts - self.offset) % size   # (floor mod: the Java code adds size for negative remainders)
        return ts - r

    def is_fired(self, window_end: int, progress: int) -> bool:
        """TimeWindowUtil.isWindowFired for a fixed-offset zone: toEpochMillsForTimer(end - 1) <= progress"""
        if window_end == JMAX:
            return False
        return window_end - 1 - self.tz <= progress

    def interval(self) -> int:
        """window ends: TUMBLE every size, HOP every slide, CUMULATE every step"""
        return self.size if self.kind == TUMBLE else self.slide

    def namespace(self, slice_end: int, progress: int) -> int:
        if self.kind == CUMULATE and self.is_fired(slice_end, progress):
            return self.window_start(slice_end - 1, self.size) + self.slide
        return slice_end

    def next_end(self, progress: int) -> int:
        iv = self.interval()
        return self.window_start(progress + self.tz, iv) + iv


def merge_acc(a: tuple, b: tuple, f64: bool) -> tuple:
    """two partial accumulators (cnt_star, cnt_val, sum bits, min bits, max bits) of one key, as
    GpuAccRows.merge does (COUNT / SUM add; MIN / MAX only over COUNT(v) > 0 sides)"""
    cs, cv = a[0] + b[0], a[1] + b[1]
    if f64:
        s = np.float64(np.int64(a[2]).view(np.float64) + np.int64(b[2]).view(np.float64)).view(np.int64)
    else:
        s = np.int64(np.int64(a[2]) + np.int64(b[2]))   # (Java long wrap-around)
    mn, mx = a[3], a[4]
    if b[1] > 0:
        if a[1] == 0:
            mn, mx = b[3], b[4]
        else:
            bv = (lambda x: np.int64(x).view(np.float64)) if f64 else (lambda x: x)
            mn = b[3] if bv(b[3]) < bv(a[3]) else a[3]
            mx = b[4] if bv(b[4]) > bv(a[4]) else a[4]
    return (int(cs), int(cv), int(s), int(mn), int(mx))


class WindowAggsState:
    """The heap backend's window-aggs ValueState + event-time timers of one subtask (a model, with
    the operation counts a checkpoint costs the task thread)."""

    def __init__(self, spec: SliceSpec, f64: bool = True, proctime: bool = False):
        self.spec, self.f64, self.proctime = spec, f64, proctime
        self.entries: dict[tuple[int, int], tuple] = {}   # (key, namespace) -> accumulator
        self.timers: set[tuple[int, int]] = set()          # (key, timestamp)
        self.namespaces: set[int] = set()                 # of the image last written / restored
        self.contrib: dict[int, set] = {}                 # namespace -> its slices at that image
        self.last_next_end = JMIN
        self.ops = dict(put=0, clear=0, timer_register=0, timer_delete=0, scan=0)

    # -- the timer service -------------------------------------------------------------------------
    def advance_watermark(self, wm: int):
        """InternalTimerServiceImpl.advanceWatermark: timers at or below the watermark fire (the
        shim's onEventTime is a no-op: the engine fired the windows)"""
        self.timers = {t for t in self.timers if t[1] > wm}

    def _register(self, key: int, window_end: int):
        """WindowTimerServiceImpl.registerEventTimeWindowTimer: the timer at
        toEpochMillsForTimer(window_end - 1) (the timer service deduplicates)"""
        self.ops["timer_register"] += 1
        self.timers.add((key, window_end - 1 - self.spec.tz))

    # -- the image -> backend ------------------------------------------------------------------------
    def _rows_of(self, image, lo: int, hi: int):
        mn = image.get("min", image["sum"])
        mx = image.get("max", image["sum"])
        for i in range(lo, hi):
            yield (int(image["key"][i]), int(image["slice_end"][i]),
                   (int(image["cnt_star"][i]), int(image["cnt_val"][i]), int(image["sum"][i]), int(mn[i]),
                    int(mx[i])))

    def _namespace_images(self, image, slices, progress, wanted=None):
        """{namespace: {key: acc}} of the namespaces in `wanted` (all if None), from the slices' rows"""
        out: dict[int, dict[int, tuple]] = {}
        for se, first, nrow in zip(slices["slice_end"].tolist(), slices["first_row"].tolist(),
                                   slices["rows"].tolist()):
            ns = self.spec.namespace(se, progress)
            if wanted is not None and ns not in wanted:
                continue
            m = out.setdefault(ns, {})
            for key, _, acc in self._rows_of(image, first, first + nrow):
                prev = m.get(key)
                m[key] = acc if prev is None else merge_acc(prev, acc, self.f64)
        return out

    def _fired_keys(self, image, slices, progress, wanted=None):
        keys = set()
        for se, first, nrow in zip(slices["slice_end"].tolist(), slices["first_row"].tolist(),
                                   slices["rows"].tolist()):
            if not self.spec.is_fired(se, progress):
                continue
            if wanted is not None and self.spec.namespace(se, progress) not in wanted:
                continue
            keys.update(int(k) for k in image["key"][first:first + nrow])
        return keys

    def write_image(self, image, slices, progress: int) -> dict:
        """writeKeyedState, incremental. `image`: the engine's snapshot columns; `slices`:
        fg_snapshot_slices; `progress`: the image's timer watermark. Returns this call's op counts."""
        before = dict(self.ops)
        sp = self.spec
        contrib: dict[int, set] = {}
        changed: dict[int, bool] = {}
        for se, ch in zip(slices["slice_end"].tolist(), slices["changed"].tolist()):
            ns = sp.namespace(se, progress)
            contrib.setdefault(ns, set()).add(se)
            changed[ns] = changed.get(ns, False) or bool(ch)
        # a namespace whose slices are not the ones it held at the last image (a CUMULATE slice that
        # fired since moved into its window's namespace, or left one) is rebuilt: cleared, then put
        reset = {ns for ns, c in contrib.items() if ns in self.contrib and self.contrib[ns] != c}
        for ns in reset:
            changed[ns] = True
        # namespaces gone since the previous image, and the ones rebuilt: cleared (their keys from
        # getKeys(state, namespace))
        for ns in sorted((self.namespaces - set(changed)) | reset):
            for kn in [kn for kn in self.entries if kn[1] == ns]:
                self.ops["scan"] += 1
                del self.entries[kn]
                self.ops["clear"] += 1
        dirty = {ns for ns, c in changed.items() if c}
        for ns, m in self._namespace_images(image, slices, progress, wanted=dirty).items():
            for key, acc in m.items():
                self.entries[(key, ns)] = acc
                self.ops["put"] += 1
                if not self.proctime and not sp.is_fired(ns, progress):
                    self._register(key, ns)
        if not self.proctime:
            nxt = sp.next_end(progress)
            moved = nxt != self.last_next_end
            for key in self._fired_keys(image, slices, progress, wanted=None if moved else dirty):
                self._register(key, nxt)
            self.last_next_end = nxt
        self.namespaces = set(changed)
        self.contrib = contrib
        return {k: self.ops[k] - before[k] for k in self.ops}

    def write_image_full(self, image, slices, progress: int) -> dict:
        """round 5's writeKeyedState: every previous entry cleared and every timer deleted, then the
        whole image put and every timer registered"""
        before = dict(self.ops)
        sp = self.spec
        self.ops["scan"] += len(self.entries)
        self.ops["clear"] += len(self.entries)
        self.entries.clear()
        self.ops["timer_delete"] += len(self.timers)
        self.timers.clear()
        for ns, m in self._namespace_images(image, slices, progress).items():
            for key, acc in m.items():
                self.entries[(key, ns)] = acc
                self.ops["put"] += 1
                if not self.proctime and not sp.is_fired(ns, progress):
                    self._register(key, ns)
        if not self.proctime:
            nxt = sp.next_end(progress)
            for key in self._fired_keys(image, slices, progress):
                self._register(key, nxt)
            self.last_next_end = nxt
        self.namespaces = {sp.namespace(se, progress) for se in slices["slice_end"].tolist()}
        self.contrib = {}
        for se in slices["slice_end"].tolist():
            self.contrib.setdefault(sp.namespace(se, progress), set()).add(se)
        return {k: self.ops[k] - before[k] for k in self.ops}

    # -- backend -> engine (initializeState) ---------------------------------------------------------
    def image(self):
        """restoreFromKeyedState: every entry as an image row, and the timer watermark = the smallest
        registered timer's time - 1 (every window ending before it has fired, none after it)."""
        items = sorted(self.entries.items(), key=lambda kv: (kv[0][1], kv[0][0]))
        n = len(items)
        cols = {c: np.zeros(n, dtype=np.int64) for c in ("key", "slice_end", "cnt_star", "cnt_val", "sum", "min", "max")}
        for i, ((key, ns), acc) in enumerate(items):
            cols["key"][i], cols["slice_end"][i] = key, ns
            cols["cnt_star"][i], cols["cnt_val"][i], cols["sum"][i], cols["min"][i], cols["max"][i] = acc
        twm = min((t for _, t in self.timers), default=None)
        self.namespaces = {ns for _, ns in self.entries}
        # (which slices made a restored namespace is not in the backend: a namespace is its own slice
        # unless a CUMULATE window fired into it -- the first image after a restore rebuilds those)
        self.contrib = {ns: {ns} for ns in self.namespaces}
        self.last_next_end = JMIN
        return cols, JMIN if twm is None else twm - 1
