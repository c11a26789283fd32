"""Host-side mirror of the reference's window-aggregation operators over libflinkgpu.

``WindowAggOperator`` keeps the operator surface of
  * SQL:  ``SlicingWindowOperator`` built by ``SlicingWindowAggOperatorBuilder``
          (TR/operators/window/slicing/SlicingWindowOperator.java:196-242,
           TR/operators/aggregate/window/SlicingWindowAggOperatorBuilder.java:127-170), and
  * DataStream: ``WindowOperator`` for ``keyBy().window(Tumbling|SlidingEventTimeWindows).sum()``
          (SJ/runtime/operators/windowing/WindowOperator.java:300-503),
with the same names, argument meaning and error behaviour:

  processElement (batched)      -> process_batch(key, rowtime, val, val_null)
  processWatermark              -> process_watermark(wm)  (returns the fired rows)
  prepareSnapshotPreBarrier     -> prepare_snapshot_pre_barrier()
  snapshotState / initializeState -> snapshot_state() / restore_state()
  getNumLateRecordsDropped      -> num_late_records_dropped

The window spec factories mirror ``SliceAssigners.tumbling/hopping/cumulative``
(TR/operators/window/slicing/SliceAssigners.java:59-96) and raise ``WindowSpecError``
(a ValueError) with the reference's IllegalArgumentException message.

All compute runs in libflinkgpu.so (HIP, gfx950). Inputs may be numpy arrays (host,
copied H2D) or device tensors (torch CUDA tensors / objects exposing
``__cuda_array_interface__``), which are consumed in place.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L

AGG_NAMES = {L.AGG_COUNT_STAR: "count_star", L.AGG_COUNT: "count", L.AGG_SUM: "sum", L.AGG_AVG: "avg",
             L.AGG_SUM0: "sum0", L.AGG_MIN: "min", L.AGG_MAX: "max"}
AGGS = {"count_star": L.AGG_COUNT_STAR, "count": L.AGG_COUNT, "sum": L.AGG_SUM, "avg": L.AGG_AVG,
        "sum0": L.AGG_SUM0, "min": L.AGG_MIN, "max": L.AGG_MAX}
# aggregates whose column has the value's type (DOUBLE for f64 values)
VALUE_TYPED = (L.AGG_SUM, L.AGG_AVG, L.AGG_SUM0, L.AGG_MIN, L.AGG_MAX)


@dataclass(frozen=True)
class Window:
    kind: int
    size: int
    slide: int = 0
    offset: int = 0


def tumbling(size_ms: int, offset_ms: int = 0) -> Window:
    """SliceAssigners.tumbling (:59-62) / TumblingEventTimeWindows.of."""
    return Window(L.TUMBLE, int(size_ms), 0, int(offset_ms))


def hopping(size_ms: int, slide_ms: int, offset_ms: int = 0) -> Window:
    """SliceAssigners.hopping (:75-79) / SlidingEventTimeWindows.of (DataStream)."""
    return Window(L.HOP, int(size_ms), int(slide_ms), int(offset_ms))


def cumulative(max_size_ms: int, step_ms: int, offset_ms: int = 0) -> Window:
    """SliceAssigners.cumulative (:92-96)."""
    return Window(L.CUMULATE, int(max_size_ms), int(step_ms), int(offset_ms))


def _dev_ptr(x):
    """(pointer, is_device) of a column: torch tensor, CUDA-array-interface object or numpy."""
    if x is None:
        return None, False, None
    if hasattr(x, "is_cuda") and hasattr(x, "data_ptr"):
        if x.is_cuda:
            assert x.is_contiguous(), "device columns must be contiguous"
            return x.data_ptr(), True, x
        x = x.numpy()
    if hasattr(x, "__cuda_array_interface__"):
        return x.__cuda_array_interface__["data"][0], True, x
    return None, False, x


class WindowAggOperator:
    """SlicingWindowOperator / WindowOperator with the buffer, state and firing on an MI355X."""

    def __init__(self, window: Window, aggs=("count_star", "count", "sum", "avg"), val_type: str = "f64",
                 mode: str = "sql", shift_tz_offset_ms: int = 0, expected_keys: int = 1 << 16,
                 buffer_records: int = 1 << 22, device: int = 0, max_parallelism: int = 128,
                 key_group_range=(0, 127), kernel_timing: bool = False, local_partials: bool = False,
                 proctime: bool = False, zone: str | None = None, windowed: bool = False,
                 allowed_lateness: int = 0, purging_trigger: bool = False):
        """allowed_lateness (DataStream): WindowedStream.allowedLateness -- a fired window keeps
        its state until maxTimestamp + allowed_lateness, and an element reaching it meanwhile
        fires it again at once; those rows are returned by the next process_watermark, ahead of
        the rows its watermark fires. purging_trigger: PurgingTrigger.of(EventTimeTrigger) (a
        firing window's state is cleared).

        windowed: rows carry their window (WindowedSliceAssigner, after a window TVF): the
        `rowtime` column of process_batch holds each row's window_end; `window` is the TVF's.

        zone: an IANA zone name (TableConfig.getLocalTimeZone() of a TIMESTAMP_LTZ window)
        whose rules -- transitions and daylight saving -- replace shift_tz_offset_ms
        (flink_amd.tz.zone_rules; a zone that never changed offset takes the fixed path).

        local_partials: the local phase of the two-phase aggregation
        (LocalSlicingWindowAggOperator + LocalAggCombiner): process_watermark returns one
        partial accumulator row per (key, fired slice) with columns count_star, count, sum
        (min / max for a MIN / MAX query; sum, min and max for a list mixing them;
        window_start/window_end = the slice), to be exchanged by key group and merged by a
        global operator's process_partials."""
        lib = L.load()
        self.window = window
        self.mode = {"sql": L.MODE_SQL, "datastream": L.MODE_DATASTREAM}[mode]
        self.val_type = {"none": L.VAL_NONE, "i64": L.VAL_I64, "f64": L.VAL_F64}[val_type]
        self.local_partials = bool(local_partials)
        if self.local_partials:
            # the partial accumulator: SUM, or the MIN / MAX of a MIN / MAX query; a list mixing
            # them carries SUM, MIN and MAX (the engine's layout for the C-ABI)
            kinds = {("min" if a in ("min", L.AGG_MIN) else "max" if a in ("max", L.AGG_MAX) else
                      "sum" if a in ("sum", "avg", "sum0", L.AGG_SUM, L.AGG_AVG, L.AGG_SUM0) else None)
                     for a in aggs} - {None}
            if len(kinds) > 1:   # several value accumulators: the partial row carries all three
                aggs = ("count_star", "count", "sum", "min", "max")
            else:
                vagg = next((a for a in aggs if a in ("min", "max", L.AGG_MIN, L.AGG_MAX)), "sum")
                aggs = ("count_star", "count", AGG_NAMES.get(vagg, vagg))
        self.aggs = tuple(AGGS[a] if isinstance(a, str) else int(a) for a in aggs)
        cfg = L.FgConfig()
        cfg.mode = self.mode
        cfg.window_kind = window.kind
        cfg.size_ms = window.size
        cfg.slide_ms = window.slide
        cfg.offset_ms = window.offset
        cfg.shift_tz_offset_ms = int(shift_tz_offset_ms)
        cfg.val_type = self.val_type
        cfg.num_aggs = len(self.aggs)
        for i, a in enumerate(self.aggs):
            cfg.aggs[i] = a
        cfg.max_parallelism = int(max_parallelism)
        cfg.key_group_start, cfg.key_group_end = int(key_group_range[0]), int(key_group_range[1])
        cfg.device_id = int(device)
        cfg.flags = ((L.FLAG_KERNEL_TIMING if kernel_timing else 0) | (L.FLAG_LOCAL_PARTIALS if local_partials else 0)
                     | (L.FLAG_PROCTIME if proctime else 0) | (L.FLAG_WINDOWED if windowed else 0)
                     | (L.FLAG_PURGING_TRIGGER if purging_trigger else 0))
        cfg.allowed_lateness_ms = int(allowed_lateness)
        cfg.expected_keys = int(expected_keys)
        cfg.buffer_records = int(buffer_records)
        self.zone = zone
        if zone is not None:
            from .tz import zone_rules
            trans, offs, dst = zone_rules(zone)
            if len(trans) == 0:
                cfg.shift_tz_offset_ms = int(offs[0])
            else:   # fg_open copies the rules
                self._tz = (np.ascontiguousarray(trans), np.ascontiguousarray(offs))
                cfg.tz_transition_ms = self._tz[0].ctypes.data
                cfg.tz_offset_ms = self._tz[1].ctypes.data
                cfg.n_tz_transitions = len(trans)
                cfg.tz_use_daylight = 1 if dst else 0
        self.cfg = cfg
        h = C.c_void_p()
        L.check(lib.fg_open(C.byref(cfg), C.byref(h)), None)
        self._h = h
        self._dev_rows = L.FgRows()   # process_watermark(device_output=True) result
        self._dev_rows_ref = C.byref(self._dev_rows)
        self._lib = lib

    # -- lifecycle -------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._lib.fg_close(self._h)   # drains the engine stream: no column is read any more
            self._h = None
            self._inflight, self._held = None, []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- processElement ---------------------------------------------------------------------
    def _after_producers(self, cols):
        """Device columns are read on the engine's stream: order it after the torch stream
        that produced them (an event wait, no host synchronization)."""
        for c in cols:
            if hasattr(c, "is_cuda") and c.is_cuda:
                import torch
                cur = torch.cuda.current_stream(c.device)
                ext = self.__dict__.get("_ext_stream")
                if ext is None or ext.device != c.device:   # made once per operator
                    ext = self._ext_stream = torch.cuda.ExternalStream(self.stream, device=c.device)
                # a producer stream with nothing left to run: the columns are complete (no barrier
                # packet on the engine stream -- it delays the batch's first kernel by ~20 us)
                if not cur.query():
                    ext.wait_stream(cur)
                return

    def process_batch(self, key, rowtime, val=None, val_null=None, rowtime_base=None):
        """processElement for every record of a micro-batch (arrival order = index order).

        Host columns may be narrow (fg_batch.format, fewer bytes over PCIe): an int32 key
        column, rowtime as uint32 offsets from `rowtime_base`, an int32 BIGINT value column."""
        self._after_producers((key, rowtime, val, val_null))
        kp, kdev, key = _dev_ptr(key)
        tp, tdev, rowtime = _dev_ptr(rowtime)
        vp, vdev, val = _dev_ptr(val)
        np_, ndev, val_null = _dev_ptr(val_null)
        keep = []
        b = L.FgBatch()
        if kdev:
            assert tdev and (val is None or vdev) and (val_null is None or ndev), "mixed host/device columns"
            b.location = L.DEVICE
            b.n = int(key.numel() if hasattr(key, "numel") else key.shape[0])
            b.key, b.rowtime, b.val, b.val_null = kp, tp, vp, np_
            if rowtime_base is not None:   # (narrow columns are FG_HOST only: the engine says so)
                b.format, b.rowtime_base = L.BATCH_ROWTIME32, int(rowtime_base)
        else:
            fmt = 0
            if getattr(key, "dtype", None) == np.int32:
                fmt |= L.BATCH_KEY32
            key = np.ascontiguousarray(key, dtype=np.int32 if fmt & L.BATCH_KEY32 else np.int64)
            if rowtime_base is not None:
                fmt |= L.BATCH_ROWTIME32
                b.rowtime_base = int(rowtime_base)
            rowtime = np.ascontiguousarray(rowtime, dtype=np.uint32 if rowtime_base is not None else np.int64)
            b.location = L.HOST
            b.n = len(key)
            b.key, b.rowtime = key.ctypes.data, rowtime.ctypes.data
            if val is not None and self.val_type != L.VAL_NONE:
                narrow = self.val_type == L.VAL_I64 and getattr(val, "dtype", None) == np.int32
                fmt |= L.BATCH_VAL32 if narrow else 0
                val = np.ascontiguousarray(val, dtype=np.float64 if self.val_type == L.VAL_F64 else
                                           np.int32 if narrow else np.int64)
                b.val = val.ctypes.data
            b.format = fmt
            if val_null is not None:
                val_null = np.ascontiguousarray(val_null, dtype=np.uint8)
                b.val_null = val_null.ctypes.data
            keep = [key, rowtime, val, val_null]
        L.check(self._lib.fg_add_batch(self._h, C.byref(b)), self._h)
        self._hold((key, rowtime, val, val_null) if kdev else None)
        del keep

    def _hold(self, cols):
        """Device columns stay in use until the work the NEXT engine call queues has run (the
        engine finishes a batch's staging there; include/flinkgpu.h, fg_batch). Keep a reference
        to them until an event recorded on the engine stream after that call has completed, so
        that torch's caching allocator cannot hand their blocks to other work earlier. (Not
        record_stream: the allocator would record events on the engine stream when the block is
        freed, which may be after fg_close destroyed that stream.)"""
        prev = self.__dict__.get("_inflight")
        if prev is None and cols is None:   # (the watermark path between batches: nothing to do)
            return
        held = self.__dict__.setdefault("_held", [])
        ext = self.__dict__.get("_ext_stream")
        if prev is not None:
            if ext is None:
                held.append((None, prev))   # not torch tensors: kept until close
            else:
                import torch
                ev = torch.cuda.Event()
                ev.record(ext)
                held.append((ev, prev))
        if cols is not None:   # a new batch: release the columns whose event completed
            self._held = [(e, c) for e, c in held if e is None or not e.query()]
        self._inflight = cols

    def process_rows(self, rows, stride: int, arity: int, key_field: int = 0, rowtime_field: int = 1,
                     val_field: int = 2):
        """processElement for packed BinaryRowData rows (the fixed-length parts, `stride` bytes
        apart: flink_amd.rows.pack_rows writes them as BinaryRowWriter does): a uint8 numpy
        array / bytes on the host, or a uint8 device tensor."""
        self._after_producers((rows,))
        b = L.FgRowBatch()
        rp, rdev, rows = _dev_ptr(rows)
        keep = None
        if rdev:
            b.location = L.DEVICE
            b.rows = rp
            nbytes = int(rows.numel())
        else:
            keep = np.ascontiguousarray(np.frombuffer(rows, dtype=np.uint8) if isinstance(rows, (bytes, bytearray))
                                        else rows, dtype=np.uint8)
            b.location = L.HOST
            b.rows = keep.ctypes.data
            nbytes = keep.size
        b.stride = int(stride)
        b.n = nbytes // int(stride)
        b.arity, b.key_field, b.rowtime_field = int(arity), int(key_field), int(rowtime_field)
        b.val_field = int(val_field) if self.val_type != L.VAL_NONE else -1
        L.check(self._lib.fg_add_rows(self._h, C.byref(b)), self._h)
        self._hold((rows,) if rdev else None)
        del keep

    # -- global phase ----------------------------------------------------------------------------
    def process_partials(self, key, slice_end, cnt_star, cnt_val, sum_bits, min_bits=None, max_bits=None):
        """GlobalAggCombiner.combine for partial accumulator rows (after the exchange): numpy
        arrays or device tensors; `sum_bits` holds i64 sums or the bits of f64 sums. An operator
        with several value accumulators (SUM family, MIN, MAX) also takes the partial MIN / MAX
        (the local phase's agg[3] / agg[4])."""
        cols = [key, slice_end, cnt_star, cnt_val, sum_bits]
        if min_bits is not None:
            cols += [min_bits, max_bits]
        self._after_producers(cols)
        ptrs = [_dev_ptr(c) for c in cols]
        b = L.FgPartials()
        keep = []
        if ptrs[0][1]:
            assert all(p[1] for p in ptrs), "mixed host/device columns"
            b.location = L.DEVICE
            x = ptrs[0][2]
            b.n = int(x.numel() if hasattr(x, "numel") else x.shape[0])
            b.key, b.slice_end, b.cnt_star, b.cnt_val, b.sum = (p[0] for p in ptrs[:5])
            if len(ptrs) > 5:
                b.min, b.max = ptrs[5][0], ptrs[6][0]
        else:
            arrs = []
            for c in cols:
                a = np.asarray(c)
                if a.dtype == np.float64:
                    a = a.view(np.int64)
                arrs.append(np.ascontiguousarray(a, dtype=np.int64))
            b.location = L.HOST
            b.n = len(arrs[0])
            b.key, b.slice_end, b.cnt_star, b.cnt_val, b.sum = (a.ctypes.data for a in arrs[:5])
            if len(arrs) > 5:
                b.min, b.max = arrs[5].ctypes.data, arrs[6].ctypes.data
            keep = arrs
        L.check(self._lib.fg_add_partials(self._h, C.byref(b)), self._h)
        self._hold(None)
        del keep

    # -- processWatermark ---------------------------------------------------------------------
    def process_watermark(self, watermark: int, device_output: bool = False, wait: bool = True):
        """Advance event time; returns the rows fired by this watermark: a structured numpy
        array, or with device_output=True the operator's FgRows (device pointers, reused and
        valid until the next call on this operator). device_output=True, wait=False is
        fg_advance_progress_async: the fires are queued and the call returns None at once;
        collect_fired() waits for them and returns their rows."""
        if device_output and not wait:
            rc = self._lib.fg_advance_progress_async(self._h, int(watermark))
            if rc:
                L.check(rc, self._h)
            self._hold(None)
            return None
        if device_output:
            # one FgRows per operator: device rows are library-owned and valid until the next
            # call on this handle anyway; no per-call allocation on the watermark path
            rc = self._lib.fg_advance_progress(self._h, int(watermark), L.DEVICE, self._dev_rows_ref)
            if rc:
                L.check(rc, self._h)
            self._hold(None)
            return self._dev_rows
        r = L.FgRows()
        L.check(self._lib.fg_advance_progress(self._h, int(watermark), L.HOST, C.byref(r)), self._h)
        self._hold(None)
        return self._host_rows(r)

    def process_watermarks(self, watermarks):
        """process_watermark(wm, device_output=True, wait=False) of each watermark in order, in
        one library call (fg_advance_progress_async_n): the watermarks a shim holds between two
        batches; collect_fired() returns their rows."""
        if len(watermarks) == 0:
            return
        wm = np.ascontiguousarray(watermarks, dtype=np.int64)
        rc = self._lib.fg_advance_progress_async_n(self._h, wm.ctypes.data, len(wm))
        if rc:
            L.check(rc, self._h)
        self._hold(None)

    def collect_fired(self, host: bool = False):
        """The rows of the process_watermark(..., wait=False) calls since the last collect
        (fg_collect_fired: waits for their fires): the operator's FgRows, device pointers valid
        until the next call that fires; host=True: a structured numpy array copied out by the
        library (fg_collect_fired_to FG_HOST, what a JVM shim takes)."""
        if host:
            r = L.FgRows()
            L.check(self._lib.fg_collect_fired_to(self._h, L.HOST, C.byref(r)), self._h)
            return self._host_rows(r)
        L.check(self._lib.fg_collect_fired(self._h, self._dev_rows_ref), self._h)
        return self._dev_rows

    def rows_to_host(self, r: L.FgRows) -> np.ndarray:
        """Host copy of device FgRows (process_watermark(device_output=True) / collect_fired) in the
        layout of the host rows."""
        import torch

        class _Col:
            def __init__(self, ptr, typestr, n):
                self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (int(ptr or 0), False),
                                                 "version": 2}

        def col(ptr, dtype, count):
            ts = "|u1" if dtype is C.c_uint8 else "<i8"
            return torch.as_tensor(_Col(ptr, ts, count), device=torch.device("cuda", self.cfg.device_id)).cpu().numpy()

        torch.cuda.synchronize(self.cfg.device_id)   # (the rows are complete once collected; torch's copy runs on its stream)
        return self._host_rows(r, col)

    def _host_rows(self, r: L.FgRows, col=None) -> np.ndarray:
        n = r.n
        fields = [("key", "<i8"), ("window_start", "<i8"), ("window_end", "<i8")]
        for a in self.aggs:
            nm = AGG_NAMES[a]
            is_f = self.val_type == L.VAL_F64 and a in VALUE_TYPED
            fields.append((nm, "<f8" if is_f else "<i8"))
            fields.append((nm + "_null", "?"))
        if self.mode == L.MODE_DATASTREAM:
            fields.append(("rowtime", "<i8"))
        out = np.zeros(n, dtype=np.dtype(fields))
        if n == 0:
            return out

        if col is None:
            def col(ptr, dtype, count):
                return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(dtype)), shape=(count,)).copy()

        out["key"] = col(r.key, C.c_int64, n)
        out["window_start"] = col(r.window_start, C.c_int64, n)
        out["window_end"] = col(r.window_end, C.c_int64, n)
        nullm = col(r.null_mask, C.c_uint8, n)
        for i, a in enumerate(self.aggs):
            nm = AGG_NAMES[a]
            raw = col(r.agg[i], C.c_int64, n)
            out[nm] = raw.view(np.float64) if out.dtype[nm] == np.float64 else raw
            out[nm + "_null"] = (nullm >> i) & 1 == 1
        if self.mode == L.MODE_DATASTREAM:
            out["rowtime"] = col(r.rowtime, C.c_int64, n)
        return out

    # -- checkpointing ----------------------------------------------------------------------------
    def prepare_snapshot_pre_barrier(self):
        """Flush the staged buffer into the GPU-resident state (RecordsWindowBuffer.flush). A local
        operator (local_partials) keeps no state: its buffer flushes to the output instead -- the
        partial rows of every buffered slice are returned (flush_partials)."""
        if self.local_partials:
            return self.flush_partials()
        L.check(self._lib.fg_flush(self._h), self._h)
        self._hold(None)

    def flush_partials(self, device_output: bool = False):
        """Local phase: every buffered slice emits its partial accumulator rows now
        (LocalSlicingWindowAggOperator.prepareSnapshotPreBarrier -> WindowBuffer.flush ->
        LocalAggCombiner, fg_flush_partials); host rows as process_watermark returns them, or
        with device_output=True the operator's FgRows (device pointers, valid until the next call)."""
        if device_output:
            L.check(self._lib.fg_flush_partials(self._h, L.DEVICE, self._dev_rows_ref), self._h)
            self._hold(None)
            return self._dev_rows
        r = L.FgRows()
        L.check(self._lib.fg_flush_partials(self._h, L.HOST, C.byref(r)), self._h)
        self._hold(None)
        return self._host_rows(r)

    def snapshot_state(self, copy: bool = True):
        """(state image dict of numpy arrays, timer watermark): the window-aggs ValueState.
        copy=False returns views of the library-owned pinned host image (what a JNI shim hands
        to the state backend), valid until the next call on this operator."""
        s = L.FgStateRows()
        wm = C.c_int64()
        L.check(self._lib.fg_snapshot_state(self._h, C.byref(s), C.byref(wm)), self._h)
        return self._image(s, wm, copy)

    def snapshot_state_async(self):
        """snapshotState's synchronous part (fg_snapshot_state_async): the state as of this call
        is exported on the GPU and its copy to the host image queued; the operator takes
        batches and watermarks meanwhile. snapshot_state_wait returns the image."""
        L.check(self._lib.fg_snapshot_state_async(self._h), self._h)

    def snapshot_state_wait(self, copy: bool = True):
        """the image of the last snapshot_state_async (as snapshot_state returns it)"""
        s = L.FgStateRows()
        wm = C.c_int64()
        L.check(self._lib.fg_snapshot_state_wait(self._h, C.byref(s), C.byref(wm)), self._h)
        return self._image(s, wm, copy)

    def _image(self, s, wm, copy):
        n = s.n

        def col(p):
            if n == 0:
                return np.zeros(0, dtype=np.int64)
            a = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int64)), shape=(n,))
            return a.copy() if copy else a

        img = dict(key=col(s.key), slice_end=col(s.slice_end), cnt_star=col(s.cnt_star), cnt_val=col(s.cnt_val),
                   sum=col(s.sum))
        if s.min:   # several value accumulators: the MIN and MAX slots too
            img["min"], img["max"] = col(s.min), col(s.max)
        return img, wm.value

    def snapshot_slices(self) -> dict:
        """fg_snapshot_slices: the slices of the image the last snapshot returned -- slice_end,
        first_row, rows (its rows in the image), changed (written since the image before)."""
        s = L.FgImageSlices()
        L.check(self._lib.fg_snapshot_slices(self._h, C.byref(s)), self._h)
        n = int(s.n)

        def col(p, ct, dt):
            if n == 0:
                return np.zeros(0, dtype=dt)
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(ct)), shape=(n,)).copy()
        return dict(slice_end=col(s.slice_end, C.c_int64, np.int64), first_row=col(s.first_row, C.c_int64, np.int64),
                    rows=col(s.rows, C.c_int64, np.int64), changed=col(s.changed, C.c_uint8, np.uint8).astype(bool))

    def restore_state(self, image, timer_watermark: int):
        names = ("key", "slice_end", "cnt_star", "cnt_val", "sum") + (("min", "max") if "min" in image else ())
        cols = {k: np.ascontiguousarray(image[k], dtype=np.int64) for k in names}
        s = L.FgStateRows()
        s.n = len(cols["key"])
        for k in names:
            setattr(s, k, cols[k].ctypes.data)
        L.check(self._lib.fg_restore(self._h, C.byref(s), int(timer_watermark)), self._h)

    # -- metrics ------------------------------------------------------------------------------------
    @property
    def num_late_records_dropped(self) -> int:
        v = C.c_int64()
        L.check(self._lib.fg_late_dropped(self._h, C.byref(v)), self._h)
        return v.value

    def stats(self) -> dict:
        s = L.FgStats()
        L.check(self._lib.fg_get_stats(self._h, C.byref(s)), self._h)
        return {k: getattr(s, k) for k, _ in s._fields_}

    def reset(self):
        """Drop all state (a fresh operator restored from an empty snapshot), keep allocations."""
        L.check(self._lib.fg_reset(self._h), self._h)

    def kernel_stats(self) -> dict:
        """{kernel: dict(launches, total_ms, records, rows)} (needs kernel_timing=True)."""
        arr = (L.FgKernelStat * 32)()
        n = C.c_int32()
        L.check(self._lib.fg_kernel_stats(self._h, arr, 32, C.byref(n)), self._h)
        return {arr[i].name.decode(): dict(launches=arr[i].launches, total_ms=arr[i].total_ms,
                                           records=arr[i].records, rows=arr[i].rows) for i in range(min(n.value, 32))}

    def set_kernel_timing(self, classes=None):
        """Time only the named kernel classes (names of kernel_stats); None: all."""
        mask = 0xFFFFFFFF
        if classes is not None:
            names = list(self.kernel_stats())
            mask = 0
            for c in classes:
                mask |= 1 << names.index(c)
        L.check(self._lib.fg_set_kernel_timing(self._h, mask), self._h)

    def synchronize(self):
        L.check(self._lib.fg_synchronize(self._h), self._h)

    @property
    def stream(self) -> int:
        return self._lib.fg_stream(self._h) or 0


def key_groups(keys, max_parallelism: int = 128, key_hash: int = L.KEYHASH_BINARYROW_BIGINT, device: int = 0):
    """KeyGroupRangeAssignment.assignToKeyGroup on the GPU (numpy in, numpy out)."""
    lib = L.load()
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    out = np.empty(len(keys), dtype=np.int32)
    L.check(lib.fg_key_groups(device, L.HOST, len(keys), keys.ctypes.data, key_hash, max_parallelism,
                              out.ctypes.data))
    return out
