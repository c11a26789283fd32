"""ORACLE -- test infrastructure only.

ctypes front-end for ``liboracle.so``, the plain-C restatement of the reference CPU
operators (see ``oracle.h``).  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the checker or
the reported CPU baseline: the product path (``flink_amd``) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

MODE_SQL, MODE_DATASTREAM = 0, 1
TUMBLE, HOP, CUMULATE = 0, 1, 2
PHASE_SINGLE, PHASE_LOCAL, PHASE_GLOBAL = 0, 1, 2
VAL_NONE, VAL_I64, VAL_F64 = 0, 1, 2
JMIN = -(1 << 63)
JMAX = (1 << 63) - 1


class Config(C.Structure):
    _fields_ = [
        ("mode", C.c_int32),
        ("kind", C.c_int32),
        ("size", C.c_int64),
        ("slide", C.c_int64),
        ("offset", C.c_int64),
        ("tz_offset_ms", C.c_int64),
        ("val_type", C.c_int32),
        ("count_star_index", C.c_int32),
        ("proctime", C.c_int32),
        ("tz_n", C.c_int32),
        ("tz_trans", C.c_void_p),
        ("tz_offs", C.c_void_p),
        ("tz_use_dst", C.c_int32),
        ("windowed", C.c_int32),
        ("phase", C.c_int32),
        ("purging", C.c_int32),
        ("allowed_lateness", C.c_int64),
    ]


class Row(C.Structure):
    _fields_ = [
        ("key", C.c_int64),
        ("window_start", C.c_int64),
        ("window_end", C.c_int64),
        ("cnt_star", C.c_int64),
        ("cnt_val", C.c_int64),
        ("sum_i", C.c_int64),
        ("sum_d", C.c_double),
        ("avg_i", C.c_int64),
        ("avg_d", C.c_double),
        ("sum_null", C.c_int32),
        ("avg_null", C.c_int32),
        ("out_ts", C.c_int64),
        ("sum0_i", C.c_int64),
        ("sum0_d", C.c_double),
        ("min_i", C.c_int64),
        ("max_i", C.c_int64),
        ("min_d", C.c_double),
        ("max_d", C.c_double),
    ]


ROW_DTYPE = np.dtype(
    [
        ("key", "<i8"), ("window_start", "<i8"), ("window_end", "<i8"),
        ("cnt_star", "<i8"), ("cnt_val", "<i8"), ("sum_i", "<i8"), ("sum_d", "<f8"),
        ("avg_i", "<i8"), ("avg_d", "<f8"), ("sum_null", "<i4"), ("avg_null", "<i4"),
        ("out_ts", "<i8"), ("sum0_i", "<i8"), ("sum0_d", "<f8"),
        ("min_i", "<i8"), ("max_i", "<i8"), ("min_d", "<f8"), ("max_d", "<f8"),
    ]
)
assert ROW_DTYPE.itemsize == C.sizeof(Row)

_lib = None


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        i64p = C.POINTER(C.c_int64)
        L.or_open.restype = P
        L.or_open.argtypes = [C.POINTER(Config), C.c_char_p, C.c_int]
        L.or_close.argtypes = [P]
        L.or_process_batch.argtypes = [P, C.c_int64, P, P, P, P]
        L.or_process_watermark.argtypes = [P, C.c_int64]
        L.or_process_partials.argtypes = [P, C.c_int64, P]
        L.or_prepare_snapshot.argtypes = [P]
        L.or_restore_copy.restype = P
        L.or_restore_copy.argtypes = [P]
        L.or_num_rows.restype = C.c_int64
        L.or_num_rows.argtypes = [P]
        L.or_rows.restype = P
        L.or_rows.argtypes = [P]
        L.or_clear_rows.argtypes = [P]
        for fn in ("or_late_dropped", "or_state_entries", "or_pending_timers"):
            getattr(L, fn).restype = C.c_int64
            getattr(L, fn).argtypes = [P]
        for fn in ("or_assign_slice_end", "or_get_window_start", "or_get_last_window_end", "or_to_utc",
                   "or_to_epoch_for_timer", "or_to_epoch", "or_next_trigger"):
            getattr(L, fn).restype = C.c_int64
            getattr(L, fn).argtypes = [P, C.c_int64]
        L.or_expired_slices.restype = C.c_int32
        L.or_expired_slices.argtypes = [P, C.c_int64, i64p]
        L.or_merge_slices.restype = C.c_int32
        L.or_merge_slices.argtypes = [P, C.c_int64, i64p, i64p, C.c_int32]
        L.or_next_trigger_window.restype = C.c_int32
        L.or_next_trigger_window.argtypes = [P, C.c_int64, C.c_int32, i64p]
        L.or_next_trigger_watermark.restype = C.c_int64
        L.or_next_trigger_watermark.argtypes = [C.c_int64, C.c_int64]
        L.or_window_start_with_offset.restype = C.c_int64
        L.or_window_start_with_offset.argtypes = [C.c_int64, C.c_int64, C.c_int64]
        for fn in ("or_binaryrow_hash_i64", "or_long_hash"):
            getattr(L, fn).restype = C.c_int32
            getattr(L, fn).argtypes = [C.c_int64]
        L.or_binaryrow_hash_bytes.restype = C.c_int32
        L.or_binaryrow_hash_bytes.argtypes = [P, C.c_int32]
        L.or_murmur_hash.restype = C.c_int32
        L.or_murmur_hash.argtypes = [C.c_int32]
        L.or_key_group.restype = C.c_int32
        L.or_key_group.argtypes = [C.c_int32, C.c_int32]
        L.or_operator_index.restype = C.c_int32
        L.or_operator_index.argtypes = [C.c_int32, C.c_int32, C.c_int32]
        L.or_default_max_parallelism.restype = C.c_int32
        L.or_default_max_parallelism.argtypes = [C.c_int32]
        L.or_key_groups_binaryrow.argtypes = [C.c_int64, P, C.c_int32, P]
        L.or_run_partitioned.restype = C.c_double
        L.or_run_partitioned.argtypes = [
            C.POINTER(Config), C.c_int32, C.c_int32, C.c_int64, P, P, P, C.c_int32, P, P,
            i64p, C.POINTER(C.c_uint64), i64p,
        ]
        L.or_run_partitioned_rows.restype = C.c_double
        L.or_run_partitioned_rows.argtypes = [
            C.POINTER(Config), C.c_int32, C.c_int32, C.c_int64, P, P, P, C.c_int32, P, P, C.c_int32,
            C.POINTER(C.c_void_p), i64p, i64p,
        ]
        L.or_free.argtypes = [P]
        L.or_ds_export_state.restype = C.c_int64
        L.or_ds_export_state.argtypes = [P, P, P, P, P, P, P]
        L.or_export_timers.restype = C.c_int64
        L.or_export_timers.argtypes = [P, P, P, P]
        L.or_ds_import.restype = P
        L.or_ds_import.argtypes = [C.POINTER(Config), C.c_int64, P, P, P, P, C.c_int64, P, P, P, C.c_char_p, C.c_int]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


class OracleOperator:
    """The reference operator restated: processElement / processWatermark /
    prepareSnapshotPreBarrier / snapshot-restore, with fired rows collected."""

    def __init__(self, mode=MODE_SQL, kind=TUMBLE, size=1000, slide=0, offset=0, tz_offset_ms=0,
                 val_type=VAL_F64, count_star_index=0, proctime=False, _handle=None, zone=None, windowed=False,
                 phase=PHASE_SINGLE, allowed_lateness=0, purging=False):
        """zone: an IANA zone name whose rules (transitions, daylight saving) replace the fixed
        tz_offset_ms (TimeWindowUtil with a ZoneId). phase: PHASE_LOCAL / PHASE_GLOBAL for the
        two halves of the two-phase plan (LocalSlicingWindowAggOperator + LocalAggCombiner;
        SlicingWindowOperator over the `sliced` assigner + GlobalAggCombiner)."""
        self.cfg = Config(mode, kind, size, slide, offset, tz_offset_ms, val_type, count_star_index,
                          1 if proctime else 0, 0)
        self.cfg.windowed = 1 if windowed else 0
        self.cfg.phase = phase
        self.cfg.allowed_lateness = int(allowed_lateness)   # DataStream WindowOperator.allowedLateness
        self.cfg.purging = 1 if purging else 0              # PurgingTrigger.of(EventTimeTrigger)
        self.zone = zone
        if zone is not None:
            from flink_amd.tz import zone_rules
            tr, of, dst = zone_rules(zone)
            self._tz = (np.ascontiguousarray(tr), np.ascontiguousarray(of))
            self.cfg.tz_n = len(tr)
            self.cfg.tz_trans = self._tz[0].ctypes.data if len(tr) else None
            self.cfg.tz_offs = self._tz[1].ctypes.data
            self.cfg.tz_use_dst = 1 if dst else 0
            if len(tr) == 0:   # a zone that never changed offset: the fixed-offset path
                self.cfg.tz_offset_ms = int(of[0])
        L = lib()
        if _handle is None:
            err = C.create_string_buffer(512)
            h = L.or_open(C.byref(self.cfg), err, 512)
            if not h:
                raise ValueError(err.value.decode())
            self._h = h
        else:
            self._h = _handle

    def close(self):
        if self._h:
            lib().or_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process_batch(self, key, ts, val=None, isnull=None):
        key = np.ascontiguousarray(key, dtype=np.int64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        if val is not None:
            val = np.ascontiguousarray(val)
            assert val.dtype.itemsize == 8
        if isnull is not None:
            isnull = np.ascontiguousarray(isnull, dtype=np.uint8)
        lib().or_process_batch(self._h, len(key), _ptr(key), _ptr(ts), _ptr(val), _ptr(isnull))

    def process_watermark(self, wm: int):
        lib().or_process_watermark(self._h, int(wm))

    def process_partials(self, rows):
        """Global phase: partial accumulator rows (ROW_DTYPE) of local-phase operators."""
        rows = np.ascontiguousarray(rows, dtype=ROW_DTYPE)
        lib().or_process_partials(self._h, len(rows), rows.ctypes.data if len(rows) else None)

    def prepare_snapshot(self):
        lib().or_prepare_snapshot(self._h)

    def restore_copy(self) -> "OracleOperator":
        h = lib().or_restore_copy(self._h)
        c = self.cfg
        return OracleOperator(c.mode, c.kind, c.size, c.slide, c.offset, c.tz_offset_ms, c.val_type,
                              c.count_star_index, _handle=h, zone=self.zone, windowed=bool(c.windowed),
                              phase=c.phase)

    # DataStream WindowOperator keyed state ("window-contents" + "window-timers")
    def ds_state_image(self, agg: str = "sum") -> dict:
        """The operator's heap-backend image: per (key, TimeWindow) the reduced value's field bits
        (agg: the aggregator's field -- "sum", "min" or "max"; "avg" / "count": the sum) and the
        record count (an aggregate function's count), and every pending timer (key, window end,
        timestamp)."""
        L = lib()
        n = self.state_entries
        a = {k: np.zeros(n, dtype=np.int64) for k in ("key", "window_end", "cnt", "sum", "min", "max")}
        L.or_ds_export_state(self._h, *(_ptr(a[k]) for k in ("key", "window_end", "cnt", "sum", "min", "max")))
        nt = self.pending_timers
        t = {k: np.zeros(nt, dtype=np.int64) for k in ("timer_key", "timer_window_end", "timer_ts")}
        L.or_export_timers(self._h, *(_ptr(t[k]) for k in ("timer_key", "timer_window_end", "timer_ts")))
        img = dict(key=a["key"], window_end=a["window_end"], window_start=a["window_end"] - self.cfg.size,
                   value=a["sum" if agg in ("avg", "count") else agg], count=a["cnt"])
        img.update(t)
        return img

    @classmethod
    def from_ds_state_image(cls, image: dict, kind=TUMBLE, size=1000, slide=0, offset=0, val_type=VAL_I64,
                            allowed_lateness=0, purging=False) -> "OracleOperator":
        """A DataStream operator restored from a ds_state_image-shaped image."""
        cfg = Config(MODE_DATASTREAM, kind, size, slide, offset, 0, val_type, 0, 0, 0)
        cfg.allowed_lateness = int(allowed_lateness)
        cfg.purging = 1 if purging else 0
        c = {k: np.ascontiguousarray(image[k], dtype=np.int64) for k in
             ("key", "window_end", "timer_key", "timer_window_end", "timer_ts")}
        n = len(c["key"])
        c["value"] = np.ascontiguousarray(image["value"], dtype=np.int64) if "value" in image else np.zeros(n, np.int64)
        cnt = np.ascontiguousarray(image["count"], dtype=np.int64) if "count" in image else None
        err = C.create_string_buffer(512)
        h = lib().or_ds_import(C.byref(cfg), n, _ptr(c["key"]), _ptr(c["window_end"]), _ptr(c["value"]), _ptr(cnt),
                               len(c["timer_key"]), _ptr(c["timer_key"]), _ptr(c["timer_window_end"]),
                               _ptr(c["timer_ts"]), err, 512)
        if not h:
            raise ValueError(err.value.decode())
        return cls(MODE_DATASTREAM, kind, size, slide, offset, 0, val_type, 0, _handle=h,
                   allowed_lateness=allowed_lateness, purging=purging)

    def take_rows(self) -> np.ndarray:
        L = lib()
        n = L.or_num_rows(self._h)
        if n == 0:
            out = np.zeros(0, dtype=ROW_DTYPE)
        else:
            buf = (C.c_char * (n * ROW_DTYPE.itemsize)).from_address(L.or_rows(self._h))
            out = np.frombuffer(bytes(buf), dtype=ROW_DTYPE).copy()
        L.or_clear_rows(self._h)
        return out

    @property
    def late_dropped(self) -> int:
        return lib().or_late_dropped(self._h)

    @property
    def state_entries(self) -> int:
        return lib().or_state_entries(self._h)

    @property
    def pending_timers(self) -> int:
        return lib().or_pending_timers(self._h)

    # slice assigner restatement
    def assign_slice_end(self, ts):
        return lib().or_assign_slice_end(self._h, ts)

    def window_start(self, w):
        return lib().or_get_window_start(self._h, w)

    # TimeWindowUtil with this operator's zone
    def to_utc(self, epoch):
        return lib().or_to_utc(self._h, epoch)

    def to_epoch_for_timer(self, local):
        return lib().or_to_epoch_for_timer(self._h, local)

    def to_epoch(self, local):
        return lib().or_to_epoch(self._h, local)

    def next_trigger(self, wm):
        return lib().or_next_trigger(self._h, wm)

    def last_window_end(self, s):
        return lib().or_get_last_window_end(self._h, s)

    def expired_slices(self, w):
        out = (C.c_int64 * 2)()
        n = lib().or_expired_slices(self._h, w, out)
        return [out[i] for i in range(n)]

    def merge_slices(self, s):
        out = (C.c_int64 * 100000)()
        mr = C.c_int64()
        n = lib().or_merge_slices(self._h, s, C.byref(mr), out, 100000)
        return (None if mr.value == JMIN else mr.value), [out[i] for i in range(n)]

    def next_trigger_window(self, w, is_empty):
        nx = C.c_int64()
        ok = lib().or_next_trigger_window(self._h, w, int(bool(is_empty)), C.byref(nx))
        return nx.value if ok else None


def next_trigger_watermark(wm, interval):
    return lib().or_next_trigger_watermark(wm, interval)


def binaryrow_hash_i64(key: int) -> int:
    return lib().or_binaryrow_hash_i64(key)


def binaryrow_hash_bytes(row: bytes) -> int:
    """BinarySection.hashCode of a serialized row (any key type)."""
    buf = (C.c_uint8 * max(len(row), 1)).from_buffer_copy(row or b"\0")
    return lib().or_binaryrow_hash_bytes(buf, len(row))


def key_group_of_row(row: bytes, max_parallelism: int) -> int:
    """KeyGroupRangeAssignment.assignToKeyGroup(keyRow, maxP) for a BinaryRowData key row."""
    return key_group(binaryrow_hash_bytes(row), max_parallelism)


def long_hash(key: int) -> int:
    return lib().or_long_hash(key)


def murmur_hash(code: int) -> int:
    return lib().or_murmur_hash(code)


def key_group(key_hash: int, max_parallelism: int) -> int:
    return lib().or_key_group(key_hash, max_parallelism)


def operator_index(max_parallelism, parallelism, kg):
    return lib().or_operator_index(max_parallelism, parallelism, kg)


def default_max_parallelism(p):
    return lib().or_default_max_parallelism(p)


def key_groups_binaryrow(keys: np.ndarray, max_parallelism: int) -> np.ndarray:
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    out = np.empty(len(keys), dtype=np.int32)
    lib().or_key_groups_binaryrow(len(keys), _ptr(keys), max_parallelism, _ptr(out))
    return out


def run_partitioned(cfg: Config, parallelism, max_parallelism, key, ts, val, wm_at, wm_val):
    """CPU baseline: `parallelism` operator instances (pthreads), records routed by key group."""
    key = np.ascontiguousarray(key, dtype=np.int64)
    ts = np.ascontiguousarray(ts, dtype=np.int64)
    val = None if val is None else np.ascontiguousarray(val)
    wm_at = np.ascontiguousarray(wm_at, dtype=np.int64)
    wm_val = np.ascontiguousarray(wm_val, dtype=np.int64)
    rows = C.c_int64()
    cs = C.c_uint64()
    late = C.c_int64()
    el = lib().or_run_partitioned(C.byref(cfg), parallelism, max_parallelism, len(key), _ptr(key), _ptr(ts),
                                  _ptr(val), len(wm_at), _ptr(wm_at), _ptr(wm_val), C.byref(rows),
                                  C.byref(cs), C.byref(late))
    return el, rows.value, cs.value, late.value


def run_partitioned_rows(cfg: Config, parallelism, max_parallelism, key, ts, val, wm_at, wm_val, snapshot_after=-1):
    """Every fired row of `parallelism` key-group-routed operator instances (ROW_DTYPE), the
    late-drop count and the elapsed seconds; snapshot_after >= 0 takes a checkpoint and
    restores from it after that watermark (or_run_partitioned_rows)."""
    key = np.ascontiguousarray(key, dtype=np.int64)
    ts = np.ascontiguousarray(ts, dtype=np.int64)
    val = None if val is None else np.ascontiguousarray(val)
    wm_at = np.ascontiguousarray(wm_at, dtype=np.int64)
    wm_val = np.ascontiguousarray(wm_val, dtype=np.int64)
    rp = C.c_void_p()
    nr = C.c_int64()
    late = C.c_int64()
    L = lib()
    el = L.or_run_partitioned_rows(C.byref(cfg), parallelism, max_parallelism, len(key), _ptr(key), _ptr(ts),
                                   _ptr(val), len(wm_at), _ptr(wm_at), _ptr(wm_val), int(snapshot_after),
                                   C.byref(rp), C.byref(nr), C.byref(late))
    n = nr.value
    try:
        if n == 0:
            rows = np.zeros(0, dtype=ROW_DTYPE)
        else:
            buf = (C.c_char * (n * ROW_DTYPE.itemsize)).from_address(rp.value)
            rows = np.frombuffer(buf, dtype=ROW_DTYPE).copy()
    finally:
        L.or_free(rp)
    return rows, late.value, el
