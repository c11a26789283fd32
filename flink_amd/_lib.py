"""ctypes binding of libflinkgpu.so (the C-ABI declared in include/flinkgpu.h).

The library is built in-tree (``flink_amd/libflinkgpu.so``, flink_amd/Makefile via __graft_entry__.build()).
There is no fallback: if the library is missing or cannot be loaded, importing the
engine raises -- the product path never runs on a CPU substitute.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FLINKGPU_LIB", os.path.join(HERE, "libflinkgpu.so"))   # override: diagnostic builds

FG_OK, FG_EINVAL, FG_EFULL, FG_EDEVICE, FG_ECAPACITY, FG_ESTATE = range(6)
MODE_SQL, MODE_DATASTREAM = 0, 1
TUMBLE, HOP, CUMULATE = 0, 1, 2
VAL_NONE, VAL_I64, VAL_F64 = 0, 1, 2
AGG_COUNT_STAR, AGG_COUNT, AGG_SUM, AGG_AVG, AGG_SUM0, AGG_MIN, AGG_MAX = 0, 1, 2, 3, 4, 5, 6
HOST, DEVICE = 0, 1
KEYHASH_BINARYROW_BIGINT, KEYHASH_JAVA_LONG, KEYHASH_DICT_ID = 0, 1, 2
MAX_AGGS = 8


class FgConfig(C.Structure):
    _fields_ = [
        ("mode", C.c_int32), ("window_kind", C.c_int32),
        ("size_ms", C.c_int64), ("slide_ms", C.c_int64), ("offset_ms", C.c_int64),
        ("shift_tz_offset_ms", C.c_int64),
        ("val_type", C.c_int32), ("num_aggs", C.c_int32), ("aggs", C.c_int32 * MAX_AGGS),
        ("max_parallelism", C.c_int32), ("key_group_start", C.c_int32), ("key_group_end", C.c_int32),
        ("device_id", C.c_int32), ("flags", C.c_int32),
        ("expected_keys", C.c_int64), ("buffer_records", C.c_int64),
        ("tz_transition_ms", C.c_void_p), ("tz_offset_ms", C.c_void_p),
        ("n_tz_transitions", C.c_int32), ("tz_use_daylight", C.c_int32),
        ("allowed_lateness_ms", C.c_int64),
    ]


class FgBatch(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("location", C.c_int32), ("format", C.c_int32),
        ("key", C.c_void_p), ("rowtime", C.c_void_p), ("val", C.c_void_p), ("val_null", C.c_void_p),
        ("rowtime_base", C.c_int64),
    ]


class FgRowBatch(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("location", C.c_int32), ("stride", C.c_int32), ("rows", C.c_void_p),
        ("arity", C.c_int32), ("key_field", C.c_int32), ("rowtime_field", C.c_int32), ("val_field", C.c_int32),
    ]


class FgRows(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("location", C.c_int32), ("num_aggs", C.c_int32),
        ("key", C.c_void_p), ("window_start", C.c_void_p), ("window_end", C.c_void_p),
        ("agg", C.c_void_p * MAX_AGGS), ("null_mask", C.c_void_p), ("rowtime", C.c_void_p),
    ]


class FgStateRows(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("key", C.c_void_p), ("slice_end", C.c_void_p), ("cnt_star", C.c_void_p),
        ("cnt_val", C.c_void_p), ("sum", C.c_void_p), ("min", C.c_void_p), ("max", C.c_void_p),
    ]


class FgPartials(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("location", C.c_int32), ("reserved0", C.c_int32),
        ("key", C.c_void_p), ("slice_end", C.c_void_p), ("cnt_star", C.c_void_p), ("cnt_val", C.c_void_p),
        ("sum", C.c_void_p), ("min", C.c_void_p), ("max", C.c_void_p),
    ]


class FgExchanged(C.Structure):
    _fields_ = [("n", C.c_int64), ("ncols", C.c_int32), ("reserved0", C.c_int32), ("cols", C.c_void_p * 8),
                ("min_watermark", C.c_int64), ("bytes_sent", C.c_int64)]


COMM_ID_BYTES = 128
ROUND_FIRED, ROUND_FLUSHED, ROUND_IDLE = 0, 1, 2


class FgRound(C.Structure):
    _fields_ = [("min_watermark", C.c_int64), ("min_epoch", C.c_int64), ("rows_sent", C.c_int64),
                ("rows_received", C.c_int64), ("bytes_sent", C.c_int64), ("failed_rank", C.c_int32),
                ("reserved0", C.c_int32)]


class FgImageSlices(C.Structure):
    _fields_ = [("n", C.c_int64), ("slice_end", C.c_void_p), ("first_row", C.c_void_p), ("rows", C.c_void_p),
                ("changed", C.c_void_p)]


class FgStats(C.Structure):
    _fields_ = [(n, C.c_int64) for n in (
        "records_in", "records_staged", "late_dropped", "rows_fired", "flushes", "live_slices",
        "state_regions", "region_capacity")]


class FgKernelStat(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_int64), ("total_ms", C.c_double),
                ("records", C.c_int64), ("rows", C.c_int64)]


FLAG_KERNEL_TIMING = 1
FLAG_LOCAL_PARTIALS = 2
FLAG_PROCTIME = 4
FLAG_WINDOWED = 8
FLAG_PURGING_TRIGGER = 16
BATCH_KEY32, BATCH_ROWTIME32, BATCH_VAL32 = 1, 2, 4   # fg_batch.format

# every symbol include/flinkgpu.h declares
EXPORTS = (
    "fg_open", "fg_add_batch", "fg_add_rows", "fg_add_partials", "fg_advance_progress", "fg_advance_progress_async",
    "fg_advance_progress_async_n",
    "fg_collect_fired", "fg_collect_fired_to", "fg_flush", "fg_flush_partials", "fg_snapshot_state",
    "fg_snapshot_state_async", "fg_snapshot_state_wait", "fg_snapshot_slices", "fg_selftest", "fg_restore", "fg_late_dropped", "fg_get_stats", "fg_synchronize", "fg_reset", "fg_kernel_stats", "fg_set_kernel_timing",
    "fg_stream",
    "fg_last_error", "fg_close", "fg_key_groups", "fg_partition_by_owner", "fg_partition_columns_by_owner",
    "fg_abi_version", "fg_key_dict_open", "fg_key_dict_intern", "fg_key_dict_intern_async",
    "fg_key_dict_intern_wait", "fg_key_dict_lookup", "fg_key_dict_arena",
    "fg_key_dict_copy_arena", "fg_key_dict_size", "fg_key_dict_stream", "fg_key_dict_set_timing",
    "fg_key_dict_kernel_stats", "fg_key_dict_last_error", "fg_key_dict_close",
    "fg_binaryrow_hash", "fg_host_register", "fg_host_unregister",
    "fg_comm_unique_id", "fg_comm_open", "fg_comm_exchange_columns", "fg_comm_exchange_partials",
    "fg_comm_exchange_fired", "fg_comm_exchange_flushed", "fg_comm_round_begin", "fg_comm_round_exchange",
    "fg_comm_round_end", "fg_comm_stream", "fg_comm_bytes_sent", "fg_comm_last_error", "fg_comm_close",
)

_lib = None


class FlinkGpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[fg error {code}] {msg}")
        self.code = code
        self.msg = msg


class WindowSpecError(ValueError):
    """IllegalArgumentException of the reference (same message)."""


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so.7 (same
    # SONAME as /opt/rocm's). Loading torch first makes libflinkgpu bind to that instance
    # instead of starting a second runtime that would hide the GPU from torch.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    L.fg_open.argtypes = [C.POINTER(FgConfig), C.POINTER(P)]
    L.fg_add_batch.argtypes = [P, C.POINTER(FgBatch)]
    L.fg_add_rows.argtypes = [P, C.POINTER(FgRowBatch)]
    L.fg_add_partials.argtypes = [P, C.POINTER(FgPartials)]
    L.fg_advance_progress.argtypes = [P, C.c_int64, C.c_int32, C.POINTER(FgRows)]
    L.fg_advance_progress_async.argtypes = [P, C.c_int64]
    L.fg_advance_progress_async_n.argtypes = [P, P, C.c_int64]
    L.fg_collect_fired.argtypes = [P, C.POINTER(FgRows)]
    L.fg_collect_fired_to.argtypes = [P, C.c_int32, C.POINTER(FgRows)]
    L.fg_flush_partials.argtypes = [P, C.c_int32, C.POINTER(FgRows)]
    L.fg_flush.argtypes = [P]
    L.fg_snapshot_state.argtypes = [P, C.POINTER(FgStateRows), C.POINTER(C.c_int64)]
    L.fg_snapshot_state_async.argtypes = [P]
    L.fg_snapshot_state_wait.argtypes = [P, C.POINTER(FgStateRows), C.POINTER(C.c_int64)]
    L.fg_restore.argtypes = [P, C.POINTER(FgStateRows), C.c_int64]
    L.fg_late_dropped.argtypes = [P, C.POINTER(C.c_int64)]
    L.fg_get_stats.argtypes = [P, C.POINTER(FgStats)]
    L.fg_synchronize.argtypes = [P]
    L.fg_reset.argtypes = [P]
    L.fg_kernel_stats.argtypes = [P, C.POINTER(FgKernelStat), C.c_int32, C.POINTER(C.c_int32)]
    L.fg_set_kernel_timing.argtypes = [P, C.c_uint32]
    L.fg_set_kernel_timing.restype = C.c_int
    L.fg_stream.argtypes = [P]
    L.fg_stream.restype = P
    L.fg_last_error.argtypes = [P]
    L.fg_last_error.restype = C.c_char_p
    L.fg_close.argtypes = [P]
    L.fg_close.restype = None
    L.fg_key_groups.argtypes = [C.c_int32, C.c_int32, C.c_int64, P, C.c_int32, C.c_int32, P]
    L.fg_partition_by_owner.argtypes = [C.c_int32, P, C.c_int64, P, P, P, C.c_int32, C.c_int32, C.c_int32,
                                        P, P, P, P]
    L.fg_partition_columns_by_owner.argtypes = [C.c_int32, P, C.c_int64, C.c_int32, P, C.c_int32, C.c_int32,
                                                C.c_int32, P, P]
    L.fg_abi_version.restype = C.c_int
    L.fg_key_dict_open.argtypes = [C.c_int32, C.c_int32, C.c_int64, C.POINTER(P)]
    L.fg_key_dict_intern.argtypes = [P, C.c_int32, C.c_int64, P, C.c_int64, P, P, P, P]
    L.fg_key_dict_intern_async.argtypes = [P, C.c_int64, P, C.c_int64, P, P, P, P]
    L.fg_key_dict_intern_wait.argtypes = [P]
    L.fg_key_dict_lookup.argtypes = [P, C.c_int32, C.c_int64, P, P, P]
    L.fg_key_dict_arena.argtypes = [P, C.POINTER(P), C.POINTER(C.c_int64)]
    L.fg_key_dict_copy_arena.argtypes = [P, C.c_int64, C.c_int64, P]
    L.fg_key_dict_size.argtypes = [P]
    L.fg_key_dict_size.restype = C.c_int64
    L.fg_key_dict_set_timing.argtypes = [P, C.c_int32]
    L.fg_key_dict_set_timing.restype = C.c_int
    L.fg_key_dict_kernel_stats.argtypes = [P, C.POINTER(FgKernelStat), C.c_int32, C.POINTER(C.c_int32)]
    L.fg_key_dict_kernel_stats.restype = C.c_int
    L.fg_key_dict_stream.argtypes = [P]
    L.fg_key_dict_stream.restype = P
    L.fg_key_dict_last_error.argtypes = [P]
    L.fg_key_dict_last_error.restype = C.c_char_p
    L.fg_key_dict_close.argtypes = [P]
    L.fg_key_dict_close.restype = None
    L.fg_binaryrow_hash.argtypes = [P, C.c_int32]
    L.fg_binaryrow_hash.restype = C.c_int32
    L.fg_host_register.argtypes = [C.c_int32, P, C.c_int64]
    L.fg_host_unregister.argtypes = [C.c_int32, P]
    L.fg_host_register.restype = L.fg_host_unregister.restype = C.c_int
    L.fg_comm_unique_id.argtypes = [P]
    L.fg_comm_open.argtypes = [C.c_int32, C.c_int32, C.c_int32, P, C.POINTER(P)]
    L.fg_comm_exchange_columns.argtypes = [P, P, C.c_int64, C.c_int32, P, C.c_int32, C.c_int32, C.c_int64,
                                           C.POINTER(FgExchanged)]
    L.fg_comm_exchange_partials.argtypes = [P, P, C.POINTER(FgRows), C.c_int32, C.c_int32, C.c_int64, P,
                                            C.POINTER(C.c_int64)]
    L.fg_comm_exchange_fired.argtypes = [P, P, C.c_int32, C.c_int32, C.c_int64, P, C.POINTER(C.c_int64)]
    L.fg_comm_exchange_flushed.argtypes = [P, P, C.c_int32, C.c_int32, C.c_int64, P, C.POINTER(C.c_int64)]
    L.fg_comm_round_begin.argtypes = [P, P, C.c_int32, C.c_int32, C.c_int32, C.c_int64, C.c_int64]
    L.fg_comm_round_exchange.argtypes = [P, C.POINTER(FgRound)]
    L.fg_comm_round_end.argtypes = [P, P]
    L.fg_snapshot_slices.argtypes = [P, C.POINTER(FgImageSlices)]
    L.fg_selftest.argtypes = [C.c_int32, C.c_char_p, C.c_int32]
    L.fg_selftest.restype = C.c_int
    L.fg_comm_bytes_sent.argtypes = [P]
    L.fg_comm_bytes_sent.restype = C.c_int64
    L.fg_comm_stream.argtypes = [P]
    L.fg_comm_stream.restype = P
    L.fg_comm_last_error.argtypes = [P]
    L.fg_comm_last_error.restype = C.c_char_p
    L.fg_comm_close.argtypes = [P]
    L.fg_comm_close.restype = None
    for fn in ("fg_comm_unique_id", "fg_comm_open", "fg_comm_exchange_columns", "fg_comm_exchange_partials",
               "fg_comm_exchange_fired", "fg_comm_exchange_flushed", "fg_comm_round_begin", "fg_comm_round_exchange",
               "fg_comm_round_end"):
        getattr(L, fn).restype = C.c_int
    for fn in ("fg_key_dict_open", "fg_key_dict_intern", "fg_key_dict_intern_async", "fg_key_dict_intern_wait",
               "fg_key_dict_lookup", "fg_key_dict_arena",
               "fg_key_dict_copy_arena"):
        getattr(L, fn).restype = C.c_int
    for fn in ("fg_open", "fg_add_batch", "fg_add_rows", "fg_add_partials", "fg_advance_progress",
               "fg_advance_progress_async", "fg_advance_progress_async_n", "fg_collect_fired", "fg_collect_fired_to", "fg_flush", "fg_flush_partials",
               "fg_snapshot_state", "fg_snapshot_state_async", "fg_snapshot_state_wait", "fg_snapshot_slices", "fg_restore", "fg_late_dropped", "fg_get_stats", "fg_synchronize", "fg_reset", "fg_kernel_stats", "fg_key_groups",
               "fg_partition_by_owner", "fg_partition_columns_by_owner"):
        getattr(L, fn).restype = C.c_int
    _lib = L
    return L


def check(rc: int, handle=None):
    if rc == FG_OK:
        return
    msg = load().fg_last_error(handle).decode(errors="replace")
    if rc == FG_EINVAL:
        raise WindowSpecError(msg)
    raise FlinkGpuError(rc, msg)


class HostRegistration:
    """fg_host_register over host arrays (numpy arrays / CPU tensors): the pages they span are
    locked while the context is open, so FG_HOST batches read from them are DMA'd directly --
    what a JNI shim does once per off-heap MemorySegment of its managed memory."""

    def __init__(self, *arrays, device: int = 0):
        self.device = int(device)
        self._ptrs = []
        self._arrays = arrays   # kept alive while registered
        L = load()
        try:
            for a in arrays:
                ptr, nbytes = (a.ctypes.data, a.nbytes) if hasattr(a, "ctypes") else \
                    (a.data_ptr(), a.numel() * a.element_size())
                check(L.fg_host_register(self.device, ptr, nbytes))
                self._ptrs.append(ptr)
        except Exception:
            self.close()
            raise

    def close(self):
        L = load()
        while self._ptrs:
            check(L.fg_host_unregister(self.device, self._ptrs.pop()))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
