"""The two-phase keyBy edge over RCCL through the C-ABI (fg_comm_*, include/flinkgpu.h ABI 14).

The same exchange as flink_amd.exchange.exchange_partials -- rows grouped by key-group owner on
the device, one all-to-all of (count, watermark) per peer, one host read, the rows moved over
xGMI -- but driven from libflinkgpu.so itself: no torch.distributed, so a JVM shim (JNI
commOpen / commExchangeFired) or any C/C++ host gets the edge with the same library. The
communicator is bootstrapped from a 128-byte id made once (fg_comm_unique_id) and handed to
every rank (a coordinator distributes it; here a file or torch.distributed broadcast).
"""
from __future__ import annotations

import ctypes as C

from . import _lib as L


def unique_id() -> bytes:
    """ncclGetUniqueId: made once, by one rank, and shipped to every rank."""
    lib = L.load()
    buf = (C.c_uint8 * L.COMM_ID_BYTES)()
    rc = lib.fg_comm_unique_id(buf)
    if rc:
        raise L.FlinkGpuError(rc, lib.fg_comm_last_error(None).decode(errors="replace"))
    return bytes(buf)


class Communicator:
    """fg_comm of one subtask: `world` ranks, one process per GPU. fg_comm_open blocks until
    every rank has joined."""

    def __init__(self, device: int, world: int, rank: int, comm_id: bytes):
        self._lib = L.load()
        self.world, self.rank, self.device = world, rank, device
        idb = (C.c_uint8 * L.COMM_ID_BYTES).from_buffer_copy(comm_id)
        h = C.c_void_p()
        rc = self._lib.fg_comm_open(device, world, rank, idb, C.byref(h))
        if rc:
            raise L.FlinkGpuError(rc, self._lib.fg_comm_last_error(None).decode(errors="replace"))
        self._h = h

    def _check(self, rc):
        if rc:
            raise L.FlinkGpuError(rc, self._lib.fg_comm_last_error(self._h).decode(errors="replace"))

    @property
    def bytes_sent(self) -> int:
        """bytes sent to other ranks by every exchange so far"""
        return self._lib.fg_comm_bytes_sent(self._h)

    @property
    def stream(self) -> int:
        return self._lib.fg_comm_stream(self._h) or 0

    def exchange_columns(self, cols, key_hash=L.KEYHASH_BINARYROW_BIGINT, max_parallelism=128, watermark=0,
                         stream=None):
        """int64 device tensors (cols[0] = key) -> (received column tensors on the device -- views of
        communicator-owned memory, valid until the next exchange, complete on `self.stream` --, the
        min watermark over the ranks). `stream`: the producer's stream (default torch's current)."""
        import torch
        dev = cols[0].device
        n = cols[0].numel()
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        ptrs = (C.c_void_p * len(cols))(*[c.data_ptr() for c in cols])
        x = L.FgExchanged()
        self._check(self._lib.fg_comm_exchange_columns(self._h, C.c_void_p(s), n, len(cols), ptrs, key_hash,
                                                       max_parallelism, int(watermark), C.byref(x)))
        from .exchange import _DeviceColumn
        out = [torch.as_tensor(_DeviceColumn(x.cols[j], int(x.n)), device=dev) for j in range(x.ncols)]
        # torch's stream orders after the collective before anything reads the views
        torch.cuda.current_stream(dev).wait_stream(torch.cuda.ExternalStream(self.stream, device=dev))
        return out, int(x.min_watermark)

    def exchange_fired(self, local, glob, watermark, key_hash=L.KEYHASH_BINARYROW_BIGINT, max_parallelism=128) -> int:
        """fg_comm_exchange_fired: the local operator's uncollected async fires -> owners ->
        fg_add_partials of `glob`; returns the combined watermark."""
        wm = C.c_int64()
        self._check(self._lib.fg_comm_exchange_fired(self._h, local._h, key_hash, max_parallelism, int(watermark),
                                                     glob._h, C.byref(wm)))
        return wm.value

    def exchange_flushed(self, local, glob, watermark, key_hash=L.KEYHASH_BINARYROW_BIGINT, max_parallelism=128) -> int:
        """fg_comm_exchange_flushed: the local buffer (fg_flush_partials, prepareSnapshotPreBarrier)
        -> owners -> fg_add_partials of `glob`; returns the combined watermark."""
        wm = C.c_int64()
        self._check(self._lib.fg_comm_exchange_flushed(self._h, local._h, key_hash, max_parallelism, int(watermark),
                                                       glob._h, C.byref(wm)))
        return wm.value

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fg_comm_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
