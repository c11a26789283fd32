"""Grouping keys of any type: the GPU key dictionary (fg_key_dict_* of include/flinkgpu.h).

The reference aggregates by the BinaryRowData key row its key selector projects
(TR/keyselector/BinaryRowDataKeySelector.java:43-50): a STRING key, or several key columns,
is one serialized row, equal keys are byte-equal rows (BinarySection.equals,
TC/data/binary/BinarySection.java:62-73) and the key group is
murmurHash(hashBytesByWords(row)) % maxParallelism (BinarySection.hashCode :76-78,
KeyGroupRangeAssignment.java:63-77). `KeyDictionary.intern` maps such rows to 64-bit ids on the
GPU (equal rows -> equal ids, exact), which the window operators aggregate as BIGINT keys;
`lookup` maps fired rows' ids back to the key rows. `key_row` / `decode_key_row` write and read
key rows the way BinaryRowWriter does (writer/BinaryRowWriter.java, AbstractBinaryWriter.java:
81-105,280-330: STRING of <= 7 bytes inline in its 8-byte slot as 0x80|len in the top byte,
longer ones in the variable part, 8-byte aligned, the slot holding offset << 32 | length).
"""
from __future__ import annotations

import ctypes as C
import struct

import numpy as np

from . import _lib as L
from .rows import HEADER_SIZE_IN_BITS, bit_set_width

def dict_kg_bits(max_parallelism: int) -> int:
    """Bits of the key group in a dictionary id: ceil(log2(max parallelism)) (fg_window.h)."""
    b = 0
    while b < 31 and (1 << b) < max_parallelism:
        b += 1
    return b


def key_row(fields, types, row_kind: int = 0) -> bytes:
    """One BinaryRowData key row. types[i] in {"string", "bigint", "int", "double", "boolean"};
    a None field is NULL (null bit set, slot zero: BinaryRowWriter.setNullAt)."""
    arity = len(fields)
    w = bit_set_width(arity)
    fixed = bytearray(w + 8 * arity)
    fixed[0] = row_kind
    var = bytearray()
    for f, (v, t) in enumerate(zip(fields, types)):
        slot = w + 8 * f
        if v is None:
            b = HEADER_SIZE_IN_BITS + f
            fixed[b >> 3] |= 1 << (b & 7)
            continue
        if t == "string":
            data = v.encode("utf-8") if isinstance(v, str) else bytes(v)
            if len(data) <= 7:   # writeBytesToFixLenPart: 0x80 | len in the top byte, data LE
                word = (0x80 | len(data)) << 56 | int.from_bytes(data, "little")
                fixed[slot:slot + 8] = word.to_bytes(8, "little")
            else:                # writeBytesToVarLenPart: offset << 32 | len, padded to 8 bytes
                off = len(fixed) + len(var)
                fixed[slot:slot + 8] = (off << 32 | len(data)).to_bytes(8, "little")
                var += data + b"\0" * (-len(data) % 8)
        elif t == "bigint":
            fixed[slot:slot + 8] = struct.pack("<q", int(v))
        elif t == "int":
            fixed[slot:slot + 4] = struct.pack("<i", int(v))
        elif t == "double":
            fixed[slot:slot + 8] = struct.pack("<d", float(v))
        elif t == "boolean":
            fixed[slot] = 1 if v else 0
        else:
            raise ValueError(f"unsupported key field type {t!r}")
    return bytes(fixed + var)


def decode_key_row(row: bytes, types):
    """Fields of a key row written by key_row (None for NULL)."""
    arity = len(types)
    w = bit_set_width(arity)
    out = []
    for f, t in enumerate(types):
        b = HEADER_SIZE_IN_BITS + f
        if row[b >> 3] >> (b & 7) & 1:
            out.append(None)
            continue
        slot = row[w + 8 * f: w + 8 * f + 8]
        word = int.from_bytes(slot, "little")
        if t == "string":
            if word >> 63:
                n = (word >> 56) & 0x7F
                out.append(slot[:n].decode("utf-8"))
            else:
                off, n = word >> 32, word & 0xFFFFFFFF
                out.append(row[off:off + n].decode("utf-8"))
        elif t == "bigint":
            out.append(struct.unpack("<q", slot)[0])
        elif t == "int":
            out.append(struct.unpack("<i", slot[:4])[0])
        elif t == "double":
            out.append(struct.unpack("<d", slot)[0])
        elif t == "boolean":
            out.append(bool(slot[0]))
    return tuple(out)


def pack_key_rows(rows):
    """(bytes uint8[], offsets int64[], lengths int32[]) of a list of key rows (8-byte aligned)."""
    lens = np.array([len(r) for r in rows], dtype=np.int32)
    pad = (-lens) % 8
    offs = np.zeros(len(rows), dtype=np.int64)
    if len(rows) > 1:
        offs[1:] = np.cumsum((lens + pad)[:-1], dtype=np.int64)
    buf = bytearray()
    for r, p in zip(rows, pad):
        buf += r + b"\0" * int(p)
    return np.frombuffer(bytes(buf) or b"\0" * 8, dtype=np.uint8), offs, lens


def key_group_of_id(ids, max_parallelism: int = 128):
    """Key group carried by a dictionary id (FG_KEYHASH_DICT_ID)."""
    mask = np.uint64((1 << dict_kg_bits(max_parallelism)) - 1)   # id = ordinal << kg_bits | key group
    return (np.asarray(ids, dtype=np.int64).view(np.uint64) & mask).astype(np.int32) % max_parallelism


def binaryrow_hash(row: bytes) -> int:
    """BinarySection.hashCode of one row, computed by the library (no device needed)."""
    lib = L.load()
    buf = (C.c_uint8 * max(len(row), 1)).from_buffer_copy(row or b"\0")
    return int(lib.fg_binaryrow_hash(buf, len(row)))


class KeyDictionary:
    """GPU-resident dictionary of key rows -> 64-bit ids (fg_key_dict)."""

    def __init__(self, max_parallelism: int = 128, expected_keys: int = 0, device: int = 0):
        lib = L.load()
        self._lib = lib
        self.max_parallelism = max_parallelism
        h = C.c_void_p()
        rc = lib.fg_key_dict_open(device, max_parallelism, expected_keys, C.byref(h))
        if rc != L.FG_OK:
            raise L.FlinkGpuError(rc, "fg_key_dict_open failed (no usable device?)")
        self._h = h

    def _check(self, rc):
        if rc == L.FG_OK:
            return
        msg = self._lib.fg_key_dict_last_error(self._h).decode(errors="replace")
        if rc == L.FG_EINVAL:
            raise L.WindowSpecError(msg)
        raise L.FlinkGpuError(rc, msg)

    def intern_async(self, packed, key_groups=False):
        """fg_key_dict_intern_async of device rows packed=(bytes u8, offsets i64, lengths i32
        tensors): the lookup is launched on the dictionary's stream and (ids, key_groups) tensors
        are returned at once -- complete after intern_wait(). The packed tensors must stay alive
        until then."""
        import torch
        buf, off, ln = packed
        n = len(off)
        ext = self.__dict__.get("_ext_stream")
        if ext is None or ext.device != buf.device:
            ext = self._ext_stream = torch.cuda.ExternalStream(self._lib.fg_key_dict_stream(self._h), device=buf.device)
        ext.wait_stream(torch.cuda.current_stream(buf.device))
        ids = torch.empty(n, dtype=torch.int64, device=buf.device)
        kg = torch.empty(n, dtype=torch.int32, device=buf.device) if key_groups else None
        self._pending = (buf, off, ln, ids, kg)
        self._check(self._lib.fg_key_dict_intern_async(self._h, n, C.c_void_p(buf.data_ptr()), buf.numel(),
                                                       C.c_void_p(off.data_ptr()), C.c_void_p(ln.data_ptr()),
                                                       C.c_void_p(ids.data_ptr()),
                                                       C.c_void_p(kg.data_ptr() if key_groups else None)))
        return ids, kg

    def intern_wait(self):
        """fg_key_dict_intern_wait: the pending intern_async's ids (and key groups) complete"""
        rc = self._lib.fg_key_dict_intern_wait(self._h)
        self._pending = None
        self._check(rc)

    def intern(self, rows=None, packed=None, key_groups=True):
        """rows: list of key-row bytes, or packed=(bytes u8[], offsets i64[], lengths i32[]) on the
        host (numpy) or the device (torch tensors). Returns (ids, key_groups) of the same kind
        (key_groups None when not asked for: an id carries its key group, FG_KEYHASH_DICT_ID)."""
        if packed is None:
            packed = pack_key_rows(rows)
        buf, off, ln = packed
        n = len(off)
        if hasattr(buf, "data_ptr"):   # torch device tensors
            import torch
            # the dictionary reads them on its own stream: order it after their producers
            ext = self.__dict__.get("_ext_stream")
            if ext is None or ext.device != buf.device:
                ext = self._ext_stream = torch.cuda.ExternalStream(self._lib.fg_key_dict_stream(self._h),
                                                                   device=buf.device)
            ext.wait_stream(torch.cuda.current_stream(buf.device))
            ids = torch.empty(n, dtype=torch.int64, device=buf.device)
            kg = torch.empty(n, dtype=torch.int32, device=buf.device) if key_groups else None
            self._check(self._lib.fg_key_dict_intern(self._h, L.DEVICE, n, C.c_void_p(buf.data_ptr()), buf.numel(),
                                                     C.c_void_p(off.data_ptr()), C.c_void_p(ln.data_ptr()),
                                                     C.c_void_p(ids.data_ptr()),
                                                     C.c_void_p(kg.data_ptr() if key_groups else None)))
            return ids, kg
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.int64)
        ln = np.ascontiguousarray(ln, dtype=np.int32)
        ids = np.empty(n, dtype=np.int64)
        kg = np.empty(n, dtype=np.int32) if key_groups else None
        self._check(self._lib.fg_key_dict_intern(self._h, L.HOST, n, buf.ctypes.data, buf.size, off.ctypes.data,
                                                 ln.ctypes.data, ids.ctypes.data,
                                                 C.c_void_p(kg.ctypes.data if key_groups else None)))
        return ids, kg

    def intern_rows(self, data, offsets, lengths):
        """ids (device int64 tensor) of the key rows in device tensors: data uint8, offsets
        int64, lengths int32 (flink_amd.exchange's receiving side of key rows)."""
        ids, _ = self.intern(packed=(data, offsets, lengths), key_groups=False)
        return ids

    def locate(self, ids):
        """Where the key rows of device ids live: (word offsets int64, words int64, arena) with
        arena an int32 device tensor view of the dictionary's arena (valid until the next
        intern on this dictionary); row i = arena[woff[i] : woff[i] + nw[i]]."""
        import torch
        n = ids.numel()
        off = torch.empty(n, dtype=torch.int64, device=ids.device)
        ln = torch.empty(n, dtype=torch.int32, device=ids.device)
        if n:
            ext = self.__dict__.get("_ext_stream")
            if ext is None or ext.device != ids.device:
                ext = self._ext_stream = torch.cuda.ExternalStream(self._lib.fg_key_dict_stream(self._h),
                                                                   device=ids.device)
            ext.wait_stream(torch.cuda.current_stream(ids.device))
            self._check(self._lib.fg_key_dict_lookup(self._h, L.DEVICE, n, C.c_void_p(ids.data_ptr()),
                                                     C.c_void_p(off.data_ptr()), C.c_void_p(ln.data_ptr())))
            if bool((ln < 0).any()):
                raise KeyError("unknown dictionary id in locate()")
        p = C.c_void_p()
        size = C.c_int64()
        self._check(self._lib.fg_key_dict_arena(self._h, C.byref(p), C.byref(size)))

        class _Arena:   # zero-copy view for torch.as_tensor
            __cuda_array_interface__ = {"shape": (max(int(size.value) // 4, 1),), "typestr": "<i4",
                                        "data": (int(p.value or 0), False), "version": 2}
        arena = torch.as_tensor(_Arena(), device=ids.device)
        return off // 4, (ln // 4).to(torch.int64), arena

    def lookup(self, ids):
        """Key rows (bytes) of the ids (host)."""
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        n = len(ids)
        if n == 0:
            return []
        off = np.empty(n, dtype=np.int64)
        ln = np.empty(n, dtype=np.int32)
        self._check(self._lib.fg_key_dict_lookup(self._h, L.HOST, n, ids.ctypes.data, off.ctypes.data, ln.ctypes.data))
        if (ln < 0).any():
            raise KeyError(f"unknown dictionary id {int(ids[np.argmax(ln < 0)])}")
        lo, hi = int(off.min()), int((off + ln).max())
        arena = np.empty(max(hi - lo, 1), dtype=np.uint8)
        self._check(self._lib.fg_key_dict_copy_arena(self._h, lo, hi - lo, arena.ctypes.data))
        raw = arena.tobytes()
        return [raw[o - lo:o - lo + n_] for o, n_ in zip(off.tolist(), ln.tolist())]

    def set_timing(self, on: bool = True):
        """HIP-event timing of the dictionary's kernels (kernel_stats)."""
        self._check(self._lib.fg_key_dict_set_timing(self._h, 1 if on else 0))

    def kernel_stats(self) -> dict:
        """{"dict_probe" | "dict_assign": dict(launches, total_ms, records, rows)}."""
        arr = (L.FgKernelStat * 4)()
        n = C.c_int32()
        self._check(self._lib.fg_key_dict_kernel_stats(self._h, arr, 4, C.byref(n)))
        return {arr[i].name.decode(): dict(launches=arr[i].launches, total_ms=arr[i].total_ms,
                                           records=arr[i].records, rows=arr[i].rows) for i in range(n.value)}

    def __len__(self):
        return int(self._lib.fg_key_dict_size(self._h))

    def close(self):
        if self._h:
            self._lib.fg_key_dict_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
