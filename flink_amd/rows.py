"""Packed BinaryRowData rows for fg_add_rows (the host-side analogue of BinaryRowWriter for
rows of fixed-length fields; TC/data/binary/BinaryRowData.java:68-76, writer/BinaryRowWriter).

Row layout (little endian): a bit set of calculateBitSetWidthInBytes(arity) =
((arity + 63 + 8) / 64) * 8 bytes -- byte 0 is the RowKind, bit 8 + f marks field f NULL
(:155-157, BinarySegmentUtils.bitGet :459-463) -- then 8 bytes per field (:119-121): BIGINT
and DOUBLE as is, TIMESTAMP(3) as its compact epoch millis (:347-352). A NULL field's 8 bytes
are zero (BinaryRowWriter.setNullAt)."""
from __future__ import annotations

import numpy as np

HEADER_SIZE_IN_BITS = 8


def bit_set_width(arity: int) -> int:
    """BinaryRowData.calculateBitSetWidthInBytes (:70-72)."""
    return ((arity + 63 + HEADER_SIZE_IN_BITS) // 64) * 8


def fixed_part_size(arity: int) -> int:
    """BinaryRowData.calculateFixPartSizeInBytes (:74-76)."""
    return bit_set_width(arity) + 8 * arity


def pack_rows(fields, nulls=None, stride: int | None = None, row_kind: int = 0) -> np.ndarray:
    """fields: list of `arity` 8-byte numpy columns (int64 / float64) of equal length; nulls:
    per field None or a bool column. Returns a uint8 array of n * stride bytes."""
    arity = len(fields)
    n = len(fields[0])
    w = bit_set_width(arity)
    stride = stride or fixed_part_size(arity)
    assert stride >= fixed_part_size(arity) and stride % 8 == 0
    out = np.zeros((n, stride // 8), dtype=np.int64)
    bits = np.zeros((n, w), dtype=np.uint8)
    bits[:, 0] = row_kind
    for f, col in enumerate(fields):
        c = np.ascontiguousarray(col)
        assert c.dtype.itemsize == 8
        v = c.view(np.int64).copy()
        nl = None if nulls is None else nulls[f]
        if nl is not None:
            nl = np.asarray(nl, dtype=bool)
            v[nl] = 0
            b = HEADER_SIZE_IN_BITS + f
            bits[nl, b >> 3] |= np.uint8(1 << (b & 7))
        out[:, w // 8 + f] = v
    out[:, : w // 8] = bits.view(np.int64).reshape(n, w // 8)
    return out.view(np.uint8).reshape(-1)
