"""CPU checks of the key-row path (no device): BinaryRowData key rows as BinaryRowWriter writes
them, and BinarySection.hashCode of any row computed by the library equal to the oracle's
restatement (MurmurHashUtils.hashBytesByWords, seed 42)."""
import struct

import numpy as np

from flink_amd import keys as K
from oracle import oracle as O


def test_key_row_layout_follows_binary_row_writer():
    # one STRING field: bit set (8 B: RowKind byte + null bits) + 8-B slot
    r = K.key_row(["a"], ["string"])
    assert len(r) == 16
    # <= 7 bytes inline: top byte 0x80 | len, data little endian (AbstractBinaryWriter.java:317-330)
    assert int.from_bytes(r[8:16], "little") == (0x80 | 1) << 56 | ord("a")
    r7 = K.key_row(["abcdefg"], ["string"])
    assert len(r7) == 16 and r7[15] == 0x87 and r7[8:15] == b"abcdefg"
    # longer: offset << 32 | length, data in the variable part padded to 8 (:280-292)
    r8 = K.key_row(["abcdefgh1"], ["string"])
    assert len(r8) == 16 + 16
    assert int.from_bytes(r8[8:16], "little") == 16 << 32 | 9
    assert r8[16:25] == b"abcdefgh1" and r8[25:] == b"\0" * 7
    # NULL field: bit 8 + f set, slot zero (BinaryRowWriter.setNullAt)
    rn = K.key_row([None], ["string"])
    assert rn[1] == 1 and rn[8:16] == b"\0" * 8
    # several key columns (STRING, BIGINT, INT)
    rm = K.key_row(["user-0001", -5, 7], ["string", "bigint", "int"])
    assert len(rm) == 8 + 3 * 8 + 16
    assert K.decode_key_row(rm, ["string", "bigint", "int"]) == ("user-0001", -5, 7)
    for v in ("", "x", "héllo wörld", "0123456789" * 5, None):
        assert K.decode_key_row(K.key_row([v], ["string"]), ["string"]) == (v,)


def test_row_hash_matches_oracle_and_bigint_path():
    rng = np.random.default_rng(7)
    for _ in range(300):
        s = "".join(chr(c) for c in rng.integers(32, 127, rng.integers(0, 40)))
        row = K.key_row([s, int(rng.integers(-2**63, 2**63 - 1))], ["string", "bigint"])
        assert K.binaryrow_hash(row) == O.binaryrow_hash_bytes(row)
    for key in (0, 1, -1, 2**63 - 1, -2**63, 123456789):
        row = struct.pack("<q", 0) + struct.pack("<q", key)   # the 16-B BIGINT key row
        assert K.binaryrow_hash(row) == O.binaryrow_hash_i64(key) == O.binaryrow_hash_bytes(row)


def test_pack_key_rows_offsets_are_word_aligned():
    rows = [K.key_row([s], ["string"]) for s in ("a", "bbbbbbbbbbbbb", "", "c" * 30)]
    buf, off, ln = K.pack_key_rows(rows)
    assert (off % 8 == 0).all() and (ln % 8 == 0).all()
    for r, o, n in zip(rows, off, ln):
        assert bytes(buf[o:o + n]) == r
