/*
 * Grouping keys of a GPU window operator: one BIGINT key column as it is, any other key row
 * (BinaryRowDataKeySelector output, BinaryRowDataKeySelector.java:43-50 -- a STRING key, several
 * columns, a NULL key) through the engine's key dictionary (fg_key_dict: equal rows -> equal ids,
 * BinarySection.equals / hashCode, BinarySection.java:62-78).
 *
 * Per micro-batch the key rows are gathered into one direct buffer and interned by ONE
 * dictIntern call; per advance the fired rows' ids become key rows through ONE dictLookup of
 * every id and ONE arena copy of the byte range they span -- never a JNI round trip per row.
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.core.memory.MemorySegment;
import org.apache.flink.core.memory.MemorySegmentFactory;
import org.apache.flink.table.data.RowData;
import org.apache.flink.table.data.binary.BinaryRowData;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;

/** Key rows <-> 64-bit engine keys for one operator. */
final class GpuKeyRows implements AutoCloseable {
    private final boolean bigint;
    private final int arity;
    private final int batch;
    private long dict;
    private ByteBuffer rows, offsets, lengths;   // the current micro-batch's key rows
    private int n;
    private int bytes;
    private ByteBuffer ids, outOff, outLen;      // lookup scratch (grown on demand)

    GpuKeyRows(GpuWindowAggSpec spec, int maxParallelism) {
        this.bigint = spec.bigintKey;
        this.arity = spec.keyArity;
        this.batch = spec.batchRecords;
        if (!bigint) {
            dict = FlinkGpu.dictOpen(spec.device, maxParallelism, spec.expectedKeys);
            rows = direct(64L * batch);
            offsets = direct(8L * batch);
            lengths = direct(4L * batch);
        }
    }

    static ByteBuffer direct(long bytes) {
        return ByteBuffer.allocateDirect((int) Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
    }

    boolean bigint() {
        return bigint;
    }

    /** room for one more key row of `len` bytes in the batch's row buffer */
    boolean fits(RowData key) {
        return bigint || bytes + ((BinaryRowData) key).getSizeInBytes() <= rows.capacity();
    }

    /** record i of the micro-batch has key `key`: BIGINT into keys[i], else its row gathered */
    void add(RowData key, int i, ByteBuffer keys) {
        if (bigint) {
            keys.putLong(8 * i, key.getLong(0));
            return;
        }
        BinaryRowData row = (BinaryRowData) key;
        int len = row.getSizeInBytes();
        rows.position(bytes);
        MemorySegment[] segs = row.getSegments();
        if (segs.length == 1) {
            segs[0].get(row.getOffset(), rows, len);
        } else {   // (a key row spanning segments: copied through a heap array)
            byte[] b = new byte[len];
            org.apache.flink.table.data.binary.BinarySegmentUtils.copyToBytes(segs, row.getOffset(), b, 0, len);
            rows.put(b);
        }
        offsets.putLong(8 * n, bytes);
        lengths.putInt(4 * n, len);
        bytes += (len + 7) & ~7;
        n++;
    }

    /** the batch's key rows -> ids in keys[0 .. count) (one dictIntern) */
    void intern(int count, ByteBuffer keys) {
        if (bigint || count == 0) {
            return;
        }
        FlinkGpu.dictIntern(dict, rows, bytes, offsets, lengths, count, keys, null);
        n = 0;
        bytes = 0;
    }

    /** the key rows of ids keys[0 .. count) (one dictLookup, one arena copy) */
    RowData[] rows(ByteBuffer keys, int count) {
        RowData[] out = new RowData[count];
        if (bigint) {
            // BinaryRowData of arity 1 (8-byte header + the long), as BinaryRowDataKeySelector
            // builds them: hashCode / equals -- and so key groups and state keys -- are the
            // selector's own (a GenericRowData would hash differently)
            MemorySegment seg = MemorySegmentFactory.wrap(new byte[16 * Math.max(count, 1)]);
            for (int i = 0; i < count; i++) {
                seg.putLong(16 * i + 8, keys.getLong(8 * i));
                BinaryRowData r = new BinaryRowData(1);
                r.pointTo(seg, 16 * i, 16);
                out[i] = r;
            }
            return out;
        }
        if (count == 0) {
            return out;
        }
        if (outOff == null || outOff.capacity() < 8 * count) {
            outOff = direct(8L * count);
            outLen = direct(4L * count);
        }
        FlinkGpu.dictLookup(dict, keys, count, outOff, outLen);
        long lo = Long.MAX_VALUE, hi = 0;
        for (int i = 0; i < count; i++) {
            long o = outOff.getLong(8 * i);
            lo = Math.min(lo, o);
            hi = Math.max(hi, o + outLen.getInt(4 * i));
        }
        ByteBuffer arena = direct(hi - lo);
        FlinkGpu.dictCopyArena(dict, lo, hi - lo, arena);
        byte[] all = new byte[(int) (hi - lo)];
        arena.get(all);
        MemorySegment seg = MemorySegmentFactory.wrap(all);
        for (int i = 0; i < count; i++) {
            BinaryRowData r = new BinaryRowData(arity);
            r.pointTo(seg, (int) (outOff.getLong(8 * i) - lo), outLen.getInt(4 * i));
            out[i] = r;
        }
        return out;
    }

    /** the key rows of the given ids (a restore re-interns the image's rows first) */
    void internRows(byte[][] keyRows, ByteBuffer keys) {
        if (bigint) {
            return;
        }
        long total = 0;
        for (byte[] b : keyRows) {
            total += (b.length + 7) & ~7;
        }
        ByteBuffer all = direct(total);
        ByteBuffer off = direct(8L * keyRows.length);
        ByteBuffer len = direct(4L * keyRows.length);
        int at = 0;
        for (int i = 0; i < keyRows.length; i++) {
            all.position(at);
            all.put(keyRows[i]);
            off.putLong(8 * i, at);
            len.putInt(4 * i, keyRows[i].length);
            at += (keyRows[i].length + 7) & ~7;
        }
        FlinkGpu.dictIntern(dict, all, at, off, len, keyRows.length, keys, null);
    }

    @Override
    public void close() {
        if (dict != 0) {
            FlinkGpu.dictClose(dict);
            dict = 0;
        }
    }
}
