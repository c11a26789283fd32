/*
 * The WindowBuffer half the two GPU window buffers share: records of (key, slice) pre-aggregated
 * on the MI355X engine, the way RecordsWindowBuffer pre-aggregates them in its managed-memory
 * hash map (RecordsWindowBuffer.java:81-119) -- on a UTC local-partials handle
 * (FG_FLAG_LOCAL_PARTIALS) that takes each record at time sliceEnd - 1, so it lands in exactly
 * the slice the operator assigned (slice ends are on the slice grid in the shifted zone's wall
 * clock; the engine never re-derives the zone).
 *
 *   addElement(key, sliceEnd, row)  the record joins a columnar micro-batch; a full batch goes to
 *                                   fg_add_batch (RecordsWindowBuffer.addElement :81-97; the
 *                                   engine's own staging replaces its EOFException flush)
 *   advanceProgress(progress)       flush() once the smallest buffered slice is fired
 *                                   (RecordsWindowBuffer.advanceProgress :100-106)
 *   flush()                         fg_flush_partials: one partial accumulator row per (key, slice)
 *                                   of everything buffered, handed to combine() with the key row
 *                                   and the accumulator row in the planner's layout (GpuAccRows)
 *   close()                         fg_close
 *
 * Subclasses: GpuLocalWindowBuffer (combine = emit, LocalAggCombiner) and GpuRecordsWindowBuffer
 * (combine = merge into "window-aggs" + window timer, AggCombiner).
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.table.data.GenericRowData;
import org.apache.flink.table.data.RowData;
import org.apache.flink.table.runtime.operators.aggregate.window.buffers.WindowBuffer;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.time.ZoneId;

import static org.apache.flink.table.runtime.util.TimeWindowUtil.isWindowFired;

/** GPU pre-aggregation of (key, slice) records, flushed as accumulator rows. */
abstract class GpuPartialsBuffer implements WindowBuffer {
    protected final GpuWindowAggSpec spec;
    protected final ZoneId shiftTimeZone;
    protected final GpuAccRows accRows;
    private final GpuKeyRows keys;
    private final long handle;
    private final ByteBuffer keyCol, timeCol, valCol, nullCol;
    private int count;
    private long minSliceEnd = Long.MAX_VALUE;

    GpuPartialsBuffer(GpuWindowAggSpec spec, int maxParallelism, ZoneId shiftTimeZone) {
        this.spec = spec;
        this.shiftTimeZone = shiftTimeZone;
        this.accRows = new GpuAccRows(spec.aggs, spec.valType);
        this.keys = new GpuKeyRows(spec, maxParallelism);
        GpuWindowAggSpec local = spec.copy();
        local.flags |= FgConfig.FLAG_LOCAL_PARTIALS;
        local.flags &= ~FgConfig.FLAG_PROCTIME;   // (the slice is assigned: nothing is late here)
        local.shiftTzOffsetMs = 0;
        local.tzTransitionsMs = null;
        local.tzOffsetsMs = null;
        this.handle = FlinkGpu.open(FgConfig.of(local, maxParallelism, 0, maxParallelism - 1, 0), null, null);
        keyCol = GpuKeyRows.direct(8L * spec.batchRecords);
        timeCol = GpuKeyRows.direct(8L * spec.batchRecords);
        valCol = GpuKeyRows.direct(8L * spec.batchRecords);
        nullCol = GpuKeyRows.direct(spec.batchRecords);
        for (ByteBuffer b : new ByteBuffer[] {keyCol, timeCol, valCol, nullCol}) {
            FlinkGpu.hostRegister(spec.device, b);
        }
    }

    @Override
    public void addElement(RowData key, long sliceEnd, RowData element) throws Exception {
        minSliceEnd = Math.min(sliceEnd, minSliceEnd);
        if (!keys.fits(key)) {
            addBatch();
        }
        keys.add(key, count, keyCol);
        timeCol.putLong(8 * count, sliceEnd - 1);
        if (spec.valueIndex >= 0) {
            boolean isNull = element.isNullAt(spec.valueIndex);
            nullCol.put(count, (byte) (isNull ? 1 : 0));
            valCol.putLong(
                    8 * count,
                    isNull ? 0L
                            : spec.valType == FgConfig.VAL_F64
                                    ? Double.doubleToRawLongBits(element.getDouble(spec.valueIndex))
                                    : element.getLong(spec.valueIndex));
        }
        if (++count == spec.batchRecords) {
            addBatch();
        }
    }

    /** the gathered micro-batch to the engine (read completely when the call returns) */
    private void addBatch() {
        if (count == 0) {
            return;
        }
        keys.intern(count, keyCol);
        FlinkGpu.addBatch(
                handle,
                keyCol,
                timeCol,
                spec.valueIndex >= 0 ? valCol : null,
                spec.valueIndex >= 0 ? nullCol : null,
                count);
        count = 0;
    }

    @Override
    public void advanceProgress(long progress) throws Exception {
        if (isWindowFired(minSliceEnd, progress, shiftTimeZone)) {
            flush();
        }
    }

    @Override
    public void flush() throws Exception {
        addBatch();
        if (minSliceEnd == Long.MAX_VALUE) {
            return;   // nothing buffered
        }
        ByteBuffer[] cols = new ByteBuffer[5 + 5];
        long n = FlinkGpu.flushPartials(handle, cols);
        for (ByteBuffer c : cols) {
            if (c != null) {
                c.order(ByteOrder.nativeOrder());
            }
        }
        // partial columns (include/flinkgpu.h FG_FLAG_LOCAL_PARTIALS): key, slice start, slice
        // end, COUNT(*), COUNT(v), then the value slot -- SUM, or MIN / MAX for a list holding only
        // that one -- or, for a list mixing them, the three slots SUM, MIN, MAX
        final boolean mv = accRows.multiValue();
        RowData[] keyRows = keys.rows(cols[0], (int) n);
        for (int i = 0; i < n; i++) {
            long v = cols[5].getLong(8 * i);
            GenericRowData acc =
                    accRows.fromPartial(
                            cols[3].getLong(8 * i),
                            cols[4].getLong(8 * i),
                            v,
                            mv ? cols[6].getLong(8 * i) : v,
                            mv ? cols[7].getLong(8 * i) : v);
            combine(keyRows[i], cols[2].getLong(8 * i), acc);
        }
        minSliceEnd = Long.MAX_VALUE;
    }

    /** one (key, slice)'s partial accumulator of the flushed records */
    protected abstract void combine(RowData key, long sliceEnd, GenericRowData acc) throws Exception;

    @Override
    public void close() throws Exception {
        for (ByteBuffer b : new ByteBuffer[] {keyCol, timeCol, valCol, nullCol}) {
            FlinkGpu.hostUnregister(spec.device, b);
        }
        FlinkGpu.close(handle);
        keys.close();
    }
}
