/*
 * SlicingWindowProcessor<Long> backed by the MI355X engine (libflinkgpu.so through
 * FlinkGpu/JNI). Replaces SliceUnsharedWindowAggProcessor / SliceSharedWindowAggProcessor +
 * RecordsWindowBuffer + AggCombiner (SlicingWindowAggOperatorBuilder.java:146-170):
 *
 *   processElement      -> the record is appended to direct column buffers; a full micro-batch
 *                          goes to fg_add_batch (AbstractWindowAggProcessor.java:135-165)
 *   advanceProgress     -> the pending micro-batch, then fg_advance_progress: the engine applies
 *                          the progress gate, flushes, fires the windows whose timers the
 *                          watermark passes and returns their rows, emitted here before
 *                          SlicingWindowOperator forwards the watermark (SlicingWindowOperator
 *                          .java:207-210)
 *   prepareCheckpoint   -> fg_flush, then the resident (key, slice) accumulators are written to
 *                          the keyed state "gpu-window-aggs" (namespace = slice end), as
 *                          AggCombiner.combine writes "window-aggs" (AggCombiner.java:76-115)
 *   fireWindow/clearWindow -> no-ops: the engine fires windows itself, no per-key timer is
 *                          registered (DESIGN.md section 3)
 *
 * Late drops: the engine counts them; advanceProgress adds the new ones to the operator's
 * numLateRecordsDropped counter, which also drives lateRecordsDroppedRate (a MeterView over
 * that counter, SlicingWindowOperator.java:159-163); watermarkLatency is the operator's own
 * gauge over its timer service's watermark and is unchanged.
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.api.common.state.ValueState;
import org.apache.flink.api.common.state.ValueStateDescriptor;
import org.apache.flink.api.common.typeutils.TypeSerializer;
import org.apache.flink.api.common.typeutils.base.LongSerializer;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.core.memory.MemorySegmentFactory;
import org.apache.flink.runtime.state.CheckpointableKeyedStateBackend;
import org.apache.flink.runtime.state.KeyGroupRange;
import org.apache.flink.runtime.state.KeyedStateBackend;
import org.apache.flink.table.data.GenericRowData;
import org.apache.flink.table.data.RowData;
import org.apache.flink.table.data.TimestampData;
import org.apache.flink.table.data.binary.BinaryRowData;
import org.apache.flink.table.data.utils.JoinedRowData;
import org.apache.flink.table.runtime.operators.window.slicing.SlicingWindowOperator;
import org.apache.flink.table.runtime.operators.window.slicing.SlicingWindowProcessor;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.List;
import java.util.stream.Collectors;

/** The slicing window processor of the GPU engine. */
public final class GpuSlicingWindowProcessor implements SlicingWindowProcessor<Long> {
    private static final long serialVersionUID = 1L;
    static final String STATE_NAME = "gpu-window-aggs";

    private final GpuWindowAggSpec spec;

    private transient Context<Long> ctx;
    private transient SlicingWindowOperator<?, ?> owner;
    private transient long handle;
    private transient long dict;
    private transient ByteBuffer keys, rowtimes, vals, nulls;
    private transient ByteBuffer keyRows, keyOffsets, keyLengths;
    private transient int count;
    private transient int keyBytes;
    private transient long droppedSeen;
    private transient ValueState<GenericRowData> state;

    public GpuSlicingWindowProcessor(GpuWindowAggSpec spec) {
        this.spec = spec;
    }

    /** the operator whose numLateRecordsDropped the engine's drop count feeds */
    public void attach(SlicingWindowOperator<?, ?> operator) {
        this.owner = operator;
    }

    @Override
    public void open(Context<Long> context) throws Exception {
        this.ctx = context;
        KeyedStateBackend<RowData> backend = ctx.getKeyedStateBackend();
        KeyGroupRange range = ((CheckpointableKeyedStateBackend<?>) backend).getKeyGroupRange();
        int maxP = ctx.getRuntimeContext().getMaxNumberOfParallelSubtasks();
        int nTz = spec.tzTransitionsMs == null ? 0 : spec.tzTransitionsMs.length;
        handle =
                FlinkGpu.open(
                        FgConfig.of(
                                spec, maxP, range.getStartKeyGroup(), range.getEndKeyGroup(), nTz),
                        spec.tzTransitionsMs,
                        spec.tzOffsetsMs);
        if (!spec.bigintKey) {
            dict = FlinkGpu.dictOpen(spec.device, maxP, spec.expectedKeys);
            keyRows = direct(64L * spec.batchRecords);
            keyOffsets = direct(8L * spec.batchRecords);
            keyLengths = direct(4L * spec.batchRecords);
        }
        keys = direct(8L * spec.batchRecords);
        rowtimes = direct(8L * spec.batchRecords);
        vals = direct(8L * spec.batchRecords);
        nulls = direct(spec.batchRecords);
        // the staging columns live for the operator's life: page-lock them once, so every
        // micro-batch is DMA'd straight from them (fg_host_register)
        for (ByteBuffer b : new ByteBuffer[] {keys, rowtimes, vals, nulls}) {
            FlinkGpu.hostRegister(spec.device, b);
        }
        state =
                backend.getPartitionedState(
                        LongSerializer.INSTANCE.createInstance(),
                        LongSerializer.INSTANCE,
                        new ValueStateDescriptor<>(STATE_NAME, GenericRowData.class));
        restoreFromKeyedState(backend);
    }

    private static ByteBuffer direct(long bytes) {
        return ByteBuffer.allocateDirect((int) Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
    }

    @Override
    public boolean processElement(RowData key, RowData element) throws Exception {
        if (spec.bigintKey) {
            keys.putLong(8 * count, key.getLong(0));
        } else {
            BinaryRowData row = (BinaryRowData) key;   // BinaryRowDataKeySelector output
            int len = row.getSizeInBytes();
            if (keyBytes + len > keyRows.capacity()) {
                flushBatch();
            }
            keyRows.position(keyBytes);   // (the selector's copy: one segment)
            row.getSegments()[0].get(row.getOffset(), keyRows, len);
            keyOffsets.putLong(8 * count, keyBytes);
            keyLengths.putInt(4 * count, len);
            keyBytes += (len + 7) & ~7;
        }
        rowtimes.putLong(8 * count, element.getTimestamp(spec.rowtimeIndex, 3).getMillisecond());
        if (spec.valueIndex >= 0) {
            boolean isNull = element.isNullAt(spec.valueIndex);
            nulls.put(count, (byte) (isNull ? 1 : 0));
            long bits =
                    isNull
                            ? 0L
                            : spec.valType == FgConfig.VAL_F64
                                    ? Double.doubleToRawLongBits(element.getDouble(spec.valueIndex))
                                    : element.getLong(spec.valueIndex);
            vals.putLong(8 * count, bits);
        }
        if (++count == spec.batchRecords) {
            flushBatch();
        }
        return false;   // late drops are counted by the engine (see advanceProgress)
    }

    /** hands the gathered micro-batch to the engine (which has read it when this returns) */
    private void flushBatch() {
        if (count == 0) {
            return;
        }
        if (!spec.bigintKey) {   // key rows -> dictionary ids (BinarySection.equals identity)
            FlinkGpu.dictIntern(dict, keyRows, keyBytes, keyOffsets, keyLengths, count, keys, null);
            keyBytes = 0;
        }
        FlinkGpu.addBatch(
                handle,
                keys,
                rowtimes,
                spec.valueIndex >= 0 ? vals : null,
                spec.valueIndex >= 0 ? nulls : null,
                count);
        count = 0;
    }

    @Override
    public void advanceProgress(long progress) throws Exception {
        flushBatch();
        ByteBuffer[] cols = new ByteBuffer[5 + spec.aggs.length];
        long n = FlinkGpu.advanceProgress(handle, progress, cols);
        for (ByteBuffer c : cols) {
            if (c != null) {
                c.order(ByteOrder.nativeOrder());
            }
        }
        for (int i = 0; i < n; i++) {
            ctx.output(outputRow(cols, i));
        }
        long dropped = FlinkGpu.lateDropped(handle);
        if (owner != null && dropped > droppedSeen) {
            owner.getNumLateRecordsDropped().inc(dropped - droppedSeen);
        }
        droppedSeen = dropped;
    }

    /** JoinedRowData(key, [aggs..., window_start, window_end]) (AbstractWindowAggProcessor.collect) */
    private RowData outputRow(ByteBuffer[] cols, int i) {
        long key = cols[0].getLong(8 * i);
        int nAggs = spec.aggs.length;
        byte nullMask = cols[3 + nAggs].get(i);
        GenericRowData aggs = new GenericRowData(nAggs + 2);
        for (int a = 0; a < nAggs; a++) {
            if ((nullMask >> a & 1) != 0) {
                continue;   // NULL
            }
            long bits = cols[3 + a].getLong(8 * i);
            int agg = spec.aggs[a];
            boolean valueTyped = agg != FgConfig.AGG_COUNT_STAR && agg != FgConfig.AGG_COUNT;
            aggs.setField(
                    a,
                    valueTyped && spec.valType == FgConfig.VAL_F64
                            ? (Object) Double.longBitsToDouble(bits)
                            : (Object) bits);
        }
        aggs.setField(nAggs, TimestampData.fromEpochMillis(cols[1].getLong(8 * i)));
        aggs.setField(nAggs + 1, TimestampData.fromEpochMillis(cols[2].getLong(8 * i)));
        return new JoinedRowData(keyRow(key), aggs);
    }

    private RowData keyRow(long key) {
        if (spec.bigintKey) {
            return GenericRowData.of(key);
        }
        ByteBuffer id = direct(8);
        id.putLong(0, key);
        ByteBuffer off = direct(8);
        ByteBuffer len = direct(4);
        FlinkGpu.dictLookup(dict, id, 1, off, len);
        int n = len.getInt(0);
        ByteBuffer bytes = direct(n);
        FlinkGpu.dictCopyArena(dict, off.getLong(0), n, bytes);
        byte[] b = new byte[n];
        bytes.get(b);
        BinaryRowData row = new BinaryRowData(spec.keyArity);
        row.pointTo(MemorySegmentFactory.wrap(b), 0, n);
        return row;
    }

    @Override
    public void prepareCheckpoint() throws Exception {
        flushBatch();
        FlinkGpu.flush(handle);
        writeKeyedState();
    }

    /**
     * The window-aggs image into keyed state: per (key, slice end) one row (cnt_star, cnt_val,
     * sum, min, max), as AggCombiner.combine leaves one accumulator per (key, slice). Entries of
     * slices fired since the last checkpoint are removed first.
     */
    private void writeKeyedState() throws Exception {
        KeyedStateBackend<RowData> backend = ctx.getKeyedStateBackend();
        List<Tuple2<RowData, Long>> old =
                backend.<Long>getKeysAndNamespaces(STATE_NAME).collect(Collectors.toList());
        for (Tuple2<RowData, Long> kn : old) {
            backend.setCurrentKey(kn.f0);
            backend.getPartitionedState(
                            kn.f1,
                            LongSerializer.INSTANCE,
                            new ValueStateDescriptor<>(STATE_NAME, GenericRowData.class))
                    .clear();
        }
        ByteBuffer[] cols = new ByteBuffer[7];
        long[] wm = new long[1];
        long n = FlinkGpu.snapshotState(handle, cols, wm);
        for (ByteBuffer c : cols) {
            if (c != null) {
                c.order(ByteOrder.nativeOrder());
            }
        }
        for (int i = 0; i < n; i++) {
            backend.setCurrentKey(keyRow(cols[0].getLong(8 * i)));
            ValueState<GenericRowData> s =
                    backend.getPartitionedState(
                            cols[1].getLong(8 * i),
                            LongSerializer.INSTANCE,
                            new ValueStateDescriptor<>(STATE_NAME, GenericRowData.class));
            s.update(
                    GenericRowData.of(
                            cols[2].getLong(8 * i),
                            cols[3].getLong(8 * i),
                            cols[4].getLong(8 * i),
                            cols[5] == null ? null : cols[5].getLong(8 * i),
                            cols[6] == null ? null : cols[6].getLong(8 * i),
                            wm[0]));
        }
    }

    /** initializeState: the keyed image of the subtask's key groups back into the engine */
    private void restoreFromKeyedState(KeyedStateBackend<RowData> backend) throws Exception {
        List<Tuple2<RowData, Long>> entries =
                backend.<Long>getKeysAndNamespaces(STATE_NAME).collect(Collectors.toList());
        if (entries.isEmpty()) {
            return;
        }
        int n = entries.size();
        List<ByteBuffer> c = new ArrayList<>();
        for (int j = 0; j < 7; j++) {
            c.add(direct(8L * n));
        }
        boolean mv = false;
        long timerWm = Long.MIN_VALUE;
        List<byte[]> rows = new ArrayList<>();
        for (int i = 0; i < n; i++) {
            Tuple2<RowData, Long> kn = entries.get(i);
            backend.setCurrentKey(kn.f0);
            GenericRowData acc =
                    backend.getPartitionedState(
                                    kn.f1,
                                    LongSerializer.INSTANCE,
                                    new ValueStateDescriptor<>(STATE_NAME, GenericRowData.class))
                            .value();
            if (spec.bigintKey) {
                c.get(0).putLong(8 * i, kn.f0.getLong(0));
            } else {
                BinaryRowData r = (BinaryRowData) kn.f0;
                byte[] b = new byte[r.getSizeInBytes()];
                r.getSegments()[0].get(r.getOffset(), b);
                rows.add(b);
            }
            c.get(1).putLong(8 * i, kn.f1);
            for (int j = 0; j < 3; j++) {
                c.get(2 + j).putLong(8 * i, acc.getLong(j));
            }
            if (!acc.isNullAt(3)) {
                mv = true;
                c.get(5).putLong(8 * i, acc.getLong(3));
                c.get(6).putLong(8 * i, acc.getLong(4));
            }
            timerWm = acc.getLong(5);
        }
        if (!spec.bigintKey) {   // the image carries key rows: re-intern them first
            ByteBuffer all = direct(rows.stream().mapToLong(b -> (b.length + 7) & ~7).sum());
            ByteBuffer off = direct(8L * n);
            ByteBuffer len = direct(4L * n);
            int at = 0;
            for (int i = 0; i < n; i++) {
                byte[] b = rows.get(i);
                all.position(at);
                all.put(b);
                off.putLong(8 * i, at);
                len.putInt(4 * i, b.length);
                at += (b.length + 7) & ~7;
            }
            FlinkGpu.dictIntern(dict, all, at, off, len, n, c.get(0), null);
        }
        FlinkGpu.restore(
                handle,
                n,
                c.get(0),
                c.get(1),
                c.get(2),
                c.get(3),
                c.get(4),
                mv ? c.get(5) : null,
                mv ? c.get(6) : null,
                timerWm);
    }

    @Override
    public void fireWindow(Long windowEnd) {}

    @Override
    public void clearWindow(Long windowEnd) {}

    @Override
    public void close() throws Exception {
        if (handle != 0) {
            FlinkGpu.close(handle);
            handle = 0;
            for (ByteBuffer b : new ByteBuffer[] {keys, rowtimes, vals, nulls}) {
                FlinkGpu.hostUnregister(spec.device, b);
            }
        }
        if (dict != 0) {
            FlinkGpu.dictClose(dict);
            dict = 0;
        }
    }

    @Override
    public TypeSerializer<Long> createWindowSerializer() {
        return LongSerializer.INSTANCE;
    }
}
