/*
 * SlicingWindowProcessor<Long> backed by the MI355X engine (libflinkgpu.so through FlinkGpu/JNI):
 * replaces SliceUnsharedWindowAggProcessor / SliceSharedWindowAggProcessor + RecordsWindowBuffer
 * + AggCombiner (SlicingWindowAggOperatorBuilder.java:146-170), and, for the global phase of the
 * two-phase plan, GlobalAggCombiner (spec.partialInput). The engine keeps the (key, slice)
 * accumulators in HBM and fires windows itself.
 *
 *   processElement      the record (or, global phase, the local phase's partial accumulator row)
 *                       joins columnar micro-batch buffers; a full micro-batch goes to
 *                       fg_add_batch / fg_add_partials with its key rows interned by ONE
 *                       dictionary call (AbstractWindowAggProcessor.java:135-165). Processing
 *                       time: the record carries the operator clock's time, and a processing-time
 *                       timer is registered once per new slice end (the reference registers one per
 *                       record, :137-140) -- its firing calls advanceProgress
 *   advanceProgress     fg_advance_progress: the engine applies the progress gate, fires the windows
 *                       the progress passes and returns their rows (one dictionary lookup + one
 *                       arena copy for every fired key row), emitted before the operator forwards
 *                       the watermark (SlicingWindowOperator.java:207-210)
 *   advanceAsync / collectHeld   fg_advance_progress_async + fg_collect_fired for an operator that
 *                       holds the watermark while the fires complete (GpuSlicingWindowAggOperator)
 *   prepareCheckpoint   fg_flush + fg_snapshot_state_async / _wait: the resident accumulators are written to the
 *                       reference's own keyed state "window-aggs" (namespace = slice end, the
 *                       accumulator row in the accSerializer layout, GpuAccRows) and the window
 *                       timers AggCombiner would hold are registered -- a savepoint the reference
 *                       processors restore, and restore from (INTEGRATION.md section 6); only the
 *                       slices written since the last checkpoint (fg_snapshot_slices) are rewritten
 *   fireWindow / clearWindow  no-ops: the engine fires windows; the timers registered at a
 *                       checkpoint fire into these no-ops
 *
 * Late drops: the engine counts them; advanceProgress adds the new ones to the operator's
 * numLateRecordsDropped counter (lateRecordsDroppedRate is a MeterView over it).
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.api.common.state.ValueState;
import org.apache.flink.api.common.state.ValueStateDescriptor;
import org.apache.flink.api.common.typeutils.TypeSerializer;
import org.apache.flink.api.common.typeutils.base.LongSerializer;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.metrics.Counter;
import org.apache.flink.runtime.state.CheckpointableKeyedStateBackend;
import org.apache.flink.runtime.state.KeyGroupRange;
import org.apache.flink.runtime.state.KeyedStateBackend;
import org.apache.flink.runtime.state.internal.InternalValueState;
import org.apache.flink.streaming.api.operators.InternalTimerService;
import org.apache.flink.table.data.GenericRowData;
import org.apache.flink.table.data.RowData;
import org.apache.flink.table.data.TimestampData;
import org.apache.flink.table.data.binary.BinaryRowData;
import org.apache.flink.table.data.utils.JoinedRowData;
import org.apache.flink.table.runtime.operators.window.TimeWindow;
import org.apache.flink.table.runtime.operators.window.slicing.SlicingWindowProcessor;
import org.apache.flink.table.runtime.operators.window.slicing.WindowTimerService;
import org.apache.flink.table.runtime.operators.window.slicing.WindowTimerServiceImpl;
import org.apache.flink.table.runtime.operators.window.state.WindowValueState;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.time.ZoneId;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.HashSet;
import java.util.List;
import java.util.Map;
import java.util.Set;
import java.util.stream.Collectors;

import static org.apache.flink.table.runtime.util.TimeWindowUtil.isWindowFired;
import static org.apache.flink.table.runtime.util.TimeWindowUtil.toUtcTimestampMills;

/** The slicing window processor of the GPU engine. */
public final class GpuSlicingWindowProcessor implements SlicingWindowProcessor<Long> {
    private static final long serialVersionUID = 1L;
    /** the reference's state name (AbstractWindowAggProcessor.java:103-107) */
    static final String STATE_NAME = "window-aggs";

    private final GpuWindowAggSpec spec;
    private final ZoneId shiftTimeZone;

    private transient Context<Long> ctx;
    private transient Counter lateDropped;
    private transient long handle;
    private transient GpuKeyRows keys;
    private transient GpuAccRows accRows;
    private transient ByteBuffer keyCol, timeCol, valCol, nullCol;
    private transient ByteBuffer csCol, cvCol, sumCol, minCol, maxCol;   // partial input
    private transient int count;
    private transient long droppedSeen;
    private transient WindowValueState<Long> windowState;
    private transient WindowTimerService<Long> timerService;
    private transient long lastProcTimer;
    private transient boolean asyncPending;
    /** an fg_snapshot_state_async not collected (a checkpoint that failed before its wait). */
    private transient boolean snapshotPending;
    private transient boolean batchHanded;
    /** the namespaces the backend holds from the last image written (or restored), and their slices */
    private transient Map<Long, Set<Long>> imageContrib;
    /** the next window end the key timers of fired state were registered at */
    private transient long lastNextEnd;

    public GpuSlicingWindowProcessor(GpuWindowAggSpec spec, ZoneId shiftTimeZone) {
        this.spec = spec;
        this.shiftTimeZone = shiftTimeZone;
    }

    /** the operator's numLateRecordsDropped, fed from the engine's drop count */
    void attach(Counter numLateRecordsDropped) {
        this.lateDropped = numLateRecordsDropped;
    }

    private boolean proctime() {
        return (spec.flags & FgConfig.FLAG_PROCTIME) != 0;
    }

    @Override
    @SuppressWarnings("unchecked")
    public void open(Context<Long> context) throws Exception {
        this.ctx = context;
        KeyedStateBackend<RowData> backend = ctx.getKeyedStateBackend();
        KeyGroupRange range = ((CheckpointableKeyedStateBackend<?>) backend).getKeyGroupRange();
        int maxP = ctx.getRuntimeContext().getMaxNumberOfParallelSubtasks();
        int nTz = spec.tzTransitionsMs == null ? 0 : spec.tzTransitionsMs.length;
        handle =
                FlinkGpu.open(
                        FgConfig.of(spec, maxP, range.getStartKeyGroup(), range.getEndKeyGroup(), nTz),
                        spec.tzTransitionsMs,
                        spec.tzOffsetsMs);
        keys = new GpuKeyRows(spec, maxP);
        accRows = new GpuAccRows(spec.aggs, spec.valType);
        int b = spec.batchRecords;
        keyCol = GpuKeyRows.direct(8L * b);
        timeCol = GpuKeyRows.direct(8L * b);
        valCol = GpuKeyRows.direct(8L * b);
        nullCol = GpuKeyRows.direct(b);
        // the staging columns live for the operator's life: page-lock them once, so every
        // micro-batch is DMA'd straight from them (fg_host_register)
        for (ByteBuffer c : new ByteBuffer[] {keyCol, timeCol, valCol, nullCol}) {
            FlinkGpu.hostRegister(spec.device, c);
        }
        if (spec.partialInput) {
            csCol = GpuKeyRows.direct(8L * b);
            cvCol = GpuKeyRows.direct(8L * b);
            sumCol = GpuKeyRows.direct(8L * b);
            minCol = GpuKeyRows.direct(8L * b);
            maxCol = GpuKeyRows.direct(8L * b);
        }
        ValueState<RowData> state =
                backend.getOrCreateKeyedState(
                        LongSerializer.INSTANCE, new ValueStateDescriptor<>(STATE_NAME, accRows.serializer()));
        windowState = new WindowValueState<>((InternalValueState<RowData, Long, RowData>) state);
        timerService = new WindowTimerServiceImpl(ctx.getTimerService(), shiftTimeZone);
        lastProcTimer = Long.MIN_VALUE;
        imageContrib = new HashMap<>();
        lastNextEnd = Long.MIN_VALUE;
        restoreFromKeyedState(backend);
    }

    // ---- input ------------------------------------------------------------------------------

    @Override
    public boolean processElement(RowData key, RowData element) throws Exception {
        if (!keys.fits(key)) {
            flushBatch();
        }
        keys.add(key, count, keyCol);
        if (spec.partialInput) {
            // LocalAggCombiner's row (key, acc..., slice_end): the accumulators from valueIndex
            long[] p = accRows.toPartial(element, spec.valueIndex);
            timeCol.putLong(8 * count, element.getLong(spec.rowtimeIndex));
            csCol.putLong(8 * count, p[0]);
            cvCol.putLong(8 * count, p[1]);
            sumCol.putLong(8 * count, p[2]);
            minCol.putLong(8 * count, p[3]);
            maxCol.putLong(8 * count, p[4]);
        } else {
            long t;
            if (proctime()) {
                t = ctx.getTimerService().currentProcessingTime();
                registerProcTimer(t);
            } else {
                t = element.getTimestamp(spec.rowtimeIndex, 3).getMillisecond();
            }
            timeCol.putLong(8 * count, t);
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
        }
        if (++count == spec.batchRecords) {
            flushBatch();
        }
        return false;   // late drops are counted by the engine (see advanceProgress)
    }

    /** the slice grid: TUMBLE size, HOP gcd(size, slide), CUMULATE step (SliceAssigners.java:59-96) */
    private long sliceSize() {
        if (spec.windowKind == FgConfig.TUMBLE) {
            return spec.sizeMs;
        }
        if (spec.windowKind == FgConfig.HOP) {
            long a = spec.sizeMs, c = spec.slideMs;
            while (c != 0) {
                long t = a % c;
                a = c;
                c = t;
            }
            return a;
        }
        return spec.slideMs;
    }

    /** window ends: TUMBLE every size, HOP every slide, CUMULATE every step (getSliceEndInterval) */
    private long windowInterval() {
        return spec.windowKind == FgConfig.TUMBLE ? spec.sizeMs : spec.slideMs;
    }

    /**
     * one processing-time timer per new slice end (under the current key: SlicingWindowOperator
     * .onProcessingTime advances the progress for any key's timer, and the engine fires every key)
     */
    private void registerProcTimer(long now) {
        long s = sliceSize();
        long end = TimeWindow.getWindowStartWithOffset(toUtcTimestampMills(now, shiftTimeZone), spec.offsetMs, s) + s;
        if (end > lastProcTimer) {
            timerService.registerProcessingTimeWindowTimer(end);
            lastProcTimer = end;
        }
    }

    /** hands the gathered micro-batch to the engine (which has read it when this returns) */
    private void flushBatch() {
        if (count == 0) {
            return;
        }
        keys.intern(count, keyCol);
        if (spec.partialInput) {
            boolean mv = accRows.multiValue();
            FlinkGpu.addPartials(
                    handle, count, keyCol, timeCol, csCol, cvCol, sumCol, mv ? minCol : null, mv ? maxCol : null);
        } else {
            FlinkGpu.addBatch(
                    handle,
                    keyCol,
                    timeCol,
                    spec.valueIndex >= 0 ? valCol : null,
                    spec.valueIndex >= 0 ? nullCol : null,
                    count);
        }
        count = 0;
        batchHanded = true;
    }

    /** a micro-batch went to the engine since the last call (the operator releases a held watermark) */
    boolean takeBatchHanded() {
        boolean b = batchHanded;
        batchHanded = false;
        return b;
    }

    // ---- progress ---------------------------------------------------------------------------

    @Override
    public void advanceProgress(long progress) throws Exception {
        flushBatch();
        collectHeld();   // (an operator's async progress: its rows first, in order)
        ByteBuffer[] cols = new ByteBuffer[5 + spec.aggs.length];
        emit(cols, FlinkGpu.advanceProgress(handle, progress, cols));
    }

    /** fg_advance_progress_async: the fires are queued; collectHeld() returns their rows */
    void advanceAsync(long progress) {
        flushBatch();
        FlinkGpu.advanceProgressAsync(handle, progress);
        asyncPending = true;
    }

    /** the rows of every async advance since the last collect (fg_collect_fired, host memory) */
    void collectHeld() {
        if (!asyncPending) {
            return;
        }
        asyncPending = false;
        ByteBuffer[] cols = new ByteBuffer[5 + spec.aggs.length];
        emit(cols, FlinkGpu.collectFired(handle, cols));
    }

    /** fired rows -> JoinedRowData(key, [aggs..., window_start, window_end]) (collect :223-226) */
    private void emit(ByteBuffer[] cols, long n) {
        for (ByteBuffer c : cols) {
            if (c != null) {
                c.order(ByteOrder.nativeOrder());
            }
        }
        int nAggs = spec.aggs.length;
        RowData[] keyRows = keys.rows(cols[0], (int) n);
        for (int i = 0; i < n; i++) {
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
            ctx.output(new JoinedRowData(keyRows[i], aggs));
        }
        long dropped = FlinkGpu.lateDropped(handle);
        if (lateDropped != null && dropped > droppedSeen) {
            lateDropped.inc(dropped - droppedSeen);
        }
        droppedSeen = dropped;
    }

    // ---- checkpoints ------------------------------------------------------------------------

    @Override
    public void prepareCheckpoint() throws Exception {
        flushBatch();
        collectHeld();
        FlinkGpu.flush(handle);
        if (snapshotPending) {   // (a failed checkpoint's image: collected and dropped)
            FlinkGpu.snapshotStateWait(handle, new ByteBuffer[7], new long[1]);
            snapshotPending = false;
        }
        // the image's export and host copy run on the GPU while the previous image is cleared
        FlinkGpu.snapshotStateAsync(handle);
        snapshotPending = true;
        writeKeyedState();
    }

    /**
     * The engine's (key, slice) accumulators into "window-aggs" as the reference keeps them, and
     * the window timers AggCombiner / SliceSharedWindowAggProcessor would hold -- incrementally: the
     * backend keeps what earlier checkpoints wrote, and a barrier rewrites only what changed since
     * (the reference's prepareCheckpoint flushes its buffer into state it already keeps,
     * AbstractWindowAggProcessor.java:195-197; AggCombiner.combine touches only the (key, slice)
     * pairs a flush saw, AggCombiner.java:76-115). Per image slice the engine says whether its table
     * was written since the previous image (fg_snapshot_slices, ABI 16):
     *  - a slice's namespace is its end; a CUMULATE slice of a fired window maps to the window's first
     *    slice, where CumulativeSliceAssigner.mergeSlices keeps the fired state (SliceAssigners.java:
     *    359-370). A namespace is rewritten -- its accumulator rows put, its window timer registered
     *    (AggCombiner.java:104-112; the timer service deduplicates) -- iff one of its slices changed;
     *    a namespace whose slices are not the ones it held at the last image is rebuilt (cleared first);
     *  - namespaces of the previous image that are gone (fired, expired) are cleared; their timers
     *    have fired: the operator forwards a watermark only after the engine fired its windows;
     *  - a key holding state of fired slices (HOP / CUMULATE) holds a timer at the next window end
     *    after the progress (fireWindow's nextTriggerWindow registration): registered for the keys of
     *    rewritten namespaces, and for every such key when that next window end moved.
     * Round 5 cleared every entry, deleted every timer and wrote the whole image at every barrier on
     * the task thread. Mirror: flink_amd/keyed_state.py (tests/test_gpu_incremental_state.py checks
     * it against that full rewrite, and a failover restored from the written backend).
     */
    private void writeKeyedState() throws Exception {
        KeyedStateBackend<RowData> backend = ctx.getKeyedStateBackend();
        ByteBuffer[] cols = new ByteBuffer[7];
        long[] wm = new long[1];
        FlinkGpu.snapshotStateWait(handle, cols, wm);
        snapshotPending = false;
        for (ByteBuffer c : cols) {
            if (c != null) {
                c.order(ByteOrder.nativeOrder());
            }
        }
        final long progress = wm[0];
        final long[] sl = FlinkGpu.snapshotSlices(handle);
        final int ns = (int) sl[0];
        // namespaces of the image: their slices, whether one changed
        Map<Long, Set<Long>> contrib = new HashMap<>();
        Map<Long, Boolean> changed = new HashMap<>();
        long[] nsOf = new long[ns];
        for (int i = 0; i < ns; i++) {
            long slice = sl[1 + i];
            nsOf[i] = namespaceOf(slice, progress);
            contrib.computeIfAbsent(nsOf[i], k -> new HashSet<>()).add(slice);
            changed.merge(nsOf[i], sl[1 + 3 * ns + i] != 0, Boolean::logicalOr);
        }
        Set<Long> rebuild = new HashSet<>();
        for (Map.Entry<Long, Set<Long>> e : contrib.entrySet()) {
            Set<Long> before = imageContrib.get(e.getKey());
            if (before != null && !before.equals(e.getValue())) {
                rebuild.add(e.getKey());
                changed.put(e.getKey(), true);
            }
        }
        Set<Long> clear = new HashSet<>(rebuild);
        for (Long n : imageContrib.keySet()) {
            if (!contrib.containsKey(n)) {
                clear.add(n);
            }
        }
        for (Long n : clear) {   // (gone, or rebuilt: its keys from the backend)
            List<RowData> keysOfNs = backend.<Long>getKeys(STATE_NAME, n).collect(Collectors.toList());
            for (RowData k : keysOfNs) {
                backend.setCurrentKey(k);
                windowState.clear(n);
            }
        }
        long interval = windowInterval();
        long nextEnd =
                TimeWindow.getWindowStartWithOffset(toUtcTimestampMills(progress, shiftTimeZone), spec.offsetMs, interval)
                        + interval;
        boolean nextMoved = nextEnd != lastNextEnd;
        // the rows of the slices to read: those of rewritten namespaces, and of fired slices when the
        // next window end moved (their keys' next-window timers)
        Map<Long, Map<BinaryRowData, RowData>> image = new HashMap<>();
        Set<BinaryRowData> needNextTimer = new HashSet<>();
        for (int i = 0; i < ns; i++) {
            long slice = sl[1 + i];
            boolean write = changed.get(nsOf[i]);
            boolean fired = isWindowFired(slice, progress, shiftTimeZone);
            if (!write && !(fired && nextMoved)) {
                continue;
            }
            int first = (int) sl[1 + ns + i], rows = (int) sl[1 + 2 * ns + i];
            RowData[] keyRows = keys.rows(slice(cols[0], first, rows), rows);
            for (int r = 0; r < rows; r++) {
                BinaryRowData key = (BinaryRowData) keyRows[r];
                if (fired && !proctime()) {
                    needNextTimer.add(key);
                }
                if (!write) {
                    continue;
                }
                int at = first + r;
                GenericRowData acc =
                        accRows.fromPartial(
                                cols[2].getLong(8 * at),
                                cols[3].getLong(8 * at),
                                cols[4].getLong(8 * at),
                                cols[5] == null ? cols[4].getLong(8 * at) : cols[5].getLong(8 * at),
                                cols[6] == null ? cols[4].getLong(8 * at) : cols[6].getLong(8 * at));
                Map<BinaryRowData, RowData> m = image.computeIfAbsent(nsOf[i], k -> new HashMap<>());
                RowData prev = m.get(key);
                m.put(key, prev == null ? acc : accRows.merge(prev, acc));
            }
        }
        for (Map.Entry<Long, Map<BinaryRowData, RowData>> e : image.entrySet()) {
            long n = e.getKey();
            boolean timer = !proctime() && !isWindowFired(n, progress, shiftTimeZone);
            for (Map.Entry<BinaryRowData, RowData> kv : e.getValue().entrySet()) {
                backend.setCurrentKey(kv.getKey());
                windowState.update(n, kv.getValue());
                if (timer) {
                    timerService.registerEventTimeWindowTimer(n);
                }
            }
        }
        for (BinaryRowData key : needNextTimer) {
            backend.setCurrentKey(key);
            timerService.registerEventTimeWindowTimer(nextEnd);
        }
        imageContrib = contrib;
        lastNextEnd = nextEnd;
    }

    /** the namespace of a slice's state at `progress` (CUMULATE: a fired slice's window's first slice) */
    private long namespaceOf(long slice, long progress) {
        if (spec.windowKind == FgConfig.CUMULATE && isWindowFired(slice, progress, shiftTimeZone)) {
            return TimeWindow.getWindowStartWithOffset(slice - 1, spec.offsetMs, spec.sizeMs) + spec.slideMs;
        }
        return slice;
    }

    /** rows [first, first + n) of an 8-byte image column, as a buffer of their own */
    private static ByteBuffer slice(ByteBuffer col, int first, int n) {
        ByteBuffer d = col.duplicate();
        d.position(8 * first);
        d.limit(8 * (first + n));
        return d.slice().order(ByteOrder.nativeOrder());
    }

    /**
     * initializeState: "window-aggs" of the subtask's key groups back into the engine (one
     * dictionary intern of every key row); the timer watermark is the smallest registered window
     * timer's time - 1: every window ending before it has fired (a key with state holds a timer
     * at its first unfired window), none after it has.
     */
    private void restoreFromKeyedState(KeyedStateBackend<RowData> backend) throws Exception {
        List<Tuple2<RowData, Long>> entries =
                backend.<Long>getKeysAndNamespaces(STATE_NAME).collect(Collectors.toList());
        if (entries.isEmpty()) {
            return;
        }
        int n = entries.size();
        ByteBuffer[] c = new ByteBuffer[7];
        for (int j = 0; j < 7; j++) {
            c[j] = GpuKeyRows.direct(8L * n);
        }
        byte[][] rows = new byte[n][];
        for (int i = 0; i < n; i++) {
            Tuple2<RowData, Long> kn = entries.get(i);
            backend.setCurrentKey(kn.f0);
            long[] p = accRows.toPartial(windowState.value(kn.f1), 0);
            if (spec.bigintKey) {
                c[0].putLong(8 * i, kn.f0.getLong(0));
            } else {
                BinaryRowData r = (BinaryRowData) kn.f0;
                rows[i] = new byte[r.getSizeInBytes()];
                r.getSegments()[0].get(r.getOffset(), rows[i]);
            }
            c[1].putLong(8 * i, kn.f1);
            for (int j = 0; j < 5; j++) {
                c[2 + j].putLong(8 * i, p[j]);
            }
        }
        keys.internRows(rows, c[0]);
        // the backend holds these namespaces (each its own slice: which slices folded into a restored
        // CUMULATE namespace is not kept -- the first checkpoint rebuilds those)
        for (Tuple2<RowData, Long> kn : entries) {
            imageContrib.computeIfAbsent(kn.f1, k -> new HashSet<>()).add(kn.f1);
        }
        long[] minTimer = {Long.MAX_VALUE};
        ctx.getTimerService()
                .forEachEventTimeTimer((w, ts) -> minTimer[0] = Math.min(minTimer[0], ts));
        long timerWm = minTimer[0] == Long.MAX_VALUE ? Long.MIN_VALUE : minTimer[0] - 1;
        boolean mv = accRows.multiValue();
        FlinkGpu.restore(handle, n, c[0], c[1], c[2], c[3], c[4], mv ? c[5] : null, mv ? c[6] : null, timerWm);
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
            for (ByteBuffer b : new ByteBuffer[] {keyCol, timeCol, valCol, nullCol}) {
                FlinkGpu.hostUnregister(spec.device, b);
            }
        }
        if (keys != null) {
            keys.close();
        }
    }

    @Override
    public TypeSerializer<Long> createWindowSerializer() {
        return LongSerializer.INSTANCE;
    }
}
