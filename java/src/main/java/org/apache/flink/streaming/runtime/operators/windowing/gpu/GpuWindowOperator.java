/*
 * DataStream keyBy(f0).window(Tumbling|SlidingEventTimeWindows).sum / min / max(1) (and minBy /
 * maxBy, which give the same Tuple2) -- GpuWindowOperator.reduce -- and .aggregate(f) with the
 * GPU's AggregateFunctions (GpuAggregateFunctions: COUNT, SUM, AVG, MIN, MAX) --
 * GpuWindowOperator.aggregate, WindowedStream.java:283-349 -> WindowOperatorBuilder.aggregate
 * :198-224, state an AggregatingState of the function's accumulator -- on Tuple2<Long, Long> or
 * Tuple2<Long, Double> as one operator backed by the GPU engine in FG_MODE_DATASTREAM. Replaces WindowOperator + EventTimeTrigger +
 * HeapReducingState (WindowOperator.java:300-503, built by WindowOperatorBuilder.java:150-172 from
 * WindowedStream.sum / min / max, WindowedStream.java:671-850), with the reference's keyed-state
 * layout on both sides of a checkpoint:
 *
 *   processElement     -> (key, timestamp, value) appended to direct buffers; a full micro-batch
 *                         goes to fg_add_batch
 *   processWatermark   -> the pending batch, fg_advance_progress: every window whose
 *                         maxTimestamp the watermark passes fires with the aggregator's result,
 *                         emitted at window.maxTimestamp() (emitWindowContents :574-579), before
 *                         the watermark is forwarded
 *   prepareSnapshotPreBarrier -> "window-contents": the ReducingState of the input type in the TimeWindow
 *                         namespace (WindowOperatorBuilder.java:71,165-167) -- one reduced Tuple2 per
 *                         (key, window), a sliding window's value the reduce of its slices -- and
 *                         "window-timers" (WindowOperator.java:225): the trigger timer of every
 *                         window not fired yet, the cleanup timer at maxTimestamp + allowedLateness
 *                         (:630-642,669-673). A CPU WindowOperator restores this image.
 *   initializeState    -> an image of the same layout (the CPU operator's or this one's) is held as
 *                         restored window contents; the engine restarts at Long.MIN_VALUE (as the
 *                         restored timer service does). A fired GPU row of a restored (key, window)
 *                         is reduced with the restored value; a restored window whose trigger timer
 *                         is pending and that fired no GPU row emits its restored value alone.
 *
 * The timers this operator registers are for the image only: the engine fires the windows, so
 * onEventTime / onProcessingTime do nothing. flink_amd/datastream.py is the Python mirror of this
 * class, tested against the oracle in tests/test_gpu_datastream_state.py.
 * The late-drop count feeds numLateRecordsDropped (WindowOperator.java:222).
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import org.apache.flink.api.common.ExecutionConfig;
import org.apache.flink.api.common.functions.ReduceFunction;
import org.apache.flink.api.common.state.ReducingStateDescriptor;
import org.apache.flink.api.common.state.StateDescriptor;
import org.apache.flink.api.common.typeinfo.BasicTypeInfo;
import org.apache.flink.api.common.typeinfo.TypeInformation;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.typeutils.TupleTypeInfo;
import org.apache.flink.metrics.Counter;
import org.apache.flink.runtime.state.CheckpointableKeyedStateBackend;
import org.apache.flink.runtime.state.KeyGroupRange;
import org.apache.flink.runtime.state.StateInitializationContext;
import org.apache.flink.runtime.state.internal.InternalAppendingState;
import org.apache.flink.streaming.api.functions.aggregation.AggregationFunction;
import org.apache.flink.streaming.api.functions.aggregation.ComparableAggregator;
import org.apache.flink.streaming.api.functions.aggregation.SumAggregator;
import org.apache.flink.streaming.api.operators.AbstractStreamOperator;
import org.apache.flink.streaming.api.operators.InternalTimer;
import org.apache.flink.streaming.api.operators.InternalTimerService;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.operators.TimestampedCollector;
import org.apache.flink.streaming.api.operators.Triggerable;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.api.windowing.windows.TimeWindow;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;
import org.apache.flink.table.runtime.operators.window.gpu.FgConfig;
import org.apache.flink.table.runtime.operators.window.gpu.FlinkGpu;
import org.apache.flink.table.runtime.operators.window.gpu.GpuWindowAggSpec;

import java.io.Serializable;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.HashMap;
import java.util.HashSet;
import java.util.Iterator;
import java.util.List;
import java.util.Map;
import java.util.Set;
import java.util.TreeMap;
import java.util.stream.Collectors;

/** keyBy(f0).window(...) reduce / aggregate over Tuple2<Long, V> (V = Long or Double) on the GPU. */
public final class GpuWindowOperator<V, ACC, OUT> extends AbstractStreamOperator<OUT>
        implements OneInputStreamOperator<Tuple2<Long, V>, OUT>, Triggerable<Long, TimeWindow> {
    private static final long serialVersionUID = 3L;
    private static final String WINDOW_STATE_NAME = "window-contents";   // WindowOperatorBuilder.java:71
    private static final String WINDOW_TIMERS_NAME = "window-timers";    // WindowOperator.java:225

    /** The WindowedStream reduce: sum(1), min(1) / minBy(1), max(1) / maxBy(1). */
    public enum Aggregation {
        SUM,
        MIN,
        MAX
    }

    /**
     * The map between a window's state value (ACC: the reduced Tuple2, or an AggregateFunction's
     * accumulator), its output and the engine's per-(key, window) accumulator: the value
     * accumulator's bits a0 (SUM / MIN / MAX of f1) and the record count a1.
     */
    public interface Accumulation<V, ACC, OUT> extends Serializable {
        /** the engine's value aggregate (FgConfig.AGG_SUM / AGG_MIN / AGG_MAX), -1: none (COUNT) */
        int valueAgg();

        /** "window-contents": WindowOperatorBuilder's descriptor for this reduce / aggregate */
        StateDescriptor<?, ACC> stateDescriptor(String name, TypeInformation<Tuple2<Long, V>> in, ExecutionConfig config);

        ACC fromBits(long key, long a0, long a1);

        long[] toBits(ACC acc);

        /** merge(a, b), a the earlier accumulator (value1 of a reduce) */
        long[] merge(long a0, long a1, long b0, long b1) throws Exception;

        OUT output(long key, long a0, long a1);
    }

    /** WindowedStream.sum / min / max: the reference's own SumAggregator / ComparableAggregator. */
    static final class ReduceAccumulation<V> implements Accumulation<V, Tuple2<Long, V>, Tuple2<Long, V>> {
        private static final long serialVersionUID = 1L;
        private final Aggregation aggregation;
        private final boolean isDouble;
        private transient ReduceFunction<Tuple2<Long, V>> reducer;

        ReduceAccumulation(Aggregation aggregation, boolean isDouble) {
            this.aggregation = aggregation;
            this.isDouble = isDouble;
        }

        @Override
        public int valueAgg() {
            return aggregation == Aggregation.SUM
                    ? FgConfig.AGG_SUM
                    : aggregation == Aggregation.MIN ? FgConfig.AGG_MIN : FgConfig.AGG_MAX;
        }

        @Override
        public StateDescriptor<?, Tuple2<Long, V>> stateDescriptor(
                String name, TypeInformation<Tuple2<Long, V>> in, ExecutionConfig config) {
            // WindowedStream.sum / min / max build exactly these aggregators (:671-850), and
            // WindowOperatorBuilder.reduce their ReducingStateDescriptor (:165-167)
            reducer =
                    aggregation == Aggregation.SUM
                            ? new SumAggregator<>(1, in, config)
                            : new ComparableAggregator<>(
                                    1,
                                    in,
                                    aggregation == Aggregation.MIN
                                            ? AggregationFunction.AggregationType.MIN
                                            : AggregationFunction.AggregationType.MAX,
                                    config);
            return new ReducingStateDescriptor<>(name, reducer, in.createSerializer(config));
        }

        private long bits(V v) {
            return isDouble ? Double.doubleToRawLongBits((Double) v) : (Long) v;
        }

        @SuppressWarnings("unchecked")
        private V value(long bits) {
            return (V) (isDouble ? (Object) Double.longBitsToDouble(bits) : (Object) bits);
        }

        @Override
        public Tuple2<Long, V> fromBits(long key, long a0, long a1) {
            return Tuple2.of(key, value(a0));
        }

        @Override
        public long[] toBits(Tuple2<Long, V> acc) {
            return new long[] {bits(acc.f1), 1L};
        }

        @Override
        public long[] merge(long a0, long a1, long b0, long b1) throws Exception {
            return new long[] {bits(reducer.reduce(fromBits(0L, a0, a1), fromBits(0L, b0, b1)).f1), a1 + b1};
        }

        @Override
        public Tuple2<Long, V> output(long key, long a0, long a1) {
            return fromBits(key, a0, a1);
        }
    }

    private final GpuWindowAggSpec spec;
    private final TypeInformation<Tuple2<Long, V>> inputType;
    private final Accumulation<V, ACC, OUT> acc;
    private final boolean isDouble;
    private final boolean hasValue;
    private final boolean purging;

    private transient long handle;
    private transient ByteBuffer keys, timestamps, vals;
    private transient int count;
    private transient long droppedSeen;
    private transient long currentWatermark;
    private transient Counter numLateRecordsDropped;
    private transient TimestampedCollector<OUT> collector;
    private transient InternalAppendingState<Long, TimeWindow, Tuple2<Long, V>, ACC, ?> windowState;
    private transient InternalTimerService<TimeWindow> timers;
    /** Restored window contents by window end (initializeState), until their cleanup time. */
    private transient TreeMap<Long, Restored> restored;
    /** window ends the backend holds from the last image written (or restored) */
    private transient Set<Long> imageWindows;

    /** A restored window: keys (sorted), accumulators (a0, a1), trigger pending, holding state. */
    private static final class Restored {
        final long[] keys;
        final long[] a0;
        final long[] a1;
        final boolean[] pending;
        final boolean[] alive;

        Restored(long[] keys, long[] a0, long[] a1, boolean[] pending) {
            this.keys = keys;
            this.a0 = a0;
            this.a1 = a1;
            this.pending = pending;
            this.alive = new boolean[keys.length];
            Arrays.fill(alive, true);
        }
    }

    /**
     * WindowedStream.sum / min / max(1). spec: windowKind TUMBLE or HOP (sliding), sizeMs /
     * slideMs / offsetMs, allowedLatenessMs, flags FgConfig.FLAG_PURGING_TRIGGER for
     * PurgingTrigger.of(EventTimeTrigger).
     */
    public static <V> GpuWindowOperator<V, Tuple2<Long, V>, Tuple2<Long, V>> reduce(
            GpuWindowAggSpec spec, TypeInformation<Tuple2<Long, V>> inputType, Aggregation aggregation) {
        return new GpuWindowOperator<>(spec, inputType, new ReduceAccumulation<>(aggregation, isDouble(inputType)));
    }

    /** WindowedStream.aggregate(f) with one of GpuAggregateFunctions' functions. */
    public static <V, ACC, R> GpuWindowOperator<V, ACC, R> aggregate(
            GpuWindowAggSpec spec,
            TypeInformation<Tuple2<Long, V>> inputType,
            GpuAggregateFunctions.GpuAggregate<V, ACC, R> function) {
        if (function.isDouble != isDouble(inputType)) {
            throw new IllegalArgumentException("the aggregate function's field type differs from the input's");
        }
        return new GpuWindowOperator<>(spec, inputType, function);
    }

    private static boolean isDouble(TypeInformation<?> inputType) {
        TypeInformation<?> f1 = ((TupleTypeInfo<?>) inputType).getTypeAt(1);
        if (!f1.equals(BasicTypeInfo.LONG_TYPE_INFO) && !f1.equals(BasicTypeInfo.DOUBLE_TYPE_INFO)) {
            throw new IllegalArgumentException("GPU window aggregation of a Long or Double field, got " + f1);
        }
        return f1.equals(BasicTypeInfo.DOUBLE_TYPE_INFO);
    }

    private GpuWindowOperator(
            GpuWindowAggSpec spec, TypeInformation<Tuple2<Long, V>> inputType, Accumulation<V, ACC, OUT> acc) {
        this.isDouble = isDouble(inputType);
        this.hasValue = acc.valueAgg() >= 0;
        spec.mode = FgConfig.MODE_DATASTREAM;
        spec.valType = !hasValue ? FgConfig.VAL_NONE : isDouble ? FgConfig.VAL_F64 : FgConfig.VAL_I64;
        spec.aggs = hasValue ? new int[] {FgConfig.AGG_COUNT_STAR, acc.valueAgg()} : new int[] {FgConfig.AGG_COUNT_STAR};
        this.spec = spec;
        this.inputType = inputType;
        this.acc = acc;
        this.purging = (spec.flags & FgConfig.FLAG_PURGING_TRIGGER) != 0;
    }

    @Override
    @SuppressWarnings({"unchecked", "rawtypes"})
    public void initializeState(StateInitializationContext context) throws Exception {
        super.initializeState(context);
        StateDescriptor desc = acc.stateDescriptor(WINDOW_STATE_NAME, inputType, getExecutionConfig());
        windowState =
                (InternalAppendingState<Long, TimeWindow, Tuple2<Long, V>, ACC, ?>)
                        getOrCreateKeyedState(new TimeWindow.Serializer(), desc);
    }

    @Override
    public void open() throws Exception {
        super.open();
        collector = new TimestampedCollector<>(output);
        numLateRecordsDropped = metrics.counter("numLateRecordsDropped");
        timers = getInternalTimerService(WINDOW_TIMERS_NAME, new TimeWindow.Serializer(), this);
        KeyGroupRange range =
                ((CheckpointableKeyedStateBackend<?>) getKeyedStateBackend()).getKeyGroupRange();
        handle =
                FlinkGpu.open(
                        FgConfig.of(
                                spec,
                                getRuntimeContext().getMaxNumberOfParallelSubtasks(),
                                range.getStartKeyGroup(),
                                range.getEndKeyGroup(),
                                0),
                        null,
                        null);
        keys = direct(8L * spec.batchRecords);
        timestamps = direct(8L * spec.batchRecords);
        vals = hasValue ? direct(8L * spec.batchRecords) : null;
        currentWatermark = Long.MIN_VALUE;
        restored = new TreeMap<>();
        imageWindows = new HashSet<>();
        restoreImage();
        imageWindows.addAll(restored.keySet());
    }

    private static ByteBuffer direct(long bytes) {
        return ByteBuffer.allocateDirect((int) Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
    }

    private long bitsOf(V v) {
        return isDouble ? Double.doubleToRawLongBits((Double) v) : (Long) v;
    }

    /** WindowOperator.cleanupTime (:669-673). */
    private long cleanupTime(long end) {
        long maxTs = end - 1;
        long c = maxTs + spec.allowedLatenessMs;
        return c >= maxTs ? c : Long.MAX_VALUE;
    }

    @Override
    public void processElement(StreamRecord<Tuple2<Long, V>> element) throws Exception {
        keys.putLong(8 * count, element.getValue().f0);
        timestamps.putLong(8 * count, element.getTimestamp());
        if (hasValue) {
            vals.putLong(8 * count, bitsOf(element.getValue().f1));
        }
        if (++count == spec.batchRecords) {
            flushBatch();
        }
    }

    private void flushBatch() {
        if (count > 0) {
            FlinkGpu.addBatch(handle, keys, timestamps, vals, null, count);
            count = 0;
        }
    }

    private void emit(long key, long end, long a0, long a1) {
        collector.setAbsoluteTimestamp(end - 1);   // window.maxTimestamp()
        collector.collect(acc.output(key, a0, a1));
    }

    @Override
    public void processWatermark(Watermark mark) throws Exception {
        flushBatch();
        long wm = mark.getTimestamp();
        ByteBuffer[] cols = new ByteBuffer[7];
        long n = FlinkGpu.advanceProgress(handle, wm, cols);
        for (ByteBuffer c : cols) {
            if (c != null) {
                c.order(ByteOrder.nativeOrder());
            }
        }
        // columns: key, window_start, window_end, COUNT(*)[, the value aggregate], null mask, rowtime
        for (int i = 0; i < n; i++) {
            long key = cols[0].getLong(8 * i);
            long end = cols[2].getLong(8 * i);
            long a1 = cols[3].getLong(8 * i);
            long a0 = hasValue ? cols[4].getLong(8 * i) : 0L;
            Restored r = restored.get(end);
            if (r != null) {
                int at = Arrays.binarySearch(r.keys, key);
                if (at >= 0 && r.alive[at]) {
                    long[] m = acc.merge(r.a0[at], r.a1[at], a0, a1);
                    a0 = m[0];
                    a1 = m[1];
                    r.pending[at] = false;
                    if (purging) {
                        r.alive[at] = false;
                    }
                }
            }
            emit(key, end, a0, a1);
        }
        for (Iterator<Map.Entry<Long, Restored>> it = restored.entrySet().iterator(); it.hasNext(); ) {
            Map.Entry<Long, Restored> e = it.next();
            long end = e.getKey();
            Restored r = e.getValue();
            if (end - 1 <= wm) {   // the trigger: pending restored contents without a GPU row
                for (int j = 0; j < r.keys.length; j++) {
                    if (r.pending[j] && r.alive[j]) {
                        emit(r.keys[j], end, r.a0[j], r.a1[j]);
                        if (purging) {
                            r.alive[j] = false;
                        }
                    }
                    r.pending[j] = false;
                }
            }
            boolean any = false;
            for (boolean a : r.alive) {
                any |= a;
            }
            if (cleanupTime(end) <= wm || !any) {
                it.remove();
            }
        }
        currentWatermark = Math.max(currentWatermark, wm);
        long dropped = FlinkGpu.lateDropped(handle);
        numLateRecordsDropped.inc(dropped - droppedSeen);
        droppedSeen = dropped;
        super.processWatermark(mark);
    }

    @Override
    public void onEventTime(InternalTimer<Long, TimeWindow> timer) {
        // the engine fires and cleans the windows; the timers describe them for the image only
    }

    @Override
    public void onProcessingTime(InternalTimer<Long, TimeWindow> timer) {}

    /**
     * The pending batch and the engine's buffer flushed, then the image written into keyed state
     * and the timer service here, before the barrier: StreamOperatorStateHandler.snapshotState
     * writes the timers to raw keyed state before it calls the operator's snapshotState
     * (StreamOperatorStateHandler.java:198-218).
     */
    @Override
    public void prepareSnapshotPreBarrier(long checkpointId) throws Exception {
        flushBatch();
        FlinkGpu.flush(handle);
        writeImage();
    }

    /**
     * The image into "window-contents" and the timers, incrementally: a window's entries are
     * rewritten only when one of its slices was written since the previous image
     * (fg_snapshot_slices, ABI 16); windows no longer in the image are cleared; the others stay as
     * an earlier barrier wrote them (round 5 cleared and rewrote the whole state every barrier).
     */
    private void writeImage() throws Exception {
        ByteBuffer[] cols = new ByteBuffer[7];
        long[] wmOut = new long[1];
        long n = FlinkGpu.snapshotState(handle, cols, wmOut);
        for (ByteBuffer c : cols) {
            if (c != null) {
                c.order(ByteOrder.nativeOrder());
            }
        }
        long wm = currentWatermark;
        long slide = spec.windowKind == FgConfig.TUMBLE ? spec.sizeMs : spec.slideMs;
        long perSlice = spec.sizeMs / slide;
        long[] sl = FlinkGpu.snapshotSlices(handle);
        int nsl = (int) sl[0];
        Set<Long> changedSlices = new HashSet<>();
        for (int i = 0; i < nsl; i++) {
            if (sl[1 + 3 * nsl + i] != 0) {
                changedSlices.add(sl[1 + i]);
            }
        }
        // per (key, window): the restored accumulator first (value1 of the merge), then every slice
        Map<Long, Map<Long, long[]>> contents = new HashMap<>();   // window end -> key -> (a0, a1)
        for (Map.Entry<Long, Restored> e : restored.entrySet()) {
            Restored r = e.getValue();
            Map<Long, long[]> w = contents.computeIfAbsent(e.getKey(), x -> new HashMap<>());
            for (int j = 0; j < r.keys.length; j++) {
                if (r.alive[j]) {
                    w.put(r.keys[j], new long[] {r.a0[j], r.a1[j]});
                }
            }
        }
        // state columns: key, slice_end, cnt_star, cnt_val, the value accumulator
        for (int i = 0; i < n; i++) {
            long key = cols[0].getLong(8 * i);
            long sliceEnd = cols[1].getLong(8 * i);
            long a1 = cols[2].getLong(8 * i);
            long a0 = hasValue ? cols[4].getLong(8 * i) : 0L;
            for (long j = 0; j < perSlice; j++) {
                long end = sliceEnd + j * slide;
                if (cleanupTime(end) <= wm || (purging && end - 1 <= wm)) {
                    continue;   // cleared (clearAllState), or fired and purged
                }
                Map<Long, long[]> w = contents.computeIfAbsent(end, x -> new HashMap<>());
                long[] prev = w.get(key);
                w.put(key, prev == null ? new long[] {a0, a1} : acc.merge(prev[0], prev[1], a0, a1));
            }
        }
        // windows gone since the previous image: cleared (their keys from the backend)
        for (Long end : imageWindows) {
            if (!contents.containsKey(end)) {
                TimeWindow window = new TimeWindow(end - spec.sizeMs, end);
                List<Long> ks =
                        getKeyedStateBackend().<TimeWindow>getKeys(WINDOW_STATE_NAME, window)
                                .map(k -> (Long) k)
                                .collect(Collectors.toList());
                for (Long k : ks) {
                    setCurrentKey(k);
                    windowState.setCurrentNamespace(window);
                    windowState.clear();
                }
            }
        }
        for (Map.Entry<Long, Map<Long, long[]>> e : contents.entrySet()) {
            long end = e.getKey();
            boolean write = !imageWindows.contains(end);
            for (long j = 0; j < perSlice && !write; j++) {
                write = changedSlices.contains(end - j * slide);
            }
            if (!write) {
                continue;   // (as an earlier barrier wrote it: none of its slices changed since)
            }
            TimeWindow window = new TimeWindow(end - spec.sizeMs, end);
            long cleanup = cleanupTime(end);
            for (Map.Entry<Long, long[]> kv : e.getValue().entrySet()) {
                setCurrentKey(kv.getKey());
                windowState.setCurrentNamespace(window);
                windowState.updateInternal(acc.fromBits(kv.getKey(), kv.getValue()[0], kv.getValue()[1]));
                if (window.maxTimestamp() > wm) {   // EventTimeTrigger.onElement's timer
                    timers.registerEventTimeTimer(window, window.maxTimestamp());
                }
                if (cleanup != Long.MAX_VALUE) {   // registerCleanupTimer
                    timers.registerEventTimeTimer(window, cleanup);
                }
            }
        }
        imageWindows = new HashSet<>(contents.keySet());
    }

    /** initializeState's image: the (key, window) accumulators and which triggers are pending. */
    private void restoreImage() throws Exception {
        List<Tuple2<Long, TimeWindow>> entries =
                getKeyedStateBackend().<TimeWindow>getKeysAndNamespaces(WINDOW_STATE_NAME)
                        .map(t -> Tuple2.of((Long) t.f0, t.f1))
                        .collect(Collectors.toList());
        if (entries.isEmpty()) {
            return;
        }
        // the pending trigger timers: (key, window) of every event-time timer at maxTimestamp
        Set<Tuple2<Long, TimeWindow>> pending = new HashSet<>();
        timers.forEachEventTimeTimer(
                (window, ts) -> {
                    if (ts == window.maxTimestamp()) {
                        pending.add(Tuple2.of((Long) getCurrentKey(), window));
                    }
                });
        Map<TimeWindow, List<long[]>> byWindow = new HashMap<>();
        for (Tuple2<Long, TimeWindow> kn : entries) {
            setCurrentKey(kn.f0);
            windowState.setCurrentNamespace(kn.f1);
            ACC a = windowState.getInternal();
            if (a == null) {
                continue;
            }
            long[] b = acc.toBits(a);
            byWindow.computeIfAbsent(kn.f1, x -> new ArrayList<>())
                    .add(new long[] {kn.f0, b[0], b[1], pending.contains(kn) ? 1 : 0});
        }
        for (Map.Entry<TimeWindow, List<long[]>> e : byWindow.entrySet()) {
            List<long[]> l = e.getValue();
            l.sort((x, y) -> Long.compare(x[0], y[0]));
            int m = l.size();
            long[] k = new long[m];
            long[] a0 = new long[m];
            long[] a1 = new long[m];
            boolean[] p = new boolean[m];
            for (int j = 0; j < m; j++) {
                k[j] = l.get(j)[0];
                a0[j] = l.get(j)[1];
                a1[j] = l.get(j)[2];
                p[j] = l.get(j)[3] != 0;
            }
            restored.put(e.getKey().getEnd(), new Restored(k, a0, a1, p));
        }
    }

    @Override
    public void close() throws Exception {
        if (handle != 0) {
            FlinkGpu.close(handle);
            handle = 0;
        }
        super.close();
    }
}
