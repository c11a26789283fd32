/*
 * DataStream keyBy(f0).window(Tumbling|SlidingEventTimeWindows).sum(1) on Tuple2<Long, Long>
 * (WindowedStream.sum -> SumAggregator, WindowedStream.java:671-674,891-893) as one operator
 * backed by the GPU engine in FG_MODE_DATASTREAM. Replaces WindowOperator + EventTimeTrigger +
 * HeapReducingState (WindowOperator.java:300-503, built by WindowOperatorBuilder.java:150-172):
 *
 *   processElement     -> (key, timestamp, value) appended to direct buffers; a full micro-batch
 *                         goes to fg_add_batch
 *   processWatermark   -> the pending batch, fg_advance_progress: every window whose
 *                         maxTimestamp the watermark passes fires with its SumAggregator result,
 *                         emitted with timestamp window.maxTimestamp() (emitWindowContents
 *                         :574-579) before the watermark is forwarded
 *   prepareSnapshotPreBarrier -> pending batch + fg_flush; snapshotState writes the resident
 *                         (key, window) sums into keyed state "gpu-window-contents"
 *   allowedLateness    -> GpuWindowAggSpec.allowedLatenessMs (fg_config.allowed_lateness_ms)
 *
 * The late-drop count feeds numLateRecordsDropped (WindowOperator.java:222).
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import org.apache.flink.api.common.state.ValueState;
import org.apache.flink.api.common.state.ValueStateDescriptor;
import org.apache.flink.api.common.typeutils.base.LongSerializer;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.metrics.Counter;
import org.apache.flink.runtime.state.CheckpointableKeyedStateBackend;
import org.apache.flink.runtime.state.KeyGroupRange;
import org.apache.flink.runtime.state.StateSnapshotContext;
import org.apache.flink.streaming.api.operators.AbstractStreamOperator;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.operators.TimestampedCollector;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;
import org.apache.flink.table.runtime.operators.window.gpu.FgConfig;
import org.apache.flink.table.runtime.operators.window.gpu.FlinkGpu;
import org.apache.flink.table.runtime.operators.window.gpu.GpuWindowAggSpec;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.List;
import java.util.stream.Collectors;

/** keyBy(f0).window(...).sum(1) over Tuple2<Long, Long> on the GPU engine. */
public final class GpuWindowOperator extends AbstractStreamOperator<Tuple2<Long, Long>>
        implements OneInputStreamOperator<Tuple2<Long, Long>, Tuple2<Long, Long>> {
    private static final long serialVersionUID = 1L;
    private static final String STATE_NAME = "gpu-window-contents";

    private final GpuWindowAggSpec spec;

    private transient long handle;
    private transient ByteBuffer keys, timestamps, vals;
    private transient int count;
    private transient long droppedSeen;
    private transient Counter numLateRecordsDropped;
    private transient TimestampedCollector<Tuple2<Long, Long>> collector;

    /** spec: mode DATASTREAM, TUMBLE or HOP (sliding), valType I64, aggs {SUM} */
    public GpuWindowOperator(GpuWindowAggSpec spec) {
        spec.mode = FgConfig.MODE_DATASTREAM;
        spec.valType = FgConfig.VAL_I64;
        spec.aggs = new int[] {FgConfig.AGG_SUM};
        this.spec = spec;
    }

    @Override
    public void open() throws Exception {
        super.open();
        collector = new TimestampedCollector<>(output);
        numLateRecordsDropped = metrics.counter("numLateRecordsDropped");
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
        vals = direct(8L * spec.batchRecords);
        restore();
    }

    private static ByteBuffer direct(long bytes) {
        return ByteBuffer.allocateDirect((int) Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
    }

    @Override
    public void processElement(StreamRecord<Tuple2<Long, Long>> element) throws Exception {
        keys.putLong(8 * count, element.getValue().f0);
        timestamps.putLong(8 * count, element.getTimestamp());
        vals.putLong(8 * count, element.getValue().f1);
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

    @Override
    public void processWatermark(Watermark mark) throws Exception {
        flushBatch();
        ByteBuffer[] cols = new ByteBuffer[6];
        long n = FlinkGpu.advanceProgress(handle, mark.getTimestamp(), cols);
        for (ByteBuffer c : cols) {
            if (c != null) {
                c.order(ByteOrder.nativeOrder());
            }
        }
        for (int i = 0; i < n; i++) {   // Tuple2(key, sum) at window.maxTimestamp()
            collector.setAbsoluteTimestamp(cols[5].getLong(8 * i));
            collector.collect(Tuple2.of(cols[0].getLong(8 * i), cols[3].getLong(8 * i)));
        }
        long dropped = FlinkGpu.lateDropped(handle);
        numLateRecordsDropped.inc(dropped - droppedSeen);
        droppedSeen = dropped;
        super.processWatermark(mark);
    }

    @Override
    public void prepareSnapshotPreBarrier(long checkpointId) throws Exception {
        flushBatch();
        FlinkGpu.flush(handle);
    }

    private ValueState<long[]> stateFor(long window) throws Exception {
        return getKeyedStateBackend()
                .getPartitionedState(
                        window,
                        LongSerializer.INSTANCE,
                        new ValueStateDescriptor<>(STATE_NAME, long[].class));
    }

    @Override
    public void snapshotState(StateSnapshotContext context) throws Exception {
        List<Tuple2<Object, Long>> old =
                getKeyedStateBackend().<Long>getKeysAndNamespaces(STATE_NAME)
                        .map(t -> Tuple2.<Object, Long>of(t.f0, t.f1))
                        .collect(Collectors.toList());
        for (Tuple2<Object, Long> kn : old) {
            setCurrentKey(kn.f0);
            stateFor(kn.f1).clear();
        }
        ByteBuffer[] cols = new ByteBuffer[7];
        long[] wm = new long[1];
        long n = FlinkGpu.snapshotState(handle, cols, wm);
        for (ByteBuffer c : cols) {
            if (c != null) {
                c.order(ByteOrder.nativeOrder());
            }
        }
        for (int i = 0; i < n; i++) {   // namespace: the slice end; value: the accumulators
            setCurrentKey(cols[0].getLong(8 * i));
            stateFor(cols[1].getLong(8 * i))
                    .update(
                            new long[] {
                                cols[2].getLong(8 * i),
                                cols[3].getLong(8 * i),
                                cols[4].getLong(8 * i),
                                wm[0]
                            });
        }
        super.snapshotState(context);
    }

    private void restore() throws Exception {
        List<Tuple2<Object, Long>> entries =
                getKeyedStateBackend().<Long>getKeysAndNamespaces(STATE_NAME)
                        .map(t -> Tuple2.<Object, Long>of(t.f0, t.f1))
                        .collect(Collectors.toList());
        if (entries.isEmpty()) {
            return;
        }
        int n = entries.size();
        ByteBuffer[] c = new ByteBuffer[5];
        for (int j = 0; j < 5; j++) {
            c[j] = direct(8L * n);
        }
        long timerWm = Long.MIN_VALUE;
        for (int i = 0; i < n; i++) {
            setCurrentKey(entries.get(i).f0);
            long[] acc = stateFor(entries.get(i).f1).value();
            c[0].putLong(8 * i, (Long) entries.get(i).f0);
            c[1].putLong(8 * i, entries.get(i).f1);
            c[2].putLong(8 * i, acc[0]);
            c[3].putLong(8 * i, acc[1]);
            c[4].putLong(8 * i, acc[2]);
            timerWm = acc[3];
        }
        FlinkGpu.restore(handle, n, c[0], c[1], c[2], c[3], c[4], null, null, timerWm);
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
