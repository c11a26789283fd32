/*
 * The window-aggregate operator of the GPU engine: the role of SlicingWindowOperator
 * (SlicingWindowOperator.java:96-242, a final class) around GpuSlicingWindowProcessor, with one
 * difference in how a watermark moves on -- it is HELD while the engine fires its windows:
 *
 *   processWatermark(mark)  the previously held watermark is released first (see below); then
 *                           fg_advance_progress_async(mark): the pending records are handed over,
 *                           the fires queued behind them and the call returns; the watermark is
 *                           held
 *   the held watermark is released -- fg_collect_fired, its rows emitted, then the watermark
 *   forwarded (timers advanced, downstream notified) -- at the first of: the next micro-batch
 *   handed to the engine (its partition passes overlap the fires), the NEXT watermark, a
 *   processing-time callback spec.maxWatermarkHoldMs after the hold began, a checkpoint barrier
 *   (prepareSnapshotPreBarrier), a processing-time timer, end of input and close.
 *
 * No row is emitted after a watermark that passes its window (rows always precede the watermark
 * that fired them), so downstream operators see the reference's output; a watermark reaches
 * them at most one watermark interval (or maxWatermarkHoldMs of processing time) later -- also on
 * a slow or idle stream, where a micro-batch fills rarely (the reference forwards at once,
 * SlicingWindowOperator.java:207-210). spec.asyncWatermarks = false forwards every watermark at
 * once, as SlicingWindowOperator does. Metrics: numLateRecordsDropped (fed by the engine's
 * count), lateRecordsDroppedRate, watermarkLatency, as SlicingWindowOperator.java:158-174.
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.api.common.functions.RuntimeContext;
import org.apache.flink.metrics.Counter;
import org.apache.flink.metrics.MeterView;
import org.apache.flink.runtime.memory.MemoryManager;
import org.apache.flink.runtime.state.KeyedStateBackend;
import org.apache.flink.streaming.api.operators.BoundedOneInput;
import org.apache.flink.streaming.api.operators.ChainingStrategy;
import org.apache.flink.streaming.api.operators.InternalTimer;
import org.apache.flink.streaming.api.operators.InternalTimerService;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.operators.TimestampedCollector;
import org.apache.flink.streaming.api.operators.Triggerable;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;
import org.apache.flink.table.data.RowData;
import org.apache.flink.table.runtime.operators.TableStreamOperator;
import org.apache.flink.table.runtime.operators.window.slicing.SlicingWindowProcessor;

/** Keyed window aggregation on the MI355X engine, watermarks held while fires complete. */
public final class GpuSlicingWindowAggOperator extends TableStreamOperator<RowData>
        implements OneInputStreamOperator<RowData, RowData>, Triggerable<RowData, Long>, BoundedOneInput {
    private static final long serialVersionUID = 1L;

    private final GpuSlicingWindowProcessor processor;
    private final boolean async;

    private transient TimestampedCollector<RowData> collector;
    private transient InternalTimerService<Long> timers;
    private transient Counter numLateRecordsDropped;
    private transient long lastTriggeredProcessingTime;
    private final long maxHoldMs;

    private transient Watermark held;
    private transient long holdSeq;   // which hold a processing-time release callback belongs to
    private transient boolean closed;

    public GpuSlicingWindowAggOperator(GpuSlicingWindowProcessor processor, boolean asyncWatermarks) {
        this(processor, asyncWatermarks, GpuWindowAggSpec.DEFAULT_MAX_WATERMARK_HOLD_MS);
    }

    public GpuSlicingWindowAggOperator(
            GpuSlicingWindowProcessor processor, boolean asyncWatermarks, long maxWatermarkHoldMs) {
        this.processor = processor;
        this.async = asyncWatermarks;
        this.maxHoldMs = maxWatermarkHoldMs;
        setChainingStrategy(ChainingStrategy.ALWAYS);
    }

    @Override
    public void open() throws Exception {
        super.open();
        closed = false;
        held = null;
        holdSeq = 0;
        lastTriggeredProcessingTime = Long.MIN_VALUE;
        collector = new TimestampedCollector<>(output);
        collector.eraseTimestamp();
        timers = getInternalTimerService("window-timers", processor.createWindowSerializer(), this);
        numLateRecordsDropped = metrics.counter("numLateRecordsDropped");
        metrics.meter("lateRecordsDroppedRate", new MeterView(numLateRecordsDropped));
        metrics.gauge(
                "watermarkLatency",
                () -> {
                    long wm = timers.currentWatermark();
                    return wm < 0 ? 0L : timers.currentProcessingTime() - wm;
                });
        processor.attach(numLateRecordsDropped);
        final Object owner = getContainingTask();
        final MemoryManager mm = getContainingTask().getEnvironment().getMemoryManager();
        final long memorySize = computeMemorySize();
        final KeyedStateBackend<RowData> backend = getKeyedStateBackend();
        final RuntimeContext rc = getRuntimeContext();
        processor.open(
                new SlicingWindowProcessor.Context<Long>() {
                    @Override
                    public Object getOperatorOwner() {
                        return owner;
                    }

                    @Override
                    public MemoryManager getMemoryManager() {
                        return mm;
                    }

                    @Override
                    public long getMemorySize() {
                        return memorySize;
                    }

                    @Override
                    public KeyedStateBackend<RowData> getKeyedStateBackend() {
                        return backend;
                    }

                    @Override
                    public InternalTimerService<Long> getTimerService() {
                        return timers;
                    }

                    @Override
                    public void output(RowData result) {
                        collector.collect(result);
                    }

                    @Override
                    public RuntimeContext getRuntimeContext() {
                        return rc;
                    }
                });
    }

    @Override
    public void processElement(StreamRecord<RowData> element) throws Exception {
        processor.processElement((RowData) getCurrentKey(), element.getValue());
        if (held != null && processor.takeBatchHanded()) {
            release();
        }
    }

    @Override
    public void processWatermark(Watermark mark) throws Exception {
        if (!async) {
            processor.advanceProgress(mark.getTimestamp());
            super.processWatermark(mark);
            return;
        }
        if (held != null) {
            release();   // a watermark waits at most one watermark interval
        }
        processor.advanceAsync(mark.getTimestamp());
        processor.takeBatchHanded();   // (the pending records went with this advance)
        held = mark;
        final long seq = ++holdSeq;
        if (maxHoldMs >= 0) {
            // and at most maxHoldMs of processing time on an idle stream (the callback runs in the
            // task's mailbox thread, like every operator call)
            getProcessingTimeService()
                    .registerTimer(
                            getProcessingTimeService().getCurrentProcessingTime() + maxHoldMs,
                            t -> {
                                if (held != null && holdSeq == seq) {
                                    release();
                                }
                            });
        }
    }

    /** the held watermark's rows, then the watermark itself */
    private void release() throws Exception {
        Watermark mark = held;
        held = null;
        processor.collectHeld();
        super.processWatermark(mark);
    }

    @Override
    public void onEventTime(InternalTimer<RowData, Long> timer) {
        // window timers exist only as part of a checkpoint image (GpuSlicingWindowProcessor
        // .writeKeyedState); the engine fires windows itself
    }

    @Override
    public void onProcessingTime(InternalTimer<RowData, Long> timer) throws Exception {
        if (held != null) {
            release();
        }
        if (timer.getTimestamp() > lastTriggeredProcessingTime) {
            lastTriggeredProcessingTime = timer.getTimestamp();
            processor.advanceProgress(timer.getTimestamp());
        }
    }

    @Override
    public void prepareSnapshotPreBarrier(long checkpointId) throws Exception {
        if (held != null) {
            release();
        }
        processor.prepareCheckpoint();
    }

    @Override
    public void endInput() throws Exception {
        if (held != null) {
            release();
        }
    }

    @Override
    public void close() throws Exception {
        if (held != null) {
            release();
        }
        super.close();
        collector = null;
        closed = true;
        processor.close();
    }

    @Override
    public void dispose() throws Exception {
        super.dispose();
        collector = null;
        if (!closed) {
            closed = true;
            processor.close();
        }
    }
}
