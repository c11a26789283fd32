/*
 * WindowBuffer.Factory of the single-phase (and global-less) window aggregation with the
 * reference's own state: a drop-in for RecordsWindowBuffer + AggCombiner behind the unchanged
 * SliceUnsharedWindowAggProcessor / SliceSharedWindowAggProcessor and SlicingWindowOperator
 * (SlicingWindowAggOperatorBuilder.java:146-170 passes `new RecordsWindowBuffer.Factory(keySer,
 * inputSer, new AggCombiner.Factory(genAggsHandler))`; with the GPU engine it passes
 * `new GpuRecordsWindowBuffer.Factory(spec)`, INTEGRATION.md section 5).
 *
 * The records of every (key, slice) are pre-aggregated on the engine; a flush merges each
 * partial accumulator into the "window-aggs" ValueState exactly as AggCombiner.combine leaves it
 * (AggCombiner.java:76-115): the state's accumulator (or createAccumulators) merged with the
 * partial by the functions' mergeExpressions, written back, and the window timer registered
 * unless the watermark has passed it. Firing, clearing, checkpoints, timers and rescaling stay
 * the reference processor's: the state and timers are the reference's, byte for byte, so a job
 * switches to this buffer (and back) across a savepoint. The fully device-resident path, with
 * the engine also firing windows, is GpuSlicingWindowProcessor.
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.api.common.functions.RuntimeContext;
import org.apache.flink.runtime.memory.MemoryManager;
import org.apache.flink.runtime.state.KeyedStateBackend;
import org.apache.flink.table.data.GenericRowData;
import org.apache.flink.table.data.RowData;
import org.apache.flink.table.runtime.operators.aggregate.window.buffers.WindowBuffer;
import org.apache.flink.table.runtime.operators.window.slicing.WindowTimerService;
import org.apache.flink.table.runtime.operators.window.state.WindowState;
import org.apache.flink.table.runtime.operators.window.state.WindowValueState;

import java.time.ZoneId;

import static org.apache.flink.table.runtime.util.TimeWindowUtil.isWindowFired;

/** The state-combining window buffer of the GPU engine. */
public final class GpuRecordsWindowBuffer extends GpuPartialsBuffer {
    private final WindowTimerService<Long> timerService;
    private final KeyedStateBackend<RowData> stateBackend;
    private final WindowValueState<Long> accState;
    private final boolean isEventTime;

    GpuRecordsWindowBuffer(
            GpuWindowAggSpec spec,
            int maxParallelism,
            WindowTimerService<Long> timerService,
            KeyedStateBackend<RowData> stateBackend,
            WindowValueState<Long> accState,
            boolean isEventTime,
            ZoneId shiftTimeZone) {
        super(spec, maxParallelism, shiftTimeZone);
        this.timerService = timerService;
        this.stateBackend = stateBackend;
        this.accState = accState;
        this.isEventTime = isEventTime;
    }

    @Override
    protected void combine(RowData key, long window, GenericRowData partial) throws Exception {
        stateBackend.setCurrentKey(key);
        RowData acc = accState.value(window);
        accState.update(window, acc == null ? partial : accRows.merge(acc, partial));
        if (isEventTime
                && !isWindowFired(window, timerService.currentWatermark(), timerService.getShiftTimeZone())) {
            timerService.registerEventTimeWindowTimer(window);
        }
        // processing-time timers: registered per record by the processor (AggCombiner.java:113-114)
    }

    /** WindowBuffer.Factory of the GPU engine (SlicingWindowAggOperatorBuilder.java:146-170). */
    public static final class Factory implements WindowBuffer.Factory {
        private static final long serialVersionUID = 1L;
        private final GpuWindowAggSpec spec;

        public Factory(GpuWindowAggSpec spec) {
            this.spec = spec;
        }

        @Override
        @SuppressWarnings("unchecked")
        public WindowBuffer create(
                Object operatorOwner,
                MemoryManager memoryManager,
                long memorySize,
                RuntimeContext runtimeContext,
                WindowTimerService<Long> timerService,
                KeyedStateBackend<RowData> stateBackend,
                WindowState<Long> windowState,
                boolean isEventTime,
                ZoneId shiftTimeZone)
                throws Exception {
            return new GpuRecordsWindowBuffer(
                    spec,
                    runtimeContext.getMaxNumberOfParallelSubtasks(),
                    timerService,
                    stateBackend,
                    (WindowValueState<Long>) windowState,
                    isEventTime,
                    shiftTimeZone);
        }
    }
}
