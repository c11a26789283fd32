/*
 * WindowBuffer of the LOCAL phase of the two-phase window aggregation: a drop-in for
 * RecordsWindowBuffer + LocalAggCombiner behind the unchanged LocalSlicingWindowAggOperator
 * (LocalSlicingWindowAggOperator.java:44-52,95-144). The planner builds
 * `new RecordsWindowBuffer.LocalFactory(keySer, valueSer, new LocalAggCombiner.Factory(..))` at
 * StreamExecLocalWindowAggregate.java:149-155; with the GPU engine it passes
 * `new GpuLocalWindowBuffer.LocalFactory(spec)` instead (INTEGRATION.md section 5).
 *
 * A flush emits one row per (key, slice) as LocalAggCombiner.combine does
 * (LocalAggCombiner.java:69-106): JoinedRowData(key, JoinedRowData(accumulators, slice_end)).
 * The operator keeps no state (prepareSnapshotPreBarrier flushes the buffer to the output), so
 * checkpoints and failover are the reference's own.
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.api.common.functions.RuntimeContext;
import org.apache.flink.runtime.memory.MemoryManager;
import org.apache.flink.table.data.GenericRowData;
import org.apache.flink.table.data.RowData;
import org.apache.flink.table.data.utils.JoinedRowData;
import org.apache.flink.table.runtime.operators.aggregate.window.buffers.WindowBuffer;
import org.apache.flink.util.Collector;

import java.time.ZoneId;

/** The local window buffer of the GPU engine. */
public final class GpuLocalWindowBuffer extends GpuPartialsBuffer {
    private final Collector<RowData> collector;

    GpuLocalWindowBuffer(GpuWindowAggSpec spec, int maxParallelism, Collector<RowData> collector, ZoneId shiftTimeZone) {
        super(spec, maxParallelism, shiftTimeZone);
        this.collector = collector;
    }

    @Override
    protected void combine(RowData key, long sliceEnd, GenericRowData acc) {
        collector.collect(new JoinedRowData(key, new JoinedRowData(acc, GenericRowData.of(sliceEnd))));
    }

    /** WindowBuffer.LocalFactory of the GPU engine (StreamExecLocalWindowAggregate.java:149-155). */
    public static final class LocalFactory implements WindowBuffer.LocalFactory {
        private static final long serialVersionUID = 1L;
        private final GpuWindowAggSpec spec;

        public LocalFactory(GpuWindowAggSpec spec) {
            this.spec = spec;
        }

        @Override
        public WindowBuffer create(
                Object operatorOwner,
                MemoryManager memoryManager,
                long memorySize,
                RuntimeContext runtimeContext,
                Collector<RowData> collector,
                ZoneId shiftTimeZone)
                throws Exception {
            return new GpuLocalWindowBuffer(
                    spec, runtimeContext.getMaxNumberOfParallelSubtasks(), collector, shiftTimeZone);
        }
    }
}
