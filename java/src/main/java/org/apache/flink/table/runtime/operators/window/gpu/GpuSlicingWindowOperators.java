/*
 * The plug points of the GPU engine in the planner's window-aggregate translation
 * (INTEGRATION.md section 5 has the builder lines):
 *
 *   create(spec, zone)        SlicingWindowAggOperatorBuilder.build (SlicingWindowAggOperatorBuilder
 *                             .java:127-170) returns this operator -- the engine holds the window
 *                             state and fires windows (single-phase, and the global phase of the
 *                             two-phase plan with spec.partialInput)
 *   recordsBuffer(spec)       the WindowBuffer.Factory the builder passes to the reference's own
 *                             processors instead of RecordsWindowBuffer.Factory: GPU
 *                             pre-aggregation, the reference's state and timers
 *   localBuffer(spec)         StreamExecLocalWindowAggregate.java:149-155: the LocalFactory of the
 *                             unchanged LocalSlicingWindowAggOperator (local phase)
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.table.runtime.operators.aggregate.window.buffers.WindowBuffer;

import java.time.ZoneId;

/** Factories of the GPU engine's window-aggregate operators and buffers. */
public final class GpuSlicingWindowOperators {
    private GpuSlicingWindowOperators() {}

    public static GpuSlicingWindowAggOperator create(GpuWindowAggSpec spec, ZoneId shiftTimeZone) {
        return new GpuSlicingWindowAggOperator(
                new GpuSlicingWindowProcessor(spec, shiftTimeZone), spec.asyncWatermarks, spec.maxWatermarkHoldMs);
    }

    public static WindowBuffer.Factory recordsBuffer(GpuWindowAggSpec spec) {
        return new GpuRecordsWindowBuffer.Factory(spec);
    }

    public static WindowBuffer.LocalFactory localBuffer(GpuWindowAggSpec spec) {
        return new GpuLocalWindowBuffer.LocalFactory(spec);
    }
}
