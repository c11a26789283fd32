/*
 * The plug point: SlicingWindowAggOperatorBuilder.build (SlicingWindowAggOperatorBuilder
 * .java:127-170) builds `new SlicingWindowOperator<>(windowProcessor)` around the processor it
 * picks at :146-170; with the GPU engine enabled it returns create(spec) instead (see
 * INTEGRATION.md for the two-line builder change). The local phase of the two-phase plan
 * (StreamExecLocalWindowAggregate.java:149-155) passes a spec with FLAG_LOCAL_PARTIALS.
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.table.data.RowData;
import org.apache.flink.table.runtime.operators.window.slicing.SlicingWindowOperator;

/** Factory of GPU-backed slicing window operators. */
public final class GpuSlicingWindowOperators {
    private GpuSlicingWindowOperators() {}

    public static SlicingWindowOperator<RowData, Long> create(GpuWindowAggSpec spec) {
        GpuSlicingWindowProcessor processor = new GpuSlicingWindowProcessor(spec);
        SlicingWindowOperator<RowData, Long> operator = new SlicingWindowOperator<>(processor);
        processor.attach(operator);
        return operator;
    }
}
