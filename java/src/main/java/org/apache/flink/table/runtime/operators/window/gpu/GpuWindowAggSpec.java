/*
 * What the planner knows about one window aggregation, in the engine's terms: the window
 * (SliceAssigners.tumbling/hopping/cumulative, SliceAssigners.java:59-96), the aggregate list
 * (Count1/Count/Sum/Avg/Sum0/Min/MaxAggFunction over one value column), the input row's
 * rowtime and value fields, and the grouping key's kind (one BIGINT column, or any key row
 * through the GPU key dictionary).
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import java.io.Serializable;

/** Serializable description of a GPU window aggregation (shipped with the operator). */
public final class GpuWindowAggSpec implements Serializable {
    private static final long serialVersionUID = 1L;

    public int mode = FgConfig.MODE_SQL;
    public int windowKind = FgConfig.TUMBLE;
    public long sizeMs;
    public long slideMs;
    public long offsetMs;
    /** fixed-offset shift zone (TIMESTAMP_LTZ); zones with transitions pass their rules. */
    public long shiftTzOffsetMs;
    public long[] tzTransitionsMs;
    public long[] tzOffsetsMs;
    public boolean tzUseDaylight;
    public int valType = FgConfig.VAL_F64;
    public int[] aggs = {FgConfig.AGG_COUNT_STAR, FgConfig.AGG_SUM, FgConfig.AGG_AVG};
    public int flags;
    public long expectedKeys;
    public long bufferRecords = 1 << 24;
    public int device;
    public long allowedLatenessMs;

    /** input row layout */
    public int rowtimeIndex;
    public int valueIndex = -1;

    /** the key row is one BIGINT column (else: interned by the key dictionary) */
    public boolean bigintKey = true;
    /** fields of the key row (BinaryRowData arity) when it is interned */
    public int keyArity = 1;

    /** records gathered before one engine call (one micro-batch) */
    public int batchRecords = 1 << 20;

    /**
     * global phase of the two-phase plan: input rows are LocalAggCombiner's (key, acc...,
     * slice_end) -- the accumulators from valueIndex, the slice end (BIGINT) at rowtimeIndex
     */
    public boolean partialInput;

    /**
     * hold each watermark while its fires complete on the GPU (fg_advance_progress_async): the
     * fired rows, then the watermark, are forwarded once the next micro-batch has been handed over
     * (or at the next watermark, checkpoint or end of input) -- GpuSlicingWindowAggOperator
     */
    public boolean asyncWatermarks = true;

    /** a held watermark is released at the latest this long (processing time) after its hold began */
    public static final long DEFAULT_MAX_WATERMARK_HOLD_MS = 200L;

    /** bound on a watermark's hold in processing time (< 0: none; the next watermark still releases it) */
    public long maxWatermarkHoldMs = DEFAULT_MAX_WATERMARK_HOLD_MS;

    /** a field-by-field copy (the arrays cloned) */
    public GpuWindowAggSpec copy() {
        GpuWindowAggSpec c = new GpuWindowAggSpec();
        c.mode = mode;
        c.windowKind = windowKind;
        c.sizeMs = sizeMs;
        c.slideMs = slideMs;
        c.offsetMs = offsetMs;
        c.shiftTzOffsetMs = shiftTzOffsetMs;
        c.tzTransitionsMs = tzTransitionsMs == null ? null : tzTransitionsMs.clone();
        c.tzOffsetsMs = tzOffsetsMs == null ? null : tzOffsetsMs.clone();
        c.tzUseDaylight = tzUseDaylight;
        c.valType = valType;
        c.aggs = aggs.clone();
        c.flags = flags;
        c.expectedKeys = expectedKeys;
        c.bufferRecords = bufferRecords;
        c.device = device;
        c.allowedLatenessMs = allowedLatenessMs;
        c.rowtimeIndex = rowtimeIndex;
        c.valueIndex = valueIndex;
        c.bigintKey = bigintKey;
        c.keyArity = keyArity;
        c.batchRecords = batchRecords;
        c.partialInput = partialInput;
        c.asyncWatermarks = asyncWatermarks;
        c.maxWatermarkHoldMs = maxWatermarkHoldMs;
        return c;
    }
}
