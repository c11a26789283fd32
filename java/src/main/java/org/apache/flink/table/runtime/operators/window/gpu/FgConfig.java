/*
 * The fg_config image (include/flinkgpu.h) handed to FlinkGpu.open. Field offsets follow the C
 * struct's layout on LP64 (checked against the library's own layout by tests/test_jni_shim.py).
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;

/** Writes an fg_config into a direct buffer. */
public final class FgConfig {

    // fg_config field offsets (bytes)
    public static final int MODE = 0;
    public static final int WINDOW_KIND = 4;
    public static final int SIZE_MS = 8;
    public static final int SLIDE_MS = 16;
    public static final int OFFSET_MS = 24;
    public static final int SHIFT_TZ_OFFSET_MS = 32;
    public static final int VAL_TYPE = 40;
    public static final int NUM_AGGS = 44;
    public static final int AGGS = 48;
    public static final int MAX_PARALLELISM = 80;
    public static final int KEY_GROUP_START = 84;
    public static final int KEY_GROUP_END = 88;
    public static final int DEVICE_ID = 92;
    public static final int FLAGS = 96;
    public static final int EXPECTED_KEYS = 104;
    public static final int BUFFER_RECORDS = 112;
    public static final int TZ_TRANSITION_MS = 120;
    public static final int TZ_OFFSET_MS = 128;
    public static final int N_TZ_TRANSITIONS = 136;
    public static final int TZ_USE_DAYLIGHT = 140;
    public static final int ALLOWED_LATENESS_MS = 144;
    public static final int SIZE = 152;
    public static final int MAX_AGGS = 8;

    // enums of include/flinkgpu.h
    public static final int MODE_SQL = 0;
    public static final int MODE_DATASTREAM = 1;
    public static final int TUMBLE = 0;
    public static final int HOP = 1;
    public static final int CUMULATE = 2;
    public static final int VAL_NONE = 0;
    public static final int VAL_I64 = 1;
    public static final int VAL_F64 = 2;
    public static final int AGG_COUNT_STAR = 0;
    public static final int AGG_COUNT = 1;
    public static final int AGG_SUM = 2;
    public static final int AGG_AVG = 3;
    public static final int AGG_SUM0 = 4;
    public static final int AGG_MIN = 5;
    public static final int AGG_MAX = 6;
    public static final int FLAG_LOCAL_PARTIALS = 2;
    public static final int FLAG_PROCTIME = 4;
    public static final int FLAG_WINDOWED = 8;
    public static final int FLAG_PURGING_TRIGGER = 16;

    private FgConfig() {}

    /** The image of spec for the subtask owning key groups [kgStart, kgEnd]. */
    public static ByteBuffer of(
            GpuWindowAggSpec spec, int maxParallelism, int kgStart, int kgEnd, int nTransitions) {
        ByteBuffer b = ByteBuffer.allocateDirect(SIZE).order(ByteOrder.nativeOrder());
        b.putInt(MODE, spec.mode);
        b.putInt(WINDOW_KIND, spec.windowKind);
        b.putLong(SIZE_MS, spec.sizeMs);
        b.putLong(SLIDE_MS, spec.slideMs);
        b.putLong(OFFSET_MS, spec.offsetMs);
        b.putLong(SHIFT_TZ_OFFSET_MS, spec.shiftTzOffsetMs);
        b.putInt(VAL_TYPE, spec.valType);
        if (spec.aggs.length > MAX_AGGS) {
            throw new IllegalArgumentException("at most " + MAX_AGGS + " aggregates");
        }
        b.putInt(NUM_AGGS, spec.aggs.length);
        for (int i = 0; i < spec.aggs.length; i++) {
            b.putInt(AGGS + 4 * i, spec.aggs[i]);
        }
        b.putInt(MAX_PARALLELISM, maxParallelism);
        b.putInt(KEY_GROUP_START, kgStart);
        b.putInt(KEY_GROUP_END, kgEnd);
        b.putInt(DEVICE_ID, spec.device);
        b.putInt(FLAGS, spec.flags);
        b.putLong(EXPECTED_KEYS, spec.expectedKeys);
        b.putLong(BUFFER_RECORDS, spec.bufferRecords);
        b.putInt(N_TZ_TRANSITIONS, nTransitions);
        b.putInt(TZ_USE_DAYLIGHT, spec.tzUseDaylight ? 1 : 0);
        b.putLong(ALLOWED_LATENESS_MS, spec.allowedLatenessMs);
        return b;
    }
}
