/*
 * Natives of libflinkgpu_jni.so (jni/flink_gpu_jni.c), one per C-ABI entry point of
 * include/flinkgpu.h. Every ByteBuffer is a direct buffer in native byte order (a wrapped
 * off-heap MemorySegment, MemorySegment.java:288,307, or ByteBuffer.allocateDirect).
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import java.nio.ByteBuffer;

/** JNI entry points of the MI355X window-aggregation engine. */
public final class FlinkGpu {

    static {
        System.loadLibrary("flinkgpu_jni");
    }

    private FlinkGpu() {}

    /** fg_open: config is an fg_config image (FgConfig); zone rules as arrays (may be null). */
    public static native long open(ByteBuffer config, long[] tzTransitions, long[] tzOffsets);

    /** fg_add_batch (FG_HOST): the buffers may be refilled as soon as the call returns. */
    public static native void addBatch(
            long h, ByteBuffer key, ByteBuffer rowtime, ByteBuffer val, ByteBuffer valNull, int n);

    /**
     * fg_add_batch with fg_batch.format: FORMAT_KEY32 (int keys), FORMAT_ROWTIME32 (rowtime as
     * unsigned int offsets from rowtimeBase), FORMAT_VAL32 (int BIGINT values) -- 16 instead of
     * 24 bytes per record over PCIe for a DOUBLE value.
     */
    public static native void addBatchNarrow(
            long h,
            int format,
            ByteBuffer key,
            ByteBuffer rowtime,
            long rowtimeBase,
            ByteBuffer val,
            ByteBuffer valNull,
            int n);

    public static final int FORMAT_KEY32 = 1;
    public static final int FORMAT_ROWTIME32 = 2;
    public static final int FORMAT_VAL32 = 4;

    /** fg_add_rows: n packed BinaryRowData fixed-length parts, stride bytes apart. */
    public static native void addRows(
            long h,
            ByteBuffer rows,
            int n,
            int stride,
            int arity,
            int keyField,
            int rowtimeField,
            int valField);

    /** fg_add_partials (GlobalAggCombiner.combine); min / max null unless several accumulators. */
    public static native void addPartials(
            long h,
            int n,
            ByteBuffer key,
            ByteBuffer sliceEnd,
            ByteBuffer cntStar,
            ByteBuffer cntVal,
            ByteBuffer sum,
            ByteBuffer min,
            ByteBuffer max);

    /**
     * fg_advance_progress: fills cols with key, window_start, window_end, agg[0..numAggs),
     * null_mask, rowtime (library-owned, valid until the next call); returns the row count.
     */
    public static native long advanceProgress(long h, long watermark, ByteBuffer[] cols);

    /**
     * fg_advance_progress_async: the watermark's fires are queued and the call returns at once; the
     * caller holds the watermark until {@link #collectFired} has returned the fired rows.
     */
    public static native void advanceProgressAsync(long h, long watermark);

    /** fg_advance_progress_async_n: watermarks[0..n) in order, as n advanceProgressAsync calls. */
    public static native void advanceProgressAsyncN(long h, long[] watermarks, int n);

    /**
     * fg_collect_fired_to(FG_HOST): waits for the fires of every async advance since the last
     * collect; fills cols as {@link #advanceProgress} (host memory); returns the row count.
     */
    public static native long collectFired(long h, ByteBuffer[] cols);

    /** fg_flush (prepareSnapshotPreBarrier). */
    public static native void flush(long h);

    /**
     * fg_flush_partials (FG_FLAG_LOCAL_PARTIALS handles): every buffered slice's partial rows, in
     * host memory; cols (length >= 10) as {@link #advanceProgress}; returns the row count.
     */
    public static native long flushPartials(long h, ByteBuffer[] cols);

    /**
     * fg_snapshot_state: cols (length 7) receives key, slice_end, cnt_star, cnt_val, sum, min, max;
     * timerWatermark[0] the timer watermark; returns the entry count.
     */
    public static native long snapshotState(long h, ByteBuffer[] cols, long[] timerWatermark);

    /**
     * fg_snapshot_state_async (ABI 15): the staged records flushed, the resident state exported on
     * the GPU and its copy into the host image queued; the handle takes further calls meanwhile.
     */
    public static native void snapshotStateAsync(long h);

    /** fg_snapshot_state_wait: the image of the last snapshotStateAsync, as snapshotState. */
    public static native long snapshotStateWait(long h, ByteBuffer[] cols, long[] timerWatermark);

    /**
     * fg_snapshot_slices (ABI 16): the slices of the image the last snapshotState / snapshotStateWait
     * returned, as [n, sliceEnd[n], firstRow[n], rows[n], changed[n] (1 / 0)].
     */
    public static native long[] snapshotSlices(long h);

    /** fg_restore. */
    public static native void restore(
            long h,
            int n,
            ByteBuffer key,
            ByteBuffer sliceEnd,
            ByteBuffer cntStar,
            ByteBuffer cntVal,
            ByteBuffer sum,
            ByteBuffer min,
            ByteBuffer max,
            long timerWatermark);

    /** fg_late_dropped (numLateRecordsDropped). */
    public static native long lateDropped(long h);

    /** fg_close. */
    public static native void close(long h);

    /** fg_key_dict_open. */
    public static native long dictOpen(int device, int maxParallelism, long expectedKeys);

    /** fg_key_dict_intern (FG_HOST); outKeyGroups may be null. */
    public static native void dictIntern(
            long d,
            ByteBuffer rows,
            long nbytes,
            ByteBuffer offsets,
            ByteBuffer lengths,
            int n,
            ByteBuffer outIds,
            ByteBuffer outKeyGroups);

    /** fg_key_dict_lookup (FG_HOST). */
    public static native void dictLookup(
            long d, ByteBuffer ids, int n, ByteBuffer outOffsets, ByteBuffer outLengths);

    /** fg_key_dict_copy_arena. */
    public static native void dictCopyArena(long d, long begin, long nbytes, ByteBuffer out);

    /** fg_key_dict_close. */
    public static native void dictClose(long d);

    /**
     * fg_host_register: page-lock a whole direct buffer (an off-heap managed-memory segment,
     * MemorySegment.wrap) once, so batches handed from it are DMA'd without staging.
     */
    public static native void hostRegister(int device, ByteBuffer segment);

    /** fg_host_unregister (at close, before the segment is released to the MemoryManager). */
    public static native void hostUnregister(int device, ByteBuffer segment);

    // ---- the keyBy edge local -> global over RCCL (fg_comm; INTEGRATION.md section 7) ----

    /** fg_key_hash: a BIGINT key hashed as its BinaryRowData key row (FG_KEYHASH_BINARYROW_BIGINT). */
    public static final int KEYHASH_BINARYROW_BIGINT = 0;

    /** Bytes of a communicator id (FG_COMM_ID_BYTES). */
    public static final int COMM_ID_BYTES = 128;

    /** fg_comm_unique_id: a new id into a direct buffer of COMM_ID_BYTES (the coordinator's). */
    public static native void commUniqueId(ByteBuffer id);

    /** fg_comm_open: this subtask's communicator (blocks until all `world` ranks joined). */
    public static native long commOpen(int device, int world, int rank, ByteBuffer id);

    /**
     * fg_comm_exchange_fired: the local handle's collected fires exchanged by key-group owner and
     * merged into the global handle; returns the combined watermark to advance the global to.
     */
    public static native long commExchangeFired(
            long comm, long local, int keyHash, int maxParallelism, long watermark, long global);

    /** fg_comm_exchange_flushed: the same for the local flush before a checkpoint barrier. */
    public static native long commExchangeFlushed(
            long comm, long local, int keyHash, int maxParallelism, long watermark, long global);

    /** fg_comm_round_begin modes (FG_ROUND_*). */
    public static final int ROUND_FIRED = 0;

    public static final int ROUND_FLUSHED = 1;
    public static final int ROUND_IDLE = 2;

    /**
     * fg_comm_round_begin (ABI 16): the local rows of the round grouped by owner (the operators are
     * touched here and in {@link #commRoundEnd}, never while {@link #commRoundExchange} waits). A
     * failed begin still takes part: call commRoundExchange after it whatever it threw.
     */
    public static native void commRoundBegin(
            long comm, long local, int mode, int keyHash, int maxParallelism, long watermark, long epoch);

    /**
     * fg_comm_round_exchange: the round's collectives; out[0..4] = min watermark, min epoch, rows
     * sent, rows received, bytes sent. Throws on every rank when one rank's round failed.
     */
    public static native void commRoundExchange(long comm, long[] out);

    /** fg_comm_round_end: the received partial rows merged into the global handle. */
    public static native void commRoundEnd(long comm, long global);

    /** fg_comm_bytes_sent. */
    public static native long commBytesSent(long comm);

    /** fg_comm_close. */
    public static native void commClose(long comm);
}
