/*
 * flink_gpu_jni.c -- JNI glue between the Java shim (java/, org.apache.flink...gpu.FlinkGpu)
 * and libflinkgpu.so (include/flinkgpu.h). Built by jni/Makefile when $JAVA_HOME is set; not
 * part of __graft_entry__.build() (this image has no JDK).
 *
 * Every native of FlinkGpu.java maps one-for-one onto a C-ABI entry point:
 *   open            fg_open              (WindowBuffer.Factory.create / SlicingWindowAggOperatorBuilder.build)
 *   addBatch        fg_add_batch         (SlicingWindowOperator.processElement, batched)
 *   addBatchNarrow  fg_add_batch         (the same with fg_batch.format: 4-byte key / rowtime / value columns)
 *   addRows         fg_add_rows          (packed BinaryRowData of a MemorySegment)
 *   addPartials     fg_add_partials      (GlobalAggCombiner.combine)
 *   advanceProgress fg_advance_progress  (processWatermark -> advanceProgress + fireWindow)
 *   advanceProgressAsync fg_advance_progress_async (the same, the fires queued: the watermark held)
 *   advanceProgressAsyncN fg_advance_progress_async_n (a batch's held watermarks in one call)
 *   collectFired    fg_collect_fired_to  (the held watermark's rows, in host memory; then the watermark is forwarded)
 *   flush           fg_flush             (prepareSnapshotPreBarrier)
 *   flushPartials   fg_flush_partials    (local phase: WindowBuffer.flush of LocalSlicingWindowAggOperator)
 *   snapshotState   fg_snapshot_state    (snapshotState: the window-aggs image)
 *   snapshotStateAsync / snapshotStateWait   fg_snapshot_state_async / _wait (the image exported
 *                   and its host copy queued; the shim clears the previous image meanwhile)
 *   restore         fg_restore           (initializeState)
 *   lateDropped     fg_late_dropped      (numLateRecordsDropped)
 *   close           fg_close
 *   dict*           fg_key_dict_*        (BinaryRowDataKeySelector rows of any key type)
 *   hostRegister    fg_host_register     (page-lock a managed-memory segment at open: direct DMA)
 *   hostUnregister  fg_host_unregister   (at close)
 *   snapshotSlices  fg_snapshot_slices   (the image's slices and which changed: the incremental keyed-state write)
 *   comm*           fg_comm_*            (the keyBy edge local -> global over RCCL: KeyGroupStreamPartitioner
 *                                         + RecordWriter + StatusWatermarkValve between co-located subtasks;
 *                                         commRoundBegin / Exchange / End: a round on the subtask's edge thread)
 *
 * Buffers: every ByteBuffer argument is a DIRECT buffer (MemorySegment.wrap of an off-heap
 * segment, MemorySegment.java:288,307, or ByteBuffer.allocateDirect) in native byte order;
 * its address is handed to the engine as FG_HOST memory, which fg_add_batch has finished
 * reading when it returns (the shim may refill the buffer at once). Output columns are
 * library-owned and wrapped with NewDirectByteBuffer: valid until the next call on the handle.
 *
 * Errors: a non-zero return code throws -- FG_EINVAL as IllegalArgumentException (the
 * reference's message, e.g. SliceAssigners' window-spec checks), FG_EFULL as EOFException
 * (RecordsWindowBuffer's "buffer full" signal), anything else as RuntimeException -- carrying
 * fg_last_error / fg_key_dict_last_error.
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flinkgpu.h"

static void throw_code(JNIEnv* env, int rc, const char* msg) {
    const char* cls = rc == FG_EINVAL ? "java/lang/IllegalArgumentException"
                    : rc == FG_EFULL  ? "java/io/EOFException"
                                      : "java/lang/RuntimeException";
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, msg ? msg : "libflinkgpu error");
}

static int check(JNIEnv* env, fg_handle* h, int rc) {
    if (rc != FG_OK) throw_code(env, rc, fg_last_error(h));
    return rc;
}

/* address of a direct buffer (NULL for a null reference); throws for a heap buffer */
static void* addr(JNIEnv* env, jobject buf) {
    if (!buf) return NULL;
    void* p = (*env)->GetDirectBufferAddress(env, buf);
    if (!p) throw_code(env, FG_EINVAL, "libflinkgpu takes direct ByteBuffers only");
    return p;
}

static jobject wrap(JNIEnv* env, const void* p, jlong bytes) {
    return (*env)->NewDirectByteBuffer(env, (void*)p, bytes > 0 ? bytes : 0);
}

#define FN(name) Java_org_apache_flink_table_runtime_operators_window_gpu_FlinkGpu_##name

/* long open(ByteBuffer config, long[] tzTransitions, long[] tzOffsets)
 * config: an fg_config image written by FgConfig.java (its pointer fields are ignored: the
 * zone rules come as the two arrays, copied by fg_open). */
JNIEXPORT jlong JNICALL FN(open)(JNIEnv* env, jclass cls, jobject config, jlongArray tzTrans, jlongArray tzOffs) {
    (void)cls;
    const fg_config* img = (const fg_config*)addr(env, config);
    if (!img) return 0;
    fg_config c = *img;
    jlong* tr = NULL;
    jlong* of = NULL;
    c.tz_transition_ms = NULL;
    c.tz_offset_ms = NULL;
    if (c.n_tz_transitions > 0) {
        if (!tzTrans || !tzOffs || (*env)->GetArrayLength(env, tzTrans) != c.n_tz_transitions ||
            (*env)->GetArrayLength(env, tzOffs) != c.n_tz_transitions + 1) {
            throw_code(env, FG_EINVAL, "zone rules need n_tz_transitions instants and n_tz_transitions + 1 offsets");
            return 0;
        }
        tr = (*env)->GetLongArrayElements(env, tzTrans, NULL);
        of = (*env)->GetLongArrayElements(env, tzOffs, NULL);
        c.tz_transition_ms = (const int64_t*)tr;
        c.tz_offset_ms = (const int64_t*)of;
    }
    fg_handle* h = NULL;
    int rc = fg_open(&c, &h);
    if (tr) (*env)->ReleaseLongArrayElements(env, tzTrans, tr, JNI_ABORT);
    if (of) (*env)->ReleaseLongArrayElements(env, tzOffs, of, JNI_ABORT);
    if (rc != FG_OK) {
        throw_code(env, rc, fg_last_error(NULL));
        return 0;
    }
    return (jlong)(intptr_t)h;
}

/* void addBatch(long h, ByteBuffer key, ByteBuffer rowtime, ByteBuffer val, ByteBuffer valNull, int n) */
JNIEXPORT void JNICALL FN(addBatch)(JNIEnv* env, jclass cls, jlong hp, jobject key, jobject rowtime, jobject val,
                                    jobject valNull, jint n) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    fg_batch b;
    memset(&b, 0, sizeof b);
    b.n = n;
    b.location = FG_HOST;
    b.key = (const int64_t*)addr(env, key);
    b.rowtime = (const int64_t*)addr(env, rowtime);
    b.val = addr(env, val);
    b.val_null = (const uint8_t*)addr(env, valNull);
    if ((*env)->ExceptionCheck(env)) return;
    check(env, h, fg_add_batch(h, &b));
}

/* void addBatchNarrow(long h, int format, ByteBuffer key, ByteBuffer rowtime, long rowtimeBase, ByteBuffer val,
 *                     ByteBuffer valNull, int n) -- fg_batch.format columns (int key, rowtime offsets from
 *                     rowtimeBase, int BIGINT values): fewer bytes per record over PCIe */
JNIEXPORT void JNICALL FN(addBatchNarrow)(JNIEnv* env, jclass cls, jlong hp, jint format, jobject key, jobject rowtime,
                                          jlong rowtimeBase, jobject val, jobject valNull, jint n) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    fg_batch b;
    memset(&b, 0, sizeof b);
    b.n = n;
    b.location = FG_HOST;
    b.format = format;
    b.key = (const int64_t*)addr(env, key);
    b.rowtime = (const int64_t*)addr(env, rowtime);
    b.rowtime_base = rowtimeBase;
    b.val = addr(env, val);
    b.val_null = (const uint8_t*)addr(env, valNull);
    if ((*env)->ExceptionCheck(env)) return;
    check(env, h, fg_add_batch(h, &b));
}

/* void addRows(long h, ByteBuffer rows, int n, int stride, int arity, int keyField, int rowtimeField, int valField)
 * rows: the fixed-length parts of n BinaryRowData (a MemorySegment of serialized records) */
JNIEXPORT void JNICALL FN(addRows)(JNIEnv* env, jclass cls, jlong hp, jobject rows, jint n, jint stride, jint arity,
                                   jint keyField, jint rowtimeField, jint valField) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    fg_row_batch b;
    memset(&b, 0, sizeof b);
    b.n = n;
    b.location = FG_HOST;
    b.stride = stride;
    b.rows = (const uint8_t*)addr(env, rows);
    b.arity = arity;
    b.key_field = keyField;
    b.rowtime_field = rowtimeField;
    b.val_field = valField;
    if ((*env)->ExceptionCheck(env)) return;
    check(env, h, fg_add_rows(h, &b));
}

/* void addPartials(long h, int n, ByteBuffer key, ByteBuffer sliceEnd, ByteBuffer cntStar,
 *                  ByteBuffer cntVal, ByteBuffer sum, ByteBuffer min, ByteBuffer max) */
JNIEXPORT void JNICALL FN(addPartials)(JNIEnv* env, jclass cls, jlong hp, jint n, jobject key, jobject sliceEnd,
                                       jobject cntStar, jobject cntVal, jobject sum, jobject min, jobject max) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    fg_partials p;
    memset(&p, 0, sizeof p);
    p.n = n;
    p.location = FG_HOST;
    p.key = (const int64_t*)addr(env, key);
    p.slice_end = (const int64_t*)addr(env, sliceEnd);
    p.cnt_star = (const int64_t*)addr(env, cntStar);
    p.cnt_val = (const int64_t*)addr(env, cntVal);
    p.sum = (const int64_t*)addr(env, sum);
    p.min = (const int64_t*)addr(env, min);
    p.max = (const int64_t*)addr(env, max);
    if ((*env)->ExceptionCheck(env)) return;
    check(env, h, fg_add_partials(h, &p));
}

/* the columns of fg_rows into cols (length >= 5 + num_aggs): key, window_start, window_end,
 * agg[0..num_aggs), null_mask, rowtime (DataStream; else null); returns the row count */
static jlong put_rows(JNIEnv* env, const fg_rows* r, jobjectArray cols, const char* who) {
    const jlong n = r->n, bytes = 8 * n;
    if ((*env)->GetArrayLength(env, cols) < 5 + r->num_aggs) {
        char msg[96];
        snprintf(msg, sizeof msg, "%s: column array too short", who);
        throw_code(env, FG_EINVAL, msg);
        return 0;
    }
    int i = 0;
    (*env)->SetObjectArrayElement(env, cols, i++, wrap(env, r->key, bytes));
    (*env)->SetObjectArrayElement(env, cols, i++, wrap(env, r->window_start, bytes));
    (*env)->SetObjectArrayElement(env, cols, i++, wrap(env, r->window_end, bytes));
    for (int a = 0; a < r->num_aggs; a++) (*env)->SetObjectArrayElement(env, cols, i++, wrap(env, r->agg[a], bytes));
    (*env)->SetObjectArrayElement(env, cols, i++, wrap(env, r->null_mask, n));
    (*env)->SetObjectArrayElement(env, cols, i++, r->rowtime ? wrap(env, r->rowtime, bytes) : NULL);
    return n;
}

/* long advanceProgress(long h, long watermark, ByteBuffer[] cols): the fired rows (put_rows) */
JNIEXPORT jlong JNICALL FN(advanceProgress)(JNIEnv* env, jclass cls, jlong hp, jlong wm, jobjectArray cols) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    fg_rows r;
    if (check(env, h, fg_advance_progress(h, wm, FG_HOST, &r))) return 0;
    return put_rows(env, &r, cols, "advanceProgress");
}

/* void advanceProgressAsync(long h, long watermark): the watermark's fires are queued; the shim
 * holds the watermark until collectFired has returned the rows of every async advance since the
 * last collect (rows before the watermark, as processWatermark emits them). */
JNIEXPORT void JNICALL FN(advanceProgressAsync)(JNIEnv* env, jclass cls, jlong hp, jlong wm) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    check(env, h, fg_advance_progress_async(h, wm));
}

/* void advanceProgressAsyncN(long h, long[] watermarks, int n): the watermarks a shim received
 * between two batches, in one call (fg_advance_progress_async_n) */
JNIEXPORT void JNICALL FN(advanceProgressAsyncN)(JNIEnv* env, jclass cls, jlong hp, jlongArray wms, jint n) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    if (n < 0 || !wms || (*env)->GetArrayLength(env, wms) < n) {
        throw_code(env, FG_EINVAL, "advanceProgressAsyncN: watermark array shorter than n");
        return;
    }
    jlong* w = (*env)->GetLongArrayElements(env, wms, NULL);
    const int rc = fg_advance_progress_async_n(h, (const int64_t*)w, n);
    (*env)->ReleaseLongArrayElements(env, wms, w, JNI_ABORT);
    check(env, h, rc);
}

/* long collectFired(long h, ByteBuffer[] cols): as advanceProgress -- the rows are copied to
 * library-owned host memory (fg_collect_fired_to FG_HOST), so the direct buffers the shim reads
 * with getLong are host memory, valid until the next call on the handle */
JNIEXPORT jlong JNICALL FN(collectFired)(JNIEnv* env, jclass cls, jlong hp, jobjectArray cols) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    fg_rows r;
    if (check(env, h, fg_collect_fired_to(h, FG_HOST, &r))) return 0;
    return put_rows(env, &r, cols, "collectFired");
}

/* void flush(long h) */
JNIEXPORT void JNICALL FN(flush)(JNIEnv* env, jclass cls, jlong hp) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    check(env, h, fg_flush(h));
}

/* long flushPartials(long h, ByteBuffer[] cols): a local-phase handle's partial rows of every
 * buffered slice, in host memory (LocalSlicingWindowAggOperator's WindowBuffer.flush) */
JNIEXPORT jlong JNICALL FN(flushPartials)(JNIEnv* env, jclass cls, jlong hp, jobjectArray cols) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    fg_rows r;
    if (check(env, h, fg_flush_partials(h, FG_HOST, &r))) return 0;
    return put_rows(env, &r, cols, "flushPartials");
}

/* long snapshotState(long h, ByteBuffer[] cols, long[] timerWatermark)
 * cols (length 7) receives key, slice_end, cnt_star, cnt_val, sum, min, max (min/max null for a
 * single-accumulator operator); timerWatermark[0] the timer service's watermark. Returns n. */
JNIEXPORT jlong JNICALL FN(snapshotState)(JNIEnv* env, jclass cls, jlong hp, jobjectArray cols, jlongArray timerWm) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    fg_state_rows s;
    int64_t wm = 0;
    if (check(env, h, fg_snapshot_state(h, &s, &wm))) return 0;
    const jlong bytes = 8 * s.n;
    const int64_t* c[7] = {s.key, s.slice_end, s.cnt_star, s.cnt_val, s.sum, s.min, s.max};
    for (int i = 0; i < 7; i++) (*env)->SetObjectArrayElement(env, cols, i, c[i] ? wrap(env, c[i], bytes) : NULL);
    jlong w = wm;
    (*env)->SetLongArrayRegion(env, timerWm, 0, 1, &w);
    return s.n;
}

/* void snapshotStateAsync(long h): fg_snapshot_state_async (ABI 15) */
JNIEXPORT void JNICALL FN(snapshotStateAsync)(JNIEnv* env, jclass cls, jlong hp) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    (void)check(env, h, fg_snapshot_state_async(h));
}

/* long snapshotStateWait(long h, ByteBuffer[] cols, long[] timerWatermark): the image of the last
 * snapshotStateAsync, as snapshotState returns it (fg_snapshot_state_wait) */
JNIEXPORT jlong JNICALL FN(snapshotStateWait)(JNIEnv* env, jclass cls, jlong hp, jobjectArray cols, jlongArray timerWm) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    fg_state_rows s;
    int64_t wm = 0;
    if (check(env, h, fg_snapshot_state_wait(h, &s, &wm))) return 0;
    const jlong bytes = 8 * s.n;
    const int64_t* c[7] = {s.key, s.slice_end, s.cnt_star, s.cnt_val, s.sum, s.min, s.max};
    for (int i = 0; i < 7; i++) (*env)->SetObjectArrayElement(env, cols, i, c[i] ? wrap(env, c[i], bytes) : NULL);
    jlong w = wm;
    (*env)->SetLongArrayRegion(env, timerWm, 0, 1, &w);
    return s.n;
}

/* long[] snapshotSlices(long h): the slices of the image the last snapshotState / snapshotStateWait
 * returned (fg_snapshot_slices, ABI 16) as one array: [n, slice_end[n], first_row[n], rows[n],
 * changed[n] (1 / 0)] -- the shim rewrites only the changed slices' keyed state */
JNIEXPORT jlongArray JNICALL FN(snapshotSlices)(JNIEnv* env, jclass cls, jlong hp) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    fg_image_slices s;
    if (check(env, h, fg_snapshot_slices(h, &s))) return NULL;
    const jsize n = (jsize)s.n;
    jlongArray out = (*env)->NewLongArray(env, 1 + 4 * n);
    if (!out) return NULL;
    jlong* buf = (jlong*)malloc(sizeof(jlong) * (size_t)(1 + 4 * n));
    if (!buf) {
        throw_code(env, FG_EDEVICE, "snapshotSlices: out of host memory");
        return NULL;
    }
    buf[0] = n;
    for (jsize i = 0; i < n; i++) {
        buf[1 + i] = s.slice_end[i];
        buf[1 + n + i] = s.first_row[i];
        buf[1 + 2 * n + i] = s.rows[i];
        buf[1 + 3 * n + i] = s.changed[i] ? 1 : 0;
    }
    (*env)->SetLongArrayRegion(env, out, 0, 1 + 4 * n, buf);
    free(buf);
    return out;
}

/* void restore(long h, int n, ByteBuffer key, ByteBuffer sliceEnd, ByteBuffer cntStar, ByteBuffer cntVal,
 *              ByteBuffer sum, ByteBuffer min, ByteBuffer max, long timerWatermark) */
JNIEXPORT void JNICALL FN(restore)(JNIEnv* env, jclass cls, jlong hp, jint n, jobject key, jobject sliceEnd,
                                   jobject cntStar, jobject cntVal, jobject sum, jobject min, jobject max,
                                   jlong timerWm) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    fg_state_rows s;
    memset(&s, 0, sizeof s);
    s.n = n;
    s.key = (const int64_t*)addr(env, key);
    s.slice_end = (const int64_t*)addr(env, sliceEnd);
    s.cnt_star = (const int64_t*)addr(env, cntStar);
    s.cnt_val = (const int64_t*)addr(env, cntVal);
    s.sum = (const int64_t*)addr(env, sum);
    s.min = (const int64_t*)addr(env, min);
    s.max = (const int64_t*)addr(env, max);
    if ((*env)->ExceptionCheck(env)) return;
    check(env, h, fg_restore(h, &s, timerWm));
}

/* long lateDropped(long h) */
JNIEXPORT jlong JNICALL FN(lateDropped)(JNIEnv* env, jclass cls, jlong hp) {
    (void)cls;
    fg_handle* h = (fg_handle*)(intptr_t)hp;
    int64_t v = 0;
    check(env, h, fg_late_dropped(h, &v));
    return v;
}

/* void close(long h) */
JNIEXPORT void JNICALL FN(close)(JNIEnv* env, jclass cls, jlong hp) {
    (void)env;
    (void)cls;
    fg_close((fg_handle*)(intptr_t)hp);
}

/* ---- key dictionary (keys of any type) ------------------------------------------------------ */

static int dcheck(JNIEnv* env, fg_key_dict* d, int rc) {
    if (rc != FG_OK) throw_code(env, rc, d ? fg_key_dict_last_error(d) : "fg_key_dict_open failed");
    return rc;
}

/* long dictOpen(int device, int maxParallelism, long expectedKeys) */
JNIEXPORT jlong JNICALL FN(dictOpen)(JNIEnv* env, jclass cls, jint device, jint maxP, jlong expected) {
    (void)cls;
    fg_key_dict* d = NULL;
    if (dcheck(env, NULL, fg_key_dict_open(device, maxP, expected, &d))) return 0;
    return (jlong)(intptr_t)d;
}

/* void dictIntern(long d, ByteBuffer rows, long nbytes, ByteBuffer offsets, ByteBuffer lengths, int n,
 *                 ByteBuffer outIds, ByteBuffer outKeyGroups) -- outKeyGroups may be null */
JNIEXPORT void JNICALL FN(dictIntern)(JNIEnv* env, jclass cls, jlong dp, jobject rows, jlong nbytes, jobject offsets,
                                      jobject lengths, jint n, jobject outIds, jobject outKg) {
    (void)cls;
    fg_key_dict* d = (fg_key_dict*)(intptr_t)dp;
    const uint8_t* r = (const uint8_t*)addr(env, rows);
    const int64_t* o = (const int64_t*)addr(env, offsets);
    const int32_t* l = (const int32_t*)addr(env, lengths);
    int64_t* ids = (int64_t*)addr(env, outIds);
    int32_t* kg = (int32_t*)addr(env, outKg);
    if ((*env)->ExceptionCheck(env)) return;
    dcheck(env, d, fg_key_dict_intern(d, FG_HOST, n, r, nbytes, o, l, ids, kg));
}

/* void dictLookup(long d, ByteBuffer ids, int n, ByteBuffer outOffsets, ByteBuffer outLengths) */
JNIEXPORT void JNICALL FN(dictLookup)(JNIEnv* env, jclass cls, jlong dp, jobject ids, jint n, jobject outOffsets,
                                      jobject outLengths) {
    (void)cls;
    fg_key_dict* d = (fg_key_dict*)(intptr_t)dp;
    const int64_t* i = (const int64_t*)addr(env, ids);
    int64_t* o = (int64_t*)addr(env, outOffsets);
    int32_t* l = (int32_t*)addr(env, outLengths);
    if ((*env)->ExceptionCheck(env)) return;
    dcheck(env, d, fg_key_dict_lookup(d, FG_HOST, n, i, o, l));
}

/* void dictCopyArena(long d, long begin, long nbytes, ByteBuffer out) */
JNIEXPORT void JNICALL FN(dictCopyArena)(JNIEnv* env, jclass cls, jlong dp, jlong begin, jlong nbytes, jobject out) {
    (void)cls;
    fg_key_dict* d = (fg_key_dict*)(intptr_t)dp;
    uint8_t* o = (uint8_t*)addr(env, out);
    if ((*env)->ExceptionCheck(env)) return;
    dcheck(env, d, fg_key_dict_copy_arena(d, begin, nbytes, o));
}

/* void dictClose(long d) */
JNIEXPORT void JNICALL FN(dictClose)(JNIEnv* env, jclass cls, jlong dp) {
    (void)env;
    (void)cls;
    fg_key_dict_close((fg_key_dict*)(intptr_t)dp);
}

/* ---- page-locked managed memory --------------------------------------------------------------- */

/* void hostRegister(int device, ByteBuffer segment): the whole direct buffer (an off-heap
 * MemorySegment wrapped whole, MemorySegment.wrap :307) is page-locked for direct DMA */
JNIEXPORT void JNICALL FN(hostRegister)(JNIEnv* env, jclass cls, jint device, jobject segment) {
    (void)cls;
    void* p = addr(env, segment);
    if ((*env)->ExceptionCheck(env)) return;
    const jlong bytes = (*env)->GetDirectBufferCapacity(env, segment);
    check(env, NULL, fg_host_register(device, p, bytes));
}

/* void hostUnregister(int device, ByteBuffer segment) */
JNIEXPORT void JNICALL FN(hostUnregister)(JNIEnv* env, jclass cls, jint device, jobject segment) {
    (void)cls;
    void* p = addr(env, segment);
    if ((*env)->ExceptionCheck(env)) return;
    check(env, NULL, fg_host_unregister(device, p));
}

/* ---- the keyBy edge over RCCL (fg_comm) ----------------------------------------------------------- */

static int ccheck(JNIEnv* env, fg_comm* c, int rc) {
    if (rc != FG_OK) throw_code(env, rc, fg_comm_last_error(c));
    return rc;
}

/* void commUniqueId(ByteBuffer id): FG_COMM_ID_BYTES bytes of a new RCCL unique id (the
 * coordinator makes it once and ships it with the deployment) */
JNIEXPORT void JNICALL FN(commUniqueId)(JNIEnv* env, jclass cls, jobject id) {
    (void)cls;
    uint8_t* p = (uint8_t*)addr(env, id);
    if ((*env)->ExceptionCheck(env)) return;
    if ((*env)->GetDirectBufferCapacity(env, id) < FG_COMM_ID_BYTES) {
        throw_code(env, FG_EINVAL, "commUniqueId: the id buffer holds FG_COMM_ID_BYTES bytes");
        return;
    }
    ccheck(env, NULL, fg_comm_unique_id(p));
}

/* long commOpen(int device, int world, int rank, ByteBuffer id): blocks until every rank joined */
JNIEXPORT jlong JNICALL FN(commOpen)(JNIEnv* env, jclass cls, jint device, jint world, jint rank, jobject id) {
    (void)cls;
    const uint8_t* p = (const uint8_t*)addr(env, id);
    if ((*env)->ExceptionCheck(env)) return 0;
    if ((*env)->GetDirectBufferCapacity(env, id) < FG_COMM_ID_BYTES) {
        throw_code(env, FG_EINVAL, "commOpen: the id buffer holds FG_COMM_ID_BYTES bytes");
        return 0;
    }
    fg_comm* c = NULL;
    if (ccheck(env, NULL, fg_comm_open(device, world, rank, p, &c))) return 0;
    return (jlong)(intptr_t)c;
}

/* long commExchangeFired(long comm, long local, int keyHash, int maxParallelism, long watermark,
 * long global): the local handle's collected async fires exchanged by key-group owner and merged
 * into `global`; returns the combined watermark (min over the ranks) to advance `global` to */
JNIEXPORT jlong JNICALL FN(commExchangeFired)(JNIEnv* env, jclass cls, jlong cp, jlong lp, jint keyHash,
                                              jint maxPar, jlong wm, jlong gp) {
    (void)cls;
    int64_t mw = 0;
    fg_comm* c = (fg_comm*)(intptr_t)cp;
    if (ccheck(env, c, fg_comm_exchange_fired(c, (fg_handle*)(intptr_t)lp, keyHash, maxPar, wm,
                                              (fg_handle*)(intptr_t)gp, &mw)))
        return 0;
    return mw;
}

/* long commExchangeFlushed(long comm, long local, int keyHash, int maxParallelism, long watermark,
 * long global): the same for the local buffer's flush before a checkpoint barrier */
JNIEXPORT jlong JNICALL FN(commExchangeFlushed)(JNIEnv* env, jclass cls, jlong cp, jlong lp, jint keyHash,
                                                jint maxPar, jlong wm, jlong gp) {
    (void)cls;
    int64_t mw = 0;
    fg_comm* c = (fg_comm*)(intptr_t)cp;
    if (ccheck(env, c, fg_comm_exchange_flushed(c, (fg_handle*)(intptr_t)lp, keyHash, maxPar, wm,
                                                (fg_handle*)(intptr_t)gp, &mw)))
        return 0;
    return mw;
}

/* void commRoundBegin(long comm, long local, int mode, int keyHash, int maxParallelism, long watermark,
 * long epoch): fg_comm_round_begin -- the local rows collected (ROUND_FIRED) or flushed
 * (ROUND_FLUSHED) and grouped by owner, or nothing (ROUND_IDLE, local may be 0). Whatever it throws,
 * the caller calls commRoundExchange next (a failed begin still takes part in the round). */
JNIEXPORT void JNICALL FN(commRoundBegin)(JNIEnv* env, jclass cls, jlong cp, jlong lp, jint mode, jint keyHash,
                                          jint maxPar, jlong wm, jlong epoch) {
    (void)cls;
    fg_comm* c = (fg_comm*)(intptr_t)cp;
    (void)ccheck(env, c, fg_comm_round_begin(c, (fg_handle*)(intptr_t)lp, mode, keyHash, maxPar, wm, epoch));
}

/* void commRoundExchange(long comm, long[] out): fg_comm_round_exchange (blocks for the peers; touches
 * no operator); out[0..4] = min watermark, min epoch, rows sent, rows received, bytes sent */
JNIEXPORT void JNICALL FN(commRoundExchange)(JNIEnv* env, jclass cls, jlong cp, jlongArray out) {
    (void)cls;
    fg_comm* c = (fg_comm*)(intptr_t)cp;
    fg_round r;
    memset(&r, 0, sizeof r);
    if (ccheck(env, c, fg_comm_round_exchange(c, &r))) return;
    jlong v[5] = {r.min_watermark, r.min_epoch, r.rows_sent, r.rows_received, r.bytes_sent};
    (*env)->SetLongArrayRegion(env, out, 0, 5, v);
}

/* void commRoundEnd(long comm, long global): fg_comm_round_end -- the received rows merged into global */
JNIEXPORT void JNICALL FN(commRoundEnd)(JNIEnv* env, jclass cls, jlong cp, jlong gp) {
    (void)cls;
    fg_comm* c = (fg_comm*)(intptr_t)cp;
    (void)ccheck(env, c, fg_comm_round_end(c, (fg_handle*)(intptr_t)gp));
}

/* long commBytesSent(long comm) */
JNIEXPORT jlong JNICALL FN(commBytesSent)(JNIEnv* env, jclass cls, jlong cp) {
    (void)env;
    (void)cls;
    return fg_comm_bytes_sent((fg_comm*)(intptr_t)cp);
}

/* void commClose(long comm) */
JNIEXPORT void JNICALL FN(commClose)(JNIEnv* env, jclass cls, jlong cp) {
    (void)env;
    (void)cls;
    fg_comm_close((fg_comm*)(intptr_t)cp);
}
