/*
 * flinkgpu.h -- C-ABI of the MI355X keyed window-aggregation engine (libflinkgpu.so).
 *
 * Drop-in boundary for Flink's window aggregation hot path.  A JNI / Panama stub on
 * the Java side binds these entry points one-for-one to the reference
 * SPI methods they replace:
 *
 *   reference (Java)                                                   C-ABI
 *   ---------------------------------------------------------------   ----------------------
 *   WindowBuffer.Factory.create(...)                                    fg_open
 *     TR/operators/aggregate/window/buffers/WindowBuffer.java:105-118
 *     + SlicingWindowAggOperatorBuilder.build  .../SlicingWindowAggOperatorBuilder.java:127-170
 *   SlicingWindowOperator.processElement -> WindowProcessor.processElement
 *     TR/operators/window/slicing/SlicingWindowOperator.java:196-204     fg_add_batch
 *     (packed BinaryRowData rows, TC/data/binary/BinaryRowData.java:68-76) fg_add_rows
 *     TR/operators/aggregate/window/processors/AbstractWindowAggProcessor.java:135-165
 *     (+ RecordsWindowBuffer.addElement  .../buffers/RecordsWindowBuffer.java:81-97)
 *   SlicingWindowOperator.processWatermark + onEventTime/onTimer
 *     SlicingWindowOperator.java:207-237                                  fg_advance_progress
 *     AbstractWindowAggProcessor.advanceProgress :178-192, fireWindow/clearWindow
 *     (SliceUnsharedWindowAggProcessor.java:46-54, SliceSharedWindowAggProcessor.java:64-118)
 *   SlicingWindowOperator.prepareSnapshotPreBarrier :240-242           fg_flush
 *     -> AbstractWindowAggProcessor.prepareCheckpoint :195-197 -> RecordsWindowBuffer.flush :108-119
 *   StreamOperatorStateHandler.snapshotState (window-aggs state + timers)   fg_snapshot_state
 *     SJ/api/operators/StreamOperatorStateHandler.java:185-241
 *   AbstractStreamOperator.initializeState (keyed state restore)         fg_restore
 *   SlicingWindowOperator.getNumLateRecordsDropped :300-303            fg_late_dropped
 *   two-phase: LocalAggCombiner.combine (local operator output)        fg_config.flags |= FG_FLAG_LOCAL_PARTIALS
 *     GlobalAggCombiner.combine  .../combines/GlobalAggCombiner.java:77-110  fg_add_partials
 *   WindowBuffer.close / SlicingWindowOperator.close :178-183           fg_close
 *   DataStream WindowOperator.processElement / processWatermark / onEventTime
 *     SJ/runtime/operators/windowing/WindowOperator.java:300-503          same entry points,
 *                                                                        fg_config.mode = FG_MODE_DATASTREAM
 *   KeyGroupRangeAssignment.assignToKeyGroup  RT/state/KeyGroupRangeAssignment.java:63-77
 *     + KeyGroupStreamPartitioner.selectChannel SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:55-65
 *                                                                        fg_key_groups
 *   BinaryRowDataKeySelector.getKey (any key type: STRING, several columns)
 *     TR/keyselector/BinaryRowDataKeySelector.java:43-50, key identity BinarySection.equals /
 *     hashCode TC/data/binary/BinarySection.java:62-78                   fg_key_dict_intern
 *
 * Conventions
 *  - Return 0 (FG_OK) on success, a positive FG_E* code otherwise; fg_last_error()
 *    holds the message (for FG_EINVAL: the reference's IllegalArgumentException text).
 *  - FG_EFULL mirrors the EOFException "buffer full, flush and retry" signal of
 *    RecordsWindowBuffer (:91-96); the engine handles it internally, it is returned only
 *    if a single batch exceeds the configured buffer capacity.
 *  - Input buffers are owned by the caller and must stay valid for the call only.
 *    Output buffers (fg_rows, fg_state_rows) are owned by the library and stay valid
 *    until the next call on the same handle.
 *  - A handle is single-threaded (Flink's mailbox model, MailboxProcessor.java:44-48);
 *    distinct handles are independent and may be used from different threads.
 *  - Times are epoch milliseconds (Java long). All integer arithmetic wraps like Java.
 */
#ifndef FLINKGPU_H
#define FLINKGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FG_ABI_VERSION 16

enum fg_status {
    FG_OK = 0,
    FG_EINVAL = 1,     /* invalid argument / window spec (IllegalArgumentException) */
    FG_EFULL = 2,      /* batch larger than the configured buffer (EOFException analogue) */
    FG_EDEVICE = 3,    /* HIP runtime error or no usable MI355X device */
    FG_ECAPACITY = 4,  /* more distinct keys in one slice than 2^13 state regions hold (~29M):
                        * raise the parallelism. Below that a region that overflows splits
                        * (BytesMap growth, BytesMap.java:229-290) and the call succeeds. */
    FG_ESTATE = 5      /* API used out of order */
};

enum fg_mode { FG_MODE_SQL = 0, FG_MODE_DATASTREAM = 1 };
enum fg_window_kind { FG_TUMBLE = 0, FG_HOP = 1, FG_CUMULATE = 2 };   /* DataStream: TUMBLE, HOP=sliding */
enum fg_val_type { FG_VAL_NONE = 0, FG_VAL_I64 = 1, FG_VAL_F64 = 2 };
/* Aggregates over the single value column (SumAggFunction, Count1AggFunction,
 * CountAggFunction, AvgAggFunction, Sum0AggFunction of TP/functions/aggfunctions/).
 * SUM0 (Sum0AggFunction.java:60-63,75-76,97-98,136-137,162-163): 0-initialised, never NULL;
 * its value is the AVG accumulator's sum. */
/* MIN / MAX (MinAggFunction.java:56-90, MaxAggFunction.java:56-96, TP/functions/aggfunctions/):
 * NULL-initialised; a non-null operand replaces the accumulator iff operand < min (> max),
 * Java primitive comparison; NULL when the window holds no non-null value. An aggregate list
 * may mix SUM / AVG / SUM0, MIN and MAX over the value column: the operator then keeps all three
 * value accumulators per (key, slice), as the reference's generated accumulator row does
 * (AggsHandlerCodeGenerator.scala:578-700), staging each record once; the two-phase operators'
 * partial rows then carry the three value accumulators too (FG_FLAG_LOCAL_PARTIALS, fg_partials). */
enum fg_agg { FG_AGG_COUNT_STAR = 0, FG_AGG_COUNT = 1, FG_AGG_SUM = 2, FG_AGG_AVG = 3, FG_AGG_SUM0 = 4,
              FG_AGG_MIN = 5, FG_AGG_MAX = 6 };
/* FG_DEVICE columns are read on the handle's stream (fg_stream): the caller orders their
 * producer before it (complete, or an event the stream waits on). fg_add_partials and
 * fg_add_rows have read them when they return; fg_add_batch's columns stay in use until the
 * work queued on the handle's stream by the NEXT call on the handle has completed (the engine
 * finishes a batch's staging in that call, so that its two partition passes run back to back
 * on the GPU): a caller that frees or reuses them orders that after the handle's stream (an
 * event recorded on fg_stream after the next call, or fg_synchronize, which releases them).
 * FG_HOST buffers (pageable or pinned) have been read completely when the call returns: the
 * caller may overwrite them at once (the H2D copy is complete; the batch's kernels may still
 * be running on the handle's stream). */
enum fg_location { FG_HOST = 0, FG_DEVICE = 1 };
/* FG_KEYHASH_DICT_ID: the key is an id of an fg_key_dict (any key type); its key group, computed
 * from the key row's bytes when it was interned, is carried in the id's low ceil(log2(max_parallelism))
 * bits. */
enum fg_key_hash { FG_KEYHASH_BINARYROW_BIGINT = 0, FG_KEYHASH_JAVA_LONG = 1, FG_KEYHASH_DICT_ID = 2 };
enum fg_flags {
    FG_FLAG_KERNEL_TIMING = 1,    /* HIP-event timing of every launch (fg_kernel_stats) */
    /* Local phase of the two-phase window aggregation (LocalSlicingWindowAggOperator +
     * LocalAggCombiner, TR/operators/aggregate/window/LocalSlicingWindowAggOperator.java:113-139,
     * combines/LocalAggCombiner.java:69-106): records are assigned to their own slice with no
     * late handling, and fg_advance_progress emits, for every slice the watermark fires, one
     * partial accumulator row per key instead of window rows: window_start/window_end = the
     * slice, agg[0] = COUNT(*), agg[1] = COUNT(v), agg[2] = SUM bits (0 when COUNT(v) = 0).
     * fg_config.aggs is ignored (the global operator's list applies), except that a MIN or
     * MAX in it makes agg[2] the partial MIN / MAX instead of the SUM; a list mixing the SUM
     * family, MIN and MAX makes the partial row carry all three value accumulators: agg[2] =
     * SUM, agg[3] = MIN, agg[4] = MAX (fg_partials.min / max of the global operator). */
    FG_FLAG_LOCAL_PARTIALS = 2,
    /* SQL processing-time windows (SliceAssigner.isEventTime() == false,
     * AbstractWindowAggProcessor.java:137-140): `rowtime` carries each record's processing
     * time, nothing is late, fg_advance_progress takes the current processing time. Records
     * are expected at or after the last progress (as processing time is). */
    FG_FLAG_PROCTIME = 4,
    /* Input rows already carry their window (SliceAssigners.windowed / WindowedSliceAssigner,
     * TR/operators/window/slicing/SliceAssigners.java:386-435, after a window TVF): `rowtime`
     * carries each row's window_end; every window is its own slice (unshared, fired and
     * expired alone, a late row is dropped once its window fired); window_start =
     * the kind's getWindowStart(window_end). The window kind/size/slide/offset describe the
     * inner assigner. window_end values must lie on the inner assigner's slice grid (as a
     * window TVF emits them), else fg_add_batch fails with FG_EINVAL. SQL event time only,
     * not the local phase. With zone rules the window_end values are local (UTC-shifted)
     * times and are taken as is. */
    FG_FLAG_WINDOWED = 8,
    /* DataStream: PurgingTrigger.of(EventTimeTrigger) -- a firing window's state is cleared
     * (FIRE_AND_PURGE), so an element of a fired, not yet cleaned window (allowed lateness)
     * fires it with itself alone (WindowOperatorTest.testLateness :1805-1886). */
    FG_FLAG_PURGING_TRIGGER = 16
};

#define FG_MAX_AGGS 8

typedef struct fg_config {
    int32_t mode;                 /* fg_mode */
    int32_t window_kind;          /* fg_window_kind */
    int64_t size_ms;              /* TUMBLE size / HOP size / CUMULATE max size */
    int64_t slide_ms;             /* HOP slide / CUMULATE step; ignored for TUMBLE */
    int64_t offset_ms;            /* window offset */
    int64_t shift_tz_offset_ms;   /* fixed-offset shift time zone (TIMESTAMP_LTZ); 0 = UTC */
    int32_t val_type;             /* fg_val_type of the aggregated column */
    int32_t num_aggs;             /* output aggregate columns, in order */
    int32_t aggs[FG_MAX_AGGS];    /* fg_agg */
    int32_t max_parallelism;      /* number of key groups (KeyGroupRangeAssignment) */
    int32_t key_group_start;      /* key-group range owned by this subtask (inclusive) */
    int32_t key_group_end;
    int32_t device_id;            /* HIP device ordinal */
    int32_t flags;                /* FG_FLAG_* */
    int64_t expected_keys;        /* distinct keys per slice on this subtask: sizes the state regions
                                   * (speed, not correctness: regions split on overflow, up to 2^13);
                                   * <= 0: unknown, 2^10 regions (117 MB per slice table), grown on demand */
    int64_t buffer_records;       /* staged records before an implicit flush (managed-memory analogue) */
    /* Shift time zone with transitions (daylight saving): the ZoneRules of the ZoneId as data
     * (ZoneRules.getTransitions() on the Java side). n_tz_transitions > 0 replaces
     * shift_tz_offset_ms: toUtcTimestampMills / toEpochMillsForTimer / getNextTriggerWatermark
     * follow TimeWindowUtil.java:53-61,70-140,187-210 with these rules. SQL mode only (incl. the
     * two-phase operators, whose partial rows carry local slice ends). Copied at fg_open. */
    const int64_t* tz_transition_ms;   /* n_tz_transitions instants, epoch ms, ascending */
    const int64_t* tz_offset_ms;       /* n_tz_transitions + 1 offsets (ms): [i] in force before transition i */
    int32_t n_tz_transitions;
    int32_t tz_use_daylight;           /* TimeZone.getTimeZone(zone).useDaylightTime() */
    /* DataStream WindowOperator.allowedLateness (WindowedStream.allowedLateness, WindowOperator.java:
     * 608-622,630-681): a window's state is kept until cleanupTime = maxTimestamp + lateness
     * (Long.MAX_VALUE on overflow); an element of a fired window not yet cleaned re-fires it
     * (EventTimeTrigger.onElement :37-46). 0 for SQL operators. */
    int64_t allowed_lateness_ms;
} fg_config;

/* fg_batch.format bits -- narrow FG_HOST columns, so a batch moves fewer bytes over PCIe (the
 * link, not the kernels, bounds a host-fed operator): a shim whose keys fit 32 bits (INT keys,
 * dictionary ordinals, most BIGINT ids) and whose micro-batch spans < 2^32 ms hands 4-byte
 * columns; the engine widens them on the device. 24 -> 16 B per record for a DOUBLE value, 12 B
 * for a BIGINT value that fits 32 bits. */
enum fg_batch_format {
    FG_BATCH_KEY32 = 1,       /* key: int32_t[n], sign-extended */
    FG_BATCH_ROWTIME32 = 2,   /* rowtime: uint32_t[n], each rowtime_base + the offset */
    FG_BATCH_VAL32 = 4        /* BIGINT val: int32_t[n], sign-extended (FG_VAL_I64 only) */
};

typedef struct fg_batch {
    int64_t n;
    int32_t location;             /* fg_location of the column pointers */
    int32_t format;               /* fg_batch_format bits; 0: 8-byte columns. Non-zero: FG_HOST only */
    const int64_t* key;           /* BIGINT grouping key (FG_BATCH_KEY32: int32_t[]) */
    const int64_t* rowtime;       /* event time, epoch ms (TIMESTAMP(3) compact form; FG_BATCH_ROWTIME32: uint32_t[]) */
    const void* val;              /* int64_t[] or double[] per fg_config.val_type; may be NULL for FG_VAL_NONE */
    const uint8_t* val_null;      /* optional: 1 = value is NULL */
    int64_t rowtime_base;         /* FG_BATCH_ROWTIME32: rowtime[i] = rowtime_base + offset[i] */
} fg_batch;

typedef struct fg_rows {
    int64_t n;
    int32_t location;             /* where the column pointers live */
    int32_t num_aggs;
    const int64_t* key;
    const int64_t* window_start;
    const int64_t* window_end;
    const int64_t* agg[FG_MAX_AGGS];   /* 8-byte columns: BIGINT, or the bits of a DOUBLE */
    const uint8_t* null_mask;          /* bit i set: agg[i] is NULL in that row */
    const int64_t* rowtime;            /* DataStream: window.maxTimestamp() (end - 1); SQL: NULL */
} fg_rows;

/* Packed BinaryRowData input: the records as Flink holds them (BinaryRowData.java:68-76): row i
 * is the fixed-length part of a BinaryRowData of `arity` fields at rows + i * stride -- a
 * header byte (RowKind) and the null bits (bit 8 + f of the little-endian bit set marks field f
 * NULL, :155-157) in calculateBitSetWidthInBytes(arity) = ((arity + 71) / 64) * 8 bytes, then
 * 8 bytes per field (:119-121): BIGINT / DOUBLE as is (:306-320), TIMESTAMP(3) as its compact
 * epoch millis (:347-352). A shim hands a MemorySegment of such rows (e.g. the serialized
 * records of a network buffer or the RecordsWindowBuffer's pages) without building columns.
 * A NULL value field is a NULL value; a NULL key or rowtime is FG_EINVAL (the columnar boundary
 * has no NULL key either: the shim maps a nullable key to a BIGINT id). */
typedef struct fg_row_batch {
    int64_t n;
    int32_t location;             /* fg_location of `rows` */
    int32_t stride;               /* bytes between rows: >= the fixed-length part, a multiple of 8 */
    const uint8_t* rows;
    int32_t arity;                /* fields per row */
    int32_t key_field;            /* BIGINT grouping key */
    int32_t rowtime_field;        /* TIMESTAMP(3) event time */
    int32_t val_field;            /* BIGINT or DOUBLE per fg_config.val_type; -1: none (FG_VAL_NONE) */
} fg_row_batch;

/* Partial accumulator rows entering the global phase (GlobalAggCombiner.combine,
 * combines/GlobalAggCombiner.java:77-110, fed through the `sliced` assigner,
 * SliceAssigners.java:494-533): the rows of a FG_FLAG_LOCAL_PARTIALS operator after the
 * key-group exchange. */
typedef struct fg_partials {
    int64_t n;
    int32_t location;             /* fg_location of the column pointers */
    int32_t reserved0;
    const int64_t* key;
    const int64_t* slice_end;     /* the partial's slice (window_end of the local row) */
    const int64_t* cnt_star;
    const int64_t* cnt_val;
    const int64_t* sum;           /* i64 or f64 bits per fg_config.val_type */
    /* a global operator whose list mixes the SUM family, MIN and MAX (several value
     * accumulators): the partial MIN and MAX (the local phase's agg[3] / agg[4]); else NULL */
    const int64_t* min;
    const int64_t* max;
} fg_partials;

/* Checkpoint image of the GPU-resident keyed state: one entry per (key, slice) accumulator,
 * the content of WindowValueState "window-aggs" (AbstractWindowAggProcessor.java:103-109). */
typedef struct fg_state_rows {
    int64_t n;
    const int64_t* key;
    const int64_t* slice_end;     /* namespace of WindowValueState */
    const int64_t* cnt_star;      /* COUNT(*) accumulator */
    const int64_t* cnt_val;       /* COUNT(v) accumulator */
    const int64_t* sum;           /* SUM/AVG sum accumulator (i64 or f64 bits); a MIN- or MAX-only
                                   * operator: its MIN / MAX accumulator */
    const int64_t* min;           /* an operator with several value accumulators (SUM family, MIN,
                                   * MAX in one aggregate list): the MIN and MAX accumulators (the
                                   * identity where absent); NULL for other operators */
    const int64_t* max;
} fg_state_rows;

typedef struct fg_stats {
    int64_t records_in;
    int64_t records_staged;
    int64_t late_dropped;
    int64_t rows_fired;
    int64_t flushes;
    int64_t live_slices;
    int64_t state_regions;        /* P */
    int64_t region_capacity;      /* entries per region in HBM */
} fg_stats;

/* Per-kernel accounting (filled when FG_FLAG_KERNEL_TIMING is set): launches, summed
 * HIP-event duration on the handle's stream, records consumed and rows emitted. */
typedef struct fg_kernel_stat {
    char name[32];
    int64_t launches;
    double total_ms;
    int64_t records;
    int64_t rows;
} fg_kernel_stat;

typedef struct fg_handle fg_handle;

int  fg_open(const fg_config* cfg, fg_handle** out);
int  fg_add_batch(fg_handle* h, const fg_batch* batch);
/* fg_add_batch for packed BinaryRowData rows (same semantics, same processElement per row). */
int  fg_add_rows(fg_handle* h, const fg_row_batch* rows);
/* Global phase: merge partial accumulators (late rules of the global operator apply to
 * the partial's slice). */
int  fg_add_partials(fg_handle* h, const fg_partials* partials);
int  fg_advance_progress(fg_handle* h, int64_t watermark, int32_t out_location, fg_rows* fired);
/* Asynchronous fg_advance_progress (ABI 11; the same processWatermark, device output): the
 * windows the watermark fires are queued on the handle's stream and the call returns without
 * waiting for them. A shim that forwards the watermark only after the fired rows (Flink emits a
 * window's rows before the watermark, SlicingWindowOperator.java:207-237 / WindowOperator
 * onEventTime) takes them with fg_collect_fired, which waits; until then the host is free to
 * deliver the next watermarks and batches. The fires' completion -- row count, region retries,
 * overflow check -- is taken by the next call that needs it: a watermark that fires again, any
 * batch, flush, snapshot or restore. Errors of a fire are reported by that call. The rows of an
 * async advance stay valid until the next call that fires windows. */
int  fg_advance_progress_async(fg_handle* h, int64_t watermark);
/* fg_advance_progress_async of n watermarks in order, as n calls would (ABI 13): the
 * watermarks a shim received since its last batch -- with no element between them -- in one
 * call instead of one JNI / C call each (configs[0]: 100 watermarks per 1M-record batch; each
 * one that fires nothing only moves the progress). Stops at the first error. */
int  fg_advance_progress_async_n(fg_handle* h, const int64_t* watermarks, int64_t n);
/* Waits for the fires of the last fg_advance_progress_async call and returns their rows (device
 * pointers, as fg_advance_progress with FG_DEVICE); n = 0 when it fired nothing. A synchronous
 * fg_advance_progress called while async rows are uncollected returns them ahead of its own rows
 * (none is dropped). */
int  fg_collect_fired(fg_handle* h, fg_rows* fired);
/* fg_collect_fired with the rows at out_location (ABI 12): FG_HOST copies them into library-owned
 * host memory (as fg_advance_progress with FG_HOST) -- what a JVM shim wraps in direct buffers;
 * FG_DEVICE is fg_collect_fired. */
int  fg_collect_fired_to(fg_handle* h, int32_t out_location, fg_rows* fired);
int  fg_flush(fg_handle* h);
/* Local phase only (FG_FLAG_LOCAL_PARTIALS; ABI 12): every buffered slice emits its partial
 * accumulator rows now, as fg_advance_progress does for the slices a watermark fires --
 * LocalSlicingWindowAggOperator.prepareSnapshotPreBarrier -> WindowBuffer.flush
 * (LocalSlicingWindowAggOperator.java:142-144, RecordsWindowBuffer.java:108-119 with
 * LocalAggCombiner.java:69-106): the local operator holds no state across a checkpoint. The
 * progress does not move. Rows as fg_advance_progress at out_location. */
int  fg_flush_partials(fg_handle* h, int32_t out_location, fg_rows* fired);
int  fg_snapshot_state(fg_handle* h, fg_state_rows* out, int64_t* timer_watermark);
/* snapshotState in two parts (ABI 15; StreamOperatorStateHandler.snapshotState's synchronous
 * part and the AsyncSnapshotCallable of a heap state backend, SnapshotStrategyRunner.snapshot):
 * _async flushes the staged records and exports every resident slice into a device image (the
 * state as of this call) and queues its copy into the pinned host image on a stream of its own;
 * the operator takes batches, watermarks and partials meanwhile. _wait returns that image (the
 * fg_snapshot_state layout, valid until the next snapshot call) once the copy has completed.
 * One snapshot at a time: fg_snapshot_state[_async] fails with FG_ESTATE while one is not
 * collected. fg_snapshot_state is _async + _wait. An image of an operator that never saw a NULL
 * value may return the same column for cnt_star and cnt_val (they are equal). */
int  fg_snapshot_state_async(fg_handle* h);
int  fg_snapshot_state_wait(fg_handle* h, fg_state_rows* out, int64_t* timer_watermark);
/* The slices of the image the last fg_snapshot_state / fg_snapshot_state_wait returned (ABI 16):
 * the image's rows are grouped by slice, ascending; `changed` tells whether the slice's state was
 * written since the previous image of this handle (a new slice, a flush or fold into it, a late
 * record; every slice of a handle's first image; a table restored into an empty handle by fg_restore
 * counts as unchanged -- the backend holds it). A shim keeps its keyed state between checkpoints and
 * rewrites only the changed slices' entries, clearing the namespaces of slices no longer in the image
 * (AbstractWindowAggProcessor.prepareCheckpoint :195-197 flushes only the buffer; AggCombiner.combine
 * :76-115 touches only the (key, slice) pairs a flush saw). Valid until the next snapshot call. */
typedef struct fg_image_slices {
    int64_t n;
    const int64_t* slice_end;   /* [n] */
    const int64_t* first_row;   /* [n] the slice's rows are image rows [first_row, first_row + rows) */
    const int64_t* rows;        /* [n] */
    const uint8_t* changed;     /* [n] 1 / 0 */
} fg_image_slices;
int  fg_snapshot_slices(fg_handle* h, fg_image_slices* out);
/* The device self-check (ABI 16): the DPP wave scans and the tile walk the fire runs, as this
 * library's code object compiled them, on inputs whose answers the host knows (msg: "ok" or what is
 * wrong). fg_open runs it once per process and device and fails with FG_EDEVICE (its message in
 * fg_last_error(NULL)) if it does not pass: a miscompiled build fails loudly instead of firing wrong
 * rows. */
int  fg_selftest(int32_t device_id, char* msg, int32_t cap);
int  fg_restore(fg_handle* h, const fg_state_rows* in, int64_t timer_watermark);
int  fg_late_dropped(fg_handle* h, int64_t* out);
int  fg_get_stats(fg_handle* h, fg_stats* out);
int  fg_synchronize(fg_handle* h);
/* Drop all resident state and staged records, keep device allocations: a fresh operator
 * after open() + initializeState() from an empty snapshot. */
int  fg_reset(fg_handle* h);
/* Copies up to `max` kernel statistics into out; *count receives the number available. */
int  fg_kernel_stats(fg_handle* h, fg_kernel_stat* out, int32_t max, int32_t* count);
/* With FG_FLAG_KERNEL_TIMING: bracket only the kernel classes whose bit is set (bit i = entry
 * i of fg_kernel_stats' list); each bracket costs two events on the stream, so a measurement
 * times the kernel it reports and leaves the others unperturbed. Default: all classes. */
int  fg_set_kernel_timing(fg_handle* h, uint32_t class_mask);
/* Device stream of the handle (hipStream_t), for callers that overlap their own work. */
void* fg_stream(fg_handle* h);
const char* fg_last_error(fg_handle* h);   /* h may be NULL: last error of fg_open */
void fg_close(fg_handle* h);

/* Key-group routing (keyBy partitioner) on the device of `device_id`:
 * out_kg[i] = murmurHash(hash(key[i])) % max_parallelism, hash per fg_key_hash.
 * Pointers are device pointers when location == FG_DEVICE. */
int  fg_key_groups(int32_t device_id, int32_t location, int64_t n, const int64_t* key,
                   int32_t key_hash, int32_t max_parallelism, int32_t* out_kg);

/* Pack a batch for the key-group exchange: records are reordered by destination
 * subtask (kg * parallelism / max_parallelism) into the caller-provided device buffers,
 * counts[parallelism] receives per-destination record counts. Device pointers only. */
int  fg_partition_by_owner(int32_t device_id, void* stream, int64_t n, const int64_t* key,
                           const int64_t* rowtime, const int64_t* val, int32_t key_hash,
                           int32_t max_parallelism, int32_t parallelism, int64_t* out_key,
                           int64_t* out_rowtime, int64_t* out_val, int64_t* counts);

/* The same for `ncols` int64 columns moved together (cols[0] = the key), e.g. the partial
 * accumulator rows (key, slice_end, cnt_star, cnt_val, sum) of the two-phase exchange.
 * ncols <= 8. Device pointers only. */
int  fg_partition_columns_by_owner(int32_t device_id, void* stream, int64_t n, int32_t ncols,
                                   const int64_t* const* cols, int32_t key_hash, int32_t max_parallelism,
                                   int32_t parallelism, int64_t* const* out_cols, int64_t* counts);

/* The keyBy edge of the two-phase plan over RCCL (ABI 14; libflinkgpu.so links librccl): replaces,
 * between co-located subtasks, KeyGroupStreamPartitioner.selectChannel
 * (SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:55-65) + RecordWriter.emit
 * (RT/io/network/api/writer/RecordWriter.java:101-128) on the edge LocalSlicingWindowAggOperator ->
 * GlobalSlicingWindowAggOperator, and StatusWatermarkValve's min over the input channels
 * (SJ/runtime/watermarkstatus/StatusWatermarkValve.java). One communicator per subtask (one process
 * per GPU): a coordinator (the JobManager) makes the id once with fg_comm_unique_id and ships its
 * bytes with the deployment; every subtask calls fg_comm_open(device, parallelism, its index, id),
 * which blocks until all have joined. Owner of a row = computeOperatorIndexForKeyGroup(key group)
 * (KeyGroupRangeAssignment.java:124-127) with fg_key_hash routing. Per exchange: the rows grouped by
 * owner on the device, ONE all-to-all of (row count, this rank's watermark) per peer, ONE host read
 * of them, grouped send / receive of each column's runs. Collective: every rank calls the same
 * exchanges in the same order (a rank with no rows still calls). Not for per-rank dictionary ids
 * (FG_KEYHASH_DICT_ID of different dictionaries): those ship key rows. */
#define FG_COMM_ID_BYTES 128
typedef struct fg_comm fg_comm;
typedef struct fg_exchanged {
    int64_t n;                        /* rows received (this rank's key groups) */
    int32_t ncols;
    int32_t reserved0;
    const int64_t* cols[8];           /* device columns, communicator-owned, valid until the next exchange;
                                       * complete in stream order on fg_comm_stream */
    int64_t min_watermark;            /* min over the ranks of the watermarks passed in (StatusWatermarkValve) */
    int64_t bytes_sent;               /* to other ranks */
} fg_exchanged;
int  fg_comm_unique_id(uint8_t* id /* FG_COMM_ID_BYTES */);
int  fg_comm_open(int32_t device_id, int32_t world, int32_t rank, const uint8_t* id, fg_comm** out);
/* ncols <= 8 int64 device columns (cols[0] = key) produced on `stream` (hipStream_t; the
 * communicator's stream waits for it), grouped by owner and exchanged. */
int  fg_comm_exchange_columns(fg_comm* c, void* stream, int64_t n, int32_t ncols, const int64_t* const* cols,
                              int32_t key_hash, int32_t max_parallelism, int64_t watermark, fg_exchanged* out);
/* The local operator's partial rows (FG_DEVICE rows of a FG_FLAG_LOCAL_PARTIALS handle: key,
 * window_end = slice end, agg[0..2] or [0..4]) exchanged and merged into this rank's global operator
 * (fg_add_partials on `global`, ordered after the collective on its stream). *min_watermark receives
 * the combined watermark the caller then advances `global` to. */
int  fg_comm_exchange_partials(fg_comm* c, fg_handle* local, const fg_rows* rows, int32_t key_hash,
                               int32_t max_parallelism, int64_t watermark, fg_handle* global, int64_t* min_watermark);
/* fg_comm_exchange_partials of the rows fg_collect_fired(local) returns (the local fires of the
 * async advances since the last collect) -- a shim's per-batch call: LocalSlicingWindowAggOperator
 * .processWatermark's output edge. */
int  fg_comm_exchange_fired(fg_comm* c, fg_handle* local, int32_t key_hash, int32_t max_parallelism,
                            int64_t watermark, fg_handle* global, int64_t* min_watermark);
/* ... of fg_flush_partials(local) (LocalSlicingWindowAggOperator.prepareSnapshotPreBarrier :142-144:
 * the local buffer crosses the edge before the barrier). */
int  fg_comm_exchange_flushed(fg_comm* c, fg_handle* local, int32_t key_hash, int32_t max_parallelism,
                              int64_t watermark, fg_handle* global, int64_t* min_watermark);
/* The exchange as a round of three calls (ABI 16), for a subtask whose edge runs on a thread of its
 * own: the operators are touched only in _begin (the local rows collected or flushed and grouped by
 * owner) and _end (the received rows merged into `global`), never while _exchange waits for the
 * peers. Every rank runs the same sequence of rounds: a rank with nothing to send still begins an
 * FG_ROUND_IDLE round. The meta words of a round carry each rank's watermark and epoch (the id of
 * the last checkpoint whose pre-barrier flush it has sent) and a failure flag: a rank whose _begin
 * failed still takes part, sending no rows, and _exchange then fails on EVERY rank with FG_EDEVICE
 * (fg_round.failed_rank) instead of leaving the peers blocked in the data collective. After a
 * _begin -- whatever it returned -- the caller calls _exchange; _end after an _exchange that
 * returned FG_OK. */
#define FG_ROUND_FIRED 0     /* the local handle's uncollected async fires (fg_collect_fired) */
#define FG_ROUND_FLUSHED 1   /* the local buffer (fg_flush_partials: before a checkpoint barrier) */
#define FG_ROUND_IDLE 2      /* nothing to send (local may be NULL) */
typedef struct fg_round {
    int64_t min_watermark;   /* min over the ranks of the watermarks passed to _begin (StatusWatermarkValve) */
    int64_t min_epoch;       /* min over the ranks of the epochs passed to _begin */
    int64_t rows_sent;       /* this rank's rows (to every rank, itself included) */
    int64_t rows_received;
    int64_t bytes_sent;      /* to other ranks */
    int32_t failed_rank;     /* -1, or the lowest rank whose round failed (world: column counts disagree) */
    int32_t reserved0;
} fg_round;
int  fg_comm_round_begin(fg_comm* c, fg_handle* local, int32_t mode, int32_t key_hash, int32_t max_parallelism,
                         int64_t watermark, int64_t epoch);
int  fg_comm_round_exchange(fg_comm* c, fg_round* out);
int  fg_comm_round_end(fg_comm* c, fg_handle* global);
void* fg_comm_stream(fg_comm* c);
int64_t fg_comm_bytes_sent(fg_comm* c);      /* bytes sent to other ranks by every exchange so far */
const char* fg_comm_last_error(fg_comm* c);   /* c may be NULL: last error of fg_comm_open / _unique_id */
void fg_comm_close(fg_comm* c);

/* Grouping keys of any type (STRING, several key columns ...): a GPU-resident dictionary of the
 * serialized key rows. The reference groups by the BinaryRowData key row the key selector
 * projects (BinaryRowDataKeySelector.java:43-50); two keys are equal iff their rows' bytes are
 * (BinarySection.equals, BinarySection.java:62-73), and the key group comes from
 * MurmurHashUtils.hashBytesByWords over those bytes, seed 42 (BinarySection.hashCode :76-78,
 * MurmurHashUtils.java:92-96,131-170) -> KeyGroupRangeAssignment. fg_key_dict_intern maps each row
 * to a 64-bit id: equal rows -> equal ids, distinct rows -> distinct ids (exact: a hash collision
 * is resolved by comparing the bytes), id = ordinal << ceil(log2(max_parallelism)) | key group (below
 * 2^31 for 16.7M keys at max parallelism 128, so the window engine stages them as 32-bit keys). The ids are the BIGINT key
 * column of fg_add_batch / the key field of fg_add_rows; FG_KEYHASH_DICT_ID routes them by the
 * carried key group; fired rows' ids map back to their rows with fg_key_dict_lookup. A handle is
 * single-threaded like fg_handle; ids are stable for the dictionary's life (a restored operator
 * re-interns the key rows of its state image first). */
typedef struct fg_key_dict fg_key_dict;
int  fg_key_dict_open(int32_t device_id, int32_t max_parallelism, int64_t expected_keys, fg_key_dict** out);
/* n key rows: row i = bytes[offsets[i], offsets[i] + lengths[i]) (nbytes = the buffer's size),
 * each length and offset a multiple of 4 (BinaryRowData rows are multiples of 8; rows may
 * overlap). out_id[n] receives the ids, out_kg[n] (optional) the rows' key groups under the
 * dictionary's max parallelism. All pointers FG_HOST or all FG_DEVICE (location). FG_DEVICE
 * inputs are read on the dictionary's stream (fg_key_dict_stream): the caller orders their
 * producer before it; the outputs are complete when the call returns. */
int  fg_key_dict_intern(fg_key_dict* d, int32_t location, int64_t n, const uint8_t* bytes, int64_t nbytes,
                        const int64_t* offsets, const int32_t* lengths, int64_t* out_id, int32_t* out_kg);
/* fg_key_dict_intern of device rows in two halves (ABI 13): _async launches the lookup of every
 * row on the dictionary's stream (fg_key_dict_stream) and returns at once; _wait synchronizes,
 * interns the rows the table did not hold yet and resolves tag collisions -- out_id / out_kg are
 * complete when it returns. A key selector interns the next micro-batch's rows while the engine
 * aggregates the current one. One call pending per dictionary (FG_ESTATE otherwise); bad rows are
 * reported by _wait, before anything is inserted. */
int  fg_key_dict_intern_async(fg_key_dict* d, int64_t n, const uint8_t* bytes, int64_t nbytes, const int64_t* offsets,
                              const int32_t* lengths, int64_t* out_id, int32_t* out_kg);
int  fg_key_dict_intern_wait(fg_key_dict* d);
/* For each id: its row's offset and length in the dictionary's arena (-1 / -1 for an unknown id). */
int  fg_key_dict_lookup(fg_key_dict* d, int32_t location, int64_t n, const int64_t* ids, int64_t* out_offsets,
                        int32_t* out_lengths);
/* The arena (device memory, rows padded to 8 bytes) and its used size; valid until the next intern. */
int  fg_key_dict_arena(fg_key_dict* d, const uint8_t** dev_bytes, int64_t* size);
int  fg_key_dict_copy_arena(fg_key_dict* d, int64_t begin, int64_t nbytes, uint8_t* host);
int64_t fg_key_dict_size(fg_key_dict* d);   /* distinct key rows interned */
void* fg_key_dict_stream(fg_key_dict* d);   /* the dictionary's device stream (hipStream_t) */
/* HIP-event timing of the dictionary's kernels (per chunk: "dict_probe", then "dict_assign" =
 * assign + verify of the rows new in the chunk); fg_key_dict_kernel_stats copies them. */
int  fg_key_dict_set_timing(fg_key_dict* d, int32_t on);
int  fg_key_dict_kernel_stats(fg_key_dict* d, fg_kernel_stat* out, int32_t max, int32_t* count);
const char* fg_key_dict_last_error(fg_key_dict* d);
void fg_key_dict_close(fg_key_dict* d);
/* BinarySection.hashCode of one row (MurmurHashUtils.hashBytesByWords, seed 42); len % 4 == 0. */
int32_t fg_binaryrow_hash(const uint8_t* row, int32_t len);

/* Page-lock a caller range for FG_HOST input (hipHostRegister): Flink's managed memory is
 * off-heap MemorySegments (MemorySegmentFactory.allocateOffHeapUnsafeMemory,
 * CO/core/memory/MemorySegmentFactory.java:130-167; address MemorySegment.getAddress :288)
 * that live for the operator's life, so a shim registers each segment it hands batches from
 * once, at open, and unregisters it at close. Batches read from a registered range are DMA'd
 * directly; pageable ranges are staged by the runtime at a lower rate. Not per handle: the
 * registration serves every handle on the device. Errors: fg_last_error(NULL). */
int  fg_host_register(int32_t device_id, void* p, int64_t bytes);
int  fg_host_unregister(int32_t device_id, void* p);

int  fg_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FLINKGPU_H */
