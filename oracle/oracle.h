/*
 * ORACLE -- test infrastructure only.
 *
 * CPU restatement (plain C) of the reference's keyed window-aggregation path:
 *   SQL:        SlicingWindowOperator + SliceAssigners + AbstractWindowAggProcessor
 *               + Slice(Un)SharedWindowAggProcessor + RecordsWindowBuffer + AggCombiner
 *               + InternalTimerServiceImpl (event time, heap timers, dedup)
 *   DataStream: WindowOperator + Tumbling/SlidingEventTimeWindows + EventTimeTrigger
 *               + SumAggregator (ReducingState)
 *   Routing:    KeyGroupRangeAssignment + MathUtils.murmurHash + BinaryRowData Murmur3.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the reported CPU baseline.  Nothing in the
 * product path (flink_amd/, include/) links or calls it.
 *
 * Parity pinning: the restatement is checked against the reference's own known-answer
 * tests transcribed under tests/golden/ (see tests/golden/make_golden.py for the
 * file:line of every vector).  Key-group routing has no literal known-answer test in
 * the reference and is pinned by restatement only.
 */
#ifndef FLINK_ORACLE_H
#define FLINK_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_MODE_SQL = 0, OR_MODE_DATASTREAM = 1 };
enum { OR_TUMBLE = 0, OR_HOP = 1, OR_CUMULATE = 2 };
enum { OR_VAL_NONE = 0, OR_VAL_I64 = 1, OR_VAL_F64 = 2 };

typedef struct or_config {
    int32_t mode;             /* OR_MODE_SQL / OR_MODE_DATASTREAM */
    int32_t kind;             /* OR_TUMBLE / OR_HOP / OR_CUMULATE (DataStream: TUMBLE / HOP=sliding) */
    int64_t size;             /* tumble size, hop size, cumulate max size (ms) */
    int64_t slide;            /* hop slide, cumulate step (ms); ignored for tumble */
    int64_t offset;           /* window offset (ms) */
    int64_t tz_offset_ms;     /* fixed-offset shift time zone (no DST); 0 = UTC */
    int32_t val_type;         /* OR_VAL_* */
    int32_t count_star_index; /* >= 0 when the agg list holds COUNT(*) (required for HOP) */
    int32_t proctime;         /* SQL processing-time windows (assigner isEventTime() == false) */
    int32_t tz_n;             /* > 0: a zone with transitions (DST); tz_offset_ms is then ignored */
    const int64_t* tz_trans;  /* tz_n transition instants (epoch ms, ascending) */
    const int64_t* tz_offs;   /* tz_n + 1 offsets (ms): [i] in force before transition i */
    int32_t tz_use_dst;       /* TimeZone.getTimeZone(zone).useDaylightTime() */
    int32_t windowed;         /* WindowedSliceAssigner over the kind's assigner: ts = window_end */
    int32_t phase;            /* OR_PHASE_*: single operator, or the local / global half of the
                               * two-phase plan (TwoStageOptimizedWindowAggregateRule) */
    int32_t purging;          /* DataStream: PurgingTrigger.of(EventTimeTrigger) (FIRE -> FIRE_AND_PURGE) */
    int64_t allowed_lateness; /* DataStream WindowOperator.allowedLateness (ms, >= 0) */
} or_config;
enum { OR_PHASE_SINGLE = 0, OR_PHASE_LOCAL = 1, OR_PHASE_GLOBAL = 2 };

/* One fired row. The aggregate set is fixed: COUNT(*), COUNT(v), SUM(v), AVG(v), SUM0(v), MIN(v), MAX(v). */
typedef struct or_row {
    int64_t key;
    int64_t window_start;
    int64_t window_end;
    int64_t cnt_star;
    int64_t cnt_val;
    int64_t sum_i;      /* SUM for i64 values (valid when !sum_null)            */
    double  sum_d;      /* SUM for f64 values (valid when !sum_null)            */
    int64_t avg_i;      /* AVG for i64 values: Java long division (valid when !avg_null) */
    double  avg_d;      /* AVG for f64 values: sum / (double) count            */
    int32_t sum_null;
    int32_t avg_null;
    int64_t out_ts;     /* DataStream: emitted StreamRecord timestamp (end - 1) */
    int64_t sum0_i;     /* SUM0 for i64 values (Sum0AggFunction: 0-initialised, never NULL) */
    double  sum0_d;     /* SUM0 for f64 values                                  */
    int64_t min_i;      /* MIN / MAX (Min/MaxAggFunction; NULL exactly when sum_null) */
    int64_t max_i;
    double  min_d;
    double  max_d;
} or_row;

typedef struct or_op or_op;

/* Returns NULL on invalid parameters; err receives the reference's exception message. */
or_op*  or_open(const or_config* cfg, char* err, int errlen);
void    or_close(or_op* op);
/* processElement for n records. val points at int64_t[] or double[] (or NULL for NONE);
 * isnull may be NULL. */
void    or_process_batch(or_op* op, int64_t n, const int64_t* key, const int64_t* ts,
                         const void* val, const uint8_t* isnull);
void    or_process_watermark(or_op* op, int64_t wm);
/* Global phase: n partial accumulator rows as the local phase emits them (key, window_end =
 * the slice end, cnt_star, cnt_val, sum/sum0/min/max, sum_null), through the `sliced`
 * assigner and GlobalAggCombiner. A local-phase operator's take_rows are such rows. */
void    or_process_partials(or_op* op, int64_t n, const or_row* rows);
/* prepareSnapshotPreBarrier: RecordsWindowBuffer.flush() (no-op for DataStream). */
void    or_prepare_snapshot(or_op* op);
/* snapshot -> close -> initializeState -> open: state and timers survive, the buffer
 * (empty after prepare_snapshot), processor progress and timer watermark reset. */
or_op*  or_restore_copy(const or_op* op);
int64_t or_num_rows(const or_op* op);
const or_row* or_rows(const or_op* op);
void    or_clear_rows(or_op* op);
int64_t or_late_dropped(const or_op* op);
int64_t or_state_entries(const or_op* op);
int64_t or_pending_timers(const or_op* op);
/* DataStream WindowOperator keyed state image ("window-contents" + "window-timers") */
int64_t or_ds_export_state(const or_op* op, int64_t* key, int64_t* end, int64_t* cnt, int64_t* sum, int64_t* mn,
                           int64_t* mx);
int64_t or_export_timers(const or_op* op, int64_t* key, int64_t* ns, int64_t* ts);
or_op*  or_ds_import(const or_config* cfg, int64_t n, const int64_t* key, const int64_t* end, const int64_t* val,
                     const int64_t* cnt, int64_t nt, const int64_t* tkey, const int64_t* tns, const int64_t* tts,
                     char* err, int errlen);

/* --- slice assigner restatement (SliceAssigners.java) ------------------------- */
int64_t or_assign_slice_end(const or_op* op, int64_t ts);
/* TimeWindowUtil with the operator's zone: toUtcTimestampMills, toEpochMillsForTimer,
 * toEpochMills, getNextTriggerWatermark(useDayLightSaving of the zone) */
int64_t or_to_utc(const or_op* op, int64_t epoch);
int64_t or_to_epoch_for_timer(const or_op* op, int64_t local);
int64_t or_to_epoch(const or_op* op, int64_t local);
int64_t or_next_trigger(const or_op* op, int64_t wm);
int64_t or_get_window_start(const or_op* op, int64_t window_end);
int64_t or_get_last_window_end(const or_op* op, int64_t slice_end);
/* writes up to 2 slices, returns count */
int32_t or_expired_slices(const or_op* op, int64_t window_end, int64_t* out);
/* HOP/CUMULATE mergeSlices: *merge_result = MIN when null namespace; returns #toBeMerged */
int32_t or_merge_slices(const or_op* op, int64_t slice_end, int64_t* merge_result, int64_t* out, int32_t cap);
/* nextTriggerWindow: returns 1 and *next when present */
int32_t or_next_trigger_window(const or_op* op, int64_t window_end, int32_t is_empty, int64_t* next);
int64_t or_next_trigger_watermark(int64_t wm, int64_t interval);
int64_t or_window_start_with_offset(int64_t ts, int64_t offset, int64_t size);

/* --- key groups (KeyGroupRangeAssignment / MathUtils / MurmurHashUtils) ------- */
int32_t or_binaryrow_hash_i64(int64_t key);
int32_t or_binaryrow_hash_bytes(const uint8_t* row, int32_t len);          /* BinaryRowData(BIGINT).hashCode() */
int32_t or_long_hash(int64_t key);                    /* java.lang.Long.hashCode() */
int32_t or_murmur_hash(int32_t code);                 /* MathUtils.murmurHash */
int32_t or_key_group(int32_t key_hash, int32_t max_parallelism);
int32_t or_operator_index(int32_t max_parallelism, int32_t parallelism, int32_t key_group);
int32_t or_default_max_parallelism(int32_t parallelism);
void    or_key_groups_binaryrow(int64_t n, const int64_t* key, int32_t max_parallelism, int32_t* out);

/* --- CPU baseline: P operator instances, one per core, records routed by key group.
 * Watermark wm_val[j] is delivered after record index wm_at[j] (exclusive prefix).
 * Returns elapsed seconds of the parallel processing region (routing excluded);
 * *rows_out receives total fired rows, *checksum an order-independent checksum. */
double  or_run_partitioned(const or_config* cfg, int32_t parallelism, int32_t max_parallelism,
                           int64_t n, const int64_t* key, const int64_t* ts, const void* val,
                           int32_t n_wm, const int64_t* wm_at, const int64_t* wm_val,
                           int64_t* rows_out, uint64_t* checksum, int64_t* late_out);

/* --- The same, keeping every fired row (parity runs at BASELINE key spaces): the rows of
 * all instances are concatenated into *rows (malloc'd; free with or_free), *n_rows their
 * count. snapshot_after >= 0: after watermark snapshot_after every instance takes a
 * checkpoint (prepareSnapshotPreBarrier) and continues as a restored copy (initializeState
 * from that snapshot), as a failover would. Returns elapsed seconds. */
double  or_run_partitioned_rows(const or_config* cfg, int32_t parallelism, int32_t max_parallelism,
                                int64_t n, const int64_t* key, const int64_t* ts, const void* val,
                                int32_t n_wm, const int64_t* wm_at, const int64_t* wm_val,
                                int32_t snapshot_after, or_row** rows, int64_t* n_rows, int64_t* late_out);
void    or_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
