/*
 * ORACLE -- test infrastructure only (see oracle.h for scope and pinning).
 *
 * Plain-C restatement of the reference CPU operators. Every function cites the
 * reference file:line it follows. Paths are abbreviated as in SURVEY.md:
 *   TR/  = flink-table/flink-table-runtime-blink/src/main/java/org/apache/flink/table/runtime/
 *   TP/  = flink-table/flink-table-planner-blink/src/main/java/org/apache/flink/table/planner/
 *   SJ/  = flink-streaming-java/src/main/java/org/apache/flink/streaming/
 *   RT/  = flink-runtime/src/main/java/org/apache/flink/runtime/
 *   CO/  = flink-core/src/main/java/org/apache/flink/
 *   TC/  = flink-table/flink-table-common/src/main/java/org/apache/flink/table/data/
 *
 * Java `long` arithmetic wraps; every add/sub on times and integer sums goes through
 * jadd/jsub (unsigned arithmetic) so C never hits signed-overflow UB.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define JMAX INT64_MAX
#define JMIN INT64_MIN

static inline int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
static inline int32_t imul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
static inline int32_t iadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t rotl32(int32_t x, int r) {
    uint32_t u = (uint32_t)x;
    return (int32_t)((u << r) | (u >> (32 - r)));
}
static inline int64_t jmod(int64_t a, int64_t b) { /* Java `%` (truncated); b > 0 here */
    return a % b;
}

/* ------------------------------------------------------------------------------------
 * Pair-keyed open-addressing map (int64,int64) -> int64. Linear probing, backward-shift
 * deletion. Stands in for the heap-state CopyOnWriteStateMap / BytesMap lookups.
 * ---------------------------------------------------------------------------------- */
typedef struct {
    int64_t* ka;
    int64_t* kb;
    int64_t* v;
    uint8_t* used;
    int64_t cap, n;
} pmap;

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static inline uint64_t phash(int64_t a, int64_t b) {
    return mix64((uint64_t)a * 0x9E3779B97F4A7C15ULL ^ mix64((uint64_t)b + 0x632BE59BD9B4E019ULL));
}
static void pmap_init(pmap* m, int64_t cap) {
    int64_t c = 16;
    while (c < cap) c <<= 1;
    m->cap = c;
    m->n = 0;
    m->ka = (int64_t*)malloc(sizeof(int64_t) * c);
    m->kb = (int64_t*)malloc(sizeof(int64_t) * c);
    m->v = (int64_t*)malloc(sizeof(int64_t) * c);
    m->used = (uint8_t*)calloc((size_t)c, 1);
}
static void pmap_free(pmap* m) {
    free(m->ka); free(m->kb); free(m->v); free(m->used);
    memset(m, 0, sizeof(*m));
}
static int64_t* pmap_find(const pmap* m, int64_t a, int64_t b) {
    uint64_t mask = (uint64_t)m->cap - 1, i = phash(a, b) & mask;
    while (m->used[i]) {
        if (m->ka[i] == a && m->kb[i] == b) return &m->v[i];
        i = (i + 1) & mask;
    }
    return NULL;
}
static void pmap_grow(pmap* m);
/* returns pointer to value; *inserted = 1 when new (value then uninitialised) */
static int64_t* pmap_upsert(pmap* m, int64_t a, int64_t b, int* inserted) {
    if ((m->n + 1) * 2 > m->cap) pmap_grow(m);
    uint64_t mask = (uint64_t)m->cap - 1, i = phash(a, b) & mask;
    while (m->used[i]) {
        if (m->ka[i] == a && m->kb[i] == b) { *inserted = 0; return &m->v[i]; }
        i = (i + 1) & mask;
    }
    m->used[i] = 1; m->ka[i] = a; m->kb[i] = b; m->n++;
    *inserted = 1;
    return &m->v[i];
}
static void pmap_grow(pmap* m) {
    pmap o = *m;
    pmap_init(m, o.cap * 2);
    for (int64_t i = 0; i < o.cap; i++) {
        if (!o.used[i]) continue;
        int ins;
        *pmap_upsert(m, o.ka[i], o.kb[i], &ins) = o.v[i];
    }
    pmap_free(&o);
}
static int pmap_remove(pmap* m, int64_t a, int64_t b, int64_t* old) {
    uint64_t mask = (uint64_t)m->cap - 1, i = phash(a, b) & mask;
    while (m->used[i]) {
        if (m->ka[i] == a && m->kb[i] == b) break;
        i = (i + 1) & mask;
    }
    if (!m->used[i]) return 0;
    if (old) *old = m->v[i];
    /* backward-shift deletion */
    uint64_t j = i;
    for (;;) {
        j = (j + 1) & mask;
        if (!m->used[j]) break;
        uint64_t h = phash(m->ka[j], m->kb[j]) & mask;
        /* can slot j's entry move to i? yes if h is cyclically outside (i, j] */
        int move = (i <= j) ? (h <= i || h > j) : (h <= i && h > j);
        if (move) {
            m->ka[i] = m->ka[j]; m->kb[i] = m->kb[j]; m->v[i] = m->v[j];
            i = j;
        }
    }
    m->used[i] = 0;
    m->n--;
    return 1;
}

/* ------------------------------------------------------------------------------------
 * Accumulators: generated NamespaceAggsHandleFunction for
 *   COUNT(*)  -> Count1AggFunction   TP/functions/aggfunctions/Count1AggFunction.java:64-79
 *   COUNT(v)  -> CountAggFunction    TP/functions/aggfunctions/CountAggFunction.java:63-83
 *   SUM(v)    -> SumAggFunction      TP/functions/aggfunctions/SumAggFunction.java:58-96 (null init)
 *   AVG(v)    -> AvgAggFunction      TP/functions/aggfunctions/AvgAggFunction.java:64-103 (0 init)
 *   SUM0(v)   -> Sum0AggFunction     TP/functions/aggfunctions/Sum0AggFunction.java:60-63,75-76
 *                (0 init :97-98/:136-137/:162-163, sum0 + v for non-null v): the same
 *                accumulator as AVG's sum, so it is read from avg_sum_* at emit
 *   MIN(v)    -> MinAggFunction      TP/functions/aggfunctions/MinAggFunction.java:56-90
 *   MAX(v)    -> MaxAggFunction      TP/functions/aggfunctions/MaxAggFunction.java:56-96
 *                null init; accumulate/merge: isNull(operand) ? acc : isNull(acc) ? operand :
 *                lessThan(operand, acc) ? operand : acc (greaterThan for MAX), Java primitive
 *                comparison. Null exactly when SUM is null, so sum_null serves all three.
 * ---------------------------------------------------------------------------------- */
typedef struct {
    int64_t cnt_star, cnt_val;
    int64_t sum_i, avg_sum_i;
    double sum_d, avg_sum_d;
    int32_t sum_null;
    int64_t min_i, max_i;
    double min_d, max_d;
} or_acc;

static inline void acc_create(or_acc* a) {   /* initialValuesExpressions */
    memset(a, 0, sizeof(*a));
    a->sum_null = 1;
}
static inline void acc_accumulate(or_acc* a, int vt, int64_t vbits, int isnull) {
    a->cnt_star = jadd(a->cnt_star, 1);                 /* count1 = count1 + 1 */
    if (isnull) return;                                  /* ifThenElse(isNull(operand(0)), ...) */
    a->cnt_val = jadd(a->cnt_val, 1);
    if (vt == OR_VAL_I64) {
        a->sum_i = a->sum_null ? vbits : jadd(a->sum_i, vbits);   /* isNull(sum) ? v : sum + v */
        a->avg_sum_i = jadd(a->avg_sum_i, vbits);
        a->min_i = a->sum_null ? vbits : (vbits < a->min_i ? vbits : a->min_i);
        a->max_i = a->sum_null ? vbits : (vbits > a->max_i ? vbits : a->max_i);
    } else if (vt == OR_VAL_F64) {
        double d;
        memcpy(&d, &vbits, 8);
        a->sum_d = a->sum_null ? d : a->sum_d + d;
        a->avg_sum_d = a->avg_sum_d + d;
        a->min_d = a->sum_null ? d : (d < a->min_d ? d : a->min_d);
        a->max_d = a->sum_null ? d : (d > a->max_d ? d : a->max_d);
    }
    a->sum_null = 0;
}
static inline void acc_merge(or_acc* a, const or_acc* o, int vt) {   /* mergeExpressions */
    a->cnt_star = jadd(a->cnt_star, o->cnt_star);
    a->cnt_val = jadd(a->cnt_val, o->cnt_val);
    if (!o->sum_null) {
        if (vt == OR_VAL_I64) {
            a->sum_i = a->sum_null ? o->sum_i : jadd(a->sum_i, o->sum_i);
            a->min_i = a->sum_null ? o->min_i : (o->min_i < a->min_i ? o->min_i : a->min_i);
            a->max_i = a->sum_null ? o->max_i : (o->max_i > a->max_i ? o->max_i : a->max_i);
        } else {
            a->sum_d = a->sum_null ? o->sum_d : a->sum_d + o->sum_d;
            a->min_d = a->sum_null ? o->min_d : (o->min_d < a->min_d ? o->min_d : a->min_d);
            a->max_d = a->sum_null ? o->max_d : (o->max_d > a->max_d ? o->max_d : a->max_d);
        }
        a->sum_null = 0;
    }
    a->avg_sum_i = jadd(a->avg_sum_i, o->avg_sum_i);
    a->avg_sum_d = a->avg_sum_d + o->avg_sum_d;
}

/* ------------------------------------------------------------------------------------
 * Operator state
 * ---------------------------------------------------------------------------------- */
typedef struct { int64_t ts, seq, key, ns; } or_timer;

struct or_op {
    or_config cfg;
    /* derived assigner parameters */
    int64_t slice_size;      /* tumble: size, hop: gcd(size, slide), cumulate: step */
    int64_t num_slices;      /* hop: size / slice_size */
    int64_t interval;        /* getSliceEndInterval */
    /* processor (AbstractWindowAggProcessor) */
    int64_t current_progress, next_trigger_progress;
    /* RecordsWindowBuffer */
    int64_t min_slice_end;
    int64_t* merge_buf;                /* hop: numSlicesPerWindow slice ends */
    pmap buf_map;                      /* (slice, key) -> entry idx */
    int64_t* be_slice; int64_t* be_key; int64_t* be_head; int64_t* be_tail;
    int64_t be_n, be_cap;
    int64_t* br_val; uint8_t* br_null; int64_t* br_next;
    or_acc* br_acc;                    /* global phase: the buffered partial accumulators */
    int64_t br_n, br_cap;
    /* WindowValueState: (key, ns) -> acc idx */
    pmap state;
    or_acc* accs; int64_t acc_n, acc_cap; int64_t* acc_free; int64_t acc_free_n, acc_free_cap;
    /* InternalTimerServiceImpl */
    int64_t timer_wm;
    or_timer* heap; int64_t heap_n, heap_cap, seq;
    pmap timer_set;                    /* (key, ns) dedup (ts is a function of ns) */
    pmap cleanup_set;                  /* DataStream with allowed lateness: the (key, window) cleanup
                                        * timers at maxTimestamp + lateness (a second timer per window) */
    /* output */
    or_row* rows; int64_t rows_n, rows_cap;
    int64_t late_dropped;
};

/* ---------------- time utilities: TR/util/TimeWindowUtil.java ---------------------- */
/* TimeWindow.getWindowStartWithOffset  TR/operators/window/TimeWindow.java:222-224
 * (same formula: SJ/api/windowing/windows/TimeWindow.java:264-266) */
int64_t or_window_start_with_offset(int64_t ts, int64_t offset, int64_t size) {
    return jsub(ts, jmod(jadd(jsub(ts, offset), size), size));
}
/* ZoneRules.getOffset(Instant): the offset in force at an epoch instant (zone with
 * transitions: the offset after the last transition at or before it) */
static int64_t zone_offset_at(const or_op* op, int64_t instant) {
    int32_t lo = 0, hi = op->cfg.tz_n;   /* number of transitions <= instant */
    while (lo < hi) {
        int32_t mid = (lo + hi) / 2;
        if (op->cfg.tz_trans[mid] <= instant) lo = mid + 1;
        else hi = mid;
    }
    return op->cfg.tz_offs[lo];
}
/* LocalDateTime.atZone(zone).toInstant().toEpochMilli() (ZonedDateTime.ofLocal with no
 * preferred offset): the unique valid offset; in an overlap the earlier one (the offset
 * before the transition); in a gap the local time moves later by the gap length and takes
 * the offset after, i.e. epoch = local - offset before. */
static int64_t zone_local_to_epoch(const or_op* op, int64_t local) {
    const int64_t W = 20LL * 3600 * 1000;   /* |offset| <= 18 h */
    const int32_t n = op->cfg.tz_n;
    const int64_t* T = op->cfg.tz_trans;
    const int64_t* O = op->cfg.tz_offs;
    int32_t k = 0;   /* first offset region that may hold local - offset: transitions <= local - W */
    while (k < n && T[k] <= jsub(local, W)) k++;
    for (; k <= n; k++) {
        const int64_t e = jsub(local, O[k]);
        const int lo_ok = k == 0 || T[k - 1] <= e;
        const int hi_ok = k == n || e < T[k];
        if (lo_ok && hi_ok) return e;                 /* first valid = earlier offset */
        if (k < n && T[k] > jadd(local, W)) break;
        if (k < n && e >= T[k] && jsub(local, O[k + 1]) < T[k]) return e;   /* gap at transition k */
    }
    return jsub(local, O[n]);
}
/* toUtcTimestampMills  TimeWindowUtil.java:53-61 */
static inline int64_t to_utc(const or_op* op, int64_t epoch) {
    if (epoch == JMAX) return epoch;
    if (op->cfg.tz_n > 0) return jadd(epoch, zone_offset_at(op, epoch));
    if (op->cfg.tz_offset_ms == 0) return epoch;
    return jadd(epoch, op->cfg.tz_offset_ms);
}
/* toEpochMillsForTimer  TimeWindowUtil.java:70-140: DST zones take the first skipped
 * instant for a local time in a gap and the later instant for one in an overlap (:107-135);
 * zones without DST -> toEpochMills (:137-139) */
static inline int64_t to_epoch_for_timer(const or_op* op, int64_t utc) {
    if (utc == JMAX) return utc;
    if (op->cfg.tz_n > 0) {
        if (!op->cfg.tz_use_dst) return zone_local_to_epoch(op, utc);
        const int64_t HOUR = 3600LL * 1000;
        int64_t t1 = zone_local_to_epoch(op, utc);
        int64_t t2 = zone_local_to_epoch(op, jadd(utc, HOUR));
        if (t1 == t2) return jsub(t1, t1 % HOUR);      /* hasNoEpoch */
        if (jsub(t2, t1) > HOUR) return jadd(t1, HOUR); /* hasTwoEpochs */
        return t1;
    }
    if (op->cfg.tz_offset_ms == 0) return utc;
    return jsub(utc, op->cfg.tz_offset_ms);
}
/* isWindowFired  TimeWindowUtil.java:176-184 */
static inline int is_window_fired(const or_op* op, int64_t window_end, int64_t progress) {
    if (window_end == JMAX) return 0;
    return progress >= to_epoch_for_timer(op, jsub(window_end, 1));
}
/* getNextTriggerWatermark  TimeWindowUtil.java:187-210 (useDayLightSaving = false) */
int64_t or_next_trigger_watermark(int64_t wm, int64_t interval) {
    if (wm == JMAX) return wm;
    int64_t start = or_window_start_with_offset(wm, 0, interval);
    int64_t trig = jsub(jadd(start, interval), 1);
    return trig > wm ? trig : jadd(trig, interval);
}
/* the same with the operator's zone: the DST branch (:194-199) when useDayLightSaving */
static int64_t next_trigger(const or_op* op, int64_t wm) {
    if (!(op->cfg.tz_n > 0 && op->cfg.tz_use_dst)) return or_next_trigger_watermark(wm, op->interval);
    if (wm == JMAX) return wm;
    int64_t utc_start = or_window_start_with_offset(to_utc(op, wm), 0, op->interval);
    int64_t trig = to_epoch_for_timer(op, jsub(jadd(utc_start, op->interval), 1));
    return trig > wm ? trig : jadd(trig, op->interval);
}

int64_t or_to_utc(const or_op* op, int64_t epoch) { return to_utc(op, epoch); }
int64_t or_to_epoch_for_timer(const or_op* op, int64_t local) { return to_epoch_for_timer(op, local); }
/* toEpochMills  TimeWindowUtil.java:149-157 */
int64_t or_to_epoch(const or_op* op, int64_t local) {
    if (local == JMAX) return local;
    if (op->cfg.tz_n > 0) return zone_local_to_epoch(op, local);
    return jsub(local, op->cfg.tz_offset_ms);
}
int64_t or_next_trigger(const or_op* op, int64_t wm) { return next_trigger(op, wm); }

/* ---------------- SliceAssigners.java ---------------------------------------------- */
/* assignSliceEnd: Tumbling :164-167, Hopping :231-234, Cumulative :318-321, via
 * AbstractSliceAssigner.assignSliceEnd :551-561 (rowtime path) */
int64_t or_assign_slice_end(const or_op* op, int64_t ts) {
    /* WindowedSliceAssigner.assignSliceEnd :402-404: the attached window end, as is */
    if (op->cfg.windowed) return ts;
    int64_t t = to_utc(op, ts);
    return jadd(or_window_start_with_offset(t, op->cfg.offset, op->slice_size), op->slice_size);
}
/* getWindowStart: Tumbling :174-176, Hopping :242-244, Cumulative :330-332 */
int64_t or_get_window_start(const or_op* op, int64_t window_end) {
    if (op->cfg.kind == OR_CUMULATE)
        return or_window_start_with_offset(jsub(window_end, 1), op->cfg.offset, op->cfg.size);
    return jsub(window_end, op->cfg.size);
}
/* getLastWindowEnd: Tumbling :170-172, Hopping :237-239, Cumulative :324-327 */
int64_t or_get_last_window_end(const or_op* op, int64_t slice_end) {
    if (op->cfg.windowed) return slice_end;   /* WindowedSliceAssigner :407-412: the window itself */
    switch (op->cfg.kind) {
        case OR_TUMBLE: return slice_end;
        case OR_HOP: return jadd(jsub(slice_end, op->slice_size), op->cfg.size);
        default: return jadd(or_get_window_start(op, slice_end), op->cfg.size);
    }
}
/* expiredSlices: Tumbling :179-182, Hopping :247-253, Cumulative :335-351 */
int32_t or_expired_slices(const or_op* op, int64_t w, int64_t* out) {
    if (op->cfg.windowed) { out[0] = w; return 1; }   /* WindowedSliceAssigner :420-423 */
    switch (op->cfg.kind) {
        case OR_TUMBLE: out[0] = w; return 1;
        case OR_HOP: out[0] = jadd(or_get_window_start(op, w), op->slice_size); return 1;
        default: {
            int64_t ws = or_get_window_start(op, w);
            int64_t first = jadd(ws, op->slice_size), last = jadd(ws, op->cfg.size);
            if (w == first) return 0;
            if (w == last) { out[0] = w; out[1] = first; return 2; }
            out[0] = w; return 1;
        }
    }
}
/* mergeSlices: Hopping :261-267 (+HoppingSlicesIterable :617-648), Cumulative :359-370 */
int32_t or_merge_slices(const or_op* op, int64_t slice_end, int64_t* merge_result, int64_t* out, int32_t cap) {
    if (op->cfg.kind == OR_HOP) {
        *merge_result = JMIN;   /* null namespace: heap accumulator */
        int32_t n = 0;
        int64_t s = slice_end;
        for (int64_t i = 0; i < op->num_slices && n < cap; i++, s = jsub(s, op->slice_size)) out[n++] = s;
        return n;
    }
    if (op->cfg.kind == OR_CUMULATE) {
        int64_t first = jadd(or_get_window_start(op, slice_end), op->slice_size);
        *merge_result = first;
        if (slice_end == first) return 0;
        if (cap > 0) out[0] = slice_end;
        return 1;
    }
    *merge_result = JMIN;
    return 0;
}
/* nextTriggerWindow: Hopping :270-276, Cumulative :373-381 */
int32_t or_next_trigger_window(const or_op* op, int64_t w, int32_t is_empty, int64_t* next) {
    if (op->cfg.kind == OR_HOP) {
        if (is_empty) return 0;
        *next = jadd(w, op->slice_size);
        return 1;
    }
    if (op->cfg.kind == OR_CUMULATE) {
        int64_t nw = jadd(w, op->slice_size);
        int64_t maxw = jadd(or_get_window_start(op, w), op->cfg.size);
        if (nw > maxw) return 0;
        *next = nw;
        return 1;
    }
    return 0;
}
/* SliceSharedWindowAggProcessor.sliceStateMergeTarget :120-131 (+ helper :172-190) */
static int64_t slice_state_merge_target(const or_op* op, int64_t slice) {
    if (op->cfg.kind == OR_CUMULATE && !op->cfg.windowed) {
        int64_t mr, tmp[1];
        or_merge_slices(op, slice, &mr, tmp, 1);
        return mr;   /* never null for cumulate */
    }
    return slice;    /* tumble: SliceUnsharedWindowAggProcessor :56-59; hop: null -> itself */
}

/* ---------------- heap timers: InternalTimerServiceImpl + HeapPriorityQueueSet -------- */
static inline int tless(const or_timer* a, const or_timer* b) {
    /* TimerHeapInternalTimer.comparePriorityTo compares timestamps only (:131-133); ties
     * break by insertion sequence here (heap order in the reference: arbitrary). */
    return a->ts < b->ts || (a->ts == b->ts && a->seq < b->seq);
}
static void heap_push(or_op* op, or_timer t) {
    if (op->heap_n == op->heap_cap) {
        op->heap_cap = op->heap_cap ? op->heap_cap * 2 : 1024;
        op->heap = (or_timer*)realloc(op->heap, sizeof(or_timer) * op->heap_cap);
    }
    int64_t i = op->heap_n++;
    while (i > 0) {
        int64_t p = (i - 1) / 2;
        if (!tless(&t, &op->heap[p])) break;
        op->heap[i] = op->heap[p];
        i = p;
    }
    op->heap[i] = t;
}
static or_timer heap_pop(or_op* op) {
    or_timer top = op->heap[0], last = op->heap[--op->heap_n];
    int64_t i = 0, n = op->heap_n;
    for (;;) {
        int64_t l = 2 * i + 1, r = l + 1, m = i;
        const or_timer* best = &last;
        if (l < n && tless(&op->heap[l], best)) { m = l; best = &op->heap[l]; }
        if (r < n && tless(&op->heap[r], best)) { m = r; }
        if (m == i) break;
        op->heap[i] = op->heap[m];
        i = m;
    }
    if (n > 0) op->heap[i] = last;
    return top;
}
/* registerEventTimeTimer  InternalTimerServiceImpl.java (queue add with dedup) */
/* HeapPriorityQueueSet dedups timers by (timestamp, key, namespace) (TimerHeapInternalTimer
 * .equals): a window's trigger timer and its cleanup timer (WindowOperator.registerCleanupTimer
 * :630-642, at cleanupTime :669-673) are distinct timers when the allowed lateness is > 0 */
static int is_cleanup_timer(const or_op* op, int64_t ns, int64_t ts);
static void register_timer(or_op* op, int64_t key, int64_t ns, int64_t ts) {
    int ins;
    int64_t* v = pmap_upsert(is_cleanup_timer(op, ns, ts) ? &op->cleanup_set : &op->timer_set, key, ns, &ins);
    if (!ins) return;           /* HeapPriorityQueueSet.add: already contained */
    *v = ts;
    or_timer t = {ts, op->seq++, key, ns};
    heap_push(op, t);
}
/* WindowTimerServiceImpl.registerEventTimeWindowTimer  :60-63 */
static void register_window_timer(or_op* op, int64_t key, int64_t window) {
    register_timer(op, key, window, to_epoch_for_timer(op, jsub(window, 1)));
}

/* ---------------- state ------------------------------------------------------------ */
static or_acc* state_get(or_op* op, int64_t key, int64_t ns) {
    int64_t* v = pmap_find(&op->state, key, ns);
    return v ? &op->accs[*v] : NULL;
}
static or_acc* state_put(or_op* op, int64_t key, int64_t ns) {
    int ins;
    int64_t* v = pmap_upsert(&op->state, key, ns, &ins);
    if (ins) {
        int64_t idx;
        if (op->acc_free_n > 0) idx = op->acc_free[--op->acc_free_n];
        else {
            if (op->acc_n == op->acc_cap) {
                op->acc_cap = op->acc_cap ? op->acc_cap * 2 : 1024;
                op->accs = (or_acc*)realloc(op->accs, sizeof(or_acc) * op->acc_cap);
            }
            idx = op->acc_n++;
        }
        *v = idx;
        acc_create(&op->accs[idx]);
    }
    return &op->accs[*v];
}
static void state_clear(or_op* op, int64_t key, int64_t ns) {
    int64_t idx;
    if (!pmap_remove(&op->state, key, ns, &idx)) return;
    if (op->acc_free_n == op->acc_free_cap) {
        op->acc_free_cap = op->acc_free_cap ? op->acc_free_cap * 2 : 1024;
        op->acc_free = (int64_t*)realloc(op->acc_free, sizeof(int64_t) * op->acc_free_cap);
    }
    op->acc_free[op->acc_free_n++] = idx;
}

/* ---------------- output ----------------------------------------------------------- */
static void emit_row(or_op* op, int64_t key, int64_t wstart, int64_t wend, const or_acc* a, int64_t out_ts) {
    if (op->rows_n == op->rows_cap) {
        op->rows_cap = op->rows_cap ? op->rows_cap * 2 : 1024;
        op->rows = (or_row*)realloc(op->rows, sizeof(or_row) * op->rows_cap);
    }
    or_row* r = &op->rows[op->rows_n++];
    memset(r, 0, sizeof(*r));
    r->key = key;
    r->window_start = wstart;
    r->window_end = wend;
    r->cnt_star = a->cnt_star;
    r->cnt_val = a->cnt_val;
    r->sum_null = a->sum_null;
    r->sum_i = a->sum_i;
    r->sum_d = a->sum_d;
    /* AvgAggFunction.getValueExpression :98-103: count == 0 ? null : sum / count */
    r->avg_null = a->cnt_val == 0;
    if (!r->avg_null) {
        r->avg_i = (a->cnt_val == -1 && a->avg_sum_i == JMIN) ? JMIN : a->avg_sum_i / a->cnt_val;
        r->avg_d = a->avg_sum_d / (double)a->cnt_val;
    }
    r->sum0_i = a->avg_sum_i;   /* Sum0AggFunction.getValueExpression :85 */
    r->sum0_d = a->avg_sum_d;
    r->min_i = a->min_i;   /* Min/MaxAggFunction.getValueExpression: the accumulator (NULL iff sum_null) */
    r->max_i = a->max_i;
    r->min_d = a->min_d;
    r->max_d = a->max_d;
    r->out_ts = out_ts;
}

/* ---------------- RecordsWindowBuffer ---------------------------------------------- */
static void buffer_add_any(or_op* op, int64_t key, int64_t slice, int64_t vbits, uint8_t isnull, const or_acc* acc) {
    /* RecordsWindowBuffer.addElement :81-97 */
    if (slice < op->min_slice_end) op->min_slice_end = slice;
    int ins;
    int64_t* e = pmap_upsert(&op->buf_map, slice, key, &ins);
    if (op->br_n == op->br_cap) {
        op->br_cap = op->br_cap ? op->br_cap * 2 : 4096;
        op->br_val = (int64_t*)realloc(op->br_val, sizeof(int64_t) * op->br_cap);
        op->br_null = (uint8_t*)realloc(op->br_null, op->br_cap);
        op->br_next = (int64_t*)realloc(op->br_next, sizeof(int64_t) * op->br_cap);
        if (op->cfg.phase == OR_PHASE_GLOBAL) op->br_acc = (or_acc*)realloc(op->br_acc, sizeof(or_acc) * op->br_cap);
    }
    int64_t r = op->br_n++;
    op->br_val[r] = vbits;
    op->br_null[r] = isnull;
    op->br_next[r] = -1;
    if (acc) op->br_acc[r] = *acc;
    if (ins) {
        /* AbstractBytesMultiMap.append :145-184 -- new key, insertion order kept */
        if (op->be_n == op->be_cap) {
            op->be_cap = op->be_cap ? op->be_cap * 2 : 4096;
            op->be_slice = (int64_t*)realloc(op->be_slice, sizeof(int64_t) * op->be_cap);
            op->be_key = (int64_t*)realloc(op->be_key, sizeof(int64_t) * op->be_cap);
            op->be_head = (int64_t*)realloc(op->be_head, sizeof(int64_t) * op->be_cap);
            op->be_tail = (int64_t*)realloc(op->be_tail, sizeof(int64_t) * op->be_cap);
        }
        int64_t ei = op->be_n++;
        *e = ei;
        op->be_slice[ei] = slice;
        op->be_key[ei] = key;
        op->be_head[ei] = op->be_tail[ei] = r;
    } else {
        op->br_next[op->be_tail[*e]] = r;
        op->be_tail[*e] = r;
    }
}
static void buffer_add(or_op* op, int64_t key, int64_t slice, int64_t vbits, uint8_t isnull) {
    buffer_add_any(op, key, slice, vbits, isnull, NULL);
}
/* RecordsWindowBuffer.flush :108-119 + AggCombiner.combine  TR/operators/aggregate/window/combines/AggCombiner.java:76-115
 * (two-phase: LocalAggCombiner.combine  combines/LocalAggCombiner.java:69-106, GlobalAggCombiner.combine
 *  combines/GlobalAggCombiner.java:77-110) */
static void buffer_flush(or_op* op) {
    if (op->be_n == 0) return;
    int vt = op->cfg.val_type;
    for (int64_t ei = 0; ei < op->be_n; ei++) {
        int64_t key = op->be_key[ei], window = op->be_slice[ei];
        if (op->cfg.phase == OR_PHASE_LOCAL) {
            /* a fresh accumulator per (key, slice), emitted as (key, acc, slice end); no state */
            or_acc acc;
            acc_create(&acc);
            for (int64_t r = op->be_head[ei]; r >= 0; r = op->br_next[r])
                acc_accumulate(&acc, vt, op->br_val[r], op->br_null[r]);
            emit_row(op, key, jsub(window, op->slice_size), window, &acc, JMIN);
            continue;
        }
        or_acc* acc = state_put(op, key, window);        /* value(window) ?: createAccumulators */
        if (op->cfg.phase == OR_PHASE_GLOBAL) {
            /* localAggregator.merge of the partials into a fresh accumulator, then
             * globalAggregator.merge into the state (:94-101) */
            or_acc part;
            acc_create(&part);
            for (int64_t r = op->be_head[ei]; r >= 0; r = op->br_next[r]) acc_merge(&part, &op->br_acc[r], vt);
            acc_merge(acc, &part, vt);
        } else {
            for (int64_t r = op->be_head[ei]; r >= 0; r = op->br_next[r])
                acc_accumulate(acc, vt, op->br_val[r], op->br_null[r]);   /* arrival order */
        }
        if (!op->cfg.proctime && !is_window_fired(op, window, op->timer_wm))   /* step 5 (:101-110), event time */
            register_window_timer(op, key, window);
    }
    pmap_free(&op->buf_map);
    pmap_init(&op->buf_map, 1024);
    op->be_n = 0;
    op->br_n = 0;
    op->min_slice_end = JMAX;
}

/* ---------------- processors ------------------------------------------------------- */
/* AbstractWindowAggProcessor.processElement  TR/operators/aggregate/window/processors/AbstractWindowAggProcessor.java:135-165 */
static int sql_process_slice(or_op* op, int64_t key, int64_t slice_end, int64_t vbits, uint8_t isnull,
                             const or_acc* acc) {
    if (op->cfg.proctime) {
        /* :137-140 processing time: a timer per element at its slice, never late */
        register_window_timer(op, key, slice_end);
        buffer_add_any(op, key, slice_end, vbits, isnull, acc);
        return 0;
    }
    if (is_window_fired(op, slice_end, op->current_progress)) {
        int64_t last = or_get_last_window_end(op, slice_end);
        if (is_window_fired(op, last, op->current_progress)) return 1;   /* dropped */
        buffer_add_any(op, key, slice_state_merge_target(op, slice_end), vbits, isnull, acc);
        int64_t unfired = slice_end;
        while (is_window_fired(op, unfired, op->current_progress)) unfired = jadd(unfired, op->interval);
        register_window_timer(op, key, unfired);
        return 0;
    }
    buffer_add_any(op, key, slice_end, vbits, isnull, acc);
    return 0;
}
static int sql_process_element(or_op* op, int64_t key, int64_t ts, int64_t vbits, uint8_t isnull) {
    int64_t slice_end = or_assign_slice_end(op, ts);
    if (op->cfg.phase == OR_PHASE_LOCAL) {
        /* LocalSlicingWindowAggOperator.processElement :113-119: its own slice, no late handling */
        buffer_add(op, key, slice_end, vbits, isnull);
        return 0;
    }
    return sql_process_slice(op, key, slice_end, vbits, isnull, NULL);
}

/* fireWindow: SliceUnsharedWindowAggProcessor.java:46-54 / SliceSharedWindowAggProcessor.java:64-118;
 * clearWindow: AbstractWindowAggProcessor.java:200-206; via SlicingWindowOperator.onTimer :230-237 */
static void sql_on_timer(or_op* op, int64_t key, int64_t w) {
    int vt = op->cfg.val_type;
    int64_t wstart = or_get_window_start(op, w);   /* windowed: innerAssigner.getWindowStart :415-417 */
    if (op->cfg.kind == OR_TUMBLE || op->cfg.windowed) {   /* SliceUnsharedWindowAggProcessor */
        or_acc tmp;
        const or_acc* a = state_get(op, key, w);
        if (!a) { acc_create(&tmp); a = &tmp; }
        emit_row(op, key, wstart, w, a, JMIN);
    } else {
        int64_t mr, *list = op->merge_buf;
        int32_t nm = or_merge_slices(op, w, &mr, list, (int32_t)op->num_slices);
        or_acc acc;
        if (mr == JMIN) acc_create(&acc);
        else {
            const or_acc* s = state_get(op, key, mr);
            if (s) acc = *s; else acc_create(&acc);
        }
        for (int32_t i = 0; i < nm; i++) {
            const or_acc* s = state_get(op, key, list[i]);
            if (s) acc_merge(&acc, s, vt);
        }
        if (mr != JMIN) *state_put(op, key, mr) = acc;
        /* isWindowEmpty :120-127 + WindowIsEmptySupplier :133-170 */
        int empty = op->cfg.count_star_index >= 0 && acc.cnt_star == 0;
        if (!empty) emit_row(op, key, wstart, w, &acc, JMIN);
        int64_t next;
        if (or_next_trigger_window(op, w, empty, &next)) register_window_timer(op, key, next);
    }
    int64_t ex[2];
    int32_t ne = or_expired_slices(op, w, ex);
    for (int32_t i = 0; i < ne; i++) state_clear(op, key, ex[i]);
}

/* ---------------- DataStream WindowOperator  SJ/runtime/operators/windowing/WindowOperator.java ---- */
/* processElement :300,413-456 with TumblingEventTimeWindows.assignWindows
 * (SJ/api/windowing/assigners/TumblingEventTimeWindows.java:70-88) or
 * SlidingEventTimeWindows.assignWindows (:70-85); EventTimeTrigger.onElement :37-46;
 * HeapReducingState.add -> SumAggregator.reduce (SJ/api/functions/aggregation/SumAggregator.java:66-76) */
/* WindowOperator.cleanupTime :669-673: maxTimestamp + allowedLateness, Long.MAX_VALUE on overflow */
static int64_t ds_cleanup_time(const or_op* op, int64_t end) {
    int64_t max_ts = jsub(end, 1);
    int64_t c = jadd(max_ts, op->cfg.allowed_lateness);
    return c >= max_ts ? c : JMAX;
}
static int is_cleanup_timer(const or_op* op, int64_t ns, int64_t ts) {
    return op->cfg.mode == OR_MODE_DATASTREAM && op->cfg.allowed_lateness > 0 && ts == ds_cleanup_time(op, ns) &&
           ts != jsub(ns, 1);
}
/* WindowedStream.min / max (minBy / maxBy) on a DOUBLE field: ComparableAggregator.reduce
 * SJ/api/functions/aggregation/ComparableAggregator.java:83-104 with Comparator.java:48-137:
 * MIN keeps value1's field iff value1.compareTo(value2) < 0, else takes value2's (MAX: > 0),
 * Double.compareTo's total order (-0.0 < +0.0, NaN above +inf, every NaN equal: the
 * doubleToLongBits canonical form, which the result carries). BIGINT: Long.compareTo, the
 * primitive order acc_accumulate applies. HeapReducingState.add keeps the first element as is. */
static int64_t ds_canon(int64_t b) {
    return (b & INT64_MAX) > 0x7FF0000000000000ll ? 0x7FF8000000000000ll : b;
}
static int64_t ds_ord(int64_t b) { return b >= 0 ? b : b ^ INT64_MAX; }
static void ds_minmax_f64(or_acc* a, int64_t vbits, int first) {
    int64_t v = ds_canon(vbits), mn, mx;
    memcpy(&mn, &a->min_d, 8);
    memcpy(&mx, &a->max_d, 8);
    if (first || !(ds_ord(mn) < ds_ord(v))) mn = v;   /* c == 0: value1.field := value2.field */
    if (first || !(ds_ord(mx) > ds_ord(v))) mx = v;
    memcpy(&a->min_d, &mn, 8);
    memcpy(&a->max_d, &mx, 8);
}
static int ds_process_element(or_op* op, int64_t key, int64_t ts, int64_t vbits, uint8_t isnull) {
    (void)isnull;
    int64_t size = op->cfg.size;
    int64_t slide = op->cfg.kind == OR_TUMBLE ? size : op->cfg.slide;
    int skipped = 1;
    int64_t last_start = or_window_start_with_offset(ts, op->cfg.offset, slide);
    for (int64_t start = last_start; start > jsub(ts, size); start = jsub(start, slide)) {
        int64_t end = jadd(start, size);
        int64_t max_ts = jsub(end, 1);
        int64_t cleanup = ds_cleanup_time(op, end);
        if (cleanup <= op->timer_wm) continue;       /* isWindowLate :608-611 */
        skipped = 0;
        or_acc* a = state_put(op, key, end);         /* windowState.add -> SumAggregator.reduce */
        const int first = a->cnt_star == 0;
        acc_accumulate(a, op->cfg.val_type, vbits, 0);
        if (op->cfg.val_type == OR_VAL_F64) ds_minmax_f64(a, vbits, first);   /* ComparableAggregator */
        /* EventTimeTrigger.onElement :37-46 (PurgingTrigger.onElement: FIRE -> FIRE_AND_PURGE) */
        if (max_ts <= op->timer_wm) {
            emit_row(op, key, start, end, a, max_ts);  /* emitWindowContents :574-579 */
            if (op->cfg.purging) state_clear(op, key, end);
        } else {
            register_timer(op, key, end, max_ts);
        }
        if (cleanup != JMAX) register_timer(op, key, end, cleanup);   /* registerCleanupTimer :630-642 */
        if (op->cfg.kind == OR_TUMBLE) break;
    }
    /* :448-456: isSkippedElement && isElementLate (:620-622: timestamp + allowedLateness <= watermark) */
    return skipped && jadd(ts, op->cfg.allowed_lateness) <= op->timer_wm;
}
/* onEventTime :459-503: EventTimeTrigger.onEventTime FIREs at maxTimestamp (:49-51) ->
 * emitWindowContents :574-579 (timestamp = window.maxTimestamp()); PurgingTrigger purges;
 * at cleanupTime clearAllState :559-570 */
static void ds_on_timer(or_op* op, int64_t key, int64_t end, int64_t time) {
    int64_t max_ts = jsub(end, 1);
    if (time == max_ts) {
        const or_acc* a = state_get(op, key, end);
        if (a) emit_row(op, key, jsub(end, op->cfg.size), end, a, max_ts);
        if (op->cfg.purging) state_clear(op, key, end);
    }
    if (time == ds_cleanup_time(op, end)) state_clear(op, key, end);
}

/* ---------------- public API --------------------------------------------------------- */
static int64_t gcd64(int64_t a, int64_t b) {
    while (b) { int64_t t = a % b; a = b; b = t; }
    return a < 0 ? -a : a;
}

or_op* or_open(const or_config* cfg, char* err, int errlen) {
    char buf[512];
    buf[0] = 0;
    int64_t size = cfg->size, slide = cfg->slide, off = cfg->offset;
    if (cfg->kind == OR_TUMBLE) {
        /* SliceAssigners.java:149-158 */
        if (!(size > 0))
            snprintf(buf, sizeof buf, "Tumbling Window parameters must satisfy size > 0, but got size %lldms.", (long long)size);
        else if (!((off < 0 ? -off : off) < size))
            snprintf(buf, sizeof buf,
                     "Tumbling Window parameters must satisfy abs(offset) < size, bot got size %lldms and offset %lldms.",
                     (long long)size, (long long)off);
    } else if (cfg->kind == OR_HOP) {
        /* SliceAssigners.java:211-222; SliceSharedWindowAggProcessor.java:138-142 */
        if (size <= 0 || slide <= 0)
            snprintf(buf, sizeof buf,
                     "Hopping Window must satisfy slide > 0 and size > 0, but got slide %lldms and size %lldms.",
                     (long long)slide, (long long)size);
        else if (size % slide != 0)
            snprintf(buf, sizeof buf,
                     "Slicing Hopping Window requires size must be an integral multiple of slide, but got size %lldms and slide %lldms.",
                     (long long)size, (long long)slide);
        else if (cfg->mode == OR_MODE_SQL && cfg->count_star_index < 0 && !cfg->windowed)
            snprintf(buf, sizeof buf, "Hopping window requires a COUNT(*) in the aggregate functions.");
    } else if (cfg->kind == OR_CUMULATE) {
        /* SliceAssigners.java:299-310 */
        if (size <= 0 || slide <= 0)
            snprintf(buf, sizeof buf,
                     "Cumulative Window parameters must satisfy maxSize > 0 and step > 0, but got maxSize %lldms and step %lldms.",
                     (long long)size, (long long)slide);
        else if (size % slide != 0)
            snprintf(buf, sizeof buf,
                     "Cumulative Window requires maxSize must be an integral multiple of step, but got maxSize %lldms and step %lldms.",
                     (long long)size, (long long)slide);
        else if (cfg->mode == OR_MODE_DATASTREAM)
            snprintf(buf, sizeof buf, "DataStream has no cumulative window assigner.");
    } else {
        snprintf(buf, sizeof buf, "unknown window kind %d", cfg->kind);
    }
    if (!buf[0] && cfg->phase != OR_PHASE_SINGLE &&
        (cfg->mode != OR_MODE_SQL || cfg->windowed || cfg->proctime || cfg->phase > OR_PHASE_GLOBAL))
        snprintf(buf, sizeof buf, "the two-phase operators are SQL event-time operators");
    if (!buf[0] && cfg->allowed_lateness < 0)   /* WindowOperatorBuilder.allowedLateness :128 */
        snprintf(buf, sizeof buf, "The allowed lateness cannot be negative.");
    if (!buf[0] && (cfg->allowed_lateness > 0 || cfg->purging) && cfg->mode != OR_MODE_DATASTREAM)
        snprintf(buf, sizeof buf, "allowed lateness and triggers are DataStream WindowOperator settings");
    if (!buf[0] && cfg->windowed && (cfg->mode != OR_MODE_SQL || cfg->proctime))
        /* WindowedSliceAssigner.isEventTime() is always true (:430-434); SQL only */
        snprintf(buf, sizeof buf, "a windowed slice assigner is an SQL event-time assigner");
    if (buf[0]) {
        if (err && errlen > 0) { strncpy(err, buf, (size_t)errlen - 1); err[errlen - 1] = 0; }
        return NULL;
    }
    or_op* op = (or_op*)calloc(1, sizeof(or_op));
    op->cfg = *cfg;
    if (cfg->tz_n > 0) {   /* the operator keeps its own copy of the zone rules */
        int64_t* tr = (int64_t*)malloc(sizeof(int64_t) * (size_t)cfg->tz_n);
        int64_t* of = (int64_t*)malloc(sizeof(int64_t) * (size_t)(cfg->tz_n + 1));
        memcpy(tr, cfg->tz_trans, sizeof(int64_t) * (size_t)cfg->tz_n);
        memcpy(of, cfg->tz_offs, sizeof(int64_t) * (size_t)(cfg->tz_n + 1));
        op->cfg.tz_trans = tr;
        op->cfg.tz_offs = of;
    } else {
        op->cfg.tz_n = 0;
        op->cfg.tz_trans = op->cfg.tz_offs = NULL;
    }
    switch (cfg->kind) {
        case OR_TUMBLE: op->slice_size = size; op->num_slices = 1; break;
        case OR_HOP: op->slice_size = gcd64(size, slide); op->num_slices = size / op->slice_size; break;
        default: op->slice_size = slide; op->num_slices = 1; break;
    }
    op->interval = op->slice_size;
    op->merge_buf = (int64_t*)malloc(sizeof(int64_t) * (size_t)(op->num_slices + 1));
    op->current_progress = JMIN;
    op->next_trigger_progress = JMIN;
    op->min_slice_end = JMAX;
    op->timer_wm = JMIN;
    pmap_init(&op->buf_map, 1024);
    pmap_init(&op->state, 1024);
    pmap_init(&op->timer_set, 1024);
    pmap_init(&op->cleanup_set, 1024);
    return op;
}

void or_close(or_op* op) {
    if (!op) return;
    pmap_free(&op->buf_map); pmap_free(&op->state); pmap_free(&op->timer_set); pmap_free(&op->cleanup_set);
    free(op->be_slice); free(op->be_key); free(op->be_head); free(op->be_tail);
    free(op->br_val); free(op->br_null); free(op->br_next); free(op->br_acc);
    free(op->accs); free(op->acc_free); free(op->heap); free(op->rows); free(op->merge_buf);
    free((void*)op->cfg.tz_trans); free((void*)op->cfg.tz_offs);
    free(op);
}

void or_process_batch(or_op* op, int64_t n, const int64_t* key, const int64_t* ts, const void* val,
                      const uint8_t* isnull) {
    const int64_t* v = (const int64_t*)val;   /* bit pattern; f64 reinterpreted in acc_accumulate */
    for (int64_t i = 0; i < n; i++) {
        int64_t vb = v ? v[i] : 0;
        uint8_t nl = isnull ? isnull[i] : 0;
        int dropped = op->cfg.mode == OR_MODE_SQL ? sql_process_element(op, key[i], ts[i], vb, nl)
                                                  : ds_process_element(op, key[i], ts[i], vb, nl);
        op->late_dropped += dropped;   /* numLateRecordsDropped (SlicingWindowOperator.java:196-204) */
    }
}

/* The global phase's input: the `sliced` assigner takes each partial row's slice end
 * (SliceAssigners.java:494-533); late rules, buffer and timers as for records; the
 * combiner merges accumulators (GlobalAggCombiner). A late row counts once. */
void or_process_partials(or_op* op, int64_t n, const or_row* rows) {
    for (int64_t i = 0; i < n; i++) {
        const or_row* r = &rows[i];
        or_acc a;
        acc_create(&a);
        a.cnt_star = r->cnt_star;
        a.cnt_val = r->cnt_val;
        a.sum_null = r->sum_null;
        a.sum_i = r->sum_i;
        a.sum_d = r->sum_d;
        a.avg_sum_i = r->sum0_i;
        a.avg_sum_d = r->sum0_d;
        a.min_i = r->min_i;
        a.max_i = r->max_i;
        a.min_d = r->min_d;
        a.max_d = r->max_d;
        op->late_dropped += sql_process_slice(op, r->key, r->window_end, 0, 0, &a);
    }
}

void or_process_watermark(or_op* op, int64_t wm) {
    if (op->cfg.phase == OR_PHASE_LOCAL) {
        /* LocalSlicingWindowAggOperator.processWatermark :121-134 (no timers) */
        if (wm > op->current_progress) {
            op->current_progress = wm;
            if (op->current_progress >= op->next_trigger_progress) {
                if (is_window_fired(op, op->min_slice_end, wm)) buffer_flush(op);   /* advanceProgress */
                op->next_trigger_progress = next_trigger(op, wm);
            }
        }
        op->timer_wm = wm;
        return;
    }
    if (op->cfg.mode == OR_MODE_SQL) {
        /* SlicingWindowOperator.processWatermark :207-210 -> AbstractWindowAggProcessor.advanceProgress :178-192 */
        if (wm > op->current_progress) {
            op->current_progress = wm;
            if (op->current_progress >= op->next_trigger_progress) {
                /* RecordsWindowBuffer.advanceProgress :100-105 */
                if (is_window_fired(op, op->min_slice_end, wm)) buffer_flush(op);
                op->next_trigger_progress = next_trigger(op, wm);
            }
        }
    }
    /* AbstractStreamOperator.processWatermark -> InternalTimerServiceImpl.advanceWatermark :294-304 */
    op->timer_wm = wm;
    while (op->heap_n > 0 && op->heap[0].ts <= wm) {
        or_timer t = heap_pop(op);
        pmap_remove(is_cleanup_timer(op, t.ns, t.ts) ? &op->cleanup_set : &op->timer_set, t.key, t.ns, NULL);
        if (op->cfg.mode == OR_MODE_SQL) sql_on_timer(op, t.key, t.ns);
        else ds_on_timer(op, t.key, t.ns, t.ts);
    }
}

void or_prepare_snapshot(or_op* op) {
    /* SlicingWindowOperator.prepareSnapshotPreBarrier :240-242 -> prepareCheckpoint :195-197 */
    if (op->cfg.mode == OR_MODE_SQL) buffer_flush(op);
}

or_op* or_restore_copy(const or_op* src) {
    char err[256];
    or_op* op = or_open(&src->cfg, err, sizeof err);
    /* keyed state (heap backend snapshot) */
    for (int64_t i = 0; i < src->state.cap; i++) {
        if (!src->state.used[i]) continue;
        *state_put(op, src->state.ka[i], src->state.kb[i]) = src->accs[src->state.v[i]];
    }
    /* timers (raw keyed state), replayed in heap order */
    for (int64_t i = 0; i < src->heap_n; i++) {
        const or_timer* t = &src->heap[i];
        register_timer(op, t->key, t->ns, t->ts);
    }
    return op;   /* progress, next trigger and timer watermark back at Long.MIN_VALUE */
}

/* DataStream WindowOperator keyed state as its heap backend holds it: "window-contents" (one
 * reduced value per (key, TimeWindow), WindowOperatorBuilder.java:71,165-167) and the
 * "window-timers" queue (WindowOperator.java:225; trigger timers at maxTimestamp, cleanup timers
 * at maxTimestamp + allowedLateness, :630-642). or_ds_export_state writes per entry the key, the
 * window end, COUNT(*) and the SUM / MIN / MAX bits of the value field (i64, or f64 bits); the
 * arrays hold or_state_entries() entries. or_export_timers: or_pending_timers() timers. */
int64_t or_ds_export_state(const or_op* op, int64_t* key, int64_t* end, int64_t* cnt, int64_t* sum, int64_t* mn,
                           int64_t* mx) {
    int64_t j = 0;
    const int f = op->cfg.val_type == OR_VAL_F64;
    for (int64_t i = 0; i < op->state.cap; i++) {
        if (!op->state.used[i]) continue;
        const or_acc* a = &op->accs[op->state.v[i]];
        key[j] = op->state.ka[i];
        end[j] = op->state.kb[i];
        cnt[j] = a->cnt_star;
        if (f) {
            memcpy(&sum[j], &a->sum_d, 8);
            memcpy(&mn[j], &a->min_d, 8);
            memcpy(&mx[j], &a->max_d, 8);
        } else {
            sum[j] = a->sum_i;
            mn[j] = a->min_i;
            mx[j] = a->max_i;
        }
        j++;
    }
    return j;
}
int64_t or_export_timers(const or_op* op, int64_t* key, int64_t* ns, int64_t* ts) {
    for (int64_t i = 0; i < op->heap_n; i++) {
        key[i] = op->heap[i].key;
        ns[i] = op->heap[i].ns;
        ts[i] = op->heap[i].ts;
    }
    return op->heap_n;
}
/* A DataStream operator restored from such an image (initializeState of the heap backend): the
 * reduced value of each (key, window) is all a reduce keeps -- its COUNT(*) is taken as 1 (never
 * emitted by a DataStream reduce) unless `cnt` gives it (an aggregate function's accumulator
 * with a count: COUNT, AVG); the timers are registered as they were. The
 * timer watermark restarts at Long.MIN_VALUE (InternalTimerServiceImpl). */
or_op* or_ds_import(const or_config* cfg, int64_t n, const int64_t* key, const int64_t* end, const int64_t* val,
                    const int64_t* cnt, int64_t nt, const int64_t* tkey, const int64_t* tns, const int64_t* tts,
                    char* err, int errlen) {
    or_op* op = or_open(cfg, err, errlen);
    if (!op) return NULL;
    const int f = cfg->val_type == OR_VAL_F64;
    for (int64_t i = 0; i < n; i++) {
        or_acc* a = state_put(op, key[i], end[i]);
        a->cnt_star = cnt ? cnt[i] : 1;   /* (an AggregateFunction's accumulator may hold its count) */
        a->cnt_val = a->cnt_star;
        a->sum_null = 0;
        if (f) {
            memcpy(&a->sum_d, &val[i], 8);
            memcpy(&a->min_d, &val[i], 8);
            memcpy(&a->max_d, &val[i], 8);
        } else {
            a->sum_i = a->min_i = a->max_i = val[i];
        }
    }
    for (int64_t i = 0; i < nt; i++) register_timer(op, tkey[i], tns[i], tts[i]);
    return op;
}

int64_t or_num_rows(const or_op* op) { return op->rows_n; }
const or_row* or_rows(const or_op* op) { return op->rows; }
void or_clear_rows(or_op* op) { op->rows_n = 0; }
int64_t or_late_dropped(const or_op* op) { return op->late_dropped; }
int64_t or_state_entries(const or_op* op) { return op->state.n; }
int64_t or_pending_timers(const or_op* op) { return op->heap_n; }

/* ---------------- key groups -------------------------------------------------------- */
/* MurmurHashUtils  TC/binary/MurmurHashUtils.java:30-32, mixK1/mixH1/fmix */
static inline int32_t mix_k1(int32_t k1) {
    k1 = imul(k1, (int32_t)0xcc9e2d51);
    k1 = rotl32(k1, 15);
    return imul(k1, 0x1b873593);
}
static inline int32_t mix_h1(int32_t h1, int32_t k1) {
    h1 ^= k1;
    h1 = rotl32(h1, 13);
    return iadd(imul(h1, 5), (int32_t)0xe6546b64);
}
static inline int32_t fmix32(int32_t h) {
    uint32_t u = (uint32_t)h;
    u ^= u >> 16; u *= 0x85ebca6bU; u ^= u >> 13; u *= 0xc2b2ae35U; u ^= u >> 16;
    return (int32_t)u;
}
/* BinarySection.hashCode TC/binary/BinarySection.java:76-78 -> BinarySegmentUtils.hash :395-400
 * -> MurmurHashUtils.hashBytes(seg, off, 16, seed 42). The key row of one BIGINT is
 * [rowkind=0][null bits=0] (8 B) + the i64 little-endian (BinaryRowData.java:68-76,121-123). */
int32_t or_binaryrow_hash_i64(int64_t key) {
    int32_t h1 = 42;
    h1 = mix_h1(h1, mix_k1(0));
    h1 = mix_h1(h1, mix_k1(0));
    h1 = mix_h1(h1, mix_k1((int32_t)(uint32_t)((uint64_t)key & 0xffffffffu)));
    h1 = mix_h1(h1, mix_k1((int32_t)(uint32_t)((uint64_t)key >> 32)));
    return fmix32(h1 ^ 16);
}
/* BinarySection.hashCode of any row (TC/data/binary/BinarySection.java:76-78 ->
 * BinarySegmentUtils.hash -> MurmurHashUtils.hashBytesByWords, MurmurHashUtils.java:92-96,
 * 131-141): the row's little-endian 4-byte words (MemorySegment.getInt, native order), seed 42,
 * fmix(h1 ^ length); len % 4 == 0 (BinaryRowData sizes are multiples of 8) */
int32_t or_binaryrow_hash_bytes(const uint8_t* row, int32_t len) {
    int32_t h1 = 42;
    for (int32_t i = 0; i < len; i += 4) {
        const uint32_t w = (uint32_t)row[i] | (uint32_t)row[i + 1] << 8 | (uint32_t)row[i + 2] << 16 |
                           (uint32_t)row[i + 3] << 24;
        h1 = mix_h1(h1, mix_k1((int32_t)w));
    }
    return fmix32(h1 ^ len);
}
int32_t or_long_hash(int64_t key) { return (int32_t)(uint32_t)((uint64_t)key ^ ((uint64_t)key >> 32)); }
/* MathUtils.murmurHash  CO/util/MathUtils.java:137-155 */
int32_t or_murmur_hash(int32_t code) {
    code = imul(code, (int32_t)0xcc9e2d51);
    code = rotl32(code, 15);
    code = imul(code, 0x1b873593);
    code = rotl32(code, 13);
    code = iadd(imul(code, 5), (int32_t)0xe6546b64);
    code ^= 4;
    code = fmix32(code);   /* bitMix :194-201 */
    if (code >= 0) return code;
    if (code != INT32_MIN) return -code;
    return 0;
}
/* KeyGroupRangeAssignment.computeKeyGroupForKeyHash  RT/state/KeyGroupRangeAssignment.java:74-77 */
int32_t or_key_group(int32_t key_hash, int32_t max_p) { return or_murmur_hash(key_hash) % max_p; }
/* computeOperatorIndexForKeyGroup :124-127 */
int32_t or_operator_index(int32_t max_p, int32_t p, int32_t kg) { return kg * p / max_p; }
/* computeDefaultMaxParallelism :137-147 */
int32_t or_default_max_parallelism(int32_t p) {
    int32_t x = p + p / 2 - 1;
    x |= x >> 1; x |= x >> 2; x |= x >> 4; x |= x >> 8; x |= x >> 16;
    x += 1;
    if (x < 128) x = 128;
    if (x > 32768) x = 32768;
    return x;
}
void or_key_groups_binaryrow(int64_t n, const int64_t* key, int32_t max_p, int32_t* out) {
    for (int64_t i = 0; i < n; i++) out[i] = or_key_group(or_binaryrow_hash_i64(key[i]), max_p);
}

/* ---------------- CPU baseline: one operator instance per core --------------------- */
typedef struct {
    const or_config* cfg;
    int64_t n;
    int64_t* key; int64_t* ts; int64_t* val; int64_t* gidx;   /* records routed to this instance */
    int32_t n_wm; const int64_t* wm_at; const int64_t* wm_val;
    int64_t rows; uint64_t checksum; int64_t late;
    int keep_rows; int32_t snapshot_after;          /* or_run_partitioned_rows */
    or_row* out; int64_t out_n, out_cap;
} part_job;

static uint64_t row_digest(const or_row* r) {
    uint64_t h = mix64((uint64_t)r->key ^ mix64((uint64_t)r->window_end));
    h ^= mix64((uint64_t)r->cnt_star + 0x1234567ULL);
    return h;
}

static void* part_worker(void* arg) {
    part_job* j = (part_job*)arg;
    char err[256];
    or_op* op = or_open(j->cfg, err, sizeof err);
    int64_t i = 0;
    for (int32_t w = 0; w <= j->n_wm; w++) {
        int64_t upto = w < j->n_wm ? j->wm_at[w] : INT64_MAX;   /* global record index bound */
        int64_t s = i;
        while (i < j->n && j->gidx[i] < upto) i++;
        if (i > s) or_process_batch(op, i - s, j->key + s, j->ts + s, j->val ? j->val + s : NULL, NULL);
        if (w < j->n_wm) or_process_watermark(op, j->wm_val[w]);
        for (int64_t r = 0; r < op->rows_n; r++) j->checksum += row_digest(&op->rows[r]);
        if (j->keep_rows && op->rows_n > 0) {
            if (j->out_n + op->rows_n > j->out_cap) {
                j->out_cap = 2 * (j->out_n + op->rows_n);
                j->out = (or_row*)realloc(j->out, sizeof(or_row) * (size_t)j->out_cap);
            }
            memcpy(j->out + j->out_n, op->rows, sizeof(or_row) * (size_t)op->rows_n);
            j->out_n += op->rows_n;
        }
        j->rows += op->rows_n;
        op->rows_n = 0;
        if (w == j->snapshot_after) {   /* checkpoint + failover: continue as the restored copy */
            or_prepare_snapshot(op);
            or_op* r = or_restore_copy(op);
            j->late += op->late_dropped;
            or_close(op);
            op = r;
        }
    }
    j->late += op->late_dropped;
    or_close(op);
    return NULL;
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static double run_partitioned(const or_config* cfg, int32_t P, int32_t max_p, int64_t n, const int64_t* key,
                              const int64_t* ts, const void* val, int32_t n_wm, const int64_t* wm_at,
                              const int64_t* wm_val, int64_t* rows_out, uint64_t* checksum, int64_t* late_out,
                              int keep_rows, int32_t snapshot_after, or_row** rows_kept) {
    /* keyBy routing: KeyGroupStreamPartitioner.selectChannel (SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:55-65) */
    int32_t* dest = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int64_t* cnt = (int64_t*)calloc((size_t)P, sizeof(int64_t));
    for (int64_t i = 0; i < n; i++) {
        int32_t h = cfg->mode == OR_MODE_SQL ? or_binaryrow_hash_i64(key[i]) : or_long_hash(key[i]);
        dest[i] = or_operator_index(max_p, P, or_key_group(h, max_p));
        cnt[dest[i]]++;
    }
    part_job* jobs = (part_job*)calloc((size_t)P, sizeof(part_job));
    const int64_t* v = (const int64_t*)val;
    for (int32_t p = 0; p < P; p++) {
        jobs[p].cfg = cfg;
        jobs[p].key = (int64_t*)malloc(sizeof(int64_t) * (size_t)(cnt[p] + 1));
        jobs[p].ts = (int64_t*)malloc(sizeof(int64_t) * (size_t)(cnt[p] + 1));
        jobs[p].val = v ? (int64_t*)malloc(sizeof(int64_t) * (size_t)(cnt[p] + 1)) : NULL;
        jobs[p].gidx = (int64_t*)malloc(sizeof(int64_t) * (size_t)(cnt[p] + 1));
        jobs[p].n_wm = n_wm; jobs[p].wm_at = wm_at; jobs[p].wm_val = wm_val;
        jobs[p].keep_rows = keep_rows; jobs[p].snapshot_after = snapshot_after;
    }
    for (int64_t i = 0; i < n; i++) {
        part_job* j = &jobs[dest[i]];
        j->key[j->n] = key[i];
        j->ts[j->n] = ts[i];
        if (v) j->val[j->n] = v[i];
        j->gidx[j->n] = i;
        j->n++;
    }
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)P);
    double t0 = now_s();
    for (int32_t p = 0; p < P; p++) pthread_create(&th[p], NULL, part_worker, &jobs[p]);
    for (int32_t p = 0; p < P; p++) pthread_join(th[p], NULL);
    double el = now_s() - t0;
    int64_t rows = 0, late = 0;
    uint64_t cs = 0;
    for (int32_t p = 0; p < P; p++) {
        rows += jobs[p].rows; cs += jobs[p].checksum; late += jobs[p].late;
        free(jobs[p].key); free(jobs[p].ts); free(jobs[p].val); free(jobs[p].gidx);
    }
    if (keep_rows) {
        or_row* all = (or_row*)malloc(sizeof(or_row) * (size_t)(rows > 0 ? rows : 1));
        int64_t at = 0;
        for (int32_t p = 0; p < P; p++) {
            if (jobs[p].out_n) memcpy(all + at, jobs[p].out, sizeof(or_row) * (size_t)jobs[p].out_n);
            at += jobs[p].out_n;
            free(jobs[p].out);
        }
        *rows_kept = all;
    }
    *rows_out = rows; *checksum = cs; *late_out = late;
    free(th); free(jobs); free(cnt); free(dest);
    return el;
}

double or_run_partitioned(const or_config* cfg, int32_t P, int32_t max_p, int64_t n, const int64_t* key,
                          const int64_t* ts, const void* val, int32_t n_wm, const int64_t* wm_at,
                          const int64_t* wm_val, int64_t* rows_out, uint64_t* checksum, int64_t* late_out) {
    return run_partitioned(cfg, P, max_p, n, key, ts, val, n_wm, wm_at, wm_val, rows_out, checksum, late_out, 0, -1,
                           NULL);
}

double or_run_partitioned_rows(const or_config* cfg, int32_t P, int32_t max_p, int64_t n, const int64_t* key,
                               const int64_t* ts, const void* val, int32_t n_wm, const int64_t* wm_at,
                               const int64_t* wm_val, int32_t snapshot_after, or_row** rows, int64_t* n_rows,
                               int64_t* late_out) {
    uint64_t cs = 0;
    return run_partitioned(cfg, P, max_p, n, key, ts, val, n_wm, wm_at, wm_val, n_rows, &cs, late_out, 1,
                           snapshot_after, rows);
}

void or_free(void* p) { free(p); }
