// fg_late.h -- launch interface of the allowed-lateness kernels (fg_late.hip), internal to
// libflinkgpu.so. DataStream WindowOperator semantics (WindowOperator.java:608-681,
// EventTimeTrigger.java:37-51), with window = the engine's slices (tumbling: one slice;
// sliding: size / slide slices, slice = slide).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fg_kernels.h"
#include "fg_window.h"

namespace fg {

// window.maxTimestamp() <= watermark: the window's trigger timer fired (EventTimeTrigger)
__host__ __device__ __forceinline__ bool ds_fired(int64_t window_end, int64_t wm) {
    return window_end != JMAX && jsub(window_end, 1) <= wm;
}
// WindowOperator.cleanupTime (:669-673): maxTimestamp + allowedLateness, Long.MAX_VALUE on overflow
__host__ __device__ __forceinline__ int64_t ds_cleanup(int64_t window_end, int64_t lateness) {
    const int64_t max_ts = jsub(window_end, 1);
    const int64_t c = jadd(max_ts, lateness);
    return c >= max_ts ? c : JMAX;
}

struct LateClass {
    int64_t slice_end;
    bool late_allowed;   // some window of the element fired and is not cleaned: it FIREs at once
    bool last_fired;     // every window of the element fired (so none takes it later)
};
// The windows of an element are those holding its slice s: ends s, s + slide, ..,
// s - slide + size (TumblingEventTimeWindows / SlidingEventTimeWindows.assignWindows). The fired
// ones are the first few; the element is late-allowed iff the latest fired one is not cleaned
// (cleanup times grow with the window end). Elements that are not late-allowed see only
// unfired or cleaned windows: the regular ingest (drop iff the last window fired) then applies
// isWindowLate to each (:608-611).
__host__ __device__ __forceinline__ LateClass late_class(const WindowSpec& w, int64_t ts, int64_t wm,
                                                         int64_t lateness) {
    LateClass c{};
    c.slice_end = assign_slice_end(w, ts);
    const int64_t slide = w.kind == TUMBLE ? w.size : w.slide;
    const int64_t first = c.slice_end;
    const int64_t nwin = w.kind == TUMBLE ? 1 : w.size / slide;
    const int64_t last = jadd(first, (nwin - 1) * slide);
    c.last_fired = ds_fired(last, wm);
    if (!ds_fired(first, wm)) return c;
    int64_t ef = last;
    if (!c.last_fired) {
        const uint64_t k = (uint64_t)jsub(wm, jsub(first, 1)) / (uint64_t)slide;   // windows fired - 1
        ef = jadd(first, (int64_t)k * slide);
    }
    c.late_allowed = ds_cleanup(ef, lateness) > wm;
    return c;
}

struct LateSplit {
    WindowSpec w;
    int64_t wm;
    int64_t lateness;
    int32_t purging;
    int32_t pad;
    int64_t n;
    const int64_t* key;
    const int64_t* ts;
    const int64_t* val;
    const uint8_t* vnull;
    unsigned long long* counts;   // [0] late, [1] regular
    // late list
    int64_t* l_mix;
    int64_t* l_se;
    int64_t* l_val;
    uint8_t* l_null;
    uint32_t* l_idx;
    // regular remainder (the order does not matter: the merge is order-free)
    int64_t* r_key;
    int64_t* r_ts;
    int64_t* r_val;
    uint8_t* r_null;
};

struct LateDir {           // slice tables of the late path, sorted by slice end
    const int64_t* se;
    const TableRef* t;
    int32_t n;
    int32_t pad;
};

struct LateRound {
    WindowSpec w;
    int64_t wm;
    int64_t lateness;
    int32_t purging;
    int32_t vt;                 // value type (1 i64, 2 f64)
    int32_t region_bits;
    int32_t P;
    int32_t cap, cols;          // table region capacity and 8-byte words per entry
    int64_t n;                  // late elements
    const int64_t* mix;
    const int64_t* se;
    const int64_t* val;
    const uint8_t* vnull;
    const uint32_t* idx;        // arrival index in the batch
    uint8_t* done;
    uint8_t* sel;               // selected in this round (one per key)
    uint32_t* slot;             // claim-table slot of the element's key
    int32_t* found;             // entry of (key, slice) in the slice table, -1 new
    unsigned long long* claim_key;   // [claim_mask + 2]
    uint32_t* claim_idx;
    uint64_t claim_mask;
    uint32_t* need;             // [dir.n * P] new entries per (table, region)
    unsigned int* flags;        // bit0 region full, bit1 missing table, bit2 output overflow
    unsigned long long* nsel;   // elements selected in this round
    LateDir dir;
    // rows
    int32_t num_aggs;
    int32_t aggs[kMaxAggs];
    int64_t* out_key;
    int64_t* out_ws;
    int64_t* out_we;
    int64_t* out_agg[kMaxAggs];
    uint8_t* out_null;
    int64_t* out_rowtime;
    unsigned long long* out_count;
    int64_t out_cap;
};

hipError_t launch_late_split(const LateSplit& p, hipStream_t s);
hipError_t launch_late_reset(const LateRound& p, hipStream_t s);   // claim table, flags, nsel
hipError_t launch_late_claim(const LateRound& p, hipStream_t s);
hipError_t launch_late_lookup(const LateRound& p, hipStream_t s);
hipError_t launch_late_update(const LateRound& p, hipStream_t s);
hipError_t launch_late_emit(const LateRound& p, hipStream_t s);

}  // namespace fg
