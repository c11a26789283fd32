// fg_window.h -- window / slice arithmetic shared by the HIP kernels and the host engine.
//
// Restates the reference's slice assigners and time utilities for the event-time path
// (UTC, a fixed-offset shift time zone, or a zone with transitions / daylight saving given
// as its rules). Java long arithmetic wraps, so every add/sub goes through unsigned
// arithmetic.
//   TimeWindow.getWindowStartWithOffset  TR/operators/window/TimeWindow.java:222-224
//   TimeWindowUtil.toUtcTimestampMills / toEpochMillsForTimer / isWindowFired /
//     getNextTriggerWatermark            TR/util/TimeWindowUtil.java:53-61,137-139,176-210
//   SliceAssigners (Tumbling/Hopping/Cumulative)  TR/operators/window/slicing/SliceAssigners.java:133-382
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fg {

constexpr int64_t JMAX = INT64_MAX;
constexpr int64_t JMIN = INT64_MIN;

enum : int { TUMBLE = 0, HOP = 1, CUMULATE = 2 };

__host__ __device__ __forceinline__ int64_t jadd(int64_t a, int64_t b) {
    return (int64_t)((uint64_t)a + (uint64_t)b);
}
__host__ __device__ __forceinline__ int64_t jsub(int64_t a, int64_t b) {
    return (int64_t)((uint64_t)a - (uint64_t)b);
}
// floor division for a positive divisor
__host__ __device__ __forceinline__ int64_t floor_div(int64_t a, int64_t b) {
    int64_t q = a / b;
    return (a % b != 0 && a < 0) ? q - 1 : q;
}

// Exact floor division / Java remainder by a positive divisor b with a precomputed
// reciprocal rb = 1.0 / b: one f64 multiply + at most two integer corrections. Falls
// back to integer division when |a| >= 2^52 (outside ~142,000 years of epoch millis).
__host__ __device__ __forceinline__ int64_t floor_div_fast(int64_t a, int64_t b, double rb) {
    if (a >= (int64_t(1) << 52) || a <= -(int64_t(1) << 52)) return floor_div(a, b);
    int64_t q = (int64_t)__builtin_floor((double)a * rb);
    int64_t r = a - q * b;
    while (r < 0) { q -= 1; r += b; }
    while (r >= b) { q += 1; r -= b; }
    return q;
}
// Java `a % b` (truncated remainder) for b > 0
__host__ __device__ __forceinline__ int64_t jrem_fast(int64_t a, int64_t b, double rb) {
    int64_t r = a - floor_div_fast(a, b, rb) * b;   // floor remainder in [0, b)
    return (a < 0 && r != 0) ? r - b : r;
}

struct WindowSpec {
    int32_t kind;       // TUMBLE / HOP / CUMULATE
    int32_t mode;       // 0 SQL, 1 DataStream
    int64_t size;       // tumble size, hop size, cumulate max size
    int64_t slide;      // hop slide, cumulate step
    int64_t offset;
    int64_t tz;         // fixed shift-zone offset in ms (0 = UTC; unused when tz_n > 0)
    int64_t slice;      // getSliceEndInterval: tumble size, hop gcd(size, slide), cumulate step
    int64_t nslices;    // hop: size / slice
    double rslice;      // 1.0 / slice
    double rsize;       // 1.0 / size
    // zone with transitions (ZoneRules as data): tz_n instants (epoch ms, ascending) and
    // tz_n + 1 offsets ([i] in force before transition i), one copy in host memory for the
    // engine and one in HBM for the kernels
    const int64_t* tz_trans_h;
    const int64_t* tz_offs_h;
    const int64_t* tz_trans_d;
    const int64_t* tz_offs_d;
    int32_t tz_n;
    int32_t tz_dst;     // TimeZone.useDaylightTime(): the DST branches of TimeWindowUtil
    // the rowtime column already holds local (UTC-shifted) times: partial rows and windowed
    // rows carry their slice / window end, which the `sliced` / `windowed` assigners take as
    // is (SliceAssigners.java:407-412, :520-524) -- set for zone rules, whose local -> epoch
    // mapping is not invertible (a fixed offset round-trips through slice_end - 1 - tz)
    int32_t local_input;
};

// the zone tables of the side this code runs on
__host__ __device__ __forceinline__ const int64_t* zone_trans(const WindowSpec& w) {
#if defined(__HIP_DEVICE_COMPILE__)
    return w.tz_trans_d;
#else
    return w.tz_trans_h;
#endif
}
__host__ __device__ __forceinline__ const int64_t* zone_offs(const WindowSpec& w) {
#if defined(__HIP_DEVICE_COMPILE__)
    return w.tz_offs_d;
#else
    return w.tz_offs_h;
#endif
}
// ZoneRules.getOffset(Instant): the offset after the last transition at or before `instant`
__host__ __device__ __forceinline__ int64_t zone_offset_at(const WindowSpec& w, int64_t instant) {
    const int64_t* T = zone_trans(w);
    int32_t lo = 0, hi = w.tz_n;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (T[mid] <= instant) lo = mid + 1;
        else hi = mid;
    }
    return zone_offs(w)[lo];
}
// LocalDateTime.atZone(zone).toInstant() for a local (UTC-shifted) time: the one valid
// offset; in an overlap the earlier offset (the one before the transition); in a gap the
// local time moves later by the gap and takes the offset after (= local - offset before).
__host__ __device__ inline int64_t zone_local_to_epoch(const WindowSpec& w, int64_t local) {
    const int64_t W = 20ll * 3600 * 1000;   // |offset| <= 18 h
    const int32_t n = w.tz_n;
    const int64_t* T = zone_trans(w);
    const int64_t* O = zone_offs(w);
    int32_t lo = 0, hi = n;                  // first offset region that can hold local - offset
    const int64_t from = jsub(local, W);
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (T[mid] <= from) lo = mid + 1;
        else hi = mid;
    }
    for (int32_t k = lo; k <= n; k++) {
        const int64_t e = jsub(local, O[k]);
        if ((k == 0 || T[k - 1] <= e) && (k == n || e < T[k])) return e;   // first valid: earlier offset
        if (k == n || T[k] > jadd(local, W)) break;
        if (e >= T[k] && jsub(local, O[k + 1]) < T[k]) return e;            // gap at transition k
    }
    return jsub(local, O[n]);
}

// TimeWindow.getWindowStartWithOffset (Java truncated remainder, kept bit for bit)
__host__ __device__ __forceinline__ int64_t window_start_with_offset(int64_t ts, int64_t off, int64_t size) {
    return jsub(ts, jadd(jsub(ts, off), size) % size);
}
// TimeWindowUtil.toUtcTimestampMills (:53-61)
__host__ __device__ __forceinline__ int64_t to_utc(const WindowSpec& w, int64_t epoch) {
    if (w.tz_n > 0) return epoch == JMAX ? epoch : jadd(epoch, zone_offset_at(w, epoch));
    return (w.tz == 0 || epoch == JMAX) ? epoch : jadd(epoch, w.tz);
}
// TimeWindowUtil.toEpochMillsForTimer (:70-140): with daylight saving, a local time in a
// gap takes the first skipped instant (hasNoEpoch) and one in an overlap the later instant
// (hasTwoEpochs); without, toEpochMills (atZone)
__host__ __device__ __forceinline__ int64_t to_epoch_for_timer(const WindowSpec& w, int64_t utc) {
    if (w.tz_n > 0) {
        if (utc == JMAX) return utc;
        const int64_t t1 = zone_local_to_epoch(w, utc);
        if (!w.tz_dst) return t1;
        const int64_t HOUR = 3600ll * 1000;
        const int64_t t2 = zone_local_to_epoch(w, jadd(utc, HOUR));
        if (t1 == t2) return jsub(t1, t1 % HOUR);
        if (jsub(t2, t1) > HOUR) return jadd(t1, HOUR);
        return t1;
    }
    return (w.tz == 0 || utc == JMAX) ? utc : jsub(utc, w.tz);
}
// trigger time of a window (the timer timestamp registered by WindowTimerServiceImpl:60-63)
__host__ __device__ __forceinline__ int64_t trigger_time(const WindowSpec& w, int64_t window_end) {
    return to_epoch_for_timer(w, jsub(window_end, 1));
}
__host__ __device__ __forceinline__ bool is_window_fired(const WindowSpec& w, int64_t window_end, int64_t progress) {
    if (window_end == JMAX) return false;
    return progress >= trigger_time(w, window_end);
}
// AbstractSliceAssigner.assignSliceEnd (rowtime path)
__host__ __device__ __forceinline__ int64_t assign_slice_end(const WindowSpec& w, int64_t ts) {
    int64_t t = w.local_input ? ts : to_utc(w, ts);
    int64_t start = jsub(t, jrem_fast(jadd(jsub(t, w.offset), w.slice), w.slice, w.rslice));
    return jadd(start, w.slice);
}
__host__ __device__ __forceinline__ int64_t window_start(const WindowSpec& w, int64_t window_end) {
    if (w.kind == CUMULATE) {
        int64_t t = jsub(window_end, 1);
        return jsub(t, jrem_fast(jadd(jsub(t, w.offset), w.size), w.size, w.rsize));
    }
    return jsub(window_end, w.size);
}
__host__ __device__ __forceinline__ int64_t last_window_end(const WindowSpec& w, int64_t slice_end) {
    if (w.kind == TUMBLE) return slice_end;
    if (w.kind == HOP) return jadd(jsub(slice_end, w.slice), w.size);
    return jadd(window_start(w, slice_end), w.size);
}
// SliceSharedWindowAggProcessor.sliceStateMergeTarget (:120-131): cumulate -> first slice
__host__ __device__ __forceinline__ int64_t merge_target(const WindowSpec& w, int64_t slice_end) {
    if (w.kind == CUMULATE) return jadd(window_start(w, slice_end), w.slice);
    return slice_end;
}
// TimeWindowUtil.getNextTriggerWatermark (useDayLightSaving = false)
__host__ __device__ __forceinline__ int64_t next_trigger_watermark(int64_t wm, int64_t interval) {
    if (wm == JMAX) return wm;
    int64_t start = window_start_with_offset(wm, 0, interval);
    int64_t trig = jsub(jadd(start, interval), 1);
    return trig > wm ? trig : jadd(trig, interval);
}
// the same with the window's zone: the daylight-saving branch (:194-199) when the zone
// observes it (AbstractWindowAggProcessor's useDayLightSaving)
__host__ __device__ __forceinline__ int64_t next_trigger_watermark(const WindowSpec& w, int64_t wm, int64_t interval) {
    if (!(w.tz_n > 0 && w.tz_dst) || wm == JMAX) return next_trigger_watermark(wm, interval);
    const int64_t start = window_start_with_offset(to_utc(w, wm), 0, interval);
    const int64_t trig = to_epoch_for_timer(w, jsub(jadd(start, interval), 1));
    return trig > wm ? trig : jadd(trig, interval);
}

// Target slice of one record under the late-record rules of
// AbstractWindowAggProcessor.processElement (:135-165). Returns false when dropped.
__host__ __device__ __forceinline__ bool target_slice(const WindowSpec& w, int64_t ts, int64_t progress,
                                                     int64_t* target) {
    int64_t s = assign_slice_end(w, ts);
    if (is_window_fired(w, s, progress)) {
        if (is_window_fired(w, last_window_end(w, s), progress)) return false;
        *target = merge_target(w, s);
        return true;
    }
    *target = s;
    return true;
}

// 64-bit finalizer (MurmurHash3 fmix64): bijective, spreads keys over state regions.
// Device state keeps every key as its mix h = fmix64(key): the top region_bits of h pick
// the state region, the low 32 bits the LDS home bucket, and no kernel past ingest hashes
// a key again; rows and images leaving the engine carry fmix64_inv(h) = the key.
__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdULL;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ULL;
    h ^= h >> 33;
    return h;
}
// inverse of fmix64 (x ^= x >> 33 is an involution; the multipliers' inverses mod 2^64)
__host__ __device__ __forceinline__ uint64_t fmix64_inv(uint64_t h) {
    h ^= h >> 33;
    h *= 0x9cb4b2f8129337dbULL;
    h ^= h >> 33;
    h *= 0x4f74430c22a54005ULL;
    h ^= h >> 33;
    return h;
}
__host__ __device__ __forceinline__ int64_t key_of(int64_t h) { return (int64_t)fmix64_inv((uint64_t)h); }
__host__ __device__ __forceinline__ int64_t mix_of(int64_t key) { return (int64_t)fmix64((uint64_t)key); }

// ---- Flink key groups (KeyGroupRangeAssignment.java:63-77, MathUtils.java:137-155,194-201,
//      MurmurHashUtils.java hashBytes over the 16-byte BinaryRowData of one BIGINT) ----------
__host__ __device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__host__ __device__ __forceinline__ uint32_t mix_k1(uint32_t k1) {
    k1 *= 0xcc9e2d51u;
    k1 = rotl32(k1, 15);
    return k1 * 0x1b873593u;
}
__host__ __device__ __forceinline__ uint32_t mix_h1(uint32_t h1, uint32_t k1) {
    h1 ^= k1;
    h1 = rotl32(h1, 13);
    return h1 * 5u + 0xe6546b64u;
}
__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
__host__ __device__ __forceinline__ int32_t binaryrow_hash_i64(int64_t key) {
    uint32_t h1 = 42u;
    h1 = mix_h1(h1, mix_k1(0u));
    h1 = mix_h1(h1, mix_k1(0u));
    h1 = mix_h1(h1, mix_k1((uint32_t)((uint64_t)key & 0xffffffffu)));
    h1 = mix_h1(h1, mix_k1((uint32_t)((uint64_t)key >> 32)));
    return (int32_t)fmix32(h1 ^ 16u);
}
__host__ __device__ __forceinline__ int32_t java_long_hash(int64_t key) {
    return (int32_t)(uint32_t)((uint64_t)key ^ ((uint64_t)key >> 32));
}
__host__ __device__ __forceinline__ int32_t murmur_hash(int32_t code) {
    uint32_t c = (uint32_t)code;
    c *= 0xcc9e2d51u;
    c = rotl32(c, 15);
    c *= 0x1b873593u;
    c = rotl32(c, 13);
    c = c * 5u + 0xe6546b64u;
    c ^= 4u;
    int32_t r = (int32_t)fmix32(c);
    if (r >= 0) return r;
    if (r != INT32_MIN) return -r;
    return 0;
}
// bits of the key group in an fg_key_dict id: ceil(log2(max parallelism))
__host__ __device__ __forceinline__ int32_t dict_kg_bits(int32_t max_p) {
    int32_t b = 0;
    while (b < 31 && (1 << b) < max_p) b++;
    return b;
}
__host__ __device__ __forceinline__ int32_t key_group_of(int64_t key, int32_t key_hash, int32_t max_p) {
    // an fg_key_dict id carries its key group in its low bits (ordinal << kg_bits | key group)
    if (key_hash == 2) return (int32_t)((uint64_t)key & ((1ull << dict_kg_bits(max_p)) - 1)) % max_p;
    int32_t h = key_hash == 0 ? binaryrow_hash_i64(key) : java_long_hash(key);
    return murmur_hash(h) % max_p;
}

}  // namespace fg
