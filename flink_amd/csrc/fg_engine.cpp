// fg_engine.cpp -- host side of libflinkgpu.so: the C-ABI of include/flinkgpu.h.
//
// Mirrors the control flow of the reference operator around the GPU hot path:
//   processElement    -> fg_add_batch: device ingest (slice assignment, late rules,
//                        bucketing) into a staged buffer  (RecordsWindowBuffer.addElement)
//   processWatermark  -> fg_advance_progress: the AbstractWindowAggProcessor.advanceProgress
//                        gate (:178-192) and RecordsWindowBuffer.advanceProgress (:100-105)
//                        decide the flush; then every window whose timer would fire
//                        (trigger in (previous watermark, watermark]) is fired from the
//                        GPU-resident slice state (fireWindow/mergeSlices/clearWindow).
//   prepareSnapshotPreBarrier -> fg_flush ; snapshot/restore -> fg_snapshot_state/fg_restore.
//
// State is kept per slice in HBM ("slice tables"); a (key, window) row fires when its
// window's timer fires and the key holds state in the window's slices -- the timers of
// the reference (one per (key, window), registered by AggCombiner step 5 and chained by
// nextTriggerWindow) fire exactly for those (key, window) pairs when offset == 0
// (DESIGN.md "Firing without per-key timers").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <csignal>
#include <execinfo.h>
#include <map>
#include <mutex>
#include <memory>
#include <string>
#include <set>
#include <vector>

#include "../../include/flinkgpu.h"
#include "fg_kernels.h"
#include "fg_late.h"

using namespace fg;

namespace {

thread_local std::string g_open_error;

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;   // one owner per device allocation
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t ensure(size_t need, hipStream_t s = nullptr, bool keep = false) {
        if (need <= bytes) return hipSuccess;
        size_t nb = std::max(need, bytes + bytes / 2);
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, nb);
        if (e != hipSuccess) return e;
        if (keep && p && bytes) {
            e = hipMemcpyAsync(q, p, bytes, hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) return e;
            e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
        }
        if (p) (void)hipFree(p);
        p = q;
        bytes = nb;
        return hipSuccess;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
    void swap(DevBuf& o) {
        std::swap(p, o.p);
        std::swap(bytes, o.bytes);
    }
};

struct HostBuf {   // pinned host memory
    void* p = nullptr;
    size_t bytes = 0;
    ~HostBuf() {
        if (p) (void)hipHostFree(p);
    }
    hipError_t ensure(size_t need, unsigned flags = hipHostMallocDefault) {
        if (need <= bytes) return hipSuccess;
        size_t nb = std::max(need, bytes + bytes / 2);
        void* q = nullptr;
        hipError_t e = hipHostMalloc(&q, nb, flags);
        if (e != hipSuccess) return e;
        if (p) (void)hipHostFree(p);
        p = q;
        bytes = nb;
        return hipSuccess;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct SliceTable {
    int64_t slice_end = 0;
    DevBuf data;          // P * 4 * kRegionCap int64
    DevBuf counts;        // P uint32
    int64_t upper = 0;    // host-side upper bound of entries
    int bits = 0;         // region bits of its layout
    bool has_null = false;   // some entry may count NULL values (else its cnt_null column is all 0)
    // 16-B entries (fg_kernels.h TableRef): written only by the tile fire with tables, read by
    // every reader; a table takes the layout of the first writer that finds it empty, and is
    // widened in place (k_widen_table) before a writer of the wide layout or a region split
    bool narrow = false;
    // written since the last snapshot image (fg_snapshot_slices: a shim rewrites only the keyed
    // state of the slices whose tables changed between two checkpoints)
    bool changed = true;
};

// One ingest pass: the bucket scan of its records over all lanes; lane l's records sit at
// [lane_start[l], lane_start[l] + lane_n[l]) of lane l's staged area.
struct Staged {
    DevBuf bucket_off;    // F + 1 uint32 (lane-major), F = lanes << bits
    int bits = 0;         // region bits the pass was bucketed at (the regions may split later)
    bool is_acc = false;  // accumulator rows (global phase) in the lanes' accumulator areas
    int64_t lane_start[kMaxLanes] = {0, 0, 0, 0};
    int64_t lane_n[kMaxLanes] = {0, 0, 0, 0};
    bool has_null = false;
    bool narrow = false;  // 12-B records {int32 key, value} (IngestParams.narrow)
    bool skew = false;    // some region may hold over kHeavyMin records of this pass (hot keys)
    int refs = 0;         // lanes still holding records of this pass
    // tile staging (fg_kernels.h): the records stay in pass-1 tiles sorted by consumer bucket
    // until a TUMBLE / local-phase fire reads them (k_tile_fire) or they are materialized
    bool tiles = false;
    DevBuf t_rec, t_dt;   // block-laid 12-B records at their batch index; per-bucket (offset, length) columns
    DevBuf t_btot;        // records per bucket of the pass (a skewed pass's fire plans its chunks from them)
    int64_t t_n = 0;
    int t_nt = 0, t_mt = 0, t_nc = 0;
    bool busy = false;    // read by a merge job not yet settled: not reused from the pool
    // a materialized tile pass: its own narrow record area (block-laid from index 0)
    bool own = false;
    DevBuf own_rec;
};

// A slice lane of the staged buffer (RecordsWindowBuffer analogue, one per live slice):
// slice index q = slice_end / slice (mod lanes == lane), records staged, and the passes
// that hold them.
constexpr int64_t kEmptyLane = INT64_MIN;
struct Lane {
    int64_t q = kEmptyLane;
    int64_t fill = 0;       // staged records
    int64_t acc_fill = 0;   // staged accumulator rows (global phase)
    std::vector<Staged*> passes;
};

struct DevCounters {     // device scratch words read back after the count pass
    unsigned long long drops;
    unsigned long long lane_mask;
    long long qmin, qmax;
    long long qnext;       // smallest occupied slice index >= the pass's filter (JMAX: none)
    unsigned long long lane_total[kMaxLanes];
    unsigned int max_bucket;   // largest per-workgroup bucket count (skew hint)
    unsigned int wide;         // pass 1: an accepted key does not fit 32 bits (narrow staging off)
};
struct Counters {        // host view: per-lane slice index ranges (min > max: lane idle)
    unsigned long long drops;
    long long qmin, qmax;
    long long qnext;       // smallest occupied slice index >= the pass's filter_hi (JMAX: none)
    long long lane_min[kMaxLanes];
    long long lane_max[kMaxLanes];
    long long lane_total[kMaxLanes];
    bool skew;
};

// skewed regions (hot keys): a region holding more than max(kHeavyMin, 8 x the mean) staged
// records at merge time is merged in kHeavyChunk-record chunks (k_heavy_plan/_chunks +
// the heavy pass), so that its work is spread over the GPU instead of one workgroup
constexpr int64_t kHeavyMin = 1 << 16;
constexpr int64_t kHeavyChunk = 1 << 16;

enum KClass { K_COUNT = 0, K_SCAN, K_SCATTER, K_PART1, K_PART2, K_FLUSH, K_FLUSH_FIRE, K_FIRE, K_EXPORT, K_RESTORE,
              K_HEAVY, K_TILE1, K_TILE_FIRE, K_TILE_MAT, K_TILE_FLUSH, K_TILE_SPLIT, K_NCLASS };
const char* const kClassName[K_NCLASS] = {"ingest_count", "ingest_scan",      "ingest_scatter", "ingest_part1",
                                           "ingest_part2", "merge_flush",      "merge_flush_fire", "merge_fire",
                                           "export",       "restore",          "merge_heavy",      "tile_part1",
                                           "tile_fire",    "tile_materialize", "tile_flush",       "tile_split_fire"};
struct KStat {
    int64_t launches = 0;
    double ms = 0;
    int64_t records = 0, rows = 0;
};
struct PendingEv {
    int cls;
    hipEvent_t a, b;
    int64_t records;
};

// Capacity growth (the BytesMap analogue: BytesMap.java:229-290 doubles its bucket area when
// full; RecordsWindowBuffer.java:89-96 flushes and retries on EOFException). A state region
// holds at most kRegionCap entries in HBM and its LDS table kSlots keys; a region that
// overflows in a merge emits and writes nothing and is reported in the fail list. Every
// merge launch is kept as a job (inputs by reference) until the synchronization that
// follows it: then the regions split (2^b -> 2^(b+1), the slice tables re-laid by
// k_split_table, staged passes read through their coarser buckets) and exactly the failed
// regions' children are merged again, until none fails.
constexpr int kMaxRegionBits = 13;
constexpr int kFailCap = 1 << 16;
constexpr int64_t kStateCapMax = (int64_t)kRegionCap << kMaxRegionBits;   // entries of a slice at most
constexpr int kDefaultRegionBits = 10;   // no key-count hint
struct JobBatch {
    Staged* s = nullptr;   // a staged pass (lane `lane`) ...
    int lane = 0;
    StagedBatch ext{};     // ... or an explicit batch (restore image) bucketed at ext_bits
    int ext_bits = 0;
};
struct PassState {
    IngestParams p{};
    std::unique_ptr<Staged> s;
    bool two_pass = false, spec = false;
    bool tiles = false;    // tile staging (k_tile_part1): no pass 2
    int64_t n = 0;
    const uint8_t* vnull = nullptr;
    int64_t flo = 0, fhi = 0;
};

struct MergeJob {
    std::vector<JobBatch> batches;
    std::vector<SliceTable*> srcs;
    SliceTable* dst = nullptr;
    bool emit = false;
    int64_t wend = 0;
    int bits = 0;          // region bits of its last launch
    int kclass = 0;
    // restore re-fire (MergeParams): marking / mark-only sources, marked emission, chain dst
    uint64_t mark_mask = 0, markonly_mask = 0;
    int emit_marked = 0, dst_mode = 0;
    bool tile = false;     // a fire straight from tile passes (k_tile_fire; batches: the passes, tbits)
    int tbits = 0;
};

}  // namespace

// A batch whose first pass is queued but not yet finished on the host (deferred staging)
struct PendingBatch {
    bool active = false;
    PassState ps;
    int64_t n = 0;
    const int64_t *key = nullptr, *ts = nullptr, *val = nullptr;
    const uint8_t* vnull = nullptr;
    int64_t flo = 0, fhi = 0;
    int slot = -1;
};

struct fg_handle {
    int32_t kvt = 0;   // kernel value op (val_type | op << 2); multi-value: the value type
    // several value accumulators (SUM family + MIN + MAX): value slots 0 SUM, 1 MIN, 2 MAX
    int mv = 0;
    int32_t vop[kNV] = {3, 3, 3};          // op per slot (0 SUM, 1 MIN, 2 MAX, 3 none)
    int32_t agg_slot[FG_MAX_AGGS] = {};    // value slot of each output aggregate
    int tcap = kRegionCap;                 // entries per region of its tables
    fg_config cfg{};
    WindowSpec w{};
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    int region_bits = 0, P = 1, lanes = 1, F = 1, grid = 256, merge_grid = 256;
    int64_t slice_phase = 0;   // slice ends are == slice_phase (mod slice)

    // processor / timer state
    int64_t current_progress = JMIN;
    int64_t next_trigger = JMIN;
    int64_t timer_wm = JMIN;
    int64_t late_dropped = 0;

    // staged buffer (RecordsWindowBuffer analogue): one area of lane_cap records per lane
    int64_t lane_cap = 0;
    int st_stride = 2;          // int64 words per staged record: {key, val} or {key}
    // narrow staging: passes write 12-B {int32 key, value} records while every key seen fits
    // 32 bits; the first wider key flushes the lanes and turns it off for good (all live
    // passes share one record format, so a lane's positions map to one byte layout)
    bool narrow = false;
    bool narrow_ok = false;   // the operator may stage narrow records (fg_reset restores `narrow`)
    DevBuf st_rec, st_null;
    Lane lane[kMaxLanes];
    // accumulator areas (global phase, fg_add_partials): SoA, acc_cap rows per lane
    int64_t acc_cap = 0;
    DevBuf acc_key, acc_cs, acc_cn, acc_sum;
    DevBuf acc_v1, acc_v2;   // multi-value operator: the partial rows' MIN / MAX
    DevBuf in_cs, in_cv, in_sum, in_slice, in_v1, in_v2;
    bool local = false;     // FG_FLAG_LOCAL_PARTIALS: fired slices emit partial accumulators
    bool local_emit_all = false;   // fg_flush_partials: every staged slice emits now
    bool proctime = false;  // FG_FLAG_PROCTIME: processing-time windows, nothing is late
    std::vector<int64_t> tz_trans, tz_offs;   // zone rules (host copy); tz_dev: the HBM copy
    DevBuf tz_dev;
    bool windowed = false;  // FG_FLAG_WINDOWED: rows carry window_end; `w` is a one-slice
    WindowSpec inner{};     // window per slice, `inner` the TVF's assigner (getWindowStart)
    DevBuf in_wts;          // windowed: pseudo rowtimes of a batch
    std::vector<std::unique_ptr<Staged>> passes;       // live passes
    std::vector<std::unique_ptr<Staged>> pass_pool;
    int64_t anchor_start = JMIN;   // a recent slice start: base of the 32-bit rowtime fast path

    // ingest scratch
    DevBuf in_key, in_ts, in_val, in_null;
    DevBuf in_rows, row_bad;   // fg_add_rows: host rows copied in; NULL key/rowtime + NULL value counts
    // FG_HOST batches: double-buffered H2D on a copy stream of its own, so that the copy of
    // batch i + 1 overlaps the kernels of batch i (the engine stream waits for the copy's
    // event; a buffer is rewritten only after the kernels that read it)
    hipStream_t copy_stream = nullptr;
    // asynchronous snapshot (fg_snapshot_state_async): the image's D2H copy runs on its own
    // stream after the export kernels (event ev_snap), collected by fg_snapshot_state_wait
    hipStream_t snap_stream = nullptr;
    hipEvent_t ev_snap = nullptr;
    bool snap_pending = false;
    bool snap_cv_alias = false;   // the pending image's cnt_val column is its cnt_star column
    int64_t snap_total = 0, snap_wm = 0;
    // the slices of the last image (fg_snapshot_slices): ends, row ranges, changed since the image
    // before (SliceTable.changed, cleared at each snapshot)
    std::vector<int64_t> img_se, img_first, img_rows;
    std::vector<uint8_t> img_changed;
    bool img_ready = false;   // an image was returned since the last snapshot call
    DevBuf hb_key[2], hb_ts[2], hb_val[2], hb_null[2];
    DevBuf hb_narrow[2];   // FG_HOST narrow columns (fg_batch.format) before widening
    hipEvent_t ev_copied[2] = {nullptr, nullptr}, ev_free[2] = {nullptr, nullptr};
    int hslot = 0;
    DevBuf part_tmp, part_tmp_null, part_dir;   // two-pass partition: pass-1 tiles + directory
    // tile staging (FG_TILE=0 turns it off, A/B): in-order TUMBLE and local-phase batches of 32-bit
    // keys stay in their pass-1 tiles until the fire; off for good once a wider key is seen
    bool tile_ok = true;
    // FG_TILE_STATE: tile passes of HOP / CUMULATE (and TUMBLE lanes with resident state) flush
    // into their slice tables straight from the tiles (k_tile_fire with tables); 0: TUMBLE and
    // local fires only, anything else materialized (the round-4 first tile build)
    bool tile_state = true;
    int tile_grid_force = 0;  // FG_TILE_GRID (test knob, tile_grid)
    bool tile_skew = false;   // a tile pass saw hot-key skew: later batches take the two-pass partition
                              // (a performance hint kept across fg_reset)
    // FG_TILE_SPLIT (default on): a skewed tile pass of a TUMBLE / local-phase operator stays on the
    // tiles; its fire splits the hot buckets into chunk items (k_tile_plan, k_tile_fire's merge)
    bool tile_split = true;
    uint32_t tile_chunk = 0;
    // FG_TILE_HOT=1: the split fire's wave pre-combine of a hot key. Off by default: configs[4]
    // A/B (profiles/r05/zipf_ab): split fire 1.485 vs 1.072 ms per 100M-record window with it on --
    // the ballot + butterflies cost more than the same-slot LDS atomics they save
    bool tile_hot = false;
    // tables written by the tile fire take 16-B entries (round 5: CUMULATE 62.7 -> 59.0 ms per 1B)
    bool narrow_tables = true;
    DevBuf tile_dir, tile_hist;
    DevBuf sp_items, sp_n, sp_split, sp_parts, sp_pkey, sp_pcs, sp_pv, sp_bfail, sp_icnt;   // split plans + partials
    // skewed-region plan and chunk partial tables
    DevBuf hv_flags, hv_list, hv_n, hv_chunk0, hv_clist, hv_v0, hv_v1, hv_key, hv_cs, hv_cn, hv_sum, hv_pn;
    DevBuf hv_mv1, hv_mv2;   // multi-value operator: value slots 1 and 2 of the chunks' partial rows
    int64_t hv_max_chunks = 0;
    DevBuf hist, totals, scan_tmp, counters;
    DevBuf plan_dev;          // k_scan_plan's lane plan (speculative pass 2)
    HostBuf h_pass;           // coherent host memory k_scan_plan writes the pass's counters + plan to
    unsigned long long pass_seq = 0;   // k_scan_plan's sequence word in h_pass
    // asynchronous advance (fg_advance_progress_async): its fires publish the scalars to h_fire
    // (k_publish_words) instead of synchronizing; the completion -- row count, region retries,
    // overflow check -- is taken by complete_fire at the next call that needs it
    HostBuf h_fire;
    unsigned long long fire_seq = 0;
    bool async_advance = false;   // the advance in progress publishes its fires
    bool fire_pending = false;    // published, not yet completed
    bool fire_rows_open = false;  // the pending fire's rows are not yet in rows_fired
    int fire_kclass = 0;          // kernel class credited with the pending fire's rows
    int64_t fire_before = 0;      // out_n when the pending fire was published
    bool async_open = false;      // rows of async advances not yet collected: the next one appends
    int64_t adv_base = 0;         // rows ahead of the current advance's in the output buffers
    int64_t fire_rows_base = 0;   // adv_base of the advance whose rows complete_fire counts
    bool fail_zeroed = false;     // the fail count was zeroed by flush_lanes' fill (job_add skips its own)
    bool counters_clean = false;   // the device counters hold their initial values
    bool speculate = true;    // FG_SPECULATE=0 turns the speculative pass 2 off (A/B)
    PendingBatch pending;     // deferred first pass of the last batch
    hipEvent_t ev_pending = nullptr;
    DevBuf sink;   // target of the stores of idle lanes (kernels keep their store counts static)
    HostBuf h_counters;

    // resident state
    std::map<int64_t, std::unique_ptr<SliceTable>> tables;
    std::vector<std::unique_ptr<SliceTable>> table_pool;
    // capacity growth: merge launches since the last synchronization (job id = index),
    // tables freed meanwhile (a job may still read them), the fail list of overflowed regions
    std::vector<MergeJob> jobs;
    std::vector<std::unique_ptr<SliceTable>> deferred;
    bool defer_free = false;
    DevBuf fail_list;
    HostBuf h_fail;
    int lanes_target = 0;   // lanes for the current region bits (reached once the upper lanes drain)
    int64_t grows = 0;
    // Restore re-fire of shared windows (HOP / CUMULATE, refire()): records flushed after a
    // restore into slices whose windows fired before the checkpoint are kept apart -- re_new
    // their state, re_delta their keys since the last watermark -- and re-fire those windows
    // for their keys only, chained as nextTriggerWindow chains the reference's timers.
    int64_t refire_hi = JMIN;   // the checkpoint's timer watermark (JMIN: nothing to re-fire)
    int64_t arrival_progress = JMIN;   // progress the staged records arrived under (set per advance)
    int64_t refire_wm = JMIN;   // the watermark the re-fire ran at last
    std::map<int64_t, std::unique_ptr<SliceTable>> re_new, re_delta;
    std::unique_ptr<SliceTable> re_chain;   // keys whose chain continues at window re_chain_w
    int64_t re_chain_w = JMIN;
    std::vector<std::unique_ptr<SliceTable>> re_tmp;   // chain tables of the running re-fire

    // descriptor arena (device + pinned mirror), reset at every sync point
    DevBuf arena;
    HostBuf h_arena;
    size_t arena_used = 0;

    // device scalars: [0] overflow flags, [1] out_count
    DevBuf scalars;
    HostBuf h_scalars;
    bool out_count_reset = false;   // out_count zeroed for the current advance

    // fired rows
    int64_t out_cap = 0, out_n = 0, pending_out = 0;
    std::set<int64_t> fused_fired;   // window ends fired by a fused flush in the current advance
    int64_t q_guess = kEmptyLane;   // first slice of the next batch's first ingest pass (kEmptyLane: all)
    DevBuf o_key, o_ws, o_we, o_null, o_rt;
    DevBuf o_agg[FG_MAX_AGGS];
    HostBuf h_key, h_ws, h_we, h_null, h_rt;
    HostBuf h_agg[FG_MAX_AGGS];

    // snapshot image
    DevBuf s_key, s_slice, s_cs, s_cv, s_sum, s_off, s_v1, s_v2;
    HostBuf hs_key, hs_slice, hs_cs, hs_cv, hs_sum, hs_counts, hs_off, hs_v1, hs_v2;

    // DataStream allowed lateness (WindowOperator.allowedLateness, fg_late.hip): a fired window's
    // slices stay resident until its cleanup time (retire_at: slice end -> the cleanup time of
    // the slice's last window); rows fired by late elements in fg_add_batch wait in the output
    // buffers for the next fg_advance_progress (late_rows of them)
    int64_t lateness = 0;
    bool purging = false;                  // FG_FLAG_PURGING_TRIGGER
    bool retain = false;                   // lateness > 0 and not purging: fired windows keep state
    std::map<int64_t, int64_t> retire_at;
    int64_t late_rows = 0;
    int64_t late_horizon = JMIN;           // after fg_restore: the checkpoint's watermark (fired windows)
    DevBuf lt_mix, lt_se, lt_val, lt_null, lt_idx, lt_done, lt_sel, lt_slot, lt_found, lt_ckey, lt_cidx, lt_need;
    DevBuf lt_dir_se, lt_dir_t, lt_words, lt_r_key, lt_r_ts, lt_r_val, lt_r_null;
    HostBuf lt_h;

    // stats
    int64_t records_in = 0, rows_fired = 0, flushes = 0;
    // bound on any (key, window)'s COUNT(*): records taken since the reset (JMAX once partial
    // accumulators or a state image, whose counts are unbounded, entered) -- gates the compact
    // merge's 32-bit LDS counts
    int64_t cnt_bound = 0;
    // every key staged since the reset fits 32 bits (narrow passes only, no partials or images):
    // the compact merge may key its LDS table by the int32 key of a resident entry's mix
    bool keys32 = true;
    bool skew_seen = false;     // some ingest pass saw hot-key skew (pass-2 units of one workgroup)
    bool timing = false;
    uint32_t timing_mask = ~0u;   // kernel classes bracketed with events (fg_set_kernel_timing)
    KStat kstat[K_NCLASS];
    std::vector<PendingEv> pend;
    std::vector<hipEvent_t> ev_pool;

    int fail(int code, const char* fmt, ...) {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
};

#define HIPCHK(h, expr)                                                                        \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess)                                                                   \
            return (h)->fail(FG_EDEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                             __FILE__, __LINE__);                                               \
    } while (0)

namespace {

int64_t gcd64(int64_t a, int64_t b) {
    while (b) {
        int64_t t = a % b;
        a = b;
        b = t;
    }
    return a < 0 ? -a : a;
}

int64_t slice_end_of(const fg_handle* h, int64_t q) { return jadd((int64_t)((uint64_t)q * (uint64_t)h->w.slice), h->slice_phase); }

// copy a small descriptor array into the arena and return its device address
template <class T>
int arena_put(fg_handle* h, const T* items, size_t n, const T** dev) {
    size_t bytes = sizeof(T) * std::max<size_t>(n, 1);
    size_t at = (h->arena_used + 255) & ~size_t(255);
    if (at + bytes > h->arena.bytes) return h->fail(FG_EDEVICE, "descriptor arena exhausted");
    std::memcpy(h->h_arena.as<char>() + at, items, sizeof(T) * n);
    HIPCHK(h, hipMemcpyAsync(h->arena.as<char>() + at, h->h_arena.as<char>() + at, bytes, hipMemcpyHostToDevice,
                             h->stream));
    *dev = reinterpret_cast<const T*>(h->arena.as<char>() + at);
    h->arena_used = at + bytes;
    return FG_OK;
}

hipEvent_t ev_get(fg_handle* h) {
    if (!h->ev_pool.empty()) {
        hipEvent_t e = h->ev_pool.back();
        h->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}
// bracket one launch call with HIP events on the handle's stream (FG_FLAG_KERNEL_TIMING): the
// events ride in the kernels' dispatch packets (fg_launch), so timing adds no queue markers
struct KTimer {
    fg_handle* h;
    int cls;
    int64_t records;
    hipEvent_t a = nullptr, b = nullptr;
    KTimer(fg_handle* hh, int c, int64_t r) : h(hh), cls(c), records(r) {
        if (h->timing && ((h->timing_mask >> cls) & 1u)) {
            a = ev_get(h);
            b = ev_get(h);
            g_launch_ev.start = a;
            g_launch_ev.stop = b;
        }
    }
    ~KTimer() {
        if (!a) return;
        const bool launched = g_launch_ev.start == nullptr;
        g_launch_ev = LaunchEvents{};
        if (!launched) {   // the call launched nothing: no span
            h->ev_pool.push_back(a);
            h->ev_pool.push_back(b);
            return;
        }
        h->pend.push_back(PendingEv{cls, a, b, records});
    }
};

// counters initialised by a kernel in stream order (no blit + queue latency before pass 1)
hipError_t init_counters(fg_handle* h, const DevCounters& init) {
    static_assert(sizeof(DevCounters) % 8 == 0 && sizeof(DevCounters) <= 16 * 8, "DevCounters words");
    Words16 w{};
    w.n = (int32_t)(sizeof(DevCounters) / 8);
    std::memcpy(w.v, &init, sizeof init);
    return launch_store_words(h->counters.as<unsigned long long>(), w, h->stream);
}

int sync(fg_handle* h, bool drain_timing = false) {
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->arena_used = 0;
    // kernel-timing events are read off the critical path (they are complete here); only a
    // long backlog, and fg_kernel_stats / fg_synchronize, drain them
    if (!drain_timing && h->pend.size() < 1024) return FG_OK;
    for (auto& p : h->pend) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) h->kstat[p.cls].ms += ms;
        h->kstat[p.cls].launches++;
        h->kstat[p.cls].records += p.records;
        h->ev_pool.push_back(p.a);
        h->ev_pool.push_back(p.b);
    }
    h->pend.clear();
    return FG_OK;
}

// an empty slice table of the current layout (from the pool when one is free)
int table_new(fg_handle* h, int64_t slice_end, std::unique_ptr<SliceTable>* out) {
    std::unique_ptr<SliceTable>& t = *out;
    if (!h->table_pool.empty()) {
        t = std::move(h->table_pool.back());
        h->table_pool.pop_back();
    } else {
        t.reset(new SliceTable());
        HIPCHK(h, t->data.ensure(sizeof(int64_t) * table_cols(h->mv) * (size_t)table_cap(h->mv) * h->P));
        HIPCHK(h, t->counts.ensure(sizeof(uint32_t) * h->P));
    }
    HIPCHK(h, hipMemsetAsync(t->counts.p, 0, sizeof(uint32_t) * h->P, h->stream));
    t->slice_end = slice_end;
    t->upper = 0;
    t->bits = h->region_bits;
    t->has_null = false;
    t->narrow = false;
    t->changed = true;
    return FG_OK;
}

int table_get(fg_handle* h, int64_t slice_end, bool create, SliceTable** out) {
    auto it = h->tables.find(slice_end);
    if (it != h->tables.end()) {
        *out = it->second.get();
        return FG_OK;
    }
    if (!create) {
        *out = nullptr;
        return FG_OK;
    }
    std::unique_ptr<SliceTable> t;
    int rc = table_new(h, slice_end, &t);
    if (rc) return rc;
    *out = t.get();
    h->tables[slice_end] = std::move(t);
    return FG_OK;
}

void table_free(fg_handle* h, int64_t slice_end) {
    auto it = h->tables.find(slice_end);
    if (it == h->tables.end()) return;
    // a merge launched since the last synchronization may still need it (region retry)
    if (h->defer_free || h->fire_pending) h->deferred.push_back(std::move(it->second));
    else h->table_pool.push_back(std::move(it->second));
    h->tables.erase(it);
}

bool refire_slice(const fg_handle* h, int64_t se) {
    return h->refire_hi != JMIN && !h->local && se != JMAX && trigger_time(h->w, se) <= h->refire_hi;
}

SliceTable* side_get(std::map<int64_t, std::unique_ptr<SliceTable>>& m, int64_t se) {
    auto it = m.find(se);
    return it == m.end() ? nullptr : it->second.get();
}

int side_create(fg_handle* h, std::map<int64_t, std::unique_ptr<SliceTable>>& m, int64_t se, SliceTable** out) {
    if ((*out = side_get(m, se))) return FG_OK;
    std::unique_ptr<SliceTable> t;
    int rc = table_new(h, se, &t);
    if (rc) return rc;
    *out = t.get();
    m[se] = std::move(t);
    return FG_OK;
}

TableRef ref_of(SliceTable* t) {
    return TableRef{t->data.as<int64_t>(), t->counts.as<uint32_t>(), t->narrow ? 1 : 0, 0};
}
int widen_table(fg_handle* h, SliceTable* t) {
    if (!t || !t->narrow) return FG_OK;
    HIPCHK(h, launch_widen_table(ref_of(t), t->bits, h->stream));
    t->narrow = false;
    return FG_OK;
}

// device scalars: [0] overflow flags (u32), [4] fail count (u32), [8] fired-row counter (u64)
// (flags and fail count adjacent: one 8-B fill zeroes both and keeps the counter)
constexpr size_t kScalarBytes = 24;
uint32_t fail_count(const fg_handle* h) { return h->h_scalars.as<uint32_t>()[1]; }
// zero the flags, the fired-row counter (with_out) and -- no job pending -- the fail count, in as
// few fills as the layout allows
int zero_scalars(fg_handle* h, bool with_out) {
    const bool fail = h->jobs.empty();
    if (fail) {
        HIPCHK(h, hipMemsetAsync(h->scalars.p, 0, with_out ? 16 : 8, h->stream));
        h->fail_zeroed = true;
    } else {
        HIPCHK(h, hipMemsetAsync(h->scalars.p, 0, 4, h->stream));
        if (with_out) HIPCHK(h, hipMemsetAsync(h->scalars.as<char>() + 8, 0, 8, h->stream));
    }
    return FG_OK;
}

// Every tile fire goes through here. FG_STAMPS builds with FG_STAMPS set in the environment print
// the fire's phase cycles per wave (k_tile_fire's FSTAMP phases) after each launch.
hipError_t tile_fire_launch(fg_handle* h, TileFire& f, int32_t workgroups, hipStream_t s) {
#ifdef FG_STAMPS
    static DevBuf d_fs;
    const bool st = getenv("FG_STAMPS") != nullptr && d_fs.ensure(64) == hipSuccess;
    if (st) {
        (void)hipMemsetAsync(d_fs.p, 0, 64, s);
        f.m.stamps = d_fs.as<unsigned long long>();
    }
    const hipError_t e = launch_tile_fire(f, workgroups, s);
    if (st) {
        unsigned long long v[8];
        (void)hipMemcpyAsync(v, d_fs.p, sizeof v, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        const double waves = (double)workgroups * kTileFireThreads / 64;
        fprintf(stderr, "[fg stamps] tile_fire split=%d merge=%d srcs=%d dst=%d passes=%d: clear %.0f walk %.0f wait %.0f "
                "insert %.0f sources %.0f barrier %.0f compact %.0f emit %.0f (cycles/wave)\n", f.split, f.merge,
                f.m.n_src, f.m.has_dst, f.n_passes, v[0] / waves, v[1] / waves, v[2] / waves, v[3] / waves,
                v[4] / waves, v[5] / waves, v[6] / waves, v[7] / waves);
        f.m.stamps = nullptr;
    }
    return e;
#else
    (void)h;
    return launch_tile_fire(f, workgroups, s);
#endif
}

int check_overflow(fg_handle* h) {
    // region overflows (bits 0 and 2) are handled by the fail list (settle_jobs)
    unsigned int fl = h->h_scalars.as<unsigned int>()[0];
    if (fl & 2u) return h->fail(FG_EDEVICE, "internal: fired-row buffer overflow");
    if (fl & 8u) return h->fail(FG_EDEVICE, "internal: a tile walk addressed a record past its pass");
    return FG_OK;
}

int lanes_for(int bits) {
    // lanes x regions bounded by the count histogram and, for the two-pass partition, by
    // pass 1's LDS histogram
    int lanes = kMaxLanes;
    while (lanes > 1 && (lanes << bits) > kMaxStageBuckets) lanes >>= 1;
    while (lanes > 2 && bits >= kFineBits && (lanes << bits) > kMaxPart1Fine) lanes >>= 1;
    return lanes;
}

// A new job set starts after every synchronization: zero its fail count.
int job_add(fg_handle* h, MergeJob&& j, int* id) {
    if (h->jobs.empty() && !h->fail_zeroed) HIPCHK(h, hipMemsetAsync(h->scalars.as<char>() + 4, 0, 4, h->stream));
    h->fail_zeroed = false;
    j.bits = h->region_bits;
    if (j.dst) j.dst->changed = true;   // (every table write goes through a job, or sets upper below)
    h->jobs.push_back(std::move(j));
    *id = (int)h->jobs.size() - 1;
    return FG_OK;
}

StagedBatch batch_of(const fg_handle* h, const JobBatch& jb) {
    StagedBatch b{};
    if (!jb.s) {
        b = jb.ext;
        b.shift = h->region_bits - jb.ext_bits;
        return b;
    }
    const Staged* s = jb.s;
    const int l = jb.lane;
    b.bucket_off = s->bucket_off.as<uint32_t>() + ((int64_t)l << s->bits);
    if (s->is_acc) {
        const int64_t at = (int64_t)l * h->acc_cap + s->lane_start[l];
        b.is_acc = 1;
        b.stride = 1;
        b.rec = h->acc_key.as<int64_t>() + at;
        b.cnt_star = h->acc_cs.as<int64_t>() + at;
        b.cnt_null = h->acc_cn.as<int64_t>() + at;
        b.val = h->acc_sum.as<int64_t>() + at;
        if (h->mv) {
            b.val1 = h->acc_v1.as<int64_t>() + at;
            b.val2 = h->acc_v2.as<int64_t>() + at;
        }
    } else if (s->own) {   // a materialized tile pass: narrow records of its own area, from index 0
        b.rec = s->own_rec.as<int64_t>();
        b.rec_first = 0;
        b.vnull = nullptr;
        b.stride = 3;
    } else {
        // narrow records: block-laid from the staged area's base (kRec12Block), the batch's
        // first record by index
        b.rec = s->narrow ? h->st_rec.as<int64_t>()
                          : h->st_rec.as<int64_t>() + ((int64_t)l * h->lane_cap + s->lane_start[l]) * h->st_stride;
        b.rec_first = s->narrow ? (int32_t)((int64_t)l * h->lane_cap + s->lane_start[l]) : 0;
        b.vnull = s->has_null ? h->st_null.as<uint8_t>() + (int64_t)l * h->lane_cap + s->lane_start[l] : nullptr;
        b.stride = s->narrow ? 3 : h->st_stride;
    }
    b.shift = h->region_bits - s->bits;
    return b;
}

void fill_emit(fg_handle* h, MergeParams& p, int64_t wend);

// the operator's value accumulators in a merge's parameters
void set_values(const fg_handle* h, MergeParams* p) {
    p->val_type = h->kvt;
    p->mv = h->mv;
    for (int k = 0; k < kNV; k++) p->vop[k] = h->vop[k];
    for (int a = 0; a < FG_MAX_AGGS; a++) p->agg_slot[a] = h->agg_slot[a];
}

// MergeParams of job `ji` at the current region bits (the general path; callers pick the
// fast variants on a first launch)
// the COUNT(*) of any key stays below 2^32 (the compact merge's u32 counts)
bool ub_cnt_fits(const fg_handle* h) { return h->cnt_bound < ((int64_t)1 << 32); }

int job_params(fg_handle* h, int ji, MergeParams* p) {
    const MergeJob& j = h->jobs[(size_t)ji];
    // the general merge writes the wide layout: a narrow destination is widened first (before the
    // sources' refs are taken -- it may be one of them)
    if (int rc = widen_table(h, j.dst)) return rc;
    std::vector<StagedBatch> sb;
    for (const JobBatch& jb : j.batches) sb.push_back(batch_of(h, jb));
    std::vector<TableRef> srcs;
    // sources known free of NULL counts are read without their cnt_null column; a destination
    // may hold NULL counts iff something merged into it may
    unsigned long long null_mask = 0;
    bool dst_null = false;
    bool src_narrow = false, all_narrow = !j.srcs.empty();
    for (size_t i = 0; i < j.srcs.size(); i++) {
        srcs.push_back(ref_of(j.srcs[i]));
        src_narrow = src_narrow || j.srcs[i]->narrow;
        all_narrow = all_narrow && j.srcs[i]->narrow;
        if (j.srcs[i]->has_null) {
            if (i < 64) null_mask |= 1ull << i;
            dst_null = true;
        }
    }
    if (j.srcs.size() > 64) null_mask = ~0ull;
    for (const JobBatch& jb : j.batches)
        dst_null = dst_null || !jb.s || jb.s->has_null || jb.s->is_acc;   // (restore images, partials)
    if (j.dst) j.dst->has_null = j.dst->has_null || dst_null;
    *p = MergeParams{};
    p->region_bits = h->region_bits;
    p->n_src = (int)srcs.size();
    p->src_narrow = all_narrow ? 2 : src_narrow ? 1 : 0;
    if (srcs.size() <= 2) {   // by value in the arguments (no descriptor copy on the stream)
        for (size_t i = 0; i < srcs.size(); i++) p->src_in[i] = srcs[i];
    } else {
        int rc = arena_put(h, srcs.data(), srcs.size(), &p->src);
        if (rc) return rc;
    }
    p->n_batches = (int)sb.size();
    if (!sb.empty()) {
        int rc = arena_put(h, sb.data(), sb.size(), &p->batches);
        if (rc) return rc;
    }
    set_values(h, p);
    p->has_dst = j.dst ? 1 : 0;
    if (j.dst) p->dst = ref_of(j.dst);
    if (j.emit) fill_emit(h, *p, j.wend);
    p->overflow = h->scalars.as<unsigned int>();
    p->out_count = reinterpret_cast<unsigned long long*>(h->scalars.as<char>() + 8);
    p->fail_list = h->fail_list.as<uint32_t>();
    p->fail_n = reinterpret_cast<uint32_t*>(h->scalars.as<char>() + 4);
    p->fail_cap = kFailCap;
    p->job = ji;
    p->mark_mask = j.mark_mask;
    p->markonly_mask = j.markonly_mask;
    p->emit_marked = j.emit_marked;
    p->dst_mode = j.dst_mode;
    p->src_null_mask = null_mask;
    return FG_OK;
}

// ---- tile staging (fg_kernels.h) ------------------------------------------------------------
TilePass tile_pass_of(const Staged* s, int lane) {
    TilePass tp{};
    tp.rec = s->t_rec.p;
    tp.dt = s->t_dt.as<uint32_t>();
    tp.n = s->t_n;
    tp.nt = s->t_nt;
    tp.mt = s->t_mt;
    tp.nc = s->t_nc;
    tp.bits = s->bits;
    tp.lane = lane;
    tp.btot = s->t_btot.p ? s->t_btot.as<uint32_t>() : nullptr;
    return tp;
}

// TileFire of tile job `ji` at the current region bits (retry: regions in retry_list)
int tile_job_params(fg_handle* h, int ji, TileFire* f) {
    const MergeJob& j = h->jobs[(size_t)ji];
    std::vector<TilePass> tps;
    for (const JobBatch& jb : j.batches) tps.push_back(tile_pass_of(jb.s, jb.lane));
    *f = TileFire{};
    MergeParams& p = f->m;
    p.region_bits = h->region_bits;
    set_values(h, &p);
    if (j.emit) {
        fill_emit(h, p, j.wend);
        p.emit = 1;
    }
    std::vector<TableRef> srcs;
    for (SliceTable* x : j.srcs) {
        srcs.push_back(ref_of(x));
        if (x->narrow) p.src_narrow = 1;
    }
    p.n_src = (int)srcs.size();
    if (srcs.size() <= 2) {   // by value in the arguments (no descriptor copy on the stream)
        for (size_t i = 0; i < srcs.size(); i++) p.src_in[i] = srcs[i];
    } else {
        int rc = arena_put(h, srcs.data(), srcs.size(), &p.src);
        if (rc) return rc;
    }
    p.has_dst = j.dst ? 1 : 0;
    if (j.dst) p.dst = ref_of(j.dst);
    p.overflow = h->scalars.as<unsigned int>();
    p.out_count = reinterpret_cast<unsigned long long*>(h->scalars.as<char>() + 8);
    p.fail_list = h->fail_list.as<uint32_t>();
    p.fail_n = reinterpret_cast<uint32_t*>(h->scalars.as<char>() + 4);
    p.fail_cap = kFailCap;
    p.job = ji;
    f->n_passes = (int32_t)tps.size();
    f->tbits = j.tbits;
    if (tps.size() <= 2) {   // (one or two passes per lane -- TUMBLE, HOP / CUMULATE flushes: in the
        f->one = tps[0];     // kernel's arguments, no descriptor copy queued before the fire)
        if (tps.size() == 2) f->two = tps[1];
        return FG_OK;
    }
    return arena_put(h, tps.data(), tps.size(), &f->passes);
}

// Split every slice table's regions 2^b -> 2^nb (k_split_table). Staged passes keep their
// bucketing (the merge reads a region's records through its parent bucket); new passes
// bucket at nb. The slice lanes stay until the lanes above lanes_for(nb) drain.
int materialize_lane(fg_handle* h, int l);
int grow(fg_handle* h, int nb) {
    const int sh = nb - h->region_bits;
    if (sh <= 0) return FG_OK;
    if (nb > kMaxRegionBits) return h->fail(FG_ECAPACITY, "internal: region bits above %d", kMaxRegionBits);
    // a staged tile pass is read at most kTileMaxSub regions per bucket by the materialize
    // kernels: a lane whose tile passes would pass that bound at nb is materialized first, at
    // the current bits (its regular staged pass is then read through its parent buckets)
    for (int l = 0; l < h->lanes; l++) {
        bool deep = false;
        for (const Staged* s : h->lane[l].passes) deep = deep || (s->tiles && nb - s->bits + kTileBits > 6);
        if (!deep) continue;
        if (int rc = materialize_lane(h, l)) return rc;
    }
    const int64_t P2 = (int64_t)1 << nb;
    std::vector<std::unique_ptr<DevBuf>> old;   // freed once the split kernels are done
    auto split = [&](SliceTable* t) -> int {
        if (int rc0 = widen_table(h, t)) return rc0;   // (the split copies the wide layout)
        std::unique_ptr<DevBuf> nd(new DevBuf()), nc(new DevBuf());
        HIPCHK(h, nd->ensure(sizeof(int64_t) * table_cols(h->mv) * (size_t)table_cap(h->mv) * P2));
        HIPCHK(h, nc->ensure(sizeof(uint32_t) * P2));
        HIPCHK(h, launch_split_table(ref_of(t), TableRef{nd->as<int64_t>(), nc->as<uint32_t>()}, t->bits,
                                     nb - t->bits, h->mv, h->stream));
        t->data.swap(*nd);
        t->counts.swap(*nc);
        t->bits = nb;
        old.push_back(std::move(nd));
        old.push_back(std::move(nc));
        return FG_OK;
    };
    int rc;
    for (auto& kv : h->tables)
        if ((rc = split(kv.second.get()))) return rc;
    for (auto& t : h->deferred)
        if ((rc = split(t.get()))) return rc;
    for (auto* m : {&h->re_new, &h->re_delta})
        for (auto& kv : *m)
            if ((rc = split(kv.second.get()))) return rc;
    if (h->re_chain && (rc = split(h->re_chain.get()))) return rc;
    for (auto& t : h->re_tmp)
        if (t && (rc = split(t.get()))) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    old.clear();
    h->table_pool.clear();   // pooled tables have the old layout
    h->region_bits = nb;
    h->P = 1 << nb;
    h->lanes_target = lanes_for(nb);
    h->F = h->lanes << nb;
    // (the ingest scratch grows at the next pass: a pass in progress keeps its buffers)
    h->grows++;
    return FG_OK;
}

int merge_grid(const fg_handle* h);

// After the synchronization that follows a job set (h_scalars read back): while regions
// failed, split the regions and redo exactly the failed ones' children. The jobs' inputs
// (staged lanes, tables) are untouched until this returns.
int retry_failed(fg_handle* h) {
    while (!h->jobs.empty() && fail_count(h) > 0) {
        const uint32_t nf = fail_count(h);
        if (nf > (uint32_t)kFailCap) return h->fail(FG_ECAPACITY, "internal: %u failed regions in one merge set", nf);
        if (h->region_bits >= kMaxRegionBits)
            return h->fail(FG_ECAPACITY,
                           "state region overflow at %d regions (> %d distinct keys of one region in a slice): "
                           "more keys per subtask than one operator holds; raise the parallelism",
                           1 << kMaxRegionBits, kRegionCap);
        HIPCHK(h, h->h_fail.ensure(4 * (size_t)nf));
        HIPCHK(h, hipMemcpyAsync(h->h_fail.p, h->fail_list.p, 4 * (size_t)nf, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        std::map<int, std::vector<int32_t>> per_job;
        for (uint32_t i = 0; i < nf; i++) {
            const uint32_t e = h->h_fail.as<uint32_t>()[i];
            per_job[(int)(e >> kFailJobShift)].push_back((int32_t)(e & ((1u << kFailJobShift) - 1)));
        }
        int rc = grow(h, h->region_bits + 1);
        if (rc) return rc;
        h->arena_used = 0;
        HIPCHK(h, hipMemsetAsync(h->scalars.p, 0, 8, h->stream));   // flags and fail count
        for (auto& kv : per_job) {
            MergeJob& j = h->jobs[(size_t)kv.first];
            const int sh = h->region_bits - j.bits;
            std::vector<int32_t> regs;
            for (int32_t r : kv.second)
                for (int c = 0; c < (1 << sh); c++) regs.push_back((r << sh) | c);
            j.bits = h->region_bits;
            if (j.tile) {   // one region per item, the bucket's records filtered by region
                TileFire f{};
                rc = tile_job_params(h, kv.first, &f);
                if (rc) return rc;
                rc = arena_put(h, regs.data(), regs.size(), &f.m.retry_list);
                if (rc) return rc;
                f.m.n_retry = (int)regs.size();
                KTimer kt(h, j.kclass, 0);
                HIPCHK(h, tile_fire_launch(h, f, std::min<int>((int)regs.size(), merge_grid(h)), h->stream));
                continue;
            }
            MergeParams p{};
            rc = job_params(h, kv.first, &p);
            if (rc) return rc;
            rc = arena_put(h, regs.data(), regs.size(), &p.retry_list);
            if (rc) return rc;
            p.n_retry = (int)regs.size();
            KTimer kt(h, j.kclass, 0);
            HIPCHK(h, launch_merge(p, std::min<int>((int)regs.size(), merge_grid(h)), h->stream));
        }
        HIPCHK(h, hipMemcpyAsync(h->h_scalars.p, h->scalars.p, kScalarBytes, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->arena_used = 0;
    }
    return FG_OK;
}
int settle_jobs(fg_handle* h) {
    const int rc = retry_failed(h);
    for (MergeJob& j : h->jobs)   // (tile passes the jobs read may be reused from the pool now)
        for (JobBatch& jb : j.batches)
            if (jb.s) jb.s->busy = false;
    h->jobs.clear();
    // tables freed while the jobs ran go back to the pool (or away, after a split)
    for (auto& t : h->deferred)
        if (t->bits == h->region_bits) h->table_pool.push_back(std::move(t));
    h->deferred.clear();
    return rc;
}

// Reduce the slice lanes to lanes_for(region bits) once the lanes above it hold nothing
// (after a split to 2^13 regions, two lanes keep the two-pass partition).
// ---- asynchronous advance: publish a fire's results, complete it later -----------------
// The fires of fg_advance_progress_async end with k_publish_words (the scalars -- overflow
// flags, fired-row count, fail count -- into coherent host memory, then a sequence word)
// instead of a D2H copy and a stream synchronization; the host's bookkeeping (tables freed,
// lanes released) is done at once, tables freed meanwhile are held (table_free) and the staged
// passes stay intact until the next ingest, which completes the fire first -- so a region retry
// still finds its inputs.
int publish_fire(fg_handle* h, int kclass) {
    h->fire_seq++;
    HIPCHK(h, launch_publish_words(h->scalars.as<unsigned long long>(), (int32_t)(kScalarBytes / 8),
                                   h->h_fire.as<unsigned long long>(), h->fire_seq, h->stream));
    h->fire_pending = true;
    h->fire_kclass = kclass;
    h->fire_before = h->out_n;
    return FG_OK;
}
int complete_fire(fg_handle* h) {
    if (!h->fire_pending) return FG_OK;
    h->fire_pending = false;
    const volatile unsigned long long* sq = h->h_fire.as<unsigned long long>() + kScalarBytes / 8;
    for (int64_t spin = 0; *sq != h->fire_seq; spin++) {
        if (spin > (1 << 12) && hipStreamQuery(h->stream) != hipErrorNotReady) {
            HIPCHK(h, hipStreamSynchronize(h->stream));
            if (*sq != h->fire_seq) return h->fail(FG_EDEVICE, "internal: fire scalars never arrived");
            break;
        }
    }
    std::memcpy(h->h_scalars.p, h->h_fire.p, kScalarBytes);
    int rc = settle_jobs(h);   // regions that overflowed: split and redone (their rows counted)
    if (rc) return rc;
    rc = check_overflow(h);
    if (rc) return rc;
    h->out_n = (int64_t)h->h_scalars.as<unsigned long long>()[1];
    h->kstat[h->fire_kclass].rows += h->out_n - h->fire_before;
    h->pending_out = 0;
    if (h->fire_rows_open) {   // the advance returned before its rows were known
        h->rows_fired += h->out_n - h->fire_rows_base;
        h->fire_rows_open = false;
    }
    return FG_OK;
}

void maybe_reduce_lanes(fg_handle* h) {
    if (h->lanes_target <= 0 || h->lanes_target >= h->lanes) return;
    for (int l = h->lanes_target; l < h->lanes; l++)
        if (h->lane[l].q != kEmptyLane) return;
    h->lanes = h->lanes_target;
    h->F = h->lanes << h->region_bits;
    h->q_guess = kEmptyLane;
}

int ensure_out(fg_handle* h, int64_t need);
int fire_collect(fg_handle* h);

// zero the overflow word and the fired-row counter once per advance
int reset_out_count(fg_handle* h) {
    if (!h->out_count_reset) {
        if (int rc = zero_scalars(h, true)) return rc;
        // rows fired by late elements, or by async advances not yet collected, lead the advance's rows
        if (h->adv_base + h->late_rows > 0) {
            Words16 w{};
            w.v[0] = (unsigned long long)(h->adv_base + h->late_rows);
            w.n = 1;
            HIPCHK(h, launch_store_words(reinterpret_cast<unsigned long long*>(h->scalars.as<char>() + 8), w, h->stream));
        }
        h->out_count_reset = true;
    }
    return FG_OK;
}

// A slice whose windows all fired: freed now, or -- with allowed lateness -- kept until the
// cleanup time of its last window (WindowOperator.registerCleanupTimer :630-642).
void retire(fg_handle* h, int64_t se, int64_t last_window_end) {
    if (!h->retain) {
        table_free(h, se);
        return;
    }
    const int64_t at = ds_cleanup(last_window_end, h->lateness);
    if (at <= h->current_progress) table_free(h, se);
    else h->retire_at[se] = at;
}

struct FireRange {   // windows whose timers fire in (prev, wm]
    int64_t prev, wm;
};

void fill_emit(fg_handle* h, MergeParams& p, int64_t wend) {
    p.emit = 1;
    // local phase: the emitted "window" is the slice itself (LocalAggCombiner emits
    // (key, acc, slice_end) rows)
    p.wstart = h->local ? jsub(wend, h->w.slice) : window_start(h->windowed ? h->inner : h->w, wend);
    p.wend = wend;
    p.out_ts = jsub(wend, 1);
    p.num_aggs = h->cfg.num_aggs;
    for (int a = 0; a < h->cfg.num_aggs; a++) {
        p.aggs[a] = h->cfg.aggs[a];
        p.out_agg[a] = h->o_agg[a].as<int64_t>();
    }
    p.out_key = h->o_key.as<int64_t>();
    p.out_ws = h->o_ws.as<int64_t>();
    p.out_we = h->o_we.as<int64_t>();
    p.out_null = h->o_null.as<uint8_t>();
    p.out_rowtime = h->cfg.mode == FG_MODE_DATASTREAM ? h->o_rt.as<int64_t>() : nullptr;
    p.out_cap = h->out_cap;
}

bool staged_any(const fg_handle* h) {
    for (int l = 0; l < h->lanes; l++)
        if (h->lane[l].q != kEmptyLane) return true;
    return false;
}
int64_t staged_records(const fg_handle* h) {
    int64_t n = 0;
    for (int l = 0; l < h->lanes; l++) n += h->lane[l].fill + h->lane[l].acc_fill;
    return n;
}
int64_t min_staged_slice_end(const fg_handle* h) {
    int64_t m = JMAX;
    for (int l = 0; l < h->lanes; l++)
        if (h->lane[l].q != kEmptyLane) m = std::min(m, slice_end_of(h, h->lane[l].q));
    return m;
}

// empty lane l; a pass returns to the pool once no lane holds its records
void release_lane(fg_handle* h, int l) {
    for (Staged* s : h->lane[l].passes) {
        if (--s->refs > 0) continue;
        for (size_t i = 0; i < h->passes.size(); i++) {
            if (h->passes[i].get() != s) continue;
            h->pass_pool.push_back(std::move(h->passes[i]));
            h->passes.erase(h->passes.begin() + (long)i);
            break;
        }
    }
    h->lane[l] = Lane{};
}

int merge_grid(const fg_handle* h) { return std::min(h->P, h->merge_grid); }

// A Staged from the pool that no unsettled job reads (or a new one)
std::unique_ptr<Staged> pass_from_pool(fg_handle* h) {
    std::unique_ptr<Staged> s;
    for (size_t i = h->pass_pool.size(); i-- > 0;) {
        if (h->pass_pool[i]->busy) continue;
        s = std::move(h->pass_pool[i]);
        h->pass_pool.erase(h->pass_pool.begin() + (long)i);
        break;
    }
    if (!s) s.reset(new Staged());
    return s;
}

// Lane l's tile passes become regular narrow staged passes (their own record areas) at the
// current regions: per-region counts (k_tile_count), their scan, the records written by region
// (k_tile_scatter). Every consumer other than the fire straight from the tiles -- a flush into
// the slice table, a checkpoint, a restore re-fire, the heavy pass -- then reads the lane as it
// reads any staged pass.
int split_buffers(fg_handle* h, int nb, int64_t fill, uint32_t chunk, bool icnt, TileSplit* out);
int materialize_lane(fg_handle* h, int l) {
    Lane& ln = h->lane[l];
    for (size_t i = 0; i < ln.passes.size(); i++) {
        Staged* s = ln.passes[i];
        if (!s->tiles) continue;
        const int bits = h->region_bits;
        if (bits - s->bits + kTileBits > 6)
            return h->fail(FG_ECAPACITY, "internal: regions split %d times since a tile pass", bits - s->bits);
        std::unique_ptr<Staged> m = pass_from_pool(h);
        const TilePass tp = tile_pass_of(s, l);
        const int64_t P = (int64_t)1 << bits;
        HIPCHK(h, h->tile_hist.ensure(4 * (size_t)(P + 1)));
        HIPCHK(h, h->scan_tmp.ensure(4 * scan_tmp_words(P)));
        HIPCHK(h, m->bucket_off.ensure(sizeof(uint32_t) * (((size_t)kMaxLanes << bits) + 1)));
        HIPCHK(h, m->own_rec.ensure((size_t)(s->lane_n[l] / 64 + 2) * kRec12Block));
        uint32_t* bo = m->bucket_off.as<uint32_t>() + ((int64_t)l << bits);
        {
            KTimer kt(h, K_TILE_MAT, s->lane_n[l]);
            // items of at most ~kTileMatChunk records (a hot key's bucket spread over many)
            TileFire f{};
            f.one = tp;
            f.n_passes = 1;
            f.tbits = s->bits;
            f.split = 1;
            f.m.overflow = h->scalars.as<unsigned int>();
            int rc = split_buffers(h, 1 << (s->bits - kTileBits), s->lane_n[l], kTileMatChunk, true, &f.sp);
            if (rc) return rc;
            f.sp.gpre[0] = 0;
            f.sp.gpre[1] = tp.nt;
            HIPCHK(h, launch_tile_plan(f, h->stream));
            const int wg = 4 * h->merge_grid;
            uint32_t* hist = h->tile_hist.as<uint32_t>();
            HIPCHK(h, hipMemsetAsync(hist, 0, 4 * (size_t)P, h->stream));
            HIPCHK(h, launch_tile_count(tp, bits, f.sp, hist, wg, h->stream));
            HIPCHK(h, launch_scan_u32(hist, bo, P, h->scan_tmp.as<uint32_t>(), h->stream));
            // (the scan's bases copied: each item reserves its regions' blocks from them)
            HIPCHK(h, hipMemcpyAsync(hist, bo, 4 * (size_t)P, hipMemcpyDeviceToDevice, h->stream));
            HIPCHK(h, launch_tile_scatter(tp, bits, f.sp, hist, m->own_rec.p, wg, h->stream));
        }
        m->bits = bits;
        m->is_acc = false;
        m->has_null = false;
        m->narrow = true;
        m->tiles = false;
        m->own = true;
        m->busy = false;
        m->skew = s->skew;
        for (int q = 0; q < kMaxLanes; q++) m->lane_start[q] = m->lane_n[q] = 0;
        m->lane_n[l] = s->lane_n[l];
        m->refs = 1;
        ln.passes[i] = m.get();
        h->passes.push_back(std::move(m));
        if (--s->refs == 0) {
            for (size_t k = 0; k < h->passes.size(); k++) {
                if (h->passes[k].get() != s) continue;
                h->pass_pool.push_back(std::move(h->passes[k]));
                h->passes.erase(h->passes.begin() + (long)k);
                break;
            }
        }
    }
    return FG_OK;
}

// Lane l fires straight from its tile passes: every pass a tile pass of the same bits, no skew,
// COUNT(*) below 2^32
// (the split fire walks at most kMaxTilePasses passes: a skewed lane of more passes is materialized;
// the plain fire takes any number -- a window of many small micro-batches stays on the tiles)
bool tile_fire_ok(const fg_handle* h, const Lane& ln, bool allow_skew = false) {
    if (ln.passes.empty() || ln.acc_fill != 0 || ln.fill >= ((int64_t)1 << 32) || h->mv) return false;
    bool skew = false;
    for (const Staged* s : ln.passes) {
        if (!s->tiles || (s->skew && !allow_skew) || s->bits != ln.passes[0]->bits) return false;
        skew = skew || s->skew;
    }
    return !(skew && ln.passes.size() > (size_t)kMaxTilePasses);
}

constexpr int64_t kTileSpreadMin = 1 << 18;     // records of a lane worth a spread (split) fire
constexpr int64_t kTileSpreadChunk = 1 << 12;   // smallest chunk item of a spread fire
// A skewed tile pass stays on the tiles (FG_TILE_SPLIT): TUMBLE windows and local-phase slices,
// whose lanes fire straight from the tiles by the split fire (anything else materializes them)
bool tile_split_ok(const fg_handle* h) { return h->tile_split && (h->w.kind == TUMBLE || h->local); }

// The split fire of a lane holding a skewed tile pass (fg_kernels.h TileSplit): k_tile_plan cuts
// the buckets above max(kTileChunk, the lane's mean) into chunk items, k_tile_fire aggregates
// every item (chunks into partial entries), and again over the split buckets (merge = 1), each
// merging its chunks -- with the job's source and destination tables when it has them
// into its rows. f is the job's TileFire (tile_job_params).
// The plan's buffers (TileSplit) for `fill` records over nb buckets in items of at least `chunk`
// records (0: kTileChunk), the counts zeroed on the stream; materialize also keeps per-item
// sub-region counts (icnt).
int split_buffers(fg_handle* h, int nb, int64_t fill, uint32_t chunk, bool icnt, TileSplit* out) {
    const int64_t max_chunks = fill / (chunk ? chunk : kTileChunk) + nb + 1;   // (chunks >= chunk records, + 1 per bucket)
    const int64_t max_items = max_chunks + nb;
    const int64_t part_cap = icnt ? 1 : std::min<int64_t>(fill, max_chunks * (kTileSlots + 1)) + 1;
    if (part_cap >= ((int64_t)1 << 32) || max_items >= ((int64_t)1 << 31))
        return h->fail(FG_ECAPACITY, "internal: split plan of %lld records above its index range", (long long)fill);
    HIPCHK(h, h->sp_items.ensure(sizeof(TileItem) * (size_t)max_items));
    HIPCHK(h, h->sp_n.ensure(16));
    HIPCHK(h, h->sp_split.ensure(4 * 3 * (size_t)nb));
    HIPCHK(h, h->sp_parts.ensure(4 * 2 * (size_t)max_chunks));
    HIPCHK(h, h->sp_pkey.ensure(4 * (size_t)part_cap));
    HIPCHK(h, h->sp_pcs.ensure(4 * (size_t)part_cap));
    HIPCHK(h, h->sp_pv.ensure(8 * (size_t)part_cap));
    HIPCHK(h, h->sp_bfail.ensure(4 * (size_t)nb));
    if (icnt) HIPCHK(h, h->sp_icnt.ensure(4 * (size_t)kTileMaxSub * (size_t)max_items));
    HIPCHK(h, hipMemsetAsync(h->sp_n.p, 0, 16, h->stream));   // n_items, n_split, part_fill, next_item
    TileSplit& sp = *out;
    sp = TileSplit{};
    sp.items = h->sp_items.as<TileItem>();
    sp.n_items = h->sp_n.as<uint32_t>();
    sp.n_split = h->sp_n.as<uint32_t>() + 1;
    sp.part_fill = h->sp_n.as<uint32_t>() + 2;
    sp.next_item = h->sp_n.as<uint32_t>() + 3;
    sp.max_items = (int32_t)max_items;
    sp.max_split = nb;
    sp.split_b = h->sp_split.as<int32_t>();
    sp.split_c0 = sp.split_b + nb;
    sp.split_k = sp.split_b + 2 * nb;
    sp.part_off = h->sp_parts.as<uint32_t>();
    sp.part_n = sp.part_off + max_chunks;
    sp.part_cap = (uint32_t)part_cap;
    sp.p_key = h->sp_pkey.as<int32_t>();
    sp.p_cs = h->sp_pcs.as<uint32_t>();
    sp.p_v = h->sp_pv.as<unsigned long long>();
    sp.bfail = h->sp_bfail.as<uint32_t>();
    sp.chunk = chunk;
    sp.icnt = icnt ? h->sp_icnt.as<uint32_t>() : nullptr;
    return FG_OK;
}

int tile_split_fire(fg_handle* h, const Lane& ln, TileFire& f, uint32_t chunk) {
    const int nb = 1 << (f.tbits - kTileBits);
    if (int rc = split_buffers(h, nb, ln.fill, chunk, false, &f.sp)) return rc;
    TileSplit& sp = f.sp;
    const int64_t max_items = sp.max_items;
    int32_t g = 0;
    for (size_t i = 0; i < ln.passes.size(); i++) {
        sp.gpre[i] = g;
        g += ln.passes[i]->t_nt;
    }
    sp.gpre[ln.passes.size()] = g;
    f.split = 1;
    f.hot = h->tile_hot ? 1 : 0;
    HIPCHK(h, launch_tile_plan(f, h->stream));
    HIPCHK(h, tile_fire_launch(h, f, (int)std::min<int64_t>(max_items, h->merge_grid), h->stream));
    TileFire fm = f;   // the split buckets: their chunks' partial entries merged (+ tables, rows)
    fm.merge = 1;
    fm.hot = 0;
    HIPCHK(h, tile_fire_launch(h, fm, std::min(nb, h->merge_grid), h->stream));
    return FG_OK;
}

// Plan the skewed regions of one lane's merge (k_heavy_plan): regions over
// max(kHeavyMin, 8 x mean) staged records, cut into kHeavyChunk-record chunks.
int plan_heavy(fg_handle* h, const StagedBatch* d_sb, int nb, int64_t fill, HeavyPlan* hp) {
    const int64_t threshold = std::max<int64_t>(kHeavyMin, 8 * fill / h->P);
    const int64_t max_chunks = fill / kHeavyChunk + fill / threshold + 2;
    if (max_chunks > h->hv_max_chunks) {
        const size_t e = (size_t)max_chunks * kPartStride;
        HIPCHK(h, h->hv_clist.ensure(4 * (size_t)max_chunks));
        HIPCHK(h, h->hv_v0.ensure(8 * (size_t)max_chunks));
        HIPCHK(h, h->hv_v1.ensure(8 * (size_t)max_chunks));
        HIPCHK(h, h->hv_pn.ensure(4 * (size_t)max_chunks));
        HIPCHK(h, h->hv_key.ensure(8 * e));
        HIPCHK(h, h->hv_cs.ensure(8 * e));
        HIPCHK(h, h->hv_cn.ensure(8 * e));
        HIPCHK(h, h->hv_sum.ensure(8 * e));
        h->hv_max_chunks = max_chunks;
    }
    if (h->mv) {
        const size_t e = (size_t)h->hv_max_chunks * kPartStride;
        HIPCHK(h, h->hv_mv1.ensure(8 * e));
        HIPCHK(h, h->hv_mv2.ensure(8 * e));
    }
    HIPCHK(h, h->hv_flags.ensure((size_t)h->P));
    HIPCHK(h, h->hv_list.ensure(4 * (size_t)h->P));
    HIPCHK(h, h->hv_chunk0.ensure(4 * ((size_t)h->P + 1)));
    HIPCHK(h, h->hv_n.ensure(8));
    hp->batches = d_sb;
    hp->n_batches = nb;
    hp->region_bits = h->region_bits;
    hp->threshold = threshold;
    hp->chunk = kHeavyChunk;
    hp->max_chunks = (int32_t)std::min<int64_t>(h->hv_max_chunks, INT32_MAX);
    hp->val_type = h->kvt;
    hp->heavy = h->hv_flags.as<uint8_t>();
    hp->region_list = h->hv_list.as<int32_t>();
    hp->n_list = h->hv_n.as<int32_t>();
    hp->chunk0 = h->hv_chunk0.as<int32_t>();
    hp->chunk_list = h->hv_clist.as<int32_t>();
    hp->chunk_v0 = h->hv_v0.as<int64_t>();
    hp->chunk_v1 = h->hv_v1.as<int64_t>();
    hp->part_key = h->hv_key.as<int64_t>();
    hp->part_cs = h->hv_cs.as<int64_t>();
    hp->part_cn = h->hv_cn.as<int64_t>();
    hp->part_sum = h->hv_sum.as<int64_t>();
    hp->part_v1 = h->mv ? h->hv_mv1.as<int64_t>() : nullptr;
    hp->part_v2 = h->mv ? h->hv_mv2.as<int64_t>() : nullptr;
    hp->mv = h->mv ? 1 : 0;
    for (int k = 0; k < kNV; k++) hp->vop[k] = h->vop[k];
    hp->part_n = h->hv_pn.as<uint32_t>();
    hp->overflow = h->scalars.as<unsigned int>();
    KTimer kt(h, K_HEAVY, 0);
    HIPCHK(h, launch_heavy_plan(*hp, h->stream));
    return FG_OK;
}

// RecordsWindowBuffer.flush (:108-119) + AggCombiner.combine (:76-115): merge staged slice
// lanes into their slice tables -- every lane, or (only_fired) the lanes whose slice is
// fired at the current progress, the only ones a window firing now can read; the others
// stay staged (their merge order does not change results beyond f64 summation order).
// With `fire` (TUMBLE only), a lane whose window's timer fires in this advance is combined
// and fired in the same pass: its rows are emitted straight from LDS and the slice is
// never written back (SliceUnsharedWindowAggProcessor.fireWindow + clearWindow, :46-54 /
// AbstractWindowAggProcessor.java:200-206).
int flush_lanes(fg_handle* h, const std::vector<int>& sel_in, const FireRange* fire) {
    if (sel_in.empty()) return FG_OK;
    if (int rc0 = complete_fire(h)) return rc0;   // (one fire's rows and scalars at a time)
    std::vector<int> sel = sel_in;   // slice order: windows fired by the flush fire in order
    std::sort(sel.begin(), sel.end(), [&](int a, int b) { return h->lane[a].q < h->lane[b].q; });
    // flags (and out_count unless this advance already counts rows; and the fail count when no
    // job is pending) zeroed by one fill: reset_out_count and job_add then need none of their own
    bool zeroed_out = false;
    if (h->out_count_reset) {
        if (int rc0 = zero_scalars(h, false)) return rc0;   // keep out_count
    } else {
        if (int rc0 = zero_scalars(h, true)) return rc0;
        zeroed_out = true;
    }
    std::vector<int64_t> fired_tables, retained;
    bool any_emit = false;
    int fire_class = K_FLUSH_FIRE;   // kernel class credited with the fired rows
    int rc;
    for (int l : sel) {
        const Lane& ln = h->lane[l];
        const int64_t se = slice_end_of(h, ln.q);
        bool lane_tiles = false;
        for (const Staged* st : ln.passes) lane_tiles = lane_tiles || st->tiles;
        if (lane_tiles) {
            // tile passes: a TUMBLE window (or a local slice) due now fires straight from the
            // tiles; anything else reads the lane's records once they are materialized
            const int64_t trig0 = trigger_time(h->w, se);
            const bool due0 = fire && se != JMAX && trig0 > fire->prev && trig0 <= fire->wm;
            const bool fire0 = fire && (h->local || (h->w.kind == TUMBLE && due0));
            SliceTable* t0 = nullptr;
            rc = table_get(h, se, false, &t0);
            if (rc) return rc;
            if (fire0 && !refire_slice(h, se) && !(h->retain && !h->local) && (!t0 || t0->upper == 0) &&
                tile_fire_ok(h, ln, tile_split_ok(h))) {
                const int64_t ub = std::min<int64_t>(ln.fill, kStateCapMax);
                if (zeroed_out && !h->out_count_reset && h->adv_base + h->late_rows == 0) h->out_count_reset = true;
                rc = reset_out_count(h);
                if (rc) return rc;
                rc = ensure_out(h, h->out_n + h->pending_out + ub);
                if (rc) return rc;
                h->pending_out += ub;
                MergeJob job;
                for (Staged* st : ln.passes) {
                    job.batches.push_back(JobBatch{st, l, StagedBatch{}, 0});
                    st->busy = true;
                }
                job.emit = true;
                job.wend = se;
                job.kclass = K_TILE_FIRE;
                job.tile = true;
                job.tbits = ln.passes[0]->bits;
                int ji = 0;
                rc = job_add(h, std::move(job), &ji);
                if (rc) return rc;
                TileFire f{};
                rc = tile_job_params(h, ji, &f);
                if (rc) return rc;
                bool skewed = false;
                for (const Staged* st : ln.passes) skewed = skewed || st->skew;
                // a lane of fewer buckets than CUs (a small key space, configs[0]) is split too, into
                // ~2 items per CU: one workgroup per bucket would leave most of the GPU idle
                const int nbk = 1 << (f.tbits - kTileBits);
                const bool spread = h->tile_split && nbk < h->merge_grid && ln.fill >= kTileSpreadMin &&
                                    ln.passes.size() <= (size_t)kMaxTilePasses;
                const uint32_t chunk =
                    skewed ? h->tile_chunk : (uint32_t)std::max<int64_t>(kTileSpreadChunk, ln.fill / (2 * h->merge_grid));
                {
                    KTimer kt(h, skewed || spread ? K_TILE_SPLIT : K_TILE_FIRE, ln.fill);
                    if (skewed || spread) {
                        rc = tile_split_fire(h, ln, f, chunk);
                        if (rc) return rc;
                    } else {
                        HIPCHK(h, tile_fire_launch(h, f, std::min(1 << (f.tbits - kTileBits), h->merge_grid), h->stream));
                    }
                }
                if (t0) fired_tables.push_back(se);
                any_emit = true;
                fire_class = K_TILE_FIRE;
                continue;
            }
            if (refire_slice(h, se) || !h->tile_state) {
                rc = materialize_lane(h, l);
                if (rc) return rc;
                lane_tiles = false;
            }
        }
        if (refire_slice(h, se)) {
            // after a restore, records of a slice whose windows fired before the checkpoint:
            // their state (re_new) and their keys (re_delta, at the window their timer chain
            // starts from: the slice's own, or for a record accepted late the first window not
            // fired at its arrival, AbstractWindowAggProcessor.java:148-156)
            SliceTable *T = nullptr, *D = nullptr;
            rc = side_create(h, h->re_new, se, &T);
            if (rc) return rc;
            int64_t U = se;
            while (U != JMAX && trigger_time(h->w, U) <= h->arrival_progress) U = jadd(U, h->w.slice);
            const bool ds = h->cfg.mode == FG_MODE_DATASTREAM;   // (per-window state: no chains)
            if (!ds) {
                rc = side_create(h, h->re_delta, U, &D);
                if (rc) return rc;
            }
            for (SliceTable* x : {T, D}) {
                if (!x) continue;
                MergeJob job;
                for (Staged* st : ln.passes) job.batches.push_back(JobBatch{st, l, StagedBatch{}, 0});
                if (x->upper > 0) job.srcs.push_back(x);
                job.dst = x;
                job.kclass = K_FLUSH;
                int ji = 0;
                rc = job_add(h, std::move(job), &ji);
                if (rc) return rc;
                MergeParams p{};
                rc = job_params(h, ji, &p);
                if (rc) return rc;
                KTimer kt(h, K_FLUSH, ln.fill);
                HIPCHK(h, launch_merge(p, merge_grid(h), h->stream));
                x->upper = std::min<int64_t>(x->upper + ln.fill + ln.acc_fill, kStateCapMax);
                x->changed = true;
            }
            continue;
        }
        const int64_t trig = trigger_time(h->w, se);
        const bool due = fire && se != JMAX && trig > fire->prev && trig <= fire->wm;
        // local phase: every fired slice lane emits its partial accumulators
        const bool fire_now = fire && (h->local || (h->w.kind == TUMBLE && due));
        // a slice fired here whose state is not kept needs no table unless one exists (no fill
        // of an empty table's counts per fire)
        SliceTable* t = nullptr;
        rc = table_get(h, se, !(fire_now && !(h->retain && !h->local)), &t);
        if (rc) return rc;
        // CUMULATE: the step window W = se fires now -- combine the staged slice with the
        // first slice's state, write the state back (unless W is the last window) and emit
        // W in one pass, instead of a flush into the slice table and a fire re-reading it
        // (CumulativeSliceAssigner.mergeSlices :359-370 + SliceSharedWindowAggProcessor.fireWindow)
        // (only when every earlier step window of this cumulative window fired in an earlier
        // advance, so that no earlier window still has to fire from the unextended state)
        // (not while a restore re-fire is pending: the re-fire folds the new state of this
        // cumulative window's earlier slices into its first slice first -- advance_progress runs
        // it after this flush -- and fire_windows then fires W from the complete state)
        bool cum_fire = !h->local && h->w.kind == CUMULATE && due && h->refire_hi == JMIN;
        if (cum_fire) {
            const int64_t ws0 = window_start(h->w, se);
            const int64_t prev_w = jsub(se, h->w.slice);
            cum_fire = se == jadd(ws0, h->w.slice) || trigger_time(h->w, prev_w) <= fire->prev;
        }
        SliceTable* F = nullptr;       // first slice's table of W's cumulative window
        SliceTable* dstt = t;          // table written by this merge (null: none)
        MergeJob job;
        if (t && t->upper > 0) job.srcs.push_back(t);
        int64_t cum_first = 0, cum_last = 0;
        if (cum_fire) {
            const int64_t ws = window_start(h->w, se);
            cum_first = jadd(ws, h->w.slice);
            cum_last = jadd(ws, h->w.size);
            if (se != cum_first) {
                rc = table_get(h, cum_first, se != cum_last, &F);
                if (rc) return rc;
                if (F && F->upper > 0) job.srcs.push_back(F);
            }
            dstt = se == cum_last ? nullptr : (se == cum_first ? t : F);
        } else if (fire_now) {
            dstt = h->retain && !h->local ? t : nullptr;   // allowed lateness: the fired window keeps its state
        }
        int64_t ub_in = ln.fill + ln.acc_fill;
        for (SliceTable* r : job.srcs) ub_in += r->upper;
        const int64_t ub = std::min<int64_t>(ub_in, kStateCapMax);
        if (fire_now || cum_fire) {
            if (zeroed_out && !h->out_count_reset && h->adv_base + h->late_rows == 0) h->out_count_reset = true;
            rc = reset_out_count(h);
            if (rc) return rc;
            rc = ensure_out(h, h->out_n + h->pending_out + ub);
            if (rc) return rc;
            h->pending_out += ub;
        }
        job.dst = dstt;
        job.emit = fire_now || cum_fire;
        job.wend = se;
        job.kclass = fire_now || cum_fire ? K_FLUSH_FIRE : K_FLUSH;
        if (lane_tiles) {
            // the lane's tile passes straight into the slice state (and the fired window's rows):
            // the resident tables the merge would read inserted first, the destination's regions
            // written back by the same workgroups -- no materialized pass, no staged pass 2
            // (an item's (source, region) ranges fit the kernel's kTileMaxRegions prefix slots)
            const int tsub = kTileBits + h->region_bits - ln.passes[0]->bits;
            bool ok = tile_fire_ok(h, ln, tile_split_ok(h)) && h->keys32 && ub_cnt_fits(h) && job.srcs.size() <= 8 &&
                      tsub <= kTileMaxRegionBits &&
                      ((int64_t)job.srcs.size() << tsub) <= (int64_t)kTileMaxRegions &&
                      !(job.emit && h->retain && !h->local);
            for (SliceTable* x : job.srcs) ok = ok && !x->has_null;
            if (ok) {
                for (Staged* st : ln.passes) {
                    job.batches.push_back(JobBatch{st, l, StagedBatch{}, 0});
                    st->busy = true;
                }
                // an empty destination takes the 16-B layout (FG_NARROW_TABLES=0: wide, A/B) -- not
                // for HOP, whose fires read the slice tables through the compact merge: A/B on one box
                // (profiles/r05/hop_narrow) 0.507 vs 0.445 ms per merge fire reading narrow vs wide
                // entries, 46.1 vs 44.4 ms per 1B records; CUMULATE's tile fire gains (59.0 vs 62.7)
#if defined(FG_HOP_WIDE)
                if (job.dst && job.dst->upper == 0 && h->narrow_tables && !h->mv && h->w.kind != HOP)
#else
                if (job.dst && job.dst->upper == 0 && h->narrow_tables && !h->mv)
#endif
                    job.dst->narrow = true;
                job.tile = true;
                job.tbits = ln.passes[0]->bits;
                job.kclass = job.emit ? K_TILE_FIRE : K_TILE_FLUSH;
                const int kc = job.kclass;
                int ji = 0;
                rc = job_add(h, std::move(job), &ji);
                if (rc) return rc;
                TileFire f{};
                rc = tile_job_params(h, ji, &f);
                if (rc) return rc;
                bool skewed = false;   // (a skewed pass: the split fire, with the job's tables)
                for (const Staged* st : ln.passes) skewed = skewed || st->skew;
                {
                    KTimer kt(h, skewed ? K_TILE_SPLIT : kc, ln.fill);
                    if (skewed) {
                        rc = tile_split_fire(h, ln, f, h->tile_chunk);
                        if (rc) return rc;
                    } else {
                        HIPCHK(h, tile_fire_launch(h, f, std::min(1 << (f.tbits - kTileBits), h->merge_grid), h->stream));
                    }
                }
                if (kc == K_TILE_FIRE) fire_class = K_TILE_FIRE;
                goto merged;
            }
            rc = materialize_lane(h, l);
            if (rc) return rc;
        }
        for (Staged* s : ln.passes) job.batches.push_back(JobBatch{s, l, StagedBatch{}, 0});
        {
        int ji = 0;
        rc = job_add(h, std::move(job), &ji);
        if (rc) return rc;
        MergeParams p{};
        rc = job_params(h, ji, &p);
        if (rc) return rc;
        // fast variants: plain staged {key, value} records bucketed at the current regions
        bool plain = h->st_stride == 2 && !ln.passes.empty() && ln.passes.size() <= (size_t)kMaxMergeBatches;
        for (Staged* s : ln.passes)
            plain = plain && !s->has_null && !s->is_acc && s->bits == h->region_bits && s->narrow == ln.passes[0]->narrow;
        p.fast_stream = plain ? 1 : 0;
        p.narrow = plain && ln.passes[0]->narrow ? 1 : 0;
        // compact LDS table (two workgroups per CU) when no resident state is read and the
        // COUNT(*) of a key cannot reach 2^32
        // (resident sources: plain ones -- no NULL counts, marks or chains -- at a COUNT(*) bound
        // below 2^32, keyed by their int32 keys under narrow staging; a fired window that keeps
        // its state (allowed lateness) takes the wide merge)
        const bool src_ok = p.n_src == 0 ||
                            (!h->mv && p.src_null_mask == 0 && !p.mark_mask && !p.markonly_mask &&
                             !p.emit_marked && p.dst_mode == 0 && p.n_src <= 64 && ub_cnt_fits(h) &&
                             (!p.narrow || h->keys32));
        p.compact = plain && src_ok && ln.fill < ((int64_t)1 << 32) && !(p.emit && p.has_dst && h->retain) ? 1 : 0;
#ifdef FG_STAMPS
        static DevBuf d_st;
        if (getenv("FG_STAMPS")) {
            HIPCHK(h, d_st.ensure(64));
            HIPCHK(h, hipMemsetAsync(d_st.p, 0, 64, h->stream));
            p.stamps = d_st.as<unsigned long long>();
        }
#endif
        // skewed regions take the chunked heavy pass (passes bucketed at the current regions)
        bool skew = false, same_bits = true;
        for (Staged* s : ln.passes) {
            skew = skew || s->skew;
            same_bits = same_bits && s->bits == h->region_bits;
        }
        p.hot_keys = skew ? 1 : 0;
        skew = skew && same_bits;
        HeavyPlan hp{};
        if (skew) {
            rc = plan_heavy(h, p.batches, p.n_batches, ln.fill + ln.acc_fill, &hp);
            if (rc) return rc;
            p.heavy = hp.heavy;
        }
        {
            KTimer kt(h, fire_now || cum_fire ? K_FLUSH_FIRE : K_FLUSH, ln.fill);
            HIPCHK(h, launch_merge(p, p.compact && !h->mv ? std::min(h->P, 2 * h->merge_grid) : merge_grid(h), h->stream));
        }
        if (skew) {
            // the heavy regions: chunk tables, then their merge with the region's state
            KTimer kt(h, K_HEAVY, 0);
            HIPCHK(h, launch_heavy_chunks(hp, h->merge_grid, h->stream));
            MergeParams q = p;
            q.compact = 0;
            q.fast_stream = 0;
            q.n_batches = 0;
            q.batches = nullptr;
            q.heavy = nullptr;
            q.region_list = hp.region_list;
            q.n_list = hp.n_list;
            q.chunk0 = hp.chunk0;
            q.part_key = hp.part_key;
            q.part_cs = hp.part_cs;
            q.part_cn = hp.part_cn;
            q.part_sum = hp.part_sum;
            q.part_v1 = hp.part_v1;
            q.part_v2 = hp.part_v2;
            q.part_n = hp.part_n;
            HIPCHK(h, launch_merge(q, merge_grid(h), h->stream));
        }
#ifdef FG_STAMPS
        if (p.stamps) {
            unsigned long long st[4];
            HIPCHK(h, hipMemcpyAsync(st, d_st.p, 32, hipMemcpyDeviceToHost, h->stream));
            HIPCHK(h, hipStreamSynchronize(h->stream));
            const int waves = (p.compact ? std::min(h->P, 2 * h->merge_grid) * kCompactMergeThreads
                                         : merge_grid(h) * kMergeThreads) / 64;
            fprintf(stderr, "[fg stamps] merge %s P=%d records=%lld: clear %.0f stream %.0f compact %.0f emit %.0f (cycles/wave)\n",
                    p.compact ? "compact" : "wide", h->P, (long long)ln.fill, (double)st[0] / waves,
                    (double)st[1] / waves, (double)st[2] / waves, (double)st[3] / waves);
        }
#endif
        }
    merged:
        if (fire_now) {
            if (h->retain && !h->local) {
                t->upper = ub;
                t->changed = true;
                retained.push_back(se);
            } else if (t) {
                fired_tables.push_back(se);
            }
            any_emit = true;
        } else if (cum_fire) {
            any_emit = true;
            h->fused_fired.insert(se);   // fire_windows must not fire W again
            if (dstt) {
                dstt->upper = ub;
                dstt->changed = true;
            }
            if (se == cum_last) {        // the cumulative window is complete
                fired_tables.push_back(se);
                if (se != cum_first) fired_tables.push_back(cum_first);
            } else if (se != cum_first) {
                fired_tables.push_back(se);   // folded into the first slice
            }
        } else {
            t->upper = std::min<int64_t>(t->upper + ln.fill + ln.acc_fill, kStateCapMax);
            t->changed = true;
        }
    }
    if (h->async_advance && any_emit) {
        // fg_advance_progress_async: the host's bookkeeping now, the device's results later
        // (complete_fire); tables freed here are held until then
        rc = publish_fire(h, fire_class);   // (first: the tables freed below are held)
        if (rc) return rc;
        for (int64_t se : fired_tables) table_free(h, se);
        for (int64_t se : retained) retire(h, se, se);
        for (int l : sel) release_lane(h, l);
        h->flushes++;
        return FG_OK;
    }
    HIPCHK(h, hipMemcpyAsync(h->h_scalars.p, h->scalars.p, kScalarBytes, hipMemcpyDeviceToHost, h->stream));
    rc = sync(h);
    if (rc) return rc;
    rc = settle_jobs(h);   // regions that overflowed: split and redone
    if (rc) return rc;
    rc = check_overflow(h);
    if (rc) return rc;
    if (any_emit) {
        const int64_t before = h->out_n;
        h->out_n = (int64_t)h->h_scalars.as<unsigned long long>()[1];
        h->kstat[fire_class].rows += h->out_n - before;
        h->pending_out = 0;
    }
    for (int64_t se : fired_tables) table_free(h, se);
    for (int64_t se : retained) retire(h, se, se);
    for (int l : sel) release_lane(h, l);
    h->flushes++;
    return FG_OK;
}

int flush(fg_handle* h, const FireRange* fire = nullptr, bool only_fired = false) {
    std::vector<int> sel;
    for (int l = 0; l < h->lanes; l++) {
        if (h->lane[l].q == kEmptyLane) continue;
        if (only_fired && !is_window_fired(h->w, slice_end_of(h, h->lane[l].q), h->current_progress)) continue;
        sel.push_back(l);
    }
    return flush_lanes(h, sel, fire);
}
int flush_lane(fg_handle* h, int l) { return flush_lanes(h, std::vector<int>{l}, nullptr); }

int ensure_out(fg_handle* h, int64_t need) {
    if (need <= h->out_cap) return FG_OK;
    int64_t nc = std::max<int64_t>(need, h->out_cap + h->out_cap / 2);
    nc = std::max<int64_t>(nc, 1024);
    HIPCHK(h, h->o_key.ensure(8 * nc, h->stream, true));
    HIPCHK(h, h->o_ws.ensure(8 * nc, h->stream, true));
    HIPCHK(h, h->o_we.ensure(8 * nc, h->stream, true));
    HIPCHK(h, h->o_null.ensure(nc, h->stream, true));
    if (h->cfg.mode == FG_MODE_DATASTREAM) HIPCHK(h, h->o_rt.ensure(8 * nc, h->stream, true));
    for (int a = 0; a < h->cfg.num_aggs; a++) HIPCHK(h, h->o_agg[a].ensure(8 * nc, h->stream, true));
    h->out_cap = nc;
    return FG_OK;
}

// Emit one window from the union of `srcs`; optionally write the merged state to `dst`.
// `defer`: no host synchronization -- the caller collects the row count (fire_collect)
// after the advance's last fire (launches stay ordered on the handle's stream).
int fire_one(fg_handle* h, int64_t wend, const std::vector<SliceTable*>& srcs, SliceTable* dst, bool defer = false) {
    if (int rc0 = complete_fire(h)) return rc0;
    int64_t ub = 0;
    for (auto* s : srcs) ub += s->upper;
    ub = std::min<int64_t>(ub, kStateCapMax);
    if (ub == 0 && dst == nullptr) return FG_OK;
    int rc = reset_out_count(h);
    if (rc) return rc;
    rc = ensure_out(h, h->out_n + h->pending_out + ub);
    if (rc) return rc;
    if (srcs.size() == 1 && !dst) {   // one table, nothing written: rows straight from it (cannot overflow)
        MergeParams p{};
        p.region_bits = h->region_bits;
        set_values(h, &p);
        fill_emit(h, p, wend);
        p.out_count = reinterpret_cast<unsigned long long*>(h->scalars.as<char>() + 8);
        p.overflow = h->scalars.as<unsigned int>();
        KTimer kt(h, K_FIRE, 0);
        HIPCHK(h, launch_emit_table(p, ref_of(srcs[0]), h->stream));
    } else {
        MergeJob j;
        j.srcs = srcs;
        j.dst = dst;
        j.emit = true;
        j.wend = wend;
        j.kclass = K_FIRE;
        int ji = 0;
        rc = job_add(h, std::move(j), &ji);
        if (rc) return rc;
        MergeParams p{};
        rc = job_params(h, ji, &p);
        if (rc) return rc;
#ifdef FG_STAMPS
        static DevBuf d_fst;
        if (getenv("FG_STAMPS")) {
            HIPCHK(h, d_fst.ensure(64));
            HIPCHK(h, hipMemsetAsync(d_fst.p, 0, 64, h->stream));
            p.stamps = d_fst.as<unsigned long long>();
        }
#endif
        // the compact merge (two workgroups per CU, 20-B LDS slots) when the window is plain
        // resident state: source tables without NULL counts or marks, nothing written back, one
        // value accumulator, COUNT(*)s below 2^32
        p.compact = !h->mv && !dst && p.n_batches == 0 && p.src_null_mask == 0 && !p.mark_mask &&
                            !p.markonly_mask && !p.emit_marked && p.dst_mode == 0 && p.n_src <= 64 &&
                            ub_cnt_fits(h)
                        ? 1
                        : 0;
        p.narrow = p.compact && h->keys32 ? 1 : 0;   // (narrow LDS table: keys from the entries' mixes)
        {
            KTimer kt(h, K_FIRE, 0);
            HIPCHK(h, launch_merge(p, p.compact ? std::min(h->P, 2 * h->merge_grid) : merge_grid(h), h->stream));
        }
#ifdef FG_STAMPS
        if (p.stamps) {
            unsigned long long st[4];
            HIPCHK(h, hipMemcpyAsync(st, d_fst.p, 32, hipMemcpyDeviceToHost, h->stream));
            HIPCHK(h, hipStreamSynchronize(h->stream));
            const int waves = merge_grid(h) * kMergeThreads / 64;
            fprintf(stderr, "[fg stamps] fire srcs=%zu dst=%d: clear %.0f stream %.0f compact %.0f emit %.0f (cycles/wave)\n",
                    srcs.size(), dst ? 1 : 0, (double)st[0] / waves, (double)st[1] / waves, (double)st[2] / waves,
                    (double)st[3] / waves);
        }
#endif
    }
    if (dst) {
        dst->upper = ub;
        dst->changed = true;
    }
    if (defer) {
        h->pending_out += ub;
        return FG_OK;
    }
    return fire_collect(h);
}

// after fires: region retries, overflow check and the fired-row count (one synchronization)
int fire_collect(fg_handle* h) {
    if (h->async_advance) {   // fg_advance_progress_async: completed by the next call that needs it
        return publish_fire(h, K_FIRE);   // (tables freed by the fires stay held until then)
    }
    HIPCHK(h, hipMemcpyAsync(h->h_scalars.p, h->scalars.p, kScalarBytes, hipMemcpyDeviceToHost, h->stream));
    int rc = sync(h);
    if (rc) return rc;
    rc = settle_jobs(h);
    if (rc) return rc;
    rc = check_overflow(h);
    if (rc) return rc;
    const int64_t before = h->out_n;
    h->out_n = (int64_t)h->h_scalars.as<unsigned long long>()[1];
    h->kstat[K_FIRE].rows += h->out_n - before;
    h->pending_out = 0;
    return FG_OK;
}

// Fire every window whose timer time lies in (prev, wm] (InternalTimerServiceImpl.advanceWatermark
// :294-304 -> SlicingWindowOperator.onTimer :230-237), in window order.
int fire_windows_launch(fg_handle* h, int64_t prev, int64_t wm, bool* fired);
int fire_windows(fg_handle* h, int64_t prev, int64_t wm) {
    bool fired = false;
    // tables freed by the loop stay alive until the fires are collected (a failed region's
    // retry reads them)
    h->defer_free = true;
    int rc = fire_windows_launch(h, prev, wm, &fired);
    h->defer_free = false;
    if (rc) return rc;
    if (fired) return fire_collect(h);
    if (h->fire_pending) return FG_OK;   // (freed tables held until the pending fire completes)
    for (auto& t : h->deferred) h->table_pool.push_back(std::move(t));
    h->deferred.clear();
    return FG_OK;
}
int fire_windows_launch(fg_handle* h, int64_t prev, int64_t wm, bool* fired) {
    const WindowSpec& w = h->w;
    auto due = [&](int64_t wend) {
        int64_t t = trigger_time(w, wend);
        return wend != JMAX && t > prev && t <= wm;
    };
    auto dead = [&](int64_t wend) { return wend != JMAX && trigger_time(w, wend) <= prev; };
    if (h->tables.empty()) return FG_OK;
    int rc;
    if (w.kind == TUMBLE) {
        std::vector<int64_t> ends;
        for (auto& kv : h->tables) ends.push_back(kv.first);
        for (int64_t e : ends) {
            if (h->retire_at.count(e)) continue;   // fired before, kept for its late elements
            if (due(e)) {
                rc = fire_one(h, e, {h->tables[e].get()}, nullptr, true);
                *fired = true;
                if (rc) return rc;
                retire(h, e, e);    // expiredSlices = [windowEnd] (with allowed lateness: at cleanup)
            } else if (dead(e)) {
                retire(h, e, e);    // no timer can fire for this slice any more
            }
        }
        return FG_OK;
    }
    if (w.kind == HOP) {
        // window ends on the slice grid; window W covers slices (W - size, W]
        int64_t lo = h->tables.begin()->first;
        int64_t hi = jadd(jsub(h->tables.rbegin()->first, w.slice), w.size);   // last window of the last slice
        for (int64_t W = lo; W <= hi; W = jadd(W, w.slice)) {
            if (trigger_time(w, W) > wm) break;
            if (h->tables.empty()) break;
            if (due(W)) {
                std::vector<SliceTable*> srcs;
                for (auto it = h->tables.upper_bound(jsub(W, w.size)); it != h->tables.end() && it->first <= W; ++it)
                    srcs.push_back(it->second.get());
                if (!srcs.empty()) {
                    rc = fire_one(h, W, srcs, nullptr, true);
                    *fired = true;
                    if (rc) return rc;
                }
            }
            if (due(W) || dead(W)) {   // expiredSlices: W was the last window of its first slice
                const int64_t first = jadd(jsub(W, w.size), w.slice);
                if (!h->retire_at.count(first)) retire(h, first, W);
            }
            // skip empty stretches
            auto nx = h->tables.upper_bound(jsub(W, w.size));
            if (nx == h->tables.end()) break;
            if (jadd(W, w.slice) <= jsub(nx->first, w.slice) && nx->first > W) W = jsub(nx->first, w.slice);
        }
        return FG_OK;
    }
    // CUMULATE: windows ws+step, ws+2step, ... ws+max of every cumulative window with state
    std::vector<int64_t> starts;
    for (auto& kv : h->tables) {
        int64_t ws = window_start(w, kv.first);
        if (starts.empty() || starts.back() != ws) starts.push_back(ws);
    }
    std::sort(starts.begin(), starts.end());
    starts.erase(std::unique(starts.begin(), starts.end()), starts.end());
    for (int64_t ws : starts) {
        const int64_t first = jadd(ws, w.slice), last = jadd(ws, w.size);
        for (int64_t W = first; W <= last; W = jadd(W, w.slice)) {
            if (trigger_time(w, W) > wm) break;
            SliceTable* F = nullptr;
            SliceTable* S = nullptr;
            rc = table_get(h, first, false, &F);
            if (rc) return rc;
            if (W != first) {
                rc = table_get(h, W, false, &S);
                if (rc) return rc;
            }
            if (!F && !S) continue;
            if (due(W) && !h->fused_fired.count(W)) {
                std::vector<SliceTable*> srcs;
                if (F) srcs.push_back(F);
                if (S) srcs.push_back(S);
                SliceTable* dst = nullptr;
                if (W != first && W != last && S) {
                    if (!F) {
                        rc = table_get(h, first, true, &F);
                        if (rc) return rc;
                    }
                    dst = F;   // merge the step slice into the first slice's state
                }
                rc = fire_one(h, W, srcs, dst, true);   // (no step slice: the state is unchanged)
                *fired = true;
                if (rc) return rc;
            } else if (S && F && W != first) {
                // window already fired before: fold the slice into the first slice without emitting
                // (only reachable for state restored below an older watermark)
            }
            if (due(W) || dead(W)) {
                if (W != first) table_free(h, W);
                if (W == last) table_free(h, first);
            }
        }
    }
    return FG_OK;
}

// ---- restore re-fire of shared windows (HOP, CUMULATE) -------------------------------
// After initializeState the reference's timer service restarts at Long.MIN_VALUE: a record
// older than the checkpoint's watermark is not late, its flush registers the timer of its
// slice's window (AggCombiner step 5), and onTimer chains the key on through
// nextTriggerWindow -- HOP while the window is non-empty, CUMULATE to the cumulative window's
// end (SliceSharedWindowAggProcessor.java:64-118) -- so those old windows fire again for the
// keys of such records only. Here those records are flushed apart (re_new: their state,
// re_delta: the keys flushed since the last watermark) and, per re-fired window W in
// ascending order, one merge emits exactly the chained keys: the keys of W's own new slice
// plus the running chain (a table of keys with zero accumulators, the merge's mark-only
// sources), with their whole state over W's slices (restored + new); the merge writes the
// chain on (HOP: the marked keys holding state in W; CUMULATE: every marked key). CUMULATE
// folds each step slice into the first slice's state as it fires (mergeSlices).
// one re-fire merge as a job (retried by region like every merge)
int refire_job(fg_handle* h, const std::vector<SliceTable*>& vals, const std::vector<SliceTable*>& marks,
               SliceTable* dst, int dst_mode, bool emit, int64_t wend) {
    MergeJob j;
    for (SliceTable* t : vals)
        if (t && t->upper > 0) j.srcs.push_back(t);
    int64_t ub = 0;
    for (SliceTable* t : j.srcs) ub += t->upper;
    for (SliceTable* t : marks) {
        if (!t || t->upper == 0) continue;
        if (j.srcs.size() >= 64) return h->fail(FG_ESTATE, "internal: re-fire merge over 64 sources");
        const uint64_t bit = 1ull << j.srcs.size();
        j.mark_mask |= bit;
        j.markonly_mask |= bit;
        j.srcs.push_back(t);
    }
    if (j.mark_mask == 0 && dst_mode != 0) return FG_OK;   // nothing chained
    int rc;
    if (emit) {
        if (j.mark_mask == 0) return FG_OK;
        rc = reset_out_count(h);
        if (rc) return rc;
        ub = std::min<int64_t>(ub, kStateCapMax);
        rc = ensure_out(h, h->out_n + h->pending_out + ub);
        if (rc) return rc;
        h->pending_out += ub;
        j.emit = true;
        j.emit_marked = 1;
        j.wend = wend;
    }
    j.dst = dst;
    j.dst_mode = dst_mode;
    j.kclass = K_FIRE;
    int ji = 0;
    rc = job_add(h, std::move(j), &ji);
    if (rc) return rc;
    MergeParams p{};
    rc = job_params(h, ji, &p);
    if (rc) return rc;
    KTimer kt(h, K_FIRE, 0);
    HIPCHK(h, launch_merge(p, merge_grid(h), h->stream));
    if (dst) {
        int64_t u = 0;
        for (SliceTable* t : h->jobs.back().srcs) u += t->upper;
        dst->upper = std::min<int64_t>(u, kStateCapMax);
        dst->changed = true;
    }
    return FG_OK;
}

// the re-fire is over (the watermark passed the checkpoint's): new state of slices that
// later windows still read joins the resident state, the rest is dropped
int refire_finish(fg_handle* h) {
    int rc;
    const WindowSpec& w = h->w;
    std::vector<std::pair<int64_t, std::unique_ptr<SliceTable>>> moved;
    for (auto& kv : h->re_new) {
        const int64_t se = kv.first;
        // the last window containing the slice (HOP: se + size - slice; CUMULATE: its window's end)
        const int64_t last = w.kind == HOP ? jadd(jsub(se, w.slice), w.size) : jadd(window_start(w, se), w.size);
        if (trigger_time(w, last) <= h->refire_hi) continue;
        // HOP: the slice's own table; CUMULATE: the first slice's state it folds into
        const int64_t into = w.kind == HOP ? se : jadd(window_start(w, se), w.slice);
        SliceTable* m = nullptr;
        rc = table_get(h, into, w.kind == CUMULATE, &m);
        if (rc) return rc;
        if (m) {
            rc = refire_job(h, {m, kv.second.get()}, {}, m, 0, false, 0);
            if (rc) return rc;
        } else {
            moved.emplace_back(se, std::move(kv.second));
        }
    }
    rc = fire_collect(h);
    if (rc) return rc;
    for (auto& mv : moved) h->tables[mv.first] = std::move(mv.second);
    auto pool = [&](std::unique_ptr<SliceTable>& t) {
        if (t && t->bits == h->region_bits) h->table_pool.push_back(std::move(t));
        t.reset();
    };
    for (auto& kv : h->re_new) pool(kv.second);
    for (auto& kv : h->re_delta) pool(kv.second);
    for (auto& t : h->re_tmp) pool(t);
    pool(h->re_chain);
    h->re_new.clear();
    h->re_delta.clear();
    h->re_tmp.clear();
    h->re_chain_w = JMIN;
    h->refire_hi = JMIN;
    return FG_OK;
}

// DataStream sliding windows (WindowOperator): a restored window that fired was purged
// (clearAllState at its cleanup time), so an element that arrives for it after the restore
// (isWindowLate against the restarted timer watermark) builds a new window state of the
// post-restore elements only, whose timer fires it again: re-fire every window up to the
// horizon from the new slices alone, for every key in them.
int refire_datastream(fg_handle* h, int64_t wm) {
    const WindowSpec& w = h->w;
    const int64_t lim = std::min(wm, h->refire_hi);
    const int64_t from = h->refire_wm;   // windows up to the last run's limit are final
    h->refire_wm = lim;
    bool fired = false;
    int rc;
    if (!h->re_new.empty()) {
        int64_t W = h->re_new.begin()->first;
        const int64_t hi = jadd(jsub(h->re_new.rbegin()->first, w.slice), w.size);
        for (; W <= hi && trigger_time(w, W) <= lim; W = jadd(W, w.slice)) {
            if (trigger_time(w, W) <= from) continue;
            std::vector<SliceTable*> srcs;
            for (auto it = h->re_new.upper_bound(jsub(W, w.size)); it != h->re_new.end() && it->first <= W; ++it)
                srcs.push_back(it->second.get());
            if (srcs.empty()) continue;
            rc = fire_one(h, W, srcs, nullptr, true);
            if (rc) return rc;
            fired = true;
        }
    }
    if (fired) {
        rc = fire_collect(h);
        if (rc) return rc;
    }
    if (wm >= h->refire_hi) return refire_finish(h);
    return FG_OK;
}

int refire(fg_handle* h, int64_t wm) {
    if (int rc0 = complete_fire(h)) return rc0;
    if (h->cfg.mode == FG_MODE_DATASTREAM) return refire_datastream(h, wm);
    const WindowSpec& w = h->w;
    const int64_t S = w.slice;
    const int64_t lim = std::min(wm, h->refire_hi);
    h->refire_wm = wm;
    int64_t W = JMAX;
    if (!h->re_delta.empty()) W = h->re_delta.begin()->first;
    if (h->re_chain) W = std::min(W, h->re_chain_w);
    const int64_t last_delta = h->re_delta.empty() ? JMIN : h->re_delta.rbegin()->first;
    SliceTable* R = nullptr;   // running chain (in re_tmp)
    int64_t R_ws = JMIN;       // CUMULATE: the cumulative window of R
    std::vector<int64_t> done_delta, folded, expired_first;
    bool any = false;
    int rc;
    auto new_chain = [&](SliceTable** out) -> int {
        std::unique_ptr<SliceTable> t;
        int r = table_new(h, JMIN, &t);
        if (r) return r;
        *out = t.get();
        h->re_tmp.push_back(std::move(t));
        return FG_OK;
    };
    for (; W != JMAX && trigger_time(w, W) <= lim; W = jadd(W, S)) {
        SliceTable* D = side_get(h->re_delta, W);
        SliceTable* Cold = h->re_chain && W == h->re_chain_w ? h->re_chain.get() : nullptr;
        if (w.kind == CUMULATE && R && window_start(w, W) != R_ws) R = nullptr;   // a new cumulative window
        if (!D && !R && !Cold) {
            if (W >= last_delta && (!h->re_chain || W >= h->re_chain_w)) break;
            continue;
        }
        if (D) done_delta.push_back(W);
        SliceTable* R2 = nullptr;
        rc = new_chain(&R2);
        if (rc) return rc;
        if (w.kind == HOP) {
            std::vector<SliceTable*> vals;   // W's slices (W - size, W]: resident and new state
            for (auto it = h->tables.upper_bound(jsub(W, w.size)); it != h->tables.end() && it->first <= W; ++it)
                vals.push_back(it->second.get());
            for (auto it = h->re_new.upper_bound(jsub(W, w.size)); it != h->re_new.end() && it->first <= W; ++it)
                vals.push_back(it->second.get());
            rc = refire_job(h, vals, {D, R, Cold}, R2, 1, true, W);   // emit + chain on (marked, non-empty)
            if (rc) return rc;
            expired_first.push_back(jadd(jsub(W, w.size), S));          // expiredSlices: W's first slice
        } else {   // CUMULATE
            const int64_t ws = window_start(w, W), first = jadd(ws, S), last = jadd(ws, w.size);
            SliceTable* F = nullptr;
            rc = table_get(h, first, true, &F);
            if (rc) return rc;
            // fold the new state of this cumulative window's slices up to W into the first
            // slice's state (mergeSlices; a late-accepted record's slice is the first one)
            std::vector<SliceTable*> fold{F};
            for (auto it = h->re_new.lower_bound(first); it != h->re_new.end() && it->first <= W; ++it) {
                if (std::find(folded.begin(), folded.end(), it->first) != folded.end()) continue;
                fold.push_back(it->second.get());
                folded.push_back(it->first);
            }
            if (fold.size() > 1) {
                rc = refire_job(h, fold, {}, F, 0, false, 0);
                if (rc) return rc;
            }
            rc = refire_job(h, {F}, {D, R, Cold}, nullptr, 0, true, W);   // emit the chained keys
            if (rc) return rc;
            rc = refire_job(h, {}, {D, R, Cold}, R2, 2, false, 0);        // the chain goes on regardless
            if (rc) return rc;
            R_ws = ws;
            if (W == last) {   // the cumulative window is complete: its state expires
                table_free(h, first);
                R2 = nullptr;
            }
        }
        R = R2;
        any = true;
    }
    if (any) {
        h->defer_free = true;   // (table_free above: held until the fires are collected)
        rc = fire_collect(h);
        h->defer_free = false;
        if (rc) return rc;
    }
    for (int64_t e : done_delta) {
        auto it = h->re_delta.find(e);
        if (it != h->re_delta.end()) {
            h->table_pool.push_back(std::move(it->second));
            h->re_delta.erase(it);
        }
    }
    for (int64_t e : folded) {
        auto it = h->re_new.find(e);
        if (it != h->re_new.end()) {
            h->table_pool.push_back(std::move(it->second));
            h->re_new.erase(it);
        }
    }
    for (int64_t e : expired_first) {
        auto it = h->re_new.find(e);
        if (it != h->re_new.end()) {
            h->table_pool.push_back(std::move(it->second));
            h->re_new.erase(it);
        }
    }
    // the chain that goes on past this watermark
    std::unique_ptr<SliceTable> keep;
    for (auto& t : h->re_tmp)
        if (t && t.get() == R) keep = std::move(t);
    for (auto& t : h->re_tmp)
        if (t && t->bits == h->region_bits) h->table_pool.push_back(std::move(t));
    h->re_tmp.clear();
    if (h->re_chain && h->re_chain.get() != R) {
        if (h->re_chain->bits == h->region_bits) h->table_pool.push_back(std::move(h->re_chain));
        h->re_chain.reset();
    }
    if (keep) {
        h->re_chain = std::move(keep);
        h->re_chain_w = W;
    } else if (!h->re_chain || h->re_chain.get() != R) {
        h->re_chain.reset();
        h->re_chain_w = JMIN;
    }
    if (wm >= h->refire_hi) return refire_finish(h);
    return FG_OK;
}

int copy_out_to_host(fg_handle* h, fg_rows* r) {
    const int64_t n = h->out_n;
    const size_t b8 = 8 * (size_t)std::max<int64_t>(n, 1);
    HIPCHK(h, h->h_key.ensure(b8));
    HIPCHK(h, h->h_ws.ensure(b8));
    HIPCHK(h, h->h_we.ensure(b8));
    HIPCHK(h, h->h_null.ensure(std::max<int64_t>(n, 1)));
    if (h->cfg.mode == FG_MODE_DATASTREAM) HIPCHK(h, h->h_rt.ensure(b8));
    for (int a = 0; a < h->cfg.num_aggs; a++) HIPCHK(h, h->h_agg[a].ensure(b8));
    if (n > 0) {
        HIPCHK(h, hipMemcpyAsync(h->h_key.p, h->o_key.p, 8 * n, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->h_ws.p, h->o_ws.p, 8 * n, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->h_we.p, h->o_we.p, 8 * n, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->h_null.p, h->o_null.p, n, hipMemcpyDeviceToHost, h->stream));
        if (h->cfg.mode == FG_MODE_DATASTREAM)
            HIPCHK(h, hipMemcpyAsync(h->h_rt.p, h->o_rt.p, 8 * n, hipMemcpyDeviceToHost, h->stream));
        for (int a = 0; a < h->cfg.num_aggs; a++)
            HIPCHK(h, hipMemcpyAsync(h->h_agg[a].p, h->o_agg[a].p, 8 * n, hipMemcpyDeviceToHost, h->stream));
        int rc = sync(h);
        if (rc) return rc;
    }
    r->key = h->h_key.as<int64_t>();
    r->window_start = h->h_ws.as<int64_t>();
    r->window_end = h->h_we.as<int64_t>();
    r->null_mask = h->h_null.as<uint8_t>();
    r->rowtime = h->cfg.mode == FG_MODE_DATASTREAM ? h->h_rt.as<int64_t>() : nullptr;
    for (int a = 0; a < h->cfg.num_aggs; a++) r->agg[a] = h->h_agg[a].as<int64_t>();
    return FG_OK;
}

// Rowtime fast path (k_ingest_*: classify): with tbase a slice start at or below the
// batch's rowtimes, assignSliceEnd(ts) = tbase + S * (floor((ts + tz - tbase) / S) + 1)
// whenever ts + tz - tbase < 2^32 (AbstractSliceAssigner.assignSliceEnd, SliceAssigners.java:573-577,
// for ts - offset + S >= 0), and the slice is not fired iff its end > progress + 1 + tz
// (isWindowFired, TimeWindowUtil.java:166-173). Everything else takes the exact 64-bit path.
void set_fast_path(fg_handle* h, IngestParams* p) {
    p->div_m = 0;
    const int64_t S = h->w.slice;
    if (h->w.tz_n > 0) return;   // zone rules: the offset varies per record, exact path
    if (h->anchor_start == JMIN || S < 2 || S >= ((int64_t)1 << 32)) return;
    const __int128 margin = (__int128)S * (((int64_t)1 << 30) / S);
    const __int128 tb = (__int128)h->anchor_start - margin;
    if (tb < (__int128)h->w.offset || tb + ((__int128)1 << 33) + 4 * (__int128)S > (__int128)JMAX) return;
    p->tbase = (int64_t)tb;
    p->div_m = ~0ull / (uint64_t)S + 1;
    p->qbase = floor_div(p->tbase, S) + 1;
    __int128 lim = (__int128)(h->local || h->proctime ? JMIN : h->current_progress) + 1 + h->w.tz;
    if (lim < (__int128)JMIN) lim = JMIN;
    if (lim > (__int128)JMAX) lim = JMAX;
    p->fired_lim = (int64_t)lim;
}

// Seed the fast-path anchor from the first rowtime when no batch has been seen yet.
int seed_anchor(fg_handle* h, const int64_t* ts_dev, const int64_t* ts_host) {
    if (h->anchor_start != JMIN) return FG_OK;
    int64_t t0;
    if (ts_host) {
        t0 = ts_host[0];
    } else {
        HIPCHK(h, hipMemcpyAsync(h->h_counters.p, ts_dev, 8, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        std::memcpy(&t0, h->h_counters.p, 8);
    }
    if (t0 == JMAX || t0 == JMIN) return FG_OK;
    const int64_t t = to_utc(h->w, t0);
    const __int128 st = (__int128)floor_div(jsub(t, h->slice_phase), h->w.slice) * h->w.slice + h->slice_phase;
    if (st > (__int128)JMIN + h->w.slice && st < (__int128)JMAX - h->w.slice) h->anchor_start = (int64_t)st;
    return FG_OK;
}

// grow the per-lane staged areas to hold `need` records per lane (all lanes empty)
int grow_lanes(fg_handle* h, int64_t need) {
    if (need <= h->lane_cap) return FG_OK;
    if (staged_any(h)) return h->fail(FG_ESTATE, "internal: staged areas grown while holding records");
    const int64_t cap = std::max<int64_t>(need, h->lane_cap + h->lane_cap / 2);
    HIPCHK(h, h->st_rec.ensure(8 * (size_t)h->st_stride * h->lanes * cap + kRec12Block));
    HIPCHK(h, h->st_null.ensure((size_t)h->lanes * cap));
    h->lane_cap = cap;
    return FG_OK;
}

// one ingest pass over the device-resident batch with a slice filter: count pass
// (slice assignment, late rules, bucket histogram), then -- once the batch's slices are
// known to fit the staged lanes -- bucket scan and scatter into the lanes' staged areas.
// Returns -1 when the batch spans more slices than the lanes can hold.
// ingest scratch for the current regions x lanes (after a split)
int ensure_scratch(fg_handle* h) {
    HIPCHK(h, h->hist.ensure(4 * (size_t)h->F * h->grid));
    HIPCHK(h, h->totals.ensure(4 * ((size_t)h->F + 1)));
    HIPCHK(h, h->scan_tmp.ensure(4 * scan_tmp_words((int64_t)h->F)));
    return FG_OK;
}

// One ingest pass in two halves: ingest_launch queues pass 1 (or the count pass), the bucket
// scan and -- speculatively -- pass 2 with the device's lane plan, then the counters' copy to
// the host; ingest_finish takes the host's decisions once the counters are there (flushes,
// the regular pass 2 when the plan said no, the lanes' bookkeeping).

// Pass 1's grid for a tile pass of n records: one workgroup per 6,144-record tile, at most one
// per CU. FG_TILE_GRID (test knob, read at fg_open) forces a grid: N > 0 exactly N workgroups (more than the
// tiles leaves empty segments), -1 the two-pass partition's rule (one per 16,384 records).
int tile_grid(const fg_handle* h, int64_t n) {
    const int force = h->tile_grid_force;
    int64_t g;
    if (force > 0) g = force;
    else if (force < 0) g = std::min<int64_t>(h->grid, (n + 16383) / 16384);
    else g = std::min<int64_t>(h->grid, (n + kTileRecs - 1) / kTileRecs);
    return (int)std::max<int64_t>(1, g);
}

int ingest_launch(fg_handle* h, int64_t n, const int64_t* key, const int64_t* ts, const int64_t* val,
                  const uint8_t* vnull, int64_t flo, int64_t fhi, bool count_drops, PassState& ps) {
    if (int rc0 = ensure_scratch(h)) return rc0;
    ps.n = n;
    ps.vnull = vnull;
    ps.flo = flo;
    ps.fhi = fhi;
    IngestParams& p = ps.p;
    p.w = h->w;
    p.n = n;
    p.key = key;
    p.ts = ts;
    p.val = val;
    p.vnull = vnull;
    p.progress = h->local || h->proctime ? JMIN : h->current_progress;   // local phase / proctime: nothing is late
    p.lanes = h->lanes;
    p.region_bits = h->region_bits;
    p.filter_lo = flo;
    p.filter_hi = fhi;
    p.count_drops = count_drops ? 1 : 0;
    int64_t g = (n + 16383) / 16384;
    p.grid = (int)std::max<int64_t>(1, std::min<int64_t>(h->grid, g));
    p.vec = ((uintptr_t)key % 16 == 0 && (uintptr_t)ts % 16 == 0 && (!val || (uintptr_t)val % 16 == 0)) ? 1 : 0;
    p.hist = h->hist.as<uint32_t>();
    p.sink = h->sink.as<int64_t>();
    set_fast_path(h, &p);
    // two-pass partition when the regions split into 64-bucket coarse groups
    const bool two_pass = h->region_bits >= kFineBits && h->F <= kMaxPart1Fine;
    ps.two_pass = two_pass;
    // tile staging: TUMBLE windows and the local phase's slices fire straight from pass 1's tiles
    // (32-bit keys, one value accumulator, no NULL values, no allowed lateness, no hot-key skew)
    const bool tiles = two_pass && h->tile_ok && !h->tile_skew && h->narrow && !vnull && !h->mv && h->lateness == 0 &&
                       (h->w.kind == TUMBLE || h->local || (h->tile_state && h->cfg.mode == FG_MODE_SQL)) &&
                       (h->F >> kTileBits) <= kMaxTileBuckets;
    ps.tiles = tiles;
    if (tiles) {
        // the pass's own Staged (its tiles live until the fire): a pooled one no unsettled job reads
        ps.s = pass_from_pool(h);
        Staged* st = ps.s.get();
        // pass 1's grid for tiles: one workgroup per tile up to one per CU (a small batch's pass
        // is then one tile's latency); the segment split (max_tiles, tiles) is carried with the
        // pass -- every consumer (k_tile_dirt, the fire's walk, materialize) reads it from there,
        // never from a grid of its own
        p.grid = tile_grid(h, n);
        // whole-tile segments: max_tiles tiles per workgroup, the grid trimmed to the workgroups
        // that get records; tile t of the pass then starts at record t * kTileRecs
        const int64_t per = (n + p.grid - 1) / p.grid;
        p.max_tiles = (int32_t)std::max<int64_t>(1, (per + kTileRecs - 1) / kTileRecs);
        const int64_t seg = (int64_t)p.max_tiles * kTileRecs;
        p.grid = (int)std::max<int64_t>(1, (n + seg - 1) / seg);
        p.n_coarse = h->F >> kTileBits;
        const int64_t NT = (int64_t)p.grid * p.max_tiles;
        HIPCHK(h, st->t_rec.ensure((size_t)(n / 64 + 2) * kRec12Block));   // (packed 12-B tile records: 12 n)
        HIPCHK(h, st->t_dt.ensure(4 * (size_t)p.n_coarse * NT));
        HIPCHK(h, st->t_btot.ensure(4 * (size_t)p.n_coarse));
        p.tile_btot = st->t_btot.as<uint32_t>();
        HIPCHK(h, h->tile_dir.ensure(2 * (size_t)NT * kTileDirStride(p.n_coarse)));
        p.tmp = st->t_rec.as<longlong2>();
        p.dir = h->tile_dir.as<uint16_t>();
        st->t_n = n;
        st->t_mt = p.max_tiles;
        st->t_nt = (int)NT;
        st->t_nc = p.n_coarse;
    } else if (two_pass) {
        p.max_tiles = part1_max_tiles(n, p.grid);
        p.n_coarse = h->F >> kFineBits;
        HIPCHK(h, h->part_tmp.ensure(16 * (size_t)n + kRec12Block));   // (+ a narrow block's tail)
        HIPCHK(h, h->part_dir.ensure(2 * (size_t)p.grid * p.max_tiles * (p.n_coarse + 1)));
        p.tmp = h->part_tmp.as<longlong2>();
        p.dir = h->part_dir.as<uint16_t>();
        if (vnull) {
            HIPCHK(h, h->part_tmp_null.ensure((size_t)n));
            p.tmp_null = h->part_tmp_null.as<uint8_t>();
        }
    }
    DevCounters init{};
    init.qmin = JMAX;
    init.qmax = JMIN;
    init.qnext = JMAX;
    if (!h->counters_clean) HIPCHK(h, init_counters(h, init));   // (else reset by the last scan)
    h->counters_clean = false;
    DevCounters* dc = h->counters.as<DevCounters>();
    p.drops = &dc->drops;
    p.lane_mask = &dc->lane_mask;
    p.qmin = &dc->qmin;
    p.qmax = &dc->qmax;
    p.qnext = &dc->qnext;
    p.lane_total = dc->lane_total;
    p.max_bucket = &dc->max_bucket;
    p.wide = &dc->wide;
    p.narrow = two_pass && h->narrow ? 1 : 0;
    if (!p.narrow) h->keys32 = false;
    // a stream seen skewed (hot keys) partitions in pass-2 units of one pass-1 workgroup: the
    // hot key's coarse bucket is then spread over as many units as there are workgroups
    p.p2_group = 0;
    if (tiles) {
        {
            KTimer kt(h, K_TILE1, n);
            HIPCHK(h, launch_tile_part1(p, h->stream));
        }
        // each bucket's (offset, length) column (before k_scan_plan resets the lane mask it reads)
        HIPCHK(h, launch_tile_dirt(p.dir, ps.s->t_nt, p.n_coarse, h->region_bits - kTileBits, p.lane_mask,
                                   ps.s->t_dt.as<uint32_t>(), p.tile_btot, h->stream));
    } else if (two_pass) {
        KTimer kt(h, K_PART1, n);
        HIPCHK(h, launch_part1(p, h->stream));
    } else {
        KTimer kt(h, K_COUNT, n);
        HIPCHK(h, launch_ingest_count(p, h->stream));
    }
    // (fg_add_batch: a pending async fire -- before a staged pass is reused below)
    if (int rc0 = complete_fire(h)) return rc0;
    // per-bucket prefix over workgroups and bucket bases: they depend on the histogram only,
    // so they are queued before the host waits for the counters (no idle GPU across the
    // round trip); a pass that stages nothing goes back to the pool
    std::unique_ptr<Staged>& s = ps.s;
    if (!s) s = pass_from_pool(h);   // (a tile pass took its Staged before pass 1)
    const int Fp = tiles ? 0 : p.lanes << p.region_bits;   // the pass's buckets (the regions may split meanwhile)
    HIPCHK(h, s->bucket_off.ensure(sizeof(uint32_t) * (Fp + 1)));
    // Speculative pass 2 (two-pass partition): the lane decision the host takes below is
    // taken on the device from pass 1's counters (k_scan_plan), and pass 2 is queued at
    // once, so the GPU does not idle across the counters' round trip. When the batch needs a
    // flush first (another slice in a lane, no room) the plan says so and pass 2 does
    // nothing; the host then takes the regular path below.
    // (a tile pass is finished at the next call too: nothing of it depends on the host's decisions)
    const bool spec = two_pass && (h->speculate || tiles);
    ps.spec = spec;
    {
        // per-bucket prefix over workgroups, then one workgroup: bucket bases, the counters
        // to the host (reset for the next pass), the lane plan
        KTimer kt(h, K_SCAN, 0);
        if (Fp > 0) HIPCHK(h, launch_hist_columns(h->hist.as<uint32_t>(), h->totals.as<uint32_t>(), Fp, p.grid, h->stream));
        PlanParams pp{};
        pp.lane_cap = h->lane_cap;
        for (int l = 0; l < kMaxLanes; l++) {
            pp.q[l] = l < h->lanes ? h->lane[l].q : kEmptyLane;
            pp.fill[l] = l < h->lanes ? h->lane[l].fill : 0;
        }
        ScanPlanArgs sa{};
        sa.totals = h->totals.as<uint32_t>();
        sa.bucket_off = s->bucket_off.as<uint32_t>();
        sa.F = Fp;
        sa.n_words = (int32_t)(sizeof(DevCounters) / 8);
        sa.counters = h->counters.as<unsigned long long>();
        sa.host = h->h_pass.as<unsigned long long>();
        sa.reset.n = sa.n_words;
        std::memcpy(sa.reset.v, &init, sizeof init);
        sa.do_plan = spec && !tiles ? 1 : 0;
        sa.plan = h->plan_dev.as<IngestPlan>();
        sa.seq = ++h->pass_seq;   // settle_pending polls for it (no event between the kernels)
        HIPCHK(h, launch_scan_plan(p, pp, sa, h->stream));
        h->counters_clean = true;
    }
    if (spec && !tiles) {
        IngestParams q = p;
        q.bucket_base = s->bucket_off.as<uint32_t>();
        // one lane's units: each workgroup takes its unit of every lane the plan finds active
        for (int l = 0; l < kMaxLanes; l++) q.lane_slot[l] = l == 0 ? 0 : -1;
        q.st_stride = h->st_stride;
        q.st_rec = h->st_rec.as<int64_t>();
        q.st_null = vnull ? h->st_null.as<uint8_t>() : nullptr;
        if (h->cfg.val_type == FG_VAL_NONE) q.val = nullptr;
        q.plan = h->plan_dev.as<IngestPlan>();
        KTimer kt(h, K_PART2, n);
        HIPCHK(h, launch_part2(q, h->stream));
    }
    return FG_OK;
}

int ingest_finish(fg_handle* h, PassState& ps, Counters* out) {
    IngestParams& p = ps.p;
    std::unique_ptr<Staged>& s = ps.s;
    struct PoolBack {   // a pass that stages nothing goes back to the pool
        fg_handle* h;
        std::unique_ptr<Staged>& s;
        ~PoolBack() {
            if (s) h->pass_pool.push_back(std::move(s));
        }
    } pool_back{h, s};
    const bool two_pass = ps.two_pass, spec = ps.spec;
    const uint8_t* vnull = ps.vnull;
    const int64_t n = ps.n, flo = ps.flo, fhi = ps.fhi;
    int rc = FG_OK;
    DevCounters got;   // written by k_scan_plan into host-visible memory
    std::memcpy(&got, h->h_pass.p, sizeof got);
    const bool tiles = ps.tiles;
    IngestPlan plan{};
    if (spec && !tiles) std::memcpy(&plan, h->h_pass.as<char>() + sizeof(DevCounters), sizeof plan);
    const bool staged_by_plan = spec && !tiles && plan.ok;
    out->drops = got.drops;
    out->qmin = got.qmin;
    out->qmax = got.qmax;
    out->qnext = got.qnext;
    // (a tile pass reports its largest bucket count of one tile: skew is > 4x the uniform mean of
    // a lane's 2^(bits - 2) buckets, and > 96 records -- 16x the mean at 1,024 buckets per lane;
    // a uniform stream over few buckets stays on the tiles, a hot key's bucket does not)
    const int64_t tile_mean = kTileRecs >> std::max(0, p.region_bits - kTileBits);
    out->skew = tiles ? (int64_t)got.max_bucket > std::max<int64_t>(kTileRecs / 64, 4 * tile_mean)
                      : (int64_t)got.max_bucket * p.grid > kHeavyMin;
    for (int l = 0; l < kMaxLanes; l++) {
        out->lane_min[l] = JMAX;
        out->lane_max[l] = JMIN;
        out->lane_total[l] = (long long)got.lane_total[l];
    }
    if (got.qmin > got.qmax) return FG_OK;   // nothing accepted
    h->anchor_start = jsub(slice_end_of(h, got.qmin), h->w.slice);
    // qmin/qmax span the batch's accepted records; the pass stages those inside the filter
    const int64_t fq0 = std::max<int64_t>(got.qmin, flo), fq1 = std::min<int64_t>(got.qmax, fhi - 1);
    if (fq0 > fq1) return FG_OK;                                            // none inside
    if (tiles && got.wide) {
        // a key wider than 32 bits: the tile pass truncated it -- void. The lanes' narrow passes go
        // into their tables, tile staging and narrow staging end for good, and the batch is staged
        // again by the two-pass partition with 16-B records (its drops were counted by this pass)
        rc = flush(h);
        if (rc) return rc;
        h->narrow = false;
        h->keys32 = false;
        h->tile_ok = false;
        PassState ps2;
        rc = ingest_launch(h, n, p.key, p.ts, p.val, vnull, flo, fhi, false, ps2);
        if (rc) return rc;
        rc = sync(h);
        if (rc) return rc;
        Counters c2{};
        rc = ingest_finish(h, ps2, &c2);
        const unsigned long long drops = out->drops;
        *out = c2;
        out->drops = drops;
        return rc;
    }
    if (tiles && out->skew && !tile_split_ok(h)) {
        // hot keys (a bucket of one tile above 16x the uniform mean): a tile pass would be fired by
        // one overloaded workgroup per hot bucket, or materialized by one (9.6 ms per 100M-record
        // Zipf(1.1) batch, round 4). Tile staging ends for good and the batch is staged again by
        // the two-pass partition, whose heavy-region path spreads hot keys (its drops were
        // counted by this pass); the pass's tiles go back to the pool unused
        h->tile_skew = true;
        h->pass_pool.push_back(std::move(ps.s));
        PassState ps2;
        rc = ingest_launch(h, n, p.key, p.ts, p.val, vnull, flo, fhi, false, ps2);
        if (rc) return rc;
        rc = sync(h);
        if (rc) return rc;
        Counters c2{};
        rc = ingest_finish(h, ps2, &c2);
        const unsigned long long drops = out->drops;
        *out = c2;
        out->drops = drops;
        return rc;
    }
    if (p.narrow && got.wide) {
        // a key wider than 32 bits under narrow staging (the device plan stopped pass 2; pass 1's
        // 12-B tile records truncated it): the lanes' narrow passes go into their tables, pass 1
        // runs again with 16-B tile records (same histogram and bucket bases; the counters it
        // adds up again are reset before the next pass) and every later pass stays on 16 B
        rc = flush(h);
        if (rc) return rc;
        h->narrow = false;
        h->keys32 = false;
        p.narrow = 0;
        {
            KTimer kt(h, K_PART1, n);
            HIPCHK(h, launch_part1(p, h->stream));
        }
        // (pass 2 reads the histogram as per-workgroup prefixes: convert the rewritten one again)
        HIPCHK(h, launch_hist_columns(h->hist.as<uint32_t>(), h->totals.as<uint32_t>(), p.lanes << p.region_bits,
                                      p.grid, h->stream));
        h->counters_clean = false;
    }
    if ((uint64_t)(fq1 - fq0) >= (uint64_t)h->lanes) return -1;              // more slices than lanes
    for (int64_t q = fq0; q <= fq1; q++) {
        const int l = (int)(q & (h->lanes - 1));
        if (got.lane_mask >> l & 1) out->lane_min[l] = out->lane_max[l] = q;
    }

    if (staged_by_plan) {   // pass 2 ran with the device's decision: the host's is the same
        for (int l = 0; l < h->lanes; l++) {
            if (out->lane_total[l] == 0) continue;
            const Lane& ln = h->lane[l];
            if (out->lane_total[l] > h->lane_cap ||
                (ln.q != kEmptyLane && (ln.q != out->lane_min[l] || ln.fill + out->lane_total[l] > h->lane_cap)))
                return h->fail(FG_ESTATE, "internal: device lane plan disagrees with the host (lane %d)", l);
        }
    }
    // make room: a lane holding another slice, or without space for the batch's records,
    // is flushed into its slice table first (the EOFException flush of RecordsWindowBuffer
    // :91-96, per lane)
    int64_t need = 0;
    for (int l = 0; l < h->lanes; l++) need = std::max<int64_t>(need, out->lane_total[l]);
    if (need > h->lane_cap) {
        rc = flush(h);
        if (rc) return rc;
        rc = grow_lanes(h, need);
        if (rc) return rc;
    }
    {
        bool any = false;
        for (int l = 0; l < h->lanes; l++) {
            if (out->lane_total[l] == 0) continue;
            const Lane& ln = h->lane[l];
            if (ln.q != kEmptyLane && (ln.q != out->lane_min[l] || ln.fill + out->lane_total[l] > h->lane_cap))
                any = true;
        }
        if (any) {
            // flush only the blocking lanes: merge them (no fire) into their tables
            for (int l = 0; l < h->lanes; l++) {
                if (out->lane_total[l] == 0) continue;
                const Lane& ln = h->lane[l];
                if (ln.q == kEmptyLane || (ln.q == out->lane_min[l] && ln.fill + out->lane_total[l] <= h->lane_cap))
                    continue;
                rc = flush_lane(h, l);
                if (rc) return rc;
            }
        }
    }

    // scatter into the lane areas at the bucket bases scanned above
    p.bucket_base = s->bucket_off.as<uint32_t>();
    // staged position of bucket b (lane l) = bucket_base[b] - (records of lanes < l) + lane l's
    // area start + its fill
    int64_t before = 0;
    for (int l = 0; l < kMaxLanes; l++) {
        p.lane_shift[l] = 0;
        s->lane_start[l] = 0;
        s->lane_n[l] = 0;
        if (l >= h->lanes) continue;
        p.lane_shift[l] = (int64_t)l * h->lane_cap + h->lane[l].fill - before;
        before += out->lane_total[l];
    }
    // tile-sorted scatter when at most two lanes are active and their buckets fit LDS
    {
        int nslots = 0;
        for (int l = 0; l < kMaxLanes; l++) p.lane_slot[l] = -1;
        for (int l = 0; l < h->lanes; l++)
            if (out->lane_total[l] > 0) p.lane_slot[l] = nslots++;
        p.sorted = (nslots >= 1 && nslots <= 2 && (nslots << p.region_bits) <= kMaxSortedBuckets) ? 1 : 0;
    }
    p.st_stride = h->st_stride;
    p.st_rec = h->st_rec.as<int64_t>();
    p.st_null = vnull ? h->st_null.as<uint8_t>() : nullptr;
    if (h->cfg.val_type == FG_VAL_NONE) p.val = nullptr;
    if (staged_by_plan || tiles) {
        // (already staged: by the speculative pass 2 at these positions, or in the pass's tiles)
    } else if (two_pass) {
        KTimer kt(h, K_PART2, n);
        HIPCHK(h, launch_part2(p, h->stream));
    } else {
        KTimer kt(h, K_SCATTER, n);
        HIPCHK(h, launch_ingest_scatter(p, h->stream));
    }
    s->has_null = vnull != nullptr;
    s->narrow = p.narrow != 0;
    s->bits = p.region_bits;   // (a flush above may have split the regions since the count)
    s->is_acc = false;
    s->tiles = tiles;
    s->own = false;
    s->busy = false;
    s->skew = out->skew;
    h->skew_seen = h->skew_seen || out->skew;
    if (tiles && out->skew && !tile_split_ok(h)) h->tile_skew = true;
    s->refs = 0;
    for (int l = 0; l < h->lanes; l++) {
        if (out->lane_total[l] == 0) continue;
        Lane& ln = h->lane[l];
        s->lane_start[l] = ln.fill;
        s->lane_n[l] = out->lane_total[l];
        s->refs++;
        ln.q = out->lane_min[l];
        ln.fill += out->lane_total[l];
        ln.passes.push_back(s.get());
    }
    if (s->refs > 0) h->passes.push_back(std::move(s));
    else h->pass_pool.push_back(std::move(s));
    return FG_OK;
}

int ingest_pass(fg_handle* h, int64_t n, const int64_t* key, const int64_t* ts, const int64_t* val,
                const uint8_t* vnull, int64_t flo, int64_t fhi, bool count_drops, Counters* out) {
    PassState ps;
    int rc = ingest_launch(h, n, key, ts, val, vnull, flo, fhi, count_drops, ps);
    if (rc) return rc;
    rc = sync(h);
    if (rc) return rc;
    return ingest_finish(h, ps, out);
}

// grow the per-lane accumulator areas to `need` rows per lane (all lanes free of acc rows)
int grow_acc(fg_handle* h, int64_t need) {
    if (need <= h->acc_cap) return FG_OK;
    for (int l = 0; l < h->lanes; l++)
        if (h->lane[l].acc_fill) return h->fail(FG_ESTATE, "internal: accumulator areas grown while in use");
    const int64_t cap = std::max<int64_t>(need, h->acc_cap + h->acc_cap / 2);
    const size_t b = 8 * (size_t)h->lanes * cap;
    HIPCHK(h, h->acc_key.ensure(b));
    HIPCHK(h, h->acc_cs.ensure(b));
    HIPCHK(h, h->acc_cn.ensure(b));
    HIPCHK(h, h->acc_sum.ensure(b));
    if (h->mv) {
        HIPCHK(h, h->acc_v1.ensure(b));
        HIPCHK(h, h->acc_v2.ensure(b));
    }
    h->acc_cap = cap;
    return FG_OK;
}

// one global-phase pass over partial accumulator rows (device columns; `ts` = the pseudo
// rowtime slice_end - 1 - tz): count pass with the global operator's late rules, then
// the rows are scattered into their slice lanes' accumulator areas. Returns -1 when the
// rows span more slices than the lanes can hold.
int acc_pass(fg_handle* h, int64_t n, const int64_t* key, const int64_t* ts, const int64_t* cs, const int64_t* cv,
             const int64_t* sum, const int64_t* v1, const int64_t* v2, int64_t flo, int64_t fhi, bool count_drops,
             Counters* out) {
    if (int rc0 = ensure_scratch(h)) return rc0;
    IngestParams p{};
    p.w = h->w;
    p.w.local_input = h->w.tz_n > 0 ? 1 : 0;   // partial rows carry local slice ends
    p.n = n;
    p.key = key;
    p.ts = ts;
    p.progress = h->current_progress;
    p.lanes = h->lanes;
    p.region_bits = h->region_bits;
    p.filter_lo = flo;
    p.filter_hi = fhi;
    p.count_drops = count_drops ? 1 : 0;
    int64_t g = (n + 16383) / 16384;
    p.grid = (int)std::max<int64_t>(1, std::min<int64_t>(h->grid, g));
    p.vec = ((uintptr_t)key % 16 == 0 && (uintptr_t)ts % 16 == 0) ? 1 : 0;
    p.hist = h->hist.as<uint32_t>();
    set_fast_path(h, &p);
    DevCounters init{};
    init.qmin = JMAX;
    init.qmax = JMIN;
    init.qnext = JMAX;
    HIPCHK(h, init_counters(h, init));
    h->counters_clean = false;
    DevCounters* dc = h->counters.as<DevCounters>();
    p.drops = &dc->drops;
    p.lane_mask = &dc->lane_mask;
    p.qmin = &dc->qmin;
    p.qmax = &dc->qmax;
    p.qnext = &dc->qnext;
    p.lane_total = dc->lane_total;
    {
        KTimer kt(h, K_COUNT, n);
        HIPCHK(h, launch_ingest_count(p, h->stream));
    }
    HIPCHK(h, hipMemcpyAsync(h->h_counters.p, h->counters.p, sizeof(DevCounters), hipMemcpyDeviceToHost, h->stream));
    int rc = sync(h);
    if (rc) return rc;
    DevCounters got;
    std::memcpy(&got, h->h_counters.p, sizeof got);
    out->drops = got.drops;
    out->qmin = got.qmin;
    out->qmax = got.qmax;
    out->qnext = got.qnext;
    for (int l = 0; l < kMaxLanes; l++) {
        out->lane_min[l] = JMAX;
        out->lane_max[l] = JMIN;
        out->lane_total[l] = (long long)got.lane_total[l];
    }
    if (got.qmin > got.qmax) return FG_OK;
    const int64_t fq0 = std::max<int64_t>(got.qmin, flo), fq1 = std::min<int64_t>(got.qmax, fhi - 1);
    if (fq0 > fq1) return FG_OK;
    if ((uint64_t)(fq1 - fq0) >= (uint64_t)h->lanes) return -1;
    for (int64_t q = fq0; q <= fq1; q++) {
        const int l = (int)(q & (h->lanes - 1));
        if (got.lane_mask >> l & 1) out->lane_min[l] = out->lane_max[l] = q;
    }
    int64_t need = 0;
    for (int l = 0; l < h->lanes; l++) need = std::max<int64_t>(need, out->lane_total[l]);
    if (need > h->acc_cap) {
        rc = flush(h);
        if (rc) return rc;
        rc = grow_acc(h, std::max<int64_t>(need, std::min<int64_t>(h->lane_cap, (int64_t)1 << 24)));
        if (rc) return rc;
    }
    for (int l = 0; l < h->lanes; l++) {
        if (out->lane_total[l] == 0) continue;
        const Lane& ln = h->lane[l];
        if (ln.q == kEmptyLane || (ln.q == out->lane_min[l] && ln.acc_fill + out->lane_total[l] <= h->acc_cap)) continue;
        rc = flush_lane(h, l);
        if (rc) return rc;
    }
    std::unique_ptr<Staged> s = pass_from_pool(h);
    const int Fp = p.lanes << p.region_bits;   // the pass's buckets (the regions may split meanwhile)
    HIPCHK(h, s->bucket_off.ensure(sizeof(uint32_t) * (Fp + 1)));
    {
        KTimer kt(h, K_SCAN, 0);
        HIPCHK(h, launch_hist_columns(h->hist.as<uint32_t>(), h->totals.as<uint32_t>(), Fp, p.grid, h->stream));
        HIPCHK(h, launch_scan_u32(h->totals.as<uint32_t>(), s->bucket_off.as<uint32_t>(), Fp,
                                  h->scan_tmp.as<uint32_t>(), h->stream));
    }
    p.bucket_base = s->bucket_off.as<uint32_t>();
    int64_t before = 0;
    for (int l = 0; l < kMaxLanes; l++) {
        p.lane_shift[l] = 0;
        s->lane_start[l] = 0;
        s->lane_n[l] = 0;
        if (l >= h->lanes) continue;
        p.lane_shift[l] = (int64_t)l * h->acc_cap + h->lane[l].acc_fill - before;
        before += out->lane_total[l];
    }
    AccColumns a{};
    a.in_cnt_star = cs;
    a.in_cnt_val = cv;
    a.in_sum = sum;
    a.key = h->acc_key.as<int64_t>();
    a.cnt_star = h->acc_cs.as<int64_t>();
    a.cnt_null = h->acc_cn.as<int64_t>();
    a.sum = h->acc_sum.as<int64_t>();
    if (h->mv) {
        a.in_v1 = v1;
        a.in_v2 = v2;
        a.v1 = h->acc_v1.as<int64_t>();
        a.v2 = h->acc_v2.as<int64_t>();
    }
    {
        KTimer kt(h, K_SCATTER, n);
        HIPCHK(h, launch_acc_scatter(p, a, h->stream));
    }
    s->has_null = false;
    s->bits = p.region_bits;
    s->is_acc = true;
    s->tiles = false;
    s->own = false;
    s->skew = false;
    s->refs = 0;
    for (int l = 0; l < h->lanes; l++) {
        if (out->lane_total[l] == 0) continue;
        Lane& ln = h->lane[l];
        s->lane_start[l] = ln.acc_fill;
        s->lane_n[l] = out->lane_total[l];
        s->refs++;
        ln.q = out->lane_min[l];
        ln.acc_fill += out->lane_total[l];
        ln.passes.push_back(s.get());
    }
    if (s->refs > 0) h->passes.push_back(std::move(s));
    else h->pass_pool.push_back(std::move(s));
    return FG_OK;
}

int validate(const fg_config* c, std::string* msg) {
    char buf[512];
    buf[0] = 0;
    const long long size = c->size_ms, slide = c->slide_ms, off = c->offset_ms;
    bool has_star = false;
    for (int a = 0; a < c->num_aggs; a++) has_star |= c->aggs[a] == FG_AGG_COUNT_STAR;
    if (c->window_kind == FG_TUMBLE) {
        if (!(size > 0))
            snprintf(buf, sizeof buf, "Tumbling Window parameters must satisfy size > 0, but got size %lldms.", size);
        else if (!((off < 0 ? -off : off) < size))
            snprintf(buf, sizeof buf,
                     "Tumbling Window parameters must satisfy abs(offset) < size, bot got size %lldms and offset %lldms.",
                     size, off);
    } else if (c->window_kind == FG_HOP) {
        if (size <= 0 || slide <= 0)
            snprintf(buf, sizeof buf,
                     "Hopping Window must satisfy slide > 0 and size > 0, but got slide %lldms and size %lldms.", slide,
                     size);
        else if (size % slide != 0)
            snprintf(buf, sizeof buf,
                     "Slicing Hopping Window requires size must be an integral multiple of slide, but got size %lldms and slide %lldms.",
                     size, slide);
        else if (c->mode == FG_MODE_SQL && !has_star && !(c->flags & FG_FLAG_WINDOWED))
            snprintf(buf, sizeof buf, "Hopping window requires a COUNT(*) in the aggregate functions.");
    } else if (c->window_kind == FG_CUMULATE) {
        if (size <= 0 || slide <= 0)
            snprintf(buf, sizeof buf,
                     "Cumulative Window parameters must satisfy maxSize > 0 and step > 0, but got maxSize %lldms and step %lldms.",
                     size, slide);
        else if (size % slide != 0)
            snprintf(buf, sizeof buf,
                     "Cumulative Window requires maxSize must be an integral multiple of step, but got maxSize %lldms and step %lldms.",
                     size, slide);
        else if (c->mode == FG_MODE_DATASTREAM)
            snprintf(buf, sizeof buf, "DataStream has no cumulative window assigner.");
    } else {
        snprintf(buf, sizeof buf, "unknown window kind %d", c->window_kind);
    }
    if (!buf[0]) {
        if (c->num_aggs < 1 || c->num_aggs > FG_MAX_AGGS)
            snprintf(buf, sizeof buf, "num_aggs must be in [1, %d]", FG_MAX_AGGS);
        for (int a = 0; a < c->num_aggs && !buf[0]; a++)
            if (c->aggs[a] < FG_AGG_COUNT_STAR || c->aggs[a] > FG_AGG_MAX) snprintf(buf, sizeof buf, "bad agg %d", c->aggs[a]);
        if (!buf[0]) {   // one value accumulator per (key, slice): SUM-family, MIN or MAX
            int kinds = 0;
            bool sum_family = false, has_min = false, has_max = false;
            for (int a = 0; a < c->num_aggs; a++) {
                sum_family |= c->aggs[a] == FG_AGG_SUM || c->aggs[a] == FG_AGG_AVG || c->aggs[a] == FG_AGG_SUM0;
                has_min |= c->aggs[a] == FG_AGG_MIN;
                has_max |= c->aggs[a] == FG_AGG_MAX;
            }
            kinds = (int)sum_family + (int)has_min + (int)has_max;
            // several kinds: a multi-value operator (value slots SUM, MIN, MAX). DataStream
            // windows reduce ONE aggregation per window (WindowedStream.sum / min / max / minBy /
            // maxBy: SumAggregator or ComparableAggregator), so one value accumulator there
            if (kinds > 1 && c->mode != FG_MODE_SQL)
                snprintf(buf, sizeof buf, "DataStream windows reduce one aggregation (sum, min or max), not a mix");
        }
        if (c->val_type < FG_VAL_NONE || c->val_type > FG_VAL_F64) snprintf(buf, sizeof buf, "bad val_type");
        if (c->val_type == FG_VAL_NONE)
            for (int a = 0; a < c->num_aggs && !buf[0]; a++)
                if (c->aggs[a] != FG_AGG_COUNT_STAR) snprintf(buf, sizeof buf, "aggregates over a value need val_type");
    }
    if (buf[0]) {
        *msg = buf;
        return FG_EINVAL;
    }
    return FG_OK;
}

// The host half of fg_add_batch once the first pass's counters are on the host: its
// decisions (the regular pass 2 when the device's plan said no), the filtered passes for
// the slices outside the first pass's filter, the late-drop count.
int finish_batch(fg_handle* h) {
    PendingBatch& pb = h->pending;
    struct SlotFree {   // every kernel reading the slot's buffers is queued when this runs
        fg_handle* h;
        int slot;
        ~SlotFree() {
            if (slot >= 0) (void)hipEventRecord(h->ev_free[slot], h->stream);
        }
    } slot_free{h, pb.slot};
    pb.slot = -1;
    const int64_t n = pb.n, flo = pb.flo, fhi = pb.fhi;
    const int64_t *key = pb.key, *ts = pb.ts, *val = pb.val;
    const uint8_t* vnull = pb.vnull;
    Counters c{};
    int rc = ingest_finish(h, pb.ps, &c);
    pb.ps = PassState{};
    h->late_dropped += (int64_t)c.drops;
    if (rc != FG_OK && rc != -1) return rc;
    if (c.qmin > c.qmax) return FG_OK;   // nothing accepted
    h->q_guess = (uint64_t)(c.qmax - c.qmin) >= (uint64_t)h->lanes ? c.qmin : kEmptyLane;
    std::vector<std::pair<int64_t, int64_t>> rest;   // slice ranges [a, b) still to stage
    if (rc == -1) {
        rest.push_back({c.qmin, c.qmax + 1});
    } else {
        if (c.qmin < flo) rest.push_back({c.qmin, flo});
        if (c.qmax >= fhi) rest.push_back({c.qnext, c.qmax + 1});   // qnext: first occupied slice >= fhi
    }
    // Each filtered pass reports the next occupied slice above its filter, so empty
    // stretches (a far-future or ancient outlier record) cost no passes.
    for (auto& r : rest) {
        int64_t lo = r.first;
        while (lo < r.second) {
            Counters c2{};
            const int64_t hi = std::min<int64_t>(lo + h->lanes, r.second);
            rc = ingest_pass(h, n, key, ts, val, vnull, lo, hi, false, &c2);
            if (rc == -1) return h->fail(FG_ESTATE, "internal: slice lanes conflict inside a filtered pass");
            if (rc) return rc;
            lo = c2.qnext;   // JMAX when nothing lies above hi
        }
    }
    return FG_OK;
}

// ---- DataStream allowed lateness (fg_late.hip) ------------------------------------------------
// The watermark the late rules compare with: the timer service's (the operator's progress); after
// fg_restore, until the watermark passes it, the checkpoint's -- windows fired before the
// checkpoint keep only their cleanup timers, and their state is resident.
int64_t late_wm(const fg_handle* h) { return std::max(h->current_progress, h->late_horizon); }

// The late elements of a batch (late-allowed: a fired window not yet cleaned), in rounds of one
// element per key, oldest first: each updates its (key, slice) state and FIREs its fired, not
// cleaned windows at once (EventTimeTrigger.onElement :37-46) -- rows appended to the output
// buffers, returned by the next fg_advance_progress ahead of its own rows.
int late_fire(fg_handle* h, int64_t nl) {
    if (int rc0 = complete_fire(h)) return rc0;
    const WindowSpec& w = h->w;
    const int64_t wm = late_wm(h);
    const int64_t nwin = w.kind == TUMBLE ? 1 : w.size / w.slide;
    std::vector<int64_t> ses(nl);
    HIPCHK(h, hipMemcpyAsync(ses.data(), h->lt_se.p, 8 * (size_t)nl, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    std::sort(ses.begin(), ses.end());
    ses.erase(std::unique(ses.begin(), ses.end()), ses.end());
    int rc;
    if (!h->purging) {   // every slice a late element updates holds a table (its windows' state)
        for (int64_t se : ses) {
            SliceTable* t = nullptr;
            rc = table_get(h, se, true, &t);
            if (rc) return rc;
            if (!h->retire_at.count(se) && ds_fired(jadd(se, (nwin - 1) * w.slide), wm))
                h->retire_at[se] = ds_cleanup(jadd(se, (nwin - 1) * w.slide), h->lateness);   // all its windows fired
        }
    }
    // rounds
    uint64_t cap = 1024;
    while (cap < 2 * (uint64_t)nl) cap <<= 1;
    HIPCHK(h, h->lt_done.ensure(nl));
    HIPCHK(h, h->lt_sel.ensure(nl));
    HIPCHK(h, h->lt_slot.ensure(4 * (size_t)nl));
    HIPCHK(h, h->lt_found.ensure(4 * (size_t)nl));
    HIPCHK(h, h->lt_ckey.ensure(8 * (size_t)(cap + 2)));
    HIPCHK(h, h->lt_cidx.ensure(4 * (size_t)(cap + 2)));
    HIPCHK(h, h->lt_h.ensure(64));
    HIPCHK(h, hipMemsetAsync(h->lt_done.p, 0, (size_t)nl, h->stream));
    rc = ensure_out(h, h->late_rows + nl * nwin + 1);
    if (rc) return rc;
    {   // the fired-row counter continues after the rows fired earlier since the last advance
        Words16 wd{};
        wd.v[0] = (unsigned long long)h->late_rows;
        wd.n = 1;
        HIPCHK(h, launch_store_words(reinterpret_cast<unsigned long long*>(h->scalars.as<char>() + 8), wd, h->stream));
    }
    h->out_count_reset = false;   // (the next advance re-bases the counter on late_rows)
    int64_t pending = nl;
    int guard = 0;
    while (pending > 0) {
        if (++guard > 64 + 4 * nl) return h->fail(FG_ESTATE, "internal: late-element rounds do not progress");
        // directory of the slice tables (sorted by slice end), rebuilt per round (a split moves them)
        std::vector<int64_t> dse;
        std::vector<TableRef> dt;
        for (auto& kv : h->tables) {
            dse.push_back(kv.first);
            dt.push_back(ref_of(kv.second.get()));
        }
        const int nd = (int)dse.size();
        HIPCHK(h, h->lt_dir_se.ensure(8 * (size_t)std::max(nd, 1)));
        HIPCHK(h, h->lt_dir_t.ensure(sizeof(TableRef) * (size_t)std::max(nd, 1)));
        HIPCHK(h, h->lt_need.ensure(4 * (size_t)std::max(nd, 1) * h->P));
        if (nd) {
            HIPCHK(h, hipMemcpyAsync(h->lt_dir_se.p, dse.data(), 8 * (size_t)nd, hipMemcpyHostToDevice, h->stream));
            HIPCHK(h, hipMemcpyAsync(h->lt_dir_t.p, dt.data(), sizeof(TableRef) * (size_t)nd, hipMemcpyHostToDevice,
                                     h->stream));
            HIPCHK(h, hipMemsetAsync(h->lt_need.p, 0, 4 * (size_t)nd * h->P, h->stream));
        }
        LateRound p{};
        p.w = w;
        p.wm = wm;
        p.lateness = h->lateness;
        p.purging = h->purging ? 1 : 0;
        p.vt = h->kvt;   // the value op (SumAggregator's sum, or a DataStream MIN / MAX)
        p.region_bits = h->region_bits;
        p.P = h->P;
        p.cap = table_cap(h->mv);
        p.cols = table_cols(h->mv);
        p.n = nl;
        p.mix = h->lt_mix.as<int64_t>();
        p.se = h->lt_se.as<int64_t>();
        p.val = h->lt_val.as<int64_t>();
        p.vnull = h->lt_null.as<uint8_t>();
        p.idx = h->lt_idx.as<uint32_t>();
        p.done = h->lt_done.as<uint8_t>();
        p.sel = h->lt_sel.as<uint8_t>();
        p.slot = h->lt_slot.as<uint32_t>();
        p.found = h->lt_found.as<int32_t>();
        p.claim_key = h->lt_ckey.as<unsigned long long>();
        p.claim_idx = h->lt_cidx.as<uint32_t>();
        p.claim_mask = cap - 1;
        p.need = h->lt_need.as<uint32_t>();
        p.flags = reinterpret_cast<unsigned int*>(h->lt_words.as<char>());
        p.nsel = reinterpret_cast<unsigned long long*>(h->lt_words.as<char>() + 8);
        p.dir = LateDir{h->lt_dir_se.as<int64_t>(), h->lt_dir_t.as<TableRef>(), nd, 0};
        p.num_aggs = h->cfg.num_aggs;
        for (int a = 0; a < h->cfg.num_aggs; a++) {
            p.aggs[a] = h->cfg.aggs[a];
            p.out_agg[a] = h->o_agg[a].as<int64_t>();
        }
        p.out_key = h->o_key.as<int64_t>();
        p.out_ws = h->o_ws.as<int64_t>();
        p.out_we = h->o_we.as<int64_t>();
        p.out_null = h->o_null.as<uint8_t>();
        p.out_rowtime = h->o_rt.as<int64_t>();
        p.out_count = reinterpret_cast<unsigned long long*>(h->scalars.as<char>() + 8);
        p.out_cap = h->out_cap;
        HIPCHK(h, launch_late_reset(p, h->stream));
        HIPCHK(h, launch_late_claim(p, h->stream));
        HIPCHK(h, launch_late_lookup(p, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->lt_h.p, h->lt_words.p, 16, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        const unsigned flags = h->lt_h.as<unsigned int>()[0];
        if (flags & 2u) return h->fail(FG_ESTATE, "internal: a late element's slice table is missing");
        if (flags & 1u) {   // a region cannot take the round's new entries: split and redo the round
            rc = grow(h, h->region_bits + 1);
            if (rc) return rc;
            continue;
        }
        const int64_t nsel = (int64_t)h->lt_h.as<unsigned long long>()[1];
        HIPCHK(h, launch_late_update(p, h->stream));
        HIPCHK(h, launch_late_emit(p, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->lt_h.p, h->lt_words.p, 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->lt_h.as<char>() + 16, h->scalars.as<char>() + 8, 8, hipMemcpyDeviceToHost,
                                 h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        if (h->lt_h.as<unsigned int>()[0] & 4u) return h->fail(FG_EDEVICE, "internal: late-row buffer overflow");
        h->late_rows = (int64_t)h->lt_h.as<unsigned long long>()[2];
        pending -= nsel;
    }
    if (!h->purging)
        for (int64_t se : ses) {
            SliceTable* t = nullptr;
            table_get(h, se, false, &t);
            if (t) {
                t->upper = std::min<int64_t>(t->upper + nl, kStateCapMax);
                t->changed = true;
            }
        }
    return FG_OK;
}

// The batch's late-allowed elements (k_late_split) are fired here; the others replace the batch
// (compacted into engine buffers). Returns the remaining record count in *n_regular.
int late_split(fg_handle* h, int64_t n, const int64_t** key, const int64_t** ts, const int64_t** val,
               const uint8_t** vnull, int64_t* n_regular) {
    // the previous batch's remainder may still be read by its queued passes: no reallocation under them
    if (h->lt_r_key.bytes < 8 * (size_t)n) HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, h->lt_mix.ensure(8 * (size_t)n));
    HIPCHK(h, h->lt_se.ensure(8 * (size_t)n));
    HIPCHK(h, h->lt_val.ensure(8 * (size_t)n));
    HIPCHK(h, h->lt_null.ensure((size_t)n));
    HIPCHK(h, h->lt_idx.ensure(4 * (size_t)n));
    HIPCHK(h, h->lt_words.ensure(64));
    HIPCHK(h, h->lt_r_key.ensure(8 * (size_t)n));
    HIPCHK(h, h->lt_r_ts.ensure(8 * (size_t)n));
    if (*val) HIPCHK(h, h->lt_r_val.ensure(8 * (size_t)n));
    if (*vnull) HIPCHK(h, h->lt_r_null.ensure((size_t)n));
    HIPCHK(h, h->lt_h.ensure(64));
    unsigned long long* counts = reinterpret_cast<unsigned long long*>(h->lt_words.as<char>() + 32);
    HIPCHK(h, hipMemsetAsync(counts, 0, 16, h->stream));
    LateSplit p{};
    p.w = h->w;
    p.wm = late_wm(h);
    p.lateness = h->lateness;
    p.purging = h->purging ? 1 : 0;
    p.n = n;
    p.key = *key;
    p.ts = *ts;
    p.val = *val;
    p.vnull = *vnull;
    p.counts = counts;
    p.l_mix = h->lt_mix.as<int64_t>();
    p.l_se = h->lt_se.as<int64_t>();
    p.l_val = h->lt_val.as<int64_t>();
    p.l_null = h->lt_null.as<uint8_t>();
    p.l_idx = h->lt_idx.as<uint32_t>();
    p.r_key = h->lt_r_key.as<int64_t>();
    p.r_ts = h->lt_r_ts.as<int64_t>();
    p.r_val = *val ? h->lt_r_val.as<int64_t>() : nullptr;
    p.r_null = *vnull ? h->lt_r_null.as<uint8_t>() : nullptr;
    HIPCHK(h, launch_late_split(p, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->lt_h.p, counts, 16, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const int64_t nl = (int64_t)h->lt_h.as<unsigned long long>()[0];
    const int64_t nr = (int64_t)h->lt_h.as<unsigned long long>()[1];
    *n_regular = n;
    if (nl == 0) return FG_OK;   // nothing late: the batch as it is
    // late elements go into the resident slice tables without pass 1's 32-bit key check: the
    // narrow LDS table (keyed by the int32 of an entry's mix) is off from here on
    h->keys32 = false;
    if (!*vnull) {   // (the late list's NULL flags are all 0)
        HIPCHK(h, hipMemsetAsync(h->lt_null.p, 0, (size_t)nl, h->stream));
    }
    int rc = late_fire(h, nl);
    if (rc) return rc;
    *n_regular = nr;
    *key = h->lt_r_key.as<int64_t>();
    *ts = h->lt_r_ts.as<int64_t>();
    if (*val) *val = h->lt_r_val.as<int64_t>();
    if (*vnull) *vnull = h->lt_r_null.as<uint8_t>();
    return FG_OK;
}

// Every entry point first completes a deferred batch (its counters were copied behind
// pass 1's plan, so the wait is usually over before pass 2 ends).
int settle_pending(fg_handle* h) {
    if (int rc0 = complete_fire(h)) return rc0;   // every entry point but a quiet async advance
    if (!h->pending.active) return FG_OK;
    h->pending.active = false;
    // k_scan_plan writes its sequence word into coherent host memory after the counters and
    // the plan: poll for it (pass 1 is done by then; pass 2 still runs). A stream error or a
    // lost write falls back to synchronizing the stream.
    const volatile unsigned long long* sq = reinterpret_cast<const volatile unsigned long long*>(
        h->h_pass.as<char>() + sizeof(DevCounters) + sizeof(IngestPlan));
    for (int64_t spin = 0; *sq != h->pass_seq; spin++) {
        if (spin > (1 << 12) && hipStreamQuery(h->stream) != hipErrorNotReady) {
            HIPCHK(h, hipStreamSynchronize(h->stream));
            if (*sq != h->pass_seq) return h->fail(FG_EDEVICE, "internal: pass counters never arrived");
            break;
        }
    }
    return finish_batch(h);
}

}  // namespace

extern "C" {

int fg_abi_version(void) { return FG_ABI_VERSION; }

int fg_selftest(int32_t device_id, char* msg, int32_t cap) {
    static std::mutex mu;
    static std::map<int, std::pair<int, std::string>> done;   // device -> (result, message)
    std::lock_guard<std::mutex> g(mu);
    auto it = done.find(device_id);
    if (it == done.end()) {
        char m[160] = "";
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || device_id < 0 || device_id >= ndev) {
            if (msg && cap > 0) snprintf(msg, (size_t)cap, "no such HIP device");
            return FG_EDEVICE;
        }
        const int r = run_selftest(device_id, m, sizeof m);
        it = done.emplace(device_id, std::make_pair(r, std::string(m))).first;
    }
    if (msg && cap > 0) snprintf(msg, (size_t)cap, "%s", it->second.second.c_str());
    return it->second.first == 0 ? FG_OK : FG_EDEVICE;
}

// Page-locking caller memory (the shim's off-heap MemorySegments): an FG_HOST batch read from
// a registered range is DMA'd straight from it by hipMemcpyAsync; pageable memory is first
// staged through the runtime's bounce buffers, chunk by chunk, at about half the link rate.
int fg_host_register(int32_t device_id, void* p, int64_t bytes) {
    if (!p || bytes <= 0) {
        g_open_error = "fg_host_register: null range";
        return FG_EINVAL;
    }
    if (hipSetDevice(device_id) != hipSuccess) {
        g_open_error = "fg_host_register: bad device";
        return FG_EDEVICE;
    }
    const hipError_t e = hipHostRegister(p, (size_t)bytes, hipHostRegisterDefault);
    if (e != hipSuccess) {
        g_open_error = std::string("hipHostRegister: ") + hipGetErrorString(e);
        return e == hipErrorHostMemoryAlreadyRegistered || e == hipErrorInvalidValue ? FG_EINVAL : FG_EDEVICE;
    }
    return FG_OK;
}

int fg_host_unregister(int32_t device_id, void* p) {
    if (!p) {
        g_open_error = "fg_host_unregister: null pointer";
        return FG_EINVAL;
    }
    if (hipSetDevice(device_id) != hipSuccess) {
        g_open_error = "fg_host_unregister: bad device";
        return FG_EDEVICE;
    }
    const hipError_t e = hipHostUnregister(p);
    if (e != hipSuccess) {
        g_open_error = std::string("hipHostUnregister: ") + hipGetErrorString(e);
        return e == hipErrorHostMemoryNotRegistered || e == hipErrorInvalidValue ? FG_EINVAL : FG_EDEVICE;
    }
    return FG_OK;
}

// FG_BACKTRACE=1 (diagnostics, standalone or Python hosts only): a host fault prints the native
// frames to stderr. Installed only while SIGSEGV has its default disposition -- a JVM (the JNI
// shim) handles SIGSEGV itself for implicit null checks and safepoint polls, and its handler is
// never replaced.
static void fg_fault_trace(int sig) {
    void* b[64];
    const int n = backtrace(b, 64);
    backtrace_symbols_fd(b, n, 2);
    std::signal(sig, SIG_DFL);
    std::raise(sig);
}

int fg_open(const fg_config* cfg, fg_handle** out) {
    if (getenv("FG_BACKTRACE")) {   // (on its own stack: a stack overflow is traced too)
        struct sigaction old{};
        sigaction(SIGSEGV, nullptr, &old);
        if (!(old.sa_flags & SA_SIGINFO) && old.sa_handler == SIG_DFL) {
            static char alt[1 << 16];
            stack_t ss{};
            ss.ss_sp = alt;
            ss.ss_size = sizeof alt;
            sigaltstack(&ss, nullptr);
            struct sigaction sa{};
            sa.sa_handler = fg_fault_trace;
            sa.sa_flags = SA_ONSTACK;
            sigaction(SIGSEGV, &sa, nullptr);
        }
    }
    if (!out) {
        g_open_error = "null handle pointer";
        return FG_EINVAL;
    }
    *out = nullptr;
    if (!cfg) {
        g_open_error = "null config";
        return FG_EINVAL;
    }
    fg_config c = *cfg;
    const bool local = (c.flags & FG_FLAG_LOCAL_PARTIALS) != 0;
    if (local) {
        // the local phase emits the accumulator layout COUNT(*), COUNT(v), SUM
        if (c.val_type == FG_VAL_NONE || c.mode != FG_MODE_SQL) {
            g_open_error = "FG_FLAG_LOCAL_PARTIALS needs an SQL operator with a value column";
            return FG_EINVAL;
        }
        // a MIN / MAX in the global operator's list makes the partial accumulator a MIN / MAX;
        // the partial row holds ONE value accumulator, so the list may name one kind only
        int32_t vagg = FG_AGG_SUM;
        bool sum_family = false, has_min = false, has_max = false;
        for (int a = 0; a < c.num_aggs && a < FG_MAX_AGGS; a++) {
            if (c.aggs[a] == FG_AGG_MIN || c.aggs[a] == FG_AGG_MAX) vagg = c.aggs[a];
            has_min |= c.aggs[a] == FG_AGG_MIN;
            has_max |= c.aggs[a] == FG_AGG_MAX;
            sum_family |= c.aggs[a] == FG_AGG_SUM || c.aggs[a] == FG_AGG_AVG || c.aggs[a] == FG_AGG_SUM0;
        }
        c.num_aggs = 3;
        c.aggs[0] = FG_AGG_COUNT_STAR;
        c.aggs[1] = FG_AGG_COUNT;
        c.aggs[2] = vagg;
        if ((int)sum_family + (int)has_min + (int)has_max > 1) {
            // several value accumulators: the partial row carries SUM, MIN and MAX
            // (agg[2..4]; a kind absent from the list travels as its identity)
            c.num_aggs = 5;
            c.aggs[2] = FG_AGG_SUM;
            c.aggs[3] = FG_AGG_MIN;
            c.aggs[4] = FG_AGG_MAX;
        }
    }
    if (c.allowed_lateness_ms < 0) {   // WindowedStream.allowedLateness: "The allowed lateness cannot be negative."
        g_open_error = "The allowed lateness cannot be negative.";
        return FG_EINVAL;
    }
    if (c.allowed_lateness_ms > 0 && c.mode != FG_MODE_DATASTREAM) {
        g_open_error = "allowed_lateness_ms is a DataStream WindowOperator setting (SQL window operators have none)";
        return FG_EINVAL;
    }
    if ((c.flags & FG_FLAG_PURGING_TRIGGER) && c.mode != FG_MODE_DATASTREAM) {
        g_open_error = "FG_FLAG_PURGING_TRIGGER is a DataStream WindowOperator trigger";
        return FG_EINVAL;
    }
    const bool proctime = (c.flags & FG_FLAG_PROCTIME) != 0;
    if (proctime && (c.mode != FG_MODE_SQL || local)) {
        g_open_error = "FG_FLAG_PROCTIME is for SQL window aggregation (not DataStream or the local phase)";
        return FG_EINVAL;
    }
    const bool windowed = (c.flags & FG_FLAG_WINDOWED) != 0;
    if (windowed && (c.mode != FG_MODE_SQL || local || proctime)) {
        // WindowedSliceAssigner.isEventTime() is always true (SliceAssigners.java:430-434)
        g_open_error = "FG_FLAG_WINDOWED is for SQL event-time window aggregation (not DataStream, processing time "
                       "or the local phase)";
        return FG_EINVAL;
    }
    if (c.n_tz_transitions < 0 || (c.n_tz_transitions > 0 && (!c.tz_transition_ms || !c.tz_offset_ms))) {
        g_open_error = "zone rules need n_tz_transitions instants and n_tz_transitions + 1 offsets";
        return FG_EINVAL;
    }
    if (c.n_tz_transitions > 0) {
        if (c.mode != FG_MODE_SQL) {
            g_open_error = "zone rules (daylight saving) are for SQL window aggregation, not DataStream";
            return FG_EINVAL;
        }
        for (int32_t i = 0; i + 1 < c.n_tz_transitions; i++)
            if (c.tz_transition_ms[i] >= c.tz_transition_ms[i + 1]) {
                g_open_error = "zone transitions must be ascending";
                return FG_EINVAL;
            }
        for (int32_t i = 0; i <= c.n_tz_transitions; i++)
            if (c.tz_offset_ms[i] < -18ll * 3600 * 1000 || c.tz_offset_ms[i] > 18ll * 3600 * 1000) {
                g_open_error = "zone offsets must lie within +-18 h (ZoneOffset)";
                return FG_EINVAL;
            }
    }
    std::string msg;
    int rc = validate(&c, &msg);
    if (rc) {
        g_open_error = msg;
        return rc;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        g_open_error = "no HIP device available (libflinkgpu needs an MI355X / gfx950)";
        return FG_EDEVICE;
    }
    if (cfg->device_id < 0 || cfg->device_id >= ndev) {
        g_open_error = "device_id out of range";
        return FG_EINVAL;
    }
    {   // the device self-check, once per process and device: a build whose scans or tile walk came
        // out wrong (a compiler fold) fails here instead of firing wrong rows
        char m[160];
        if (fg_selftest(cfg->device_id, m, sizeof m) != FG_OK) {
            g_open_error = m;
            return FG_EDEVICE;
        }
    }
    std::unique_ptr<fg_handle> h(new fg_handle());
    h->cfg = c;
    h->kvt = c.val_type;   // kernel value op: val_type | op << 2 (op 1 MIN, 2 MAX; fg_kernels.hip lds_add)
    {
        bool sum_family = false, has_min = false, has_max = false;
        for (int a = 0; a < c.num_aggs; a++) {
            sum_family |= c.aggs[a] == FG_AGG_SUM || c.aggs[a] == FG_AGG_AVG || c.aggs[a] == FG_AGG_SUM0;
            has_min |= c.aggs[a] == FG_AGG_MIN;
            has_max |= c.aggs[a] == FG_AGG_MAX;
        }
        if ((int)sum_family + (int)has_min + (int)has_max > 1) {
            // the reference's generated accumulator row holds every aggregate's accumulator
            // (AggsHandlerCodeGenerator.scala:578-700): one operator, one staging, value slots
            // 0 SUM (SUM / AVG / SUM0), 1 MIN, 2 MAX
            h->mv = 1;
            h->tcap = kRegionCapMV;
            h->vop[0] = sum_family ? 0 : 3;
            h->vop[1] = has_min ? 1 : 3;
            h->vop[2] = has_max ? 2 : 3;
            for (int a = 0; a < c.num_aggs; a++)
                h->agg_slot[a] = c.aggs[a] == FG_AGG_MIN ? 1 : c.aggs[a] == FG_AGG_MAX ? 2 : 0;
        } else {
            // DataStream DOUBLE MIN / MAX compare by Double.compareTo (ComparableAggregator:
            // ops 3 / 4, fg_kernels.hip kVtMinT); SQL's and BIGINT's by the primitive comparison
            const int ds_f64 = c.mode == FG_MODE_DATASTREAM && c.val_type == FG_VAL_F64 ? 2 : 0;
            for (int a = 0; a < c.num_aggs; a++) {
                if (c.aggs[a] == FG_AGG_MIN) h->kvt = c.val_type | ((1 + ds_f64) << 2);
                if (c.aggs[a] == FG_AGG_MAX) h->kvt = c.val_type | ((2 + ds_f64) << 2);
            }
        }
    }
    h->local = local;
    h->proctime = proctime;
    h->lateness = c.mode == FG_MODE_DATASTREAM ? c.allowed_lateness_ms : 0;
    h->purging = c.mode == FG_MODE_DATASTREAM && (c.flags & FG_FLAG_PURGING_TRIGGER) != 0;
    h->retain = h->lateness > 0 && !h->purging;
    if (h->lateness > 0 && h->mv) {
        g_open_error = "allowed lateness: one value accumulator (DataStream SumAggregator)";
        return FG_EINVAL;
    }
    h->device = cfg->device_id;
    h->timing = (cfg->flags & FG_FLAG_KERNEL_TIMING) != 0;
    if (const char* e = getenv("FG_KERNEL_TIMING")) h->timing = h->timing && std::atoi(e) != 0;   // A/B of the events' cost
    if (hipSetDevice(h->device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        g_open_error = "hipSetDevice/hipStreamCreate failed";
        return FG_EDEVICE;
    }
    if (h->timing) {   // timing events made up front: none is created on the launch path
        h->ev_pool.reserve(2304);
        for (int i = 0; i < 2304; i++) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) break;
            h->ev_pool.push_back(e);
        }
    }
    WindowSpec& w = h->w;
    w.kind = cfg->window_kind;
    w.mode = cfg->mode;
    w.size = cfg->size_ms;
    w.slide = cfg->window_kind == FG_TUMBLE ? cfg->size_ms : cfg->slide_ms;
    w.offset = cfg->offset_ms;
    w.tz = cfg->mode == FG_MODE_DATASTREAM ? 0 : cfg->shift_tz_offset_ms;
    w.slice = cfg->window_kind == FG_HOP ? gcd64(w.size, w.slide) : w.slide;
    w.nslices = w.size / w.slice;
    w.rslice = 1.0 / (double)w.slice;
    w.rsize = 1.0 / (double)w.size;
    if (c.n_tz_transitions > 0) {   // zone rules: host copy + HBM copy for the kernels
        const size_t n = (size_t)c.n_tz_transitions;
        h->tz_trans.assign(c.tz_transition_ms, c.tz_transition_ms + n);
        h->tz_offs.assign(c.tz_offset_ms, c.tz_offset_ms + n + 1);
        if (h->tz_dev.ensure(8 * (2 * n + 1)) != hipSuccess ||
            hipMemcpy(h->tz_dev.p, h->tz_trans.data(), 8 * n, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(h->tz_dev.as<int64_t>() + n, h->tz_offs.data(), 8 * (n + 1), hipMemcpyHostToDevice) != hipSuccess) {
            g_open_error = "zone rules: device copy failed";
            return FG_EDEVICE;
        }
        w.tz = 0;
        w.tz_n = c.n_tz_transitions;
        w.tz_dst = c.tz_use_daylight ? 1 : 0;
        w.tz_trans_h = h->tz_trans.data();
        w.tz_offs_h = h->tz_offs.data();
        w.tz_trans_d = h->tz_dev.as<int64_t>();
        w.tz_offs_d = h->tz_dev.as<int64_t>() + n;
    }
    h->slice_phase = ((w.offset % w.slice) + w.slice) % w.slice;
    if (windowed) {   // each window its own slice: a tumbling spec of the inner slice interval
        h->windowed = true;
        h->inner = w;
        w.kind = TUMBLE;
        w.size = w.slide = w.slice;
        w.nslices = 1;
        w.rsize = w.rslice;
        if (w.tz_n > 0) w.local_input = 1;   // window ends are local times (zone rules)
    }

    // Regions: keys per region ~35 % of the kSlots LDS slots, so linear probes stay short (a
    // wave's probe loop runs at its lanes' probe counts), up to 2^13 regions. A region that
    // overflows later splits (settle_jobs / grow), so the hint sizes for speed, not for
    // correctness. expected_keys <= 0 (a shim without a key-count hint): 2^10 regions
    // (~1.4M keys per slice at that load, 117 MB per slice table), grown on demand.
    int bits = 0;
    if (cfg->expected_keys > 0) {
        const int slots = h->mv ? kSlotsMV : kSlots;
        while (bits < kMaxRegionBits && ((int64_t)1 << bits) * (int64_t)(slots * 0.35) < cfg->expected_keys) bits++;
        // a merge runs one region per workgroup: an operator of a few thousand keys would fire
        // each window on a handful of CUs, so from 4,096 expected keys it takes at least
        // 2^FG_MIN_REGION_BITS regions (more, emptier LDS tables; every CU busy at a fire)
        // (TUMBLE and the local phase: 2^10 -- their windows fire straight from the tile passes,
        // one workgroup per bucket of 4 regions, so 256 buckets per slice keep every CU busy and
        // a tile's fragment of a bucket at ~24 records; their slice tables are rarely written)
        int min_bits = (w.kind == TUMBLE || local) && h->lateness == 0 ? 10 : 8;
        if (const char* e = getenv("FG_MIN_REGION_BITS")) min_bits = std::max(0, std::min(kMaxRegionBits, std::atoi(e)));
        if (cfg->expected_keys >= 4096 && bits < min_bits) bits = min_bits;
    } else {
        bits = kDefaultRegionBits;
    }
    h->region_bits = bits;
    h->P = 1 << bits;
    // the staging buckets are the state regions: one region per merge workgroup pass
    h->lanes = lanes_for(bits);
    h->lanes_target = h->lanes;
    h->F = h->lanes << h->region_bits;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, h->device) == hipSuccess) {
        h->grid = std::max(1, prop.multiProcessorCount);
        h->merge_grid = std::max(1, prop.multiProcessorCount);
    }
    // per-lane staged areas: buffer_records records per lane
    h->lane_cap = cfg->buffer_records > 0 ? cfg->buffer_records : (int64_t)1 << 26;
    fg_handle* hp = h.get();
    auto chk = [&](hipError_t e) { return e == hipSuccess; };
    hp->st_stride = cfg->val_type == FG_VAL_NONE ? 1 : 2;
    bool ok = chk(hp->st_rec.ensure(8 * (size_t)hp->st_stride * hp->lanes * hp->lane_cap + kRec12Block)) &&
              chk(hp->st_null.ensure((size_t)hp->lanes * hp->lane_cap)) &&
              chk(hp->hist.ensure(4 * (size_t)hp->F * hp->grid)) &&
              chk(hp->totals.ensure(4 * ((size_t)hp->F + 1))) &&
              chk(hp->scan_tmp.ensure(4 * scan_tmp_words((int64_t)hp->F))) &&
              chk(hp->counters.ensure(sizeof(Counters))) &&
              chk(hp->h_counters.ensure(sizeof(Counters) + sizeof(IngestPlan))) &&
              chk(hp->plan_dev.ensure(sizeof(IngestPlan))) && chk(hp->row_bad.ensure(16)) &&
              chk(hp->h_pass.ensure(sizeof(DevCounters) + sizeof(IngestPlan) + 8, hipHostMallocCoherent)) &&
              chk(hp->h_fire.ensure(kScalarBytes + 8, hipHostMallocCoherent)) &&
              chk(hp->arena.ensure(1 << 20)) && chk(hp->h_arena.ensure(1 << 20)) && chk(hp->scalars.ensure(64)) && chk(hp->sink.ensure(256)) &&
              chk(hp->h_scalars.ensure(64)) && chk(hp->fail_list.ensure(4 * (size_t)kFailCap));
    if (!ok) {
        g_open_error = "device allocation failed";
        return FG_EDEVICE;
    }
    if (const char* e = getenv("FG_SPECULATE")) hp->speculate = std::atoi(e) != 0;
    // narrow 12-B staging for the two-pass partition of a one-value operator
    hp->narrow = hp->st_stride == 2 && !hp->mv && hp->region_bits >= kFineBits;
    hp->narrow_ok = hp->narrow;
    if (const char* e = getenv("FG_TILE_STATE")) hp->tile_state = std::atoi(e) != 0;
    if (const char* e = getenv("FG_TILE_GRID")) hp->tile_grid_force = std::atoi(e);
    if (const char* e = getenv("FG_TILE_SPLIT")) hp->tile_split = std::atoi(e) != 0;
    if (const char* e = getenv("FG_TILE_HOT")) hp->tile_hot = std::atoi(e) != 0;
    hp->tile_ok = true;
    if (hipEventCreateWithFlags(&hp->ev_pending, hipEventDisableTiming) != hipSuccess) {
        g_open_error = "hipEventCreate failed";
        return FG_EDEVICE;
    }
    *out = h.release();
    return FG_OK;
}

int fg_add_batch(fg_handle* h, const fg_batch* b) {
    if (!h || !b) return FG_EINVAL;
    if (b->n <= 0) return FG_OK;
    if (b->n > (int64_t)0x7fffffff) return h->fail(FG_EINVAL, "batch larger than 2^31-1 records");
    if (!b->key || !b->rowtime) return h->fail(FG_EINVAL, "batch key/rowtime columns are required");
    if (h->cfg.val_type != FG_VAL_NONE && !b->val) return h->fail(FG_EINVAL, "batch value column is required");
    h->cnt_bound = b->n > JMAX - h->cnt_bound ? JMAX : h->cnt_bound + b->n;
    const int fmt = b->format;
    if (fmt & ~(FG_BATCH_KEY32 | FG_BATCH_ROWTIME32 | FG_BATCH_VAL32)) return h->fail(FG_EINVAL, "bad fg_batch.format %d", fmt);
    if (fmt && b->location != FG_HOST) return h->fail(FG_EINVAL, "narrow fg_batch columns are for FG_HOST batches");
    if ((fmt & FG_BATCH_VAL32) && h->cfg.val_type != FG_VAL_I64)
        return h->fail(FG_EINVAL, "FG_BATCH_VAL32 needs a BIGINT value column");
    HIPCHK(h, hipSetDevice(h->device));
    // A fire queued by fg_advance_progress_async completes once this batch's pass 1 is queued
    // behind it (ingest_launch): pass 1 touches nothing a region retry of the fire reads.
    if (!(h->fire_pending && !h->pending.active && !h->windowed && h->lateness == 0)) {
        if (int rc0 = settle_pending(h)) return rc0;
        maybe_reduce_lanes(h);
    }
    int64_t n = b->n;
    const int64_t *key = b->key, *ts = b->rowtime;
    const int64_t* val = h->cfg.val_type != FG_VAL_NONE ? static_cast<const int64_t*>(b->val) : nullptr;
    const uint8_t* vnull = b->val_null;
    int slot = -1;   // FG_HOST: the device buffer set this batch was copied into
    if (b->location == FG_HOST) {
        // double-buffered H2D (RecordsWindowBuffer.addElement receives the records from the
        // JVM, :81-97; the shim hands a micro-batch of them): the copy runs on the copy stream
        // while the previous batch's kernels run on the engine stream
        if (!h->copy_stream) {
            HIPCHK(h, hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking));
            for (int i = 0; i < 2; i++) {
                HIPCHK(h, hipEventCreateWithFlags(&h->ev_copied[i], hipEventDisableTiming));
                HIPCHK(h, hipEventCreateWithFlags(&h->ev_free[i], hipEventDisableTiming));
                HIPCHK(h, hipEventRecord(h->ev_free[i], h->stream));
            }
        }
        slot = h->hslot;
        h->hslot ^= 1;
        const bool grow = h->hb_key[slot].bytes < (size_t)(8 * n) || (val && h->hb_val[slot].bytes < (size_t)(8 * n)) ||
                          (vnull && h->hb_null[slot].bytes < (size_t)n);
        if (grow) HIPCHK(h, hipEventSynchronize(h->ev_free[slot]));   // the old buffers are freed
        HIPCHK(h, h->hb_key[slot].ensure(8 * n));
        HIPCHK(h, h->hb_ts[slot].ensure(8 * n));
        if (val) HIPCHK(h, h->hb_val[slot].ensure(8 * n));
        HIPCHK(h, hipStreamWaitEvent(h->copy_stream, h->ev_free[slot], 0));
        // a narrow column (fg_batch.format) crosses the link at 4 bytes a record into
        // hb_narrow, and is widened into the 8-byte column on the copy stream
        uint8_t* nw = nullptr;
        if (fmt) {
            HIPCHK(h, h->hb_narrow[slot].ensure(12 * n));
            nw = h->hb_narrow[slot].as<uint8_t>();
        }
        auto h2d = [&](DevBuf& wide, const void* src, int bit, int k) -> hipError_t {
            if (fmt & bit) return hipMemcpyAsync(nw + 4 * n * k, src, 4 * n, hipMemcpyHostToDevice, h->copy_stream);
            return hipMemcpyAsync(wide.p, src, 8 * n, hipMemcpyHostToDevice, h->copy_stream);
        };
        HIPCHK(h, h2d(h->hb_key[slot], key, FG_BATCH_KEY32, 0));
        HIPCHK(h, h2d(h->hb_ts[slot], ts, FG_BATCH_ROWTIME32, 1));
        if (val) HIPCHK(h, h2d(h->hb_val[slot], val, FG_BATCH_VAL32, 2));
        key = h->hb_key[slot].as<int64_t>();
        ts = h->hb_ts[slot].as<int64_t>();
        if (val) val = h->hb_val[slot].as<int64_t>();
        if (fmt)
            HIPCHK(h, launch_widen_columns((fmt & FG_BATCH_KEY32) ? reinterpret_cast<const int32_t*>(nw) : nullptr,
                                           (fmt & FG_BATCH_ROWTIME32) ? reinterpret_cast<const uint32_t*>(nw + 4 * n) : nullptr,
                                           (fmt & FG_BATCH_VAL32) && val ? reinterpret_cast<const int32_t*>(nw + 8 * n) : nullptr,
                                           n, b->rowtime_base, const_cast<int64_t*>(key), const_cast<int64_t*>(ts),
                                           const_cast<int64_t*>(val), h->copy_stream));
        if (vnull) {
            HIPCHK(h, h->hb_null[slot].ensure(n));
            HIPCHK(h, hipMemcpyAsync(h->hb_null[slot].p, vnull, n, hipMemcpyHostToDevice, h->copy_stream));
            vnull = h->hb_null[slot].as<uint8_t>();
        }
        HIPCHK(h, hipEventRecord(h->ev_copied[slot], h->copy_stream));
        HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_copied[slot], 0));
    }
    struct SlotFree {   // every kernel reading the slot's buffers is queued when this runs
        fg_handle* h;
        int slot;
        ~SlotFree() {
            if (slot >= 0) (void)hipEventRecord(h->ev_free[slot], h->stream);
        }
    } slot_free{h, slot};
    // The caller's host columns are read by the DMA until ev_copied: the call returns only
    // after it (the header's contract -- a shim recycles its pinned staging ring right away,
    // as RecordsWindowBuffer's callers reuse their row objects, RecordsWindowBuffer.java:81-97).
    // The kernels of this batch are queued first, so the GPU keeps working on the engine
    // stream while the host waits for the copy.
    struct CopyWait {
        hipEvent_t e;
        ~CopyWait() {
            if (e) (void)hipEventSynchronize(e);
        }
    } copy_wait{slot >= 0 ? h->ev_copied[slot] : nullptr};
    if (h->windowed) {   // window_end -> pseudo rowtime (every end on the slice grid)
        HIPCHK(h, h->in_wts.ensure(8 * n + 8));
        unsigned long long* bad = reinterpret_cast<unsigned long long*>(h->in_wts.as<int64_t>() + n);
        HIPCHK(h, hipMemsetAsync(bad, 0, 8, h->stream));
        HIPCHK(h, launch_window_end_rowtime(ts, n, h->w.tz, h->w.slice, h->slice_phase, h->in_wts.as<int64_t>(), bad,
                                            h->stream));
        HIPCHK(h, hipMemcpyAsync(h->h_counters.p, bad, 8, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        unsigned long long nbad = 0;
        std::memcpy(&nbad, h->h_counters.p, 8);
        if (nbad)
            return h->fail(FG_EINVAL, "windowed input: %llu window_end values off the slice grid of the window", nbad);
        ts = h->in_wts.as<int64_t>();
    }
    // DataStream allowed lateness: elements of fired, not yet cleaned windows FIRE them now
    // (late_split / late_fire); the rest go on as the batch
    if (h->lateness > 0) {
        h->records_in += n;
        int64_t nr = n;
        int rcl = late_split(h, n, &key, &ts, &val, &vnull, &nr);
        if (rcl) return rcl;
        if (nr == 0) return FG_OK;
        h->records_in -= nr;   // (counted below)
        n = nr;
    }
    // EOFException semantics (RecordsWindowBuffer.java:91-96) are applied per lane inside
    // ingest_pass: a lane without room is flushed into its slice table, then the pass stages
    h->records_in += n;
    {
        int64_t t_first = 0;   // the batch's first rowtime as the caller holds it
        if (b->location == FG_HOST && !h->windowed)
            t_first = (fmt & FG_BATCH_ROWTIME32)
                          ? (int64_t)((uint64_t)b->rowtime_base + *reinterpret_cast<const uint32_t*>(b->rowtime))
                          : b->rowtime[0];
        int rc0 = b->location == FG_HOST && !h->windowed ? seed_anchor(h, nullptr, &t_first) : seed_anchor(h, ts, nullptr);
        if (rc0) return rc0;
    }
    // First pass: every slice -- or, while batches span more slices than the staged lanes
    // (out-of-order jitter, long batches), the `lanes` slices from the previous batch's
    // first one. Slices outside the pass's filter are staged by filtered passes of `lanes`
    // slices each; a lane holding another slice is flushed to its table first (ingest_pass).
    PendingBatch& pb = h->pending;
    pb.ps = PassState{};
    pb.n = n;
    pb.key = key;
    pb.ts = ts;
    pb.val = val;
    pb.vnull = vnull;
    pb.slot = slot;
    slot_free.slot = -1;   // recorded by finish_batch, after the last kernel reading the slot
    pb.flo = JMIN;
    pb.fhi = JMAX;
    if (h->q_guess != kEmptyLane) {
        pb.flo = h->q_guess;
        pb.fhi = pb.flo + h->lanes;
    }
    int rc = ingest_launch(h, n, key, ts, val, vnull, pb.flo, pb.fhi, true, pb.ps);
    if (rc) {
        if (slot >= 0) (void)hipEventRecord(h->ev_free[slot], h->stream);
        return rc;
    }
    if (pb.ps.spec) {
        // Deferred: pass 2 is queued with the device's lane plan; the host takes the
        // counters at its next call on the handle (settle_pending: ev_pending follows the
        // scan, so it waits for pass 1 only) while the GPU runs pass 2 -- no round trip inside
        // the batch.
        pb.active = true;
        return FG_OK;
    }
    rc = sync(h);
    if (rc) return rc;
    return finish_batch(h);
}

int fg_add_rows(fg_handle* h, const fg_row_batch* b) {
    if (!h || !b) return FG_EINVAL;
    if (b->n <= 0) return FG_OK;
    if (b->n > (int64_t)0x7fffffff) return h->fail(FG_EINVAL, "batch larger than 2^31-1 rows");
    if (!b->rows) return h->fail(FG_EINVAL, "rows pointer is required");
    // BinaryRowData.calculateBitSetWidthInBytes / calculateFixPartSizeInBytes (:70-76)
    const int64_t bits_w = ((int64_t)b->arity + 63 + 8) / 64 * 8;
    const int64_t fixed = bits_w + 8 * (int64_t)b->arity;
    const bool has_val = h->cfg.val_type != FG_VAL_NONE;
    auto field_ok = [&](int32_t f) { return f >= 0 && f < b->arity; };
    if (b->arity < 1 || !field_ok(b->key_field) || !field_ok(b->rowtime_field))
        return h->fail(FG_EINVAL, "row layout: arity %d, key field %d, rowtime field %d", b->arity, b->key_field,
                       b->rowtime_field);
    if (has_val ? !field_ok(b->val_field) : b->val_field != -1)
        return h->fail(FG_EINVAL, "row layout: value field %d (val_type %d)", b->val_field, h->cfg.val_type);
    if (b->stride < fixed || b->stride % 8 != 0)
        return h->fail(FG_EINVAL, "row stride %d: at least the fixed-length part (%lld bytes), a multiple of 8",
                       b->stride, (long long)fixed);
    HIPCHK(h, hipSetDevice(h->device));
    if (int rc0 = settle_pending(h)) return rc0;
    const int64_t n = b->n;
    const uint8_t* rows = b->rows;
    if (b->location == FG_HOST) {
        HIPCHK(h, h->in_rows.ensure((size_t)n * b->stride));
        HIPCHK(h, hipMemcpyAsync(h->in_rows.p, rows, (size_t)n * b->stride, hipMemcpyHostToDevice, h->stream));
        rows = h->in_rows.as<uint8_t>();
    }
    RowLayout L{};
    L.stride = b->stride;
    L.key_off = (int32_t)(bits_w + 8 * b->key_field);
    L.ts_off = (int32_t)(bits_w + 8 * b->rowtime_field);
    L.val_off = has_val ? (int32_t)(bits_w + 8 * b->val_field) : -1;
    L.key_bit = 8 + b->key_field;   // HEADER_SIZE_IN_BITS + field (:155-157)
    L.ts_bit = 8 + b->rowtime_field;
    L.val_bit = has_val ? 8 + b->val_field : 0;
    HIPCHK(h, h->in_key.ensure(8 * (size_t)n));
    HIPCHK(h, h->in_ts.ensure(8 * (size_t)n));
    if (has_val) {
        HIPCHK(h, h->in_val.ensure(8 * (size_t)n));
        HIPCHK(h, h->in_null.ensure((size_t)n));
    }
    unsigned long long* bad = h->row_bad.as<unsigned long long>();
    HIPCHK(h, hipMemsetAsync(bad, 0, 16, h->stream));
    HIPCHK(h, launch_rows_to_columns(rows, n, L, h->in_key.as<int64_t>(), h->in_ts.as<int64_t>(),
                                     has_val ? h->in_val.as<int64_t>() : nullptr,
                                     has_val ? h->in_null.as<uint8_t>() : nullptr, bad, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->h_counters.p, bad, 16, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    unsigned long long cnt[2];
    std::memcpy(cnt, h->h_counters.p, sizeof cnt);
    if (cnt[0]) return h->fail(FG_EINVAL, "%llu rows with a NULL key or rowtime", cnt[0]);
    fg_batch cb{};
    cb.n = n;
    cb.location = FG_DEVICE;
    cb.key = h->in_key.as<int64_t>();
    cb.rowtime = h->in_ts.as<int64_t>();
    cb.val = has_val ? h->in_val.as<int64_t>() : nullptr;
    cb.val_null = has_val && cnt[1] ? h->in_null.as<uint8_t>() : nullptr;   // no NULLs: the plain path
    return fg_add_batch(h, &cb);
}

static int add_partials(fg_handle* h, const fg_partials* b);

int fg_add_partials(fg_handle* h, const fg_partials* b) {
    const int rc = add_partials(h, b);
    // FG_DEVICE columns have been read when the call returns (include/flinkgpu.h): the last
    // pass's scatter reads them after the counters' round trip, so wait for it -- a caller's
    // allocator may hand the columns' blocks to other work on another stream at once
    if (rc == FG_OK && b && b->n > 0 && b->location == FG_DEVICE) HIPCHK(h, hipStreamSynchronize(h->stream));
    return rc;
}

static int add_partials(fg_handle* h, const fg_partials* b) {
    if (h) {
        h->cnt_bound = JMAX;
        h->keys32 = false;
    }
    if (!h || !b) return FG_EINVAL;
    if (b->n <= 0) return FG_OK;
    if (h->local) return h->fail(FG_ESTATE, "fg_add_partials on a FG_FLAG_LOCAL_PARTIALS (local phase) operator");
    if (b->n > (int64_t)0x7fffffff) return h->fail(FG_EINVAL, "batch larger than 2^31-1 rows");
    if (!b->key || !b->slice_end || !b->cnt_star || !b->cnt_val || !b->sum)
        return h->fail(FG_EINVAL, "partials need key, slice_end, cnt_star, cnt_val and sum columns");
    if (h->mv && (!b->min || !b->max))
        return h->fail(FG_EINVAL, "a global operator with several value accumulators (SUM family, MIN, MAX) needs "
                                  "the partial rows' min and max columns");
    HIPCHK(h, hipSetDevice(h->device));
    if (int rc0 = settle_pending(h)) return rc0;
    maybe_reduce_lanes(h);
    const int64_t n = b->n;
    const int64_t *key = b->key, *se = b->slice_end, *cs = b->cnt_star, *cv = b->cnt_val, *sum = b->sum;
    const int64_t *v1 = h->mv ? b->min : nullptr, *v2 = h->mv ? b->max : nullptr;
    if (b->location == FG_HOST) {
        DevBuf* bufs[7] = {&h->in_key, &h->in_slice, &h->in_cs, &h->in_cv, &h->in_sum, &h->in_v1, &h->in_v2};
        const int64_t* src[7] = {key, se, cs, cv, sum, v1, v2};
        for (int i = 0; i < (h->mv ? 7 : 5); i++) {
            HIPCHK(h, bufs[i]->ensure(8 * n));
            HIPCHK(h, hipMemcpyAsync(bufs[i]->p, src[i], 8 * n, hipMemcpyHostToDevice, h->stream));
        }
        key = h->in_key.as<int64_t>();
        se = h->in_slice.as<int64_t>();
        cs = h->in_cs.as<int64_t>();
        cv = h->in_cv.as<int64_t>();
        sum = h->in_sum.as<int64_t>();
        if (h->mv) {
            v1 = h->in_v1.as<int64_t>();
            v2 = h->in_v2.as<int64_t>();
        }
    }
    HIPCHK(h, h->in_ts.ensure(8 * n));
    int64_t* ts = h->in_ts.as<int64_t>();
    // fixed offset: pseudo rowtime slice_end - 1 - tz; zone rules: slice_end - 1 in local
    // time, assigned without the zone shift (WindowSpec::local_input, set in acc_pass)
    HIPCHK(h, launch_pseudo_rowtime(se, n, h->w.tz_n > 0 ? 0 : h->w.tz, ts, h->stream));
    h->records_in += n;
    int rc0 = seed_anchor(h, ts, nullptr);
    if (rc0) return rc0;
    Counters c{};
    int rc = acc_pass(h, n, key, ts, cs, cv, sum, v1, v2, JMIN, JMAX, true, &c);
    h->late_dropped += (int64_t)c.drops;
    if (rc == FG_OK) return FG_OK;
    if (rc != -1) return rc;
    const int64_t qlo = c.qmin, qhi = c.qmax;
    rc = flush(h);
    if (rc) return rc;
    // filtered passes over the occupied slices only (each pass reports the next one)
    for (int64_t lo = qlo; lo <= qhi;) {
        Counters c2{};
        rc = acc_pass(h, n, key, ts, cs, cv, sum, v1, v2, lo, lo + h->lanes, false, &c2);
        if (rc == -1) return h->fail(FG_ESTATE, "internal: slice lanes conflict inside a filtered pass");
        if (rc) return rc;
        lo = c2.qnext;
        if (lo <= qhi) {
            rc = flush(h);
            if (rc) return rc;
        }
    }
    return FG_OK;
}

int fg_flush(fg_handle* h) {
    if (!h) return FG_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    if (int rc0 = settle_pending(h)) return rc0;
    return flush(h);
}

// (static: inside the extern "C" block an exported `advance` is interposed by libc's)
// processWatermark without the output: flushes, re-fires, fires, cleanup timers
static int advance_progress(fg_handle* h, int64_t wm) {
    if (int rc0 = settle_pending(h)) return rc0;
    // rows of async advances not collected yet lead this advance's rows (an async advance appends
    // to them; a synchronous one returns them ahead of its own)
    h->adv_base = h->async_open ? h->out_n : 0;
    h->out_n = h->adv_base + h->late_rows;   // rows fired by late elements since the last advance come first
    h->pending_out = 0;
    h->out_count_reset = false;
    h->fused_fired.clear();
    if (h->late_rows > 0) {
        int rcr = reset_out_count(h);
        if (rcr) return rcr;
    }
    int rc;
    const int64_t prev = h->timer_wm;
    const FireRange fr{prev, wm};
    const FireRange* fuse = wm > prev ? &fr : nullptr;
    if (h->local) {
        // LocalSlicingWindowAggOperator.processWatermark (:113-139): once the watermark fires
        // the smallest buffered slice, the combiner emits partial accumulators; here every
        // fired slice lane emits its partials, and slices flushed earlier to make room are
        // emitted from their tables
        // (fg_flush_partials: prepareSnapshotPreBarrier -> RecordsWindowBuffer.flush, every
        // buffered slice emits its partials now, the local operator keeps no state)
        const bool every = h->local_emit_all;
        if (wm > h->current_progress) h->current_progress = wm;
        if (staged_any(h) && (every || is_window_fired(h->w, min_staged_slice_end(h), wm))) {
            const FireRange all{JMIN, every ? JMAX : wm};
            rc = flush(h, &all, !every);
            if (rc) return rc;
        }
        std::vector<int64_t> ends;
        for (auto& kv : h->tables)
            if (every || is_window_fired(h->w, kv.first, wm)) ends.push_back(kv.first);
        for (int64_t e : ends) {
            rc = fire_one(h, e, {h->tables[e].get()}, nullptr);
            if (rc) return rc;
            table_free(h, e);
        }
    } else if (h->cfg.mode == FG_MODE_SQL) {
        // AbstractWindowAggProcessor.advanceProgress :178-192
        if (wm > h->current_progress) {
            h->arrival_progress = h->current_progress;   // the staged records arrived under it
            h->current_progress = wm;
            if (h->current_progress >= h->next_trigger) {
                if (staged_any(h) && is_window_fired(h->w, min_staged_slice_end(h), wm)) {
                    rc = flush(h, fuse, true);
                    if (rc) return rc;
                }
                h->next_trigger = next_trigger_watermark(h->w, wm, h->w.slice);
            }
        }
    } else {
        // DataStream WindowOperator: records are in state before any timer fires
        if (wm > h->current_progress) h->current_progress = wm;
        if (staged_any(h) && is_window_fired(h->w, min_staged_slice_end(h), wm)) {
            rc = flush(h, fuse, true);
            if (rc) return rc;
        }
    }
    h->arrival_progress = h->current_progress;
    if (h->refire_hi != JMIN && wm > h->refire_wm) {   // restore re-fire (timers below prev)
        rc = refire(h, wm);
        if (rc) return rc;
    }
    if (wm > prev && !h->local) {
        rc = fire_windows(h, prev, wm);
        if (rc) return rc;
    }
    if (wm > h->timer_wm) h->timer_wm = wm;
    if (!h->retire_at.empty()) {   // cleanup timers (WindowOperator.onEventTime :493-496 -> clearAllState)
        for (auto it = h->retire_at.begin(); it != h->retire_at.end();) {
            if (it->second <= h->current_progress) {
                table_free(h, it->first);
                it = h->retire_at.erase(it);
            } else {
                ++it;
            }
        }
    }
    if (h->late_horizon != JMIN && h->current_progress >= h->late_horizon) h->late_horizon = JMIN;
    h->late_rows = 0;
    return FG_OK;
}

// A watermark that can neither flush, fire, re-fire nor free anything (between window ends:
// no window timer in (timer watermark, wm], the staged slices not yet fired): with a
// fire pending, fg_advance_progress_async takes only its progress bookkeeping -- the fire's
// completion is left to the call that needs it, so the host does not wait for the fire here.
// true when a window end on the slice grid may have its timer in (prev, wm]: exact for zones
// without rules (trigger_time(e) = e - 1 - tz, increasing in e), assumed otherwise
static bool trigger_between(const fg_handle* h, int64_t prev, int64_t wm) {
    const WindowSpec& w = h->w;
    if (wm <= prev) return false;
    const int64_t lim = (int64_t)1 << 61;
    if (w.tz_n > 0 || prev < -lim || prev > lim || wm > lim) return true;
    const int64_t q = floor_div(prev + 1 + w.tz - h->slice_phase, w.slice);
    for (int64_t k = q - 1; k <= q + 2; k++) {
        const int64_t t = trigger_time(w, k * w.slice + h->slice_phase);
        if (t > prev) return t <= wm;
    }
    return true;
}

static bool quiet_advance(const fg_handle* h, int64_t wm) {
    if (!h->fire_pending || h->pending.active || h->late_rows > 0 || h->local || h->refire_hi != JMIN ||
        !h->retire_at.empty() || h->lateness > 0)
        return false;
    if (!h->tables.empty()) {   // resident slices: no window may come due, and (TUMBLE) none is overdue
        if (trigger_between(h, h->timer_wm, wm)) return false;
        if (h->w.kind == TUMBLE && trigger_time(h->w, h->tables.begin()->first) <= h->timer_wm) return false;
    }
    if (!staged_any(h)) return true;
    const bool fired = is_window_fired(h->w, min_staged_slice_end(h), wm);
    if (h->cfg.mode == FG_MODE_SQL)   // (advance: flush iff progress moves past the next trigger onto a fired slice)
        return !(wm > h->current_progress && wm >= h->next_trigger && fired);
    return !fired;
}
static void quiet_progress(fg_handle* h, int64_t wm) {   // advance()'s bookkeeping on the quiet path
    if (h->cfg.mode == FG_MODE_SQL) {
        if (wm > h->current_progress) {
            h->current_progress = wm;
            if (h->current_progress >= h->next_trigger) h->next_trigger = next_trigger_watermark(h->w, wm, h->w.slice);
        }
    } else if (wm > h->current_progress) {
        h->current_progress = wm;
    }
    h->arrival_progress = h->current_progress;
    if (wm > h->timer_wm) h->timer_wm = wm;
    if (h->late_horizon != JMIN && h->current_progress >= h->late_horizon) h->late_horizon = JMIN;
}

int fg_advance_progress_async(fg_handle* h, int64_t wm) {
    if (!h) return FG_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    if (quiet_advance(h, wm)) {
        quiet_progress(h, wm);
        return FG_OK;
    }
    if (h->lateness > 0)   // (late elements fire rows at fg_add_batch, ahead of any advance's)
        return h->fail(FG_EINVAL, "fg_advance_progress_async: allowed lateness needs fg_advance_progress");
    h->async_advance = true;
    const int rc = advance_progress(h, wm);
    h->async_advance = false;
    if (rc) return rc;
    h->async_open = true;
    if (h->fire_pending) {   // rows_fired at completion
        h->fire_rows_open = true;
        h->fire_rows_base = h->adv_base;
    } else {
        h->rows_fired += h->out_n - h->adv_base;
    }
    return FG_OK;
}

int fg_advance_progress_async_n(fg_handle* h, const int64_t* wms, int64_t n) {
    if (!h || n < 0 || (n > 0 && !wms)) return FG_EINVAL;
    for (int64_t i = 0; i < n; i++)
        if (int rc = fg_advance_progress_async(h, wms[i])) return rc;
    return FG_OK;
}

static void device_rows(fg_handle* h, int32_t out_location, fg_rows* fired) {
    std::memset(fired, 0, sizeof *fired);
    fired->n = h->out_n;
    fired->num_aggs = h->cfg.num_aggs;
    fired->location = out_location;
    fired->key = h->o_key.as<int64_t>();
    fired->window_start = h->o_ws.as<int64_t>();
    fired->window_end = h->o_we.as<int64_t>();
    fired->null_mask = h->o_null.as<uint8_t>();
    fired->rowtime = h->cfg.mode == FG_MODE_DATASTREAM ? h->o_rt.as<int64_t>() : nullptr;
    for (int a = 0; a < h->cfg.num_aggs; a++) fired->agg[a] = h->o_agg[a].as<int64_t>();
}

int fg_collect_fired_to(fg_handle* h, int32_t out_location, fg_rows* fired) {
    if (!h || !fired || (out_location != FG_HOST && out_location != FG_DEVICE)) return FG_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    if (int rc = complete_fire(h)) return rc;
    if (!h->async_open) h->out_n = 0;   // (every async advance since the last collect fired nothing)
    h->async_open = false;
    if (out_location == FG_HOST) {
        std::memset(fired, 0, sizeof *fired);
        fired->n = h->out_n;
        fired->num_aggs = h->cfg.num_aggs;
        fired->location = FG_HOST;
        return copy_out_to_host(h, fired);
    }
    device_rows(h, FG_DEVICE, fired);
    return FG_OK;
}

int fg_collect_fired(fg_handle* h, fg_rows* fired) { return fg_collect_fired_to(h, FG_DEVICE, fired); }

int fg_flush_partials(fg_handle* h, int32_t out_location, fg_rows* fired) {
    if (!h || !fired || (out_location != FG_HOST && out_location != FG_DEVICE)) return FG_EINVAL;
    if (!h->local) return h->fail(FG_ESTATE, "fg_flush_partials on an operator without FG_FLAG_LOCAL_PARTIALS");
    HIPCHK(h, hipSetDevice(h->device));
    h->local_emit_all = true;
    const int rc = advance_progress(h, h->current_progress);   // (the progress does not move)
    h->local_emit_all = false;
    if (rc) return rc;
    h->rows_fired += h->out_n - h->adv_base;
    h->async_open = false;
    std::memset(fired, 0, sizeof *fired);
    fired->n = h->out_n;
    fired->num_aggs = h->cfg.num_aggs;
    fired->location = out_location;
    if (out_location == FG_HOST) return copy_out_to_host(h, fired);
    device_rows(h, out_location, fired);
    return FG_OK;
}

int fg_advance_progress(fg_handle* h, int64_t wm, int32_t out_location, fg_rows* fired) {
    if (!h) return FG_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    int rc = advance_progress(h, wm);   // (uncollected async rows lead its rows: adv_base)
    if (rc) return rc;
    h->rows_fired += h->out_n - h->adv_base;   // (the async rows were counted by their advances)
    h->async_open = false;
    if (fired) {
        std::memset(fired, 0, sizeof *fired);
        fired->n = h->out_n;
        fired->num_aggs = h->cfg.num_aggs;
        fired->location = out_location;
        if (out_location == FG_HOST) {
            rc = copy_out_to_host(h, fired);
            if (rc) return rc;
        } else {
            device_rows(h, out_location, fired);
        }
    }
    return FG_OK;
}

// snapshotState's synchronous part: the staged records flushed, every resident slice exported
// into the device image columns (s_*, in stream order: the image is the state as of this call)
// and their copy into the pinned host image (hs_*) queued on the snapshot stream
static int snapshot_begin(fg_handle* h) {
    if (int rc0 = settle_pending(h)) return rc0;
    int rc = flush(h);
    if (rc) return rc;
    // a restore re-fire still pending: its new state joins the image (the chained timers
    // of its keys are not part of it)
    if (h->refire_hi != JMIN) {
        rc = refire_finish(h);
        if (rc) return rc;
    }
    // region counts of every resident slice
    const size_t nt = h->tables.size();
    HIPCHK(h, h->hs_counts.ensure(sizeof(uint32_t) * h->P * std::max<size_t>(nt, 1)));
    size_t ti = 0;
    for (auto& kv : h->tables) {
        HIPCHK(h, hipMemcpyAsync(h->hs_counts.as<uint32_t>() + ti * h->P, kv.second->counts.p, 4 * h->P,
                                 hipMemcpyDeviceToHost, h->stream));
        ti++;
    }
    rc = sync(h);
    if (rc) return rc;
    int64_t total = 0;
    HIPCHK(h, h->hs_off.ensure(sizeof(uint64_t) * h->P * std::max<size_t>(nt, 1)));
    for (size_t t = 0; t < nt; t++) {
        for (int r = 0; r < h->P; r++) {
            h->hs_off.as<uint64_t>()[t * h->P + r] = (uint64_t)total;
            total += h->hs_counts.as<uint32_t>()[t * h->P + r];
        }
    }
    // the image's slices: its rows are grouped by slice, in the tables' (ascending) order
    h->img_ready = false;
    h->img_se.clear();
    h->img_first.clear();
    h->img_rows.clear();
    h->img_changed.clear();
    {
        size_t t = 0;
        for (auto& kv : h->tables) {
            const int64_t first = (int64_t)h->hs_off.as<uint64_t>()[t * h->P];
            const int64_t next = t + 1 < nt ? (int64_t)h->hs_off.as<uint64_t>()[(t + 1) * h->P] : total;
            h->img_se.push_back(kv.first);
            h->img_first.push_back(first);
            h->img_rows.push_back(next - first);
            h->img_changed.push_back(kv.second->changed ? 1 : 0);
            kv.second->changed = false;
            t++;
        }
    }
    const size_t b8 = 8 * (size_t)std::max<int64_t>(total, 1);
    HIPCHK(h, h->s_key.ensure(b8));
    HIPCHK(h, h->s_slice.ensure(b8));
    HIPCHK(h, h->s_cs.ensure(b8));
    HIPCHK(h, h->s_cv.ensure(b8));
    HIPCHK(h, h->s_sum.ensure(b8));
    if (h->mv) {
        HIPCHK(h, h->s_v1.ensure(b8));
        HIPCHK(h, h->s_v2.ensure(b8));
    }
    HIPCHK(h, h->s_off.ensure(sizeof(uint64_t) * h->P * std::max<size_t>(nt, 1)));
    HIPCHK(h, hipMemcpyAsync(h->s_off.p, h->hs_off.p, sizeof(uint64_t) * h->P * nt, hipMemcpyHostToDevice, h->stream));
    ti = 0;
    for (auto& kv : h->tables) {
        ExportParams p{};
        p.t = ref_of(kv.second.get());
        p.region_off = h->s_off.as<uint64_t>() + ti * h->P;
        p.slice_end = kv.first;
        p.out_key = h->s_key.as<int64_t>();
        p.out_slice = h->s_slice.as<int64_t>();
        p.out_cnt_star = h->s_cs.as<int64_t>();
        p.out_cnt_val = h->s_cv.as<int64_t>();
        p.out_sum = h->s_sum.as<int64_t>();
        p.mv = h->mv;
        p.out_v1 = h->s_v1.as<int64_t>();
        p.out_v2 = h->s_v2.as<int64_t>();
        {
            KTimer kt(h, K_EXPORT, 0);
            HIPCHK(h, launch_export(p, h->P, h->stream));
        }
        ti++;
    }
    HIPCHK(h, h->hs_key.ensure(b8));
    HIPCHK(h, h->hs_slice.ensure(b8));
    HIPCHK(h, h->hs_cs.ensure(b8));
    HIPCHK(h, h->hs_cv.ensure(b8));
    HIPCHK(h, h->hs_sum.ensure(b8));
    if (h->mv) {
        HIPCHK(h, h->hs_v1.ensure(b8));
        HIPCHK(h, h->hs_v2.ensure(b8));
    }
    if (total > 0) {
        if (!h->snap_stream) {
            // (the runtime copies device -> host with blit kernels that share the CUs with a
            // concurrent fire or pass 1; restricting the copy's stream to 8-64 CUs kept the kernels'
            // speed but slowed the copy more than it saved, round 5: profiles/r05/zipf_ab/snap_cus)
            HIPCHK(h, hipStreamCreateWithFlags(&h->snap_stream, hipStreamNonBlocking));
            HIPCHK(h, hipEventCreateWithFlags(&h->ev_snap, hipEventDisableTiming));
        }
        HIPCHK(h, hipEventRecord(h->ev_snap, h->stream));   // (after the export kernels)
        HIPCHK(h, hipStreamWaitEvent(h->snap_stream, h->ev_snap, 0));
        hipStream_t cs = h->snap_stream;
        const hipMemcpyKind kd = hipMemcpyDeviceToHost;
        if (h->mv) {
            HIPCHK(h, hipMemcpyAsync(h->hs_v1.p, h->s_v1.p, 8 * total, kd, cs));
            HIPCHK(h, hipMemcpyAsync(h->hs_v2.p, h->s_v2.p, 8 * total, kd, cs));
        }
        HIPCHK(h, hipMemcpyAsync(h->hs_key.p, h->s_key.p, 8 * total, kd, cs));
        HIPCHK(h, hipMemcpyAsync(h->hs_slice.p, h->s_slice.p, 8 * total, kd, cs));
        HIPCHK(h, hipMemcpyAsync(h->hs_cs.p, h->s_cs.p, 8 * total, kd, cs));
        // no table counts NULL values: COUNT(v) = COUNT(*) for every entry, and the image's
        // cnt_val column is its cnt_star column (a fifth less to copy while the job runs on)
        bool any_null = false;
        for (auto& kv : h->tables) any_null = any_null || kv.second->has_null;
        h->snap_cv_alias = !any_null;
        if (any_null) HIPCHK(h, hipMemcpyAsync(h->hs_cv.p, h->s_cv.p, 8 * total, kd, cs));
        HIPCHK(h, hipMemcpyAsync(h->hs_sum.p, h->s_sum.p, 8 * total, kd, cs));
    }
    h->snap_pending = true;
    h->snap_total = total;
    h->snap_wm = h->timer_wm;
    return FG_OK;
}

// snapshotState's asynchronous part: the host image once its copy has completed
static int snapshot_end(fg_handle* h, fg_state_rows* out, int64_t* timer_watermark) {
    if (!h->snap_pending) return h->fail(FG_ESTATE, "fg_snapshot_state_wait without fg_snapshot_state_async");
    if (h->snap_stream) HIPCHK(h, hipStreamSynchronize(h->snap_stream));
    h->snap_pending = false;
    const int64_t total = h->snap_total;
    out->n = total;
    out->key = h->hs_key.as<int64_t>();
    out->slice_end = h->hs_slice.as<int64_t>();
    out->cnt_star = h->hs_cs.as<int64_t>();
    out->cnt_val = h->snap_cv_alias ? h->hs_cs.as<int64_t>() : h->hs_cv.as<int64_t>();
    out->sum = h->hs_sum.as<int64_t>();
    out->min = h->mv ? h->hs_v1.as<int64_t>() : nullptr;   // multi-value operators: the MIN / MAX slots
    out->max = h->mv ? h->hs_v2.as<int64_t>() : nullptr;
    if (timer_watermark) *timer_watermark = h->snap_wm;
    h->img_ready = true;
    return FG_OK;
}

int fg_snapshot_slices(fg_handle* h, fg_image_slices* out) {
    if (!h || !out) return FG_EINVAL;
    if (!h->img_ready) return h->fail(FG_ESTATE, "fg_snapshot_slices: no image returned since the last snapshot call");
    out->n = (int64_t)h->img_se.size();
    out->slice_end = h->img_se.data();
    out->first_row = h->img_first.data();
    out->rows = h->img_rows.data();
    out->changed = h->img_changed.data();
    return FG_OK;
}

int fg_snapshot_state_async(fg_handle* h) {
    if (!h) return FG_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    if (h->snap_pending) return h->fail(FG_ESTATE, "an asynchronous snapshot is not collected yet (fg_snapshot_state_wait)");
    return snapshot_begin(h);
}

int fg_snapshot_state_wait(fg_handle* h, fg_state_rows* out, int64_t* timer_watermark) {
    if (!h || !out) return FG_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    return snapshot_end(h, out, timer_watermark);
}

int fg_snapshot_state(fg_handle* h, fg_state_rows* out, int64_t* timer_watermark) {
    if (!h || !out) return FG_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    if (h->snap_pending) return h->fail(FG_ESTATE, "an asynchronous snapshot is not collected yet (fg_snapshot_state_wait)");
    if (int rc = snapshot_begin(h)) return rc;
    return snapshot_end(h, out, timer_watermark);
}

int fg_restore(fg_handle* h, const fg_state_rows* in, int64_t timer_watermark) {
    if (!h || !in) return FG_EINVAL;
    const bool was_empty = h->tables.empty();   // (restored into a new handle: its tables equal the image)
    h->cnt_bound = JMAX;
    h->keys32 = false;
    HIPCHK(h, hipSetDevice(h->device));
    if (int rc0 = settle_pending(h)) return rc0;
    int rc = flush(h);
    if (rc) return rc;
    // group entries by slice, bucket by region on the host (restore is off the hot path)
    std::map<int64_t, std::vector<int64_t>> by_slice;
    for (int64_t i = 0; i < in->n; i++) by_slice[in->slice_end[i]].push_back(i);
    // regions sized for the image first: the smallest split whose fullest region keeps the
    // LDS tables at most ~70 % full (a slice restored into a live table may still split more)
    {
        int need = h->region_bits;
        for (auto& kv : by_slice) {
            std::vector<uint32_t> c13((size_t)1 << kMaxRegionBits, 0);
            for (int64_t i : kv.second) c13[fmix64((uint64_t)in->key[i]) >> (64 - kMaxRegionBits)]++;
            for (int b = need; b <= kMaxRegionBits; b++) {
                uint32_t mx = 0;
                const int per = 1 << (kMaxRegionBits - b);
                for (size_t r = 0; r < c13.size(); r += (size_t)per) {
                    uint32_t sum = 0;
                    for (int c = 0; c < per; c++) sum += c13[r + (size_t)c];
                    mx = std::max(mx, sum);
                }
                need = b;
                if (mx <= (uint32_t)(0.7 * h->tcap)) break;
            }
        }
        rc = grow(h, need);
        if (rc) return rc;
    }
    for (auto& kv : by_slice) {
        const auto& idx = kv.second;
        const int64_t m = (int64_t)idx.size();
        const int NB = 1 << h->region_bits;
        std::vector<uint32_t> off(NB + 1, 0);
        std::vector<uint32_t> reg(m);
        for (int64_t j = 0; j < m; j++) {
            const uint64_t hk = fmix64((uint64_t)in->key[idx[j]]);
            reg[j] = h->region_bits == 0 ? 0u : (uint32_t)(hk >> (64 - h->region_bits));
            off[reg[j] + 1]++;
        }
        for (int r = 0; r < NB; r++) off[r + 1] += off[r];
        if (h->mv && (!in->min || !in->max))
            return h->fail(FG_EINVAL, "a multi-value operator's image needs the min and max columns");
        std::vector<int64_t> k(m), cs(m), cn(m), sm(m), v1(h->mv ? m : 0), v2(h->mv ? m : 0);
        std::vector<uint32_t> cur(off.begin(), off.end() - 1);
        for (int64_t j = 0; j < m; j++) {
            const int64_t i = idx[j];
            const uint32_t at = cur[reg[j]]++;
            k[at] = mix_of(in->key[i]);   // state keeps the key's mix (fg_window.h)
            cs[at] = in->cnt_star[i];
            cn[at] = in->cnt_star[i] - in->cnt_val[i];
            sm[at] = in->sum[i];
            if (h->mv) {
                v1[at] = in->min[i];
                v2[at] = in->max[i];
            }
        }
        DevBuf dk, dcs, dcn, dsm, doff, dv1, dv2;
        if (h->mv) {
            HIPCHK(h, dv1.ensure(8 * std::max<int64_t>(m, 1)));
            HIPCHK(h, dv2.ensure(8 * std::max<int64_t>(m, 1)));
            HIPCHK(h, hipMemcpy(dv1.p, v1.data(), 8 * m, hipMemcpyHostToDevice));
            HIPCHK(h, hipMemcpy(dv2.p, v2.data(), 8 * m, hipMemcpyHostToDevice));
        }
        HIPCHK(h, dk.ensure(8 * std::max<int64_t>(m, 1)));
        HIPCHK(h, dcs.ensure(8 * std::max<int64_t>(m, 1)));
        HIPCHK(h, dcn.ensure(8 * std::max<int64_t>(m, 1)));
        HIPCHK(h, dsm.ensure(8 * std::max<int64_t>(m, 1)));
        HIPCHK(h, doff.ensure(4 * (NB + 1)));
        HIPCHK(h, hipMemcpy(dk.p, k.data(), 8 * m, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(dcs.p, cs.data(), 8 * m, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(dcn.p, cn.data(), 8 * m, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(dsm.p, sm.data(), 8 * m, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(doff.p, off.data(), 4 * (NB + 1), hipMemcpyHostToDevice));
        SliceTable* t = nullptr;
        rc = table_get(h, kv.first, true, &t);
        if (rc) return rc;
        MergeJob j;
        JobBatch jb;
        jb.ext.rec = dk.as<int64_t>();
        jb.ext.stride = 1;
        jb.ext.val = dsm.as<int64_t>();
        jb.ext.cnt_star = dcs.as<int64_t>();
        jb.ext.cnt_null = dcn.as<int64_t>();
        jb.ext.bucket_off = doff.as<uint32_t>();
        jb.ext.is_acc = 1;
        jb.ext.val1 = dv1.as<int64_t>();
        jb.ext.val2 = dv2.as<int64_t>();
        jb.ext_bits = h->region_bits;
        j.batches.push_back(jb);
        j.srcs.push_back(t);
        j.dst = t;
        j.kclass = K_RESTORE;
        if (int rc0 = zero_scalars(h, true)) return rc0;
        int ji = 0;
        rc = job_add(h, std::move(j), &ji);
        if (rc) return rc;
        MergeParams p{};
        rc = job_params(h, ji, &p);
        if (rc) return rc;
        {
            KTimer kt(h, K_RESTORE, m);
            HIPCHK(h, launch_merge(p, merge_grid(h), h->stream));
        }
        HIPCHK(h, hipMemcpyAsync(h->h_scalars.p, h->scalars.p, kScalarBytes, hipMemcpyDeviceToHost, h->stream));
        rc = sync(h);
        if (rc) return rc;
        rc = settle_jobs(h);   // the device buffers above stay alive until this returns
        if (rc) return rc;
        rc = check_overflow(h);
        if (rc) return rc;
        t->upper = std::min<int64_t>(t->upper + m, kStateCapMax);
        t->changed = true;
    }
    // open(): processor progress restarts at Long.MIN_VALUE, and so does the restored timer
    // service's watermark (InternalTimerServiceImpl.currentWatermark is not part of the
    // snapshot): a record older than the checkpoint's watermark is not late, its flush
    // registers a timer (AggCombiner step 5 checks isWindowFired against the timer
    // watermark) and the window fires again on the next watermark.
    // Unshared slices (TUMBLE, windowed inputs): every restored (key, slice) entry holds a
    // pending timer (a fired slice is cleared), so firing every window with state whose
    // trigger is <= the watermark is exactly the timers that fire -- the timer watermark
    // restarts at Long.MIN_VALUE here too.
    // Shared slices (HOP, CUMULATE, DataStream sliding): restored slices may also belong to
    // windows that fired before the checkpoint, for keys without pending timers, so the
    // checkpoint's timer watermark is kept (divergence 2).
    h->current_progress = JMIN;
    h->arrival_progress = JMIN;
    h->next_trigger = JMIN;
    h->timer_wm = h->w.kind == TUMBLE ? JMIN : timer_watermark;
    // shared slices: windows at or below the checkpoint's watermark re-fire for the keys of
    // records that arrive for them (refire)
    h->refire_hi = h->w.kind != TUMBLE && !h->local && !h->proctime ? timer_watermark : JMIN;
    h->refire_wm = JMIN;
    if (h->lateness > 0) {
        // allowed lateness: windows that fired before the checkpoint keep only their cleanup
        // timers (WindowOperator.onEventTime fired their trigger timers); their slices stay
        // resident until then and fire again only for elements that reach them (the late path,
        // against the checkpoint's watermark until the watermark passes it)
        h->late_horizon = timer_watermark;
        const int64_t nwin = h->w.kind == TUMBLE ? 1 : h->w.size / h->w.slide;
        for (auto& kv : h->tables) {
            const int64_t last = jadd(kv.first, (nwin - 1) * h->w.slide);
            if (ds_fired(last, timer_watermark)) h->retire_at[kv.first] = ds_cleanup(last, h->lateness);
        }
    }
    // the keyed state backend holds exactly this image: a restored table is not "changed" until a
    // write reaches it (the shim's next checkpoint rewrites only the slices that change)
    if (was_empty)
        for (auto& kv : h->tables) kv.second->changed = false;
    return FG_OK;
}

int fg_late_dropped(fg_handle* h, int64_t* out) {
    if (!h || !out) return FG_EINVAL;
    if (int rc0 = settle_pending(h)) return rc0;
    *out = h->late_dropped;
    return FG_OK;
}

int fg_get_stats(fg_handle* h, fg_stats* out) {
    if (!h || !out) return FG_EINVAL;
    if (int rc0 = settle_pending(h)) return rc0;
    out->records_in = h->records_in;
    out->records_staged = staged_records(h);
    out->late_dropped = h->late_dropped;
    out->rows_fired = h->rows_fired;
    out->flushes = h->flushes;
    out->live_slices = (int64_t)h->tables.size();
    out->state_regions = h->P;
    out->region_capacity = h->tcap;
    return FG_OK;
}

int fg_synchronize(fg_handle* h) {
    if (!h) return FG_EINVAL;
    if (int rc0 = settle_pending(h)) return rc0;
    return sync(h, true);
}

int fg_reset(fg_handle* h) {
    if (!h) return FG_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    if (int rc0 = settle_pending(h)) return rc0;
    int rc = sync(h);
    if (rc) return rc;
    std::vector<int64_t> ends;
    for (auto& kv : h->tables) ends.push_back(kv.first);
    for (int64_t e : ends) table_free(h, e);
    for (int l = 0; l < h->lanes; l++) release_lane(h, l);
    h->anchor_start = JMIN;
    h->q_guess = kEmptyLane;
    h->cnt_bound = 0;
    h->keys32 = true;
    h->skew_seen = false;
    h->current_progress = JMIN;
    h->arrival_progress = JMIN;
    h->next_trigger = JMIN;
    h->timer_wm = JMIN;
    h->late_dropped = 0;
    h->out_n = 0;
    h->pending_out = 0;
    h->async_open = false;
    h->re_new.clear();
    h->re_delta.clear();
    h->re_tmp.clear();
    h->re_chain.reset();
    h->re_chain_w = JMIN;
    h->refire_hi = JMIN;
    h->refire_wm = JMIN;
    h->retire_at.clear();
    h->late_rows = 0;
    h->late_horizon = JMIN;
    h->narrow = h->narrow_ok;
    h->tile_ok = true;
    return FG_OK;
}

int fg_kernel_stats(fg_handle* h, fg_kernel_stat* out, int32_t max, int32_t* count) {
    if (!h || !count) return FG_EINVAL;
    if (int rc0 = settle_pending(h)) return rc0;
    int rc = sync(h, true);
    if (rc) return rc;
    *count = K_NCLASS;
    for (int c = 0; c < K_NCLASS && c < max; c++) {
        std::memset(&out[c], 0, sizeof(fg_kernel_stat));
        std::snprintf(out[c].name, sizeof out[c].name, "%s", kClassName[c]);
        out[c].launches = h->kstat[c].launches;
        out[c].total_ms = h->kstat[c].ms;
        out[c].records = h->kstat[c].records;
        out[c].rows = h->kstat[c].rows;
    }
    return FG_OK;
}

int fg_set_kernel_timing(fg_handle* h, uint32_t class_mask) {
    if (!h) return FG_EINVAL;
    h->timing_mask = class_mask;
    return FG_OK;
}

void* fg_stream(fg_handle* h) { return h ? (void*)h->stream : nullptr; }

const char* fg_last_error(fg_handle* h) { return h ? h->err.c_str() : g_open_error.c_str(); }

void fg_close(fg_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipStreamSynchronize(h->stream);
    {
        // release device memory before the stream
        h->tables.clear();
        h->table_pool.clear();
        for (int l = 0; l < kMaxLanes; l++) h->lane[l] = Lane{};
        h->passes.clear();
        h->pass_pool.clear();
    }
    for (auto& p : h->pend) {
        h->ev_pool.push_back(p.a);
        h->ev_pool.push_back(p.b);
    }
    for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
    if (h->ev_pending) (void)hipEventDestroy(h->ev_pending);
    for (int i = 0; i < 2; i++) {
        if (h->ev_copied[i]) (void)hipEventDestroy(h->ev_copied[i]);
        if (h->ev_free[i]) (void)hipEventDestroy(h->ev_free[i]);
    }
    if (h->copy_stream) {
        (void)hipStreamSynchronize(h->copy_stream);
        (void)hipStreamDestroy(h->copy_stream);
    }
    if (h->snap_stream) {
        (void)hipStreamSynchronize(h->snap_stream);
        (void)hipStreamDestroy(h->snap_stream);
    }
    if (h->ev_snap) (void)hipEventDestroy(h->ev_snap);
    hipStream_t s = h->stream;
    delete h;
    if (s) (void)hipStreamDestroy(s);
}

int fg_key_groups(int32_t device_id, int32_t location, int64_t n, const int64_t* key, int32_t key_hash,
                  int32_t max_parallelism, int32_t* out_kg) {
    if (n <= 0) return FG_OK;
    if (!key || !out_kg || max_parallelism <= 0) return FG_EINVAL;
    if (hipSetDevice(device_id) != hipSuccess) return FG_EDEVICE;
    if (location == FG_DEVICE) {
        if (launch_key_groups(key, n, key_hash, max_parallelism, out_kg, nullptr) != hipSuccess) return FG_EDEVICE;
        return hipDeviceSynchronize() == hipSuccess ? FG_OK : FG_EDEVICE;
    }
    int64_t* dk = nullptr;
    int32_t* dout = nullptr;
    if (hipMalloc(&dk, 8 * n) != hipSuccess) return FG_EDEVICE;
    if (hipMalloc(&dout, 4 * n) != hipSuccess) {
        (void)hipFree(dk);
        return FG_EDEVICE;
    }
    int rc = FG_OK;
    if (hipMemcpy(dk, key, 8 * n, hipMemcpyHostToDevice) != hipSuccess ||
        launch_key_groups(dk, n, key_hash, max_parallelism, dout, nullptr) != hipSuccess ||
        hipMemcpy(out_kg, dout, 4 * n, hipMemcpyDeviceToHost) != hipSuccess)
        rc = FG_EDEVICE;
    (void)hipFree(dk);
    (void)hipFree(dout);
    return rc;
}

int fg_partition_columns_by_owner(int32_t device_id, void* stream, int64_t n, int32_t ncols, const int64_t* const* cols,
                                  int32_t key_hash, int32_t max_parallelism, int32_t parallelism, int64_t* const* out_cols,
                                  int64_t* counts) {
    if (n < 0 || n > (int64_t)0x7fffffff || parallelism < 1 || max_parallelism < parallelism || ncols < 1 ||
        ncols > kMaxOwnerCols || !cols || !out_cols || !counts)
        return FG_EINVAL;
    if (hipSetDevice(device_id) != hipSuccess) return FG_EDEVICE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    OwnerCols c{};
    c.ncols = ncols;
    for (int j = 0; j < ncols; j++) {
        c.in[j] = cols[j];
        c.out[j] = out_cols[j];
    }
    const size_t words = partition_scratch_words(n, parallelism);
    uint32_t* scratch = nullptr;
    if (hipMallocAsync((void**)&scratch, 4 * words, s) != hipSuccess) return FG_EDEVICE;
    hipError_t e = launch_partition_cols_by_owner(c, n, key_hash, max_parallelism, parallelism, counts, scratch, words, s);
    (void)hipFreeAsync(scratch, s);
    if (e != hipSuccess) return FG_EDEVICE;
    return hipStreamSynchronize(s) == hipSuccess ? FG_OK : FG_EDEVICE;
}

int fg_partition_by_owner(int32_t device_id, void* stream, int64_t n, const int64_t* key, const int64_t* rowtime,
                          const int64_t* val, int32_t key_hash, int32_t max_parallelism, int32_t parallelism,
                          int64_t* out_key, int64_t* out_rowtime, int64_t* out_val, int64_t* counts) {
    if (n < 0 || n > (int64_t)0x7fffffff || parallelism < 1 || max_parallelism < parallelism) return FG_EINVAL;
    if (hipSetDevice(device_id) != hipSuccess) return FG_EDEVICE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t words = partition_scratch_words(n, parallelism);
    uint32_t* scratch = nullptr;
    if (hipMallocAsync((void**)&scratch, 4 * words, s) != hipSuccess) return FG_EDEVICE;
    hipError_t e = launch_partition_by_owner(key, rowtime, val, n, key_hash, max_parallelism, parallelism, out_key,
                                             out_rowtime, out_val, counts, scratch, words, s);
    (void)hipFreeAsync(scratch, s);
    if (e != hipSuccess) return FG_EDEVICE;
    return hipStreamSynchronize(s) == hipSuccess ? FG_OK : FG_EDEVICE;
}

}  // extern "C"
