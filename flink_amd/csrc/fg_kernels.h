// fg_kernels.h -- launch interface of the gfx950 kernels (internal to libflinkgpu.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <hip/hip_ext.h>

#include "fg_window.h"

namespace fg {

// Kernel timing (FG_FLAG_KERNEL_TIMING): the engine's KTimer arms these events and the next
// launches on this thread carry them in their own dispatch packets (hipExtLaunchKernel) --
// the first launch of the bracketed call records `start`, every launch `stop` (the last one
// wins). Separate hipEventRecord markers each cost a queue round of 6-20 us between kernels.
struct LaunchEvents {
    hipEvent_t start = nullptr;
    hipEvent_t stop = nullptr;
};
extern thread_local LaunchEvents g_launch_ev;
template <class K, class... A>
inline void fg_launch(K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t s, A... a) {
    if (g_launch_ev.stop) {
        hipExtLaunchKernelGGL(kernel, grid, block, lds, s, g_launch_ev.start, g_launch_ev.stop, 0u, a...);
        g_launch_ev.start = nullptr;
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, s, a...);
    }
}

// LDS hash table of one state region: kSlots open-addressing slots + 1 slot reserved
// for the key that equals the EMPTY sentinel (Long.MIN_VALUE).
constexpr int kSlotBits = 12;
constexpr int kSlots = 1 << kSlotBits;        // 4096 slots x 32 B = 128 KiB of LDS
constexpr int kRegionCap = 3584;              // max entries per region in HBM (87.5 % of kSlots)
constexpr int kMergeThreads = 1024;           // persistent merge: one 1024-thread workgroup per CU
constexpr int kCompactSlots = 3584;           // compact merge table: 3,584 x 20 B = 70 KiB of LDS
#ifndef FG_COMPACT_T
#define FG_COMPACT_T 512
#endif
constexpr int kCompactMergeThreads = FG_COMPACT_T;   // compact merge: two 512-thread workgroups per CU
// Several value accumulators over the one value column (SUM family + MIN + MAX in one
// operator, the reference's generated accumulator row, AggsHandlerCodeGenerator.scala:578-700):
// three value slots per entry, so the LDS tables hold fewer slots and regions fewer entries
constexpr int kNV = 3;                        // value slots per entry of a multi-value operator
constexpr int kSlotsMV = 3072;                // wide LDS table: 3,072 x 48 B = 144 KiB
constexpr int kCompactSlotsMV = 3072;         // compact LDS table: 3,072 x 36 B = 108 KiB
constexpr int kRegionCapMV = 2688;            // entries per region in HBM (87.5 % of kSlotsMV)
constexpr int kIngestThreads = 1024;
constexpr int kMaxLanes = 4;
constexpr int kMaxStageBuckets = 32768;       // lanes << region_bits (count / direct scatter LDS)
constexpr int kMaxSortedBuckets = 8192;       // lane slots << region_bits (tile-sorted scatter LDS)
constexpr int kTile = 8192;                   // records per sorted-scatter tile (8 per thread)
constexpr int kMaxAggs = 8;
// two-pass partition (regions >= 64): pass 1 sorts tiles by coarse bucket (= fine >> 6)
// into a tile-private buffer, pass 2 sorts each (coarse bucket, workgroup) unit by fine
// bucket into the staged areas
constexpr int kFineBits = 6;                  // fine buckets per coarse bucket = 64
#ifndef FG_P1_T
#define FG_P1_T 768
#endif
#ifndef FG_P1_R
#define FG_P1_R 6
#endif
constexpr int kPart1Threads = FG_P1_T;        // one workgroup per CU (LDS: fine histogram + tile)
constexpr int kPart1Tile = FG_P1_R * kPart1Threads;   // pass-1 records per tile (FG_P1_R per thread, one LDS round)
constexpr int kMaxPart1Fine = 16384;          // lanes << region_bits for the two-pass path
constexpr int kMaxCoarse = kMaxPart1Fine >> kFineBits;   // 256
#ifndef FG_P2_T
#define FG_P2_T 512
#endif
constexpr int kPart2Threads = FG_P2_T;
constexpr int kPart2Tile = 8 * kPart2Threads;  // pass-2 records per sub-tile (8 per thread)

// One slice table in HBM: P regions, each region an SoA block of kRegionCap entries:
//   [key i64 x cap][cnt_star i64 x cap][cnt_null i64 x cap][sum (i64 | f64 bits) x cap]
// cnt_val = cnt_star - cnt_null. A multi-value operator's regions hold kRegionCapMV entries
// and kNV value columns: [key][cnt_star][cnt_null][v0][v1][v2].
// A narrow table (round 5: `narrow`, keys32 operators without NULL counts, one value slot, COUNT(*)
// below 2^32) keeps 16 B per entry in the first half of each region's block: [int32 key][u32
// cnt_star][value] (cap 4-B keys, cap 4-B counts, then cap 8-B values; the region stride stays
// the wide one). Its readers recompute the key's mix.
struct TableRef {
    int64_t* base;
    uint32_t* counts;   // entries per region
    int32_t narrow;
    int32_t pad;
};


// One staged batch of one slice lane. The records of region r are
//   rec[bucket_off[r] - bucket_off[0] .. bucket_off[r + 1] - bucket_off[0])
// (bucket_off points at the batch's lane slice of its [lanes * P + 1] bucket scan).
// Records are AoS {key, value bits} (stride 2) or {key} (stride 1, COUNT(*)-only).
// Restore images (is_acc) are SoA accumulators: rec = keys, val / cnt_star / cnt_null.
struct StagedBatch {
    const int64_t* rec;
    const int64_t* val;        // is_acc only: the `sum` accumulator
    const uint8_t* vnull;      // NULL flags aligned with rec (may be null)
    const int64_t* cnt_star;   // is_acc only
    const int64_t* cnt_null;   // is_acc only
    const uint32_t* bucket_off;
    int32_t is_acc;
    int32_t stride;            // int64 words per record (1 or 2); 3: narrow 12-B records {int32 key,
                               // value bits} in 64-record blocks (rec: the staged area's base; the
                               // batch's records are rec_first, rec_first + 1, ...)
    // regions split since the batch was staged (MergeParams.region_bits - the batch's bits):
    // region r's records are those of bucket r >> shift whose key mix lies in region r
    // (general merge path only)
    int32_t shift;
    int32_t rec_first;         // stride 3: block index of the batch's first record
    const int64_t* val1;       // is_acc of a multi-value operator: value slots 1 and 2
    const int64_t* val2;
};

// Narrow staged record: {int32 key, value bits} in 12 bytes (4-B aligned). The state keeps a
// key as its fmix64 mix (fg_window.h), recomputed from the 32-bit key by its readers.
constexpr int kRec12Block = 64 * 12;   // 64 narrow records: 64 int32 keys, then 64 values
struct __attribute__((packed, aligned(4))) Rec12 {
    uint32_t k, lo, hi;
};
__host__ __device__ __forceinline__ Rec12 rec12_of(int64_t mix, int64_t val) {
    Rec12 r;
    r.k = (uint32_t)key_of(mix);
    r.lo = (uint32_t)(uint64_t)val;
    r.hi = (uint32_t)((uint64_t)val >> 32);
    return r;
}
__host__ __device__ __forceinline__ int64_t rec12_mix(const Rec12& r) { return mix_of((int64_t)(int32_t)r.k); }
__host__ __device__ __forceinline__ int64_t rec12_val(const Rec12& r) { return (int64_t)((uint64_t)r.hi << 32 | r.lo); }

struct IngestParams {
    WindowSpec w;
    int64_t n;
    const int64_t* key;
    const int64_t* ts;
    const int64_t* val;
    const uint8_t* vnull;
    int64_t progress;          // current progress (watermark) for the late check
    // fast path (host-precomputed): d = rowtime + tz - tbase in [0, 2^32) -> slice end
    // tbase + S * (umulhi64(d, div_m) + 1); not late iff that end > fired_lim
    int64_t tbase;             // a slice start (== offset mod S); fast path off when div_m == 0
    uint64_t div_m;            // ceil(2^64 / S)
    int64_t qbase;             // floor_div(tbase, S) + 1
    int64_t fired_lim;         // progress + 1 + tz (saturated): slice ends <= fired_lim are fired
    int32_t lanes;             // power of two <= kMaxLanes
    int32_t region_bits;       // log2(P); bucket = (slice lane, top region_bits of fmix64(key))
    int64_t filter_lo;         // slice-index filter [lo, hi): floor_div(target, slice)
    int64_t filter_hi;
    int32_t count_drops;
    int32_t grid;              // number of workgroups (segments)
    int32_t vec;               // 1: key/ts/val 16-byte aligned -> paired 16-B loads
    int32_t sorted;            // scatter variant: 1 tile-sorted (<= 2 lane slots), 0 direct
    int32_t lane_slot[kMaxLanes];  // sorted scatter: lane -> slot (-1 inactive)
    // count outputs
    uint32_t* hist;            // [grid][F] (workgroup-major); after k_hist_columns: per-wg prefix
    unsigned long long* drops;
    long long* qmin;           // min / max slice index of the accepted records
    long long* qmax;
    long long* qnext;          // min slice index >= filter_hi of the accepted records (JMAX: none)
    unsigned long long* lane_mask;    // bit l: some record has slice index == l (mod lanes)
    unsigned long long* lane_total;   // [kMaxLanes] accepted records per lane
    unsigned int* max_bucket;  // max over workgroups and buckets of a workgroup's bucket count (skew hint)
    unsigned int* wide;        // pass 1: set when an accepted record's key does not fit 32 bits (the word
                               // after max_bucket in the counter block)
    // scatter inputs/outputs
    const uint32_t* bucket_base; // [F + 1] exclusive scan of bucket totals (lane-major)
    int64_t lane_shift[kMaxLanes];  // staged position = bucket_base[b] + prefix + lane_shift[lane]
    int64_t* st_rec;           // staged record area (all lanes), AoS {key, val} or {key}
    int32_t st_stride;
    // narrow staging: pass 1's tile records and pass 2's staged records are 12 B {int32 key,
    // value bits} at byte 12 * position, while every key seen fits 32 bits (pass 1 reports a
    // wider one in *wide: the plan then stops the speculative pass 2, the host reruns pass 1
    // with 16-B records and the operator stays on them)
    int32_t narrow;
    uint8_t* st_null;          // NULL flags at the same positions (may be null)
    // two-pass partition
    longlong2* tmp;            // pass-1 output: tile (g, j) sorted by coarse bucket at its input offset
    uint8_t* tmp_null;         // NULL flags of tmp (when vnull)
    uint16_t* dir;             // [grid * max_tiles][n_coarse + 1] coarse offsets within each tile
    int32_t max_tiles;         // tiles per workgroup segment (ceil(segment / kPart1Tile))
    uint32_t* tile_btot;       // tile pass: [n_coarse] per-bucket totals, zeroed by k_tile_part1's
                               // workgroup 0 (k_tile_dirt adds into them after it); may be null
    int32_t p2_group;          // pass-1 workgroups per pass-2 unit (0: part2_group's default); 1 for
                               // skewed input, whose hot coarse bucket would load a few units
    int32_t n_coarse;          // lanes << (region_bits - kFineBits)
    int64_t* sink;             // >= 32 B of scratch: idle lanes store here (static store counts)
    // speculative pass 2 (launched right after pass 1, no host round trip): the staged
    // positions come from k_ingest_plan's verdict instead of lane_shift; not ok -> no-op
    const struct IngestPlan* plan;
};

// Lane decision of one ingest pass taken on the device (k_ingest_plan) from pass 1's
// counters and the host's lane state, exactly as the host takes it (fg_engine.cpp
// ingest_pass): ok iff the pass's slices fit the lanes without a flush.
struct IngestPlan {
    int32_t ok;
    int32_t active;            // bit l: lane l receives records (the counters are reset by then)
    int64_t lane_shift[kMaxLanes];
};
struct PlanParams {
    int64_t lane_cap;
    int64_t q[kMaxLanes];      // slice index a lane holds (INT64_MIN: empty)
    int64_t fill[kMaxLanes];   // records staged in the lane
};

constexpr int kMaxMergeBatches = 32;         // pipelined merge: staged batches held in LDS
constexpr int kPartStride = kSlots + 1;      // heavy chunks: partial-table entries per chunk

struct MergeParams {
    int32_t region_bits;       // log2(P): state regions
    int32_t fast_stream;       // every batch plain AoS {key, value}, n_batches <= kMaxMergeBatches
    int32_t narrow;            // fast stream of narrow 12-B records (every batch stride 3)
    int32_t compact;           // compact LDS table (fast_stream, no src tables, < 2^32 records)
    int32_t n_src;
    int32_t src_narrow;        // 1: some source table holds narrow (16-B) entries; 2: every one does
    const TableRef* src;       // device array [n_src]; null: n_src <= 2, the tables in src_in
    TableRef src_in[2];        // up to two source tables by value (no descriptor copy per merge)
    int32_t n_batches;
    int32_t val_type;          // 0 none, 1 i64, 2 f64
    const StagedBatch* batches;  // device array [n_batches]
    int32_t has_dst;
    int32_t emit;
    TableRef dst;
    unsigned long long* dst_total;  // += entries written to dst (may be null)
    // emit
    int64_t wstart, wend, out_ts;
    int32_t num_aggs;
    int32_t aggs[kMaxAggs];
    int64_t* out_key;
    int64_t* out_ws;
    int64_t* out_we;
    int64_t* out_agg[kMaxAggs];
    uint8_t* out_null;
    int64_t* out_rowtime;      // may be null
    unsigned long long* out_count;
    int64_t out_cap;
    unsigned int* overflow;    // bit0: region overflow, bit1: output overflow, bit2: LDS table full
    unsigned long long* stamps;  // diagnostic builds only (FG_STAMPS): per-phase cycles summed over waves
    // skewed (heavy) regions, split off by k_heavy_plan (may be null):
    const uint8_t* heavy;      // [P] 1: the region is merged by the heavy pass, skipped here
    // heavy pass (wide kernel only): regions = region_list[0 .. *n_list), each with the
    // partial tables of its chunks [chunk0[i], chunk0[i + 1]) as an extra source
    const int32_t* region_list;
    const int32_t* n_list;
    const int32_t* chunk0;
    const int64_t* part_key;   // [chunk * kSlots + e]
    const int64_t* part_cs;
    const int64_t* part_cn;
    const int64_t* part_sum;
    const int64_t* part_v1;    // multi-value operator: value slots 1 and 2 of the partial rows
    const int64_t* part_v2;
    const uint32_t* part_n;    // entries per chunk (kChunkFailed: the chunk's table overflowed)
    // Region overflow (LDS table full, or more than kRegionCap entries for a table write): the
    // region emits and writes nothing, and (job << kFailJobShift | region) is appended to
    // fail_list, so the host can split the regions and redo exactly the failed ones
    // (BytesMap growth, BytesMap.java:229-290). A retry launch names its regions in retry_list.
    uint32_t* fail_list;
    uint32_t* fail_n;
    int32_t fail_cap;
    int32_t job;
    const int32_t* retry_list;
    int32_t n_retry;
    // restore re-fire of shared windows (wide merge only): entries of source j with bit j of
    // mark_mask set are marked; emit_marked emits marked entries holding state only; dst_mode
    // 1 writes the marked entries holding state, 2 every marked entry, both as keys with zero
    // accumulators (a chain table of the keys whose timers chain on)
    int32_t emit_marked;
    unsigned long long src_null_mask;   // source j (< 64) may hold NULL counts (else its cnt_null column is 0)
    int32_t hot_keys;          // skewed staging (Zipf): compact merges pre-combine a wave's equal keys
    unsigned long long mark_mask;
    unsigned long long markonly_mask;   // sources that only mark (their accumulators are not added)
    int32_t dst_mode;
    // multi-value operator (mv): value slot k accumulates with op vop[k] (0 SUM, 1 MIN,
    // 2 MAX, 3 none) over the value type in val_type; output aggregate a reads slot agg_slot[a];
    // tables have kNV value columns and kRegionCapMV entries per region
    int32_t mv;
    int32_t vop[kNV];
    int32_t agg_slot[kMaxAggs];
};
// region capacity and 8-byte words per entry of an operator's tables
__host__ __device__ __forceinline__ int table_cap(int mv) { return mv ? kRegionCapMV : kRegionCap; }
__host__ __device__ __forceinline__ int table_cols(int mv) { return mv ? 3 + kNV : 4; }
constexpr int kFailJobShift = 14;             // region < 2^13
constexpr uint32_t kChunkFailed = 0xFFFFFFFFu;

// Skewed regions (Zipf hot keys): a region whose staged records exceed `threshold` is
// merged in chunks of `chunk` records by k_heavy_chunks (one LDS table per chunk, with a
// wave-level pre-reduction of equal keys), then the chunks' partial tables (and the
// region's resident state) by the heavy pass of the wide merge, so that no region's work
// lands on one workgroup.
struct HeavyPlan {
    const StagedBatch* batches;
    int32_t n_batches;
    int32_t region_bits;
    int64_t threshold;
    int64_t chunk;
    int32_t max_chunks;
    int32_t val_type;
    uint8_t* heavy;            // [P]
    int32_t* region_list;      // [P]
    int32_t* n_list;           // [2]: heavy regions, chunks
    int32_t* chunk0;           // [P + 1]
    int32_t* chunk_list;       // [max_chunks]: list index of the chunk's region
    int64_t* chunk_v0;         // [max_chunks]: first record of the chunk within the region's
    int64_t* chunk_v1;         //   records, batches concatenated in order
    int64_t* part_key;         // [max_chunks * kSlots]
    int64_t* part_cs;
    int64_t* part_cn;
    int64_t* part_sum;
    int64_t* part_v1;          // multi-value operator: value slots 1 and 2
    int64_t* part_v2;
    uint32_t* part_n;          // [max_chunks]
    unsigned int* overflow;
    // multi-value operator: val_type is the value type, slot k folds with op vop[k] (as MergeParams)
    int32_t mv;
    int32_t vop[kNV];
};

// Accumulator rows of the global phase: input columns and the SoA staged area (all lanes)
struct AccColumns {
    const int64_t* in_cnt_star;
    const int64_t* in_cnt_val;
    const int64_t* in_sum;
    int64_t* key;
    int64_t* cnt_star;
    int64_t* cnt_null;
    int64_t* sum;
    const int64_t* in_v1;      // multi-value operator: the partial MIN / MAX (else null)
    const int64_t* in_v2;
    int64_t* v1;
    int64_t* v2;
};

struct ExportParams {
    TableRef t;
    const uint64_t* region_off;  // [P] exclusive prefix of counts
    int64_t slice_end;
    int64_t* out_key;
    int64_t* out_slice;
    int64_t* out_cnt_star;
    int64_t* out_cnt_val;
    int64_t* out_sum;
    int64_t* out_v1;             // multi-value operator: value slots 1 and 2
    int64_t* out_v2;
    int32_t mv;
    int32_t pad;
};

hipError_t launch_ingest_count(const IngestParams& p, hipStream_t s);
// global phase: rowtime = slice_end - 1 - tz for partial rows; scatter of accumulator rows
hipError_t launch_pseudo_rowtime(const int64_t* slice_end, int64_t n, int64_t tz, int64_t* out, hipStream_t s);
// a few words stored by a kernel (scratch counters initialised in stream order: a small
// host-to-device copy costs a blit plus ~20 us of queue latency before the next kernel)
struct Words16 {
    unsigned long long v[16];
    int32_t n;
};
hipError_t launch_store_words(unsigned long long* dst, const Words16& w, hipStream_t s);
hipError_t launch_publish_words(const unsigned long long* src, int32_t n, unsigned long long* host,
                                unsigned long long seq, hipStream_t s);
hipError_t launch_widen_columns(const int32_t* k32, const uint32_t* t32, const int32_t* v32, int64_t n, int64_t tbase,
                                int64_t* key, int64_t* ts, int64_t* val, hipStream_t s);
hipError_t launch_window_end_rowtime(const int64_t* wend, int64_t n, int64_t tz, int64_t S, int64_t phase,
                                     int64_t* out, unsigned long long* off_grid, hipStream_t s);
hipError_t launch_acc_scatter(const IngestParams& p, const AccColumns& a, hipStream_t s);
// packed BinaryRowData fixed-length parts -> key / rowtime / value / NULL columns; bad[0]
// counts rows whose key or rowtime is NULL, bad[1] NULL values
struct RowLayout {
    int32_t stride, key_off, ts_off, val_off;   // byte offsets of the fields (val_off < 0: none)
    int32_t key_bit, ts_bit, val_bit;           // null-bit indices (8 + field)
    int32_t pad;
};
hipError_t launch_rows_to_columns(const uint8_t* rows, int64_t n, const RowLayout& L, int64_t* key, int64_t* ts,
                                  int64_t* val, uint8_t* vnull, unsigned long long* bad, hipStream_t s);
// two-pass partition: pass 1 does the count pass's work (drops, slice range, lane totals,
// fine histogram per workgroup) while sorting tiles by coarse bucket into p.tmp / p.dir
hipError_t launch_part1(const IngestParams& p, hipStream_t s);
// pass 2: one workgroup per (active coarse bucket, pass-1 workgroup); p.bucket_base, p.hist
// (column prefixes), p.lane_shift and p.lane_slot as for the scatter
hipError_t launch_part2(const IngestParams& p, hipStream_t s);
// After pass 1 (or the count pass) and k_hist_columns, one workgroup: the exclusive scan of
// the bucket totals into bucket_off[F + 1]; the pass's counter words (`counters`, n_words)
// copied to host-visible memory `host` and reset to `reset` for the next pass; with `pp`,
// the lane plan of the speculative pass 2 (into plan, and after the counters in `host`).
struct ScanPlanArgs {
    const uint32_t* totals;
    uint32_t* bucket_off;
    int32_t F;
    int32_t n_words;
    unsigned long long* counters;
    unsigned long long* host;          // n_words counter words, then an IngestPlan
    Words16 reset;
    int32_t do_plan;
    int32_t pad;
    IngestPlan* plan;
    unsigned long long seq;            // written after everything else: the host polls for it
};
hipError_t launch_scan_plan(const IngestParams& p, const PlanParams& pp, const ScanPlanArgs& a, hipStream_t s);
int32_t part1_max_tiles(int64_t n, int32_t grid);
hipError_t launch_ingest_scatter(const IngestParams& p, hipStream_t s);   // picks the variant by p.sorted
// exclusive scan of n u32 (n < 2^32 total); out has n + 1 entries; tmp >= scan_tmp_words(n)
size_t scan_tmp_words(int64_t n);
hipError_t launch_scan_u32(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* tmp, hipStream_t s);
// per bucket b: hist[g][b] <- sum_{g' < g} hist[g'][b]; totals[b] <- sum_g hist[g][b]
hipError_t launch_hist_columns(uint32_t* hist, uint32_t* totals, int32_t F, int32_t grid, hipStream_t s);
// persistent merge over the P regions: `workgroups` <= P workgroups, each a strided set of
// regions (p.compact: two workgroups fit a CU)
hipError_t launch_merge(const MergeParams& p, int32_t workgroups, hipStream_t s);
// fire one window straight from a single slice table (no combine): p's emit fields
hipError_t launch_emit_table(const MergeParams& p, const TableRef& t, hipStream_t s);
hipError_t launch_export(const ExportParams& p, int32_t regions, hipStream_t s);
// region split: the table `src` at old_bits -> `dst` at old_bits + shift (each region's
// entries go to its 2^shift child regions by the next bits of their key mix)
// a narrow table rewritten wide in place (regions 2^bits)
hipError_t launch_widen_table(const TableRef& t, int32_t bits, hipStream_t s);
hipError_t launch_split_table(const TableRef& src, const TableRef& dst, int32_t old_bits, int32_t shift, int32_t mv,
                              hipStream_t s);
hipError_t launch_heavy_plan(const HeavyPlan& hp, hipStream_t s);
hipError_t launch_heavy_chunks(const HeavyPlan& hp, int32_t workgroups, hipStream_t s);
// ---- tile staging: a TUMBLE window (or a local-phase slice) fired straight from pass-1 tiles ----
// Pass 1 (k_tile_part1) sorts each tile of kTileRecs records by CONSUMER BUCKET -- (lane, region
// >> kTileBits): 4 state regions, ~4.9k keys at 10M keys / 2^13 regions -- and writes it back in
// place (block-laid 12-B records {int32 key, value}, absolute record index) with a directory row
// of bucket offsets; k_tile_dirt transposes the directory into one (offset, length) column per
// bucket. At the fire, k_tile_fire gives each bucket one workgroup: it gathers the bucket's
// fragment of every tile, aggregates its keys in an LDS table and emits the fired rows -- the
// staged area of pass 2 is never written nor read back (RecordsWindowBuffer.flush + AggCombiner
// + fireWindow in one kernel). Anything else that needs the lane's records (a flush into a slice
// table, a checkpoint, a re-fire after restore) first converts the pass into a regular staged
// pass (k_tile_count + scan + k_tile_scatter).
constexpr int kTileBits = 2;                  // state regions per consumer bucket = 4
#ifndef FG_TILE_T
#define FG_TILE_T 768
#endif
#ifndef FG_TILE_R
#define FG_TILE_R 8
#endif
#ifndef FG_TILE_H
#define FG_TILE_H 1
#endif
constexpr int kTileThreads = FG_TILE_T;       // tile pass 1: one classification round of R records per
constexpr int kTileR = FG_TILE_R;             // thread (768 x 8: no spills at 170 VGPRs; more spill)
constexpr int kTileH = FG_TILE_H;             // rounds (halves) per tile
constexpr int kTileRecs = kTileH * kTileR * kTileThreads;   // records per pass-1 tile (6,144; even R: paired loads)
// directory row of one tile: nc u16 bucket offsets, the tile's total, padded to 4-B alignment
__host__ __device__ constexpr int64_t kTileDirStride(int nc) { return nc + 2; }
constexpr int kMaxTileBuckets = 4096;         // lanes << (region_bits - kTileBits)
constexpr int kTileSlots = 8192;              // consumer LDS table (~4.9k keys: 60 % load)
constexpr int kTileFireThreads = 1024;
constexpr int kTileMaxSub = 64;               // regions of one bucket at the current bits (materialize)
constexpr int kTileMaxRegionBits = 8;         // tile jobs with tables: at most 2^8 regions per item
constexpr int kTileMaxRegions = 1 << kTileMaxRegionBits;

// One tile-staged pass as the fire / materialize kernels read it (lane `lane`'s buckets)
struct TilePass {
    const void* rec;          // packed 12-B tile records at their absolute batch index (ld_tile_rec)
    const uint32_t* dt;       // [nc][nt]: offset | length << 16 of bucket c's fragment of tile t
    int64_t n;                // records of the pass (tile t holds records [t * kTileRecs, ...): pass 1's
                              // segments are whole tiles, so a tile's first record needs no division)
    int32_t nt, mt;           // tiles, tiles per pass-1 segment
    int32_t nc;               // buckets of the pass (all lanes)
    int32_t bits;             // region bits of the pass
    int32_t lane;
    int32_t pad;
    const uint32_t* btot;     // [nc] records per bucket of the pass (k_tile_dirt); may be null
};
// Skewed tile passes (hot keys, Zipf): a bucket whose records exceed kTileChunk is fired by
// several workgroups -- chunk items over equal ranges of its tiles, each aggregating its range in
// an LDS table (hot keys pre-combined across the wave) and writing the table as partial entries
// -- and the chunks' partials are then merged per bucket (k_tile_fire with merge = 1) into the
// rows / the destination table; the
// other buckets fire as usual. k_tile_plan lists the items on the device.
constexpr int kTileChunk = 1 << 16;           // records per chunk item of a split bucket
constexpr int kMaxTilePasses = 8;             // passes one split fire walks
struct TileItem {
    int32_t bucket;           // the lane's bucket (item of the plain fire)
    int32_t g_lo, g_hi;       // tiles [g_lo, g_hi) of the passes' concatenated tile sequence
    int32_t part;             // chunk ordinal of a split bucket (its partials); -1: rows directly
};
struct TileSplit {
    TileItem* items;          // [max_items], *n_items listed by k_tile_plan
    uint32_t* n_items;
    int32_t max_items;
    int32_t max_split;
    int32_t* split_b;         // split entry i: its bucket, first chunk ordinal, chunks
    int32_t* split_c0;
    int32_t* split_k;
    uint32_t* n_split;
    uint32_t* part_off;       // per chunk ordinal: first partial entry, entries (kChunkFailed: failed)
    uint32_t* part_n;
    uint32_t* part_fill;      // partial entries written (reservation counter)
    uint32_t* next_item;      // the fire's dynamic item counter (zeroed with the counts)
    uint32_t chunk;           // records per chunk item; 0: max(kTileChunk, the lane's mean bucket)
    uint32_t* icnt;           // materialize: [items][kTileMaxSub] records per sub-region of an item
    uint32_t part_cap;
    int32_t* p_key;           // partial entries: int32 key, COUNT(*), value bits (the LDS repr)
    uint32_t* p_cs;
    unsigned long long* p_v;
    uint32_t* bfail;          // [buckets] a chunk of the bucket failed: the merge skips it (the
                              // regions are redone by the split-and-retry protocol, listed once)
    int32_t gpre[kMaxTilePasses + 1];   // tiles before pass pi in the concatenated sequence
};
struct TileFire {
    MergeParams m;            // emit fields, value op, overflow / out_count / fail list, job, region_bits
    const TilePass* passes;   // device array [n_passes], all at bits `tbits` (n_passes > 2)
    TilePass one;             // the pass, by value, when n_passes == 1 (no descriptor copy)
    TilePass two;             // n_passes == 2: the passes are `one` and `two` (by value, no copy either)
    int32_t n_passes;
    int32_t tbits;
    // items: the lane's buckets 0 .. (1 << (tbits - kTileBits)) - 1, or (retry) regions at
    // m.region_bits: m.retry_list[0 .. m.n_retry), or (split) sp.items[0 .. *sp.n_items)
    int32_t split;            // sp holds a plan (k_tile_plan): a skewed pass's fire
    int32_t hot;              // split fire: pre-combine a wave's records of a hot key (SUM-family ops)
    int32_t merge;            // split fire, second launch: items = the split buckets (sp.split_b), each
                              // merging its chunks' partial entries (with its tables, rows, destination)
    TileSplit sp;
};
hipError_t launch_tile_part1(const IngestParams& p, hipStream_t s);
// directory transpose of a tile pass: dir [tiles][nc + 1] -> dt [nc][tiles] (lanes absent from
// *lane_mask skipped)
hipError_t launch_tile_dirt(const uint16_t* dir, int32_t tiles, int32_t nc, int32_t lane_shift,
                            const unsigned long long* lane_mask, uint32_t* dt, uint32_t* btot, hipStream_t s);
hipError_t launch_tile_fire(const TileFire& f, int32_t workgroups, hipStream_t s);
// the device self-check of the DPP scans and the tile walk (fg_selftest): 0 when they are right
int run_selftest(int device, char* msg, size_t cap);
// a split fire: the plan (one workgroup), then launch_tile_fire over its items and again with
// merge = 1 over the split buckets
hipError_t launch_tile_plan(const TileFire& f, hipStream_t s);

// materialize, over the items of a plan (launch_tile_plan of the one pass with sp.chunk =
// kTileMatChunk): per-region counts of the pass's lane added into hist[P] at `bits` (zeroed
// first) and kept per item in plan.icnt, then -- after the exclusive scan into bucket_off, copied
// into `cursor` -- the records into a regular narrow staged area (each item reserves its regions'
// blocks from cursor)
constexpr uint32_t kTileMatChunk = 1u << 14;
hipError_t launch_tile_count(const TilePass& tp, int32_t bits, const TileSplit& plan, uint32_t* hist,
                             int32_t workgroups, hipStream_t s);
hipError_t launch_tile_scatter(const TilePass& tp, int32_t bits, const TileSplit& plan, uint32_t* cursor, void* out_rec,
                               int32_t workgroups, hipStream_t s);

constexpr int kMaxOwnerCols = 8;
struct OwnerCols {
    int32_t ncols;
    const int64_t* in[kMaxOwnerCols];   // in[0] = key
    int64_t* out[kMaxOwnerCols];
};
hipError_t launch_partition_cols_by_owner(const OwnerCols& c, int64_t n, int32_t key_hash, int32_t max_p,
                                          int32_t par, int64_t* counts, uint32_t* scratch, size_t scratch_words,
                                          hipStream_t s);
hipError_t launch_key_groups(const int64_t* key, int64_t n, int32_t key_hash, int32_t max_p, int32_t* out,
                             hipStream_t s);
hipError_t launch_partition_by_owner(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n,
                                     int32_t key_hash, int32_t max_p, int32_t parallelism, int64_t* out_key,
                                     int64_t* out_ts, int64_t* out_val, int64_t* counts, uint32_t* scratch,
                                     size_t scratch_words, hipStream_t s);
size_t partition_scratch_words(int64_t n, int32_t parallelism);

}  // namespace fg
