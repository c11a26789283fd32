// fg_kernels.hip -- gfx950 kernels of the keyed window-aggregation engine.
//
// Hot path:
//   k_ingest_count / k_ingest_scatter  a1 slice assignment + a2 late rules + a3 key hashing,
//                                      bucketing records by (slice lane, state region):
//                                      replaces RecordsWindowBuffer.addElement
//                                      (TR/operators/aggregate/window/buffers/RecordsWindowBuffer.java:81-97)
//   k_merge                            a4/a5/a7: a persistent workgroup per CU walks state regions;
//                                      per region it builds an LDS open-addressing table from
//                                      resident slice regions and the staged records, then writes
//                                      the region back (flush =
//                                      AggCombiner.combine, combines/AggCombiner.java:76-115)
//                                      and/or emits fired rows (fireWindow + mergeSlices,
//                                      processors/SliceSharedWindowAggProcessor.java:64-118)
//   k_export                           checkpoint image of the resident state
//   k_key_groups / k_owner_*           KeyGroupRangeAssignment routing for the key-group exchange
//
// All global traffic is streaming and coalesced; per-key read-modify-write happens in LDS
// (ds_cmpst_rtn_b64 / ds_add_u64 / ds_add_f64), never as global atomics.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include <type_traits>

#include "fg_kernels.h"

namespace fg {

thread_local LaunchEvents g_launch_ev;

typedef long long RecV2 __attribute__((ext_vector_type(2)));
typedef const RecV2 __attribute__((address_space(1)))* GlobalRec;

// 16-B record loads / stores (non-temporal forms measured within +-2 % or slower)
__device__ __forceinline__ longlong2 ld2(const void* q) {
    const RecV2 v = *static_cast<const RecV2*>(q);
    return make_longlong2(v.x, v.y);
}
__device__ __forceinline__ void st2(void* q, longlong2 a) {
    RecV2 v;
    v.x = a.x;
    v.y = a.y;
    *static_cast<RecV2*>(q) = v;
}
// a pointer that was itself loaded from memory is generic (flat) to the compiler: view it in
// the global address space so its loads are global_load (see `load` below)
template <class T>
__device__ __forceinline__ const T __attribute__((address_space(1)))* gbl(const T* q) {
    return (const T __attribute__((address_space(1)))*)q;
}

// Narrow 12-B records {int32 key, value bits} in blocks of 64 (kRec12Block bytes): the block's
// 64 keys (256 B), then its 64 values (512 B), record i in block i / 64 at lane i % 64. A
// wave's consecutive records are then one 4-B and one 8-B coalesced, naturally aligned access
// each (a packed 12-B record took unaligned dwordx3 accesses: pass 2's stores ran 1.7x slower
// than its 16-B ones). Indices are absolute from the buffer's base (a staged batch's first
// record is StagedBatch.rec_first), so batches appended to a lane share its blocks.
__device__ __forceinline__ Rec12 ld_rec12(const void* base, uint64_t i) {
    const char __attribute__((address_space(1)))* b =
        (const char __attribute__((address_space(1)))*)base + (i >> 6) * kRec12Block;
    const uint32_t k = *((const uint32_t __attribute__((address_space(1)))*)b + (i & 63));
    const uint64_t v = *((const uint64_t __attribute__((address_space(1)))*)(b + 256) + (i & 63));
    Rec12 r;
    r.k = k;
    r.lo = (uint32_t)v;
    r.hi = (uint32_t)(v >> 32);
    return r;
}
// narrow record {int32 key, value} i of a block-laid record array
__device__ __forceinline__ void st_rec12(void* base, uint64_t i, int64_t key, int64_t val) {
    char __attribute__((address_space(1)))* b = (char __attribute__((address_space(1)))*)base + (i >> 6) * kRec12Block;
    *((uint32_t __attribute__((address_space(1)))*)b + (i & 63)) = (uint32_t)key;
    *((uint64_t __attribute__((address_space(1)))*)(b + 256) + (i & 63)) = (uint64_t)val;
}

// Slice-table entry i of a region block b, wide ([mix][cnt_star][cnt_null][v0..]) or narrow
// ([int32 key][u32 cnt_star][v], fg_kernels.h TableRef)
typedef const int64_t __attribute__((address_space(1)))* gtab_t;
__device__ __forceinline__ int64_t tab_mix(gtab_t b, int cap, uint32_t i, bool nar) {
    return nar ? mix_of((int64_t)((const int32_t __attribute__((address_space(1)))*)b)[i]) : b[i];
}
__device__ __forceinline__ int32_t tab_key32(gtab_t b, int cap, uint32_t i, bool nar) {
    return nar ? ((const int32_t __attribute__((address_space(1)))*)b)[i] : (int32_t)key_of(b[i]);
}
__device__ __forceinline__ int64_t tab_cs(gtab_t b, int cap, uint32_t i, bool nar) {
    return nar ? (int64_t)((const uint32_t __attribute__((address_space(1)))*)b)[cap + i] : b[cap + i];
}
__device__ __forceinline__ int64_t tab_cn(gtab_t b, int cap, uint32_t i, bool nar) { return nar ? 0 : b[2 * cap + i]; }
__device__ __forceinline__ int64_t tab_v(gtab_t b, int cap, uint32_t i, bool nar, int q = 0) {
    return nar ? b[cap + i] : b[(3 + q) * cap + i];
}

// Tile-staged records (k_tile_part1 -> k_tile_fire / k_tile_mat): packed 12-B records {value bits,
// int32 key} at 12 * i, one dwordx3 access each (4-B aligned). The tiles are written whole and in
// order (a wave's stores are 768 contiguous bytes), and the fire gathers a bucket's fragments of a
// few records each: a fragment is one contiguous range. The value comes first so that a record
// loads into three VGPRs whose first two are an aligned 64-bit pair: with the key first the
// compiler realigned the value with two moves right after each load -- and waited for the load
// there (s_waitcnt vmcnt(0) per record: the fire's gathers were never in flight across its inserts)
__device__ __forceinline__ Rec12 ld_tile_rec(const void* base, uint64_t i) {
    const uint32_t __attribute__((address_space(1)))* q = (const uint32_t __attribute__((address_space(1)))*)base + 3 * i;
    Rec12 r;   // (three adjacent dwords: one global_load_dwordx3)
    r.lo = q[0];
    r.hi = q[1];
    r.k = q[2];
    return r;
}
__device__ __forceinline__ void st_tile_rec(void* base, uint64_t i, int64_t key, int64_t val) {
    uint32_t __attribute__((address_space(1)))* q = (uint32_t __attribute__((address_space(1)))*)base + 3 * i;
    q[0] = (uint32_t)val;   // (one global_store_dwordx3)
    q[1] = (uint32_t)((uint64_t)val >> 32);
    q[2] = (uint32_t)key;
}

// A pointer every lane of the wave holds (loaded from LDS, so the compiler cannot tell):
// moved to SGPRs, so loads off it take the scalar-base + 32-bit-offset form (no 64-bit
// address arithmetic per lane).
template <class T>
__device__ __forceinline__ T* wave_uniform(T* q) {
    const uint64_t v = (uint64_t)q;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (T*)(((uint64_t)hi << 32) | lo);
}

// A 0 the compiler cannot see through (an SGPR): `(&kernel_arg)[opaque_zero()]` re-reads a kernel
// argument where it is used instead of at the kernel's entry (loop-invariant loads are hoisted).
__device__ __forceinline__ int opaque_zero() {
    int z = 0;
    asm volatile("" : "+s"(z));
    return z;
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS ops, not for its
// global loads/stores (a __syncthreads() also drains vmcnt, stalling on in-flight stores).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}


// ----------------------------------------------------------------------------------------
// record classification shared by count and scatter (must agree exactly)
// ----------------------------------------------------------------------------------------
// returns bucket >= 0, -1 when the record is late-dropped, -2 when outside the slice filter;
// *h_out = fmix64(key), the form in which the key is staged and kept (fg_window.h)
__device__ __forceinline__ int classify(const IngestParams& p, int64_t key, int64_t ts, int64_t* q_out,
                                        int64_t* h_out) {
    int64_t q;
    const uint64_t d = (uint64_t)ts + (uint64_t)p.w.tz - (uint64_t)p.tbase;
    const uint64_t qq = __umul64hi(d, p.div_m);
    const int64_t end_fast = p.tbase + (int64_t)((qq + 1) * (uint64_t)p.w.slice);
    if (p.div_m != 0 && d < (1ull << 32) && ts != JMAX && end_fast > p.fired_lim) {
        q = p.qbase + (int64_t)qq;              // assignSliceEnd, not fired: no late handling
    } else {
        int64_t target;
        if (!target_slice(p.w, ts, p.progress, &target)) return -1;
        q = floor_div_fast(target, p.w.slice, p.w.rslice);
    }
    *q_out = q;   // also for records outside the filter: the batch's whole slice range is counted
    if (q < p.filter_lo || q >= p.filter_hi) return -2;
    const int lane = (int)(q & (int64_t)(p.lanes - 1));
    const uint64_t h = fmix64((uint64_t)key);
    *h_out = (int64_t)h;
    const uint32_t rb = p.region_bits == 0 ? 0u : (uint32_t)(h >> (64 - p.region_bits));
    return (lane << p.region_bits) | (int)rb;
}
__device__ __forceinline__ int classify(const IngestParams& p, int64_t key, int64_t ts, int64_t* q_out) {
    int64_t h;
    return classify(p, key, ts, q_out, &h);
}

__device__ __forceinline__ void seg_bounds(int64_t n, int grid, int g, int64_t* b, int64_t* e) {
    int64_t per = (n + grid - 1) / grid;
    per = (per + 1) & ~int64_t(1);   // even, so pair loads stay aligned
    *b = per * g < n ? per * g : n;
    *e = *b + per < n ? *b + per : n;
}

// ----------------------------------------------------------------------------------------
// exclusive scan of u32 (reduce-then-scan, 4096 items per block)
// ----------------------------------------------------------------------------------------
constexpr int kScanThreads = 1024;
constexpr int kScanItems = 4;
constexpr int kScanChunk = kScanThreads * kScanItems;

template <bool kLdsOnly>
__device__ __forceinline__ uint32_t block_exclusive_scan_t(uint32_t v, uint32_t* s_wave, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) s_wave[wave] = x;
    if (kLdsOnly) lds_barrier(); else __syncthreads();
    if (wave == 0) {
        const int nw = blockDim.x >> 6;
        uint32_t w = lane < nw ? s_wave[lane] : 0u;
        for (int off = 1; off < 64; off <<= 1) {
            uint32_t y = __shfl_up(w, off);
            if (lane >= off) w += y;
        }
        if (lane < nw) s_wave[lane] = w;   // inclusive
    }
    if (kLdsOnly) lds_barrier(); else __syncthreads();
    const uint32_t wave_base = wave ? s_wave[wave - 1] : 0u;
    *total = s_wave[(blockDim.x >> 6) - 1];
    if (kLdsOnly) lds_barrier(); else __syncthreads();
    return wave_base + x - v;
}
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* s_wave, uint32_t* total) {
    return block_exclusive_scan_t<false>(v, s_wave, total);
}

// ----------------------------------------------------------------------------------------
// ingest: count (a1 slice assignment + a2 late rules + bucket histogram per workgroup)
// ----------------------------------------------------------------------------------------
constexpr int kMaxBuckets = kMaxStageBuckets;

__global__ __launch_bounds__(kIngestThreads) void k_ingest_count(IngestParams p) {
    __shared__ uint32_t s_hist[kMaxBuckets];
    __shared__ unsigned long long s_drop;
    __shared__ long long s_qmin, s_qmax, s_qnext;
    __shared__ uint32_t s_mask;
    __shared__ uint32_t s_lane[kMaxLanes];
    const int F = p.lanes << p.region_bits;
    const int tid = threadIdx.x;
    for (int i = tid; i < F; i += kIngestThreads) s_hist[i] = 0;
    if (tid == 0) { s_drop = 0; s_qmin = JMAX; s_qmax = JMIN; s_qnext = JMAX; s_mask = 0; }
    if (tid < kMaxLanes) s_lane[tid] = 0;
    __syncthreads();

    int64_t beg, end;
    seg_bounds(p.n, p.grid, blockIdx.x, &beg, &end);
    uint32_t drops = 0, mask = 0;
    long long qmin = JMAX, qmax = JMIN, qnext = JMAX;
    const int lm = p.lanes - 1;

    // pairs of records per thread: 16-byte loads of key and rowtime, 4 pairs in flight
    const int64_t npairs = (end - beg) >> 1;
    auto account = [&](int64_t k, int64_t ts) {
        int64_t q;
        const int b = classify(p, k, ts, &q);
        if (b >= 0) {
            atomicAdd(&s_hist[b], 1u);
            qmin = q < qmin ? q : qmin;
            qmax = q > qmax ? q : qmax;
            mask |= 1u << ((int)q & lm);
        } else if (b == -1) {
            drops++;
        } else {   // outside the slice filter: in the batch's slice range only
            qmin = q < qmin ? q : qmin;
            qmax = q > qmax ? q : qmax;
            if (q >= p.filter_hi) qnext = q < qnext ? q : qnext;   // next occupied slice above the filter
        }
    };
    constexpr int kU = 4;
    for (int64_t p0 = 0; p0 < npairs; p0 += kU * kIngestThreads) {
        longlong2 k2[kU], t2[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int64_t pi = p0 + u * kIngestThreads + tid;
            if (pi >= npairs) continue;
            const int64_t i = beg + 2 * pi;
            if (p.vec) {
                k2[u] = *reinterpret_cast<const longlong2*>(p.key + i);
                t2[u] = *reinterpret_cast<const longlong2*>(p.ts + i);
            } else {
                k2[u].x = p.key[i]; k2[u].y = p.key[i + 1];
                t2[u].x = p.ts[i]; t2[u].y = p.ts[i + 1];
            }
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int64_t pi = p0 + u * kIngestThreads + tid;
            if (pi >= npairs) continue;
            account(k2[u].x, t2[u].x);
            account(k2[u].y, t2[u].y);
        }
    }
    if (((end - beg) & 1) && tid == 0) account(p.key[end - 1], p.ts[end - 1]);
    // wave reductions, then one LDS atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        drops += __shfl_down(drops, off);
        mask |= __shfl_down(mask, off);
        const long long oa = __shfl_down(qmin, off), oz = __shfl_down(qmax, off), on = __shfl_down(qnext, off);
        qmin = oa < qmin ? oa : qmin;
        qmax = oz > qmax ? oz : qmax;
        qnext = on < qnext ? on : qnext;
    }
    if ((tid & 63) == 0) {
        if (drops) atomicAdd(&s_drop, (unsigned long long)drops);
        if (mask) atomicOr(&s_mask, mask);
        if (qmin != JMAX) atomicMin(&s_qmin, qmin);
        if (qmax != JMIN) atomicMax(&s_qmax, qmax);
        if (qnext != JMAX) atomicMin(&s_qnext, qnext);
    }
    __syncthreads();
    // workgroup-major histogram: hist[g * F + b] (contiguous stores) + per-lane totals
    uint32_t lane_part = 0, bmax = 0;
    int lane_of = -1;
    for (int b = tid; b < F; b += kIngestThreads) {
        const uint32_t c = s_hist[b];
        p.hist[(int64_t)blockIdx.x * F + b] = c;
        bmax = c > bmax ? c : bmax;
        const int l = b >> p.region_bits;
        if (l != lane_of) {
            if (lane_part) atomicAdd(&s_lane[lane_of], lane_part);
            lane_of = l;
            lane_part = 0;
        }
        lane_part += c;
    }
    if (lane_part) atomicAdd(&s_lane[lane_of], lane_part);
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t y = __shfl_xor(bmax, off);
        bmax = y > bmax ? y : bmax;
    }
    if ((tid & 63) == 0 && p.max_bucket && bmax) atomicMax(p.max_bucket, bmax);
    __syncthreads();
    if (tid < p.lanes && s_lane[tid]) atomicAdd(&p.lane_total[tid], (unsigned long long)s_lane[tid]);
    if (tid == 0) {
        if (p.count_drops && s_drop) atomicAdd(p.drops, s_drop);
        if (s_mask) atomicOr(p.lane_mask, (unsigned long long)s_mask);
        if (s_qmin != JMAX) atomicMin(p.qmin, s_qmin);
        if (s_qmax != JMIN) atomicMax(p.qmax, s_qmax);
        if (s_qnext != JMAX) atomicMin(p.qnext, s_qnext);
    }
}

// ----------------------------------------------------------------------------------------
// ingest: scatter into the per-lane staged areas (bucket-major within each batch; within
// a (bucket, workgroup) run the order is arrival order up to LDS atomic ordering)
// ----------------------------------------------------------------------------------------
// Direct scatter (any number of active lanes): one 16-B store per record at its
// bucket cursor (LDS atomic); used when a batch touches more than two slice lanes.
__global__ __launch_bounds__(kIngestThreads) void k_ingest_scatter_direct(IngestParams p) {
    __shared__ uint32_t s_cur[kMaxBuckets];
    const int F = p.lanes << p.region_bits;
    const int tid = threadIdx.x;
    for (int b = tid; b < F; b += kIngestThreads)
        s_cur[b] = (uint32_t)((int64_t)p.bucket_base[b] + p.hist[(int64_t)blockIdx.x * F + b] +
                              p.lane_shift[b >> p.region_bits]);
    __syncthreads();
    int64_t beg, end;
    seg_bounds(p.n, p.grid, blockIdx.x, &beg, &end);
    const bool has_val = p.val != nullptr;
    const bool has_null = p.vnull != nullptr;
    const bool aos = p.st_stride == 2;
    for (int64_t i = beg + tid; i < end; i += kIngestThreads) {
        const int64_t k = p.key[i];
        int64_t q, h;
        const int b = classify(p, k, p.ts[i], &q, &h);
        if (b < 0) continue;
        const uint32_t pos = atomicAdd(&s_cur[b], 1u);
        if (aos) *reinterpret_cast<longlong2*>(p.st_rec + 2 * (int64_t)pos) = make_longlong2(h, has_val ? p.val[i] : 0);
        else p.st_rec[pos] = h;
        if (has_null) p.st_null[pos] = p.vnull[i];
    }
}

// Tile-sorted scatter (<= 2 active slice lanes). Per tile of kTile records (8 per thread,
// kept in registers): rank each record in its bucket with an LDS atomic, scan the tile
// counts (each thread owns 8 consecutive buckets), advance the buckets' staged cursors,
// then stage the tile bucket-sorted through LDS in rounds of kRound slots and write
// every bucket run with consecutive lanes (slot i of bucket b goes to
// cursor[b] - offset[b + 1] + i). Only LDS is ordered by the barriers: stores stay in
// flight.
constexpr int kPerThread = kTile / kIngestThreads;   // 8
constexpr int kRound = 4096;                         // slots staged per round

template <int BPT>   // slot buckets per thread: FS <= BPT * kIngestThreads
__global__ __launch_bounds__(kIngestThreads) void k_ingest_scatter_sorted(IngestParams p) {
    __shared__ longlong2 s_rec[kRound];                // 64 KiB
    __shared__ uint16_t s_bkt[kRound];                 // 8 KiB: bucket of each slot
    __shared__ uint32_t s_off[kMaxSortedBuckets + 1];  // 32 KiB: tile counts, then tile offsets
    __shared__ uint32_t s_cur[kMaxSortedBuckets];      // 32 KiB: staged cursor (end of the tile's run)
    __shared__ uint32_t s_wave[16];
    const int P = 1 << p.region_bits;
    const int F = p.lanes << p.region_bits;
    const int tid = threadIdx.x;
    int nslots = 0;
    {
        for (int l = 0; l < kMaxLanes; l++) {
            const int sl = p.lane_slot[l];
            if (sl < 0) continue;
            nslots++;
            for (int r = tid; r < P; r += kIngestThreads) {
                const int bf = l * P + r;
                s_cur[sl * P + r] =
                    (uint32_t)((int64_t)p.bucket_base[bf] + p.hist[(int64_t)blockIdx.x * F + bf] + p.lane_shift[l]);
            }
        }
        for (int b = tid; b <= kMaxSortedBuckets; b += kIngestThreads) s_off[b] = 0;
    }
    // thread tid owns the slot buckets [tid * BPT, tid * BPT + BPT); bucket FS is the total
    const int FS = nslots << p.region_bits;
    constexpr int bpt = BPT;
    __syncthreads();
    int64_t beg, end;
    seg_bounds(p.n, p.grid, blockIdx.x, &beg, &end);
    const bool has_val = p.val != nullptr;
    const bool has_null = p.vnull != nullptr;
    const bool aos = p.st_stride == 2;

    for (int64_t t0 = beg; t0 < end; t0 += kTile) {
        const int64_t tn = end - t0 < kTile ? end - t0 : kTile;
        int64_t rk[kPerThread], rv[kPerThread];
        uint32_t rbr[kPerThread];   // (rank << 13) | slot bucket, 0xffffffff = not staged
        // 1) load (pairs: records t0 + 2*(tid + j*1024) + {0,1}) + classify + rank
        if (tn == kTile && p.vec) {
            longlong2 k2[kPerThread / 2], t2[kPerThread / 2];
#pragma unroll
            for (int j = 0; j < kPerThread / 2; j++) {
                const int64_t i = t0 + 2 * ((int64_t)tid + (int64_t)j * kIngestThreads);
                k2[j] = *reinterpret_cast<const longlong2*>(p.key + i);
                t2[j] = *reinterpret_cast<const longlong2*>(p.ts + i);
            }
#pragma unroll
            for (int j = 0; j < kPerThread / 2; j++) {
                int64_t q;
                int b0 = classify(p, k2[j].x, t2[j].x, &q, &rk[2 * j]);
                int b1 = classify(p, k2[j].y, t2[j].y, &q, &rk[2 * j + 1]);
                if (b0 >= 0) b0 = p.lane_slot[b0 >> p.region_bits] * P + (b0 & (P - 1));
                if (b1 >= 0) b1 = p.lane_slot[b1 >> p.region_bits] * P + (b1 & (P - 1));
                rbr[2 * j] = b0 >= 0 ? (atomicAdd(&s_off[b0], 1u) << 13) | (uint32_t)b0 : 0xffffffffu;
                rbr[2 * j + 1] = b1 >= 0 ? (atomicAdd(&s_off[b1], 1u) << 13) | (uint32_t)b1 : 0xffffffffu;
            }
            // values are not needed until staging: their latency hides behind the scan
            if (has_val) {
#pragma unroll
                for (int j = 0; j < kPerThread / 2; j++) {
                    const int64_t i = t0 + 2 * ((int64_t)tid + (int64_t)j * kIngestThreads);
                    const longlong2 v2 = *reinterpret_cast<const longlong2*>(p.val + i);
                    rv[2 * j] = v2.x;
                    rv[2 * j + 1] = v2.y;
                }
            } else {
#pragma unroll
                for (int j = 0; j < kPerThread; j++) rv[j] = 0;
            }
        } else {
#pragma unroll
            for (int j = 0; j < kPerThread / 2; j++) {
                const int64_t li = 2 * ((int64_t)tid + (int64_t)j * kIngestThreads);
                const int64_t i = t0 + li;
                longlong2 k2 = {0, 0}, t2 = {0, 0};
                if (li < tn) {
                    k2.x = p.key[i];
                    t2.x = p.ts[i];
                }
                if (li + 1 < tn) {
                    k2.y = p.key[i + 1];
                    t2.y = p.ts[i + 1];
                }
                rk[2 * j] = rk[2 * j + 1] = 0;
                int64_t q;
                int b0 = li < tn ? classify(p, k2.x, t2.x, &q, &rk[2 * j]) : -3;
                int b1 = li + 1 < tn ? classify(p, k2.y, t2.y, &q, &rk[2 * j + 1]) : -3;
                if (b0 >= 0) b0 = p.lane_slot[b0 >> p.region_bits] * P + (b0 & (P - 1));
                if (b1 >= 0) b1 = p.lane_slot[b1 >> p.region_bits] * P + (b1 & (P - 1));
                rbr[2 * j] = b0 >= 0 ? (atomicAdd(&s_off[b0], 1u) << 13) | (uint32_t)b0 : 0xffffffffu;
                rbr[2 * j + 1] = b1 >= 0 ? (atomicAdd(&s_off[b1], 1u) << 13) | (uint32_t)b1 : 0xffffffffu;
            }
#pragma unroll
            for (int j = 0; j < kPerThread; j++) {
                const int64_t li = 2 * ((int64_t)tid + (int64_t)(j >> 1) * kIngestThreads) + (j & 1);
                rv[j] = has_val && li < tn ? p.val[t0 + li] : 0;
            }
        }
        lds_barrier();
        // 2) tile offsets (exclusive scan over the slot buckets, s_off[FS] = tile total);
        //    the cursors advance past this tile's runs
        {
            uint32_t local = 0;
#pragma unroll
            for (int q = 0; q < bpt; q++) {
                const int b = tid * bpt + q;
                if (b < FS) local += s_off[b];
            }
            uint32_t total;
            uint32_t run = block_exclusive_scan_t<true>(local, s_wave, &total);
#pragma unroll
            for (int q = 0; q < bpt; q++) {   // each thread rewrites only its own buckets
                const int b = tid * bpt + q;
                if (b >= FS) break;
                const uint32_t c = s_off[b];
                s_off[b] = run;
                s_cur[b] += c;
                run += c;
            }
            if (tid == 0) s_off[FS] = total;
        }
        lds_barrier();
        const uint32_t tile_total = s_off[FS];
        // 3) rounds: stage the slots of one round in bucket order, write the runs
        for (uint32_t lo = 0; lo < tile_total; lo += kRound) {
#pragma unroll
            for (int j = 0; j < kPerThread; j++) {
                if (rbr[j] == 0xffffffffu) continue;
                const int b = (int)(rbr[j] & 8191u);
                const uint32_t slot = s_off[b] + (rbr[j] >> 13);
                if (slot - lo >= (uint32_t)kRound) continue;
                s_rec[slot - lo] = make_longlong2(rk[j], rv[j]);
                s_bkt[slot - lo] = (uint16_t)b;
            }
            lds_barrier();
            const uint32_t hi = tile_total - lo < (uint32_t)kRound ? tile_total - lo : (uint32_t)kRound;
            for (uint32_t i = tid; i < hi; i += kIngestThreads) {
                const longlong2 r = s_rec[i];
                const int b = s_bkt[i];   // run of bucket b = [cursor - count, cursor)
                const int64_t pos = (int64_t)(s_cur[b] - s_off[b + 1] + lo + i);
                if (aos) *reinterpret_cast<longlong2*>(p.st_rec + 2 * pos) = r;
                else p.st_rec[pos] = r.x;
            }
            if (lo + kRound < tile_total) lds_barrier();
        }
        if (has_null) {   // rare path: NULL flags go straight to their staged position
#pragma unroll
            for (int j = 0; j < kPerThread; j++) {
                if (rbr[j] == 0xffffffffu) continue;
                const int b = (int)(rbr[j] & 8191u);
                const int64_t li = 2 * ((int64_t)tid + (int64_t)(j >> 1) * kIngestThreads) + (j & 1);
                p.st_null[s_cur[b] - (s_off[b + 1] - s_off[b]) + (rbr[j] >> 13)] = p.vnull[t0 + li];
            }
        }
        lds_barrier();   // every write-out has read the offsets
        // 4) clear the tile counts for the next tile
#pragma unroll
        for (int q = 0; q < bpt; q++) {
            const int b = tid * bpt + q;
            if (b < FS) s_off[b] = 0;
        }
        lds_barrier();
    }
}

// ----------------------------------------------------------------------------------------
// two-pass partition (regions >= 64). A single tile-sorted pass over 4,096+ buckets writes
// ~2-record runs; two passes of 64-way sorting write sequential tiles, then 512-B+ runs.
// ----------------------------------------------------------------------------------------
// Pass 1: the count pass's bookkeeping (drops, slice range, lane totals, fine histogram per
// workgroup) plus a tile sort by coarse bucket (fine >> 6) written back to the tile's own
// input offset in p.tmp (fully sequential stores); p.dir holds each tile's coarse offsets.
// Software-pipelined: the next tile's key / rowtime / value loads are issued right after the
// current tile is classified, so they are in flight across its scan, LDS staging and
// write-out (barriers here order LDS only); one LDS staging round per tile.
__global__ __launch_bounds__(kPart1Threads) void k_part1(IngestParams p) {
    constexpr int T = kPart1Threads;
    constexpr int R = FG_P1_R;                       // records per thread per tile (even: 16-B pairs)
    constexpr int TILE = kPart1Tile;
    static_assert(R % 2 == 0, "pairs of records per thread");
    __shared__ uint32_t s_hist[kMaxPart1Fine];       // 64 KiB: fine histogram of this workgroup
    __shared__ longlong2 s_rec[TILE];                // the tile, coarse-bucket sorted
    __shared__ uint8_t s_nul[TILE];
    __shared__ uint32_t s_cc[kMaxCoarse + 1];        // tile coarse counts, then offsets
    __shared__ uint32_t s_wave[T / 64];
    __shared__ unsigned long long s_drop;
    __shared__ long long s_qmin, s_qmax, s_qnext;
    __shared__ uint32_t s_mask;
    __shared__ uint32_t s_lane[kMaxLanes];
    const int F = p.lanes << p.region_bits;
    const int NC = p.n_coarse;
    const int tid = threadIdx.x;
    for (int i = tid; i < F; i += T) s_hist[i] = 0;
    for (int i = tid; i <= NC; i += T) s_cc[i] = 0;
    if (tid == 0) { s_drop = 0; s_qmin = JMAX; s_qmax = JMIN; s_qnext = JMAX; s_mask = 0; }
    if (tid < kMaxLanes) s_lane[tid] = 0;
    __syncthreads();
    int64_t beg, end;
    seg_bounds(p.n, p.grid, blockIdx.x, &beg, &end);
    const bool has_val = p.val != nullptr;
    const bool has_null = p.vnull != nullptr;
    uint32_t drops = 0, mask = 0;
    bool wide = false;
    long long qmin = JMAX, qmax = JMIN, qnext = JMAX;
    const int lm = p.lanes - 1;

    // record u of this thread in a tile: pair u / 2 at 2 * (tid + (u / 2) * T), element u & 1
    auto li_of = [&](int u) -> int64_t { return 2 * ((int64_t)tid + (int64_t)(u >> 1) * T) + (u & 1); };
    // loads of the tile at t0 (records past the segment's end are not loaded: tn < TILE)
    auto load = [&](int64_t t0, longlong2 (&k2)[R / 2], longlong2 (&t2)[R / 2], longlong2 (&v2)[R / 2]) {
        const int64_t tn = end - t0 < TILE ? end - t0 : TILE;
        if (tn == TILE && p.vec) {
#pragma unroll
            for (int u = 0; u < R / 2; u++) {
                const int64_t i = t0 + li_of(2 * u);
                k2[u] = ld2(p.key + i);
                t2[u] = ld2(p.ts + i);
                v2[u] = has_val ? ld2(p.val + i) : make_longlong2(0, 0);
            }
        } else {
#pragma unroll
            for (int u = 0; u < R / 2; u++) {
                const int64_t l0 = li_of(2 * u);
                k2[u] = t2[u] = v2[u] = make_longlong2(0, 0);
                if (l0 < tn) {
                    k2[u].x = p.key[t0 + l0]; t2[u].x = p.ts[t0 + l0];
                    if (has_val) v2[u].x = p.val[t0 + l0];
                }
                if (l0 + 1 < tn) {
                    k2[u].y = p.key[t0 + l0 + 1]; t2[u].y = p.ts[t0 + l0 + 1];
                    if (has_val) v2[u].y = p.val[t0 + l0 + 1];
                }
            }
        }
    };
    longlong2 ka[R / 2], ta[R / 2], va[R / 2];
    if (beg < end) load(beg, ka, ta, va);
    int j = 0;
    for (int64_t t0 = beg; t0 < end; t0 += TILE, j++) {
        const int64_t tn = end - t0 < TILE ? end - t0 : TILE;
        // 1) classify + rank the current tile (LDS atomics); keys become their mixes
        uint32_t rcr[R];   // (rank << 9) | coarse, 0xffffffff = not staged
        int64_t hk[R];
        uint32_t nb = 0;   // NULL flags of the thread's records
#pragma unroll
        for (int u = 0; u < R; u++) {
            const int64_t li = li_of(u);
            rcr[u] = 0xffffffffu;
            hk[u] = 0;
            if (li >= tn) continue;
            const int64_t k = (u & 1) ? ka[u >> 1].y : ka[u >> 1].x;
            const int64_t ts = (u & 1) ? ta[u >> 1].y : ta[u >> 1].x;
            int64_t q;
            const int b = classify(p, k, ts, &q, &hk[u]);
            if (b >= 0) {
                wide |= k != (int64_t)(int32_t)k;   // (narrow staging needs 32-bit keys)
                if (p.narrow) hk[u] = k;            // narrow tiles carry the key, not its mix
                atomicAdd(&s_hist[b], 1u);
                qmin = q < qmin ? q : qmin;
                qmax = q > qmax ? q : qmax;
                mask |= 1u << ((int)q & lm);
                const uint32_t c = (uint32_t)b >> kFineBits;
                rcr[u] = (atomicAdd(&s_cc[c], 1u) << 9) | c;
                if (has_null && p.vnull[t0 + li]) nb |= 1u << u;
            } else if (b == -1) {
                drops++;
            } else {   // outside the slice filter: in the batch's slice range only
                qmin = q < qmin ? q : qmin;
                qmax = q > qmax ? q : qmax;
                if (q >= p.filter_hi) qnext = q < qnext ? q : qnext;   // next occupied slice above the filter
            }
        }
        int64_t rv[R];
#pragma unroll
        for (int u = 0; u < R; u++) rv[u] = (u & 1) ? va[u >> 1].y : va[u >> 1].x;
        // 2) prefetch the next tile: in flight across this tile's scan, staging and write-out
        if (t0 + TILE < end) load(t0 + TILE, ka, ta, va);
        lds_barrier();
        {   // exclusive scan of the tile's coarse counts; the offsets go to the directory
            const uint32_t c = tid < NC ? s_cc[tid] : 0u;
            uint32_t total;
            const uint32_t off = block_exclusive_scan_t<true>(c, s_wave, &total);
            if (tid < NC) s_cc[tid] = off;
            if (tid == 0) s_cc[NC] = total;
        }
        lds_barrier();
        uint16_t* drow = p.dir + ((int64_t)blockIdx.x * p.max_tiles + j) * (NC + 1);
        for (int c = tid; c <= NC; c += T) drow[c] = (uint16_t)s_cc[c];
        const uint32_t tile_total = s_cc[NC];
        // 3) stage the tile coarse-bucket sorted, then write it back sequentially
#pragma unroll
        for (int u = 0; u < R; u++) {
            if (rcr[u] == 0xffffffffu) continue;
            const uint32_t slot = s_cc[rcr[u] & 511u] + (rcr[u] >> 9);
            s_rec[slot] = make_longlong2(hk[u], rv[u]);
            if (has_null) s_nul[slot] = (uint8_t)((nb >> u) & 1u);
        }
        lds_barrier();
        if (p.narrow) {   // 12-B tile records {int32 key, value} (a wider key: the host reruns the pass)
            for (uint32_t i = tid; i < tile_total; i += T) {
                const longlong2 r = s_rec[i];
                st_rec12(p.tmp, (uint64_t)(t0 + i), r.x, r.y);
                if (has_null) p.tmp_null[t0 + i] = s_nul[i];
            }
        } else {
            for (uint32_t i = tid; i < tile_total; i += T) {
                st2(&p.tmp[t0 + i], s_rec[i]);
                if (has_null) p.tmp_null[t0 + i] = s_nul[i];
            }
        }
        lds_barrier();   // staging and the directory row have read the offsets
        for (int c = tid; c <= NC; c += T) s_cc[c] = 0;
        lds_barrier();
    }
    // bookkeeping as in k_ingest_count
    for (int off = 32; off > 0; off >>= 1) {
        drops += __shfl_down(drops, off);
        mask |= __shfl_down(mask, off);
        const long long oa = __shfl_down(qmin, off), oz = __shfl_down(qmax, off), on = __shfl_down(qnext, off);
        qmin = oa < qmin ? oa : qmin;
        qmax = oz > qmax ? oz : qmax;
        qnext = on < qnext ? on : qnext;
    }
    if ((tid & 63) == 0) {
        if (drops) atomicAdd(&s_drop, (unsigned long long)drops);
        if (mask) atomicOr(&s_mask, mask);
        if (qmin != JMAX) atomicMin(&s_qmin, qmin);
        if (qmax != JMIN) atomicMax(&s_qmax, qmax);
        if (qnext != JMAX) atomicMin(&s_qnext, qnext);
    }
    if (p.wide && __ballot(wide) != 0 && (tid & 63) == 0) atomicOr(p.wide, 1u);
    __syncthreads();
    uint32_t lane_part = 0, bmax = 0;
    int lane_of = -1;
    for (int b = tid; b < F; b += T) {
        const uint32_t c = s_hist[b];
        p.hist[(int64_t)blockIdx.x * F + b] = c;
        bmax = c > bmax ? c : bmax;
        const int l = b >> p.region_bits;
        if (l != lane_of) {
            if (lane_part) atomicAdd(&s_lane[lane_of], lane_part);
            lane_of = l;
            lane_part = 0;
        }
        lane_part += c;
    }
    if (lane_part) atomicAdd(&s_lane[lane_of], lane_part);
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t y = __shfl_xor(bmax, off);
        bmax = y > bmax ? y : bmax;
    }
    if ((tid & 63) == 0 && p.max_bucket && bmax) atomicMax(p.max_bucket, bmax);
    __syncthreads();
    if (tid < p.lanes && s_lane[tid]) atomicAdd(&p.lane_total[tid], (unsigned long long)s_lane[tid]);
    if (tid == 0) {
        if (p.count_drops && s_drop) atomicAdd(p.drops, s_drop);
        if (s_mask) atomicOr(p.lane_mask, (unsigned long long)s_mask);
        if (s_qmin != JMAX) atomicMin(p.qmin, s_qmin);
        if (s_qmax != JMIN) atomicMax(p.qmax, s_qmax);
        if (s_qnext != JMAX) atomicMin(p.qnext, s_qnext);
    }
}

// Pass 2: workgroup (active coarse bucket ca, group of K consecutive pass-1 workgroups
// [g0, g0 + K)) gathers the coarse bucket's fragment of every tile of the group, sorts it by
// fine bucket in sub-tiles of kPart2Tile and writes each fine bucket's run at its cursor.
// Within a bucket the staged layout is workgroup-major, so the K workgroups' records of
// bucket b own the one contiguous range starting at the column prefix of g0 (their order
// inside it is immaterial): one cursor per fine bucket serves the whole group.
constexpr int kPart2MaxFrags = 512;    // fragments (group tiles) per unit held in LDS

int32_t part2_group(int32_t max_tiles) {
    int32_t k = kPart2MaxFrags / (max_tiles > 0 ? max_tiles : 1);
    return k < 1 ? 1 : (k > 8 ? 8 : k);
}

template <bool AOS, bool NARROW = false>
__global__ __launch_bounds__(kPart2Threads) void k_part2(IngestParams p, int32_t group) {
    constexpr int NF = 1 << kFineBits;
    constexpr int R = kPart2Tile / kPart2Threads;   // 8
    constexpr int FPT = kPart2MaxFrags / kPart2Threads;   // fragments per thread
    __shared__ longlong2 s_rec[kPart2Tile];          // 32 KiB
    __shared__ uint8_t s_fb[kPart2Tile];             // fine bucket | NULL flag << 7
    __shared__ uint32_t s_fstart[kPart2MaxFrags + 1];  // prefix of fragment lengths
    __shared__ uint32_t s_fsrc[kPart2MaxFrags];        // tmp position of each fragment
    __shared__ uint32_t s_cnt[NF], s_off[NF + 1], s_cur[NF];
    __shared__ uint32_t s_wave[kPart2Threads / 64];
    // u16 fragment of each record of the sub-tile being loaded (4 KiB): aliases s_rec, which
    // is free from the end of one sub-tile's write-out to the staging of the next
    uint4* s_map4 = reinterpret_cast<uint4*>(s_rec);
    uint16_t* s_map = reinterpret_cast<uint16_t*>(s_rec);
    const int tid = threadIdx.x;
    const int P = 1 << p.region_bits;
    const int F = p.lanes << p.region_bits;
    const int NC = p.n_coarse;
    const int MT = p.max_tiles;
    const int cpl = 1 << (p.region_bits - kFineBits);   // coarse buckets per lane
    const int ngroups = (p.grid + group - 1) / group;
    const int gi = blockIdx.x % ngroups;
    const int ca = blockIdx.x / ngroups;
    const int g0 = gi * group;
    const int g1 = g0 + group < p.grid ? g0 + group : p.grid;
    // regular launch: one unit per workgroup, slot ca / cpl; speculative launch (p.plan): one
    // lane's units, each workgroup taking its unit of every lane the plan found active
    int lane = 0;
    uint32_t more = 0;   // further active lanes (speculative launch)
    int64_t lane_shift;
    if (p.plan) {
        if (!gbl(&p.plan->ok)[0]) return;
        more = (uint32_t)gbl(&p.plan->active)[0];
        if (!more) return;
        lane = __ffs(more) - 1;
        more &= more - 1;
        lane_shift = gbl(p.plan->lane_shift)[lane];
    } else {
        const int sl = ca / cpl;
        for (int l = 0; l < kMaxLanes; l++)
            if (p.lane_slot[l] == sl) lane = l;
        lane_shift = p.lane_shift[lane];
    }
    for (;;) {   // (one iteration per lane; the body keeps its original indentation)
    const int cl = ca % cpl;
    const int c = lane * cpl + cl;
    // fragment q = (workgroup g0 + q / MT, tile q % MT); missing tiles are empty fragments
    const int nfr = (g1 - g0) * MT;
    uint32_t len[FPT], fst[FPT];
    uint32_t local = 0;
#pragma unroll
    for (int k = 0; k < FPT; k++) {
        const int q = tid * FPT + k;
        len[k] = 0;
        if (q >= nfr) continue;
        const int g = g0 + q / MT, jt = q % MT;
        int64_t beg, end;
        seg_bounds(p.n, p.grid, g, &beg, &end);
        if (beg + (int64_t)jt * kPart1Tile >= end) continue;
        const uint16_t* drow = p.dir + ((int64_t)g * MT + jt) * (NC + 1);
        const uint32_t a = drow[c], b = drow[c + 1];
        len[k] = b - a;
        s_fsrc[q] = (uint32_t)(beg + (int64_t)jt * kPart1Tile + a);
        local += len[k];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(local, s_wave, &total);
#pragma unroll
    for (int k = 0; k < FPT; k++) {
        const int q = tid * FPT + k;
        if (q < nfr) s_fstart[q] = run;
        fst[k] = run;
        run += len[k];
    }
    if (tid < NF) {
        const int b = lane * P + cl * NF + tid;
        s_cur[tid] = (uint32_t)((int64_t)p.bucket_base[b] + p.hist[(int64_t)g0 * F + b] + lane_shift);
        s_cnt[tid] = 0;
    }
    __syncthreads();
    const bool has_null = p.vnull != nullptr;
    // records of a sub-tile: idx = base + u * T + tid; the next sub-tile's loads are issued
    // before this one is ranked, staged and written. The fragment of each idx comes from a
    // per-sub-tile map: every fragment marks its first record in the sub-tile, and an
    // inclusive max-scan fills the map forward (fragment numbers grow with idx).
    auto build_map = [&](uint32_t base) {
        s_map4[tid] = make_uint4(0u, 0u, 0u, 0u);
        lds_barrier();
#pragma unroll
        for (int k = 0; k < FPT; k++) {
            const int q = tid * FPT + k;
            if (q < nfr && len[k] > 0 && fst[k] < base + kPart2Tile && fst[k] + len[k] > base)
                s_map[fst[k] > base ? fst[k] - base : 0u] = (uint16_t)q;
        }
        lds_barrier();
        const uint4 w = s_map4[tid];
        uint32_t e[8] = {w.x & 0xffffu, w.x >> 16, w.y & 0xffffu, w.y >> 16,
                         w.z & 0xffffu, w.z >> 16, w.w & 0xffffu, w.w >> 16};
#pragma unroll
        for (int j = 1; j < 8; j++) e[j] = e[j] > e[j - 1] ? e[j] : e[j - 1];
        uint32_t x = e[7];
        const int ln = tid & 63;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x, off);
            if (ln >= off) x = x > y ? x : y;
        }
        if (ln == 63) s_wave[tid >> 6] = x;
        uint32_t pre = __shfl_up(x, 1);
        if (ln == 0) pre = 0;
        lds_barrier();
        for (int wv = 0; wv < (tid >> 6); wv++) pre = pre > s_wave[wv] ? pre : s_wave[wv];
#pragma unroll
        for (int j = 0; j < 8; j++) e[j] = e[j] > pre ? e[j] : pre;
        s_map4[tid] = make_uint4(e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16), e[6] | (e[7] << 16));
        lds_barrier();
    };
    // every lane issues all R loads (past the end: record 0, unused) and all R stores (idle
    // lanes into p.sink), and the two record buffers alternate statically (the loop is
    // unrolled by two): the number of memory operations between a prefetch and its use is
    // then the same on every path, so the wait for it leaves the stores in flight
    // NULL flags (rare) are gathered into a bit mask at load time
    auto load = [&](longlong2 (&rr)[R], uint32_t& rn, uint32_t base) {
        rn = 0;
#pragma unroll
        for (int u = 0; u < R; u++) {
            const uint32_t idx = base + (uint32_t)(u * kPart2Threads + tid);
            const bool ok = idx < total;
            const int q = ok ? (int)s_map[idx - base] : 0;
            const uint32_t src = ok ? s_fsrc[q] + (idx - s_fstart[q]) : 0u;
            if constexpr (NARROW) {   // {int32 key, value}: the key sign-extended, its mix recomputed below
                const Rec12 r = ld_rec12(p.tmp, src);
                rr[u] = make_longlong2((long long)(int32_t)r.k, (long long)rec12_val(r));
            } else {
                rr[u] = ld2(&p.tmp[src]);
            }
            if (has_null && p.tmp_null[src] != 0) rn |= 1u << u;
        }
    };
    // sub-tile at `base` (records in cr, NULL bits cn); loads the next one into nr/nn
    // first; cr is reused for the write-out once its records are staged in LDS
    auto step = [&](longlong2 (&cr)[R], const uint32_t cn, longlong2 (&nr)[R], uint32_t& nn, uint32_t base) {
        if (base + kPart2Tile < total) build_map(base + kPart2Tile);
        load(nr, nn, base + kPart2Tile);
        uint32_t rf[R];   // (rank << 6) | fine, 0xffffffff = none
#pragma unroll
        for (int u = 0; u < R; u++) {
            rf[u] = 0xffffffffu;
            if (base + (uint32_t)(u * kPart2Threads + tid) >= total) continue;
            const int64_t mix = NARROW ? mix_of(cr[u].x) : cr[u].x;   // staged mix (narrow: of the key)
            const uint32_t f = (uint32_t)((uint64_t)mix >> (64 - p.region_bits)) & (NF - 1);
            rf[u] = (atomicAdd(&s_cnt[f], 1u) << 6) | f;
        }
        lds_barrier();
        if (tid < 64) {   // one wave: exclusive scan of the 64 fine counts
            const uint32_t v = s_cnt[tid];
            uint32_t x = v;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off);
                if (tid >= off) x += y;
            }
            s_off[tid] = x - v;
            if (tid == 63) s_off[NF] = x;
        }
        lds_barrier();
#pragma unroll
        for (int u = 0; u < R; u++) {
            if (rf[u] == 0xffffffffu) continue;
            const uint32_t slot = s_off[rf[u] & (NF - 1)] + (rf[u] >> 6);
            s_rec[slot] = cr[u];
            s_fb[slot] = (uint8_t)((rf[u] & (NF - 1)) | (((cn >> u) & 1u) << 7));
        }
        lds_barrier();
        // write-out: all of the thread's LDS reads first, then its stores back to back
        const uint32_t sub = s_off[NF];
        uint32_t wfb[R];
        longlong2 (&wv)[R] = cr;
#pragma unroll
        for (int u = 0; u < R; u++) {
            const uint32_t i = (uint32_t)(u * kPart2Threads + tid);
            const bool live = i < sub;
            wfb[u] = live ? (uint32_t)s_fb[i] : 0xffffffffu;
            wv[u] = s_rec[live ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < R; u++) {
            const bool live = wfb[u] != 0xffffffffu;
            const uint32_t i = (uint32_t)(u * kPart2Threads + tid);
            const int f = (int)(wfb[u] & (NF - 1));
            const int64_t pos = live ? (int64_t)(s_cur[f] + (i - s_off[f])) : 0;
            if constexpr (NARROW) {   // 12-B record {int32 key, value}
                st_rec12(live ? (void*)p.st_rec : (void*)p.sink, live ? (uint64_t)pos : 0u, wv[u].x, wv[u].y);
            } else if constexpr (AOS) {
                st2(live ? p.st_rec + 2 * pos : p.sink, wv[u]);
            } else {
                *(live ? p.st_rec + pos : p.sink) = wv[u].x;
            }
        }
        if (has_null) {
#pragma unroll
            for (int u = 0; u < R; u++) {
                const bool live = wfb[u] != 0xffffffffu;
                const uint32_t i = (uint32_t)(u * kPart2Threads + tid);
                const int f = (int)(wfb[u] & (NF - 1));
                uint8_t* dst = live ? p.st_null + (int64_t)(s_cur[f] + (i - s_off[f]))
                                    : reinterpret_cast<uint8_t*>(p.sink);
                *dst = (uint8_t)(wfb[u] >> 7);
            }
        }
        lds_barrier();
        if (tid < NF) {
            s_cur[tid] += s_cnt[tid];
            s_cnt[tid] = 0;
        }
        lds_barrier();
    };
    longlong2 ra[R], rb[R];
    uint32_t na = 0, nb = 0;
    if (total > 0) {
        build_map(0);
        load(ra, na, 0);
        lds_barrier();   // every wave has read the map before build_map(kPart2Tile) clears it
    }
    for (uint32_t base = 0; base < total; base += 2 * kPart2Tile) {
        step(ra, na, rb, nb, base);
        if (base + kPart2Tile >= total) break;
        step(rb, nb, ra, na, base + kPart2Tile);
    }
    if (!more) break;
    lane = __ffs(more) - 1;   // the next active lane's unit (speculative launch)
    more &= more - 1;
    lane_shift = gbl(p.plan->lane_shift)[lane];
    __syncthreads();
    }
}

// The host's lane decision of ingest_pass, restated (pass 1's counters against the lane
// state handed over in pp): ok iff the accepted slices inside the filter span fewer slices
// than lanes and every active lane is empty or holds that slice with room left.
__device__ void ingest_plan(const IngestParams& p, const PlanParams& pp, long long qmin, long long qmax,
                            unsigned long long mask, const unsigned long long* lane_total, IngestPlan* out) {
    int ok = 1;
    if (qmin <= qmax) {
        const long long fq0 = qmin > p.filter_lo ? qmin : p.filter_lo;
        const long long fq1 = qmax < p.filter_hi - 1 ? qmax : p.filter_hi - 1;
        if (fq0 <= fq1) {
            if ((unsigned long long)(fq1 - fq0) >= (unsigned long long)p.lanes) {
                ok = 0;
            } else {
                for (int l = 0; l < p.lanes; l++) {
                    const long long tot = (long long)lane_total[l];
                    if (tot == 0) continue;
                    long long ql = JMAX;   // the lane's slice among [fq0, fq1]
                    for (long long q = fq0; q <= fq1; q++)
                        if ((int)(q & (p.lanes - 1)) == l && ((mask >> l) & 1)) ql = q;
                    if (tot > pp.lane_cap) ok = 0;
                    if (pp.q[l] != JMIN && (pp.q[l] != ql || pp.fill[l] + tot > pp.lane_cap)) ok = 0;
                }
            }
        }
    }
    int64_t before = 0;
    int active = 0;
    for (int l = 0; l < kMaxLanes; l++) {
        out->lane_shift[l] = l < p.lanes ? (int64_t)l * pp.lane_cap + pp.fill[l] - before : 0;
        if (l < p.lanes) before += (int64_t)lane_total[l];
        if (l < p.lanes && lane_total[l] > 0) active |= 1 << l;
    }
    out->active = active;
    out->ok = ok;
}

constexpr int kScanPlanThreads = 1024;
__global__ __launch_bounds__(kScanPlanThreads) void k_scan_plan(IngestParams p, PlanParams pp, ScanPlanArgs a) {
    __shared__ uint32_t s_wave[kScanPlanThreads / 64];
    __shared__ unsigned long long s_words[16];
    const int tid = threadIdx.x;
    // 1) bucket bases: thread t scans a run of consecutive totals (loaded at once)
    constexpr int kPer = kMaxStageBuckets / kScanPlanThreads;
    const int per = (a.F + kScanPlanThreads - 1) / kScanPlanThreads;
    const int b0 = tid * per;
    uint32_t v[kPer];
    uint32_t run = 0;
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        v[j] = (j < per && b0 + j < a.F) ? a.totals[b0 + j] : 0u;
        run += v[j];
    }
    uint32_t total;
    uint32_t ex = block_exclusive_scan(run, s_wave, &total);
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        if (j < per && b0 + j < a.F) a.bucket_off[b0 + j] = ex;
        ex += v[j];
    }
    if (tid == 0) a.bucket_off[a.F] = total;
    // 2) the pass's counters to the host, reset for the next pass; the lane plan
    if (tid < a.n_words) s_words[tid] = a.counters[tid];
    __syncthreads();
    if (tid < a.n_words) {
        a.host[tid] = s_words[tid];
        if (tid < a.reset.n) a.counters[tid] = a.reset.v[tid];
    }
    if (tid == 0 && a.do_plan) {
        // the counter words hold DevCounters (fg_engine.cpp): read through the pass's pointers'
        // offsets into the block
        auto word = [&](const void* q) {
            return s_words[(reinterpret_cast<const char*>(q) - reinterpret_cast<const char*>(a.counters)) / 8];
        };
        const long long qmin = (long long)word(p.qmin), qmax = (long long)word(p.qmax);
        const unsigned long long mask = word(p.lane_mask);
        unsigned long long lt[kMaxLanes];
        for (int l = 0; l < kMaxLanes; l++) lt[l] = word(p.lane_total + l);
        IngestPlan pl;
        ingest_plan(p, pp, qmin, qmax, mask, lt, &pl);
        // a key wider than 32 bits under narrow staging: the host switches to 16-B records
        // (max_bucket and the wide flag share one counter word: max_bucket low, wide high)
        if (p.narrow && (word(p.max_bucket) >> 32) != 0) pl.ok = 0;
        *a.plan = pl;
        IngestPlan* hp = reinterpret_cast<IngestPlan*>(a.host + a.n_words);
        *hp = pl;
    }
    if (tid == 0) {   // the host polls the sequence word (after the counters and the plan)
        __threadfence_system();
        volatile unsigned long long* sq = a.host + a.n_words + sizeof(IngestPlan) / 8;
        *sq = a.seq;
        __threadfence_system();
    }
}

hipError_t launch_scan_plan(const IngestParams& p, const PlanParams& pp, const ScanPlanArgs& a, hipStream_t s) {
    if (a.n_words < 1 || a.n_words > 16 || a.reset.n > a.n_words) return hipErrorInvalidValue;
    fg_launch(k_scan_plan, dim3(1), dim3(kScanPlanThreads), 0, s, p, pp, a);
    return hipGetLastError();
}

int32_t part1_max_tiles(int64_t n, int32_t grid) {
    int64_t per = (n + grid - 1) / grid;
    per = (per + 1) & ~int64_t(1);
    return (int32_t)((per + kPart1Tile - 1) / kPart1Tile);
}

hipError_t launch_part1(const IngestParams& p, hipStream_t s) {
    if (p.n_coarse < 1 || p.n_coarse > kMaxCoarse || (p.lanes << p.region_bits) > kMaxPart1Fine ||
        p.region_bits < kFineBits || p.max_tiles > kPart2MaxFrags)
        return hipErrorInvalidValue;
    fg_launch(k_part1, dim3(p.grid), dim3(kPart1Threads), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_part2(const IngestParams& p, hipStream_t s) {
    int nslots = 0;
    for (int l = 0; l < kMaxLanes; l++) nslots += p.lane_slot[l] >= 0 ? 1 : 0;
    const int32_t group = p.p2_group > 0 ? std::min(p.p2_group, part2_group(p.max_tiles)) : part2_group(p.max_tiles);
    const int64_t units = (int64_t)nslots * (1 << (p.region_bits - kFineBits)) * ((p.grid + group - 1) / group);
    if (units == 0) return hipSuccess;
    if (p.narrow) {
        if (p.st_stride != 2) return hipErrorInvalidValue;
        fg_launch((k_part2<true, true>), dim3((unsigned)units), dim3(kPart2Threads), 0, s, p, group);
    } else if (p.st_stride == 2) {
        fg_launch(k_part2<true>, dim3((unsigned)units), dim3(kPart2Threads), 0, s, p, group);
    } else {
        fg_launch(k_part2<false>, dim3((unsigned)units), dim3(kPart2Threads), 0, s, p, group);
    }
    return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// global phase: partial accumulators (LocalAggCombiner rows) -> per-lane accumulator areas
// ----------------------------------------------------------------------------------------
// A partial row of slice `slice_end` is classified like a record with rowtime
// slice_end - 1 - tz (the `sliced` assigner: assignSliceEnd = the row's window end,
// SliceAssigners.java:494-533), so the late rules of the global operator apply unchanged.
__global__ void k_pseudo_rowtime(const int64_t* slice_end, int64_t n, int64_t tz, int64_t* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = slice_end[i];
        out[i] = e == JMAX ? JMAX : jsub(jsub(e, 1), tz);
    }
}

// Packed BinaryRowData rows (BinaryRowData.java:68-76): the fixed-length part of row i at
// rows + i * stride; field f's null bit is bit 8 + f of the row's leading bit set (:155-157,
// BinarySegmentUtils.bitGet :459-463), its 8 bytes at the bit set's width + 8 f (:119-121).
// One thread per row; the row's 8-byte words are read as aligned 8-B loads.
__global__ void k_rows_to_columns(const uint8_t* rows, int64_t n, RowLayout L, int64_t* key, int64_t* ts,
                                  int64_t* val, uint8_t* vnull, unsigned long long* bad) {
    unsigned long long nbad = 0, nnull = 0;   // rows with a NULL key or rowtime; NULL values
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t* r = rows + i * (int64_t)L.stride;
        auto bit = [&](int b) { return (r[b >> 3] >> (b & 7)) & 1; };
        key[i] = *reinterpret_cast<const int64_t*>(r + L.key_off);
        ts[i] = *reinterpret_cast<const int64_t*>(r + L.ts_off);
        if (bit(L.key_bit) | bit(L.ts_bit)) nbad++;
        if (L.val_off >= 0) {
            val[i] = *reinterpret_cast<const int64_t*>(r + L.val_off);
            const int nl = bit(L.val_bit);
            vnull[i] = (uint8_t)nl;
            nnull += (unsigned long long)nl;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        nbad += __shfl_down(nbad, off);
        nnull += __shfl_down(nnull, off);
    }
    if ((threadIdx.x & 63) == 0 && nbad) atomicAdd(bad, nbad);
    if ((threadIdx.x & 63) == 0 && nnull) atomicAdd(bad + 1, nnull);
}

hipError_t launch_rows_to_columns(const uint8_t* rows, int64_t n, const RowLayout& L, int64_t* key, int64_t* ts,
                                  int64_t* val, uint8_t* vnull, unsigned long long* bad, hipStream_t s) {
    const int64_t blocks = (n + 255) / 256;
    fg_launch(k_rows_to_columns, dim3((unsigned)(blocks < 4096 ? (blocks > 0 ? blocks : 1) : 4096)), dim3(256),
                       0, s, rows, n, L, key, ts, val, vnull, bad);
    return hipGetLastError();
}

// Windowed input (WindowedSliceAssigner): the attached window_end of a row is its slice,
// classified like a record with rowtime window_end - 1 - tz; ends off the inner assigner's
// slice grid are counted (the caller fails loudly on any)
__global__ void k_window_end_rowtime(const int64_t* wend, int64_t n, int64_t tz, int64_t S, int64_t phase,
                                     int64_t* out, unsigned long long* off_grid) {
    unsigned long long bad = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = wend[i];
        int64_t r = jsub(e, phase) % S;
        if (r < 0) r += S;
        bad += (r != 0 || e == JMAX) ? 1ull : 0ull;
        out[i] = jsub(jsub(e, 1), tz);
    }
    if (bad) atomicAdd(off_grid, bad);
}

// narrow FG_HOST columns (fg_batch.format), copied H2D into buffers of their own, widened
// into the batch's 8-byte device columns
__global__ void k_widen_columns(const int32_t* k32, const uint32_t* t32, const int32_t* v32, int64_t n, int64_t tbase,
                                int64_t* key, int64_t* ts, int64_t* val) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (k32) key[i] = (int64_t)k32[i];
    if (t32) ts[i] = (int64_t)((uint64_t)tbase + (uint64_t)t32[i]);   // Java long wrap
    if (v32) val[i] = (int64_t)v32[i];
}
hipError_t launch_widen_columns(const int32_t* k32, const uint32_t* t32, const int32_t* v32, int64_t n, int64_t tbase,
                                int64_t* key, int64_t* ts, int64_t* val, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    fg_launch(k_widen_columns, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, k32, t32, v32, n, tbase,
                       key, ts, val);
    return hipGetLastError();
}

hipError_t launch_window_end_rowtime(const int64_t* wend, int64_t n, int64_t tz, int64_t S, int64_t phase,
                                     int64_t* out, unsigned long long* off_grid, hipStream_t s) {
    int64_t blocks = (n + 255) / 256;
    blocks = blocks > 8192 ? 8192 : (blocks < 1 ? 1 : blocks);
    fg_launch(k_window_end_rowtime, dim3((unsigned)blocks), dim3(256), 0, s, wend, n, tz, S, phase, out, off_grid);
    return hipGetLastError();
}

__global__ void k_store_words(unsigned long long* dst, Words16 w) {
    if ((int)threadIdx.x < w.n) dst[threadIdx.x] = w.v[threadIdx.x];
}

hipError_t launch_store_words(unsigned long long* dst, const Words16& w, hipStream_t s) {
    if (w.n < 0 || w.n > 16) return hipErrorInvalidValue;
    fg_launch(k_store_words, dim3(1), dim3(64), 0, s, dst, w);
    return hipGetLastError();
}

// n device words to coherent host memory, then the sequence word after them: the host polls
// for `seq` instead of synchronizing the stream (no interrupt wake-up, no D2H blit)
__global__ void k_publish_words(const unsigned long long* src, int32_t n, unsigned long long* host,
                                unsigned long long seq) {
    if ((int)threadIdx.x < n) host[threadIdx.x] = src[threadIdx.x];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        *reinterpret_cast<volatile unsigned long long*>(host + n) = seq;
        __threadfence_system();
    }
}

hipError_t launch_publish_words(const unsigned long long* src, int32_t n, unsigned long long* host,
                                unsigned long long seq, hipStream_t s) {
    if (n < 0 || n > 64) return hipErrorInvalidValue;
    fg_launch(k_publish_words, dim3(1), dim3(64), 0, s, src, n, host, seq);
    return hipGetLastError();
}

hipError_t launch_pseudo_rowtime(const int64_t* slice_end, int64_t n, int64_t tz, int64_t* out, hipStream_t s) {
    int64_t blocks = (n + 255) / 256;
    blocks = blocks > 8192 ? 8192 : (blocks < 1 ? 1 : blocks);
    fg_launch(k_pseudo_rowtime, dim3((unsigned)blocks), dim3(256), 0, s, slice_end, n, tz, out);
    return hipGetLastError();
}

// Direct scatter of accumulator rows (key, COUNT(*), NULL count, sum) into the SoA areas
// at their bucket cursors (the count pass's histogram, k_hist_columns, scan).
__global__ __launch_bounds__(kIngestThreads) void k_acc_scatter(IngestParams p, AccColumns a) {
    __shared__ uint32_t s_cur[kMaxStageBuckets];
    const int F = p.lanes << p.region_bits;
    const int tid = threadIdx.x;
    for (int b = tid; b < F; b += kIngestThreads)
        s_cur[b] = (uint32_t)((int64_t)p.bucket_base[b] + p.hist[(int64_t)blockIdx.x * F + b] +
                              p.lane_shift[b >> p.region_bits]);
    __syncthreads();
    int64_t beg, end;
    seg_bounds(p.n, p.grid, blockIdx.x, &beg, &end);
    for (int64_t i = beg + tid; i < end; i += kIngestThreads) {
        const int64_t k = p.key[i];
        int64_t q, h;
        const int b = classify(p, k, p.ts[i], &q, &h);
        if (b < 0) continue;
        const uint32_t pos = atomicAdd(&s_cur[b], 1u);
        const int64_t cs = a.in_cnt_star[i];
        a.key[pos] = h;
        a.cnt_star[pos] = cs;
        a.cnt_null[pos] = cs - a.in_cnt_val[i];
        a.sum[pos] = a.in_sum[i];
        if (a.v1) {
            a.v1[pos] = a.in_v1[i];
            a.v2[pos] = a.in_v2[i];
        }
    }
}

hipError_t launch_acc_scatter(const IngestParams& p, const AccColumns& a, hipStream_t s) {
    fg_launch(k_acc_scatter, dim3(p.grid), dim3(kIngestThreads), 0, s, p, a);
    return hipGetLastError();
}

// per bucket: exclusive prefix over workgroups (column of the workgroup-major histogram)
// 64 buckets per workgroup, four threads per bucket: each sums a quarter of the workgroup
// rows (held in registers), the quarter sums are scanned in LDS, then each thread writes its
// rows' prefixes. F / 64 workgroups keep the chip's memory pipes busy (one thread per bucket
// over all rows left three quarters of the CUs idle and serialized the loads).
constexpr int kHcRows = 64;   // rows per thread held in registers (grid <= 4 * kHcRows)
__global__ __launch_bounds__(256) void k_hist_columns(uint32_t* hist, uint32_t* totals, int32_t F, int32_t grid) {
    __shared__ uint32_t s_q[4][64];
    const int j = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int b = blockIdx.x * 64 + j;
    const int per = (grid + 3) / 4;
    const int g0 = q * per;
    uint32_t v[kHcRows];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kHcRows; k++) {
        const int g = g0 + k;
        v[k] = (b < F && k < per && g < grid) ? hist[(int64_t)g * F + b] : 0u;
        sum += v[k];
    }
    s_q[q][j] = sum;
    __syncthreads();
    uint32_t run = 0;
    for (int k = 0; k < q; k++) run += s_q[k][j];
    if (b >= F) return;
#pragma unroll
    for (int k = 0; k < kHcRows; k++) {
        const int g = g0 + k;
        if (k < per && g < grid) hist[(int64_t)g * F + b] = run;
        run += v[k];
    }
    if (q == 3) totals[b] = run;
}

hipError_t launch_hist_columns(uint32_t* hist, uint32_t* totals, int32_t F, int32_t grid, hipStream_t s) {
    if (grid > 4 * kHcRows) return hipErrorInvalidValue;
    fg_launch(k_hist_columns, dim3((F + 63) / 64), dim3(256), 0, s, hist, totals, F, grid);
    return hipGetLastError();
}

__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const uint32_t* in, int64_t n, uint32_t* sums) {
    __shared__ uint32_t s_wave[16];
    const int64_t base = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * kScanItems;
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; j++) v += (base + j < n) ? in[base + j] : 0u;
    uint32_t total;
    block_exclusive_scan(v, s_wave, &total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_blocks(uint32_t* sums, int64_t nb) {
    __shared__ uint32_t s_wave[16];
    __shared__ uint32_t s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int64_t b0 = 0; b0 < nb; b0 += kScanThreads) {
        const int64_t i = b0 + threadIdx.x;
        uint32_t v = i < nb ? sums[i] : 0u;
        uint32_t total;
        uint32_t ex = block_exclusive_scan(v, s_wave, &total);
        const uint32_t carry = s_carry;
        if (i < nb) sums[i] = carry + ex;
        __syncthreads();
        if (threadIdx.x == 0) s_carry = carry + total;
        __syncthreads();
    }
}

__global__ __launch_bounds__(kScanThreads) void k_scan_final(const uint32_t* in, int64_t n, const uint32_t* sums,
                                                             uint32_t* out) {
    __shared__ uint32_t s_wave[16];
    const int64_t base = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t t = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        v[j] = (base + j < n) ? in[base + j] : 0u;
        t += v[j];
    }
    uint32_t total;
    uint32_t ex = block_exclusive_scan(t, s_wave, &total) + sums[blockIdx.x];
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        if (base + j < n) out[base + j] = ex;
        ex += v[j];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = sums[blockIdx.x] + total;
}

size_t scan_tmp_words(int64_t n) { return (size_t)((n + kScanChunk - 1) / kScanChunk) + 1; }

hipError_t launch_scan_u32(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* tmp, hipStream_t s) {
    const int64_t nb = (n + kScanChunk - 1) / kScanChunk;
    if (nb == 0) return hipMemsetAsync(out, 0, sizeof(uint32_t), s);
    fg_launch(k_scan_reduce, dim3((unsigned)nb), dim3(kScanThreads), 0, s, in, n, tmp);
    fg_launch(k_scan_blocks, dim3(1), dim3(kScanThreads), 0, s, tmp, nb);
    fg_launch(k_scan_final, dim3((unsigned)nb), dim3(kScanThreads), 0, s, in, n, tmp, out);
    return hipGetLastError();
}

hipError_t launch_ingest_count(const IngestParams& p, hipStream_t s) {
    fg_launch(k_ingest_count, dim3(p.grid), dim3(kIngestThreads), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_ingest_scatter(const IngestParams& p, hipStream_t s) {
    int nslots = 0;
    for (int l = 0; l < kMaxLanes; l++) nslots += p.lane_slot[l] >= 0 ? 1 : 0;
    const int FS = nslots << p.region_bits;
    if (p.sorted && FS <= 4 * kIngestThreads)
        fg_launch(k_ingest_scatter_sorted<4>, dim3(p.grid), dim3(kIngestThreads), 0, s, p);
    else if (p.sorted)
        fg_launch(k_ingest_scatter_sorted<kMaxSortedBuckets / kIngestThreads>, dim3(p.grid),
                           dim3(kIngestThreads), 0, s, p);
    else fg_launch(k_ingest_scatter_direct, dim3(p.grid), dim3(kIngestThreads), 0, s, p);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// merge: persistent, one 1024-thread workgroup per CU walking a strided set of regions
// ----------------------------------------------------------------------------------------
// LDS table layouts. Wide: 4,096 slots of {key, COUNT(*) u64, NULL count, sum} (128 KiB,
// one 1,024-thread workgroup per CU) for every merge. Compact: 3,584 slots of {key, sum,
// COUNT(*) u32} (70 KiB, two 512-thread workgroups per CU) for the common fire/flush of
// plain staged records (no NULLs, no resident state, < 2^32 records).
//
// staged-stream chunk of the compact merge: 16-B loads per thread (overridable for experiments)
// staged records per thread per chunk (compact and wide merges; 1, 3 and 4 measured slower,
// DESIGN.md section 9 v10)
constexpr int kMergeRecsPerThread = 2;

template <bool C, bool MV = false>
struct MergeCfg;
template <>
struct MergeCfg<false, false> {
    static constexpr int kSlotsT = kSlots;
    static constexpr int kThreads = kMergeThreads;
    static constexpr int kU = kMergeRecsPerThread;   // 1,024 threads: 128 VGPRs
    static constexpr int kWavesPerEu = 4;
};
template <>
struct MergeCfg<true, false> {
    static constexpr int kSlotsT = kCompactSlots;
    static constexpr int kThreads = kCompactMergeThreads;
    static constexpr int kU = kMergeRecsPerThread;
    static constexpr int kWavesPerEu = kCompactMergeThreads / 128;   // two workgroups per CU
};
template <>
struct MergeCfg<false, true> {   // multi-value: one 1,024-thread workgroup per CU
    static constexpr int kSlotsT = kSlotsMV;
    static constexpr int kThreads = kMergeThreads;
    static constexpr int kU = kMergeRecsPerThread;
    static constexpr int kWavesPerEu = 4;
};
template <>
struct MergeCfg<true, true> {    // multi-value compact: 108 KiB, one 1,024-thread workgroup per CU
    static constexpr int kSlotsT = kCompactSlotsMV;
    static constexpr int kThreads = kMergeThreads;
    static constexpr int kU = kMergeRecsPerThread;
    static constexpr int kWavesPerEu = 4;
};

// v[k][slot]: value slot k (one slot; kNV for a multi-value operator)
template <bool C, bool MV = false>
struct LdsTableT;
template <>
struct LdsTableT<false, false> {
    alignas(16) int64_t key[kSlots + 1];      // slot kSlots: the key equal to the sentinel
    unsigned long long cs[kSlots + 1];        // COUNT(*)
    unsigned long long cn[kSlots + 1];        // records whose value was NULL
    unsigned long long v[1][kSlots + 1];      // SUM / AVG sum (i64, or f64 bits) or MIN / MAX
};
template <>
struct LdsTableT<true, false> {
    alignas(16) int64_t key[kCompactSlots + 1];
    unsigned long long v[1][kCompactSlots + 1];
    uint32_t cs[kCompactSlots + 1];
};
template <>
struct LdsTableT<false, true> {
    alignas(16) int64_t key[kSlotsMV + 1];
    unsigned long long cs[kSlotsMV + 1];
    unsigned long long cn[kSlotsMV + 1];
    unsigned long long v[kNV][kSlotsMV + 1];
};
template <>
struct LdsTableT<true, true> {
    alignas(16) int64_t key[kCompactSlotsMV + 1];
    unsigned long long v[kNV][kCompactSlotsMV + 1];
    uint32_t cs[kCompactSlotsMV + 1];
};
// Narrow compact table (staged 12-B records: keys within 32 bits): the slot holds the key
// itself, so a 4-slot home bucket is ONE 16-B LDS read with an exact compare (the 64-bit mix
// table reads 32 B). Empty = INT32_MIN; the key INT32_MIN takes the sentinel slot. The home
// bucket is still picked by the key's mix (its low word; the region is its top bits).
struct LdsTableN {
    alignas(16) int32_t key[kCompactSlots + 1];
    unsigned long long v[1][kCompactSlots + 1];
    uint32_t cs[kCompactSlots + 1];
};
constexpr int32_t kEmpty32 = INT32_MIN;
// linear probe of the narrow table from `slot` (as lds_find_or_insert_from)
__device__ __forceinline__ int lds_find_or_insert_from32(LdsTableN& t, int32_t k, uint32_t slot, bool& full) {
    constexpr int S = kCompactSlots;
    for (int probe = 0; probe < S; probe++) {
        const int32_t cur = t.key[slot];
        if (cur == k) return (int)slot;
        if (cur == kEmpty32) {
            const int old = atomicCAS(&t.key[slot], kEmpty32, k);
            if (old == kEmpty32 || old == k) return (int)slot;
        }
        slot = slot + 1 == (uint32_t)S ? 0u : slot + 1;
    }
    full = true;
    return -1;
}
// slot of the 32-bit key k in the narrow table given its home bucket's four keys (read
// beforehand): a match, else a CAS on the bucket's first empty slot, else the linear probe
__device__ __forceinline__ int nt_bucket_slot(LdsTableN& t, int32_t k, uint32_t home, int4 b, bool& full) {
    constexpr uint32_t S_ = (uint32_t)kCompactSlots;
    if (k == kEmpty32) return (int)S_;
    const int32_t q[4] = {b.x, b.y, b.z, b.w};
    int hit = -1, empty = -1;
#pragma unroll
    for (int j = 3; j >= 0; j--) {
        if (q[j] == k) hit = j;
        if (q[j] == kEmpty32) empty = j;
    }
    if (hit >= 0 && (empty < 0 || hit < empty)) return (int)home + hit;
    if (empty >= 0) {
        const uint32_t e = home + (uint32_t)empty;
        const int old = atomicCAS(&t.key[e], kEmpty32, k);
        if (old == kEmpty32 || old == k) return (int)e;
        return lds_find_or_insert_from32(t, k, e + 1 >= S_ ? 0u : e + 1, full);
    }
    const uint32_t nx = home + 4;
    return lds_find_or_insert_from32(t, k, nx >= S_ ? 0u : nx, full);
}

// Home bucket: the low 32 bits of the key's mix h (the region is its top bits; the low
// word is independent of them) pick an aligned bucket of kBucket slots -- one 32-bit
// multiply-high, no hashing in the merge -- read with one 32-byte LDS access; probing is
// linear, slot by slot, from the bucket's first slot. At the regions' load factor (<= ~0.35)
// a key sits in its home bucket ~99 % of the time, against ~84 % for a single home slot, so
// a wave's lanes rarely leave the fast path.
// (2-slot buckets, one 16-B read, measured slower: more probes leave the home bucket; odd buckets
// read half-swapped to spread banks measured slower too -- DESIGN.md section 9)
constexpr int kBucket = 4;   // slots per home bucket (two 16-B reads of 64-bit keys)
template <bool C, bool MV>
__device__ __forceinline__ uint32_t lds_home(int64_t h) {
    constexpr uint32_t NB = (uint32_t)(MergeCfg<C, MV>::kSlotsT / kBucket);
    return __umulhi((uint32_t)(uint64_t)h, NB) * kBucket;
}

// linear probe from `slot` (keys never leave the table during a region, so a key is at the
// first slot from its home that was empty or held it when it was inserted)
// The narrow (int32-keyed) LDS table's home bucket: a multiplicative hash of the key itself -- the
// records, narrow entries and wide entries of one merge all reach it from the int32 key, so a narrow
// entry needs no fmix64 of its key (the wide one's stored mix was its home: a 64-bit mix per narrow
// entry made HOP's fires over narrow tables slower than over wide ones, round 5)
template <bool C, bool MV>
__device__ __forceinline__ uint32_t nt_home(int32_t k) {
    constexpr uint32_t NB = (uint32_t)(MergeCfg<C, MV>::kSlotsT / kBucket);
#if defined(FG_NT_HOME_MIX)
    return lds_home<C, MV>(mix_of((int64_t)k));
#else
    return __umulhi((uint32_t)k * 0x9E3779B1u, NB) * kBucket;
#endif
}
template <bool C, bool MV>
__device__ __forceinline__ int lds_find_or_insert_from(LdsTableT<C, MV>& t, int64_t k, uint32_t slot, bool& full) {
    constexpr int S = MergeCfg<C, MV>::kSlotsT;
    for (int probe = 0; probe < S; probe++) {
        const int64_t cur = t.key[slot];
        if (cur == k) return (int)slot;
        if (cur == JMIN) {
            const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long*>(&t.key[slot]),
                                                     (unsigned long long)JMIN, (unsigned long long)k);
            if (old == (unsigned long long)JMIN || old == (unsigned long long)k) return (int)slot;
        }
        slot = slot + 1 == (uint32_t)S ? 0u : slot + 1;
    }
    full = true;
    return -1;
}

template <bool C, bool MV>
__device__ __forceinline__ int lds_find_or_insert(LdsTableT<C, MV>& t, int64_t k, bool& full) {
    if (k == JMIN) return MergeCfg<C, MV>::kSlotsT;
    return lds_find_or_insert_from<C, MV>(t, k, lds_home<C, MV>(k), full);
}

// slot of key k given its home bucket's keys (read beforehand): a match, else a CAS on the
// bucket's first empty slot, else (full bucket / lost CAS) the linear probe
template <bool C, bool MV>
__device__ __forceinline__ int lds_bucket_slot(LdsTableT<C, MV>& t, int64_t k, uint32_t home, RecV2 b01, RecV2 b23,
                                               bool& full) {
    constexpr uint32_t S_ = (uint32_t)MergeCfg<C, MV>::kSlotsT;
    if (k == JMIN) return (int)S_;
    const int64_t q[kBucket] = {b01.x, b01.y, b23.x, b23.y};
    int hit = -1, empty = -1;
#pragma unroll
    for (int j = kBucket - 1; j >= 0; j--) {
        if (q[j] == k) hit = j;
        if (q[j] == JMIN) empty = j;
    }
    if (hit >= 0 && (empty < 0 || hit < empty)) return (int)home + hit;
    if (empty >= 0) {
        const uint32_t e = home + (uint32_t)empty;
        const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long*>(&t.key[e]),
                                                 (unsigned long long)JMIN, (unsigned long long)k);
        if (old == (unsigned long long)JMIN || old == (unsigned long long)k) return (int)e;
        return lds_find_or_insert_from<C, MV>(t, k, e + 1 >= S_ ? 0u : e + 1, full);
    }
    const uint32_t nx = home + kBucket;
    return lds_find_or_insert_from<C, MV>(t, k, nx >= S_ ? 0u : nx, full);
}
// one fired row: key, window bounds, (DataStream) output timestamp and the aggregates of
// the accumulator {COUNT(*), NULL count, sum} (a6: Count1/Count/Sum/AvgAggFunction)
// v: the entry's value slots (one; kNV for a multi-value operator, aggregate a reading slot
// p.agg_slot[a]); vt: the kernel value op (its low bits the value type)
// NT: the row columns stored non-temporally (past L2 and the Infinity Cache). The CUMULATE fold +
// fire (the tile fire with tables) emits ~1.2 rows per record, and cached rows evicted the next
// batch's input and tiles: 52.8-54.8 -> 51.4-52.1 ms per 1B records, its pass 1 0.17 -> 0.15 ms. The
// TUMBLE fire (0.1 row per record: 0.654 vs 0.666 ms with NT) and k_merge's HOP window fires (0.37
// vs 0.38 ms) store as usual (A/B round 6, profiles/r06/ab/r6x, r6z_*)
template <bool NT>
__device__ __forceinline__ void row_st(int64_t& dst, int64_t v) {
    if constexpr (NT) __builtin_nontemporal_store(v, &dst);
    else dst = v;
}
template <bool NT>
__device__ __forceinline__ void row_st(uint8_t& dst, uint8_t v) {
    if constexpr (NT) __builtin_nontemporal_store(v, &dst);
    else dst = v;
}
#define ROW_ST(dst, v) row_st<NT>((dst), (v))
template <bool NT = false>
__device__ __forceinline__ void write_row_k(const MergeParams& p, unsigned long long o, int64_t key,
                                            unsigned long long cs, unsigned long long cn, const int64_t* vals, int vt) {
    ROW_ST(p.out_key[o], key);
    ROW_ST(p.out_ws[o], p.wstart);
    ROW_ST(p.out_we[o], p.wend);
    if (p.out_rowtime) ROW_ST(p.out_rowtime[o], p.out_ts);
    const int64_t cv = (int64_t)(cs - cn);
    uint8_t nm = 0;
#pragma unroll
    for (int a = 0; a < kMaxAggs; a++) {
        if (a >= p.num_aggs) break;
        int64_t v = 0;
        const int64_t sum = vals[p.mv ? p.agg_slot[a] : 0];
        switch (p.aggs[a]) {
            case 0: v = (int64_t)cs; break;   // COUNT(*)
            case 1: v = cv; break;            // COUNT(v)
            case 2:                           // SUM(v): NULL when no non-null value
                if (cv == 0) nm |= (uint8_t)(1u << a);
                else v = sum;
                break;
            case 4: v = sum; break;           // SUM0(v): 0-initialised, never NULL
            case 5:                           // MIN(v) / MAX(v): NULL when no non-null value
            case 6:
                if (cv == 0) nm |= (uint8_t)(1u << a);
                else v = sum;
                break;
            default:                          // AVG(v): count == 0 ? NULL : sum / count
                if (cv == 0) nm |= (uint8_t)(1u << a);
                else if ((vt & 3) == 2) v = __double_as_longlong(__longlong_as_double(sum) / (double)cv);
                else v = sum / cv;
                break;
        }
        ROW_ST(p.out_agg[a][o], v);
    }
    ROW_ST(p.out_null[o], nm);
}
#undef ROW_ST
__device__ __forceinline__ void write_row(const MergeParams& p, unsigned long long o, int64_t h,
                                          unsigned long long cs, unsigned long long cn, const int64_t* vals, int vt) {
    write_row_k(p, o, key_of(h), cs, cn, vals, vt);   // state holds the key's mix
}

// source table j of a merge: by value in the arguments (n_src <= 2) or from the device array
// (static indices into the arguments: a runtime index would copy them to scratch)
__device__ __forceinline__ TableRef src_at(const MergeParams& p, int j) {
    if (p.src) return p.src[j];
    return j == 0 ? p.src_in[0] : p.src_in[1];
}
constexpr int kSrcU = 2;   // source-table entries per thread per round (1, 3, 4 measured +-2 % or slower)
constexpr unsigned long long kMarkBit = 1ull << 63;   // wide table: entry touched by a marking source (NULL-count word)
constexpr int kMaxSrcFlat = 64;   // source tables of one merge (hop: size / slide)

// Value accumulator of an entry (kernel vt = val_type | op << 2; val_type 1 BIGINT, 2 DOUBLE;
// op 0 SUM/AVG/SUM0, 1 MIN, 2 MAX). MIN/MAX restate Min/MaxAggFunction
// (TP/functions/aggfunctions/MinAggFunction.java:61-90, MaxAggFunction.java:61-96):
// the operand replaces the accumulator iff `operand < min` (`>` for MAX), Java primitive
// comparison; a NULL accumulator is the identity (+inf / Long.MAX_VALUE for MIN), and an
// entry without non-null values (COUNT(v) = 0) emits NULL, so the identity is never seen.
// Ops 3 / 4 (DOUBLE only): the DataStream MIN / MAX of ComparableAggregator
// (SJ/api/functions/aggregation/ComparableAggregator.java:83-104 with Comparator.java:48-137),
// which compare by Double.compareTo: a total order in which -0.0 < +0.0 and NaN (every NaN
// canonicalised, as doubleToLongBits does) is above +inf -- MAX picks a NaN, MIN avoids it.
// Their identities are the canonical order's top and bottom: NaN and -inf.
constexpr int kOpShift = 2;
constexpr int kVtMinT = 2 | (3 << kOpShift), kVtMaxT = 2 | (4 << kOpShift);
__device__ __forceinline__ int64_t f64_ord(int64_t b) { return b >= 0 ? b : b ^ 0x7FFFFFFFFFFFFFFFll; }
__device__ __forceinline__ int64_t f64_canon(int64_t b) {   // Double.doubleToLongBits
    return (b & 0x7FFFFFFFFFFFFFFFll) > 0x7FF0000000000000ll ? 0x7FF8000000000000ll : b;
}
__device__ __forceinline__ int64_t val_identity(int vt) {
    switch (vt) {
        case 1 | (1 << kOpShift): return INT64_MAX;
        case 1 | (2 << kOpShift): return JMIN;
        case 2 | (1 << kOpShift): return 0x7FF0000000000000ll;    // +inf
        case 2 | (2 << kOpShift): return (int64_t)0xFFF0000000000000ull;   // -inf
        // the top / bottom of the canonical total order (canonical themselves, so a combine
        // that canonicalises its operands keeps them neutral): NaN, -inf
        case kVtMinT: return 0x7FF8000000000000ll;
        case kVtMaxT: return (int64_t)0xFFF0000000000000ull;
        default: return 0;
    }
}
// a op b (wave pre-reduction of hot keys)
__device__ __forceinline__ int64_t val_combine(int64_t a, int64_t b, int vt) {
    switch (vt) {
        case 1: return (int64_t)((uint64_t)a + (uint64_t)b);
        case 2: return __double_as_longlong(__longlong_as_double(a) + __longlong_as_double(b));
        case 1 | (1 << kOpShift): return b < a ? b : a;
        case 1 | (2 << kOpShift): return b > a ? b : a;
        case 2 | (1 << kOpShift): return __longlong_as_double(b) < __longlong_as_double(a) ? b : a;
        case 2 | (2 << kOpShift): return __longlong_as_double(b) > __longlong_as_double(a) ? b : a;
        case kVtMinT: a = f64_canon(a); b = f64_canon(b); return f64_ord(b) < f64_ord(a) ? b : a;
        case kVtMaxT: a = f64_canon(a); b = f64_canon(b); return f64_ord(b) > f64_ord(a) ? b : a;
        default: return 0;
    }
}
// DOUBLE MIN/MAX in LDS: an LDS slot of a DOUBLE MIN / MAX holds the value's bits mapped to an
// order-preserving int64 (f64_ord: non-negative doubles as they are, negative ones with the
// magnitude bits flipped; an involution), so one ds_min_i64 / ds_max_i64 replaces a
// compare-and-swap loop. The operand replaces the accumulator iff operand < min (> max) as
// Java's primitive comparison, except that a NaN operand never wins (Java keeps a NaN that
// arrived first) and -0.0 < +0.0 (Java keeps whichever zero came first): DESIGN.md section 3.
__device__ __forceinline__ bool is_f64_minmax(int op) {
    return op == (2 | (1 << kOpShift)) || op == (2 | (2 << kOpShift)) || op == kVtMinT || op == kVtMaxT;
}
// the LDS form of a value slot's bits (and back: f64_ord is its own inverse)
__device__ __forceinline__ int64_t lds_repr(int op, int64_t b) { return is_f64_minmax(op) ? f64_ord(b) : b; }
template <bool kMin>
__device__ __forceinline__ void lds_minmax_f64(unsigned long long* a, int64_t bits) {
    if ((bits & 0x7FFFFFFFFFFFFFFFll) > 0x7FF0000000000000ll) return;   // NaN: never wins
    if (kMin) atomicMin(reinterpret_cast<long long*>(a), (long long)f64_ord(bits));
    else atomicMax(reinterpret_cast<long long*>(a), (long long)f64_ord(bits));
}

// one value slot: `bits` into *a with the kernel value op vtk (val_type | op << 2; 0: none).
// MIN / MAX skip an accumulator with COUNT(v) = 0 (it holds no value: has_value false).
__device__ __forceinline__ void lds_val(unsigned long long* a, int64_t bits, int vtk, bool has_value) {
    if (vtk == 2) {
        atomicAdd(reinterpret_cast<double*>(a), __longlong_as_double(bits));
    } else if (vtk == 1) {
        atomicAdd(a, (unsigned long long)bits);
    } else if (vtk > 3 && has_value) {
        switch (vtk) {
            case 1 | (1 << kOpShift): atomicMin(reinterpret_cast<long long*>(a), (long long)bits); break;
            case 1 | (2 << kOpShift): atomicMax(reinterpret_cast<long long*>(a), (long long)bits); break;
            case 2 | (1 << kOpShift): lds_minmax_f64<true>(a, bits); break;
            case 2 | (2 << kOpShift): lds_minmax_f64<false>(a, bits); break;
            case kVtMinT: atomicMin(reinterpret_cast<long long*>(a), (long long)f64_ord(f64_canon(bits))); break;
            case kVtMaxT: atomicMax(reinterpret_cast<long long*>(a), (long long)f64_ord(f64_canon(bits))); break;
            default: break;
        }
    }
}

// Accumulate {COUNT(*), NULL count, values} into a slot. vt: the kernel value op for a
// single-value table; for a multi-value table the value type (0: a NULL record, no value),
// slot k taking op p.vop[k]. vals: one value per slot (a record's value repeated).
template <bool C, bool MV, class PV, class TT>   // PV: MergeParams or HeavyPlan (vop); TT: the LDS table
__device__ __forceinline__ void lds_add(TT& t, int slot, unsigned long long cs, unsigned long long cn,
                                        const int64_t* vals, int vt, const PV& p) {
    if constexpr (C) {
        atomicAdd(&t.cs[slot], (uint32_t)cs);
    } else {
        atomicAdd(&t.cs[slot], cs);
        if (cn) atomicAdd(&t.cn[slot], cn);
    }
    if constexpr (!MV) {
        lds_val(&t.v[0][slot], vals[0], vt, cn < cs);
    } else if (vt) {
#pragma unroll
        for (int k = 0; k < kNV; k++)
            if (p.vop[k] < 3) lds_val(&t.v[k][slot], vals[k], (vt & 3) | (p.vop[k] << kOpShift), cn < cs);
    }
}
// the same with one value for every slot (a staged record)
template <bool C, bool MV, class TT>
__device__ __forceinline__ void lds_add1(TT& t, int slot, unsigned long long cs, unsigned long long cn,
                                         int64_t bits, int vt, const MergeParams& p) {
    const int64_t vals[kNV] = {bits, bits, bits};
    lds_add<C, MV>(t, slot, cs, cn, vals, vt, p);
}


// Pipelined staged stream (every batch plain {key, value} AoS, <= kMaxMergeBatches): the
// workgroup walks its regions r0, r0 + G, ... as one stream of chunks (chunks never span
// batches). Region ranges are loaded two regions ahead into LDS, and the chunk after a
// region's last one -- the next region's first -- is loaded while that region is
// inserted, compacted and emitted, so no region starts on a cold load.
struct MergeCursor {
    int ri;          // region ordinal of this workgroup (region = blockIdx.x + ri * gridDim.x)
    int j;           // batch
    uint32_t i0;     // first record of the chunk (batch-relative)
    uint32_t end;    // end of region ri in batch j
    bool ok;         // settled on a chunk (false: walked past the regions whose ranges are known)
};

// VTC >= 0: the value op compiled in (kernel vt = val_type | op << 2: the LDS adds, identity and
// row arithmetic of that op only -- a small straight-line stream loop); -1: read p.val_type
// N12: the fast stream's records are narrow 12-B {int32 key, value} (every batch stride 3)
template <bool C, int VTC, bool MV = false, bool N12 = false>
// waves_per_eu(4): 128 VGPRs, so two 512-thread compact workgroups (16 waves) fit a CU (8 and 64
// VGPRs for two 1,024-thread ones, FG_COMPACT_T)
__global__ __launch_bounds__((MergeCfg<C, MV>::kThreads)) __attribute__((amdgpu_waves_per_eu(MergeCfg<C, MV>::kWavesPerEu))) void k_merge(MergeParams pa) {
    const MergeParams& p = pa;
    constexpr int S = MergeCfg<C, MV>::kSlotsT;
    constexpr int T = MergeCfg<C, MV>::kThreads;
    constexpr int kWaves = T / 64;
    constexpr int kRounds = (S + T - 1) / T + 1;    // + 1: the sentinel slot (thread 0)
    constexpr int kMergeU = MergeCfg<C, MV>::kU;
    constexpr uint32_t kChunk = kMergeU * T;
    // narrow table: the compact single-value merge over 12-B records keys its LDS table by the
    // 32-bit key (records then travel as {key, value}; the mix is recomputed for the home bucket)
    constexpr bool NT = N12 && C && !MV;
    using Tab = std::conditional_t<NT, LdsTableN, LdsTableT<C, MV>>;
    __shared__ Tab t;
    __shared__ uint32_t s_grp[kRounds * kWaves];   // per (round, wave) row counts -> offsets
    __shared__ uint16_t s_map[S + 1];              // rank -> slot of the region's emitted entries
    __shared__ unsigned int s_flags;
    __shared__ uint32_t s_total;
    __shared__ unsigned long long s_out_base;
    __shared__ const longlong2* s_brec[kMaxMergeBatches];     // fast path: batch record bases
    __shared__ uint32_t s_bfirst[kMaxMergeBatches];            //   and (narrow) their first record
    __shared__ uint32_t s_rng[3][kMaxMergeBatches][2];         // fast path: [ri % 3][batch] = (beg, end)
    __shared__ uint32_t s_soff[kMaxSrcFlat + 1];               // source tables: entry prefix of the region
    __shared__ const int64_t* s_sbase[kMaxSrcFlat];            //   and each table's region base
    __shared__ uint8_t s_snar[kMaxSrcFlat];                     //   and layout (narrow tables)
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    constexpr int cap = MV ? kRegionCapMV : kRegionCap;   // table entries per region
    constexpr int cols = MV ? 3 + kNV : 4;               // 8-byte words per table entry
    constexpr int NVS = MV ? kNV : 1;                    // value slots
    const int vt = VTC >= 0 ? VTC : p.val_type;          // (MV: the value type; slot k has op p.vop[k])
    int64_t vinit[NVS];
    int vops[NVS];   // the op of each value slot (kernel value op form)
#pragma unroll
    for (int k = 0; k < NVS; k++) {
        // MV with VTC >= 0: the slots' ops compiled in as SUM, MIN, MAX (launch_merge)
        vops[k] = MV ? (VTC >= 0 ? (VTC | (k << kOpShift)) : p.vop[k] < 3 ? (vt & 3) | (p.vop[k] << kOpShift) : 0) : vt;
        vinit[k] = val_identity(vops[k]);
    }
    const int P = 1 << p.region_bits;
    const int G = gridDim.x;
    // regions: all P (strided over the grid), the heavy pass's list, or a retry's list
    const int NR = p.region_list ? *gbl(p.n_list) : p.retry_list ? p.n_retry : P;
    const int nreg = ((int)blockIdx.x < NR) ? (NR - 1 - (int)blockIdx.x) / G + 1 : 0;
    auto region_at = [&](int ri) -> int {
        const int x = (int)blockIdx.x + ri * G;
        return p.region_list ? gbl(p.region_list)[x] : p.retry_list ? gbl(p.retry_list)[x] : x;
    };
    // heavy regions are left to the heavy pass (no state read, nothing emitted or written)
    auto skipped = [&](int r) -> bool { return p.heavy != nullptr && gbl(p.heavy)[r] != 0; };
    // the compact merge streams plain staged records, or (a fire of resident slice tables only:
    // HOP windows) reads source tables alone
    const bool fast = C ? p.n_batches > 0 : p.fast_stream != 0;
    const int nb = p.n_batches;

    // fast path state
    auto range_of = [&](int ri, int j, uint32_t& beg, uint32_t& end) {
        const int r = region_at(ri);
        const auto bo = gbl(p.batches[j].bucket_off);
        const uint32_t b0 = bo[0];
        beg = bo[r] - b0;
        end = skipped(r) ? beg : bo[r + 1] - b0;
    };
    // first non-empty chunk at or after (ri, j, i0) within regions <= maxri (whose ranges
    // are in LDS); ri == nreg: stream exhausted
    auto settle = [&](MergeCursor& c, int maxri) {
        c.ok = false;
        while (c.ri < nreg && c.ri <= maxri) {
            const uint32_t* rg = s_rng[c.ri % 3][c.j];
            if (c.i0 < rg[1]) {
                c.end = rg[1];
                c.ok = true;
                return;
            }
            if (++c.j >= nb) {
                c.j = 0;
                if (++c.ri > maxri || c.ri >= nreg) return;   // i0 is set when re-settled
            }
            c.i0 = s_rng[c.ri % 3][c.j][0];
        }
    };
    longlong2 ca[kMergeU], cb[kMergeU];
    auto load = [&](longlong2 (&c)[kMergeU], const MergeCursor& m) {
        // the base comes back from LDS: cast to the global address space so these are
        // global_load_dwordx4 (a flat load is waited for with vmcnt(0) AND lgkmcnt(0),
        // serializing every LDS probe behind the loads in flight)
        if constexpr (N12) {   // 12-B records: the key's mix recomputed from its 32 bits
            const void* rec = wave_uniform(s_brec[m.j]);
            const uint32_t first = __builtin_amdgcn_readfirstlane(s_bfirst[m.j]);
            Rec12 v[kMergeU];
#pragma unroll
            for (int u = 0; u < kMergeU; u++) {
                const uint32_t i = m.i0 + u * T + tid;
                v[u] = ld_rec12(rec, (uint64_t)first + (i < m.end ? i : m.end - 1));
            }
#pragma unroll
            for (int u = 0; u < kMergeU; u++)
                c[u] = make_longlong2(NT ? (int64_t)(int32_t)v[u].k : rec12_mix(v[u]), rec12_val(v[u]));
        } else {
        const GlobalRec rec = (GlobalRec)wave_uniform(s_brec[m.j]);   // the cursor is workgroup-uniform
#pragma unroll
        for (int u = 0; u < kMergeU; u++) {
            const uint32_t i = m.i0 + u * T + tid;
            const RecV2 v = rec[i < m.end ? i : m.end - 1];
            c[u] = make_longlong2(v.x, v.y);
        }
        }
    };
    // The home buckets of the chunk's records are read together. A record whose key is in
    // its bucket (every repeat of a key, nearly always) is added at once; a new key claims
    // the bucket's first empty slot with one CAS; only a full bucket or a lost CAS probes on.
    auto insert = [&](const longlong2 (&c)[kMergeU], const MergeCursor& m, bool& full) {
        uint32_t home[kMergeU];
        RecV2 b01[kMergeU], b23[kMergeU];
        int4 bq[kMergeU];   // narrow table: the home bucket's four keys (one 16-B read)
#pragma unroll
        for (int u = 0; u < kMergeU; u++) {
            if constexpr (NT) {
                home[u] = nt_home<C, MV>((int32_t)c[u].x);
                bq[u] = *reinterpret_cast<const int4*>(&t.key[home[u]]);
            } else {
            home[u] = lds_home<C, MV>(c[u].x);
            const RecV2* kb = reinterpret_cast<const RecV2*>(&t.key[home[u]]);
            b01[u] = kb[0];
            b23[u] = kb[1];
            }
        }
        // Hot keys (Zipf regions below the heavy threshold: one key can fill most of a wave):
        // the wave's records equal to its first lane's key are combined with cross-lane
        // reductions and inserted once, by the first of them, instead of serializing a
        // wave's worth of LDS atomics on one slot. Wave-uniform: every lane takes part.
        uint32_t pcnt[kMergeU];        // records this lane inserts (0: combined into another lane)
        int64_t pval[kMergeU][NVS];    // their combined value per value slot
#pragma unroll
        for (int u = 0; u < kMergeU; u++) {
            const bool valid = m.i0 + u * T + tid < m.end;
            pcnt[u] = valid ? 1u : 0u;
#pragma unroll
            for (int q = 0; q < NVS; q++) pval[u][q] = C ? c[u].y : 0;
            if (C && p.hot_keys) {   // (compact merges only, and only over skewed staging: a
                                     // uniform stream has no equal keys in a wave to combine)
            const int64_t k0 = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)c[u].x) |
                                         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)c[u].x >> 32)) << 32));
            const uint64_t msk = __ballot(valid && c[u].x == k0);
            if (__popcll(msk) > 1) {
                const bool in = (msk >> lane) & 1;
#pragma unroll
                for (int q = 0; q < NVS; q++) {
                    const int op = vops[q];
                    if (op == 0) continue;
                    int64_t x = in ? c[u].y : val_identity(op);
                    for (int off = 32; off > 0; off >>= 1) x = val_combine(x, __shfl_xor(x, off), op);
                    if (in) pval[u][q] = x;   // (the others keep their own value)
                }
                if (in) pcnt[u] = lane == __ffsll((long long)msk) - 1 ? (uint32_t)__popcll(msk) : 0u;
            }
            }
        }
#pragma unroll
        for (int u = 0; u < kMergeU; u++) {
            if (pcnt[u] == 0) continue;
            if constexpr (NT) {   // exact 32-bit keys, one bucket read
                const int slot = nt_bucket_slot(t, (int32_t)c[u].x, home[u], bq[u], full);
                if (slot >= 0) lds_add<C, MV>(t, slot, (unsigned long long)pcnt[u], 0ull, pval[u], vt, p);
            } else {
            const int64_t k = c[u].x;
            const int64_t q[kBucket] = {b01[u].x, b01[u].y, b23[u].x, b23[u].y};
            int hit = -1, empty = -1;
#pragma unroll
            for (int j = kBucket - 1; j >= 0; j--) {   // the first match / first empty slot
                if (q[j] == k) hit = j;
                if (q[j] == JMIN) empty = j;
            }
            constexpr uint32_t S_ = (uint32_t)MergeCfg<C, MV>::kSlotsT;
            int slot;
            if (k == JMIN) {
                slot = (int)S_;
            } else if (hit >= 0 && (empty < 0 || hit < empty)) {
                slot = (int)home[u] + hit;
            } else if (empty >= 0) {   // claim the first empty slot; a lost CAS probes on
                const uint32_t e = home[u] + (uint32_t)empty;
                const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long*>(&t.key[e]),
                                                         (unsigned long long)JMIN, (unsigned long long)k);
                if (old == (unsigned long long)JMIN || old == (unsigned long long)k) slot = (int)e;
                else slot = lds_find_or_insert_from<C, MV>(t, k, e + 1 >= S_ ? 0u : e + 1, full);
            } else {                   // full bucket: probe on from the next one
                const uint32_t nx = home[u] + kBucket;
                slot = lds_find_or_insert_from<C, MV>(t, k, nx >= S_ ? 0u : nx, full);
            }
            if constexpr (MV && VTC >= 0) {   // SUM, MIN, MAX slots, straight-line
                if (slot >= 0) {
                    if constexpr (C) atomicAdd(&t.cs[slot], pcnt[u]);
                    else atomicAdd(&t.cs[slot], 1ull);
#pragma unroll
                    for (int k = 0; k < NVS; k++) lds_val(&t.v[k][slot], C ? pval[u][k] : c[u].y, vops[k], true);
                }
            } else if (slot >= 0) {
                if constexpr (C) lds_add<C, MV>(t, slot, (unsigned long long)pcnt[u], 0ull, pval[u], vt, p);
                else lds_add1<C, MV>(t, slot, 1ull, 0ull, c[u].y, vt, p);
            }
            }
        }
    };
#ifdef FG_STAMPS
    // diagnostic build only: cycles per phase, summed over this workgroup's regions
    unsigned long long st_acc[4] = {0, 0, 0, 0};
    unsigned long long st_prev = __builtin_amdgcn_s_memtime();
#define MSTAMP(i)                                                     \
    do {                                                              \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        st_acc[i] += now_ - st_prev;                                  \
        st_prev = now_;                                               \
    } while (0)
#else
#define MSTAMP(i) \
    do {          \
    } while (0)
#endif
    // one chunk in flight while the current one is inserted. The buffer roles are static
    // (the loop is unrolled by two): selecting a buffer at run time made the compiler copy
    // registers, waiting for the loads in flight. At a region's end the next region's first
    // chunk is in flight in buffer `nbuf`.
    MergeCursor cur{nreg, 0, 0, 0, false};
    int nbuf = 0;
    auto step = [&](const longlong2 (&in)[kMergeU], longlong2 (&next)[kMergeU], int ri, bool& full) -> bool {
        MergeCursor nx = cur;
        nx.i0 += kChunk;
        settle(nx, ri + 1);
        // issued unconditionally (a dummy reload of this chunk past the stream's end): the
        // counter-based wait before the inserts must know these loads are the newest
        load(next, nx.ok ? nx : cur);
        insert(in, cur, full);
        cur = nx;
        return cur.ri == ri && cur.ok;
    };
    if (fast) {
        if (tid < nb) {
            s_brec[tid] = reinterpret_cast<const longlong2*>(p.batches[tid].rec);
            s_bfirst[tid] = (uint32_t)p.batches[tid].rec_first;
        }
        for (int q = tid; q < 2 * nb; q += T) {   // ranges of regions 0 and 1
            const int ri = q / nb, j = q % nb;
            uint32_t beg = 0, end = 0;
            if (ri < nreg) range_of(ri, j, beg, end);
            s_rng[ri][j][0] = beg;
            s_rng[ri][j][1] = end;
        }
        __syncthreads();
        cur = MergeCursor{0, 0, s_rng[0][0][0], 0, false};
        settle(cur, 1);
        if (cur.ok) load(ca, cur);
    }

    for (int ri = 0; ri < nreg; ri++) {
#if !defined(FG_MERGE_HOIST)
        // (the arguments re-read per region, as in the tile fire: hoisted to the kernel's entry they
        // are held -- and spilled -- across the region's loops)
        const MergeParams& p = (&pa)[opaque_zero()];
#endif
        const int r = region_at(ri);
        const bool skip = skipped(r);
        for (int i = tid; i <= S; i += T) {
            if constexpr (NT) t.key[i] = kEmpty32;
            else t.key[i] = JMIN;
            t.cs[i] = 0;
            if constexpr (!C) t.cn[i] = 0;
#pragma unroll
            for (int k = 0; k < NVS; k++) t.v[k][i] = (unsigned long long)lds_repr(vops[k], vinit[k]);
        }
        if (tid == 0) s_flags = 0;
        if ((!C || p.n_src > 0) && tid < 64) {   // source tables: per-region entry counts -> flat prefix
            const int nsrc = p.n_src <= kMaxSrcFlat ? p.n_src : 0;
            const uint32_t v = tid < nsrc ? gbl(src_at(p, tid).counts)[r] : 0u;
            uint32_t x = v;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off);
                if (tid >= off) x += y;
            }
            if (tid < nsrc) {
                s_soff[tid + 1] = x;
                s_sbase[tid] = src_at(p, tid).base + (int64_t)r * cols * cap;
                s_snar[tid] = src_at(p, tid).narrow ? 1 : 0;
            }
            if (tid == 0) s_soff[0] = 0;
        }
        // fast path: ranges of region ri + 2 (written to LDS after this region's inserts)
        uint32_t nbeg = 0, nend = 0;
        if (fast && tid < nb && ri + 2 < nreg) range_of(ri + 2, tid, nbeg, nend);
        lds_barrier();
        bool full = false;

        MSTAMP(0);   // clear + barrier
        // 1) resident slice regions (state) ------------------------------------------
        //    the entries of all source tables form one flat sequence (prefix of the
        //    tables' counts in s_soff), loaded kSrcU per thread at a time and inserted with
        //    the bucketed probe (compact: plain sources only -- no NULL counts, no marks)
        if constexpr (NT) if (p.n_src > 0 && !p.src_narrow) {   // wide sources only (HOP's tables)
            // (a loop of its own: the narrow-aware one below costs the wide case 12 %, round 5 --
            // 0.429 vs 0.384 ms per HOP fire)
            const uint32_t NE = skip ? 0u : s_soff[p.n_src];
            for (uint32_t i0 = 0; i0 < NE; i0 += kSrcU * T) {
                int64_t k[kSrcU], cs[kSrcU], sm[kSrcU][1];
                int j = 0;
                {
                    const uint32_t f = i0 + tid;
                    int lo = 0, hi = p.n_src;
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (s_soff[mid] <= f) lo = mid;
                        else hi = mid;
                    }
                    j = lo;
                }
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    const uint32_t f = i0 + u * T + tid;
                    k[u] = 0;
                    cs[u] = 0;
                    sm[u][0] = 0;
                    if (f >= NE) continue;
                    while (s_soff[j + 1] <= f) j++;
                    const uint32_t i = f - s_soff[j];
                    const auto base = gbl(s_sbase[j]);
                    k[u] = base[i];
                    cs[u] = base[cap + i];
                    sm[u][0] = base[3 * cap + i];
                }
                uint32_t home[kSrcU];
                int4 bq[kSrcU];
                int32_t k32[kSrcU];   // (the operator's keys fit 32 bits: the mix's key is its int32 sign-extended)
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    k32[u] = (int32_t)key_of(k[u]);
                    home[u] = nt_home<C, MV>(k32[u]);
                    bq[u] = *reinterpret_cast<const int4*>(&t.key[home[u]]);
                }
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    if (i0 + u * T + tid >= NE) continue;
                    const int slot = nt_bucket_slot(t, k32[u], home[u], bq[u], full);
                    if (slot >= 0 && cs[u]) lds_add<C, MV>(t, slot, (unsigned long long)cs[u], 0ull, sm[u], vt, p);
                }
            }
        }
        if constexpr (NT) if (p.n_src > 0 && p.src_narrow == 2) {   // every source narrow (HOP's slice tables)
            // (a loop of its own: the entry's three columns loaded at clamped indices, no per-entry
            // layout test; the layout-aware loop below made HOP's fires over narrow tables slower
            // than over wide ones)
            const uint32_t NE = skip ? 0u : s_soff[p.n_src];
            for (uint32_t i0 = 0; i0 < NE; i0 += kSrcU * T) {
                int32_t k32[kSrcU];
                uint32_t cs[kSrcU];
                int64_t sm[kSrcU][1];
                int j = 0;
                {   // (the clamped index, as below: past NE the search would land on an empty last table,
                    // whose first entry lies past the clamped index)
                    const uint32_t f = i0 + tid < NE ? i0 + tid : NE - 1;
                    int lo = 0, hi = p.n_src;
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (s_soff[mid] <= f) lo = mid;
                        else hi = mid;
                    }
                    j = lo;
                }
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    const uint32_t f0 = i0 + u * T + tid;
                    const uint32_t f = f0 < NE ? f0 : NE - 1;   // (clamped: every load issued)
                    while (s_soff[j + 1] <= f) j++;
                    const uint32_t i = f - s_soff[j];
                    const auto base = gbl(s_sbase[j]);
                    k32[u] = reinterpret_cast<const int32_t __attribute__((address_space(1)))*>(base)[i];
                    cs[u] = reinterpret_cast<const uint32_t __attribute__((address_space(1)))*>(base)[cap + i];
                    sm[u][0] = base[cap + i];
                }
                uint32_t home[kSrcU];
                int4 bq[kSrcU];
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    home[u] = nt_home<C, MV>(k32[u]);
                    bq[u] = *reinterpret_cast<const int4*>(&t.key[home[u]]);
                }
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    if (i0 + u * T + tid >= NE) continue;
                    const int slot = nt_bucket_slot(t, k32[u], home[u], bq[u], full);
                    if (slot >= 0 && cs[u]) lds_add<C, MV>(t, slot, (unsigned long long)cs[u], 0ull, sm[u], vt, p);
                }
            }
        }
        if constexpr (NT) if (p.n_src > 0 && p.src_narrow == 1) {   // narrow and wide tables: per entry
            const uint32_t NE = skip ? 0u : s_soff[p.n_src];   // (compact: n_src <= kMaxSrcFlat)
            for (uint32_t i0 = 0; i0 < NE; i0 += kSrcU * T) {
                int64_t k[kSrcU], cs[kSrcU], sm[kSrcU][1];
                int32_t k32[kSrcU];   // (the int32 key: loaded from a narrow table, the mix's from a wide one)
                int j = 0;
                {
                    const uint32_t f = i0 + tid;
                    int lo = 0, hi = p.n_src;
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (s_soff[mid] <= f) lo = mid;
                        else hi = mid;
                    }
                    j = lo;
                }
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    const uint32_t f = i0 + u * T + tid;
                    k[u] = 0;
                    k32[u] = 0;
                    cs[u] = 0;
                    sm[u][0] = 0;
                    if (f >= NE) continue;
                    while (s_soff[j + 1] <= f) j++;
                    const uint32_t i = f - s_soff[j];
                    const auto base = gbl(s_sbase[j]);
                    const bool nar = s_snar[j] != 0;
                    if (nar) {
                        k32[u] = tab_key32(base, cap, i, true);
                    } else {   // (the operator's keys fit 32 bits: the mix's key is its int32 sign-extended)
                        k32[u] = (int32_t)key_of(base[i]);
                    }
                    cs[u] = tab_cs(base, cap, i, nar);
                    sm[u][0] = tab_v(base, cap, i, nar);
                }
                uint32_t home[kSrcU];
                int4 bq[kSrcU];
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    home[u] = nt_home<C, MV>(k32[u]);
                    bq[u] = *reinterpret_cast<const int4*>(&t.key[home[u]]);
                }
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    if (i0 + u * T + tid >= NE) continue;
                    const int slot = nt_bucket_slot(t, k32[u], home[u], bq[u], full);
                    if (slot >= 0 && cs[u]) lds_add<C, MV>(t, slot, (unsigned long long)cs[u], 0ull, sm[u], vt, p);
                }
            }
        }
        if constexpr (!NT) if (!C || p.n_src > 0) {
            const uint32_t NT = skip ? 0u : s_soff[p.n_src <= kMaxSrcFlat ? p.n_src : 0];
            for (uint32_t i0 = 0; i0 < NT; i0 += kSrcU * T) {
                int64_t k[kSrcU], cs[kSrcU], cn[kSrcU], sm[kSrcU][NVS];
                int j = 0;
                {   // table of this thread's first entry (binary search), later ones advance
                    const uint32_t f = i0 + tid;
                    int lo = 0, hi = p.n_src;
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (s_soff[mid] <= f) lo = mid;
                        else hi = mid;
                    }
                    j = lo;
                }
                bool mk[kSrcU];
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    const uint32_t f = i0 + u * T + tid;
                    k[u] = JMIN;
                    mk[u] = false;
                    if (f >= NT) continue;
                    while (s_soff[j + 1] <= f) j++;
                    const uint32_t i = f - s_soff[j];
                    const auto base = gbl(s_sbase[j]);
                    const bool nar = s_snar[j] != 0;   // (narrow: one value slot, no NULL counts)
                    k[u] = tab_mix(base, cap, i, nar);
                    cs[u] = tab_cs(base, cap, i, nar);
                    cn[u] = ((p.src_null_mask >> j) & 1ull) ? tab_cn(base, cap, i, nar) : 0;
#pragma unroll
                    for (int q = 0; q < NVS; q++) sm[u][q] = tab_v(base, cap, i, nar, q);
                    mk[u] = ((p.mark_mask >> j) & 1ull) != 0;
                    if ((p.markonly_mask >> j) & 1ull) cs[u] = 0;   // a mark-only source adds nothing
                }
                uint32_t home[kSrcU];
                RecV2 b01[kSrcU], b23[kSrcU];
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    home[u] = lds_home<C, MV>(k[u]);
                    const RecV2* kb = reinterpret_cast<const RecV2*>(&t.key[home[u]]);
                    b01[u] = kb[0];
                    b23[u] = kBucket == 4 ? kb[1] : b01[u];
                }
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    if (i0 + u * T + tid >= NT) continue;
                    const int slot = lds_bucket_slot<C, MV>(t, k[u], home[u], b01[u], b23[u], full);
                    if (slot < 0) continue;
                    // (a zero accumulator -- a chain table's key -- adds nothing, only its mark)
                    if (cs[u]) lds_add<C, MV>(t, slot, (unsigned long long)cs[u], (unsigned long long)cn[u], sm[u], vt, p);
                    if constexpr (!C) if (mk[u]) atomicOr(&t.cn[slot], kMarkBit);
                }
            }
            for (int j = 0; !skip && p.n_src > kMaxSrcFlat && j < p.n_src; j++) {   // many tables: one by one
                const TableRef src = src_at(p, j);
                const uint32_t n = gbl(src.counts)[r];
                const auto base = gbl(src.base + (int64_t)r * cols * cap);
                const bool nar = src.narrow != 0;
                const bool mkj = j < 64 && ((p.mark_mask >> j) & 1ull) != 0;
                const bool moj = j < 64 && ((p.markonly_mask >> j) & 1ull) != 0;
                for (uint32_t i = tid; i < n; i += T) {
                    const int slot = lds_find_or_insert<C, MV>(t, tab_mix(base, cap, i, nar), full);
                    if (slot < 0) continue;
                    const int64_t csi = tab_cs(base, cap, i, nar);
                    if (csi && !moj) {
                        int64_t vv[NVS];
#pragma unroll
                        for (int q = 0; q < NVS; q++) vv[q] = tab_v(base, cap, i, nar, q);
                        lds_add<C, MV>(t, slot, (unsigned long long)csi, (unsigned long long)tab_cn(base, cap, i, nar),
                                       vv, vt, p);
                    }
                    if constexpr (!C) if (mkj) atomicOr(&t.cn[slot], kMarkBit);
                }
            }
        }
        // 2) staged records of region r over the lane's staged batches ------------------
        if (fast) {
            if (cur.ri == ri && !cur.ok) {   // walked past empty regions: settle now (cold load)
                cur.j = 0;
                cur.i0 = s_rng[ri % 3][0][0];
                settle(cur, ri + 1);
                nbuf = 0;
                // (the chunk is loaded even when it lies in region ri + 1 -- this region empty:
                // region ri + 1 then streams from buffer ca without another settle. Loading it
                // only for region ri left ca holding an earlier region's records, which region
                // ri + 1 inserted in place of its first chunk: rows lost, rows with foreign keys
                // -- found in round 4 with sparse regions, FG_MIN_REGION_BITS=10/12)
                if (cur.ok) load(ca, cur);
            }
            bool go = cur.ri == ri && cur.ok;
            if (go && nbuf == 1) {
                go = step(cb, ca, ri, full);
                nbuf = 0;
            }
            while (go) {
                go = step(ca, cb, ri, full);
                if (!go) {
                    nbuf = 1;
                    break;
                }
                go = step(cb, ca, ri, full);
            }
        } else if constexpr (!C) {
            if (p.region_list) {   // heavy pass: the partial tables of the region's chunks
                const int li = (int)blockIdx.x + ri * G;
                const int c0 = gbl(p.chunk0)[li], c1 = gbl(p.chunk0)[li + 1];
                for (int c = c0; c < c1; c++) {
                    const uint32_t n = gbl(p.part_n)[c];
                    if (n == kChunkFailed) {   // the chunk's table overflowed: the region fails
                        full = true;
                        continue;
                    }
                    const int64_t at = (int64_t)c * kPartStride;
                    for (uint32_t i = tid; i < n; i += T) {
                        const int slot = lds_find_or_insert<C, MV>(t, gbl(p.part_key)[at + i], full);
                        if (slot < 0) continue;
                        int64_t vv[NVS];
                        vv[0] = gbl(p.part_sum)[at + i];
                        if constexpr (MV) {
                            vv[1] = gbl(p.part_v1)[at + i];
                            vv[2] = gbl(p.part_v2)[at + i];
                        }
                        lds_add<C, MV>(t, slot, (unsigned long long)gbl(p.part_cs)[at + i],
                                       (unsigned long long)gbl(p.part_cn)[at + i], vv, vt, p);
                    }
                }
            }
            for (int j = 0; !skip && j < nb; j++) {
                const StagedBatch sb = p.batches[j];
                const auto bo = gbl(sb.bucket_off);
                const uint32_t b0 = bo[0];
                // a batch staged before the regions split: its bucket r >> shift holds region
                // r's records among its siblings' (keys are staged as their mix, whose top
                // region_bits are the region)
                const int sh = sb.shift;
                const uint32_t beg = bo[r >> sh] - b0;
                const uint32_t end = bo[(r >> sh) + 1] - b0;
                auto mine = [&](int64_t h) { return sh == 0 || (int)((uint64_t)h >> (64 - p.region_bits)) == r; };
                const auto srec = gbl(sb.rec);
                const auto vnull = sb.vnull != nullptr ? gbl(sb.vnull) : nullptr;
                if (sb.is_acc) {
                    const auto cst = gbl(sb.cnt_star), cnl = gbl(sb.cnt_null), sval = gbl(sb.val);
                    for (uint32_t i = beg + tid; i < end; i += T) {
                        if (!mine(srec[i])) continue;
                        const int slot = lds_find_or_insert<C, MV>(t, srec[i], full);
                        if (slot < 0) continue;
                        int64_t vv[NVS];
                        vv[0] = sval[i];
                        if constexpr (MV) {
                            vv[1] = gbl(sb.val1)[i];
                            vv[2] = gbl(sb.val2)[i];
                        }
                        lds_add<C, MV>(t, slot, (unsigned long long)cst[i], (unsigned long long)cnl[i], vv, vt, p);
                    }
                } else if (sb.stride == 2) {
                    const GlobalRec rec = (GlobalRec)sb.rec;
                    for (uint32_t i = beg + tid; i < end; i += T) {
                        const RecV2 rc = rec[i];
                        if (!mine(rc.x)) continue;
                        const int slot = lds_find_or_insert<C, MV>(t, rc.x, full);
                        if (slot < 0) continue;
                        const bool isnull = vnull != nullptr && vnull[i] != 0;
                        lds_add1<C, MV>(t, slot, 1ull, isnull ? 1ull : 0ull, isnull ? 0 : rc.y, isnull ? 0 : vt, p);
                    }
                } else if (sb.stride == 3) {   // narrow 12-B records
                    for (uint32_t i = beg + tid; i < end; i += T) {
                        const Rec12 rc = ld_rec12(sb.rec, (uint64_t)sb.rec_first + i);
                        const int64_t k = rec12_mix(rc);
                        if (!mine(k)) continue;
                        const int slot = lds_find_or_insert<C, MV>(t, k, full);
                        if (slot < 0) continue;
                        const bool isnull = vnull != nullptr && vnull[i] != 0;
                        lds_add1<C, MV>(t, slot, 1ull, isnull ? 1ull : 0ull, isnull ? 0 : rec12_val(rc), isnull ? 0 : vt, p);
                    }
                } else {
                    for (uint32_t i = beg + tid; i < end; i += T) {
                        if (!mine(srec[i])) continue;
                        const int slot = lds_find_or_insert<C, MV>(t, srec[i], full);
                        if (slot < 0) continue;
                        const bool isnull = vnull != nullptr && vnull[i];
                        lds_add1<C, MV>(t, slot, 1ull, isnull ? 1ull : 0ull, 0, 0, p);
                    }
                }
            }
        }
        MSTAMP(1);   // staged stream (this wave's share)
        if (full) atomicOr(&s_flags, 4u);
        if (fast && tid < nb && ri + 2 < nreg) {
            s_rng[(ri + 2) % 3][tid][0] = nbeg;
            s_rng[(ri + 2) % 3][tid][1] = nend;
        }
        lds_barrier();

        // 3) compaction: round k covers slots [k*T, (k+1)*T) (round kRounds-1: the
        //    sentinel slot, thread 0); rows of one (round, wave) are consecutive lanes, so the
        //    row stores of a wave are contiguous
        uint64_t occ_mask = 0;   // bit k: this thread's slot of round k is occupied
        // occupied: holds state (COUNT(*) > 0); marked modes (restore re-fire): marked and
        // holding state, or marked at all for a chain table of every marked key
        const int omode = C ? 0 : (p.dst_mode == 2 ? 2 : (p.dst_mode == 1 || p.emit_marked) ? 1 : 0);
#pragma unroll
        for (int k = 0; k < kRounds; k++) {
            const int slot = k < kRounds - 1 ? k * T + tid : S;
            bool occ = (k < kRounds - 1 ? slot < S : tid == 0);
            if (occ) {
                bool marked = false;
                if constexpr (!C) marked = (t.cn[slot] & kMarkBit) != 0;
                occ = omode == 2 ? marked : (t.cs[slot] != 0 && (omode == 0 || marked));
            }
            const uint64_t bal = __ballot(occ);
            if (occ) occ_mask |= 1ull << k;
            if (lane == 0) s_grp[k * kWaves + wave] = (uint32_t)__popcll(bal);
        }
        lds_barrier();
        if (wave == 0) {   // exclusive scan of the kRounds * kWaves group counts (<= 128)
            constexpr int NG = kRounds * kWaves;
            const uint32_t a = 2 * lane < NG ? s_grp[2 * lane] : 0u;
            const uint32_t b = 2 * lane + 1 < NG ? s_grp[2 * lane + 1] : 0u;
            uint32_t x = a + b;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off);
                if (lane >= off) x += y;
            }
            const uint32_t ex = x - a - b;
            if (2 * lane < NG) s_grp[2 * lane] = ex;
            if (2 * lane + 1 < NG) s_grp[2 * lane + 1] = ex + a;
            const uint32_t total = __shfl(x, 63);
            if (lane == 0) {
                unsigned int fl = s_flags;
                if (p.has_dst && total > (uint32_t)cap) fl |= 1u;
                if (p.emit && !(fl & 5u)) {   // (a failed region reserves no rows)
                    const unsigned long long ob = atomicAdd(p.out_count, (unsigned long long)total);
                    s_out_base = ob;
                    if ((int64_t)(ob + total) > p.out_cap) fl |= 2u;
                }
                s_flags = fl;
                s_total = total;
                if (fl) atomicOr(p.overflow, fl);
                if ((fl & 5u) && p.fail_list) {   // the region does nothing; the host redoes it split
                    const uint32_t at = atomicAdd(p.fail_n, 1u);
                    if (at < (uint32_t)p.fail_cap) p.fail_list[at] = ((uint32_t)p.job << kFailJobShift) | (uint32_t)r;
                }
            }
        }
        lds_barrier();
        MSTAMP(2);   // compaction + scan + barriers
        const unsigned int fl = s_flags;
        const bool write_dst = !skip && p.has_dst && !(fl & 5u);
        const bool write_out = p.emit && !(fl & 7u);
        int64_t* dbase = p.has_dst ? p.dst.base + (int64_t)r * cols * cap : nullptr;
        const unsigned long long obase = s_out_base;
        // one entry out: its table write-back and / or its fired row, at rank `at`
        auto emit_one = [&](int slot, uint32_t at) {
            // (the state's form of the key: its mix; a narrow table holds the key itself)
            const int64_t key = NT ? mix_of(slot == S ? (int64_t)kEmpty32 : (int64_t)t.key[slot])
                                   : slot == S ? JMIN : (int64_t)t.key[slot];
            unsigned long long cs = t.cs[slot], cn = 0;
            if constexpr (!C) cn = t.cn[slot] & ~kMarkBit;
            int64_t vv[NVS];
#pragma unroll
            for (int q = 0; q < NVS; q++) vv[q] = lds_repr(vops[q], (int64_t)t.v[q][slot]);
            if (write_dst) {
                const bool chain = !C && p.dst_mode != 0;   // a chain table holds keys with zero accumulators
                dbase[at] = key;
                dbase[cap + at] = chain ? 0 : (int64_t)cs;
                dbase[2 * cap + at] = chain ? 0 : (int64_t)cn;
#pragma unroll
                for (int q = 0; q < NVS; q++) dbase[(3 + q) * cap + at] = chain ? vinit[q] : vv[q];
            }
            if (write_out) write_row(p, obase + at, key, cs, cn, vv, vt);
        };
        // per round: the wave's occupied lanes below this lane give the rank within the group
        // the ranks are gathered into a rank -> slot map first, then every lane writes one
        // entry at consecutive ranks (full-width stores instead of the ~1/3 of a wave that a
        // round's occupied lanes fill)
#pragma unroll
        for (int k = 0; k < kRounds; k++) {
            const bool occ = (occ_mask >> k) & 1;
            const uint64_t bal = __ballot(occ);
            if (!occ) continue;
            const int slot = k < kRounds - 1 ? k * T + tid : S;
            s_map[s_grp[k * kWaves + wave] + (uint32_t)__popcll(bal & ((1ull << lane) - 1))] = (uint16_t)slot;
        }
        lds_barrier();
        if (write_dst || write_out) {
            const uint32_t total = s_total;
            for (uint32_t i = tid; i < total; i += T) emit_one(s_map[i], i);
        }
        if (tid == 0 && write_dst) {
            const uint32_t total = s_total;
            const uint32_t old = p.dst.counts[r];
            p.dst.counts[r] = total;
            if (p.dst_total) atomicAdd(p.dst_total, (unsigned long long)((int64_t)total - (int64_t)old));
        }
        lds_barrier();   // the table is cleared for the next region
        MSTAMP(3);   // emit + barrier
    }
#ifdef FG_STAMPS
    if (p.stamps && (tid & 63) == 0)
        for (int i = 0; i < 4; i++) atomicAdd(&p.stamps[i], st_acc[i]);
#endif
}

// Fire straight from one slice table (a window whose state is a single table and is not
// written back: tumble windows flushed before their fire, cumulate windows re-fired with
// no new step slice, hop windows of one slice): no LDS combine, one row per entry.
constexpr int kEmitThreads = 256;
__global__ __launch_bounds__(kEmitThreads) void k_emit_table(MergeParams p, TableRef t) {
    __shared__ unsigned long long s_base;
    const int r = blockIdx.x;
    const uint32_t n = gbl(t.counts)[r];
    if (n == 0) return;
    if (threadIdx.x == 0) {
        const unsigned long long b = atomicAdd(p.out_count, (unsigned long long)n);
        s_base = b;
        if ((int64_t)(b + n) > p.out_cap) atomicOr(p.overflow, 2u);
    }
    __syncthreads();
    const unsigned long long b = s_base;
    if ((int64_t)(b + n) > p.out_cap) return;
    const int cap = table_cap(p.mv);
    const auto base = gbl(t.base + (int64_t)r * table_cols(p.mv) * cap);
    const bool nar = t.narrow != 0;
    for (uint32_t i = threadIdx.x; i < n; i += kEmitThreads) {
        int64_t vv[kNV];
        for (int q = 0; q < (p.mv ? kNV : 1); q++) vv[q] = tab_v(base, cap, i, nar, q);
        write_row(p, b + i, tab_mix(base, cap, i, nar), (unsigned long long)tab_cs(base, cap, i, nar),
                  (unsigned long long)tab_cn(base, cap, i, nar), vv, p.val_type);
    }
}

hipError_t launch_emit_table(const MergeParams& p, const TableRef& t, hipStream_t s) {
    fg_launch(k_emit_table, dim3(1u << p.region_bits), dim3(kEmitThreads), 0, s, p, t);
    return hipGetLastError();
}

hipError_t launch_merge(const MergeParams& p, int32_t workgroups, hipStream_t s) {
    if (p.mv) {   // multi-value operator
        if (p.compact) {
            if (!p.fast_stream || p.n_src != 0) return hipErrorInvalidValue;
            // the common list (SUM family, MIN and MAX) over BIGINT / DOUBLE: ops compiled in
            const bool all3 = p.vop[0] == 0 && p.vop[1] == 1 && p.vop[2] == 2;
            constexpr int MT = MergeCfg<true, true>::kThreads;
            if (all3 && p.val_type == 2) fg_launch((k_merge<true, 2, true>), dim3(workgroups), dim3(MT), 0, s, p);
            else if (all3 && p.val_type == 1) fg_launch((k_merge<true, 1, true>), dim3(workgroups), dim3(MT), 0, s, p);
            else fg_launch((k_merge<true, -1, true>), dim3(workgroups), dim3(MT), 0, s, p);
        } else {
            fg_launch((k_merge<false, -1, true>), dim3(workgroups), dim3(kMergeThreads), 0, s, p);
        }
        return hipGetLastError();
    }
    // narrow 12-B staged records (a compact merge of resident sources alone: narrow keys, p.narrow)
    const bool n12 = p.narrow && (p.fast_stream || (p.compact && p.n_batches == 0));
    if (p.compact) {
        // staged records alone, or plain source tables alone (no NULL counts, marks, chains or
        // destination: a HOP window's fire)
        // staged records and / or plain source tables (no NULL counts, marks or chains)
        const bool plain_src = !p.mark_mask && !p.markonly_mask && !p.src_null_mask && !p.dst_mode && !p.emit_marked &&
                               p.n_src <= kMaxSrcFlat && (p.n_batches == 0 || p.fast_stream);
        if (p.n_src == 0 ? !p.fast_stream : !plain_src) return hipErrorInvalidValue;
        // the compact merge (the TUMBLE fire of plain staged records) per value op
        if (n12) {
            switch (p.val_type) {
                case 1: fg_launch((k_merge<true, 1, false, true>), dim3(workgroups), dim3(kCompactMergeThreads), 0, s, p); break;
                case 2: fg_launch((k_merge<true, 2, false, true>), dim3(workgroups), dim3(kCompactMergeThreads), 0, s, p); break;
                default: fg_launch((k_merge<true, -1, false, true>), dim3(workgroups), dim3(kCompactMergeThreads), 0, s, p); break;
            }
            return hipGetLastError();
        }
        switch (p.val_type) {
            case 0: fg_launch((k_merge<true, 0>), dim3(workgroups), dim3(kCompactMergeThreads), 0, s, p); break;
            case 1: fg_launch((k_merge<true, 1>), dim3(workgroups), dim3(kCompactMergeThreads), 0, s, p); break;
            case 2: fg_launch((k_merge<true, 2>), dim3(workgroups), dim3(kCompactMergeThreads), 0, s, p); break;
            default: fg_launch((k_merge<true, -1>), dim3(workgroups), dim3(kCompactMergeThreads), 0, s, p); break;
        }
    } else if (n12) {
        fg_launch((k_merge<false, -1, false, true>), dim3(workgroups), dim3(kMergeThreads), 0, s, p);
    } else {
        fg_launch((k_merge<false, -1>), dim3(workgroups), dim3(kMergeThreads), 0, s, p);
    }
    return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// skewed regions (hot keys): plan, chunk tables; the heavy pass is k_merge with a region list
// ----------------------------------------------------------------------------------------
constexpr int kPlanThreads = 1024;
constexpr int kPlanPer = (1 << 13) / kPlanThreads;   // regions per thread (P <= 8192)

// One workgroup: staged records per region over the batches; regions above the threshold
// are listed with ceil(records / chunk) chunks each. A plan that would exceed max_chunks
// lists nothing (every region then takes the regular merge: slower, same result).
__global__ __launch_bounds__(kPlanThreads) void k_heavy_plan(HeavyPlan hp) {
    __shared__ uint32_t s_wave[kPlanThreads / 64];
    const int tid = threadIdx.x;
    const int P = 1 << hp.region_bits;
    int64_t size[kPlanPer];
    uint32_t nh = 0, nc = 0;
#pragma unroll
    for (int k = 0; k < kPlanPer; k++) {
        const int r = tid * kPlanPer + k;
        size[k] = 0;
        if (r >= P) continue;
        for (int j = 0; j < hp.n_batches; j++) {
            const auto bo = gbl(hp.batches[j].bucket_off);
            size[k] += (int64_t)(bo[r + 1] - bo[r]);
        }
        if (size[k] > hp.threshold) {
            nh++;
            nc += (uint32_t)((size[k] + hp.chunk - 1) / hp.chunk);
        }
    }
    uint32_t tot_h, tot_c;
    const uint32_t hbase = block_exclusive_scan(nh, s_wave, &tot_h);
    const uint32_t cbase = block_exclusive_scan(nc, s_wave, &tot_c);
    const bool ok = tot_c <= (uint32_t)hp.max_chunks;
    uint32_t hi = hbase, ci = cbase;
#pragma unroll
    for (int k = 0; k < kPlanPer; k++) {
        const int r = tid * kPlanPer + k;
        if (r >= P) continue;
        const bool heavy = ok && size[k] > hp.threshold;
        hp.heavy[r] = heavy ? 1 : 0;
        if (!heavy) continue;
        hp.region_list[hi] = r;
        hp.chunk0[hi] = (int32_t)ci;
        for (int64_t v = 0; v < size[k]; v += hp.chunk) {
            hp.chunk_list[ci] = (int32_t)hi;
            hp.chunk_v0[ci] = v;
            hp.chunk_v1[ci] = v + hp.chunk < size[k] ? v + hp.chunk : size[k];
            ci++;
        }
        hi++;
    }
    if (tid == 0) {
        hp.n_list[0] = ok ? (int32_t)tot_h : 0;
        hp.n_list[1] = ok ? (int32_t)tot_c : 0;
        hp.chunk0[ok ? tot_h : 0] = ok ? (int32_t)tot_c : 0;
    }
}

// Persistent over the chunks: each chunk's records (its slice of the region's records,
// batches in order) are combined in a wide LDS table and the table is written out as the
// chunk's partial rows {key, COUNT(*), NULL count, value slots}. Equal keys within a wave (the
// hot key of a Zipf region fills most lanes) are reduced with cross-lane adds (min / max) first,
// so the LDS atomics of a hot slot drop from one per record to one per wave. MV: a multi-value
// operator's table (kNV value slots, slot k folding with op vop[k]).
template <bool MV>
__global__ __launch_bounds__(kMergeThreads) void k_heavy_chunks(HeavyPlan hp) {
    constexpr int T = kMergeThreads;
    constexpr int S = MergeCfg<false, MV>::kSlotsT;
    constexpr int NVS = MV ? kNV : 1;
    __shared__ LdsTableT<false, MV> t;
    __shared__ uint32_t s_n;
    __shared__ unsigned int s_full;
    const int tid = threadIdx.x, lane = tid & 63;
    const int vt = hp.val_type;   // MV: the value type; else the kernel value op
    int vops[NVS];                // the op of each slot (kernel value op form)
    int64_t vinit[NVS];
#pragma unroll
    for (int k = 0; k < NVS; k++) {
        vops[k] = MV ? (hp.vop[k] < 3 ? (vt & 3) | (hp.vop[k] << kOpShift) : 0) : vt;
        vinit[k] = val_identity(vops[k]);
    }
    const int nch = *gbl(hp.n_list + 1);
    for (int c = blockIdx.x; c < nch; c += gridDim.x) {
        for (int i = tid; i <= S; i += T) {
            t.key[i] = JMIN;
            t.cs[i] = 0;
            t.cn[i] = 0;
#pragma unroll
            for (int k = 0; k < NVS; k++) t.v[k][i] = (unsigned long long)lds_repr(vops[k], vinit[k]);
        }
        if (tid == 0) {
            s_n = 0;
            s_full = 0;
        }
        lds_barrier();
        bool full = false;
        const int r = gbl(hp.region_list)[gbl(hp.chunk_list)[c]];
        const int64_t v0 = gbl(hp.chunk_v0)[c], v1 = gbl(hp.chunk_v1)[c];
        int64_t acc = 0;
        for (int j = 0; j < hp.n_batches && acc < v1; j++) {
            const StagedBatch sb = hp.batches[j];
            const auto bo = gbl(sb.bucket_off);
            const int64_t beg = (int64_t)(bo[r] - bo[0]);
            const int64_t len = (int64_t)(bo[r + 1] - bo[r]);
            const int64_t lo = acc > v0 ? acc : v0;
            const int64_t hi = acc + len < v1 ? acc + len : v1;
            for (int64_t xb = lo; xb < hi; xb += T) {   // wave-uniform trip count
                const int64_t x = xb + tid;
                const bool valid = x < hi;
                const int64_t i = beg + (x - acc);
                int64_t k = JMIN;
                int64_t vals[NVS];
#pragma unroll
                for (int q = 0; q < NVS; q++) vals[q] = 0;
                unsigned long long cs = 1, cn = 0;
                if (valid) {
                    if (sb.is_acc) {
                        k = gbl(sb.rec)[i];
                        cs = (unsigned long long)gbl(sb.cnt_star)[i];
                        cn = (unsigned long long)gbl(sb.cnt_null)[i];
                        vals[0] = gbl(sb.val)[i];
                        if constexpr (MV) {
                            vals[1] = gbl(sb.val1)[i];
                            vals[2] = gbl(sb.val2)[i];
                        }
                    } else if (sb.stride == 2) {
                        const RecV2 rc = ((GlobalRec)sb.rec)[i];
                        k = rc.x;
#pragma unroll
                        for (int q = 0; q < NVS; q++) vals[q] = rc.y;
                    } else if (sb.stride == 3) {   // narrow 12-B records
                        const Rec12 rc = ld_rec12(sb.rec, (uint64_t)sb.rec_first + (uint64_t)i);
                        k = rec12_mix(rc);
#pragma unroll
                        for (int q = 0; q < NVS; q++) vals[q] = rec12_val(rc);
                    } else {
                        k = gbl(sb.rec)[i];
                    }
                    if (!sb.is_acc && sb.vnull != nullptr && gbl(sb.vnull)[i] != 0) {
                        cn = 1;
#pragma unroll
                        for (int q = 0; q < NVS; q++) vals[q] = 0;
                    }
                }
                // a record without a value column or a NULL record adds no value
                const bool novalue = !sb.is_acc && (sb.stride < 2 || cn == 1);
                // wave pre-reduction of the records equal to the first lane's key (no NULLs)
                bool done = !valid;
                const int64_t k0 = __builtin_amdgcn_readfirstlane(k);
                const uint64_t m = __ballot(valid && cn == 0 && k == k0 && !sb.is_acc);
                if (__popcll(m) > 1) {
                    const bool in = (m >> lane) & 1;
                    int64_t part[NVS];
#pragma unroll
                    for (int q = 0; q < NVS; q++) {
                        const int op = vops[q];
                        part[q] = in && sb.stride >= 2 ? vals[q] : vinit[q];
                        if (op == 2) {
                            double d = __longlong_as_double(part[q]);
                            for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off);
                            part[q] = __double_as_longlong(d);
                        } else if (op != 0) {
                            for (int off = 32; off > 0; off >>= 1) part[q] = val_combine(part[q], __shfl_xor(part[q], off), op);
                        }
                    }
                    if (in) {
                        done = true;
                        if (lane == __ffsll((long long)m) - 1) {
                            const int slot = lds_find_or_insert<false, MV>(t, k0, full);
                            if (slot >= 0)
                                lds_add<false, MV>(t, slot, (unsigned long long)__popcll(m), 0ull, part,
                                                   sb.stride >= 2 ? vt : 0, hp);
                        }
                    }
                }
                if (!done) {
                    const int slot = lds_find_or_insert<false, MV>(t, k, full);
                    if (slot >= 0) lds_add<false, MV>(t, slot, cs, cn, vals, novalue ? 0 : vt, hp);
                }
            }
            acc += len;
        }
        if (full) atomicOr(&s_full, 1u);
        lds_barrier();
        const int64_t at = (int64_t)c * kPartStride;
        for (int i = tid; i <= S; i += T) {
            if (t.cs[i] == 0) continue;
            const uint32_t o = atomicAdd(&s_n, 1u);
            hp.part_key[at + o] = i == S ? JMIN : t.key[i];
            hp.part_cs[at + o] = (int64_t)t.cs[i];
            hp.part_cn[at + o] = (int64_t)t.cn[i];
            hp.part_sum[at + o] = lds_repr(vops[0], (int64_t)t.v[0][i]);
            if constexpr (MV) {
                hp.part_v1[at + o] = lds_repr(vops[1], (int64_t)t.v[1][i]);
                hp.part_v2[at + o] = lds_repr(vops[2], (int64_t)t.v[2][i]);
            }
        }
        lds_barrier();
        if (tid == 0) {
            // an overflowed chunk fails its region in the heavy pass (which then redoes it split)
            hp.part_n[c] = s_full ? kChunkFailed : s_n;
            if (s_full) atomicOr(hp.overflow, 4u);
        }
        lds_barrier();   // the table is cleared for the next chunk
    }
}

hipError_t launch_heavy_plan(const HeavyPlan& hp, hipStream_t s) {
    if (hp.region_bits > 13 || hp.n_batches < 1 || hp.chunk < 1) return hipErrorInvalidValue;
    fg_launch(k_heavy_plan, dim3(1), dim3(kPlanThreads), 0, s, hp);
    return hipGetLastError();
}

hipError_t launch_heavy_chunks(const HeavyPlan& hp, int32_t workgroups, hipStream_t s) {
    if (hp.mv) fg_launch(k_heavy_chunks<true>, dim3(workgroups), dim3(kMergeThreads), 0, s, hp);
    else fg_launch(k_heavy_chunks<false>, dim3(workgroups), dim3(kMergeThreads), 0, s, hp);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// export (checkpoint image)
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_export(ExportParams p) {
    const int r = blockIdx.x;
    const uint32_t n = p.t.counts[r];
    const int cap = table_cap(p.mv);
    const auto base = gbl(p.t.base + (int64_t)r * table_cols(p.mv) * cap);
    const bool nar = p.t.narrow != 0;
    const uint64_t o = p.region_off[r];
    for (uint32_t i = threadIdx.x; i < n; i += 256) {
        const int64_t cs = tab_cs(base, cap, i, nar), cn = tab_cn(base, cap, i, nar);
        p.out_key[o + i] = nar ? (int64_t)tab_key32(base, cap, i, nar) : key_of(base[i]);
        p.out_slice[o + i] = p.slice_end;
        p.out_cnt_star[o + i] = cs;
        p.out_cnt_val[o + i] = cs - cn;
        p.out_sum[o + i] = tab_v(base, cap, i, nar);
        if (p.mv) {
            p.out_v1[o + i] = base[4 * cap + i];
            p.out_v2[o + i] = base[5 * cap + i];
        }
    }
}

hipError_t launch_export(const ExportParams& p, int32_t regions, hipStream_t s) {
    fg_launch(k_export, dim3(regions), dim3(256), 0, s, p);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// region split (capacity growth): one workgroup per old region appends each entry to the
// child region named by the next `shift` bits of its key mix (a child holds a subset of its
// parent, so it never exceeds kRegionCap); entry order inside a region is irrelevant (the
// merge rebuilds its LDS table from the entries)
// ----------------------------------------------------------------------------------------
constexpr int kSplitThreads = 256;
__global__ __launch_bounds__(kSplitThreads) void k_split_table(TableRef src, TableRef dst, int32_t old_bits,
                                                               int32_t shift, int32_t mv) {
    __shared__ uint32_t s_cnt[1 << 13];
    const int r = blockIdx.x;
    const int nch = 1 << shift;
    const int new_bits = old_bits + shift;
    for (int c = threadIdx.x; c < nch; c += kSplitThreads) s_cnt[c] = 0;
    __syncthreads();
    const uint32_t n = gbl(src.counts)[r];
    const int cap = table_cap(mv), cols = table_cols(mv);
    const auto sb = gbl(src.base + (int64_t)r * cols * cap);
    for (uint32_t i = threadIdx.x; i < n; i += kSplitThreads) {
        const int64_t h = sb[i];
        const int c = (int)(((uint64_t)h >> (64 - new_bits)) & (uint64_t)(nch - 1));
        const uint32_t at = atomicAdd(&s_cnt[c], 1u);
        int64_t* db = dst.base + ((int64_t)r * nch + c) * cols * cap;
        for (int w = 0; w < cols; w++) db[w * cap + at] = sb[w * cap + i];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < nch; c += kSplitThreads) dst.counts[(int64_t)r * nch + c] = s_cnt[c];
}

// A narrow table widened in place (a writer that writes the wide layout -- the general merge --
// or a region split): one workgroup per region reads its entries (the narrow block is the first
// half of the wide one), then writes them wide.
constexpr int kWidenThreads = 1024;
__global__ __launch_bounds__(kWidenThreads) void k_widen_table(TableRef t) {
    constexpr int PER = (kRegionCap + kWidenThreads - 1) / kWidenThreads;
    const int r = blockIdx.x;
    constexpr int cap = kRegionCap;
    const uint32_t n = gbl(t.counts)[r];
    int64_t* b = t.base + (int64_t)r * 4 * cap;
    int32_t k[PER];
    int64_t cs[PER], v[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const uint32_t i = threadIdx.x + q * kWidenThreads;
        if (i < n) {
            k[q] = tab_key32(gbl(b), cap, i, true);
            cs[q] = tab_cs(gbl(b), cap, i, true);
            v[q] = tab_v(gbl(b), cap, i, true);
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const uint32_t i = threadIdx.x + q * kWidenThreads;
        if (i < n) {
            b[i] = mix_of((int64_t)k[q]);
            b[cap + i] = cs[q];
            b[2 * cap + i] = 0;
            b[3 * cap + i] = v[q];
        }
    }
}

hipError_t launch_widen_table(const TableRef& t, int32_t bits, hipStream_t s) {
    if (!t.narrow || bits < 0 || bits > 13) return hipErrorInvalidValue;
    fg_launch(k_widen_table, dim3(1u << bits), dim3(kWidenThreads), 0, s, t);
    return hipGetLastError();
}

hipError_t launch_split_table(const TableRef& src, const TableRef& dst, int32_t old_bits, int32_t shift, int32_t mv,
                              hipStream_t s) {
    if (shift < 1 || old_bits < 0 || old_bits + shift > 13 || src.narrow || dst.narrow) return hipErrorInvalidValue;
    fg_launch(k_split_table, dim3(1u << old_bits), dim3(kSplitThreads), 0, s, src, dst, old_bits, shift, mv);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// key groups and owner partitioning (keyBy exchange)
// ----------------------------------------------------------------------------------------
__global__ void k_key_groups(const int64_t* key, int64_t n, int32_t key_hash, int32_t max_p, int32_t* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = key_group_of(key[i], key_hash, max_p);
}

hipError_t launch_key_groups(const int64_t* key, int64_t n, int32_t key_hash, int32_t max_p, int32_t* out,
                             hipStream_t s) {
    int64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    fg_launch(k_key_groups, dim3((unsigned)blocks), dim3(256), 0, s, key, n, key_hash, max_p, out);
    return hipGetLastError();
}

constexpr int kOwnerGrid = 512;
constexpr int kOwnerThreads = 256;
constexpr int kMaxOwners = 1024;

__device__ __forceinline__ int owner_of(int64_t key, int32_t key_hash, int32_t max_p, int32_t par) {
    return key_group_of(key, key_hash, max_p) * par / max_p;   // computeOperatorIndexForKeyGroup
}

__global__ __launch_bounds__(kOwnerThreads) void k_owner_count(const int64_t* key, int64_t n, int32_t key_hash,
                                                                int32_t max_p, int32_t par, uint32_t* hist) {
    __shared__ uint32_t s[kMaxOwners];
    for (int i = threadIdx.x; i < par; i += kOwnerThreads) s[i] = 0;
    __syncthreads();
    int64_t beg, end;
    seg_bounds(n, kOwnerGrid, blockIdx.x, &beg, &end);
    for (int64_t i = beg + threadIdx.x; i < end; i += kOwnerThreads) atomicAdd(&s[owner_of(key[i], key_hash, max_p, par)], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < par; i += kOwnerThreads) hist[(int64_t)i * kOwnerGrid + blockIdx.x] = s[i];
}

__global__ __launch_bounds__(kOwnerThreads) void k_owner_scatter(const int64_t* key, const int64_t* ts,
                                                                  const int64_t* val, int64_t n, int32_t key_hash,
                                                                  int32_t max_p, int32_t par, const uint32_t* offsets,
                                                                  int64_t* ok, int64_t* ot, int64_t* ov) {
    __shared__ uint32_t s[kMaxOwners];
    for (int i = threadIdx.x; i < par; i += kOwnerThreads) s[i] = offsets[(int64_t)i * kOwnerGrid + blockIdx.x];
    __syncthreads();
    int64_t beg, end;
    seg_bounds(n, kOwnerGrid, blockIdx.x, &beg, &end);
    for (int64_t i = beg + threadIdx.x; i < end; i += kOwnerThreads) {
        const int64_t k = key[i];
        const uint32_t pos = atomicAdd(&s[owner_of(k, key_hash, max_p, par)], 1u);
        ok[pos] = k;
        ot[pos] = ts[i];
        if (val) ov[pos] = val[i];
    }
}

// generic form for the partial-accumulator exchange: up to kMaxOwnerCols int64 columns
// (key first) moved together by destination subtask
__global__ __launch_bounds__(kOwnerThreads) void k_owner_scatter_cols(OwnerCols c, int64_t n, int32_t key_hash,
                                                                       int32_t max_p, int32_t par,
                                                                       const uint32_t* offsets) {
    __shared__ uint32_t s[kMaxOwners];
    for (int i = threadIdx.x; i < par; i += kOwnerThreads) s[i] = offsets[(int64_t)i * kOwnerGrid + blockIdx.x];
    __syncthreads();
    int64_t beg, end;
    seg_bounds(n, kOwnerGrid, blockIdx.x, &beg, &end);
    for (int64_t i = beg + threadIdx.x; i < end; i += kOwnerThreads) {
        const int64_t k = c.in[0][i];
        const uint32_t pos = atomicAdd(&s[owner_of(k, key_hash, max_p, par)], 1u);
        for (int j = 0; j < c.ncols; j++) c.out[j][pos] = c.in[j][i];
    }
}

__global__ void k_owner_counts(const uint32_t* offsets, int32_t par, int64_t* counts) {
    const int i = threadIdx.x;
    if (i < par) counts[i] = (int64_t)offsets[(int64_t)(i + 1) * kOwnerGrid] - (int64_t)offsets[(int64_t)i * kOwnerGrid];
}

hipError_t launch_partition_cols_by_owner(const OwnerCols& c, int64_t n, int32_t key_hash, int32_t max_p,
                                          int32_t par, int64_t* counts, uint32_t* scratch, size_t scratch_words,
                                          hipStream_t s) {
    if (par < 1 || par > kMaxOwners || c.ncols < 1 || c.ncols > kMaxOwnerCols ||
        scratch_words < partition_scratch_words(n, par))
        return hipErrorInvalidValue;
    const int64_t m = (int64_t)par * kOwnerGrid;
    uint32_t* hist = scratch;
    uint32_t* offs = scratch + m;
    uint32_t* tmp = scratch + 2 * m + 1;
    fg_launch(k_owner_count, dim3(kOwnerGrid), dim3(kOwnerThreads), 0, s, c.in[0], n, key_hash, max_p, par,
                       hist);
    hipError_t e = launch_scan_u32(hist, offs, m, tmp, s);
    if (e != hipSuccess) return e;
    fg_launch(k_owner_scatter_cols, dim3(kOwnerGrid), dim3(kOwnerThreads), 0, s, c, n, key_hash, max_p, par,
                       offs);
    fg_launch(k_owner_counts, dim3(1), dim3(kMaxOwners), 0, s, offs, par, counts);
    return hipGetLastError();
}

size_t partition_scratch_words(int64_t n, int32_t par) {
    const int64_t m = (int64_t)par * kOwnerGrid;
    return (size_t)(2 * m + 1) + scan_tmp_words(m);
}

hipError_t launch_partition_by_owner(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n,
                                     int32_t key_hash, int32_t max_p, int32_t par, int64_t* out_key,
                                     int64_t* out_ts, int64_t* out_val, int64_t* counts, uint32_t* scratch,
                                     size_t scratch_words, hipStream_t s) {
    if (par < 1 || par > kMaxOwners || scratch_words < partition_scratch_words(n, par)) return hipErrorInvalidValue;
    const int64_t m = (int64_t)par * kOwnerGrid;
    uint32_t* hist = scratch;
    uint32_t* offs = scratch + m;
    uint32_t* tmp = scratch + 2 * m + 1;
    fg_launch(k_owner_count, dim3(kOwnerGrid), dim3(kOwnerThreads), 0, s, key, n, key_hash, max_p, par, hist);
    hipError_t e = launch_scan_u32(hist, offs, m, tmp, s);
    if (e != hipSuccess) return e;
    fg_launch(k_owner_scatter, dim3(kOwnerGrid), dim3(kOwnerThreads), 0, s, key, ts, val, n, key_hash, max_p,
                       par, offs, out_key, out_ts, out_val);
    fg_launch(k_owner_counts, dim3(1), dim3(kMaxOwners), 0, s, offs, par, counts);
    return hipGetLastError();
}


// ----------------------------------------------------------------------------------------
// tile staging (fg_kernels.h): pass 1 by consumer bucket, directory transpose, fire straight
// from the tiles, and the conversion of a tile pass into a regular staged pass
// ----------------------------------------------------------------------------------------
// Pass 1 of a tile-staged batch: k_part1's bookkeeping (slice assignment with the late rules,
// drops, slice range, lane totals, the 32-bit key check) and a sort of each tile by consumer
// bucket (lane << (region_bits - kTileBits) | region >> kTileBits), written back in place as
// block-laid 12-B records at their absolute batch index, with the tile's bucket offsets in
// p.dir (rows of kTileDirStride u16). A tile is kTileH halves of R records per thread: the
// second half's keys and rowtimes are loaded while the first is classified, the values are read
// once the tile's ranks are known (straight into the sorted tile), and the next tile's first
// half is prefetched across the write-out -- so a tile holds twice the records the registers of
// one classification round allow, and the fire reads half as many fragments. Bucket counts are
// u16 pairs in one LDS word (ds_add_u32 of 1 << 16 * (b & 1): a tile has < 2^16 records).
// *p.max_bucket: the largest bucket count of one tile (skew).
__global__ __launch_bounds__(kTileThreads) void k_tile_part1(IngestParams p) {
    constexpr int T = kTileThreads;
    constexpr int R = kTileR;
    constexpr int H = kTileH;
    constexpr int HALF = T * R;
    constexpr int TILE = kTileRecs;
    static_assert(R % 2 == 0 && H >= 1 && H <= 2 && TILE == H * HALF, "tile shape");
    static_assert(TILE < (1 << 16) && kMaxTileBuckets <= (1 << 12), "u16 counts and offsets; rank << 12 | bucket");
    __shared__ uint32_t s_k[TILE];                       // the tile, bucket sorted: keys
    __shared__ unsigned long long s_v[TILE];             //   and value bits
    __shared__ uint32_t s_cw[kMaxTileBuckets / 2 + 1];   // bucket counts, then offsets (u16 pairs); [NC/2] total
    __shared__ uint32_t s_wave[T / 64];
    __shared__ unsigned long long s_drop;
    __shared__ long long s_qmin, s_qmax, s_qnext;
    __shared__ uint32_t s_mask, s_bmax;
    __shared__ uint32_t s_lane[kMaxLanes];
    const int NC = p.n_coarse;   // (even: >= 16 buckets)
    const int NW = NC / 2;
    const int tid = threadIdx.x;
    for (int i = tid; i <= NW; i += T) s_cw[i] = 0;
    if (tid == 0) { s_drop = 0; s_qmin = JMAX; s_qmax = JMIN; s_qnext = JMAX; s_mask = 0; s_bmax = 0; }
    if (p.tile_btot && blockIdx.x == 0)
        for (int i = tid; i < NC; i += T) p.tile_btot[i] = 0u;
    if (tid < kMaxLanes) s_lane[tid] = 0;
    __syncthreads();
    // whole-tile segments (the host trims the grid): tile j of this workgroup is tile
    // blockIdx.x * max_tiles + j of the pass and starts at record (that tile) * TILE
    const int64_t seg = (int64_t)p.max_tiles * TILE;
    const int64_t beg = (int64_t)blockIdx.x * seg < p.n ? (int64_t)blockIdx.x * seg : p.n;
    const int64_t end = beg + seg < p.n ? beg + seg : p.n;
    const bool has_val = p.val != nullptr;
    uint32_t drops = 0, mask = 0, bmax = 0;
    uint32_t lc[kMaxLanes] = {0u, 0u, 0u, 0u};
    bool wide = false;
    long long qmin = JMAX, qmax = JMIN, qnext = JMAX;
    const int lm = p.lanes - 1;
    const int pw = (NW + T - 1) / T;   // count words per thread in the scan
    auto li_of = [&](int u) -> int64_t { return 2 * ((int64_t)tid + (int64_t)(u >> 1) * T) + (u & 1); };
    // keys and rowtimes of the half at h0 (classification)
    auto load = [&](int64_t h0, longlong2 (&k2)[R / 2], longlong2 (&t2)[R / 2]) {
        const int64_t hn = end - h0 < HALF ? end - h0 : HALF;
        if (hn == HALF && p.vec) {
#pragma unroll
            for (int u = 0; u < R / 2; u++) {
                const int64_t i = h0 + li_of(2 * u);
                k2[u] = ld2(p.key + i);
                t2[u] = ld2(p.ts + i);
            }
        } else {
#pragma unroll
            for (int u = 0; u < R / 2; u++) {
                const int64_t l0 = li_of(2 * u);
                k2[u] = t2[u] = make_longlong2(0, 0);
                if (l0 < hn) {
                    k2[u].x = p.key[h0 + l0];
                    t2[u].x = p.ts[h0 + l0];
                }
                if (l0 + 1 < hn) {
                    k2[u].y = p.key[h0 + l0 + 1];
                    t2[u].y = p.ts[h0 + l0 + 1];
                }
            }
        }
    };
    auto load_vals = [&](int64_t h0, longlong2 (&v2)[R / 2]) {
        const int64_t hn = end - h0 < HALF ? end - h0 : HALF;
        if (hn == HALF && p.vec && has_val) {
#pragma unroll
            for (int u = 0; u < R / 2; u++) v2[u] = ld2(p.val + h0 + li_of(2 * u));
        } else {
#pragma unroll
            for (int u = 0; u < R / 2; u++) {
                const int64_t l0 = li_of(2 * u);
                v2[u] = make_longlong2(0, 0);
                if (has_val && l0 < hn) v2[u].x = p.val[h0 + l0];
                if (has_val && l0 + 1 < hn) v2[u].y = p.val[h0 + l0 + 1];
            }
        }
    };
    // classify + rank the half's records by bucket (LDS atomics on the u16 pairs)
    auto classify_half = [&](int64_t h0, const longlong2 (&k2)[R / 2], const longlong2 (&t2)[R / 2],
                             uint32_t (&rcb)[R], uint32_t (&k32)[R]) {
        const int64_t hn = end - h0 < HALF ? end - h0 : HALF;
#pragma unroll
        for (int u = 0; u < R; u++) {
            const int64_t li = li_of(u);
            rcb[u] = 0xffffffffu;
            const int64_t k = (u & 1) ? k2[u >> 1].y : k2[u >> 1].x;
            k32[u] = (uint32_t)k;
            if (li >= hn) continue;
            const int64_t ts = (u & 1) ? t2[u >> 1].y : t2[u >> 1].x;
            int64_t q, h;
            const int b = classify(p, k, ts, &q, &h);
            if (b >= 0) {
                wide |= k != (int64_t)(int32_t)k;
                qmin = q < qmin ? q : qmin;
                qmax = q > qmax ? q : qmax;
                mask |= 1u << ((int)q & lm);
                const int ln = b >> p.region_bits;   // (selects: a dynamic register index would go to scratch)
#pragma unroll
                for (int l = 0; l < kMaxLanes; l++) lc[l] += ln == l ? 1u : 0u;
                const uint32_t cb = (uint32_t)b >> kTileBits;
                const uint32_t sh = (cb & 1u) * 16u;
                const uint32_t old = atomicAdd(&s_cw[cb >> 1], 1u << sh);
                rcb[u] = (((old >> sh) & 0xffffu) << 12) | cb;
            } else if (b == -1) {
                drops++;
            } else {   // outside the slice filter: in the batch's slice range only
                qmin = q < qmin ? q : qmin;
                qmax = q > qmax ? q : qmax;
                if (q >= p.filter_hi) qnext = q < qnext ? q : qnext;
            }
        }
    };
    longlong2 ka[R / 2], ta[R / 2];
    if (beg < end) load(beg, ka, ta);
    int j = 0;
    for (int64_t t0 = beg; t0 < end; t0 += TILE, j++) {
        uint32_t rcb[H][R], k32[H][R];
        {
            longlong2 kb[R / 2], tb[R / 2];
            if (H > 1 && t0 + HALF < end) load(t0 + HALF, kb, tb);   // (in flight across the first half's ranking)
            classify_half(t0, ka, ta, rcb[0], k32[0]);
            if (H > 1) {
                // the first half's ranks and keys wait in LDS (s_k is free until the staging): a tile of
                // two halves then holds one half's classification state in registers at a time
#pragma unroll
                for (int u = 0; u < R; u++)
                    reinterpret_cast<uint2*>(s_k)[u * T + tid] = make_uint2(rcb[0][u], k32[0][u]);
                if (t0 + HALF < end) {
                    classify_half(t0 + HALF, kb, tb, rcb[H - 1], k32[H - 1]);
                } else {
#pragma unroll
                    for (int u = 0; u < R; u++) rcb[H - 1][u] = 0xffffffffu;
                }
            }
        }
        if (H > 1) asm volatile("" ::: "memory");   // (the value loads not hoisted into the classification)
        longlong2 va[H][R / 2];
#pragma unroll
        for (int hh = 0; hh < H; hh++) load_vals(t0 + (int64_t)hh * HALF, va[hh]);   // (in flight across the scan)
        lds_barrier();
        if (H > 1) {   // (each thread its own stash entries, read before the barrier that precedes the staging)
#pragma unroll
            for (int u = 0; u < R; u++) {
                const uint2 q = reinterpret_cast<const uint2*>(s_k)[u * T + tid];
                rcb[0][u] = q.x;
                k32[0][u] = q.y;
            }
        }
        {   // exclusive scan of the tile's bucket counts, u16 pairs per word, consecutive words per thread
            constexpr int kPw = (kMaxTileBuckets / 2 + T - 1) / T;
            uint32_t c[kPw], run = 0;
#pragma unroll
            for (int q = 0; q < kPw; q++) {
                const int w = tid * pw + q;
                c[q] = (q < pw && w < NW) ? s_cw[w] : 0u;
                const uint32_t lo = c[q] & 0xffffu, hi = c[q] >> 16;
                run += lo + hi;
                bmax = lo > bmax ? lo : bmax;
                bmax = hi > bmax ? hi : bmax;
            }
            uint32_t total;
            uint32_t ex = block_exclusive_scan_t<true>(run, s_wave, &total);
#pragma unroll
            for (int q = 0; q < kPw; q++) {
                const int w = tid * pw + q;
                const uint32_t lo = c[q] & 0xffffu, hi = c[q] >> 16;
                if (q < pw && w < NW) s_cw[w] = ex | ((ex + lo) << 16);
                ex += lo + hi;
            }
            if (tid == 0) s_cw[NW] = total;
        }
        lds_barrier();
        {   // the directory row: the offsets (u16 pairs) and the tile's total
            uint32_t* drow = reinterpret_cast<uint32_t*>(p.dir + ((int64_t)blockIdx.x * p.max_tiles + j) * kTileDirStride(NC));
            for (int w = tid; w <= NW; w += T) drow[w] = s_cw[w];
        }
        const uint32_t tile_total = s_cw[NW];
        // stage the tile bucket sorted (the values arrive here), then write it back in place
#pragma unroll
        for (int hh = 0; hh < H; hh++) {
#pragma unroll
            for (int u = 0; u < R; u++) {
                const uint32_t rc = rcb[hh][u];
                if (rc == 0xffffffffu) continue;
                const uint32_t cb = rc & 4095u;
                const uint32_t slot = ((s_cw[cb >> 1] >> ((cb & 1u) * 16u)) & 0xffffu) + (rc >> 12);
                s_k[slot] = k32[hh][u];
                s_v[slot] = (unsigned long long)((u & 1) ? va[hh][u >> 1].y : va[hh][u >> 1].x);
            }
        }
        if (H > 1) asm volatile("" ::: "memory");   // (the next tile's loads not hoisted into the staging)
        if (t0 + TILE < end) load(t0 + TILE, ka, ta);   // the next tile's first half, across the write-out
        lds_barrier();
        for (uint32_t i = tid; i < tile_total; i += T) st_tile_rec(p.tmp, (uint64_t)(t0 + i), (int64_t)s_k[i], (int64_t)s_v[i]);
        lds_barrier();   // staging and the directory row have read the offsets
        for (int w = tid; w <= NW; w += T) s_cw[w] = 0;
        lds_barrier();
    }
    // tiles past the segment's end (a short last segment, or none): empty directory rows -- the
    // fire reads every workgroup's max_tiles rows, and the buffer holds the last batch's
    for (; j < p.max_tiles; j++) {
        uint32_t* drow = reinterpret_cast<uint32_t*>(p.dir + ((int64_t)blockIdx.x * p.max_tiles + j) * kTileDirStride(NC));
        for (int w = tid; w <= NW; w += T) drow[w] = 0u;
    }
    for (int off = 32; off > 0; off >>= 1) {
        drops += __shfl_down(drops, off);
        mask |= __shfl_down(mask, off);
        const uint32_t bm = __shfl_down(bmax, off);
        bmax = bm > bmax ? bm : bmax;
#pragma unroll
        for (int l = 0; l < kMaxLanes; l++) lc[l] += __shfl_down(lc[l], off);
        const long long oa = __shfl_down(qmin, off), oz = __shfl_down(qmax, off), on = __shfl_down(qnext, off);
        qmin = oa < qmin ? oa : qmin;
        qmax = oz > qmax ? oz : qmax;
        qnext = on < qnext ? on : qnext;
    }
    if ((tid & 63) == 0) {
        if (drops) atomicAdd(&s_drop, (unsigned long long)drops);
        if (mask) atomicOr(&s_mask, mask);
        if (bmax) atomicMax(&s_bmax, bmax);
#pragma unroll
        for (int l = 0; l < kMaxLanes; l++)
            if (lc[l]) atomicAdd(&s_lane[l], lc[l]);
        if (qmin != JMAX) atomicMin(&s_qmin, qmin);
        if (qmax != JMIN) atomicMax(&s_qmax, qmax);
        if (qnext != JMAX) atomicMin(&s_qnext, qnext);
    }
    if (p.wide && __ballot(wide) != 0 && (tid & 63) == 0) atomicOr(p.wide, 1u);
    __syncthreads();
    if (tid < p.lanes && s_lane[tid]) atomicAdd(&p.lane_total[tid], (unsigned long long)s_lane[tid]);
    if (tid == 0) {
        if (p.count_drops && s_drop) atomicAdd(p.drops, s_drop);
        if (s_mask) atomicOr(p.lane_mask, (unsigned long long)s_mask);
        if (s_bmax && p.max_bucket) atomicMax(p.max_bucket, s_bmax);
        if (s_qmin != JMAX) atomicMin(p.qmin, s_qmin);
        if (s_qmax != JMIN) atomicMax(p.qmax, s_qmax);
        if (s_qnext != JMAX) atomicMin(p.qnext, s_qnext);
    }
}

hipError_t launch_tile_part1(const IngestParams& p, hipStream_t s) {
    if (p.n_coarse < 2 || p.n_coarse % 2 != 0 || p.n_coarse > kMaxTileBuckets || p.region_bits < kTileBits || !p.tmp ||
        !p.dir || p.vnull != nullptr || p.max_tiles < 1 || p.grid < 1 ||
        (int64_t)p.grid * p.max_tiles * kTileRecs < p.n)   // (whole-tile segments cover the batch)
        return hipErrorInvalidValue;
    fg_launch(k_tile_part1, dim3(p.grid), dim3(kTileThreads), 0, s, p);
    return hipGetLastError();
}

// dir [tiles][kTileDirStride(nc)] (u16 offsets, [nc] the total) -> dt [nc][tiles] = offset | length << 16, 64 x 64 blocks
// through LDS; buckets of lanes without records (lane_mask) are skipped
__global__ __launch_bounds__(256) void k_tile_dirt(const uint16_t* dir, int32_t NT, int32_t NC, int32_t lshift,
                                                   const unsigned long long* lane_mask, uint32_t* dt, uint32_t* btot) {
    __shared__ uint16_t s[64][67];
    __shared__ uint32_t s_q[4][64];   // btot: quarter sums of the block's 64 tiles per column
    const int tb = blockIdx.x * 64, cb = blockIdx.y * 64;
    const unsigned long long lm = *gbl(lane_mask);
    const int l0 = cb >> lshift, l1 = (cb + 63 < NC ? cb + 63 : NC - 1) >> lshift;
    bool any = false;
    for (int l = l0; l <= l1; l++) any = any || ((lm >> l) & 1);
    if (!any) return;
    // the block's 64 rows of 65 offsets as 33 4-B words each (rows start 4-B aligned: the row
    // stride and the block's first bucket are even; a word past the row's NC + 2 entries is not
    // read), instead of 2-B loads
    for (int i = threadIdx.x; i < 64 * 33; i += 256) {
        const int tt = i / 33, k = i % 33;
        const int t = tb + tt, c = cb + 2 * k;
        uint32_t w = 0;
        if (t < NT && c <= NC) w = *gbl(reinterpret_cast<const uint32_t*>(dir + (int64_t)t * kTileDirStride(NC) + c));
        s[tt][2 * k] = (uint16_t)w;
        s[tt][2 * k + 1] = (uint16_t)(w >> 16);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int cc = i / 64, tt = i % 64;
        const int t = tb + tt, c = cb + cc;
        if (t < NT && c < NC && ((lm >> (c >> lshift)) & 1)) {
            const uint32_t a = s[tt][cc], b = s[tt][cc + 1];
            dt[(int64_t)c * NT + t] = a | ((b - a) << 16);
        }
    }
    // btot: the block's records per bucket column -- 4 threads per column sum 16 tiles each
    // (conflict-free LDS reads), then one global add per column. Per-lane LDS adds into the column's
    // counter (64 lanes, one address) took 164 vs 76 us per 100M-record pass (round 5)
    if (btot) {
        const int cc = threadIdx.x & 63, q = threadIdx.x >> 6;
        uint32_t sum = 0;
        for (int j = 0; j < 16; j++) {
            const int tt = q * 16 + j;
            if (tb + tt < NT) sum += (uint32_t)s[tt][cc + 1] - s[tt][cc];
        }
        s_q[q][cc] = sum;
        __syncthreads();
        const int c = cb + (int)threadIdx.x;
        if (threadIdx.x < 64 && c < NC && ((lm >> (c >> lshift)) & 1)) {
            const uint32_t t4 = s_q[0][threadIdx.x] + s_q[1][threadIdx.x] + s_q[2][threadIdx.x] + s_q[3][threadIdx.x];
            if (t4) atomicAdd(&btot[c], t4);
        }
    }
}

// The same transpose in wide blocks of TT tiles x TC buckets (nc >= TC): a block reads TT row
// segments of TC + 2 offsets (516 B at TC = 256: whole 64-B lines, where the 64 x 64 blocks read
// 132-B pieces of 4-KB rows, each line shared with a block launched far away) and writes TC
// columns of TT entries (one 128-B line each at TT = 32)
template <int TT, int TC>
__global__ __launch_bounds__(256) void k_tile_dirt_w(const uint16_t* dir, int32_t NT, int32_t NC, int32_t lshift,
                                                     const unsigned long long* lane_mask, uint32_t* dt,
                                                     uint32_t* btot) {
    static_assert(TC % 64 == 0 && 256 % TC == 0 || TC == 256, "dirt block shape");
    constexpr int RS = TC + 4;        // LDS row stride (u16): TC + 1 entries, padded
    constexpr int WPR = TC / 2 + 1;   // 4-B words per row segment: entries [cb, cb + TC + 2)
    constexpr int Q = 256 / TC;       // threads per column summing btot
    __shared__ uint16_t s[TT][RS];
    __shared__ uint32_t s_q[Q][TC];
    const int tb = blockIdx.x * TT, cb = blockIdx.y * TC;
    const unsigned long long lm = *gbl(lane_mask);
    const int l0 = cb >> lshift, l1 = (cb + TC - 1 < NC ? cb + TC - 1 : NC - 1) >> lshift;
    bool any = false;
    for (int l = l0; l <= l1; l++) any = any || ((lm >> l) & 1);
    if (!any) return;
    for (int i = threadIdx.x; i < TT * WPR; i += 256) {
        const int tt = i / WPR, k = i % WPR;
        const int t = tb + tt, c = cb + 2 * k;
        uint32_t w = 0;
        if (t < NT && c <= NC) w = *gbl(reinterpret_cast<const uint32_t*>(dir + (int64_t)t * kTileDirStride(NC) + c));
        *reinterpret_cast<uint32_t*>(&s[tt][2 * k]) = w;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < TT * TC; i += 256) {
        const int cc = i / TT, tt = i % TT;
        const int t = tb + tt, c = cb + cc;
        if (t < NT && c < NC && ((lm >> (c >> lshift)) & 1)) {
            const uint32_t a = s[tt][cc], b = s[tt][cc + 1];
            dt[(int64_t)c * NT + t] = a | ((b - a) << 16);
        }
    }
    if (btot) {
        const int cc = threadIdx.x % TC, q = threadIdx.x / TC;
        uint32_t sum = 0;
        for (int j = q; j < TT; j += Q)
            if (tb + j < NT) sum += (uint32_t)s[j][cc + 1] - s[j][cc];
        s_q[q][cc] = sum;
        __syncthreads();
        const int c = cb + (int)threadIdx.x;
        if ((int)threadIdx.x < TC && c < NC && ((lm >> (c >> lshift)) & 1)) {
            uint32_t t4 = 0;
#pragma unroll
            for (int j = 0; j < Q; j++) t4 += s_q[j][threadIdx.x];
            if (t4) atomicAdd(&btot[c], t4);
        }
    }
}

hipError_t launch_tile_dirt(const uint16_t* dir, int32_t tiles, int32_t nc, int32_t lane_shift,
                            const unsigned long long* lane_mask, uint32_t* dt, uint32_t* btot, hipStream_t s) {
    if (tiles <= 0 || nc <= 0) return hipSuccess;
    if (nc >= 256) {   // (A/B round 6, 64 x 128 blocks alike: 15.9-16.0 vs 16.1 ms per step)
        fg_launch((k_tile_dirt_w<32, 256>), dim3((unsigned)((tiles + 31) / 32), (unsigned)((nc + 255) / 256)), dim3(256),
                  0, s, dir, tiles, nc, lane_shift, lane_mask, dt, btot);
    } else {
        fg_launch(k_tile_dirt, dim3((unsigned)((tiles + 63) / 64), (unsigned)((nc + 63) / 64)), dim3(256), 0, s, dir,
                  tiles, nc, lane_shift, lane_mask, dt, btot);
    }
    return hipGetLastError();
}

// pass pi of a tile fire: one or two passes ride in the kernel arguments, more in a device array
__device__ __forceinline__ TilePass tile_pass(const TileFire& f, int pi) {
    if (f.n_passes == 1 || (f.n_passes == 2 && pi == 0)) return f.one;
    if (f.n_passes == 2) return f.two;
    return f.passes[pi];
}

// Order a wave's LDS writes before its other lanes' reads (wave-private scratch, no barrier).
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// A wave's walk over the fragments of one bucket (column `col` of a tile pass): groups of
// 64 * kTileTPL tiles (kTileTPL consecutive tiles per lane, this wave's every W-th group), each
// cut into windows of up to kTileWin records; next() fills the window's records (kTileWin / 64
// per lane, loads in flight on return) -- a wave-private map from a window position to its
// fragment (the fragments mark their first position, an inclusive max-scan fills the map)
// gives each record its source.
#ifndef FG_TILE_WIN
#define FG_TILE_WIN 256
#endif
#ifndef FG_TILE_TPL
#define FG_TILE_TPL 2   // tiles per lane of a walk group (A/B round 4: 2 -> tile_fire 0.852 vs 0.888 ms per 100M)
#endif
constexpr int kTileWin = FG_TILE_WIN;
constexpr int kTileRpl = kTileWin / 64;
constexpr int kTileTPL = FG_TILE_TPL;
constexpr int kTileGroup = 64 * kTileTPL;   // tiles per group (<= 256: u8 fragment ids)
static_assert(kTileGroup <= 256 && kTileWin % 64 == 0, "tile walk shape");
struct TileWalk {
    const uint32_t* col;
    const void* rec;
    uint32_t n;                 // records of the pass: a source at or past it is a walk error
    bool bad;                   // (reported as overflow flag 8, the record not read)
    int32_t nt;                 // the walk's end tile (exclusive)
    int32_t t0, tn;             // current group's first tile, the next group's (its entries in xn)
    int32_t t_base, ng;         // the walk's first tile, its groups
    int32_t gk, wave, W;        // groups taken (static assignment: group wave + W * k)
    uint32_t* q;                // LDS group counter the waves take groups from (nullptr: static)
    int32_t gsz;                // tiles per group (kTileGroup, fewer for a short tile range)
    uint32_t xn[kTileTPL];      // the next group's directory entries (prefetched)
    uint32_t g_len[kTileTPL], g_st[kTileTPL], g_tot, b;
};
// Wave-wide inclusive scans on the DPP network (row_shr 1/2/4/8 inside each row of 16 lanes, then
// row_bcast 15 / 31 across rows): one fused VALU op per step, no LDS round trip (a __shfl_up
// step is a ds_bpermute plus a select).
template <bool MAX>
__device__ __forceinline__ uint32_t dpp_op(uint32_t a, uint32_t b) { return MAX ? (a > b ? a : b) : a + b; }
template <bool MAX>
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    // lanes without a DPP source (or masked) read 0: the identity of max (values >= 0) and of +
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return v;
}
// the value of the lane below (0 for lane 0): DPP wave_shr:1
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}

// the walk's next group: from the workgroup's LDS counter (the waves of an item finish together:
// a wave that ran ahead takes more groups -- with a fixed share per wave the item's slowest wave
// held the others at the barrier after the inserts, 14 % of the headline fire's wave cycles, 5 %
// with the counter; fire 0.727 -> 0.677 ms per 100M records, round 6), or the static share
__device__ __forceinline__ int32_t tile_walk_grab(TileWalk& w, int lane) {
    if (!w.q) return w.wave + w.W * (w.gk++);
    uint32_t g = 0;
    if (lane == 0) g = atomicAdd(w.q, 1u);
    return (int32_t)__builtin_amdgcn_readfirstlane(g);
}
// (the walk covers the pass's tiles [t_lo, t_hi): all of them, or a split bucket's chunk)
__device__ __forceinline__ void tile_walk_begin(TileWalk& w, const TilePass& tp, int32_t cb, int wave, int W,
                                                int lane, int32_t t_lo, int32_t t_hi, uint32_t* q = nullptr) {
    w.col = tp.dt + (int64_t)cb * tp.nt;
    w.rec = tp.rec;
    w.n = (uint32_t)tp.n;
    w.bad = false;
    w.nt = t_hi;
    // a short tile range (a small batch: a few hundred tiles) is spread over every wave -- groups
    // of kTileGroup tiles would leave most waves without one
    const int32_t per = (t_hi - t_lo + W - 1) / W;
    w.gsz = per >= kTileGroup ? kTileGroup : (per + kTileTPL - 1) / kTileTPL * kTileTPL;
    if (w.gsz < kTileTPL) w.gsz = kTileTPL;
    w.t_base = t_lo;
    w.ng = t_hi > t_lo ? (t_hi - t_lo + w.gsz - 1) / w.gsz : 0;
    w.gk = 0;
    w.wave = wave;
    w.W = W;
    // (passes of a few groups per wave keep the static share: the table fires' 2-3K-tile passes
    // ran 5-15 % slower taking groups from the counter, A/B round 6)
    w.q = w.ng >= 4 * W ? q : nullptr;
    const int32_t g0 = tile_walk_grab(w, lane);
    w.tn = g0 < w.ng ? t_lo + g0 * w.gsz : t_hi;
#pragma unroll
    for (int q4 = 0; q4 < kTileTPL; q4++) {
        // (every load issued, the index clamped and the entry masked: a load under a branch would
        // keep the compiler from counting the wave's loads in flight -- s_waitcnt vmcnt(0))
        const int t = w.tn + lane * kTileTPL + q4;
        const bool ok = t < w.nt && lane * kTileTPL + q4 < w.gsz;
        const uint32_t x = gbl(w.col)[ok ? t : 0];
        w.xn[q4] = ok ? x : 0u;
        w.g_len[q4] = w.g_st[q4] = 0;
    }
    w.g_tot = w.b = 0;
}
// the next window of the walk: records in kr / vr (lanes at or past nrec: garbage, masked by the
// caller), false when done. Every record load is issued unconditionally (lanes past nrec read
// record 0), so the loads in flight are counted and the previous window's inserts wait only for
// their own loads.
__device__ __forceinline__ bool tile_walk_next(TileWalk& w, uint8_t* fm, uint32_t* dl, int lane,
                                               int32_t (&kr)[kTileRpl], int64_t (&vr)[kTileRpl], uint32_t& nrec) {
    static_assert(kTileRpl == 4, "one fragment-map word per lane");
    // (every path issues the window's loads, also the one that ends the walk: the caller's
    // inserts then wait for exactly their own loads -- a path without them would make the
    // compiler count the loads of the window just issued as possibly absent)
    bool done = false;
    while (w.b >= w.g_tot) {   // the next group with records
        w.t0 = w.tn;
        if (w.t0 >= w.nt) {
            done = true;
            break;
        }
        const int32_t gn = tile_walk_grab(w, lane);
        w.tn = gn < w.ng ? w.t_base + gn * w.gsz : w.nt;
        uint32_t base[kTileTPL], sum = 0;
#pragma unroll
        for (int q = 0; q < kTileTPL; q++) {
            const int t = w.t0 + lane * kTileTPL + q;
            const uint32_t x = w.xn[q];
            const int tn = w.tn + lane * kTileTPL + q;
            const bool okn = tn < w.nt && lane * kTileTPL + q < w.gsz;
            const uint32_t xn = gbl(w.col)[okn ? tn : 0];
            w.xn[q] = okn ? xn : 0u;
            w.g_len[q] = x >> 16;
            base[q] = (uint32_t)t * (uint32_t)kTileRecs + (x & 0xffffu);   // (whole-tile segments)
            w.g_st[q] = sum;   // (local prefix; the wave's exclusive prefix added below)
            sum += w.g_len[q];
        }
        uint32_t inc = wave_incl_scan<false>(sum);
        // (the scan materialized: the compiler otherwise folds `base - (prefix + inc - sum)` into a
        // chain of DPP subtracts, which produced wrong fragment bases -- DESIGN section 8)
        asm volatile("" : "+v"(inc));
        const uint32_t ex = inc - sum;
        w.g_tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        w.b = 0;
        wave_lds_sync();   // (the last window's reads of dl are done: its loads were issued)
#pragma unroll
        for (int q = 0; q < kTileTPL; q++) {
            w.g_st[q] += ex;
            dl[lane * kTileTPL + q] = base[q] - w.g_st[q];
        }
    }
    // the fragment map of the window: each position's fragment (the fragments mark their first
    // position, then an inclusive max-scan), one 4-byte word of 4 positions per lane
    if (done) {
        w.b = w.g_tot = 0;   // (nrec = 0 below: the loads read record 0)
    }
    uint32_t* fm32 = reinterpret_cast<uint32_t*>(fm);
    fm32[lane] = 0;
    wave_lds_sync();
#pragma unroll
    for (int q = 0; q < kTileTPL; q++) {
        const uint32_t st = w.g_st[q], len = w.g_len[q];
        if (len > 0 && st < w.b + kTileWin && st + len > w.b) fm[st > w.b ? st - w.b : 0] = (uint8_t)(lane * kTileTPL + q);
    }
    wave_lds_sync();
    const uint32_t e4 = fm32[lane];
    uint32_t e0 = e4 & 255u, e1 = (e4 >> 8) & 255u, e2 = (e4 >> 16) & 255u, e3 = e4 >> 24;
    e1 = e1 > e0 ? e1 : e0;
    e2 = e2 > e1 ? e2 : e1;
    e3 = e3 > e2 ? e3 : e2;
    const uint32_t pre = wave_shr1(wave_incl_scan<true>(e3));
    e0 = e0 > pre ? e0 : pre;
    e1 = e1 > pre ? e1 : pre;
    e2 = e2 > pre ? e2 : pre;
    e3 = e3 > pre ? e3 : pre;
    fm32[lane] = e0 | e1 << 8 | e2 << 16 | e3 << 24;
    wave_lds_sync();
    nrec = w.g_tot - w.b < (uint32_t)kTileWin ? w.g_tot - w.b : (uint32_t)kTileWin;
    // every position's fragment, then every fragment's base: two LDS round trips for the window's
    // records, no branch (a position past nrec reads a garbage map entry, masked below)
    uint32_t fq[kTileRpl], dq[kTileRpl];
#pragma unroll
    for (int u = 0; u < kTileRpl; u++) fq[u] = fm[lane + 64 * u] & (uint32_t)(kTileGroup - 1);
#pragma unroll
    for (int u = 0; u < kTileRpl; u++) dq[u] = dl[fq[u]];
#pragma unroll
    for (int u = 0; u < kTileRpl; u++) {
        const uint32_t jr = lane + 64 * u;
        uint32_t src = jr < nrec ? dq[u] + w.b + jr : 0u;
        if (src >= w.n) {   // (never, if the directory and the walk agree: reported, not read)
#ifdef FG_DEBUG_WALK
            if (!w.bad)
                printf("walk: lane %d u %d jr %u nrec %u b %u g_tot %u t0 %d nt %d n %u src %u fm %u dl %u "
                       "g_st %u %u g_len %u %u xn %u %u\n", lane, u, jr, nrec, w.b, w.g_tot, w.t0, w.nt, w.n, src,
                       (uint32_t)fm[jr], dl[fm[jr]], w.g_st[0], w.g_st[1], w.g_len[0], w.g_len[1], w.xn[0], w.xn[1]);
#endif
            w.bad = true;
            src = 0;
        }
#if defined(FG_DIAG_FIRE) && (FG_DIAG_FIRE & 1)   // (diagnostic: no record loads, keys from the source index)
        kr[u] = (int32_t)((src * 2654435761u) >> 20);
        vr[u] = (int64_t)src;
#else
        const Rec12 r = ld_tile_rec(w.rec, (uint64_t)src);
        kr[u] = (int32_t)r.k;
        vr[u] = rec12_val(r);
#endif
    }
    w.b += kTileWin;
    return !done;
}

// ---- device self-check (fg_selftest): the DPP wave scans and the tile walk as compiled here -----
// Round 5 found the compiler folding the walk's DPP scan into a wrong subtract chain;
// these kernels run the SAME inline functions the fire runs, on inputs whose answer the host knows.
__global__ __launch_bounds__(256) void k_selftest_scan(const uint32_t* in, uint32_t* out) {
    const uint32_t v = in[threadIdx.x];
    const uint32_t a = wave_incl_scan<false>(v);
    const uint32_t m = wave_incl_scan<true>(v & 255u);
    out[3 * threadIdx.x] = a;
    out[3 * threadIdx.x + 1] = m;
    out[3 * threadIdx.x + 2] = wave_shr1(m);
}
// one wave per bucket column: the walk's records in walk order (the key of record i is i)
__global__ __launch_bounds__(64) void k_selftest_walk(TilePass tp, uint32_t cap, uint32_t* out, uint32_t* n_out,
                                                      unsigned int* bad) {
    __shared__ __attribute__((aligned(16))) uint8_t s_fm[kTileWin];
    __shared__ uint32_t s_dl[kTileGroup];
    const int lane = threadIdx.x;
    const int32_t cb = blockIdx.x;
    TileWalk w;
    tile_walk_begin(w, tp, cb, 0, 1, lane, 0, tp.nt);
    int32_t kr[kTileRpl];
    int64_t vr[kTileRpl];
    uint32_t nrec = 0, pos = 0;
    while (tile_walk_next(w, s_fm, s_dl, lane, kr, vr, nrec)) {
#pragma unroll
        for (int u = 0; u < kTileRpl; u++) {
            const uint32_t jr = lane + 64 * u;
            if (jr < nrec && pos + jr < cap) out[(uint64_t)cb * cap + pos + jr] = (uint32_t)kr[u];
        }
        pos += nrec;
    }
    if (lane == 0) n_out[cb] = pos;
    if (__ballot(w.bad) != 0 && lane == 0) atomicOr(bad, 1u);
}
__global__ void k_selftest_fill(uint32_t* rec, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        rec[3 * i] = (uint32_t)i;   // (value lo = hi = the index's low word: only the key is checked)
        rec[3 * i + 1] = 0u;
        rec[3 * i + 2] = (uint32_t)i;
    }
}

int run_selftest(int device, char* msg, size_t cap_msg) {
    auto say = [&](const char* m) {
        if (msg && cap_msg) snprintf(msg, cap_msg, "%s", m);
    };
    if (hipSetDevice(device) != hipSuccess) {
        say("hipSetDevice failed");
        return 1;
    }
    uint64_t x = 0x5EEDF11Cull;
    auto rnd = [&]() {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        return (uint32_t)(x >> 33);
    };
    // 1. the scans over 4 waves of random values
    std::vector<uint32_t> in(256), got(3 * 256);
    for (auto& v : in) v = rnd() & 1023u;
    // 2. a tile pass of NT tiles, NB buckets; fragment lengths 0..20 (a fifth empty), offsets packed
    constexpr int NT = 300, NB = 3;
    std::vector<uint32_t> dt((size_t)NB * NT);
    std::vector<std::vector<uint32_t>> want(NB);
    for (int t = 0; t < NT; t++) {
        uint32_t off = rnd() % 64;
        for (int b = 0; b < NB; b++) {
            const uint32_t len = rnd() % 5 == 0 ? 0 : rnd() % 21;
            dt[(size_t)b * NT + t] = off | len << 16;
            for (uint32_t i = 0; i < len; i++) want[b].push_back((uint32_t)t * (uint32_t)kTileRecs + off + i);
            off += len;
        }
    }
    const uint64_t nrec = (uint64_t)NT * kTileRecs;
    uint32_t cap = 0;
    for (auto& v : want) cap = std::max<uint32_t>(cap, (uint32_t)v.size());
    void *d_in = nullptr, *d_out = nullptr, *d_rec = nullptr, *d_dt = nullptr, *d_w = nullptr, *d_n = nullptr,
         *d_bad = nullptr;
    int rc = 0;
    const char* what = nullptr;
    auto cleanup = [&]() {
        for (void* q : {d_in, d_out, d_rec, d_dt, d_w, d_n, d_bad})
            if (q) (void)hipFree(q);
    };
    if (hipMalloc(&d_in, 4 * 256) != hipSuccess || hipMalloc(&d_out, 4 * 3 * 256) != hipSuccess ||
        hipMalloc(&d_rec, 12 * nrec) != hipSuccess || hipMalloc(&d_dt, 4 * dt.size()) != hipSuccess ||
        hipMalloc(&d_w, 4 * (size_t)NB * cap + 4) != hipSuccess || hipMalloc(&d_n, 4 * NB) != hipSuccess ||
        hipMalloc(&d_bad, 4) != hipSuccess) {
        cleanup();
        say("self-check: device allocation failed");
        return 1;
    }
    (void)hipMemcpy(d_in, in.data(), 4 * 256, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_dt, dt.data(), 4 * dt.size(), hipMemcpyHostToDevice);
    (void)hipMemset(d_bad, 0, 4);
    k_selftest_scan<<<1, 256>>>(static_cast<const uint32_t*>(d_in), static_cast<uint32_t*>(d_out));
    k_selftest_fill<<<256, 256>>>(static_cast<uint32_t*>(d_rec), nrec);
    TilePass tp{};
    tp.rec = d_rec;
    tp.dt = static_cast<const uint32_t*>(d_dt);
    tp.n = (int64_t)nrec;
    tp.nt = NT;
    tp.mt = NT;
    tp.nc = NB;
    k_selftest_walk<<<NB, 64>>>(tp, cap, static_cast<uint32_t*>(d_w), static_cast<uint32_t*>(d_n),
                                static_cast<unsigned int*>(d_bad));
    std::vector<uint32_t> walk((size_t)NB * cap), wn(NB);
    unsigned int bad = 0;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(got.data(), d_out, 4 * 3 * 256, hipMemcpyDeviceToHost) ||
        hipMemcpy(walk.data(), d_w, 4 * walk.size(), hipMemcpyDeviceToHost) ||
        hipMemcpy(wn.data(), d_n, 4 * NB, hipMemcpyDeviceToHost) || hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost)) {
        cleanup();
        say("self-check: a kernel or copy failed");
        return 1;
    }
    cleanup();
    for (int wv = 0; wv < 4 && !what; wv++) {
        uint32_t a = 0, m = 0, prev = 0;
        for (int l = 0; l < 64; l++) {
            const uint32_t v = in[64 * wv + l];
            a += v;
            m = (v & 255u) > m ? (v & 255u) : m;
            const uint32_t* o = &got[3 * (64 * wv + l)];
            if (o[0] != a) what = "self-check: the DPP add scan (wave_incl_scan) is wrong";
            else if (o[1] != m) what = "self-check: the DPP max scan (wave_incl_scan) is wrong";
            else if (o[2] != (l ? prev : 0u)) what = "self-check: the DPP lane shift (wave_shr1) is wrong";
            if (what) break;
            prev = m;
        }
    }
    for (int b = 0; b < NB && !what; b++) {
        if (wn[b] != want[b].size()) what = "self-check: the tile walk visited a wrong number of records";
        for (size_t i = 0; !what && i < want[b].size(); i++)
            if (walk[(size_t)b * cap + i] != want[b][i]) what = "self-check: the tile walk read a wrong record";
    }
    if (!what && bad) what = "self-check: the tile walk addressed a record past its pass";
    if (what) {
        say(what);
        rc = 1;
    } else {
        say("ok");
    }
    return rc;
}

// Fire from tile passes: one workgroup per item -- a bucket of the lane (4 << (bits - tbits)
// regions at the current bits), or on a retry one region (its bucket's records filtered by the
// key's region) -- gathers the item's records from every pass, aggregates them in an LDS table
// of kTileSlots 32-bit keys (COUNT(*) u32, one value slot; the home bucket of 4 slots from a
// 32-bit multiplicative hash) and emits one row per key (a6 arithmetic: write_row_k). Two
// windows in flight per wave: the next window's loads are issued before this one's inserts. A
// full table emits nothing and lists the item's regions in the fail list (the host splits the
// regions and redoes them one region per item, MergeParams fail protocol).
// With resident state (m.n_src > 0: slice tables -- a HOP slice's own table, a CUMULATE window's
// first slice, AggCombiner's accState) the item's regions of every source table are inserted
// first (their COUNT(*) and value accumulator, the keys from their mixes); with m.has_dst the
// item's aggregate is written back as the destination table's regions -- each key into its
// region's block, the regions' counts replaced (RecordsWindowBuffer.flush + AggCombiner.combine
// straight from the tiles, no staged pass 2). A region holding more than kRegionCap keys fails
// the item like a full table: nothing is written or emitted and its regions are redone.
// m.emit = 0: a flush (the table written, no rows).
// HOT (a skewed pass's split fire, SUM-family value ops): the insert pre-combines a wave's records of
// a hot key; the plain fire keeps the one-probe-loop-per-record insert (A/B, round 5: 0.89 vs 1.08
// ms per 100M records for the branch-free insert with a dummy slot)
// SM: 0 the plain fire (no split code: the split and merge paths cost it 4 spilled VGPRs, round 5),
// 1 a split fire's launches (chunk items, then the merge launch), 2 chunk items with HOT
template <int VTC, bool TAB, int SM>   // TAB: source / destination tables (compiled out of the plain fire)
__global__ __launch_bounds__(kTileFireThreads) void k_tile_fire(TileFire fa) {
    const TileFire& f = fa;
    constexpr bool HOT = SM == 2;
    constexpr int T = kTileFireThreads, W = T / 64, S = kTileSlots;
    constexpr int kRounds = S / T + 1;   // + 1: the sentinel slot (thread 0)
    static_assert(S % T == 0 && (S & (S - 1)) == 0, "table rounds");
    // slot S: the key INT32_MIN (the empty sentinel); slot S + 1: a dummy that window lanes without
    // a record (or whose key found no slot) add into, so the inserts need no branch (never emitted)
    constexpr int kDummy = S + 1;
    __shared__ __attribute__((aligned(16))) int32_t t_key[S + 2];
    __shared__ uint32_t t_cs[S + 2];
    __shared__ unsigned long long t_v[S + 2];
    __shared__ __attribute__((aligned(16))) uint8_t s_fm[W][kTileWin];
    __shared__ uint32_t s_dl[W][kTileGroup];
    __shared__ uint32_t s_grp[kRounds * W];
    __shared__ uint16_t s_map[S + 1];
    __shared__ unsigned int s_flags;
    __shared__ uint32_t s_total;
    __shared__ unsigned long long s_out_base;
    __shared__ uint32_t s_rc[kTileMaxRegions];   // destination: keys per region of the item
    __shared__ uint32_t s_rb[kTileMaxRegions];   // destination: each region's first rank
    __shared__ uint32_t s_gnext[kMaxTilePasses];  // per pass: the next tile group a wave takes
    const MergeParams& p = f.m;
    const bool dst = TAB && p.has_dst != 0;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef FG_STAMPS
    // diagnostic build only: cycles per phase summed over the waves -- 0 table clear, 1 tile walk
    // (fragment map, sources, loads issued), 2 waiting for a window's records, 3 inserts, 4 resident
    // sources / chunk partials, 5 the barrier after the inserts (the item's slowest wave), 6
    // compaction (occupancy ranks, row reservation, rank -> slot map), 7 emit / write-back
    unsigned long long fst_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long fst_prev = __builtin_amdgcn_s_memtime();
#define FSTAMP(i)                                                     \
    do {                                                              \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        fst_acc[i] += now_ - fst_prev;                                \
        fst_prev = now_;                                              \
    } while (0)
#define FWAIT(kk, vv) asm volatile("" ::"v"(kk[kTileRpl - 1]), "v"(vv[kTileRpl - 1]))
#else
#define FSTAMP(i) \
    do {          \
    } while (0)
#define FWAIT(kk, vv) \
    do {              \
    } while (0)
#endif
    const int vt = VTC >= 0 ? VTC : p.val_type;
    const int64_t vinit = lds_repr(vt, val_identity(vt));
    const int sub = p.region_bits - f.tbits;          // current region bits above the passes'
    const bool retry = p.retry_list != nullptr;
    const bool split = SM != 0 && f.split != 0;       // items planned by k_tile_plan (a skewed pass)
    const bool merge = split && f.merge != 0;         // the split buckets' merge of their chunks' partials
    __shared__ int s_item;   // split: the item fetched by workgroup (dynamic: chunk items vary in size)
    const int NI = retry ? p.n_retry
                   : merge ? (int)*gbl(f.sp.n_split)
                   : split ? (int)*gbl(f.sp.n_items)
                           : 1 << (f.tbits - kTileBits);
    const int G = gridDim.x;
    const bool xcd = !retry && !split && G % 8 == 0;  // consecutive buckets on one XCD (shared L2 lines)
    for (int k = 0;; k++) {
        const int b = (int)blockIdx.x;
        int x = xcd ? k * G + (b % 8) * (G / 8) + b / 8 : b + k * G;
        if (split && !merge) {   // (s_item's previous value was read before this iteration's barriers)
            if (tid == 0) s_item = (int)atomicAdd(f.sp.next_item, 1u);
            __syncthreads();
            x = s_item;
            if (x >= NI) break;
        } else if (k * G >= NI) {
            break;
        }
        bool live = x < NI;
#if !defined(FG_FIRE_HOIST)
        // (the parameters re-read through an opaque offset per item and again for the compaction:
        // hoisted to the kernel's entry they held ~100 SGPRs across the record loop, 80 of them
        // spilled to VGPR lanes, and left one SGPR pair for every compare of the probe loop)
        const TileFire& f = (&fa)[opaque_zero()];
        const MergeParams& p = f.m;
#endif
        int r_lo = 0, r_hi = 0, item = 0;
        int32_t g_lo = 0, g_hi = 0x7fffffff, part = -1;   // (split: the item's tile range, chunk ordinal)
        int32_t mc0 = 0, mck = 0;                          // (merge: the bucket's chunks)
        if (live) {
            if (merge) {
                item = f.sp.split_b[x];
                mc0 = f.sp.split_c0[x];
                mck = f.sp.split_k[x];
                r_lo = item << (sub + kTileBits);
                r_hi = (item + 1) << (sub + kTileBits);
                live = *gbl(&f.sp.bfail[item]) == 0u;   // (a failed chunk: the retry redoes the bucket)
            } else if (retry) {
                r_lo = gbl(p.retry_list)[x];
                r_hi = r_lo + 1;
                item = r_lo >> (sub + kTileBits);
            } else if (split) {
                const TileItem it = f.sp.items[x];
                item = it.bucket;
                g_lo = it.g_lo;
                g_hi = it.g_hi;
                part = it.part;
                r_lo = item << (sub + kTileBits);
                r_hi = (item + 1) << (sub + kTileBits);
            } else {
                item = x;
                r_lo = x << (sub + kTileBits);
                r_hi = (x + 1) << (sub + kTileBits);
            }
        }
        // a chunk of a split bucket writes partial entries only (no resident state, rows or table)
        const bool to_part = split && !merge && part >= 0;
        for (int i = tid; i <= S + 1; i += T) {
            t_key[i] = kEmpty32;
            t_cs[i] = 0;
            t_v[i] = (unsigned long long)vinit;
        }
        if (TAB)
            for (int i = tid; i < kTileMaxRegions; i += T) s_rc[i] = 0;
        if (tid < kMaxTilePasses) s_gnext[tid] = 0;
        if (tid == 0) s_flags = 0;
        __syncthreads();
        FSTAMP(0);
        bool full = false;
#if defined(FG_DIAG_FIRE)
        uint64_t diag_sink = 0;
#endif
        // the slot of `key` in the table (claimed if new), -1 when the table is full
        auto slot_of = [&](int32_t key) -> int {
            if (key == kEmpty32) return S;
            uint32_t home = __umulhi((uint32_t)key * 0x9E3779B1u, (uint32_t)(S / 4)) * 4;
            for (int probe = 0; probe < S / 4; probe++) {
                const int4 q4 = *reinterpret_cast<const int4*>(&t_key[home]);
                const int32_t qq[4] = {q4.x, q4.y, q4.z, q4.w};
                int hit = -1, emp = -1;
#pragma unroll
                for (int z = 3; z >= 0; z--) {
                    if (qq[z] == key) hit = z;
                    if (qq[z] == kEmpty32) emp = z;
                }
                if (hit >= 0 && (emp < 0 || hit < emp)) return (int)home + hit;
                if (emp >= 0) {
                    const int old = atomicCAS(&t_key[home + emp], kEmpty32, key);
                    if (old == kEmpty32 || old == key) return (int)home + emp;
                    continue;   // (lost the slot to another key: the same bucket again)
                }
                home = (home + 4) & (S - 1);
            }
            return -1;
        };
        if (TAB && p.n_src > 0 && !to_part) {
            // resident state first: the item's regions of every source table (keys as mixes; the
            // operator's keys fit 32 bits, so a mix's key is its int32) -- one flat sequence over
            // the (source, region) ranges (their counts' exclusive prefix in s_rb, wave 0), every
            // thread kSrcU entries per round, their loads issued before any insert
            constexpr int cap = kRegionCap;
            const int nreg = r_hi - r_lo, nrange = live ? p.n_src * nreg : 0;   // (host: <= kTileMaxRegions)
            if (wave == 0) {
                constexpr int RPL = kTileMaxRegions / 64;
                uint32_t c[RPL], x = 0;
#pragma unroll
                for (int q = 0; q < RPL; q++) {
                    const int g = RPL * lane + q;
                    c[q] = g < nrange ? gbl(src_at(p, g / nreg).counts)[r_lo + g % nreg] : 0u;
                    x += c[q];
                }
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t y = __shfl_up(x, off);
                    if (lane >= off) x += y;
                }
                uint32_t ex = x;
#pragma unroll
                for (int q = 0; q < RPL; q++) ex -= c[q];
#pragma unroll
                for (int q = 0; q < RPL; q++) {
                    if (RPL * lane + q < nrange) s_rb[RPL * lane + q] = ex;
                    ex += c[q];
                }
                if (lane == 63) s_total = x;
            }
            __syncthreads();
            const uint32_t NE = nrange ? s_total : 0u;
            for (uint32_t i0 = 0; !p.src_narrow && i0 < NE; i0 += kSrcU * T) {   // wide sources (a loop of its own)
                int64_t mk[kSrcU], cs[kSrcU], v[kSrcU];
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    const uint32_t i = i0 + u * T + tid;
                    mk[u] = cs[u] = v[u] = 0;
                    if (i >= NE) continue;
                    int lo = 0, hi = nrange;   // the range of entry i: the last base <= i
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (s_rb[mid] <= i) lo = mid;
                        else hi = mid;
                    }
                    const auto base = gbl(src_at(p, lo / nreg).base + (int64_t)(r_lo + lo % nreg) * 4 * cap);
                    const uint32_t e = i - s_rb[lo];
                    mk[u] = base[e];
                    cs[u] = base[cap + e];
                    v[u] = base[3 * cap + e];
                }
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    if (i0 + u * T + tid >= NE) continue;
                    const int sl = slot_of((int32_t)key_of(mk[u]));   // (keys32: a mix's key is its int32)
                    if (sl < 0) {
                        full = true;
                        continue;
                    }
                    atomicAdd(&t_cs[sl], (uint32_t)cs[u]);
                    lds_val(&t_v[sl], v[u], vt, true);
                }
            }
            for (uint32_t i0 = 0; p.src_narrow && i0 < NE; i0 += kSrcU * T) {
                int64_t cs[kSrcU], v[kSrcU];
                int32_t mk[kSrcU];
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    const uint32_t i = i0 + u * T + tid;
                    mk[u] = 0;
                    cs[u] = v[u] = 0;
                    if (i >= NE) continue;
                    int lo = 0, hi = nrange;   // the range of entry i: the last base <= i
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (s_rb[mid] <= i) lo = mid;
                        else hi = mid;
                    }
                    const TableRef sr = src_at(p, lo / nreg);
                    const auto base = gbl(sr.base + (int64_t)(r_lo + lo % nreg) * 4 * cap);
                    const uint32_t e = i - s_rb[lo];
                    const bool nar = sr.narrow != 0;   // (the operator's keys fit 32 bits: a mix's key is its int32)
                    mk[u] = tab_key32(base, cap, e, nar);
                    cs[u] = tab_cs(base, cap, e, nar);
                    v[u] = tab_v(base, cap, e, nar);
                }
#pragma unroll
                for (int u = 0; u < kSrcU; u++) {
                    if (i0 + u * T + tid >= NE) continue;
                    const int sl = slot_of(mk[u]);
                    if (sl < 0) {
                        full = true;
                        continue;
                    }
                    atomicAdd(&t_cs[sl], (uint32_t)cs[u]);
                    lds_val(&t_v[sl], v[u], vt, true);
                }
            }
        }
        FSTAMP(4);
        if (live && merge) {
            // the split bucket's chunks: their partial entries (int32 key, COUNT(*), the value's LDS
            // form) into the table -- the value combined as the chunks combined their records.
            // Up to kTileMaxRegions chunks at a time form one flat sequence (their counts' exclusive
            // prefix in s_rb, wave 0), every thread kPartU entries per round with their loads issued
            // before any insert: a hot bucket has hundreds of chunks of a few thousand entries each,
            // which chunk by chunk left one load round trip per few entries
            constexpr int kPartU = 4;
            for (int c0 = mc0; c0 < mc0 + mck; c0 += kTileMaxRegions) {
                const int nc = min(kTileMaxRegions, mc0 + mck - c0);
                __syncthreads();   // (s_rb: the source ranges' or the previous group's readers are done)
                if (wave == 0) {
                    constexpr int RPL = kTileMaxRegions / 64;
                    uint32_t c[RPL], x = 0;
#pragma unroll
                    for (int q = 0; q < RPL; q++) {
                        const int g = RPL * lane + q;
                        c[q] = 0;
                        if (g < nc) {
                            const uint32_t off = f.sp.part_off[c0 + g], n = f.sp.part_n[c0 + g];
                            if ((uint64_t)off + n <= (uint64_t)f.sp.part_cap) c[q] = n;
                            else atomicOr(p.overflow, 2u);   // (never: a failed chunk fails its bucket)
                        }
                        x += c[q];
                    }
                    for (int off = 1; off < 64; off <<= 1) {
                        const uint32_t y = __shfl_up(x, off);
                        if (lane >= off) x += y;
                    }
                    uint32_t ex = x;
#pragma unroll
                    for (int q = 0; q < RPL; q++) ex -= c[q];
#pragma unroll
                    for (int q = 0; q < RPL; q++) {
                        if (RPL * lane + q < nc) s_rb[RPL * lane + q] = ex;
                        ex += c[q];
                    }
                    if (lane == 63) s_total = x;
                }
                __syncthreads();
                const uint32_t NE = s_total;
                for (uint32_t i0 = 0; i0 < NE; i0 += kPartU * T) {
                    int32_t pk[kPartU];
                    uint32_t pc[kPartU];
                    unsigned long long pv[kPartU];
#pragma unroll
                    for (int u = 0; u < kPartU; u++) {
                        const uint32_t i = i0 + u * T + tid;
                        pk[u] = kEmpty32;
                        pc[u] = 0;
                        pv[u] = 0;
                        if (i >= NE) continue;
                        int lo = 0, hi = nc;   // the chunk of entry i: the last base <= i
                        while (hi - lo > 1) {
                            const int mid = (lo + hi) >> 1;
                            if (s_rb[mid] <= i) lo = mid;
                            else hi = mid;
                        }
                        const uint32_t e = f.sp.part_off[c0 + lo] + (i - s_rb[lo]);
                        pk[u] = f.sp.p_key[e];
                        pc[u] = f.sp.p_cs[e];
                        pv[u] = f.sp.p_v[e];
                    }
#pragma unroll
                    for (int u = 0; u < kPartU; u++) {
                        if (i0 + u * T + tid >= NE) continue;
                        const int sl = slot_of(pk[u]);
                        if (sl < 0) {
                            full = true;
                            continue;
                        }
                        atomicAdd(&t_cs[sl], pc[u]);
                        lds_val(&t_v[sl], lds_repr(vt, (int64_t)pv[u]), vt, true);
                    }
                }
            }
        } else if (live) {
            // one window's records into the table, one probe loop per record (the plain fire)
            // (FULL: a whole window, every lane's records present; RETRY: the region filter --
            // compile-time tags, so the common case's loop carries neither per-record test)
            auto insert_plain = [&](auto FULL, auto RETRY, const int32_t (&kr)[kTileRpl], const int64_t (&vr)[kTileRpl],
                                    uint32_t nrec) {
#if defined(FG_DIAG_FIRE) && (FG_DIAG_FIRE & 2)   // (diagnostic: no inserts, the records consumed)
#pragma unroll
                for (int u = 0; u < kTileRpl; u++)
                    if (lane + 64 * u < nrec) diag_sink ^= (uint64_t)kr[u] ^ (uint64_t)vr[u];
                return;
#endif
                uint32_t hm[kTileRpl];
                int4 bq[kTileRpl];
#pragma unroll
                for (int u = 0; u < kTileRpl; u++) {   // every home bucket read first, then resolved
                    hm[u] = __umulhi((uint32_t)kr[u] * 0x9E3779B1u, (uint32_t)(S / 4)) * 4;
                    bq[u] = *reinterpret_cast<const int4*>(&t_key[hm[u]]);
                }
#pragma unroll
                for (int u = 0; u < kTileRpl; u++) {
                    if (!decltype(FULL)::value && lane + 64 * u >= nrec) continue;
                    const int32_t key = kr[u];
                    if (decltype(RETRY)::value && retry &&
                        (int)((uint64_t)mix_of((int64_t)key) >> (64 - p.region_bits)) != r_lo)
                        continue;
                    int sl = -1;
                    if (key == kEmpty32) {
                        sl = S;
                    } else {
                        uint32_t home = hm[u];
                        int4 q4 = bq[u];
                        for (int probe = 0; probe < S / 4; probe++) {
                            const int32_t qq[4] = {q4.x, q4.y, q4.z, q4.w};
                            int hit = -1, emp = -1;
#pragma unroll
                            for (int z = 3; z >= 0; z--) {
                                if (qq[z] == key) hit = z;
                                if (qq[z] == kEmpty32) emp = z;
                            }
                            if (hit >= 0 && (emp < 0 || hit < emp)) {
                                sl = (int)home + hit;
                                break;
                            }
                            if (emp >= 0) {
                                const int old = atomicCAS(&t_key[home + emp], kEmpty32, key);
                                if (old == kEmpty32 || old == key) {
                                    sl = (int)home + emp;
                                    break;
                                }
                            } else {
                                home = (home + 4) & (S - 1);
                            }
                            q4 = *reinterpret_cast<const int4*>(&t_key[home]);
                        }
                    }
                    if (sl < 0) {
                        full = true;
                        continue;
                    }
                    atomicAdd(&t_cs[sl], 1u);
                    lds_val(&t_v[sl], vr[u], vt, true);
                }
            };
            // the split fire's insert. A bucket fills in slot order and keys are never
            // removed, so a key present in a bucket sits before its first empty slot: the common
            // case -- the key in its home bucket -- is four compares and a select, no branch; the
            // lanes whose key is not there (its first record in this fire, or a full home bucket)
            // claim a slot by CAS or probe on, in a loop entered only when some lane needs it; the
            // adds are unconditional (lanes without a record add into the dummy slot)
            auto insert_hot = [&](const int32_t (&kr)[kTileRpl], const int64_t (&vr)[kTileRpl], uint32_t nrec) {
                const bool hot = vt >= 0 && vt <= 2;   // (SUM-family value ops: pre-combine hot keys)
                uint32_t hm[kTileRpl];
                int4 bq[kTileRpl];
                int sl[kTileRpl];
                uint32_t cn[kTileRpl];   // records a lane adds (> 1: a hot key's wave pre-combined)
                int64_t va[kTileRpl];
#pragma unroll
                for (int u = 0; u < kTileRpl; u++) {   // every home bucket read first, then resolved
                    hm[u] = __umulhi((uint32_t)kr[u] * 0x9E3779B1u, (uint32_t)(S / 4)) * 4;
                    bq[u] = *reinterpret_cast<const int4*>(&t_key[hm[u]]);
                    cn[u] = 1u;
                    va[u] = vr[u];
                }
                bool pend[kTileRpl];
#pragma unroll
                for (int u = 0; u < kTileRpl; u++) {
                    const int32_t key = kr[u];
                    bool valid = lane + 64 * u < (int)nrec;
                    if (retry) valid = valid && (int)((uint64_t)mix_of((int64_t)key) >> (64 - p.region_bits)) == r_lo;
                    if (hot) {
                        // skewed pass: the records of the wave's first key (a hot key, when it is
                        // the key of 16+ lanes) are added once, by one lane, with their count and
                        // value sum (SUM-family value ops only); the other lanes of it add nothing
                        const int32_t k0 = __builtin_amdgcn_readfirstlane(key);
                        const bool mine = valid && key == k0;
                        const uint64_t m = __ballot(mine);
                        if (__popcll(m) >= 16) {   // (uniform)
                            int64_t sv = mine ? vr[u] : 0;   // (0 bits: +0.0 and 0, the sum identity)
#pragma unroll
                            for (int off = 32; off > 0; off >>= 1) {
                                const int64_t o = __shfl_xor(sv, off);
                                if (vt == 2) sv = __double_as_longlong(__longlong_as_double(sv) + __longlong_as_double(o));
                                else sv += o;
                            }
                            const int leader = __ffsll((long long)m) - 1;
                            if (mine) {
                                if (lane == leader) {
                                    cn[u] = (uint32_t)__popcll(m);
                                    va[u] = sv;
                                } else {
                                    valid = false;
                                }
                            }
                        }
                    }
                    const int4 q4 = bq[u];
                    int z = q4.w == key ? 3 : -1;
                    z = q4.z == key ? 2 : z;
                    z = q4.y == key ? 1 : z;
                    z = q4.x == key ? 0 : z;
                    int s0 = z >= 0 ? (int)hm[u] + z : -1;
                    s0 = key == kEmpty32 ? S : s0;
                    pend[u] = valid && s0 < 0;
                    sl[u] = valid ? s0 : kDummy;
                }
#pragma unroll
                for (int u = 0; u < kTileRpl; u++) {
                    if (__ballot(pend[u]) == 0) continue;   // (uniform)
                    if (!pend[u]) continue;
                    const int32_t key = kr[u];
                    uint32_t home = hm[u];
                    int4 q4 = bq[u];
                    int found = -1;
                    for (int probe = 0; probe < S / 4 && found < 0; probe++) {
                        const int32_t qq[4] = {q4.x, q4.y, q4.z, q4.w};
                        int hit = -1, emp = -1;
#pragma unroll
                        for (int z = 3; z >= 0; z--) {
                            if (qq[z] == key) hit = z;
                            if (qq[z] == kEmpty32) emp = z;
                        }
                        if (hit >= 0 && (emp < 0 || hit < emp)) {
                            found = (int)home + hit;
                        } else if (emp >= 0) {
                            const int old = atomicCAS(&t_key[home + emp], kEmpty32, key);
                            if (old == kEmpty32 || old == key) found = (int)home + emp;
                            else q4 = *reinterpret_cast<const int4*>(&t_key[home]);   // (lost the slot: again)
                        } else {
                            home = (home + 4) & (S - 1);
                            q4 = *reinterpret_cast<const int4*>(&t_key[home]);
                        }
                    }
                    if (found < 0) full = true;
                    sl[u] = found >= 0 ? found : kDummy;
                }
#pragma unroll
                for (int u = 0; u < kTileRpl; u++) {
                    atomicAdd(&t_cs[sl[u]], cn[u]);
                    lds_val(&t_v[sl[u]], va[u], vt, true);
                }
            };
            auto insert = [&](const int32_t (&kr)[kTileRpl], const int64_t (&vr)[kTileRpl], uint32_t nrec) {
                if constexpr (HOT) {
                    insert_hot(kr, vr, nrec);
                } else {
#if defined(FG_INSERT_GENERIC)
                    insert_plain(std::false_type{}, std::true_type{}, kr, vr, nrec);
#else
                    if (retry) insert_plain(std::false_type{}, std::true_type{}, kr, vr, nrec);
                    else if (nrec == (uint32_t)kTileWin) insert_plain(std::true_type{}, std::false_type{}, kr, vr, nrec);
                    else insert_plain(std::false_type{}, std::false_type{}, kr, vr, nrec);
#endif
                }
            };
            for (int pi = 0; pi < f.n_passes; pi++) {
                const TilePass tp = tile_pass(f, pi);
                int32_t t_lo = 0, t_hi = tp.nt;
                if (split) {   // the item's range of the concatenated tile sequence, in this pass
                    t_lo = g_lo - f.sp.gpre[pi] > 0 ? g_lo - f.sp.gpre[pi] : 0;
                    t_hi = g_hi - f.sp.gpre[pi] < tp.nt ? g_hi - f.sp.gpre[pi] : tp.nt;
                    if (t_lo >= t_hi) continue;
                }
                TileWalk w;
                tile_walk_begin(w, tp, (tp.lane << (f.tbits - kTileBits)) | item, wave, W, lane, t_lo, t_hi,
#if defined(FG_WALK_STATIC)
                                nullptr);
#else
                                pi < kMaxTilePasses ? &s_gnext[pi] : nullptr);
#endif
                int32_t ka[kTileRpl], kb[kTileRpl];
                int64_t va[kTileRpl], vb[kTileRpl];
                uint32_t na = 0, nb = 0;
                bool more = tile_walk_next(w, s_fm[wave], s_dl[wave], lane, ka, va, na);
                FSTAMP(1);
                while (more) {   // (buffer roles static: the loop is unrolled by two)
                    const bool hb = tile_walk_next(w, s_fm[wave], s_dl[wave], lane, kb, vb, nb);
                    FSTAMP(1);
                    FWAIT(ka, va);
                    FSTAMP(2);
                    insert(ka, va, na);
                    FSTAMP(3);
                    if (!hb) break;
                    more = tile_walk_next(w, s_fm[wave], s_dl[wave], lane, ka, va, na);
                    FSTAMP(1);
                    FWAIT(kb, vb);
                    FSTAMP(2);
                    insert(kb, vb, nb);
                    FSTAMP(3);
                }
                if (__ballot(w.bad) != 0 && lane == 0) atomicOr(p.overflow, 8u);
            }
        }
        if (full) atomicOr(&s_flags, 4u);
#if defined(FG_DIAG_FIRE)
        if (diag_sink == 0x5EEDull) atomicOr(p.overflow, 0u);
#endif
        FSTAMP(4);
        __syncthreads();
        FSTAMP(5);
        {
#if !defined(FG_FIRE_HOIST)
        const TileFire& f = (&fa)[opaque_zero()];
        const MergeParams& p = f.m;
#endif
        // compaction: the occupied slots' ranks (round k covers slots [k*T, (k+1)*T); the last
        // round the sentinel slot), a dense rank -> slot map, then one row per lane
        uint32_t occ_mask = 0;
        // a key's region at the current bits, relative to the item's first
        auto region_of = [&](int slot) -> int {
            const int64_t key = slot == S ? (int64_t)kEmpty32 : (int64_t)t_key[slot];
            return (int)((uint64_t)mix_of(key) >> (64 - p.region_bits)) - r_lo;
        };
#pragma unroll
        for (int r = 0; r < kRounds; r++) {
            const int slot = r < kRounds - 1 ? r * T + tid : S;
            const bool occ = (r < kRounds - 1 || tid == 0) && t_cs[slot] != 0;
            const uint64_t bal = __ballot(occ);
            if (occ) occ_mask |= 1u << r;
            if (lane == 0) s_grp[r * W + wave] = (uint32_t)__popcll(bal);
            if (dst && !to_part && occ && live) atomicAdd(&s_rc[region_of(slot)], 1u);
        }
        __syncthreads();
        if (wave == 0) {
            constexpr int NG = kRounds * W;
            constexpr int GPL = (NG + 63) / 64;   // groups per lane
            uint32_t gv[GPL], xs = 0;
#pragma unroll
            for (int q = 0; q < GPL; q++) {
                gv[q] = GPL * lane + q < NG ? s_grp[GPL * lane + q] : 0u;
                xs += gv[q];
            }
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(xs, off);
                if (lane >= off) xs += y;
            }
            uint32_t ex = xs;
#pragma unroll
            for (int q = 0; q < GPL; q++) ex -= gv[q];
#pragma unroll
            for (int q = 0; q < GPL; q++) {
                if (GPL * lane + q < NG) s_grp[GPL * lane + q] = ex;
                ex += gv[q];
            }
            const uint32_t total = __shfl(xs, 63);
            bool over = false;   // a destination region above its capacity: the item fails
            if (dst && !to_part)
                for (int q = lane; q < r_hi - r_lo; q += 64) over = over || s_rc[q] > (uint32_t)kRegionCap;
            over = __ballot(over) != 0;
            if (lane == 0) {
                unsigned int fl = s_flags | (over ? 4u : 0u);
                if (live && !(fl & 4u) && !to_part && (!TAB || p.emit)) {
                    const unsigned long long ob = atomicAdd(p.out_count, (unsigned long long)total);
                    s_out_base = ob;
                    if ((int64_t)(ob + total) > p.out_cap) fl |= 2u;
                }
                if (live && !(fl & 4u) && to_part) {   // a chunk of a split bucket: its partial entries
                    const uint32_t ob = atomicAdd(f.sp.part_fill, total);
                    s_out_base = ob;
                    if ((uint64_t)ob + total > (uint64_t)f.sp.part_cap) fl |= 2u;
                    f.sp.part_off[part] = ob;
                    f.sp.part_n[part] = total;
                }
                if (live && to_part && (fl & 4u)) f.sp.part_n[part] = kChunkFailed;
                s_flags = fl;
                s_total = total;
                if (fl) atomicOr(p.overflow, fl);
                // the item does nothing; the host redoes its regions (a split bucket's regions are
                // listed by its first failing chunk only, and its merge skips it)
                if (live && (fl & 4u) && p.fail_list && (!to_part || atomicExch(&f.sp.bfail[item], 1u) == 0u)) {
                    const uint32_t nr = (uint32_t)(r_hi - r_lo);
                    const uint32_t at = atomicAdd(p.fail_n, nr);
                    for (uint32_t q = 0; q < nr; q++)
                        if (at + q < (uint32_t)p.fail_cap)
                            p.fail_list[at + q] = ((uint32_t)p.job << kFailJobShift) | (uint32_t)(r_lo + (int)q);
                }
            }
        }
        __syncthreads();
        const unsigned int fl = s_flags;
#pragma unroll
        for (int r = 0; r < kRounds; r++) {
            const bool occ = (occ_mask >> r) & 1;
            const uint64_t bal = __ballot(occ);
            if (occ) s_map[s_grp[r * W + wave] + (uint32_t)__popcll(bal & ((1ull << lane) - 1))] =
                (uint16_t)(r < kRounds - 1 ? r * T + tid : S);
        }
        __syncthreads();
        FSTAMP(6);
        if (live && to_part && !(fl & 6u)) {   // partial entries (LDS repr), merged later
            const uint32_t total = s_total;
            const uint32_t ob = (uint32_t)s_out_base;
            for (uint32_t i = tid; i < total; i += T) {
                const int sl = s_map[i];
                f.sp.p_key[ob + i] = sl == S ? kEmpty32 : t_key[sl];
                f.sp.p_cs[ob + i] = t_cs[sl];
                f.sp.p_v[ob + i] = t_v[sl];
            }
        } else if (live && (!TAB || p.emit) && !(fl & 6u)) {
            const uint32_t total = s_total;
            const unsigned long long ob = s_out_base;
            for (uint32_t i = tid; i < total; i += T) {
                const int sl = s_map[i];
                const int64_t v = lds_repr(vt, (int64_t)t_v[sl]);
                write_row_k<TAB>(p, ob + i, sl == S ? (int64_t)kEmpty32 : (int64_t)t_key[sl], t_cs[sl], 0ull, &v, vt);
            }
        }
        if (TAB && dst && live && !to_part && !(fl & 5u)) {
            // the regions' counts and bases (exclusive prefix, wave 0), the rank -> slot map
            // rebuilt region-major (s_map is free once the rows are out), then every region's
            // entries written at consecutive ranks: full-width stores into each SoA column
            constexpr int cap = kRegionCap;
            const int nreg = r_hi - r_lo;
            __syncthreads();   // (the emit's reads of s_map are done)
            if (wave == 0) {
                constexpr int RPL = kTileMaxRegions / 64;
                uint32_t c[RPL], x = 0;
#pragma unroll
                for (int q = 0; q < RPL; q++) {
                    c[q] = RPL * lane + q < nreg ? s_rc[RPL * lane + q] : 0u;
                    x += c[q];
                }
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t y = __shfl_up(x, off);
                    if (lane >= off) x += y;
                }
                uint32_t ex = x;
#pragma unroll
                for (int q = 0; q < RPL; q++) ex -= c[q];
#pragma unroll
                for (int q = 0; q < RPL; q++) {
                    const int rr = RPL * lane + q;
                    if (rr < nreg) {
                        const uint32_t old = p.dst.counts[r_lo + rr];
                        p.dst.counts[r_lo + rr] = c[q];
                        if (p.dst_total) atomicAdd(p.dst_total, (unsigned long long)((int64_t)c[q] - (int64_t)old));
                        s_rb[rr] = ex;   // region rr's first rank
                        s_rc[rr] = ex;   // (its cursor)
                    }
                    ex += c[q];
                }
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < kRounds; r++) {
                if (!((occ_mask >> r) & 1)) continue;
                const int slot = r < kRounds - 1 ? r * T + tid : S;
                s_map[atomicAdd(&s_rc[region_of(slot)], 1u)] = (uint16_t)slot;
            }
            __syncthreads();
            const uint32_t total = s_total;
            for (uint32_t i = tid; i < total; i += T) {
                int lo = 0, hi = nreg;   // the region of rank i: the last base <= i
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (s_rb[mid] <= i) lo = mid;
                    else hi = mid;
                }
                const int sl = s_map[i];
                const uint32_t at = i - s_rb[lo];
                int64_t* db = p.dst.base + (int64_t)(r_lo + lo) * 4 * cap;
                const int32_t k32 = sl == S ? kEmpty32 : t_key[sl];
                if (p.dst.narrow) {   // 16-B entries: [int32 key][u32 COUNT(*)][value]
                    reinterpret_cast<int32_t*>(db)[at] = k32;
                    reinterpret_cast<uint32_t*>(db)[cap + at] = t_cs[sl];
                    db[cap + at] = lds_repr(vt, (int64_t)t_v[sl]);
                } else {
                    db[at] = mix_of((int64_t)k32);
                    db[cap + at] = (int64_t)t_cs[sl];
                    db[2 * cap + at] = 0;
                    db[3 * cap + at] = lds_repr(vt, (int64_t)t_v[sl]);
                }
            }
        }
        }
        __syncthreads();   // the table is cleared for the next item
        FSTAMP(7);
    }
#ifdef FG_STAMPS
    if (fa.m.stamps && lane == 0)
        for (int i = 0; i < 8; i++) atomicAdd(&fa.m.stamps[i], fst_acc[i]);
#endif
#undef FSTAMP
#undef FWAIT
}

hipError_t launch_tile_fire(const TileFire& f, int32_t workgroups, hipStream_t s) {
    if (f.n_passes < 1 || f.tbits < kTileBits || f.m.region_bits < f.tbits || f.m.mv) return hipErrorInvalidValue;
    if (f.m.has_dst || f.m.n_src > 0) {
        // s_rc holds an item's regions and s_rb its (source, region) ranges: an item is one
        // region on a retry, else the 2^(kTileBits + sub) regions of its bucket
        if (f.m.src_null_mask) return hipErrorInvalidValue;   // (sources without NULL counts)
        const int sub = kTileBits + f.m.region_bits - f.tbits;
        if (!f.m.retry_list && sub > kTileMaxRegionBits) return hipErrorInvalidValue;
        const int64_t nreg = f.m.retry_list ? 1 : (int64_t)1 << sub;
        if ((int64_t)f.m.n_src * nreg > kTileMaxRegions) return hipErrorInvalidValue;
    }
    const dim3 g((unsigned)workgroups), b(kTileFireThreads);
    const bool tab = f.m.has_dst || f.m.n_src > 0;
    // the value op compiled in: SUM / AVG over DOUBLE, BIGINT, or COUNT only
    if (f.split && !f.merge && !f.sp.next_item) return hipErrorInvalidValue;
    if (f.merge && (!f.split || !f.sp.split_b || !f.sp.n_split)) return hipErrorInvalidValue;
    const bool hot = f.hot && f.split && !f.merge && f.m.val_type >= 0 && f.m.val_type <= 2;
    const int sm = !f.split ? 0 : hot ? 2 : 1;
#define FG_TILE_FIRE_SM(V, TB)                                                     \
    do {                                                                           \
        if (sm == 0) fg_launch((k_tile_fire<V, TB, 0>), g, b, 0, s, f);            \
        else if (sm == 1) fg_launch((k_tile_fire<V, TB, 1>), g, b, 0, s, f);       \
        else fg_launch((k_tile_fire<V, TB, 2>), g, b, 0, s, f);                    \
    } while (0)
#define FG_TILE_FIRE(V)                          \
    do {                                         \
        if (tab) FG_TILE_FIRE_SM(V, true);       \
        else FG_TILE_FIRE_SM(V, false);          \
    } while (0)
    switch (f.m.val_type) {
        case 2: FG_TILE_FIRE(2); break;
        case 1: FG_TILE_FIRE(1); break;
        case 0: FG_TILE_FIRE(0); break;
        default: FG_TILE_FIRE(-1); break;
    }
#undef FG_TILE_FIRE
#undef FG_TILE_FIRE_SM
    return hipGetLastError();
}

// ---- split (skewed) tile fires ---------------------------------------------------------------
// k_tile_plan (one workgroup): per bucket of the lane, its records over the fire's passes (the
// passes' btot); a bucket above kTileChunk records becomes K = ceil(records / kTileChunk) chunk
// items over equal ranges of the passes' concatenated tiles (records of a Zipf hot key spread
// evenly over the tiles, as the stream does), the others one item each; the items, the split
// entries and the counts are written for k_tile_fire (its items, then its merge of the split
// buckets).
constexpr int kTilePlanThreads = 1024;
__global__ __launch_bounds__(kTilePlanThreads) void k_tile_plan(TileFire f) {
    __shared__ uint32_t s_wave[kTilePlanThreads / 64];
    const TileSplit& sp = f.sp;
    const int nb = 1 << (f.tbits - kTileBits);
    const int tid = threadIdx.x;
    const int32_t G = sp.gpre[f.n_passes];
    constexpr int BPT = kMaxTileBuckets / kTilePlanThreads;   // buckets per thread (consecutive)
    uint32_t kk[BPT], tb[BPT], mine = 0, nitem = 0, nsplit = 0, nchunk = 0;
#pragma unroll
    for (int q = 0; q < BPT; q++) {
        const int bk = tid * BPT + q;
        tb[q] = 0;
        if (bk >= nb) continue;
        for (int pi = 0; pi < f.n_passes; pi++) {
            const TilePass tp = tile_pass(f, pi);
            if (tp.btot) tb[q] += gbl(tp.btot)[(tp.lane << (f.tbits - kTileBits)) | bk];
        }
        mine += tb[q];
    }
    // chunk size: kTileChunk records, at least the lane's mean bucket -- a split bucket's chunks are
    // items of a normal bucket's size (the fire fetches items dynamically)
    uint32_t lane_total;
    (void)block_exclusive_scan(mine, s_wave, &lane_total);
    const uint64_t chunk = sp.chunk ? (uint64_t)sp.chunk : max((uint64_t)kTileChunk, (uint64_t)lane_total / (uint64_t)nb);
#pragma unroll
    for (int q = 0; q < BPT; q++) {
        const int bk = tid * BPT + q;
        kk[q] = 0;
        if (bk >= nb) continue;
        uint64_t k = tb[q] > chunk ? (tb[q] + chunk - 1) / chunk : 1;
        if (k > (uint64_t)G) k = G > 0 ? (uint64_t)G : 1;
        kk[q] = (uint32_t)k;
        nitem += (uint32_t)k;
        if (k > 1) {
            nsplit++;
            nchunk += (uint32_t)k;
        }
    }
    uint32_t t_item, t_split, t_chunk;
    const uint32_t b_item = block_exclusive_scan(nitem, s_wave, &t_item);
    const uint32_t b_split = block_exclusive_scan(nsplit, s_wave, &t_split);
    const uint32_t b_chunk = block_exclusive_scan(nchunk, s_wave, &t_chunk);
    const bool fits = t_item <= (uint32_t)sp.max_items && t_split <= (uint32_t)sp.max_split;
    if (tid == 0) {
        *sp.n_items = fits ? t_item : 0u;
        *sp.n_split = fits ? t_split : 0u;
        if (!fits) atomicOr(f.m.overflow, 2u);   // (the host sized the lists from the lane's records)
    }
    if (!fits) return;
    uint32_t it = b_item, si = b_split, ci = b_chunk;
#pragma unroll
    for (int q = 0; q < BPT; q++) {
        const int bk = tid * BPT + q;
        const uint32_t k = kk[q];
        if (k == 0) continue;
        if (k > 1) {
            sp.split_b[si] = bk;
            sp.split_c0[si] = (int32_t)ci;
            sp.split_k[si] = (int32_t)k;
            sp.bfail[bk] = 0u;
            si++;
        }
        for (uint32_t c = 0; c < k; c++) {
            TileItem x;
            x.bucket = bk;
            x.g_lo = k > 1 ? (int32_t)((int64_t)G * c / k) : 0;
            x.g_hi = k > 1 ? (int32_t)((int64_t)G * (c + 1) / k) : G;
            x.part = k > 1 ? (int32_t)(ci + c) : -1;
            sp.items[it + c] = x;
        }
        it += k;
        if (k > 1) ci += k;
    }
}

hipError_t launch_tile_plan(const TileFire& f, hipStream_t s) {
    if (!f.split || f.n_passes < 1 || f.n_passes > kMaxTilePasses || (1 << (f.tbits - kTileBits)) > kMaxTileBuckets ||
        !f.sp.items || !f.sp.n_items || !f.sp.split_b || !f.sp.n_split || !f.sp.bfail)
        return hipErrorInvalidValue;
    fg_launch(k_tile_plan, dim3(1), dim3(kTilePlanThreads), 0, s, f);
    return hipGetLastError();
}

// Materialize a tile pass's lane into a regular narrow staged pass, over the items of a plan
// (k_tile_plan with sp.chunk = kTileMatChunk: a bucket above that many records is cut into equal
// tile ranges, so a hot key's bucket is spread over many workgroups and no workgroup gets more
// than ~kTileMatChunk records). Persistent workgroups take items in turn; an item's tiles are
// walked kTileMatThreads at a time (one directory entry per thread, their lengths scanned into a
// flat record sequence, kTileMatU records in flight per thread). COUNT: the item's records per
// region at `bits` into icnt[item][sub-region] and added into hist (zeroed by the host). SCATTER:
// each region's block of the item reserved at once from cursor[region] (the exclusive scan of
// hist, copied) by its icnt, the records written at their rank (order inside a region is
// immaterial).
constexpr int kTileMatThreads = 256;
constexpr int kTileMatU = 4;
template <bool SCATTER>
__global__ __launch_bounds__(kTileMatThreads) void k_tile_mat(TilePass tp, int32_t bits, const TileItem* items,
                                                              const uint32_t* n_items, uint32_t* icnt,
                                                              uint32_t* hist_or_cursor, void* out) {
    constexpr int T = kTileMatThreads, U = kTileMatU;
    __shared__ uint32_t s_c[kTileMaxSub];
    __shared__ uint32_t s_pre[T + 1];
    __shared__ uint32_t s_x[T];
    __shared__ uint32_t s_wave[T / 64];
    const int sub = bits - tp.bits;
    const int nsub = 1 << (kTileBits + sub);   // (host: kTileBits + sub <= 6)
    const int tid = threadIdx.x;
    const uint32_t NI = *gbl(n_items);
    for (uint32_t x = blockIdx.x; x < NI; x += gridDim.x) {
        const TileItem it = items[x];
        const int r_lo = it.bucket << (kTileBits + sub);
        const uint32_t* col = tp.dt + (int64_t)((tp.lane << (tp.bits - kTileBits)) | it.bucket) * tp.nt;
        if (tid < nsub) {
            uint32_t c0 = 0;
            if (SCATTER) {
                const uint32_t c = icnt[(uint64_t)x * kTileMaxSub + tid];
                if (c) c0 = atomicAdd(&hist_or_cursor[r_lo + tid], c);
            }
            s_c[tid] = c0;
        }
        const int32_t g_hi = it.g_hi < tp.nt ? it.g_hi : tp.nt;
        for (int32_t t0 = it.g_lo; t0 < g_hi; t0 += T) {
            const uint32_t xd = t0 + tid < g_hi ? gbl(col)[t0 + tid] : 0u;
            uint32_t total;
            const uint32_t ex = block_exclusive_scan(xd >> 16, s_wave, &total);   // (synchronizes)
            s_pre[tid] = ex;
            s_x[tid] = xd;
            if (tid == 0) s_pre[T] = total;
            __syncthreads();
            if (total > 0) {   // (uniform)
                auto rec_at = [&](uint32_t i) -> uint64_t {   // its tile: the last prefix <= i
                    int lo = 0, hi = T;
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (s_pre[mid] <= i) lo = mid;
                        else hi = mid;
                    }
                    return (uint64_t)(t0 + lo) * kTileRecs + (s_x[lo] & 0xffffu) + (i - s_pre[lo]);
                };
                for (uint32_t i0 = 0; i0 < total; i0 += U * T) {
                    Rec12 r[U];
                    int rg[U];
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const uint32_t i = i0 + u * T + tid;
                        if (i < total) r[u] = ld_tile_rec(tp.rec, rec_at(i));
                    }
#pragma unroll
                    for (int u = 0; u < U; u++)
                        rg[u] = i0 + u * T + tid < total
                                    ? (int)((uint64_t)mix_of((int64_t)(int32_t)r[u].k) >> (64 - bits)) - r_lo : -1;
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        if (rg[u] < 0) continue;
                        const uint32_t pos = atomicAdd(&s_c[rg[u]], 1u);
                        if (SCATTER) st_rec12(out, pos, (int64_t)(int32_t)r[u].k, rec12_val(r[u]));
                    }
                }
            }
            __syncthreads();   // (s_pre / s_x are rewritten by the next tile range)
        }
        if (!SCATTER && tid < nsub) {
            const uint32_t c = s_c[tid];
            icnt[(uint64_t)x * kTileMaxSub + tid] = c;
            if (c) atomicAdd(&hist_or_cursor[r_lo + tid], c);
        }
        __syncthreads();   // (s_c is reset by the next item)
    }
}

hipError_t launch_tile_count(const TilePass& tp, int32_t bits, const TileSplit& plan, uint32_t* hist,
                             int32_t workgroups, hipStream_t s) {
    if (bits - tp.bits + kTileBits > 6 || tp.nt <= 0 || !plan.items || !plan.n_items || !plan.icnt || workgroups < 1)
        return hipErrorInvalidValue;   // (kTileMaxSub regions per bucket)
    fg_launch(k_tile_mat<false>, dim3((unsigned)workgroups), dim3(kTileMatThreads), 0, s, tp, bits,
              (const TileItem*)plan.items, (const uint32_t*)plan.n_items, plan.icnt, hist, (void*)nullptr);
    return hipGetLastError();
}

hipError_t launch_tile_scatter(const TilePass& tp, int32_t bits, const TileSplit& plan, uint32_t* cursor, void* out_rec,
                               int32_t workgroups, hipStream_t s) {
    if (bits - tp.bits + kTileBits > 6 || tp.nt <= 0 || !plan.items || !plan.n_items || !plan.icnt || workgroups < 1)
        return hipErrorInvalidValue;
    fg_launch(k_tile_mat<true>, dim3((unsigned)workgroups), dim3(kTileMatThreads), 0, s, tp, bits,
              (const TileItem*)plan.items, (const uint32_t*)plan.n_items, plan.icnt, cursor, out_rec);
    return hipGetLastError();
}

}  // namespace fg
