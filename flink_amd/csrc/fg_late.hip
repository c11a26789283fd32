// fg_late.hip -- DataStream allowed lateness (WindowedStream.allowedLateness) on the GPU.
//
// WindowOperator with allowedLateness L > 0 (SJ/runtime/operators/windowing/WindowOperator.java):
//   * a window is late once cleanupTime = maxTimestamp + L (Long.MAX_VALUE on overflow,
//     :669-673) <= the watermark (isWindowLate :608-611); an element skipped by all of its
//     windows counts as dropped when timestamp + L <= watermark (isElementLate :620-622);
//   * a fired window keeps its state until the cleanup timer (:630-642, onEventTime :493-496);
//   * an element of a fired window that is not late FIREs it at once (EventTimeTrigger.onElement
//     :37-46): the window's contents are emitted right after the element joined them
//     (emitWindowContents :574-579, timestamp maxTimestamp); a PurgingTrigger then clears them
//     (FIRE_AND_PURGE), so the next element fires with itself alone.
//
// The ingest splits every batch (k_late_split): elements of a fired, not yet cleaned window
// ("late-allowed") go to a late list, the rest take the regular path (whose late rule -- drop
// when the last window fired -- is then exactly isWindowLate for every window). The late list
// is processed in rounds, one element per key per round, oldest first (k_late_claim: the
// smallest arrival index per key), so that a key's rows come out in arrival order with the
// state each element saw: per round k_late_lookup finds the key's entry in the element's slice
// table (and reserves room for the new ones), k_late_update adds the element, k_late_emit sums
// the key's entries over every fired, not cleaned window holding the slice and writes the row.
// Slice tables are the engine's (regions of SoA entries keyed by fmix64 mix); a region is
// scanned by one wave (64 keys per step).
#include <hip/hip_runtime.h>

#include "fg_late.h"

namespace fg {

namespace {

constexpr int kLateThreads = 256;
constexpr unsigned long long kClaimEmpty = 0x8000000000000000ull;   // (the mix equal to it has its own slot)

__device__ __forceinline__ unsigned long long wave_reserve(unsigned long long* ctr, uint32_t amount) {
    const int lane = threadIdx.x & 63;
    uint32_t x = amount;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    const uint32_t total = __shfl(x, 63);
    unsigned long long base = 0;
    if (lane == 63 && total) base = atomicAdd(ctr, (unsigned long long)total);
    base = __shfl(base, 63);
    return base + x - amount;
}

__device__ __forceinline__ int64_t region_of(int64_t mix, int bits) {
    return bits == 0 ? 0 : (int64_t)((uint64_t)mix >> (64 - bits));
}

// table of the slice ending at se (binary search over the sorted directory), or -1
__device__ __forceinline__ int dir_find(const LateDir& d, int64_t se) {
    int lo = 0, hi = d.n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (d.se[mid] < se) lo = mid + 1;
        else hi = mid;
    }
    return lo < d.n && d.se[lo] == se ? lo : -1;
}

// one wave scans region r of table t for `mix`: its entry index, or -1 (all lanes agree)
__device__ __forceinline__ int wave_find(const TableRef& t, int64_t r, int cap, int cols, int64_t mix) {
    const int lane = threadIdx.x & 63;
    const uint32_t n = t.counts[r];
    const int64_t* keys = t.base + r * cols * cap;
    for (uint32_t b = 0; b < n; b += 64) {
        const uint32_t i = b + lane;
        const bool hit = i < n && keys[i] == mix;
        const uint64_t m = __ballot(hit);
        if (m) return (int)(b + __ffsll((long long)m) - 1);
    }
    return -1;
}

// acc (+) v under the kernel value op vt = val_type | op << 2: op 0 the sum (SumAggregator),
// 1 / 2 BIGINT MIN / MAX, 3 / 4 DOUBLE MIN / MAX by Double.compareTo (ComparableAggregator,
// fg_kernels.hip kVtMinT): the order of canonical bits mapped to ordered integers
__device__ __forceinline__ int64_t canon_bits(int64_t b) {   // Double.doubleToLongBits
    return (b & 0x7FFFFFFFFFFFFFFFll) > 0x7FF0000000000000ll ? 0x7FF8000000000000ll : b;
}
__device__ __forceinline__ int64_t ord_of(int64_t b) { return b >= 0 ? b : b ^ 0x7FFFFFFFFFFFFFFFll; }
__device__ __forceinline__ int64_t add_value(int vt, int64_t acc, int64_t v) {
    switch (vt >> 2) {
        case 1: return v < acc ? v : acc;
        case 2: return v > acc ? v : acc;
        case 3: acc = canon_bits(acc); v = canon_bits(v); return ord_of(v) < ord_of(acc) ? v : acc;
        case 4: acc = canon_bits(acc); v = canon_bits(v); return ord_of(v) > ord_of(acc) ? v : acc;
        default: break;
    }
    if ((vt & 3) == 2) return __double_as_longlong(__longlong_as_double(acc) + __longlong_as_double(v));
    return (int64_t)((uint64_t)acc + (uint64_t)v);   // Java long wrap
}

}  // namespace

// ---- split ----------------------------------------------------------------------------------
__global__ __launch_bounds__(kLateThreads) void k_late_split(LateSplit p) {
    const int64_t i0 = (int64_t)blockIdx.x * kLateThreads + threadIdx.x;
    const bool valid = i0 < p.n;
    const int64_t i = valid ? i0 : 0;
    const int64_t key = p.key[i], ts = p.ts[i];
    const int64_t val = p.val ? p.val[i] : 0;
    const uint8_t nul = p.vnull ? p.vnull[i] : 0;
    const LateClass c = late_class(p.w, ts, p.wm, p.lateness);
    const bool late = valid && c.late_allowed;
    const bool regular = valid && (!c.late_allowed || (p.purging && !c.last_fired));
    const unsigned long long at_l = wave_reserve(&p.counts[0], late ? 1u : 0u);
    const unsigned long long at_r = wave_reserve(&p.counts[1], regular ? 1u : 0u);
    if (late) {
        p.l_mix[at_l] = mix_of(key);
        p.l_se[at_l] = c.slice_end;
        p.l_val[at_l] = val;
        p.l_null[at_l] = nul;
        p.l_idx[at_l] = (uint32_t)i;
    }
    if (regular) {
        p.r_key[at_r] = key;
        p.r_ts[at_r] = ts;
        if (p.val) p.r_val[at_r] = val;
        if (p.vnull) p.r_null[at_r] = nul;
    }
}

// ---- rounds -----------------------------------------------------------------------------------
__global__ __launch_bounds__(kLateThreads) void k_late_reset(LateRound p) {
    const uint64_t i = (uint64_t)blockIdx.x * kLateThreads + threadIdx.x;
    if (i <= p.claim_mask + 1) {
        p.claim_key[i] = kClaimEmpty;
        p.claim_idx[i] = 0xFFFFFFFFu;
    }
    if (i == 0) {
        *p.flags = 0;
        *p.nsel = 0;
    }
}

// the smallest arrival index of every pending key (insert-or-min into an open-addressing table)
__global__ __launch_bounds__(kLateThreads) void k_late_claim(LateRound p) {
    const int64_t j = (int64_t)blockIdx.x * kLateThreads + threadIdx.x;
    if (j >= p.n || p.done[j]) return;
    const unsigned long long k = (unsigned long long)p.mix[j];
    uint64_t s;
    if (k == kClaimEmpty) {
        s = p.claim_mask + 1;   // the sentinel mix: its own slot
    } else {
        s = fmix64(k ^ 0x9E3779B97F4A7C15ull) & p.claim_mask;
        for (;;) {
            const unsigned long long old = atomicCAS(&p.claim_key[s], kClaimEmpty, k);
            if (old == kClaimEmpty || old == k) break;
            s = (s + 1) & p.claim_mask;
        }
    }
    p.slot[j] = (uint32_t)s;
    atomicMin(&p.claim_idx[s], p.idx[j]);
}

// this round's elements (one per key): their entry in the slice table, and the room new
// entries need (need[table * P + region] counts them; the host splits regions when full)
__global__ __launch_bounds__(kLateThreads) void k_late_lookup(LateRound p) {
    const int64_t j = ((int64_t)blockIdx.x * kLateThreads + threadIdx.x) >> 6;   // one wave per element
    if (j >= p.n) return;
    const int lane = threadIdx.x & 63;
    const bool sel = !p.done[j] && p.claim_idx[p.slot[j]] == p.idx[j];
    if (lane == 0) {
        p.sel[j] = sel ? 1 : 0;
        if (sel) atomicAdd(p.nsel, 1ull);
    }
    if (!sel || p.purging) return;
    const int d = dir_find(p.dir, p.se[j]);
    if (d < 0) {
        if (lane == 0) atomicOr(p.flags, 2u);   // (the host creates the tables first: never)
        return;
    }
    const int64_t r = region_of(p.mix[j], p.region_bits);
    const int f = wave_find(p.dir.t[d], r, p.cap, p.cols, p.mix[j]);
    if (lane == 0) {
        p.found[j] = f;
        if (f < 0) {
            const uint32_t need = atomicAdd(&p.need[(int64_t)d * p.P + r], 1u) + 1;
            if (p.dir.t[d].counts[r] + need > (uint32_t)p.cap) atomicOr(p.flags, 1u);   // region full: split
        }
    }
}

// add each selected element to its (key, slice) entry: found -> in place, new -> appended
__global__ __launch_bounds__(kLateThreads) void k_late_update(LateRound p) {
    const int64_t j = (int64_t)blockIdx.x * kLateThreads + threadIdx.x;
    if (j >= p.n || !p.sel[j] || p.purging) return;
    const int d = dir_find(p.dir, p.se[j]);
    const TableRef t = p.dir.t[d];
    const int64_t r = region_of(p.mix[j], p.region_bits);
    int64_t* base = t.base + r * p.cols * p.cap;
    int64_t v = p.vnull && p.vnull[j] ? 0 : p.val[j];
    if ((p.vt >> 2) >= 3) v = canon_bits(v);   // DOUBLE MIN / MAX by compareTo: canonical NaN
    const int64_t nul = p.vnull ? p.vnull[j] : 0;
    int f = p.found[j];
    if (f < 0) {
        f = (int)atomicAdd(&t.counts[r], 1u);
        base[f] = p.mix[j];
        base[p.cap + f] = 1;
        base[2 * p.cap + f] = nul;
        base[3 * p.cap + f] = (p.vt & 3) == 2 && nul ? __double_as_longlong(0.0) : v;
        return;
    }
    base[p.cap + f] += 1;
    base[2 * p.cap + f] += nul;
    if (!nul) base[3 * p.cap + f] = add_value(p.vt, base[3 * p.cap + f], v);
}

// the rows: per selected element, every fired and not cleaned window holding its slice, with
// the key's state summed over the window's slices (PurgingTrigger: the element alone)
__global__ __launch_bounds__(kLateThreads) void k_late_emit(LateRound p) {
    const int64_t j = ((int64_t)blockIdx.x * kLateThreads + threadIdx.x) >> 6;   // one wave per element
    if (j >= p.n || !p.sel[j]) return;
    const int lane = threadIdx.x & 63;
    const WindowSpec& w = p.w;
    const int64_t se = p.se[j];
    const int64_t mix = p.mix[j];
    const int64_t r = region_of(mix, p.region_bits);
    const int64_t nwin = w.kind == TUMBLE ? 1 : w.size / w.slide;
    for (int64_t k = 0; k < nwin; k++) {
        const int64_t e = jadd(se, k * w.slide);   // windows holding the slice: ends se .. se + size - slide
        if (!ds_fired(e, p.wm) || ds_cleanup(e, p.lateness) <= p.wm) continue;
        int64_t cs = 0, cn = 0, sum = (p.vt & 3) == 2 ? __double_as_longlong(0.0) : 0;
        bool have = false;   // the first slice's accumulator is taken as it is (no identity)
        if (p.purging) {
            cs = 1;
            cn = p.vnull ? p.vnull[j] : 0;
            sum = cn ? sum : (p.vt >> 2) >= 3 ? canon_bits(p.val[j]) : p.val[j];
        } else {
            const int64_t ns = w.kind == TUMBLE ? 1 : w.size / w.slice;
            for (int64_t q = 0; q < ns; q++) {   // slices of window e: e - size + slice .. e
                const int64_t s2 = jsub(e, q * w.slice);
                const int d = dir_find(p.dir, s2);
                if (d < 0) continue;
                const int f = wave_find(p.dir.t[d], r, p.cap, p.cols, mix);
                if (f < 0) continue;
                const int64_t* base = p.dir.t[d].base + r * p.cols * p.cap;
                cs += base[p.cap + f];
                cn += base[2 * p.cap + f];
                sum = have ? add_value(p.vt, sum, base[3 * p.cap + f]) : base[3 * p.cap + f];
                have = true;
            }
        }
        if (lane != 0 || cs == 0) continue;
        const unsigned long long o = atomicAdd(p.out_count, 1ull);
        if ((int64_t)o >= p.out_cap) {
            atomicOr(p.flags, 4u);
            continue;
        }
        p.out_key[o] = key_of(mix);
        p.out_ws[o] = jsub(e, w.size);
        p.out_we[o] = e;
        p.out_rowtime[o] = jsub(e, 1);   // window.maxTimestamp()
        const int64_t cv = cs - cn;
        uint8_t nm = 0;
        for (int a = 0; a < p.num_aggs; a++) {
            int64_t v = 0;
            switch (p.aggs[a]) {
                case 0: v = cs; break;
                case 1: v = cv; break;
                case 4: v = sum; break;
                case 3:
                    if (cv == 0) nm |= (uint8_t)(1u << a);
                    else if ((p.vt & 3) == 2) v = __double_as_longlong(__longlong_as_double(sum) / (double)cv);
                    else v = sum / cv;
                    break;
                default:   // SUM (SumAggregator: the sum of the window's values)
                    if (cv == 0) nm |= (uint8_t)(1u << a);
                    else v = sum;
                    break;
            }
            p.out_agg[a][o] = v;
        }
        p.out_null[o] = nm;
    }
    if (lane == 0) p.done[j] = 1;
}

// ---- launches -------------------------------------------------------------------------------
namespace {
inline unsigned grid_of(int64_t n, int per_block) { return (unsigned)((n + per_block - 1) / per_block); }
}

hipError_t launch_late_split(const LateSplit& p, hipStream_t s) {
    if (p.n <= 0) return hipSuccess;
    fg_launch(k_late_split, dim3(grid_of(p.n, kLateThreads)), dim3(kLateThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_late_reset(const LateRound& p, hipStream_t s) {
    fg_launch(k_late_reset, dim3(grid_of((int64_t)p.claim_mask + 2, kLateThreads)), dim3(kLateThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_late_claim(const LateRound& p, hipStream_t s) {
    fg_launch(k_late_claim, dim3(grid_of(p.n, kLateThreads)), dim3(kLateThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_late_lookup(const LateRound& p, hipStream_t s) {
    fg_launch(k_late_lookup, dim3(grid_of(p.n, kLateThreads / 64)), dim3(kLateThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_late_update(const LateRound& p, hipStream_t s) {
    fg_launch(k_late_update, dim3(grid_of(p.n, kLateThreads)), dim3(kLateThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_late_emit(const LateRound& p, hipStream_t s) {
    fg_launch(k_late_emit, dim3(grid_of(p.n, kLateThreads / 64)), dim3(kLateThreads), 0, s, p);
    return hipGetLastError();
}

}  // namespace fg
