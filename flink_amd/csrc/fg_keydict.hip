// fg_keydict.hip -- grouping keys of any type: a GPU-resident dictionary of serialized key
// rows (BinaryRowData bytes), for the C-ABI fg_key_dict_* of include/flinkgpu.h.
//
// The reference groups by the key row the BinaryRowDataKeySelector projects
// (TR/keyselector/BinaryRowDataKeySelector.java:43-50): key identity is byte equality of the
// row (BinarySection.equals, TC/data/binary/BinarySection.java:62-73) and its hash is
// MurmurHashUtils.hashBytesByWords over the row's bytes, seed 42 (BinarySection.java:76-78 ->
// BinarySegmentUtils.hash -> MurmurHashUtils.java:92-96,131-170), which KeyGroupStreamPartitioner
// turns into a key group (KeyGroupRangeAssignment.java:63-77). The window engine aggregates
// 64-bit keys; this dictionary interns each distinct key row once and hands out an id
// (ordinal << kg_bits | key group): equal rows get equal ids, distinct rows distinct ids, so the
// aggregation by id is the aggregation by key row, and the id carries the row's key group
// (FG_KEYHASH_DICT_ID routes by it).
//
// Layout in HBM: an open-addressing table of `cap` 64-B slots -- one memory line -- {tag u64
// (a 64-bit hash of the row, 0 = empty), loc u64 (where the row's arena entry lives, and its
// length), id i64, the row's first 40 bytes}; the arena holds one entry per id, [id i64][row
// bytes padded to 8]. A steady-state lookup is one random access: the slot holds the tag, the
// id and the bytes to compare (rows of up to 40 bytes -- BinaryRowData key rows of a short
// string and a fixed field or two). One intern call: k_dict_lookup over every row (both hashes
// in one pass over its words, the slot of its tag, the byte comparison, the id; rows whose tag
// is not in the table go to a miss list -- none in a steady state), then over the misses only,
// in chunks the table has room for: k_dict_probe (the slot of its tag or a CAS claiming an
// empty one), k_dict_assign (the first claimer of a new slot allocates the id and writes the
// slot and the entry) and k_dict_verify (the byte comparison of the rows whose slot is new).
// Reservations (miss and pending lists, ids, arena bytes) take one atomic per wave. A 64-bit
// tag shared by distinct rows fails the comparison and is resolved on the host, so ids stay
// exact whatever the hash.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/flinkgpu.h"
#include "fg_window.h"

using namespace fg;

namespace {

constexpr int kDictThreads = 256;
#ifndef FG_DICT_GROW
#define FG_DICT_GROW 4   // table rebuilt at FG_DICT_GROW x (ids + 1M) slots (>= 2: room for a chunk)
#endif
static_assert(FG_DICT_GROW >= 2, "FG_DICT_GROW: the table must stay at most half full after a rebuild");
#ifndef FG_DICT_INIT
#define FG_DICT_INIT 2   // slots at open: FG_DICT_INIT x expected keys, rounded up to a power of two
#endif
// id = ordinal << kg_bits | key group, kg_bits = dict_kg_bits(max parallelism) (7 at Flink's
// default 128): ids stay below 2^31 for 16.7M keys, so the window engine stages them as narrow
// 32-bit keys (fg_window.h key_group_of reads the key group back from the low bits)

__host__ __device__ __forceinline__ uint32_t load_u32(const uint8_t* p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

// MurmurHashUtils.hashBytesByWords(segment, offset, len) (MurmurHashUtils.java:92-96,131-141,
// 143-161): little-endian 4-byte words (MemorySegment.getInt is native order), seed 42
__host__ __device__ __forceinline__ int32_t binaryrow_hash_bytes(const uint8_t* p, int32_t len) {
    uint32_t h1 = 42u;
    for (int32_t i = 0; i < len; i += 4) h1 = mix_h1(h1, mix_k1(load_u32(p + i)));
    return (int32_t)fmix32(h1 ^ (uint32_t)len);
}

constexpr uint64_t kNoLoc = ~0ull;   // a slot whose entry is not written yet

// Table slot (one 64-B line): the row's 64-bit tag, where its entry lives in the arena (entry
// offset << 24 | row length), its id and its first kSlotWords 4-byte words (zero padded). An
// arena entry is [id i64][row bytes, padded to 8].
constexpr int kSlotWords = 10;
struct alignas(64) Slot {
    unsigned long long tag;   // 0: empty
    unsigned long long loc;   // kNoLoc until the entry (and id, row words) are written
    long long id;
    uint32_t row[kSlotWords];
};
static_assert(sizeof(Slot) == 64, "one slot per 64-B line");
__host__ __device__ __forceinline__ uint64_t loc_of(uint64_t entry, int32_t len) { return entry << 24 | (uint32_t)len; }

struct DictDev {
    Slot* slots;         // [cap]
    uint32_t* slot_row;  // [cap] first claimer of a new slot in this call
    int64_t* ent_off;    // [ids] arena offset of the id's row bytes (its entry + 8)
    int32_t* ent_len;    // [ids]
    uint64_t* ent_tag;   // [ids] tag (0: resolved on the host, not in the table)
    uint8_t* arena;
    unsigned long long* counters;   // [0] ids, [1] arena bytes, [2] collisions, [3] bad rows, [4] pending rows,
                                    // [5] entry bytes of the lookup's misses, [6] lookup misses
    uint64_t mask;       // cap - 1
    int32_t kg_bits;     // id = ordinal << kg_bits | key group
};

// one atomic per wave: lane-exclusive offsets of `amount` (0 for a lane that takes nothing)
// reserved from *ctr; every lane of the wave must call it (inactive lanes count as 0)
__device__ __forceinline__ unsigned long long wave_reserve(unsigned long long* ctr, uint32_t amount) {
    const int lane = threadIdx.x & 63;
    uint32_t x = amount;   // inclusive scan over the wave
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

struct RowsIn {
    const uint8_t* bytes;   // 4-byte aligned; every row at a multiple of 4, of 4-byte words
    const int64_t* off;
    const int32_t* len;
    const uint32_t* idx;    // rows idx[0..n) of off / len (the miss list), or null: rows 0..n
    int64_t n;
    int64_t nbytes;
    int32_t max_p;
    int32_t tag_bits;
    int32_t check;          // device rows: k_dict_lookup checks them (bad rows -> counters[3])
};

// arena bytes an entry of a row of `len` bytes takes: [id i64][row bytes, padded to 8]
__host__ __device__ __forceinline__ uint64_t entry_bytes(int32_t len) { return 8 + (((uint64_t)len + 7) & ~7ull); }

// Both hashes of a row in one pass over its 4-byte words: the Flink hash (hashBytesByWords,
// seed 42) and the table's own 64-bit tag (independent of it: equal Flink hashes are common at
// 10M keys; equal tags are ~1e-5 there, and resolved exactly anyway).
__device__ __forceinline__ void row_hashes(const uint32_t* w, int32_t len, int tag_bits, uint64_t* tag, int32_t* fh) {
    uint32_t h1 = 42u;
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)len * 0xff51afd7ed558ccdull;
    const int32_t nw = len >> 2;
    int32_t k = 0;
    for (; k + 2 <= nw; k += 2) {
        const uint32_t a = w[k], b = w[k + 1];
        h1 = mix_h1(mix_h1(h1, mix_k1(a)), mix_k1(b));
        h = fmix64(h ^ ((uint64_t)a | (uint64_t)b << 32)) + 0x632BE59BD9B4E019ull;
    }
    if (k < nw) {
        const uint32_t a = w[k];
        h1 = mix_h1(h1, mix_k1(a));
        h = fmix64(h ^ (uint64_t)a ^ 0xA0761D6478BD642Full);
    }
    h = fmix64(h);
    if (tag_bits < 64) h &= (1ull << tag_bits) - 1;   // diagnostic: force collisions (tests)
    *tag = h ? h : 1;
    *fh = (int32_t)fmix32(h1 ^ (uint32_t)len);
}

// the id of the entry at `loc` if its row equals the row at w, else -1
__device__ __forceinline__ int64_t entry_id_if_equal(const DictDev& d, uint64_t loc, const uint32_t* w, int32_t len) {
    if ((int32_t)(loc & 0xFFFFFF) != len) return -1;
    const uint8_t* e = d.arena + (loc >> 24);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(e + 8);
    bool eq = true;
    for (int32_t k = 0; eq && k < (len >> 2); k++) eq = w[k] == q[k];
    return eq ? *reinterpret_cast<const int64_t*>(e) : -1;
}

// Rows of up to kRegWords words (BinaryRowData key rows of one or two fixed fields and a short
// string: 16-32 bytes) are read once into registers -- 8-byte loads when the row is 8-byte
// aligned -- and hashed and compared from there; longer rows take the word loops above.
constexpr int kRegWords = 8;
__device__ __forceinline__ void row_words(const uint8_t* p, int32_t len, uint32_t (&r)[kRegWords]) {
    const int32_t nw = len >> 2;
    if (((uintptr_t)p & 15) == 0 && nw == kRegWords) {   // the common 32-B row, 16-B aligned
        const uint4 a = *reinterpret_cast<const uint4*>(p), b = *reinterpret_cast<const uint4*>(p + 16);
        r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
        r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
        return;
    }
    const bool a8 = ((uintptr_t)p & 7) == 0;
#pragma unroll
    for (int k = 0; k < kRegWords; k += 2) {
        r[k] = r[k + 1] = 0;
        if (a8 && k + 2 <= nw) {
            const uint2 v = *reinterpret_cast<const uint2*>(p + 4 * k);
            r[k] = v.x;
            r[k + 1] = v.y;
        } else {
            if (k < nw) r[k] = *reinterpret_cast<const uint32_t*>(p + 4 * k);
            if (k + 1 < nw) r[k + 1] = *reinterpret_cast<const uint32_t*>(p + 4 * k + 4);
        }
    }
}
// row_hashes over register words (the same arithmetic, unrolled)
__device__ __forceinline__ void row_hashes_reg(const uint32_t (&r)[kRegWords], int32_t len, int tag_bits, uint64_t* tag,
                                               int32_t* fh) {
    uint32_t h1 = 42u;
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)len * 0xff51afd7ed558ccdull;
    const int32_t nw = len >> 2;
#pragma unroll
    for (int k = 0; k < kRegWords; k += 2) {
        if (k + 2 <= nw) {
            h1 = mix_h1(mix_h1(h1, mix_k1(r[k])), mix_k1(r[k + 1]));
            h = fmix64(h ^ ((uint64_t)r[k] | (uint64_t)r[k + 1] << 32)) + 0x632BE59BD9B4E019ull;
        } else if (k < nw) {
            h1 = mix_h1(h1, mix_k1(r[k]));
            h = fmix64(h ^ (uint64_t)r[k] ^ 0xA0761D6478BD642Full);
        }
    }
    h = fmix64(h);
    if (tag_bits < 64) h &= (1ull << tag_bits) - 1;
    *tag = h ? h : 1;
    *fh = (int32_t)fmix32(h1 ^ (uint32_t)len);
}
// The id of a written slot if its row equals the row (register words r when `small`, else the
// words at w): the slot's words first, an entry's bytes past them only for rows longer than the
// slot holds; -1 for a distinct row with an equal tag.
__device__ __forceinline__ int64_t slot_id_if_equal(const DictDev& d, const Slot& sl, const uint32_t (&r)[kRegWords],
                                                    const uint32_t* w, bool small, int32_t len) {
    if ((int32_t)(sl.loc & 0xFFFFFF) != len) return -1;
    const int32_t nw = len >> 2;
    uint32_t diff = 0;
    if (small) {
        static_assert(kRegWords <= kSlotWords, "register rows fit the slot");
#pragma unroll
        for (int k = 0; k < kRegWords; k++)
            if (k < nw) diff |= r[k] ^ sl.row[k];
    } else {
        for (int k = 0; k < nw && k < kSlotWords; k++) diff |= w[k] ^ sl.row[k];
        if (diff == 0 && nw > kSlotWords) {
            const uint32_t* q = reinterpret_cast<const uint32_t*>(d.arena + (sl.loc >> 24) + 8);
            for (int k = kSlotWords; k < nw; k++) diff |= w[k] ^ q[k];
        }
    }
    return diff == 0 ? (int64_t)sl.id : -1;
}

// a slot as four 16-B loads issued together (the line is fetched once)
__device__ __forceinline__ Slot load_slot(const Slot* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1], c = q[2], e = q[3];
    Slot sl;
    sl.tag = (unsigned long long)a.x | (unsigned long long)a.y << 32;
    sl.loc = (unsigned long long)a.z | (unsigned long long)a.w << 32;
    sl.id = (long long)((unsigned long long)b.x | (unsigned long long)b.y << 32);
    sl.row[0] = b.z; sl.row[1] = b.w;
    sl.row[2] = c.x; sl.row[3] = c.y; sl.row[4] = c.z; sl.row[5] = c.w;
    sl.row[6] = e.x; sl.row[7] = e.y; sl.row[8] = e.z; sl.row[9] = e.w;
    return sl;
}

// Lookup of every row of the call (no claims): both hashes, the slot of its tag (one 64-B line
// holds tag, length, id and the row's first 40 bytes), the byte comparison, the id. A row whose
// tag is not in the table joins the miss list (counters[6]); a distinct row with an equal tag
// gets -1 (counters[2], resolved on the host). kg_out (optional) takes every row's key group.
// Each thread takes kLookupRows rows (a block's rows in kLookupRows coalesced strides) and issues
// all their slot loads before resolving any.
#ifndef FG_DICT_ROWS
#define FG_DICT_ROWS 1   // rows per thread (A/B in DESIGN.md)
#endif
constexpr int kLookupRows = FG_DICT_ROWS;
__global__ __launch_bounds__(kDictThreads) void k_dict_lookup(DictDev d, RowsIn in, int32_t* kg_out, int64_t* id_out,
                                                              uint32_t* miss) {
    constexpr int R = kLookupRows;
    const int64_t b0 = (int64_t)blockIdx.x * kDictThreads * R + threadIdx.x;
    int64_t ii[R];
    bool valid[R], small[R];
    int32_t len[R], fh[R];
    const uint8_t* rp[R];
    uint32_t r[R][kRegWords];
    uint64_t t[R], s[R];
    uint32_t nbad = 0;
#pragma unroll
    for (int u = 0; u < R; u++) {   // (every lane stays for the wave-wide reservations below)
        const int64_t i0 = b0 + (int64_t)u * kDictThreads;
        valid[u] = i0 < in.n;
        ii[u] = valid[u] ? i0 : 0;
        len[u] = in.len[ii[u]];
        const int64_t off = in.off[ii[u]];
        if (in.check && valid[u]) {   // device rows: inside the buffer, 4-byte words (BinaryRowData)
            const bool bad = len[u] < 0 || len[u] >= (1 << 24) || (len[u] & 3) != 0 || off < 0 || (off & 3) != 0 ||
                             off + len[u] > in.nbytes;
            if (bad) {
                nbad++;
                valid[u] = false;   // (not looked up; the call fails before anything is inserted)
                len[u] = 0;
            }
        }
        rp[u] = in.bytes + (valid[u] ? off : 0);
    }
    if (in.check) {
        uint32_t b = nbad;
        for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o);
        if ((threadIdx.x & 63) == 0 && b) atomicAdd(&d.counters[3], (unsigned long long)b);
    }
#pragma unroll
    for (int u = 0; u < R; u++) {
        small[u] = len[u] <= 4 * kRegWords;
        if (small[u]) {
            row_words(rp[u], len[u], r[u]);
            row_hashes_reg(r[u], len[u], in.tag_bits, &t[u], &fh[u]);
        } else {
#pragma unroll
            for (int k = 0; k < kRegWords; k++) r[u][k] = 0;
            row_hashes(reinterpret_cast<const uint32_t*>(rp[u]), len[u], in.tag_bits, &t[u], &fh[u]);
        }
        s[u] = fmix64(t[u]) & d.mask;
    }
    Slot sl[R];
#pragma unroll
    for (int u = 0; u < R; u++) sl[u] = load_slot(&d.slots[s[u]]);   // every row's line in flight
#pragma unroll
    for (int u = 0; u < R; u++) {
        bool found = false;
        int64_t id = -1;
        if (valid[u]) {
            Slot cur = sl[u];
            uint64_t at = s[u];
            for (;;) {   // (the home slot resolves almost every row; probing past it is rare)
                if (cur.tag == t[u]) {   // (every slot is written: no claims run beside the lookup)
                    found = true;
                    id = slot_id_if_equal(d, cur, r[u], reinterpret_cast<const uint32_t*>(rp[u]), small[u], len[u]);
                    break;
                }
                if (cur.tag == 0) break;
                at = (at + 1) & d.mask;
                cur = load_slot(&d.slots[at]);
            }
            if (kg_out) kg_out[ii[u]] = murmur_hash(fh[u]) % in.max_p;
            if (found) {
                if (id < 0) atomicAdd(&d.counters[2], 1ull);
                id_out[ii[u]] = id;
            }
        }
        const bool m = valid[u] && !found;
        const unsigned long long w = wave_reserve(&d.counters[6], m ? 1u : 0u);
        if (m) miss[w] = (uint32_t)ii[u];
        // the arena bytes the misses may take as new entries (counters[5], one atomic per wave)
        uint64_t eb = m ? entry_bytes(len[u]) : 0;
        for (int o = 32; o > 0; o >>= 1) eb += __shfl_xor(eb, o);
        if ((threadIdx.x & 63) == 0 && eb) atomicAdd(&d.counters[5], (unsigned long long)eb);
    }
}

// Pending rows (their slot is new in this call): row index, slot and key group, for
// k_dict_assign / k_dict_verify.
struct Pending {
    uint32_t* row;
    uint64_t* slot;
    int32_t* kg;
};

// One pass per row: both hashes, the slot holding the row's tag or an empty one claimed with a
// CAS (one 16-B load reads a slot's tag and entry location together), and -- when the slot's
// entry was written by an earlier call -- the byte comparison with that entry (its id, or -1: a
// distinct row with an equal tag, left to the host). Rows whose slot is new in this call (claimed
// by them or by an equal-tagged row) join the pending list (none in a steady state). kg_out
// (optional) takes every row's key group.
__global__ __launch_bounds__(kDictThreads) void k_dict_probe(DictDev d, RowsIn in, int64_t* id_out, Pending pend_out) {
    const int64_t j0 = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    const bool valid = j0 < in.n;   // (every lane stays for the wave-wide reservation below)
    const int64_t i = in.idx ? (int64_t)in.idx[valid ? j0 : 0] : (valid ? j0 : 0);
    const int32_t len = in.len[i];
    const uint8_t* rp = in.bytes + in.off[i];
    const bool small = len <= 4 * kRegWords;
    uint32_t r[kRegWords];
    uint64_t t;
    int32_t fh;
    if (small) {
        row_words(rp, len, r);
        row_hashes_reg(r, len, in.tag_bits, &t, &fh);
    } else {
#pragma unroll
        for (int k = 0; k < kRegWords; k++) r[k] = 0;
        row_hashes(reinterpret_cast<const uint32_t*>(rp), len, in.tag_bits, &t, &fh);
    }
    uint64_t s = fmix64(t) & d.mask;
    uint64_t loc = kNoLoc;
    int64_t sid = -1;
    for (; valid;) {
        // the whole line in four 16-B loads: a written slot holds the row's first kSlotWords
        // words and its id, so a row of up to 40 bytes is compared and resolved from the slot
        // alone -- no second random access into the arena (the 32-B key rows of a STRING key)
        const Slot cur = load_slot(&d.slots[s]);
        if (cur.tag == t) {   // (a slot claimed earlier in this call still has no entry: kNoLoc)
            loc = cur.loc;
            if (loc != kNoLoc) sid = slot_id_if_equal(d, cur, r, reinterpret_cast<const uint32_t*>(rp), small, len);
            break;
        }
        if (cur.tag == 0) {
            const unsigned long long old = atomicCAS(&d.slots[s].tag, 0ull, (unsigned long long)t);
            if (old == 0) {   // claimed: this row owns the new slot (no other row can claim it)
                d.slot_row[s] = (uint32_t)i;
                break;
            }
            if (old == t) break;   // claimed in this call by an equal-tagged row
        }
        s = (s + 1) & d.mask;
    }
    const int32_t kg = murmur_hash(fh) % in.max_p;
    if (valid) {
        if (loc != kNoLoc) {   // written by an earlier call, or an earlier chunk of this one
            if (sid < 0) atomicAdd(&d.counters[2], 1ull);
            id_out[i] = sid;
        }
    }
    const bool pend = valid && loc == kNoLoc;
    const unsigned long long at = wave_reserve(&d.counters[4], pend ? 1u : 0u);
    if (pend) {
        pend_out.row[at] = (uint32_t)i;
        pend_out.slot[at] = s;
        pend_out.kg[at] = kg;
    }
}

// pending rows: the claimer of a new slot allocates its id and writes its entry
__global__ __launch_bounds__(kDictThreads) void k_dict_assign(DictDev d, RowsIn in, Pending pend) {
    const uint64_t np = d.counters[4];
    const int lane = threadIdx.x & 63;
    // wave-uniform trip count (the reservations are wave-wide)
    for (uint64_t wb = (uint64_t)blockIdx.x * kDictThreads + (threadIdx.x & ~63u); wb < np;
         wb += (uint64_t)gridDim.x * kDictThreads) {
        const uint64_t j = wb + lane;
        const int64_t i = j < np ? pend.row[j] : 0;
        const uint64_t s = j < np ? pend.slot[j] : 0;
        const bool own = j < np && d.slot_row[s] == (uint32_t)i;
        const int32_t len = own ? in.len[i] : 0;
        const unsigned long long ord = wave_reserve(&d.counters[0], own ? 1u : 0u);
        const unsigned long long at = wave_reserve(&d.counters[1], own ? (uint32_t)(8 + ((len + 7) & ~7)) : 0u);
        if (!own) continue;
        const int64_t id = (int64_t)(ord << d.kg_bits | (uint64_t)pend.kg[j]);
        *reinterpret_cast<int64_t*>(d.arena + at) = id;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(in.bytes + in.off[i]);
        uint32_t* dst = reinterpret_cast<uint32_t*>(d.arena + at + 8);
        for (int32_t k = 0; k < (len >> 2); k++) dst[k] = src[k];
        if (len & 4) dst[len >> 2] = 0;   // (zero padding to 8 bytes)
        d.ent_off[ord] = (int64_t)at + 8;
        d.ent_len[ord] = len;
        d.ent_tag[ord] = d.slots[s].tag;
        Slot& sl = d.slots[s];
        sl.id = id;
        for (int k = 0; k < kSlotWords; k++) sl.row[k] = k < (len >> 2) ? src[k] : 0u;
        __threadfence();   // the slot's id and words before its loc (read by later chunks' probes)
        sl.loc = loc_of(at, len);
    }
}

// pending rows compare their bytes with their slot's (new) entry; a mismatch is left to the host
__global__ __launch_bounds__(kDictThreads) void k_dict_verify(DictDev d, RowsIn in, Pending pend, int64_t* id_out) {
    const uint64_t np = d.counters[4];
    for (uint64_t j = (uint64_t)blockIdx.x * kDictThreads + threadIdx.x; j < np; j += (uint64_t)gridDim.x * kDictThreads) {
        const int64_t i = pend.row[j];
        const int64_t id = entry_id_if_equal(d, d.slots[pend.slot[j]].loc,
                                             reinterpret_cast<const uint32_t*>(in.bytes + in.off[i]), in.len[i]);
        if (id < 0) atomicAdd(&d.counters[2], 1ull);
        id_out[i] = id;
    }
}

// rebuild the table at a larger capacity from the entries (ids keep their values)
__global__ __launch_bounds__(kDictThreads) void k_dict_rehash(DictDev d, int64_t nids) {
    const int64_t o = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    if (o >= nids) return;
    const uint64_t t = d.ent_tag[o];
    if (t == 0) return;   // a host-resolved row: not in the table
    uint64_t s = fmix64(t) & d.mask;
    for (;;) {
        const unsigned long long old = atomicCAS(&d.slots[s].tag, 0ull, (unsigned long long)t);
        if (old == 0) break;
        s = (s + 1) & d.mask;
    }
    const int32_t len = d.ent_len[o];
    const uint8_t* e = d.arena + d.ent_off[o] - 8;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(e + 8);
    Slot& sl = d.slots[s];
    sl.id = *reinterpret_cast<const long long*>(e);
    for (int k = 0; k < kSlotWords; k++) sl.row[k] = k < (len >> 2) ? w[k] : 0u;
    sl.loc = loc_of((uint64_t)(d.ent_off[o] - 8), len);
}

__global__ __launch_bounds__(kDictThreads) void k_dict_gather(DictDev d, int64_t n, const int64_t* ids, int64_t nids,
                                                              int64_t* off_out, int32_t* len_out) {
    const int64_t i = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    if (i >= n) return;
    const uint64_t ord = (uint64_t)ids[i] >> d.kg_bits;
    const bool ok = ids[i] >= 0 && (int64_t)ord < nids;
    off_out[i] = ok ? d.ent_off[ord] : -1;
    len_out[i] = ok ? d.ent_len[ord] : -1;
}

__global__ __launch_bounds__(kDictThreads) void k_slots_clear(Slot* p, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    if (i < n) {
        uint4* q = reinterpret_cast<uint4*>(p + i);
        q[0] = make_uint4(0u, 0u, 0xffffffffu, 0xffffffffu);   // tag 0, loc kNoLoc
        q[1] = q[2] = q[3] = make_uint4(0u, 0u, 0u, 0u);
    }
}

inline unsigned grid_of(int64_t n) { return (unsigned)((n + kDictThreads - 1) / kDictThreads); }

struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    Buf() = default;
    Buf(const Buf&) = delete;
    Buf& operator=(const Buf&) = delete;
    ~Buf() {
        if (p) (void)hipFree(p);
    }
    // grow to `need` bytes, keeping the first `keep` bytes
    hipError_t ensure(size_t need, hipStream_t s, size_t keep = 0) {
        if (need <= bytes) return hipSuccess;
        const size_t nb = std::max(need, bytes + bytes / 2);
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, nb);
        if (e != hipSuccess) return e;
        if (keep && p) {
            e = hipMemcpyAsync(q, p, std::min(keep, bytes), hipMemcpyDeviceToDevice, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) {
                (void)hipFree(q);
                return e;
            }
        }
        if (p) (void)hipFree(p);
        p = q;
        bytes = nb;
        return hipSuccess;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

}  // namespace

struct fg_key_dict {
    int device = 0;
    int32_t max_p = 128;
    int tag_bits = 64;
    hipStream_t stream = nullptr;
    uint64_t cap = 0;   // table slots (power of two)
    int64_t nids = 0;   // ids handed out (host mirror of counters[0])
    int64_t arena_used = 0;
    Buf slots, slot_row, ent_off, ent_len, ent_tag, arena, counters;
    Buf in_bytes, in_off, in_len, row_tag, row_kg, row_slot, row_pkg, row_id, miss;   // per-call scratch
    std::unordered_map<std::string, int64_t> side;   // rows whose tag another row holds
    std::string err;
    // kernel timing (fg_key_dict_set_timing): HIP events around each chunk's probe and its
    // assign + verify, on the dictionary's stream; summed into the two classes below
    bool timing = false;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    fg_kernel_stat kstat[2] = {};
    // fg_key_dict_intern_async: the lookup launched, the rest of the call taken by _wait
    struct Pending {
        bool active = false, host = false;
        int64_t n = 0, nbytes = 0;
        RowsIn in{};
        int64_t* ids = nullptr;
        int32_t* kg_dev = nullptr;
        const uint8_t* bytes = nullptr;
        const int64_t* offsets = nullptr;
        const int32_t* lengths = nullptr;
        int64_t* out_id = nullptr;
        int32_t* out_kg = nullptr;
        uint64_t entry_need = 0;   // host rows: every row as a new entry
    } pend;

    int fail(int rc, const std::string& m) {
        err = m;
        return rc;
    }
    DictDev dev() const {
        DictDev d;
        d.slots = slots.as<Slot>();
        d.slot_row = slot_row.as<uint32_t>();
        d.ent_off = ent_off.as<int64_t>();
        d.ent_len = ent_len.as<int32_t>();
        d.ent_tag = ent_tag.as<uint64_t>();
        d.arena = arena.as<uint8_t>();
        d.counters = counters.as<unsigned long long>();
        d.mask = cap - 1;
        d.kg_bits = dict_kg_bits(max_p);
        return d;
    }
};

#define DCHK(d, x)                                                                     \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return (d)->fail(FG_EDEVICE, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)

namespace {

// table at `ncap` slots (power of two) holding every entry
int rebuild(fg_key_dict* d, uint64_t ncap) {
    hipStream_t s = d->stream;
    Buf nslots, nrow;
    DCHK(d, nslots.ensure(sizeof(Slot) * ncap, s));
    DCHK(d, nrow.ensure(4 * ncap, s));
    hipLaunchKernelGGL(k_slots_clear, dim3(grid_of((int64_t)ncap)), dim3(kDictThreads), 0, s, nslots.as<Slot>(),
                       (int64_t)ncap);
    DCHK(d, hipGetLastError());
    std::swap(d->slots.p, nslots.p);
    std::swap(d->slots.bytes, nslots.bytes);
    std::swap(d->slot_row.p, nrow.p);
    std::swap(d->slot_row.bytes, nrow.bytes);
    d->cap = ncap;
    if (d->nids)
        hipLaunchKernelGGL(k_dict_rehash, dim3(grid_of(d->nids)), dim3(kDictThreads), 0, s, d->dev(), d->nids);
    DCHK(d, hipGetLastError());
    DCHK(d, hipStreamSynchronize(s));
    return FG_OK;
}

// Rows of one chunk whose 64-bit tag another row holds (ids -1): exact ids from the host-side
// map, new rows appended to the arena (ent_tag 0: never rehashed into the table). `bytes`,
// `offsets`, `lengths` are the caller's (host or device) arrays for the chunk's rows.
int resolve_collisions(fg_key_dict* d, bool host, int64_t n, const uint8_t* bytes, int64_t nbytes,
                       const int64_t* offsets, const int32_t* lengths, int64_t* ids) {
    hipStream_t s = d->stream;
    std::vector<int64_t> hid(n);
    DCHK(d, hipMemcpy(hid.data(), ids, 8 * (size_t)n, hipMemcpyDeviceToHost));
    // device rows: one copy of the buffer and the chunk's offsets / lengths, not one per row
    std::vector<uint8_t> hbytes;
    std::vector<int64_t> hoff;
    std::vector<int32_t> hlen;
    if (!host) {
        hbytes.resize((size_t)nbytes);
        hoff.resize(n);
        hlen.resize(n);
        if (nbytes) DCHK(d, hipMemcpy(hbytes.data(), bytes, (size_t)nbytes, hipMemcpyDeviceToHost));
        DCHK(d, hipMemcpy(hoff.data(), offsets, 8 * (size_t)n, hipMemcpyDeviceToHost));
        DCHK(d, hipMemcpy(hlen.data(), lengths, 4 * (size_t)n, hipMemcpyDeviceToHost));
    }
    const uint8_t* rb = host ? bytes : hbytes.data();
    const int64_t* ro = host ? offsets : hoff.data();
    const int32_t* rl = host ? lengths : hlen.data();
    for (int64_t i = 0; i < n; i++) {
        if (hid[i] >= 0) continue;
        const int32_t l = rl[i];
        const uint8_t* row = rb + ro[i];
        std::string k(row, row + l);
        auto it = d->side.find(k);
        int64_t id;
        if (it != d->side.end()) {
            id = it->second;
        } else {
            // its entry ([id][row bytes, padded]) appended to the arena, out of the table
            const int64_t ord = d->nids++;
            const int64_t at = d->arena_used;
            d->arena_used += 8 + ((l + 7) & ~7);
            DCHK(d, d->ent_off.ensure(8 * (size_t)d->nids, s, 8 * (size_t)ord));
            DCHK(d, d->ent_len.ensure(4 * (size_t)d->nids, s, 4 * (size_t)ord));
            DCHK(d, d->ent_tag.ensure(8 * (size_t)d->nids, s, 8 * (size_t)ord));
            DCHK(d, d->arena.ensure((size_t)d->arena_used, s, (size_t)at));
            const int32_t kg = murmur_hash(binaryrow_hash_bytes(row, l)) % d->max_p;
            id = (int64_t)((uint64_t)ord << dict_kg_bits(d->max_p) | (uint64_t)kg);
            std::vector<uint8_t> entry(8 + ((l + 7) & ~7), 0);
            std::memcpy(entry.data(), &id, 8);
            std::memcpy(entry.data() + 8, row, (size_t)l);
            const uint64_t zero = 0;
            const int64_t row_off = at + 8;
            DCHK(d, hipMemcpy(d->arena.as<uint8_t>() + at, entry.data(), entry.size(), hipMemcpyHostToDevice));
            DCHK(d, hipMemcpy(d->ent_off.as<int64_t>() + ord, &row_off, 8, hipMemcpyHostToDevice));
            DCHK(d, hipMemcpy(d->ent_len.as<int32_t>() + ord, &l, 4, hipMemcpyHostToDevice));
            DCHK(d, hipMemcpy(d->ent_tag.as<uint64_t>() + ord, &zero, 8, hipMemcpyHostToDevice));
            d->side.emplace(std::move(k), id);
        }
        hid[i] = id;
    }
    DCHK(d, hipMemcpy(ids, hid.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
    const unsigned long long c2[3] = {(unsigned long long)d->nids, (unsigned long long)d->arena_used, 0ull};
    DCHK(d, hipMemcpy(d->counters.p, c2, sizeof c2, hipMemcpyHostToDevice));
    return FG_OK;
}

uint64_t pow2_at_least(uint64_t x) {
    uint64_t c = 1024;
    while (c < x) c <<= 1;
    return c;
}

}  // namespace

extern "C" {

int fg_key_dict_open(int32_t device_id, int32_t max_parallelism, int64_t expected_keys, fg_key_dict** out) {
    if (!out || max_parallelism <= 0 || max_parallelism > (1 << 15)) return FG_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device_id < 0 || device_id >= ndev) return FG_EDEVICE;
    if (hipSetDevice(device_id) != hipSuccess) return FG_EDEVICE;
    std::unique_ptr<fg_key_dict> d(new fg_key_dict());
    d->device = device_id;
    d->max_p = max_parallelism;
    if (const char* e = getenv("FG_DICT_TAG_BITS")) d->tag_bits = std::max(1, std::min(64, std::atoi(e)));   // tests
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) return FG_EDEVICE;
    if (d->counters.ensure(64, d->stream) != hipSuccess) return FG_EDEVICE;
    if (hipMemsetAsync(d->counters.p, 0, 64, d->stream) != hipSuccess) return FG_EDEVICE;
    if (rebuild(d.get(), pow2_at_least(FG_DICT_INIT * (uint64_t)std::max<int64_t>(expected_keys, 1)))) return FG_EDEVICE;
    *out = d.release();
    return FG_OK;
}

// The first half of an intern call: arguments checked, scratch sized, the lookup of every row
// launched (device rows are checked by the lookup itself: a bad row is counted, not looked up,
// and the call fails in intern_finish before anything is inserted). No host synchronization.
static int intern_begin(fg_key_dict* d, int32_t location, int64_t n, const uint8_t* bytes, int64_t nbytes,
                        const int64_t* offsets, const int32_t* lengths, int64_t* out_id, int32_t* out_kg) {
    if (!d) return FG_EINVAL;
    if (d->pend.active) return d->fail(FG_ESTATE, "fg_key_dict_intern: an async intern is pending (fg_key_dict_intern_wait)");
    if (n < 0 || n > 0x7fffffff || !bytes || nbytes < 0 || !offsets || !lengths || !out_id)
        return d->fail(FG_EINVAL, "fg_key_dict_intern: invalid arguments");
    if (hipSetDevice(d->device) != hipSuccess) return d->fail(FG_EDEVICE, "hipSetDevice failed");
    hipStream_t s = d->stream;
    const bool host = location == FG_HOST;
    if (!host && (uintptr_t)bytes % 4 != 0)
        return d->fail(FG_EINVAL, "fg_key_dict_intern: the row buffer must be 4-byte aligned");
    uint64_t entry_need = 0;   // host rows: arena bytes if every row is new
    if (host) {   // validate on the host: every row inside the buffer, 4-byte words
        for (int64_t i = 0; i < n; i++) {
            if (lengths[i] < 0 || lengths[i] >= (1 << 24) || (lengths[i] & 3) || (offsets[i] & 3) || offsets[i] < 0 ||
                offsets[i] + lengths[i] > nbytes)
                return d->fail(FG_EINVAL, "key row " + std::to_string(i) +
                                              ": offset/length outside the buffer or not a multiple of 4 bytes");
            entry_need += entry_bytes(lengths[i]);
        }
    }
    const size_t ents = (size_t)(d->nids + n);
    DCHK(d, d->ent_off.ensure(8 * ents, s, 8 * (size_t)d->nids));
    DCHK(d, d->ent_len.ensure(4 * ents, s, 4 * (size_t)d->nids));
    DCHK(d, d->ent_tag.ensure(8 * ents, s, 8 * (size_t)d->nids));
    RowsIn in{};
    in.n = n;
    in.nbytes = nbytes;
    in.max_p = d->max_p;
    in.tag_bits = d->tag_bits;
    in.check = host ? 0 : 1;
    if (host) {
        DCHK(d, d->in_bytes.ensure((size_t)nbytes + 8, s));
        DCHK(d, d->in_off.ensure(8 * (size_t)n, s));
        DCHK(d, d->in_len.ensure(4 * (size_t)n, s));
        DCHK(d, hipMemcpyAsync(d->in_bytes.p, bytes, (size_t)nbytes, hipMemcpyHostToDevice, s));
        DCHK(d, hipMemcpyAsync(d->in_off.p, offsets, 8 * (size_t)n, hipMemcpyHostToDevice, s));
        DCHK(d, hipMemcpyAsync(d->in_len.p, lengths, 4 * (size_t)n, hipMemcpyHostToDevice, s));
        in.bytes = d->in_bytes.as<uint8_t>();
        in.off = d->in_off.as<int64_t>();
        in.len = d->in_len.as<int32_t>();
    } else {
        in.bytes = bytes;
        in.off = offsets;
        in.len = lengths;
    }
    int64_t* ids = out_id;
    if (host) {
        DCHK(d, d->row_id.ensure(8 * (size_t)n, s));
        ids = d->row_id.as<int64_t>();
    }
    int32_t* kg_dev = nullptr;   // every row's key group, when asked for
    if (out_kg) {
        if (host) {
            DCHK(d, d->row_kg.ensure(4 * (size_t)n, s));
            kg_dev = d->row_kg.as<int32_t>();
        } else {
            kg_dev = out_kg;
        }
    }
    // 1) lookup of every row: one random 64-B slot per row; the misses are listed, their arena
    // bytes summed (counters[5]), bad device rows counted (counters[3])
    DCHK(d, d->miss.ensure(4 * (size_t)std::max<int64_t>(n, 1), s));
    unsigned long long* ctr = d->counters.as<unsigned long long>();
    DCHK(d, hipMemsetAsync(ctr + 5, 0, 16, s));   // [5] miss entry bytes, [6] misses
    if (n > 0) {
        if (d->timing) DCHK(d, hipEventRecord(d->ev[0], s));
        hipLaunchKernelGGL(k_dict_lookup, dim3((unsigned)((n + (int64_t)kDictThreads * kLookupRows - 1) /
                                                    ((int64_t)kDictThreads * kLookupRows))),
                           dim3(kDictThreads), 0, s, d->dev(), in, kg_dev, ids, d->miss.as<uint32_t>());
        if (d->timing) DCHK(d, hipEventRecord(d->ev[1], s));
        DCHK(d, hipGetLastError());
    }
    auto& pc = d->pend;
    pc.active = true;
    pc.host = host;
    pc.n = n;
    pc.nbytes = nbytes;
    pc.in = in;
    pc.ids = ids;
    pc.kg_dev = kg_dev;
    pc.bytes = bytes;
    pc.offsets = offsets;
    pc.lengths = lengths;
    pc.out_id = out_id;
    pc.out_kg = out_kg;
    pc.entry_need = entry_need;
    return FG_OK;
}

// The second half: the lookup's counters (one synchronization), then the misses -- none in a
// steady state -- in chunks, and the collisions.
static int intern_finish(fg_key_dict* d) {
    if (!d) return FG_EINVAL;
    if (!d->pend.active) return FG_OK;
    auto pc = d->pend;
    d->pend.active = false;
    hipStream_t s = d->stream;
    const int64_t n = pc.n;
    RowsIn in = pc.in;
    int64_t* ids = pc.ids;
    unsigned long long* ctr = d->counters.as<unsigned long long>();
    unsigned long long cnt[7];
    DCHK(d, hipMemcpyAsync(cnt, ctr, sizeof cnt, hipMemcpyDeviceToHost, s));
    DCHK(d, hipStreamSynchronize(s));
    if (n == 0) return FG_OK;
    if (cnt[3]) {   // bad device rows: nothing was inserted
        DCHK(d, hipMemsetAsync(ctr + 3, 0, 8, s));
        DCHK(d, hipStreamSynchronize(s));
        return d->fail(FG_EINVAL, "fg_key_dict_intern: " + std::to_string(cnt[3]) +
                                      " key rows outside the buffer or not a multiple of 4 bytes");
    }
    if (d->timing) {
        float ms = 0.f;
        DCHK(d, hipEventElapsedTime(&ms, d->ev[0], d->ev[1]));
        d->kstat[0].launches++;
        d->kstat[0].total_ms += ms;
        d->kstat[0].records += n;
    }
    uint64_t collisions = cnt[2];
    const int64_t nmiss = (int64_t)cnt[6];
    if (nmiss > 0) {
        // k_dict_assign writes a new row's entry at a reserved arena offset without a bound check:
        // the arena holds every missed row of the call as a new entry
        const uint64_t need = pc.host ? pc.entry_need : cnt[5];
        DCHK(d, d->arena.ensure((size_t)d->arena_used + (size_t)need + 16, s, (size_t)d->arena_used));
    }
    // 2) the misses, in chunks the table has room for: it stays at most half full even if every
    // row of a chunk is new. It grows when that room falls under an eighth of the ids (and 1M
    // rows): to FG_DICT_GROW x (ids + 1M) slots rounded up -- sized by the distinct keys.
    for (int64_t pos = 0; pos < nmiss;) {
        const int64_t room = (int64_t)(d->cap / 2) - d->nids;
        if (room < std::max<int64_t>(1 << 20, d->nids / 8))
            if (int rc = rebuild(d, pow2_at_least(FG_DICT_GROW * (uint64_t)(d->nids + (1 << 20))))) return rc;
        const int64_t m = std::min<int64_t>(nmiss - pos, (int64_t)(d->cap / 2) - d->nids);
        DCHK(d, d->row_tag.ensure(4 * (size_t)m, s));   // the pending list
        DCHK(d, d->row_slot.ensure(8 * (size_t)m, s));
        DCHK(d, d->row_pkg.ensure(4 * (size_t)m, s));
        RowsIn c = in;
        c.idx = d->miss.as<uint32_t>() + pos;
        c.n = m;
        const Pending pend{d->row_tag.as<uint32_t>(), d->row_slot.as<uint64_t>(), d->row_pkg.as<int32_t>()};
        const DictDev dv = d->dev();
        const unsigned gm = grid_of(m);
        DCHK(d, hipMemsetAsync(dv.counters + 4, 0, 8, s));
        if (d->timing) DCHK(d, hipEventRecord(d->ev[1], s));
        hipLaunchKernelGGL(k_dict_probe, dim3(gm), dim3(kDictThreads), 0, s, dv, c, ids, pend);
        const unsigned gp = std::min(gm, 1024u);
        hipLaunchKernelGGL(k_dict_assign, dim3(gp), dim3(kDictThreads), 0, s, dv, c, pend);
        hipLaunchKernelGGL(k_dict_verify, dim3(gp), dim3(kDictThreads), 0, s, dv, c, pend, ids);
        if (d->timing) DCHK(d, hipEventRecord(d->ev[2], s));
        DCHK(d, hipGetLastError());
        DCHK(d, hipMemcpyAsync(cnt, ctr, sizeof cnt, hipMemcpyDeviceToHost, s));
        DCHK(d, hipStreamSynchronize(s));
        if (d->timing) {
            float ms = 0.f;
            DCHK(d, hipEventElapsedTime(&ms, d->ev[1], d->ev[2]));
            d->kstat[1].launches++;
            d->kstat[1].total_ms += ms;
            d->kstat[1].records += m;
        }
        d->nids = (int64_t)cnt[0];
        d->arena_used = (int64_t)cnt[1];
        pos += m;
    }
    collisions = cnt[2];
    if (collisions) {   // rows whose tag another row holds: exact ids from the host-side map
        DCHK(d, hipMemsetAsync(ctr + 2, 0, 8, s));
        if (int rc = resolve_collisions(d, pc.host, n, pc.bytes, pc.nbytes, pc.offsets, pc.lengths, ids)) return rc;
    }
    if (pc.host) DCHK(d, hipMemcpy(pc.out_id, ids, 8 * (size_t)n, hipMemcpyDeviceToHost));
    if (pc.out_kg && pc.host) DCHK(d, hipMemcpy(pc.out_kg, pc.kg_dev, 4 * (size_t)n, hipMemcpyDeviceToHost));
    return FG_OK;
}

int fg_key_dict_intern(fg_key_dict* d, int32_t location, int64_t n, const uint8_t* bytes, int64_t nbytes,
                       const int64_t* offsets, const int32_t* lengths, int64_t* out_id, int32_t* out_kg) {
    if (!d) return FG_EINVAL;
    if (n == 0 && !d->pend.active) return FG_OK;
    if (int rc = intern_begin(d, location, n, bytes, nbytes, offsets, lengths, out_id, out_kg)) return rc;
    return intern_finish(d);
}

int fg_key_dict_intern_async(fg_key_dict* d, int64_t n, const uint8_t* bytes, int64_t nbytes, const int64_t* offsets,
                             const int32_t* lengths, int64_t* out_id, int32_t* out_kg) {
    if (!d) return FG_EINVAL;
    return intern_begin(d, FG_DEVICE, n, bytes, nbytes, offsets, lengths, out_id, out_kg);
}

int fg_key_dict_intern_wait(fg_key_dict* d) {
    if (!d) return FG_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess) return d->fail(FG_EDEVICE, "hipSetDevice failed");
    return intern_finish(d);
}

int fg_key_dict_lookup(fg_key_dict* d, int32_t location, int64_t n, const int64_t* ids, int64_t* out_offsets,
                       int32_t* out_lengths) {
    if (!d) return FG_EINVAL;
    if (n == 0) return FG_OK;
    if (d->pend.active) return d->fail(FG_ESTATE, "fg_key_dict_lookup: an async intern is pending (fg_key_dict_intern_wait)");
    if (n < 0 || !ids || !out_offsets || !out_lengths) return d->fail(FG_EINVAL, "fg_key_dict_lookup: invalid arguments");
    if (hipSetDevice(d->device) != hipSuccess) return d->fail(FG_EDEVICE, "hipSetDevice failed");
    hipStream_t s = d->stream;
    const bool host = location == FG_HOST;
    const int64_t* di = ids;
    int64_t* doff = out_offsets;
    int32_t* dlen = out_lengths;
    Buf bi, bo, bl;
    if (host) {
        DCHK(d, bi.ensure(8 * (size_t)n, s));
        DCHK(d, bo.ensure(8 * (size_t)n, s));
        DCHK(d, bl.ensure(4 * (size_t)n, s));
        DCHK(d, hipMemcpyAsync(bi.p, ids, 8 * (size_t)n, hipMemcpyHostToDevice, s));
        di = bi.as<int64_t>();
        doff = bo.as<int64_t>();
        dlen = bl.as<int32_t>();
    }
    hipLaunchKernelGGL(k_dict_gather, dim3(grid_of(n)), dim3(kDictThreads), 0, s, d->dev(), n, di, d->nids, doff, dlen);
    DCHK(d, hipGetLastError());
    if (host) {
        DCHK(d, hipMemcpyAsync(out_offsets, doff, 8 * (size_t)n, hipMemcpyDeviceToHost, s));
        DCHK(d, hipMemcpyAsync(out_lengths, dlen, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
    }
    DCHK(d, hipStreamSynchronize(s));
    return FG_OK;
}

int fg_key_dict_arena(fg_key_dict* d, const uint8_t** dev_bytes, int64_t* size) {
    if (!d || !dev_bytes || !size) return FG_EINVAL;
    *dev_bytes = d->arena.as<uint8_t>();
    *size = d->arena_used;
    return FG_OK;
}

int fg_key_dict_copy_arena(fg_key_dict* d, int64_t begin, int64_t nbytes, uint8_t* host) {
    if (d && d->pend.active)
        return d->fail(FG_ESTATE, "fg_key_dict_copy_arena: an async intern is pending (fg_key_dict_intern_wait)");
    if (!d || begin < 0 || nbytes < 0 || begin + nbytes > d->arena_used || (nbytes && !host))
        return d ? d->fail(FG_EINVAL, "fg_key_dict_copy_arena: range outside the arena") : FG_EINVAL;
    if (!nbytes) return FG_OK;
    if (hipSetDevice(d->device) != hipSuccess) return d->fail(FG_EDEVICE, "hipSetDevice failed");
    DCHK(d, hipMemcpy(host, d->arena.as<uint8_t>() + begin, (size_t)nbytes, hipMemcpyDeviceToHost));
    return FG_OK;
}

int64_t fg_key_dict_size(fg_key_dict* d) { return d ? d->nids : -1; }

void* fg_key_dict_stream(fg_key_dict* d) { return d ? (void*)d->stream : nullptr; }

int fg_key_dict_set_timing(fg_key_dict* d, int32_t on) {
    if (!d) return FG_EINVAL;
    if (on && !d->ev[0]) {
        if (hipSetDevice(d->device) != hipSuccess) return d->fail(FG_EDEVICE, "hipSetDevice failed");
        for (auto& e : d->ev) DCHK(d, hipEventCreate(&e));
        std::snprintf(d->kstat[0].name, sizeof d->kstat[0].name, "dict_probe");
        std::snprintf(d->kstat[1].name, sizeof d->kstat[1].name, "dict_assign");
    }
    d->timing = on != 0;
    return FG_OK;
}

int fg_key_dict_kernel_stats(fg_key_dict* d, fg_kernel_stat* out, int32_t max, int32_t* count) {
    if (!d || !count || (max > 0 && !out)) return FG_EINVAL;
    *count = d->ev[0] ? 2 : 0;
    for (int i = 0; i < *count && i < max; i++) out[i] = d->kstat[i];
    return FG_OK;
}

const char* fg_key_dict_last_error(fg_key_dict* d) { return d ? d->err.c_str() : "null dictionary"; }

void fg_key_dict_close(fg_key_dict* d) {
    if (!d) return;
    (void)hipSetDevice(d->device);
    hipStream_t s = d->stream;
    if (s) (void)hipStreamSynchronize(s);
    for (auto e : d->ev)
        if (e) (void)hipEventDestroy(e);
    delete d;
    if (s) (void)hipStreamDestroy(s);
}

int32_t fg_binaryrow_hash(const uint8_t* row, int32_t len) {
    if (!row || len < 0 || (len & 3)) return 0;
    return binaryrow_hash_bytes(row, len);
}

}  // extern "C"
