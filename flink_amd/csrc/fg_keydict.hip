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
// (key group << 40 | ordinal): equal rows get equal ids, distinct rows distinct ids, so the
// aggregation by id is the aggregation by key row, and the id carries the row's key group
// (FG_KEYHASH_DICT_ID routes by it).
//
// Layout in HBM: an open-addressing table of `cap` slots {tag u64 (a 64-bit hash of the row,
// 0 = empty), id i64, claiming row u32}; per id its row's offset and length in a byte arena
// (rows padded to 8 bytes). One intern call: k_dict_hash (both hashes per row), k_dict_claim
// (a CAS per new tag), k_dict_assign (the first claimer of a new slot allocates the id and
// copies its bytes), k_dict_verify (every row compares its bytes with its slot's row: a 64-bit
// hash collision between distinct rows is caught here and resolved on the host, so ids stay
// exact whatever the hash).
#include <hip/hip_runtime.h>

#include <algorithm>
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
constexpr int kIdShift = 40;   // id = key group << kIdShift | ordinal
constexpr uint64_t kOrdMask = (1ull << kIdShift) - 1;

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

// the table's own 64-bit hash of the row (independent of the Flink hash: two keys with equal
// Flink hashes are common at 10M keys; equal 64-bit tags are ~1e-5 there, and exact anyway)
__host__ __device__ __forceinline__ uint64_t table_hash(const uint8_t* p, int32_t len, int tag_bits) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)len * 0xff51afd7ed558ccdull;
    int32_t i = 0;
    for (; i + 8 <= len; i += 8) {
        const uint64_t w = (uint64_t)load_u32(p + i) | (uint64_t)load_u32(p + i + 4) << 32;
        h = fmix64(h ^ w) + 0x632BE59BD9B4E019ull;
    }
    if (i < len) h = fmix64(h ^ (uint64_t)load_u32(p + i) ^ 0xA0761D6478BD642Full);
    h = fmix64(h);
    if (tag_bits < 64) h &= (1ull << tag_bits) - 1;   // diagnostic: force collisions (tests)
    return h ? h : 1;
}

struct DictDev {
    uint64_t* tag;       // [cap]
    int64_t* slot_id;    // [cap] -1: no id yet
    uint32_t* slot_row;  // [cap] first claimer of a new slot in this call
    int64_t* ent_off;    // [ids] arena offset of the id's row
    int32_t* ent_len;    // [ids]
    uint64_t* ent_tag;   // [ids] tag (0: resolved on the host, not in the table)
    uint8_t* arena;
    unsigned long long* counters;   // [0] ids, [1] arena bytes, [2] collisions, [3] bad rows
    uint64_t mask;       // cap - 1
};

struct RowsIn {
    const uint8_t* bytes;
    const int64_t* off;
    const int32_t* len;
    int64_t n;
    int64_t nbytes;
    int32_t max_p;
    int32_t tag_bits;
};

__global__ __launch_bounds__(kDictThreads) void k_dict_hash(RowsIn in, uint64_t* tag_out, int32_t* kg_out,
                                                            unsigned long long* counters) {
    const int64_t i = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    if (i >= in.n) return;
    const int32_t len = in.len[i];
    const int64_t off = in.off[i];
    if (len < 0 || (len & 3) != 0 || off < 0 || (off & 3) != 0 || off + len > in.nbytes) {
        atomicAdd(&counters[3], 1ull);   // (BinaryRowData rows are 8-byte multiples)
        tag_out[i] = 1;
        kg_out[i] = 0;
        return;
    }
    const uint8_t* p = in.bytes + off;
    tag_out[i] = table_hash(p, len, in.tag_bits);
    kg_out[i] = murmur_hash(binaryrow_hash_bytes(p, len)) % in.max_p;
}

// a slot for every row: the slot holding its tag, or an empty slot it claimed (CAS)
__global__ __launch_bounds__(kDictThreads) void k_dict_claim(DictDev d, int64_t n, const uint64_t* tag_in,
                                                             uint64_t* slot_out) {
    const int64_t i = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    if (i >= n) return;
    const uint64_t t = tag_in[i];
    uint64_t s = fmix64(t) & d.mask;
    for (;;) {
        const uint64_t cur = d.tag[s];
        if (cur == t) break;
        if (cur == 0) {
            const unsigned long long old =
                atomicCAS(reinterpret_cast<unsigned long long*>(&d.tag[s]), 0ull, (unsigned long long)t);
            if (old == 0) {   // claimed: this row owns the new slot (no other row can claim it)
                d.slot_row[s] = (uint32_t)i;
                break;
            }
            if (old == t) break;
        }
        s = (s + 1) & d.mask;
    }
    slot_out[i] = s;
}

// the claimer of a new slot allocates its id and copies its row into the arena
__global__ __launch_bounds__(kDictThreads) void k_dict_assign(DictDev d, RowsIn in, const uint64_t* slot_in,
                                                              const uint64_t* tag_in, const int32_t* kg_in) {
    const int64_t i = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    if (i >= in.n) return;
    const uint64_t s = slot_in[i];
    if (d.slot_id[s] >= 0 || d.slot_row[s] != (uint32_t)i) return;
    const int32_t len = in.len[i];
    const unsigned long long ord = atomicAdd(&d.counters[0], 1ull);
    const unsigned long long at = atomicAdd(&d.counters[1], (unsigned long long)((len + 7) & ~7));
    const uint8_t* p = in.bytes + in.off[i];
    uint32_t* dst = reinterpret_cast<uint32_t*>(d.arena + at);
    for (int32_t b = 0; b < len; b += 4) dst[b >> 2] = load_u32(p + b);
    if (len & 4) dst[len >> 2] = 0;   // (zero padding to 8 bytes)
    d.ent_off[ord] = (int64_t)at;
    d.ent_len[ord] = len;
    d.ent_tag[ord] = tag_in[i];
    d.slot_id[s] = (int64_t)((uint64_t)kg_in[i] << kIdShift | ord);
}

// every row compares its bytes with its slot's row; a mismatch (distinct rows, equal tags) is
// left to the host (-1)
__global__ __launch_bounds__(kDictThreads) void k_dict_verify(DictDev d, RowsIn in, const uint64_t* slot_in,
                                                              int64_t* id_out) {
    const int64_t i = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    if (i >= in.n) return;
    const int32_t len = in.len[i];
    const int64_t id = d.slot_id[slot_in[i]];
    const uint64_t ord = (uint64_t)id & kOrdMask;
    bool eq = d.ent_len[ord] == len;
    const uint8_t* p = in.bytes + in.off[i];
    const uint32_t* q = reinterpret_cast<const uint32_t*>(d.arena + d.ent_off[ord]);
    for (int32_t b = 0; eq && b < len; b += 4) eq = load_u32(p + b) == q[b >> 2];
    if (!eq) atomicAdd(&d.counters[2], 1ull);
    id_out[i] = eq ? id : -1;
}

// rebuild the table at a larger capacity from the entries (ids keep their values)
__global__ __launch_bounds__(kDictThreads) void k_dict_rehash(DictDev d, int64_t nids, const int64_t* ids_kg) {
    const int64_t o = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    if (o >= nids) return;
    const uint64_t t = d.ent_tag[o];
    if (t == 0) return;   // a host-resolved row: not in the table
    uint64_t s = fmix64(t) & d.mask;
    for (;;) {
        const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long*>(&d.tag[s]), 0ull,
                                                 (unsigned long long)t);
        if (old == 0) break;
        s = (s + 1) & d.mask;
    }
    d.slot_id[s] = ids_kg[o];
}

__global__ __launch_bounds__(kDictThreads) void k_dict_gather(DictDev d, int64_t n, const int64_t* ids, int64_t nids,
                                                              int64_t* off_out, int32_t* len_out) {
    const int64_t i = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    if (i >= n) return;
    const uint64_t ord = (uint64_t)ids[i] & kOrdMask;
    const bool ok = ids[i] >= 0 && (int64_t)ord < nids;
    off_out[i] = ok ? d.ent_off[ord] : -1;
    len_out[i] = ok ? d.ent_len[ord] : -1;
}

__global__ __launch_bounds__(kDictThreads) void k_fill_u64(uint64_t* p, int64_t n, uint64_t v) {
    const int64_t i = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    if (i < n) p[i] = v;
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
    Buf tag, slot_id, slot_row, ent_off, ent_len, ent_tag, ent_id, arena, counters;
    Buf in_bytes, in_off, in_len, row_tag, row_kg, row_slot, row_id;   // per-call scratch
    std::unordered_map<std::string, int64_t> side;   // rows whose tag another row holds
    std::string err;

    int fail(int rc, const std::string& m) {
        err = m;
        return rc;
    }
    DictDev dev() const {
        DictDev d;
        d.tag = tag.as<uint64_t>();
        d.slot_id = slot_id.as<int64_t>();
        d.slot_row = slot_row.as<uint32_t>();
        d.ent_off = ent_off.as<int64_t>();
        d.ent_len = ent_len.as<int32_t>();
        d.ent_tag = ent_tag.as<uint64_t>();
        d.arena = arena.as<uint8_t>();
        d.counters = counters.as<unsigned long long>();
        d.mask = cap - 1;
        return d;
    }
};

#define DCHK(d, x)                                                                     \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return (d)->fail(FG_EDEVICE, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)

namespace {

// ids of every entry (key group bits included), for a rebuild
__global__ __launch_bounds__(kDictThreads) void k_dict_ids(DictDev d, uint64_t cap, int64_t* ids_kg) {
    const int64_t s = (int64_t)blockIdx.x * kDictThreads + threadIdx.x;
    if (s >= (int64_t)cap) return;
    const int64_t id = d.slot_id[s];
    if (id >= 0) ids_kg[(uint64_t)id & kOrdMask] = id;
}

// table at `ncap` slots (power of two) holding every entry
int rebuild(fg_key_dict* d, uint64_t ncap) {
    hipStream_t s = d->stream;
    // the ids' key-group bits: from the old table (host-resolved ids are kept in ent_id)
    DCHK(d, d->ent_id.ensure(8 * (size_t)std::max<int64_t>(d->nids, 1), s, 8 * (size_t)d->nids));
    if (d->cap && d->nids)
        hipLaunchKernelGGL(k_dict_ids, dim3(grid_of((int64_t)d->cap)), dim3(kDictThreads), 0, s, d->dev(), d->cap,
                           d->ent_id.as<int64_t>());
    DCHK(d, hipGetLastError());
    Buf ntag, nid, nrow;
    DCHK(d, ntag.ensure(8 * ncap, s));
    DCHK(d, nid.ensure(8 * ncap, s));
    DCHK(d, nrow.ensure(4 * ncap, s));
    DCHK(d, hipMemsetAsync(ntag.p, 0, 8 * ncap, s));
    hipLaunchKernelGGL(k_fill_u64, dim3(grid_of((int64_t)ncap)), dim3(kDictThreads), 0, s, nid.as<uint64_t>(),
                       (int64_t)ncap, ~0ull);
    DCHK(d, hipGetLastError());
    std::swap(d->tag.p, ntag.p);
    std::swap(d->tag.bytes, ntag.bytes);
    std::swap(d->slot_id.p, nid.p);
    std::swap(d->slot_id.bytes, nid.bytes);
    std::swap(d->slot_row.p, nrow.p);
    std::swap(d->slot_row.bytes, nrow.bytes);
    d->cap = ncap;
    if (d->nids)
        hipLaunchKernelGGL(k_dict_rehash, dim3(grid_of(d->nids)), dim3(kDictThreads), 0, s, d->dev(), d->nids,
                           d->ent_id.as<int64_t>());
    DCHK(d, hipGetLastError());
    DCHK(d, hipStreamSynchronize(s));
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
    if (rebuild(d.get(), pow2_at_least(2 * (uint64_t)std::max<int64_t>(expected_keys, 1)))) return FG_EDEVICE;
    *out = d.release();
    return FG_OK;
}

int fg_key_dict_intern(fg_key_dict* d, int32_t location, int64_t n, const uint8_t* bytes, int64_t nbytes,
                       const int64_t* offsets, const int32_t* lengths, int64_t* out_id, int32_t* out_kg) {
    if (!d) return FG_EINVAL;
    if (n == 0) return FG_OK;
    if (n < 0 || n > 0x7fffffff || !bytes || nbytes < 0 || !offsets || !lengths || !out_id)
        return d->fail(FG_EINVAL, "fg_key_dict_intern: invalid arguments");
    if (hipSetDevice(d->device) != hipSuccess) return d->fail(FG_EDEVICE, "hipSetDevice failed");
    hipStream_t s = d->stream;
    const bool host = location == FG_HOST;
    if (host) {   // validate on the host: every row inside the buffer, 4-byte words
        for (int64_t i = 0; i < n; i++) {
            if (lengths[i] < 0 || (lengths[i] & 3) || (offsets[i] & 3) || offsets[i] < 0 ||
                offsets[i] + lengths[i] > nbytes)
                return d->fail(FG_EINVAL, "key row " + std::to_string(i) +
                                              ": offset/length outside the buffer or not a multiple of 4 bytes");
        }
    }
    // room: the table stays at most half full, the arena takes every row of the call
    if ((uint64_t)(d->nids + n) * 2 > d->cap)
        if (int rc = rebuild(d, pow2_at_least(4 * (uint64_t)(d->nids + n)))) return rc;
    const size_t ents = (size_t)(d->nids + n);
    DCHK(d, d->ent_off.ensure(8 * ents, s, 8 * (size_t)d->nids));
    DCHK(d, d->ent_len.ensure(4 * ents, s, 4 * (size_t)d->nids));
    DCHK(d, d->ent_tag.ensure(8 * ents, s, 8 * (size_t)d->nids));
    DCHK(d, d->arena.ensure((size_t)d->arena_used + (size_t)nbytes + 8 * (size_t)n + 8, s, (size_t)d->arena_used));
    RowsIn in{};
    in.n = n;
    in.nbytes = nbytes;
    in.max_p = d->max_p;
    in.tag_bits = d->tag_bits;
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
    DCHK(d, d->row_tag.ensure(8 * (size_t)n, s));
    DCHK(d, d->row_kg.ensure(4 * (size_t)n, s));
    DCHK(d, d->row_slot.ensure(8 * (size_t)n, s));
    int64_t* ids = out_id;
    if (host) {
        DCHK(d, d->row_id.ensure(8 * (size_t)n, s));
        ids = d->row_id.as<int64_t>();
    }
    const DictDev dv = d->dev();
    const unsigned g = grid_of(n);
    hipLaunchKernelGGL(k_dict_hash, dim3(g), dim3(kDictThreads), 0, s, in, d->row_tag.as<uint64_t>(),
                       d->row_kg.as<int32_t>(), dv.counters);
    DCHK(d, hipGetLastError());
    if (!host) {   // device rows are checked on the device before anything is inserted
        unsigned long long bad = 0;
        DCHK(d, hipMemcpyAsync(&bad, dv.counters + 3, 8, hipMemcpyDeviceToHost, s));
        DCHK(d, hipStreamSynchronize(s));
        if (bad) {
            DCHK(d, hipMemsetAsync(dv.counters + 3, 0, 8, s));
            DCHK(d, hipStreamSynchronize(s));
            return d->fail(FG_EINVAL, "fg_key_dict_intern: " + std::to_string(bad) +
                                          " key rows outside the buffer or not a multiple of 4 bytes");
        }
    }
    hipLaunchKernelGGL(k_dict_claim, dim3(g), dim3(kDictThreads), 0, s, dv, n, d->row_tag.as<uint64_t>(),
                       d->row_slot.as<uint64_t>());
    hipLaunchKernelGGL(k_dict_assign, dim3(g), dim3(kDictThreads), 0, s, dv, in, d->row_slot.as<uint64_t>(),
                       d->row_tag.as<uint64_t>(), d->row_kg.as<int32_t>());
    hipLaunchKernelGGL(k_dict_verify, dim3(g), dim3(kDictThreads), 0, s, dv, in, d->row_slot.as<uint64_t>(), ids);
    DCHK(d, hipGetLastError());
    unsigned long long cnt[4];
    DCHK(d, hipMemcpyAsync(cnt, d->counters.p, sizeof cnt, hipMemcpyDeviceToHost, s));
    DCHK(d, hipStreamSynchronize(s));
    d->nids = (int64_t)cnt[0];
    d->arena_used = (int64_t)cnt[1];
    if (cnt[2]) {
        // rows whose 64-bit tag another row holds: exact ids from the host-side map, their rows
        // appended to the arena (ent_tag 0: never rehashed into the table)
        std::vector<int64_t> hid(n);
        std::vector<int32_t> hkg(n);
        DCHK(d, hipMemcpy(hid.data(), ids, 8 * (size_t)n, hipMemcpyDeviceToHost));
        DCHK(d, hipMemcpy(hkg.data(), d->row_kg.p, 4 * (size_t)n, hipMemcpyDeviceToHost));
        std::vector<uint8_t> row;
        for (int64_t i = 0; i < n; i++) {
            if (hid[i] >= 0) continue;
            const int32_t len = host ? lengths[i] : 0;
            int64_t off = 0;
            int32_t l = len;
            if (host) {
                off = offsets[i];
                row.assign(bytes + off, bytes + off + len);
            } else {
                DCHK(d, hipMemcpy(&off, offsets + i, 8, hipMemcpyDeviceToHost));
                DCHK(d, hipMemcpy(&l, lengths + i, 4, hipMemcpyDeviceToHost));
                row.resize(l);
                if (l) DCHK(d, hipMemcpy(row.data(), bytes + off, (size_t)l, hipMemcpyDeviceToHost));
            }
            std::string k(row.begin(), row.end());
            auto it = d->side.find(k);
            int64_t id;
            if (it != d->side.end()) {
                id = it->second;
            } else {
                const int64_t ord = d->nids++;
                const int64_t at = d->arena_used;
                d->arena_used += (l + 7) & ~7;
                DCHK(d, d->ent_off.ensure(8 * (size_t)d->nids, s, 8 * (size_t)ord));
                DCHK(d, d->ent_len.ensure(4 * (size_t)d->nids, s, 4 * (size_t)ord));
                DCHK(d, d->ent_tag.ensure(8 * (size_t)d->nids, s, 8 * (size_t)ord));
                DCHK(d, d->arena.ensure((size_t)d->arena_used, s, (size_t)at));
                std::vector<uint8_t> padded((l + 7) & ~7, 0);
                std::copy(row.begin(), row.end(), padded.begin());
                const uint64_t zero = 0;
                if (!padded.empty()) DCHK(d, hipMemcpy(d->arena.as<uint8_t>() + at, padded.data(), padded.size(), hipMemcpyHostToDevice));
                DCHK(d, hipMemcpy(d->ent_off.as<int64_t>() + ord, &at, 8, hipMemcpyHostToDevice));
                DCHK(d, hipMemcpy(d->ent_len.as<int32_t>() + ord, &l, 4, hipMemcpyHostToDevice));
                DCHK(d, hipMemcpy(d->ent_tag.as<uint64_t>() + ord, &zero, 8, hipMemcpyHostToDevice));
                id = (int64_t)((uint64_t)hkg[i] << kIdShift | (uint64_t)ord);
                d->side.emplace(std::move(k), id);
            }
            hid[i] = id;
        }
        DCHK(d, hipMemcpy(ids, hid.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
        const unsigned long long c2[3] = {(unsigned long long)d->nids, (unsigned long long)d->arena_used, 0ull};
        DCHK(d, hipMemcpy(d->counters.p, c2, sizeof c2, hipMemcpyHostToDevice));
    }
    if (host) DCHK(d, hipMemcpy(out_id, ids, 8 * (size_t)n, hipMemcpyDeviceToHost));
    if (out_kg) {
        DCHK(d, hipMemcpy(out_kg, d->row_kg.p, 4 * (size_t)n, host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice));
    }
    return FG_OK;
}

int fg_key_dict_lookup(fg_key_dict* d, int32_t location, int64_t n, const int64_t* ids, int64_t* out_offsets,
                       int32_t* out_lengths) {
    if (!d) return FG_EINVAL;
    if (n == 0) return FG_OK;
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
    if (!d || begin < 0 || nbytes < 0 || begin + nbytes > d->arena_used || (nbytes && !host))
        return d ? d->fail(FG_EINVAL, "fg_key_dict_copy_arena: range outside the arena") : FG_EINVAL;
    if (!nbytes) return FG_OK;
    if (hipSetDevice(d->device) != hipSuccess) return d->fail(FG_EDEVICE, "hipSetDevice failed");
    DCHK(d, hipMemcpy(host, d->arena.as<uint8_t>() + begin, (size_t)nbytes, hipMemcpyDeviceToHost));
    return FG_OK;
}

int64_t fg_key_dict_size(fg_key_dict* d) { return d ? d->nids : -1; }

const char* fg_key_dict_last_error(fg_key_dict* d) { return d ? d->err.c_str() : "null dictionary"; }

void fg_key_dict_close(fg_key_dict* d) {
    if (!d) return;
    (void)hipSetDevice(d->device);
    hipStream_t s = d->stream;
    if (s) (void)hipStreamSynchronize(s);
    delete d;
    if (s) (void)hipStreamDestroy(s);
}

int32_t fg_binaryrow_hash(const uint8_t* row, int32_t len) {
    if (!row || len < 0 || (len & 3)) return 0;
    return binaryrow_hash_bytes(row, len);
}

}  // extern "C"
