// Prototype (experiment, not product): TUMBLE fire straight from pass-1 tiles.
//
// Pass 1 sorts each tile by CONSUMER bucket (4 state regions = region >> 2: 2,048 buckets at
// 2^13 regions) and writes it back sequentially (block-laid 12-B records) with a directory row
// per tile; a transpose gives each consumer its fragments' (offset, length) column; the consumer
// (one workgroup per bucket, persistent) gathers its fragment of every tile, aggregates the
// bucket's ~4.9k keys in an LDS table and emits the fired rows -- no staged area written and
// read back (pass 2 + merge of the engine). Measures the three kernels on 100M records / 10M keys.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o scripts/exp/tile_proto scripts/exp/tile_proto.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__);   \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

constexpr int NB = 13;                 // region bits
constexpr int CBITS = 2;               // regions per consumer bucket = 4
constexpr int NC = 1 << (NB - CBITS);  // 2,048 consumer buckets
#ifndef P1T
#define P1T 1024
#endif
#ifndef P1R
#define P1R 8
#endif
constexpr int T1 = P1T, R1 = P1R, TILE = T1 * R1;
constexpr int G1 = 256;                // pass-1 workgroups
constexpr int TC = 1024;               // consumer threads
#ifndef SLOTS
#define SLOTS 8192
#endif
constexpr int S = SLOTS;               // LDS table slots
#ifndef WIN
#define WIN 256                        // consumer: records per wave window (WIN / 64 per lane)
#endif
constexpr int kBlk = 768;              // 64 narrow records: 64 int32 keys, then 64 values
#ifndef PACKED
#define PACKED 1                       // 1: packed 12-B records {key, value lo, value hi}; 0: block-laid
#endif

__host__ __device__ inline uint64_t fmix64(uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdULL;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ULL;
    h ^= h >> 33;
    return h;
}
__host__ __device__ inline uint64_t splitmix(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_gen(int64_t n, int64_t K, int64_t* key, int64_t* ts, double* val) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t u = splitmix(0x5EEDF11Cull ^ (uint64_t)i), u2 = splitmix((0x5EEDF11Cull * 3 + 1) ^ (uint64_t)i);
        key[i] = (int64_t)(u % (uint64_t)K);
        ts[i] = 1600000000000ll + i / 100000;
        val[i] = (double)(u2 >> 11) * (1000.0 / 9007199254740992.0);
    }
}

__device__ inline void seg(int64_t n, int g, int64_t* b, int64_t* e) {
    int64_t per = (n + G1 - 1) / G1;
    per = (per + 63) & ~int64_t(63);   // whole 64-record blocks per segment
    *b = per * g < n ? per * g : n;
    *e = *b + per < n ? *b + per : n;
}

__device__ inline void st12(char* base, uint64_t i, uint32_t k, uint64_t v) {
    char* b = base + (i >> 6) * kBlk;
    reinterpret_cast<uint32_t*>(b)[i & 63] = k;
    reinterpret_cast<uint64_t*>(b + 256)[i & 63] = v;
}

// ---- pass 1: tile sort by consumer bucket ------------------------------------------------
__global__ __launch_bounds__(T1) void k_p1(int64_t n, const int64_t* key, const int64_t* ts, const double* val,
                                          char* tmp, uint16_t* dir, int MT) {
#if PACKED
    __shared__ uint4 s_w4[(TILE * 3 + 3) / 4];       // the sorted tile as packed 12-B records
    uint32_t* s_w = reinterpret_cast<uint32_t*>(s_w4);
#else
    __shared__ uint32_t s_k[TILE];
    __shared__ uint64_t s_v[TILE];
#endif
    __shared__ uint32_t s_cc[NC + 1];
    __shared__ uint32_t s_wave[T1 / 64];
    const int tid = threadIdx.x;
    int64_t beg, end;
    seg(n, blockIdx.x, &beg, &end);
    for (int i = tid; i <= NC; i += T1) s_cc[i] = 0;
    __syncthreads();
    int64_t kk[R1], vv[R1];
    auto load = [&](int64_t t0) {
#pragma unroll
        for (int u = 0; u < R1; u++) {
            const int64_t i = t0 + u * T1 + tid;
            kk[u] = i < end ? key[i] : 0;
            vv[u] = i < end ? __double_as_longlong(val[i]) : 0;
            if (i < end && ts[i] < 0) kk[u] = -1;   // (keeps the rowtime stream read: 24 B per record)
        }
    };
    if (beg < end) load(beg);
    int j = 0;
    for (int64_t t0 = beg; t0 < end; t0 += TILE, j++) {
        uint32_t rc[R1];
        uint32_t k32[R1];
        uint64_t v64[R1];
#pragma unroll
        for (int u = 0; u < R1; u++) {
            const int64_t i = t0 + u * T1 + tid;
            rc[u] = 0xffffffffu;
            k32[u] = (uint32_t)kk[u];
            v64[u] = (uint64_t)vv[u];
            if (i >= end) continue;
            const uint64_t h = fmix64((uint64_t)kk[u]);
            const uint32_t c = (uint32_t)(h >> (64 - (NB - CBITS)));
            rc[u] = (atomicAdd(&s_cc[c], 1u) << 11) | c;
        }
        if (t0 + TILE < end) load(t0 + TILE);
        __syncthreads();
        {   // exclusive scan of NC counts, 2 per thread
            const uint32_t a = s_cc[2 * tid], b = s_cc[2 * tid + 1];
            uint32_t x = a + b;
            const int ln = tid & 63, w = tid >> 6;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off);
                if (ln >= off) x += y;
            }
            if (ln == 63) s_wave[w] = x;
            __syncthreads();
            uint32_t wb = 0;
            for (int q = 0; q < w; q++) wb += s_wave[q];
            const uint32_t ex = wb + x - a - b;
            __syncthreads();
            s_cc[2 * tid] = ex;
            s_cc[2 * tid + 1] = ex + a;
            if (tid == T1 - 1) s_cc[NC] = ex + a + b;
        }
        __syncthreads();
        uint16_t* drow = dir + ((int64_t)blockIdx.x * MT + j) * (NC + 1);
        for (int c = tid; c <= NC; c += T1) drow[c] = (uint16_t)s_cc[c];
        const uint32_t total = s_cc[NC];
#pragma unroll
        for (int u = 0; u < R1; u++) {
            if (rc[u] == 0xffffffffu) continue;
            const uint32_t slot = s_cc[rc[u] & 2047u] + (rc[u] >> 11);
#if PACKED
            s_w[3 * slot] = k32[u];
            s_w[3 * slot + 1] = (uint32_t)v64[u];
            s_w[3 * slot + 2] = (uint32_t)(v64[u] >> 32);
#else
            s_k[slot] = k32[u];
            s_v[slot] = v64[u];
#endif
        }
        __syncthreads();
#if PACKED
        {   // the tile's bytes as aligned 16-B stores (12 * t0 is 16-B aligned: TILE % 4 == 0)
            uint4* dst = reinterpret_cast<uint4*>(tmp + 12 * (uint64_t)t0);
            const uint32_t nch = (total * 12 + 15) / 16;
            for (uint32_t i = tid; i < nch; i += T1) dst[i] = s_w4[i];
        }
#else
        for (uint32_t i = tid; i < total; i += T1) st12(tmp, (uint64_t)(t0 + i), s_k[i], s_v[i]);
#endif
        __syncthreads();
        for (int c = tid; c <= NC; c += T1) s_cc[c] = 0;
        __syncthreads();
    }
}

// ---- directory transpose: dt[c][t] = off | len << 16 ------------------------------------
__global__ __launch_bounds__(256) void k_dirt(const uint16_t* dir, int NT, uint32_t* dt) {
    __shared__ uint16_t s[64][65 + 1];
    const int tb = blockIdx.x * 64, cb = blockIdx.y * 64;
    for (int i = threadIdx.x; i < 64 * 65; i += 256) {
        const int tt = i / 65, cc = i % 65;
        const int t = tb + tt, c = cb + cc;
        s[tt][cc] = (t < NT && c <= NC) ? dir[(int64_t)t * (NC + 1) + c] : 0;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int cc = i / 64, tt = i % 64;
        const int t = tb + tt, c = cb + cc;
        if (t < NT && c < NC) {
            const uint32_t a = s[tt][cc], b = s[tt][cc + 1];
            dt[(int64_t)c * NT + t] = a | ((b - a) << 16);
        }
    }
}

// ---- consumer: gather + LDS aggregate + emit ------------------------------------------------
struct Out {
    int64_t *key, *ws, *we, *cs, *sum, *avg;
    uint8_t* nul;
    unsigned long long* count;
};
constexpr int32_t kEmpty = INT32_MIN;
// order a wave's LDS writes before its other lanes' reads (no workgroup barrier)
__device__ inline void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(TC) void k_tm(int64_t n, const char* tmp, const uint32_t* dt, int NT, int MT, Out o,
                                          int64_t ws, int64_t we, int mode) {
    __shared__ int32_t t_key[S];
    __shared__ uint32_t t_cs[S];
    __shared__ double t_v[S];
    __shared__ uint8_t s_fm[TC / 64][WIN];           // per-wave fragment map (u8 lane ids)
    __shared__ uint32_t s_dl[TC / 64][64];           // per-wave fragment delta (src - idx)
    __shared__ uint32_t s_grp[(S / TC + 1) * (TC / 64)];
    __shared__ uint16_t s_map[S];
    __shared__ uint32_t s_total;
    __shared__ unsigned long long s_base;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int W = TC / 64;
    const int G = gridDim.x;
    const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8, per_xcd = G / 8;
    const int per = NC / 8;
    int64_t per1 = (n + G1 - 1) / G1;
    per1 = (per1 + 63) & ~int64_t(63);
    for (int k = 0;; k++) {
        const int ci = slot + k * per_xcd;
        if (ci >= per) break;
        const int c = xcd * per + ci;
        for (int i = tid; i < S; i += TC) {
            t_key[i] = kEmpty;
            t_cs[i] = 0;
            t_v[i] = 0.0;
        }
        __syncthreads();
        const uint32_t* col = dt + (int64_t)c * NT;
        constexpr int RPL = WIN / 64;   // records per lane per window
        // home bucket: a multiplicative 32-bit hash of the key (keys of one consumer share the
        // top bits of their fmix64 mix, not of the key itself)
        auto home_of = [&](int32_t k) -> uint32_t {
            return __umulhi((uint32_t)k * 0x9E3779B1u, (uint32_t)(S / 4)) * 4;
        };
        auto resolve = [&](int32_t k, uint32_t home, int4 q4) -> int {
            for (int probe = 0; probe < S / 4; probe++) {
                const int32_t qq[4] = {q4.x, q4.y, q4.z, q4.w};
                int hit = -1, emp = -1;
#pragma unroll
                for (int z = 3; z >= 0; z--) {
                    if (qq[z] == k) hit = z;
                    if (qq[z] == kEmpty) emp = z;
                }
                if (hit >= 0 && (emp < 0 || hit < emp)) return home + hit;
                if (emp >= 0) {
                    const int old = atomicCAS(&t_key[home + emp], kEmpty, k);
                    if (old == kEmpty || old == k) return home + emp;
                } else {
                    home = (home + 4) & (S - 1);
                }
                q4 = *reinterpret_cast<const int4*>(&t_key[home]);
            }
            return -1;
        };
        // window iterator over this wave's groups of 64 tiles (group gi: tiles t0 .. t0 + 63,
        // t0 = (wave + gi * W) * 64); a window = up to WIN consecutive records of a group
        int t0 = wave * 64 - W * 64;   // (advanced to the first group below)
        uint32_t xn = wave * 64 + lane < NT ? col[wave * 64 + lane] : 0u;   // next group's entry, prefetched
        uint32_t g_len = 0, g_st = 0, g_tot = 0, b = 0;
        auto next_window = [&](int32_t (&kr)[RPL], double (&vr)[RPL], uint32_t& nrec) -> bool {
            while (b >= g_tot) {   // the next non-empty group
                t0 += W * 64;
                if (t0 >= NT) return false;
                const int t = t0 + lane;
                const uint32_t x = xn;
                xn = t + W * 64 < NT ? col[t + W * 64] : 0u;
                const uint32_t off = x & 0xffffu;
                g_len = x >> 16;
                const int g = t / MT, jj = t % MT;
                const uint32_t base = (uint32_t)(per1 * g + (int64_t)jj * TILE) + off;
                uint32_t inc = g_len;
                for (int s = 1; s < 64; s <<= 1) {
                    const uint32_t y = __shfl_up(inc, s);
                    if (lane >= s) inc += y;
                }
                g_st = inc - g_len;
                g_tot = __shfl(inc, 63);
                b = 0;
                wave_sync();   // (the previous group's reads of s_dl are done: its loads are issued)
                s_dl[wave][lane] = base - g_st;
            }
#pragma unroll
            for (int q = 0; q < RPL; q++) s_fm[wave][lane * RPL + q] = 0;
            wave_sync();
            if (g_len > 0 && g_st < b + WIN && g_st + g_len > b) s_fm[wave][g_st > b ? g_st - b : 0] = (uint8_t)lane;
            wave_sync();
            uint32_t e[RPL];
#pragma unroll
            for (int q = 0; q < RPL; q++) e[q] = s_fm[wave][lane * RPL + q];
#pragma unroll
            for (int q = 1; q < RPL; q++) e[q] = e[q] > e[q - 1] ? e[q] : e[q - 1];
            uint32_t m = e[RPL - 1];
            for (int s = 1; s < 64; s <<= 1) {
                const uint32_t y = __shfl_up(m, s);
                if (lane >= s) m = m > y ? m : y;
            }
            uint32_t pre = __shfl_up(m, 1);
            if (lane == 0) pre = 0;
#pragma unroll
            for (int q = 0; q < RPL; q++) s_fm[wave][lane * RPL + q] = (uint8_t)(e[q] > pre ? e[q] : pre);
            wave_sync();
            nrec = g_tot - b < WIN ? g_tot - b : WIN;
#pragma unroll
            for (int u = 0; u < RPL; u++) {
                const uint32_t jr = lane + 64 * u;
                kr[u] = 0;
                vr[u] = 0;
                if (jr < nrec) {
                    const uint32_t src = s_dl[wave][s_fm[wave][jr]] + b + jr;
                    // (round 4 had a "mode 2" no-gather diagnostic here that synthesised
                    // c * 4096 + (src & 4095) keys: more distinct keys than the consumer's
                    // table holds, so its probe ran past the table -- the illegal access in
                    // gpurun_out/proto3.log. Removed in round 5.)
                    {
#if PACKED
                        const uint3 w = *reinterpret_cast<const uint3*>(tmp + 12 * (uint64_t)src);
                        kr[u] = (int32_t)w.x;
                        vr[u] = __longlong_as_double((long long)(((uint64_t)w.z << 32) | w.y));
#else
                        const char* blk = tmp + (uint64_t)(src >> 6) * kBlk;
                        kr[u] = reinterpret_cast<const int32_t*>(blk)[src & 63];
                        vr[u] = reinterpret_cast<const double*>(blk + 256)[src & 63];
#endif
                    }
                }
            }
            b += WIN;
            return true;
        };
        auto insert_window = [&](const int32_t (&kr)[RPL], const double (&vr)[RPL], uint32_t nrec) {
            if (mode & 1) {
#pragma unroll
                for (int u = 0; u < RPL; u++)
                    if (lane + 64 * u < nrec && vr[u] == -1.0 && kr[u] == 7) o.count[1] = 1;
                return;
            }
            // every home bucket read first (RPL 16-B LDS reads in flight), then resolved
            uint32_t hm[RPL];
            int4 bq[RPL];
#pragma unroll
            for (int u = 0; u < RPL; u++) {
                hm[u] = home_of(kr[u]);
                bq[u] = *reinterpret_cast<const int4*>(&t_key[hm[u]]);
            }
#pragma unroll
            for (int u = 0; u < RPL; u++) {
                if (lane + 64 * u >= nrec) continue;
                const int sl = resolve(kr[u], hm[u], bq[u]);
                atomicAdd(&t_cs[sl], 1u);
                atomicAdd(&t_v[sl], vr[u]);
            }
        };
        {   // two windows in flight: the next window's loads are issued before this one's inserts
            int32_t ka[RPL], kb[RPL];
            double va[RPL], vb[RPL];
            uint32_t na = 0, nb = 0;
            bool more = next_window(ka, va, na);
            while (more) {
                const bool hb = next_window(kb, vb, nb);
                insert_window(ka, va, na);
                if (!hb) break;
                more = next_window(ka, va, na);
                insert_window(kb, vb, nb);
            }
        }
        __syncthreads();
        // emit: dense rank -> slot map, then one row per occupied slot
        constexpr int RN = S / TC;
        uint32_t occm = 0;
#pragma unroll
        for (int r = 0; r < RN; r++) {
            const bool occ = t_cs[r * TC + tid] != 0;
            const uint64_t bal = __ballot(occ);
            if (occ) occm |= 1u << r;
            if (lane == 0) s_grp[r * W + wave] = (uint32_t)__popcll(bal);
        }
        __syncthreads();
        if (wave == 0) {
            constexpr int NG = RN * W;   // 128
            const uint32_t a = 2 * lane < NG ? s_grp[2 * lane] : 0u, b = 2 * lane + 1 < NG ? s_grp[2 * lane + 1] : 0u;
            uint32_t x = a + b;
            for (int s = 1; s < 64; s <<= 1) {
                const uint32_t y = __shfl_up(x, s);
                if (lane >= s) x += y;
            }
            const uint32_t ex = x - a - b;
            if (2 * lane < NG) s_grp[2 * lane] = ex;
            if (2 * lane + 1 < NG) s_grp[2 * lane + 1] = ex + a;
            const uint32_t total = __shfl(x, 63);
            if (lane == 0) {
                s_total = total;
                s_base = atomicAdd(o.count, (unsigned long long)total);
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RN; r++) {
            const bool occ = (occm >> r) & 1;
            const uint64_t bal = __ballot(occ);
            if (occ) s_map[s_grp[r * W + wave] + (uint32_t)__popcll(bal & ((1ull << lane) - 1))] = (uint16_t)(r * TC + tid);
        }
        __syncthreads();
        const uint32_t total = s_total;
        const unsigned long long ob = s_base;
        for (uint32_t i = tid; i < total; i += TC) {
            const int sl = s_map[i];
            const uint64_t r = ob + i;
            const uint32_t cnt = t_cs[sl];
            const double sm = t_v[sl];
            o.key[r] = (int64_t)t_key[sl];
            o.ws[r] = ws;
            o.we[r] = we;
            o.cs[r] = cnt;
            o.sum[r] = __double_as_longlong(sm);
            o.avg[r] = __double_as_longlong(sm / (double)cnt);
            o.nul[r] = 0;
        }
        __syncthreads();
    }
}

__global__ void k_check(const int64_t* cs, const double* sum, int64_t rows, unsigned long long* tot_cnt, double* tot_sum) {
    unsigned long long c = 0;
    double s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows; i += (int64_t)gridDim.x * blockDim.x) {
        c += (unsigned long long)cs[i];
        s += sum[i];
    }
    atomicAdd(tot_cnt, c);
    atomicAdd(tot_sum, s);
}
__global__ void k_sumv(const double* v, int64_t n, double* out) {
    double s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) s += v[i];
    atomicAdd(out, s);
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
    const int64_t K = argc > 2 ? atoll(argv[2]) : 10000000;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int mode = argc > 4 ? atoi(argv[4]) : 0;
    int64_t *key, *ts;
    double* val;
    CK(hipMalloc(&key, 8 * n));
    CK(hipMalloc(&ts, 8 * n));
    CK(hipMalloc(&val, 8 * n));
    k_gen<<<4096, 256>>>(n, K, key, ts, val);
    int64_t per1 = (n + G1 - 1) / G1;
    per1 = (per1 + 63) & ~int64_t(63);
    const int MT = (int)((per1 + TILE - 1) / TILE);
    const int NT = G1 * MT;
    char* tmp;
    uint16_t* dir;
    uint32_t* dt;
    CK(hipMalloc(&tmp, (size_t)(n / 64 + 2) * kBlk + 64));
    CK(hipMalloc(&dir, (size_t)NT * (NC + 1) * 2));
    CK(hipMalloc(&dt, (size_t)NT * NC * 4));
    CK(hipMemset(dir, 0, (size_t)NT * (NC + 1) * 2));
    Out o;
    const int64_t cap = K + K / 8 + 1024;
    CK(hipMalloc(&o.key, 8 * cap));
    CK(hipMalloc(&o.ws, 8 * cap));
    CK(hipMalloc(&o.we, 8 * cap));
    CK(hipMalloc(&o.cs, 8 * cap));
    CK(hipMalloc(&o.sum, 8 * cap));
    CK(hipMalloc(&o.avg, 8 * cap));
    CK(hipMalloc(&o.nul, cap));
    CK(hipMalloc(&o.count, 64));
    hipEvent_t e[4];
    for (auto& x : e) CK(hipEventCreate(&x));
    float t1 = 0, t2 = 0, t3 = 0;
    unsigned long long rows = 0;
    for (int r = 0; r < reps + 1; r++) {
        CK(hipMemsetAsync(o.count, 0, 8));
        CK(hipEventRecord(e[0]));
        k_p1<<<G1, T1>>>(n, key, ts, val, tmp, dir, MT);
        CK(hipEventRecord(e[1]));
        k_dirt<<<dim3((NT + 63) / 64, (NC + 63) / 64 + 1), 256>>>(dir, NT, dt);
        CK(hipEventRecord(e[2]));
        k_tm<<<256, TC>>>(n, tmp, dt, NT, MT, o, 1600000000000ll, 1600000001000ll, mode);
        CK(hipEventRecord(e[3]));
        CK(hipEventSynchronize(e[3]));
        float a, b, c;
        CK(hipEventElapsedTime(&a, e[0], e[1]));
        CK(hipEventElapsedTime(&b, e[1], e[2]));
        CK(hipEventElapsedTime(&c, e[2], e[3]));
        if (r > 0) {
            t1 += a;
            t2 += b;
            t3 += c;
        }
        CK(hipMemcpy(&rows, o.count, 8, hipMemcpyDeviceToHost));
    }
    unsigned long long* tc;
    double *tsum, *vsum;
    CK(hipMalloc(&tc, 8));
    CK(hipMalloc(&tsum, 8));
    CK(hipMalloc(&vsum, 8));
    CK(hipMemset(tc, 0, 8));
    CK(hipMemset(tsum, 0, 8));
    CK(hipMemset(vsum, 0, 8));
    k_check<<<1024, 256>>>(o.cs, (const double*)o.sum, (int64_t)rows, tc, tsum);
    k_sumv<<<1024, 256>>>(val, n, vsum);
    unsigned long long hc;
    double hs, hv;
    CK(hipMemcpy(&hc, tc, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hs, tsum, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hv, vsum, 8, hipMemcpyDeviceToHost));
    const double exp_rows = (double)K * (1.0 - exp(-(double)n / (double)K));
    printf("n=%lld K=%lld tile=%d MT=%d NT=%d slots=%d\n", (long long)n, (long long)K, TILE, MT, NT, S);
    printf("rows %llu (expected ~%.0f)  count sum %llu (n %lld)  value sum rel diff %.3g\n", rows, exp_rows, hc,
           (long long)n, fabs(hs - hv) / hv);
    printf("pass1 %.3f ms  (%.2f TB/s at 36 B/rec)\n", t1 / reps, 36.0 * n / (t1 / reps * 1e-3) / 1e12);
    printf("dir^T %.3f ms\n", t2 / reps);
    printf("tile merge %.3f ms  (%.2f TB/s at 12 B/rec + 49 B/row)\n", t3 / reps,
           (12.0 * n + 49.0 * rows) / (t3 / reps * 1e-3) / 1e12);
    printf("total %.3f ms per %lld records\n", (t1 + t2 + t3) / reps, (long long)n);
    return 0;
}
