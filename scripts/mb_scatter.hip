// Microbenchmark (not product code): how fast can 16-B records be partitioned into F
// buckets on gfx950? Measures, for 50M records (key, ts, val i64 columns):
//   copy      : read 24 B, write 16 B sequentially (upper bound)
//   loadonly  : read 24 B, classify, LDS histogram (the count pass shape)
//   direct    : read 24 B, write 16 B to cursor[b]++ (per-WG cursors in LDS, bases from a count pass)
// for several F and workgroup shapes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__host__ __device__ inline uint64_t fmix64(uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdULL;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ULL;
    h ^= h >> 33;
    return h;
}

__device__ inline void seg(int64_t n, int g, int G, int64_t* b, int64_t* e) {
    int64_t per = (n + G - 1) / G;
    per = (per + 1) & ~int64_t(1);
    *b = std::min<int64_t>(per * g, n);
    *e = std::min<int64_t>(*b + per, n);
}

template <int T>
__global__ __launch_bounds__(T) void k_copy(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n,
                                            longlong2* out) {
    for (int64_t i = (int64_t)blockIdx.x * T + threadIdx.x; i < n / 2; i += (int64_t)gridDim.x * T) {
        longlong2 k = reinterpret_cast<const longlong2*>(key)[i];
        longlong2 t = reinterpret_cast<const longlong2*>(ts)[i];
        longlong2 v = reinterpret_cast<const longlong2*>(val)[i];
        out[2 * i] = make_longlong2(k.x + (t.x & 1), v.x);
        out[2 * i + 1] = make_longlong2(k.y + (t.y & 1), v.y);
    }
}

template <int T>
__global__ __launch_bounds__(T) void k_count(const int64_t* key, const int64_t* ts, int64_t n, int bits,
                                             uint32_t* hist) {
    __shared__ uint32_t h[8192];
    const int F = 1 << bits;
    for (int i = threadIdx.x; i < F; i += T) h[i] = 0;
    __syncthreads();
    int64_t b, e;
    seg(n, blockIdx.x, gridDim.x, &b, &e);
    const int64_t np = (e - b) / 2;
    for (int64_t p0 = 0; p0 < np; p0 += 4 * T) {
        longlong2 k[4], t[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            int64_t p = p0 + u * T + threadIdx.x;
            if (p < np) {
                k[u] = reinterpret_cast<const longlong2*>(key + b)[p];
                t[u] = reinterpret_cast<const longlong2*>(ts + b)[p];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            int64_t p = p0 + u * T + threadIdx.x;
            if (p < np) {
                atomicAdd(&h[(fmix64(k[u].x + (t[u].x >> 62)) >> (64 - bits))], 1u);
                atomicAdd(&h[(fmix64(k[u].y + (t[u].y >> 62)) >> (64 - bits))], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < F; i += T) hist[(int64_t)blockIdx.x * F + i] = h[i];
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_direct(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n,
                                              int bits, const uint32_t* base, longlong2* out) {
    __shared__ uint32_t cur[8192];
    const int F = 1 << bits;
    for (int i = threadIdx.x; i < F; i += T) cur[i] = base[(int64_t)blockIdx.x * F + i];
    __syncthreads();
    int64_t b, e;
    seg(n, blockIdx.x, gridDim.x, &b, &e);
    const int64_t np = (e - b) / 2;
    for (int64_t p0 = 0; p0 < np; p0 += U * T) {
        longlong2 k[U], t[U], v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            int64_t p = p0 + u * T + threadIdx.x;
            if (p < np) {
                k[u] = reinterpret_cast<const longlong2*>(key + b)[p];
                t[u] = reinterpret_cast<const longlong2*>(ts + b)[p];
                v[u] = reinterpret_cast<const longlong2*>(val + b)[p];
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            int64_t p = p0 + u * T + threadIdx.x;
            if (p < np) {
                uint32_t p1 = atomicAdd(&cur[fmix64(k[u].x + (t[u].x >> 62)) >> (64 - bits)], 1u);
                uint32_t p2 = atomicAdd(&cur[fmix64(k[u].y + (t[u].y >> 62)) >> (64 - bits)], 1u);
                out[p1] = make_longlong2(k[u].x, v[u].x);
                out[p2] = make_longlong2(k[u].y, v[u].y);
            }
        }
    }
}


template <int NT_>
__device__ inline uint32_t block_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    if (w == 0) {
        uint32_t q = lane < NT_ / 64 ? s_w[lane] : 0;
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t y = __shfl_up(q, o);
            if (lane >= o) q += y;
        }
        if (lane < NT_ / 64) s_w[lane] = q;
    }
    __syncthreads();
    uint32_t base = w ? s_w[w - 1] : 0;
    *total = s_w[NT_ / 64 - 1];
    __syncthreads();
    return base + x - v;
}

// tile-sorted scatter: R records per thread in registers, LDS rounds of RS slots
template <int NT_, int R, int RS, int FMAX, bool NTS, bool NTL = false>
__global__ __launch_bounds__(NT_) void k_tiled(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n,
                                               int bits, const uint32_t* base, longlong2* out) {
    constexpr int T = NT_ * R;
    __shared__ longlong2 s_rec[RS];
    __shared__ uint16_t s_bkt[RS];
    __shared__ uint32_t s_cur[FMAX], s_off[FMAX + 1];
    __shared__ uint32_t s_w[16];
    const int F = 1 << bits;
    const int tid = threadIdx.x;
    for (int i = tid; i < F; i += NT_) { s_cur[i] = base[(int64_t)blockIdx.x * F + i]; s_off[i] = 0; }
    __syncthreads();
    int64_t b, e;
    seg(n, blockIdx.x, gridDim.x, &b, &e);
    for (int64_t t0 = b; t0 < e; t0 += T) {
        const int64_t tn = std::min<int64_t>(T, e - t0);
        int64_t rk[R], rv[R];
        uint32_t rb[R];
#pragma unroll
        for (int j = 0; j < R / 2; j++) {
            const int64_t li = 2 * ((int64_t)tid + (int64_t)j * NT_);
            longlong2 k2 = {0, 0}, t2 = {0, 0}, vv = {0, 0};
            if (li + 1 < tn) {
                if (NTL) {
                    typedef long long v2 __attribute__((ext_vector_type(2)));
                    v2 a = __builtin_nontemporal_load(reinterpret_cast<const v2*>(key + t0 + li));
                    v2 c = __builtin_nontemporal_load(reinterpret_cast<const v2*>(ts + t0 + li));
                    v2 d = __builtin_nontemporal_load(reinterpret_cast<const v2*>(val + t0 + li));
                    k2 = make_longlong2(a.x, a.y); t2 = make_longlong2(c.x, c.y); vv = make_longlong2(d.x, d.y);
                } else {
                    k2 = *reinterpret_cast<const longlong2*>(key + t0 + li);
                    t2 = *reinterpret_cast<const longlong2*>(ts + t0 + li);
                    vv = *reinterpret_cast<const longlong2*>(val + t0 + li);
                }
            }
            rk[2 * j] = k2.x; rk[2 * j + 1] = k2.y; rv[2 * j] = vv.x; rv[2 * j + 1] = vv.y;
            rb[2 * j] = li < tn ? (uint32_t)(fmix64(k2.x + (t2.x >> 62)) >> (64 - bits)) : 0xffffu;
            rb[2 * j + 1] = li + 1 < tn ? (uint32_t)(fmix64(k2.y + (t2.y >> 62)) >> (64 - bits)) : 0xffffu;
        }
#pragma unroll
        for (int j = 0; j < R; j++)
            if (rb[j] != 0xffffu) rb[j] |= atomicAdd(&s_off[rb[j]], 1u) << 16;
        __syncthreads();
        {
            constexpr int PER = (FMAX + NT_ - 1) / NT_;
            uint32_t c[PER], loc = 0;
#pragma unroll
            for (int q = 0; q < PER; q++) { const int i = tid * PER + q; c[q] = i < F ? s_off[i] : 0; loc += c[q]; }
            uint32_t tot;
            uint32_t run = block_scan<NT_>(loc, s_w, &tot);
#pragma unroll
            for (int q = 0; q < PER; q++) { const int i = tid * PER + q; if (i < F) s_off[i] = run; run += c[q]; }
            if (tid == 0) s_off[F] = tot;
        }
        __syncthreads();
        const uint32_t tot = s_off[F];
        for (uint32_t lo = 0; lo < tot; lo += RS) {
#pragma unroll
            for (int j = 0; j < R; j++) {
                if ((rb[j] & 0xffffu) == 0xffffu) continue;
                const uint32_t bk = rb[j] & 0xffffu;
                const uint32_t slot = s_off[bk] + (rb[j] >> 16) - lo;
                if (slot < (uint32_t)RS) { s_rec[slot] = make_longlong2(rk[j], rv[j]); s_bkt[slot] = (uint16_t)bk; }
            }
            __syncthreads();
            const uint32_t hi = std::min<uint32_t>(RS, tot - lo);
            for (uint32_t i = tid; i < hi; i += NT_) {
                const uint32_t bk = s_bkt[i];
                const uint32_t pos = s_cur[bk] + (lo + i - s_off[bk]);
                if (NTS) { typedef long long v2 __attribute__((ext_vector_type(2))); const longlong2 r_ = s_rec[i]; v2 q_ = {r_.x, r_.y}; __builtin_nontemporal_store(q_, reinterpret_cast<v2*>(&out[pos])); }
                else out[pos] = s_rec[i];
            }
            __syncthreads();
        }
        for (int i = tid; i < F; i += NT_) { s_cur[i] += s_off[i + 1] - s_off[i]; }
        __syncthreads();
        for (int i = tid; i < F; i += NT_) s_off[i] = 0;
        __syncthreads();
    }
}

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
template <int NT_>
__device__ inline uint32_t block_scan_lds(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    lds_barrier();
    if (w == 0) {
        uint32_t q = lane < NT_ / 64 ? s_w[lane] : 0;
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t y = __shfl_up(q, o);
            if (lane >= o) q += y;
        }
        if (lane < NT_ / 64) s_w[lane] = q;
    }
    lds_barrier();
    uint32_t base = w ? s_w[w - 1] : 0;
    *total = s_w[NT_ / 64 - 1];
    lds_barrier();
    return base + x - v;
}

// tiled2: LDS-only barriers (stores stay in flight), optional register prefetch of the next tile
template <int NT_, int R, int RS, int FMAX, bool PF>
__global__ __launch_bounds__(NT_) void k_tiled2(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n,
                                                int bits, const uint32_t* base, longlong2* out) {
    constexpr int T = NT_ * R;
    __shared__ longlong2 s_rec[RS];
    __shared__ uint16_t s_bkt[RS];
    __shared__ uint32_t s_cur[FMAX], s_off[FMAX + 1];
    __shared__ uint32_t s_w[16];
    const int F = 1 << bits;
    const int tid = threadIdx.x;
    for (int i = tid; i < F; i += NT_) { s_cur[i] = base[(int64_t)blockIdx.x * F + i]; s_off[i] = 0; }
    __syncthreads();
    int64_t b, e;
    seg(n, blockIdx.x, gridDim.x, &b, &e);
    longlong2 pk[R / 2], pt[R / 2], pv[R / 2];
    auto load = [&](int64_t t0) {
        const int64_t tn = std::min<int64_t>(T, e - t0);
#pragma unroll
        for (int j = 0; j < R / 2; j++) {
            const int64_t li = 2 * ((int64_t)tid + (int64_t)j * NT_);
            if (li + 1 < tn) {
                pk[j] = *reinterpret_cast<const longlong2*>(key + t0 + li);
                pt[j] = *reinterpret_cast<const longlong2*>(ts + t0 + li);
                pv[j] = *reinterpret_cast<const longlong2*>(val + t0 + li);
            }
        }
    };
    if (PF && b < e) load(b);
    for (int64_t t0 = b; t0 < e; t0 += T) {
        const int64_t tn = std::min<int64_t>(T, e - t0);
        if (!PF) load(t0);
        int64_t rk[R], rv[R];
        uint32_t rb[R];
#pragma unroll
        for (int j = 0; j < R / 2; j++) {
            const int64_t li = 2 * ((int64_t)tid + (int64_t)j * NT_);
            const longlong2 k2 = pk[j], t2 = pt[j], v2 = pv[j];
            rk[2 * j] = k2.x; rk[2 * j + 1] = k2.y; rv[2 * j] = v2.x; rv[2 * j + 1] = v2.y;
            rb[2 * j] = li < tn ? (uint32_t)(fmix64(k2.x + (t2.x >> 62)) >> (64 - bits)) : 0xffffu;
            rb[2 * j + 1] = li + 1 < tn ? (uint32_t)(fmix64(k2.y + (t2.y >> 62)) >> (64 - bits)) : 0xffffu;
        }
        if (PF && t0 + T < e) load(t0 + T);
#pragma unroll
        for (int j = 0; j < R; j++)
            if (rb[j] != 0xffffu) rb[j] |= atomicAdd(&s_off[rb[j]], 1u) << 16;
        lds_barrier();
        {
            constexpr int PER = (FMAX + NT_ - 1) / NT_;
            uint32_t c[PER], loc = 0;
#pragma unroll
            for (int q = 0; q < PER; q++) { const int i = tid * PER + q; c[q] = i < F ? s_off[i] : 0; loc += c[q]; }
            uint32_t tot;
            uint32_t run = block_scan_lds<NT_>(loc, s_w, &tot);
#pragma unroll
            for (int q = 0; q < PER; q++) { const int i = tid * PER + q; if (i < F) s_off[i] = run; run += c[q]; }
            if (tid == 0) s_off[F] = tot;
        }
        lds_barrier();
        const uint32_t tot = s_off[F];
        for (uint32_t lo = 0; lo < tot; lo += RS) {
#pragma unroll
            for (int j = 0; j < R; j++) {
                if ((rb[j] & 0xffffu) == 0xffffu) continue;
                const uint32_t bk = rb[j] & 0xffffu;
                const uint32_t slot = s_off[bk] + (rb[j] >> 16) - lo;
                if (slot < (uint32_t)RS) { s_rec[slot] = make_longlong2(rk[j], rv[j]); s_bkt[slot] = (uint16_t)bk; }
            }
            lds_barrier();
            const uint32_t hi = std::min<uint32_t>(RS, tot - lo);
            for (uint32_t i = tid; i < hi; i += NT_) {
                const uint32_t bk = s_bkt[i];
                out[s_cur[bk] + (lo + i - s_off[bk])] = s_rec[i];
            }
            lds_barrier();
        }
        for (int i = tid; i < F; i += NT_) { s_cur[i] += s_off[i + 1] - s_off[i]; }
        lds_barrier();
        for (int i = tid; i < F; i += NT_) s_off[i] = 0;
        lds_barrier();
    }
}

// tile-sorted scatter that only writes whole 64-B segments: per bucket, the <= 3 records
// past the last aligned segment boundary are carried (LDS) into the next tile's run.
template <int NT_, int R, int RS, int FMAX>
__global__ __launch_bounds__(NT_) void k_carry(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n,
                                               int bits, const uint32_t* base, longlong2* out) {
    constexpr int T = NT_ * R;
    __shared__ longlong2 s_rec[RS];
    __shared__ uint16_t s_bkt[RS];
    __shared__ longlong2 s_cx[FMAX * 3];
    __shared__ uint32_t s_gs[FMAX], s_off[FMAX + 1], s_cn[FMAX], s_em[FMAX];
    __shared__ uint32_t s_w[16];
    const int F = 1 << bits;
    const int tid = threadIdx.x;
    for (int i = tid; i < F; i += NT_) { s_gs[i] = base[(int64_t)blockIdx.x * F + i]; s_off[i] = 0; s_cn[i] = 0; }
    __syncthreads();
    int64_t b, e;
    seg(n, blockIdx.x, gridDim.x, &b, &e);
    for (int64_t t0 = b; t0 < e; t0 += T) {
        const int64_t tn = std::min<int64_t>(T, e - t0);
        const bool last = t0 + T >= e;
        int64_t rk[R], rv[R];
        uint32_t rb[R];
#pragma unroll
        for (int j = 0; j < R / 2; j++) {
            const int64_t li = 2 * ((int64_t)tid + (int64_t)j * NT_);
            longlong2 k2 = {0, 0}, t2 = {0, 0}, vv = {0, 0};
            if (li + 1 < tn) {
                k2 = *reinterpret_cast<const longlong2*>(key + t0 + li);
                t2 = *reinterpret_cast<const longlong2*>(ts + t0 + li);
                vv = *reinterpret_cast<const longlong2*>(val + t0 + li);
            }
            rk[2 * j] = k2.x; rk[2 * j + 1] = k2.y; rv[2 * j] = vv.x; rv[2 * j + 1] = vv.y;
            rb[2 * j] = li < tn ? (uint32_t)(fmix64(k2.x + (t2.x >> 62)) >> (64 - bits)) : 0xffffu;
            rb[2 * j + 1] = li + 1 < tn ? (uint32_t)(fmix64(k2.y + (t2.y >> 62)) >> (64 - bits)) : 0xffffu;
        }
#pragma unroll
        for (int j = 0; j < R; j++)
            if (rb[j] != 0xffffu) rb[j] |= atomicAdd(&s_off[rb[j]], 1u) << 16;
        __syncthreads();
        {
            constexpr int PER = (FMAX + NT_ - 1) / NT_;
            uint32_t c[PER], loc = 0;
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const int i = tid * PER + q;
                c[q] = i < F ? s_off[i] + s_cn[i] : 0;   // carry + tile records
                loc += c[q];
            }
            uint32_t tot;
            uint32_t run = block_scan<NT_>(loc, s_w, &tot);
#pragma unroll
            for (int q = 0; q < PER; q++) {
                const int i = tid * PER + q;
                if (i < F) {
                    s_off[i] = run;
                    const uint32_t g0 = s_gs[i], g1 = g0 + c[q];
                    const uint32_t a1 = last ? g1 : (g1 & ~3u);
                    s_em[i] = a1 > g0 ? a1 - g0 : 0;
                }
                run += c[q];
            }
            if (tid == 0) s_off[F] = tot;
        }
        __syncthreads();
        const uint32_t tot = s_off[F];
        for (uint32_t lo = 0; lo < tot; lo += RS) {
            // carries of the previous tile lead their bucket's run
            for (int i = tid; i < F; i += NT_) {
                const uint32_t cn = s_cn[i];
                for (uint32_t q = 0; q < cn; q++) {
                    const uint32_t slot = s_off[i] + q - lo;
                    if (slot < (uint32_t)RS) { s_rec[slot] = s_cx[i * 3 + q]; s_bkt[slot] = (uint16_t)i; }
                }
            }
#pragma unroll
            for (int j = 0; j < R; j++) {
                if ((rb[j] & 0xffffu) == 0xffffu) continue;
                const uint32_t bk = rb[j] & 0xffffu;
                const uint32_t slot = s_off[bk] + s_cn[bk] + (rb[j] >> 16) - lo;
                if (slot < (uint32_t)RS) { s_rec[slot] = make_longlong2(rk[j], rv[j]); s_bkt[slot] = (uint16_t)bk; }
            }
            __syncthreads();
            const uint32_t hi = std::min<uint32_t>(RS, tot - lo);
            for (uint32_t i = tid; i < hi; i += NT_) {
                const uint32_t bk = s_bkt[i];
                const uint32_t k = lo + i - s_off[bk];
                if (k < s_em[bk]) out[s_gs[bk] + k] = s_rec[i];
                else s_cx[bk * 3 + (k - s_em[bk])] = s_rec[i];
            }
            __syncthreads();
        }
        for (int i = tid; i < F; i += NT_) {
            const uint32_t m = s_off[i + 1] - s_off[i];
            s_gs[i] += s_em[i];
            s_cn[i] = m - s_em[i];
        }
        __syncthreads();
        for (int i = tid; i < F; i += NT_) s_off[i] = 0;
        __syncthreads();
    }
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 50000000;
    const int keys = 10000000;
    std::vector<int64_t> hk(n), ht(n), hv(n);
    uint64_t x = 0x5EEDF11C;
    for (int64_t i = 0; i < n; i++) {
        x = fmix64(x + 0x9E3779B97F4A7C15ull);
        hk[i] = (int64_t)(x % keys);
        ht[i] = 1600000000000LL + i / 100000;
        hv[i] = (int64_t)(x >> 11);
    }
    int64_t *key, *ts, *val;
    longlong2* out;
    uint32_t* hist;
    CK(hipMalloc(&key, 8 * n));
    CK(hipMalloc(&ts, 8 * n));
    CK(hipMalloc(&val, 8 * n));
    CK(hipMalloc(&out, 16 * n + 4096));
    CK(hipMalloc(&hist, 4 * 8192 * 4096));
    CK(hipMemcpy(key, hk.data(), 8 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(ts, ht.data(), 8 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(val, hv.data(), 8 * n, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, double bytes, auto&& fn) {
        fn();
        CK(hipDeviceSynchronize());
        const int R = 5;
        CK(hipEventRecord(a));
        for (int r = 0; r < R; r++) fn();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= R;
        printf("%-40s %8.3f ms  %7.0f GB/s\n", name, ms, bytes / ms / 1e6);
        fflush(stdout);
    };

    std::vector<longlong2> ho(n);
    auto verify = [&](int F, int G) {
        CK(hipMemcpy(ho.data(), out, 16 * n, hipMemcpyDeviceToHost));
        const int bits = __builtin_ctz(F);
        // bucket order: records of bucket f occupy [sum_{f'<f} cnt, ...)
        std::vector<uint64_t> cnt(F, 0);
        for (int64_t i = 0; i < n; i++) cnt[fmix64(hk[i] + (ht[i] >> 62)) >> (64 - bits)]++;
        uint64_t s1 = 0, s2 = 0, x1 = 0, x2 = 0;
        for (int64_t i = 0; i < n; i++) { s1 += (uint64_t)hk[i] * 3 + (uint64_t)hv[i]; x1 ^= fmix64(hk[i] ^ hv[i]); }
        int64_t at = 0;
        bool ok = true;
        for (int f = 0; f < F && ok; f++) {
            for (uint64_t j = 0; j < cnt[f]; j++, at++) {
                const longlong2 r = ho[at];
                if ((fmix64(r.x) >> (64 - bits)) != (uint64_t)f) { ok = false; break; }
                s2 += (uint64_t)r.x * 3 + (uint64_t)r.y; x2 ^= fmix64(r.x ^ r.y);
            }
        }
        CK(hipMemset(out, 0, 16 * n));
        return ok && s1 == s2 && x1 == x2;
    };
    timeit("copy 24->16 (256x1024 thr)", 40.0 * n, [&] { hipLaunchKernelGGL((k_copy<256>), dim3(1024 * 8), dim3(256), 0, 0, key, ts, val, n, out); });
    for (int bits : {10, 12}) {
        const int F = 1 << bits;
        for (int G : {256}) {
            char nm[128];
            snprintf(nm, sizeof nm, "count F=%d G=%d T=256", F, G);
            timeit(nm, 16.0 * n, [&] { hipLaunchKernelGGL((k_count<256>), dim3(G), dim3(256), 0, 0, key, ts, n, bits, hist); });
            std::vector<uint32_t> h((size_t)G * F);
            CK(hipMemcpy(h.data(), hist, 4 * h.size(), hipMemcpyDeviceToHost));
            for (int K : {1, 8, 32, 256}) {
            // K groups of G/K workgroups, each group its own bucket-major area
            std::vector<uint32_t> base((size_t)G * F);
            uint32_t run = 0;
            const int per = G / K;
            for (int k = 0; k < K; k++)
                for (int f = 0; f < F; f++)
                    for (int g = k * per; g < (k + 1) * per; g++) {
                        base[(size_t)g * F + f] = run;
                        run += h[(size_t)g * F + f];
                    }
            if (run != (uint32_t)n) printf("bad total %u\n", run);
            CK(hipMemcpy(hist, base.data(), 4 * base.size(), hipMemcpyHostToDevice));
            printf("K=%d groups\n", K);
#define TILED(NT_, R, RS, NTS)                                                                                  \
    snprintf(nm, sizeof nm, "tiled F=%d G=%d thr=%d R=%d RS=%d nt=%d", F, G, NT_, R, RS, NTS);                \
    timeit(nm, 40.0 * n, [&] { hipLaunchKernelGGL((k_tiled<NT_, R, RS, 4096, NTS>), dim3(G), dim3(NT_), 0, 0, key, ts, val, n, bits, hist, out); });
#define TILED2(NT_, R, RS, FM, PF)                                                                                  \
    snprintf(nm, sizeof nm, "tiled2 F=%d G=%d thr=%d R=%d RS=%d pf=%d", F, G, NT_, R, RS, PF);                \
    timeit(nm, 40.0 * n, [&] { hipLaunchKernelGGL((k_tiled2<NT_, R, RS, FM, PF>), dim3(G), dim3(NT_), 0, 0, key, ts, val, n, bits, hist, out); });
#define TILEDN(NT_, R, RS, NTL)                                                                                  \
    snprintf(nm, sizeof nm, "tiled F=%d G=%d thr=%d R=%d RS=%d ntl=%d", F, G, NT_, R, RS, NTL);                \
    timeit(nm, 40.0 * n, [&] { hipLaunchKernelGGL((k_tiled<NT_, R, RS, 4096, false, NTL>), dim3(G), dim3(NT_), 0, 0, key, ts, val, n, bits, hist, out); });
#define CARRY(NT_, R, RS, FM)                                                                                  \
    snprintf(nm, sizeof nm, "carry F=%d G=%d thr=%d R=%d RS=%d", F, G, NT_, R, RS);                \
    timeit(nm, 40.0 * n, [&] { hipLaunchKernelGGL((k_carry<NT_, R, RS, FM>), dim3(G), dim3(NT_), 0, 0, key, ts, val, n, bits, hist, out); }); \

            if (G == 256) {
                TILEDN(1024, 12, 4096, false)
                if (F <= 1024) { CARRY(1024, 8, 4096, 1024) }
            }
            }
        }
    }
    return 0;
}
