// Microbenchmark (not product code): read side of two staging layouts for F buckets.
//   seq  : bucket-major layout (count + scatter): WG b streams bucket b's contiguous range
//   frag : tile-sorted layout (tiles of T records, each sorted by bucket, written sequentially):
//          WG b gathers its fragment from every tile (offsets transposed [b][t])
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

template <int NT, bool BIG>
__global__ __launch_bounds__(NT) void k_seq(const longlong2* rec, const uint32_t* bo, int team, unsigned long long* out) {
    __shared__ unsigned long long s_big[BIG ? 15000 : 1];
    // team members on one XCD: blocks x + 8 * (j + team * m) -> bucket 8 m + x, part j
    const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
    const int part = k % team, b = (k / team) * 8 + x;
    const uint32_t beg = bo[b], end = bo[b + 1];
    unsigned long long acc = 0;
    constexpr int U = 8;
    for (uint32_t i0 = beg; i0 < end; i0 += U * NT) {
        longlong2 r[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = i0 + u * NT + threadIdx.x;
            r[u] = i < end ? rec[i] : make_longlong2(0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; u++)
            if ((fmix64(r[u].x) & (team - 1)) == (uint64_t)part) acc += (uint64_t)r[u].x ^ (uint64_t)r[u].y;
    }
    if (BIG) { s_big[threadIdx.x] = acc; __syncthreads(); acc = s_big[(threadIdx.x + 1) % NT]; }
    atomicAdd(out, acc);
}

// 16 lanes per fragment; a wave covers 4 tiles per step
template <int NT, bool BIG>
__global__ __launch_bounds__(NT) void k_frag(const longlong2* rec, const uint32_t* offT, int ntiles, int team,
                                             unsigned long long* out) {
    __shared__ unsigned long long s_big[BIG ? 15000 : 1];
    const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
    const int part = k % team, b = (k / team) * 8 + x;
    const uint32_t* o0 = offT + (size_t)b * (ntiles + 1);   // [b][t]: start of fragment b in tile t
    const uint32_t* o1 = offT + (size_t)(b + 1) * (ntiles + 1);
    unsigned long long acc = 0;
    const int sub = threadIdx.x & 15, grp = threadIdx.x >> 4;   // NT/16 groups
    constexpr int G = NT / 16;
    constexpr int U = 4;
    for (int t0 = 0; t0 < ntiles; t0 += U * G) {
        longlong2 r[U][2];
        uint32_t bg[U], en[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + u * G + grp;
            bg[u] = t < ntiles ? o0[t] : 0;
            en[u] = t < ntiles ? o1[t] : 0;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t i = bg[u] + sub + 16 * h;
                r[u][h] = i < en[u] ? rec[i] : make_longlong2(0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
#pragma unroll
            for (int h = 0; h < 2; h++)
                if ((fmix64(r[u][h].x) & (team - 1)) == (uint64_t)part) acc += (uint64_t)r[u][h].x ^ (uint64_t)r[u][h].y;
            for (uint32_t i = bg[u] + sub + 32; i < en[u]; i += 16) {   // long fragments
                const longlong2 q = rec[i];
                if ((fmix64(q.x) & (team - 1)) == (uint64_t)part) acc += (uint64_t)q.x ^ (uint64_t)q.y;
            }
        }
    }
    if (BIG) { s_big[threadIdx.x] = acc; __syncthreads(); acc = s_big[(threadIdx.x + 1) % NT]; }
    atomicAdd(out, acc);
}

int main() {
    const int64_t n = 50000000;
    const int keys = 10000000;
    std::vector<longlong2> recs(n);
    uint64_t x = 0x5EEDF11C;
    for (int64_t i = 0; i < n; i++) {
        x = fmix64(x + 0x9E3779B97F4A7C15ull);
        recs[i] = make_longlong2((int64_t)(x % keys), (int64_t)(x >> 11));
    }
    longlong2 *d_seq, *d_frag;
    uint32_t *d_bo, *d_off;
    unsigned long long* d_out;
    CK(hipMalloc(&d_seq, 16 * n));
    CK(hipMalloc(&d_frag, 16 * n));
    CK(hipMalloc(&d_out, 8));
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
        unsigned long long v = 0;
        CK(hipMemcpy(&v, d_out, 8, hipMemcpyDeviceToHost));
        printf("%-44s %8.3f ms  %7.0f GB/s  (chk %llx)\n", name, ms, bytes / ms / 1e6, v);
        fflush(stdout);
    };
    for (int bits : {10, 11, 12}) {
        const int F = 1 << bits;
        // seq layout
        std::vector<uint32_t> cnt(F + 1, 0);
        for (int64_t i = 0; i < n; i++) cnt[(fmix64(recs[i].x) >> (64 - bits)) + 1]++;
        for (int f = 0; f < F; f++) cnt[f + 1] += cnt[f];
        std::vector<longlong2> seq(n);
        std::vector<uint32_t> cur(cnt.begin(), cnt.end() - 1);
        for (int64_t i = 0; i < n; i++) seq[cur[fmix64(recs[i].x) >> (64 - bits)]++] = recs[i];
        CK(hipMemcpy(d_seq, seq.data(), 16 * n, hipMemcpyHostToDevice));
        CK(hipMalloc(&d_bo, 4 * (F + 1)));
        CK(hipMemcpy(d_bo, cnt.data(), 4 * (F + 1), hipMemcpyHostToDevice));
        for (int T : {12288}) {
            const int ntiles = (int)((n + T - 1) / T);
            std::vector<longlong2> frag(n);
            std::vector<uint32_t> offT((size_t)(F + 1) * (ntiles + 1));
            std::vector<uint32_t> tc(F + 1);
            for (int t = 0; t < ntiles; t++) {
                const int64_t lo = (int64_t)t * T, hi = std::min<int64_t>(n, lo + T);
                std::fill(tc.begin(), tc.end(), 0);
                for (int64_t i = lo; i < hi; i++) tc[(fmix64(recs[i].x) >> (64 - bits)) + 1]++;
                for (int f = 0; f < F; f++) tc[f + 1] += tc[f];
                for (int f = 0; f <= F; f++) offT[(size_t)f * (ntiles + 1) + t] = (uint32_t)(lo + tc[f]);
                for (int64_t i = lo; i < hi; i++) frag[lo + tc[fmix64(recs[i].x) >> (64 - bits)]++] = recs[i];
            }
            CK(hipMalloc(&d_off, 4 * offT.size()));
            CK(hipMemcpy(d_frag, frag.data(), 16 * n, hipMemcpyHostToDevice));
            CK(hipMemcpy(d_off, offT.data(), 4 * offT.size(), hipMemcpyHostToDevice));
            for (int team : {1, 2, 4}) {
                char nm[128];
#define RUN(KN, NT, BIG, ...)                                                                            \
    snprintf(nm, sizeof nm, #KN " F=%d T=%d team=%d thr=%d big=%d", F, T, team, NT, BIG);               \
    timeit(nm, 16.0 * n, [&] { CK(hipMemset(d_out, 0, 8)); hipLaunchKernelGGL((KN<NT, BIG>), dim3(F * team), dim3(NT), 0, 0, __VA_ARGS__); });
                if (T == 12288) {
                    RUN(k_seq, 256, false, d_seq, d_bo, team, d_out)
                    RUN(k_seq, 1024, true, d_seq, d_bo, team, d_out)
                    RUN(k_seq, 512, true, d_seq, d_bo, team, d_out)
                }
                RUN(k_frag, 256, false, d_frag, d_off, ntiles, team, d_out)
                RUN(k_frag, 1024, true, d_frag, d_off, ntiles, team, d_out)
                RUN(k_frag, 512, true, d_frag, d_off, ntiles, team, d_out)
            }
            CK(hipFree(d_off));
        }
        CK(hipFree(d_bo));
    }
    return 0;
}
