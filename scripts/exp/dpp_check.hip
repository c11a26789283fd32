// Checks the DPP wave scans of fg_kernels.hip (wave_incl_scan, wave_shr1) against a host
// reference: pure register arithmetic, no data-dependent addressing. Prints PASS / FAIL.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <bool MAX>
__device__ __forceinline__ uint32_t dpp_op(uint32_t a, uint32_t b) { return MAX ? (a > b ? a : b) : a + b; }
template <bool MAX>
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = dpp_op<MAX>(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}
__global__ void k(const uint32_t* in, uint32_t* out, int reps) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int r = 0; r < reps; r++) {
        const uint32_t v = in[(r * 256 + threadIdx.x) % 4096];
        const uint32_t a = wave_incl_scan<false>(v);
        const uint32_t m = wave_incl_scan<true>(v & 255u);
        const uint32_t s = wave_shr1(m);
        uint32_t* o = out + ((size_t)r * 256 + w * 64 + lane) * 3;
        o[0] = a; o[1] = m; o[2] = s;
    }
}
// the tile walk's group setup (fg_kernels.hip tile_walk_next): per lane two directory entries
// x = offset | len << 16 of tiles t = t0 + 2 lane + q; dl[q] = base[q] - g_st[q]
template <bool OPAQUE>
__global__ void kg(const uint32_t* xs, uint32_t* dl_out, uint32_t* tot_out, int t0) {
    const int lane = threadIdx.x & 63;
    uint32_t base[2], g_st[2], g_len[2], sum = 0;
    for (int q = 0; q < 2; q++) {
        const int t = t0 + lane * 2 + q;
        const uint32_t x = xs[lane * 2 + q];
        g_len[q] = x >> 16;
        base[q] = (uint32_t)t * 6144u + (x & 0xffffu);
        g_st[q] = sum;
        sum += g_len[q];
    }
    uint32_t inc = wave_incl_scan<false>(sum);
    if (OPAQUE) asm volatile("" : "+v"(inc));
    const uint32_t ex = inc - sum;
    tot_out[lane] = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    for (int q = 0; q < 2; q++) {
        g_st[q] += ex;
        dl_out[lane * 2 + q] = base[q] - g_st[q];
    }
}
static int check_group(bool opaque) {
    std::vector<uint32_t> xs(128);
    uint64_t x = 99;
    for (auto& v : xs) { x = x * 6364136223846793005ull + 1442695040888963407ull; v = ((uint32_t)(x >> 33) % 7) << 16 | ((uint32_t)(x >> 45) % 6000); }
    uint32_t *dx, *dd, *dt;
    hipMalloc(&dx, 4 * 128); hipMalloc(&dd, 4 * 128); hipMalloc(&dt, 4 * 64);
    hipMemcpy(dx, xs.data(), 4 * 128, hipMemcpyHostToDevice);
    if (opaque) kg<true><<<1, 64>>>(dx, dd, dt, 4096); else kg<false><<<1, 64>>>(dx, dd, dt, 4096);
    std::vector<uint32_t> dl(128), tot(64);
    hipMemcpy(dl.data(), dd, 4 * 128, hipMemcpyDeviceToHost);
    hipMemcpy(tot.data(), dt, 4 * 64, hipMemcpyDeviceToHost);
    uint32_t st = 0;
    int bad = 0;
    for (int i = 0; i < 128; i++) {
        const uint32_t base = (uint32_t)(4096 + i) * 6144u + (xs[i] & 0xffffu);
        if (dl[i] != base - st) { if (bad < 5) printf("group%s: entry %d dl %u want %u\n", opaque ? "(opaque)" : "", i, dl[i], base - st); bad++; }
        st += xs[i] >> 16;
    }
    for (int l = 0; l < 64; l++) if (tot[l] != st) { if (bad < 8) printf("group: tot %u want %u\n", tot[l], st); bad++; }
    printf("group setup%s: %s\n", opaque ? " (opaque scan)" : "", bad ? "FAIL" : "PASS");
    return bad;
}
int main() {
    int gb = check_group(false) + check_group(true);
    const int reps = 16;
    std::vector<uint32_t> in(4096);
    uint64_t x = 12345;
    for (auto& v : in) { x = x * 6364136223846793005ull + 1442695040888963407ull; v = (uint32_t)(x >> 40) & 1023u; }
    uint32_t *din, *dout;
    hipMalloc(&din, 4 * in.size());
    hipMalloc(&dout, 4 * 3 * 256 * reps);
    hipMemcpy(din, in.data(), 4 * in.size(), hipMemcpyHostToDevice);
    k<<<1, 256>>>(din, dout, reps);
    std::vector<uint32_t> out(3 * 256 * reps);
    if (hipMemcpy(out.data(), dout, 4 * out.size(), hipMemcpyDeviceToHost) != hipSuccess) { printf("FAIL: copy\n"); return 1; }
    int bad = 0;
    for (int r = 0; r < reps; r++)
        for (int w = 0; w < 4; w++) {
            uint32_t a = 0, m = 0, prev_m = 0;
            for (int l = 0; l < 64; l++) {
                const uint32_t v = in[(r * 256 + w * 64 + l) % 4096];
                a += v;
                const uint32_t mm = (v & 255u) > m ? (v & 255u) : m;
                const uint32_t* o = &out[((size_t)r * 256 + w * 64 + l) * 3];
                const uint32_t sh = l == 0 ? 0u : prev_m;
                if (o[0] != a || o[1] != mm || o[2] != sh) {
                    if (bad < 10) printf("r%d w%d lane %d: add %u/%u max %u/%u shr %u/%u\n", r, w, l, o[0], a, o[1], mm, o[2], sh);
                    bad++;
                }
                m = mm;
                prev_m = mm;
            }
        }
    printf(bad ? "FAIL: %d mismatches\n" : "PASS (%d)\n", bad);
    return bad || gb ? 1 : 0;
}
