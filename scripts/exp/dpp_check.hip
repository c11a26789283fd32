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
int main() {
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
    return bad ? 1 : 0;
}
