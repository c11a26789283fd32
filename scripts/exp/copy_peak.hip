// HBM ceiling of streaming patterns on this box (experiment): read-only, copy, and the
// pass-1 shape (three 8-B columns read, one 16-B record written). Prints GB/s per pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef long long v2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_read(const v2* __restrict__ a, size_t n, long long* sink) {
    long long acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        v2 x = a[i];
        acc ^= x.x + x.y;
    }
    if (acc == 0x123456789) sink[0] = acc;
}
template <int U>
__global__ __launch_bounds__(256) void k_copy(const v2* __restrict__ a, v2* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += stride * U) {
        v2 x[U];
#pragma unroll
        for (int u = 0; u < U; u++) if (i + u * stride < n) x[u] = a[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; u++) if (i + u * stride < n) b[i + u * stride] = x[u];
    }
}
// pass-1 shape: key, ts, val columns (2 records per lane per 16-B load) -> 16-B records
template <int U>
__global__ __launch_bounds__(256) void k_p1(const v2* __restrict__ k, const v2* __restrict__ t, const v2* __restrict__ v,
                                            v2* __restrict__ out, size_t npairs) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < npairs; i += stride * U) {
        v2 a[U], b[U], c[U];
#pragma unroll
        for (int u = 0; u < U; u++) if (i + u * stride < npairs) { a[u] = k[i + u * stride]; b[u] = t[i + u * stride]; c[u] = v[i + u * stride]; }
#pragma unroll
        for (int u = 0; u < U; u++) if (i + u * stride < npairs) {
            v2 r0 = {a[u].x ^ b[u].x, c[u].x}, r1 = {a[u].y ^ b[u].y, c[u].y};
            out[2 * (i + u * stride)] = r0;
            out[2 * (i + u * stride) + 1] = r1;
        }
    }
}

int main() {
    const size_t bytes = (size_t)2 << 30;   // 2 GiB per buffer
    const size_t n = bytes / 16;
    v2 *a, *b, *c, *d, *o;
    long long* sink;
    hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMalloc(&c, bytes); hipMalloc(&d, bytes); hipMalloc(&o, 2 * bytes);
    hipMalloc(&sink, 8);
    hipMemset(a, 1, bytes); hipMemset(b, 2, bytes); hipMemset(c, 3, bytes); hipMemset(d, 4, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto timeit = [&](const char* name, double gb, auto launch) {
        launch(); hipDeviceSynchronize();
        float best = 1e9;
        for (int r = 0; r < 5; r++) {
            hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); best = ms < best ? ms : best;
        }
        printf("%-28s %8.3f ms  %7.0f GB/s\n", name, best, gb / best * 1e3);
    };
    for (int g : {1024, 2048, 4096, 8192}) {
        char nm[64];
        snprintf(nm, 64, "read grid %d", g);
        timeit(nm, bytes / 1e9, [&] { hipLaunchKernelGGL(k_read, dim3(g), dim3(256), 0, 0, a, n, sink); });
        snprintf(nm, 64, "copy U1 grid %d", g);
        timeit(nm, 2 * bytes / 1e9, [&] { hipLaunchKernelGGL(k_copy<1>, dim3(g), dim3(256), 0, 0, a, b, n); });
        snprintf(nm, 64, "copy U4 grid %d", g);
        timeit(nm, 2 * bytes / 1e9, [&] { hipLaunchKernelGGL(k_copy<4>, dim3(g), dim3(256), 0, 0, a, b, n); });
        snprintf(nm, 64, "p1 U1 grid %d", g);
        timeit(nm, (3 * bytes + 2 * bytes) / 1e9, [&] { hipLaunchKernelGGL(k_p1<1>, dim3(g), dim3(256), 0, 0, b, c, d, o, n); });
        snprintf(nm, 64, "p1 U2 grid %d", g);
        timeit(nm, (3 * bytes + 2 * bytes) / 1e9, [&] { hipLaunchKernelGGL(k_p1<2>, dim3(g), dim3(256), 0, 0, b, c, d, o, n); });
    }
    return 0;
}
