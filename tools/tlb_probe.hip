// Probe: W waves each read C random "cells" (4 KB contiguous) from a buffer of
// S bytes, one cell after another (the k_kpp_eval item pattern).  Time per
// launch vs S: a TLB/page-walk bound shows as a strong dependence on S.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
__global__ __launch_bounds__(256) void k_cells(const float *__restrict__ buf, unsigned long long ncell, int per_wave,
                                               unsigned seed, float *out) {
    const int lane = threadIdx.x & 63;
    const unsigned long long wid = (blockIdx.x * 256ull + threadIdx.x) >> 6;
    float acc = 0.f;
    unsigned long long h = wid * 0x9E3779B97F4A7C15ull + seed;
    for (int c = 0; c < per_wave; ++c) {
        h ^= h >> 31; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 29;
        const unsigned long long cell = (unsigned long long)__shfl((long long)(h % ncell), 0);
        const float *p = buf + cell * 1024;   // 4 KB cell
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = p[u * 64 + lane];
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += v[u];
    }
    if (acc == 1234.5f) out[0] = acc;
}
int main() {
    const size_t total = 1ull << 31;   // 2 GiB
    float *buf, *out;
    hipMalloc(&buf, total);
    hipMalloc(&out, 64);
    hipMemset(buf, 0, total);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (size_t S : {size_t(8) << 20, size_t(32) << 20, size_t(128) << 20, size_t(512) << 20, total}) {
        for (int pw : {1, 2, 4}) {
            const unsigned long long ncell = S / 4096;
            float best = 1e9f;
            for (int rep = 0; rep < 5; ++rep) {
                hipEventRecord(a);
                k_cells<<<512, 256>>>(buf, ncell, pw, 17u + rep, out);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                best = ms < best ? ms : best;
            }
            printf("span %5zu MiB  cells/wave %d (2048 waves): %7.2f us\n", S >> 20, pw, best * 1e3f);
        }
    }
    return 0;
}
