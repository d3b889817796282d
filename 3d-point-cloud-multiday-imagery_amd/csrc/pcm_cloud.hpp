// pcm_cloud.hpp — per-pair point-cloud assembly on gfx950 (SURVEY.md §8 rows
// a1-a4 / f2): the float64 pipeline of members/rafael/disparity/plugin.py:147-192.
//
//   k_cloud_flags    height = -disp/16; valid = finite & |h| <= limit & validity
//   (rocprim scan)   row-major output slots of the valid pixels (np.where order)
//   k_cloud_compact  P = [x, y, z] of every valid pixel
//   k_cloud_sums     per-block sums of x, y, z (then of the 6 centred products)
//   (host)           mean, 3x3 covariance, Jacobi eigen-solve: the plane normal
//                    is the eigenvector of the smallest eigenvalue (= Vh[2] of the
//                    SVD of the centred points), oriented to +z
//   k_cloud_project  relative height P_c . n
//   (rocprim sort)   2nd / 98th percentiles (numpy 'linear')
//   k_cloud_output   points (z - h_min, y, x) and h_norm clipped to [0, 1]
// All HBM-bound byte/elementwise work; sums are float64 block trees (parity with
// numpy to float64 rounding, not bit-exact).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pcm {

constexpr int CLOUD_TPB = 256;

__global__ __launch_bounds__(CLOUD_TPB) void k_cloud_flags(const double *__restrict__ disp,
                                                           const uint8_t *__restrict__ validity, long long n,
                                                           double limit, uint32_t *__restrict__ flags,
                                                           double *__restrict__ height) {
    const long long i = blockIdx.x * (long long)CLOUD_TPB + threadIdx.x;
    if (i >= n) return;
    const double h = -disp[i] / 16.0;
    const bool v = __builtin_isfinite(h) && fabs(h) <= limit && (validity ? validity[i] != 0 : true);
    flags[i] = v ? 1u : 0u;
    height[i] = h;
}

__global__ __launch_bounds__(CLOUD_TPB) void k_cloud_compact(const uint32_t *__restrict__ flags,
                                                             const uint32_t *__restrict__ pos,
                                                             const double *__restrict__ height, long long n,
                                                             long long W, double *__restrict__ P) {
    const long long i = blockIdx.x * (long long)CLOUD_TPB + threadIdx.x;
    if (i >= n || !flags[i]) return;
    const long long j = pos[i];
    P[3 * j + 0] = (double)(i % W);
    P[3 * j + 1] = (double)(i / W);
    P[3 * j + 2] = height[i];
}

// MODE 0: sums of x, y, z.  MODE 1: sums of the 6 products of centred coordinates.
template <int MODE>
__global__ __launch_bounds__(CLOUD_TPB) void k_cloud_sums(const double *__restrict__ P, long long m, double cx,
                                                          double cy, double cz, double *__restrict__ part) {
    constexpr int NV = MODE == 0 ? 3 : 6;
    double acc[NV];
    for (int v = 0; v < NV; ++v) acc[v] = 0.0;
    for (long long j = blockIdx.x * (long long)CLOUD_TPB + threadIdx.x; j < m;
         j += (long long)gridDim.x * CLOUD_TPB) {
        const double x = P[3 * j], y = P[3 * j + 1], z = P[3 * j + 2];
        if (MODE == 0) {
            acc[0] += x; acc[1] += y; acc[2] += z;
        } else {
            const double a = x - cx, b = y - cy, c = z - cz;
            acc[0] += a * a; acc[1] += a * b; acc[2] += a * c;
            acc[3] += b * b; acc[4] += b * c; acc[5] += c * c;
        }
    }
    __shared__ double red[NV][CLOUD_TPB / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int v = 0; v < NV; ++v) {
        double s = acc[v];
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) red[v][wv] = s;
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        double s = 0.0;
        for (int w = 0; w < CLOUD_TPB / 64; ++w) s += red[threadIdx.x][w];
        part[(size_t)blockIdx.x * NV + threadIdx.x] = s;
    }
}

__global__ __launch_bounds__(CLOUD_TPB) void k_cloud_project(const double *__restrict__ P, long long m, double cx,
                                                             double cy, double cz, double n0, double n1, double n2,
                                                             double *__restrict__ zrel) {
    const long long j = blockIdx.x * (long long)CLOUD_TPB + threadIdx.x;
    if (j >= m) return;
    zrel[j] = ((P[3 * j] - cx) * n0 + (P[3 * j + 1] - cy) * n1) + (P[3 * j + 2] - cz) * n2;
}

__global__ __launch_bounds__(CLOUD_TPB) void k_cloud_output(const double *__restrict__ P,
                                                            const double *__restrict__ zrel, long long m,
                                                            double h_min, double h_max,
                                                            double *__restrict__ points,
                                                            double *__restrict__ hnorm) {
    const long long j = blockIdx.x * (long long)CLOUD_TPB + threadIdx.x;
    if (j >= m) return;
    const double z = zrel[j];
    const double hn = (z - h_min) / (h_max - h_min + 1e-6);
    hnorm[j] = hn < 0.0 ? 0.0 : (hn > 1.0 ? 1.0 : hn);
    points[3 * j + 0] = z - h_min;
    points[3 * j + 1] = P[3 * j + 1];
    points[3 * j + 2] = P[3 * j];
}

}  // namespace pcm
