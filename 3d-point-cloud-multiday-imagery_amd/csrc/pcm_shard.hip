// pcm_shard.hip — spatial slab sharding of a row-sharded cloud.
//
// The multi-GPU fit receives contiguous ROW shards (rank r holds rows
// [gidx0, gidx0 + n)).  Every shard of a uniform cloud spans the whole bounding
// box, so each rank's pruning grid would be a coarse one over the full box and
// its per-iteration fixed work (candidate lists for every cell of that box)
// would not shrink with the number of ranks.  At layout time the driver
// (pcm_amd/lloyd.py) therefore moves every point to the rank owning its slab of
// the longest axis:
//
//   pcm_shard_hist        histogram of the slab coordinate over nbins bins
//                         (SUM all-reduced; equal-count cut points on the host)
//   pcm_shard_partition   stable partition of the local rows by destination rank
//                         (rows keep their original order inside every
//                         destination), with each row's global index
//   (all_to_all of rows and indices; the engine lays out its slab and keeps
//    the global indices for the relocation tie-break, pcm_layout_shard)
//   pcm_shard_scatter_labels  labels returned by the reverse all_to_all ->
//                         the caller's original row order
//
// The bin of a point is floor((x_axis - lo) * inv) in fp64 from the exact
// input value, clamped to [0, nbins) -- restated by tests/cpu_engine.py.
// HBM-bound streaming kernels run once per cloud.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <string>

#include "pcm_common.hpp"
#include "pcm_kmeans.h"

namespace pcm_shard {

constexpr int TPB = 256;
constexpr int ROUNDS = 16;                  // points per thread per block
constexpr int CHUNK = TPB * ROUNDS;         // points per partition block (contiguous rows)
constexpr int HIST_BINS_MAX = 16384;        // LDS histogram (64 KB of uint32)

template <typename T> __device__ __forceinline__ double to_d(T v);
template <> __device__ __forceinline__ double to_d<float>(float v) { return (double)v; }
template <> __device__ __forceinline__ double to_d<__half>(__half v) { return (double)__half2float(v); }

__device__ __forceinline__ int bin_of(double x, double lo, double inv, int nbins) {
    const double t = (x - lo) * inv;
    int b = (int)floor(t);
    return b < 0 ? 0 : (b >= nbins ? nbins - 1 : b);
}

template <typename T>
__global__ __launch_bounds__(TPB) void k_shard_hist(const T *__restrict__ X, long long n, int d, int axis, double lo,
                                                    double inv, int nbins, unsigned long long *__restrict__ hist) {
    __shared__ unsigned int h[HIST_BINS_MAX];
    for (int b = threadIdx.x; b < nbins; b += TPB) h[b] = 0u;
    __syncthreads();
    for (long long i = blockIdx.x * (long long)TPB + threadIdx.x; i < n; i += (long long)gridDim.x * TPB)
        atomicAdd(&h[bin_of(to_d<T>(X[i * d + axis]), lo, inv, nbins)], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < nbins; b += TPB)
        if (h[b]) atomicAdd(hist + b, (unsigned long long)h[b]);
}

// Pass 1: rows of block b's chunk per destination -> cnt[dest * nblk + b].
template <typename T>
__global__ __launch_bounds__(TPB) void k_shard_count(const T *__restrict__ X, long long n, int d, int axis, double lo,
                                                     double inv, int nbins, const uint8_t *__restrict__ owner, int P,
                                                     uint32_t *__restrict__ cnt) {
    __shared__ unsigned int c[PCM_SHARD_MAXP];
    if (threadIdx.x < PCM_SHARD_MAXP) c[threadIdx.x] = 0u;
    __syncthreads();
    const long long base = (long long)blockIdx.x * CHUNK;
    for (int r = 0; r < ROUNDS; ++r) {
        const long long i = base + (long long)r * TPB + threadIdx.x;
        if (i < n) atomicAdd(&c[owner[bin_of(to_d<T>(X[i * d + axis]), lo, inv, nbins)]], 1u);
    }
    __syncthreads();
    if ((int)threadIdx.x < P) cnt[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = c[threadIdx.x];
}

// Destination totals from the exclusive scan of cnt (dest-major): tot[p].
__global__ void k_shard_totals(const uint32_t *__restrict__ off, const uint32_t *__restrict__ cnt, int nblk, int P,
                               long long *__restrict__ tot) {
    const int p = threadIdx.x;
    if (p >= P) return;
    const long long a = off[(size_t)p * nblk];
    const long long b = (p + 1 < P) ? (long long)off[(size_t)(p + 1) * nblk]
                                     : (long long)off[(size_t)P * nblk - 1] + cnt[(size_t)P * nblk - 1];
    tot[p] = b - a;
}

// Pass 2: stable scatter.  Each round of 256 rows ranks its rows per
// destination by wave ballots + a 4-wave prefix, so rows keep their original
// order inside each destination segment.
template <typename T>
__global__ __launch_bounds__(TPB) void k_shard_scatter(const T *__restrict__ X, long long n, int d, int axis, double lo,
                                                       double inv, int nbins, const uint8_t *__restrict__ owner, int P,
                                                       const uint32_t *__restrict__ off, long long gidx0,
                                                       T *__restrict__ Xout, uint32_t *__restrict__ rows_out) {
    __shared__ unsigned int basep[PCM_SHARD_MAXP];
    __shared__ unsigned int wc[TPB / 64][PCM_SHARD_MAXP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < P) basep[tid] = off[(size_t)tid * gridDim.x + blockIdx.x];
    const long long base = (long long)blockIdx.x * CHUNK;
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int r = 0; r < ROUNDS; ++r) {
        const long long i = base + (long long)r * TPB + tid;
        const bool valid = i < n;
        const int dest = valid ? (int)owner[bin_of(to_d<T>(X[i * d + axis]), lo, inv, nbins)] : -1;
        unsigned int mine = 0;
        for (int p = 0; p < P; ++p) {
            const unsigned long long m = __ballot(dest == p);
            if (dest == p) mine = (unsigned int)__popcll(m & below);
            if (lane == 0) wc[wave][p] = (unsigned int)__popcll(m);
        }
        __syncthreads();
        if (valid) {
            unsigned int pos = basep[dest] + mine;
            for (int w = 0; w < wave; ++w) pos += wc[w][dest];
            for (int a = 0; a < d; ++a) Xout[(size_t)pos * d + a] = X[i * d + a];
            rows_out[pos] = (uint32_t)(gidx0 + i);
        }
        __syncthreads();
        if (tid < P) {
            unsigned int s = 0;
            for (int w = 0; w < TPB / 64; ++w) s += wc[w][tid];
            basep[tid] += s;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(TPB) void k_shard_labels(const int32_t *__restrict__ lab, const uint32_t *__restrict__ rows,
                                                      long long n, long long gidx0, int32_t *__restrict__ out) {
    const long long i = blockIdx.x * (long long)TPB + threadIdx.x;
    if (i < n) out[(long long)rows[i] - gidx0] = lab[i];
}

int blocks(long long n, int per) { return (int)std::max(1LL, (n + per - 1) / per); }

size_t align256(size_t v) { return (v + 255) / 256 * 256; }

size_t scan_bytes(size_t m) {
    size_t b = 0;
    if (rocprim::exclusive_scan(nullptr, b, (uint32_t *)nullptr, (uint32_t *)nullptr, 0u, m, rocprim::plus<uint32_t>(),
                                (hipStream_t)0) != hipSuccess)
        return 0;
    return b;
}

}  // namespace pcm_shard

using namespace pcm_shard;

extern "C" {

int pcm_shard_hist(const void *X, int dtype, int64_t n, int d, int axis, double lo, double inv, int nbins,
                   uint64_t *hist, void *stream) {
    if ((!X && n > 0) || !hist || n < 0 || d < 1 || d > 4 || axis < 0 || axis >= d || nbins < 1 ||
        nbins > HIST_BINS_MAX)
        return pcm_fail(PCM_E_ARG, "pcm_shard_hist: bad argument");
    hipStream_t s = (hipStream_t)stream;
    if (hipError_t e = hipMemsetAsync(hist, 0, (size_t)nbins * 8, s))
        return pcm_fail(PCM_E_HIP, std::string("pcm_shard_hist: ") + hipGetErrorString(e));
    if (n == 0) return 0;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1)
        ncu = 256;
    const int g = std::min(blocks(n, TPB), 2 * ncu);
    if (dtype == PCM_F32)
        k_shard_hist<float><<<g, TPB, 0, s>>>((const float *)X, n, d, axis, lo, inv, nbins,
                                              (unsigned long long *)hist);
    else if (dtype == PCM_F16)
        k_shard_hist<__half><<<g, TPB, 0, s>>>((const __half *)X, n, d, axis, lo, inv, nbins,
                                               (unsigned long long *)hist);
    else
        return pcm_fail(PCM_E_ARG, "pcm_shard_hist: dtype must be PCM_F32 or PCM_F16");
    if (hipError_t e = hipGetLastError()) return pcm_fail(PCM_E_HIP, std::string("k_shard_hist: ") + hipGetErrorString(e));
    return 0;
}

int pcm_shard_partition_workspace(int64_t n, int P, size_t *bytes) {
    if (!bytes || n < 0 || P < 1 || P > PCM_SHARD_MAXP) return pcm_fail(PCM_E_ARG, "pcm_shard_partition_workspace: bad argument");
    const size_t nblk = (size_t)blocks(n, CHUNK), m = nblk * P;
    *bytes = 2 * align256(m * 4) + align256((size_t)P * 8) + align256(scan_bytes(m));
    return 0;
}

int pcm_shard_partition(const void *X, int dtype, int64_t n, int d, int axis, double lo, double inv, int nbins,
                        const uint8_t *owner, int P, int64_t gidx0, void *X_out, uint32_t *rows_out, int64_t *counts,
                        void *workspace, size_t workspace_bytes, void *stream) {
    if ((!X && n > 0) || !owner || !counts || d < 1 || d > 4 || axis < 0 || axis >= d || nbins < 1 || P < 1 ||
        P > PCM_SHARD_MAXP || n < 0 || (n > 0 && (!X_out || !rows_out)) || gidx0 < 0 ||
        gidx0 + n > (int64_t)0xffffffffLL)
        return pcm_fail(PCM_E_ARG, "pcm_shard_partition: bad argument");
    if (dtype != PCM_F32 && dtype != PCM_F16) return pcm_fail(PCM_E_ARG, "pcm_shard_partition: dtype must be PCM_F32 or PCM_F16");
    for (int p = 0; p < P; ++p) counts[p] = 0;
    if (n == 0) return 0;
    size_t need = 0;
    if (int rc = pcm_shard_partition_workspace(n, P, &need)) return rc;
    if (!workspace || workspace_bytes < need) return pcm_fail(PCM_E_ARG, "pcm_shard_partition: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const int nblk = blocks(n, CHUNK);
    const size_t m = (size_t)nblk * P;
    char *w = (char *)workspace;
    uint32_t *cnt = (uint32_t *)w, *off = (uint32_t *)(w + align256(m * 4));
    long long *tot = (long long *)(w + 2 * align256(m * 4));
    void *tmp = w + 2 * align256(m * 4) + align256((size_t)P * 8);
    size_t tb = scan_bytes(m);
    auto launch = [&](auto T) -> int {
        using TT = decltype(T);
        k_shard_count<TT><<<nblk, TPB, 0, s>>>((const TT *)X, n, d, axis, lo, inv, nbins, owner, P, cnt);
        if (hipError_t e = hipGetLastError()) return pcm_fail(PCM_E_HIP, std::string("k_shard_count: ") + hipGetErrorString(e));
        if (hipError_t e = rocprim::exclusive_scan(tmp, tb, cnt, off, 0u, m, rocprim::plus<uint32_t>(), s))
            return pcm_fail(PCM_E_HIP, std::string("pcm_shard_partition scan: ") + hipGetErrorString(e));
        k_shard_totals<<<1, 64, 0, s>>>(off, cnt, nblk, P, tot);
        k_shard_scatter<TT><<<nblk, TPB, 0, s>>>((const TT *)X, n, d, axis, lo, inv, nbins, owner, P, off, gidx0,
                                                 (TT *)X_out, rows_out);
        if (hipError_t e = hipGetLastError()) return pcm_fail(PCM_E_HIP, std::string("k_shard_scatter: ") + hipGetErrorString(e));
        return 0;
    };
    int rc = dtype == PCM_F16 ? launch(__half{}) : launch(float{});
    if (rc) return rc;
    if (hipError_t e = hipMemcpyAsync(counts, tot, (size_t)P * 8, hipMemcpyDeviceToHost, s))
        return pcm_fail(PCM_E_HIP, std::string("pcm_shard_partition counts: ") + hipGetErrorString(e));
    if (hipError_t e = hipStreamSynchronize(s))
        return pcm_fail(PCM_E_HIP, std::string("pcm_shard_partition: ") + hipGetErrorString(e));
    return 0;
}

int pcm_shard_scatter_labels(const int32_t *labels, const uint32_t *rows, int64_t n, int64_t gidx0, int32_t *out,
                             void *stream) {
    if ((n > 0 && (!labels || !rows || !out)) || n < 0) return pcm_fail(PCM_E_ARG, "pcm_shard_scatter_labels: bad argument");
    if (n == 0) return 0;
    k_shard_labels<<<blocks(n, TPB), TPB, 0, (hipStream_t)stream>>>(labels, rows, n, gidx0, out);
    if (hipError_t e = hipGetLastError()) return pcm_fail(PCM_E_HIP, std::string("k_shard_labels: ") + hipGetErrorString(e));
    return 0;
}

}  // extern "C"
