// pcm_sort.hpp — the layout's cell sort: an LSD radix sort (digits of <= 8
// bits) that carries the point records {coordinates, caller row} through every
// pass, so the cloud lands in cell order without a random row gather.  Keys
// come from sort_key_f (the same fp64 binning as everywhere else).
//
// Per pass, over chunks of RS_TPB * IPT consecutive items:
//   k_rs_count    per-chunk digit histogram -> hist[chunk][digit]
//   k_rs_colscan, k_rs_segscan   every (chunk, digit)'s output base: column
//                 scans over segments of chunks, then segment and digit bases
//   k_rs_scatter  stable rank of each item inside its chunk (per wave: digit
//                 peer masks by ballots, running per-digit counters in LDS;
//                 across waves: digit-wise prefix), the chunk staged in LDS in
//                 digit order, then written out run by run (consecutive lanes
//                 write consecutive addresses)
// The first pass reads the caller's rows (row index = item index); the last
// writes the AoSoA-4 `xs` and `perm` (cell starts then come from a binary
// search over xs, k_cell_starts_xs: no key array at all).  Stable passes from
// the lowest digit up give the (key, row) order of the previous pairs sort.
// Reads/writes per point at config 3 (fp32 D = 3, 15-bit keys, 2 passes):
// 12 (count) + 12 + 16 (scatter) + 16 (count) + 16 + 16 (scatter) = 88 B.
#pragma once
#include "pcm_kernels.hpp"

namespace pcm {

#ifndef PCM_RS_TPB
#define PCM_RS_TPB 512   // 256: scatters 885 / 975 us, 512: 652 / 799 us at config 3 (profiles/rd6_sort_tpb512.txt)
#endif
constexpr int RS_TPB = PCM_RS_TPB;   // threads per scatter block (256 or 512; chunks stay RsCfg::CH items)
constexpr int RS_NWV = RS_TPB / 64;
constexpr int RS_DIG = 256;          // digit values per pass (<= 8 bits)

template <typename T, int D> struct RsCfg {
    // items per thread: the LDS staging of a chunk (record + digit per item) <= 68 KB.  Longer
    // chunks give longer output runs per digit: 4096 items measured 858 / 1185 us for the two
    // config-3 scatters, 3072 (with a 4-B key staged and written per item) 1376 / 2084 us,
    // 2048 slower overall (layout 5.37 vs 4.95 ms)
    static constexpr int CH = sizeof(PRec<T, D>) <= 16 ? 4096 : 3072;   // items per chunk
    static constexpr int IPT = CH / RS_TPB;                               // (16 / 12 at 256 threads)
};

// Item i of a pass: the first pass reads the caller's row i, later passes the
// record the previous pass wrote.  Keys are recomputed from the coordinates in
// every pass (fp64 binning, ~36 flops per point): writing them beside the
// records costs more, since a chunk's 4-B keys land in short runs (partial
// lines; measured above).
template <typename T, int D, bool FROM_X>
__device__ __forceinline__ void rs_load(const T *__restrict__ X, const PRec<T, D> *__restrict__ rin, long long i,
                                        PRec<T, D> &r) {
    if constexpr (FROM_X) {
#pragma unroll
        for (int a = 0; a < D; ++a) r.c[a] = X[i * D + a];
        r.row = (uint32_t)i;
    } else {
        r = rin[i];
    }
}

template <typename T, int D>
__device__ __forceinline__ uint32_t rs_key(const PRec<T, D> &r, const Grid &g, int with_sub, int zlev) {
    float x[D];
#pragma unroll
    for (int a = 0; a < D; ++a) x[a] = to_f<T>(r.c[a]);
    return sort_key_f<D>(x, g, with_sub, zlev);
}

// Per-chunk digit histogram.  PCM_RS_CTPB: threads per count block (the
// chunk stays RsCfg::CH items; A/B of the count's occupancy)
#ifndef PCM_RS_CTPB
#define PCM_RS_CTPB 512   // 256: 383 -> 512: 325 us for the record pass at config 3 (profiles/rd6_sort_count_vec.txt)
#endif
constexpr int RS_CTPB = PCM_RS_CTPB;
template <typename T, int D, bool FROM_X>
__global__ __launch_bounds__(RS_CTPB) void k_rs_count(const T *__restrict__ X, const PRec<T, D> *__restrict__ rin,
                                                     long long n, Grid g, int with_sub, int zlev, int shift, int width,
                                                     uint32_t *__restrict__ hist, int vec) {
    constexpr int CH = RsCfg<T, D>::CH, CNWV = RS_CTPB / 64, IPT = CH / RS_CTPB;
    static_assert(CH % RS_CTPB == 0 && RS_CTPB >= RS_DIG, "count block geometry");
    __shared__ uint32_t h[CNWV][RS_DIG];
    const int tid = threadIdx.x, wv = tid >> 6;
    for (int k = tid; k < CNWV * RS_DIG; k += RS_CTPB) (&h[0][0])[k] = 0u;
    __syncthreads();
    const long long base = (long long)blockIdx.x * CH;
    const uint32_t mask = (1u << width) - 1u;
    if constexpr (FROM_X && sizeof(T) == 4 && D == 3 && IPT % 4 == 0) {
        if (vec) {   // (X 16-B aligned) 4 consecutive rows per thread and group: three 16-B loads instead of 12 4-B ones
            constexpr int G = IPT / 4;
            float4 q[G][3];
#pragma unroll
            for (int u = 0; u < G; ++u) {
                const long long r0 = base + 4LL * (u * RS_CTPB + tid);
                if (r0 + 3 < n) {
                    const float4 *p = reinterpret_cast<const float4 *>(X + r0 * 3);
                    q[u][0] = p[0]; q[u][1] = p[1]; q[u][2] = p[2];
                }
            }
#pragma unroll
            for (int u = 0; u < G; ++u) {
                const long long r0 = base + 4LL * (u * RS_CTPB + tid);
                if (r0 >= n) continue;
                float f[12];
                if (r0 + 3 < n) {
                    f[0] = q[u][0].x; f[1] = q[u][0].y; f[2] = q[u][0].z; f[3] = q[u][0].w;
                    f[4] = q[u][1].x; f[5] = q[u][1].y; f[6] = q[u][1].z; f[7] = q[u][1].w;
                    f[8] = q[u][2].x; f[9] = q[u][2].y; f[10] = q[u][2].z; f[11] = q[u][2].w;
                } else {
                    for (int k = 0; k < 12; ++k) f[k] = r0 * 3 + k < n * 3 ? (float)X[r0 * 3 + k] : 0.f;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (r0 + k >= n) break;
                    const float x[3] = {f[3 * k], f[3 * k + 1], f[3 * k + 2]};
                    atomicAdd(&h[wv][(sort_key_f<3>(x, g, with_sub, zlev) >> shift) & mask], 1u);
                }
            }
            __syncthreads();
            if (tid < RS_DIG) {
                uint32_t t = 0u;
#pragma unroll
                for (int w = 0; w < CNWV; ++w) t += h[w][tid];
                hist[(long long)blockIdx.x * RS_DIG + tid] = t;
            }
            return;
        }
    }
    PRec<T, D> r[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const long long i = base + (long long)j * RS_CTPB + tid;
        if (i < n) rs_load<T, D, FROM_X>(X, rin, i, r[j]);
    }
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const long long i = base + (long long)j * RS_CTPB + tid;
        if (i < n) atomicAdd(&h[wv][(rs_key<T, D>(r[j], g, with_sub, zlev) >> shift) & mask], 1u);
    }
    __syncthreads();
    if (tid < RS_DIG) {
        uint32_t t = 0u;
#pragma unroll
        for (int w = 0; w < CNWV; ++w) t += h[w][tid];
        hist[(long long)blockIdx.x * RS_DIG + tid] = t;   // chunk-major: one coalesced 1-KB row per chunk
    }
}

// Output bases, chunk-major like hist: goff[chunk][d] (exclusive over the
// chunks of its segment of RS_SEG chunks) + segb[segment][d] (all earlier
// chunks and all smaller digits) = where chunk's first item of digit d goes.
constexpr int RS_SEG = 256;

__global__ __launch_bounds__(RS_DIG) void k_rs_colscan(const uint32_t *__restrict__ hist, long long nblk,
                                                       uint32_t *__restrict__ goff, uint32_t *__restrict__ segt) {
    const int t = threadIdx.x;
    const long long r0 = (long long)blockIdx.x * RS_SEG, r1 = min(r0 + RS_SEG, nblk);
    uint32_t acc = 0u;
    long long r = r0;
    for (; r + 8 <= r1; r += 8) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = hist[(r + u) * RS_DIG + t];
#pragma unroll
        for (int u = 0; u < 8; ++u) { goff[(r + u) * RS_DIG + t] = acc; acc += v[u]; }
    }
    for (; r < r1; ++r) {
        const uint32_t v = hist[r * RS_DIG + t];
        goff[r * RS_DIG + t] = acc;
        acc += v;
    }
    segt[(long long)blockIdx.x * RS_DIG + t] = acc;
}

// One block: segment bases per digit, then every digit's global base (an
// exclusive scan over the digits of their totals), folded into segb.
__global__ __launch_bounds__(RS_DIG) void k_rs_segscan(uint32_t *__restrict__ segb, long long nseg) {
    __shared__ uint32_t wtot[RS_DIG / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint32_t acc = 0u;
    long long q = 0;
    for (; q + 8 <= nseg; q += 8) {   // 8 loads in flight per step
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = segb[(q + u) * RS_DIG + t];
#pragma unroll
        for (int u = 0; u < 8; ++u) { segb[(q + u) * RS_DIG + t] = acc; acc += v[u]; }
    }
    for (; q < nseg; ++q) {
        const uint32_t v = segb[q * RS_DIG + t];
        segb[q * RS_DIG + t] = acc;
        acc += v;
    }
    uint32_t v = acc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)v, o);
        if (lane >= o) v += u;
    }
    if (lane == 63) wtot[wv] = v;
    __syncthreads();
    uint32_t pre = 0u;
    for (int w = 0; w < wv; ++w) pre += wtot[w];
    const uint32_t dbase = pre + v - acc;
    for (long long q2 = 0; q2 < nseg; ++q2) segb[q2 * RS_DIG + t] += dbase;
}

template <typename T, int D, bool FROM_X, bool TO_XS>
__global__ __launch_bounds__(RS_TPB) void k_rs_scatter(const T *__restrict__ X, const PRec<T, D> *__restrict__ rin,
                                                       long long n, Grid g, int with_sub, int zlev, int shift,
                                                       int width,
                                                       const uint32_t *__restrict__ goff,
                                                       const uint32_t *__restrict__ segb,
                                                       PRec<T, D> *__restrict__ rout, T *__restrict__ xs,
                                                       uint32_t *__restrict__ perm, uint32_t *__restrict__ dmap,
                                                       int xcd) {
    constexpr int IPT = RsCfg<T, D>::IPT, CH = RsCfg<T, D>::CH, PW = CH / RS_NWV;
    __shared__ PRec<T, D> stage[CH];
    __shared__ uint8_t sdig[CH];
    __shared__ uint32_t wc[RS_NWV][RS_DIG];
    __shared__ uint32_t dstart[RS_DIG];
    __shared__ long long gdelta[RS_DIG];
    __shared__ uint32_t wtot[4];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int k = tid; k < RS_NWV * RS_DIG; k += RS_TPB) (&wc[0][0])[k] = 0u;
    // chunk through xcd_block: a chunk's digit runs end in lines shared with the
    // next chunk's runs of the same digits, and those partial lines merge in one
    // L2 when both chunks run on the same XCD
    const unsigned chunk = xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const long long base = (long long)chunk * CH;
    const uint32_t mask = (1u << width) - 1u;
    const unsigned long long lt = (1ull << lane) - 1ull;
    // wave wv owns the PW consecutive items [base + wv * PW, ...), 64 per round
    PRec<T, D> r[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const long long i = base + wv * PW + j * 64 + lane;
        if (i < n) rs_load<T, D, FROM_X>(X, rin, i, r[j]);
    }
    __syncthreads();
    uint32_t dk[IPT];   // digit | (rank in the wave's run of that digit) << 8
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const long long i = base + wv * PW + j * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = valid ? (rs_key<T, D>(r[j], g, with_sub, zlev) >> shift) & mask : 0u;
        unsigned long long peers = __ballot(valid);
        for (int b = 0; b < width; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t rk = (uint32_t)__popcll(peers & lt);
        const uint32_t prior = wc[wv][d];
        if (valid && rk == 0u) wc[wv][d] = prior + (uint32_t)__popcll(peers);
        dk[j] = d | ((prior + rk) << 8);
    }
    __syncthreads();
    {
        // digit tid (< RS_DIG): offsets of the waves' runs, the chunk's digit starts, output bases
        uint32_t tot = 0u, v = 0u;
        if (tid < RS_DIG) {
#pragma unroll
            for (int w = 0; w < RS_NWV; ++w) {
                const uint32_t cw = wc[w][tid];
                wc[w][tid] = tot;
                tot += cw;
            }
            v = tot;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = (uint32_t)__shfl_up((int)v, o);
                if (lane >= o) v += u;
            }
            if (lane == 63) wtot[wv] = v;
        }
        __syncthreads();
        if (tid < RS_DIG) {
            uint32_t pre = 0u;
            for (int w = 0; w < wv; ++w) pre += wtot[w];
            const uint32_t ex = pre + v - tot;
            dstart[tid] = ex;
            gdelta[tid] = (long long)goff[(long long)chunk * RS_DIG + tid] +
                          (long long)segb[(long long)(chunk / RS_SEG) * RS_DIG + tid] - (long long)ex;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const long long i = base + wv * PW + j * 64 + lane;
        if (i < n) {
            const uint32_t d = dk[j] & 0xffu;
            const uint32_t p = dstart[d] + wc[wv][d] + (dk[j] >> 8);
            stage[p] = r[j];
            sdig[p] = (uint8_t)d;
            if (dmap) dmap[i] = (uint32_t)(p + gdelta[d]);   // this pass's input position -> output position
        }
    }
    __syncthreads();
    const int cnt = (int)min((long long)CH, n - base);
    for (int p = tid; p < cnt; p += RS_TPB) {
        const PRec<T, D> rec = stage[p];
        const long long dst = p + gdelta[sdig[p]];
        if constexpr (TO_XS) {
            perm[dst] = rec.row;
#pragma unroll
            for (int a = 0; a < D; ++a) xs[xs_index<D>(dst, a)] = rec.c[a];
        } else {
            rout[dst] = rec;
        }
    }
}

// start[c] = first sorted position whose key (recomputed from xs) >> shift is
// >= c, for c in [0, ncells]: one thread per cell, ~log2(n) probes.
template <typename T, int D>
__global__ __launch_bounds__(256) void k_cell_starts_xs(const T *__restrict__ xs, long long n, Grid g, int with_sub,
                                                        int zlev, long long ncells, uint32_t *__restrict__ start,
                                                        int shift) {
    const long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (c > ncells) return;
    long long lo = 0, hi = n;
    while (lo < hi) {
        const long long mid = (lo + hi) >> 1;
        float x[D];
#pragma unroll
        for (int a = 0; a < D; ++a) x[a] = to_f<T>(xs[xs_index<D>(mid, a)]);
        if ((long long)(sort_key_f<D>(x, g, with_sub, zlev) >> shift) < c) lo = mid + 1; else hi = mid;
    }
    start[c] = (uint32_t)lo;
}

// Labels back to the caller's row order through the sort's per-pass position
// maps (dmap_q: input position of pass q -> its output position), one gather
// per pass from the last to the first: a pass's outputs are runs of its input
// order, so the gathers read runs instead of single random words.
// 4 consecutive outputs per thread: the map as one 16-B load
// (VM: the map is 16-B aligned) and the outputs as one 8-B / 16-B store (VO:
// the destination is aligned), the 4 run-wise source reads in flight together
// (one output per thread moved ~1.9 TB/s: two dependent 2-B accesses a lane).
template <typename LT, typename OT, bool VM, bool VO>
__global__ __launch_bounds__(256) void k_lab_gather4(const uint32_t *__restrict__ dmap, const LT *__restrict__ src,
                                                     long long n, OT *__restrict__ dst, int xcd) {
    // xcd_block: the source runs of neighbouring sort chunks are adjacent and
    // share lines, which then come into one L2
    const unsigned b = xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const long long i4 = (b * (long long)blockDim.x + threadIdx.x) * 4;
    if (i4 >= n) return;
    if (i4 + 4 > n) {
        for (long long i = i4; i < n; ++i) dst[i] = (OT)src[dmap[i]];
        return;
    }
    uint32_t m[4];
    if constexpr (VM) {
        const uint4 v = *reinterpret_cast<const uint4 *>(dmap + i4);
        m[0] = v.x; m[1] = v.y; m[2] = v.z; m[3] = v.w;
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) m[k] = dmap[i4 + k];
    }
    OT o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (OT)src[m[k]];
    if constexpr (VO && sizeof(OT) == 2) {
        uint2 w;
        w.x = (uint32_t)(uint16_t)o[0] | ((uint32_t)(uint16_t)o[1] << 16);
        w.y = (uint32_t)(uint16_t)o[2] | ((uint32_t)(uint16_t)o[3] << 16);
        *reinterpret_cast<uint2 *>(dst + i4) = w;
    } else if constexpr (VO && sizeof(OT) == 4) {
        *reinterpret_cast<int4 *>(dst + i4) = make_int4((int)o[0], (int)o[1], (int)o[2], (int)o[3]);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[i4 + k] = o[k];
    }
}

// xs padding [n, npad): zeros
template <typename T, int D>
__global__ void k_xs_pad(long long n, long long npad, T *__restrict__ xs) {
    const long long i = n + threadIdx.x;
    if (i < npad)
#pragma unroll
        for (int a = 0; a < D; ++a) xs[xs_index<D>(i, a)] = (T)0.0f;
}

}  // namespace pcm
