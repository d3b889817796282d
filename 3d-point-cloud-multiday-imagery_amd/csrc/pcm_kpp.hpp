// pcm_kpp.hpp — k-means++ seeding on gfx950.
//
// Restates scikit-learn's _kmeans_plusplus (sklearn/cluster/_kmeans.py:174-272,
// the KMeans default init, :1012-1019) with the canonical arithmetic of
// oracle/kpp_ref.py: float32 direct-form distances, integer point weights
// w = trunc(ldexp(double(d), s)), exact integer potentials and cumulative sums,
// targets floor(u * pot) computed exactly from u's 53-bit mantissa.
//
// Per centre (one step), three stream-ordered launches:
//   k_kpp_pass    one pass over X: closest := min(closest, d(x, previous best));
//                 per block, for each of the L candidates, the sum of the
//                 weights of min(closest, d(x, cand)) -> bsum[block][l]
//   k_kpp_select  one block: potentials, first argmin (the new centre); for the
//                 next step's L targets, the block whose prefix crosses each
//   k_kpp_locate  one block per target: exact index inside its block (scan)
#pragma once
#include "pcm_kernels.hpp"

namespace pcm {

constexpr int KPP_LMAX = 16;
constexpr int KPP_BS = 8192;     // points per pass block (256 threads x 32)

struct KppState {
    float4 best;                  // centre chosen at the previous step
    float4 cand[KPP_LMAX];        // this step's candidates
    long long cand_idx[KPP_LMAX];
    long long loc_block[KPP_LMAX];
    unsigned long long resid[KPP_LMAX];
    unsigned long long pot;
    int Lc, has_best, first, pad_;
};

__device__ __forceinline__ unsigned long long kpp_w(float d, int s) {
    return (unsigned long long)__builtin_ldexp((double)d, s);   // d >= 0: truncation
}

template <int D>
__device__ __forceinline__ float4 row4(const float *X, long long i) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < D; ++a) v[a] = X[i * D + a];
    return make_float4(v[0], v[1], v[2], v[3]);
}

template <int D>
__device__ __forceinline__ float kdist(const float *X, long long i, const float4 &c) {
    float x[D];
#pragma unroll
    for (int a = 0; a < D; ++a) x[a] = X[i * D + a];
    return dist_canon<D>(x, c);
}

template <int D>
__global__ __launch_bounds__(256) void k_kpp_pass(const float *__restrict__ X, long long n, float *__restrict__ closest,
                                                  const KppState *__restrict__ st, int s,
                                                  unsigned long long *__restrict__ bsum) {
    const int tid = threadIdx.x;
    const long long b0 = (long long)blockIdx.x * KPP_BS;
    const int Lc = st->Lc;
    const bool first = st->first != 0, has_best = st->has_best != 0;
    const float4 best = st->best;
    float4 cand[KPP_LMAX];
#pragma unroll
    for (int l = 0; l < KPP_LMAX; ++l) cand[l] = st->cand[l];
    unsigned long long acc[KPP_LMAX];
#pragma unroll
    for (int l = 0; l < KPP_LMAX; ++l) acc[l] = 0ull;
    for (int e = tid; e < KPP_BS; e += 256) {
        const long long i = b0 + e;
        if (i >= n) break;
        float x[D];
#pragma unroll
        for (int a = 0; a < D; ++a) x[a] = X[i * D + a];
        float cl = first ? __builtin_inff() : closest[i];
        if (has_best) cl = fminf(cl, dist_canon<D>(x, best));
        closest[i] = cl;
#pragma unroll
        for (int l = 0; l < KPP_LMAX; ++l)
            if (l < Lc) acc[l] += kpp_w(fminf(cl, dist_canon<D>(x, cand[l])), s);
    }
    __shared__ unsigned long long red[KPP_LMAX][4];
    const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
    for (int l = 0; l < KPP_LMAX; ++l) {
        if (l >= Lc) break;
        unsigned long long v = acc[l];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) red[l][wv] = v;
    }
    __syncthreads();
    if (tid < Lc) bsum[(size_t)blockIdx.x * KPP_LMAX + tid] = red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3];
}

// One block of 1024 threads.  umant: the next step's L uniforms as exact
// 53-bit mantissas (nullptr after the last centre).
__global__ __launch_bounds__(1024) void k_kpp_select(const unsigned long long *__restrict__ bsum, long long nblk,
                                                     KppState *__restrict__ st, long long *__restrict__ indices,
                                                     int c, const unsigned long long *__restrict__ umant, int Lnext) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int Lc = st->Lc;
    __shared__ unsigned long long wp[16][KPP_LMAX];
    __shared__ unsigned long long tsum[1024];
    __shared__ int s_best;
    // potentials (exact integer sums: any order)
    unsigned long long p[KPP_LMAX];
#pragma unroll
    for (int l = 0; l < KPP_LMAX; ++l) p[l] = 0ull;
    for (long long b = tid; b < nblk; b += 1024)
#pragma unroll
        for (int l = 0; l < KPP_LMAX; ++l)
            if (l < Lc) p[l] += bsum[(size_t)b * KPP_LMAX + l];
#pragma unroll
    for (int l = 0; l < KPP_LMAX; ++l) {
        unsigned long long v = p[l];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) wp[wv][l] = v;
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long bp = 0ull;
        int bl = -1;
        for (int l = 0; l < Lc; ++l) {
            unsigned long long v = 0ull;
            for (int w = 0; w < 16; ++w) v += wp[w][l];
            if (bl < 0 || v < bp) { bp = v; bl = l; }   // first argmin (np.argmin)
        }
        s_best = bl;
        st->pot = bp;
        st->best = st->cand[bl];
        st->has_best = 1;
        st->first = 0;
        indices[c] = st->cand_idx[bl];
    }
    __syncthreads();
    if (!umant) return;
    const int bl = s_best;
    const unsigned long long pot = st->pot;
    // thread tid owns the contiguous block range [b0, b1)
    const long long per = (nblk + 1023) / 1024;
    const long long b0 = tid * per < nblk ? tid * per : nblk, b1 = b0 + per < nblk ? b0 + per : nblk;
    unsigned long long loc = 0ull;
    for (long long b = b0; b < b1; ++b) loc += bsum[(size_t)b * KPP_LMAX + bl];
    tsum[tid] = loc;
    __syncthreads();
    // inclusive scan of the thread sums (Hillis-Steele in LDS)
    for (int o = 1; o < 1024; o <<= 1) {
        const unsigned long long v = tid >= o ? tsum[tid - o] : 0ull;
        __syncthreads();
        tsum[tid] += v;
        __syncthreads();
    }
    unsigned long long run = tsum[tid] - loc;   // exclusive prefix of this thread's range
    for (int t = 0; t < Lnext; ++t) {
        const unsigned long long m = umant[t];
        const unsigned long long lo = m * pot, hi = __umul64hi(m, pot);
        const unsigned long long tg = (hi << 11) | (lo >> 53);   // floor(u * pot)
        // first block b with inclusive prefix >= tg (np.searchsorted side='left')
        unsigned long long r = run;
        for (long long b = b0; b < b1; ++b) {
            const unsigned long long v = bsum[(size_t)b * KPP_LMAX + bl];
            if (r + v >= tg && (b == 0 || r < tg)) {
                st->loc_block[t] = b;
                st->resid[t] = tg - r;
            }
            r += v;
        }
        if (tid == 1023 && r < tg) {   // past the end: np.searchsorted -> n, clipped to n-1
            st->loc_block[t] = -1;
            st->resid[t] = 0ull;
        }
    }
    if (tid == 0) st->Lc = Lnext;
}

template <int D>
__global__ void k_kpp_init(const float *__restrict__ X, long long first, KppState *__restrict__ st) {
    if (threadIdx.x != 0) return;
    st->cand[0] = row4<D>(X, first);
    st->cand_idx[0] = first;
    st->Lc = 1;
    st->first = 1;
    st->has_best = 0;
    st->pot = 0ull;
}

// One block (1024 threads) per target: the exact index inside its block.
template <int D>
__global__ __launch_bounds__(1024) void k_kpp_locate(const float *__restrict__ X, long long n,
                                                     const float *__restrict__ closest, KppState *__restrict__ st,
                                                     int s) {
    const int t = blockIdx.x, tid = threadIdx.x;
    const long long b = st->loc_block[t];
    if (b < 0) {
        if (tid == 0) {
            st->cand_idx[t] = n - 1;
            st->cand[t] = row4<D>(X, n - 1);
        }
        return;
    }
    const unsigned long long rs = st->resid[t];
    const float4 best = st->best;
    constexpr int PER = KPP_BS / 1024;   // 8 consecutive points per thread
    unsigned long long w[PER], loc = 0ull;
#pragma unroll
    for (int e = 0; e < PER; ++e) {
        const long long i = b * KPP_BS + (long long)tid * PER + e;
        w[e] = i < n ? kpp_w(fminf(closest[i], kdist<D>(X, i, best)), s) : 0ull;
        loc += w[e];
    }
    __shared__ unsigned long long tsum[1024];
    __shared__ long long found;
    if (tid == 0) found = 0x7fffffffffffffffll;
    tsum[tid] = loc;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const unsigned long long v = tid >= o ? tsum[tid - o] : 0ull;
        __syncthreads();
        tsum[tid] += v;
        __syncthreads();
    }
    unsigned long long r = tsum[tid] - loc;
#pragma unroll
    for (int e = 0; e < PER; ++e) {
        const long long i = b * KPP_BS + (long long)tid * PER + e;
        if (i < n && r + w[e] >= rs) atomicMin(&found, i);   // first inclusive prefix >= rs
        r += w[e];
    }
    __syncthreads();
    if (tid == 0) {
        long long i = found;
        if (i >= n) i = n - 1;
        st->cand_idx[t] = i;
        st->cand[t] = row4<D>(X, i);
    }
}

}  // namespace pcm
