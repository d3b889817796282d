// pcm_dense.hip — generic-D Lloyd K-means + k-means++ on gfx950 for the
// reference's only executed K-means call site:
// members/jasraj/land_use_classification/core.py:227-228,
// KMeans(n_clusters=5, random_state=42, n_init=10).fit_predict(StandardScaler(X))
// on ~1500 x 20 float64 superpixel features.
//
// The point-cloud engine (pcm_engine.hip) prunes candidates on a D <= 4 grid;
// feature vectors (D up to PCM_DENSE_DMAX) have no useful grid, so this path is
// brute force over all K (centres staged in LDS) and computes in the INPUT
// precision (float64 stays float64, like scikit-learn).  Canonical arithmetic
// (oracle/dense_ref.py):
//  * distance: sequential sum over features of (x_a - c_a)^2, every op rounded
//    in T (no FMA); argmin strict '<' in ascending centroid index
//    (_k_means_lloyd.pyx:168-213);
//  * sums: exact int64 fixed point trunc(ldexp(x_a, q_a)), q_a = 62 - e_a -
//    bits(n) with max|x_a| < 2^e_a (order-independent; the sums cannot overflow);
//  * centre: (T)((double(S) * 2^-q) * (1.0 / count))  (_average_centers'
//    alpha = 1 / weight, _k_means_common.pyx:274-295);
//  * empty clusters: the farthest points (distance desc, row asc) move in,
//    the list of empty clusters fixed first (_k_means_common.pyx:167-211);
//  * shift: per centre sqrt of _euclidean_dense_dense's 4-grouped sum, total
//    = sequential sum of squares (_k_means_common.pyx:17-43, 298-311,
//    _kmeans.py:724-732); convergence: labels unchanged or shift <= tol;
//  * inertia: exact limbs of trunc(d * 2^s) (as the point-cloud engine).
// Everything runs on the device; per iteration: k_dense_assign (grid) +
// k_dense_update (one block), gated on the control block so the host can
// enqueue iterations in chunks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "pcm_common.hpp"
#include "pcm_kmeans.h"

namespace pcm {

struct DenseCtrl {
    uint32_t done, iter, max_iter, relocs;
    double tol;
    unsigned long long changed;       // labels changed by the last assign (accumulated, read by update)
    unsigned long long last_changed;
    double last_shift;
    unsigned long long inert[4];      // inertia limbs (final E-step)
};

template <typename T> __device__ __forceinline__ T dense_dist(const T *__restrict__ x, const T *__restrict__ c, int d) {
    T diff = x[0] - c[0];
    T acc = diff * diff;
    for (int a = 1; a < d; ++a) {
        diff = x[a] - c[a];
        const T sq = diff * diff;
        acc = acc + sq;
    }
    return acc;
}

__device__ __forceinline__ long long dense_fixed(double x, int q) { return (long long)__builtin_ldexp(x, q); }

// E-step (+ statistics when `stats`, + inertia limbs when `inert`); labels
// hold the previous labels on entry (-1 before the first iteration).
template <typename T>
__global__ __launch_bounds__(256) void k_dense_assign(const T *__restrict__ X, long long n, int d,
                                                      const T *__restrict__ C, int k, const int *__restrict__ q,
                                                      int32_t *__restrict__ labels, T *__restrict__ dist,
                                                      unsigned long long *__restrict__ stats, int lds_stats,
                                                      DenseCtrl *__restrict__ ctrl, int gate,
                                                      unsigned long long *__restrict__ inert, int iscale, int lds_c) {
    if (gate && (ctrl->done != 0u)) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
    // centres staged in LDS when they fit (k * d * sizeof(T) <= 64 KB), else read
    // from global memory (L2/L1-resident: every thread scans them in the same order)
    const size_t cb = lds_c ? (((size_t)k * d * sizeof(T) + 15) / 16) * 16 : 0;
    T *scl = (T *)sm;
    const T *sc = lds_c ? scl : C;                                     // [k * d]
    unsigned long long *ls = (unsigned long long *)(sm + cb);         // [k * (d + 1)]
    const int nstat = k * (d + 1);
    if (lds_c)
        for (int j = threadIdx.x; j < k * d; j += blockDim.x) scl[j] = C[j];
    if (stats && lds_stats)
        for (int j = threadIdx.x; j < nstat; j += blockDim.x) ls[j] = 0ull;
    __syncthreads();
    unsigned long long changed = 0ull, ilo = 0ull, ihi = 0ull;
    unsigned iovf = 0u;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const T *x = X + i * d;
        T bd = dense_dist<T>(x, sc, d);
        int bj = 0;
        for (int j = 1; j < k; ++j) {
            const T dd = dense_dist<T>(x, sc + (size_t)j * d, d);
            if (dd < bd) { bd = dd; bj = j; }
        }
        if (labels[i] != bj) ++changed;
        labels[i] = bj;
        if (dist) dist[i] = bd;
        if (stats) {
            unsigned long long *p = (lds_stats ? ls : stats) + (size_t)bj * (d + 1);
            for (int a = 0; a < d; ++a) atomicAdd(p + a, (unsigned long long)dense_fixed((double)x[a], q[a]));
            atomicAdd(p + d, 1ull);
        }
        if (inert) {
            const double v = __builtin_ldexp((double)bd, iscale);
            unsigned long long w;
            if (v < 18446744073709551616.0) {
                w = (unsigned long long)v;
            } else {
                w = ~0ull;
                ++iovf;
            }
            ilo += w;
            ihi += (ilo < w) ? 1ull : 0ull;
        }
    }
    for (int o = 32; o > 0; o >>= 1) changed += __shfl_xor(changed, o);
    if ((threadIdx.x & 63) == 0 && changed) atomicAdd(&ctrl->changed, changed);
    if (inert) {
        unsigned long long l[4] = {ilo & 0xffffffffull, ilo >> 32, ihi, (unsigned long long)iovf};
        for (int t = 0; t < 4; ++t) {
            for (int o = 32; o > 0; o >>= 1) l[t] += __shfl_xor(l[t], o);
            if ((threadIdx.x & 63) == 0 && l[t]) atomicAdd(inert + t, l[t]);
        }
    }
    if (stats && lds_stats) {
        __syncthreads();
        for (int j = threadIdx.x; j < nstat; j += blockDim.x)
            if (ls[j]) atomicAdd(stats + j, ls[j]);
    }
}

// Centre update, relocation, shift, convergence (one block of 256 threads).
template <typename T>
__global__ __launch_bounds__(256) void k_dense_update(const T *__restrict__ X, long long n, int d, T *__restrict__ C,
                                                      int k, const int *__restrict__ q, const int32_t *__restrict__ labels,
                                                      const T *__restrict__ dist, unsigned long long *__restrict__ stats,
                                                      int *__restrict__ empty_idx, long long *__restrict__ picked,
                                                      unsigned long long *__restrict__ hist_changed,
                                                      double *__restrict__ hist_shift, DenseCtrl *__restrict__ ctrl) {
    if (ctrl->done != 0u) return;
    const int tid = threadIdx.x;
    __shared__ int s_nempty;
    __shared__ double s_bv[256];
    __shared__ long long s_bi[256];
    const unsigned long long changed = ctrl->changed;
    if (tid == 0) s_nempty = 0;
    __syncthreads();
    if (tid == 0)
        for (int j = 0; j < k; ++j)
            if (stats[(size_t)j * (d + 1) + d] == 0ull) empty_idx[s_nempty++] = j;
    __syncthreads();
    const int ne = s_nempty;
    if (ne > 0) {
        // farthest points from their centre, (distance desc, row asc); picked[] keeps the chosen rows
        int m = 0;
        for (; m < ne && m < (int)n; ++m) {
            double bv = -1.0;
            long long bi = 0x7fffffffffffffffll;
            for (long long i = tid; i < n; i += blockDim.x) {
                bool taken = false;
                for (int t = 0; t < m; ++t) taken |= (picked[t] == i);
                if (taken) continue;
                const double v = (double)dist[i];
                if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
            }
            s_bv[tid] = bv;
            s_bi[tid] = bi;
            __syncthreads();
            for (int st = 128; st > 0; st >>= 1) {
                if (tid < st) {
                    const double ov = s_bv[tid + st];
                    const long long oi = s_bi[tid + st];
                    if (ov > s_bv[tid] || (ov == s_bv[tid] && oi < s_bi[tid])) { s_bv[tid] = ov; s_bi[tid] = oi; }
                }
                __syncthreads();
            }
            if (tid == 0) picked[m] = s_bi[0];
            const double top = s_bv[0];
            __syncthreads();
            if (m == 0 && !(top > 0.0)) break;   // all points at their centres: nothing to move (pyx:189-192)
        }
        if (tid == 0 && m > 0) {
            for (int t = 0; t < m; ++t) {
                const int j = empty_idx[t];
                const long long p = picked[t];
                const int old = labels[p];
                unsigned long long *so = stats + (size_t)old * (d + 1), *sn = stats + (size_t)j * (d + 1);
                for (int a = 0; a < d; ++a) {
                    const unsigned long long u = (unsigned long long)dense_fixed((double)X[p * d + a], q[a]);
                    so[a] -= u;
                    sn[a] = u;
                }
                so[d] -= 1ull;
                sn[d] = 1ull;
            }
            ctrl->relocs += 1u;
        }
        __syncthreads();
    }
    // argmax of the counts (first) for clusters still empty
    if (tid == 0) {
        unsigned long long bmax = 0ull;
        int arg = 0;
        for (int j = 0; j < k; ++j) {
            const unsigned long long c = stats[(size_t)j * (d + 1) + d];
            if (c > bmax) { bmax = c; arg = j; }
        }
        s_bi[0] = arg;
        s_bv[0] = (double)bmax;
    }
    __syncthreads();
    const int arg = (int)s_bi[0];
    const bool any = s_bv[0] > 0.0;
    // new centres staged after the statistics: a still-empty cluster takes the
    // (averaged) centre of the first largest one, or keeps its own if all are empty
    T *stage = (T *)(stats + (size_t)k * (d + 1));
    for (int e = tid; e < k * d; e += blockDim.x) {
        const int j = e / d, a = e % d;
        const int src = (stats[(size_t)j * (d + 1) + d] > 0ull || !any) ? j : arg;
        const unsigned long long *row = stats + (size_t)src * (d + 1);
        const unsigned long long c = row[d];
        T cn = C[e];
        if (c > 0ull) {
            const double sm = (double)(long long)row[a] * __builtin_ldexp(1.0, -q[a]);
            cn = (T)(sm * (1.0 / (double)c));
        }
        stage[e] = cn;
    }
    __syncthreads();
    if (tid == 0) {
        // shift: per centre sqrt(_euclidean_dense_dense's 4-grouped sum), total = sequential sum of squares
        double shift_tot = 0.0;
        for (int j = 0; j < k; ++j) {
            double res = 0.0;
            int a0 = 0;
            for (; a0 + 4 <= d; a0 += 4) {
                double g = 0.0;
                for (int a = a0; a < a0 + 4; ++a) {
                    const double df = (double)stage[(size_t)j * d + a] - (double)C[(size_t)j * d + a];
                    const double sq = df * df;
                    g = (a == a0) ? sq : g + sq;
                }
                res = res + g;
            }
            for (int a = a0; a < d; ++a) {
                const double df = (double)stage[(size_t)j * d + a] - (double)C[(size_t)j * d + a];
                const double sq = df * df;
                res = res + sq;
            }
            const double r = sqrt(res);
            shift_tot = shift_tot + r * r;
        }
        s_bv[1] = shift_tot;
    }
    __syncthreads();
    for (int e = tid; e < k * d; e += blockDim.x) C[e] = stage[e];
    // zero the statistics for the next iteration; flags
    for (int e = tid; e < k * (d + 1); e += blockDim.x) stats[e] = 0ull;
    if (tid == 0) {
        const double sh = s_bv[1];
        const uint32_t it = ctrl->iter;
        if (it < ctrl->max_iter) {
            hist_changed[it] = changed;
            hist_shift[it] = sh;
        }
        ctrl->last_changed = changed;
        ctrl->last_shift = sh;
        ctrl->changed = 0ull;
        uint32_t done = 0;
        if (changed == 0ull) done = 1u;
        else if (sh <= ctrl->tol) done = 2u;
        if (!done && it + 1 >= ctrl->max_iter) done = 3u;
        ctrl->done = done;
        ctrl->iter = it + 1;
    }
}

// ------------------------------------------------------------------ k-means++
constexpr int DKPP_LMAX = 16;
constexpr int DKPP_BS = 4096;   // rows per pass block

template <typename T>
struct DKppState {
    long long cand_idx[DKPP_LMAX];
    long long loc_block[DKPP_LMAX];
    unsigned long long resid[DKPP_LMAX];
    unsigned long long pot;
    long long best_idx;
    int Lc, has_best, first, pad_;
};

__device__ __forceinline__ unsigned long long dkpp_w(double d, int s) {
    return (unsigned long long)__builtin_ldexp(d, s);   // d >= 0: truncation
}

template <typename T>
__global__ __launch_bounds__(256) void k_dkpp_pass(const T *__restrict__ X, long long n, int d, T *__restrict__ closest,
                                                   const DKppState<T> *__restrict__ st, int s,
                                                   unsigned long long *__restrict__ bsum) {
    const int tid = threadIdx.x;
    const long long b0 = (long long)blockIdx.x * DKPP_BS;
    const int Lc = st->Lc;
    const bool first = st->first != 0, has_best = st->has_best != 0;
    const T *best = has_best ? X + st->best_idx * d : nullptr;
    unsigned long long acc[DKPP_LMAX];
    for (int l = 0; l < DKPP_LMAX; ++l) acc[l] = 0ull;
    for (int e = tid; e < DKPP_BS; e += 256) {
        const long long i = b0 + e;
        if (i >= n) break;
        const T *x = X + i * d;
        T cl = first ? (T)__builtin_inf() : closest[i];
        if (has_best) {
            const T db = dense_dist<T>(x, best, d);
            cl = db < cl ? db : cl;
        }
        closest[i] = cl;
        for (int l = 0; l < Lc; ++l) {
            const T dc = dense_dist<T>(x, X + st->cand_idx[l] * d, d);
            acc[l] += dkpp_w((double)(dc < cl ? dc : cl), s);
        }
    }
    __shared__ unsigned long long red[DKPP_LMAX][4];
    const int lane = tid & 63, wv = tid >> 6;
    for (int l = 0; l < Lc; ++l) {
        unsigned long long v = acc[l];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) red[l][wv] = v;
    }
    __syncthreads();
    if (tid < Lc) bsum[(size_t)blockIdx.x * DKPP_LMAX + tid] = red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3];
}

// One block of 1024 threads: potentials, first argmin (the new centre); for
// the next step's L targets, the pass block whose prefix reaches each.
template <typename T>
__global__ __launch_bounds__(1024) void k_dkpp_select(const unsigned long long *__restrict__ bsum, long long nblk,
                                                      DKppState<T> *__restrict__ st, long long *__restrict__ indices,
                                                      int c, const unsigned long long *__restrict__ umant, int Lnext) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int Lc = st->Lc;
    __shared__ unsigned long long wp[16][DKPP_LMAX];
    __shared__ unsigned long long tsum[1024];
    __shared__ int s_best;
    unsigned long long p[DKPP_LMAX];
    for (int l = 0; l < DKPP_LMAX; ++l) p[l] = 0ull;
    for (long long b = tid; b < nblk; b += 1024)
        for (int l = 0; l < Lc; ++l) p[l] += bsum[(size_t)b * DKPP_LMAX + l];
    for (int l = 0; l < DKPP_LMAX; ++l) {
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
        st->best_idx = st->cand_idx[bl];
        st->has_best = 1;
        st->first = 0;
        indices[c] = st->cand_idx[bl];
    }
    __syncthreads();
    if (!umant) return;
    const int bl = s_best;
    const unsigned long long pot = st->pot;
    const long long per = (nblk + 1023) / 1024;
    const long long b0 = tid * per < nblk ? tid * per : nblk, b1 = b0 + per < nblk ? b0 + per : nblk;
    unsigned long long loc = 0ull;
    for (long long b = b0; b < b1; ++b) loc += bsum[(size_t)b * DKPP_LMAX + bl];
    tsum[tid] = loc;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const unsigned long long v = tid >= o ? tsum[tid - o] : 0ull;
        __syncthreads();
        tsum[tid] += v;
        __syncthreads();
    }
    const unsigned long long run = tsum[tid] - loc;
    for (int t = 0; t < Lnext; ++t) {
        const unsigned long long m = umant[t];
        const unsigned long long lo = m * pot, hi = __umul64hi(m, pot);
        const unsigned long long tg = (hi << 11) | (lo >> 53);   // floor(u * pot)
        unsigned long long r = run;
        for (long long b = b0; b < b1; ++b) {
            const unsigned long long v = bsum[(size_t)b * DKPP_LMAX + bl];
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

template <typename T>
__global__ void k_dkpp_init(long long first, DKppState<T> *__restrict__ st, long long *__restrict__ indices) {
    if (threadIdx.x != 0) return;
    st->cand_idx[0] = first;
    st->Lc = 1;
    st->first = 1;
    st->has_best = 0;
    st->pot = 0ull;
    indices[0] = first;
}

// One block (1024 threads) per target: the exact row inside its pass block.
template <typename T>
__global__ __launch_bounds__(1024) void k_dkpp_locate(const T *__restrict__ X, long long n, int d,
                                                      const T *__restrict__ closest, DKppState<T> *__restrict__ st,
                                                      int s) {
    const int t = blockIdx.x, tid = threadIdx.x;
    const long long b = st->loc_block[t];
    if (b < 0) {
        if (tid == 0) st->cand_idx[t] = n - 1;
        return;
    }
    const unsigned long long rs = st->resid[t];
    const T *best = X + st->best_idx * d;
    constexpr int PER = DKPP_BS / 1024;
    unsigned long long w[PER], loc = 0ull;
    for (int e = 0; e < PER; ++e) {
        const long long i = b * DKPP_BS + (long long)tid * PER + e;
        if (i < n) {
            const T db = dense_dist<T>(X + i * d, best, d);
            const T cl = closest[i];
            w[e] = dkpp_w((double)(db < cl ? db : cl), s);
        } else {
            w[e] = 0ull;
        }
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
    for (int e = 0; e < PER; ++e) {
        const long long i = b * DKPP_BS + (long long)tid * PER + e;
        if (i < n && r + w[e] >= rs) atomicMin(&found, i);
        r += w[e];
    }
    __syncthreads();
    if (tid == 0) st->cand_idx[t] = found < n ? found : n - 1;
}

}  // namespace pcm

using namespace pcm;

struct pcm_dense {
    int device = 0, d = 0, k = 0, dtype = PCM_F64, max_iter_cap = 300;
    long long n = 0;
    const void *X = nullptr;     // caller's rows (kept for the fit's duration)
    void *C = nullptr;           // [k * d] T
    int32_t *labels = nullptr;
    void *dist = nullptr;        // [n] T
    unsigned long long *stats = nullptr;   // [k * (d + 1)] + staging [k * d] T
    int *q = nullptr;
    int qh[PCM_DENSE_DMAX] = {0};
    int iscale = 0;
    int *empty_idx = nullptr;
    long long *picked = nullptr;
    unsigned long long *hist_changed = nullptr;
    double *hist_shift = nullptr;
    DenseCtrl *ctrl = nullptr;
    int num_cu = 256;
};

namespace {
size_t tsz(int dtype) { return dtype == PCM_F64 ? 8 : 4; }

template <typename F>
int dispatch_t(int dtype, F &&f) {
    if (dtype == PCM_F64) return f(double{});
    if (dtype == PCM_F32) return f(float{});
    return pcm_fail(PCM_E_ARG, "dense dtype must be PCM_F32 or PCM_F64");
}

int dense_grid(const pcm_dense *e) {
    return (int)std::max(1LL, std::min<long long>((e->n + 255) / 256, (long long)e->num_cu * 4));
}

bool dense_lds_c(const pcm_dense *e) { return (size_t)e->k * e->d * tsz(e->dtype) <= 64 * 1024; }

size_t dense_lds(const pcm_dense *e, bool with_stats) {
    const size_t cbytes = dense_lds_c(e) ? (((size_t)e->k * e->d * tsz(e->dtype) + 15) / 16) * 16 : 0;
    const size_t sbytes = (size_t)e->k * (e->d + 1) * 8;
    return cbytes + (with_stats && cbytes + sbytes <= 64 * 1024 ? sbytes : 0);
}
}  // namespace

extern "C" {

int pcm_dense_create(int device, int64_t n, int d, int k, int dtype, int max_iter, pcm_dense **out) {
    if (!out) return pcm_fail(PCM_E_ARG, "out is null");
    *out = nullptr;
    if (d < 1 || d > PCM_DENSE_DMAX) return pcm_fail(PCM_E_ARG, "d must be 1..PCM_DENSE_DMAX");
    if (k < 1 || n < 1 || k > n) return pcm_fail(PCM_E_ARG, "need 1 <= k <= n");
    if (dtype != PCM_F32 && dtype != PCM_F64) return pcm_fail(PCM_E_ARG, "dtype must be PCM_F32 or PCM_F64");
    if (max_iter < 1) return pcm_fail(PCM_E_ARG, "max_iter must be >= 1");
    if (n >= (1LL << 31)) return pcm_fail(PCM_E_ARG, "n must be < 2^31");
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != device) return pcm_fail(PCM_E_STATE, "current HIP device != device");
    pcm_dense *e = new pcm_dense();
    e->device = device;
    e->n = n;
    e->d = d;
    e->k = k;
    e->dtype = dtype;
    e->max_iter_cap = max_iter;
    if (hipDeviceGetAttribute(&e->num_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || e->num_cu < 1)
        e->num_cu = 256;
    const size_t ts = tsz(dtype);
    hipError_t err = hipSuccess;
    err = err ? err : hipMalloc(&e->C, (size_t)k * d * ts);
    err = err ? err : hipMalloc(&e->labels, (size_t)n * 4);
    err = err ? err : hipMalloc(&e->dist, (size_t)n * ts);
    err = err ? err : hipMalloc(&e->stats, (size_t)k * (d + 1) * 8 + (size_t)k * d * ts);
    err = err ? err : hipMalloc(&e->q, PCM_DENSE_DMAX * sizeof(int));
    err = err ? err : hipMalloc(&e->empty_idx, (size_t)k * sizeof(int));
    err = err ? err : hipMalloc(&e->picked, (size_t)k * sizeof(long long));
    err = err ? err : hipMalloc(&e->hist_changed, (size_t)max_iter * 8);
    err = err ? err : hipMalloc(&e->hist_shift, (size_t)max_iter * 8);
    err = err ? err : hipMalloc(&e->ctrl, sizeof(DenseCtrl));
    if (err != hipSuccess) {
        pcm_dense_destroy(e);
        return pcm_fail(PCM_E_NOMEM, std::string("dense allocation: ") + hipGetErrorString(err));
    }
    *out = e;
    return 0;
}

int pcm_dense_destroy(pcm_dense *e) {
    if (!e) return 0;
    void *ps[] = {e->C, e->labels, e->dist, e->stats, e->q, e->empty_idx, e->picked, e->hist_changed, e->hist_shift, e->ctrl};
    for (void *p : ps)
        if (p) (void)hipFree(p);
    delete e;
    return 0;
}

int pcm_dense_begin(pcm_dense *e, const void *X, const double *maxabs, const void *C0, double tol, int max_iter,
                    void *stream) {
    if (!e || !X || !maxabs || !C0) return pcm_fail(PCM_E_ARG, "bad argument");
    if (max_iter < 1 || max_iter > e->max_iter_cap) return pcm_fail(PCM_E_ARG, "max_iter exceeds the cap");
    if (!(tol >= 0.0)) return pcm_fail(PCM_E_ARG, "tol must be >= 0");
    hipStream_t s = (hipStream_t)stream;
    e->X = X;
    // q_a = 62 - e_a - bits(n): |sum| < n 2^(62 - bits(n)) <= 2^62
    int nb = 0;
    for (unsigned long long v = (unsigned long long)e->n; v; v >>= 1) ++nb;
    double bound = 0.0;
    for (int a = 0; a < e->d; ++a) {
        int ea = 0;
        if (maxabs[a] > 0.0) (void)std::frexp(maxabs[a], &ea);
        if (!std::isfinite(maxabs[a])) return pcm_fail(PCM_E_NONFINITE, "input contains NaN or Inf");
        e->qh[a] = 62 - ea - nb;
        bound += std::ldexp(1.0, 2 * (ea + 1));   // (2 * 2^e_a)^2
    }
    int eb = 0;
    (void)std::frexp(bound * (1.0 + std::ldexp(1.0, -20)), &eb);
    e->iscale = 64 - eb;
    DenseCtrl h{};
    h.max_iter = (uint32_t)max_iter;
    h.tol = tol;
    const size_t ts = tsz(e->dtype);
    if (hipMemcpyAsync(e->q, e->qh, sizeof(e->qh), hipMemcpyHostToDevice, s) ||
        hipMemcpyAsync(e->C, C0, (size_t)e->k * e->d * ts, hipMemcpyDeviceToDevice, s) ||
        hipMemsetAsync(e->labels, 0xff, (size_t)e->n * 4, s) ||
        hipMemsetAsync(e->stats, 0, (size_t)e->k * (e->d + 1) * 8, s) ||
        hipMemsetAsync(e->hist_changed, 0, (size_t)e->max_iter_cap * 8, s) ||
        hipMemsetAsync(e->hist_shift, 0, (size_t)e->max_iter_cap * 8, s) ||
        hipMemcpyAsync(e->ctrl, &h, sizeof(h), hipMemcpyHostToDevice, s) || hipStreamSynchronize(s))
        return pcm_fail(PCM_E_HIP, "pcm_dense_begin");
    return 0;
}

int pcm_dense_iterate(pcm_dense *e, int n_iter, void *stream) {
    if (!e || !e->X || n_iter < 0) return pcm_fail(PCM_E_ARG, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    return dispatch_t(e->dtype, [&](auto TT) -> int {
        using T = decltype(TT);
        const size_t lds = dense_lds(e, true);
        const int lds_stats = lds > dense_lds(e, false) ? 1 : 0;
        const int lds_c = dense_lds_c(e) ? 1 : 0;
        for (int it = 0; it < n_iter; ++it) {
            k_dense_assign<T><<<dense_grid(e), 256, lds, s>>>((const T *)e->X, e->n, e->d, (const T *)e->C, e->k, e->q,
                                                             e->labels, (T *)e->dist, e->stats, lds_stats, e->ctrl, 1,
                                                             nullptr, 0, lds_c);
            if (hipGetLastError() != hipSuccess) return pcm_fail(PCM_E_HIP, "k_dense_assign launch");
            k_dense_update<T><<<1, 256, 0, s>>>((const T *)e->X, e->n, e->d, (T *)e->C, e->k, e->q, e->labels,
                                                (const T *)e->dist, e->stats, e->empty_idx, e->picked,
                                                e->hist_changed, e->hist_shift, e->ctrl);
            if (hipGetLastError() != hipSuccess) return pcm_fail(PCM_E_HIP, "k_dense_update launch");
        }
        return 0;
    });
}

int pcm_dense_final(pcm_dense *e, void *stream) {
    if (!e || !e->X) return pcm_fail(PCM_E_ARG, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(e->ctrl->inert, 0, sizeof(e->ctrl->inert), s)) return pcm_fail(PCM_E_HIP, "final memset");
    return dispatch_t(e->dtype, [&](auto TT) -> int {
        using T = decltype(TT);
        k_dense_assign<T><<<dense_grid(e), 256, dense_lds(e, false), s>>>(
            (const T *)e->X, e->n, e->d, (const T *)e->C, e->k, e->q, e->labels, nullptr, nullptr, 0, e->ctrl, 0,
            e->ctrl->inert, e->iscale, dense_lds_c(e) ? 1 : 0);
        if (hipGetLastError() != hipSuccess) return pcm_fail(PCM_E_HIP, "final assign launch");
        return 0;
    });
}

int pcm_dense_status(pcm_dense *e, pcm_status *out, void *stream) {
    if (!e || !out) return pcm_fail(PCM_E_ARG, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    DenseCtrl h{};
    if (hipMemcpyAsync(&h, e->ctrl, sizeof(h), hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s))
        return pcm_fail(PCM_E_HIP, "pcm_dense_status");
    std::memset(out, 0, sizeof(*out));
    out->done = h.done;
    out->iter = h.iter;
    out->last_changed = h.last_changed;
    out->last_shift = h.last_shift;
    for (int t = 0; t < 3; ++t) out->inertia_limbs[t] = h.inert[t];
    out->inertia_scale = e->iscale;
    out->inertia_overflow = (uint32_t)h.inert[3];
    out->inertia = pcm_inertia_value(out->inertia_limbs, e->iscale, out->inertia_overflow);
    out->list_rebuilds = h.relocs;   // dense path: relocation events
    return 0;
}

int pcm_dense_outputs(pcm_dense *e, int32_t *labels, void *centers, uint64_t *changed, double *shift, int cap,
                      void *stream) {
    if (!e) return pcm_fail(PCM_E_ARG, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    if (labels && hipMemcpyAsync(labels, e->labels, (size_t)e->n * 4, hipMemcpyDeviceToDevice, s))
        return pcm_fail(PCM_E_HIP, "dense labels");
    if (centers && hipMemcpyAsync(centers, e->C, (size_t)e->k * e->d * tsz(e->dtype), hipMemcpyDeviceToDevice, s))
        return pcm_fail(PCM_E_HIP, "dense centers");
    const int c = std::min(cap, e->max_iter_cap);
    if (changed && c > 0 && hipMemcpyAsync(changed, e->hist_changed, (size_t)c * 8, hipMemcpyDeviceToHost, s))
        return pcm_fail(PCM_E_HIP, "dense history");
    if (shift && c > 0 && hipMemcpyAsync(shift, e->hist_shift, (size_t)c * 8, hipMemcpyDeviceToHost, s))
        return pcm_fail(PCM_E_HIP, "dense history");
    if (hipStreamSynchronize(s)) return pcm_fail(PCM_E_HIP, "dense outputs");
    return 0;
}

int pcm_dense_kmeanspp_workspace(int64_t n, int d, int dtype, int k, int n_local_trials, size_t *bytes) {
    if (!bytes || n < 1 || d < 1 || k < 1 || n_local_trials < 1 || n_local_trials > DKPP_LMAX)
        return pcm_fail(PCM_E_ARG, "bad argument");
    const long long nblk = (n + DKPP_BS - 1) / DKPP_BS;
    *bytes = (size_t)n * tsz(dtype) + 256 + (size_t)nblk * DKPP_LMAX * 8 + 256 + sizeof(DKppState<double>) + 256 +
             (size_t)std::max(1, (k - 1) * n_local_trials) * 8;
    return 0;
}

int pcm_dense_kmeanspp(const void *X, int64_t n, int d, int dtype, int k, int n_local_trials, int64_t first_index,
                       const uint64_t *umant, int scale, int64_t *indices, void *workspace, size_t workspace_bytes,
                       void *stream) {
    if (!X || !indices || n < 1 || k < 1 || k > n || d < 1 || d > PCM_DENSE_DMAX) return pcm_fail(PCM_E_ARG, "bad argument");
    if (n_local_trials < 1 || n_local_trials > DKPP_LMAX) return pcm_fail(PCM_E_ARG, "n_local_trials must be 1..16");
    if (first_index < 0 || first_index >= n) return pcm_fail(PCM_E_ARG, "first_index out of range");
    if (k > 1 && !umant) return pcm_fail(PCM_E_ARG, "umant is null");
    size_t need = 0;
    if (int rc = pcm_dense_kmeanspp_workspace(n, d, dtype, k, n_local_trials, &need)) return rc;
    if (!workspace || workspace_bytes < need) return pcm_fail(PCM_E_ARG, "workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const int L = n_local_trials;
    const long long nblk = (n + DKPP_BS - 1) / DKPP_BS;
    char *wb = (char *)workspace;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t at = o; o += ((bytes + 255) / 256) * 256; return wb + at; };
    void *closest = take((size_t)n * tsz(dtype));
    unsigned long long *bsum = (unsigned long long *)take((size_t)nblk * DKPP_LMAX * 8);
    void *st = take(sizeof(DKppState<double>));
    unsigned long long *um = (unsigned long long *)take((size_t)std::max(1, (k - 1) * L) * 8);
    if (k > 1 && hipMemcpy(um, umant, (size_t)(k - 1) * L * 8, hipMemcpyHostToDevice))
        return pcm_fail(PCM_E_HIP, "dense kmeanspp uniforms");
    return dispatch_t(dtype, [&](auto TT) -> int {
        using T = decltype(TT);
        DKppState<T> *S = (DKppState<T> *)st;
        k_dkpp_init<T><<<1, 64, 0, s>>>(first_index, S, (long long *)indices);
        for (int c = 0; c < k; ++c) {
            k_dkpp_pass<T><<<(int)nblk, 256, 0, s>>>((const T *)X, n, d, (T *)closest, S, scale, bsum);
            const bool more = c + 1 < k;
            k_dkpp_select<T><<<1, 1024, 0, s>>>(bsum, nblk, S, (long long *)indices, c, more ? um + (size_t)c * L : nullptr,
                                                L);
            if (more) k_dkpp_locate<T><<<L, 1024, 0, s>>>((const T *)X, n, d, (const T *)closest, S, scale);
            if (hipGetLastError() != hipSuccess) return pcm_fail(PCM_E_HIP, "dense kmeanspp launch");
        }
        return 0;
    });
}

}  // extern "C"
