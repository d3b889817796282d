// pcm_kpp.hpp — k-means++ seeding on gfx950 with exact
// cell-grid skipping.
//
// Restates scikit-learn's _kmeans_plusplus (sklearn/cluster/_kmeans.py:174-272,
// the KMeans default init, :1012-1019) with the canonical arithmetic of
// oracle/kpp_ref.py: float32 direct-form distances, integer point weights
// w = trunc(ldexp(double(d), s)), exact integer potentials and cumulative sums
// (in the caller's row order), targets floor(u * pot) computed exactly from u's
// 53-bit mantissa.
//
// The cloud is laid out in pruning-grid cell order (the Lloyd engine's record
// sort, pcm_sort.hpp: AoSoA-4 points + perm).  Per centre c = 1 .. k-1, three
// stream-ordered launches:
//   k_kpp_search  L blocks: target t's original-order weight block by an exact
//                 prefix over the block sums `bsum`, then the first row of that
//                 block whose inclusive prefix reaches the target (searchsorted
//                 side='left'; the rows' weights from `crow`, the caller-order
//                 copy of the closest distances); extra blocks reduce the per-cell maxima of
//                 `closest` to gmax (a bound on every point's closest distance)
//   k_kpp_eval    per candidate, the potential drop sum_i w(closest_i) -
//                 w(min(closest_i, d(x_i, cand))) over the cells the candidate
//                 can reach: cells of the cube of radius sqrt(gmax) around it
//                 whose box lower bound on the fp32 distance is below the cell's
//                 max closest -- every other point's term is exactly 0
//   k_kpp_apply   the first argmin of the potentials becomes centre c; the
//                 closest distances, cell maxima and block sums of the cells it
//                 reaches are updated
// so a step touches only the neighbourhood of its L + 1 candidates (early
// steps, with gmax large, are full passes).  Potentials are exact unsigned
// integers: the sampled indices are the oracle's for any launch geometry.
#pragma once
#include "pcm_kernels.hpp"

namespace pcm {

constexpr int KPP_LMAX = 16;
#ifndef PCM_KPP_PPL
#define PCM_KPP_PPL 8
#endif
constexpr int KPP_PPL = PCM_KPP_PPL;           // points per lane per pass of one-candidate cell visits
constexpr int KPP_OB_LOG = 12;                 // original-order weight blocks of 4096 rows
constexpr int KPP_OB = 1 << KPP_OB_LOG;
constexpr int KPP_CELL_PTS = 256;              // target points per pruning cell
constexpr int KPP_STPB = 1024;                 // k_kpp_search block size
constexpr int KPP_RED_BLOCKS = 64;             // gmax reduction blocks of k_kpp_search
constexpr int KPP_SCU = 32;                    // k_kpp_search: 64-wide chunks of block sums kept in registers per wave
// Same-address device atomics serialise at the memory side (~12 ns each,
// MI355X_MICROARCH.md "fanin") and stall the loads queued behind them: 1024
// per-wave atomicMax on one gmax word held k_kpp_search's block-sum loads for
// ~10 us, thousands of per-wave adds on the 8 candidate potentials held
// k_kpp_eval's cell loads.  Reductions therefore go through LDS, then per-block
// plain stores (gmax) or adds spread over KPP_DREP replica lines (potentials).
constexpr int KPP_DREP = 32;

struct KppCtl {
    float4 cand[KPP_LMAX];
    long long cand_idx[KPP_LMAX];
    unsigned long long pot[2];                 // potential at the start of step c: pot[c & 1]
    unsigned long long drep[KPP_DREP][KPP_LMAX];   // potential drop of each candidate: sum of the replicas (k_kpp_eval)
    unsigned int gpart[KPP_RED_BLOCKS];        // float bits: max closest per reduction block of step c's search
};

// gmax = max of the reduction blocks' parts (whole block must call)
__device__ __forceinline__ float kpp_gmax(const KppCtl *__restrict__ ctl, unsigned *s_g) {
    if (threadIdx.x < 64) {
        unsigned m = threadIdx.x < KPP_RED_BLOCKS ? ctl->gpart[threadIdx.x] : 0u;
        for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
        if (threadIdx.x == 0) *s_g = m;
    }
    __syncthreads();
    return __uint_as_float(*s_g);
}

// w = trunc(ldexp(double(d), s)) for d >= 0, from the fp32 fields with integer
// ops (exact: d = mant * 2^e2 before scaling; w < 2^64 by the choice of s).
__device__ __forceinline__ unsigned long long kpp_w(float d, int s) {
    const unsigned bits = __float_as_uint(d);
    const int E = (int)(bits >> 23);
    const unsigned long long mant = (unsigned long long)((bits & 0x7fffffu) | (E ? 0x800000u : 0u));
    const int e2 = (E ? E - 150 : -149) + s;
    if (e2 >= 0) return mant << e2;
    return e2 > -64 ? mant >> (-e2) : 0ull;
}

template <int D>
__device__ __forceinline__ void kpp_point(const float *__restrict__ xs, long long i, float (&x)[D]) {
#pragma unroll
    for (int a = 0; a < D; ++a) x[a] = xs[xs_index<D>(i, a)];
}

// Conservative reach test: true iff some point of the cell may have a
// canonical fp32 distance to c strictly below cmax (the cell's max closest).
// The cell is given by its fine coordinates f (its fp64 box computed here) or,
// for a box tested against several candidates, by the box itself.
template <int D>
__device__ __forceinline__ bool kpp_reaches_box(const double (&blo)[MAXD], const double (&bhi)[MAXD], const float4 &c,
                                                float cmax) {
    double m = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        const double ca = (double)comp(c, a);
        const double t = ca < blo[a] ? blo[a] - ca : (ca > bhi[a] ? ca - bhi[a] : 0.0);
        m += t * t;
    }
    // d~ >= d (1 - 5u) - 3 * 2^-150 (DESIGN.md "Exactness of pruning")
    return m * (1.0 - PEPS) - PTAU < (double)cmax;
}

template <int D>
__device__ __forceinline__ bool kpp_reaches_f(const Grid &g, const int (&f)[MAXD], const float4 &c, float cmax) {
    double blo[MAXD], bhi[MAXD];
    cell_box<D>(g, f, f, blo, bhi);
    return kpp_reaches_box<D>(blo, bhi, c, cmax);
}

// fine coordinates of a cell id with 32-bit divisions (the k-means++ grid holds
// <= 2^20 cells): the 64-bit div/mod of `decode` expand to long sequences, and
// the late steps run one reach test per lane on their critical path
template <int D>
__device__ __forceinline__ void decode32(unsigned c, const int *G, int (&f)[MAXD]) {
#pragma unroll
    for (int a = D - 1; a >= 0; --a) {
        const unsigned gd = (unsigned)G[a];
        f[a] = (int)(c % gd);
        c /= gd;
    }
}

// Cell-index cube around c of half-width sqrt(gmax) (+ one cell of binning slack).
template <int D>
__device__ __forceinline__ void kpp_cube(const Grid &g, const float4 &c, float gmax, int (&i0)[MAXD], int (&i1)[MAXD],
                                         long long &vol) {
    const double R = sqrt((double)gmax * (1.0 + 1.52587890625e-05) + 1e-36);
    vol = 1;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        if (g.G[a] <= 1 || !(g.inv[a] > 0.0)) {
            i0[a] = 0;
            i1[a] = g.G[a] - 1;
        } else {
            const double ca = (double)comp(c, a);
            const double lo = floor((ca - R - g.lo[a]) * g.inv[a]) - 1.0, hi = floor((ca + R - g.lo[a]) * g.inv[a]) + 1.0;
            i0[a] = lo < 0.0 ? 0 : (lo > (double)(g.G[a] - 1) ? g.G[a] - 1 : (int)lo);
            i1[a] = hi < 0.0 ? 0 : (hi > (double)(g.G[a] - 1) ? g.G[a] - 1 : (int)hi);
        }
        vol *= (long long)(i1[a] - i0[a] + 1);
    }
}

// Cube item `local` (< 2^31: a cube never exceeds the grid) -> its fine
// coordinates f and cell id, 32-bit divisions.
template <int D>
__device__ __forceinline__ long long kpp_cube_cell(const Grid &g, const int (&i0)[MAXD], const int (&i1)[MAXD],
                                                   unsigned local, int (&f)[MAXD]) {
#pragma unroll
    for (int a = D - 1; a >= 0; --a) {
        const unsigned w = (unsigned)(i1[a] - i0[a] + 1);
        f[a] = i0[a] + (int)(local % w);
        local /= w;
    }
    return encode(f, g.G, D);
}

// Inclusive wave scan of a u64 by DPP moves of both halves (row_shr 1/2/4/8
// inside rows of 16, then row_bcast 15 / 31 across rows; out-of-row sources
// read 0): VALU-only, no LDS crossbar round trips -- the ds_bpermute chains of
// 64-bit shuffles cost ~7 us of k_kpp_search's 33 (tools/kpp_timing.py).
// The whole wave must be active.
__device__ __forceinline__ unsigned long long wave_scan_u64(unsigned long long v) {
#define PCM_DPP_ADD(ctrl, rmask)                                                                              \
    {                                                                                                         \
        const unsigned lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)v, ctrl, rmask, 0xF, false);          \
        const unsigned hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(v >> 32), ctrl, rmask, 0xF, false);  \
        v += ((unsigned long long)hi << 32) | lo;                                                             \
    }
    PCM_DPP_ADD(0x111, 0xF)
    PCM_DPP_ADD(0x112, 0xF)
    PCM_DPP_ADD(0x114, 0xF)
    PCM_DPP_ADD(0x118, 0xF)
    PCM_DPP_ADD(0x142, 0xA)
    PCM_DPP_ADD(0x143, 0xC)
#undef PCM_DPP_ADD
    return v;
}

// lane 63 of the inclusive scan, broadcast (uniform)
__device__ __forceinline__ unsigned long long wave_last_u64(unsigned long long v) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), 63);
    return ((unsigned long long)hi << 32) | lo;
}

// lane `src`'s value (uniform src), broadcast
__device__ __forceinline__ unsigned long long wave_bcast_u64(unsigned long long v, int src) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), src);
    return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    return wave_last_u64(wave_scan_u64(v));
}

__device__ __forceinline__ float wave_max_f(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// Visit the points [b, e) of one cell with a wave, PPL points per lane per
// pass: the coordinate and `closest` loads of the PPL points are all issued
// before any is used (one memory latency per 64 PPL points instead of PPL
// dependent rounds).  f(i, x, closest_i) per point.  The grid's cells hold ~380
// points at config 3 (2^18 cells): PPL = 8 visits most of them in one pass
// (one-candidate items: eval's per-(candidate, cell) items and apply); PPL = 4
// where registers are scarce (eval's whole-cell walk keeps 16 candidate sums).
template <int D, int PPL = 4, typename F>
__device__ __forceinline__ void kpp_cell_points(const float *__restrict__ xs, const float *__restrict__ closest,
                                                uint32_t b, uint32_t e, int lane, F &&f) {
    for (uint32_t i0 = b + lane; i0 < e; i0 += 64u * PPL) {
        float x[PPL][D], cl[PPL];
#pragma unroll
        for (int u = 0; u < PPL; ++u) {
            const uint32_t i = i0 + 64u * u;
            const uint32_t ii = i < e ? i : i0;
            kpp_point<D>(xs, ii, x[u]);
            cl[u] = closest[ii];
        }
#pragma unroll
        for (int u = 0; u < PPL; ++u)
            if (i0 + 64u * u < e) f(i0 + 64u * u, x[u], cl[u]);
    }
}

// kpp_cell_points that also loads each point's caller row (perm) in the same
// batch, so that apply's row-order updates (crow, block sums) do not wait for a
// dependent perm load after the distances
template <int D, int PPL, typename F>
__device__ __forceinline__ void kpp_cell_points_rows(const float *__restrict__ xs, const float *__restrict__ closest,
                                                     const uint32_t *__restrict__ perm, uint32_t b, uint32_t e,
                                                     int lane, F &&f) {
    for (uint32_t i0 = b + lane; i0 < e; i0 += 64u * PPL) {
        float x[PPL][D], cl[PPL];
        uint32_t rw[PPL];
#pragma unroll
        for (int u = 0; u < PPL; ++u) {
            const uint32_t i = i0 + 64u * u;
            const uint32_t ii = i < e ? i : i0;
            kpp_point<D>(xs, ii, x[u]);
            cl[u] = closest[ii];
            rw[u] = perm[ii];
        }
#pragma unroll
        for (int u = 0; u < PPL; ++u)
            if (i0 + 64u * u < e) f(i0 + 64u * u, x[u], cl[u], rw[u]);
    }
}

__device__ __forceinline__ float4 kpp_row_centre(const float *__restrict__ X, long long r, int D) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int a = 0; a < D; ++a) v[a] = X[r * D + a];
    return make_float4(v[0], v[1], v[2], v[3]);
}

// Step 0, cell order: closest := d(x, c0) for every point and the cell maxima.
// One wave per cell (strided).
template <int D>
__global__ __launch_bounds__(256) void k_kpp_init(const float *__restrict__ xs, const uint32_t *__restrict__ cell_start,
                                                  long long ncells, const float *__restrict__ X, long long first,
                                                  float *__restrict__ closest, float *__restrict__ cmax,
                                                  long long *__restrict__ indices) {
    if (blockIdx.x == 0 && threadIdx.x == 0) indices[0] = first;
    const float4 c0 = kpp_row_centre(X, first, D);
    const int lane = threadIdx.x & 63;
    const long long wid = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    for (long long cell = wid; cell < ncells; cell += nw) {
        const uint32_t b = cell_start[cell], e = cell_start[cell + 1];
        float mx = 0.f;
        for (uint32_t i = b + lane; i < e; i += 64) {
            float x[D];
            kpp_point<D>(xs, i, x);
            const float d = dist_canon<D>(x, c0);
            closest[i] = d;
            mx = fmaxf(mx, d);
        }
        mx = wave_max_f(mx);
        if (lane == 0) cmax[cell] = mx;
    }
}

// Step 0, row order: crow[j] := d(X_j, c0) (the caller-order copy of `closest`
// that k_kpp_search reads), the weight sum of every KPP_OB-row block (a block
// reduction, plain store: no atomics) and the potential (one atomic per
// workgroup).  The same canonical distance as k_kpp_init: bitwise equal values.
template <int D>
__global__ __launch_bounds__(256) void k_kpp_init_rows(const float *__restrict__ X, long long n, long long first, int s,
                                                       float *__restrict__ crow, unsigned long long *__restrict__ bsum,
                                                       KppCtl *__restrict__ ctl) {
    __shared__ unsigned long long wtot[4];
    const float4 c0 = kpp_row_centre(X, first, D);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long long nb = (n + KPP_OB - 1) / KPP_OB;
    unsigned long long pot = 0ull;
    for (long long b = blockIdx.x; b < nb; b += gridDim.x) {
        unsigned long long acc = 0ull;
#pragma unroll 4
        for (int e = 0; e < KPP_OB / 256; ++e) {
            const long long j = b * KPP_OB + e * 256 + tid;
            if (j < n) {
                float x[D];
#pragma unroll
                for (int a = 0; a < D; ++a) x[a] = X[j * D + a];
                const float d = dist_canon<D>(x, c0);
                crow[j] = d;
                acc += kpp_w(d, s);
            }
        }
        acc = wave_sum_u64(acc);
        if (lane == 0) wtot[wv] = acc;
        __syncthreads();
        if (tid == 0) {
            const unsigned long long t = wtot[0] + wtot[1] + wtot[2] + wtot[3];
            bsum[b] = t;
            pot += t;
        }
        __syncthreads();
    }
    if (tid == 0 && pot) atomicAdd(&ctl->pot[1], pot);
}

// Inclusive scan of one u64 per thread over a KPP_STPB-thread block: wave
// scans (shfl_up), one LDS pass over the wave totals.  Returns the EXCLUSIVE
// prefix of this thread.
__device__ __forceinline__ unsigned long long kpp_block_exscan(unsigned long long v, unsigned long long *wtot) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const unsigned long long inc = wave_scan_u64(v);
    if (lane == 63) wtot[wv] = inc;
    __syncthreads();
    unsigned long long base = 0ull;
    for (int w = 0; w < wv; ++w) base += wtot[w];
    __syncthreads();
    return base + inc - v;
}

// Step c (>= 1): blocks t < L locate candidate t; blocks >= L reduce gmax.
//  1. the original-order weight block holding target tg: wave w owns a
//     contiguous segment of the block sums and reads it coalesced (lane l,
//     chunk u: sum index seg + 64 u + l), KPP_SCU chunks kept in registers; the
//     wave totals give each segment's exclusive base, and the one wave whose
//     segment holds the target scans its chunks (wave prefix sums) for the
//     unique block with  incl >= tg  and  (first block or excl < tg);
//  2. the same unique-row test inside that block (4096 rows, 4 per thread,
//     a block prefix scan): a plain LDS store, no atomic.
// Measured per-phase (tools/kpp_timing.py): per-thread ranges of 24 sums
// (uncoalesced, one latency each) and an LDS atomicMin of every row past the
// target made this launch 45-54 us per centre.
template <int D>
__global__ __launch_bounds__(KPP_STPB) void k_kpp_search(const unsigned long long *__restrict__ bsum, long long nb,
                                                         const float *__restrict__ crow, const float *__restrict__ X,
                                                         long long n, const unsigned long long *__restrict__ umant,
                                                         int L, int s, int c, const float *__restrict__ cmax,
                                                         long long ncells, KppCtl *__restrict__ ctl) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    DBG_T(0);
    constexpr int NWV = KPP_STPB / 64;
    if ((int)blockIdx.x >= L) {   // gmax part: max over a slice of the cells' max closest
        __shared__ unsigned int s_m[NWV];
        unsigned int m = 0u;
        for (long long cl = (blockIdx.x - L) * (long long)KPP_STPB + tid; cl < ncells;
             cl += (long long)(gridDim.x - L) * KPP_STPB)
            m = max(m, __float_as_uint(cmax[cl]));
        for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, o));
        if (lane == 0) s_m[wv] = m;
        __syncthreads();
        if (tid == 0) {
            for (int w = 1; w < NWV; ++w) m = max(m, s_m[w]);
            ctl->gpart[blockIdx.x - L] = m;
        }
        DBG_T(8);
        return;
    }
    const int t = blockIdx.x;
    if (t == 0)
        for (int l = tid; l < KPP_DREP * KPP_LMAX; l += KPP_STPB) (&ctl->drep[0][0])[l] = 0ull;
    __shared__ unsigned long long wtot[NWV];
    __shared__ unsigned long long s_tr[KPP_SCU][64];   // the target wave's chunks, transposed (16 KB)
    __shared__ long long s_blk;
    __shared__ unsigned long long s_res;
    __shared__ long long s_found;
    const unsigned long long pot = ctl->pot[c & 1];
    const unsigned long long m = umant[t];
    if (tid == 0) { s_blk = -1; s_found = 0x7fffffffffffffffll; }
    // 1. this wave's segment [sb, se) of the block sums, 64-wide chunks (issued
    // before the target is computed: the loads do not wait for pot / umant)
    const long long seg = ((nb + NWV * 64 - 1) / (NWV * 64)) * 64;
    const long long sb = min((long long)wv * seg, nb), se = min(sb + seg, nb);
    const int nch = (int)((se - sb + 63) / 64);
    constexpr int CU = KPP_SCU;
    unsigned long long v[CU];
    unsigned long long lsum = 0ull;
#pragma unroll
    for (int u = 0; u < CU; ++u) {
        const long long b = sb + 64LL * u + lane;
        v[u] = (u < nch && b < se) ? bsum[b] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < CU; ++u) lsum += v[u];
    for (int u = CU; u < nch; ++u) {   // segments longer than the register cache (n > ~134M points)
        const long long b = sb + 64LL * u + lane;
        lsum += b < se ? bsum[b] : 0ull;
    }
    const unsigned long long lo = m * pot, hi = __umul64hi(m, pot);
    const unsigned long long tg = (hi << 11) | (lo >> 53);   // floor(u * pot), u = m / 2^53
    const unsigned long long wsum = wave_sum_u64(lsum);
    if (lane == 0) wtot[wv] = wsum;
    __syncthreads();
    DBG_T(2);
    unsigned long long base = 0ull;
    for (int w = 0; w < wv; ++w) base += wtot[w];
    const bool mine = (tg == 0ull) ? (sb == 0 && se > 0) : (base < tg && tg <= base + wsum);
    if (mine) {   // wave-uniform
        // the chunk holding the target: the wave's register cache transposed
        // through LDS, lane u < CU sums chunk u (one 8-B read per lane and step,
        // rotated so that the 32 lanes hit distinct banks), one wave scan over the
        // chunk totals; then one wave scan of that chunk (round 6: 32 dependent
        // wave scans of the chunks in registers took 3.6 us of the launch's 10.6,
        // tools/kpp_timing.py)
#pragma unroll
        for (int u = 0; u < CU; ++u) s_tr[u][lane] = v[u];
        unsigned long long ct = 0ull;
        if (lane < CU) {
#pragma unroll 16
            for (int j = 0; j < 64; ++j) ct += s_tr[lane][(j + lane) & 63];
        }
        const unsigned long long ci = wave_scan_u64(ct);   // inclusive over the chunks (lanes >= CU add 0)
        const bool hit = lane < CU && lane < nch && base + ci >= tg;
        const unsigned long long hb = __ballot(hit);
        unsigned long long r = base, x = 0ull, xi = 0ull;
        int uc = -1;
        if (hb) {
            uc = __builtin_ctzll(hb);
            const unsigned long long cu = wave_bcast_u64(ci, uc), tu = wave_bcast_u64(ct, uc);
            r = base + cu - tu;   // everything before chunk uc
            x = s_tr[uc][lane];
            xi = wave_scan_u64(x);
        } else {
            r = base + wave_bcast_u64(ci, CU - 1);   // past the register chunks
        }
        for (int u = CU; uc < 0 && u < nch; ++u) {   // past the register cache (n > ~134M points)
            const long long b = sb + 64LL * u + lane;
            const unsigned long long y = b < se ? bsum[b] : 0ull;
            const unsigned long long inc = wave_scan_u64(y);
            const unsigned long long ct2 = wave_last_u64(inc);
            if (r + ct2 >= tg) { uc = u; x = y; xi = inc; } else { r += ct2; }
        }
        if (uc >= 0) {
            const long long b = sb + 64LL * uc + lane;
            const unsigned long long inc = xi;
            const unsigned long long ex = r + inc - x;
            if (b < se && r + inc >= tg && (b == 0 || ex < tg)) {   // first block whose inclusive prefix reaches tg
                s_blk = b;
                s_res = tg - ex;
            }
        }
    }
    __syncthreads();
    DBG_T(4);
    const long long blk = s_blk;
    long long idx = n - 1;   // past the end (np.searchsorted -> n, clipped): not reachable, tg < pot
    if (blk >= 0) {
        // 2. first row of the block whose inclusive prefix reaches the residual
        const unsigned long long rs = s_res;
        constexpr int PER = KPP_OB / KPP_STPB;
        unsigned long long w[PER];
        unsigned long long l2 = 0ull;
        float cr[PER];
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            const long long j = blk * KPP_OB + (long long)tid * PER + e;
            cr[e] = j < n ? crow[j] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            const long long j = blk * KPP_OB + (long long)tid * PER + e;
            w[e] = j < n ? kpp_w(cr[e], s) : 0ull;
            l2 += w[e];
        }
        DBG_T(5);
        unsigned long long q = kpp_block_exscan(l2, wtot);
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            const long long j = blk * KPP_OB + (long long)tid * PER + e;
            if (j < n && q + w[e] >= rs && (j == blk * KPP_OB || q < rs)) s_found = j;   // unique row
            q += w[e];
        }
        __syncthreads();
        idx = s_found < n ? s_found : n - 1;
    }
    DBG_T(6);
    if (tid == 0) {
        float vv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a = 0; a < D; ++a) vv[a] = X[idx * D + a];
        ctl->cand[t] = make_float4(vv[0], vv[1], vv[2], vv[3]);
        ctl->cand_idx[t] = idx;
    }
    DBG_T(7);
}

// Step c: potential drop of every candidate over the cells it reaches.  While
// the candidates' cubes together cover more items than the grid has cells
// (early steps), every wave walks whole cells and evaluates all reaching
// candidates on one load of each point; later, one wave per (candidate, cube
// cell) item.  Per-lane, per-candidate partial sums in registers, one wave
// reduction and atomic per candidate at the end.
// LM: the candidate accumulators kept per lane (8 when n_local_trials <= 8, as
// sklearn's 2 + int(log(k)) is up to k = 2980; else KPP_LMAX)
// eval with 8 candidate sums at 6 waves per SIMD (79 VGPRs, no spill): 91.3-91.5
// -> 90.6 ms per seeding at config 3 (round 5, profiles/rd5_kpp_steps.txt)
#ifndef PCM_KPP_EVAL_WPE
#define PCM_KPP_EVAL_WPE 6
#endif
template <int D, int LM = KPP_LMAX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LM <= 8 ? PCM_KPP_EVAL_WPE : 1, 8))) void k_kpp_eval(const float *__restrict__ xs, const uint32_t *__restrict__ cell_start,
                                                  Grid g, const float *__restrict__ closest,
                                                  const float *__restrict__ cmax, int L, int s, int c,
                                                  KppCtl *__restrict__ ctl) {
    __shared__ int s_i0[KPP_LMAX][MAXD], s_i1[KPP_LMAX][MAXD];
    __shared__ long long s_off[KPP_LMAX + 1];
    __shared__ float4 s_cand[KPP_LMAX];
    __shared__ unsigned s_g;
    __shared__ unsigned long long s_red[4][KPP_LMAX];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    DBG_E(0);
    const float4 cd = ctl->cand[tid < L ? tid : 0];   // issued together with the gmax parts
    const float gmax = kpp_gmax(ctl, &s_g);
    if (tid < L) {
        int i0[MAXD], i1[MAXD];
        long long vol;
        kpp_cube<D>(g, cd, gmax, i0, i1, vol);
#pragma unroll
        for (int a = 0; a < D; ++a) { s_i0[tid][a] = i0[a]; s_i1[tid][a] = i1[a]; }
        s_off[tid + 1] = vol;
        s_cand[tid] = cd;
    }
    __syncthreads();
    if (tid == 0) {
        s_off[0] = 0;
        for (int l = 0; l < L; ++l) s_off[l + 1] += s_off[l];
    }
    __syncthreads();
    const long long total = s_off[L];
    DBG_E(1);
    DBG_EV(5, total);
    const long long wid = (blockIdx.x * (long long)blockDim.x + tid) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    unsigned dbg_cells = 0;
    unsigned long long dw[LM];
#pragma unroll
    for (int q = 0; q < LM; ++q) dw[q] = 0ull;
    if (total > g.ncells) {
        // this wave's cells wid, wid + nw, ...: one per lane, each lane tests its
        // cell against every candidate (cmax and the bounds of up to 64 cells
        // loaded together), then the reached cells one after another
        const long long cpw = g.ncells > wid ? (g.ncells - wid + nw - 1) / nw : 0;
        for (long long k0 = 0; k0 < cpw; k0 += 64) {
            unsigned lmask = 0u;
            uint32_t cb = 0u, ce = 0u;
            if (k0 + lane < cpw) {
                const long long cl = wid + (k0 + lane) * nw;
                const float cm = cmax[cl];
                cb = cell_start[cl];
                ce = cell_start[cl + 1];
                // the cell's box once, then every candidate against it
                int f[MAXD];
                decode32<D>((unsigned)cl, g.G, f);
                double blo[MAXD], bhi[MAXD];
                cell_box<D>(g, f, f, blo, bhi);
                for (int q = 0; q < L; ++q)
                    if (kpp_reaches_box<D>(blo, bhi, s_cand[q], cm)) lmask |= 1u << q;
            }
            unsigned long long bits = __ballot(lmask != 0u);
            if (lane == 0) {
                DBG_KPP(c, 0, (unsigned)min(64LL, cpw - k0));
                DBG_KPP(c, 1, __popcll(bits));
            }
            while (bits) {
                const int src = __builtin_ctzll(bits);
                bits &= bits - 1ull;
                const unsigned mask = (unsigned)__shfl((int)lmask, src);
                const uint32_t b = (uint32_t)__shfl((int)cb, src), e = (uint32_t)__shfl((int)ce, src);
                // the candidates are re-read from LDS per cell: hoisted out of the
                // cell loop they held 16 x 4 VGPRs for the whole launch
                asm volatile("" ::: "memory");
                kpp_cell_points<D>(xs, closest, b, e, lane, [&](uint32_t, const float (&x)[D], float cl) {
                    const unsigned long long wcl = kpp_w(cl, s);
#pragma unroll
                    for (int q = 0; q < LM; ++q) {
                        if (!((mask >> q) & 1u)) continue;
                        const float d = dist_canon<D>(x, s_cand[q]);
                        if (d < cl) dw[q] += wcl - kpp_w(d, s);
                    }
                });
            }
        }
    } else {
        // this wave's items wid, wid + nw, ... (ipw of them): their reach tests
        // run one per lane (cmax and the cell bounds of up to 64 items loaded
        // together: one memory latency), then the reached cells one after
        // another (wave-uniform)
        const long long ipw = total > wid ? (total - wid + nw - 1) / nw : 0;
        for (long long k0 = 0; k0 < ipw; k0 += 64) {
            const long long it = wid + (k0 + lane) * nw;
            long long cell = 0;
            bool reach = false;
            uint32_t cb = 0u, ce = 0u;
            int l = 0;
            if (k0 + lane < ipw) {
                while (it >= s_off[l + 1]) ++l;
                int i0[MAXD], i1[MAXD];
#pragma unroll
                for (int a = 0; a < D; ++a) { i0[a] = s_i0[l][a]; i1[a] = s_i1[l][a]; }
                int f[MAXD];
                cell = kpp_cube_cell<D>(g, i0, i1, (unsigned)(it - s_off[l]), f);
                const float cm = cmax[cell];
                cb = cell_start[cell];
                ce = cell_start[cell + 1];
                reach = kpp_reaches_f<D>(g, f, s_cand[l], cm);
            }
            unsigned long long bits = __ballot(reach);
            if (k0 == 0) DBG_E(3);
            dbg_cells += (unsigned)__popcll(bits);
            if (lane == 0) {
                DBG_KPP(c, 0, (unsigned)min(64LL, ipw - k0));
                DBG_KPP(c, 1, __popcll(bits));
            }
            while (bits) {
                const int src = __builtin_ctzll(bits);
                bits &= bits - 1ull;
                const int lq = __shfl(l, src);
                const uint32_t b = (uint32_t)__shfl((int)cb, src), e = (uint32_t)__shfl((int)ce, src);
                const float4 cd = s_cand[lq];
                unsigned long long v = 0ull;
                kpp_cell_points<D, KPP_PPL>(xs, closest, b, e, lane, [&](uint32_t, const float (&x)[D], float cl) {
                    const float d = dist_canon<D>(x, cd);
                    if (d < cl) v += kpp_w(cl, s) - kpp_w(d, s);
                });
#pragma unroll
                for (int q = 0; q < LM; ++q)
                    if (q == lq) dw[q] += v;
                if (dbg_cells > 0u && k0 == 0) DBG_E(6);
            }
        }
    }
    DBG_E(2);
    DBG_EV(4, dbg_cells);
    (void)dbg_cells;
    // waves that reached no cell hold zeros: skip their L wave reductions (in the
    // late steps most of the grid's waves have no item, and 8 x 12 cross-lane
    // moves per idle wave were a large share of the launch)
    unsigned long long nz = 0ull;
#pragma unroll
    for (int q = 0; q < LM; ++q) nz |= dw[q];
    if (__ballot(nz != 0ull) != 0ull) {   // wave-uniform
#pragma unroll
        for (int q = 0; q < LM; ++q) {
            if (q >= L) break;
            const unsigned long long v = wave_sum_u64(dw[q]);
            if (lane == 0) s_red[wv][q] = v;
        }
    } else if (lane < KPP_LMAX) {
        s_red[wv][lane] = 0ull;
    }
    __syncthreads();
    if (tid < L) {
        const unsigned long long v = s_red[0][tid] + s_red[1][tid] + s_red[2][tid] + s_red[3][tid];
        if (v) atomicAdd(&ctl->drep[blockIdx.x % KPP_DREP][tid], v);
    }
    DBG_E(7);
}

// Step c: select (first argmin of the candidates' potentials) and, unless this
// is the last centre, apply the new centre to the cells it reaches.
template <int D>
__global__ __launch_bounds__(256) void k_kpp_apply(const float *__restrict__ xs, const uint32_t *__restrict__ perm,
                                                   const uint32_t *__restrict__ cell_start, Grid g,
                                                   float *__restrict__ closest, float *__restrict__ crow,
                                                   float *__restrict__ cmax, unsigned long long *__restrict__ bsum,
                                                   const float *__restrict__ X, long long n,
                                                   int L, int s, int c, int apply, long long *__restrict__ indices,
                                                   KppCtl *__restrict__ ctl) {
    __shared__ unsigned s_g;
    __shared__ unsigned long long s_w[4];
    __shared__ unsigned long long s_del[KPP_LMAX];
    const int tid = threadIdx.x, lane = tid & 63;
    const unsigned long long pot = ctl->pot[c & 1];
    if (tid < L) {   // candidate tid's potential drop: the sum of the replicas
        unsigned long long v[KPP_DREP];
#pragma unroll
        for (int r = 0; r < KPP_DREP; ++r) v[r] = ctl->drep[r][tid];
        unsigned long long sum = 0ull;
#pragma unroll
        for (int r = 0; r < KPP_DREP; ++r) sum += v[r];
        s_del[tid] = sum;
    }
    const float gmax = kpp_gmax(ctl, &s_g);   // (its barrier publishes s_del)
    int bl = 0;
    unsigned long long bp = pot - s_del[0];
    for (int q = 1; q < L; ++q) {
        const unsigned long long v = pot - s_del[q];
        if (v < bp) { bp = v; bl = q; }   // first argmin (np.argmin)
    }
    const float4 best = ctl->cand[bl];
    if (blockIdx.x == 0 && tid == 0) {
        indices[c] = ctl->cand_idx[bl];
        ctl->pot[(c + 1) & 1] = bp;
    }
    if (!apply) return;
    int i0[MAXD], i1[MAXD];
    long long vol;
    kpp_cube<D>(g, best, gmax, i0, i1, vol);
    // Dense step (the cube covers >= 7/8 of the grid: the first ~10-20
    // centres): the caller-order copy `crow` and the block sums are rebuilt by a
    // streaming pass over the caller's rows at the end of this launch instead
    // of one random 4-B write and one random atomic per updated point (every
    // point outside the cube keeps its value: its distance exceeds gmax).
    const bool dense = 8 * vol >= 7 * g.ncells;
    const long long wid = (blockIdx.x * (long long)blockDim.x + tid) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    // this wave's cube cells wid, wid + nw, ...: reach tests one per lane (one
    // memory latency for up to 64), then the reached cells one after another
    const long long ipw = vol > wid ? (vol - wid + nw - 1) / nw : 0;
    for (long long k0 = 0; k0 < ipw; k0 += 64) {
        const long long itl = wid + (k0 + lane) * nw;
        long long celll = 0;
        bool reach = false;
        uint32_t cbl = 0u, cel = 0u;
        if (k0 + lane < ipw) {
            int f[MAXD];
            celll = kpp_cube_cell<D>(g, i0, i1, (unsigned)itl, f);
            const float cm = cmax[celll];
            cbl = cell_start[celll];
            cel = cell_start[celll + 1];
            reach = kpp_reaches_f<D>(g, f, best, cm);
        }
        unsigned long long bits = __ballot(reach);
        if (lane == 0) {
            DBG_KPP(c, 2, (unsigned)min(64LL, ipw - k0));
            DBG_KPP(c, 3, __popcll(bits));
        }
        while (bits) {
            const int src = __builtin_ctzll(bits);
            bits &= bits - 1ull;
            const long long cell = (long long)__shfl((int)celll, src);   // cell ids < 2^31 (kpp grid <= 2^20 cells)
            const uint32_t b = (uint32_t)__shfl((int)cbl, src), e = (uint32_t)__shfl((int)cel, src);
            float mx = 0.f;
            if (dense) {   // (block-uniform) rows are rebuilt below
                kpp_cell_points<D, KPP_PPL>(xs, closest, b, e, lane, [&](uint32_t i, const float (&x)[D], float cl) {
                    const float d = dist_canon<D>(x, best);
                    if (d < cl) closest[i] = d;
                    mx = fmaxf(mx, fminf(d, cl));
                });
            } else {
                kpp_cell_points_rows<D, KPP_PPL>(xs, closest, perm, b, e, lane,
                                                 [&](uint32_t i, const float (&x)[D], float cl, uint32_t r) {
                    const float d = dist_canon<D>(x, best);
                    if (d < cl) {
                        closest[i] = d;
                        crow[r] = d;
                        atomicAdd(&bsum[r >> KPP_OB_LOG], ~(kpp_w(cl, s) - kpp_w(d, s)) + 1ull);   // -= (mod 2^64)
                    }
                    mx = fmaxf(mx, fminf(d, cl));
                });
            }
            mx = wave_max_f(mx);
            if (lane == 0) cmax[cell] = mx;
        }
    }
    if (!dense) return;
    // rows: crow[j] = min(crow[j], d(X_j, best)), bsum[b] = its block's weight sum
    const long long nb = (n + KPP_OB - 1) / KPP_OB;
    const int wv = tid >> 6;
    for (long long b = blockIdx.x; b < nb; b += gridDim.x) {
        unsigned long long acc = 0ull;
#pragma unroll 4
        for (int e = 0; e < KPP_OB / 256; ++e) {
            const long long j = b * KPP_OB + e * 256 + tid;
            if (j < n) {
                float x[D];
#pragma unroll
                for (int a = 0; a < D; ++a) x[a] = X[j * D + a];
                const float cl = crow[j];
                const float d = dist_canon<D>(x, best);
                const float m = d < cl ? d : cl;
                if (d < cl) crow[j] = d;
                acc += kpp_w(m, s);
            }
        }
        acc = wave_sum_u64(acc);
        if (lane == 0) s_w[wv] = acc;
        __syncthreads();
        if (tid == 0) bsum[b] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
        __syncthreads();
    }
}

}  // namespace pcm
