// pcm_kernels.hpp — gfx950 kernels of the multi-day point-cloud Lloyd engine.
//
// Hot path: per iteration
//   k_cand             exact candidate lists per grid cell (fp64 bisector bound)
//   k_lloyd1           nearest centroid over the cell's candidates + LDS-privatised
//                      fixed-point accumulation (replaces _k_means_lloyd.pyx:168-218)
//   k_label            final E-step: labels + inertia (_kmeans.py:736-750)
//   k_global           averaging / shift / convergence (_k_means_common.pyx:274-311,
//                      _kmeans.py:717-732)
// Layout (once per cloud): k_bbox*, the record sort of pcm_sort.hpp (cell
// order, AoSoA-4), k_cell_starts_xs, k_tiles.
//
// Canonical arithmetic (oracle/lloyd_ref.py): fp32 distance
// ((d0*d0 + d1*d1) + d2*d2) + d3*d3 with every op rounded (-ffp-contract=off),
// strict '<' scan in ascending centroid index, int64 fixed-point sums.
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pcm_debug.hpp"   // DBG_* phase stamps (debug builds only)

namespace pcm {

constexpr int MAXD = 4;
constexpr int CAPC = 512;          // coarse candidate capacity (12.5M shard: coarse lists p90 243, max > 256)
constexpr int CAPF = 64;           // fine candidate capacity
constexpr int MSLOT = 4;           // LDS-privatised slots per lane (nearest-to-centre ranks)
#ifndef PCM_TPB
#define PCM_TPB 128   // 128 measured 9% faster than 256 at 100M (two-wave barriers), 10% at 12.5M
#endif
constexpr int TPB = PCM_TPB;       // assign block size
#ifndef PCM_TILE_PTS
#define PCM_TILE_PTS (32 * PCM_TPB)
#endif
constexpr int TILE = PCM_TILE_PTS;  // max points per tile: <= 32 per lane, 64 per shared LDS word (see AccL)
static_assert(TILE <= 64 * (TPB >= 128 ? TPB / 2 : TPB), "an LDS word sums <= 64 points (int32-exact)");
constexpr uint32_t FULL = 0xFFFFFFFFu;
constexpr int TLCAP = 256;        // tile lists staged whole in k_lloyd1's LDS (slot-map path)
constexpr int TLMAX = 1024;       // tile-list capacity (longer lists: FULL); lists past TLCAP scan in LDS chunks
constexpr uint32_t TL_MIN = 16;   // crowded layouts: tiles of cells with longer lists (or FULL) get tile lists
constexpr int QBITS = 25;
// Pruning margins (see DESIGN.md "Exactness of pruning").
constexpr double PEPS = 7.62939453125e-06;   // 2^-17  >> 6 * 2^-24 (fp32 distance error)
constexpr double PTAU = 1e-36;               // >> fp32 underflow error of a distance
constexpr double DRIFT_SAFE = 1.0 + 6.103515625e-05;   // 1 + 2^-14 >= (1 + PEPS) * fp64 rounding slack

struct Grid {
    int d;
    int prune;
    int F;
    int pad_;
    int G[MAXD];
    int GC[MAXD];
    double lo[MAXD], w[MAXD], inv[MAXD], mg[MAXD], ext[MAXD];
    long long ncells, ncoarse;
};

// Device control block (one per engine).
constexpr int INERT_REP = 32;
struct Ctrl {
    uint32_t halt, done, iter, max_iter;
    uint32_t n_empty, resume, status, pad0;
    double tol;
    unsigned long long inert[4];    // exact inertia: 32-bit limbs of sum trunc(d * 2^s), [3] = overflow count
    unsigned long long neq_saved;   // stat words changed at a halted iteration (used on resume)
    unsigned long long last_changed;
    double last_shift;
    unsigned int ref_sel;           // candidate lists: which reference-centre buffer (cref[ref_sel]) they were built at
    double budget;                  // ... and the centre drift they tolerate (0: exact for the reference only)
    unsigned int rebuilds;          // candidate-list rebuilds of this fit (diagnostics)
    unsigned int pad1;
    // k_upd: arrival counter of its blocks (the last one reduces their records and
    // resets it) and the list work it hands to k_lists
    unsigned int u_arrive, pad3;
    unsigned int lists, pad2;       // k_lists: 0 nothing, 1 refresh the records, 2 rebuild the lists
    double lists_dl;                // the rebuilt lists' drift budget
    // Same-address device atomics serialise at the memory side (~12 ns each, MI355X_MICROARCH.md
    // "fanin") and hold back loads queued behind them, so bulk per-wave adds are spread instead:
    // k_label: exact-inertia limbs added per block into replica lines (folded by k_inert_fold)
    alignas(128) unsigned long long inert_rep[INERT_REP][16];
};

// Arrival of block blockIdx.x among gridDim.x on one counter: true for the last
// one.  Release: the block's prior loads and stores precede its arrival (the
// last block then takes an acquire fence).  Round 5 measured a two-level
// arrival (8 group counters, then one) at config 3: "centres + arrival" 6.2 ->
// 7.3 us per block, so the single counter stays (profiles/rd5_updlists_phases_c3.txt).
// k_updlists' arrival, issued early and read late: a relaxed agent-scope
// fetch-add by lane 0 of the calling wave (EXEC = lane 0, or no lane when `on`
// is 0) whose returned value stays in flight -- hipcc's waitcnt pass does not
// see the asm, and __syncthreads waits only on LDS -- until arrive_read's
// explicit vmcnt(0).  (The compiler's own atomic would be rewritten into a
// wave-aggregated form whose broadcast waits for the return on the spot.)
__device__ __forceinline__ unsigned arrive_issue(unsigned *p, unsigned long long on) {
    unsigned old = 0u;
    unsigned long long save;
    asm volatile(
        "s_mov_b64 %1, exec\n\t"
        "s_mov_b64 exec, %4\n\t"
        "global_atomic_add %0, %2, %3, off sc0\n\t"
        "s_mov_b64 exec, %1"
        : "+v"(old), "=&s"(save)
        : "v"(p), "v"(1u), "s"(on)
        : "memory");
    return old;
}
__device__ __forceinline__ unsigned arrive_read(unsigned v) {
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(v) : : "memory");
    return (unsigned)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ bool arrive_last(Ctrl *ctrl) {
    const unsigned p = __hip_atomic_fetch_add(&ctrl->u_arrive, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    return p == gridDim.x - 1u;
}

// Fixed-point exponents q_a (identical on every rank).
struct QExp {
    int q[MAXD];
};

// Control words are written by earlier kernels on the same stream; the kernel
// boundary orders them, so plain loads suffice.
__device__ __forceinline__ bool gated(const Ctrl *c) { return (c->halt | c->done) != 0u; }

// ------------------------------------------------------------------ helpers
template <int D>
__device__ __forceinline__ float dist_canon(const float (&x)[D], const float4 &c) {
    float a = x[0] - c.x;
    float acc = a * a;
    if (D > 1) { float b = x[1] - c.y; float s = b * b; acc = acc + s; }
    if (D > 2) { float b = x[2] - c.z; float s = b * b; acc = acc + s; }
    if (D > 3) { float b = x[3] - c.w; float s = b * b; acc = acc + s; }
    return acc;
}

__device__ __forceinline__ float comp(const float4 &c, int a) {
    return a == 0 ? c.x : a == 1 ? c.y : a == 2 ? c.z : c.w;
}

// Fixed-point coordinate: trunc(x * 2^q) (exact scaling, truncation toward 0).
__device__ __forceinline__ int fixed_i(float x, int q) { return (int)__builtin_ldexpf(x, q); }

__device__ __forceinline__ void decode(long long c, const int *G, int d, int *idx) {
    for (int a = d - 1; a >= 0; --a) {
        idx[a] = (int)(c % G[a]);
        c /= G[a];
    }
}

__device__ __forceinline__ long long encode(const int *idx, const int *G, int d) {
    long long c = 0;
    for (int a = 0; a < d; ++a) c = c * G[a] + idx[a];
    return c;
}

// fine-cell range [f0, f1] on every axis -> fp64 box containing every point binned there
template <int D>
__device__ __forceinline__ void cell_box(const Grid &g, const int *f0, const int *f1, double *blo, double *bhi) {
#pragma unroll
    for (int a = 0; a < D; ++a) {
        blo[a] = g.lo[a] + (double)f0[a] * g.w[a] - g.mg[a];
        bhi[a] = (f1[a] == g.G[a] - 1) ? g.lo[a] + g.ext[a] + g.mg[a]
                                       : g.lo[a] + (double)(f1[a] + 1) * g.w[a] + g.mg[a];
    }
}

template <int D>
__device__ __forceinline__ double maxdist(const double *blo, const double *bhi, const float4 &c) {
    double s = 0.0;
    for (int a = 0; a < D; ++a) {
        double ca = (double)comp(c, a);
        double l = blo[a] - ca, h = bhi[a] - ca;
        s += fmax(l * l, h * h);
    }
    return s;
}

// True iff every point of the box is provably (with margin PEPS/PTAU) strictly
// closer, in the canonical fp32 distance, to r than to c.  The objective
// (1-e)|x-c|^2 - (1+e)|x-r|^2 is separable and concave per axis, so its box
// minimum is the sum of per-axis endpoint minima.
//
// Drift budget dl > 0 (lists reused while every centre stays within dl of the
// reference position the list was built at): with |x-c| <= Mc and |x-r| <= Mr
// over the box, (1-e)(|x-c|-dl)^2 - (1+e)(|x-r|+dl)^2 >= S - 2 dl (1+e)(Mc+Mr)
// - 2 e dl^2, so S > tau + 2 dl (Mc+Mr) (1+e) + 2 dl^2 keeps c dominated by r
// for any moved centres c', r' (and forces |x-c| > 2 dl).  mr = Mr.
template <int D>
__device__ __forceinline__ bool prunable(const double *blo, const double *bhi, const float4 &c, const float4 &r,
                                         double dl = 0.0, double mr = 0.0) {
    const double em = 1.0 - PEPS, ep = 1.0 + PEPS;
    double s = 0.0;
    for (int a = 0; a < D; ++a) {
        double ca = (double)comp(c, a), ra = (double)comp(r, a);
        double cl = blo[a] - ca, ch = bhi[a] - ca, rl = blo[a] - ra, rh = bhi[a] - ra;
        double gl = em * (cl * cl) - ep * (rl * rl);
        double gh = em * (ch * ch) - ep * (rh * rh);
        s += fmin(gl, gh);
    }
    if (!(dl > 0.0)) return s > PTAU;
    const double mc = sqrt(maxdist<D>(blo, bhi, c));
    return s > PTAU + (2.0 * dl * (mc + mr) + 2.0 * dl * dl) * DRIFT_SAFE;
}

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<__half>(__half v) { return __half2float(v); }

// Up to 5 buffers of 64-bit words := 0 in one launch (pcm_fit_begin).
struct ZeroSpans {
    unsigned long long *p[5];
    long long n[5];
};
__global__ __launch_bounds__(256) void k_zero_spans(ZeroSpans z) {
    const long long st = (long long)gridDim.x * blockDim.x;
#pragma unroll
    for (int q = 0; q < 5; ++q)
        for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < z.n[q]; i += st) z.p[q][i] = 0ull;
}

// ------------------------------------------------------------------ layout
// Per-block min/max/maxabs (+ non-finite flag) of an AoS (n, D) array.
template <typename T, int D>
__global__ __launch_bounds__(256) void k_bbox_partial(const T *__restrict__ X, long long n, float *__restrict__ part,
                                                      unsigned *__restrict__ nonfinite) {
    float mn[D], mx[D];
    for (int a = 0; a < D; ++a) { mn[a] = __builtin_inff(); mx[a] = -__builtin_inff(); }
    bool bad = false;
    const long long st = (long long)gridDim.x * blockDim.x;
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    for (; i + 3 * st < n; i += 4 * st) {   // 4 rows' loads in flight per round
        float v[4][D];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int a = 0; a < D; ++a) v[u][a] = to_f<T>(X[(i + u * st) * D + a]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int a = 0; a < D; ++a) {
                bad |= !__builtin_isfinite(v[u][a]);
                mn[a] = fminf(mn[a], v[u][a]);
                mx[a] = fmaxf(mx[a], v[u][a]);
            }
    }
    for (; i < n; i += st) {
        for (int a = 0; a < D; ++a) {
            float v = to_f<T>(X[i * D + a]);
            bad |= !__builtin_isfinite(v);
            mn[a] = fminf(mn[a], v);
            mx[a] = fmaxf(mx[a], v);
        }
    }
    __shared__ float smn[D][256], smx[D][256];
    for (int a = 0; a < D; ++a) { smn[a][threadIdx.x] = mn[a]; smx[a][threadIdx.x] = mx[a]; }
    if (bad) atomicOr(nonfinite, 1u);
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s)
            for (int a = 0; a < D; ++a) {
                smn[a][threadIdx.x] = fminf(smn[a][threadIdx.x], smn[a][threadIdx.x + s]);
                smx[a][threadIdx.x] = fmaxf(smx[a][threadIdx.x], smx[a][threadIdx.x + s]);
            }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int a = 0; a < D; ++a) {
            part[(size_t)blockIdx.x * 2 * D + a] = smn[a][0];
            part[(size_t)blockIdx.x * 2 * D + D + a] = smx[a][0];
        }
}

template <int D>
__global__ __launch_bounds__(256) void k_bbox_final(const float *__restrict__ part, int nblk, double *__restrict__ out) {
    // out: lo[D], hi[D]; one block, strided per-thread pass then an LDS tree
    __shared__ float smn[D][256], smx[D][256];
    const int tid = threadIdx.x;
    for (int a = 0; a < D; ++a) {
        float mn = __builtin_inff(), mx = -__builtin_inff();
        for (int b = tid; b < nblk; b += 256) {
            mn = fminf(mn, part[(size_t)b * 2 * D + a]);
            mx = fmaxf(mx, part[(size_t)b * 2 * D + D + a]);
        }
        smn[a][tid] = mn;
        smx[a][tid] = mx;
    }
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (tid < st)
            for (int a = 0; a < D; ++a) {
                smn[a][tid] = fminf(smn[a][tid], smn[a][tid + st]);
                smx[a][tid] = fmaxf(smx[a][tid], smx[a][tid + st]);
            }
        __syncthreads();
    }
    if (tid == 0)
        for (int a = 0; a < D; ++a) {
            out[a] = smn[a][0];
            out[D + a] = smx[a][0];
        }
}

// Sort key of the Lloyd layout: the cell id << D | the sub-cell (bit D-1-a set
// when the point lies in the upper half of its cell along axis a), so that
// within a cell the points of one sub-cell are contiguous.  The half test uses
// the same fp64 cell coordinate as the binning (clamped cells: a point on the
// top face lands in the upper half); sub-cell boxes carry the binning margin on
// both sides of the split (k_lloyd1).  Crowded layouts (zlev > 0) instead append
// a Morton code of zlev bisections of the cell (level 1 = the sub-cell bits,
// then the next finer halves, axis 0 first within a level), so the tiles of a
// crowded cell are compact boxes (tile lists, k_tile_cand).
template <int D>
__device__ __forceinline__ uint32_t sort_key_f(const float (&x)[D], const Grid &g, int with_sub, int zlev) {
    int idx[MAXD];
    uint32_t sub = 0, fz[MAXD];
#pragma unroll
    for (int a = 0; a < D; ++a) {
        double t = ((double)x[a] - g.lo[a]) * g.inv[a];
        int v = (int)floor(t);
        v = v < 0 ? 0 : (v >= g.G[a] ? g.G[a] - 1 : v);
        idx[a] = v;
        const double fr = t - (double)v;
        sub = (sub << 1) | ((fr >= 0.5) ? 1u : 0u);
        fz[a] = 0u;
        if (zlev > 0) {
            const int top = (1 << zlev) - 1;
            int m = (int)floor(fr * (double)(1 << zlev));
            fz[a] = (uint32_t)(m < 0 ? 0 : (m > top ? top : m));
        }
    }
    const uint32_t cell = (uint32_t)encode(idx, g.G, D);
    if (zlev > 0) {
        uint32_t z = 0;
        for (int l = zlev - 1; l >= 0; --l)
#pragma unroll
            for (int a = 0; a < D; ++a) z = (z << 1) | ((fz[a] >> l) & 1u);
        return (cell << (D * zlev)) | z;
    }
    return with_sub ? (cell << D) | sub : cell;
}

// Point record carried through the layout sort (coordinates + caller row), so
// that the sort itself moves the points and no random row gather follows.
template <typename T, int D> struct PRec {
    T c[D];
    uint32_t row;
};

// cell_start[c] = sub_start[c << d], c in [0, ncells]
__global__ __launch_bounds__(256) void k_cell_from_sub(const uint32_t *__restrict__ sub_start, long long ncells, int d,
                                                       uint32_t *__restrict__ cell_start) {
    long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (c <= ncells) cell_start[c] = sub_start[c << d];
}

// Sorted point layout "AoSoA-4": the points in cell order, in groups of 4
// consecutive points stored coordinate-major -- [x0 x1 x2 x3][y0 .. y3][z0 .. z3]
// -- so one lane's 4 points arrive from b128 loads already paired for the
// packed (v_pk_*) distance arithmetic, with no register shuffling.
template <int D>
__device__ __forceinline__ long long xs_index(long long i, int a) {
    return ((i >> 2) * D + a) * 4 + (i & 3);
}

__global__ __launch_bounds__(256) void k_tile_counts(const uint32_t *__restrict__ start, long long ncells,
                                                     uint32_t *__restrict__ cnt, uint32_t cap) {
    long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (c >= ncells) return;
    uint32_t n = start[c + 1] - start[c];
    cnt[c] = (n + cap - 1) / cap;
}

// tile_off[nc] and the tile count (the scan is exclusive: add the last cell's count)
__global__ void k_tile_total(uint32_t *__restrict__ off, const uint32_t *__restrict__ cnt, long long ncells,
                             uint32_t *__restrict__ ntiles) {
    if (threadIdx.x != 0) return;
    const uint32_t t = off[ncells - 1] + cnt[ncells - 1];
    off[ncells] = t;
    *ntiles = t;
}

__global__ __launch_bounds__(256) void k_tile_write(const uint32_t *__restrict__ start, const uint32_t *__restrict__ off,
                                                    long long ncells, uint4 *__restrict__ tiles, uint32_t cap) {
    long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (c >= ncells) return;
    uint32_t s = start[c], e = start[c + 1];
    uint32_t n = e - s;
    if (n == 0) return;
    uint32_t nt = (n + cap - 1) / cap;
    uint32_t per = (n + nt - 1) / nt;
    uint32_t o = off[c];
    for (uint32_t t = 0; t < nt; ++t) {
        uint32_t a = s + t * per;
        uint32_t b = a + per < e ? a + per : e;
        tiles[o + t] = make_uint4((uint32_t)c, a, b, 0u);
    }
}

// Longest-list-first tile order (pcm_fit_begin): key = 0xffff - the list
// length of the tile's cell at the first lists (FULL: the longest), value = the
// tile; a stable radix sort, then the records gathered in that order.
__global__ __launch_bounds__(256) void k_tile_lpt_keys(const uint4 *__restrict__ tiles, const uint32_t *__restrict__ fc_cnt,
                                                       unsigned nt, uint32_t *__restrict__ key, uint32_t *__restrict__ idx) {
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (t >= nt) return;
    const uint32_t c = fc_cnt[tiles[t].x];
    key[t] = 0xffffu - (c == FULL ? 0xffffu : min(c, 0xfffeu));
    idx[t] = t;
}

__global__ __launch_bounds__(256) void k_tile_gather(const uint4 *__restrict__ tiles, const uint4 *__restrict__ tmeta,
                                                     const uint32_t *__restrict__ idx, unsigned nt,
                                                     uint4 *__restrict__ t2, uint4 *__restrict__ m2) {
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (t >= nt) return;
    const uint32_t j = idx[t];
    t2[t] = tiles[j];
    if (tmeta) m2[t] = tmeta[j];
}

// Compressed point stream (fp32, D = 3).  Inside one tile (one cell, <= TILE
// points) each axis spans a short range, so every coordinate's fp32 bit pattern
// is the tile's minimum pattern on that axis plus a small unsigned delta (the
// patterns of same-signed floats are ordered by magnitude).  When every axis is
// single-signed over the tile and the three delta widths sum to <= 64 bits, the
// tile's points are stored as 8-byte records d0 | d1 << w0 | d2 << (w0 + w1) in
// `xz` (lo and hi words, zword() below); k_lloyd1 then streams 8 instead of 12 bytes per point and
// rebuilds the EXACT fp32 values (lossless: labels and sums are unchanged).
// tmeta[t] = {min0, min1, min2, 1 << 31 | w0 | w1 << 8 | w2 << 16}, or .w = 0
// (raw tile: 12-B AoSoA-4 `xs`).  Uniform [0,1)^3 cloud with 32^3 cells: cells
// with an axis index >= 1 need <= 23 + 21 + 20 bits; ~91 % of the points.
__device__ __forceinline__ unsigned zwidth(unsigned span) { return span ? 32u - (unsigned)__clz(span) : 0u; }

// Word offset in `xz` of the lo word of point i (its hi word: + ZHI).  PCM_ZWAVE
// (default): blocks of 256 points, 1 KB of lo words then 1 KB of hi words, each
// group of 4 points' words 16 B at (i % 256) / 4 -- a wave's 64 lanes x 4 points
// load 2 x 1 KB of consecutive bytes (two b128 per lane, each instruction one
// contiguous run).  PCM_ZWAVE=0: [lo0..lo3][hi0..hi3] per group (32 B per lane:
// each b128 instruction reads every other 16 B).
#ifndef PCM_ZWAVE
#define PCM_ZWAVE 1
#endif
// Record fields: x = bits [0, w0), y = [w0, w0 + w1), z = the top w2 bits (x by
// a mask, y by one funnel shift of the two words, z by one shift of the high
// word: 7 VALU per point; z after y took two 64-bit shifts, ~11 VALU, and
// measured ~1.5 % slower per k_lloyd1 launch at config 3, profiles/rd4_ztop_ab.txt).
#if PCM_ZWAVE
constexpr unsigned ZHI = 256;
__host__ __device__ __forceinline__ size_t zword(size_t i) { return (i >> 8) * 512u + (i & 255u); }
#else
constexpr unsigned ZHI = 4;
__host__ __device__ __forceinline__ size_t zword(size_t i) { return (i >> 2) * 8u + (i & 3u); }
#endif

__global__ __launch_bounds__(256) void k_tile_compress(const float *__restrict__ xs, const uint4 *__restrict__ tiles,
                                                       const uint32_t *__restrict__ ntiles, uint4 *__restrict__ tmeta,
                                                       unsigned *__restrict__ xz, unsigned long long *__restrict__ zpts) {
    const unsigned t = blockIdx.x;
    if (t >= *ntiles) return;
    const uint4 tr = tiles[t];
    const unsigned start = tr.y, end = tr.z;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // the whole tile (<= TILE = 16 x 256 points) in registers: every load in
    // flight at once, one read of xs (a strided loop waited one latency per
    // round, twice: 505-530 us for 100M points).  Round 6: a thread takes whole
    // AoSoA-4 groups -- 4 consecutive points, three 16-B loads (x4, y4, z4) --
    // instead of one coordinate word per point and axis (4-B loads at a 12-B
    // lane stride), and writes a full group's records as two 16-B stores
    constexpr int GPT = TILE / 1024 + 1;   // groups per thread (a tile spans <= TILE / 4 + 1 groups)
    const unsigned g0 = start >> 2, g1 = (end + 3u) >> 2;
    const float4 *xs4 = reinterpret_cast<const float4 *>(xs);
    float4 q[GPT][3];
#pragma unroll
    for (int u = 0; u < GPT; ++u) {
        const unsigned gg = g0 + (unsigned)tid + 256u * u;
        if (gg < g1) {
#pragma unroll
            for (int a = 0; a < 3; ++a) q[u][a] = xs4[(size_t)gg * 3 + a];
        } else {
#pragma unroll
            for (int a = 0; a < 3; ++a) q[u][a] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    auto word = [&](int u, int a, int k) -> unsigned {
        const float4 &v = q[u][a];
        return __float_as_uint(k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w)));
    };
    unsigned mn[3] = {~0u, ~0u, ~0u}, mx[3] = {0u, 0u, 0u}, sor[3] = {0u, 0u, 0u}, sand[3] = {1u, 1u, 1u};
#pragma unroll
    for (int u = 0; u < GPT; ++u) {
        const unsigned gg = g0 + (unsigned)tid + 256u * u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned i = 4u * gg + (unsigned)k;
            if (gg >= g1 || i < start || i >= end) continue;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const unsigned b = word(u, a, k);
                mn[a] = min(mn[a], b);
                mx[a] = max(mx[a], b);
                sor[a] |= b >> 31;
                sand[a] &= b >> 31;
            }
        }
    }
    __shared__ unsigned smn[4][3], smx[4][3], sso[4][3], ssa[4][3];
    __shared__ uint4 meta;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        for (int o = 32; o > 0; o >>= 1) {
            mn[a] = min(mn[a], (unsigned)__shfl_xor((int)mn[a], o));
            mx[a] = max(mx[a], (unsigned)__shfl_xor((int)mx[a], o));
            sor[a] |= (unsigned)__shfl_xor((int)sor[a], o);
            sand[a] &= (unsigned)__shfl_xor((int)sand[a], o);
        }
        if (lane == 0) { smn[wv][a] = mn[a]; smx[wv][a] = mx[a]; sso[wv][a] = sor[a]; ssa[wv][a] = sand[a]; }
    }
    __syncthreads();
    if (tid == 0) {
        unsigned w[3], lo[3], total = 0;
        bool ok = true;
        for (int a = 0; a < 3; ++a) {
            unsigned m0 = ~0u, m1 = 0u, so = 0u, sa = 1u;
            for (int k = 0; k < 4; ++k) { m0 = min(m0, smn[k][a]); m1 = max(m1, smx[k][a]); so |= sso[k][a]; sa &= ssa[k][a]; }
            lo[a] = m0;
            w[a] = zwidth(m1 - m0);
            ok = ok && (so == sa) && w[a] <= 31u;
            total += w[a];
        }
        // the z field sits at the top of the 64-bit record (decoded by one shift of
        // the high word): at least 1 bit wide, so the shift stays below 32
        // (w0 + w1 <= 62: the extra bit always fits)
        if (w[2] == 0u) { w[2] = 1u; ++total; }
        ok = ok && total <= 64u;
        meta = make_uint4(lo[0], lo[1], lo[2], ok ? (0x80000000u | w[0] | (w[1] << 8) | (w[2] << 16)) : 0u);
        tmeta[t] = meta;
        if (ok) atomicAdd(zpts + (t % 32u) * 16u, (unsigned long long)(end - start));   // 32 replica lines
    }
    __syncthreads();
    const uint4 m = meta;
    if (!(m.w >> 31)) return;
    const unsigned w0 = m.w & 0xffu, w2 = (m.w >> 16) & 0xffu;
#pragma unroll
    for (int u = 0; u < GPT; ++u) {
        const unsigned gg = g0 + (unsigned)tid + 256u * u;
        if (gg >= g1) continue;
        unsigned lw[4], hw[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned long long d0 = word(u, 0, k) - m.x;
            const unsigned long long d1 = word(u, 1, k) - m.y;
            const unsigned long long d2 = word(u, 2, k) - m.z;
            const unsigned long long v = d0 | (d1 << w0) | (d2 << (64u - w2));
            lw[k] = (unsigned)v;
            hw[k] = (unsigned)(v >> 32);
        }
        const unsigned i0 = 4u * gg;
        const size_t zg = zword(i0);   // 4 consecutive words, 16-B aligned (i0 % 4 == 0, same 256-point block)
        if (i0 >= start && i0 + 4u <= end) {
            *reinterpret_cast<uint4 *>(xz + zg) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
            *reinterpret_cast<uint4 *>(xz + zg + ZHI) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
        } else {   // a group at the tile's edge: only this tile's points
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const unsigned i = i0 + (unsigned)k;
                if (i < start || i >= end) continue;
                xz[zg + k] = lw[k];
                xz[zg + k + ZHI] = hw[k];
            }
        }
    }
}

// ------------------------------------------------------------------ crowded cells: tile lists
// A uniform grid cannot follow tight clusters: a cell that holds a whole
// cluster holds its hundreds of centres too, its list overflows CAPF (FULL) and
// every point of it scans all K (a 16-cluster K = 4096 cloud: 20 ms per
// iteration, VALU-bound).  When the layout finds crowded cells (an occupancy
// sample, pcm_layout_build) it orders each cell's points by a Morton code of
// `zlev` further bisections (sort_key), so a tile -- a run of <= TILE points of
// one cell -- covers a compact piece of the cell; k_tile_box records each
// tile's exact point box, and before every assign launch k_tile_cand builds,
// for the tiles of FULL cells, a list over that box with the same exact
// dominance test as the cell lists (any box holding the points is valid).

// Occupancy sample: counts[cell of point i * stride] += 1, i < m; counts[ncells]
// := the largest count afterwards (k_umax).
template <typename T, int D>
__global__ __launch_bounds__(256) void k_zsample(const T *__restrict__ X, long long m, long long stride, Grid g,
                                                 uint32_t *__restrict__ counts) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= m) return;
    const long long p = i * stride;
    int idx[MAXD];
#pragma unroll
    for (int a = 0; a < D; ++a) {
        const double t = ((double)to_f<T>(X[p * D + a]) - g.lo[a]) * g.inv[a];
        int v = (int)floor(t);
        idx[a] = v < 0 ? 0 : (v >= g.G[a] ? g.G[a] - 1 : v);
    }
    atomicAdd(counts + encode(idx, g.G, D), 1u);
}

__global__ __launch_bounds__(256) void k_umax(const uint32_t *__restrict__ v, long long n, uint32_t *__restrict__ out) {
    uint32_t m = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        m = max(m, v[i]);
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    if ((threadIdx.x & 63) == 0 && m) atomicMax(out, m);
}

// Exact fp32 box of every tile's points: tbox[2t] = lower, tbox[2t + 1] = upper corner.
template <typename T, int D>
__global__ __launch_bounds__(256) void k_tile_box(const T *__restrict__ xs, const uint4 *__restrict__ tiles,
                                                  const uint32_t *__restrict__ ntiles, float4 *__restrict__ tbox) {
    const unsigned t = blockIdx.x;
    if (t >= *ntiles) return;
    const uint4 tr = tiles[t];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    float mn[D], mx[D];
#pragma unroll
    for (int a = 0; a < D; ++a) { mn[a] = __builtin_inff(); mx[a] = -__builtin_inff(); }
    for (unsigned i = tr.y + tid; i < tr.z; i += 256)
#pragma unroll
        for (int a = 0; a < D; ++a) {
            const float v = to_f<T>(xs[xs_index<D>(i, a)]);
            mn[a] = fminf(mn[a], v);
            mx[a] = fmaxf(mx[a], v);
        }
    __shared__ float smn[4][MAXD], smx[4][MAXD];
#pragma unroll
    for (int a = 0; a < D; ++a) {
        for (int o = 32; o > 0; o >>= 1) {
            mn[a] = fminf(mn[a], __shfl_xor(mn[a], o));
            mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], o));
        }
        if (lane == 0) { smn[wv][a] = mn[a]; smx[wv][a] = mx[a]; }
    }
    __syncthreads();
    if (tid == 0) {
        float lo[4] = {0.f, 0.f, 0.f, 0.f}, hi[4] = {0.f, 0.f, 0.f, 0.f};
        for (int a = 0; a < D; ++a) {
            lo[a] = fminf(fminf(smn[0][a], smn[1][a]), fminf(smn[2][a], smn[3][a]));
            hi[a] = fmaxf(fmaxf(smx[0][a], smx[1][a]), fmaxf(smx[2][a], smx[3][a]));
        }
        tbox[2 * (size_t)t] = make_float4(lo[0], lo[1], lo[2], lo[3]);
        tbox[2 * (size_t)t + 1] = make_float4(hi[0], hi[1], hi[2], hi[3]);
    }
}

// List of one tile of a crowded cell (list FULL or longer than TL_MIN) over its
// point box, at the current centres:
// reference r = a centre of least max distance to the box, then every centre
// not provably dominated by r (prunable), compacted in ascending centroid index
// (the strict-'<' scan keeps the lowest index on ties).  tl_cnt[t] = the length,
// or FULL when it is not shorter than the cell's list or exceeds CAPF.  Tiles of
// other cells are skipped (k_lloyd1 reads tl_cnt only for cells past TL_MIN).
template <int D>
__global__ __launch_bounds__(256) void k_tile_cand(const uint4 *__restrict__ tiles, const uint32_t *__restrict__ ntiles,
                                                   const uint32_t *__restrict__ fc_cnt, const float4 *__restrict__ tbox,
                                                   const float4 *__restrict__ C, int K, uint32_t *__restrict__ tl_cnt,
                                                   float4 *__restrict__ tl_rec, int32_t *__restrict__ tl_lab,
                                                   const Ctrl *__restrict__ ctrl, int gate) {
    const unsigned t = blockIdx.x;
    if (gate && gated(ctrl)) return;
    if (t >= *ntiles) return;
    const uint4 tr = tiles[t];
    const uint32_t cc = fc_cnt[tr.x];
    if (cc <= TL_MIN) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const float4 lo4 = tbox[2 * (size_t)t], hi4 = tbox[2 * (size_t)t + 1];
    double blo[MAXD], bhi[MAXD];
#pragma unroll
    for (int a = 0; a < D; ++a) { blo[a] = (double)comp(lo4, a); bhi[a] = (double)comp(hi4, a); }
    double best = __builtin_inf();
    int bj = 0;
    for (int j = tid; j < K; j += 256) {
        const double md = maxdist<D>(blo, bhi, C[j]);
        if (md < best) { best = md; bj = j; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double ob = __shfl_xor(best, o);
        const int oj = __shfl_xor(bj, o);
        if (ob < best || (ob == best && oj < bj)) { best = ob; bj = oj; }
    }
    __shared__ double s_b[4];
    __shared__ int s_j[4];
    __shared__ unsigned s_w[4];
    if (lane == 0) { s_b[wv] = best; s_j[wv] = bj; }
    __syncthreads();
    int rj = s_j[0];
    double rb = s_b[0];
    for (int w = 1; w < 4; ++w)
        if (s_b[w] < rb || (s_b[w] == rb && s_j[w] < rj)) { rb = s_b[w]; rj = s_j[w]; }
    const float4 r = C[rj];
    unsigned base = 0;
    for (int j0 = 0; j0 < K; j0 += 256) {
        const int j = j0 + tid;
        const bool keep = j < K && !prunable<D>(blo, bhi, C[j < K ? j : 0], r);
        const unsigned long long bal = __ballot(keep);
        if (lane == 0) s_w[wv] = (unsigned)__popcll(bal);
        __syncthreads();
        unsigned off = base, total = 0;
        for (int w = 0; w < 4; ++w) {
            off += (w < wv) ? s_w[w] : 0u;
            total += s_w[w];
        }
        const unsigned pos = off + (unsigned)__popcll(bal & ((1ull << lane) - 1ull));
        if (keep && pos < (unsigned)TLMAX) {
            tl_rec[(size_t)t * TLMAX + pos] = C[j];
            tl_lab[(size_t)t * TLMAX + pos] = j;
        }
        base += total;
        __syncthreads();   // s_w is rewritten by the next chunk
        if (base > (unsigned)TLMAX) break;   // block-uniform
    }
    // FULL: no shorter list than the cell's (the tile scans the cell list, or all K)
    if (tid == 0) tl_cnt[t] = (base <= (unsigned)TLMAX && base < cc) ? base : FULL;
}

// Tile-list summary: out[0] += tiles of cells past TL_MIN, out[1] += those with a
// tile list, out[2] += the lengths of those lists; out[3] += tile lists longer
// than TLCAP (k_lloyd1 scans them through LDS chunks), out[4] += all-K tiles (a
// FULL cell whose tile got no list either), out[5] = the longest tile list.
__global__ __launch_bounds__(256) void k_tile_list_stats(const uint4 *__restrict__ tiles,
                                                         const uint32_t *__restrict__ ntiles,
                                                         const uint32_t *__restrict__ fc_cnt,
                                                         const uint32_t *__restrict__ tl_cnt,
                                                         unsigned long long *__restrict__ out) {
    const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (t >= *ntiles) return;
    const uint32_t cc = fc_cnt[tiles[t].x];
    if (cc <= TL_MIN) return;
    atomicAdd(out, 1ull);
    const uint32_t c = tl_cnt[t];
    if (c != FULL) {
        atomicAdd(out + 1, 1ull);
        atomicAdd(out + 2, (unsigned long long)c);
        if (c > (uint32_t)TLCAP) atomicAdd(out + 3, 1ull);
        atomicMax(out + 5, (unsigned long long)c);
    } else if (cc == FULL) {
        atomicAdd(out + 4, 1ull);
    }
}

// ------------------------------------------------------------------ candidates
// Candidate lists of every fine cell, in one launch, without global-memory
// round trips inside the per-cell work.  Block (I, b) owns coarse cell I
// (F^D fine cells) and children [b*cpb, (b+1)*cpb):
//  1. coarse list (block-wide, into LDS): reference r = a centre minimising the
//     max distance to the coarse box (LDS atomic min of a packed key: any centre
//     is a valid reference, the choice only affects pruning power); every
//     centre not provably dominated by r is marked in an LDS bitmap, and one
//     wave compacts the bitmap in ascending centroid index.  More than CAPC
//     survivors -> all K (FULL parent);
//  2. one wave per child cell: reference = a parent candidate nearest the cell
//     centre (again an LDS atomic-min key), keep the parent candidates it does
//     not dominate, in ascending centroid order (the scan's tie rule); the count
//     goes to fc_cnt[cell] (FULL = more than CAPF, or pruning disabled).
// D = 4: a coarse cell has 4^4 = 256 fine cells and a longer coarse list
template <int D> constexpr int cand_capc() { return D >= 4 ? 1024 : CAPC; }
#ifndef PCM_CAND_TPB
#define PCM_CAND_TPB 512   // round-2 fused update at config 3: 25.7 vs 28.7 us (the pair passes are latency-bound)
#endif
constexpr int CAND_TPB = PCM_CAND_TPB;   // threads per candidate block (one child cell per wave at a time)
constexpr int CAND_KBITS = 4096;         // bitmap capacity (larger K: direct ballot compaction)
constexpr int CAND_CBW = 512;            // pair path: child bitmap words (4 KB)
constexpr int CAND_MAXCH = 64;           // pair path: children per block


// Wave-wide minimum through DPP (row_shr 1/2/4/8 scan, then row_bcast 15/31;
// lane 63 ends with the minimum).  The whole wave must be active.  Used only to
// pick pruning references, where any candidate is correct (callers clamp).
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    const int id = -1;   // 0xFFFFFFFF: the identity of unsigned min
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x111, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x112, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x114, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x118, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x142, 0xA, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x143, 0xC, 0xF, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// C: the K centres, in global memory (k_cand, k_lists, k_coarse).
// Coarse lists computed once per coarse cell (CoarseL, D = 4 layouts): k_coarse
// writes them (out); the blocks of the next level read them (in).
struct CoarseL {
    const uint32_t *in_cnt = nullptr;   // [ncoarse] list length or FULL
    const int32_t *in_idx = nullptr;    // [ncoarse][cand_capc] centroid ids, ascending
    uint32_t *out_cnt = nullptr;
    int32_t *out_idx = nullptr;
};
// FC: fine cells per axis of the block's cell.  FC = 4: a coarse cell (4^D
// children) whose list is computed from all K centres (or read from k_coarse);
// FC = 2: a mid cell (2^D children, D = 4 layouts) whose list REFINES its
// coarse parent's k_coarse list -- the same exact test against the mid box --
// so the fine lists prune ~2^D-times shorter lists than the coarse ones.
template <int D, int FC = 4, int TPB = CAND_TPB>
__device__ __forceinline__ void cand_body(const Grid &g, const float4 *C, int K, uint32_t *__restrict__ fc_cnt,
                                          float4 *__restrict__ fc_rec, int32_t *__restrict__ fc_lab, int BPC,
                                          double dl = 0.0, CoarseL cl = CoarseL{}) {
    static_assert(FC == 4 || FC == 2, "children per axis");
    constexpr int CAP = cand_capc<D>();
    constexpr int FS = FC == 4 ? 2 : 1;   // log2(FC)
    const long long I = blockIdx.x / BPC;
    const int bsub = blockIdx.x % BPC;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    __shared__ float4 prec[CAP];
    __shared__ int pidx[CAP];
    __shared__ int sidx[FC == 2 ? CAP : 1];   // refine: the coarse parent's list
    __shared__ unsigned long long kbits[CAND_KBITS / 64];
    __shared__ unsigned long long rkey;
    __shared__ uint32_t s_mp, s_np;
    __shared__ unsigned long long cbits[CAND_CBW];   // pair path: per-child keep bitmaps over the coarse list
    int ci[MAXD];
    long long Ipar = I;   // the coarse cell whose k_coarse list this block reads
    if (FC == 4) {
        decode(I, g.GC, D, ci);
    } else {
        int GM[MAXD], pc[MAXD];
        for (int a = 0; a < MAXD; ++a) GM[a] = a < D ? (g.G[a] + 1) / 2 : 1;
        decode(I, GM, D, ci);
        for (int a = 0; a < D; ++a) pc[a] = ci[a] / 2;
        Ipar = encode(pc, g.GC, D);
    }
    int nchild = 1;
    for (int a = 0; a < D; ++a) nchild *= FC;
    const int cpb = (nchild + BPC - 1) / BPC;
    const bool refine = FC == 2 && cl.in_cnt != nullptr;

    // ---- 1. this block's cell list
    if (cl.in_cnt && !refine) {   // computed by k_coarse for this iteration's centres
        for (int w = tid; w < CAND_CBW; w += TPB) cbits[w] = 0ull;
        if (tid == 0) s_mp = cl.in_cnt[I];
        __syncthreads();
        const uint32_t m0 = s_mp;
        if (m0 != FULL)
            for (uint32_t l = tid; l < m0; l += TPB) {
                const int j = cl.in_idx[(size_t)I * CAP + l];
                pidx[l] = j;
                prec[l] = C[j];
            }
    } else if (g.prune) {
        int f0[MAXD], f1[MAXD];
        for (int a = 0; a < D; ++a) {
            f0[a] = ci[a] * FC;
            f1[a] = min(f0[a] + FC, g.G[a]) - 1;
        }
        double blo[MAXD], bhi[MAXD];
        cell_box<D>(g, f0, f1, blo, bhi);
        // source candidates: every centre, or (refine) the coarse parent's list
        int nsrc = K;
        bool from_list = false;
        if (refine) {
            if (tid == 0) s_np = cl.in_cnt[Ipar];
            __syncthreads();
            const uint32_t m0 = s_np;
            if (m0 != FULL) {
                nsrc = (int)m0;
                from_list = true;
                for (int l = tid; l < nsrc; l += TPB) sidx[l] = cl.in_idx[(size_t)Ipar * CAP + l];
            }
        }
        auto src = [&](int p) -> int { return from_list ? sidx[p] : p; };
        const bool bitmap = nsrc <= CAND_KBITS;
        if (tid == 0) rkey = ~0ull;
        if (bitmap)
            for (int w = tid; w < CAND_KBITS / 64; w += TPB) kbits[w] = 0ull;
        for (int w = tid; w < CAND_CBW; w += TPB) cbits[w] = 0ull;
        __syncthreads();
        // reference key: fp32 bits of the max distance (any centre is a valid
        // reference; the key only ranks them) with the low 11 bits replaced by
        // j's wave-local rank -> per-wave DPP minimum, then one LDS atomic per wave
        uint32_t best = ~0u;
        int bjj = 0;
        for (int p = tid; p < nsrc; p += TPB) {
            const int j = src(p);
            const float m = (float)maxdist<D>(blo, bhi, C[j]);
            if (__float_as_uint(m) < best) { best = __float_as_uint(m); bjj = j; }
        }
        const uint32_t wbest = wave_min_u32(best);
        const unsigned long long bal = __ballot(best == wbest);
        if (lane == (int)(__ffsll((long long)bal) - 1)) atomicMin(&rkey, ((unsigned long long)wbest << 32) | (unsigned)bjj);
        __syncthreads();
        DBG_T(4);
        const float4 r = C[(int)min((unsigned long long)(K - 1), rkey & 0xFFFFFFFFull)];
        const double mr = dl > 0.0 ? sqrt(maxdist<D>(blo, bhi, r)) : 0.0;
        if (bitmap) {
            // a wave's 64 consecutive source positions fill one bitmap word: a
            // ballot and a plain store (no 64-way contended LDS atomic)
            for (int p0 = 0; p0 < nsrc; p0 += TPB) {
                const int p = p0 + tid;
                const bool keep = p < nsrc && !prunable<D>(blo, bhi, C[src(p < nsrc ? p : 0)], r, dl, mr);
                const unsigned long long bal = __ballot(keep);
                if (lane == 0 && p0 + wv * 64 < nsrc) kbits[(p0 >> 6) + wv] = bal;
            }
            __syncthreads();
            DBG_T(5);
            // ordered compaction (ascending source position = ascending centroid
            // index): word prefix counts by one wave-wide scan, then every wave
            // compacts the words w = wv (mod waves) in parallel
            __shared__ uint32_t wpre[CAND_KBITS / 64];
            const int nwk = (nsrc + 63) / 64;   // <= 64
            if (wv == 0) {
                const uint32_t c = lane < nwk ? (uint32_t)__popcll(kbits[lane]) : 0u;
                uint32_t x = c;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(x, o);
                    if (lane >= o) x += y;
                }
                wpre[lane] = x - c;
                if (lane == 63) s_mp = x <= (uint32_t)CAP ? x : FULL;
            }
            __syncthreads();
            for (int w = wv; w < nwk; w += TPB / 64) {
                const unsigned long long word = kbits[w];
                const uint32_t pos = wpre[w] + __popcll(word & ((1ull << lane) - 1ull));
                if (((word >> lane) & 1ull) && pos < (uint32_t)CAP) {
                    const int j = src(w * 64 + lane);
                    prec[pos] = C[j];
                    pidx[pos] = j;
                }
            }
        } else {
            // large K: ordered compaction by ballots (one barrier pair per TPB centres)
            __shared__ uint32_t wcnt[TPB / 64];
            uint32_t total = 0;
            for (int base = 0; base < nsrc; base += TPB) {
                const int p = base + tid;
                const int j = src(p < nsrc ? p : 0);
                const bool keep = p < nsrc && !prunable<D>(blo, bhi, C[j], r, dl, mr);
                const unsigned long long bal = __ballot(keep);
                if (lane == 0) wcnt[wv] = __popcll(bal);
                __syncthreads();
                uint32_t woff = 0;
                for (int w = 0; w < wv; ++w) woff += wcnt[w];
                const uint32_t pos = total + woff + __popcll(bal & ((1ull << lane) - 1ull));
                if (keep && pos < (uint32_t)CAP) {
                    prec[pos] = C[j];
                    pidx[pos] = j;
                }
                for (int w = 0; w < TPB / 64; ++w) total += wcnt[w];
                __syncthreads();
            }
            if (tid == 0) s_mp = total <= (uint32_t)CAP ? total : FULL;
        }
    } else if (tid == 0) {
        s_mp = FULL;
    }
    __syncthreads();
    uint32_t mp = s_mp;
    const bool pfull = (mp == FULL);
    if (cl.out_cnt) {   // k_coarse: publish the coarse list, no children
        if (tid == 0) cl.out_cnt[I] = mp;
        if (!pfull)
            for (uint32_t l = tid; l < mp; l += TPB) cl.out_idx[(size_t)I * CAP + l] = pidx[l];
        return;
    }
    if (pfull) mp = (uint32_t)K;
    DBG_T(1);
    DBG_V(8, mp);

    // ---- 2. children (FC per axis) of this block: c0 .. c1-1
    const int c0 = bsub * cpb, c1 = min(nchild, (bsub + 1) * cpb);
    const int nwc = (int)((mp + 63u) / 64u);   // bitmap words per child
    // pair path when each wave would otherwise walk >= 8 children one after the
    // other (100M: 64 children per block, 15 -> 9.6 us); with few children per
    // block (12.5M shard: 8) the wave path's two chains per wave are shorter
    // (mid blocks, FC = 2: 16 children over lists of tens to hundreds: the pair path too)
    if (!pfull && ((c1 - c0) >= 2 * TPB / 16 || FC == 2) && (c1 - c0) <= CAND_MAXCH &&
        (c1 - c0) * nwc <= CAND_CBW) {
        // Pair path: one thread per (child, coarse-list position) in three
        // block-wide passes -- (A) reference = a parent candidate nearest the
        // child's centre (LDS atomic min of the key of the wave path below),
        // (B) keep bits of the candidates that reference does not dominate,
        // (C) ordered compaction (ascending centroid index) by popcounts.  The
        // lists equal the wave path's; all pairs run in parallel instead of one
        // child per wave after another (100M: 15 -> ~2 us per block).
        const int nch = c1 - c0, npair = nch * (int)mp;
        const int dch = TPB / (int)mp, dlp = TPB % (int)mp;
        constexpr uint32_t LM = CAP > 256 ? 0x3FFu : 0xFFu;
        // (0) per-child cell id, fp64 box and centre, once per child
        __shared__ double s_blo[CAND_MAXCH][D], s_bhi[CAND_MAXCH][D];
        __shared__ float s_ctr[CAND_MAXCH][D];
        __shared__ long long s_cell[CAND_MAXCH];
        __shared__ float4 s_ref[CAND_MAXCH];   // the child's reference centre (pass A)
        __shared__ double s_mr[CAND_MAXCH];    // max distance from the child's box to it (drift budget > 0)
        for (int ch = tid; ch < nch; ch += TPB) {
            int f[MAXD];
            bool inside = true;
#pragma unroll
            for (int a = D - 1, t = c0 + ch; a >= 0; --a, t >>= FS) {
                f[a] = ci[a] * FC + (t & (FC - 1));
                inside &= f[a] < g.G[a];
            }
            double blo[MAXD], bhi[MAXD];
            cell_box<D>(g, f, f, blo, bhi);
#pragma unroll
            for (int a = 0; a < D; ++a) {
                s_blo[ch][a] = blo[a];
                s_bhi[ch][a] = bhi[a];
                s_ctr[ch][a] = (float)(0.5 * (blo[a] + bhi[a]));
            }
            s_cell[ch] = inside ? encode(f, g.G, D) : -1ll;
        }
        __syncthreads();
        DBG_T(10);
        // (A) reference per child: TPC threads per child scan its share of
        // the coarse list, then a min over the TPC lanes (shuffles, no atomics:
        // an LDS atomic per pair serialised ~25-way on the child's word)
        {
            int tpc = 64;
            while (tpc > 1 && tpc * nch > TPB) tpc >>= 1;
            const int ch = tid / tpc, sub = tid % tpc;
            uint32_t best = ~0u;
            if (ch < nch && s_cell[ch] >= 0)
                for (int l = sub; l < (int)mp; l += tpc) {
                    const float4 c = prec[l];
                    float dsum = 0.f;
#pragma unroll
                    for (int a = 0; a < D; ++a) {
                        const float dd = s_ctr[ch][a] - comp(c, a);
                        dsum += dd * dd;
                    }
                    const uint32_t key = (__float_as_uint(dsum) & ~LM) | (uint32_t)l;
                    best = key < best ? key : best;
                }
            for (int o = 1; o < tpc; o <<= 1) {
                const uint32_t ob = (uint32_t)__shfl_xor((int)best, o);
                best = ob < best ? ob : best;
            }
            if (ch < nch && sub == 0 && s_cell[ch] >= 0) {
                uint32_t bl = best & LM;
                if (bl >= mp) bl = 0;
                const float4 r = prec[bl];
                s_ref[ch] = r;
                if (dl > 0.0) {
                    double blo[MAXD], bhi[MAXD];
#pragma unroll
                    for (int a = 0; a < D; ++a) { blo[a] = s_blo[ch][a]; bhi[a] = s_bhi[ch][a]; }
                    s_mr[ch] = sqrt(maxdist<D>(blo, bhi, r));
                } else {
                    s_mr[ch] = 0.0;
                }
            }
        }
        __syncthreads();
        DBG_T(11);
        // (B) keep bits; the lanes of one (child, bitmap word) are contiguous in a
        // wave, so one ballot and one LDS atomic per segment
        {
            const int iters = (npair + TPB - 1) / TPB;
            int ch = tid / (int)mp, l = tid % (int)mp;
            for (int it = 0, p = tid; it < iters; ++it, p += TPB) {
                bool keep = false;
                const bool valid = p < npair && s_cell[ch < nch ? ch : 0] >= 0 && ch < nch;
                if (valid) {
                    double blo[MAXD], bhi[MAXD];
#pragma unroll
                    for (int a = 0; a < D; ++a) { blo[a] = s_blo[ch][a]; bhi[a] = s_bhi[ch][a]; }
                    keep = !prunable<D>(blo, bhi, prec[l], s_ref[ch], dl, s_mr[ch]);
                }
                const unsigned long long bal = __ballot(keep);
                const int k = min(lane, l & 63);   // lanes before this one in its segment
                if (valid && k == 0) {
                    const int len = min(64 - lane, min(64 - (l & 63), (int)mp - l));
                    const unsigned long long seg = (bal >> lane) & (len >= 64 ? ~0ull : ((1ull << len) - 1ull));
                    if (seg) atomicOr(&cbits[ch * nwc + (l >> 6)], seg << (l & 63));
                }
                l += dlp;
                ch += dch;
                if (l >= (int)mp) { l -= (int)mp; ++ch; }
            }
        }
        __syncthreads();
        DBG_T(12);
        // (C)
        for (int p = tid, ch = tid / (int)mp, l = tid % (int)mp; p < npair; p += TPB) {
            const long long cell = s_cell[ch];
            if (cell >= 0) {
                const unsigned long long *wb = cbits + ch * nwc;
                const unsigned long long word = wb[l >> 6];
                uint32_t before = 0;
                for (int w = 0; w < (l >> 6); ++w) before += __popcll(wb[w]);
                if ((word >> (l & 63)) & 1ull) {
                    const uint32_t pos = before + __popcll(word & ((1ull << (l & 63)) - 1ull));
                    if (pos < (uint32_t)CAPF) {
                        fc_rec[cell * CAPF + pos] = prec[l];
                        fc_lab[cell * CAPF + pos] = pidx[l];
                    }
                }
                if (l == 0) {
                    uint32_t total = 0;
                    for (int w = 0; w < nwc; ++w) total += __popcll(wb[w]);
                    fc_cnt[cell] = total <= (uint32_t)CAPF ? total : FULL;
                }
            }
            l += dlp;
            ch += dch;
            if (l >= (int)mp) { l -= (int)mp; ++ch; }
        }
        DBG_T(2);
        return;
    }
    // wave path (FULL parent, or more pairs than the LDS bitmaps hold): one wave per child cell
    auto child = [&](auto PFc) {
        constexpr bool PF = decltype(PFc)::value;
        for (int ch = c0 + wv; ch < c1; ch += TPB / 64) {
            int f[MAXD];
            bool inside = true;
#pragma unroll
            for (int a = D - 1, t = ch; a >= 0; --a, t >>= FS) {
                f[a] = ci[a] * FC + (t & (FC - 1));
                inside &= f[a] < g.G[a];
            }
            if (!inside) continue;   // wave-uniform
            const long long cell = encode(f, g.G, D);
            if (!g.prune) {
                if (lane == 0) fc_cnt[cell] = FULL;
                continue;
            }
            double blo[MAXD], bhi[MAXD];
            cell_box<D>(g, f, f, blo, bhi);
            float ctr[MAXD];
#pragma unroll
            for (int a = 0; a < D; ++a) ctr[a] = (float)(0.5 * (blo[a] + bhi[a]));
            // reference: a parent candidate nearest the centre
            int bl;
            if constexpr (PF) {   // exact wave argmin (K may exceed a packed key's index field)
                float bd = __builtin_inff();
                bl = 0x7fffffff;
                for (uint32_t l = lane; l < mp; l += 64) {
                    const float4 c = C[l];
                    float dsum = 0.f;
#pragma unroll
                    for (int a = 0; a < D; ++a) {
                        const float dd = ctr[a] - comp(c, a);
                        dsum += dd * dd;
                    }
                    if (dsum < bd) { bd = dsum; bl = (int)l; }
                }
                for (int sft = 32; sft > 0; sft >>= 1) {
                    const float ob = __shfl_xor(bd, sft);
                    const int ol = __shfl_xor(bl, sft);
                    if (ob < bd || (ob == bd && ol < bl)) { bd = ob; bl = ol; }
                }
            } else {   // key = distance bits (low bits dropped) | list position (< CAP)
                uint32_t best = ~0u;
                for (uint32_t l = lane; l < mp; l += 64) {
                    const float4 c = prec[l];
                    float dsum = 0.f;
#pragma unroll
                    for (int a = 0; a < D; ++a) {
                        const float dd = ctr[a] - comp(c, a);
                        dsum += dd * dd;
                    }
                    const uint32_t key = (__float_as_uint(dsum) & (CAP > 256 ? 0xFFFFFC00u : 0xFFFFFF00u)) | l;
                    best = key < best ? key : best;
                }
                bl = (int)(wave_min_u32(best) & (CAP > 256 ? 0x3FFu : 0xFFu));
                if (bl >= (int)mp) bl = 0;
            }
            const float4 r = PF ? C[bl] : prec[bl];
            const double mr = dl > 0.0 ? sqrt(maxdist<D>(blo, bhi, r)) : 0.0;
            uint32_t total = 0;
            for (uint32_t base = 0; base < mp; base += 64) {
                const uint32_t l = base + lane;
                const bool in = l < mp;
                const uint32_t lc = in ? l : (uint32_t)bl;
                const float4 c = PF ? C[lc] : prec[lc];
                const int j = PF ? (int)lc : pidx[lc];
                const bool keep = in && !prunable<D>(blo, bhi, c, r, dl, mr);
                const unsigned long long bal = __ballot(keep);
                const uint32_t pos = total + __popcll(bal & ((1ull << lane) - 1ull));
                if (keep && pos < (uint32_t)CAPF) {
                    fc_rec[cell * CAPF + pos] = c;
                    fc_lab[cell * CAPF + pos] = j;
                }
                total += __popcll(bal);
            }
            if (lane == 0) fc_cnt[cell] = total <= (uint32_t)CAPF ? total : FULL;
        }
    };
    if (pfull) child(std::integral_constant<bool, true>{});
    else child(std::integral_constant<bool, false>{});
    DBG_T(2);
}

// Standalone candidate lists, exact for the current centres C (drift budget 0;
// fit start, relocation resume, final E-step): the reference
// buffer cref[ctrl->ref_sel] := C so that k_upd measures drift from C.
template <int D, int FC = 4>
__global__ __launch_bounds__(CAND_TPB) void k_cand(Grid g, const float4 *__restrict__ C, int K,
                                              uint32_t *__restrict__ fc_cnt, float4 *__restrict__ fc_rec,
                                              int32_t *__restrict__ fc_lab, Ctrl *__restrict__ ctrl, int gate,
                                              int bpc, float4 *__restrict__ cref, CoarseL cl) {
    if (gate && gated(ctrl)) return;
    float4 *ref = cref + (size_t)ctrl->ref_sel * K;
    for (long long j = blockIdx.x * (long long)CAND_TPB + threadIdx.x; j < K; j += (long long)gridDim.x * CAND_TPB)
        ref[j] = C[j];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctrl->budget = 0.0;
        if (gate) ctrl->rebuilds += 1u;   // lists rebuilt at a relocation resume
    }
    cand_body<D, FC>(g, C, K, fc_cnt, fc_rec, fc_lab, bpc, 0.0, cl);
}

// Coarse lists only (one block per coarse cell), for the child blocks of
// k_cand / k_lists to read.  C: the centres the lists are for; lists: gate on
// the k_lists work flag (the iteration path) or 0 (k_cand's callers).
template <int D>
__global__ __launch_bounds__(CAND_TPB) void k_coarse(Grid g, const float4 *__restrict__ C, int K,
                                                const Ctrl *__restrict__ ctrl, int lists, uint32_t *__restrict__ cl_cnt,
                                                int32_t *__restrict__ cl_idx) {
    double dl = 0.0;
    if (lists) {
        unsigned halt = ctrl->halt;
        unsigned mode = ctrl->lists;
        dl = ctrl->lists_dl;
        asm volatile("" : "+s"(halt), "+s"(mode), "+s"(dl));
        if (halt != 0u || mode != 2u) return;   // only a rebuild needs coarse lists
    }
    CoarseL cl;
    cl.out_cnt = cl_cnt;
    cl.out_idx = cl_idx;
    cand_body<D>(g, C, K, nullptr, nullptr, nullptr, 1, dl, cl);
}

// Candidate records refreshed to the new centres (lists still valid under the
// drift budget): every fine cell's records, grid-stride over the cells with 16
// threads per cell, every load of a cell's count and ids issued in parallel.
template <int D, int TPB = CAND_TPB>
__device__ __forceinline__ void refresh_body(const Grid &g, const float4 *cn, const uint32_t *__restrict__ fc_cnt,
                                             float4 *__restrict__ fc_rec, const int32_t *__restrict__ fc_lab,
                                             unsigned nblk = 0u) {   // list blocks (0: gridDim.x)
    constexpr int PER = 16, CPB = TPB / PER;   // threads per cell, cells per block pass
    const int sub = (int)threadIdx.x % PER;
    const unsigned nb = nblk ? nblk : gridDim.x;
    for (long long cell = (long long)blockIdx.x * CPB + (int)threadIdx.x / PER; cell < g.ncells;
         cell += (long long)nb * CPB) {
        const uint32_t m = fc_cnt[cell];
        if (m == FULL) continue;
        for (uint32_t p = sub; p < m; p += PER) fc_rec[cell * CAPF + p] = cn[fc_lab[cell * CAPF + p]];
    }
}

// ------------------------------------------------------------------ assign
// Nearest of mm candidates for 4 points per lane: strict '<' in ascending
// candidate order, so the lowest index wins ties (_k_means_lloyd.pyx:205-213).
template <int D, typename P>
__device__ __forceinline__ void scan4(P rec, int mm, const float (&x)[4][D], float (&bd)[4], int (&bj)[4]) {
    {
        const float4 c = rec[0];
        for (int e = 0; e < 4; ++e) { bd[e] = dist_canon<D>(x[e], c); bj[e] = 0; }
    }
#pragma unroll 2
    for (int j = 1; j < mm; ++j) {
        const float4 c = rec[j];
        for (int e = 0; e < 4; ++e) {
            float dd = dist_canon<D>(x[e], c);
            bool lt = dd < bd[e];
            bd[e] = lt ? dd : bd[e];
            bj[e] = lt ? j : bj[e];
        }
    }
}

// Same scan over the list positions set in a wave-uniform mask (ascending, so
// the lowest index still wins ties); m has at least one bit set.
template <int D, typename P>
__device__ __forceinline__ void scan4_m(P rec, unsigned long long m, const float (&x)[4][D], float (&bd)[4],
                                        int (&bj)[4]) {
    {
        const int j = __builtin_ctzll(m);
        m &= m - 1ull;
        const float4 c = rec[j];
        for (int e = 0; e < 4; ++e) { bd[e] = dist_canon<D>(x[e], c); bj[e] = j; }
    }
    while (m) {
        const int j = __builtin_ctzll(m);
        m &= m - 1ull;
        const float4 c = rec[j];
        for (int e = 0; e < 4; ++e) {
            float dd = dist_canon<D>(x[e], c);
            bool lt = dd < bd[e];
            bd[e] = lt ? dd : bd[e];
            bj[e] = lt ? j : bj[e];
        }
    }
}

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ rsrc_t make_rsrc(const void *base, unsigned long long bytes) {
    const unsigned long long b = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    const unsigned nb = __builtin_amdgcn_readfirstlane((unsigned)(bytes > 0xffffffffull ? 0xffffffffull : bytes));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((unsigned long long)hi << 32) | lo), (short)0, (int)nb,
                                             0x00020000);
}

// Lane-local 4 consecutive points in the packed AoS layout ([npad][D] of T):
// 4*D*sizeof(T) bytes = NW 32-bit words, loaded as b128 pieces (+ a b64 tail).
template <typename T, int D> struct Raw {
    static constexpr int NW = 4 * D * (int)sizeof(T) / 4;
    unsigned w[NW];
};
template <typename LT> struct RawLab;
template <> struct RawLab<uint16_t> {
    u32x2 w;
};
template <> struct RawLab<int32_t> {
    u32x4 w;
};

// Cache policy of the point stream (0 = default; 2 = NT measured 22% slower:
// 349 vs 282 us per launch, and no gain in the other kernels).
#ifndef PCM_XLOAD_CPOL
#define PCM_XLOAD_CPOL 0
#endif

// off_pt = index of the lane's first point; one descriptor for the whole AoS array.
template <typename T, int D>
__device__ __forceinline__ void load_x(Raw<T, D> &r, rsrc_t rs, unsigned off_pt) {
    constexpr int NW = Raw<T, D>::NW;
    const unsigned boff = off_pt * (unsigned)(D * sizeof(T));
    for (int k = 0; k + 4 <= NW; k += 4) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, boff + 4u * k, 0, PCM_XLOAD_CPOL);
        r.w[k] = v[0]; r.w[k + 1] = v[1]; r.w[k + 2] = v[2]; r.w[k + 3] = v[3];
    }
    if (NW % 4 == 2) {
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, boff + 4u * (NW - 2), 0, PCM_XLOAD_CPOL);
        r.w[NW - 2] = v[0]; r.w[NW - 1] = v[1];
    }
}
#define LOAD_X(dst, off) load_x<T, D>(dst, rx, off)
// compressed item: 4 points' 8-B records, lo words then hi words (AoSoA-4)
// (templated so that k_lloyd1's other instances, which never call it, compile)
template <typename R>
__device__ __forceinline__ void load_z2(R &r, rsrc_t rA, unsigned off_pt) {
    static_assert(sizeof(r.w) >= 8 * sizeof(unsigned), "compressed items fill 8 words");
    // off_pt is a multiple of 4 (or the out-of-range 0x0ffffff0: offsets past any
    // buffer, zeros without memory traffic)
    const unsigned boff = off_pt >= 0x0ffffff0u ? 0xfffff000u : (unsigned)zword(off_pt) * 4u;
    const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rA, boff, 0, PCM_XLOAD_CPOL);
    const u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(rA, boff + 4u * ZHI, 0, PCM_XLOAD_CPOL);
    r.w[0] = v0[0]; r.w[1] = v0[1]; r.w[2] = v0[2]; r.w[3] = v0[3];
    r.w[4] = v1[0]; r.w[5] = v1[1]; r.w[6] = v1[2]; r.w[7] = v1[3];
}
// exact fp32 coordinates of a compressed item (k_tile_compress): base + delta bits
// (sh1 = w0, sh2 = 32 - w2)
template <typename R, int DD>
__device__ __forceinline__ void unpack_z(const R &r, float (&x)[4][DD], const uint4 &zm, unsigned sh1,
                                         unsigned sh2, unsigned m0, unsigned m1) {
    static_assert(DD == 3 && sizeof(r.w) >= 8 * sizeof(unsigned), "compressed tiles: fp32 D = 3");
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const unsigned lo = r.w[e], hi = r.w[4 + e];
        x[e][0] = __uint_as_float(zm.x + (lo & m0));
        x[e][1] = __uint_as_float(zm.y + (__builtin_amdgcn_alignbit(hi, lo, sh1) & m1));
        x[e][2] = __uint_as_float(zm.z + (hi >> sh2));
    }
}
// AoSoA-4 (xs_index): word a*4 + e holds coordinate a of the lane's point e
template <int D>
__device__ __forceinline__ void unpack_x(const Raw<float, D> &r, float (&x)[4][D]) {
    for (int e = 0; e < 4; ++e)
        for (int a = 0; a < D; ++a) x[e][a] = __uint_as_float(r.w[a * 4 + e]);
}
template <int D>
__device__ __forceinline__ void unpack_x(const Raw<__half, D> &r, float (&x)[4][D]) {
    for (int e = 0; e < 4; ++e)
        for (int a = 0; a < D; ++a) {
            const int k = a * 4 + e;
            const unsigned word = r.w[k >> 1];
            const unsigned short hb = (unsigned short)((k & 1) ? (word >> 16) : (word & 0xffffu));
            x[e][a] = __half2float(__ushort_as_half(hb));
        }
}
__device__ __forceinline__ void store_l4(rsrc_t rs, unsigned off, const int (&l)[4], const bool (&v)[4],
                                         RawLab<uint16_t> *) {
    if (v[0] & v[1] & v[2] & v[3]) {
        u32x2 w;
        w[0] = ((unsigned)l[0] & 0xffffu) | ((unsigned)l[1] << 16);
        w[1] = ((unsigned)l[2] & 0xffffu) | ((unsigned)l[3] << 16);
        __builtin_amdgcn_raw_buffer_store_b64(w, rs, off * 2u, 0, 0);
    } else {
        for (int e = 0; e < 4; ++e)
            if (v[e]) __builtin_amdgcn_raw_buffer_store_b16((unsigned short)l[e], rs, (off + e) * 2u, 0, 0);
    }
}
__device__ __forceinline__ void store_l4(rsrc_t rs, unsigned off, const int (&l)[4], const bool (&v)[4],
                                         RawLab<int32_t> *) {
    if (v[0] & v[1] & v[2] & v[3]) {
        u32x4 w;
        for (int e = 0; e < 4; ++e) w[e] = (unsigned)l[e];
        __builtin_amdgcn_raw_buffer_store_b128(w, rs, off * 4u, 0, 0);
    } else {
        for (int e = 0; e < 4; ++e)
            if (v[e]) __builtin_amdgcn_raw_buffer_store_b32((unsigned)l[e], rs, (off + e) * 4u, 0, 0);
    }
}

#ifndef PCM_LSLOT
#define PCM_LSLOT 16
#endif
constexpr int LSLOT = PCM_LSLOT;

// Lane-minor accumulator words shared by threads tid and tid + AW = TPB / 2 (different
// waves, so an instruction never hits one word twice): word (slot, a) of column
// c = tid & 127 at (slot*(D+1)+a)*128 + c -- a wave's ds_add_u32 hits 32 distinct
// banks per half-wave whatever the slots.  A word sums <= 2 x 32 points of
// |xq| < 2^25 per tile: < 2^31, exact in int32.
constexpr int AW = TPB >= 128 ? TPB / 2 : TPB;   // one wave per block: no sharing (same-instruction lanes must not collide)
template <int D, int LS = LSLOT> struct AccL {
    static constexpr int rows = (LS + 1) * (D + 1);   // + junk slot
    static constexpr int words = AW * rows;
    // crowded layouts launch k_lloyd1 with this much more dynamic LDS: int64
    // words of long tile lists' positions (LDS atomics, one global atomic per
    // word and tile at the end instead of one per point: contended global
    // atomics made a 16-cluster K = 4096 cloud L2-atomic-bound)
    static constexpr int gwords = TLCAP * (D + 1);
    static constexpr size_t bytes_crowded = ((size_t)words * 4 + 7) / 8 * 8 + (size_t)gwords * 8;
};

// XCD-aware block order (a speed choice only: every kernel using it is
// correct under any dispatch).  The dispatcher deals a grid's blocks round-robin
// over the 8 XCDs, each with its own L2, so by default neighbouring chunks or
// tiles -- which share the cache lines at their boundaries and often their
// cell's records -- run on different XCDs.  This maps the blocks one XCD
// receives (b % 8 labels them) onto one contiguous range of chunk ids, in
// dispatch order; bijective on [0, nb) for any nb.
__device__ __forceinline__ unsigned xcd_block(unsigned b, unsigned nb) {
    const unsigned q = nb >> 3, r = nb & 7u, x = b & 7u, k = b >> 3;
    return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + k;
}

struct LloydArgs {
    const void *xs;                 // packed AoS [npad][D] of T, cell order
    const unsigned *xz;             // compressed 8-B records (fp32 D = 3 tiles with tmeta .w bit 31), or null
    const uint4 *tmeta;             // per-tile compression record (k_tile_compress), or null
    long long npad;
    const uint4 *tiles;             // {cell, start, end, -}
    const uint32_t *fc_cnt;         // candidate count per cell (FULL: all K)
    const uint32_t *ntiles;         // device: tile count of the layout
    const float4 *fc_rec;
    const int32_t *fc_lab;
    const float4 *C;                // all centres (FULL cells)
    int K;
    int q[MAXD];
    unsigned long long *partials;   // accumulation target: + (iter & 1) * pstride
    long long pstride;              // K*(D+1): single-GPU parity halves; 0: the all-reduce buffer itself
    const Ctrl *ctrl;
    const uint32_t *sub_start;      // [(ncells << D) + 1] sub-cell starts (k_lloyd1's per-round candidate masks)
    int sub;                        // the layout is sorted by sub-cell (else sub_start is [ncells + 1])
    Grid g;
    const uint32_t *tl_cnt;         // crowded layouts: per-tile list length for tiles of FULL cells (or FULL), else null
    const float4 *tl_rec;           // [tile][TLCAP] records of the tile lists (k_tile_cand)
    const float4 *tbox;             // crowded layouts: [tile][2] exact point box (lo, hi), else null
    const int32_t *tl_lab;
    int xcd;                        // k_lloyd1 takes its tile through xcd_block
};

struct TileL {
    unsigned cell, start, end, base0;
    int mm, full, nr, pad_;
};

// t.w = the cell's candidate count (fc_cnt[t.x], or FULL)
__device__ __forceinline__ TileL make_tile(const uint4 &t, int K) {
    TileL h;
    h.cell = t.x;
    h.start = t.y;
    h.end = t.z;
    h.full = (t.w == FULL) ? 1 : 0;
    h.mm = h.full ? K : (int)t.w;
    h.base0 = h.start & ~3u;
    h.nr = (int)((h.end - h.base0 + 4 * TPB - 1) / (4 * TPB));
    h.pad_ = 0;
    return h;
}

// Exact, order-independent inertia: a point adds w = trunc(d * 2^s) (d the
// canonical fp32 distance; s from the global fixed-point exponents so that
// w < 2^64, see inertia_scale); per-thread 128-bit sums are split into three
// 32-bit limbs, which are summed with integer atomics.  The total is the same
// integer for any block order, grid size or number of ranks
// (oracle/lloyd_ref.py inertia_exact).
__device__ __forceinline__ void inert_add(unsigned long long &lo, unsigned long long &hi, unsigned &ovf, float d,
                                          int s) {
    const double v = __builtin_ldexp((double)d, s);
    unsigned long long w;
    if (v < 18446744073709551616.0) {
        w = (unsigned long long)v;   // truncation (d >= 0)
    } else {
        w = ~0ull;
        ++ovf;
    }
    lo += w;
    hi += (lo < w) ? 1ull : 0ull;
}

// Block-wide: the limbs of all threads summed, then one add per limb into the
// block's replica line out[blockIdx % INERT_REP][0..3] (k_inert_fold sums them).
__device__ __forceinline__ void inert_flush(unsigned long long lo, unsigned long long hi, unsigned ovf,
                                            unsigned long long *__restrict__ out) {
    __shared__ unsigned long long s_l[TPB / 64][4];
    unsigned long long l[4] = {lo & 0xffffffffull, lo >> 32, hi, (unsigned long long)ovf};
    const int wv = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        for (int o = 32; o > 0; o >>= 1) l[q] += __shfl_xor(l[q], o);
        if ((threadIdx.x & 63) == 0) s_l[wv][q] = l[q];
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned long long v = 0ull;
        for (int w = 0; w < TPB / 64; ++w) v += s_l[w][threadIdx.x];
        if (v) atomicAdd(out + (size_t)(blockIdx.x % INERT_REP) * 16 + threadIdx.x, v);
    }
}

// inert[0..3] += the replica sums; replicas := 0 (one 64-thread block)
__global__ void k_inert_fold(unsigned long long *__restrict__ rep, unsigned long long *__restrict__ inert) {
    const int q = threadIdx.x;
    if (q >= 4) return;
    unsigned long long v = 0ull;
    for (int r = 0; r < INERT_REP; ++r) {
        v += rep[r * 16 + q];
        rep[r * 16 + q] = 0ull;
    }
    inert[q] += v;
}

// E-step with the current centres writing labels (sorted order) and the
// inertia (final E-step of _kmeans.py:736-750, relocation keys).  Not gated.
// Same tiles and candidate lists as k_lloyd1 (blocks walk tiles b, b + G, ...;
// the engine launches one block per tile); 4 points per lane per round,
// the loads of the next round in flight while one is computed; compressed
// tiles read their 8-B records (round 4), like k_lloyd1.
template <typename T, int D, typename LT>
__global__ __launch_bounds__(TPB) void k_label(LloydArgs A, void *lab, unsigned long long *inert_out, int iscale) {
    __shared__ float4 crec[CAPF];
    __shared__ int32_t cid[CAPF];
    const int tid = threadIdx.x;
    const unsigned G = gridDim.x;
    const unsigned nt = *A.ntiles;
    const float4 *lrec = A.fc_rec;
    const int32_t *llab = A.fc_lab;
    const rsrc_t rx = make_rsrc(A.xs, (unsigned long long)A.npad * D * sizeof(T));
    const rsrc_t rl = make_rsrc(lab, (unsigned long long)A.npad * sizeof(LT));
    constexpr bool ZOK = sizeof(T) == 4 && D == 3;   // compressed tiles exist only for fp32 D = 3
    const rsrc_t rz = make_rsrc(A.xz ? (const void *)A.xz : A.xs,
                                A.xz ? (unsigned long long)(A.npad + 255) / 256 * 256 * 8 : 0ull);
    unsigned long long ilo = 0ull, ihi = 0ull;
    unsigned iovf = 0u;
    for (unsigned t = blockIdx.x; t < nt; t += G) {
        uint4 tr = A.tiles[t];
        tr.w = A.fc_cnt[tr.x];
        const float4 *trec = lrec + (size_t)tr.x * CAPF;
        const int32_t *tlab = llab + (size_t)tr.x * CAPF;
        const float4 *Cs = A.C;             // all-K / long-list scans read these records
        const int32_t *glab = nullptr;      // long tile list: position -> centroid index
        if (tr.w > TL_MIN && A.tl_cnt && A.tl_cnt[t] != FULL) {   // crowded cell: the tile's own list
            const uint32_t tc = A.tl_cnt[t];
            trec = A.tl_rec + (size_t)t * TLMAX;
            tlab = A.tl_lab + (size_t)t * TLMAX;
            tr.w = tc;
            if (tc > (uint32_t)CAPF) { Cs = trec; glab = tlab; }
        }
        TileL h = make_tile(tr, A.K);
        if (glab) { h.full = 1; h.mm = (int)tr.w; }
        // compressed tile (fp32 D = 3): its 8-B records, decoded exactly as in k_lloyd1
        uint4 zm = make_uint4(0u, 0u, 0u, 0u);
        if (ZOK && A.tmeta) zm = A.tmeta[t];
        __syncthreads();
        if (!h.full && tid < h.mm) {
            crec[tid] = trec[tid];
            cid[tid] = tlab[tid];
        }
        __syncthreads();
        // one instance per point format (block-uniform per tile), so each keeps a
        // constant load count per item for hipcc's waitcnt pass
        auto run = [&](auto ZCc) {
            constexpr bool ZC = decltype(ZCc)::value;
            const unsigned zw0 = zm.w & 0xffu, zw1 = (zm.w >> 8) & 0xffu, zw2 = (zm.w >> 16) & 0xffu;
            const unsigned zsh1 = zw0, zsh2 = 32u - zw2, zm0 = (1u << zw0) - 1u, zm1 = (1u << zw1) - 1u;
            auto ldx = [&](Raw<T, D> &dst, unsigned off) {
                if constexpr (ZC) load_z2(dst, rz, off);
                else load_x<T, D>(dst, rx, off);
            };
            Raw<T, D> cur, nxt;
            ldx(cur, h.base0 + 4u * tid);
            for (int r = 0; r < h.nr; ++r) {
                const unsigned i0 = h.base0 + (unsigned)r * 4u * TPB + 4u * tid;
                ldx(nxt, r + 1 < h.nr ? i0 + 4u * TPB : 0x0ffffff0u);
                float x[4][D];
                if constexpr (ZC) unpack_z(cur, x, zm, zsh1, zsh2, zm0, zm1);
                else unpack_x<D>(cur, x);
                float bd[4];
                int bj[4];
                if (h.full) scan4<D>(Cs, h.mm, x, bd, bj);
                else scan4<D>(crec, h.mm, x, bd, bj);
                int lbl[4];
                bool v[4];
                for (int e = 0; e < 4; ++e) {
                    lbl[e] = h.full ? (glab ? glab[bj[e]] : bj[e]) : cid[bj[e]];
                    v[e] = (i0 + e >= h.start) && (i0 + e < h.end);
                    if (v[e] && inert_out) inert_add(ilo, ihi, iovf, bd[e], iscale);
                }
                if (i0 < h.end) store_l4(rl, i0, lbl, v, (RawLab<LT> *)nullptr);
                cur = nxt;
            }
        };
        if constexpr (ZOK) {
            if (zm.w >> 31) run(std::true_type{});
            else run(std::false_type{});
        } else {
            run(std::false_type{});
        }
    }
    if (inert_out) inert_flush(ilo, ihi, iovf, inert_out);
}

// ------------------------------------------------------------------ Lloyd iteration
// One Lloyd iteration's E-step + accumulation (sklearn's lloyd_iter_chunked_dense
// with update_centers=True, _k_means_lloyd.pyx:23-165).  It streams ONLY the
// points (12 B/pt at fp32 D=3): no label array is read or written.  sklearn's
// strict-convergence test (labels equal, _kmeans.py:717-723) is replaced by
// "the raw integer statistics equal the previous iteration's" in k_global: equal
// labels give equal statistics, and equal statistics give equal centres, i.e.
// shift 0 <= tol, so sklearn stops at that same iteration either way (DESIGN.md
// "Convergence").
//
// Per tile (a run of one cell's points): the candidate list (ascending centroid
// index, so the strict-'<' scan keeps the lowest index on ties,
// _k_means_lloyd.pyx:205-213) in LDS; a winner's fixed-point coordinates and
// count are summed into LDS words of its lane slot (ds_add_u32, lane-minor:
// conflict-free), winners without a slot into int64 words; out-of-tile lanes of
// a partial round add into a junk slot (never read).
// Nearest of mm centres read through scalar loads (FULL tiles: the whole
// uniform centre array); same scan order and tie rule as scan4.
template <int D>
__device__ __forceinline__ void scan4_s(const float4 *__restrict__ C, int mm, const float (&x)[4][D], float (&bd)[4],
                                        int (&bj)[4]) {
    {
        const float4 c = C[0];
        for (int e = 0; e < 4; ++e) { bd[e] = dist_canon<D>(x[e], c); bj[e] = 0; }
    }
    for (int j = 1; j < mm; ++j) {
        const float4 c = C[j];
        for (int e = 0; e < 4; ++e) {
            float dd = dist_canon<D>(x[e], c);
            bool lt = dd < bd[e];
            bd[e] = lt ? dd : bd[e];
            bj[e] = lt ? j : bj[e];
        }
    }
}

#ifndef PCM_WPE
#define PCM_WPE 4
#endif
#ifndef PCM_WPE_FINE
#define PCM_WPE_FINE 7
#endif
#ifndef PCM_WPE_D4
#define PCM_WPE_D4 6
#endif
#ifndef PCM_D4_OVF_LDS
#define PCM_D4_OVF_LDS 0
#endif
// One Lloyd iteration's E-step + accumulation, ONE TILE PER BLOCK (the round-1
// persistent tile walk, removed in round 5, measured 211 vs 238 us at config 3).
// The block's start-up: the tile record, the candidate count and the first
// LSPEC list records (vector loads, speculative: the count is not known yet)
// and the first two work items' point loads are all issued before anything
// is waited for, so a block starts scanning one point-load latency after it
// starts (the tile record -> count -> records chain cost ~3.8 us per block,
// a quarter of its lifetime at config 3).  The list loads precede the point
// loads, so the in-order vmcnt wait for the first work item covers them.
constexpr int LSPEC = 16;   // list records loaded before the count is known
#ifndef PCM_MASK_MIN
#define PCM_MASK_MIN 2
#endif
constexpr int MASK_MIN = PCM_MASK_MIN;   // sub-cell masks for lists of at least this length
// Minimum waves per SIMD the compiler must fit (a VGPR budget): the fine-grid
// fp32 variant (LS = 8, no masks) fits 6 without spilling (70 VGPRs instead of
// 82 at 4: 10 -> 12 resident blocks per CU; config 3 assign 214.7 -> 209.8 us
// on one box, tools/wpe_sweep.sh -- across boxes the rocprof average moved
// only 212.5 -> 211.3 us: the kernel is memory-bound, residency was not the
// limit); the masked 16-slot variant spills at 6 (12.5M shard
// 42.0 -> 45.5 us) and D = 4 gains nothing, so they keep 4.  Round 5: once the
// D <= 3 overflow words left LDS (10.9 KB per block), the fine-grid variant at
// 7 waves (71 VGPRs, 94 SGPRs; 4 VGPRs spilled outside the rounds) measured
// 198.3-199.0 -> 195.0-196.3 us per launch at config 3 (events, one box,
// profiles/rd5_wpe7_ab.txt), so PCM_WPE_FINE is 7.  Likewise the D = 4
// 8-slot variant without its LDS overflow words (PCM_D4_OVF_LDS 0; positions
// past the slots go to global atomics) fits 6 waves at 74 VGPRs: config-5
// 62.5M shard assign 332.7 -> 308.8-312.2 us, 8-way slab ~195 -> ~188 us per
// rank (profiles/rd5_d4_wpe6_ab.txt), so PCM_WPE_D4 is 6.
// Work items of a compressed tile in flight while one is computed (raw tiles: 2).
#ifndef PCM_ZPF
#define PCM_ZPF 2
#endif
constexpr int ZPF = PCM_ZPF;
template <typename T, int D, int LS, bool MASK>
constexpr int lloyd1_wpe() {
    return (sizeof(T) == 4 && D <= 3 && LS < LSLOT && !MASK) ? (ZPF > 2 ? 5 : PCM_WPE_FINE)
                                                             : ((D == 4 && LS < LSLOT && !MASK) ? PCM_WPE_D4 : PCM_WPE);
}
// the crowded-layout instance (tile lists, LDS-chunked long lists) does not fit
// a 6-wave budget: 80 VGPRs spilled 6 to scratch (round 5), so it keeps 5
template <typename T, int D, int LS, bool MASK, bool CROWD>
constexpr int lloyd1_wpe_c() { return CROWD ? (lloyd1_wpe<T, D, LS, MASK>() > 5 ? 5 : lloyd1_wpe<T, D, LS, MASK>()) : lloyd1_wpe<T, D, LS, MASK>(); }

// CROWD: the crowded-layout instance (tile lists, long lists, AccL::gwords of
// dynamic LDS); the other instances compile without that code.
template <typename T, int D, int LS, bool MASK, bool CROWD = false>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(lloyd1_wpe_c<T, D, LS, MASK, CROWD>(), 8))) void k_lloyd1(
    LloydArgs A, const uint4 *__restrict__ tiles, const float4 *__restrict__ fc_rec, const int32_t *__restrict__ fc_lab,
    const float4 *__restrict__ Call, const uint32_t *__restrict__ fc_cnt, const float4 *__restrict__ tl_rec) {
    extern __shared__ __attribute__((aligned(16))) uint32_t acc[];   // [(LS+1)*(D+1)][AW]
    // crowded layouts stage tile lists of up to TLCAP records in LDS (the long
    // lists of clustered clouds scan from LDS instead of one scalar load per
    // candidate) and sum list positions >= LS into the block-shared int64 words
    // AccL::gwords (one global atomic per word and tile at the end, not one per point)
    constexpr int LCAP = CROWD ? TLCAP : CAPF;
    __shared__ float4 crec[LCAP];
    __shared__ int32_t cid[LCAP];
    // Lists longer than LS: the LS candidates nearest the tile's centre own the
    // lane slots (smap: list position -> slot; sid: slot -> centroid), the
    // rest sum into int64 words per list position -- LDS words (8 slots, D = 4)
    // or global atomics (12 / 16 slots, rare positions), AccL::gwords when
    // crowded.  Points mostly pick a candidate near their tile, so the lane
    // slots take nearly all of them whatever the list's length.
    // (D <= 3, 8 slots: lists past 8 are rare on the fine grids that take 8
    // slots, so their overflow goes to global atomics; dropping the 2 KB of LDS
    // words, 13.0 -> 10.9 KB per block, gave config 3's assign 203.6-204.3 ->
    // 199.3-199.6 us on one box, round 5, profiles/rd5_lds_ovf_ab.txt)
    constexpr bool kOvf = !CROWD && D >= 4 && PCM_D4_OVF_LDS;
    __shared__ unsigned long long ovf[kOvf ? CAPF * (D + 1) : 1];
    __shared__ uint16_t smap[LCAP];
    __shared__ float skey[LCAP];
    __shared__ int32_t sid[LS];
    const int tid = threadIdx.x;
    const unsigned t = A.xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    // the gate flags, the device tile count and the tile record are loaded
    // together (one memory latency, not three in a row): the tiles buffer holds
    // ntiles_cap >= gridDim.x records, so the record load is in bounds before
    // the count says whether this block has work
    uint4 tr = tiles[t];
    unsigned nt = *A.ntiles;
    unsigned gate = A.ctrl->halt | A.ctrl->done;
    constexpr bool ZOK = sizeof(T) == 4 && D == 3;   // compressed tiles exist only for fp32 D = 3
    uint4 zm = make_uint4(0u, 0u, 0u, 0u);
    if (ZOK && A.tmeta) zm = A.tmeta[t];
    asm volatile("" : "+s"(tr.x), "+s"(tr.y), "+s"(tr.z), "+s"(nt), "+s"(gate));   // keep the loads above the exits
    asm volatile("" : "+s"(zm.x), "+s"(zm.y), "+s"(zm.z), "+s"(zm.w));
    if (gate != 0u || t >= nt) return;
    DBG_L(0);
    DBG_LV(5, __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)));    // HW_REG_HW_ID, 32 bits
    DBG_LV(6, __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)));   // HW_REG_XCC_ID, 16 bits
    const unsigned cell = tr.x, start = tr.y, end = tr.z;
    float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f);
    int l0 = 0;
    if (tid < LSPEC) {
        r0 = fc_rec[(size_t)cell * CAPF + tid];
        l0 = fc_lab[(size_t)cell * CAPF + tid];
    }
    uint32_t cnt = fc_cnt[cell];
    DBG_LV(7, (unsigned long long)(cnt & 0xFFFFu) | ((unsigned long long)(end - start) << 16));
    // crowded cell (list FULL or past TL_MIN): the tile's own list when k_tile_cand built a shorter one
    // (lists past TLCAP and all-K scans go through LDS in chunks, below)
    const float4 *lrec = fc_rec + (size_t)cell * CAPF;
    const int32_t *llab = fc_lab + (size_t)cell * CAPF;
    bool tl = false;
    if (CROWD && cnt > TL_MIN) {
        const uint32_t tc = A.tl_cnt[t];
        if (tc != FULL) {
            cnt = tc;
            lrec = tl_rec + (size_t)t * TLMAX;
            llab = A.tl_lab + (size_t)t * TLMAX;
            tl = true;
        }
    }
    constexpr int NSUB = 1 << D;
    uint32_t ss[NSUB + 1];   // the cell's sub-cell starts (uniform: scalar loads)
#pragma unroll
    for (int o = 0; o <= NSUB; ++o) ss[o] = (MASK && A.sub) ? A.sub_start[((size_t)cell << D) + o] : 0u;
    const unsigned base0 = start & ~3u;
    const int nr = (int)((end - base0 + 4 * TPB - 1) / (4 * TPB));
    const rsrc_t rx = make_rsrc(A.xs, (unsigned long long)A.npad * D * sizeof(T));
    // compressed tile (k_tile_compress): 8-B records from xz, decoded exactly
    const bool zc = ZOK && (zm.w >> 31);
    const unsigned zw0 = zm.w & 0xffu, zw1 = (zm.w >> 8) & 0xffu, zw2 = (zm.w >> 16) & 0xffu;
    const unsigned zsh1 = zw0, zsh2 = 32u - zw2;
    const unsigned zm0 = (1u << zw0) - 1u, zm1 = (1u << zw1) - 1u;
    const unsigned bpp = zc ? 8u : (unsigned)(D * sizeof(T));
    const rsrc_t rA = make_rsrc(zc ? (const void *)A.xz : A.xs, (unsigned long long)(zc ? (A.npad + 255) / 256 * 256 : A.npad) * bpp);
    // lanes past the tile's end get the out-of-range offset: zeros, no memory traffic
    auto item_off = [&](int rr) -> unsigned {
        const unsigned o = base0 + (unsigned)rr * 4u * TPB + 4u * tid;
        return (rr < nr && o < end) ? o : 0x0ffffff0u;
    };
    __shared__ unsigned long long omask[NSUB];
    __shared__ uint32_t okey[NSUB];
    __shared__ unsigned long long rmask[TILE / (4 * TPB) + 1];   // rounds of one tile
    // The rest of the kernel, instantiated per point format: compressed tiles
    // (fp32 D = 3, 8-B records) issue 2 b128 loads per work item, raw tiles
    // D * sizeof(T) / 4 -- one constant load count per instance keeps hipcc's
    // waitcnt bookkeeping exact, and compressed items no longer issue a third,
    // out-of-range load just to match the raw path's count.
    auto body = [&](auto ZCc) {
    constexpr bool ZC = decltype(ZCc)::value;
    auto ldx = [&](Raw<T, D> &dst, unsigned off) {
        if constexpr (ZC) load_z2(dst, rA, off);
        else load_x<T, D>(dst, rx, off);
    };
    // work items r+1 .. r+PF in flight while item r is computed: a ring of PF+1
    // register sets (compile-time indices after unrolling)
    constexpr int PF = ZC ? ZPF : 2;
    Raw<T, D> xr[PF + 1];
#pragma unroll
    for (int k = 0; k < PF; ++k) ldx(xr[k], item_off(k));
    for (int e = tid; e < AccL<D, LS>::words; e += TPB) acc[e] = 0u;
    // long tile lists: block-shared int64 words per list position (AccL::gwords, crowded launches only)
    unsigned long long *const govf =
        reinterpret_cast<unsigned long long *>(acc + (AccL<D, LS>::words + 1) / 2 * 2);
    const bool full = (cnt == FULL);
    const int mm = (cnt == FULL) ? A.K : (int)cnt;
    // crowded: an all-K scan or a tile list longer than the LDS list: scanned in
    // LDS chunks (below), no list staging
    const bool chunked = CROWD && (full || mm > LCAP);
    // block-uniform: the list is longer than the lane slots (not an all-K scan)
    const bool use_map = !full && !chunked && mm > LS;
    // block-uniform: a winner can lack a lane slot only in an all-K scan or a
    // list longer than the slots (the per-round test below is skipped otherwise)
    const bool can_over = full || mm > LS;
    if (kOvf && use_map)
        for (int e = tid; e < mm * (D + 1); e += TPB) ovf[e] = 0ull;
    if (full || chunked) {
        if (tid < LS) sid[tid] = tid;
        // (crowded: positions >= LS of an all-K scan go to global atomics, as the 16-slot variant's)
    } else {
        if (tid < LSPEC && tid < mm) {
            int lab = l0;
            if (tl) {   // block-uniform: crowded cells only (r0/l0 hold the cell list)
                crec[tid] = lrec[tid];
                lab = llab[tid];
            } else {
                crec[tid] = r0;
            }
            cid[tid] = lab;
            if (!use_map) sid[tid] = lab;   // short list: position p owns lane slot p
        }
        for (int j = LSPEC + tid; j < mm; j += TPB) {   // long lists (rare at D <= 3)
            crec[j] = lrec[j];
            cid[j] = llab[j];
        }
        if (CROWD && use_map)
            for (int j = tid; j < mm * (D + 1); j += TPB) govf[j] = 0ull;
    }
    uint32_t *const myacc = acc + (tid & (AW - 1));
    unsigned long long *prep = A.partials + (size_t)(A.ctrl->iter & 1u) * A.pstride;
    __syncthreads();
    if constexpr (CROWD) {
        if (chunked) {   // block-uniform
            // Crowded tile with a list longer than TLCAP (up to TLMAX), or FULL (no
            // list: every centre): the candidates are staged through LDS in chunks
            // of TLCAP -- the scalar-load scan of a 64-KB centre array missed the
            // scalar cache every few candidates (~2 ms per 4096-point tile at
            // K = 4096) -- in ascending centroid index with the strict '<' of scan4
            // (ties: lowest index).  Winners sum into a direct-mapped LDS table of
            // int64 words (govf, TLCAP entries tagged with the centroid; a slot
            // taken by another centroid sends the point to global atomics), folded
            // into the statistics once at the end.
            constexpr uint32_t EMPTY = 0xFFFFFFFFu;
            __shared__ uint32_t htag[TLCAP];
            for (int h = tid; h < TLCAP; h += TPB) htag[h] = EMPTY;
            for (int e = tid; e < TLCAP * (D + 1); e += TPB) govf[e] = 0ull;
            const rsrc_t rxf = make_rsrc(A.xs, (unsigned long long)A.npad * D * sizeof(T));
            for (int r = 0; r < nr; ++r) {
                const unsigned rbase = base0 + (unsigned)r * 4u * TPB;
                const unsigned i0 = rbase + 4u * tid;
                const unsigned off = (i0 < end) ? i0 : 0x0ffffff0u;
                float x[4][D];
                if constexpr (ZOK) {
                    Raw<float, 3> raw;
                    if (zc) {
                        load_z2(raw, rA, off);
                        unpack_z(raw, x, zm, zsh1, zsh2, zm0, zm1);
                    } else {
                        load_x<float, 3>(raw, rxf, off);
                        unpack_x<3>(raw, x);
                    }
                } else {
                    Raw<T, D> raw;
                    load_x<T, D>(raw, rxf, off);
                    unpack_x<D>(raw, x);
                }
                float bd[4];
                int bj[4];
                for (int c0 = 0; c0 < mm; c0 += TLCAP) {
                    const int mc = min(TLCAP, mm - c0);
                    __syncthreads();   // the previous chunk has been scanned
                    if (full) {
                        for (int j = tid; j < mc; j += TPB) { crec[j] = Call[c0 + j]; cid[j] = c0 + j; }
                    } else {
                        for (int j = tid; j < mc; j += TPB) { crec[j] = lrec[c0 + j]; cid[j] = llab[c0 + j]; }
                    }
                    __syncthreads();
                    int j = 0;
                    if (c0 == 0) {
                        const float4 c = crec[0];
                        const int cj = cid[0];
                        for (int e = 0; e < 4; ++e) { bd[e] = dist_canon<D>(x[e], c); bj[e] = cj; }
                        j = 1;
                    }
                    for (; j < mc; ++j) {
                        const float4 c = crec[j];
                        const int cj = cid[j];
                        for (int e = 0; e < 4; ++e) {
                            const float dd = dist_canon<D>(x[e], c);
                            const bool lt = dd < bd[e];
                            bd[e] = lt ? dd : bd[e];
                            bj[e] = lt ? cj : bj[e];
                        }
                    }
                }
                for (int e = 0; e < 4; ++e) {
                    if (!((i0 + e >= start) && (i0 + e < end))) continue;
                    const uint32_t h = (uint32_t)bj[e] & (uint32_t)(TLCAP - 1);
                    const uint32_t old = atomicCAS(&htag[h], EMPTY, (uint32_t)bj[e]);
                    if (old == EMPTY || old == (uint32_t)bj[e]) {
                        unsigned long long *pp = govf + h * (D + 1);
                        for (int a = 0; a < D; ++a) atomicAdd(pp + a, (unsigned long long)(long long)fixed_i(x[e][a], A.q[a]));
                        atomicAdd(pp + D, 1ull);
                    } else {
                        unsigned long long *pp = prep + (size_t)bj[e] * (D + 1);
                        for (int a = 0; a < D; ++a)
                            atomicAdd(pp + a, (unsigned long long)(long long)fixed_i(x[e][a], A.q[a]));
                        atomicAdd(pp + D, 1ull);
                    }
                }
            }
            __syncthreads();
            for (int i = tid; i < TLCAP * (D + 1); i += TPB) {
                const uint32_t c = htag[i / (D + 1)];
                const unsigned long long w = govf[i];
                if (c != EMPTY && w) atomicAdd(prep + (size_t)c * (D + 1) + i % (D + 1), w);
            }
            return;
        }
    }
    if (use_map) {
        // rank the list by the fp32 squared distance of each candidate to the
        // tile's centre (ties by position): ranks < LS get the lane slots
        float ctr[D];
        if (CROWD && tl && A.tbox) {   // crowded tile: its exact point box
            const float4 blo = A.tbox[(size_t)t * 2], bhi = A.tbox[(size_t)t * 2 + 1];
#pragma unroll
            for (int a = 0; a < D; ++a) ctr[a] = 0.5f * (comp(blo, a) + comp(bhi, a));
        } else {   // the cell's centre
            int ci[MAXD];
            for (int a = D - 1, c = (int)cell; a >= 0; --a) {
                ci[a] = (int)((unsigned)c % (unsigned)A.g.G[a]);
                c = (int)((unsigned)c / (unsigned)A.g.G[a]);
            }
#pragma unroll
            for (int a = 0; a < D; ++a) ctr[a] = (float)(A.g.lo[a] + ((double)ci[a] + 0.5) * A.g.w[a]);
        }
        for (int j = tid; j < mm; j += TPB) skey[j] = dist_canon<D>(ctr, crec[j]);
        __syncthreads();
        for (int j = tid; j < mm; j += TPB) {
            const float kj = skey[j];
            int rank = 0;
            for (int q = 0; q < mm; ++q) {
                const float kq = skey[q];
                rank += (kq < kj || (kq == kj && q < j)) ? 1 : 0;
            }
            smap[j] = (uint16_t)(rank < LS ? rank : LS + j);
            if (rank < LS) sid[rank] = cid[j];
        }
        __syncthreads();
    }
    // Sub-cell candidate masks: for every half-cell box (one per axis
    // combination) the list positions its reference does not dominate (the
    // exact test of the candidate lists, at the current centres), then per
    // round the union over the sub-cells the round's points occupy.  Points are
    // sorted by sub-cell within the cell, so a round (512 points) spans one or
    // two sub-cells and scans ~the candidates of a cell half as wide; any
    // superset of the undominated candidates, scanned in ascending order, gives
    // the exact labels (a dominated candidate is strictly farther for every
    // point of the box, so every tied minimiser is kept).
    // only coarse grids (MASK: the 16-slot D <= 3 variant, lists of ~6 at a
    // 12.5M shard: 47.8 -> 43.5 us per launch); at config 3 (lists of ~2.7)
    // and D = 4 (16 sub-cells) the mask phase at the block's start cost more
    // than the shorter scans saved (217 -> 225 us, 415 -> 488 us)
    const bool use_mask = MASK && A.sub && !full && !tl && mm >= MASK_MIN && A.g.prune;
    if (use_mask) {
        int ci[MAXD];
        for (int a = D - 1, c = (int)cell; a >= 0; --a) {   // cell ids fit 32 bits (sort keys)
            ci[a] = (int)((unsigned)c % (unsigned)A.g.G[a]);
            c = (int)((unsigned)c / (unsigned)A.g.G[a]);
        }
        double cblo[MAXD], cbhi[MAXD], mid[MAXD];
        cell_box<D>(A.g, ci, ci, cblo, cbhi);
#pragma unroll
        for (int a = 0; a < D; ++a) mid[a] = A.g.lo[a] + ((double)ci[a] + 0.5) * A.g.w[a];
        auto sub_box = [&](int o, double *blo, double *bhi) {
#pragma unroll
            for (int a = 0; a < D; ++a) {
                const bool up = (o >> (D - 1 - a)) & 1;
                blo[a] = up ? mid[a] - A.g.mg[a] : cblo[a];
                bhi[a] = up ? cbhi[a] : mid[a] + A.g.mg[a];
            }
        };
        if (tid < NSUB) { okey[tid] = ~0u; omask[tid] = 0ull; }
        __syncthreads();
        // (sub-cell o, list position j) pairs: reference = a candidate nearest
        // the sub-cell's centre (LDS atomic min of the key of the candidate lists. children)
        const int np = NSUB * mm;
        for (int p = tid; p < np; p += TPB) {
            const int o = p / mm, j = p - o * mm;
            double blo[MAXD], bhi[MAXD];
            sub_box(o, blo, bhi);
            const float4 c = crec[j];
            float dsum = 0.f;
#pragma unroll
            for (int a = 0; a < D; ++a) {
                const float dd = (float)(0.5 * (blo[a] + bhi[a])) - comp(c, a);
                dsum += dd * dd;
            }
            atomicMin(&okey[o], (__float_as_uint(dsum) & ~0x3Fu) | (uint32_t)j);
        }
        __syncthreads();
        for (int p = tid; p < np; p += TPB) {
            const int o = p / mm, j = p - o * mm;
            double blo[MAXD], bhi[MAXD];
            sub_box(o, blo, bhi);
            uint32_t bl = okey[o] & 0x3Fu;
            if (bl >= (uint32_t)mm) bl = 0;
            if (!prunable<D>(blo, bhi, crec[j], crec[bl])) atomicOr(&omask[o], 1ull << j);
        }
        __syncthreads();
        if (tid < nr) {
            const unsigned rb = base0 + (unsigned)tid * 4u * TPB;
            const unsigned rbeg = rb > start ? rb : start;
            const unsigned rend = rb + 4u * TPB < end ? rb + 4u * TPB : end;
            unsigned long long m = 0ull;
#pragma unroll
            for (int o = 0; o < NSUB; ++o)
                if (ss[o] < rend && ss[o + 1] > rbeg) m |= omask[o];
            rmask[tid] = m;
        }
        __syncthreads();
    }
    DBG_L(1);

    // loads per work item; after item r+PF's are issued, items r+1 .. r+PF may
    // stay outstanding while r is computed
    constexpr int NL = ZC ? 2 : Raw<T, D>::NW / 4 + (Raw<T, D>::NW % 4 ? 1 : 0);
    constexpr int VM = PF * NL;
    constexpr int WAIT_PREV = 0x0F70 | (VM & 0xF) | ((VM >> 4) << 14);   // vmcnt(VM) expcnt(7) lgkmcnt(15)
    auto step = [&](Raw<T, D> &cx, Raw<T, D> &nx, int r) {
        ldx(nx, item_off(r + PF));
        if (r >= nr) {
            // padding step (nr not a multiple of 3): no compute, but the same
            // wait as a computing step, so that every path reaches the loop
            // latch with the same outstanding loads (a skipped step left the
            // waitcnt pass a pessimistic merge: vmcnt(0) before each prefetch)
            __builtin_amdgcn_s_waitcnt(WAIT_PREV);
            return;
        }
        const unsigned rbase = base0 + (unsigned)r * 4u * TPB;
        const unsigned i0 = rbase + 4u * tid;
        float x[4][D];
        if constexpr (ZC) unpack_z(cx, x, zm, zsh1, zsh2, zm0, zm1);
        else unpack_x<D>(cx, x);
        int bj[4];
        if (mm == 1) {
            for (int e = 0; e < 4; ++e) bj[e] = 0;
        } else if (use_mask) {
            const unsigned long long m0 = rmask[r];
            const unsigned long long m = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(m0 >> 32)) << 32) |
                                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)m0);
            if ((m & (m - 1ull)) == 0ull) {   // one candidate for the whole round
                const int j = m ? __builtin_ctzll(m) : 0;
                for (int e = 0; e < 4; ++e) bj[e] = j;
            } else {
                float bd[4];
                scan4_m<D>(crec, m, x, bd, bj);
            }
        } else {
            float bd[4];
            if (full) {
                scan4_s<D>(Call, mm, x, bd, bj);
            } else {
                scan4<D>(crec, mm, x, bd, bj);
            }
        }
        // block-uniform: every point of the round lies inside the tile
        const bool whole = (rbase >= start) && (rbase + 4u * TPB <= end);
        // slot of each point's winner: its lane slot (< LS), else LS + its list
        // position (use_map) or, in an all-K scan, LS + (centroid - LS)
        int sl[4], so[4];
        bool over = false;
        for (int e = 0; e < 4; ++e) {
            const bool v = whole || ((i0 + e >= start) && (i0 + e < end));
            const int sm = use_map ? (int)smap[bj[e]] : bj[e];
            const bool hi = sm >= LS;
            over |= v && hi;
            sl[e] = (v && !hi) ? sm : LS;
            so[e] = (v && hi) ? (use_map ? sm - LS : bj[e]) : -1;
        }
        for (int e = 0; e < 4; ++e) {
            uint32_t *ap = myacc + sl[e] * ((D + 1) * AW);
            for (int a = 0; a < D; ++a) atomicAdd(ap + a * AW, (uint32_t)fixed_i(x[e][a], A.q[a]));
            atomicAdd(ap + D * AW, 1u);
        }
        if (can_over && over) {   // winners without a lane slot (long lists only)
            for (int e = 0; e < 4; ++e) {
                const int o = so[e];   // list position (use_map) or centroid (all-K scan)
                if (o < 0) continue;
                // one address space per branch (a pointer select would make FLAT
                // atomics, which count in vmcnt and lgkmcnt and drain the prefetch)
                if (CROWD && !full) {   // crowded list: block-shared words, folded at the end
                    unsigned long long *pp = govf + o * (D + 1);
                    for (int a = 0; a < D; ++a) atomicAdd(pp + a, (unsigned long long)(long long)fixed_i(x[e][a], A.q[a]));
                    atomicAdd(pp + D, 1ull);
                } else if (full || !kOvf) {
                    unsigned long long *pp = prep + (size_t)(full ? o : cid[o]) * (D + 1);
                    for (int a = 0; a < D; ++a)
                        atomicAdd(pp + a, (unsigned long long)(long long)fixed_i(x[e][a], A.q[a]));
                    atomicAdd(pp + D, 1ull);
                } else {
                    unsigned long long *pp = ovf + o * (D + 1);
                    for (int a = 0; a < D; ++a) atomicAdd(pp + a, (unsigned long long)(long long)fixed_i(x[e][a], A.q[a]));
                    atomicAdd(pp + D, 1ull);
                }
            }
        }
    };
    // PF+1 rotating register sets; a tile spans at most TILE / (4 TPB) + 1 = 9 rounds
    for (int r = 0; r < nr; r += PF + 1) {
#pragma unroll
        for (int k = 0; k <= PF; ++k) step(xr[k], xr[(k + PF) % (PF + 1)], r + k);
    }
    DBG_L(2);
    // fold the slot words into the int64 statistics: 16 threads per (slot, a) row
    __syncthreads();
    {
        const int nslots = mm < LS ? mm : LS;
        const int npairs = nslots * (D + 1);
        for (int p0 = 0; p0 < npairs; p0 += TPB / 16) {
            const int pi = p0 + tid / 16, sub = tid & 15;
            long long sacc = 0;
            if (pi < npairs) {
                const bool isc = (pi % (D + 1) == D);
                const uint32_t *row = acc + pi * AW;
                for (int k = 0; k < AW / 16; ++k) {
                    const uint32_t w = row[sub + 16 * k];
                    sacc += isc ? (long long)w : (long long)(int32_t)w;
                }
            }
            sacc += __shfl_down(sacc, 8, 16);
            sacc += __shfl_down(sacc, 4, 16);
            sacc += __shfl_down(sacc, 2, 16);
            sacc += __shfl_down(sacc, 1, 16);
            if (pi < npairs && sub == 0 && sacc) {
                const int slot = pi / (D + 1), qq = pi % (D + 1);
                atomicAdd(prep + (size_t)sid[slot] * (D + 1) + qq, (unsigned long long)sacc);
            }
        }
        // the int64 words of the positions without a lane slot (use_map lists)
        if (CROWD && use_map)
            for (int i = tid; i < mm * (D + 1); i += TPB) {
                const unsigned long long w = govf[i];
                if (w) atomicAdd(prep + (size_t)cid[i / (D + 1)] * (D + 1) + i % (D + 1), w);
            }
        if (kOvf && use_map)
            for (int i = tid; i < mm * (D + 1); i += TPB) {
                const unsigned long long w = ovf[i];
                if (w) atomicAdd(prep + (size_t)cid[i / (D + 1)] * (D + 1) + i % (D + 1), w);
            }
    }
    DBG_L(3);
    };
    if constexpr (ZOK) {
        if (zc) body(std::true_type{});
        else body(std::false_type{});
    } else {
        body(std::false_type{});
    }
}

// Single block of 1024 threads.  Optionally first folds partials[parity] into
// `stats` (single-GPU path: no all-reduce in between).  Then
// reads the (all-reduced) statistics, halts for relocation when a cluster is
// empty (unless resuming), otherwise averages, computes the shift with the
// fixed reduction tree (per-thread sums over j = tid + 1024 r, then the halving
// tree 512..1, as oracle/lloyd_ref.py shift_total) and sets convergence flags.
template <int D>
__global__ __launch_bounds__(1024) void k_global(unsigned long long *__restrict__ partials,
                                                 unsigned long long *__restrict__ stats, int K, QExp qe,
                                                 unsigned long long *__restrict__ held,
                                                 unsigned long long *__restrict__ prev,
                                                 float4 *__restrict__ C, float4 *__restrict__ Cn,
                                                 unsigned long long *__restrict__ hist_changed,
                                                 double *__restrict__ hist_shift, Ctrl *__restrict__ ctrl) {
    if (gated(ctrl)) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int *q = qe.q;
    const int n = K * (D + 1);
    __shared__ unsigned cnt_empty;
    __shared__ unsigned long long neq_s;
    __shared__ unsigned long long wmax[16];
    __shared__ int warg[16];
    __shared__ double ssum[1024];
    if (tid == 0) { cnt_empty = 0; neq_s = 0ull; }
    __syncthreads();
    const uint32_t resume = ctrl->resume;
    // Thread tid owns centroids j = tid + 1024 r: every load of a row (and of
    // the previous statistics) is issued before any is consumed, so a pass
    // costs one memory round trip.
    // Convergence (sklearn: labels equal, _kmeans.py:717-723): the raw statistics
    // of this iteration (before any relocation move) equal the previous ones.
    unsigned long long neq = 0, bmax = 0;
    int barg = 0x7fffffff;
    unsigned ne = 0;
    for (int j = tid; j < K; j += 1024) {
        unsigned long long row[D + 1], pv[D + 1];
        const size_t o = (size_t)j * (D + 1);
        if (partials) {
            unsigned long long *src = partials + (size_t)(ctrl->iter & 1u) * n;
#pragma unroll
            for (int a = 0; a <= D; ++a) { row[a] = src[o + a]; pv[a] = prev[o + a]; }
#pragma unroll
            for (int a = 0; a <= D; ++a) {
                src[o + a] = 0ull;
                stats[o + a] = row[a];
            }
        } else {
#pragma unroll
            for (int a = 0; a <= D; ++a) { row[a] = stats[o + a]; pv[a] = prev[o + a]; }
        }
        if (!resume) {
#pragma unroll
            for (int a = 0; a <= D; ++a) {
                neq += (row[a] != pv[a]) ? 1ull : 0ull;
                prev[o + a] = row[a];
            }
        }
        const unsigned long long c = row[D];
        if (c == 0) ne++;
        if (c > bmax) { bmax = c; barg = j; }
    }
    if (partials && tid == 0) stats[n] = 0ull;
    if (neq) atomicAdd(&neq_s, neq);
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long ob = __shfl_xor(bmax, o);
        const int oa = __shfl_xor(barg, o);
        if (ob > bmax || (ob == bmax && oa < barg)) { bmax = ob; barg = oa; }
    }
    if (lane == 0) { wmax[wv] = bmax; warg[wv] = barg; }
    if (ne) atomicAdd(&cnt_empty, ne);
    __syncthreads();
    if (cnt_empty > 0 && !resume) {
        // Snapshot the reduced statistics: the no-op iterations queued behind a
        // halt still run their all-reduce on `stats`.
        for (int i = tid; i < n + 1; i += 1024) held[i] = stats[i];
        if (tid == 0) {
            ctrl->halt = 1u;
            ctrl->n_empty = cnt_empty;
            ctrl->neq_saved = neq_s;
        }
        return;
    }
    unsigned long long gmax = wmax[0];
    int argmax = warg[0];
    for (int w = 1; w < 16; ++w)
        if (wmax[w] > gmax || (wmax[w] == gmax && warg[w] < argmax)) { gmax = wmax[w]; argmax = warg[w]; }
    // average + shift (thread tid owns j = tid + 1024 r in every loop below);
    // shift: per-thread sequential sum over its j, then the fixed tree below
    auto average_row = [&](int j, float4 &cn) -> bool {
        unsigned long long row[D + 1];
#pragma unroll
        for (int a = 0; a <= D; ++a) row[a] = stats[(size_t)j * (D + 1) + a];
        const unsigned long long c = row[D];
        float out[4] = {0.f, 0.f, 0.f, 0.f};
        if (c > 0) {
#pragma unroll
            for (int a = 0; a < D; ++a) {
                const long long sv = (long long)row[a];   // exact signed sum
                const double m = ((double)sv * __builtin_ldexp(1.0, -q[a])) / (double)c;
                out[a] = (float)m;
            }
        }
        cn = make_float4(out[0], out[1], out[2], out[3]);
        return c > 0;
    };
    auto shift_of = [&](const float4 &a4, const float4 &b4) -> double {
        double sh = 0.0;
#pragma unroll
        for (int a = 0; a < D; ++a) {
            const double dd = (double)comp(a4, a) - (double)comp(b4, a);
            const double sq = dd * dd;
            sh = (a == 0) ? sq : sh + sq;
        }
        return sh;
    };
    double acc = 0.0;
    if (cnt_empty == 0) {   // the common case: no empty cluster, one pass
        for (int j = tid; j < K; j += 1024) {
            const float4 b4 = C[j];
            float4 cn;
            average_row(j, cn);
            acc = acc + shift_of(cn, b4);
            C[j] = cn;
        }
    } else {   // resumed after relocation: an empty cluster copies the largest one's centre
        for (int j = tid; j < K; j += 1024) {
            float4 cn;
            if (average_row(j, cn)) Cn[j] = cn;
        }
        __syncthreads();   // Cn[argmax] is read by other threads
        for (int j = tid; j < K; j += 1024) {
            const unsigned long long c = stats[(size_t)j * (D + 1) + D];
            if (c == 0) Cn[j] = (gmax > 0) ? Cn[argmax] : C[j];
            const float4 a4 = Cn[j], b4 = C[j];
            acc = acc + shift_of(a4, b4);
            C[j] = Cn[j];
        }
    }
    ssum[tid] = acc;
    __syncthreads();
    // statistics read in place (all-reduce buffer / resume): zero them for the
    // next iteration's accumulation (every read above precedes the barrier)
    if (!partials)
        for (int i = tid; i < n + 1; i += 1024) stats[i] = 0ull;
    for (int st = 512; st >= 64; st >>= 1) {
        if (tid < st) ssum[tid] = ssum[tid] + ssum[tid + st];
        __syncthreads();
    }
    if (wv == 0) {
        double v = ssum[lane];
        for (int st = 32; st > 0; st >>= 1) v = v + __shfl_down(v, st);   // lane t: v_t + v_{t+st}
        if (lane == 0) {
            const unsigned long long changed = resume ? ctrl->neq_saved : neq_s;
            const double shift = v;
            const uint32_t it = ctrl->iter;
            if (it < ctrl->max_iter) {
                hist_changed[it] = changed;
                hist_shift[it] = shift;
            }
            ctrl->last_changed = changed;
            ctrl->last_shift = shift;
            ctrl->resume = 0u;
            uint32_t done = 0;
            if (changed == 0ull) done = 1u;
            else if (shift <= ctrl->tol) done = 2u;
            ctrl->iter = it + 1;
            if (!done && it + 1 >= ctrl->max_iter) done = 3u;
            ctrl->done = done;
        }
    }
}

// ------------------------------------------------------------------ centre update + candidate lists
// One Lloyd iteration's M-step (_average_centers, _center_shift, the
// convergence tests; _k_means_common.pyx:274-311, _kmeans.py:717-732) and the
// next iteration's candidate lists, in two launches:
//
//  k_upd   one thread per centroid: its row of the (all-reduced) integer
//          statistics -> the new centre Cn[j] (computed ONCE per iteration),
//          the statistics-equality test against the previous iteration, the
//          relocation snapshot `held`, zeroing of the next accumulation target,
//          its squared shift sh[j] and drift from the lists' reference centre.
//          Block sums/maxima go to ctrl by agent-scope atomics; the last block
//          to arrive reduces the shift with the fixed 1024-lane tree of
//          oracle/lloyd_ref.py shift_total, halts on an empty cluster (the host
//          relocates, then k_global + k_cand resume), or publishes the history,
//          flags and the list work: REFRESH the lists' records when every
//          centre is still within the lists' drift budget of the reference
//          position they were built at (the lists stay exact, see prunable),
//          else REBUILD them at the new centres with budget alpha * (largest
//          shift), capped at kappa * the smallest cell width (budget 0 above).
//  k_lists C := Cn (and the new reference buffer when rebuilding), then the
//          refresh or rebuild of this block's cells (cand_body / refresh_body
//          reading the new centres from global memory).
//
// Hand-off inside k_upd (MI355X_MICROARCH.md, hand-off table row 1): sh[] is
// written with sc1 stores, every storing wave drains them (vmcnt(0)) before
// the block barrier, one lane per block adds to the arrival counter, and the
// last arriver reads sh[] and the atomics with sc1 loads.
constexpr int UPD_TPB = 128;
constexpr int SHIFT_LANES = 1024;   // oracle/lloyd_ref.py SHIFT_LANES
constexpr int UPD_LPT = SHIFT_LANES / UPD_TPB;   // tree lanes per thread of the last block
static_assert(UPD_TPB == 128, "k_upd's last tree steps: one LDS step (h = 64), then wave shuffles");
// per-block record of k_upd: changed words, empty clusters, max squared drift, max squared shift
struct UpdPart {
    unsigned long long neq, nempty, dmax_bits, smax_bits;
};
// centroid j's loads: its statistics row, the previous row, the lists'
// reference position and the current centre
template <int D>
__device__ __forceinline__ void upd_load(int j, int K, const unsigned long long *src, const unsigned long long *prev,
                                         const float4 *cref, unsigned sel, const float4 *C,
                                         unsigned long long (&row)[D + 1], unsigned long long (&pv)[D + 1],
                                         float4 &rj, float4 &oj) {
    const size_t o = (size_t)j * (D + 1);
#pragma unroll
    for (int a = 0; a <= D; ++a) { row[a] = src[o + a]; pv[a] = prev[o + a]; }
    rj = cref[(size_t)sel * K + j];
    oj = C[j];
}
// its new centre (_average_centers: one fp64 division, one rounding to fp32),
// changed statistic words, emptiness, squared drift and squared shift
template <int D>
__device__ __forceinline__ void upd_row(const unsigned long long (&row)[D + 1], const unsigned long long (&pv)[D + 1],
                                        const float4 &rj, const float4 &oj, const QExp &qe, float4 &cnew,
                                        unsigned long long &neq, unsigned &ne, double &dr, double &ds) {
#pragma unroll
    for (int a = 0; a <= D; ++a) neq += (row[a] != pv[a]) ? 1ull : 0ull;   // raw statistics vs the previous ones
    const unsigned long long c = row[D];
    float out[4] = {0.f, 0.f, 0.f, 0.f};
    if (c > 0) {
#pragma unroll
        for (int a = 0; a < D; ++a) {
            const double m = ((double)(long long)row[a] * __builtin_ldexp(1.0, -qe.q[a])) / (double)c;
            out[a] = (float)m;
        }
    } else {
        ne += 1u;
    }
    cnew = make_float4(out[0], out[1], out[2], out[3]);
#pragma unroll
    for (int a = 0; a < D; ++a) {
        const double e1 = (double)comp(cnew, a) - (double)comp(rj, a);
        const double e2 = (double)comp(cnew, a) - (double)comp(oj, a);
        dr += e1 * e1;
        ds += e2 * e2;
    }
}
// one lane: history, convergence flags and the list work of the next launch
// (it, max_iter, budget, tol: the control words as this launch found them)
__device__ __forceinline__ void upd_publish(Ctrl *ctrl, unsigned long long changed, double shift, double dmax,
                                            double smax, unsigned sel, double alpha, double dl_cap,
                                            unsigned long long *hist_changed, double *hist_shift, uint32_t it,
                                            uint32_t max_iter, double budget, double tol) {
    if (it < max_iter) {
        hist_changed[it] = changed;
        hist_shift[it] = shift;
    }
    ctrl->last_changed = changed;
    ctrl->last_shift = shift;
    ctrl->resume = 0u;
    const double slack = 1.0 + 9.094947017729282e-13;   // 1 + 2^-40: fp64 rounding of the drift norms
    const bool rebuild = !(sqrt(dmax) * slack <= budget);
    double dl_new = alpha * sqrt(smax) * slack;
    if (!(dl_new <= dl_cap)) dl_new = 0.0;
    if (rebuild) {
        ctrl->ref_sel = sel ^ 1u;
        ctrl->budget = dl_new;
        ctrl->rebuilds += 1u;
    }
    ctrl->lists = rebuild ? 2u : 1u;
    ctrl->lists_dl = rebuild ? dl_new : budget;
    uint32_t done = 0;
    if (changed == 0ull) done = 1u;
    else if (shift <= tol) done = 2u;
    if (!done && it + 1 >= max_iter) done = 3u;
    ctrl->done = done;
    ctrl->iter = it + 1;
}

template <int D>
__global__ __launch_bounds__(UPD_TPB) void k_upd(unsigned long long *__restrict__ stats_in,
                                                 unsigned long long *__restrict__ partials, int K, QExp qe,
                                                 unsigned long long *__restrict__ held,
                                                 unsigned long long *__restrict__ prev, const float4 *__restrict__ C,
                                                 float4 *__restrict__ Cn, const float4 *__restrict__ cref,
                                                 double *__restrict__ sh, UpdPart *__restrict__ upart,
                                                 unsigned long long *__restrict__ hist_changed,
                                                 double *__restrict__ hist_shift, Ctrl *__restrict__ ctrl, double alpha,
                                                 double dl_cap) {
    // the gate flags and the control words this launch reads, in one memory latency
    unsigned gate = ctrl->halt | ctrl->done;
    unsigned par = ctrl->iter & 1u;
    unsigned sel = ctrl->ref_sel;
    asm volatile("" : "+s"(gate), "+s"(par), "+s"(sel));   // keep the loads above the exit
    if (gate != 0u) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = K * (D + 1);
    const int j = blockIdx.x * UPD_TPB + tid;
    unsigned long long *src = stats_in ? stats_in : partials + (size_t)par * n;
    unsigned long long neq = 0ull;
    unsigned ne = 0u;
    double dr = 0.0, ds = 0.0;
    unsigned long long row[D + 1], pv[D + 1];
    float4 rj, oj;
    float4 cnew = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j < K) {
        upd_load<D>(j, K, src, prev, cref, sel, C, row, pv, rj, oj);
        upd_row<D>(row, pv, rj, oj, qe, cnew, neq, ne, dr, ds);
        __hip_atomic_store(sh + j, ds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // only sh[] is handed to the last block inside this launch: drain it now;
    // the other stores below are read by later launches (the kernel boundary)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (j < K) {
        const size_t o = (size_t)j * (D + 1);
        unsigned long long *pnext = stats_in ? stats_in : partials + (size_t)(par ^ 1u) * n;
#pragma unroll
        for (int a = 0; a <= D; ++a) {
            prev[o + a] = row[a];
            held[o + a] = row[a];   // the relocation snapshot, should this iteration halt
            pnext[o + a] = 0ull;    // the next accumulation starts from zero
        }
        Cn[j] = cnew;
    }
    if (j == 0) {
        held[n] = 0ull;
        if (stats_in) stats_in[n] = 0ull;
    }
    for (int o = 32; o > 0; o >>= 1) {
        neq += __shfl_xor(neq, o);
        ne += __shfl_xor(ne, o);
        dr = fmax(dr, __shfl_xor(dr, o));
        ds = fmax(ds, __shfl_xor(ds, o));
    }
    __shared__ unsigned long long s_neq[UPD_TPB / 64];
    __shared__ unsigned s_ne[UPD_TPB / 64];
    __shared__ double s_dr[UPD_TPB / 64], s_ds[UPD_TPB / 64];
    __shared__ unsigned s_last;
    if (lane == 0) { s_neq[wv] = neq; s_ne[wv] = ne; s_dr[wv] = dr; s_ds[wv] = ds; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < UPD_TPB / 64; ++w) {
            neq += s_neq[w]; ne += s_ne[w]; dr = fmax(dr, s_dr[w]); ds = fmax(ds, s_ds[w]);
        }
        // this block's record (sc1 stores, drained before the arrival like sh[])
        UpdPart *pp = upart + blockIdx.x;
        __hip_atomic_store(&pp->neq, neq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&pp->nempty, (unsigned long long)ne, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&pp->dmax_bits, (unsigned long long)__double_as_longlong(dr), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&pp->smax_bits, (unsigned long long)__double_as_longlong(ds), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // release (arrive_last): this block's sh[] and record stores are ordered
        // before its arrival (the sc1 stores above are drained anyway)
        s_last = arrive_last(ctrl) ? 1u : 0u;
    }
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // every other block's published stores are visible
    // ---- the last block: every other block's sh[] and record have landed
    unsigned long long changed = 0ull, n_empty = 0ull;
    double dmax = 0.0, smax = 0.0;
    for (int b = tid; b < (int)gridDim.x; b += UPD_TPB) {
        const UpdPart *pp = upart + b;
        changed += __hip_atomic_load(&pp->neq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        n_empty += __hip_atomic_load(&pp->nempty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dmax = fmax(dmax, __longlong_as_double(
                              (long long)__hip_atomic_load(&pp->dmax_bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
        smax = fmax(smax, __longlong_as_double(
                              (long long)__hip_atomic_load(&pp->smax_bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
    }
    for (int o = 32; o > 0; o >>= 1) {
        changed += __shfl_xor(changed, o);
        n_empty += __shfl_xor(n_empty, o);
        dmax = fmax(dmax, __shfl_xor(dmax, o));
        smax = fmax(smax, __shfl_xor(smax, o));
    }
    __syncthreads();   // s_* of the arrival phase are reused below
    if (lane == 0) { s_neq[wv] = changed; s_ne[wv] = (unsigned)n_empty; s_dr[wv] = dmax; s_ds[wv] = smax; }
    __syncthreads();
    changed = s_neq[0];
    n_empty = s_ne[0];
    dmax = s_dr[0];
    smax = s_ds[0];
    for (int w = 1; w < UPD_TPB / 64; ++w) {
        changed += s_neq[w]; n_empty += s_ne[w]; dmax = fmax(dmax, s_dr[w]); smax = fmax(smax, s_ds[w]);
    }
    if (tid == 0) __hip_atomic_store(&ctrl->u_arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n_empty > 0ull) {   // empty cluster: the host relocates, then k_global + k_cand resume
        if (tid == 0) {
            ctrl->n_empty = (unsigned)n_empty;
            ctrl->neq_saved = changed;
            ctrl->lists = 0u;
            ctrl->halt = 1u;
        }
        return;
    }
    // total shift: lane L sums sh[L + 1024 r] in ascending r, then the halving tree
    double v[UPD_LPT];
#pragma unroll
    for (int u = 0; u < UPD_LPT; ++u) v[u] = 0.0;
    for (int r = 0; r * SHIFT_LANES < K; ++r)
#pragma unroll
        for (int u = 0; u < UPD_LPT; ++u) {
            const int idx = r * SHIFT_LANES + tid + UPD_TPB * u;
            if (idx < K) v[u] = v[u] + __hip_atomic_load(sh + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
    for (int h = UPD_LPT / 2; h >= 1; h >>= 1)   // lanes L and L + UPD_TPB * h live in this thread
#pragma unroll
        for (int u = 0; u < h; ++u) v[u] = v[u] + v[u + h];
    __shared__ double s_tree[UPD_TPB];
    s_tree[tid] = v[0];
    __syncthreads();
    if (wv == 0) {
        double x = s_tree[lane];
        x = x + s_tree[lane + 64];
        for (int st = 32; st > 0; st >>= 1) x = x + __shfl_down(x, st);   // lane t: x_t + x_{t+st}
        if (lane == 0)
            upd_publish(ctrl, changed, x, dmax, smax, sel, alpha, dl_cap, hist_changed, hist_shift, ctrl->iter,
                        ctrl->max_iter, ctrl->budget, ctrl->tol);
    }
}

// k_upd in ONE block of SHIFT_LANES threads (K <= UPD1_MAX: configs 1-4): thread L owns centroids L + 1024 r, so its tree lane's
// sum (ascending r) stays in registers and the halving tree runs in LDS -- no
// per-block records, no arrival counter, no second pass over sh[] (the
// multi-block k_upd's hand-off cost ~4 memory latencies: 9.5 us at K = 1024).
// Same arithmetic, stores and published words as k_upd.
// R = rows per thread = ceil(K / 1024).  K = 4096 (config 5) keeps the
// multi-block k_upd: one block doing 4 rows per thread (in batches, to stay
// within 128 VGPRs) measured 28 us against k_upd's 15 at an 8-way config-5 slab.
constexpr int UPD1_MAX = 2 * SHIFT_LANES;
template <int D, int R>
__global__ __launch_bounds__(SHIFT_LANES) void k_upd1(unsigned long long *__restrict__ stats_in,
                                                      unsigned long long *__restrict__ partials, int K, QExp qe,
                                                      unsigned long long *__restrict__ held,
                                                      unsigned long long *__restrict__ prev,
                                                      const float4 *__restrict__ C, float4 *__restrict__ Cn,
                                                      const float4 *__restrict__ cref,
                                                      unsigned long long *__restrict__ hist_changed,
                                                      double *__restrict__ hist_shift, Ctrl *__restrict__ ctrl,
                                                      double alpha, double dl_cap) {
    // every load of the launch in ONE memory latency: the control words, the
    // rows of both parity halves of `partials` and both reference buffers
    // (selected once the words are in, instead of a second dependent round)
    unsigned gate = ctrl->halt | ctrl->done;
    const uint32_t it = ctrl->iter, max_iter = ctrl->max_iter;
    const unsigned sel = ctrl->ref_sel;
    const double budget = ctrl->budget, tol = ctrl->tol;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = K * (D + 1);
    // (R > 2: too many registers for both halves -- the rows follow the control
    // words, one more latency)
    static_assert(R >= 1 && R <= 2, "K <= UPD1_MAX");
    unsigned long long row[R][D + 1], alt[R][D + 1], pv[R][D + 1];
    float4 rj[R], rk[R], oj[R];
    const unsigned par = it & 1u;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = tid + SHIFT_LANES * r;
        if (j < K) {
            const size_t o = (size_t)j * (D + 1);
#pragma unroll
            for (int a = 0; a <= D; ++a) {
                row[r][a] = stats_in ? stats_in[o + a] : partials[o + a];
                alt[r][a] = stats_in ? 0ull : partials[(size_t)n + o + a];
                pv[r][a] = prev[o + a];
            }
            rj[r] = cref[j];
            rk[r] = cref[(size_t)K + j];
            oj[r] = C[j];
        }
    }
    if (gate != 0u) return;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!stats_in && par)
#pragma unroll
            for (int a = 0; a <= D; ++a) row[r][a] = alt[r][a];
        if (sel) rj[r] = rk[r];
    }
    unsigned long long neq = 0ull;
    unsigned ne = 0u;
    double dr = 0.0, ds = 0.0, v = 0.0;
    float4 cnew[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = tid + SHIFT_LANES * r;
        if (j < K) {
            double drj = 0.0, dsj = 0.0;
            upd_row<D>(row[r], pv[r], rj[r], oj[r], qe, cnew[r], neq, ne, drj, dsj);
            dr = fmax(dr, drj);
            ds = fmax(ds, dsj);
            v = v + dsj;   // tree lane tid: sh[tid + 1024 r] in ascending r
        }
    }
    unsigned long long *pnext = stats_in ? stats_in : partials + (size_t)(par ^ 1u) * n;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = tid + SHIFT_LANES * r;
        if (j < K) {
            const size_t o = (size_t)j * (D + 1);
#pragma unroll
            for (int a = 0; a <= D; ++a) {
                prev[o + a] = row[r][a];
                held[o + a] = row[r][a];   // the relocation snapshot, should this iteration halt
                pnext[o + a] = 0ull;       // the next accumulation starts from zero
            }
            Cn[j] = cnew[r];
        }
    }
    if (tid == 0) {
        held[n] = 0ull;
        if (stats_in) stats_in[n] = 0ull;
    }
    for (int o = 32; o > 0; o >>= 1) {
        neq += __shfl_xor(neq, o);
        ne += __shfl_xor(ne, o);
        dr = fmax(dr, __shfl_xor(dr, o));
        ds = fmax(ds, __shfl_xor(ds, o));
    }
    constexpr int NW = SHIFT_LANES / 64;
    __shared__ unsigned long long s_neq[NW];
    __shared__ unsigned s_ne[NW];
    __shared__ double s_dr[NW], s_ds[NW];
    __shared__ double s_tree[SHIFT_LANES];
    if (lane == 0) { s_neq[wv] = neq; s_ne[wv] = ne; s_dr[wv] = dr; s_ds[wv] = ds; }
    s_tree[tid] = v;
    __syncthreads();
    unsigned long long changed = 0ull, n_empty = 0ull;
    double dmax = 0.0, smax = 0.0;
    for (int w = 0; w < NW; ++w) {
        changed += s_neq[w]; n_empty += s_ne[w]; dmax = fmax(dmax, s_dr[w]); smax = fmax(smax, s_ds[w]);
    }
    if (n_empty > 0ull) {   // empty cluster: the host relocates, then k_global + k_cand resume
        if (tid == 0) {
            ctrl->n_empty = (unsigned)n_empty;
            ctrl->neq_saved = changed;
            ctrl->lists = 0u;
            ctrl->halt = 1u;
        }
        return;
    }
    // the halving tree of oracle/lloyd_ref.py shift_total: lane L += lane L + h
    for (int h = SHIFT_LANES / 2; h >= 64; h >>= 1) {
        if (tid < h) s_tree[tid] = s_tree[tid] + s_tree[tid + h];
        __syncthreads();
    }
    if (wv == 0) {
        double x = s_tree[lane];
        for (int st = 32; st > 0; st >>= 1) x = x + __shfl_down(x, st);   // lane t: x_t + x_{t+st}
        if (lane == 0)
            upd_publish(ctrl, changed, x, dmax, smax, sel, alpha, dl_cap, hist_changed, hist_shift, it, max_iter,
                        budget, tol);
    }
}

// C := Cn (the centres k_upd published) and the next iteration's candidate
// lists: a rebuild at Cn with the published budget (the new reference buffer
// cref[ref_sel] := Cn) or a refresh of the records.  Runs after a completed
// k_upd: halted iterations leave C untouched (the relocation needs the old
// centres); queued no-op launches after convergence repeat the same copy and
// lists (idempotent).
constexpr int LISTS_STAGE_MAX = 2048;   // k_lists stages the centres in LDS up to this K (32 KB)
template <int D, int FC = 4, bool STAGE = false, int TPB = CAND_TPB>
__global__ __launch_bounds__(TPB) void k_lists(Grid g, const float4 *__restrict__ Cn, float4 *__restrict__ C,
                                                    float4 *__restrict__ cref, int K, const Ctrl *__restrict__ ctrl,
                                                    uint32_t *__restrict__ fc_cnt, float4 *__restrict__ fc_rec,
                                                    int32_t *__restrict__ fc_lab, int bpc, CoarseL cl) {
    unsigned halt = ctrl->halt;
    unsigned mode = ctrl->lists;
    unsigned sel = ctrl->ref_sel;
    double dl = ctrl->lists_dl;
    // STAGE: all K new centres staged in LDS by one coalesced pass, issued with
    // the control-word loads (one memory latency for both; a gated launch
    // leaves the LDS copy unused): the list phases' reads of them (references,
    // tests, compaction) become LDS reads instead of dependent global round trips
    extern __shared__ __attribute__((aligned(16))) float4 cstage[];
    if constexpr (STAGE)
        for (int j = threadIdx.x; j < K; j += TPB) cstage[j] = Cn[j];
    asm volatile("" : "+s"(halt), "+s"(mode), "+s"(sel), "+s"(dl));
    if (halt != 0u || mode == 0u) return;
    DBG_T(0);
    if constexpr (STAGE) __syncthreads();
    for (int j = blockIdx.x * TPB + threadIdx.x; j < K; j += gridDim.x * TPB) {
        const float4 c = STAGE ? cstage[j] : Cn[j];
        C[j] = c;
        if (mode == 2u) cref[(size_t)sel * K + j] = c;
    }
    if (mode != 2u) {
        refresh_body<D, TPB>(g, Cn, fc_cnt, fc_rec, fc_lab);
        return;
    }
    if constexpr (STAGE) cand_body<D, FC, TPB>(g, cstage, K, fc_cnt, fc_rec, fc_lab, bpc, dl, cl);
    else cand_body<D, FC, TPB>(g, Cn, K, fc_cnt, fc_rec, fc_lab, bpc, dl, cl);
}

// Centre update and candidate lists in ONE launch (D <= 3, K <= CAND_TPB * 2 =
// 1024: configs 1-4).  Every block loads all K statistics rows (both parity
// halves of `partials`, or the all-reduced buffer), the previous rows, the old
// centres and both reference buffers together with the control words -- one
// memory latency -- and computes all K new centres into LDS plus the
// order-independent decisions every block needs identically (an empty cluster
// halts; the largest drift and shift give rebuild-or-refresh and the new
// budget).  Then one agent-scope arrival per block; the LAST block to arrive
// (every other block's loads have returned by then) publishes what k_upd does
// -- prev, held, the zeroed next accumulation target, C and the new reference
// buffer, the shift tree of oracle/lloyd_ref.py shift_total, history and flags
// -- and every block rebuilds or refreshes its own cells' lists from the LDS
// centres.  Replaces k_upd1 + k_lists (two launches, ~16 us at an 8-way slab).
// PUB (round 6; the host takes it when one more block fits the residency, e.g.
// the 8-way slab's 256 list blocks): the LAST block of the grid builds no lists
// and is the publisher -- it waits (bounded, s_sleep) until the list blocks have
// arrived, right after their centres, and publishes while they still build
// their lists, instead of after its own lists; a wait past 2 s sets done = 5.
template <int D, int R, bool PUB = false>
__global__ __launch_bounds__(CAND_TPB) void k_updlists(
    unsigned long long *__restrict__ stats_in, unsigned long long *__restrict__ partials, int K, QExp qe,
    unsigned long long *__restrict__ held, unsigned long long *__restrict__ prev, float4 *__restrict__ C,
    float4 *__restrict__ cref, unsigned long long *__restrict__ hist_changed, double *__restrict__ hist_shift,
    Ctrl *__restrict__ ctrl, double alpha, double dl_cap, Grid g, uint32_t *__restrict__ fc_cnt,
    float4 *__restrict__ fc_rec, int32_t *__restrict__ fc_lab, int bpc) {
    static_assert(R * CAND_TPB <= SHIFT_LANES && SHIFT_LANES % CAND_TPB == 0, "one tree lane per row");
    extern __shared__ __attribute__((aligned(16))) float4 cstage[];   // the K new centres
    DBG_T(13);
    unsigned gate = ctrl->halt | ctrl->done;
    const uint32_t it = ctrl->iter, max_iter = ctrl->max_iter;
    const unsigned sel = ctrl->ref_sel;
    const double budget = ctrl->budget, tol = ctrl->tol;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = K * (D + 1);
    // row r of this thread: centroid j = tid + CAND_TPB * r (tree lane j).  (The
    // publisher alone loading the previous rows, for the changed-word count,
    // measured slower: its extra latency sits on the launch's tail.)
    unsigned long long row[R][D + 1], alt[R][D + 1], pv[R][D + 1];
    float4 rj[R], rk[R], oj[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = tid + CAND_TPB * r;
        if (j < K) {
            const size_t o = (size_t)j * (D + 1);
#pragma unroll
            for (int a = 0; a <= D; ++a) {
                row[r][a] = stats_in ? stats_in[o + a] : partials[o + a];
                alt[r][a] = stats_in ? 0ull : partials[(size_t)n + o + a];
                pv[r][a] = prev[o + a];
            }
            rj[r] = cref[j];
            rk[r] = cref[(size_t)K + j];
            oj[r] = C[j];
        }
    }
    if (gate != 0u) return;
    DBG_T(0);
    const unsigned par = it & 1u;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!stats_in && par)
#pragma unroll
            for (int a = 0; a <= D; ++a) row[r][a] = alt[r][a];
        if (sel) rj[r] = rk[r];
    }
    unsigned long long neq = 0ull;
    unsigned ne = 0u;
    double dr = 0.0, ds = 0.0, sh[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = tid + CAND_TPB * r;
        sh[r] = 0.0;
        if (j < K) {
            double drj = 0.0, dsj = 0.0;
            float4 cnew;
            upd_row<D>(row[r], pv[r], rj[r], oj[r], qe, cnew, neq, ne, drj, dsj);
            dr = fmax(dr, drj);
            ds = fmax(ds, dsj);
            sh[r] = dsj;
            cstage[j] = cnew;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        neq += __shfl_xor(neq, o);
        ne += __shfl_xor(ne, o);
        dr = fmax(dr, __shfl_xor(dr, o));
        ds = fmax(ds, __shfl_xor(ds, o));
    }
    constexpr int NW = CAND_TPB / 64;
    __shared__ unsigned long long s_neq[NW];
    __shared__ unsigned s_ne[NW];
    __shared__ double s_dr[NW], s_ds[NW];
    __shared__ unsigned s_last;
    // the shift tree's lanes: L < 1024 holds sh[L] (K <= 1024); the first halving
    // step (lane t += lane t + 512) runs in this thread's registers.  Kept in LDS
    // for the publisher, so that nothing of the centre phase stays live in
    // registers through the lists (a 2-blocks-per-CU residency at 512 blocks)
    static_assert(CAND_TPB == SHIFT_LANES / 2, "thread t holds tree lanes t and t + 512");
    __shared__ double s_tree[CAND_TPB];
    s_tree[tid] = sh[0] + (R > 1 ? sh[R > 1 ? 1 : 0] : 0.0);
    if (lane == 0) { s_neq[wv] = neq; s_ne[wv] = ne; s_dr[wv] = dr; s_ds[wv] = ds; }
    __syncthreads();   // every load of this block has returned (its values are used above)
    // The arrival: issued now, its returned place read after this block's lists.
    // One same-address atomic per block (512 of them serialise at the memory
    // side, ~12 ns each): waiting for it here held every block's lists for its
    // place in that queue ("centres + arrival" 6.2 us of a ~17 us block at
    // config 3, rd5_updlists_phases_c3.txt).  No release fence: the rows, prev,
    // C and control words the publisher overwrites were consumed above, and the
    // lists read only the LDS centres.  The publisher is the last block to
    // ARRIVE (here), not the last to finish its lists, so its extra work lands
    // on a block of ordinary length.
    const bool pub_blk = PUB && blockIdx.x == gridDim.x - 1u;   // the dedicated publisher (PUB)
    const unsigned nlist = PUB ? gridDim.x - 1u : gridDim.x;
    unsigned tk = 0u;
    if constexpr (PUB) {
        if (!pub_blk && tid == 0) __hip_atomic_fetch_add(&ctrl->u_arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        tk = arrive_issue(&ctrl->u_arrive, (unsigned long long)__builtin_amdgcn_readfirstlane(wv == 0 ? 1 : 0));
    }
    // the decisions of upd_publish, identical in every block (same data, order-free maxima)
    auto decide = [&](unsigned long long &n_empty, double &dmax, double &smax, bool &rebuild, double &dl_new) {
        n_empty = 0ull; dmax = 0.0; smax = 0.0;
        for (int w = 0; w < NW; ++w) {
            n_empty += s_ne[w]; dmax = fmax(dmax, s_dr[w]); smax = fmax(smax, s_ds[w]);
        }
        const double slack = 1.0 + 9.094947017729282e-13;
        rebuild = !(sqrt(dmax) * slack <= budget);
        dl_new = alpha * sqrt(smax) * slack;
        if (!(dl_new <= dl_cap)) dl_new = 0.0;
    };
    {
        unsigned long long n_empty;
        double dmax, smax, dl_new;
        bool rebuild;
        decide(n_empty, dmax, smax, rebuild, dl_new);
        // this block's share of the writes nobody reads in this launch: the
        // relocation snapshot `held` and, on a rebuild, the new reference buffer
        // (the blocks read cref[sel ^ 1] only speculatively, and use cref[sel])
        const int share = (K + (int)gridDim.x - 1) / (int)gridDim.x;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int j = tid + CAND_TPB * r;
            if (j < K && j / share == (int)blockIdx.x) {
                const size_t o = (size_t)j * (D + 1);
#pragma unroll
                for (int a = 0; a <= D; ++a) held[o + a] = row[r][a];
                if (n_empty == 0ull && rebuild) cref[(size_t)(sel ^ 1u) * K + j] = cstage[j];
            }
        }
        DBG_T(15);
        // a halted iteration (identical decision in every block) builds no lists
        if (n_empty == 0ull && !pub_blk) {
            DBG_T(14);
            // this block's cells: rebuilt at the new centres with the new budget, or refreshed
            if (rebuild) cand_body<D, 4>(g, cstage, K, fc_cnt, fc_rec, fc_lab, bpc, dl_new, CoarseL{});
            else refresh_body<D>(g, cstage, fc_cnt, fc_rec, fc_lab, nlist);
        }
    }
    if constexpr (PUB) {
        if (!pub_blk) return;
        if (wv == 0) {   // every list block arrives right after its centres: a bounded wait
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
            unsigned ok = 1u;
            while (__hip_atomic_load(&ctrl->u_arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nlist) {
                __builtin_amdgcn_s_sleep(2);
                if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { ok = 0u; break; }
            }
            if (lane == 0) s_last = ok;
        }
        __syncthreads();   // s_last
        if (!s_last) {
            if (tid == 0) ctrl->done = 5u;   // the fit is void (lloyd.run raises)
            return;
        }
    } else {
        if (wv == 0) {
            const unsigned place = arrive_read(tk);
            if (lane == 0) s_last = place == gridDim.x - 1u;
        }
        __syncthreads();   // s_last
        if (!s_last) return;
    }
    DBG_T(3);
    // ---- the publisher: every other block's loads have returned.  It reads the
    // rows again (L2; nobody has written them): prev := rows, the next
    // accumulation target := 0 and (unless halted: the relocation needs the old
    // C) C := the new centres.  Invariant the zeroing relies on: every
    // block consumed its loads of prev, C and the statistics rows (their values
    // feed the centres above) before it arrived; a load left in flight at an
    // arrival is one whose value is discarded -- the `alt` half of `partials`,
    // issued only when stats_in is null, a path no engine entry takes since
    // round 6 (pcm_iterate / pcm_iter_global always pass the statistics buffer).
    unsigned long long n_empty;
    double dmax, smax, dl_new;
    bool rebuild;
    decide(n_empty, dmax, smax, rebuild, dl_new);
    const unsigned long long *src = stats_in ? stats_in : partials + (size_t)par * n;
    unsigned long long *pnext = stats_in ? stats_in : partials + (size_t)(par ^ 1u) * n;
    unsigned long long v[R][D + 1];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = tid + CAND_TPB * r;
        const size_t o = (size_t)(j < K ? j : 0) * (D + 1);
#pragma unroll
        for (int a = 0; a <= D; ++a) v[r][a] = src[o + a];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = tid + CAND_TPB * r;
        if (j < K) {
            const size_t o = (size_t)j * (D + 1);
#pragma unroll
            for (int a = 0; a <= D; ++a) prev[o + a] = v[r][a];
#pragma unroll
            for (int a = 0; a <= D; ++a) pnext[o + a] = 0ull;   // the next accumulation starts from zero
            if (n_empty == 0ull) C[j] = cstage[j];
        }
    }
    unsigned long long changed = 0ull;
    for (int w = 0; w < NW; ++w) changed += s_neq[w];
    if (tid == 0) {
        held[n] = 0ull;
        if (stats_in) stats_in[n] = 0ull;
        __hip_atomic_store(&ctrl->u_arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (n_empty > 0ull) {
        if (tid == 0) {
            ctrl->n_empty = (unsigned)n_empty;
            ctrl->neq_saved = changed;
            ctrl->lists = 0u;
            ctrl->halt = 1u;
        }
    } else {
        for (int h = SHIFT_LANES / 4; h >= 64; h >>= 1) {
            if (tid < h) s_tree[tid] = s_tree[tid] + s_tree[tid + h];
            __syncthreads();
        }
        if (wv == 0) {
            double x = s_tree[lane];
            for (int st = 32; st > 0; st >>= 1) x = x + __shfl_down(x, st);   // lane t: x_t + x_{t+st}
            if (lane == 0)
                upd_publish(ctrl, changed, x, dmax, smax, sel, alpha, dl_cap, hist_changed, hist_shift, it,
                            max_iter, budget, tol);
        }
    }
    DBG_T(6);
}

// ------------------------------------------------------------------ relocation
// This rank's m farthest points from their centre (_k_means_common.pyx:185-187)
// by an exact radix SELECT over unique 64-bit keys (no sort, no N-sized
// allocation: the keys live in the layout's scratch arena):
//   key = dist_bits << 32 | (0xffffffff - global index)   (distance desc, row asc)
// 8 passes pick the m-th largest key T one byte at a time (MSB first); then
// every point with key >= T writes its record (any order: k_reloc_apply ranks
// the records it receives).
template <typename T, int D, typename LT>
__global__ __launch_bounds__(256) void k_reloc_keys(const T *__restrict__ xs, long long n,
                                                    const LT *__restrict__ lab, const uint32_t *__restrict__ perm,
                                                    const float4 *__restrict__ C, long long gidx0,
                                                    const uint32_t *__restrict__ grows,
                                                    unsigned long long *__restrict__ keys) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x[D];
    for (int a = 0; a < D; ++a) x[a] = to_f<T>(xs[xs_index<D>(i, a)]);
    float d = dist_canon<D>(x, C[(int)lab[i]]);
    const uint32_t r = perm[i];
    unsigned long long g = grows ? (unsigned long long)grows[r] : (unsigned long long)(gidx0 + r);
    keys[i] = ((unsigned long long)__float_as_uint(d) << 32) | (0xffffffffull - (g & 0xffffffffull));
}

struct RselState {
    unsigned long long prefix;    // selected high bytes of T
    unsigned long long m_rem;     // how many of the keys matching `prefix` still belong to the top m
    unsigned int hist[256];
    unsigned int count_out;
    unsigned int pad;
};

// Histogram of byte `pass` (0 = most significant) of the keys whose higher bytes equal the prefix.
__global__ __launch_bounds__(256) void k_rsel_hist(const unsigned long long *__restrict__ keys, long long n,
                                                   RselState *__restrict__ st, int pass) {
    __shared__ unsigned int h[256];
    h[threadIdx.x] = 0u;
    __syncthreads();
    const int shift = 56 - 8 * pass;
    const unsigned long long hmask = pass ? (~0ull << (64 - 8 * pass)) : 0ull;
    const unsigned long long prefix = st->prefix;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const unsigned long long k = keys[i];
        if ((k & hmask) == prefix) atomicAdd(&h[(k >> shift) & 0xffu], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&st->hist[threadIdx.x], h[threadIdx.x]);
}

// One thread: the byte value holding the m_rem-th largest matching key.
__global__ void k_rsel_pick(RselState *__restrict__ st, int pass) {
    if (threadIdx.x != 0) return;
    unsigned long long above = 0ull;
    int v = 255;
    for (; v > 0; --v) {
        if (above + st->hist[v] >= st->m_rem) break;
        above += st->hist[v];
    }
    st->prefix |= (unsigned long long)v << (56 - 8 * pass);
    st->m_rem -= above;
    for (int b = 0; b < 256; ++b) st->hist[b] = 0u;
}

struct RelocRec {
    unsigned long long key;
    int32_t label;
    int32_t valid;
    int32_t xq[4];
};

// Every point with key >= T (the top m; keys are unique) writes its record.
template <typename T, int D, typename LT>
__global__ __launch_bounds__(256) void k_reloc_gather(const unsigned long long *__restrict__ keys, long long n,
                                                      const T *__restrict__ xs, const LT *__restrict__ lab, QExp qe,
                                                      RselState *__restrict__ st, int m, RelocRec *__restrict__ out) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long k = keys[i];
    if (k < st->prefix) return;
    const unsigned int slot = atomicAdd(&st->count_out, 1u);
    if (slot >= (unsigned)m) return;   // cannot happen (exactly min(m, n) keys >= T)
    RelocRec r;
    r.key = k;
    r.label = (int)lab[i];
    r.valid = 1;
    r.xq[0] = r.xq[1] = r.xq[2] = r.xq[3] = 0;
    for (int a = 0; a < D; ++a) r.xq[a] = fixed_i(to_f<T>(xs[xs_index<D>(i, a)]), qe.q[a]);
    out[slot] = r;
}

// Single block: global top-n_empty over all ranks' records, moves applied to
// the (all-reduced, offset-encoded) statistics in cluster order; then resume.
template <int D>
__global__ __launch_bounds__(256) void k_reloc_apply(const RelocRec *__restrict__ recs, int nrec,
                                                     unsigned long long *__restrict__ stats, int K,
                                                     int *__restrict__ rank_buf, int *__restrict__ empty_idx,
                                                     Ctrl *__restrict__ ctrl) {
    const int tid = threadIdx.x;
    // rank of each valid record by (key desc); keys are globally unique
    for (int i = tid; i < nrec; i += 256) {
        int r = 0;
        if (recs[i].valid) {
            for (int j = 0; j < nrec; ++j)
                if (recs[j].valid && recs[j].key > recs[i].key) ++r;
        } else {
            r = 0x7fffffff;
        }
        rank_buf[i] = r;
    }
    __syncthreads();
    if (tid == 0) {
        // max distance == 0 -> nothing to relocate (sklearn _k_means_common.pyx:189-192)
        int top = -1;
        for (int i = 0; i < nrec; ++i)
            if (rank_buf[i] == 0) top = i;
        bool doit = top >= 0 && (recs[top].key >> 32) != 0ull;
        if (doit) {
            // the empty clusters are fixed before any move (sklearn iterates a
            // precomputed list, _k_means_common.pyx:177-178): a donor cluster
            // emptied by a move is not refilled in this pass
            int n_empty = 0;
            for (int j = 0; j < K; ++j)
                if (stats[(size_t)j * (D + 1) + D] == 0ull) empty_idx[n_empty++] = j;
            int done_moves = 0;
            for (int ei = 0; ei < n_empty; ++ei) {
                const int j = empty_idx[ei];
                int pick = -1;
                for (int i = 0; i < nrec; ++i)
                    if (rank_buf[i] == done_moves) { pick = i; break; }
                if (pick < 0) break;
                const RelocRec &r = recs[pick];
                unsigned long long *so = stats + (size_t)r.label * (D + 1);
                unsigned long long *sn = stats + (size_t)j * (D + 1);
                for (int a = 0; a < D; ++a) {
                    unsigned long long u = (unsigned long long)(long long)r.xq[a];
                    so[a] -= u;
                    sn[a] = u;
                }
                so[D] -= 1ull;
                sn[D] = 1ull;
                ++done_moves;
            }
        }
        ctrl->halt = 0u;
        ctrl->resume = 1u;
    }
}

// ------------------------------------------------------------------ misc
template <typename LT>
__global__ __launch_bounds__(256) void k_unpermute(const LT *__restrict__ lab, const uint32_t *__restrict__ perm,
                                                   long long n, int32_t *__restrict__ out) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i < n) out[perm ? perm[i] : (uint32_t)i] = (int32_t)lab[i];
}

// Scatter of the sorted-order labels into row order restricted to the rows
// [r0, r1) (destination windows small enough to stay in the Infinity Cache
// while the random writes land: partial lines merge on-die instead of each
// 2-4 B write costing an HBM burst).
template <typename LT, typename OT>
__global__ __launch_bounds__(256) void k_unpermute_win(const LT *__restrict__ lab, const uint32_t *__restrict__ perm,
                                                       long long n, uint32_t r0, uint32_t r1, OT *__restrict__ out) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = perm[i];
    if (r >= r0 && r < r1) out[r] = (OT)lab[i];
}

// uint16 row-order labels -> int32 (0xffff stays -1 only where K > 65535, which never takes this path)
__global__ __launch_bounds__(256) void k_widen_u16(const uint16_t *__restrict__ in, long long n, int32_t *__restrict__ out) {
    long long i = (blockIdx.x * (long long)blockDim.x + threadIdx.x) * 4;
    if (i + 4 <= n) {
        const uint2 w = *reinterpret_cast<const uint2 *>(in + i);
        *reinterpret_cast<int4 *>(out + i) = make_int4((int)(w.x & 0xffffu), (int)(w.x >> 16), (int)(w.y & 0xffffu), (int)(w.y >> 16));
    } else {
        for (; i < n; ++i) out[i] = (int32_t)in[i];
    }
}

template <int D>
__global__ void k_centers_in(const float *__restrict__ Cin, int K, float4 *__restrict__ C) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= K) return;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int a = 0; a < D; ++a) v[a] = Cin[(size_t)j * D + a];
    C[j] = make_float4(v[0], v[1], v[2], v[3]);
}

template <int D>
__global__ void k_centers_out(const float4 *__restrict__ C, int K, float *__restrict__ out) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= K) return;
    float4 c = C[j];
    for (int a = 0; a < D; ++a) out[(size_t)j * D + a] = comp(c, a);
}

__global__ __launch_bounds__(256) void k_fill_i32(int32_t *__restrict__ p, long long n, int32_t v) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

__device__ __forceinline__ float synth_value(unsigned long long ctr, unsigned long long seed) {
    unsigned long long z = seed * 0xD1B54A32D192ED03ull + (ctr + 1ull) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    return (float)(uint32_t)(z >> 40) * 5.9604644775390625e-08f;
}

__global__ __launch_bounds__(256) void k_synth(float *__restrict__ out, long long n, int d, unsigned long long seed,
                                               long long start) {
    long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (e >= n * d) return;
    out[e] = synth_value((unsigned long long)(start * d + e), seed);
}

__global__ __launch_bounds__(256) void k_synth_rows(float *__restrict__ out, const long long *__restrict__ rows,
                                                    long long m, int d, unsigned long long seed) {
    long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (e >= m * d) return;
    long long r = rows[e / d];
    out[e] = synth_value((unsigned long long)(r * d + e % d), seed);
}

// Candidate-list statistics for diagnostics.
__global__ __launch_bounds__(256) void k_cand_stats(const uint32_t *__restrict__ fc_cnt, long long ncells,
                                                    unsigned long long *__restrict__ out /* sum, max, full */) {
    long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (c >= ncells) return;
    uint32_t m = fc_cnt[c];
    if (m == FULL) { atomicAdd(out + 2, 1ull); return; }
    atomicAdd(out, (unsigned long long)m);
    atomicMax(out + 1, (unsigned long long)m);
}

// ------------------------------------------------------------------ brute force
// Stateless brute-force operator: centres staged in LDS (K*4 floats), each
// thread one point; statistics via global atomics (exactness over speed).
template <int D>
__global__ __launch_bounds__(256) void k_bruteforce(const float *__restrict__ X, long long n, const float *__restrict__ Cg,
                                                    int K, QExp qe, int32_t *__restrict__ labels,
                                                    unsigned long long *__restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) float4 sc[];
    for (int j = threadIdx.x; j < K; j += blockDim.x) {
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        for (int a = 0; a < D; ++a) v[a] = Cg[(size_t)j * D + a];
        sc[j] = make_float4(v[0], v[1], v[2], v[3]);
    }
    __syncthreads();
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        float x[D];
        for (int a = 0; a < D; ++a) x[a] = X[i * D + a];
        float bd = dist_canon<D>(x, sc[0]);
        int bj = 0;
        for (int j = 1; j < K; ++j) {
            float dd = dist_canon<D>(x, sc[j]);
            if (dd < bd) { bd = dd; bj = j; }
        }
        labels[i] = bj;
        if (stats) {
            unsigned long long *p = stats + (size_t)bj * (D + 1);
            for (int a = 0; a < D; ++a) atomicAdd(p + a, (unsigned long long)(long long)fixed_i(x[a], qe.q[a]));
            atomicAdd(p + D, 1ull);
        }
    }
}

}  // namespace pcm
