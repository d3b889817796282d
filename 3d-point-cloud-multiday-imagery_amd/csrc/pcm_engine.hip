// pcm_engine.hip — host runtime + C ABI (include/pcm_kmeans.h) of the MI355X
// multi-day point-cloud Lloyd engine.  All device work is stream-ordered; the
// per-iteration entry points allocate nothing and never synchronise, so a
// caller may capture them into a HIP graph.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <vector>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "pcm_kernels.hpp"
#include "pcm_kpp.hpp"
#include "pcm_sort.hpp"
#include "pcm_cloud.hpp"
#include "pcm_common.hpp"
#include "pcm_kmeans.h"
#include "pcm_xchg.hpp"

using namespace pcm;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
}  // namespace

int pcm_fail(int code, const std::string &msg) { return fail(code, msg); }

#define HIPCHK(expr)                                                                             \
    do {                                                                                         \
        hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess)                                                                    \
            return fail(PCM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e) + " @" +   \
                                       std::to_string(__LINE__));                               \
    } while (0)

#define LAUNCHCHK() HIPCHK(hipGetLastError())

struct pcm_engine {
    int device = 0, d = 3, k = 1, dtype = PCM_F32, max_iter_cap = 300;
    long long n = 0, npad = 0, gidx0 = 0;
    long long n_global = 0;          // points over all ranks (pcm_layout_shard; = n for a single-process fit)
    uint32_t *grows = nullptr;       // global row of every local point (spatial shard) or null: gidx0 + i
    size_t cap_grows = 0;
    bool has_rows = false;
    double lo[MAXD] = {0}, hi[MAXD] = {0}, maxabs[MAXD] = {0};
    bool have_bbox = false, layout_ready = false, fit_ready = false;
    Grid g{};
    QExp qe{};
    long long ntiles = 0;            // host copy: -1 = not read back yet (pcm_layout_info reads it)
    long long ntiles_cap = 0;        // upper bound on the tiles of the current layout (grid sizing)
    uint32_t tile_cap = TILE;        // points per tile
    uint32_t *ntiles_host = nullptr; // pinned: the layout's tile count, read back at the end of pcm_layout_build
    Ctrl *ctrl_pin = nullptr;        // pinned snapshot of ctrl (pcm_status_post / pcm_status_wait)
    hipEvent_t st_ev = nullptr;
    // device buffers (persistent: grown on demand, reused by later layouts, freed at destroy)
    void *xs = nullptr;
    unsigned *xz = nullptr;          // compressed 8-B point records (fp32 D = 3, k_tile_compress)
    uint4 *tmeta = nullptr;          // per-tile compression records
    unsigned long long *zpts = nullptr;   // points in compressed tiles (device counter)
    bool use_xz = false;             // the current layout has a compressed stream
    bool tiles_lpt = false;          // tiles ordered longest candidate list first (PCM_TILE_LPT, A/B)
    size_t cap_xz = 0, cap_tmeta = 0;
    // crowded layouts (tight clusters): Morton levels of the in-cell order and the tile lists
    int zlev = 0;
    float4 *tbox = nullptr;          // [tile][2] exact point box
    uint32_t *tl_cnt = nullptr;      // [tile] list length (tiles of FULL cells) or FULL
    float4 *tl_rec = nullptr;        // [tile][TLMAX]
    int32_t *tl_lab = nullptr;       // [tile][TLMAX]
    uint32_t *zcnt = nullptr;        // occupancy sample counts [ncells + 1]
    size_t cap_tbox = 0, cap_tlc = 0, cap_tlr = 0, cap_tll = 0, cap_zcnt = 0;
    uint32_t *perm = nullptr;
    uint32_t *dmap = nullptr;        // [2][n] the layout sort's per-pass position maps (labels back to row order)
    size_t cap_dmap = 0;
    bool has_dmap = false;           // the current layout kept them (2-pass sorts)
    void *lab = nullptr;             // sorted-order labels: uint16 when k <= 65535, else int32
    uint32_t *cell_start = nullptr;
    uint32_t *sub_start = nullptr;   // [(ncells << d) + 1]: first sorted point of every sub-cell (half-cell per axis)
    int sub = 0;                     // the current layout is sorted by sub-cell
    size_t cap_sub = 0;
    uint32_t *tile_off = nullptr;    // [ncells+1] first tile of each cell
    uint4 *tiles = nullptr;
    int num_cu = 256;
    uint32_t *fc_cnt = nullptr;
    float4 *fc_rec = nullptr;
    int32_t *fc_lab = nullptr;
    float4 *C = nullptr, *Cn = nullptr;
    float4 *cref = nullptr;                    // [2][K] reference centres of the candidate lists (k_upd / k_lists)
    double *shbuf = nullptr;                   // [K] squared centre shifts of one iteration (k_upd's shift tree)
    UpdPart *upart = nullptr;                  // [ceil(K / UPD_TPB)] k_upd's per-block records
    uint32_t *cl_cnt = nullptr;                // [ncoarse] coarse candidate lists (k_coarse; split layouts)
    int32_t *cl_idx = nullptr;                 // [ncoarse][cand_capc]
    size_t cap_clc = 0, cap_cli = 0;
    double drift_alpha = 2.0, drift_kappa = 0.05;  // candidate-list reuse policy (see k_upd)
    unsigned long long *prev = nullptr;        // raw statistics of the previous iteration
    int iscale = 0;                  // exact-inertia weight exponent (from the global q)
    unsigned long long *partials = nullptr, *stats = nullptr, *hist_changed = nullptr;
    unsigned long long *stats_own = nullptr;   // engine-owned; `stats` may point at a bound buffer
    unsigned long long *held = nullptr;        // statistics of a halted iteration
    double *hist_shift = nullptr;
    Ctrl *ctrl = nullptr;
    float *bbox_part = nullptr;
    unsigned *nonfinite = nullptr;
    double *bbox_out = nullptr;
    unsigned long long *cand_stats = nullptr;
    int *rank_buf = nullptr;
    int rank_cap = 0;
    int *empty_idx = nullptr;        // [K] scratch of the relocation kernel
    uint32_t *ntiles_dev = nullptr;  // tile count of the current layout (written by k_tile_total)
    size_t cap_xs = 0, cap_lab = 0, cap_perm = 0, cap_cells = 0, cap_fc = 0, cap_tiles = 0, cap_ws = 0;
    void *ws = nullptr;              // layout / relocation scratch arena
    Ctrl ctrl_host{};
    // optional kernel timing: event pairs per iteration, summed on read
    static constexpr int TEV = 64;
    bool timing = false;
    hipEvent_t ev[TEV][4] = {};
    int ev_next = 0, ev_pending = 0;
    double t_sum[3] = {0, 0, 0};
    long long t_count = 0;
};

namespace {

const int BBOX_BLOCKS = 1024;

size_t tsize(int dtype) { return dtype == PCM_F16 ? 2 : 4; }

// Internal sorted-order labels are uint16 when every label fits (saves 4 B/pt/iter of HBM).
#ifdef PCM_DBG_LABEL32
bool small_labels(const pcm_engine *) { return false; }
#else
bool small_labels(const pcm_engine *e) { return e->k <= 65535; }
#endif
size_t lsize(const pcm_engine *e) { return small_labels(e) ? 2 : 4; }

int check_device(pcm_engine *e) {
    int cur = -1;
    HIPCHK(hipGetDevice(&cur));
    if (cur != e->device)
        return fail(PCM_E_STATE, "current HIP device " + std::to_string(cur) + " != engine device " +
                                     std::to_string(e->device));
    return 0;
}

template <typename F>
int dispatch_d(int d, F &&f) {
    switch (d) {
        case 1: return f(std::integral_constant<int, 1>{});
        case 2: return f(std::integral_constant<int, 2>{});
        case 3: return f(std::integral_constant<int, 3>{});
        case 4: return f(std::integral_constant<int, 4>{});
    }
    return fail(PCM_E_ARG, "d must be 1..4");
}

template <typename F>
int dispatch_td(int dtype, int d, F &&f) {
    if (dtype == PCM_F16)
        return dispatch_d(d, [&](auto DD) { return f(__half{}, DD); });
    return dispatch_d(d, [&](auto DD) { return f(float{}, DD); });
}

template <typename F>
int dispatch_l(const pcm_engine *e, F &&f) {
    if (small_labels(e)) return f(uint16_t{});
    return f(int32_t{});
}

// LSD record sort (pcm_sort.hpp): passes, chunking and workspace offsets.
struct RsPlan {
    int npass = 1, wb = 8;
    long long nblk = 1, ent = RS_DIG;
    long long nseg = 1;
    size_t o_ra = 0, o_rb = 0, o_hist = 0, o_goff = 0, o_segb = 0, total = 0;
};

template <typename TT, int D>
void rs_plan(long long n, unsigned bits, RsPlan &p) {
    using R = PRec<TT, D>;
    constexpr int CH = RsCfg<TT, D>::CH;
    p.npass = std::max(1, (int)((bits + 7) / 8));
    p.wb = (int)((bits + p.npass - 1) / p.npass);
    p.nblk = std::max(1LL, (n + CH - 1) / CH);
    p.ent = (long long)RS_DIG * p.nblk;
    p.nseg = (p.nblk + RS_SEG - 1) / RS_SEG;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t at = o; o = (o + std::max<size_t>(bytes, 8) + 255) / 256 * 256; return at; };
    p.o_ra = take(p.npass >= 2 ? n * sizeof(R) : 0);
    p.o_rb = take(p.npass >= 3 ? n * sizeof(R) : 0);
    p.o_hist = take(p.ent * 4);
    p.o_goff = take(p.ent * 4);
    p.o_segb = take((size_t)p.nseg * RS_DIG * 4);
    p.total = o;
}

// XCD-aware block orders (xcd_block), a bit mask: 1 the sort scatters, 2 k_lloyd1's tiles, 4 the label
// gathers
static int xcd_mode() {
    static const int m = [] { const char *v = std::getenv("PCM_XCD"); return v ? std::atoi(v) : 7; }();
    return m;
}

// 16-B row loads of the caller's X in the sort's first count pass (X 16-B aligned; PCM_SORT_VEC=0: the
// 4-B loads, A/B).  The same staged through LDS in the first scatter measured 899-901 -> 909-916 us
// (profiles/rd6_sort_count_vec.txt), so the scatter keeps its 4-B loads.
static int sort_vec(const void *X) {
    static const int m = [] { const char *v = std::getenv("PCM_SORT_VEC"); return v ? std::atoi(v) : 1; }();
    return ((uintptr_t)X & 15u) == 0u ? m : 0;
}

// Sort the caller's rows X into cell order: AoSoA-4 xs (zero padded to npad)
// and perm (sorted position -> row).
template <typename TT, int D>
int rs_sort(const TT *X, long long n, long long npad, const Grid &g, int with_sub, int zlev, unsigned bits,
            const RsPlan &p, char *wb, TT *xs, uint32_t *perm, hipStream_t s, uint32_t *dmaps = nullptr) {
    using R = PRec<TT, D>;
    R *ra = (R *)(wb + p.o_ra), *rb = (R *)(wb + p.o_rb);
    uint32_t *hist = (uint32_t *)(wb + p.o_hist), *goff = (uint32_t *)(wb + p.o_goff),
             *segb = (uint32_t *)(wb + p.o_segb);
    const int grid = (int)p.nblk;
    for (int q = 0; q < p.npass; ++q) {
        const int shift = q * p.wb, width = std::min(p.wb, (int)bits - shift);
        const bool from_x = q == 0, to_xs = q == p.npass - 1;
        const R *rin = from_x ? nullptr : (((q - 1) & 1) ? rb : ra);
        R *rout = to_xs ? nullptr : ((q & 1) ? rb : ra);
        if (from_x)
            k_rs_count<TT, D, true><<<grid, RS_CTPB, 0, s>>>(X, rin, n, g, with_sub, zlev, shift, width, hist,
                                                             sort_vec(X) & 1);
        else
            k_rs_count<TT, D, false><<<grid, RS_CTPB, 0, s>>>(X, rin, n, g, with_sub, zlev, shift, width, hist, 0);
        LAUNCHCHK();
        k_rs_colscan<<<(int)p.nseg, RS_DIG, 0, s>>>(hist, p.nblk, goff, segb);
        LAUNCHCHK();
        k_rs_segscan<<<1, RS_DIG, 0, s>>>(segb, p.nseg);
        LAUNCHCHK();
#define PCM_RS_SCATTER(FX, TX)                                                                                      \
    k_rs_scatter<TT, D, FX, TX><<<grid, RS_TPB, 0, s>>>(X, rin, n, g, with_sub, zlev, shift, width, goff, segb, rout, \
                                                        xs, perm, dmaps ? dmaps + (size_t)q * n : nullptr, xcd_mode() & 1)
        if (from_x && to_xs) PCM_RS_SCATTER(true, true);
        else if (from_x) PCM_RS_SCATTER(true, false);
        else if (to_xs) PCM_RS_SCATTER(false, true);
        else PCM_RS_SCATTER(false, false);
#undef PCM_RS_SCATTER
        LAUNCHCHK();
    }
    if (npad > n) {
        k_xs_pad<TT, D><<<1, 64, 0, s>>>(n, npad, xs);
        LAUNCHCHK();
    }
    return 0;
}

// The layout's buffers persist across layouts (a later cloud reuses them when
// they are large enough); invalidating a layout frees nothing.
void free_layout(pcm_engine *e) {
    e->layout_ready = false;
    e->fit_ready = false;
    e->has_dmap = false;
}

void free_buffers(pcm_engine *e) {
    void *ps[] = {e->xs, e->perm, e->lab, e->cell_start, e->tiles, e->fc_cnt, e->fc_rec, e->fc_lab, e->tile_off, e->ws,
                  e->sub_start, e->xz, e->tmeta, e->tbox, e->tl_cnt, e->tl_rec, e->tl_lab, e->zcnt, e->dmap,
                  e->cl_cnt, e->cl_idx};
    for (void *p : ps)
        if (p) (void)hipFree(p);
    e->dmap = nullptr; e->cap_dmap = 0; e->has_dmap = false;
    e->xs = nullptr; e->perm = nullptr; e->lab = nullptr; e->cell_start = nullptr; e->tiles = nullptr;
    e->tile_off = nullptr; e->ws = nullptr; e->sub_start = nullptr; e->cap_sub = 0;
    e->xz = nullptr; e->tmeta = nullptr; e->cap_xz = e->cap_tmeta = 0; e->use_xz = false;
    e->tbox = nullptr; e->tl_cnt = nullptr; e->tl_rec = nullptr; e->tl_lab = nullptr; e->zcnt = nullptr;
    e->cap_tbox = e->cap_tlc = e->cap_tlr = e->cap_tll = e->cap_zcnt = 0; e->zlev = 0;
    e->fc_cnt = nullptr; e->fc_rec = nullptr; e->fc_lab = nullptr;
    e->cl_cnt = nullptr; e->cl_idx = nullptr; e->cap_clc = e->cap_cli = 0;
    e->cap_xs = e->cap_lab = e->cap_perm = e->cap_cells = e->cap_fc = e->cap_tiles = e->cap_ws = 0;
    free_layout(e);
}

// Grow-only device buffer: reallocates (after freeing the old one) only when
// `need` bytes exceed the capacity.
template <typename P>
hipError_t ensure(P *&p, size_t &cap, size_t need) {
    if (p && need <= cap) return hipSuccess;
    if (p) {
        hipError_t err = hipFree((void *)p);
        p = nullptr;
        cap = 0;
        if (err != hipSuccess) return err;
    }
    void *q = nullptr;
    hipError_t err = hipMalloc(&q, std::max<size_t>(need, 256));
    if (err != hipSuccess) return err;
    p = static_cast<P *>(q);
    cap = std::max<size_t>(need, 256);
    return hipSuccess;
}

size_t align_up(size_t v, size_t a = 256) { return (v + a - 1) / a * a; }

// Roughly cubic grid of about `target` cells over the box [lo, hi]
// (degenerate axes get one cell); F = 4 fine cells per coarse cell per axis.
void make_grid(Grid &g, int d, const double *lo, const double *hi, double target) {
    g = Grid{};
    g.d = d;
    g.F = 4;   // fixed: k_cand assumes 4 fine cells per coarse cell per axis
    target = std::max(1.0, std::min(target, (double)(1 << 18)));
    double vol = 1.0;
    int nondeg = 0;
    double maxext = 0.0;
    for (int a = 0; a < MAXD; ++a) {
        g.G[a] = 1;
        g.GC[a] = 1;
    }
    for (int a = 0; a < d; ++a) {
        double ex = hi[a] - lo[a];
        g.ext[a] = ex;
        g.lo[a] = lo[a];
        maxext = std::max(maxext, ex);
        if (ex > 0) {
            vol *= ex;
            nondeg++;
        }
    }
    if (nondeg > 0) {
        double sz = std::pow(vol / target, 1.0 / nondeg);
        for (int a = 0; a < d; ++a) {
            if (g.ext[a] > 0) {
                long long G = std::llround(g.ext[a] / sz);
                g.G[a] = (int)std::max(1LL, std::min(G, 4096LL));
            }
        }
    }
    long long nc = 1;
    for (int a = 0; a < d; ++a) nc *= g.G[a];
    while (nc > (1LL << 20)) {   // keep keys and candidate tables bounded
        int amax = 0;
        for (int a = 1; a < d; ++a)
            if (g.G[a] > g.G[amax]) amax = a;
        g.G[amax] = std::max(1, g.G[amax] / 2);
        nc = 1;
        for (int a = 0; a < d; ++a) nc *= g.G[a];
    }
    long long ncc = 1;
    for (int a = 0; a < d; ++a) {
        g.w[a] = g.ext[a] / g.G[a];
        g.inv[a] = g.ext[a] > 0 ? (double)g.G[a] / g.ext[a] : 0.0;
        g.mg[a] = 1e-7 * g.ext[a];
        g.GC[a] = (g.G[a] + g.F - 1) / g.F;
        ncc *= g.GC[a];
    }
    g.ncells = nc;
    g.ncoarse = ncc;
    // fp32 distances overflow beyond ~1.8e19: no pruning then (brute force is exact)
    g.prune = (maxext < 1e18) ? 1 : 0;
}

// The Lloyd engine's pruning grid: about min(32 K, n / 2800) cells -- ~2.8k
// points per cell: fewer, fuller tiles (a tile round is 1024 points) outweigh
// the slightly longer candidate lists (swept on 12.5M / 100M clouds).
void choose_grid(pcm_engine *e) {
    // D = 4: smaller cells (~1k points) shorten the lists more than the tiles
    // cost (config-5 shape: 20736 -> 65536 cells, 913 -> 846 us per iteration)
    // (a spatial shard holds about n / n_global of the centres: the cap scales with it)
    // D = 4 slabs: 48 cells per centre (config-5 8-way slab, 13718 -> 27783 cells,
    // lists 7.1 -> 5.3, one tile per cell: 280 -> 250 us per rank; 36501 cells 265,
    // profiles/rd4_c5_slab_grid.txt); D <= 3: 32 (the config-4 slab sweep)
    const double share = e->n_global > 0 ? std::min(1.0, (double)e->n / (double)e->n_global) : 1.0;
    const double per_centre = e->d >= 4 ? 48.0 : 32.0;
    double target = std::min(per_centre * e->k * share, (double)e->n / (e->d >= 4 ? 1000.0 : 2800.0));
    if (const char *ov = std::getenv("PCM_CELL_TARGET")) target = std::atof(ov);   // tuning sweeps only
    make_grid(e->g, e->d, e->lo, e->hi, target);
    if (e->k <= 1) e->g.prune = 0;
}

int blocks_for(long long n, int bs = 256) { return (int)std::max(1LL, (n + bs - 1) / bs); }

// Exact-inertia exponent s (oracle/lloyd_ref.py inertia_scale): the global
// exponents give |x_a|, |c_a| < 2^(QBITS - q_a), so every canonical distance
// is below bound = sum_a 4^(QBITS + 1 - q_a) (times 1 + 2^-20 for rounding);
// s = 64 - e with bound' < 2^e keeps trunc(d * 2^s) < 2^64.
int inertia_scale(const int32_t *q, int d) {
    double bound = 0.0;
    for (int a = 0; a < d; ++a) bound += std::ldexp(1.0, 2 * (QBITS + 1 - q[a]));
    int e = 0;
    (void)std::frexp(bound * (1.0 + std::ldexp(1.0, -20)), &e);
    return 64 - e;
}

}  // namespace

extern "C" {

int pcm_abi_version(void) { return PCM_ABI_VERSION; }

double pcm_inertia_value(const uint64_t *limbs, int scale, uint32_t overflow) {
    if (!limbs) return 0.0;
    if (overflow) return HUGE_VAL;
    const unsigned __int128 v = (unsigned __int128)limbs[0] + ((unsigned __int128)limbs[1] << 32) +
                                ((unsigned __int128)limbs[2] << 64);
    return std::ldexp((double)v, -scale);   // one correctly rounded conversion, exact scaling
}

int pcm_last_error(char *buf, size_t n) {
    if (!buf || n == 0) return PCM_E_ARG;
    std::snprintf(buf, n, "%s", g_err.c_str());
    return 0;
}

int pcm_engine_create(int device, int d, int k, int dtype, int max_iter, pcm_engine **out) {
    if (!out) return fail(PCM_E_ARG, "out is null");
    *out = nullptr;
    if (d < 1 || d > MAXD) return fail(PCM_E_ARG, "d must be 1..4");
    if (k < 1 || k > (1 << 20)) return fail(PCM_E_ARG, "k out of range");
    if (dtype != PCM_F32 && dtype != PCM_F16) return fail(PCM_E_ARG, "dtype must be PCM_F32 or PCM_F16");
    if (max_iter < 1) return fail(PCM_E_ARG, "max_iter must be >= 1");
    pcm_engine *e = new pcm_engine();
    e->device = device;
    e->d = d;
    e->k = k;
    e->dtype = dtype;
    e->max_iter_cap = max_iter;
    int rc = check_device(e);
    if (rc) { delete e; return rc; }
    if (hipDeviceGetAttribute(&e->num_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        e->num_cu < 1)
        e->num_cu = 256;
    const size_t nstat = (size_t)k * (d + 1) + 1;
    hipError_t err = hipSuccess;
    err = err ? err : hipMalloc(&e->C, (size_t)k * sizeof(float4));
    err = err ? err : hipMalloc(&e->Cn, (size_t)k * sizeof(float4));
    err = err ? err : hipMalloc(&e->cref, (size_t)2 * k * sizeof(float4));
    err = err ? err : hipMalloc(&e->shbuf, (size_t)k * sizeof(double));
    err = err ? err : hipMalloc(&e->upart, (size_t)blocks_for(k, UPD_TPB) * sizeof(UpdPart));
    err = err ? err : hipMalloc(&e->prev, nstat * sizeof(unsigned long long));
    err = err ? err : hipMalloc(&e->partials, (size_t)2 * k * (d + 1) * sizeof(unsigned long long));
    err = err ? err : hipMalloc(&e->stats_own, nstat * sizeof(unsigned long long));
    e->stats = e->stats_own;
    err = err ? err : hipMalloc(&e->held, nstat * sizeof(unsigned long long));
    err = err ? err : hipMalloc(&e->hist_changed, (size_t)max_iter * sizeof(unsigned long long));
    err = err ? err : hipMalloc(&e->hist_shift, (size_t)max_iter * sizeof(double));
    err = err ? err : hipMalloc(&e->ctrl, sizeof(Ctrl));
    err = err ? err : hipMalloc(&e->bbox_part, (size_t)BBOX_BLOCKS * 2 * MAXD * sizeof(float));
    err = err ? err : hipMalloc(&e->nonfinite, sizeof(unsigned));
    err = err ? err : hipMalloc(&e->bbox_out, 2 * MAXD * sizeof(double));
    err = err ? err : hipMalloc(&e->cand_stats, 6 * sizeof(unsigned long long));
    err = err ? err : hipMalloc(&e->empty_idx, (size_t)k * sizeof(int));
    err = err ? err : hipMalloc(&e->ntiles_dev, 2 * sizeof(uint32_t));
    err = err ? err : hipMalloc(&e->zpts, 32 * 16 * sizeof(unsigned long long));
    err = err ? err : hipHostMalloc((void **)&e->ntiles_host, sizeof(uint32_t), hipHostMallocDefault);
    err = err ? err : hipHostMalloc((void **)&e->ctrl_pin, sizeof(Ctrl), hipHostMallocDefault);
    err = err ? err : hipEventCreateWithFlags(&e->st_ev, hipEventDisableTiming);
    err = err ? err : hipMemset(e->partials, 0, (size_t)2 * k * (d + 1) * sizeof(unsigned long long));
    err = err ? err : hipMemset(e->ctrl, 0, sizeof(Ctrl));
    if (err != hipSuccess) {
        pcm_engine_destroy(e);
        return fail(PCM_E_NOMEM, std::string("engine allocation: ") + hipGetErrorString(err));
    }
    // candidate-list reuse: budget = alpha x the last centre shift, at most kappa x
    // the smallest cell width (tuning sweeps may override; alpha = 0 disables reuse)
    if (const char *v = std::getenv("PCM_DRIFT_ALPHA")) e->drift_alpha = std::atof(v);
    if (const char *v = std::getenv("PCM_DRIFT_KAPPA")) e->drift_kappa = std::atof(v);
    *out = e;
    return 0;
}

int pcm_engine_destroy(pcm_engine *e) {
    if (!e) return 0;
    for (int i = 0; i < pcm_engine::TEV; ++i)
        for (int j = 0; j < 4; ++j)
            if (e->ev[i][j]) (void)hipEventDestroy(e->ev[i][j]);
    free_buffers(e);
    void *ps[] = {e->C, e->Cn, e->cref, e->shbuf, e->upart, e->prev, e->partials, e->stats_own, e->held, e->hist_changed, e->hist_shift, e->ctrl,
                  e->bbox_part, e->nonfinite, e->bbox_out, e->cand_stats, e->rank_buf, e->empty_idx, e->ntiles_dev,
                  e->grows, e->zpts};
    for (void *p : ps)
        if (p) (void)hipFree(p);
    if (e->ntiles_host) (void)hipHostFree(e->ntiles_host);
    if (e->ctrl_pin) (void)hipHostFree(e->ctrl_pin);
    if (e->st_ev) (void)hipEventDestroy(e->st_ev);
    delete e;
    return 0;
}

int pcm_layout_bbox(pcm_engine *e, const void *X, int64_t n, void *stream, double *lo, double *hi, double *maxabs) {
    if (!e || (!X && n > 0) || n < 0 || !lo || !hi || !maxabs) return fail(PCM_E_ARG, "bad argument");
    if (n >= (1LL << 32) - 8) return fail(PCM_E_ARG, "n must be < 2^32 per engine");
    if (int rc = check_device(e)) return rc;
    hipStream_t s = (hipStream_t)stream;
    e->n = n;
    e->n_global = n;
    e->has_rows = false;
    e->have_bbox = false;
    free_layout(e);
    if (n == 0) {
        for (int a = 0; a < e->d; ++a) lo[a] = hi[a] = maxabs[a] = e->lo[a] = e->hi[a] = e->maxabs[a] = 0.0;
        e->have_bbox = true;
        return 0;
    }
    HIPCHK(hipMemsetAsync(e->nonfinite, 0, sizeof(unsigned), s));
    int nblk = (int)std::min<long long>(BBOX_BLOCKS, (n + 255) / 256);
    int rc = dispatch_td(e->dtype, e->d, [&](auto T, auto DD) -> int {
        using TT = decltype(T);
        constexpr int D = decltype(DD)::value;
        k_bbox_partial<TT, D><<<nblk, 256, 0, s>>>((const TT *)X, n, e->bbox_part, e->nonfinite);
        LAUNCHCHK();
        k_bbox_final<D><<<1, 256, 0, s>>>(e->bbox_part, nblk, e->bbox_out);
        LAUNCHCHK();
        return 0;
    });
    if (rc) return rc;
    double hb[2 * MAXD];
    unsigned nf = 0;
    HIPCHK(hipMemcpyAsync(hb, e->bbox_out, 2 * e->d * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&nf, e->nonfinite, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (nf) return fail(PCM_E_NONFINITE, "input points contain NaN or Inf");
    for (int a = 0; a < e->d; ++a) {
        e->lo[a] = lo[a] = hb[a];
        e->hi[a] = hi[a] = hb[e->d + a];
        e->maxabs[a] = maxabs[a] = std::max(std::fabs(hb[a]), std::fabs(hb[e->d + a]));
    }
    e->have_bbox = true;
    return 0;
}

static int lloyd_slots(const pcm_engine *e);

int pcm_layout_shard(pcm_engine *e, const uint32_t *rows, int64_t n_global, void *stream) {
    if (!e || (!rows && e->n > 0)) return fail(PCM_E_ARG, "bad argument");
    if (!e->have_bbox) return fail(PCM_E_STATE, "pcm_layout_bbox must run first");
    if (n_global < e->n || n_global >= (1LL << 32)) return fail(PCM_E_ARG, "n_global must be in [n, 2^32)");
    if (int rc = check_device(e)) return rc;
    free_layout(e);
    e->n_global = n_global;
    e->has_rows = true;
    if (e->n == 0) return 0;
    HIPCHK(ensure(e->grows, e->cap_grows, (size_t)e->n * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(e->grows, rows, (size_t)e->n * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                          (hipStream_t)stream));
    return 0;
}

static unsigned cell_bits(long long nc) {
    unsigned b = 0;
    while ((1LL << b) < nc) ++b;
    return b;
}

// Crowded-cell detection (tile lists, k_tile_cand): the cell counts of a strided
// sample of up to 2^20 points, scaled to n.  A cell expected to hold more than
// ZCROWD tiles' worth of points gets its points ordered by zlev Morton levels,
// enough that a level-zlev box of the fullest cell holds ~1/8 tile (the lists
// are only needed when K exceeds CAPF).  One host read-back of 4 bytes.
// PCM_ZLEV forces the level count (tests: crowded order on small clouds).
static int choose_zlev(pcm_engine *e, const void *X, hipStream_t s) {
    e->zlev = 0;
    const long long n = e->n, nc = e->g.ncells;
    const int d = e->d;
    const unsigned cb = cell_bits(nc);
    const int zmax = std::min(6, (int)((32 - (int)cb) / d));
    if (const char *v = std::getenv("PCM_ZLEV")) {
        e->zlev = std::max(0, std::min(zmax, std::atoi(v)));
        return 0;
    }
    constexpr double ZCROWD = 4.0;
    if (!e->g.prune || e->k <= CAPF || n < (long long)(ZCROWD * e->tile_cap) || zmax < 1) return 0;
    const long long m = std::min(n, 1LL << 20), stride = n / m;
    HIPCHK(ensure(e->zcnt, e->cap_zcnt, (size_t)(nc + 1) * sizeof(uint32_t)));
    HIPCHK(hipMemsetAsync(e->zcnt, 0, (size_t)(nc + 1) * sizeof(uint32_t), s));
    int rc = dispatch_td(e->dtype, d, [&](auto T, auto DD) -> int {
        using TT = decltype(T);
        constexpr int D = decltype(DD)::value;
        k_zsample<TT, D><<<blocks_for(m), 256, 0, s>>>((const TT *)X, m, stride, e->g, e->zcnt);
        LAUNCHCHK();
        return 0;
    });
    if (rc) return rc;
    k_umax<<<(int)std::min<long long>(1024, std::max(1LL, (nc + 255) / 256)), 256, 0, s>>>(e->zcnt, nc, e->zcnt + nc);
    LAUNCHCHK();
    uint32_t mx = 0;
    HIPCHK(hipMemcpyAsync(&mx, e->zcnt + nc, sizeof(mx), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const double est = (double)mx * (double)n / (double)m;
    if (est <= ZCROWD * e->tile_cap) return 0;
    int z = 1;
    while (z < zmax && std::ldexp(1.0, d * z) < 8.0 * est / e->tile_cap) ++z;
    e->zlev = z;
    return 0;
}

// Grow the point-sized persistent buffers for a cloud of up to n points and
// touch them, so that the first layout of a process allocates nothing large.
// The first allocations of a fresh process map and clear new VRAM (~17 ms for
// config 3's ~5 GB); the buffers are the ones pcm_layout_build
// grows: points (xs), labels, perm, the sort's records (ws, sized for the
// worst-case 4-pass plan plus the per-cell arrays of the largest grid), its
// position maps (dmap) and the compressed stream (xz, fp32 D = 3).  Crowded
// layouts' tile-list storage is sized by the tiles and stays lazy.
int pcm_engine_reserve(pcm_engine *e, int64_t n, void *stream) {
    if (!e || n < 0) return fail(PCM_E_ARG, "bad argument");
    if (n >= (1LL << 28) - 32) return fail(PCM_E_ARG, "at most 2^28 - 32 points per engine");
    if (int rc = check_device(e)) return rc;
    if (n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const long long npad = ((n + 3) / 4) * 4 + 4;
    const size_t ts = tsize(e->dtype);
    size_t scan_bytes = 0;
    if (rocprim::exclusive_scan(nullptr, scan_bytes, (uint32_t *)nullptr, (uint32_t *)nullptr, 0u, (size_t)1 << 20,
                                rocprim::plus<uint32_t>(), s) != hipSuccess)
        return fail(PCM_E_HIP, "reserve: rocprim size query failed");
    size_t ws_need = 0;
    dispatch_td(e->dtype, e->d, [&](auto T, auto DD) -> int {
        RsPlan p;
        rs_plan<decltype(T), decltype(DD)::value>(n, 32, p);
        ws_need = align_up(p.total) + align_up(((size_t)1 << 20) * 4) + scan_bytes;
        return 0;
    });
    struct Buf { void **p; size_t *cap; size_t need; };
    Buf bufs[] = {
        {(void **)&e->xs, &e->cap_xs, (size_t)e->d * npad * ts},
        {(void **)&e->lab, &e->cap_lab, (size_t)npad * lsize(e)},
        {(void **)&e->perm, &e->cap_perm, (size_t)n * sizeof(uint32_t)},
        {(void **)&e->ws, &e->cap_ws, ws_need},
        {(void **)&e->dmap, &e->cap_dmap, (size_t)2 * n * sizeof(uint32_t)},
        {(void **)&e->xz, &e->cap_xz, (e->dtype == PCM_F32 && e->d == 3) ? (size_t)align_up(npad) * 8 : 0},
    };
    free_layout(e);   // a grown buffer no longer holds the old layout
    for (const Buf &b : bufs) {
        if (b.need == 0) continue;
        HIPCHK(ensure(*b.p, *b.cap, b.need));
        HIPCHK(hipMemsetAsync(*b.p, 0, *b.cap, s));
    }
    return 0;
}

int pcm_layout_build(pcm_engine *e, const void *X, const int32_t *q, int64_t gidx0, void *stream) {
    if (!e || !q) return fail(PCM_E_ARG, "bad argument");
    if (!e->have_bbox) return fail(PCM_E_STATE, "pcm_layout_bbox must run first");
    if (int rc = check_device(e)) return rc;
    hipStream_t s = (hipStream_t)stream;
    free_layout(e);
    for (int a = 0; a < MAXD; ++a) e->qe.q[a] = a < e->d ? q[a] : 0;
    e->iscale = inertia_scale(q, e->d);
    e->gidx0 = gidx0;
    const long long n = e->n;
    e->npad = ((n + 3) / 4) * 4 + 4;
    // the assign kernel addresses points with 32-bit offsets and uses offset
    // 0x0ffffff0 (points) as its always-out-of-range prefetch
    if (e->npad >= 0x0ffffff0LL) return fail(PCM_E_ARG, "at most 2^28 - 32 points per engine (shard larger clouds)");
    choose_grid(e);
    const long long nc = e->g.ncells;
    const size_t ts = tsize(e->dtype);
    // points per tile (<= TILE): PCM_TILE_CAP for tuning sweeps only
    static const uint32_t tcap = [] {
        const char *v = std::getenv("PCM_TILE_CAP");
        const int c = v ? std::atoi(v) : TILE;
        return (uint32_t)std::min(TILE, std::max(4 * TPB, c));
    }();
    e->tile_cap = tcap;
    // every cell holds ceil(count / cap) <= count / cap + 1 tiles
    e->ntiles_cap = nc + n / e->tile_cap + 1;
    e->ntiles = -1;

    // persistent layout buffers (no allocation when an earlier layout was as large)
    HIPCHK(ensure(e->xs, e->cap_xs, (size_t)e->d * e->npad * ts));
    HIPCHK(ensure(e->lab, e->cap_lab, (size_t)e->npad * lsize(e)));
    HIPCHK(ensure(e->perm, e->cap_perm, (size_t)std::max(1LL, n) * sizeof(uint32_t)));
    {
        // cell_start, tile_off: nc + 1 each; fc_cnt: nc -- one grow-only allocation each
        size_t need = (size_t)(nc + 1) * sizeof(uint32_t);
        size_t c0 = e->cap_cells, c1 = e->cap_cells;
        HIPCHK(ensure(e->cell_start, c0, need));
        HIPCHK(ensure(e->tile_off, c1, need));
        size_t c2 = e->cap_cells;
        HIPCHK(ensure(e->fc_cnt, c2, need));
        e->cap_cells = std::min(c0, std::min(c1, c2));
        size_t f0 = e->cap_fc, f1 = e->cap_fc;
        HIPCHK(ensure(e->sub_start, e->cap_sub, (size_t)((nc << e->d) + 1) * sizeof(uint32_t)));
        HIPCHK(ensure(e->fc_rec, f0, (size_t)nc * CAPF * sizeof(float4)));
        HIPCHK(ensure(e->fc_lab, f1, (size_t)nc * CAPF * sizeof(float4)));   // sized like fc_rec: one capacity
        e->cap_fc = std::min(f0, f1);
    }
    HIPCHK(ensure(e->tiles, e->cap_tiles, (size_t)e->ntiles_cap * sizeof(uint4)));
    HIPCHK(hipMemsetAsync(e->fc_rec, 0, (size_t)nc * CAPF * sizeof(float4), s));
    HIPCHK(hipMemsetAsync(e->fc_lab, 0, (size_t)nc * CAPF * sizeof(int32_t), s));
    HIPCHK(hipMemsetAsync(e->fc_cnt, 0, (size_t)nc * sizeof(uint32_t), s));

    if (n == 0) {
        HIPCHK(hipMemsetAsync(e->tile_off, 0, (size_t)(nc + 1) * sizeof(uint32_t), s));
        HIPCHK(hipMemsetAsync(e->cell_start, 0, (size_t)(nc + 1) * sizeof(uint32_t), s));
        HIPCHK(hipMemsetAsync(e->lab, 0xff, (size_t)e->npad * lsize(e), s));
        HIPCHK(hipMemsetAsync(e->xs, 0, (size_t)e->d * e->npad * ts, s));
        HIPCHK(hipMemsetAsync(e->ntiles_dev, 0, sizeof(uint32_t), s));
        e->ntiles = 0;
        e->ntiles_cap = 0;
        e->layout_ready = true;
        return 0;
    }

    // sort key: cell id << d | sub-cell (which half of the cell per axis) on the
    // coarse grids whose k_lloyd1 variant uses sub-cell masks (the 16-slot D <= 3
    // one, see lloyd_slots); else the cell id
    e->sub = (e->d <= 3 && lloyd_slots(e) == LSLOT) ? 1 : 0;
    if (int rc = choose_zlev(e, X, s)) return rc;
    if (e->zlev > 0) e->sub = 0;
    const int sh = e->sub ? e->d : 0;
    const long long nsub = nc << sh;
    // Key order: the LSD record sort of pcm_sort.hpp (no random row gather, no
    // key array).  Measured at config 3: (key, row) pairs sort +
    // 12-B row gather 1.4 + 2.9 ms; rocprim pairs sort with 16-B point records
    // as values 3.4 ms in all; counting sorts slower still (global-atomic
    // counters 3.65 + 7.35 ms, LDS-privatised 0.39 + 7.55 ms: single-point
    // writes into 32768 key ranges do not merge).
    unsigned bits = 1;
    while ((1LL << bits) < nsub) ++bits;
    if (e->zlev > 0) bits = cell_bits(nc) + (unsigned)(e->d * e->zlev);   // <= 32 (choose_zlev)
    uint32_t *tcnt = nullptr;
    void *tmp = nullptr;
    size_t scan_bytes = 0;
    if (rocprim::exclusive_scan(nullptr, scan_bytes, (uint32_t *)nullptr, (uint32_t *)nullptr, 0u, (size_t)nc,
                                rocprim::plus<uint32_t>(), s) != hipSuccess)
        return fail(PCM_E_HIP, "layout: rocprim size query failed");
    int rc = dispatch_td(e->dtype, e->d, [&](auto T, auto DD) -> int {
        using TT = decltype(T);
        constexpr int D = decltype(DD)::value;
        RsPlan p;
        rs_plan<TT, D>(n, bits, p);
        const size_t o_tcnt = align_up(p.total), o_tmp = align_up(o_tcnt + nc * 4), ws_need = o_tmp + scan_bytes;
        if (ensure(e->ws, e->cap_ws, ws_need) != hipSuccess) return fail(PCM_E_NOMEM, "layout scratch");
        char *wb = (char *)e->ws;
        tcnt = (uint32_t *)(wb + o_tcnt);
        tmp = wb + o_tmp;
        // 2-pass sorts keep their position maps for pcm_labels
        e->has_dmap = p.npass == 2 && ensure(e->dmap, e->cap_dmap, (size_t)2 * n * sizeof(uint32_t)) == hipSuccess;
        if (int rc2 = rs_sort<TT, D>((const TT *)X, n, e->npad, e->g, e->sub, e->zlev, bits, p, wb, (TT *)e->xs,
                                     e->perm, s, e->has_dmap ? e->dmap : nullptr))
            return rc2;
        // cell (or sub-cell) starts by binary search over the sorted points
        if (e->zlev > 0)   // Morton-ordered cells: the keys' cell bits
            k_cell_starts_xs<TT, D><<<blocks_for(nc + 1), 256, 0, s>>>((const TT *)e->xs, n, e->g, 0, e->zlev, nc,
                                                                      e->cell_start, e->d * e->zlev);
        else
            k_cell_starts_xs<TT, D><<<blocks_for(nsub + 1), 256, 0, s>>>((const TT *)e->xs, n, e->g, e->sub, 0, nsub,
                                                                        e->sub_start, 0);
        LAUNCHCHK();
        return 0;
    });
    if (rc) return rc;
    if (e->zlev == 0) {
        k_cell_from_sub<<<blocks_for(nc + 1), 256, 0, s>>>(e->sub_start, nc, sh, e->cell_start);
        LAUNCHCHK();
    }
    k_tile_counts<<<blocks_for(nc), 256, 0, s>>>(e->cell_start, nc, tcnt, e->tile_cap);
    LAUNCHCHK();
    size_t sb = scan_bytes;
    if (rocprim::exclusive_scan(tmp, sb, tcnt, e->tile_off, 0u, (size_t)nc, rocprim::plus<uint32_t>(), s) != hipSuccess)
        return fail(PCM_E_HIP, "layout: tile scan");
    k_tile_total<<<1, 64, 0, s>>>(e->tile_off, tcnt, nc, e->ntiles_dev);
    LAUNCHCHK();
    k_tile_write<<<blocks_for(nc), 256, 0, s>>>(e->cell_start, e->tile_off, nc, e->tiles, e->tile_cap);
    LAUNCHCHK();
    e->tiles_lpt = false;
    // the exact tile count for the grids of the per-tile kernels (the bound
    // ntiles_cap launched ~1.7x as many blocks at config 3, the excess exiting
    // after one memory latency: a drain tail on every assign launch)
    HIPCHK(hipMemcpyAsync(e->ntiles_host, e->ntiles_dev, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    // compressed point stream for k_lloyd1 (fp32, D = 3; PCM_XZ=0 disables it: A/B measurement only)
    static const bool xz_on = [] { const char *v = std::getenv("PCM_XZ"); return !(v && std::atoi(v) == 0); }();
    e->use_xz = xz_on && e->dtype == PCM_F32 && e->d == 3;
    HIPCHK(hipMemsetAsync(e->zpts, 0, 32 * 16 * sizeof(unsigned long long), s));
    if (e->use_xz) {
        HIPCHK(ensure(e->xz, e->cap_xz, (size_t)align_up(e->npad) * 8));   // whole 256-point blocks (zword)
        HIPCHK(ensure(e->tmeta, e->cap_tmeta, (size_t)e->ntiles_cap * sizeof(uint4)));
        k_tile_compress<<<(int)std::max(1LL, e->ntiles_cap), 256, 0, s>>>((const float *)e->xs, e->tiles, e->ntiles_dev, e->tmeta,
                                                           e->xz, e->zpts);
        LAUNCHCHK();
    }
    if (e->zlev > 0) {   // crowded layout: exact tile boxes and tile-list storage
        HIPCHK(ensure(e->tbox, e->cap_tbox, (size_t)e->ntiles_cap * 2 * sizeof(float4)));
        HIPCHK(ensure(e->tl_cnt, e->cap_tlc, (size_t)e->ntiles_cap * sizeof(uint32_t)));
        HIPCHK(ensure(e->tl_rec, e->cap_tlr, (size_t)e->ntiles_cap * TLMAX * sizeof(float4)));
        HIPCHK(ensure(e->tl_lab, e->cap_tll, (size_t)e->ntiles_cap * TLMAX * sizeof(int32_t)));
        rc = dispatch_td(e->dtype, e->d, [&](auto T, auto DD) -> int {
            using TT = decltype(T);
            constexpr int D = decltype(DD)::value;
            k_tile_box<TT, D><<<(int)e->ntiles_cap, 256, 0, s>>>((const TT *)e->xs, e->tiles, e->ntiles_dev, e->tbox);
            LAUNCHCHK();
            return 0;
        });
        if (rc) return rc;
    }
    // one host synchronisation at the end (the tile count; and choose_zlev's
    // occupancy read-back): X must not be modified by other streams meanwhile
    HIPCHK(hipStreamSynchronize(s));
    e->ntiles = (long long)*e->ntiles_host;
    if (e->ntiles > e->ntiles_cap) return fail(PCM_E_HIP, "layout: tile count exceeds its bound");
    e->layout_ready = true;
    return 0;
}

static int launch_candidates(pcm_engine *e, hipStream_t s, int gate);

// Longest-list-first tile order: the tile records (and their compression
// records) sorted by descending candidate-list length of their cell at the
// first lists, so k_lloyd1 dispatches its longest-lived blocks first and the
// short ones fill the tail (a block's lifetime follows its list length,
// DESIGN.md §4).  Where the tiles are few generations of resident blocks (the
// 8-way slab: 4096 tiles, 37.1 vs 39.1 us per assign) or D = 4 (config-5 shard,
// 299 vs 307 us) it pays; config 3's 32768 D = 3 tiles keep their spatial order
// and the XCD ranges (profiles/rd6_tile_lpt_ab.txt).  The statistics are exact
// integers, so the order changes no result.  PCM_TILE_LPT = 0 / 1 forces it.
static int tiles_order_lpt(pcm_engine *e, hipStream_t s) {
    static const int mode = [] { const char *v = std::getenv("PCM_TILE_LPT"); return v ? std::atoi(v) : -1; }();
    const bool want = mode == 1 || (mode < 0 && (e->d >= 4 || e->ntiles <= 16LL * e->num_cu));
    if (!want || e->zlev > 0 || e->ntiles < 2) return 0;   // crowded layouts: tile boxes and lists are per tile
    const unsigned nt = (unsigned)e->ntiles;
    size_t sort_bytes = 0;
    if (rocprim::radix_sort_pairs(nullptr, sort_bytes, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                  (uint32_t *)nullptr, (size_t)nt, 0u, 16u, s) != hipSuccess)
        return fail(PCM_E_HIP, "tile order: sort size");
    const size_t o_k1 = align_up((size_t)nt * 4), o_v0 = o_k1 + align_up((size_t)nt * 4), o_v1 = o_v0 + align_up((size_t)nt * 4),
                 o_t2 = o_v1 + align_up((size_t)nt * 4), o_m2 = o_t2 + align_up((size_t)nt * 16),
                 o_tmp = o_m2 + align_up((size_t)nt * 16), need = o_tmp + sort_bytes;
    if (ensure(e->ws, e->cap_ws, need) != hipSuccess) return fail(PCM_E_NOMEM, "tile order scratch");
    char *wb = (char *)e->ws;
    uint32_t *k0 = (uint32_t *)wb, *k1 = (uint32_t *)(wb + o_k1), *v0 = (uint32_t *)(wb + o_v0), *v1 = (uint32_t *)(wb + o_v1);
    uint4 *t2 = (uint4 *)(wb + o_t2), *m2 = (uint4 *)(wb + o_m2);
    k_tile_lpt_keys<<<blocks_for(nt), 256, 0, s>>>(e->tiles, e->fc_cnt, nt, k0, v0);
    LAUNCHCHK();
    size_t sb = sort_bytes;
    if (rocprim::radix_sort_pairs((void *)(wb + o_tmp), sb, k0, k1, v0, v1, (size_t)nt, 0u, 16u, s) != hipSuccess)
        return fail(PCM_E_HIP, "tile order: sort");
    k_tile_gather<<<blocks_for(nt), 256, 0, s>>>(e->tiles, e->use_xz ? e->tmeta : nullptr, v1, nt, t2, m2);
    LAUNCHCHK();
    HIPCHK(hipMemcpyAsync(e->tiles, t2, (size_t)nt * sizeof(uint4), hipMemcpyDeviceToDevice, s));
    if (e->use_xz) HIPCHK(hipMemcpyAsync(e->tmeta, m2, (size_t)nt * sizeof(uint4), hipMemcpyDeviceToDevice, s));
    e->tiles_lpt = true;
    return 0;
}

int pcm_fit_begin(pcm_engine *e, const float *C0, double tol, int max_iter, void *stream) {
    if (!e || !C0) return fail(PCM_E_ARG, "bad argument");
    if (!e->layout_ready) return fail(PCM_E_STATE, "layout not built");
    if (max_iter < 1 || max_iter > e->max_iter_cap) return fail(PCM_E_ARG, "max_iter exceeds the engine's cap");
    if (!(tol >= 0.0)) return fail(PCM_E_ARG, "tol must be >= 0");
    if (int rc = check_device(e)) return rc;
    hipStream_t s = (hipStream_t)stream;
    int rc = dispatch_d(e->d, [&](auto DD) -> int {
        constexpr int D = decltype(DD)::value;
        k_centers_in<D><<<blocks_for(e->k), 256, 0, s>>>(C0, e->k, e->C);
        LAUNCHCHK();
        return 0;
    });
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(e->lab, 0xff, (size_t)e->npad * lsize(e), s));   // "no label yet" (-1 / 0xffff)
    // previous raw statistics := 0: iteration 0 "converges" only for an empty cloud,
    // as sklearn's labels-vs-(-1) comparison does
    {   // prev, partials, stats and the histories := 0 in one launch (five memsets: ~5 us each)
        const long long w = (long long)e->k * (e->d + 1);
        ZeroSpans z{};
        z.p[0] = e->prev;         z.n[0] = w + 1;
        z.p[1] = e->partials;     z.n[1] = 2 * w;
        z.p[2] = e->stats;        z.n[2] = w + 1;
        z.p[3] = e->hist_changed; z.n[3] = e->max_iter_cap;
        z.p[4] = reinterpret_cast<unsigned long long *>(e->hist_shift); z.n[4] = e->max_iter_cap;   // 0.0 = all-zero bits
        long long tot = 0;
        for (int q = 0; q < 5; ++q) tot += z.n[q];
        k_zero_spans<<<(int)std::min<long long>(1024, (tot + 255) / 256), 256, 0, s>>>(z);
        LAUNCHCHK();
    }
    e->ctrl_host = Ctrl{};
    e->ctrl_host.max_iter = (uint32_t)max_iter;
    e->ctrl_host.tol = tol;
    HIPCHK(hipMemcpyAsync(e->ctrl, &e->ctrl_host, sizeof(Ctrl), hipMemcpyHostToDevice, s));
    e->fit_ready = true;
    // candidate lists of C0 (later iterations get theirs from k_lists / the resume path)
    if (int rc2 = launch_candidates(e, s, 0)) return rc2;
    return tiles_order_lpt(e, s);
}

// Candidate blocks per coarse cell: enough blocks to fill the chip on small
// (sharded) clouds; D = 4 coarse cells hold 256 fine cells.
// Measured (round-2 bpc sweep, tools/sweep.sh PCM_CAND_BPC_RT): 12.5M-point shard (64 coarse cells) 8 -> 39 us
// vs 4 -> 47 us per update; 100M (512 coarse cells) 1; D = 4, K = 4096: 32.
// Fine grids (short lists, the 8-slot k_lloyd1: an 8-way slab, 64 coarse cells)
// want about one block per CU (round-3 slab sweep, profiles/r3x_slab_sweep.txt:
// bpc 4 -> 18.6 us, 2 -> 19.2, 8 -> 21.0, 16 -> 31.2 per update).
static int lloyd_slots(const pcm_engine *e);
static int cand_bpc(const pcm_engine *e) {
    if (const char *ov = std::getenv("PCM_CAND_BPC_RT")) return std::max(1, std::atoi(ov));   // tuning sweeps only
    if (e->d >= 4) return 32;
    const long long per = (lloyd_slots(e) == 8 ? 1LL : 2LL) * e->num_cu;
    long long b = (per + e->g.ncoarse - 1) / std::max(1LL, e->g.ncoarse);
    return (int)std::max(1LL, std::min(8LL, b));
}

// D = 4 coarse cells hold 4^4 = 256 fine cells and long lists: their lists are
// built in three levels -- k_coarse (one block per coarse cell, all K centres,
// once) -> one block per mid cell (2^4 fine cells) refining its coarse parent's
// list -> its 16 fine cells (k_cand / k_lists with FC = 2) -- instead of 32
// blocks per coarse cell each recomputing the coarse list and then pruning it
// per fine cell (config-5 shard: 252 us of k_cand per iteration).
static bool split_coarse(const pcm_engine *e) { return e->g.prune && e->d >= 4; }
static long long n_mid(const pcm_engine *e) {
    long long m = 1;
    for (int a = 0; a < e->d; ++a) m *= (e->g.G[a] + 1) / 2;
    return m;
}

// coarse-list storage of the current layout (split layouts only)
static int ensure_coarse(pcm_engine *e) {
    if (!split_coarse(e)) return 0;
    const int cap = e->d >= 4 ? cand_capc<4>() : cand_capc<3>();
    HIPCHK(ensure(e->cl_cnt, e->cap_clc, (size_t)e->g.ncoarse * sizeof(uint32_t)));
    HIPCHK(ensure(e->cl_idx, e->cap_cli, (size_t)e->g.ncoarse * cap * sizeof(int32_t)));
    return 0;
}

// k_lloyd1 and the per-tile kernels: one block per tile of the layout (the
// exact count, read back at layout time).  Measured at config 3: 211 us per
// launch with one tile per block vs 238 us for as many persistent blocks as are
// co-resident walking tiles b, b + G, ... (each tile's list install stalled its
// block; with one tile per block the other resident blocks keep streaming);
// config-5 shape 485 vs 536 us.
static int lloyd_grid(const pcm_engine *e) { return (int)std::max(1LL, e->ntiles >= 0 ? e->ntiles : e->ntiles_cap); }

static int launch_candidates(pcm_engine *e, hipStream_t s, int gate) {
    return dispatch_d(e->d, [&](auto DD) -> int {
        constexpr int D = decltype(DD)::value;
        const int bpc = cand_bpc(e);
        if (split_coarse(e)) {
            if (int rc = ensure_coarse(e)) return rc;
            k_coarse<D><<<(int)e->g.ncoarse, CAND_TPB, 0, s>>>(e->g, e->C, e->k, e->ctrl, 0, e->cl_cnt, e->cl_idx);
            LAUNCHCHK();
            CoarseL cl;
            cl.in_cnt = e->cl_cnt;
            cl.in_idx = e->cl_idx;
            k_cand<D, 2><<<(int)n_mid(e), CAND_TPB, 0, s>>>(e->g, e->C, e->k, e->fc_cnt, e->fc_rec, e->fc_lab, e->ctrl,
                                                             gate, 1, e->cref, cl);
            LAUNCHCHK();
            return 0;
        }
        k_cand<D><<<(int)(e->g.ncoarse * bpc), CAND_TPB, 0, s>>>(e->g, e->C, e->k, e->fc_cnt, e->fc_rec, e->fc_lab,
                                                                 e->ctrl, gate, bpc, e->cref, CoarseL{});
        LAUNCHCHK();
        return 0;
    });
}

// Tile lists of the crowded cells at the current centres (before every assign
// launch of a crowded layout; gate: skip when the fit has halted or finished).
static int launch_tile_lists(pcm_engine *e, hipStream_t s, int gate) {
    if (e->zlev <= 0 || e->n == 0) return 0;
    return dispatch_d(e->d, [&](auto DD) -> int {
        constexpr int D = decltype(DD)::value;
        k_tile_cand<D><<<lloyd_grid(e), 256, 0, s>>>(e->tiles, e->ntiles_dev, e->fc_cnt, e->tbox, e->C, e->k,
                                                          e->tl_cnt, e->tl_rec, e->tl_lab, e->ctrl, gate);
        LAUNCHCHK();
        return 0;
    });
}

// Persistent grid: as many 256-thread blocks as are co-resident (occupancy
// query), never more blocks than tiles.
// k_label's grid: one block per tile (round 6: 247-249 -> 235-237 us per final
// E-step at config 3 against the co-resident persistent grid, as k_lloyd1
// measured in round 2; profiles/rd6_klabel_grid_ab.txt).  PCM_ASSIGN_BLOCKS_PER_CU
// (A/B) restores a persistent grid of that many blocks per CU.
static int assign_grid(pcm_engine *e, const void *kern, size_t lds) {
    (void)kern;
    (void)lds;
    const long long nt = e->ntiles >= 0 ? e->ntiles : e->ntiles_cap;
    if (const char *ov = std::getenv("PCM_ASSIGN_BLOCKS_PER_CU"))
        return (int)std::max(1LL, std::min<long long>(nt, (long long)std::max(1, std::atoi(ov)) * e->num_cu));
    return (int)std::max(1LL, nt);
}

static int lloyd_slots(const pcm_engine *e) {
    if (const char *ov = std::getenv("PCM_LSLOT_RT")) return std::atoi(ov) == 8 ? 8 : LSLOT;   // tuning sweeps only
    // cells per centre of the whole cloud (a spatial shard's cells cover ~n / n_global of the centres)
    const double share = e->n_global > 0 ? std::min(1.0, (double)e->n / (double)e->n_global) : 1.0;
    return (e->g.prune && (double)e->g.ncells >= 8.0 * e->k * share) ? 8 : LSLOT;
}

// Lane slots of the launched k_lloyd1: 8 on fine grids, else LSLOT.  D = 4
// (config 5: lists of ~8, up to 27) takes 8 slots since the slot map gives them
// to the candidates nearest each tile (k_lloyd1): 11.5 instead of 21.8 KB of
// LDS words per block, 5 instead of 3 waves per SIMD -- config-5 shard 404 ->
// 325 us per launch, 8-way slab 270 -> 220 us (round 4; PCM_D4_LS8=0 restores 16).
static int assign_ls(const pcm_engine *e) {
    static const bool d4_ls8 = [] { const char *v = std::getenv("PCM_D4_LS8"); return !v || std::atoi(v); }();
    return ((e->d <= 3 || d4_ls8) && lloyd_slots(e) == 8) ? 8 : LSLOT;
}

static LloydArgs lloyd_args(pcm_engine *e) {
    LloydArgs A{};
    A.xcd = ((xcd_mode() >> 1) & 1) && !e->tiles_lpt;   // an ordered tile list is dealt round-robin
    A.xs = e->xs;
    A.xz = e->use_xz ? e->xz : nullptr;
    A.tmeta = e->use_xz ? e->tmeta : nullptr;
    A.npad = e->npad;
    A.tiles = e->tiles;
    A.ntiles = e->ntiles_dev;
    A.fc_rec = e->fc_rec;
    A.fc_lab = e->fc_lab;
    A.C = e->C;
    A.fc_cnt = e->fc_cnt;
    A.K = e->k;
    for (int a = 0; a < MAXD; ++a) A.q[a] = e->qe.q[a];
    A.partials = e->partials;
    A.pstride = (long long)e->k * (e->d + 1);
    A.ctrl = e->ctrl;
    A.sub_start = e->sub_start;
    A.sub = e->sub;
    A.g = e->g;
    A.tl_cnt = e->zlev > 0 ? e->tl_cnt : nullptr;
    A.tl_rec = e->zlev > 0 ? e->tl_rec : nullptr;
    A.tl_lab = e->zlev > 0 ? e->tl_lab : nullptr;
    A.tbox = e->zlev > 0 ? e->tbox : nullptr;
    return A;
}

// E-step with the current centres: candidate lists, then labels (sorted
// order, e->lab) and, when inert is non-null, the exact inertia limbs added
// into inert[0..3].  Not gated.
static int launch_labels(pcm_engine *e, hipStream_t s, unsigned long long *inert) {
    if (int rc = launch_candidates(e, s, 0)) return rc;
    if (int rc = launch_tile_lists(e, s, 0)) return rc;
    LloydArgs A = lloyd_args(e);
    return dispatch_td(e->dtype, e->d, [&](auto T, auto DD) -> int {
        using TT = decltype(T);
        constexpr int D = decltype(DD)::value;
        if (e->n == 0) return 0;
        return dispatch_l(e, [&](auto L) -> int {
            using LT = decltype(L);
            // inertia limbs: per-block replica lines, folded into inert[] afterwards
            unsigned long long *rep = inert ? &e->ctrl->inert_rep[0][0] : nullptr;
            k_label<TT, D, LT><<<assign_grid(e, (const void *)k_label<TT, D, LT>, 0), TPB, 0, s>>>(A, e->lab, rep, e->iscale);
            LAUNCHCHK();
            if (inert) {
                k_inert_fold<<<1, 64, 0, s>>>(rep, inert);
                LAUNCHCHK();
            }
            return 0;
        });
    });
}

// Fold completed event pairs into the sums (non-blocking unless the ring is full).
static int timing_drain(pcm_engine *e, bool block) {
    while (e->ev_pending > 0) {
        int slot = (e->ev_next - e->ev_pending + pcm_engine::TEV) % pcm_engine::TEV;
        if (block) HIPCHK(hipEventSynchronize(e->ev[slot][3]));
        else if (hipEventQuery(e->ev[slot][3]) != hipSuccess) return 0;
        float a = 0, b = 0, c = 0;
        HIPCHK(hipEventElapsedTime(&a, e->ev[slot][0], e->ev[slot][1]));
        HIPCHK(hipEventElapsedTime(&b, e->ev[slot][1], e->ev[slot][2]));
        HIPCHK(hipEventElapsedTime(&c, e->ev[slot][2], e->ev[slot][3]));
        e->t_sum[1] += a;   // candidates
        e->t_sum[0] += b;   // assign
        e->t_sum[2] += c;   // fold + global
        e->t_count++;
        e->ev_pending--;
    }
    return 0;
}

static int timing_mark(pcm_engine *e, int which, hipStream_t s) {
    if (!e->timing) return 0;
    if (which == 0) {
        if (e->ev_pending == pcm_engine::TEV)
            if (int rc = timing_drain(e, true)) return rc;
        if (!e->ev[e->ev_next][0])
            for (int j = 0; j < 4; ++j) HIPCHK(hipEventCreate(&e->ev[e->ev_next][j]));
    }
    HIPCHK(hipEventRecord(e->ev[e->ev_next][which], s));
    if (which == 3) {
        e->ev_next = (e->ev_next + 1) % pcm_engine::TEV;
        e->ev_pending++;
    }
    return 0;
}

// k_lloyd (its candidate lists were built by the previous k_lists, the resume
// path or pcm_fit_begin).  to_stats: accumulate straight into `stats` (the
// statistics buffer every fit iterates through -- one GPU or the all-reduce /
// peer-exchange buffer of several -- zeroed by the previous update's
// publisher, k_global or fit_begin); otherwise into partials[iter & 1], which
// only the assign-timing calibration (pcm_time_assign) still uses.
static int iter_local_impl(pcm_engine *e, hipStream_t s, bool to_stats) {
    if (int rc = timing_mark(e, 0, s)) return rc;
    if (int rc = launch_tile_lists(e, s, 1)) return rc;   // crowded layouts only
    if (int rc = timing_mark(e, 1, s)) return rc;
    LloydArgs A = lloyd_args(e);
    if (to_stats) {
        A.partials = e->stats;
        A.pstride = 0;
    }
    return dispatch_td(e->dtype, e->d, [&](auto T, auto DD) -> int {
        using TT = decltype(T);
        constexpr int D = decltype(DD)::value;
        if (e->n > 0) {
            // lane slots per thread: 8 on fine grids (>= 8 cells per centre: lists
            // of ~3 at config 3; 13.5 KB of LDS -> 5 waves/SIMD, 247 -> 237 us),
            // else 16 (12.5M-point shard: lists of ~6, 53 vs 57 us)
            auto launch = [&](auto LSc) {
                constexpr int LS = decltype(LSc)::value;
                // crowded layouts: + the long tile lists' int64 words (AccL::gwords)
                const size_t lds = e->zlev > 0 ? AccL<D, LS>::bytes_crowded
                                                : (size_t)AccL<D, LS>::words * sizeof(uint32_t);
                if (e->zlev > 0)   // crowded layout (sub-cell masks off: e->sub = 0)
                    k_lloyd1<TT, D, LS, false, true><<<lloyd_grid(e), TPB, lds, s>>>(
                        A, e->tiles, e->fc_rec, e->fc_lab, e->C, e->fc_cnt, e->tl_rec);
                else
                    k_lloyd1<TT, D, LS, (D <= 3 && LS == LSLOT)><<<lloyd_grid(e), TPB, lds, s>>>(
                        A, e->tiles, e->fc_rec, e->fc_lab, e->C, e->fc_cnt, e->C);
            };
            // coarse grids keep 16 slots with masks: 8 slots + LDS int64 words 42.0 -> 51.2 us,
            // 12 slots + global atomics 42.6 -> 65.7 us at 12.5M (tools/mls_sweep.sh)
            if (assign_ls(e) == 8) launch(std::integral_constant<int, 8>{});
            else launch(std::integral_constant<int, LSLOT>{});
            LAUNCHCHK();
        }
        return timing_mark(e, 2, s);
    });
}

int pcm_iter_local(pcm_engine *e, void *stream) {
    if (!e) return fail(PCM_E_ARG, "null engine");
    if (!e->fit_ready) return fail(PCM_E_STATE, "pcm_fit_begin must run first");
    return iter_local_impl(e, (hipStream_t)stream, true);   // into `stats`: the caller all-reduces it
}

// Centre update + next candidate lists.  from_partials = false (every fit): the
// kernels read `stats` (the summed statistics); true: partials[iter & 1].  Every K: k_upd (the
// K new centres once, convergence, history) then k_lists (C := new centres,
// this block's lists rebuilt or refreshed).  The relocation resume takes
// k_global (it handles `resume`) + k_cand.
static int iter_global_impl(pcm_engine *e, hipStream_t s, bool from_partials, bool resume_path) {
    int rc = dispatch_d(e->d, [&](auto DD) -> int {
        constexpr int D = decltype(DD)::value;
        if (!resume_path) {
            double wmin = 0.0;
            for (int a = 0; a < D; ++a)
                if (e->g.ext[a] > 0 && (wmin == 0.0 || e->g.w[a] < wmin)) wmin = e->g.w[a];
            // D <= 3, K <= 1024: update and lists in one launch (k_updlists)
            // (PCM_FUSED_UPD=0: k_upd1 + k_lists instead -- A/B and tests; read per
            // launch so tests can switch it between fits, captured graphs keep theirs)
            const char *fz = std::getenv("PCM_FUSED_UPD");
            const bool fused_on = !(fz && std::atoi(fz) == 0);
            if (fused_on && D <= 3 && !split_coarse(e) && e->k <= 2 * CAND_TPB) {
                const int bpc = cand_bpc(e);
                const int nlist = (int)(e->g.ncoarse * bpc);
                auto fused = [&](auto RR) {
                    constexpr int RV = decltype(RR)::value;
                    const size_t lds = (size_t)e->k * sizeof(float4);
                    // a dedicated publisher block when one more block still fits the residency
                    // (PCM_UPD_PUB=0: always the last arriver -- A/B only)
                    static const int pub_env = [] { const char *v = std::getenv("PCM_UPD_PUB"); return v ? std::atoi(v) : 1; }();
                    int per_cu = 0;
                    const bool pub = pub_env &&
                        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)k_updlists<D, RV, true>,
                                                                     CAND_TPB, lds) == hipSuccess &&
                        (long long)nlist + 1 <= (long long)per_cu * e->num_cu;
                    if (pub)
                        k_updlists<D, RV, true><<<nlist + 1, CAND_TPB, lds, s>>>(
                            from_partials ? nullptr : e->stats, e->partials, e->k, e->qe, e->held, e->prev, e->C, e->cref,
                            e->hist_changed, e->hist_shift, e->ctrl, e->drift_alpha, e->drift_kappa * wmin, e->g,
                            e->fc_cnt, e->fc_rec, e->fc_lab, bpc);
                    else
                        k_updlists<D, RV, false><<<nlist, CAND_TPB, lds, s>>>(
                            from_partials ? nullptr : e->stats, e->partials, e->k, e->qe, e->held, e->prev, e->C, e->cref,
                            e->hist_changed, e->hist_shift, e->ctrl, e->drift_alpha, e->drift_kappa * wmin, e->g,
                            e->fc_cnt, e->fc_rec, e->fc_lab, bpc);
                };
                if (e->k <= CAND_TPB) fused(std::integral_constant<int, 1>{});
                else fused(std::integral_constant<int, 2>{});
                LAUNCHCHK();
                return 0;
            }
            // one block (the shift tree in LDS, no hand-off between blocks) up to UPD1_MAX centres
            auto upd1 = [&](auto RR) {
                k_upd1<D, decltype(RR)::value><<<1, SHIFT_LANES, 0, s>>>(
                    from_partials ? nullptr : e->stats, e->partials, e->k, e->qe, e->held, e->prev, e->C, e->Cn,
                    e->cref, e->hist_changed, e->hist_shift, e->ctrl, e->drift_alpha, e->drift_kappa * wmin);
            };
            if (e->k <= SHIFT_LANES)
                upd1(std::integral_constant<int, 1>{});
            else if (e->k <= UPD1_MAX)
                upd1(std::integral_constant<int, 2>{});
            else
                k_upd<D><<<blocks_for(e->k, UPD_TPB), UPD_TPB, 0, s>>>(
                    from_partials ? nullptr : e->stats, e->partials, e->k, e->qe, e->held, e->prev, e->C, e->Cn,
                    e->cref, e->shbuf, e->upart, e->hist_changed, e->hist_shift, e->ctrl, e->drift_alpha,
                    e->drift_kappa * wmin);
            LAUNCHCHK();
            if (split_coarse(e)) {
                if (int rc = ensure_coarse(e)) return rc;
                k_coarse<D><<<(int)e->g.ncoarse, CAND_TPB, 0, s>>>(e->g, e->Cn, e->k, e->ctrl, 1, e->cl_cnt, e->cl_idx);
                LAUNCHCHK();
                CoarseL cl;
                cl.in_cnt = e->cl_cnt;
                cl.in_idx = e->cl_idx;
                // mid-cell blocks of 256 threads (PCM_LISTS4_TPB=512: the round-4 start's size, A/B only)
                const char *lt = std::getenv("PCM_LISTS4_TPB");
                if (lt && std::atoi(lt) == 512)
                    k_lists<D, 2><<<(int)n_mid(e), CAND_TPB, 0, s>>>(e->g, e->Cn, e->C, e->cref, e->k, e->ctrl,
                                                                      e->fc_cnt, e->fc_rec, e->fc_lab, 1, cl);
                else
                    k_lists<D, 2, false, 256><<<(int)n_mid(e), 256, 0, s>>>(e->g, e->Cn, e->C, e->cref, e->k, e->ctrl,
                                                                             e->fc_cnt, e->fc_rec, e->fc_lab, 1, cl);
            } else if (e->k <= LISTS_STAGE_MAX) {   // centres staged in LDS
                const int bpc = cand_bpc(e);
                k_lists<D, 4, true><<<(int)(e->g.ncoarse * bpc), CAND_TPB, (size_t)e->k * sizeof(float4), s>>>(
                    e->g, e->Cn, e->C, e->cref, e->k, e->ctrl, e->fc_cnt, e->fc_rec, e->fc_lab, bpc, CoarseL{});
            } else {
                const int bpc = cand_bpc(e);
                k_lists<D><<<(int)(e->g.ncoarse * bpc), CAND_TPB, 0, s>>>(e->g, e->Cn, e->C, e->cref, e->k, e->ctrl,
                                                                           e->fc_cnt, e->fc_rec, e->fc_lab, bpc,
                                                                           CoarseL{});
            }
            LAUNCHCHK();
            return 0;
        }
        k_global<D><<<1, 1024, 0, s>>>(nullptr, e->stats, e->k, e->qe, e->held, e->prev, e->C, e->Cn,
                                       e->hist_changed, e->hist_shift, e->ctrl);
        LAUNCHCHK();
        return launch_candidates(e, s, 1);
    });
    if (rc) return rc;
    return timing_mark(e, 3, s);
}

int pcm_iter_global(pcm_engine *e, void *stream) {
    if (!e) return fail(PCM_E_ARG, "null engine");
    if (!e->fit_ready) return fail(PCM_E_STATE, "pcm_fit_begin must run first");
    return iter_global_impl(e, (hipStream_t)stream, false, false);
}

int pcm_timing(pcm_engine *e, int enable) {
    if (!e) return fail(PCM_E_ARG, "null engine");
    if (int rc = timing_drain(e, true)) return rc;
    e->timing = enable != 0;
    e->t_sum[0] = e->t_sum[1] = e->t_sum[2] = 0.0;
    e->t_count = 0;
    return 0;
}

int pcm_timing_read(pcm_engine *e, double *ms, int *count) {
    if (!e || !ms || !count) return fail(PCM_E_ARG, "bad argument");
    if (int rc = timing_drain(e, true)) return rc;
    for (int i = 0; i < 3; ++i) ms[i] = e->t_count ? e->t_sum[i] / (double)e->t_count : 0.0;
    *count = (int)e->t_count;
    return 0;
}

// Calibration of the assign kernel's launch duration: `reps` back-to-back
// launches on the current layout, lists and centres between ONE HIP event pair
// (no per-launch events, no k_step between them).  The statistics they add are
// discarded: the fit must restart with pcm_fit_begin.
int pcm_time_assign(pcm_engine *e, int reps, void *stream, double *ms) {
    if (!e || !ms || reps < 1) return fail(PCM_E_ARG, "bad argument");
    if (!e->fit_ready) return fail(PCM_E_STATE, "pcm_fit_begin must run first");
    hipStream_t s = (hipStream_t)stream;
    if (int rc = timing_drain(e, true)) return rc;
    // a halted or finished fit gates k_lloyd1 off: its launches would time nothing
    uint32_t flags[2] = {0u, 0u};
    HIPCHK(hipMemcpyAsync(flags, e->ctrl, sizeof(flags), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (flags[0] | flags[1]) return fail(PCM_E_STATE, "the fit has halted or finished: nothing to time");
    // events and the engine's timing flag are restored on every exit path
    struct Guard {
        pcm_engine *e;
        bool was;
        hipEvent_t a = nullptr, b = nullptr;
        ~Guard() {
            if (a) (void)hipEventDestroy(a);
            if (b) (void)hipEventDestroy(b);
            e->timing = was;
        }
    } g{e, e->timing};
    e->timing = false;
    HIPCHK(hipEventCreate(&g.a));
    HIPCHK(hipEventCreate(&g.b));
    HIPCHK(hipEventRecord(g.a, s));
    int rc = 0;
    for (int i = 0; i < reps && !rc; ++i) rc = iter_local_impl(e, s, false);
    e->fit_ready = false;   // the partial statistics now hold extra sums
    if (rc) return rc;
    HIPCHK(hipEventRecord(g.b, s));
    HIPCHK(hipEventSynchronize(g.b));
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, g.a, g.b));
    *ms = (double)t / reps;
    return 0;
}

// Single-process iterations: the multi-GPU sequence without the all-reduce --
// k_lloyd1 into the statistics buffer, then the update reading it in place (its
// publisher zeroes it once every block has read it).  (Round 5 retired the
// parity halves of `partials` on this path: they made every k_updlists block
// load both halves, 32 of its 144 B per centroid row; round 6 removed the A/B
// switch that kept them.)
int pcm_iterate(pcm_engine *e, int n, void *stream) {
    if (!e || n < 0) return fail(PCM_E_ARG, "bad argument");
    if (!e->fit_ready) return fail(PCM_E_STATE, "pcm_fit_begin must run first");
    hipStream_t s = (hipStream_t)stream;
    for (int i = 0; i < n; ++i) {
        if (int rc = iter_local_impl(e, s, true)) return rc;
        if (int rc = iter_global_impl(e, s, false, false)) return rc;
    }
    return 0;
}

// The cross-rank SUM of the statistics by peer-memory writes (pcm_xchg.hip),
// between pcm_iter_local and pcm_iter_global in place of the RCCL all-reduce;
// gated by the control block like both of them.
int pcm_iter_exchange(pcm_engine *e, pcm_xchg *x, int phase, void *stream) {
    if (!e || !x) return fail(PCM_E_ARG, "null engine or exchange");
    if (!e->fit_ready) return fail(PCM_E_STATE, "pcm_fit_begin must run first");
    return pcm_xchg_launch(x, e->stats, &e->ctrl->halt, phase, (hipStream_t)stream);
}

int pcm_stats_ptr(pcm_engine *e, void **ptr, int64_t *count) {
    if (!e || !ptr || !count) return fail(PCM_E_ARG, "bad argument");
    *ptr = e->stats;
    *count = (int64_t)e->k * (e->d + 1) + 1;
    return 0;
}

int pcm_bind_stats(pcm_engine *e, void *ptr) {
    if (!e) return fail(PCM_E_ARG, "null engine");
    e->stats = ptr ? (unsigned long long *)ptr : e->stats_own;
    return 0;
}

int pcm_reloc_candidates(pcm_engine *e, int m, void *records, void *stream) {
    if (!e || m < 1 || !records) return fail(PCM_E_ARG, "bad argument");
    if (!e->fit_ready) return fail(PCM_E_STATE, "no fit in progress");
    hipStream_t s = (hipStream_t)stream;
    const long long n = e->n;
    HIPCHK(hipMemsetAsync(records, 0, (size_t)m * sizeof(RelocRec), s));
    if (n == 0) return 0;
    // keys (8 B/pt) + selection state in the layout's scratch arena (>= 12 B/pt)
    const size_t need = align_up((size_t)n * 8) + sizeof(RselState);
    if (ensure(e->ws, e->cap_ws, need) != hipSuccess) return fail(PCM_E_NOMEM, "reloc scratch");
    unsigned long long *keys = (unsigned long long *)e->ws;
    RselState *st = (RselState *)((char *)e->ws + align_up((size_t)n * 8));
    RselState h{};
    h.prefix = 0ull;
    h.m_rem = (unsigned long long)std::min<long long>(m, n);
    HIPCHK(hipMemcpyAsync(st, &h, sizeof(h), hipMemcpyHostToDevice, s));
    // labels of the halted iteration (the iterations keep no label array)
    if (int rc = launch_labels(e, s, nullptr)) return rc;
    const int hblk = (int)std::min<long long>((n + 255) / 256, (long long)e->num_cu * 4);
    int rc = dispatch_td(e->dtype, e->d, [&](auto T, auto DD) -> int {
        using TT = decltype(T);
        constexpr int D = decltype(DD)::value;
        return dispatch_l(e, [&](auto L) -> int {
            using LT = decltype(L);
            k_reloc_keys<TT, D, LT><<<blocks_for(n), 256, 0, s>>>((const TT *)e->xs, n, (const LT *)e->lab, e->perm,
                                                                 e->C, e->gidx0, e->has_rows ? e->grows : nullptr,
                                                                 keys);
            LAUNCHCHK();
            if (m < n)   // exactly the top m; m >= n takes every point (T = 0)
                for (int pass = 0; pass < 8; ++pass) {
                    k_rsel_hist<<<hblk, 256, 0, s>>>(keys, n, st, pass);
                    LAUNCHCHK();
                    k_rsel_pick<<<1, 64, 0, s>>>(st, pass);
                    LAUNCHCHK();
                }
            k_reloc_gather<TT, D, LT><<<blocks_for(n), 256, 0, s>>>(keys, n, (const TT *)e->xs, (const LT *)e->lab,
                                                                   e->qe, st, m, (RelocRec *)records);
            LAUNCHCHK();
            return 0;
        });
    });
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

int pcm_reloc_apply(pcm_engine *e, const void *records, int n_rec, void *stream) {
    if (!e || !records || n_rec < 1) return fail(PCM_E_ARG, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    if (n_rec > e->rank_cap) {
        if (e->rank_buf) HIPCHK(hipFree(e->rank_buf));
        e->rank_buf = nullptr;
        HIPCHK(hipMalloc(&e->rank_buf, (size_t)n_rec * sizeof(int)));
        e->rank_cap = n_rec;
    }
    int rc = dispatch_d(e->d, [&](auto DD) -> int {
        constexpr int D = decltype(DD)::value;
        k_reloc_apply<D><<<1, 256, 0, s>>>((const RelocRec *)records, n_rec, e->held, e->k, e->rank_buf,
                                           e->empty_idx, e->ctrl);
        LAUNCHCHK();
        return 0;
    });
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(e->stats, e->held, ((size_t)e->k * (e->d + 1) + 1) * sizeof(unsigned long long),
                          hipMemcpyDeviceToDevice, s));
    return iter_global_impl(e, s, false, true);
}

int pcm_final(pcm_engine *e, void *stream) {
    if (!e) return fail(PCM_E_ARG, "null engine");
    if (!e->fit_ready) return fail(PCM_E_STATE, "pcm_fit_begin must run first");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemsetAsync(e->ctrl->inert, 0, sizeof(e->ctrl->inert), s));
    return launch_labels(e, s, e->ctrl->inert);
}

int pcm_labels(pcm_engine *e, int32_t *out, void *stream) {
    if (!e || (!out && e->n > 0)) return fail(PCM_E_ARG, "bad argument");
    if (!e->layout_ready) return fail(PCM_E_STATE, "layout not built");
    if (e->n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    // uint16 labels (K <= 65535): scatter into a 2 B/pt scratch that stays in the
    // Infinity Cache while the random writes land, then one sequential widen to
    // int32 -- 100M points: 1.52 vs 2.11 ms for the direct int32 scatter
    // (tools/unperm_sweep.sh; windows of 64M/32M rows: 1.88/1.93 ms).
    // PCM_UNPERM / PCM_UNPERM_WIN: tuning sweeps only.
    static const int mode = [] { const char *v = std::getenv("PCM_UNPERM"); return v ? std::atoi(v) : 3; }();
    static const long long win = [] { const char *v = std::getenv("PCM_UNPERM_WIN"); return v ? std::atoll(v) : (1LL << 40); }();
    return dispatch_l(e, [&](auto L) -> int {
        using LT = decltype(L);
        const bool a16 = ((uintptr_t)out & 15u) == 0;
        if (mode == 3 && e->has_dmap) {
            // the sort's two position maps, inverted by two run-wise gathers:
            // sorted -> between the passes -> caller rows
            if (ensure(e->ws, e->cap_ws, (size_t)e->n * sizeof(LT) + 64) != hipSuccess)
                return fail(PCM_E_NOMEM, "labels scratch");
            LT *mid = (LT *)e->ws;   // 256-B aligned scratch
            const uint32_t *m1 = e->dmap + e->n;   // the second pass's map: 16-B aligned iff n % 4 == 0
            const int g4 = (int)blocks_for((e->n + 3) / 4);
            const int xg = (xcd_mode() >> 2) & 1;
            if (((uintptr_t)m1 & 15u) == 0)
                k_lab_gather4<LT, LT, true, true><<<g4, 256, 0, s>>>(m1, (const LT *)e->lab, e->n, mid, xg);
            else
                k_lab_gather4<LT, LT, false, true><<<g4, 256, 0, s>>>(m1, (const LT *)e->lab, e->n, mid, xg);
            LAUNCHCHK();
            if (a16)
                k_lab_gather4<LT, int32_t, true, true><<<g4, 256, 0, s>>>(e->dmap, mid, e->n, out, xg);
            else
                k_lab_gather4<LT, int32_t, true, false><<<g4, 256, 0, s>>>(e->dmap, mid, e->n, out, xg);
            LAUNCHCHK();
            return 0;
        }
        if (mode >= 1 && std::is_same<LT, uint16_t>::value && a16) {
            // uint16 scatter into scratch (n * 2 B), in destination windows, then a sequential widen
            if (ensure(e->ws, e->cap_ws, (size_t)e->n * 2 + 64) != hipSuccess) return fail(PCM_E_NOMEM, "labels scratch");
            uint16_t *t16 = (uint16_t *)e->ws;
            for (long long r0 = 0; r0 < e->n; r0 += win) {
                const long long r1 = std::min<long long>(e->n, r0 + win);
                k_unpermute_win<LT, uint16_t><<<blocks_for(e->n), 256, 0, s>>>((const LT *)e->lab, e->perm, e->n,
                                                                               (uint32_t)r0, (uint32_t)r1, t16);
                LAUNCHCHK();
            }
            k_widen_u16<<<blocks_for((e->n + 3) / 4), 256, 0, s>>>(t16, e->n, out);
            LAUNCHCHK();
            return 0;
        }
        if (mode == 2) {
            for (long long r0 = 0; r0 < e->n; r0 += win) {
                const long long r1 = std::min<long long>(e->n, r0 + win);
                k_unpermute_win<LT, int32_t><<<blocks_for(e->n), 256, 0, s>>>((const LT *)e->lab, e->perm, e->n,
                                                                              (uint32_t)r0, (uint32_t)r1, out);
                LAUNCHCHK();
            }
            return 0;
        }
        k_unpermute<LT><<<blocks_for(e->n), 256, 0, s>>>((const LT *)e->lab, e->perm, e->n, out);
        LAUNCHCHK();
        return 0;
    });
}

int pcm_get_centers(pcm_engine *e, float *out, void *stream) {
    if (!e || !out) return fail(PCM_E_ARG, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    return dispatch_d(e->d, [&](auto DD) -> int {
        constexpr int D = decltype(DD)::value;
        k_centers_out<D><<<blocks_for(e->k), 256, 0, s>>>(e->C, e->k, out);
        LAUNCHCHK();
        return 0;
    });
}

int pcm_history(pcm_engine *e, uint64_t *changed, double *shift, int cap, void *stream) {
    if (!e || !changed || !shift || cap < 0) return fail(PCM_E_ARG, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    int c = std::min(cap, e->max_iter_cap);
    HIPCHK(hipMemcpyAsync(changed, e->hist_changed, (size_t)c * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(shift, e->hist_shift, (size_t)c * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

static void status_fill(const pcm_engine *e, const Ctrl &h, pcm_status *out) {
    out->halt = h.halt;
    out->done = h.done;
    out->iter = h.iter;
    out->n_empty = h.n_empty;
    for (int q = 0; q < 3; ++q) out->inertia_limbs[q] = h.inert[q];
    out->inertia_scale = e->iscale;
    out->inertia_overflow = (uint32_t)h.inert[3];
    out->inertia = pcm_inertia_value(out->inertia_limbs, e->iscale, out->inertia_overflow);
    out->list_rebuilds = h.rebuilds;
    out->pad_ = 0;
    out->last_changed = h.last_changed;
    out->last_shift = h.last_shift;
}

int pcm_read_status(pcm_engine *e, pcm_status *out, void *stream) {
    if (!e || !out) return fail(PCM_E_ARG, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    Ctrl h{};
    HIPCHK(hipMemcpyAsync(&h, e->ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    status_fill(e, h, out);
    return 0;
}

// Status without draining the stream: post = a snapshot of ctrl queued behind
// the work enqueued so far (pinned copy + event); wait = until that snapshot
// has landed.  Lets the host queue the next chunk of iterations before it
// reads the previous chunk's status (lloyd.run), so the GPU does not idle for
// the round trip.  One snapshot in flight per engine.
int pcm_status_post(pcm_engine *e, void *stream) {
    if (!e) return fail(PCM_E_ARG, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(e->ctrl_pin, e->ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(e->st_ev, s));
    return 0;
}

int pcm_status_wait(pcm_engine *e, pcm_status *out) {
    if (!e || !out) return fail(PCM_E_ARG, "bad argument");
    HIPCHK(hipEventSynchronize(e->st_ev));
    status_fill(e, *e->ctrl_pin, out);
    return 0;
}

int pcm_layout_info(pcm_engine *e, int64_t *ncells, int64_t *ntiles, int *grid) {
    if (!e || !ncells || !ntiles || !grid) return fail(PCM_E_ARG, "bad argument");
    *ncells = e->g.ncells;
    if (e->layout_ready && e->ntiles < 0) {   // read back lazily (synchronises the device)
        uint32_t nt = 0;
        HIPCHK(hipMemcpy(&nt, e->ntiles_dev, sizeof(uint32_t), hipMemcpyDeviceToHost));
        e->ntiles = nt;
    }
    *ntiles = e->ntiles;
    for (int a = 0; a < MAXD; ++a) grid[a] = e->g.G[a];
    return 0;
}

int pcm_layout_stream_bytes(pcm_engine *e, double *bytes, int64_t *compressed_points) {
    if (!e || !bytes || !compressed_points) return fail(PCM_E_ARG, "bad argument");
    if (!e->layout_ready) return fail(PCM_E_STATE, "layout not built");
    unsigned long long zr[32 * 16], z = 0;   // replica lines of k_tile_compress
    HIPCHK(hipMemcpy(zr, e->zpts, sizeof(zr), hipMemcpyDeviceToHost));
    for (int r = 0; r < 32; ++r) z += zr[r * 16];
    const double raw = (double)e->d * (double)tsize(e->dtype);
    *compressed_points = (int64_t)z;
    *bytes = (double)z * 8.0 + (double)(e->n - (long long)z) * raw;
    return 0;
}

int pcm_assign_kernel_name(pcm_engine *e, char *buf, size_t n) {
    if (!e || !buf || n == 0) return fail(PCM_E_ARG, "bad argument");
    if (!e->layout_ready) return fail(PCM_E_STATE, "layout not built");
    const int ls = assign_ls(e);
    const bool mask = e->d <= 3 && ls == LSLOT && e->zlev == 0;
    std::snprintf(buf, n, "k_lloyd1<%s,%d,%d,%s%s>", e->dtype == PCM_F16 ? "__half" : "float", e->d, ls,
                  mask ? "true" : "false", e->zlev > 0 ? ",crowded" : "");
    return 0;
}

int pcm_candidate_stats(pcm_engine *e, double *mean, int *mx, int64_t *full_cells, void *stream) {
    if (!e || !mean || !mx || !full_cells) return fail(PCM_E_ARG, "bad argument");
    if (!e->layout_ready) return fail(PCM_E_STATE, "layout not built");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemsetAsync(e->cand_stats, 0, 3 * sizeof(unsigned long long), s));
    k_cand_stats<<<blocks_for(e->g.ncells), 256, 0, s>>>(e->fc_cnt, e->g.ncells, e->cand_stats);
    LAUNCHCHK();
    unsigned long long h[3];
    HIPCHK(hipMemcpyAsync(h, e->cand_stats, sizeof(h), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    long long nonfull = e->g.ncells - (long long)h[2];
    *mean = nonfull > 0 ? (double)h[0] / (double)nonfull : 0.0;
    *mx = (int)h[1];
    *full_cells = (int64_t)h[2];
    return 0;
}

int pcm_tile_list_stats(pcm_engine *e, int *zlev, int64_t *crowded_tiles, int64_t *listed_tiles, int64_t *listed_len,
                        void *stream) {
    if (!e || !zlev || !crowded_tiles || !listed_tiles || !listed_len) return fail(PCM_E_ARG, "bad argument");
    if (!e->layout_ready) return fail(PCM_E_STATE, "layout not built");
    *zlev = e->zlev;
    *crowded_tiles = *listed_tiles = *listed_len = 0;
    if (e->zlev <= 0 || e->n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemsetAsync(e->cand_stats, 0, 6 * sizeof(unsigned long long), s));
    k_tile_list_stats<<<blocks_for(e->ntiles_cap), 256, 0, s>>>(e->tiles, e->ntiles_dev, e->fc_cnt, e->tl_cnt,
                                                                 e->cand_stats);
    LAUNCHCHK();
    unsigned long long h[3];
    HIPCHK(hipMemcpyAsync(h, e->cand_stats, sizeof(h), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *crowded_tiles = (int64_t)h[0];
    *listed_tiles = (int64_t)h[1];
    *listed_len = (int64_t)h[2];
    return 0;
}

int pcm_tile_list_detail(pcm_engine *e, int64_t *long_lists, int64_t *allk_tiles, int64_t *max_len, void *stream) {
    if (!e || !long_lists || !allk_tiles || !max_len) return fail(PCM_E_ARG, "bad argument");
    if (!e->layout_ready) return fail(PCM_E_STATE, "layout not built");
    *long_lists = *allk_tiles = *max_len = 0;
    if (e->zlev <= 0 || e->n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemsetAsync(e->cand_stats, 0, 6 * sizeof(unsigned long long), s));
    k_tile_list_stats<<<blocks_for(e->ntiles_cap), 256, 0, s>>>(e->tiles, e->ntiles_dev, e->fc_cnt, e->tl_cnt,
                                                                 e->cand_stats);
    LAUNCHCHK();
    unsigned long long h[6];
    HIPCHK(hipMemcpyAsync(h, e->cand_stats, sizeof(h), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *long_lists = (int64_t)h[3];
    *allk_tiles = (int64_t)h[4];
    *max_len = (int64_t)h[5];
    return 0;
}

int pcm_synth_uniform(float *out, int64_t n, int d, uint64_t seed, int64_t start, void *stream) {
    if ((!out && n > 0) || n < 0 || d < 1) return fail(PCM_E_ARG, "bad argument");
    if (n == 0) return 0;
    k_synth<<<blocks_for(n * d), 256, 0, (hipStream_t)stream>>>(out, n, d, seed, start);
    LAUNCHCHK();
    return 0;
}

// Debug (not in the public header): copy the sorted layout to device buffers
// (xs in the AoSoA-4 order of pcm_kernels.hpp xs_index).
int pcm_debug_layout(pcm_engine *e, void *xs_out, int32_t *lab_out, uint32_t *perm_out, void *stream) {
    if (!e || !e->layout_ready) return fail(PCM_E_STATE, "layout not built");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(xs_out, e->xs, (size_t)e->d * e->npad * tsize(e->dtype), hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(perm_out, e->perm, (size_t)e->n * 4, hipMemcpyDeviceToDevice, s));
    return dispatch_l(e, [&](auto L) -> int {
        using LT = decltype(L);
        k_unpermute<LT><<<blocks_for(e->n), 256, 0, s>>>((const LT *)e->lab, nullptr, e->n, lab_out);
        LAUNCHCHK();
        return 0;
    });
}

int pcm_synth_rows(float *out, const int64_t *rows, int64_t m, int d, uint64_t seed, void *stream) {
    if ((!out || !rows) && m > 0) return fail(PCM_E_ARG, "bad argument");
    if (m == 0) return 0;
    k_synth_rows<<<blocks_for(m * d), 256, 0, (hipStream_t)stream>>>(out, (const long long *)rows, m, d, seed);
    LAUNCHCHK();
    return 0;
}

int pcm_assign_bruteforce(const float *X, int64_t n, int d, const float *C, int k, const int32_t *q, int32_t *labels,
                          uint64_t *stats, void *stream) {
    if ((!X && n > 0) || !C || !q || (!labels && n > 0) || k < 1 || n < 0) return fail(PCM_E_ARG, "bad argument");
    if ((size_t)k * sizeof(float4) > 160 * 1024) return fail(PCM_E_ARG, "k too large for LDS staging");
    if (n == 0) return 0;
    QExp qe{};
    for (int a = 0; a < MAXD; ++a) qe.q[a] = a < d ? q[a] : 0;
    hipStream_t s = (hipStream_t)stream;
    int nblk = (int)std::min<long long>((n + 255) / 256, 2048);
    return dispatch_d(d, [&](auto DD) -> int {
        constexpr int D = decltype(DD)::value;
        k_bruteforce<D><<<nblk, 256, (size_t)k * sizeof(float4), s>>>(X, n, C, k, qe, labels,
                                                                       (unsigned long long *)stats);
        LAUNCHCHK();
        return 0;
    });
}

// k-means++ seeding (oracle/kpp_ref.py; sklearn/cluster/_kmeans.py:174-272):
// cell layout of X, then 3 launches per centre (csrc/pcm_kpp.hpp).  All
// device memory comes from the caller's workspace (pcm_kmeanspp_workspace).
namespace {
struct KppWs {   // byte offsets into the workspace
    size_t bbox_part, bbox_out, nonfinite, sort, perm, crow, xs, closest, cell_start, cmax, bsum, ctl, um, total;
    long long nc_max;
    RsPlan plan;   // the cell sort's plan at the largest grid (kpp_cells_max)
};

long long kpp_cells_max(long long n, int d) {
    const double target = std::max(1.0, (double)n / KPP_CELL_PTS);
    return std::min<long long>(1LL << 20, (long long)std::ceil(std::pow(1.5, d) * target) + 2);
}

int kpp_layout(long long n, int d, int k, int L, KppWs &w) {
    const long long npad = ((n + 3) / 4) * 4 + 4;
    const long long nb = (n + KPP_OB - 1) / KPP_OB;
    w.nc_max = kpp_cells_max(n, d);
    if (int rc = dispatch_d(d, [&](auto DD) -> int {
            constexpr int D = decltype(DD)::value;
            rs_plan<float, D>(n, cell_bits(w.nc_max), w.plan);
            return 0;
        }))
        return rc;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t at = o; o = align_up(o + std::max<size_t>(bytes, 8)); return at; };
    w.bbox_part = take((size_t)BBOX_BLOCKS * 2 * MAXD * sizeof(float));
    w.bbox_out = take(2 * MAXD * sizeof(double));
    w.nonfinite = take(sizeof(unsigned));
    w.sort = take(w.plan.total);
    w.perm = take(n * 4);
    w.crow = take(n * 4);
    w.xs = take((size_t)npad * d * sizeof(float));
    w.closest = take(n * 4);
    w.cell_start = take((w.nc_max + 1) * 4);
    w.cmax = take(w.nc_max * 4);
    w.bsum = take(nb * 8);
    w.ctl = take(sizeof(KppCtl));
    w.um = take((size_t)std::max(1, (k - 1) * L) * 8);
    w.total = o;
    return 0;
}

// oracle/kpp_ref.py kpp_scale: n * 2^s * maxd * (1 + 2^-20) < 2^62
int kpp_scale(long long n, double maxd) {
    if (!(maxd > 0.0) || n <= 0) return 0;
    int e = 0;
    (void)std::frexp(maxd * (1.0 + std::ldexp(1.0, -20)), &e);
    int nb = 0;
    for (unsigned long long v = (unsigned long long)(n - 1); v; v >>= 1) ++nb;
    return 62 - std::max(1, nb) - e;
}
}  // namespace

int pcm_kmeanspp_workspace(int64_t n, int d, int k, int n_local_trials, size_t *bytes) {
    if (!bytes || n < 1 || d < 1 || d > MAXD || k < 1 || n_local_trials < 1) return fail(PCM_E_ARG, "bad argument");
    KppWs w;
    if (int rc = kpp_layout(n, d, k, n_local_trials, w)) return rc;
    *bytes = w.total;
    return 0;
}

int pcm_kmeanspp(const float *X, int64_t n, int d, int k, int n_local_trials, int64_t first_index,
                 const uint64_t *umant, int64_t *indices, void *workspace, size_t workspace_bytes, void *stream) {
    if (!X || !indices || n < 1 || k < 1 || k > n || d < 1 || d > MAXD) return fail(PCM_E_ARG, "bad argument");
    if (n_local_trials < 1 || n_local_trials > KPP_LMAX) return fail(PCM_E_ARG, "n_local_trials must be 1..16");
    if (first_index < 0 || first_index >= n) return fail(PCM_E_ARG, "first_index out of range");
    if (k > 1 && !umant) return fail(PCM_E_ARG, "umant is null");
    if (n >= (1LL << 32) - 8) return fail(PCM_E_ARG, "n must be < 2^32");
    const int L = n_local_trials;
    KppWs w;
    if (int rc = kpp_layout(n, d, k, L, w)) return rc;
    if (!workspace || workspace_bytes < w.total) return fail(PCM_E_ARG, "workspace too small (pcm_kmeanspp_workspace)");
    hipStream_t s = (hipStream_t)stream;
    char *wb = (char *)workspace;
    float *bbox_part = (float *)(wb + w.bbox_part), *xs = (float *)(wb + w.xs), *closest = (float *)(wb + w.closest),
          *cmax = (float *)(wb + w.cmax);
    double *bbox_out = (double *)(wb + w.bbox_out);
    unsigned *nonfinite = (unsigned *)(wb + w.nonfinite);
    uint32_t *perm = (uint32_t *)(wb + w.perm), *cell_start = (uint32_t *)(wb + w.cell_start);
    float *crow = (float *)(wb + w.crow);
    unsigned long long *bsum = (unsigned long long *)(wb + w.bsum), *um = (unsigned long long *)(wb + w.um);
    KppCtl *ctl = (KppCtl *)(wb + w.ctl);
    const long long npad = ((n + 3) / 4) * 4 + 4;
    const long long nb = (n + KPP_OB - 1) / KPP_OB;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1)
        ncu = 256;
    // bounding box (+ non-finite check) -> pruning grid of ~n / KPP_CELL_PTS cells, weight scale
    const int nblk = (int)std::min<long long>(BBOX_BLOCKS, (n + 255) / 256);
    HIPCHK(hipMemsetAsync(nonfinite, 0, sizeof(unsigned), s));
    int rc = dispatch_d(d, [&](auto DD) -> int {
        constexpr int D = decltype(DD)::value;
        k_bbox_partial<float, D><<<nblk, 256, 0, s>>>(X, n, bbox_part, nonfinite);
        LAUNCHCHK();
        k_bbox_final<D><<<1, 256, 0, s>>>(bbox_part, nblk, bbox_out);
        LAUNCHCHK();
        return 0;
    });
    if (rc) return rc;
    double hb[2 * MAXD];
    unsigned nf = 0;
    HIPCHK(hipMemcpyAsync(hb, bbox_out, 2 * d * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&nf, nonfinite, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (nf) return fail(PCM_E_NONFINITE, "input points contain NaN or Inf");
    double maxd = 0.0;
    for (int a = 0; a < d; ++a) maxd += (hb[d + a] - hb[a]) * (hb[d + a] - hb[a]);
    const int scale = kpp_scale(n, maxd);
    Grid g;
    make_grid(g, d, hb, hb + d, std::max(1.0, (double)n / KPP_CELL_PTS));
    const long long nc = g.ncells;
    if (nc > w.nc_max) return fail(PCM_E_STATE, "kmeanspp: grid exceeds the workspace bound");
    unsigned bits = 1;
    while ((1LL << bits) < nc) ++bits;
    if (k > 1) HIPCHK(hipMemcpy(um, umant, (size_t)(k - 1) * L * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemsetAsync(bsum, 0, nb * 8, s));
    HIPCHK(hipMemsetAsync(ctl, 0, sizeof(KppCtl), s));
    return dispatch_d(d, [&](auto DD) -> int {
        constexpr int D = decltype(DD)::value;
        // cell layout (the Lloyd engine's record sort, pcm_sort.hpp), cell starts
        RsPlan p;
        rs_plan<float, D>(n, bits, p);
        if (p.total > w.plan.total) return fail(PCM_E_STATE, "kmeanspp: sort plan exceeds the workspace bound");
        if (int rc2 = rs_sort<float, D>(X, n, npad, g, 0, 0, bits, p, wb + w.sort, xs, perm, s)) return rc2;
        k_cell_starts_xs<float, D><<<blocks_for(nc + 1), 256, 0, s>>>(xs, n, g, 0, 0, nc, cell_start, 0);
        LAUNCHCHK();
        const int pgrid = ncu * 8;
        k_kpp_init<D><<<pgrid, 256, 0, s>>>(xs, cell_start, nc, X, first_index, closest, cmax, (long long *)indices);
        LAUNCHCHK();
        k_kpp_init_rows<D><<<(int)std::min<long long>(nb, pgrid), 256, 0, s>>>(X, n, first_index, scale, crow, bsum, ctl);
        LAUNCHCHK();
        // from centre 64 on a step touches a neighbourhood: a quarter of the grid
        // (2048 -> 512 blocks) for eval/apply, 163.3 -> 159.1 ms at config 3
        // (tools/kpp_grid_sweep.sh; 1/8: 162.6 ms); re-swept after the round-3
        // atomics fix: 1/4 109.3-110.2, 1/2 113.3, 1/8 123.4 ms (tools/r4j.sh).
        // PCM_KPP_LATE_*: tuning only
        // round 5 (eval at 86 VGPRs, 5 waves/SIMD): eval keeps the whole grid, apply
        // 1/4 -- 94.5 ms vs 95.1 (1/2, 1/4), 94.9 (1/2, 1/2), 95.9 (1/1, 1/8)
        // (tools/rd5q.sh, profiles/rd5_kpp_steps.txt)
        static const int late_div = [] { const char *v = std::getenv("PCM_KPP_LATE_DIV"); return v ? std::max(1, std::atoi(v)) : 1; }();
        static const int apply_div = [] { const char *v = std::getenv("PCM_KPP_APPLY_DIV"); return v ? std::max(1, std::atoi(v)) : 4; }();
        static const int late_c = [] { const char *v = std::getenv("PCM_KPP_LATE_C"); return v ? std::atoi(v) : 64; }();
        for (int c = 1; c < k; ++c) {
            const int eg = c >= late_c ? std::max(ncu, pgrid / late_div) : pgrid;
            const int ag = c >= late_c ? std::max(ncu, pgrid / apply_div) : pgrid;
            k_kpp_search<D><<<L + KPP_RED_BLOCKS, KPP_STPB, 0, s>>>(bsum, nb, crow, X, n,
                                                                    um + (size_t)(c - 1) * L, L, scale, c, cmax, nc,
                                                                    ctl);
            LAUNCHCHK();
            if (L <= 8) k_kpp_eval<D, 8><<<eg, 256, 0, s>>>(xs, cell_start, g, closest, cmax, L, scale, c, ctl);
            else k_kpp_eval<D><<<eg, 256, 0, s>>>(xs, cell_start, g, closest, cmax, L, scale, c, ctl);
            LAUNCHCHK();
            k_kpp_apply<D><<<ag, 256, 0, s>>>(xs, perm, cell_start, g, closest, crow, cmax, bsum, X, n, L, scale, c,
                                              c + 1 < k ? 1 : 0, (long long *)indices, ctl);
            LAUNCHCHK();
        }
        return 0;
    });
}

#ifdef PCM_DBG_TIMING
int pcm_debug_timing(unsigned long long *out, int nblocks) {
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg_t), (size_t)nblocks * 16 * sizeof(unsigned long long)));
    return 0;
}
int pcm_debug_timing_eval(unsigned long long *out, int nblocks) {
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg_e), (size_t)nblocks * 8 * sizeof(unsigned long long)));
    return 0;
}
int pcm_debug_kpp_counts(unsigned long long *out, int ncentres) {
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg_kpp), (size_t)ncentres * 4 * sizeof(unsigned long long)));
    return 0;
}
int pcm_debug_timing_lloyd(unsigned long long *out, int nblocks) {
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg_l), (size_t)nblocks * 8 * sizeof(unsigned long long)));
    return 0;
}
#endif

namespace {
// Symmetric 3x3 eigen-solve (cyclic Jacobi, float64): eigenvector of the smallest eigenvalue.
void smallest_eigvec3(const double cov[6], double out[3]) {
    double a[3][3] = {{cov[0], cov[1], cov[2]}, {cov[1], cov[3], cov[4]}, {cov[2], cov[4], cov[5]}};
    double v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int sweep = 0; sweep < 64; ++sweep) {
        const double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
        const double diag = a[0][0] * a[0][0] + a[1][1] * a[1][1] + a[2][2] * a[2][2];
        if (off <= 1e-40 * (diag > 0 ? diag : 1.0)) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                if (a[p][q] == 0.0) continue;
                const double th = (a[q][q] - a[p][p]) / (2.0 * a[p][q]);
                const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), sn = t * c;
                for (int k = 0; k < 3; ++k) {   // A := A J (columns p, q)
                    const double akp = a[k][p], akq = a[k][q];
                    a[k][p] = c * akp - sn * akq;
                    a[k][q] = sn * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {   // A := J^T A (rows p, q)
                    const double apk = a[p][k], aqk = a[q][k];
                    a[p][k] = c * apk - sn * aqk;
                    a[q][k] = sn * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {   // V := V J
                    const double vkp = v[k][p], vkq = v[k][q];
                    v[k][p] = c * vkp - sn * vkq;
                    v[k][q] = sn * vkp + c * vkq;
                }
            }
    }
    int m = 0;
    for (int k = 1; k < 3; ++k)
        if (a[k][k] < a[m][m]) m = k;
    double nrm = std::sqrt(v[0][m] * v[0][m] + v[1][m] * v[1][m] + v[2][m] * v[2][m]);
    for (int k = 0; k < 3; ++k) out[k] = v[k][m] / nrm;
}

// numpy.percentile(..., method='linear') on an ascending array (numpy's _lerp form).
double percentile_linear(const double *sorted_host_lo_hi, long long n, double q, long long lo) {
    const double vi = q / 100.0 * (double)(n - 1);
    const double g = vi - (double)lo;
    const double a = sorted_host_lo_hi[0], b = sorted_host_lo_hi[1];
    const double d = b - a;
    return g >= 0.5 ? b - d * (1.0 - g) : a + d * g;
}
}  // namespace

// Per-pair cloud assembly (members/rafael/disparity/plugin.py:147-192).
int pcm_cloud_assemble(const double *disparity, const uint8_t *validity, int64_t H, int64_t W, double limit,
                       double *points, double *hnorm, int64_t *m_out, double *normal_out, void *stream) {
    if (!disparity || !points || !hnorm || !m_out || H < 1 || W < 1) return fail(PCM_E_ARG, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    const long long n = (long long)H * W;
    uint32_t *flags = nullptr, *pos = nullptr;
    double *height = nullptr, *P = nullptr, *part = nullptr, *zrel = nullptr, *zsort = nullptr;
    void *tmp = nullptr;
    int rc = 0;
    const int nb = blocks_for(n, CLOUD_TPB);
    const int sb = 1024;   // reduction blocks
    *m_out = 0;
    do {
        hipError_t err;
        if ((err = hipMalloc(&flags, n * 4)) || (err = hipMalloc(&pos, n * 4)) || (err = hipMalloc(&height, n * 8)) ||
            (err = hipMalloc(&P, n * 24)) || (err = hipMalloc(&part, (size_t)sb * 6 * 8)) ||
            (err = hipMalloc(&zrel, n * 8)) || (err = hipMalloc(&zsort, n * 8))) {
            rc = fail(PCM_E_NOMEM, "cloud workspace");
            break;
        }
        k_cloud_flags<<<nb, CLOUD_TPB, 0, s>>>(disparity, validity, n, limit, flags, height);
        if ((err = hipGetLastError())) { rc = fail(PCM_E_HIP, "k_cloud_flags"); break; }
        size_t tb = 0, tb2 = 0;
        if ((err = rocprim::exclusive_scan(nullptr, tb, flags, pos, 0u, (size_t)n, rocprim::plus<uint32_t>(), s)) ||
            (err = rocprim::radix_sort_keys(nullptr, tb2, zrel, zsort, (size_t)n, 0, 64, s)) ||
            (err = hipMalloc(&tmp, std::max(tb, tb2)))) {
            rc = fail(PCM_E_HIP, "cloud scan/sort setup");
            break;
        }
        if ((err = rocprim::exclusive_scan(tmp, tb, flags, pos, 0u, (size_t)n, rocprim::plus<uint32_t>(), s))) {
            rc = fail(PCM_E_HIP, "cloud scan");
            break;
        }
        uint32_t last_pos = 0, last_flag = 0;
        if ((err = hipMemcpyAsync(&last_pos, pos + n - 1, 4, hipMemcpyDeviceToHost, s)) ||
            (err = hipMemcpyAsync(&last_flag, flags + n - 1, 4, hipMemcpyDeviceToHost, s)) ||
            (err = hipStreamSynchronize(s))) {
            rc = fail(PCM_E_HIP, "cloud count");
            break;
        }
        const long long m = (long long)last_pos + last_flag;
        *m_out = m;
        if (m == 0) break;
        k_cloud_compact<<<nb, CLOUD_TPB, 0, s>>>(flags, pos, height, n, W, P);
        const int rb = (int)std::min<long long>(sb, (m + CLOUD_TPB - 1) / CLOUD_TPB);
        double hp[sb * 6];
        k_cloud_sums<0><<<rb, CLOUD_TPB, 0, s>>>(P, m, 0, 0, 0, part);
        if ((err = hipMemcpyAsync(hp, part, (size_t)rb * 3 * 8, hipMemcpyDeviceToHost, s)) ||
            (err = hipStreamSynchronize(s))) {
            rc = fail(PCM_E_HIP, "cloud mean");
            break;
        }
        double c[3] = {0, 0, 0};
        for (int b = 0; b < rb; ++b)
            for (int a = 0; a < 3; ++a) c[a] += hp[b * 3 + a];
        for (int a = 0; a < 3; ++a) c[a] /= (double)m;
        k_cloud_sums<1><<<rb, CLOUD_TPB, 0, s>>>(P, m, c[0], c[1], c[2], part);
        if ((err = hipMemcpyAsync(hp, part, (size_t)rb * 6 * 8, hipMemcpyDeviceToHost, s)) ||
            (err = hipStreamSynchronize(s))) {
            rc = fail(PCM_E_HIP, "cloud covariance");
            break;
        }
        double cov[6] = {0, 0, 0, 0, 0, 0};
        for (int b = 0; b < rb; ++b)
            for (int a = 0; a < 6; ++a) cov[a] += hp[b * 6 + a];
        double nv[3];
        smallest_eigvec3(cov, nv);
        if (nv[2] < 0) for (int a = 0; a < 3; ++a) nv[a] = -nv[a];   // plugin.py:167-168
        if (normal_out) for (int a = 0; a < 3; ++a) normal_out[a] = nv[a];
        const int mb = blocks_for(m, CLOUD_TPB);
        k_cloud_project<<<mb, CLOUD_TPB, 0, s>>>(P, m, c[0], c[1], c[2], nv[0], nv[1], nv[2], zrel);
        size_t tbs = tb2;
        if ((err = rocprim::radix_sort_keys(tmp, tbs, zrel, zsort, (size_t)m, 0, 64, s))) {
            rc = fail(PCM_E_HIP, "cloud sort");
            break;
        }
        double q[2] = {2.0, 98.0}, hq[2];
        for (int t = 0; t < 2; ++t) {
            const double vi = q[t] / 100.0 * (double)(m - 1);
            long long lo = (long long)std::floor(vi);
            const long long hi = std::min(lo + 1, m - 1);
            double ab[2];
            if ((err = hipMemcpyAsync(&ab[0], zsort + lo, 8, hipMemcpyDeviceToHost, s)) ||
                (err = hipMemcpyAsync(&ab[1], zsort + hi, 8, hipMemcpyDeviceToHost, s)) ||
                (err = hipStreamSynchronize(s))) {
                rc = fail(PCM_E_HIP, "cloud percentile");
                break;
            }
            hq[t] = percentile_linear(ab, m, q[t], lo);
        }
        if (rc) break;
        k_cloud_output<<<mb, CLOUD_TPB, 0, s>>>(P, zrel, m, hq[0], hq[1], points, hnorm);
        if ((err = hipGetLastError()) || (err = hipStreamSynchronize(s))) {
            rc = fail(PCM_E_HIP, std::string("cloud output: ") + hipGetErrorString(err));
            break;
        }
    } while (0);
    void *ps[] = {flags, pos, height, P, part, zrel, zsort, tmp};
    for (void *p : ps)
        if (p) (void)hipFree(p);
    return rc;
}

}  // extern "C"
