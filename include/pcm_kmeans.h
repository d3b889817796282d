/* pcm_kmeans.h — C ABI of the MI355X multi-day point-cloud K-means (Lloyd) engine.
 *
 * Drop-in boundary for the "Multi-day 3D Point Cloud" K-means step
 * (SURVEY.md §8b).  The reference has no K-means of its own: the step slots in
 * after the per-pair cloud assembly of members/rafael/disparity/plugin.py:147-192,
 * and its arithmetic follows scikit-learn's Lloyd, the only K-means the reference
 * executes (members/jasraj/land_use_classification/core.py:227-228):
 *
 *   pcm_fit_begin / pcm_iter_* / pcm_iterate   replace one call of
 *       sklearn/cluster/_kmeans.py:623-752 _kmeans_single_lloyd (its loop body is
 *       _k_means_lloyd.pyx:23-165 lloyd_iter_chunked_dense: E-step :168-213,
 *       accumulation :215-218 + :118-152, relocation _k_means_common.pyx:167-211,
 *       averaging :274-295, shift :298-311, convergence _kmeans.py:717-732);
 *   pcm_final                                 replaces the final E-step and
 *       inertia of _kmeans.py:736-750;
 *   pcm_labels / pcm_get_centers              return the fit outputs (labels in
 *       the caller's original row order, centres (K, D) float32).
 *
 * Conventions (modelled on lloyd_iter_chunked_dense's in-place contract,
 * _k_means_lloyd.pyx:23-32): caller-owned device buffers (torch tensors),
 * outputs written in place, no allocation and no host synchronisation in the
 * per-iteration entry points (pcm_iter_*, pcm_iterate, pcm_final), all work
 * ordered on the hipStream_t passed as `stream` (NULL = default stream).
 * Every function returns 0 on success or a negative PCM_E* code; the message of
 * the last failure on the calling thread is available from pcm_last_error.
 * Nothing throws across this ABI.  One engine must not be used from two
 * threads at once; distinct engines are independent.
 * Load this library after the process has loaded libamdhip64.so.7 (e.g. after
 * `import torch`) so that one HIP runtime serves both.
 */
#ifndef PCM_KMEANS_H
#define PCM_KMEANS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCM_ABI_VERSION 6

enum pcm_dtype { PCM_F32 = 0, PCM_F16 = 1, PCM_F64 = 2 /* dense path only */ };

#define PCM_DENSE_DMAX 64   /* features of the generic-D (dense) path */

enum pcm_err {
    PCM_OK = 0,
    PCM_E_ARG = -1,      /* invalid argument / shape */
    PCM_E_HIP = -2,      /* HIP runtime or kernel launch failure */
    PCM_E_STATE = -3,    /* call out of order (e.g. iterate before layout) */
    PCM_E_NONFINITE = -4,/* input points contain NaN or Inf */
    PCM_E_NOMEM = -5
};

/* Device-side iteration status, copied to the host by pcm_read_status. */
typedef struct pcm_status {
    uint32_t halt;       /* 1: empty clusters need relocation (pcm_reloc_*) */
    uint32_t done;       /* 0 running, 1 strict label convergence, 2 shift<=tol, 3 max_iter,
                            4 a peer exchange timed out (pcm_iter_exchange; the fit is void),
                            5 the update's publisher block timed out waiting for its list blocks (void) */
    uint32_t iter;       /* completed Lloyd iterations */
    uint32_t n_empty;    /* empty clusters seen by the halted iteration */
    double inertia;      /* local inertia of the last pcm_final (= pcm_inertia_value of the fields below) */
    uint64_t last_changed;   /* statistic words (of K*(D+1)) that differ from the previous iteration's:
                                NOT a count of changed labels -- 0 exactly when no label changed */
    double last_shift;
    /* Exact, order-independent inertia: sum over points of trunc(d * 2^scale)
     * (d = canonical fp32 distance to the final centre) as 32-bit limbs
     * inertia_limbs[0] + 2^32 [1] + 2^64 [2].  Sum-all-reduce the limbs over
     * ranks, then pcm_inertia_value gives the global inertia; the result is
     * bit-identical for any world size. */
    uint64_t inertia_limbs[3];
    int32_t inertia_scale;
    uint32_t inertia_overflow;   /* > 0: a distance exceeded the bound (inertia = +inf) */
    uint32_t list_rebuilds;      /* candidate-list rebuilds so far in this fit (the other iterations
                                    only refreshed the lists' centre records) */
    uint32_t pad_;
} pcm_status;

typedef struct pcm_engine pcm_engine;

int pcm_abi_version(void);
/* Inertia from (all-reduced) limbs: ldexp((double)(l0 + l1 2^32 + l2 2^64), -scale),
 * one correctly rounded conversion; +inf when overflow > 0. */
double pcm_inertia_value(const uint64_t *limbs, int scale, uint32_t overflow);
int pcm_last_error(char *buf, size_t n);

/* Create an engine for D-dimensional points (1..4), K clusters, on HIP device
 * `device`.  `max_iter` sizes the per-iteration history. */
int pcm_engine_create(int device, int d, int k, int dtype, int max_iter, pcm_engine **out);
int pcm_engine_destroy(pcm_engine *e);

/* Layout, step 1 (host-synchronising, once per point cloud): local bounding box
 * of X (n rows, row-major, dtype given at create) on device.  Writes lo[d],
 * hi[d], maxabs[d] (host arrays).  Returns PCM_E_NONFINITE for NaN/Inf input. */
int pcm_layout_bbox(pcm_engine *e, const void *X, int64_t n, void *stream,
                    double *lo, double *hi, double *maxabs);

/* Layout, step 2 (host-synchronising, once): bin rows into the pruning grid,
 * sort them into cell order (AoSoA-4: groups of 4 points stored coordinate-major)
 * and build the tile list.  `q` are the
 * GLOBAL fixed-point exponents (identical on every rank), `gidx0` the global row
 * index of local row 0 (relocation tie-break).  X must stay unchanged until
 * this call returns. */
int pcm_layout_build(pcm_engine *e, const void *X, const int32_t *q, int64_t gidx0, void *stream);

/* Optional, at engine setup: grow (and zero) the point-sized device buffers a
 * layout of up to `n` points needs, so that the first pcm_layout_build of a
 * process allocates nothing large (a fresh process's first allocations map
 * and clear new VRAM).  Buffers only grow; invalidates the current layout.
 * No reference counterpart (the reference allocates per call). */
int pcm_engine_reserve(pcm_engine *e, int64_t n, void *stream);

/* Layout, optional step between pcm_layout_bbox and pcm_layout_build: the
 * engine's cloud is a SPATIAL shard of a fit over `n_global` points on all
 * ranks (pcm_shard_* below).  `rows` (device uint32[n], copied) is each local
 * point's global row index -- the relocation tie-break (distance desc, global
 * row asc, _k_means_common.pyx:185-187) -- and n_global scales the pruning-grid
 * policy (cells per centre) to the whole cloud.  Reset by pcm_layout_bbox. */
int pcm_layout_shard(pcm_engine *e, const uint32_t *rows, int64_t n_global, void *stream);

/* Start a fit from centres C0 (device, K*D float32): labels := -1, history
 * cleared, absolute shift tolerance `tol`, iteration cap `max_iter`. */
int pcm_fit_begin(pcm_engine *e, const float *C0, double tol, int max_iter, void *stream);

/* One Lloyd iteration split at the all-reduce:
 *   pcm_iter_local   assign + exact accumulation of the local integer
 *                    statistics straight into the buffer of pcm_stats_ptr;
 *   (caller all-reduces that buffer with SUM over ranks when world size > 1)
 *   pcm_iter_global  empty-cluster check (may set halt), averaging, shift,
 *                    convergence flags, the next iteration's candidate lists;
 *                    zeroes the statistics buffer for the next iteration.
 * Both are gated on the device: after convergence or halt they are no-ops. */
int pcm_iter_local(pcm_engine *e, void *stream);
int pcm_iter_global(pcm_engine *e, void *stream);
/* n x (local, global) on one device without any host synchronisation. */
int pcm_iterate(pcm_engine *e, int n, void *stream);

/* Device pointer + element count (int64) of the per-iteration statistics
 * buffer: K*(D+1) offset-encoded fixed-point sums and counts, then 1 change
 * count.  Sum-all-reduce it between pcm_iter_local and pcm_iter_global. */
int pcm_stats_ptr(pcm_engine *e, void **ptr, int64_t *count);
/* Use a caller-owned device buffer of pcm_stats_ptr's count int64 elements
 * (e.g. a torch tensor handed to torch.distributed.all_reduce) instead of the
 * engine's own; NULL reverts to the engine buffer. */
int pcm_bind_stats(pcm_engine *e, void *ptr);

/* Empty-cluster relocation (run only after pcm_read_status reports halt):
 * write this rank's `m` farthest-from-centre points as 32-byte records to
 * `records` (device, m*32 bytes); the caller concatenates every rank's records
 * (all-gather) and passes all `n_rec` of them to pcm_reloc_apply, which picks
 * the global farthest, moves them into the empty clusters, clears halt and
 * completes the iteration. */
int pcm_reloc_candidates(pcm_engine *e, int m, void *records, void *stream);
int pcm_reloc_apply(pcm_engine *e, const void *records, int n_rec, void *stream);

/* Final E-step with the final centres (labels + local inertia). */
int pcm_final(pcm_engine *e, void *stream);
/* Labels in the caller's original row order (device int32[n]). */
int pcm_labels(pcm_engine *e, int32_t *out, void *stream);
/* Current centres (device float32[K*D]). */
int pcm_get_centers(pcm_engine *e, float *out, void *stream);
/* Per-iteration history (host arrays of length >= iter): changed statistic words
 * (as pcm_status.last_changed; 0 exactly when no label changed), shifts. */
int pcm_history(pcm_engine *e, uint64_t *changed, double *shift, int cap, void *stream);
/* Synchronise `stream` and copy the device status. */
int pcm_read_status(pcm_engine *e, pcm_status *out, void *stream);
/* The same without draining the stream (round 6): pcm_status_post queues a
 * snapshot of the status behind the work enqueued so far; pcm_status_wait
 * blocks until that snapshot has landed and decodes it.  One snapshot in flight
 * per engine (a post overwrites the previous one). */
int pcm_status_post(pcm_engine *e, void *stream);
int pcm_status_wait(pcm_engine *e, pcm_status *out);

/* Layout facts for diagnostics: cells, tiles, grid dims (host ints). */
int pcm_layout_info(pcm_engine *e, int64_t *ncells, int64_t *ntiles, int *grid /*[4]*/);
/* Bytes the assign kernel streams per iteration for the current layout (points
 * in compressed tiles at 8 B, the others at d * sizeof(dtype)) and the number
 * of compressed points (synchronising; see DESIGN.md §3, compressed stream). */
int pcm_layout_stream_bytes(pcm_engine *e, double *bytes, int64_t *compressed_points);
/* Name of the assign-kernel variant the current layout launches per iteration
 * (e.g. "k_lloyd1<float,3,8,false>"), for measurement records. */
int pcm_assign_kernel_name(pcm_engine *e, char *buf, size_t n);
/* Mean/max fine candidate-list length of the last iteration (synchronising). */
int pcm_candidate_stats(pcm_engine *e, double *mean, int *max, int64_t *full_cells, void *stream);
/* Crowded layouts (cells holding many tiles' worth of points, e.g. tight
 * clusters): the Morton levels of the in-cell point order (0: not crowded),
 * the tiles of cells whose list is FULL or longer than 16 at the last
 * iteration, how many of them got a shorter tile list and those lists' summed
 * length (synchronising). */
int pcm_tile_list_stats(pcm_engine *e, int *zlev, int64_t *crowded_tiles, int64_t *listed_tiles, int64_t *listed_len,
                        void *stream);
/* Crowded layouts, the long-list paths of the assign kernel: tile lists longer
 * than 256 (scanned through LDS chunks), all-K tiles (a FULL cell's tile with no
 * list of at most 1024) and the longest tile list (synchronising; 0 when not
 * crowded). */
int pcm_tile_list_detail(pcm_engine *e, int64_t *long_lists, int64_t *allk_tiles, int64_t *max_len, void *stream);

/* Kernel timing on the engine's launch stream (HIP events around every launch
 * of the assign kernel and of the candidate and tail kernels).  enable=1 starts
 * recording (resets the sums), pcm_timing_read synchronises and returns mean
 * milliseconds per iteration for: [0] assign, [1] candidates, [2] fold+global,
 * and the number of iterations timed. */
int pcm_timing(pcm_engine *e, int enable);
int pcm_timing_read(pcm_engine *e, double *ms /*[3]*/, int *count);

/* Calibration: mean milliseconds of `reps` back-to-back assign launches on the
 * current layout and centres, between one HIP event pair.  The statistics they
 * add are discarded; the engine needs pcm_fit_begin before iterating again. */
int pcm_time_assign(pcm_engine *e, int reps, void *stream, double *ms);

/* Rows `rows[0..m)` (device int64) of the synthetic cloud, device float32[m*d]. */
int pcm_synth_rows(float *out, const int64_t *rows, int64_t m, int d, uint64_t seed, void *stream);

/* Counter-based U[0,1) synthetic cloud (identical to oracle.splitmix_uniform):
 * out[(i)*d + a] for rows [start, start+n), device float32. */
int pcm_synth_uniform(float *out, int64_t n, int d, uint64_t seed, int64_t start, void *stream);

/* Stateless operator (sklearn lloyd_iter_chunked_dense shape, unit weights,
 * brute force over all K, LDS-staged centres): labels (device int32[n]) and
 * integer statistics (device uint64[K*(D+1)], accumulated, caller zeroes)
 * for centres C (device float32[K*D]).  q = fixed-point exponents. */
int pcm_assign_bruteforce(const float *X, int64_t n, int d, const float *C, int k,
                          const int32_t *q, int32_t *labels, uint64_t *stats, void *stream);

/* ---------------------------------------------------------------- slab sharding
 * Multi-GPU layout (no reference counterpart -- the reference is
 * single-process): the row shards the ranks receive are regrouped into slabs
 * of the longest axis so that each rank's pruning grid covers only its slab.
 * X: device n*d rows (dtype PCM_F32/PCM_F16) whose global row index is gidx0 + i.
 * bin(x) = clamp(floor((x[axis] - lo) * inv), 0, nbins - 1), computed in fp64.
 *   pcm_shard_hist       hist[nbins] (device uint64, overwritten), nbins <= 16384;
 *   pcm_shard_partition  stable partition by owner[bin] (device uint8[nbins],
 *                        values < P): X_out (device n*d) holds the rows grouped
 *                        by destination rank in original order, rows_out
 *                        (device uint32[n]) their global indices, counts (host
 *                        int64[P]) the group sizes; synchronises `stream`;
 *   pcm_shard_scatter_labels  out[rows[i] - gidx0] = labels[i] (device int32):
 *                        labels returned in the partition's order -> row order. */
#define PCM_SHARD_MAXP 16
int pcm_shard_hist(const void *X, int dtype, int64_t n, int d, int axis, double lo, double inv, int nbins,
                   uint64_t *hist, void *stream);
int pcm_shard_partition_workspace(int64_t n, int P, size_t *bytes);
int pcm_shard_partition(const void *X, int dtype, int64_t n, int d, int axis, double lo, double inv, int nbins,
                        const uint8_t *owner, int P, int64_t gidx0, void *X_out, uint32_t *rows_out, int64_t *counts,
                        void *workspace, size_t workspace_bytes, void *stream);
int pcm_shard_scatter_labels(const int32_t *labels, const uint32_t *rows, int64_t n, int64_t gidx0, int32_t *out,
                             void *stream);

/* ---------------------------------------------------------------- peer exchange
 * One-sided SUM of the per-iteration statistics over the ranks (SURVEY.md §8e;
 * no reference counterpart -- the reference is single-process): it replaces the
 * RCCL all-reduce between pcm_iter_local and pcm_iter_global by writes into the
 * peers' memory.  Each rank creates one exchange of `words` int64 (pcm_stats_ptr's
 * count); its receive buffer (2 x P slots + flags, uncached device memory) is made
 * reachable to the other ranks by pcm_xchg_handle -> pcm_xchg_open (another
 * process: IPC) or pcm_xchg_link (an exchange of the same process).  Every rank
 * must run the same sequence of exchanges.
 *   pcm_xchg_allreduce  buf (device uint64[words]) := SUM over ranks, in place,
 *                       stream-ordered, no host synchronisation (graph-capturable);
 *                       phase 1 = push only, 2 = wait + sum only, 3 = both;
 *   pcm_iter_exchange   the same on the engine's statistics buffer, gated by the
 *                       engine's device control block like pcm_iter_*; a wait
 *                       longer than timeout_s sets status done = 4 (exchange
 *                       failed) and gates the rest of the fit;
 *   pcm_xchg_status     synchronises `stream`: err (1 = a wait timed out), and
 *                       the number of exchanges completed. */
#define PCM_XCHG_MAXP 16
#define PCM_XCHG_HANDLE_BYTES 64
typedef struct pcm_xchg pcm_xchg;
int pcm_xchg_create(int device, int64_t words, int nranks, int rank, double timeout_s, pcm_xchg **out);
int pcm_xchg_destroy(pcm_xchg *x);
int pcm_xchg_handle(pcm_xchg *x, void *handle /* PCM_XCHG_HANDLE_BYTES */);
int pcm_xchg_open(pcm_xchg *x, int peer, const void *handle);
int pcm_xchg_link(pcm_xchg *x, int peer, pcm_xchg *other);
int pcm_xchg_allreduce(pcm_xchg *x, uint64_t *buf, int phase, void *stream);
int pcm_xchg_status(pcm_xchg *x, uint32_t *err, uint64_t *epoch, void *stream);
int pcm_iter_exchange(pcm_engine *e, pcm_xchg *x, int phase, void *stream);

/* k-means++ seeding, replacing scikit-learn's _kmeans_plusplus
 * (sklearn/cluster/_kmeans.py:174-272; KMeans' default init, :1012-1019; the
 * reference's call site members/jasraj/land_use_classification/core.py:227-228)
 * with the canonical arithmetic of oracle/kpp_ref.py.  X: device float32[n*d]
 * (row order = the caller's); first_index: the first centre (sklearn's
 * random_state.choice draw, computed by the host); umant: host uint64
 * [(k-1)*n_local_trials], each uniform of random_state.uniform(size=L) for
 * centres 1..k-1 as its exact 53-bit mantissa (u * 2^53).  The weight
 * exponent is kpp_scale(n, sum_a (max_a - min_a)^2) of the device bounding box.
 * Writes indices (device int64[k]), stream-ordered; synchronises once (bounding
 * box -> pruning grid) and returns PCM_E_NONFINITE for NaN/Inf input.
 * workspace: caller-owned device memory of pcm_kmeanspp_workspace bytes. */
int pcm_kmeanspp_workspace(int64_t n, int d, int k, int n_local_trials, size_t *bytes);
int pcm_kmeanspp(const float *X, int64_t n, int d, int k, int n_local_trials, int64_t first_index,
                 const uint64_t *umant, int64_t *indices, void *workspace, size_t workspace_bytes, void *stream);

/* Per-pair point-cloud assembly, replacing the float64 NumPy block of
 * members/rafael/disparity/plugin.py:147-192 (height = -disparity/16, validity
 * mask, np.where row-major compaction, SVD plane fit oriented to +z, relative
 * height, 2/98 percentiles, points (z - h_min, y, x) + 'height' property).
 * disparity: device float64[H*W]; validity: device uint8[H*W] or NULL;
 * limit = MAX_DISP/2.  points: device float64[3*H*W] capacity, hnorm:
 * device float64[H*W] capacity; *m_out = number of points; normal_out (host
 * double[3], nullable) = the fitted plane normal.  Synchronises the stream. */
int pcm_cloud_assemble(const double *disparity, const uint8_t *validity, int64_t H, int64_t W, double limit,
                       double *points, double *hnorm, int64_t *m_out, double *normal_out, void *stream);

/* ---------------------------------------------------------------- stereo gathers
 * Per-pixel consistency maps of a rectified pair (H x W, row-major, device):
 * pcm_photoconsistency replaces members/rafael/disparity/processing.py:94-115
 * photoconsistency_map (left/right images PCM_F32 or PCM_F64, left_disp
 * float64 = disparity / 16; out float64 |right[y, rint(x - d)] - left[y, x]| / 255,
 * 0 where undefined); pcm_lr_consistency replaces disparity.py:229-250
 * left_right_consistency (out float64 |rd[y, rint(x - d)] + ld[y, x]|, max_disp
 * where undefined; below (nullable) uint8 = out < threshold, the caller's
 * `< 3` of disparity.py:170-172; out may be NULL when only the mask is
 * wanted).  Undefined: d NaN, rint(x - d) outside [0, W), or d < min_disp.
 * Stream-ordered, no synchronisation. */
int pcm_photoconsistency(const void *left, const void *right, int img_dtype, const double *left_disp, int64_t H,
                         int64_t W, double min_disp, double *out, void *stream);
int pcm_lr_consistency(const double *left_disp, const double *right_disp, int64_t H, int64_t W, double min_disp,
                       double max_disp, double *out, uint8_t *below, double threshold, void *stream);

/* ---------------------------------------------------------------- dense path
 * Generic-D Lloyd K-means for feature vectors (D <= PCM_DENSE_DMAX, float32 or
 * float64, computed in that precision), replacing one _kmeans_single_lloyd
 * call (sklearn/cluster/_kmeans.py:623-752) at the reference's KMeans call site
 * members/jasraj/land_use_classification/core.py:227-228 (~1500 x 20 float64).
 * Brute force over all K with the centres staged in LDS when k*d*sizeof <= 64 KB (else read from L2);
 * canonical arithmetic of oracle/dense_ref.py; everything on the device, one
 * process (no sharding).  X (device, n*d, row-major) must stay valid and
 * unchanged from pcm_dense_begin to the last call of the fit.  maxabs (host
 * double[d]) = max |X[:, a]| fixes the exact fixed-point sums. */
typedef struct pcm_dense pcm_dense;
int pcm_dense_create(int device, int64_t n, int d, int k, int dtype, int max_iter, pcm_dense **out);
int pcm_dense_destroy(pcm_dense *e);
/* centres C0: device k*d of dtype; labels := -1, history cleared (synchronises). */
int pcm_dense_begin(pcm_dense *e, const void *X, const double *maxabs, const void *C0, double tol, int max_iter,
                    void *stream);
/* n_iter Lloyd iterations (E-step + update), gated on the device after convergence. */
int pcm_dense_iterate(pcm_dense *e, int n_iter, void *stream);
/* Final E-step with the final centres: labels + exact inertia limbs. */
int pcm_dense_final(pcm_dense *e, void *stream);
/* Status (synchronises): done/iter/last_*, inertia; list_rebuilds = relocation events. */
int pcm_dense_status(pcm_dense *e, pcm_status *out, void *stream);
/* Outputs (synchronises): labels device int32[n], centres device k*d dtype,
 * history host uint64/double[cap]; any pointer may be NULL. */
int pcm_dense_outputs(pcm_dense *e, int32_t *labels, void *centers, uint64_t *changed, double *shift, int cap,
                      void *stream);
/* k-means++ for the dense path (oracle/kpp_ref.py canonical seeding in the
 * input precision), brute force; scale = kpp_scale(n, max distance bound). */
int pcm_dense_kmeanspp_workspace(int64_t n, int d, int dtype, int k, int n_local_trials, size_t *bytes);
int pcm_dense_kmeanspp(const void *X, int64_t n, int d, int dtype, int k, int n_local_trials, int64_t first_index,
                       const uint64_t *umant, int scale, int64_t *indices, void *workspace, size_t workspace_bytes,
                       void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PCM_KMEANS_H */
