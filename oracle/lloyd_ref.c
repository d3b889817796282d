/* Scalar/OpenMP C restatement of the canonical Lloyd E-step + exact accumulation.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ (as the bit-exact checker at sizes
 * where numpy is too slow) and by bench.py's cpu_baseline leg (timed on the GPU
 * box's host cores).  Never linked into or called by the product path.
 *
 * Semantics are those of oracle/lloyd_ref.py (which cites the scikit-learn
 * lines it follows): _k_means_lloyd.pyx:168-218 (argmin with strict '<', lowest
 * index wins; per-cluster sums), with the build's canonical fp32 distance
 * ((d0*d0 + d1*d1) + d2*d2) + d3*d3 and int64 fixed-point sums.
 * Compile with -ffp-contract=off (no FMA contraction) and without -ffast-math.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define PB 16   /* points per vector block */

static inline float dist_canon(const float *x, const float *c, int d) {
    float a = x[0] - c[0];
    float acc = a * a;
    for (int t = 1; t < d; ++t) {
        float b = x[t] - c[t];
        float sq = b * b;
        acc = acc + sq;
    }
    return acc;
}

/* labels[i] = argmin_j dist(x_i, c_j); also counts changes vs labels_old
 * (nullable) and, when sums/counts are non-null, accumulates exact int64
 * fixed-point sums: xq = trunc(ldexpf(x, q[a])).  Returns n_changed. */
int64_t ref_lloyd_stats(const float *X, int64_t n, int d, const float *C, int k,
                        const int32_t *q, const int32_t *labels_old,
                        int32_t *labels, int64_t *sums, int64_t *counts,
                        int nthreads) {
    int64_t n_changed = 0;
    if (nthreads <= 0) nthreads = 1;
    int nt = nthreads;
    int64_t *tsums = NULL, *tcnt = NULL;
    if (sums) {
        tsums = (int64_t *)calloc((size_t)nt * k * d, sizeof(int64_t));
        tcnt = (int64_t *)calloc((size_t)nt * k, sizeof(int64_t));
    }
    /* transpose centroids to [d][k] for contiguous inner loops */
    float *Ct = (float *)malloc((size_t)k * d * sizeof(float));
    for (int j = 0; j < k; ++j)
        for (int t = 0; t < d; ++t) Ct[(size_t)t * k + j] = C[(size_t)j * d + t];

#pragma omp parallel num_threads(nt) reduction(+ : n_changed)
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        int64_t *ms = sums ? tsums + (size_t)tid * k * d : NULL;
        int64_t *mc = sums ? tcnt + (size_t)tid * k : NULL;
        int64_t nblk = (n + PB - 1) / PB;
#pragma omp for schedule(static)
        for (int64_t b = 0; b < nblk; ++b) {
            int64_t i0 = b * PB;
            int np_ = (int)((n - i0) < PB ? (n - i0) : PB);
            float xs[4][PB];
            float bestd[PB];
            int32_t bestj[PB];
            for (int p = 0; p < PB; ++p)
                for (int t = 0; t < 4; ++t)
                    xs[t][p] = (p < np_ && t < d) ? X[(i0 + p) * d + t] : 0.0f;
            for (int p = 0; p < PB; ++p) {
                float a = xs[0][p] - Ct[0];
                float acc = a * a;
                for (int t = 1; t < d; ++t) {
                    float bb = xs[t][p] - Ct[(size_t)t * k];
                    float sq = bb * bb;
                    acc = acc + sq;
                }
                bestd[p] = acc;
                bestj[p] = 0;
            }
            for (int j = 1; j < k; ++j) {
                float c0 = Ct[j];
                float c1 = d > 1 ? Ct[(size_t)k + j] : 0.0f;
                float c2 = d > 2 ? Ct[(size_t)2 * k + j] : 0.0f;
                float c3 = d > 3 ? Ct[(size_t)3 * k + j] : 0.0f;
                if (d == 3) {
#pragma omp simd
                    for (int p = 0; p < PB; ++p) {
                        float e0 = xs[0][p] - c0, e1 = xs[1][p] - c1, e2 = xs[2][p] - c2;
                        float s0 = e0 * e0, s1 = e1 * e1, s2 = e2 * e2;
                        float acc = s0 + s1;
                        acc = acc + s2;
                        int m = acc < bestd[p];
                        bestd[p] = m ? acc : bestd[p];
                        bestj[p] = m ? j : bestj[p];
                    }
                } else if (d == 4) {   /* config 5: the same canonical order, vectorised over the block */
#pragma omp simd
                    for (int p = 0; p < PB; ++p) {
                        float e0 = xs[0][p] - c0, e1 = xs[1][p] - c1, e2 = xs[2][p] - c2, e3 = xs[3][p] - c3;
                        float s0 = e0 * e0, s1 = e1 * e1, s2 = e2 * e2, s3 = e3 * e3;
                        float acc = s0 + s1;
                        acc = acc + s2;
                        acc = acc + s3;
                        int m = acc < bestd[p];
                        bestd[p] = m ? acc : bestd[p];
                        bestj[p] = m ? j : bestj[p];
                    }
                } else {
                    for (int p = 0; p < PB; ++p) {
                        float e0 = xs[0][p] - c0;
                        float acc = e0 * e0;
                        if (d > 1) { float e1 = xs[1][p] - c1; float s1 = e1 * e1; acc = acc + s1; }
                        if (d > 2) { float e2 = xs[2][p] - c2; float s2 = e2 * e2; acc = acc + s2; }
                        if (d > 3) { float e3 = xs[3][p] - c3; float s3 = e3 * e3; acc = acc + s3; }
                        int m = acc < bestd[p];
                        bestd[p] = m ? acc : bestd[p];
                        bestj[p] = m ? j : bestj[p];
                    }
                }
            }
            for (int p = 0; p < np_; ++p) {
                int64_t i = i0 + p;
                int32_t lab = bestj[p];
                labels[i] = lab;
                if (labels_old && labels_old[i] != lab) n_changed++;
                if (!labels_old) n_changed++;
                if (ms) {
                    mc[lab] += 1;
                    for (int t = 0; t < d; ++t)
                        ms[(size_t)lab * d + t] += (int64_t)ldexpf(xs[t][p], q[t]);   /* trunc */
                }
            }
        }
    }
    if (sums) {
        memset(sums, 0, (size_t)k * d * sizeof(int64_t));
        memset(counts, 0, (size_t)k * sizeof(int64_t));
        for (int t = 0; t < nt; ++t) {
            for (size_t e = 0; e < (size_t)k * d; ++e) sums[e] += tsums[(size_t)t * k * d + e];
            for (int j = 0; j < k; ++j) counts[j] += tcnt[(size_t)t * k + j];
        }
        free(tsums);
        free(tcnt);
    }
    free(Ct);
    (void)dist_canon;
    return n_changed;
}

int ref_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
