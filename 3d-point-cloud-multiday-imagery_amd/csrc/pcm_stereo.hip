// pcm_stereo.hip — stereo consistency gathers on gfx950.
//
//   k_photo  members/rafael/disparity/processing.py:94-115 photoconsistency_map
//   k_lrc    members/rafael/disparity/disparity.py:229-250 left_right_consistency
//
// One thread per pixel of an H x W row-major image.  xd = rint(x - d) (round
// half to even, as np.round); the pixel is undefined when d is NaN, xd falls
// outside [0, W) or d < min_disp.  Photoconsistency: |right[y, xd] -
// left[y, x]| / 255 in float64 (0 when undefined); L/R consistency:
// |right_disp[y, xd] + left_disp[y, x]| (max_disp when undefined), optionally
// thresholded (< threshold, disparity.py:170-172) into a uint8 mask in the same
// pass.  HBM-bound streaming kernels: the gather stays within the pixel's own
// row (cache-resident); 24 B/px (photo, float32 images) and 32 B/px (+1 for
// the mask) of algorithmic traffic.
#include <hip/hip_runtime.h>

#include <string>

#include "pcm_common.hpp"
#include "pcm_kmeans.h"

namespace pcm {

__device__ __forceinline__ bool stereo_gather(double d, long long x, long long W, double min_disp, long long &xd) {
    const double f = __builtin_rint((double)x - d);
    const bool undefined = __builtin_isnan(d) || !(f >= 0.0) || !(f < (double)W) || d < min_disp;
    xd = undefined ? x : (long long)f;
    return undefined;
}

template <typename T>
__global__ __launch_bounds__(256) void k_photo(const T *__restrict__ left, const T *__restrict__ right,
                                               const double *__restrict__ disp, long long H, long long W,
                                               double min_disp, double *__restrict__ out) {
    for (long long y = blockIdx.y; y < H; y += gridDim.y) {
        const long long row = y * W;
        for (long long x = blockIdx.x * (long long)blockDim.x + threadIdx.x; x < W; x += (long long)gridDim.x * blockDim.x) {
            long long xd;
            const bool und = stereo_gather(disp[row + x], x, W, min_disp, xd);
            const double v = __builtin_fabs((double)right[row + xd] - (double)left[row + x]) / 255.0;
            out[row + x] = und ? 0.0 : v;
        }
    }
}

__global__ __launch_bounds__(256) void k_lrc(const double *__restrict__ ld, const double *__restrict__ rd, long long H,
                                             long long W, double min_disp, double max_disp, double *__restrict__ out,
                                             uint8_t *__restrict__ below, double threshold) {
    for (long long y = blockIdx.y; y < H; y += gridDim.y) {
        const long long row = y * W;
        for (long long x = blockIdx.x * (long long)blockDim.x + threadIdx.x; x < W; x += (long long)gridDim.x * blockDim.x) {
            long long xd;
            const double d = ld[row + x];
            const bool und = stereo_gather(d, x, W, min_disp, xd);
            const double v = und ? max_disp : __builtin_fabs(rd[row + xd] + d);
            if (out) out[row + x] = v;
            if (below) below[row + x] = v < threshold ? 1 : 0;
        }
    }
}

}  // namespace pcm

using namespace pcm;

namespace {
dim3 stereo_grid(long long H, long long W) {
    const long long bx = (W + 255) / 256;
    return dim3((unsigned)std::min<long long>(bx, 1 << 16), (unsigned)std::min<long long>(H, 65535), 1);
}
}  // namespace

extern "C" {

int pcm_photoconsistency(const void *left, const void *right, int img_dtype, const double *left_disp, int64_t H,
                         int64_t W, double min_disp, double *out, void *stream) {
    if (!left || !right || !left_disp || !out || H < 1 || W < 1) return pcm_fail(PCM_E_ARG, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    if (img_dtype == PCM_F32)
        k_photo<float><<<stereo_grid(H, W), 256, 0, s>>>((const float *)left, (const float *)right, left_disp, H, W,
                                                        min_disp, out);
    else if (img_dtype == PCM_F64)
        k_photo<double><<<stereo_grid(H, W), 256, 0, s>>>((const double *)left, (const double *)right, left_disp, H, W,
                                                         min_disp, out);
    else
        return pcm_fail(PCM_E_ARG, "img_dtype must be PCM_F32 or PCM_F64");
    if (hipError_t e = hipGetLastError()) return pcm_fail(PCM_E_HIP, std::string("k_photo: ") + hipGetErrorString(e));
    return 0;
}

int pcm_lr_consistency(const double *left_disp, const double *right_disp, int64_t H, int64_t W, double min_disp,
                       double max_disp, double *out, uint8_t *below, double threshold, void *stream) {
    if (!left_disp || !right_disp || (!out && !below) || H < 1 || W < 1) return pcm_fail(PCM_E_ARG, "bad argument");
    k_lrc<<<stereo_grid(H, W), 256, 0, (hipStream_t)stream>>>(left_disp, right_disp, H, W, min_disp, max_disp, out,
                                                              below, threshold);
    if (hipError_t e = hipGetLastError()) return pcm_fail(PCM_E_HIP, std::string("k_lrc: ") + hipGetErrorString(e));
    return 0;
}

}  // extern "C"
