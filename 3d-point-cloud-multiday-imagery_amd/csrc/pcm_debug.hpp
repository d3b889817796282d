// pcm_debug.hpp — calibration-only phase stamps of the kernels (debug builds:
// tools/build_variant.sh NAME -DPCM_DBG_TIMING, read back by the pcm_debug_*
// entry points and tools/*_timing.py).  Product builds compile every macro
// below to nothing.
#pragma once
#include <hip/hip_runtime.h>

namespace pcm {

#ifdef PCM_DBG_TIMING
__device__ unsigned long long g_dbg_t[8192][16];
#define DBG_T(k) do { if (threadIdx.x == 0 && blockIdx.x < 8192) g_dbg_t[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define DBG_V(k, v) do { if (threadIdx.x == 0 && blockIdx.x < 8192) g_dbg_t[blockIdx.x][k] = (unsigned long long)(v); } while (0)
__device__ unsigned long long g_dbg_l[65536][8];
#define DBG_L(k) do { if (threadIdx.x == 0 && blockIdx.x < 65536) g_dbg_l[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
// k_lloyd1 block info: [5] HW_ID (cu/sh/se), [6] XCC_ID, [7] list length | tile points << 16
#define DBG_LV(k, v) do { if (threadIdx.x == 0 && blockIdx.x < 65536) g_dbg_l[blockIdx.x][k] = (unsigned long long)(v); } while (0)
__device__ unsigned long long g_dbg_e[8192][8];
// k-means++ per-step work counters [centre][eval items, eval reached cells, apply items, apply reached]
__device__ unsigned long long g_dbg_kpp[4096][4];
#define DBG_KPP(c, k, v) do { if ((c) < 4096 && (v)) atomicAdd(&g_dbg_kpp[c][k], (unsigned long long)(v)); } while (0)
#define DBG_E(k) do { if (threadIdx.x == 0 && blockIdx.x < 8192) g_dbg_e[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define DBG_EV(k, v) do { if (threadIdx.x == 0 && blockIdx.x < 8192) g_dbg_e[blockIdx.x][k] = (unsigned long long)(v); } while (0)
#else
#define DBG_E(k) do { } while (0)
#define DBG_EV(k, v) do { } while (0)
#define DBG_KPP(c, k, v) do { } while (0)
#define DBG_T(k) do { } while (0)
#define DBG_V(k, v) do { } while (0)
#define DBG_L(k) do { } while (0)
#define DBG_LV(k, v) do { } while (0)
#endif

}  // namespace pcm
