// pcm_xchg.hpp — internal entry of the one-sided statistics exchange
// (pcm_xchg.hip), shared with the engine's pcm_iter_exchange.
#pragma once
#include <hip/hip_runtime.h>

#include "pcm_kmeans.h"

// phase bit 1: push this rank's `buf` into every peer's slot; bit 2: wait for
// the peers' pushes and add their slots into `buf`.  `gate` (nullable) points
// at the engine control block's {halt, done} words: both kernels are no-ops
// when either is set, and a timed-out wait sets done = 4.
int pcm_xchg_launch(pcm_xchg *x, unsigned long long *buf, unsigned int *gate, int phase, hipStream_t s);
