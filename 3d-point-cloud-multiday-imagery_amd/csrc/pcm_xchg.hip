// pcm_xchg.hip — one-sided cross-rank SUM of the per-iteration statistics.
//
// The multi-GPU Lloyd iteration (lloyd.run) sums K*(D+1)+1
// int64 statistics over the ranks between the assign kernel and the update.
// Through RCCL that is a 32 KiB all-reduce whose fixed cost (14-15 us even for a
// group of one inside a captured graph, profiles/rd5_split_graph_vs_eager.txt)
// is a quarter of an 8-way slab's iteration.  This exchange replaces it by
// peer-memory writes: every rank owns a receive buffer of 2 x P slots (one per
// sender, double-buffered by exchange parity) plus 2 x 16 flag words and the
// exchange's state words (epoch, block arrivals, error), allocated fine-grained
// (hipDeviceMallocFinegrained: coherent for the system-scope accesses of other
// agents) and exposed to the other ranks by IPC handle (other processes) or
// directly (engines of one process: the 1-GPU slab proxy of bench.py).
//
//   k_xpush    one block per peer: the rank's statistics (its own buffer, written
//              by the assign kernel) into slot [parity][rank] of that peer's
//              buffer, every storing wave drains its stores, one lane issues a
//              system-scope release and then the flag word [parity][rank] := epoch + 1
//   k_xsum     wave 0 of every block polls the P - 1 flags of its parity
//              (system-scope loads, s_sleep between polls, bounded by a wall-clock
//              timeout), a system-scope acquire, then the block sums its slice of the words -- the own
//              statistics plus every peer slot -- into the own buffer, which the
//              update kernel reads as the all-reduced statistics.  The last block
//              to finish advances the local epoch.
//
// Integer sums are order-independent, so the result is bit-identical to the
// RCCL all-reduce (and to one GPU).  Double buffering is enough: a rank starts
// its push of exchange e + 2 (same parity as e) only after its sum of e + 1,
// which needed every peer's push of e + 1, which each peer issued after its sum
// of e.  Flags are never reset (epoch + 1 is unique per parity), so no rank has
// to clear anything another rank might already have written.  Both kernels are
// gated by the engine's control block (halt | done, identical on every rank) and
// by the exchange's own error word; a timed-out wait sets that word and done = 4
// ("exchange failed"), which gates every later kernel of the fit.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "pcm_common.hpp"
#include "pcm_kmeans.h"
#include "pcm_xchg.hpp"

namespace pcm_xc {

constexpr int MAXP = PCM_XCHG_MAXP;
constexpr long long FLAG_WORDS = 512;        // 2 x 16 flags, padded to 4 KB: the slots start page-aligned
constexpr int PUSH_TPB = 1024;
constexpr int SUM_TPB = 256;
constexpr int SUM_WORDS = 2;                 // words per thread of k_xsum
constexpr int PUSH_VEC = 8;                  // 8-B words per thread per batch of k_xpush (8192 per batch)

// Exchange state words, in the fine-grained buffer's header beside the flags (one
// 128-B line each) and only touched by system-scope atomics: no L1/L2/scalar
// cache ever holds them, so every block of every later kernel reads the value
// the last writer left (a cached epoch line could hand an early block of the
// next k_xsum the previous parity).
constexpr long long EPOCH_W = 64;            // exchanges completed (identical on every rank)
constexpr long long ARRIVE_W = 80;           // k_xsum's block arrivals
constexpr long long ERR_W = 96;              // 1: a wait timed out (gates every later exchange)
constexpr long long ZERO_W = 112;            // two zero words: the gate of an exchange without an engine

__device__ __forceinline__ unsigned long long ld_sys(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct XArgs {
    unsigned long long *peer[MAXP];          // receive buffers of every rank (peer[rank] = own)
    int P, rank;
    long long Ws;                            // words per slot (>= W, 32-word multiple)
    long long W;                             // words exchanged
    unsigned long long timeout;              // s_memrealtime ticks (100 MHz)
    unsigned int *gate;                      // engine Ctrl {halt, done}, else the zero word ZERO_W
    int engine;                              // gate is an engine's control block
    int acq;                                 // system-scope acquire between the flag poll and the slot loads (A/B)
};

__device__ __forceinline__ unsigned long long *slot(const XArgs &a, unsigned long long *base, unsigned par, int s) {
    return base + FLAG_WORDS + ((long long)par * a.P + s) * a.Ws;
}

// One block per peer (blockIdx.x = 0 .. P - 2): destination (rank + 1 + b) % P.
// The control words (engine gate, error word, epoch) and the first batch of the
// statistics are all in flight before any of them is waited for: nothing
// branches on the gate before the first stores (a gated push writes its batch
// into the own buffer's never-read slot [par][rank] instead), so hipcc cannot
// sink the statistics loads behind the control words' latency.  WT: 8-B
// system-scope (sc0 sc1) write-through stores; once every storing wave has
// drained them (vmcnt(0)) and met the others at the barrier, one lane raises the
// flag -- no release fence (MI355X_MICROARCH.md "Valid forms", producer, the
// sc1-stores form).  !WT: plain stores + a system release fence (A/B).
template <bool WT, int TPB, int VEC>
__device__ __forceinline__ void push_body(const unsigned long long *__restrict__ src, const XArgs &a, int blk) {
    unsigned long long *mine = a.peer[a.rank];
    const int tid = threadIdx.x;
    const long long last = a.W - 1;
    unsigned long long v[VEC];
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
        const long long i = (long long)tid + (long long)u * TPB;
        v[u] = src[i < last ? i : last];
    }
    const unsigned gate = a.gate[0] | a.gate[1];
    const unsigned long long err = ld_sys(mine + ERR_W);
    const unsigned long long e = ld_sys(mine + EPOCH_W);
    const bool go = (gate | (unsigned)err) == 0u;
    const unsigned par = (unsigned)(e & 1ull);
    const int dst = (a.rank + 1 + blk) % a.P;
    unsigned long long *base = a.peer[dst];
    unsigned long long *out = go ? slot(a, base, par, a.rank) : slot(a, mine, par, a.rank);
    for (long long b = 0;;) {
#pragma unroll
        for (int u = 0; u < VEC; ++u) {
            const long long i = b + tid + (long long)u * TPB;
            if (i < a.W) {
                if constexpr (WT) st_sys(out + i, v[u]);
                else out[i] = v[u];
            }
        }
        b += (long long)VEC * TPB;
        if (b >= a.W) break;
#pragma unroll
        for (int u = 0; u < VEC; ++u) {
            const long long i = b + tid + (long long)u * TPB;
            v[u] = src[i < last ? i : last];
        }
    }
    if (!go) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        if constexpr (!WT) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        st_sys(base + (long long)par * MAXP + a.rank, e + 1ull);
    }
}

// Wait for the P - 1 peers' flags of this exchange, then buf[i] += every peer slot
// (NP = P rounded up to a power of two).  Wave 0 loads the gate, the error word,
// the epoch and the flags of BOTH parities in one round trip (lane s: sender s),
// then polls only if a flag is not there yet; the other waves wait at the
// barrier.  The slot loads are 8-B system-scope loads of words the producers
// stored write-through, issued after the barrier that follows the matched poll
// (the consumer's sc1-loads form: no acquire fence; a.acq = 1 adds one, A/B).
template <int NP, int TPB>
__device__ __forceinline__ void sum_body(unsigned long long *__restrict__ buf, const XArgs &a, int blk, int nblk) {
    __shared__ int s_state;                  // 0 go, 1 gated, 2 timed out
    __shared__ unsigned long long s_e;
    unsigned long long *mine = a.peer[a.rank];
    const int tid = threadIdx.x, lane = tid & 63;
    // the own statistics (the previous kernel's) load while wave 0 polls
    const long long i0 = ((long long)blk * TPB + tid) * SUM_WORDS;
    long long ix[SUM_WORDS];
#pragma unroll
    for (int w = 0; w < SUM_WORDS; ++w) ix[w] = i0 + w < a.W ? i0 + w : a.W - 1;
    unsigned long long acc[SUM_WORDS], v[NP][SUM_WORDS];
#pragma unroll
    for (int w = 0; w < SUM_WORDS; ++w) acc[w] = buf[ix[w]];
    if (tid < 64) {
        const unsigned gate = a.gate[0] | a.gate[1];
        const unsigned long long err = ld_sys(mine + ERR_W);
        const unsigned long long e = ld_sys(mine + EPOCH_W);
        const bool mine_lane = lane < a.P && lane != a.rank;
        const int fl = mine_lane ? lane : a.rank;            // the own flag is never written: 0
        const unsigned long long f0 = ld_sys(mine + fl), f1 = ld_sys(mine + MAXP + fl);
        int state = (gate | (unsigned)err) ? 1 : 0;
        if (state == 0 && mine_lane) {
            const unsigned par = (unsigned)(e & 1ull);
            unsigned long long f = par ? f1 : f0;
            if (f != e + 1ull) {
                const unsigned long long *fp = mine + (long long)par * MAXP + lane;
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                do {
                    __builtin_amdgcn_s_sleep(2);
                    if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
                        state = 2;
                        break;
                    }
                    f = ld_sys(fp);
                } while (f != e + 1ull);
            }
        }
        const bool gated = __any(state == 1), fail = __any(state == 2);
        if (lane == 0) {
            s_state = gated ? 1 : (fail ? 2 : 0);
            s_e = e;
        }
    }
    __syncthreads();
    const int state = s_state;
    if (state) {
        if (state == 2 && tid == 0) {
            st_sys(mine + ERR_W, 1ull);
            if (a.engine) a.gate[1] = 4u;   // plain store: later kernels read the control block plainly
        }
        return;
    }
    const unsigned long long e = s_e;
    const unsigned par = (unsigned)(e & 1ull);
    if (a.acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    // branch-free loads, all in flight at once: NP slots per word (slots past P and
    // the own index read slot [par][rank] of the own buffer, which nobody writes: 0)
#pragma unroll
    for (int s = 0; s < NP; ++s) {
        const unsigned long long *sl = slot(a, mine, par, (s < a.P && s != a.rank) ? s : a.rank);
#pragma unroll
        for (int w = 0; w < SUM_WORDS; ++w)
            v[s][w] = ld_sys(sl + ix[w]);
    }
#pragma unroll
    for (int s = 0; s < NP; ++s)
#pragma unroll
        for (int w = 0; w < SUM_WORDS; ++w) acc[w] += v[s][w];
#pragma unroll
    for (int w = 0; w < SUM_WORDS; ++w)
        if (i0 + w < a.W) buf[i0 + w] = acc[w];
    // the last block to finish advances the epoch (every block has read it by then)
    __syncthreads();
    if (tid == 0) {
        const unsigned long long old =
            __hip_atomic_fetch_add(mine + ARRIVE_W, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (old == (unsigned long long)nblk - 1ull) {
            st_sys(mine + ARRIVE_W, 0ull);
            st_sys(mine + EPOCH_W, e + 1ull);
        }
    }
}

// Push and sum stay two launches: in one launch the summing blocks would
// overwrite the statistics while this rank's pushing blocks may still be
// reading them (a 3-rank self-test caught exactly that, round 6).
template <bool WT>
__global__ __launch_bounds__(PUSH_TPB) void k_xpush(const unsigned long long *__restrict__ src, XArgs a) {
    push_body<WT, PUSH_TPB, PUSH_VEC>(src, a, (int)blockIdx.x);
}

template <int NP>
__global__ __launch_bounds__(SUM_TPB) void k_xsum(unsigned long long *__restrict__ buf, XArgs a) {
    sum_body<NP, SUM_TPB>(buf, a, (int)blockIdx.x, (int)gridDim.x);
}

}  // namespace pcm_xc

using namespace pcm_xc;

struct pcm_xchg {
    int device = 0, P = 1, rank = 0;
    long long W = 0, Ws = 0;
    size_t bytes = 0;
    unsigned long long *buf = nullptr;       // own receive buffer (fine-grained)
    void *opened[MAXP] = {};                 // hipIpcOpenMemHandle mappings (closed at destroy)
    unsigned long long *peer[MAXP] = {};
    unsigned long long timeout = 0;
};

#define XCHK(expr)                                                                                       \
    do {                                                                                                 \
        hipError_t _e = (expr);                                                                          \
        if (_e != hipSuccess)                                                                            \
            return pcm_fail(PCM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));             \
    } while (0)

namespace {
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(d);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};
}  // namespace

int pcm_xchg_create(int device, int64_t words, int nranks, int rank, double timeout_s, pcm_xchg **out) {
    if (!out || words < 1 || nranks < 1 || nranks > MAXP || rank < 0 || rank >= nranks || !(timeout_s > 0.0))
        return pcm_fail(PCM_E_ARG, "pcm_xchg_create: bad argument");
    *out = nullptr;
    DeviceGuard g(device);
    pcm_xchg *x = new pcm_xchg();
    x->device = device;
    x->P = nranks;
    x->rank = rank;
    x->W = words;
    x->Ws = (words + 31) / 32 * 32;
    x->timeout = (unsigned long long)(timeout_s * 1e8);
    x->bytes = (size_t)(FLAG_WORDS + 2ll * nranks * x->Ws) * sizeof(unsigned long long);
    // fine-grained device memory (coherent for system-scope accesses of other
    // agents).  PCM_XCHG_ALLOC (A/B only): 0 uncached, 2 plain hipMalloc.  Measured
    // (tools/xchg_alloc_ab.sh, profiles/rd6_xchg_alloc_ab.txt): the uncached
    // allocation returned stale slot words once the buffers of earlier exchanges
    // had been freed and reallocated; fine-grained and plain memory gave exact sums.
    const char *am = std::getenv("PCM_XCHG_ALLOC");
    const int amode = am ? std::atoi(am) : 1;
    hipError_t e = amode == 2 ? hipMalloc((void **)&x->buf, x->bytes)
                              : hipExtMallocWithFlags((void **)&x->buf, x->bytes,
                                                      amode == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached);
    if (e == hipSuccess) e = hipMemset(x->buf, 0, x->bytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();   // zeroed before any peer can learn the handle
    if (e != hipSuccess) {
        if (x->buf) (void)hipFree(x->buf);
        delete x;
        return pcm_fail(PCM_E_HIP, std::string("pcm_xchg_create: ") + hipGetErrorString(e));
    }
    x->peer[rank] = x->buf;
    *out = x;
    return 0;
}

int pcm_xchg_destroy(pcm_xchg *x) {
    if (!x) return 0;
    DeviceGuard g(x->device);
    (void)hipDeviceSynchronize();
    for (int r = 0; r < MAXP; ++r)
        if (x->opened[r]) (void)hipIpcCloseMemHandle(x->opened[r]);
    if (x->buf) (void)hipFree(x->buf);
    delete x;
    return 0;
}

int pcm_xchg_handle(pcm_xchg *x, void *handle) {
    if (!x || !handle) return pcm_fail(PCM_E_ARG, "pcm_xchg_handle: bad argument");
    DeviceGuard g(x->device);
    hipIpcMemHandle_t h;
    XCHK(hipIpcGetMemHandle(&h, x->buf));
    static_assert(sizeof(h) == PCM_XCHG_HANDLE_BYTES, "IPC handle size");
    __builtin_memcpy(handle, &h, sizeof(h));
    return 0;
}

int pcm_xchg_open(pcm_xchg *x, int peer, const void *handle) {
    if (!x || !handle || peer < 0 || peer >= x->P || peer == x->rank)
        return pcm_fail(PCM_E_ARG, "pcm_xchg_open: bad argument");
    if (x->opened[peer]) return pcm_fail(PCM_E_STATE, "pcm_xchg_open: peer already linked");
    DeviceGuard g(x->device);
    hipIpcMemHandle_t h;
    __builtin_memcpy(&h, handle, sizeof(h));
    void *p = nullptr;
    XCHK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    x->opened[peer] = p;
    x->peer[peer] = (unsigned long long *)p;
    return 0;
}

int pcm_xchg_link(pcm_xchg *x, int peer, pcm_xchg *other) {
    if (!x || !other || peer < 0 || peer >= x->P || peer == x->rank || other->rank != peer || other->P != x->P ||
        other->W != x->W)
        return pcm_fail(PCM_E_ARG, "pcm_xchg_link: bad argument");
    x->peer[peer] = other->buf;
    return 0;
}

int pcm_xchg_launch(pcm_xchg *x, unsigned long long *buf, unsigned int *gate, int phase, hipStream_t s) {
    if (!x || !buf || phase < 1 || phase > 3) return pcm_fail(PCM_E_ARG, "pcm_xchg: bad argument");
    if (x->P == 1) return 0;
    XArgs a{};
    for (int r = 0; r < x->P; ++r) {
        if (!x->peer[r]) return pcm_fail(PCM_E_STATE, "pcm_xchg: a peer buffer is not linked");
        a.peer[r] = x->peer[r];
    }
    a.P = x->P;
    a.rank = x->rank;
    a.Ws = x->Ws;
    a.W = x->W;
    a.timeout = x->timeout;
    a.gate = gate ? gate : (unsigned int *)(x->buf + ZERO_W);
    a.engine = gate != nullptr;
    // write-through slot stores + system-scope slot loads need no fences
    // (PCM_XCHG_WT=0: plain stores + a release fence; PCM_XCHG_ACQ=1: an acquire
    // fence before the slot loads -- A/B, profiles/rd6_xchg_*)
    static const int wt = [] { const char *v = std::getenv("PCM_XCHG_WT"); return v ? std::atoi(v) : 1; }();
    static const int acq = [] { const char *v = std::getenv("PCM_XCHG_ACQ"); return v ? std::atoi(v) : 0; }();
    a.acq = acq || !wt;
    if (phase & 1) {
        if (wt) k_xpush<true><<<x->P - 1, PUSH_TPB, 0, s>>>(buf, a);
        else k_xpush<false><<<x->P - 1, PUSH_TPB, 0, s>>>(buf, a);
        XCHK(hipGetLastError());
    }
    if (phase & 2) {
        const long long per = (long long)SUM_TPB * SUM_WORDS;
        const int grid = (int)((x->W + per - 1) / per);
        if (x->P <= 2) k_xsum<2><<<grid, SUM_TPB, 0, s>>>(buf, a);
        else if (x->P <= 4) k_xsum<4><<<grid, SUM_TPB, 0, s>>>(buf, a);
        else if (x->P <= 8) k_xsum<8><<<grid, SUM_TPB, 0, s>>>(buf, a);
        else k_xsum<16><<<grid, SUM_TPB, 0, s>>>(buf, a);
        XCHK(hipGetLastError());
    }
    return 0;
}

int pcm_xchg_allreduce(pcm_xchg *x, uint64_t *buf, int phase, void *stream) {
    return pcm_xchg_launch(x, (unsigned long long *)buf, nullptr, phase, (hipStream_t)stream);
}

int pcm_xchg_status(pcm_xchg *x, uint32_t *err, uint64_t *epoch, void *stream) {
    if (!x) return pcm_fail(PCM_E_ARG, "pcm_xchg_status: bad argument");
    unsigned long long h[ERR_W + 1] = {};
    hipStream_t s = (hipStream_t)stream;
    XCHK(hipMemcpyAsync(h, x->buf, sizeof(h), hipMemcpyDeviceToHost, s));
    XCHK(hipStreamSynchronize(s));
    if (err) *err = (uint32_t)h[ERR_W];
    if (epoch) *epoch = h[EPOCH_W];
    return 0;
}
