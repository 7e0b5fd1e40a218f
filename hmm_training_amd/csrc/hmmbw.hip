// hmmbw.hip — MI355X (gfx950, CDNA4) Baum-Welch engine behind the C ABI in include/hmmbw.h.
//
// Replaces the hot path of DemianMArin/HMM_Training HMM/hmm_training.py:265-541 (hmm_training):
//   E-step  :351-410  forward alpha / backward beta (calculate_log_alpha :122-160,
//                     calculate_log_beta :163-199), gamma, xi
//   M-step  :415-500  pi, A, B re-estimation (incl. the 1e-20 floor at :497)
//   converge:503-514  L = LSE_r log P_r, diff, stop rule of :346
//   finalise:524-541  safe_exp + normalisation
// and the forward-only scorer of HMM/hmm_testing.py:49-104.
//
// Numerics.  The reference works in the log domain.  Here every recursion is
// fp64 *scaled linear*: alpha_t is renormalised by an exact power of two 2^-e_t (frexp/ldexp, no
// rounding), log P = log(sum alpha_hat_{T-1}) + ln2 * sum_t e_t, beta_hat shares the same scale
// factors (Rabiner scaling with c_t = 2^e_t), so gamma_t = alpha_hat_t * beta_hat_t and
// xi_t(i,j) = a_ij * alpha_hat_t(i) * v_{t+1}(j) with v = b(o_{t+1}) * beta_hat_{t+1} * 2^-e_{t+1}.
// The reference's "-inf term dropped" rules are exactly "zero term adds nothing" here.
//
// Kernel map:
//   k_estep_small<N,G,LR,LDSTAB,FWD_ONLY>  N <= 16: a sequence is a group of G = pow2ceil(N) lanes,
//        lane j = state j, 64/G sequences per wavefront.  Cross-lane exchange by DPP (quad_perm,
//        row_shr/shl, row_half_mirror, row_mirror, row_newbcast); B^T and the B-numerator histogram
//        in LDS; the forward sweep stores one alpha_hat checkpoint per 8-step chunk plus the int16
//        scale exponents, the backward sweep recomputes each chunk's alpha_hat in registers
//        (bit-identical) and fuses beta, gamma, xi and the histogram scatter.
//   k_estep_wide<NP,FWD_ONLY>              16 < N <= 64: one sequence per wavefront, lane = state,
//        A / A^T in LDS, alpha / v exchanged through a per-wave LDS row.
//   k_reduce_local  (multi-rank) sum the statistics copies into the all-reduce buffer + the rank's
//                   (max, sum exp) pair of log P_r.
//   k_mstep / k_mstep_staged  one workgroup: L, M-step, convergence record, zero the statistics
//                   (staged: all statistics gathered into LDS with one batch of loads).
//   k_mstep_grid    large N x K (wide path): B re-estimated by the whole grid, the rest by workgroup 0.
//   k_finalise  the reference's return-path normalisation (:524-541).
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <rccl/rccl.h>

#include "hmmbw_device.hpp"
#include "hmmbw_kernels.hpp"

namespace hmmbw {

// Multi-rank: sum this rank's statistics copies into the caller's buffer (for the all-reduce),
// zero the copies, and write the rank's (max, sum exp) pair of log P into its slot.
__global__ void __launch_bounds__(256) k_reduce_local(double *copies, int ncopies, long long copy_len,
                                                      const double *llpart, long long nblocks, double *stats,
                                                      long long off_ll, int world, int rank,
                                                      const IterState *state) {
    __shared__ double sh[16];
    if (state->done) return;
    for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < copy_len;
         idx += (long long)gridDim.x * blockDim.x) {
        double v = 0.0;
        for (int c = 0; c < ncopies; ++c) {
            v += copies[c * copy_len + idx];
            copies[c * copy_len + idx] = 0.0;
        }
        stats[idx] = v;
    }
    if (blockIdx.x == 0) {
        double m, s;
        combine_ll_pairs(llpart, nblocks, sh, &m, &s);
        if (threadIdx.x < 2 * world) stats[off_ll + threadIdx.x] = 0.0;
        __syncthreads();
        if (threadIdx.x == 0) {
            stats[off_ll + 2 * rank] = (s > 0.0) ? m : 0.0;
            stats[off_ll + 2 * rank + 1] = s;
        }
    }
}

// Deterministic mode: sum the per-workgroup partial statistics [blocks][n] in workgroup order.
__global__ void __launch_bounds__(256) k_det_reduce(const double *part, long long nblocks, long long n, double *out,
                                                    const IterState *state) {
    if (state->done) return;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        double v = 0.0;
        for (long long b = 0; b < nblocks; ++b) v += part[b * n + i];
        out[i] = v;
    }
}

__global__ void __launch_bounds__(256) k_mstep(MArgs m) {
    if (carry_if_done(m)) return;
    mstep_block<false>(m);
}

__global__ void __launch_bounds__(256) k_mstep_grid(MArgs m) {
    if (carry_if_done(m)) return;
    mstep_grid(m);
}

// single-rank M-step with the statistics staged in dynamic LDS (copy_len doubles)
__global__ void __launch_bounds__(256) k_mstep_staged(MArgs m) {
    extern __shared__ double sSt[];
    if (carry_if_done(m)) return;
    mstep_staged<false>(m, sSt);
}

// Status snapshot for hmmbw_status_post: the state record and the iteration records [first, iteration)
// written straight into pinned host memory (one small launch on the stream instead of DMA copies).
__global__ void __launch_bounds__(256) k_snapshot(const IterState *st, const double *hist, long long first,
                                                   IterState *hst, double *hrec) {
    const IterState s = *st;
    const long long n = min(max(s.iteration - first, 0LL), (long long)kHist);
    for (long long i = threadIdx.x; i < n; i += blockDim.x) {
        const long long k = (first + i) % kHist;
        hrec[2 * i] = hist[2 * k];
        hrec[2 * i + 1] = hist[2 * k + 1];
    }
    if (threadIdx.x == 0) *hst = s;
}

// safe_exp + normalisation of the returned parameters (:524-541)
__global__ void k_finalise(const double *pi, const double *A, const double *B, int N, int K, double *out) {
    double *opi = out, *oA = out + N, *oB = out + N + N * N;
    const int tid = threadIdx.x;
    if (tid == 0) {
        double s = 0.0;
        for (int i = 0; i < N; ++i) s += pi[i];
        for (int i = 0; i < N; ++i) opi[i] = pi[i] / s;
    }
    for (int i = tid; i < N; i += blockDim.x) {
        double s = 0.0;
        for (int k = 0; k < N; ++k) s += A[i * N + k];
        for (int k = 0; k < N; ++k) oA[i * N + k] = s > 0.0 ? A[i * N + k] / s : A[i * N + k];
        double sb = 0.0;
        for (int k = 0; k < K; ++k) sb += B[(long long)i * K + k];
        for (int k = 0; k < K; ++k) oB[(long long)i * K + k] = sb > 0.0 ? B[(long long)i * K + k] / sb : B[(long long)i * K + k];
    }
}

// ---------------------------------------------------------------------------------------------
// Peer all-reduce (HMMBW_OPT_ALLREDUCE = 1; include/hmmbw.h).  The reference's sums over all recordings
// (hmm_training.py:415-424 pi over the global R, :429-500 A and B, :503 L) become ONE elementwise sum of
// the ranks' statistics buffers per EM iteration.  Every rank owns a receive region in its HBM:
//   [2 iteration parities][world slots][slot doubles], then flags [world][chunks] (uint64 sequence numbers)
// The buffer is cut into chunks of kPeerThreads x dpt doubles (dpt chosen so a payload has <= 32 chunks).
//   push   workgroup (chunk c, peer p) writes chunk c of this rank's buffer into slot `rank` of p's region
//          with system-scope write-through stores, waits for them (vmcnt(0) in every wave, then the
//          barrier) and release-stores the iteration's sequence number into p's flag (rank, c);
//   reduce workgroup c's first wave polls its region's W flags of chunk c (system-scope loads + s_sleep,
//          bounded by wall-clock ticks: on expiry the iteration state records HMMBW_E_TIMEOUT and stops
//          EM), then the workgroup sums the W slots in rank order into the buffer, so every rank holds
//          bitwise-identical sums.
// k_peer_allreduce does both in ONE launch (hmmbw_iterate's loop: one kernel boundary, as RCCL's);
// the split ABI runs them as k_peer_push (in _begin) and k_peer_reduce (in _end), so several ranks that
// share one stream (the in-process tests) never wait on a push queued behind them.
// Parity double-buffering is enough: a rank can push iteration e + 2 into p's slot only after its own
// reduce of e + 1, which needs p's push of e + 1, which p enqueues after its reduce of e.
// ---------------------------------------------------------------------------------------------
constexpr int kMaxPeers = 16;
constexpr int kPeerThreads = 256;
constexpr int kPeerMaxChunks = 32;

struct PeerArgs {
    double *region[kMaxPeers];  // every rank's receive region, as addressable from this device
    long long n;                // payload doubles
    long long slot;             // slot stride (n rounded up to 256 B)
    long long nch;              // chunks
    int dpt;                    // doubles per thread per chunk (chunk = kPeerThreads x dpt)
    int world, rank;
    double perturb;             // diagnostics (HMMBW_DIAG_PEER_PERTURB): element 0 of this rank's push x (1 + perturb)
};

__device__ __forceinline__ unsigned long long *peer_flags(double *region, const PeerArgs &P) {
    return reinterpret_cast<unsigned long long *>(region + 2LL * P.world * P.slot);
}

__device__ __forceinline__ void peer_push_chunk(const double *src, const PeerArgs &P, unsigned long long seq,
                                                long long c, int p) {
    const long long base = c * kPeerThreads * P.dpt + threadIdx.x;
    double *dst = P.region[p] + ((long long)(seq & 1) * P.world + P.rank) * P.slot;
    for (int k = 0; k < P.dpt; ++k) {
        const long long i = base + (long long)k * kPeerThreads;
        if (i < P.n) __hip_atomic_store(dst + i, i == 0 ? src[i] * (1.0 + P.perturb) : src[i], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's write-through stores are acknowledged
    __syncthreads();
    // The flag is a write-through store too, issued after every payload store of the workgroup was
    // acknowledged: that orders it after them.  A release would add an L2 write-back at system scope
    // (every dirty line of this XCD, e.g. the E-step's checkpoints), which the payload does not need.
    if (threadIdx.x == 0)
        __hip_atomic_store(peer_flags(P.region[p], P) + (long long)P.rank * P.nch + c, seq, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// returns false (and stops EM with HMMBW_E_TIMEOUT) when a flag did not arrive in time
__device__ __forceinline__ bool peer_reduce_chunk(double *dst, const PeerArgs &P, unsigned long long seq,
                                                  IterState *state, long long timeout_ticks, long long c) {
    __shared__ int ok;
    const int tid = threadIdx.x;
    double *reg = P.region[P.rank];
    if (tid < 64) {  // one wave polls: lane q watches rank q's flag of this chunk
        const unsigned long long *fl = peer_flags(reg, P) + c;
        bool got = tid >= P.world;
        const unsigned long long t0 = wall_clock64();
        while (true) {
            if (!got) got = __hip_atomic_load(fl + (long long)tid * P.nch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= seq;
            if (__all(got)) break;
            if ((long long)(wall_clock64() - t0) > timeout_ticks) break;
            __builtin_amdgcn_s_sleep(2);
        }
        const int all = __all(got);
        if (tid == 0) ok = all;
    }
    __syncthreads();
    if (!ok) {
        if (tid == 0) {
            state->error = HMMBW_E_TIMEOUT;
            state->error_src = kErrPeer;
            state->done = 1;
        }
        return false;
    }
    // no acquire fence (it would invalidate this XCD's L2): the slot loads below are system-scope loads,
    // which bypass the caches and are issued after the flags were seen
    const double *slots = reg + (long long)(seq & 1) * P.world * P.slot;
    const long long base = c * kPeerThreads * P.dpt + tid;
    for (int k = 0; k < P.dpt; ++k) {
        const long long i = base + (long long)k * kPeerThreads;
        if (i < P.n) {
            double v = 0.0;
            for (int q = 0; q < P.world; ++q)
                v += __hip_atomic_load(slots + q * P.slot + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            dst[i] = v;
        }
    }
    return true;
}

__global__ void __launch_bounds__(kPeerThreads) k_peer_push(const double *src, PeerArgs P, unsigned long long seq,
                                                            const IterState *state) {
    if (state->done) return;  // identical on every rank: no rank pushes, none waits
    peer_push_chunk(src, P, seq, blockIdx.x, blockIdx.y);
}

__global__ void __launch_bounds__(kPeerThreads) k_peer_reduce(double *dst, PeerArgs P, unsigned long long seq,
                                                              IterState *state, long long timeout_ticks) {
    if (state->done) return;
    (void)peer_reduce_chunk(dst, P, seq, state, timeout_ticks, blockIdx.x);
}

// push + wait + sum in one launch: workgroup (c, p) pushes chunk c to rank p; the one whose p is this
// rank (its own slot, the nearest memory) then waits for chunk c's W flags and sums them into `sum` (not
// into buf, which the other workgroups of this launch may still be pushing).  At most 32 x 16 workgroups
// of 256 threads, all resident at once, so a waiting workgroup never holds a slot a pushing one needs
// (and every wait is bounded anyway).
__global__ void __launch_bounds__(kPeerThreads) k_peer_allreduce(const double *buf, double *sum, PeerArgs P,
                                                                 unsigned long long seq, IterState *state,
                                                                 long long timeout_ticks) {
    if (state->done) return;
    peer_push_chunk(buf, P, seq, blockIdx.x, blockIdx.y);
    if ((int)blockIdx.y != P.rank) return;
    (void)peer_reduce_chunk(sum, P, seq, state, timeout_ticks, blockIdx.x);
}

// Validation of a new uncached / fine-grained peer region (peer_region_alloc): the pattern is written with the
// push's system-scope stores, then read back with the reduce's system-scope loads and with ordinary loads;
// every mismatch is counted.  Recycled pages can return stale data to kernel loads after a change of memory
// type (see peer_region_alloc), which this catches before the region carries any statistics.
__device__ __forceinline__ double region_pattern(long long i, unsigned seed) {
    return (double)(((unsigned long long)i * 2654435761ull + seed) & 0xFFFFFFull) + 0.5;
}
__global__ void k_region_fill(double *r, long long n, unsigned seed) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        __hip_atomic_store(r + i, region_pattern(i, seed), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_region_check(const double *r, long long n, unsigned seed, unsigned *bad) {
    unsigned nb = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const double want = region_pattern(i, seed);
        nb += __hip_atomic_load(r + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != want;
        nb += r[i] != want;
    }
    if (nb) atomicAdd(bad, nb);
}

__global__ void k_init_state(IterState *st, double eps, long long max_it) {
    st->prev_L = -INFINITY;
    st->last_L = -INFINITY;
    st->last_diff = INFINITY;
    st->epsilon = eps;
    st->iteration = 0;
    st->max_iterations = max_it;
    st->done = max_it <= 0 ? 1 : 0;
    st->converged = 0;
    st->error = 0;
    st->error_src = 0;
}

// ---------------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------------
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                            \
    do {                                                                                         \
        hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess)                                                                    \
            return fail(HMMBW_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));         \
    } while (0)

// Block cache of the small device buffers and the pinned snapshot blocks.  The drop-in API builds and
// destroys one context per hmm_training call (HMM/hmm_training.py:265-267), and hipFree /
// hipHostFree synchronise the device and return memory to the driver: a word-sized context (20
// utterances) spent about 1 ms in hmmbw_ctx_destroy, as long as its 30 EM iterations.  Blocks up to
// kCacheMaxBlock bytes are rounded up to a power of two and kept per (device, kind, size) for the next
// context, up to kCacheMaxBytes per kind and device (a word-sized context holds well under 1 MB);
// larger buffers go straight to the driver.  hmmbw_cache_trim returns every cached block.
// Reused blocks are not cleared: every buffer is initialised by its owner, as after hipMalloc.
constexpr size_t kCacheMaxBlock = size_t(4) << 20;
constexpr size_t kCacheMaxBytes = size_t(32) << 20;
struct BlockCache {
    std::mutex mu;
    std::map<std::tuple<int, int, size_t>, std::vector<void *>> free;  // (device, kind, bytes) -> blocks
    std::map<void *, std::pair<int, size_t>> size_of;                   // cached-class block -> (kind, bytes)
    std::map<std::pair<int, int>, size_t> held;                          // (device, kind) -> bytes cached
};
BlockCache &block_cache() {
    static BlockCache *bc = new BlockCache;  // never destroyed: blocks may be released at process exit
    return *bc;
}
size_t cache_class(size_t bytes) {
    size_t c = 256;
    while (c < bytes) c <<= 1;
    return c;
}
enum { kDevBlock = 0, kPinnedBlock = 1 };

// Allocation ledger (HMMBW_DEBUG_ALLOC=1, diagnostics): every driver allocation the library holds, with the
// blocks the cache has handed out; a new allocation that overlaps a held one, a block handed out twice and a
// free of an unknown block are reported on stderr.
struct Ledger {
    std::mutex mu;
    std::map<uintptr_t, std::pair<size_t, std::string>> held;  // start -> (bytes, what)
    std::map<uintptr_t, int> out;                              // cached blocks handed out
};
bool ledger_on() {
    static const bool on = std::getenv("HMMBW_DEBUG_ALLOC") && std::atoi(std::getenv("HMMBW_DEBUG_ALLOC")) != 0;
    return on;
}
Ledger &ledger() {
    static Ledger *l = new Ledger;
    return *l;
}
void ledger_add(const void *p, size_t bytes, const char *what) {
    if (!ledger_on() || !p) return;
    Ledger &L = ledger();
    std::lock_guard<std::mutex> lk(L.mu);
    const uintptr_t a = (uintptr_t)p;
    auto it = L.held.upper_bound(a);
    if (it != L.held.end() && it->first < a + bytes)
        fprintf(stderr, "HMMBW_DEBUG_ALLOC: %s [%#lx, +%zu) overlaps held %s [%#lx, +%zu)\n", what, (unsigned long)a, bytes,
                it->second.second.c_str(), (unsigned long)it->first, it->second.first);
    if (it != L.held.begin()) {
        auto jt = std::prev(it);
        if (jt->first + jt->second.first > a)
            fprintf(stderr, "HMMBW_DEBUG_ALLOC: %s [%#lx, +%zu) overlaps held %s [%#lx, +%zu)\n", what, (unsigned long)a,
                    bytes, jt->second.second.c_str(), (unsigned long)jt->first, jt->second.first);
    }
    L.held[a] = std::make_pair(bytes, std::string(what));
}
void ledger_remove(const void *p, const char *what) {
    if (!ledger_on() || !p) return;
    Ledger &L = ledger();
    std::lock_guard<std::mutex> lk(L.mu);
    if (!L.held.erase((uintptr_t)p)) fprintf(stderr, "HMMBW_DEBUG_ALLOC: %s of unknown %p\n", what, p);
}
void ledger_out(const void *p, bool take) {
    if (!ledger_on() || !p) return;
    Ledger &L = ledger();
    std::lock_guard<std::mutex> lk(L.mu);
    int &n = L.out[(uintptr_t)p];
    n += take ? 1 : -1;
    if (n > 1) fprintf(stderr, "HMMBW_DEBUG_ALLOC: cached block %p handed out twice\n", p);
    if (n < 0) fprintf(stderr, "HMMBW_DEBUG_ALLOC: cached block %p freed twice\n", p);
}

hipError_t cached_alloc(void **p, size_t bytes, int kind) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (bytes > kCacheMaxBlock) {
        const hipError_t e = kind == kDevBlock ? hipMalloc(p, bytes)
                                               : hipHostMalloc(p, bytes, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess && kind == kDevBlock) ledger_add(*p, bytes, "hipMalloc (large)");
        return e;
    }
    const size_t cls = cache_class(bytes);
    BlockCache &bc = block_cache();
    {
        std::lock_guard<std::mutex> lk(bc.mu);
        auto it = bc.free.find(std::make_tuple(dev, kind, cls));
        if (it != bc.free.end() && !it->second.empty()) {
            *p = it->second.back();
            it->second.pop_back();
            bc.held[std::make_pair(dev, kind)] -= cls;
            if (kind == kDevBlock) ledger_out(*p, true);
            return hipSuccess;
        }
    }
    const hipError_t e = kind == kDevBlock ? hipMalloc(p, cls)
                                           : hipHostMalloc(p, cls, hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> lk(bc.mu);
        bc.size_of[*p] = std::make_pair(kind, cls);
    }
    if (e == hipSuccess && kind == kDevBlock) {
        ledger_add(*p, cls, "hipMalloc (cached class)");
        ledger_out(*p, true);
    }
    return e;
}
void cached_free(void *p, int kind) {
    if (!p) return;
    int dev = 0;
    (void)hipGetDevice(&dev);
    BlockCache &bc = block_cache();
    if (kind == kDevBlock && bc.size_of.count(p)) ledger_out(p, false);
    {
        std::lock_guard<std::mutex> lk(bc.mu);
        auto it = bc.size_of.find(p);
        if (it != bc.size_of.end()) {
            const size_t cls = it->second.second;
            size_t &held = bc.held[std::make_pair(dev, kind)];
            if (held + cls <= kCacheMaxBytes) {
                bc.free[std::make_tuple(dev, kind, cls)].push_back(p);
                held += cls;
                return;
            }
            bc.size_of.erase(it);
        }
    }
    if (kind == kDevBlock) {
        ledger_remove(p, "hipFree");
        (void)hipFree(p);
    } else {
        (void)hipHostFree(p);
    }
}
// Release every cached block (all devices); returns the bytes given back to the driver.
size_t cache_trim() {
    BlockCache &bc = block_cache();
    std::vector<std::tuple<int, int, void *>> out;
    size_t bytes = 0;
    {
        std::lock_guard<std::mutex> lk(bc.mu);
        for (auto &kv : bc.free) {
            for (void *p : kv.second) {
                out.emplace_back(std::get<0>(kv.first), std::get<1>(kv.first), p);
                bytes += std::get<2>(kv.first);
                bc.size_of.erase(p);
            }
        }
        bc.free.clear();
        bc.held.clear();
    }
    int dev0 = 0;
    (void)hipGetDevice(&dev0);
    for (auto &t : out) {
        (void)hipSetDevice(std::get<0>(t));
        if (std::get<1>(t) == kDevBlock) {
            ledger_remove(std::get<2>(t), "hipFree (trim)");
            (void)hipFree(std::get<2>(t));
        } else {
            (void)hipHostFree(std::get<2>(t));
        }
    }
    (void)hipSetDevice(dev0);
    return bytes;
}

template <class T>
int dalloc(T **p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    HIP_TRY(cached_alloc(reinterpret_cast<void **>(p), n * sizeof(T), kDevBlock));
    return HMMBW_OK;
}

template <class T>
void dfree(T *&p) {
    cached_free(p, kDevBlock);
    p = nullptr;
}

// E-step kernel pointers live in the instantiation units (hmmbw_kernels.hpp)
template <bool LR, bool LDSTAB>
Kernels pick_small_n(int N) {
    switch (N) {
#define CASE(n) \
    case n: return small_kernels_n<n>(LR, LDSTAB);
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
        CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
        default: return Kernels{};
    }
}

}  // namespace hmmbw

using namespace hmmbw;

struct hmmbw_ctx {
    int device = 0, N = 0, K = 0, G = 0, U = 0;
    bool wide = false;
    int NP = 0;
    int topo_req = HMMBW_TOPOLOGY_AUTO, topo = HMMBW_TOPOLOGY_DENSE;
    int rank = 0, world = 1;
    hipStream_t stream = nullptr;
    // parameters (linear, working copy)
    double *d_pi = nullptr, *d_A = nullptr, *d_B = nullptr, *d_Bt = nullptr, *d_out = nullptr;
    std::vector<double> h_A;
    bool has_params = false;
    // training state
    IterState *d_state = nullptr;  // [2]: the current slot is scur; every M-step writes the other
    int scur = 0;
    double *d_hist = nullptr;
    // hmmbw_status_post / _wait: two pinned snapshots (state + record ring) taken on the stream
    struct Snap {
        hipEvent_t ev = nullptr;
        IterState *st = nullptr;
        double *hist = nullptr;  // records [first, st->iteration)
        long long first = 0;
        long long ticket = -1;
    } snaps[2];
    long long snap_next = 0;
    // HMMBW_OPT_LIVE_STATUS: the host mirror every recording M-step writes (hmmbw_status_live_wait)
    LiveBlock *h_live = nullptr;
    unsigned live_epoch = 1;
    double *d_copies = nullptr;   // [3][ncopies][copy_len] E-step accumulators (iteration e uses e % 3)
    int ncopies = 2;              // HMMBW_OPT_STAT_COPIES default: halves the flush atomics per address (measured -3 %)
    bool merge_mstep = true;      // run each M-step in the prologue of the next E-step launch
    bool det = false;             // HMMBW_OPT_DETERMINISTIC: no floating-point atomics (LDS-table or wide kernels)
    double *d_part = nullptr;     // det: per-workgroup partial statistics [blocks][off_bnum]
    bool armed = false;
    long long e_count = 0;        // E-step launches since the statistics were last cleared
    // an M-step whose statistics are ready but which has not run yet (it runs in the next merged
    // E-step launch, or on its own in flush_mstep before anything reads parameters or state)
    struct Pending {
        bool on = false;
        bool local = true;        // statistics are this context's copies (single rank)
        const double *src = nullptr;
        int nsrc = 1;
        const double *ll = nullptr;  // (max, sum exp) pairs of log P
        long long nll = 0;
        double *ext = nullptr;    // multi-rank: the caller's all-reduced buffer
        long long R = 0;
    } pend;
    // observations
    long long R = 0, nwaves = 0;
    long long nblocks = 0;
    long long nfull = 0;          // small kernels: workgroups with 4 active waves (then xact-wave ones)
    int xact = 4;
    int prio = -1;                // wave priority of the small kernels (EArgs::prio): -1 auto (left-to-right 2,
                                  // dense 0: profiles/r5/spread_knobs.txt); HMMBW_PRIO overrides it
    int split_extra = 1;          // EArgs::split_extra (HMMBW_SPLIT_EXTRA=0 turns it off)
    int join = 1;                 // left-to-right E-step on the joined spread map (k_estep_join; HMMBW_JOIN=0 off)
    int join_dense = 1;           // the dense E-step on it too (HMMBW_JOIN_DENSE=0 off)
    bool fits_cus = false;        // the launch map's workgroups fit one per CU (set_observations)
    long long last_nll = 0;       // per-workgroup log-likelihood pairs written by the last E-step launch
    uint16_t *d_sym = nullptr;
    long long *d_wsym = nullptr, *d_wckoff = nullptr, *d_wspoff = nullptr;
    int *d_wT = nullptr, *d_wfull = nullptr, *d_slen = nullptr, *d_sseq = nullptr;
    double *d_ck = nullptr, *d_logp = nullptr, *d_llpart = nullptr;  // llpart: [2][nblocks][2]
    long long cktot = 0;          // checkpoint doubles of the layout
    double *d_zf = nullptr;       // dense small kernels: every z_t, kChunk x cktot (allocated on first use)
    // wide path: gamma rows per position and the symbol -> rows index of k_bnum_gather
    double *d_gam = nullptr;
    long long *d_bptr = nullptr;
    unsigned *d_brows = nullptr;
    unsigned *d_wq = nullptr;  // wide work queue (EArgs::wq): 2 counters + a flag per tile, or nullptr
    long long wq_grid = 0;     // its grid (a workgroup per unit: 2 x tiles)
    int wq_mode = -1;          // HMMBW_OPT_WIDE_WQ: -1 auto (from 4 tiles per CU), 0 off, 1 on (more tiles than CUs)
    long long wq_timeout_ms = 10000;  // HMMBW_OPT_WQ_TIMEOUT_MS: bound of a backward unit's wait
    uint4 *d_sp = nullptr;
    int *d_ebuf = nullptr;
    // native RCCL communicator (hmmbw_comm_init): the multi-rank hmmbw_iterate all-reduces d_ext
    ncclComm_t comm = nullptr;
    double *d_ext = nullptr;      // non-fused multi-rank paths: the packed statistics to all-reduce
    long long ext_len = 0;
    // hmmbw_iterate_begin / _end: one multi-rank iteration split at its all-reduce (the same enqueue
    // sequence hmmbw_iterate runs around ncclAllReduce); open between the two calls
    bool ar_open = false;
    bool ar_fused = false;
    double *ar_cur = nullptr;
    long long ar_R = 0;
    // fused native path (small kernels): the E-step accumulates straight into a triple-buffered
    // all-reduce buffer [3][xlen] = {ncopies statistics copies, (max, sum exp) per rank}; the last
    // workgroup of each launch writes the rank's pair (d_ctr: completion counter)
    double *d_xbuf = nullptr;
    // peer all-reduce (HMMBW_OPT_ALLREDUCE = 1): this rank's receive region, every rank's region as
    // addressable here (attached), the IPC mappings to close, and the iteration sequence number
    int ar_kind = HMMBW_ALLREDUCE_RCCL;
    double *d_peer = nullptr;
    size_t peer_bytes = 0;
    long long peer_n = 0, peer_slot = 0, peer_nch = 0;
    int peer_dpt = 1;
    double *d_xsum = nullptr;     // the all-reduced sums the pending M-step reads (peer mode)
    int peer_world = 0;
    bool peer_on = false;
    bool peer_revoked = false;
    bool peer_special = false;
    double peer_perturb = 0.0;    // diagnostics: HMMBW_DIAG_PEER_PERTURB=<rank>:<value> (bench's leg check)    // the region is uncached / fine-grained (HMMBW_PEER_MEM)    // a region this context was attached to was freed by its owner
    std::vector<double *> peer_regions;
    std::vector<void *> peer_mapped;
    unsigned long long peer_seq = 0;
    long long peer_timeout_ms = 30000;
    long long wall_khz = 100000;  // hipDeviceAttributeWallClockRate (100 MHz on MI355X)
    long long ar_len_last = 0;    // doubles in the last all-reduce hmmbw_iterate enqueued
    long long xlen = 0;
    int *d_ctr = nullptr;
    // all-reduce timing (hmmbw_comm_info): event pairs around ncclAllReduce, same schedule as timing
    long long ar_seq = 0;
    std::vector<hipEvent_t> ar_free, ar_pending;
    double ar_ms = 0.0;
    long long ar_n = 0;
    long long R_global = 0;
    bool has_obs = false;
    int force_safe = 0;
    int ablate = 0;
    // timing
    int timing = 0;              // 0: off; k >= 1: time every k-th E-step launch
    long long timing_seq = 0;
    std::vector<hipEvent_t> ev_free, ev_pending;  // pairs (start, stop)
    double timed_ms = 0.0;
    long long timed_n = 0;
    // launches with a follow-up kernel (wide: k_bnum_gather): an event between the E-step kernel and
    // it, one entry per pending pair (nullptr: none), so hmmbw_timing_split can price the E-step alone
    std::vector<hipEvent_t> mid_free, mid_pending;
    double timed_main_ms = 0.0;
    long long timed_main_n = 0;

    long long off_S() const { return N; }
    long long off_gex() const { return N + (long long)N * N; }
    long long off_gall() const { return off_gex() + N; }
    long long off_bnum() const { return off_gall() + N; }
    long long off_ll() const { return off_bnum() + (long long)K * N; }
    long long stats_len() const { return off_ll() + 2LL * world; }
    long long copy_len() const { return off_ll(); }
    // emission table + B-numerator histogram in LDS ([K][G+1] fp64 each) when they fit 48 KiB
    // emission P/H tables in LDS (two [K][G + kTabPad] tables of 16-B entries kHistOff bytes apart, see
    // hmmbw_device.hpp) when the first fits below kHistOff (the row offsets then fit the uint16 packs)
    bool lds_tables() const { return !wide && lds_tables_fit(K, G + kTabPad); }
    // LDS doubles of the small kernels' tables
    size_t lds_table_doubles() const { return lds_tables() ? lds_table_bytes(K, G + kTabPad) / sizeof(double) : 0; }
    bool can_merge() const { return merge_mstep && lds_tables() && copy_len() <= kMergedMaxStats && nwaves > 0; }
    // statistics copies in the fused all-reduce buffer: the wide path's B numerator is written once (by
    // k_bnum_gather, into copy 0), and its tiles finish at different times, so its atomics need no
    // spreading: one copy, and the all-reduce carries no K x N block of zeros (cfg5: 0.56 MB, not 1.1)
    int xcopies() const { return wide ? 1 : ncopies; }
    // doubles of the per-iteration multi-rank all-reduce: the fused buffer (copies + one (max, sum exp)
    // pair per rank, 256-B aligned) or, in deterministic mode, the packed statistics
    long long ar_payload() const {
        return det ? stats_len() : ((long long)xcopies() * copy_len() + 2LL * world + 31) / 32 * 32;
    }
    bool peer_mode() const { return ar_kind == HMMBW_ALLREDUCE_PEER && peer_on; }
    IterState *state() const { return d_state + scur; }
    double *copies(long long e) const { return d_copies + (e % 3) * (long long)ncopies * copy_len(); }
    double *llpart(long long e) const { return d_llpart + (e % 2) * 2 * std::max(nblocks, 1LL); }
};

namespace {

int set_device(hmmbw_ctx *c) {
    HIP_TRY(hipSetDevice(c->device));
    return HMMBW_OK;
}

// the block cache hands a freed block to the next allocation at once (hipFree used to synchronise the
// device): the context's queued work must be done with a block before it is freed
void sync_ctx(hmmbw_ctx *c) {
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    else (void)hipDeviceSynchronize();
}

// wall-clock ticks of a bound in ms, saturated (a huge bound must not wrap to a negative count, which
// would end every wait at once)
long long ms_to_ticks(const hmmbw_ctx *c, long long ms) {
    const long long khz = std::max(1LL, c->wall_khz);
    if (ms <= 0) return 0;
    return ms > LLONG_MAX / khz ? LLONG_MAX : ms * khz;
}

// In-process attachments (hmmbw_peer_attach): region -> the contexts whose peer_regions hold it.  A context
// that frees its region detaches every context still attached to it, so a later push of theirs fails with
// HMMBW_E_STATE instead of writing into memory the allocator may already have handed to another buffer.
struct PeerLinks {
    std::mutex mu;
    std::map<const void *, std::vector<hmmbw_ctx *>> users;
};
PeerLinks &peer_links() {
    static PeerLinks *p = new PeerLinks;  // never destroyed
    return *p;
}

// drop the attached peer regions (closing the IPC mappings of other ranks' regions)
void peer_detach(hmmbw_ctx *c) {
    for (void *p : c->peer_mapped) (void)hipIpcCloseMemHandle(p);
    c->peer_mapped.clear();
    {
        PeerLinks &pl = peer_links();
        std::lock_guard<std::mutex> lk(pl.mu);
        for (double *r : c->peer_regions) {
            auto it = pl.users.find(r);
            if (it == pl.users.end()) continue;
            auto &v = it->second;
            v.erase(std::remove(v.begin(), v.end(), c), v.end());
            if (v.empty()) pl.users.erase(it);
        }
    }
    c->peer_regions.clear();
    c->peer_on = false;
}

std::string peer_off_msg(const hmmbw_ctx *c) {
    return c->peer_revoked ? "peer all-reduce: a rank's region this context was attached to has been freed "
                             "(its context was destroyed or re-sized its region); attach again"
                           : "peer all-reduce selected but no regions attached (hmmbw_peer_open / _attach)";
}

// this context's region is about to be freed: detach every other context attached to it (in-process)
void peer_revoke(hmmbw_ctx *c) {
    if (!c->d_peer) return;
    PeerLinks &pl = peer_links();
    std::lock_guard<std::mutex> lk(pl.mu);
    auto it = pl.users.find(c->d_peer);
    if (it == pl.users.end()) return;
    for (hmmbw_ctx *u : it->second) {
        if (u == c) continue;
        for (double *r : u->peer_regions) {  // u's other links go too: its exchange is broken as a whole
            if (r == c->d_peer) continue;
            auto jt = pl.users.find(r);
            if (jt == pl.users.end()) continue;
            auto &w = jt->second;
            w.erase(std::remove(w.begin(), w.end(), u), w.end());
            if (w.empty()) pl.users.erase(jt);
        }
        u->peer_regions.clear();
        u->peer_on = false;
        u->peer_revoked = true;
    }
    pl.users.erase(it);
}

void free_obs(hmmbw_ctx *c) {
    sync_ctx(c);
    dfree(c->d_sym); dfree(c->d_wsym); dfree(c->d_wckoff); dfree(c->d_wspoff);
    dfree(c->d_wT); dfree(c->d_wfull); dfree(c->d_slen); dfree(c->d_sseq);
    dfree(c->d_ck); dfree(c->d_sp); dfree(c->d_ebuf); dfree(c->d_logp); dfree(c->d_llpart); dfree(c->d_zf);
    dfree(c->d_gam); dfree(c->d_bptr); dfree(c->d_brows); dfree(c->d_part); dfree(c->d_wq);
    c->wq_grid = 0;
    c->has_obs = false;
}

int realloc_stats(hmmbw_ctx *c) {
    sync_ctx(c);
    dfree(c->d_copies);
    c->pend.on = false;
    c->e_count = 0;
    const size_t n = 3 * (size_t)c->ncopies * c->copy_len();
    if (int rc = dalloc(&c->d_copies, n)) return rc;
    HIP_TRY(hipMemsetAsync(c->d_copies, 0, sizeof(double) * n, c->stream));
    return HMMBW_OK;
}

EArgs make_eargs(hmmbw_ctx *c) {
    EArgs a{};
    a.L = Layout{c->d_sym, c->d_wsym, c->d_wckoff, c->d_wspoff, c->d_wT, c->d_wfull, c->d_slen, c->d_sseq,
                 c->nwaves};
    a.pi = c->d_pi;
    a.A = c->d_A;
    a.Bt = c->d_Bt;
    a.ckpt = c->d_ck;
    a.gam = c->d_gam;
    a.gdst = c->wide ? c->d_brows : nullptr;
    a.part = c->d_part;
    a.spack = c->d_sp;
    a.ebuf = c->d_ebuf;
    a.copies = c->copies(0);
    a.copy_len = c->copy_len();
    a.ncopies = c->ncopies;
    a.logp = c->d_logp;
    a.llpart = c->llpart(0);
    a.force_safe = c->force_safe;
    a.ablate = c->ablate;
    a.state = c->state();
    a.K = c->K;
    a.N = c->N;
    a.off_S = c->off_S();
    a.off_gex = c->off_gex();
    a.off_gall = c->off_gall();
    a.off_bnum = c->off_bnum();
    a.nfull = c->nfull;
    a.xact = c->xact;
    a.prio = c->prio >= 0 ? c->prio : (c->topo == HMMBW_TOPOLOGY_LEFT_TO_RIGHT ? 2 : 0);
    a.split_extra = c->split_extra;
    return a;
}

// M-step arguments for the pending statistics: this context's copies (single rank) or the caller's
// all-reduced buffer with one (max, sum exp) pair per rank
MArgs make_margs(hmmbw_ctx *c, const hmmbw_ctx::Pending &p) {
    MArgs m{};
    m.src = p.src;
    m.zero_ll = p.local ? nullptr : const_cast<double *>(p.ll);
    m.nsrc = p.nsrc;
    m.copy_len = c->copy_len();
    m.pi = c->d_pi;
    m.A = c->d_A;
    m.B = c->d_B;
    m.Bt = c->d_Bt;
    m.llpart = p.ll;
    m.nblocks = p.nll;
    m.R_global = p.R;
    m.state = c->state();
    m.state_out = c->d_state + (c->scur ^ 1);
    m.hist = c->d_hist;
    m.N = c->N;
    m.K = c->K;
    m.G = c->G;
    m.world = c->world;
    m.local_lse = p.local ? 1 : 0;
    m.bt_perm = c->wide ? 1 : 0;
    m.off_S = c->off_S();
    m.off_gex = c->off_gex();
    m.off_gall = c->off_gall();
    m.live = c->h_live;
    m.live_epoch = c->live_epoch;
    m.off_bnum = c->off_bnum();
    m.off_ll = c->off_ll();
    return m;
}

// run the pending M-step as its own one-workgroup kernel
int flush_mstep(hmmbw_ctx *c) {
    if (!c->pend.on) return HMMBW_OK;
    c->pend.on = false;
    if (c->ablate & 4) return HMMBW_OK;  // diagnostics (HMMBW_OPT_ABLATE bit 2): no separate M-step kernel
    const MArgs m = make_margs(c, c->pend);
    const size_t staged = sizeof(double) * (size_t)c->copy_len();
    const long long nb = (long long)c->N * c->K;
    if (m.local_lse && staged <= 64 * 1024 && c->N * c->N <= 256)
        hipLaunchKernelGGL(k_mstep_staged, dim3(1), dim3(256), staged, c->stream, m);
    else if (nb > 8192)  // large B: the whole grid re-estimates it (one workgroup took 150 us at 64 x 1024)
        hipLaunchKernelGGL(k_mstep_grid, dim3((unsigned)std::min<long long>((nb + 1023) / 1024, 256)), dim3(256), 0,
                           c->stream, m);
    else
        hipLaunchKernelGGL(k_mstep, dim3(1), dim3(256), 0, c->stream, m);
    HIP_TRY(hipGetLastError());
    c->scur ^= 1;
    return HMMBW_OK;
}

// The largest dynamic LDS each kernel has been allowed so far on each device: hipFuncSetAttribute once
// per kernel and size, not on every launch (the LR cfg3 launch asks for 66,880 B every EM iteration).
struct LdsGrants {
    std::mutex mu;
    std::map<std::pair<int, const void *>, size_t> have;
};
LdsGrants &lds_grants() {
    static LdsGrants g;
    return g;
}

int allow_lds(const void *f, size_t lds) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    LdsGrants &g = lds_grants();
    std::lock_guard<std::mutex> lk(g.mu);
    size_t &have = g.have[std::make_pair(dev, f)];
    if (have >= lds) return HMMBW_OK;
    HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    have = lds;
    return HMMBW_OK;
}

template <class F>
int launch_lds(F f, unsigned grid, size_t lds, hipStream_t stream, const EArgs &a, unsigned block = kBlock) {
    if (lds > 64 * 1024)
        if (int rc = allow_lds(reinterpret_cast<const void *>(f), lds)) return rc;
    hipLaunchKernelGGL(f, dim3(grid), dim3(block), lds, stream, a);
    HIP_TRY(hipGetLastError());
    return HMMBW_OK;
}

// One E-step / scorer launch of a context, resolved but not yet enqueued (launch_estep enqueues it
// alone, group_launch concatenates several contexts' plans into one grouped launch).
struct Plan {
    EArgs a{};
    KernelFn fn = nullptr;
    GroupFn gfn = nullptr;
    unsigned grid = 0, block = kBlock;
    size_t lds = 0;
    bool flip = false;
    long long nll = 0;  // per-workgroup log-likelihood pairs the launch writes (tiles on the wide work queue)
};

// E-step launch e accumulates into copies and llpart; it clears `zero` (zero_len doubles) and, when
// `merge` is set, first runs the pending M-step in its prologue (which consumes c->pend).
// Dense small kernels store every z_t (ZF, hmmbw_device.hpp): kChunk x the checkpoint layout.  Allocated
// as soon as observations and a dense A are both known (set_observations / set_params), so an
// out-of-memory surfaces there rather than in the first training call.
int ensure_zf(hmmbw_ctx *c) {
    if (!HMMBW_ZFULL || c->wide || !c->has_obs || !c->has_params || c->topo == HMMBW_TOPOLOGY_LEFT_TO_RIGHT || c->d_zf)
        return HMMBW_OK;
    if (int rc = dalloc(&c->d_zf, (size_t)std::max(c->cktot * kChunk, 1LL)))
        return fail(rc, "dense A: the forward's every-step store (" + std::to_string(8 * c->cktot * kChunk) +
                            " bytes) does not fit: " + g_err);
    return HMMBW_OK;
}

// Wide path with many tiles per CU: a workgroup per forward and per backward sweep, taken from a queue
// in dispatch order (k_estep_mfma<..., WQ>), so the CUs' loads even out in sweeps instead of whole
// tiles.  Measured (round 4): whole cfg5 (3,125 tiles) 12.06 against 12.37 ms per iteration; the cfg5
// shard (391 tiles, 1.5 per CU) 2.17 against 1.85 ms: with so few tiles per CU the backward sweeps
// (0.63 of a tile) start late and form the tail, so by default (HMMBW_OPT_WIDE_WQ = -1) the queue is
// used from 4 tiles per CU; 1 uses it whenever there are more tiles than CUs, 0 never (the environment
// variable HMMBW_WIDE_WQ = 0 / 1 gives the default of a new context).  (Re)allocates or frees the queue
// to match the current observations; the counters and flags start cleared.
int ensure_wq(hmmbw_ctx *c) {
    bool want = false;
    if (c->has_obs && c->wide && !c->det && c->nblocks < (1LL << 30)) {
        int ncu = 0;
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
        if (ncu > 0 && c->wq_mode != 0) want = c->nblocks > (c->wq_mode == 1 ? ncu : 4LL * ncu);
    }
    if (c->d_wq && (!want || c->wq_grid != 2 * c->nblocks)) {
        sync_ctx(c);
        dfree(c->d_wq);
        c->wq_grid = 0;
    }
    if (want && !c->d_wq) {
        if (int rc = dalloc(&c->d_wq, (size_t)c->nblocks + 2)) return rc;
        HIP_TRY(hipMemset(c->d_wq, 0, sizeof(unsigned) * ((size_t)c->nblocks + 2)));
        c->wq_grid = 2 * c->nblocks;
    }
    return HMMBW_OK;
}

// The left-to-right E-step runs the joined spread map (k_estep_join): every extra workgroup of the spread map
// (at most one per CU) becomes waves 4.. of the full workgroup with its index, so each CU runs one 8-wave
// workgroup: one M-step prologue, one set of LDS tables and one histogram flush instead of two on the CUs
// that host an extra workgroup.  cfg3: 32.2 -> 30.9 us per iteration (profiles/r5/join_ab.txt).
// Round 6: the dense E-step joins too (HMMBW_JOIN_DENSE=0 keeps its separate extra workgroups); its split B
// waves take A's hand-over through an LDS flag, so the joined workgroup's full waves are never held.
#ifndef HMMBW_JOIN_ALL
#define HMMBW_JOIN_ALL 1
#endif
bool joined_map(const hmmbw_ctx *c) {
    const bool topo_ok = c->topo == HMMBW_TOPOLOGY_LEFT_TO_RIGHT || (c->topo == HMMBW_TOPOLOGY_DENSE && c->join_dense);
    const int xw = (c->topo == HMMBW_TOPOLOGY_DENSE && c->split_extra && 2 * c->xact <= kBlock / kWave) ? 2 * c->xact
                                                                                                     : c->xact;
    // Round 6: left-to-right without extra groups too (at most 4 groups per CU, one workgroup per CU), the idle waves
    // 4-7 then only sharing the prologue's table build and the flush: T = 8 at 8,192 sequences 13.51 -> 12.96 us,
    // 8,192 x 200 27.59 -> 27.32, 4,096 x 200 24.30 -> 23.72 (profiles/r6/join_all_ab.txt)
    const bool all = HMMBW_JOIN_ALL && c->topo == HMMBW_TOPOLOGY_LEFT_TO_RIGHT && c->nblocks == c->nfull && c->fits_cus;
    return c->join && topo_ok && !c->wide && !c->det && c->lds_tables() && (c->nblocks > c->nfull || all) &&
           c->nblocks - c->nfull <= c->nfull && xw <= kBlock / kWave;
}

// The split extra waves run (estep_small_body SPLITOK, "split"): dense, and left-to-right on the joined map.
bool split_extra_map(const hmmbw_ctx *c) {
    const bool topo_ok = c->topo == HMMBW_TOPOLOGY_DENSE || (c->topo == HMMBW_TOPOLOGY_LEFT_TO_RIGHT && joined_map(c));
    return c->split_extra && !c->wide && !c->det && topo_ok && c->lds_tables() && c->nblocks > c->nfull &&
           2 * c->xact <= kBlock / kWave;
}

int plan_estep(hmmbw_ctx *c, bool fwd_only, const IterState *state, double *copies, double *llpart, double *zero,
               long long zero_len, bool merge, Plan *P, double *rank_ll = nullptr, int ncopies = 0,
               bool allow_join = true) {
    Plan &p = *P;
    p = Plan{};
    EArgs &a = p.a;
    a = make_eargs(c);
    a.state = state;
    if (ncopies > 0) a.ncopies = ncopies;
    if (copies) a.copies = copies;
    if (llpart) a.llpart = llpart;
    a.zero = zero;
    a.zero_len = zero ? zero_len : 0;
    a.rank_ll = rank_ll;
    a.done_ctr = c->d_ctr;
    const int wpb = kBlock / kWave;
    p.grid = (unsigned)c->nblocks;
    p.nll = c->nblocks;
    if (c->wide) {
        // exchange images [2][2 NP][17] (+ the backward's masked-z images [2][NP][17]) and the per-block
        // reduction scratch (estep_mfma.hpp)
        const int nt = c->NP / 16;
        p.lds = sizeof(double) * ((fwd_only ? 4 * (size_t)c->NP * 17 : 6 * (size_t)c->NP * 17) + (size_t)nt * 16 + 16);
        const Kernels kw = wide_kernels(c->NP);
        p.fn = fwd_only ? kw.score : (c->det ? kw.det_estep : kw.estep);
        p.block = (unsigned)(nt * kWave);
        if (!p.fn) return fail(HMMBW_E_UNSUPPORTED, "no wide kernel for N");
        if (!fwd_only && !c->det && c->d_wq) {  // more tiles than CUs: the work-queue form (estep_mfma.hpp)
            p.fn = wide_wq_kernel(c->NP);
            p.grid = (unsigned)c->wq_grid;
            a.wq = c->d_wq;
            a.wq_flag = c->d_wq + 2;
            a.wq_units = (int)c->nblocks;
            a.wq_timeout_ticks = ms_to_ticks(c, c->wq_timeout_ms);
            if (!p.fn) return fail(HMMBW_E_UNSUPPORTED, "no wide work-queue kernel for N");
        }
    } else {
        const bool lr = c->topo == HMMBW_TOPOLOGY_LEFT_TO_RIGHT;
        const bool lds_tab = c->lds_tables();
        {
            Kernels ks = lr ? (lds_tab ? pick_small_n<true, true>(c->N) : pick_small_n<true, false>(c->N))
                            : (lds_tab ? pick_small_n<false, true>(c->N) : pick_small_n<false, false>(c->N));
            p.fn = fwd_only ? ks.score : (c->det ? ks.det_estep : ks.estep);
            p.gfn = fwd_only ? ks.group_score : (c->det ? nullptr : ks.group_estep);
            if (!p.fn) return fail(HMMBW_E_UNSUPPORTED, "no kernel for N");
            const int NV = (lr ? 2 : c->N) + 3;
            const size_t tabs = c->lds_table_doubles();
            p.lds = sizeof(double) * (tabs + (size_t)wpb * c->G * NV + 8);
            // joined spread map: extra workgroup b's waves become waves 4.. of full workgroup b
            if (!fwd_only && allow_join && joined_map(c) && ks.join_estep) {
                p.fn = ks.join_estep;
                p.grid = (unsigned)c->nfull;
                p.nll = c->nfull;
                p.block = 2 * kBlock;
                p.lds = sizeof(double) * (tabs + (size_t)(2 * wpb) * c->G * NV + 16);  // + [8 waves][2] LL pairs
            }
            // left-to-right: split extra waves on the joined map only (round 6, cfg3 29.63 -> 28.33 us,
            // profiles/r6/split_lr_ab.txt); beside separate extra workgroups they cost more than they save
            // (round 5: 34.0 -> 35.6 us)
            if (lr && p.fn != ks.join_estep) a.split_extra = 0;
            if (HMMBW_ZFULL && !lr && !fwd_only) {  // dense: the forward stores every z_t (hmmbw_device.hpp)
                if (int rc = ensure_zf(c)) return rc;
                a.ckpt = c->d_zf;
            }
        }
    }
    if (p.grid > 0 && merge && !fwd_only && c->pend.on && c->can_merge()) {
        a.merged = 1;
        a.m = make_margs(c, c->pend);
        c->pend.on = false;
        p.flip = true;  // the launch's M-step writes the other state slot
    }
    return HMMBW_OK;
}

int launch_estep(hmmbw_ctx *c, bool fwd_only, const IterState *state, double *copies = nullptr,
                 double *llpart = nullptr, double *zero = nullptr, long long zero_len = 0, bool merge = false,
                 double *rank_ll = nullptr, int ncopies = 0) {
    Plan p;
    if (int rc = plan_estep(c, fwd_only, state, copies, llpart, zero, zero_len, merge, &p, rank_ll, ncopies)) return rc;
    if (p.grid == 0) return HMMBW_OK;
    const EArgs &a = p.a;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (c->timing && !fwd_only && (c->timing_seq++ % c->timing) == 0) {
        if (c->ev_free.size() < 2) {
            hipEvent_t x, y;
            HIP_TRY(hipEventCreate(&x));
            HIP_TRY(hipEventCreate(&y));
            c->ev_free.push_back(x);
            c->ev_free.push_back(y);
        }
        e1 = c->ev_free.back(); c->ev_free.pop_back();
        e0 = c->ev_free.back(); c->ev_free.pop_back();
        HIP_TRY(hipEventRecord(e0, c->stream));
    }
    if (int rc = launch_lds(p.fn, p.grid, p.lds, c->stream, a, p.block)) return rc;
    if (!fwd_only) c->last_nll = p.nll;
    hipEvent_t em = nullptr;
    if (e0 && (c->wide || c->det)) {
        if (c->mid_free.empty()) {
            hipEvent_t x;
            HIP_TRY(hipEventCreate(&x));
            c->mid_free.push_back(x);
        }
        em = c->mid_free.back();
        c->mid_free.pop_back();
        HIP_TRY(hipEventRecord(em, c->stream));
    }
    if (c->wide && !fwd_only) {  // B numerator: per-symbol gather of the gamma rows (estep_mfma.hpp)
        if (c->det) {  // deterministic mode: the other statistics from the partials, in workgroup order
            const long long n = c->off_bnum();
            hipLaunchKernelGGL(k_det_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, c->d_part,
                               (long long)p.grid, n, a.copies, a.state);
        }
        hipLaunchKernelGGL(bnum_gather_kernel(true), dim3((unsigned)c->K), dim3(256), 0, c->stream, c->d_gam,
                           nullptr, c->d_bptr, c->NP, c->N, 1, a.copies + c->off_bnum(), a.state);
        HIP_TRY(hipGetLastError());
    } else if (c->det && !fwd_only) {  // deterministic mode: fixed-order sums of the partials and gamma rows
        const long long n = c->off_bnum();
        hipLaunchKernelGGL(k_det_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, c->d_part,
                           (long long)p.grid, n, a.copies, a.state);
        hipLaunchKernelGGL(bnum_gather_kernel(false), dim3((unsigned)c->K), dim3(256), 0, c->stream, c->d_gam,
                           c->d_brows, c->d_bptr, c->G, c->N, 0, a.copies + c->off_bnum(), a.state);
        HIP_TRY(hipGetLastError());
    }
    if (p.flip) c->scur ^= 1;
    if (e1) {
        HIP_TRY(hipEventRecord(e1, c->stream));
        c->ev_pending.push_back(e0);
        c->ev_pending.push_back(e1);
        c->mid_pending.push_back(em);
    }
    return HMMBW_OK;
}

int drain_timing(hmmbw_ctx *c) {
    for (size_t i = 0; i + 1 < c->ev_pending.size(); i += 2) {
        HIP_TRY(hipEventSynchronize(c->ev_pending[i + 1]));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev_pending[i], c->ev_pending[i + 1]));
        c->timed_ms += ms;
        c->timed_n += 1;
        if (hipEvent_t em = c->mid_pending[i / 2]) {
            HIP_TRY(hipEventElapsedTime(&ms, c->ev_pending[i], em));
            c->timed_main_ms += ms;
            c->timed_main_n += 1;
            c->mid_free.push_back(em);
        }
        c->ev_free.push_back(c->ev_pending[i]);
        c->ev_free.push_back(c->ev_pending[i + 1]);
    }
    c->ev_pending.clear();
    c->mid_pending.clear();
    return HMMBW_OK;
}

int check_ready(hmmbw_ctx *c, bool need_armed) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (!c->has_obs) return fail(HMMBW_E_STATE, "observations not set");
    if (!c->has_params) return fail(HMMBW_E_STATE, "parameters not set");
    if (need_armed && !c->armed) return fail(HMMBW_E_STATE, "training not armed (hmmbw_reset_training)");
    return set_device(c);
}

// RCCL entry points, resolved at run time from the RCCL library already in the process (the one
// torch loaded), so that one RCCL instance serves torch.distributed and the engine.
struct Rccl {
    bool ok = false;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    ncclResult_t (*comm_count)(ncclComm_t, int *) = nullptr;  // optional (hmmbw_comm_info)
};

// HIP event pair from a pool (timing only)
int take_events(std::vector<hipEvent_t> &pool, hipEvent_t *e0, hipEvent_t *e1) {
    while (pool.size() < 2) {
        hipEvent_t x;
        HIP_TRY(hipEventCreate(&x));
        pool.push_back(x);
    }
    *e1 = pool.back(); pool.pop_back();
    *e0 = pool.back(); pool.pop_back();
    return HMMBW_OK;
}

int drain_pairs(std::vector<hipEvent_t> &pending, std::vector<hipEvent_t> &pool, double *ms_sum, long long *n) {
    for (size_t i = 0; i + 1 < pending.size(); i += 2) {
        HIP_TRY(hipEventSynchronize(pending[i + 1]));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, pending[i], pending[i + 1]));
        *ms_sum += ms;
        *n += 1;
        pool.push_back(pending[i]);
        pool.push_back(pending[i + 1]);
    }
    pending.clear();
    return HMMBW_OK;
}

int rccl_load(const char *path, Rccl **out) {
    static Rccl r;
    static std::string err;
    if (!r.ok) {
        void *h = nullptr;
        if (path && *path) h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return fail(HMMBW_E_UNSUPPORTED, std::string("cannot load RCCL: ") + dlerror());
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
        r.comm_count = reinterpret_cast<decltype(r.comm_count)>(dlsym(h, "ncclCommCount"));
        if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce || !r.error_string)
            return fail(HMMBW_E_UNSUPPORTED, "RCCL library lacks the ncclGetUniqueId / ncclCommInitRank / "
                                             "ncclCommDestroy / ncclAllReduce / ncclGetErrorString symbols");
        r.ok = true;
    }
    *out = &r;
    return HMMBW_OK;
}

int rccl_fail(const Rccl *r, ncclResult_t e, const char *what) {
    return fail(HMMBW_E_HIP, std::string(what) + ": " + (r && r->error_string ? r->error_string(e) : "RCCL error"));
}

void resolve_topology(hmmbw_ctx *c) {
    int t = c->topo_req;
    if (c->wide) t = HMMBW_TOPOLOGY_DENSE;
    if (t == HMMBW_TOPOLOGY_AUTO || t == HMMBW_TOPOLOGY_LEFT_TO_RIGHT) {
        bool lr = true;
        for (int i = 0; i < c->N && lr; ++i)
            for (int k = 0; k < c->N; ++k)
                if (c->h_A[(size_t)i * c->N + k] != 0.0 && k != i && k != i + 1) { lr = false; break; }
        t = lr ? HMMBW_TOPOLOGY_LEFT_TO_RIGHT : HMMBW_TOPOLOGY_DENSE;
    }
    c->topo = t;
}

// Memory of the peer receive regions (HMMBW_PEER_MEM).  Other GPUs write payload and flags into a region
// over xGMI while this GPU's reduce kernel polls it.  coarse (default): hipMalloc, allocated and freed with
// its context; the writers' stores are system-scope write-through and the reader's loads system-scope.
// uncached / finegrained: the hipExtMallocWithFlags kinds RCCL keeps its flags in.
// The cause of round 5's failures (wrong statistics in later contexts of one process, once a
// MEMORY_APERTURE_VIOLATION), measured in round 6 (tools/uc_stale.py, profiles/r6/uc_stale.txt, tools/peer_diag.py,
// profiles/r6/peer_diag.txt): the driver hands a freed ordinary block's addresses to the next uncached /
// fine-grained allocation, and kernel loads from such a region (system-scope and ordinary alike) can then
// return stale or foreign data while hipMemcpy reads what was written; an L2 write-back + invalidate between
// the two lives does not clear it.  In the suite, the wide path's 2.2 MB region of rank 0 landed on the
// addresses of the previous test's freed coarse region: every push landed (checked by hipMemcpy), but the
// reduce kernel read zeros and 1e-20 (another context's B floor) for some entries, so the M-step's A and B
// were wrong; the reverse transition (a freed special region's pages back as an ordinary buffer that kernels
// read) fits the aperture violation, an address formed from offsets that came back as foreign data.
// Fp64 atomics themselves sum exactly on every kind (tools/uc_probe.py).  Hence: special regions come from a
// per-process pool and never go back to the driver (no special -> ordinary transition), and a new one is
// validated with the push's stores and the reduce's loads before use (catches the ordinary -> special one;
// a region that fails is quarantined, kept allocated and unused).  Separately, in-process attachments
// (hmmbw_peer_attach) are revoked when their region is freed (peer_revoke), so no context can push through a
// pointer to a freed region.  Cross-GPU coherence of either kind over xGMI is unmeasured here.
struct PeerPool {
    std::mutex mu;
    std::vector<std::tuple<int, unsigned, size_t, void *>> free;  // (device, flags, bytes, region)
    std::map<void *, std::tuple<int, unsigned, size_t>> owned;
    std::vector<void *> quarantined;
    long long validated = 0, rejected = 0;
};
PeerPool &peer_pool() {
    static PeerPool *p = new PeerPool;  // never destroyed (its regions live for the process)
    return *p;
}

// 0: the region reads back what was written; > 0: mismatching reads; < 0: HIP error
long long validate_region(void *p, size_t bytes) {
    const long long n = (long long)(bytes / sizeof(double));
    unsigned *d_bad = nullptr;
    if (hipMalloc(reinterpret_cast<void **>(&d_bad), sizeof(unsigned)) != hipSuccess) return -1;
    unsigned bad = 0;
    long long rc = 0;
    for (unsigned seed = 1; seed <= 2 && rc == 0; ++seed) {
        if (hipMemset(d_bad, 0, sizeof(unsigned)) != hipSuccess) { rc = -1; break; }
        hipLaunchKernelGGL(k_region_fill, dim3(256), dim3(256), 0, nullptr, static_cast<double *>(p), n, seed);
        if (hipDeviceSynchronize() != hipSuccess) { rc = -1; break; }
        hipLaunchKernelGGL(k_region_check, dim3(256), dim3(256), 0, nullptr, static_cast<const double *>(p), n, seed, d_bad);
        if (hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(&bad, d_bad, sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess) { rc = -1; break; }
        rc = bad;
    }
    (void)hipFree(d_bad);
    return rc;
}

int peer_region_alloc(hmmbw_ctx *c, size_t b) {
    c->peer_special = false;
    const char *pm = std::getenv("HMMBW_PEER_MEM");
    const std::string kind = pm ? pm : "coarse";
    if (kind == "coarse") {
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&c->d_peer), b));
        ledger_add(c->d_peer, b, "peer region (coarse)");
        return HMMBW_OK;
    }
    if (kind != "uncached" && kind != "finegrained")
        return fail(HMMBW_E_INVALID, "HMMBW_PEER_MEM must be coarse, uncached or finegrained");
    const unsigned fl = kind == "finegrained" ? hipDeviceMallocFinegrained : hipDeviceMallocUncached;
    c->peer_special = true;
    PeerPool &pp = peer_pool();
    std::lock_guard<std::mutex> lk(pp.mu);
    size_t best = SIZE_MAX;
    long long bi = -1;
    for (size_t i = 0; i < pp.free.size(); ++i) {  // smallest free region of this device and kind that fits
        const auto &f = pp.free[i];
        if (std::get<0>(f) == c->device && std::get<1>(f) == fl && std::get<2>(f) >= b && std::get<2>(f) < best) {
            best = std::get<2>(f);
            bi = (long long)i;
        }
    }
    if (bi >= 0) {
        c->d_peer = static_cast<double *>(std::get<3>(pp.free[(size_t)bi]));
        pp.free.erase(pp.free.begin() + bi);
        return HMMBW_OK;
    }
    // whole 2 MB units: in the probe only allocations past 2 MB that were not a multiple of it (2.25 MB, the
    // wide path's region at world 2) read back wrong after an ordinary -> special reuse (uc_stale.txt)
    const size_t nb = (b + (size_t(2) << 20) - 1) / (size_t(2) << 20) * (size_t(2) << 20);
    for (int attempt = 0; attempt < 8; ++attempt) {
        void *p = nullptr;
        HIP_TRY(hipExtMallocWithFlags(&p, nb, fl));
        ledger_add(p, nb, kind == "finegrained" ? "peer region (fine-grained)" : "peer region (uncached)");
        const long long bad = validate_region(p, nb);
        if (bad < 0) return fail(HMMBW_E_HIP, "validating a new peer region failed");
        if (bad == 0) {
            pp.validated += 1;
            pp.owned[p] = std::make_tuple(c->device, fl, nb);
            c->d_peer = static_cast<double *>(p);
            return HMMBW_OK;
        }
        pp.rejected += 1;
        pp.quarantined.push_back(p);  // stale pages: never used, never freed
    }
    return fail(HMMBW_E_HIP, "no " + kind + " peer region read back what was written (8 attempts quarantined): use "
                "HMMBW_PEER_MEM=coarse");
}

// callers synchronise the device first (no launch of this context still writes the region)
void peer_region_free(hmmbw_ctx *c) {
    if (!c->d_peer) return;
    peer_revoke(c);
    if (c->peer_special) {  // back to the pool, never to the driver
        PeerPool &pp = peer_pool();
        std::lock_guard<std::mutex> lk(pp.mu);
        auto it = pp.owned.find(c->d_peer);
        if (it != pp.owned.end())
            pp.free.emplace_back(std::get<0>(it->second), std::get<1>(it->second), std::get<2>(it->second), c->d_peer);
        c->d_peer = nullptr;
        return;
    }
    ledger_remove(c->d_peer, "hipFree (peer region)");
    (void)hipFree(c->d_peer);
    c->d_peer = nullptr;
}

// message of a device-side stop (IterState::error, set with done by a bounded wait that expired)
std::string device_error(const IterState &h) {
    if (h.error_src == kErrWorkQueue)
        return "EM stopped on a device-side failure: a wide work-queue backward sweep did not see its tile's "
               "forward sweep finish within HMMBW_OPT_WQ_TIMEOUT_MS";
    return "EM stopped on a device-side failure: a rank did not deliver its statistics to the peer all-reduce "
           "within HMMBW_OPT_PEER_TIMEOUT_MS";
}

}  // namespace

extern "C" {

int hmmbw_abi_version(void) { return HMMBW_ABI_VERSION; }

const char *hmmbw_last_error(void) { return g_err.c_str(); }

int hmmbw_device_count(int *out) {
    if (!out) return fail(HMMBW_E_INVALID, "null out");
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    *out = n;
    return HMMBW_OK;
}

int hmmbw_cache_trim(int64_t *bytes_released) {
    const size_t b = cache_trim();
    if (bytes_released) *bytes_released = (int64_t)b;
    return HMMBW_OK;
}

int hmmbw_ctx_create(int device, int n_states, int n_symbols, hmmbw_ctx **out) {
    if (!out) return fail(HMMBW_E_INVALID, "null out");
    *out = nullptr;
    if (n_states < 1 || n_symbols < 1) return fail(HMMBW_E_INVALID, "N and M must be >= 1");
    if (n_states > 64) return fail(HMMBW_E_UNSUPPORTED, "N > 64 states is not implemented");
    if (n_symbols > 65536) return fail(HMMBW_E_UNSUPPORTED, "M > 65536 symbols is not implemented");
    hmmbw_ctx *c = new hmmbw_ctx();
    c->device = device;
    c->N = n_states;
    c->K = n_symbols;
    c->wide = n_states > 16;
    // wide: 16-state MFMA blocks, a tile of 16 sequences per workgroup (estep_mfma.hpp)
    c->NP = c->wide ? 16 * ((n_states + 15) / 16) : 0;
    c->G = c->wide ? c->NP : (n_states <= 2 ? 2 : n_states <= 4 ? 4 : n_states <= 8 ? 8 : 16);
    c->U = c->wide ? 16 : kWave / c->G;
    if (const char *we = std::getenv("HMMBW_WIDE_WQ")) c->wq_mode = std::atoi(we) == 0 ? 0 : (std::atoi(we) == 1 ? 1 : -1);
    int rc = set_device(c);
    if (!rc) {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
            c->wall_khz = khz;
    }
    if (!rc) rc = dalloc(&c->d_pi, c->N);
    if (!rc) rc = dalloc(&c->d_A, (size_t)c->N * c->N);
    if (!rc) rc = dalloc(&c->d_B, (size_t)c->N * c->K);
    if (!rc) rc = dalloc(&c->d_Bt, (size_t)c->K * c->G + c->G);
    if (!rc) rc = dalloc(&c->d_out, (size_t)c->N + (size_t)c->N * c->N + (size_t)c->N * c->K);
    if (!rc) rc = dalloc(&c->d_state, 2);
    if (!rc) rc = dalloc(&c->d_hist, 2 * (size_t)kHist);
    if (!rc) rc = dalloc(&c->d_ctr, 1);
    if (!rc) {
        const hipError_t e = hipMemset(c->d_ctr, 0, sizeof(int));
        if (e != hipSuccess) rc = fail(HMMBW_E_HIP, std::string("init: ") + hipGetErrorString(e));
    }
    if (!rc) rc = realloc_stats(c);
    if (!rc) {
        hipLaunchKernelGGL(k_init_state, dim3(1), dim3(1), 0, c->stream, c->d_state, 0.0, 0LL);
        hipLaunchKernelGGL(k_init_state, dim3(1), dim3(1), 0, c->stream, c->d_state + 1, 0.0, 0LL);
        hipError_t e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) rc = fail(HMMBW_E_HIP, std::string("init: ") + hipGetErrorString(e));
    }
    if (rc) {
        hmmbw_ctx_destroy(c);
        return rc;
    }
    *out = c;
    return HMMBW_OK;
}

int hmmbw_ctx_destroy(hmmbw_ctx *c) {
    if (!c) return HMMBW_OK;
    (void)hipSetDevice(c->device);
    // the whole device, not just the context stream: a caller may still use a buffer the context
    // handed out (hmmbw_iterate_begin) on its own stream, and the block cache reuses freed blocks at
    // once (hipFree used to synchronise the device implicitly)
    (void)hipDeviceSynchronize();
    dfree(c->d_pi); dfree(c->d_A); dfree(c->d_B); dfree(c->d_Bt); dfree(c->d_out);
    for (auto &sn : c->snaps) {
        if (sn.ev) (void)hipEventDestroy(sn.ev);
        cached_free(sn.st, kPinnedBlock);
        cached_free(sn.hist, kPinnedBlock);
    }
    dfree(c->d_state); dfree(c->d_hist); dfree(c->d_copies); dfree(c->d_ext); dfree(c->d_xbuf); dfree(c->d_ctr);
    cached_free(c->h_live, kPinnedBlock);
    if (c->comm) {
        Rccl *r = nullptr;
        if (rccl_load(nullptr, &r) == HMMBW_OK) (void)r->comm_destroy(c->comm);
        c->comm = nullptr;
    }
    peer_detach(c);
    peer_region_free(c);
    dfree(c->d_xsum);
    free_obs(c);
    for (auto e : c->ev_free) (void)hipEventDestroy(e);
    for (auto e : c->ev_pending) (void)hipEventDestroy(e);
    for (auto e : c->mid_free) (void)hipEventDestroy(e);
    for (auto e : c->mid_pending)
        if (e) (void)hipEventDestroy(e);
    for (auto e : c->ar_free) (void)hipEventDestroy(e);
    for (auto e : c->ar_pending) (void)hipEventDestroy(e);
    delete c;
    return HMMBW_OK;
}

int hmmbw_set_stream(hmmbw_ctx *c, void *stream) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (s != c->stream) {
        // later frees synchronise only the NEW stream: the block cache must not hand a buffer that work
        // queued on the old one still uses to another context
        if (int rc = set_device(c)) return rc;
        if (c->stream) HIP_TRY(hipStreamSynchronize(c->stream));
        else HIP_TRY(hipDeviceSynchronize());
    }
    c->stream = s;
    return HMMBW_OK;
}

int hmmbw_set_rank(hmmbw_ctx *c, int rank, int world) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    if (world < 1 || rank < 0 || rank >= world) return fail(HMMBW_E_INVALID, "bad rank/world");
    if (int rc = set_device(c)) return rc;
    if (int rc = flush_mstep(c)) return rc;
    if (c->rank != rank || c->world != world) peer_detach(c);  // the regions are sized for the old world
    c->rank = rank;
    c->world = world;
    return realloc_stats(c);
}

int hmmbw_set_topology(hmmbw_ctx *c, int topology) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (topology < HMMBW_TOPOLOGY_AUTO || topology > HMMBW_TOPOLOGY_LEFT_TO_RIGHT)
        return fail(HMMBW_E_INVALID, "bad topology");
    c->topo_req = topology;
    if (c->has_params) {
        resolve_topology(c);
        if (topology == HMMBW_TOPOLOGY_LEFT_TO_RIGHT && c->topo != HMMBW_TOPOLOGY_LEFT_TO_RIGHT)
            return fail(HMMBW_E_INVALID, "A is not left-to-right (nonzero a_ij with j not in {i, i+1})");
    }
    return HMMBW_OK;
}

int hmmbw_get_topology(const hmmbw_ctx *c, int *out) {
    if (!c || !out) return fail(HMMBW_E_INVALID, "null argument");
    *out = c->topo;
    return HMMBW_OK;
}

int hmmbw_set_observations(hmmbw_ctx *c, const int64_t *offsets, const int32_t *symbols, int64_t R) {
    if (!c || !offsets || (R > 0 && !symbols && offsets[R] > 0)) return fail(HMMBW_E_INVALID, "null argument");
    if (R < 0) return fail(HMMBW_E_INVALID, "negative sequence count");
    if (offsets[0] != 0) return fail(HMMBW_E_INVALID, "offsets[0] must be 0");
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    std::vector<int> len((size_t)R);
    for (int64_t r = 0; r < R; ++r) {
        const int64_t T = offsets[r + 1] - offsets[r];
        if (T < 0) return fail(HMMBW_E_INVALID, "offsets must be non-decreasing");
        if (T == 0) return fail(HMMBW_E_EMPTY_SEQUENCE, "sequence " + std::to_string(r) + " is empty");
        if (T > (1 << 28)) return fail(HMMBW_E_UNSUPPORTED, "sequence too long");
        len[(size_t)r] = (int)T;
    }
    const int64_t total = offsets[R];
    for (int64_t i = 0; i < total; ++i)
        if (symbols[i] < 0 || symbols[i] >= c->K)
            return fail(HMMBW_E_SYMBOL_RANGE, "symbol " + std::to_string(symbols[i]) + " at position " +
                                                  std::to_string(i) + " is outside [0, M)");
    if (int rc = set_device(c)) return rc;
    if (int rc = flush_mstep(c)) return rc;      // it reads this layout's log-likelihood pairs
    HIP_TRY(hipStreamSynchronize(c->stream));  // buffers may still be in use by enqueued work
    // length-sorted (descending, stable) assignment of sequences to wave slots: the sequences that
    // share a wave have near-equal lengths, so the lockstep time loop wastes little
    std::vector<int64_t> perm((size_t)R);
    std::iota(perm.begin(), perm.end(), 0);
    std::stable_sort(perm.begin(), perm.end(), [&](int64_t x, int64_t y) { return len[x] > len[y]; });
    const int U = c->U;
    const long long nwaves = (R + U - 1) / U;
    std::vector<long long> wsym((size_t)nwaves), wck((size_t)nwaves), wsp((size_t)nwaves);
    std::vector<int> wT((size_t)nwaves), wfull((size_t)nwaves), slen((size_t)(nwaves * U), 0),
        sseq((size_t)(nwaves * U), -1);
    long long symtot = 0, cktot = 0, sptot = 0;
    for (long long w = 0; w < nwaves; ++w) {
        int Tw = 0, Tmin = 1 << 30;
        for (int u = 0; u < U; ++u) {
            const long long s = w * U + u;
            if (s < R) {
                slen[(size_t)s] = len[(size_t)perm[(size_t)s]];
                sseq[(size_t)s] = (int)perm[(size_t)s];
                Tw = std::max(Tw, slen[(size_t)s]);
                Tmin = std::min(Tmin, slen[(size_t)s]);
            }
        }
        const long long nch = (Tw + kChunk - 1) / kChunk;
        wT[(size_t)w] = Tw;
        wfull[(size_t)w] = (Tmin == Tw) ? 1 : 0;
        wsym[(size_t)w] = symtot;
        wck[(size_t)w] = cktot;
        wsp[(size_t)w] = sptot;
        symtot += nch * U * kChunk;
        if (c->wide) {  // full alpha_hat [t][NP/16 waves][4][64 lanes] + exponents [t][16]
            cktot += nch * kChunk * (long long)c->NP * 16;
            sptot += nch * kChunk * 16;
        } else {        // one checkpoint per chunk [c][64] + exponent packs [c][u]
            cktot += nch * kWave;
            sptot += nch * U;
        }
    }
    // packs hold LDS byte offsets of the emission record rows when the tables live in LDS (< 64 KiB,
    // so they fit uint16), symbol ids otherwise
    const bool lds_off = c->lds_tables();
    const long long row_bytes = (long long)(c->G + kTabPad) * 16;  // 16-B table entries
    std::vector<uint16_t> hsym((size_t)std::max(symtot, 1LL), 0);
    for (long long w = 0; w < nwaves; ++w)
        for (int u = 0; u < U; ++u) {
            const long long s = w * U + u;
            if (s >= R) continue;
            const int64_t r = perm[(size_t)s];
            const int T = len[(size_t)r];
            for (int t = 0; t < T; ++t)
                hsym[(size_t)(wsym[(size_t)w] + ((long long)(t / kChunk) * U + u) * kChunk + t % kChunk)] =
                    (uint16_t)(lds_off ? symbols[offsets[r] + t] * row_bytes : symbols[offsets[r] + t]);
        }
    free_obs(c);
    const int wpb = kBlock / kWave;
    long long nblocks = c->wide ? nwaves : (nwaves + wpb - 1) / wpb;  // wide: one tile per block
    // Small kernels, more waves than SIMDs: one full 4-wave workgroup per CU, then the remaining waves
    // in workgroups of xact = 2 active waves (one per CU while they fit), so the SIMDs that must run a
    // second wave are spread over twice as many CUs, which then share their LDS and memory pipes among
    // 6 waves instead of 8.  cfg3 (1,250 waves): 38.2 -> 36.5 us per iteration; xact = 1 (a prologue
    // and histogram flush per extra wave) and 3 measured no better.  HMMBW_XACT
    // overrides it (diagnostics: 1..4, 4 = every workgroup full).
    // A/B switches (read before the map, which depends on the split)
    if (const char *pe = std::getenv("HMMBW_PRIO")) c->prio = std::atoi(pe);
    if (const char *se = std::getenv("HMMBW_SPLIT_EXTRA")) c->split_extra = std::atoi(se) != 0;
    if (const char *je = std::getenv("HMMBW_JOIN")) c->join = std::atoi(je) != 0;
    if (const char *jd = std::getenv("HMMBW_JOIN_DENSE")) c->join_dense = std::atoi(jd) != 0;
    long long nfull = nblocks;
    int xact = wpb;
    if (!c->wide && !c->det) {
        int ncu = 0;
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
        if (ncu > 0 && nwaves > (long long)ncu * wpb) {
            const long long extra = nwaves - (long long)ncu * wpb;
            const char *xe = std::getenv("HMMBW_XACT");
            int xa = extra <= 2LL * ncu ? 2 : wpb;
            // dense (as requested before the observations) with the split extra waves: one group per extra
            // workgroup while they fit one per CU (cfg3 dense 63.5 -> 62.2 us, profiles/r5/spread_knobs.txt)
            if (c->topo_req == HMMBW_TOPOLOGY_DENSE && c->split_extra && extra <= ncu) xa = 1;
            if (xe) xa = std::max(1, std::min(wpb, std::atoi(xe)));
            // left-to-right on the joined map: past 2 extra groups per CU they still join the full workgroups,
            // up to 4 per CU (cfg4 shard, 12,500 sequences: 135 workgroups of 8 waves instead of 2 x 135 of 4)
            const bool join4 = !xe && xa == wpb && c->join && c->topo_req != HMMBW_TOPOLOGY_DENSE;
            if ((xa < wpb || join4) && (extra + xa - 1) / xa <= ncu) {
                nfull = ncu;
                xact = xa;
                nblocks = nfull + (extra + xa - 1) / xa;
            }
        }
    }
    int rc = dalloc(&c->d_sym, (size_t)std::max(symtot, 1LL));
    if (!rc) rc = dalloc(&c->d_wsym, (size_t)nwaves);
    if (!rc) rc = dalloc(&c->d_wckoff, (size_t)nwaves);
    if (!rc) rc = dalloc(&c->d_wspoff, (size_t)nwaves);
    if (!rc) rc = dalloc(&c->d_wT, (size_t)nwaves);
    if (!rc) rc = dalloc(&c->d_wfull, (size_t)nwaves);
    if (!rc) rc = dalloc(&c->d_slen, (size_t)(nwaves * U));
    if (!rc) rc = dalloc(&c->d_sseq, (size_t)(nwaves * U));
    if (!rc) rc = dalloc(&c->d_ck, (size_t)std::max(cktot, 1LL));
    c->cktot = cktot;
    if (!rc) {
        if (c->wide) rc = dalloc(&c->d_ebuf, (size_t)std::max(sptot, 1LL));
        else rc = dalloc(&c->d_sp, (size_t)std::max(sptot, 1LL));
    }
    std::vector<long long> bptr;
    std::vector<unsigned> brows;
    if (c->wide) {
        // position -> its row in symbol order (positions of one symbol in tile-row order): the E-step writes
        // the gamma row of tile row wck / NP + t * 16 + u there (brows, indexed by tile row), so symbol k's
        // rows are [bptr[k], bptr[k+1]) and k_bnum_gather streams them
        if (cktot / c->NP >= (1LL << 32)) return fail(HMMBW_E_UNSUPPORTED, "too many positions for the wide path");
        bptr.assign((size_t)c->K + 1, 0);
        for (int64_t i = 0; i < total; ++i) ++bptr[(size_t)symbols[i] + 1];
        for (int k = 0; k < c->K; ++k) bptr[(size_t)k + 1] += bptr[(size_t)k];
        std::vector<long long> fill(bptr.begin(), bptr.end() - 1);
        // rows of padding slots (a tile's slots past the last sequence: full-tile code paths store their
        // exact-zero gamma rows unmasked) all go to one scratch row past the real ones
        brows.assign((size_t)std::max(cktot / c->NP, 1LL), (unsigned)total);
        for (long long w = 0; w < nwaves; ++w)
            for (int u = 0; u < U; ++u) {
                const long long sl = w * U + u;
                if (sl >= R) continue;
                const int64_t r = perm[(size_t)sl];
                for (int t = 0; t < len[(size_t)r]; ++t)
                    brows[(size_t)(wck[(size_t)w] / c->NP + (long long)t * U + u)] =
                        (unsigned)fill[(size_t)symbols[offsets[r] + t]]++;
            }
        if (!rc) rc = dalloc(&c->d_gam, (size_t)(total + 1) * c->NP);
        if (!rc) rc = dalloc(&c->d_bptr, bptr.size());
        if (!rc) rc = dalloc(&c->d_brows, brows.size());
        if (!rc && c->det) rc = dalloc(&c->d_part, (size_t)std::max(nblocks, 1LL) * (size_t)c->off_bnum());
    } else if (c->det) {  // deterministic mode: symbol -> pack positions (gamma row = pack index), stable
        if (symtot >= (1LL << 32)) return fail(HMMBW_E_UNSUPPORTED, "too many positions for the deterministic mode");
        bptr.assign((size_t)c->K + 1, 0);
        for (int64_t i = 0; i < total; ++i) ++bptr[(size_t)symbols[i] + 1];
        for (int k = 0; k < c->K; ++k) bptr[(size_t)k + 1] += bptr[(size_t)k];
        std::vector<long long> fill(bptr.begin(), bptr.end() - 1);
        brows.resize((size_t)std::max<int64_t>(total, 1));
        for (long long w = 0; w < nwaves; ++w)
            for (int u = 0; u < U; ++u) {
                const long long sl = w * U + u;
                if (sl >= R) continue;
                const int64_t r = perm[(size_t)sl];
                for (int t = 0; t < len[(size_t)r]; ++t)
                    brows[(size_t)fill[(size_t)symbols[offsets[r] + t]]++] =
                        (unsigned)(wsym[(size_t)w] + ((long long)(t / kChunk) * U + u) * kChunk + t % kChunk);
            }
        if (!rc) rc = dalloc(&c->d_gam, (size_t)std::max(symtot, 1LL) * c->G);
        if (!rc) rc = dalloc(&c->d_bptr, bptr.size());
        if (!rc) rc = dalloc(&c->d_brows, brows.size());
        if (!rc) rc = dalloc(&c->d_part, (size_t)std::max(nblocks, 1LL) * (size_t)c->off_bnum());
    }
    if (!rc) rc = dalloc(&c->d_logp, (size_t)std::max<int64_t>(R, 1));
    if (!rc) rc = dalloc(&c->d_llpart, 4 * (size_t)std::max(nblocks, 1LL));
    if (rc) return rc;
    HIP_TRY(hipMemcpy(c->d_sym, hsym.data(), sizeof(uint16_t) * hsym.size(), hipMemcpyHostToDevice));
    if (c->wide || c->det) {
        HIP_TRY(hipMemcpy(c->d_bptr, bptr.data(), sizeof(long long) * bptr.size(), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_brows, brows.data(), sizeof(unsigned) * brows.size(), hipMemcpyHostToDevice));
    }
    if (nwaves > 0) {
        HIP_TRY(hipMemcpy(c->d_wsym, wsym.data(), sizeof(long long) * nwaves, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_wckoff, wck.data(), sizeof(long long) * nwaves, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_wspoff, wsp.data(), sizeof(long long) * nwaves, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_wT, wT.data(), sizeof(int) * nwaves, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_wfull, wfull.data(), sizeof(int) * nwaves, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_slen, slen.data(), sizeof(int) * nwaves * U, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_sseq, sseq.data(), sizeof(int) * nwaves * U, hipMemcpyHostToDevice));
    }
    std::vector<double> ninf((size_t)std::max<int64_t>(R, 1), -INFINITY);
    HIP_TRY(hipMemcpy(c->d_logp, ninf.data(), sizeof(double) * ninf.size(), hipMemcpyHostToDevice));
    std::vector<double> zpairs(4 * (size_t)std::max(nblocks, 1LL), 0.0);
    HIP_TRY(hipMemcpy(c->d_llpart, zpairs.data(), sizeof(double) * zpairs.size(), hipMemcpyHostToDevice));
    c->R = R;
    c->nwaves = nwaves;
    c->nblocks = nblocks;
    c->nfull = nfull;
    {
        int ncu = 0;
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
        c->fits_cus = ncu > 0 && nblocks <= ncu;
    }
    c->xact = xact;
    c->has_obs = true;
    if (int rc2 = ensure_wq(c)) return rc2;
    return ensure_zf(c);
}

int hmmbw_set_option(hmmbw_ctx *c, int key, int64_t value) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    if (key == HMMBW_OPT_SAFE_SCALING) {
        c->force_safe = value != 0;
        return HMMBW_OK;
    }
    if (key == HMMBW_OPT_STAT_COPIES) {
        if (value < 1 || value > 1024) return fail(HMMBW_E_INVALID, "statistics copies must be in [1, 1024]");
        if (int rc = set_device(c)) return rc;
        if (int rc = flush_mstep(c)) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));
        c->ncopies = (int)value;
        return realloc_stats(c);
    }
    if (key == HMMBW_OPT_DETERMINISTIC) {
        if (c->has_obs) return fail(HMMBW_E_STATE, "set the deterministic mode before hmmbw_set_observations");
        if (value != 0 && !c->wide && !c->lds_tables())
            return fail(HMMBW_E_UNSUPPORTED, "deterministic mode needs the LDS emission tables (N <= 16) or the wide path");
        c->det = value != 0;
        return HMMBW_OK;
    }
    if (key == HMMBW_OPT_MERGE_MSTEP) {
        if (int rc = set_device(c)) return rc;
        if (int rc = flush_mstep(c)) return rc;
        c->merge_mstep = value != 0;
        return HMMBW_OK;
    }
    if (key == HMMBW_OPT_ALLREDUCE) {
        if (value != HMMBW_ALLREDUCE_RCCL && value != HMMBW_ALLREDUCE_PEER)
            return fail(HMMBW_E_INVALID, "HMMBW_OPT_ALLREDUCE: 0 (RCCL / caller) or 1 (peer)");
        c->ar_kind = (int)value;
        return HMMBW_OK;
    }
    if (key == HMMBW_OPT_PEER_TIMEOUT_MS) {
        if (value < 1) return fail(HMMBW_E_INVALID, "peer timeout must be >= 1 ms");
        c->peer_timeout_ms = value;
        return HMMBW_OK;
    }
    if (key == HMMBW_OPT_LIVE_STATUS) {
        if (int rc = set_device(c)) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));  // no launch of the old setting is still in flight
        if (value == 0) {
            cached_free(c->h_live, kPinnedBlock);
            c->h_live = nullptr;
            return HMMBW_OK;
        }
        if (c->h_live) return HMMBW_OK;
        HIP_TRY(cached_alloc(reinterpret_cast<void **>(&c->h_live), sizeof(LiveBlock), kPinnedBlock));
        // seed the mirror with the state as it stands (records of a pending M-step follow when it runs)
        IterState h{};
        HIP_TRY(hipMemcpy(&h, c->state(), sizeof(IterState), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(c->h_live->hist, c->d_hist, sizeof(double) * 2 * (size_t)kHist, hipMemcpyDeviceToHost));
        c->h_live->slot[h.iteration & 1] = h;
        std::atomic_thread_fence(std::memory_order_release);
        reinterpret_cast<volatile unsigned long long &>(c->h_live->pub) =
            ((unsigned long long)c->live_epoch << 32) | (unsigned long long)(unsigned)h.iteration;
        return HMMBW_OK;
    }
    if (key == HMMBW_OPT_WQ_TIMEOUT_MS) {
        if (value < 0) return fail(HMMBW_E_INVALID, "work-queue timeout must be >= 0 ms");
        c->wq_timeout_ms = value;
        return HMMBW_OK;
    }
    if (key == HMMBW_OPT_WIDE_WQ) {
        if (value < -1 || value > 1) return fail(HMMBW_E_INVALID, "HMMBW_OPT_WIDE_WQ: -1 (auto), 0 (off) or 1 (on)");
        if (int rc = set_device(c)) return rc;
        c->wq_mode = (int)value;
        return ensure_wq(c);
    }
    if (key == HMMBW_OPT_ABLATE) {  // diagnostics: results are wrong while set
        c->ablate = (int)value;
        return HMMBW_OK;
    }
    return fail(HMMBW_E_INVALID, "unknown option " + std::to_string(key));
}

int hmmbw_get_option(const hmmbw_ctx *c, int key, int64_t *value) {
    if (!c || !value) return fail(HMMBW_E_INVALID, "null argument");
    switch (key) {
        case HMMBW_OPT_SAFE_SCALING: *value = c->force_safe; return HMMBW_OK;
        case HMMBW_OPT_ABLATE: *value = c->ablate; return HMMBW_OK;
        case HMMBW_OPT_STAT_COPIES: *value = c->ncopies; return HMMBW_OK;
        case HMMBW_OPT_MERGE_MSTEP: *value = c->merge_mstep ? 1 : 0; return HMMBW_OK;
        case HMMBW_OPT_DETERMINISTIC: *value = c->det ? 1 : 0; return HMMBW_OK;
        case HMMBW_OPT_ALLREDUCE: *value = c->ar_kind; return HMMBW_OK;
        case HMMBW_OPT_PEER_TIMEOUT_MS: *value = c->peer_timeout_ms; return HMMBW_OK;
        case HMMBW_OPT_LIVE_STATUS: *value = c->h_live ? 1 : 0; return HMMBW_OK;
        case HMMBW_OPT_WQ_TIMEOUT_MS: *value = c->wq_timeout_ms; return HMMBW_OK;
        case HMMBW_OPT_WIDE_WQ: *value = c->wq_mode; return HMMBW_OK;
        case HMMBW_INFO_WIDE_WQ_ACTIVE: *value = c->d_wq ? 1 : 0; return HMMBW_OK;
        case HMMBW_INFO_WAVES: *value = c->wide ? c->nblocks * (c->NP / 16) : c->nwaves; return HMMBW_OK;
        case HMMBW_INFO_WORKGROUPS: *value = c->d_wq ? c->wq_grid : c->nblocks; return HMMBW_OK;
        case HMMBW_INFO_WAVES_PER_WORKGROUP: *value = c->wide ? c->NP / 16 : kBlock / kWave; return HMMBW_OK;
        case HMMBW_INFO_FULL_WORKGROUPS: *value = c->wide ? c->nblocks : std::min(c->nfull, c->nblocks); return HMMBW_OK;
        case HMMBW_INFO_EXTRA_WAVES: *value = c->wide ? 0 : c->xact; return HMMBW_OK;
        case HMMBW_INFO_PEER_CHUNKS: *value = c->d_peer ? c->peer_nch : 0; return HMMBW_OK;
        case HMMBW_INFO_JOINED: *value = c->has_obs && joined_map(c) ? 1 : 0; return HMMBW_OK;
        case HMMBW_INFO_SPLIT_EXTRA: *value = c->has_obs && split_extra_map(c) ? 1 : 0; return HMMBW_OK;
        case HMMBW_INFO_PEER_SUM_PTR: *value = (int64_t)(intptr_t)c->d_xsum; return HMMBW_OK;
        case HMMBW_INFO_PEER_REGIONS_VALIDATED:
        case HMMBW_INFO_PEER_REGIONS_REJECTED: {
            PeerPool &pp = peer_pool();
            std::lock_guard<std::mutex> lk(pp.mu);
            *value = key == HMMBW_INFO_PEER_REGIONS_VALIDATED ? pp.validated : pp.rejected;
            return HMMBW_OK;
        }
        default: return fail(HMMBW_E_INVALID, "unknown option " + std::to_string(key));
    }
}

int hmmbw_set_params(hmmbw_ctx *c, const double *pi, const double *A, const double *B) {
    if (!c || !pi || !A || !B) return fail(HMMBW_E_INVALID, "null argument");
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    if (int rc = set_device(c)) return rc;
    if (int rc = flush_mstep(c)) return rc;  // it would overwrite the new parameters later
    HIP_TRY(hipStreamSynchronize(c->stream));
    const int N = c->N, K = c->K, G = c->G;
    // safe_log semantics (hmm_training.py:46-54): x <= 0 (and NaN) is a zero probability
    auto clean = [](double x) { return x > 0.0 ? x : 0.0; };
    std::vector<double> hpi(N), hA((size_t)N * N), hB((size_t)N * K), hBt((size_t)K * G + G, 0.0);
    for (int i = 0; i < N; ++i) hpi[i] = clean(pi[i]);
    for (size_t i = 0; i < hA.size(); ++i) hA[i] = clean(A[i]);
    for (int jj = 0; jj < N; ++jj)
        for (int k = 0; k < K; ++k) {
            const double v = clean(B[(size_t)jj * K + k]);
            hB[(size_t)jj * K + k] = v;
            hBt[(size_t)k * G + (c->wide ? bt_col(jj) : jj)] = v;
        }
    HIP_TRY(hipMemcpy(c->d_pi, hpi.data(), sizeof(double) * N, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_A, hA.data(), sizeof(double) * hA.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_B, hB.data(), sizeof(double) * hB.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_Bt, hBt.data(), sizeof(double) * hBt.size(), hipMemcpyHostToDevice));
    c->h_A = hA;
    c->has_params = true;
    resolve_topology(c);
    return ensure_zf(c);
}

int hmmbw_reset_training(hmmbw_ctx *c, double epsilon, int64_t max_iterations) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    if (int rc = set_device(c)) return rc;
    if (int rc = flush_mstep(c)) return rc;
    hipLaunchKernelGGL(k_init_state, dim3(1), dim3(1), 0, c->stream, c->state(), epsilon, (long long)max_iterations);
    HIP_TRY(hipGetLastError());
    ++c->live_epoch;  // the mirror's records of the previous run no longer count (hmmbw_status_live_wait)
    HIP_TRY(hipMemsetAsync(c->d_copies, 0, sizeof(double) * 3 * c->ncopies * c->copy_len(), c->stream));
    if (c->d_xbuf) HIP_TRY(hipMemsetAsync(c->d_xbuf, 0, sizeof(double) * 3 * (size_t)c->xlen, c->stream));
    // the work queue's counters and flags: a run stopped by a work-queue timeout leaves them armed (the
    // workgroups that start after the stop return at once and never reach the re-arm)
    if (c->d_wq) HIP_TRY(hipMemsetAsync(c->d_wq, 0, sizeof(unsigned) * ((size_t)c->nblocks + 2), c->stream));
    // the fused multi-rank completion counter: workgroups that start after a device-side stop return
    // before counting their log-likelihood pair, so a stopped launch leaves it part-way; the next run's
    // last-workgroup fold must start from zero
    HIP_TRY(hipMemsetAsync(c->d_ctr, 0, sizeof(int), c->stream));
    c->e_count = 0;
    c->armed = true;
    return HMMBW_OK;
}

int hmmbw_stats_len(const hmmbw_ctx *c, int64_t *n) {
    if (!c || !n) return fail(HMMBW_E_INVALID, "null argument");
    *n = c->stats_len();
    return HMMBW_OK;
}

int hmmbw_estep(hmmbw_ctx *c, double *stats_dev) {
    if (int rc = check_ready(c, true)) return rc;
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    if (!stats_dev) return fail(HMMBW_E_INVALID, "null stats buffer");
    if (c->pend.on && !c->can_merge())
        if (int rc = flush_mstep(c)) return rc;
    const long long e = c->e_count++;
    double *llp = c->llpart(e);
    // multi-rank: one copy set, cleared by k_reduce_local
    if (int rc = launch_estep(c, false, c->state(), c->copies(0), llp, nullptr, 0, true)) return rc;
    const long long n = c->copy_len();
    const unsigned grid = (unsigned)std::min<long long>((n + 255) / 256, 64);
    hipLaunchKernelGGL(k_reduce_local, dim3(grid), dim3(256), 0, c->stream, c->copies(0), c->det ? 1 : c->ncopies, n, llp,
                       c->last_nll, stats_dev, c->off_ll(), c->world, c->rank, c->state());
    HIP_TRY(hipGetLastError());
    return HMMBW_OK;
}

int hmmbw_mstep(hmmbw_ctx *c, double *stats_dev, int64_t n_seq_global) {
    if (int rc = check_ready(c, true)) return rc;
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    if (!stats_dev) return fail(HMMBW_E_INVALID, "null stats buffer");
    if (int rc = flush_mstep(c)) return rc;
    hmmbw_ctx::Pending &p = c->pend;
    p.on = true;
    p.local = false;
    p.src = stats_dev;
    p.nsrc = 1;
    p.ll = stats_dev + c->off_ll();
    p.nll = c->world;
    p.ext = stats_dev;
    p.R = n_seq_global;
    // deferred into the next hmmbw_estep launch when that can merge it; queries flush it
    return c->can_merge() ? HMMBW_OK : flush_mstep(c);
}

// First half of one multi-rank EM iteration: this rank's E-step, leaving in *buf (*len doubles, device
// memory of the context) the partial statistics that every rank must all-reduce (sum) before mr_end.
// Small kernels: fused (the E-step accumulates straight into a triple-buffered all-reduce buffer and
// its last workgroup writes the rank's (max, sum exp) pair; no k_reduce_local launch).  Wide and
// deterministic paths: hmmbw_estep + k_reduce_local into d_ext.  The layout is rank-independent: every
// rank all-reduces the same buffer shape, also a rank whose shard is empty.
static int mr_begin(hmmbw_ctx *c, long long n_seq_global, double **buf, long long *len) {
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    const bool fused = !c->det;  // the small and the wide E-step accumulate into the all-reduce buffer
    if (fused) {
        // rounded to 256 B so all three buffers keep the copies' alignment (a 16-B shift splits the
        // B-numerator rows' 64-B segments over two cache lines; ~0.7 us per launch at cfg3)
        const int nc = c->xcopies();
        const long long xl = c->ar_payload();
        if (c->xlen != xl) {
            if (int rc = flush_mstep(c)) return rc;
            // the caller may still read or write the old buffer on its own stream (its all-reduce)
            HIP_TRY(hipDeviceSynchronize());
            dfree(c->d_xbuf);
            if (int rc = dalloc(&c->d_xbuf, 3 * (size_t)xl)) return rc;
            HIP_TRY(hipMemsetAsync(c->d_xbuf, 0, sizeof(double) * 3 * (size_t)xl, c->stream));
            c->xlen = xl;
            c->e_count = 0;
        }
        if (c->pend.on && !c->can_merge())
            if (int rc = flush_mstep(c)) return rc;
        const long long e = c->e_count++;
        double *X = c->d_xbuf + (e % 3) * c->xlen, *Xn = c->d_xbuf + ((e + 1) % 3) * c->xlen;
        const long long ll_off = (long long)nc * c->copy_len();
        // accumulate into X (the merged M-step reads the previous, all-reduced X), clear the next
        if (c->nblocks > 0) {
            if (int rc = launch_estep(c, false, c->state(), X, c->llpart(e), Xn, c->xlen, true,
                                      X + ll_off + 2LL * c->rank, nc))
                return rc;
        } else {  // empty shard: contribute zeros (no E-step launch clears the buffers)
            HIP_TRY(hipMemsetAsync(X, 0, sizeof(double) * (size_t)c->xlen, c->stream));
        }
        *buf = X;
        *len = c->xlen;
    } else {
        if (c->ext_len != c->stats_len()) {  // sized by the world of hmmbw_set_rank
            if (int rc = flush_mstep(c)) return rc;
            HIP_TRY(hipStreamSynchronize(c->stream));
            dfree(c->d_ext);
            if (int rc = dalloc(&c->d_ext, (size_t)c->stats_len())) return rc;
            HIP_TRY(hipMemsetAsync(c->d_ext, 0, sizeof(double) * (size_t)c->stats_len(), c->stream));
            c->ext_len = c->stats_len();
        }
        if (int rc = hmmbw_estep(c, c->d_ext)) return rc;
        *buf = c->d_ext;
        *len = c->ext_len;
    }
    c->ar_open = true;
    c->ar_fused = fused;
    c->ar_cur = *buf;
    c->ar_R = n_seq_global;
    return HMMBW_OK;
}

// Peer all-reduce halves (kernels above): push this rank's buffer to every rank's slot `rank` after the
// E-step, and wait for / sum every rank's slot before the M-step.
static PeerArgs peer_args(const hmmbw_ctx *c) {
    PeerArgs P{};
    for (int r = 0; r < c->peer_world; ++r) P.region[r] = c->peer_regions[(size_t)r];
    P.n = c->peer_n;
    P.slot = c->peer_slot;
    P.nch = c->peer_nch;
    P.dpt = c->peer_dpt;
    P.world = c->peer_world;
    P.rank = c->rank;
    P.perturb = c->peer_perturb;
    return P;
}

static int peer_push(hmmbw_ctx *c, const double *buf, long long len) {
    if (len != c->peer_n || c->peer_world != c->world)
        return fail(HMMBW_E_STATE, "the all-reduce payload changed after hmmbw_peer_region (rank, world or options "
                                   "set after it): set up the peer regions again");
    c->peer_seq += 1;
    hipLaunchKernelGGL(k_peer_push, dim3((unsigned)c->peer_nch, (unsigned)c->peer_world), dim3(kPeerThreads), 0,
                       c->stream, buf, peer_args(c), c->peer_seq, c->state());
    HIP_TRY(hipGetLastError());
    return HMMBW_OK;
}

// hmmbw_iterate's loop: push, wait and sum in one launch (k_peer_allreduce)
static int peer_allreduce(hmmbw_ctx *c, double *buf, long long len) {
    if (len != c->peer_n || c->peer_world != c->world)
        return fail(HMMBW_E_STATE, "the all-reduce payload changed after hmmbw_peer_region (rank, world or options "
                                   "set after it): set up the peer regions again");
    c->peer_seq += 1;
    const long long ticks = ms_to_ticks(c, std::max(1LL, c->peer_timeout_ms));
    hipLaunchKernelGGL(k_peer_allreduce, dim3((unsigned)c->peer_nch, (unsigned)c->peer_world), dim3(kPeerThreads), 0,
                       c->stream, buf, c->d_xsum, peer_args(c), c->peer_seq, c->state(), ticks);
    HIP_TRY(hipGetLastError());
    c->ar_cur = c->d_xsum;  // the pending M-step reads the sums
    return HMMBW_OK;
}

// the sums go to d_xsum, which becomes the pending M-step's source (mr_end)
static int peer_reduce(hmmbw_ctx *c) {
    const long long ticks = ms_to_ticks(c, std::max(1LL, c->peer_timeout_ms));
    hipLaunchKernelGGL(k_peer_reduce, dim3((unsigned)c->peer_nch), dim3(kPeerThreads), 0, c->stream, c->d_xsum,
                       peer_args(c), c->peer_seq, c->state(), ticks);
    HIP_TRY(hipGetLastError());
    c->ar_cur = c->d_xsum;
    return HMMBW_OK;
}

// Second half: the M-step from the all-reduced buffer (merged into the next E-step launch when it can).
static int mr_end(hmmbw_ctx *c) {
    if (!c->ar_open) return fail(HMMBW_E_STATE, "no open iteration (hmmbw_iterate_begin first)");
    c->ar_open = false;
    if (!c->ar_fused) return hmmbw_mstep(c, c->ar_cur, c->ar_R);
    hmmbw_ctx::Pending &p = c->pend;
    p.on = true;
    p.local = false;
    p.src = c->ar_cur;
    p.nsrc = c->xcopies();
    p.ll = c->ar_cur + (long long)c->xcopies() * c->copy_len();
    p.nll = c->world;
    p.ext = c->ar_cur;
    p.R = c->ar_R;
    return c->can_merge() ? HMMBW_OK : flush_mstep(c);
}

int hmmbw_iterate_begin(hmmbw_ctx *c, int64_t n_seq_global, double **buf, int64_t *n_doubles) {
    if (int rc = check_ready(c, true)) return rc;
    if (!buf || !n_doubles) return fail(HMMBW_E_INVALID, "null argument");
    if (n_seq_global < 0) return fail(HMMBW_E_INVALID, "negative sequence count");
    if (c->ar_kind == HMMBW_ALLREDUCE_PEER && !c->peer_on) return fail(HMMBW_E_STATE, peer_off_msg(c));
    long long len = 0;
    if (int rc = mr_begin(c, n_seq_global, buf, &len)) return rc;
    if (c->peer_mode()) {  // the whole exchange is the engine's: push now, wait + sum in _end
        if (int rc = peer_push(c, *buf, len)) {
            c->ar_open = false;
            return rc;
        }
        c->ar_len_last = len;
    }
    *n_doubles = len;
    return HMMBW_OK;
}

int hmmbw_iterate_end(hmmbw_ctx *c) {
    if (int rc = check_ready(c, true)) return rc;
    if (c->ar_open && c->peer_mode())
        if (int rc = peer_reduce(c)) {
            c->ar_open = false;
            return rc;
        }
    return mr_end(c);
}

int hmmbw_peer_region(hmmbw_ctx *c, void **region, int64_t *bytes) {
    if (!c || !region || !bytes) return fail(HMMBW_E_INVALID, "null argument");
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    if (c->world > kMaxPeers) return fail(HMMBW_E_UNSUPPORTED, "peer all-reduce: at most 16 ranks");
    if (int rc = set_device(c)) return rc;
    const long long n = c->ar_payload();
    const long long dpt = std::min(64LL, std::max(1LL, (n + (long long)kPeerThreads * kPeerMaxChunks - 1) /
                                                       ((long long)kPeerThreads * kPeerMaxChunks)));
    const long long slot = (n + 31) / 32 * 32, nch = (n + kPeerThreads * dpt - 1) / (kPeerThreads * dpt);
    const size_t b = sizeof(double) * 2 * (size_t)c->world * (size_t)slot +
                     sizeof(unsigned long long) * (size_t)c->world * (size_t)nch;
    if (!c->d_peer || c->peer_n != n || c->peer_world != c->world) {
        peer_detach(c);
        HIP_TRY(hipDeviceSynchronize());
        peer_region_free(c);
        // its own allocation (exported with hipIpcGetMemHandle), never a block of the cache
        if (int rc = peer_region_alloc(c, b)) return rc;
        HIP_TRY(hipMemset(c->d_peer, 0, b));
        dfree(c->d_xsum);
        if (int rc = dalloc(&c->d_xsum, (size_t)slot)) return rc;
        HIP_TRY(hipMemset(c->d_xsum, 0, sizeof(double) * (size_t)slot));
        c->peer_bytes = b;
        c->peer_n = n;
        c->peer_slot = slot;
        c->peer_nch = nch;
        c->peer_dpt = (int)dpt;
        c->peer_world = c->world;
    }
    *region = c->d_peer;
    *bytes = (int64_t)c->peer_bytes;
    return HMMBW_OK;
}

int hmmbw_peer_ipc_handle(hmmbw_ctx *c, void *handle_out) {
    if (!c || !handle_out) return fail(HMMBW_E_INVALID, "null argument");
    if (!c->d_peer) return fail(HMMBW_E_STATE, "no peer region (hmmbw_peer_region first)");
    if (int rc = set_device(c)) return rc;
    hipIpcMemHandle_t h;
    HIP_TRY(hipIpcGetMemHandle(&h, c->d_peer));
    static_assert(sizeof(h) == 64, "HIP IPC handles are 64 bytes");
    std::memcpy(handle_out, &h, sizeof(h));
    return HMMBW_OK;
}

static int peer_attach_impl(hmmbw_ctx *c, const std::vector<double *> &regions, int64_t n_seq_global) {
    HIP_TRY(hipDeviceSynchronize());
    // a fresh exchange: clear this rank's slots and flags (every rank attaches before any iterates)
    HIP_TRY(hipMemset(c->d_peer, 0, c->peer_bytes));
    c->peer_regions = regions;
    {
        PeerLinks &pl = peer_links();
        std::lock_guard<std::mutex> lk(pl.mu);
        for (double *r : regions) pl.users[r].push_back(c);
    }
    c->peer_seq = 0;
    c->peer_on = true;
    c->peer_revoked = false;
    // diagnostics: one rank pushes a wrong payload, so the exchange disagrees with any other all-reduce
    // (tests/test_bench.py drives bench.py's leg check with it)
    c->peer_perturb = 0.0;
    if (const char *pe = std::getenv("HMMBW_DIAG_PEER_PERTURB")) {
        const char *colon = std::strchr(pe, ':');
        if (colon && std::atoi(pe) == c->rank) c->peer_perturb = std::atof(colon + 1);
    }
    c->R_global = n_seq_global;  // the R of hmm_training.py:424 for hmmbw_iterate's loop
    return HMMBW_OK;
}

int hmmbw_peer_attach(hmmbw_ctx *c, void *const *regions, int64_t n_seq_global) {
    if (!c || !regions) return fail(HMMBW_E_INVALID, "null argument");
    if (n_seq_global < 0) return fail(HMMBW_E_INVALID, "negative sequence count");
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    if (!c->d_peer || c->peer_world != c->world || c->peer_n != c->ar_payload())
        return fail(HMMBW_E_STATE, "no current peer region (hmmbw_peer_region first, after set_rank and options)");
    if (regions[c->rank] != c->d_peer) return fail(HMMBW_E_INVALID, "regions[rank] must be this context's own region");
    std::vector<double *> reg((size_t)c->world);
    for (int r = 0; r < c->world; ++r) {
        if (!regions[r]) return fail(HMMBW_E_INVALID, "null peer region");
        reg[(size_t)r] = static_cast<double *>(regions[r]);
    }
    if (int rc = set_device(c)) return rc;
    peer_detach(c);
    return peer_attach_impl(c, reg, n_seq_global);
}

int hmmbw_peer_open(hmmbw_ctx *c, const void *handles, int64_t n_seq_global) {
    if (!c || !handles) return fail(HMMBW_E_INVALID, "null argument");
    if (n_seq_global < 0) return fail(HMMBW_E_INVALID, "negative sequence count");
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    if (!c->d_peer || c->peer_world != c->world || c->peer_n != c->ar_payload())
        return fail(HMMBW_E_STATE, "no current peer region (hmmbw_peer_region first, after set_rank and options)");
    if (int rc = set_device(c)) return rc;
    peer_detach(c);
    std::vector<double *> reg((size_t)c->world, nullptr);
    const char *hb = static_cast<const char *>(handles);
    for (int r = 0; r < c->world; ++r) {
        if (r == c->rank) {
            reg[(size_t)r] = c->d_peer;
            continue;
        }
        hipIpcMemHandle_t h;
        std::memcpy(&h, hb + 64 * (size_t)r, sizeof(h));
        void *p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            peer_detach(c);
            return fail(HMMBW_E_HIP, "hipIpcOpenMemHandle (rank " + std::to_string(r) + "): " + hipGetErrorString(e));
        }
        c->peer_mapped.push_back(p);
        reg[(size_t)r] = static_cast<double *>(p);
    }
    return peer_attach_impl(c, reg, n_seq_global);
}

int hmmbw_allreduce_kind(const hmmbw_ctx *c, int *kind) {
    if (!c || !kind) return fail(HMMBW_E_INVALID, "null argument");
    if (c->peer_mode()) *kind = HMMBW_ALLREDUCE_PEER;
    else if (c->world > 1 || c->comm) *kind = HMMBW_ALLREDUCE_RCCL;
    else *kind = -1;
    return HMMBW_OK;
}

int hmmbw_iterate(hmmbw_ctx *c, int64_t n_iter) {
    if (int rc = check_ready(c, true)) return rc;
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    if (c->world != 1 || c->comm || c->peer_mode()) {
        // multi-rank with the engine's own all-reduce: estep -> ncclAllReduce (this stream) or the peer
        // push / wait + sum -> mstep
        const bool peer = c->peer_mode();
        if (c->ar_kind == HMMBW_ALLREDUCE_PEER && !peer) return fail(HMMBW_E_STATE, peer_off_msg(c));
        if (!peer && !c->comm)
            return fail(HMMBW_E_STATE, "multi-rank hmmbw_iterate needs hmmbw_comm_init or the peer all-reduce "
                                       "(or use hmmbw_iterate_begin / all-reduce / _end)");
        Rccl *r = nullptr;
        if (!peer)
            if (int rc = rccl_load(nullptr, &r)) return rc;
        for (int64_t i = 0; i < n_iter; ++i) {
            double *ar = nullptr;
            long long ar_len = 0;
            if (int rc = mr_begin(c, c->R_global, &ar, &ar_len)) return rc;
            // between mr_begin and mr_end: any failure closes the iteration again, or every later
            // training call would fail with HMMBW_E_STATE
            auto collective = [&]() -> int {
                hipEvent_t e0 = nullptr, e1 = nullptr;
                if (c->timing && (c->ar_seq++ % c->timing) == 0) {
                    if (int rc = take_events(c->ar_free, &e0, &e1)) return rc;
                    HIP_TRY(hipEventRecord(e0, c->stream));
                }
                // also at world 1 (RCCL's in-place 1-rank sum is a copy kernel, ~2 us): the 1-rank
                // communicator tests then exercise the same ncclAllReduce call as an 8-GPU run
                c->ar_len_last = ar_len;
                if (peer) {
                    if (int rc = peer_allreduce(c, ar, ar_len)) return rc;
                } else {
                    ncclResult_t e = r->all_reduce(ar, ar, (size_t)ar_len, ncclFloat64, ncclSum, c->comm, c->stream);
                    if (e != ncclSuccess) return rccl_fail(r, e, "ncclAllReduce");
                }
                if (e1) {
                    HIP_TRY(hipEventRecord(e1, c->stream));
                    c->ar_pending.push_back(e0);
                    c->ar_pending.push_back(e1);
                    if (c->ar_pending.size() >= 256)
                        if (int rc = drain_pairs(c->ar_pending, c->ar_free, &c->ar_ms, &c->ar_n)) return rc;
                }
                return HMMBW_OK;
            };
            if (int rc = collective()) {
                c->ar_open = false;
                return rc;
            }
            if (int rc = mr_end(c)) return rc;
        }
        return HMMBW_OK;
    }
    const long long nz = (long long)c->ncopies * c->copy_len();
    for (int64_t i = 0; i < n_iter; ++i) {
        if (c->pend.on && !c->can_merge())
            if (int rc = flush_mstep(c)) return rc;
        const long long e = c->e_count++;
        // statistics triple buffer: this launch adds into e, the merged M-step reads e - 1, and e + 1
        // (read by launch e - 2) is cleared for the next launch
        if (int rc = launch_estep(c, false, c->state(), c->copies(e), c->llpart(e), c->copies(e + 1), nz, true))
            return rc;
        hmmbw_ctx::Pending &p = c->pend;
        p.on = true;
        p.local = true;
        p.src = c->copies(e);
        p.nsrc = c->det ? 1 : c->ncopies;
        p.ll = c->llpart(e);
        p.nll = c->last_nll;
        p.ext = nullptr;
        p.R = c->R;
        if (!c->can_merge())
            if (int rc = flush_mstep(c)) return rc;
        if (c->timing && c->ev_pending.size() >= 256)
            if (int rc = drain_timing(c)) return rc;
    }
    return HMMBW_OK;
}

static void fill_status(const IterState &h, hmmbw_status *st) {
    st->iterations = h.iteration;
    st->done = h.done;
    st->converged = h.converged;
    st->last_log_likelihood = h.last_L;
    st->last_diff = h.last_diff;
}

int hmmbw_get_status(hmmbw_ctx *c, hmmbw_status *st, hmmbw_iter_record *rec, int64_t first, int64_t count) {
    if (!c || !st) return fail(HMMBW_E_INVALID, "null argument");
    if (int rc = set_device(c)) return rc;
    if (int rc = flush_mstep(c)) return rc;
    IterState h{};
    HIP_TRY(hipMemcpyAsync(&h, c->state(), sizeof(IterState), hipMemcpyDeviceToHost, c->stream));
    std::vector<double> hist(2 * (size_t)kHist);
    if (rec && count > 0)
        HIP_TRY(hipMemcpyAsync(hist.data(), c->d_hist, sizeof(double) * hist.size(), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    fill_status(h, st);
    if (h.error) return fail(h.error, device_error(h));
    if (rec && count > 0) {
        if (first < 0 || first + count > h.iteration || first < h.iteration - kHist)
            return fail(HMMBW_E_INVALID, "requested iteration records are not available");
        for (int64_t i = 0; i < count; ++i) {
            const int64_t k = (first + i) % kHist;
            rec[i].log_likelihood = hist[2 * k];
            rec[i].diff = hist[2 * k + 1];
        }
    }
    return HMMBW_OK;
}

int hmmbw_status_post(hmmbw_ctx *c, int64_t first, int64_t *ticket) {
    if (!c || !ticket) return fail(HMMBW_E_INVALID, "null argument");
    if (first < 0) return fail(HMMBW_E_INVALID, "negative first iteration");
    if (int rc = set_device(c)) return rc;
    hmmbw_ctx::Snap &sn = c->snaps[c->snap_next % 2];
    if (!sn.ev) {
        HIP_TRY(hipEventCreateWithFlags(&sn.ev, hipEventDisableTiming));
        // fine-grained host memory the snapshot kernel writes (visible once its event has completed)
        HIP_TRY(cached_alloc(reinterpret_cast<void **>(&sn.st), sizeof(IterState), kPinnedBlock));
        HIP_TRY(cached_alloc(reinterpret_cast<void **>(&sn.hist), sizeof(double) * 2 * (size_t)kHist, kPinnedBlock));
    } else {
        HIP_TRY(hipEventSynchronize(sn.ev));  // the slot's previous snapshot has landed (two posts ago)
    }
    // no flush: a pending (merged) M-step stays pending, so the snapshot holds the records of every
    // iteration enqueued so far except the last one
    hipLaunchKernelGGL(k_snapshot, dim3(1), dim3(256), 0, c->stream, c->state(), c->d_hist, (long long)first, sn.st,
                       sn.hist);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(sn.ev, c->stream));
    sn.first = first;
    sn.ticket = c->snap_next++;
    *ticket = sn.ticket;
    return HMMBW_OK;
}

int hmmbw_status_wait(hmmbw_ctx *c, int64_t ticket, hmmbw_status *st, hmmbw_iter_record *rec, int64_t first,
                      int64_t count) {
    if (!c || !st) return fail(HMMBW_E_INVALID, "null argument");
    if (ticket < 0 || ticket >= c->snap_next || ticket < c->snap_next - 2)
        return fail(HMMBW_E_INVALID, "status ticket is not one of the last two posted");
    if (int rc = set_device(c)) return rc;
    hmmbw_ctx::Snap &sn = c->snaps[ticket % 2];
    HIP_TRY(hipEventSynchronize(sn.ev));  // this snapshot only, not the work enqueued after it
    const IterState h = *sn.st;
    fill_status(h, st);
    if (h.error) return fail(h.error, device_error(h));
    if (rec && count > 0) {
        if (first < sn.first || first + count > h.iteration || first + count > sn.first + kHist ||
            first < h.iteration - kHist)  // overwritten in the ring before the snapshot was taken
            return fail(HMMBW_E_INVALID, "requested iteration records are not in this snapshot");
        for (int64_t i = 0; i < count; ++i) {
            const int64_t k = first + i - sn.first;
            rec[i].log_likelihood = sn.hist[2 * k];
            rec[i].diff = sn.hist[2 * k + 1];
        }
    }
    return HMMBW_OK;
}

int hmmbw_status_live_wait(hmmbw_ctx *c, int64_t iterations, hmmbw_status *st, hmmbw_iter_record *rec,
                           int64_t first, int64_t count) {
    if (!c || !st) return fail(HMMBW_E_INVALID, "null argument");
    if (!c->h_live) return fail(HMMBW_E_STATE, "HMMBW_OPT_LIVE_STATUS is off");
    if (int rc = set_device(c)) return rc;
    volatile LiveBlock *lv = c->h_live;
    IterState h{};
    bool have = false;
    for (long long spin = 0;; ++spin) {
        const unsigned long long p0 = lv->pub;
        std::atomic_thread_fence(std::memory_order_acquire);
        if ((unsigned)(p0 >> 32) == c->live_epoch) {
            const long long n = (long long)(unsigned)(p0 & 0xffffffffULL);
            const volatile IterState &sl = lv->slot[n & 1];
            h.prev_L = sl.prev_L;
            h.last_L = sl.last_L;
            h.last_diff = sl.last_diff;
            h.epsilon = sl.epsilon;
            h.iteration = sl.iteration;
            h.max_iterations = sl.max_iterations;
            h.done = sl.done;
            h.converged = sl.converged;
            h.error = sl.error;
            std::atomic_thread_fence(std::memory_order_acquire);
            const unsigned long long p1 = lv->pub;
            // the slot is rewritten only by the record after next: two publications apart
            const bool stable = (unsigned)(p1 >> 32) == c->live_epoch && (long long)(unsigned)(p1 & 0xffffffffULL) <= n + 1;
            if (stable && h.iteration == n && (n >= iterations || h.done)) {
                have = true;
                break;
            }
        }
        // the stream ran dry without the record (a pending M-step, a device-side stop the mirror does not
        // carry, or a reset): the device state is the answer
        if ((spin & 63) == 63 && hipStreamQuery(c->stream) == hipSuccess) {
            const unsigned long long p2 = lv->pub;
            if ((unsigned)(p2 >> 32) == c->live_epoch && (long long)(unsigned)(p2 & 0xffffffffULL) >= iterations) continue;
            break;
        }
    }
    std::vector<double> dh;
    if (!have) {
        HIP_TRY(hipMemcpy(&h, c->state(), sizeof(IterState), hipMemcpyDeviceToHost));
        if (rec && count > 0) {
            dh.resize(2 * (size_t)kHist);
            HIP_TRY(hipMemcpy(dh.data(), c->d_hist, sizeof(double) * dh.size(), hipMemcpyDeviceToHost));
        }
    }
    fill_status(h, st);
    if (h.error) return fail(h.error, device_error(h));
    if (rec && count > 0) {
        if (first < 0 || first + count > h.iteration || first < h.iteration - kHist)
            return fail(HMMBW_E_INVALID, "requested iteration records are not available");
        for (int64_t i = 0; i < count; ++i) {
            const int64_t k = (first + i) % kHist;
            rec[i].log_likelihood = have ? lv->hist[2 * k] : dh[2 * k];
            rec[i].diff = have ? lv->hist[2 * k + 1] : dh[2 * k + 1];
        }
    }
    return HMMBW_OK;
}

int hmmbw_get_params(hmmbw_ctx *c, double *pi, double *A, double *B, int normalise) {
    if (!c || !pi || !A || !B) return fail(HMMBW_E_INVALID, "null argument");
    if (!c->has_params) return fail(HMMBW_E_STATE, "parameters not set");
    if (int rc = set_device(c)) return rc;
    if (int rc = flush_mstep(c)) return rc;
    const size_t N = c->N, K = c->K;
    if (normalise) {
        hipLaunchKernelGGL(k_finalise, dim3(1), dim3(64), 0, c->stream, c->d_pi, c->d_A, c->d_B, c->N, c->K, c->d_out);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(pi, c->d_out, sizeof(double) * N, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(A, c->d_out + N, sizeof(double) * N * N, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(B, c->d_out + N + N * N, sizeof(double) * N * K, hipMemcpyDeviceToHost, c->stream));
    } else {
        HIP_TRY(hipMemcpyAsync(pi, c->d_pi, sizeof(double) * N, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(A, c->d_A, sizeof(double) * N * N, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(B, c->d_B, sizeof(double) * N * K, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return HMMBW_OK;
}

int hmmbw_get_loglik(hmmbw_ctx *c, double *out) {
    if (!c || !out) return fail(HMMBW_E_INVALID, "null argument");
    if (!c->has_obs) return fail(HMMBW_E_STATE, "observations not set");
    if (int rc = set_device(c)) return rc;
    if (c->R > 0)
        HIP_TRY(hipMemcpyAsync(out, c->d_logp, sizeof(double) * c->R, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return HMMBW_OK;
}

int hmmbw_score(hmmbw_ctx *c, double *out) {
    if (int rc = check_ready(c, false)) return rc;
    if (!out) return fail(HMMBW_E_INVALID, "null argument");
    if (c->ar_open) return fail(HMMBW_E_STATE, "an iteration is open (hmmbw_iterate_end first)");
    if (int rc = flush_mstep(c)) return rc;
    if (int rc = launch_estep(c, true, nullptr)) return rc;
    return hmmbw_get_loglik(c, out);
}

int hmmbw_timing(hmmbw_ctx *c, int enable, double *total_ms, int64_t *count) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (int rc = set_device(c)) return rc;
    if (int rc = drain_timing(c)) return rc;
    if (total_ms) *total_ms = c->timed_ms;
    if (count) *count = c->timed_n;
    if (enable >= 0) {
        c->timing = enable;
        c->timing_seq = 0;
        c->timed_ms = 0.0;
        c->timed_n = 0;
        c->timed_main_ms = 0.0;
        c->timed_main_n = 0;
    }
    return HMMBW_OK;
}

int hmmbw_timing_split(hmmbw_ctx *c, double *main_ms, int64_t *count) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (int rc = set_device(c)) return rc;
    if (int rc = drain_timing(c)) return rc;
    if (main_ms) *main_ms = c->timed_main_ms;
    if (count) *count = c->timed_main_n;
    return HMMBW_OK;
}



// ---------------------------------------------------------------------------------------------
// Groups: several single-rank contexts of one shape advanced by ONE grouped launch per EM iteration
// (k_estep_small_group).  The reference trains its word models one after another (HMM/main.py:147-152
// -> training_with_save, hmm_training.py:215-247) and scores every (recording, model) pair with its
// own forward pass (hmm_testing.py:139-161); a group does each in one launch.
// ---------------------------------------------------------------------------------------------
}  // extern "C"

struct hmmbw_group {
    std::vector<hmmbw_ctx *> m;
    // argument slabs ([n_launch][n] EArgs + [n_launch][n + 1] first-workgroup tables): pinned staging,
    // device copy, and the event after the last launch that reads it; reused round-robin
    struct Slab {
        char *host = nullptr, *dev = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;
    };
    std::vector<Slab> slabs;
    size_t next = 0;
    std::vector<hipEvent_t> ev_free, ev_pending;  // timing pairs (start, stop)
    int timing = 0;
    double timed_ms = 0.0;
    long long timed_n = 0, timing_seq = 0;
};

namespace {

int group_check(hmmbw_group *g, bool need_armed) {
    if (!g || g->m.empty()) return fail(HMMBW_E_INVALID, "null or empty group");
    hmmbw_ctx *c0 = g->m[0];
    for (hmmbw_ctx *c : g->m) {
        if (int rc = check_ready(c, need_armed)) return rc;
        if (c->world != 1) return fail(HMMBW_E_STATE, "group members are single-rank contexts");
        if (c->ar_open) return fail(HMMBW_E_STATE, "a group member has an open iteration (hmmbw_iterate_end first)");
        if (c->device != c0->device || c->stream != c0->stream)
            return fail(HMMBW_E_INVALID, "group members must share the device and the stream");
        if (c->N != c0->N || c->K != c0->K || c->topo != c0->topo || c->wide || !c->lds_tables())
            return fail(HMMBW_E_UNSUPPORTED, "group members must share N, M and topology (small-N path with LDS tables)");
    }
    return HMMBW_OK;
}

// Enqueue n_launch grouped launches; plans[l * n + i] is member i's plan for launch l.
int group_launch(hmmbw_group *g, const std::vector<Plan> &plans, int n_launch, bool timed) {
    const int n = (int)g->m.size();
    hipStream_t st = g->m[0]->stream;
    const size_t args_b = sizeof(EArgs) * (size_t)n, start_b = sizeof(long long) * (size_t)(n + 1);
    const size_t per = (args_b + start_b + 255) & ~(size_t)255;
    const size_t need = per * (size_t)n_launch;
    if (g->slabs.size() < 4) g->slabs.resize(4);
    hmmbw_group::Slab &sl = g->slabs[g->next];
    g->next = (g->next + 1) % g->slabs.size();
    if (sl.ev) HIP_TRY(hipEventSynchronize(sl.ev));  // its previous launches have read it
    else HIP_TRY(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
    if (sl.cap < need) {
        if (sl.host) HIP_TRY(hipHostFree(sl.host));
        if (sl.dev) {
            ledger_remove(sl.dev, "hipFree (group args)");
            HIP_TRY(hipFree(sl.dev));
        }
        sl.host = sl.dev = nullptr;
        sl.cap = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&sl.host), need));
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&sl.dev), need));
        ledger_add(sl.dev, need, "hipMalloc (group args)");
        sl.cap = need;
    }
    std::vector<unsigned> grid((size_t)n_launch, 0);
    size_t lds = 0;
    for (int l = 0; l < n_launch; ++l) {
        EArgs *A = reinterpret_cast<EArgs *>(sl.host + per * l);
        long long *S = reinterpret_cast<long long *>(sl.host + per * l + args_b);
        long long b = 0;
        for (int i = 0; i < n; ++i) {
            const Plan &p = plans[(size_t)l * n + i];
            A[i] = p.a;
            S[i] = b;
            b += p.grid;
            lds = std::max(lds, p.lds);
        }
        S[n] = b;
        grid[(size_t)l] = (unsigned)b;
    }
    HIP_TRY(hipMemcpyAsync(sl.dev, sl.host, need, hipMemcpyHostToDevice, st));
    const GroupFn f = plans[0].gfn;
    if (lds > 64 * 1024)
        HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
    for (int l = 0; l < n_launch; ++l) {
        if (grid[(size_t)l] == 0) continue;
        GroupArgs ga{reinterpret_cast<const EArgs *>(sl.dev + per * l),
                     reinterpret_cast<const long long *>(sl.dev + per * l + args_b), n};
        const bool t = timed && g->timing && (g->timing_seq++ % g->timing) == 0;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (t) {
            while (g->ev_free.size() < 2) {
                hipEvent_t x;
                HIP_TRY(hipEventCreate(&x));
                g->ev_free.push_back(x);
            }
            e1 = g->ev_free.back(); g->ev_free.pop_back();
            e0 = g->ev_free.back(); g->ev_free.pop_back();
            HIP_TRY(hipEventRecord(e0, st));
        }
        hipLaunchKernelGGL(f, dim3(grid[(size_t)l]), dim3(kBlock), lds, st, ga);
        HIP_TRY(hipGetLastError());
        if (t) {
            HIP_TRY(hipEventRecord(e1, st));
            g->ev_pending.push_back(e0);
            g->ev_pending.push_back(e1);
        }
    }
    HIP_TRY(hipEventRecord(sl.ev, st));
    return HMMBW_OK;
}

}  // namespace

extern "C" {

int hmmbw_comm_probe(const char *rccl_path) {
    Rccl *r = nullptr;
    return rccl_load(rccl_path, &r);
}

int hmmbw_comm_unique_id(const char *rccl_path, void *id_out) {
    if (!id_out) return fail(HMMBW_E_INVALID, "null argument");
    Rccl *r = nullptr;
    if (int rc = rccl_load(rccl_path, &r)) return rc;
    ncclUniqueId id;
    ncclResult_t e = r->get_unique_id(&id);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclGetUniqueId");
    std::memcpy(id_out, &id, sizeof(id));
    return HMMBW_OK;
}

int hmmbw_comm_init(hmmbw_ctx *c, const char *rccl_path, const void *id, int rank, int world, int64_t n_seq_global) {
    if (!c || !id) return fail(HMMBW_E_INVALID, "null argument");
    if (world < 1 || rank < 0 || rank >= world) return fail(HMMBW_E_INVALID, "need 0 <= rank < world");
    if (c->world != world || c->rank != rank) return fail(HMMBW_E_STATE, "hmmbw_set_rank first, with the same rank/world");
    if (n_seq_global < 0) return fail(HMMBW_E_INVALID, "negative sequence count");
    Rccl *r = nullptr;
    if (int rc = rccl_load(rccl_path, &r)) return rc;
    if (int rc = set_device(c)) return rc;
    if (c->comm) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        (void)r->comm_destroy(c->comm);
        c->comm = nullptr;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    ncclResult_t e = r->comm_init_rank(&comm, world, uid, rank);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclCommInitRank");
    sync_ctx(c);
    dfree(c->d_ext);
    if (int rc = dalloc(&c->d_ext, (size_t)c->stats_len())) {
        (void)r->comm_destroy(comm);
        return rc;
    }
    HIP_TRY(hipMemset(c->d_ext, 0, sizeof(double) * (size_t)c->stats_len()));
    c->ext_len = c->stats_len();
    c->comm = comm;
    c->R_global = n_seq_global;
    return HMMBW_OK;
}

int hmmbw_comm_payload(const hmmbw_ctx *c, int64_t *n_doubles) {
    if (!c || !n_doubles) return fail(HMMBW_E_INVALID, "null argument");
    *n_doubles = c->ar_len_last;
    return HMMBW_OK;
}

int hmmbw_comm_info(hmmbw_ctx *c, int *n_ranks, double *total_ms, int64_t *count, int reset) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (int rc = set_device(c)) return rc;
    int n = 0;
    if (c->comm) {
        Rccl *r = nullptr;
        if (int rc = rccl_load(nullptr, &r)) return rc;
        n = -1;  // communicator exists but this RCCL has no ncclCommCount
        if (r->comm_count) {
            ncclResult_t e = r->comm_count(c->comm, &n);
            if (e != ncclSuccess) return rccl_fail(r, e, "ncclCommCount");
        }
    }
    if (int rc = drain_pairs(c->ar_pending, c->ar_free, &c->ar_ms, &c->ar_n)) return rc;
    if (n_ranks) *n_ranks = n;
    if (total_ms) *total_ms = c->ar_ms;
    if (count) *count = c->ar_n;
    if (reset) {
        c->ar_ms = 0.0;
        c->ar_n = 0;
        c->ar_seq = 0;
    }
    return HMMBW_OK;
}

int hmmbw_vq_encode(void *stream, const double *frames, int64_t n_frames, int frame_stride, int first_dim, int dims,
                    const double *centroids, int n_centroids, int32_t *symbols, double *distances) {
    if (n_frames < 0) return fail(HMMBW_E_INVALID, "negative frame count");
    if (n_frames == 0) return HMMBW_OK;
    if (!frames || !centroids || !symbols) return fail(HMMBW_E_INVALID, "null argument");
    if (dims < 1 || dims > 64 || first_dim < 0 || frame_stride < first_dim + dims)
        return fail(HMMBW_E_INVALID, "need 1 <= dims <= 64 and first_dim + dims <= frame_stride");
    if (n_centroids < 1) return fail(HMMBW_E_INVALID, "empty codebook");
    if ((long long)n_centroids * dims > 20480) return fail(HMMBW_E_UNSUPPORTED, "codebook larger than 160 KiB of LDS");
    if (n_frames > (1LL << 40)) return fail(HMMBW_E_UNSUPPORTED, "too many frames");
    hipError_t e = launch_vq(reinterpret_cast<hipStream_t>(stream), frames, n_frames, frame_stride, first_dim, dims,
                             centroids, n_centroids, symbols, distances);
    if (e != hipSuccess) return fail(HMMBW_E_HIP, std::string("vq launch: ") + hipGetErrorString(e));
    return HMMBW_OK;
}

int hmmbw_group_create(hmmbw_ctx *const *ctxs, int n, hmmbw_group **out) {
    if (!out || (!ctxs && n > 0)) return fail(HMMBW_E_INVALID, "null argument");
    if (n <= 0) return fail(HMMBW_E_INVALID, "a group needs at least one context");
    *out = nullptr;
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i]) return fail(HMMBW_E_INVALID, "null context in group");
        for (int k = 0; k < i; ++k)
            if (ctxs[k] == ctxs[i]) return fail(HMMBW_E_INVALID, "a context appears twice in the group");
    }
    hmmbw_group *g = new hmmbw_group();
    g->m.assign(ctxs, ctxs + n);
    if (int rc = group_check(g, false)) {  // members must be set up and of one groupable shape
        delete g;
        return rc;
    }
    *out = g;
    return HMMBW_OK;
}

int hmmbw_group_destroy(hmmbw_group *g) {
    if (!g) return HMMBW_OK;
    if (!g->m.empty()) (void)hipSetDevice(g->m[0]->device);
    for (auto &sl : g->slabs) {
        if (sl.ev) {
            (void)hipEventSynchronize(sl.ev);
            (void)hipEventDestroy(sl.ev);
        }
        if (sl.host) (void)hipHostFree(sl.host);
        if (sl.dev) {
            ledger_remove(sl.dev, "hipFree (group args)");
            (void)hipFree(sl.dev);
        }
    }
    for (hipEvent_t e : g->ev_free) (void)hipEventDestroy(e);
    for (hipEvent_t e : g->ev_pending) (void)hipEventDestroy(e);
    delete g;
    return HMMBW_OK;
}

int hmmbw_group_iterate(hmmbw_group *g, int64_t n_iter) {
    if (int rc = group_check(g, true)) return rc;
    if (n_iter <= 0) return HMMBW_OK;
    const int n = (int)g->m.size();
    constexpr int64_t kBatch = 64;  // launches per argument slab
    std::vector<Plan> plans;
    for (int64_t i0 = 0; i0 < n_iter; i0 += kBatch) {
        const int nl = (int)std::min<int64_t>(kBatch, n_iter - i0);
        plans.assign((size_t)nl * n, Plan{});
        // Members whose M-step cannot run in the E-step prologue need their own M-step kernel
        // between two grouped launches; then the batch is one launch at a time.
        bool all_merge = true;
        for (hmmbw_ctx *c : g->m) all_merge = all_merge && c->can_merge();
        const int step = all_merge ? nl : 1;
        for (int l0 = 0; l0 < nl; l0 += step) {
            for (int l = l0; l < l0 + step; ++l)
                for (int i = 0; i < n; ++i) {
                    hmmbw_ctx *c = g->m[(size_t)i];
                    if (c->pend.on && !c->can_merge())
                        if (int rc = flush_mstep(c)) return rc;
                    const long long e = c->e_count++;
                    const long long nz = (long long)c->ncopies * c->copy_len();
                    Plan &p = plans[(size_t)l * n + i];
                    if (int rc = plan_estep(c, false, c->state(), c->copies(e), c->llpart(e), c->copies(e + 1), nz,
                                            true, &p, nullptr, 0, false))
                        return rc;
                    if (!p.gfn || p.gfn != plans[0].gfn || p.block != kBlock)
                        return fail(HMMBW_E_UNSUPPORTED, "group members need the same grouped kernel");
                    if (p.flip) c->scur ^= 1;  // slots are read by the launch through the plan's pointers
                    hmmbw_ctx::Pending &q = c->pend;
                    q.on = true;
                    q.local = true;
                    q.src = c->copies(e);
                    q.nsrc = c->ncopies;
                    q.ll = c->llpart(e);
                    q.nll = c->nblocks;
                    q.ext = nullptr;
                    q.R = c->R;
                }
            if (step == nl) {
                if (int rc = group_launch(g, plans, nl, true)) return rc;
            } else {
                std::vector<Plan> one(plans.begin() + (size_t)l0 * n, plans.begin() + (size_t)(l0 + 1) * n);
                if (int rc = group_launch(g, one, 1, true)) return rc;
                for (hmmbw_ctx *c : g->m)
                    if (!c->can_merge())
                        if (int rc = flush_mstep(c)) return rc;
            }
        }
    }
    return HMMBW_OK;
}

int hmmbw_group_score(hmmbw_group *g, double *out) {
    if (int rc = group_check(g, false)) return rc;
    if (!out) return fail(HMMBW_E_INVALID, "null argument");
    const int n = (int)g->m.size();
    std::vector<Plan> plans((size_t)n);
    for (int i = 0; i < n; ++i) {
        hmmbw_ctx *c = g->m[(size_t)i];
        if (int rc = flush_mstep(c)) return rc;
        if (int rc = plan_estep(c, true, nullptr, nullptr, nullptr, nullptr, 0, false, &plans[(size_t)i]))
            return rc;
        if (!plans[(size_t)i].gfn || plans[(size_t)i].gfn != plans[0].gfn)
            return fail(HMMBW_E_UNSUPPORTED, "group members need the same grouped kernel");
    }
    if (int rc = group_launch(g, plans, 1, false)) return rc;
    long long off = 0;
    for (hmmbw_ctx *c : g->m) {
        if (c->R > 0)
            HIP_TRY(hipMemcpyAsync(out + off, c->d_logp, sizeof(double) * c->R, hipMemcpyDeviceToHost, c->stream));
        off += c->R;
    }
    HIP_TRY(hipStreamSynchronize(g->m[0]->stream));
    return HMMBW_OK;
}

int hmmbw_group_timing(hmmbw_group *g, int enable, double *total_ms, int64_t *count) {
    if (!g || g->m.empty()) return fail(HMMBW_E_INVALID, "null or empty group");
    if (int rc = set_device(g->m[0])) return rc;
    for (size_t i = 0; i + 1 < g->ev_pending.size(); i += 2) {
        HIP_TRY(hipEventSynchronize(g->ev_pending[i + 1]));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, g->ev_pending[i], g->ev_pending[i + 1]));
        g->timed_ms += ms;
        g->timed_n += 1;
        g->ev_free.push_back(g->ev_pending[i]);
        g->ev_free.push_back(g->ev_pending[i + 1]);
    }
    g->ev_pending.clear();
    if (total_ms) *total_ms = g->timed_ms;
    if (count) *count = g->timed_n;
    if (enable >= 0) {
        g->timing = enable;
        g->timing_seq = 0;
        g->timed_ms = 0.0;
        g->timed_n = 0;
    }
    return HMMBW_OK;
}

}  // extern "C"
