// hmmbw_device.hpp — device code of the MI355X Baum-Welch engine (kernels, reductions, M-step
// building blocks), shared by the host translation unit (hmmbw.hip) and the per-N instantiation
// units (estep_small_inst.hip, estep_wide_inst.hip) that the build compiles in parallel.
// See hmmbw.hip for the kernel map and DESIGN.md for the numerics.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/hmmbw.h"

namespace hmmbw {

// Diagnostics build only (-DHMMBW_PHASE_TIMES, tools/phase_times.py): per-wave wall-clock stamps of
// the small E-step's phases, read back with hmmbw_debug_phase_times.
#ifdef HMMBW_PHASE_TIMES
constexpr int kPhaseWaves = 1 << 16;
constexpr int kPhaseSlots = 16;
static __device__ unsigned long long g_phase[kPhaseWaves][kPhaseSlots];
#define PHASE(k)                                                                               \
    do {                                                                                       \
        const long long w_ = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);   \
        if ((threadIdx.x & 63) == 0 && w_ < kPhaseWaves) g_phase[w_][k] = wall_clock64();      \
    } while (0)
// diagnostics: where the wave runs: HW_ID (wave, SIMD, CU, shader array, engine fields) in slot 15, XCC_ID
// in slot 14
#define PHASE_HWID()                                                                                    \
    do {                                                                                                \
        const long long w_ = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);            \
        if ((threadIdx.x & 63) == 0 && w_ < kPhaseWaves) {                                              \
            g_phase[w_][15] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);                      \
            g_phase[w_][14] = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20);                     \
        }                                                                                               \
    } while (0)
// diagnostics: wait for every outstanding memory operation of the wave, then stamp
#define PHASE_DRAIN(k)                   \
    do {                                 \
        __builtin_amdgcn_s_waitcnt(0);   \
        PHASE(k);                        \
    } while (0)
// shader-clock stamp at the start of forward (d = 0) / backward (d = 1) chunk c (c < 64); only with
// -DHMMBW_CHUNK_TIMES too: its conditional stores inside the sweeps change their s_waitcnt placement
static __device__ unsigned long long g_chunk[4096][2][64];
#ifdef HMMBW_CHUNK_TIMES
#define CHUNKSTAMP(d, c)                                                                       \
    do {                                                                                       \
        const long long w_ = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);   \
        if ((threadIdx.x & 63) == 0 && w_ < 4096 && (c) < 64) g_chunk[w_][d][c] = clock64();   \
    } while (0)
#else
#define CHUNKSTAMP(d, c) \
    do {                 \
    } while (0)
#endif
#else
#define CHUNKSTAMP(d, c) \
    do {                 \
    } while (0)
#define PHASE(k) \
    do {         \
    } while (0)
#define PHASE_HWID() \
    do {             \
    } while (0)
#define PHASE_DRAIN(k) \
    do {               \
    } while (0)
#endif

// 1: the dense path's stored z_t (written once, read once) nontemporal.  Measured worse (cfg3 dense 79.7-80.5
// against 73.6-73.8 us): the backward reads them back while the caches still hold them.
#ifndef HMMBW_ZF_NT
#define HMMBW_ZF_NT 0
#endif

constexpr int kWave = 64;
constexpr int kChunk = 8;  // time steps per packed symbol load (8 x uint16 = 16 B)
#ifndef HMMBW_KSCALE
#define HMMBW_KSCALE 8
#endif
constexpr int kScale = HMMBW_KSCALE;  // lagged mode: the forward rescales every kScale steps
constexpr int kHist = 4096;
constexpr int kBlock = 256;  // threads per E-step workgroup (4 waves)

struct IterState {
    double prev_L;
    double last_L;
    double last_diff;
    double epsilon;
    long long iteration;
    long long max_iterations;
    int done;
    int converged;
    int error;      // HMMBW_E_* of a device-side failure; done is set with it
    int error_src;  // which bounded wait failed: kErrPeer (peer all-reduce) or kErrWorkQueue (wide work queue)
};
constexpr int kErrPeer = 1;
constexpr int kErrWorkQueue = 2;

// Observation layout in HBM (built once by hmmbw_set_observations).
//   slot = wave * U + u  ->  caller sequence slot_seq[slot] (-1: padding), length slot_len[slot]
//   sym    : per wave, chunk-major [chunk][u][8] uint16  (one 16-B load = 8 steps of one sequence)
//   ckpt   : per wave [chunk][64 lanes] fp64 — alpha_hat at the first step of every chunk (small N)
//   spack  : per wave [chunk][u] 8 x int16 — the power-of-two scale exponent of every step
//   alpha  : per wave [t][64 lanes] fp64 + ebuf [t][u] int32 — full alpha_hat (wide kernel only)
struct Layout {
    const uint16_t *sym;
    const long long *wave_symoff;
    const long long *wave_ckoff;   // doubles (small) | alpha doubles (wide)
    const long long *wave_spoff;   // uint4 units (small) | ebuf ints (wide)
    const int *wave_T;
    const int *wave_full;          // 1: every real slot of the wave has length wave_T
    const int *slot_len;
    const int *slot_seq;
    long long nwaves;
};

// Host-visible mirror of the convergence state (HMMBW_OPT_LIVE_STATUS), in fine-grained pinned host
// memory: every M-step that records an iteration also writes the record and the new state here with
// write-through stores, then publishes pub = epoch << 32 | iteration.  The state goes to slot
// iteration % 2, so a reader that sees pub unchanged around its copy of that slot read one record.
struct LiveBlock {
    unsigned long long pub;
    unsigned long long pad_[7];
    IterState slot[2];
    double hist[2 * kHist];  // (L, diff) of iteration i at 2 (i % kHist)
};

struct MArgs {
    const double *src;     // statistics: the copies (single rank) or the all-reduced buffer
    double *zero_ll;       // LL slots to clear (multi-rank) or nullptr
    int nsrc;
    long long copy_len;
    double *pi, *A, *B, *Bt;
    const double *llpart;
    long long nblocks;
    long long R_global;
    const IterState *state;  // convergence state entering this M-step
    IterState *state_out;    // ... and after it (double-buffered: the host flips the slots per M-step)
    double *hist;
    int N, K, G, world;
    int local_lse;
    int bt_perm;           // 1: B^T columns in the wide kernels' order (wide_col)
    long long off_S, off_gex, off_gall, off_bnum, off_ll;
    LiveBlock *live;       // HMMBW_OPT_LIVE_STATUS: the host mirror (or nullptr)
    unsigned live_epoch;   // the host's reset count: records of an earlier run never match
};

struct EArgs {
    Layout L;
    const double *pi;
    const double *A;
    const double *Bt;  // [K][G] + G zero pad
    double *ckpt;      // small: checkpoints | wide: alpha_hat
    double *gam;       // wide: gamma rows [position][NP] (bt_col order) for k_bnum_gather
    const unsigned *gdst;  // wide: row of position (tile row = wave_ckoff / NP + t * 16 + s) in symbol order
    uint4 *spack;      // small: scale exponents
    int *ebuf;         // wide: scale exponents
    double *copies;    // [ncopies][copy_len] statistics accumulators (workgroup b adds into copy b % ncopies)
    long long copy_len;
    int ncopies;
    double *logp;
    double *llpart;    // [blocks][2]: per-block (max, sum exp) of log P
    const IterState *state;
    int K;
    int N;
    int force_safe;    // 1: per-step normalisation (no lagged scaling)
    int ablate;        // diagnostics only: bit 0 skips the statistics flush, bit 1 the backward sweep
    int merged;        // 1: run the previous iteration's M-step (m) in the prologue of every workgroup
    double *zero;      // statistics buffer of the NEXT iteration, cleared by this launch (or nullptr)
    long long zero_len;
    double *part;      // deterministic mode: per-workgroup partial statistics [blocks][off_bnum]
    double *rank_ll;   // multi-rank fused: this rank's (max, sum exp) slot in the all-reduce buffer (or nullptr)
    int *done_ctr;     // ... and the workgroup completion counter that picks the workgroup forming it
    MArgs m;
    long long off_S, off_gex, off_gall, off_bnum;
    // wave -> workgroup map of the small kernels: workgroups [0, nfull) run 4 sequence-group waves each,
    // the workgroups after them only xact (the waves beyond one per SIMD spread over more CUs)
    long long nfull;
    int xact;
    // wave priority (HMMBW_PRIO overrides): 2 (default) = s_setprio 1 for the spread map's extra waves, the
    // second wave on their SIMDs (cfg3 34.5-34.7 us per iteration against 36.0-36.8 at 0, two interleaved
    // rounds; no effect without extra waves, e.g. 12,500 sequences); 1 = for the full workgroups' waves
    int prio;
    // split extra waves (small kernels, LDS tables): the idle waves of the spread map's extra workgroups run
    // the lower half of their partner's backward sweep (estep_small_body, "split"); 0 off
    int split_extra;
    // wide work queue (k_estep_mfma<..., WQ>): [0] next unit, [1] workgroups done; per-tile forward flags
    unsigned *wq;
    unsigned *wq_flag;
    int wq_units;  // tiles
    long long wq_timeout_ticks;  // bound (wall-clock ticks) of a backward unit's wait for its forward
};

// Grouped launch (k_estep_small_group): per-model arguments and first workgroups (start[nm] = grid)
struct GroupArgs {
    const EArgs *__restrict__ args;
    const long long *__restrict__ start;
    int nm;
};

// ---------------------------------------------------------------------------------------------
// Cross-lane helpers (DPP on gfx950; 64-bit operands are split or use v_mov_b64_dpp)
// ---------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    long long x = __builtin_bit_cast(long long, v);
    x = __builtin_amdgcn_update_dpp(0ll, x, CTRL, 0xF, 0xF, true);
    return __builtin_bit_cast(double, x);
}

template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}

// lane ^ 16 / lane ^ 32 partners of a double without LDS: v_permlane16_swap / v_permlane32_swap (VALU) on
// both halves.  Each returns (own, partner) in an order that depends on the row, so combine the pair with a
// commutative operation only (every lane of the pair then gets the bitwise-identical result).
template <bool P32>
__device__ __forceinline__ void swap_pair(double v, double &a, double &b) {
    const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
    const auto l = P32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                       : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = P32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                       : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a = __hiloint2double((int)h[0], (int)l[0]);
    b = __hiloint2double((int)h[1], (int)l[1]);
}
template <bool P32>
__device__ __forceinline__ double add_swap(double v) {
    double a, b;
    swap_pair<P32>(v, a, b);
    return a + b;
}
template <bool P32>
__device__ __forceinline__ double max_swap(double v) {
    double a, b;
    swap_pair<P32>(v, a, b);
    return fmax(a, b);
}

// Sum over a group of G lanes (butterfly; every lane gets the bitwise-identical result because
// each level adds the same two partial sums, only commuted).  No LDS round trip: DPP within a row,
// permlane swaps across rows (round 6: the ds_bpermute of __shfl_xor cost ~120 cycles per level).
template <int G>
__device__ __forceinline__ double gsum(double x) {
    if constexpr (G >= 2) x += dpp<0xB1>(x);   // quad_perm [1,0,3,2]
    if constexpr (G >= 4) x += dpp<0x4E>(x);   // quad_perm [2,3,0,1]
    if constexpr (G >= 8) x += dpp<0x141>(x);  // row_half_mirror
    if constexpr (G >= 16) x += dpp<0x140>(x); // row_mirror
    if constexpr (G >= 32) x = add_swap<false>(x);
    if constexpr (G >= 64) x = add_swap<true>(x);
    return x;
}

// Sum over the lanes of a wave that share (lane mod G), e.g. the U sequences of a G-lane-group layout: the
// result is complete in every lane (the order of the additions may differ between lanes).
template <int G>
__device__ __forceinline__ double usum(double x) {
    if constexpr (G <= 2) x += __shfl_xor(x, 2);
    if constexpr (G <= 4) x += dpp<0x124>(x);   // row_ror:4
    if constexpr (G <= 8) x += dpp<0x128>(x);   // row_ror:8
    if constexpr (G <= 16) x = add_swap<false>(x);
    return add_swap<true>(x);
}

// min over the lanes of a wave that share (lane mod G), ints (DPP in the row, permlane swaps across rows)
template <int G>
__device__ __forceinline__ int umin_i32(int x) {
    if constexpr (G <= 2) x = min(x, __shfl_xor(x, 2));
    if constexpr (G <= 4) x = min(x, dpp_i32<0x124>(x));  // row_ror:4
    if constexpr (G <= 8) x = min(x, dpp_i32<0x128>(x));  // row_ror:8
    if constexpr (G <= 16) {
        const auto r = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
        x = min((int)r[0], (int)r[1]);
    }
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
    return min((int)r[0], (int)r[1]);
}

template <int G>
__device__ __forceinline__ int gmax_i32(int e) {
    if constexpr (G >= 2) e = max(e, dpp_i32<0xB1>(e));
    if constexpr (G >= 4) e = max(e, dpp_i32<0x4E>(e));
    if constexpr (G >= 8) e = max(e, dpp_i32<0x141>(e));
    if constexpr (G >= 16) e = max(e, dpp_i32<0x140>(e));
    return e;
}

// Exponent that steers the power-of-two scaling: frexp exponent of the group's largest entry
// (entries are >= 0), kZeroExp when the whole group is zero.
constexpr int kZeroExp = -8192;
template <int G>
__device__ __forceinline__ int group_exp(double z) {
    return gmax_i32<G>(z > 0.0 ? __builtin_amdgcn_frexp_exp(z) : kZeroExp);
}

// Value of lane I of this lane's G-group.
template <int G, int I>
__device__ __forceinline__ double gbcast(double v, int lane) {
    if constexpr (G == 2) {
        return dpp<(I) | ((I) << 2) | ((2 + I) << 4) | ((2 + I) << 6)>(v);
    } else if constexpr (G == 4) {
        return dpp<(I) * 0x55>(v);
    } else if constexpr (G == 8) {
        const double lo = dpp<0x150 + I>(v);
        const double hi = dpp<0x150 + 8 + I>(v);
        return (lane & 8) ? hi : lo;
    } else {
        static_assert(G == 16, "group size");
        return dpp<0x150 + I>(v);  // row_newbcast:I
    }
}

template <int B, int E, class F>
__device__ __forceinline__ void sfor(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}

// Dense-A cross-lane products with the broadcast fused into the multiply-add: gfx950's 64-bit DPP
// ("DP ALU DPP") has only row_newbcast, which broadcasts lane L of every 16-lane row, so for G-lane
// groups (G = 4, 8, 16) one v_fmac_f64_dpp per group position Q, with bank_mask restricting the write
// to that group's lanes, gives  acc += z(lane I of this lane's group) * a  in 16 / G instructions, in
// place of a broadcast, a select and an fma per group (the compiler does not fuse 64-bit DPP moves).
template <int G, int I, int Q>
__device__ __forceinline__ void fmac_bcast1(double &acc, double z, double a) {
    constexpr int lane = Q * G + I;
    constexpr int bm = ((1 << (G / 4)) - 1) << (Q * G / 4);
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:%4"
                 : "+v"(acc) : "v"(z), "v"(a), "i"(lane), "i"(bm));
}
// VALU write -> DPP read of that VGPR needs 2 wait states; the compiler does not see the DPP read
// inside the asm, so the first fused product after z is written goes behind this.
__device__ __forceinline__ void dpp_guard(double z) { asm volatile("s_nop 1" ::"v"(z)); }

// acc0 += sum over even i of a[i] z(lane i), acc1 the odd i (two chains), per G-lane group.  (Four
// chains, i mod 4, measured slower at dense cfg3: 76-77 against 71-73 us, profiles/r5/ab_dense_dot4.txt.)
template <int G, int N>
__device__ __forceinline__ void bcast_dot(double &acc0, double &acc1, double z, const double (&a)[N]) {
    dpp_guard(z);
    sfor<0, (N + 1) / 2>([&](auto P) {
        constexpr int i0 = 2 * decltype(P)::value, i1 = i0 + 1;
        sfor<0, 16 / G>([&](auto Q) {
            fmac_bcast1<G, i0, decltype(Q)::value>(acc0, z, a[i0]);
            if constexpr (i1 < N) fmac_bcast1<G, i1, decltype(Q)::value>(acc1, z, a[i1]);
        });
    });
}

// Dense xi partial sums of a G = 8 wave (lane = 8 u + j) on the 4x4x4 f64 MFMA: its block is lane
// bits 2-3, A lane 16k + 4blk + m holds A[m][k], B lane 16k + 4blk + n holds B[k][n], D lane
// 16m + 4blk + n holds D[m][n] (tools/ubench_mfma4.hip, profiles/r3/ubench_mfma4x4x4.txt).  With
// z as A and v as B, block (j >> 2, u & 1) sums over the seqs u >> 1:
//   X[0] lane 16m + 4jh + 8u0 + n:  sum z_t(4jh + m) v_{t+1}(4jh + n)            (diagonal 4x4 blocks)
//   X[1] with v row_half_mirrored (state j -> 7 - j):  ... v_{t+1}(4(1 - jh) + 3 - n)  (off-diagonal)
// The accumulation is off the forward/backward chains, so the MFMA's ~44-cycle SrcC latency is
// hidden; it replaces 16 v_fmac_f64_dpp per step (bcast_acc).
__device__ __forceinline__ void xi_mfma8(double (&X)[2], double zs, double vd) {
    X[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(zs, vd, X[0], 0, 0, 0);
    X[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(zs, dpp<0x141>(vd), X[1], 0, 0, 0);  // row_half_mirror
}

// S[i] += z(lane i) * w for every state i of the group
template <int G, int N, int NS>
__device__ __forceinline__ void bcast_acc(double (&S)[NS], double z, double w) {
    dpp_guard(z);
    sfor<0, 16 / G>([&](auto Q) {
        sfor<0, N>([&](auto I) { fmac_bcast1<G, decltype(I)::value, decltype(Q)::value>(S[decltype(I)::value], z, w); });
    });
}

__device__ __forceinline__ int sym_of(const uint4 &p, int s) {
    const unsigned w = s < 2 ? p.x : (s < 4 ? p.y : (s < 6 ? p.z : p.w));
    return (s & 1) ? int(w >> 16) : int(w & 0xFFFFu);
}

__device__ __forceinline__ int exp_of(const uint4 &p, int s) {  // signed int16 lanes of a pack
    const unsigned w = s < 2 ? p.x : (s < 4 ? p.y : (s < 6 ? p.z : p.w));
    return (s & 1) ? int((int)w >> 16) : int((int)(w << 16) >> 16);
}

__device__ __forceinline__ uint4 pack_exps(const int *e) {
    uint4 p;
    p.x = (unsigned)(e[0] & 0xFFFF) | ((unsigned)e[1] << 16);
    p.y = (unsigned)(e[2] & 0xFFFF) | ((unsigned)e[3] << 16);
    p.z = (unsigned)(e[4] & 0xFFFF) | ((unsigned)e[5] << 16);
    p.w = (unsigned)(e[6] & 0xFFFF) | ((unsigned)e[7] << 16);
    return p;
}

__device__ __forceinline__ double pow2_scale(double x, int e) { return __builtin_amdgcn_ldexp(x, -e); }

// 32-bit LDS byte address of a pointer into shared memory, and back (kept in one VGPR instead of
// being re-derived from its parts)
typedef __attribute__((address_space(3))) char lds_char;
__device__ __forceinline__ unsigned lds_addr(const char *p) {
    return (unsigned)(size_t)(const lds_char *)p;
}
__device__ __forceinline__ char *lds_ptr(unsigned a) {
    return (char *)(lds_char *)(size_t)a;
}

// Per-block (max, sum exp(x - max)) of the sequences' log P (each sequence contributes from
// exactly one lane with valid = true).  All threads of the block call it.
__device__ __forceinline__ double wave_max(double x);
__device__ __forceinline__ void block_ll_partial(double lp, bool valid, double *sh, double *out) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
    double m = wave_max(valid ? lp : -INFINITY);
    if (lane == 0) sh[wv] = m;
    __syncthreads();
    double M = -INFINITY;
    for (int w = 0; w < nw; ++w) M = fmax(M, sh[w]);
    const double s = gsum<64>((valid && M != -INFINITY && lp != -INFINITY) ? exp(lp - M) : 0.0);
    __syncthreads();
    if (lane == 0) sh[wv] = s;
    __syncthreads();
    if (tid == 0) {
        double S = 0.0;
        for (int w = 0; w < nw; ++w) S += sh[w];
        // memory-side atomics: the fused M-step of the last workgroup reads these with atomics too
        atomicExch(&out[0], (S > 0.0) ? M : 0.0);
        atomicExch(&out[1], S);
    }
}

// ---------------------------------------------------------------------------------------------
// Small-N E-step / scorer.  One G-lane group per sequence (lane j = state j), 64/G per wave.
//
// Forward: z_t = alpha_t / 2^{C_t}, C_t = s_0 + ... + s_t.  In the default (lagged) mode only every
// kScale-th step rescales, by s_t = M_{t-kScale} - 1023 with M = the biased exponent of the group's
// largest entry measured kScale steps earlier, so the per-step dependency chain is just
// (DPP shift || multiply) -> fma; the scaling itself is folded into the emission factor
// b_j(o_t) * 2^{-s_t} (exact).  If a wave's magnitudes ever leave [2^-900, 2^900]
// (pathological parameters) the wave re-runs its forward in the safe mode, which normalises every
// step by its own group maximum.  Only z at the first step of every 8-step chunk (the checkpoint)
// and the s_t are stored; the backward sweep recomputes each chunk's z_t in registers with the
// identical instruction sequence (bit-identical), so alpha never round-trips through HBM.
//
// Backward (Rabiner scaling with c_t = 2^{s_t}): beta_hat_{T-1} = 1/phat, phat = sum_j z_{T-1}(j);
//   v_j = b_j(o_{t+1}) 2^{-s_{t+1}} beta_hat_{t+1}(j),  beta_hat_t(i) = sum_j a_ij v_j,
//   gamma_t(i) = z_t(i) beta_hat_t(i),  xi_t(i,j) = a_ij z_t(i) v_j  (accumulated as S_ij = xi/a_ij).
// gamma is scattered into the per-workgroup LDS histogram B_num[o_t][j] (ds_add_f64).
// ---------------------------------------------------------------------------------------------
// LDS emission tables of the small kernels: two [K x GP] tables of 16-byte entries (GP = G + kTabPad
// columns, the columns past N zero), the second kHistOff bytes after the first:
//   P-table {x, y}: left-to-right x = a_jj b_j(o), y = a_{j-1,j} b_j(o) (the two products of the
//                   forward step); dense x = b_j(o), y = 0;
//   H-table {h, b}: h = the workgroup's B-numerator histogram (hmm_training.py:474-485), b = b_j(o).
// The symbol packs hold the byte offset of the symbol's row, o * GP * 16, so ONE lane address per step
// serves the emission read (ds_read_b128, offset 0) and the histogram add (ds_add_f64, offset
// kHistOff): the constant distance is the instructions' immediate offset.
// Rows are 8 x 16 B for G = 8 (no pad column): a ds_read_b128 lane group (4 windows of 4 states of 4
// sequences) then meets 1.74 bank conflicts per 16 lanes on uniform symbols, against 2.44 with a pad
// column (simulated with the MI355X_MICROARCH.md grouping; tools/lds_banks.py).  Padding slots of
// ragged waves read row 0 (any finite entry: their steps are masked and add 0 to the histogram).
#ifndef HMMBW_TAB_PAD
#define HMMBW_TAB_PAD 0
#endif
constexpr int kTabPad = HMMBW_TAB_PAD;
#ifndef HMMBW_XI_MFMA
#define HMMBW_XI_MFMA 1
#endif
#ifndef HMMBW_ZFULL
#define HMMBW_ZFULL 1
#endif
#ifndef HMMBW_FLUSH_VMWAIT  // explicit vmcnt(0) before the histogram flush (round 6 A/B)
#define HMMBW_FLUSH_VMWAIT 1
#endif
#ifndef HMMBW_SPLIT_LR  // split extra waves in the left-to-right kernels too (the host enables them on the joined map)
#define HMMBW_SPLIT_LR 1
#endif
#ifndef HMMBW_KARG_TOUCH  // touch every line of the kernel arguments at entry, in one batch (round 6 A/B)
#define HMMBW_KARG_TOUCH 1
#endif

// The prologue reads the kernel arguments in several dependent rounds (the zero loop's, then the M-step's, then
// the launch map's), and the first read of each 64-B line of the argument segment misses the scalar cache:
// ~0.4 us per round at cfg3 (phase stamps, profiles/r6/phase_lr_cfg3.json).  One load per line, all issued
// before the first wait, makes it one miss latency: LR cfg3 29.72 -> 29.62 us, T = 8 13.69 -> 13.56
// (profiles/r6/prologue_ab.txt).
template <class Args>
__device__ __forceinline__ void touch_kernargs() {
    typedef const __attribute__((address_space(4))) unsigned karg_u32;
    karg_u32 *p = (karg_u32 *)__builtin_amdgcn_kernarg_segment_ptr();
    constexpr int n = (int)((sizeof(Args) + 63) / 64);
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < n; ++i) acc ^= p[i * 16];
    asm volatile("" ::"s"(acc));
}
constexpr int kHistOff = kTabPad ? 40960 : 32768;
__host__ __device__ constexpr bool lds_tables_fit(int K, int GP) { return (size_t)K * GP * 16 <= (size_t)kHistOff; }
__host__ __device__ constexpr size_t lds_table_bytes(int K, int GP) { return (size_t)kHistOff + (size_t)K * GP * 16; }

// Entry i = k * GP + c (symbol k, state column c) of the LDS emission tables, 16 B each:
// P {a_cc b_c(k), a_{c-1,c} b_c(k)} (left-to-right, PT) or {b_c(k), 0} (dense); H {histogram, b_c(k)}.
// Round 4 measured two alternatives, both reverted: a dense layout with two 8-B copies of b per row (one
// per sequence-slot parity, to spread the ds_read_b64 lane groups over more banks: 74.0-76.7 us at cfg3
// against 73.4), and H entries {h, h'} with the even / odd sequence slots adding into their own half (a
// ds_add_f64 serves 16 contiguous lanes = two slots x 8 states, and both slots' adds otherwise hit the same
// 8 even banks), b(o_0) then coming from the statistics: LR cfg3 36.96-36.98 us against 35.23-35.58.
template <bool PT, int GP>
__device__ __forceinline__ void tab_put(double *sP, double *sH, int i, double px, double py, double b) {
    reinterpret_cast<double2 *>(sP)[i] = PT ? double2{px, py} : double2{b, 0.0};
    reinterpret_cast<double2 *>(sH)[i] = double2{0.0, b};
}

template <int N, int G, int GP, bool PT, int BLK = kBlock>
__device__ __forceinline__ bool merged_mstep(const EArgs &a, double *sP, double *sH, double *sPA, long long bid);
__device__ __forceinline__ int rank_ll_count(const EArgs &a);
__device__ __forceinline__ void rank_ll_fold(const EArgs &a, long long nblk);
__device__ __forceinline__ void ll_merge(double &M, double &S, double m2, double s2);

// Body of the small-N E-step / scorer for workgroup `bid` of the `nblk` workgroups that cover one
// model's sequences: the whole grid of k_estep_small, or one model's slice of a grouped launch
// (k_estep_small_group, several models of the same shape in one launch).
// DET (deterministic-reduction mode, LDS tables, E-step only): no floating-point atomics anywhere, so
// repeated runs are bitwise identical: gamma goes to per-position rows in HBM (summed per symbol in a
// fixed order by k_bnum_gather, as on the wide path) instead of the LDS histogram, and each workgroup
// writes its partial statistics with plain stores (summed over workgroups in order by k_det_reduce).
// BLK = 2 kBlock (k_estep_join, left-to-right E-step): the spread map's extra workgroup bid runs as waves
// 4.. of full workgroup bid (one 8-wave workgroup per CU), so each CU builds one set of LDS tables, runs
// one M-step prologue and flushes one histogram.
template <int N, int G, bool LR, bool LDSTAB, bool FWD_ONLY, bool DET = false, int BLK = kBlock>
__device__ __forceinline__ void estep_small_body(const EArgs &a, const long long bid, const long long nblk) {
    static_assert(!DET || (LDSTAB && !FWD_ONLY), "deterministic mode: E-step with LDS tables");
    constexpr bool JOIN = BLK > kBlock;
    static_assert(!JOIN || (BLK == 2 * kBlock && LDSTAB && !FWD_ONLY && !DET), "joined map: E-step with LDS tables");
    constexpr int U = kWave / G;
    // dense G = 8: xi on the 4x4x4 MFMA (xi_mfma8), two accumulators per lane in its D layout
    constexpr bool XM = !LR && G == 8 && !FWD_ONLY && HMMBW_XI_MFMA;
    constexpr int NSR = LR ? 2 : N;     // S columns per state in the block reduction (row j of S)
    constexpr int NS = XM ? 2 : NSR;    // per-lane S accumulators
    constexpr int NV = NSR + 3;         // + gamma_den_excl, gamma_den_all, pi_num
    // dense: the forward stores every z_t ([chunk][8 steps][64 lanes], kChunk x the checkpoint
    // layout; the host sizes it), so the backward loads z instead of recomputing it: the recompute is
    // 16 of the dense step's ~70 VALU instructions; the 128 MB at cfg3 go through HBM (275 MB of
    // traffic per launch, 0.46 of the HBM peak over the kernel: not the bound, profiles/r3)
    constexpr bool ZF = !LR && !FWD_ONLY && HMMBW_ZFULL;
    constexpr int GP = LDSTAB ? G + kTabPad : G;  // row stride of the emission / histogram tables
    // left-to-right with LDS tables: per (symbol, state) products {a_jj b_j(o), a_{j-1,j} b_j(o)}
    constexpr bool PT = LR && LDSTAB;
    // split extra waves possible in this instantiation: dense E-step with LDS tables and atomic statistics
    // (dense cfg3 69.4 -> 64.3 us), left-to-right on the joined map only (round 6: cfg3 29.63 -> 28.33 us,
    // profiles/r6/split_lr_ab.txt; beside separate extra workgroups 34.0 -> 35.6 us and its code costs
    // registers, profiles/r5/split_extra_ab.txt)
    // (joined map: the split groups hand over through an LDS flag instead of a workgroup barrier, which would
    // also hold the full workgroup's waves)
    constexpr bool SPLITOK = (!LR || (HMMBW_SPLIT_LR && JOIN)) && LDSTAB && !FWD_ONLY && !DET;
    extern __shared__ __attribute__((aligned(256))) double smem[];  // 256-B aligned whatever the static LDS (ds_read_b128 rows)
    __shared__ double sPA[G + N * N];  // pi (zero-padded to G) and A of this iteration
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // joined map, split groups: A's hand-over flags (cleared here; the prologue's barriers order it before use)
    __shared__ int sXflag[SPLITOK && JOIN ? kBlock / kWave / 2 : 1];
    if constexpr (SPLITOK && JOIN)
        if (tid < kBlock / kWave / 2) sXflag[tid] = 0;
    PHASE(0);
    PHASE_HWID();
    if constexpr (!FWD_ONLY)  // clear the next iteration's statistics (single rank: triple buffer)
        for (long long i = bid * blockDim.x + tid; i < a.zero_len; i += nblk * blockDim.x)
            a.zero[i] = 0.0;
    PHASE(13);
    const int j = lane & (G - 1), u = lane / G;
    const int K = a.K;
    double *sP = smem;                   // LDSTAB: P-table [K][GP] {x, y} (see kHistOff)
    double *sH = smem + kHistOff / 8;    // LDSTAB: H-table [K][GP] {h, b}
    double *sRed = smem + (LDSTAB ? lds_table_bytes(K, GP) / 8 : 0);  // [waves][G][NV] + ll scratch
    bool merged = false;
    if constexpr (LDSTAB && !FWD_ONLY) merged = a.merged != 0;
    const int wpb = JOIN ? kBlock / kWave : blockDim.x >> 6;  // waves of a full (sequence-group) workgroup
    const bool xblk = JOIN ? wv >= wpb : bid >= a.nfull;     // this wave runs an extra group
    const int wx = JOIN ? wv - wpb : wv;                      // index among the extra group's waves
    // split extra waves: with 2 xact <= 4 extra waves, extra wave wx in [xact, 2 xact) is the B partner of extra
    // wave wx - xact (same sequence group): it runs the lower half of the group's backward
    const bool split_wg = SPLITOK && xblk && a.split_extra != 0 && 2 * a.xact <= wpb;
    const bool brole = split_wg && wx >= a.xact && wx < 2 * a.xact;
    const int wvg = brole ? wv - a.xact : wv;
    const int xs = JOIN ? wvg - wpb : wvg;                    // the group's hand-over slot
    const long long wave = JOIN ? (xblk ? a.nfull * wpb + bid * a.xact + (wvg - wpb) : bid * wpb + wv)
                                : (xblk ? a.nfull * wpb + (bid - a.nfull) * a.xact + wvg : bid * wpb + wv);
    const bool wactive = !xblk || wx < a.xact || brole;
    if (merged) {
        // the previous iteration's M-step, computed redundantly by every workgroup straight into
        // its LDS tables (no separate M-step kernel, no parameter round trip through HBM)
        if constexpr (LDSTAB && !FWD_ONLY)
            if (!merged_mstep<N, G, GP, PT, BLK>(a, sP, sH, sPA, bid)) return;  // done or stopped (:346)
    } else {
        if (a.state != nullptr && a.state->done) return;  // converged: device-side no-op
        if (tid < G) sPA[tid] = tid < N ? a.pi[tid] : 0.0;
        if (tid < N * N) sPA[G + tid] = a.A[tid];
        if constexpr (LDSTAB) {
            if constexpr (PT) __syncthreads();  // the records fold a_jj, a_{j-1,j} in
            // 16 independent loads in flight per thread before the first LDS store
            constexpr int TB = 16;
            const int nt = K * GP;
            for (int i0 = 0; i0 < nt; i0 += TB * BLK) {
                double x[TB];
#pragma unroll
                for (int q = 0; q < TB; ++q) {
                    const int i = i0 + q * BLK + tid;
                    const int k = i / GP, c = i - k * GP;
                    const bool ok = i < nt && k < K && c < G;
                    x[q] = a.Bt[ok ? (size_t)k * G + c : 0];
                    x[q] = ok ? x[q] : 0.0;
                }
#pragma unroll
                for (int q = 0; q < TB; ++q) {
                    const int i = i0 + q * BLK + tid;
                    if (i < nt) {
                        if constexpr (PT) {
                            const int c = i % GP;
                            const double ad = c < N ? sPA[G + c * N + c] : 0.0;
                            const double ai = (c >= 1 && c < N) ? sPA[G + (c - 1) * N + c] : 0.0;
                            tab_put<PT, GP>(sP, sH, i, ad * x[q], ai * x[q], x[q]);
                        } else {
                            tab_put<PT, GP>(sP, sH, i, 0.0, 0.0, x[q]);
                        }
                    }
                }
            }
        }
        __syncthreads();
    }
    PHASE(1);

    if (a.prio == 1 && !xblk) __builtin_amdgcn_s_setprio(1);
    if (a.prio == 2 && xblk) __builtin_amdgcn_s_setprio(1);
    double *accb = a.copies + (bid % a.ncopies) * a.copy_len;
    double S[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) S[k] = 0.0;
    double gex = 0.0, gall = 0.0, pin = 0.0;
    double logp_lane = -INFINITY;
    bool ll_valid = false;

    if (wactive && wave < a.L.nwaves) {
        const long long slot = wave * U + u;
#ifdef HMMBW_DIAG_XHALF  // diagnostics (timing only, results wrong): the spread map's extra waves run half their steps
        const int Tw = xblk ? max(kChunk, (a.L.wave_T[wave] / 2) & ~(kChunk - 1)) : a.L.wave_T[wave];
        const int T = min(a.L.slot_len[slot], Tw);
#else
        const int T = a.L.slot_len[slot];
        const int Tw = a.L.wave_T[wave];
#endif
        const int seq = a.L.slot_seq[slot];
        const bool full = a.L.wave_full[wave] != 0;
        const int nch = (Tw + kChunk - 1) / kChunk;
        const long long symbase = a.L.wave_symoff[wave] + u * kChunk;  // pack index of this slot's chunk-0 entry
        const uint16_t *symw = a.L.sym + symbase;
        double *ckw = a.ckpt + (FWD_ONLY ? 0 : a.L.wave_ckoff[wave] * (ZF ? kChunk : 1)) + lane;
        uint4 *spw = a.spack + (FWD_ONLY ? 0 : a.L.wave_spoff[wave]) + u;
        const bool jv = j < N;
        // shortest sequence of the wave: in a ragged wave the chunks every lane is still inside of run
        // unmasked.  Padding slots (T = 0; empty sequences are rejected at the ABI) do not count: their
        // z starts at 0 in the (masked) first chunk and their beta at 1/P = 0, so every term they
        // add in an unmasked chunk is an exact zero.
        int Tmin = T > 0 ? T : INT_MAX;
        Tmin = umin_i32<G>(Tmin);

        // transition coefficients of this lane (state j)
        double acol[LR ? 1 : N], arow[LR ? 1 : N];
        double a_dg = 0.0, a_in = 0.0, a_up = 0.0;
        const double *sA = sPA + G;
        if constexpr (LR) {
            a_dg = jv ? sA[j * N + j] : 0.0;
            a_in = (jv && j >= 1) ? sA[(j - 1) * N + j] : 0.0;
            a_up = (j + 1 < N) ? sA[j * N + j + 1] : 0.0;
        } else {
#pragma unroll
            for (int i = 0; i < N; ++i) {
                acol[i] = jv ? sA[i * N + j] : 0.0;
                arow[i] = jv ? sA[j * N + i] : 0.0;
            }
        }
        const double pij = sPA[j];

        auto loadpack = [&](int c) -> uint4 {
            return *reinterpret_cast<const uint4 *>(symw + (long long)c * U * kChunk);
        };
        // This lane's P-table entry for packed entry k.  With LDS tables the packs hold the byte
        // offset of the symbol's row (o * GP * 16, precomputed on the host), else the symbol.
        char *pj = reinterpret_cast<char *>(sP) + j * 16;
        auto pent = [&](const uint4 &p, int k) -> char * { return pj + sym_of(p, k); };
        auto brow = [&](const uint4 &p, int k) -> const double * {  // b_j(o) (and b_{j+1}(o) after it, global)
            if constexpr (LDSTAB) return reinterpret_cast<const double *>(pent(p, k));
            else return a.Bt + j + (size_t)sym_of(p, k) * G;
        };
        // the emission operand of one step: the product pair (PT) or b_j(o)
        using Em = typename std::conditional<PT, double2, double>::type;
        auto ld_em = [&](const uint4 &p, int k) -> Em {
            if constexpr (PT) return *reinterpret_cast<const double2 *>(pent(p, k));
            else return *brow(p, k);
        };
        // One forward step (hmm_training.py:122-160 without the 2^-s rescale, which the caller
        // applies): PT  a_jj b_j z_{t-1}(j) + a_{j-1,j} b_j z_{t-1}(j-1);  LR  the same from a and b;
        // dense  (A^T z_{t-1})_j b_j.  Used verbatim by the forward sweep and the backward recompute,
        // so both produce bit-identical z_t.
        auto step = [&](double zp, Em e) -> double {
            if constexpr (PT) {
                const double prev = dpp<0x111>(zp);  // row_shr:1 -> z_{t-1}(j-1); 0 in lane 0 of a group
                return fma(e.y, prev, e.x * zp);
            } else if constexpr (LR) {
                const double prev = dpp<0x111>(zp);  // row_shr:1 -> z_{t-1}(j-1); a_in = 0 for j = 0
                return fma(a_in * e, prev, (a_dg * e) * zp);
            } else {
                const double bs = e;
                double acc0 = 0.0, acc1 = 0.0;
                if constexpr (G >= 4) {
                    bcast_dot<G, N>(acc0, acc1, zp, acol);
                } else {
                    sfor<0, N>([&](auto I) {
                        const double zi = gbcast<G, I.value>(zp, lane);
                        if constexpr ((I.value & 1) == 0) acc0 = fma(acol[I.value], zi, acc0);
                        else acc1 = fma(acol[I.value], zi, acc1);
                    });
                }
                return (acc0 + acc1) * bs;
            }
        };
        // Biased exponent field of the group's largest entry (entries are >= 0; 0 for an all-zero
        // group).  Integer-only: bit-field extract + DPP max.
        auto group_bexp = [&](double x) -> int {
            return gmax_i32<G>((int)__builtin_amdgcn_ubfe((unsigned)__double2hiint(x), 20, 11));
        };

        // ---------------- forward sweep (hmm_training.py:357-368) ----------------
        // Lagged mode: only steps t = 0 mod kScale rescale; s_t = M_{t-kScale}, the group exponent
        // measured right after step t-kScale, so C_t = log2|alpha_{t-kScale}| and the stored z stay
        // within a few steps' growth of 1.
        // split: the group's backward is cut at chunk hc (the B partner takes chunks [0, hc)); full waves of
        // at least two chunks only
        const bool spl = split_wg && full && nch >= 2;
        const int hc = spl ? nch / 2 : -1;
        int Ch = 0;  // C after step 8 hc (the forward records it)
        // B partner: beta over t = Tw - 1 .. h with its own power-of-two scaling (beta_t = bt 2^Eb), no
        // statistics (the recursion of :163-199 needs no alpha): the lower half's starting vector
        auto presweep = [&](int h, int &Eb) -> double {
            double bt = jv ? 1.0 : 0.0;
            Eb = 0;
            const int ctop = (Tw - 1) / kChunk, cbot = h / kChunk;
            auto pchunk = [&](int c, const uint4 &p) {
                Em ev[kChunk];
#pragma unroll
                for (int k = 0; k < kChunk; ++k) ev[k] = ld_em(p, k);
#pragma unroll
                for (int k = kChunk - 1; k >= 0; --k) {
                    const int t1 = c * kChunk + k;  // beta_{t1 - 1} from beta_{t1} and b(o_{t1})
                    double bn = bt;
                    if constexpr (PT) {
                        bn = fma(ev[k].x, bt, dpp<0x101>(ev[k].y * bt));  // row_shl:1: state j + 1
                    } else if constexpr (!LR) {
                        const double vd = ev[k] * bt;
                        double b0 = 0.0, b1 = 0.0;
                        if constexpr (G >= 4) {
                            bcast_dot<G, N>(b0, b1, vd, arow);
                        } else {
                            sfor<0, N>([&](auto I) {
                                const double vk = gbcast<G, I.value>(vd, lane);
                                if constexpr ((I.value & 1) == 0) b0 = fma(arow[I.value], vk, b0);
                                else b1 = fma(arow[I.value], vk, b1);
                            });
                        }
                        bn = b0 + b1;
                    }
                    bt = (t1 >= h + 1 && t1 <= Tw - 1) ? bn : bt;
                }
                const int M = group_bexp(bt);
                const int e = M == 0 ? 0 : M - 1023;
                bt = pow2_scale(bt, e);
                Eb += e;
            };
            // 4-deep pack ring, unrolled by 4 (no dynamic register indexing)
            uint4 Q0 = loadpack(ctop), Q1 = loadpack(max(ctop - 1, cbot)), Q2 = loadpack(max(ctop - 2, cbot)),
                  Q3 = loadpack(max(ctop - 3, cbot));
            int c = ctop;
            for (; c - 3 >= cbot; c -= 4) {
                pchunk(c, Q0);
                Q0 = loadpack(max(c - 4, cbot));
                pchunk(c - 1, Q1);
                Q1 = loadpack(max(c - 5, cbot));
                pchunk(c - 2, Q2);
                Q2 = loadpack(max(c - 6, cbot));
                pchunk(c - 3, Q3);
                Q3 = loadpack(max(c - 7, cbot));
            }
            if (c >= cbot) {
                pchunk(c, Q0);
                if (c - 1 >= cbot) {
                    pchunk(c - 1, Q1);
                    if (c - 2 >= cbot) pchunk(c - 2, Q2);
                }
            }
            return bt;
        };
        double z = 0.0;
        int C = 0;
        auto forward = [&](auto SAFE_, auto RAG_) -> bool {
            constexpr bool SAFE = decltype(SAFE_)::value;
            constexpr bool RAG = decltype(RAG_)::value;
            z = 0.0;
            C = 0;
            int pend[kChunk / kScale] = {};  // lagged: exponents to apply at the coming scale steps
            int minM = 4096, maxM = 0;       // extreme group exponents seen (fallback trigger)
            // Symbol packs travel through a 4-deep register ring (the pack of chunk c + 4 is loaded
            // while chunk c runs) and the emissions through a 2-deep one (chunk c + 1's LDS reads are
            // issued before chunk c computes); the sweep is unrolled by 4 so no ring slot is ever
            // copied, which would wait on the load that just filled it.
            uint4 Q[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) Q[i] = loadpack(i < nch ? i : nch - 1);
            double b00;  // b_j(o_0) for pi_j b_j(o_0) (:357-360)
            if constexpr (PT) b00 = *reinterpret_cast<const double *>(pent(Q[0], 0) + kHistOff + 8);  // H.b
            else b00 = *brow(Q[0], 0);
            Em E[2][kChunk];
#pragma unroll
            for (int k = 0; k < kChunk; ++k) E[0][k] = ld_em(Q[0], k);
            auto chunk = [&](int c, const Em (&bv)[kChunk], auto MASK_, auto FIRST_) {
                constexpr bool MASK = decltype(MASK_)::value;
                constexpr bool FIRST = decltype(FIRST_)::value;  // chunk 0: step 0 is pi_j b_j(o_0)
                const int Tend = RAG ? T : Tw;
                int sp[kChunk];
#pragma unroll
                for (int k = 0; k < kChunk; ++k) {
                    const int t = c * kChunk + k;
                    double zn;
                    int st = 0;
                    if constexpr (SAFE) {
                        const double x = (FIRST && k == 0) ? pij * b00 : step(z, bv[k]);
                        const int M = group_bexp(x);
                        st = M == 0 ? 0 : M - 1023;
                        zn = pow2_scale(x, st);
                    } else if (k % kScale == 0) {
                        st = pend[k / kScale];
                        zn = pow2_scale((FIRST && k == 0) ? pij * b00 : step(z, bv[k]), st);
                        const int M = group_bexp(zn);
                        // applied kScale steps later; clamped so an all-zero (dead) group can never
                        // scale itself to inf (the fallback below catches it)
                        pend[k / kScale] = min(max(M - 1023, -600), 600);
                        if (!RAG || t < T) {
                            minM = min(minM, M);
                            maxM = max(maxM, M);
                        }
                    } else {
                        zn = step(z, bv[k]);
                    }
                    if constexpr (MASK) {
                        const bool act = t < Tend;
                        z = act ? zn : z;
                        C += act ? st : 0;
                    } else {
                        z = zn;
                        C += st;
                    }
                    if (SPLITOK && k == 0) Ch = (c == hc) ? C : Ch;  // split: C_h, h = 8 hc
                    sp[k] = st;
                    if constexpr (!FWD_ONLY) {
                        if (ZF) {  // every z_t
                            if constexpr (HMMBW_ZF_NT) __builtin_nontemporal_store(z, &ckw[((long long)c * kChunk + k) * kWave]);
                            else ckw[((long long)c * kChunk + k) * kWave] = z;
                        } else if (k == 0) {
                            ckw[(long long)c * kWave] = z;  // checkpoint z_{8c}
                        }
                    }
                }
                if constexpr (!FWD_ONLY) spw[(long long)c * U] = pack_exps(sp);
            };
            // chunk c uses ring slot r = c % 4.  The steady loop runs 4 chunks per trip with no
            // branches around loads or stores, so the compiler's s_waitcnt vmcnt counts stay exact
            // (a conditional chunk makes it wait for every store of the previous chunks).
            using F0 = std::false_type;
            using F1 = std::true_type;
            auto body = [&](int c, auto R_, auto MASK_, auto FIRST_) {
                constexpr int r = decltype(R_)::value;
                __builtin_amdgcn_sched_barrier(0);  // one chunk at a time: registers stay per chunk
                CHUNKSTAMP(0, c);
#pragma unroll
                for (int k = 0; k < kChunk; ++k) E[(r + 1) & 1][k] = ld_em(Q[(r + 1) & 3], k);
                Q[r] = loadpack(c + 4 < nch ? c + 4 : nch - 1);
                chunk(c, E[r & 1], MASK_, FIRST_);
            };
            auto tail_body = [&](int c, auto R_) {  // masked where the wave's last chunk is partial
                if (RAG || (c == nch - 1 && (Tw % kChunk) != 0)) body(c, R_, F1{}, F0{});
                else body(c, R_, F0{}, F0{});
            };
            using I0 = std::integral_constant<int, 0>;
            using I1 = std::integral_constant<int, 1>;
            using I2 = std::integral_constant<int, 2>;
            using I3 = std::integral_constant<int, 3>;
            if (RAG || (nch == 1 && (Tw % kChunk) != 0)) body(0, I0{}, F1{}, F1{});
            else body(0, I0{}, F0{}, F1{});
            const int lim = RAG ? nch : ((Tw % kChunk) != 0 ? nch - 1 : nch);  // chunks [1, lim) unmasked (full)
            int c = 1;
            using Mk = std::integral_constant<bool, RAG>;
            if constexpr (RAG) {  // ragged wave: chunks [1, Tmin / 8) have every lane active
                for (; c + 4 <= Tmin / kChunk; c += 4) {
                    body(c, I1{}, F0{}, F0{});
                    body(c + 1, I2{}, F0{}, F0{});
                    body(c + 2, I3{}, F0{}, F0{});
                    body(c + 3, I0{}, F0{}, F0{});
                }
            }
            auto trip = [&](int c0) {
                body(c0, I1{}, Mk{}, F0{});
                body(c0 + 1, I2{}, Mk{}, F0{});
                body(c0 + 2, I3{}, Mk{}, F0{});
                body(c0 + 3, I0{}, Mk{}, F0{});
            };
            for (; c + 4 <= lim; c += 4) trip(c);
            if (c < nch) {
                tail_body(c, I1{});
                if (c + 1 < nch) {
                    tail_body(c + 1, I2{});
                    if (c + 2 < nch) {
                        tail_body(c + 2, I3{});
                        if (c + 3 < nch) tail_body(c + 3, I0{});
                    }
                }
            }
            return (!SAFE) && (minM < 1023 - 900 || maxM > 1023 + 900);
        };
        bool safe = a.force_safe != 0;
        if (!brole) {  // the B partner of a split group runs no forward
            if (!safe) {
                const bool bad = full ? forward(std::false_type{}, std::false_type{})
                                      : forward(std::false_type{}, std::true_type{});
                safe = __any(bad && T > 0) != 0;  // wave-uniform: redo the wave with per-step normalisation
            }
            if (safe) {
                if (full) forward(std::true_type{}, std::false_type{});
                else forward(std::true_type{}, std::true_type{});
            }
        }

        PHASE(2);
        // log P(O|lambda) = log(sum_j z_{T-1}(j)) + ln2 * C   (:375-377)
        double phat = 0.0;
        bool alive = false;
        if (!brole) {
            phat = gsum<G>(z);
            alive = (T > 0) && (phat > 0.0);
            const double lp = alive ? (log(phat) + (double)C * 0.69314718055994530942) : -INFINITY;
            if (T > 0 && j == 0 && seq >= 0) a.logp[seq] = lp;
            logp_lane = lp;
            ll_valid = (T > 0) && (j == 0);
        }

        // ---- split extra waves: B's starting vector for the lower half, beta_hat at h = 8 hc ----
        // beta_hat_t = beta_t 2^{C_t} / P (the forward's scaling), P = phat 2^{C_{T-1}}, so
        // beta_hat_h = bt 2^{Eb - (C_{T-1} - C_h)} / phat.  One workgroup barrier (every wave of the
        // workgroup passes it once) orders the forward's checkpoints, exponents and (1/phat, C_{T-1} - C_h,
        // safe) before B reads them.
        double beta_h = 0.0;
        if constexpr (SPLITOK) if (split_wg) {
            __shared__ double sXinv[kBlock / kWave / 2][kWave];
            __shared__ int sXd[kBlock / kWave / 2][kWave];
            __shared__ int sXsafe[kBlock / kWave / 2];
            int Eb = 0;
            double bt = 0.0;
            if (brole && spl) bt = presweep(hc * kChunk, Eb);
            if (!brole && spl) {
                sXinv[xs][lane] = alive ? 1.0 / phat : 0.0;
                sXd[xs][lane] = C - Ch;
                if (lane == 0) sXsafe[xs] = safe ? 1 : 0;
            }
            if constexpr (JOIN) {
                // A releases its slot's flag; B waits for it (the full waves of the workgroup are not held)
                if (!brole && spl) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0) __hip_atomic_store(&sXflag[xs], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                if (brole && spl) {
                    while (__hip_atomic_load(&sXflag[xs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                        __builtin_amdgcn_s_sleep(1);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                }
            } else {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __syncthreads();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            if (brole && spl) {
                safe = sXsafe[xs] != 0;
                beta_h = __builtin_amdgcn_ldexp(bt, Eb - sXd[xs][lane]) * sXinv[xs][lane];
            }
        }

        if constexpr (!FWD_ONLY) if (!(a.ablate & 2)) if (!brole || spl) {
            // ------------- backward sweep fused with gamma / xi / M-step numerators -------------
            const double inv_p = alive ? 1.0 / phat : 0.0;  // beta_hat_{T-1}: folds 1/P (:392,:407)
            // chunks ctop down to clo, entering with beta_hat_{8 ctop + 8} = beta0 (the whole sweep: the top
            // chunk (Tw - 1) / 8 down to 0 from 1/phat; split: A the top down to hc, B hc - 1 down to 0)
            auto backward = [&](auto SAFE_, auto RAG_, auto SPLIT_, const int ctop_, const int clo_, const double beta0) {
                constexpr bool SAFE = decltype(SAFE_)::value;
                constexpr bool RAG = decltype(RAG_)::value;
                // SPLIT: a part of the sweep (split groups only); otherwise the whole sweep, fixed at compile
                // time, so the unsplit waves run the same code as without the split
                constexpr bool SPLIT = decltype(SPLIT_)::value;
                double beta = SPLIT ? beta0 : inv_p;
                const int cl = SPLIT ? ctop_ : (Tw - 1) / kChunk;
                const int clo = SPLIT ? clo_ : 0;
                // per-chunk inputs (checkpoint, scale exponents, symbol pack) through a 4-deep register
                // ring: chunk c - 4's are loaded as soon as chunk c is done with its slot; emissions
                // through a 2-deep one; unrolled by 4 so no slot is copied (see the forward)
                struct Ld {
                    double ck;  // the checkpoint (not with ZF)
                    uint4 sp, pk;
                };
                auto ldset = [&](int c) -> Ld {
                    Ld x;
                    x.ck = ZF ? 0.0 : ckw[(long long)c * kWave];
                    x.sp = spw[(long long)c * U];
                    x.pk = loadpack(c);
                    return x;
                };
                // ZF: the chunk's stored z_t through a 2-deep ring (chunk c - 2 loaded once chunk c is
                // done; 4 deep would not fit 2 waves per SIMD)
                double ZR[ZF ? 2 : 1][ZF ? kChunk : 1];
                auto ldz = [&](double (&zz)[ZF ? kChunk : 1], int c) {
                    if constexpr (ZF) {
#pragma unroll
                        for (int k = 0; k < kChunk; ++k) {
                            if constexpr (HMMBW_ZF_NT) zz[k] = __builtin_nontemporal_load(&ckw[((long long)c * kChunk + k) * kWave]);
                            else zz[k] = ckw[((long long)c * kChunk + k) * kWave];
                        }
                    }
                };
                Ld X[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) X[i] = ldset(cl - i >= 0 ? cl - i : 0);
                if constexpr (ZF) {
                    ldz(ZR[0], cl);
                    ldz(ZR[ZF ? 1 : 0], cl >= 1 ? cl - 1 : 0);
                }
                Em E[2][kChunk];
                double BU[2][kChunk];
                // LDSTAB: this lane's table-row byte offsets of a chunk's symbols, computed once when the
                // chunk's emission rows are read (one chunk ahead) and reused by its histogram atomics
                // (32-bit LDS byte addresses, the table base included, so the atomics need no add)
                unsigned HA[2][kChunk];
                auto ldrows = [&](Em (&bv)[kChunk], double (&bu)[kChunk], unsigned (&ha)[kChunk], const uint4 &p) {
#pragma unroll
                    for (int k = 0; k < kChunk; ++k) {
                        if constexpr (LDSTAB) ha[k] = lds_addr(pj) + (unsigned)sym_of(p, k);
                        if constexpr (PT) {
                            bv[k] = *reinterpret_cast<const double2 *>(lds_ptr(ha[k]));
                        } else {
                            const double *r = LDSTAB ? reinterpret_cast<const double *>(lds_ptr(ha[k])) : brow(p, k);
                            bv[k] = r[0];
                            if constexpr (LR) bu[k] = r[1];  // b_{j+1}(o): the neighbour's emission
                        }
                    }
                };
                ldrows(E[0], BU[0], HA[0], X[0].pk);
                double f_hi = 0.0, fu_hi = 0.0;  // scaled emissions at o_{8c+8} (from chunk c+1)
                Em e_hi{};                       // PT: product pair at o_{8c+8} ...
                int s_hi = 0;                    // ... and that step's scale exponent
                if (SPLIT && cl < (Tw - 1) / kChunk) {  // a lower range: step 8 cl + 8 is chunk cl + 1's first
                    const uint4 pn = loadpack(cl + 1);
                    const int sn = exp_of(spw[(long long)(cl + 1) * U], 0);  // k = 0: always a scale step
                    if constexpr (PT) {
                        e_hi = ld_em(pn, 0);
                        s_hi = sn;
                    } else {
                        const double *r = brow(pn, 0);
                        f_hi = pow2_scale(r[0], sn);
                        if constexpr (LR) fu_hi = pow2_scale(r[1], sn);
                    }
                }
                auto chunk = [&](int c, const Ld &cur, const double (&zst)[ZF ? kChunk : 1], const uint4 &pkn, const Em (&bv)[kChunk],
                                 const double (&bu)[kChunk], Em (&bvn)[kChunk], double (&bun)[kChunk],
                                 const unsigned (&hac)[kChunk], unsigned (&han)[kChunk], auto MASK_) {
                    constexpr bool MASK = decltype(MASK_)::value;
                    const uint4 &spA = cur.sp, &pkA = cur.pk;
                    int sk[kChunk];
                    double fs[kChunk], fus[kChunk];  // non-PT: b(o_t) / c_t for t = 8c .. 8c+7
#pragma unroll
                    for (int k = 0; k < kChunk; ++k) {
                        const bool scaled = SAFE || (k % kScale == 0);
                        sk[k] = scaled ? exp_of(spA, k) : 0;
                        if constexpr (!PT) {
                            fs[k] = scaled ? pow2_scale(bv[k], sk[k]) : bv[k];
                            if constexpr (LR) fus[k] = scaled ? pow2_scale(bu[k], sk[k]) : bu[k];
                        }
                    }
                    // recompute z_{8c .. 8c+7} from the checkpoint (identical ops to the forward); PT keeps
                    // the diagonal products ux[k] = a_jj b_j(o_{8c+k}) z_{8c+k-1}(j): xi_t(j,j) = ux[t+1] v_j
                    double zr[kChunk];
                    double ux[kChunk];
                    zr[0] = ZF ? zst[0] : cur.ck;
                    ux[0] = 0.0;
#pragma unroll
                    for (int k = 1; k < kChunk; ++k) {
                        if constexpr (ZF) {
                            zr[k] = zst[k];
                            continue;
                        }
                        double x;
                        if constexpr (PT) {
                            ux[k] = bv[k].x * zr[k - 1];
                            x = fma(bv[k].y, dpp<0x111>(zr[k - 1]), ux[k]);  // = step(zr[k - 1], bv[k])
                        } else {
                            x = step(zr[k - 1], bv[k]);
                        }
                        zr[k] = (SAFE || (k % kScale == 0)) ? pow2_scale(x, sk[k]) : x;
                    }
                    double gk[kChunk];
#pragma unroll
                    for (int k = kChunk - 1; k >= 0; --k) {
                        const int t = c * kChunk + k;
                        const double zt = zr[k];
                        // regular step (t <= T-2) / gamma_{T-1} (t == T-1) / past the end; per lane in
                        // ragged waves, wave-uniform otherwise; only boundary chunks are masked.
                        // zs = 0 leaves S and gex unchanged.
                        const bool reg = !MASK || (RAG ? (t <= T - 2) : (t <= Tw - 2));
                        const bool ini = MASK && (RAG ? (t == T - 1) : (t == Tw - 1));
                        const double zs = reg ? zt : 0.0;
                        double bn;
                        if constexpr (PT) {
                            // beta_hat_t(j) = a_jj b_j(o') beta'(j) + a_j,j+1 b_j+1(o') beta'(j+1) with
                            // beta' = beta_hat_{t+1} / c_{t+1} (:163-199); the second term is the
                            // neighbour's a_{j,j+1} b_{j+1} beta' product, shifted down one lane (zero
                            // past the last state: a_{N-1,N} does not exist, Bi(., 0) = 0)
                            const Em e = (k == kChunk - 1) ? e_hi : bv[k + 1];
                            const int s1 = (k == kChunk - 1) ? s_hi : sk[(k + 1) & (kChunk - 1)];
                            const bool sc1 = SAFE || ((k + 1) % kScale == 0);
                            const double bp = sc1 ? pow2_scale(beta, s1) : beta;
                            const double vu = dpp<0x101>(e.y * bp);  // row_shl:1
                            bn = fma(e.x, bp, vu);
                            // a_jj b_j(o_{t+1}) z_t(j): from the recompute, or (t = 8c+7) one product
                            const double uk = (k == kChunk - 1) ? e.x * zt : ux[(k + 1) & (kChunk - 1)];
                            S[0] = fma(reg ? uk : 0.0, bp, S[0]);  // xi_t(j,j)   (:396-410)
                            S[1] = fma(zs, vu, S[1]);              // xi_t(j,j+1)
                        } else if constexpr (LR) {
                            const double f = (k == kChunk - 1) ? f_hi : fs[k + 1];  // b(o_{t+1}) / c_{t+1}
                            const double fu = (k == kChunk - 1) ? fu_hi : fus[k + 1];
                            const double bup = dpp<0x101>(beta);  // row_shl:1 -> beta(j+1)
                            const double vd = f * beta, vu = fu * bup;
                            bn = fma(a_up, vu, a_dg * vd);       // :182-197
                            S[0] = fma(zs, vd, S[0]);             // xi_t(j,j)   / a_jj
                            S[1] = fma(zs, vu, S[1]);             // xi_t(j,j+1) / a_j,j+1 (scaled at the end)
                        } else {
                            const double f = (k == kChunk - 1) ? f_hi : fs[k + 1];  // b(o_{t+1}) / c_{t+1}
                            const double vd = f * beta;
                            double b0 = 0.0, b1 = 0.0;
                            if constexpr (G >= 4) {
                                bcast_dot<G, N>(b0, b1, vd, arow);   // :182-193
                                if constexpr (XM) xi_mfma8(S, zs, vd);  // :402-408
                                else bcast_acc<G, N>(S, vd, zs);
                            } else {
                                sfor<0, N>([&](auto I) {
                                    const double vk = gbcast<G, I.value>(vd, lane);
                                    if constexpr ((I.value & 1) == 0) b0 = fma(arow[I.value], vk, b0);
                                    else b1 = fma(arow[I.value], vk, b1);
                                    S[I.value] = fma(zs, vk, S[I.value]);   // :402-408
                                });
                            }
                            bn = b0 + b1;
                        }
                        double g;  // gamma_t(j) (:392)
                        // PT: sum_{t <= T-2} gamma_t(j) = S_jj + S_j,j+1 (the xi row sums, :431-441),
                        // formed after the sweep instead of one add per step
                        if constexpr (MASK) {
                            g = reg ? zt * bn : (ini ? zt * inv_p : 0.0);
                            beta = reg ? bn : beta;
                            if constexpr (!PT) gex = fma(zs, bn, gex);
                            gall += ini ? g : 0.0;
                        } else {
                            g = zt * bn;
                            beta = bn;
                            if constexpr (!PT) gex += g;
                        }
                        if (t == 0) pin = g;  // :420
                        gk[k] = g;
                    }
                    if constexpr (PT) {
                        e_hi = bv[0];
                        s_hi = sk[0];
                    }
                    // next chunk's emission rows go to LDS before this chunk's histogram atomics, so
                    // they are not queued behind them
                    ldrows(bvn, bun, han, pkn);
#ifndef HMMBW_NO_HIST  // diagnostics build: no B-numerator histogram
                    if constexpr (DET) {
                        // gamma row of every position (position = index of the symbol in the pack layout)
                        double *gr = a.gam + (symbase + (long long)c * U * kChunk) * G + j;
#pragma unroll
                        for (int k = 0; k < kChunk; ++k) gr[k * G] = gk[k];
                    } else if constexpr (LDSTAB) {
                        // every lane, no branch (the pad lanes j >= N add their zero gamma to the pad
                        // columns), so the compiler's lgkmcnt bookkeeping stays exact
#pragma unroll
                        for (int k = 0; k < kChunk; ++k)  // :474-485
                            atomicAdd(reinterpret_cast<double *>(lds_ptr(hac[k]) + kHistOff), gk[k]);  // H.h of o_t
                    } else if (N == G || jv) {
#pragma unroll
                        for (int k = 0; k < kChunk; ++k)
                            if (gk[k] != 0.0) unsafeAtomicAdd(&accb[a.off_bnum + (long long)sym_of(pkA, k) * N + j], gk[k]);
                    }
#endif
                    if constexpr (!PT) {
                        f_hi = fs[0];
                        if constexpr (LR) fu_hi = fus[0];
                    }
                };
                auto body = [&](int c, auto R_, auto MASK_) {
                    constexpr int r = decltype(R_)::value;
                    constexpr int rn = (r + 1) & 3;
                    __builtin_amdgcn_sched_barrier(0);  // one chunk at a time: registers stay per chunk
                    CHUNKSTAMP(1, c);
                    chunk(c, X[r], ZR[ZF ? (r & 1) : 0], X[rn].pk, E[r & 1], BU[r & 1], E[(r + 1) & 1], BU[(r + 1) & 1],
                          HA[r & 1], HA[(r + 1) & 1], MASK_);
                    X[r] = ldset(c >= 4 ? c - 4 : 0);  // branch-free: exact vmcnt accounting
                    if constexpr (ZF) ldz(ZR[r & 1], c >= 2 ? c - 2 : 0);
                };
                using Mk = std::integral_constant<bool, RAG>;  // only the first chunk is masked in full waves
                using I0 = std::integral_constant<int, 0>;
                using I1 = std::integral_constant<int, 1>;
                using I2 = std::integral_constant<int, 2>;
                using I3 = std::integral_constant<int, 3>;
                body(cl, I0{}, std::true_type{});  // holds t = Tw - 1
                if constexpr (LDSTAB) {
                    // steady loop: 4 chunks per trip, no branches around the loads or the LDS
                    // atomics, so the compiler's vmcnt / lgkmcnt waits stay exact
                    int c = cl - 1;
                    if constexpr (RAG) {
                        // ragged wave: masked while a trip holds some lane's last frames, then the
                        // chunks with t <= Tmin - 2 for every lane (c <= (Tmin - 9) / 8) unmasked
                        const int cr = Tmin >= kChunk + 1 ? (Tmin - kChunk - 1) / kChunk : -1;
                        for (; c >= clo + 3 && c > cr; c -= 4) {
                            body(c, I1{}, Mk{});
                            body(c - 1, I2{}, Mk{});
                            body(c - 2, I3{}, Mk{});
                            body(c - 3, I0{}, Mk{});
                        }
                        using U0 = std::false_type;
                        for (; c >= clo + 3; c -= 4) {
                            body(c, I1{}, U0{});
                            body(c - 1, I2{}, U0{});
                            body(c - 2, I3{}, U0{});
                            body(c - 3, I0{}, U0{});
                        }
                    }
                    auto trip = [&](int c0) {
                        body(c0, I1{}, Mk{});
                        body(c0 - 1, I2{}, Mk{});
                        body(c0 - 2, I3{}, Mk{});
                        body(c0 - 3, I0{}, Mk{});
                    };
                    for (; c >= clo + 3; c -= 4) trip(c);
                    if (c >= clo) {
                        body(c, I1{}, Mk{});
                        if (c - 1 >= clo) {
                            body(c - 1, I2{}, Mk{});
                            if (c - 2 >= clo) body(c - 2, I3{}, Mk{});
                        }
                    }
                } else {  // global histogram atomics (skipped for zero gamma): the compact loop
                    for (int c = cl - 1; c >= 0; c -= 4) {
                        body(c, I1{}, Mk{});
                        if (c >= 1) body(c - 1, I2{}, Mk{});
                        if (c >= 2) body(c - 2, I3{}, Mk{});
                        if (c >= 3) body(c - 3, I0{}, Mk{});
                    }
                }
            };
            using NoSp = std::false_type;
            if (SPLITOK && spl) {  // full waves only: A the chunks from the top down to hc, B hc - 1 down to 0
                const int ctop = brole ? hc - 1 : (Tw - 1) / kChunk;
                const int clo = brole ? 0 : hc;
                const double beta0 = brole ? beta_h : inv_p;
                if (safe) backward(std::true_type{}, std::false_type{}, std::true_type{}, ctop, clo, beta0);
                else backward(std::false_type{}, std::false_type{}, std::true_type{}, ctop, clo, beta0);
            } else if (safe) {
                if (full) backward(std::true_type{}, std::false_type{}, NoSp{}, 0, 0, 0.0);
                else backward(std::true_type{}, std::true_type{}, NoSp{}, 0, 0, 0.0);
            } else {
                if (full) backward(std::false_type{}, std::false_type{}, NoSp{}, 0, 0, 0.0);
                else backward(std::false_type{}, std::true_type{}, NoSp{}, 0, 0, 0.0);
            }
            if constexpr (PT) gex = S[0] + S[1];
            gall += gex;
            PHASE(3);
            // xi_t(i,j) = a_ij * (the accumulated S_ij): scale once per sequence group (PT already
            // accumulates xi itself)
            if constexpr (!PT && !XM) {  // XM: a_ij applied per element at the flush
#pragma unroll
                for (int k = 0; k < NS; ++k) {
                    if constexpr (LR) S[k] *= (k == 0 ? a_dg : a_up);
                    else S[k] *= arow[k];
                }
            }
        }
    } else if (split_wg && !JOIN) {  // no sequence group here: the split barrier still counts every wave
        __syncthreads();
    }

    __syncthreads();
#if HMMBW_FLUSH_VMWAIT
    // every load of the sweeps has landed long ago; saying so here keeps the compiler from waiting on the
    // flush's global atomics below: at the join of the active and idle waves' paths it otherwise counts a
    // ring load as possibly in flight and, before reusing its register, waits vmcnt(2), i.e. for the
    // round trips of all but two of the histogram atomics issued after it
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#endif
    // the B-numerator histogram's atomics first: their round trips overlap the reductions below
    if constexpr (!FWD_ONLY && !DET && LDSTAB) if (!(a.ablate & 1)) {
        // (round 4: starting each workgroup's pass at a different row, so that workgroups finishing together
        // hit different addresses, measured no faster: 35.1-35.7 against 34.8-35.5 us at cfg3)
        for (int idx = tid; idx < K * G; idx += blockDim.x) {
            const int k = idx / G, jj = idx - k * G;
            if (jj >= N) continue;
            const double x = sH[((size_t)k * GP + jj) * 2];
            if (x != 0.0) unsafeAtomicAdd(&accb[a.off_bnum + (long long)k * N + jj], x);
        }
    }
    PHASE(11);
    // per-block (max, sum exp) of log P for the convergence scalar.  E-step (round 6): each wave forms its own
    // (max, sum exp) pair and writes it beside its statistics partials, and thread 0 merges the waves' pairs
    // after the one barrier the statistics need anyway (block_ll_partial took three more).
    const int nwv = blockDim.x >> 6;
    double *sLL = sRed + (size_t)(BLK / kWave) * G * NV;  // [waves][2] (the host sizes the scratch)
    if constexpr (FWD_ONLY) {
        block_ll_partial(logp_lane, ll_valid, sRed, a.llpart + 2 * bid);
    } else {
        const double wm = wave_max(ll_valid ? logp_lane : -INFINITY);
        const double ws = gsum<64>((ll_valid && wm != -INFINITY && logp_lane != -INFINITY) ? exp(logp_lane - wm) : 0.0);
        if (lane == 0) {
            sLL[2 * wv] = wm;
            sLL[2 * wv + 1] = ws;
        }
    }
    PHASE(4);
    // fused multi-rank launch: thread 0 counts this workgroup's pair in during the statistics flush (the
    // ticket's round trip overlaps the flush), and wave 0 of the last one folds the pairs at the end
    const bool fused_ll = !FWD_ONLY && !DET && a.rank_ll != nullptr;
    int ticket = 0;
    bool counted = false;
    // the waves' log-likelihood pairs merged by wave 0 (after the barrier below), lane w taking wave w's pair:
    // one exp per lane in parallel (a serial merge by one thread put ~0.5 us on the tail)
    auto ll_out = [&]() {
        if (wv == 0) {
            double mw = -INFINITY, sw = 0.0;
            if (lane < nwv) {
                mw = sLL[2 * lane];
                sw = sLL[2 * lane + 1];
            }
            const bool ok = sw > 0.0;
            const double M = wave_max(ok ? mw : -INFINITY);
            const double S = gsum<64>((ok && M != -INFINITY) ? sw * exp(mw - M) : 0.0);
            // memory-side atomics: the fused M-step of the last workgroup reads these with atomics too
            if (lane == 0) {
                atomicExch(&a.llpart[2 * bid], (S > 0.0) ? M : 0.0);
                atomicExch(&a.llpart[2 * bid + 1], S);
            }
        }
    };

    if constexpr (!FWD_ONLY) if (a.ablate & 1) {
        __syncthreads();
        ll_out();
    }
    if constexpr (!FWD_ONLY) if (!(a.ablate & 1)) {
        // ---- reduce per-lane accumulators over the U sequences of the wave, then the block ----
        constexpr int K0 = XM ? NSR : 0;  // XM: the S columns come from the MFMA lanes below
        double vals[NV];
#pragma unroll
        for (int k = 0; k < NS && !XM; ++k) vals[k] = S[k];
        vals[NSR] = gex;
        vals[NSR + 1] = gall;
        vals[NSR + 2] = pin;
#pragma unroll
        for (int k = K0; k < NV; ++k) vals[k] = usum<G>(vals[k]);
        double xd = 0.0, xo = 0.0;
        if constexpr (XM) {  // sum the two seq parities (lane bit 3)
            xd = S[0] + dpp<0x128>(S[0]);  // row_ror:8 = lane ^ 8 within the row
            xo = S[1] + dpp<0x128>(S[1]);
        }
        if (u == 0) {
#pragma unroll
            for (int k = K0; k < NV; ++k) sRed[(wv * G + j) * NV + k] = vals[k];
        }
        if constexpr (XM) {
            if ((lane & 8) == 0) {
                const int jh = (lane >> 2) & 1, from = 4 * jh + (lane >> 4);
                const int td = 4 * jh + (lane & 3), to = 4 * (1 - jh) + 3 - (lane & 3);
                if (from < N) {
                    const double *sA = sPA + G;  // xi_t(i,j) = a_ij S_ij
                    if (td < N) sRed[(wv * G + from) * NV + td] = xd * sA[from * N + td];
                    if (to < N) sRed[(wv * G + from) * NV + to] = xo * sA[from * N + to];
                }
            }
        }
        double *sPart = smem;  // DET: this workgroup's statistics [off_bnum] (the tables are dead now)
        if constexpr (DET)
            for (long long i = tid; i < a.off_bnum; i += blockDim.x) sPart[i] = 0.0;
        __syncthreads();
        ll_out();
        if (fused_ll && tid == 0) ticket = rank_ll_count(a);
        counted = true;
        const int nw = blockDim.x >> 6;
        for (int idx = tid; idx < G * NV; idx += blockDim.x) {
            const int jj = idx / NV, k = idx % NV;
            if (jj >= N) continue;
            double x = 0.0;
            for (int w = 0; w < nw; ++w) x += sRed[(w * G + jj) * NV + k];
            if (x == 0.0) continue;
            long long dst;
            if (k < NSR) {
                const int col = LR ? jj + k : k;
                if (col >= N) continue;
                dst = a.off_S + (long long)jj * N + col;
            } else if (k == NSR) {
                dst = a.off_gex + jj;
            } else if (k == NSR + 1) {
                dst = a.off_gall + jj;
            } else {
                dst = jj;  // pi_num at offset 0
            }
            if constexpr (DET) sPart[dst] = x;
            else unsafeAtomicAdd(&accb[dst], x);
        }
        if constexpr (DET) {
            __syncthreads();
            for (long long i = tid; i < a.off_bnum; i += blockDim.x) a.part[bid * a.off_bnum + i] = sPart[i];
        }
    }
    PHASE(5);
    if (fused_ll && wv == 0) {
        if (!counted && tid == 0) ticket = rank_ll_count(a);
        if (__shfl(ticket, 0) == (int)(nblk - 1)) rank_ll_fold(a, nblk);
    }
}

template <int N, int G, bool LR, bool LDSTAB, bool FWD_ONLY, bool DET = false>
__global__ void __launch_bounds__(kBlock, 2) k_estep_small(EArgs a) {  // 2 waves per SIMD (<= 256 VGPRs)
#if HMMBW_KARG_TOUCH
    touch_kernargs<EArgs>();
#endif
    estep_small_body<N, G, LR, LDSTAB, FWD_ONLY, DET>(a, blockIdx.x, gridDim.x);
}

// Joined spread map (E-step with LDS tables): one 8-wave workgroup per CU, grid = nfull; waves 4.. of
// workgroup b run extra workgroup b's xact sequence groups (estep_small_body, JOIN), and on the dense path
// their split B partners (hand-over by LDS flag).
template <int N, int G, bool LR>
__global__ void __launch_bounds__(2 * kBlock, 1) k_estep_join(EArgs a) {
#if HMMBW_KARG_TOUCH
    touch_kernargs<EArgs>();
#endif
    estep_small_body<N, G, LR, true, false, false, 2 * kBlock>(a, blockIdx.x, gridDim.x);
}

// Grouped launch: g.nm models of one shape (same N, topology and tables), model m owning workgroups
// [start[m], start[m+1]) with its own arguments args[m] (observations, parameters, statistics,
// convergence state).  Replaces the per-word loop of HMM/main.py:147-152 (train) and the per-model
// loop of HMM/hmm_testing.py:139-161 (test) with one launch per EM iteration / per scoring pass.
template <int N, int G, bool LR, bool LDSTAB, bool FWD_ONLY>
__global__ void __launch_bounds__(kBlock, 2) k_estep_small_group(GroupArgs g) {
    const long long b = blockIdx.x;
    int lo = 0, hi = g.nm - 1;  // the last model whose first workgroup is <= b (uniform search)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (g.start[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    const long long b0 = g.start[lo];
    estep_small_body<N, G, LR, LDSTAB, FWD_ONLY>(g.args[lo], b - b0, g.start[lo + 1] - b0);
}

// ---------------------------------------------------------------------------------------------
// Block reductions
// ---------------------------------------------------------------------------------------------
__device__ double block_reduce(double x, double *sh, bool is_max) {
    const int tid = threadIdx.x;
    x = is_max ? wave_max(x) : gsum<64>(x);
    __syncthreads();
    if ((tid & 63) == 0) sh[tid >> 6] = x;
    __syncthreads();
    if (tid < 64) {
        const int nw = blockDim.x >> 6;
        double y = tid < nw ? sh[tid] : (is_max ? -INFINITY : 0.0);
        y = is_max ? wave_max(y) : gsum<64>(y);
        if (tid == 0) sh[0] = y;
    }
    __syncthreads();
    const double r = sh[0];
    __syncthreads();
    return r;
}

// Combine per-block (max, sum exp) pairs into this rank's pair (log_sum_exp :66-79 over :503).
// ATOMIC: read with returning memory-side atomics (inside the producing kernel, where the per-XCD
// L2s give no cross-workgroup visibility for plain loads).
template <bool ATOMIC = false>
__device__ __forceinline__ double rd(const double *p) {
    if constexpr (ATOMIC) return unsafeAtomicAdd(const_cast<double *>(p), 0.0);
    else return *p;
}

template <bool ATOMIC = false>
__device__ void combine_ll_pairs(const double *pairs, long long n, double *sh, double *m_out, double *s_out) {
    double mx = -INFINITY;
    for (long long r = threadIdx.x; r < n; r += blockDim.x)
        if (rd<ATOMIC>(&pairs[2 * r + 1]) > 0.0) mx = fmax(mx, rd<ATOMIC>(&pairs[2 * r]));
    mx = block_reduce(mx, sh, true);
    double s = 0.0;
    if (mx != -INFINITY)
        for (long long r = threadIdx.x; r < n; r += blockDim.x) {
            const double sr = rd<ATOMIC>(&pairs[2 * r + 1]);
            if (sr > 0.0) s += sr * exp(rd<ATOMIC>(&pairs[2 * r]) - mx);
        }
    s = block_reduce(s, sh, false);
    *m_out = mx;
    *s_out = s;
}



// sum of one statistic over the copies, clearing them for the next iteration
template <bool ATOMIC>
__device__ __forceinline__ double take(const MArgs &m, long long idx) {
    double v = 0.0;
    double *p = const_cast<double *>(m.src) + idx;
    for (int c = 0; c < m.nsrc; ++c) {
        if constexpr (ATOMIC) {
            v += atomicExch(p + c * m.copy_len, 0.0);
        } else {
            v += p[c * m.copy_len];
            p[c * m.copy_len] = 0.0;
        }
    }
    return v;
}

// B entry from its numerator and the reciprocal of its row's denominator (:460-497): 1e-20 floor when
// no gamma term carries the symbol, 0 for an empty row.  Shared by every M-step variant, so they
// produce bit-identical parameters.
// Column of state j in the wide kernels' emission table (estep_mfma.hpp): j = 16m + 4r + g is stored
// at 16m + 4g + r, so the 4 states one lane owns are contiguous.
__host__ __device__ inline int bt_col(int j) { return (j & ~15) | ((j & 3) << 2) | ((j >> 2) & 3); }

__device__ __forceinline__ double mstep_inv(double den) { return den > 0.0 ? 1.0 / den : 0.0; }
__device__ __forceinline__ double bnum_to_b(double num, double inv) {
    return inv > 0.0 ? (num > 0.0 ? num * inv : 1e-20) : 0.0;
}

// Convergence record of one EM iteration (hmm_training.py:503-514): L of the parameters that entered
// it, diff (+inf on the first iteration), the stop rule of :346; written to the next state slot.
__device__ bool record_iteration(const MArgs &m, const IterState &in, double L) {
    const double diff = (in.prev_L != -INFINITY) ? fabs(L - in.prev_L) : INFINITY;  // :505-508
    const long long it = in.iteration;
    const bool cont = (diff >= in.epsilon) && (it + 1 < in.max_iterations);
    m.hist[2 * (it % kHist)] = L;
    m.hist[2 * (it % kHist) + 1] = diff;
    IterState o = in;
    o.prev_L = L;
    o.last_L = L;
    o.last_diff = diff;
    o.iteration = it + 1;
    if (!cont) {
        o.done = 1;
        o.converged = (it + 1 < in.max_iterations) ? 1 : 0;
    }
    *m.state_out = o;
    if (m.live != nullptr) {  // the host mirror: record and state first, then (acknowledged) the publication
        auto sys = [](auto *p, auto v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
        sys(&m.live->hist[2 * (it % kHist)], L);
        sys(&m.live->hist[2 * (it % kHist) + 1], diff);
        IterState *sl = &m.live->slot[o.iteration & 1];
        sys(&sl->prev_L, o.prev_L);
        sys(&sl->last_L, o.last_L);
        sys(&sl->last_diff, o.last_diff);
        sys(&sl->epsilon, o.epsilon);
        sys(&sl->iteration, o.iteration);
        sys(&sl->max_iterations, o.max_iterations);
        sys(&sl->done, o.done);
        sys(&sl->converged, o.converged);
        sys(&sl->error, o.error);
        sys(&sl->error_src, o.error_src);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): every store above is acknowledged
        sys(&m.live->pub, ((unsigned long long)m.live_epoch << 32) | (unsigned long long)(unsigned)o.iteration);
    }
    return cont;
}

// L = LSE_r log P_r (:503) from one all-reduced (max, sum exp) pair per rank, by ONE thread in rank
// order.  Every multi-rank M-step variant (the merged prologue, k_mstep, k_mstep_grid) forms L with
// this function, so ranks that run different variants (an empty shard cannot merge its M-step) still
// hold bitwise-identical L and diff and take the same stop decision (:346).
__device__ __forceinline__ double lse_rank_pairs(const double *ll, long long n) {
    double mx = -INFINITY;
    for (long long r = 0; r < n; ++r)
        if (ll[2 * r + 1] > 0.0) mx = fmax(mx, ll[2 * r]);
    double s = 0.0;
    if (mx != -INFINITY)
        for (long long r = 0; r < n; ++r)
            if (ll[2 * r + 1] > 0.0) s += ll[2 * r + 1] * exp(ll[2 * r] - mx);
    return (s > 0.0) ? mx + log(s) : -INFINITY;
}

// M-step kernels entered after convergence carry the state over to the next slot and do nothing else
__device__ __forceinline__ bool carry_if_done(const MArgs &m) {
    if (!m.state->done) return false;
    if (threadIdx.x == 0 && blockIdx.x == 0) *m.state_out = *m.state;
    return true;
}

// M-step + convergence by one workgroup of 256 threads (hmm_training.py:415-514).
template <bool ATOMIC>
__device__ void mstep_block(const MArgs &m) {
    __shared__ double sh[16];
    __shared__ double sL;
    __shared__ double sPi[64], sGex[64], sGall[64];
    const IterState *st = m.state;
    const int tid = threadIdx.x;
    // L = LSE_r log P_r over all ranks (:503)
    if (m.local_lse) {
        double mx, s;
        combine_ll_pairs<ATOMIC>(m.llpart, m.nblocks, sh, &mx, &s);
        if (tid == 0) sL = (s > 0.0) ? mx + log(s) : -INFINITY;
    } else if (tid == 0) {
        sL = lse_rank_pairs(m.llpart, m.nblocks);  // one (max, sum exp) pair per rank, all-reduced
        for (long long r = 0; r < 2 * m.nblocks; ++r) m.zero_ll[r] = 0.0;
    }
    const int N = m.N, K = m.K;
    for (int i = tid; i < N; i += blockDim.x) {
        sPi[i] = take<ATOMIC>(m, i);
        sGex[i] = take<ATOMIC>(m, m.off_gex + i);
        sGall[i] = take<ATOMIC>(m, m.off_gall + i);
    }
    __syncthreads();
    // pi (:415-424): LSE_r gamma_0 - log R ; no term -> -inf
    for (int i = tid; i < N; i += blockDim.x) m.pi[i] = sPi[i] > 0.0 ? sPi[i] / (double)m.R_global : 0.0;
    // A (:429-455): xi numerator; denominator excludes the last frame
    for (int idx = tid; idx < N * N; idx += blockDim.x) {
        const double den = sGex[idx / N];
        const double num = take<ATOMIC>(m, m.off_S + idx);
        m.A[idx] = (den > 0.0 && num > 0.0) ? num / den : 0.0;
    }
    // B (:460-497): floor 1e-20 when no gamma term carries the symbol; empty denominator -> row 0
    for (long long idx = tid; idx < (long long)N * K; idx += blockDim.x) {
        const int jj = (int)(idx % N), k = (int)(idx / N);  // symbol-major: coalesced over the copies
        const double num = take<ATOMIC>(m, m.off_bnum + idx);
        const double v = bnum_to_b(num, mstep_inv(sGall[jj]));
        m.B[(long long)jj * K + k] = v;
        m.Bt[(long long)k * m.G + (m.bt_perm ? bt_col(jj) : jj)] = v;
    }
    __syncthreads();
    if (tid == 0) record_iteration(m, *st, sL);
}



// M-step + convergence spread over the whole grid (large N x K, e.g. the wide path's 64 x 1024 B):
// every workgroup re-estimates its grid-stride share of B (:460-497) and A (:429-455) from the
// statistics summed over the copies; workgroup 0 also does pi (:415-424), L and the convergence
// record (:503-514).  The statistics are only read (each E-step launch clears the buffer it will fill), so
// no workgroup depends on another.
__device__ __forceinline__ double peek(const MArgs &m, long long idx) {
    double v = 0.0;
    for (int c = 0; c < m.nsrc; ++c) v += m.src[c * m.copy_len + idx];
    return v;
}

__device__ void mstep_grid(const MArgs &m) {
    __shared__ double sh[16];
    __shared__ double sL;
    __shared__ double sGall[64];
    const int tid = threadIdx.x;
    const int N = m.N, K = m.K;
    for (int i = tid; i < N; i += blockDim.x) sGall[i] = mstep_inv(peek(m, m.off_gall + i));
    __syncthreads();
    for (long long idx = (long long)blockIdx.x * blockDim.x + tid; idx < (long long)N * K;
         idx += (long long)gridDim.x * blockDim.x) {
        const int jj = (int)(idx % N), k = (int)(idx / N);  // symbol-major: coalesced reads
        const double v = bnum_to_b(peek(m, m.off_bnum + idx), sGall[jj]);
        m.B[(long long)jj * K + k] = v;
        m.Bt[(long long)k * m.G + (m.bt_perm ? bt_col(jj) : jj)] = v;
    }
    for (long long idx = (long long)blockIdx.x * blockDim.x + tid; idx < (long long)N * N;
         idx += (long long)gridDim.x * blockDim.x) {  // A (:429-455)
        const double den = peek(m, m.off_gex + idx / N);
        const double num = peek(m, m.off_S + idx);
        m.A[idx] = (den > 0.0 && num > 0.0) ? num / den : 0.0;
    }
    if (blockIdx.x != 0) return;
    if (m.local_lse) {
        double mx, s;
        combine_ll_pairs<false>(m.llpart, m.nblocks, sh, &mx, &s);
        if (tid == 0) sL = (s > 0.0) ? mx + log(s) : -INFINITY;
    } else if (tid == 0) {
        sL = lse_rank_pairs(m.llpart, m.nblocks);  // one (max, sum exp) pair per rank, all-reduced
    }
    for (int i = tid; i < N; i += blockDim.x) {
        const double pn = peek(m, i);
        m.pi[i] = pn > 0.0 ? pn / (double)m.R_global : 0.0;
    }
    __syncthreads();
    if (tid == 0) record_iteration(m, *m.state, sL);
}

// merge (max, sum exp) pairs: online log-sum-exp
__device__ __forceinline__ void ll_merge(double &M, double &S, double m2, double s2) {
    if (!(s2 > 0.0)) return;
    if (!(S > 0.0)) { M = m2; S = s2; return; }
    if (m2 > M) { S = S * exp(M - m2) + s2; M = m2; }
    else S += s2 * exp(m2 - M);
}

// M-step staged through LDS (sSt: copy_len doubles): the statistics (summed over the copies, which
// are cleared) and the per-workgroup log-likelihood pairs are gathered in independent batches, then
// the update runs from LDS.  ATOMIC (fused into the E-step): gathered with returning memory-side
// atomics; otherwise (its own kernel, after a kernel boundary) with plain loads.
template <bool ATOMIC>
__device__ void mstep_staged(const MArgs &m, double *sSt) {
    __shared__ double sM[16], sS[16];
    __shared__ double sL;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
    const int N = m.N, K = m.K;
    const long long len = m.copy_len;
    // ---- one batch of independent loads: convergence state, LL pairs, statistics ----
    IterState in{};
    if (tid == 0) in = *m.state;
    // Branch-free, clamped addresses so the compiler issues every load of a batch before the first
    // wait (a guarded load inside a runtime loop serialises on its own s_waitcnt).
    constexpr int PB = 4;
    double pm[PB], ps[PB];
    double M = -INFINITY, S = 0.0;
    const long long nb = m.nblocks;  // >= 1 (a launch with no workgroups leaves nothing pending)
    for (long long r0 = 0; r0 < nb; r0 += (long long)PB * blockDim.x) {
#pragma unroll
        for (int u = 0; u < PB; ++u) {
            const long long r = r0 + (long long)u * blockDim.x + tid;
            const long long rc = r < nb ? r : nb - 1;
            pm[u] = rd<ATOMIC>(m.llpart + 2 * rc);
            ps[u] = rd<ATOMIC>(m.llpart + 2 * rc + 1);
        }
#pragma unroll
        for (int u = 0; u < PB; ++u) {
            const bool ok = r0 + (long long)u * blockDim.x + tid < nb;
            ll_merge(M, S, ok ? pm[u] : -INFINITY, ok ? ps[u] : 0.0);
        }
    }
    constexpr int B = 16;
    double *src = const_cast<double *>(m.src);
    for (long long base = 0; base < len; base += (long long)B * blockDim.x) {
        double v[B];
#pragma unroll
        for (int u = 0; u < B; ++u) v[u] = 0.0;
        for (int c = 0; c < m.nsrc; ++c) {
            double x[B];
#pragma unroll
            for (int u = 0; u < B; ++u) {
                const long long idx = base + (long long)u * blockDim.x + tid;
                double *q = src + c * len + (idx < len ? idx : len - 1);
                if constexpr (ATOMIC) x[u] = idx < len ? atomicExch(q, 0.0) : 0.0;
                else x[u] = *q;
            }
#pragma unroll
            for (int u = 0; u < B; ++u) v[u] += x[u];
        }
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const long long idx = base + (long long)u * blockDim.x + tid;
            if (idx < len) {
                sSt[idx] = v[u];
                if constexpr (!ATOMIC)
                    for (int c = 0; c < m.nsrc; ++c) src[c * len + idx] = 0.0;
            }
        }
    }
    // ---- L = LSE_r log P_r (:503) ----
    for (int k = 32; k >= 1; k >>= 1) ll_merge(M, S, __shfl_xor(M, k), __shfl_xor(S, k));
    if (lane == 0) { sM[wv] = M; sS[wv] = S; }
    __syncthreads();
    if (tid == 0) {
        double MM = -INFINITY, SS = 0.0;
        for (int w = 0; w < nw; ++w) ll_merge(MM, SS, sM[w], sS[w]);
        sL = (SS > 0.0) ? MM + log(SS) : -INFINITY;
    }
    __syncthreads();
    const double *sPi = sSt, *sS_ = sSt + m.off_S, *sGex = sSt + m.off_gex, *sGall = sSt + m.off_gall,
                 *sBn = sSt + m.off_bnum;
    // pi (:415-424), A (:429-455), B (:460-497)
    if (tid < N) m.pi[tid] = sPi[tid] > 0.0 ? sPi[tid] / (double)m.R_global : 0.0;
    if (tid < N * N) {
        const double den = sGex[tid / N];
        const double num = sS_[tid];
        m.A[tid] = (den > 0.0 && num > 0.0) ? num / den : 0.0;
    }
    for (int idx = tid; idx < N * K; idx += blockDim.x) {
        const int k = idx / N, jj = idx - k * N;
        const double v = bnum_to_b(sBn[idx], mstep_inv(sGall[jj]));
        m.B[(long long)jj * K + k] = v;
        m.Bt[(long long)k * m.G + (m.bt_perm ? bt_col(jj) : jj)] = v;
    }
    if (tid == 0) record_iteration(m, in, sL);
}

// The previous iteration's M-step + convergence step (hmm_training.py:415-514), run by EVERY
// workgroup of the merged E-step launch, straight into its LDS tables: every workgroup reads the same
// statistics and log-likelihood pairs and applies the same arithmetic in the same order, so all of
// them hold bit-identical parameters and reach the same stop decision.  Workgroup 0 also writes the
// parameters back to HBM (for the queries) and records the iteration in the other state slot.
// Returns false when EM stops here (or had stopped before).
constexpr int kMergedMaxStats = 16 * kBlock;  // statistics per launch the prologue holds in registers

__device__ __forceinline__ double wave_max(double x) {
    x = fmax(x, dpp<0xB1>(x));
    x = fmax(x, dpp<0x4E>(x));
    x = fmax(x, dpp<0x141>(x));
    x = fmax(x, dpp<0x140>(x));
    x = max_swap<false>(x);
    return max_swap<true>(x);
}

// Multi-rank fused E-step (hmmbw_iterate with the engine communicator): the workgroups accumulate
// straight into the all-reduce buffer, and wave 0 of the LAST workgroup to count its pair in (completion
// counter) folds the per-workgroup (max, sum exp) pairs into this rank's slot (what k_reduce_local did
// in its own launch).  No __threadfence: a device-scope release writes back the XCD's L2 (this launch's
// checkpoints), which cost ~20 us per launch; the pairs are memory-side atomics, so thread 0 only has
// to see its own pair land (vmcnt(0)) before it counts, and the folding wave reads them with atomics.
__device__ __forceinline__ int rank_ll_count(const EArgs &a) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // s_waitcnt vmcnt(0): block_ll_partial's atomicExch has landed
    return atomicAdd(a.done_ctr, 1);
}

__device__ __forceinline__ void rank_ll_fold(const EArgs &a, long long nblk) {  // one wave
    const int lane = threadIdx.x & 63;
    double tm = -INFINITY, ts = 0.0;
    for (long long r0 = 0; r0 < nblk; r0 += 4 * 64) {
        double pm[4], ps[4];  // every round's memory-side reads issued together
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const long long r = r0 + lane + q * 64;
            pm[q] = r < nblk ? rd<true>(&a.llpart[2 * r]) : 0.0;
            ps[q] = r < nblk ? rd<true>(&a.llpart[2 * r + 1]) : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (!(ps[q] > 0.0)) continue;
            if (pm[q] > tm) {
                ts = (tm == -INFINITY) ? ps[q] : ps[q] + ts * exp(tm - pm[q]);
                tm = pm[q];
            } else {
                ts += ps[q] * exp(pm[q] - tm);
            }
        }
    }
    const double mx = wave_max(tm);
    const double s = gsum<64>((mx != -INFINITY && ts > 0.0) ? ts * exp(tm - mx) : 0.0);
    if (lane == 0) {
        atomicExch(&a.rank_ll[0], (s > 0.0) ? mx : 0.0);
        atomicExch(&a.rank_ll[1], s);
        atomicExch(a.done_ctr, 0);
    }
}

template <int N, int G, int GP, bool PT, int BLK>
__device__ __forceinline__ bool merged_mstep(const EArgs &a, double *sP, double *sH, double *sPA, long long bid) {
    constexpr int NSM = N + N * N + 2 * N;  // pi_num, xi, gamma_den_excl, gamma_den_all
    constexpr int NW = BLK / 64;
    constexpr int SB = kMergedMaxStats / BLK;
    constexpr int PB = 2;                   // log-likelihood pairs per thread per pass
    __shared__ double sSm[NSM];
    __shared__ double sMx[NW], sSum[NW];
    __shared__ double sLr;  // multi-rank: L from the per-rank pairs (lse_rank_pairs)
    __shared__ IterState sIn;
    const MArgs &m = a.m;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int K = a.K;
    const long long len = m.copy_len;
    PHASE(8);
    // ---- every load issued before any use: statistics, log-likelihood pairs, convergence state (the
    // pairs and the state before the other copies' statistics are waited for: one latency, not two) ----
    double v[SB];
#pragma unroll
    for (int q = 0; q < SB; ++q) {
        const long long idx = (long long)q * BLK + tid;
        v[q] = m.src[idx < len ? idx : len - 1];
    }
    const long long nb = m.nblocks;  // >= 1
    double pm[PB], ps[PB];
#pragma unroll
    for (int q = 0; q < PB; ++q) {
        const long long r = (long long)q * BLK + tid;
        const long long rc = r < nb ? r : nb - 1;
        pm[q] = m.llpart[2 * rc];
        ps[q] = m.llpart[2 * rc + 1];
    }
    IterState in{};
    if (tid == 0) {
        in.prev_L = m.state->prev_L;
        in.epsilon = m.state->epsilon;
        in.iteration = m.state->iteration;
        in.max_iterations = m.state->max_iterations;
        in.done = m.state->done;
        in.converged = m.state->converged;
        in.error = m.state->error;
        in.error_src = m.state->error_src;
        in.last_L = m.state->last_L;
        in.last_diff = m.state->last_diff;
    }
    for (int c = 1; c < m.nsrc; ++c) {
        double x[SB];
#pragma unroll
        for (int q = 0; q < SB; ++q) {
            const long long idx = (long long)q * BLK + tid;
            x[q] = m.src[c * len + (idx < len ? idx : len - 1)];
        }
#pragma unroll
        for (int q = 0; q < SB; ++q) v[q] += x[q];
    }
    PHASE_DRAIN(9);
    // ---- L = LSE_r log P_r (:503) in two passes: max, then sum of exp(m - max) ----
    double mx = -INFINITY;
#pragma unroll
    for (int q = 0; q < PB; ++q) {
        const bool ok = (long long)q * BLK + tid < nb && ps[q] > 0.0;
        mx = ok ? fmax(mx, pm[q]) : mx;
    }
    for (long long r = (long long)PB * BLK + tid; r < nb; r += BLK)  // > 512 workgroups
        if (m.llpart[2 * r + 1] > 0.0) mx = fmax(mx, m.llpart[2 * r]);
    mx = wave_max(mx);
    if (lane == 0) sMx[wv] = mx;
#pragma unroll
    for (int q = 0; q < SB; ++q) {
        const int idx = q * BLK + tid;
        if (idx < NSM) sSm[idx] = (idx < len) ? v[q] : 0.0;
    }
    if (tid == 0) {
        sIn = in;
        // multi-rank: the same fixed-order fold as the standalone M-step kernels of other ranks
        if (!m.local_lse) sLr = lse_rank_pairs(m.llpart, nb);
    }
    __syncthreads();
    PHASE(6);
    if (sIn.done) {  // converged before this launch: device-side no-op
        if (tid == 0 && bid == 0) *m.state_out = sIn;
        return false;
    }
    double Mb = sMx[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) Mb = fmax(Mb, sMx[w]);
    double sum = 0.0;
    if (Mb != -INFINITY) {
#pragma unroll
        for (int q = 0; q < PB; ++q) {
            const bool ok = (long long)q * BLK + tid < nb && ps[q] > 0.0;
            sum += ok ? ps[q] * exp(pm[q] - Mb) : 0.0;
        }
        for (long long r = (long long)PB * BLK + tid; r < nb; r += BLK)
            if (m.llpart[2 * r + 1] > 0.0) sum += m.llpart[2 * r + 1] * exp(m.llpart[2 * r] - Mb);
    }
    sum = gsum<64>(sum);
    if (lane == 0) sSum[wv] = sum;
    PHASE(7);
    // pi (:415-424), A (:429-455) into LDS
    if (tid < G) sPA[tid] = (tid < N && sSm[tid] > 0.0) ? sSm[tid] / (double)m.R_global : 0.0;
    if (tid < N * N) {
        const double den = sSm[N + N * N + tid / N];
        const double num = sSm[N + tid];
        sPA[G + tid] = (den > 0.0 && num > 0.0) ? num / den : 0.0;
    }
    // B (:460-497) from the registers straight into the emission table (and HBM, workgroup 0).
    // Element e = q * BLK + tid - NSM is symbol e / N, state e % N; with N | BLK the state (and
    // so the denominator) is the same for every q of a thread: one reciprocal per thread.
    const bool w0 = bid == 0;
    const int e0 = tid - NSM;
    constexpr bool kSameState = (BLK % N) == 0;
    const int jj0 = ((e0 % N) + N) % N;
    const double inv0 = kSameState ? mstep_inv(sSm[N + N * N + N + jj0]) : 0.0;
    // PT: a_jj and a_{j-1,j} of the element's state, the same arithmetic as sPA's A (:429-455)
    auto a_of = [&](int r, int c) -> double {
        const double den = sSm[N + N * N + r];
        const double num = sSm[N + r * N + c];
        return (den > 0.0 && num > 0.0) ? num / den : 0.0;
    };
    double ad0 = 0.0, ai0 = 0.0;
    if constexpr (PT && kSameState) {
        ad0 = a_of(jj0, jj0);
        ai0 = jj0 >= 1 ? a_of(jj0 - 1, jj0) : 0.0;
    }
    double bval[SB];
#pragma unroll
    for (int q = 0; q < SB; ++q) {
        const int e = q * BLK + e0;
        const int jj = kSameState ? jj0 : ((e % N) + N) % N;
        const double inv = kSameState ? inv0 : mstep_inv(sSm[N + N * N + N + jj]);
        bval[q] = bnum_to_b(v[q], inv);
        if (e >= 0 && e < K * N) {
            const int i = (e / N) * GP + jj;
            if constexpr (PT) {
                const double ad = kSameState ? ad0 : a_of(jj, jj);
                const double ai = kSameState ? ai0 : (jj >= 1 ? a_of(jj - 1, jj) : 0.0);
                tab_put<PT, GP>(sP, sH, i, ad * bval[q], ai * bval[q], bval[q]);  // histogram zeroed, b
            } else {
                tab_put<PT, GP>(sP, sH, i, 0.0, 0.0, bval[q]);
            }
        }
    }
    if (w0) {
#pragma unroll
        for (int q = 0; q < SB; ++q) {
            const int e = q * BLK + e0;
            if (e >= 0 && e < K * N) {
                const int k = e / N, jj = e - k * N;
                m.B[(long long)jj * K + k] = bval[q];
                m.Bt[(long long)k * G + jj] = bval[q];
            }
        }
    }
    PHASE(10);
    // zero the pad columns [N, GP) of every row (products, histogram, b)
    if constexpr (GP > N) {
        for (int i = tid; i < K * (GP - N); i += BLK) {
            const int k = i / (GP - N), c = N + (i - k * (GP - N));
            tab_put<PT, GP>(sP, sH, k * GP + c, 0.0, 0.0, 0.0);
        }
    }
    __syncthreads();
    double S = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) S += sSum[w];
    const double L = m.local_lse ? ((S > 0.0) ? Mb + log(S) : -INFINITY) : sLr;
    const double diff = (sIn.prev_L != -INFINITY) ? fabs(L - sIn.prev_L) : INFINITY;  // :505-508
    const bool cont = (diff >= sIn.epsilon) && (sIn.iteration + 1 < sIn.max_iterations);  // :346
    if (w0) {
        if (tid < N) m.pi[tid] = sPA[tid];
        if (tid < N * N) m.A[tid] = sPA[G + tid];
        if (tid == 0) record_iteration(m, sIn, L);
    }
    return cont;
}

}  // namespace hmmbw
