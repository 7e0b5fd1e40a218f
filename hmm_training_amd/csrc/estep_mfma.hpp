// estep_mfma.hpp — E-step / scorer for 16 < N <= 64 states on the fp64 matrix cores (gfx950).
//
// Replaces the per-utterance forward / backward loops of HMM/hmm_training.py:351-410
// (calculate_log_alpha :122-160, calculate_log_beta :163-199, gamma :388-394, xi :396-410) and the
// forward-only scorer of HMM/hmm_testing.py:49-104 for the dense large-state models (BASELINE cfg5:
// N=64, K=1024, T=400).
//
// Mapping.  A workgroup owns a TILE of 16 sequences (the MFMA column dimension) and has NT = NP/16
// waves; wave m owns the 16-state block [16m, 16m+16) of the (zero-padded) state vector.  With
// v_mfma_f64_16x16x4_f64 (C/D: col = lane&15, row = (lane>>4) + 4*reg; A/B one f64 per lane, A[l&15][l>>4],
// B[l>>4][l&15]) a 16x16 block of Z^T = [state][sequence] in C/D form is exactly the B operand of the
// next product over states, so the recursions never move data across lanes:
//   forward   Zt^T[o, s] = sum_i A[i][o] Z_{t-1}^T[i, s]           (16-state block m: 4NT MFMAs)
//   backward  beta_t[i, s] = sum_j A[i][j] V_{t+1}[j, s]            (4NT MFMAs)
//   xi        S[i][j] += sum_s z_t[i, s] V_{t+1}[j, s]               (NT x 4 MFMAs: k = sequence)
// Lane (s = lane&15, g = lane>>4) holds states 16m + g + 4r (r = 0..3) of sequence s.  The blocks of
// the other waves come through a double-buffered LDS image [state][16] (row stride 17 doubles: both the
// C/D-form and the transposed reads of the xi operands are bank-conflict free), one s_barrier per step.
//
// Numerics (same scaled-linear fp64 scheme as the small kernel): z_t = x_t 2^{-s_t} with
// the exact power-of-two s_t = (largest biased exponent of z_{t-1} over the sequence's states) - 1023,
// so z stays within one step's growth of 1 (no lag, no fallback needed); log P = log(sum z_{T-1}) +
// ln2 * sum s_t; the backward uses Rabiner scaling with the same s_t.  alpha_hat (fp64) and s_t go to
// HBM in the forward and come back in the backward (the recursions here are bound by the fp64 matrix
// rate, not by these bytes).
//
// B numerator (:474-485).  With K = 1024 symbols x 64 states the per-symbol histogram (512 KB) cannot
// live in LDS, and scattering every gamma_t(j) into it with global fp64 atomics costs more than the
// whole forward.  Instead each gamma row (one position, NP states, bt_col order) is stored once to a
// per-position buffer, and k_bnum_gather (one workgroup per symbol, the host's symbol -> positions
// index) sums the rows of each symbol: deterministic, and HBM-streaming rather than atomic-bound.
#pragma once

#include "hmmbw_device.hpp"

namespace hmmbw {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kTileSeqs = 16;  // sequences per tile = MFMA columns
// The gamma rows (1.28 GB per cfg5-shard iteration, written once by the E-step, read once by the gather)
// move with nontemporal stores and loads: E-step + gather 1,714 -> 1,672 us (the gather 233 -> 193 us).
#ifndef HMMBW_GAMMA_NT
#define HMMBW_GAMMA_NT 1
#endif
// alpha_hat (written by the forward, read once by the backward) likewise: E-step 1,480-1,488 -> 1,476-1,481 us
// The work queue hands alpha_hat and s_t from the forward unit to the backward unit with agent-scope
// stores / loads (write-through past the non-coherent XCD L2s; the flag follows vmcnt(0)) instead of a
// release fence (an XCD-wide L2 write-back per forward unit) and an acquire (an L2 invalidate per
// backward unit): whole cfg5 11.78 -> 11.57 ms per iteration (profiles/r4/wide_work_queue_ab.txt).
#ifndef HMMBW_WQ_WT
#define HMMBW_WQ_WT 1
#endif
#ifndef HMMBW_ALPHA_NT
#define HMMBW_ALPHA_NT 1
#endif

// Profiling ablations of the inner loops (results wrong by construction) exist only in a diagnostics
// build (-DHMMBW_WIDE_ABLATE): a runtime test inside the step loops costs the release build its
// counted vmcnt waits (the join points after such branches drain every prefetch with vmcnt(0)).
#ifdef HMMBW_WIDE_ABLATE
#define WIDE_ABL(a, bit) (((a).ablate & (bit)) != 0)
#elif defined(HMMBW_WIDE_ABLATE_CT)  // compile-time mask: the ablated build keeps the release schedule
#define WIDE_ABL(a, bit) ((HMMBW_WIDE_ABLATE_CT & (bit)) != 0)
#else
#define WIDE_ABL(a, bit) false
#endif
constexpr int kXs = 17;        // LDS row stride (doubles) of a [state][16 sequences] image

// every helper lambda of the kernel is force-inlined: a lambda left out of line keeps the f64x4
// state it captures by reference (beta, gamma sums) in scratch memory
#define HMMBW_AI __attribute__((always_inline))

// max over the 4 rows (16 lanes each) of a wave, for every in-row lane: one v_permlane16_swap (rows
// 0<->1, 2<->3) and one v_permlane32_swap (halves); each returns the pair (own, partner)
__device__ __forceinline__ int row_max4(int x) {
    const auto r16 = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
    x = max((int)r16[0], (int)r16[1]);
    const auto r32 = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
    return max((int)r32[0], (int)r32[1]);
}

__device__ __forceinline__ f64x4 mfma_f64(double a, double b, f64x4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// DET (deterministic-reduction mode): no floating-point atomics; every statistic of the block's
// prefix [0, off_bnum) is owned by exactly one lane, accumulated in registers in a fixed order and
// stored once into the workgroup's partial a.part[block][off_bnum] (k_det_reduce sums the partials in
// workgroup order; the B numerator is the gather's, deterministic already).
// WQ (work queue): 2 ntile workgroups, each taking the next work unit from a counter as it starts:
// units [0, ntile) are the tiles' forward sweeps, [ntile, 2 ntile) their backward sweeps, each backward
// waiting for its tile's forward (a per-tile flag; alpha_hat and s_t pass through HBM, released at agent
// scope).  The dispatcher starts a workgroup wherever one finished, so with more tiles than CUs the CUs'
// loads even out in units of a sweep instead of a whole tile (cfg5 shard: 391 tiles on 256 CUs left 135
// CUs two tiles and the others one).  A unit only waits for a unit taken before it, by a workgroup that
// is running, so the waits always end.
template <int NT, bool FWD_ONLY, bool DET = false, bool WQ = false>
__global__ void __launch_bounds__(NT * 64, 2) k_estep_mfma(EArgs a) {  // 2 waves per SIMD: <= 256 VGPRs
    static_assert(!(DET && FWD_ONLY), "deterministic mode is an E-step option");
    static_assert(!WQ || (!DET && !FWD_ONLY), "the work queue is an E-step option (atomic statistics)");
    constexpr int NP = 16 * NT, KB = 4 * NT, IMG = NP * kXs, IMGX = 2 * IMG;
    extern __shared__ __attribute__((aligned(256))) double smem[];  // 256-B aligned whatever the static LDS (ds_read_b128 rows)
    // [2][2 NP][kXs]: z (forward) / v (backward) images, every row stored twice (rows r and r + NP), so that
    // wave m reads the other blocks in the order 16m + 16, ..., 16m + NP - 1 without wrapping (below)
    double *X0 = smem;
    double *Z0 = smem + 2 * IMGX;                        // [2][NP][kXs] masked z (backward xi operand)
    double *sRed = smem + (FWD_ONLY ? 2 * IMGX : 2 * IMGX + 2 * IMG);  // [NT][16] partial sums + block LL scratch
    if constexpr (!FWD_ONLY)  // clear the next iteration's statistics (single rank: triple buffer)
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < a.zero_len;
             i += (long long)gridDim.x * blockDim.x)
            a.zero[i] = 0.0;
    if (a.state != nullptr && a.state->done) return;    // converged: device-side no-op (:346)
    CHUNKSTAMP(0, 62);  // diagnostics build only (tools/wide_chunk_times.py): shader-clock stamps per chunk
    const int tid = threadIdx.x, lane = tid & 63, m = tid >> 6;
    const int s = lane & 15, g = lane >> 4;
    const int N = a.N;
    const long long ntile = WQ ? (long long)a.wq_units : (long long)gridDim.x;
    bool do_f = true;  // this workgroup runs the tile's forward sweep ...
    bool do_b = true;  // ... and its backward sweep
    long long tile = blockIdx.x;
    if constexpr (WQ) {
        __shared__ int s_unit;
        if (tid == 0) s_unit = (int)atomicAdd(a.wq, 1u);
        __syncthreads();
        const long long u = s_unit;
        do_f = u < ntile;
        do_b = !do_f;
        tile = do_f ? u : u - ntile;
    }
    const long long slot = tile * kTileSeqs + s;
    const int T = a.L.slot_len[slot];
    const int seq = a.L.slot_seq[slot];
    const int Tw = a.L.wave_T[tile];
    const bool full = a.L.wave_full[tile] != 0;          // every sequence of the tile has length Tw
    const int nch = (Tw + kChunk - 1) / kChunk;
    const uint16_t *symw = a.L.sym + a.L.wave_symoff[tile] + s * kChunk;
    double *ckw = a.ckpt + (FWD_ONLY ? 0 : a.L.wave_ckoff[tile]) + (long long)m * 4 * 64 + lane;
    int *ew = a.ebuf + (FWD_ONLY ? 0 : a.L.wave_spoff[tile]) + s;
    const int col0 = 16 * m + 4 * g;  // this lane's 4 emission columns (bt_col order)
    // gamma row of position (t, s): row gdw[t * 16] of the symbol-sorted row buffer (the host's
    // position -> rank map), so that k_bnum_gather streams each symbol's rows contiguously
    const unsigned *gdw = a.gdst + (FWD_ONLY ? 0 : a.L.wave_ckoff[tile] / NP) + s;
    auto putg = [&](unsigned row, const f64x4 &v) HMMBW_AI {
        double2 *q = reinterpret_cast<double2 *>(a.gam + (long long)row * NP + col0);
        if constexpr (HMMBW_GAMMA_NT) {  // written once here, read once by the gather
            typedef double d2 __attribute__((ext_vector_type(2)));
            d2 *qq = reinterpret_cast<d2 *>(q);
            __builtin_nontemporal_store(d2{v[0], v[1]}, qq);
            __builtin_nontemporal_store(d2{v[2], v[3]}, qq + 1);
        } else {
            q[0] = double2{v[0], v[1]};
            q[1] = double2{v[2], v[3]};
        }
    };

    auto loadpack = [&](int c) HMMBW_AI -> uint4 {
        return *reinterpret_cast<const uint4 *>(symw + (long long)c * kTileSeqs * kChunk);
    };
    auto emis = [&](int o) HMMBW_AI -> f64x4 {  // b_j(o) for j = 16m + g + 4r, r = 0..3
        const double2 *p = reinterpret_cast<const double2 *>(a.Bt + (long long)o * NP + col0);
        const double2 lo = p[0], hi = p[1];
        return f64x4{lo.x, lo.y, hi.x, hi.y};
    };
    // Backward: own block first.  The recursion contracts over all NP states in k-blocks of 4, and the C/D
    // registers of this wave's block ARE the B operands of its own 4 k-blocks (4m + r: states 16m + 4r + g),
    // so publish issues those 4 MFMAs of the next step's beta straight from registers, before the barrier
    // and the LDS reads of the other waves' blocks, which consume then reads in the rotated order 16m + 16,
    // ..., 16m + NP - 1 (mod NP, hence the doubled v-image rows), with the A operands loaded in the same
    // rotated k-block order (backward 3,210 -> 3,096 cycles per step for a lone tile).  The forward keeps
    // the natural order and one copy: the same reordering there cost 46 cycles per step (its extra LDS
    // writes sit in front of the barrier and its exchange has no independent MFMAs to hide behind).
    double *const putb = X0 + (16 * m + g) * kXs + s;   // this wave's block (put2: both copies)
    auto put1 = [&](int p, const f64x4 &v) HMMBW_AI {
#pragma unroll
        for (int r = 0; r < 4; ++r) putb[p * IMGX + 4 * r * kXs] = v[r];
    };
    auto put2 = [&](int p, const f64x4 &v) HMMBW_AI {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            putb[p * IMGX + 4 * r * kXs] = v[r];
            putb[p * IMGX + NP * kXs + 4 * r * kXs] = v[r];
        }
    };
    double *const putz = Z0 + (16 * m + g) * kXs + s;
    auto putzs = [&](int p, const f64x4 &v) HMMBW_AI {
#pragma unroll
        for (int r = 0; r < 4; ++r) putz[p * IMG + 4 * r * kXs] = v[r];
    };
    const double *const bopb = X0 + g * kXs + s;             // + 4 kb kXs: k-block kb of image p (forward)
    const double *const bopr = X0 + (16 * m + g) * kXs + s;  // + 4 kb' kXs: rotated k-block kb' (>= 4) of image p
    const double *const topb = X0 + (lane & 15) * kXs + (lane >> 4);
    const double *const topz = Z0 + (lane & 15) * kXs + (lane >> 4);
    auto bexp = [](double x) HMMBW_AI -> int { return (int)__builtin_amdgcn_ubfe((unsigned)__double2hiint(x), 20, 11); };
    // sum over the 16 sequences of a 16-lane row
    auto rowsum = [](double x) HMMBW_AI -> double {
#pragma unroll
        for (int q = 1; q < kTileSeqs; q <<= 1) x += __shfl_xor(x, q);
        return x;
    };

    // forward A operands of this wave's 16-state block: A^T[o][i] = a_io (o = 16m + (lane&15),
    // i = 4kb + (lane>>4))
    double aop[KB];
    if (do_f) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            const int o = 16 * m + (lane & 15), i = 4 * kb + (lane >> 4);
            aop[kb] = (i < N && o < N) ? a.A[i * N + o] : 0.0;
        }
    }

    // ---------------- forward (hmm_training.py:357-368; hmm_testing.py:70-92) ----------------
    f64x4 z = {0.0, 0.0, 0.0, 0.0};
    int C = 0;
    // b(o_t) in slot t % 4, loaded kLook steps ahead; symbol packs one chunk ahead of their use
    constexpr int kLook = 3;
    f64x4 bring[4];
    // STEADY: a step of a chunk in which every step runs (t >= 1): no branch in the step, so the
    // compiler can count the in-flight prefetches and stores (a conditional block makes it wait for
    // them: gfx9 counts stores in vmcnt)
    auto fstep = [&](int t, const f64x4 &b, auto MASK_, auto STEADY_) HMMBW_AI {
        constexpr bool MASK = decltype(MASK_)::value;
        constexpr bool STEADY = decltype(STEADY_)::value;
        f64x4 x;
        int sc = 0;
        if (!STEADY && t == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = 16 * m + g + 4 * r;
                x[r] = (j < N && T > 0) ? a.pi[j] * b[r] : 0.0;  // pi_j b_j(o_0) (:357-360)
            }
        } else {
            const double *src = bopb + ((t - 1) & 1) * IMGX;
            double zb[KB];
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) zb[kb] = src[4 * kb * kXs];
            // one accumulation chain: a dependent v_mfma_f64_16x16x4 issues every 64 cycles, its full
            // rate (tools/ubench_mfma.hip), and a second chain would cost 8 VGPRs
            f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) acc = mfma_f64(aop[kb], zb[kb], acc);
            // s_t from z_{t-1} over all NP states of the sequence (4 lanes x KB values)
            int M = 0;
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) M = max(M, bexp(zb[kb]));
            // across the 4 lane rows: gfx950's row-swap permutes are VALU ops (ds_bpermute put two LDS
            // round trips in front of the MFMA chain, which the compiler schedules after them)
            M = row_max4(M);
            // the exponent's VALU work between the chain's MFMAs (each waits ~64 cycles for the last)
            // instead of in front of the first one
            __builtin_amdgcn_sched_group_barrier(0x100, KB / 2, 0);
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            }
            sc = M == 0 ? 0 : M - 1023;
            // rescale before the emission factor: z_{t-1} and b(o_t) may both be ~1e-200 (no underflow)
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = __builtin_amdgcn_ldexp(acc[r], -sc) * b[r];
        }
        if constexpr (MASK) {
            const bool act = t < T;  // past the sequence's end: z frozen at z_{T-1}
#pragma unroll
            for (int r = 0; r < 4; ++r) z[r] = act ? x[r] : z[r];
            sc = act ? sc : 0;
        } else {
            z = x;
        }
        C += sc;
        put1(t & 1, z);
        if constexpr (!FWD_ONLY) {
            if (!WIDE_ABL(a, 8)) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if constexpr (WQ && HMMBW_WQ_WT)
                        __hip_atomic_store(&ckw[((long long)t * NT * 4 + r) * 64], z[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    else if constexpr (HMMBW_ALPHA_NT) __builtin_nontemporal_store(z[r], &ckw[((long long)t * NT * 4 + r) * 64]);
                    else ckw[((long long)t * NT * 4 + r) * 64] = z[r];
                }
            }
            // every wave computes the same s_t from all NP states: one lane group stores it (STEADY: all
            // lanes, the same value to the same 16 words, so the store needs no exec branch)
            if (STEADY || (m == 0 && g == 0)) {
                if constexpr (WQ && HMMBW_WQ_WT) __hip_atomic_store(&ew[t * kTileSeqs], sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else ew[t * kTileSeqs] = sc;
            }
        }
        if (!WIDE_ABL(a, 16)) __syncthreads();
    };
    uint4 p0, p1;  // symbol packs of chunks c and c + 1
    auto fchunk = [&](int c, auto MASK_, auto STEADY_) HMMBW_AI {
        constexpr bool STEADY = decltype(STEADY_)::value;
        CHUNKSTAMP(0, c);
        const uint4 p2 = loadpack(c + 2 < nch ? c + 2 : nch - 1);
#pragma unroll
        for (int k = 0; k < kChunk; ++k) {
            const int t = c * kChunk + k;
            // b(o_{t + kLook}) into the slot step t - 1 has consumed
            bring[(k + kLook) & 3] = emis(k + kLook < kChunk ? sym_of(p0, k + kLook) : sym_of(p1, k + kLook - kChunk));
            if (!STEADY && t >= Tw) continue;  // tile-uniform
            fstep(t, bring[k & 3], MASK_, STEADY_);
        }
        p0 = p1;
        p1 = p2;
    };
    auto forward = [&](auto MASK_) HMMBW_AI {
        p0 = loadpack(0);
        p1 = loadpack(nch > 1 ? 1 : 0);
#pragma unroll
        for (int i = 0; i < kLook; ++i) bring[i] = emis(sym_of(p0, i));
        const int cf = Tw / kChunk;  // chunks [1, cf) run all their steps
        fchunk(0, MASK_, std::false_type{});
        for (int c = 1; c < cf; ++c) fchunk(c, MASK_, std::true_type{});
        for (int c = cf > 1 ? cf : 1; c < nch; ++c) fchunk(c, MASK_, std::false_type{});
    };
    if (do_f) {
        if (full) forward(std::false_type{});
        else forward(std::true_type{});
    } else if constexpr (WQ) {
        // backward unit: wait for the tile's forward (it runs on a resident workgroup, so the wait ends),
        // then z_{Tw-1} (masked per sequence, as the forward left it in its registers) from alpha_hat.
        // The wait is bounded (HMMBW_OPT_WQ_TIMEOUT_MS, wall-clock ticks from the host): past it the unit
        // records HMMBW_E_TIMEOUT in the iteration state, stops EM (done: the gather, the M-step and every
        // later launch become no-ops, the status calls return the error) and skips its backward sweep, as
        // the peer all-reduce does; it never reads an alpha_hat that may not be there.  A 0-ms bound
        // expires before the first look at the flag.
        __shared__ int s_ok;
        if (tid == 0) {
            const unsigned long long t0 = wall_clock64();
            int ok = 1;
            while (true) {
                if ((long long)(wall_clock64() - t0) >= a.wq_timeout_ticks) {
                    ok = 0;
                    break;
                }
                if (__hip_atomic_load(a.wq_flag + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
                __builtin_amdgcn_s_sleep(8);
            }
            if (!ok) {
                IterState *st = const_cast<IterState *>(a.state);
                __hip_atomic_store(&st->error, (int)HMMBW_E_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&st->error_src, kErrWorkQueue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&st->done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            s_ok = ok;
        }
        __syncthreads();
        do_b = s_ok != 0;
        if constexpr (!HMMBW_WQ_WT) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (do_b && Tw > 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double *q = &ckw[((long long)(Tw - 1) * NT * 4 + r) * 64];
                if constexpr (HMMBW_WQ_WT) z[r] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if constexpr (HMMBW_ALPHA_NT) z[r] = __builtin_nontemporal_load(q);
                else z[r] = *q;
            }
        }
    }

    CHUNKSTAMP(0, 61);
    // log P(O|lambda) = log(sum_j z_{T-1}(j)) + ln2 * C   (:375-377)
    double ps = (z[0] + z[1]) + (z[2] + z[3]);
    ps += __shfl_xor(ps, 16);
    ps += __shfl_xor(ps, 32);
    if (g == 0) sRed[m * kTileSeqs + s] = ps;
    __syncthreads();
    double phat = 0.0;
#pragma unroll
    for (int mm = 0; mm < NT; ++mm) phat += sRed[mm * kTileSeqs + s];
    const bool alive = (T > 0) && (phat > 0.0);
    const double lp = alive ? (log(phat) + (double)C * 0.69314718055994530942) : -INFINITY;
    if (do_f && m == 0 && g == 0 && T > 0 && seq >= 0) a.logp[seq] = lp;
    const bool ll_valid = (m == 0) && (g == 0) && (T > 0);

    if constexpr (!FWD_ONLY) if (do_b && !(a.ablate & 2)) {
        // ------------- backward fused with gamma / xi / M-step numerators (:370-410, :474-485) -------------
        double *accb = a.copies + (long long)(blockIdx.x % a.ncopies) * a.copy_len;
        double dgall[4] = {0.0, 0.0, 0.0, 0.0}, dpin[4] = {0.0, 0.0, 0.0, 0.0};  // DET: this lane's sums
        const double inv_p = alive ? 1.0 / phat : 0.0;  // beta_hat_{T-1}: folds 1/P (:392, :407)
        // gamma_{T-1} = z_{T-1} / P (:392 at t = T-1): its gamma row, gamma_den_all, pi_num when T = 1
        {
            f64x4 gT;
#pragma unroll
            for (int r = 0; r < 4; ++r) gT[r] = z[r] * inv_p;
            if (T > 0 && !WIDE_ABL(a, 4)) putg(gdw[(T - 1) * kTileSeqs], gT);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = 16 * m + g + 4 * r;
                const double x1 = rowsum(gT[r]), x2 = rowsum(T == 1 ? gT[r] : 0.0);
                if constexpr (DET) {
                    dgall[r] = x1;
                    dpin[r] = x2;
                } else if (s == 0 && j < N) {
                    if (x1 != 0.0) unsafeAtomicAdd(&accb[a.off_gall + j], x1);
                    if (x2 != 0.0) unsafeAtomicAdd(&accb[j], x2);  // pi_num at offset 0
                }
            }
        }
        // backward A operands A[i][j] (i = 16m + (lane&15), j = 4kb + (lane>>4))
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {  // rotated k-block order, as the forward's
            const int i = 16 * m + (lane & 15), jj = 4 * ((kb + 4 * m) % KB) + (lane >> 4);
            aop[kb] = (i < N && jj < N) ? a.A[i * N + jj] : 0.0;
        }
        f64x4 beta = {inv_p, inv_p, inv_p, inv_p};
        double gex[4] = {0.0, 0.0, 0.0, 0.0};  // plain array: an f64x4 with element-wise updates stays in scratch
        f64x4 S[NT];
#pragma unroll
        for (int mm = 0; mm < NT; ++mm) S[mm] = f64x4{0.0, 0.0, 0.0, 0.0};
        // rings (two slots each, indexed by step parity: fewer VGPRs, two waves per SIMD): alpha_hat_t
        // (HBM), loaded two visits before the publish that uses it; b(o_t) (L2-resident table) and s_t,
        // loaded one visit before
        f64x4 zring[2], bring1[2];
        int sring[2];
        unsigned dring[2];  // gamma row of step t in slot t % 2, loaded in the visit before consume(t)
        f64x4 zs;  // z_t masked to the regular steps: gamma_t of the step that consumes the image
        f64x4 accn;  // beta of the next step to consume: its own-block MFMAs, issued by publish
        auto ldew = [&](int t) HMMBW_AI -> int {
            if constexpr (WQ && HMMBW_WQ_WT) return __hip_atomic_load(&ew[t * kTileSeqs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else return ew[t * kTileSeqs];
        };
        auto ldz = [&](int t) HMMBW_AI -> f64x4 {
            f64x4 v;
            if (WIDE_ABL(a, 8)) return f64x4{0.5, 0.5, 0.5, 0.5};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if constexpr (WQ && HMMBW_WQ_WT)
                    v[r] = __hip_atomic_load(&ckw[((long long)t * NT * 4 + r) * 64], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if constexpr (HMMBW_ALPHA_NT) v[r] = __builtin_nontemporal_load(&ckw[((long long)t * NT * 4 + r) * 64]);
                else v[r] = ckw[((long long)t * NT * 4 + r) * 64];
            }
            return v;
        };
        // publish(t): the image of step t <= Tw - 2 (MASK: per-sequence t <= T - 2 in ragged tiles) into
        // LDS buffer t % 2: v_{t+1}(j) = b_j(o_{t+1}) 2^{-s_{t+1}} beta_hat_{t+1}(j) (:182-197) and z_t
        auto publish = [&](int t, const f64x4 &zt, const f64x4 &b1, int s1, auto MASK_) HMMBW_AI {
            constexpr bool MASK = decltype(MASK_)::value;
            const bool reg = !MASK || t <= T - 2;
            f64x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = __builtin_amdgcn_ldexp(b1[r] * beta[r], -s1);
                if constexpr (MASK) {
                    v[r] = reg ? v[r] : 0.0;
                    zs[r] = reg ? zt[r] : 0.0;
                } else {
                    zs[r] = zt[r];
                }
            }
            put2(t & 1, v);
            putzs(t & 1, zs);
            // the own-block part of beta_hat_t = A v_{t+1}: this wave's v is its own k-blocks' B operand
            accn = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int r = 0; r < 4; ++r) accn = mfma_f64(aop[r], v[r], accn);
        };
        // consume(t): after the barrier, beta_hat_t = A v_{t+1} (:163-199, this wave's 16 rows), gamma_t,
        // then the xi MFMAs of the same image.  The xi products are off the beta chain: they are made
        // to follow it (a register dependency on beta_t), so that the next step's image is computed
        // and published (VALU, LDS writes) between them instead of after them, and the wave reaches
        // the next barrier right after its last MFMA issues.
        auto consume = [&](int t, unsigned grow, auto MASK_, auto STEADY_, auto &&next) HMMBW_AI {
            constexpr bool MASK = decltype(MASK_)::value;
            constexpr bool STEADY = decltype(STEADY_)::value;
            const bool reg = !MASK || t <= T - 2;
            const int p = t & 1;
            if (!WIDE_ABL(a, 16)) __syncthreads();
            const double *vsrc = bopr + p * IMGX;
            f64x4 acc = accn;  // own blocks done (publish), the other waves' blocks now
#pragma unroll
            for (int kb = 4; kb < KB; ++kb) acc = mfma_f64(aop[kb], vsrc[4 * kb * kXs], acc);
            // S_ij += sum_s z_t(i, s) v_{t+1}(j, s): xi_t(i,j) / a_ij (:396-410)
            const double *tsrc = topb + p * IMGX;
            double za[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) za[kk] = topz[p * IMG + 16 * m * kXs + 4 * kk];
            asm volatile("" : "+v"(za[0]) : "v"(acc[0]));  // xi after the beta chain (see above)
            f64x4 gm;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double bn = acc[r];
                gm[r] = zs[r] * bn;  // gamma_t (:392); 0 past the sequence's end
                if constexpr (MASK) beta[r] = reg ? bn : beta[r];
                else beta[r] = bn;
                gex[r] += gm[r];
            }
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int mj = 0; mj < NT; ++mj) S[mj] = mfma_f64(za[kk], tsrc[16 * mj * kXs + 4 * kk], S[mj]);
            if ((!MASK || reg) && !WIDE_ABL(a, 4)) putg(grow, gm);  // B numerator row (:474-485)
            if (!STEADY && t == 0) {  // pi_num (:415-420): gamma_0 summed over the tile's sequences
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = 16 * m + g + 4 * r;
                    const double x = rowsum(gm[r]);
                    if constexpr (DET) dpin[r] += x;
                    else if (s == 0 && j < N && x != 0.0) unsafeAtomicAdd(&accb[j], x);
                }
            }
            next();  // publish(t - 1), when there is a step t - 1
        };
        uint4 pc;  // chunk c's symbol pack; chunk c - 1's is loaded at the top of chunk c
        // visit t: consume(t) for t <= Tw - 2, publish(t - 1) for 1 <= t <= Tw - 1 (with b(o_t), s_t
        // from slot t % 2), then b(o_{t-1}), s_{t-1} and alpha_hat_{t-3} into the slots just consumed
        auto bchunk = [&](int c, auto MASK_, auto STEADY_) HMMBW_AI {
            constexpr bool STEADY = decltype(STEADY_)::value;  // c >= 1 and every step t <= Tw - 2
            CHUNKSTAMP(1, c);
            const uint4 pp = loadpack(c >= 1 ? c - 1 : 0);
#pragma unroll
            for (int k = kChunk - 1; k >= 0; --k) {
                const int t = c * kChunk + k;
                auto pub = [&]() HMMBW_AI {
                    if (STEADY || (t >= 1 && t <= Tw - 1))
                        publish(t - 1, zring[(k + 1) & 1], bring1[k & 1], sring[k & 1], MASK_);
                };
                // tile-uniform; gamma_{T-1} is done above
                if (STEADY || t <= Tw - 2) consume(t, dring[k & 1], MASK_, STEADY_, pub);
                else pub();
                if (STEADY || t >= 1) dring[(k + 1) & 1] = gdw[(t - 1) * kTileSeqs];  // row of step t - 1
                if (STEADY || t >= 2) {
                    bring1[(k + 1) & 1] = emis(k >= 1 ? sym_of(pc, k - 1) : sym_of(pp, kChunk - 1));  // b(o_{t-1})
                    sring[(k + 1) & 1] = ldew(t - 1);  // s_{t-1}
                }
                if (STEADY || t >= 3) zring[(k + 1) & 1] = ldz(t - 3);
            }
            pc = pp;
        };
        auto backward = [&](auto MASK_) HMMBW_AI {
            const int ttop = nch * kChunk;  // steps ttop - 1 .. 0 are visited (those > Tw - 2 skip)
            pc = loadpack(nch - 1);
            // alpha_hat for the first two visits' publish: z_{ttop-2}, z_{ttop-3}
#pragma unroll
            for (int i = 2; i < 4; ++i) {
                const int s0 = ttop - i;
                zring[s0 & 1] = s0 >= 0 ? ldz(s0) : f64x4{0.0, 0.0, 0.0, 0.0};
            }
            // b(o_{ttop-1}), s_{ttop-1} for the first visit (slot 1: ttop - 1 is odd)
            bring1[1] = emis(sym_of(pc, kChunk - 1));
            sring[1] = ldew(ttop - 1);
            dring[1] = gdw[(ttop - 1) * kTileSeqs];
            // chunks [1, cs] have every step t <= Tw - 2 (c * kChunk + kChunk - 1 <= Tw - 2)
            const int cs = Tw >= kChunk + 1 ? (Tw - kChunk - 1) / kChunk : 0;
            int c = nch - 1;
            for (; c > cs && c >= 1; --c) bchunk(c, MASK_, std::false_type{});
            for (; c >= 1; --c) bchunk(c, MASK_, std::true_type{});
            bchunk(0, MASK_, std::false_type{});
        };
        if (full) backward(std::false_type{});
        else backward(std::true_type{});
        CHUNKSTAMP(1, 62);
        // ---- flush: xi = a_ij S_ij; gamma sums reduced over the tile's sequences ----
        double *part = DET ? a.part + (long long)blockIdx.x * a.off_bnum : nullptr;
#pragma unroll
        for (int mj = 0; mj < NT; ++mj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * m + g + 4 * r, jj = 16 * mj + (lane & 15);
                if constexpr (DET) {
                    if (i < N && jj < N) part[a.off_S + (long long)i * N + jj] = S[mj][r] * a.A[i * N + jj];
                } else if (i < N && jj < N && S[mj][r] != 0.0) {
                    const double x = S[mj][r] * a.A[i * N + jj];
                    if (x != 0.0) unsafeAtomicAdd(&accb[a.off_S + (long long)i * N + jj], x);
                }
            }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double x0 = rowsum(gex[r]);
            const int j = 16 * m + g + 4 * r;
            if constexpr (DET) {
                if (s == 0 && j < N) {
                    part[j] = dpin[r];
                    part[a.off_gex + j] = x0;
                    part[a.off_gall + j] = dgall[r] + x0;
                }
            } else if (s == 0 && j < N && x0 != 0.0) {
                unsafeAtomicAdd(&accb[a.off_gex + j], x0);
                unsafeAtomicAdd(&accb[a.off_gall + j], x0);  // gamma_den_all = excl + the last frames
            }
        }
    }
    if constexpr (WQ) {
        if (do_f) {  // the tile's log P pair, then the release of alpha_hat and s_t to its backward unit
            __syncthreads();
            block_ll_partial(lp, ll_valid, sRed + NT * kTileSeqs, a.llpart + 2 * tile);
            if constexpr (HMMBW_WQ_WT) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the stores have landed
            else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __syncthreads();
            if (tid == 0) __hip_atomic_store(a.wq_flag + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (a.rank_ll != nullptr) {
            __syncthreads();
            int ticket = 0;
            if (threadIdx.x == 0) ticket = rank_ll_count(a);
            if ((threadIdx.x >> 6) == 0 && __shfl(ticket, 0) == (int)(ntile - 1)) rank_ll_fold(a, ntile);
        }
        // the last workgroup out re-arms the queue and the flags for the next launch
        __shared__ int s_last;
        if (tid == 0) s_last = atomicAdd(a.wq + 1, 1u) == gridDim.x - 1;
        __syncthreads();
        if (s_last) {
            for (long long i = tid; i < ntile; i += blockDim.x) a.wq_flag[i] = 0u;
            if (tid == 0) {
                a.wq[0] = 0u;
                a.wq[1] = 0u;
            }
        }
        return;
    }
    __syncthreads();
    block_ll_partial(lp, ll_valid, sRed + NT * kTileSeqs, a.llpart + 2 * (long long)blockIdx.x);
    if constexpr (!DET && !FWD_ONLY) {
        // fused multi-rank launch (hmmbw_iterate / hmmbw_iterate_begin): the statistics went straight
        // into the all-reduce buffer; the last tile to finish folds the tiles' (max, sum exp) pairs
        // into this rank's slot (as the small kernels do), so no k_reduce_local pass is needed
        if (a.rank_ll != nullptr) {
            int ticket = 0;
            if (threadIdx.x == 0) ticket = rank_ll_count(a);
            if ((threadIdx.x >> 6) == 0 && __shfl(ticket, 0) == (int)(gridDim.x - 1)) rank_ll_fold(a, gridDim.x);
        }
    }
    CHUNKSTAMP(1, 63);
}

// B numerator of the wide kernels (:474-485): B_num[k][j] = sum of the gamma rows of every position
// whose symbol is k (rows[ptr[k] .. ptr[k+1]): row indices into the gamma buffer, NP doubles each,
// bt_col order).  One workgroup per symbol, lane = column; it walks the list in batches of 256
// positions: wave w's lane l loads the row index of position 64 w + l of the batch (one coalesced load,
// the next batch's prefetched), then the wave streams those 64 rows, 16 loads in flight, with the row
// index broadcast from its lane (readlane: the row base is a scalar).  Fixed order (each wave sums its
// positions in list order, the four waves in wave order), plain stores into the symbol-major [K][N]
// statistics block.  Also the small kernels' deterministic mode (NP = G columns in state order,
// perm = 0).  Round 3: 234.5 us at the cfg5 shard against 237.0 for one index load per 4 rows.
// SORTED (the wide path): the E-step wrote every position's row at its rank in symbol order, so symbol k's
// rows are the contiguous rows [ptr[k], ptr[k+1]) and the walk is a stream (no row index to load).
template <bool SORTED>
__global__ void __launch_bounds__(256) k_bnum_gather(const double *gam, const unsigned *rows, const long long *ptr,
                                                       int NP, int N, int perm, double *bnum, const IterState *state) {
    __shared__ double sh[4][64];
    if (state != nullptr && state->done) return;
    const int k = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long b = ptr[k], e = ptr[k + 1];
    const int q = lane < NP ? lane : 0;
    constexpr int U = 16;
    auto ldidx = [&](long long p0) -> unsigned {
        const long long p = p0 + 64 * wv + lane;
        return SORTED ? 0u : rows[p < e ? p : b];
    };
    double acc = 0.0;
    unsigned idx = b < e ? ldidx(b) : 0u;
    for (long long p0 = b; p0 < e; p0 += 256) {
        const unsigned cur = idx;
        if (!SORTED && p0 + 256 < e) idx = ldidx(p0 + 256);
        const long long pw = p0 + 64 * wv;  // this wave's first position of the batch
#pragma unroll
        for (int g = 0; g < 64; g += U) {
            double x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const long long r = SORTED ? (pw + g + u < e ? pw + g + u : b) : (long long)__builtin_amdgcn_readlane(cur, g + u);
                if constexpr (HMMBW_GAMMA_NT) x[u] = __builtin_nontemporal_load(&gam[r * NP + q]);
                else x[u] = gam[r * NP + q];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc += (pw + g + u < e) ? x[u] : 0.0;
        }
    }
    sh[wv][lane] = acc;
    __syncthreads();
    if (wv == 0 && lane < NP) {
        const double v = (sh[0][lane] + sh[1][lane]) + (sh[2][lane] + sh[3][lane]);
        const int j = perm ? bt_col(lane) : lane;  // bt_col is an involution: column -> state
        if (j < N) bnum[(long long)k * N + j] = v;
    }
}

}  // namespace hmmbw
