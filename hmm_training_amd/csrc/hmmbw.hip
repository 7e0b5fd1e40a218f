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
//        in LDS; alpha_hat spilled to HBM coalesced (512 B per wave-step) and re-read by the
//        backward sweep, which fuses beta, gamma, xi and the histogram scatter.
//   k_estep_wide<NP,FWD_ONLY>              16 < N <= 64: one sequence per wavefront, lane = state,
//        A / A^T in LDS, alpha / v exchanged through a per-wave LDS row.
//   k_seq_lse   per-rank (max, sum exp) pair of log P_r into the rank's statistics slot.
//   k_mstep     one workgroup: L, M-step, convergence record, zero the statistics.
//   k_finalise  the reference's return-path normalisation (:524-541).
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

constexpr int kWave = 64;
constexpr int kChunk = 8;  // time steps per packed symbol load (8 x uint16 = 16 B)
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
};

// Observation layout in HBM (built once by hmmbw_set_observations).
//   slot = wave * U + u  ->  caller sequence slot_seq[slot] (-1: padding), length slot_len[slot]
//   symbols: per wave, chunk-major [chunk][u][8] uint16  (one 16-B load = 8 steps of one sequence)
//   alpha_hat: per wave [t][64 lanes] fp64 ; exponents: per wave [t][u] int32 (+1 chunk pad)
struct Layout {
    const uint16_t *sym;
    const long long *wave_symoff;
    const long long *wave_aoff;
    const long long *wave_eoff;
    const int *wave_T;
    const int *slot_len;
    const int *slot_seq;
    long long nwaves;
};

struct EArgs {
    Layout L;
    const double *pi;
    const double *A;
    const double *Bt;  // [K][G]
    double *alpha;
    int *ebuf;
    double *stats;
    double *logp;
    const IterState *state;
    int K;
    int N;
    long long off_S, off_gex, off_gall, off_bnum;
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

// Sum over a group of G lanes (butterfly; every lane gets the bitwise-identical result because
// each level adds the same two partial sums, only commuted).
template <int G>
__device__ __forceinline__ double gsum(double x) {
    if constexpr (G >= 2) x += dpp<0xB1>(x);   // quad_perm [1,0,3,2]
    if constexpr (G >= 4) x += dpp<0x4E>(x);   // quad_perm [2,3,0,1]
    if constexpr (G >= 8) x += dpp<0x141>(x);  // row_half_mirror
    if constexpr (G >= 16) x += dpp<0x140>(x); // row_mirror
    if constexpr (G >= 32) x += __shfl_xor(x, 16);
    if constexpr (G >= 64) x += __shfl_xor(x, 32);
    return x;
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

__device__ __forceinline__ int sym_of(const uint4 &p, int s) {
    const unsigned w = s < 2 ? p.x : (s < 4 ? p.y : (s < 6 ? p.z : p.w));
    return (s & 1) ? int(w >> 16) : int(w & 0xFFFFu);
}

__device__ __forceinline__ double pow2_scale(double x, int e) { return __builtin_amdgcn_ldexp(x, -e); }

// ---------------------------------------------------------------------------------------------
// Small-N E-step / scorer.  One G-lane group per sequence.
// ---------------------------------------------------------------------------------------------
template <int N, int G, bool LR, bool LDSTAB, bool FWD_ONLY>
__global__ void __launch_bounds__(kBlock) k_estep_small(EArgs a) {
    constexpr int U = kWave / G;
    constexpr int NS = LR ? 2 : N;      // per-lane S accumulators (row j of S)
    constexpr int NV = NS + 3;          // + gamma_den_excl, gamma_den_all, pi_num
    extern __shared__ double smem[];
    if (a.state != nullptr && a.state->done) return;  // converged: device-side no-op

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int j = lane & (G - 1), u = lane / G;
    const int K = a.K;
    double *sBt = smem;                                  // [K][G]
    double *sBn = LDSTAB ? smem + (size_t)K * G : nullptr; // [K][G]
    double *sRed = smem + (LDSTAB ? 2 : 0) * (size_t)K * G; // [waves][G][NV]
    if constexpr (LDSTAB) {
        for (int i = tid; i < K * G; i += blockDim.x) {
            sBt[i] = a.Bt[i];
            if constexpr (!FWD_ONLY) sBn[i] = 0.0;
        }
    }
    __syncthreads();
    const double *Btab = LDSTAB ? sBt : a.Bt;

    const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + wv;
    double S[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) S[k] = 0.0;
    double gex = 0.0, gall = 0.0, pin = 0.0;

    if (wave < a.L.nwaves) {
        const long long slot = wave * U + u;
        const int T = a.L.slot_len[slot];
        const int seq = a.L.slot_seq[slot];
        const int Tw = a.L.wave_T[wave];
        const int nch = (Tw + kChunk - 1) / kChunk;
        const uint16_t *symw = a.L.sym + a.L.wave_symoff[wave] + u * kChunk;
        double *aw = a.alpha + (FWD_ONLY ? 0 : a.L.wave_aoff[wave]) + lane;
        int *ew = a.ebuf + (FWD_ONLY ? 0 : a.L.wave_eoff[wave]) + u;
        const bool jv = j < N;

        // transition coefficients for this lane (state j)
        double acol[LR ? 1 : N], arow[LR ? 1 : N];
        double a_dg = 0.0, a_in = 0.0, a_up = 0.0;
        if constexpr (LR) {
            a_dg = jv ? a.A[j * N + j] : 0.0;
            a_in = (jv && j >= 1) ? a.A[(j - 1) * N + j] : 0.0;
            a_up = (j + 1 < N) ? a.A[j * N + j + 1] : 0.0;
        } else {
#pragma unroll
            for (int i = 0; i < N; ++i) {
                acol[i] = jv ? a.A[i * N + j] : 0.0;
                arow[i] = jv ? a.A[j * N + i] : 0.0;
            }
        }
        const double pij = jv ? a.pi[j] : 0.0;

        auto loadpack = [&](int c) -> uint4 {
            return *reinterpret_cast<const uint4 *>(symw + (long long)c * U * kChunk);
        };

        // ---------------- forward: alpha_hat_t, e_t  (hmm_training.py:357-368) ----------------
        double alpha = 0.0;
        int E = 0;
        uint4 pk = loadpack(0);
        for (int c = 0; c < nch; ++c) {
            const uint4 pkn = (c + 1 < nch) ? loadpack(c + 1) : pk;
#pragma unroll
            for (int s = 0; s < kChunk; ++s) {
                const int t = c * kChunk + s;
                const int o = sym_of(pk, s);
                const double b = Btab[o * G + j];
                double x;
                if (t == 0) {
                    x = pij * b;                                            // :360
                } else if constexpr (LR) {
                    double prev = dpp<0x111>(alpha);                        // row_shr:1 -> alpha(j-1)
                    prev = (j == 0) ? 0.0 : prev;
                    x = fma(a_in, prev, a_dg * alpha) * b;                 // :141-156
                } else {
                    double acc0 = 0.0, acc1 = 0.0;
                    sfor<0, N>([&](auto I) {
                        const double ai = gbcast<G, I.value>(alpha, lane);
                        if constexpr ((I.value & 1) == 0) acc0 = fma(acol[I.value], ai, acc0);
                        else acc1 = fma(acol[I.value], ai, acc1);
                    });
                    x = (acc0 + acc1) * b;
                }
                const double sum = gsum<G>(x);
                const int e = __builtin_amdgcn_frexp_exp(sum);  // 0 for sum == 0
                x = pow2_scale(x, e);
                if (t < T) {
                    alpha = x;
                    E += e;
                    if constexpr (!FWD_ONLY) {
                        aw[(long long)t * kWave] = x;
                        if (j == 0) ew[(long long)t * U] = e;
                    }
                }
            }
            pk = pkn;
        }
        // log P(O|lambda) = log(sum_j alpha_hat_{T-1}(j)) + ln2 * sum_t e_t   (:375-377)
        const double phat = gsum<G>(alpha);
        const bool alive = (T > 0) && (phat > 0.0);
        if (T > 0 && j == 0 && seq >= 0)
            a.logp[seq] = alive ? (log(phat) + (double)E * 0.69314718055994530942) : -INFINITY;

        if constexpr (!FWD_ONLY) {
            // ---------------- backward sweep fused with gamma / xi / M-step numerators ----------
            double beta = 1.0 / phat;  // beta_hat_{T-1} = 1/phat folds the 1/P of :392,:407
            const int tl = T > 0 ? T - 1 : 0;
            const int olast = symw[(long long)(tl / kChunk) * U * kChunk + (tl % kChunk)];
            {
                const double g = alpha * beta;  // gamma_{T-1}
                if (alive) {
                    gall = g;
                    if (T == 1) pin = g;
                    if (jv) {
                        if constexpr (LDSTAB) atomicAdd(&sBn[olast * G + j], g);
                        else unsafeAtomicAdd(&a.stats[a.off_bnum + (long long)olast * N + j], g);
                    }
                }
            }
            double ca[kChunk], na[kChunk];
            int ce[kChunk], ne[kChunk];
            const int clast = (Tw >= 2) ? (Tw - 2) / kChunk : -1;
            if (clast >= 0) {
#pragma unroll
                for (int s = 0; s < kChunk; ++s) {
                    const long long t = (long long)clast * kChunk + s;
                    ca[s] = aw[t * kWave];
                    ce[s] = ew[(t + 1) * U];
                }
            }
            uint4 pkhi = (clast + 1 < nch) ? loadpack(clast + 1) : pk;
            for (int c = clast; c >= 0; --c) {
                const uint4 pkc = loadpack(c);
                const int cn = c > 0 ? c - 1 : 0;  // prefetch the next (lower) chunk
#pragma unroll
                for (int s = 0; s < kChunk; ++s) {
                    const long long t = (long long)cn * kChunk + s;
                    na[s] = aw[t * kWave];
                    ne[s] = ew[(t + 1) * U];
                }
#pragma unroll
                for (int s = kChunk - 1; s >= 0; --s) {
                    const int t = c * kChunk + s;
                    const int o1 = (s == kChunk - 1) ? sym_of(pkhi, 0) : sym_of(pkc, s + 1);
                    const int o0 = sym_of(pkc, s);
                    const double at = ca[s];
                    const double b1 = Btab[o1 * G + j];
                    const double v = pow2_scale(b1 * beta, ce[s]);  // b_j(o_{t+1}) beta_{t+1}(j) / c_{t+1}
                    const bool act = alive && (t <= T - 2);
                    double bn;
                    if constexpr (LR) {
                        double vup = dpp<0x101>(v);  // row_shl:1 -> v(j+1)
                        vup = (j + 1 < N) ? vup : 0.0;
                        bn = fma(a_up, vup, a_dg * v);       // :182-197
                        if (act) {
                            S[0] = fma(at, v, S[0]);         // xi_t(j,j)   / a_jj
                            S[1] = fma(at, vup, S[1]);       // xi_t(j,j+1) / a_j,j+1
                        }
                    } else {
                        double b0 = 0.0, bb = 0.0;
                        sfor<0, N>([&](auto I) {
                            const double vk = gbcast<G, I.value>(v, lane);
                            if constexpr ((I.value & 1) == 0) b0 = fma(arow[I.value], vk, b0);
                            else bb = fma(arow[I.value], vk, bb);
                            if (act) S[I.value] = fma(at, vk, S[I.value]);   // :402-408
                        });
                        bn = b0 + bb;
                    }
                    if (act) {
                        const double g = at * bn;  // gamma_t(j)  (:392)
                        beta = bn;
                        gex += g;
                        if (t == 0) pin = g;
                        if (jv) {
                            if constexpr (LDSTAB) atomicAdd(&sBn[o0 * G + j], g);   // :474-485
                            else unsafeAtomicAdd(&a.stats[a.off_bnum + (long long)o0 * N + j], g);
                        }
                    }
                }
                pkhi = pkc;
#pragma unroll
                for (int s = 0; s < kChunk; ++s) { ca[s] = na[s]; ce[s] = ne[s]; }
            }
            gall += gex;
        }
    }

    if constexpr (!FWD_ONLY) {
        // ---- reduce per-lane accumulators over the U sequences of the wave, then the block ----
        double vals[NV];
#pragma unroll
        for (int k = 0; k < NS; ++k) vals[k] = S[k];
        vals[NS] = gex;
        vals[NS + 1] = gall;
        vals[NS + 2] = pin;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            double x = vals[k];
            for (int m = G; m < kWave; m <<= 1) x += __shfl_xor(x, m);
            vals[k] = x;
        }
        if (u == 0) {
#pragma unroll
            for (int k = 0; k < NV; ++k) sRed[(wv * G + j) * NV + k] = vals[k];
        }
        __syncthreads();
        const int nw = blockDim.x >> 6;
        for (int idx = tid; idx < G * NV; idx += blockDim.x) {
            const int jj = idx / NV, k = idx % NV;
            if (jj >= N) continue;
            double x = 0.0;
            for (int w = 0; w < nw; ++w) x += sRed[(w * G + jj) * NV + k];
            if (x == 0.0) continue;
            long long dst;
            if (k < NS) {
                const int col = LR ? jj + k : k;
                if (col >= N) continue;
                dst = a.off_S + (long long)jj * N + col;
            } else if (k == NS) {
                dst = a.off_gex + jj;
            } else if (k == NS + 1) {
                dst = a.off_gall + jj;
            } else {
                dst = jj;  // pi_num at offset 0
            }
            unsafeAtomicAdd(&a.stats[dst], x);
        }
        if constexpr (LDSTAB) {
            for (int idx = tid; idx < K * G; idx += blockDim.x) {
                const int jj = idx & (G - 1);
                if (jj >= N) continue;
                const double x = sBn[idx];
                if (x != 0.0) unsafeAtomicAdd(&a.stats[a.off_bnum + (long long)(idx / G) * N + jj], x);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Wide E-step / scorer: 16 < N <= 64, one sequence per wavefront, lane = state.
// ---------------------------------------------------------------------------------------------
template <int NP, bool FWD_ONLY>
__global__ void __launch_bounds__(kBlock) k_estep_wide(EArgs a) {
    extern __shared__ double smem[];
    if (a.state != nullptr && a.state->done) return;
    const int N = a.N;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int j = lane;
    double *sA = smem;              // [NP][64]  a_ij at [i][j]
    double *sAT = smem + NP * 64;   // [NP][64]  a_jk at [k][j]
    double *sX = smem + 2 * NP * 64 + wv * 64;  // per-wave exchange row
    for (int idx = tid; idx < NP * 64; idx += blockDim.x) {
        const int r = idx / 64, c = idx % 64;
        sA[idx] = (r < N && c < N) ? a.A[r * N + c] : 0.0;
        sAT[idx] = (r < N && c < N) ? a.A[c * N + r] : 0.0;
    }
    __syncthreads();
    const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + wv;
    if (wave >= a.L.nwaves) return;
    const int T = a.L.slot_len[wave];
    const int seq = a.L.slot_seq[wave];
    if (T <= 0) return;
    const int nch = (T + kChunk - 1) / kChunk;
    const uint16_t *symw = a.L.sym + a.L.wave_symoff[wave];
    double *aw = a.alpha + (FWD_ONLY ? 0 : a.L.wave_aoff[wave]) + lane;
    int *ew = a.ebuf + (FWD_ONLY ? 0 : a.L.wave_eoff[wave]);
    const bool jv = j < N;
    const double pij = jv ? a.pi[j] : 0.0;
    auto loadpack = [&](int c) -> uint4 { return *reinterpret_cast<const uint4 *>(symw + (long long)c * kChunk); };
    auto xchg = [&](double v) {
        __builtin_amdgcn_wave_barrier();
        sX[lane] = v;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };

    double alpha = 0.0;
    int E = 0;
    uint4 pk = loadpack(0);
    for (int c = 0; c < nch; ++c) {
        const uint4 pkn = (c + 1 < nch) ? loadpack(c + 1) : pk;
        for (int s = 0; s < kChunk; ++s) {
            const int t = c * kChunk + s;
            if (t >= T) break;
            const int o = sym_of(pk, s);
            const double b = a.Bt[(long long)o * 64 + j];
            double x;
            if (t == 0) {
                x = pij * b;
            } else {
                xchg(alpha);
                double acc0 = 0.0, acc1 = 0.0;
#pragma unroll 8
                for (int i = 0; i < NP; i += 2) {
                    acc0 = fma(sX[i], sA[i * 64 + j], acc0);
                    acc1 = fma(sX[i + 1], sA[(i + 1) * 64 + j], acc1);
                }
                x = (acc0 + acc1) * b;
            }
            const double sum = gsum<64>(x);
            const int e = __builtin_amdgcn_frexp_exp(sum);
            x = pow2_scale(x, e);
            alpha = x;
            E += e;
            if constexpr (!FWD_ONLY) {
                aw[(long long)t * kWave] = x;
                if (j == 0) ew[t] = e;
            }
        }
        pk = pkn;
    }
    const double phat = gsum<64>(alpha);
    const bool alive = phat > 0.0;
    if (j == 0 && seq >= 0) a.logp[seq] = alive ? (log(phat) + (double)E * 0.69314718055994530942) : -INFINITY;
    if constexpr (!FWD_ONLY) {
        if (!alive) return;
        double S[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) S[k] = 0.0;
        double gex = 0.0, pin = 0.0;
        double beta = 1.0 / phat;
        auto symat = [&](int t) -> int { return symw[(long long)(t / kChunk) * kChunk + (t % kChunk)]; };
        const double glast = alpha * beta;
        double gall = glast;
        if (T == 1) pin = glast;
        if (jv) unsafeAtomicAdd(&a.stats[a.off_bnum + (long long)symat(T - 1) * N + j], glast);
        int o1 = symat(T - 1);
        for (int t = T - 2; t >= 0; --t) {
            const int o0 = symat(t);
            const double at = aw[(long long)t * kWave];
            const int e1 = ew[t + 1];
            const double b1 = a.Bt[(long long)o1 * 64 + j];
            const double v = pow2_scale(b1 * beta, e1);
            xchg(v);
            double b0 = 0.0, bb = 0.0;
#pragma unroll
            for (int k = 0; k < NP; k += 2) {
                const double v0 = sX[k], v1 = sX[k + 1];
                b0 = fma(sAT[k * 64 + j], v0, b0);
                bb = fma(sAT[(k + 1) * 64 + j], v1, bb);
                S[k] = fma(at, v0, S[k]);
                S[k + 1] = fma(at, v1, S[k + 1]);
            }
            const double bn = b0 + bb;
            const double g = at * bn;
            beta = bn;
            gex += g;
            if (t == 0) pin = g;
            if (jv) unsafeAtomicAdd(&a.stats[a.off_bnum + (long long)o0 * N + j], g);
            o1 = o0;
        }
        gall += gex;
        if (jv) {
#pragma unroll
            for (int k = 0; k < NP; ++k)
                if (k < N && S[k] != 0.0) unsafeAtomicAdd(&a.stats[a.off_S + (long long)j * N + k], S[k]);
            if (gex != 0.0) unsafeAtomicAdd(&a.stats[a.off_gex + j], gex);
            if (gall != 0.0) unsafeAtomicAdd(&a.stats[a.off_gall + j], gall);
            if (pin != 0.0) unsafeAtomicAdd(&a.stats[j], pin);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Block reductions
// ---------------------------------------------------------------------------------------------
__device__ double block_reduce(double x, double *sh, bool is_max) {
    const int tid = threadIdx.x;
    for (int m = 32; m >= 1; m >>= 1) {
        const double y = __shfl_xor(x, m);
        x = is_max ? fmax(x, y) : x + y;
    }
    __syncthreads();
    if ((tid & 63) == 0) sh[tid >> 6] = x;
    __syncthreads();
    if (tid < 64) {
        const int nw = blockDim.x >> 6;
        double y = tid < nw ? sh[tid] : (is_max ? -INFINITY : 0.0);
        for (int m = 32; m >= 1; m >>= 1) {
            const double z = __shfl_xor(y, m);
            y = is_max ? fmax(y, z) : y + z;
        }
        if (tid == 0) sh[0] = y;
    }
    __syncthreads();
    const double r = sh[0];
    __syncthreads();
    return r;
}

// (max, sum exp(x - max)) over the finite log P_r of this rank  (log_sum_exp :66-79 over :503)
__device__ void seq_lse_pair(const double *logp, long long R, double *sh, double *m_out, double *s_out) {
    double mx = -INFINITY;
    for (long long r = threadIdx.x; r < R; r += blockDim.x) mx = fmax(mx, logp[r]);
    mx = block_reduce(mx, sh, true);
    double s = 0.0;
    if (mx != -INFINITY)
        for (long long r = threadIdx.x; r < R; r += blockDim.x) {
            const double x = logp[r];
            if (x != -INFINITY) s += exp(x - mx);
        }
    s = block_reduce(s, sh, false);
    *m_out = mx;
    *s_out = s;
}

__global__ void __launch_bounds__(1024) k_seq_lse(const double *logp, long long R, double *stats, long long off_ll,
                                                  int rank, const IterState *state) {
    __shared__ double sh[16];
    if (state->done) return;
    double m, s;
    seq_lse_pair(logp, R, sh, &m, &s);
    if (threadIdx.x == 0) {
        stats[off_ll + 2 * rank] = (s > 0.0) ? m : 0.0;
        stats[off_ll + 2 * rank + 1] = s;
    }
}

struct MArgs {
    double *stats;
    long long stats_len;
    double *pi, *A, *B, *Bt;
    const double *logp;
    long long R_local;
    long long R_global;
    IterState *state;
    double *hist;
    int N, K, G, world;
    int local_lse;
    long long off_S, off_gex, off_gall, off_bnum, off_ll;
};

__global__ void __launch_bounds__(1024) k_mstep(MArgs m) {
    __shared__ double sh[16];
    __shared__ double sL;
    IterState *st = m.state;
    if (st->done) return;
    const int tid = threadIdx.x;
    // L = LSE_r log P_r over all ranks (:503)
    if (m.local_lse) {
        double mx, s;
        seq_lse_pair(m.logp, m.R_local, sh, &mx, &s);
        if (tid == 0) sL = (s > 0.0) ? mx + log(s) : -INFINITY;
    } else if (tid == 0) {
        double mx = -INFINITY;
        for (int r = 0; r < m.world; ++r)
            if (m.stats[m.off_ll + 2 * r + 1] > 0.0) mx = fmax(mx, m.stats[m.off_ll + 2 * r]);
        double s = 0.0;
        if (mx != -INFINITY)
            for (int r = 0; r < m.world; ++r) {
                const double sr = m.stats[m.off_ll + 2 * r + 1];
                if (sr > 0.0) s += sr * exp(m.stats[m.off_ll + 2 * r] - mx);
            }
        sL = (s > 0.0) ? mx + log(s) : -INFINITY;
    }
    const int N = m.N, K = m.K;
    const double *st_ = m.stats;
    // pi (:415-424): LSE_r gamma_0 - log R ; no term -> -inf
    for (int i = tid; i < N; i += blockDim.x) {
        const double num = st_[i];
        m.pi[i] = num > 0.0 ? num / (double)m.R_global : 0.0;
    }
    // A (:429-455): xi numerator = a_ij * S_ij ; denominator excludes the last frame
    for (int idx = tid; idx < N * N; idx += blockDim.x) {
        const int i = idx / N;
        const double den = st_[m.off_gex + i];
        const double num = m.A[idx] * st_[m.off_S + idx];
        m.A[idx] = (den > 0.0 && num > 0.0) ? num / den : 0.0;
    }
    // B (:460-497): floor 1e-20 when no gamma term carries the symbol; empty denominator -> row 0
    for (long long idx = tid; idx < (long long)N * K; idx += blockDim.x) {
        const int jj = (int)(idx / K), k = (int)(idx % K);
        const double den = st_[m.off_gall + jj];
        const double num = st_[m.off_bnum + (long long)k * N + jj];
        const double v = den > 0.0 ? (num > 0.0 ? num / den : 1e-20) : 0.0;
        m.B[idx] = v;
        m.Bt[(long long)k * m.G + jj] = v;
    }
    __syncthreads();
    if (tid == 0) {
        const double L = sL;
        const double prev = st->prev_L;
        const double diff = (prev != -INFINITY) ? fabs(L - prev) : INFINITY;  // :505-508
        const long long it = st->iteration;
        m.hist[2 * (it % kHist)] = L;
        m.hist[2 * (it % kHist) + 1] = diff;
        st->prev_L = L;
        st->last_L = L;
        st->last_diff = diff;
        st->iteration = it + 1;
        const bool cont = (diff >= st->epsilon) && (it + 1 < st->max_iterations);  // :346
        if (!cont) {
            st->done = 1;
            st->converged = (it + 1 < st->max_iterations) ? 1 : 0;
        }
    }
    // zero the statistics for the next iteration
    for (long long idx = tid; idx < m.stats_len; idx += blockDim.x) m.stats[idx] = 0.0;
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

__global__ void k_init_state(IterState *st, double eps, long long max_it) {
    st->prev_L = -INFINITY;
    st->last_L = -INFINITY;
    st->last_diff = INFINITY;
    st->epsilon = eps;
    st->iteration = 0;
    st->max_iterations = max_it;
    st->done = max_it <= 0 ? 1 : 0;
    st->converged = 0;
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

template <class T>
int dalloc(T **p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(p), n * sizeof(T)));
    return HMMBW_OK;
}

template <class T>
void dfree(T *&p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

using KernelFn = void (*)(EArgs);

struct Kernels {
    KernelFn estep = nullptr, score = nullptr;
};

template <int N, int G, bool LR, bool LDSTAB>
Kernels small_kernels() {
    return Kernels{k_estep_small<N, G, LR, LDSTAB, false>, k_estep_small<N, G, LR, LDSTAB, true>};
}

template <int N, bool LR, bool LDSTAB>
Kernels pick_small_g() {
    constexpr int G = N <= 2 ? 2 : (N <= 4 ? 4 : (N <= 8 ? 8 : 16));
    return small_kernels<N, G, LR, LDSTAB>();
}

template <bool LR, bool LDSTAB>
Kernels pick_small_n(int N) {
    switch (N) {
#define CASE(n) \
    case n: return pick_small_g<n, LR, LDSTAB>();
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
    IterState *d_state = nullptr;
    double *d_hist = nullptr;
    double *d_stats = nullptr;
    bool armed = false;
    // observations
    long long R = 0, nwaves = 0;
    uint16_t *d_sym = nullptr;
    long long *d_wsym = nullptr, *d_waoff = nullptr, *d_weoff = nullptr;
    int *d_wT = nullptr, *d_slen = nullptr, *d_sseq = nullptr;
    double *d_alpha = nullptr, *d_logp = nullptr;
    int *d_ebuf = nullptr;
    bool has_obs = false;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev_free, ev_pending;  // pairs (start, stop)
    double timed_ms = 0.0;
    long long timed_n = 0;

    long long off_S() const { return N; }
    long long off_gex() const { return N + (long long)N * N; }
    long long off_gall() const { return off_gex() + N; }
    long long off_bnum() const { return off_gall() + N; }
    long long off_ll() const { return off_bnum() + (long long)K * N; }
    long long stats_len() const { return off_ll() + 2LL * world; }
    bool lds_tables() const { return !wide && (size_t)2 * K * G * sizeof(double) <= 48 * 1024; }
};

namespace {

int set_device(hmmbw_ctx *c) {
    HIP_TRY(hipSetDevice(c->device));
    return HMMBW_OK;
}

int realloc_stats(hmmbw_ctx *c) {
    dfree(c->d_stats);
    if (int rc = dalloc(&c->d_stats, (size_t)c->stats_len())) return rc;
    HIP_TRY(hipMemsetAsync(c->d_stats, 0, sizeof(double) * c->stats_len(), c->stream));
    return HMMBW_OK;
}

EArgs make_eargs(hmmbw_ctx *c, double *stats) {
    EArgs a{};
    a.L = Layout{c->d_sym, c->d_wsym, c->d_waoff, c->d_weoff, c->d_wT, c->d_slen, c->d_sseq, c->nwaves};
    a.pi = c->d_pi;
    a.A = c->d_A;
    a.Bt = c->d_Bt;
    a.alpha = c->d_alpha;
    a.ebuf = c->d_ebuf;
    a.stats = stats;
    a.logp = c->d_logp;
    a.state = c->d_state;
    a.K = c->K;
    a.N = c->N;
    a.off_S = c->off_S();
    a.off_gex = c->off_gex();
    a.off_gall = c->off_gall();
    a.off_bnum = c->off_bnum();
    return a;
}

template <class F>
int launch_lds(F f, unsigned grid, size_t lds, hipStream_t stream, const EArgs &a) {
    if (lds > 64 * 1024)
        HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
    hipLaunchKernelGGL(f, dim3(grid), dim3(kBlock), lds, stream, a);
    HIP_TRY(hipGetLastError());
    return HMMBW_OK;
}

int launch_estep(hmmbw_ctx *c, double *stats, bool fwd_only, const IterState *state) {
    EArgs a = make_eargs(c, stats);
    a.state = state;
    const int wpb = kBlock / kWave;
    const unsigned grid = (unsigned)((c->nwaves + wpb - 1) / wpb);
    if (grid == 0) return HMMBW_OK;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (c->timing && !fwd_only) {
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
    if (c->wide) {
        const size_t lds = sizeof(double) * (2 * (size_t)c->NP * 64 + (size_t)wpb * 64);
        KernelFn f = c->NP == 32 ? (fwd_only ? k_estep_wide<32, true> : k_estep_wide<32, false>)
                                 : (fwd_only ? k_estep_wide<64, true> : k_estep_wide<64, false>);
        if (int rc = launch_lds(f, grid, lds, c->stream, a)) return rc;
    } else {
        const bool lr = c->topo == HMMBW_TOPOLOGY_LEFT_TO_RIGHT;
        const bool lds_tab = c->lds_tables();
        Kernels ks = lr ? (lds_tab ? pick_small_n<true, true>(c->N) : pick_small_n<true, false>(c->N))
                        : (lds_tab ? pick_small_n<false, true>(c->N) : pick_small_n<false, false>(c->N));
        KernelFn f = fwd_only ? ks.score : ks.estep;
        if (!f) return fail(HMMBW_E_UNSUPPORTED, "no kernel for N");
        const int NV = (lr ? 2 : c->N) + 3;
        const size_t lds = sizeof(double) * ((lds_tab ? 2 * (size_t)c->K * c->G : 0) + (size_t)wpb * c->G * NV);
        if (int rc = launch_lds(f, grid, lds, c->stream, a)) return rc;
    }
    if (e1) {
        HIP_TRY(hipEventRecord(e1, c->stream));
        c->ev_pending.push_back(e0);
        c->ev_pending.push_back(e1);
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
        c->ev_free.push_back(c->ev_pending[i]);
        c->ev_free.push_back(c->ev_pending[i + 1]);
    }
    c->ev_pending.clear();
    return HMMBW_OK;
}

int launch_mstep(hmmbw_ctx *c, double *stats, long long R_global, bool local) {
    MArgs m{};
    m.stats = stats;
    m.stats_len = c->stats_len();
    m.pi = c->d_pi;
    m.A = c->d_A;
    m.B = c->d_B;
    m.Bt = c->d_Bt;
    m.logp = c->d_logp;
    m.R_local = c->R;
    m.R_global = R_global;
    m.state = c->d_state;
    m.hist = c->d_hist;
    m.N = c->N;
    m.K = c->K;
    m.G = c->G;
    m.world = c->world;
    m.local_lse = local ? 1 : 0;
    m.off_S = c->off_S();
    m.off_gex = c->off_gex();
    m.off_gall = c->off_gall();
    m.off_bnum = c->off_bnum();
    m.off_ll = c->off_ll();
    hipLaunchKernelGGL(k_mstep, dim3(1), dim3(1024), 0, c->stream, m);
    HIP_TRY(hipGetLastError());
    return HMMBW_OK;
}

int check_ready(hmmbw_ctx *c, bool need_armed) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (!c->has_obs) return fail(HMMBW_E_STATE, "observations not set");
    if (!c->has_params) return fail(HMMBW_E_STATE, "parameters not set");
    if (need_armed && !c->armed) return fail(HMMBW_E_STATE, "training not armed (hmmbw_reset_training)");
    return set_device(c);
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
    c->G = c->wide ? 64 : (n_states <= 2 ? 2 : n_states <= 4 ? 4 : n_states <= 8 ? 8 : 16);
    c->U = kWave / c->G;
    c->NP = c->wide ? (n_states <= 32 ? 32 : 64) : 0;
    int rc = set_device(c);
    if (!rc) rc = dalloc(&c->d_pi, c->N);
    if (!rc) rc = dalloc(&c->d_A, (size_t)c->N * c->N);
    if (!rc) rc = dalloc(&c->d_B, (size_t)c->N * c->K);
    if (!rc) rc = dalloc(&c->d_Bt, (size_t)c->K * c->G);
    if (!rc) rc = dalloc(&c->d_out, (size_t)c->N + (size_t)c->N * c->N + (size_t)c->N * c->K);
    if (!rc) rc = dalloc(&c->d_state, 1);
    if (!rc) rc = dalloc(&c->d_hist, 2 * (size_t)kHist);
    if (!rc) rc = realloc_stats(c);
    if (!rc) {
        hipLaunchKernelGGL(k_init_state, dim3(1), dim3(1), 0, c->stream, c->d_state, 0.0, 0LL);
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
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    else (void)hipDeviceSynchronize();
    dfree(c->d_pi); dfree(c->d_A); dfree(c->d_B); dfree(c->d_Bt); dfree(c->d_out);
    dfree(c->d_state); dfree(c->d_hist); dfree(c->d_stats);
    dfree(c->d_sym); dfree(c->d_wsym); dfree(c->d_waoff); dfree(c->d_weoff);
    dfree(c->d_wT); dfree(c->d_slen); dfree(c->d_sseq);
    dfree(c->d_alpha); dfree(c->d_logp); dfree(c->d_ebuf);
    for (auto e : c->ev_free) (void)hipEventDestroy(e);
    for (auto e : c->ev_pending) (void)hipEventDestroy(e);
    delete c;
    return HMMBW_OK;
}

int hmmbw_set_stream(hmmbw_ctx *c, void *stream) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    c->stream = reinterpret_cast<hipStream_t>(stream);
    return HMMBW_OK;
}

int hmmbw_set_rank(hmmbw_ctx *c, int rank, int world) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (world < 1 || rank < 0 || rank >= world) return fail(HMMBW_E_INVALID, "bad rank/world");
    if (int rc = set_device(c)) return rc;
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
    std::vector<int> len((size_t)R);
    for (int64_t r = 0; r < R; ++r) {
        const int64_t T = offsets[r + 1] - offsets[r];
        if (T < 0) return fail(HMMBW_E_INVALID, "offsets must be non-decreasing");
        if (T == 0) return fail(HMMBW_E_EMPTY_SEQUENCE, "sequence " + std::to_string(r) + " is empty");
        if (T > (1 << 30)) return fail(HMMBW_E_UNSUPPORTED, "sequence too long");
        len[(size_t)r] = (int)T;
    }
    const int64_t total = offsets[R];
    for (int64_t i = 0; i < total; ++i)
        if (symbols[i] < 0 || symbols[i] >= c->K)
            return fail(HMMBW_E_SYMBOL_RANGE, "symbol " + std::to_string(symbols[i]) + " at position " +
                                                  std::to_string(i) + " is outside [0, M)");
    if (int rc = set_device(c)) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));  // buffers may still be in use by enqueued work
    // length-sorted (descending, stable) assignment of sequences to wave slots
    std::vector<int64_t> perm((size_t)R);
    std::iota(perm.begin(), perm.end(), 0);
    std::stable_sort(perm.begin(), perm.end(), [&](int64_t x, int64_t y) { return len[x] > len[y]; });
    const int U = c->U;
    const long long nwaves = (R + U - 1) / U;
    std::vector<long long> wsym((size_t)nwaves), waoff((size_t)nwaves), weoff((size_t)nwaves);
    std::vector<int> wT((size_t)nwaves), slen((size_t)(nwaves * U), 0), sseq((size_t)(nwaves * U), -1);
    long long symtot = 0, atot = 0, etot = 0;
    for (long long w = 0; w < nwaves; ++w) {
        int Tw = 0;
        for (int u = 0; u < U; ++u) {
            const long long s = w * U + u;
            if (s < R) {
                slen[(size_t)s] = len[(size_t)perm[(size_t)s]];
                sseq[(size_t)s] = (int)perm[(size_t)s];
                Tw = std::max(Tw, slen[(size_t)s]);
            }
        }
        const long long nch = (Tw + kChunk - 1) / kChunk;
        wT[(size_t)w] = Tw;
        wsym[(size_t)w] = symtot;
        waoff[(size_t)w] = atot;
        weoff[(size_t)w] = etot;
        symtot += nch * U * kChunk;
        atot += nch * kChunk * kWave;
        etot += (nch * kChunk + kChunk) * U;
    }
    std::vector<uint16_t> hsym((size_t)std::max(symtot, 1LL), 0);
    for (long long w = 0; w < nwaves; ++w)
        for (int u = 0; u < U; ++u) {
            const long long s = w * U + u;
            if (s >= R) continue;
            const int64_t r = perm[(size_t)s];
            const int T = len[(size_t)r];
            for (int t = 0; t < T; ++t)
                hsym[(size_t)(wsym[(size_t)w] + ((long long)(t / kChunk) * U + u) * kChunk + t % kChunk)] =
                    (uint16_t)symbols[offsets[r] + t];
        }
    dfree(c->d_sym); dfree(c->d_wsym); dfree(c->d_waoff); dfree(c->d_weoff);
    dfree(c->d_wT); dfree(c->d_slen); dfree(c->d_sseq);
    dfree(c->d_alpha); dfree(c->d_logp); dfree(c->d_ebuf);
    c->has_obs = false;
    int rc = dalloc(&c->d_sym, (size_t)std::max(symtot, 1LL));
    if (!rc) rc = dalloc(&c->d_wsym, (size_t)nwaves);
    if (!rc) rc = dalloc(&c->d_waoff, (size_t)nwaves);
    if (!rc) rc = dalloc(&c->d_weoff, (size_t)nwaves);
    if (!rc) rc = dalloc(&c->d_wT, (size_t)nwaves);
    if (!rc) rc = dalloc(&c->d_slen, (size_t)(nwaves * U));
    if (!rc) rc = dalloc(&c->d_sseq, (size_t)(nwaves * U));
    if (!rc) rc = dalloc(&c->d_alpha, (size_t)std::max(atot, 1LL));
    if (!rc) rc = dalloc(&c->d_ebuf, (size_t)std::max(etot, 1LL));
    if (!rc) rc = dalloc(&c->d_logp, (size_t)std::max<int64_t>(R, 1));
    if (rc) return rc;
    HIP_TRY(hipMemcpy(c->d_sym, hsym.data(), sizeof(uint16_t) * hsym.size(), hipMemcpyHostToDevice));
    if (nwaves > 0) {
        HIP_TRY(hipMemcpy(c->d_wsym, wsym.data(), sizeof(long long) * nwaves, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_waoff, waoff.data(), sizeof(long long) * nwaves, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_weoff, weoff.data(), sizeof(long long) * nwaves, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_wT, wT.data(), sizeof(int) * nwaves, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_slen, slen.data(), sizeof(int) * nwaves * U, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_sseq, sseq.data(), sizeof(int) * nwaves * U, hipMemcpyHostToDevice));
    }
    std::vector<double> ninf((size_t)std::max<int64_t>(R, 1), -INFINITY);
    HIP_TRY(hipMemcpy(c->d_logp, ninf.data(), sizeof(double) * ninf.size(), hipMemcpyHostToDevice));
    c->R = R;
    c->nwaves = nwaves;
    c->has_obs = true;
    return HMMBW_OK;
}

int hmmbw_set_params(hmmbw_ctx *c, const double *pi, const double *A, const double *B) {
    if (!c || !pi || !A || !B) return fail(HMMBW_E_INVALID, "null argument");
    if (int rc = set_device(c)) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    const int N = c->N, K = c->K, G = c->G;
    // safe_log semantics (hmm_training.py:46-54): x <= 0 (and NaN) is a zero probability
    auto clean = [](double x) { return x > 0.0 ? x : 0.0; };
    std::vector<double> hpi(N), hA((size_t)N * N), hB((size_t)N * K), hBt((size_t)K * G, 0.0);
    for (int i = 0; i < N; ++i) hpi[i] = clean(pi[i]);
    for (size_t i = 0; i < hA.size(); ++i) hA[i] = clean(A[i]);
    for (int jj = 0; jj < N; ++jj)
        for (int k = 0; k < K; ++k) {
            const double v = clean(B[(size_t)jj * K + k]);
            hB[(size_t)jj * K + k] = v;
            hBt[(size_t)k * G + jj] = v;
        }
    HIP_TRY(hipMemcpy(c->d_pi, hpi.data(), sizeof(double) * N, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_A, hA.data(), sizeof(double) * hA.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_B, hB.data(), sizeof(double) * hB.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_Bt, hBt.data(), sizeof(double) * hBt.size(), hipMemcpyHostToDevice));
    c->h_A = hA;
    c->has_params = true;
    resolve_topology(c);
    return HMMBW_OK;
}

int hmmbw_reset_training(hmmbw_ctx *c, double epsilon, int64_t max_iterations) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (int rc = set_device(c)) return rc;
    hipLaunchKernelGGL(k_init_state, dim3(1), dim3(1), 0, c->stream, c->d_state, epsilon, (long long)max_iterations);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemsetAsync(c->d_stats, 0, sizeof(double) * c->stats_len(), c->stream));
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
    if (!stats_dev) return fail(HMMBW_E_INVALID, "null stats buffer");
    if (int rc = launch_estep(c, stats_dev, false, c->d_state)) return rc;
    hipLaunchKernelGGL(k_seq_lse, dim3(1), dim3(1024), 0, c->stream, c->d_logp, c->R, stats_dev, c->off_ll(),
                       c->rank, c->d_state);
    HIP_TRY(hipGetLastError());
    return HMMBW_OK;
}

int hmmbw_mstep(hmmbw_ctx *c, double *stats_dev, int64_t n_seq_global) {
    if (int rc = check_ready(c, true)) return rc;
    if (!stats_dev) return fail(HMMBW_E_INVALID, "null stats buffer");
    return launch_mstep(c, stats_dev, n_seq_global, false);
}

int hmmbw_iterate(hmmbw_ctx *c, int64_t n_iter) {
    if (int rc = check_ready(c, true)) return rc;
    if (c->world != 1) return fail(HMMBW_E_STATE, "hmmbw_iterate is single-rank; use estep/all-reduce/mstep");
    for (int64_t i = 0; i < n_iter; ++i) {
        if (int rc = launch_estep(c, c->d_stats, false, c->d_state)) return rc;
        if (int rc = launch_mstep(c, c->d_stats, c->R, true)) return rc;
        if (c->timing && c->ev_pending.size() >= 256)
            if (int rc = drain_timing(c)) return rc;
    }
    return HMMBW_OK;
}

int hmmbw_get_status(hmmbw_ctx *c, hmmbw_status *st, hmmbw_iter_record *rec, int64_t first, int64_t count) {
    if (!c || !st) return fail(HMMBW_E_INVALID, "null argument");
    if (int rc = set_device(c)) return rc;
    IterState h{};
    HIP_TRY(hipMemcpyAsync(&h, c->d_state, sizeof(IterState), hipMemcpyDeviceToHost, c->stream));
    std::vector<double> hist(2 * (size_t)kHist);
    if (rec && count > 0)
        HIP_TRY(hipMemcpyAsync(hist.data(), c->d_hist, sizeof(double) * hist.size(), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    st->iterations = h.iteration;
    st->done = h.done;
    st->converged = h.converged;
    st->last_log_likelihood = h.last_L;
    st->last_diff = h.last_diff;
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

int hmmbw_get_params(hmmbw_ctx *c, double *pi, double *A, double *B, int normalise) {
    if (!c || !pi || !A || !B) return fail(HMMBW_E_INVALID, "null argument");
    if (!c->has_params) return fail(HMMBW_E_STATE, "parameters not set");
    if (int rc = set_device(c)) return rc;
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
    if (int rc = launch_estep(c, c->d_stats, true, nullptr)) return rc;
    return hmmbw_get_loglik(c, out);
}

int hmmbw_timing(hmmbw_ctx *c, int enable, double *total_ms, int64_t *count) {
    if (!c) return fail(HMMBW_E_INVALID, "null context");
    if (int rc = set_device(c)) return rc;
    if (int rc = drain_timing(c)) return rc;
    if (total_ms) *total_ms = c->timed_ms;
    if (count) *count = c->timed_n;
    if (enable >= 0) {
        c->timing = enable != 0;
        c->timed_ms = 0.0;
        c->timed_n = 0;
    }
    return HMMBW_OK;
}

}  // extern "C"
