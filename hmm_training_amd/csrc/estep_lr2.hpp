// estep_lr2.hpp — left-to-right E-step / scorer with TWO states per lane (5 <= N <= 8), gfx950.
//
// Replaces the per-utterance loops of HMM/hmm_training.py:351-410 (calculate_log_alpha :122-160,
// calculate_log_beta :163-199, gamma :388-394, xi :396-410, B numerator :474-485) and the forward-only
// scorer of HMM/hmm_testing.py:49-104 for the reference's left-to-right topology (:307-312).
//
// Why.  The one-state-per-lane kernel (k_estep_small: 8 lanes per sequence, 8 sequences per wave) is
// bound by the latency of its per-step chain (DPP shift -> fma), not by issue: at the headline size
// (10,000 sequences = 1,250 waves on 1,024 SIMDs) the SIMDs that hold two waves set the kernel time,
// and one wave per SIMD costs as much as 16,384 sequences would (measured: 8,192 sequences 39 us,
// 10,000 50 us, 16,384 55 us).  With two states per lane a wave carries 16 sequences: 625 waves, at
// most one per SIMD, and the extra arithmetic hides in the same latency chain.
//
// Mapping.  A wave owns a tile of 16 sequences = two consecutive waves of the small kernel's layout
// (so this kernel shares its packs, checkpoints, LDS tables and merged M-step prologue; a workgroup of
// 2 waves covers the small kernel's 4 waves, so the grid and the log-likelihood pairs are the same).
// Lane = 4 s + q: sequence s (0..15), states j0 = 2q and j1 = 2q + 1.  With the product tables
// Bd_j(o) = a_jj b_j(o), Bi_j(o) = a_{j-1,j} b_j(o) (Bi_0 = 0):
//   forward   z_t(j0) = Bd_j0 z(j0) + Bi_j0 z(j0 - 1)   [z(j0 - 1) = lane - 1's z(j1): row_shr:1]
//             z_t(j1) = Bd_j1 z(j1) + Bi_j1 z(j0)       [in lane]
//   backward  beta_t(j0) = Bd_j0 b'(j0) + Bi_j1 b'(j1)  [in lane]
//             beta_t(j1) = Bd_j1 b'(j1) + Bi_j0' b'(j0')  [lane + 1's j0: row_shl:1; 0 past the last state]
// Numerics are the small kernel's: lagged power-of-two scaling every kScale steps with a per-wave
// fall back to per-step scaling, checkpoints every 8 steps and a bit-identical recompute.
//
// Status: experimental, off by default (HMMBW_OPT_LR_PAIRS).  Parity-green (tests/test_gpu_lr2.py) but
// measured slower than k_estep_small: 68.8 vs 35.0 us at 4,096 sequences and 90.4 vs 49.6 us at
// 10,000 — a wave with two states per lane takes about twice as long as one with one, so the latency
// hypothesis above does not hold for this form; k_estep_small's register rings and unroll-by-4
// prefetch, which this kernel does not have, are the likely difference.
#pragma once

#include "hmmbw_device.hpp"

namespace hmmbw {

constexpr int kL2Block = 128;  // two waves = two 16-sequence tiles per workgroup

// helper lambdas are force-inlined: one left out of line keeps its by-reference state in scratch
#define L2_AI __attribute__((always_inline))

template <int N, bool FWD_ONLY>
__global__ void __launch_bounds__(kL2Block) k_estep_lr2(EArgs a) {
    static_assert(N >= 5 && N <= 8, "tiles pair two 8-lane-group waves of the small layout");
    constexpr int G = 8, GP = G + 1, U = kWave / G;
    constexpr int NS = 4;  // per-lane xi accumulators: (j0,j0), (j0,j0+1), (j1,j1), (j1,j1+1)
    constexpr int NV = 3;  // gamma_den_excl, gamma_den_all, pi_num
    extern __shared__ double smem[];
    __shared__ double sPA[G + N * N];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long long bid = blockIdx.x;
    if constexpr (!FWD_ONLY)  // clear the next iteration's statistics (single rank: triple buffer)
        for (long long i = bid * blockDim.x + tid; i < a.zero_len; i += (long long)gridDim.x * blockDim.x)
            a.zero[i] = 0.0;
    const int K = a.K;
    const size_t ntab = (((size_t)K + 1) * GP + 1) & ~(size_t)1;
    double *sBt = smem;                                                // [K+1][GP] b_j(o)
    double2 *sBP = reinterpret_cast<double2 *>(smem + ntab);           // [K+1][GP] (Bd, Bi)
    double *sBn = smem + 3 * ntab;                                     // [K][GP] B numerator histogram
    double *sRed = sBn + (FWD_ONLY ? 0 : (size_t)K * GP);              // [2 waves][G][NS+NV] + ll scratch
    if (!FWD_ONLY && a.merged != 0) {
        if (!merged_mstep<N, G, GP, !FWD_ONLY, true, kL2Block>(a, sBt, sBP, sBn, sPA, bid)) return;
    } else {
        if (a.state != nullptr && a.state->done) return;
        if (tid < G) sPA[tid] = tid < N ? a.pi[tid] : 0.0;
        if (tid < N * N) sPA[G + tid] = a.A[tid];
        for (int i = tid; i < (K + 1) * GP; i += kL2Block) {
            const int k = i / GP, c = i - k * GP;
            sBt[i] = (k < K && c < G) ? a.Bt[(size_t)k * G + c] : 0.0;
            if constexpr (!FWD_ONLY)
                if (i < K * GP) sBn[i] = 0.0;
        }
        __syncthreads();
        for (int i = tid; i < (K + 1) * GP; i += kL2Block) {
            const int c = i % GP;
            const double b = sBt[i];
            const double ad = c < N ? sPA[G + c * N + c] : 0.0;
            const double ai = (c >= 1 && c < N) ? sPA[G + (c - 1) * N + c] : 0.0;
            sBP[i] = double2{ad * b, ai * b};
        }
        __syncthreads();
    }

    const int s = lane >> 2, q = lane & 3;
    const int j0 = 2 * q, j1 = 2 * q + 1;
    const long long tile = bid * 2 + wv;
    const long long w0 = 2 * tile;
    const long long wl = w0 + (s >> 3);
    const bool wok = wl < a.L.nwaves;
    const long long wc = wok ? wl : a.L.nwaves - 1;  // clamped for addressing; lanes of a missing wave
    const int u = s & 7;                               // have T = 0 and store nothing
    const long long slot = wc * U + u;
    const int T = wok ? a.L.slot_len[slot] : 0;
    const int seq = wok ? a.L.slot_seq[slot] : -1;
    const bool t1ok = w0 + 1 < a.L.nwaves;
    const int T0 = w0 < a.L.nwaves ? a.L.wave_T[w0] : 0, T1 = t1ok ? a.L.wave_T[w0 + 1] : 0;
    const int Tw = max(T0, T1);
    // every sequence of the tile has length Tw: no per-lane masks in the sweeps
    const bool full = t1ok && a.L.wave_full[w0] && a.L.wave_full[w0 + 1] && T0 == T1;
    const int nch = (Tw + kChunk - 1) / kChunk;
    const int nchw = (a.L.wave_T[wc] + kChunk - 1) / kChunk;
    const uint16_t *symw = a.L.sym + a.L.wave_symoff[wc] + u * kChunk;
    double *ckw = a.ckpt + (FWD_ONLY ? 0 : a.L.wave_ckoff[wc]) + u * G + j0;  // + c * kWave; j0, j1 adjacent
    uint4 *spw = a.spack + (FWD_ONLY ? 0 : a.L.wave_spoff[wc]) + u;            // + c * U
    double *accb = a.copies + (bid % a.ncopies) * a.copy_len;
    const double pij0 = sPA[j0], pij1 = sPA[j1];  // zero-padded to G

    auto loadpack = [&](int c) L2_AI -> uint4 {
        const int cc = c < nchw ? c : nchw - 1;
        return *reinterpret_cast<const uint4 *>(symw + (long long)cc * U * kChunk);
    };
    // product pairs of this lane's two states at the symbol whose packed entry is off (o * GP * 16 B)
    const char *tabP = reinterpret_cast<const char *>(sBP + j0);
    struct E2 {
        double2 e0, e1;
    };
    auto ld_em = [&](int off) L2_AI -> E2 {
        const double2 *p = reinterpret_cast<const double2 *>(tabP + off);
        return E2{p[0], p[1]};
    };
    // forward step (both states) from z_{t-1}: the small kernel's PT arithmetic
    auto step = [&](double z0, double z1, const E2 &e) L2_AI -> double2 {
        const double prev = dpp<0x111>(z1);  // row_shr:1 -> lane - 1's z(j1) = z(j0 - 1); Bi_0 = 0
        return double2{fma(e.e0.y, prev, e.e0.x * z0), fma(e.e1.y, z0, e.e1.x * z1)};
    };
    // biased exponent of the sequence's largest entry (4 lanes x 2 states), 0 for an all-zero group
    auto group_bexp = [&](double x0, double x1) L2_AI -> int {
        const int e = max((int)__builtin_amdgcn_ubfe((unsigned)__double2hiint(x0), 20, 11),
                          (int)__builtin_amdgcn_ubfe((unsigned)__double2hiint(x1), 20, 11));
        return gmax_i32<4>(e);
    };

    // ---------------- forward sweep (hmm_training.py:357-368) ----------------
    double z0 = 0.0, z1 = 0.0;
    int C = 0;
    auto forward = [&](auto SAFE_, auto MASK_) L2_AI -> bool {
        constexpr bool SAFE = decltype(SAFE_)::value;
        constexpr bool MASK = decltype(MASK_)::value;
        z0 = 0.0;
        z1 = 0.0;
        C = 0;
        int pend[kChunk / kScale] = {};
        int minM = 4096, maxM = 0;
        uint4 pk = loadpack(0);
        for (int c = 0; c < nch; ++c) {
            const uint4 pkn = loadpack(c + 1 < nch ? c + 1 : c);
            int sp[kChunk];
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                const int t = c * kChunk + k;
                sp[k] = 0;
                if (t >= Tw) continue;  // tile-uniform
                double n0, n1;
                int st = 0;
                if (t == 0) {
                    const double *row = reinterpret_cast<const double *>(reinterpret_cast<const char *>(sBt) +
                                                                         (sym_of(pk, 0) >> 1));
                    n0 = pij0 * row[j0];  // pi_j b_j(o_0) (:357-360)
                    n1 = pij1 * row[j1];
                } else {
                    const double2 nn = step(z0, z1, ld_em(sym_of(pk, k)));
                    n0 = nn.x;
                    n1 = nn.y;
                }
                if constexpr (SAFE) {
                    const int M = group_bexp(n0, n1);
                    st = M == 0 ? 0 : M - 1023;
                    n0 = pow2_scale(n0, st);
                    n1 = pow2_scale(n1, st);
                } else if (k % kScale == 0) {
                    st = pend[k / kScale];
                    n0 = pow2_scale(n0, st);
                    n1 = pow2_scale(n1, st);
                    const int M = group_bexp(n0, n1);
                    pend[k / kScale] = min(max(M - 1023, -600), 600);
                    if (!MASK || t < T) {
                        minM = min(minM, M);
                        maxM = max(maxM, M);
                    }
                }
                if constexpr (MASK) {
                    const bool act = t < T;
                    z0 = act ? n0 : z0;
                    z1 = act ? n1 : z1;
                    st = act ? st : 0;
                } else {
                    z0 = n0;
                    z1 = n1;
                }
                C += st;
                sp[k] = st;
                if constexpr (!FWD_ONLY)
                    if (k == 0 && wok && c < nchw)  // checkpoint z_{8c}
                        *reinterpret_cast<double2 *>(ckw + (long long)c * kWave) = double2{z0, z1};
            }
            if constexpr (!FWD_ONLY)
                if (q == 0 && wok && c < nchw) spw[(long long)c * U] = pack_exps(sp);
            pk = pkn;
        }
        return (!SAFE) && (minM < 1023 - 900 || maxM > 1023 + 900);
    };
    bool safe = a.force_safe != 0;
    if (!safe) {
        const bool bad = full ? forward(std::false_type{}, std::false_type{}) : forward(std::false_type{}, std::true_type{});
        safe = __any(bad && T > 0) != 0;  // wave-uniform: redo with per-step normalisation
    }
    if (safe) {
        if (full) forward(std::true_type{}, std::false_type{});
        else forward(std::true_type{}, std::true_type{});
    }

    // log P(O|lambda) = log(sum_j z_{T-1}(j)) + ln2 * C   (:375-377)
    double ps = z0 + z1;
    ps += dpp<0xB1>(ps);  // quad_perm [1,0,3,2]
    ps += dpp<0x4E>(ps);  // quad_perm [2,3,0,1]
    const bool alive = (T > 0) && (ps > 0.0);
    const double lp = alive ? (log(ps) + (double)C * 0.69314718055994530942) : -INFINITY;
    if (q == 0 && T > 0 && seq >= 0) a.logp[seq] = lp;
    const bool ll_valid = (q == 0) && (T > 0);

    double S[NS] = {0.0, 0.0, 0.0, 0.0};
    double gex0 = 0.0, gex1 = 0.0, gall0 = 0.0, gall1 = 0.0, pin0 = 0.0, pin1 = 0.0;
    if constexpr (!FWD_ONLY) if (!(a.ablate & 2)) {
        // ------------- backward sweep fused with gamma / xi / B numerator (:370-410, :474-485) -------------
        const double inv_p = alive ? 1.0 / ps : 0.0;  // beta_hat_{T-1}: folds 1/P (:392, :407)
        char *hist0 = reinterpret_cast<char *>(sBn + j0);
        auto backward = [&](auto SAFE_, auto MASK_) L2_AI {
            constexpr bool SAFE = decltype(SAFE_)::value;
            constexpr bool MASK = decltype(MASK_)::value;
            double beta0 = inv_p, beta1 = inv_p;
            E2 e_hi{};  // product pairs at o_{8c+8} and that step's exponent (from chunk c + 1)
            int s_hi = 0;
            const int cl = (Tw - 1) / kChunk;
            uint4 pk = loadpack(cl), sp = (wok && cl < nchw) ? spw[(long long)cl * U] : uint4{0u, 0u, 0u, 0u};
            double2 ck = (wok && cl < nchw) ? *reinterpret_cast<const double2 *>(ckw + (long long)cl * kWave)
                                            : double2{0.0, 0.0};
            for (int c = cl; c >= 0; --c) {
                // next (lower) chunk's inputs, one chunk ahead
                const int cn = c > 0 ? c - 1 : 0;
                const uint4 pkn = loadpack(cn);
                const uint4 spn = (wok && cn < nchw) ? spw[(long long)cn * U] : uint4{0u, 0u, 0u, 0u};
                const double2 ckn = (wok && cn < nchw) ? *reinterpret_cast<const double2 *>(ckw + (long long)cn * kWave)
                                                       : double2{0.0, 0.0};
                E2 ev[kChunk];
                int sk[kChunk];
#pragma unroll
                for (int k = 0; k < kChunk; ++k) {
                    ev[k] = ld_em(sym_of(pk, k));
                    sk[k] = (SAFE || (k % kScale == 0)) ? exp_of(sp, k) : 0;
                }
                // recompute z_{8c .. 8c+7} (identical ops to the forward)
                double zr0[kChunk], zr1[kChunk];
                zr0[0] = ck.x;
                zr1[0] = ck.y;
#pragma unroll
                for (int k = 1; k < kChunk; ++k) {
                    const double2 nn = step(zr0[k - 1], zr1[k - 1], ev[k]);
                    double n0 = nn.x, n1 = nn.y;
                    if (SAFE || (k % kScale == 0)) {
                        n0 = pow2_scale(n0, sk[k]);
                        n1 = pow2_scale(n1, sk[k]);
                    }
                    zr0[k] = n0;
                    zr1[k] = n1;
                }
                double g0[kChunk], g1[kChunk];
#pragma unroll
                for (int k = kChunk - 1; k >= 0; --k) {
                    const int t = c * kChunk + k;
                    if (t > Tw - 1) {
                        g0[k] = 0.0;
                        g1[k] = 0.0;
                        continue;
                    }
                    const double zt0 = zr0[k], zt1 = zr1[k];
                    const bool reg = !MASK ? (t <= Tw - 2) : (t <= T - 2);
                    const bool ini = !MASK ? (t == Tw - 1) : (t == T - 1);
                    double bn0 = 0.0, bn1 = 0.0;
                    if (t <= Tw - 2) {  // tile-uniform: a step t + 1 exists for some sequence
                        const E2 &e = (k == kChunk - 1) ? e_hi : ev[k + 1];
                        const int s1 = (k == kChunk - 1) ? s_hi : sk[(k + 1) & (kChunk - 1)];
                        const bool sc1 = SAFE || ((k + 1) % kScale == 0);
                        const double bp0 = sc1 ? pow2_scale(beta0, s1) : beta0;
                        const double bp1 = sc1 ? pow2_scale(beta1, s1) : beta1;
                        const double vd0 = e.e0.x * bp0, vd1 = e.e1.x * bp1;
                        const double vu0 = e.e1.y * bp1;               // a_{j0,j1} b_j1 beta'(j1): in lane
                        const double vu1 = dpp<0x101>(e.e0.y * bp0);   // row_shl:1: lane + 1's j0 term
                        bn0 = vd0 + vu0;
                        bn1 = vd1 + vu1;
                        const double zs0 = reg ? zt0 : 0.0, zs1 = reg ? zt1 : 0.0;
                        S[0] = fma(zs0, vd0, S[0]);  // xi_t(j0, j0)  (:396-410)
                        S[1] = fma(zs0, vu0, S[1]);  // xi_t(j0, j1)
                        S[2] = fma(zs1, vd1, S[2]);  // xi_t(j1, j1)
                        S[3] = fma(zs1, vu1, S[3]);  // xi_t(j1, j1 + 1)
                    }
                    // gamma_t (:392), branch-free: regular step, gamma_{T-1}, or past the end
                    const double fz = reg ? 1.0 : 0.0, fi = ini ? inv_p : 0.0;
                    const double gr0 = zt0 * bn0, gr1 = zt1 * bn1;
                    const double gi0 = zt0 * fi, gi1 = zt1 * fi;
                    const double gg0 = reg ? gr0 : gi0, gg1 = reg ? gr1 : gi1;
                    gex0 = fma(fz, gr0, gex0);
                    gex1 = fma(fz, gr1, gex1);
                    gall0 += gi0;
                    gall1 += gi1;
                    beta0 = reg ? bn0 : beta0;
                    beta1 = reg ? bn1 : beta1;
                    if (t == 0) {  // :420 (tile-uniform test)
                        pin0 = gg0;
                        pin1 = gg1;
                    }
                    g0[k] = gg0;
                    g1[k] = gg1;
                }
                e_hi = ev[0];
                s_hi = sk[0];
                if (!(a.ablate & 4)) {
#pragma unroll
                    for (int k = 0; k < kChunk; ++k) {  // :474-485
                        double *h = reinterpret_cast<double *>(hist0 + (sym_of(pk, k) >> 1));
                        if (N == 8 || j0 < N) atomicAdd(h, g0[k]);
                        if (N == 8 || j1 < N) atomicAdd(h + 1, g1[k]);
                    }
                }
                pk = pkn;
                sp = spn;
                ck = ckn;
            }
        };
        if (safe) {
            if (full) backward(std::true_type{}, std::false_type{});
            else backward(std::true_type{}, std::true_type{});
        } else {
            if (full) backward(std::false_type{}, std::false_type{});
            else backward(std::false_type{}, std::true_type{});
        }
        gall0 += gex0;
        gall1 += gex1;
    }

    __syncthreads();
    block_ll_partial(lp, ll_valid, sRed + 2 * G * (NS + NV), a.llpart + 2 * bid);

    if constexpr (!FWD_ONLY) if (!(a.ablate & 1)) {
        // ---- reduce over the 16 sequences of the wave (lanes with the same q), then the two waves ----
        double vals[2][NS / 2 + NV] = {{S[0], S[1], gex0, gall0, pin0}, {S[2], S[3], gex1, gall1, pin1}};
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int k = 0; k < NS / 2 + NV; ++k) {
                double x = vals[h][k];
                for (int m = 4; m < kWave; m <<= 1) x += __shfl_xor(x, m);
                vals[h][k] = x;
            }
        constexpr int NR = NS / 2 + NV;  // per state: xi(j,j), xi(j,j+1), gex, gall, pin
        __syncthreads();
        if (s == 0) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int k = 0; k < NR; ++k) sRed[(wv * G + 2 * q + h) * NR + k] = vals[h][k];
        }
        __syncthreads();
        for (int idx = tid; idx < N * NR; idx += kL2Block) {
            const int jj = idx / NR, k = idx % NR;
            const double x = sRed[jj * NR + k] + sRed[(G + jj) * NR + k];
            if (x == 0.0) continue;
            long long dst;
            if (k < 2) {
                const int col = jj + k;
                if (col >= N) continue;
                dst = a.off_S + (long long)jj * N + col;
            } else if (k == 2) {
                dst = a.off_gex + jj;
            } else if (k == 3) {
                dst = a.off_gall + jj;
            } else {
                dst = jj;  // pi_num at offset 0
            }
            unsafeAtomicAdd(&accb[dst], x);
        }
        for (int idx = tid; idx < K * G; idx += kL2Block) {
            const int k = idx / G, jj = idx - k * G;
            if (jj >= N) continue;
            const double x = sBn[k * GP + jj];
            if (x != 0.0) unsafeAtomicAdd(&accb[a.off_bnum + (long long)k * N + jj], x);
        }
    }
}

}  // namespace hmmbw
