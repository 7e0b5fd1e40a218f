// estep_dmfma.hpp — E-step / scorer for DENSE transition matrices with 5 <= N <= 8 states on the fp64
// matrix cores (gfx950).
//
// Replaces the per-utterance loops of HMM/hmm_training.py:351-410 (calculate_log_alpha :122-160,
// calculate_log_beta :163-199, gamma :388-394, xi :396-410, B numerator :474-485) and the forward-only
// scorer of HMM/hmm_testing.py:49-104 when A is dense.  The VALU kernel (k_estep_small) spends most
// of a dense step on cross-lane broadcasts (every state needs every other state); here the
// recursions are 16 x 16 x 4 fp64 MFMAs instead, and no value crosses a lane in the recursions.
//
// Mapping.  A wave owns a TILE of 16 sequences (the MFMA columns) = two consecutive waves of the small
// kernel's observation layout (8 sequences each), so this kernel shares that layout, its emission
// tables and histogram in LDS, and its merged M-step prologue; a workgroup has 2 waves = the small
// kernel's 4 waves of sequences, so the grid and the per-workgroup log-likelihood pairs are the same.
// Lane (s = lane & 15, g = lane >> 4) holds states g and g + 4 (C/D registers 0 and 1; registers 2,
// 3 are the zero padding rows 8..15) of sequence s.  With v_mfma_f64_16x16x4_f64 (C/D: col =
// lane & 15, row = (lane >> 4) + 4 * reg; A/B operands A[lane & 15][lane >> 4], B[lane >> 4][lane & 15])
// the C/D register kb of Z^T = [state][sequence] is exactly the B operand of k-block kb, so
//   forward   Z_t^T  = b(o_t) * (A^T Z_{t-1}^T)       2 MFMAs (k-blocks of states 0-3, 4-7)
//   backward  beta_t = A V_{t+1}                        2 MFMAs
//   xi        S     += Z_t V_{t+1}^T (k = sequence)     4 MFMAs, operands transposed through LDS
// Scaling: the same exact power-of-two scheme as the small kernel in its per-step form (s_t from the
// largest biased exponent of z_{t-1}); the forward stores one checkpoint per 8-step chunk plus the
// exponents, the backward recomputes each chunk (identical MFMA sequence: bit-identical z).
#pragma once

#include "hmmbw_device.hpp"

namespace hmmbw {

typedef double d64x4 __attribute__((ext_vector_type(4)));

constexpr int kDmBlock = 128;  // two waves = two 16-sequence tiles per workgroup
constexpr int kDmXs = 17;      // LDS row stride (doubles) of a [state][16 sequences] image

__device__ __forceinline__ d64x4 dm_mfma(double a, double b, d64x4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <int N, bool FWD_ONLY>
__global__ void __launch_bounds__(kDmBlock) k_estep_dmfma(EArgs a) {
    static_assert(N >= 5 && N <= 8, "tiles pair two 8-lane-group waves of the small layout");
    constexpr int G = 8, GP = G + 1, U = kWave / G;  // the small kernel's layout for 5 <= N <= 8
    constexpr int NV = 3;                             // gamma_den_excl, gamma_den_all, pi_num rows
    extern __shared__ double smem[];
    __shared__ double sPA[G + N * N];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long long bid = blockIdx.x;
    if constexpr (!FWD_ONLY)  // clear the next iteration's statistics (single rank: triple buffer)
        for (long long i = bid * blockDim.x + tid; i < a.zero_len; i += (long long)gridDim.x * blockDim.x)
            a.zero[i] = 0.0;
    const int K = a.K;
    const size_t ntab = (((size_t)K + 1) * GP + 1) & ~(size_t)1;
    double *sBt = smem;                                        // [K+1][GP] b_j(o)
    double *sBn = smem + ntab;                                 // [K][GP] B numerator histogram
    double *sImg = sBn + (FWD_ONLY ? 0 : (size_t)K * GP);      // [2 waves][2][16][kDmXs] z / v images
    double *sRed = sImg + (FWD_ONLY ? 0 : 2 * 2 * 16 * kDmXs); // [2 waves][G][NV] + ll scratch
    if constexpr (!FWD_ONLY) {
        if (a.merged != 0) {
            if (!merged_mstep<N, G, GP, true, false, kDmBlock>(a, sBt, nullptr, sBn, sPA, bid)) return;
        } else {
            if (a.state != nullptr && a.state->done) return;
            if (tid < G) sPA[tid] = tid < N ? a.pi[tid] : 0.0;
            if (tid < N * N) sPA[G + tid] = a.A[tid];
            for (int i = tid; i < (K + 1) * GP; i += kDmBlock) {
                const int k = i / GP, c = i - k * GP;
                sBt[i] = (k < K && c < G) ? a.Bt[(size_t)k * G + c] : 0.0;
                if (i < K * GP) sBn[i] = 0.0;
            }
            __syncthreads();
        }
    } else {
        if (tid < G) sPA[tid] = tid < N ? a.pi[tid] : 0.0;
        if (tid < N * N) sPA[G + tid] = a.A[tid];
        for (int i = tid; i < (K + 1) * GP; i += kDmBlock) {
            const int k = i / GP, c = i - k * GP;
            sBt[i] = (k < K && c < G) ? a.Bt[(size_t)k * G + c] : 0.0;
        }
        __syncthreads();
    }

    const int s = lane & 15, g = lane >> 4;
    const long long tile = bid * 2 + wv;
    const long long w0 = 2 * tile;                    // the two small-layout waves of this tile
    const long long wl = w0 + (s >> 3);               // this lane's sequence's wave
    const bool wok = wl < a.L.nwaves;
    const long long wc = wok ? wl : a.L.nwaves - 1;   // clamped for addressing
    const int u = s & 7;
    const long long slot = wc * U + u;
    const int T = wok ? a.L.slot_len[slot] : 0;
    const int seq = wok ? a.L.slot_seq[slot] : -1;
    const bool t0ok = w0 < a.L.nwaves, t1ok = w0 + 1 < a.L.nwaves;
    const int T0 = t0ok ? a.L.wave_T[w0] : 0, T1 = t1ok ? a.L.wave_T[w0 + 1] : 0;
    const int Tw = max(T0, T1);                       // tile-uniform step count
    const int nch = (Tw + kChunk - 1) / kChunk;
    const int nchw = (a.L.wave_T[wc] + kChunk - 1) / kChunk;  // chunks stored for this lane's wave
    const uint16_t *symw = a.L.sym + a.L.wave_symoff[wc] + u * kChunk;
    double *ckw = a.ckpt + (FWD_ONLY ? 0 : a.L.wave_ckoff[wc]) + u * G;  // + state j, chunk stride kWave
    uint4 *spw = a.spack + (FWD_ONLY ? 0 : a.L.wave_spoff[wc]) + u;       // chunk stride U
    double *accb = a.copies + (bid % a.ncopies) * a.copy_len;
    const int r0 = g, r1 = g + 4;                     // this lane's states (C/D rows of registers 0, 1)
    const bool v0 = r0 < N, v1 = r1 < N;

    // MFMA A operands: forward A^T[o][i] = a_io (o = lane & 15, i = 4 kb + g); backward A[i][j]
    // (i = lane & 15, j = 4 kb + g); rows / columns >= N are zero
    double aF[2], aB[2];
    {
        const double *sA = sPA + G;
        const int o = lane & 15;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            const int i = 4 * kb + g;
            aF[kb] = (o < N && i < N) ? sA[i * N + o] : 0.0;
            aB[kb] = (o < N && i < N) ? sA[o * N + i] : 0.0;
        }
    }
    const double pi0 = v0 ? sPA[r0] : 0.0, pi1 = v1 ? sPA[r1] : 0.0;

    auto loadpack = [&](int c) -> uint4 {  // chunk c of this lane's sequence (clamped to its wave's chunks)
        const int cc = c < nchw ? c : nchw - 1;
        return *reinterpret_cast<const uint4 *>(symw + (long long)cc * U * kChunk);
    };
    // b_{r0}(o), b_{r1}(o) from the LDS table: packs hold o * (G + 1) * 16 bytes; sBt rows are half that
    const char *tab = reinterpret_cast<const char *>(sBt);
    auto emis = [&](int off) -> double2 {
        const double *row = reinterpret_cast<const double *>(tab + (off >> 1));
        return double2{row[r0], row[r1]};
    };
    auto bexp = [](double x) -> int { return (int)__builtin_amdgcn_ubfe((unsigned)__double2hiint(x), 20, 11); };
    // largest biased exponent over this sequence's states (2 registers x 4 lanes g)
    auto colmax_exp = [&](const d64x4 &z) -> int {
        int M = max(bexp(z[0]), bexp(z[1]));
        M = max(M, __shfl_xor(M, 16));
        return max(M, __shfl_xor(M, 32));
    };
    // one forward step from z_{t-1} (t >= 1) with the emission pair e = b(o_t) and exponent sc
    auto fstep = [&](const d64x4 &zp, double2 e, int sc) -> d64x4 {
        d64x4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = dm_mfma(aF[0], zp[0], acc);
        acc = dm_mfma(aF[1], zp[1], acc);
        return d64x4{__builtin_amdgcn_ldexp(acc[0], -sc) * e.x, __builtin_amdgcn_ldexp(acc[1], -sc) * e.y, 0.0, 0.0};
    };

    // ---------------- forward (hmm_training.py:357-368) ----------------
    d64x4 z = {0.0, 0.0, 0.0, 0.0};
    int C = 0;
    for (int c = 0; c < nch; ++c) {
        const uint4 pk = loadpack(c);
        int sp[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; ++k) {
            const int t = c * kChunk + k;
            sp[k] = 0;
            if (t >= Tw) continue;  // tile-uniform
            const double2 e = emis(sym_of(pk, k));
            d64x4 x;
            int sc = 0;
            if (t == 0) {
                x = d64x4{pi0 * e.x, pi1 * e.y, 0.0, 0.0};  // pi_j b_j(o_0) (:357-360)
            } else {
                const int M = colmax_exp(z);
                sc = M == 0 ? 0 : M - 1023;
                x = fstep(z, e, sc);
            }
            const bool act = t < T;  // past the sequence's end: z frozen at z_{T-1}
            z = act ? x : z;
            sc = act ? sc : 0;
            C += sc;
            sp[k] = sc;
            if constexpr (!FWD_ONLY)
                if (k == 0 && wok && c < nchw) {  // checkpoint z_{8c} (lanes of a missing wave store nothing)
                    if (v0) ckw[(long long)c * kWave + r0] = z[0];
                    if (v1) ckw[(long long)c * kWave + r1] = z[1];
                }
        }
        if constexpr (!FWD_ONLY)
            if (g == 0 && wok && c < nchw) spw[(long long)c * U] = pack_exps(sp);
    }

    // log P(O|lambda) = log(sum_j z_{T-1}(j)) + ln2 * C   (:375-377)
    double ps = z[0] + z[1];
    ps += __shfl_xor(ps, 16);
    ps += __shfl_xor(ps, 32);
    const bool alive = (T > 0) && (ps > 0.0);
    const double lp = alive ? (log(ps) + (double)C * 0.69314718055994530942) : -INFINITY;
    if (g == 0 && T > 0 && seq >= 0) a.logp[seq] = lp;
    const bool ll_valid = (g == 0) && (T > 0);

    double gex0 = 0.0, gex1 = 0.0, gall0 = 0.0, gall1 = 0.0, pin0 = 0.0, pin1 = 0.0;
    d64x4 S = {0.0, 0.0, 0.0, 0.0};  // S[r] = sum_t xi_t(i, j) / a_ij, i = g + 4r, j = lane & 15 (C/D)
    if constexpr (!FWD_ONLY) if (!(a.ablate & 2)) {
        // ------------- backward fused with gamma / xi / B numerator (:370-410, :474-485) -------------
        const double inv_p = alive ? 1.0 / ps : 0.0;  // beta_hat_{T-1}: folds 1/P (:392, :407)
        double *img = sImg + (size_t)wv * 2 * 16 * kDmXs;
        double *imgZ = img, *imgV = img + 16 * kDmXs;
        d64x4 beta = {inv_p, inv_p, 0.0, 0.0};
        // v_{t+1} of the step after, with its symbol: consumed by step t
        for (int c = nch - 1; c >= 0; --c) {
            const uint4 pk = loadpack(c);
            const uint4 pkn = loadpack(c + 1 < nch ? c + 1 : c);
            const uint4 spk = c < nchw ? spw[(long long)c * U] : uint4{0u, 0u, 0u, 0u};
            const uint4 spn = (c + 1 < nch && c + 1 < nchw) ? spw[(long long)(c + 1) * U] : uint4{0u, 0u, 0u, 0u};
            // recompute z_{8c .. 8c+7} from the checkpoint (the forward's exact operation sequence)
            d64x4 zr[kChunk];
            zr[0] = d64x4{(v0 && c < nchw) ? ckw[(long long)c * kWave + r0] : 0.0,
                          (v1 && c < nchw) ? ckw[(long long)c * kWave + r1] : 0.0, 0.0, 0.0};
#pragma unroll
            for (int k = 1; k < kChunk; ++k) {
                const int t = c * kChunk + k;
                if (t >= Tw) {
                    zr[k] = zr[k - 1];
                    continue;
                }
                const int sc = exp_of(spk, k);
                const d64x4 x = fstep(zr[k - 1], emis(sym_of(pk, k)), sc);
                zr[k] = (t < T) ? x : zr[k - 1];
            }
#pragma unroll
            for (int k = kChunk - 1; k >= 0; --k) {
                const int t = c * kChunk + k;
                if (t > Tw - 1) continue;  // tile-uniform
                const d64x4 zt = zr[k];
                const int o_t = sym_of(pk, k);
                if (t == Tw - 1 || t >= T - 1) {
                    // gamma_{T-1} = z_{T-1} / P for the lanes whose last step this is (:392 at t = T-1)
                    if (t == T - 1) {
                        const double g0 = zt[0] * inv_p, g1 = zt[1] * inv_p;
                        gall0 += g0;
                        gall1 += g1;
                        if (t == 0) {
                            pin0 += g0;
                            pin1 += g1;
                        }
                        if (v0) atomicAdd(reinterpret_cast<double *>(reinterpret_cast<char *>(sBn + r0) + (o_t >> 1)), g0);
                        if (v1) atomicAdd(reinterpret_cast<double *>(reinterpret_cast<char *>(sBn + r1) + (o_t >> 1)), g1);
                    }
                    if (t == Tw - 1) continue;  // no later step in the tile: nothing to recur from
                }
                // regular step t <= T - 2 (per lane): v_j = b_j(o_{t+1}) 2^{-s_{t+1}} beta_hat_{t+1}(j)
                const bool reg = t <= T - 2;
                const int o1 = (k + 1 < kChunk) ? sym_of(pk, k + 1) : sym_of(pkn, 0);
                const int s1 = (k + 1 < kChunk) ? exp_of(spk, k + 1) : exp_of(spn, 0);
                const double2 e1 = emis(o1);
                const double vA = reg ? __builtin_amdgcn_ldexp(e1.x * beta[0], -s1) : 0.0;
                const double vB = reg ? __builtin_amdgcn_ldexp(e1.y * beta[1], -s1) : 0.0;
                const double zA = reg ? zt[0] : 0.0, zB = reg ? zt[1] : 0.0;
                // beta_hat_t = A v (:163-199)
                d64x4 bn = {0.0, 0.0, 0.0, 0.0};
                bn = dm_mfma(aB[0], vA, bn);
                bn = dm_mfma(aB[1], vB, bn);
                // xi: S_ij += sum_s z_t(i, s) v_{t+1}(j, s) through [state][sequence] images (:396-410)
                imgZ[r0 * kDmXs + s] = zA;
                imgZ[r1 * kDmXs + s] = zB;
                imgV[r0 * kDmXs + s] = vA;
                imgV[r1 * kDmXs + s] = vB;
                __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the wave's image writes are done
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int ir = lane & 15, sc4 = 4 * kk + g;
                    const double za = ir < 8 ? imgZ[ir * kDmXs + sc4] : 0.0;
                    const double vb = ir < 8 ? imgV[ir * kDmXs + sc4] : 0.0;
                    S = dm_mfma(za, vb, S);
                }
                __builtin_amdgcn_wave_barrier();
                const double gm0 = zA * bn[0], gm1 = zB * bn[1];  // gamma_t (:392); 0 unless regular
                beta = reg ? d64x4{bn[0], bn[1], 0.0, 0.0} : beta;
                gex0 += gm0;
                gex1 += gm1;
                if (t == 0) {
                    pin0 += gm0;
                    pin1 += gm1;
                }
                if (reg) {
                    if (v0) atomicAdd(reinterpret_cast<double *>(reinterpret_cast<char *>(sBn + r0) + (o_t >> 1)), gm0);
                    if (v1) atomicAdd(reinterpret_cast<double *>(reinterpret_cast<char *>(sBn + r1) + (o_t >> 1)), gm1);
                }
            }
        }
        gall0 += gex0;
        gall1 += gex1;
    }
    __syncthreads();
    block_ll_partial(lp, ll_valid, sRed + 2 * G * NV, a.llpart + 2 * bid);

    if constexpr (!FWD_ONLY) if (!(a.ablate & 1)) {
        // ---- flush: xi = a_ij S_ij (S is already summed over the tile's sequences); gamma sums over
        // the 16 sequences (lanes with the same g), then both waves through LDS, then fp64 atomics ----
        const double *sA = sPA + G;
        const int jj = lane & 15;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int i = g + 4 * r;
            if (i < N && jj < N) {
                const double x = S[r] * sA[i * N + jj];
                if (x != 0.0) unsafeAtomicAdd(&accb[a.off_S + (long long)i * N + jj], x);
            }
        }
        double vals[2][NV] = {{gex0, gall0, pin0}, {gex1, gall1, pin1}};
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                double x = vals[r][q];
                for (int m = 1; m < 16; m <<= 1) x += __shfl_xor(x, m);
                vals[r][q] = x;
            }
        __syncthreads();
        if (s == 0) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int q = 0; q < NV; ++q) sRed[(wv * G + g + 4 * r) * NV + q] = vals[r][q];
        }
        __syncthreads();
        for (int idx = tid; idx < N * NV; idx += kDmBlock) {
            const int j = idx / NV, q = idx % NV;
            const double x = sRed[j * NV + q] + sRed[(G + j) * NV + q];
            if (x == 0.0) continue;
            const long long dst = q == 0 ? a.off_gex + j : (q == 1 ? a.off_gall + j : j);
            unsafeAtomicAdd(&accb[dst], x);
        }
        for (int idx = tid; idx < K * G; idx += kDmBlock) {
            const int k = idx / G, j = idx - k * G;
            if (j >= N) continue;
            const double x = sBn[k * GP + j];
            if (x != 0.0) unsafeAtomicAdd(&accb[a.off_bnum + (long long)k * N + j], x);
        }
    }
}

}  // namespace hmmbw
