// vq.hip — vector-quantisation encoder (the step before the Baum-Welch path) for gfx950.
//
// Replaces get_observations, HMM/hmm_training.py:82-120: for every frame, the index of the nearest
// centroid by Euclidean distance over the MFCC coefficients [1, 13) (the power coefficient 0 is
// skipped, :98 and :106), scanning centroids in order and keeping the FIRST minimum (strict '<',
// :111).  Bit-exact with the reference: its distance is np.linalg.norm(frame - centroid) (:109) =
// sqrt(x.dot(x)), and for these 12-element vectors OpenBLAS's ddot is a sequential fused
// multiply-add from element 0 (its vector kernel starts at 32 elements); oracle/bw_oracle.c restates
// that and tests/test_oracle_golden.py pins it to numpy bit for bit.  So each distance here is
//     d = fma(x_11, x_11, ... fma(x_1, x_1, x_0 * x_0)),  x_i = f_i - c_i,   s = sqrt(d)
// with the correctly rounded fp64 sqrt, and the comparison is on s, as in the reference (two
// different d can round to the same s, and then the earlier centroid wins).  sqrt is monotone, so
// s < s_best needs d < d_best: the sqrt is only evaluated for those candidates.
//
// Mapping: one lane per frame (fp64 VALU; the scan is a dependent fma chain per centroid, not a
// GEMM: a -2 f.c + |c|^2 reformulation would round differently).  Every lane of a wave scans the same
// centroid at the same time, so the centroid is a wave-uniform operand (scalar loads for the
// reference's 12 dims, an LDS-staged codebook for other widths).  The frame's D values stay in
// registers.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace hmmbw {

// DMAX = D (exact, the reference's 12 dims): the codebook is read with wave-uniform SCALAR loads
// (s_load into SGPRs, one copy per wave, which v_add_f64 takes as its operand), so the scan costs no
// LDS bandwidth: a broadcast ds_read still returns 8 bytes per lane, and with 24 fp64 VALU ops per
// (frame, centroid) the LDS return path, not the fp64 pipe, bounded the LDS-staged form (measured).
template <int D, int FPL>
__global__ void __launch_bounds__(256) k_vq_encode_s(const double *__restrict__ frames, long long F, int stride,
                                                     int col0, const double *__restrict__ cents, int K,
                                                     int *__restrict__ out, double *__restrict__ dist) {
    // FPL frames per lane: independent fma chains against the same (scalar) centroid row
    const long long f0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * FPL;
    if (f0 >= F) return;
    double x[FPL][D];
#pragma unroll
    for (int q = 0; q < FPL; ++q) {
        const long long f = f0 + q < F ? f0 + q : F - 1;
#pragma unroll
        for (int d = 0; d < D; ++d) x[q][d] = frames[f * stride + col0 + d];
    }
    double best_s[FPL], best_d[FPL];
    int arg[FPL];
#pragma unroll
    for (int q = 0; q < FPL; ++q) {
        best_s[q] = INFINITY;
        best_d[q] = INFINITY;
        arg[q] = 0;
    }
    const double *c = cents + col0;
    // centroid k + 1's row is loaded (into SGPRs) while centroid k is scanned
    double cn[D];
#pragma unroll
    for (int d = 0; d < D; ++d) cn[d] = c[d];
    for (int k = 0; k < K; ++k) {
        double cc[D];
#pragma unroll
        for (int d = 0; d < D; ++d) cc[d] = cn[d];
        c += stride;
        if (k + 1 < K) {
#pragma unroll
            for (int d = 0; d < D; ++d) cn[d] = c[d];
        }
        double acc[FPL];
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int q = 0; q < FPL; ++q) {
                const double e = x[q][d] - cc[d];
                acc[q] = (d == 0) ? e * e : __builtin_fma(e, e, acc[q]);
            }
        // only candidates with acc < best_d can have sqrt(acc) < best_s (sqrt is monotone); after the
        // first few centroids that is rare, so the sqrt sits behind a real branch
        bool any = false;
#pragma unroll
        for (int q = 0; q < FPL; ++q) any = any || (acc[q] < best_d[q]);
        if (__builtin_expect(__any(any), 0)) {
#pragma unroll
            for (int q = 0; q < FPL; ++q) {
                if (acc[q] < best_d[q]) {
                    const double sq = __builtin_sqrt(acc[q]);
                    if (sq < best_s[q]) {
                        best_s[q] = sq;
                        best_d[q] = acc[q];
                        arg[q] = k;
                    }
                }
            }
        }
    }
#pragma unroll
    for (int q = 0; q < FPL; ++q) {
        if (f0 + q >= F) break;
        out[f0 + q] = arg[q];
        if (dist) dist[f0 + q] = best_s[q];  // the reference's min_distance (:112)
    }
}

// Any D <= DMAX: codebook staged in LDS.
template <int DMAX>
__global__ void __launch_bounds__(256) k_vq_encode(const double *__restrict__ frames, long long F, int stride,
                                                   int col0, int D, const double *__restrict__ cents, int K,
                                                   int *__restrict__ out, double *__restrict__ dist) {
    extern __shared__ double sC[];  // [K][D] codebook (columns col0 .. col0 + D)
    for (int i = threadIdx.x; i < K * D; i += blockDim.x) {
        const int k = i / D, d = i - k * D;
        sC[i] = cents[(long long)k * stride + col0 + d];
    }
    __syncthreads();
    const long long f = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= F) return;
    double x[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) x[d] = (d < D) ? frames[f * stride + col0 + d] : 0.0;
    double best_s = INFINITY, best_d = INFINITY;
    int arg = 0;
    for (int k = 0; k < K; ++k) {
        const double *c = sC + k * D;
        double acc = 0.0;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
            if (d >= D) break;
            const double e = x[d] - c[d];
            acc = (d == 0) ? e * e : __builtin_fma(e, e, acc);
        }
        if (acc < best_d) {
            const double s = __builtin_sqrt(acc);
            if (s < best_s) {
                best_s = s;
                best_d = acc;
                arg = k;
            }
        }
    }
    out[f] = arg;
    if (dist) dist[f] = best_s;
}

// Enqueue the encoder (arguments validated by hmmbw_vq_encode in hmmbw.hip).
hipError_t launch_vq(hipStream_t st, const double *frames, long long n_frames, int stride, int col0, int dims,
                     const double *centroids, int n_centroids, int *symbols, double *dist) {
    const unsigned grid = (unsigned)((n_frames + 255) / 256);
    if (dims == 12) {
        constexpr int FPL = 2;  // measured: 1 -> 0.61 ms, 2 -> 0.59 ms, 4 -> 0.69 ms (2M frames x 256)
        const unsigned g2 = (unsigned)((n_frames + 256 * FPL - 1) / (256 * FPL));
        auto kern = k_vq_encode_s<12, FPL>;
        hipLaunchKernelGGL(kern, dim3(g2), dim3(256), 0, st, frames, n_frames, stride, col0, centroids, n_centroids,
                           symbols, dist);
        return hipGetLastError();
    }
    const size_t lds = sizeof(double) * (size_t)n_centroids * dims;
    auto f = k_vq_encode<64>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(f),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(f, dim3(grid), dim3(256), lds, st, frames, n_frames, stride, col0, dims, centroids,
                       n_centroids, symbols, dist);
    return hipGetLastError();
}

}  // namespace hmmbw
