// Latency / issue micro-benchmark of the E-step's per-step dependency chains on gfx950.
// One workgroup; 64 * W threads -> W waves (W = 4: one per SIMD, W = 8: two per SIMD).
// Prints cycles per step (s_memtime, shader clock) for each chain variant.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_chain.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    long long x = __builtin_bit_cast(long long, v);
    x = __builtin_amdgcn_update_dpp(0ll, x, CTRL, 0xF, 0xF, true);
    return __builtin_bit_cast(double, x);
}

constexpr int kSteps = 4096;

template <int V>
__global__ void k_chain(const double *in, double *out, long long *cyc) {
    double x = in[threadIdx.x], y = in[threadIdx.x + 1], e0 = in[threadIdx.x + 2], e1 = in[threadIdx.x + 3];
    double x2 = x * 0.5, y2 = y * 0.25;
    __syncthreads();
    const long long t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < kSteps; ++i) {
        if constexpr (V == 0) {  // fp64 fma chain
            x = fma(x, e0, e1);
        } else if constexpr (V == 1) {  // forward step: fma(e1, dpp_shr(x), e0 * x)
            x = fma(e1, dpp<0x111>(x), e0 * x);
        } else if constexpr (V == 7) {  // backward beta step: fma(e0, x, dpp_shl(e1 * x)) (product, then the shift)
            x = fma(e0, x, dpp<0x101>(e1 * x));
        } else if constexpr (V == 2) {  // two independent forward steps (ILP 2)
            x = fma(e1, dpp<0x111>(x), e0 * x);
            x2 = fma(e1, dpp<0x111>(x2), e0 * x2);
        } else if constexpr (V == 3) {  // DPP chain only (64-bit move as 2 x 32)
            x = dpp<0x111>(x);
        } else if constexpr (V == 4) {  // fp64 mul chain
            x = x * e0;
        } else if constexpr (V == 5) {  // four independent forward steps (ILP 4)
            x = fma(e1, dpp<0x111>(x), e0 * x);
            x2 = fma(e1, dpp<0x111>(x2), e0 * x2);
            y = fma(e1, dpp<0x111>(y), e0 * y);
            y2 = fma(e1, dpp<0x111>(y2), e0 * y2);
        } else if constexpr (V == 6) {  // fp32 fma chain
            float f = (float)x;
            f = fmaf(f, (float)e0, (float)e1);
            x = f;
        }
    }
    const long long t1 = clock64();
    out[threadIdx.x] = x + x2 + y + y2;
    if ((threadIdx.x & 63) == 0) cyc[threadIdx.x / 64] = t1 - t0;
}

template <int V>
void run(const char *name, double *din, double *dout, long long *dcyc, int waves) {
    hipLaunchKernelGGL(k_chain<V>, dim3(1), dim3(64 * waves), 0, 0, din, dout, dcyc);
    hipLaunchKernelGGL(k_chain<V>, dim3(1), dim3(64 * waves), 0, 0, din, dout, dcyc);
    long long h[16];
    (void)hipMemcpy(h, dcyc, sizeof(long long) * waves, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int w = 0; w < waves; ++w) mx = h[w] > mx ? h[w] : mx;
    printf("%-34s waves %2d  %7.2f cycles/step (s_memtime)\n", name, waves, mx / kSteps);
}

int main() {
    double *din, *dout;
    long long *dcyc;
    (void)hipMalloc(&din, 2048 * sizeof(double));
    (void)hipMalloc(&dout, 2048 * sizeof(double));
    (void)hipMalloc(&dcyc, 16 * sizeof(long long));
    double h[2048];
    for (int i = 0; i < 2048; ++i) h[i] = 1.0 + 1e-9 * i;
    (void)hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    for (int w : {1, 4, 8}) {
        run<0>("fp64 fma chain", din, dout, dcyc, w);
        run<4>("fp64 mul chain", din, dout, dcyc, w);
        run<6>("fp32 fma chain (+cvt)", din, dout, dcyc, w);
        run<3>("dpp row_shr 64-bit chain", din, dout, dcyc, w);
        run<1>("forward step (dpp+mul+fma)", din, dout, dcyc, w);
        run<7>("backward beta step (mul+dpp+fma)", din, dout, dcyc, w);
        run<2>("forward step x2 ILP", din, dout, dcyc, w);
        run<5>("forward step x4 ILP", din, dout, dcyc, w);
    }
    return 0;
}
