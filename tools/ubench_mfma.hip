// Micro-benchmark: v_mfma_f64_16x16x4_f64 issue rate on gfx950 (independent accumulators vs one
// dependent chain), one wave per SIMD and two waves per SIMD.   hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int CHAINS>
__global__ void k_mfma(double *out, int iters, long long *cyc) {
    f64x4 acc[CHAINS];
    for (int c = 0; c < CHAINS; ++c) acc[c] = f64x4{0.0, 0.0, 0.0, 0.0};
    double a = 1.0 + threadIdx.x * 1e-9, b = 0.5 + threadIdx.x * 1e-9;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    }
    long long t1 = clock64();
    double s = 0;
    for (int c = 0; c < CHAINS; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_fma(double *out, int iters, long long *cyc) {  // 8 independent v_fma_f64 chains
    double x[8];
    for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 1e-9 + c;
    const double a = 0.999999, b = 1e-7;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < 8; ++c) x[c] = fma(x[c], a, b);
    long long t1 = clock64();
    double s = 0;
    for (int c = 0; c < 8; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class F>
void run(const char *name, F f, int blocks, int threads, int iters, double flop_per_iter_wave, double *d, long long *c) {
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, iters, c);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, iters, c);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long cy; hipMemcpy(&cy, c, sizeof(cy), hipMemcpyDeviceToHost);
    const double waves = blocks * (threads / 64);
    printf("%-28s blocks %5d x %4d thr: %.3f ms, %.1f TFLOP/s, %.2f cycles/instr/wave (clock64 of block 0)\n", name, blocks,
           threads, ms, waves * iters * flop_per_iter_wave / (ms * 1e-3) / 1e12, (double)cy / iters);
}

int main() {
    double *d; long long *c;
    hipMalloc(&d, 1 << 24); hipMalloc(&c, 1 << 16);
    const int it = 20000;
    const double mf = 16 * 16 * 4 * 2;
    run("mfma f64 1 chain", k_mfma<1>, 256, 256, it, mf * 1, d, c);
    run("mfma f64 2 chains", k_mfma<2>, 256, 256, it, mf * 2, d, c);
    run("mfma f64 4 chains", k_mfma<4>, 256, 256, it, mf * 4, d, c);
    run("mfma f64 4 chains 2w/SIMD", k_mfma<4>, 512, 256, it, mf * 4, d, c);
    run("fma f64 8 chains", k_fma, 256, 256, it, 64.0 * 2 * 8, d, c);
    run("fma f64 8 chains 2w/SIMD", k_fma, 512, 256, it, 64.0 * 2 * 8, d, c);
    return 0;
}
