// PMC calibration for the access widths the E-step uses (MI355X_MICROARCH.md §HBM: FETCH_SIZE /
// WRITE_SIZE are only calibrated for 16-B-per-lane streams).  Streams a known byte count with
// 8-B-per-lane (dwordx2) loads and stores, and with 16-B-per-lane loads, over buffers larger than the
// 256 MiB Infinity Cache, so the counters' bytes can be converted to real bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_read8(const double* __restrict__ src, double* __restrict__ sink, long long n) {
    double acc = 0.0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        acc += src[i];
    if (acc == 12345.678) sink[0] = acc;
}
__global__ void k_write8(double* __restrict__ dst, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        dst[i] = (double)i;
}
__global__ void k_read16(const double2* __restrict__ src, double* __restrict__ sink, long long n) {
    double acc = 0.0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        acc += src[i].x + src[i].y;
    if (acc == 12345.678) sink[0] = acc;
}

int main() {
    const long long bytes = 1LL << 30;  // 1 GiB per buffer, 4x the Infinity Cache
    const long long n = bytes / 8;
    double *a, *b, *sink;
    if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&sink, 64)) { printf("alloc failed\n"); return 1; }
    hipMemset(a, 0, bytes);
    hipMemset(b, 0, bytes);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_read8, dim3(4096), dim3(256), 0, 0, a, sink, n);
        hipLaunchKernelGGL(k_write8, dim3(4096), dim3(256), 0, 0, b, n);
        hipLaunchKernelGGL(k_read16, dim3(4096), dim3(256), 0, 0, (const double2*)a, sink, n / 2);
    }
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    printf("{\"bytes_per_kernel\": %lld}\n", bytes);
    hipFree(a); hipFree(b); hipFree(sink);
    return 0;
}
