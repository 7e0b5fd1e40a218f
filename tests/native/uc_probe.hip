// Test-only probe (not part of the product library): what becomes of device memory that was allocated
// uncached / fine-grained (hipExtMallocWithFlags, the kinds HMMBW_PEER_MEM selects for the peer receive
// regions) and then freed, and whether the fp64 atomics the E-step uses (global_atomic_add_f64, this unit is
// built with -munsafe-fp-atomics like libhmmbw.so) give exact sums on each kind of memory.
// Built by tests/native/build_probe.py into tests/native/libucprobe.so; driven by tests/test_gpu_peer.py.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace {

// every thread adds 1.0 to slot (global id mod nslots), `reps` times: the exact sums are known
__global__ void k_add_f64(double *p, long long nslots, int reps) {
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (int r = 0; r < reps; ++r) atomicAdd(p + (g + r) % nslots, 1.0);
}

__global__ void k_add_u32(unsigned *p, long long nslots, int reps) {
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (int r = 0; r < reps; ++r) atomicAdd(p + (g + r) % nslots, 1u);
}

}  // namespace

extern "C" {

// kind 0 hipMalloc, 1 hipExtMallocWithFlags(uncached), 2 hipExtMallocWithFlags(fine-grained)
int ucp_alloc(int kind, size_t bytes, void **out) {
    *out = nullptr;
    if (kind == 0) return (int)hipMalloc(out, bytes);
    return (int)hipExtMallocWithFlags(out, bytes, kind == 1 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained);
}

int ucp_free(void *p) { return (int)hipFree(p); }

// base and size of the allocation that holds p (a sub-allocation shows base != p or a larger size)
int ucp_range(void *p, void **base, size_t *size) {
    hipDeviceptr_t b = nullptr;
    size_t s = 0;
    const hipError_t e = hipMemGetAddressRange(&b, &s, reinterpret_cast<hipDeviceptr_t>(p));
    *base = reinterpret_cast<void *>(b);
    *size = s;
    return (int)e;
}

int ucp_flags(void *p, unsigned *flags) {
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, p);
    *flags = a.allocationFlags;
    return (int)e;
}

// fp64 and u32 atomic sums on nslots slots of p (bytes >= 8 * nslots): counts the slots whose sum is wrong
int ucp_atomics(void *p, long long nslots, long long *wrong_f64, long long *wrong_u32) {
    const int blocks = 1024, threads = 256, reps = 8;
    const long long total = (long long)blocks * threads * reps;
    hipError_t e = hipMemset(p, 0, sizeof(double) * (size_t)nslots);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_add_f64, dim3(blocks), dim3(threads), 0, 0, static_cast<double *>(p), nslots, reps);
    if ((e = hipDeviceSynchronize()) != hipSuccess) return (int)e;
    std::vector<double> hd((size_t)nslots);
    if ((e = hipMemcpy(hd.data(), p, sizeof(double) * (size_t)nslots, hipMemcpyDeviceToHost)) != hipSuccess) return (int)e;
    *wrong_f64 = 0;
    for (long long i = 0; i < nslots; ++i) {
        // slot i receives one add per (g, r) with (g + r) mod nslots == i
        long long want = 0;
        for (int r = 0; r < reps; ++r) {
            const long long g0 = ((i - r) % nslots + nslots) % nslots;  // first g with (g + r) % nslots == i
            const long long n = (long long)blocks * threads;
            want += g0 < n ? (n - 1 - g0) / nslots + 1 : 0;
        }
        if (hd[(size_t)i] != (double)want) ++*wrong_f64;
    }
    if ((e = hipMemset(p, 0, sizeof(unsigned) * (size_t)nslots)) != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_add_u32, dim3(blocks), dim3(threads), 0, 0, static_cast<unsigned *>(p), nslots, reps);
    if ((e = hipDeviceSynchronize()) != hipSuccess) return (int)e;
    std::vector<unsigned> hu((size_t)nslots);
    if ((e = hipMemcpy(hu.data(), p, sizeof(unsigned) * (size_t)nslots, hipMemcpyDeviceToHost)) != hipSuccess) return (int)e;
    *wrong_u32 = 0;
    long long sum = 0;
    for (long long i = 0; i < nslots; ++i) sum += hu[(size_t)i];
    for (long long i = 0; i < nslots; ++i) {
        long long want = 0;
        for (int r = 0; r < reps; ++r) {
            const long long g0 = ((i - r) % nslots + nslots) % nslots;
            const long long n = (long long)blocks * threads;
            want += g0 < n ? (n - 1 - g0) / nslots + 1 : 0;
        }
        if ((long long)hu[(size_t)i] != want) ++*wrong_u32;
    }
    (void)total;
    (void)sum;
    return 0;
}

}  // extern "C"
