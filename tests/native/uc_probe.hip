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

__global__ void k_fill(double *p, long long n, double base) {  // ordinary (cached) stores
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        p[i] = base + (double)i;
}

__global__ void k_sum_read(const double *p, long long n, double *out) {  // ordinary loads (lines into L2)
    double s = 0.0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        s += p[i];
    if (s == -1.0) out[0] = s;  // keeps the loads
}

__global__ void k_fill_sys(double *p, long long n, double base) {  // the peer push's system-scope stores
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        __hip_atomic_store(p + i, base + (double)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_copy_sys(const double *p, long long n, double *out) {  // the peer reduce's system-scope loads
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        out[i] = __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_copy_plain(const double *p, long long n, double *out) {  // ordinary loads
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        out[i] = p[i];
}

__global__ void k_l2_flush() {  // system-scope release + acquire on every XCD
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
}

}  // namespace

extern "C" {

// A page's life as ordinary (cached) memory, then as an uncached / fine-grained region (kind 1 / 2):
//   1. c = hipMalloc(bytes), pattern A (1e6 + i) by a kernel, read back by a kernel (lines in the L2), free c
//   2. u = the special allocation (same_va: u == c); hipMemset(u, 0); pattern B (2e6 + i) with system-scope stores
//   3. read u with system-scope loads (sys) and with ordinary loads (plain) into a fresh buffer, and by hipMemcpy
// counts[0..2] = elements != B for sys / plain / hipMemcpy; counts[3..5] = elements equal to pattern A;
// counts[6] = same_va.  flush bit 0: an L2 write-back + invalidate kernel after step 1, bit 1 after step 2;
// bit 2: a validation-like pass (kernel stores, then kernel loads) right after the allocation.
int ucp_stale(int kind, size_t bytes, int flush, long long *counts) {
    const long long n = (long long)(bytes / 8);
    double *c = nullptr, *u = nullptr, *o = nullptr;
    hipError_t e;
    for (int i = 0; i < 7; ++i) counts[i] = 0;
    if ((e = hipMalloc(reinterpret_cast<void **>(&o), bytes)) != hipSuccess) return (int)e;
    if ((e = hipMalloc(reinterpret_cast<void **>(&c), bytes)) != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, c, n, 1e6);
    hipLaunchKernelGGL(k_sum_read, dim3(1024), dim3(256), 0, 0, c, n, o);
    if ((e = hipDeviceSynchronize()) != hipSuccess) return (int)e;
    if ((e = hipFree(c)) != hipSuccess) return (int)e;
    if (flush & 1) {
        hipLaunchKernelGGL(k_l2_flush, dim3(1024), dim3(64), 0, 0);
        if ((e = hipDeviceSynchronize()) != hipSuccess) return (int)e;
    }
    if ((e = hipExtMallocWithFlags(reinterpret_cast<void **>(&u), bytes,
                                   kind == 2 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached)) != hipSuccess)
        return (int)e;
    counts[6] = (u == c) ? 1 : 0;
    if (flush & 4) {  // the engine's validation pass before first use: kernel stores, then kernel loads
        hipLaunchKernelGGL(k_fill_sys, dim3(1024), dim3(256), 0, 0, u, n, 3e6);
        hipLaunchKernelGGL(k_copy_sys, dim3(1024), dim3(256), 0, 0, u, n, o);
        hipLaunchKernelGGL(k_copy_plain, dim3(1024), dim3(256), 0, 0, u, n, o);
        if ((e = hipDeviceSynchronize()) != hipSuccess) return (int)e;
    }
    if ((e = hipMemset(u, 0, bytes)) != hipSuccess) return (int)e;
    if ((e = hipDeviceSynchronize()) != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_fill_sys, dim3(1024), dim3(256), 0, 0, u, n, 2e6);
    if ((e = hipDeviceSynchronize()) != hipSuccess) return (int)e;
    if (flush & 2) {
        hipLaunchKernelGGL(k_l2_flush, dim3(1024), dim3(64), 0, 0);
        if ((e = hipDeviceSynchronize()) != hipSuccess) return (int)e;
    }
    std::vector<double> h((size_t)n);
    for (int mode = 0; mode < 3; ++mode) {
        if (mode == 0) hipLaunchKernelGGL(k_copy_sys, dim3(1024), dim3(256), 0, 0, u, n, o);
        if (mode == 1) hipLaunchKernelGGL(k_copy_plain, dim3(1024), dim3(256), 0, 0, u, n, o);
        if ((e = hipDeviceSynchronize()) != hipSuccess) return (int)e;
        if ((e = hipMemcpy(h.data(), mode < 2 ? o : u, bytes, hipMemcpyDeviceToHost)) != hipSuccess) return (int)e;
        for (long long i = 0; i < n; ++i) {
            counts[mode] += h[(size_t)i] != 2e6 + (double)i;
            counts[3 + mode] += h[(size_t)i] == 1e6 + (double)i;
        }
    }
    (void)hipFree(u);
    (void)hipFree(o);
    return 0;
}


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
