// v_mfma_f64_4x4x4_4b_f64 on gfx950: operand/result lane layout probe, then latency of the chains a
// dense N = 8 forward step would run (MFMA -> MFMA through SrcC, MFMA -> VALU -> MFMA through SrcB,
// with v_permlane32_swap between them).  Diagnostics only.   hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>

// probe[p][l]: D lane l when A = e_p (1 at lane p) and B lane k holds k + 1; probeB likewise with
// B = e_p and A lane k holding k + 1.
__global__ void k_probe(double *pa, double *pb) {
    const int l = threadIdx.x;
    for (int p = 0; p < 64; ++p) {
        double a = l == p ? 1.0 : 0.0, b = l + 1.0;
        pa[p * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
        a = l + 1.0; b = l == p ? 1.0 : 0.0;
        pb[p * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    }
}

static __device__ __forceinline__ double swap32(double x) {
    const unsigned long long u = __double_as_longlong(x);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)u, (unsigned)u, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(u >> 32), (unsigned)(u >> 32), false, false);
    return __longlong_as_double(((unsigned long long)hi[0] << 32) | lo[0]);
}

// MODE 0: acc chain through SrcC; 1: chain through SrcB (D feeds the next B); 2: forward-step shape
// (MFMA, swap, MFMA accumulate, v_mul); 3: two independent forward chains interleaved.
template <int MODE>
__global__ void k_chain(double *out, int iters, long long *cyc) {
    const int l = threadIdx.x & 63;
    double a = 0.25 + l * 1e-6, a2 = 0.25 - l * 1e-6, z = 1.0 + l * 1e-3, y = 1.0 - l * 1e-3, acc = 0.0;
    const double bm = 0.999 + l * 1e-7;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {
            acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a, z, acc, 0, 0, 0);
        } else if (MODE == 1) {
            z = __builtin_amdgcn_mfma_f64_4x4x4f64(a, z, 0.0, 0, 0, 0);
        } else if (MODE == 2) {
            const double zs = swap32(z);
            double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, z, 0.0, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f64_4x4x4f64(a2, zs, d, 0, 0, 0);
            z = d * bm;
        } else {
            const double zs = swap32(z), ys = swap32(y);
            double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, z, 0.0, 0, 0, 0);
            double e = __builtin_amdgcn_mfma_f64_4x4x4f64(a, y, 0.0, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f64_4x4x4f64(a2, zs, d, 0, 0, 0);
            e = __builtin_amdgcn_mfma_f64_4x4x4f64(a2, ys, e, 0, 0, 0);
            z = d * bm;
            y = e * bm;
        }
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc + z + y;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// Dense N = 8 step shapes with 16 sequences per wave (states j & 3 in lane bits 4-5, j >> 2 in the
// register: zl / zh; sequences in bits 0-3): MODE 0 forward (4 MFMAs, two SrcC pairs, 2 v_mul);
// MODE 1 backward shape: the beta chain (4 MFMAs) + the transposed v through LDS (write, read) +
// 4 xi MFMAs accumulating.
template <int MODE>
__global__ void k_dense16(double *out, int iters, long long *cyc) {
    __shared__ double sx[4][2][64];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double a0 = 0.11 + l * 1e-6, a1 = 0.12 - l * 1e-6, a2 = 0.13 + l * 1e-7, a3 = 0.14 - l * 1e-7;
    double zl = 1.0 + l * 1e-3, zh = 1.0 - l * 1e-3, s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    const double bl = 0.999 + l * 1e-7, bh = 1.001 - l * 1e-7;
    const int tl = ((l & 3) << 4) | (l & 12) | (l >> 4);  // transposed lane: bits 0-1 <-> 4-5
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        double nl = __builtin_amdgcn_mfma_f64_4x4x4f64(a0, zl, 0.0, 0, 0, 0);
        double nh = __builtin_amdgcn_mfma_f64_4x4x4f64(a2, zl, 0.0, 0, 0, 0);
        nl = __builtin_amdgcn_mfma_f64_4x4x4f64(a1, zh, nl, 0, 0, 0);
        nh = __builtin_amdgcn_mfma_f64_4x4x4f64(a3, zh, nh, 0, 0, 0);
        if (MODE == 1) {
            sx[w][0][l] = zl;
            sx[w][1][l] = zh;
            const double vl = sx[w][0][tl], vh = sx[w][1][tl];
            s0 = __builtin_amdgcn_mfma_f64_4x4x4f64(vl, vl, s0, 0, 0, 0);
            s1 = __builtin_amdgcn_mfma_f64_4x4x4f64(vl, vh, s1, 0, 0, 0);
            s2 = __builtin_amdgcn_mfma_f64_4x4x4f64(vh, vl, s2, 0, 0, 0);
            s3 = __builtin_amdgcn_mfma_f64_4x4x4f64(vh, vh, s3, 0, 0, 0);
        }
        zl = nl * bl;
        zh = nh * bh;
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = zl + zh + s0 + s1 + s2 + s3;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// The VALU dense N = 8 step it would replace (8 sequences per wave, lane = 8 u + j): acc0/acc1 over
// even/odd states, one bank-masked v_fmac_f64_dpp row_newbcast per 8-lane group and state, then * b.
template <int L, int BM>
__device__ __forceinline__ void fmacb(double &acc, double z, double a) {
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:%4" : "+v"(acc) : "v"(z), "v"(a), "i"(L), "i"(BM));
}
__global__ void k_dppstep(double *out, int iters, long long *cyc) {
    const int l = threadIdx.x & 63;
    double a[8];
    for (int i = 0; i < 8; ++i) a[i] = 0.12 + 0.001 * i + l * 1e-7;
    double z = 1.0 + l * 1e-3;
    const double bm = 0.999 + l * 1e-7;
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        double a0 = 0.0, a1 = 0.0;
        asm volatile("s_nop 1" ::"v"(z));
        fmacb<0, 3>(a0, z, a[0]); fmacb<8, 12>(a0, z, a[0]); fmacb<1, 3>(a1, z, a[1]); fmacb<9, 12>(a1, z, a[1]);
        fmacb<2, 3>(a0, z, a[2]); fmacb<10, 12>(a0, z, a[2]); fmacb<3, 3>(a1, z, a[3]); fmacb<11, 12>(a1, z, a[3]);
        fmacb<4, 3>(a0, z, a[4]); fmacb<12, 12>(a0, z, a[4]); fmacb<5, 3>(a1, z, a[5]); fmacb<13, 12>(a1, z, a[5]);
        fmacb<6, 3>(a0, z, a[6]); fmacb<14, 12>(a0, z, a[6]); fmacb<7, 3>(a1, z, a[7]); fmacb<15, 12>(a1, z, a[7]);
        z = (a0 + a1) * bm;
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = z;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class F>
void run(const char *name, F f, int blocks, int threads, int iters, double *d, long long *c) {
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, iters, c);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, iters, c);
    hipDeviceSynchronize();
    long long cy;
    hipMemcpy(&cy, c, sizeof(cy), hipMemcpyDeviceToHost);
    printf("%-40s %4d x %3d thr: %.2f cycles/iter (clock64, block 0)\n", name, blocks, threads, (double)cy / iters);
}

int main() {
    double *pa, *pb;
    hipMalloc(&pa, 64 * 64 * 8);
    hipMalloc(&pb, 64 * 64 * 8);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, pa, pb);
    static double ha[64 * 64], hb[64 * 64];
    hipMemcpy(ha, pa, sizeof(ha), hipMemcpyDeviceToHost);
    hipMemcpy(hb, pb, sizeof(hb), hipMemcpyDeviceToHost);
    // A probe: D lanes touched by A lane p, with the B lane (value - 1) that multiplied it
    for (int p = 0; p < 64; ++p) {
        printf("A%02d:", p);
        for (int l = 0; l < 64; ++l)
            if (ha[p * 64 + l] != 0.0) printf(" D%02d<-B%02d", l, (int)ha[p * 64 + l] - 1);
        printf("\n");
    }
    for (int p = 0; p < 64; ++p) {
        printf("B%02d:", p);
        for (int l = 0; l < 64; ++l)
            if (hb[p * 64 + l] != 0.0) printf(" D%02d<-A%02d", l, (int)hb[p * 64 + l] - 1);
        printf("\n");
    }
    double *d; long long *c;
    hipMalloc(&d, 1 << 24); hipMalloc(&c, 1 << 16);
    const int it = 20000;
    run("4x4x4 chain through SrcC", k_chain<0>, 256, 256, it, d, c);
    run("4x4x4 chain through SrcB", k_chain<1>, 256, 256, it, d, c);
    run("forward step (mfma,swap,mfma,mul)", k_chain<2>, 256, 256, it, d, c);
    run("forward step x2 interleaved", k_chain<3>, 256, 256, it, d, c);
    run("forward step, 2 waves/SIMD", k_chain<2>, 512, 256, it, d, c);
    run("forward step x2, 2 waves/SIMD", k_chain<3>, 512, 256, it, d, c);
    run("VALU dense step (16 fmac_dpp), 8 seqs", k_dppstep, 256, 256, it, d, c);
    run("VALU dense step, 2 waves/SIMD", k_dppstep, 512, 256, it, d, c);
    run("dense16 forward step", k_dense16<0>, 256, 256, it, d, c);
    run("dense16 backward shape", k_dense16<1>, 256, 256, it, d, c);
    run("dense16 backward shape, 2 waves/SIMD", k_dense16<1>, 512, 256, it, d, c);
    return 0;
}
