// hmmbw_kernels.hpp — E-step kernel entry points exported by the instantiation units.
//
// The small-N kernel k_estep_small<N, G, LR, LDSTAB, FWD_ONLY> has 128 instantiations (N = 1..16 x
// topology x LDS tables x E-step/scorer), plus 64 of the grouped form k_estep_small_group (LDS tables
// only); each N lives in its own translation unit
// (estep_small_inst.hip compiled with -DHMMBW_INST_N=n) so the build compiles them in parallel.
// The pointers returned here are the kernels' host stubs, registered by their own unit's module.
#pragma once

#include "hmmbw_device.hpp"

namespace hmmbw {

using KernelFn = void (*)(EArgs);
using GroupFn = void (*)(GroupArgs);

struct Kernels {
    KernelFn estep = nullptr, score = nullptr;
    GroupFn group_estep = nullptr, group_score = nullptr;  // grouped launches (LDS tables only)
    KernelFn det_estep = nullptr;                          // deterministic-reduction E-step (LDS tables, wide)
    KernelFn join_estep = nullptr;                         // joined spread map (left-to-right, LDS tables)
};

// E-step and scorer kernels for N states (1 <= N <= 16), left-to-right or dense, with or without the
// LDS emission tables.
template <int N>
Kernels small_kernels_n(bool lr, bool ldstab);

// Wide kernels (16 < N <= 64) for the padded state count NP (32, 48 or 64).
Kernels wide_kernels(int NP);
KernelFn wide_wq_kernel(int NP);  // the work-queue E-step (persistent grid, forward / backward units)

// The wide path's B-numerator gather (estep_mfma.hpp).
using BnumFn = void (*)(const double *, const unsigned *, const long long *, int, int, int, double *, const IterState *);
BnumFn bnum_gather_kernel(bool sorted);  // sorted: the wide path's symbol-ordered rows

// The VQ encoder (vq.hip).
hipError_t launch_vq(hipStream_t st, const double *frames, long long n_frames, int stride, int col0, int dims,
                     const double *centroids, int n_centroids, int *symbols, double *dist);

}  // namespace hmmbw
