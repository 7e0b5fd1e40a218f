// estep_small_inst.hip — instantiates the small-N E-step / scorer kernels for N = HMMBW_INST_N
// (the build compiles this file once per N = 1..16, in parallel).
#include "hmmbw_kernels.hpp"

#ifndef HMMBW_INST_N
#error "compile with -DHMMBW_INST_N=<states>"
#endif

namespace hmmbw {

template <>
Kernels small_kernels_n<HMMBW_INST_N>(bool lr, bool ldstab) {
    constexpr int N = HMMBW_INST_N;
    constexpr int G = N <= 2 ? 2 : (N <= 4 ? 4 : (N <= 8 ? 8 : 16));
    if (lr) {
        if (ldstab)
            return Kernels{k_estep_small<N, G, true, true, false>, k_estep_small<N, G, true, true, true>,
                           k_estep_small_group<N, G, true, true, false>, k_estep_small_group<N, G, true, true, true>,
                           k_estep_small<N, G, true, true, false, true>, k_estep_join<N, G, true>};
        return Kernels{k_estep_small<N, G, true, false, false>, k_estep_small<N, G, true, false, true>};
    }
    if (ldstab)
        return Kernels{k_estep_small<N, G, false, true, false>, k_estep_small<N, G, false, true, true>,
                       k_estep_small_group<N, G, false, true, false>, k_estep_small_group<N, G, false, true, true>,
                       k_estep_small<N, G, false, true, false, true>, k_estep_join<N, G, false>};
    return Kernels{k_estep_small<N, G, false, false, false>, k_estep_small<N, G, false, false, true>};
}

}  // namespace hmmbw

#if defined(HMMBW_PHASE_TIMES) && HMMBW_INST_N == 8
// Diagnostics build: the phase / chunk stamps live in this unit's device module (the N = 8 kernels
// write them), so their readback is defined here.
using namespace hmmbw;
extern "C" {
int hmmbw_debug_phase_times(unsigned long long *out, int64_t nwaves) {
    if (!out || nwaves < 0 || nwaves > kPhaseWaves) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * kPhaseSlots * nwaves) != hipSuccess)
        return -2;
    return 0;
}

int hmmbw_debug_chunk_times(unsigned long long *out, int64_t nwaves) {
    if (!out || nwaves < 0 || nwaves > 4096) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chunk), sizeof(unsigned long long) * 128 * nwaves) != hipSuccess)
        return -2;
    return 0;
}
}
#endif
