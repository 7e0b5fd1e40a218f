// estep_wide_inst.hip — instantiates the wide (16 < N <= 64) E-step / scorer kernels (fp64 MFMA,
// estep_mfma.hpp) for NT = 2, 3, 4 sixteen-state blocks.
#include "estep_mfma.hpp"
#include "hmmbw_kernels.hpp"

namespace hmmbw {

Kernels wide_kernels(int NP) {
    Kernels k;
    if (NP == 32) k = Kernels{k_estep_mfma<2, false>, k_estep_mfma<2, true>, nullptr, nullptr, k_estep_mfma<2, false, true>};
    if (NP == 48) k = Kernels{k_estep_mfma<3, false>, k_estep_mfma<3, true>, nullptr, nullptr, k_estep_mfma<3, false, true>};
    if (NP == 64) k = Kernels{k_estep_mfma<4, false>, k_estep_mfma<4, true>, nullptr, nullptr, k_estep_mfma<4, false, true>};
    return k;
}

KernelFn wide_wq_kernel(int NP) {
    if (NP == 32) return k_estep_mfma<2, false, false, true>;
    if (NP == 48) return k_estep_mfma<3, false, false, true>;
    if (NP == 64) return k_estep_mfma<4, false, false, true>;
    return nullptr;
}

BnumFn bnum_gather_kernel(bool sorted) { return sorted ? k_bnum_gather<true> : k_bnum_gather<false>; }

}  // namespace hmmbw

#if defined(HMMBW_PHASE_TIMES) && defined(HMMBW_CHUNK_TIMES)
// Diagnostics build: the wide kernel's chunk stamps live in this unit's device module.
extern "C" int hmmbw_debug_wide_chunk_times(unsigned long long *out, int64_t nwaves) {
    using namespace hmmbw;
    if (!out || nwaves < 0 || nwaves > 4096) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chunk), sizeof(unsigned long long) * 128 * nwaves) != hipSuccess)
        return -2;
    return 0;
}
#endif
