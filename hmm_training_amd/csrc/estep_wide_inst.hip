// estep_wide_inst.hip — instantiates the wide (16 < N <= 64) E-step / scorer kernels.
#include "hmmbw_kernels.hpp"

namespace hmmbw {

Kernels wide_kernels(int NP) {
    if (NP == 32) return Kernels{k_estep_wide<32, false>, k_estep_wide<32, true>};
    if (NP == 64) return Kernels{k_estep_wide<64, false>, k_estep_wide<64, true>};
    return Kernels{};
}

}  // namespace hmmbw
