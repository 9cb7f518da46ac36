// gol_wg_deep_a.hip -- k_step_wg on helix tiles at depths 17..24: wg_waves(K) = 5 or 6
// wavefronts of at most 4 stages each (72 VGPRs, 7 waves per SIMD).  Own translation unit
// so the deep instantiations compile in parallel with the others.
#include "gol_wg.h"

namespace golk {

void *wg_deep_kernel_a(int turns)
{
    switch (turns) {
    case 17: return reinterpret_cast<void *>(&k_step_wg<17, wg_waves(17), 2, 7, true>);
    case 18: return reinterpret_cast<void *>(&k_step_wg<18, wg_waves(18), 2, 7, true>);
    case 19: return reinterpret_cast<void *>(&k_step_wg<19, wg_waves(19), 2, 7, true>);
    case 20: return reinterpret_cast<void *>(&k_step_wg<20, wg_waves(20), 2, 7, true>);
    case 21: return reinterpret_cast<void *>(&k_step_wg<21, wg_waves(21), 2, 7, true>);
    case 22: return reinterpret_cast<void *>(&k_step_wg<22, wg_waves(22), 2, 7, true>);
    case 23: return reinterpret_cast<void *>(&k_step_wg<23, wg_waves(23), 2, 7, true>);
    case 24: return reinterpret_cast<void *>(&k_step_wg<24, wg_waves(24), 2, 7, true>);
    default: return nullptr;
    }
}

}  // namespace golk
