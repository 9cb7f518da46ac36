// gol_wg_deep_b.hip -- k_step_wg on helix tiles at depths 25..32: wg_waves(K) = 7 or 8
// wavefronts of at most 4 stages each (72 VGPRs, 7 waves per SIMD).  Own translation unit
// so the deep instantiations compile in parallel with the others.
#include "gol_wg.h"

namespace golk {

void *wg_deep_kernel_b(int turns)
{
    switch (turns) {
    case 25: return reinterpret_cast<void *>(&k_step_wg<25, wg_waves(25), 2, 7, true>);
    case 26: return reinterpret_cast<void *>(&k_step_wg<26, wg_waves(26), 2, 7, true>);
    case 27: return reinterpret_cast<void *>(&k_step_wg<27, wg_waves(27), 2, 7, true>);
    case 28: return reinterpret_cast<void *>(&k_step_wg<28, wg_waves(28), 2, 7, true>);
    case 29: return reinterpret_cast<void *>(&k_step_wg<29, wg_waves(29), 2, 7, true>);
    case 30: return reinterpret_cast<void *>(&k_step_wg<30, wg_waves(30), 2, 7, true>);
    case 31: return reinterpret_cast<void *>(&k_step_wg<31, wg_waves(31), 2, 7, true>);
    case 32: return reinterpret_cast<void *>(&k_step_wg<32, wg_waves(32), 2, 7, true>);
    default: return nullptr;
    }
}

}  // namespace golk
