// gol_wg_hx.hip -- the k_step_wg instantiation table for helix tiling (kMultiWgHx; see HX in
// gol_wg.h).  Its own translation unit so it compiles in parallel with gol_wg.hip.
#include "gol_wg.h"

namespace golk {

template <int MINW, bool PG>
static void *wg_hx_fn(int turns)
{
    switch (turns) {
    case 4: return reinterpret_cast<void *>(&k_step_wg<4, 4, 2, MINW, true, PG>);
    case 5: return reinterpret_cast<void *>(&k_step_wg<5, 4, 2, MINW, true, PG>);
    case 6: return reinterpret_cast<void *>(&k_step_wg<6, 4, 2, MINW, true, PG>);
    case 7: return reinterpret_cast<void *>(&k_step_wg<7, 4, 2, MINW, true, PG>);
    case 8: return reinterpret_cast<void *>(&k_step_wg<8, 4, 2, MINW, true, PG>);
    case 9: return reinterpret_cast<void *>(&k_step_wg<9, 4, 2, MINW, true, PG>);
    case 10: return reinterpret_cast<void *>(&k_step_wg<10, 4, 2, MINW, true, PG>);
    case 11: return reinterpret_cast<void *>(&k_step_wg<11, 4, 2, MINW, true, PG>);
    case 12: return reinterpret_cast<void *>(&k_step_wg<12, 4, 2, MINW, true, PG>);
    case 13: return reinterpret_cast<void *>(&k_step_wg<13, 4, 2, MINW, true, PG>);
    case 14: return reinterpret_cast<void *>(&k_step_wg<14, 4, 2, MINW, true, PG>);
    case 15: return reinterpret_cast<void *>(&k_step_wg<15, 4, 2, MINW, true, PG>);
    case 16: return reinterpret_cast<void *>(&k_step_wg<16, 4, 2, MINW, true, PG>);
    default: return nullptr;
    }
}

// the register caps of kMultiWg: 8 waves per SIMD at K <= 12 (64 VGPRs), 7 at K >= 13 (72);
// K > 16 (tools build): helix only (launch_wg runs kMultiWgPg as kMultiWgHx there), wg_waves(K)
// waves
void *wg_hx_kernel(int turns, bool pg)
{
#if GOL_TOOLS   // depths 17..32 measured slower per turn than 16: tools build only
    if (turns > 16) return pg ? nullptr : turns <= 24 ? wg_deep_kernel_a(turns) : wg_deep_kernel_b(turns);
#else
    if (turns > 16) return nullptr;
#endif
    if (pg) return turns >= 13 ? wg_hx_fn<7, true>(turns) : wg_hx_fn<8, true>(turns);
    return turns >= 13 ? wg_hx_fn<7, false>(turns) : wg_hx_fn<8, false>(turns);
}

}  // namespace golk
