// gol_wg.hip -- the k_step_wg instantiation table (band tiling; gol_wg_hx.hip: helix)
#include "gol_wg.h"

namespace golk {

template <int NW, int SYNC, int MINW = 1>
static void *wg_fn_nw(int turns)
{
    switch (turns) {
    case 4: return reinterpret_cast<void *>(&k_step_wg<4, NW, SYNC, MINW>);
    case 5: return reinterpret_cast<void *>(&k_step_wg<5, NW, SYNC, MINW>);
    case 6: return reinterpret_cast<void *>(&k_step_wg<6, NW, SYNC, MINW>);
    case 7: return reinterpret_cast<void *>(&k_step_wg<7, NW, SYNC, MINW>);
    case 8: return reinterpret_cast<void *>(&k_step_wg<8, NW, SYNC, MINW>);
    case 9: return reinterpret_cast<void *>(&k_step_wg<9, NW, SYNC, MINW>);
    case 10: return reinterpret_cast<void *>(&k_step_wg<10, NW, SYNC, MINW>);
    case 11: return reinterpret_cast<void *>(&k_step_wg<11, NW, SYNC, MINW>);
    case 12: return reinterpret_cast<void *>(&k_step_wg<12, NW, SYNC, MINW>);
    case 13: return reinterpret_cast<void *>(&k_step_wg<13, NW, SYNC, MINW>);
    case 14: return reinterpret_cast<void *>(&k_step_wg<14, NW, SYNC, MINW>);
    case 15: return reinterpret_cast<void *>(&k_step_wg<15, NW, SYNC, MINW>);
    case 16: return reinterpret_cast<void *>(&k_step_wg<16, NW, SYNC, MINW>);
    default: return nullptr;
    }
}

// kMultiWg: 4 waves per band, capped where that costs no spills: 64 VGPRs (8 waves per
// SIMD) at K <= 12 (60 uncapped), 72 (7 waves) at K >= 13 (75 uncapped; 64 spills 28 B);
// kMultiWgNoBar / kMultiWgDiag: timing ablation / wait diagnostics (GOL_TOOLS build only)
static void *wg_fn(int turns, int variant)
{
    switch (variant) {
#if GOL_TOOLS
    case kMultiWgNoBar: return turns == 8 || turns == 16 ? wg_fn_nw<4, 0>(turns) : nullptr;
    case kMultiWgDiag: return turns == 8 || turns == 16 ? wg_fn_nw<4, 3>(turns) : nullptr;
#else
    case kMultiWgNoBar:
    case kMultiWgDiag: return nullptr;                  // wrong-result builds: tools only
#endif
    case kMultiWgHx: return wg_hx_kernel(turns, false);
    case kMultiWgPg: return wg_hx_kernel(turns, true);
    case kMultiWgHxS: return wg_ser_kernel(turns, false);
    case kMultiWgPgS: return wg_ser_kernel(turns, true);
    default: return turns >= 13 ? wg_fn_nw<4, 2, 7>(turns) : wg_fn_nw<4, 2, 8>(turns);
    }
}

void *wg_kernel(int turns, int variant) { return wg_fn(turns, variant); }

}  // namespace golk
