// gol_wg_ser.hip -- k_step_wg on helix tiles with each wave's stages in order within a step
// (kMultiWgHxS / kMultiWgPgS; SER in gol_wg.h).  Own translation unit (parallel builds).
#include "gol_wg.h"

namespace golk {

template <int MINW, bool PG>
static void *wg_ser_fn(int turns)
{
    switch (turns) {
    case 4: return reinterpret_cast<void *>(&k_step_wg<4, 4, 2, MINW, true, PG, true>);
    case 5: return reinterpret_cast<void *>(&k_step_wg<5, 4, 2, MINW, true, PG, true>);
    case 6: return reinterpret_cast<void *>(&k_step_wg<6, 4, 2, MINW, true, PG, true>);
    case 7: return reinterpret_cast<void *>(&k_step_wg<7, 4, 2, MINW, true, PG, true>);
    case 8: return reinterpret_cast<void *>(&k_step_wg<8, 4, 2, MINW, true, PG, true>);
    case 9: return reinterpret_cast<void *>(&k_step_wg<9, 4, 2, MINW, true, PG, true>);
    case 10: return reinterpret_cast<void *>(&k_step_wg<10, 4, 2, MINW, true, PG, true>);
    case 11: return reinterpret_cast<void *>(&k_step_wg<11, 4, 2, MINW, true, PG, true>);
    case 12: return reinterpret_cast<void *>(&k_step_wg<12, 4, 2, MINW, true, PG, true>);
    case 13: return reinterpret_cast<void *>(&k_step_wg<13, 4, 2, MINW, true, PG, true>);
    case 14: return reinterpret_cast<void *>(&k_step_wg<14, 4, 2, MINW, true, PG, true>);
    case 15: return reinterpret_cast<void *>(&k_step_wg<15, 4, 2, MINW, true, PG, true>);
    case 16: return reinterpret_cast<void *>(&k_step_wg<16, 4, 2, MINW, true, PG, true>);
    default: return nullptr;
    }
}

// In-order stages keep XS out of the live state across steps: K = 16 needs 61 VGPRs instead
// of 72, so the helix build fits 8 waves per SIMD at every K; the parallelogram build (K = 4,
// 8, 12, 16 only, pg_ok) keeps 8 up to K = 12 and 7 (67 VGPRs) at K = 16.
void *wg_ser_kernel(int turns, bool pg)
{
    if (pg) {
        if (turns % 4) return nullptr;
        return turns >= 13 ? wg_ser_fn<7, true>(turns) : wg_ser_fn<8, true>(turns);
    }
    return wg_ser_fn<8, false>(turns);
}

}  // namespace golk
