// gol_tile.hip -- the k_step_tile instantiation table (K1t, gol_tile.h) and its launcher.
#include "gol_tile.h"

namespace golk {

void *tile_kernel(int seg)
{
    switch (seg) {
    case 2: return reinterpret_cast<void *>(&k_step_tile<2>);
    case 3: return reinterpret_cast<void *>(&k_step_tile<3>);
    case 4: return reinterpret_cast<void *>(&k_step_tile<4>);
    case 6: return reinterpret_cast<void *>(&k_step_tile<6>);
    case 8: return reinterpret_cast<void *>(&k_step_tile<8>);
    case 12: return reinterpret_cast<void *>(&k_step_tile<12>);
    case 16: return reinterpret_cast<void *>(&k_step_tile<16>);
    case 24: return reinterpret_cast<void *>(&k_step_tile<24>);
    case 32: return reinterpret_cast<void *>(&k_step_tile<32>);
    case 40: return reinterpret_cast<void *>(&k_step_tile<40>);
    case 48: return reinterpret_cast<void *>(&k_step_tile<48>);
    default: return nullptr;
    }
}

bool tile_shape_ok(int nw, int turns, int tile_h, int tile_w, int seg)
{
    if (turns < 2 || turns > 64 || tile_h < 1 || tile_w < 1 || tile_w + 2 > 64 || !tile_kernel(seg))
        return false;
    (void)nw;
    const int C = tile_w + 2, G = 64 / C;
    const int nseg = (tile_h + 2 * turns + seg - 1) / seg;
    return (nseg + G - 1) / G <= kTileMaxWaves;
}

int tile_waves(int turns, int tile_h, int tile_w, int seg)
{
    const int C = tile_w + 2, G = 64 / C;
    const int nseg = (tile_h + 2 * turns + seg - 1) / seg;
    return (nseg + G - 1) / G;
}

long long tile_count(int nw, int rows, int tile_h, int tile_w)
{
    const long long ntx = (nw + tile_w - 1) / tile_w;
    return ntx * ((rows + tile_h - 1) / tile_h);
}

hipError_t launch_tile(const StepArgs &a, int turns, hipStream_t s)
{
    const int rows = a.row_hi - a.row_lo;
    if (!tile_shape_ok(a.nw, turns, a.band, a.tile_w, a.tile_seg)) return hipErrorInvalidValue;
    const int ntx = (a.nw + a.tile_w - 1) / a.tile_w;
    const long long ntiles = (long long)ntx * ((rows + a.band - 1) / a.band);
    if (ntiles <= 0 || ntiles > (1 << 24)) return hipErrorInvalidValue;
    const unsigned blocks = (unsigned)((ntiles + 7) / 8 * 8);
    const int threads = 64 * tile_waves(turns, a.band, a.tile_w, a.tile_seg);
    void *fn = tile_kernel(a.tile_seg);
    StepArgs args = a;
    const uint64_t *in = a.in;
    uint64_t *out = a.out;
    int k = turns, ntx_arg = ntx, nt = (int)ntiles;
    void *params[] = {&in, &out, &args, &k, &ntx_arg, &nt};
    return hipLaunchKernel(fn, dim3(blocks), dim3(threads), params, tile_lds_bytes(threads), s);
}

}  // namespace golk
