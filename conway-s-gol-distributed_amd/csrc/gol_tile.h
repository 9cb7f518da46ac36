// gol_tile.h -- K1t k_step_tile: K turns per launch on a 2-D tile held in registers, for
// boards too small to fill the GPU with K1s / K1w band pipelines (BASELINE configs[1],
// 5120^2: 80 words per row, 409 600 words in all -- a K1w band pipeline per workgroup leaves
// most CUs idle or runs 16-row bands that are mostly pipeline fill: 1.6 us per turn at best,
// tools/sweep.py).
//
// One workgroup per tile of TH rows x TW words (the reference's calculateNextState over a
// sub-rectangle, SubServer/distributor.go:119-208, advanced K turns at once):
//   * Tile + halo.  The workgroup loads rows [y0 - K, y0 + TH + K) of words
//     [x0 - 1, x0 + TW + 1) (torus wrap), C = TW + 2 words per row: K halo rows above and
//     below, one halo word (64 cells) left and right.  Cells next to the loaded region are
//     unknown; the error they cause moves one cell (row) per turn, so after K <= 64 turns it
//     is still inside the halos and the TH x TW interior is exact.
//   * Lanes.  A wave holds G = 64 / C row segments side by side: lane = group * C + column.
//     Each lane keeps SEG consecutive rows of its word column in registers (2 dwords per
//     row, interleaved layout) for all K turns: the tile never round-trips through memory
//     between turns.  Horizontal neighbours come from the adjacent lanes by DPP (the lanes
//     at a group edge read another group's word: only the halo columns see that); the
//     1-bit funnel shifts and the 7-op rule are K1s's (gol_device.h, life_rule7).
//   * Vertical neighbours.  Per turn each lane sums its segment's first and last row (the
//     3-cell horizontal sums every rule needs) and publishes the two sums in LDS
//     (double-buffered by turn parity: one barrier per turn), then reads the sums of the row
//     above its segment (the previous segment's last) and of the row below (the next one's
//     first), and sweeps its segment top to bottom with a 3-row window of row sums,
//     overwriting each row in place once its sums are taken.  Every row is summed once per
//     turn (exchanging raw rows cost each lane 2 extra row sums a turn: +33 % at SEG = 4).
//   * After K turns the lanes holding interior rows and columns store them.
// Work per turn and lane: SEG row sums (2 DPP, 2 v_alignbit, 4 v_bitop3) + SEG rules
// (14 v_bitop3) + 4 16-B LDS accesses; waste = the (TH + 2K) / TH halo rows, C / TW halo
// columns and the 64 - G C idle lanes.  The engine (tile_candidates + autotune) picks TW, TH,
// SEG and K.
#pragma once
#include "gol_device.h"

namespace golk {

constexpr int kTileMaxWaves = 16;                       // 1024 threads per workgroup
// dynamic LDS of a workgroup of `threads` threads: row sums of the segments' edge rows,
// first and last row, two turn parities, 16 B each
constexpr size_t tile_lds_bytes(int threads) { return (size_t)threads * 4 * 16; }

template <int SEG>
__global__ __launch_bounds__(1024, 1) void k_step_tile(const uint64_t *__restrict__ in,
                                                     uint64_t *__restrict__ out, StepArgs a,
                                                     int turns, int ntx, int ntiles)
{
    // per turn parity: the 3-cell row sums (4 dwords) of the first / last row of every segment,
    // segment-major, C slots per segment (dynamic LDS: 2 x 2 x waves x 64 x 16 B)
    extern __shared__ uint4 xsh[];
    const int nslot = (int)(blockDim.x);                 // waves x 64 >= segments x C
    const int TW = a.tile_w, C = TW + 2, G = 64 / C;
    const int K = turns, TH = a.band;
    // XCD-aware tile order: blockIdx b runs on XCD b % 8, which gets a contiguous run of
    // tiles (whole tile rows, so most halo rows were written by the same XCD's L2)
    const int per = (ntiles + 7) / 8;
    const int tile = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
    if (tile >= ntiles) return;                          // the whole workgroup
    const int ty = tile / ntx, tx = tile - ty * ntx;
    const int y0 = a.row_lo + ty * TH;
    const int x0 = tx * TW;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int group = lane / C, col = lane - group * C;
    const bool live = group < G;                         // lanes past G groups: idle
    const int seg = wave * G + group;                    // segment index within the tile
    const int nseg = (TH + 2 * K + SEG - 1) / SEG;       // segments the tile needs
    const int slot = seg * C + col;

    // word column (torus wrap) and the lane's rows: tile row t = seg * SEG + i is buffer row
    // y0 - K + t (mod modrows; rows past the tile are read, never stored)
    int gx = x0 - 1 + (live ? col : 0);
    while (gx < 0) gx += a.nw;
    while (gx >= a.nw) gx -= a.nw;
    const int M = a.modrows;
    const uint32_t pitch_b = (uint32_t)a.pitch * 8u;
    const uint32_t span = (uint32_t)M * pitch_b;
    int r = y0 - K + (live ? seg : 0) * SEG;
    while (r < 0) r += M;
    while (r >= M) r -= M;
    uint32_t off = (uint32_t)r * pitch_b + (uint32_t)gx * 8u;
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc((void *)in, (short)0, (int)span, kBufFlags);
    const __amdgpu_buffer_rsrc_t rout =
        __builtin_amdgcn_make_buffer_rsrc((void *)out, (short)0, (int)span, kBufFlags);

    uint32_t v[SEG][2];
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
        const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(rin, off, 0, 0);
        v[i][0] = w.x;
        v[i][1] = w.y;
        off += pitch_b;
        off = off >= span ? off - span : off;            // (the column stays < pitch_b)
    }

    // 3-cell row sums of one row (even dword: s0e/s1e, odd dword: s0o/s1o): K1s's stage
    auto rsum = [](const uint32_t (&x)[2], uint32_t (&s)[4]) {
        const uint32_t L = dpp_from_lower_z(x[1]);       // west word's odd cells
        const uint32_t Rt = dpp_from_upper_z(x[0]);      // east word's even cells
        const uint32_t wl0 = __builtin_amdgcn_alignbit(x[1], L, 31);
        const uint32_t er1 = __builtin_amdgcn_alignbit(Rt, x[0], 1);
        s[0] = xor3(wl0, x[0], x[1]);
        s[1] = maj(wl0, x[0], x[1]);
        s[2] = xor3(x[0], x[1], er1);
        s[3] = maj(x[0], x[1], er1);
    };
    uint4 *xtop[2] = {xsh, xsh + nslot};
    uint4 *xbot[2] = {xsh + 2 * nslot, xsh + 3 * nslot};
    const bool has_up = seg > 0, has_dn = seg + 1 < nseg;
    for (int t = 0; t < K; ++t) {
        const int p = t & 1;
        // the segment's first and last row sums go to the neighbours (row sums, not rows: no
        // lane sums a row twice -- SEG row sums and SEG rules per turn)
        uint32_t F[4], Lr[4];
        rsum(v[0], F);
        if (SEG > 1) rsum(v[SEG - 1], Lr);
        else {
#pragma unroll
            for (int k = 0; k < 4; ++k) Lr[k] = F[k];
        }
        if (live) {
            xtop[p][slot] = make_uint4(F[0], F[1], F[2], F[3]);
            xbot[p][slot] = make_uint4(Lr[0], Lr[1], Lr[2], Lr[3]);
        }
        __syncthreads();
        uint32_t A[4] = {0, 0, 0, 0}, D[4] = {0, 0, 0, 0};
        if (live && has_up) {
            const uint4 u = xbot[p][slot - C];
            A[0] = u.x; A[1] = u.y; A[2] = u.z; A[3] = u.w;
        }
        if (live && has_dn) {
            const uint4 d = xtop[p][slot + C];
            D[0] = d.x; D[1] = d.y; D[2] = d.z; D[3] = d.w;
        }
        // sweep: A = sums of the row above, B = this row's, Cs = the row below's
        uint32_t B[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) B[k] = F[k];
#pragma unroll
        for (int i = 0; i < SEG; ++i) {
            uint32_t Cs[4];
            if (i + 1 == SEG) {
#pragma unroll
                for (int k = 0; k < 4; ++k) Cs[k] = D[k];
            } else if (i + 2 == SEG) {
#pragma unroll
                for (int k = 0; k < 4; ++k) Cs[k] = Lr[k];
            } else {
                rsum(v[i + 1], Cs);
            }
            const uint32_t n0 = life_rule7(A[0], B[0], Cs[0], A[1], B[1], Cs[1], v[i][0]);
            const uint32_t n1 = life_rule7(A[2], B[2], Cs[2], A[3], B[3], Cs[3], v[i][1]);
            v[i][0] = n0;
            v[i][1] = n1;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                A[k] = B[k];
                B[k] = Cs[k];
            }
        }
    }
    // interior rows [K, K + TH) of the tile, below row_hi; interior columns inside the row
    if (!live || col < 1 || col > TW || x0 + col - 1 >= a.nw) return;
    const int t0 = seg * SEG;
    // per-lane byte offset (the segment differs between the lane groups of a wave); rows
    // y0 - K + t0 + i are stored only once inside [row_lo, row_hi): no wrap, and the
    // unsigned sum is exact there even if the first row of the segment lies above row 0
    uint32_t so = (uint32_t)(y0 - K + t0) * pitch_b + (uint32_t)(x0 + col - 1) * 8u;
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
        const int tr = t0 + i;
        if (tr >= K && tr < K + TH && y0 - K + tr < a.row_hi) {
            const uint32_t o[2] = {v[i][0], v[i][1]};
            buf_store(o, rout, so, 0);
        }
        so += pitch_b;
    }
}

}  // namespace golk
