// gol_kernels.hip — gfx950 (MI355X) kernels of the Game of Life engine.
//
// Hot path: one B3/S23 toroidal turn of a bit-packed board, the MI355X
// replacement for the reference's byte-per-cell, branchy
//   calculateNextState     SubServer/distributor.go:119-208
// run over row strips by   SubServerDistributor/worker  SubServer/distributor.go:48-117
// and the Server strips     Server/gol/distributor.go:104-134,185-224.
//
// Board layout in HBM: row-major, 64 cells per uint64 word, LSB = lowest x
// (cell x of row y = bit x%64 of word y*pitch + x/64), bit set <=> byte == 255.
//
// K1 k_step_fast (width % 128 == 0, width >= 256) — the hot kernel.
//   One wavefront owns a tile of 128 words (64 lanes x 16 B, one coalesced
//   1 KiB dwordx4 access per row) and a band of `band` rows.  It walks the band
//   top to bottom with a 3-row sliding window kept in registers, so every input
//   row is read from HBM once per wavefront (plus 2 halo rows per band).
//   Horizontal neighbour bits come from the adjacent lanes by DPP wave_shl /
//   wave_shr (no LDS, no barriers: wavefronts are fully independent); the two
//   tile-edge dwords are wave-uniform loads.  Cells are bit-sliced 32 per dword:
//   per row  W = C<<1, E = C>>1 via v_alignbit, the 3-cell row sum (s0, s1) =
//   (xor3, majority) — v_bitop3 on gfx950 — and per output row the 9-cell total
//   T = sum of three 2-bit row sums; next = (T == 3) | (alive & T == 4), which is
//   B3/S23 with the centre included.  ~14 VALU ops per 32 cells: the kernel is
//   HBM-bound at 0.25 B per cell-update (1 bit read + 1 bit written).
// K1g k_step_generic — any width >= 2 (16x16, 64x64 fixtures), one thread per
//   word with explicit torus wrap for a partial last word.
// K2 k_popcount — AliveCellsCount (Server/gol/distributor.go:173-183).
// K3 k_row_popcount + k_alive_scatter — FinalTurnComplete's row-major alive
//   list (Local/gol/distributor.go:229-239) by stream compaction.
// K4 k_pack / k_unpack — PGM bytes <-> bits, with the non-binary mask.
#include "gol_device.h"

#include <type_traits>

namespace golk {

// ------------------------------------------------------- K1: fast stencil
struct RowSums {
    uint32_t s0[4], s1[4];
};

// 3-cell horizontal sums of one 128-cell lane segment.  L = the dword left of
// c.x (bit 31 used), R = the dword right of c.w (bit 0 used).
__device__ __forceinline__ RowSums row_sums(uint4 c, uint32_t L, uint32_t R)
{
    const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
    uint32_t w[4], e[4];
    w[0] = __builtin_amdgcn_alignbit(cc[0], L, 31);      // cell x-1
    w[1] = __builtin_amdgcn_alignbit(cc[1], cc[0], 31);
    w[2] = __builtin_amdgcn_alignbit(cc[2], cc[1], 31);
    w[3] = __builtin_amdgcn_alignbit(cc[3], cc[2], 31);
    e[0] = __builtin_amdgcn_alignbit(cc[1], cc[0], 1);   // cell x+1
    e[1] = __builtin_amdgcn_alignbit(cc[2], cc[1], 1);
    e[2] = __builtin_amdgcn_alignbit(cc[3], cc[2], 1);
    e[3] = __builtin_amdgcn_alignbit(R, cc[3], 1);
    RowSums s;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        s.s0[k] = w[k] ^ cc[k] ^ e[k];
        s.s1[k] = maj3(w[k], cc[k], e[k]);
    }
    return s;
}

template <bool BLK, bool CNT>
__global__ __launch_bounds__(256) void k_step_fast(const uint64_t *__restrict__ in,
                                                   uint64_t *__restrict__ out,
                                                   const uint64_t *__restrict__ blocked,
                                                   unsigned long long *__restrict__ counts,
                                                   StepArgs a, int ntx)
{
    const int lane = threadIdx.x & 63;
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);   // wavefront id (uniform)
    const int tx = wv % ntx;
    const int by = wv / ntx;
    const int y0 = a.row_lo + by * a.band;
    if (y0 >= a.row_hi) return;                            // whole wavefront
    const int y1 = min(y0 + a.band, a.row_hi);

    const int nd = a.nw * 2;                               // dwords per row
    const int tile0 = tx * (kTileWords * 2);
    const int tile_end = min(tile0 + kTileWords * 2, nd);
    const int d0 = tile0 + lane * 4;                       // this lane's first dword
    const bool act = d0 < nd;
    const int last_lane = ((tile_end - tile0) >> 2) - 1;
    const int lidx = tile0 == 0 ? nd - 1 : tile0 - 1;      // torus wrap in x
    const int ridx = tile_end == nd ? 0 : tile_end;

    const uint32_t *in32 = reinterpret_cast<const uint32_t *>(in);
    uint32_t *out32 = reinterpret_cast<uint32_t *>(out);
    const uint32_t *blk32 = reinterpret_cast<const uint32_t *>(blocked);
    const size_t pitch32 = (size_t)a.pitch * 2;
    const int M = a.modrows;
    auto rowbase = [&](int r) -> size_t {
        r = r < 0 ? r + M : (r >= M ? r - M : r);
        return (size_t)r * pitch32;
    };
    auto load_row = [&](size_t base, uint4 &v, uint32_t &hl, uint32_t &hr) {
        v = act ? *reinterpret_cast<const uint4 *>(in32 + base + d0) : make_uint4(0, 0, 0, 0);
        hl = in32[base + lidx];
        hr = in32[base + ridx];
    };
    auto sums = [&](uint4 v, uint32_t hl, uint32_t hr) -> RowSums {
        const uint32_t L = dpp_from_lower(hl, v.w);
        uint32_t R = dpp_from_upper(hr, v.x);
        R = lane == last_lane ? hr : R;
        return row_sums(v, L, R);
    };

    uint4 vp, vc, vn;
    uint32_t lp, rp, lc, rc, ln, rn;
    load_row(rowbase(y0 - 1), vp, lp, rp);
    load_row(rowbase(y0), vc, lc, rc);
    load_row(rowbase(y0 + 1), vn, ln, rn);
    RowSums A = sums(vp, lp, rp);
    RowSums B = sums(vc, lc, rc);
    unsigned long long acc = 0;

    for (int y = y0; y < y1; ++y) {
        uint4 vq = make_uint4(0, 0, 0, 0);
        uint32_t lq = 0, rq = 0;
        if (y + 2 <= y1) load_row(rowbase(y + 2), vq, lq, rq);   // prefetch
        const RowSums C = sums(vn, ln, rn);
        const uint32_t al[4] = {vc.x, vc.y, vc.z, vc.w};
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o[k] = life_rule(A.s0[k], A.s1[k], B.s0[k], B.s1[k], C.s0[k], C.s1[k], al[k]);
        const size_t ob = rowbase(y);
        if (BLK) {
            const uint4 m = act ? *reinterpret_cast<const uint4 *>(blk32 + ob + d0)
                                : make_uint4(0, 0, 0, 0);
            o[0] &= ~m.x; o[1] &= ~m.y; o[2] &= ~m.z; o[3] &= ~m.w;
        }
        if (act) *reinterpret_cast<uint4 *>(out32 + ob + d0) = make_uint4(o[0], o[1], o[2], o[3]);
        if (CNT && act && y >= a.cnt_lo && y < a.cnt_hi)
            acc += __builtin_popcount(o[0]) + __builtin_popcount(o[1]) +
                   __builtin_popcount(o[2]) + __builtin_popcount(o[3]);
        A = B; B = C; vc = vn;
        vn = vq; ln = lq; rn = rq;
    }
    if (CNT) {
        acc = wave_sum(acc);
        if (lane == 0 && acc) atomicAdd(counts + (wv & (kShards - 1)), acc);
    }
}


struct Slot {
    uint4 v;            // the lane's 4 dwords of this row
    uint32_t hl, hr;    // tile-edge dwords (left of lane 0, right of the last lane)
    uint32_t s0[4], s1[4];
};

template <bool BLK, bool CNT, int D, bool NT>
__global__ __launch_bounds__(256) void k_step_ring(const uint64_t *__restrict__ in,
                                                   uint64_t *__restrict__ out,
                                                   const uint64_t *__restrict__ blocked,
                                                   unsigned long long *__restrict__ counts,
                                                   StepArgs a, int ntx)
{
    constexpr int Q = D + 3;
    const int lane = threadIdx.x & 63;
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int tx = wv % ntx;
    const int by = wv / ntx;
    const int y0 = a.row_lo + by * a.band;
    if (y0 >= a.row_hi) return;
    const int y1 = min(y0 + a.band, a.row_hi);       // outputs [y0, y1); inputs [y0-1, y1]

    const int nd = a.nw * 2;
    const int tile0 = tx * (kTileWords * 2);
    const int tile_end = min(tile0 + kTileWords * 2, nd);
    const int d0 = tile0 + lane * 4;
    const bool act = d0 < nd;
    const int last_lane = ((tile_end - tile0) >> 2) - 1;
    const int lidx = tile0 == 0 ? nd - 1 : tile0 - 1;
    const int ridx = tile_end == nd ? 0 : tile_end;

    const uint32_t *in32 = reinterpret_cast<const uint32_t *>(in);
    const_u32p in32s = (const_u32p)in32;   // wave-uniform edge dwords via the scalar path
    uint32_t *out32 = reinterpret_cast<uint32_t *>(out);
    const uint32_t *blk32 = reinterpret_cast<const uint32_t *>(blocked);
    const size_t pitch32 = (size_t)a.pitch * 2;
    const int M = a.modrows;
    auto rowbase = [&](int r) -> size_t {
        r = r < 0 ? r + M : (r >= M ? r - M : r);
        return (size_t)r * pitch32;
    };
    auto load = [&](Slot &sl, int r) {
        const size_t b = rowbase(r);
        sl.v = act ? *reinterpret_cast<const uint4 *>(in32 + b + d0) : make_uint4(0, 0, 0, 0);
        sl.hl = in32s[b + lidx];
        sl.hr = in32s[b + ridx];
    };
    auto sums = [&](Slot &sl) {
        const uint32_t L = dpp_from_lower(sl.hl, sl.v.w);
        uint32_t R = dpp_from_upper(sl.hr, sl.v.x);
        R = lane == last_lane ? sl.hr : R;
        const uint32_t c[4] = {sl.v.x, sl.v.y, sl.v.z, sl.v.w};
        uint32_t w[4], e[4];
        w[0] = __builtin_amdgcn_alignbit(c[0], L, 31);
        w[1] = __builtin_amdgcn_alignbit(c[1], c[0], 31);
        w[2] = __builtin_amdgcn_alignbit(c[2], c[1], 31);
        w[3] = __builtin_amdgcn_alignbit(c[3], c[2], 31);
        e[0] = __builtin_amdgcn_alignbit(c[1], c[0], 1);
        e[1] = __builtin_amdgcn_alignbit(c[2], c[1], 1);
        e[2] = __builtin_amdgcn_alignbit(c[3], c[2], 1);
        e[3] = __builtin_amdgcn_alignbit(R, c[3], 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            sl.s0[k] = xor3(w[k], c[k], e[k]);
            sl.s1[k] = maj(w[k], c[k], e[k]);
        }
    };

    Slot ring[Q];
    // prologue: rows y0-1 .. y0+D into slots 0 .. D+1; sums of y0-1 and y0
#pragma unroll
    for (int k = 0; k < D + 2; ++k)
        if (y0 - 1 + k <= y1) load(ring[k], y0 - 1 + k);
    sums(ring[0]);
    sums(ring[1]);
    unsigned long long acc = 0;

    // output row y uses slots (y-y0)%Q (row y-1), +1 (row y), +2 (row y+1); it prefetches
    // row y+1+D into slot (y-y0+Q-1)%Q, which held row y-2.
    auto body = [&](auto I, int y) {
        constexpr int i = decltype(I)::value;
        constexpr int sa = i % Q, sb = (i + 1) % Q, sc = (i + 2) % Q, sp = (i + Q - 1) % Q;
        if (y + 1 + D <= y1) load(ring[sp], y + 1 + D);
        sums(ring[sc]);
        const uint32_t al[4] = {ring[sb].v.x, ring[sb].v.y, ring[sb].v.z, ring[sb].v.w};
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t u0 = xor3(ring[sa].s0[k], ring[sb].s0[k], ring[sc].s0[k]);
            const uint32_t u1 = maj(ring[sa].s0[k], ring[sb].s0[k], ring[sc].s0[k]);
            const uint32_t v0 = xor3(ring[sa].s1[k], ring[sb].s1[k], ring[sc].s1[k]);
            const uint32_t v1 = maj(ring[sa].s1[k], ring[sb].s1[k], ring[sc].s1[k]);
            const uint32_t h1 = bitop3<0x14>(u1, v0, v1);      // (u1 ^ v0) & ~v1   : H == 1
            const uint32_t h2 = bitop3<0x42>(u1, v0, v1);      // H == 2
            const uint32_t x = bitop3<0x08>(u0, al[k], h2);     // ~u0 & alive & h2
            o[k] = bitop3<0xea>(u0, h1, x);                     // (u0 & h1) | x
        }
        const size_t ob = rowbase(y);
        if (BLK) {
            const uint4 m = act ? *reinterpret_cast<const uint4 *>(blk32 + ob + d0)
                                : make_uint4(0, 0, 0, 0);
            o[0] &= ~m.x; o[1] &= ~m.y; o[2] &= ~m.z; o[3] &= ~m.w;
        }
        if (act) {
            const uint4 ov = make_uint4(o[0], o[1], o[2], o[3]);
            uint4 *dst = reinterpret_cast<uint4 *>(out32 + ob + d0);
            if (NT) {
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 nv = {ov.x, ov.y, ov.z, ov.w};
                __builtin_nontemporal_store(nv, reinterpret_cast<u32x4 *>(dst));
            } else {
                *dst = ov;
            }
        }
        if (CNT && act && y >= a.cnt_lo && y < a.cnt_hi)
            acc += __builtin_popcount(o[0]) + __builtin_popcount(o[1]) +
                   __builtin_popcount(o[2]) + __builtin_popcount(o[3]);
    };

    int y = y0;
    for (; y + Q <= y1; y += Q)
        unroll_seq(std::make_integer_sequence<int, Q>{}, [&](auto I) { body(I, y + I); });
    // remainder (< Q rows), continuing the ring phase from 0
    unroll_seq(std::make_integer_sequence<int, Q - 1>{}, [&](auto I) {
        if (y + I < y1) body(I, y + I);
    });
    if (CNT) {
        acc = wave_sum(acc);
        if (lane == 0 && acc) atomicAdd(counts + (wv & (kShards - 1)), acc);
    }
}


// ---------------------------------------------------- K1g: generic stencil
__device__ __forceinline__ uint64_t west_word(const uint64_t *row, int j, int nw, int nb)
{
    const uint64_t carry = j > 0 ? (row[j - 1] >> 63) : ((row[nw - 1] >> (nb - 1)) & 1ull);
    return (row[j] << 1) | carry;
}
__device__ __forceinline__ uint64_t east_word(const uint64_t *row, int j, int nw, int nb)
{
    if (j < nw - 1) return (row[j] >> 1) | (row[j + 1] << 63);
    return (row[j] >> 1) | ((row[0] & 1ull) << (nb - 1));
}

template <bool BLK, bool CNT>
__global__ __launch_bounds__(256) void k_step_generic(const uint64_t *__restrict__ in,
                                                      uint64_t *__restrict__ out,
                                                      const uint64_t *__restrict__ blocked,
                                                      unsigned long long *__restrict__ counts,
                                                      StepArgs a)
{
    const int nb = a.width - 64 * (a.nw - 1);
    const uint64_t lm = nb == 64 ? ~0ull : ((1ull << nb) - 1);
    const long long total = (long long)(a.row_hi - a.row_lo) * a.nw;
    unsigned long long acc = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int y = a.row_lo + (int)(i / a.nw);
        const int j = (int)(i % a.nw);
        const int yn = y == 0 ? a.modrows - 1 : y - 1;
        const int ys = y == a.modrows - 1 ? 0 : y + 1;
        const uint64_t *rn = in + (size_t)yn * a.pitch;
        const uint64_t *rc = in + (size_t)y * a.pitch;
        const uint64_t *rs = in + (size_t)ys * a.pitch;
        uint64_t s0[3], s1[3];
        const uint64_t *rr[3] = {rn, rc, rs};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint64_t w = west_word(rr[k], j, a.nw, nb), c = rr[k][j],
                           e = east_word(rr[k], j, a.nw, nb);
            s0[k] = w ^ c ^ e;
            s1[k] = maj3(w, c, e);
        }
        uint64_t o = life_rule(s0[0], s1[0], s0[1], s1[1], s0[2], s1[2], rc[j]);
        if (j == a.nw - 1) o &= lm;
        if (BLK) o &= ~blocked[(size_t)y * a.pitch + j];
        out[(size_t)y * a.pitch + j] = o;
        if (CNT && y >= a.cnt_lo && y < a.cnt_hi) acc += __builtin_popcountll(o);
    }
    if (CNT) block_count(acc, counts);
}

// ------------------------------------------------------------ K2: popcount
__global__ __launch_bounds__(256) void k_popcount(const uint64_t *__restrict__ w, int nw,
                                                  int pitch, int row_lo, int row_hi,
                                                  unsigned long long *__restrict__ counts)
{
    const long long total = (long long)(row_hi - row_lo) * nw;
    unsigned long long acc = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int y = row_lo + (int)(i / nw), j = (int)(i % nw);
        acc += __builtin_popcountll(w[(size_t)y * pitch + j]);
    }
    block_count(acc, counts);
}

// ------------------------------------------------------- K4: pack / unpack
__global__ __launch_bounds__(256) void k_pack(const uint8_t *__restrict__ bytes, int width,
                                              int nrows, uint64_t *__restrict__ words,
                                              uint64_t *__restrict__ blocked, int nw, int pitch,
                                              int row0, unsigned long long *__restrict__ nonbin)
{
    const long long total = (long long)nrows * nw;
    unsigned long long acc = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int y = (int)(i / nw), j = (int)(i % nw);
        const uint8_t *src = bytes + (size_t)y * width + (size_t)64 * j;
        const int n = min(64, width - 64 * j);
        uint64_t al = 0, bl = 0;
        if (n == 64 && (width & 15) == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 v = reinterpret_cast<const uint4 *>(src)[q];
                const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const uint32_t b = (d[k >> 2] >> (8 * (k & 3))) & 0xffu;
                    al |= (uint64_t)(b == 255u) << (16 * q + k);
                    bl |= (uint64_t)(b != 255u && b != 0u) << (16 * q + k);
                }
            }
        } else {
            for (int k = 0; k < n; ++k) {
                const uint32_t b = src[k];
                al |= (uint64_t)(b == 255u) << k;
                bl |= (uint64_t)(b != 255u && b != 0u) << k;
            }
        }
        words[(size_t)(row0 + y) * pitch + j] = al;
        if (blocked) blocked[(size_t)(row0 + y) * pitch + j] = bl;
        acc += __builtin_popcountll(bl);
    }
    block_count(acc, nonbin);
}

__global__ __launch_bounds__(256) void k_unpack(const uint64_t *__restrict__ words, int width,
                                                int nw, int pitch, int row0, int nrows,
                                                uint8_t *__restrict__ bytes)
{
    const long long total = (long long)nrows * nw;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int y = (int)(i / nw), j = (int)(i % nw);
        const uint64_t w = words[(size_t)(row0 + y) * pitch + j];
        uint8_t *dst = bytes + (size_t)y * width + (size_t)64 * j;
        const int n = min(64, width - 64 * j);
        if (n == 64 && (width & 15) == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t d[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const uint32_t bits = (uint32_t)(w >> (16 * q + 4 * m)) & 0xfu;
                    d[m] = ((bits & 1u) ? 0xffu : 0u) | ((bits & 2u) ? 0xff00u : 0u) |
                           ((bits & 4u) ? 0xff0000u : 0u) | ((bits & 8u) ? 0xff000000u : 0u);
                }
                reinterpret_cast<uint4 *>(dst)[q] = make_uint4(d[0], d[1], d[2], d[3]);
            }
        } else {
            for (int k = 0; k < n; ++k) dst[k] = ((w >> k) & 1ull) ? 255 : 0;
        }
    }
}

__global__ __launch_bounds__(256) void k_fill_random(uint64_t *__restrict__ words, int width,
                                                     int nw, int pitch, int nrows,
                                                     long long grow0, int gheight,
                                                     uint64_t seed)
{
    const int nb = width - 64 * (nw - 1);
    const uint64_t lm = nb == 64 ? ~0ull : ((1ull << nb) - 1);
    const long long total = (long long)nrows * nw;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int b = (int)(i / nw), j = (int)(i % nw);
        long long g = (grow0 + b) % gheight;
        if (g < 0) g += gheight;
        uint64_t v = splitmix64((seed << 40) + (uint64_t)g * nw + j);
        if (j == nw - 1) v &= lm;
        words[(size_t)b * pitch + j] = v;
    }
}

// ------------------------------------------------------- K3: alive list
// ------------------------------------------- layout: standard <-> interleaved words
// The interleaved layout (k_step_skew<IL>, 2 dwords per lane) keeps each 64-cell word's
// even cells in its low dword (cell 2i -> bit i) and its odd cells in the high dword
// (cell 2i+1 -> bit 32+i): the inverse perfect shuffle, five delta swaps (Hacker's
// Delight 7-2).  Row pitches are in words; one thread per word, grid-stride.
__device__ __forceinline__ uint64_t dswap(uint64_t x, int s, uint64_t m)
{
    const uint64_t t = (x ^ (x >> s)) & m;
    return x ^ t ^ (t << s);
}
__device__ __forceinline__ uint64_t il_unshuffle(uint64_t x)
{
    x = dswap(x, 1, 0x2222222222222222ull);
    x = dswap(x, 2, 0x0C0C0C0C0C0C0C0Cull);
    x = dswap(x, 4, 0x00F000F000F000F0ull);
    x = dswap(x, 8, 0x0000FF000000FF00ull);
    return dswap(x, 16, 0x00000000FFFF0000ull);
}
__device__ __forceinline__ uint64_t il_shuffle(uint64_t x)
{
    x = dswap(x, 16, 0x00000000FFFF0000ull);
    x = dswap(x, 8, 0x0000FF000000FF00ull);
    x = dswap(x, 4, 0x00F000F000F000F0ull);
    x = dswap(x, 2, 0x0C0C0C0C0C0C0C0Cull);
    return dswap(x, 1, 0x2222222222222222ull);
}

template <bool TO_IL>
__global__ __launch_bounds__(256) void k_il_convert(const uint64_t *__restrict__ in, int in_pitch,
                                                    uint64_t *__restrict__ out, int out_pitch,
                                                    int nrows, int nw)
{
    const long long total = (long long)nrows * nw;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int r = (int)(i / nw), j = (int)(i % nw);
        const uint64_t v = in[(size_t)r * in_pitch + j];
        out[(size_t)r * out_pitch + j] = TO_IL ? il_unshuffle(v) : il_shuffle(v);
    }
}

// One wavefront per row.
__global__ __launch_bounds__(256) void k_row_popcount(const uint64_t *__restrict__ w, int nw,
                                                      int pitch, int row0, int nrows,
                                                      long long *__restrict__ row_counts)
{
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= nrows) return;
    const uint64_t *row = w + (size_t)(row0 + r) * pitch;
    unsigned long long acc = 0;
    for (int j = lane; j < nw; j += 64) acc += __builtin_popcountll(row[j]);
    acc = wave_sum(acc);
    if (lane == 0) row_counts[r] = (long long)acc;
}

__global__ __launch_bounds__(256) void k_alive_scatter(const uint64_t *__restrict__ w, int nw,
                                                       int pitch, int row0, int nrows,
                                                       long long grow0,
                                                       const long long *__restrict__ row_off,
                                                       long long *__restrict__ xy)
{
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= nrows) return;
    const uint64_t *row = w + (size_t)(row0 + r) * pitch;
    long long base = row_off[r];
    const long long y = grow0 + r;
    for (int j0 = 0; j0 < nw; j0 += 64) {
        const int j = j0 + lane;
        uint64_t v = j < nw ? row[j] : 0ull;
        const int c = __builtin_popcountll(v);
        // inclusive scan of c across the wavefront
        int incl = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(incl, off, 64);
            if (lane >= off) incl += t;
        }
        long long o = base + incl - c;
        while (v) {
            const int b = __builtin_ctzll(v);
            xy[2 * o] = 64LL * j + b;
            xy[2 * o + 1] = y;
            ++o;
            v &= v - 1;
        }
        base += __shfl(incl, 63, 64);
    }
}

// ------------------------------------------------------------- launchers
static inline int grid_for(long long total, int cap = 2048)
{
    long long g = (total + 255) / 256;
    if (g < 1) g = 1;
    return (int)(g > cap ? cap : g);
}

bool fast_path_ok(int width) { return width >= 256 && (width % 128) == 0; }

int auto_band(int width, int rows)
{
    const int nw = (width + 63) / 64;
    const long long ntx = fast_path_ok(width) ? (nw + kTileWords - 1) / kTileWords : 1;
    const long long row_tiles = (long long)rows * ntx;
    // Measured on MI355X (tools/sweep.py): short bands win -- 16 rows at 65536^2
    // (32768 wavefronts, ~8 residency rounds at 4 waves/SIMD), 8 rows at 16384^2.
    // The 2 halo rows per band are L2/MALL re-reads, not HBM traffic.
    long long b = row_tiles / 32768;
    if (b < 8) b = 8;
    if (b > 64) b = 64;
    return (int)b;
}

const int kVariantDefault = kVariantRing3;

template <bool BLK, bool CNT>
static void launch_fast(const StepArgs &a, int ntx, int blocks, hipStream_t s)
{
    switch (a.variant) {
    case kVariantWindow:
        hipLaunchKernelGGL((k_step_fast<BLK, CNT>), dim3(blocks), dim3(256), 0, s, a.in, a.out,
                           a.blocked, a.counts, a, ntx);
        break;
    case kVariantRing2:
        hipLaunchKernelGGL((k_step_ring<BLK, CNT, 2, false>), dim3(blocks), dim3(256), 0, s,
                           a.in, a.out, a.blocked, a.counts, a, ntx);
        break;
    case kVariantRing3NT:
        hipLaunchKernelGGL((k_step_ring<BLK, CNT, 3, true>), dim3(blocks), dim3(256), 0, s,
                           a.in, a.out, a.blocked, a.counts, a, ntx);
        break;
    case kVariantRing5:
        hipLaunchKernelGGL((k_step_ring<BLK, CNT, 5, false>), dim3(blocks), dim3(256), 0, s,
                           a.in, a.out, a.blocked, a.counts, a, ntx);
        break;
    case kVariantRing7:
        hipLaunchKernelGGL((k_step_ring<BLK, CNT, 7, false>), dim3(blocks), dim3(256), 0, s,
                           a.in, a.out, a.blocked, a.counts, a, ntx);
        break;
    case kVariantRing5NT:
        hipLaunchKernelGGL((k_step_ring<BLK, CNT, 5, true>), dim3(blocks), dim3(256), 0, s,
                           a.in, a.out, a.blocked, a.counts, a, ntx);
        break;
    case kVariantRing3:
    default:
        hipLaunchKernelGGL((k_step_ring<BLK, CNT, 3, false>), dim3(blocks), dim3(256), 0, s,
                           a.in, a.out, a.blocked, a.counts, a, ntx);
        break;
    }
}

template <bool BLK, bool CNT>
static void launch_generic(const StepArgs &a, hipStream_t s)
{
    const int g = grid_for((long long)(a.row_hi - a.row_lo) * a.nw);
    hipLaunchKernelGGL((k_step_generic<BLK, CNT>), dim3(g), dim3(256), 0, s, a.in, a.out,
                       a.blocked, a.counts, a);
}

hipError_t launch_step(const StepArgs &a, bool fast, hipStream_t s)
{
    if (a.row_hi <= a.row_lo) return hipSuccess;
    const bool blk = a.blocked != nullptr, cnt = a.counts != nullptr;
    if (fast) {
        const int ntx = (a.nw + kTileWords - 1) / kTileWords;
        const int nbands = (a.row_hi - a.row_lo + a.band - 1) / a.band;
        const long long nwaves = (long long)ntx * nbands;
        const int blocks = (int)((nwaves + 3) / 4);
        if (blk && cnt) launch_fast<true, true>(a, ntx, blocks, s);
        else if (blk) launch_fast<true, false>(a, ntx, blocks, s);
        else if (cnt) launch_fast<false, true>(a, ntx, blocks, s);
        else launch_fast<false, false>(a, ntx, blocks, s);
    } else {
        if (blk && cnt) launch_generic<true, true>(a, s);
        else if (blk) launch_generic<true, false>(a, s);
        else if (cnt) launch_generic<false, true>(a, s);
        else launch_generic<false, false>(a, s);
    }
    return hipGetLastError();
}

int multi_max_turns(int variant)
{
    if (variant == kMultiTile) return kMaxTileTurns;
    if (variant == kMultiWgHx || variant == kMultiWgPg) return GOL_TOOLS ? kWgDeepMax : 16;
    if (variant == kMultiWgHxS || variant == kMultiWgPgS) return 16;
    return is_wg_variant(variant) ? 16 : variant == kMultiSkewILW16 ? 12 : 8;
}

int multi_waves_per_band(int variant, int turns)
{
    return is_wg_variant(variant) ? wg_waves(turns) : 1;
}

int multi_pipes_per_block(int variant) { return is_wg_variant(variant) ? 1 : 4; }

bool multi_is_il(int words_per_lane, int variant)
{
    return (is_il_variant(variant) || variant >= kMultiAblate) && words_per_lane == 1;
}

int multi_lane_dwords(int words_per_lane, int variant)
{
    return variant == kMultiSkewD1 ? 1 : 2 * words_per_lane;
}

long long multi_tiles(int width, int lane_dwords)
{
    const long long nd = 2ll * ((width + 63) / 64);
    return (nd + 62 * lane_dwords - 1) / (62 * lane_dwords);
}

long long multi_pipes(int width, int rows, int band, int lane_dwords, int variant)
{
    const long long nb = (rows + band - 1) / band;
    if (is_helix_variant(variant)) {
        // stored virtual lanes run up to nb (nw + 4) - 3; tile t stores [62t + 1, 62t + 62]
        const long long nwv = (width + 63) / 64 + 4;
        return (nb * nwv - 3 + 61) / 62;
    }
    return multi_tiles(width, lane_dwords) * nb;
}

int auto_band_multi(int width, int rows, int lane_dwords)
{
    // a band re-reads 2K halo rows and runs 2K pipeline fill steps, so bands are taller
    // than for k=1: 64 rows at 65536^2 (9216 wavefronts), 16 at 16384^2 (measured).
    long long b = (long long)rows * multi_tiles(width, lane_dwords) / 9216;
    if (b < 16) b = 16;
    if (b > 64) b = 64;
    return (int)b;
}

bool multi_ok(int width, int turns, int variant)
{
    return fast_path_ok(width) && turns >= 2 && turns <= multi_max_turns(variant);
}

bool multi_fits(int nw, int pitch, int rows)
{
    (void)nw;
    return (long long)rows * pitch * 8 < (1ll << 31);   // k_step_skew buffer ranges < 2 GiB
}

// k_step_wg: one workgroup (4 waves) per (tile, band) pipeline; depths 2, 3 run on
// k_step_skew (same interleaved layout and tiles)
static hipError_t launch_wg(const StepArgs &a0, int turns, hipStream_t s)
{
    StepArgs a = a0;                                    // other shapes / no scratch: helix
    const bool ser = a.multi_variant == kMultiWgPgS;
    if (is_pg_variant(a.multi_variant) &&
        (!pg_ok(turns, a.band, ser) || !a.xrows || !a.xflags))
        a.multi_variant = ser ? kMultiWgHxS : kMultiWgHx;
    const bool hx = is_helix_variant(a.multi_variant);
    const long long blocks =
        multi_pipes(a.width, a.row_hi - a.row_lo, a.band, 2, a.multi_variant);
    // band tiling: tiles per band; helix: the tile count itself (blockIdx.x = tile)
    const int ntx = hx ? (int)blocks : (int)multi_tiles(a.width, 2);
    void *fn = wg_kernel(turns, a.multi_variant);
    if (!fn) return hipErrorInvalidValue;
    const int threads = 64 * multi_waves_per_band(a.multi_variant, turns);
    StepArgs args = a;
    const uint64_t *in = a.in;
    uint64_t *out = a.out;
    int ntx_arg = ntx;
    void *params[] = {&in, &out, &args, &ntx_arg};
    return hipLaunchKernel(fn, dim3((unsigned)blocks), dim3(threads), params, 0, s);
}

template <int V>
static hipError_t launch_multi_v(const StepArgs &a, int turns, hipStream_t s)
{
    int var = a.multi_variant;                          // depths D1 lacks: 2 dwords per lane
    if (is_wg_variant(var)) {
        if (V == 1 && turns >= 4) return launch_wg(a, turns, s);
        var = kMultiSkewILW16;                          // same layout and tiles
    }
    if (var == kMultiSkewD1 && !(V == 1 && (turns == 4 || turns == 6 || turns == 8)))
        var = kMultiSkew;
    if (is_il_variant(var) && V != 1) var = kMultiSkew;  // multi_is_il() is false for V = 2
    const int ntx = (int)multi_tiles(a.width, multi_lane_dwords(V, var));
    const int nbands = (a.row_hi - a.row_lo + a.band - 1) / a.band;
    const long long nwaves = (long long)ntx * nbands;
    const int blocks = (int)((nwaves + 3) / 4);
    void *fn = skew_kernel(V, turns, var);
    if (!fn) return hipErrorInvalidValue;
    StepArgs args = a;
    const uint64_t *in = a.in;
    uint64_t *out = a.out;
    int ntx_arg = ntx;
    void *params[] = {&in, &out, &args, &ntx_arg};
    return hipLaunchKernel(fn, dim3(blocks), dim3(256), params, 0, s);
}

template <int V>
static int multi_blocks_per_cu_v(int turns, int variant)
{
    if (variant == kMultiTile) return 1;                // shape-dependent: the engine plans it
    int blocks = 0;
    void *fn = is_wg_variant(variant) ? (V == 1 ? wg_kernel(turns, variant) : nullptr)
                                      : skew_kernel(V, turns, variant);
    if (!fn) return 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn,
                                                        64 * multi_waves_per_band(variant, turns),
                                                        0) == hipSuccess
               ? blocks
               : 0;
}

int multi_blocks_per_cu(int turns, int words_per_lane, int variant)
{
    return words_per_lane == 1 ? multi_blocks_per_cu_v<1>(turns, variant)
                               : multi_blocks_per_cu_v<2>(turns, variant);
}

int pick_band_multi(int width, int rows, int lane_dwords, int turns, int capacity_waves,
                    int variant)
{
    // Every wavefront of a launch does the same work, so a launch takes ~ rounds x
    // (per-wavefront time), rounds = ceil(waves / resident capacity): a grid that spills
    // a few waves into an extra round wastes most of that round (measured: the 65536^2
    // K=6 launch at 4.25 rounds).  Per-wavefront time ~ K x band + K (K + 1) stage-steps
    // (band rows, 2K halo rows, minus the skipped pipeline fill).  Pick the band that
    // minimises rounds x per-wave time, charging at least 2 rounds (a single round that
    // starts and ends every wavefront together measured slower: 65536^2 K=6 band 274 vs
    // 137, 60.6 vs 58.0 us/turn); ties go to the smaller band.
    if (capacity_waves <= 0) return auto_band_multi(width, rows, lane_dwords);
    long long best_cost = -1;
    int best = 16;
    for (int band = 16; band <= 1024; ++band) {
        const long long nb = (rows + band - 1) / band;
        const long long waves = multi_pipes(width, rows, band, lane_dwords, variant);
        long long rounds = (waves + capacity_waves - 1) / capacity_waves;
        if (rounds < 2) rounds = 2;
        const long long cost = rounds * ((long long)turns * band + (long long)turns * (turns + 1));
        if (best_cost < 0 || cost < best_cost) {
            best_cost = cost;
            best = band;
        }
        if (nb == 1) break;
    }
    return best;
}

hipError_t launch_step_multi(const StepArgs &a, int turns, hipStream_t s)
{
    if (a.row_hi <= a.row_lo) return hipSuccess;
    if (a.multi_variant == kMultiTile) return launch_tile(a, turns, s);
    if (!GOL_TOOLS && a.multi_words != 1) return hipErrorInvalidValue;   // tools build only
    return a.multi_words == 1 ? launch_multi_v<1>(a, turns, s) : launch_multi_v<2>(a, turns, s);
}

hipError_t launch_popcount(const uint64_t *w, int nw, int pitch, int row_lo, int row_hi,
                           unsigned long long *counts, hipStream_t s)
{
    const int g = grid_for((long long)(row_hi - row_lo) * nw, 1024);
    hipLaunchKernelGGL(k_popcount, dim3(g), dim3(256), 0, s, w, nw, pitch, row_lo, row_hi,
                       counts);
    return hipGetLastError();
}

hipError_t launch_pack(const uint8_t *bytes, int width, int nrows, uint64_t *words,
                       uint64_t *blocked, int nw, int pitch, int row0,
                       unsigned long long *nonbin, hipStream_t s)
{
    const int g = grid_for((long long)nrows * nw);
    hipLaunchKernelGGL(k_pack, dim3(g), dim3(256), 0, s, bytes, width, nrows, words, blocked,
                       nw, pitch, row0, nonbin);
    return hipGetLastError();
}

hipError_t launch_unpack(const uint64_t *words, int width, int nw, int pitch, int row0,
                         int nrows, uint8_t *bytes, hipStream_t s)
{
    const int g = grid_for((long long)nrows * nw);
    hipLaunchKernelGGL(k_unpack, dim3(g), dim3(256), 0, s, words, width, nw, pitch, row0, nrows,
                       bytes);
    return hipGetLastError();
}

hipError_t launch_il_convert(const uint64_t *in, int in_pitch, uint64_t *out, int out_pitch,
                             int nrows, int nw, bool to_il, hipStream_t s)
{
    if (nrows <= 0) return hipSuccess;
    const int g = grid_for((long long)nrows * nw);
    if (to_il)
        hipLaunchKernelGGL(k_il_convert<true>, dim3(g), dim3(256), 0, s, in, in_pitch, out,
                           out_pitch, nrows, nw);
    else
        hipLaunchKernelGGL(k_il_convert<false>, dim3(g), dim3(256), 0, s, in, in_pitch, out,
                           out_pitch, nrows, nw);
    return hipGetLastError();
}

hipError_t launch_fill_random(uint64_t *words, int width, int nw, int pitch, int nrows,
                              long long grow0, int gheight, uint64_t seed, hipStream_t s)
{
    const int g = grid_for((long long)nrows * nw);
    hipLaunchKernelGGL(k_fill_random, dim3(g), dim3(256), 0, s, words, width, nw, pitch, nrows,
                       grow0, gheight, seed);
    return hipGetLastError();
}

hipError_t launch_row_popcount(const uint64_t *w, int nw, int pitch, int row0, int nrows,
                               long long *row_counts, hipStream_t s)
{
    const int blocks = (nrows + 3) / 4;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_row_popcount, dim3(blocks), dim3(256), 0, s, w, nw, pitch, row0, nrows,
                       row_counts);
    return hipGetLastError();
}

hipError_t launch_alive_scatter(const uint64_t *w, int nw, int pitch, int row0, int nrows,
                                long long grow0, const long long *row_offsets, long long *xy,
                                hipStream_t s)
{
    const int blocks = (nrows + 3) / 4;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_alive_scatter, dim3(blocks), dim3(256), 0, s, w, nw, pitch, row0,
                       nrows, grow0, row_offsets, xy);
    return hipGetLastError();
}

}  // namespace golk
