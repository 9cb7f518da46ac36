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
#include "gol_kernels.h"

#include <type_traits>

namespace golk {

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t dpp_from_lower(uint32_t old_v, uint32_t v)
{
    // DPP wave_shr:1 — lane i receives lane i-1; lane 0 keeps old_v.
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old_v, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_from_upper(uint32_t old_v, uint32_t v)
{
    // DPP wave_shl:1 — lane i receives lane i+1; lane 63 keeps old_v.
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old_v, (int)v, 0x130, 0xf, 0xf, false);
}

// bound_ctrl forms: the lane without a source (0 / 63) reads 0 -- no `old` operand to
// materialise (the update_dpp(0, ...) form costs a v_mov per use)
__device__ __forceinline__ uint32_t dpp_from_lower_z(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t dpp_from_upper_z(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, true);
}

template <typename T>
__device__ __forceinline__ T maj3(T a, T b, T c) { return (a & b) | (c & (a | b)); }

// next state from three 2-bit row sums (above a, current b, below c) and the
// centre bits: T = a + b + c over the 3x3 window incl. the centre.
template <typename T>
__device__ __forceinline__ T life_rule(T a0, T a1, T b0, T b1, T c0, T c1, T alive)
{
    const T u0 = a0 ^ b0 ^ c0;          // bit 0 of T
    const T u1 = maj3(a0, b0, c0);      // carry of the low bits (weight 2)
    const T v0 = a1 ^ b1 ^ c1;          // weight 2
    const T v1 = maj3(a1, b1, c1);      // weight 4
    // H = u1 + v0 + 2 v1 ;  T = u0 + 2 H
    const T h1 = (u1 ^ v0) & ~v1;                       // H == 1
    const T h2 = (u1 & v0 & ~v1) | (~(u1 | v0) & v1);   // H == 2
    return (u0 & h1) | (~u0 & alive & h2);              // T == 3  |  (alive & T == 4)
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// block-wide sum (blockDim.x == 256) into one of kShards accumulators
__device__ __forceinline__ void block_count(unsigned long long acc, unsigned long long *counts)
{
    __shared__ unsigned long long part[4];
    acc = wave_sum(acc);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) part[w] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long s = part[0] + part[1] + part[2] + part[3];
        if (s) atomicAdd(counts + (blockIdx.x & (kShards - 1)), s);
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

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


// ------------------------------------------- K1 v2: register ring, D rows in flight
// Same algorithm as k_step_fast; the sliding window is a ring of Q = D + 3 row slots
// (rows y-1, y, y+1 summed + D raw rows in flight) so each wavefront keeps D KiB of
// loads outstanding, and the loop is unrolled by Q so every slot index is a
// compile-time constant (no register rotation moves).  xor3 / majority are single
// v_bitop3_b32 (truth tables 0x96 / 0xE8, symmetric in their operands).
// v_bitop3_b32 through the compiler builtin (no inline asm: no conservative hazard
// s_nops, and the scheduler sees the dependencies).  Truth-table index is
// (src0 << 2) | (src1 << 1) | src2 (checked against the compiler's own lowering of
// a & ~b & ~c -> bitop3:0x10).
template <int IMM>
__device__ __forceinline__ uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, IMM);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return bitop3<0x96>(a, b, c);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c)
{
    return bitop3<0xe8>(a, b, c);
}

// B3/S23 from the three rows' 3-cell sums (a, b, c: low bits a0 b0 c0, high bits a1 b1
// c1; the window's middle row b includes the centre) and the centre bit C.
// T = L + 2H with L = a0 + b0 + c0, H = a1 + b1 + c1; next = (T == 3) | (C & T == 4).
// life_rule8: L and H in binary (4 ops), then H' = L/2 + H compared with 1 and 2 (4 ops).
__device__ __forceinline__ uint32_t life_rule8(uint32_t a0, uint32_t b0, uint32_t c0, uint32_t a1,
                                               uint32_t b1, uint32_t c1, uint32_t C)
{
    const uint32_t u0 = xor3(a0, b0, c0);
    const uint32_t u1 = maj(a0, b0, c0);
    const uint32_t v0 = xor3(a1, b1, c1);
    const uint32_t v1 = maj(a1, b1, c1);
    const uint32_t h1 = bitop3<0x14>(u1, v0, v1);      // (u1 ^ v0) & ~v1   : H' == 1
    const uint32_t h2 = bitop3<0x42>(u1, v0, v1);      // H' == 2
    const uint32_t xx = bitop3<0x08>(u0, C, h2);       // ~u0 & C & h2
    return bitop3<0xea>(u0, h1, xx);                   // (u0 & h1) | xx
}
// life_rule7: 7 ops.  L is encoded as (L >= 2, L in {1,2}) -- majority and "not all
// equal" of the low bits -- and H as (H >= 2, H odd); the three final LUTs were found by
// an exhaustive search over 3-gate circuits on those 5 signals (no 2-gate circuit
// exists for any injective encoding) and are checked on all 512 3x3 windows by
// tests/test_host_cpu.py::test_rule7_truth_tables.
__device__ __forceinline__ uint32_t life_rule7(uint32_t a0, uint32_t b0, uint32_t c0, uint32_t a1,
                                               uint32_t b1, uint32_t c1, uint32_t C)
{
    const uint32_t lm = maj(a0, b0, c0);               // L >= 2
    const uint32_t lx = bitop3<0x7e>(a0, b0, c0);      // L in {1, 2}
    const uint32_t hm = maj(a1, b1, c1);               // H >= 2
    const uint32_t hx = xor3(a1, b1, c1);              // H odd
    const uint32_t g1 = bitop3<0x16>(lm, lx, C);
    const uint32_t g2 = bitop3<0x86>(hm, C, g1);
    return bitop3<0x82>(lx, hx, g2);
}

template <typename F, int... Is>
__device__ __forceinline__ void unroll_seq(std::integer_sequence<int, Is...>, F &&f)
{
    (f(std::integral_constant<int, Is>{}), ...);
}

struct Slot {
    uint4 v;            // the lane's 4 dwords of this row
    uint32_t hl, hr;    // tile-edge dwords (left of lane 0, right of the last lane)
    uint32_t s0[4], s1[4];
};

typedef const __attribute__((address_space(4))) uint32_t *const_u32p;
typedef __attribute__((address_space(3))) void lds_void;

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


// ------------------------------------- K1m: K turns per launch (temporal blocking)
// A wavefront owns a tile of 128 words (64 lanes x 2 words) whose first and last lane
// are halo lanes: only lanes 1..62 (124 words) are stored, tiles advance by 124 words.
// The tile edges are never loaded: DPP brings zeros into lane 0 / past the last lane,
// and that error travels one cell per turn, so after K <= 64 turns it is still inside
// the halo lanes (128 cells each).  Vertically, a band of `band` output rows reads
// input rows [y0-K, y1+K) once; stage j (j = 0..K-1) turns its input row stream into
// the stream of turn t+j+1 rows one row later, all in registers.  HBM traffic per
// launch is one read + one write of the board for K turns: 0.25/K B per cell-update.
// V = words per lane (2: 16-B accesses, 128-word tiles; 1: 8-B accesses, 64-word tiles,
// half the per-stage registers -> higher occupancy).  Tiles store lanes 1..62.
template <int V> struct LaneVec;
template <> struct LaneVec<2> { using T = uint4; };
template <> struct LaneVec<1> { using T = uint2; };

template <int V>
__device__ __forceinline__ void vec_get(const typename LaneVec<V>::T &v, uint32_t (&c)[2 * V]);
template <>
__device__ __forceinline__ void vec_get<2>(const uint4 &v, uint32_t (&c)[4])
{
    c[0] = v.x; c[1] = v.y; c[2] = v.z; c[3] = v.w;
}
template <>
__device__ __forceinline__ void vec_get<1>(const uint2 &v, uint32_t (&c)[2])
{
    c[0] = v.x; c[1] = v.y;
}
__device__ __forceinline__ uint4 vec_make(const uint32_t (&c)[4]) { return make_uint4(c[0], c[1], c[2], c[3]); }
__device__ __forceinline__ uint2 vec_make(const uint32_t (&c)[2]) { return make_uint2(c[0], c[1]); }

#ifndef MULTI_MIN_WAVES
#define MULTI_MIN_WAVES 1   // forcing 4-5 waves/SIMD spills (measured with -Rpass-analysis)
#endif
template <int K, int V>
__global__ __launch_bounds__(256, MULTI_MIN_WAVES) void k_step_multi(const uint64_t *__restrict__ in,
                                                    uint64_t *__restrict__ out, StepArgs a,
                                                    int ntx)
{
    constexpr int ND = 2 * V;                          // dwords per lane
    constexpr int STRIDE = 62 * V;                     // stored words per tile
    using Vec = typename LaneVec<V>::T;
    const int lane = threadIdx.x & 63;
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int tx = wv % ntx;
    const int by = wv / ntx;
    const int y0 = a.row_lo + by * a.band;
    if (y0 >= a.row_hi) return;
    const int y1 = min(y0 + a.band, a.row_hi);         // outputs [y0, y1)

    const int nw = a.nw;
    const int t0 = tx * STRIDE;                        // first stored word
    const int t1 = min(t0 + STRIDE, nw);               // end of stored words
    const int last = (t1 - t0 + V - 1) / V + 1;        // right halo lane
    const bool st = lane >= 1 && lane < last;
    // every lane loads (its word index wraps mod nw, so lanes past the right halo lane hold
    // the true torus neighbours): no exec-masked loads; only stores are masked
    int w = t0 - V + V * lane;                         // lane's first word (torus wrap)
    while (w < 0) w += nw;
    while (w >= nw) w -= nw;
    // dword offsets fit 32 bits: the host only launches this kernel on buffers of
    // < 2^31 dwords (multi_ok)
    const uint32_t pitch32 = (uint32_t)a.pitch * 2u;
    const uint32_t *in32 = reinterpret_cast<const uint32_t *>(in) + 2 * (size_t)w;
    uint32_t *out32 = reinterpret_cast<uint32_t *>(out) + 2 * (size_t)w;
    const int M = a.modrows;
    auto rowoff = [&](int r) -> uint32_t {   // r in [-K, M + K): may wrap more than once
        while (r < 0) r += M;
        while (r >= M) r -= M;
        return (uint32_t)r * pitch32;
    };
    // Row offsets advance by one row per step: keep them as wave-uniform running values
    // (a per-step rowoff() of a computed row turned into a VALU urem sequence).
    const uint32_t span = (uint32_t)M * pitch32;
    auto adv = [&](uint32_t &o) {
        o += pitch32;
        o = o >= span ? o - span : o;
    };
    auto load_at = [&](uint32_t off, uint32_t (&c)[ND]) {
        vec_get<V>(*reinterpret_cast<const Vec *>(in32 + off), c);
    };
    auto load = [&](int r, uint32_t (&c)[ND]) { load_at(rowoff(r), c); };
    // per stage: ring of 3 row sums and 3 raw input rows (phase = step % 3)
    uint32_t S0[K][3][ND], S1[K][3][ND], X[K][3][ND];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int k = 0; k < ND; ++k) S0[j][p][k] = S1[j][p][k] = X[j][p][k] = 0;
    uint32_t raw[3][ND];
    const int r_first = y0 - K, r_end = y1 + K;         // input rows [r_first, r_end)
    uint32_t ld_off = rowoff(r_first + 3);              // row prefetched by the next step
    uint32_t st_off = rowoff(r_first - K);              // row r - K stored by the next step
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        if (r_first + p < r_end) {
            load(r_first + p, raw[p]);
        } else {
#pragma unroll
            for (int k = 0; k < ND; ++k) raw[p][k] = 0;
        }
    }

    // One pipeline step: input row r enters stage 0, every active stage advances one row.
    // I = ring phase (step % 3), NS = active stages (compile-time).
    auto step = [&](auto I, auto NSc, int r) {
        constexpr int i = decltype(I)::value;
        constexpr int NS = decltype(NSc)::value;
        constexpr int pn = i % 3, p1 = (i + 2) % 3, p2 = (i + 1) % 3;
        uint32_t x[ND];
#pragma unroll
        for (int k = 0; k < ND; ++k) x[k] = raw[pn][k];
        if (r + 3 < r_end) load_at(ld_off, raw[pn]);
        adv(ld_off);
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            // row sums of the new input row, dword by dword, each consumed right away by
            // the rule so the oldest row's sums die early (register pressure)
            const uint32_t L = dpp_from_lower_z(x[ND - 1]);
            const uint32_t R = dpp_from_upper_z(x[0]);
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                const uint32_t wl = __builtin_amdgcn_alignbit(x[k], k == 0 ? L : x[k - 1], 31);
                const uint32_t er = __builtin_amdgcn_alignbit(k == ND - 1 ? R : x[k + 1], x[k], 1);
                S0[j][pn][k] = xor3(wl, x[k], er);
                S1[j][pn][k] = maj(wl, x[k], er);
                X[j][pn][k] = x[k];
            }
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                const uint32_t u0 = xor3(S0[j][p2][k], S0[j][p1][k], S0[j][pn][k]);
                const uint32_t u1 = maj(S0[j][p2][k], S0[j][p1][k], S0[j][pn][k]);
                const uint32_t v0 = xor3(S1[j][p2][k], S1[j][p1][k], S1[j][pn][k]);
                const uint32_t v1 = maj(S1[j][p2][k], S1[j][p1][k], S1[j][pn][k]);
                const uint32_t h1 = bitop3<0x14>(u1, v0, v1);
                const uint32_t h2 = bitop3<0x42>(u1, v0, v1);
                const uint32_t xx = bitop3<0x08>(u0, X[j][p1][k], h2);
                x[k] = bitop3<0xea>(u0, h1, xx);         // stage j output = row r-1-j
            }
        }
        if constexpr (NS == K) {
            const int ry = r - K;                        // final output row
            if (st && ry >= y0) *reinterpret_cast<Vec *>(out32 + st_off) = vec_make(x);
        }
        adv(st_off);
    };

    // Prologue: stage j's first needed output (row y0-K+1+j) comes at step 2j+2 and its
    // window fills in the two steps before, so step s runs stages 0 .. s/2 only.  The
    // band always has >= 2K steps, so the prologue (2K-2 steps) never overruns it.
    int r = r_first;
    unroll_seq(std::make_integer_sequence<int, 2 * K - 2>{}, [&](auto S) {
        constexpr int sidx = decltype(S)::value;
        step(std::integral_constant<int, sidx % 3>{}, std::integral_constant<int, sidx / 2 + 1>{},
             r + sidx);
    });
    r += 2 * K - 2;
    constexpr int P0 = (2 * K - 2) % 3;                 // ring phase of the first steady step
    using Kc = std::integral_constant<int, K>;
    for (; r + 3 <= r_end; r += 3) {
        step(std::integral_constant<int, P0>{}, Kc{}, r);
        step(std::integral_constant<int, (P0 + 1) % 3>{}, Kc{}, r + 1);
        step(std::integral_constant<int, (P0 + 2) % 3>{}, Kc{}, r + 2);
    }
    if (r < r_end) step(std::integral_constant<int, P0>{}, Kc{}, r);
    if (r + 1 < r_end) step(std::integral_constant<int, (P0 + 1) % 3>{}, Kc{}, r + 1);
}

// ------------------------- K1s: K turns per launch, skewed stage pipeline (the default)
// Same tiles, halo lanes and bit-sliced rule as k_step_multi; three changes:
//  * Skew.  Stage j consumes the row stage j-1 produced in the PREVIOUS step, so the K
//    stages of one step are independent dependency chains (K-wide ILP per wavefront)
//    instead of one serial chain of ~7K levels.  Stage j outputs row r_first + s - 1 - 2j
//    at step s; it fills its 3-row window at steps 3j, 3j+1 and computes from 3j+2 on.
//    All stages share ring phase s % 3.
//  * Wave-uniform bookkeeping.  The wavefront id goes through readfirstlane, so band,
//    tile, row offsets and loop control live in SGPRs and branches are scalar; loads are
//    unconditional (rows past the band wrap in-bounds and feed only unstored outputs).
//  * LDS-DMA prefetch.  Row s + PD is loaded at the end of step s, by global_load_lds,
//    into the LDS slot of row s - 1 (a per-wavefront ring of RQ = PD + 1 slots) and read
//    back with a counted vmcnt wait when stage 0 consumes it.  Register-destination
//    prefetches became loop-carried register copies that the compiler guarded with
//    vmcnt waits for every row in flight; LDS slots carry no registers across the loop.
//    The steady loop is unrolled by U = lcm(3, RQ) so slot offsets are immediates.
// Steps: prologue [0, 3K-3) with compile-time stage ranges, steady [3K-3, nr) unrolled by
// U, epilogue K-1 steps (stage j active while j > e).  nr = input rows, padded so the
// steady part is a multiple of U; rows past r_end feed only outputs >= y1 (not stored).
constexpr int cgcd(int a, int b) { return b == 0 ? a : cgcd(b, a % b); }

constexpr int kBufFlags = 0x00020000;                  // raw buffer, dword3 (CDNA)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void buf_store(const uint32_t (&o)[1], __amdgpu_buffer_rsrc_t r,
                                          uint32_t voff, uint32_t soff)
{
    __builtin_amdgcn_raw_buffer_store_b32(o[0], r, voff, soff, 0);
}
__device__ __forceinline__ void buf_store(const uint32_t (&o)[2], __amdgpu_buffer_rsrc_t r,
                                          uint32_t voff, uint32_t soff)
{
    const u32x2 d = {o[0], o[1]};
    __builtin_amdgcn_raw_buffer_store_b64(d, r, voff, soff, 0);
}
__device__ __forceinline__ void buf_store(const uint32_t (&o)[4], __amdgpu_buffer_rsrc_t r,
                                          uint32_t voff, uint32_t soff)
{
    const u32x4 d = {o[0], o[1], o[2], o[3]};
    __builtin_amdgcn_raw_buffer_store_b128(d, r, voff, soff, 0);
}

template <int ND> struct LaneDw;
template <> struct LaneDw<1> { using T = uint32_t; };
template <> struct LaneDw<2> { using T = uint2; };
template <> struct LaneDw<4> { using T = uint4; };
__device__ __forceinline__ uint32_t vec_make(const uint32_t (&c)[1]) { return c[0]; }

// ND = dwords per lane (1, 2 or 4: 32, 64 or 128 cells); tiles advance by 62 * ND dwords.
// IL: the lane's 32 * ND cells are stored interleaved -- dword r holds the cells whose
// offset in the lane's range is = r (mod ND), bit i <-> offset ND * i + r (the engine's
// interleaved board layout, il_lane_dwords == ND).  Then the west neighbours of dword r
// are dword r - 1 as is and the east neighbours dword r + 1 as is; only dword 0's west
// and dword ND-1's east need a 1-bit funnel shift (v_alignbit, half-rate on gfx950 like
// DPP: tools/calib/valu_issue.hip), i.e. 2 instead of 2 * ND shifts per lane-row.
// (ND == 1 makes both layouts the same.)
// BUF: row loads (LDS-DMA) and stores through buffer resources -- per-lane byte offset in
// one VGPR, the row (+ dword) offset in an SGPR (soffset): no
// 64-bit VALU address adds, ~5 VGPRs freed (num_records = the buffer size: < 2 GiB,
// multi_fits).  Halo lanes skip their stores by exec mask (2 % faster than dropping them
// with an out-of-range offset).
// ABL: timing ablations (tools only, wrong results): 1 = no row DMA, 2 = no LDS read-back
// (and no DMA wait), 4 = no output stores (kept live behind a runtime-false branch).
// W16 (ND = 2, BUF): one 16-B LDS-DMA per row from lanes 0..31 (word pairs) instead of two
// 4-B DMAs from all lanes.  Tiles start one word later (lane 0 holds an even word, so no
// pair straddles the row's wrap; the last tile stores word 0), and the slot holds the row's
// 64 words in order (read back as one ds_read_b64 per lane).
template <int K, int ND, int PD, int MINW, bool R7, bool IL = false, bool BUF = false,
          int ABL = 0, bool W16 = false>
__global__ __launch_bounds__(256, MINW) void k_step_skew(const uint64_t *__restrict__ in,
                                                   uint64_t *__restrict__ out, StepArgs a,
                                                   int ntx)
{
    static_assert(K >= 2, "one turn per launch is k_step_ring");
    static_assert(K <= 32 * ND, "the edge error must stay inside the halo lanes");
    static_assert(!W16 || (ND == 2 && BUF), "wide row DMA: 2 dwords per lane, buffer path");
    constexpr int STRIDE = 62 * ND;                     // stored dwords per tile
    constexpr int RQ = PD + 1;                          // prefetch ring slots
    constexpr int U = 3 * RQ / cgcd(3, RQ);             // steady-loop unroll
    constexpr int S0_ = 3 * K - 3;                      // first steady step
    using Vec = typename LaneDw<ND>::T;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    const int tx = wv % ntx;
    const int by = wv / ntx;
    const int y0 = a.row_lo + by * a.band;
    if (y0 >= a.row_hi) return;
    const int y1 = min(y0 + a.band, a.row_hi);          // stored outputs [y0, y1)
    int nr = max(y1 - y0, K) + 2 * K;                   // >= S0_ + 3
    nr = S0_ + (nr - S0_ + U - 1) / U * U;

    const int nd = 2 * a.nw;                            // dwords per row
    constexpr int SHIFT = W16 ? ND : 0;                 // W16: tiles start one word later
    const int t0 = tx * STRIDE + SHIFT;
    const int t1 = min(t0 + STRIDE, nd + SHIFT);
    const int last = (t1 - t0 + ND - 1) / ND + 1;       // right halo lane
    const bool st = lane >= 1 && lane < last;
    int w = t0 - ND + ND * lane;                        // lane's first dword (torus wrap)
    while (w < 0) w += nd;
    while (w >= nd) w -= nd;
    const uint32_t lane_b = (uint32_t)w * 4u;
    uint32_t lane_dma = 0;                              // W16: word pair of lanes 2L, 2L+1
    if constexpr (W16) {
        int pw = t0 - ND + 4 * (lane & 31);
        while (pw >= nd) pw -= nd;
        lane_dma = (uint32_t)pw * 4u;
    }
    // byte offsets fit 32 bits: the host launches this kernel only on buffers < 4 GiB
    const uint32_t pitch_b = (uint32_t)a.pitch * 8u;
    const int M = a.modrows;
    const uint32_t span = (uint32_t)M * pitch_b;
    auto rowoff = [&](int r) -> uint32_t {
        while (r < 0) r += M;
        while (r >= M) r -= M;
        return (uint32_t)r * pitch_b;
    };
    auto adv = [&](uint32_t &o) {
        o += pitch_b;
        o = o >= span ? o - span : o;
    };
    const char *inb = reinterpret_cast<const char *>(in);
    char *outb = reinterpret_cast<char *>(out);
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc((void *)in, (short)0, (int)span, kBufFlags);
    const __amdgpu_buffer_rsrc_t rout =
        __builtin_amdgcn_make_buffer_rsrc((void *)out, (short)0, (int)span, kBufFlags);
    // prefetch ring in LDS: each wavefront owns RQ row slots of 64 lanes x ND dwords,
    // filled by LDS-DMA (global_load_lds_dword, dword k of every lane into plane k)
    __shared__ uint32_t lds_rows[4][RQ][ND][64];
    uint32_t(*slots)[ND][64] = lds_rows[__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))];
    auto issue = [&](uint32_t off, auto Qc) {
        constexpr int q = decltype(Qc)::value;
        if constexpr ((ABL & 1) != 0) return;
        if constexpr (W16) {
            if (lane < 32)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_void *)&slots[q][0][0], 16,
                                                         lane_dma, off, 0, 0);
        } else if constexpr (BUF) {
            unroll_seq(std::make_integer_sequence<int, ND>{}, [&](auto Kc) {
                constexpr int k = decltype(Kc)::value;
                // (the immediate offset would move the LDS destination too: use soffset)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_void *)&slots[q][k][0], 4,
                                                         lane_b, off + 4 * k, 0, 0);
            });
        } else {
            const uint32_t *g = reinterpret_cast<const uint32_t *>((inb + off) + lane_b);
#pragma unroll
            for (int k = 0; k < ND; ++k)
                __builtin_amdgcn_global_load_lds(g + k, (lds_void *)&slots[q][k][0], 4, 0, 0);
        }
    };
    // row in slot q: wait until at most ND*(PD-1) vector-memory ops are outstanding -- the
    // ND*(PD-1) DMA dwords of the PD-1 later rows were issued after it (stores, when
    // present, only make the wait earlier), then read it back
    auto fetch = [&](auto Qc, uint32_t (&c)[ND]) {
        constexpr int q = decltype(Qc)::value;
        constexpr int n = (W16 ? 1 : ND) * (PD - 1);
        if constexpr ((ABL & 2) != 0) {
#pragma unroll
            for (int k = 0; k < ND; ++k) c[k] = lane_b * (q + k + 1);
            return;
        }
        __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8));
        if constexpr (W16) {
            const uint32_t *sp = &slots[q][0][0] + 2 * lane;
            c[0] = sp[0];
            c[1] = sp[1];
        } else {
#pragma unroll
            for (int k = 0; k < ND; ++k) c[k] = slots[q][k][lane];
        }
    };

    uint32_t S0[K][3][ND], S1[K][3][ND], X[K][3][ND], XS[K][ND];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int k = 0; k < ND; ++k) {
            XS[j][k] = 0;
#pragma unroll
            for (int p = 0; p < 3; ++p) S0[j][p][k] = S1[j][p][k] = X[j][p][k] = 0;
        }
    uint32_t ld_off = rowoff(y0 - K);                   // input row r_first = y0 - K
    unroll_seq(std::make_integer_sequence<int, PD>{}, [&](auto Qc) {
        issue(ld_off, Qc);
        adv(ld_off);
    });
    uint32_t st_off = 0;
    int ry = 0;                                          // row stage K-1 outputs this step

    // one stage: input row x enters stage j's window at phase P; if RULE, the window's
    // middle row advances one turn into `o`
    auto stage = [&](auto Jc, auto Pc, auto RULEc, const uint32_t (&x)[ND], uint32_t (&o)[ND]) {
        constexpr int j = decltype(Jc)::value;
        constexpr int P = decltype(Pc)::value;
        constexpr int pm = (P + 2) % 3, po = (P + 1) % 3;   // middle, oldest row
        const uint32_t L = dpp_from_lower_z(x[ND - 1]);
        const uint32_t R = dpp_from_upper_z(x[0]);
#pragma unroll
        for (int k = 0; k < ND; ++k) {
            uint32_t wl, er;
            if constexpr (IL) {
                wl = k == 0 ? __builtin_amdgcn_alignbit(x[ND - 1], L, 31) : x[k - 1];
                er = k == ND - 1 ? __builtin_amdgcn_alignbit(R, x[0], 1) : x[k + 1];
            } else {
                wl = __builtin_amdgcn_alignbit(x[k], k == 0 ? L : x[k - 1], 31);
                er = __builtin_amdgcn_alignbit(k == ND - 1 ? R : x[k + 1], x[k], 1);
            }
            S0[j][P][k] = xor3(wl, x[k], er);
            S1[j][P][k] = maj(wl, x[k], er);
            X[j][P][k] = x[k];
        }
        if constexpr (decltype(RULEc)::value) {
#pragma unroll
            for (int k = 0; k < ND; ++k) {
                if constexpr (R7)
                    o[k] = life_rule7(S0[j][po][k], S0[j][pm][k], S0[j][P][k], S1[j][po][k],
                                      S1[j][pm][k], S1[j][P][k], X[j][pm][k]);
                else
                    o[k] = life_rule8(S0[j][po][k], S0[j][pm][k], S0[j][P][k], S1[j][po][k],
                                      S1[j][pm][k], S1[j][P][k], X[j][pm][k]);
            }
        }
    };

    // step s (compile-time s mod U as SM): stages [JA, JB) active, stages < JR compute the
    // rule (JR <= JB); LD = stage 0 consumes slot s % RQ and row s + PD is loaded after it.
    // Stages run in descending order so stage j+1 reads XS[j+1] before stage j rewrites it.
    auto step = [&](auto SMc, auto JAc, auto JBc, auto JRc, auto LDc) {
        constexpr int SM = decltype(SMc)::value;
        constexpr int P = SM % 3;
        constexpr int JA = decltype(JAc)::value, JB = decltype(JBc)::value;
        constexpr int JR = decltype(JRc)::value;
        constexpr bool LD = decltype(LDc)::value;
        using Pc = std::integral_constant<int, P>;
        unroll_seq(std::make_integer_sequence<int, JB - JA>{}, [&](auto I) {
            constexpr int j = JB - 1 - decltype(I)::value;
            using RULE = std::integral_constant<bool, (j < JR)>;
            uint32_t x[ND];
            if constexpr (j == 0) {
                fetch(std::integral_constant<int, SM % RQ>{}, x);
            } else {
#pragma unroll
                for (int k = 0; k < ND; ++k) x[k] = XS[j][k];
            }
            if constexpr (j == K - 1) {
                uint32_t o[ND];
                stage(std::integral_constant<int, j>{}, Pc{}, RULE{}, x, o);
                if constexpr (RULE::value) {
                    if constexpr ((ABL & 4) != 0) {
                        if (a.cnt_hi == 0x7fffffff) buf_store(o, rout, lane_b, st_off);
                    } else if constexpr (BUF) {
                        if (st && ry >= y0 && ry < y1) buf_store(o, rout, lane_b, st_off);
                    } else if (st && ry >= y0 && ry < y1) {
                        *reinterpret_cast<Vec *>((outb + st_off) + lane_b) = vec_make(o);
                    }
                }
            } else {
                stage(std::integral_constant<int, j>{}, Pc{}, RULE{}, x, XS[j + 1]);
            }
        });
        if constexpr (LD) {                             // row s + PD into row s-1's slot
            issue(ld_off, std::integral_constant<int, (SM + PD) % RQ>{});
            adv(ld_off);
        }
        if constexpr (JR == K) {                         // stage K-1 produced row ry
            adv(st_off);
            ++ry;
        }
    };
    using T = std::true_type;
    using F = std::false_type;
    using Z = std::integral_constant<int, 0>;
    using Kc = std::integral_constant<int, K>;

    // prologue: steps 0 .. 3K-4
    unroll_seq(std::make_integer_sequence<int, S0_>{}, [&](auto Sc) {
        constexpr int s = decltype(Sc)::value;
        constexpr int JB = s / 3 + 1;
        constexpr int JR = s >= 2 ? (s - 2) / 3 + 1 : 0;
        step(std::integral_constant<int, s % U>{}, Z{}, std::integral_constant<int, JB>{},
             std::integral_constant<int, JR>{}, T{});
    });
    // steady state: every stage active; step s outputs row y0 + s - 3K + 1
    ry = y0 - 2;
    st_off = rowoff(ry);
    for (int s = S0_; s < nr; s += U) {
        unroll_seq(std::make_integer_sequence<int, U>{}, [&](auto Ic) {
            constexpr int i = decltype(Ic)::value;
            step(std::integral_constant<int, (S0_ + i) % U>{}, Z{}, Kc{}, Kc{}, T{});
        });
    }
    // epilogue: step nr + e runs stages e+1 .. K-1 (nr == S0_ mod U)
    unroll_seq(std::make_integer_sequence<int, K - 1>{}, [&](auto Ec) {
        constexpr int e = decltype(Ec)::value;
        step(std::integral_constant<int, (S0_ + e) % U>{}, std::integral_constant<int, e + 1>{},
             Kc{}, Kc{}, F{});
    });
    // the last PD prefetches (rows past the band) must land before the LDS is released
    __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));
}

// -------------------- K1w: K turns per launch, one band's stage pipeline split over a workgroup
// k_step_skew gives every wavefront a whole K-stage pipeline over its own band, so the
// machine is filled with many short bands, each paying the 2K halo rows and the pipeline
// fill again (the K^2 + K stage-rows per band), and each wave holds K x 12 VGPRs of stage
// state (4 waves/SIMD at K = 8).  Here the NW wavefronts of a workgroup share ONE band:
// wave w runs stages [J_w, J_w + G_w) of the same skewed pipeline (G_w = K/NW, the first
// K%NW waves one more) and hands its last stage's rows to wave w+1 through an LDS ring.
// For the same number of resident waves the bands are NW times taller, and a wave holds
// ~G_w x 12 VGPRs: more waves per SIMD, or K = 16 (half the HBM bytes per turn of K = 8).
//   * Hand-off.  Each wave boundary is a single-producer / single-consumer ring of kWgR
//     row slots in LDS with two counters: `produced` (rows written) and `consumed` (rows
//     read).  The producer waits for a free slot, writes the row, releases (lgkmcnt(0))
//     and bumps `produced`; the consumer waits for `produced`, reads the row and bumps
//     `consumed`.  Both remember the last value they saw, so in steady state most steps
//     read no counter at all, and waves drift up to kWgR rows apart without waiting.
//     A per-step s_barrier (lockstep) measured 22-37 % slower than no synchronisation at
//     all; the ring keeps only the true dependencies.  The graph is a chain (wave 0 never
//     waits upstream, the last wave never downstream), so it cannot deadlock.
//   * Timeline.  Wave w's local pipeline is k_step_skew's with G_w stages over the
//     nr - 2 J_w rows its first stage receives: prologue 3G-3 steps, steady loop (unroll
//     U, a guarded tail), epilogue G-1 steps.  Its first stage consumes input row q at
//     local step q; its last stage emits row q at local step q + 3G - 1.
//   * Memory.  Wave 0 alone streams input rows (16-B LDS-DMA from lanes 0..31 into its
//     RQ-slot ring, counted vmcnt wait: it issues no stores, so the count is exact); the
//     last wave alone stores output rows.  Tiles, halo lanes, interleaved layout, rule and
//     buffer addressing are k_step_skew's (IL, W16, BUF, R7).
template <int K, int NW>
struct WgSplit {
    static constexpr int G(int w) { return K / NW + (w < K % NW ? 1 : 0); }
    static constexpr int J(int w) { return w == 0 ? 0 : J(w - 1) + G(w - 1); }
};

// Ring slots are compile-time (immediate LDS offsets): the steady loop is unrolled by
// U = lcm(3, kWgRQ, kWgR) = 6.  Runtime slot indices (to deepen the rings to 12 DMA rows
// and 8 hand-off slots without a longer unroll) measured no faster and cost ~10 VGPRs
// (K = 16: 86, i.e. 5 waves/SIMD instead of 6).
constexpr int kWgPD = 5;                                // wave 0's rows in flight
constexpr int kWgRQ = kWgPD + 1;                        // its LDS-DMA ring slots
constexpr int kWgR = 6;                                 // hand-off ring slots per boundary
// A wait gives up after this many polls (~2^22 x 64 cycles, >0.1 s): a broken hand-off then
// ends the launch with a wrong board (caught by the parity tests) instead of hanging the GPU.
constexpr int kWgSpinLimit = 1 << 22;
constexpr int kWgLag = 3;                               // SYNC 2: consumer's initial lag (rows)

struct WgShared {
    uint32_t dma[kWgRQ][128];                           // wave 0's input rows (64 words each)
    uint32_t xfer[3][kWgR][128];                        // wave w -> w+1 rows (NW <= 4)
    uint32_t produced[4], consumed[4];                  // per boundary: rows written / read
};

__device__ __forceinline__ uint32_t lds_load_counter(const uint32_t *p)
{
    return (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void lds_store_counter(uint32_t *p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// SYNC: 0 = timing ablation only (no hand-off synchronisation: wrong results); 1 = counters
// with hardware release/acquire (s_waitcnt lgkmcnt(0) around every hand-off); 2 = counters
// ordered by the LDS itself (it executes a CU's requests in arrival order, and each wave's
// in issue order: a row written before its counter is visible to a reader that saw the
// counter; a slot read before its `consumed` store is read before the producer can see
// that store and overwrite it) with compiler-only fences, and a consumer that starts
// kWgLag rows behind its producer so the ring absorbs rate jitter both ways.  3 = 2 plus
// per-wave wait timing into a.counts (tools only: GOL_MULTI_VARIANT=kMultiWgDiag).
template <int K, int NW, int W, int SYNC>
__device__ __forceinline__ void wg_wave(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                        const StepArgs &a, WgShared &sh, int tx, int y0, int y1,
                                        int nr)
{
    constexpr int ND = 2;
    constexpr int G = WgSplit<K, NW>::G(W);
    constexpr int J = WgSplit<K, NW>::J(W);
    constexpr bool FIRST = W == 0, LAST = W == NW - 1;
    constexpr int RQ = kWgRQ, PD = kWgPD, R = kWgR;
    constexpr int U = 6;                                 // lcm(3, RQ, R): slots are immediates
    static_assert(U % 3 == 0 && U % RQ == 0 && U % R == 0, "steady unroll");
    constexpr int S0_ = 3 * G - 3;                       // local prologue steps
    constexpr int EMIT0 = 3 * G - 1;                     // first local step the last stage emits
    constexpr int STRIDE = 62 * ND, SHIFT = ND;
    static_assert(NW >= 2 && NW <= 4 && G >= 1, "2..4 waves, every wave a stage");
    const int lane = threadIdx.x & 63;
    const int nl = nr - 2 * J;                           // rows this wave's first stage takes

    const int nd = 2 * a.nw;
    const int t0 = tx * STRIDE + SHIFT;
    const int t1 = min(t0 + STRIDE, nd + SHIFT);
    const int last = (t1 - t0 + ND - 1) / ND + 1;        // right halo lane
    const bool st = lane >= 1 && lane < last;
    int w = t0 - ND + ND * lane;                         // lane's first dword (torus wrap)
    while (w >= nd) w -= nd;
    const uint32_t lane_b = (uint32_t)w * 4u;
    int pw = t0 - ND + 4 * (lane & 31);                  // W16 DMA: words 2L, 2L+1
    while (pw >= nd) pw -= nd;
    const uint32_t lane_dma = (uint32_t)pw * 4u;
    const uint32_t pitch_b = (uint32_t)a.pitch * 8u;
    const int M = a.modrows;
    const uint32_t span = (uint32_t)M * pitch_b;
    auto rowoff = [&](int r) -> uint32_t {
        while (r < 0) r += M;
        while (r >= M) r -= M;
        return (uint32_t)r * pitch_b;
    };
    auto adv = [&](uint32_t &o) {
        o += pitch_b;
        o = o >= span ? o - span : o;
    };
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc((void *)in, (short)0, (int)span, kBufFlags);
    const __amdgpu_buffer_rsrc_t rout =
        __builtin_amdgcn_make_buffer_rsrc((void *)out, (short)0, (int)span, kBufFlags);

    uint32_t ld_off = 0;
    auto issue = [&](auto Qc) {                          // wave 0: next input row -> slot Q
        constexpr int q = decltype(Qc)::value;
        if (lane < 32)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_void *)&sh.dma[q][0], 16,
                                                     lane_dma, ld_off, 0, 0);
        adv(ld_off);
    };
    // priorities graded down the chain: upstream waves outrank their consumers (equal
    // priorities left the followers waiting for the head's rows at ~93 % of their steps,
    // tools/wg_diag.py; graded: 65536^2 K=16 44.6 -> 38.2 us/turn)
    if constexpr (SYNC >= 2) __builtin_amdgcn_s_setprio(NW - 1 - W);
    uint32_t avail = 0;                                  // consumer: rows known to be written
    uint32_t room = R;                                   // producer: rows it may write
    constexpr bool DIAG = SYNC == 3;
    unsigned long long d_t0 = DIAG ? __builtin_amdgcn_s_memtime() : 0, d_fw = 0, d_ew = 0,
                       d_nf = 0, d_ne = 0, d_first = 0;
    // input row q of local step l == q (SM = l mod U): wave 0 from its DMA ring, the others
    // from the upstream hand-off ring
    auto lds_order = [] { __atomic_signal_fence(__ATOMIC_SEQ_CST); };   // compiler-only
    auto fetch = [&](auto SMc, int q, uint32_t (&c)[ND]) {
        constexpr int SM = decltype(SMc)::value;
        if constexpr (FIRST) {
            __builtin_amdgcn_s_waitcnt(((PD - 1) & 15) | (((PD - 1) >> 4) << 14) | (7 << 4) |
                                       (15 << 8));
            const uint32_t *sp = &sh.dma[SM % RQ][2 * lane];
            c[0] = sp[0];
            c[1] = sp[1];
        } else {
            if constexpr (SYNC != 0) {
                uint32_t need = (uint32_t)q + 1;
                if constexpr (SYNC >= 2)
                    if (q == 0) need = (uint32_t)min(kWgLag + 1, nl);   // start behind
                unsigned long long tw = 0;
                if (DIAG && avail < need) tw = __builtin_amdgcn_s_memtime();
                for (int spin = 0; avail < need && spin < kWgSpinLimit; ++spin) {
                    avail = lds_load_counter(&sh.produced[W - 1]);
                    if (avail < need) __builtin_amdgcn_s_sleep(1);
                }
                if (DIAG && tw) {
                    const unsigned long long dt = __builtin_amdgcn_s_memtime() - tw;
                    if (q == 0) d_first += dt;
                    else { d_fw += dt; ++d_nf; }
                }
                if constexpr (SYNC == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                else lds_order();
            }
            const uint32_t *sp = &sh.xfer[W - 1][SM % R][2 * lane];
            c[0] = sp[0];
            c[1] = sp[1];
            if constexpr (SYNC != 0) {
                // the row is read before the slot is handed back
                if constexpr (SYNC == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                else lds_order();
                if (lane == 0) lds_store_counter(&sh.consumed[W - 1], (uint32_t)q + 1);
            }
        }
    };
    auto emit = [&](auto SMc, int q, const uint32_t (&o)[ND]) {   // non-last waves: row q
        constexpr int SM = decltype(SMc)::value;
        constexpr int slot = ((SM - EMIT0) % R + R) % R;
        if constexpr (SYNC != 0) {
            unsigned long long tw = 0;
            if (DIAG && room <= (uint32_t)q) tw = __builtin_amdgcn_s_memtime();
            for (int spin = 0; room <= (uint32_t)q && spin < kWgSpinLimit; ++spin) {
                room = lds_load_counter(&sh.consumed[W]) + R;
                if (room <= (uint32_t)q) __builtin_amdgcn_s_sleep(1);
            }
            if (DIAG && tw) {
                d_ew += __builtin_amdgcn_s_memtime() - tw;
                ++d_ne;
            }
            if constexpr (SYNC == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
            else lds_order();
        }
        uint32_t *dp = &sh.xfer[W][slot][2 * lane];
        dp[0] = o[0];
        dp[1] = o[1];
        if constexpr (SYNC != 0) {
            if constexpr (SYNC == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            else lds_order();
            if (lane == 0) lds_store_counter(&sh.produced[W], (uint32_t)q + 1);
        }
    };

    uint32_t S0[G][3][ND], S1[G][3][ND], X[G][3][ND], XS[G][ND];
#pragma unroll
    for (int j = 0; j < G; ++j)
#pragma unroll
        for (int k = 0; k < ND; ++k) {
            XS[j][k] = 0;
#pragma unroll
            for (int p = 0; p < 3; ++p) S0[j][p][k] = S1[j][p][k] = X[j][p][k] = 0;
        }
    uint32_t st_off = 0;
    int ry = 0;                                          // last wave: row its last stage outputs

    auto stage = [&](auto Jc, auto Pc, auto RULEc, const uint32_t (&x)[ND], uint32_t (&o)[ND]) {
        constexpr int j = decltype(Jc)::value;
        constexpr int P = decltype(Pc)::value;
        constexpr int pm = (P + 2) % 3, po = (P + 1) % 3;
        const uint32_t L = dpp_from_lower_z(x[ND - 1]);
        const uint32_t Rt = dpp_from_upper_z(x[0]);
        const uint32_t wl0 = __builtin_amdgcn_alignbit(x[1], L, 31);
        const uint32_t er1 = __builtin_amdgcn_alignbit(Rt, x[0], 1);
        S0[j][P][0] = xor3(wl0, x[0], x[1]);
        S1[j][P][0] = maj(wl0, x[0], x[1]);
        S0[j][P][1] = xor3(x[0], x[1], er1);
        S1[j][P][1] = maj(x[0], x[1], er1);
        X[j][P][0] = x[0];
        X[j][P][1] = x[1];
        if constexpr (decltype(RULEc)::value) {
#pragma unroll
            for (int k = 0; k < ND; ++k)
                o[k] = life_rule7(S0[j][po][k], S0[j][pm][k], S0[j][P][k], S1[j][po][k],
                                  S1[j][pm][k], S1[j][P][k], X[j][pm][k]);
        }
    };

    // local step l (SM = l mod U): local stages [JA, JB) active, stages < JR apply the rule
    auto step = [&](auto SMc, auto JAc, auto JBc, auto JRc, auto LDc, int l) {
        constexpr int SM = decltype(SMc)::value;
        constexpr int P = SM % 3;
        constexpr int JA = decltype(JAc)::value, JB = decltype(JBc)::value;
        constexpr int JR = decltype(JRc)::value;
        using Pc = std::integral_constant<int, P>;
        unroll_seq(std::make_integer_sequence<int, JB - JA>{}, [&](auto I) {
            constexpr int j = JB - 1 - decltype(I)::value;
            using RULE = std::integral_constant<bool, (j < JR)>;
            uint32_t x[ND];
            if constexpr (j == 0) {
                fetch(SMc, l, x);
            } else {
#pragma unroll
                for (int k = 0; k < ND; ++k) x[k] = XS[j][k];
            }
            if constexpr (j == G - 1) {
                uint32_t o[ND];
                stage(std::integral_constant<int, j>{}, Pc{}, RULE{}, x, o);
                if constexpr (RULE::value) {
                    if constexpr (LAST) {
                        if (st && ry >= y0 && ry < y1) buf_store(o, rout, lane_b, st_off);
                    } else if (l >= EMIT0) {
                        // (the last stage's first two rule steps, S0_ and S0_ + 1, still
                        // fill its window: k_step_skew drops those rows by the row check)
                        emit(SMc, l - EMIT0, o);
                    }
                }
            } else {
                stage(std::integral_constant<int, j>{}, Pc{}, RULE{}, x, XS[j + 1]);
            }
        });
        if constexpr (FIRST && decltype(LDc)::value) issue(std::integral_constant<int, (SM + PD) % RQ>{});
        if constexpr (LAST && JR == G) {
            adv(st_off);
            ++ry;
        }
    };
    using Tt = std::true_type;
    using Ft = std::false_type;
    using Z = std::integral_constant<int, 0>;
    using Gc = std::integral_constant<int, G>;

    if constexpr (FIRST) {
        ld_off = rowoff(y0 - K);                         // input row r_first = y0 - K
        unroll_seq(std::make_integer_sequence<int, PD>{},
                   [&](auto Qc) { issue(std::integral_constant<int, decltype(Qc)::value>{}); });
    }
    unroll_seq(std::make_integer_sequence<int, S0_>{}, [&](auto Sc) {
        constexpr int s = decltype(Sc)::value;
        constexpr int JB = s / 3 + 1;
        constexpr int JR = s >= 2 ? (s - 2) / 3 + 1 : 0;
        step(std::integral_constant<int, s % U>{}, Z{}, std::integral_constant<int, JB>{},
             std::integral_constant<int, JR>{}, Tt{}, s);
    });
    // steady: the last stage of the last wave outputs row y0 + (global step) - 3K + 1
    if constexpr (LAST) {
        ry = y0 - 2;
        st_off = rowoff(ry);
    }
    int l = S0_;
    for (; l + U <= nl; l += U) {
        unroll_seq(std::make_integer_sequence<int, U>{}, [&](auto Ic) {
            constexpr int i = decltype(Ic)::value;
            step(std::integral_constant<int, (S0_ + i) % U>{}, Z{}, Gc{}, Gc{}, Tt{}, l + i);
        });
    }
    unroll_seq(std::make_integer_sequence<int, U - 1>{}, [&](auto Ic) {   // guarded tail
        constexpr int i = decltype(Ic)::value;
        if (l + i < nl)
            step(std::integral_constant<int, (S0_ + i) % U>{}, Z{}, Gc{}, Gc{}, Tt{}, l + i);
    });
    // epilogue: local step nl + e runs stages e+1 .. G-1; its ring phase is (nl + e) mod U,
    // a runtime value here -- dispatch it
    const int ph = nl % U;
    unroll_seq(std::make_integer_sequence<int, G - 1>{}, [&](auto Ec) {
        constexpr int e = decltype(Ec)::value;
        unroll_seq(std::make_integer_sequence<int, U>{}, [&](auto Pc2) {
            constexpr int p0 = decltype(Pc2)::value;
            if (ph == p0)
                step(std::integral_constant<int, (p0 + e) % U>{},
                     std::integral_constant<int, e + 1>{}, Gc{}, Gc{}, Ft{}, nl + e);
        });
    });
    if constexpr (FIRST) __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));   // DMAs landed
    if constexpr (DIAG) {
        if (lane == 0 && a.counts) {
            unsigned long long *d = a.counts + ((size_t)blockIdx.x * NW + W) * 8;
            d[0] = __builtin_amdgcn_s_memtime() - d_t0;
            d[1] = d_first;
            d[2] = d_fw;
            d[3] = d_nf;
            d[4] = d_ew;
            d[5] = d_ne;
            d[6] = (unsigned long long)nl;
            d[7] = d_t0;
        }
    }
}

template <int K, int NW, int SYNC = 2, int MINW = 1>
__global__ __launch_bounds__(64 * NW, MINW) void k_step_wg(const uint64_t *__restrict__ in,
                                                   uint64_t *__restrict__ out, StepArgs a,
                                                   int ntx)
{
    static_assert(K >= NW, "every wave needs a stage");
    static_assert(K <= 64, "the edge error must stay inside the halo lanes");
    __shared__ WgShared sh;
    const int pipe = blockIdx.x;                         // one band pipeline per workgroup
    const int tx = pipe % ntx;
    const int by = pipe / ntx;
    const int y0 = a.row_lo + by * a.band;
    if (y0 >= a.row_hi) return;                          // the whole workgroup
    const int y1 = min(y0 + a.band, a.row_hi);
    const int nr = max(y1 - y0, K) + 2 * K;              // input rows of the whole pipeline
    if (threadIdx.x < 4) sh.produced[threadIdx.x] = sh.consumed[threadIdx.x] = 0;
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    switch (wave) {
    case 0: wg_wave<K, NW, 0, SYNC>(in, out, a, sh, tx, y0, y1, nr); break;
    case 1: wg_wave<K, NW, 1, SYNC>(in, out, a, sh, tx, y0, y1, nr); break;
    case 2: if constexpr (NW > 2) wg_wave<K, NW, 2, SYNC>(in, out, a, sh, tx, y0, y1, nr); break;
    default: if constexpr (NW > 3) wg_wave<K, NW, 3, SYNC>(in, out, a, sh, tx, y0, y1, nr); break;
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

constexpr bool is_wg_variant(int v)
{
    return v == kMultiWg || v == kMultiWgNoBar || v == kMultiWgDiag;
}

constexpr bool is_il_variant(int v)
{
    return v == kMultiSkewIL || v == kMultiSkewILW16 || is_wg_variant(v);
}

int multi_max_turns(int variant) { return is_wg_variant(variant) ? 16 : 8; }

int multi_waves_per_band(int variant) { return is_wg_variant(variant) ? 4 : 1; }

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

// skew-kernel configurations (kMulti* variants): rows in flight, min waves per SIMD
// (MINW 4 = at most 128 VGPRs: 4 waves per SIMD; only 2 dwords per lane at K < 8 fits
// without spills -- K = 8 needs 132 VGPRs, and forcing 128 spilled and ran 17 % slower)
template <int Var, int K, int ND> struct SkewCfg;
template <int K, int ND> struct SkewCfg<kMultiSkew, K, ND> {
    static constexpr int PD = 8, MINW = (ND == 2 && K < 8) ? 4 : 1;
    static constexpr bool R7 = true;
};
template <int K, int ND> struct SkewCfg<kMultiSkewPD5, K, ND> {
    static constexpr int PD = 5, MINW = 1;
    static constexpr bool R7 = true;
};
template <int K, int ND> struct SkewCfg<kMultiSkewW1, K, ND> {
    static constexpr int PD = 8, MINW = 1;
    static constexpr bool R7 = true;
};
template <int K, int ND> struct SkewCfg<kMultiSkewRule8, K, ND> {
    static constexpr int PD = 8, MINW = ND == 2 ? 4 : 1;
    static constexpr bool R7 = false;
};
template <int K, int ND> struct SkewCfg<kMultiSkewD1, K, ND> {
    static constexpr int PD = 8, MINW = 1;
    static constexpr bool R7 = true;
};
// the interleaved build at K = 8 wants 129 VGPRs; capped at 128 (4 waves/SIMD) it spills 2
// outside the steady loop and ran 37.1 vs 40.2 us/turn at 3 waves/SIMD (65536^2, band 274)
template <int K, int ND> struct SkewCfg<kMultiSkewIL, K, ND> {
    static constexpr int PD = 8, MINW = 4;
    static constexpr bool R7 = true;
};
template <int K, int ND> struct SkewCfg<kMultiSkewILW16, K, ND> {
    static constexpr int PD = 8, MINW = 4;
    static constexpr bool R7 = true;
};



template <int ABL>
static void *abl_fn()
{
    return reinterpret_cast<void *>(&k_step_skew<8, 2, 8, 4, true, true, true, ABL>);
}

template <int K, int ND, int Var>
static void *skew_fn()
{
    using C = SkewCfg<Var, K, ND>;
    return reinterpret_cast<void *>(
        &k_step_skew<K, ND, C::PD, C::MINW, C::R7, is_il_variant(Var), is_il_variant(Var), 0,
                     Var == kMultiSkewILW16>);
}

// kernel for (turns, words per lane, variant); experimental variants exist for V = 1 and
// K in {6, 8} only (kMultiSkewD1: K in {4, 6, 8}) and fall back to kMultiSkew elsewhere
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

// kMultiWg: 4 waves per band, capped at 64 VGPRs (8 waves per SIMD) where that costs no
// spills (K <= 12: 65 -> 64; 65536^2 K = 12 38.2 vs 40.0 us/turn uncapped; K >= 13 needs
// 76+ and spilled 74-285 VGPRs capped); kMultiWgNoBar / kMultiWgDiag: timing ablation /
// wait diagnostics (tools only)
static void *wg_fn(int turns, int variant)
{
    switch (variant) {
    case kMultiWgNoBar: return turns == 8 || turns == 16 ? wg_fn_nw<4, 0>(turns) : nullptr;
    case kMultiWgDiag: return turns == 8 || turns == 16 ? wg_fn_nw<4, 3>(turns) : nullptr;
    default: return turns >= 13 ? wg_fn_nw<4, 2>(turns) : wg_fn_nw<4, 2, 8>(turns);
    }
}

template <int V>
static void *multi_fn(int turns, int variant)
{
    if (variant == kMultiSerial) {
        switch (turns) {
        case 2: return reinterpret_cast<void *>(&k_step_multi<2, V>);
        case 3: return reinterpret_cast<void *>(&k_step_multi<3, V>);
        case 4: return reinterpret_cast<void *>(&k_step_multi<4, V>);
        case 5: return reinterpret_cast<void *>(&k_step_multi<5, V>);
        case 6: return reinterpret_cast<void *>(&k_step_multi<6, V>);
        case 7: return reinterpret_cast<void *>(&k_step_multi<7, V>);
        case 8: return reinterpret_cast<void *>(&k_step_multi<8, V>);
        default: return nullptr;
        }
    }
    if (V == 1 && turns == 8 && variant >= kMultiAblate) {   // timing ablations (tools only)
        switch (variant - kMultiAblate) {
        case 1: return abl_fn<1>();
        case 2: return abl_fn<2>();
        case 3: return abl_fn<3>();
        case 4: return abl_fn<4>();
        case 7: return abl_fn<7>();
        default: return nullptr;
        }
    }
    if (V == 1 && variant == kMultiSkewILW16) {
        switch (turns) {
        case 2: return skew_fn<2, 2, kMultiSkewILW16>();
        case 3: return skew_fn<3, 2, kMultiSkewILW16>();
        case 4: return skew_fn<4, 2, kMultiSkewILW16>();
        case 5: return skew_fn<5, 2, kMultiSkewILW16>();
        case 6: return skew_fn<6, 2, kMultiSkewILW16>();
        case 7: return skew_fn<7, 2, kMultiSkewILW16>();
        case 8: return skew_fn<8, 2, kMultiSkewILW16>();
        default: return nullptr;
        }
    }
    if (V == 1 && variant == kMultiSkewIL) {
        switch (turns) {
        case 2: return skew_fn<2, 2, kMultiSkewIL>();
        case 3: return skew_fn<3, 2, kMultiSkewIL>();
        case 4: return skew_fn<4, 2, kMultiSkewIL>();
        case 5: return skew_fn<5, 2, kMultiSkewIL>();
        case 6: return skew_fn<6, 2, kMultiSkewIL>();
        case 7: return skew_fn<7, 2, kMultiSkewIL>();
        case 8: return skew_fn<8, 2, kMultiSkewIL>();
        default: return nullptr;
        }
    }
    if (V == 1 && variant == kMultiSkewD1) {
        switch (turns) {
        case 4: return skew_fn<4, 1, kMultiSkewD1>();
        case 6: return skew_fn<6, 1, kMultiSkewD1>();
        case 8: return skew_fn<8, 1, kMultiSkewD1>();
        default: return nullptr;
        }
    }
    if (V == 1 && (turns == 6 || turns == 8)) {
#define GOL_SKEW_VAR(VAR)                                                                     \
    case VAR: return turns == 6 ? skew_fn<6, 2, VAR>() : skew_fn<8, 2, VAR>();
        switch (variant) {
            GOL_SKEW_VAR(kMultiSkewPD5)
            GOL_SKEW_VAR(kMultiSkewW1)
            GOL_SKEW_VAR(kMultiSkewRule8)
        default: break;
        }
#undef GOL_SKEW_VAR
    }
    switch (turns) {
    case 2: return skew_fn<2, 2 * V, kMultiSkew>();
    case 3: return skew_fn<3, 2 * V, kMultiSkew>();
    case 4: return skew_fn<4, 2 * V, kMultiSkew>();
    case 5: return skew_fn<5, 2 * V, kMultiSkew>();
    case 6: return skew_fn<6, 2 * V, kMultiSkew>();
    case 7: return skew_fn<7, 2 * V, kMultiSkew>();
    case 8: return skew_fn<8, 2 * V, kMultiSkew>();
    default: return nullptr;
    }
}

// k_step_wg: one workgroup (4 waves) per (tile, band) pipeline; depths 2, 3 run on
// k_step_skew (same interleaved layout and tiles)
static hipError_t launch_wg(const StepArgs &a, int turns, hipStream_t s)
{
    const int ntx = (int)multi_tiles(a.width, 2);
    const int nbands = (a.row_hi - a.row_lo + a.band - 1) / a.band;
    const long long blocks = (long long)ntx * nbands;
    void *fn = wg_fn(turns, a.multi_variant);
    if (!fn) return hipErrorInvalidValue;
    const int threads = 64 * multi_waves_per_band(a.multi_variant);
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
    void *fn = multi_fn<V>(turns, var);
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
    int blocks = 0;
    void *fn = is_wg_variant(variant) ? (V == 1 ? wg_fn(turns, variant) : nullptr)
                                      : multi_fn<V>(turns, variant);
    if (!fn) return 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn,
                                                        64 * multi_waves_per_band(variant),
                                                        0) == hipSuccess
               ? blocks
               : 0;
}

int multi_blocks_per_cu(int turns, int words_per_lane, int variant)
{
    return words_per_lane == 1 ? multi_blocks_per_cu_v<1>(turns, variant)
                               : multi_blocks_per_cu_v<2>(turns, variant);
}

int pick_band_multi(int width, int rows, int lane_dwords, int turns, int capacity_waves)
{
    // Every wavefront of a launch does the same work, so a launch takes ~ rounds x
    // (per-wavefront time), rounds = ceil(waves / resident capacity): a grid that spills
    // a few waves into an extra round wastes most of that round (measured: the 65536^2
    // K=6 launch at 4.25 rounds).  Per-wavefront time ~ K x band + K (K + 1) stage-steps
    // (band rows, 2K halo rows, minus the skipped pipeline fill).  Pick the band that
    // minimises rounds x per-wave time, charging at least 2 rounds (a single round that
    // starts and ends every wavefront together measured slower: 65536^2 K=6 band 274 vs
    // 137, 60.6 vs 58.0 us/turn); ties go to the smaller band.
    const long long ntx = multi_tiles(width, lane_dwords);
    if (capacity_waves <= 0) return auto_band_multi(width, rows, lane_dwords);
    long long best_cost = -1;
    int best = 16;
    for (int band = 16; band <= 1024; ++band) {
        const long long nb = (rows + band - 1) / band;
        const long long waves = ntx * nb;
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
