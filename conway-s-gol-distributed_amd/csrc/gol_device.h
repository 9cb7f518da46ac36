// gol_device.h -- device-side building blocks shared by the gfx950 kernel files
// (gol_kernels.hip, gol_skew.hip, gol_wg.hip): DPP lane shifts, v_bitop3 truth tables,
// the B3/S23 rules, wave reductions, buffer-resource stores and compile-time unrolling.
// Internal: included by the kernel translation units only.
#pragma once
#include "gol_kernels.h"

#include <type_traits>
#include <utility>

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

typedef const __attribute__((address_space(4))) uint32_t *const_u32p;
typedef __attribute__((address_space(3))) void lds_void;

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

// (A/B builds: the cache policy of k_step_tile's final stores and first loads, the aux operand
// of the buffer instruction -- gfx950: 1 = sc0, 2 = nt, 16 = sc1; 0 in the product)
#ifndef GOL_TILE_STORE_AUX
#define GOL_TILE_STORE_AUX 0
#endif
#ifndef GOL_TILE_LOAD_AUX
#define GOL_TILE_LOAD_AUX 0
#endif
template <int AUX>
__device__ __forceinline__ void buf_store_aux(const uint32_t (&o)[2], __amdgpu_buffer_rsrc_t r,
                                              uint32_t voff)
{
    const u32x2 d = {o[0], o[1]};
    __builtin_amdgcn_raw_buffer_store_b64(d, r, voff, 0, AUX);
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
constexpr bool is_il_variant(int v)
{
    return v == kMultiSkewIL || v == kMultiSkewILW16 || is_wg_variant(v) || v == kMultiTile;
}

// kernel entry points built in their own translation units (parallel builds)
void *skew_kernel(int words_per_lane, int turns, int variant);   // gol_skew.hip
void *wg_kernel(int turns, int variant);                          // gol_wg.hip
void *wg_hx_kernel(int turns, bool pg);                           // gol_wg_hx.hip
void *wg_ser_kernel(int turns, bool pg);                          // gol_wg_ser.hip
void *wg_deep_kernel_a(int turns);                                // gol_wg_deep_a.hip (17..24)
void *wg_deep_kernel_b(int turns);                                // gol_wg_deep_b.hip (25..32)

}  // namespace golk
