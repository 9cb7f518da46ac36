// gol_skew.hip -- the temporal-blocking kernels with one band pipeline per wavefront:
// K1m k_step_multi (serial stages) and K1s k_step_skew (skewed stages, the shipped
// K <= 12 kernel), their A/B variants and the instantiation table the launchers use.
// Split from gol_kernels.hip so the kernel families compile in parallel.
#include "gol_device.h"

namespace golk {

#if GOL_TOOLS   // K1m: superseded by K1s, tools build only
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

#endif  // GOL_TOOLS

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

// skew-kernel configurations (kMulti* variants): rows in flight, min waves per SIMD
// (MINW 4 = at most 128 VGPRs: 4 waves per SIMD; only 2 dwords per lane at K < 8 fits
// without spills -- K = 8 needs 132 VGPRs, and forcing 128 spilled and ran 17 % slower)
template <int Var, int K, int ND> struct SkewCfg;
#if GOL_TOOLS   // superseded k_step_skew variants (A/B history in DESIGN.md): tools build only
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
#endif  // GOL_TOOLS
// K = 9..12 (deeper launches, fewer of them): 3 waves/SIMD up to K = 10, 2 beyond
template <int K, int ND> struct SkewCfg<kMultiSkewILW16, K, ND> {
    static constexpr int PD = 8, MINW = K <= 8 ? 4 : (K <= 10 ? 3 : 2);
    static constexpr bool R7 = true;
};



template <int K, int ND, int Var>
static void *skew_fn()
{
    using C = SkewCfg<Var, K, ND>;
    return reinterpret_cast<void *>(
        &k_step_skew<K, ND, C::PD, C::MINW, C::R7, is_il_variant(Var), is_il_variant(Var), 0,
                     Var == kMultiSkewILW16>);
}

// the shipped k_step_skew: interleaved layout, 16-B row DMA, one word per lane, K = 2..12
static void *ilw16_fn(int turns)
{
    switch (turns) {
    case 2: return skew_fn<2, 2, kMultiSkewILW16>();
    case 3: return skew_fn<3, 2, kMultiSkewILW16>();
    case 4: return skew_fn<4, 2, kMultiSkewILW16>();
    case 5: return skew_fn<5, 2, kMultiSkewILW16>();
    case 6: return skew_fn<6, 2, kMultiSkewILW16>();
    case 7: return skew_fn<7, 2, kMultiSkewILW16>();
    case 8: return skew_fn<8, 2, kMultiSkewILW16>();
    case 9: return skew_fn<9, 2, kMultiSkewILW16>();
    case 10: return skew_fn<10, 2, kMultiSkewILW16>();
    case 11: return skew_fn<11, 2, kMultiSkewILW16>();
    case 12: return skew_fn<12, 2, kMultiSkewILW16>();
    default: return nullptr;
    }
}

#if GOL_TOOLS
template <int ABL>
static void *abl_fn()
{
    return reinterpret_cast<void *>(&k_step_skew<8, 2, 8, 4, true, true, true, ABL>);
}

// tools build: every variant for (turns, words per lane); experimental variants exist for
// V = 1 and K in {6, 8} only (kMultiSkewD1: K in {4, 6, 8}) and fall back to kMultiSkew
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
    if (V == 1 && turns == 8 && variant >= kMultiAblate) {   // timing ablations
        switch (variant - kMultiAblate) {
        case 1: return abl_fn<1>();
        case 2: return abl_fn<2>();
        case 3: return abl_fn<3>();
        case 4: return abl_fn<4>();
        case 7: return abl_fn<7>();
        default: return nullptr;
        }
    }
    if (V == 1 && variant == kMultiSkewILW16) return ilw16_fn(turns);
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

void *skew_kernel(int words_per_lane, int turns, int variant)
{
    return words_per_lane == 1 ? multi_fn<1>(turns, variant) : multi_fn<2>(turns, variant);
}
#else
void *skew_kernel(int words_per_lane, int turns, int variant)
{
    return words_per_lane == 1 && variant == kMultiSkewILW16 ? ilw16_fn(turns) : nullptr;
}
#endif  // GOL_TOOLS

}  // namespace golk
