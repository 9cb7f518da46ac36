// gol_wg.h -- K1w k_step_wg: one band's K-stage pipeline split over the 4 wavefronts of
// a workgroup.  Included by gol_wg.hip (band tiling) and gol_wg_hx.hip (helix tiling),
// which compile in parallel.
#pragma once
#include "gol_device.h"

namespace golk {

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
//     U) through the G-1 epilogue steps, padded to a multiple of U.  Its first stage consumes input row q at
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
constexpr int kWgPD = kWgDmaRows;                       // wave 0's rows in flight
constexpr int kWgRQ = kWgPD + 1;                        // its LDS-DMA ring slots
constexpr int kWgR = 6;                                 // hand-off ring slots per boundary
// A wait gives up after this many polls (~2^22 x 64 cycles, >0.1 s) instead of hanging the
// GPU, and records that in the engine's error word (StepArgs::err): the engine then fails its
// next synchronising call with GOL_EHIP rather than hand back the wrong board it computed.
// (GOL_WG_SPIN_LIMIT: the test build libgolamd_spin0.so sets 0, so every wait gives up.)
#ifndef GOL_WG_SPIN_LIMIT
#define GOL_WG_SPIN_LIMIT (1 << 22)
#endif
constexpr int kWgSpinLimit = GOL_WG_SPIN_LIMIT;

// a wait gave up: one store of the code from lane 0 into host-mapped memory (system scope,
// so the host sees it after the launch completes; a plain store, no PCIe atomics needed)
__device__ __forceinline__ void wg_report(unsigned *err, unsigned code)
{
    if (err && (threadIdx.x & 63) == 0)
        __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// SYNC 2: consumer's initial lag (rows).  Each wave boundary adds it to the pipeline fill;
// 1 measured as fast as 3 or slightly faster (16384^2 K = 16: 3.25 vs 3.27-3.33 us/turn; the
// 8-strip shape 5.62 vs 5.66-5.95; 65536^2 equal)
constexpr int kWgLag = 1;

template <int NW, bool PG = false>
struct WgShared {
    uint32_t dma[kWgRQ][128];                           // wave 0's input rows (64 words each)
    uint32_t xfer[NW - 1][kWgR][128];                   // wave w -> w+1 rows
    uint32_t produced[NW], consumed[NW];                // per boundary: rows written / read
    // PG: each wave's rows from below, 2 stages at a time (stage j in slot j % 2): 8 KB, not
    // 16, keeps 7 workgroups (of K = 16) per CU
    uint32_t nb[PG ? NW : 1][PG ? 2 : 1][2][128];
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
// HX (kMultiWgHx): helix tiling.  Tiles of 64 lanes (62 stored) waste the row's remainder:
// 16384 cells = 256 words -> 5 tiles of 64 lanes, 80 % of the lanes stored.  Instead, the
// row bands are laid end to end as one virtual lane sequence, band m contributing the
// nw + 4 words [nw-2, nw-1, 0, 1, ..., nw-1, 0, 1] (its row's torus wrap as 2 halo words
// on each side) and rows [y0 + m band, +band); the tiles cut that sequence every 62
// lanes.  A lane's vertical neighbours stay in the lane (it streams its own column of its
// own band), so a tile may span two bands: the lanes of each band address their own rows
// (per-lane row offsets for the DMA and the stores).  Where two bands meet, the 2 + 2 halo
// words absorb the wrong neighbours exactly as a tile's edge lanes do (K <= 64 bits of
// error); word pairs stay 16-B aligned (nw even, bands of even length), so the 16-B DMA
// still works.  Stored fraction 256/260 x 62/64 = 95 % at 16384^2, and any band height
// gives a full grid (the last band may be short: its lanes mask their stores).
// PG (kMultiWgPg, helix only): parallelogram bands.  With the trapezoid above, stage j of a
// band recomputes 2(K-1-j) rows of its neighbours' outputs (a 2K-row halo: 16384^2, K = 16,
// 68-row bands: 84 stage rows per 68 output rows).  Here stage j of band m outputs exactly
// its rows [y0 - K + 1 + j, y1 - K + 1 + j) -- the region slides down one row per stage, so
// the bands of one stage still partition the board -- and takes the last 2 of its band + 2
// input rows from stage j-1 of band m+1, whose FIRST 2 output rows they are.  So each
// stage publishes its first 2 output rows (e = 0, 1) to memory early in the pipeline and
// substitutes the 2 rows published by the band below for its own outputs e = band, band+1
// near the end (its computed ones would need rows it does not have).  Tiles run in reverse
// order (blockIdx 0 = the last tile), and a tile only waits for tiles after it, which were
// dispatched first and wait for nothing before publishing: no deadlock at any occupancy.
// The band of the last block (and every tile holding some of its lanes) keeps the
// trapezoid: it breaks the torus cycle and, in strips, ends at the halo.  Published rows
// and flags live in uncached memory (hipDeviceMallocUncached): visible across the XCDs'
// L2s without cache maintenance.  Flags carry the launch epoch, so they are never reset.
template <int K, int NW, int W, int SYNC, bool HX, bool PG = false, bool SER = false>
__device__ __forceinline__ void wg_wave(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                        const StepArgs &a, WgShared<NW, PG> &sh, int tx, int y0,
                                        int y1, int nr, bool trap, int ntx)
{
    constexpr int ND = 2;
    constexpr int G = WgSplit<K, NW>::G(W);
    constexpr int J = WgSplit<K, NW>::J(W);
    constexpr bool FIRST = W == 0, LAST = W == NW - 1;
    constexpr int RQ = kWgRQ, PD = kWgPD, R = kWgR;
    constexpr int U = kWgU;                              // lcm(3, RQ, R): slots are immediates
    static_assert(U % 3 == 0 && U % RQ == 0 && U % R == 0, "steady unroll");
    // SER: the wave's stages run in order within a step (stage j takes stage j-1's output of
    // the same step), so a stage starts 2 steps after the one before it instead of 3: the
    // pipeline fills and drains a third faster, and XS is no longer live across steps; the
    // skewed order keeps the G stages of a step independent (ILP).  STG = steps per stage.
    constexpr int STG = SER ? 2 : 3;
    constexpr int S0_ = STG * G - STG;                   // local prologue steps
    constexpr int EMIT0 = STG * G - STG + 2;             // first local step the last stage emits
    constexpr int STRIDE = 62 * ND, SHIFT = ND;
    static_assert(NW >= 2 && NW <= 8 && G >= 1, "2..8 waves, every wave a stage");
    const int lane = threadIdx.x & 63;
    const bool pgt = PG && !trap;                        // parallelogram tile
    // rows this wave's first stage takes, rows it hands on
    const int nl = pgt ? nr : nr - 2 * J;

    const uint32_t pitch_b = (uint32_t)a.pitch * 8u;
    const int M = a.modrows;
    const uint32_t span = (uint32_t)M * pitch_b;
    auto rowoff = [&](int r) -> uint32_t {
        while (r < 0) r += M;
        while (r >= M) r -= M;
        return (uint32_t)r * pitch_b;
    };
    bool st;
    uint32_t lane_b, lane_dma;
    int hy0 = 0, hh = 0, hy0d = 0;                       // HX: lane's band start / height, DMA lane's
    // PG: publishing lane / lane taking rows from below, their byte offsets in a published row,
    // the tiles that publish this tile's rows from below
    bool pub_ok = false, sub_ok = false;
    uint32_t pub_b = 0, cons_b = 0;
    int t_a = 0, t_b = -1;
    if constexpr (HX) {
        const int nwv = a.nw + 4;
        const int nblk = (a.row_hi - a.row_lo + a.band - 1) / a.band;
        // virtual lane v -> band m (clamped: lanes past the last band load real rows and
        // store nothing), column, stored?
        auto map = [&](int v, int &m, int &col) -> bool {
            m = v / nwv;
            const int p = v - m * nwv;
            col = p - 2;
            if (col < 0) col += a.nw;
            if (col >= a.nw) col -= a.nw;
            const bool useful = p >= 2 && p < a.nw + 2 && m < nblk;
            if (m >= nblk) m = nblk - 1;
            return useful;
        };
        int m, col, md, cold;
        const bool useful = map(62 * tx + lane, m, col);
        (void)map(62 * tx + 2 * (lane & 31), md, cold);
        st = lane >= 1 && lane < 63 && useful;
        lane_b = (uint32_t)col * 8u;
        lane_dma = (uint32_t)cold * 8u;
        hy0 = a.row_lo + m * a.band;
        hh = min(a.band, a.row_hi - hy0);
        hy0d = a.row_lo + md * a.band;
        if constexpr (PG) {
            const int u = 62 * tx + lane;                // virtual lane (interior ones publish)
            pub_ok = lane >= 1 && lane < 63 && u < nblk * nwv;
            pub_b = (uint32_t)u * 8u;
            // every lane of a band with a band below -- halo lanes too: they have no rows
            // past the band either, and feed the stored lanes' last rows
            sub_ok = m < nblk - 1;
            cons_b = (uint32_t)(62 * tx + 2 * (lane & 31) + nwv) * 8u;   // 16-B DMA pairs
            t_a = (62 * tx + nwv - 1) / 62;              // publisher of u: (u - 1) / 62
            t_b = min((62 * tx + nwv + 62) / 62, ntx - 1);
        }
    } else {
        const int nd = 2 * a.nw;
        const int t0 = tx * STRIDE + SHIFT;
        const int t1 = min(t0 + STRIDE, nd + SHIFT);
        const int last = (t1 - t0 + ND - 1) / ND + 1;    // right halo lane
        st = lane >= 1 && lane < last;
        int w = t0 - ND + ND * lane;                     // lane's first dword (torus wrap)
        while (w >= nd) w -= nd;
        lane_b = (uint32_t)w * 4u;
        int pw = t0 - ND + 4 * (lane & 31);              // W16 DMA: words 2L, 2L+1
        while (pw >= nd) pw -= nd;
        lane_dma = (uint32_t)pw * 4u;
    }
    auto adv = [&](uint32_t &o) {
        o += pitch_b;
        o = o >= span ? o - span : o;
    };
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc((void *)in, (short)0, (int)span, kBufFlags);
    const __amdgpu_buffer_rsrc_t rout =
        __builtin_amdgcn_make_buffer_rsrc((void *)out, (short)0, (int)span, kBufFlags);

    uint32_t ld_off = 0;                                 // HX: per lane, lane_dma included
    auto issue = [&](auto Qc) {                          // wave 0: next input row -> slot Q
        constexpr int q = decltype(Qc)::value;
        if (lane < 32) {
            if constexpr (HX)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_void *)&sh.dma[q][0], 16,
                                                         ld_off, 0, 0, 0);
            else
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_void *)&sh.dma[q][0], 16,
                                                         lane_dma, ld_off, 0, 0);
        }
        adv(ld_off);
    };
    // priorities graded down the chain: upstream waves outrank their consumers (equal
    // priorities left the followers waiting for the head's rows at ~93 % of their steps,
    // tools/wg_diag.py; graded: 65536^2 K=16 44.6 -> 38.2 us/turn)
    if constexpr (SYNC >= 2) {
        const unsigned pr = NW == 4 && a.wg_prio ? (a.wg_prio >> (2 * W)) & 3u
                                                 : (unsigned)((NW - 1 - W) * 3 / (NW - 1));
        switch (pr) {                                    // (s_setprio takes an immediate)
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
        }
    }
    uint32_t avail = 0;                                  // consumer: rows known to be written
    uint32_t room = R;                                   // producer: rows it may write
    unsigned gave_up = 0;                                // kDevErr* of a wait that gave up
                                                         //   (wave-uniform: reported at the end)
    constexpr bool DIAG = SYNC == 3;
    const unsigned long long d_r0 = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
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
                // rows past the upstream's last (the padded steps below) are not waited for
                uint32_t need = (uint32_t)min(q + 1, nl);
                if constexpr (SYNC >= 2)
                    if (q == 0) need = (uint32_t)min(kWgLag + 1, nl);   // start behind
                unsigned long long tw = 0;
                if (DIAG && avail < need) tw = __builtin_amdgcn_s_memtime();
                for (int spin = 0; avail < need && spin < kWgSpinLimit; ++spin) {
                    avail = lds_load_counter(&sh.produced[W - 1]);
                    if (avail < need) __builtin_amdgcn_s_sleep(1);
                }
                if (avail < need) gave_up = kDevErrHandoff;
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
    const int nemit = pgt ? nl : nl - 2 * G;             // rows the downstream wave takes
    auto emit = [&](auto SMc, int q, const uint32_t (&o)[ND]) {   // non-last waves: row q
        constexpr int SM = decltype(SMc)::value;
        constexpr int slot = ((SM - EMIT0) % R + R) % R;
        if (q >= nemit) return;                          // a padded step's row
        if constexpr (SYNC != 0) {
            unsigned long long tw = 0;
            if (DIAG && room <= (uint32_t)q) tw = __builtin_amdgcn_s_memtime();
            for (int spin = 0; room <= (uint32_t)q && spin < kWgSpinLimit; ++spin) {
                room = lds_load_counter(&sh.consumed[W]) + R;
                if (room <= (uint32_t)q) __builtin_amdgcn_s_sleep(1);
            }
            if (room <= (uint32_t)q) gave_up = kDevErrHandoff;
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
    uint32_t st_off = 0;                                 // HX: per lane, lane_b included
    int ry = 0;                                          // last wave: row its last stage outputs
                                                         //   (HX: relative to the lane's band)

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

    // PG: stage jl's output e = l - 3 jl - 2 (its first rule step is 3 jl + 2).  Its outputs
    // e = 0, 1 are published (steps 3 jl + 2, 3 jl + 3: prologue or the peeled first steady
    // iteration, compile-time); its outputs e = band, band + 1 are the rows of the band below
    // (steps band + 3 jl + 2, + 3: the epilogue, compile-time -- the host runs PG only with
    // band + 2 = S0_ mod U, so the steady loop ends exactly at step band + 2).  The global
    // last stage does neither: its rows are the launch's output.
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.xrows, (short)0, PG ? (int)(2u * kPgStages * a.xlanes * 8u) : 0, kBufFlags);
    auto rowb = [&](int jg, int r) -> uint32_t { return (uint32_t)(2 * jg + r) * a.xlanes * 8u; };
    constexpr int NS = (J + G <= K - 1) ? G : G - 1;     // PG: stages that publish / take
    constexpr int XPUB = 1 << 16;                        // step flags: publish e = 0, 1;
    // bits 0..7 / 8..15: stage j's output this step is row 0 / 1 from below
    auto publish = [&](auto Jc, int l, const uint32_t (&o)[ND]) {
        constexpr int jl = decltype(Jc)::value;
        if constexpr (PG && jl < NS) {
            const int e = l - STG * jl - 2;              // a constant in the steps that publish
            if ((e == 0 || e == 1) && pub_ok) buf_store(o, rx, pub_b, rowb(J + jl, e));
        }
    };
    // once per wave, after its last publication store (stage G-1's e = 1, step 3G): the flags
    auto publish_flags = [&]() {
        if constexpr (PG && NS > 0) {
            // Ordering without cache maintenance: rows and flags live in uncached memory, so
            // a row store is visible to every XCD once it has completed.  The wait completes
            // the row stores before a flag store issues; the flag store's release order (at
            // workgroup scope: no L2 write-back -- an agent-scope release would write back the
            // XCD's whole L2, which holds this launch's board output) keeps the compiler from
            // moving a row store below it.  (Compiler-only fences around the wait cost K <= 12
            // one VGPR: 65 > 64, one wave per SIMD less.)
            __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));   // the stores are done
            if (lane == 0)
                for (int jl = 0; jl < NS; ++jl)
                    __hip_atomic_store(&a.xflags[tx * kPgStages + J + jl], a.epoch,
                                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    // stage jl's 2 rows from below into LDS slot jl % 2 (16-B DMA from lanes 0..31)
    auto nb_load = [&](int jl) {
#if defined(__HIP_DEVICE_COMPILE__)
        // (device pass only: clang's host pass rejects the second kernel instantiating this
        // wave body -- a deferred-diagnostic quirk -- and the host never runs it)
        if constexpr (PG)
            if (lane < 32)
                for (int r = 0; r < 2; ++r)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        rx, (lds_void *)&sh.nb[W][jl & 1][r][0], 16, cons_b, rowb(J + jl, r), 0, 0);
#endif
    };
    // once per wave, a few steps before the first substitution: wait for the tiles below and
    // pull the rows of the first 2 stages into LDS (the epilogue loads the others)
    auto take_rows = [&]() {
        if constexpr (PG && NS > 0) {
            for (int jl = 0; jl < NS; ++jl)
                for (int t = t_a; t <= t_b; ++t) {
                    unsigned *f = &a.xflags[t * kPgStages + J + jl];
                    bool seen = false;
                    for (int spin = 0; !seen && spin < kWgSpinLimit; ++spin) {
                        const unsigned v = (unsigned)__builtin_amdgcn_readfirstlane((int)
                            __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                        seen = v == a.epoch;
                        if (!seen) __builtin_amdgcn_s_sleep(1);
                    }
                    if (!seen) gave_up = kDevErrPgFlag;
                }
            // the row loads stay below the flag checks (the loop exits on the loaded value, so
            // the hardware issues them after the flags arrived)
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            for (int jl = 0; jl < NS && jl < 2; ++jl) nb_load(jl);
            __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));   // rows landed
        }
    };

    // local step l (SM = l mod U): local stages [JA, JB) active, stages < JR apply the rule;
    // XF: PG flags (XPUB, substitution masks)
    auto step = [&](auto SMc, auto JAc, auto JBc, auto JRc, auto LDc, int l, auto XFc) {
        constexpr int SM = decltype(SMc)::value;
        constexpr int P = SM % 3;
        constexpr int JA = decltype(JAc)::value, JB = decltype(JBc)::value;
        constexpr int JR = decltype(JRc)::value;
        constexpr int XF = decltype(XFc)::value;
        using Pc = std::integral_constant<int, P>;
        unroll_seq(std::make_integer_sequence<int, JB - JA>{}, [&](auto I) {
            constexpr int j = SER ? JA + decltype(I)::value : JB - 1 - decltype(I)::value;
            using RULE = std::integral_constant<bool, (j < JR)>;
            constexpr int SUBR = (XF >> j) & 1 ? 0 : (XF >> (8 + j)) & 1 ? 1 : -1;
            uint32_t x[ND];
            if constexpr (SUBR < 0) {
                if constexpr (j == 0) {
                    fetch(SMc, l, x);
                } else {
#pragma unroll
                    for (int k = 0; k < ND; ++k) x[k] = XS[j][k];
                }
            }
            if constexpr (j == G - 1) {
                uint32_t o[ND];
                if constexpr (SUBR >= 0) {
                    if (pgt) {                           // (trapezoid tiles: past their end)
                        o[0] = sh.nb[W][j & 1][SUBR][2 * lane];
                        o[1] = sh.nb[W][j & 1][SUBR][2 * lane + 1];
                    } else {
                        o[0] = o[1] = 0;
                    }
                } else {
                    stage(std::integral_constant<int, j>{}, Pc{}, RULE{}, x, o);
                    if constexpr (RULE::value && (XF & XPUB) != 0)
                        publish(std::integral_constant<int, j>{}, l, o);
                }
                if constexpr (RULE::value) {
                    if constexpr (LAST) {
                        if constexpr (HX) {
                            if (st && ry >= 0 && ry < hh) buf_store(o, rout, st_off, 0);
                        } else {
                            if (st && ry >= y0 && ry < y1) buf_store(o, rout, lane_b, st_off);
                        }
                    } else if (l >= EMIT0) {
                        // (the last stage's first two rule steps, S0_ and S0_ + 1, still
                        // fill its window: k_step_skew drops those rows by the row check)
                        emit(SMc, l - EMIT0, o);
                    }
                }
            } else if constexpr (SUBR >= 0) {
                if (pgt) {
                    XS[j + 1][0] = sh.nb[W][j & 1][SUBR][2 * lane];
                    XS[j + 1][1] = sh.nb[W][j & 1][SUBR][2 * lane + 1];
                }
            } else {
                stage(std::integral_constant<int, j>{}, Pc{}, RULE{}, x, XS[j + 1]);
                if constexpr (RULE::value && (XF & XPUB) != 0)
                    publish(std::integral_constant<int, j>{}, l, XS[j + 1]);
            }
        });
        if constexpr (FIRST && decltype(LDc)::value) issue(std::integral_constant<int, (SM + PD) % RQ>{});
        if constexpr (LAST && JR == G) {
            adv(st_off);
            ++ry;
        }
        if constexpr (PG && (XF & XPUB) != 0)
            if (l == STG * (G - 1) + 3) publish_flags();
    };
    using Tt = std::true_type;
    using Ft = std::false_type;
    using Z = std::integral_constant<int, 0>;
    using Gc = std::integral_constant<int, G>;
    using XP = std::integral_constant<int, PG ? XPUB : 0>;
    using X0 = std::integral_constant<int, 0>;

    if constexpr (FIRST) {
        if constexpr (HX) ld_off = lane_dma + rowoff(hy0d - K);
        else ld_off = rowoff(y0 - K);                    // input row r_first = y0 - K
        unroll_seq(std::make_integer_sequence<int, PD>{},
                   [&](auto Qc) { issue(std::integral_constant<int, decltype(Qc)::value>{}); });
    }
    unroll_seq(std::make_integer_sequence<int, S0_>{}, [&](auto Sc) {
        constexpr int s = decltype(Sc)::value;
        constexpr int JB = s / STG + 1;
        constexpr int JR = s >= 2 ? (s - 2) / STG + 1 : 0;
        step(std::integral_constant<int, s % U>{}, Z{}, std::integral_constant<int, JB>{},
             std::integral_constant<int, JR>{}, Tt{}, s, XP{});
    });
    // steady: the last stage of the last wave outputs row y0 + (global step) - 3K + 1
    if constexpr (LAST) {
        if constexpr (HX) {
            ry = -2;
            st_off = lane_b + rowoff(hy0 - 2);
        } else {
            ry = y0 - 2;
            st_off = rowoff(ry);
        }
    }
    // The steady loop runs every remaining local step, S0_ .. nl + G - 2, padded up to a
    // multiple of U: the epilogue's steps (local step nl + e needs only stages e+1 .. G-1)
    // run all stages, the idle ones on rows past the band -- fetch does not wait for those
    // rows, emit drops them, the last wave's row check masks them, wave 0's DMA reads real
    // rows below the band -- and the rows they spoil are all past the last valid output of
    // each stage.  Every step's ring phase is a compile-time constant and the loop has one
    // exit: a guarded tail plus an epilogue dispatched on the runtime phase nl mod U kept
    // all three window slots of every stage live across the loop (K = 16: 92 instead of 74
    // VGPRs, 5 instead of 6 waves/SIMD; K = 12: 71 vs 63, 7 vs 8).
    // PG: the first steady iteration is peeled (it holds the last publications and the flag
    // step 3G).  A parallelogram tile's loop then ends at step band + 2 (a multiple of U
    // past S0_, by the host's choice of band), with the wave's rows from below taken in the
    // iteration holding step band - 3, and the epilogue's step ep (local step band + 2 + ep)
    // substitutes stage ep / 3's output row ep % 3 (ep % 3 < 2) and runs the stages above
    // it.  A trapezoid tile (last band) runs the padded loop without substitutions.
    int l0 = S0_;
    if constexpr (PG) {
        unroll_seq(std::make_integer_sequence<int, U>{}, [&](auto Ic) {
            constexpr int i = decltype(Ic)::value;
            step(std::integral_constant<int, (S0_ + i) % U>{}, Z{}, Gc{}, Gc{}, Tt{}, S0_ + i,
                 XP{});
        });
        l0 = S0_ + U;
    }
    if constexpr (PG) {
        // one loop + epilogue for both tile kinds (two alternative loops in one kernel cost
        // 129 VGPRs against 79 and 75 apart).  A trapezoid tile ends its loop once stage 0
        // is done (L >= nl) and skips the substitutions: the epilogue step that would
        // substitute stage js comes after its last needed output there.
        const int L = pgt ? a.band + 2 : S0_ + U + (max(nl - S0_ - U, 0) + U - 1) / U * U;
        const int pf = pgt ? a.band - 3 : -1;
        for (int l = l0; l < L; l += U) {
            if (pf >= l && pf < l + U) take_rows();
            unroll_seq(std::make_integer_sequence<int, U>{}, [&](auto Ic) {
                constexpr int i = decltype(Ic)::value;
                step(std::integral_constant<int, (S0_ + i) % U>{}, Z{}, Gc{}, Gc{}, Tt{}, l + i,
                     X0{});
            });
        }
        if (pgt && pf < l0) take_rows();
        constexpr int GS = LAST ? G - 1 : G;             // stages that substitute
        unroll_seq(std::make_integer_sequence<int, STG * G - STG + 2>{}, [&](auto Ec) {
            constexpr int ep = decltype(Ec)::value;
            constexpr int js = ep / STG, r = ep % STG;
            constexpr int XF = (js < GS && r < 2) ? (1 << (js + 8 * r)) : 0;
            // stage js >= 2: its rows were loaded 4 steps ago into the slot stage js - 2 freed
            if constexpr (r == 0 && js >= 2 && js < NS)
                __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));
            step(std::integral_constant<int, (S0_ + ep) % U>{},
                 std::integral_constant<int, SER ? ep / 2 : (ep + 1) / 3>{}, Gc{}, Gc{}, Ft{},
                 L + ep,
                 std::integral_constant<int, XF>{});
            if constexpr (r == STG - 1 && js + 2 < NS)
                if (pgt) nb_load(js + 2);
        });
    } else {
        const int l_end = SER ? nl : nl + G - 1;
        for (int l = l0; l < l_end; l += U) {
            unroll_seq(std::make_integer_sequence<int, U>{}, [&](auto Ic) {
                constexpr int i = decltype(Ic)::value;
                step(std::integral_constant<int, (S0_ + i) % U>{}, Z{}, Gc{}, Gc{}, Tt{}, l + i,
                     X0{});
            });
        }
    }
    if constexpr (FIRST) __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));   // DMAs landed
    if (gave_up) wg_report(a.err, gave_up);
    if constexpr (DIAG) {
        if (lane == 0 && a.counts) {
            unsigned long long *d = a.counts + ((size_t)blockIdx.x * NW + W) * 10;
            d[8] = d_r0;                                 // 100 MHz clock: comparable across XCDs
            d[9] = __builtin_amdgcn_s_memrealtime();
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

template <int K, int NW, int SYNC = 2, int MINW = 1, bool HX = false, bool PG = false,
          bool SER = false>
__global__ __launch_bounds__(64 * NW, MINW) void k_step_wg(const uint64_t *__restrict__ in,
                                                   uint64_t *__restrict__ out, StepArgs a,
                                                   int ntx)
{
    static_assert(K >= NW, "every wave needs a stage");
    static_assert(K <= 64, "the edge error must stay inside the halo lanes");
    static_assert(!PG || (HX && K <= kPgStages && K <= 4 * NW), "PG: helix, <= 4 stages a wave");
    __shared__ WgShared<NW, PG> sh;
    const int pipe = blockIdx.x;                         // one band pipeline per workgroup
    // HX: one helix tile per workgroup (ntx = the tile count), every lane its own band;
    // PG: the last tile first
    const int tx = HX ? (PG ? ntx - 1 - pipe : pipe) : pipe % ntx;
    const int by = HX ? 0 : pipe / ntx;
    const int y0 = a.row_lo + by * a.band;
    if (HX ? pipe >= ntx : y0 >= a.row_hi) return;       // the whole workgroup
    const int y1 = min(y0 + a.band, a.row_hi);
    // PG: tiles holding lanes of the last band run the trapezoid (band + 2K input rows)
    bool trap = true;
    if constexpr (PG) {
        const int nblk = (a.row_hi - a.row_lo + a.band - 1) / a.band;
        trap = (62 * tx + 63) / (a.nw + 4) >= nblk - 1;
    }
    const int nr = trap ? max(y1 - y0, K) + 2 * K : a.band + 2;   // input rows of the pipeline
    if (threadIdx.x < NW) sh.produced[threadIdx.x] = sh.consumed[threadIdx.x] = 0;
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    switch (wave) {
    case 0: wg_wave<K, NW, 0, SYNC, HX, PG, SER>(in, out, a, sh, tx, y0, y1, nr, trap, ntx); break;
    case 1: wg_wave<K, NW, 1, SYNC, HX, PG, SER>(in, out, a, sh, tx, y0, y1, nr, trap, ntx); break;
    case 2: if constexpr (NW > 2) wg_wave<K, NW, 2, SYNC, HX, PG, SER>(in, out, a, sh, tx, y0, y1, nr, trap, ntx); break;
    case 3: if constexpr (NW > 3) wg_wave<K, NW, 3, SYNC, HX, PG, SER>(in, out, a, sh, tx, y0, y1, nr, trap, ntx); break;
    case 4: if constexpr (NW > 4) wg_wave<K, NW, 4, SYNC, HX, PG, SER>(in, out, a, sh, tx, y0, y1, nr, trap, ntx); break;
    case 5: if constexpr (NW > 5) wg_wave<K, NW, 5, SYNC, HX, PG, SER>(in, out, a, sh, tx, y0, y1, nr, trap, ntx); break;
    case 6: if constexpr (NW > 6) wg_wave<K, NW, 6, SYNC, HX, PG, SER>(in, out, a, sh, tx, y0, y1, nr, trap, ntx); break;
    default: if constexpr (NW > 7) wg_wave<K, NW, 7, SYNC, HX, PG, SER>(in, out, a, sh, tx, y0, y1, nr, trap, ntx); break;
    }
}

}  // namespace golk
