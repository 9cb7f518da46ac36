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
#if GOL_TOOLS
#include "gol_tile_turn.h"   // (ORD 8 / 9's generated inline-asm turns: tools build only)
#else
namespace golk {
// (declared only: ORD 8 / 9 are instantiated in the tools build alone)
template <int SEG, int V>
__device__ __forceinline__ void tile_turn_asm(uint32_t (&v)[SEG][2], uint32_t (&ad)[4], uint32_t ps,
                                              uint32_t ba);
}  // namespace golk
#endif

#include <type_traits>

#ifndef GOL_TILE_PAIRS_MAX   // (experiments: the longest segment that runs turns in pairs)
#define GOL_TILE_PAIRS_MAX 12
#endif
// West funnel shift by lane-mask carry (one word per lane): wl = (o << 1) | (west lane's o >>
// 31) as o + o + carry, the carry-in being the odd dwords' sign bits as a lane mask (one VOPC
// compare) shifted up one lane on the scalar unit, instead of a DPP move and a v_alignbit.
// It issues no faster (the isolated stream: 69.4-73.5 SIMD cycles per 4096 cell-updates
// against 67.8-70.8 for DPP + v_alignbit, tools/calib/stencil_issue.hip) but it drops the
// DPP's data hazard (s_nop) from each row's dependency chain, which pays where the turn is
// latency-bound: SEG 6 at 16384^2 3.02 against 3.22 us per turn, SEG 12 on the 8448-row
// strip 5.63 against 6.06, 33024-row strip 19.2 against 21.0; SEG 24 (issue-bound, 6 waves per
// SIMD) loses 1-3 %, SEG 3 about 1 % (profiles/r05_west_carry_ab.log).  So segments of 4..16
// rows take it.  GOL_TILE_WEST_CARRY=0: never (A/B builds).
// K1t ORD 8 / 9 (the turn in inline asm, gol_tile_turn.h): bit 1 = the workgroup barrier after
// rows 1 and 2 instead of right after the edge sums' stores, bit 2 = LDS slots 16 B apart
// instead of 64 (A/B builds: make variant VDEFS=-DGOL_TURN_VAR=n)
#ifndef GOL_TURN_VAR
#define GOL_TURN_VAR 4
#endif
#ifndef GOL_TILE_WEST_CARRY
#define GOL_TILE_WEST_CARRY 1
#endif
// Raw edge rows (ORD 0-2, one word per lane, segments of up to GOL_TILE_RAW rows; 0 = never):
// each lane publishes its first and last row as they are -- one 16-B LDS slot, one
// ds_write_b128 -- instead of their two 3-cell row sums (two slots, two ds_write_b128), and
// sums the rows it reads from the segments above and below itself (two more row sums a turn).
// Half the LDS bytes per turn for 8 more VALU per neighbour row: the trade pays where a turn's
// LDS stores, not its VALU, are the critical path -- short segments on small boards.
#ifndef GOL_TILE_RAW
#define GOL_TILE_RAW 0
#endif
// ORD 3 = two tiles per workgroup, software-pipelined (tile_pass_pair; A/B builds: make variant
// VDEFS=-DGOL_TILE_PAIR=1).  Without it ORD 3 is the tools build's no-barrier timing ablation.
#ifndef GOL_TILE_PAIR
#define GOL_TILE_PAIR 0
#endif
// (K1p / K1q / K1r: polls of a neighbour tile's flag before a wait gives up; the test build
// libgolamd_spin0.so sets 0)
#ifndef GOL_TILE_SPIN_LIMIT
#define GOL_TILE_SPIN_LIMIT (1 << 22)
#endif
template <int SEG, int W>
constexpr bool tile_west_carry() { return GOL_TILE_WEST_CARRY && W == 1 && SEG >= 4 && SEG <= 16; }

namespace golk {

constexpr int kTileMaxWaves = 16;                       // 1024 threads per workgroup
// dynamic LDS of a workgroup of `threads` threads: row sums of the segments' edge rows (16 B
// per word of the lane), first and last row, two turn parities; then one progress flag per
// wave (ORD 4), 64 B
constexpr size_t tile_lds_bytes(int threads, int words)
{
    return (size_t)threads * 4 * 16 * words + 4 * kTileMaxWaves;
}
// tile_seg = SEG + 100 * ORD + 1000 * (W - 1): rows per lane segment, turn order (0: in order;
// 1: interior rows, then the edge rows; 2: the same with the barrier after the interior rows;
// 4: ORD 1 with no workgroup barrier -- each wave waits only for its two neighbour waves'
// published edge sums, through per-wave progress flags in LDS; 5: ORD 1 with the edge sums
// read back from LDS instead of kept in registers; 6: ORD 5 with the barrier after the
// interior rows; 7: ORD 5 with the tile's two halo segments in wave 0, which skips the rows
// the shrinking trapezoid no longer needs -- see tile_pass; 8: ORD 5's turn as generated
// inline asm with a hand-made, parity-aware VGPR assignment; 9: ORD 8 with ds_bpermute lane
// shifts -- 7, 8 and 9 in the tools build only), words per lane
constexpr int tile_seg_rows(int code) { return code % 100; }
constexpr int tile_seg_words(int code) { return code / 1000 + 1; }
// ORD 8 / 9 with the 16-B slot layout: the slot count rounded up to a power of two (the turn
// parity is an XOR of the addresses)
constexpr int tile_slots_pow2(int threads)
{
    int n = 64;
    while (n < threads) n *= 2;
    return n;
}
constexpr size_t tile_lds_bytes_code(int threads, int code)
{
    const int ord = code / 100 % 10;
    return (ord == 8 || ord == 9) && (GOL_TURN_VAR & 4)
               ? tile_lds_bytes(tile_slots_pow2(threads), 1)
           : ord == 3 && GOL_TILE_PAIR ? 2 * tile_lds_bytes(threads, 1)   // (two tiles' slots)
                                       : tile_lds_bytes(threads, tile_seg_words(code));
}

// W words per lane (2W dwords, interleaved layout word by word).  With W = 2 the lane's two
// words are neighbours, so only the outer edges need a lane shift: per row 2 DPP + 2W funnel
// shifts + 4W v_bitop3 instead of W x (2 + 2 + 4) -- 48 instead of 52 SIMD cycles per 4096
// cell-updates with the rule.
// One pass of K turns over one tile (the body of k_step_tile, and of each block of
// k_tile_persist / item of k_tile_stream).  PERSIST: the workgroup stays for further passes,
// so no wave leaves the trapezoid early -- every wave runs every turn (a wave past the
// trapezoid computes halo rows nobody reads) and the pass returns on every path.  (A leaving
// wave would have to meet the barriers of its remaining turns, and that exit path alone took
// the SEG 24 pass from 80 to 126 VGPRs.)
// K1r (RING): the tile stays in registers across blocks; between blocks only its ring is
// exchanged (k_tile_ring below)
struct RingArgs {
    uint64_t *u0, *u1;          // board-layout edge buffers, block b writes u[b % 2]
    unsigned *flags;            // per tile: epoch + b + 1 once its block-b edges are stored
    unsigned epoch;
    int turns;                  // turns of the launch, in blocks of <= K
    unsigned *gcount;           // (tools, GOL_RING=2) non-null: a grid-wide barrier per block
    unsigned gbase;             // instead of the 8 neighbours: *gcount at the launch's start
    int ablate;                 // (tools timing ablations, wrong boards: 1 no edge stores, 2 no
                                // flag wait, 4 no ring loads)
};
template <int SEG, int ORD, int W, bool PERSIST, bool RING = false>
__device__ __forceinline__ void tile_pass(const uint64_t *__restrict__ in,
                                          uint64_t *__restrict__ out, const StepArgs &a,
                                          int turns, int tile, int ntx,
                                          RingArgs ra = RingArgs{})
{
    constexpr int ND = 2 * W;                            // dwords per lane and row
    constexpr int NS = 2 * ND;                           // row-sum dwords (2 bits per dword)
    static_assert(SEG >= 2, "two edge rows per segment");
    // per turn parity: the 3-cell row sums of the first / last row of every segment,
    // segment-major, C slots per segment (dynamic LDS, W uint4 per slot)
    extern __shared__ uint4 xsh[];
    const int nslot = (int)(blockDim.x);                 // waves x 64 >= segments x C
    const int TW = a.tile_w, C = TW + 2, G = 64 / C;     // (in lanes of W words)
    const int K = turns, TH = a.band;
    const int nl = a.nw / W;                             // lane columns per row
    const int ty = tile / ntx, tx = tile - ty * ntx;
    const int y0 = a.row_lo + ty * TH;
    const int x0 = tx * TW;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int group = lane / C, col = lane - group * C;
    const bool live = group < G;                         // lanes past G groups: idle
    const int nseg = (TH + 2 * K + SEG - 1) / SEG;       // segments the tile needs
    // ORD 7 (G == 2, nseg >= 3; host-checked): wave 0 holds the top segment (group 0) and the
    // bottom one (group 1, its rows in reverse order), the other waves the segments between,
    // in order.  Both of wave 0's segments then leave the trapezoid from their local row 0
    // on: turn t changes tile rows [t + 1, 2K + TH - 1 - t), so local rows 0 .. t of either
    // segment are outside it, and wave 0 can skip them for both groups at once (turn4 below).
    // The rule is symmetric in up and down, so a reversed segment runs the same body; only
    // its loads, stores and LDS edge slots are mirrored.
    constexpr bool kHalo = ORD == 7;
    static_assert(!kHalo || W == 1, "ORD 7: one word per lane");
    const int seg = !kHalo ? wave * G + group
                           : wave == 0 ? (group == 0 ? 0 : nseg - 1) : (wave - 1) * G + group + 1;
    const bool rev = kHalo && wave == 0 && group == 1;   // (a lane-varying flag: group 1 only)
    const int slot = seg * C + col;

    // lane column (torus wrap) and the lane's rows: tile row t = seg * SEG + i is buffer row
    // y0 - K + t (mod modrows; rows past the tile are read, never stored)
    int gx = x0 - 1 + (live ? col : 0);
    while (gx < 0) gx += nl;
    while (gx >= nl) gx -= nl;
    const int M = a.modrows;
    const uint32_t pitch_b = (uint32_t)a.pitch * 8u;
    const uint32_t span = (uint32_t)M * pitch_b;
    int r = y0 - K + (live ? seg : 0) * SEG + (rev ? SEG - 1 : 0);
    while (r < 0) r += M;
    while (r >= M) r -= M;
    uint32_t off = (uint32_t)r * pitch_b + (uint32_t)gx * (8u * W);
    [[maybe_unused]] const uint32_t off_first = off;     // (RING: the segment's first row)
    const uint32_t lstep = rev ? span - pitch_b : pitch_b;   // (a reversed segment loads upwards)
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc((void *)in, (short)0, (int)span, kBufFlags);
    const __amdgpu_buffer_rsrc_t rout =
        __builtin_amdgcn_make_buffer_rsrc((void *)out, (short)0, (int)span, kBufFlags);

    // PERSIST: loads bypass this CU's vector L1 (sc1): block b reads rows other CUs wrote
    // since block b - 2 left lines of the same buffer in it, and the L1 is never refreshed
    // by another CU's stores
    constexpr int kLoadAux = PERSIST ? 16 : GOL_TILE_LOAD_AUX;
    uint32_t v[SEG][ND];
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
        if constexpr (W == 1) {
            const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(rin, off, 0, kLoadAux);
            v[i][0] = w.x;
            v[i][1] = w.y;
        } else {
            const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, kLoadAux);
            v[i][0] = w.x;
            v[i][1] = w.y;
            v[i][2] = w.z;
            v[i][3] = w.w;
        }
        off += lstep;
        off = off >= span ? off - span : off;            // (the column stays < pitch_b)
    }

    // 3-cell row sums of one row: per word w (even dword e, odd dword o) the sums of the even
    // cells (s[4w], s[4w+1]) and of the odd cells (s[4w+2], s[4w+3]); K1s's stage, with the
    // neighbour words inside the lane taken as they are
    auto rsum = [&](const uint32_t (&x)[ND], uint32_t (&s)[NS]) {
        const uint32_t Rt = dpp_from_upper_z(x[0]);      // east lane's first even cells
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint32_t e = x[2 * w], o = x[2 * w + 1];
            uint32_t wl;
            if constexpr (tile_west_carry<SEG, W>()) {
                // every lane is active here (the idle lanes run the turn too), so the mask
                // holds every lane's sign bit; lane 0 gets carry 0, as the DPP's bound_ctrl
                const uint64_t m = __builtin_amdgcn_ballot_w64((int)o < 0) << 1;
                uint64_t co;
                asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(wl), "=&s"(co) : "v"(o), "s"(m));
            } else {
                const uint32_t L = dpp_from_lower_z(x[ND - 1]);   // west lane's last odd cells
                wl = __builtin_amdgcn_alignbit(o, w == 0 ? L : x[2 * w - 1], 31);
            }
            const uint32_t er = __builtin_amdgcn_alignbit(w == W - 1 ? Rt : x[2 * w + 2], e, 1);
            s[4 * w + 0] = xor3(wl, e, o);
            s[4 * w + 1] = maj(wl, e, o);
            s[4 * w + 2] = xor3(e, o, er);
            s[4 * w + 3] = maj(e, o, er);
        }
    };
    // next state of the lane's row from the sums of the rows above (A), at (B) and below (Cs)
    auto rule = [&](const uint32_t (&A)[NS], const uint32_t (&B)[NS], const uint32_t (&Cs)[NS],
                   uint32_t (&x)[ND]) {
        uint32_t n[ND];
#pragma unroll
        for (int d = 0; d < ND; ++d)
            n[d] = life_rule7(A[2 * d], B[2 * d], Cs[2 * d], A[2 * d + 1], B[2 * d + 1],
                              Cs[2 * d + 1], x[d]);
#pragma unroll
        for (int d = 0; d < ND; ++d) x[d] = n[d];
    };
    auto put = [&](uint4 *base, const uint32_t (&S)[NS]) {
#pragma unroll
        for (int q = 0; q < W; ++q)
            base[(size_t)q * nslot * 4] =
                make_uint4(S[4 * q], S[4 * q + 1], S[4 * q + 2], S[4 * q + 3]);
    };
    auto get = [&](const uint4 *base, uint32_t (&S)[NS]) {
#pragma unroll
        for (int q = 0; q < W; ++q) {
            const uint4 u = base[(size_t)q * nslot * 4];
            S[4 * q] = u.x;
            S[4 * q + 1] = u.y;
            S[4 * q + 2] = u.z;
            S[4 * q + 3] = u.w;
        }
    };
    // Slot arrays: [q][parity][top / bottom][slot], q = the word of the lane.  Every lane
    // writes and reads every turn, with no mask: the idle lanes (group >= G) own the slots
    // past the tile's (waves x G x C .. waves x 64), and a segment with no neighbour above
    // (below) reads its own slot.  What it reads there is junk, but it only reaches the tile's
    // outermost row, whose error moves inward one row per turn like that of any halo row.
    const int nlive = (int)(blockDim.x >> 6) * G * C;
    const int myslot = live ? slot : nlive + wave * (64 - G * C) + (lane - G * C);
    const int s_up = live && seg > 0 ? slot - C : myslot;
    const int s_dn = live && seg + 1 < nseg ? slot + C : myslot;
    // a lane's own edge slots and its neighbours', by the lane's local row order: its first
    // row's sums go to the top-edge array and its last row's to the bottom-edge array, and it
    // reads the bottom edge of the segment above and the top edge of the one below -- all
    // mirrored for a reversed segment (ORD 7), whose first row is physically its bottom one
    const int o_wt = (rev ? (int)nslot : 0) + myslot, o_wb = (rev ? 0 : (int)nslot) + myslot;
    const int o_up = rev ? s_dn : (int)nslot + s_up, o_dn = rev ? (int)nslot + s_up : s_dn;
    // Turn parity p uses the slots 2 p nslot further on.  Short segments run two turns per
    // loop iteration with p a compile-time constant (the parity's addresses hoisted out of the
    // loop: 11 % faster turns at SEG 3-4); long ones one turn body with the offset added per
    // turn -- the doubled body of a long segment ran 10-14 % slower (instruction fetch,
    // profiles/r03_tile_unroll_ab.log).  The threshold 12: pairs at SEG 8 are 2-3 % faster
    // than one body, at SEG 16 11-28 % slower (profiles/r03b_tile_pairs_threshold.log).
    constexpr bool kPairs = SEG * W <= GOL_TILE_PAIRS_MAX;
    constexpr bool kRaw = ORD < 4 && W == 1 && SEG <= GOL_TILE_RAW;
    // (with pairs the lane's four LDS addresses of each parity are loop-invariant registers;
    // one body forms them per turn -- precomputed there, the long bodies ran 4-8 % slower)
    uint4 *const wtop2[2] = {xsh + o_wt, xsh + 2 * nslot + o_wt};
    uint4 *const wbot2[2] = {xsh + o_wb, xsh + 2 * nslot + o_wb};
    const uint4 *const rup2[2] = {xsh + o_up, xsh + 2 * nslot + o_up};
    const uint4 *const rdn2[2] = {xsh + o_dn, xsh + 2 * nslot + o_dn};
    auto wtop = [&](int p, int off) { return kPairs ? wtop2[p] : xsh + off + o_wt; };
    auto wbot = [&](int p, int off) { return kPairs ? wbot2[p] : xsh + off + o_wb; };
    auto rup = [&](int p, int off) { return kPairs ? rup2[p] : (const uint4 *)(xsh + off + o_up); };
    auto rdn = [&](int p, int off) { return kPairs ? rdn2[p] : (const uint4 *)(xsh + off + o_dn); };
    // A wave whose rows are all outside the turn's trapezoid leaves: the tile's rows
    // [t + 1, 2K + TH - 1 - t) change at turn t (t = 0 .. K-1) and need the sums of the rows
    // one further out; a wave above row t (below row 2K + TH - 1 - t) holds no row that any
    // later turn or the final store needs (its rows are < K, resp. >= K + TH), and the
    // workgroup barrier no longer counts it once it has ended.
    // the wave's tile rows (ORD 7: wave 0 spans the whole tile -- it never leaves; wave w > 0
    // holds segments (w - 1) G + 1 ..)
    const int wrow0 = !kHalo ? wave * G * SEG : wave == 0 ? 0 : ((wave - 1) * G + 1) * SEG;
    const int wrow1 = !kHalo ? wrow0 + G * SEG : wave == 0 ? 1 << 30 : wrow0 + G * SEG;
    // ORD 4: per-wave progress flags after the slot arrays.  flag[w] = the last turn whose
    // edge sums wave w has published (-1 before the first; INT_MAX once it has left), written
    // by lane 0 after its sums: the LDS serves one wave's requests in issue order, so a wave
    // that reads flag[w] >= t reads w's turn-t sums (the K1w hand-off assumption).
    // The sums are double-buffered by turn parity: a wave overwrites its turn-(t-2) slots only
    // after both neighbours published turn t-1, i.e. after they finished reading turn t-2.
    const int nwaves = (int)(blockDim.x >> 6);
    volatile int *const flag = (volatile int *)(xsh + 4 * (size_t)nslot * W);
    if constexpr (ORD == 4) {
        if (lane == 0) flag[wave] = -1;
        __syncthreads();                                  // (once per launch)
    }
    auto publish = [&](int t) {
        if constexpr (ORD == 4) {
            asm volatile("" ::: "memory");
            if (lane == 0) flag[wave] = t;
        }
    };
    auto await_neighbours = [&](int t) {
        if constexpr (ORD == 4) {
            const int up = wave > 0 ? wave - 1 : wave, dn = wave + 1 < nwaves ? wave + 1 : wave;
            for (;;) {
                const int a = __builtin_amdgcn_readfirstlane(flag[up]);
                const int b = __builtin_amdgcn_readfirstlane(flag[dn]);
                if (a >= t && b >= t) break;
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
    };
    // ORD 4's turn: the edge sums F (row 0) and Lr (row SEG-1) go to LDS and are read back
    // from the wave's own slots when needed, instead of staying live across the interior rows
    // and the wait (64 VGPRs at SEG 16: 8 waves per SIMD).  ORD 5: the same turn with ORD 1's
    // workgroup barrier after the puts instead of the flags (80 VGPRs at SEG 24: 6 waves per
    // SIMD, where the stencil's instruction mix issues fastest -- tools/calib/valu_issue.hip
    // occupancy sweep).  ORD 6: the barrier where ORD 4 waits, after the interior rows (ORD
    // 2's placement: a wave that arrives early has done all the work that needs no neighbour;
    // the turn-parity double buffer still needs only the one barrier per turn)
    // ORD 7's wave 0 updates, at turn t, only its rows lo = t + 1 (at most SEG - 2) and above:
    // local rows 0 .. t of both its segments are outside the trapezoid.  The rules of the rows
    // below lo (14 of a row's 22 VALU) and row 0's neighbour read are skipped by wave-uniform
    // scalar branches (the other waves pass lo = 0 and never take one); the row sums stay
    // unconditional -- skipping them too made the sliding window's values conditional, and
    // the compiler paid 4 v_mov per row on every wave's path to merge them.  A skipped row goes
    // stale exactly when the trapezoid makes it junk, and row lo reads only rows lo - 1 ..,
    // which were updated at turn t - 1 (their lo was t).  For every other turn order lo is the
    // constant 0.
    auto turn4 = [&](auto P, int poff, int t, int lo_rt) {
        constexpr int p = decltype(P)::value;
        const int lo = ORD == 7 ? lo_rt : 0;
        const int off = poff;
        uint32_t Pw[NS], Q[NS], S1[NS];
        {
            uint32_t F[NS], Lr[NS];
            rsum(v[0], F);
            rsum(v[SEG - 1], Lr);
            put(wtop(p, off), F);
            put(wbot(p, off), Lr);
            if constexpr (ORD == 5 || ORD == 7) __syncthreads();
            else if constexpr (ORD == 4) publish(t);
#pragma unroll
            for (int k = 0; k < NS; ++k) Pw[k] = F[k];
        }
        rsum(v[1], Q);
#pragma unroll
        for (int k = 0; k < NS; ++k) S1[k] = Q[k];
#pragma unroll
        for (int i = 1; i + 1 < SEG; ++i) {
            uint32_t R[NS];
            if (i + 2 == SEG) get(wbot(p, off), R);   // (own bottom slot: Lr)
            else rsum(v[i + 1], R);
            if (i >= lo) rule(Pw, Q, R, v[i]);
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                Pw[k] = Q[k];
                Q[k] = R[k];
            }
        }
        // (keep the wait after the interior rows: the compiler would otherwise sink them
        // below the poll loop)
#pragma unroll
        for (int i = 1; i + 1 < SEG; ++i)
#pragma unroll
            for (int d = 0; d < ND; ++d) asm volatile("" : "+v"(v[i][d]));
        if constexpr (ORD == 6) __syncthreads();
        else await_neighbours(t);
        uint32_t U[NS], D[NS], F[NS];
        if (lo == 0) {
            get(rup(p, off), U);
            get(wtop(p, off), F);
            rule(U, F, S1, v[0]);
        }
        get(rdn(p, off), D);
        get(wbot(p, off), F);                                 // (Lr)
        rule(Pw, F, D, v[SEG - 1]);
    };
    auto turn = [&](auto P, int poff, int t) {
        if constexpr (ORD >= 4) {
            turn4(P, poff, t, kHalo && wave == 0 ? min(t + 1, SEG - 2) : 0);
            return;
        }
        constexpr int p = decltype(P)::value;
        const int off = poff;
        // the segment's first and last row sums go to the neighbours (row sums, not rows: no
        // lane sums a row twice -- SEG row sums and SEG rules per turn); kRaw: the rows
        uint32_t F[NS], Lr[NS];
        rsum(v[0], F);
        rsum(v[SEG - 1], Lr);
        if constexpr (kRaw) {
            *wtop(p, off) = make_uint4(v[0][0], v[0][1], v[SEG - 1][0], v[SEG - 1][1]);
        } else {
            put(wtop(p, off), F);
            put(wbot(p, off), Lr);
        }
        uint32_t U[NS], D[NS];
        // kRaw: the last row of the segment above (the z, w half of its slot) and the first
        // row of the one below (x, y), summed here
        auto get_raw = [&](uint32_t (&Us)[NS], uint32_t (&Ds)[NS]) {
            const uint4 *const base = kPairs ? xsh + 2 * nslot * p : xsh + off;
            const uint2 a = *(reinterpret_cast<const uint2 *>(base + s_up) + 1);
            const uint2 b = *reinterpret_cast<const uint2 *>(base + s_dn);
            const uint32_t ra[ND] = {a.x, a.y}, rb[ND] = {b.x, b.y};
            rsum(ra, Us);
            rsum(rb, Ds);
        };
        if constexpr (ORD < 2 || ORD == 3) {
            if constexpr (ORD != 3) __syncthreads();   // ORD 3: timing ablation (tools build)
            if constexpr (kRaw) {
                get_raw(U, D);
            } else {
                get(rup(p, off), U);
                get(rdn(p, off), D);
            }
        }
        if constexpr (ORD == 0 || ORD == 3) {
            // in order: A, B, Cs = sums of rows i-1, i, i+1
            uint32_t A[NS], B[NS];
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                A[k] = U[k];
                B[k] = F[k];
            }
#pragma unroll
            for (int i = 0; i < SEG; ++i) {
                uint32_t Cs[NS];
                if (i + 1 == SEG) {
#pragma unroll
                    for (int k = 0; k < NS; ++k) Cs[k] = D[k];
                } else if (i + 2 == SEG) {
#pragma unroll
                    for (int k = 0; k < NS; ++k) Cs[k] = Lr[k];
                } else {
                    rsum(v[i + 1], Cs);
                }
                rule(A, B, Cs, v[i]);
#pragma unroll
                for (int k = 0; k < NS; ++k) {
                    A[k] = B[k];
                    B[k] = Cs[k];
                }
            }
        } else {
            // ORD 1: interior rows 1 .. SEG-2 first (their sums are all local), so the LDS
            // reads land while they compute; window P, Q, R = sums of rows i-1, i, i+1
            uint32_t Pw[NS], Q[NS], S1[NS];
#pragma unroll
            for (int k = 0; k < NS; ++k) Pw[k] = F[k];
            if constexpr (SEG >= 3) {
                rsum(v[1], Q);
#pragma unroll
                for (int k = 0; k < NS; ++k) S1[k] = Q[k];
            } else {
#pragma unroll
                for (int k = 0; k < NS; ++k) S1[k] = Q[k] = Lr[k];
            }
#pragma unroll
            for (int i = 1; i + 1 < SEG; ++i) {
                uint32_t R[NS];
                if (i + 2 == SEG) {
#pragma unroll
                    for (int k = 0; k < NS; ++k) R[k] = Lr[k];
                } else {
                    rsum(v[i + 1], R);
                }
                rule(Pw, Q, R, v[i]);
#pragma unroll
                for (int k = 0; k < NS; ++k) {
                    Pw[k] = Q[k];
                    Q[k] = R[k];
                }
            }
            // (Pw = the sums of row SEG-2, or of row 0 when SEG == 2)
            if constexpr (ORD == 2) {
                // ORD 2: the barrier after the interior rows -- a wave that arrives early has
                // already done all the work that needs no neighbour
                __syncthreads();
                if constexpr (kRaw) {
                    get_raw(U, D);
                } else {
                    get(rup(p, off), U);
                    get(rdn(p, off), D);
                }
            }
            rule(U, F, S1, v[0]);
            rule(Pw, Lr, D, v[SEG - 1]);
        }
    };
    const int lastrow = 2 * K + TH - 1;
    // a wave leaving the trapezoid at turn t: its rows are all < K or >= K + TH, so it has
    // nothing to store.  It ends (the barrier stops counting it; ORD 4: its flag says it has
    // gone).  Persistent passes keep every wave to the end of the pass.
    auto leave = [&](int t) {
        if constexpr (ORD == 4) {
            if (lane == 0) flag[wave] = 0x7fffffff;
        }
    };
    bool gone = false;
    if constexpr (RING) {
        // K1r: ceil(turns / K) blocks of near-equal depth <= K on the tile held in v.  After
        // block b the TH x TW interior is exact and everything else is stale; the tile stores
        // its ring's sources -- interior rows within K of its top or bottom edge and its first
        // and last interior columns -- into u[b % 2] at their board positions, flags them, waits
        // for its 8 neighbours' flags, and reloads from u[b % 2] what its neighbours stored: the
        // K rows above and below its interior (halo lanes included) and the two halo lanes.
        // Lanes and rows further out (a ragged tile's columns past the east halo lane, rows past
        // the bottom halo) stay stale: their error moves one cell per turn and the refreshed
        // halo word / K halo rows are as deep as a plain launch's.  Every tile's interior spans
        // >= K rows (host-checked), so each ring cell comes from one of the 8 neighbours.
        // Memory: K1p's uncached buffers (no cache maintenance; loads bypass the vector L1).
        static_assert(PERSIST && W == 1 && ORD != 4 && ORD != 7 && ORD < 8, "K1r: one word per lane");
        const int THv = min(TH, a.row_hi - y0), TWv = min(TW, nl - x0);
        const int nty = (a.row_hi - a.row_lo + TH - 1) / TH;
        const int nblocks = (ra.turns + K - 1) / K, kbase = ra.turns / nblocks,
                  kextra = ra.turns % nblocks;
        bool gave_up = false;
        for (int b = 0; b < nblocks; ++b) {
            const int kb = kbase + (b < kextra ? 1 : 0);
            if constexpr (!kPairs) {
                for (int t = 0; t < kb; ++t) turn(std::integral_constant<int, 0>{}, (t & 1) * 2 * nslot, t);
            } else {
                for (int t = 0; t < kb; t += 2) {
                    turn(std::integral_constant<int, 0>{}, 0, t);
                    if (t + 1 == kb) break;
                    turn(std::integral_constant<int, 1>{}, 0, t + 1);
                }
            }
            if (b + 1 == nblocks) break;
            uint64_t *const X = (b & 1) ? ra.u1 : ra.u0;
            const __amdgpu_buffer_rsrc_t rx =
                __builtin_amdgcn_make_buffer_rsrc((void *)X, (short)0, (int)span, kBufFlags);
            // (the lane's values pass through an empty asm here, so that what the exchange
            // derives from them -- two predicates per row -- is formed per exchange instead of
            // hoisted out of the block loop and held in registers across the turns)
            int ln = lane, thv = THv, twv = TWv, kk = K;
            uint32_t off0 = off_first;
            asm volatile("" : "+v"(ln), "+v"(off0), "+s"(thv), "+s"(twv), "+s"(kk));
            const int gr = ln / C, cl = ln - gr * C;
            const bool lv = gr < G;
            const int tr0 = (wave * G + gr) * SEG;       // the lane's first tile row
            if (lv && cl >= 1 && cl <= twv && !(ra.ablate & 1)) {
                const bool side = cl == 1 || cl == twv;
                uint32_t so = off0;
#pragma unroll
                for (int i = 0; i < SEG; ++i) {
                    const int j = tr0 + i - kk;           // interior row of the tile
                    if (j >= 0 && j < thv && (side || j < kk || j >= thv - kk))
                        buf_store(v[i], rx, so, 0);
                    so += pitch_b;
                    so = so >= span ? so - span : so;
                }
            }
            __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));   // this wave's stores are done
            __syncthreads();                                     // ... and every wave's
            // (u0 / u1 are uncached: completed stores are in memory, visible to every XCD)
            if (threadIdx.x == 0) {
                __hip_atomic_store(ra.flags + tile, ra.epoch + (unsigned)b + 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            if (ra.gcount && threadIdx.x == 0) {        // (every tile: a grid-wide barrier)
                __hip_atomic_fetch_add(ra.gcount, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned want = ra.gbase + (unsigned)(b + 1) * (unsigned)(nty * ntx);
                bool seen = false;
                for (int spin = 0; !seen && spin < GOL_TILE_SPIN_LIMIT; ++spin) {
                    const unsigned fv = __hip_atomic_load(ra.gcount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    seen = (int)(fv - want) >= 0;
                    if (!seen) __builtin_amdgcn_s_sleep(1);
                }
                gave_up |= !seen;
            }
            if (!ra.gcount && threadIdx.x < 8 && !(ra.ablate & 2)) {   // one neighbour per lane 0..7
                const int jn = (int)threadIdx.x + (threadIdx.x >= 4 ? 1 : 0);   // skip (0, 0)
                const int ny = (ty + jn / 3 - 1 + nty) % nty, nx = (tx + jn % 3 - 1 + ntx) % ntx;
                const unsigned want = ra.epoch + (unsigned)b + 1u;
                const unsigned *f = ra.flags + ny * ntx + nx;
                bool seen = false;
                for (int spin = 0; !seen && spin < GOL_TILE_SPIN_LIMIT; ++spin) {
                    const unsigned fv = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    seen = (int)(fv - want) >= 0;
                    if (!seen) __builtin_amdgcn_s_sleep(1);
                }
                gave_up |= !seen;
            }
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            __syncthreads();
            if (lv && !(ra.ablate & 4)) {
                const bool hl = cl == 0 || cl == twv + 1;
                uint32_t lo = off0;
#pragma unroll
                for (int i = 0; i < SEG; ++i) {
                    const int tr = tr0 + i;
                    if (tr < 2 * kk + thv && (hl || tr < kk || tr >= kk + thv)) {
                        const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(rx, lo, 0, kLoadAux);
                        v[i][0] = w.x;
                        v[i][1] = w.y;
                    }
                    lo += pitch_b;
                    lo = lo >= span ? lo - span : lo;
                }
            }
        }
        if (gave_up && a.err)
            __hip_atomic_store(a.err, kDevErrTileFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if constexpr (ORD == 8 || ORD == 9) {
        // ORD 8: ORD 5's turn as one inline-asm block with a hand-made VGPR assignment
        // (gol_tile_turn.h, generated by gen_tile_turn.py: every v_bitop3 reads registers of
        // both parities, which the compiler's allocation does not ensure -- a v_bitop3 whose
        // sources all have one parity issues at half rate).  LDS: 64 B per slot, [slot][top,
        // bottom][turn parity]; the asm toggles the parity (bit 4) of the three addresses.
        // ORD 9: the same with the lane shifts' neighbour words fetched by ds_bpermute_b32 (the
        // LDS pipe) one row ahead instead of DPP moves (half-rate VALU instructions); lane l
        // reads lane l - 1 at address ba and lane l + 1 at ba + 8 (the wrap reaches only halo
        // and idle lanes, whose cells are junk anyway)
        static_assert(W == 1 && !PERSIST && SEG % 3 == 0, "ORD 8/9: one word per lane, plain launches");
        // Registers: the asm holds v0 .. v(2 SEG + 25); everything else live across the turn
        // loop must fit the rest of the 80-VGPR budget (6 waves per SIMD): the three addresses,
        // a scalar turn count (the turn the wave leaves the trapezoid at, computed once), and
        // the store stage's lane values recomputed after the loop rather than kept.
        // (k_step_tile has no static LDS: the dynamic slots start at LDS address 0, so the
        // parity toggle is an XOR of each address with ps)
        constexpr int TV = (GOL_TURN_VAR & 6) | (ORD == 9 ? 1 : 0);
        const uint32_t base = (uint32_t)(uintptr_t)(lds_void *)xsh;
        uint32_t ad[4];
        uint32_t ps;
        if constexpr ((TV & 4) != 0) {
            // [parity][top, bottom][slot], 16 B per slot, the slot count a power of two
            // (tile_lds_bytes_code)
            const uint32_t ns = (uint32_t)tile_slots_pow2(nslot);
            ad[0] = base + 16u * (uint32_t)myslot;
            ad[1] = base + 16u * (ns + (uint32_t)myslot);
            ad[2] = base + 16u * (ns + (uint32_t)s_up);     // the segment above's last-row sums
            ad[3] = base + 16u * (uint32_t)s_dn;            // the segment below's first-row sums
            ps = 32u * ns;
        } else {
            // [slot][top, bottom][parity], 64 B per slot
            ad[0] = base + 64u * (uint32_t)myslot;
            ad[1] = 0u;
            ad[2] = base + 64u * (uint32_t)s_up + 32u;
            ad[3] = base + 64u * (uint32_t)s_dn;
            ps = 16u;
        }
        // the wave leaves at the first turn t with wrow1 <= t or wrow0 > lastrow - t
        const int tend = __builtin_amdgcn_readfirstlane(
            max(0, min(K, min(wrow1, lastrow - wrow0 + 1))));
        const uint32_t ba = ORD == 9 ? (uint32_t)((lane + 63) & 63) * 4u : 0u;
        ps = __builtin_amdgcn_readfirstlane(ps);
        for (int t = 0; t < tend; ++t) tile_turn_asm<SEG, TV>(v, ad, ps, ba);
        if (tend < K) return;
        // interior rows [K, K + TH) of the tile, below row_hi; interior columns inside the row
        // (the lane's values from the lane count of an opaque all-ones mask, formed after the
        // loop: neither the thread index nor anything derived from it stays live across it)
        uint32_t all = ~0u;
        asm volatile("" : "+v"(all));
        const int ln = (int)__builtin_amdgcn_mbcnt_hi(all, __builtin_amdgcn_mbcnt_lo(all, 0u));
        const int gr = ln / C, cl = ln - gr * C;
        if (gr >= G || cl < 1 || cl > TW || x0 + cl - 1 >= nl) return;
        const int t0 = (wave * G + gr) * SEG;
        uint32_t so = (uint32_t)(y0 - K + t0) * pitch_b + (uint32_t)(x0 + cl - 1) * 8u;
#pragma unroll
        for (int i = 0; i < SEG; ++i) {
            const int tr = t0 + i;
            if (tr >= K && tr < K + TH && y0 - K + tr < a.row_hi) buf_store(v[i], rout, so, 0);
            so += pitch_b;
        }
        return;
    } else if constexpr (kHalo) {
        static_assert(!kPairs, "ORD 7: long segments");
        for (int t = 0; t < K; ++t) {
            // (wave 0 spans the whole tile and never leaves: wrow1 is out of reach)
            if (!PERSIST && (wrow1 <= t || wrow0 > lastrow - t)) {   // (wave-uniform)
                leave(t);
                gone = true;
                break;
            }
            turn(std::integral_constant<int, 0>{}, (t & 1) * 2 * nslot, t);
        }
    } else if constexpr (!kPairs) {
        for (int t = 0; t < K; ++t) {
            if (!PERSIST && (wrow1 <= t || wrow0 > lastrow - t)) {   // (wave-uniform)
                leave(t);
                gone = true;
                break;
            }
            turn(std::integral_constant<int, 0>{}, (t & 1) * 2 * nslot, t);
        }
    } else {
        for (int t = 0; t < K; t += 2) {
            if (!PERSIST && (wrow1 <= t || wrow0 > lastrow - t)) {
                leave(t);
                gone = true;
                break;
            }
            turn(std::integral_constant<int, 0>{}, 0, t);
            if (t + 1 == K) break;
            if (!PERSIST && (wrow1 <= t + 1 || wrow0 > lastrow - t - 1)) {
                leave(t + 1);
                gone = true;
                break;
            }
            turn(std::integral_constant<int, 1>{}, 0, t + 1);
        }
    }
    if (!PERSIST && gone) return;
    // interior rows [K, K + TH) of the tile, below row_hi; interior columns inside the row
    if (gone || !live || col < 1 || col > TW || x0 + col - 1 >= nl) return;
    const int t0 = seg * SEG + (rev ? SEG - 1 : 0);
    const int dr = rev ? -1 : 1;
    const uint32_t sstep = rev ? 0u - pitch_b : pitch_b;
    // per-lane byte offset (the segment differs between the lane groups of a wave); rows
    // y0 - K + t0 + i are stored only once inside [row_lo, row_hi): no wrap, and the
    // unsigned sum is exact there even if the first row of the segment lies above row 0
    uint32_t so = (uint32_t)(y0 - K + t0) * pitch_b + (uint32_t)(x0 + col - 1) * (8u * W);
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
        const int tr = t0 + dr * i;
        if (tr >= K && tr < K + TH && y0 - K + tr < a.row_hi) {
            if constexpr (W == 1 && GOL_TILE_STORE_AUX != 0)
                buf_store_aux<GOL_TILE_STORE_AUX>(v[i], rout, so);
            else
                buf_store(v[i], rout, so, 0);
        }
        so += sstep;
    }
}

// ORD 3 (round 6): two tiles per workgroup, software-pipelined (the round-5 verdict's ask for
// small boards, whose turn is a serial chain: one barrier, the LDS round trip of the edge sums,
// the edge rules, the next turn's row sums and stores, then the barrier again -- the waves of a
// workgroup all reach each phase together, so the VALU idles while the LDS works and back).
// Every lane holds one SEG-row segment of tile A and one of tile B (the same local rows of two
// tiles), and each turn is split in two halves:
//   H1(X) -- the row sums of the segment's first and last rows, their stores to LDS, and the
//            interior rows (everything that needs no neighbour);
//   H2(X) -- the neighbours' edge sums read back and the first and last rows' rules.
// Between two workgroup barriers a lane runs H2 of one tile beside H1 of the other, so one
// tile's LDS reads are in flight while the other tile's VALU work issues:
//   H1(A, 0) | H2(A, t), H1(B, t) | H2(B, t), H1(A, t + 1) | ...
// Two barriers per turn for two tiles: one per tile-turn, as for one tile.  The edge sums stay
// double-buffered by turn parity per tile ([tile][parity][top, bottom][slot]).  One word per
// lane; segments of 2..8 rows.
template <int SEG>
__device__ __forceinline__ void tile_pass_pair(const uint64_t *__restrict__ in,
                                               uint64_t *__restrict__ out, const StepArgs &a,
                                               int turns, int tileA, int tileB, bool storeB,
                                               int ntx)
{
    constexpr int ND = 2, NS = 4;
    static_assert(SEG >= 2 && SEG <= 8, "ORD 3: short segments");
    extern __shared__ uint4 xsh[];
    const int nslot = (int)blockDim.x;
    const int TW = a.tile_w, C = TW + 2, G = 64 / C;
    const int K = turns, TH = a.band;
    const int nl = a.nw;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int group = lane / C, col = lane - group * C;
    const bool live = group < G;
    const int nseg = (TH + 2 * K + SEG - 1) / SEG;
    const int seg = wave * G + group;
    const int slot = seg * C + col;
    const int M = a.modrows;
    const uint32_t pitch_b = (uint32_t)a.pitch * 8u;
    const uint32_t span = (uint32_t)M * pitch_b;
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc((void *)in, (short)0, (int)span, kBufFlags);
    const __amdgpu_buffer_rsrc_t rout =
        __builtin_amdgcn_make_buffer_rsrc((void *)out, (short)0, (int)span, kBufFlags);
    const int tiles[2] = {tileA, tileB};
    uint32_t v[2][SEG][ND];
    int y0s[2], x0s[2];
#pragma unroll
    for (int X = 0; X < 2; ++X) {
        const int ty = tiles[X] / ntx, tx = tiles[X] - ty * ntx;
        y0s[X] = a.row_lo + ty * TH;
        x0s[X] = tx * TW;
        int gx = x0s[X] - 1 + (live ? col : 0);
        while (gx < 0) gx += nl;
        while (gx >= nl) gx -= nl;
        int r = y0s[X] - K + (live ? seg : 0) * SEG;
        while (r < 0) r += M;
        while (r >= M) r -= M;
        uint32_t off = (uint32_t)r * pitch_b + (uint32_t)gx * 8u;
#pragma unroll
        for (int i = 0; i < SEG; ++i) {
            const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(rin, off, 0, 0);
            v[X][i][0] = w.x;
            v[X][i][1] = w.y;
            off += pitch_b;
            off = off >= span ? off - span : off;
        }
    }
    auto rsum = [&](const uint32_t (&x)[ND], uint32_t (&s)[NS]) {
        const uint32_t Rt = dpp_from_upper_z(x[0]);
        const uint32_t e = x[0], o = x[1];
        uint32_t wl;
        if constexpr (tile_west_carry<SEG, 1>()) {
            const uint64_t m = __builtin_amdgcn_ballot_w64((int)o < 0) << 1;
            uint64_t co;
            asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(wl), "=&s"(co) : "v"(o), "s"(m));
        } else {
            wl = __builtin_amdgcn_alignbit(o, dpp_from_lower_z(o), 31);
        }
        const uint32_t er = __builtin_amdgcn_alignbit(Rt, e, 1);
        s[0] = xor3(wl, e, o);
        s[1] = maj(wl, e, o);
        s[2] = xor3(e, o, er);
        s[3] = maj(e, o, er);
    };
    auto rule = [&](const uint32_t (&A)[NS], const uint32_t (&B)[NS], const uint32_t (&Cs)[NS],
                    uint32_t (&x)[ND]) {
        uint32_t n[ND];
#pragma unroll
        for (int d = 0; d < ND; ++d)
            n[d] = life_rule7(A[2 * d], B[2 * d], Cs[2 * d], A[2 * d + 1], B[2 * d + 1],
                              Cs[2 * d + 1], x[d]);
#pragma unroll
        for (int d = 0; d < ND; ++d) x[d] = n[d];
    };
    auto put = [&](uint4 *p, const uint32_t (&S)[NS]) { *p = make_uint4(S[0], S[1], S[2], S[3]); };
    auto get = [&](const uint4 *p, uint32_t (&S)[NS]) {
        const uint4 u = *p;
        S[0] = u.x;
        S[1] = u.y;
        S[2] = u.z;
        S[3] = u.w;
    };
    // slots as in tile_pass: idle lanes own the slots past the tile's, a segment with no
    // neighbour reads its own (junk that reaches only the tile's outermost row)
    const int nlive = (int)(blockDim.x >> 6) * G * C;
    const int myslot = live ? slot : nlive + wave * (64 - G * C) + (lane - G * C);
    const int s_up = live && seg > 0 ? slot - C : myslot;
    const int s_dn = live && seg + 1 < nseg ? slot + C : myslot;
    // [tile X][parity p][top 0 / bottom 1][slot]
    auto at = [&](int X, int p, int bt, int sl) { return xsh + ((X * 2 + p) * 2 + bt) * nslot + sl; };
    uint32_t F[2][NS], Lr[2][NS], S1[2][NS], Pl[2][NS];
    auto h1 = [&](auto XX, auto PP) {
        constexpr int X = decltype(XX)::value, p = decltype(PP)::value;
        rsum(v[X][0], F[X]);
        rsum(v[X][SEG - 1], Lr[X]);
        put(at(X, p, 0, myslot), F[X]);
        put(at(X, p, 1, myslot), Lr[X]);
        uint32_t Pw[NS], Q[NS];
#pragma unroll
        for (int k = 0; k < NS; ++k) Pw[k] = F[X][k];
        if constexpr (SEG >= 3) {
            rsum(v[X][1], Q);
        } else {
#pragma unroll
            for (int k = 0; k < NS; ++k) Q[k] = Lr[X][k];
        }
#pragma unroll
        for (int k = 0; k < NS; ++k) S1[X][k] = Q[k];
#pragma unroll
        for (int i = 1; i + 1 < SEG; ++i) {
            uint32_t R[NS];
            if (i + 2 == SEG) {
#pragma unroll
                for (int k = 0; k < NS; ++k) R[k] = Lr[X][k];
            } else {
                rsum(v[X][i + 1], R);
            }
            rule(Pw, Q, R, v[X][i]);
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                Pw[k] = Q[k];
                Q[k] = R[k];
            }
        }
#pragma unroll
        for (int k = 0; k < NS; ++k) Pl[X][k] = Pw[k];   // sums of row SEG-2 (row 0 at SEG 2)
    };
    auto h2 = [&](auto XX, auto PP) {
        constexpr int X = decltype(XX)::value, p = decltype(PP)::value;
        uint32_t U[NS], D[NS];
        get(at(X, p, 1, s_up), U);
        get(at(X, p, 0, s_dn), D);
        rule(U, F[X], S1[X], v[X][0]);
        rule(Pl[X], Lr[X], D, v[X][SEG - 1]);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    const int lastrow = 2 * K + TH - 1;
    const int wrow0 = wave * G * SEG, wrow1 = wrow0 + G * SEG;
    auto leaves = [&](int t) { return wrow1 <= t || wrow0 > lastrow - t; };   // (wave-uniform)
    h1(I0{}, I0{});
    __syncthreads();
    bool gone = false;
    for (int t = 0; t < K; t += 2) {
        if (leaves(t)) {
            gone = true;
            break;
        }
        h2(I0{}, I0{});
        h1(I1{}, I0{});
        __syncthreads();
        h2(I1{}, I0{});
        if (t + 1 == K) break;
        h1(I0{}, I1{});
        __syncthreads();
        if (leaves(t + 1)) {
            gone = true;
            break;
        }
        h2(I0{}, I1{});
        h1(I1{}, I1{});
        __syncthreads();
        h2(I1{}, I1{});
        if (t + 2 == K) break;
        h1(I0{}, I0{});
        __syncthreads();
    }
    if (gone || !live || col < 1 || col > TW) return;
    // interior rows [K, K + TH) of each tile below row_hi, interior columns inside the row
    const int t0 = seg * SEG;
#pragma unroll
    for (int X = 0; X < 2; ++X) {
        if (X == 1 && !storeB) break;
        if (x0s[X] + col - 1 >= nl) continue;
        uint32_t so = (uint32_t)(y0s[X] - K + t0) * pitch_b + (uint32_t)(x0s[X] + col - 1) * 8u;
#pragma unroll
        for (int i = 0; i < SEG; ++i) {
            const int tr = t0 + i;
            if (tr >= K && tr < K + TH && y0s[X] - K + tr < a.row_hi) buf_store(v[X][i], rout, so, 0);
            so += pitch_b;
        }
    }
}

// XCD-aware tile order: blockIdx b runs on XCD b % 8, which gets a contiguous run of tiles
// (whole tile rows, so most halo rows were written by the same XCD's L2)
__device__ __forceinline__ int tile_of_block(int ntiles)
{
    const int per = (ntiles + 7) / 8;
    return (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
}

// (ORD 4 up to SEG 16: 64 VGPRs, 8 waves per SIMD -- two 16-wave workgroups per CU)
template <int SEG, int ORD, int W>
__global__ __launch_bounds__(1024, (ORD == 7 ? 6 : 1)) void k_step_tile(const uint64_t *__restrict__ in,
                                                     uint64_t *__restrict__ out, StepArgs a,
                                                     int turns, int ntx, int ntiles)
{
    const int tile = tile_of_block(ntiles);
    if (tile >= ntiles) return;                          // the whole workgroup
    tile_pass<SEG, ORD, W, false>(in, out, a, turns, tile, ntx);
}

// ORD 3: tile pairs (tile_pass_pair).  Pair j runs tiles 2j and 2j + 1; with an odd count the
// last pair repeats its first tile and stores it once.
template <int SEG>
__global__ __launch_bounds__(1024, 1) void k_step_tile_pair(const uint64_t *__restrict__ in,
                                                            uint64_t *__restrict__ out, StepArgs a,
                                                            int turns, int ntx, int ntiles)
{
    const int npairs = (ntiles + 1) / 2;
    const int pair = tile_of_block(npairs);
    if (pair >= npairs) return;                          // the whole workgroup
    const int tA = 2 * pair, tB = 2 * pair + 1 < ntiles ? 2 * pair + 1 : 2 * pair;
    tile_pass_pair<SEG>(in, out, a, turns, tA, tB, 2 * pair + 1 < ntiles, ntx);
}

// K1p k_tile_persist: `turns` turns in blocks of K on tiles that stay resident for the whole
// launch (small boards: every tile is one resident workgroup, checked by the host).  A block
// is one tile_pass; between blocks a tile exchanges its borders with its 8 neighbours through
// memory instead of ending the launch: block b reads buffer u[(b-1) % 2] (block 0: `in`) and
// writes u[b % 2] (the last block: `out`); u0 / u1 are uncached (visible across the XCDs' L2s
// without cache maintenance, like the k_step_wg parallelogram rows) and read with sc1 loads
// that bypass the CU's vector L1.  flags[tile] = epoch + b
// + 1 once the tile's block-b stores completed; a tile starts block b when its 8 neighbours
// are there -- which also means they finished reading the buffer it is about to overwrite.
// A wait that gives up after kTileSpinLimit polls marks the error word (GOL_EHIP at the next
// synchronising call) and goes on with a wrong board rather than hang.
template <int SEG, int ORD, int W>
__global__ __launch_bounds__(1024, 1) void k_tile_persist(
    const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t *u0, uint64_t *u1,
    StepArgs a, int turns, int K, int ntx, int ntiles, unsigned *flags, unsigned epoch)
{
    const int tile = tile_of_block(ntiles);
    if (tile >= ntiles) return;                          // (never waited for)
    const int nty = ntiles / ntx, ty = tile / ntx, tx = tile - ty * ntx;
    // ceil(turns / K) blocks of near-equal depth (<= K): 1000 turns at K = 32 run as
    // 8 x 32 + 24 x 31, not 31 x 32 + 8
    const int nblocks = (turns + K - 1) / K, base = turns / nblocks, extra = turns % nblocks;
    bool gave_up = false;
    for (int b = 0; b < nblocks; ++b) {
        const int k = base + (b < extra ? 1 : 0);
        if (b > 0) {
            if (threadIdx.x < 8) {                        // one neighbour per lane 0..7
                const int j = (int)threadIdx.x + (threadIdx.x >= 4 ? 1 : 0);   // skip (0, 0)
                const int dy = j / 3 - 1, dx = j % 3 - 1;
                const int ny = (ty + dy + nty) % nty, nx = (tx + dx + ntx) % ntx;
                const unsigned want = epoch + (unsigned)b;
                unsigned *f = flags + ny * ntx + nx;
                bool seen = false;
                for (int spin = 0; !seen && spin < GOL_TILE_SPIN_LIMIT; ++spin) {
                    const unsigned v =
                        __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    seen = (int)(v - want) >= 0;
                    if (!seen) __builtin_amdgcn_s_sleep(2);
                }
                gave_up |= !seen;
            }
            // (the loads of the block stay below the waits: the barrier and the fence)
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            __syncthreads();
        }
        const uint64_t *src = b == 0 ? in : ((b & 1) ? u0 : u1);
        uint64_t *dst = b + 1 == nblocks ? out : ((b & 1) ? u1 : u0);
        tile_pass<SEG, ORD, W, true>(src, dst, a, k, tile, ntx);
        if (b + 1 == nblocks) break;
        __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));   // this wave's stores are done
        __syncthreads();                                     // ... and every wave's
        // (u0 / u1 are uncached: completed stores are in memory; the flag is an agent-scope
        // store, a workgroup-scope release would order nothing across CUs)
        if (threadIdx.x == 0)
            __hip_atomic_store(flags + tile, epoch + (unsigned)b + 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (gave_up && a.err)
        __hip_atomic_store(a.err, kDevErrTileFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}


// K1r k_tile_ring: K1p's resident tiles without the round trip of the whole tile -- between
// blocks a tile stores and reloads only its ring (tile_pass RING).  Small torus boards: every
// tile one resident workgroup (host-checked: a wait for a tile that never runs gives up after
// GOL_TILE_SPIN_LIMIT polls and marks the error word).  u0 / u1: uncached board-layout buffers.
template <int SEG, int ORD>
__global__ __launch_bounds__(1024, 1) void k_tile_ring(
    const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t *u0, uint64_t *u1,
    StepArgs a, int turns, int K, int ntx, int ntiles, unsigned *flags, unsigned epoch,
    unsigned *gcount, unsigned gbase, int ablate)
{
    const int tile = tile_of_block(ntiles);
    if (tile >= ntiles) return;                          // (never waited for)
    tile_pass<SEG, ORD, 1, true, true>(in, out, a, K, tile, ntx,
                                       RingArgs{u0, u1, flags, epoch, turns, gcount, gbase, ablate});
}

// K1q k_tile_stream: K1p's blocks for boards whose tiles do not all fit at once.  One launch
// runs `turns` turns as blocks of <= K turns; the (block, tile) items are taken in order from
// a device counter by a grid of resident workgroups, so one launch has one start and one tail
// instead of one per K turns (a K1t launch costs ~55 us besides its turns at 65536^2).  Item
// i = b * ntiles + j is tile row (j / ntx + 2 b) mod nty, column j % ntx of block b: every
// item of block b is taken before any of block b + 1, and an item waits only for its 8
// neighbours' block b - 1 (flags as K1p: epoch + b once a tile's block-b stores completed),
// and on its own block b - 1 (it ran on another workgroup), all taken earlier and so running
// or done -- no deadlock whatever the residency.
// Rotating the tile rows by 2 per block puts the first items of a block on rows whose
// neighbours were among the first of the block before (the torus wrap would otherwise make
// the first row wait for the previous block's last).  Block b reads u[(b-1) % 2] (block 0:
// `in`) and writes u[b % 2] (the last block: `out`), as K1p.  counter counts across
// launches: each workgroup takes one item past the end before it leaves, so a launch
// advances it by items + grid; `base` is its value at the launch (unsigned wrap).
// (the item loop holds registers across items: bound them to k_step_tile's budget -- 80
// VGPRs at SEG 24, 6 waves per SIMD; 64 below, 8)
template <int SEG, int ORD, int W>
__global__ __launch_bounds__(1024, (SEG >= 20 ? 6 : 8)) void k_tile_stream(
    const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t *u0, uint64_t *u1,
    StepArgs a, int turns, int K, int ntx, int ntiles, unsigned *flags, unsigned epoch,
    unsigned *counter, unsigned base)
{
    __shared__ unsigned next_item;
    const int nty = ntiles / ntx;
    const int nblocks = (turns + K - 1) / K, kbase = turns / nblocks, extra = turns % nblocks;
    const unsigned nitems = (unsigned)nblocks * (unsigned)ntiles;
    bool gave_up = false;
    if (threadIdx.x == 0)
        next_item = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - base;
    __syncthreads();
    for (;;) {
        const unsigned item = next_item;
        __syncthreads();                                  // (everyone has read next_item)
        if (item >= nitems) break;                        // (workgroup-uniform)
        // the next item's fetch overlaps this one (its latency is a memory round trip, in
        // flight with the tile loads); thread 0 hands it over at the end of the item
        unsigned nxt = 0;
        if (threadIdx.x == 0)
            nxt = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - base;
        const int b = (int)(item / (unsigned)ntiles), j = (int)(item % (unsigned)ntiles);
        const int ty = (j / ntx + 2 * b) % nty, tx = j % ntx;
        const int tile = ty * ntx + tx;
        const int k = kbase + (b < extra ? 1 : 0);
        if (b > 0) {
            // the 8 neighbours AND the tile itself: unlike K1p, the tile's own block b - 1 ran
            // on some other workgroup, which may still be reading the buffer this item is about
            // to overwrite, and wrote the interior this item reads
            if (threadIdx.x < 9) {                        // one tile per lane 0..8
                const int jj = (int)threadIdx.x;
                const int dy = jj / 3 - 1, dx = jj % 3 - 1;
                const int ny = (ty + dy + nty) % nty, nx = (tx + dx + ntx) % ntx;
                const unsigned want = epoch + (unsigned)b;
                unsigned *f = flags + ny * ntx + nx;
                bool seen = false;
                for (int spin = 0; !seen && spin < GOL_TILE_SPIN_LIMIT; ++spin) {
                    const unsigned v =
                        __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    seen = (int)(v - want) >= 0;
                    if (!seen) __builtin_amdgcn_s_sleep(2);
                }
                gave_up |= !seen;
            }
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            // cached block buffers (MI355X_MICROARCH, inter-workgroup visibility, consumer
            // form): one agent acquire in the polling wave, its wait, then the barrier
            if (threadIdx.x < 64) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
        }
        const uint64_t *src = b == 0 ? in : ((b & 1) ? u0 : u1);
        uint64_t *dst = b + 1 == nblocks ? out : ((b & 1) ? u1 : u0);
        // (the shape's scalars pass through an empty asm every item, so the lane constants
        // tile_pass derives from them are recomputed per item rather than hoisted out of the
        // loop and held in VGPRs across it: that spilled at SEG 24)
        StepArgs aa = a;
        asm volatile("" : "+s"(aa.tile_w), "+s"(aa.band), "+s"(aa.nw), "+s"(aa.pitch),
                     "+s"(aa.modrows));
        tile_pass<SEG, ORD, W, true>(src, dst, aa, k, tile, ntx);
        if (b + 1 < nblocks) {
            __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));   // this wave's stores are done
            __syncthreads();                                     // ... and every wave's
            // (producer form: lane 0 writes the XCD L2's dirty lines back, waits, then flags)
            if (threadIdx.x == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(flags + tile, epoch + (unsigned)b + 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (threadIdx.x == 0) next_item = nxt;
        __syncthreads();                                  // (and the LDS slots are free again)
    }
    if (gave_up && a.err)
        __hip_atomic_store(a.err, kDevErrTileFlag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace golk
