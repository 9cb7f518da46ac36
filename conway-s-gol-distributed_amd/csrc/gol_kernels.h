// Internal launch interface of the gfx950 kernels (gol_kernels.hip).
// Not part of the C ABI; the engine (gol_engine.cpp) is the only caller.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace golk {

constexpr int kShards = 64;            // popcount accumulator shards (one 512-B line)
constexpr int kTileWords = 128;        // fast stencil: words per wavefront tile (64 lanes x 2)

// One turn over rows [row_lo, row_hi) of a buffer of `modrows` rows (row index
// wraps mod modrows: torus engines; strip engines never reach the wrap).
struct StepArgs {
    const uint64_t *in;
    uint64_t *out;
    const uint64_t *blocked;           // non-binary mask (turn 1 only) or nullptr
    unsigned long long *counts;        // kShards accumulators or nullptr
    int width;                         // cells per row
    int nw;                            // words per row
    int pitch;                         // row stride in words
    int modrows;
    int row_lo, row_hi;
    int cnt_lo, cnt_hi;                // rows whose outputs are counted
    int band;                          // rows per wavefront (fast) / per thread (generic)
    int variant;                       // fast-path kernel variant (kVariant*)
    int multi_words;                   // k_step_multi words per lane (1 or 2)
    int multi_variant;                 // temporal-blocking kernel (kMulti*)
    // kMultiWgPg: boundary rows published between neighbouring bands (engine-owned, uncached)
    uint64_t *xrows;                   // 2 rows per stage, kPgStages stages, xlanes words each
    unsigned *xflags;                  // per (tile, stage): epoch of its last publication
    unsigned xlanes;                   // virtual lanes per published row
    unsigned epoch;                    // this launch's epoch (above every earlier launch's)
    // k_step_wg wave priorities (4-wave workgroups): wave w runs at s_setprio
    // (wg_prio >> 2w) & 3; 0 = the built-in grading
    unsigned wg_prio;
    // engine-owned error word (host-mapped pinned memory, or nullptr): a k_step_wg wait that
    // gives up stores a kDevErr* code here, and the engine reports it as GOL_EHIP at its next
    // synchronising call instead of returning a corrupt board with GOL_OK
    unsigned *err;
    // k_step_tile (kMultiTile): tile width in words (the tile height is `band`) and rows per
    // lane segment
    int tile_w;
    int tile_seg;
};

// device error codes (StepArgs::err)
constexpr unsigned kDevErrHandoff = 1u;    // k_step_wg: LDS hand-off wait timed out
constexpr unsigned kDevErrPgFlag = 2u;     // k_step_wg parallelogram: flag wait timed out
constexpr unsigned kDevErrTileFlag = 3u;   // k_tile_persist: a neighbour tile's flag wait timed out

// temporal-blocking kernels (A/B-able via GOL_MULTI_VARIANT; kMultiSkewILW16 is shipped)
enum : int {
    kMultiSerial = 0,       // k_step_multi: stages chained within a step
    kMultiSkew = 1,         // k_step_skew: stages one step apart, LDS-DMA prefetch of 8 rows,
                            //   4 waves/SIMD (V = 1, K < 8; 3 at K = 8), 7-op rule
    kMultiSkewPD5 = 2,      // k_step_skew, 5 rows in flight, no wave floor (V = 1, K = 6/8 only)
    kMultiSkewW1 = 3,       // k_step_skew, no wave floor                   (V = 1, K = 6/8 only)
    kMultiSkewRule8 = 4,    // k_step_skew with the 8-op rule               (V = 1, K = 6/8 only)
    kMultiSkewD1 = 5,       // k_step_skew, 1 dword (32 cells) per lane     (V = 1, K = 4/6/8 only)
    kMultiSkewIL = 6,       // k_step_skew on the interleaved board layout (V = 1)
    kMultiSkewILW16 = 7,    // kMultiSkewIL, one 16-B row DMA from half the lanes (V = 1; default)
    kMultiWg = 8,           // k_step_wg: one band's stages split over the 4 waves of a workgroup
                            //   (interleaved layout, V = 1, K = 4..16; K = 2, 3: kMultiSkewILW16)
    kMultiWgHx = 9,         // k_step_wg on helix tiles: the row bands end to end, cut every 62
                            //   lanes (no per-row remainder tile; needs nw even)
    kMultiWgNoBar = 10,     // k_step_wg without hand-off sync: timing ablation (wrong results)
    kMultiWgDiag = 11,      // k_step_wg with per-wave wait timing (tools/wg_diag.py)
    kMultiWgPg = 12,        // kMultiWgHx with parallelogram bands: a band's stages take their
                            //   last 2 input rows from the band below (published through
                            //   memory) instead of recomputing a 2K-row halo (band >= kPgMinBand)
    kMultiWgHxS = 13,       // kMultiWgHx with each wave's stages in order within a step (fill
                            //   and drain of 2 instead of 3 steps per stage)
    kMultiWgPgS = 14,       // kMultiWgPg, stages in order (band rule: golk::pg_ok(.., true))
    kMultiTile = 15,        // k_step_tile: a 2-D tile per workgroup, resident in registers for
                            //   all K turns (small boards: gol_tile.h)
    kMultiUserEnd = 16,     // variants 0 .. kMultiUserEnd - 1 may be requested (GOL_MULTI_VARIANT);
                            //   the ids from here on are engine-internal launch kinds
    kMultiTilePersist = 16, // K1p k_tile_persist: k_step_tile's tiles resident across blocks of
                            //   K turns (engine-internal; tools build only)
    kMultiTileStream = 17,  // K1q k_tile_stream: blocks of K turns over (block, tile) items taken
                            //   in order by resident workgroups (engine-internal; tools build only)
    kMultiInternalEnd = 18, // one past the engine-internal launch kinds (size of any table by kind)
    kMultiAblate = 100,     // 100 + ABL mask: k_step_skew<8> timing ablations (K = 8 only)
};

static_assert(kMultiTile < kMultiUserEnd && kMultiWgPgS < kMultiUserEnd,
              "every requestable variant lies below the engine-internal launch kinds");
static_assert(kMultiTilePersist >= kMultiUserEnd && kMultiTileStream < kMultiInternalEnd &&
              kMultiInternalEnd < kMultiAblate, "engine-internal kinds between the two ranges");

#ifndef GOL_TOOLS
#define GOL_TOOLS 0   // 1: the tools build (libgolamd_tools.so, see the Makefile)
#endif

// the kernels the product library ships (gol_create_ex rejects the others unless GOL_TOOLS):
// k_step_skew on the interleaved layout with 16-B row DMA, the k_step_wg families and the
// LDS tile kernel.  The superseded skew variants (kMultiSerial .. kMultiSkewIL), the timing
// ablations and the wait diagnostics exist in the tools build only.
constexpr bool multi_variant_shipped(int v)
{
    return v == kMultiSkewILW16 || v == kMultiWg || v == kMultiWgHx || v == kMultiWgPg ||
           v == kMultiWgHxS || v == kMultiWgPgS || v == kMultiTile;
}

// the k_step_wg variants (one band pipeline per workgroup)
constexpr bool is_wg_variant(int v)
{
    return v == kMultiWg || v == kMultiWgHx || v == kMultiWgPg || v == kMultiWgNoBar ||
           v == kMultiWgDiag || v == kMultiWgHxS || v == kMultiWgPgS;
}

// fast-path stencil variants (A/B-able in one process; kVariantDefault is shipped)
enum : int {
    kVariantWindow = 0,     // k_step_fast: 3-row window, 1 row in flight
    kVariantRing2 = 1,      // k_step_ring<D=2>
    kVariantRing3 = 2,      // k_step_ring<D=3>
    kVariantRing3NT = 3,    // k_step_ring<D=3>, non-temporal stores
    kVariantRing5 = 4,      // k_step_ring<D=5>
    kVariantRing7 = 5,      // k_step_ring<D=7>
    kVariantRing5NT = 6,    // k_step_ring<D=5>, non-temporal stores
    kVariantCount = 7,
};
extern const int kVariantDefault;

bool fast_path_ok(int width);

// K turns per launch (temporal blocking): outputs rows [row_lo, row_hi) after `turns`
// turns, reading rows [row_lo - turns, row_hi + turns) (mod modrows).  No blocked mask,
// no counts.  turns in 2 .. multi_max_turns(variant).
constexpr int kMaxTurnsPerLaunch = 32;
// k_step_tile alone goes deeper: its halo word (64 cells) and K halo rows stay exact up to 64
// turns (the planner's per-depth tables stop at kMaxTurnsPerLaunch; deeper K1t launches are
// pinned or requested, never searched)
constexpr int kMaxTileTurns = 64;
// 32 for the helix k_step_wg variants, 16 for band-tiled k_step_wg, 8..12 for k_step_skew
int multi_max_turns(int variant);
// k_step_wg on helix tiles: wavefronts per workgroup at depth `turns` -- 4 up to K = 16, then
// one more per 4 stages (K = 17..32: 5..8 waves of at most 4 stages, <= 72 VGPRs each)
constexpr int wg_waves(int turns) { return turns <= 16 ? 4 : (turns + 3) / 4; }
constexpr int kWgDeepMax = 32;
// band height of the boundary launches of an overlapped step (rows next to the halos)
constexpr int kOverlapBand = 16;
// kMultiWgPg: stages per tile in the flag array, smallest band; it runs at depths K = 4, 8,
// 12, 16 (every wave the same stage count) with band = 3K/4 - 5 (mod kWgU) (its steady loop
// then ends on a whole unrolled iteration); other launches run as kMultiWgHx
constexpr int kPgStages = 16;
constexpr int kPgMinBand = 32;
// k_step_wg's steady-loop unroll (its LDS ring slots are immediates) and wave 0's input rows
// in flight (LDS-DMA ring of kWgDmaRows + 1 slots; kWgU a multiple of 3, of that and of 6).
// 11 rows in flight (unroll 12) measured no faster than 5 at 65536^2, K = 4..16 (the launch
// is not bound by the head's DMA latency) and cost PG 8-11 VGPRs: 5 / 6 stay.
constexpr int kWgDmaRows = 5;
constexpr int kWgU = 6;
// (ser: kMultiWgPgS, prologue 2G - 2 steps instead of 3G - 3, G = turns / 4)
constexpr bool pg_ok(int turns, int band, bool ser = false)
{
    return turns % 4 == 0 && turns <= kPgStages && band >= kPgMinBand &&
           (band + 2 - (ser ? 2 : 3) * (turns / 4 - 1)) % kWgU == 0;
}
// the nearest band >= `band` kMultiWgPg / kMultiWgPgS runs at depth `turns` (0: none)
constexpr int pg_band(int turns, int band, bool ser = false)
{
    for (int b = band < kPgMinBand ? kPgMinBand : band; b < band + kWgU + kPgMinBand; ++b)
        if (pg_ok(turns, b, ser)) return b;
    return 0;
}
constexpr bool is_pg_variant(int v) { return v == kMultiWgPg || v == kMultiWgPgS; }
constexpr bool is_helix_variant(int v)
{
    return v == kMultiWgHx || v == kMultiWgPg || v == kMultiWgHxS || v == kMultiWgPgS;
}
bool multi_ok(int width, int turns, int variant);
// waves sharing one band pipeline at depth `turns` (k_step_wg: wg_waves, else 1)
int multi_waves_per_band(int variant, int turns);
// band pipelines per thread block (k_step_skew: 4 single-wave pipelines; k_step_wg: 1)
int multi_pipes_per_block(int variant);
bool multi_fits(int nw, int pitch, int rows);   // buffer < 2 GiB (k_step_skew buffer ranges)
// the temporal-blocking kernel for (words per lane, variant) runs on the interleaved layout
bool multi_is_il(int words_per_lane, int variant);
// standard <-> interleaved rows (row pitches in words; in and out may not alias)
hipError_t launch_il_convert(const uint64_t *in, int in_pitch, uint64_t *out, int out_pitch,
                             int nrows, int nw, bool to_il, hipStream_t s);
// dwords per lane of the temporal-blocking kernel (tiles advance by 62 x that many dwords)
int multi_lane_dwords(int words_per_lane, int variant);
// wavefront tiles per row band of the temporal-blocking kernel
long long multi_tiles(int width, int lane_dwords);
// band pipelines of one launch over `rows` rows in bands of `band` (workgroups for the
// k_step_wg variants, wavefronts for k_step_skew): tiles x bands, or the helix tile count
long long multi_pipes(int width, int rows, int band, int lane_dwords, int variant);
int auto_band_multi(int width, int rows, int lane_dwords);
// resident 256-thread blocks per CU of the temporal-blocking kernel (0 on error)
int multi_blocks_per_cu(int turns, int words_per_lane, int variant);
// band height minimising (residency rounds x per-wavefront work) for the multi kernel
int pick_band_multi(int width, int rows, int lane_dwords, int turns, int capacity_waves,
                    int variant);
hipError_t launch_step_multi(const StepArgs &a, int turns, hipStream_t s);
// k_step_tile (gol_tile.hip): a launch of `turns` turns on tiles of band x tile_w words with
// tile_seg rows per lane; shape check, workgroup waves, tile count
constexpr int kTileMaxWavesHost = 16;  // k_step_tile: waves per workgroup (gol_tile.h)
// The k_step_tile segment codes (SEG + 100 * ORD + 1000 * (W - 1), gol_tile.h) the product
// library runs: every code the engine's shape searches can pick (tile_candidates, tile_search)
// and nothing else.  Each one is pinned by its own oracle parity test
// (tests/test_gpu_engine.py::test_tile_code_pinned, read through gol_tile_codes), and
// tile_shape_ok rejects the others outside the tools build.
constexpr int kTileCodes[] = {
    2,    3,    4,    6,    8,    12,   16,   24,   32,   40,   48,             // ORD 0, W 1
    102,  103,  104,  106,  108,  112,  116,  124,  132,  140,                  // ORD 1
    203,  204,  206,  208,  212,  216,  224,  232,  240,                        // ORD 2
    403,  404,  406,  408,  412,  416,  424,  432,  440,                        // ORD 4
    503,  504,  506,  508,  512,  516,  524,  532,  540,                        // ORD 5
    612,  616,  624,                                                            // ORD 6
    1002, 1003, 1004, 1006, 1008,                                               // W 2
    1102, 1103, 1104, 1106, 1108,
    1204, 1206, 1208,
};
// the codes k_tile_persist (K1p) is instantiated for in the tools build (gol_tile.hip
// persist_fn; each pinned by tests/test_gpu_engine.py::test_tile_persist_pinned through
// gol_tile_persist_codes, which reports none in the product library: K1p never won its
// autotune and its uncached hand-off shares K1q's unexplained wrong-board runs)
constexpr int kTilePersistCodes[] = {102, 103, 104, 106, 108, 112, 116,
                                     403, 404, 406, 408, 412, 416,
                                     2, 3, 4, 6, 8,
                                     503, 504, 506, 508};
// the codes k_tile_stream (K1q) is instantiated for (gol_tile.hip stream_fn; each pinned by
// tests/test_gpu_engine.py::test_tile_stream_pinned through gol_tile_stream_codes)
constexpr int kTileStreamCodes[] = {106, 506, 512, 524};
// the codes k_tile_ring (K1r) is instantiated for in the tools build (gol_tile.hip ring_fn)
constexpr int kTileRingCodes[] = {103, 203, 503, 504, 506, 508, 512, 516, 112, 116};
constexpr bool tile_code_shipped(int code)
{
    for (int c : kTileCodes)
        if (c == code) return true;
    return false;
}
bool tile_shape_ok(int nw, int turns, int tile_h, int tile_w, int seg);
int tile_waves(int turns, int tile_h, int tile_w, int seg);
// resident workgroups per CU of that launch (occupancy API: VGPRs, LDS; 0 on error)
int tile_blocks_per_cu(int turns, int tile_h, int tile_w, int seg);
long long tile_count(int nw, int rows, int tile_h, int tile_w, int seg);
hipError_t launch_tile(const StepArgs &a, int turns, hipStream_t s);
// K1p k_tile_persist (gol_tile.h): `turns` turns in blocks of K on tiles resident for the whole
// launch, exchanging borders between blocks through u0 / u1 (uncached, board-sized) and
// per-tile flags (uncached, one per tile; epoch above every earlier launch's flags).
// tile_persist_ok: an instantiated code, K within the tile rows, every tile resident at once.
bool tile_persist_ok(int nw, int rows, int turns, int K, int tile_h, int tile_w, int seg, int ncu);
hipError_t launch_tile_persist(const StepArgs &a, int turns, int K, uint64_t *u0, uint64_t *u1,
                               unsigned *flags, unsigned epoch, hipStream_t s);
// K1q k_tile_stream (gol_tile.h): `turns` turns in blocks of K over (block, tile) items taken
// from *counter (value `base` at the launch) by min(items, CUs x occupancy, max_grid if > 0)
// workgroups, whose count goes to *grid (the counter advances by items + grid).  Same u0 / u1 / flags contract
// as K1p; tile_stream_ok: an instantiated code and K within the tile rows (no residency need).
bool tile_stream_ok(int nw, int rows, int K, int tile_h, int tile_w, int seg);
hipError_t launch_tile_stream(const StepArgs &a, int turns, int K, uint64_t *u0, uint64_t *u1,
                              unsigned *flags, unsigned epoch, unsigned *counter, unsigned base,
                              int ncu, int max_grid, unsigned *grid, hipStream_t s);
// K1r k_tile_ring (gol_tile.h): K1p's contract (flags, epoch) with the tiles kept in registers
// across blocks; only their rings pass through u0 / u1 (uncached, board-sized).
bool tile_ring_ok(int nw, int rows, int K, int tile_h, int tile_w, int seg, int ncu);
// gcount (tools experiments, else nullptr): a grid-wide barrier per block on that counter,
// whose value at the launch is gbase (it advances by tiles x (blocks - 1))
hipError_t launch_tile_ring(const StepArgs &a, int turns, int K, uint64_t *u0, uint64_t *u1,
                            unsigned *flags, unsigned epoch, unsigned *gcount, unsigned gbase,
                            hipStream_t s);
int auto_band(int width, int rows);
hipError_t launch_step(const StepArgs &a, bool fast, hipStream_t s);

// Popcount of rows [row_lo, row_hi) into kShards accumulators (caller zeroes).
hipError_t launch_popcount(const uint64_t *w, int nw, int pitch, int row_lo, int row_hi,
                           unsigned long long *counts, hipStream_t s);

// bytes (nrows x width, row-major, device) -> words rows [row0, row0+nrows).
// blocked (nullable) gets the non-binary mask; nonbin accumulates its popcount.
hipError_t launch_pack(const uint8_t *bytes, int width, int nrows, uint64_t *words,
                       uint64_t *blocked, int nw, int pitch, int row0,
                       unsigned long long *nonbin, hipStream_t s);
// words rows [row0, row0+nrows) -> bytes (nrows x width, 0/255)
hipError_t launch_unpack(const uint64_t *words, int width, int nw, int pitch, int row0,
                         int nrows, uint8_t *bytes, hipStream_t s);

// Random board: buffer row b is global row (grow0 + b) mod gheight.
hipError_t launch_fill_random(uint64_t *words, int width, int nw, int pitch, int nrows,
                              long long grow0, int gheight, uint64_t seed, hipStream_t s);

// Alive list: per-row popcounts, then a row-major scatter of {x, y} int64 pairs.
hipError_t launch_row_popcount(const uint64_t *w, int nw, int pitch, int row0, int nrows,
                               long long *row_counts, hipStream_t s);
hipError_t launch_alive_scatter(const uint64_t *w, int nw, int pitch, int row0, int nrows,
                                long long grow0, const long long *row_offsets,
                                long long *xy, hipStream_t s);

}  // namespace golk
