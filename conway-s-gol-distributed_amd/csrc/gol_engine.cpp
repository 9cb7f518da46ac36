// gol_engine.cpp — the per-GPU engine behind include/gol_amd.h.
//
// One gol_ctx = one MI355X holding either the whole torus board or one row
// strip of it (the reference's SubServer strip, Server/gol/distributor.go:
// 106-116 split; here the strip lives on the GPU for the whole run and only
// `halo` boundary rows move between strips every `halo` turns).
//
// Device memory per engine (owned here, freed in gol_destroy):
//   board[2]   double-buffered packed board, buffer_rows x pitch uint64
//   blocked    packed mask of the cells that were neither 0 nor 255 at load
//              (only while turn 1 is pending; reference quirk,
//              SubServer/distributor.go:178-200 + :122-125)
//   counts     popcount shards (kShards u64) x kRing slots for the per-turn
//              series (GOL_FLAG_COUNT_EVERY_TURN) and one slot for snapshots
//   staging    byte / alive-list staging, allocated on demand
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <iterator>
#include <map>
#include <tuple>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "gol_amd.h"
#include "gol_kernels.h"
#include "gol_internal.h"

using golk::kShards;

namespace {

constexpr int kRing = 4096;                 // per-turn count ring (turn t -> slot t % kRing)
constexpr size_t kStagingBytes = 256u << 20;  // byte staging chunk for load / read

}  // namespace

// one temporal-blocking launch: depth, kernel (golk::kMulti*), band, and for k_step_tile the
// tile width and segment code it was timed at (a plan may hold a tile family other than the
// engine's own pick: each launch carries its shape)
struct Launch {
    int k = 0, var = 0, band = 0;
    int tw = 0, seg = 0;
    int blk = 0;                             // kMultiTilePersist: turns per block
};
constexpr int kPlanMax = 128;               // launch plans cover gol_step / halo windows up to this
constexpr int kSeqMax = 32;                 // gol_step calls this short run a timed sequence
constexpr size_t kLastCap = 4096;           // gol_last_launches records at most this many

// a read-only call (gol_snapshot, gol_read_*, ...) run by a stepping thread at a launch boundary
struct Job {
    std::function<int()> fn;
    int rc = 0;
    bool done = false;
};

struct gol_ctx {
    gol_config cfg{};
    int device = 0;
    int nw = 0, pitch = 0, buf_rows = 0;
    bool fast = false;
    int band = 8;
    int variant = golk::kVariantDefault;
    int tpl = 1;                             // turns per stencil launch (temporal blocking)
    int multi_words = 2;                     // k_step_multi words per lane
    unsigned wg_prio = 0;                    // k_step_wg priority override (GOL_WG_PRIO, tools)
    int multi_variant = golk::kMultiSkewILW16;  // temporal-blocking kernel (kMulti*)
    int band_multi = 64;                     // band height of the multi-turn kernel (depth tpl)
    int band_at[golk::kMaxTurnsPerLaunch + 1] = {};   // band_for_depth cache (0 = not yet)
    // a pinned k_step_tile shape's tile height for launches of depth <= short_k (0: none): a
    // short step's one shallow launch takes the taller tile its depth allows
    int short_k = 0, short_band = 0;
    // launch planner (autotuned engines): plan[t] = the first launch of the fastest measured
    // sequence of launches for t turns (t <= kPlanMax; k = 0: no plan, use the even split)
    std::vector<Launch> plan;
    // seq[r] (r <= kSeqMax, torus engines): the launch sequence of a gol_step of exactly r
    // turns, chosen by timing whole candidate sequences the way gol_step runs them (empty:
    // follow `plan`)
    std::vector<std::vector<Launch>> seq;
    std::vector<Launch> last;                // launches of the last gol_step (gol_last_launches)
    long long last_n = 0;
    int ncu = 0;                             // compute units of the device
    float tuned_us_per_turn = 0.f;           // autotune's best measurement (0 = not tuned)
    int shape_source = 0;                    // gol_info.shape_source: 1 = searched, 2 = kKnownShapes
    uint64_t *board[2] = {nullptr, nullptr};
    int cur = 0;
    bool il = false;                         // board[cur] is in the interleaved layout
    uint64_t *blocked = nullptr;
    bool blocked_pending = false;
    long long nonbinary = 0;
    std::vector<uint8_t> raw_turn0;          // loaded bytes, kept only while non-binary & turn == 0
    unsigned long long *counts = nullptr;    // (kRing + 1) * kShards
    unsigned long long *h_counts = nullptr;  // pinned mirror of one slot
    uint8_t *staging = nullptr;
    size_t staging_size = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;              // boundary-band launches of gol_step_overlap
    hipEvent_t ev_side = nullptr, ev_main = nullptr;
    long long turn = 0;
    long long launches = 0;
    int halo_valid = 0;
    bool blocking_limited = false;           // temporal blocking off: buffer >= 2 GiB
    // kMultiWgPg: published boundary rows and per-(tile, stage) flags (uncached, grow-only)
    uint64_t *pg_rows = nullptr;
    unsigned *pg_flags = nullptr;
    size_t pg_lanes = 0, pg_tiles = 0;
    unsigned pg_epoch = 0;
    // control word (gol_set_control): read by gol_step between launches, written by any
    // thread without the engine lock (the reference's CFput flag channel)
    std::atomic<int> control{GOL_CONTROL_RUN};
    std::atomic<bool> control_used{false};
    std::atomic<long long> progress{0};      // lock-free mirror of `turn` (gol_get_progress)
    std::atomic<bool> parked{false};         // gol_step is parked on GOL_CONTROL_PAUSE
    // k_step_tile shape (kMultiTile): tile width in words, rows per lane segment (the tile
    // height is the launch's band)
    int tile_w = 0, tile_seg = 0;
    // K1p (k_tile_persist, small torus boards): turns per block (0 = off), the uncached block
    // buffers and per-tile flags, and the flags' epoch (grows by blocks + 1 per launch)
    int persist_k = 0;
    int persist_seg = 0;                     // K1p's segment code (plain launches keep tile_seg)
    bool persist_forced = false;             // GOL_PERSIST (tests): also on a shared device
    bool persist_ring = false;               // GOL_RING (tools build): K1r instead of K1p
    uint64_t *pu[2] = {nullptr, nullptr};
    unsigned *pflags = nullptr;
    size_t pflags_n = 0;
    unsigned pepoch = 0;
    // K1q (k_tile_stream, large torus boards): turns per block (0 = off) and its tile shape;
    // the item counter (uncached) and its host mirror (the value the next launch starts from)
    int stream_k = 0;
    bool stream_forced = false;              // GOL_STREAM (tests): also on a shared device
    int stream_tw = 0, stream_th = 0, stream_seg = 0;
    unsigned *pcounter = nullptr;
    unsigned pcount = 0;
    uint64_t *su[2] = {nullptr, nullptr};     // K1q block buffers (cached: hipMalloc)
    // device error word (host-mapped pinned memory; golk::kDevErr*): a k_step_wg wait that gave
    // up writes it, every synchronising call checks it
    unsigned *h_err = nullptr, *d_err = nullptr;
    bool registered = false;                 // counted in g_dev_engines
    hipEvent_t ev_copy = nullptr;            // gol_copy_halo_from_*: ordering between engines
    std::string err;
    std::recursive_mutex mu;                 // engine state; held by gol_step except while parked
    // read-only calls from other threads while gol_step runs (run_read): served by the stepping
    // thread at its next launch boundary
    std::mutex jm;
    std::condition_variable jcv;
    std::vector<Job *> jobs;
    bool stepping = false;                   // (under jm) a gol_step holds `mu`
    std::atomic<bool> jobs_pending{false};
    std::atomic<bool> readers{false};        // a reader was served during a step: keep the queue short
};

namespace {

int fail(gol_ctx *c, int code, const char *fmt, ...)
{
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return code;
}

#define HIP_OR_FAIL(c, expr)                                                                   \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail((c), e_ == hipErrorOutOfMemory ? GOL_ENOMEM : GOL_EHIP, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(e_), __FILE__, __LINE__);                     \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        int now = -1;
        if (prev >= 0 && hipGetDevice(&now) == hipSuccess && now != prev) (void)hipSetDevice(prev);
    }
};

// engines alive per device in this process: kMultiWgPg runs only on a device with one engine
// (two concurrent parallelogram grids can each fill an XCD with tiles waiting for tiles of
// their own launch that sit undispatched behind the other grid's: the waits would time out),
// and not at all when GOL_SHARED_DEVICE is set (other processes share the GPU: torchrun ranks
// on one device).  The rows it would have published are recomputed as plain helix bands.
std::mutex g_dev_mu;
std::map<int, int> g_dev_engines;

// Create-time autotune results, per (device, width, buffer rows, requested depth, what was
// tuned): engines of one shape in one process -- the strips of a run, the engines a test suite
// or a sweep creates -- time their candidates once (GOL_AUTOTUNE_CACHE=0: always re-time).
struct TuneKey {
    int dev, width, rows, tpl_req, mode;
    bool operator<(const TuneKey &o) const
    {
        return std::tie(dev, width, rows, tpl_req, mode) <
               std::tie(o.dev, o.width, o.rows, o.tpl_req, o.mode);
    }
};
struct TuneVal {
    int var, tpl, band, tile_w, tile_seg, persist_k, persist_seg;
    int stream_k, stream_tw, stream_th, stream_seg;
    float us;
    std::vector<Launch> plan;
    std::vector<std::vector<Launch>> seq;
};
std::mutex g_tune_mu;
std::map<TuneKey, TuneVal> g_tune;

// Pinned shapes whose create-time check (check_pinned) has run in this process, per (device,
// width, buffer rows): later engines of the same shape -- the strips of a run, a bench's second
// measurement, a gol.Run after an Engine -- skip it (its ~60 ms of launches are a cost of the
// first engine only).
std::mutex g_pin_mu;
std::set<std::tuple<int, int, int>> g_pin_checked;

bool device_exclusive(int dev)
{
    static const bool shared = getenv("GOL_SHARED_DEVICE") && atoi(getenv("GOL_SHARED_DEVICE"));
    if (shared) return false;
    std::lock_guard<std::mutex> lk(g_dev_mu);
    auto it = g_dev_engines.find(dev);
    return it == g_dev_engines.end() || it->second <= 1;
}

bool is_strip(const gol_ctx *c) { return c->cfg.halo > 0; }

// The device error word after a synchronisation: a k_step_wg hand-off or parallelogram flag
// wait gave up (a preempted or starved workgroup), so the board of that launch is wrong.  The
// word stays set until the board is replaced (gol_load*, gol_fill_random): every synchronising
// call reports it (the reference ignored its RPC errors, Server/gol/distributor.go:219).
int check_dev_err(gol_ctx *c)
{
    const unsigned e = c->h_err ? *(volatile unsigned *)c->h_err : 0u;
    if (!e) return GOL_OK;
    return fail(c, GOL_EHIP,
                "a %s wait timed out (device error word %u): the board is corrupt; reload it",
                e == golk::kDevErrPgFlag     ? "k_step_wg parallelogram flag"
                : e == golk::kDevErrTileFlag ? "k_tile_persist neighbour-tile flag"
                                             : "k_step_wg hand-off",
                e);
}

int sync_checked(gol_ctx *c)
{
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    return check_dev_err(c);
}

void clear_dev_err(gol_ctx *c)
{
    if (c->h_err) *(volatile unsigned *)c->h_err = 0u;
}

// Serve the read-only calls posted by run_read (the stepping thread, holding `mu`).
void serve_jobs(gol_ctx *c)
{
    std::vector<Job *> js;
    {
        std::lock_guard<std::mutex> jl(c->jm);
        js.swap(c->jobs);
        c->jobs_pending.store(false);
    }
    for (Job *j : js) {
        const int rc = j->fn();
        std::lock_guard<std::mutex> jl(c->jm);
        j->rc = rc;
        j->done = true;                      // (j lives on the waiter's stack: not touched again)
    }
    if (!js.empty()) c->jcv.notify_all();
}

void set_stepping(gol_ctx *c, bool on)
{
    std::lock_guard<std::mutex> jl(c->jm);
    c->stepping = on;
}

// Run a read-only engine call.  No gol_step in progress: now, under the engine lock.  While
// another thread's gol_step runs: by that thread at its next launch boundary, on the board the
// step has enqueued so far (turn-consistent), so AliveCellsCount / GetWorld never wait for
// the whole step -- the reference's Alivecount and GetWorld take the Server mutex only around
// the per-turn commit (Server/gol/distributor.go:62-75,131-134).  While the step is parked on
// PAUSE it has released the engine, and the call runs now.
template <class F>
int run_read(gol_ctx *c, F &&fn)
{
    for (;;) {
        std::unique_lock<std::mutex> jl(c->jm);
        if (c->stepping) {
            Job j;
            j.fn = std::function<int()>(fn);
            c->jobs.push_back(&j);
            c->jobs_pending.store(true);
            c->readers.store(true);
            c->jcv.wait(jl, [&] { return j.done; });
            return j.rc;
        }
        if (c->mu.try_lock()) {              // (the owner of a recursive lock gets it too)
            jl.unlock();
            std::lock_guard<std::recursive_mutex> lk(c->mu, std::adopt_lock);
            return fn();
        }
        jl.unlock();                         // a short call holds the engine, or a step is
        std::this_thread::sleep_for(std::chrono::microseconds(50));   // about to flag itself
    }
}

// rows of the owned region inside the buffer
int own_lo(const gol_ctx *c) { return c->cfg.halo; }
int own_hi(const gol_ctx *c) { return c->cfg.halo + c->cfg.rows; }

int ensure_staging(gol_ctx *c, size_t bytes)
{
    if (c->staging_size >= bytes) return GOL_OK;
    if (c->staging) (void)hipFree(c->staging);
    c->staging = nullptr;
    c->staging_size = 0;
    HIP_OR_FAIL(c, hipMalloc(&c->staging, bytes));
    c->staging_size = bytes;
    return GOL_OK;
}

void release_blocked(gol_ctx *c)
{
    if (c->blocked) (void)hipFree(c->blocked);
    c->blocked = nullptr;
    c->blocked_pending = false;
}

// The temporal-blocking kernel runs on the interleaved word layout (gol_kernels.h,
// multi_is_il); everything else -- the k = 1 stencils, PGM pack/unpack, the alive list,
// reads, loads, halo rows crossing the API -- sees the standard layout.  The engine
// converts lazily, whole buffer, when the next consumer needs the other layout (one read
// and one write of the board: at most twice per gol_step, never inside a run of
// multi-turn launches).  Popcounts do not depend on the layout.
int ensure_layout(gol_ctx *c, bool il)
{
    if (c->il == il) return GOL_OK;
    HIP_OR_FAIL(c, golk::launch_il_convert(c->board[c->cur], c->pitch, c->board[c->cur ^ 1],
                                           c->pitch, c->buf_rows, c->nw, il, c->stream));
    c->cur ^= 1;
    c->il = il;
    return GOL_OK;
}

// The band a kernel tuned at (K0, band0) runs at depth k.  A launch of another depth -- the
// even split's shallower launches, a short gol_step, the last block before a halo exchange,
// a planned launch -- runs a kernel with another residency (k_step_wg: 4..8 waves per
// workgroup at 7 or 8 waves per SIMD; k_step_skew: 2..4 waves per SIMD), where band0 would
// leave resident slots idle or spill a few pipelines into one more round (65536^2: K = 16's
// band 607 fills 1791 of 1792 slots; a K = 20 launch has 1280).  Keep the tuned number of
// rounds instead: the smallest band whose grid fits them at depth k (kMultiWgPg: the next
// band it runs at).
int band_same_rounds(const gol_ctx *c, int var, int K0, int band0, int k)
{
    if (k == K0 || k < 2 || k > golk::kMaxTurnsPerLaunch || var == golk::kMultiTile)
        return band0;                        // (k_step_tile: the tile height stays)
    const int lane_dw = golk::multi_lane_dwords(c->multi_words, var);
    const int per = golk::multi_pipes_per_block(var);
    const long long cap_t = (long long)c->ncu * golk::multi_blocks_per_cu(K0, c->multi_words, var) * per;
    const long long cap_k = (long long)c->ncu * golk::multi_blocks_per_cu(k, c->multi_words, var) * per;
    if (cap_t <= 0 || cap_k <= 0) return band0;
    const int W = c->cfg.width, rows = c->buf_rows;
    const long long pipes = golk::multi_pipes(W, rows, band0, lane_dw, var);
    const long long rounds = std::max(1ll, (pipes + cap_t - 1) / cap_t);
    int b = band0;
    for (int band = 16; band <= std::max(rows, 16); ++band)
        if (golk::multi_pipes(W, rows, band, lane_dw, var) <= rounds * cap_k) {
            b = band;
            break;
        }
    const bool ser = var == golk::kMultiWgPgS;
    if (golk::is_pg_variant(var) && golk::pg_ok(k, golk::pg_band(k, b, ser), ser))
        b = golk::pg_band(k, b, ser);
    return b;
}

// band_same_rounds for the engine's kernel and depth (cached); a band the caller fixed
// (gol_config.band_rows) is kept
int band_for_depth(gol_ctx *c, int k)
{
    if (c->short_k > 0 && c->multi_variant == golk::kMultiTile && c->cfg.band_rows <= 0 &&
        k >= 2 && k <= c->short_k)
        return c->short_band;
    if (k == c->tpl || c->cfg.band_rows > 0 || k < 2 || k > golk::kMaxTurnsPerLaunch)
        return c->band_multi;
    int &b = c->band_at[k];
    if (b <= 0) b = band_same_rounds(c, c->multi_variant, c->tpl, c->band_multi, k);
    return b;
}

// The next launch when `room` turns remain before the next sync point (end of the gol_step
// call, or the next halo exchange of a strip engine).  k = 1: the one-turn kernel.
//  * Autotuned engines follow the launch plan for room <= kPlanMax: the sequence of launches
//    (depth and kernel) the create-time timing table says is fastest.  A short launch costs
//    nearly as much as a full one and the kernels differ in that fixed cost (65536^2,
//    profiles/r02_launch_table_65536.log: k_step_skew 260 us at K = 6 and 384 at K = 10;
//    k_step_wg 413 us at K = 4, 459 at 12, 595 at 16), so 20 turns run best as 10 + 10 on
//    k_step_skew although k_step_wg at K = 16 is the fastest per turn.  Longer stretches run
//    full launches of the tuned kernel and depth first.
//  * Otherwise the turns are spread over ceil(room / tpl) launches of near-equal depth: 128
//    turns at tpl 6 run as 18 x 6 + 4 x 5, not 21 x 6 + 2.
// gol_step and gol_halo_buffers both use this rule (the zero-copy halo layout must be the
// layout the first launch after an exchange runs on; every planned kernel runs on the
// interleaved layout).
Launch plan_launch(gol_ctx *c, int64_t room)
{
    Launch L{1, c->multi_variant, c->band, 0, 0};
    if (c->tpl <= 1 || room < 2 || (c->cfg.flags & GOL_FLAG_COUNT_EVERY_TURN) ||
        c->blocked_pending)
        return L;
    // (another engine on the device could hold CUs the resident tiles need: then plain
    // launches -- a starved wait would give up and report GOL_EHIP, but never hang)
    if (c->persist_k > 0 && !is_strip(c) && room >= 2 * c->persist_k &&
        (c->persist_forced || device_exclusive(c->device))) {
        // K1p: blocks of <= persist_k turns in one launch, up to ~1 ms of work per launch so
        // the control word and readers are still served every millisecond or so
        const double us = c->tuned_us_per_turn > 0.f ? c->tuned_us_per_turn : 1.0;
        const int64_t cap = std::max<int64_t>(2 * c->persist_k, (int64_t)(1000.0 / us));
        return Launch{(int)std::min<int64_t>(room, cap), golk::kMultiTilePersist, c->band_multi,
                      c->tile_w, c->persist_seg ? c->persist_seg : c->tile_seg, c->persist_k};
    }
    if (c->stream_k > 0 && !is_strip(c) && room >= 2 * c->stream_k) {
        // K1q: blocks of <= stream_k turns in one launch, up to ~8 ms of work per launch (the
        // control word and readers are served between launches)
        const double us = c->tuned_us_per_turn > 0.f ? c->tuned_us_per_turn : 1.0;
        const int64_t cap = std::max<int64_t>(2 * c->stream_k, (int64_t)(8000.0 / us));
        return Launch{(int)std::min<int64_t>(room, cap), golk::kMultiTileStream, c->stream_th,
                      c->stream_tw, c->stream_seg, c->stream_k};
    }
    if (!c->plan.empty()) {
        if (room > kPlanMax)
            return Launch{c->tpl, c->multi_variant, c->band_multi, c->tile_w, c->tile_seg};
        if (c->plan[room].k >= 2) return c->plan[room];
    }
    const int64_t nl = (room + c->tpl - 1) / c->tpl;
    const int k = (int)((room + nl - 1) / nl);
    if (!golk::multi_ok(c->cfg.width, k, c->multi_variant)) return L;
    return Launch{k, c->multi_variant, band_for_depth(c, k), c->tile_w, c->tile_seg};
}

int launch_depth(gol_ctx *c, int64_t room) { return plan_launch(c, room).k; }

// the word layout a launch of depth k runs on
bool stepping_il(const gol_ctx *c, int k)
{
    return k > 1 && golk::multi_is_il(c->multi_words, c->multi_variant);
}

// popcount of owned rows of the current board -> *alive (synchronous)
int count_now(gol_ctx *c, long long *alive)
{
    unsigned long long *slot = c->counts + (size_t)kRing * kShards;
    HIP_OR_FAIL(c, hipMemsetAsync(slot, 0, kShards * sizeof(unsigned long long), c->stream));
    HIP_OR_FAIL(c, golk::launch_popcount(c->board[c->cur], c->nw, c->pitch, own_lo(c), own_hi(c),
                                         slot, c->stream));
    HIP_OR_FAIL(c, hipMemcpyAsync(c->h_counts, slot, kShards * sizeof(unsigned long long),
                                  hipMemcpyDeviceToHost, c->stream));
    if (int rc = sync_checked(c)) return rc;
    unsigned long long s = 0;
    for (int i = 0; i < kShards; i++) s += c->h_counts[i];
    *alive = (long long)s;
    return GOL_OK;
}

// kMultiWgPg: the published-row scratch and flags for a launch of `a`, grown on demand (the
// engine's streams are drained first: a running launch may still use the old buffers), and
// a fresh epoch.  Other variants, and bands the kernel runs as kMultiWgHx, need nothing.
static hipError_t pg_prepare(gol_ctx *c, golk::StepArgs &a, int k)
{
    a.xrows = nullptr;
    a.xflags = nullptr;
    if (!golk::is_pg_variant(a.multi_variant) ||
        !golk::pg_ok(k, a.band, a.multi_variant == golk::kMultiWgPgS))
        return hipSuccess;
    if (!device_exclusive(c->device)) {      // (launch_wg runs it as plain helix bands)
        a.multi_variant = a.multi_variant == golk::kMultiWgPgS ? golk::kMultiWgHxS
                                                               : golk::kMultiWgHx;
        return hipSuccess;
    }
    const long long T =
        golk::multi_pipes(a.width, a.row_hi - a.row_lo, a.band, 2, a.multi_variant);
    const size_t lanes = (size_t)T * 62 + 64;
    if (lanes > c->pg_lanes || (size_t)T > c->pg_tiles) {
        if (2ull * golk::kPgStages * lanes * 8 >= (1ull << 31)) return hipSuccess;   // helix
        hipError_t e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess && c->side) e = hipStreamSynchronize(c->side);
        if (e != hipSuccess) return e;
        if (c->pg_rows) (void)hipFree(c->pg_rows);
        if (c->pg_flags) (void)hipFree(c->pg_flags);
        c->pg_rows = nullptr;
        c->pg_flags = nullptr;
        c->pg_lanes = c->pg_tiles = 0;
        e = hipExtMallocWithFlags((void **)&c->pg_rows, 2ull * golk::kPgStages * lanes * 8,
                                  hipDeviceMallocUncached);
        if (e == hipSuccess)
            e = hipExtMallocWithFlags((void **)&c->pg_flags,
                                      (size_t)T * golk::kPgStages * sizeof(unsigned),
                                      hipDeviceMallocUncached);
        if (e == hipSuccess)
            e = hipMemset(c->pg_flags, 0, (size_t)T * golk::kPgStages * sizeof(unsigned));
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (e != hipSuccess) return e;
        c->pg_lanes = lanes;
        c->pg_tiles = (size_t)T;
    }
    a.xrows = c->pg_rows;
    a.xflags = c->pg_flags;
    a.xlanes = (unsigned)c->pg_lanes;
    a.epoch = ++c->pg_epoch;
    return hipSuccess;
}

// K1p / K1q: the uncached block buffers (board-sized), per-tile flags and the item counter,
// allocated on first use (the engine's streams drained first)
static hipError_t persist_buffers(gol_ctx *c, long long ntiles)
{
    const size_t words = (size_t)c->buf_rows * c->pitch;
    if (c->pu[0] && c->pu[1] && (size_t)ntiles <= c->pflags_n && c->pcounter) return hipSuccess;
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return e;
    for (auto *&u : c->pu)
        if (!u && (e = hipExtMallocWithFlags((void **)&u, words * 8, hipDeviceMallocUncached)) !=
                      hipSuccess)
            return e;
    if (!c->pcounter) {
        if ((e = hipExtMallocWithFlags((void **)&c->pcounter, 64, hipDeviceMallocUncached)) !=
                hipSuccess ||
            (e = hipMemset(c->pcounter, 0, 64)) != hipSuccess ||
            (e = hipDeviceSynchronize()) != hipSuccess)
            return e;
        c->pcount = 0;
    }
    if ((size_t)ntiles > c->pflags_n) {
        if (c->pflags) (void)hipFree(c->pflags);
        c->pflags = nullptr;
        c->pflags_n = 0;
        if ((e = hipExtMallocWithFlags((void **)&c->pflags, (size_t)ntiles * sizeof(unsigned),
                                       hipDeviceMallocUncached)) != hipSuccess ||
            (e = hipMemset(c->pflags, 0, (size_t)ntiles * sizeof(unsigned))) != hipSuccess ||
            (e = hipDeviceSynchronize()) != hipSuccess)
            return e;
        c->pflags_n = (size_t)ntiles;
        c->pepoch = 0;
    }
    return hipSuccess;
}

// K1p: one launch of `turns` turns in blocks of K on resident tiles
hipError_t persist_launch(gol_ctx *c, golk::StepArgs a, int turns, int K)
{
    const long long ntiles = golk::tile_count(c->nw, a.row_hi - a.row_lo, a.band, a.tile_w,
                                              a.tile_seg);
    if (hipError_t e = persist_buffers(c, ntiles)) return e;
    // flags of earlier launches are at most their epoch + blocks - 1: start above them all
    const unsigned nblocks = (unsigned)((turns + K - 1) / K);
    const unsigned epoch = c->pepoch + 1;
    c->pepoch = epoch + nblocks;
    if (c->persist_ring) {                   // K1r: only the rings pass through u0 / u1
        // (GOL_RING=2, experiments: a grid-wide barrier per block on K1q's counter)
        const bool grid = getenv("GOL_RING") && atoi(getenv("GOL_RING")) == 2;
        const unsigned base = c->pcount;
        if (grid) c->pcount += (unsigned)ntiles * (nblocks - 1);
        return golk::launch_tile_ring(a, turns, K, c->pu[0], c->pu[1], c->pflags, epoch,
                                      grid ? c->pcounter : nullptr, base, c->stream);
    }
    return golk::launch_tile_persist(a, turns, K, c->pu[0], c->pu[1], c->pflags, epoch, c->stream);
}

// K1q: one launch of `turns` turns in blocks of K, (block, tile) items taken from the counter
hipError_t stream_launch(gol_ctx *c, golk::StepArgs a, int turns, int K)
{
    const long long ntiles = golk::tile_count(c->nw, a.row_hi - a.row_lo, a.band, a.tile_w,
                                              a.tile_seg);
    if (hipError_t e = persist_buffers(c, ntiles)) return e;
    for (auto *&u : c->su)
        if (!u) {
            hipError_t e = hipStreamSynchronize(c->stream);
            if (e == hipSuccess) e = hipMalloc((void **)&u, (size_t)c->buf_rows * c->pitch * 8);
            if (e != hipSuccess) return e;
        }
    const unsigned nblocks = (unsigned)((turns + K - 1) / K);
    const unsigned epoch = c->pepoch + 1;
    unsigned grid = 0;
    // GOL_STREAM_GRID (tests): cap the workgroups, so that each takes many items
    const int max_grid = getenv("GOL_STREAM_GRID") ? atoi(getenv("GOL_STREAM_GRID")) : 0;
    const hipError_t e = golk::launch_tile_stream(a, turns, K, c->su[0], c->su[1], c->pflags,
                                                  epoch, c->pcounter, c->pcount, c->ncu, max_grid,
                                                  &grid, c->stream);
    if (e != hipSuccess) return e;
    c->pepoch = epoch + nblocks;
    c->pcount += (unsigned)(ntiles * nblocks) + grid;   // items + one overshoot per workgroup
    return hipSuccess;
}

// ---------------------------------------------------------------- k_step_tile planning
// every segment code a search below can pick is one the product ships (and tests)
template <size_t N>
constexpr bool all_shipped(const int (&codes)[N])
{
    for (int c : codes)
        if (!golk::tile_code_shipped(c)) return false;
    return true;
}

struct TileShape {
    int K = 0, th = 0, tw = 0, seg = 0;
    double model_us = 0;                     // modelled time per turn
};

// Modelled time per turn of k_step_tile at one shape, fitted to the
// measured shapes of profiles/r03_tile_*.log: a wave issues (SEG + 2) row sums (8 VALU) and
// SEG rules (14 VALU) per turn, at ~2.36 SIMD cycles per instruction (18 full-rate v_bitop3,
// 4 half-rate v_alignbit / DPP moves per row pair); a SIMD shares its issue between its
// resident waves, one wave alone issues at most every ~5 cycles, and each turn adds a barrier
// and the LDS exchange -- cheaper to hide with >= 2 workgroups per CU (~80 % of the issue
// rate and ~700 cycles a turn) than with one (~70 %, ~900).  Residency from the occupancy
// API (the kernel's VGPRs and dynamic LDS).
double tile_model_us(int ncu, int nw, int rows, int K, int th, int tw, int seg)
{
    if (!golk::tile_shape_ok(nw, K, th, tw, seg)) return 0;
    const long long tiles = golk::tile_count(nw, rows, th, tw, seg);
    const int waves = golk::tile_waves(K, th, tw, seg);
    const int wgpc = golk::tile_blocks_per_cu(K, th, tw, seg);         // VGPRs, LDS
    if (wgpc <= 0) return 0;
    const long long slots = (long long)ncu * wgpc;
    const long long rounds = (tiles + slots - 1) / slots;
    const long long per_cu = std::min<long long>((tiles + ncu - 1) / ncu, wgpc);
    const double instr = (seg % 100) * 22.0;                           // per wave and turn
    const double issue = (double)(per_cu * waves) * instr * 2.36 / 4.0;
    const bool two = per_cu >= 2;
    const double turn_cyc = std::max(issue / (two ? 0.8 : 0.7), instr * 5.0) + (two ? 700 : 900);
    const double launch_us = rounds * (K * turn_cyc + 2500.0) / 2400.0 + 3.0;
    return launch_us / K;
}

// The shapes the model ranks best for a board of nw words x rows (the best TH and SEG per
// (K, TW)), fastest first.  TW: every width that splits a row into ntx near-equal tiles; TH:
// the tallest tile the workgroup holds (16 waves) and the heights whose tile count fills 1..4
// resident tiles per CU or a few more tile rows.
std::vector<TileShape> tile_candidates(int ncu, int nw, int rows, int keep)
{
    // SEG, and SEG + 100 for the interior-rows-first turn order (gol_tile.hip)
    static constexpr int kSegs[] = {2, 3, 4, 6, 8, 12, 16, 24, 32, 40, 48,
                                    106, 108, 112, 116, 124, 132, 140};
    static_assert(all_shipped(kSegs), "a tile code outside golk::kTileCodes");
    std::vector<TileShape> all;
    std::vector<int> tws;
    for (int ntx = 1; ntx <= nw; ++ntx) {
        const int tw = (nw + ntx - 1) / ntx;
        if (tw <= 62 && (tws.empty() || tws.back() != tw)) tws.push_back(tw);
    }
    for (int K : {8, 12, 16, 20, 24, 32}) {
        for (int tw : tws) {
            TileShape best;
            const int C = tw + 2, G = 64 / C;
            const long long ntx = (nw + tw - 1) / tw;
            for (int seg : kSegs) {
                const int thmax = golk::kTileMaxWavesHost * G * (seg % 100) - 2 * K;
                if (thmax < 1) continue;
                std::vector<long long> ntys;
                const long long nty0 = (rows + thmax - 1) / thmax;
                for (long long n = nty0; n < nty0 + 4; ++n) ntys.push_back(n);
                for (int per_cu = 1; per_cu <= 4; ++per_cu)
                    ntys.push_back(std::max(nty0, ((long long)ncu * per_cu + ntx - 1) / ntx));
                for (long long nty : ntys) {
                    const int th = (int)std::max<long long>(1, (rows + nty - 1) / nty);
                    const double m = tile_model_us(ncu, nw, rows, K, th, tw, seg);
                    if (m > 0 && (best.K == 0 || m < best.model_us)) best = {K, th, tw, seg, m};
                }
            }
            if (best.K) all.push_back(best);
        }
    }
    std::sort(all.begin(), all.end(),
              [](const TileShape &x, const TileShape &y) { return x.model_us < y.model_us; });
    // the model ranks, the autotune decides: keep the list diverse (at most 2 depths per tile
    // width among the first picks)
    std::vector<TileShape> out;
    std::map<int, int> per_tw;
    for (const TileShape &t : all)
        if (per_tw[t.tw]++ < 2 && (int)out.size() < keep) out.push_back(t);
    for (const TileShape &t : all)
        if ((int)out.size() < keep && per_tw[t.tw] > 2) {
            out.push_back(t);
            per_tw[t.tw] = 0;               // (each width once more at most)
        }
    return out;
}

void apply_tile(gol_ctx *c, const TileShape &t)
{
    c->multi_variant = golk::kMultiTile;
    c->tpl = t.K;
    c->band_multi = t.th;
    c->tile_w = t.tw;
    c->tile_seg = t.seg;
    c->short_k = c->short_band = 0;
    for (int &b : c->band_at) b = 0;
    c->plan.clear();
    c->seq.clear();
    c->persist_k = 0;
    c->persist_seg = 0;
}

// Measured search for the k_step_tile shape (coordinate descent over the launch parameters;
// the model above only seeds the widths): from (the best-filled tile width, 8 waves per
// workgroup, K = 32 or the requested depth, SEG 16), improve one parameter at a time -- SEG
// (both turn orders), tile width, waves per workgroup (the tile height follows: the tallest
// tile that many waves hold), K -- and keep each improvement.  The grid sweeps of
// profiles/r03_tile_grid_*.log put the best shapes at 8-wave workgroups (2 per CU) at every
// board size, with SEG from 4-6 (5120^2) to 16-40 (65536^2).  Returns the best measured
// shape (K == 0: none ran) and its time per turn in *us.
TileShape tile_search(gol_ctx *c, int kfix, float *us, int W)
{
    *us = 0.f;
    const int nw = c->nw, rows = c->buf_rows;
    if (nw % W) return TileShape{};
    const int nl = nw / W;                           // lane columns (W words each)
    struct WOpt { double useful; int tw; };
    std::vector<WOpt> wopt;
    for (int tw = 1; tw <= 62; ++tw) {
        const int G = 64 / (tw + 2);
        const long long ntx = (nl + tw - 1) / tw;
        wopt.push_back({(double)G * tw / 64.0 * nl / (double)(ntx * tw), tw});
    }
    std::sort(wopt.begin(), wopt.end(), [](const WOpt &x, const WOpt &y) {
        return x.useful > y.useful || (x.useful == y.useful && x.tw > y.tw);
    });
    std::vector<int> tws, tws_wide;                  // the 3 best-filled widths; 8 within 80 %
    for (const WOpt &w : wopt) {
        if ((int)tws.size() < 3 && w.useful >= wopt[0].useful * 0.9) tws.push_back(w.tw);
        if ((int)tws_wide.size() < 8 && w.useful >= wopt[0].useful * 0.8) tws_wide.push_back(w.tw);
    }
    static constexpr int kSegs1[] = {2, 3, 4, 6, 8, 12, 16, 24, 32, 40, 48,
                                     106, 108, 112, 116, 124, 132, 140,
                                     203, 204, 206, 208, 212, 216, 224, 232, 240,
                                     506, 512, 516, 524, 612, 616, 624};
    static constexpr int kSegs2[] = {1002, 1003, 1004, 1006, 1008, 1106, 1108, 1204, 1206, 1208};
    static_assert(all_shipped(kSegs1) && all_shipped(kSegs2), "a tile code outside kTileCodes");
    std::vector<int> segs = W == 1 ? std::vector<int>(std::begin(kSegs1), std::end(kSegs1))
                                   : std::vector<int>(std::begin(kSegs2), std::end(kSegs2));
    struct P { int K, wv, tw, seg, th = 0; };          // th > 0: this height (<= wv's)
    auto shape = [&](const P &p) -> TileShape {
        const int G = 64 / (p.tw + 2);
        int th = p.wv * G * (p.seg % 100) - 2 * p.K;
        if (p.th > 0) th = std::min(th, p.th);
        th = std::min(th, rows);
        if (th < std::min(8, rows) ||
            !golk::tile_shape_ok(nw, p.K, th, p.tw, p.seg))
            return TileShape{};
        return TileShape{p.K, th, p.tw, p.seg, 0};
    };
    golk::StepArgs a{};
    a.width = c->cfg.width;
    a.nw = nw;
    a.pitch = c->pitch;
    a.modrows = rows;
    a.row_lo = 0;
    a.row_hi = rows;
    a.multi_words = 1;
    a.multi_variant = golk::kMultiTile;
    a.err = c->d_err;
    if (golk::launch_fill_random(c->board[0], c->cfg.width, nw, c->pitch, rows, 0, rows, 12345,
                                 c->stream) != hipSuccess)
        return TileShape{};
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess) return TileShape{};
    if (hipEventCreate(&e1) != hipSuccess) { (void)hipEventDestroy(e0); return TileShape{}; }
    int reps = 16;
    auto time_one = [&](const TileShape &t, int n) -> float {
        a.band = t.th;
        a.tile_w = t.tw;
        a.tile_seg = t.seg;
        bool ok = hipEventRecord(e0, c->stream) == hipSuccess;
        for (int rep = 0; rep < n && ok; ++rep) {
            a.in = c->board[rep & 1];
            a.out = c->board[(rep + 1) & 1];
            ok = golk::launch_step_multi(a, t.K, c->stream) == hipSuccess;
        }
        ok = ok && hipEventRecord(e1, c->stream) == hipSuccess &&
             hipEventSynchronize(e1) == hipSuccess;
        float ms = 0.f;
        if (!ok || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 0.f;
        return ms / ((float)n * t.K);
    };
    std::map<std::tuple<int, int, int, int>, float> memo;
    auto measure = [&](const P &p) -> float {
        const TileShape t = shape(p);
        if (!t.K) return 0.f;
        auto key = std::make_tuple(t.K, t.th, t.tw, t.seg);
        auto it = memo.find(key);
        if (it != memo.end()) return it->second;
        float best = 0.f;
        for (int pass = 0; pass < 2; ++pass) {      // best of two (clock noise)
            const float v = time_one(t, reps);
            if (v > 0.f && (best == 0.f || v < best)) best = v;
        }
        memo[key] = best;
        if (getenv("GOL_AUTOTUNE_LOG"))
            fprintf(stderr, "autotune tile %dx%d K=%d th=%d tw=%d seg=%d us_per_turn=%.4f\n",
                    c->cfg.width, rows, t.K, t.th, t.tw, t.seg, best * 1000.f);
        return best;
    };
    P cur{kfix > 0 ? kfix : 32, 8, tws.empty() ? 30 : tws[0], W == 1 ? 16 : 1008};
    // clock ramp, and the repetitions that make a measurement ~0.5 ms of launches
    {
        TileShape t0 = shape(cur);
        if (!t0.K) {                          // (tiny boards: shallower SEG)
            for (int sg : {8, 4, 2}) {
                cur.seg = sg + 1000 * (W - 1);
                if ((t0 = shape(cur)).K) break;
            }
        }
        if (t0.K) {
            const float v = time_one(t0, 8) * 1000.f * t0.K;   // us per launch
            if (v > 0.f) reps = std::max(2, std::min(16, (int)(500.f / v) + 1));
            (void)time_one(t0, reps);
        }
    }
    float best = measure(cur);
    auto improve = [&](P p) {
        const float v = measure(p);
        if (v > 0.f && (best == 0.f || v < best * 0.995f)) {
            best = v;
            cur = p;
        }
    };
    if ((long long)nw * rows < (1ll << 23)) {
        // boards up to 16384^2: SEG x width x waves jointly first (one turn order) -- one
        // parameter at a time settled on 5120^2 at 18-word tiles of SEG 8 (0.76 us per turn)
        // while 14 x 128 tiles of SEG 6 ran 0.64 (profiles/r03b_tile_search_5120.log)
        static constexpr int kJoint1[] = {102, 103, 104, 106, 108, 112, 116, 124};
        static constexpr int kJoint2[] = {1102, 1103, 1104, 1106, 1108};
        static_assert(all_shipped(kJoint1) && all_shipped(kJoint2), "tile code outside kTileCodes");
        const P base = cur;
        const int *js = W == 1 ? kJoint1 : kJoint2;
        const int nj = W == 1 ? (int)std::size(kJoint1) : (int)std::size(kJoint2);
        for (int i = 0; i < nj; ++i)
            for (int tw : tws_wide)
                for (int wv : {8, 12, 16}) improve(P{base.K, wv, tw, js[i]});
    } else if (W == 1) {
        // larger boards: the short-segment family on 14-word tiles (4 groups of 16 lanes, 16
        // waves at <= 64 VGPRs: 8 waves per SIMD) -- 11 % faster than 62-word SEG 32 tiles on
        // the 8-strip shape, 8 % slower at 65536^2 (profiles/r03_tile_small_seg_65536.log)
        const P base = cur;
        static constexpr int kShort[] = {104, 106, 206, 108};
        static_assert(all_shipped(kShort), "a tile code outside kTileCodes");
        for (int sg : kShort)
            for (int tw : {14, tws.empty() ? 14 : tws[0]})
                for (int wv : {8, 16}) improve(P{base.K, wv, tw, sg});
        // ... and the 80-VGPR family: ORD 5 (edge sums read back from LDS) at SEG 16-24 holds
        // 6 waves per SIMD -- two 12-wave workgroups per CU, the occupancy at which the
        // stencil's instruction mix issues fastest (tools/calib/valu_issue occupancy: 1.66
        // cycles per instruction against 2.43 at 4 waves); 30 x 536 tiles of SEG 24 ran 34.6
        // us per turn at 65536^2 against 36.3 for the best 4-wave shape
        // (profiles/r04_sweep_65536_ord5.log)
        static constexpr int kSix[] = {524, 624, 516, 616};
        static_assert(all_shipped(kSix), "a tile code outside kTileCodes");
        for (int sg : kSix)
            for (int tw : {tws.empty() ? 30 : tws[0], 14})
                for (int wv : {12, 8}) improve(P{base.K, wv, tw, sg});
    }
    {
        const P base = cur;
        for (int sg : segs) improve(P{base.K, base.wv, base.tw, sg});
    }
    {
        const P base = cur;
        for (int tw : tws) improve(P{base.K, base.wv, tw, base.seg});
    }
    {
        const P base = cur;
        for (int wv : {4, 6, 8, 12, 16}) improve(P{base.K, wv, base.tw, base.seg});
    }
    if (kfix <= 0) {
        const P base = cur;
        for (int K : {12, 16, 20, 24, 32}) improve(P{K, base.wv, base.tw, base.seg});
    }
    {
        // width x waves jointly (the tile height follows both: 5120^2 ran best at 10 words x
        // 12 waves, a width the fill ranking puts 4th, profiles/r03_tile_grid_5.log)
        const P base = cur;
        for (int tw : tws_wide)
            for (int wv : {8, 12, 16}) improve(P{base.K, wv, tw, base.seg});
    }
    {
        const P base = cur;
        for (int sg : segs) improve(P{base.K, base.wv, base.tw, sg});
    }
    // round balance: the tallest tile is not always the best -- 525 tiles on 512 slots run 2
    // rounds (8448-row strips at height 576); shorter tiles that fill the same rounds evenly
    // take fewer waves each.  Try the heights whose tile count just fits 1..4 residency rounds.
    {
        const P base = cur;
        const TileShape t0 = shape(base);
        if (t0.K) {
            const long long ntx = (nl + base.tw - 1) / base.tw;
            for (int r = 1; r <= 4; ++r) {
                for (long long nty = (rows + t0.th - 1) / t0.th; nty <= 4ll * rows; ++nty) {
                    const int th = (int)((rows + nty - 1) / nty);
                    if (th < 8) break;
                    const int wg = golk::tile_blocks_per_cu(base.K, th, base.tw, base.seg);
                    if (wg <= 0) continue;
                    if (ntx * nty <= (long long)r * c->ncu * wg) {
                        if (th != t0.th) improve(P{base.K, base.wv, base.tw, base.seg, th});
                        break;
                    }
                }
            }
        }
    }
    // the search kept whatever beat the incumbent by 0.5 % on a best-of-2 timing; shapes
    // within noise of each other can trade places from box to box, so the 4 fastest seen are
    // timed again (best of 3) and the fastest of that final round is the pick
    TileShape pick = best > 0.f ? shape(cur) : TileShape{};
    if (pick.K) {
        std::vector<std::pair<float, TileShape>> top;
        for (const auto &m : memo)
            if (m.second > 0.f)
                top.push_back({m.second, TileShape{std::get<0>(m.first), std::get<1>(m.first),
                                                   std::get<2>(m.first), std::get<3>(m.first), 0}});
        std::sort(top.begin(), top.end(),
                  [](const auto &x, const auto &y) { return x.first < y.first; });
        if (top.size() > 4) top.resize(4);
        // ... and among the shapes within 1 % of the fastest of that round (timing noise from
        // box to box), a fixed order decides -- the deepest K, then the lowest segment code,
        // the widest tile, the tallest -- so two boxes that time the same shapes within noise
        // pick the same one
        std::vector<std::pair<float, TileShape>> fin;
        float fbest = 0.f;
        for (const auto &c2 : top) {
            float v = 0.f;
            for (int pass = 0; pass < 3; ++pass) {
                const float u = time_one(c2.second, reps);
                if (u > 0.f && (v == 0.f || u < v)) v = u;
            }
            if (v > 0.f) {
                fin.push_back({v, c2.second});
                if (fbest == 0.f || v < fbest) fbest = v;
            }
        }
        auto before = [](const TileShape &x, const TileShape &y) {
            return std::make_tuple(-x.K, x.seg, -x.tw, -x.th) < std::make_tuple(-y.K, y.seg, -y.tw, -y.th);
        };
        bool have = false;
        for (const auto &f : fin)
            if (f.first <= 1.01f * fbest && (!have || before(f.second, pick))) {
                pick = f.second;
                best = f.first;
                have = true;
            }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipGetLastError();
    *us = best * 1000.f;
    return pick;
}

// Pinned launch shapes for the BASELINE board sizes on an MI355X (gfx950, 256 CUs): an engine
// of one of these widths and buffer heights (a torus, or a row strip with its halos) with
// nothing pinned by the caller runs this k_step_tile shape and skips the create-time search.  The search's 0.5 ms timings put a dozen shapes within
// ~1.5 % of each other and picked different ones from box to box (round 4: 65536^2 K = 20 on
// 336-row tiles on one box, K = 32 on 512-row tiles or k_step_skew K = 8 on others; 16384^2
// bands 316 / 320), so the kernel a bench line timed was not reliably the one profiles/
// measured.  These are the search winners of the round-4 sweeps, each pinned by a full-size
// oracle digest (tests/test_gpu_engine.py::test_pinned_shape_digest) and profiled as is
// (profiles/r05_*_summary.json).  GOL_AUTOTUNE=2 measures instead.
struct KnownShape {
    int width, rows;
    TileShape t;                             // K, tile height, tile width (lanes), segment code
    float us_per_turn;                       // measured steady state (round-4 sweeps)
    int short_K = 0, short_th = 0;           // launches of depth <= short_K: tiles short_th tall
};
constexpr KnownShape kKnownShapes[] = {
#ifdef GOL_PIN_OVERRIDE   // (A/B builds: an entry ahead of the table, e.g. 65536,65536,{20,472,30,516,0},34.f)
    {GOL_PIN_OVERRIDE},
#endif
    // configs[3..4]: 30-lane tiles of ORD 5 SEG 16 in 16-wave workgroups (2 per CU, 8 waves
    // per SIMD).  Long steps: K = 30 on 30 x 452 tiles, 33.09-33.12 us per turn against
    // 33.72-33.75 for K = 20 (profiles/r06_c3_deep_k.log, 65536 sweep).  Launches of <= 20
    // turns -- the driver's 20-turn call is one launch of exactly 20 -- keep 30 x 472 tiles:
    // the fastest of 30 K = 20 shapes (33.6 us per turn; profiles/r06_headline_pin_ab.log) and,
    // in the bench, 118.3-121.0k against 117.7-119.4k for 30 x 536 SEG 24 12-wave tiles and
    // 115.9-118.4k for round 5's K = 24 on 30 x 336 8-wave tiles (alternating on one box)
    {65536, 65536, {30, 452, 30, 516, 0}, 33.1f, 20, 472},
    // configs[2]: ORD 5, SEG 16, 8-wave workgroups, 14 x 410 tiles, K = 51 (deeper than the
    // planner's tables: k_step_tile runs up to 64 turns): 760 tiles, at most 3 per CU, 2.726-2.730
    // us per turn against 2.742 for K = 48 on 14 x 416 and 2.83-2.84 for round 6's first pin,
    // 14 x 448 at K = 32 (703 tiles), which was the fastest of 36 K = 32 shapes
    // (profiles/r06_c3_deep_k.log; before it round 5's 14 x 320 ORD 1 SEG 12,
    // profiles/r06_headline_pin_ab.log)
    {16384, 16384, {51, 410, 14, 516, 0}, 2.73f},
    // configs[1]: ORD 2, SEG 3, 16-wave workgroups of 10-lane tiles (5 groups per wave), 10 x
    // 160 at K = 40: 8 x 32 = 256 tiles, one per CU with none idle (80 words = 8 x 10 exactly),
    // 0.524-0.530 us per turn against 0.550-0.553 for the earlier 14 x 128 at K = 32 (240
    // tiles; profiles/r06_c3_deep_k.log, C2 section)
    {5120, 5120, {40, 160, 10, 203, 0}, 0.53f},
    // configs[3..4] as row strips with 128-row halos (buffer = H / N + 256 rows):
    // N = 8 ORD 1 SEG 12 (west carry) on 14 x 352 tiles, 8 launches of 16 turns per window
    // (5.44-5.46 us per turn against 5.69-5.70 for ORD 5 SEG 12 on the same tiles,
    // profiles/r05_strip_seg12_ab.log; 5.61-5.71 for round 4's searched picks); N = 4 and 2
    // ORD 5 SEG 16 since round 6: 14 x 448 tiles K = 32 (9.14 against 9.21 us per turn for
    // round 5's 14 x 704 SEG 24) and 14 x 480 tiles K = 16 (16.97 against 17.91)
    // (profiles/r06_strip_sweep.log)
    {65536, 8448, {16, 352, 14, 112, 0}, 5.3f},
    {65536, 16640, {32, 448, 14, 516, 0}, 9.14f},
    {65536, 33024, {16, 480, 14, 516, 0}, 16.97f},
    // configs[3..4] as row strips with the bench's default halo for its 20-turn command
    // (min(128, turns): 20 rows, one exchange and one 20-turn launch per window; buffer = H / N
    // + 40 rows), K = 20, the fastest of 40-50 shapes swept per buffer
    // (profiles/r06_strip_sweep.log): N = 8 ORD 1 SEG 12 (west carry) on 14 x 344 tiles, 4.95
    // us per turn; N = 4 and 2 the headline's ORD 5 SEG 16 on 30 x 472 tiles in 16-wave
    // workgroups, 9.04 / 17.56 against 9.28-9.36 / 18.16 for 14 x 344 ORD 1 SEG 12
    {65536, 8232, {20, 344, 14, 112, 0}, 4.95f},
    {65536, 16424, {20, 472, 30, 516, 0}, 9.04f},
    {65536, 32808, {20, 472, 30, 516, 0}, 17.56f},
    // configs[2] on 2 GPUs: 16384^2 as 2 strips with 128-row halos (16384 x 8448): ORD 5 SEG 12
    // on 30 x 320 tiles, K = 32, 16-wave workgroups: 1.72 us per turn (30 x 320 ORD 1 SEG 12
    // 1.73, 14 x 704 ORD 5 SEG 12 1.74, the 14 x 320 ORD 1 torus pin slower;
    // profiles/r06_strip_sweep.log)
    {16384, 8448, {32, 320, 30, 512, 0}, 1.72f},
};

bool known_shape(const gol_ctx *c, KnownShape *out)
{
    if (c->ncu != 256) return false;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->device) != hipSuccess ||
        std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return false;
    for (const KnownShape &k : kKnownShapes)
        if (k.width == c->cfg.width && k.rows == c->buf_rows &&
            golk::tile_shape_ok(c->nw, k.t.K, k.t.th, k.t.tw, k.t.seg)) {
            *out = k;
            return true;
        }
    return false;
}

// A pinned shape is applied whenever the device, width and buffer rows match: the shape never
// depends on timing or load (round-5 advice: a slow or shared box must not change the kernel
// the tests and profiles pin).  The first engine of a pinned shape in a process then runs
// ~GOL_PIN_VERIFY_MS (default 60; 0 = off) ms of its launches on its own buffers and compares
// the median time per turn with the table's figure; more than 1.35x is only reported (stderr),
// a device unlike the one the table was measured on.  The check also keeps the GPU busy right
// before the caller's first steps: an MI355X that idled drops its clock, and a 20-turn 65536^2
// call then takes 810-850 us instead of 700 (profiles/r04_clock_ramp_20turn.log,
// profiles/r05_prewarm_probe.log).  Later engines of the same (device, width, buffer rows) skip
// it (g_pin_checked).  Returns the median us per turn (0 when it did not run).
float check_pinned(gol_ctx *c, const KnownShape &ks)
{
    const char *v = getenv("GOL_PIN_VERIFY_MS");
    const double budget_ms = v ? atof(v) : 60.0;
    if (budget_ms <= 0) return 0.f;
    const auto key = std::make_tuple(c->device, c->cfg.width, c->buf_rows);
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        if (g_pin_checked.count(key)) return 0.f;
    }
    golk::StepArgs a{};
    a.width = c->cfg.width;
    a.nw = c->nw;
    a.pitch = c->pitch;
    a.modrows = c->buf_rows;
    a.row_lo = 0;
    a.row_hi = c->buf_rows;
    a.multi_words = 1;
    a.multi_variant = golk::kMultiTile;
    a.err = c->d_err;
    a.band = ks.t.th;
    a.tile_w = ks.t.tw;
    a.tile_seg = ks.t.seg;
    if (golk::launch_fill_random(c->board[0], c->cfg.width, c->nw, c->pitch, c->buf_rows, 0,
                                 c->buf_rows, 12345, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return 0.f;
    // groups of ~1 ms of launches
    const int n = std::max(1, (int)std::ceil(1000.0 / (ks.t.K * ks.us_per_turn)));
    std::vector<float> us;
    // (default) one queue of back-to-back launches, an event pair per group, one sync at the
    // end: the GPU stays busy for the whole check (bench20 116.5-118.0k against 116.1-117.2k
    // with a sync after every burst, profiles/r05_verify_mode_ab.log); GOL_PIN_VERIFY_MODE=0:
    // bursts of ~1 ms, each ended by a sync
    const char *vm = getenv("GOL_PIN_VERIFY_MODE");
    const bool queued = !(vm && atoi(vm) == 0);
    if (queued) {
        const int groups = std::max(8, (int)std::ceil(budget_ms * 1000.0 / (n * ks.t.K * ks.us_per_turn)));
        std::vector<hipEvent_t> ev(groups + 1);
        for (auto &e : ev)
            if (hipEventCreate(&e) != hipSuccess) return 0.f;
        bool ok = hipEventRecord(ev[0], c->stream) == hipSuccess;
        for (int i = 0; ok && i < groups; ++i) {
            for (int j = 0; ok && j < n; ++j) {
                a.in = c->board[j & 1];
                a.out = c->board[(j + 1) & 1];
                ok = golk::launch_step_multi(a, ks.t.K, c->stream) == hipSuccess;
            }
            ok = ok && hipEventRecord(ev[i + 1], c->stream) == hipSuccess;
        }
        ok = ok && hipStreamSynchronize(c->stream) == hipSuccess;
        for (int i = 0; ok && i < groups; ++i) {
            float ms = 0.f;
            ok = hipEventElapsedTime(&ms, ev[i], ev[i + 1]) == hipSuccess;
            us.push_back(ms * 1e3f / (n * ks.t.K));
        }
        for (auto &e : ev) (void)hipEventDestroy(e);
        if (!ok) return 0.f;
    }
    // GOL_PIN_VERIFY_MODE=0: bursts of ~1 ms of launches, each ended by a sync (host wall time,
    // as gol_step runs)
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; !queued && i < 2000; ++i) {
        const auto s0 = std::chrono::steady_clock::now();
        for (int j = 0; j < n; ++j) {
            a.in = c->board[j & 1];
            a.out = c->board[(j + 1) & 1];
            if (golk::launch_step_multi(a, ks.t.K, c->stream) != hipSuccess) return 0.f;
        }
        if (hipStreamSynchronize(c->stream) != hipSuccess) return 0.f;
        const auto s1 = std::chrono::steady_clock::now();
        us.push_back(std::chrono::duration<float, std::micro>(s1 - s0).count() / (n * ks.t.K));
        if (std::chrono::duration<double, std::milli>(s1 - t0).count() >= budget_ms && i >= 8) break;
    }
    (void)hipGetLastError();
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        g_pin_checked.insert(key);
    }
    if (check_dev_err(c) != GOL_OK || us.empty()) return 0.f;
    std::vector<float> tail(us.begin() + us.size() / 2, us.end());
    std::sort(tail.begin(), tail.end());
    const float med = tail[tail.size() / 2];
    const bool slow = med > 1.35f * ks.us_per_turn;
    if (slow || getenv("GOL_AUTOTUNE_LOG"))
        fprintf(stderr, "%spinned shape %dx%d K=%d tile=%dx%d code=%d: %zu launches, median %.3f us per "
                "turn (table %.3f)%s\n", slow ? "gol: warning: " : "", c->cfg.width, c->buf_rows,
                ks.t.K, ks.t.tw, ks.t.th, ks.t.seg, us.size(), med, ks.us_per_turn,
                slow ? " -- more than 1.35x the table: not the device the table was measured on, "
                       "or a shared / throttled one (the pinned shape is kept)" : "");
    return med;
}

// Boards below 2^20 words (5120^2: 409 600) cannot fill the GPU with band pipelines: they run
// k_step_tile at the measured-best shape.
// K1p for a small torus board at the tuned tile shape: 256 turns as one k_tile_persist launch
// (blocks of Kp turns, tiles resident between blocks) against the same turns as k_step_tile
// launches of the tuned depth, best of 3 each; the persistent mode is kept (at its fastest
// block depth) when it is >= 2 % faster.  Only on a device this engine has to itself: every
// tile must be resident at once.
void persist_tune(gol_ctx *c)
{
    c->persist_k = 0;
    c->persist_seg = 0;
    const bool log = getenv("GOL_AUTOTUNE_LOG") != nullptr;
    if (is_strip(c) || c->multi_variant != golk::kMultiTile || !device_exclusive(c->device) ||
        getenv("GOL_NO_PERSIST")) {
        if (log)
            fprintf(stderr, "autotune persist skipped (strip %d variant %d exclusive %d)\n",
                    (int)is_strip(c), c->multi_variant, (int)device_exclusive(c->device));
        return;
    }
    golk::StepArgs a{};
    a.width = c->cfg.width;
    a.nw = c->nw;
    a.pitch = c->pitch;
    a.modrows = c->buf_rows;
    a.row_lo = 0;
    a.row_hi = c->buf_rows;
    a.multi_words = 1;
    a.multi_variant = golk::kMultiTile;
    a.band = c->band_multi;
    a.tile_w = c->tile_w;
    a.tile_seg = c->tile_seg;
    a.err = c->d_err;
    const int N = 256;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess) return;
    if (hipEventCreate(&e1) != hipSuccess) { (void)hipEventDestroy(e0); return; }
    auto timed = [&](auto &&launches) -> float {       // us per turn, best of 3
        float best = 0.f;
        for (int pass = 0; pass < 3; ++pass) {
            bool ok = hipEventRecord(e0, c->stream) == hipSuccess && launches() &&
                      hipEventRecord(e1, c->stream) == hipSuccess &&
                      hipEventSynchronize(e1) == hipSuccess;
            float ms = 0.f;
            if (!ok || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 0.f;
            const float us = ms * 1000.f / N;
            if (best == 0.f || us < best) best = us;
        }
        return best;
    };
    const float plain = timed([&]() {
        const int n = (N + c->tpl - 1) / c->tpl;
        for (int i = 0; i < n; ++i) {
            a.in = c->board[i & 1];
            a.out = c->board[(i + 1) & 1];
            const int k = N / n + (i < N % n ? 1 : 0);
            if (golk::launch_step_multi(a, k, c->stream) != hipSuccess) return false;
        }
        return true;
    });
    // the tuned code and its siblings with the same rows per segment (K1p is instantiated for
    // ORD 0, 1, 4 and 5 only: an ORD 2 pick runs persistent as one of those)
    float best = 0.f;
    int best_k = 0, best_code = 0;
    const int sg = c->tile_seg % 100;
    const int codes[] = {c->tile_seg, 100 + sg, 500 + sg, 400 + sg, sg};
    for (int ci = 0; ci < (int)std::size(codes); ++ci) {
        const int code = codes[ci];
        if (c->tile_seg >= 1000 || (ci > 0 && code == c->tile_seg)) continue;   // (W = 1 only)
        a.tile_seg = code;
        for (int Kp : {c->tpl, 8, 12, 16, 20, 24, 32}) {
            if (Kp < 2 || !golk::tile_persist_ok(c->nw, c->buf_rows, N, Kp, c->band_multi,
                                                 c->tile_w, code, c->ncu)) {
                if (log)
                    fprintf(stderr, "autotune persist K=%d: shape %d:%d:%d not persistent-capable\n",
                            Kp, c->tile_w, c->band_multi, code);
                continue;
            }
            const float us = timed([&]() {
                a.in = c->board[0];
                a.out = c->board[1];
                return persist_launch(c, a, N, Kp) == hipSuccess;
            });
            if (log)
                fprintf(stderr, "autotune persist %dx%d code=%d K=%d us_per_turn=%.4f (plain K=%d %.4f)\n",
                        c->cfg.width, c->buf_rows, code, Kp, us, c->tpl, plain);
            if (us > 0.f && (best == 0.f || us < best)) {
                best = us;
                best_k = Kp;
                best_code = code;
            }
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipGetLastError();
    // (a wait that gave up while timing: no persistent mode, and the junk board's error word
    // is cleared -- the board is refilled before use)
    const bool bad = check_dev_err(c) != GOL_OK;
    if (bad) clear_dev_err(c);
    if (best > 0.f && plain > 0.f && best < 0.98f * plain && !bad) {
        c->persist_k = best_k;
        c->persist_seg = best_code;          // (plain launches keep the code they were timed at)
        c->tuned_us_per_turn = best;
    }
}

void autotune_small(gol_ctx *c)
{
    float us1 = 0.f, us2 = 0.f;
    const TileShape t1 = tile_search(c, 0, &us1, 1);
    const TileShape t2 = tile_search(c, 0, &us2, 2);   // two words per lane
    const bool two = t2.K && (!t1.K || us2 < us1);
    if (!t1.K && !t2.K) return;
    apply_tile(c, two ? t2 : t1);
    c->tuned_us_per_turn = two ? us2 : us1;
    persist_tune(c);
}

// Create-time timing sweep of the temporal-blocking kernel, its depth K and its band on
// the engine's own buffers.  The fastest choice depends on grid/residency quantisation and
// on whether the two boards fit the 256 MiB MALL (tools/sweep.py, tools/strip_emulate.py:
// 65536^2 -> k_step_skew K = 8 band 137-274; 16384^2 and 8448-row strips -> k_step_wg
// K = 12), which no closed form captured, so large engines measure.  Both kernels run on
// the interleaved layout and every candidate computes the same bits.  `tune_variant`:
// choose between k_step_skew and k_step_wg (otherwise keep c->multi_variant).
void autotune_multi(gol_ctx *c, bool tune_k, bool tune_variant)
{
    const long long words = (long long)c->buf_rows * c->pitch;
    if (words < (1ll << 20)) return;                 // < 64 Mi cells: keep the defaults
    std::vector<int> vars{c->multi_variant};
    if (tune_variant)
        vars = {golk::kMultiSkewILW16, golk::kMultiWg, golk::kMultiWgHx, golk::kMultiWgPg,
                golk::kMultiWgHxS, golk::kMultiWgPgS, golk::kMultiTile};
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
    struct Cand {
        int var, K, band;
        int tw = 0, seg = 0;                         // k_step_tile shape
    };
    std::vector<Cand> cand;
    for (int var : vars) {
        if (var == golk::kMultiTile) {
            // the measured-best tile shape (tile_search), timed again beside the rest
            for (int W : {1, 2}) {
                float us = 0.f;
                const TileShape ts = tile_search(c, tune_k ? 0 : c->tpl, &us, W);
                if (ts.K) cand.push_back({var, ts.K, ts.th, ts.tw, ts.seg});
            }
            continue;
        }
        // K = 7 measured no faster than 6 / 8 on k_step_skew (DESIGN); k_step_wg goes to 16
        std::vector<int> ks = !golk::is_wg_variant(var) ? std::vector<int>{6, 8, 10}
                                                  : std::vector<int>{8, 12, 16};
        if (!tune_k) ks = {c->tpl};
        static const int kBands[] = {16, 20, 24, 32, 40, 48, 64, 96, 137, 192};
        const int lane_dw = golk::multi_lane_dwords(c->multi_words, var);
        for (int K : ks) {
            if (!golk::multi_ok(c->cfg.width, K, var)) continue;
            // plus the bands whose grid just fits 1..4 rounds of resident band pipelines
            // (k_step_skew: one per wave, k_step_wg: one per workgroup; 65536^2 at 4
            // waves/SIMD: 274 -> 4080 of 4096 waves, 137 -> 8160 of 8192)
            std::vector<int> bands(std::begin(kBands), std::end(kBands));
            const long long cap = (long long)ncu *
                                  golk::multi_blocks_per_cu(K, c->multi_words, var) *
                                  golk::multi_pipes_per_block(var);
            for (int r = 1; r <= 4 && cap > 0; ++r) {
                // the smallest band whose launch fits r rounds
                for (int b = 16; b <= 1024 && b <= c->cfg.rows; ++b)
                    if (golk::multi_pipes(c->cfg.width, c->cfg.rows, b, lane_dw, var) <= r * cap) {
                        bands.push_back(b);
                        break;
                    }
            }
            if (golk::is_pg_variant(var)) {   // the nearest bands it runs at (golk::pg_ok)
                for (int &b : bands) b = golk::pg_band(K, b, var == golk::kMultiWgPgS);
                bands.erase(std::remove(bands.begin(), bands.end(), 0), bands.end());
            }
            std::sort(bands.begin(), bands.end());
            bands.erase(std::unique(bands.begin(), bands.end()), bands.end());
            for (int band : bands) {
                if (band > c->cfg.rows && band != bands[0]) break;
                cand.push_back({var, K, band});
            }
        }
    }
    if (cand.empty()) return;
    golk::StepArgs a{};
    a.width = c->cfg.width;
    a.nw = c->nw;
    a.pitch = c->pitch;
    a.modrows = c->buf_rows;
    a.row_lo = 0;
    a.row_hi = c->buf_rows;
    a.cnt_lo = 0;
    a.cnt_hi = 0;
    a.variant = c->variant;
    a.multi_words = c->multi_words;
    a.wg_prio = c->wg_prio;
    a.err = c->d_err;
    if (golk::launch_fill_random(c->board[0], c->cfg.width, c->nw, c->pitch, c->buf_rows, 0,
                                 c->buf_rows, 12345, c->stream) != hipSuccess)
        return;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess) return;
    if (hipEventCreate(&e1) != hipSuccess) { (void)hipEventDestroy(e0); return; }
    // time `reps` launches of one candidate on the engine's stream, per turn (0 on error)
    auto time_one = [&](const Cand &cd, int reps) -> float {
        a.band = cd.band;
        a.multi_variant = cd.var;
        a.tile_w = cd.tw;
        a.tile_seg = cd.seg;
        bool ok = hipEventRecord(e0, c->stream) == hipSuccess;
        for (int rep = 0; rep < reps && ok; ++rep) {
            a.in = c->board[rep & 1];
            a.out = c->board[(rep + 1) & 1];
            ok = pg_prepare(c, a, cd.K) == hipSuccess &&
                 golk::launch_step_multi(a, cd.K, c->stream) == hipSuccess;
        }
        ok = ok && hipEventRecord(e1, c->stream) == hipSuccess &&
             hipEventSynchronize(e1) == hipSuccess;
        float ms = 0.f;
        if (!ok || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 0.f;
        return ms / ((float)reps * cd.K);
    };
    // the clock ramps over the first milliseconds of load: warm up, then two interleaved
    // passes over the candidates, best of the two per candidate (one pass picked bands
    // 73 / 137 / 218 at 65536^2 on three runs); each candidate times >= ~1 ms of launches
    // (strips of 8192 rows launch in ~50 us)
    std::vector<float> t(cand.size(), 0.f);
    int reps = 3;
    {
        const float us = time_one(cand.back(), 12) * 1000.f * cand.back().K;   // per launch
        if (us > 0.f) reps = std::max(3, std::min(24, (int)(1000.f / us) + 1));
    }
    auto measure = [&](size_t from) {
        for (int pass = 0; pass < 2; ++pass)
            for (size_t i = from; i < cand.size(); ++i) {
                const float v = time_one(cand[i], reps);
                if (v > 0.f && (t[i] == 0.f || v < t[i])) t[i] = v;
            }
    };
    measure(0);
    // refine: the bands next to the best of each (kernel, K) (the coarse list steps by up to
    // 50 %, and a one-round grid's fill changes with every band: 16384^2 parallelogram K = 16
    // ran 3.35 / 3.25 / 3.70 us per turn at bands 43 / 55 / 67)
    {
        const size_t n0 = cand.size();
        for (size_t j = 0; j < n0; ++j) {
            // the best band of each (kernel, K)
            const int var = cand[j].var;
            int bi = -1;
            for (size_t i = 0; i < n0; ++i)
                if (cand[i].var == var && cand[i].K == cand[j].K && t[i] > 0.f &&
                    (bi < 0 || t[i] < t[bi]))
                    bi = (int)i;
            if (bi != (int)j || var == golk::kMultiTile) continue;
            const Cand b = cand[bi];
            const int step = golk::is_pg_variant(var) ? golk::kWgU : std::max(2, b.band / 16);
            for (int d : {-2, -1, 1, 2}) {
                int band = b.band + d * step;
                if (golk::is_pg_variant(var))
                    band = golk::pg_band(b.K, band, var == golk::kMultiWgPgS);
                if (band < 16 || band > std::max(c->cfg.rows, 16)) continue;
                bool seen = false;
                for (const Cand &x : cand)
                    seen |= x.var == var && x.K == b.K && x.band == band;
                if (!seen) {
                    cand.push_back({var, b.K, band, 0, 0});
                    t.push_back(0.f);
                }
            }
        }
        measure(n0);
    }
    float best = 0.f;
    for (size_t i = 0; i < cand.size(); ++i)
        if (t[i] > 0.f && (best == 0.f || t[i] < best)) best = t[i];
    if (getenv("GOL_AUTOTUNE_LOG"))   // tools only: the measured table on stderr
        for (size_t i = 0; i < cand.size(); ++i)
            fprintf(stderr, "autotune %dx%d var=%d K=%d band=%d tile=%d,%d us_per_turn=%.3f "
                    "reps=%d\n", c->cfg.width, c->buf_rows, cand[i].var, cand[i].K, cand[i].band,
                    cand[i].tw, cand[i].seg, t[i] * 1000.f, reps);
    // within 1.5 % of the best, the deepest K wins: the same steady rate with fewer launches
    // when a run is short (65536^2, 20 turns: K = 10 -> 2 launches, 104.7k GCUPS; K = 8 ->
    // 7 + 7 + 6, 100.8k; steady state 36.0 vs 36.2 us/turn)
    Cand pick{c->multi_variant, c->tpl, c->band_multi, c->tile_w, c->tile_seg};
    float pick_t = 0.f;
    for (size_t i = 0; i < cand.size(); ++i) {
        if (t[i] <= 0.f || t[i] > best * 1.015f) continue;
        if (pick_t == 0.f || cand[i].K > pick.K || (cand[i].K == pick.K && t[i] < pick_t)) {
            pick = cand[i];
            pick_t = t[i];
        }
    }
    if (pick_t > 0.f) best = pick_t;
    // Launch planner (tune_k and tune_variant only: nothing pinned).  For each kernel, its
    // fastest (K, band) is a family; time one launch of every family at every depth 2..16
    // (band_same_rounds), then plan, for every t <= kPlanMax turns, the sequence of launches
    // with the least total measured time (plan_launch).  All candidates run on the
    // interleaved layout, so launches of different kernels mix freely.
    std::vector<Launch> plan;
    float stream_best = 0.f;
    if (tune_k && tune_variant && pick_t > 0.f) {
        struct Fam {
            int var, K, band, tw, seg;
            float T[golk::kMaxTurnsPerLaunch + 1];
            int band_k[golk::kMaxTurnsPerLaunch + 1];
        };
        std::vector<Fam> fams;
        for (int var : vars) {
            int bi = -1;
            for (size_t i = 0; i < cand.size(); ++i)
                if (cand[i].var == var && t[i] > 0.f && (bi < 0 || t[i] < t[bi])) bi = (int)i;
            if (bi < 0 || !golk::multi_is_il(c->multi_words, var)) continue;
            Fam f{var, cand[bi].K, cand[bi].band, cand[bi].tw, cand[bi].seg, {}, {}};
            for (int k = 2; k <= golk::kMaxTurnsPerLaunch; ++k) {
                f.T[k] = 0.f;
                f.band_k[k] = 0;
                // (k_step_wg runs depths 2, 3 as k_step_skew: that family covers them; the
                // tile kernel's depth is a runtime loop: it is timed up to 32)
                if ((k > 16 && var != golk::kMultiTile) || !golk::multi_ok(c->cfg.width, k, var) ||
                    (golk::is_wg_variant(var) && k < 4))
                    continue;
                f.band_k[k] = band_same_rounds(c, var, f.K, f.band, k);
                for (int pass = 0; pass < 2; ++pass) {
                    const float v =
                        time_one(Cand{var, k, f.band_k[k], f.tw, f.seg}, reps) * (float)k;
                    if (v > 0.f && (f.T[k] == 0.f || v < f.T[k])) f.T[k] = v;
                }
            }
            fams.push_back(f);
        }
        const float inf = 1e30f;
        std::vector<float> cost(kPlanMax + 1, inf);
        plan.assign(kPlanMax + 1, Launch{});
        cost[0] = 0.f;
        for (int r = 2; r <= kPlanMax; ++r)
            for (const Fam &f : fams)
                for (int k = 2; k <= std::min(r, golk::kMaxTurnsPerLaunch); ++k) {
                    if (f.T[k] <= 0.f || r - k == 1 || cost[r - k] >= inf) continue;
                    const float v = cost[r - k] + f.T[k];
                    if (v < cost[r]) {
                        cost[r] = v;
                        plan[r] = Launch{k, f.var, f.band_k[k], f.tw, f.seg};
                    }
                }
        // K1q for the tile family: 240 turns as one k_tile_stream launch in blocks of Kp
        // turns (one start and one tail instead of one per launch), against the tuned
        // steady rate; kept when >= 2 % faster.  Torus engines only (a strip's halo window
        // shrinks its rows from launch to launch).
        c->stream_k = 0;
        if (!is_strip(c) && !getenv("GOL_NO_STREAM")) {
            const Fam *tf = nullptr;
            for (const Fam &f : fams)
                if (f.var == golk::kMultiTile) tf = &f;
            const int N = 240;
            float sbest = 0.f;
            int sk = 0, sband = 0;
            for (int Kp : {tf ? tf->K : 0, 24}) {
                if (!tf || Kp < 2 || Kp > golk::kMaxTurnsPerLaunch || tf->band_k[Kp] <= 0)
                    continue;
                // equal tile rows (the same count): a last tile row shorter than K would take
                // its halo from two tile rows up
                const int nty = (c->buf_rows + tf->band_k[Kp] - 1) / tf->band_k[Kp];
                const int th = (c->buf_rows + nty - 1) / nty;
                if (!golk::tile_stream_ok(c->nw, c->buf_rows, Kp, th, tf->tw, tf->seg)) continue;
                a.band = th;
                a.multi_variant = golk::kMultiTile;
                a.tile_w = tf->tw;
                a.tile_seg = tf->seg;
                a.in = c->board[0];
                a.out = c->board[1];
                float v = 0.f;
                for (int pass = 0; pass < 3; ++pass) {
                    float ms = 0.f;
                    const bool ok = hipEventRecord(e0, c->stream) == hipSuccess &&
                                    stream_launch(c, a, N, Kp) == hipSuccess &&
                                    hipEventRecord(e1, c->stream) == hipSuccess &&
                                    hipEventSynchronize(e1) == hipSuccess &&
                                    hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
                    if (ok && (v == 0.f || ms / N < v)) v = ms / N;
                }
                if (getenv("GOL_AUTOTUNE_LOG"))
                    fprintf(stderr, "autotune stream %dx%d K=%d band=%d tile=%d,%d us_per_turn=%.3f "
                            "(tuned %.3f)\n", c->cfg.width, c->buf_rows, Kp, a.band, tf->tw, tf->seg,
                            v * 1000.f, best * 1000.f);
                if (v > 0.f && (sbest == 0.f || v < sbest)) {
                    sbest = v;
                    sk = Kp;
                    sband = a.band;
                }
            }
            // (a wait that gave up while timing: no K1q, and the junk board's error word is
            // cleared -- the board is refilled before use)
            const bool bad = check_dev_err(c) != GOL_OK;
            if (bad) clear_dev_err(c);
            if (sk && sbest < 0.98f * best && !bad) {
                c->stream_k = sk;
                c->stream_tw = tf->tw;
                c->stream_th = sband;
                c->stream_seg = tf->seg;
                stream_best = sbest;
            }
        }
        // Short steps (r <= kSeqMax turns, e.g. the bench's 20-turn call): the DP adds
        // back-to-back launch times, but a gol_step of r turns starts from a synchronised
        // stream, and two plans within a few % of each other by the sum traded places as the
        // bench's single timed call (65536^2 x 20: 2 x k_step_skew K = 10 vs 1 x k_step_tile
        // K = 20, profiles/r03b_plan_choice.log).  So for every r the DP's plan, the best plan
        // of each family alone and each family's single launch of depth r are timed as whole
        // sequences the way gol_step runs them -- host wall time from a synchronised stream
        // to the last launch's completion, best of 5, candidates interleaved -- and the
        // fastest is kept in seq[r].
        std::vector<std::vector<Launch>> seqs(kSeqMax + 1);
        {
            auto chain = [&](const std::vector<Launch> &pl, int r) {
                std::vector<Launch> out;
                for (int q = r; q >= 2 && pl[q].k >= 2; q -= pl[q].k) out.push_back(pl[q]);
                int n = 0;
                for (const Launch &L : out) n += L.k;
                if (n != r) out.clear();
                return out;
            };
            std::vector<std::vector<Launch>> fam_plan;
            for (const Fam &f : fams) {
                std::vector<float> cf(kSeqMax + 1, inf);
                std::vector<Launch> pf(kSeqMax + 1, Launch{});
                cf[0] = 0.f;
                for (int r = 2; r <= kSeqMax; ++r)
                    for (int k = 2; k <= std::min(r, golk::kMaxTurnsPerLaunch); ++k) {
                        if (f.T[k] <= 0.f || r - k == 1 || cf[r - k] >= inf) continue;
                        if (cf[r - k] + f.T[k] < cf[r]) {
                            cf[r] = cf[r - k] + f.T[k];
                            pf[r] = Launch{k, f.var, f.band_k[k], f.tw, f.seg};
                        }
                    }
                fam_plan.push_back(std::move(pf));
            }
            auto same = [](const std::vector<Launch> &x, const std::vector<Launch> &y) {
                if (x.size() != y.size()) return false;
                for (size_t i = 0; i < x.size(); ++i)
                    if (x[i].k != y[i].k || x[i].var != y[i].var || x[i].band != y[i].band ||
                        x[i].tw != y[i].tw || x[i].seg != y[i].seg || x[i].blk != y[i].blk)
                        return false;
                return true;
            };
            auto time_seq = [&](const std::vector<Launch> &sq) -> float {
                if (hipStreamSynchronize(c->stream) != hipSuccess) return 0.f;
                const auto t0 = std::chrono::steady_clock::now();
                bool ok = true;
                int rep = 0;
                for (const Launch &L : sq) {
                    a.band = L.band;
                    a.multi_variant = L.var == golk::kMultiTileStream ? golk::kMultiTile : L.var;
                    a.tile_w = L.tw;
                    a.tile_seg = L.seg;
                    a.in = c->board[rep & 1];
                    a.out = c->board[(rep + 1) & 1];
                    ++rep;
                    if (L.var == golk::kMultiTileStream)
                        ok = ok && stream_launch(c, a, L.k, L.blk) == hipSuccess;
                    else
                        ok = ok && pg_prepare(c, a, L.k) == hipSuccess &&
                             golk::launch_step_multi(a, L.k, c->stream) == hipSuccess;
                }
                ok = ok && hipStreamSynchronize(c->stream) == hipSuccess;
                const std::chrono::duration<float, std::micro> d =
                    std::chrono::steady_clock::now() - t0;
                return ok ? d.count() : 0.f;
            };
            for (int r = 2; r <= kSeqMax; ++r) {
                std::vector<std::vector<Launch>> cands;
                auto add = [&](std::vector<Launch> sq) {
                    if (sq.empty()) return;
                    for (const auto &x : cands)
                        if (same(x, sq)) return;
                    cands.push_back(std::move(sq));
                };
                add(chain(plan, r));
                // K1q (when tuned): the r turns as one launch of 2 or 3 near-equal blocks --
                // shallower blocks carry fewer halo rows, and the launch starts only once
                if (c->stream_k > 0)
                    for (int nb : {2, 3}) {
                        const int blk = (r + nb - 1) / nb;
                        if (blk >= 4 && golk::tile_stream_ok(c->nw, c->buf_rows, blk, c->stream_th,
                                                             c->stream_tw, c->stream_seg))
                            add({Launch{r, golk::kMultiTileStream, c->stream_th, c->stream_tw,
                                        c->stream_seg, blk}});
                    }
                for (size_t fi = 0; fi < fams.size(); ++fi) {
                    add(chain(fam_plan[fi], r));
                    if (r <= golk::kMaxTurnsPerLaunch && fams[fi].T[r] > 0.f)
                        add({Launch{r, fams[fi].var, fams[fi].band_k[r], fams[fi].tw,
                                    fams[fi].seg}});
                }
                if (cands.size() <= 1) {
                    if (!cands.empty()) seqs[r] = cands[0];
                    continue;
                }
                std::vector<float> tt(cands.size(), 0.f);
                for (int pass = 0; pass < 5; ++pass)
                    for (size_t i = 0; i < cands.size(); ++i) {
                        const float v = time_seq(cands[i]);
                        if (v > 0.f && (tt[i] == 0.f || v < tt[i])) tt[i] = v;
                    }
                size_t bi = 0;
                for (size_t i = 1; i < cands.size(); ++i)
                    if (tt[i] > 0.f && (tt[bi] == 0.f || tt[i] < tt[bi])) bi = i;
                if (tt[bi] > 0.f) seqs[r] = cands[bi];
                if (getenv("GOL_AUTOTUNE_LOG") && (r == 8 || r == 16 || r == 20 || r == 32))
                    for (size_t i = 0; i < cands.size(); ++i) {
                        fprintf(stderr, "autotune seq %d turns%s %.1f us =", r,
                                i == bi ? " (pick)" : "", tt[i]);
                        for (const Launch &L : cands[i])
                            fprintf(stderr, " %d(var %d, band %d, tile %d,%d, blk %d)", L.k,
                                    L.var, L.band, L.tw, L.seg, L.blk);
                        fprintf(stderr, "\n");
                    }
            }
        }
        c->seq = std::move(seqs);
        if (getenv("GOL_AUTOTUNE_LOG")) {
            for (const Fam &f : fams)
                for (int k = 2; k <= golk::kMaxTurnsPerLaunch; ++k)
                    if (f.T[k] > 0.f)
                        fprintf(stderr, "autotune launch var=%d K=%d band=%d us=%.1f\n", f.var, k,
                                f.band_k[k], f.T[k] * 1000.f);
            for (int r : {8, 16, 20, 32, 64, 128})
                if (r <= kPlanMax) {
                    fprintf(stderr, "autotune plan %d turns: %.1f us =", r, cost[r] * 1000.f);
                    for (int q = r; q >= 2 && plan[q].k >= 2; q -= plan[q].k)
                        fprintf(stderr, " %d(var %d, band %d)", plan[q].k, plan[q].var, plan[q].band);
                    fprintf(stderr, "\n");
                }
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipGetLastError();
    c->multi_variant = pick.var;
    c->tpl = pick.K;
    c->band_multi = pick.band;
    if (pick.var == golk::kMultiTile) {
        c->tile_w = pick.tw;
        c->tile_seg = pick.seg;
    }
    for (int &b : c->band_at) b = 0;
    if (plan.empty()) c->seq.clear();
    c->plan = std::move(plan);
    c->tuned_us_per_turn = (stream_best > 0.f ? stream_best : best) * 1000.f;
}

}  // namespace

// ================================================================ C ABI
extern "C" {

const char *gol_strerror(int code)
{
    switch (code) {
    case GOL_OK: return "ok";
    case GOL_EINVAL: return "invalid argument";
    case GOL_EHIP: return "HIP runtime error";
    case GOL_ENOMEM: return "out of memory";
    case GOL_ESTATE: return "invalid state";
    case GOL_ENODEV: return "no HIP device";
    case GOL_EIO: return "I/O error";
    case GOL_ECLOSED: return "channel closed";
    case GOL_ETIMEDOUT: return "timed out";
    default: return "unknown error";
    }
}

const char *gol_last_error(const gol_ctx *ctx) { return ctx ? ctx->err.c_str() : ""; }

int gol_create(int32_t width, int32_t height, uint32_t flags, gol_ctx **out)
{
    gol_config cfg{};
    cfg.width = width;
    cfg.height = height;
    cfg.device = -1;
    cfg.row_offset = 0;
    cfg.rows = height;
    cfg.halo = 0;
    cfg.flags = flags;
    cfg.band_rows = 0;
    return gol_create_ex(&cfg, out);
}

int gol_create_ex(const gol_config *cfg, gol_ctx **out)
{
    if (!cfg || !out) return GOL_EINVAL;
    *out = nullptr;
    if (cfg->width < 2 || cfg->height < 1 || cfg->rows < 1 || cfg->halo < 0) return GOL_EINVAL;
    if (cfg->halo == 0 && (cfg->rows != cfg->height || cfg->row_offset != 0)) return GOL_EINVAL;
    if (cfg->halo > 0 && (cfg->halo > cfg->rows || cfg->row_offset < 0 ||
                          cfg->row_offset + cfg->rows > cfg->height))
        return GOL_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return GOL_ENODEV;
    int dev = cfg->device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return GOL_ENODEV;
    if (dev >= ndev) return GOL_ENODEV;

    gol_ctx *c = new (std::nothrow) gol_ctx();
    if (!c) return GOL_ENOMEM;
    c->cfg = *cfg;
    c->cfg.device = dev;
    c->device = dev;
    c->nw = (cfg->width + 63) / 64;
    c->pitch = c->nw;
    c->buf_rows = cfg->rows + 2 * cfg->halo;
    c->fast = golk::fast_path_ok(cfg->width) && !(cfg->flags & GOL_FLAG_FORCE_GENERIC);
    c->band = cfg->band_rows > 0 ? cfg->band_rows : golk::auto_band(cfg->width, cfg->rows);
    if (const char *v = getenv("GOL_STENCIL_VARIANT")) {   // A/B experiments only
        const int k = atoi(v);
        if (k >= 0 && k < golk::kVariantCount) c->variant = k;
    }
    // temporal blocking defaults (tools/sweep.py on MI355X): 1 word per lane (more waves,
    // 87 VGPRs at K=4), K = 6 on large boards (64-row bands), K = 4 on smaller ones
    c->multi_words = 1;
    if (const char *v = getenv("GOL_MULTI_WORDS")) c->multi_words = atoi(v) == 1 ? 1 : 2;
    if (!GOL_TOOLS && c->multi_words != 1) {  // 2 words per lane: a superseded build
        delete c;
        return GOL_EINVAL;
    }
    if (const char *v = getenv("GOL_WG_PRIO")) {          // A/B experiments only: "3210" =
        for (int w = 0; w < 4 && v[w] >= '0' && v[w] <= '3'; ++w)   // wave 0..3's priority
            c->wg_prio |= (unsigned)(v[w] - '0') << (2 * w);
        if (!c->wg_prio) c->wg_prio = 0x100;              // all zero: still an override
    }
    if (const char *v = getenv("GOL_MULTI_VARIANT")) {    // A/B experiments only
        const int k = atoi(v);
        const bool known = (k >= 0 && k < golk::kMultiUserEnd) || k > golk::kMultiAblate;
        // the product library ships only the kernels that compute the right board
        // (multi_variant_shipped); ablations, diagnostics and superseded variants need the
        // tools build (libgolamd_tools.so via GOL_AMD_LIB)
        if (!known || (!GOL_TOOLS && !golk::multi_variant_shipped(k))) {
            delete c;
            return GOL_EINVAL;
        }
        c->multi_variant = k;
    }
    const int lane_dw = golk::multi_lane_dwords(c->multi_words, c->multi_variant);
    const int auto_bm = golk::auto_band_multi(cfg->width, cfg->rows, lane_dw);
    const bool wg = golk::is_wg_variant(c->multi_variant);
    c->tpl = cfg->turns_per_launch > 0 ? cfg->turns_per_launch
                                       : (wg ? 16 : (auto_bm >= 48 ? 8 : 6));
    if (const char *v = getenv("GOL_TURNS_PER_LAUNCH")) c->tpl = atoi(v);
    c->tpl = std::max(1, std::min(c->tpl, golk::multi_max_turns(c->multi_variant)));
    if (c->fast && c->tpl > 1 && !golk::multi_fits(c->nw, c->pitch, c->buf_rows))
        c->blocking_limited = true;   // reported in gol_info.blocking_limited
    if (!c->fast || c->blocking_limited) c->tpl = 1;
    c->halo_valid = cfg->halo;

    DeviceGuard g(dev);
    (void)hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, dev);
    c->band_multi = cfg->band_rows;
    if (c->band_multi <= 0 && c->tpl > 1) {
        const int ncu = c->ncu;
        const int bpc = golk::multi_blocks_per_cu(c->tpl, c->multi_words, c->multi_variant);
        c->band_multi = golk::pick_band_multi(cfg->width, cfg->rows, lane_dw, c->tpl,
                                              ncu * bpc *
                                                  golk::multi_pipes_per_block(c->multi_variant),
                                              c->multi_variant);
    }
    if (c->band_multi <= 0) c->band_multi = golk::auto_band_multi(cfg->width, cfg->rows, lane_dw);
    const size_t words = (size_t)c->buf_rows * c->pitch;
    int rc = GOL_OK;
    auto bail = [&](int code) {
        gol_destroy(c);
        return code;
    };
    hipError_t e;
    if ((e = hipMalloc(&c->board[0], words * 8)) != hipSuccess ||
        (e = hipMalloc(&c->board[1], words * 8)) != hipSuccess ||
        (e = hipMalloc(&c->counts, (size_t)(kRing + 1) * kShards * 8)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_counts, kShards * 8, hipHostMallocDefault)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->ev_side, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->ev_main, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->ev_copy, hipEventDisableTiming)) != hipSuccess ||
        (e = hipHostMalloc((void **)&c->h_err, sizeof(unsigned),
                           hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&c->d_err, c->h_err, 0)) != hipSuccess) {
        rc = e == hipErrorOutOfMemory ? GOL_ENOMEM : GOL_EHIP;
        return bail(rc);
    }
    clear_dev_err(c);
    {
        std::lock_guard<std::mutex> lk(g_dev_mu);
        ++g_dev_engines[dev];
        c->registered = true;
    }
    c->stream = c->own_stream;
    // small boards (and k_step_tile pinned by GOL_MULTI_VARIANT): k_step_tile at the model's
    // best shape for the requested or default depth; the autotune below times the model's best
    // shapes
    const bool small = c->fast && c->tpl > 1 && (long long)c->buf_rows * c->pitch < (1ll << 20);
    const bool pinned = getenv("GOL_MULTI_VARIANT") != nullptr;
    if (c->fast && c->tpl > 1 &&
        ((small && !pinned && cfg->band_rows <= 0) || c->multi_variant == golk::kMultiTile)) {
        int K = cfg->turns_per_launch > 0 ? std::min(cfg->turns_per_launch, golk::kMaxTileTurns) : 0;
        if (const char *v = getenv("GOL_TURNS_PER_LAUNCH"))
            K = std::max(2, std::min(atoi(v), golk::kMaxTileTurns));
        std::vector<TileShape> cand = tile_candidates(c->ncu, c->nw, c->buf_rows, 1 << 20);
        for (const TileShape &t : cand)
            if (K == 0 || t.K == K) {
                apply_tile(c, t);
                break;
            }
        if (K > 0 && c->multi_variant == golk::kMultiTile && c->tpl != K) {
            // no ranked shape at this depth (K not in the candidate list): best TW / TH at K
            TileShape best;
            for (const TileShape &t : cand) {
                const double m = tile_model_us(c->ncu, c->nw, c->buf_rows, K, t.th, t.tw, t.seg);
                if (m > 0 && (best.K == 0 || m < best.model_us)) best = {K, t.th, t.tw, t.seg, m};
            }
            if (best.K) apply_tile(c, best);
        }
        if (c->multi_variant == golk::kMultiTile && cfg->band_rows > 0)
            c->band_multi = cfg->band_rows;  // tile height pinned by the caller
        if (const char *v = getenv("GOL_TILE")) {           // experiments: "TW,SEG"
            int tw = 0, seg = 0;
            if (sscanf(v, "%d,%d", &tw, &seg) == 2 && tw > 0 && seg > 0) {
                c->multi_variant = golk::kMultiTile;
                c->tile_w = tw;
                c->tile_seg = seg;
            }
        }
        if (c->multi_variant == golk::kMultiTile &&
            !golk::tile_shape_ok(c->nw, c->tpl, c->band_multi, c->tile_w, c->tile_seg))
            return bail(GOL_EINVAL);
        if (const char *v = getenv("GOL_PERSIST")) {       // tests / experiments: K1p blocks
            const int pk = atoi(v);
            if (pk > 0) {
                const char *rv = getenv("GOL_RING");
                const bool ring = rv && atoi(rv) > 0;
                if (c->multi_variant != golk::kMultiTile || is_strip(c) ||
                    !(ring ? golk::tile_ring_ok(c->nw, c->buf_rows, pk, c->band_multi, c->tile_w,
                                                c->tile_seg, c->ncu)
                           : golk::tile_persist_ok(c->nw, c->buf_rows, 2 * pk, pk, c->band_multi,
                                                   c->tile_w, c->tile_seg, c->ncu)))
                    return bail(GOL_EINVAL);
                c->persist_k = pk;
                c->persist_forced = true;
                c->persist_ring = ring;
            }
        }
        if (const char *v = getenv("GOL_STREAM")) {        // tests / experiments: K1q blocks
            const int sk = atoi(v);
            if (sk > 0) {
                if (c->multi_variant != golk::kMultiTile || is_strip(c) ||
                    !golk::tile_stream_ok(c->nw, c->buf_rows, sk, c->band_multi, c->tile_w,
                                          c->tile_seg))
                    return bail(GOL_EINVAL);
                c->stream_k = sk;
                c->stream_forced = true;
                c->stream_tw = c->tile_w;
                c->stream_th = c->band_multi;
                c->stream_seg = c->tile_seg;
            }
        }
    }
    const char *at = getenv("GOL_AUTOTUNE");
    bool tuning = !(cfg->flags & GOL_FLAG_NO_AUTOTUNE) && (!at || atoi(at) != 0) &&
                  cfg->band_rows <= 0 && c->tpl > 1;
    // a BASELINE board size on an MI355X: the pinned shape, no search (GOL_AUTOTUNE=2: search);
    // the first engine of the shape in this process times it once (check_pinned: a warning
    // when slow, never a different shape)
    KnownShape ks{};
    if (tuning && !pinned && cfg->turns_per_launch <= 0 && !getenv("GOL_TILE") &&
        !(at && atoi(at) == 2) && known_shape(c, &ks)) {
        apply_tile(c, ks.t);
        if (ks.short_K >= 2 && ks.short_K < ks.t.K &&
            golk::tile_shape_ok(c->nw, ks.short_K, ks.short_th, ks.t.tw, ks.t.seg)) {
            c->short_k = ks.short_K;
            c->short_band = ks.short_th;
        }
        c->tuned_us_per_turn = ks.us_per_turn;
        c->shape_source = 2;
        tuning = false;
        (void)check_pinned(c, ks);
    }
    const bool tune_small = small && c->multi_variant == golk::kMultiTile && !pinned &&
                            cfg->turns_per_launch <= 0;
    // the kernel is tuned too unless an experiment pins it (GOL_MULTI_VARIANT) or the requested
    // depth only one of them runs
    const bool tune_var = !pinned && c->multi_words == 1 &&
                          (cfg->turns_per_launch <= 0 || cfg->turns_per_launch <= 8);
    const TuneKey key{dev, cfg->width, c->buf_rows, cfg->turns_per_launch,
                      (tune_small ? 4 : 0) | (tune_var ? 2 : 0) | (pinned ? 1 : 0) |
                          (c->multi_variant << 3)};
    const char *tc = getenv("GOL_AUTOTUNE_CACHE");
    const bool use_cache = !tc || atoi(tc) != 0;
    bool cached = false;
    if (tuning && use_cache) {
        std::lock_guard<std::mutex> lk(g_tune_mu);
        auto it = g_tune.find(key);
        if (it != g_tune.end()) {
            const TuneVal &v = it->second;
            c->multi_variant = v.var;
            c->tpl = v.tpl;
            c->band_multi = v.band;
            c->tile_w = v.tile_w;
            c->tile_seg = v.tile_seg;
            c->persist_k = v.persist_k;
            c->persist_seg = v.persist_seg;
            c->stream_k = v.stream_k;
            c->stream_tw = v.stream_tw;
            c->stream_th = v.stream_th;
            c->stream_seg = v.stream_seg;
            c->plan = v.plan;
            c->seq = v.seq;
            c->tuned_us_per_turn = v.us;
            for (int &b : c->band_at) b = 0;
            c->shape_source = 1;
            cached = true;
        }
    }
    if (tuning && !cached && (tune_small || !small)) {
        if (tune_small) autotune_small(c);
        else autotune_multi(c, cfg->turns_per_launch <= 0, tune_var);
        c->shape_source = 1;
        // a wait that gave up while timing the candidates: fail loudly at create
        (void)hipStreamSynchronize(c->stream);
        if (check_dev_err(c)) return bail(GOL_EHIP);
        if (use_cache) {
            std::lock_guard<std::mutex> lk(g_tune_mu);
            g_tune[key] = TuneVal{c->multi_variant, c->tpl, c->band_multi, c->tile_w,
                                  c->tile_seg, c->persist_k, c->persist_seg, c->stream_k, c->stream_tw,
                                  c->stream_th, c->stream_seg, c->tuned_us_per_turn, c->plan,
                                  c->seq};
        }
    }
    if ((e = hipMemsetAsync(c->board[0], 0, words * 8, c->stream)) != hipSuccess ||
        (e = hipMemsetAsync(c->board[1], 0, words * 8, c->stream)) != hipSuccess ||
        (e = hipMemsetAsync(c->counts, 0, (size_t)(kRing + 1) * kShards * 8, c->stream)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return bail(GOL_EHIP);
    *out = c;
    return GOL_OK;
}

void gol_destroy(gol_ctx *c)
{
    if (!c) return;
    if (c->registered) {
        std::lock_guard<std::mutex> lk(g_dev_mu);
        if (--g_dev_engines[c->device] <= 0) g_dev_engines.erase(c->device);
    }
    {
        DeviceGuard g(c->device);
        if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
        if (c->stream && c->stream != c->own_stream) (void)hipStreamSynchronize(c->stream);
        if (c->side) (void)hipStreamSynchronize(c->side);
        if (c->board[0]) (void)hipFree(c->board[0]);
        if (c->board[1]) (void)hipFree(c->board[1]);
        if (c->pg_rows) (void)hipFree(c->pg_rows);
        if (c->pg_flags) (void)hipFree(c->pg_flags);
        for (auto *u : c->pu)
            if (u) (void)hipFree(u);
        for (auto *u : c->su)
            if (u) (void)hipFree(u);
        if (c->pcounter) (void)hipFree(c->pcounter);
        if (c->pflags) (void)hipFree(c->pflags);
        if (c->blocked) (void)hipFree(c->blocked);
        if (c->counts) (void)hipFree(c->counts);
        if (c->staging) (void)hipFree(c->staging);
        if (c->h_counts) (void)hipHostFree(c->h_counts);
        if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
        if (c->side) (void)hipStreamDestroy(c->side);
        if (c->ev_side) (void)hipEventDestroy(c->ev_side);
        if (c->ev_main) (void)hipEventDestroy(c->ev_main);
        if (c->ev_copy) (void)hipEventDestroy(c->ev_copy);
        if (c->h_err) (void)hipHostFree(c->h_err);
    }
    delete c;
}

int gol_get_info(gol_ctx *c, gol_info *info)
{
    if (!c || !info) return GOL_EINVAL;
    return run_read(c, [&]() -> int {
        info->width = c->cfg.width;
        info->height = c->cfg.height;
        info->row_offset = c->cfg.row_offset;
        info->rows = c->cfg.rows;
        info->halo = c->cfg.halo;
        info->words_per_row = c->nw;
        info->pitch_words = c->pitch;
        info->buffer_rows = c->buf_rows;
        info->fast_path = c->fast ? 1 : 0;
        info->band_rows = c->tpl > 1 ? c->band_multi : c->band;   // band of the kernel in use
        info->halo_valid = c->halo_valid;
        info->turns_per_launch = c->tpl;
        info->device = c->device;
        info->turn = c->turn;
        info->nonbinary_cells = c->nonbinary;
        info->launches = c->launches;
        info->blocking_limited = c->blocking_limited ? 1 : 0;
        info->shape_source = c->shape_source;
        return GOL_OK;
    });
}

int gol_set_stream(gol_ctx *c, void *s)
{
    if (!c) return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    // order the switch: everything queued on the old stream completes first
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return GOL_OK;
}

void *gol_get_stream(gol_ctx *c) { return c ? (void *)c->stream : nullptr; }

int gol_sync(gol_ctx *c)
{
    if (!c) return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    return sync_checked(c);
}

int gol_load(gol_ctx *c, const uint8_t *bytes)
{
    if (!c || !bytes) return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    const int W = c->cfg.width;
    const size_t row_bytes = (size_t)W;
    int chunk_rows = (int)std::max<size_t>(1, std::min<size_t>(kStagingBytes / row_bytes,
                                                               (size_t)c->buf_rows));
    int rc = ensure_staging(c, (size_t)chunk_rows * row_bytes);
    if (rc) return rc;
    release_blocked(c);
    const size_t words = (size_t)c->buf_rows * c->pitch;
    HIP_OR_FAIL(c, hipMalloc(&c->blocked, words * 8));
    unsigned long long *nb = c->counts + (size_t)kRing * kShards;
    HIP_OR_FAIL(c, hipMemsetAsync(nb, 0, kShards * 8, c->stream));
    uint64_t *dst = c->board[0];
    for (int r0 = 0; r0 < c->buf_rows; r0 += chunk_rows) {
        const int nr = std::min(chunk_rows, c->buf_rows - r0);
        HIP_OR_FAIL(c, hipMemcpyAsync(c->staging, bytes + (size_t)r0 * row_bytes,
                                      (size_t)nr * row_bytes, hipMemcpyHostToDevice, c->stream));
        HIP_OR_FAIL(c, golk::launch_pack(c->staging, W, nr, dst, c->blocked, c->nw, c->pitch, r0,
                                         nb, c->stream));
    }
    HIP_OR_FAIL(c, hipMemcpyAsync(c->h_counts, nb, kShards * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    unsigned long long s = 0;
    for (int i = 0; i < kShards; i++) s += c->h_counts[i];
    c->nonbinary = (long long)s;
    c->cur = 0;
    c->il = false;
    clear_dev_err(c);                        // a new board: earlier hand-off failures are moot
    c->turn = 0;
    c->progress.store(0);
    c->launches = 0;
    c->halo_valid = c->cfg.halo;
    c->raw_turn0.clear();
    if (s == 0) {
        release_blocked(c);
    } else {
        c->blocked_pending = true;
        // the reference returns the raw bytes unchanged at Turns = 0 (Server loop never runs)
        const size_t own_bytes = (size_t)c->cfg.rows * row_bytes;
        c->raw_turn0.assign(bytes + (size_t)own_lo(c) * row_bytes,
                            bytes + (size_t)own_lo(c) * row_bytes + own_bytes);
    }
    return GOL_OK;
}

int gol_load_packed(gol_ctx *c, const uint64_t *words)
{
    if (!c || !words) return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    release_blocked(c);
    HIP_OR_FAIL(c, hipMemcpy2DAsync(c->board[0], (size_t)c->pitch * 8, words, (size_t)c->nw * 8,
                                    (size_t)c->nw * 8, c->buf_rows, hipMemcpyHostToDevice,
                                    c->stream));
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    c->cur = 0;
    c->il = false;
    clear_dev_err(c);                        // a new board: earlier hand-off failures are moot
    c->turn = 0;
    c->progress.store(0);
    c->launches = 0;
    c->nonbinary = 0;
    c->raw_turn0.clear();
    c->halo_valid = c->cfg.halo;
    return GOL_OK;
}

int gol_fill_random(gol_ctx *c, uint64_t seed)
{
    if (!c) return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    release_blocked(c);
    const long long grow0 = (long long)c->cfg.row_offset - c->cfg.halo;
    HIP_OR_FAIL(c, golk::launch_fill_random(c->board[0], c->cfg.width, c->nw, c->pitch,
                                            c->buf_rows, grow0, c->cfg.height, seed, c->stream));
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    c->cur = 0;
    c->il = false;
    clear_dev_err(c);                        // a new board: earlier hand-off failures are moot
    c->turn = 0;
    c->progress.store(0);
    c->launches = 0;
    c->nonbinary = 0;
    c->raw_turn0.clear();
    c->halo_valid = c->cfg.halo;
    return GOL_OK;
}

namespace {

#if GOL_TOOLS
// Tools build only (GOL_MULTI_VARIANT=kMultiWgDiag): one k_step_wg launch with per-wave wait
// timing, summarised by wave role on stderr.
int wg_diag_launch(gol_ctx *c, golk::StepArgs a, int k)
{
    const long long ntx = golk::multi_tiles(c->cfg.width, 2);
    const long long pipes = ntx * ((a.row_hi - a.row_lo + a.band - 1) / a.band);
    const size_t n = (size_t)pipes * 4 * 10;
    unsigned long long *d = nullptr;
    HIP_OR_FAIL(c, hipMalloc(&d, n * 8));
    HIP_OR_FAIL(c, hipMemsetAsync(d, 0, n * 8, c->stream));
    a.counts = d;
    HIP_OR_FAIL(c, golk::launch_step_multi(a, k, c->stream));
    std::vector<unsigned long long> h(n);
    HIP_OR_FAIL(c, hipMemcpyAsync(h.data(), d, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    (void)hipFree(d);
    unsigned long long t0min = ~0ull, t1max = 0;
    std::vector<unsigned long long> starts, ends;        // wave 0's start / wave 3's end
    for (long long p = 0; p < pipes; ++p)
        for (int w = 0; w < 4; ++w) {
            const unsigned long long *e = &h[((size_t)p * 4 + w) * 10];
            if (e[8] == 0) continue;                     // a workgroup past the last band
            t0min = std::min(t0min, e[8]);
            t1max = std::max(t1max, e[9]);
            if (w == 0) starts.push_back(e[8]);
            if (w == 3) ends.push_back(e[9]);
        }
    auto pct = [](std::vector<unsigned long long> v, unsigned long long base, double q) {
        if (v.empty()) return 0.0;
        std::sort(v.begin(), v.end());
        return (double)(v[(size_t)(q * (double)(v.size() - 1))] - base);
    };
    fprintf(stderr,
            "wg_diag starts (100 MHz ticks after the first) p10 %.0f p50 %.0f p90 %.0f max %.0f; "
            "ends p10 %.0f p50 %.0f p90 %.0f max %.0f\n",
            pct(starts, t0min, 0.1), pct(starts, t0min, 0.5), pct(starts, t0min, 0.9),
            pct(starts, t0min, 1.0), pct(ends, t0min, 0.1), pct(ends, t0min, 0.5),
            pct(ends, t0min, 0.9), pct(ends, t0min, 1.0));
    for (int w = 0; w < 4; ++w) {
        double life = 0, first = 0, fw = 0, nf = 0, ew = 0, ne = 0, nl = 0;
        for (long long p = 0; p < pipes; ++p) {
            const unsigned long long *e = &h[((size_t)p * 4 + w) * 10];
            life += (double)e[0]; first += (double)e[1]; fw += (double)e[2];
            nf += (double)e[3]; ew += (double)e[4]; ne += (double)e[5]; nl += (double)e[6];
        }
        fprintf(stderr,
                "wg_diag K=%d band=%d pipes=%lld wave %d: life %.0f ticks, first-row wait %.1f%%, "
                "fetch waits %.1f%% (%.2f per row), emit waits %.1f%% (%.2f per row)\n",
                k, a.band, pipes, w, life / pipes, 100 * first / life, 100 * fw / life, nf / nl,
                100 * ew / life, ne / nl);
    }
    fprintf(stderr, "wg_diag launch span %llu ticks of 100 MHz\n", t1max - t0min);
    return GOL_OK;
}
#endif  // GOL_TOOLS

constexpr int kCtlDepth = 2;   // launches queued ahead while a control word is in use

// gol_step / gol_step_overlap.  xstream != null: the first launch is split -- the rows
// whose k-turn dependency cone stays inside the owned rows run on the engine stream at
// once, the rows next to the halos run on the side stream after everything queued on
// xstream (the caller's halo receives) -- and the engine stream joins the side stream
// before the next launch.
int step_impl(gol_ctx *c, int64_t turns, hipStream_t xstream,
              std::unique_lock<std::recursive_mutex> &lk)
{
    if (is_strip(c) && turns > c->halo_valid)
        return fail(c, GOL_ESTATE, "strip engine: %lld turns requested, halos valid for %d",
                    (long long)turns, c->halo_valid);
    DeviceGuard g(c->device);
    const bool cnt = (c->cfg.flags & GOL_FLAG_COUNT_EVERY_TURN) != 0;
    golk::StepArgs a{};
    a.width = c->cfg.width;
    a.nw = c->nw;
    a.pitch = c->pitch;
    a.modrows = c->buf_rows;
    a.cnt_lo = own_lo(c);
    a.cnt_hi = own_hi(c);
    a.band = c->band;
    a.variant = c->variant;
    a.multi_words = c->multi_words;
    a.wg_prio = c->wg_prio;
    a.multi_variant = c->multi_variant;
    a.err = c->d_err;
    a.tile_w = c->tile_w;
    a.tile_seg = c->tile_seg;
    // read-only calls from other threads are served at launch boundaries from here on
    struct Stepping {
        gol_ctx *c;
        explicit Stepping(gol_ctx *c_) : c(c_) { set_stepping(c, true); }
        ~Stepping()
        {
            set_stepping(c, false);          // later readers take the lock themselves
            serve_jobs(c);
        }
    } stepping(c);
    // control word: with a controlling thread present, keep at most kCtlDepth launches
    // queued so a pause / stop takes effect within that many launches (and so does a reader:
    // once one has been served during a step, steps keep the queue this short)
    struct EventRing {
        hipEvent_t ev[kCtlDepth] = {};
        int n = 0;
        ~EventRing()
        {
            for (int i = 0; i < std::min(n, kCtlDepth); ++i) (void)hipEventDestroy(ev[i]);
        }
    } ring;
    const bool ctl = c->control_used.load();
    // a reader served during an earlier step does not shorten this one's queue: the bound
    // comes back when a reader is served during this step (a ticker's snapshot)
    c->readers.store(false);
    // a short torus step runs the sequence the autotune timed for exactly this many turns
    const std::vector<Launch> *fixed =
        !is_strip(c) && !cnt && !c->blocked_pending && turns >= 2 && turns <= kSeqMax &&
                turns < (int64_t)c->seq.size() && !c->seq[turns].empty()
            ? &c->seq[turns]
            : nullptr;
    size_t fi = 0;
    c->last.clear();
    c->last_n = 0;
    for (int64_t t = 0; t < turns;) {
        if (c->jobs_pending.load(std::memory_order_relaxed)) serve_jobs(c);
        if (ctl) {
            int w = c->control.load();
            if (w == GOL_CONTROL_PAUSE) {
                // park at this launch boundary with the board complete (Server/gol/
                // distributor.go:147-156: the turn loop blocks until the second 'p'); the
                // engine is released while parked, so AliveCellsCount / GetWorld calls from
                // other threads run at once (the reference's ticker keeps firing while paused,
                // Local/gol/distributor.go:117-130,154-167)
                if (int rc = sync_checked(c)) return rc;
                set_stepping(c, false);
                serve_jobs(c);
                c->parked.store(true);
                lk.unlock();
                while ((w = c->control.load()) == GOL_CONTROL_PAUSE)
                    std::this_thread::sleep_for(std::chrono::microseconds(200));
                lk.lock();
                set_stepping(c, true);
                c->parked.store(false);
            }
            if (w == GOL_CONTROL_STOP)   // quit / kill (distributor.go:143-146,157-164)
                return GOL_STOPPED;
        }
        int64_t room = turns - t;
        if (is_strip(c)) room = std::min<int64_t>(room, c->halo_valid);
        const Launch plan = fixed && fi < fixed->size() ? (*fixed)[fi++] : plan_launch(c, room);
        const int k = plan.k;
        // rows computed: torus -> all; strip -> [s, buf_rows - s) after turn s since exchange
        const int s0 = is_strip(c) ? c->cfg.halo - c->halo_valid : 0;
        if (is_strip(c)) {
            a.row_lo = s0 + k;
            a.row_hi = c->buf_rows - s0 - k;
        } else {
            a.row_lo = 0;
            a.row_hi = c->buf_rows;
        }
        if (int rc = ensure_layout(c, stepping_il(c, k))) return rc;
        a.in = c->board[c->cur];
        a.out = c->board[c->cur ^ 1];
        // split this launch around the incoming halos (first launch of an overlapped step;
        // with per-turn counts the launch waits for the receives whole instead)
        const bool split = xstream && t == 0 && is_strip(c) && !cnt;
        if (xstream && t == 0 && !split) {
            HIP_OR_FAIL(c, hipEventRecord(c->ev_side, xstream));
            HIP_OR_FAIL(c, hipStreamWaitEvent(c->stream, c->ev_side, 0));
        }
        const int H = c->cfg.halo;
        const int in_lo = H + k, in_hi = H + c->cfg.rows - k;   // interior output rows
        if (split) {
            // side stream: after the caller's receives (and the engine's queued work)
            HIP_OR_FAIL(c, hipEventRecord(c->ev_main, c->stream));
            HIP_OR_FAIL(c, hipStreamWaitEvent(c->side, c->ev_main, 0));
            HIP_OR_FAIL(c, hipEventRecord(c->ev_side, xstream));
            HIP_OR_FAIL(c, hipStreamWaitEvent(c->side, c->ev_side, 0));
        }
        if (k > 1) {
            a.blocked = nullptr;
            a.counts = nullptr;
            a.band = plan.band;
            a.multi_variant = plan.var;
            if (plan.var == golk::kMultiTile || plan.var == golk::kMultiTilePersist ||
                plan.var == golk::kMultiTileStream) {
                a.tile_w = plan.tw;
                a.tile_seg = plan.seg;
            }
#if GOL_TOOLS
            if (c->multi_variant == golk::kMultiWgDiag && !split) {
                if (int rc = wg_diag_launch(c, a, k)) return rc;
            } else
#endif
            if (plan.var == golk::kMultiTilePersist) {
                HIP_OR_FAIL(c, persist_launch(c, a, k, plan.blk));
            } else if (plan.var == golk::kMultiTileStream) {
                HIP_OR_FAIL(c, stream_launch(c, a, k, plan.blk));
            } else if (split && in_lo < in_hi) {
                golk::StepArgs b = a;
                // concurrent launches cannot share the published-row scratch
                if (b.multi_variant == golk::kMultiWgPg) b.multi_variant = golk::kMultiWgHx;
                if (b.multi_variant == golk::kMultiWgPgS) b.multi_variant = golk::kMultiWgHxS;
                b.row_lo = in_lo;
                b.row_hi = in_hi;
                HIP_OR_FAIL(c, golk::launch_step_multi(b, k, c->stream));
                // boundary rows: short bands so the few rows still spread over many waves
                b.band = std::min(c->band_multi, golk::kOverlapBand);
                b.row_lo = a.row_lo;
                b.row_hi = in_lo;
                HIP_OR_FAIL(c, golk::launch_step_multi(b, k, c->side));
                b.row_lo = in_hi;
                b.row_hi = a.row_hi;
                HIP_OR_FAIL(c, golk::launch_step_multi(b, k, c->side));
            } else {
                HIP_OR_FAIL(c, pg_prepare(c, a, k));
                HIP_OR_FAIL(c, golk::launch_step_multi(a, k, split ? c->side : c->stream));
            }
            a.band = c->band;
            a.multi_variant = c->multi_variant;
            a.tile_w = c->tile_w;
            a.tile_seg = c->tile_seg;
        } else if (split) {
            // one-turn launches: interior now, the 2 x (halo) boundary rows after the receives
            a.blocked = c->blocked_pending ? c->blocked : nullptr;
            a.counts = nullptr;
            golk::StepArgs b = a;
            if (in_lo < in_hi) {
                b.row_lo = in_lo;
                b.row_hi = in_hi;
                HIP_OR_FAIL(c, golk::launch_step(b, c->fast, c->stream));
                b.row_lo = a.row_lo;
                b.row_hi = in_lo;
                HIP_OR_FAIL(c, golk::launch_step(b, c->fast, c->side));
                b.row_lo = in_hi;
                b.row_hi = a.row_hi;
                HIP_OR_FAIL(c, golk::launch_step(b, c->fast, c->side));
            } else {
                HIP_OR_FAIL(c, golk::launch_step(a, c->fast, c->side));
            }
        } else {
            a.blocked = c->blocked_pending ? c->blocked : nullptr;
            a.counts = nullptr;
            if (cnt) {
                const long long next_turn = c->turn + 1;
                const size_t slot = (size_t)(next_turn % kRing);
                if (slot == 0 || t == 0) {
                    // zero the slots of the next min(turns - t, kRing - slot) turns
                    const size_t nslots =
                        (size_t)std::min<int64_t>(turns - t, (int64_t)(kRing - slot));
                    HIP_OR_FAIL(c, hipMemsetAsync(c->counts + slot * kShards, 0,
                                                  nslots * kShards * 8, c->stream));
                }
                a.counts = c->counts + slot * kShards;
            }
            HIP_OR_FAIL(c, golk::launch_step(a, c->fast, c->stream));
        }
        if (split) {   // join: the next launch overwrites rows the side launches read
            HIP_OR_FAIL(c, hipEventRecord(c->ev_side, c->side));
            HIP_OR_FAIL(c, hipStreamWaitEvent(c->stream, c->ev_side, 0));
        }
        c->cur ^= 1;
        c->turn += k;
        c->progress.store(c->turn);
        c->launches += 1;
        if (c->last.size() < kLastCap)
            c->last.push_back(k > 1 ? plan : Launch{1, 0, c->band, 0, 0});
        ++c->last_n;
        t += k;
        if (is_strip(c)) c->halo_valid -= k;
        if (c->blocked_pending) {
            // every cell is 0/255 after the first turn; the mask is dead from here on
            c->blocked_pending = false;
            c->raw_turn0.clear();
        }
        if (ctl || c->readers.load(std::memory_order_relaxed)) {
            // bound the queue: wait for the launch kCtlDepth back
            hipEvent_t &e = ring.ev[ring.n % kCtlDepth];
            if (ring.n >= kCtlDepth) {
                HIP_OR_FAIL(c, hipEventSynchronize(e));
                if (int rc = check_dev_err(c)) return rc;
            } else {
                HIP_OR_FAIL(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
            }
            HIP_OR_FAIL(c, hipEventRecord(e, c->stream));
            ++ring.n;
        }
    }
    if (c->blocked && !c->blocked_pending) {
        HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
        release_blocked(c);
    }
    return GOL_OK;
}

}  // namespace

int gol_step(gol_ctx *c, int64_t turns)
{
    if (!c || turns < 0) return GOL_EINVAL;
    std::unique_lock<std::recursive_mutex> lk(c->mu);
    return step_impl(c, turns, nullptr, lk);
}

int gol_last_launches(gol_ctx *c, int32_t *turns, int32_t *kernel, int32_t *band, int32_t cap)
{
    if (!c || cap < 0 || (cap > 0 && (!turns || !kernel || !band))) return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    const int n = (int)std::min<size_t>((size_t)cap, c->last.size());
    for (int i = 0; i < n; ++i) {
        turns[i] = c->last[i].k;
        kernel[i] = c->last[i].var;
        band[i] = c->last[i].band;
    }
    return (int)std::min<long long>(c->last_n, 0x7fffffff);
}

int gol_last_launch_tiles(gol_ctx *c, int32_t *tile_w, int32_t *tile_seg, int32_t *waves,
                          int32_t *block_turns, int32_t cap)
{
    if (!c || cap < 0 || (cap > 0 && (!tile_w || !tile_seg || !waves || !block_turns)))
        return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    const int n = (int)std::min<size_t>((size_t)cap, c->last.size());
    for (int i = 0; i < n; ++i) {
        const Launch &L = c->last[i];
        const bool p = L.var == golk::kMultiTilePersist || L.var == golk::kMultiTileStream;
        const bool t = L.k > 1 && (L.var == golk::kMultiTile || p);
        const int depth = p ? L.blk : L.k;               // (K1p / K1q: the waves fit one block)
        tile_w[i] = t ? L.tw : 0;
        tile_seg[i] = t ? L.seg : 0;
        waves[i] = t ? golk::tile_waves(depth, L.band, L.tw, L.seg) : 0;
        block_turns[i] = t ? depth : 0;
    }
    return (int)std::min<long long>(c->last_n, 0x7fffffff);
}

int gol_tile_codes(int32_t *codes, int32_t cap)
{
    const int n = (int)std::size(golk::kTileCodes);
    if (cap < 0 || (cap > 0 && !codes)) return GOL_EINVAL;
    for (int i = 0; i < std::min(n, (int)cap); ++i) codes[i] = golk::kTileCodes[i];
    return n;
}

int gol_tile_persist_codes(int32_t *codes, int32_t cap)
{
    const int n = GOL_TOOLS ? (int)std::size(golk::kTilePersistCodes) : 0;   // (tools build)
    if (cap < 0 || (cap > 0 && !codes)) return GOL_EINVAL;
    for (int i = 0; i < std::min(n, (int)cap); ++i) codes[i] = golk::kTilePersistCodes[i];
    return n;
}

int gol_tile_stream_codes(int32_t *codes, int32_t cap)
{
    const int n = GOL_TOOLS ? (int)std::size(golk::kTileStreamCodes) : 0;   // (tools build)
    if (cap < 0 || (cap > 0 && !codes)) return GOL_EINVAL;
    for (int i = 0; i < std::min(n, (int)cap); ++i) codes[i] = golk::kTileStreamCodes[i];
    return n;
}

int gol_step_overlap(gol_ctx *c, int64_t turns, void *recv_stream)
{
    if (!c || turns < 0 || !recv_stream) return GOL_EINVAL;
    std::unique_lock<std::recursive_mutex> lk(c->mu);
    if (!is_strip(c)) return fail(c, GOL_ESTATE, "not a strip engine");
    c->halo_valid = c->cfg.halo;   // the receives queued on recv_stream refresh the halos
    return step_impl(c, turns, (hipStream_t)recv_stream, lk);
}

int gol_stream_wait(gol_ctx *c, void *stream)
{
    if (!c || !stream) return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    DeviceGuard g(c->device);
    HIP_OR_FAIL(c, hipEventRecord(c->ev_main, c->stream));
    HIP_OR_FAIL(c, hipStreamWaitEvent((hipStream_t)stream, c->ev_main, 0));
    return GOL_OK;
}

int gol_set_control(gol_ctx *c, int32_t word)
{
    if (!c || word < GOL_CONTROL_RUN || word > GOL_CONTROL_STOP) return GOL_EINVAL;
    c->control_used.store(true);
    c->control.store(word);
    return GOL_OK;
}

int gol_get_progress(gol_ctx *c, int64_t *turn, int32_t *parked)
{
    if (!c) return GOL_EINVAL;
    if (turn) *turn = c->progress.load();
    if (parked) *parked = c->parked.load() ? 1 : 0;
    return GOL_OK;
}

int gol_snapshot(gol_ctx *c, int64_t *turn, int64_t *alive)
{
    if (!c || !turn || !alive) return GOL_EINVAL;
    return run_read(c, [&]() -> int {
        DeviceGuard g(c->device);
        long long n = 0;
        int rc = count_now(c, &n);
        if (rc) return rc;
        *turn = c->turn;
        *alive = n;
        return GOL_OK;
    });
}

int gol_turn_counts(gol_ctx *c, int64_t first_turn, int64_t n, int64_t *out)
{
    if (!c || !out || n < 0) return GOL_EINVAL;
    return run_read(c, [&]() -> int {
        if (!(c->cfg.flags & GOL_FLAG_COUNT_EVERY_TURN))
            return fail(c, GOL_ESTATE, "engine created without GOL_FLAG_COUNT_EVERY_TURN");
        if (n == 0) return GOL_OK;
        if (first_turn < 1 || first_turn + n - 1 > c->turn || first_turn <= c->turn - kRing)
            return fail(c, GOL_EINVAL, "turns %lld..%lld not in the recorded window",
                        (long long)first_turn, (long long)(first_turn + n - 1));
        DeviceGuard g(c->device);
        std::vector<unsigned long long> h((size_t)kRing * kShards);
        HIP_OR_FAIL(c, hipMemcpyAsync(h.data(), c->counts, h.size() * 8, hipMemcpyDeviceToHost,
                                      c->stream));
        if (int rc = sync_checked(c)) return rc;
        for (int64_t i = 0; i < n; ++i) {
            const size_t slot = (size_t)((first_turn + i) % kRing);
            unsigned long long s = 0;
            for (int k = 0; k < kShards; k++) s += h[slot * kShards + k];
            out[i] = (int64_t)s;
        }
        return GOL_OK;
    });
}

namespace {
// owned rows as 0/255 bytes (the caller holds the engine: run_read)
int read_board_bytes(gol_ctx *c, uint8_t *out)
{
    {
        const size_t row_bytes = (size_t)c->cfg.width;
        if (!c->raw_turn0.empty()) {
            std::memcpy(out, c->raw_turn0.data(), c->raw_turn0.size());
            return GOL_OK;
        }
        DeviceGuard g(c->device);
        if (int rc_ = ensure_layout(c, false)) return rc_;
        const int chunk_rows = (int)std::max<size_t>(
            1, std::min<size_t>(kStagingBytes / row_bytes, (size_t)c->cfg.rows));
        int rc = ensure_staging(c, (size_t)chunk_rows * row_bytes);
        if (rc) return rc;
        for (int r0 = 0; r0 < c->cfg.rows; r0 += chunk_rows) {
            const int nr = std::min(chunk_rows, c->cfg.rows - r0);
            HIP_OR_FAIL(c, golk::launch_unpack(c->board[c->cur], c->cfg.width, c->nw, c->pitch,
                                               own_lo(c) + r0, nr, c->staging, c->stream));
            HIP_OR_FAIL(c, hipMemcpyAsync(out + (size_t)r0 * row_bytes, c->staging,
                                          (size_t)nr * row_bytes, hipMemcpyDeviceToHost, c->stream));
            if (int rc2 = sync_checked(c)) return rc2;
        }
        return GOL_OK;
    }
}
}  // namespace

int gol_read_board(gol_ctx *c, uint8_t *out)
{
    if (!c || !out) return GOL_EINVAL;
    return run_read(c, [&]() -> int { return read_board_bytes(c, out); });
}

int gol_get_world(gol_ctx *c, uint8_t *out, int64_t *turn)
{
    if (!c || !out || !turn) return GOL_EINVAL;
    return run_read(c, [&]() -> int {
        const int rc = read_board_bytes(c, out);
        if (rc == GOL_OK) *turn = c->turn;
        return rc;
    });
}

int gol_read_packed(gol_ctx *c, uint64_t *out)
{
    if (!c || !out) return GOL_EINVAL;
    return run_read(c, [&]() -> int {
        DeviceGuard g(c->device);
        if (int rc_ = ensure_layout(c, false)) return rc_;
        HIP_OR_FAIL(c, hipMemcpy2DAsync(out, (size_t)c->nw * 8,
                                        c->board[c->cur] + (size_t)own_lo(c) * c->pitch,
                                        (size_t)c->pitch * 8, (size_t)c->nw * 8, c->cfg.rows,
                                        hipMemcpyDeviceToHost, c->stream));
        return sync_checked(c);
    });
}

int gol_alive_cells(gol_ctx *c, int64_t *xy, int64_t cap, int64_t *n)
{
    if (!c || !n || cap < 0 || (cap > 0 && !xy)) return GOL_EINVAL;
    return run_read(c, [&]() -> int {
        DeviceGuard g(c->device);
        if (int rc_ = ensure_layout(c, false)) return rc_;
        const int rows = c->cfg.rows;
        std::vector<long long> rc((size_t)rows), off((size_t)rows);
        long long *d_rc = nullptr;
        HIP_OR_FAIL(c, hipMalloc((void **)&d_rc, (size_t)rows * 8 * 2));
        long long *d_off = d_rc + rows;
        int err = GOL_OK;
        auto done = [&](int code) {
            (void)hipStreamSynchronize(c->stream);
            (void)hipFree(d_rc);
            return code;
        };
        hipError_t e = golk::launch_row_popcount(c->board[c->cur], c->nw, c->pitch, own_lo(c), rows,
                                                 d_rc, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(rc.data(), d_rc, (size_t)rows * 8, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return done(fail(c, GOL_EHIP, "alive count: %s", hipGetErrorString(e)));
        if (int rc2 = check_dev_err(c)) return done(rc2);
        long long total = 0;
        for (int r = 0; r < rows; r++) {
            off[(size_t)r] = total;
            total += rc[(size_t)r];
        }
        *n = total;
        if (cap == 0 || total == 0) return done(GOL_OK);
        // scatter in row chunks so the device list stays within the staging budget
        const long long per_cell = 16;
        long long r0 = 0;
        while (r0 < rows && off[(size_t)r0] < cap) {
            // rows [r0, r1) whose cells fit in kStagingBytes
            long long r1 = r0;
            while (r1 < rows && (off[(size_t)r1] + rc[(size_t)r1] - off[(size_t)r0]) * per_cell <=
                                    (long long)kStagingBytes)
                ++r1;
            if (r1 == r0) r1 = r0 + 1;  // a single row larger than the budget
            const long long cells = off[(size_t)r1 - 1] + rc[(size_t)r1 - 1] - off[(size_t)r0];
            err = ensure_staging(c, (size_t)std::max<long long>(cells * per_cell, 16));
            if (err) return done(err);
            // offsets relative to this chunk: subtract off[r0] via a shifted copy
            std::vector<long long> rel((size_t)(r1 - r0));
            for (long long r = r0; r < r1; r++) rel[(size_t)(r - r0)] = off[(size_t)r] - off[(size_t)r0];
            e = hipMemcpyAsync(d_off + r0, rel.data(), rel.size() * 8, hipMemcpyHostToDevice,
                               c->stream);
            if (e == hipSuccess)
                e = golk::launch_alive_scatter(c->board[c->cur], c->nw, c->pitch,
                                               own_lo(c) + (int)r0, (int)(r1 - r0),
                                               (long long)c->cfg.row_offset + r0, d_off + r0,
                                               (long long *)c->staging, c->stream);
            const long long want = std::min<long long>(cells, cap - off[(size_t)r0]);
            if (e == hipSuccess)
                e = hipMemcpyAsync(xy + 2 * off[(size_t)r0], c->staging, (size_t)want * per_cell,
                                   hipMemcpyDeviceToHost, c->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
            if (e != hipSuccess)
                return done(fail(c, GOL_EHIP, "alive scatter: %s", hipGetErrorString(e)));
            r0 = r1;
        }
        return done(GOL_OK);
    });
}

// ------------------------------------------------------------ halo exchange
int gol_export_halo(gol_ctx *c, void *top, void *bottom, void *s)
{
    if (!c || !top || !bottom) return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (!is_strip(c)) return fail(c, GOL_ESTATE, "not a strip engine");
    DeviceGuard g(c->device);
    hipStream_t st = s ? (hipStream_t)s : c->stream;
    if (st != c->stream) {
        // make the caller's stream wait for the engine's queued turns
        hipEvent_t ev;
        HIP_OR_FAIL(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_OR_FAIL(c, hipEventRecord(ev, c->stream));
        HIP_OR_FAIL(c, hipStreamWaitEvent(st, ev, 0));
        (void)hipEventDestroy(ev);
    }
    const int K = c->cfg.halo;
    const size_t rowb = (size_t)c->nw * 8;
    const uint64_t *b = c->board[c->cur];
    if (c->il) {   // halo rows cross the API in the standard layout
        HIP_OR_FAIL(c, golk::launch_il_convert(b + (size_t)own_lo(c) * c->pitch, c->pitch,
                                               (uint64_t *)top, c->nw, K, c->nw, false, st));
        HIP_OR_FAIL(c, golk::launch_il_convert(b + (size_t)(own_hi(c) - K) * c->pitch, c->pitch,
                                               (uint64_t *)bottom, c->nw, K, c->nw, false, st));
        return GOL_OK;
    }
    HIP_OR_FAIL(c, hipMemcpy2DAsync(top, rowb, b + (size_t)own_lo(c) * c->pitch,
                                    (size_t)c->pitch * 8, rowb, K, hipMemcpyDeviceToDevice, st));
    HIP_OR_FAIL(c, hipMemcpy2DAsync(bottom, rowb, b + (size_t)(own_hi(c) - K) * c->pitch,
                                    (size_t)c->pitch * 8, rowb, K, hipMemcpyDeviceToDevice, st));
    return GOL_OK;
}

int gol_import_halo(gol_ctx *c, const void *top, const void *bottom, void *s)
{
    if (!c || !top || !bottom) return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (!is_strip(c)) return fail(c, GOL_ESTATE, "not a strip engine");
    DeviceGuard g(c->device);
    hipStream_t st = s ? (hipStream_t)s : c->stream;
    const int K = c->cfg.halo;
    const size_t rowb = (size_t)c->nw * 8;
    uint64_t *b = c->board[c->cur];
    if (c->il) {
        HIP_OR_FAIL(c, golk::launch_il_convert((const uint64_t *)top, c->nw, b, c->pitch, K, c->nw,
                                               true, st));
        HIP_OR_FAIL(c, golk::launch_il_convert((const uint64_t *)bottom, c->nw,
                                               b + (size_t)own_hi(c) * c->pitch, c->pitch, K,
                                               c->nw, true, st));
    } else {
        HIP_OR_FAIL(c, hipMemcpy2DAsync(b, (size_t)c->pitch * 8, top, rowb, rowb, K,
                                        hipMemcpyDeviceToDevice, st));
        HIP_OR_FAIL(c, hipMemcpy2DAsync(b + (size_t)own_hi(c) * c->pitch, (size_t)c->pitch * 8,
                                        bottom, rowb, rowb, K, hipMemcpyDeviceToDevice, st));
    }
    if (st != c->stream) {
        hipEvent_t ev;
        HIP_OR_FAIL(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_OR_FAIL(c, hipEventRecord(ev, st));
        HIP_OR_FAIL(c, hipStreamWaitEvent(c->stream, ev, 0));
        (void)hipEventDestroy(ev);
    }
    c->halo_valid = K;
    return GOL_OK;
}

static int copy_rows_between(gol_ctx *dst, int dst_row, gol_ctx *src, int src_row, int K)
{
    if (dst->nw != src->nw) return fail(dst, GOL_EINVAL, "width mismatch");
    if (src->il != dst->il) {   // raw row copies need one layout on both sides
        DeviceGuard gs(src->device);
        if (int rc = ensure_layout(src, dst->il)) return rc;
    }
    // dst stream waits for src's queued work (src's event, on src's device); copy on dst's
    // stream; then src's stream waits for the copy (dst's event)
    {
        DeviceGuard g(src->device);
        HIP_OR_FAIL(dst, hipEventRecord(src->ev_copy, src->stream));
    }
    DeviceGuard g(dst->device);
    HIP_OR_FAIL(dst, hipStreamWaitEvent(dst->stream, src->ev_copy, 0));
    const size_t rowb = (size_t)dst->nw * 8;
    uint64_t *d = dst->board[dst->cur] + (size_t)dst_row * dst->pitch;
    const uint64_t *s = src->board[src->cur] + (size_t)src_row * src->pitch;
    if (dst->device == src->device) {
        HIP_OR_FAIL(dst, hipMemcpy2DAsync(d, (size_t)dst->pitch * 8, s, (size_t)src->pitch * 8,
                                          rowb, K, hipMemcpyDeviceToDevice, dst->stream));
    } else {
        // rows are contiguous when pitch == nw (always true for engines created here)
        HIP_OR_FAIL(dst, hipMemcpyPeerAsync(d, dst->device, s, src->device, rowb * K,
                                            dst->stream));
    }
    // src must not overwrite these rows before the copy lands
    HIP_OR_FAIL(dst, hipEventRecord(dst->ev_copy, dst->stream));
    {
        DeviceGuard g2(src->device);
        HIP_OR_FAIL(dst, hipStreamWaitEvent(src->stream, dst->ev_copy, 0));
    }
    return GOL_OK;
}

int gol_copy_halo_from_upper(gol_ctx *dst, gol_ctx *src)
{
    if (!dst || !src || !is_strip(dst) || !is_strip(src) || dst->cfg.halo != src->cfg.halo)
        return GOL_EINVAL;
    // both engines at once, deadlock-free in any order (a ring pair exchanging both ways from
    // two host threads); dst == src (one strip exchanging with itself) is one recursive lock
    std::scoped_lock lk(dst->mu, src->mu);
    const int K = dst->cfg.halo;
    return copy_rows_between(dst, 0, src, own_hi(src) - K, K);
}

int gol_copy_halo_from_lower(gol_ctx *dst, gol_ctx *src)
{
    if (!dst || !src || !is_strip(dst) || !is_strip(src) || dst->cfg.halo != src->cfg.halo)
        return GOL_EINVAL;
    std::scoped_lock lk(dst->mu, src->mu);
    const int K = dst->cfg.halo;
    return copy_rows_between(dst, own_hi(dst), src, own_lo(src), K);
}

int gol_halo_done(gol_ctx *c)
{
    if (!c || !is_strip(c)) return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    c->halo_valid = c->cfg.halo;
    return GOL_OK;
}

int gol_halo_buffers(gol_ctx *c, void **send_top, void **send_bottom, void **recv_top,
                     void **recv_bottom, int32_t *layout)
{
    if (!c || !send_top || !send_bottom || !recv_top || !recv_bottom || !layout)
        return GOL_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (!is_strip(c)) return fail(c, GOL_ESTATE, "not a strip engine");
    DeviceGuard g(c->device);
    // the layout the first launch after a full exchange runs on: gol_step's own rule
    // (launch_depth) with halo turns to go -- whatever the step after the exchange asks
    // for, its first launch has depth launch_depth(min(turns, halo)); the layout is the
    // same for every depth >= 2, and a function of width, halo and flags only, so equal
    // on every rank
    const bool il = stepping_il(c, launch_depth(c, c->cfg.halo));
    if (int rc = ensure_layout(c, il)) return rc;
    uint64_t *b = c->board[c->cur];
    const int K = c->cfg.halo;
    *send_top = b + (size_t)own_lo(c) * c->pitch;
    *send_bottom = b + (size_t)(own_hi(c) - K) * c->pitch;
    *recv_top = b;
    *recv_bottom = b + (size_t)own_hi(c) * c->pitch;
    *layout = c->il ? 1 : 0;
    return GOL_OK;
}

}  // extern "C"

// ------------------------------------------------- internal (driver) access
namespace golint {
long long engine_turn(gol_ctx *c) { return c->turn; }
int engine_device(gol_ctx *c) { return c->device; }
}  // namespace golint
