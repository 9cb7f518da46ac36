// gol_run.cpp — C++ host driver mirroring the reference's controller:
//
//   gol.Run(p, events, keyPresses)          Local/gol/gol.go:12-40
//   distributor(p, c, keyPresses)           Local/gol/distributor.go:55-227
//   readPgmImage / writePgmImage            Local/gol/io.go:42-121
//   Server turn loop + control handshake    Server/gol/distributor.go:104-171
//
// Differences from the reference, all deliberate and documented in DESIGN.md:
//   * the board lives on the GPU(s) for the whole run; there is no per-turn RPC;
//   * CompletedTurns counts the turns of THIS run (the reference's Server keeps a
//     process-global `turn` that is never reset: Server/gol/distributor.go:30,133);
//   * TurnComplete{t} is emitted for every turn when enabled (event.go:55-60
//     contract; the reference emits none: Local/gol/distributor.go:184-185);
//   * control keys are sampled at kernel-launch boundaries (a launch fuses up to
//     turns_per_launch turns; multi-strip runs: chunk boundaries, ~2 chunks of ~1-4 ms
//     each in flight) instead of after every single turn;
//   * boards need not be square (the reference reads H x H bytes:
//     Local/gol/distributor.go:80).
#include <hip/hip_runtime.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gol_amd.h"
#include "gol_internal.h"

namespace {

using Clock = std::chrono::steady_clock;

// The reference Server keeps `world` and `turn` in process globals across controller
// runs (Server/gol/distributor.go:29-30) so that CONT=yes can resume
// (Local/gol/distributor.go:171-178).  Here: the last run's final packed board.
struct RetainedState {
    std::mutex mu;
    bool valid = false;
    int W = 0, H = 0;
    long long turn = 0;
    std::vector<uint64_t> words;     // H x ceil(W/64)
};
RetainedState &retained()
{
    static RetainedState r;
    return r;
}

struct Item {
    gol_event ev;
    std::shared_ptr<std::vector<int64_t>> cells;   // FinalTurnComplete.Alive
};

// Host image bytes in page-locked memory (hipHostMalloc), so PGM payloads move to and
// from the device by DMA (hipMemcpyAsync without a pageable bounce); plain malloc if the
// pinning fails.  The reference's io goroutine moves the image byte by byte over a
// channel (Local/gol/io.go:88-121, 42-85).
struct HostBuf {
    uint8_t *p = nullptr;
    size_t n = 0;
    bool pinned = false;
    HostBuf() = default;
    HostBuf(const HostBuf &) = delete;
    HostBuf &operator=(const HostBuf &) = delete;
    HostBuf(HostBuf &&o) noexcept : p(o.p), n(o.n), pinned(o.pinned) { o.p = nullptr; o.n = 0; }
    HostBuf &operator=(HostBuf &&o) noexcept
    {
        if (this != &o) {
            release();
            p = o.p;
            n = o.n;
            pinned = o.pinned;
            o.p = nullptr;
            o.n = 0;
        }
        return *this;
    }
    ~HostBuf() { release(); }
    bool alloc(size_t bytes)
    {
        if (p && n == bytes) return true;
        release();
        if (bytes == 0) return true;
        if (hipHostMalloc((void **)&p, bytes, hipHostMallocDefault) == hipSuccess) {
            pinned = true;
        } else {
            (void)hipGetLastError();
            p = (uint8_t *)std::malloc(bytes);
            pinned = false;
            if (!p) return false;
        }
        n = bytes;
        return true;
    }
    void release()
    {
        if (p) {
            if (pinned) (void)hipHostFree(p);
            else std::free(p);
        }
        p = nullptr;
        n = 0;
    }
    uint8_t *data() { return p; }
    const uint8_t *data() const { return p; }
    size_t size() const { return n; }
};

bool is_space(unsigned char ch) { return ch == ' ' || (ch >= '\t' && ch <= '\r'); }

// strings.Fields-like split of the first 5 fields (Local/gol/io.go:93-114):
// fields[4] is the payload, which ends at the next whitespace byte.  On success
// `payload` is the payload's offset in `data` (W*H bytes).
int parse_pgm(const uint8_t *data, size_t size, int W, int H, size_t &payload, std::string &err)
{
    size_t pos = 0;
    std::string f[4];
    for (int k = 0; k < 4; k++) {
        while (pos < size && is_space(data[pos])) pos++;
        size_t s = pos;
        while (pos < size && !is_space(data[pos])) pos++;
        f[k].assign((const char *)data + s, pos - s);
    }
    if (f[0] != "P5") { err = "Not a pgm file"; return GOL_EIO; }
    if (atoi(f[1].c_str()) != W) { err = "Incorrect width"; return GOL_EIO; }
    if (atoi(f[2].c_str()) != H) { err = "Incorrect height"; return GOL_EIO; }
    if (atoi(f[3].c_str()) != 255) { err = "Incorrect maxval/bit depth"; return GOL_EIO; }
    while (pos < size && is_space(data[pos])) pos++;
    size_t s = pos;
    while (pos < size && !is_space(data[pos])) pos++;
    const size_t need = (size_t)W * H;
    if (pos - s < need) {
        err = "PGM payload shorter than width*height (the reference would block on inputQ)";
        return GOL_EIO;
    }
    payload = s;
    return GOL_OK;
}

int write_pgm(const std::string &dir, const std::string &name, int W, int H,
              const HostBuf &pix, std::string &err)
{
    ::mkdir(dir.c_str(), 0777);                   // os.Mkdir("out", ...) (io.go:46)
    const std::string path = dir + "/" + name + ".pgm";
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) { err = "cannot create " + path; return GOL_EIO; }
    fprintf(f, "P5\n%d %d\n255\n", W, H);        // io.go:50-57
    const size_t n = fwrite(pix.data(), 1, pix.size(), f);
    const bool ok = n == pix.size() && fflush(f) == 0;
    fclose(f);
    if (!ok) { err = "short write " + path; return GOL_EIO; }
    return GOL_OK;
}

}  // namespace

struct gol_run {
    gol_params p{};
    std::string image_dir = "images", out_dir = "out";
    int ngpus = 1;
    std::vector<int> devices;
    int halo = 0;
    int resume = -1;
    int ticker_ms = 2000;
    size_t capacity = 1;
    bool emit_turn_complete = false;
    bool emit_cell_flipped = false;
    uint32_t engine_flags = 0;

    std::thread th;
    std::mutex mu;
    std::condition_variable cv_push, cv_pop;
    std::deque<Item> q;
    bool closed = false;
    std::atomic<bool> abort{false};

    std::mutex kmu;
    std::condition_variable kcv;
    std::deque<int> keys;

    std::shared_ptr<std::vector<int64_t>> last_final;
    std::string error;

    // single-engine runs: a key press interrupts the running chunk through the engine's
    // control word (gol_set_control), so keys take effect within 2 kernel launches
    std::mutex ctl_mu;
    gol_ctx *ctl_engine = nullptr;
    void interrupt()
    {
        std::lock_guard<std::mutex> lk(ctl_mu);
        if (ctl_engine) (void)gol_set_control(ctl_engine, GOL_CONTROL_STOP);
    }
    void set_ctl_engine(gol_ctx *e)
    {
        std::lock_guard<std::mutex> lk(ctl_mu);
        ctl_engine = e;
        if (e) (void)gol_set_control(e, GOL_CONTROL_RUN);
    }

    // ----------------------------------------------------------- channel
    bool send(const gol_event &ev, std::shared_ptr<std::vector<int64_t>> cells = nullptr)
    {
        std::unique_lock<std::mutex> lk(mu);
        cv_push.wait(lk, [&] { return q.size() < capacity || abort.load(); });
        if (abort.load()) return false;
        q.push_back(Item{ev, std::move(cells)});
        cv_pop.notify_one();
        return true;
    }
    void close()
    {
        std::lock_guard<std::mutex> lk(mu);
        closed = true;
        cv_pop.notify_all();
    }
    bool pop_key(int &k)
    {
        std::lock_guard<std::mutex> lk(kmu);
        if (keys.empty()) return false;
        k = keys.front();
        keys.pop_front();
        return true;
    }

    void run();
};

namespace {

gol_event make_ev(int type, long long turns)
{
    gol_event e;
    std::memset(&e, 0, sizeof e);
    e.type = type;
    e.completed_turns = turns;
    return e;
}

// Row strips over `n` engines with the reference Server's split (:106-116).
struct Strips {
    std::vector<gol_ctx *> eng;
    std::vector<int> off, rows;
    int W = 0, H = 0, K = 0;
    std::string err;

    ~Strips()
    {
        for (auto *e : eng) gol_destroy(e);
    }
    bool strip_mode() const { return eng.size() > 1; }

    int fail_from(gol_ctx *e, int rc)
    {
        err = std::string(gol_strerror(rc)) + ": " + (e ? gol_last_error(e) : "");
        return rc;
    }

    int create(int width, int height, int n, const std::vector<int> &devs, int halo,
               uint32_t flags)
    {
        W = width;
        H = height;
        if (n < 1) n = 1;
        if (n > H) n = H;
        const int base = H / n, slack = H % n;
        int o = 0;
        for (int i = 0; i < n; i++) {
            const int r = base + (i < slack ? 1 : 0);
            off.push_back(o);
            rows.push_back(r);
            o += r;
        }
        const int min_rows = *std::min_element(rows.begin(), rows.end());
        K = n > 1 ? std::max(1, std::min(halo > 0 ? halo : 16, min_rows)) : 0;
        for (int i = 0; i < n; i++) {
            gol_config cfg{};
            cfg.width = W;
            cfg.height = H;
            cfg.device = devs[(size_t)i];
            cfg.row_offset = n > 1 ? off[(size_t)i] : 0;
            cfg.rows = n > 1 ? rows[(size_t)i] : H;
            cfg.halo = K;
            cfg.flags = flags;
            gol_ctx *e = nullptr;
            int rc = gol_create_ex(&cfg, &e);
            if (rc) {
                err = std::string("gol_create_ex: ") + gol_strerror(rc);
                return rc;
            }
            eng.push_back(e);
        }
        return GOL_OK;
    }

    int load(const uint8_t *pix)
    {
        if (!strip_mode()) {
            int rc = gol_load(eng[0], pix);
            return rc ? fail_from(eng[0], rc) : GOL_OK;
        }
        HostBuf buf;
        for (size_t i = 0; i < eng.size(); i++) {
            const int br = rows[i] + 2 * K;
            if (!buf.alloc((size_t)br * W)) {
                err = "out of host memory";
                return GOL_ENOMEM;
            }
            for (int b = 0; b < br; b++) {
                int g = (off[i] - K + b) % H;
                if (g < 0) g += H;
                std::memcpy(buf.data() + (size_t)b * W, pix + (size_t)g * W, (size_t)W);
            }
            int rc = gol_load(eng[i], buf.data());
            if (rc) return fail_from(eng[i], rc);
        }
        return GOL_OK;
    }

    int nwords() const { return (W + 63) / 64; }

    // load a global packed board (H x nw words) into every strip (with halo rows)
    int load_packed(const std::vector<uint64_t> &g)
    {
        const size_t nw = (size_t)nwords();
        if (!strip_mode()) {
            int rc = gol_load_packed(eng[0], g.data());
            return rc ? fail_from(eng[0], rc) : GOL_OK;
        }
        for (size_t i = 0; i < eng.size(); i++) {
            const int br = rows[i] + 2 * K;
            std::vector<uint64_t> buf((size_t)br * nw);
            for (int b = 0; b < br; b++) {
                int gr = (off[i] - K + b) % H;
                if (gr < 0) gr += H;
                std::memcpy(buf.data() + (size_t)b * nw, g.data() + (size_t)gr * nw, nw * 8);
            }
            int rc = gol_load_packed(eng[i], buf.data());
            if (rc) return fail_from(eng[i], rc);
        }
        return GOL_OK;
    }

    int read_packed(std::vector<uint64_t> &g)
    {
        const size_t nw = (size_t)nwords();
        g.assign((size_t)H * nw, 0);
        for (size_t i = 0; i < eng.size(); i++) {
            const int o = strip_mode() ? off[i] : 0;
            int rc = gol_read_packed(eng[i], g.data() + (size_t)o * nw);
            if (rc) return fail_from(eng[i], rc);
        }
        return GOL_OK;
    }

    int halo_valid()
    {
        gol_info info;
        gol_get_info(eng[0], &info);
        return info.halo_valid;
    }

    int exchange()
    {
        const size_t n = eng.size();
        for (size_t i = 0; i < n; i++) {
            gol_ctx *up = eng[(i + n - 1) % n], *dn = eng[(i + 1) % n];
            int rc = gol_copy_halo_from_upper(eng[i], up);
            if (!rc) rc = gol_copy_halo_from_lower(eng[i], dn);
            if (rc) return fail_from(eng[i], rc);
        }
        for (auto *e : eng) gol_halo_done(e);
        return GOL_OK;
    }

    long long engine_turn() { return golint::engine_turn(eng[0]); }

    // advance `turns` turns (asynchronous on the engines' streams); a single engine stops
    // early when its control word says so (engine_turn() tells how far it got)
    int step(long long turns)
    {
        if (!strip_mode()) {
            int rc = gol_step(eng[0], turns);
            return rc < 0 ? fail_from(eng[0], rc) : GOL_OK;
        }
        while (turns > 0) {
            int hv = halo_valid();
            if (hv == 0) {
                int rc = exchange();
                if (rc) return rc;
                hv = K;
            }
            const long long n = std::min<long long>(turns, hv);
            for (auto *e : eng) {
                int rc = gol_step(e, n);
                if (rc < 0) return fail_from(e, rc);   // (strip engines have no control word)
            }
            turns -= n;
        }
        return GOL_OK;
    }

    int sync()
    {
        for (auto *e : eng) {
            int rc = gol_sync(e);
            if (rc) return fail_from(e, rc);
        }
        return GOL_OK;
    }

    int snapshot(long long &turn, long long &alive)
    {
        alive = 0;
        for (auto *e : eng) {
            int64_t t = 0, a = 0;
            int rc = gol_snapshot(e, &t, &a);
            if (rc) return fail_from(e, rc);
            turn = t;
            alive += a;
        }
        return GOL_OK;
    }

    int read_board(HostBuf &pix)
    {
        if (!pix.alloc((size_t)W * H)) {
            err = "out of host memory";
            return GOL_ENOMEM;
        }
        for (size_t i = 0; i < eng.size(); i++) {
            const int o = strip_mode() ? off[i] : 0;
            int rc = gol_read_board(eng[i], pix.data() + (size_t)o * W);
            if (rc) return fail_from(eng[i], rc);
        }
        return GOL_OK;
    }

    int alive_cells(std::vector<int64_t> &xy)
    {
        xy.clear();
        for (auto *e : eng) {
            int64_t n = 0;
            int rc = gol_alive_cells(e, nullptr, 0, &n);
            if (rc) return fail_from(e, rc);
            const size_t base = xy.size();
            xy.resize(base + (size_t)n * 2);
            if (n) {
                rc = gol_alive_cells(e, xy.data() + base, n, &n);
                if (rc) return fail_from(e, rc);
            }
        }
        return GOL_OK;
    }
};

}  // namespace

void gol_run::run()
{
    const int W = p.image_width, H = p.image_height;
    auto die = [&](const std::string &msg) {
        {
            std::lock_guard<std::mutex> lk(mu);
            error = msg;
        }
        close();
    };
    if (W < 2 || H < 1 || p.turns < 0) return die("invalid Params");

    // ioInput: read images/{W}x{H}.pgm (distributor.go:73-83, io.go:88-121)
    const std::string fname = std::to_string(W) + "x" + std::to_string(H);
    HostBuf file;                                     // the whole file, pinned
    size_t payload = 0;
    {
        const std::string path = image_dir + "/" + fname + ".pgm";
        FILE *f = fopen(path.c_str(), "rb");
        if (!f) return die("cannot open " + path);
        long sz = -1;
        if (fseek(f, 0, SEEK_END) == 0) sz = ftell(f);
        if (sz < 0 || fseek(f, 0, SEEK_SET) != 0 || !file.alloc((size_t)sz) ||
            fread(file.data(), 1, (size_t)sz, f) != (size_t)sz) {
            fclose(f);
            return die("cannot read " + path);
        }
        fclose(f);
        std::string err;
        if (parse_pgm(file.data(), file.size(), W, H, payload, err)) return die(err);
    }
    const uint8_t *pix = file.data() + payload;

    Strips st;
    if (st.create(W, H, ngpus, devices, halo, engine_flags)) return die(st.err);
    if (st.load(pix)) return die(st.err);

    long long turn = 0;
    bool cont = resume > 0;
    if (resume < 0) {
        const char *e = getenv("CONT");                // distributor.go:171
        cont = e && std::string(e) == "yes";
    }
    if (cont) {
        // GetWorld -> {SWorld, TurnCur}; run Turns - TurnCur more turns (distributor.go:172-177)
        RetainedState &rs = retained();
        std::lock_guard<std::mutex> lk(rs.mu);
        if (!rs.valid || rs.W != W || rs.H != H)
            return die("CONT=yes: no retained board of this size to resume from");
        if (st.load_packed(rs.words)) return die(st.err);
        turn = rs.turn;
    }
    const long long turn0 = turn;   // engines count from 0; events report turn0 + engine turn
    gol_event ev = make_ev(GOL_EV_STATE_CHANGE, turn);
    ev.new_state = GOL_EXECUTING;
    if (!send(ev)) return close();

    if (emit_cell_flipped) {
        // "send this event for all cells that are alive when the image is loaded" (event.go:49-51)
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++)
                if (pix[(size_t)y * W + x] == 255) {
                    gol_event cf = make_ev(GOL_EV_CELL_FLIPPED, 0);
                    cf.x = x;
                    cf.y = y;
                    if (!send(cf)) return close();
                }
    }

    auto next_tick = Clock::now() + std::chrono::milliseconds(ticker_ms);
    auto tick_now = [&]() -> bool {                   // the tick that is due, unconditionally
        next_tick += std::chrono::milliseconds(ticker_ms);
        long long t = 0, a = 0;
        if (st.snapshot(t, a)) { die(st.err); return false; }
        gol_event e = make_ev(GOL_EV_ALIVE_CELLS_COUNT, turn0 + t);
        e.cells_count = a;
        return send(e);
    };
    auto tick = [&]() -> bool { return Clock::now() < next_tick || tick_now(); };
    auto save_image = [&](long long t) -> bool {      // 's' and the final output
        HostBuf out;
        if (st.read_board(out)) { die(st.err); return false; }
        const std::string name = fname + "x" + std::to_string(t);
        std::string err;
        if (write_pgm(out_dir, name, W, H, out, err)) { die(err); return false; }
        gol_event e = make_ev(GOL_EV_IMAGE_OUTPUT_COMPLETE, t);
        std::snprintf(e.filename, sizeof e.filename, "%s", name.c_str());
        return send(e);
    };

    HostBuf prev;                                     // CellFlipped: previous board
    if (emit_cell_flipped) {
        if (!prev.alloc((size_t)W * H)) return die("out of host memory");
        std::memcpy(prev.data(), pix, (size_t)W * H);
    }
    pix = nullptr;
    file.release();

    long long chunk = 1;
    bool quit = false, killed = false;
    // Chunks in flight: the engines' launches are enqueued without a host sync per chunk; the
    // host waits only for the chunk before the newest one, so the GPUs never idle between
    // chunks (a sync per chunk left a launch-latency bubble each ~4 ms) and a key or a tick is
    // served within ~2 chunks.  Strip runs get the same bound as a single engine's control
    // word gives it (their engines stay in lockstep: no per-engine STOP).
    struct Chunk {
        long long first = 0, n = 0;
        std::vector<hipEvent_t> ev;
    };
    std::deque<Chunk> inflight;
    auto drop_events = [&]() {
        for (Chunk &c : inflight)
            for (hipEvent_t e : c.ev) (void)hipEventDestroy(e);
        inflight.clear();
    };
    struct InflightScope {
        std::function<void()> f;
        ~InflightScope() { f(); }
    } inflight_scope{drop_events};
    // wait until at most `keep` chunks are in flight; TurnComplete for the retired turns
    auto retire = [&](size_t keep) -> bool {
        while (inflight.size() > keep) {
            Chunk &c = inflight.front();
            for (size_t i = 0; i < c.ev.size(); i++) {
                const hipError_t e = hipEventSynchronize(c.ev[i]);
                (void)hipEventDestroy(c.ev[i]);
                c.ev[i] = nullptr;
                if (e != hipSuccess) {
                    for (size_t j = i + 1; j < c.ev.size(); j++) (void)hipEventDestroy(c.ev[j]);
                    c.ev.clear();
                    inflight.pop_front();
                    die(std::string("chunk wait: ") + hipGetErrorString(e));
                    return false;
                }
            }
            if (emit_turn_complete)
                for (long long t = 1; t <= c.n; t++)
                    if (!send(make_ev(GOL_EV_TURN_COMPLETE, c.first + t))) {
                        c.ev.clear();
                        inflight.pop_front();
                        return false;
                    }
            c.ev.clear();
            inflight.pop_front();
        }
        return true;
    };
    struct CtlScope {   // the key thread may interrupt this run's engine while it lives
        gol_run *r;
        CtlScope(gol_run *r_, gol_ctx *e) : r(r_) { r->set_ctl_engine(e); }
        ~CtlScope() { r->set_ctl_engine(nullptr); }
    } ctl_scope(this, st.strip_mode() ? nullptr : st.eng[0]);
    while (turn < p.turns && !quit) {
        if (abort.load()) return close();
        // re-arm before draining the keys: a key pushed from here on stops the next chunk
        if (!st.strip_mode()) (void)gol_set_control(st.eng[0], GOL_CONTROL_RUN);
        int k;
        bool drained = false;
        while (!quit && pop_key(k)) {
            // a key sees every enqueued turn done, and its events follow their TurnComplete
            // events: drain after the pop (checking for a key first and popping later let a key
            // that arrived in between be served with the previous chunk still in flight)
            if (!drained) {
                if (!retire(0)) return close();
                if (st.sync()) return die(st.err);
                drained = true;
            }
            if (k == 's') {                           // distributor.go:131-144
                if (!save_image(turn)) return close();
            } else if (k == 'q' || k == 'k') {        // :113-115, :146-150
                quit = true;
                killed = killed || k == 'k';
            } else if (k == 'p') {                    // :117-130, Server :147-156
                gol_event e = make_ev(GOL_EV_STATE_CHANGE, turn);
                e.new_state = GOL_PAUSED;
                if (!send(e)) return close();
                for (;;) {
                    if (abort.load()) return close();
                    if (!tick()) return close();
                    std::unique_lock<std::mutex> lk(kmu);
                    kcv.wait_for(lk, std::chrono::milliseconds(20), [&] { return !keys.empty(); });
                    if (keys.empty()) continue;
                    const int k2 = keys.front();
                    keys.pop_front();
                    if (k2 == 'p') break;             // other keys are swallowed while paused
                }
                e = make_ev(GOL_EV_STATE_CHANGE, turn);
                e.new_state = GOL_EXECUTING;
                if (!send(e)) return close();
            }
        }
        if (quit) break;
        if (Clock::now() >= next_tick) {              // one clock read decides: drain, then tick
            if (!retire(0)) return close();
            if (!tick_now()) return close();
        }

        const long long want = std::min(chunk, p.turns - turn);
        const auto t0 = Clock::now();
        const long long before = st.engine_turn();
        if (st.step(want)) return die(st.err);
        const long long n = st.engine_turn() - before;   // < want if a key interrupted it
        if (!emit_cell_flipped) {
            Chunk c;
            c.first = turn;
            c.n = n;
            for (auto *e : st.eng) {
                hipEvent_t ev = nullptr;
                if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
                    hipEventRecord(ev, (hipStream_t)gol_get_stream(e)) != hipSuccess) {
                    if (ev) (void)hipEventDestroy(ev);
                    for (hipEvent_t x : c.ev) (void)hipEventDestroy(x);
                    return die("chunk event: HIP error");
                }
                c.ev.push_back(ev);
            }
            inflight.push_back(std::move(c));
            turn += n;
            if (!retire(1)) return close();
            // aim for ~2 ms of GPU work per chunk: with one chunk queued behind the running
            // one, an iteration takes about a chunk's GPU time
            const double ms =
                std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
            if (ms < 1.0) chunk = std::min<long long>(chunk * 2, 1 << 20);
            else if (ms > 4.0 && chunk > 1) chunk /= 2;
            continue;
        }
        if (st.sync()) return die(st.err);
        {
            HostBuf cur;
            if (st.read_board(cur)) return die(st.err);
            // with CellFlipped on, chunks are single turns so every flip is reported
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++)
                    if (cur.data()[(size_t)y * W + x] != prev.data()[(size_t)y * W + x]) {
                        gol_event cf = make_ev(GOL_EV_CELL_FLIPPED, turn + 1);
                        cf.x = x;
                        cf.y = y;
                        if (!send(cf)) return close();
                    }
            std::swap(prev, cur);
        }
        if (emit_turn_complete)
            for (long long t = 1; t <= n; t++)
                if (!send(make_ev(GOL_EV_TURN_COMPLETE, turn + t))) return close();
        turn += n;
    }
    if (!retire(0)) return close();
    if (st.sync()) return die(st.err);

    // retain the final board for a later CONT=yes run; 'k' kills the "server" and its state
    {
        RetainedState &rs = retained();
        std::lock_guard<std::mutex> lk(rs.mu);
        rs.valid = false;
        if (!killed) {
            if (st.read_packed(rs.words)) return die(st.err);
            rs.W = W;
            rs.H = H;
            rs.turn = turn;
            rs.valid = true;
        } else {
            rs.words.clear();
        }
    }

    // FinalTurnComplete{turn, calculateAliveCells} -> StateChange Quitting ->
    // PGM out/WxHxT -> ImageOutputComplete -> close  (distributor.go:187-226)
    auto cells = std::make_shared<std::vector<int64_t>>();
    if (st.alive_cells(*cells)) return die(st.err);
    gol_event fe = make_ev(GOL_EV_FINAL_TURN_COMPLETE, turn);
    fe.cells_count = (int64_t)(cells->size() / 2);
    if (!send(fe, cells)) return close();
    gol_event qe = make_ev(GOL_EV_STATE_CHANGE, turn);
    qe.new_state = GOL_QUITTING;
    if (!send(qe)) return close();
    if (!save_image(turn)) return close();
    close();
}

// why the calling thread's last gol_run_start failed after it had validated its arguments
// (gol_run_error(NULL)); cleared by a start that succeeds
thread_local std::string t_start_error;

extern "C" {

int gol_run_start(const gol_params *p, const gol_run_options *o, gol_run **out)
{
    if (!p || !out) return GOL_EINVAL;
    *out = nullptr;
    if (p->image_width < 2 || p->image_height < 1 || p->turns < 0) return GOL_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return GOL_ENODEV;
    gol_run *r = new (std::nothrow) gol_run();
    if (!r) return GOL_ENOMEM;
    r->p = *p;
    if (o) {
        if (o->image_dir) r->image_dir = o->image_dir;
        if (o->out_dir) r->out_dir = o->out_dir;
        if (o->ngpus > 0) r->ngpus = o->ngpus;
        r->halo = o->halo;
        if (o->ticker_ms > 0) r->ticker_ms = o->ticker_ms;
        if (o->event_capacity > 0) r->capacity = (size_t)o->event_capacity;
        r->emit_turn_complete = o->emit_turn_complete != 0;
        r->emit_cell_flipped = o->emit_cell_flipped != 0;
        r->engine_flags = o->engine_flags;
        r->resume = o->resume;
    }
    for (int i = 0; i < r->ngpus; i++)
        r->devices.push_back(o && o->devices ? o->devices[i] : i % ndev);
    for (int d : r->devices)
        if (d < 0 || d >= ndev) {
            delete r;
            return GOL_ENODEV;
        }
    // peer access between the strips' devices (xGMI); same-device strips need none.  A device
    // pair that reports peer access but refuses to enable it fails the start with GOL_EHIP and
    // the reason in gol_run_error(NULL) -- the reference's dial-or-fatal for a SubServer it
    // cannot reach (Server/gol/distributor.go:87-97) -- instead of halo copies that fail or
    // silently stage through the host later.  A pair without peer access at all still runs:
    // hipMemcpyPeerAsync stages its copies.
    for (size_t i = 0; i < r->devices.size(); i++)
        for (size_t j = 0; j < r->devices.size(); j++) {
            const int a = r->devices[i], b = r->devices[j];
            if (a == b) continue;
            int can = 0;
            const hipError_t qe = hipDeviceCanAccessPeer(&can, a, b);
            int rc = GOL_OK;
            char msg[256];
            if (qe != hipSuccess) {
                rc = gol_internal_peer_access_status("hipDeviceCanAccessPeer", (int)qe,
                                                     hipGetErrorName(qe), a, b, msg, sizeof msg);
            } else if (can) {
                int prev = 0;
                (void)hipGetDevice(&prev);
                (void)hipSetDevice(a);
                const hipError_t pe = hipDeviceEnablePeerAccess(b, 0);
                (void)hipGetLastError();
                (void)hipSetDevice(prev);
                rc = gol_internal_peer_access_status("hipDeviceEnablePeerAccess", (int)pe,
                                                     hipGetErrorName(pe), a, b, msg, sizeof msg);
            }
            if (rc != GOL_OK) {
                t_start_error = msg;
                delete r;
                return rc;
            }
        }
    t_start_error.clear();
    r->th = std::thread([r] { r->run(); });
    *out = r;
    return GOL_OK;
}

int gol_run_next_event(gol_run *r, gol_event *ev, int32_t timeout_ms)
{
    if (!r || !ev) return GOL_EINVAL;
    std::unique_lock<std::mutex> lk(r->mu);
    auto ready = [&] { return !r->q.empty() || r->closed; };
    if (timeout_ms < 0) r->cv_pop.wait(lk, ready);
    else if (!r->cv_pop.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready))
        return GOL_ETIMEDOUT;
    if (r->q.empty()) return GOL_ECLOSED;
    Item it = std::move(r->q.front());
    r->q.pop_front();
    r->cv_push.notify_one();
    *ev = it.ev;
    if (it.ev.type == GOL_EV_FINAL_TURN_COMPLETE) r->last_final = it.cells;
    return GOL_OK;
}

int64_t gol_run_final_alive(gol_run *r, int64_t *xy, int64_t cap)
{
    if (!r) return GOL_EINVAL;
    std::lock_guard<std::mutex> lk(r->mu);
    if (!r->last_final) return GOL_ESTATE;
    const int64_t n = (int64_t)(r->last_final->size() / 2);
    if (xy && cap > 0)
        std::memcpy(xy, r->last_final->data(), (size_t)std::min(n, cap) * 2 * sizeof(int64_t));
    return n;
}

int gol_run_key(gol_run *r, int32_t rune)
{
    if (!r) return GOL_EINVAL;
    {
        std::lock_guard<std::mutex> lk(r->kmu);
        r->keys.push_back(rune);
        r->kcv.notify_all();
    }
    if (rune == 's' || rune == 'p' || rune == 'q' || rune == 'k') r->interrupt();
    return GOL_OK;
}

// The result of one peer-access call between two strips' devices, mapped to a return code and
// a message: success and "already enabled" (an earlier run in the process enabled it) are
// GOL_OK, anything else GOL_EHIP with the call, the HIP error and the device pair.  Pure (no
// HIP call), so the CPU tests check the mapping (tests/test_abi.py).
int gol_internal_peer_access_status(const char *call, int hip_error, const char *hip_name,
                                    int dev_a, int dev_b, char *msg, size_t cap)
{
    if (hip_error == (int)hipSuccess || hip_error == (int)hipErrorPeerAccessAlreadyEnabled) {
        if (msg && cap) msg[0] = '\0';
        return GOL_OK;
    }
    if (msg && cap)
        snprintf(msg, cap, "%s(%d -> %d) failed: %s (%d): the strips on devices %d and %d "
                 "cannot exchange halos by peer copies", call ? call : "peer access", dev_a, dev_b,
                 hip_name ? hip_name : "?", hip_error, dev_a, dev_b);
    return GOL_EHIP;
}

const char *gol_run_error(gol_run *r)
{
    if (!r) return t_start_error.c_str();
    std::lock_guard<std::mutex> lk(r->mu);
    return r->error.c_str();
}

void gol_run_destroy(gol_run *r)
{
    if (!r) return;
    r->abort.store(true);
    {
        std::lock_guard<std::mutex> lk(r->mu);
        r->cv_push.notify_all();
    }
    r->kcv.notify_all();
    if (r->th.joinable()) r->th.join();
    delete r;
}

}  // extern "C"
