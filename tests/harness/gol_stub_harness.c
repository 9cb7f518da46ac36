/* gol_stub_harness.c -- the cgo stub of INTEGRATION.md ("Go binding"), goroutine for
 * goroutine, in C with pthreads over libgolamd.so, so its control flow runs somewhere: no Go
 * toolchain exists in this image or on the GPU box.  Test infrastructure only
 * (tests/test_gpu_run.py::test_stub_harness_*).
 *
 * The reference controller (Local/gol/distributor.go:55-227) has three goroutines, and so does
 * this harness:
 *   main    -- reads the PGM, creates the engine, emits StateChange{0, Executing}, then runs
 *              the WHOLE game in one call, as the reference's one API.ServerDistributor RPC
 *              (:182): gol_step(ctx, Turns), which returns early (GOL_STOPPED) after 'q' / 'k'.
 *              Then Alivecount for the end turn (:188-190), FinalTurnComplete, StateChange
 *              Quitting, the PGM out/WxHxT, ImageOutputComplete, close (:194-226).
 *   keys    -- (:107-152) 'q' / 'k': the control word STOP (CFput{2} / {5});
 *              'p': PAUSE, wait until gol_step is parked at a launch boundary, StateChange
 *              {turn, Paused}, swallow keys until the next 'p', StateChange{turn, Executing},
 *              RUN (CFput{0} twice);
 *              's': gol_get_world -- the GetWorld pair {SWorld, TurnCur} (:131-144), served
 *              while gol_step runs -- written as out/WxHxTurnCur.pgm, ImageOutputComplete.
 *   ticker  -- (:154-167) every ticker_ms: gol_snapshot (Alivecount) -> AliveCellsCount.  No
 *              STOP: the snapshot is served at the next launch boundary while gol_step runs,
 *              and at once while it is parked, so the ticker keeps firing while paused.  It
 *              ends on the unbuffered `done` channel (:59, :162-163, :198): main's send returns
 *              only once the ticker is back in its select, i.e. after any tick in flight has
 *              emitted its AliveCellsCount.  Here main sends right after gol_step returns, so
 *              no AliveCellsCount follows FinalTurnComplete / StateChange Quitting.  That order
 *              is STRICTER than the reference, not a copy of it: distributor.go sends
 *              FinalTurnComplete and Quitting (:194-195) before ticker.Stop and done <- true
 *              (:197-198), so in the reference a tick that fires in between can still emit an
 *              AliveCellsCount after Quitting.  Every event sequence this harness produces is
 *              one the reference can produce.
 * GOL_HARNESS_TICK_DELAY_MS (tests): sleep between a tick's snapshot and its event, so a tick is
 * in flight when the run ends.
 *
 * usage: gol_stub_harness W H TURNS IMAGE_DIR OUT_DIR TICKER_MS [TURN_COMPLETE]
 * stdin: one key rune per line.  stdout: one event per line, then "CLOSED":
 *   StateChange <turn> Executing|Paused|Quitting     AliveCellsCount <turn> <cells>
 *   ImageOutputComplete <turn> <name>                FinalTurnComplete <turn> <cells>
 *   TurnComplete <turn>   (TURN_COMPLETE = 1: every turn, after the run -- the reference
 *                          emits none, Local/gol/distributor.go:184-185)
 * Exit status 0, or 2 with "ERROR ..." on stdout. */
#include <errno.h>
#include <poll.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "gol_amd.h"

static pthread_mutex_t g_out = PTHREAD_MUTEX_INITIALIZER;   /* the events channel */
static pthread_mutex_t g_ctx = PTHREAD_MUTEX_INITIALIZER;   /* engine lifetime vs key thread */
static gol_ctx *g_e;
static int g_w, g_h;
static const char *g_out_dir;
static volatile int g_step_done;                             /* gol_step returned */
static volatile int g_finished;                              /* ... and main owns the engine */

/* an unbuffered Go channel of one value type, for `done` (distributor.go:59): chan_send
 * blocks until a receiver has taken the value; chan_recv_timeout is one `select` with a timer */
struct chan0 {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int full, taken;
};
static struct chan0 g_done = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, 0, 0};

static void chan_send(struct chan0 *c)
{
    pthread_mutex_lock(&c->mu);
    c->full = 1;
    c->taken = 0;
    pthread_cond_broadcast(&c->cv);
    while (!c->taken) pthread_cond_wait(&c->cv, &c->mu);
    pthread_mutex_unlock(&c->mu);
}

/* 1: received; 0: `ms` elapsed first (the ticker's case) */
static int chan_recv_timeout(struct chan0 *c, int ms)
{
    struct timespec dl;
    clock_gettime(CLOCK_REALTIME, &dl);
    dl.tv_sec += ms / 1000;
    dl.tv_nsec += (long)(ms % 1000) * 1000000L;
    if (dl.tv_nsec >= 1000000000L) {
        dl.tv_sec++;
        dl.tv_nsec -= 1000000000L;
    }
    pthread_mutex_lock(&c->mu);
    int got = 0;
    while (!c->full)
        if (pthread_cond_timedwait(&c->cv, &c->mu, &dl) == ETIMEDOUT) break;
    if (c->full) {
        c->full = 0;
        c->taken = 1;
        got = 1;
        pthread_cond_broadcast(&c->cv);
    }
    pthread_mutex_unlock(&c->mu);
    return got;
}

static void emit(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    pthread_mutex_lock(&g_out);
    vprintf(fmt, ap);
    putchar('\n');
    fflush(stdout);
    pthread_mutex_unlock(&g_out);
    va_end(ap);
}

static void die(const char *what, int rc)
{
    emit("ERROR %s: %s %s", what, gol_strerror(rc), g_e ? gol_last_error(g_e) : "");
    exit(2);
}

static void sleep_ms(int ms)
{
    struct timespec ts = {ms / 1000, (long)(ms % 1000) * 1000000L};
    while (nanosleep(&ts, &ts) == -1 && errno == EINTR) {
    }
}

/* the io goroutine's PGM reader (Local/gol/io.go:88-121): whitespace-separated fields */
static uint8_t *read_pgm(const char *path, int w, int h)
{
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    char magic[3] = {0};
    int fw = 0, fh = 0, maxv = 0;
    if (fscanf(f, "%2s %d %d %d", magic, &fw, &fh, &maxv) != 4 || strcmp(magic, "P5") ||
        fw != w || fh != h || maxv != 255 || fgetc(f) == EOF) {
        fclose(f);
        return NULL;
    }
    uint8_t *b = malloc((size_t)w * h);
    if (b && fread(b, 1, (size_t)w * h, f) != (size_t)w * h) {
        free(b);
        b = NULL;
    }
    fclose(f);
    return b;
}

/* the io goroutine's writer (io.go:42-76): out/{name}.pgm, header "P5\nW H\n255\n" */
static int write_pgm(const char *name, const uint8_t *b)
{
    char path[1024];
    snprintf(path, sizeof path, "%s/%s.pgm", g_out_dir, name);
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    fprintf(f, "P5\n%d %d\n255\n", g_w, g_h);
    const size_t n = fwrite(b, 1, (size_t)g_w * g_h, f);
    return fclose(f) == 0 && n == (size_t)g_w * g_h ? 0 : -1;
}

static int next_key(void)       /* one rune per stdin line; -1 at EOF or once the run ended */
{
    char line[64];
    for (;;) {
        struct pollfd p = {0, POLLIN, 0};
        const int r = poll(&p, 1, 50);
        if (g_finished) return -1;
        if (r <= 0) continue;
        if (!fgets(line, sizeof line, stdin)) return -1;
        if (line[0] && line[0] != '\n') return (unsigned char)line[0];
    }
}

static void *ticker(void *arg)
{
    const int ms = *(const int *)arg;
    const char *d = getenv("GOL_HARNESS_TICK_DELAY_MS");
    const int delay = d ? atoi(d) : 0;
    for (;;) {
        if (chan_recv_timeout(&g_done, ms)) return NULL;     /* case <-done: return */
        int64_t t = 0, alive = 0;                            /* case <-ticker.C: */
        const int rc = gol_snapshot(g_e, &t, &alive);          /* API.Alivecount */
        if (rc) die("gol_snapshot", rc);
        if (delay > 0) sleep_ms(delay);
        emit("AliveCellsCount %lld %lld", (long long)t, (long long)alive);
    }
}

static void *keys(void *arg)
{
    (void)arg;
    uint8_t *world = malloc((size_t)g_w * g_h);
    for (int k; (k = next_key()) >= 0;) {
        pthread_mutex_lock(&g_ctx);
        if (g_finished) {                                     /* the run is over: ignored */
            pthread_mutex_unlock(&g_ctx);
            break;
        }
        if (k == 'q' || k == 'k') {                           /* CFput{2} / CFput{5} */
            gol_set_control(g_e, GOL_CONTROL_STOP);
        } else if (k == 's') {                                /* GetWorld -> out/WxHxTurnCur */
            int64_t t = 0;
            const int rc = gol_get_world(g_e, world, &t);
            if (rc) die("gol_get_world", rc);
            char name[128];
            snprintf(name, sizeof name, "%dx%dx%lld", g_w, g_h, (long long)t);
            if (write_pgm(name, world)) die("write_pgm", GOL_EIO);
            emit("ImageOutputComplete %lld %s", (long long)t, name);
        } else if (k == 'p') {                                /* CFput{0}: pause */
            gol_set_control(g_e, GOL_CONTROL_PAUSE);
            int64_t t = 0;
            int32_t parked = 0;
            int over = 0;                      /* the step ended before it parked */
            while (!parked && !over) {
                gol_get_progress(g_e, &t, &parked);
                if (g_step_done) over = !parked;
                else if (!parked) sleep_ms(1);
            }
            if (over) {                        /* (main is waiting for g_ctx to finish) */
                pthread_mutex_unlock(&g_ctx);
                continue;
            }
            pthread_mutex_unlock(&g_ctx);
            emit("StateChange %lld Paused", (long long)t);
            int k2;
            while ((k2 = next_key()) >= 0 && k2 != 'p') {   /* other keys: swallowed */
            }
            pthread_mutex_lock(&g_ctx);
            emit("StateChange %lld Executing", (long long)t);
            if (!g_finished) gol_set_control(g_e, GOL_CONTROL_RUN);   /* CFput{0}: resume */
        }
        pthread_mutex_unlock(&g_ctx);
    }
    free(world);
    return NULL;
}

int main(int argc, char **argv)
{
    if (argc != 7 && argc != 8) {
        fprintf(stderr, "usage: %s W H TURNS IMAGE_DIR OUT_DIR TICKER_MS [TURN_COMPLETE]\n",
                argv[0]);
        return 1;
    }
    g_w = atoi(argv[1]);
    g_h = atoi(argv[2]);
    const long long turns = atoll(argv[3]);
    g_out_dir = argv[5];
    int ticker_ms = atoi(argv[6]);
    const int turn_complete = argc == 8 && atoi(argv[7]) != 0;
    char path[1024];
    snprintf(path, sizeof path, "%s/%dx%d.pgm", argv[4], g_w, g_h);
    uint8_t *world = read_pgm(path, g_w, g_h);                /* ioInput */
    if (!world) die(path, GOL_EIO);

    int rc = gol_create(g_w, g_h, 0, &g_e);
    if (rc) die("gol_create", rc);
    if ((rc = gol_load(g_e, world))) die("gol_load", rc);
    gol_set_control(g_e, GOL_CONTROL_RUN);                    /* arm the control word */
    emit("StateChange 0 Executing");

    pthread_t tk, kt;
    pthread_create(&tk, NULL, ticker, &ticker_ms);
    pthread_create(&kt, NULL, keys, NULL);

    rc = gol_step(g_e, turns);                                /* API.ServerDistributor */
    g_step_done = 1;
    if (rc < 0) die("gol_step", rc);
    pthread_mutex_lock(&g_ctx);                               /* (a key being served ends) */
    g_finished = 1;
    pthread_mutex_unlock(&g_ctx);
    chan_send(&g_done);                                       /* ticker.Stop(); done <- true */

    int64_t turn = 0, alive = 0;
    if ((rc = gol_snapshot(g_e, &turn, &alive))) die("gol_snapshot", rc);   /* Alivecount */
    for (long long t = 1; turn_complete && t <= turn; t++) emit("TurnComplete %lld", t);
    emit("FinalTurnComplete %lld %lld", (long long)turn, (long long)alive);
    emit("StateChange %lld Quitting", (long long)turn);
    if ((rc = gol_read_board(g_e, world))) die("gol_read_board", rc);
    char name[128];
    snprintf(name, sizeof name, "%dx%dx%lld", g_w, g_h, (long long)turn);
    if (write_pgm(name, world)) die("write_pgm", GOL_EIO);
    emit("ImageOutputComplete %lld %s", (long long)turn, name);
    pthread_join(kt, NULL);
    pthread_join(tk, NULL);                                   /* (returned at the done receive) */
    gol_destroy(g_e);
    free(world);
    emit("CLOSED");
    return 0;
}
