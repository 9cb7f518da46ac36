/*
 * oracle/refcpu.c — CPU restatement of the reference's per-turn board update.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (conway-s-gol-distributed_amd/)
 * links, loads or calls this file.  It is imported only by tests/, by
 * __graft_entry__.smoke() as a checker, and by bench.py's `cpu_baseline` leg.
 *
 * What it restates (all paths relative to the reference repo
 * joyce-leesw/Conway-s-GOL-Distributed):
 *   - calculateNextState              SubServer/distributor.go:119-208
 *       byte cells, alive iff == 255, x-wrap inside the row (:136-145),
 *       y-neighbours from the strip's halo rows (:148-149), B3/S23 rule
 *       (:178-200), output rows zero-initialised (:122-125) so a centre cell
 *       that is neither 0 nor 255 always produces 0.
 *   - SubServer thread split          SubServer/distributor.go:48-117
 *       base = len/T, first len%T workers +1 (:53-63); worker slices with the
 *       "wrap inside the strip" quirk (:96-112) whose halo-row outputs are
 *       garbage and are discarded by the Server.
 *   - Server row-strip split          Server/gol/distributor.go:104-134,185-224
 *       base = H/N, first H%N strips +1 (:106-116); haloed strip assembly with
 *       global torus wrap (:197-213); part[1:len-1] (:223); gather (:124-129).
 *   - Alive count / alive list        Server/gol/distributor.go:173-183,
 *                                     Local/gol/distributor.go:229-239
 *
 * The Go reference cannot be built here (no Go toolchain), so
 * this restatement is pinned by the reference's own golden fixtures
 * (Local/check/images/ and Local/check/alive/) in tests/test_oracle.py.
 *
 * Threading: every (strip, worker) pair of one turn is one OpenMP task, the
 * way every SubServer worker is one goroutine.  The per-turn gob/HTTP
 * serialisation of the reference is NOT reproduced, so timings from this file
 * are an optimistic upper bound on the reference's own speed.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* calculateNextState — SubServer/distributor.go:119-208.
 * world: `len` row pointers (row 0 and row len-1 are the halo rows).
 * out:   len-2 row pointers, each `width` bytes. */
static void calculate_next_state(const uint8_t *const *world, int len, int width,
                                 uint8_t *const *out)
{
    for (int y = 0; y < len - 2; y++) {               /* :129 range tempW */
        const uint8_t *s = world[y + 1];               /* tempW = world[1:len-1] (:127) */
        const uint8_t *up = world[y];                  /* lastY = y      (:149) */
        const uint8_t *dn = world[y + 2];              /* nextY = y + 2  (:148) */
        uint8_t *o = out[y];
        memset(o, 0, (size_t)width);                   /* make([]uint8, W) (:124) */
        for (int x = 0; x < width; x++) {
            int nextX, lastX;
            if (x == width - 1) { nextX = 0; lastX = x - 1; }        /* :136-138 */
            else if (x == 0)    { nextX = x + 1; lastX = width - 1; }/* :139-141 */
            else                { nextX = x + 1; lastX = x - 1; }    /* :142-144 */
            int counter = 0;
            if (s[nextX] == 255) counter++;            /* E  :151 */
            if (s[lastX] == 255) counter++;            /* W  :154 */
            if (up[lastX] == 255) counter++;           /* NW :158 */
            if (up[x] == 255) counter++;               /* N  :161 */
            if (up[nextX] == 255) counter++;           /* NE :164 */
            if (dn[lastX] == 255) counter++;           /* SW :168 */
            if (dn[x] == 255) counter++;               /* S  :171 */
            if (dn[nextX] == 255) counter++;           /* SE :174 */
            const uint8_t sl = s[x];
            if (sl == 255)                             /* :179-186 */
                o[x] = (counter < 2 || counter > 3) ? 0 : 255;
            if (sl == 0)                               /* :191-198 */
                o[x] = (counter == 3) ? 255 : 0;
            /* any other value: stays 0 from the zero-initialised row */
        }
    }
}

/* base/remainder split used by both the Server (:106-116) and the SubServer (:53-63). */
static void split_lines(int total, int parts, int *lines)
{
    int base = total / parts, slack = total % parts;
    for (int i = 0; i < parts; i++) lines[i] = base + (i < slack ? 1 : 0);
}

/* One SubServer worker's slice (SubServer/distributor.go:86-117), returned as
 * a freshly built row-pointer list `go` of length *golen. */
static void subserver_worker_slice(const uint8_t *const *strip, int L, const int *lines,
                                   int T, int j, const uint8_t **go, int *golen)
{
    int comp = 0;
    for (int i = 0; i < j; i++) comp += lines[i];
    int n = 0;
    if (j == 0) {                                       /* :96-105 */
        go[n++] = strip[L - 1];
        if (T == 1) {
            for (int r = 0; r < L; r++) go[n++] = strip[r];
            go[n++] = strip[0];
        } else {
            for (int r = 0; r < lines[0] + 1; r++) go[n++] = strip[r];
        }
    } else if (j == T - 1) {                            /* :107-109 */
        for (int r = comp - 1; r < L; r++) go[n++] = strip[r];
        go[n++] = strip[0];
    } else {                                            /* :110-111 */
        for (int r = comp - 1; r < comp + lines[j] + 1; r++) go[n++] = strip[r];
    }
    *golen = n;
}

/* Server worker's haloed strip (Server/gol/distributor.go:185-213). */
static int server_strip(const uint8_t *const *world, int H, const int *lines, int N, int i,
                        const uint8_t **strip)
{
    int comp = 0;
    for (int k = 0; k < i; k++) comp += lines[k];
    int n = 0;
    if (i == 0) {                                       /* :197-206 */
        strip[n++] = world[H - 1];
        if (N == 1) {
            for (int r = 0; r < H; r++) strip[n++] = world[r];
            strip[n++] = world[0];
        } else {
            for (int r = 0; r < lines[0] + 1; r++) strip[n++] = world[r];
        }
    } else if (i == N - 1) {                            /* :208-210 */
        for (int r = comp - 1; r < H; r++) strip[n++] = world[r];
        strip[n++] = world[0];
    } else {                                            /* :211-212 */
        for (int r = comp - 1; r < comp + lines[i] + 1; r++) strip[n++] = world[r];
    }
    return n;
}

/*
 * ref_run — `turns` turns of the reference Server turn loop
 * (Server/gol/distributor.go:104-134) over an H x W byte board, with `nsub`
 * sub-servers each splitting their strip over `threads` workers, executed on
 * `ncores` OpenMP threads (0 = library default).  board is updated in place.
 * Returns 0, -1 on bad arguments / allocation failure, or -2 when the
 * reference itself would panic: a SubServer worker slices
 * world[compLines-1 : compLines+lines[i]+1] (SubServer/distributor.go:111),
 * which runs past the strip whenever threads > strip rows + 2 (Go: "slice
 * bounds out of range"); e.g. a 16x16 board on 4 sub-servers with Threads > 6.
 */
int ref_run(uint8_t *board, int W, int H, long long turns, int nsub, int threads, int ncores)
{
    if (!board || W < 2 || H < 1 || nsub < 1 || threads < 1 || nsub > H) return -1;
    uint8_t *next = (uint8_t *)malloc((size_t)W * H);
    const uint8_t **world = (const uint8_t **)malloc(sizeof(void *) * (size_t)H);
    int *slines = (int *)malloc(sizeof(int) * (size_t)nsub);
    /* per strip: the strip row list, its thread split, and per worker its slice */
    int maxL = H + 2;
    const uint8_t **strips = (const uint8_t **)malloc(sizeof(void *) * (size_t)nsub * (maxL + 2));
    int *slen = (int *)malloc(sizeof(int) * (size_t)nsub);
    int *tlines = (int *)malloc(sizeof(int) * (size_t)nsub * threads);
    int ntask = nsub * threads;
    /* scratch output rows for the discarded halo outputs: 2 per strip */
    uint8_t *scratch = (uint8_t *)malloc((size_t)W * 2 * nsub);
    if (!next || !world || !slines || !strips || !slen || !tlines || !scratch) {
        free(next); free(world); free(slines); free(strips); free(slen); free(tlines); free(scratch);
        return -1;
    }
#ifdef _OPENMP
    if (ncores > 0) omp_set_num_threads(ncores);
#else
    (void)ncores;
#endif
    uint8_t *cur = board, *nxt = next;
    split_lines(H, nsub, slines);
    for (int i = 0; i < nsub; i++)
        if (threads > 1 && threads > slines[i] + 2) {
            free(next); free(world); free(slines); free(strips); free(slen); free(tlines);
            free(scratch);
            return -2;
        }
    for (long long t = 0; t < turns; t++) {
        for (int y = 0; y < H; y++) world[y] = cur + (size_t)y * W;
        int off = 0;
        for (int i = 0; i < nsub; i++) {
            const uint8_t **st = strips + (size_t)i * (maxL + 2);
            slen[i] = server_strip(world, H, slines, nsub, i, st);
            split_lines(slen[i], threads, tlines + (size_t)i * threads);
            (void)off;
        }
        #pragma omp parallel for schedule(dynamic, 1)
        for (int task = 0; task < ntask; task++) {
            int i = task / threads, j = task % threads;
            const uint8_t **st = strips + (size_t)i * (maxL + 2);
            int L = slen[i];
            const int *tl = tlines + (size_t)i * threads;
            const uint8_t **go = (const uint8_t **)malloc(sizeof(void *) * (size_t)(L + 3));
            uint8_t **out = (uint8_t **)malloc(sizeof(void *) * (size_t)(L + 3));
            int golen = 0;
            subserver_worker_slice(st, L, tl, threads, j, go, &golen);
            int comp = 0;
            for (int k = 0; k < j; k++) comp += tl[k];
            int soff = 0;
            for (int k = 0; k < i; k++) soff += slines[k];
            /* worker j produces strip rows [comp, comp + golen - 2); strip row k
             * (1 <= k <= L-2) is global row soff + k - 1; rows 0 and L-1 are the
             * halo outputs the Server discards (:223). */
            for (int k = 0; k < golen - 2; k++) {
                int srow = comp + k;
                if (srow >= 1 && srow <= L - 2)
                    out[k] = nxt + (size_t)(soff + srow - 1) * W;
                else
                    out[k] = scratch + (size_t)W * (2 * i + (srow == 0 ? 0 : 1));
            }
            if (golen > 2) calculate_next_state(go, golen, W, out);
            free(go); free(out);
        }
        uint8_t *tmp = cur; cur = nxt; nxt = tmp;
    }
    if (cur != board) memcpy(board, cur, (size_t)W * H);
    free(next); free(world); free(slines); free(strips); free(slen); free(tlines); free(scratch);
    return 0;
}

/* calculateAliveCells — Server/gol/distributor.go:173-183 (the reference
 * iterates x < len(world), i.e. square boards only; this iterates x < W). */
long long ref_alive_count(const uint8_t *board, int W, int H)
{
    long long n = 0;
    for (size_t i = 0; i < (size_t)W * H; i++) n += board[i] == 255;
    return n;
}

/* calculateAliveCells — Local/gol/distributor.go:229-239: row-major {X,Y}
 * list of cells == 255.  Writes at most cap pairs, returns the total count. */
long long ref_alive_cells(const uint8_t *board, int W, int H, long long *xy, long long cap)
{
    long long n = 0;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++)
            if (board[(size_t)y * W + x] == 255) {
                if (n < cap) { xy[2 * n] = x; xy[2 * n + 1] = y; }
                n++;
            }
    return n;
}
