/*
 * gol_amd.h — C ABI of the MI355X-native Game of Life engine (libgolamd.so).
 *
 * Drop-in boundary for the reference's per-turn board update
 * (joyce-leesw/Conway-s-GOL-Distributed).  The reference crosses this boundary
 * with Go net/rpc calls whose payload is a gob-encoded [][]uint8 board; here it
 * is a plain C ABI (opaque handles, pointers + sizes, int error codes, no
 * exceptions and no torch types), so a cgo / ctypes / JNI binding is a thin stub
 * (INTEGRATION.md shows the cgo one).
 *
 * Two layers:
 *
 *  1. Engine (gol_ctx): one MI355X, one board or one row strip of a board.
 *     Owns every device buffer (double-buffered bit-packed board, 64 cells per
 *     uint64 word, LSB = lowest x; optional non-binary "blocked" mask; popcount
 *     shards).  Replaces, per GPU:
 *       API.SubServerDistributor          SubServer/distributor.go:48-84
 *       calculateNextState                SubServer/distributor.go:119-208
 *       the Server turn loop + commit     Server/gol/distributor.go:104-134
 *       API.Alivecount / calculateAliveCells  Server/gol/distributor.go:69-75,173-183
 *       API.GetWorld                      Server/gol/distributor.go:62-67
 *       Local calculateAliveCells         Local/gol/distributor.go:229-239
 *
 *  2. Run driver (gol_run): the C++ host mirror of
 *       gol.Run(Params, events chan<- Event, keyPresses <-chan rune)
 *                                         Local/gol/gol.go:12-40
 *     with the distributor's event sequence (Local/gol/distributor.go:55-227),
 *     the 2 s AliveCellsCount ticker (:58,154-167), the s/p/q/k key handling
 *     (:107-152, Server/gol/distributor.go:136-164) and the PGM I/O goroutine
 *     (Local/gol/io.go:42-143).
 *
 * Threading: one thread drives an engine (gol_step, loads, halo calls).  The read-only
 * calls (gol_snapshot, gol_get_info, gol_read_board, gol_get_world, gol_read_packed,
 * gol_alive_cells, gol_turn_counts) may come from other threads at any time: during a gol_step the stepping
 * thread serves them at its next launch boundary, on a turn-consistent board; while the
 * step is parked on GOL_CONTROL_PAUSE they run at once (the reference Server's mutex is
 * held only around the per-turn commit: Server/gol/distributor.go:62-75,131-134).  A run
 * driver owns its engines on its own thread; gol_run_* calls are thread-safe.
 *
 * Return codes: GOL_OK or a negative GOL_E* code; gol_step returns GOL_STOPPED (> 0) when
 * the control word stopped it, gol_last_launches a count.  Test failures with rc < 0.
 * GOL_EHIP also reports a corrupt board: a k_step_wg pipeline wait that gave up (a starved
 * workgroup) sets the engine's device error word, and every synchronising call fails until
 * the board is replaced (gol_load*, gol_fill_random).
 */
#ifndef GOL_AMD_H
#define GOL_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------ error codes */
#define GOL_OK          0
#define GOL_EINVAL     -1   /* bad argument (size, null pointer, W < 2, ...)        */
#define GOL_EHIP       -2   /* HIP runtime error (message in gol_last_error)         */
#define GOL_ENOMEM     -3   /* device or host allocation failed                      */
#define GOL_ESTATE     -4   /* call not valid now (e.g. halo exhausted in strip mode)*/
#define GOL_ENODEV     -5   /* no usable HIP device                                  */
#define GOL_EIO        -6   /* PGM file missing / malformed (reference: panic)       */
#define GOL_ECLOSED    -7   /* run driver: event channel closed                      */
#define GOL_ETIMEDOUT  -8   /* run driver: no event within the timeout               */
#define GOL_STOPPED     1   /* gol_step returned early on GOL_CONTROL_STOP (not an error:
                               the turns done so far are in gol_info.turn)            */

/* ----------------------------------------------------------------- engine */
typedef struct gol_ctx gol_ctx;

/* flags */
#define GOL_FLAG_COUNT_EVERY_TURN  0x1u  /* fuse a popcount into every turn (per-turn series) */
#define GOL_FLAG_FORCE_GENERIC     0x2u  /* use the generic stencil even when the fast one applies */
#define GOL_FLAG_NO_AUTOTUNE       0x4u  /* skip the create-time (turns per launch, band) timing
                                            sweep on large boards (results never depend on it) */

typedef struct gol_config {
    int32_t  width;       /* Params.ImageWidth  (>= 2)                                   */
    int32_t  height;      /* Params.ImageHeight of the WHOLE board (>= 1)                */
    int32_t  device;      /* HIP device ordinal; -1 = current device                     */
    int32_t  row_offset;  /* first global row owned by this engine                        */
    int32_t  rows;        /* rows owned; rows == height and halo == 0 => torus engine      */
    int32_t  halo;        /* strip mode: halo depth K in rows (1 <= K <= rows)            */
    uint32_t flags;       /* GOL_FLAG_*                                                   */
    int32_t  band_rows;   /* rows per wavefront band in the stencil; 0 = auto             */
    int32_t  turns_per_launch; /* temporal blocking: turns fused per stencil pass (1 = off;
                                  0 = default); results are identical for every value   */
} gol_config;

typedef struct gol_info {
    int32_t  width, height, row_offset, rows, halo;
    int32_t  words_per_row;     /* ceil(width / 64)                                  */
    int32_t  pitch_words;       /* row stride of the device board in uint64 words    */
    int32_t  buffer_rows;       /* rows + 2 * halo                                   */
    int32_t  fast_path;         /* 1 = the LDS-free DPP stencil (width % 128 == 0, >= 256) */
    int32_t  band_rows;         /* effective band height                              */
    int32_t  halo_valid;        /* strip mode: turns left before the next exchange    */
    int32_t  turns_per_launch;  /* effective temporal-blocking depth                   */
    int32_t  device;
    int64_t  turn;              /* completed turns since load                          */
    int64_t  nonbinary_cells;   /* cells that were neither 0 nor 255 at load           */
    int64_t  launches;          /* stencil kernel launches since load                  */
    int32_t  blocking_limited;  /* 1 = temporal blocking is off because a board buffer is
                                   >= 2 GiB (the multi-turn kernel's 32-bit buffer offsets):
                                   every launch runs one turn                          */
    int32_t  shape_source;      /* where the multi-turn launch shape came from: 0 = defaults
                                   or the caller (gol_config / GOL_* experiments), 1 = the
                                   create-time timing search, 2 = the pinned table of
                                   MI355X shapes for the BASELINE board sizes            */
} gol_info;

/* Whole-board (torus) engine on the current device. */
int  gol_create(int32_t width, int32_t height, uint32_t flags, gol_ctx **out);
/* Whole-board or row-strip engine (see gol_config). */
int  gol_create_ex(const gol_config *cfg, gol_ctx **out);
void gol_destroy(gol_ctx *ctx);
const char *gol_last_error(const gol_ctx *ctx);   /* per engine; "" if none            */
const char *gol_strerror(int code);
/* Build stamp: 16 hex digits of the sha256 of the library's sources (csrc/Makefile SRCS), so
 * a test can tell a library built from other sources than the tree it ships with. */
const char *gol_source_id(void);
int  gol_get_info(gol_ctx *ctx, gol_info *info);

/* Stream: the engine creates its own HIP stream; gol_set_stream makes it enqueue
 * on the caller's stream instead (e.g. torch.cuda.current_stream().cuda_stream).
 * NULL restores the engine's own stream. */
int   gol_set_stream(gol_ctx *ctx, void *hip_stream);
void *gol_get_stream(gol_ctx *ctx);
int   gol_sync(gol_ctx *ctx);

/* Load a board from host bytes (0 = dead, 255 = alive, anything else: the
 * reference's non-binary semantics).  Torus engine: height x width bytes.
 * Strip engine: (rows + 2*halo) x width bytes = global rows
 * row_offset-halo .. row_offset+rows+halo-1 (mod height).  Resets turn to 0. */
int gol_load(gol_ctx *ctx, const uint8_t *bytes);
/* Synthetic board: word (y, j) = splitmix64((seed << 40) + y*words_per_row + j),
 * y the GLOBAL row (oracle/bitref.c uses the same definition).  Resets turn. */
int gol_fill_random(gol_ctx *ctx, uint64_t seed);
/* Load / read packed words for the buffer rows (strip: incl. halos), row stride
 * words_per_row, for checkers that work on packed boards.  Packed words crossing
 * the ABI (here, gol_read_packed and the halo rows of gol_export_halo /
 * gol_import_halo) are always in the standard layout (cell x = bit x % 64 of word
 * x / 64), whatever internal layout the temporal-blocking kernel runs on. */
int gol_load_packed(gol_ctx *ctx, const uint64_t *words);

/* Advance `turns` turns.  Torus engine: any turns >= 0.  Strip engine:
 * turns <= halo_valid (then exchange halos; see gol_export_halo).  Returns GOL_OK, or
 * GOL_STOPPED when the control word (below) said stop between two launches. */
int gol_step(gol_ctx *ctx, int64_t turns);

/* Control word, the engine-level mirror of the reference's CFput flag handshake
 * (Server/gol/distributor.go:54-60,136-164): any thread may set it at any time, without
 * the engine lock.  gol_step reads it before every kernel launch (a launch fuses up to
 * turns_per_launch turns): RUN continues, PAUSE parks gol_step at that launch boundary
 * with the board complete until the word changes, STOP makes gol_step return GOL_STOPPED.
 * Once an engine has seen gol_set_control, gol_step keeps at most 2 launches queued so
 * the word takes effect within 2 launches.  The word stays set until changed. */
#define GOL_CONTROL_RUN    0
#define GOL_CONTROL_PAUSE  1
#define GOL_CONTROL_STOP   2
int gol_set_control(gol_ctx *ctx, int32_t word);

/* The launches the last gol_step / gol_step_overlap call ran (planner introspection for
 * benchmarks and tests; no reference counterpart): up to `cap` entries of turns fused, kernel
 * (the engine's temporal-blocking kernel id; turns == 1: the one-turn stencil, kernel 0) and
 * band rows.  Returns the number of launches (may exceed cap; entries past 4096 are not
 * recorded), or a negative GOL_E* code. */
int gol_last_launches(gol_ctx *ctx, int32_t *turns, int32_t *kernel, int32_t *band, int32_t cap);
/* The same launches' k_step_tile shapes (kernel 15, and 16 = the same tiles resident across
 * blocks of turns): tile width in lanes, the segment code (SEG + 100 * turn order + 1000 *
 * (words per lane - 1)), the waves per workgroup and the turns per block (kernel 15: the
 * launch's turns); 0 for the other kernels.  Returns the launch count like
 * gol_last_launches. */
int gol_last_launch_tiles(gol_ctx *ctx, int32_t *tile_w, int32_t *tile_seg, int32_t *waves,
                          int32_t *block_turns, int32_t cap);
/* The k_step_tile segment codes this library runs (planner introspection for the parity
 * tests: every code the shape search can pick has an oracle test).  Writes min(n, cap) codes,
 * returns n.  Needs no device. */
int gol_tile_codes(int32_t *codes, int32_t cap);
/* The subset of those the persistent tile kernel (K1p: small torus boards, tiles resident
 * across blocks of turns) runs; same convention. */
int gol_tile_persist_codes(int32_t *codes, int32_t cap);
/* The subset the streamed tile kernel (K1q: large torus boards, blocks of turns over
 * (block, tile) items taken in order by resident workgroups) runs; same convention.  Empty
 * in the product library (K1q is a tools-build experiment). */
int gol_tile_stream_codes(int32_t *codes, int32_t cap);
/* Lock-free progress read for a controlling thread: *turn = turns enqueued so far (the
 * board reaches it at the next gol_sync), *parked = 1 while gol_step is parked on PAUSE
 * (the board is then complete at *turn).  Either pointer may be NULL. */
int gol_get_progress(gol_ctx *ctx, int64_t *turn, int32_t *parked);

/* Halo exchange overlapped with compute (strip engines; the zero-copy path of
 * gol_halo_buffers).  gol_stream_wait makes `hip_stream` (the transport's stream) wait for
 * the work queued on the engine so far -- the send rows are final.  The caller then
 * enqueues its sends and receives on that stream and calls gol_step_overlap, which marks
 * the halos fresh and advances `turns` (<= halo) turns: the first launch's interior rows
 * (those whose dependency cone stays inside the owned rows) start on the engine stream at
 * once, the rows next to the halos run on a second engine stream after the work queued on
 * `recv_stream`, and the engine stream joins it before the next launch.  Replaces the
 * reference's blocking fan-out / gather of every strip every turn
 * (Server/gol/distributor.go:118-129). */
int gol_stream_wait(gol_ctx *ctx, void *hip_stream);
int gol_step_overlap(gol_ctx *ctx, int64_t turns, void *recv_stream);

/* Consistent (turn, alive) pair of the current board (owned rows only). */
int gol_snapshot(gol_ctx *ctx, int64_t *turn, int64_t *alive);
/* Per-turn alive counts recorded by GOL_FLAG_COUNT_EVERY_TURN for turns
 * first_turn .. first_turn+n-1 (must be among the last 4096 turns). */
int gol_turn_counts(gol_ctx *ctx, int64_t first_turn, int64_t n, int64_t *out);

/* Owned rows as bytes (rows x width, 0/255; at turn 0 the loaded bytes as-is,
 * matching the reference's Turns = 0 output). */
int gol_read_board(gol_ctx *ctx, uint8_t *out);
/* GetWorld (Server/gol/distributor.go:62-67, the reply ItemW{SWorld, TurnCur}): the owned
 * rows as bytes, as gol_read_board, and the turn that board is at -- one consistent pair,
 * callable from another thread while gol_step runs (served at a launch boundary) or is
 * parked.  The 's' key of a controller that runs the whole game in one gol_step uses it. */
int gol_get_world(gol_ctx *ctx, uint8_t *out, int64_t *turn);
/* Owned rows as packed words (rows x words_per_row). */
int gol_read_packed(gol_ctx *ctx, uint64_t *out);
/* Row-major alive-cell list {x, y} (y = global row) of the owned rows, as
 * int64 pairs; writes min(n, cap) pairs and sets *n to the total. */
int gol_alive_cells(gol_ctx *ctx, int64_t *xy, int64_t cap, int64_t *n);

/* Strip mode halo exchange.  export: copy the first and the last `halo` owned
 * rows (packed, halo x words_per_row uint64 each) to device buffers `top` and
 * `bottom` on `hip_stream` (NULL = engine stream).  import: copy the neighbour
 * rows into this engine's halos (top = the rows above, from rank r-1's bottom;
 * bottom = the rows below, from rank r+1's top) and reset halo_valid to halo. */
int gol_export_halo(gol_ctx *ctx, void *top, void *bottom, void *hip_stream);
int gol_import_halo(gol_ctx *ctx, const void *top, const void *bottom, void *hip_stream);
/* In-process exchange between two strip engines (any devices, peer copies):
 * dst's top halo <- src's last `halo` owned rows (src is dst's upper neighbour). */
int gol_copy_halo_from_upper(gol_ctx *dst, gol_ctx *src);
/* dst's bottom halo <- src's first `halo` owned rows (src is dst's lower neighbour). */
int gol_copy_halo_from_lower(gol_ctx *dst, gol_ctx *src);
/* Mark the halos fresh after all copies into this engine are enqueued. */
int gol_halo_done(gol_ctx *ctx);
/* Zero-copy exchange (the RCCL path: the transport reads and writes the board
 * itself).  Device pointers into the current board buffer: send_top / send_bottom =
 * the first / last `halo` owned rows, recv_top / recv_bottom = the top / bottom halo
 * rows, each halo x words_per_row uint64 with row stride words_per_row.  The rows
 * are in the engine's stepping layout (converted to it here if needed), returned in
 * *layout (0 standard, 1 interleaved): both ends of an exchange must report the
 * same layout -- engines created with the same width, halo and flags do.  The
 * pointers are valid until the next gol_step / gol_load*.  Order the transport after
 * the engine's stream, and the next gol_step after the receives, then call
 * gol_halo_done.  Replaces the per-turn strip+halo RPC copy
 * (reference Server/gol/distributor.go:185-224). */
int gol_halo_buffers(gol_ctx *ctx, void **send_top, void **send_bottom, void **recv_top,
                     void **recv_bottom, int32_t *layout);

/* -------------------------------------------------------------- run driver */
typedef struct gol_params {          /* Local/gol/gol.go:4-9 */
    int64_t turns;
    int32_t threads;                 /* kept for API parity; the GPU result is independent of it */
    int32_t image_width;
    int32_t image_height;
} gol_params;

typedef enum gol_event_type {        /* Local/gol/event.go:9-68 */
    GOL_EV_ALIVE_CELLS_COUNT    = 1,
    GOL_EV_IMAGE_OUTPUT_COMPLETE = 2,
    GOL_EV_STATE_CHANGE         = 3,
    GOL_EV_CELL_FLIPPED         = 4,
    GOL_EV_TURN_COMPLETE        = 5,
    GOL_EV_FINAL_TURN_COMPLETE  = 6
} gol_event_type;

typedef enum gol_state { GOL_PAUSED = 0, GOL_EXECUTING = 1, GOL_QUITTING = 2 } gol_state;

typedef struct gol_event {
    int32_t type;                    /* gol_event_type                                  */
    int32_t new_state;               /* StateChange.NewState                            */
    int64_t completed_turns;         /* every event's GetCompletedTurns()               */
    int64_t cells_count;             /* AliveCellsCount.CellsCount; FinalTurnComplete: len(Alive) */
    int64_t x, y;                    /* CellFlipped.Cell                                */
    char    filename[256];           /* ImageOutputComplete.Filename                    */
} gol_event;

typedef struct gol_run_options {
    const char *image_dir;           /* where {W}x{H}.pgm is read ("images")            */
    const char *out_dir;             /* where {W}x{H}x{T}.pgm is written ("out")        */
    int32_t ngpus;                   /* row strips = engines (the reference's len(SUB)); 0 = 1 */
    const int32_t *devices;          /* exactly ngpus device ordinals (the array is read at
                                        indices 0..ngpus-1); NULL = 0..ngpus-1 (mod count)  */
    int32_t halo;                    /* strip halo depth K; 0 = auto                    */
    int32_t ticker_ms;               /* AliveCellsCount period; 0 = 2000 (distributor.go:58) */
    int32_t event_capacity;          /* bounded event channel; 0 = 1 (unbuffered-like)  */
    int32_t emit_turn_complete;      /* 1 = TurnComplete{t} for every turn (event.go:55-60) */
    int32_t emit_cell_flipped;       /* 1 = CellFlipped for initial cells and each flip  */
    uint32_t engine_flags;           /* GOL_FLAG_* for the engines                      */
    int32_t resume;                  /* 1 = CONT=yes (Local/gol/distributor.go:171-178): continue
                                        from the board and turn the previous run in this
                                        process ended with (the reference Server's retained
                                        world/turn), running Turns - turn more turns; -1 =
                                        read the CONT environment variable                 */
} gol_run_options;

typedef struct gol_run gol_run;

/* Start a run (non-blocking, like gol.Run).  opts may be NULL (defaults). */
int gol_run_start(const gol_params *p, const gol_run_options *opts, gol_run **out);
/* Receive the next event: GOL_OK, GOL_ECLOSED once the channel is closed and
 * drained, GOL_ETIMEDOUT after timeout_ms (< 0 = wait forever). */
int gol_run_next_event(gol_run *r, gol_event *ev, int32_t timeout_ms);
/* FinalTurnComplete.Alive of the most recently received FinalTurnComplete:
 * writes min(n, cap) {x, y} int64 pairs, returns n (or < 0 on error). */
int64_t gol_run_final_alive(gol_run *r, int64_t *xy, int64_t cap);
/* keyPresses <- rune ('s', 'p', 'q', 'k'). */
int gol_run_key(gol_run *r, int32_t rune);
/* Error text of a run that failed (the events channel is closed early).  NULL: why the calling
 * thread's last gol_run_start failed after validating its arguments (e.g. GOL_EHIP: two strip
 * devices that report peer access but refuse to enable it); "" after a successful start. */
const char *gol_run_error(gol_run *r);
/* Join the driver thread and free the run. */
void gol_run_destroy(gol_run *r);

#ifdef __cplusplus
}
#endif
#endif /* GOL_AMD_H */
