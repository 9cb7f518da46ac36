"""Engine: a Python handle on one gol_ctx (include/gol_amd.h).

One Engine = one MI355X holding the whole torus board or one row strip of it —
the GPU-resident replacement for the reference's SubServer
(``API.SubServerDistributor``, reference ``SubServer/distributor.go:48-84``)
plus the Server's per-turn commit and counters
(``Server/gol/distributor.go:62-75,104-134,173-183``).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N


class Engine:
    def __init__(self, width: int, height: int, *, device: int = -1, row_offset: int = 0,
                 rows: int | None = None, halo: int = 0, count_every_turn: bool = False,
                 force_generic: bool = False, band_rows: int = 0, turns_per_launch: int = 0,
                 autotune: bool = True):
        L = N.lib()
        cfg = N.gol_config()
        cfg.width, cfg.height = int(width), int(height)
        cfg.device = int(device)
        cfg.row_offset = int(row_offset)
        cfg.rows = int(height if rows is None else rows)
        cfg.halo = int(halo)
        cfg.flags = ((N.GOL_FLAG_COUNT_EVERY_TURN if count_every_turn else 0) |
                     (N.GOL_FLAG_FORCE_GENERIC if force_generic else 0) |
                     (0 if autotune else N.GOL_FLAG_NO_AUTOTUNE))
        cfg.band_rows = int(band_rows)
        cfg.turns_per_launch = int(turns_per_launch)
        h = ctypes.c_void_p()
        N.check(L.gol_create_ex(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self._L = L
        info = self.info()
        self.width, self.height = info.width, info.height
        self.rows, self.halo = info.rows, info.halo
        self.row_offset = info.row_offset
        self.words_per_row = info.words_per_row
        self.buffer_rows = info.buffer_rows

    # -- lifetime
    def close(self):
        if getattr(self, "_h", None):
            self._L.gol_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    def _c(self, rc):
        return N.check(rc, self._h)

    # -- info / streams
    def info(self) -> N.gol_info:
        i = N.gol_info()
        self._c(self._L.gol_get_info(self._h, ctypes.byref(i)))
        return i

    @property
    def turn(self) -> int:
        return int(self.info().turn)

    @property
    def halo_valid(self) -> int:
        return int(self.info().halo_valid)

    def set_stream(self, stream_ptr: int | None):
        self._c(self._L.gol_set_stream(self._h, ctypes.c_void_p(stream_ptr or 0)))

    def stream(self) -> int:
        return int(self._L.gol_get_stream(self._h) or 0)

    def sync(self):
        self._c(self._L.gol_sync(self._h))

    # -- boards
    def load(self, board: np.ndarray):
        """bytes (buffer_rows, width): whole board, or the haloed strip."""
        b = np.ascontiguousarray(board, dtype=np.uint8)
        if b.shape != (self.buffer_rows, self.width):
            raise ValueError(f"expected {(self.buffer_rows, self.width)}, got {b.shape}")
        self._c(self._L.gol_load(self._h, b.ctypes.data_as(N._u8p)))

    def load_packed(self, words: np.ndarray):
        w = np.ascontiguousarray(words, dtype=np.uint64)
        if w.shape != (self.buffer_rows, self.words_per_row):
            raise ValueError(f"expected {(self.buffer_rows, self.words_per_row)}, got {w.shape}")
        self._c(self._L.gol_load_packed(self._h, w.ctypes.data_as(N._u64p)))

    def fill_random(self, seed: int):
        self._c(self._L.gol_fill_random(self._h, ctypes.c_uint64(int(seed))))

    def step(self, turns: int = 1) -> bool:
        """Advance `turns` turns; False if the control word stopped it early."""
        return self._c(self._L.gol_step(self._h, int(turns))) != N.GOL_STOPPED

    # -- control word (reference CFput handshake, Server/gol/distributor.go:54-60,136-164)
    def set_control(self, word: int):
        """GOL_CONTROL_RUN / _PAUSE / _STOP; safe from any thread while step() runs."""
        self._c(self._L.gol_set_control(self._h, int(word)))

    def progress(self):
        """Lock-free (turns enqueued so far, parked on PAUSE)."""
        t, p = ctypes.c_int64(), ctypes.c_int32()
        self._c(self._L.gol_get_progress(self._h, ctypes.byref(t), ctypes.byref(p)))
        return int(t.value), bool(p.value)

    def last_launches(self, cap: int = 4096):
        """[(turns, kernel id, band rows)] of the launches the last step() ran."""
        arrs = [(ctypes.c_int32 * cap)() for _ in range(3)]
        n = self._c(self._L.gol_last_launches(self._h, *arrs, int(cap)))
        return [(arrs[0][i], arrs[1][i], arrs[2][i]) for i in range(min(n, cap))]

    def last_launch_tiles(self, cap: int = 4096, blocks: bool = False):
        """[(tile width, segment code, waves per workgroup)] of the same launches (k_step_tile
        and its persistent form; zeros for the other kernels); blocks=True adds the turns per
        block as a fourth element."""
        arrs = [(ctypes.c_int32 * cap)() for _ in range(4)]
        n = self._c(self._L.gol_last_launch_tiles(self._h, *arrs, int(cap)))
        k = 4 if blocks else 3
        return [tuple(arrs[j][i] for j in range(k)) for i in range(min(n, cap))]

    # -- overlapped halo exchange (gol_stream_wait / gol_step_overlap)
    def stream_wait(self, stream_ptr: int):
        """Make `stream_ptr` wait for the work queued on the engine so far."""
        self._c(self._L.gol_stream_wait(self._h, ctypes.c_void_p(int(stream_ptr))))

    def step_overlap(self, turns: int, recv_stream_ptr: int):
        """Mark the halos fresh and advance `turns` turns, the first launch's interior
        rows at once and its boundary rows after the work queued on recv_stream_ptr."""
        self._c(self._L.gol_step_overlap(self._h, int(turns),
                                         ctypes.c_void_p(int(recv_stream_ptr))))

    def snapshot(self):
        """(completed turns, alive cells) — the reference's Alivecount pair."""
        t, a = ctypes.c_int64(), ctypes.c_int64()
        self._c(self._L.gol_snapshot(self._h, ctypes.byref(t), ctypes.byref(a)))
        return int(t.value), int(a.value)

    def turn_counts(self, first_turn: int, n: int) -> np.ndarray:
        out = np.zeros(max(int(n), 1), dtype=np.int64)
        self._c(self._L.gol_turn_counts(self._h, int(first_turn), int(n),
                                        out.ctypes.data_as(N._i64p)))
        return out[: int(n)]

    def read_board(self) -> np.ndarray:
        out = np.zeros((self.rows, self.width), dtype=np.uint8)
        self._c(self._L.gol_read_board(self._h, out.ctypes.data_as(N._u8p)))
        return out

    def get_world(self):
        """(board bytes, turn): the reference's GetWorld reply {SWorld, TurnCur}, one
        consistent pair even while another thread's step() runs."""
        out = np.zeros((self.rows, self.width), dtype=np.uint8)
        t = ctypes.c_int64()
        self._c(self._L.gol_get_world(self._h, out.ctypes.data_as(N._u8p), ctypes.byref(t)))
        return out, int(t.value)

    def read_packed(self) -> np.ndarray:
        out = np.zeros((self.rows, self.words_per_row), dtype=np.uint64)
        self._c(self._L.gol_read_packed(self._h, out.ctypes.data_as(N._u64p)))
        return out

    def alive_cells(self) -> np.ndarray:
        """Row-major (n, 2) int64 {x, y} list (Local/gol/distributor.go:229-239)."""
        n = ctypes.c_int64()
        self._c(self._L.gol_alive_cells(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros((max(n.value, 1), 2), dtype=np.int64)
        if n.value:
            self._c(self._L.gol_alive_cells(self._h, out.ctypes.data_as(N._i64p), n.value,
                                            ctypes.byref(n)))
        return out[: n.value]

    # -- strip halo exchange (device pointers)
    def export_halo(self, top_ptr: int, bottom_ptr: int, stream_ptr: int | None = None):
        self._c(self._L.gol_export_halo(self._h, ctypes.c_void_p(top_ptr),
                                        ctypes.c_void_p(bottom_ptr),
                                        ctypes.c_void_p(stream_ptr or 0)))

    def import_halo(self, top_ptr: int, bottom_ptr: int, stream_ptr: int | None = None):
        self._c(self._L.gol_import_halo(self._h, ctypes.c_void_p(top_ptr),
                                        ctypes.c_void_p(bottom_ptr),
                                        ctypes.c_void_p(stream_ptr or 0)))

    def copy_halo_from_upper(self, upper: "Engine"):
        self._c(self._L.gol_copy_halo_from_upper(self._h, upper._h))

    def copy_halo_from_lower(self, lower: "Engine"):
        self._c(self._L.gol_copy_halo_from_lower(self._h, lower._h))

    def halo_done(self):
        self._c(self._L.gol_halo_done(self._h))

    def halo_buffers(self):
        """Zero-copy exchange: device pointers (send_top, send_bottom, recv_top,
        recv_bottom) into the current board, each halo x words_per_row uint64, and the
        rows' layout (0 standard, 1 interleaved).  Valid until the next step."""
        p = [ctypes.c_void_p() for _ in range(4)]
        lay = ctypes.c_int32()
        self._c(self._L.gol_halo_buffers(self._h, *(ctypes.byref(x) for x in p),
                                         ctypes.byref(lay)))
        return tuple(int(x.value or 0) for x in p), int(lay.value)


def strip_split(height: int, n: int):
    """The reference Server's row split (Server/gol/distributor.go:106-116):
    base = H // n rows each, the first H % n strips one more.  Returns [(offset, rows)]."""
    base, slack = divmod(int(height), int(n))
    out, off = [], 0
    for i in range(int(n)):
        r = base + (1 if i < slack else 0)
        out.append((off, r))
        off += r
    return out


def haloed_rows(board: np.ndarray, offset: int, rows: int, halo: int) -> np.ndarray:
    """Global rows offset-halo .. offset+rows+halo-1 (mod H) of a byte board."""
    H = board.shape[0]
    idx = (np.arange(offset - halo, offset + rows + halo) % H)
    return np.ascontiguousarray(board[idx])
