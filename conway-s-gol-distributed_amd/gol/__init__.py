"""gol — host-side mirror of the reference's ``gol`` package on the MI355X engine.

Same surface as the reference (joyce-leesw/Conway-s-GOL-Distributed, ``Local/gol``):

* ``Params{Turns, Threads, ImageWidth, ImageHeight}``      Local/gol/gol.go:4-9
* ``Run(p, events, keyPresses)`` — non-blocking; events is a channel closed at
  the end of the run                                       Local/gol/gol.go:12-40
* events ``AliveCellsCount``, ``ImageOutputComplete``, ``StateChange``,
  ``CellFlipped``, ``TurnComplete``, ``FinalTurnComplete`` and ``State``
                                                            Local/gol/event.go:9-131
* ``Cell{X, Y}``                                            Local/util/cell.go:10-12

Go channels are mirrored by ``Channel`` (bounded, closable, iterable).  The turn
loop, the 2 s ticker, the key handling and the PGM I/O run in the native C++
driver (``csrc/gol_run.cpp``) over the HIP engine; this module only pumps its
events into the caller's channel.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import enum
import queue
import threading
from dataclasses import dataclass, field
from typing import Any, NamedTuple, Optional

import numpy as np

from . import _native as N
from .engine import Engine, haloed_rows, strip_split  # noqa: F401


# ------------------------------------------------------------------ params
@dataclass
class Params:
    Turns: int = 0
    Threads: int = 8
    ImageWidth: int = 512
    ImageHeight: int = 512


class Cell(NamedTuple):
    X: int
    Y: int


class State(enum.IntEnum):
    Paused = 0
    Executing = 1
    Quitting = 2

    def __str__(self):
        return self.name


# ------------------------------------------------------------------ events
class Event:
    CompletedTurns: int

    def GetCompletedTurns(self) -> int:
        return self.CompletedTurns


@dataclass
class AliveCellsCount(Event):
    CompletedTurns: int
    CellsCount: int

    def __str__(self):
        return f"Alive Cells {self.CellsCount}"


@dataclass
class ImageOutputComplete(Event):
    CompletedTurns: int
    Filename: str

    def __str__(self):
        return f"File {self.Filename} output complete"


@dataclass
class StateChange(Event):
    CompletedTurns: int
    NewState: State

    def __str__(self):
        return str(self.NewState)


@dataclass
class CellFlipped(Event):
    CompletedTurns: int
    Cell: Cell

    def __str__(self):
        return ""


@dataclass
class TurnComplete(Event):
    CompletedTurns: int

    def __str__(self):
        return ""


@dataclass
class FinalTurnComplete(Event):
    CompletedTurns: int
    Alive: Any = field(repr=False)        # list[Cell] (or (n, 2) int64 array)

    def __str__(self):
        return ""


# ----------------------------------------------------------------- channel
class RunError(RuntimeError):
    """A run ended on an error (the reference panics: util.Check / log.Fatal,
    Local/util/check.go:3-7, Server/gol/distributor.go:89-92)."""


class Channel:
    """A Go-like channel: bounded FIFO (capacity 0 behaves as capacity 1),
    ``close()``, ``recv() -> (value, ok)`` and iteration until closed+drained.
    ``close(error)`` closes it with an error: once the queued values are drained,
    ``recv`` and iteration raise ``RunError`` instead of reporting a clean close."""

    _CLOSED = object()

    def __init__(self, capacity: int = 0):
        self._q: queue.Queue = queue.Queue(maxsize=max(int(capacity), 1))
        self._closed = threading.Event()
        self.error: Optional[str] = None

    def send(self, v):
        if self._closed.is_set():
            raise RuntimeError("send on closed channel")
        self._q.put(v)

    def close(self, error: Optional[str] = None):
        if not self._closed.is_set():
            self.error = error
            self._closed.set()
            self._q.put(Channel._CLOSED)

    def recv(self, timeout: Optional[float] = None):
        v = self._q.get(timeout=timeout)
        if v is Channel._CLOSED:
            self._q.put(Channel._CLOSED)      # stay closed for other receivers
            if self.error:
                raise RunError(self.error)
            return None, False
        return v, True

    def __iter__(self):
        while True:
            v, ok = self.recv()
            if not ok:
                return
            yield v


# --------------------------------------------------------------------- run
class RunHandle:
    """Returned by Run(): the native run plus its pump threads."""

    def __init__(self, h, L):
        self._h, self._L = h, L
        self._lock = threading.Lock()
        self._live = True
        self.error: Optional[str] = None
        self.threads: list = []

    def key(self, rune) -> bool:
        """keyPresses <- rune; False once the run has finished."""
        with self._lock:
            if not self._live:
                return False
            N.check(self._L.gol_run_key(self._h, ord(rune) if isinstance(rune, str) else int(rune)))
            return True

    def _destroy(self):
        with self._lock:
            if self._live:
                self._live = False
                self._L.gol_run_destroy(self._h)

    def wait(self, timeout: Optional[float] = None):
        """Join the pump threads; raises RunError if the run failed."""
        for t in self.threads:
            t.join(timeout)
        if self.error:
            raise RunError(self.error)


def _to_event(ev: N.gol_event, h, L, alive_as_array: bool):
    t = int(ev.completed_turns)
    if ev.type == N.GOL_EV_ALIVE_CELLS_COUNT:
        return AliveCellsCount(t, int(ev.cells_count))
    if ev.type == N.GOL_EV_IMAGE_OUTPUT_COMPLETE:
        return ImageOutputComplete(t, ev.filename.decode())
    if ev.type == N.GOL_EV_STATE_CHANGE:
        return StateChange(t, State(int(ev.new_state)))
    if ev.type == N.GOL_EV_CELL_FLIPPED:
        return CellFlipped(t, Cell(int(ev.x), int(ev.y)))
    if ev.type == N.GOL_EV_TURN_COMPLETE:
        return TurnComplete(t)
    if ev.type == N.GOL_EV_FINAL_TURN_COMPLETE:
        n = int(ev.cells_count)
        xy = np.zeros((max(n, 1), 2), dtype=np.int64)
        got = L.gol_run_final_alive(h, xy.ctypes.data_as(N._i64p), n)
        N.check(int(got))
        xy = xy[:n]
        alive = xy if alive_as_array else [Cell(int(x), int(y)) for x, y in xy]
        return FinalTurnComplete(t, alive)
    raise ValueError(f"unknown event type {ev.type}")


def Run(p: Params, events: Channel, keyPresses: Optional[Channel] = None, *,
        image_dir: str = "images", out_dir: str = "out", ngpus: int = 1,
        devices: Optional[list] = None, halo: int = 0, ticker_ms: int = 2000,
        event_capacity: int = 1, emit_turn_complete: bool = True,
        emit_cell_flipped: bool = False, count_every_turn: bool = False,
        alive_as_array: bool = False, resume: Optional[bool] = None) -> RunHandle:
    """Start a run and return immediately (reference ``gol.Run``, Local/gol/gol.go:12-40).

    Events arrive on ``events`` in the reference's order
    (Local/gol/distributor.go:180-226): StateChange{0, Executing},
    [TurnComplete{t} per turn], AliveCellsCount every ``ticker_ms``,
    FinalTurnComplete, StateChange{T, Quitting}, ImageOutputComplete{T, "WxHxT"},
    then the channel is closed.  ``ngpus`` = number of row strips (the
    reference's ``len(SUB)``), one engine each.  ``resume`` = the reference's
    ``CONT=yes`` (None: read the CONT environment variable).
    """
    if devices is not None and len(devices) != int(ngpus):
        # gol_run_start reads devices[0..ngpus-1]
        raise ValueError(f"devices lists {len(devices)} ordinals for ngpus={ngpus}")
    L = N.lib()
    prm = N.gol_params(int(p.Turns), int(p.Threads), int(p.ImageWidth), int(p.ImageHeight))
    opts = N.gol_run_options()
    opts.image_dir = image_dir.encode()
    opts.out_dir = out_dir.encode()
    opts.ngpus = int(ngpus)
    dev_arr = None
    if devices is not None:
        dev_arr = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
        opts.devices = ctypes.cast(dev_arr, ctypes.POINTER(ctypes.c_int32))
    opts.halo = int(halo)
    opts.ticker_ms = int(ticker_ms)
    opts.event_capacity = int(event_capacity)
    opts.emit_turn_complete = 1 if emit_turn_complete else 0
    opts.emit_cell_flipped = 1 if emit_cell_flipped else 0
    opts.engine_flags = N.GOL_FLAG_COUNT_EVERY_TURN if count_every_turn else 0
    opts.resume = -1 if resume is None else (1 if resume else 0)
    h = ctypes.c_void_p()
    rc = L.gol_run_start(ctypes.byref(prm), ctypes.byref(opts), ctypes.byref(h))
    if rc < 0:
        detail = L.gol_run_error(None)          # the start's own reason (e.g. peer access)
        msg = L.gol_strerror(rc).decode()
        raise N.GolError(rc, msg + (": " + detail.decode() if detail else ""))
    handle = RunHandle(h, L)
    done = threading.Event()

    def pump():
        ev = N.gol_event()
        try:
            while True:
                rc = L.gol_run_next_event(h, ctypes.byref(ev), -1)
                if rc == N.GOL_ECLOSED:
                    break
                N.check(rc)
                events.send(_to_event(ev, h, L, alive_as_array))
        except Exception as e:              # a native error code while pumping
            handle.error = str(e)
        finally:
            err = L.gol_run_error(h)
            if err and not handle.error:
                handle.error = err.decode()
            done.set()
            handle._destroy()
            events.close(handle.error)

    def keys():
        while not done.is_set():
            try:
                k, ok = keyPresses.recv(timeout=0.05)
            except queue.Empty:
                continue
            if not ok:
                return
            if not handle.key(k):
                return

    t = threading.Thread(target=pump, name="gol-events", daemon=True)
    t.start()
    handle.threads.append(t)
    if keyPresses is not None:
        tk = threading.Thread(target=keys, name="gol-keys", daemon=True)
        tk.start()
        handle.threads.append(tk)
    handle._dev_arr = dev_arr
    return handle


__all__ = [
    "Params", "Run", "RunHandle", "RunError", "Channel", "Cell", "State", "Event", "AliveCellsCount",
    "ImageOutputComplete", "StateChange", "CellFlipped", "TurnComplete", "FinalTurnComplete",
    "Engine", "strip_split", "haloed_rows",
]
