"""CPU oracle for the per-turn Game of Life board update — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product (``conway-s-gol-distributed_amd/``) never imports it; its HIP path
fails loudly when the native library is missing instead of falling back here.

Three independent restatements of the reference algorithm:

* ``ref_run``       — ``oracle/refcpu.c``: literal byte-per-cell restatement of
  ``calculateNextState`` (reference ``SubServer/distributor.go:119-208``) driven
  by the Server strip split (``Server/gol/distributor.go:104-134,185-224``) and the
  SubServer thread split (``SubServer/distributor.go:48-117``).
* ``bit_run``       — ``oracle/bitref.c``: bit-packed CPU oracle (64 cells/word),
  8-neighbour carry-save count; for large boards.
* ``np_step``       — pure numpy ``np.roll`` restatement for small boards.

All three are pinned against the reference's golden fixtures
(``Local/check/images``, ``Local/check/alive``) by ``tests/test_oracle.py``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    """Compile oracle/build/liboracle.so (gcc + OpenMP)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        i64p = ctypes.POINTER(ctypes.c_longlong)
        L.ref_run.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_longlong,
                              ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.ref_run.restype = ctypes.c_int
        L.ref_alive_count.argtypes = [u8p, ctypes.c_int, ctypes.c_int]
        L.ref_alive_count.restype = ctypes.c_longlong
        L.ref_alive_cells.argtypes = [u8p, ctypes.c_int, ctypes.c_int, i64p, ctypes.c_longlong]
        L.ref_alive_cells.restype = ctypes.c_longlong
        L.bit_splitmix64.argtypes = [ctypes.c_uint64]
        L.bit_splitmix64.restype = ctypes.c_uint64
        L.bit_gen_random.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, u64p]
        L.bit_gen_random.restype = None
        L.bit_pack.argtypes = [u8p, ctypes.c_int, ctypes.c_int, u64p, u64p]
        L.bit_pack.restype = ctypes.c_longlong
        L.bit_unpack.argtypes = [u64p, ctypes.c_int, ctypes.c_int, u8p]
        L.bit_unpack.restype = None
        L.bit_step.argtypes = [u64p, u64p, ctypes.c_int, ctypes.c_int, u64p]
        L.bit_step.restype = None
        L.bit_popcount.argtypes = [u64p, ctypes.c_int, ctypes.c_int]
        L.bit_popcount.restype = ctypes.c_uint64
        L.bit_run.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_longlong, u64p, u64p,
                              ctypes.c_int]
        L.bit_run.restype = ctypes.c_int
        _lib = L
    return _lib


class RefPanic(RuntimeError):
    """The Go reference would panic on these arguments (see refcpu.c ref_run)."""


def _p(a: np.ndarray, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def nwords(width: int) -> int:
    return (width + 63) // 64


# ----------------------------------------------------------------- literal ref
def ref_run(board: np.ndarray, turns: int, nsub: int = 4, threads: int = 8,
            ncores: int = 0) -> np.ndarray:
    """Run the literal restatement; returns a new (H, W) uint8 board."""
    b = np.ascontiguousarray(board, dtype=np.uint8).copy()
    H, W = b.shape
    rc = lib().ref_run(_p(b, ctypes.c_uint8), W, H, int(turns), int(nsub), int(threads),
                       int(ncores))
    if rc == -2:
        raise RefPanic(f"reference would panic: threads={threads} > strip rows + 2 "
                       f"(SubServer/distributor.go:111 slice bounds)")
    if rc != 0:
        raise ValueError("ref_run rejected its arguments")
    return b


def ref_alive_count(board: np.ndarray) -> int:
    b = np.ascontiguousarray(board, dtype=np.uint8)
    H, W = b.shape
    return int(lib().ref_alive_count(_p(b, ctypes.c_uint8), W, H))


def ref_alive_cells(board: np.ndarray) -> np.ndarray:
    """Row-major (n, 2) int64 array of (x, y) where the byte == 255."""
    b = np.ascontiguousarray(board, dtype=np.uint8)
    H, W = b.shape
    n = ref_alive_count(b)
    out = np.zeros((max(n, 1), 2), dtype=np.int64)
    lib().ref_alive_cells(_p(b, ctypes.c_uint8), W, H, _p(out, ctypes.c_longlong), n)
    return out[:n]


# ------------------------------------------------------------- bit-packed ref
def gen_random(seed: int, width: int, height: int) -> np.ndarray:
    """Deterministic Bernoulli(0.5) board, packed (H, nw) uint64 (see bitref.c)."""
    w = np.zeros((height, nwords(width)), dtype=np.uint64)
    lib().bit_gen_random(seed, width, height, _p(w, ctypes.c_uint64))
    return w


def pack(board: np.ndarray):
    """bytes (H, W) -> (packed words, blocked words, number of non-binary cells)."""
    b = np.ascontiguousarray(board, dtype=np.uint8)
    H, W = b.shape
    w = np.zeros((H, nwords(W)), dtype=np.uint64)
    blk = np.zeros_like(w)
    n = lib().bit_pack(_p(b, ctypes.c_uint8), W, H, _p(w, ctypes.c_uint64),
                       _p(blk, ctypes.c_uint64))
    return w, blk, int(n)


def unpack(words: np.ndarray, width: int) -> np.ndarray:
    w = np.ascontiguousarray(words, dtype=np.uint64)
    H = w.shape[0]
    out = np.zeros((H, width), dtype=np.uint8)
    lib().bit_unpack(_p(w, ctypes.c_uint64), width, H, _p(out, ctypes.c_uint8))
    return out


def bit_run(words: np.ndarray, width: int, turns: int, blocked: np.ndarray | None = None,
            counts: bool = False, ncores: int = 0):
    """Run ``turns`` turns on a packed board. Returns the new board (and per-turn counts)."""
    w = np.ascontiguousarray(words, dtype=np.uint64).copy()
    H = w.shape[0]
    c = np.zeros(max(int(turns), 1), dtype=np.uint64) if counts else None
    blk = None if blocked is None else np.ascontiguousarray(blocked, dtype=np.uint64)
    rc = lib().bit_run(_p(w, ctypes.c_uint64), width, H, int(turns),
                       None if blk is None else _p(blk, ctypes.c_uint64),
                       None if c is None else _p(c, ctypes.c_uint64), int(ncores))
    if rc != 0:
        raise ValueError("bit_run rejected its arguments")
    if counts:
        return w, c[: int(turns)]
    return w


def popcount(words: np.ndarray, width: int) -> int:
    w = np.ascontiguousarray(words, dtype=np.uint64)
    return int(lib().bit_popcount(_p(w, ctypes.c_uint64), width, w.shape[0]))


# ------------------------------------------------------------------ numpy ref
def np_step(board: np.ndarray) -> np.ndarray:
    """One turn on a byte board (np.roll torus); non-binary centres -> 0."""
    alive = (board == 255).astype(np.uint8)
    n = np.zeros(board.shape, dtype=np.uint8)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dy or dx:
                n += np.roll(np.roll(alive, dy, axis=0), dx, axis=1)
    out = np.zeros_like(board)
    out[(board == 255) & ((n == 2) | (n == 3))] = 255
    out[(board == 0) & (n == 3)] = 255
    return out


def np_run(board: np.ndarray, turns: int) -> np.ndarray:
    b = np.asarray(board, dtype=np.uint8)
    for _ in range(int(turns)):
        b = np_step(b)
    return b.copy()
