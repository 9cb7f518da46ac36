"""ctypes binding of the C ABI in include/gol_amd.h (libgolamd.so, built for gfx950).

There is no fallback: if the native library is missing this module raises, and
every engine call goes to the HIP kernels.  The library is built in-tree by
``__graft_entry__.build()`` (``make -C conway-s-gol-distributed_amd/csrc``).
"""
from __future__ import annotations

import ctypes
import os
import re

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.environ.get("GOL_AMD_LIB", os.path.join(PKG_ROOT, "build", "libgolamd.so"))
HEADER_PATH = os.path.join(REPO_ROOT, "include", "gol_amd.h")

GOL_OK = 0
GOL_EINVAL = -1
GOL_EHIP = -2
GOL_ENOMEM = -3
GOL_ESTATE = -4
GOL_ENODEV = -5
GOL_EIO = -6
GOL_ECLOSED = -7
GOL_ETIMEDOUT = -8
GOL_STOPPED = 1

GOL_CONTROL_RUN = 0
GOL_CONTROL_PAUSE = 1
GOL_CONTROL_STOP = 2

GOL_FLAG_COUNT_EVERY_TURN = 0x1
GOL_FLAG_FORCE_GENERIC = 0x2
GOL_FLAG_NO_AUTOTUNE = 0x4

GOL_EV_ALIVE_CELLS_COUNT = 1
GOL_EV_IMAGE_OUTPUT_COMPLETE = 2
GOL_EV_STATE_CHANGE = 3
GOL_EV_CELL_FLIPPED = 4
GOL_EV_TURN_COMPLETE = 5
GOL_EV_FINAL_TURN_COMPLETE = 6


class GolError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"gol error {code}: {msg}")


class gol_config(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("device", ctypes.c_int32), ("row_offset", ctypes.c_int32),
                ("rows", ctypes.c_int32), ("halo", ctypes.c_int32),
                ("flags", ctypes.c_uint32), ("band_rows", ctypes.c_int32),
                ("turns_per_launch", ctypes.c_int32)]


class gol_info(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("row_offset", ctypes.c_int32), ("rows", ctypes.c_int32),
                ("halo", ctypes.c_int32), ("words_per_row", ctypes.c_int32),
                ("pitch_words", ctypes.c_int32), ("buffer_rows", ctypes.c_int32),
                ("fast_path", ctypes.c_int32), ("band_rows", ctypes.c_int32),
                ("halo_valid", ctypes.c_int32), ("turns_per_launch", ctypes.c_int32),
                ("device", ctypes.c_int32),
                ("turn", ctypes.c_int64), ("nonbinary_cells", ctypes.c_int64),
                ("launches", ctypes.c_int64), ("blocking_limited", ctypes.c_int32),
                ("shape_source", ctypes.c_int32)]


class gol_params(ctypes.Structure):
    _fields_ = [("turns", ctypes.c_int64), ("threads", ctypes.c_int32),
                ("image_width", ctypes.c_int32), ("image_height", ctypes.c_int32)]


class gol_event(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("new_state", ctypes.c_int32),
                ("completed_turns", ctypes.c_int64), ("cells_count", ctypes.c_int64),
                ("x", ctypes.c_int64), ("y", ctypes.c_int64),
                ("filename", ctypes.c_char * 256)]


class gol_run_options(ctypes.Structure):
    _fields_ = [("image_dir", ctypes.c_char_p), ("out_dir", ctypes.c_char_p),
                ("ngpus", ctypes.c_int32), ("devices", ctypes.POINTER(ctypes.c_int32)),
                ("halo", ctypes.c_int32), ("ticker_ms", ctypes.c_int32),
                ("event_capacity", ctypes.c_int32), ("emit_turn_complete", ctypes.c_int32),
                ("emit_cell_flipped", ctypes.c_int32), ("engine_flags", ctypes.c_uint32),
                ("resume", ctypes.c_int32)]


_lib = None

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i64p = ctypes.POINTER(ctypes.c_int64)

# name -> (restype, argtypes); must cover every function declared in the header
SIGNATURES = {
    "gol_create": (_i32, [_i32, _i32, ctypes.c_uint32, ctypes.POINTER(_vp)]),
    "gol_create_ex": (_i32, [ctypes.POINTER(gol_config), ctypes.POINTER(_vp)]),
    "gol_destroy": (None, [_vp]),
    "gol_last_error": (ctypes.c_char_p, [_vp]),
    "gol_strerror": (ctypes.c_char_p, [_i32]),
    "gol_source_id": (ctypes.c_char_p, []),
    "gol_get_info": (_i32, [_vp, ctypes.POINTER(gol_info)]),
    "gol_set_stream": (_i32, [_vp, _vp]),
    "gol_get_stream": (_vp, [_vp]),
    "gol_sync": (_i32, [_vp]),
    "gol_load": (_i32, [_vp, _u8p]),
    "gol_fill_random": (_i32, [_vp, ctypes.c_uint64]),
    "gol_load_packed": (_i32, [_vp, _u64p]),
    "gol_step": (_i32, [_vp, _i64]),
    "gol_set_control": (_i32, [_vp, _i32]),
    "gol_get_progress": (_i32, [_vp, _i64p, ctypes.POINTER(ctypes.c_int32)]),
    "gol_last_launches": (_i32, [_vp, ctypes.POINTER(ctypes.c_int32),
                                 ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                 ctypes.c_int32]),
    "gol_last_launch_tiles": (_i32, [_vp, ctypes.POINTER(ctypes.c_int32),
                                     ctypes.POINTER(ctypes.c_int32),
                                     ctypes.POINTER(ctypes.c_int32),
                                     ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]),
    "gol_tile_codes": (_i32, [ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]),
    "gol_tile_persist_codes": (_i32, [ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]),
    "gol_tile_stream_codes": (_i32, [ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]),
    "gol_stream_wait": (_i32, [_vp, _vp]),
    "gol_step_overlap": (_i32, [_vp, _i64, _vp]),
    "gol_snapshot": (_i32, [_vp, _i64p, _i64p]),
    "gol_turn_counts": (_i32, [_vp, _i64, _i64, _i64p]),
    "gol_read_board": (_i32, [_vp, _u8p]),
    "gol_get_world": (_i32, [_vp, _u8p, _i64p]),
    "gol_read_packed": (_i32, [_vp, _u64p]),
    "gol_alive_cells": (_i32, [_vp, _i64p, _i64, _i64p]),
    "gol_export_halo": (_i32, [_vp, _vp, _vp, _vp]),
    "gol_import_halo": (_i32, [_vp, _vp, _vp, _vp]),
    "gol_copy_halo_from_upper": (_i32, [_vp, _vp]),
    "gol_copy_halo_from_lower": (_i32, [_vp, _vp]),
    "gol_halo_done": (_i32, [_vp]),
    "gol_halo_buffers": (_i32, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                ctypes.POINTER(ctypes.c_int32)]),
    "gol_run_start": (_i32, [ctypes.POINTER(gol_params), ctypes.POINTER(gol_run_options),
                             ctypes.POINTER(_vp)]),
    "gol_run_next_event": (_i32, [_vp, ctypes.POINTER(gol_event), _i32]),
    "gol_run_final_alive": (_i64, [_vp, _i64p, _i64]),
    "gol_run_key": (_i32, [_vp, _i32]),
    "gol_run_error": (ctypes.c_char_p, [_vp]),
    "gol_run_destroy": (None, [_vp]),
}


def header_functions(path: str = HEADER_PATH) -> list:
    """Function names declared in include/gol_amd.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(gol_[a-z_]+)\s*\(", text)
    return sorted(set(names))


def lib() -> ctypes.CDLL:
    """Load libgolamd.so (raises if it has not been built: no CPU fallback)."""
    global _lib
    if _lib is None:
        # torch (when present) ships its own libamdhip64 whose NEEDED name differs from
        # ours (libamdhip64.so vs .so.7); loading ours first would put two HIP runtimes
        # in the process and torch would see no GPU.  Loading torch first makes our
        # libamdhip64.so.7 dependency resolve to torch's already-loaded runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"native engine {LIB_PATH} is missing; build it with "
                f"`python -c 'import __graft_entry__ as g; g.build()'` "
                f"(make -C conway-s-gol-distributed_amd/csrc)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, ctx=None) -> int:
    if rc < 0:
        L = lib()
        msg = L.gol_strerror(rc).decode()
        if ctx:
            detail = L.gol_last_error(ctx)
            if detail:
                msg += ": " + detail.decode()
        raise GolError(rc, msg)
    return rc
