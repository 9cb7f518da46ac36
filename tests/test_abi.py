"""The C-ABI library loads and exports every symbol include/gol_amd.h declares.
No compute calls here (no GPU in the build container)."""
import ctypes
import os
import subprocess
import sys

import pytest


def test_header_symbols_exported():
    from gol import _native as N
    L = N.lib()
    declared = N.header_functions()
    assert len(declared) >= 25
    missing = [n for n in declared if not hasattr(L, n)]
    assert missing == []
    assert set(declared) == set(N.SIGNATURES)
    nm = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = {line.split()[-1] for line in nm.splitlines() if " T " in line}
    assert set(declared) <= exported


def _tree_source_id():
    """csrc/Makefile's SRCS hash, recomputed from the tree."""
    import glob
    import hashlib
    from gol import _native as N
    csrc = os.path.join(os.path.dirname(os.path.dirname(N.LIB_PATH)), "csrc")
    files = sorted(os.path.basename(f) for e in ("hip", "h", "cpp")
                   for f in glob.glob(os.path.join(csrc, "*." + e)))
    files = [os.path.join(csrc, f) for f in files] + [N.HEADER_PATH, os.path.join(csrc, "Makefile")]
    h = hashlib.sha256()
    for f in files:
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def _check_libraries_match_sources():
    from gol import _native as N
    want = _tree_source_id()
    assert N.lib().gol_source_id().decode() == want, "libgolamd.so is stale: rebuild (make -C csrc)"
    build = os.path.dirname(N.LIB_PATH)
    for extra in ("libgolamd_spin0.so",):
        p = os.path.join(build, extra)
        if os.path.exists(p):
            # (in a child: two copies of the library in one process would share nothing, but
            # a child keeps the test's own process clean)
            code = ("import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); "
                    "L.gol_source_id.restype=ctypes.c_char_p; print(L.gol_source_id().decode())")
            got = subprocess.run([sys.executable, "-c", code, p], capture_output=True,
                                 text=True, check=True).stdout.strip()
            assert got == want, f"{extra} is stale"


def test_libraries_match_sources():
    """The shipped libraries were built from the sources in this tree (gol_source_id)."""
    _check_libraries_match_sources()


@pytest.mark.gpu
def test_libraries_match_sources_on_box():
    """Same check on the GPU box: the binaries the GPU tests load match the pushed tree."""
    _check_libraries_match_sources()


def test_tile_codes_are_the_pinned_list():
    """Every k_step_tile instantiation the product can run (gol_tile_codes; needs no device)
    is one that test_gpu_engine.py::test_tile_code_pinned checks against the oracle."""
    import ctypes as C
    from conftest import TILE_CODES
    from gol import _native as N
    L = N.lib()
    n = L.gol_tile_codes(None, 0)
    buf = (C.c_int32 * n)()
    assert L.gol_tile_codes(buf, n) == n
    assert tuple(buf) == TILE_CODES
    from conftest import TILE_PERSIST_CODES
    n = L.gol_tile_persist_codes(None, 0)
    buf = (C.c_int32 * n)()
    assert L.gol_tile_persist_codes(buf, n) == n
    assert tuple(buf) == TILE_PERSIST_CODES and set(buf) <= set(TILE_CODES)
    from conftest import TILE_STREAM_CODES
    n = L.gol_tile_stream_codes(None, 0)
    buf = (C.c_int32 * n)()
    assert L.gol_tile_stream_codes(buf, n) == n
    assert tuple(buf) == TILE_STREAM_CODES and set(buf) <= set(TILE_CODES)


def test_lib_is_gfx950_code_object():
    """The fat binary embeds a gfx950 (MI355X) code object."""
    from gol import _native as N
    data = open(N.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data or b"gfx950" in data


def test_strerror_and_no_device_paths():
    from gol import _native as N
    L = N.lib()
    assert L.gol_strerror(N.GOL_EINVAL) == b"invalid argument"
    assert L.gol_strerror(N.GOL_ENODEV) == b"no HIP device"
    h = ctypes.c_void_p()
    # argument validation happens before device discovery
    assert L.gol_create(1, 16, 0, ctypes.byref(h)) == N.GOL_EINVAL
    cfg = N.gol_config(64, 64, -1, 0, 32, 0, 0, 0)   # strip rows without halo
    assert L.gol_create_ex(ctypes.byref(cfg), ctypes.byref(h)) == N.GOL_EINVAL
    assert L.gol_step(None, 1) == N.GOL_EINVAL
    assert L.gol_last_error(None) == b""
    import torch
    if not torch.cuda.is_available():
        assert L.gol_create(64, 64, 0, ctypes.byref(h)) == N.GOL_ENODEV


def test_peer_access_error_mapping():
    """Round-5 verdict #6: gol_run_start maps each peer-access call between two strips'
    devices through gol_internal_peer_access_status (gol_run.cpp; pure, no HIP call): success
    and hipErrorPeerAccessAlreadyEnabled (704) start the run, anything else fails it with
    GOL_EHIP and a message naming the call, the HIP error and the device pair (returned by
    gol_run_error(NULL))."""
    from gol import _native as N
    L = N.lib()
    f = L.gol_internal_peer_access_status
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                  ctypes.c_char_p, ctypes.c_size_t]
    buf = ctypes.create_string_buffer(256)
    assert f(b"hipDeviceEnablePeerAccess", 0, b"hipSuccess", 0, 1, buf, 256) == N.GOL_OK
    assert buf.value == b""
    assert f(b"hipDeviceEnablePeerAccess", 704, b"hipErrorPeerAccessAlreadyEnabled", 2, 3,
             buf, 256) == N.GOL_OK
    rc = f(b"hipDeviceEnablePeerAccess", 217, b"hipErrorPeerAccessUnsupported", 0, 5, buf, 256)
    assert rc == N.GOL_EHIP
    msg = buf.value.decode()
    assert msg.startswith("hipDeviceEnablePeerAccess(0 -> 5) failed: "
                          "hipErrorPeerAccessUnsupported (217)"), msg
    assert "devices 0 and 5" in msg
    assert f(b"hipDeviceCanAccessPeer", 101, b"hipErrorInvalidDevice", 1, 9, buf, 16) == N.GOL_EHIP
    assert len(buf.value) == 15                          # truncated to the buffer, NUL-ended
    # no failed start on this thread yet: gol_run_error(NULL) is empty
    L.gol_run_error.restype = ctypes.c_char_p
    assert L.gol_run_error(None) == b""


def test_struct_layouts_match_header():
    """ctypes mirrors of the header structs have the C sizes (compiled probe)."""
    from gol import _native as N
    src = r'''
    #include <stdio.h>
    #include "gol_amd.h"
    int main(void){printf("%zu %zu %zu %zu %zu\n", sizeof(gol_config), sizeof(gol_info),
      sizeof(gol_params), sizeof(gol_event), sizeof(gol_run_options)); return 0;}'''
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-I", os.path.dirname(N.HEADER_PATH), c, "-o", exe], check=True)
        sizes = [int(x) for x in subprocess.run([exe], capture_output=True, text=True,
                                                check=True).stdout.split()]
    assert sizes == [ctypes.sizeof(N.gol_config), ctypes.sizeof(N.gol_info),
                     ctypes.sizeof(N.gol_params), ctypes.sizeof(N.gol_event),
                     ctypes.sizeof(N.gol_run_options)]


def test_product_does_not_import_oracle():
    """The product package never imports or links oracle/ (test infrastructure only)."""
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "conway-s-gol-distributed_amd")
    bad = ("import oracle", "from oracle", "liboracle", "oracle.py", "refcpu(", "bit_run(")
    for dp, _, files in os.walk(root):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")) or f == "Makefile":
                text = open(os.path.join(dp, f)).read()
                for b in bad:
                    assert b not in text, (f, b)


def test_pinned_shapes_match_the_tests():
    """The pinned MI355X launch shapes (gol_engine.cpp kKnownShapes) are the ones the GPU
    digests assert (test_gpu_engine.py PINNED_SHAPES / PINNED_STRIP_SHAPES), every code is a
    shipped instantiation, and profile_bench.sh can profile them (read from the source: no
    device needed)."""
    import re
    from conftest import TILE_CODES
    from gol import _native as N
    src = open(os.path.join(os.path.dirname(os.path.dirname(N.LIB_PATH)), "csrc",
                            "gol_engine.cpp")).read()
    body = src[src.index("constexpr KnownShape kKnownShapes[] = {"):]
    body = body[:body.index("};")]
    rows = re.findall(r"\{(\d+), (\d+), \{(\d+), (\d+), (\d+), (\d+), 0\}, [\d.]+f(?:, (\d+), (\d+))?\}",
                      body)
    got = {(int(w), int(r)): (int(k), int(th), int(tw), int(code))
           for w, r, k, th, tw, code, _, _ in rows}
    short = {int(w): (int(sk), int(sth)) for w, r, _, _, _, _, sk, sth in rows if sk}
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import test_gpu_engine as T
    want = {(s, s): v for s, v in T.PINNED_SHAPES.items()}
    want.update(T.PINNED_STRIP_SHAPES)
    assert got == want
    assert short == T.PINNED_SHORT
    assert all(v[3] in TILE_CODES for v in got.values())


def test_tile_turn_header_is_generated():
    """gol_tile_turn.h (K1t ORD 8 / 9: the turn as inline asm with a hand-made VGPR assignment)
    is exactly what gen_tile_turn.py writes, and every v_bitop3 in it reads registers of both
    parities (a v_bitop3 whose three sources share one register-number parity issues at half
    rate on gfx950: profiles/r05_vgpr_bank_probe.log)."""
    import re
    import subprocess
    import sys
    csrc = os.path.join(os.path.dirname(__file__), "..", "conway-s-gol-distributed_amd", "csrc")
    gen = subprocess.run([sys.executable, os.path.join(csrc, "gen_tile_turn.py")],
                         capture_output=True, text=True, check=True).stdout
    with open(os.path.join(csrc, "gol_tile_turn.h")) as f:
        assert f.read() == gen
    n = 0
    for m in re.finditer(r'"v_bitop3_b32 v(\d+), v(\d+), v(\d+), v(\d+)', gen):
        srcs = [int(m.group(i)) for i in (2, 3, 4)]
        assert len({r % 2 for r in srcs}) == 2, m.group(0)
        n += 1
    assert n > 1000
