import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "conway-s-gol-distributed_amd")
for p in (os.path.join(ROOT, "tests"), PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


# The product library ships only the kernels the engine selects; superseded variants,
# timing ablations and depths 17..32 are in the tools build (make tools), which the tests of
# those kernels need: GOL_AMD_LIB=.../build/libgolamd_tools.so python -m pytest ...
TOOLS_LIB = os.environ.get("GOL_AMD_LIB", "").endswith("libgolamd_tools.so")
tools_only = pytest.mark.skipif(not TOOLS_LIB, reason="tools-build kernel (GOL_AMD_LIB=libgolamd_tools.so)")


# The k_step_tile segment codes the product library runs (golk::kTileCodes, reported by
# gol_tile_codes): SEG + 100 * turn order + 1000 * (words per lane - 1).  Each one has its own
# oracle parity test (test_gpu_engine.py::test_tile_code_pinned); test_abi.py checks that the
# library's list is this one, so a code added to the engine without a test fails on the CPU.
TILE_CODES = (2, 3, 4, 6, 8, 12, 16, 24, 32, 40, 48,
              102, 103, 104, 106, 108, 112, 116, 124, 132, 140,
              203, 204, 206, 208, 212, 216, 224, 232, 240,
              403, 404, 406, 408, 412, 416, 424, 432, 440,
              503, 504, 506, 508, 512, 516, 524, 532, 540,
              612, 616, 624,
              1002, 1003, 1004, 1006, 1008,
              1102, 1103, 1104, 1106, 1108,
              1204, 1206, 1208)


# the subset the streamed tile kernel (K1q) runs (gol_tile_stream_codes): tools build only
TILE_STREAM_CODES = (106, 506, 512, 524) if TOOLS_LIB else ()

# the subset the persistent tile kernel (K1p) runs (gol_tile_persist_codes): tools build only
# since round 5 (it never won its autotune; its uncached hand-off is K1q's unproven scheme)
TILE_PERSIST_CODES = (102, 103, 104, 106, 108, 112, 116, 403, 404, 406, 408, 412, 416,
                      2, 3, 4, 6, 8, 503, 504, 506, 508) if TOOLS_LIB else ()

# the codes the ring-exchange tile kernel (K1r, round 6) runs (gol_tile.hip ring_fn): tools
# build only (it measured slower than plain launches, DESIGN.md "K1r")
TILE_RING_CODES = (103, 203, 503, 504, 506, 508, 512, 516, 112, 116) if TOOLS_LIB else ()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O
