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


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O
