"""bench.py takes `traffic` and the clock under load only from a committed profile summary
whose launch shape equals the launch it timed.  CPU only: reads the
committed profiles/r04_* summaries."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def test_summary_matches_shape_exactly():
    b = _bench()
    d = json.load(open(os.path.join(ROOT, "profiles", "r04_k20_65536_h2_summary.json")))
    got, src = b.pmc_summary(65536, 20, d["shape"])
    # (the newest summary of that exact shape: h2's, or the bench-run pass h of the same shape)
    assert src.startswith(os.path.join("profiles", "r04_k20_65536_h")), src
    assert got["shape"] == d["shape"]
    assert got["traffic_bytes_per_launch"] > 0 and 1.9 < got["clock_ghz"] < 2.5
    other = json.loads(json.dumps(d["shape"]))
    other["band_rows"] += 1
    other["tile"]["height_rows"] += 1
    assert b.pmc_summary(65536, 20, other) == (None, None)
    traffic, src = b.pmc_traffic(65536, 20, d["shape"])
    assert traffic == got["traffic_bytes_per_launch"]


def test_every_r04_summary_has_one_kernel():
    """Each pinned pass measured one instantiation (its FETCH / WRITE kernel sets are one name)."""
    import glob
    files = glob.glob(os.path.join(ROOT, "profiles", "r04_k*_summary.json"))
    assert len(files) >= 4
    for f in files:
        d = json.load(open(f))
        assert len(d["FETCH_SIZE_kernels"]) == 1 and d["FETCH_SIZE_kernels"] == d["WRITE_SIZE_kernels"], f
        assert "shape" in d, f
