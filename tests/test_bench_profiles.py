"""bench.py takes `traffic` and the clock under load only from a committed profile summary
whose launch shape equals the launch it timed.  CPU only: reads the
committed profiles/r04_* / r05_* summaries."""
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
    # (the newest summary of that exact shape: round 5's pass of the pinned shape, or round 4's
    # h / h2 of the same shape)
    assert src.startswith((os.path.join("profiles", "r05_k20_65536_h"),
                           os.path.join("profiles", "r04_k20_65536_h"))), src
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
    files = glob.glob(os.path.join(ROOT, "profiles", "r0[45]_k*_summary.json"))
    assert len(files) >= 4
    for f in files:
        d = json.load(open(f))
        assert len(d["FETCH_SIZE_kernels"]) == 1 and d["FETCH_SIZE_kernels"] == d["WRITE_SIZE_kernels"], f
        assert "shape" in d, f


def test_pinned_shapes_have_profiles():
    """Every BASELINE config the bench measures at N = 1 runs a pinned shape, and profiles/ holds a
    PMC summary of exactly that shape, so `traffic` is never null (round-4 verdict item 2)."""
    b = _bench()
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_gpu_engine as T
    for size, (K, th, tw, code) in T.PINNED_SHAPES.items():
        seg = code % 100
        G = 64 // (tw + 2)
        waves = -(-(-(-(th + 2 * K) // seg)) // G)
        shape = {"kernel": 15, "turns": K, "band_rows": th,
                 "tile": {"code": code, "width_words": tw, "width_lanes": tw, "height_rows": th,
                          "seg_rows": seg, "turn_order": code // 100 % 10, "words_per_lane": 1,
                          "waves_per_workgroup": waves}}
        traffic, src = b.pmc_traffic(size, K, shape)
        assert traffic and traffic > 0, (size, shape)
