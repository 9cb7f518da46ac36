#!/usr/bin/env python3
"""Parity of the ORD 3 tile-pair kernel (k_step_tile_pair, a GOL_TILE_PAIR=1 library via
GOL_AMD_LIB) against the CPU oracle: ragged tiles both ways, odd and even tile counts (the last
pair repeating its first tile), launches of even and odd depth, C2's own shape.
usage: GOL_AMD_LIB=.../libgolamd_pair.so python tools/pair_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import gol  # noqa: E402
from oracle import oracle as O  # noqa: E402

CASES = [  # (width, height, tile_w, tile_h, K, turns, code)
    (4224, 157, 14, 100, 8, 23, 303), (4224, 157, 14, 100, 8, 23, 302),
    (4224, 157, 14, 60, 8, 23, 304), (4224, 157, 10, 80, 8, 23, 306),
    (4224, 157, 14, 64, 16, 31, 308), (896, 90, 14, 30, 10, 31, 303),
    (1024, 64, 14, 64, 8, 35, 303), (5120, 5120, 14, 128, 32, 100, 303),
    (5120, 640, 14, 128, 32, 64, 304), (2048, 300, 30, 40, 12, 37, 303),
]


def main():
    os.environ["GOL_MULTI_VARIANT"] = "15"
    bad = 0
    for w, h, tw, th, K, turns, code in CASES:
        os.environ["GOL_TILE"] = f"{tw},{code}"
        start = O.gen_random(code + w + h, w, h)
        e = gol.Engine(w, h, device=0, band_rows=th, turns_per_launch=K)
        e.load_packed(start)
        e.step(turns)
        got = e.read_packed()
        tiles = {(a, b) for a, b, _ in e.last_launch_tiles()}
        e.close()
        ok = np.array_equal(got, O.bit_run(start, w, turns, ncores=8))
        bad += not ok
        print(f"{w}x{h} tile {tw}x{th} code {code} K={K} turns={turns} tiles={sorted(tiles)}: "
              f"{'OK' if ok else 'MISMATCH'}", flush=True)
    print("ALL_OK" if bad == 0 else f"{bad} MISMATCHES")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
