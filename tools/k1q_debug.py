#!/usr/bin/env python3
"""K1q (tools build) on the 8192 x 2048 board of test_tile_stream_pinned[4-*], repeated: where
do the wrong words sit (tile row / column, block-edge rows)?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import gol  # noqa: E402
from oracle import oracle as O  # noqa: E402

w, h, tw, th, K, turns = 8192, 2048, 30, 128, 20, 62
for code in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "524,512,506,106").split(",")]:
    os.environ["GOL_MULTI_VARIANT"] = "15"
    os.environ["GOL_TILE"] = f"{tw},{code}"
    os.environ["GOL_STREAM"] = str(K)
    start = O.gen_random(code * 5 + 4, w, h)
    want = O.bit_run(start, w, turns)
    for rep in range(4):
        e = gol.Engine(w, h, device=0, band_rows=th, turns_per_launch=K)
        e.load_packed(start)
        e.step(turns)
        got = e.read_packed()
        e.close()
        bad = np.argwhere(got != want)
        if len(bad) == 0:
            print(code, rep, "ok", flush=True)
            continue
        rows = sorted(set(int(r) for r, _ in bad))
        cols = sorted(set(int(c) for _, c in bad))
        print(code, rep, "bad words", len(bad), "rows", rows[:12], "..." if len(rows) > 12 else "",
              "tile rows", sorted(set(r // th for r in rows)), "cols", cols[:16],
              "tile cols", sorted(set(c // tw for c in cols)), flush=True)
