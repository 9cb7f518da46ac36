#!/usr/bin/env python3
"""A/B sweep of the fast stencil: kernel variant x band height, interleaved rounds in one
process (all engines resident at once), HIP-event timing on one stream.
usage: python tools/sweep.py [--size 65536] [--turns 100] [--rounds 3] [--variants 0,1,2,3,4]
       [--bands 0,16,32,64,128]"""
import argparse
import json
import math
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
import torch  # noqa: E402

import gol  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=65536)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--turns", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0,1,2,3,4")
    ap.add_argument("--bands", default="0,32,64,128")
    ap.add_argument("--tpl", default="1", help="turns per launch values")
    ap.add_argument("--mw", default="2", help="k_step_multi words per lane values")
    ap.add_argument("--mv", default="1", help="temporal-blocking kernel variants (kMulti*)")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    W, H = a.size, a.height or a.size
    stream = torch.cuda.Stream()
    engines = {}
    # warm-up turns: a multiple of every turns-per-launch, so all engines stay on one turn
    warm = 2 * math.lcm(*[int(x) for x in a.tpl.split(",")])
    for v in [int(x) for x in a.variants.split(",")]:
        for b in [int(x) for x in a.bands.split(",")]:
            for k in [int(x) for x in a.tpl.split(",")]:
                for mw in ([int(x) for x in a.mw.split(",")] if k > 1 else [2]):
                    for mv in ([int(x) for x in a.mv.split(",")] if k > 1 else [1]):
                        os.environ["GOL_STENCIL_VARIANT"] = str(v)
                        os.environ["GOL_MULTI_WORDS"] = str(mw)
                        os.environ["GOL_MULTI_VARIANT"] = str(mv)
                        e = gol.Engine(W, H, device=0, band_rows=b, turns_per_launch=k)
                        e.set_stream(stream.cuda_stream)
                        e.fill_random(3)
                        e.step(warm)
                        engines[(v, e.info().band_rows, k, mw, mv)] = e
    torch.cuda.synchronize()
    res = {k: [] for k in engines}
    for _ in range(a.rounds):
        for k, e in engines.items():
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            e.step(a.turns)       # turns: a multiple of every tpl keeps launches uniform
            e1.record(stream)
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1e3 / a.turns)
    ref = None
    out = []
    for k, ts in res.items():
        us = statistics.median(ts)
        gbs = 0.25 * W * H / (us * 1e-6) / 1e9
        out.append({"variant": k[0], "band": k[1], "tpl": k[2], "mw": k[3], "mv": k[4],
                    "us_per_turn": round(us, 2),
                    "min_us": round(min(ts), 2), "GBs": round(gbs, 1),
                    "GCUPS": round(W * H / us / 1e3, 1)})
        print(json.dumps(out[-1]), flush=True)
    # all engines advanced the same number of turns from the same board: equal boards
    boards = [e.read_packed() for e in engines.values()]
    same = all((b == boards[0]).all() for b in boards[1:])
    print(json.dumps({"all_variants_identical": bool(same)}))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
