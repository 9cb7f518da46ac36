#!/usr/bin/env python3
"""k_step_tile shape sweep (K1t): time `--turns` turns per shape, interleaved rounds, HIP
events on one stream, and check every shape computed the same board.
usage: python tools/tile_sweep.py --size 5120 --shapes 10:160:4:32,10:80:4:16 [--auto]
       shape = tile_w:tile_h:seg:K[:p|:r] ; --auto adds the engine's own autotuned pick;
       :p = K1p resident tiles (GOL_PERSIST=K), :r = K1r ring exchange (GOL_PERSIST=K GOL_RING=1), :g = K1r with a
       grid-wide barrier per block (GOL_RING=2),
       both tools build only (GOL_AMD_LIB=.../libgolamd_tools.so)"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
import torch  # noqa: E402

import gol  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=5120)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--turns", type=int, default=960)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="")
    ap.add_argument("--auto", action="store_true")
    ap.add_argument("--grid", default="",
                    help="tws/segs/Ks/waves, e.g. '10,14/2,3,4,106/16,32/8,16': every combination, "
                         "tile height = the tallest the workgroup of that many waves holds")
    a = ap.parse_args()
    W, H = a.size, a.height or a.size
    if a.grid:
        tws, segs, ks, wvs = ([int(x) for x in part.split(",")] for part in a.grid.split("/"))
        extra = []
        for tw in tws:
            G = 64 // (tw + 2)
            for seg in segs:
                for K in ks:
                    for wv in wvs:
                        th = wv * G * (seg % 100) - 2 * K
                        if th >= 8:
                            extra.append(f"{tw}:{min(th, H)}:{seg}:{K}")
        a.shapes = ",".join([x for x in a.shapes.split(",") if x] + extra)
    stream = torch.cuda.Stream()
    engines = {}
    for sh in [x for x in a.shapes.split(",") if x]:
        parts = sh.split(":")
        tw, th, seg, K = (int(v) for v in parts[:4])
        mode = parts[4] if len(parts) > 4 else ""
        os.environ["GOL_MULTI_VARIANT"] = "15"
        os.environ["GOL_TILE"] = f"{tw},{seg}"
        if mode in ("p", "r", "g"):
            os.environ["GOL_PERSIST"] = str(K)
        if mode in ("r", "g"):
            os.environ["GOL_RING"] = "1" if mode == "r" else "2"
        e = gol.Engine(W, H, device=0, band_rows=th, turns_per_launch=K)
        engines[sh] = e
        os.environ.pop("GOL_PERSIST", None)
        os.environ.pop("GOL_RING", None)
    os.environ.pop("GOL_MULTI_VARIANT", None)
    os.environ.pop("GOL_TILE", None)
    if a.auto:
        e = gol.Engine(W, H, device=0)
        i = e.info()
        engines[f"auto(K={i.turns_per_launch},th={i.band_rows})"] = e
    for e in engines.values():
        e.set_stream(stream.cuda_stream)
        e.fill_random(3)
        e.step(64)
    torch.cuda.synchronize()
    res = {k: [] for k in engines}
    for _ in range(a.rounds):
        for k, e in engines.items():
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            e.step(a.turns)
            e1.record(stream)
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1e3 / a.turns)
    for k, ts in res.items():
        us = statistics.median(ts)
        plan = engines[k].last_launches()
        print(json.dumps({"shape": k, "us_per_turn": round(us, 4), "min_us": round(min(ts), 4),
                          "GCUPS": round(W * H / us / 1e3, 1), "launches": len(plan),
                          "first": plan[0] if plan else None}), flush=True)
    boards = [e.read_packed() for e in engines.values()]
    print(json.dumps({"all_identical": bool(all((b == boards[0]).all() for b in boards[1:]))}))


if __name__ == "__main__":
    main()
