#!/usr/bin/env python3
"""Run ONE pinned stencil configuration (no create-time autotune) for `--turns` turns, for
profiler passes that must see only the shipped kernel (rocprofv3 --pmc / --kernel-trace).
usage: python tools/kernel_run.py --size 65536 --mv 7 --tpl 10 --band 137 --turns 100
       [--tile TW,SEG] [--persist K | --stream K]  (mv 15 = k_step_tile, band = tile height;
       --persist: the same tiles resident across blocks of K turns, k_tile_persist; --stream:
       blocks of K turns over items taken in order, k_tile_stream)"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=65536)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--mv", type=int, required=True)
    ap.add_argument("--tpl", type=int, required=True)
    ap.add_argument("--band", type=int, required=True)
    ap.add_argument("--tile", default="")
    ap.add_argument("--persist", type=int, default=0,
                    help="k_tile_persist blocks of this many turns (mv 15 only)")
    ap.add_argument("--stream", type=int, default=0,
                    help="k_tile_stream blocks of this many turns (mv 15 only)")
    ap.add_argument("--turns", type=int, default=100)
    a = ap.parse_args()
    os.environ["GOL_MULTI_VARIANT"] = str(a.mv)
    if a.tile:
        os.environ["GOL_TILE"] = a.tile
    if a.persist:
        os.environ["GOL_PERSIST"] = str(a.persist)
    if a.stream:
        os.environ["GOL_STREAM"] = str(a.stream)
    import torch
    import gol
    W, H = a.size, a.height or a.size
    e = gol.Engine(W, H, device=0, band_rows=a.band, turns_per_launch=a.tpl)
    e.fill_random(3)
    # (a k_tile_stream launch runs a whole step: warm up with a launch of the timed size, so
    # every dispatch a profiler pass sees has the same shape)
    e.step(a.turns if a.stream else 2 * a.tpl)
    e.sync()
    t0 = time.perf_counter()
    e.step(a.turns)
    e.sync()
    dt = time.perf_counter() - t0
    print(f"{W}x{H} mv={a.mv} K={a.tpl} band={a.band} tile={a.tile or '-'}: "
          f"{dt * 1e6 / a.turns:.3f} us/turn, {W * H * a.turns / dt / 1e9:.1f} GCUPS, "
          f"launches {len(e.last_launches())}", flush=True)
    e.close()
    del torch


if __name__ == "__main__":
    main()
