#!/usr/bin/env python3
"""Prototype: one board on ONE GPU as n row sub-strips (K-row halos, device copies every
`halo` turns), each sub-strip engine on its own HIP stream, with the sub-strips' launches
offset in phase (sub-strip i starts its first window with a shorter step), so one
sub-strip's pipeline fill / drain overlaps another's steady state.  Prints us per turn and
checks the board against a single torus engine.
usage: python tools/substrip_proto.py [--size 16384] [--n 2] [--halo 128] [--windows 8]
                                      [--offset 8]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gol  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--halo", type=int, default=128)
    ap.add_argument("--windows", type=int, default=8)
    ap.add_argument("--offset", type=int, default=8, help="turns of sub-strip i's first step "
                    "= i * offset (0: all in phase)")
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    W = H = a.size
    parts = gol.strip_split(H, a.n)
    engs = [gol.Engine(W, H, device=0, row_offset=o, rows=r, halo=a.halo) for o, r in parts]
    streams = [torch.cuda.Stream() for _ in engs]
    for e, s in zip(engs, streams):
        _ = s.cuda_stream
        e.set_stream(s.cuda_stream)
        e.fill_random(3)
    torch.cuda.synchronize()

    def exchange():
        n = len(engs)
        for i, e in enumerate(engs):
            e.copy_halo_from_upper(engs[(i - 1) % n])
            e.copy_halo_from_lower(engs[(i + 1) % n])
        for e in engs:
            e.halo_done()

    def window(first):
        for i, e in enumerate(engs):
            off = (i * a.offset) % a.halo if first else 0
            if off:
                e.step(off)
                e.step(a.halo - off)
            else:
                e.step(a.halo)
        exchange()

    window(True)                      # warm-up window (also sets the phase offsets)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for w in range(a.windows):
        window(False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    turns = a.windows * a.halo
    out = {"size": W, "n": a.n, "halo": a.halo, "offset": a.offset,
           "us_per_turn": round(dt * 1e6 / turns, 3),
           "GCUPS": round(W * H * turns / dt / 1e9, 1),
           "plans": [e.last_launches()[:3] for e in engs]}
    if a.check:
        ref = gol.Engine(W, H, device=0)
        ref.fill_random(3)
        ref.step((a.windows + 1) * a.halo)
        want = ref.read_packed()
        got = np.concatenate([e.read_packed() for e in engs])
        out["matches_torus_engine"] = bool(np.array_equal(got, want))
        ref.close()
    print(json.dumps(out), flush=True)
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
