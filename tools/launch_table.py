#!/usr/bin/env python3
"""Per-launch time T(k) of the temporal-blocking kernels at depth k (band autotuned per k),
one launch per gol_step call, HIP events on one stream: the fixed cost per launch vs the
per-turn rate, which decide how a short gol_step (e.g. the bench's 20 turns) should split.
usage: python tools/launch_table.py [--size 65536] [--mv 7,9,12] [--k 4,6,8,10,12,16,20]"""
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
    ap.add_argument("--size", type=int, default=65536)
    ap.add_argument("--mv", default="7,9,12")
    ap.add_argument("--k", default="4,6,8,10,12,16,20")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--band", type=int, default=0, help="fixed band rows (0: autotuned per k)")
    a = ap.parse_args()
    W = H = a.size
    stream = torch.cuda.Stream()
    for mv in a.mv.split(","):
        os.environ["GOL_MULTI_VARIANT"] = mv
        for k in [int(x) for x in a.k.split(",")]:
            e = gol.Engine(W, H, device=0, turns_per_launch=k, band_rows=a.band)
            inf = e.info()
            if inf.turns_per_launch != k:
                e.close()
                continue
            e.set_stream(stream.cuda_stream)
            e.fill_random(3)
            e.step(2 * k)
            ts = []
            for _ in range(a.reps):
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                e.step(k)
                e1.record(stream)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            us = statistics.median(ts)
            print(json.dumps({"mv": int(mv), "k": k, "band": e.info().band_rows,
                              "launch_us": round(us, 1), "us_per_turn": round(us / k, 2),
                              "min_us": round(min(ts), 1)}), flush=True)
            e.close()


if __name__ == "__main__":
    main()
