#!/usr/bin/env python3
"""Per-call time of repeated short gol_step calls on one autotuned engine (HIP events), with
the GPU's current shader clock from rocm-smi every few calls: shows whether sustained load
(power / thermal management) slows the same launches down over time.
usage: python tools/clock_drift.py [--size 65536] [--turns 20] [--calls 60] [--idle-ms 0]"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
import torch  # noqa: E402

import gol  # noqa: E402


def sclk():
    try:
        out = subprocess.run(["rocm-smi", "--showclocks"], capture_output=True, text=True,
                             timeout=20).stdout
        return " ".join(l.strip() for l in out.splitlines() if "sclk" in l.lower())[:120]
    except Exception as e:  # noqa: BLE001
        return f"n/a ({e})"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=65536)
    ap.add_argument("--turns", type=int, default=20)
    ap.add_argument("--calls", type=int, default=60)
    ap.add_argument("--idle-ms", type=float, default=0.0)
    a = ap.parse_args()
    stream = torch.cuda.Stream()
    t0 = time.perf_counter()
    e = gol.Engine(a.size, a.size, device=0)
    print(json.dumps({"create_s": round(time.perf_counter() - t0, 2), "sclk": sclk()}), flush=True)
    e.set_stream(stream.cuda_stream)
    e.fill_random(3)
    for i in range(a.calls):
        torch.cuda.synchronize()
        if a.idle_ms:
            time.sleep(a.idle_ms / 1e3)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        e.step(a.turns)
        e1.record(stream)
        e1.synchronize()
        rec = {"call": i, "us": round(e0.elapsed_time(e1) * 1e3, 1),
               "plan": e.last_launches()[:4]}
        if i % 15 == 0:
            rec["sclk"] = sclk()
        print(json.dumps(rec), flush=True)
    e.close()


if __name__ == "__main__":
    main()
