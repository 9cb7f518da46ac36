#!/usr/bin/env python3
"""How a 20-turn K1t launch's time depends on what the GPU did before (clock ramp).
Pinned 65536^2 shape (no autotune); HIP events around each gol_step on one stream.
  A: 40 calls of 20 turns back to back (after 1 s idle)
  B: 20 calls, 50 ms host sleep before each
  C: 20 calls, each after 20 ms of back-to-back turns (busy GPU right up to the call)
  D: one call of 2000 turns, then 20 calls back to back
  E: 10 times: ~60 synchronised short calls (2..32 turns, the autotune's sequence timing),
     then one 20-turn call
  F: as E, then 4 ms of back-to-back turns, then the 20-turn call
  G: as E, then a synchronised 5-turn call (bench.py's warm-up), then the 20-turn call"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
import torch  # noqa: E402

import gol  # noqa: E402

tw, th, code, K = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "30:336:524:20").split(":"))
os.environ["GOL_MULTI_VARIANT"] = "15"
os.environ["GOL_TILE"] = f"{tw},{code}"
s = torch.cuda.Stream()
e = gol.Engine(65536, 65536, device=0, band_rows=th, turns_per_launch=K)
e.set_stream(s.cuda_stream)
e.fill_random(3)
e.step(40)
e.sync()


def call(n=20):
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record(s)
    e.step(n)
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) * 1e3


def show(tag, xs):
    print(f"{tag}: n={len(xs)} first5={[round(x) for x in xs[:5]]} median={statistics.median(xs):.0f} "
          f"min={min(xs):.0f} max={max(xs):.0f} us", flush=True)


time.sleep(1.0)


def a_to_d():
    show("A back-to-back after 1 s idle", [call() for _ in range(40)])
    xs = []
    for _ in range(20):
        time.sleep(0.05)
        xs.append(call())
    show("B 50 ms idle before each", xs)
    xs = []
    for _ in range(20):
        e.step(560)                      # ~20 ms of turns, not waited for
        xs.append(call())
    show("C busy right up to each call", xs)
    long = call(2000)
    show("D long call (per 20 turns)", [long / 100])
    show("D then back-to-back", [call() for _ in range(20)])


if not os.environ.get("ONLY_EF"):
    a_to_d()


def short_calls():
    for r in range(2, 33, 1):
        e.step(r)
        e.sync()
        e.step(r)
        e.sync()


xs = []
for _ in range(10):
    short_calls()
    xs.append(call())
show("E after synchronised short calls", xs)
xs = []
for _ in range(10):
    short_calls()
    e.step(120)
    xs.append(call())
show("F after short calls + 4 ms busy", xs)
xs = []
for _ in range(10):
    short_calls()
    e.step(5)                        # the bench: 5 warm-up turns, synchronise, time 20
    e.sync()
    xs.append(call())
show("G after short calls + the bench's 5-turn warm-up", xs)
e.close()
