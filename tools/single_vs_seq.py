#!/usr/bin/env python3
"""Why one 20-turn call (the driver's headline) costs more per launch than the same launch in a
back-to-back sequence: 65536^2 with the pinned shape, warmed; then (a) single calls, each
between synchronisations, (b) ten calls back to back timed as one, (c) ten calls back to back
with an event pair around each.  Run it under rocprofv3 --kernel-trace to see each kernel's
own duration beside the event times."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
import torch  # noqa: E402

import gol  # noqa: E402

s = torch.cuda.Stream()
e = gol.Engine(65536, 65536, device=0)
e.set_stream(s.cuda_stream)
e.fill_random(3)
for _ in range(60):
    e.step(20)
torch.cuda.synchronize()


def ev():
    x = torch.cuda.Event(enable_timing=True)
    x.record(s)
    return x


single = []
for _ in range(6):
    e.step(5)
    torch.cuda.synchronize()
    t = time.perf_counter()
    a = ev()
    e.step(20)
    b = ev()
    torch.cuda.synchronize()
    single.append((a.elapsed_time(b) * 1e3, (time.perf_counter() - t) * 1e6))
print("single calls (event us, wall us):", [(round(x), round(y)) for x, y in single], flush=True)

torch.cuda.synchronize()
a = ev()
for _ in range(10):
    e.step(20)
b = ev()
torch.cuda.synchronize()
print("10 back to back: %.1f us per call" % (a.elapsed_time(b) * 1e3 / 10), flush=True)

pairs = []
for _ in range(10):
    pairs.append((ev(), None))
    e.step(20)
    pairs[-1] = (pairs[-1][0], ev())
torch.cuda.synchronize()
per = [x.elapsed_time(y) * 1e3 for x, y in pairs]
print("back to back, each evented:", [round(p) for p in per], "median %.1f" % statistics.median(per),
      flush=True)
e.close()

# (d) fresh random board against an evolved one, alternating, after the same GPU load: both
# run 1200 turns first; "fresh" then refills the board (one fast kernel) -- is the single
# call's cost data-dependent (its instruction stream is not)?
e = gol.Engine(65536, 65536, device=0)
e.set_stream(s.cuda_stream)
res = {"fresh": [], "evolved": []}
for rep in range(4):
    for kind in ("fresh", "evolved"):
        e.fill_random(3 + rep)
        for _ in range(60):
            e.step(20)
        if kind == "fresh":
            e.fill_random(3 + rep)
        e.step(5)
        torch.cuda.synchronize()
        a = ev()
        e.step(20)
        b = ev()
        torch.cuda.synchronize()
        res[kind].append(round(a.elapsed_time(b) * 1e3))
print("fresh vs evolved board, single 20-turn calls (us):", res, flush=True)
e.close()
