#!/usr/bin/env python3
"""bench.py's 65536^2 x 20-turn measurement, step by step, repeated: autotuned engine, fill,
W warm-up turns, synchronise, time 20 turns (HIP events + wall), then the same again 5 times
in the same process -- is the first timed call slower than later ones, and why."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
import torch  # noqa: E402

import gol  # noqa: E402

dev = torch.device("cuda", 0)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
stream.synchronize()
_ = stream.cuda_stream
t = time.perf_counter()
eng = gol.Engine(65536, 65536, device=0)
print(f"create {time.perf_counter() - t:.2f} s", flush=True)
eng.set_stream(stream.cuda_stream)
eng.fill_random(3)
for rep in range(6):
    eng.step(5)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    eng.step(20)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    print(f"rep {rep}: events {ev0.elapsed_time(ev1) * 1e3:.0f} us, wall {wall * 1e6:.0f} us, "
          f"plan {eng.last_launches()} tiles {eng.last_launch_tiles()}", flush=True)
    if rep == 2:
        time.sleep(0.05)
eng.close()
