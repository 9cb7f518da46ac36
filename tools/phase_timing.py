#!/usr/bin/env python3
"""Host-side time of each phase of bench.py's setup (engine create, stream switch, fill,
warm-up, timed steps): a long host stall leaves the GPU idle, and an idle MI355X lowers its
clock (profiles/r02_clock_pmc_bench20.txt)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "conway-s-gol-distributed_amd"))
import torch  # noqa: E402

import gol  # noqa: E402

stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
T = [("start", time.perf_counter())]
e = gol.Engine(65536, 65536, device=0)
T.append(("create", time.perf_counter()))
sp = stream.cuda_stream
T.append(("cuda_stream", time.perf_counter()))
e.set_stream(sp)
T.append(("set_stream", time.perf_counter()))
e.set_stream(sp)
T.append(("set_stream2", time.perf_counter()))
e.fill_random(3)
T.append(("fill", time.perf_counter()))
e.step(5)
torch.cuda.synchronize()
T.append(("warm5", time.perf_counter()))
for i in range(3):
    e.step(20)
    torch.cuda.synchronize()
    T.append((f"step20_{i}", time.perf_counter()))
for (n, t), (_, p) in zip(T[1:], T):
    print(f"{n:12s} {(t - p) * 1e3:9.2f} ms")
