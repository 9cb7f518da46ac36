#!/usr/bin/env python3
"""How the driver's 20-turn headline depends on GPU activity right before it (clock ramp),
with the pinned 65536^2 shape (no create-time search): for each pre-load X ms (synchronised
20-turn calls, like a create-time timing pass), after 1 s idle: create the engine, fill, X ms
of calls, refill, the bench's 5-turn warm-up, then the timed 20-turn call (HIP events)."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
os.environ["GOL_PIN_VERIFY_MS"] = "0"     # (the engine's own pre-load is what X stands in for)
import torch  # noqa: E402

import gol  # noqa: E402

s = torch.cuda.Stream()
res = {}
xs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,20,50,100,300").split(",")]
for rep in range(3):
    for X in xs:
        time.sleep(1.0)
        e = gol.Engine(65536, 65536, device=0)
        e.set_stream(s.cuda_stream)
        e.fill_random(3)
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < X:
            e.step(20)
            e.sync()
        e.fill_random(3)
        e.step(5)
        e.sync()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        e.step(20)
        b.record(s)
        b.synchronize()
        res.setdefault(X, []).append(a.elapsed_time(b) * 1e3)
        e.close()
for X in xs:
    v = res[X]
    print(f"pre-load {X:4d} ms: 20-turn call {[round(x) for x in v]} us, median {statistics.median(v):.0f} "
          f"-> {65536 * 65536 * 20 / statistics.median(v) / 1e3:.0f} GCUPS", flush=True)
