#!/usr/bin/env python3
"""Host-side cost of one halo window as bench.py times it at N > 1 (DistStrip.start_window +
step(halo): the exchange first, then one launch), on ONE GPU: rank 0's strip of an N-way split,
RCCL self-exchange at world size 1.  Prints, per window, the wall time from a synchronised idle
GPU to the end of the window, the GPU time between events recorded around it, and the host time
spent before the first GPU work is enqueued (exchange preparation).
usage: python tools/xchg_overhead.py [--n 8] [--halo 20] [--windows 20]"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gol.distributed import DistStrip, EngineStrip, make_engine_strip  # noqa: E402
from gol.rccl import RcclComm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=65536)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--halo", type=int, default=20)
    ap.add_argument("--windows", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29651")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    comm = RcclComm(0, 1, dev)
    stream = torch.cuda.Stream(dev)
    eng = make_engine_strip(a.size, a.size, 0, a.n, a.halo, 0)
    eng.fill_random(3)
    ds = DistStrip(EngineStrip(eng, dev, stream), 0, 1, rccl=comm)
    ds.exchange()
    ds.step(3 * a.halo)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    e1.record(stream)
    walls, gpus, preps = [], [], []
    for _ in range(a.windows):
        torch.cuda.synchronize()
        ds.start_window()
        e0.record(stream)
        t0 = time.perf_counter()
        ds.exchange()                           # (what step() does first, timed on its own)
        t1 = time.perf_counter()
        ds.step(a.halo)
        e1.record(stream)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        walls.append((t2 - t0) * 1e6)
        preps.append((t1 - t0) * 1e6)
        gpus.append(e0.elapsed_time(e1) * 1e3)
    med = statistics.median
    print(f"n={a.n} halo={a.halo}: window wall {med(walls):.1f} us, GPU {med(gpus):.1f} us, "
          f"exchange host call {med(preps):.1f} us (medians of {a.windows})", flush=True)
    comm.close()
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
