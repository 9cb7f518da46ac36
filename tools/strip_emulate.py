#!/usr/bin/env python3
"""Per-rank cost of the N-GPU strip path, measured on ONE GPU: rank 0's strip
(H/N rows + halo) of the W x H board, stepped exactly as DistStrip steps it, with the
halo exchange replaced by local device copies (export -> import of the strip's own
boundary rows, i.e. the N=1 torus of that strip: same bytes moved on-device, no RCCL).
Prints per-turn time and the implied aggregate GCUPS at N GPUs (an upper bound: the
RCCL transfer itself is not included)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
import torch  # noqa: E402

import gol  # noqa: E402
from gol.distributed import EngineStrip, make_engine_strip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=65536)
    ap.add_argument("--n", default="2,4,8")
    ap.add_argument("--halo", default="64,128,256")
    ap.add_argument("--full", action="store_true", help="also time the N=1 torus engine")
    ap.add_argument("--turns", type=int, default=768)
    ap.add_argument("--tpl", default="0")
    ap.add_argument("--band", default="0")
    ap.add_argument("--rccl", choices=("", "direct", "torch"), default="",
                    help="exchange through RCCL at world size 1 (rank 0 is its own neighbour, "
                         "zero-copy board views): direct RCCL calls on the engine stream, or "
                         "torch batch_isend_irecv; default: local copies")
    ap.add_argument("--overlap", action="store_true",
                    help="--rccl direct: overlapped exchange (gol_step_overlap)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ds_for = None
    if a.rccl:
        import torch.distributed as dist
        from gol.distributed import DistStrip
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29641")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        comm = None
        if a.rccl == "direct":
            from gol.rccl import RcclComm
            comm = RcclComm(0, 1, dev)
        ds_for = lambda es: DistStrip(es, 0, 1, rccl=comm, overlap=a.overlap)  # noqa: E731
    if a.full:
        e = gol.Engine(a.size, a.size, device=0)
        e.fill_random(3)
        s = torch.cuda.Stream()
        e.set_stream(s.cuda_stream)
        e.step(16)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        e.step(a.turns)
        e1.record(s)
        e1.synchronize()
        info = e.info()
        us = e0.elapsed_time(e1) * 1e3 / a.turns
        print(json.dumps({"n": 1, "rows": a.size, "band": info.band_rows,
                          "tpl": info.turns_per_launch, "us_per_turn": round(us, 2),
                          "GCUPS": round(a.size * a.size / us / 1e3, 1)}), flush=True)
        e.close()
    for n in [int(x) for x in a.n.split(",")]:
        for halo, tpl, band in [(int(h), int(t), int(b)) for h in a.halo.split(",")
                                for t in a.tpl.split(",") for b in a.band.split(",")]:
            eng = make_engine_strip(a.size, a.size, 0, n, halo, 0, turns_per_launch=tpl,
                                    band_rows=band)
            es = EngineStrip(eng, dev)
            eng.fill_random(3)
            ds = ds_for(es) if ds_for else None
            with torch.cuda.stream(es.stream):
                def run(turns):
                    if ds is not None:
                        return ds.step(turns)
                    left = turns
                    while left:
                        if es.halo_valid == 0:
                            top, bot = es.export_rows()
                            es.import_rows(bot, top)        # local stand-in for the exchange
                        m = min(left, es.halo_valid)
                        es.step(m)
                        left -= m
                run(2 * halo)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(es.stream)
                run(a.turns)
                e1.record(es.stream)
                e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.turns
            info = eng.info()
            print(json.dumps({"n": n, "halo": info.halo, "rows": info.rows, "band": info.band_rows,
                              "tpl": info.turns_per_launch, "us_per_turn": round(us, 2),
                              "aggregate_GCUPS_upper": round(a.size * a.size / us / 1e3, 1),
                              "exchange": f"rccl-self-{a.rccl}" if ds else "local-copy"}),
                  flush=True)
            eng.close()


if __name__ == "__main__":
    main()
