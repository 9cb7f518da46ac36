#!/usr/bin/env python3
"""Issue efficiency of the temporal-blocking kernel vs resident waves per SIMD.

A 63488-wide board has exactly 16 wavefront tiles per row band (62 words stored per
tile), so with 256-row bands a launch has 16 x 64 x W = 1024 x W equal wavefronts: W per
SIMD on the 1024 SIMDs, one round, no tail.  Per launch the VALU issues
  waves x stage-steps x 52 cycles   (18 full-rate + 4 half-rate instructions per stage-row,
                                     bench.py VALU model)
so efficiency = that / (1024 SIMDs x launch time x clock), printed at the 2.4 GHz peak.
usage: python tools/occupancy_probe.py [--waves 1,2,3,4] [--band 256] [--tpl 8]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
import torch  # noqa: E402

import gol  # noqa: E402


def stage_steps(band, K, U=9):
    nr = max(band, K) + 2 * K
    s0 = 3 * K - 3
    nr = s0 + -(-(nr - s0) // U) * U
    return K * nr - K * (K - 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--waves", default="1,2,3,4")
    ap.add_argument("--band", type=int, default=256)
    ap.add_argument("--tpl", type=int, default=8)
    ap.add_argument("--launches", type=int, default=40)
    a = ap.parse_args()
    W = 16 * 62 * 64
    s = torch.cuda.Stream()
    for w in [int(x) for x in a.waves.split(",")]:
        H = 64 * w * a.band
        e = gol.Engine(W, H, device=0, band_rows=a.band, turns_per_launch=a.tpl)
        e.set_stream(s.cuda_stream)
        e.fill_random(3)
        e.step(a.tpl * 20)                              # warm: clocks, caches
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        e.step(a.tpl * a.launches)
        e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.launches
        waves = 16 * (H // a.band)
        cyc = waves * stage_steps(a.band, a.tpl) * 52.0
        eff = cyc / (1024 * us * 1e-6 * 2.4e9)
        print(json.dumps({"waves_per_simd": w, "rows": H, "band": a.band, "tpl": a.tpl,
                          "us_per_launch": round(us, 1),
                          "GCUPS": round(W * H * a.tpl / us / 1e3, 1),
                          "valu_eff_at_2.4GHz": round(eff, 3)}), flush=True)
        e.close()


if __name__ == "__main__":
    main()
