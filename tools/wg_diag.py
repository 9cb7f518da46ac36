#!/usr/bin/env python3
"""Per-wave wait timing of k_step_wg (GOL_MULTI_VARIANT=11, kMultiWgDiag): prints, per wave
role of the split pipeline, the share of its lifetime spent waiting for its first row,
for upstream rows and for downstream ring space (the engine writes the summary to stderr)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
os.environ["GOL_MULTI_VARIANT"] = "11"
import gol  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=65536)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--bands", default="274,874")
    ap.add_argument("--tpl", default="16")
    a = ap.parse_args()
    for k in [int(x) for x in a.tpl.split(",")]:
        for b in [int(x) for x in a.bands.split(",")]:
            e = gol.Engine(a.size, a.height or a.size, device=0, band_rows=b, turns_per_launch=k)
            e.fill_random(3)
            for _ in range(2):
                e.step(k)
                e.sync()
            e.close()
            print(f"done K={k} band={b}", flush=True)


if __name__ == "__main__":
    main()
