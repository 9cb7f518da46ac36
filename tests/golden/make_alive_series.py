"""Per-turn AliveCellsCount series for the BASELINE.json GPU configs C2 (5120^2, seed 1,
1000 turns) and C3 (16384^2, seed 2, 10000 turns), computed with the CPU bit-packed
oracle (oracle/bitref.c, pinned to the reference's fixtures by tests/test_oracle.py).

Written in the format of the reference's own series fixtures
(Local/check/alive/*.csv: header ``completed_turns,alive_cells``, rows 1..T), gzipped,
to tests/golden/alive/{W}x{H}_seed{S}.csv.gz.  Run in the build container; output
committed.  tests/test_gpu_run.py checks the run driver's AliveCellsCount events at
these sizes against them."""
import gzip
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

CASES = [(5120, 5120, 1, 1000), (16384, 16384, 2, 10000)]


def main():
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "alive")
    for w, h, seed, turns in CASES:
        t0 = time.time()
        _, counts = O.bit_run(O.gen_random(seed, w, h), w, turns, counts=True)
        lines = ["completed_turns,alive_cells"]
        lines += [f"{t + 1},{int(c)}" for t, c in enumerate(counts)]
        path = os.path.join(here, f"{w}x{h}_seed{seed}.csv.gz")
        with gzip.open(path, "wt", compresslevel=9) as f:
            f.write("\n".join(lines) + "\n")
        print(path, int(counts[-1]), f"{time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
