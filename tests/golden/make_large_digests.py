"""Golden digests for the BASELINE.json sizes, computed with the CPU bit-packed
oracle (oracle/bitref.c, itself pinned to the reference fixtures by
tests/test_oracle.py).  Digest = sha256 of the packed board (rows x ceil(W/64)
little-endian uint64 words, LSB = lowest x) after `turns` turns from
oracle.gen_random(seed, W, H).  Run in the build container; output committed."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

CASES = [("5120x5120_seed1_t1000", 5120, 5120, 1, 1000),
         ("16384x16384_seed2_t10000", 16384, 16384, 2, 10000),
         ("65536x65536_seed3_t4", 65536, 65536, 3, 4),
         # the driver's bench command: 5 warm-up turns + 20 timed turns
         ("65536x65536_seed3_t25", 65536, 65536, 3, 25),
         ("65536x65536_seed3_t1000", 65536, 65536, 3, 1000)]


def main():
    """usage: make_large_digests.py [key ...]  (no keys: every case; keys: recompute those and
    keep the other committed entries)"""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "large_digests.json")
    only = set(sys.argv[1:])
    out = {}
    if only:
        with open(path) as f:
            out = json.load(f)
    for key, w, h, seed, turns in CASES:
        if only and key not in only:
            continue
        t0 = time.time()
        words = O.bit_run(O.gen_random(seed, w, h), w, turns)
        out[key] = {"width": w, "height": h, "seed": seed, "turns": turns,
                    "alive": O.popcount(words, w),
                    "sha256": hashlib.sha256(words.tobytes()).hexdigest()}
        print(key, out[key]["alive"], f"{time.time() - t0:.1f}s", flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
