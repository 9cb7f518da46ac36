#!/usr/bin/env python3
"""K1p debug: variants of a failing persistent-tile shape against the oracle, printing which
match and where the first wrong rows are.  usage: python tools/persist_debug.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import gol  # noqa: E402
from oracle import oracle as O  # noqa: E402

CASES = [  # name, w, h, tw, th, K, turns, code, persist
    ("A 896x90 K10 t31", 896, 90, 14, 30, 10, 31, 103, 1),
    ("B 896x90 K8 t32", 896, 90, 14, 30, 8, 32, 103, 1),
    ("C plain 896x90 K10 t31", 896, 90, 14, 30, 10, 31, 103, 0),
    ("D 1792x90 K10 t31", 1792, 90, 14, 30, 10, 31, 103, 1),
    ("E 896x150 K10 t31", 896, 150, 14, 50, 10, 31, 103, 1),
    ("F 896x90 tw7 K10 t31", 896, 90, 7, 30, 10, 31, 103, 1),
    ("G 896x90 K10 t40", 896, 90, 14, 30, 10, 40, 103, 1),
    ("H 896x90 K10 t10", 896, 90, 14, 30, 10, 20, 103, 1),
    ("I 896x90 K10 t31 416", 896, 90, 14, 30, 10, 31, 416, 1),
]
for name, w, h, tw, th, K, turns, code, persist in CASES:
    os.environ["GOL_MULTI_VARIANT"] = "15"
    os.environ["GOL_TILE"] = f"{tw},{code}"
    if persist:
        os.environ["GOL_PERSIST"] = str(K)
    else:
        os.environ.pop("GOL_PERSIST", None)
    start = O.gen_random(17, w, h)
    try:
        with gol.Engine(w, h, device=0, band_rows=th, turns_per_launch=K) as e:
            e.load_packed(start)
            e.step(turns)
            plan = e.last_launches()
            got = e.read_packed()
    except Exception as ex:  # noqa: BLE001
        print(name, "ERROR", ex, flush=True)
        continue
    want = O.bit_run(start, w, turns)
    bad = np.nonzero((got != want).any(axis=1))[0]
    print(f"{name}: plan {plan} match {len(bad) == 0} bad_rows {len(bad)} "
          f"first {bad[:8].tolist()} bad_words_row0 {int((got[bad[0]] != want[bad[0]]).sum()) if len(bad) else 0}",
          flush=True)
