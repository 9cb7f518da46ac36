#!/usr/bin/env python3
"""Per-kernel medians of a tools/pmc_sq.sh pass (gpurun_out/pmc_sq*/run_counter_collection.csv)."""
import collections
import csv
import statistics
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_sq/run_counter_collection.csv"
rows = list(csv.DictReader(open(path)))
by = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    by[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, c in by.items():
    if "step" not in k and "tile_stream" not in k and "tile_persist" not in k:
        continue
    m = {n: statistics.median(v) for n, v in c.items()}
    us = statistics.median(dur[k])
    print(k, f"dispatches~{len(c['SQ_WAVES'])} dur_us={us:.1f}")
    for n in sorted(m):
        print(f"  {n:24s} {m[n]:.4g}")
    if "GRBM_GUI_ACTIVE" in m:
        print(f"  clock_GHz(GUI_ACTIVE/8/dur) {m['GRBM_GUI_ACTIVE'] / 8 / (us * 1e3):.3f}")
    if "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVE_CYCLES" in m:
        print(f"  valu_active/wave_cycles   {m['SQ_ACTIVE_INST_VALU'] / m['SQ_WAVE_CYCLES']:.3f}")
    if "SQ_WAIT_ANY" in m:
        print(f"  wait_any/wave_cycles      {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
        print(f"  wait_inst/wave_cycles     {m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
