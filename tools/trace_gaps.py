#!/usr/bin/env python3
"""Print the last N dispatches of a rocprofv3 kernel trace (run_kernel_trace.csv) with
durations and the idle gap before each, in microseconds: shows where a halo exchange
(rcclGenericKernel) leaves the GPU idle between stencil launches."""
import csv
import sys


def main(path, n=40):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    prev = None
    for r in rows[-int(n):]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000 if prev is not None else 0.0
        print(f"{r['Kernel_Name'][:48]:48s} {(e - s) / 1000:8.2f} us  gap {gap:7.2f} us  "
              f"grid {r['Grid_Size_X']}")
        prev = e


if __name__ == "__main__":
    main(*sys.argv[1:])
