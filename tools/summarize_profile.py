#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof) into profiles/<tag>_*.{csv,json}.

traffic per launch = (FETCH_SIZE x 2 + WRITE_SIZE) x 1024 bytes for the stencil kernel,
medians over the last 20 dispatches of the top kernel (the timed launches):
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads exactly half of a wide
(16 B/lane) coalesced stream (MI355X_MICROARCH.md, HBM section) and of the stencil's own
4-B/lane LDS-DMA row stream (tools/calib/calib_fetch.hip: 0.501 GiB for 1 GiB), so it is
doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.  Infinity-Cache hits are included in
both, so this is fabric traffic out of the XCD L2s (an upper bound on HBM bytes)."""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag, src=os.path.join(ROOT, "gpurun_out", "prof"), kernel="k_step"):
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"),
                os.path.join(out, f"{tag}_kernel_stats.csv"))
    stats = list(csv.DictReader(open(os.path.join(src, "kt", "run_kernel_stats.csv"))))
    top = max(stats, key=lambda r: float(r["TotalDurationNs"]))
    res = {"kernel": top["Name"], "calls": int(top["Calls"]),
           "avg_ns": float(top["AverageNs"]), "min_ns": float(top["MinNs"]),
           "max_ns": float(top["MaxNs"]), "share_pct": float(top["Percentage"])}
    # the bench's timed region = its last `launches` dispatches of the top kernel: average
    # exactly those (the trace also holds autotune / warm-up dispatches of the same kernel)
    import re
    log = os.path.join(src, "kt.log")
    trace = os.path.join(src, "kt", "run_kernel_trace.csv")
    if os.path.exists(log) and os.path.exists(trace):
        m = re.search(r'"launches": (\d+)', open(log).read())
        if m:
            n = int(m.group(1))
            disp = [r for r in csv.DictReader(open(trace)) if r["Kernel_Name"] == top["Name"]]
            disp.sort(key=lambda r: int(r["Start_Timestamp"]))
            last = disp[-n:]
            durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in last]
            res["timed_launches"] = len(last)
            res["timed_avg_ns"] = statistics.mean(durs)
            res["timed_span_avg_ns"] = (int(last[-1]["End_Timestamp"]) -
                                        int(last[0]["Start_Timestamp"])) / len(last)
            for ln in open(log).read().splitlines():
                if ln.startswith('{"metric"'):
                    res["bench_line"] = json.loads(ln)
    for name, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        p = os.path.join(src, name, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        # the bench's timed launches are the last dispatches of the top kernel; the
        # engine's create-time autotune dispatches the same kernel on other bands first
        rows = [r for r in csv.DictReader(open(p))
                if r["Kernel_Name"] == top["Name"] and r["Counter_Name"] == counter]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        rows = rows[-20:]
        res[counter + "_kib_median"] = statistics.median(float(r["Counter_Value"]) for r in rows)
        res[counter + "_launches"] = len(rows)
    if "FETCH_SIZE_kib_median" in res and "WRITE_SIZE_kib_median" in res:
        rd = res["FETCH_SIZE_kib_median"] * 2 * 1024
        wr = res["WRITE_SIZE_kib_median"] * 1024
        res["read_bytes_per_launch"] = rd
        res["write_bytes_per_launch"] = wr
        res["traffic_bytes_per_launch"] = rd + wr
    with open(os.path.join(out, f"{tag}_summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
