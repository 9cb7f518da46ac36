#!/usr/bin/env python3
"""Summarise a rocprofv3 run of bench.py into profiles/<tag>_*.{csv,json}.

Usage: summarize_profile.py TAG SRC KT [FETCH WRITE] [BOARD] [KERNEL] [SHAPE_JSON] [SQ] [KTPIN]
  SRC    the pass directory root (tools/profile_r02.sh: gpurun_out/prof2)
  KT     the --kernel-trace --stats pass (KT/ + KT.log holding the bench line), or - for
         a PMC-only summary
  FETCH / WRITE  the --pmc FETCH_SIZE / WRITE_SIZE passes of the same workload
  BOARD  which board of the bench run: 0 = the headline board, 1 = configs_measured[0]
  KERNEL (PMC passes of tools/kernel_run.py, which loads no board): the last 20 dispatches
         whose name contains this text instead of the first board's
  SHAPE_JSON  the bench's launch_shape that the pinned PMC passes ran (stored as `shape`)
  SQ     a --pmc pass of GRBM_GUI_ACTIVE + SQ_* counters of the same pinned run: the clock
         under load (GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration) and the VALU counts
  KTPIN  a --kernel-trace pass of the same pinned run: the pinned kernel's average duration

Timed dispatches: bench.py loads each board (k_il_convert), steps the warm-up turns, then
the timed turns, so the timed launches are the last `launches` stencil dispatches
(k_step*) before the next board's k_fill_random (the engine's create-time autotune also
dispatches the stencil, on other bands, so "the last N of the top kernel" is not enough).
Their names can mix K: the engine spreads T turns evenly over ceil(T / K) launches.

traffic per launch = (FETCH_SIZE x 2 + WRITE_SIZE) x 1024 bytes, medians over the last 20
stencil dispatches of the PMC pass's first board (a run with --c3-size 0, one board):
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads exactly half of a wide
(16 B/lane) coalesced stream (MI355X_MICROARCH.md, HBM section) and of the stencil's own
4-B/lane LDS-DMA row stream (tools/calib/calib_fetch.hip: 0.501 GiB for 1 GiB), so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Infinity-Cache hits are included
in both, so this is fabric traffic out of the XCD L2s (an upper bound on HBM bytes)."""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def board_segments(rows):
    """Split time-ordered dispatch rows into per-board stepping segments: the dispatches
    after each k_il_convert (board load) up to the next k_fill_random (next engine)."""
    segs, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "k_il_convert" in name:
            cur = []
            segs.append(cur)
        elif "k_fill_random" in name:
            cur = None
        elif cur is not None and ("k_step" in name or "k_tile_persist" in name or
                                  "k_tile_stream" in name):
            cur.append(r)
    return segs


def load_rows(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def main(tag, src, kt, fetch=None, write=None, board="0", kernel=None, shape=None, sq=None,
         ktpin=None):
    board = int(board)
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    res = {"source": f"{os.path.relpath(src, ROOT)}/{kt}", "board": board}
    if shape:
        # the launch shape (bench.py launch_shape) the PMC passes pinned: bench.py reports
        # `traffic` from this summary only for a launch of exactly this shape
        res["shape"] = json.loads(shape)
    line = None
    if kt != "-":
        shutil.copy(os.path.join(src, kt, "run_kernel_stats.csv"),
                    os.path.join(out, f"{tag}_kernel_stats.csv"))
        for ln in open(os.path.join(src, kt + ".log")).read().splitlines():
            if ln.startswith('{"metric"'):
                line = json.loads(ln)
    if line is not None:
        res["bench_line"] = line
        if board == 0:
            n, bench_us = line["roofline"]["launches"], line["roofline"]["launch_us"]
        else:
            c = line["configs_measured"][board - 1]
            n, bench_us = c["launches"], c["launch_us"]
        segs = board_segments(load_rows(os.path.join(src, kt, "run_kernel_trace.csv")))
        last = segs[board][-n:]
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last]
        names = {}
        for r in last:
            names[r["Kernel_Name"]] = names.get(r["Kernel_Name"], 0) + 1
        res.update({
            "timed_launches": len(last), "timed_kernels": names,
            "timed_avg_ns": statistics.mean(durs),
            "timed_span_avg_ns": (int(last[-1]["End_Timestamp"]) -
                                  int(last[0]["Start_Timestamp"])) / len(last),
            "bench_hip_event_launch_us": bench_us})
    for name, counter in ((fetch, "FETCH_SIZE"), (write, "WRITE_SIZE")):
        if not name or name == "-":
            continue
        rows = [r for r in load_rows(os.path.join(src, name, "run_counter_collection.csv"))
                if r["Counter_Name"] == counter]
        if kernel:
            seg = [r for r in rows if kernel in r["Kernel_Name"]][-20:]
        else:
            seg = board_segments(rows)[0][-20:]
        res[counter + "_kernels"] = sorted({r["Kernel_Name"] for r in seg})
        res[counter + "_kib_median"] = statistics.median(float(r["Counter_Value"]) for r in seg)
        res[counter + "_launches"] = len(seg)
    if "FETCH_SIZE_kib_median" in res and "WRITE_SIZE_kib_median" in res:
        rd = res["FETCH_SIZE_kib_median"] * 2 * 1024
        wr = res["WRITE_SIZE_kib_median"] * 1024
        res["read_bytes_per_launch"] = rd
        res["write_bytes_per_launch"] = wr
        res["traffic_bytes_per_launch"] = rd + wr
    if sq and sq != "-":
        rows = load_rows(os.path.join(src, sq, "run_counter_collection.csv"))
        if kernel:
            rows = [r for r in rows if kernel in r["Kernel_Name"]]
        else:
            rows = board_segments(rows)[0]
        by, dur = {}, {}
        for r in rows:
            by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        med = {n: statistics.median(v[-20:]) for n, v in by.items()}
        us = statistics.median(list(dur.values())[-20:])
        res["sq_counters_median"] = med
        res["sq_dispatch_us_median"] = us
        if "GRBM_GUI_ACTIVE" in med and us >= 90:
            # (GRBM_GUI_ACTIVE spans more than a short dispatch: 5120^2's 17 us launches read
            # 3.3 GHz, above the 2.4 GHz maximum; no clock from dispatches under 90 us -- the
            # N = 8 strip's 20-turn launch takes ~99)
            res["clock_ghz"] = round(med["GRBM_GUI_ACTIVE"] / 8 / (us * 1e3), 4)
        if "SQ_ACTIVE_INST_VALU" in med and "SQ_WAVE_CYCLES" in med:
            res["valu_active_per_wave_cycle"] = round(med["SQ_ACTIVE_INST_VALU"] /
                                                      med["SQ_WAVE_CYCLES"], 4)
    if ktpin and ktpin != "-":
        rows = load_rows(os.path.join(src, ktpin, "run_kernel_trace.csv"))
        rows = [r for r in rows if kernel in r["Kernel_Name"]] if kernel else rows
        # the timed call of tools/kernel_run.py: its last turns / K launches
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[-10:]]
        res["pinned_trace_launches"] = len(durs)
        res["pinned_trace_avg_ns"] = statistics.mean(durs) if durs else None
        res["pinned_trace_kernels"] = sorted({r["Kernel_Name"] for r in rows[-10:]})
    with open(os.path.join(out, f"{tag}_summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    show = {k: v for k, v in res.items() if k != "bench_line"}
    print(json.dumps(show, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
