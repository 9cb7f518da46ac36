#!/usr/bin/env python3
"""Headline benchmark: GoL cell updates/s (GCUPS) on MI355X.

Workload (BASELINE.json configs[3], the metric's headline size): one 65536 x 65536
random torus board (seed 3, oracle/bitref.c generator), `--steps` turns timed
after `--warmup` untimed turns.  One step = one turn = one pass of the per-turn
board update (reference calculateNextState, SubServer/distributor.go:119-208)
over the whole board.  The board is resident in HBM (bit-packed, 512 MiB per
buffer) before the timed region; no PGM I/O or alive-list work is timed.

N = 1: one torus engine.  N > 1 (torchrun, one rank per GPU): the board's rows
are split as the reference Server splits them (Server/gol/distributor.go:106-116)
and each rank exchanges `halo` boundary rows with its ring neighbours over RCCL every
`halo` turns ("strong" scaling: the total board is fixed).  The halo defaults to
min(128, turns timed), the deepest whose windows the timed turns hold whole, and the timed
region starts at a window boundary: it holds one exchange per `halo` turns, the run's own
cadence (the driver's 20 turns: one 20-row exchange, then one 20-turn launch;
config.exchanges_timed, per-rank exchange times in config.exchange_us_per_rank, and the
stencil alone, with no exchange timed, in config.compute_only).

Printed (rank 0): one JSON line with the driver's contract fields plus
`roofline` (the dominant kernel's algorithmic HBM bytes per launch -- one read + one
write of the packed board, 0.25/k B per cell-update for k fused turns -- per average
launch time, vs 8 TB/s; PMC-measured bytes in `traffic`), `k1_equivalent` (the k = 1
bytes of SURVEY 8(d), which exceed any HBM roof once k > 1), `valu_roofline` (the
binding roof of the blocked kernel: the 52-cycle VALU issue model, at 2.4 GHz and at the
clock measured under load, with the kernel's SIMD cycles per VALU and its VALU inflation
from the SQ pass of the same launch), `configs_measured` and `cpu_baseline`:
  * config.create_ms: the engine's create time (the first engine of a pinned shape in a
    process also runs ~60 ms of its launches: gol_engine.cpp check_pinned);
    config.cold_first_call (N = 1): the same 20 turns in an engine created with that check
    off, before anything else ran on the GPU;
  * configs_measured: BASELINE configs[2] (16384^2, 10000 turns; at N = 1 and 2, the GPU
    counts configs[2] is quoted on); at N = 1 configs[1] (5120^2 seed 1, 1000 turns, with
    the final AliveCellsCount snapshot inside the timed region) and configs[0] on the GPU
    (the reference's 512^2 image, 100 turns, checked byte-exact against
    Local/check/images/512x512x100.pgm).
  * cpu_baseline: oracle/refcpu.c, the C restatement of the reference's CPU path, on a
    bounded sample of the headline board on this host's CPU share, plus configs[0] in full
    (512^2 x 100 turns, Threads = 8) checked byte-exact against the same golden image.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "conway-s-gol-distributed_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "cell updates/sec (GCUPS) at 16384² & 65536², 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
BYTES_PER_CELL_UPDATE = 0.25   # 1 bit read + 1 bit written per cell per turn
# VALU-issue roofline of the temporal-blocking tile kernel: one row of one wavefront (64 lanes
# x 64 cells = 4096 cell-updates) issues 22 VALU -- 18 v_bitop3 and 4 lane-shift instructions
# (2 DPP moves + 2 v_alignbit, or the west carry's v_cmp + v_addc).  The roof is the issue
# model: v_bitop3 at the 2-cycle wave64 floor, the 4 half-rate lane shifts at 4 cycles = 52
# SIMD cycles per 4096 cell-updates; 1024 SIMDs x 2.4 GHz -> 193.6 T cell-updates/s per GPU.
# No measured stream beats it (round-5 verdict: the 144k "ceiling" measured on the isolated
# stream at 69.9 cycles is beaten by the production kernel's own 2.83 cycles per VALU, so it
# is reported as `algorithmic_ceiling`, not as the roof).
VALU_SIMDS, VALU_CLOCK_HZ = 1024, 2.4e9
VALU_PER_ROW = 22
VALU_MODEL_CYCLES_PER_4096 = 52.0
VALU_PEAK_GCUPS = VALU_SIMDS * VALU_CLOCK_HZ / VALU_MODEL_CYCLES_PER_4096 * 4096 / 1e9
# tools/calib/stencil_issue.hip (profiles/r05_stencil_issue_calib.json): the stencil's exact
# stream in registers, SEG 24, 6 waves per SIMD, no LDS / barrier / memory: 69.9 cycles
STREAM_CYCLES_PER_4096 = 69.9
STREAM_CEILING_GCUPS = VALU_SIMDS * VALU_CLOCK_HZ / STREAM_CYCLES_PER_4096 * 4096 / 1e9
# N > 1: the deepest strip halo (rows per side = turns between exchanges) the bench uses
HALO_MAX = 128


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--size", type=int, default=65536, help="board side (default 65536)")
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--halo", type=int, default=0,
                    help="strip halo depth (rows exchanged every `halo` turns, N > 1); 0 = "
                         f"min({HALO_MAX}, turns timed): the deepest halo whose windows the "
                         "timed turns hold whole")
    ap.add_argument("--band", type=int, default=0, help="stencil band rows (0 = auto)")
    ap.add_argument("--tpl", type=int, default=0,
                    help="turns per stencil launch (temporal blocking; 0 = engine default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-turns", type=int, default=2)
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="threads for the CPU baseline (0 = this host's CPU share: the "
                         "affinity mask, capped by OMP_NUM_THREADS when that is set)")
    ap.add_argument("--c3-size", type=int, default=16384,
                    help="board side of the second measured config (BASELINE configs[2]; "
                         "0 = skip)")
    ap.add_argument("--c3-turns", type=int, default=10000,
                    help="turns of the second config (configs[2]: 10000)")
    ap.add_argument("--c2-size", type=int, default=5120,
                    help="board side of BASELINE configs[1] (N = 1 only; 0 = skip)")
    ap.add_argument("--c2-turns", type=int, default=1000)
    ap.add_argument("--no-cold", action="store_true",
                    help="N = 1: skip the cold first-call figure (config.cold_first_call)")
    ap.add_argument("--no-c1", action="store_true",
                    help="skip BASELINE configs[0] (512^2 image, 100 turns) on GPU and CPU")
    ap.add_argument("--overlap", type=int, default=0,
                    help="N > 1, direct RCCL: 1 = overlap the halo exchange with the first "
                         "launch's interior rows (gol_step_overlap, RCCL on its own stream); "
                         "0 (default) = exchange on the engine stream, serialised: measured "
                         "faster at halo 128 (8-strip shape, one GPU exchanging with itself: "
                         "6.12 vs 6.52 us/turn, profiles/r02_overlap_strip8.log)")
    ap.add_argument("--transport", choices=("rccl", "torch"), default="rccl",
                    help="N > 1 halo transport on the nccl backend: direct RCCL send/recv on "
                         "the engine's stream (default) or torch batch_isend_irecv")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="N > 1 transport: nccl (= RCCL over xGMI); gloo stages halos through "
                         "host memory and lets ranks share a GPU (tests only)")
    return ap.parse_args()


def pmc_summary(size, k, shape=None):
    """The newest committed rocprofv3 PMC summary for this board size, depth k and -- when the
    summary records one -- launch shape (profiles/rNN_k{k}_{size}*_summary.json, written by
    tools/profile_r04.sh + tools/summarize_profile.py): a summary whose `shape` differs from
    the launch that ran is not used, so `traffic` (and the clock under load) always come from
    the kernel the bench timed.  (None, None) if no pass."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_k{k}_{size}*_summary.json")))
    for path in reversed(files):                 # the newest pass that holds PMC bytes
        with open(path) as f:
            d = json.load(f)
        if not d.get("traffic_bytes_per_launch"):
            continue
        if "shape" in d and shape is not None and d["shape"] != shape:
            continue
        if "shape" not in d and shape is not None and shape.get("kernel") == 15:
            continue                             # (older passes: shape unknown)
        return d, os.path.relpath(path, ROOT)
    return None, None


def pmc_traffic(size, k, shape=None):
    """HBM traffic per launch of the stencil from pmc_summary; (None, None) if no pass."""
    d, src = pmc_summary(size, k, shape)
    return (d["traffic_bytes_per_launch"], src) if d else (None, None)


def cpu_share():
    """(threads to use, affinity-mask CPUs, OMP_NUM_THREADS or None): the GPU box's CPU
    share for one GPU is OMP_NUM_THREADS (16) while its affinity mask lists every CPU of
    the host, so the share caps the mask."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    share = min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff
    return share, aff, (int(omp) if omp and omp.isdigit() else None)


def cpu_baseline(size, seed, turns, cores):
    """oracle/refcpu.c (literal restatement of the reference's Server/SubServer CPU path,
    4 sub-servers as in the reference's default SUB list, Threads = the core count) on the
    same board for a bounded number of turns."""
    from oracle import oracle as O
    share, aff, omp = cpu_share()
    if cores <= 0:
        cores = share
    board = O.unpack(O.gen_random(seed, size, size), size)
    t0 = time.perf_counter()
    O.ref_run(board, turns, nsub=4, threads=cores, ncores=cores)
    dt = time.perf_counter() - t0
    del board
    return {"value": round(size * size * turns / dt / 1e9, 4), "unit": "GCUPS",
            "cores": cores, "kind": "port",
            "sample": f"{size}x{size} random board seed {seed}, {turns} turns, oracle/refcpu.c "
                      f"(4 sub-servers x Threads={cores} goroutine-equivalents on {cores} "
                      f"OpenMP threads; host affinity mask {aff} CPUs, OMP_NUM_THREADS "
                      f"{omp}; no gob/HTTP: optimistic), {dt:.1f} s"}


def measure(a, size, steps, warmup, world, rank, gpu, dev, dev_ids, stream, seed=None,
            snapshot=False, halo=None, compute_only=False):
    """Time `steps` turns of one size x size torus board (whole board at N = 1, this rank's
    row strip at N > 1) after `warmup` turns.  `snapshot`: the AliveCellsCount pair of the
    final turn (gol_snapshot) is taken inside the timed region.

    N > 1: the strip keeps `halo` rows per side and exchanges them every `halo` turns.  The
    timed region starts at a window boundary (DistStrip.start_window: its first action is an
    exchange), so it holds ceil(steps / halo) exchanges -- one per `halo` turns, the cadence of
    the run -- each bracketed by HIP events (per-rank exchange time).  `compute_only`: then
    time the same strip again over min(steps, halo) turns right after an untimed exchange (no
    exchange inside: the stencil alone, a labelled secondary figure).  Returns the timing and
    roofline inputs."""
    seed = a.seed if seed is None else seed
    import gol
    from gol.distributed import DistStrip, EngineStrip, make_engine_strip

    W = H = size
    comm = None
    t_create = time.perf_counter()
    if world == 1:
        eng = gol.Engine(W, H, device=gpu, band_rows=a.band, turns_per_launch=a.tpl)
        create_ms = (time.perf_counter() - t_create) * 1e3
        eng.set_stream(stream.cuda_stream)
        eng.fill_random(seed)
        runner = eng
        rows_local = H
        transport = ""
        fallback = None
    else:
        eng = make_engine_strip(W, H, rank, world, halo, gpu, band_rows=a.band,
                                turns_per_launch=a.tpl)
        create_ms = (time.perf_counter() - t_create) * 1e3
        eng.fill_random(seed)
        transport = a.transport
        fallback = None
        if a.backend == "nccl" and transport == "rccl":
            from gol.rccl import RcclComm, RcclTimeout
            try:
                comm = RcclComm(rank, world, dev)   # raises on every rank together
            except RcclTimeout as e:
                # a bootstrap that cannot complete: no other transport would reach the peers
                # either -- end this rank now, non-zero (torchrun then stops the others)
                print(f"rank {rank}: {e}", file=sys.stderr, flush=True)
                os._exit(3)
            except (OSError, RuntimeError) as e:
                if rank == 0:
                    print(f"direct RCCL unavailable ({e}); using torch batch_isend_irecv",
                          file=sys.stderr)
                comm, transport = None, "torch"
                fallback = f"direct RCCL failed, fell back to torch batch_isend_irecv: {e}"[:300]
        runner = DistStrip(EngineStrip(eng, dev, stream), rank, world,
                           stage_on_host=a.backend == "gloo", rccl=comm,
                           overlap=bool(a.overlap))
        rows_local = eng.rows
        # set up the RCCL p2p connections outside the timed region: one halo exchange now
        # (all strips hold their true halo rows after fill_random, so it changes nothing)
        runner.exchange()
    runner.step(warmup)
    if world > 1:
        runner.start_window()
        runner.time_exchanges(-(-steps // max(eng.halo, 1)) + 1)
    # torch creates an event's HIP event at its first record: do that outside the timed region
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    ev1.record(stream)
    launches0 = eng.info().launches
    exchanges0 = getattr(runner, "exchanges", 0)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier(device_ids=dev_ids)
        torch.cuda.synchronize(dev)

    # (ev0 is recorded on the idle stream just before the clock starts: its host call is
    # instrumentation, not part of the timed steps; ev1's overlaps the running kernels)
    ev0.record(stream)
    t0 = time.perf_counter()
    runner.step(steps)
    ev1.record(stream)
    alive = eng.snapshot() if snapshot else None
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier(device_ids=dev_ids)
        torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    plan = eng.last_launches()          # the last gol_step call's launches (N > 1: one window)
    tiles = eng.last_launch_tiles(blocks=True)   # (tile width in lanes, segment code, waves,
                                                 # turns per block) of each
    info = eng.info()
    launches = info.launches - launches0
    exchanges = getattr(runner, "exchanges", 0) - exchanges0
    xus = runner.exchange_us() if world > 1 else []
    if world > 1 and steps > eng.halo:
        # the timed region's last gol_step ran only the last (partial) window: take the launch
        # shape from one more whole window, untimed (every rank: it exchanges first)
        runner.start_window()
        runner.step(eng.halo)
        plan = eng.last_launches()
        tiles = eng.last_launch_tiles(blocks=True)
    comp = None
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64,
                         device=dev if a.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        # every rank's mean exchange time and count, to rank 0
        mine = torch.tensor([sum(xus) / len(xus) if xus else -1.0, float(len(xus)),
                             max(xus) if xus else -1.0], dtype=torch.float64,
                            device=dev if a.backend == "nccl" else "cpu")
        allx = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allx, mine)
        xus = [[round(float(x[0]), 2), int(x[1]), round(float(x[2]), 2)] for x in allx]
        if compute_only:
            cturns = min(steps, eng.halo)
            runner.exchange()                   # untimed: the halos are fresh for cturns
            launches1 = eng.info().launches
            ex1 = runner.exchanges
            torch.cuda.synchronize(dev)
            dist.barrier(device_ids=dev_ids)
            torch.cuda.synchronize(dev)
            ev0.record(stream)
            c0 = time.perf_counter()
            runner.step(cturns)
            ev1.record(stream)
            torch.cuda.synchronize(dev)
            dist.barrier(device_ids=dev_ids)
            torch.cuda.synchronize(dev)
            cw = torch.tensor([time.perf_counter() - c0], dtype=torch.float64,
                              device=dev if a.backend == "nccl" else "cpu")
            dist.all_reduce(cw, op=dist.ReduceOp.MAX)
            comp = {"steps": cturns, "wall": float(cw.item()), "gpu_ms": ev0.elapsed_time(ev1),
                    "launches": eng.info().launches - launches1,
                    "exchanges": runner.exchanges - ex1}
    overlap = bool(getattr(runner, "overlap", False))
    if comm is not None:
        comm.close()
    out = {"W": W, "H": H, "steps": steps, "wall": wall, "gpu_ms": gpu_ms,
           "launches": launches, "K": info.turns_per_launch, "rows_local": rows_local,
           "buffer_rows": int(info.buffer_rows),
           "band": info.band_rows, "fast": bool(info.fast_path), "halo": info.halo,
           "transport": transport, "overlap": overlap, "plan": plan, "tiles": tiles,
           "seed": seed, "fallback": fallback,
           "shape_source": SHAPE_SOURCES.get(int(info.shape_source), "?"),
           "exchanges": exchanges, "alive": alive, "create_ms": round(create_ms, 2),
           "exchange_us": xus, "compute_only": comp}
    eng.close()
    return out


def measure_cold(a, gpu, stream):
    """The headline board's timed turns with no create-time check of the pinned shape
    (GOL_PIN_VERIFY_MS=0: no ~60 ms of launches right before the first steps), in a process
    whose GPU has done nothing else yet: what a caller that creates one engine and steps it at
    once sees.  Run before the headline engine, whose own check then runs as usual."""
    import gol
    old = os.environ.get("GOL_PIN_VERIFY_MS")
    os.environ["GOL_PIN_VERIFY_MS"] = "0"
    try:
        t0 = time.perf_counter()
        eng = gol.Engine(a.size, a.size, device=gpu, band_rows=a.band, turns_per_launch=a.tpl)
        create_ms = (time.perf_counter() - t0) * 1e3
    finally:
        if old is None:
            os.environ.pop("GOL_PIN_VERIFY_MS", None)
        else:
            os.environ["GOL_PIN_VERIFY_MS"] = old
    eng.set_stream(stream.cuda_stream)
    eng.fill_random(a.seed)
    eng.step(a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.step(a.steps)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    eng.close()
    return {"value": round(a.size * a.size * a.steps / wall / 1e9, 2), "unit": "GCUPS",
            "ms_per_step": round(wall * 1e3 / a.steps, 5), "create_ms": round(create_ms, 2),
            "definition": "the same board, turns and warm-up in a fresh engine created with "
                          "GOL_PIN_VERIFY_MS=0 before anything else ran on the GPU: no "
                          "create-time check of the pinned shape (and so no GPU clock warm-up) "
                          "before the first steps"}


# gol_info.shape_source: where the launch shape the timed region ran came from
SHAPE_SOURCES = {0: "defaults", 1: "create-time timing search",
                 2: "pinned MI355X shape table (gol_engine.cpp kKnownShapes)"}

KERNELS = {16: "k_tile_persist<K> (k_step_tile's 2-D tiles resident across blocks of turns)",
           17: "k_tile_stream<K> (k_step_tile's 2-D tiles in blocks of turns, items taken in "
               "order by resident workgroups: one launch start and tail per step)",
           7: "k_step_skew<K> (interleaved layout, one pipeline per wave)",
           8: "k_step_wg<K> (pipeline split over a workgroup, band tiles)",
           9: "k_step_wg<K> (pipeline split over a workgroup, helix tiles)",
           12: "k_step_wg<K> (helix tiles, parallelogram bands)",
           13: "k_step_wg<K> (helix tiles, in-order stages)",
           14: "k_step_wg<K> (parallelogram bands, in-order stages)",
           15: "k_step_tile<K> (2-D tile resident in registers for all K turns)",
           0: "k_step_ring<D=3> (one turn per launch)"}


def kernel_depth(plan, default):
    """(run-length summary, dominant kernel id, its deepest planned launch)."""
    text, kvar = plan_summary(plan)
    return text, kvar, max((k for k, v, _ in plan if v == kvar), default=default)


def launch_shape(plan, tiles, kvar, kdepth, buffer_rows=None):
    """The shape of the dominant kernel's deepest launch: kernel, turns, band rows, the
    engine's buffer rows (a strip's owned rows + 2 x halo) and, for k_step_tile, the tile
    (width in words, height, rows per lane segment, turn order, words per lane, waves per
    workgroup) -- what the profiles in profiles/ must have measured."""
    for (k, v, band), t in zip(plan, tiles or [(0, 0, 0, 0)] * len(plan)):
        if v == kvar and k == kdepth:
            sh = {"kernel": v, "turns": k, "band_rows": band}
            if buffer_rows is not None:
                sh["buffer_rows"] = int(buffer_rows)
            if v in (15, 16, 17) and t[0] > 0:
                tw, code, waves, blk = t
                if v in (16, 17):
                    sh["block_turns"] = blk
                words = code // 1000 + 1
                sh["tile"] = {"code": code, "width_words": tw * words, "width_lanes": tw,
                              "height_rows": band, "seg_rows": code % 100,
                              "turn_order": code // 100 % 10, "words_per_lane": words,
                              "waves_per_workgroup": waves}
            return sh
    return {"kernel": kvar, "turns": kdepth}


def valu_figures(d, cells, turns):
    """From a PMC summary's SQ pass of the launch (profiles/..._summary.json): SIMD cycles per
    VALU instruction (dispatch time x the clock under load / VALU per SIMD) and the VALU
    inflation (SQ_INSTS_VALU / the useful 22 per 4096 cell-updates of `cells` x `turns`)."""
    if not d:
        return None, None
    sq = d.get("sq_counters_median") or {}
    n = sq.get("SQ_INSTS_VALU")
    if not n:
        return None, None
    cpi = None
    if d.get("clock_ghz") and d.get("sq_dispatch_us_median"):
        cycles = d["sq_dispatch_us_median"] * 1e3 * d["clock_ghz"]
        cpi = round(cycles / (n / VALU_SIMDS), 3)
    useful = cells * turns / 4096 * VALU_PER_ROW
    return cpi, round(n / useful, 4)


def config_entry(c, label, world, parallel):
    """configs_measured entry: GCUPS, launch plan, roofline fractions of one measure()."""
    g = c["W"] * c["H"] * c["steps"] / c["wall"] / 1e9
    lu = c["gpu_ms"] * 1e3 / max(c["launches"], 1)
    b = BYTES_PER_CELL_UPDATE * c["rows_local"] * c["W"]
    text, kvar, kd = kernel_depth(c["plan"], c["K"])
    shape = launch_shape(c["plan"], c.get("tiles"), kvar, kd, c.get("buffer_rows"))
    d, src = pmc_summary(c["W"], kd, shape)
    traffic = d["traffic_bytes_per_launch"] if d else None
    cpi, infl = valu_figures(d, c["rows_local"] * c["W"], kd)
    e = {"workload": label, "value": round(g, 2), "unit": "GCUPS", "n_gpus": world,
         "ms_per_step": round(c["wall"] * 1e3 / c["steps"], 6), "parallelism": parallel,
         "band_rows": shape.get("band_rows", c["band"]), "temporal_blocking_k": kd,
         "launch_shape": shape, "shape_source": c.get("shape_source"),
         "create_ms": c.get("create_ms"),
         "kernel": KERNELS.get(kvar, f"kernel {kvar}").replace("<K>", f"<K={kd}>"),
         "launch_plan": text[:300], "traffic": traffic, "traffic_source": src,
         "launch_us": round(lu, 3), "launches": c["launches"],
         "roofline_frac": round(b / (lu * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
         "valu_roofline_frac": round(g / world / VALU_PEAK_GCUPS, 4),
         "valu_cycles_per_instr": cpi, "valu_inflation": infl}
    if world > 1:
        e.update(exchange_fields(c))
        e["transport_fallback"] = c.get("fallback")
    if c.get("alive") is not None:
        e["alive_cells_final"] = list(c["alive"])
    return e


def exchange_fields(c):
    """N > 1: the exchanges inside the timed region, each rank's mean / max exchange time
    (HIP events around the transport on its stream: the transfer plus any wait for the
    neighbours) and the halo cadence."""
    out = {"exchanges_timed": c["exchanges"], "halo": c["halo"],
           "exchange_us_per_rank": [{"rank": r, "mean_us": x[0], "count": x[1], "max_us": x[2]}
                                    for r, x in enumerate(c.get("exchange_us") or [])]}
    comp = c.get("compute_only")
    if comp:
        out["compute_only"] = {
            "value": round(c["W"] * c["H"] * comp["steps"] / comp["wall"] / 1e9, 2),
            "unit": "GCUPS", "turns": comp["steps"], "exchanges_timed": comp["exchanges"],
            "ms_per_step": round(comp["wall"] * 1e3 / comp["steps"], 6),
            "definition": "the same strips over min(turns, halo) turns right after an untimed "
                          "exchange: the stencil alone, no exchange inside the timed region "
                          "(secondary figure; `value` includes the exchanges)"}
    return out


def measure_c1(gpu, stream):
    """BASELINE configs[0] on the GPU: the reference's Local/images/512x512.pgm, 100 turns,
    gol_load -> gol_step -> gol_read_board, byte-compared with Local/check/images/
    512x512x100.pgm (tests/golden fixtures).  Timed from the loaded board to the read-back
    bytes (one warm run first)."""
    import numpy as np
    import gol
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import golden_data as G
    board, want = G.input_board(512), G.check_board(512, 100)
    eng = gol.Engine(512, 512, device=gpu)
    eng.set_stream(stream.cuda_stream)
    best, exact = None, True
    for _ in range(3):
        eng.load(board)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.step(100)
        got = eng.read_board()
        dt = time.perf_counter() - t0
        exact = exact and bool(np.array_equal(got, want))
        best = dt if best is None else min(best, dt)
    plan = eng.last_launches()
    tiles = eng.last_launch_tiles(blocks=True)
    eng.close()
    _, kvar, kd = kernel_depth(plan, 0)
    return {"workload": "512x512 Local/images/512x512.pgm, 100 turns (BASELINE configs[0]) "
                        "on the GPU, load excluded, read-back of the 0/255 bytes included",
            "value": round(512 * 512 * 100 / best / 1e9, 3), "unit": "GCUPS", "n_gpus": 1,
            "ms_per_step": round(best * 1e3 / 100, 6), "launch_plan": plan_summary(plan)[0],
            "launch_shape": launch_shape(plan, tiles, kvar, kd),
            # (the packed board is 32 KiB: it stays in the L2 between launches, and the run is
            # bound by launch latency and the read-back, not by HBM)
            "traffic": None, "traffic_note": "32 KiB board, L2-resident across launches: "
                                             "launch-latency bound, no HBM roofline",
            "bit_exact_vs_check_image": exact, "best_of": 3}


def cpu_c1(cores_note):
    """BASELINE configs[0] on the CPU in full: oracle/refcpu.c (the reference's byte-per-cell
    calculateNextState with its Server strip split and SubServer thread split), Threads = 8
    on 8 OpenMP threads, 100 turns of the 512^2 image, byte-compared with the golden."""
    import numpy as np
    from oracle import oracle as O
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import golden_data as G
    board, want = G.input_board(512), G.check_board(512, 100)
    t0 = time.perf_counter()
    got = O.ref_run(board, 100, nsub=4, threads=8, ncores=8)
    dt = time.perf_counter() - t0
    return {"value": round(512 * 512 * 100 / dt / 1e9, 4), "unit": "GCUPS", "cores": 8,
            "kind": "port", "seconds": round(dt, 4),
            "bit_exact_vs_check_image": bool(np.array_equal(got, want)),
            "sample": "BASELINE configs[0] in full: Local/images/512x512.pgm, 100 turns, "
                      "oracle/refcpu.c with 4 sub-servers x Threads=8 on 8 OpenMP threads "
                      f"({cores_note}; no gob/HTTP: optimistic)"}


def plan_summary(plan):
    """Run-length summary of the engine's launches, e.g. '2 x (10 turns, kernel 7, band 137)',
    and the kernel id that ran the most turns."""
    runs, turns = [], {}
    for k, var, band in plan:
        turns[var] = turns.get(var, 0) + k
        if runs and runs[-1][1] == (k, var, band):
            runs[-1][0] += 1
        else:
            runs.append([1, (k, var, band)])
    text = ", ".join(f"{n} x ({k} turns, kernel {v}, band {b})" for n, (k, v, b) in runs)
    return text, (max(turns, key=turns.get) if turns else 0)


def parallelism(a, world, m):
    if world == 1:
        return "row-strips x1"
    how = ({"rccl": "RCCL send/recv on the engine stream" + (
                ", overlapped with the interior rows" if m["overlap"] else ""),
            "torch": "RCCL via torch batch_isend_irecv"}[m["transport"]]
           if a.backend == "nccl" else "gloo host-staged")
    return f"row-strips x{world}, halo {m['halo']}, {how}"


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    gpu = local if a.backend == "nccl" else local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    dev_ids = [gpu] if a.backend == "nccl" else None
    # a dedicated (non-default) stream shared by the engine, the events and RCCL
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    # torch creates the HIP stream on first use (~8 ms on the GPU box): do that now, not
    # between the engine's create-time autotune and the warm-up -- an idle MI355X lowers its
    # clock, and the short timed region then runs before it has ramped back
    # (profiles/r02_clock_pmc_bench20.txt, tools/phase_timing.py)
    stream.synchronize()
    _ = stream.cuda_stream

    if a.backend == "gloo" and world > max(torch.cuda.device_count(), 1):
        # ranks share a GPU: no parallelogram bands (their cross-workgroup waits assume one
        # grid per device at a time; the engine cannot see other processes' grids)
        os.environ["GOL_SHARED_DEVICE"] = "1"
    cold = None
    if world == 1 and not a.no_cold:
        cold = measure_cold(a, gpu, stream)
    # N > 1: halo = turns between exchanges; by default the deepest whose windows the timed
    # turns hold whole (the driver's 20 turns: one 20-row exchange, then one 20-turn launch)
    halo = a.halo or min(HALO_MAX, a.steps)
    m = measure(a, a.size, a.steps, a.warmup, world, rank, gpu, dev, dev_ids, stream, halo=halo,
                compute_only=True)
    c3 = None
    # (BASELINE configs[2] is quoted on 1 and 2 GPUs)
    if a.c3_size > 0 and a.c3_size != a.size and world <= 2:
        c3 = measure(a, a.c3_size, a.c3_turns, max(a.warmup, 60), world, rank, gpu, dev,
                     dev_ids, stream, halo=a.halo or min(HALO_MAX, a.c3_turns))
    c2 = None
    if world == 1 and a.c2_size > 0 and a.c2_size != a.size:
        c2 = measure(a, a.c2_size, a.c2_turns, max(a.warmup, 64), world, rank, gpu, dev,
                     dev_ids, stream, seed=1, snapshot=True)
    c1 = measure_c1(gpu, stream) if world == 1 and not a.no_c1 else None

    if rank == 0:
        W, H, K = m["W"], m["H"], m["K"]
        gcups = W * H * a.steps / m["wall"] / 1e9
        # Dominant kernel: one launch = turns/launches turns over this rank's rows.
        # Roofline (HBM): the bytes the blocked kernel must move per launch are one read and
        # one write of the packed board -- 0.25/k B per cell-update x k turns x cells =
        # 0.25 B x cells -- divided by the average launch duration (HIP events on the
        # engine's stream over the timed region / launches, inter-kernel gaps included; at
        # N > 1 the exchanges inside the region too).
        # `traffic` = the PMC-measured HBM bytes per launch of the same kernel (profiles/).
        # The k = 1 equivalent (0.25 B per cell-update x all cell-updates) is reported
        # separately: it exceeds the HBM peak once k > 1, so it is not a fraction of a roof.
        cells_local = m["rows_local"] * W
        launch_us = m["gpu_ms"] * 1e3 / max(m["launches"], 1)
        turns_per_launch = a.steps / max(m["launches"], 1)
        bytes_board = BYTES_PER_CELL_UPDATE * cells_local
        bytes_k1 = BYTES_PER_CELL_UPDATE * turns_per_launch * cells_local
        achieved = bytes_board / (launch_us * 1e-6) / 1e9
        plan_text, kvar, kdepth = kernel_depth(m["plan"], K)
        shape = launch_shape(m["plan"], m.get("tiles"), kvar, kdepth, m["buffer_rows"])
        d, traffic_src = pmc_summary(W, kdepth, shape)
        traffic = d["traffic_bytes_per_launch"] if d else None
        out = {
            "metric": METRIC,
            "value": round(gcups, 2),
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(m["wall"] * 1e3 / a.steps, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": f"{W}x{H} random torus board (seed {a.seed}), "
                                   f"{a.steps} turns, bit-packed stencil, up to {kdepth} turns "
                                   f"per launch",
                       "board": [W, H], "turns": a.steps,
                       "parallelism": parallelism(a, world, m),
                       "band_rows": shape.get("band_rows", m["band"]), "fast_path": m["fast"],
                       "temporal_blocking_k": kdepth,
                       "launch_shape": shape, "shape_source": m["shape_source"],
                       "create_ms": m["create_ms"],
                       "launch_plan": plan_text},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "definition": f"algorithmic HBM bytes of one blocked launch: 0.25/k B "
                                       f"per cell-update x k turns x cells = one read + one "
                                       f"write of the packed board ({int(bytes_board)} B), k = "
                                       f"{turns_per_launch:g} turns per launch on average, per "
                                       f"average launch time",
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": KERNELS.get(kvar, f"kernel {kvar}").replace("<K>", f"<K={kdepth}>"),
                         "launch_us": round(launch_us, 2), "launches": m["launches"],
                         "turns_per_launch": round(turns_per_launch, 3),
                         "bytes_per_launch": int(bytes_board)},
            "k1_equivalent": {"achieved": round(bytes_k1 / (launch_us * 1e-6) / 1e9, 1),
                              "unit": "GB/s",
                              "definition": "0.25 B per cell-update (SURVEY 8d, k = 1) x every "
                                            "cell-update of a launch, per launch time: the HBM "
                                            "bandwidth a one-turn-per-pass kernel would need "
                                            "to match this rate"},
            "valu_roofline": None,
            "cpu_baseline": None,
        }
        if K > 1:
            per_gpu = gcups / world
            cpi, infl = valu_figures(d, cells_local, kdepth)
            out["valu_roofline"] = {
                "bound": "valu", "achieved": round(per_gpu, 1), "peak": round(VALU_PEAK_GCUPS, 1),
                "unit": "GCUPS per GPU", "frac": round(per_gpu / VALU_PEAK_GCUPS, 4),
                "model": "issue model: 22 VALU per 4096 cell-updates (one wave row), 18 "
                         "v_bitop3 at the 2-cycle wave64 floor + 4 half-rate lane shifts at 4 "
                         "cycles = 52 SIMD cycles; 1024 SIMDs x 2.4 GHz; useful cell-updates "
                         "only (halo lanes, tile halos and syncs count against it)",
                "clock_ghz_measured": None, "peak_at_measured_clock": None,
                "frac_at_measured_clock": None, "clock_source": None,
                "valu_cycles_per_instr": cpi, "valu_inflation": infl,
                "valu_source": traffic_src if cpi or infl else None,
                "algorithmic_ceiling": {
                    "peak": round(STREAM_CEILING_GCUPS, 1), "unit": "GCUPS per GPU",
                    "frac": round(per_gpu / STREAM_CEILING_GCUPS, 4),
                    "definition": "the stencil's exact stream in registers (no LDS, barrier or "
                                  "memory; SEG 24, 6 waves per SIMD) measured at 69.9 SIMD cycles "
                                  "per 4096 cell-updates (tools/calib/stencil_issue.hip, "
                                  "profiles/r05_stencil_issue_calib.json) -- a measured reference "
                                  "point, not a roof: the production kernel issues faster "
                                  "(valu_cycles_per_instr)"}}
            if d and d.get("clock_ghz"):
                # the same model at the clock the kernel ran at under load (GRBM_GUI_ACTIVE
                # per XCD over the dispatch time, the SQ pass of the pinned shape)
                pk = VALU_PEAK_GCUPS * d["clock_ghz"] / (VALU_CLOCK_HZ / 1e9)
                out["valu_roofline"].update({
                    "clock_ghz_measured": d["clock_ghz"], "peak_at_measured_clock": round(pk, 1),
                    "frac_at_measured_clock": round(per_gpu / pk, 4), "clock_source": traffic_src})
        if world > 1:
            out["config"].update(exchange_fields(m))
            # which halo transport the timed region used, and why when it is not the requested
            # one: a scaling run on the slower fallback transport must not pass unnoticed
            out["config"]["halo_transport"] = m["transport"] if a.backend == "nccl" else "gloo"
            out["config"]["transport_fallback"] = m["fallback"]
        if cold is not None:
            out["config"]["cold_first_call"] = cold
        cm = []
        if c3 is not None:
            cm.append(config_entry(c3, f"{c3['W']}x{c3['H']} random torus board (seed "
                                       f"{a.seed}), {c3['steps']} turns (BASELINE configs[2])",
                                   world, parallelism(a, world, c3)))
        if c2 is not None:
            cm.append(config_entry(c2, f"{c2['W']}x{c2['H']} random torus board (seed 1), "
                                       f"{c2['steps']} turns + the final AliveCellsCount "
                                       f"snapshot (BASELINE configs[1])",
                                   world, parallelism(a, world, c2)))
        if c1 is not None:
            cm.append(c1)
        if cm:
            out["configs_measured"] = cm
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(W, a.seed, a.cpu_turns, a.cpu_cores)
            if not a.no_c1:
                share, aff, omp = cpu_share()
                out["cpu_baseline"]["c1"] = cpu_c1(f"host CPU share {share} of an affinity "
                                                   f"mask of {aff}")
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
