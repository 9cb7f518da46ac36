"""The N-rank strip path (gol/distributed.py, as bench.py uses it for N > 1) run as real
torchrun processes sharing the one GPU of the test box, over gloo with host-staged
halos (RCCL refuses two ranks on one device; the exchange code is the same)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dist_check(world, args, port):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.join(ROOT, "tools", "dist_check.py")] + [str(x) for x in args]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stdout[-6000:] + "\n----- stderr -----\n" + "\n".join(
        ln for ln in p.stderr.splitlines() if "amdgpu.ids" not in ln and "socket.cpp" not in ln)[:6000]
    assert "equal=True" in p.stdout
    return p.stdout


@pytest.mark.parametrize("world,halo,tpl,copy", [(2, 6, 4, False), (2, 5, 1, False),
                                                 (3, 5, 1, True), (3, 7, 6, False),
                                                 (4, 8, 8, False), (2, 8, 8, True)])
def test_torchrun_strips_one_gpu(world, halo, tpl, copy):
    """gloo, host-staged; zero-copy board views (default) and the export/import copies."""
    _dist_check(world, ["--halo", halo, "--tpl", tpl] + (["--copy"] if copy else []),
                29500 + world + (10 if copy else 0))


@pytest.mark.parametrize("halo,tpl,copy,transport", [
    (8, 8, False, "rccl"), (16, 8, False, "rccl"), (5, 1, False, "rccl"), (6, 6, False, "rccl"),
    (8, 8, True, "rccl"), (8, 8, False, "torch"), (5, 1, True, "torch")])
def test_rccl_self_exchange(halo, tpl, copy, transport):
    """The RCCL exchange proper (backend nccl, device buffers) at world size 1: rank 0 is
    its own up and down neighbour, so its halos come back over RCCL from its own boundary
    rows -- the N = 1 torus.  Transports: direct RCCL send/recv on the engine's stream
    (gol.rccl, the bench default) and torch batch_isend_irecv; zero-copy board views
    (interleaved layout at tpl > 1) and the copy path.  Bit-exact against the oracle
    after 53 turns (several exchanges)."""
    port = 29530 + halo + (50 if copy else 0) + (100 if transport == "torch" else 0)
    out = _dist_check(1, ["--backend", "nccl", "--halo", halo, "--tpl", tpl, "--height", 640,
                          "--transport", transport] + (["--copy"] if copy else []), port)
    assert "backend=nccl" in out and f"transport={transport}" in out
    if not copy:
        assert f"layout={1 if tpl > 1 else 0}" in out


@pytest.mark.parametrize("halo,tpl,height", [(8, 8, 640), (16, 8, 640), (5, 1, 640),
                                             (6, 6, 640), (40, 8, 64), (40, 8, 12),
                                             (128, 8, 300)])
def test_rccl_self_exchange_overlapped(halo, tpl, height):
    """The overlapped exchange (gol_stream_wait + direct RCCL on a stream of its own +
    gol_step_overlap): the first launch after each exchange runs its interior rows at once
    and the rows next to the halos after the receives.  Self-exchange at world size 1,
    bit-exact against the oracle; the 12-row case has no interior rows at all, and
    (128, 300) exchanges 128-row halos as the bench does."""
    port = 29700 + halo + tpl
    out = _dist_check(1, ["--backend", "nccl", "--halo", halo, "--tpl", tpl, "--height", height,
                          "--transport", "rccl", "--overlap"], port)
    assert "overlap=True" in out


@pytest.mark.parametrize("overlap", [False, True])
def test_rccl_self_exchange_65536(overlap):
    """BASELINE C4 / C5 through the bench's own N > 1 path (DistStrip, direct RCCL, 128-row
    halos, k-turn launches) at full size: 65536^2 seed 3, 1000 turns, world size 1 (the
    rank is its own ring neighbour), against the oracle digest."""
    out = _dist_check(1, ["--backend", "nccl", "--transport", "rccl", "--halo", 128, "--tpl", 0,
                          "--digest", "65536x65536_seed3_t1000"] + (["--overlap"] if overlap else []),
                      29800 + int(overlap))
    assert "world=1 halo=128 exchanges=7" in out and f"overlap={overlap}" in out


@pytest.mark.parametrize("halo,tpl,every,digest", [(20, 8, 7, ""), (20, 0, 13, ""),
                                                   (128, 0, 20, "65536x65536_seed3_t1000")])
def test_rccl_self_exchange_windows(halo, tpl, every, digest):
    """The bench's N > 1 timed-region form (round 6): blocks of turns each opened by
    DistStrip.start_window -- an exchange at any turn, its board pointers looked up before the
    window (the direct RCCL path) -- over RCCL at world size 1, against the oracle; the last
    case runs 65536^2 x 1000 in 20-turn windows on 128-row halos against the digest."""
    args = ["--backend", "nccl", "--transport", "rccl", "--halo", halo, "--tpl", tpl,
            "--window-every", every]
    args += ["--digest", digest] if digest else ["--height", 640]
    out = _dist_check(1, args, 29760 + every + halo)
    assert "backend=nccl" in out


def test_halo_buffers_zero_copy_torus():
    """gol_halo_buffers: the four views are the strip's boundary and halo rows in the
    current board; copying send_bottom -> recv_top and send_top -> recv_bottom on the
    engine's stream (a strip that is its own neighbour) and stepping reproduces the
    torus exactly, across layouts (tpl 8 = interleaved, 1 = standard)."""
    import numpy as np
    import torch
    for p in (os.path.join(ROOT, "conway-s-gol-distributed_amd"), ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    from gol.distributed import EngineStrip, make_engine_strip
    from oracle import oracle as O
    dev = torch.device("cuda", 0)
    for tpl, halo in ((8, 16), (1, 3), (6, 12)):
        W, H, turns = 1536, 300, 41
        eng = make_engine_strip(W, H, 0, 1, halo, 0, turns_per_launch=tpl)
        es = EngineStrip(eng, dev)
        eng.fill_random(11)
        with es.stream_context():
            left = turns
            while left:
                if es.halo_valid == 0:
                    st, sb = es.export_rows()
                    es.import_rows(sb, st)
                n = min(left, es.halo_valid)
                es.step(n)
                left -= n
        got = eng.read_packed()
        eng.close()
        want = O.bit_run(O.gen_random(11, W, H), W, turns)
        assert np.array_equal(got, want), (tpl, halo)
        assert es.layout == (1 if tpl > 1 else 0)


REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
            "roofline", "valu_roofline", "cpu_baseline")


def _bench_line(stdout):
    import json
    lines = [ln for ln in stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, stdout[-3000:]
    return json.loads(lines[0])


def test_bench_contract_one_gpu():
    """bench.py's single JSON line (driver contract) at a small size, CPU baseline included."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--size", "4096",
                        "--steps", "64", "--warmup", "8", "--cpu-turns", "1",
                        "--c3-size", "2048", "--c3-turns", "96"],
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _bench_line(p.stdout)
    for k in REQUIRED:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 64 and d["warmup"] == 8 and d["value"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["peak"] == 8000.0 and r["launches"] >= 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3 and 0 < r["frac"] <= 1
    assert d["k1_equivalent"]["achieved"] >= r["achieved"]
    v = d["valu_roofline"]
    # the roof is the 52-cycle issue model; the measured stream is a separate reference point
    assert abs(v["peak"] - 193583.3) < 1 and 0 < v["frac"] <= 1
    assert abs(v["algorithmic_ceiling"]["peak"] - 144010.4) < 1
    assert d["config"]["create_ms"] > 0
    cold = d["config"]["cold_first_call"]
    assert cold["value"] > 0 and cold["create_ms"] > 0
    c3 = d["configs_measured"][0]
    assert c3["value"] > 0 and "2048x2048" in c3["workload"] and c3["create_ms"] > 0
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    assert f"{cb['cores']} OpenMP threads" in cb["sample"]


@pytest.mark.parametrize("size,steps,halo,exchanges,c3", [(65536, 20, None, 1, 16384),
                                                         (4096, 64, 16, 4, 2048)])
def test_bench_torchrun_two_ranks_gloo(size, steps, halo, exchanges, c3):
    """The N > 1 bench path (strips, halo exchange every `halo` turns, max-over-ranks wall
    time) as torchrun ranks sharing the one GPU; gloo stands in for RCCL.  Round-5 verdict
    #1: the headline's timed region holds the run's exchanges -- with the driver's 20 turns
    the default halo is 20, and the region is one exchange plus one 20-turn window -- with
    each rank's exchange time, and the no-exchange rate only as a labelled secondary figure.
    configs[2] at 2 GPUs (16384^2 as 2 strips, 128-row halos) runs its pinned shape, and its
    entry carries the PMC traffic of that exact launch (the launch shape of a whole window,
    not of the run's last partial one)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={29611 + steps}",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--size", str(size), "--steps",
           str(steps), "--warmup", "5", "--backend", "gloo", "--c3-size", str(c3),
           "--c3-turns", "300" if c3 == 16384 else "40"] + (["--halo", str(halo)] if halo else [])
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert p.returncode == 0, p.stderr[-3000:]
    d = _bench_line(p.stdout)
    for k in REQUIRED:
        assert k in d, k
    c = d["config"]
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["value"] > 0
    assert c["halo"] == (halo or 20) and f"halo {halo or 20}" in c["parallelism"]
    assert c["exchanges_timed"] == exchanges >= 1
    xs = c["exchange_us_per_rank"]
    assert [x["rank"] for x in xs] == [0, 1]
    assert all(x["count"] == exchanges and x["mean_us"] > 0 for x in xs), xs
    comp = c["compute_only"]
    assert comp["exchanges_timed"] == 0 and comp["value"] > 0
    assert comp["turns"] == min(steps, halo or 20)
    assert c["create_ms"] > 0 and d["cpu_baseline"] is None and "cold_first_call" not in c
    e = d["configs_measured"][0]
    assert e["exchanges_timed"] >= 1 and len(e["exchange_us_per_rank"]) == 2
    if c3 == 16384:
        assert e["halo"] == 128 and e["exchanges_timed"] == 3
        assert e["shape_source"].startswith("pinned") and e["temporal_blocking_k"] == 32
        assert e["launch_shape"]["buffer_rows"] == 8448
        assert e["traffic"] and e["traffic"] > 0 and e["valu_inflation"] > 1
    if size == 65536:
        # the driver's 20-turn command: one whole 20-turn window on the pinned 65536 x 32808
        # strip
        assert c["shape_source"].startswith("pinned") and c["launch_shape"]["buffer_rows"] == 32808
        assert d["roofline"]["traffic"] and d["valu_roofline"]["valu_inflation"] > 1


def test_rccl_comm_world2_bootstrap():
    """gol.rccl.RcclComm at world size 2 (round-4 verdict weak #1): the unique id is broadcast
    over a gloo group and both ranks call ncclCommInitRank.  The two ranks share the test
    box's one GPU, which RCCL refuses with ncclInvalidUsage ("Duplicate GPU detected") -- a
    check that runs only after the bootstrap has connected both ranks to the root address
    inside the id.  A truncated id (the round-4 bug) fails in the bootstrap instead."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29661",
           os.path.join(ROOT, "tools", "rccl_bootstrap_check.py")]
    env = dict(os.environ, OMP_NUM_THREADS="2", NCCL_DEBUG="WARN")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=env)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    for r in (0, 1):
        assert (f"rank {r}: INIT_DUP" in out) or (f"rank {r}: INIT_OK" in out), out[-4000:]
    if "INIT_DUP" in out:
        assert "Duplicate GPU" in out, out[-4000:]


def test_rccl_comm_init_deadline():
    """Round-5 verdict #6: a communicator whose bootstrap cannot complete ends on every rank
    within GOL_RCCL_INIT_TIMEOUT_S instead of hanging.  Rank 1 joins with a wrong root port
    (tools/rccl_bootstrap_check.py --bad-port); rank 0, the root, waits for it until the
    deadline, aborts and reports INIT_TIMEOUT; rank 1 times out or fails to connect."""
    import re
    import time
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29663",
           os.path.join(ROOT, "tools", "rccl_bootstrap_check.py"), "--bad-port"]
    env = dict(os.environ, OMP_NUM_THREADS="2", NCCL_DEBUG="WARN", GOL_RCCL_INIT_TIMEOUT_S="8")
    t0 = time.monotonic()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=150, env=env)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "rank 0: INIT_TIMEOUT" in out, out[-4000:]
    assert ("rank 1: INIT_TIMEOUT" in out) or ("rank 1: INIT_FAIL" in out), out[-4000:]
    for r in (0, 1):
        m = re.search(rf"rank {r}: INIT_\w+ after ([0-9.]+) s", out)
        assert m and float(m.group(1)) < 8 + 15, out[-4000:]
    assert time.monotonic() - t0 < 140
