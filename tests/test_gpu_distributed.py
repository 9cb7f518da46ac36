"""The N-rank strip path (gol/distributed.py, as bench.py uses it for N > 1) run as real
torchrun processes sharing the one GPU of the test box, over gloo with host-staged
halos (RCCL refuses two ranks on one device; the exchange code is the same)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world,halo,tpl", [(2, 6, 4), (2, 5, 1), (3, 5, 1), (3, 7, 6), (4, 8, 8)])
def test_torchrun_strips_one_gpu(world, halo, tpl):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1", f"--master-port={29500 + world}",
           os.path.join(ROOT, "tools", "dist_check.py"), "--halo", str(halo), "--tpl", str(tpl)]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stdout[-6000:] + "\n----- stderr -----\n" + "\n".join(
        ln for ln in p.stderr.splitlines() if "amdgpu.ids" not in ln and "socket.cpp" not in ln)[:6000]
    assert "equal=True" in p.stdout


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
                        "--steps", "64", "--warmup", "8", "--cpu-turns", "1"],
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _bench_line(p.stdout)
    for k in REQUIRED:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 64 and d["warmup"] == 8 and d["value"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["peak"] == 8000.0 and r["launches"] >= 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert d["cpu_baseline"]["kind"] == "port" and d["cpu_baseline"]["value"] > 0


def test_bench_torchrun_two_ranks_gloo():
    """The N > 1 bench path (strips, halo exchange every `halo` turns, max-over-ranks wall
    time) as torchrun ranks sharing the one GPU; gloo stands in for RCCL."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29611", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--size", "4096", "--steps", "64", "--warmup", "8", "--halo", "16",
           "--backend", "gloo"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert p.returncode == 0, p.stderr[-3000:]
    d = _bench_line(p.stdout)
    for k in REQUIRED:
        assert k in d, k
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["value"] > 0
    assert "halo 16" in d["config"]["parallelism"] and d["cpu_baseline"] is None
