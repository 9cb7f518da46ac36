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
