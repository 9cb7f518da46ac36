"""torchrun helper for tests/test_gpu_distributed.py::test_rccl_comm_world2_bootstrap: two
ranks on the test box's one GPU build gol.rccl.RcclComm at world size 2, the unique id
broadcast over a gloo group.  RCCL refuses two ranks on one device ("Duplicate GPU
detected", ncclInvalidUsage = 5), but only after its bootstrap has connected every rank to
the root address carried in the unique id -- so INIT_DUP (or INIT_OK, should RCCL accept the
pair) proves the id arrived intact; a damaged id fails earlier, in the bootstrap's connect
(a system or remote error)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conway-s-gol-distributed_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gol.rccl import RcclComm  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    try:
        c = RcclComm(rank, world, torch.device("cuda", 0))
        c.close()
        print(f"rank {rank}: INIT_OK", flush=True)
    except RuntimeError as e:
        msg = str(e)
        tag = "INIT_DUP" if "RCCL error 5" in msg else "INIT_FAIL"
        print(f"rank {rank}: {tag} {msg}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
