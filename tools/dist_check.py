#!/usr/bin/env python3
"""Multi-rank strip rehearsal on ONE GPU: torchrun N ranks, every rank's engine on
cuda:0, halos exchanged through gol.distributed.DistStrip over gloo (staged via host
memory), final board gathered to rank 0 and compared with the CPU oracle.
`--backend nccl` runs the RCCL path proper (zero-copy board views, batch_isend_irecv);
on a one-GPU box that is world size 1, where rank 0 exchanges with itself.
Used by tests/test_gpu_distributed.py."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "conway-s-gol-distributed_amd"), ROOT):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--height", type=int, default=1000)
    ap.add_argument("--turns", type=int, default=53)
    ap.add_argument("--halo", type=int, default=6)
    ap.add_argument("--tpl", type=int, default=4)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--backend", choices=("gloo", "nccl"), default="gloo")
    ap.add_argument("--copy", action="store_true", help="export/import copies, not zero-copy")
    ap.add_argument("--transport", choices=("rccl", "torch"), default="rccl",
                    help="nccl backend: direct RCCL on the engine stream, or batch_isend_irecv")
    ap.add_argument("--digest", default="",
                    help="check against tests/golden/large_digests.json[KEY] (size, height, "
                         "seed and turns from there) instead of running the CPU oracle")
    ap.add_argument("--overlap", action="store_true",
                    help="direct RCCL: exchange on its own stream, overlapped with the first "
                         "launch's interior rows (gol_step_overlap)")
    ap.add_argument("--window-every", type=int, default=0,
                    help="step in blocks of this many turns, each opened by DistStrip.start_window "
                         "(an exchange at any turn, as bench.py's timed region starts)")
    a = ap.parse_args()
    want_digest = None
    if a.digest:
        import json
        d = json.load(open(os.path.join(ROOT, "tests", "golden", "large_digests.json")))[a.digest]
        a.size, a.height, a.seed, a.turns = d["width"], d["height"], d["seed"], d["turns"]
        want_digest = d["sha256"]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if a.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    gdev = dev if a.backend == "nccl" else "cpu"
    import gol
    from gol.distributed import DistStrip, EngineStrip, make_engine_strip
    eng = make_engine_strip(a.size, a.height, rank, world, a.halo, 0, turns_per_launch=a.tpl)
    eng.fill_random(a.seed)
    comm = None
    if a.backend == "nccl" and a.transport == "rccl":
        from gol.rccl import RcclComm
        comm = RcclComm(rank, world, dev)
    ds = DistStrip(EngineStrip(eng, dev, zero_copy=not a.copy), rank, world,
                   stage_on_host=a.backend == "gloo", rccl=comm, overlap=a.overlap)
    if a.window_every > 0:
        left = a.turns
        while left:
            n = min(left, a.window_every)
            ds.start_window()
            ds.step(n)
            left -= n
    else:
        ds.step(a.turns)
    split = gol.strip_split(a.height, world)
    maxr = max(r for _, r in split)
    mine = torch.zeros((maxr, eng.words_per_row), dtype=torch.int64)   # gather: equal sizes
    mine[: eng.rows] = torch.from_numpy(eng.read_packed().view(np.int64))
    mine = mine.to(gdev)
    parts = [torch.zeros((maxr, eng.words_per_row), dtype=torch.int64, device=gdev)
             for _ in split]
    if rank == 0:
        dist.gather(mine, parts, dst=0)
        got = np.concatenate([p.cpu().numpy()[:r]
                              for p, (_, r) in zip(parts, split)]).view(np.uint64)
        if want_digest:
            import hashlib
            ok = hashlib.sha256(got.tobytes()).hexdigest() == want_digest
        else:
            from oracle import oracle as O
            want = O.bit_run(O.gen_random(a.seed, a.size, a.height), a.size, a.turns)
            ok = np.array_equal(got, want)
        print(f"dist_check backend={a.backend} transport={a.transport if comm else 'torch'} world={world} halo={eng.halo} "
              f"exchanges={ds.exchanges} tpl={a.tpl} layout={ds.strip.layout} "
              f"overlap={ds.overlap} equal={ok}",
              flush=True)
        if not ok:
            sys.exit(1)
    else:
        dist.gather(mine, dst=0)
    if comm is not None:
        comm.close()
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    except Exception:
        import traceback
        print(f"RANK {os.environ.get('RANK')} FAILED:\n" + traceback.format_exc(), flush=True)
        raise
