"""One rank of the frame-sharded front-end on the GPU (configs[2]), for
tests/test_sharded_gpu.py: `python tests/sharded_gpu_job.py OUT.npz [gloo|nccl]` with RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT set. Every rank runs
slam_framework_amd.sharded.ShardedFrontend -- the object bench.py times -- on cuda:0; rank 0 writes
what it gathered to OUT.npz (per field, [world * F, bytes]).

* gloo (default): two ranks on one GPU, the gather goes through host memory (RCCL needs one GPU
  per rank).
* nccl: one rank, an RCCL process group created before any other GPU work, the job's gather on
  the device (dist.gather, async, two slots: five steps make slot reuse wait on a live Work)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# the job's shape, shared with the test (world-2: 2 contexts of 3 frames per rank, 4 owned frames)
SEED, RENDERS, BATCH, STREAMS, STEPS = 1000, 9, 6, 2, 3
# the RCCL world-1 job: the shape of the test's world-1 fixture (2 contexts of 5, 8 owned frames)
NCCL_BATCH, NCCL_STEPS = 10, 5


def main(out, backend="gloo"):
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    if backend == "gloo":
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from slam_framework_amd import synthetic as S
    from slam_framework_amd.sharded import ShardedFrontend

    nccl = backend == "nccl"
    Ls, Rs = S.layered_sequence(SEED, RENDERS)
    job = ShardedFrontend(Ls, Rs, S.KITTI_CAM, NCCL_BATCH if nccl else BATCH, dev,
                          streams=STREAMS, inflight=2, rank=rank, world=world, gather=True,
                          host_gather=not nccl)
    assert job.gat.active and len(job.gat.send) == 2
    for _ in range(NCCL_STEPS if nccl else STEPS):
        job.step()
    job.sync()
    got = job.gathered()
    info = job.check_gather()
    if rank == 0:
        slot = (job.gat.k - 1) % len(job.gat.send)
        np.savez(out, **{k: job.gat.field(slot, k).cpu().numpy() for k in job.fields()},
                 frames=np.array([d["frame"] for d in got]), lo_hi=np.array([job.lo, job.hi]),
                 gframe=job.gframe, steps=np.array(job.gat.k),
                 checked=np.array(info["frames_checked_vs_rank0"]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "gloo")
