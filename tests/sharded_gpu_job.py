"""One rank of the frame-sharded front-end on the GPU (configs[2]), for
tests/test_sharded_gpu.py: `python tests/sharded_gpu_job.py OUT.npz` with RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT set. Every rank runs slam_framework_amd.sharded.ShardedFrontend -- the
object bench.py times -- on cuda:0 over a gloo process group (two ranks on one GPU: RCCL needs
one GPU per rank, so the gather goes through host memory here); rank 0 writes what it gathered
to OUT.npz (per field, [world * F, bytes])."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# the job's shape, shared with the test (world-2: 2 contexts of 3 frames per rank, 4 owned frames)
SEED, RENDERS, BATCH, STREAMS, STEPS = 1000, 9, 6, 2, 3


def main(out):
    import torch
    import torch.distributed as dist
    from slam_framework_amd import synthetic as S
    from slam_framework_amd.sharded import ShardedFrontend

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    Ls, Rs = S.layered_sequence(SEED, RENDERS)
    job = ShardedFrontend(Ls, Rs, S.KITTI_CAM, BATCH, dev, streams=STREAMS, inflight=2,
                          rank=rank, world=world, gather=True, host_gather=True)
    for _ in range(STEPS):
        job.step()
    job.sync()
    got = job.gathered()
    if rank == 0:
        slot = (job.gat.k - 1) % len(job.gat.send)
        np.savez(out, **{k: job.gat.field(slot, k).numpy() for k in job.fields()},
                 frames=np.array([d["frame"] for d in got]), lo_hi=np.array([job.lo, job.hi]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
