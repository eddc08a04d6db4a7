"""World-size-2 gloo test of the frame-sharded multi-rank path (runs on CPU)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from slam_framework_amd import dist as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = D.shard(1000, rank, world)
    elapsed = 0.25 * (rank + 1)
    mx = D.max_over_ranks(elapsed)
    summ = D.gather_summary([lo, hi, rank])
    dist.barrier()
    q.put((rank, lo, hi, mx, summ.tolist()))
    dist.destroy_process_group()


def test_shard_balanced():
    for n in (0, 1, 7, 1000, 4541):
        for w in (1, 2, 3, 8):
            rs = [D.shard(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_two_rank_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, lo0, hi0, mx0, s0), (r1, lo1, hi1, mx1, s1) = res
    assert (lo0, hi0, lo1, hi1) == (0, 500, 500, 1000)
    assert mx0 == mx1 == 0.5
    assert s0 == s1 == [[0, 500, 0], [500, 1000, 1]]


def _job_worker(rank, world, port, n_owned, q):
    import sharded_job
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = sharded_job.run_job(n_owned)
    dist.barrier()
    q.put((rank, out))
    dist.destroy_process_group()


def test_shard_with_halo():
    # frames 1..8 over 2 ranks: rank 0 computes 0..4 (owns 1..4), rank 1 computes 4..8
    assert D.shard_with_halo(8, 0, 2, first=1) == (0, 1, 5)
    assert D.shard_with_halo(8, 1, 2, first=1) == (4, 5, 9)
    assert D.shard_with_halo(10, 0, 3) == (0, 0, 4)
    for n, w in ((4541, 8), (17, 3)):
        rs = [D.shard_with_halo(n, r, w, first=1) for r in range(w)]
        assert all(s == lo - 1 for s, lo, _ in rs)


def test_sharded_job_gathers_sequence_order(oracle):
    """World-2 gloo run of the sharded front-end (shard + halo + FrameGather): rank 0's gathered
    per-frame results are those of a world-1 run, byte for byte, in sequence order."""
    import sharded_job
    n_owned = 6
    ref = sharded_job.run_job(n_owned)  # world 1, no process group
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_job_worker, args=(r, 2, port, n_owned, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] is None
    got = res[0]
    assert set(got) == set(ref)
    for k in ref:
        assert got[k].shape == ref[k].shape == (n_owned, sharded_job.fields()[k])
        assert np.array_equal(got[k], ref[k]), k
    nm = got["nmatches"].view(np.int32).reshape(-1)
    assert (nm > 0).all(), "every owned frame (incl. each shard's first) must match its t-1"
