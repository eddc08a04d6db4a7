"""World-size-2 gloo test of the frame-sharded multi-rank path (runs on CPU)."""
import os
import socket

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
