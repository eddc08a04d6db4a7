"""Frame sharding and timing helpers for the multi-GPU path (one process per GPU).

Stereo frames are independent units of the front-end, so a job shards frames across ranks with
no data-path collective: each rank extracts and matches its own frames.
The only collectives are the bench's barrier, the max-over-ranks of the elapsed time, and an
optional gather of per-rank result summaries to rank 0 -- RCCL ("nccl") on GPUs, gloo in tests.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(n_units: int, rank: int, world: int):
    """Contiguous unit range [lo, hi) of this rank (balanced to within one unit)."""
    q, r = divmod(n_units, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def max_over_ranks(x: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_summary(values, device=None):
    """All ranks' small int64 summaries, stacked [world, len(values)] (on every rank)."""
    t = torch.tensor(list(values), dtype=torch.int64, device=device)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return t[None].cpu()
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return torch.stack(out).cpu()
