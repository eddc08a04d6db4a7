"""Frame sharding, result gather and timing helpers for the multi-GPU path (one process per GPU).

Stereo frames are independent units of the front-end: one sequence is
cut into contiguous shards, one per rank; each rank also recomputes the frame before its shard
(the halo) because the tracker's motion-model search pairs frame t with t-1. The only data-path
collective is the gather of every owned frame's results to rank 0 (FrameGather); the rest are the
bench's barrier and max-over-ranks timing -- RCCL ("nccl") on GPUs, gloo in tests.
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


def collective_device(device=None):
    """Where a small collective's tensor lives: the process group's device for RCCL ("nccl"),
    host memory for gloo (the CPU backend; bench.py --dist-backend gloo, the CPU tests)."""
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "gloo":
        return torch.device("cpu")
    return device


def max_over_ranks(x: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=collective_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_summary(values, device=None):
    """All ranks' small int64 summaries, stacked [world, len(values)] (on every rank)."""
    t = torch.tensor(list(values), dtype=torch.int64, device=collective_device(device))
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return t[None].cpu()
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return torch.stack(out).cpu()


def shard_with_halo(n_frames: int, rank: int, world: int, first: int = 0, halo: int = 1):
    """Contiguous shard of the sequence frames [first, first + n_frames) for one rank, plus the
    `halo` frames before it that its first frames' frame-to-frame search reads (SURVEY.md
    section 8(e): Tracker's motion-model search pairs frame t with t-1, tracker.cpp:756-824).

    Returns (start, lo, hi): the rank computes frames [start, hi) and owns [lo, hi); the halo
    frames [start, lo) are recomputed here and owned (and gathered) by the previous rank."""
    a, b = shard(n_frames, rank, world)
    lo, hi = first + a, first + b
    return max(0, lo - halo), lo, hi


class FrameGather:
    """Gathers per-frame results of a frame-sharded job to rank 0 (RCCL over xGMI on GPUs, gloo
    on CPU): each rank packs the frames it owns, field by field, into one contiguous send slab;
    one `dist.gather` lands the slabs rank by rank on rank 0, so field `name` of the whole job is
    `recv[:, off:off + frames * bytes].view(world * frames, bytes)` -- sequence order, since the
    shards are contiguous and rank-ordered.

    fields: {name: bytes per frame}; frames: frames each rank owns per gather (equal on every
    rank; the last shard of a ragged split is padded by its caller). `slots` send/receive buffers
    rotate so that gather k can still be in flight while the compute of k+1 packs the next slot
    (gather k+slots waits for it on the compute stream, never on the host).

    host_staging: the process group's backend is a CPU one (gloo) while the producers write
    device slots -- start() copies the slot to host memory and gathers there, synchronously."""

    def __init__(self, fields: dict, frames: int, device=None, slots: int = 2,
                 host_staging: bool = False):
        self.fields = dict(fields)
        self.frames = frames
        self.offsets, off = {}, 0
        for k, bpf in self.fields.items():
            self.offsets[k] = off
            off += (frames * bpf + 255) // 256 * 256  # 256-B aligned slabs
        self.nbytes = off
        self.active = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size() if self.active else 1
        self.rank = dist.get_rank() if self.active else 0
        self.device = device
        self.host_staging = host_staging
        self.send = [torch.empty(self.nbytes, dtype=torch.uint8, device=device)
                     for _ in range(slots)]
        rdev = "cpu" if host_staging else device
        self.recv = [torch.empty((self.world, self.nbytes), dtype=torch.uint8, device=rdev)
                     if self.rank == 0 else None for _ in range(slots)]
        self.work = [None] * slots
        self.k = 0

    def _slot(self):
        return self.k % len(self.send)

    def begin(self):
        """Claim the next send slot: the gather that last used it must be done reading it (the
        current stream waits for it on the device; the host does not block)."""
        s = self._slot()
        if self.work[s] is not None:
            self.work[s].wait()
            self.work[s] = None
        return s

    def slab(self, name: str):
        """The claimed send slot's bytes of field `name`, [frames, bytes per frame] uint8, for a
        producer to write into directly."""
        off, bpf = self.offsets[name], self.fields[name]
        return self.send[self._slot()][off:off + self.frames * bpf].view(self.frames, bpf)

    def pack(self, arrays: dict):
        """begin() + copy this rank's owned frames into the slot. arrays[name] is a uint8 tensor
        (any shape) of exactly frames * bytes-per-frame bytes, frames in sequence order."""
        s = self.begin()
        for k, bpf in self.fields.items():
            a = arrays[k].reshape(-1)
            assert a.numel() == self.frames * bpf and a.dtype == torch.uint8, (k, a.numel())
            self.slab(k).view(-1).copy_(a)
        return s

    def start(self, async_op: bool = True):
        """Gather the packed slot to rank 0; returns the slot index."""
        s = self._slot()
        if self.host_staging:
            host = self.send[s].cpu()   # waits for the producers on the current stream
            glist = list(self.recv[s].unbind(0)) if self.rank == 0 else None
            if self.world > 1:
                dist.gather(host, glist, dst=0)
            else:
                glist[0].copy_(host)
        elif self.active:
            # any initialised process group takes the collective, world 1 included, so the
            # RCCL gather and the Work.wait() ordering that slot reuse relies on are exercised
            # by a one-GPU run (tests/test_sharded_gpu.py::test_world1_rccl_gather)
            glist = list(self.recv[s].unbind(0)) if self.rank == 0 else None
            self.work[s] = dist.gather(self.send[s], glist, dst=0, async_op=async_op)
            if not async_op:
                self.work[s] = None
        else:   # no process group: a local copy
            self.recv[s][0].copy_(self.send[s])
        self.k += 1
        return s

    def wait_all(self):
        for i, w in enumerate(self.work):
            if w is not None:
                w.wait()
                self.work[i] = None

    def field(self, slot: int, name: str):
        """Rank 0: field `name` of every gathered frame, [world * frames, bytes] uint8 (sequence
        order). None on other ranks."""
        if self.rank != 0:
            return None
        off, bpf = self.offsets[name], self.fields[name]
        return self.recv[slot][:, off:off + self.frames * bpf].reshape(self.world * self.frames,
                                                                        bpf)
