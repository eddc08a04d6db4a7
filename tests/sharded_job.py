"""The frame-sharded front-end job of SURVEY.md section 8(e) with the oracle as the per-frame
compute (test infrastructure): shard one contiguous stereo sequence over the ranks, recompute
each shard's halo frame (t-1) for its first frame-to-frame search, and gather every owned frame's
results to rank 0 with slam_framework_amd.dist.FrameGather -- the same packing and gather
bench.py runs over RCCL, here over gloo on CPU tensors.

Per frame: left+right keypoints (padded to KC), descriptors, counts, stereo u_right/depth, the
frame-to-frame map-point assignment against frame t-1's stereo points (Tracker's visual-odometry
points, tracker.cpp:695-753 + SearchByProjection(CurrentFrame, LastFrame, 7), orb_matcher.cpp:
1312-1453) and its match count -- what Frame's stereo ctor (frame.cpp:61-111) and the tracker's
motion-model search produce."""
import numpy as np
import torch

import oracle_lib as O
import scenario
from slam_framework_amd import dist as D
from slam_framework_amd import synthetic as S

COLS, ROWS, NFEAT, KC = 320, 240, 500, 640
CAM = S.KITTI_CAM


def fields(kc=KC):
    return {"kps": 2 * kc * 28, "desc": 2 * kc * 32, "nkps": 8, "u_right": kc * 4,
            "depth": kc * 4, "map_point": kc * 4, "nmatches": 4}


def frame_results(L, R, frames, t):
    """Oracle results of sequence frames `frames` (consecutive); frame f's search reads f-1's
    results when f-1 is among them (the halo), else it has no last frame."""
    g = O.grid_geom(COLS, ROWS)
    out, prev = {}, None
    for f in frames:
        kl, dl, pl = O.extract(t, L[f], True)
        kr, dr, pr = O.extract(t, R[f], True)
        ur, depth, _ = O.stereo(t, kl, dl, kr, dr, pl, pr, CAM[0], CAM[4])
        mp = np.full(len(kl), -1, np.int32)
        nm = 0
        if prev is not None:
            q, lmp, lout, xyz, md, nobs = scenario.vo_queries(prev[0], prev[1], prev[2], f - 1)
            p = scenario.pose(f)
            nm = O.search_frame(t, g, kl, dl, ur, mp, prev[0], lmp, lout, xyz, md, nobs,
                                p["Rcw"][0].reshape(3, 3), p["tcw"][0], 0.0,
                                float(p["baseline"][0]), CAM, 7.0, 0, 1)
        rec = {k: np.zeros(v, np.uint8) for k, v in fields().items()}
        for v, (k_, d_) in enumerate(((kl, dl), (kr, dr))):
            assert len(k_) <= KC
            rec["kps"][v * KC * 28:v * KC * 28 + len(k_) * 28] = k_.view(np.uint8)
            rec["desc"][v * KC * 32:v * KC * 32 + d_.size] = d_.reshape(-1)
        rec["nkps"][:] = np.array([len(kl), len(kr)], np.int32).view(np.uint8)
        rec["u_right"][:len(kl) * 4] = ur.view(np.uint8)
        rec["depth"][:len(kl) * 4] = depth.view(np.uint8)
        rec["map_point"][:len(kl) * 4] = mp.view(np.uint8)
        rec["nmatches"][:] = np.array([nm], np.int32).view(np.uint8)
        out[f] = rec
        prev = (kl, dl, depth)
    return out


def run_job(n_owned, seed=77):
    """Runs on every rank of the (possibly absent) process group; returns rank 0's gathered
    {field: [n_owned, bytes]} arrays (None elsewhere). Frames 1..n_owned of the sequence are
    sharded; frame 0 is the sequence's first frame, the halo of rank 0."""
    rank, world = (torch.distributed.get_rank(), torch.distributed.get_world_size()) \
        if torch.distributed.is_initialized() else (0, 1)
    L, R = S.sequence(seed, n_owned + 1, COLS, ROWS)
    start, lo, hi = D.shard_with_halo(n_owned, rank, world, first=1)
    res = frame_results(L, R, range(start, hi), O.tables(nfeatures=NFEAT))
    g = D.FrameGather(fields(), hi - lo)
    g.pack({k: torch.from_numpy(np.concatenate([res[f][k] for f in range(lo, hi)]))
            for k in fields()})
    s = g.start(async_op=False)
    if rank != 0:
        return None
    return {k: g.field(s, k).numpy().copy() for k in fields()}
