"""One rank's share of the frame-sharded front-end job (SURVEY.md section 8(e), configs[2]).

ONE contiguous stereo sequence is cut into contiguous shards, one per rank: rank r owns the
frames [r*F + 1, (r+1)*F + 1) (F = frames completed per rank per step) and recomputes frame r*F,
the halo its first frame-to-frame search reads (Tracker's motion-model search pairs frame t with
t-1, tracker.cpp:756-824). Inside a rank, the batch of B frames is split over `streams` contexts
(each with its own HIP stream; its first frame is the halo of its second), and `inflight` groups
of such contexts take consecutive steps in turn, so up to `inflight` batches are in flight.

One step per context: the stereo Frame ctor's extract L+R + ComputeStereoMatches + grid
(slamgpu_frontend_device, frame.cpp:61-111), the last frame's stereo points as visual-odometry
map points (slamgpu_make_vo_queries_device, tracker.cpp:695-753) and
SearchByProjection(CurrentFrame, LastFrame, th=7) (slamgpu_search_by_projection_frame_device,
orb_matcher.cpp:1312-1453). With a gather, every owned frame's results (keypoints + descriptors
of both views, u_right / depth, map-point ids, match count) are packed on the device
(slamgpu_pack_frame_records_device) into a FrameGather slot and gathered to rank 0 on the
collective's stream (RCCL over xGMI; over gloo through host memory in CPU-collective tests).

bench.py times `step()`; tests/test_sharded_gpu.py runs the same object and compares what rank 0
gathers with the oracle frame by frame.
"""
from __future__ import annotations

import numpy as np
import torch

from . import dist as SD
from . import slamgpu as G
from . import synthetic as S

PITCH = 1280  # device row pitch of the resident input images (>= 1241, 256-B multiple)


def render_of(g, D):
    """Render of global frame g in a sequence of D renders played back and forth (0, 1, ..,
    D - 1, D - 2, .., 1, 0, 1, ..): consecutive frames are always neighbouring renders, so every
    frame-to-frame search sees the sequence's one-render motion (a cyclic order would pair render
    D - 1 with render 0 once per D frames: a jump with few matches)."""
    if D <= 1:
        return 0
    u = int(g) % (2 * (D - 1))
    return u if u < D else 2 * (D - 1) - u


def sequence_poses(gframe, D, cam):
    """F2F pose records of the global frames `gframe` of a D-render layered sequence (frame g is
    render render_of(g, D); its last frame is g - 1)."""
    poses = np.zeros(len(gframe), G.F2F_POSE_DTYPE)
    for f, g in enumerate(gframe):
        t, tl = render_of(g, D), render_of(int(g) - 1, D)
        Rf, tf = S.layered_pose(t)
        poses["Rcw"][f] = Rf.astype(np.float32).reshape(-1)
        poses["tcw"][f] = tf.astype(np.float32)
        poses["tlc_z"][f] = np.float32((S.rotation(tl) @ (S.camera_center(t) -
                                                          S.camera_center(tl)))[2])
    poses["baseline"] = np.float32(cam[4]) / np.float32(cam[0])
    poses["th"] = 7.0
    poses["check_ori"] = 1
    return poses


class ShardedFrontend:
    """Ls, Rs: the D distinct renders of the sequence (frame g = render_of(g, D)), uploaded once so
    the inputs are resident in HBM before any timed step. batch: stereo frames per rank per step
    (split into `streams` parts of >= 2 frames). gather: pack + gather every step's owned frames
    to rank 0 (FrameGather; host_gather stages the slots through host memory for a CPU (gloo)
    process group)."""

    def __init__(self, Ls, Rs, cam, batch, device, streams=1, inflight=2, rank=0, world=1,
                 gather=False, host_gather=False, nfeatures=2000, scale_factor=1.2, nlevels=8,
                 ini_th=20, min_th=7):
        cols, rows = Ls.shape[2], Ls.shape[1]
        assert Ls.shape == Rs.shape and cols <= PITCH
        self.cam, self.device, self.rank, self.world = cam, device, rank, world
        NS = max(1, streams)
        Bs = batch // NS
        if Bs < 2 or Bs * NS != batch:
            raise ValueError("batch must split into `streams` parts of >= 2 frames")
        self.NS, self.Bs, self.B = NS, Bs, batch
        self.F = F = NS * (Bs - 1)      # frames this rank completes (owns) per step
        self.D = D = len(Ls)
        first, lo, hi = SD.shard_with_halo(world * F, rank, world, first=1)
        assert hi - lo == F and first == lo - 1
        self.lo, self.hi = lo, hi
        # context si computes global frames lo - 1 + si*(Bs-1) + [0, Bs): its slot 0 is the halo
        # of its slot 1 (the previous context's last frame, or the previous rank's for si = 0)
        self.gframe = np.array([first + si * (Bs - 1) + i for si in range(NS) for i in range(Bs)])
        self.host_l = np.zeros((batch, rows, PITCH), np.uint8)
        self.host_r = np.zeros((batch, rows, PITCH), np.uint8)
        for f in range(batch):
            self.host_l[f, :, :cols] = Ls[render_of(self.gframe[f], D)]
            self.host_r[f, :, :cols] = Rs[render_of(self.gframe[f], D)]
        self.d_l = torch.from_numpy(self.host_l).to(device)
        self.d_r = torch.from_numpy(self.host_r).to(device)
        self.stride = rows * PITCH
        self.poses = sequence_poses(self.gframe, D, cam)
        self.d_poses = torch.from_numpy(self.poses.view(np.uint8).copy()).to(device)
        self.INF = max(1, inflight)
        self.groups = []
        pbytes = G.F2F_POSE_DTYPE.itemsize
        for _ in range(self.INF):
            ctxs = [G.Context(cols, rows, nfeatures, scale_factor, nlevels, ini_th, min_th,
                              max_frames=Bs, device=device.index) for _ in range(NS)]
            streams_ = [torch.cuda.Stream(device=device) for _ in range(NS)]
            kc = ctxs[0].kp_cap
            parts = []
            for si in range(NS):
                e = lambda n, dt: torch.empty(n, dtype=dt, device=device)
                parts.append({"q": e(Bs * kc * G.F2F_QUERY_DTYPE.itemsize, torch.uint8),
                              "qs": e(Bs, torch.int32), "qc": e(Bs, torch.int32),
                              "mp": e(Bs * kc, torch.int32), "blk": e(Bs * kc, torch.uint8),
                              "nm": e(Bs, torch.int32),
                              "poses": self.d_poses[si * Bs * pbytes:(si + 1) * Bs * pbytes]})
            self.groups.append((ctxs, streams_, parts))
        self.kc = self.groups[0][0][0].kp_cap
        self.record_bytes = self.groups[0][0][0].record_bytes
        self.gat = None
        if gather:
            self.gat = SD.FrameGather(self.fields(), F, device, host_staging=host_gather)
        self.k = 0

    def fields(self):
        return {"frontend": self.record_bytes, "map_point": self.kc * 4, "nmatches": 4}

    @property
    def contexts(self):
        """The contexts of in-flight group 0 (the one `step(group=0)` runs)."""
        return self.groups[0][0]

    @property
    def parts(self):
        return self.groups[0][2]

    def step(self, group=None):
        """Enqueue one step (no host synchronisation): the group's contexts on their streams,
        forked from and joined back into the group's first stream, then the gather."""
        gi = self.k % self.INF if group is None else group
        self.k += 1
        ctxs, streams_, parts = self.groups[gi]
        main = streams_[0]
        NS, Bs, kc, gat = self.NS, self.Bs, self.kc, self.gat
        if gat is not None:
            with torch.cuda.stream(main):
                gat.begin()
        for si in range(NS):
            st = streams_[si]
            if si:
                st.wait_stream(main)
            with torch.cuda.stream(st):
                c, pt, h = ctxs[si], parts[si], st.cuda_stream
                off = si * Bs * self.stride
                c.frontend_device(int(self.d_l.data_ptr()) + off, int(self.d_r.data_ptr()) + off,
                                  self.stride, PITCH, Bs, self.cam, h)
                c.make_vo_queries_device(pt["poses"], 1, pt["q"], pt["qs"], pt["qc"], Bs, h)
                pt["mp"].fill_(-1)
                pt["blk"].zero_()
                c.search_by_projection_frame_device(pt["q"], Bs * kc, pt["qs"], pt["qc"], kc,
                                                    pt["poses"], pt["mp"], pt["blk"], kc,
                                                    pt["nm"], Bs, h)
                if gat is not None:   # owned frames = slots 1..Bs-1 of this context
                    o = si * (Bs - 1)
                    c.pack_frame_records_device(1, Bs - 1, gat.slab("frontend")[o:o + Bs - 1], h)
                    gat.slab("map_point")[o:o + Bs - 1].view(-1).copy_(
                        pt["mp"][kc:].view(torch.uint8))
                    gat.slab("nmatches")[o:o + Bs - 1].view(-1).copy_(
                        pt["nm"][1:].view(torch.uint8))
        for si in range(1, NS):
            main.wait_stream(streams_[si])
        if gat is not None:
            with torch.cuda.stream(main):
                gat.start()
        return gi

    def sync(self):
        if self.gat is not None:
            self.gat.wait_all()
        torch.cuda.synchronize(self.device)
        for ctxs, _, _ in self.groups:
            for c in ctxs:
                c.sync()

    def gathered(self):
        """Rank 0, after sync(): the last gathered slot as one dict per owned frame of the whole
        job, in sequence order (global frames 1 .. world*F): the unpacked frontend record plus
        `map_point` (trimmed to the left keypoint count) and `nmatches`. None elsewhere."""
        if self.gat is None or self.rank != 0:
            return None
        slot = (self.gat.k - 1) % len(self.gat.send)
        recs = self.gat.field(slot, "frontend").cpu().numpy()
        mps = self.gat.field(slot, "map_point").cpu().numpy().view(np.int32)
        nms = self.gat.field(slot, "nmatches").cpu().numpy().view(np.int32).reshape(-1)
        out = []
        for j in range(len(recs)):
            d = G.unpack_frame_record(recs[j], self.kc)
            d["map_point"] = mps[j][:len(d["kps_left"])].copy()
            d["nmatches"] = int(nms[j])
            d["frame"] = j + 1
            out.append(d)
        return out

    def own_results(self, group=0):
        """This rank's own owned-frame results of in-flight group `group` (after sync()), keyed
        by global frame: the same dict as gathered() -- packed again on the device, then
        unpacked."""
        ctxs, _, parts = self.groups[group]
        Bs, kc = self.Bs, self.kc
        own = {}
        for si, c in enumerate(ctxs):
            rec = torch.empty((Bs - 1, c.record_bytes), dtype=torch.uint8, device=self.device)
            c.pack_frame_records_device(1, Bs - 1, rec, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize(self.device)
            rec = rec.cpu().numpy()
            mp = parts[si]["mp"].cpu().numpy().reshape(Bs, kc)
            nm = parts[si]["nm"].cpu().numpy()
            for i in range(1, Bs):
                d = G.unpack_frame_record(rec[i - 1], kc)
                d["map_point"] = mp[i][:len(d["kps_left"])].copy()
                d["nmatches"] = int(nm[i])
                d["frame"] = int(self.gframe[si * Bs + i])
                own[d["frame"]] = d
        return own

    def check_gather(self):
        """Rank 0, after sync(): every gathered frame must equal, byte for byte, rank 0's own
        result for the same render pair (frames play D renders back and forth: the frontend
        output depends only on the render, the frame-to-frame search only on (t-1, t)). Up to 64
        frames spread over the other ranks' shards (at world 1: rank 0's own) are checked."""
        got = self.gathered()
        if got is None:
            return None
        own = {}
        for g, d in self.own_results(0).items():
            own.setdefault((render_of(g, self.D), render_of(g - 1, self.D)), d)
        F, world = self.F, self.world
        j0 = F if world > 1 else 0
        checked = 0
        for j in range(j0, world * F, max(1, (world * F - j0) // 64)):
            g = j + 1
            b = own.get((render_of(g, self.D), render_of(g - 1, self.D)))
            if b is None:   # rank 0 owns fewer frames than the sequence has render pairs
                continue
            a = got[j]
            if not frame_results_equal(a, b):
                raise AssertionError(f"gathered frame {g} differs from rank 0's own result")
            checked += 1
        return {"bytes_per_rank_per_step": self.gat.nbytes, "frames_per_rank_per_step": F,
                "record_bytes_per_frame": int(self.record_bytes) + 4 * self.kc + 4,
                "frames_checked_vs_rank0": checked, "identical": True}


def frame_results_equal(a, b):
    keys = ("kps_left", "kps_right", "desc_left", "desc_right", "u_right", "depth", "map_point")
    return all(a[k].tobytes() == b[k].tobytes() for k in keys) and a["nmatches"] == b["nmatches"]
