"""The batched, device-resident path bench.py times, against the oracle -- including the launch
shapes the bench itself uses.

slamgpu_frontend_device (extract L+R + stereo + grid for a batch), slamgpu_make_vo_queries_device
(Tracker::UpdateLastFrame's stereo points as frame-to-frame queries, tracker.cpp:695-753) and
slamgpu_search_by_projection_frame_device (orb_matcher.cpp:1312-1453), issued twice back to back
on one stream with no host synchronisation in between, as bench.py issues its steps. Each checked
frame of the batch must equal the oracle's per-frame result: keypoints, descriptors, stereo, and
the frame-to-frame map-point assignment computed from the queries the device built.

Batch sizes: 5 frames (10 images: natural block order), 4 and 8 frames (image counts that are
multiples of 8, so pyr_down / blur7 / fast_cells / orient_desc use the XCD-aware (image, block)
remap of device_math.h xcd_image_block, as the bench's 512-image launches do), 64 frames with 8
spread frames checked, two contexts on two HIP streams (bench.py --streams 2), and uniform-noise
frames whose FAST candidate counts overflow the octree's LDS kernel into octree_global."""
import numpy as np
import pytest

from slam_framework_amd import synthetic as S

pytestmark = pytest.mark.gpu
CAM = S.KITTI_CAM
COLS, ROWS, PITCH = S.KITTI_COLS, S.KITTI_ROWS, 1280


def _poses(G, B, t_of, layered=False):
    poses = np.zeros(B, G.F2F_POSE_DTYPE)
    for f in range(B):
        if layered:  # rotation + forward motion (synthetic.layered_pose); tlc_z vs frame f - 1
            t, tl = t_of(f), t_of(f - 1) if f else t_of(f)
            R, tc = S.layered_pose(t)
            poses["Rcw"][f] = R.astype(np.float32).reshape(-1)
            poses["tcw"][f] = tc.astype(np.float32)
            poses["tlc_z"][f] = np.float32((S.rotation(tl) @ (S.camera_center(t) -
                                                              S.camera_center(tl)))[2])
        else:
            poses["Rcw"][f] = S.rotation(t_of(f)).astype(np.float32).reshape(-1)
    poses["baseline"] = np.float32(CAM[4]) / np.float32(CAM[0])
    poses["th"] = 7.0
    poses["check_ori"] = 1
    return poses


class _Part:
    """One context + its matcher buffers over Bs consecutive frames of the batch."""

    def __init__(self, G, torch, dev, Bs, poses):
        self.ctx = G.Context(COLS, ROWS, 2000, 1.2, 8, 20, 7, max_frames=Bs)
        kc = self.kc = self.ctx.kp_cap
        self.Bs = Bs
        e = lambda n, dt: torch.empty(n, dtype=dt, device=dev)
        self.d_poses = torch.from_numpy(poses.view(np.uint8).copy()).to(dev)
        self.q = e(Bs * kc * G.F2F_QUERY_DTYPE.itemsize, torch.uint8)
        self.qs, self.qc = e(Bs, torch.int32), e(Bs, torch.int32)
        self.mp, self.blk, self.nm = e(Bs * kc, torch.int32), e(Bs * kc, torch.uint8), e(Bs, torch.int32)

    def step(self, d_l, d_r, off, stream):
        Bs, kc, s = self.Bs, self.kc, stream.cuda_stream
        self.ctx.frontend_device(int(d_l.data_ptr()) + off, int(d_r.data_ptr()) + off, ROWS * PITCH,
                                 PITCH, Bs, CAM, s)
        self.ctx.make_vo_queries_device(self.d_poses, 1, self.q, self.qs, self.qc, Bs, s)
        self.mp.fill_(-1)
        self.blk.zero_()
        self.ctx.search_by_projection_frame_device(self.q, Bs * kc, self.qs, self.qc, kc,
                                                   self.d_poses, self.mp, self.blk, kc, self.nm,
                                                   Bs, s)


def run_batch(G, L, R, t_of, n_parts=1, layered=False):
    """Two back-to-back device steps over the batch, split over n_parts contexts on their own
    streams (each part's first frame is the halo of its second, as in bench.py)."""
    import torch
    B = len(L)
    dev = torch.device("cuda", 0)
    hl = np.zeros((B, ROWS, PITCH), np.uint8)
    hr = np.zeros((B, ROWS, PITCH), np.uint8)
    hl[:, :, :COLS] = L
    hr[:, :, :COLS] = R
    poses = _poses(G, B, t_of, layered)
    Bs = B // n_parts
    main = torch.cuda.Stream(device=dev)
    streams = [main] + [torch.cuda.Stream(device=dev) for _ in range(n_parts - 1)]
    with torch.cuda.stream(main):
        d_l = torch.from_numpy(hl).to(dev)
        d_r = torch.from_numpy(hr).to(dev)
        parts = [_Part(G, torch, dev, Bs, poses[i * Bs:(i + 1) * Bs]) for i in range(n_parts)]
        for _ in range(2):
            for i, p in enumerate(parts):
                if i:
                    streams[i].wait_stream(main)
                with torch.cuda.stream(streams[i]):
                    p.step(d_l, d_r, i * Bs * ROWS * PITCH, streams[i])
            for i in range(1, n_parts):
                main.wait_stream(streams[i])
    main.synchronize()
    for p in parts:
        p.ctx.sync()
    return parts, poses


def check_frames(G, oracle, parts, poses, L, R, frames):
    """Compare the listed batch frames with the oracle (frame f's search against frame f-1, the
    oracle's own result for f-1; a part's first frame has no search)."""
    t = oracle.tables()
    g = oracle.grid_geom(COLS, ROWS)
    Bs = parts[0].Bs
    total = 0
    cache = {}

    def orc(f):
        if f not in cache:
            kl, dl, pl = oracle.extract(t, L[f], True)
            kr, dr, pr = oracle.extract(t, R[f], True)
            ur, depth, _ = oracle.stereo(t, kl, dl, kr, dr, pl, pr, CAM[0], CAM[4])
            cache[f] = (kl, dl, kr, dr, ur, depth)
        return cache[f]

    for f in frames:
        p, i = parts[f // Bs], f % Bs
        kc = p.kc
        kl, dl, kr, dr, ur, depth = orc(f)
        gkl, gdl = p.ctx.keypoints(2 * i)
        gkr, gdr = p.ctx.keypoints(2 * i + 1)
        assert gkl.tobytes() == kl.tobytes() and gkr.tobytes() == kr.tobytes(), f"frame {f}"
        assert np.array_equal(gdl, dl) and np.array_equal(gdr, dr), f"frame {f}"
        gur, gdepth = p.ctx.stereo(i)
        assert gur.tobytes() == ur.tobytes() and gdepth.tobytes() == depth.tobytes(), f"frame {f}"
        qs, qc = p.qs.cpu().numpy(), p.qc.cpu().numpy()
        nm_all = p.nm.cpu().numpy()
        if i == 0:
            assert qc[0] == 0 and nm_all[0] == 0
            continue
        pkl, pdl, _, _, _, pdepth = orc(f - 1)
        q = p.q.cpu().numpy().view(G.F2F_QUERY_DTYPE)[qs[i]:qs[i] + qc[i]]
        idx = np.nonzero(pdepth > 0)[0]
        # queries: last-frame stereo points in keypoint order
        assert np.array_equal(q["mp_id"], idx)
        assert np.array_equal(q["desc"], pdl[idx])
        assert np.array_equal(q["last_octave"], pkl["octave"][idx])
        assert q["last_angle"].tobytes() == pkl["angle"][idx].tobytes()
        assert (q["blocks"] == 1).all()
        # matcher on the device's queries (map point id = last-frame keypoint index)
        n_last = len(pkl)
        last_mp = np.full(n_last, -1, np.int32)
        last_mp[idx] = idx
        xyz = np.zeros((n_last, 3), np.float32)
        xyz[idx] = q["xyz"]
        mdesc = np.zeros((n_last, 32), np.uint8)
        mdesc[idx] = q["desc"]
        nobs = np.zeros(n_last, np.int32)
        nobs[idx] = 1
        mp_o = np.full(len(kl), -1, np.int32)
        nm_o = oracle.search_frame(t, g, kl, dl, ur, mp_o, pkl, last_mp,
                                   np.zeros(n_last, np.uint8), xyz, mdesc, nobs,
                                   poses["Rcw"][f].reshape(3, 3), poses["tcw"][f],
                                   float(poses["tlc_z"][f]), float(poses["baseline"][f]), CAM,
                                   7.0, 0, 1)
        assert nm_all[i] == nm_o, f"frame {f}"
        np.testing.assert_array_equal(p.mp.cpu().numpy()[i * kc:i * kc + len(kl)], mp_o)
        total += nm_o
    return total


@pytest.mark.parametrize("B", [5, 4, 8])
def test_batched_device_path_matches_oracle(oracle, gpu_lib, B):
    L, R = S.sequence(3000, B)
    parts, poses = run_batch(gpu_lib, L, R, lambda f: f)
    total = check_frames(gpu_lib, oracle, parts, poses, L, R, range(B))
    assert total > 100, "scenario should produce real frame-to-frame matches"


def test_layered_scene_with_forward_motion(oracle, gpu_lib):
    """The bench's scene (synthetic.layered_sequence: ~50 % stereo yield, turning + 0.3 m/frame
    forward, so the queries' map points are unprojected with a translation) in an 8-frame batch."""
    B = 8
    L, R = S.layered_sequence(1000, B)
    parts, poses = run_batch(gpu_lib, L, R, lambda f: f, layered=True)
    total = check_frames(gpu_lib, oracle, parts, poses, L, R, range(B))
    assert total > 500 * (B - 1), "the layered scene should give ~700-800 matches per frame"


def test_batch64_spread_frames(oracle, gpu_lib):
    """64 frames (128-image launches, XCD remap) of an 8-render cyclic sequence, as bench.py
    cycles its renders; 8 frames spread over the batch checked (incl. the wrap 7 -> 0)."""
    D, B = 8, 64
    Ls, Rs = S.sequence(3100, D)
    L, R = Ls[np.arange(B) % D], Rs[np.arange(B) % D]
    parts, poses = run_batch(gpu_lib, L, R, lambda f: f % D)
    total = check_frames(gpu_lib, oracle, parts, poses, L, R, [0, 8, 9, 18, 27, 36, 45, 54, 63])
    assert total > 100


def test_two_contexts_two_streams(oracle, gpu_lib):
    """bench.py --streams 2: two contexts, each on its own HIP stream, overlapping."""
    B = 8
    L, R = S.sequence(3200, B)
    parts, poses = run_batch(gpu_lib, L, R, lambda f: f, n_parts=2)
    check_frames(gpu_lib, oracle, parts, poses, L, R, range(B))


def test_noise_frames_take_global_octree(oracle, gpu_lib):
    """Uniform-noise frames: FAST candidates far beyond the octree LDS kernel's key capacity, so
    their levels are redone by octree_global; mixed into a 4-frame (XCD-remapped) batch."""
    L, R = S.sequence(3300, 4)
    rng = np.random.default_rng(9)
    L[1] = rng.integers(0, 256, L[1].shape, dtype=np.uint8)
    R[1] = L[1]
    L[2] = rng.integers(0, 256, L[2].shape, dtype=np.uint8)
    R[2] = np.roll(L[2], -7, axis=1)
    parts, poses = run_batch(gpu_lib, L, R, lambda f: f)
    ctx = parts[0].ctx
    for img in (2, 4):  # the noise images produce many more level-0 candidates than fit in LDS
        assert len(ctx.debug_level_keys(img, 0, 0)) > 20000
    check_frames(gpu_lib, oracle, parts, poses, L, R, range(4))


def test_level0_fast_fork_off_identical(gpu_lib):
    """slamgpu_set_extract_fork(0) (level 0's FAST after the pyramid on the call's stream, as
    bench.py's alone breakdown pass runs it) gives the same keypoints, descriptors and stereo as
    the default side-stream fork, frame for frame, on a 9-frame (18-image) batch."""
    import torch
    B = 9
    L = np.zeros((B, ROWS, PITCH), np.uint8)
    R = np.zeros((B, ROWS, PITCH), np.uint8)
    for f in range(B):
        L[f, :, :COLS], R[f, :, :COLS] = S.stereo_pair(6000 + f)
    dev = torch.device("cuda", 0)
    d_l, d_r = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    torch.cuda.synchronize()
    ctx = gpu_lib.Context(COLS, ROWS, 2000, 1.2, 8, 20, 7, max_frames=B)
    out = []
    for fork in (True, False):
        ctx.set_extract_fork(fork)
        ctx.frontend_device(d_l, d_r, ROWS * PITCH, PITCH, B, CAM)
        ctx.sync()
        out.append([(ctx.keypoints(i), ctx.stereo(i // 2) if i % 2 == 0 else None)
                    for i in range(2 * B)])
    ctx.set_extract_fork(True)
    for i, ((a, sa), (b, sb)) in enumerate(zip(*out)):
        for f in a[0].dtype.names:
            np.testing.assert_array_equal(a[0][f], b[0][f], err_msg=f"image {i} field {f}")
        np.testing.assert_array_equal(a[1], b[1], err_msg=f"image {i} descriptors")
        if sa is not None:
            for x, y in zip(sa, sb):
                np.testing.assert_array_equal(x, y, err_msg=f"frame {i // 2} stereo")
