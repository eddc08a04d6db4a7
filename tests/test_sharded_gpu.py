"""configs[2] on the GPU: the frame-sharded front-end job through its
device half -- slamgpu_pack_frame_records_device -> FrameGather -> unpack_frame_record -- with
the object bench.py times (slam_framework_amd.sharded.ShardedFrontend).

* world 1, two contexts per step (each one's first frame the halo of its second), two batches in
  flight, three steps: every frame rank 0 gathered equals the oracle byte for byte -- left/right
  keypoints and descriptors, u_right / depth, the frame-to-frame map-point ids and match count
  (frame.cpp:61-111, tracker.cpp:756-824, orb_matcher.cpp:1312-1453) -- and the bench's own
  gather self-check (ShardedFrontend.check_gather) passes.
* world 1 over RCCL (a "nccl" process group in a child process): FrameGather's dist.gather
  branch, five steps over two slots, every gathered frame against the oracle.
* world 2 (two processes on cuda:0, gloo through host memory, since RCCL needs a GPU per rank):
  the shards + halos gathered to rank 0 reassemble exactly the world-1 job's gathered bytes."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import sharded_gpu_job as J
from slam_framework_amd import slamgpu as G
from slam_framework_amd.sharded import render_of
from slam_framework_amd import synthetic as S

pytestmark = pytest.mark.gpu
CAM = S.KITTI_CAM
COLS, ROWS = S.KITTI_COLS, S.KITTI_ROWS


@pytest.fixture(scope="module")
def world1(gpu_lib):
    """The world-1 job over the same 8 owned frames (1..8) as the world-2 run: 2 contexts of 5."""
    import torch
    from slam_framework_amd.sharded import ShardedFrontend
    dev = torch.device("cuda", 0)
    Ls, Rs = S.layered_sequence(J.SEED, J.RENDERS)
    with torch.cuda.stream(torch.cuda.Stream(device=dev)):
        job = ShardedFrontend(Ls, Rs, CAM, 10, dev, streams=2, inflight=2, gather=True)
        last = [job.step() for _ in range(J.STEPS)][-1]
        job.sync()
    return job, last, Ls, Rs


def _check_vs_oracle(oracle, got, gframe, Bs, poses, D, Ls, Rs, parts=None):
    """Every gathered frame against the oracle: left/right keypoints and descriptors, u_right /
    depth, and the frame-to-frame search against f - 1 (poses[b] of the batch slot b owning f).
    The search needs `parts`, the device buffers of a job that ran in this process (its VO
    queries are checked and searched by the oracle); without them only the extraction and
    stereo fields are checked."""
    t = oracle.tables()
    g = oracle.grid_geom(COLS, ROWS)
    cache = {}

    def orc(f):
        if f not in cache:
            kl, dl, pl = oracle.extract(t, Ls[render_of(f, D)], True)
            kr, dr, pr = oracle.extract(t, Rs[render_of(f, D)], True)
            ur, depth, _ = oracle.stereo(t, kl, dl, kr, dr, pl, pr, CAM[0], CAM[4])
            cache[f] = (kl, dl, kr, dr, ur, depth)
        return cache[f]

    for d in got:
        f = d["frame"]
        kl, dl, kr, dr, ur, depth = orc(f)
        assert d["kps_left"].tobytes() == kl.tobytes(), f"frame {f} left keypoints"
        assert d["kps_right"].tobytes() == kr.tobytes(), f"frame {f} right keypoints"
        assert np.array_equal(d["desc_left"], dl) and np.array_equal(d["desc_right"], dr)
        assert d["u_right"].tobytes() == ur.tobytes() and d["depth"].tobytes() == depth.tobytes()
        if parts is None:   # the search is checked against a job of this process instead
            continue
        # the batch slot that owns frame f (f also appears as the next context's halo slot 0)
        b = [int(x) for x in np.nonzero(gframe == f)[0] if x % Bs != 0][0]
        si, i = divmod(b, Bs)
        pt = parts[si]
        qs, qc = pt["qs"].cpu().numpy(), pt["qc"].cpu().numpy()
        q = pt["q"].cpu().numpy().view(G.F2F_QUERY_DTYPE)[qs[i]:qs[i] + qc[i]]
        pkl, pdl, _, _, _, pdepth = orc(f - 1)
        idx = np.nonzero(pdepth > 0)[0]
        assert np.array_equal(q["mp_id"], idx) and np.array_equal(q["desc"], pdl[idx])
        n_last = len(pkl)
        last_mp = np.full(n_last, -1, np.int32)
        last_mp[idx] = idx
        xyz = np.zeros((n_last, 3), np.float32)
        xyz[idx] = q["xyz"]
        mdesc = np.zeros((n_last, 32), np.uint8)
        mdesc[idx] = q["desc"]
        nobs = np.zeros(n_last, np.int32)
        nobs[idx] = 1
        p = poses[b]
        mp_o = np.full(len(kl), -1, np.int32)
        nm_o = oracle.search_frame(t, g, kl, dl, ur, mp_o, pkl, last_mp,
                                   np.zeros(n_last, np.uint8), xyz, mdesc, nobs,
                                   p["Rcw"].reshape(3, 3), p["tcw"], float(p["tlc_z"]),
                                   float(p["baseline"]), CAM, 7.0, 0, 1)
        assert d["nmatches"] == nm_o > 300, f"frame {f}: {d['nmatches']} vs {nm_o}"
        np.testing.assert_array_equal(d["map_point"], mp_o)


def test_world1_gather_matches_oracle(oracle, world1):
    job, last, Ls, Rs = world1
    got = job.gathered()
    assert [d["frame"] for d in got] == list(range(1, 9))
    _, _, parts = job.groups[last]
    _check_vs_oracle(oracle, got, job.gframe, job.Bs, job.poses, job.D, Ls, Rs, parts)
    info = job.check_gather()
    assert info["identical"] and info["frames_checked_vs_rank0"] == 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_world2_shards_reassemble_world1(world1, tmp_path):
    job, _, _, _ = world1
    out = str(tmp_path / "rank0.npz")
    rcs = _run_ranks(out, 2, "gloo")
    assert rcs == [0, 0], rcs
    w2 = np.load(out)
    assert w2["frames"].tolist() == list(range(1, 9))
    slot = (job.gat.k - 1) % len(job.gat.send)
    for k in job.fields():
        ref = job.gat.field(slot, k).cpu().numpy()
        assert w2[k].shape == ref.shape, k
        if k == "frontend":   # records are compared up to their padding
            for j in range(len(ref)):
                a, b = G.unpack_frame_record(w2[k][j], job.kc), G.unpack_frame_record(ref[j], job.kc)
                assert all(a[n].tobytes() == b[n].tobytes() for n in a), f"frame {j + 1}"
        elif k == "map_point":
            recs = job.gat.field(slot, "frontend").cpu().numpy()
            nkl = [len(G.unpack_frame_record(r, job.kc)["kps_left"]) for r in recs]
            for j, n in enumerate(nkl):
                assert np.array_equal(w2[k][j].view(np.int32)[:n], ref[j].view(np.int32)[:n]), j
        else:
            assert np.array_equal(w2[k], ref), k


def _run_ranks(out, world, backend):
    port = _free_port()
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sharded_gpu_job.py")
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", script, out, backend], env=env))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=100))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    return rcs


def test_world1_rccl_gather(oracle, world1, tmp_path):
    """FrameGather's collective branch on RCCL: a world-1 "nccl" process group (created before
    any other GPU work, TCP store on 127.0.0.1), ShardedFrontend(gather=True, inflight=2) for 5
    steps over 2 gather slots, so steps 3-5 reuse a slot whose async dist.gather Work was waited
    on the compute stream. Every frame rank 0 gathered equals the oracle (extraction, stereo) and
    the world-1 local-copy job, whose frame-to-frame search the oracle checked, byte for byte."""
    job, _, Ls, Rs = world1
    out = str(tmp_path / "rccl.npz")
    assert _run_ranks(out, 1, "nccl") == [0]
    w = np.load(out)
    assert int(w["steps"]) == J.NCCL_STEPS and int(w["checked"]) == 8
    assert w["frames"].tolist() == list(range(1, 9))
    assert np.array_equal(w["gframe"], job.gframe)
    recs = [G.unpack_frame_record(r, job.kc) for r in w["frontend"]]
    mps, nms = w["map_point"].view(np.int32), w["nmatches"].view(np.int32).reshape(-1)
    got = []
    for j, d in enumerate(recs):
        d["map_point"] = mps[j][:len(d["kps_left"])].copy()
        d["nmatches"] = int(nms[j])
        d["frame"] = j + 1
        got.append(d)
    _check_vs_oracle(oracle, got, job.gframe, job.Bs, job.poses, job.D, Ls, Rs)
    ref = {d["frame"]: d for d in job.gathered()}
    from slam_framework_amd.sharded import frame_results_equal
    for d in got:
        assert frame_results_equal(d, ref[d["frame"]]), f"frame {d['frame']}"


def test_bench_shape_gather_matches_oracle(oracle, gpu_lib):
    """configs[2] at the bench's own shape: one context of 256 frames (255 owned), two batches in
    flight, three steps with the gather on (what bench.py times with SLAMGPU_BENCH_GATHER=1 or at
    world > 1): the bench's self-check holds for 64 frames spread over the batch, and frames at the
    start, middle and end of it equal the oracle (extraction, stereo, frame-to-frame search)."""
    import torch
    from slam_framework_amd.sharded import ShardedFrontend
    dev = torch.device("cuda", 0)
    Ls, Rs = S.layered_sequence(J.SEED, 16)
    with torch.cuda.stream(torch.cuda.Stream(device=dev)):
        job = ShardedFrontend(Ls, Rs, CAM, 256, dev, streams=1, inflight=2, gather=True)
        last = [job.step() for _ in range(3)][-1]
        job.sync()
    got = job.gathered()
    assert [d["frame"] for d in got] == list(range(1, 256))
    info = job.check_gather()
    assert info["identical"] and info["frames_checked_vs_rank0"] >= 15
    _, _, parts = job.groups[last]
    # frames at the start, at the turns of the back-and-forth sequence (frames 15, 16: renders
    # 15 -> 14; frames 30, 31: renders 0 -> 1), in the middle and at the end
    pick = [got[i] for i in (0, 1, 14, 15, 29, 30, 126, 200, 254)]
    _check_vs_oracle(oracle, pick, job.gframe, job.Bs, job.poses, job.D, Ls, Rs, parts)


def test_bench_two_ranks_gloo():
    """`bench.py --gpus 2` end to end on one GPU: spawn_ranks starts two rank
    processes before any GPU call, each runs the timed job on its shard with the gather staged
    through host memory (gloo), max_over_ranks / gather_summary run over the group, and rank 0
    prints ONE JSON line whose n_gpus / parallelism describe the 2-rank job and whose gather check
    found the other rank's frames identical to its own. Only the RCCL transport itself is left to
    the driver's multi-GPU runs."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--steps", "2", "--warmup", "1", "--batch", "32", "--no-cpu-baseline",
           "--no-optimizer", "--no-bow", "--no-latency"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=150,
                       env=dict(os.environ, PYTHONUNBUFFERED="1"))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = __import__("json").loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["dist_backend"] == "gloo" and "x2" in d["config"]["parallelism"]
    assert d["config"]["frames_per_gpu_per_step"] == 31
    g = d["gather"]
    assert g["identical"] is True and g["frames_checked_vs_rank0"] > 0, g
    assert len(d["per_rank_matches_per_step"]) == 2 and min(d["per_rank_matches_per_step"]) > 0
    assert d["value"] > 0 and d["roofline"]["avg_launch_us"] > 0
