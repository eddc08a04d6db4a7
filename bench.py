#!/usr/bin/env python3
"""bench.py -- stereo frames/s of the ORB extract + match hot path on MI355X.

One step = one pass of the hot path over one batch of B synthetic 1241x376 stereo frames that are
already resident in HBM (BASELINE.json configs[1]): ORBextractor::Compute on both views
(2000 features, 8 levels), Frame::ComputeStereoMatches, the 64x48 keypoint grid, the previous
frame's stereo points as visual-odometry map points, and OrbMatcher::SearchByProjection(
CurrentFrame, LastFrame, th=7) -- the tracker's per-frame motion-model search. Frame 0 of a batch
is the halo frame of frame 1's search, so a step completes B-1 frames.

Multi-GPU (configs[2]; `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`,
or `python bench.py --gpus N`, which starts the N ranks itself before touching the GPU): ONE
contiguous synthetic sequence is sharded over the ranks -- rank r owns frames
[r*F + 1, (r+1)*F + 1) (F = frames completed per rank per step) and recomputes frame r*F, the halo
its first frame-to-frame search reads. Inside every timed step each rank packs its owned frames'
results (keypoints + descriptors of both views, stereo u_right/depth, frame-to-frame map-point ids
and match counts; slamgpu_pack_frame_records_device) and RCCL-gathers them to rank 0 on the
collective's own stream, double-buffered so the gather of step k overlaps the compute of k+1
(slam_framework_amd.dist.FrameGather). Weak scaling: F is fixed per rank.

Prints ONE JSON line on rank 0 (driver contract), with `roofline` for the dominant kernel
(HIP-event timed inside the timed region) and `cpu_baseline` (the oracle/ restatement on host
cores, rank 0 only). Per-kernel breakdowns go to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

# Algorithmic HBM bytes per launch unit of each kernel (DESIGN.md "Roofline model"); unit = one
# image, except stereo/grid/search kernels whose unit is one stereo frame.
LEVEL_PX = None  # filled from the context geometry


TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


# bench.py's timing names -> kernel symbols where they differ (the octree timing is the per-image
# kernel; octree_kernel is its global-memory fallback; the batches' pyramid levels run
# pyr_ring_kernel, the single-frame call pyr_down_kernel)
KERNEL_SYMBOL = {"octree": ("octree_img",), "octree_global": ("octree",),
                 "pyr_down": ("pyr_down", "pyr_ring", "pyr_cascade")}


def _symbol_matches(sym, kernel):
    return sym.split("<")[0].replace("_kernel", "") in KERNEL_SYMBOL.get(kernel, (kernel,))


# Sustained VALU issue rate of one MI355X, measured (tools/valu_rates.hip, profiles/r5d_valu_rates.txt):
# at 8 waves per SIMD, chains of v_dot4 / v_dot2 / v_alignbit / v_perm / v_lerp_u8 / v_bfe /
# v_pk_* / v_cvt issue at 0.44-0.48 of the nominal one-wave64-instruction-per-2-cycles peak
# (256 CUs x 4 SIMD x 2.4 GHz / 2), v_add / v_xor / v_bitop3 / f32 add, mul, fma at 0.70-0.83.
# A kernel's VALU roof is the rate its own instruction mix sustains: the harmonic mean of the
# class rates weighted by its ISA's class histogram (tools/isa_mix.py -> profiles/isa_mix.json);
# `valu_mix_frac` is its measured issue rate over that roof.
PIPES_FILE = os.path.join(ROOT, "profiles", "pipes.json")
ISA_MIX_FILE = os.path.join(ROOT, "profiles", "isa_mix.json")


def _load_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def _kernel_entries(d, kernel):
    return [v for k, v in (d or {}).get("kernels", {}).items() if _symbol_matches(k, kernel)]


def measured_pipes(kernel, batch):
    """The batch instantiation's entry of profiles/pipes.json (tools/pmc_pipes.sh +
    tools/pipes.py: per-dispatch instruction counts and pipe busy fractions from PMC passes of
    this bench configuration); None when absent or measured on another batch size."""
    d = _load_json(PIPES_FILE)
    if not d or d.get("batch") != batch:
        return None
    ents = _kernel_entries(d, kernel)
    # several instantiations may match (orient_desc_kernel<4> serves the single-frame call): the
    # batch launches are the largest
    return max(ents, key=lambda v: v.get("sq_insts_valu_per_dispatch") or 0) if ents else None


def mix_roof(kernel):
    """The VALU roof of the kernel's instruction mix, as a fraction of the nominal issue peak."""
    ents = _kernel_entries(_load_json(ISA_MIX_FILE), kernel)
    # the batch instantiation: the largest body
    return max(ents, key=lambda v: v["valu_static_instr"])["mix_roof_frac_of_nominal"] \
        if ents else None


def measured_valu(kernel, batch):
    """SQ_INSTS_VALU per dispatch of `kernel` (profiles/pipes.json) and the chip's nominal VALU
    issue peak; (None, None) when absent or measured on another batch size."""
    e = measured_pipes(kernel, batch)
    if not e or not e.get("sq_insts_valu_per_dispatch"):
        return None, None
    return e["sq_insts_valu_per_dispatch"], _load_json(PIPES_FILE).get("valu_issue_peak_per_s")


def binding_pipe(kernel, batch, hbm_frac):
    """The pipe nearest its roof: HBM (live) against the PMC pipe fractions of pipes.json."""
    e = measured_pipes(kernel, batch)
    # throughput roofs only: issue activity and the TA / TD busy counters measure occupancy
    # (latency included), not a pipe's rate (tools/pipes.py)
    fr = {k: v for k, v in (e or {}).get("pipe_frac", {}).items() if k in ("valu_mix", "lds", "mfma")}
    if hbm_frac is not None:
        fr["hbm"] = hbm_frac
    if not fr:
        return None, {}
    return max(fr, key=fr.get), fr


def measured_traffic(kernel, batch):
    """HBM bytes per dispatch of `kernel` measured by tools/pmc_traffic.sh + tools/traffic.py on
    this bench configuration (rocprofv3 FETCH_SIZE/WRITE_SIZE passes, gfx950 read calibration),
    committed as profiles/traffic.json; None when absent or measured on another batch size."""
    try:
        with open(TRAFFIC_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if d.get("batch") != batch:
        return None, None
    vals = [v.get("hbm_bytes_per_dispatch") or 0 for k, v in d.get("kernels", {}).items()
            if _symbol_matches(k, kernel)]  # the batch instantiation: the largest
    return (max(vals), d.get("source")) if vals else (None, None)


def path_bytes_per_frame(level_px, kp_per_image):
    """algorithmic HBM bytes of one stereo frame through the whole path --
    both views' pyramids read once (2 * sum_l W_l H_l) + the left / right / last-frame keypoints
    and descriptors the matchers read (3 * K * (28 + 32))."""
    return 2 * sum(level_px) + 3 * kp_per_image * 60


def kernel_bytes(name, n_images, n_frames, kp_per_image, level_px, n_queries, fast_cand=None):
    """Algorithmic (compulsory) HBM bytes one step moves through the named kernel (all its
    launches): every input byte the kernel needs read once, every output written once -- the
    per-kernel split of section 8(d)'s per-frame figure, not the bytes the kernel re-reads."""
    px = sum(level_px)
    if name == "pyr_down":       # read level l-1, write level l
        return n_images * sum(level_px[l - 1] + level_px[l] for l in range(1, len(level_px)))
    if name == "fast_cells":     # read every level once (+ small candidate writes)
        return n_images * px
    if name == "orient_desc":    # the image's pyramid (the keypoint windows cover the levels;
        # section 8(d) counts each level read once) + keypoint (28 B) and descriptor (32 B) out
        return n_images * (px + kp_per_image * 60)
    if name == "stereo_match":   # left+right kps/desc (60 B each) + SAD windows (11x11 + 11x21)
        return n_frames * kp_per_image * (2 * 60 + 121 + 231)
    if name == "search_cand":    # query (64 B) + window candidates' kps/desc (~60 B each, ~8)
        return n_queries * (64 + 8 * 60)
    if name == "octree":         # every FAST survivor of the image read (4 B key; the per-cell
        # counts ~5 KB per image are left out), the kept keys written (4 B each)
        if fast_cand is None:
            return None
        return n_images * 4 * (fast_cand + kp_per_image)
    return None


def stereo_line_bytes(ctx, level_px, line=128, pitch0=1280):
    """Compulsory bytes of stereo_match for the batch's frame 0 at cache-line granularity: the
    distinct `line`-byte lines its SAD windows touch (left 11 x 11 at the keypoint, right 11 x 21
    at u_right, both at the left keypoint's level; levels >= 1 at pitch round_up(w, 64) from
    256-aligned bases) plus every left / right keypoint and descriptor (60 B each) and the row
    table entries (4 B per (right keypoint, row) pair). Matches whose SAD step was rejected are
    not counted, so this is a lower bound."""
    kl, _ = ctx.keypoints(0)
    kr, _ = ctx.keypoints(1)
    ur, _ = ctx.stereo(0)
    dims = [ctx.pyramid_level(0, l).shape for l in range(8)]
    pitches = [pitch0] + [(w + 63) // 64 * 64 for (_, w) in dims[1:]]
    bases, off = [0], 1 << 30
    for l in range(1, 8):
        bases.append(off)
        off += (pitches[l] * dims[l][0] + 255) // 256 * 256
    lines = set()
    for i in np.nonzero(ur >= 0)[0]:
        lv = int(kl["octave"][i])
        inv = 1.0 / (1.2 ** lv)
        xl, yc, xr = (int(round(float(kl["x"][i]) * inv)), int(round(float(kl["y"][i]) * inv)),
                      int(round(float(ur[i]) * inv)))
        for side, x0, x1 in ((0, xl - 5, xl + 5), (1 << 40, xr - 10, xr + 10)):
            for y in range(yc - 5, yc + 6):
                a = side + bases[lv] + y * pitches[lv]
                lines.update(range((a + x0) // line, (a + x1) // line + 1))
    rows = sum(int(np.ceil(k["y"] + 2 * 1.2 ** k["octave"])) - int(np.floor(k["y"] - 2 * 1.2 ** k["octave"])) + 1
               for k in kr)
    return len(lines) * line + 60 * (len(kl) + len(kr)) + 4 * rows


def working_set_bytes(name, n_images, kp_per_image):
    """Bytes a kernel's work-items fetch counting overlaps (each keypoint's 43 x 43 raw window
    for orient_desc): an upper bound on its L2 -> CU traffic, not HBM bytes."""
    if name == "orient_desc":
        return n_images * kp_per_image * (43 * 43 + 60)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="stereo frames per GPU per step")
    ap.add_argument("--distinct", type=int, default=16, help="distinct synthetic renders of the sequence")
    ap.add_argument("--cpu-frames", type=int, default=0, help="oracle sample size (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streams", type=int, default=1,
                    help="split each step's batch over this many contexts on their own HIP streams")
    ap.add_argument("--inflight", type=int, default=int(os.environ.get("SLAMGPU_INFLIGHT", "2")),
                    help="batches in flight: consecutive steps alternate between this many "
                         "context groups, each on its own streams")
    ap.add_argument("--no-optimizer", action="store_true",
                    help="skip the PoseOptimization / LocalBundleAdjustment measurements")
    ap.add_argument("--no-bow", action="store_true",
                    help="skip the ComputeBoW / SearchByBoW measurement")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the single-frame drop-in latency and the PCIe-inclusive rate")
    ap.add_argument("--no-alone", action="store_true",
                    help="skip the second breakdown pass (level 0's FAST after the pyramid): the "
                         "PMC passes use it so that every kernel's dispatches are the step's")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"),
                    default=os.environ.get("SLAMGPU_BENCH_BACKEND", "nccl"),
                    help="process-group backend for N > 1: nccl (RCCL, one GPU per rank; the "
                         "driver's runs) or gloo (the gather staged through host memory; ranks "
                         "may share a GPU -- exercises the N-rank path on a one-GPU box)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    gloo = world > 1 and args.dist_backend == "gloo"
    if gloo:  # ranks share the visible GPUs round-robin (torch.cuda.device_count() makes no HIP call)
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # One explicit stream for torch ops and library launches alike: a null stream handle would
    # put the library's kernels on the context's own (non-blocking) stream, unordered with torch.
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        world = dist.get_world_size()
        # the CPU baseline and the optimizer / BoW legs are N=1 measurements
        args.no_cpu_baseline = args.no_optimizer = args.no_bow = args.no_latency = True

    from slam_framework_amd import slamgpu as G
    from slam_framework_amd import synthetic as S

    cols, rows, B, D = S.KITTI_COLS, S.KITTI_ROWS, args.batch, args.distinct
    cam = S.KITTI_CAM
    # ---- ONE synthetic sequence for the whole job (D distinct renders played back and forth,
    # frame g = render_of(g, D)), sharded contiguously with a one-frame halo, resident in HBM
    # before timing
    # (slam_framework_amd/sharded.py; the same object tests/test_sharded_gpu.py checks)
    Ls, Rs = S.layered_sequence(1000, D)
    from slam_framework_amd import dist as SD
    from slam_framework_amd.sharded import ShardedFrontend, render_of
    # per-frame results of the owned frames -> rank 0 (world > 1 only; SLAMGPU_BENCH_GATHER=1
    # runs the pack + gather path at world 1 too, as a local copy)
    gather = world > 1 or os.environ.get("SLAMGPU_BENCH_GATHER") == "1"
    job = ShardedFrontend(Ls, Rs, cam, B, dev, streams=args.streams, inflight=args.inflight,
                          rank=rank, world=world, gather=gather, host_gather=gloo)
    NS, Bs, INF = job.NS, job.Bs, job.INF
    host_l, host_r, poses = job.host_l, job.host_r, job.poses
    ctxs, parts = job.contexts, job.parts
    ctx = ctxs[0]
    kc = ctx.kp_cap
    gat = job.gat
    step = job.step

    for _ in range(max(1, args.warmup) * INF):
        step()
    job.sync()
    # sanity of what the timed steps compute (not timed)
    nk = np.array([ctx.keypoints(i)[0].shape[0] for i in range(min(4, 2 * Bs))])
    nm = np.concatenate([pt["nm"].cpu().numpy() for pt in parts])
    nq = np.concatenate([pt["qc"].cpu().numpy() for pt in parts])
    print(f"[rank {rank}] keypoints/image {nk.tolist()} queries/frame {nq[1:5].tolist()} "
          f"matches/frame {nm[1:5].tolist()}", file=sys.stderr)

    # ---- per-kernel breakdown pass (untimed) to pick the dominant kernel
    names = ["pyr_down", "fast_cells", "octree", "octree_global", "orient_desc", "stereo_rows",
             "stereo_match", "stereo_median", "grid_build", "vo_queries", "search_cand",
             "search_resolve"]
    torch.cuda.synchronize()
    ctx.timing_start("*", 4096)
    step(group=0)
    ctx.timing_stop()
    brk = {n: ctx.timing_read(n) for n in names}
    tot = sum(v[0] for v in brk.values())
    print("[rank %d] kernel ms/step: " % rank + ", ".join(
        f"{n} {brk[n][0]:.3f} ({100 * brk[n][0] / tot:.0f}%)" for n in names), file=sys.stderr)
    dominant = max(names, key=lambda n: brk[n][0])
    # the same pass with level 0's FAST after the pyramid instead of beside it (a side stream in
    # the step): every kernel alone, the basis of the per-kernel pipe fractions (the PMC pass
    # serialises dispatches too); the step itself keeps the fork
    alone = brk
    if not args.no_alone:
        for c in ctxs:
            c.set_extract_fork(False)
        torch.cuda.synchronize()
        ctx.timing_start("*", 4096)
        step(group=0)
        ctx.timing_stop()
        alone = {n: ctx.timing_read(n) for n in names}
        for c in ctxs:
            c.set_extract_fork(True)

    # ---- timed region
    launches_per_step = max(1, brk[dominant][1])
    ctx.timing_start(dominant, launches_per_step * args.steps + 16)
    bench_stream = torch.cuda.current_stream(dev).cuda_stream
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    G.trace_marker(1, bench_stream)  # brackets the timed launches in a rocprofv3 kernel trace
    torch.cuda.synchronize()        # (tools/stats_timed.py); outside the timed interval
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if gat is not None:
        gat.wait_all()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    G.trace_marker(2, bench_stream)
    ctx.timing_stop()
    job.sync()
    elapsed = SD.max_over_ranks(t1 - t0, dev)
    dom_ms, dom_n = ctx.timing_read(dominant)
    # per-rank result summary gathered to every rank (validation, outside the timed region)
    summ = SD.gather_summary([int(nk.sum()), int(nm.sum()), int(nq.sum())], dev)

    frames = world * NS * (Bs - 1) * args.steps
    value = frames / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    gather_info = job.check_gather() if gat is not None else None
    if rank == 0:
        level_px = [ctx.pyramid_level(0, l).size for l in range(8)]
        kp_img = float(nk.mean())
        nqueries = int(nq.sum())
        # FAST survivors per image (what the octree reads): images 0-3 of the batch, all levels
        cand_lv = np.array([[len(ctx.debug_level_keys(i, l, 0)) for l in range(8)]
                            for i in range(min(4, 2 * Bs))])
        fast_cand = float(cand_lv.sum(1).mean())
        dom_bytes = kernel_bytes(dominant, 2 * Bs, Bs, kp_img, level_px, nqueries // NS, fast_cand)
        avg_launch_s = dom_ms / 1000.0 / max(1, dom_n)
        per_launch_bytes = dom_bytes / max(1, launches_per_step) if dom_bytes else None
        achieved = (per_launch_bytes / avg_launch_s / 1e9) if per_launch_bytes else None
        roofline = {
            "kernel": dominant, "bound": "hbm",
            "achieved": round(achieved, 2) if achieved else None,
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
            "traffic": None,
            "avg_launch_us": round(avg_launch_s * 1e6, 2), "launches": dom_n,
            "algorithmic_bytes_per_launch": per_launch_bytes,
            "bytes_model": "section 8(d): compulsory bytes (pyramid read once + outputs), see "
                           "kernel_bytes()",
        }
        ws = working_set_bytes(dominant, 2 * Bs, kp_img)
        if ws:
            roofline["working_set_bytes_per_launch"] = ws / max(1, launches_per_step)
        # the whole path against HBM: section 8(d)'s bytes per stereo frame x frames/s
        pbf = path_bytes_per_frame(level_px, kp_img)
        path_roof = {"bytes_per_stereo_frame": round(pbf),
                     "achieved": round(pbf * value / 1e9, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(pbf * value / 1e9 / HBM_PEAK_GBS, 5)}
        traffic, tsrc = measured_traffic(dominant, B)
        if traffic is not None:
            roofline["traffic"] = round(traffic)
            roofline["traffic_source"] = tsrc
        # the dominant kernel against each pipe over the timed region (co-running with the other
        # batch's kernels): HBM above, VALU issue against its own mix's roof (PMC instruction
        # count per dispatch over the live launch time); the binding pipe is chosen below on the
        # standalone basis of kernels_standalone
        vi, vpeak = measured_valu(dominant, B)
        mr = mix_roof(dominant)
        hbm = {k: roofline[k] for k in ("achieved", "peak", "unit", "frac", "traffic")}
        if traffic is not None:
            hbm["traffic_frac"] = round(traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS, 5)
        roofline["hbm"] = hbm
        if vi is not None and mr:
            rate = vi / avg_launch_s
            roofline["valu_mix"] = {"wave_instr_per_launch": round(vi), "achieved": rate,
                                    "peak": vpeak * mr, "unit": "wave-instr/s",
                                    "frac": round(rate / (vpeak * mr), 4),
                                    "nominal_peak": vpeak, "mix_roof_frac_of_nominal": mr,
                                    "basis": "timed region (co-running launches)",
                                    "source": "SQ_INSTS_VALU: profiles/pipes.json; mix roof: "
                                              "profiles/isa_mix.json (tools/isa_mix.py)"}
        cpu = None
        if not args.no_cpu_baseline:
            dk, dd = ctx.keypoints(0)   # the left view of the batch's frame 0
            cpu = cpu_baseline(Ls, Rs, args.cpu_frames,
                               device_check=(render_of(int(job.gframe[0]), D), dk, dd))
        # the drop-in legs run before the optimizer legs: run after them, the host-fed step's
        # copies and kernels overlap less (batched_h2d 56k -> 39k frames/s, the copy and compute
        # times unchanged; profiles/r8m_h2d_leg_ab.log -- the cause is not isolated)
        drop_in = None
        if not args.no_latency:
            drop_in = {"single_frame": bench_frame_latency(Ls, Rs, cam, local),
                       "batched_h2d": bench_h2d(ctxs[0], host_l, host_r, poses, cam, dev, args)}
        opt = None
        if not args.no_optimizer:
            opt = {"pose_optimization": bench_pose(dev, not args.no_cpu_baseline),
                   "local_bundle_adjustment": bench_local_ba(dev, not args.no_cpu_baseline)}
        bow_leg = None
        if not args.no_bow:
            bow_leg = bench_bow(ctx, Bs, dev, not args.no_cpu_baseline)
        # every frontend kernel on its roofs: standalone launch times of the breakdown pass (one
        # batch, nothing else in flight), algorithmic bytes, PMC traffic and VALU counts
        # every frontend kernel on its roofs, from the breakdown passes (one batch, nothing else
        # in flight): `ms_per_step` as the step runs it (level 0's FAST beside the pyramid),
        # `alone_ms_per_step` with each kernel alone -- the basis of the fractions, per step
        # (bytes and instructions per launch x launches, over the alone time), like the PMC pass
        kernels = {}
        for n in names:
            ms, nl = brk[n]
            if ms <= 0 or nl <= 0:
                continue
            avg_s = ms / 1000.0 / nl
            ent = {"ms_per_step": round(ms, 4), "launches_per_step": nl,
                   "avg_launch_us": round(avg_s * 1e6, 2)}
            ams = alone[n][0] if alone[n][0] > 0 else ms
            ent["alone_ms_per_step"] = round(ams, 4)
            step_s = ams / 1000.0
            kb = kernel_bytes(n, 2 * Bs, Bs, kp_img, level_px, nqueries // NS, fast_cand)
            if kb:
                ent["algorithmic_bytes_per_launch"] = kb / nl
                ent["hbm_frac"] = round(kb / step_s / 1e9 / HBM_PEAK_GBS, 4)
            tr, _ = measured_traffic(n, B)
            if tr is not None:
                ent["traffic_bytes_per_launch"] = round(tr)
                ent["traffic_frac"] = round(tr * nl / step_s / 1e9 / HBM_PEAK_GBS, 4)
            vi, vpeak = measured_valu(n, B)
            mr = mix_roof(n)
            if vi is not None:
                ent["valu_wave_instr_per_launch"] = round(vi)
                ent["valu_issue_frac"] = round(vi * nl / step_s / vpeak, 4)
                if mr:
                    ent["valu_mix_roof_frac_of_nominal"] = mr
                    ent["valu_mix_frac"] = round(vi * nl / step_s / (vpeak * mr), 4)
            bp, fr = binding_pipe(n, B, ent.get("traffic_frac", ent.get("hbm_frac")))
            if bp:
                if "valu_mix_frac" in ent:
                    fr["valu_mix"] = ent["valu_mix_frac"]
                    bp = max(fr, key=fr.get)
                ent["pipes"] = {k: round(v, 4) for k, v in fr.items()}
                ent["binding_pipe"] = bp
            pe = measured_pipes(n, B)
            if pe and pe.get("lds_conflict_per_instr") is not None:
                ent["lds_conflict_per_instr"] = pe["lds_conflict_per_instr"]
            kernels[n] = ent
        if "octree" in kernels:
            kernels["octree"]["fast_candidates_per_image"] = round(fast_cand)
            kernels["octree"]["fast_candidates_per_level_max"] = cand_lv.max(0).tolist()
        if "stereo_match" in kernels:
            # HBM moves lines: the windows' distinct 128-B lines (frame 0 of the batch) + the
            # keypoint/descriptor/row-table reads, per launch (tools/stereo_lines.py restates it)
            lb = stereo_line_bytes(ctx, level_px)
            kernels["stereo_match"]["line_granular_bytes_per_launch"] = lb * Bs
        # the binding pipe of the dominant kernel, every fraction on one (standalone) basis: the
        # breakdown pass's launch time for HBM traffic and VALU, the PMC pass's serialised
        # dispatch for the LDS / MFMA busy fractions
        ke = kernels.get(dominant, {})
        if ke.get("pipes"):
            fr = ke["pipes"]
            bp = max(fr, key=fr.get)
            roofline["pipes"] = fr
            roofline["bound"] = {"valu_mix": "valu"}.get(bp, bp)
            if bp == "valu_mix":
                ra = (ke["valu_wave_instr_per_launch"] * ke["launches_per_step"]
                      / (ke["alone_ms_per_step"] * 1e-3))
                roofline.update(achieved=round(ra / 1e9, 2),
                                peak=round(vpeak * ke["valu_mix_roof_frac_of_nominal"] / 1e9, 2),
                                unit="G wave-instr/s", frac=fr[bp])
            elif bp != "hbm":
                roofline.update(achieved=fr[bp], peak=1.0, unit="busy fraction", frac=fr[bp])
            roofline["bound_source"] = (
                "largest pipe fraction of kernels_standalone[kernel].pipes (HBM traffic and VALU "
                "over the kernel's alone time per step, LDS / MFMA busy of the PMC pass's "
                "serialised dispatch, profiles/pipes.json); the timed-region figures are in hbm / "
                "valu_mix")
        line = {
            "metric": "stereo frames/sec ORB extract+match @1241x376, 2000 kp/frame",
            "value": round(value, 2), "unit": "stereo frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded layered-surfaces scene: ~50% of keypoints with stereo "
                    "depth, ~1000 frame-to-frame queries/frame; camera turning + 0.3 m/frame "
                    "forward; one sequence of 16 renders played back and forth, sharded over the "
                    "ranks)",
            "config": {"workload": "configs[1]: synthetic 1241x376 stereo stream, 2000 kp/frame, "
                                   "extract L+R + stereo match + frame-to-frame match",
                       "frames_per_gpu_per_step": NS * (Bs - 1), "batch": B, "streams": NS,
                       "batches_in_flight": INF,
                       "nfeatures": 2000,
                       "nlevels": 8, "scale_factor": 1.2, "fast_th": [20, 7],
                       "parallelism": f"frame-sharded x{world}" + (
                           ", contiguous shards + 1 halo frame, " + (
                               "gloo gather through host memory to rank 0" if gloo else
                               "RCCL gather to rank 0") if world > 1 else ""),
                       "dist_backend": (args.dist_backend if world > 1 else None)},
            "gather": gather_info,
            "roofline": roofline,
            "path_roofline": path_roof,
            "cpu_baseline": cpu,
            "kernel_ms_per_step": {n: round(brk[n][0], 4) for n in names},
            "kernels_standalone": kernels,
            "optimizer": opt,
            "bow": bow_leg,
            "drop_in": drop_in,
            "per_rank_matches_per_step": summ[:, 1].tolist(),
        }
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (RANK /
    LOCAL_RANK / WORLD_SIZE, rendezvous on 127.0.0.1) before this process makes any GPU call,
    wait for all of them and return the worst exit code. Only rank 0 prints the JSON line."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    return max(abs(p.wait()) for p in procs)


def bench_frame_latency(Ls, Rs, cam, device, reps=40):
    """The unmodified Tracker's call pattern (tracker.cpp:104-141 -> the stereo Frame ctor,
    frame.cpp:61-111): ONE frame per call from host images -- slamgpu_frame_stereo (H2D of both
    views, extract L+R, stereo, grid) plus the download of both views' keypoints + descriptors
    and the stereo coordinates the Frame holds. Median wall time per frame."""
    from slam_framework_amd import slamgpu as G
    from slam_framework_amd import synthetic as S
    c = G.Context(S.KITTI_COLS, S.KITTI_ROWS, 2000, 1.2, 8, 20, 7, max_frames=1, device=device)
    ms = []
    for i in range(reps + 3):
        f = i % len(Ls)
        t0 = time.perf_counter()
        c.frame_stereo(Ls[f], Rs[f], cam)
        c.keypoints(0)
        c.keypoints(1)
        c.stereo(0)
        ms.append(1e3 * (time.perf_counter() - t0))
    c.close()
    ms = np.array(ms[3:])
    return {"workload": "one stereo frame per call from host memory (slamgpu_frame_stereo + "
                        "download of keypoints, descriptors, u_right/depth)",
            "median_ms": round(float(np.median(ms)), 3), "p90_ms": round(float(np.percentile(ms, 90)), 3),
            "frames_per_s": round(1e3 / float(np.median(ms)), 1), "calls": reps}


def bench_h2d(ctx, host_l, host_r, poses, cam, dev, args, steps=10):
    """Batched throughput with the input crossing PCIe inside the timed region: every step's B
    stereo frames are copied from pinned host memory on a copy stream into one of two device
    buffers while the previous step computes on the other (the same step as the headline)."""
    import torch
    from slam_framework_amd import slamgpu as G
    from slam_framework_amd import synthetic as S
    B, rows, pitch = host_l.shape
    cols = S.KITTI_COLS
    stride = rows * pitch
    kc = ctx.kp_cap
    # the frames cross PCIe at their own 1241-byte rows (the bytes a caller's images hold) and
    # are spread to the 1280-byte device pitch by one strided device copy on the compute stream
    pin = [torch.from_numpy(np.ascontiguousarray(h[:, :, :cols])).pin_memory()
           for h in (host_l, host_r)]
    stage = [[torch.empty_like(p, device=dev) for p in pin] for _ in range(2)]
    bufs = [[torch.zeros((B, rows, pitch), dtype=torch.uint8, device=dev) for _ in pin]
            for _ in range(2)]
    main = torch.cuda.current_stream()
    cp = torch.cuda.Stream(device=dev)
    d_poses = torch.from_numpy(poses.view(np.uint8).copy()).to(dev)
    q = torch.empty(B * kc * G.F2F_QUERY_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    qs, qc, nm = (torch.empty(B, dtype=torch.int32, device=dev) for _ in range(3))
    mp = torch.empty(B * kc, dtype=torch.int32, device=dev)
    blk = torch.empty(B * kc, dtype=torch.uint8, device=dev)
    done = [torch.cuda.Event(), torch.cuda.Event()]
    for e in done:
        e.record(main)
    ev = []  # per timed step: copy start / end on the copy stream, compute start / end on main

    def step(k, timed=False):
        dl, dr = bufs[k % 2]
        sl, sr = stage[k % 2]
        cp.wait_event(done[k % 2])           # the step that last read these buffers is done
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if timed else None
        with torch.cuda.stream(cp):
            if e:
                e[0].record(cp)
            sl.copy_(pin[0], non_blocking=True)
            sr.copy_(pin[1], non_blocking=True)
            if e:
                e[1].record(cp)
        main.wait_stream(cp)
        h = main.cuda_stream
        if e:
            e[2].record(main)
        dl[:, :, :cols].copy_(sl)
        dr[:, :, :cols].copy_(sr)
        ctx.frontend_device(dl, dr, stride, pitch, B, cam, h)
        ctx.make_vo_queries_device(d_poses, 1, q, qs, qc, B, h)
        mp.fill_(-1)
        blk.zero_()
        ctx.search_by_projection_frame_device(q, B * kc, qs, qc, kc, d_poses, mp, blk, kc, nm,
                                              B, h)
        if e:
            e[3].record(main)
            ev.append(e)
        done[k % 2].record(main)
    for k in range(2):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    h2d_bytes = 2 * pin[0].numel()
    for k in range(4):  # the split (untimed): copy and compute durations while they overlap
        step(k, timed=True)
    torch.cuda.synchronize()
    copy_ms = float(np.median([e[0].elapsed_time(e[1]) for e in ev]))
    comp_ms = float(np.median([e[2].elapsed_time(e[3]) for e in ev]))
    pair_bytes = 2 * S.KITTI_COLS * S.KITTI_ROWS
    return {"workload": "the headline step with both views copied from pinned host memory each "
                        "step at 1241-byte rows (copy stream, double-buffered) and spread to the "
                        "1280-byte device pitch on the compute stream",
            "value": round(steps * (B - 1) / dt, 1), "unit": "stereo frames/s",
            "ms_per_step": round(1e3 * dt / steps, 3),
            "h2d_bytes_per_step": int(h2d_bytes),
            "h2d_GBps": round(h2d_bytes * steps / dt / 1e9, 2),
            "copy_engine_ceiling": "profiles/r8e_h2d_ceiling.log: 54-57 GB/s pinned host -> HBM "
                                   "alone (1-4 copy streams, DMA engines or blit kernels alike)",
            "copy_ms_per_step": round(copy_ms, 3), "compute_ms_per_step": round(comp_ms, 3),
            "image_bytes_per_pair": pair_bytes}


FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak (MI355X_MICROARCH.md)
# Algorithmic FP64 flops per pose edge: a linearise pass (error ~60, Jacobian ~40, H/b ~160)
# and a trial pass (error + Huber ~60) per LM iteration (DESIGN.md "Optimizer rows").
POSE_FLOPS_PER_EDGE_ITER = 320


def _events_ms(fn, stream, reps):
    """Median HIP-event time of fn() on `stream` (the stream the kernel is launched on)."""
    import torch
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        fn()
        b.record(stream)
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return float(np.median(ms))


def bench_pose(dev, with_cpu):
    """configs[3]: Optimizer::PoseOptimization on SURVEY.md section 8(d) C4 problems (2000 edges,
    60% stereo, 10% gross outliers, start 2 deg / 0.3 m off; seeds 7, 8, ...), batched over 2048
    frames and as a single-frame call; the oracle on host cores."""
    import torch
    from slam_framework_amd import slamgpu as G
    from slam_framework_amd import synthetic as S

    B, distinct = 2048, 64
    probs = [S.c4_problem(7 + i) for i in range(distinct)]
    edges = np.concatenate([p[0] for p in probs])
    start = np.zeros(distinct + 1, np.int64)
    start[1:] = np.cumsum([len(p[0]) for p in probs])
    poses = np.stack([p[1] for p in probs])
    isig = probs[0][3]
    k = B // distinct
    E = np.concatenate([edges] * k)
    st = np.concatenate([start[:-1] + i * start[-1] for i in range(k)] + [[k * start[-1]]])
    stream = torch.cuda.current_stream()
    d_e = torch.from_numpy(E.view(np.uint8).copy()).to(dev)
    d_s = torch.from_numpy(st.astype(np.int32)).to(dev)
    d_T0 = torch.from_numpy(np.concatenate([poses] * k)).to(dev)
    d_T = d_T0.clone()
    d_o = torch.zeros(len(E), dtype=torch.uint8, device=dev)
    d_r = torch.zeros(B, dtype=torch.int32, device=dev)
    d_it = torch.zeros(B, dtype=torch.int32, device=dev)

    def run(n):
        d_T.copy_(d_T0)
        G.pose_optimization_device(S.KITTI_CAM, isig, d_e, d_s, n, d_T, d_o, d_r, d_it,
                                   stream.cuda_stream)
    run(B)
    torch.cuda.synchronize()
    ms = _events_ms(lambda: run(B), stream, 5)
    its = d_it.cpu().numpy()
    flops = float((its.astype(np.float64) * np.diff(st)).sum()) * POSE_FLOPS_PER_EDGE_ITER
    ms1 = _events_ms(lambda: run(1), stream, 10)
    out = {"workload": "configs[3]: PoseOptimization on SURVEY 8(d) C4 (2000 edges/frame, 60% "
                       "stereo, 10% gross outliers, 2 deg / 0.3 m start), 4 rounds x 10 LM "
                       "iterations (FP64)",
           "frames_per_s": round(B / ms * 1e3, 1), "batch_frames": B,
           "ms_per_batch": round(ms, 3), "single_frame_ms": round(ms1, 4),
           "lm_iterations_per_frame": round(float(its.mean()), 2),
           "roofline": {"kernel": "pose_opt", "bound": "fp64 valu",
                        "achieved": round(flops / (ms * 1e-3) / 1e12, 3),
                        "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(flops / (ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFLOPS, 4),
                        "flops_per_edge_iteration": POSE_FLOPS_PER_EDGE_ITER},
           "cpu_baseline": None}
    if with_cpu:
        import concurrent.futures as cf
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        O.build()
        threads = host_cpu_share()[0]
        per = 16

        def work(t):
            for i in range(per):
                p = probs[(t * per + i) % distinct]
                O.pose_optimization(S.KITTI_CAM, isig, p[0], p[1])
            return per
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            done = sum(ex.map(work, range(threads)))
        wall = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(done / wall, 1), "unit": "frames/s",
                               "cores": threads, "kind": "port",
                               "sample": f"{done} frames of 2000 edges ({threads} threads x "
                                         f"{per}); oracle/pose_oracle.c FP64 restatement"}
    return out


def bench_local_ba(dev, with_cpu):
    """configs[4]: Optimizer::LocalBundleAdjustment on SURVEY.md section 8(d) C5 (20 local + 5
    fixed keyframes at 1 m spacing, 3000 map points seen by 2-6 keyframes, ~12k observations;
    seed 11), one problem and a batch of 256 (one per CU); the oracle on host cores."""
    import torch
    from slam_framework_amd import slamgpu as G
    from slam_framework_amd import synthetic as S

    P = S.c5_problem(11)
    nk, npn, no = len(P["kf_mode"]), len(P["points"]), len(P["obs"])
    stream = torch.cuda.current_stream()
    res = {}
    BB = int(os.environ.get("SLAMGPU_BA_BATCH", "256"))  # problems per batch (a workgroup each)
    for B in (1, BB):
        desc = np.array([(i * nk, nk, i * npn, npn) for i in range(B)], np.int32)
        start = np.concatenate([P["point_obs_start"][:-1] + i * no for i in range(B)] +
                               [[B * no]]).astype(np.int32)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)
        d_desc, d_mode, d_start = t(desc), t(np.tile(P["kf_mode"], B)), t(start)
        d_obs = t(np.tile(P["obs"], B))
        kf0, pts0 = t(np.tile(P["kf_Tcw"], (B, 1, 1))), t(np.tile(P["points"], (B, 1)))
        d_kf, d_pts = kf0.clone(), pts0.clone()
        d_er = torch.zeros(B * no, dtype=torch.uint8, device=dev)
        d_st = torch.zeros(B, dtype=torch.int32, device=dev)
        d_ws = torch.empty(G.local_ba_workspace_bytes(B * nk, B * npn, B * no),
                           dtype=torch.uint8, device=dev)

        def run():
            d_kf.copy_(kf0)
            d_pts.copy_(pts0)
            G.local_bundle_adjustment_device(S.KITTI_CAM, P["inv_sigma2"], d_desc, B, d_kf,
                                             d_mode, d_pts, d_start, d_obs, d_er, d_st, d_ws,
                                             B * nk, B * npn, B * no, stream=stream.cuda_stream)
        run()
        torch.cuda.synchronize()
        res[B] = (_events_ms(run, stream, 3), int(d_st[0].item()))
    # the batched reprojection residual / Jacobian / normal-equation build on its own (one
    # computeActiveErrors + buildSystem of the first optimize() per problem), 256 problems
    BL = 256
    desc = np.array([(i * nk, nk, i * npn, npn) for i in range(BL)], np.int32)
    start = np.concatenate([P["point_obs_start"][:-1] + i * no for i in range(BL)] +
                           [[BL * no]]).astype(np.int32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)
    d_desc, d_mode, d_start = t(desc), t(np.tile(P["kf_mode"], BL)), t(start)
    d_obs, d_kf, d_pts = t(np.tile(P["obs"], BL)), t(np.tile(P["kf_Tcw"], (BL, 1, 1))), t(
        np.tile(P["points"], (BL, 1)))
    f64 = lambda *sh: torch.empty(sh, dtype=torch.float64, device=dev)
    lin = {"chi2": f64(BL * no), "hpl": f64(BL * no, 18), "hll": f64(BL * npn, 6),
           "bl": f64(BL * npn, 3), "hpp": f64(BL * nk, 21), "bp": f64(BL * nk, 6), "chi": f64(BL)}
    d_st = torch.zeros(BL, dtype=torch.int32, device=dev)
    d_ws = torch.empty(G.local_ba_workspace_bytes(BL * nk, BL * npn, BL * no), dtype=torch.uint8,
                       device=dev)

    def lin_run():
        G.local_ba_linearize_device(S.KITTI_CAM, P["inv_sigma2"], d_desc, BL, d_kf, d_mode, d_pts,
                                    d_start, d_obs, lin, d_st, d_ws, BL * nk, BL * npn, BL * no,
                                    stream=stream.cuda_stream)
    lin_run()
    torch.cuda.synchronize()
    lms = _events_ms(lin_run, stream, 5)
    # algorithmic bytes: observation in (20 B) + chi2 and the 6x3 block out (8 + 144 B); point in
    # (12 B) + its 3x3 block and b out (72 B); keyframe pose in (64 B) + 6x6 block and b out (216 B)
    lin_bytes = BL * (no * (20 + 8 + 144) + npn * (12 + 72) + nk * (64 + 216))
    lin_gbs = lin_bytes / (lms * 1e-3) / 1e9
    out_lin = {"workload": "LocalBA residual/Jacobian/normal-equation build (computeActiveErrors + "
                           f"buildSystem), {BL} C5 problems", "batch_problems": BL,
               "ms_per_batch": round(lms, 3), "observations_per_s": round(BL * no / lms * 1e3),
               "roofline": {"kernel": "local_ba_linearize", "bound": "hbm",
                            "achieved": round(lin_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(lin_gbs / HBM_PEAK_GBS, 4),
                            "algorithmic_bytes_per_launch": lin_bytes}}
    del d_ws, lin
    # the drop-in calls (host buffers in and out, synchronous): slamgpu_local_bundle_adjustment
    # and slamgpu_global_bundle_adjustment, one problem spread over the CUs (csrc/ba_coop.hip)
    def wall_ms(fn, reps=10):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = fn()
            ts.append(1e3 * (time.perf_counter() - t0))
        return float(np.median(ts)), r
    drop = {}
    P48 = S.ba_problem(12, n_local=48, n_fixed=6, n_points=5000, spacing=0.6)
    for name, PP in (("C5", P), ("local_window_48", P48)):
        ms, r = wall_ms(lambda: G.Optimizer.LocalBundleAdjustment(
            PP["kf_Tcw"], PP["kf_mode"], PP["points"], PP["point_obs_start"], PP["obs"],
            S.KITTI_CAM, PP["inv_sigma2"]))
        drop[name] = {"ms": round(ms, 3), "lm_iterations": r[3],
                      "keyframes": int(len(PP["kf_mode"])), "points": int(len(PP["points"])),
                      "observations": int(len(PP["obs"]))}
    for nkf, npt in ((30, 4000), (100, 12000)):
        PG = S.ba_problem(34, n_local=nkf, n_fixed=0, n_points=npt, first_local_fixed=True,
                          spacing=0.8)
        ms, r = wall_ms(lambda: G.Optimizer.BundleAdjustment(
            PG["kf_Tcw"], PG["kf_mode"], PG["points"], PG["point_obs_start"], PG["obs"],
            S.KITTI_CAM, PG["inv_sigma2"], n_iterations=10), reps=5)
        drop[f"global_ba_{nkf}kf"] = {"ms": round(ms, 3), "lm_iterations": r[2], "keyframes": nkf,
                                      "points": npt, "observations": int(len(PG["obs"]))}
    # a map-scale global BA after a loop closure (GlobalBundleAdjustemnt over every keyframe,
    # optimizer.cpp:18-31): a closed loop of 1500 keyframes, S in block-profile storage
    PM = S.map_problem(1540, 1500)
    ms, r = wall_ms(lambda: G.Optimizer.BundleAdjustment(
        PM["kf_Tcw"], PM["kf_mode"], PM["points"], PM["point_obs_start"], PM["obs"],
        S.KITTI_CAM, PM["inv_sigma2"], n_iterations=10), reps=2)
    drop["global_ba_1500kf_loop"] = {"ms": round(ms, 3), "lm_iterations": r[2], "keyframes": 1500,
                                     "points": int(len(PM["points"])),
                                     "observations": int(len(PM["obs"]))}
    # the loop closer's optimisers: OptimizeSim3 on one loop candidate and
    # OptimizeEssentialGraph over a 400-keyframe loop, with the oracle on one host thread beside
    isig = S.level_inv_sigma2()
    m3, S3, _, _, _ = S.sim3_problem(340, 300, outlier_frac=0.2)
    ms, r = wall_ms(lambda: G.Optimizer.OptimizeSim3(m3, S3, S.KITTI_CAM, S.KITTI_CAM, isig,
                                                     isig, 10.0, False))
    drop["optimize_sim3_300"] = {"ms": round(ms, 3), "n_inliers": r[0], "matches": int(len(m3))}
    Seg, fx, Eeg, _, _ = S.essential_graph_problem(460, 400, fix_scale=True, old_loop=(200, 80))
    ms, r = wall_ms(lambda: G.Optimizer.OptimizeEssentialGraph(Seg, fx, Eeg, True, 20), reps=5)
    drop["essential_graph_400kf"] = {"ms": round(ms, 3), "lm_iterations": r[3], "keyframes": 400,
                                     "edges": int(len(Eeg))}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        O.build()
        t0 = time.perf_counter()
        O.global_ba(S.KITTI_CAM, PM, 10, True)
        drop["global_ba_1500kf_loop"]["oracle_1thread_ms"] = round(
            1e3 * (time.perf_counter() - t0), 1)
        t0 = time.perf_counter()
        O.optimize_sim3(S.KITTI_CAM, S.KITTI_CAM, isig, isig, m3, S3, 10.0, False)
        drop["optimize_sim3_300"]["oracle_1thread_ms"] = round(1e3 * (time.perf_counter() - t0), 3)
        t0 = time.perf_counter()
        O.optimize_essential_graph(Seg, fx, Eeg, True, 20)
        drop["essential_graph_400kf"]["oracle_1thread_ms"] = round(
            1e3 * (time.perf_counter() - t0), 3)
    out = {"linearize": out_lin, "drop_in": drop,
           "workload": "configs[4]: LocalBundleAdjustment on SURVEY 8(d) C5, 20 local + 5 fixed "
                       f"keyframes x 3000 map points ({no} observations), 5 robust + 10 LM "
                       "iterations (FP64)",
           "problems_per_s": round(BB / res[BB][0] * 1e3, 1), "batch_problems": BB,
           "single_problem_ms": drop["C5"]["ms"],
           "batched_kernel_one_problem_ms": round(res[1][0], 3), "lm_iterations": res[1][1],
           "cpu_baseline": None}
    if with_cpu:
        import concurrent.futures as cf
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        O.build()
        threads = host_cpu_share()[0]
        per = 2
        probs = [S.c5_problem(11 + i) for i in range(4)]

        def work(tid):
            for i in range(per):
                O.local_ba(S.KITTI_CAM, probs[(tid + i) % len(probs)])
            return per
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            done = sum(ex.map(work, range(threads)))
        wall = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(done / wall, 2), "unit": "problems/s",
                               "cores": threads, "kind": "port",
                               "sample": f"{done} problems ({threads} threads x {per}); "
                                         "oracle/ba_oracle.c FP64 restatement"}
    return out


# Compulsory bytes of one descriptor through Frame::ComputeBoW: the descriptor in (32 B), the
# per-feature leaf / node written and read back (16 B), the feature's word, weight, value, node
# and feature-list entries (28 B). The descent itself reads, per level of an ORBvoc-shaped
# vocabulary (k = 10, L = 6), the k children's descriptors and slots (10 x 48 B): 2880 B per
# descriptor that L2 / MALL serve (the vocabulary is 53 MB; its top levels are shared by all).
BOW_BYTES_PER_DESC = 32 + 16 + 28
BOW_VOCAB_BYTES_PER_DESC = 6 * 10 * 48


def bench_bow(ctx, Bs, dev, with_cpu):
    """SURVEY.md section 8(f) row 1 on the batch the timed step just extracted: Frame::ComputeBoW
    (DBoW2 transform, levelsup 4) of every left view straight from the frontend's device outputs,
    then OrbMatcher::SearchByBoW(KeyFrame = frame f, whose stereo keypoints carry map points;
    Frame = frame f + 1) for every consecutive pair. The vocabulary is ORBvoc.txt's shape (k 10,
    L 6, 1.1M nodes, L1 / TF-IDF), seeded, its top two levels from real descriptors: the reference
    ships none."""
    import torch
    from slam_framework_amd import bow
    from slam_framework_amd import synthetic as S

    V = S.vocabulary(31, k=10, L=6, pool=ctx.keypoints(0)[1])
    voc = bow.ORBVocabulary.from_arrays(V, device=dev.index)
    view = ctx.device_results()
    kc = view.kp_cap
    cap = min(kc, bow.MAX_FEATURES)
    sets = bow.DeviceBowSets(Bs, cap, dev)
    stream = torch.cuda.current_stream()

    def transform():
        voc.transform_device(view.desc, 2 * kc, view.nkps, 2, Bs, 4, sets, stream.cuda_stream)
    transform()
    # SearchByBoW views: A = left view of frame f (valid = has stereo depth), B = frame f + 1
    valid = np.zeros((Bs, kc), np.uint8)
    for f in range(Bs):
        d = ctx.stereo(f)[1]
        valid[f, :len(d)] = d > 0
    d_valid = torch.from_numpy(valid).to(dev)
    va = np.zeros(Bs - 1, bow.VIEW_DTYPE)
    vb = np.zeros(Bs - 1, bow.VIEW_DTYPE)
    for f in range(Bs - 1):
        for rec, fr, vld in ((va, f, int(d_valid.data_ptr()) + f * kc), (vb, f + 1, 0)):
            rec["desc"][f] = view.desc + 2 * fr * kc * 32
            rec["kps"][f] = view.kps + 2 * fr * kc * 28
            rec["valid"][f] = vld
            rec["n"][f] = view.nkps + 4 * 2 * fr
            for k, a in sets.view_of(fr).items():
                rec[k][f] = a
    d_va = torch.from_numpy(va.view(np.uint8).copy()).to(dev)
    d_vb = torch.from_numpy(vb.view(np.uint8).copy()).to(dev)
    d_match = torch.empty((Bs - 1, cap), dtype=torch.int32, device=dev)
    d_nm = torch.empty(Bs - 1, dtype=torch.int32, device=dev)

    def search():
        bow.search_by_bow_device(d_va, d_vb, Bs - 1, False, 0.7, True, d_match, cap, d_nm,
                                 stream.cuda_stream)
    search()
    torch.cuda.synchronize()
    t_ms = _events_ms(transform, stream, 5)
    s_ms = _events_ms(search, stream, 5)
    n_desc = sum(ctx.keypoints(2 * f)[0].shape[0] for f in range(Bs))
    nm = d_nm.cpu().numpy()
    gbs = n_desc * BOW_BYTES_PER_DESC / (t_ms * 1e-3) / 1e9
    out = {"workload": "SURVEY 8(f) row 1: Frame::ComputeBoW (DBoW2 transform, levelsup 4, "
                       "ORBvoc-shaped k 10 / L 6 vocabulary) of each frame's left view + "
                       "SearchByBoW(KeyFrame f, Frame f+1), from the frontend's device outputs",
           "frames": Bs, "descriptors": n_desc, "transform_ms": round(t_ms, 3),
           "transform_frames_per_s": round(Bs / t_ms * 1e3, 1),
           "search_ms": round(s_ms, 3), "search_pairs_per_s": round((Bs - 1) / s_ms * 1e3, 1),
           "matches_per_pair": round(float(nm.mean()), 1),
           "roofline": {"kernel": "bow_descend + bow_vectors", "bound": "hbm",
                        "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4),
                        "algorithmic_bytes_per_descriptor": BOW_BYTES_PER_DESC,
                        "cache_served_vocabulary_bytes_per_s": round(
                            n_desc * BOW_VOCAB_BYTES_PER_DESC / (t_ms * 1e-3)),
                        "note": "compulsory HBM bytes only; the 6-level descent's vocabulary "
                                "reads (2880 B per descriptor) are L2/MALL hits"},
           "cpu_baseline": None}
    if with_cpu:
        import concurrent.futures as cf
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        O.build()
        ov = O.OracleVocab(V)
        frames = [ctx.keypoints(2 * f) for f in range(min(Bs, 17))]
        threads = host_cpu_share()[0]
        per = 4

        def work(tid):
            for i in range(per):
                f = (tid + i) % (len(frames) - 1)
                wa = O.bow_transform(ov, frames[f][1], 4)
                wb = O.bow_transform(ov, frames[f + 1][1], 4)
                O.search_by_bow(frames[f][1], frames[f][0], valid[f][:len(frames[f][1])],
                                wa[2:], frames[f + 1][1], frames[f + 1][0], None, wb[2:], False,
                                0.7, True)
            return per
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            done = sum(ex.map(work, range(threads)))
        wall = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(done / wall, 1), "unit": "frames/s",
                               "cores": threads, "kind": "port",
                               "sample": f"{done} frames ({threads} threads x {per}): transform "
                                         "of two frames + SearchByBoW; oracle/bow_oracle.c"}
    out["keyframe_matchers"] = bench_kfmatch(ctx, Bs, dev, view, sets, with_cpu)
    return out


def bench_kfmatch(ctx, Bs, dev, view, sets, with_cpu):
    """SURVEY.md section 8(f) row 3 on the same batch, every frame taken as a keyframe at the
    pose it was rendered at (synthetic.layered_pose: turning + 0.3 m forward per frame):
    SearchForTriangulation(KF f, KF f+1) with 30% of the keypoints already carrying map points,
    and Fuse of KF f's stereo points (unprojected from its depths) into KF f+1, th = 3."""
    import torch
    from slam_framework_amd import kfmatch as K
    from slam_framework_amd import synthetic as S
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import kf_scenario as KS

    kc = view.kp_cap
    D = 16

    def layered_T(t):
        R, tc = S.layered_pose(t)
        T = np.eye(4, dtype=np.float32)
        T[:3, :3], T[:3, 3] = R, tc
        return T
    Ts = [layered_T(f % D) for f in range(Bs)]
    host = [ctx.keypoints(2 * f) for f in range(Bs)]
    depth = [ctx.stereo(f)[1] for f in range(Bs)]
    nn = sets.n_nodes.cpu().numpy()
    rng = np.random.default_rng(5)
    has_mp = torch.from_numpy((rng.random((Bs, kc)) < 0.3).astype(np.uint8)).to(dev)
    kfs = np.zeros(Bs, K.KF_DTYPE)
    for f in range(Bs):
        h = K.host_kf(host[f][0][:1], host[f][1][:1], np.zeros(1, np.float32), Ts[f])[0]
        kfs[f]["kps"] = view.kps + 2 * f * kc * 28
        kfs[f]["desc"] = view.desc + 2 * f * kc * 32
        kfs[f]["u_right"] = view.u_right + f * kc * 4
        kfs[f]["has_mp"] = int(has_mp.data_ptr()) + f * kc
        for k, a in sets.view_of(f).items():
            if k != "n_nodes":
                kfs[f][k] = a
        kfs[f]["n"], kfs[f]["n_nodes"] = len(host[f][1]), nn[f]
        kfs[f]["Rcw"], kfs[f]["tcw"], kfs[f]["Ow"] = list(h.Rcw), list(h.tcw), list(h.Ow)
    d_kfs = torch.from_numpy(kfs.view(np.uint8).copy()).to(dev)
    # Fuse projects KF f's points with the poses the frames were rendered at
    Tr = Ts
    d_kfs_r = d_kfs
    pairs = np.zeros(Bs - 1, K.TRI_PAIR_DTYPE)
    for f in range(Bs - 1):
        pairs[f] = (f, f + 1, KS.fundamental(Ts[f], Ts[f + 1]).reshape(-1), 0)
    d_pairs = torch.from_numpy(pairs.view(np.uint8).copy()).to(dev)
    d_m = torch.empty((Bs - 1, kc), dtype=torch.int32, device=dev)
    d_nm = torch.empty(Bs - 1, dtype=torch.int32, device=dev)
    lv = K.levels()
    stream = torch.cuda.current_stream()

    def tri():
        K.search_for_triangulation_device(d_kfs, d_pairs, Bs - 1, S.KITTI_CAM, lv, True, d_m, kc,
                                          d_nm, stream.cuda_stream)
    # Fuse points of KF f into KF f + 1
    pts, pkf = [], []
    for f in range(Bs - 1):
        p = KS.fuse_points({"kps": host[f][0], "desc": host[f][1], "depth": depth[f]}, Tr[f],
                           n_extra=0)
        pts.append(p)
        pkf.append(np.full(len(p), f + 1, np.int32))
    pts, pkf = np.concatenate(pts), np.concatenate(pkf)
    d_pts = torch.from_numpy(pts.view(np.uint8).copy()).to(dev)
    d_pkf = torch.from_numpy(pkf).to(dev)
    d_bi = torch.empty(len(pts), dtype=torch.int32, device=dev)
    d_bd = torch.empty(len(pts), dtype=torch.int32, device=dev)
    grid = K.kf_grid(S.KITTI_COLS, S.KITTI_ROWS)

    def fuse():
        K.fuse_device(d_kfs_r, d_pts, d_pkf, len(pts), 3.0, S.KITTI_CAM, lv, grid, d_bi, d_bd,
                      stream.cuda_stream)
    tri()
    fuse()
    torch.cuda.synchronize()
    t_ms, f_ms = _events_ms(tri, stream, 5), _events_ms(fuse, stream, 5)
    nm, bi = d_nm.cpu().numpy(), d_bi.cpu().numpy()
    out = {"workload": "SURVEY 8(f) row 3: SearchForTriangulation(KF f, KF f+1) and Fuse(KF f+1, "
                       "KF f's stereo points, th 3) over the batch, from the frontend's device "
                       "outputs and the BoW leg's FeatureVectors",
           "pairs": Bs - 1, "triangulation_ms": round(t_ms, 3),
           "triangulation_pairs_per_s": round((Bs - 1) / t_ms * 1e3, 1),
           "triangulation_matches_per_pair": round(float(nm.mean()), 1),
           "fuse_points": int(len(pts)), "fuse_ms": round(f_ms, 3),
           "fuse_points_per_s": round(len(pts) / f_ms * 1e3),
           "fused_per_keyframe": round(float((bi >= 0).sum()) / (Bs - 1), 1),
           "cpu_baseline": None}
    if with_cpu:
        import concurrent.futures as cf
        import oracle_lib as O
        O.build()
        sc, s2, isg, _ = KS.levels_arrays()
        g = O.grid_geom(S.KITTI_COLS, S.KITTI_ROWS)
        ur = [ctx.stereo(f)[0] for f in range(min(Bs, 17))]
        mp = has_mp.cpu().numpy()
        fvs = [sets.host(f)[1].arrays() for f in range(min(Bs, 17))]
        kd = [dict(kps=host[f][0], desc=host[f][1], ur=ur[f], mp=mp[f][:len(host[f][1])],
                   fv=fvs[f]) for f in range(min(Bs, 17))]
        threads = host_cpu_share()[0]
        per = 4

        def work(tid):
            for i in range(per):
                f = (tid + i) % (len(kd) - 1)
                T2 = Ts[f + 1]
                T2w = np.concatenate([T2[:3, :3].reshape(-1), T2[:3, 3]]).astype(np.float32)
                O.search_for_triangulation(kd[f], kd[f + 1], kfs[f]["Ow"], T2w, S.KITTI_CAM[:4],
                                           sc, s2, pairs[f]["F12"], 0, 1)
                sel = pkf == f + 1
                O.fuse(kd[f + 1]["kps"], kd[f + 1]["desc"], kd[f + 1]["ur"], g,
                       Tr[f + 1][:3, :3].reshape(-1), Tr[f + 1][:3, 3], kfs[f + 1]["Ow"],
                       S.KITTI_CAM, sc, isg,
                       float(lv.log_scale_factor), pts[sel], 3.0)
            return per
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            done = sum(ex.map(work, range(threads)))
        wall = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(done / wall, 1), "unit": "keyframe pairs/s",
                               "cores": threads, "kind": "port",
                               "sample": f"{done} pairs ({threads} threads x {per}): "
                                         "SearchForTriangulation + Fuse; oracle/kfmatch_oracle.c"}
    return out


def cpu_model():
    """The host CPU's model name (lscpu's "Model name") and logical CPU count."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip(), os.cpu_count()
    except OSError:
        pass
    return None, os.cpu_count()


def host_cpu_share():
    """(usable threads, evidence): the CPUs this process may run on (sched affinity), capped by
    the GPU pool's per-GPU CPU share, which the box advertises through OMP_NUM_THREADS (16 per
    GPU; os.cpu_count() there reports the whole machine); plus the cgroup CPU quota if any."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    share = int(os.environ.get("OMP_NUM_THREADS") or 0) or aff
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    n = min(aff, share, int(quota) if quota else aff)
    return max(1, n), {"affinity_cpus": aff, "omp_num_threads": share, "cgroup_cpu_quota": quota}


def build_native_oracle():
    """gcc -O3 -march=native build of oracle/ for THIS host's CPU (oracle/Makefile `native`),
    into a temporary directory; returns its path."""
    import subprocess
    import tempfile
    out = os.path.join(tempfile.mkdtemp(prefix="slamgpu_oracle_"), "liborb_oracle_native.so")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native",
                    f"NATIVE_OUT={out}"], check=True, stdout=subprocess.DEVNULL,
                   stderr=subprocess.DEVNULL)
    return out


def cpu_baseline(Ls, Rs, n_frames, device_check=None):
    """The oracle/ restatement (C) built -O3 -march=native for this host on host threads:
    throughput -- each thread runs its own consecutive frames (extract L+R, stereo,
    frame-to-frame search against the previous frame's stereo points), wall time over all -- at
    the thread count a sweep over 1, 2, 4, ... up to the host's CPU share picks (the sweep is in
    the result); reference threading -- one frame at a time, its left and right extraction on
    two threads as the stereo Frame ctor runs them (frame.cpp:86-89), then stereo and search.
    device_check: (render index, keypoints, descriptors) of a left view from the device, which
    the native build must reproduce byte for byte before it is timed."""
    import concurrent.futures as cf

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    import scenario
    from slam_framework_amd import synthetic as S
    from slam_framework_amd.sharded import render_of

    O.build()
    native = None
    if O._lib is None:
        try:
            native = build_native_oracle()
            O.use_lib(native)
        except Exception as e:  # no gcc on the host: the prebuilt x86-64-v3 build
            print(f"cpu_baseline: native build failed ({e}); using liborb_oracle_fast.so",
                  file=sys.stderr)
            O.use_fast()
    t = O.tables()
    g = O.grid_geom(S.KITTI_COLS, S.KITTI_ROWS)
    cam = S.KITTI_CAM
    D = len(Ls)
    identical = None
    if device_check is not None:
        f, dk, dd = device_check
        kl, dl, _ = O.extract(t, Ls[f], True)
        identical = kl.tobytes() == dk.tobytes() and np.array_equal(dl, dd)
        if not identical:
            raise SystemExit("cpu_baseline: the native oracle build differs from the device")

    def search(f, kl, dl, ur, prev):
        q, lmp, lout, xyz, md, nobs = scenario.vo_queries(prev[0], prev[1], prev[2], prev[3],
                                                          layered=True)
        p = scenario.pose(f, layered=True, t_last=prev[3])
        mp = np.full(len(kl), -1, np.int32)
        O.search_frame(t, g, kl, dl, ur, mp, prev[0], lmp, lout, xyz, md, nobs,
                       p["Rcw"][0].reshape(3, 3), p["tcw"][0], float(p["tlc_z"][0]),
                       float(p["baseline"][0]), cam, 7.0, 0, 1)

    def throughput(threads, per_thread):
        def run(tid):
            prev = None
            for k in range(per_thread):
                f = render_of(tid * per_thread + k, D)  # the bench's back-and-forth order
                kl, dl, pl = O.extract(t, Ls[f], True)
                kr, dr, pr = O.extract(t, Rs[f], True)
                ur, depth, _ = O.stereo(t, kl, dl, kr, dr, pl, pr, cam[0], cam[4])
                if prev is not None:
                    search(f, kl, dl, ur, prev)
                prev = (kl, dl, depth, f)
            return per_thread
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            done = sum(ex.map(run, range(threads)))
        return done, time.perf_counter() - t0

    max_threads, share = host_cpu_share()
    sweep = {}
    tc = 1
    while True:
        done, wall = throughput(tc, 3)
        sweep[tc] = round(done / wall, 2)
        if tc >= max_threads:
            break
        tc = min(2 * tc, max_threads)
    threads = max(sweep, key=sweep.get)
    # a ~15 s sample at the chosen thread count (n_frames overrides)
    per_thread = max(2, (n_frames or int(15 * sweep[threads])) // threads)
    done, wall = throughput(threads, per_thread)

    # the reference's own threading: frames in sequence, L and R extracted concurrently
    n_seq = 24
    prev = None
    t1 = time.perf_counter()
    with cf.ThreadPoolExecutor(2) as ex:
        for k in range(n_seq):
            f = render_of(k, D)
            fl, fr = ex.submit(O.extract, t, Ls[f], True), ex.submit(O.extract, t, Rs[f], True)
            (kl, dl, pl), (kr, dr, pr) = fl.result(), fr.result()
            ur, depth, _ = O.stereo(t, kl, dl, kr, dr, pl, pr, cam[0], cam[4])
            if prev is not None:
                search(f, kl, dl, ur, prev)
            prev = (kl, dl, depth, f)
    seq = time.perf_counter() - t1
    model, ncpu = cpu_model()
    return {"value": round(done / wall, 2), "unit": "stereo frames/s", "cores": threads,
            "kind": "port", "cpu_model": model, "host_logical_cpus": ncpu,
            "cpu_share": share,
            "thread_sweep_frames_per_s": {str(k): v for k, v in sweep.items()},
            "threads_chosen_by": "best of the sweep over 1..min(affinity, OMP_NUM_THREADS, cgroup "
                                 "quota): the GPU pool gives each GPU's jobs a 16-CPU share of "
                                 "the host (cgroup cpu.max), so more threads only time-slice",
            "build": ("gcc -O3 -march=native -ffp-contract=off (oracle/Makefile native, built on "
                      "this host)" if native else
                      "oracle/liborb_oracle_fast.so: gcc -O3 -march=x86-64-v3 -ffp-contract=off"),
            "native_matches_device": identical,
            "sample": f"{done} synthetic stereo frames ({threads} threads x {per_thread}); "
                      f"oracle/ C restatement: extract L+R + stereo + frame-to-frame",
            "wall_s": round(wall, 2),
            "reference_threading": {
                "value": round(n_seq / seq, 2), "unit": "stereo frames/s", "cores": 2,
                "ms_per_frame": round(1e3 * seq / n_seq, 2),
                "sample": f"{n_seq} frames in sequence, left/right extraction on 2 threads "
                          "(frame.cpp:86-89), then stereo + frame-to-frame search"}}


if __name__ == "__main__":
    main()
