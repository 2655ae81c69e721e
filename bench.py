"""Benchmark: frames/sec of the extract -> match hot path (BASELINE.json configs[1]).

One STEP = one candidate search of the reference's findGoodFrameFromBatch
(batch.cpp:59-99) over a batch of `--batch` (default 210, the reference
README's framesBatchSize and configs[3]'s) 1920x1080 BGR frames already in HBM:
gray + FAST-9 + SIFT descriptors for every candidate, BF-L2 kNN (k = 2) + ratio
test (knnMatcherDistance 0.7) of every candidate against the previous good
frame's descriptors, the selection rule on the host, the winner's keypoints and
matches returned to the host, and hand-over of the winner's descriptors as the
next step's query set.  BA is off in this config (configs[1]); `with_ba` /
`value_with_ba` add a BAMaxFramesCnt = 8 window per 8 searches.  A frame = one
candidate processed end to end; value = frames / s over all ranks.

Multi-GPU (torchrun, one rank per GPU, RCCL): the global batch is sharded,
candidate k on rank k % world (the reference's thread stride, batch.cpp:183-187;
ragged when world does not divide it), so the total work per step is fixed
(strong scaling); per step the previous good frame's descriptors are broadcast
from the rank that found them, the per-candidate counts are all-gathered so
every rank makes the same selection, and the winner's keypoints and matches are
broadcast device to device from its owner.

Roofline: HIP events bracket every launch of each kernel family on the launch
stream inside the timed region; the dominant family is reported against its
bound (kNN: int8 MFMA dense peak; FAST: HBM).  cpu_baseline: the oracle's
restatement of the reference's useFM-SIFT-FLANN CPU path (gray, FAST, SIFT,
FLANN-style KD-forest kNN, ratio) on a bounded sample of the same frames.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))

W, H = 1920, 1080
THRESHOLD = 33            # FAST threshold giving 10k +- 6 % keypoints on every frame of the steady 1080p sequence
PIPE_THRESHOLD = 31       # the pipeline leg's drift-path frames 100..123 (~9k keypoints)
SYNTH_PATH = 1            # slamhip.SYNTH_STEADY: a bounded camera loop, every candidate near 10k keypoints
RATIO = 0.7
REQUIRED_MATCHES = 500    # requiredMatchedPointsCount of the reference's example config (README.md)
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8 TB/s HBM3E
I8_MFMA_PEAK_TOPS = 5000.0  # dense int8 MFMA: 2x the ~2.5 PF dense bf16 rate (MI355X_MICROARCH.md, Matrix cores)
F32_VALU_PEAK_TF = 157.3    # MI355X_MICROARCH.md: peak FP32 vector
# calcSIFTDescriptor f32 operations per contributing window sample (DESIGN.md
# "SIFT descriptor"): rotation 6, bin coords 4, exp argument 4, exp32f 12,
# obin + weighted magnitude 3, fractional parts 3, trilinear split 14, 8 adds
SIFT_FLOP_PER_SAMPLE = 54
# SURVEY.md 8(d)'s own count ("N x ~2.8k contributing samples x ~40 flop"): the
# headline roofline's `frac` follows it; the 54-flop count
# above is reported beside it as `frac_54flop`
SIFT_FLOP_PER_SAMPLE_SURVEY = 40
LDS_READ_B64_TBS = 150.0      # 256 B/clk/CU x 256 CUs x 2.4 GHz (guide: ~150 TB/s chip-wide)
LDS_WRITE_B64_TBS = 52.2      # ~85 B/clk/CU (6 cycles per wave-instruction) x 256 x 2.4 GHz
FAMILIES = {0: "fast_detect", 1: "sift_desc", 2: "knn_mfma", 3: "orb_desc", 4: "sift_blur_grad", 5: "knn_finish"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=210,
                    help="candidate frames per search over all GPUs (framesBatchSize; 210 = the reference README)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the ORB and BA legs")
    ap.add_argument("--overlap", default="desc_start", choices=["knn", "desc_end", "desc_start"],
                    help="where the next search's extraction may start (PipelinedScan overlap)")
    ap.add_argument("--sift-kernel", default="auto", choices=["auto", "colw", "band", "tab"],
                    help="SIFT descriptor kernel for FAST keypoints (all bit-identical; auto = band)")
    ap.add_argument("--check-launch", action="store_true",
                    help="launch the ranks, shard the batch and print the rank layout, no GPU work "
                         "(gloo; the CPU test of the launcher)")
    return ap.parse_args()


def launch(args):
    """`--gpus N` without a torch.distributed launcher: start N ranks as a child
    `torch.distributed.run` (before anything touches the GPU) and exit with its
    status; the child's rank 0 prints the JSON line.  Under a launcher, WORLD_SIZE
    must equal --gpus (a mismatch would print a line for the wrong rank count)."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None:
        if args.gpus > 1:
            import socket
            import subprocess
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
                   "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
            sys.exit(subprocess.call(cmd))
        return
    if int(world_env) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world_env} ranks")


def check_launch(args):
    """the rank layout of a launch, without GPU work: every rank's candidate
    shard (k -> rank k % world) gathered over gloo, printed by rank 0"""
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
    mine = [k for k in range(args.batch) if k % world == rank]
    info = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "candidates": len(mine),
            "first": mine[0] if mine else None}
    allinfo = [None] * world
    if world > 1:
        dist.all_gather_object(allinfo, info)
    else:
        allinfo = [info]
    if rank == 0:
        print(json.dumps({"metric": "launch check", "n_gpus": world,
                          "world_size": dist.get_world_size() if world > 1 else 1,
                          "frames_per_step": args.batch, "ranks": allinfo}))
    if world > 1:
        dist.destroy_process_group()


def sift_samples_per_kp(size=7.0, angle=-1.0):
    """window samples inside the 4x4 histogram footprint (rbin, cbin in (-1, 4))
    for FAST keypoints, the per-keypoint work unit of the descriptor kernel"""
    f = np.float32
    ori = f(360.0) - f(angle)
    hist_width = f(3.0) * f(size) * f(0.5)
    radius = int(np.rint(hist_width * f(1.4142135623730951) * f(2.5)))
    cos_t = f(np.cos(np.float32(ori * f(np.pi / 180)))) / hist_width
    sin_t = f(np.sin(np.float32(ori * f(np.pi / 180)))) / hist_width
    i, j = np.mgrid[-radius:radius + 1, -radius:radius + 1].astype(np.float32)
    c_rot = j * cos_t - i * sin_t
    r_rot = j * sin_t + i * cos_t
    rb, cb = r_rot + f(1.5), c_rot + f(1.5)
    return int(np.count_nonzero((rb > -1) & (rb < 4) & (cb > -1) & (cb < 4)))


def orb_leg(pscan, db, frames, first, batch, pad_to, steps, warmup):
    """configs[2]'s front end (ORB FAST-9 + rBRIEF + Hamming BF, ratio 0.7) on the
    same resident frames: candidate frames per second of one search per step
    (the headline's PipelinedScan searches, counts exchanged and the frame
    selected; the query stays the first frame's descriptors)."""
    import torch
    import slamhip
    from slamhip.batch import Conditions
    db.extract(first, THRESHOLD, slamhip.ORB_BF)
    prev = torch.zeros(slamhip.lib().slam_batch_desc_bytes(slamhip.ORB_BF, 64 * 1024), dtype=torch.uint8,
                       device=frames.device)
    _, nprev = db.export_desc(0, prev)
    cond = Conditions(featureExtractingThreshold=THRESHOLD, requiredExtractedPointsCount=0, frameBatchSize=batch,
                      requiredMatchedPointsCount=REQUIRED_MATCHES, matcherType=slamhip.ORB_BF,
                      knnMatcherDistance=RATIO)

    def run(n):
        for i in range(n):
            pscan.search(frames, prev, nprev, 0, cond, pad_to=pad_to, next_frames=frames if i + 1 < n else None)

    run(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"config": "configs[2] front end: ORB FAST-9 + rBRIEF + Hamming BF kNN k=2, ratio 0.7, 1920x1080; "
                      "step = one pipelined search (extract + match + counts + selection)",
            "frames_per_s": frames.shape[0] * steps / el, "ms_per_step": el / steps * 1e3,
            "mean_kps_after_border_filter": float(np.mean(pscan.db.batch_counts())), "prev_kps": nprev}


def sift4k_leg(ctx, steps=8, warmup=2, nframes=16, target=20000, check=True):
    """configs[4]'s front end on one GPU: 3840x2160 SIFT + BF-L2 kNN k=2, ratio
    0.7, with the FAST threshold bisected on frame 0 to ~20k keypoints (SURVEY
    8(d): target +-10 %); candidate frames per second of one search per step."""
    import torch
    import slamhip
    from slamhip.batch import DeviceBatch
    w4, h4 = 3840, 2160
    db = DeviceBatch(ctx)
    host = synth(0, nframes + 1, w4, h4)
    frames = torch.from_numpy(host[1:]).cuda()
    first = torch.from_numpy(host[:1]).cuda()
    lo, hi = 1, 255                               # FAST count falls as the threshold rises
    while lo < hi:
        mid = (lo + hi) // 2
        if db.extract(first, mid, slamhip.SIFT_FLANN)[0] > target:
            lo = mid + 1
        else:
            hi = mid
    thr = lo if abs(db.extract(first, lo, slamhip.SIFT_FLANN)[0] - target) <= \
        abs(db.extract(first, max(lo - 1, 1), slamhip.SIFT_FLANN)[0] - target) else max(lo - 1, 1)
    n0 = db.extract(first, thr, slamhip.SIFT_FLANN)[0]
    prev = torch.zeros(slamhip.lib().slam_batch_desc_bytes(slamhip.SIFT_FLANN, 256 * 1024), dtype=torch.uint8,
                       device=frames.device)
    _, nprev = db.export_desc(0, prev)
    # the headline's pipelined searches (two contexts, desc_start overlap); the
    # query stays frame 0's descriptors, as the checked step below assumes
    from slamhip.batch import Conditions, PipelinedScan
    pscan = PipelinedScan(0, 1, frames.device.index or 0, overlap="desc_start")
    cond = Conditions(featureExtractingThreshold=thr, requiredExtractedPointsCount=0, frameBatchSize=nframes,
                      requiredMatchedPointsCount=REQUIRED_MATCHES, matcherType=slamhip.SIFT_FLANN,
                      knnMatcherDistance=RATIO)

    def run(n):
        kp_all = None
        for i in range(n):
            _, kp_all, _, _, _ = pscan.search(frames, prev, nprev, 0, cond, pad_to=nframes,
                                              next_frames=frames if i + 1 < n else None)
        return kp_all

    run(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kp = run(steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    db = pscan.db                                  # the last search's batch (checked below)
    out = {"config": "configs[4] front end on one GPU: SIFT + BF-L2 kNN k=2, ratio 0.7, 3840x2160, FAST threshold "
                     "bisected on frame 0 to ~20k keypoints; step = one pipelined search over the 16 frames",
           "frames_per_s": nframes * steps / el, "ms_per_step": el / steps * 1e3, "frames_per_step": nframes,
           "fast_threshold": int(thr), "frame0_kps": int(n0), "mean_kps": float(np.mean(kp)), "prev_kps": nprev}
    if check:
        # the last step's first candidate against the oracle: FAST keypoints, SIFT
        # descriptors, and the ~20k x 20k kNN (packed-key splits merged by
        # knn_finish) + ratio test, all bit-exact
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ffi as O
        kq = O.fast(host[0], thr, True)
        dq = O.sift(host[0], kq)
        k1 = O.fast(host[1], thr, True)
        d1 = O.sift(host[1], k1)
        ri, rd = O.knn2(dq, d1, O.NORM_L2)
        ref_m = O.ratio(ri, rd, RATIO)
        gk = db.keypoints(0)
        kp_ok = len(gk) == len(k1) and all(np.array_equal(gk[f], k1[f]) for f in ("x", "y", "response"))
        desc_ok = kp_ok and np.array_equal(db.descriptors(0), d1)
        gm = db.matches(0, nprev)
        out["oracle"] = {"frame": 1, "keypoints": int(len(k1)), "query": int(len(kq)), "matches": int(len(ref_m)),
                         "keypoints_ok": bool(kp_ok), "descriptors_ok": bool(desc_ok),
                         "matches_ok": bool(np.array_equal(gm, ref_m)), "bar": "bit-exact"}
        out["oracle"]["parity_ok"] = out["oracle"]["keypoints_ok"] and out["oracle"]["descriptors_ok"] and \
            out["oracle"]["matches_ok"]
    pscan.close()
    return out


def ba_window(nframes=8, npoints=10000, k4k=False):
    from slamhip import synthba
    kw = dict(width=3840, height=2160, K4=synthba.K_4K) if k4k else {}
    return synthba.make_window(nframes=nframes, npoints=npoints, seed=7, **kw)


def ba_oracle(w):
    """oracle/ba.c on a window (the checker of ba_leg, and its CPU baseline):
    (summary, seconds)"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    t0 = time.perf_counter()
    r = O.ba(w["K4"], w["ext"], w["pts"], w["obs_frame"], w["obs_point"], w["obs_xy"], O.LOSS_HUBER, 4.0)
    return r[3], time.perf_counter() - t0


def ba_leg(ctx, nframes=8, npoints=10000, k4k=False, reps=5, check=True):
    """One BAMaxFramesCnt window on the GPU: W = 8 at 1080p (configs[2]/[3]) or
    W = 16 at 4K with samsung-hv-4k intrinsics (configs[4]); synthetic scene with
    the reference's observation pattern (slamhip/synthba.py), Huber 4.0, Ceres LM
    defaults.  RMSE as the reference logs it: sqrt(cost / #residuals).  check:
    the same window through the oracle; final cost and RMSE compared (bars of
    tests/test_gpu_parity.py: 1e-6 relative, 1e-4 px)."""
    import math
    import torch
    import slamhip
    w = ba_window(nframes, npoints, k4k)
    times, sm = [], None
    for rep in range(reps + 1):                  # the first solve includes code-object load warm-up
        K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sm = slamhip.bundle_adjust_arrays(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"],
                                          slamhip.LOSS_HUBER, 4.0, ctx=ctx)
        if rep:
            times.append(time.perf_counter() - t0)
    rmse = math.sqrt(sm.final_cost / max(1, sm.num_residuals))
    out = {"frames": nframes, "points": int(w["pts"].shape[0]), "observations": int(len(w["obs_frame"])),
           "loss": "huber 4.0", "ms_per_window": float(np.median(times)) * 1e3,
           "ms_per_window_min": float(np.min(times)) * 1e3, "iterations": int(sm.iterations),
           "initial_rmse": math.sqrt(sm.initial_cost / max(1, sm.num_residuals)), "final_rmse": rmse,
           "final_cost": sm.final_cost, "usable": bool(sm.usable)}
    if check:
        rs, el = ba_oracle(w)
        r_rmse = math.sqrt(rs.final_cost / max(1, rs.num_residuals))
        out["oracle"] = {"final_cost": rs.final_cost, "final_rmse": r_rmse, "iterations": int(rs.iterations),
                         "final_cost_rel_diff": abs(sm.final_cost - rs.final_cost) / rs.final_cost,
                         "rmse_abs_diff_px": abs(rmse - r_rmse),
                         "parity_ok": bool(abs(sm.final_cost - rs.final_cost) <= 1e-6 * rs.final_cost + 1e-9
                                           and abs(rmse - r_rmse) <= 1e-4)}
        out["cpu_baseline"] = {"ms_per_window": el * 1e3, "iterations": int(rs.iterations), "cores": 1,
                               "kind": "port", "cpu_model": cpu_model(),
                               "sample": f"the same {nframes}-frame window, {out['points']} points, Huber 4.0; "
                                         "oracle/ba.c is single-threaded (the reference runs Ceres on "
                                         "BAThreadsCnt threads)"}
        out["speedup_vs_cpu_baseline"] = el * 1e3 / out["ms_per_window"]
    return out


def with_ba_leg(pscan, scan, frames, first, batch, pad_to, matcher, outer=4, W=8, check=False):
    """extract + match + BA end to end on the resident frames, the metric's
    "(extract+match+BA)": SIFT + BF-L2 (configs[3]: framesBatchSize 210 sharded
    over the ranks, RCCL exchanges, BA on) or ORB FAST-9 + rBRIEF + Hamming BF
    (configs[2]).  One outer step = W = BAMaxFramesCnt
    searches (each over the global batch of candidates, winner handed over as
    the next query) + one BA solve of a W-frame window (non-overlapping
    windows, mainCycle.cpp:201-210): the synthetic 1080p window of ba_leg (10k
    points, Huber 4) stands for the window the W good frames build.

    The searches run through the headline's PipelinedScan (each search's
    extraction queued on the other context while the host takes the previous
    one); the outer steps' boundaries queue nothing ahead, so the timed region
    holds exactly its searches' extractions.

    BA overlaps the searches: the next findGoodFrameFromBatch needs only the
    previous good frame (mainCycle.cpp:117-123), and the first consumer of BA's
    K and points is the PnP after it (:155-161), so window k is solved on its
    own context (own HIP stream, host thread) while window k + 1's searches
    run; window k + 1's solve starts after window k's has been taken (windows
    are sequential: K and points mutate in place).  With more ranks one rank
    (0) solves and broadcasts K / extrinsics / points (replicas only, SURVEY
    8(e)).  The last window is taken inside the timed region.  frames/s = W x
    global batch candidate frames per outer step; good frames/s = the W
    winners per outer step (one per search, whatever the rank count)."""
    import math
    from concurrent.futures import ThreadPoolExecutor
    import torch
    import torch.distributed as dist
    import slamhip
    from slamhip.batch import Conditions
    db = scan.db
    db.extract(first, THRESHOLD, matcher)
    prev = torch.zeros(slamhip.lib().slam_batch_desc_bytes(matcher, 64 * 1024), dtype=torch.uint8,
                       device=frames.device)
    _, nprev = db.export_desc(0, prev)
    cond = Conditions(featureExtractingThreshold=THRESHOLD, requiredExtractedPointsCount=0, frameBatchSize=batch,
                      requiredMatchedPointsCount=REQUIRED_MATCHES, matcherType=matcher,
                      knnMatcherDistance=RATIO)
    w = ba_window()
    owner = 0
    ba_ctx = slamhip.Context(frames.device.index or 0) if scan.rank == 0 else None
    pool = ThreadPoolExecutor(1) if scan.rank == 0 else None
    npts = w["pts"].shape[0]
    sol = torch.empty(4 + 6 * W + 3 * npts, dtype=torch.float64, device=frames.device)

    def solve():
        K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
        sm = slamhip.bundle_adjust_arrays(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"],
                                          slamhip.LOSS_HUBER, 4.0, ctx=ba_ctx)
        return sm, K4, ext, pts

    def take(fut):
        """the window's K / extrinsics / points on every rank"""
        out = fut.result() if fut is not None else None
        if scan.world > 1:
            if out is not None:
                sol.copy_(torch.from_numpy(np.concatenate([out[1], out[2].ravel(), out[3].ravel()])))
            dist.broadcast(sol, src=0)
        return out

    t_search = t_wait = 0.0
    sm = None
    fut = None
    for k in range(outer + 1):
        if k == 1:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            t_search = t_wait = 0.0
        ts = time.perf_counter()
        for i in range(W):
            edge = i == W - 1 and k in (0, outer)       # nothing queued across the timed region's edges
            good, kp_all, mc_all, in_batch, dc_all = pscan.search(frames, prev, nprev, owner, cond, pad_to=pad_to,
                                                                  next_frames=None if edge else frames)
            owner, nprev = pscan.advance(good, in_batch, dc_all, prev, owner, nprev)
        tb = time.perf_counter()
        if k > 0 or fut is not None:
            r = take(fut)
            if r is not None:
                sm = r[0]
        te = time.perf_counter()
        fut = pool.submit(solve) if pool is not None else None
        t_search += tb - ts
        t_wait += te - tb
    r = take(fut)
    if r is not None:
        sm = r[0]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if pool is not None:
        pool.shutdown()
        ba_ctx.close()
    nf = W * batch * outer
    name = ("configs[2]: ORB FAST-9 + rBRIEF + Hamming BF kNN k=2" if matcher == slamhip.ORB_BF else
            f"configs[3]: SIFT + BF-L2 kNN k=2, framesBatchSize {batch} sharded over {scan.world} GPU(s)")
    out = {"config": f"{name}, ratio 0.7, 1920x1080, ~10k kpts, BA on (BAMaxFramesCnt={W}, Huber 4); outer step = "
                     f"{W} searches of {batch} candidates + one {W}-frame BA window (10k points) solved on its own "
                     "stream while the next window's searches run",
           "frames_per_s": nf / el, "good_frames_per_s": W * outer / el,
           "ms_per_outer_step": el / outer * 1e3, "search_ms_per_outer_step": t_search / outer * 1e3,
           "ba_wait_ms_per_outer_step": t_wait / outer * 1e3,
           "mean_kps_after_border_filter": float(np.mean(pscan.db.batch_counts()))}
    if sm is not None:
        out["ba_final_rmse"] = math.sqrt(sm.final_cost / max(1, sm.num_residuals))
        out["ba_solve_ms"] = sm.total_time_in_seconds * 1e3
        if check:
            # the same window through the oracle (oracle/ba.c, ba_leg's bars)
            rs, _ = ba_oracle(w)
            r_rmse = math.sqrt(rs.final_cost / max(1, rs.num_residuals))
            out["oracle"] = {"final_rmse": r_rmse, "rmse_abs_diff_px": abs(out["ba_final_rmse"] - r_rmse),
                             "final_cost_rel_diff": abs(sm.final_cost - rs.final_cost) / rs.final_cost,
                             "iterations": [int(sm.iterations), int(rs.iterations)]}
            out["oracle"]["parity_ok"] = bool(out["oracle"]["final_cost_rel_diff"] <= 1e-6 and
                                              out["oracle"]["rmse_abs_diff_px"] <= 1e-4)
    return out


def siftdet_leg(ctx, reps=6):
    """the full SIFT detector: siftDetectAndCompute per
    1080p frame through the host-buffer C ABI (image H2D, keypoints +
    descriptors D2H, host-side duplicate filter included)"""
    import slamhip
    frames = slamhip.synth_frames(W, H, 0, 3, seed=1234)
    slamhip.siftDetectAndCompute(frames[0], ctx=ctx)
    t0 = time.perf_counter()
    n = 0
    for r in range(reps):
        k, _ = slamhip.siftDetectAndCompute(frames[r % 3], ctx=ctx)
        n += len(k)
    el = time.perf_counter() - t0
    out = {"config": "cv::SIFT detectAndCompute defaults (3 layers, contrast 0.04, edge 10, sigma 1.6, "
                     "doubled base), 1920x1080, host buffers", "frames_per_s": reps / el,
           "ms_per_frame": el / reps * 1e3, "mean_kps": n / reps}
    # the device-resident batch path (slam_sift_detect_batch): 16 frames in HBM per
    # call, every pyramid / extrema / refinement / descriptor launch covers the batch;
    # keypoints and descriptors returned to the host as siftDetectAndCompute does
    import torch
    nb = 16
    dev = torch.from_numpy(slamhip.synth_frames(W, H, 0, nb, seed=1234)).cuda()
    slamhip.siftDetectAndComputeBatch(dev, ctx=ctx)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nk = 0
    breps = 8                              # ~11 ms per call: 8 calls keep the number steady
    for _ in range(breps):
        nk += int(slamhip.siftDetectAndComputeBatch(dev, ctx=ctx).counts.sum())
    el = time.perf_counter() - t0
    out["batch"] = {"config": f"the same detector over {nb} 1920x1080 frames resident in HBM per call "
                              "(slam_sift_detect_batch), keypoints and descriptors left in HBM",
                    "frames_per_s": breps * nb / el, "ms_per_frame": el / (breps * nb) * 1e3,
                    "mean_kps": nk / (breps * nb), "calls": breps}
    return out


def geom_leg(ctx, n=10000, reps=20):
    """two-view DLT triangulation (reconstruct, triangulate.cpp:74-100) of n
    matched points through the host-buffer C ABI"""
    import slamhip
    rng = np.random.default_rng(3)
    K = np.array([[1724.676, 0, 995.966], [0, 1730.482, 550.192], [0, 0, 1.0]])
    a = np.deg2rad(3.0)
    R2 = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    t2 = np.array([-0.2, 0.01, 0.02])
    X = np.stack([rng.uniform(-2, 2, n), rng.uniform(-1, 1, n), rng.uniform(3, 8, n)], 1)

    def proj(R, t):
        u = (X @ R.T + t) @ K.T
        return (u[:, :2] / u[:, 2:]).astype(np.float32)
    p1, p2 = proj(np.eye(3), np.zeros(3)), proj(R2, t2)
    slamhip.reconstruct(K, np.eye(3), np.zeros(3), R2, t2, p1, p2, ctx=ctx)
    t0 = time.perf_counter()
    for _ in range(reps):
        slamhip.reconstruct(K, np.eye(3), np.zeros(3), R2, t2, p1, p2, ctx=ctx)
    el = (time.perf_counter() - t0) / reps
    # estimateTransformation (findEssentialMat RANSAC + recoverPose) on the same
    # correspondences with 30 % of them replaced by outliers, 0.5 px noise
    q1 = p1 + rng.normal(0, 0.5, p1.shape).astype(np.float32)
    q2 = p2 + rng.normal(0, 0.5, p2.shape).astype(np.float32)
    bad = rng.random(n) < 0.3
    q2[bad] = rng.uniform([0, 0], [W, H], (int(bad.sum()), 2)).astype(np.float32)
    slamhip.estimateTransformation(q1, q2, K, ctx=ctx)
    t0 = time.perf_counter()
    for _ in range(5):
        ok, Rg, tg, cm, rm = slamhip.estimateTransformation(q1, q2, K, ctx=ctx)
    el_rp = (time.perf_counter() - t0) / 5
    rerr = float(np.degrees(np.arccos(np.clip((np.trace(Rg.T @ R2) - 1) / 2, -1, 1))))
    return {"config": f"reconstruct(): {n} matched points, host buffers", "ms_per_call": el * 1e3,
            "points_per_s": n / el,
            "relative_pose": {"config": f"estimateTransformation(): {n} matches, 30 % outliers, RANSAC 0.999 / 5 px "
                                        "(1000 speculative hypotheses)", "ms_per_call": el_rp * 1e3,
                              "ransac_inliers": int(rm.sum()), "rotation_error_deg": rerr},
            "scene": (K, R2, t2, p1, p2, q1, q2)}


K_1080 = np.array([[1724.676, 0, 995.966], [0, 1730.482, 550.192], [0, 0, 1.0]])   # config/samsung-hv.xml


def pipeline_cfg():
    import slamhip
    d = slamhip.reference_example()
    d.update({"featureExtractingThreshold": PIPE_THRESHOLD, "requiredExtractedPointsCount": 1000, "framesBatchSize": 2,
              "requiredMatchedPointsCount": REQUIRED_MATCHES, "useFM-SIFT-FLANN": False, "useFM-ORB": True,
              "useBundleAdjustment": True, "BAMaxFramesCnt": 8})
    return slamhip.ConfigService(d)


PIPE_RUNS = 5          # timed runs of the 24-frame pipeline leg (median reported)


def pipeline_leg(ctx, nframes=24):
    """the reference's whole per-frame pipeline (slamhip.cycle: mainCycle / slamMain)
    on a 1080p synthetic sequence with configs[2]'s settings (ORB + Hamming BF,
    BA on, BAMaxFramesCnt 8, Huber 4): FAST batch filter, candidate search, first
    pair (essential RANSAC + recoverPose + triangulation), PnP RANSAC +
    triangulation per good frame, BA windows, output structures.  Frames are
    uploaded to HBM once (GpuOps.ingest) and each search is one device pass
    (GpuOps.search); poses, points and BA are compared with the oracle run."""
    import slamhip
    from slamhip import cycle
    frames = slamhip.synth_frames(W, H, 100, nframes, seed=1234)
    # warm-up: one whole run on the ops object the timed run uses, so its
    # post-search and BA worker contexts exist and every buffer (BA windows
    # included: the first opens at frame 8) has its size before the clock starts
    # (the query cache keys on the device frame, so no result carries over)
    gops = cycle.GpuOps(ctx)
    cycle.slam_main(cycle.MediaSources(frames), K_1080.copy(), pipeline_cfg(), gops)
    stats = {"record_ba": True}

    class Timed:
        """per-operation wall time of the run (host-side, includes the boundary copies)"""
        def __init__(self, ops):
            self.ops, self.t = ops, {}

        def __getattr__(self, name):
            f = getattr(self.ops, name)

            def g(*a, **k):
                t = time.perf_counter()
                r = f(*a, **k)
                self.t[name] = self.t.get(name, 0.0) + (time.perf_counter() - t) * 1e3
                return r
            return g
    ops = Timed(gops)
    t0 = time.perf_counter()
    gd, logs = cycle.slam_main(cycle.MediaSources(frames), K_1080.copy(), pipeline_cfg(), ops, stats=stats)
    el = time.perf_counter() - t0
    # the run is ~40 ms of host-threaded work, so one run's time moves with host
    # jitter (565-700 frames/s across runs of one tree): RUNS more identical
    # runs, the median reported beside every run's time; the first run's outputs
    # and per-operation times are the ones checked and reported
    els = [el]
    for _ in range(PIPE_RUNS - 1):
        t0 = time.perf_counter()
        cycle.slam_main(cycle.MediaSources(frames), K_1080.copy(), pipeline_cfg(), Timed(gops),
                        stats={"record_ba": True})      # the same wrapping as the first run
        els.append(time.perf_counter() - t0)
    el = sorted(els)[len(els) // 2]
    gops.close()
    import math
    by_op = {k: round(v, 2) for k, v in ops.t.items()}
    # BA windows solve on their own stream behind the next search (ba_async
    # returns at once): their GPU solve time is the summaries' own clock
    by_op["ba_solve"] = round(sum(s.total_time_in_seconds for s in stats.get("ba", [])) * 1e3, 2)
    return {"config": "slamMain/mainCycle end to end, configs[2] settings (ORB, BA on, BAMaxFramesCnt 8, Huber 4), "
                      f"1920x1080 synthetic, {nframes} frames, framesBatchSize 2, frames resident in HBM, each BA "
                      "window solved while the next search runs",
            "frames_per_s": nframes / el, "ms_per_frame": el / nframes * 1e3, "runs": len(els),
            "frames_per_s_runs": [round(nframes / e, 1) for e in els], "poses": len(logs.pose_list),
            "points": len(gd.spatialPoints), "ba_windows": len(stats.get("ba", [])),
            "ba_final_rmse": [math.sqrt(s.final_cost / max(1, s.num_residuals)) for s in stats.get("ba", [])],
            "ms_by_op": by_op, "frames": frames,
            "_result": (gd, logs, stats)}


EARLY_EXIT_CHUNK = 27     # pipeline_b210_early_exit: candidates per tail-first chunk (configs[3]'s per-rank shard at N = 8)


def pipeline_b210_leg(ctx, nframes=3800, check=True, orb=False, early_exit=0):
    """slamMain at the reference's example configuration (README.md:160-196:
    framesBatchSize 210, requiredMatchedPointsCount 500, knnMatcherDistance
    0.7, useFM-SIFT-FLANN, first fit) with BA on (BAMaxFramesCnt 8, Huber 4:
    configs[3] at N = 1; orb: useFM-ORB instead, configs[2] with the README's
    framesBatchSize) over the steady 1080p sequence, rendered into HBM
    before the run (the decoded video; slam_synth_sequence_dev): per search,
    fillVideoFrameBatch FAST-counts the frames the batch still needs in one
    device pass, every candidate is described and matched in one device pass,
    then PnP + triangulation of the good frame; every 8 good frames a BA window
    solved on its own stream while the next search runs.  Extract, match and
    BA all on the same frames.  frames_per_s = video frames consumed per second
    (each one FAST-filtered, described and matched at least once);
    candidate_frames_per_s counts every candidate evaluation.  early_exit = C:
    first-fit searches run tail-first in chunks of C candidates and stop at the
    first chunk that holds a qualifying one (the reference's single-thread
    break, batch.cpp:120-146; GpuOps(early_exit=C))."""
    import math
    import torch
    import slamhip
    from slamhip import cycle
    d = slamhip.reference_example()
    d.update({"featureExtractingThreshold": THRESHOLD, "requiredExtractedPointsCount": 9000, "framesBatchSize": 210,
              "requiredMatchedPointsCount": REQUIRED_MATCHES, "useFM-SIFT-FLANN": not orb, "useFM-SIFT-BF": False,
              "useFM-ORB": orb, "useBundleAdjustment": True, "BAMaxFramesCnt": 8, "knnMatcherDistance": RATIO})
    cfg = slamhip.ConfigService(d)
    dev = slamhip.synth_frames_dev(W, H, 0, nframes, seed=1234, path=SYNTH_PATH, ctx=ctx)
    # warm-up (code objects, buffers at size): two searches over the sequence's head
    ops = cycle.GpuOps(ctx, early_exit=early_exit)   # warmed on the object the timed run uses (its worker contexts exist)
    cycle.slam_main(cycle.DeviceMedia(None, dev[:640]), K_1080.copy(), cfg, ops)
    searches = []
    inner = ops.search

    def search(cond, batch, prev_frame, prev_holder):
        n, q = len(batch), prev_frame.seq[1]
        idx = [el.frame.seq[1] for el in batch]
        out = inner(cond, batch, prev_frame, prev_holder)
        searches.append({"query": q, "frames": idx, "counts": ops.last_counts.copy(), "good": int(out[0]),
                         "processed": int(ops.last_processed)})
        return out
    ops.search = search
    stats = {"record_ba": True}
    media = cycle.DeviceMedia(None, dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gd, logs = cycle.slam_main(media, K_1080.copy(), cfg, ops, stats=stats)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ops.close()
    dump = os.environ.get("SLAMHIP_BA_DUMP")
    if dump:
        # diagnostics (scripts/diag/ba_window_dump.sh): every window's inputs, the
        # GPU's solution and summary, for offline study against the oracle
        arr = {}
        for k, (io, sm) in enumerate(zip(stats.get("ba_io", []), stats.get("ba", []))):
            for name, v in io["in"].items():
                arr[f"w{k}_in_{name}"] = np.asarray(v)
            for name, v in zip(("K4", "ext", "pts"), io["out"]):
                arr[f"w{k}_out_{name}"] = np.asarray(v)
            arr[f"w{k}_summary"] = np.array([sm.initial_cost, sm.final_cost, sm.iterations, sm.num_residuals], np.float64)
        np.savez_compressed(f"{dump}_{'orb' if orb else 'sift'}.npz", **arr)
    cand = sum(x["processed"] for x in searches)
    fm = "ORB + Hamming BF" if orb else "SIFT-FLANN as exact BF-L2"
    out = {"config": "slamMain, the reference's example config (framesBatchSize 210, first fit, "
                     f"requiredMatchedPointsCount 500, {fm}, ratio 0.7) with BA on "
                     "(BAMaxFramesCnt 8, Huber 4): " + ("configs[2]" if orb else "configs[3] at N = 1") +
                     "; steady 1920x1080 sequence rendered into "
                     f"HBM before the run ({nframes} frames, FAST threshold {THRESHOLD})",
           "frames_per_s": media.i / el, "candidate_frames_per_s": cand / el, "frames": media.i,
           "searches": len(searches), "candidates": cand, "ms_per_search": el / max(1, len(searches)) * 1e3,
           "good_frame_gaps": [x["good"] + 1 for x in searches[:12]],
           "poses": len(logs.pose_list), "points": len(gd.spatialPoints), "ba_windows": len(stats.get("ba", [])),
           "ba_final_rmse": [math.sqrt(s.final_cost / max(1, s.num_residuals)) for s in stats.get("ba", [])],
           "ba_observations": [int(s.num_residuals) // 2 for s in stats.get("ba", [])],
           "candidates_per_search": cand / max(1, len(searches)), "early_exit_chunk": early_exit or None,
           "_result": {"searches": [(x["query"], x["good"], len(x["frames"])) for x in searches],
                       "poses": [np.asarray(p).copy() for p in logs.pose_list],
                       "rotations": [np.asarray(r).copy() for r in logs.rotation_list],
                       "points": np.asarray(gd.spatialPoints).copy(),
                       "ba": [(s.initial_cost, s.final_cost, s.iterations) for s in stats.get("ba", [])]}}
    if check:
        # (1) every BA window against oracle/ba.c on the same window inputs
        # (tests/ba_envelope.py: 1e-6 / 1e-4 px where the oracle converges, its
        # raw reordering envelope where it runs into the 50-iteration cap; a window
        # outside it fails; north_star's 1e-4 px reprojection RMSE bar beside it)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from ba_envelope import window_vs_oracle
        import oracle_ffi as O
        def resolve(w, iters):
            # a window outside the capped envelope, solved again on the GPU without the cap
            return slamhip.bundle_adjust_arrays(w["K4"].copy(), w["ext"].copy(), w["pts"].copy(), w["obs_frame"],
                                                w["obs_point"], w["obs_xy"], int(w["loss"]), float(w["loss_param"]),
                                                max_iters=iters, ctx=ctx)
        wc = [window_vs_oracle(io, s, resolve=resolve) for io, s in zip(stats.get("ba_io", []), stats.get("ba", []))]
        out["ba_window_checks"] = [{k: c.get(k) for k in ("ok", "tier", "north_star_ok", "bar",
                                                          "final_cost_rel_diff", "rmse_abs_diff_px",
                                                          "oracle_rmse_spread_px", "north_star_attainable",
                                                          "envelope", "converged")} for c in wc]
        # (2) the first search's match counts on candidates spread over its batch
        # (oracle FAST + SIFT / ORB + exact kNN + ratio, the same frames from HBM)
        s0 = searches[0] if searches else None
        samp = []

        def describe(img):
            k = O.fast(img, THRESHOLD, True)
            return O.orb(img, k)[1] if orb else O.sift(img, k)
        if s0:
            q = dev[s0["query"]].cpu().numpy()
            dq = describe(q)
            for bi in sorted(set(np.linspace(0, len(s0["frames"]) - 1, 6).round().astype(int).tolist())):
                f = dev[s0["frames"][bi]].cpu().numpy()
                ri, rd = O.knn2(dq, describe(f), O.NORM_HAMMING if orb else O.NORM_L2)
                samp.append([int(bi), int(s0["counts"][bi]), int(len(O.ratio(ri, rd, RATIO)))])
        out["first_search_counts_vs_oracle"] = samp
        out["parity_ok"] = bool(wc and all(c["ok"] for c in wc) and samp and all(a == b for _, a, b in samp))
        out["ba_north_star_ok"] = bool(wc and all(c["north_star_ok"] for c in wc))
        # windows that miss north_star's 1e-4 px where the oracle's own orders spread
        # their RMSE wider than it: the bar is unattainable there by any summation order
        out["ba_north_star_misses"] = [
            {"window": i, "rmse_abs_diff_px": c["rmse_abs_diff_px"], "oracle_rmse_spread_px": c.get("oracle_rmse_spread_px"),
             "unattainable_by_any_order": c.get("north_star_attainable") is False}
            for i, c in enumerate(wc) if not c["north_star_ok"]]
    del dev
    return out


def pipeline_cpu_baseline(frames):
    """the same sequence through the same control flow on the oracle's operations"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    from oracle_ops import OracleOps
    from slamhip import cycle
    t0 = time.perf_counter()
    stats = {}
    gd, logs = cycle.slam_main(cycle.MediaSources(frames), K_1080.copy(), pipeline_cfg(), OracleOps(), stats=stats)
    el = time.perf_counter() - t0
    return {"frames_per_s": len(frames) / el, "ms_per_frame": el / len(frames) * 1e3,
            "_result": (gd, logs, stats),
            "cores": int(O.oracle().orc_get_threads()), "kind": "port",
            "sample": f"the same {len(frames)}-frame sequence, oracle operations (OpenMP where the oracle has it)"}


def pipeline_compare(gpu, ref):
    """the GPU run against the oracle run of the same sequence.  The bar
    (parity_ok): the poses before the first BA window bit-exact (FAST, ORB,
    kNN, essential RANSAC, triangulation and PnP are all bit-exact), and EVERY
    BA window of the GPU run inside tests/ba_envelope.py's bar against the
    oracle's solve of the same window inputs: 1e-6 relative cost and 1e-4 px
    RMSE where the oracle converges, the oracle's reordering envelope where it
    runs into the 50-iteration cap.  After a capped window the two pipelines
    follow different (equally valid) trajectories; their end-to-end pose and
    point differences are reported, not barred."""
    import math
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from ba_envelope import window_vs_oracle
    (gg, lg, sg), (go, lo, so) = gpu, ref
    res = {"poses": [len(lg.pose_list), len(lo.pose_list)], "points": [len(gg.spatialPoints), len(go.spatialPoints)]}
    if len(lg.pose_list) == len(lo.pose_list) and lg.pose_list:
        res["pose_t_max_abs_diff"] = float(max(np.abs(a - b).max() for a, b in zip(lg.pose_list, lo.pose_list)))
        res["pose_R_max_abs_diff"] = float(max(np.abs(a - b).max() for a, b in zip(lg.rotation_list, lo.rotation_list)))
    if len(gg.spatialPoints) == len(go.spatialPoints) and len(gg.spatialPoints):
        res["points_max_abs_diff"] = float(np.abs(gg.spatialPoints - go.spatialPoints).max())
    if len(lg.pose_list) == len(lo.pose_list):
        res["pose_t_diff_by_pose"] = [float(np.abs(a - b).max()) for a, b in zip(lg.pose_list, lo.pose_list)]
    res["ba_windows"] = [{"gpu": [s.initial_cost, s.final_cost, s.iterations, s.num_residuals],
                          "oracle": [o.initial_cost, o.final_cost, o.iterations, o.num_residuals]}
                         for s, o in zip(sg.get("ba", []), so.get("ba", []))]
    rg = [math.sqrt(s.final_cost / max(1, s.num_residuals)) for s in sg.get("ba", [])]
    ro = [math.sqrt(s.final_cost / max(1, s.num_residuals)) for s in so.get("ba", [])]
    res["ba_rmse_gpu"], res["ba_rmse_oracle"] = rg, ro
    if len(rg) == len(ro) and rg:
        res["ba_rmse_max_abs_diff_px"] = max(abs(a - b) for a, b in zip(rg, ro))
    pre = 8                     # poses logged before the first window (BAMaxFramesCnt, pipeline_cfg)
    d = res.get("pose_t_diff_by_pose", [])
    res["poses_before_first_ba_bitexact"] = bool(d) and max(d[:pre] or [0.0]) == 0.0
    # every window of the GPU run against the oracle on the same inputs
    res["ba_window_checks"] = [window_vs_oracle(io, s) for io, s in zip(sg.get("ba_io", []), sg.get("ba", []))]
    res["ba_windows_ok"] = bool(res["ba_window_checks"]) and all(c["ok"] for c in res["ba_window_checks"])
    res["parity_ok"] = bool(res["poses"][0] == res["poses"][1] and res["poses_before_first_ba_bitexact"]
                            and res["ba_windows_ok"])
    return res


def geom_cpu_baseline(scene):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    K, R2, t2, p1, p2, q1, q2 = scene
    t0 = time.perf_counter()
    O.reconstruct(K, np.eye(3), np.zeros(3), R2, t2, p1, p2)
    el = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.estimate_transformation(q1, q2, K, True, 0.999, 5.0, 200.0)
    el_rp = time.perf_counter() - t0
    return {"ms_per_call": el * 1e3, "relative_pose_ms_per_call": el_rp * 1e3,
            "cores": int(O.oracle().orc_get_threads()), "kind": "port",
            "sample": f"one reconstruct() and one estimateTransformation() of {len(p1)} points "
                      "(relative pose: 1 thread, sequential RANSAC with early exit)"}


def siftdet_cpu_baseline():
    """oracle/siftdet.c on the same frame (OpenMP blurs, scalar extrema /
    orientation / descriptors)"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    import slamhip
    f = slamhip.synth_frames(W, H, 0, 1, seed=1234)[0]
    t0 = time.perf_counter()
    k, _ = O.sift_detect(f)
    el = time.perf_counter() - t0
    return {"ms_per_frame": el * 1e3, "kps": int(len(k)), "cores": int(O.oracle().orc_get_threads()),
            "kind": "port", "sample": "one 1920x1080 synthetic frame"}


def synth(first, count, w=W, h=H):
    """the bench's synthetic 1080p sequence (steady camera loop, seed 1234)"""
    import slamhip
    return slamhip.synth_frames(w, h, first, count, seed=1234, path=SYNTH_PATH)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads_all():
    """the host threads this process may use: OMP_NUM_THREADS when set (16 on
    the GPU box), else the affinity mask"""
    ev = os.environ.get("OMP_NUM_THREADS")
    if ev and ev.isdigit() and int(ev) > 0:
        return int(ev)
    return len(os.sched_getaffinity(0))


def cpu_baseline(frames, query, budget_s, threads=None, query_label=""):
    """oracle (restated OpenCV-semantics CPU path, not OpenCV): per candidate
    frame gray + FAST + SIFT + FLANN-forest kNN vs the query frame + ratio.
    frames: a sample spread over the GPU step's candidates; query: the frame
    whose descriptors the GPU step's kNN uses as its query set (the previous
    good frame of the timed steps), described once outside the timed loop, as
    the GPU step receives it already described."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    Oc = O.oracle()
    if threads is not None:
        Oc.orc_set_threads(int(threads))
    threads = Oc.orc_get_threads()
    kq = O.fast(query, THRESHOLD, True)
    dq = O.sift(query, kq)
    n, t0 = 0, time.perf_counter()
    kps = []
    while True:
        f = frames[n % len(frames)]
        kp = O.fast(f, THRESHOLD, True)
        d = O.sift(f, kp)
        idx = np.zeros((len(dq), 2), np.int32)
        dist = np.zeros((len(dq), 2), np.float32)
        Oc.orc_flann_knn2(O.vp(dq), len(dq), O.vp(d), len(d), 128, 4, 32, 1, O.vp(idx), O.vp(dist))
        O.ratio(idx, dist, RATIO)
        kps.append(len(kp))
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 4 * len(frames):
            break
    return {"value": n / el, "unit": "frames/s", "cores": int(threads), "kind": "port", "cpu_model": cpu_model(),
            "frames_timed": n, "mean_kps": float(np.mean(kps)), "query_kps": int(len(kq)),
            "sample": f"{n} of the GPU step's own 1920x1080 candidates (a {len(frames)}-frame sample spread evenly "
                      f"over the batch, taken in turn; {np.mean(kps):.0f} FAST kps on average) against the GPU "
                      f"step's query set ({query_label}{len(kq)} kps): gray+FAST+SIFT+FLANN(4 trees, 32 checks)+"
                      f"ratio per frame, oracle C restatement (-O3, OpenMP {threads} threads)"}


def main():
    args = parse()
    launch(args)
    if args.check_launch:
        check_launch(args)
        return
    import torch
    import torch.distributed as dist
    import slamhip
    from slamhip.batch import Conditions, PipelinedScan, ShardedScan

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SLAMHIP_DIST_BACKEND=gloo + more ranks than GPUs: a rehearsal of the
    # multi-rank step on one card (ranks share a device); the bench line uses RCCL
    backend = os.environ.get("SLAMHIP_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    props = torch.cuda.get_device_properties(local)
    my_dev = {"rank": rank, "local_rank": local, "device": f"cuda:{local}", "name": props.name,
              "pci_bus_id": getattr(props, "pci_bus_id", None)}
    devices = [my_dev]
    if world > 1:
        devices = [None] * world
        dist.all_gather_object(devices, my_dev)
    ctx = slamhip.Context(local)
    from slamhip import _lib as L
    if args.sift_kernel != "auto":
        ctx.set_option(L.OPT_SIFT_KERNEL, {"colw": L.SIFT_KERNEL_COLW, "band": L.SIFT_KERNEL_BAND,
                                               "tab": L.SIFT_KERNEL_TAB}[args.sift_kernel])
    scan = ShardedScan(rank, world, ctx=ctx)       # candidate sharding (RCCL when world > 1)
    db = scan.db
    # the headline loop: two contexts whose searches overlap (PipelinedScan: the
    # next search's extraction is queued before this one's counts are taken)
    pscan = PipelinedScan(rank, world, local, overlap=args.overlap)
    if args.sift_kernel != "auto":
        for c in pscan.ctxs:
            c.set_option(L.OPT_SIFT_KERNEL, {"colw": L.SIFT_KERNEL_COLW, "band": L.SIFT_KERNEL_BAND,
                                               "tab": L.SIFT_KERNEL_TAB}[args.sift_kernel])
    B = args.batch                                  # global candidates per search (framesBatchSize)
    mine = scan.shard(B)                            # candidate k lives on rank k % world (batch.cpp:183-187)
    pad_to = (B + world - 1) // world               # the largest shard: the all-gather's row count
    if len(mine) == 0:
        raise SystemExit(f"--batch {B} leaves rank {rank} of {world} without candidates")

    # synthetic sequence: this rank's candidates + the first previous frame
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(min(16, cpu_threads_all())) as ex:     # ctypes drops the GIL per frame
        host = np.concatenate(list(ex.map(lambda k: synth(1 + int(k), 1), mine)))
    frames = torch.from_numpy(host).to(dev)
    first = torch.from_numpy(synth(0, 1)).to(dev)
    db.extract(first, THRESHOLD, slamhip.SIFT_FLANN)
    prev_cap = 64 * 1024
    prev = torch.zeros(slamhip.lib().slam_batch_desc_bytes(slamhip.SIFT_FLANN, prev_cap), dtype=torch.uint8,
                       device=dev)
    _, nprev = db.export_desc(0, prev)
    owner = 0

    ops = [0.0]        # kNN int8 ops of this rank's launches (accumulated per step)
    winner = [None]    # the last search's (keypoints, matches), on every rank
    pending = [None]   # the last search's winner transfer in flight (ShardedScan.winner_begin)
    kps_desc = [0]     # keypoints this rank described (accumulated per step)

    cond = Conditions(featureExtractingThreshold=THRESHOLD, requiredExtractedPointsCount=0, frameBatchSize=B,
                      skipFramesFromBatchHead=0, useFirstFitInBatch=True,
                      requiredMatchedPointsCount=REQUIRED_MATCHES, matcherType=slamhip.SIFT_FLANN,
                      knnMatcherDistance=RATIO)

    def step(nxt):
        nonlocal nprev, owner
        # PipelinedScan.search: (1) the previous good frame's descriptors, owner ->
        # all ranks (RCCL broadcast; only this rank's kNN waits for it); the kNN of
        # this rank's candidates, whose extraction was queued during the previous
        # search; the NEXT search's extraction (nxt) queued on the other context;
        # one host wait; (2) per-candidate (keypoint, match, descriptor) counts
        # all-gathered; the same selection on every rank
        nq = nprev
        good, kp_all, mc_all, in_batch, dc_all = pscan.search(frames, prev, nprev, owner, cond, pad_to=pad_to,
                                                              next_frames=nxt)
        dc = pscan.db.batch_counts()
        kps_desc[0] += int(np.sum(dc))
        ops[0] += 2.0 * nq * float(np.sum(dc)) * 128
        # (3) the winner's keypoints and matches to the host of every rank: what
        # findGoodFrameFromBatch returns to its caller (batch.cpp:92-97).  The
        # copies (one rank) or the owner's device broadcast (more ranks) are
        # queued behind this search and taken after the next search's wait (the
        # last one inside the timed region)
        if pending[0] is not None:
            winner[0] = pscan.winner_end(pending[0])
        pending[0] = pscan.winner_begin(good, in_batch, dc_all, mc_all, nq)
        # hand-over: the winner's owner exports its descriptors (next broadcast root)
        owner, nprev = pscan.advance(good, in_batch, dc_all, prev, owner, nprev)
        return kp_all, mc_all, good

    def drain():
        if pending[0] is not None:
            winner[0] = pscan.winner_end(pending[0])
            pending[0] = None

    def run(n):
        """n searches, each extraction queued during the previous search; the
        first is queued here and the last search queues none, so the n
        extractions and n matches all happen inside the caller's region"""
        pscan.queue(frames, cond)
        out = None
        for i in range(n):
            out = step(frames if i + 1 < n else None)
        drain()
        return out

    kp_all, mc_all, good = run(args.warmup)
    ops[0] = 0.0
    kps_desc[0] = 0
    for c in pscan.ctxs:
        slamhip.lib().slam_profile_enable(c.handle, 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kp_all, mc_all, good = run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    # work of the timed region only (the H2D leg below calls step() again)
    ops_timed, kps_timed = ops[0], kps_desc[0]

    # kernel timings (HIP events on the launch stream, timed region only)
    import ctypes

    def read_prof(nsteps):
        out = {}
        for fam, name in FAMILIES.items():
            tot, cnt = 0.0, 0
            for c in pscan.ctxs:                    # both contexts' launches
                ms, n = ctypes.c_double(0), ctypes.c_int(0)
                slamhip.lib().slam_profile_read(c.handle, fam, ctypes.byref(ms), ctypes.byref(n))
                tot += ms.value * n.value
                cnt += n.value
            if cnt:
                out[name] = {"avg_ms": tot / cnt, "launches": cnt, "ms_per_step": tot / nsteps}
        return out

    prof = read_prof(args.steps)
    for c in pscan.ctxs:
        slamhip.lib().slam_profile_enable(c.handle, 0)   # the h2d leg below stays out of the kernel timings
    # with an overlap other than "knn" the next search's gray / FAST / blur wait
    # for CUs that this search's descriptor tail frees, so their event times
    # include that wait: the per-family rooflines come from a short pass on the
    # sequential schedule (same kernels, same inputs) right after the timed region
    prof_seq, ops_seq, kps_seq, nseq = prof, ops_timed, kps_timed, args.steps
    if pscan.overlap != "knn":
        pscan.overlap = "knn"
        ops[0], kps_desc[0] = 0.0, 0
        nseq = max(2, min(args.steps, 8))
        for c in pscan.ctxs:
            slamhip.lib().slam_profile_enable(c.handle, 1)
        run(nseq)
        torch.cuda.synchronize()
        prof_seq, ops_seq, kps_seq = read_prof(nseq), ops[0], kps_desc[0]
        for c in pscan.ctxs:
            slamhip.lib().slam_profile_enable(c.handle, 0)
        pscan.overlap = args.overlap

    # PCIe-inclusive rate (host-buffer boundary): the same steps with this rank's
    # frames copied from pinned host memory inside the timed region (never `value`)
    host_pinned = torch.from_numpy(host).pin_memory()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        frames.copy_(host_pinned, non_blocking=True)
        torch.cuda.current_stream().synchronize()   # the library's streams read the frames next
        run(1)
    torch.cuda.synchronize()
    el_h2d = time.perf_counter() - t1
    if world > 1:
        t = torch.tensor([el_h2d], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el_h2d = float(t.item())

    # the copy alone (pinned host -> HBM), to check the PCIe-inclusive number
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for _ in range(3):
        frames.copy_(host_pinned, non_blocking=True)
    torch.cuda.synchronize()
    h2d_gbps = 3 * host.nbytes / (time.perf_counter() - t2) / 1e9

    nloc = len(mine)
    value = B * args.steps / el                             # global candidates over the max-over-ranks time
    mean_kp = float(np.mean(kp_all))
    # roofline of every kernel family (sequential-schedule launch times); the
    # dominant one is the headline, priced on its timed-region launches
    spk = sift_samples_per_kp()
    per_frame_hbm = 3 * W * H + 12 * mean_kp + 2 * 128 * mean_kp + 16 * mean_kp

    def roofline(name, pf, ops_n, kps_n):
        sec = pf["avg_ms"] * 1e-3
        if name == "knn_mfma":
            alg = ops_n / pf["launches"]                       # 2 * N_prev * sum_f N_f * 128 int8 ops
            r = {"bound": "mfma", "achieved": alg / sec / 1e12, "peak": I8_MFMA_PEAK_TOPS, "unit": "TOPS",
                 "algorithmic_per_launch": alg, "per_unit": "2*128 int8 ops per (query, train) pair"}
        elif name == "sift_desc":
            alg = float(kps_n) / pf["launches"] * spk * SIFT_FLOP_PER_SAMPLE_SURVEY
            alg54 = float(kps_n) / pf["launches"] * spk * SIFT_FLOP_PER_SAMPLE
            r = {"bound": "valu", "achieved": alg / sec / 1e12, "peak": F32_VALU_PEAK_TF, "unit": "TFLOP/s",
                 "algorithmic_per_launch": alg,
                 "per_unit": f"{SIFT_FLOP_PER_SAMPLE_SURVEY} f32 flop (SURVEY 8(d)) x {spk} samples per keypoint",
                 "frac_survey": alg / sec / 1e12 / F32_VALU_PEAK_TF,
                 "frac_54flop": alg54 / sec / 1e12 / F32_VALU_PEAK_TF,
                 "bound_of_record": "lds (the 8 ordered bin read-add-writes per keypoint-sample; see lds.frac_of_floor)"}
            # the LDS view: every keypoint-sample reads and writes its 8
            # bins (32 B each way); the guide's chip-wide ds_read_b64 / ds_write_b64
            # rates give the time those bytes take at best
            rw = float(kps_n) / pf["launches"] * spk * 32
            floor_ms = (rw / LDS_READ_B64_TBS + rw / LDS_WRITE_B64_TBS) / 1e12 * 1e3
            r["lds"] = {"bin_bytes_read_per_launch": rw, "bin_bytes_written_per_launch": rw,
                        "floor_ms": floor_ms, "frac_of_floor": floor_ms / pf["avg_ms"],
                        "basis": f"ds_read_b64 {LDS_READ_B64_TBS} TB/s + ds_write_b64 {LDS_WRITE_B64_TBS} TB/s "
                                 "(MI355X_MICROARCH.md LDS table, 256 CUs x 2.4 GHz)"}
        else:
            per = {"fast_detect": 3 * W * H,                       # BGR read once
                   "sift_blur_grad": W * H * (1 + 8),              # gray in, {mag, ori} f32 out
                   "knn_finish": 16 * mean_kp}.get(name, per_frame_hbm)
            alg = per * nloc
            r = {"bound": "hbm", "achieved": alg / sec / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "algorithmic_per_launch": alg}
        r["frac"] = r["achieved"] / r["peak"]
        r["avg_ms"] = pf["avg_ms"]
        return r

    roofs = {name: roofline(name, pf, ops_seq, kps_seq) for name, pf in prof_seq.items()}
    dom = max(prof_seq, key=lambda k: prof_seq[k]["ms_per_step"]) if prof_seq else None
    roof = None
    if dom is not None and dom in prof:
        rd = roofline(dom, prof[dom], ops_timed, kps_timed)     # the timed region's own launches
        roof = dict(kernel=dom, **{k: rd[k] for k in ("bound", "achieved", "peak", "unit", "frac")},
                    traffic=None, algorithmic_per_launch=rd["algorithmic_per_launch"], avg_ms=rd["avg_ms"])
        for k in ("lds", "frac_survey", "frac_54flop", "bound_of_record", "per_unit"):
            if k in rd:
                roof[k] = rd[k]
        if "lds" in rd:
            roof["lds_frac_of_floor"] = rd["lds"]["frac_of_floor"]
    traffic_file = os.path.join(ROOT, "profiles", "traffic.json")
    if roof is not None and os.path.exists(traffic_file):
        try:
            tr = json.load(open(traffic_file)).get("per_launch_bytes", {})
            roof["traffic"] = tr.get(roof["kernel"])
            for name, r in roofs.items():
                r["traffic"] = tr.get(name)
        except (OSError, ValueError):
            pass

    # extract + match + BA over the same global batch (configs[3] at any rank
    # count): every rank joins (RCCL exchanges, BA solved on rank 0 and broadcast)
    wba = with_ba_leg(pscan, scan, frames, first, B, pad_to, slamhip.SIFT_FLANN, check=rank == 0) \
        if not args.no_extra else None
    # single-GPU legs (the N = 1 run): configs[2], configs[4]'s front end and BA
    # window, the BA windows alone, the detector, geometry, the whole pipeline
    solo = not args.no_extra and world == 1
    orb = orb_leg(pscan, db, frames, first, B, pad_to, steps=max(2, args.steps // 2), warmup=1) if solo else None
    ba = ba_leg(ctx, check=True) if solo else None
    c2 = with_ba_leg(pscan, scan, frames, first, B, pad_to, slamhip.ORB_BF, check=False) if solo else None
    pscan.close()                                   # its two contexts' buffers go back before the other legs
    if c2 is not None and ba is not None and "oracle" in ba:
        c2["ba_rmse_vs_oracle_px"] = abs(c2["ba_final_rmse"] - ba["oracle"]["final_rmse"])
    s4k = sift4k_leg(ctx) if solo else None
    ba16 = ba_leg(ctx, nframes=16, npoints=40000, k4k=True, check=False) if solo else None
    sdet = siftdet_leg(ctx) if solo else None
    geom = geom_leg(ctx) if solo else None
    geom_scene = geom.pop("scene") if geom else None
    pipe = pipeline_leg(ctx) if solo else None
    pipe210 = pipeline_b210_leg(ctx, check=rank == 0) if solo else None
    pipe210_orb = pipeline_b210_leg(ctx, check=rank == 0, orb=True) if solo else None
    pipe210_ee = pipeline_b210_leg(ctx, check=False, early_exit=EARLY_EXIT_CHUNK) if solo else None
    if pipe210_ee is not None:
        # the early-exit scan against the full scan of the same sequence: the same
        # winners (query, good index, batch size per search), poses, points and BA
        # windows, bit for bit
        a, b = pipe210["_result"], pipe210_ee.pop("_result")
        same = {"searches": a["searches"] == b["searches"],
                "poses": len(a["poses"]) == len(b["poses"]) and all(np.array_equal(x, y) for x, y in
                                                                     zip(a["poses"], b["poses"])),
                "rotations": len(a["rotations"]) == len(b["rotations"]) and all(
                    np.array_equal(x, y) for x, y in zip(a["rotations"], b["rotations"])),
                "points": a["points"].shape == b["points"].shape and np.array_equal(a["points"], b["points"]),
                "ba_windows": a["ba"] == b["ba"]}
        pipe210_ee["identical_to_full_scan"] = same
        pipe210_ee["parity_ok"] = all(same.values())
        pipe210_ee["speedup_vs_full_scan"] = pipe210_ee["frames_per_s"] / pipe210["frames_per_s"]
    for leg in (pipe210, pipe210_orb):
        if leg is not None:
            leg.pop("_result", None)
    pipe_frames = pipe.pop("frames") if pipe else None
    pipe_res = pipe.pop("_result") if pipe else None

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            # all host threads (the reported baseline) and one thread, same sample
            # a sample spread over the batch, against the query the timed steps used
            # (the last search's winner: candidate `good` is synthetic frame 1 + good)
            pick = np.unique(np.linspace(0, nloc - 1, min(nloc, 24)).round().astype(int))
            qf = 1 + int(good) if good is not None and int(good) >= 0 else 0
            qframe = synth(qf, 1)[0]
            lbl = f"synthetic frame {qf}, "
            cpu = cpu_baseline(host[pick], qframe, args.cpu_seconds, threads=cpu_threads_all(), query_label=lbl)
            cpu["one_thread"] = cpu_baseline(host[pick], qframe, args.cpu_seconds, threads=1, query_label=lbl)
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import oracle_ffi as O
            O.oracle().orc_set_threads(cpu_threads_all())
        out = {
            "metric": "frames/sec (extract+match+BA) @1080p 10k kpts, 1/2/4/8 GPU; final reproj RMSE",
            "value": value, "unit": "frames/s", "n_gpus": world,
            "world_size": dist.get_world_size() if world > 1 else 1, "devices": devices,
            "dist_backend": backend if world > 1 else None, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u8/i8 (int8 MFMA distances, f32 SIFT)", "data": "synthetic",
            "config": {"workload": f"configs[1] (N = 1) / configs[3]'s front end (N > 1): SIFT + BF-L2 kNN k=2, "
                                   f"1920x1080, ~10k kpts/frame, knnMatcherDistance=0.7, BA off; step = one "
                                   f"findGoodFrameFromBatch search over framesBatchSize={B} candidates (the "
                                   f"reference README's value), sharded k -> rank k % {world}, the winner's "
                                   f"keypoints and matches returned to the host",
                       "frames_per_step": B, "frames_per_step_this_rank": nloc, "mean_kps": mean_kp,
                       "min_kps": int(np.min(kp_all)), "max_kps": int(np.max(kp_all)),
                       "prev_kps": nprev, "query_frame": 1 + int(good) if int(good) >= 0 else 0,
                       "fast_threshold": THRESHOLD,
                       # the descriptor kernel each context's last extraction ran
                       "sift_desc_kernel": sorted({{L.SIFT_KERNEL_COLW: "sift_desc_colw", L.SIFT_KERNEL_BAND: "sift_desc_band",
                                                    L.SIFT_KERNEL_TAB: "sift_desc_tab"}.get(k, str(k))
                                                   for k in (slamhip.lib().slam_last_sift_kernel(c.handle)
                                                             for c in [ctx] + list(pscan.ctxs))}),
                       "sequence": "steady camera loop (slamhip.SYNTH_STEADY): every candidate and the query at "
                                   "10k +- 10 % FAST keypoints at one threshold, as configs[1] states",
                       "parallelism": f"candidate sharding x{world}"},
            # the metric's extract + match + BA figure and its final reprojection RMSE
            "value_with_ba": wba["frames_per_s"] if wba else None,
            "final_reproj_rmse": wba.get("ba_final_rmse") if wba else None,
            "rmse_vs_oracle_px": wba["oracle"]["rmse_abs_diff_px"] if wba and "oracle" in wba else None,
            "with_ba": wba,
            # extract + match + BA with every BA window built from the searched frames
            # (slamMain at framesBatchSize 210, SIFT, BA on: pipeline_b210): candidate
            # frames evaluated per second, and its windows' RMSE
            "value_with_ba_searched_frames": pipe210.get("candidate_frames_per_s") if pipe210 else None,
            "final_reproj_rmse_searched_frames": (pipe210.get("ba_final_rmse") or [None])[-1] if pipe210 else None,
            # PCIe-inclusive (host-buffer boundary), serialized: step time + the
            # measured pinned H2D time of this rank's frames; never `value`
            "value_incl_h2d": B / (el / args.steps + host.nbytes / (h2d_gbps * 1e9)),
            "h2d_GBps": h2d_gbps, "value_h2d_loop": B * args.steps / el_h2d,
            "config2_with_ba": c2,
            "orb": orb, "sift_4k": s4k, "ba_window": ba, "ba_window_w16_4k": ba16, "sift_detector": sdet,
            "triangulation": geom, "pipeline": pipe, "pipeline_b210": pipe210, "pipeline_b210_orb": pipe210_orb,
            "pipeline_b210_early_exit": pipe210_ee,
            "overlap": args.overlap, "kernels": prof, "kernels_sequential": prof_seq if prof_seq is not prof else None,
            "roofline": roof, "rooflines": roofs, "cpu_baseline": cpu,
        }
        if cpu:
            out["speedup_vs_cpu_baseline"] = value / cpu["value"]
        if cpu and geom:
            geom["cpu_baseline"] = geom_cpu_baseline(geom_scene)
            geom["speedup_vs_cpu_baseline"] = geom["cpu_baseline"]["ms_per_call"] / geom["ms_per_call"]
        if cpu and sdet:
            sdet["cpu_baseline"] = siftdet_cpu_baseline()
            sdet["speedup_vs_cpu_baseline"] = sdet["cpu_baseline"]["ms_per_frame"] / sdet["ms_per_frame"]
        if cpu and pipe:
            pipe["cpu_baseline"] = pipeline_cpu_baseline(pipe_frames)
            pipe["speedup_vs_cpu_baseline"] = pipe["frames_per_s"] / pipe["cpu_baseline"]["frames_per_s"]
            pipe["oracle_check"] = pipeline_compare(pipe_res, pipe["cpu_baseline"].pop("_result"))
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
