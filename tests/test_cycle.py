"""The per-frame pipeline (slamhip.cycle = mainCycle / slamMain) end to end.

CPU tests run the product's control flow over the oracle's operations
(tests/oracle_ops.py) -- the CPU plumbing case of BASELINE.json configs[0]
(640x480 synthetic 16-frame sequence, useFM-SIFT-FLANN, requiredExtractedPointsCount
2000, BA off) -- and pin the host-side pieces (Rodrigues, rawOutput format).
GPU tests run the same sequence twice, once on the HIP path (GpuOps) and once on
the oracle, and compare the reference's output files:
  BA off: poses.txt, rotations.txt, points.txt, colors.txt byte-identical;
  BA on (ORB, BAMaxFramesCnt 4): poses / rotations within 1e-6, every BA window's
  reprojection RMSE within 1e-4 px (final cost 1e-6 relative), colors identical,
  points within 1e-2 relative and the refined intrinsics within 1e-5 (the weakly
  constrained depth of the planar scene).
"""
import os

import numpy as np
import pytest

import oracle_ffi as O
import slamhip
from oracle_ops import OracleOps
from slamhip import cycle

K_VGA = np.array([[1724.676 / 3, 0, 995.966 / 3], [0, 1730.482 / 3, 550.192 / 3], [0, 0, 1.0]])


def _cfg(**kw):
    d = slamhip.reference_example()
    d.update({"featureExtractingThreshold": 10, "requiredExtractedPointsCount": 2000, "framesBatchSize": 4,
              "requiredMatchedPointsCount": 300, "useFM-SIFT-FLANN": True, "useFM-SIFT-BF": False,
              "useFM-ORB": False, "useBundleAdjustment": False, "BAMaxFramesCnt": 4})
    d.update(kw)
    return slamhip.ConfigService(d)


@pytest.fixture(scope="module")
def seq16():
    return slamhip.synth_frames(640, 480, 0, 16, seed=1234)


def _run(frames, cfg, ops, out_dir):
    K = K_VGA.copy()
    stats = {}
    gd, logs = cycle.slam_main(cycle.MediaSources(list(frames)), K, cfg, ops, out_dir=str(out_dir), stats=stats)
    files = {f: open(os.path.join(out_dir, f)).read() for f in ("poses.txt", "rotations.txt", "points.txt",
                                                                "colors.txt")}
    return gd, logs, K, files, stats


# ---------------- CPU: host logic and the configs[0] plumbing run ----------------

def test_rodrigues_matches_oracle():
    """slam_rodrigues (host code, both directions) against oracle/pnp.c, bit-exact."""
    rng = np.random.default_rng(5)
    vecs = [np.zeros(3), np.array([1e-17, 0, 0]), np.array([np.pi, 0, 0]), np.array([0, 0, 1e-3])]
    vecs += list(rng.normal(0, 1.5, (200, 3)))
    for v in vecs:
        R = slamhip.rodrigues_to_matrix(v)
        np.testing.assert_array_equal(R, O.rodrigues(v)[0])
        np.testing.assert_array_equal(slamhip.rodrigues_to_vector(R), O.rodrigues(R))
    # near-identity and 180-degree branches of the matrix -> vector direction
    for R in (np.eye(3), np.diag([1.0, -1.0, -1.0]), np.diag([-1.0, 1.0, -1.0]), np.eye(3) * 1000):
        np.testing.assert_array_equal(slamhip.rodrigues_to_vector(R), O.rodrigues(R))


def test_raw_output_format(tmp_path):
    p = tmp_path / "x.txt"
    with open(p, "w") as f:
        cycle.raw_output(np.array([[1.0, -2.5, 1e-13], [3, 4, 5]]), f)
        cycle.raw_output([(255, 0, 7)], f)
    assert p.read_text() == ("1.000000000000 -2.500000000000 0.000000000000\n"
                             "3.000000000000 4.000000000000 5.000000000000\n"
                             "255.000000000000 0.000000000000 7.000000000000\n")


def test_cycle_cpu_configs0(seq16, tmp_path):
    """BASELINE configs[0]: the CPU path (useFM-SIFT-FLANN as the reference's CPU
    build runs it: approximate KD-forest) through the product's control flow."""
    gd, logs, K, files, stats = _run(seq16, _cfg(), OracleOps(flann=True), tmp_path)
    poses = np.loadtxt(tmp_path / "poses.txt").reshape(-1, 3)
    rots = np.loadtxt(tmp_path / "rotations.txt").reshape(-1, 3, 3)
    assert len(poses) >= 3 and len(rots) == len(poses)
    np.testing.assert_array_equal(poses[0], 0)
    np.testing.assert_array_equal(rots[0], np.eye(3))
    for R in rots:
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-9)
    pts = np.loadtxt(tmp_path / "points.txt").reshape(-1, 3)
    cols = np.loadtxt(tmp_path / "colors.txt").reshape(-1, 3)
    assert len(pts) == len(cols) == len(gd.spatialPoints) > 100
    assert np.all((cols >= 0) & (cols <= 255)) and np.all(cols == np.round(cols))
    # every line: 12 digits after the point
    for line in files["points.txt"].splitlines()[:50]:
        assert all(len(v.split(".")[1]) == 12 for v in line.split())
    assert len(gd.cameraRotations) == len(poses)
    assert stats["frames"] == len(poses) - 2


def test_cycle_cpu_post_worker_matches_sequential(seq16, tmp_path):
    """the post-search worker's control flow (GpuOps.post_worker: each frame's
    "< 4" exit decided on the worker right after the previous frame's work, then
    that frame's PnP / triangulation / BA window) gives the output files of the
    sequential loop, with BA windows and with an exit taken on the worker"""
    from concurrent.futures import ThreadPoolExecutor

    class WorkerOps(OracleOps):
        def __init__(self, **kw):
            super().__init__(**kw)
            self.pool = ThreadPoolExecutor(1)

        def post_worker(self):
            return self.pool

    for kw in ({}, {"useFM-SIFT-FLANN": False, "useFM-ORB": True, "useBundleAdjustment": True,
                    "BAMaxFramesCnt": 4}):
        cfg = _cfg(**kw)
        _, la, _, fa, sa = _run(seq16, cfg, OracleOps(flann=not kw), tmp_path / ("s" + str(len(kw))))
        ops = WorkerOps(flann=not kw)
        _, lb, _, fb, sb = _run(seq16, cfg, ops, tmp_path / ("w" + str(len(kw))))
        ops.pool.shutdown()
        assert fa == fb and sa.get("frames") == sb.get("frames")
        assert len(la.pose_list) == len(lb.pose_list) >= 3
    # an exit on the worker: every frame's correspondences below 4 after the first pair
    class StopOps(WorkerOps):
        def solve_pnp(self, obj, img, K):
            raise AssertionError("no PnP after a < 4 exit")
    cfg = _cfg()
    ops = StopOps(flann=True)
    # force the exit: no previous frame keypoint has a spatial point
    cycle_main = cycle.main_cycle

    def patched(media, K, cond, deque, gd, logs, ops_, stats=None):
        orig = cycle.processing_first_pair_frames

        def first_pair(*a, **k):
            r = orig(*a, **k)
            a[4][1].correspondSpatialPointIdx[:] = -1      # deque[1]: the next search's previous frame
            return r
        cycle.processing_first_pair_frames = first_pair
        try:
            return cycle_main(media, K, cond, deque, gd, logs, ops_, stats)
        finally:
            cycle.processing_first_pair_frames = orig
    cycle.main_cycle = patched
    try:
        _, lc, _, fc, sc = _run(seq16, cfg, ops, tmp_path / "stop")
    finally:
        cycle.main_cycle = cycle_main
        ops.pool.shutdown()
    # only first-pair poses (slam_main restarts after each exit), no PnP ran
    assert len(lc.pose_list) >= 2 and len(lc.pose_list) % 2 == 0 and sc.get("frames", 0) == 0


def test_cycle_cpu_empty_and_short_sequences(tmp_path):
    """EMPTY_BATCH paths: no frame passes the FAST filter / a single frame."""
    f = slamhip.synth_frames(640, 480, 0, 3, seed=1234)
    gd, logs, K, files, _ = _run(f, _cfg(requiredExtractedPointsCount=10 ** 6), OracleOps(), tmp_path / "a")
    assert files["poses.txt"] == "" and files["points.txt"] == ""
    gd, logs, K, files, _ = _run(f[:1], _cfg(), OracleOps(), tmp_path / "b")
    assert files["poses.txt"] == "" and len(gd.spatialPoints) == 0


def test_batch_tail_and_first_fit_semantics():
    """find_good_frame_from_batch: first-fit scans from the tail, the tail after
    the good index is carried, elements before it are dropped (batch.cpp:90-97)."""
    class FakeOps:
        def __init__(self, counts):
            self.counts = counts

        def fast(self, frame, thr):
            return np.zeros(int(frame[0, 0, 0]), slamhip.KEYPOINT_DTYPE)

        def describe(self, frame, kps, matcher):
            return kps, np.zeros((len(kps), 128), np.float32)

        def match_frame(self, prev_desc, frame, kps, matcher, ratio):
            return kps, np.zeros(self.counts[int(frame[0, 0, 1])], slamhip.DMATCH_DTYPE)

    def frames(n):
        out = []
        for i in range(n):
            f = np.zeros((4, 4, 3), np.uint8)
            f[0, 0, 0] = 50
            f[0, 0, 1] = i
            out.append(f)
        return out
    cond = cycle.Conditions(_cfg(requiredExtractedPointsCount=10, requiredMatchedPointsCount=5, framesBatchSize=5))
    prev = cycle.TemporalImageData()
    prev.allExtractedFeatures = np.zeros(50, slamhip.KEYPOINT_DTYPE)
    # counts per frame id: tail-first scan, first fit -> the last qualifying index from the tail
    ops = FakeOps([9, 9, 3, 7, 1, 9, 9])
    media = cycle.MediaSources(frames(7))
    batch = []
    idx, frame, feats, m = cycle.find_good_frame_from_batch(media, cond, batch, frames(1)[0], prev, ops)
    assert idx == 3 and len(m) == 7 and [int(e.frame[0, 0, 1]) for e in batch] == [4]
    # best-count mode (useFirstFitInBatch false): max count, ties -> lowest index
    cond.useFirstFitInBatch = False
    idx, frame, feats, m = cycle.find_good_frame_from_batch(media, cond, batch, frames(1)[0], prev, ops)
    assert [int(frame[0, 0, 1])] == [5] and idx == 1 and [int(e.frame[0, 0, 1]) for e in batch] == [6]
    # nothing qualifies: FRAME_NOT_FOUND, batch untouched
    ops.counts = [0] * 7
    idx, *_ = cycle.find_good_frame_from_batch(media, cond, batch, frames(1)[0], prev, ops)
    assert idx == cycle.FRAME_NOT_FOUND and len(batch) == 1


# ---------------- GPU: the HIP path against the oracle, output files ----------------

@pytest.mark.gpu
def test_cycle_gpu_matches_oracle_sift_bf(gpu_ctx, seq16, tmp_path):
    cfg = _cfg(**{"useFM-SIFT-FLANN": False, "useFM-SIFT-BF": True})
    _, lg, Kg, fg, sg = _run(seq16, cfg, cycle.GpuOps(gpu_ctx), tmp_path / "gpu")
    _, lo, Ko, fo, so = _run(seq16, cfg, OracleOps(), tmp_path / "cpu")
    assert len(lg.pose_list) >= 3 and sg["frames"] == so["frames"]
    for name in fg:
        assert fg[name] == fo[name], name


@pytest.mark.gpu
def test_cycle_gpu_matches_oracle_orb_ba(gpu_ctx, seq16, tmp_path):
    cfg = _cfg(**{"useFM-SIFT-FLANN": False, "useFM-ORB": True, "useBundleAdjustment": True,
                  "requiredMatchedPointsCount": 200})
    gg, lg, Kg, fg, sg = _run(seq16, cfg, cycle.GpuOps(gpu_ctx), tmp_path / "gpu")
    go, lo, Ko, fo, so = _run(seq16, cfg, OracleOps(), tmp_path / "cpu")
    assert len(sg.get("ba", [])) >= 1 and len(sg["ba"]) == len(so["ba"])
    for name in ("poses.txt", "rotations.txt"):
        a = np.loadtxt(tmp_path / "gpu" / name)
        b = np.loadtxt(tmp_path / "cpu" / name)
        assert a.shape == b.shape, name
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6, err_msg=name)
    # BA bar (north_star): the reprojection error of every window within 1e-4 px of
    # the oracle's; the final costs within 1e-6 relative
    for a, b in zip(sg["ba"], so["ba"]):
        assert abs(a.final_cost - b.final_cost) <= 1e-6 * max(1.0, b.final_cost)
        ra = np.sqrt(a.final_cost / max(1, a.num_residuals))
        rb = np.sqrt(b.final_cost / max(1, b.num_residuals))
        assert abs(ra - rb) <= 1e-4
    # points: the synthetic scene is a plane seen over a short baseline, so depth is
    # weakly constrained; BA solutions agree to the same cost but drift along that
    # valley (measured up to 1.3e-3 relative), hence the looser bound on positions
    a = np.loadtxt(tmp_path / "gpu" / "points.txt")
    b = np.loadtxt(tmp_path / "cpu" / "points.txt")
    assert a.shape == b.shape
    np.testing.assert_allclose(a, b, rtol=1e-2, atol=1e-3)
    assert fg["colors.txt"] == fo["colors.txt"]
    # the intrinsics BA refines ride the same weakly constrained valley as the
    # points: a different (fixed) summation order on the device moves them by
    # up to ~2e-6 relative at equal cost (measured), hence 1e-5
    np.testing.assert_allclose(Kg, Ko, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("matcher", ["useFM-SIFT-BF", "useFM-ORB"])
@pytest.mark.parametrize("skip", [False, True])
def test_cycle_device_media_matches_oracle(gpu_ctx, seq16, tmp_path, matcher, skip):
    """The sequence decoded into HBM up front (cycle.DeviceMedia): fillVideoFrameBatch
    takes the frames a batch still needs and FAST-counts them in one device
    pass (GpuOps.fast_batch / slam_batch_fast), the batch is a view of the
    sequence when nothing was skipped (device_frames), the elements' FAST sets
    are recomputed only where read.  Output files byte-identical with the
    oracle run over MediaSources.  skip: requiredExtractedPointsCount at the
    median FAST count, so about half the frames fail the batch filter (stacked,
    non-contiguous batches).  Without skips the sequence has no host copy at
    all (DeviceMedia(None, dev)): point colours are gathered in HBM."""
    import torch
    req = int(np.median([len(O.fast(f, 10, True)) for f in seq16])) if skip else 2000
    flags = {"useFM-SIFT-FLANN": False, "useFM-SIFT-BF": False, "useFM-ORB": False, matcher: True,
             "requiredExtractedPointsCount": req}
    if matcher == "useFM-ORB":
        flags["requiredMatchedPointsCount"] = 200
    cfg = _cfg(**flags)
    dev = torch.from_numpy(np.ascontiguousarray(seq16)).cuda()
    ops = cycle.GpuOps(gpu_ctx)
    calls = []
    fb = ops.fast_batch
    ops.fast_batch = lambda frames, thr: calls.append(len(frames)) or fb(frames, thr)
    stats = {}
    out = tmp_path / "dev"
    media = cycle.DeviceMedia(seq16 if skip else None, dev)
    gd, lg = cycle.slam_main(media, K_VGA.copy(), cfg, ops, out_dir=str(out), stats=stats)
    assert calls and max(calls) > 1                        # batched intake ran
    _, lo, Ko, fo, so = _run(seq16, cfg, OracleOps(), tmp_path / "cpu")
    assert len(lg.pose_list) == len(lo.pose_list)
    if not skip:
        assert len(lg.pose_list) >= 3
    for name in fo:
        assert open(out / name).read() == fo[name], name


K_1080 = np.array([[1724.676, 0, 995.966], [0, 1730.482, 550.192], [0, 0, 1.0]])   # config/samsung-hv.xml


@pytest.mark.gpu
@pytest.mark.parametrize("matcher", ["useFM-SIFT-FLANN", "useFM-ORB"])
def test_search_early_exit_matches_full_scan(gpu_ctx, matcher):
    """GpuOps(early_exit=C) scans first-fit searches
    tail-first in chunks of C and stops at the first chunk holding a qualifying
    candidate (the single-thread break, batch.cpp:120-146).  On a drifting VGA
    sequence whose match counts fall with the distance from the query, with
    requiredMatchedPointsCount set so that the TAIL candidates FAIL (winners in
    the 2nd..4th chunk), so that none qualifies, so that all do, and with
    skipFramesFromBatchHead: the same goodIndex, winner features and matches,
    scanned-element marks, ORB border-filtered features and remaining batch as
    the full one-pass scan; fewer candidates processed when the tail qualifies"""
    frames = slamhip.synth_frames(640, 480, 0, 25, seed=1234)
    thr = 10

    def setup(ops):
        q = ops.ingest(frames[0])
        prev = cycle.TemporalImageData()
        prev.allExtractedFeatures = ops.fast(q, thr)
        els = []
        for i in range(1, len(frames)):
            f = ops.ingest(frames[i])
            els.append(cycle.BatchElement(f, ops.fast(f, thr)))
        return q, prev, els

    def run(early, required, skip=0):
        ops = cycle.GpuOps(gpu_ctx, early_exit=early)
        cond = cycle.Conditions(_cfg(**{matcher: True, "useFM-SIFT-FLANN": matcher == "useFM-SIFT-FLANN",
                                        "featureExtractingThreshold": thr, "requiredMatchedPointsCount": required,
                                        "skipFramesFromBatchHead": skip, "framesBatchSize": 24}))
        q, prev, batch = setup(ops)
        out = ops.search(cond, batch, q, prev)
        # frames are identified by their pixels' address (ingest views the same host arrays)
        res = {"good": out[0], "processed": ops.last_processed, "counts": ops.last_counts.copy(),
               "rest": [(e.frame.__array_interface__["data"][0], e.estimated, e.features.tobytes()) for e in batch]}
        if out[0] >= 0:
            res["features"], res["matches"] = out[2].tobytes(), out[3].tobytes()
        ops.close()
        return res, batch

    full0, _ = run(0, 0)
    c = full0["counts"]
    assert (c >= 0).all() and c[0] > c[-1]          # counts fall along the drift
    # thresholds: the tail fails and the winner sits 5 / 9 / 13 candidates below it
    # (chunks of 4), none qualifies, everything qualifies
    cases = [(int(c[len(c) - 1 - k]), 0) for k in (5, 9, 13)] + [(int(c.max()) + 1, 0), (0, 0), (int(c[4]), 6)]
    tail_failed = 0
    for required, skip in cases:
        full, _ = run(0, required, skip)
        ee, _ = run(4, required, skip)
        for k in ("good", "rest", "features", "matches"):
            assert full.get(k) == ee.get(k), (required, skip, k)
        if full["good"] >= 0:
            tail_failed += int(c[-1] < required)
            # the early scan stops in the chunk that holds the winner: chunks
            # [20, 24), [16, 20), ... clipped at skipFramesFromBatchHead
            lo = max(skip, 24 - 4 * ((24 - full["good"] + 3) // 4))
            assert ee["processed"] == 24 - lo
            assert (ee["counts"][lo:] == full["counts"][lo:]).all() and (ee["counts"][:lo] == -1).all()
        else:
            assert ee["processed"] == 24 - skip
    assert tail_failed >= 3
    # the tail qualifies: one chunk
    ee, _ = run(4, 0)
    assert ee["good"] == 23 and ee["processed"] == 4


@pytest.mark.gpu
def test_cycle_1080p_configs2_ba_windows(gpu_ctx):
    """configs[2]'s settings through the whole pipeline at 1920x1080 (ORB +
    Hamming BF, BA on, BAMaxFramesCnt 8, Huber 4), 24 frames as bench.py's
    pipeline leg runs them, each BA window solved on its own stream while the
    next search runs (GpuOps.ba_async).  Bars:
      * every pose before the first window bit-exact with the oracle pipeline
        (FAST, ORB, kNN, essential RANSAC, triangulation, PnP are bit-exact);
      * every BA window of the GPU run against oracle/ba.c on the SAME window
        inputs (tests/ba_envelope.py): 1e-6 relative cost and 1e-4 px RMSE
        where the oracle converges; inside the oracle's own reordering
        envelope (raw [min, max] over 16, then 64 orders) where it runs into
        the 50-iteration cap (north_star's 1e-4 px RMSE bar reported beside);
      * the asynchronous BA gives the same windows, poses and points as the
        synchronous sequence on the GPU."""
    from ba_envelope import window_vs_oracle
    frames = slamhip.synth_frames(1920, 1080, 100, 24, seed=1234)
    d = slamhip.reference_example()
    d.update({"featureExtractingThreshold": 31, "requiredExtractedPointsCount": 1000, "framesBatchSize": 2,
              "requiredMatchedPointsCount": 500, "useFM-SIFT-FLANN": False, "useFM-ORB": True,
              "useBundleAdjustment": True, "BAMaxFramesCnt": 8})
    cfg = slamhip.ConfigService(d)
    ops = cycle.GpuOps(gpu_ctx)
    sg = {"record_ba": True}
    gg, lg = cycle.slam_main(cycle.MediaSources(list(frames)), K_1080.copy(), cfg, ops, stats=sg)
    ops.close()
    assert len(sg["ba"]) >= 2 and len(sg["ba_io"]) == len(sg["ba"])
    # the synchronous sequence (plain ops.ba) on the GPU: identical results
    class SyncOps:
        def __init__(self, o):
            self.o = o

        def __getattr__(self, n):
            if n == "ba_async":
                raise AttributeError(n)
            return getattr(self.o, n)
    s2 = {}
    g2, l2 = cycle.slam_main(cycle.MediaSources(list(frames)), K_1080.copy(), cfg, SyncOps(cycle.GpuOps(gpu_ctx)),
                             stats=s2)
    assert [s.final_cost for s in s2["ba"]] == [s.final_cost for s in sg["ba"]]
    assert all(np.array_equal(a, b) for a, b in zip(l2.pose_list, lg.pose_list))
    np.testing.assert_array_equal(g2.spatialPoints, gg.spatialPoints)
    # the oracle pipeline: bit-exact up to the first window
    O.oracle().orc_set_threads(16)
    so = {}
    go, lo = cycle.slam_main(cycle.MediaSources(list(frames)), K_1080.copy(), cfg, OracleOps(), stats=so)
    assert len(lo.pose_list) == len(lg.pose_list)
    for a, b in list(zip(lg.pose_list, lo.pose_list))[:8]:
        np.testing.assert_array_equal(a, b)
    for a, b in list(zip(lg.rotation_list, lo.rotation_list))[:8]:
        np.testing.assert_array_equal(a, b)
    checks = [window_vs_oracle(io, s) for io, s in zip(sg["ba_io"], sg["ba"])]
    for c in checks:
        assert c["ok"], c
    # the first window's inputs are the oracle pipeline's own: same initial cost
    assert checks[0]["initial_cost_rel_diff"] <= 1e-12
