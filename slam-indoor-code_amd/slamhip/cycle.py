"""The reference's per-frame pipeline around the hot path: mainCycle and slamMain.

Restates, call for call, the host control flow that drives the extract ->
match -> pose -> triangulate -> BA path, so that a sequence run through this
module produces the reference's output files (points / colors / poses /
rotations .txt, rawOutput's 12-digit fixed format):

  slam_main                     src/main.cpp:71-107 (slamMain: restart loop, final outputs)
  main_cycle                    cycleProcessing/mainCycle.cpp:73-238
  processing_first_pair_frames  mainCycle.cpp:241-275
  define_first_pair_frames      mainCycle.cpp:278-306
  find_good_frame_from_batch    cycleProcessing/batch.cpp:59-99 (+ :101-160 scan, :228-267 fill)
  find_first_good_frame         mainCycleInternals.cpp:137-156
  compute_transformation_and_filter_points   mainCycleInternals.cpp:159-175
  define_features_correspond_spatial_indices mainCycleInternals.cpp:178-204
  get_old_spatial_points_and_new_frame_feature_coords  mainCycleInternals.cpp:207-219
  push_new_spatial_points       mainCycleInternals.cpp:222-246
  refine_transformation_for_global_coords    translation/cameraTranslation.cpp:71-77

Every numeric step goes through an `ops` object.  The default, GpuOps, is the
product path: the HIP kernels behind the C ABI (FAST, SIFT / ORB, kNN + ratio,
essential-matrix RANSAC + recoverPose, PnP RANSAC, DLT triangulation, BA),
with every BGR frame uploaded to HBM once and each candidate search run as one
device pass over the batch (GpuOps.search, the slam_batch_* calls).
The parity tests pass an object with the same methods backed by the CPU
oracle; this module never imports the oracle.

Reference semantics kept on purpose:
  * descriptors of the previous good frame are recomputed on every search and
    ORB's border filter mutates the keypoint lists in place (batch.cpp:113,178);
  * window entries pushed for BA are snapshots: keypoint and index lists are
    copied, R / t arrays are shared (cv::Mat shallow copies), so BA's in-place
    update reaches the deque (bundleAdjustment.cpp:178-201);
  * poses.txt / rotations.txt are written when a pose is estimated, before BA
    refines it (mainCycle.cpp:93-96, :172-177); BA mutates K in place.
"""
import ctypes
import os
import threading

import numpy as np

from . import _lib as L
from ._lib import DMATCH_DTYPE, KEYPOINT_DTYPE
from .api import (bundle_adjust_arrays, estimateTransformation, extractDescriptor,
                  fastExtractor, getMatcherTypeIndex, loss_from_config, matchFramesPairFeatures, reconstruct,
                  rodrigues_to_matrix, rodrigues_to_vector, solvePnPRansac)

EMPTY_BATCH = L.EMPTY_BATCH          # batch.h:5
FRAME_NOT_FOUND = L.FRAME_NOT_FOUND  # batch.h:6
OPTIMAL_DEQUE_SIZE = 8               # main.cpp:15, mainCycle.cpp:20


class ResidentFrame(np.ndarray):
    """A frame in host memory (the reference's cv::Mat, read for point colours)
    that also lives in HBM: GpuOps.ingest uploads it once.  Frames are never
    written after decoding, so the pipeline passes them on as the reference
    passes cv::Mat (a shallow, shared copy), not as deep copies."""

    def __array_finalize__(self, obj):
        self._dev = getattr(obj, "_dev", None)
        self.fast_kps = getattr(obj, "fast_kps", None)
        self.seq = getattr(obj, "seq", None)      # (sequence tensor, index): DeviceMedia frames
        self.host_valid = getattr(obj, "host_valid", True)   # False: the pixels live in HBM only

    @property
    def dev(self):
        """the frame's HBM copy; for a DeviceMedia frame the view of its sequence,
        made on first use (a batch of consecutive frames is used as one range,
        device_frames, and never needs the per-frame views)"""
        d = self._dev
        if d is None and self.seq is not None:
            d = self._dev = self.seq[0][self.seq[1]]
        return d

    @dev.setter
    def dev(self, v):
        self._dev = v

    @property
    def resident(self):
        return self._dev is not None or self.seq is not None


def device_frames(frames):
    """the HBM copies of `frames` as one (n, h, w, 3) tensor: a view when they
    are consecutive frames of one DeviceMedia sequence (a batch whose filter
    skipped nothing), else a stacked copy.  Returns (tensor, stacked)."""
    import torch
    seqs = [getattr(f, "seq", None) for f in frames]
    if frames and all(q is not None and q[0] is seqs[0][0] for q in seqs):
        i0 = seqs[0][1]
        if all(q[1] == i0 + k for k, q in enumerate(seqs)):
            return seqs[0][0][i0:i0 + len(frames)], False
    return torch.stack([f.dev for f in frames]), True


class GpuOps:
    """The product path: every numeric step on the GPU through libslamhip, with
    the frames resident in HBM.

    ingest() uploads a frame once when it leaves MediaSources; FAST runs on that
    copy (slam_fast_dev), and each findGoodFrameFromBatch search is one
    slam_batch_extract_match over the batch's device frames (search()), matched
    against the previous good frame's descriptors, which stay in HBM from the
    search that selected it (the reference recomputes them per search,
    batch.cpp:113: the same values).  Only keypoints, match lists and counts
    cross PCIe.  The host-buffer entry points (describe / match_frame) remain
    for callers that hold plain arrays."""

    def __init__(self, ctx=None, early_exit=0):
        """early_exit: 0 = every search describes and matches its whole batch in
        one device pass (the reference's multi-thread scan, batch.cpp:162-226,
        computes every candidate speculatively too); C > 0 = first-fit searches
        run tail-first in chunks of C candidates and stop at the first chunk that
        holds a qualifying candidate (the single-thread scan's break,
        batch.cpp:120-146).  The same winner, features, matches and batch
        mutations either way (tests/test_gpu_parity.py)."""
        from .api import default_context
        self.ctx = ctx or default_context()
        self.early_exit = int(early_exit)
        self.last_processed = 0   # candidates described + matched by the last search
        self._db = None
        self._qdb = None
        self._q = None          # (source device frame, descriptors in HBM, count, matcher)
        self._ba_pool = self._ba_ctx = None   # ba_async: one host thread, one context
        self._post_pool = self._pctx = None   # post_worker: one host thread, one context

    # ---- residency ---------------------------------------------------------
    @staticmethod
    def _torch():
        import torch  # device memory + streams (plumbing only)
        return torch

    def _stream(self):
        return ctypes.c_void_p(self._torch().cuda.current_stream().cuda_stream)

    def ingest(self, frame):
        if isinstance(frame, ResidentFrame) and frame.dev is not None:
            return frame
        if frame.ndim != 3 or frame.shape[2] != 3:
            return frame                # the device batch path takes BGR frames; others use host buffers
        torch = self._torch()
        f = np.ascontiguousarray(frame, np.uint8)
        dev = torch.from_numpy(f).to(torch.device("cuda", self.ctx.device))
        torch.cuda.current_stream().synchronize()
        r = f.view(ResidentFrame)
        r.dev = dev
        return r

    def _batches(self):
        if self._db is None:
            from .batch import DeviceBatch
            self._db, self._qdb = DeviceBatch(self.ctx), DeviceBatch(self.ctx)
        return self._db, self._qdb

    def prefetched(self, media, threshold, depth=3):
        """media whose next frames are uploaded and FAST-detected ahead of the
        pipeline on a worker thread (a context and stream of its own): the
        per-frame upload and fastExtractor leave the critical path.  Frames are
        still taken from `media` in order; each carries its FAST result."""
        return PrefetchedMedia(self, media, threshold, depth)

    # ---- fastExtractor -------------------------------------------------------
    def fast(self, frame, threshold):
        pre = getattr(frame, "fast_kps", None)
        if pre is not None and pre[0] == int(threshold):
            return pre[1].copy()                   # detected ahead (PrefetchedMedia)
        dev = getattr(frame, "dev", None)
        if dev is None:
            return fastExtractor(frame, threshold, True, ctx=self.ctx)
        return fast_dev(self.ctx, self._stream(), frame, threshold)

    # ---- findGoodFrameFromBatch (batch.cpp:59-160) on the device ---------------
    def _query(self, prev_frame, prev_holder, cond):
        """previous good frame's descriptors in HBM: kept from the search that
        selected it, else described once on the device"""
        dev = prev_frame.dev
        if self._q is not None and self._q[0] is dev and self._q[3] == cond.matcherType:
            return self._q[1], self._q[2]
        _, qdb = self._batches()
        raw = int(qdb.extract(dev.unsqueeze(0), cond.featureExtractingThreshold, cond.matcherType)[0])
        feats = qdb.keypoints(0).copy()
        # the holder keeps the frame's FAST set, or (ORB) its border-filtered part
        if len(prev_holder.allExtractedFeatures) not in (raw, len(feats)):
            raise RuntimeError("previous frame's keypoints differ from its FAST set")
        # ORB's in-place border filter (batch.cpp:113).  The holder is replaced only
        # when the contents differ: the post-search worker may be reading this
        # holder's array for its previous frame at the same time
        cur = np.asarray(prev_holder.allExtractedFeatures)
        if len(cur) != len(feats) or cur.dtype != feats.dtype or cur.tobytes() != feats.tobytes():
            prev_holder.allExtractedFeatures = feats
        q, nq = qdb.export_desc(0)
        self._q = (dev, q, nq, cond.matcherType)
        return q, nq

    def fast_batch(self, frames, threshold):
        """fillVideoFrameBatch's FAST over several resident frames in one device
        pass (slam_batch_fast): their keypoint counts, for the batch filter.
        The keypoints themselves are not copied out: a batch element's FAST set
        is recomputed (the same values) only where the pipeline reads it."""
        db, _ = self._batches()
        dev, stacked = device_frames(frames)
        if stacked:
            self._torch().cuda.current_stream().synchronize()
        # a view of the resident sequence is immutable, so the search's extraction
        # of the same view may take these results; a stacked copy is freed after
        # this call, and another stack may come back at its address
        return db.fast(dev, threshold, reuse=not stacked)

    def search(self, cond, batch, prev_frame, prev_holder):
        """the scan of batch.cpp:101-160 over the already filled batch: every
        candidate described and matched in one device pass (or, with
        early_exit, tail-first chunks until one holds the first fit), then the
        reference's selection (tail to skipFramesFromBatchHead, first fit) on the
        counts.  Returns (goodIndex, frame, features, matches) like the host
        scan, with the same batch mutations (scanned ORB candidates keep their
        border-filtered keypoints; the batch drops everything up to the winner)."""
        torch = self._torch()
        db, _ = self._batches()
        q, nq = self._query(prev_frame, prev_holder, cond)
        n, head = len(batch), cond.skipFramesFromBatchHead
        # first fit: the highest qualifying index wins, so once a tail chunk holds
        # one, no lower candidate can change the result (batch.cpp:140-141's break)
        chunk = self.early_exit if (self.early_exit > 0 and cond.useFirstFitInBatch and nq > 0) else 0
        counts = np.full(n, -1, np.int32)
        good, good_n = FRAME_NOT_FOUND, 0
        hi, lo, processed = n, 0, 0
        while True:
            lo = max(head, hi - chunk, 0) if chunk else 0
            if lo >= hi:
                break                       # nothing (left) at or above skipFramesFromBatchHead
            frames, stacked = device_frames([el.frame for el in batch[lo:hi]])
            if stacked:
                # the stack runs on torch's stream: complete before the batch kernels start
                torch.cuda.current_stream().synchronize()
            if nq > 0:
                _, mc = db.extract_match(frames, cond.featureExtractingThreshold, cond.matcherType, q, nq,
                                         cond.knnMatcherDistance)
            else:
                db.extract(frames, cond.featureExtractingThreshold, cond.matcherType)
                mc = np.zeros(hi - lo, np.int32)
            counts[lo:hi] = mc
            processed += hi - lo
            scanned = []
            for bi in range(hi - 1, max(head, lo) - 1, -1):
                scanned.append(bi)
                m = int(mc[bi - lo])
                if m >= cond.requiredMatchedPointsCount and m >= good_n:
                    good, good_n = bi, m
                    if cond.useFirstFitInBatch:
                        break
            for bi in scanned:
                batch[bi].estimated = True
                if cond.matcherType == L.ORB_BF:
                    batch[bi].features = db.keypoints(bi - lo).copy()
            if not chunk or good >= 0 or lo <= head:
                break
            hi = lo
        self.last_counts = counts        # per-candidate match counts (-1: not processed; bench checks)
        self.last_processed = processed
        if good < 0:
            return good, None, None, None
        el = batch[good]
        if nq > 0:
            k, m = db.result(good - lo, nq)                  # one sync for both
            el.features, el.matches = k.copy(), m.copy()
        else:
            el.features, el.matches = db.keypoints(good - lo).copy(), np.zeros(0, DMATCH_DTYPE)
        if len(el.features) > 0:
            qn, nqn = db.export_desc(good - lo)              # the next search's query, kept in HBM
            self._q = (el.frame.dev, qn, nqn, cond.matcherType)
        # the element leaves the batch here, so its fresh arrays are the returned copies
        out = (good, el.frame, el.features, el.matches)   # cv::Mat: shared
        del batch[:good + 1]
        return out

    # ---- the other operations (host buffers: small per-frame arrays) -----------
    def describe(self, frame, kps, matcher):
        return extractDescriptor(_host_pixels(frame), kps, matcher, ctx=self.ctx)

    def match_frame(self, prev_desc, frame, kps, matcher, ratio):
        return matchFramesPairFeatures(prev_desc, _host_pixels(frame), kps, matcher, ratio, ctx=self.ctx)

    def estimate_transformation(self, p1, p2, K, use_ransac, prob, threshold, distance):
        ok, R, t, chir, _ = estimateTransformation(p1, p2, K, use_ransac, prob, threshold, distance, ctx=self.ctx)
        return ok, R, t, chir

    # the per-frame work after a search runs on one host thread with a context of
    # its own (main_cycle: the next search runs meanwhile on self.ctx); a
    # context is used by one thread at a time (include/slamhip.h)
    def _post_ctx(self):
        # a high-priority stream (SLAMHIP_POST_PRIO=0: normal): the pose work is
        # a chain of small launches each frame waits on, and the next search's
        # batch kernels run beside it on the main context
        if self._pctx is None:
            from .api import Context
            self._pctx = Context(self.ctx.device, priority=int(os.environ.get("SLAMHIP_POST_PRIO", "1")))
            sums = os.environ.get("SLAMHIP_PNP_SUMS")
            if sums is not None:
                self._pctx.set_option(L.OPT_PNP_SUMS, int(sums))
        return self._pctx

    def post_worker(self):
        if self._post_pool is None:
            from concurrent.futures import ThreadPoolExecutor
            self._post_ctx()
            self._post_pool = ThreadPoolExecutor(1, thread_name_prefix="slamhip-post")
        return self._post_pool

    def reconstruct(self, K, R1, t1, R2, t2, p1, p2):
        return reconstruct(K, R1, t1, R2, t2, p1, p2, ctx=self._post_ctx())

    def solve_pnp(self, obj, img, K):
        found, rvec, tvec, _ = solvePnPRansac(obj, img, K, None, ctx=self._post_ctx())
        return found, rvec.reshape(3), tvec.reshape(3)

    def rodrigues(self, rvec):
        return rodrigues_to_matrix(rvec)

    def ba(self, K4, ext, pts, obs_frame, obs_point, obs_xy, loss, loss_param):
        return bundle_adjust_arrays(K4, ext, pts, obs_frame, obs_point, obs_xy, loss, loss_param, ctx=self.ctx)

    def ba_async(self, K4, ext, pts, obs_frame, obs_point, obs_xy, loss, loss_param):
        """ba() started on a context of its own (its own HIP stream) from a host
        thread: the caller's next search runs on the GPU meanwhile (ctypes drops
        the GIL inside slam_ba).  Returns a future of the summary; K4 / ext /
        pts are written when it completes."""
        if self._ba_pool is None:
            from concurrent.futures import ThreadPoolExecutor
            from .api import Context
            self._ba_ctx = Context(self.ctx.device, priority=int(os.environ.get("SLAMHIP_POST_PRIO", "1")))
            self._ba_pool = ThreadPoolExecutor(1, thread_name_prefix="slamhip-ba")
        return self._ba_pool.submit(bundle_adjust_arrays, K4, ext, pts, obs_frame, obs_point, obs_xy, loss,
                                    loss_param, ctx=self._ba_ctx)

    def close(self):
        if self._post_pool is not None:
            self._post_pool.shutdown(wait=True)
            self._post_pool = None
        if self._pctx is not None:
            self._pctx.close()
            self._pctx = None
        if self._ba_pool is not None:
            self._ba_pool.shutdown(wait=True)
            self._ba_ctx.close()
            self._ba_pool = self._ba_ctx = None


def fast_dev(ctx, stream, frame, threshold):
    """fastExtractor on a ResidentFrame's HBM copy (slam_fast_dev on `stream`)"""
    dev = frame.dev
    h, w = frame.shape[:2]
    ch = 1 if frame.ndim == 2 else frame.shape[2]
    cap = max(4096, w * h // 16)
    while True:
        out = np.empty(cap, KEYPOINT_DTYPE)   # the first n are written
        n = ctypes.c_int(0)
        rc = L.lib().slam_fast_dev(ctx.handle, stream, ctypes.c_void_p(dev.data_ptr()), w, h,
                                   w * ch, ch, int(threshold), 1, L.TYPE_9_16, L.ptr(out), cap, ctypes.byref(n))
        if rc == L.SLAM_E_CAPACITY:
            cap = n.value
            continue
        L.check(rc, ctx.handle)
        return out[:n.value].copy()


class PrefetchedMedia:
    """MediaSources read `depth` frames ahead: each frame is uploaded to HBM and
    FAST-detected on a worker thread with its own context and stream (ctypes
    releases the GIL inside the library), so getNextFrame's frame arrives
    resident with its keypoints while the pipeline's previous operations run.
    Same frames, same order, same keypoints as ingest() + fast()."""

    def __init__(self, ops, media, threshold, depth=3):
        from collections import deque
        from concurrent.futures import ThreadPoolExecutor
        from .api import Context
        self.ops, self.media, self.threshold = ops, media, int(threshold)
        self.ctx = Context(ops.ctx.device)
        self.pool = ThreadPoolExecutor(1, thread_name_prefix="slamhip-media")
        self.q = deque()
        self.done = False
        self._s = None
        for _ in range(max(1, depth)):
            self._submit()

    def _submit(self):
        if self.done:
            return
        f = self.media.next_frame()           # the source is read in order, on the caller's thread
        if f is None:
            self.done = True
            return
        self.q.append(self.pool.submit(self._work, f))

    def _work(self, frame):
        if frame.ndim != 3 or frame.shape[2] != 3:
            return frame                       # host-buffer frames: nothing ahead
        torch = GpuOps._torch()
        d = torch.device("cuda", self.ctx.device)
        if self._s is None:
            self._s = torch.cuda.Stream(d)
        f = np.ascontiguousarray(frame, np.uint8)
        with torch.cuda.stream(self._s):
            dev = torch.from_numpy(f).to(d, non_blocking=False)
            r = f.view(ResidentFrame)
            r.dev = dev
            kps = fast_dev(self.ctx, ctypes.c_void_p(self._s.cuda_stream), r, self.threshold)
        self._s.synchronize()
        dev.record_stream(torch.cuda.default_stream(d))   # used on the pipeline's stream from here on
        r.fast_kps = (self.threshold, kps)
        return r

    def next_frame(self):
        if not self.q:
            return None
        r = self.q.popleft().result()
        self._submit()
        return r

    def close(self):
        self.pool.shutdown(wait=True)
        self.ctx.close()


class Conditions:
    """DataProcessingConditions (mainCycleStructures.h:21-33), filled as
    defineProcessingEnvironment does (mainCycleInternals.cpp:80-104)."""

    def __init__(self, cfg):
        g = cfg.getValue
        self.featureExtractingThreshold = int(g("featureExtractingThreshold"))
        self.threadsCount = int(g("threadsCount"))
        self.frameBatchSize = int(g("framesBatchSize"))
        self.skipFramesFromBatchHead = int(g("skipFramesFromBatchHead"))
        self.useFirstFitInBatch = bool(g("useFirstFitInBatch"))
        self.requiredExtractedPointsCount = int(g("requiredExtractedPointsCount"))
        self.requiredMatchedPointsCount = int(g("requiredMatchedPointsCount"))
        self.matcherType = getMatcherTypeIndex(cfg)
        self.useBundleAdjustment = bool(g("useBundleAdjustment"))
        self.maxProcessedFramesVectorSz = int(g("BAMaxFramesCnt"))
        self.knnMatcherDistance = float(g("knnMatcherDistance"))
        self.rpUseRansac = bool(g("RPUseRANSAC"))
        self.rpProb = float(g("RPRANSACProb"))
        self.rpThreshold = float(g("RPRANSACThreshold"))
        self.rpDistance = float(g("RPDistanceThreshold"))
        self.loss, self.lossParam = loss_from_config(cfg)


class DeviceMedia:
    """MediaSources over a sequence already decoded into HBM: `dev` (n x h x w
    x 3 uint8 tensor) and its host copy `host` (the reference reads point
    colours from the cv::Mat).  getNextFrame hands out ResidentFrames whose
    device copy is a view of the sequence, so the consecutive frames of a batch
    are one contiguous range (device_frames: no stack per search), and take(n)
    gives fillVideoFrameBatch the next n frames for one FAST pass."""

    def __init__(self, host, dev):
        if host is not None and len(host) != len(dev):
            raise ValueError("host and device sequences differ in length")
        self.host, self.dev, self.i = host, dev, 0
        # host None: frames rendered / decoded into HBM only (colours gathered there)
        self._blank = np.broadcast_to(np.zeros(1, np.uint8), tuple(dev.shape[1:])) if host is None else None

    def next_frame(self):
        if self.i >= len(self.dev):
            return None
        if self.host is not None:
            r = self.host[self.i].view(ResidentFrame)
        else:
            r = self._blank.view(ResidentFrame)
            r.host_valid = False
        r.seq = (self.dev, self.i)              # r.dev: the view, made on first use
        self.i += 1
        return r

    def take(self, n):
        out = []
        while len(out) < n:
            f = self.next_frame()
            if f is None:
                break
            out.append(f)
        return out


class MediaSources:
    """MediaSources + getNextFrame (mainCycleInternals.cpp:107-120) over an
    in-memory sequence, a list of image paths (decoded with PIL, as imread
    would give BGR) or .npy frames.  Video decoding is out of scope."""

    def __init__(self, frames=None, paths=None):
        self._frames = list(frames) if frames is not None else []
        self._paths = list(paths) if paths is not None else []

    def next_frame(self):
        if self._frames:
            return np.ascontiguousarray(self._frames.pop(0), np.uint8)
        while self._paths:
            p = self._paths.pop(0)
            if p.endswith(".npy"):
                return np.ascontiguousarray(np.load(p), np.uint8)
            from PIL import Image
            rgb = np.asarray(Image.open(p).convert("RGB"))
            return np.ascontiguousarray(rgb[:, :, ::-1])
        return None


class TemporalImageData:
    """mainCycleStructures.h:38-45."""

    def __init__(self):
        self.allExtractedFeatures = np.zeros(0, KEYPOINT_DTYPE)
        self.allMatches = np.zeros(0, DMATCH_DTYPE)
        self.rotation = None
        self.motion = None
        self.correspondSpatialPointIdx = np.zeros(0, np.int64)

    def snapshot(self):
        """std::vector push_back copy: vectors deep, cv::Mat shallow."""
        s = TemporalImageData()
        s.allExtractedFeatures = self.allExtractedFeatures.copy()
        s.allMatches = self.allMatches.copy()
        s.rotation = self.rotation
        s.motion = self.motion
        s.correspondSpatialPointIdx = self.correspondSpatialPointIdx.copy()
        return s


class GlobalData:
    """mainCycleStructures.h:49-54 (points as an N x 3 float64 array, colors N x 3 uint8)."""

    def __init__(self):
        # std::vector storage: rows [0, n) of a buffer grown by doubling, so a
        # push_back of a frame's new points does not copy every earlier point
        self._pts, self._npts = np.zeros((0, 3), np.float64), 0      # Point3d rows
        self._cols, self._ncols = np.zeros((0, 3), np.uint8), 0      # Vec3b (b, g, r)
        self.spatialCameraPositions = []
        self.cameraRotations = []

    @property
    def spatialPoints(self):
        return self._pts[:self._npts]

    @spatialPoints.setter
    def spatialPoints(self, v):
        self._pts = np.ascontiguousarray(v, np.float64).reshape(-1, 3)
        self._npts = len(self._pts)

    @property
    def spatialPointsColors(self):
        return self._cols[:self._ncols]

    @spatialPointsColors.setter
    def spatialPointsColors(self, v):
        self._cols = np.ascontiguousarray(v, np.uint8).reshape(-1, 3)
        self._ncols = len(self._cols)

    @staticmethod
    def _append(buf, n, rows):
        if n + len(rows) > len(buf):
            grown = np.empty((max(2 * len(buf), n + len(rows), 1024), 3), buf.dtype)
            grown[:n] = buf[:n]
            buf = grown
        buf[n:n + len(rows)] = rows
        return buf, n + len(rows)

    def push_points(self, pts, colors):
        self._pts, self._npts = self._append(self._pts, self._npts, np.asarray(pts, np.float64).reshape(-1, 3))
        self._cols, self._ncols = self._append(self._cols, self._ncols, np.asarray(colors, np.uint8).reshape(-1, 3))


class BatchElement:
    """mainCycleStructures.h:59-64.  `lazy` = (ops, threshold): the element's
    FAST set was counted in a batched intake pass (GpuOps.fast_batch) and is
    recomputed by ops.fast on first read -- the same keypoints."""

    def __init__(self, frame, features, lazy=None):
        self.frame = frame
        self._features = features
        self._lazy = lazy
        self.matches = np.zeros(0, DMATCH_DTYPE)
        self.estimated = False

    @property
    def features(self):
        if self._features is None and self._lazy is not None:
            ops, thr = self._lazy
            self._features = ops.fast(self.frame, thr)
        return self._features

    @features.setter
    def features(self, v):
        self._features = v


def raw_output(rows, f):
    """IOmisc.cpp:88-109 rawOutput: rows of doubles, std::fixed, 12 digits."""
    for r in np.atleast_2d(np.asarray(rows, np.float64)):
        f.write(" ".join("%.12f" % v for v in r) + "\n")


class Logs:
    """openLogsStreams (IOmisc.cpp:10-25): the four result files of outputDataDir."""

    def __init__(self, out_dir):
        self.poses = self.rotations = None
        self.out_dir = out_dir
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
            self.poses = open(os.path.join(out_dir, "poses.txt"), "w")
            self.rotations = open(os.path.join(out_dir, "rotations.txt"), "w")
        self.pose_list, self.rotation_list = [], []

    def pose(self, R, t):
        self.pose_list.append(np.asarray(t, np.float64).reshape(3).copy())
        self.rotation_list.append(np.asarray(R, np.float64).reshape(3, 3).copy())
        if self.poses:
            raw_output(np.asarray(t, np.float64).reshape(1, 3), self.poses)
            raw_output(np.asarray(R, np.float64).reshape(3, 3), self.rotations)

    def close(self, gd):
        if self.out_dir:
            self.poses.close()
            self.rotations.close()
            with open(os.path.join(self.out_dir, "points.txt"), "w") as f:
                if len(gd.spatialPoints):
                    raw_output(gd.spatialPoints, f)
            with open(os.path.join(self.out_dir, "colors.txt"), "w") as f:
                if len(gd.spatialPointsColors):
                    raw_output(gd.spatialPointsColors, f)


def _pts(kps, idx):
    return np.stack([kps["x"][idx], kps["y"][idx]], 1).astype(np.float32) if len(idx) else np.zeros((0, 2), np.float32)


def _colors(frame, kps):
    # frame.at<Vec3b>(pt.y, pt.x): float -> int conversion (truncation) of the keypoint coordinates
    ys, xs = kps["y"].astype(np.int64), kps["x"].astype(np.int64)
    if not getattr(frame, "host_valid", True):
        # a DeviceMedia frame without a host copy: the same pixels gathered in HBM
        import torch
        d = frame.dev
        idx = torch.from_numpy(ys * frame.shape[1] + xs).to(d.device)
        return d.reshape(-1, 3).index_select(0, idx).cpu().numpy()
    return np.asarray(frame[ys, xs]).reshape(-1, 3)


def _assign_last(dst, idx, val):
    """dst[idx[i]] = val[i] for i in order (a repeated index keeps the last value):
    each index's last position by a max-scatter of the positions, O(n)"""
    n = len(idx)
    if n == 0:
        return
    pos = np.arange(n)
    w = np.full(len(dst), -1, np.int64)
    np.maximum.at(w, idx, pos)
    last = w[idx] == pos
    dst[idx[last]] = val[last]


# ---- batch.cpp ----------------------------------------------------------------

def fill_video_frame_batch(media, cond, batch, ops):
    """batch.cpp:228-267: FAST-filtered frames appended up to frameBatchSize."""
    skipped = 0
    fast_batch = getattr(ops, "fast_batch", None)
    if fast_batch is not None and getattr(media, "take", None) is not None:
        # frames already in HBM (DeviceMedia): the frames still missing are taken
        # in order and FAST-counted in one pass; the filter and the media
        # consumption are those of the frame-by-frame loop below
        while len(batch) < cond.frameBatchSize:
            frames = media.take(cond.frameBatchSize - len(batch))
            if not frames:
                break
            counts = fast_batch(frames, cond.featureExtractingThreshold)
            for f, c in zip(frames, counts):
                if c < cond.requiredExtractedPointsCount:
                    skipped += 1
                    continue
                batch.append(BatchElement(f, None, lazy=(ops, cond.featureExtractingThreshold)))
        return skipped
    ingest = getattr(ops, "ingest", None)
    while len(batch) < cond.frameBatchSize:
        frame = media.next_frame()
        if frame is None:
            break
        if ingest is not None:
            frame = ingest(frame)       # GpuOps: the frame's one upload to HBM
        feats = ops.fast(frame, cond.featureExtractingThreshold)
        if len(feats) < cond.requiredExtractedPointsCount:
            skipped += 1
            continue
        batch.append(BatchElement(frame, feats))
    return skipped


def _host_pixels(frame):
    """the frame's host pixels; a ResidentFrame whose pixels live in HBM only
    (DeviceMedia without a host copy) has none, and raises instead of handing on
    its placeholder zeros"""
    if not getattr(frame, "host_valid", True):
        raise ValueError("frame has no host pixels (DeviceMedia without a host copy): "
                         "this operation needs host pixels or ops with a device search")
    return np.asarray(frame)


def _resident(f):
    r = getattr(f, "resident", None)
    return r if r is not None else getattr(f, "dev", None) is not None


def find_good_frame_from_batch(media, cond, batch, prev_frame, prev_holder, ops):
    """batch.cpp:59-99 + the scan of :101-160.  prev_holder.allExtractedFeatures
    is mutated in place by the descriptor step (ORB border filter), as the
    reference's std::vector<KeyPoint>& is.  Returns (goodIndex, frame, features,
    matches)."""
    fill_video_frame_batch(media, cond, batch, ops)
    n = len(batch)
    if n == 0:
        return EMPTY_BATCH, None, None, None
    if getattr(ops, "search", None) is not None and _resident(prev_frame) and all(_resident(el.frame) for el in batch):
        return ops.search(cond, batch, prev_frame, prev_holder)   # GpuOps: the scan in one device pass
    # the host scan reads host pixels: a frame that lives in HBM only (DeviceMedia
    # without its host copy) cannot take this path
    for f in [prev_frame] + [el.frame for el in batch]:
        _host_pixels(f)
    feats, prev_desc = ops.describe(prev_frame, prev_holder.allExtractedFeatures, cond.matcherType)
    prev_holder.allExtractedFeatures = feats
    good, good_n = FRAME_NOT_FOUND, 0
    for bi in range(n - 1, cond.skipFramesFromBatchHead - 1, -1):
        el = batch[bi]
        el.features, el.matches = ops.match_frame(prev_desc, el.frame, el.features, cond.matcherType,
                                                  cond.knnMatcherDistance)
        el.estimated = True
        m = len(el.matches)
        if m >= cond.requiredMatchedPointsCount and m >= good_n:
            good, good_n = bi, m
            if cond.useFirstFitInBatch:
                break
    if good < 0:
        return good, None, None, None
    el = batch[good]
    out = (good, el.frame, el.features.copy(), el.matches.copy())   # cv::Mat: shared
    del batch[:good + 1]
    return out


# ---- mainCycleInternals.cpp ----------------------------------------------------

def find_first_good_frame(media, cond, holder, ops):
    ingest = getattr(ops, "ingest", None)
    while True:
        frame = media.next_frame()
        if frame is None:
            return None
        if ingest is not None:
            frame = ingest(frame)
        holder.allExtractedFeatures = ops.fast(frame, cond.featureExtractingThreshold)
        if len(holder.allExtractedFeatures) >= cond.requiredExtractedPointsCount:
            return frame


def key_point_coords(f1, f2, matches):
    """getKeyPointCoordsFromFramePair: (queryIdx pts of frame 1, trainIdx pts of frame 2)."""
    return _pts(f1, matches["queryIdx"]), _pts(f2, matches["trainIdx"])


def compute_transformation_and_filter_points(cond, K, d0, d1, ops):
    p1, p2 = key_point_coords(d0.allExtractedFeatures, d1.allExtractedFeatures, d1.allMatches)
    ok, R, t, chir = ops.estimate_transformation(p1, p2, K, cond.rpUseRansac, cond.rpProb, cond.rpThreshold,
                                                 cond.rpDistance)
    if R is None:
        raise RuntimeError("findEssentialMat returned no model for the first pair")
    d1.rotation = np.array(R, np.float64).reshape(3, 3)
    d1.motion = np.array(t, np.float64).reshape(3, 1)
    keep = np.asarray(chir, np.uint8) > 0
    return p1[keep], p2[keep], keep


def refine_transformation_for_global_coords(R0, t0, d1):
    d1.motion = t0 + d1.rotation @ d1.motion
    d1.rotation = R0 @ d1.rotation


def define_features_correspond_spatial_indices(mask, second_frame, d0, d1):
    """returns the colors of the new points (mask order)"""
    d0.correspondSpatialPointIdx = np.full(len(d0.allExtractedFeatures), -1, np.int64)
    d1.correspondSpatialPointIdx = np.full(len(d1.allExtractedFeatures), -1, np.int64)
    m = d1.allMatches[np.asarray(mask, bool)]
    k = np.arange(len(m), dtype=np.int64)
    _assign_last(d0.correspondSpatialPointIdx, m["queryIdx"].astype(np.int64), k)
    _assign_last(d1.correspondSpatialPointIdx, m["trainIdx"].astype(np.int64), k)
    return _colors(second_frame, d1.allExtractedFeatures[m["trainIdx"]])


def old_spatial_points_and_new_coords(matches, prev_idx, points, new_kps):
    sel = prev_idx[matches["queryIdx"]] if len(matches) else np.zeros(0, np.int64)
    keep = sel >= 0
    obj = points[sel[keep]].astype(np.float32) if keep.any() else np.zeros((0, 3), np.float32)
    img = _pts(new_kps, matches["trainIdx"][keep]) if keep.any() else np.zeros((0, 2), np.float32)
    return obj, img


def push_new_spatial_points(new_frame, new_points, gd, prev_idx, d1):
    """every match in order: a query without a point gets the match's new point
    (appended); the train keypoint takes the query's point index (queryIdx values
    are unique: one kNN match per query)."""
    d1.correspondSpatialPointIdx = np.full(len(d1.allExtractedFeatures), -1, np.int64)
    q = d1.allMatches["queryIdx"].astype(np.int64)
    t = d1.allMatches["trainIdx"].astype(np.int64)
    sid = prev_idx[q]
    new = sid < 0
    base = len(gd.spatialPoints)
    nid = base + np.arange(int(new.sum()), dtype=np.int64)
    gd.push_points(np.asarray(new_points, np.float64).reshape(-1, 3)[new],
                   _colors(new_frame, d1.allExtractedFeatures[t[new]]))
    prev_idx[q[new]] = nid
    val = sid.copy()
    val[new] = nid
    _assign_last(d1.correspondSpatialPointIdx, t, val)


class PendingBA:
    """One BA window whose solve may still be running (GpuOps.ba_async) while
    the next findGoodFrameFromBatch search runs: that search needs only the
    previous good frame (mainCycle.cpp:117-123), and the first consumer of BA's
    K / R / t / points is the PnP of the frame it returns (:155-161).  finish()
    writes the solution back in place (bundleAdjustment.cpp:153-201), moves the
    window to the global structure (mainCycle.cpp:203-210) and logs the summary,
    exactly as the synchronous sequence does."""

    def __init__(self, K, window, gd, result, K4, ext, pts, inputs, stats):
        self.K, self.window, self.gd, self.result = K, window, gd, result
        self.K4, self.ext, self.pts, self.inputs, self.stats = K4, ext, pts, inputs, stats

    def finish(self):
        summary = self.result.result() if hasattr(self.result, "result") else self.result
        K, K4, ext = self.K, self.K4, self.ext
        K[0, 0], K[1, 1], K[0, 2], K[1, 2] = K4
        for i, im in enumerate(self.window):
            im.rotation[...] = rodrigues_to_matrix(ext[i, :3])
            im.motion[...] = ext[i, 3:].reshape(3, 1)
        self.gd.spatialPoints = self.pts
        move_processed_data_to_global_struct(self.window, self.gd)
        if self.stats is not None:
            self.stats.setdefault("ba", []).append(summary)
            if self.stats.get("record_ba"):
                self.stats.setdefault("ba_io", []).append(
                    {"in": self.inputs, "out": (K4.copy(), ext.copy(), self.pts.copy())})
        return summary


def start_bundle_adjustment(K, window, gd, cond, ops, stats=None):
    """bundleAdjustment.cpp:73-129 over the processed-frames window: observations
    in AddResidualBlock order (frame, then keypoint), frame 0 held constant.
    Started on ops.ba_async when the ops have it (GpuOps), else solved here;
    PendingBA.finish() applies it.  stats["record_ba"]: keep each window's
    inputs and solution (stats["ba_io"]) for an oracle re-run on the same input."""
    K4 = np.array([K[0, 0], K[1, 1], K[0, 2], K[1, 2]], np.float64)
    ext = np.zeros((len(window), 6), np.float64)
    of, op, oxy = [], [], []
    for i, im in enumerate(window):
        ext[i, :3] = rodrigues_to_vector(im.rotation)
        ext[i, 3:] = im.motion.reshape(3)
        kps = im.allExtractedFeatures
        p = np.nonzero(im.correspondSpatialPointIdx >= 0)[0]
        of.append(np.full(len(p), i, np.int32))
        op.append(im.correspondSpatialPointIdx[p].astype(np.int32))
        oxy.append(np.stack([kps["x"][p], kps["y"][p]], 1).astype(np.float64))
    pts = np.ascontiguousarray(gd.spatialPoints, np.float64).copy()
    of, op, oxy = np.concatenate(of), np.concatenate(op), np.concatenate(oxy).reshape(-1, 2)
    inputs = None
    if stats is not None and stats.get("record_ba"):
        inputs = dict(K4=K4.copy(), ext=ext.copy(), pts=pts.copy(), obs_frame=of, obs_point=op, obs_xy=oxy,
                      loss=cond.loss, loss_param=cond.lossParam)
    run = getattr(ops, "ba_async", None) or ops.ba
    result = run(K4, ext, pts, of, op, oxy, cond.loss, cond.lossParam)
    return PendingBA(K, list(window), gd, result, K4, ext, pts, inputs, stats)


def bundle_adjustment(K, window, gd, cond, ops, stats=None):
    """the synchronous form: solve, write back, move the window; returns the summary"""
    pending = start_bundle_adjustment(K, window, gd, cond, ops, stats)
    window.clear()
    return pending.finish()


def move_processed_data_to_global_struct(processed, gd):
    for fd in processed:
        gd.cameraRotations.append(fd.rotation.copy())
        gd.spatialCameraPositions.append(fd.motion.copy())
    processed.clear()


# ---- mainCycle.cpp -------------------------------------------------------------

def define_first_pair_frames(cond, media, batch, deque, ops):
    first = find_first_good_frame(media, cond, deque[0], ops)
    if first is None:
        return EMPTY_BATCH, None
    while True:
        idx, frame, feats, matches = find_good_frame_from_batch(media, cond, batch, first, deque[0], ops)
        if idx == EMPTY_BATCH:
            return EMPTY_BATCH, None
        if idx >= 0:
            deque[1].allExtractedFeatures, deque[1].allMatches = feats, matches
            return idx, frame
        first = batch[0].frame
        deque[0].allExtractedFeatures = batch[0].features.copy()
        del batch[0]


def processing_first_pair_frames(media, K, cond, batch, deque, gd, logs, ops):
    idx, second = define_first_pair_frames(cond, media, batch, deque, ops)
    if idx == EMPTY_BATCH:
        return EMPTY_BATCH, None
    p1, p2, mask = compute_transformation_and_filter_points(cond, K, deque[0], deque[1], ops)
    refine_transformation_for_global_coords(deque[0].rotation, deque[0].motion, deque[1])
    pts = ops.reconstruct(K, deque[0].rotation, deque[0].motion, deque[1].rotation, deque[1].motion, p1, p2)
    colors = define_features_correspond_spatial_indices(mask, second, deque[0], deque[1])
    gd.push_points(pts, colors)
    return idx, second


def main_cycle(media, K, cond, deque, gd, logs, ops, stats=None):
    batch = []
    processed = []
    idx, last_good = processing_first_pair_frames(media, K, cond, batch, deque, gd, logs, ops)
    if idx == EMPTY_BATCH:
        return EMPTY_BATCH
    processed.append(deque[0].snapshot())
    processed.append(deque[1].snapshot())
    logs.pose(deque[0].rotation, deque[0].motion)
    logs.pose(deque[1].rotation, deque[1].motion)

    last = 1
    bidx = FRAME_NOT_FOUND
    pending = None          # the last window's BA, solving while the next search runs
    # GpuOps: the work after a search (BA write-back, PnP, triangulation, point
    # bookkeeping, the next BA window's start) runs on a host thread with a
    # context of its own while the main thread runs the NEXT search, which needs
    # only the good frame and the batch (mainCycle.cpp:117-123).  The loop's
    # exits stay where the reference takes them: a search's outcome and the
    # "< 4 correspondences" test (:150-153, which reads correspondence indices
    # only) are decided on this thread before the next search starts, so no
    # search runs that the reference would not run.
    worker = getattr(ops, "post_worker", None)
    worker = worker() if worker is not None else None
    inflight = None

    def post_search(pending, prev, nxt, frame):
        """mainCycle.cpp:128-210 for one good frame; returns the BA window it
        started (or None)"""
        if pending is not None:
            pending.finish()            # K / R / t / points before PnP reads them
        obj, img = old_spatial_points_and_new_coords(nxt.allMatches, prev.correspondSpatialPointIdx,
                                                     gd.spatialPoints, nxt.allExtractedFeatures)
        found, rvec, tvec = ops.solve_pnp(obj, img, K)
        nxt.motion = np.asarray(tvec, np.float64).reshape(3, 1).copy()
        nxt.rotation = ops.rodrigues(rvec)
        logs.pose(nxt.rotation, nxt.motion)

        p1, p2 = key_point_coords(prev.allExtractedFeatures, nxt.allExtractedFeatures, nxt.allMatches)
        new_points = ops.reconstruct(K, prev.rotation, prev.motion, nxt.rotation, nxt.motion, p1, p2)
        push_new_spatial_points(frame, new_points, gd, prev.correspondSpatialPointIdx, nxt)

        processed.append(nxt.snapshot())
        if len(processed) >= cond.maxProcessedFramesVectorSz:
            if cond.useBundleAdjustment:
                started = start_bundle_adjustment(K, processed, gd, cond, ops, stats)
                processed.clear()
                return started
            move_processed_data_to_global_struct(processed, gd)
        return None

    def too_few(prev, matches):
        # PnP's "< 4 correspondences" exit (mainCycle.cpp:150-153)
        return len(matches) == 0 or int((prev.correspondSpatialPointIdx[matches["queryIdx"]] >= 0).sum()) < 4

    # With the worker, each good frame's task is queued behind the previous
    # frame's post-search work on the one worker thread, which decides the
    # frame's "< 4" exit as soon as that work is done and goes straight on to
    # this frame's (no round trip through this thread); this thread waits only
    # for the decision before it starts the next search.
    wstate = {"pending": None}

    def checked_post(prev, nxt, frame, decided, verdict):
        try:
            if "error" in wstate:            # an earlier frame's work failed: stop with its error
                raise wstate["error"]
            verdict["stop"] = too_few(prev, nxt.allMatches)
        finally:
            decided.set()
        if not verdict["stop"]:
            p, wstate["pending"] = wstate["pending"], None
            try:
                wstate["pending"] = post_search(p, prev, nxt, frame)
            except BaseException as e:
                wstate["error"] = e
                raise

    try:
        while True:
            nxt, prev = deque[last + 1], deque[last]
            bidx, frame, feats, matches = find_good_frame_from_batch(media, cond, batch, last_good, prev, ops)
            if bidx == EMPTY_BATCH or bidx == FRAME_NOT_FOUND:
                break
            nxt.allExtractedFeatures, nxt.allMatches = feats, matches
            if worker is not None:
                decided, verdict = threading.Event(), {}
                fut = worker.submit(checked_post, prev, nxt, frame, decided, verdict)
                decided.wait()
                if verdict.get("stop", True):
                    fut.result()                 # (re-raises a failure of the decision itself)
                    break
                inflight = fut
            else:
                if too_few(prev, matches):
                    break
                pending = post_search(pending, prev, nxt, frame)

            last_good = frame
            if last == OPTIMAL_DEQUE_SIZE - 2:
                deque.pop(0)
                deque.append(TemporalImageData())
            else:
                last += 1
            if stats is not None:
                stats["frames"] = stats.get("frames", 0) + 1
    finally:
        if inflight is not None:
            inflight.result()                    # FIFO worker: every queued task is done after the last
        if worker is not None:
            pending = wstate["pending"]

    if pending is not None:             # a loop exit right after a window (PnP's < 4 points)
        pending.finish()
    if processed:
        if cond.useBundleAdjustment:
            bundle_adjustment(K, processed, gd, cond, ops, stats)
        else:
            move_processed_data_to_global_struct(processed, gd)
    if bidx == EMPTY_BATCH:
        return EMPTY_BATCH
    return last


def define_camera_position(old_deque, last_id, fd):
    """mainCycleInternals.cpp:123-134."""
    if last_id < 0 or not old_deque:
        fd.rotation = np.eye(3)
        fd.motion = np.zeros((3, 1))
    else:
        fd.rotation = old_deque[last_id].rotation.copy()
        fd.motion = old_deque[last_id].motion.copy()


def slam_main(media, K, cfg, ops=None, out_dir=None, stats=None):
    """src/main.cpp:71-107 slamMain: mainCycle restarts from the last pose until
    the sequence ends, then points.txt / colors.txt.  K (3x3 float64) is
    updated in place by BA, as the reference's calibrationMatrix is.  Returns
    (GlobalData, Logs)."""
    ops = ops or GpuOps()
    cond = Conditions(cfg)
    logs = Logs(out_dir if out_dir is not None else None)
    gd = GlobalData()
    old, last_id = [], -1
    prefetch = getattr(ops, "prefetched", None)
    if getattr(media, "take", None) is not None:
        prefetch = None                 # DeviceMedia: the frames are resident already
    if prefetch is not None:
        media = prefetch(media, cond.featureExtractingThreshold)
    try:
        while True:
            deque = [TemporalImageData() for _ in range(OPTIMAL_DEQUE_SIZE)]
            define_camera_position(old, last_id, deque[0])
            ngd = GlobalData()
            last_id = main_cycle(media, K, cond, deque, ngd, logs, ops, stats)
            old = deque
            gd.push_points(ngd.spatialPoints, ngd.spatialPointsColors)
            gd.cameraRotations += ngd.cameraRotations
            gd.spatialCameraPositions += ngd.spatialCameraPositions
            if last_id <= 0:
                break
    finally:
        if prefetch is not None:
            media.close()
    logs.close(gd)
    return gd, logs
