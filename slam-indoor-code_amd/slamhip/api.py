"""Host-side mirror of the reference's hot-path interface, over libslamhip.

Names, argument meaning and error behaviour follow the reference's mainModule
headers so that a caller (or a parity test) reads like the reference:

  fastExtractor            src/mainModule/featureExtraction/fastExtractor.h:19-21
  extractDescriptor        src/mainModule/featureMatching/featureMatching.h:12-17
  matchFramesPairFeatures  featureMatching.h:47-53 (the 5-arg overload the batch uses)
  matchFeatures            featureMatchingCPU.cpp:17-43 (static in the reference)
  getGoodMatches           featureMatchingCommon.h:45-48
  getMatcherTypeIndex      featureMatchingCommon.h:19
  bundleAdjustment         src/mainModule/bundleAdjustment/bundleAdjustment.h:50-54

C++ passes containers by reference and mutates them; here the outputs are
returned (numpy arrays cannot shrink in place): ORB's border filter returns the
filtered keypoint array, exactly the vector the reference's caller ends up with.
Every computation runs in the HIP library on the GPU; there is no CPU path.
"""
import ctypes
import math

import numpy as np

from . import _lib as L
from ._lib import DMATCH_DTYPE, KEYPOINT_DTYPE, check, lib, ptr


class MatcherTypeError(Exception):
    """getMatcherTypeIndex / extractDescriptor with an invalid type (the reference
    throws std::exception, featureMatchingCommon.cpp:20, featureMatchingCPU.cpp:37,63)."""


_default_ctx = None


class Context:
    """One HIP stream + device workspace (slam_ctx).  Not thread-safe: the
    reference's worker threads (batch.cpp:181-200) each need their own."""

    def __init__(self, device=0, priority=0):
        """priority > 0: the stream gets the device's highest priority
        (slam_create_prio)"""
        self.device = device
        self._det_out = None     # siftDetectAndCompute's reusable host output space (key, kps, desc)
        self.handle = lib().slam_create_prio(device, int(priority)) if priority else lib().slam_create(device)
        if not self.handle:
            raise L.SlamError(L.SLAM_E_NO_DEVICE, f"cannot open HIP device {device}")

    def set_option(self, option, value):
        """slam_set_option: per-context choices (all but L.OPT_PNP_SUMS never change results; e.g.
        L.OPT_SIFT_KERNEL -> L.SIFT_KERNEL_BAND / _TAB / _GENERAL / _AUTO)."""
        L.check(lib().slam_set_option(self.handle, int(option), int(value)), self.handle)

    def close(self):
        self._det_out = None
        if self.handle:
            lib().slam_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


def _img(a):
    a = np.ascontiguousarray(a)
    if a.dtype != np.uint8:
        raise TypeError("frames are 8-bit (CV_8UC1/3/4)")
    if a.ndim == 2:
        return a, a.shape[1], a.shape[0], 1
    if a.ndim == 3 and a.shape[2] in (3, 4):
        return a, a.shape[1], a.shape[0], a.shape[2]
    raise ValueError("frame must be HxW, HxWx3 (BGR) or HxWx4")


def _ctx(ctx):
    return (ctx or default_context()).handle


def fastExtractor(srcImage, threshold=10, suppression=True, type=L.TYPE_9_16, ctx=None):
    """FAST keypoints of a BGR (or gray) frame, raster order (fastExtractor.cpp:7-13)."""
    c = _ctx(ctx)
    img, w, h, ch = _img(srcImage)
    cap = max(4096, w * h // 16)
    while True:
        out = np.empty(cap, KEYPOINT_DTYPE)      # the library writes the first n (no zero fill: cap is ~w*h/16)
        n = ctypes.c_int(0)
        rc = lib().slam_fast(c, ptr(img), w, h, img.strides[0], ch, int(threshold), int(bool(suppression)),
                             int(type), ptr(out), cap, ctypes.byref(n))
        if rc == L.SLAM_E_CAPACITY:
            cap = n.value
            continue
        check(rc, c)
        return out[:n.value].copy()


def getMatcherTypeIndex(config):
    """featureMatchingCommon.cpp:13-21: SIFT_BF > SIFT_FLANN > ORB."""
    t = lib().slam_matcher_type(int(bool(config.getValue("useFM-SIFT-BF"))),
                                int(bool(config.getValue("useFM-SIFT-FLANN"))),
                                int(bool(config.getValue("useFM-ORB"))))
    if t < 0:
        raise MatcherTypeError("no feature matcher selected")
    return t


def _check_type(t):
    if t not in (L.SIFT_BF, L.SIFT_FLANN, L.ORB_BF):
        raise MatcherTypeError(f"invalid matcher type {t}")


def extractDescriptor(frame, features, extractorType, ctx=None):
    """SIFT (n x 128 float32, integer values) or ORB (n x 32 uint8) descriptors.
    Returns (features, desc); ORB returns the border-filtered keypoints."""
    _check_type(extractorType)
    c = _ctx(ctx)
    img, w, h, ch = _img(frame)
    kps = np.ascontiguousarray(np.asarray(features, KEYPOINT_DTYPE)).copy()
    n = ctypes.c_int(len(kps))
    if extractorType == L.ORB_BF:
        desc = np.empty((max(len(kps), 1), 32), np.uint8)      # the first n rows are written
    else:
        desc = np.empty((max(len(kps), 1), 128), np.float32)
    rc = lib().slam_describe(c, ptr(img), w, h, img.strides[0], ch, int(extractorType), ptr(kps), ctypes.byref(n),
                             ptr(desc))
    check(rc, c)
    return kps[:n.value].copy(), desc[:n.value].copy()


def siftDetectAndCompute(frame, ctx=None, with_descriptors=True):
    """cv::SIFT::create()->detectAndCompute(frame, noArray(), kps, desc): the full
    detector (DoG pyramid on the doubled image, extrema, orientation histogram)
    + 128-D descriptors (n x 128 float32, integer values).  Returns (kps, desc)."""
    cobj = ctx or default_context()
    c = cobj.handle
    img, w, h, ch = _img(frame)
    cap = max(4096, w * h // 16)
    while True:
        # output space kept on the context between its calls and freed by
        # Context.close() (the first n rows are copied out): a fresh
        # w * h / 16-row array per frame cost its page faults
        key = (cap, bool(with_descriptors))
        det = cobj._det_out
        if det is None or det[0] != key:
            det = (key, np.empty(cap, KEYPOINT_DTYPE), np.empty((cap, 128), np.float32) if with_descriptors else None)
            cobj._det_out = det
        _, kps, desc = det
        n = ctypes.c_int(0)
        rc = lib().slam_sift_detect(c, ptr(img), w, h, img.strides[0], ch, ptr(kps), cap, ctypes.byref(n),
                                    ptr(desc) if desc is not None else None)
        if rc == L.SLAM_E_CAPACITY and n.value > cap:
            cap = n.value
            continue
        check(rc, c)
        k = kps[:n.value].copy()
        return k, (desc[:n.value].copy() if desc is not None else None)


class SiftBatch:
    """siftDetectAndComputeBatch's result: keypoints (n, cap) and descriptors
    (n, cap, 128) float32 in device memory (torch tensors; frame f's first
    counts[f] rows are its keypoints / descriptors), counts (n,) on the host."""

    def __init__(self, kps_dev, desc_dev, counts):
        self.kps_dev, self.desc_dev, self.counts = kps_dev, desc_dev, counts

    def __len__(self):
        return len(self.counts)

    def host(self, f):
        """frame f's (keypoints, descriptors) as siftDetectAndCompute returns them"""
        n = int(self.counts[f])
        k = self.kps_dev[f, :n].cpu().numpy().reshape(-1).view(KEYPOINT_DTYPE).copy()
        d = self.desc_dev[f, :n].cpu().numpy().copy() if self.desc_dev is not None else None
        return k, d


def siftDetectAndComputeBatch(frames, ctx=None, with_descriptors=True, cap=None):
    """siftDetectAndCompute over a device-resident batch: frames is a CUDA uint8
    tensor (n, h, w, 3) or (n, h, w), already in HBM (slam_sift_detect_batch;
    every kernel launch covers the batch).  The keypoints and descriptors stay
    in device memory: returns a SiftBatch (SiftBatch.host(f) gives frame f's
    (kps, desc) as siftDetectAndCompute returns them)."""
    import torch
    c = _ctx(ctx)
    if not (frames.is_cuda and frames.dtype == torch.uint8 and frames.dim() in (3, 4)):
        raise ValueError("frames: a CUDA uint8 tensor (n, h, w[, 3])")
    frames = frames.contiguous()
    n, h, w = frames.shape[:3]
    ch = frames.shape[3] if frames.dim() == 4 else 1
    torch.cuda.current_stream(frames.device).synchronize()   # the library's stream reads the frames next
    cap = cap or max(4096, w * h // 32)
    while True:
        kps = torch.empty((n, cap, KEYPOINT_DTYPE.itemsize), dtype=torch.uint8, device=frames.device)
        desc = torch.empty((n, cap, 128), dtype=torch.float32, device=frames.device) if with_descriptors else None
        cnt = np.zeros(n, np.int32)
        rc = lib().slam_sift_detect_batch(c, None, ctypes.c_void_p(frames.data_ptr()), n, w, h, ch,
                                          ctypes.c_void_p(kps.data_ptr()), cap, ptr(cnt),
                                          ctypes.c_void_p(desc.data_ptr()) if desc is not None else None)
        if rc == L.SLAM_E_CAPACITY and n and int(cnt.max()) > cap:
            cap = int(cnt.max())
            continue
        check(rc, c)
        return SiftBatch(kps, desc, cnt)


def reconstruct(calibration, rotation1, transition1, rotation2, transition2, points1, points2, ctx=None):
    """triangulate.cpp:74-100 reconstruct(): DLT triangulation of matched
    points (Point2f, n x 2) seen from two cameras [R | t] with intrinsics K.
    Returns spatialPoints as an n x 3 float64 array (Point3d)."""
    c = _ctx(ctx)
    K = np.ascontiguousarray(calibration, np.float64).reshape(3, 3)
    R1 = np.ascontiguousarray(rotation1, np.float64).reshape(3, 3)
    R2 = np.ascontiguousarray(rotation2, np.float64).reshape(3, 3)
    t1 = np.ascontiguousarray(transition1, np.float64).reshape(3)
    t2 = np.ascontiguousarray(transition2, np.float64).reshape(3)
    p1 = np.ascontiguousarray(points1, np.float32).reshape(-1, 2)
    p2 = np.ascontiguousarray(points2, np.float32).reshape(-1, 2)
    if len(p1) != len(p2):
        raise ValueError("points1 and points2 differ in length")
    out = np.zeros((max(len(p1), 1), 3), np.float64)
    check(lib().slam_reconstruct(c, ptr(K), ptr(R1), ptr(t1), ptr(R2), ptr(t2), ptr(p1), ptr(p2), len(p1),
                                 ptr(out)), c)
    return out[:len(p1)].copy()


def estimateTransformation(points1, points2, calibrationMatrix, useRANSAC=True, RANSACProb=0.999,
                           RANSACThreshold=5.0, distanceThreshold=200.0, ctx=None):
    """cameraTranslation.cpp:32-69 estimateTransformation(): findEssentialMat
    (RANSAC) + recoverPose on matched points (n x 2).  The config keys
    RPUseRANSAC / RPRANSACProb / RPRANSACThreshold / RPDistanceThreshold are
    the keyword arguments.  Returns (ok, R 3x3, t 3, chiralityMask, ransacMask)."""
    c = _ctx(ctx)
    p1 = np.ascontiguousarray(points1, np.float32).reshape(-1, 2)
    p2 = np.ascontiguousarray(points2, np.float32).reshape(-1, 2)
    if len(p1) != len(p2):
        raise ValueError("points1 and points2 differ in length")
    n = len(p1)
    K = np.ascontiguousarray(calibrationMatrix, np.float64).reshape(3, 3)
    R = np.zeros((3, 3))
    t = np.zeros(3)
    cm = np.zeros(max(n, 1), np.uint8)
    rm = np.zeros(max(n, 1), np.uint8)
    passed = ctypes.c_int(0)
    check(lib().slam_estimate_transformation(c, ptr(p1), ptr(p2), n, ptr(K), int(bool(useRANSAC)),
                                             float(RANSACProb), float(RANSACThreshold), float(distanceThreshold),
                                             ptr(R), ptr(t), ptr(cm), ptr(rm), ctypes.byref(passed)), c)
    return passed.value > 0, R, t, cm[:n].copy(), rm[:n].copy()


def solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs=None, iterationsCount=100,
                   reprojectionError=8.0, confidence=0.99, ctx=None):
    """mainCycle.cpp:155-161 solvePnPRansac(objectPoints, imagePoints,
    calibrationMatrix, distortionCoeffs, rvec, tvec) with OpenCV's defaults:
    EPnP RANSAC + SOLVEPNP_ITERATIVE refinement on the inliers.  Returns
    (retval, rvec (3, 1), tvec (3, 1), inliers (k, 1) int32 or None) as cv2
    does.  distCoeffs must be empty / zero (the reference never sets it)."""
    if distCoeffs is not None and np.any(np.asarray(distCoeffs, np.float64) != 0):
        raise ValueError("solvePnPRansac: only zero distortion is supported (the reference passes an empty Mat)")
    c = _ctx(ctx)
    op = np.ascontiguousarray(objectPoints, np.float32).reshape(-1, 3)
    ip = np.ascontiguousarray(imagePoints, np.float32).reshape(-1, 2)
    if len(op) != len(ip):
        raise ValueError("objectPoints and imagePoints differ in length")
    n = len(op)
    K = np.ascontiguousarray(cameraMatrix, np.float64).reshape(3, 3)
    rvec = np.zeros(3)
    tvec = np.zeros(3)
    mask = np.zeros(max(n, 1), np.uint8)
    ninl = ctypes.c_int(0)
    found = ctypes.c_int(0)
    check(lib().slam_solve_pnp_ransac(c, ptr(op), ptr(ip), n, ptr(K), int(iterationsCount), float(reprojectionError),
                                      float(confidence), ptr(rvec), ptr(tvec), ptr(mask), ctypes.byref(ninl),
                                      ctypes.byref(found)), c)
    inl = np.flatnonzero(mask[:n]).astype(np.int32).reshape(-1, 1) if found.value else None
    return bool(found.value), rvec.reshape(3, 1), tvec.reshape(3, 1), inl


def _desc_arg(desc, t):
    if t == L.ORB_BF:
        return np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    return np.ascontiguousarray(desc, np.float32).reshape(-1, 128)


def knnMatch2(queryDescriptors, trainDescriptors, matcherType, norm=L.NORM_DEFAULT, ctx=None):
    """DescriptorMatcher::knnMatch(query, train, k = 2): (idx nq x 2, dist nq x 2)."""
    _check_type(matcherType)
    c = _ctx(ctx)
    q, t = _desc_arg(queryDescriptors, matcherType), _desc_arg(trainDescriptors, matcherType)
    idx = np.zeros((len(q), 2), np.int32)
    dist = np.zeros((len(q), 2), np.float32)
    if len(q):
        check(lib().slam_knn2(c, ptr(q), len(q), ptr(t), len(t), int(matcherType), int(norm), ptr(idx), ptr(dist)), c)
    return idx, dist


def getGoodMatches(idx, dist, knnMatcherDistance):
    """featureMatchingCommon.cpp:37-50 on knnMatch2 output (query order)."""
    ok = (idx[:, 0] >= 0) & (idx[:, 1] >= 0)
    ok &= dist[:, 0].astype(np.float64) < knnMatcherDistance * dist[:, 1].astype(np.float64)
    q = np.nonzero(ok)[0]
    out = np.zeros(len(q), DMATCH_DTYPE)
    out["queryIdx"] = q
    out["trainIdx"] = idx[q, 0]
    out["distance"] = dist[q, 0]
    return out


def matchFeatures(prevDesc, curDesc, extractorType, knnMatcherDistance, norm=L.NORM_DEFAULT, ctx=None):
    """knnMatch(prev = query, cur = train, 2) + getGoodMatches, fused on the GPU."""
    _check_type(extractorType)
    c = _ctx(ctx)
    q, t = _desc_arg(prevDesc, extractorType), _desc_arg(curDesc, extractorType)
    cap = max(len(q), 1)
    out = np.zeros(cap, DMATCH_DTYPE)
    n = ctypes.c_int(0)
    check(lib().slam_match(c, ptr(q), len(q), ptr(t), len(t), int(extractorType), int(norm),
                           float(knnMatcherDistance), ptr(out), cap, ctypes.byref(n)), c)
    return out[:n.value].copy()


def matchFramesPairFeatures(firstFrameDescriptor, secondFrame, secondFeatures, matcherType, knnMatcherDistance,
                            norm=L.NORM_DEFAULT, ctx=None):
    """featureMatchingCPU.cpp:83-95: describe the candidate, then match against the
    previous frame's descriptors.  Returns (secondFeatures, matches)."""
    _check_type(matcherType)
    kps, desc = extractDescriptor(secondFrame, secondFeatures, matcherType, ctx=ctx)
    if len(firstFrameDescriptor) == 0 or len(kps) == 0:
        return kps, np.zeros(0, DMATCH_DTYPE)
    return kps, matchFeatures(firstFrameDescriptor, desc, matcherType, knnMatcherDistance, norm=norm, ctx=ctx)


def selectGoodFrame(match_counts, requiredMatchedPointsCount, skipFramesFromBatchHead, useFirstFitInBatch):
    """batch.cpp:136-146 / :280-316 selection rule (index or FRAME_NOT_FOUND)."""
    a = np.ascontiguousarray(match_counts, np.int32)
    return lib().slam_select_good(ptr(a), len(a), int(requiredMatchedPointsCount), int(skipFramesFromBatchHead),
                                  int(bool(useFirstFitInBatch)))


# ---- bundle adjustment -------------------------------------------------------

def rodrigues_to_vector(R):
    """cv::Rodrigues(3x3 -> 3x1) (cvRodrigues2 restated, host code in
    libslamhip), as used by convertDataForBA (bundleAdjustment.cpp:167)."""
    src = np.ascontiguousarray(R, np.float64).reshape(9).copy()
    out = np.zeros(3)
    check(lib().slam_rodrigues(ptr(src), 9, ptr(out)))
    return out


def rodrigues_to_matrix(r):
    """cv::Rodrigues(3x1 -> 3x3) (cvRodrigues2 restated, host code in
    libslamhip), as used by convertDataFromBA (bundleAdjustment.cpp:195) and
    after solvePnPRansac (mainCycle.cpp:162)."""
    src = np.ascontiguousarray(r, np.float64).reshape(3).copy()
    out = np.zeros(9)
    check(lib().slam_rodrigues(ptr(src), 3, ptr(out)))
    return out.reshape(3, 3)


def loss_from_config(config):
    """getLossFunction (bundleAdjustment.cpp:131-151): priority
    Trivial > Huber > Cauchy > Arctan > Tukey > none."""
    g = config.getValue
    if g("BAUseTrivialLossFunction"):
        return L.LOSS_TRIVIAL, 0.0
    for flag, par, kind in (("BAUseHuberLossFunction", "BAHuberLossFunctionParameter", L.LOSS_HUBER),
                            ("BAUseCauchyLossFunction", "BACauchyLossFunctionParameter", L.LOSS_CAUCHY),
                            ("BAUseArctanLossFunction", "BAArctanLossFunctionParameter", L.LOSS_ARCTAN),
                            ("BAUseTukeyLossFunction", "BATukeyLossFunctionParameter", L.LOSS_TUKEY)):
        if g(flag):
            return kind, float(g(par))
    return L.LOSS_NONE, 0.0


def bundle_adjust_arrays(K4, ext6, pts3, obs_frame, obs_point, obs_xy, loss=L.LOSS_NONE, loss_param=0.0,
                         max_iters=50, ctx=None):
    """slam_ba on plain arrays; K4, ext6 (nf x 6), pts3 (np x 3) are updated IN PLACE."""
    c = _ctx(ctx)
    for a in (K4, ext6, pts3):
        if a.dtype != np.float64 or not a.flags.c_contiguous:
            raise TypeError("BA parameter arrays must be C-contiguous float64")
    of = np.ascontiguousarray(obs_frame, np.int32)
    op = np.ascontiguousarray(obs_point, np.int32)
    oxy = np.ascontiguousarray(obs_xy, np.float64).reshape(-1, 2)
    s = L.BASummary()
    check(lib().slam_ba(c, ptr(K4), ext6.shape[0], ptr(ext6), pts3.shape[0], ptr(pts3), len(of), ptr(of), ptr(op),
                        ptr(oxy), int(loss), float(loss_param), int(max_iters), ctypes.byref(s)), c)
    return s


class TemporalImageData:
    """mainCycleStructures.h:38-45 (the fields BA reads and writes)."""

    def __init__(self, allExtractedFeatures, correspondSpatialPointIdx, rotation, motion):
        self.allExtractedFeatures = allExtractedFeatures
        self.correspondSpatialPointIdx = np.asarray(correspondSpatialPointIdx, np.int64)
        self.rotation = np.asarray(rotation, np.float64)
        self.motion = np.asarray(motion, np.float64).reshape(3, 1)


class GlobalData:
    """mainCycleStructures.h:49-54 (spatialPoints as an N x 3 float64 array)."""

    def __init__(self, spatialPoints):
        self.spatialPoints = np.ascontiguousarray(spatialPoints, np.float64)


def bundleAdjustment(calibrationMatrix, imagesDataForAdjustment, globalData, config, ctx=None):
    """bundleAdjustment.cpp:73-129: builds the observation list in the reference's
    AddResidualBlock order (frame, then keypoint), solves, writes K, R, t and the
    points back in place.  Returns the summary (RMSE as logged at :125-126)."""
    K = calibrationMatrix
    K4 = np.array([K[0, 0], K[1, 1], K[0, 2], K[1, 2]], np.float64)
    ext = np.zeros((len(imagesDataForAdjustment), 6), np.float64)
    of, op, oxy = [], [], []
    for i, im in enumerate(imagesDataForAdjustment):
        ext[i, :3] = rodrigues_to_vector(im.rotation)
        ext[i, 3:] = im.motion.reshape(3)
        kps = im.allExtractedFeatures
        for p, idx in enumerate(im.correspondSpatialPointIdx):
            if idx < 0:
                continue
            of.append(i)
            op.append(int(idx))
            oxy.append((float(kps[p]["x"]), float(kps[p]["y"])))
    loss, par = loss_from_config(config)
    pts = globalData.spatialPoints
    summary = bundle_adjust_arrays(K4, ext, pts, np.array(of, np.int32), np.array(op, np.int32),
                                   np.array(oxy, np.float64).reshape(-1, 2), loss, par, ctx=ctx)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = K4
    for i, im in enumerate(imagesDataForAdjustment):
        im.rotation[...] = rodrigues_to_matrix(ext[i, :3])
        im.motion[...] = ext[i, 3:].reshape(3, 1)
    return summary


def ba_rmse(summary):
    """the reference's logged 'RMSE' = sqrt(cost / num_residuals) (:125-126)."""
    if summary.num_residuals == 0:
        return 0.0
    return math.sqrt(summary.initial_cost / summary.num_residuals), math.sqrt(summary.final_cost / summary.num_residuals)


SYNTH_DRIFT, SYNTH_STEADY = 0, 1


def synth_frames(w, h, first, count, seed=1234, path=SYNTH_DRIFT):
    """Deterministic synthetic indoor sequence (count x h x w x 3 BGR uint8).
    path: SYNTH_DRIFT (the camera zooms in along the sequence, so the FAST count
    falls with the frame index; the fixtures' path) or SYNTH_STEADY (a bounded
    loop: every frame near frame 0's FAST count; the bench's configs[1] batches)."""
    out = np.zeros((count, h, w, 3), np.uint8)
    check(lib().slam_synth_sequence(w, h, first, count, ctypes.c_uint64(seed), int(path), ptr(out)))
    return out


def synth_frames_dev(w, h, first, count, seed=1234, path=SYNTH_DRIFT, ctx=None, out=None):
    """synth_frames rendered on the device (slam_synth_sequence_dev): a torch
    uint8 tensor (count, h, w, 3) in HBM, byte-identical to synth_frames."""
    import torch
    ctx = ctx or default_context()
    if out is None:
        out = torch.empty((count, h, w, 3), dtype=torch.uint8, device=torch.device("cuda", ctx.device))
    assert out.is_contiguous() and tuple(out.shape) == (count, h, w, 3) and out.dtype == torch.uint8
    torch.cuda.current_stream(out.device).synchronize()
    check(lib().slam_synth_sequence_dev(ctx.handle, None, w, h, first, count, ctypes.c_uint64(seed), int(path),
                                        ctypes.c_void_p(out.data_ptr()) if count else None), ctx.handle)
    return out
