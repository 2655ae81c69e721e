"""ctypes access to the CPU oracle (oracle/_build/liboracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this, as
the checker / CPU baseline.  The product (slam-indoor-code_amd/) never loads it.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "liboracle.so")

KP = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
               ("octave", "<i4"), ("class_id", "<i4")])
DM = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"), ("distance", "<f4")])
NORM_L1, NORM_L2, NORM_HAMMING = 2, 4, 6
LOSS_NONE, LOSS_TRIVIAL, LOSS_HUBER, LOSS_CAUCHY, LOSS_ARCTAN, LOSS_TUKEY = range(6)


class BASummary(ctypes.Structure):
    _fields_ = [("initial_cost", ctypes.c_double), ("final_cost", ctypes.c_double),
                ("num_residuals", ctypes.c_int), ("iterations", ctypes.c_int),
                ("successful_steps", ctypes.c_int), ("termination", ctypes.c_int), ("usable", ctypes.c_int)]


_O = None


def oracle():
    global _O
    if _O is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        O = ctypes.CDLL(ORACLE_SO)
        O.orc_fast_atan2_deg.restype = ctypes.c_float
        O.orc_fast_atan2_deg.argtypes = [ctypes.c_float, ctypes.c_float]
        O.orc_exp32f.restype = ctypes.c_float
        O.orc_exp32f.argtypes = [ctypes.c_float]
        O.orc_sift_sigma_diff.restype = ctypes.c_float
        O.orc_gauss_kernel_f32.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
        O.orc_fast_bgr.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        O.orc_fast.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_int]
        O.orc_fast_type.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        O.orc_fast_bgr_type.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        O.orc_bgr2gray.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
        O.orc_sift_compute.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                       ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        O.orc_orb_compute.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        O.orc_knn2.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        O.orc_knn2_l2_u8.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_void_p]
        O.orc_ratio.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
        O.orc_flann_knn2.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_void_p]
        O.orc_select_good.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        O.orc_ba.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                             ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                             ctypes.c_double, ctypes.c_int, ctypes.POINTER(BASummary)]
        O.orc_ba_set_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
        O.orc_ba_set_solver.argtypes = [ctypes.c_int, ctypes.c_void_p]
        O.orc_ba_cost.restype = ctypes.c_double
        O.orc_ba_cost.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_double]
        O.orc_aa_rotate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        O.orc_loss_eval.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
        O.orc_set_threads.argtypes = [ctypes.c_int]
        O.orc_sift_detect.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        O.orc_gauss_blur_f32.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                         ctypes.c_void_p]
        O.orc_resize2x_linear.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        O.orc_resize_half_nearest.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        O.orc_sift_sigmas.argtypes = [ctypes.c_void_p]
        O.orc_sift_sigma_diff2x.restype = ctypes.c_float
        O.orc_blur_ksize.argtypes = [ctypes.c_double]
        O.orc_sift_pyr_dims.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        O.orc_sift_pyramid.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p]
        O.orc_sift_ori_hist.restype = ctypes.c_float
        O.orc_sift_ori_hist.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_float, ctypes.c_void_p]
        O.orc_sift_peaks.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p]
        O.orc_kp_dedup_sorted.argtypes = [ctypes.c_void_p, ctypes.c_int]
        O.orc_reconstruct.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_int, ctypes.c_void_p]
        O.orc_projection.argtypes = [ctypes.c_void_p] * 4
        O.orc_estimate_transformation.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                  ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.POINTER(ctypes.c_int)]
        O.orc_five_point.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        O.orc_find_essential.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_double, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.POINTER(ctypes.c_int)]
        O.orc_ep_subsets.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        O.orc_ransac_update_iters.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int]
        O.orc_rodrigues_v2m.argtypes = [ctypes.c_void_p] * 3
        O.orc_rodrigues_m2v.argtypes = [ctypes.c_void_p] * 2
        O.orc_epnp.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5
        O.orc_pnp_iterative.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 3
        O.orc_solve_pnp_ransac.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_int, ctypes.c_float, ctypes.c_double, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        _O = O
    return _O


def vp(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def gray(bgr):
    h, w = bgr.shape[:2]
    out = np.zeros((h, w), np.uint8)
    b = np.ascontiguousarray(bgr)
    oracle().orc_bgr2gray(vp(b), w, h, b.strides[0], vp(out))
    return out


FAST_5_8, FAST_7_12, FAST_9_16 = range(3)


def fast(img, threshold, nms=True, type=FAST_9_16):
    img = np.ascontiguousarray(img)
    h, w = img.shape[:2]
    cap = max(1024, w * h // 8)
    while True:
        out = np.zeros(cap, KP)
        if img.ndim == 3:
            n = oracle().orc_fast_bgr_type(vp(img), w, h, img.strides[0], int(threshold), int(nms), int(type),
                                           vp(out), cap)
        else:
            n = oracle().orc_fast_type(vp(img), w, h, int(threshold), int(nms), int(type), vp(out), cap)
        if n <= cap:
            return out[:n].copy()
        cap = n


def _bgr(img):
    """the oracle's compute entry points take BGR; a 1-channel frame is what
    OpenCV uses as is (no cvtColor), and B = G = R = g converts back to exactly g
    ((1868 + 9617 + 4899) g + 8192) >> 14 = g), so it is expanded losslessly"""
    img = np.ascontiguousarray(img)
    if img.ndim == 2:
        img = np.ascontiguousarray(np.repeat(img[..., None], 3, 2))
    return img


def sift(bgr, kps):
    bgr = _bgr(bgr)
    h, w = bgr.shape[:2]
    k = np.ascontiguousarray(kps, KP)
    d = np.zeros((max(len(k), 1), 128), np.float32)
    oracle().orc_sift_compute(vp(bgr), w, h, bgr.strides[0], vp(k), len(k), vp(d))
    return d[:len(k)]


def sift_detect(bgr, with_desc=True):
    """full SIFT detector + descriptors (oracle/siftdet.c): (keypoints, N x 128 f32)"""
    bgr = _bgr(bgr)
    h, w = bgr.shape[:2]
    cap = max(4096, w * h // 16)
    out = np.zeros(cap, KP)
    d = np.zeros((cap, 128), np.float32) if with_desc else None
    n = oracle().orc_sift_detect(vp(bgr), w, h, bgr.strides[0], vp(out), cap, vp(d))
    assert n <= cap
    return out[:n].copy(), (d[:n].copy() if with_desc else None)


def sift_pyramid(gray_img):
    """[(gauss[6], dog[5]) per octave] of the detector's pyramid (doubled base)"""
    g = np.ascontiguousarray(gray_img, np.uint8)
    h, w = g.shape
    ow = np.zeros(32, np.int32)
    oh = np.zeros(32, np.int32)
    n = oracle().orc_sift_pyr_dims(w, h, vp(ow), vp(oh))
    tot = int(sum(int(ow[o]) * int(oh[o]) for o in range(n)))
    gauss = np.zeros(tot * 6, np.float32)
    dog = np.zeros(tot * 5, np.float32)
    oracle().orc_sift_pyramid(vp(g), w, h, vp(gauss), vp(dog))
    out, go, do = [], 0, 0
    for o in range(n):
        px = int(ow[o]) * int(oh[o])
        gs = [gauss[go + i * px: go + (i + 1) * px].reshape(int(oh[o]), int(ow[o])) for i in range(6)]
        ds = [dog[do + i * px: do + (i + 1) * px].reshape(int(oh[o]), int(ow[o])) for i in range(5)]
        go += 6 * px
        do += 5 * px
        out.append((gs, ds))
    return out


def gauss_blur_f32(img, sigma):
    a = np.ascontiguousarray(img, np.float32)
    h, w = a.shape
    out = np.zeros_like(a)
    oracle().orc_gauss_blur_f32(vp(a), w, h, float(sigma), vp(out))
    return out


def resize2x_linear(img):
    a = np.ascontiguousarray(img, np.float32)
    h, w = a.shape
    out = np.zeros((2 * h, 2 * w), np.float32)
    oracle().orc_resize2x_linear(vp(a), w, h, vp(out))
    return out


def reconstruct(K, R1, t1, R2, t2, p1, p2):
    """triangulate.cpp reconstruct(): n x 3 float64 (oracle/geom.c)"""
    a = [np.ascontiguousarray(v, np.float64).ravel() for v in (K, R1, t1, R2, t2)]
    q1 = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
    q2 = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
    out = np.zeros((max(len(q1), 1), 3), np.float64)
    oracle().orc_reconstruct(*[vp(v) for v in a], vp(q1), vp(q2), len(q1), vp(out))
    return out[:len(q1)]


def estimate_transformation(p1, p2, K, use_ransac=True, prob=0.999, threshold=5.0, dist=200.0):
    """cameraTranslation.cpp estimateTransformation: (ok, R 3x3, t 3, chirality mask, ransac mask, passed)"""
    q1 = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
    q2 = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
    n = len(q1)
    Kd = np.ascontiguousarray(K, np.float64).ravel()
    R = np.zeros(9)
    t = np.zeros(3)
    cm = np.zeros(max(n, 1), np.uint8)
    rm = np.zeros(max(n, 1), np.uint8)
    passed = ctypes.c_int(0)
    ok = oracle().orc_estimate_transformation(vp(q1), vp(q2), n, vp(Kd), int(use_ransac), prob, threshold, dist,
                                              vp(R), vp(t), vp(cm), vp(rm), ctypes.byref(passed))
    return bool(ok), R.reshape(3, 3), t, cm[:n], rm[:n], passed.value


def rodrigues(v):
    """cvRodrigues2 both ways: 3-vector -> (R 3x3, J 3x9); 3x3 -> rvec"""
    a = np.ascontiguousarray(v, np.float64)
    if a.size == 3:
        R = np.zeros(9)
        J = np.zeros(27)
        oracle().orc_rodrigues_v2m(vp(a), vp(R), vp(J))
        return R.reshape(3, 3), J.reshape(3, 9)
    r = np.zeros(3)
    oracle().orc_rodrigues_m2v(vp(a.ravel().copy()), vp(r))
    return r


def epnp(op, ip, K):
    """solvePnP(SOLVEPNP_EPNP) core: (R 3x3, t 3)"""
    o = np.ascontiguousarray(op, np.float64).reshape(-1, 3)
    m = np.ascontiguousarray(ip, np.float32).reshape(-1, 2)
    Kd = np.ascontiguousarray(K, np.float64).ravel()
    R = np.zeros(9)
    t = np.zeros(3)
    oracle().orc_epnp(len(o), vp(o), vp(m), vp(Kd), vp(R), vp(t))
    return R.reshape(3, 3), t


def pnp_iterative(op, ip, K, rvec, tvec):
    """cvFindExtrinsicCameraParams2 with an extrinsic guess: (rvec, tvec, iterations)"""
    o = np.ascontiguousarray(op, np.float64).reshape(-1, 3)
    m = np.ascontiguousarray(ip, np.float64).reshape(-1, 2)
    Kd = np.ascontiguousarray(K, np.float64).ravel()
    r = np.array(rvec, np.float64).ravel().copy()
    t = np.array(tvec, np.float64).ravel().copy()
    it = oracle().orc_pnp_iterative(vp(o), vp(m), len(o), vp(Kd), vp(r), vp(t))
    return r, t, it


def solve_pnp_ransac(op, ip, K, iterations=100, reproj=8.0, confidence=0.99):
    """solvePnPRansac with the reference's defaults: (status, rvec, tvec, inlier mask, n inliers)"""
    o = np.ascontiguousarray(op, np.float32).reshape(-1, 3)
    m = np.ascontiguousarray(ip, np.float32).reshape(-1, 2)
    n = len(o)
    Kd = np.ascontiguousarray(K, np.float64).ravel()
    r = np.zeros(3)
    t = np.zeros(3)
    mask = np.zeros(max(n, 1), np.uint8)
    ninl = ctypes.c_int(0)
    st = oracle().orc_solve_pnp_ransac(vp(o), vp(m), n, vp(Kd), iterations, reproj, confidence, vp(r), vp(t),
                                       vp(mask), ctypes.byref(ninl))
    return st, r, t, mask[:n], ninl.value


def five_point(q1, q2):
    a = np.ascontiguousarray(q1, np.float64).reshape(5, 2)
    b = np.ascontiguousarray(q2, np.float64).reshape(5, 2)
    E = np.zeros((10, 9))
    n = oracle().orc_five_point(vp(a), vp(b), vp(E))
    return E[:n].reshape(n, 3, 3)


def orb(bgr, kps):
    bgr = _bgr(bgr)
    h, w = bgr.shape[:2]
    k = np.ascontiguousarray(kps, KP).copy()
    d = np.zeros((max(len(k), 1), 32), np.uint8)
    n = oracle().orc_orb_compute(vp(bgr), w, h, bgr.strides[0], vp(k), len(k), vp(d))
    return k[:n].copy(), d[:n].copy()


def _u8_valued(a):
    return a.dtype == np.float32 and a.ndim == 2 and a.shape[1] == 128 and \
        bool(np.all((a >= 0) & (a <= 255) & (a == np.floor(a))))


def knn2(q, t, norm, exact_f32=False):
    """orc_knn2 (k = 2 brute force).  Integer-valued 128-D f32 L2 inputs (SIFT
    descriptors) take orc_knn2_l2_u8, which is exactly the same computation
    (oracle/knn.c); exact_f32 forces the f32 scan."""
    q = np.ascontiguousarray(q)
    t = np.ascontiguousarray(t)
    dim = q.shape[1] if q.ndim == 2 else (t.shape[1] if t.ndim == 2 else 0)
    idx = np.zeros((len(q), 2), np.int32)
    dist = np.zeros((len(q), 2), np.float32)
    if (norm == NORM_L2 and not exact_f32 and len(q) and len(t) and _u8_valued(q) and _u8_valued(t)):
        qu, tu = q.astype(np.uint8), t.astype(np.uint8)
        oracle().orc_knn2_l2_u8(vp(qu), len(q), vp(tu), len(t), vp(idx), vp(dist))
        return idx, dist
    oracle().orc_knn2(vp(q), len(q), vp(t), len(t), dim, norm, vp(idx), vp(dist))
    return idx, dist


def ratio(idx, dist, r):
    out = np.zeros(max(len(idx), 1), DM)
    n = oracle().orc_ratio(vp(np.ascontiguousarray(idx)), vp(np.ascontiguousarray(dist)), len(idx), float(r),
                           vp(out))
    return out[:n].copy()


def select_good(counts, required, skip_head, first_fit):
    c = np.ascontiguousarray(counts, np.int32)
    return oracle().orc_select_good(vp(c), len(c), int(required), int(skip_head), int(bool(first_fit)))


BA_SOLVER_LLT, BA_SOLVER_LDLT, BA_SOLVER_GAUSS_FMA = 0, 1, 2


def ba(K4, ext, pts, of, op, oxy, loss=LOSS_NONE, a=0.0, max_iters=50, trace=None, solver=BA_SOLVER_LLT):
    """trace: optional float64 array, filled with the cost after each LM
    iteration (trace[k - 1] = what a run capped at k iterations reports).
    solver: the reduced camera system's factorisation (oracle/ba.c): the dense
    LL' restatement (default), Eigen SimplicialLDLT's arithmetic (Ceres 2.2's
    SPARSE_SCHUR on EIGEN_SPARSE, the reference's configuration), or the GPU
    solve's arithmetic (diagnostics).  Set for this call on this thread only."""
    K4 = np.array(K4, np.float64)
    ext = np.array(ext, np.float64)
    pts = np.array(pts, np.float64)
    of = np.ascontiguousarray(of, np.int32)
    op = np.ascontiguousarray(op, np.int32)
    oxy = np.ascontiguousarray(oxy, np.float64)
    s = BASummary()
    if trace is not None:
        assert trace.dtype == np.float64 and trace.flags.c_contiguous
        oracle().orc_ba_set_trace(vp(trace), len(trace))
    if solver != BA_SOLVER_LLT:
        oracle().orc_ba_set_solver(int(solver), None)
    try:
        oracle().orc_ba(vp(K4), ext.shape[0], vp(ext), pts.shape[0], vp(pts), len(of), vp(of), vp(op), vp(oxy),
                        int(loss), float(a), int(max_iters), ctypes.byref(s))
    finally:
        if trace is not None:
            oracle().orc_ba_set_trace(None, 0)
        if solver != BA_SOLVER_LLT:
            oracle().orc_ba_set_solver(BA_SOLVER_LLT, None)
    return K4, ext, pts, s


def ba_cost(K4, ext, pts, of, op, oxy, loss=LOSS_NONE, a=0.0):
    K4 = np.ascontiguousarray(K4, np.float64)
    ext = np.ascontiguousarray(ext, np.float64)
    pts = np.ascontiguousarray(pts, np.float64)
    return oracle().orc_ba_cost(vp(K4), vp(ext), vp(pts), len(of), vp(np.ascontiguousarray(of, np.int32)),
                                vp(np.ascontiguousarray(op, np.int32)), vp(np.ascontiguousarray(oxy, np.float64)),
                                int(loss), float(a))


def flann_knn2(q, t, trees=4, checks=32, seed=1):
    """FlannBasedMatcher knnMatch(k = 2) restatement (KD-forest, approximate; oracle/flann.c)"""
    q = np.ascontiguousarray(q, np.float32)
    t = np.ascontiguousarray(t, np.float32)
    idx = np.zeros((len(q), 2), np.int32)
    dist = np.zeros((len(q), 2), np.float32)
    oracle().orc_flann_knn2(vp(q), len(q), vp(t), len(t), q.shape[1], trees, checks, seed, vp(idx), vp(dist))
    return idx, dist
