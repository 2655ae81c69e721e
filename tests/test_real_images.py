"""Parity on natural images: the reference's own calibration photos
(docs/artifact/calibration, decoded once into tests/golden/real_*.npz by
tests/golden/make_real_fixtures.py).  The synthetic indoor sequence has sharp,
axis-aligned texture; these frames exercise FAST, the SIFT orientation wrap,
ORB and the matchers on real image statistics (JPEG noise, blur, a fisheye
lens).  The oracle computes the expected values at test time; the fixtures
also hold the oracle's FAST counts, re-checked on the CPU."""
import os

import numpy as np
import pytest

import oracle_ffi as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="module")
def real():
    v, h = _load("real_vga.npz"), _load("real_1080p.npz")
    return {"vga": v["bgr"], "gray": v["gray"], "hd": h["bgr"]}


def test_real_fixture_fast_counts_cpu(real):
    """the committed oracle FAST counts still hold (CPU, no GPU)"""
    v, h = _load("real_vga.npz"), _load("real_1080p.npz")
    ims = list(real["vga"]) + list(real["gray"])
    got = [[len(O.fast(im, t, True)) for t in (10, 20)] for im in ims]
    np.testing.assert_array_equal(got, v["fast_counts"])
    np.testing.assert_array_equal([[len(O.fast(real["hd"][0], t, True)) for t in (10, 20)]], h["fast_counts"])


def kp_equal(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        np.testing.assert_array_equal(a[f], b[f], err_msg=f)


@pytest.mark.gpu
@pytest.mark.parametrize("thr", [10, 20, 40])
@pytest.mark.parametrize("nms", [True, False])
def test_real_fast(gpu_ctx, real, thr, nms):
    import slamhip
    for im in list(real["vga"]) + list(real["gray"]) + list(real["hd"]):
        kp_equal(slamhip.fastExtractor(im, thr, nms, ctx=gpu_ctx), O.fast(im, thr, nms))


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["auto", "tab"])
def test_real_sift_bitexact(real, kernel):
    """SIFT descriptors of FAST keypoints (the reference path) on every real
    frame, 1080p included, through the host-buffer entry point: bit-exact"""
    import slamhip
    from slamhip import _lib as L
    ctx = slamhip.Context(0)
    if kernel == "tab":
        ctx.set_option(L.OPT_SIFT_KERNEL, L.SIFT_KERNEL_TAB)
    try:
        for im in list(real["vga"]) + list(real["gray"]) + list(real["hd"]):
            kps = O.fast(im, 10, True)
            ko, d = slamhip.extractDescriptor(im, kps, slamhip.SIFT_FLANN, ctx=ctx)
            kp_equal(ko, kps)
            np.testing.assert_array_equal(d, O.sift(im, kps))
    finally:
        ctx.close()


@pytest.mark.gpu
def test_real_orb_bitexact(gpu_ctx, real):
    import slamhip
    for im in list(real["vga"]) + list(real["gray"]) + list(real["hd"]):
        kps = O.fast(im, 10, True)
        rk, rd = O.orb(im, kps)
        ko, d = slamhip.extractDescriptor(im, kps, slamhip.ORB_BF, ctx=gpu_ctx)
        kp_equal(ko, rk)                       # in-place border filter
        np.testing.assert_array_equal(d, rd)


@pytest.mark.gpu
@pytest.mark.parametrize("matcher", ["sift", "orb"])
def test_real_match_pairs(gpu_ctx, real, matcher):
    """kNN (k = 2) + ratio between consecutive real frames, and between the
    1080p frame and each VGA crop: every DMatch bit-exact"""
    import slamhip
    m = slamhip.SIFT_FLANN if matcher == "sift" else slamhip.ORB_BF
    norm = O.NORM_L2 if matcher == "sift" else O.NORM_HAMMING
    ims = list(real["vga"]) + list(real["hd"])
    desc = []
    for im in ims:
        k = O.fast(im, 10, True)
        desc.append(O.sift(im, k) if matcher == "sift" else O.orb(im, k)[1])
    pairs = [(0, 1), (1, 2), (2, 3), (4, 0), (4, 3)]
    for a, b in pairs:
        ri, rd = O.knn2(desc[a], desc[b], norm)
        ref = O.ratio(ri, rd, 0.7)
        got = slamhip.matchFeatures(desc[a], desc[b], m, 0.7, ctx=gpu_ctx)
        np.testing.assert_array_equal(got, ref)
        # and through matchFramesPairFeatures (describe + match on the device)
        k = O.fast(ims[b], 10, True)
        _, got2 = slamhip.matchFramesPairFeatures(desc[a], ims[b], k, m, 0.7, ctx=gpu_ctx)
        np.testing.assert_array_equal(got2, ref)


@pytest.mark.gpu
def test_real_batch_path(gpu_ctx, real):
    """the device batch (FAST + SIFT + kNN of every frame against frame 0) on
    the four real VGA frames"""
    import torch
    from slamhip.batch import DeviceBatch
    db = DeviceBatch(gpu_ctx)
    fr = real["vga"]
    kc = db.extract(torch.from_numpy(fr).cuda(), 10, 1)
    ref_d = []
    for i, im in enumerate(fr):
        k = O.fast(im, 10, True)
        assert kc[i] == len(k)
        kp_equal(db.keypoints(i), k)
        ref_d.append(O.sift(im, k))
        np.testing.assert_array_equal(db.descriptors(i), ref_d[-1])
    q, nq = db.export_desc(0)
    mc = db.match(q, nq, 0.7)
    for i in range(len(fr)):
        ri, rd = O.knn2(ref_d[0], ref_d[i], O.NORM_L2)
        ref = O.ratio(ri, rd, 0.7)
        assert mc[i] == len(ref)
        np.testing.assert_array_equal(db.matches(i, nq), ref)


@pytest.mark.gpu
def test_real_sift_detector(gpu_ctx, real):
    """the full SIFT detector (8(f) rank 2) on a real frame and a fisheye frame"""
    import slamhip
    for im in (real["vga"][0], real["gray"][0]):
        rk, rd = O.sift_detect(im if im.ndim == 3 else np.repeat(im[..., None], 3, 2))
        gk, gd = slamhip.siftDetectAndCompute(im, ctx=gpu_ctx)
        assert len(rk) > 50
        kp_equal(gk, rk)
        np.testing.assert_array_equal(gd, rd)
