"""GPU parity: the HIP library (through the C ABI) against the CPU oracle.

Bars (north_star / SURVEY 8c):
  FAST corners, ORB descriptors, kNN indices + distances, ratio-test matches: bit-exact;
  SIFT descriptors: |delta| <= 1 per element and >= 99.5 % elements exact (f32
      histogram accumulation order differs; the oracle follows OpenCV's order);
  BA: final cost relative difference <= 1e-6, RMSE difference <= 1e-4 px.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

import oracle_ffi as O
import slamhip
from slamhip import _lib as L
from slamhip import synthba

pytestmark = pytest.mark.gpu

SIFT_ABS_TOL = 1.0
SIFT_EXACT_FRAC = 0.995


@pytest.fixture(scope="module")
def vga():
    return slamhip.synth_frames(640, 480, 0, 4, seed=1234)


@pytest.fixture(scope="module")
def hd():
    return slamhip.synth_frames(1920, 1080, 0, 2, seed=1234)


def kp_equal(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        np.testing.assert_array_equal(a[f], b[f], err_msg=f)


@pytest.mark.parametrize("thr", [0, 10, 20, 40])
@pytest.mark.parametrize("nms", [True, False])
def test_fast_vga_bitexact(gpu_ctx, vga, thr, nms):
    for f in vga[:2]:
        ref = O.fast(f, thr, nms)
        got = slamhip.fastExtractor(f, thr, nms, ctx=gpu_ctx)
        kp_equal(got, ref)


def test_fast_1080p_bitexact(gpu_ctx, hd):
    for f in hd:
        ref = O.fast(f, 31, True)
        got = slamhip.fastExtractor(f, 31, True, ctx=gpu_ctx)
        assert len(ref) > 5000
        kp_equal(got, ref)


def test_fast_known_answers(gpu_ctx):
    img = np.zeros((32, 32), np.uint8)
    img[16, 16] = 255
    got = slamhip.fastExtractor(img, 10, True, ctx=gpu_ctx)
    assert len(got) == 1 and got[0]["x"] == 16 and got[0]["y"] == 16 and got[0]["response"] == 254
    assert len(slamhip.fastExtractor(np.full((40, 40), 77, np.uint8), 0, True, ctx=gpu_ctx)) == 0
    for shape in [(7, 7), (6, 50), (50, 6), (9, 65), (65, 9)]:
        rnd = np.random.default_rng(sum(shape)).integers(0, 256, shape, dtype=np.uint8)
        kp_equal(slamhip.fastExtractor(rnd, 5, True, ctx=gpu_ctx), O.fast(rnd, 5, True))
    # gray input and a strided (ROI) BGR view
    g = O.gray(slamhip.synth_frames(200, 120, 3, 1)[0])
    kp_equal(slamhip.fastExtractor(g, 12, True, ctx=gpu_ctx), O.fast(g, 12, True))
    big = slamhip.synth_frames(300, 200, 5, 1)[0]
    roi = big[10:170, 20:250]
    kp_equal(slamhip.fastExtractor(roi, 12, True, ctx=gpu_ctx), O.fast(np.ascontiguousarray(roi), 12, True))
    # a strided view above 256 KB: the rows go through the pinned staging copy
    big2 = slamhip.synth_frames(1920, 1080, 7, 1)[0]
    roi2 = big2[40:1040, 100:1800]
    kp_equal(slamhip.fastExtractor(roi2, 20, True, ctx=gpu_ctx), O.fast(np.ascontiguousarray(roi2), 20, True))


@pytest.mark.parametrize("ftype", [L.TYPE_7_12, L.TYPE_5_8])
@pytest.mark.parametrize("nms", [True, False])
def test_fast_types_bitexact(gpu_ctx, vga, hd, ftype, nms):
    """fastExtractor's `type` (fastExtractor.h:19-21; docs/FastExtractor.md:13-16):
    FAST_t<12> / FAST_t<8> with their cornerScore, bit-exact against the oracle
    on VGA and 1080p frames, noise (isolated peaks: TYPE_5_8 needs all 8
    neighbours, OpenCV's pair prefilter), odd sizes, gray input, the KAT"""
    img = np.zeros((32, 32), np.uint8)
    img[16, 16] = 255
    got = slamhip.fastExtractor(img, 10, nms, ftype, ctx=gpu_ctx)
    assert len(got) == 1 and got[0]["x"] == 16 and got[0]["y"] == 16
    total = 0
    frames = list(vga[:2]) + [hd[0]]
    frames += [np.random.default_rng(s).integers(0, 256, sh, dtype=np.uint8) for s, sh in
               ((1, (480, 640)), (2, (77, 131)), (3, (9, 65)))]
    for f in frames:
        for thr in (8, 20):
            ref = O.fast(f, thr, nms, ftype)
            kp_equal(slamhip.fastExtractor(f, thr, nms, ftype, ctx=gpu_ctx), ref)
            total += len(ref)
    assert total > 1000


def sift_close(got, ref):
    assert got.shape == ref.shape
    d = np.abs(got.astype(np.int32) - ref.astype(np.int32))
    assert d.max() <= SIFT_ABS_TOL, d.max()
    assert (d == 0).mean() >= SIFT_EXACT_FRAC, (d == 0).mean()
    return (d == 0).mean()


def test_sift_vga(gpu_ctx, vga):
    f = vga[0]
    kps = O.fast(f, 12, True)
    ref = O.sift(f, kps)
    kp_out, got = slamhip.extractDescriptor(f, kps, slamhip.SIFT_FLANN, ctx=gpu_ctx)
    kp_equal(kp_out, kps)
    # FAST keypoints (one angle, one size) take the gather kernel: every histogram
    # bin accumulates in the reference's sample order -> bit-exact
    np.testing.assert_array_equal(got, ref)


def test_sift_1080p_bitexact(gpu_ctx, hd):
    f = hd[0]
    kps = O.fast(f, 31, True)
    _, got = slamhip.extractDescriptor(f, kps, slamhip.SIFT_FLANN, ctx=gpu_ctx)
    np.testing.assert_array_equal(got, O.sift(f, kps))


def test_sift_1080p_position_plane_bitexact(gpu_ctx, hd, monkeypatch):
    """the opt-in gradient-map form of the band kernel (SLAMHIP_SIFT_POSPLANE=1:
    fract(obin) and the slot-position byte plane, read per launch), host-buffer
    and frame-batch paths"""
    monkeypatch.setenv("SLAMHIP_SIFT_POSPLANE", "1")
    f = hd[0]
    kps = O.fast(f, 31, True)
    _, got = slamhip.extractDescriptor(f, kps, slamhip.SIFT_FLANN, ctx=gpu_ctx)
    np.testing.assert_array_equal(got, O.sift(f, kps))
    from slamhip.batch import DeviceBatch
    import torch
    db = DeviceBatch(gpu_ctx)
    db.extract(torch.from_numpy(hd).cuda(), 31, slamhip.SIFT_FLANN)
    for i in range(2):
        np.testing.assert_array_equal(db.descriptors(i), O.sift(hd[i], O.fast(hd[i], 31, True)))


@pytest.mark.parametrize("kernel", ["band", "tab", "general", "cols", "colw"])
def test_sift_1080p_kernels_bitexact(hd, kernel):
    """every SIFT descriptor kernel (sift_desc_band, the default for FAST keypoints,
    the sift_desc_tab fallback, the general per-keypoint kernel and the
    one-keypoint-per-lane A/B kernel sift_desc_cols, the column-per-wave kernel
    sift_desc_colw) on the batch path and the
    host-buffer path, forced with slam_set_option"""
    from slamhip import _lib as L
    gpu_ctx = slamhip.Context(0)
    gpu_ctx.set_option(L.OPT_SIFT_KERNEL, {"band": L.SIFT_KERNEL_BAND, "tab": L.SIFT_KERNEL_TAB,
                                           "general": L.SIFT_KERNEL_GENERAL, "cols": L.SIFT_KERNEL_COLS,
                                           "colw": L.SIFT_KERNEL_COLW}[kernel])
    f = hd[1]
    kps = O.fast(f, 31, True)
    _, got = slamhip.extractDescriptor(f, kps, slamhip.SIFT_FLANN, ctx=gpu_ctx)
    ref = O.sift(f, kps)
    # the table kernels accumulate every bin in the reference's order (bit-exact);
    # the general kernel (any angle per keypoint) meets the SIFT bar
    same = np.testing.assert_array_equal if kernel != "general" else sift_close
    same(got, ref)
    forced = {"band": L.SIFT_KERNEL_BAND, "tab": L.SIFT_KERNEL_TAB, "general": L.SIFT_KERNEL_GENERAL,
              "cols": L.SIFT_KERNEL_COLS, "colw": L.SIFT_KERNEL_COLW}[kernel]
    assert slamhip.lib().slam_last_sift_kernel(gpu_ctx.handle) == forced
    from slamhip.batch import DeviceBatch
    import torch
    db = DeviceBatch(gpu_ctx)
    db.extract(torch.from_numpy(hd).cuda(), 31, slamhip.SIFT_FLANN)
    same(db.descriptors(1), ref)
    assert slamhip.lib().slam_last_sift_kernel(gpu_ctx.handle) == forced
    gpu_ctx.close()


def test_batch_fast_then_extract_reuses_fast(hd):
    """fillVideoFrameBatch's FAST pass (slam_batch_fast) followed by the batch
    extraction of the same device frames: the extraction takes the pass's FAST
    results (slam_batch_fast_reused) and its keypoints, descriptors and matches
    are the oracle's; a different threshold, other frames, or a FAST launch in
    between detect again"""
    from slamhip.batch import DeviceBatch
    import torch
    ctx = slamhip.Context(0)
    db = DeviceBatch(ctx)
    dev = torch.from_numpy(hd).cuda()
    kps = [O.fast(hd[i], 31, True) for i in range(len(hd))]
    counts = db.fast(dev, 31)
    assert list(counts) == [len(k) for k in kps]
    db.extract(dev, 31, slamhip.SIFT_FLANN)
    assert slamhip.lib().slam_batch_fast_reused(ctx.handle) == 0      # opt-in only (SLAM_OPT_FAST_REUSE)
    db.fast(dev, 31, reuse=True)
    db.extract(dev, 31, slamhip.SIFT_FLANN)
    assert slamhip.lib().slam_batch_fast_reused(ctx.handle) == 1
    for i in range(len(hd)):
        kp_equal(db.keypoints(i), kps[i])
        np.testing.assert_array_equal(db.descriptors(i), O.sift(hd[i], kps[i]))
    # the fused extract + match after a FAST pass: the same matches as the oracle
    q, nq = db.export_desc(0)
    q = q.clone()
    db.fast(dev, 31, reuse=True)
    _, mc = db.extract_match(dev, 31, slamhip.SIFT_FLANN, q, nq, 0.7)
    assert slamhip.lib().slam_batch_fast_reused(ctx.handle) == 1
    d0 = O.sift(hd[0], kps[0])
    for i in range(len(hd)):
        ri, rd = O.knn2(d0, O.sift(hd[i], kps[i]), O.NORM_L2)
        assert mc[i] == len(O.ratio(ri, rd, 0.7))
    # not taken: another threshold, a single-frame FAST in between, other frames
    db.fast(dev, 31, reuse=True)
    db.extract(dev, 30, slamhip.SIFT_FLANN)
    assert slamhip.lib().slam_batch_fast_reused(ctx.handle) == 0
    db.fast(dev, 31, reuse=True)
    slamhip.fastExtractor(hd[1], 31, True, ctx=ctx)
    db.extract(dev, 31, slamhip.SIFT_FLANN)
    assert slamhip.lib().slam_batch_fast_reused(ctx.handle) == 0
    kp_equal(db.keypoints(1), kps[1])
    db.fast(dev, 31, reuse=True)
    db.extract(dev[1:], 31, slamhip.SIFT_FLANN)
    assert slamhip.lib().slam_batch_fast_reused(ctx.handle) == 0
    np.testing.assert_array_equal(db.descriptors(0), O.sift(hd[1], kps[1]))
    ctx.close()


def test_batch_fast_refilled_buffer_not_reused(hd):
    """FAST reuse is opt-in.  A buffer refilled with other frames
    between slam_batch_fast and the extraction (same pointer, count and size)
    is detected again by default -- the extraction's keypoints and descriptors
    are the NEW frames' -- and the reuse flag stays 0"""
    from slamhip.batch import DeviceBatch
    import torch
    ctx = slamhip.Context(0)
    db = DeviceBatch(ctx)
    dev = torch.from_numpy(hd).cuda()
    db.fast(dev, 31)
    other = np.ascontiguousarray(hd[::-1])
    dev.copy_(torch.from_numpy(other).cuda())
    torch.cuda.synchronize()
    db.extract(dev, 31, slamhip.SIFT_FLANN)
    assert slamhip.lib().slam_batch_fast_reused(ctx.handle) == 0
    for i in range(len(other)):
        k = O.fast(other[i], 31, True)
        kp_equal(db.keypoints(i), k)
        np.testing.assert_array_equal(db.descriptors(i), O.sift(other[i], k))
    ctx.close()


@pytest.mark.parametrize("mode", ["all", "all4", "off", "auto"])
def test_sift_band_split_parts_bitexact(hd, mode):
    """sift_desc_band's part-walks (SLAM_OPT_SIFT_BAND_SPLIT): ALL runs every
    keypoint group as two part-walks (descriptor rows 0-1 over bands -1..1, rows
    2-3 over bands 1..3), ALL4 as four (row d over bands d - 1, d), merged through
    split_raw by the last to arrive; OFF none, AUTO (the default) the last partial
    round only -- each bit-exact to the oracle on the batch path, twice in a row
    (the arrival counters reset)"""
    from slamhip import _lib as L
    from slamhip.batch import DeviceBatch
    import torch
    ctx = slamhip.Context(0)
    ctx.set_option(L.OPT_SIFT_KERNEL, L.SIFT_KERNEL_BAND)
    ctx.set_option(L.OPT_SIFT_BAND_SPLIT, {"all": L.BAND_SPLIT_ALL, "all4": L.BAND_SPLIT_ALL4,
                                           "off": L.BAND_SPLIT_OFF, "auto": L.BAND_SPLIT_AUTO}[mode])
    db = DeviceBatch(ctx)
    dev = torch.from_numpy(hd).cuda()
    refs = [O.sift(hd[i], O.fast(hd[i], 31, True)) for i in range(len(hd))]
    for _ in range(2):
        db.extract(dev, 31, slamhip.SIFT_FLANN)
        for i in range(len(hd)):
            np.testing.assert_array_equal(db.descriptors(i), refs[i])
        assert slamhip.lib().slam_last_sift_kernel(ctx.handle) == L.SIFT_KERNEL_BAND
    ctx.close()


def test_sift_forced_kernels_rebuild_their_tables(hd):
    """one context switched between the forced column kernel, the band kernel and
    AUTO on the same frames: each run is bit-exact and reports the kernel that ran
    (the column tables of one geometry never leak into a rebuild that does not
    make them); AUTO runs sift_desc_band unless SLAMHIP_SIFT_COLW=1"""
    from slamhip.batch import DeviceBatch
    import torch
    ctx = slamhip.Context(0)
    f = hd[0]
    kps = O.fast(f, 31, True)
    ctx.set_option(L.OPT_SIFT_KERNEL, L.SIFT_KERNEL_COLW)
    _, got = slamhip.extractDescriptor(f, kps, slamhip.SIFT_FLANN, ctx=ctx)
    np.testing.assert_array_equal(got, O.sift(f, kps))
    assert slamhip.lib().slam_last_sift_kernel(ctx.handle) == L.SIFT_KERNEL_COLW
    auto = L.SIFT_KERNEL_COLW if os.environ.get("SLAMHIP_SIFT_COLW", "") == "1" else L.SIFT_KERNEL_BAND
    db = DeviceBatch(ctx)
    dev = torch.from_numpy(hd).cuda()
    for opt, want in ((L.SIFT_KERNEL_COLW, L.SIFT_KERNEL_COLW), (L.SIFT_KERNEL_BAND, L.SIFT_KERNEL_BAND),
                      (L.SIFT_KERNEL_COLW, L.SIFT_KERNEL_COLW), (L.SIFT_KERNEL_AUTO, auto)):
        ctx.set_option(L.OPT_SIFT_KERNEL, opt)
        db.extract(dev, 31, slamhip.SIFT_FLANN)
        assert slamhip.lib().slam_last_sift_kernel(ctx.handle) == want
        for i in range(len(hd)):
            np.testing.assert_array_equal(db.descriptors(i), O.sift(hd[i], O.fast(hd[i], 31, True)))
    ctx.close()


def test_forced_sift_kernel_refuses_instead_of_substituting(vga):
    """a forced table kernel whose schedule cannot apply (keypoints with
    different angles) fails loudly (SLAM_E_UNSUPPORTED); AUTO falls back to the
    general kernel for the same keypoints"""
    f = vga[0]
    kps = O.fast(f, 12, True)[:64].copy()
    kps["angle"] = np.linspace(0, 300, len(kps)).astype(np.float32)
    for forced in (L.SIFT_KERNEL_BAND, L.SIFT_KERNEL_TAB, L.SIFT_KERNEL_COLS, L.SIFT_KERNEL_COLW):
        ctx = slamhip.Context(0)
        ctx.set_option(L.OPT_SIFT_KERNEL, forced)
        with pytest.raises(L.SlamError) as e:
            slamhip.extractDescriptor(f, kps, slamhip.SIFT_FLANN, ctx=ctx)
        assert e.value.code == L.SLAM_E_UNSUPPORTED
        ctx.close()
    ctx = slamhip.Context(0)
    _, got = slamhip.extractDescriptor(f, kps, slamhip.SIFT_FLANN, ctx=ctx)
    assert slamhip.lib().slam_last_sift_kernel(ctx.handle) == L.SIFT_KERNEL_GENERAL
    sift_close(got, O.sift(f, kps))
    ctx.close()


def test_fast_sift_4k_batch_bitexact(gpu_ctx):
    """configs[4] sizing: 3840x2160 frames, ~20k FAST keypoints each, through the
    device batch path (FAST + SIFT band kernel), bit-exact against the oracle"""
    import torch
    from slamhip.batch import DeviceBatch
    fr = slamhip.synth_frames(3840, 2160, 0, 2, seed=1234)
    db = DeviceBatch(gpu_ctx)
    kp = db.extract(torch.from_numpy(fr).cuda(), 31, slamhip.SIFT_FLANN)
    for i in range(2):
        ref_k = O.fast(fr[i], 31, True)
        assert kp[i] == len(ref_k) and len(ref_k) > 10000
        kp_equal(db.keypoints(i), ref_k)
        np.testing.assert_array_equal(db.descriptors(i), O.sift(fr[i], ref_k))


def test_sift_gradient_border_reuse(hd, vga):
    """sift_blur_grad writes the gradient map's zero border once per buffer and
    geometry and later launches skip the border-only tiles: SIFT stays bit-exact
    on a repeat of the same geometry (border reused), on fewer frames (reused),
    after a switch to another geometry (rewritten) and back (rewritten again)"""
    import torch
    from slamhip.batch import DeviceBatch
    ctx = slamhip.Context(0)
    db = DeviceBatch(ctx)
    steps = [hd, hd, hd[:1], vga[:2], hd[1:]]
    for fr in steps:
        db.extract(torch.from_numpy(np.ascontiguousarray(fr)).cuda(), 31, slamhip.SIFT_FLANN)
        for i in range(len(fr)):
            ref_k = O.fast(fr[i], 31, True)
            kp_equal(db.keypoints(i), ref_k)
            np.testing.assert_array_equal(db.descriptors(i), O.sift(fr[i], ref_k))
    ctx.close()


def test_configs4_4k_match_bitexact(gpu_ctx):
    """configs[4] at size: two 3840x2160 frames at ~20k FAST keypoints, FAST +
    SIFT + the kNN (k = 2, ~20k x 20k: >= 20 packed-key splits of <= 1024 train
    rows, merged by knn_finish) + ratio test through the device batch, bit-exact
    against the oracle's brute-force L2 kNN and ratio test"""
    import torch
    from slamhip.batch import DeviceBatch
    fr = slamhip.synth_frames(3840, 2160, 40, 2, seed=1234)
    thr = 55                       # ~21k keypoints on these frames (bench.py bisects to ~20k)
    db = DeviceBatch(gpu_ctx)
    dev = torch.from_numpy(fr).cuda()
    db.extract(dev[:1], thr, slamhip.SIFT_FLANN)
    q, nq = db.export_desc(0)
    q = q.clone()
    O.oracle().orc_set_threads(16)
    kq = O.fast(fr[0], thr, True)
    dq = O.sift(fr[0], kq)
    k1 = O.fast(fr[1], thr, True)
    d1 = O.sift(fr[1], k1)
    assert nq == len(kq) and len(k1) > 20 * 1024 - 1024, (nq, len(k1))
    for rep in range(2):           # two-call path, then the fused one sized on the first
        kc, mc = db.extract_match(dev[1:], thr, slamhip.SIFT_FLANN, q, nq, 0.7)
        kp_equal(db.keypoints(0), k1)
        np.testing.assert_array_equal(db.descriptors(0), d1)
        ri, rd = O.knn2(dq, d1, O.NORM_L2)
        ref = O.ratio(ri, rd, 0.7)
        assert mc[0] == len(ref) > 1000
        np.testing.assert_array_equal(db.matches(0, nq), ref)


@pytest.mark.parametrize("angle", [0.0, 359.5, 1.0, 45.0, 90.0, 200.0])
def test_sift_uniform_angle_tables(gpu_ctx, vga, angle):
    """one shared angle: the band kernel where its band order holds (small
    rotations, generic orientation wrap) and the tab kernel otherwise -- both
    accumulate in the reference's order, so both are bit-exact"""
    f = vga[2]
    kps = O.fast(f, 12, True)
    kps["angle"] = np.float32(angle)
    ref = O.sift(f, kps)
    _, got = slamhip.extractDescriptor(f, kps, slamhip.SIFT_BF, ctx=gpu_ctx)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("size", [0.5, 0.6, 1.0, 2.0])
def test_sift_tiny_uniform_keypoints(gpu_ctx, vga, size):
    """keypoints so small that a band of the band schedule holds no
    sample (size < ~0.67 at angle 0 leaves bands -1 and 3 empty) must not reach
    the band kernel (it closes a band after the band's last chunk); AUTO then
    picks a kernel whose descriptors are the oracle's"""
    f = vga[2]
    kps = O.fast(f, 12, True)[:500].copy()
    kps["angle"] = np.float32(0.0)
    kps["size"] = np.float32(size)
    ref = O.sift(f, kps)
    _, got = slamhip.extractDescriptor(f, kps, slamhip.SIFT_BF, ctx=gpu_ctx)
    np.testing.assert_array_equal(got, ref)


def test_sift_arbitrary_angles_and_edges(gpu_ctx, vga):
    f = vga[1]
    kps = O.fast(f, 12, True)[:300].copy()
    rng = np.random.default_rng(3)
    kps["angle"] = rng.uniform(0, 360, len(kps)).astype(np.float32)
    kps["angle"][:10] = 0.0
    # keypoints hugging the border exercise the r/c window clipping
    kps["x"][10:20] = [0, 1, 2, 3, 639, 638, 637, 0, 639, 5]
    kps["y"][10:20] = [0, 1, 2, 479, 478, 0, 479, 240, 240, 1]
    ref = O.sift(f, kps)
    _, got = slamhip.extractDescriptor(f, kps, slamhip.SIFT_BF, ctx=gpu_ctx)
    sift_close(got, ref)


def test_sift_constant_image_zero(gpu_ctx):
    img = np.full((100, 120, 3), 90, np.uint8)
    kps = np.zeros(3, O.KP)
    kps["x"], kps["y"], kps["size"], kps["angle"] = [50, 10, 119], [50, 10, 99], 7, -1
    _, got = slamhip.extractDescriptor(img, kps, slamhip.SIFT_BF, ctx=gpu_ctx)
    assert np.all(got == 0)


def test_orb_bitexact(gpu_ctx, vga):
    for f in vga[:2]:
        kps = O.fast(f, 12, True)
        rk, rd = O.orb(f, kps)
        gk, gd = slamhip.extractDescriptor(f, kps, slamhip.ORB_BF, ctx=gpu_ctx)
        assert len(gk) < len(kps)           # border filter applied in place
        kp_equal(gk, rk)
        np.testing.assert_array_equal(gd, rd)


def test_orb_arbitrary_angles(gpu_ctx, vga):
    f = vga[2]
    kps = O.fast(f, 12, True)[:500].copy()
    kps["angle"] = np.random.default_rng(5).uniform(0, 360, len(kps)).astype(np.float32)
    rk, rd = O.orb(f, kps)
    gk, gd = slamhip.extractDescriptor(f, kps, slamhip.ORB_BF, ctx=gpu_ctx)
    kp_equal(gk, rk)
    np.testing.assert_array_equal(gd, rd)


def planted_sift(nq, nt, seed):
    rng = np.random.default_rng(seed)
    t = rng.integers(0, 40, (nt, 128)).astype(np.float32)
    q = rng.integers(0, 40, (nq, 128)).astype(np.float32)
    if nt >= 4:
        # exact duplicates -> equal distances: the lower trainIdx must win
        t[nt // 2] = t[1]
        t[nt - 1] = t[2]
        q[: min(nq, 8)] = t[1]
    return q, t


@pytest.mark.parametrize("nq,nt", [(1, 2), (7, 3), (64, 33), (300, 257), (513, 1000), (2048, 2100)])
def test_knn_sift_bitexact(gpu_ctx, nq, nt):
    q, t = planted_sift(nq, nt, nq + nt)
    ri, rd = O.knn2(q, t, O.NORM_L2)
    gi, gd = slamhip.knnMatch2(q, t, slamhip.SIFT_BF, ctx=gpu_ctx)
    np.testing.assert_array_equal(gi, ri)
    np.testing.assert_array_equal(gd, rd)


@pytest.mark.parametrize("nq,nt", [(1, 2), (7, 3), (300, 257), (513, 1000), (2048, 2100)])
def test_knn_sift_l1_bitexact(gpu_ctx, nq, nt):
    """NORM_L1 (the reference's CUDA-build SIFT_BF, featureMatchingCUDA.cpp:28):
    v_sad_u8 integer distances, planted ties (lower trainIdx wins), full 0..255
    range, and the ratio-test match list"""
    q, t = planted_sift(nq, nt, 3 * nq + nt)
    rng = np.random.default_rng(nq)
    q[8:] = rng.integers(0, 256, q[8:].shape)
    ri, rd = O.knn2(q, t, O.NORM_L1)
    gi, gd = slamhip.knnMatch2(q, t, slamhip.SIFT_BF, norm=slamhip._lib.NORM_L1, ctx=gpu_ctx)
    np.testing.assert_array_equal(gi, ri)
    np.testing.assert_array_equal(gd, rd)
    m = slamhip.matchFeatures(q, t, slamhip.SIFT_BF, 0.8, norm=slamhip._lib.NORM_L1, ctx=gpu_ctx)
    np.testing.assert_array_equal(m, O.ratio(ri, rd, 0.8))


def test_batch_l1_matches_oracle(gpu_ctx, hd):
    """the batch matcher with NORM_L1 (CUDA-build SIFT_BF) over 1080p frames:
    per-frame matches equal the oracle's L1 kNN + ratio"""
    import torch
    from slamhip import _lib as L
    from slamhip.batch import DeviceBatch
    dev = torch.from_numpy(hd).cuda()
    db = DeviceBatch(gpu_ctx)
    db.extract(dev[:1], 31, slamhip.SIFT_BF)
    q, nq = db.export_desc(0)
    q = q.clone()
    d0 = db.descriptors(0)
    kc, mc = db.extract_match(dev, 31, slamhip.SIFT_BF, q, nq, 0.7, norm=L.NORM_L1)
    for i in range(len(hd)):
        ri, rd = O.knn2(d0, db.descriptors(i), O.NORM_L1)
        ref = O.ratio(ri, rd, 0.7)
        assert mc[i] == len(ref)
        np.testing.assert_array_equal(db.matches(i, nq), ref)


def test_knn_sift_large_norms_sqrt_keys(gpu_ctx):
    # norms beyond 1024 switch the kernel to f32-sqrt keys; still bit-exact
    rng = np.random.default_rng(11)
    q = rng.integers(150, 256, (300, 128)).astype(np.float32)
    t = rng.integers(150, 256, (700, 128)).astype(np.float32)
    t[500] = t[10]
    q[0] = t[10]
    ri, rd = O.knn2(q, t, O.NORM_L2)
    gi, gd = slamhip.knnMatch2(q, t, slamhip.SIFT_BF, ctx=gpu_ctx)
    np.testing.assert_array_equal(gi, ri)
    np.testing.assert_array_equal(gd, rd)


@pytest.mark.parametrize("nq,nt", [(1, 2), (50, 40), (777, 1500)])
def test_knn_orb_bitexact(gpu_ctx, nq, nt):
    rng = np.random.default_rng(nq * 7 + nt)
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    if nt > 10:
        t[nt - 1] = t[3]
        q[0] = t[3]
    ri, rd = O.knn2(q, t, O.NORM_HAMMING)
    gi, gd = slamhip.knnMatch2(q, t, slamhip.ORB_BF, ctx=gpu_ctx)
    np.testing.assert_array_equal(gi, ri)
    np.testing.assert_array_equal(gd, rd)


def test_knn_edge_sizes(gpu_ctx):
    q, t = planted_sift(10, 1, 1)
    gi, gd = slamhip.knnMatch2(q, t, slamhip.SIFT_BF, ctx=gpu_ctx)
    assert np.all(gi[:, 0] == 0) and np.all(gi[:, 1] == -1)
    assert len(slamhip.matchFeatures(q, t, slamhip.SIFT_BF, 0.7, ctx=gpu_ctx)) == 0   # single train row: rejected
    assert len(slamhip.matchFeatures(q, t[:0], slamhip.SIFT_BF, 0.7, ctx=gpu_ctx)) == 0
    assert len(slamhip.matchFeatures(q[:0], t, slamhip.SIFT_BF, 0.7, ctx=gpu_ctx)) == 0


def test_match_frame_pair_sift(gpu_ctx, vga):
    f0, f1 = vga[0], vga[1]
    k0, k1 = O.fast(f0, 12, True), O.fast(f1, 12, True)
    d0 = O.sift(f0, k0)
    kout, m = slamhip.matchFramesPairFeatures(d0, f1, k1, slamhip.SIFT_FLANN, 0.7, ctx=gpu_ctx)
    # reference semantics on the GPU's own descriptors: exact
    _, d1 = slamhip.extractDescriptor(f1, k1, slamhip.SIFT_FLANN, ctx=gpu_ctx)
    ri, rd = O.knn2(d0, d1, O.NORM_L2)
    ref = O.ratio(ri, rd, 0.7)
    np.testing.assert_array_equal(m, ref)
    assert len(m) > 0.5 * len(k0)
    # and against the oracle's own descriptors: the same matches up to the SIFT tolerance
    ri2, rd2 = O.knn2(d0, O.sift(f1, k1), O.NORM_L2)
    ref2 = O.ratio(ri2, rd2, 0.7)
    common = len(np.intersect1d(ref2["queryIdx"] * 100000 + ref2["trainIdx"], m["queryIdx"] * 100000 + m["trainIdx"]))
    assert common >= 0.99 * len(ref2)


def test_match_frame_pair_orb(gpu_ctx, vga):
    f0, f1 = vga[0], vga[2]
    k0, d0 = O.orb(f0, O.fast(f0, 12, True))
    k1 = O.fast(f1, 12, True)
    rk1, rd1 = O.orb(f1, k1)
    kout, m = slamhip.matchFramesPairFeatures(d0, f1, k1, slamhip.ORB_BF, 0.7, ctx=gpu_ctx)
    kp_equal(kout, rk1)
    ri, rd = O.knn2(d0, rd1, O.NORM_HAMMING)
    np.testing.assert_array_equal(m, O.ratio(ri, rd, 0.7))


def test_batch_pipeline_sift(gpu_ctx):
    import torch
    from slamhip.batch import DeviceBatch, find_good_frame, Conditions
    frames = slamhip.synth_frames(640, 480, 0, 6, seed=99)
    db = DeviceBatch(gpu_ctx)
    dev = torch.from_numpy(frames).cuda()
    kc = db.extract(dev, 12, slamhip.SIFT_FLANN)
    for i in range(len(frames)):
        ref = O.fast(frames[i], 12, True)
        assert kc[i] == len(ref)
        kp_equal(db.keypoints(i), ref)
        np.testing.assert_array_equal(db.descriptors(i), O.sift(frames[i], ref))
    prev, nprev = db.export_desc(0)
    counts = db.match(prev, nprev, 0.7)
    d0 = db.descriptors(0)
    for i in range(len(frames)):
        ri, rd = O.knn2(d0, db.descriptors(i), O.NORM_L2)
        ref = O.ratio(ri, rd, 0.7)
        assert counts[i] == len(ref)
        np.testing.assert_array_equal(db.matches(i, nprev), ref)
    cond = Conditions(12, 1500, 6, 0, True, 500, slamhip.SIFT_FLANN, 0.7)
    good, kp, mc, inb = find_good_frame(db, dev, prev, nprev, cond)
    assert good == O.select_good(mc[inb], 500, 0, True)


@pytest.mark.parametrize("matcher", [slamhip.SIFT_FLANN, slamhip.ORB_BF])
def test_batch_extract_match_fused(gpu_ctx, hd, matcher):
    """slam_batch_extract_match (one host sync, kNN sized on the previous
    batch) gives the two-call results: counts, every match, and the oracle's
    kNN + ratio -- with a fitting estimate, and after a sparse batch whose
    estimate is too small for the packed-key splits (the match is redone)"""
    import torch
    from slamhip.batch import DeviceBatch
    dev = torch.from_numpy(hd).cuda()
    db = DeviceBatch(gpu_ctx)
    db.extract(dev[:1], 31, matcher)
    q, nq = db.export_desc(0)
    q = q.clone()
    kc_ref = db.extract(dev, 31, matcher)
    mc_ref = db.match(q, nq, 0.7)
    m_ref = [db.matches(i, nq) for i in range(len(hd))]
    d0 = db.descriptors(0)
    norm = O.NORM_HAMMING if matcher == slamhip.ORB_BF else O.NORM_L2
    for i in range(len(hd)):
        ri, rd = O.knn2(d0, db.descriptors(i), norm)
        np.testing.assert_array_equal(m_ref[i], O.ratio(ri, rd, 0.7))
    for pre in (31, 90):          # 90: a sparse batch first, so the estimate is too small
        db.extract(dev, pre, matcher)
        kc, mc = db.extract_match(dev, 31, matcher, q, nq, 0.7)
        np.testing.assert_array_equal(kc, kc_ref)
        np.testing.assert_array_equal(mc, mc_ref)
        for i in range(len(hd)):
            np.testing.assert_array_equal(db.matches(i, nq), m_ref[i])
            k1, m1 = db.result(i, nq)              # slam_batch_get_result: both, one sync
            np.testing.assert_array_equal(m1, m_ref[i])
            np.testing.assert_array_equal(k1, db.keypoints(i))
        # the two-halves form, with the next batch's extract + match run in between
        # (the bench's overlap): frame 1's result queued, then taken
        db.result_begin(1, nq)
        db.extract_match(dev, 31, matcher, q, nq, 0.7)
        k2, m2 = db.result_end()
        np.testing.assert_array_equal(m2, m_ref[1])
        np.testing.assert_array_equal(k2, db.keypoints(1))
    assert slamhip.lib().slam_batch_result_end(gpu_ctx.handle, None, 0, None, None, 0, None) == L.SLAM_E_INVALID_ARG
    # an empty query set: no matches, counts still reported
    kc, mc = db.extract_match(dev, 31, matcher, q, 0, 0.7)
    np.testing.assert_array_equal(kc, kc_ref)
    assert not mc.any()


@pytest.mark.parametrize("matcher", [slamhip.SIFT_FLANN, slamhip.ORB_BF])
def test_batch_async_rematch(gpu_ctx, hd, matcher):
    """the asynchronous halves (slam_batch_extract_async /
    _match_async / _finish) size the kNN on the previous batch's largest frame;
    after a sparse batch (threshold 120: a few hundred keypoints) every frame of
    the next (threshold 31: thousands, > 1024 rows, i.e. several packed-key
    splits for both key formats) outgrows that estimate, so the queued match is
    discarded and redone at the real size -- matches must equal the oracle's"""
    import torch
    from slamhip.batch import DeviceBatch
    dev = torch.from_numpy(hd).cuda()
    db = DeviceBatch(gpu_ctx)
    db.extract(dev[:1], 31, matcher)
    q, nq = db.export_desc(0)
    q = q.clone()
    d0 = db.descriptors(0)
    norm = O.NORM_HAMMING if matcher == slamhip.ORB_BF else O.NORM_L2
    kc_sparse = db.extract(dev, 120, matcher)
    assert kc_sparse.max() < 1024
    for c in (gpu_ctx,):
        slamhip.lib().slam_profile_enable(c.handle, 1)
    db.extract_async(dev, 31, matcher)
    db.match_async(q, nq, 0.7)
    kc, mc = db.finish()
    assert db.batch_counts().min() > 1024
    for i in range(len(hd)):
        ri, rd = O.knn2(d0, db.descriptors(i), norm)
        ref = O.ratio(ri, rd, 0.7)
        assert mc[i] == len(ref)
        np.testing.assert_array_equal(db.matches(i, nq), ref)
    ms, n = ctypes.c_double(0), ctypes.c_int(0)
    slamhip.lib().slam_profile_read(gpu_ctx.handle, 2, ctypes.byref(ms), ctypes.byref(n))
    slamhip.lib().slam_profile_enable(gpu_ctx.handle, 0)
    assert n.value == 2                   # the speculative kNN and the redone one


def test_batch_pipeline_orb(gpu_ctx):
    import torch
    from slamhip.batch import DeviceBatch
    frames = slamhip.synth_frames(640, 480, 10, 3, seed=5)
    db = DeviceBatch(gpu_ctx)
    kc = db.extract(torch.from_numpy(frames).cuda(), 12, slamhip.ORB_BF)
    for i in range(len(frames)):
        raw = O.fast(frames[i], 12, True)
        assert kc[i] == len(raw)          # batch filter sees FAST's count
        rk, rd = O.orb(frames[i], raw)
        kp_equal(db.keypoints(i), rk)     # descriptor-bearing keypoints: border filtered
        np.testing.assert_array_equal(db.descriptors(i), rd)
    # slam_batch_counts: every frame's raw and descriptor-bearing counts in one call
    raw = np.zeros(len(frames), np.int32)
    desc = np.zeros(len(frames), np.int32)
    assert slamhip.lib().slam_batch_counts(gpu_ctx.handle, L.ptr(raw), L.ptr(desc), len(frames)) == len(frames)
    np.testing.assert_array_equal(raw, kc)
    np.testing.assert_array_equal(desc, [db.keypoint_count(i) for i in range(len(frames))])
    np.testing.assert_array_equal(db.batch_counts(), desc)
    assert slamhip.lib().slam_batch_counts(gpu_ctx.handle, None, None, len(frames) - 1) == L.SLAM_E_CAPACITY
    prev, nprev = db.export_desc(0)
    counts = db.match(prev, nprev, 0.7)
    r0 = db.descriptors(0)
    for i in range(len(frames)):
        ri, rd = O.knn2(r0, db.descriptors(i), O.NORM_HAMMING)
        assert counts[i] == len(O.ratio(ri, rd, 0.7))


@pytest.mark.parametrize("loss,a", [(O.LOSS_NONE, 0.0), (O.LOSS_HUBER, 4.0), (O.LOSS_CAUCHY, 4.0)])
def test_ba_matches_oracle(gpu_ctx, loss, a):
    w = synthba.make_window(nframes=5, npoints=400, seed=3)
    rK, rE, rP, rs = O.ba(w["K4"], w["ext"], w["pts"], w["obs_frame"], w["obs_point"], w["obs_xy"], loss, a)
    K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
    gs = slamhip.bundle_adjust_arrays(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"], loss, a,
                                      ctx=gpu_ctx)
    assert gs.num_residuals == rs.num_residuals == 2 * len(w["obs_frame"])
    assert abs(gs.initial_cost - rs.initial_cost) <= 1e-9 * rs.initial_cost
    assert gs.final_cost < 0.5 * gs.initial_cost
    assert abs(gs.final_cost - rs.final_cost) <= 1e-6 * rs.final_cost + 1e-9
    rmse_g = np.sqrt(gs.final_cost / gs.num_residuals)
    rmse_r = np.sqrt(rs.final_cost / rs.num_residuals)
    assert abs(rmse_g - rmse_r) <= 1e-4
    # cost re-evaluated by the oracle at the GPU solution agrees with the GPU's
    c = O.ba_cost(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"], loss, a)
    assert abs(c - gs.final_cost) <= 1e-9 * c + 1e-12
    assert np.all(ext[0] == w["ext"][0])      # frame 0 held constant


@pytest.mark.parametrize("nf", [10, 14, 16, 20])
def test_ba_wide_windows(gpu_ctx, nf):
    # nc = 4 + 6 (nf - 1) = 58 / 82 / 94 / 118: 4-, 6-, 6-, 9-wide register tiles in the camera
    # reductions; one-wave Cholesky at 64 / 96 / 96, the LDS-tiled one at 118
    w = synthba.make_window(nframes=nf, npoints=300, seed=nf)
    rK, rE, rP, rs = O.ba(w["K4"], w["ext"], w["pts"], w["obs_frame"], w["obs_point"], w["obs_xy"],
                          O.LOSS_HUBER, 4.0)
    K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
    gs = slamhip.bundle_adjust_arrays(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"],
                                      O.LOSS_HUBER, 4.0, ctx=gpu_ctx)
    assert abs(gs.initial_cost - rs.initial_cost) <= 1e-9 * rs.initial_cost
    assert abs(gs.final_cost - rs.final_cost) <= 1e-6 * rs.final_cost + 1e-9
    assert gs.usable == 1


# ---------------- full SIFT detector (siftdet.hip vs oracle/siftdet.c) ----------------
@pytest.mark.parametrize("wh", [(640, 480), (333, 251), (1920, 1080)])
def test_sift_detect_matches_oracle(gpu_ctx, wh):
    w, h = wh
    f = slamhip.synth_frames(w, h, 2, 1, seed=77)[0]
    rk, rd = O.sift_detect(f)
    gk, gd = slamhip.siftDetectAndCompute(f, ctx=gpu_ctx)
    assert len(rk) > 100
    kp_equal(gk, rk)            # pyramid, extrema, refinement, orientation: bit-exact
    np.testing.assert_array_equal(gd, rd)     # gather-form descriptors: bit-exact


def test_sift_detect_golden_and_edges(gpu_ctx):
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "siftdet_160x120.npz"), allow_pickle=False)
    gk, gd = slamhip.siftDetectAndCompute(z["image"], ctx=gpu_ctx)
    np.testing.assert_array_equal(gk.view(np.uint8).reshape(len(gk), 28), z["expected_kps"])
    np.testing.assert_array_equal(gd, z["expected"])
    # flat and tiny frames: no keypoints; gray input == BGR of the same gray
    assert len(slamhip.siftDetectAndCompute(np.full((64, 64, 3), 90, np.uint8), ctx=gpu_ctx)[0]) == 0
    assert len(slamhip.siftDetectAndCompute(np.zeros((12, 12), np.uint8), ctx=gpu_ctx)[0]) == 0
    g = O.gray(slamhip.synth_frames(300, 200, 4, 1, seed=3)[0])
    gk, gd = slamhip.siftDetectAndCompute(g, ctx=gpu_ctx)
    rk, rd = O.sift_detect(np.repeat(g[..., None], 3, 2))
    kp_equal(gk, rk)
    np.testing.assert_array_equal(gd, rd)


@pytest.mark.parametrize("wh,n", [((640, 480), 3), ((1920, 1080), 2)])
def test_sift_detect_batch_matches_oracle(gpu_ctx, wh, n):
    """slam_sift_detect_batch on frames resident in HBM (one launch per pyramid
    stage for the whole batch): every frame's keypoints and descriptors
    bit-exact against the oracle's detectAndCompute of that frame"""
    import torch
    w, h = wh
    host = slamhip.synth_frames(w, h, 5, n, seed=91)
    out = slamhip.siftDetectAndComputeBatch(torch.from_numpy(host).cuda(), ctx=gpu_ctx)
    assert len(out) == n
    for f in range(n):
        rk, rd = O.sift_detect(host[f])
        assert len(rk) > 100
        gk, gd = out.host(f)
        kp_equal(gk, rk)
        np.testing.assert_array_equal(gd, rd)


def test_sift_detect_batch_gray_and_edges(gpu_ctx):
    import torch
    # gray frames, a flat frame between textured ones (no keypoints), a tight cap
    g = np.stack([O.gray(f) for f in slamhip.synth_frames(300, 200, 4, 2, seed=3)])
    frames = np.concatenate([g[:1], np.full((1, 200, 300), 90, np.uint8), g[1:]])
    out = slamhip.siftDetectAndComputeBatch(torch.from_numpy(frames).cuda(), ctx=gpu_ctx, cap=16)
    assert out.counts[1] == 0 and len(out.host(1)[0]) == 0
    for f in (0, 2):
        rk, rd = O.sift_detect(np.repeat(frames[f][..., None], 3, 2))
        gk, gd = out.host(f)
        kp_equal(gk, rk)
        np.testing.assert_array_equal(gd, rd)
    assert len(slamhip.siftDetectAndComputeBatch(torch.zeros((0, 8, 8), dtype=torch.uint8, device="cuda"),
                                                 ctx=gpu_ctx)) == 0



# ---------------- two-view triangulation (geom.hip vs oracle/geom.c) ----------------
def test_reconstruct_bitexact(gpu_ctx):
    from test_oracle import two_view_scene
    for n, seed, noise in [(10000, 5, 0.5), (1, 6, 0.0), (777, 7, 2.0)]:
        K, R1, t1, R2, t2, p1, p2, X = two_view_scene(n, seed, noise)
        ref = O.reconstruct(K, R1, t1, R2, t2, p1, p2)
        got = slamhip.reconstruct(K, R1, t1, R2, t2, p1, p2, ctx=gpu_ctx)
        np.testing.assert_array_equal(got, ref)
    # zero baseline (rank-deficient systems): same bits, NaN / inf included
    K, R1, t1, R2, t2, p1, p2, X = two_view_scene(64, 8)
    np.testing.assert_array_equal(slamhip.reconstruct(K, R1, t1, R1, t1, p1, p1, ctx=gpu_ctx),
                                  O.reconstruct(K, R1, t1, R1, t1, p1, p1))
    assert len(slamhip.reconstruct(K, R1, t1, R2, t2, np.zeros((0, 2)), np.zeros((0, 2)), ctx=gpu_ctx)) == 0



# ---------------- relative pose (essential.hip vs oracle/essential.c) ----------------
@pytest.mark.parametrize("n,seed,outliers,ransac", [(1500, 1, 0.3, True), (4000, 2, 0.5, True), (600, 3, 0.0, False),
                                                    (5, 4, 0.0, True), (40, 5, 0.2, True)])
def test_estimate_transformation_bitexact(gpu_ctx, n, seed, outliers, ransac):
    from test_oracle import relpose_scene
    K, R, t, p1, p2, out = relpose_scene(n, seed, outliers=outliers)
    ok, Rr, tr, cr, rr, passed = O.estimate_transformation(p1, p2, K, ransac, 0.999, 5.0, 200.0)
    gok, Rg, tg, cg, rg = slamhip.estimateTransformation(p1, p2, K, ransac, 0.999, 5.0, 200.0, ctx=gpu_ctx)
    assert gok == ok
    np.testing.assert_array_equal(Rg, Rr)
    np.testing.assert_array_equal(tg, tr)
    np.testing.assert_array_equal(cg, cr)
    np.testing.assert_array_equal(rg, rr)
    assert int(cg.sum()) == passed


# ---------------- solvePnPRansac (pnp.hip vs oracle/pnp.c) ----------------
@pytest.mark.parametrize("n,seed,outliers,kw", [(1500, 1, 0.3, {}), (4000, 2, 0.5, {}), (300, 3, 0.0, {}),
                                                (5, 4, 0.0, {}), (40, 5, 0.2, {}), (9, 6, 0.0, {}),
                                                (2000, 7, 0.6, {"iterationsCount": 500, "reprojectionError": 3.0,
                                                                "confidence": 0.999})])
def test_solve_pnp_ransac_bitexact(gpu_ctx, n, seed, outliers, kw):
    from test_oracle import pnp_scene
    K, rv, t, X, uv, out = pnp_scene(n, seed, outliers=outliers)
    st, r, tt, mask, ni = O.solve_pnp_ransac(X, uv, K, kw.get("iterationsCount", 100),
                                             kw.get("reprojectionError", 8.0), kw.get("confidence", 0.99))
    ok, rg, tg, inl = slamhip.solvePnPRansac(X, uv, K, None, ctx=gpu_ctx, **kw)
    assert ok == (st == 1)
    np.testing.assert_array_equal(rg.ravel(), r)
    np.testing.assert_array_equal(tg.ravel(), tt)
    np.testing.assert_array_equal(inl.ravel(), np.flatnonzero(mask))


@pytest.mark.parametrize("n,seed,outliers", [(1500, 1, 0.3), (4000, 2, 0.5), (300, 3, 0.0), (40, 5, 0.2),
                                             (1800, 8, 0.03)])
def test_solve_pnp_ransac_pairwise_sums(n, seed, outliers):
    """SLAM_PNP_SUMS_PAIRWISE: the refinement's J'J / J'e / |e|^2 as per-thread
    partials and a fixed tree instead of the oracle's sequential order -- the
    same inlier mask, rvec / tvec within 1e-9 (relative to |t| for tvec), and
    the same value on every run"""
    from slamhip import _lib as L
    from test_oracle import pnp_scene
    ctx = slamhip.Context(0)
    ctx.set_option(L.OPT_PNP_SUMS, L.PNP_SUMS_PAIRWISE)
    K, rv, t, X, uv, out = pnp_scene(n, seed, outliers=outliers)
    st, r, tt, mask, ni = O.solve_pnp_ransac(X, uv, K, 100, 8.0, 0.99)
    ok, rg, tg, inl = slamhip.solvePnPRansac(X, uv, K, None, ctx=ctx)
    assert ok == (st == 1)
    np.testing.assert_array_equal(inl.ravel(), np.flatnonzero(mask))
    assert np.abs(rg.ravel() - r).max() <= 1e-9, (rg.ravel(), r)
    assert np.abs(tg.ravel() - tt).max() <= 1e-9 * max(1.0, np.linalg.norm(tt)), (tg.ravel(), tt)
    ok2, rg2, tg2, _ = slamhip.solvePnPRansac(X, uv, K, None, ctx=ctx)
    np.testing.assert_array_equal(rg2, rg)
    np.testing.assert_array_equal(tg2, tg)
    ctx.close()


def test_solve_pnp_ransac_edges(gpu_ctx):
    from test_oracle import pnp_scene
    K, rv, t, X, uv, out = pnp_scene(40, 11, outliers=0.0)
    with pytest.raises(slamhip.SlamError):
        slamhip.solvePnPRansac(X[:4], uv[:4], K, ctx=gpu_ctx)      # P3P (npoints == 4) not restated
    with pytest.raises(slamhip.SlamError):
        slamhip.solvePnPRansac(X[:3], uv[:3], K, ctx=gpu_ctx)
    # pure noise: same verdict, pose and mask as the oracle (often "no model")
    rng = np.random.default_rng(12)
    Xn = rng.uniform(-3, 3, (200, 3)).astype(np.float32) + [0, 0, 8]
    un = rng.uniform(0, 1900, (200, 2)).astype(np.float32)
    st, r, tt, mask, ni = O.solve_pnp_ransac(Xn, un, K)
    ok, rg, tg, inl = slamhip.solvePnPRansac(Xn, un, K, ctx=gpu_ctx)
    assert ok == (st == 1)
    np.testing.assert_array_equal(rg.ravel(), r)
    np.testing.assert_array_equal(tg.ravel(), tt)
    # degenerate: all object points coplanar and collinear in the image
    Xd = np.zeros((30, 3), np.float32)
    Xd[:, 0] = np.linspace(-1, 1, 30)
    Xd[:, 2] = 5
    ud = (Xd[:, :2] / Xd[:, 2:] * [K[0, 0], K[1, 1]] + [K[0, 2], K[1, 2]]).astype(np.float32)
    st, r, tt, mask, ni = O.solve_pnp_ransac(Xd, ud, K)
    ok, rg, tg, inl = slamhip.solvePnPRansac(Xd, ud, K, ctx=gpu_ctx)
    assert ok == (st == 1)
    np.testing.assert_array_equal(rg.ravel(), r)
    np.testing.assert_array_equal(tg.ravel(), tt)


# ---------------- configured windows, configs[2]-[4] (BAMaxFramesCnt 8 / 16) ----------------
def _ba_vs_oracle(ctx, w, loss, a):
    rK, rE, rP, rs = O.ba(w["K4"], w["ext"], w["pts"], w["obs_frame"], w["obs_point"], w["obs_xy"], loss, a)
    K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
    gs = slamhip.bundle_adjust_arrays(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"], loss, a, ctx=ctx)
    assert gs.num_residuals == rs.num_residuals == 2 * len(w["obs_frame"])
    assert abs(gs.initial_cost - rs.initial_cost) <= 1e-9 * rs.initial_cost
    assert abs(gs.final_cost - rs.final_cost) <= 1e-6 * rs.final_cost + 1e-9
    rmse_g = np.sqrt(gs.final_cost / gs.num_residuals)
    rmse_r = np.sqrt(rs.final_cost / rs.num_residuals)
    assert abs(rmse_g - rmse_r) <= 1e-4, (rmse_g, rmse_r)
    assert gs.usable == rs.usable and gs.iterations == rs.iterations
    assert np.all(ext[0] == w["ext"][0])
    # the GPU's solution re-evaluated by the oracle has the GPU's final cost
    c = O.ba_cost(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"], loss, a)
    assert abs(c - gs.final_cost) <= 1e-9 * c + 1e-12
    return gs, rs


@pytest.mark.parametrize("loss,a", [(O.LOSS_NONE, 0.0), (O.LOSS_HUBER, 4.0), (O.LOSS_CAUCHY, 4.0),
                                    (O.LOSS_ARCTAN, 4.0)])
def test_ba_bench_window_w8_losses(gpu_ctx, loss, a):
    """bench.py's BA window (BAMaxFramesCnt = 8, 10k points, ~21.6k observations,
    1080p samsung-hv intrinsics) with the getLossFunction losses
    (bundleAdjustment.cpp:131-151): cost 1e-6 rel, RMSE within 1e-4 px"""
    w = synthba.make_window(nframes=8, npoints=10000, seed=7)
    assert len(w["obs_frame"]) > 20000
    gs, rs = _ba_vs_oracle(gpu_ctx, w, loss, a)
    assert gs.final_cost < 0.5 * gs.initial_cost


@pytest.mark.parametrize("nf,npts,seed", [(5, 400, 3), (8, 2000, 7)])
def test_ba_tukey_converging_windows(gpu_ctx, nf, npts, seed):
    """Tukey where LM converges: the oracle's bars"""
    w = synthba.make_window(nframes=nf, npoints=npts, seed=seed)
    _ba_vs_oracle(gpu_ctx, w, O.LOSS_TUKEY, 4.0)


def test_ba_tukey_bench_window(gpu_ctx):
    """Tukey on the bench window does not converge in 50 iterations and its LM
    path is chaotic: the oracle's OWN final cost moves by several percent when
    only the order of the residual blocks changes (a summation order Ceres does
    not fix either: BAThreadsCnt threads).  Bars: the first iterations agree
    to 1e-9 (before rounding differences grow), then tests/ba_envelope.py's:
    the GPU's 50-iteration cost inside the oracle's raw reordering envelope
    [min, max] (16 orders, 64 if outside the 16), two-sided.  The converging
    Tukey windows above hold the strict 1e-6 / 1e-4 px bars."""
    from ba_envelope import window_vs_oracle
    w = synthba.make_window(nframes=8, npoints=10000, seed=7)
    of, op, oxy = w["obs_frame"], w["obs_point"], w["obs_xy"]
    for it in (1, 2, 3):
        rs = O.ba(w["K4"], w["ext"], w["pts"], of, op, oxy, O.LOSS_TUKEY, 4.0, max_iters=it)[3]
        K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
        gs = slamhip.bundle_adjust_arrays(K4, ext, pts, of, op, oxy, O.LOSS_TUKEY, 4.0, max_iters=it, ctx=gpu_ctx)
        assert abs(gs.final_cost - rs.final_cost) <= 1e-9 * rs.final_cost
        assert gs.successful_steps == rs.successful_steps
    K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
    gs = slamhip.bundle_adjust_arrays(K4, ext, pts, of, op, oxy, O.LOSS_TUKEY, 4.0, ctx=gpu_ctx)
    io = {"in": dict(w, loss=O.LOSS_TUKEY, loss_param=4.0), "out": (K4, ext, pts)}
    res = window_vs_oracle(io, gs, threads=16)
    assert res["ok"], {k: res.get(k) for k in ("final_cost_rel_diff", "rmse_abs_diff_px", "envelope")}
    assert gs.final_cost < 0.85 * gs.initial_cost and gs.usable == 1


def _b210_windows():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_ba_b210 import load
    g = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    return {m: load(os.path.join(g, f"ba_b210_{m}.npz")) for m in ("sift", "orb")}


@pytest.mark.parametrize("matcher,wi", [(m, i) for m in ("sift", "orb") for i in range(3)])
def test_ba_b210_searched_frame_windows(gpu_ctx, matcher, wi):
    """The BA windows slamMain builds at framesBatchSize 210 (mainCycle.cpp:193-210:
    non-overlapping BAMaxFramesCnt-8 windows over the frames the candidate
    search selected, Huber 4), dumped from bench.py's pipeline_b210 legs
    (tests/golden/make_ba_b210.py): SIFT (configs[3] at N = 1) and ORB
    (configs[2]).  Most of their points are born-once tracks and every window
    runs into the 50-iteration cap.  Each is solved through slam_ba and checked
    by tests/ba_envelope.py against oracle/ba.c on the same inputs: 1e-6 / 1e-4
    px, else inside the oracle's raw reordering envelope (16, then 64 orders).
    The round-4 bench's red SIFT window is (sift, 1)."""
    from ba_envelope import window_vs_oracle
    w = _b210_windows()[matcher][wi]
    K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
    gs = slamhip.bundle_adjust_arrays(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"], w["loss"],
                                      w["loss_param"], ctx=gpu_ctx)
    assert gs.usable == 1 and gs.final_cost < gs.initial_cost
    res = window_vs_oracle({"in": w, "out": (K4, ext, pts)}, gs, threads=16)
    print(matcher, wi, {k: res.get(k) for k in ("tier", "north_star_ok", "final_cost_rel_diff", "rmse_abs_diff_px",
                                                 "envelope")})
    assert res["ok"], {k: res.get(k) for k in ("final_cost_rel_diff", "rmse_abs_diff_px", "envelope")}


@pytest.mark.parametrize("matcher,wi", [(m, i) for m in ("sift", "orb") for i in range(3)])
def test_ba_b210_lm_path_per_iteration(gpu_ctx, matcher, wi):
    """the LM path, not only its end.  For each searched-frame
    fixture window the GPU solve capped at k = 1, 2, 3, 5, 10 iterations
    (slam_ba's max_iters) must lie inside the oracle's envelope at the same k
    (tests/ba_envelope.py lm_path_check: 16 observation orders under each of the
    oracle's two factorisations of the reduced camera system -- its LL'
    restatement and Eigen SimplicialLDLT's arithmetic, the reference's solver --
    then 64 where a k falls outside).  A formula-level difference shows as a
    one-sided offset from an early k (round 5 found the Schur accumulation order
    this way: 8 widths outside at k = 1); a different but valid summation order
    stays inside.  The endpoint bar (test_ba_b210_searched_frame_windows) is
    unchanged."""
    from ba_envelope import lm_path_check
    w = _b210_windows()[matcher][wi]
    ks = [1, 2, 3, 5, 10]
    g = []
    for k in ks:
        s = slamhip.bundle_adjust_arrays(w["K4"].copy(), w["ext"].copy(), w["pts"].copy(), w["obs_frame"],
                                         w["obs_point"], w["obs_xy"], w["loss"], w["loss_param"], max_iters=k,
                                         ctx=gpu_ctx)
        assert s.usable == 1
        g.append(s.final_cost)
    res = lm_path_check(w, g, ks, threads=16)
    for r in res["rows"]:
        print(matcher, wi, r)
    assert res["ok"], res["rows"]


def test_ba_window_w16_4k_huber(gpu_ctx):
    """configs[4]: BAMaxFramesCnt = 16, samsung-hv-4k intrinsics, Huber, >= 10k points"""
    w = synthba.make_window(nframes=16, npoints=12000, seed=16, width=3840, height=2160, K4=synthba.K_4K)
    gs, rs = _ba_vs_oracle(gpu_ctx, w, O.LOSS_HUBER, 4.0)
    assert gs.usable == 1


# ---------------- sharded scan and large batches (configs[3]) ----------------
def _oracle_desc(f, thr, matcher=slamhip.SIFT_FLANN):
    k = O.fast(f, thr, True)
    return O.orb(f, k)[1] if matcher == slamhip.ORB_BF else O.sift(f, k)


def _oracle_search(frames, prev_desc, thr, required_kp, required_mc, ratio=0.7, matcher=slamhip.SIFT_FLANN):
    kc, mc, dc, ds = [], [], [], []
    norm = O.NORM_HAMMING if matcher == slamhip.ORB_BF else O.NORM_L2
    for f in frames:
        k = O.fast(f, thr, True)
        d = O.orb(f, k)[1] if matcher == slamhip.ORB_BF else O.sift(f, k)
        idx, dist = O.knn2(prev_desc, d, norm)
        kc.append(len(k)); dc.append(len(d)); ds.append(d)
        mc.append(len(O.ratio(idx, dist, ratio)))
    kc, mc = np.array(kc), np.array(mc)
    in_batch = np.nonzero(kc >= required_kp)[0]
    good = O.select_good(mc[in_batch], required_mc, 0, True) if len(in_batch) else L.EMPTY_BATCH
    return good, kc, mc, np.array(dc), in_batch, ds


def test_sharded_search_nccl_world1(gpu_ctx):
    """ShardedScan.search + advance on the GPU with an RCCL process group of one
    rank: the broadcast / all-gather path, the event that orders only the kNN
    behind the broadcast, and the winner hand-over, checked against the oracle
    over two consecutive searches at 1080p"""
    import socket
    import torch
    import torch.distributed as dist
    from slamhip.batch import Conditions, ShardedScan
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        host = slamhip.synth_frames(1920, 1080, 300, 9, seed=21)
        frames = torch.from_numpy(host).cuda()
        scan = ShardedScan(0, 1, ctx=gpu_ctx)
        assert scan._collective()
        scan.db.extract(frames[:1], 60, slamhip.SIFT_FLANN)
        prev = torch.zeros(slamhip.lib().slam_batch_desc_bytes(slamhip.SIFT_FLANN, 64 * 1024), dtype=torch.uint8,
                           device="cuda")
        _, nprev = scan.db.export_desc(0, prev)
        owner = 0
        cond = Conditions(featureExtractingThreshold=60, requiredExtractedPointsCount=1000,
                          requiredMatchedPointsCount=150, matcherType=slamhip.SIFT_FLANN, knnMatcherDistance=0.7)
        ref_prev = O.sift(host[0], O.fast(host[0], 60, True))
        pending = None      # winner_begin / winner_end as the bench runs them: taken after the next search
        for lo, hi in [(1, 5), (5, 9)]:
            good, kp_all, mc_all, in_batch, dc_all = scan.search(frames[lo:hi], prev, nprev, owner, cond)
            if pending is not None:
                dk, dm = scan.winner_end(pending[0])
                np.testing.assert_array_equal(dk, pending[1])
                np.testing.assert_array_equal(dm, pending[2])
                pending = None
            rg, rkc, rmc, rdc, rin, rds = _oracle_search(host[lo:hi], ref_prev, 60, 1000, 150)
            np.testing.assert_array_equal(kp_all, rkc)
            np.testing.assert_array_equal(mc_all, rmc)
            np.testing.assert_array_equal(dc_all, rdc)
            assert good == rg
            wk, wm = scan.winner(good, in_batch, dc_all, mc_all, nprev)
            if good >= 0:
                gi = int(rin[good])
                kp_equal(wk, O.fast(host[lo + gi], 60, True))
                ri, rd = O.knn2(ref_prev, rds[gi], O.NORM_L2)
                np.testing.assert_array_equal(wm, O.ratio(ri, rd, 0.7))
                pending = (scan.winner_begin(good, in_batch, dc_all, mc_all, nprev), wk.copy(), wm.copy())
            owner, nprev = scan.advance(good, in_batch, dc_all, prev, owner, nprev)
            if good >= 0:
                ref_prev = rds[int(rin[good])]
                assert nprev == len(ref_prev)
        if pending is not None:
            dk, dm = scan.winner_end(pending[0])
            np.testing.assert_array_equal(dk, pending[1])
            np.testing.assert_array_equal(dm, pending[2])
        assert rg >= 0
    finally:
        dist.destroy_process_group()


def test_batch_1080p_64_candidates(gpu_ctx):
    """one search over 64 candidate 1080p frames (configs[3]'s framesBatchSize
    210 over 8 GPUs is ~27 per rank): per-candidate keypoint counts, match
    counts and the selection against the oracle"""
    import torch
    from slamhip.batch import Conditions, DeviceBatch, find_good_frame
    host = slamhip.synth_frames(1920, 1080, 200, 65, seed=77)
    dev = torch.from_numpy(host).cuda()
    db = DeviceBatch(gpu_ctx)
    db.extract(dev[:1], 70, slamhip.SIFT_FLANN)
    q, nq = db.export_desc(0)
    q = q.clone()
    cond = Conditions(70, 1500, 64, 0, True, 200, slamhip.SIFT_FLANN, 0.7)
    O.oracle().orc_set_threads(16)
    ref_prev = O.sift(host[0], O.fast(host[0], 70, True))
    rg, rkc, rmc, rdc, rin, _ = _oracle_search(host[1:], ref_prev, 70, 1500, 200)
    for rep in range(2):          # first call: two-call path; second: fused, sized on the first
        good, kc, mc, inb = find_good_frame(db, dev[1:], q, nq, cond)
        np.testing.assert_array_equal(kc, rkc)
        np.testing.assert_array_equal(mc, rmc)
        np.testing.assert_array_equal(db.batch_counts(), rdc)
        assert good == rg and list(inb) == list(rin)
    assert rg >= 0 and len(rin) > 32


def _gloo_gpu_rank(rank, world, port, outdir, host, batches, thr, req_kp, req_mc, pipelined=False):
    """one rank of a world-2 ShardedScan on ONE GPU over gloo: the owner's
    descriptor export must land before the next search's broadcast reads it,
    and the winner travels device to device (slam_batch_result_dev + broadcast)"""
    import json
    import os
    import torch
    import torch.distributed as dist
    from slamhip.batch import Conditions, PipelinedScan, ShardedScan
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = slamhip.Context(0)
        first = ShardedScan(rank, world, ctx=ctx, device="cuda")
        scan = PipelinedScan(rank, world, 0, overlap=pipelined) if pipelined else first
        frames = torch.from_numpy(host).cuda()
        prev = torch.zeros(slamhip.lib().slam_batch_desc_bytes(slamhip.SIFT_FLANN, 64 * 1024), dtype=torch.uint8,
                           device="cuda")
        nprev = 0
        if rank == 0:
            first.db.extract(frames[:1], thr, slamhip.SIFT_FLANN)
            _, nprev = first.db.export_desc(0, prev)
        t = torch.tensor([nprev], dtype=torch.int32)
        dist.broadcast(t, src=0)
        nprev, owner = int(t.item()), 0
        cond = Conditions(featureExtractingThreshold=thr, requiredExtractedPointsCount=req_kp,
                          requiredMatchedPointsCount=req_mc, matcherType=slamhip.SIFT_FLANN, knnMatcherDistance=0.7)
        out = []
        locs = []
        for lo, hi in batches:
            idx = torch.from_numpy(first.shard(hi - lo)).cuda()
            locs.append(frames[lo:hi].index_select(0, idx).contiguous())
        for b, (lo, hi) in enumerate(batches):
            local = locs[b]
            kw = {"next_frames": locs[b + 1] if b + 1 < len(batches) else None} if pipelined else {}
            good, kp_all, mc_all, in_batch, dc_all = scan.search(local, prev, nprev, owner, cond,
                                                                 pad_to=(hi - lo + world - 1) // world, **kw)
            tok = scan.winner_begin(good, in_batch, dc_all, mc_all, nprev)
            owner, nprev = scan.advance(good, in_batch, dc_all, prev, owner, nprev)
            wk, wm = scan.winner_end(tok) if good >= 0 else (None, None)
            out.append({"good": int(good), "kp": kp_all.tolist(), "mc": mc_all.tolist(), "dc": dc_all.tolist(),
                        "owner": owner, "nprev": nprev, "token": "pipelined" if pipelined else tok[0],
                        "wk": None if wk is None else wk.tobytes().hex(),
                        "wm": None if wm is None else wm.tobytes().hex()})
        # the last hand-over, broadcast as the next search would: every rank's query bytes
        dist.broadcast(prev[:nprev * 132], src=owner)
        torch.cuda.synchronize()
        out.append({"query": prev[:nprev * 128].cpu().numpy().tobytes().hex()})
        json.dump(out, open(os.path.join(outdir, f"g{rank}.json"), "w"))
        if pipelined:
            scan.close()
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pipelined", [False, "knn", "desc_start"])
def test_sharded_search_gloo_world2_one_gpu(pipelined):
    """ShardedScan (and PipelinedScan: each search's extraction queued on the
    other context before the previous search is taken) at world 2 on one GPU
    (gloo carries the device tensors):
    per-candidate counts, selection and winners against the oracle over three
    ragged searches whose winners alternate owners, so every hand-over's export
    is broadcast to the other rank (the export is ordered before the
    broadcast), and the winner's keypoints / matches travel device to device"""
    import json
    import socket
    import tempfile
    import torch.multiprocessing as mp
    host = slamhip.synth_frames(640, 480, 0, 16, seed=1234)
    thr, req_kp, req_mc = 12, 1000, 100
    batches = [(1, 7), (7, 11), (11, 16)]        # 6 / 4 / 5 candidates: 3+3, 2+2, 3+2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gloo_gpu_rank, args=(2, port, d, host, batches, thr, req_kp, req_mc, pipelined), nprocs=2,
                 join=True)
        res = [json.load(open(f"{d}/g{r}.json")) for r in range(2)]
    ref_prev = O.sift(host[0], O.fast(host[0], thr, True))
    owners = []
    for (lo, hi), r0, r1 in zip(batches, res[0], res[1]):
        rg, rkc, rmc, rdc, rin, rds = _oracle_search(host[lo:hi], ref_prev, thr, req_kp, req_mc)
        for r in (r0, r1):
            assert r["kp"] == rkc.tolist() and r["mc"] == rmc.tolist() and r["dc"] == rdc.tolist()
            assert r["good"] == rg
        if rg >= 0:
            gi = int(rin[rg])
            assert r0["token"] == r1["token"] == ("pipelined" if pipelined else "device")
            ri, rd = O.knn2(ref_prev, rds[gi], O.NORM_L2)
            wk = O.fast(host[lo + gi], thr, True)
            for r in (r0, r1):
                assert r["wk"] == wk.tobytes().hex() and r["wm"] == O.ratio(ri, rd, 0.7).tobytes().hex()
            owners.append(gi % 2)
            ref_prev = rds[gi]
    assert set(owners) == {0, 1}, owners
    q = ref_prev.astype(np.uint8).tobytes().hex()
    assert res[0][-1]["query"] == res[1][-1]["query"] == q


def test_order_after_stage_contract():
    """slam_order_after_stage: INVALID_ARG before the context's first extraction
    and for an unknown stage; after an extraction both stages order a stream
    without a host wait, and work queued behind them sees the finished batch"""
    import torch
    from slamhip.batch import DeviceBatch
    ctx = slamhip.Context(0)
    try:
        lib = slamhip.lib()
        waiter = torch.cuda.Stream()
        ws = ctypes.c_void_p(waiter.cuda_stream)
        assert lib.slam_order_after_stage(ctx.handle, ws, L.STAGE_DESC_START) == L.SLAM_E_INVALID_ARG
        host = slamhip.synth_frames(640, 480, 0, 2, seed=3)
        db = DeviceBatch(ctx)
        db.extract(torch.from_numpy(host).cuda(), 12, slamhip.SIFT_FLANN)
        assert lib.slam_order_after_stage(ctx.handle, ws, 2) == L.SLAM_E_INVALID_ARG
        assert lib.slam_order_after_stage(ctx.handle, ws, -1) == L.SLAM_E_INVALID_ARG
        for stage in (L.STAGE_DESC_START, L.STAGE_DESC_END):
            assert lib.slam_order_after_stage(ctx.handle, ws, stage) == 0
        waiter.synchronize()
        np.testing.assert_array_equal(db.descriptors(1), O.sift(host[1], O.fast(host[1], 12, True)))
    finally:
        ctx.close()


@pytest.mark.parametrize("matcher,overlap", [(slamhip.SIFT_FLANN, "knn"), (slamhip.ORB_BF, "knn"),
                                             (slamhip.SIFT_FLANN, "desc_end"), (slamhip.SIFT_FLANN, "desc_start"),
                                             (slamhip.ORB_BF, "desc_start")])
def test_pipelined_scan_world1_matches_oracle(gpu_ctx, matcher, overlap):
    """PipelinedScan on one rank without a process group: four 1080p searches,
    each one's extraction queued on the other context before the previous
    search is taken (slam_batch_extract_async / _match_async / _finish), the
    winner hand-over and the winner's keypoints / matches (taken after the next
    search, as bench.py does) against the oracle's sequential searches; SIFT +
    BF-L2 (the headline) and ORB + Hamming (bench.py's configs[2] legs)"""
    import torch
    from slamhip.batch import Conditions, PipelinedScan
    host = slamhip.synth_frames(1920, 1080, 400, 17, seed=5)
    frames = torch.from_numpy(host).cuda()
    scan = PipelinedScan(0, 1, 0, overlap=overlap)
    first = scan.scans[1].db                   # any idle batch describes the first previous frame
    first.extract(frames[:1], 60, matcher)
    prev = torch.zeros(slamhip.lib().slam_batch_desc_bytes(matcher, 64 * 1024), dtype=torch.uint8, device="cuda")
    _, nprev = first.export_desc(0, prev)
    cond = Conditions(featureExtractingThreshold=60, requiredExtractedPointsCount=1000,
                      requiredMatchedPointsCount=150, matcherType=matcher, knnMatcherDistance=0.7)
    norm = O.NORM_HAMMING if matcher == slamhip.ORB_BF else O.NORM_L2
    batches = [(1, 5), (5, 9), (9, 13), (13, 17)]
    ref_prev = _oracle_desc(host[0], 60, matcher)
    owner, pending, wins = 0, None, 0
    for c in scan.ctxs:
        slamhip.lib().slam_profile_enable(c.handle, 1)
    scan.queue(frames[1:5], cond)
    for b, (lo, hi) in enumerate(batches):
        nxt = frames[batches[b + 1][0]:batches[b + 1][1]] if b + 1 < len(batches) else None
        good, kp_all, mc_all, in_batch, dc_all = scan.search(frames[lo:hi], prev, nprev, owner, cond, next_frames=nxt)
        if pending is not None:
            dk, dm = scan.winner_end(pending[0])
            np.testing.assert_array_equal(dk, pending[1])
            np.testing.assert_array_equal(dm, pending[2])
            pending = None
        rg, rkc, rmc, rdc, rin, rds = _oracle_search(host[lo:hi], ref_prev, 60, 1000, 150, matcher=matcher)
        np.testing.assert_array_equal(kp_all, rkc)
        np.testing.assert_array_equal(mc_all, rmc)
        np.testing.assert_array_equal(dc_all, rdc)
        assert good == rg
        if good >= 0:
            gi = int(rin[good])
            ri, rd = O.knn2(ref_prev, rds[gi], norm)
            wk = O.fast(host[lo + gi], 60, True)
            if matcher == slamhip.ORB_BF:
                wk = O.orb(host[lo + gi], wk)[0]     # the winner's descriptor-bearing keypoints
            pending = (scan.winner_begin(good, in_batch, dc_all, mc_all, nprev), wk, O.ratio(ri, rd, 0.7))
            wins += 1
        owner, nprev = scan.advance(good, in_batch, dc_all, prev, owner, nprev)
        if good >= 0:
            ref_prev = rds[int(rin[good])]
            assert nprev == len(ref_prev)
    if pending is not None:
        dk, dm = scan.winner_end(pending[0])
        np.testing.assert_array_equal(dk, pending[1])
        np.testing.assert_array_equal(dm, pending[2])
    assert wins >= 3
    # one kNN launch per search: no speculative match discarded and redone (the
    # estimate of each search is the previous search's, and these frames stay
    # inside it; test_batch_async_rematch covers a frame that outgrows it)
    launches = 0
    for c in scan.ctxs:
        ms, n = ctypes.c_double(0), ctypes.c_int(0)
        slamhip.lib().slam_profile_read(c.handle, 2, ctypes.byref(ms), ctypes.byref(n))    # family 2: knn_mfma
        launches += n.value
    assert launches == len(batches)
    scan.close()


def test_pipelined_scan_waits_for_torch_producer(gpu_ctx):
    """the queued extraction runs on the context's own
    stream, so it must be ordered after the torch kernels that produce its
    frames.  Each search's candidates are built on torch's current stream right
    before queue() (a long matmul chain ahead of an add + cast), then compared
    with the oracle on the same frames."""
    import torch
    from slamhip.batch import Conditions, PipelinedScan
    host = slamhip.synth_frames(1920, 1080, 400, 9, seed=5)
    src = torch.from_numpy(host).cuda()
    scan = PipelinedScan(0, 1, 0, overlap="desc_start")
    first = scan.scans[1].db
    first.extract(src[:1], 60, slamhip.SIFT_FLANN)
    prev = torch.zeros(slamhip.lib().slam_batch_desc_bytes(slamhip.SIFT_FLANN, 64 * 1024), dtype=torch.uint8,
                       device="cuda")
    _, nprev = first.export_desc(0, prev)
    ref_prev = _oracle_desc(host[0], 60)
    cond = Conditions(featureExtractingThreshold=60, requiredExtractedPointsCount=1000,
                      requiredMatchedPointsCount=150, matcherType=slamhip.SIFT_FLANN, knnMatcherDistance=0.7)
    a = torch.randn(4096, 4096, device="cuda")
    torch.cuda.synchronize()

    def produce(lo, hi):
        # ~tens of ms of queued work on torch's stream, then the frames themselves
        x = a
        for _ in range(12):
            x = x @ a
        z = (x[:1, :1] * 0).to(torch.int16)                # 0, but only after the chain
        return (src[lo:hi].to(torch.int16) + z).to(torch.uint8).contiguous()

    batches = [(1, 5), (5, 9)]
    scan.queue(produce(*batches[0]), cond)
    owner = 0
    for b, (lo, hi) in enumerate(batches):
        nxt = produce(*batches[b + 1]) if b + 1 < len(batches) else None
        good, kp_all, mc_all, in_batch, dc_all = scan.search(src[lo:hi], prev, nprev, owner, cond, next_frames=nxt)
        rg, rkc, rmc, rdc, rin, rds = _oracle_search(host[lo:hi], ref_prev, 60, 1000, 150)
        np.testing.assert_array_equal(kp_all, rkc)
        np.testing.assert_array_equal(mc_all, rmc)
        assert good == rg
        owner, nprev = scan.advance(good, in_batch, dc_all, prev, owner, nprev)
        if good >= 0:
            ref_prev = rds[int(rin[good])]
    scan.close()


@pytest.mark.parametrize("path", [slamhip.SYNTH_DRIFT, slamhip.SYNTH_STEADY])
def test_synth_frames_dev_matches_host(gpu_ctx, path):
    """the synthetic sequence rendered in HBM (slam_synth_sequence_dev, the
    device-resident pipeline's "decoded video") is byte-identical to the host
    generator, at 1080p (frames spread over the sequence) and at an odd size"""
    for (w, h, first, count) in ((1920, 1080, 0, 2), (1920, 1080, 777, 1), (333, 251, 5, 3)):
        dev = slamhip.synth_frames_dev(w, h, first, count, seed=1234, path=path, ctx=gpu_ctx)
        np.testing.assert_array_equal(dev.cpu().numpy(), slamhip.synth_frames(w, h, first, count, seed=1234,
                                                                                path=path))
