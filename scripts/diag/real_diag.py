import os, sys
sys.path.insert(0, "slam-indoor-code_amd"); sys.path.insert(0, "tests")
import numpy as np
import oracle_ffi as O
import slamhip
v = np.load("tests/golden/real_vga.npz"); h = np.load("tests/golden/real_1080p.npz")
ctx = slamhip.Context(0)
cases = {}
for i, im in enumerate(v["bgr"]): cases[f"vga{i}"] = im
for i, im in enumerate(v["gray"]):
    cases[f"gray{i}"] = im
    cases[f"gray{i}_bgr"] = np.ascontiguousarray(np.repeat(im[..., None], 3, 2))
    cases[f"gray{i}_640"] = np.ascontiguousarray(im[:, :640])
cases["hd"] = h["bgr"][0]
syn = slamhip.synth_frames(748, 480, 0, 1, seed=5)[0]
cases["synth748"] = syn
for name, im in cases.items():
    kps = O.fast(im, 10, True)
    _, d = slamhip.extractDescriptor(im, kps, slamhip.SIFT_FLANN, ctx=ctx)
    r = O.sift(im, kps)
    rk, rd = O.orb(im, kps)
    ko, od = slamhip.extractDescriptor(im, kps, slamhip.ORB_BF, ctx=ctx)
    print(name, im.shape, len(kps), "sift mism", float((d != r).mean()), "orb mism", float((od != rd).mean()) if len(rd) else None, flush=True)
