"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The reference ships no golden vectors, so these are known
answers of the restated algorithms: they pin the oracle against regressions and
give the GPU tests fixed inputs.  Inputs are synthetic (slamhip.synth_frames) or
seeded random; nothing here comes from the reference tree.
Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_ffi as O  # noqa: E402
import slamhip  # noqa: E402
from slamhip import synthba  # noqa: E402


def save(name, **kw):
    np.savez_compressed(os.path.join(HERE, name), **kw)


def main():
    f = slamhip.synth_frames(96, 64, 3, 1, seed=2024)[0]
    for thr, nms in [(10, True), (25, True), (10, False)]:
        k = O.fast(f, thr, nms)
        save(f"fast_96x64_t{thr}_{'nms' if nms else 'raw'}.npz", kind="fast", image=f, threshold=thr, nms=nms,
             expected=np.stack([k["x"], k["y"], k["response"]], 1))
    kat = np.zeros((32, 32), np.uint8)
    kat[16, 16] = 255
    k = O.fast(kat, 10, True)
    save("fast_kat_single_pixel.npz", kind="fast", image=kat, threshold=10, nms=True,
         expected=np.stack([k["x"], k["y"], k["response"]], 1))

    g = slamhip.synth_frames(160, 120, 5, 1, seed=77)[0]
    k = O.fast(g, 10, True)[:32]
    save("sift_160x120_32kp.npz", kind="sift", image=g, keypoints=k.view(np.uint8).reshape(len(k), 28),
         expected=O.sift(g, k))
    k = O.fast(g, 8, True)
    kk, d = O.orb(g, k)
    save("orb_160x120.npz", kind="orb", image=g, keypoints=k.view(np.uint8).reshape(len(k), 28), expected=d,
         expected_kps=kk.view(np.uint8).reshape(len(kk), 28))

    rng = np.random.default_rng(512)
    q = rng.integers(0, 24, (512, 128)).astype(np.float32)
    t = rng.integers(0, 24, (512, 128)).astype(np.float32)
    t[300], t[400], q[:4] = t[5], t[6], t[5]          # planted ties: lower trainIdx wins
    idx, dist = O.knn2(q, t, O.NORM_L2)
    save("knn_l2_512x512_ties.npz", kind="knn", query=q, train=t, norm=O.NORM_L2, expected_idx=idx,
         expected_dist=dist)
    qb = rng.integers(0, 256, (256, 32), dtype=np.uint8)
    tb = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    tb[299] = tb[1]
    qb[0] = tb[1]
    idx, dist = O.knn2(qb, tb, O.NORM_HAMMING)
    save("knn_hamming_256x300.npz", kind="knn", query=qb, train=tb, norm=O.NORM_HAMMING, expected_idx=idx,
         expected_dist=dist)

    w = synthba.make_window(nframes=3, npoints=200, seed=11)
    for loss, a, tag in [(O.LOSS_NONE, 0.0, "none"), (O.LOSS_HUBER, 4.0, "huber")]:
        _, _, _, s = O.ba(w["K4"], w["ext"], w["pts"], w["obs_frame"], w["obs_point"], w["obs_xy"], loss, a)
        save(f"ba_3f_200p_{tag}.npz", kind="ba", K4=w["K4"], ext=w["ext"], pts=w["pts"], obs_frame=w["obs_frame"],
             obs_point=w["obs_point"], obs_xy=w["obs_xy"], loss=loss, loss_param=a, final_cost=s.final_cost,
             initial_cost=s.initial_cost)
    siftdet_golden()
    print("golden fixtures written to", HERE)


def siftdet_golden():
    """full SIFT detector (oracle/siftdet.c) on a textured 160 x 120 frame"""
    f = slamhip.synth_frames(160, 120, 7, 1, seed=31)[0]
    k, d = O.sift_detect(f)
    save("siftdet_160x120.npz", kind="siftdet", image=f, expected_kps=k.view(np.uint8).reshape(len(k), 28),
         expected=d)


if __name__ == "__main__":
    if sys.argv[1:] == ["siftdet"]:
        siftdet_golden()
    else:
        main()
