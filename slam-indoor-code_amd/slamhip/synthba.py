"""Synthetic bundle-adjustment windows with the reference's observation pattern.

The reference feeds Ceres one window of BAMaxFramesCnt frames (mainCycle.cpp:
201-210, non-overlapping windows).  Because window entries are snapshots taken
before a frame later serves as "prev" (mainCycle.cpp:92-93, :193-200;
mainCycleInternals.cpp:178-246), a point born at pair (i, i+1) is observed in
the window by frame i+1 and by the frames that later re-match it; the first
pair observes its points twice.  Observations are FAST keypoint positions, i.e.
integer pixels.  This generator reproduces that structure from a ground-truth
scene (SURVEY.md 8d "BA synthetic problems"):
  - camera: 2 cm/frame forward, 0.5 deg/frame yaw;
  - points 2..8 m in front of the first camera, inside the image;
  - track lengths 1..4 frames (a share of single-observation points);
  - observation noise sigma 0.5 px, then rounded to integer pixels;
  - initial perturbation: rotation 0.5 deg, translation 1 cm, points 2 cm, K 0.5 %.
Deterministic for a given seed.  Pure numpy (host-side data preparation).
"""
import math

import numpy as np

# config/samsung-hv.xml:3-9 (1080p) and config/samsung-hv-4k.xml:3-9 (4K) intrinsics
K_1080P = (1724.676, 1730.482, 995.966, 550.192)
K_4K = (3441.214, 3453.929, 2009.931, 1130.607)


def _aa_rotate(aa, p):
    th2 = float(aa @ aa)
    if th2 > np.finfo(np.float64).eps:
        th = math.sqrt(th2)
        w = aa / th
        c, s = math.cos(th), math.sin(th)
        return p * c + np.cross(w, p) * s + np.outer(p @ w, w) * (1 - c)
    return p + np.cross(aa, p)


def project(K4, ext, X):
    fx, fy, cx, cy = K4
    Xc = _aa_rotate(ext[:3], X) + ext[3:]
    return np.stack([fx * Xc[:, 0] / Xc[:, 2] + cx, fy * Xc[:, 1] / Xc[:, 2] + cy], 1), Xc[:, 2]


def make_window(nframes=8, npoints=2000, width=1920, height=1080, K4=K_1080P, seed=7, noise=0.5,
                single_share=0.3, perturb=True):
    """Returns dict(K4, ext, pts, obs_frame, obs_point, obs_xy, gt_*) ready for BA.
    ext[i] = (angle-axis, t) mapping world -> camera i; frame 0 = identity."""
    rng = np.random.default_rng(seed)
    K4 = np.array(K4, np.float64)
    ext = np.zeros((nframes, 6))
    for i in range(nframes):
        yaw = math.radians(0.5 * i)
        ext[i, :3] = (0.0, yaw, 0.0)
        ext[i, 3:] = (0.0, 0.0, -0.02 * i)
    # points: back-project random pixels of frame 0 at random depth
    u = rng.uniform(40, width - 40, npoints)
    v = rng.uniform(40, height - 40, npoints)
    z = rng.uniform(2.0, 8.0, npoints)
    pts = np.stack([(u - K4[2]) / K4[0] * z, (v - K4[3]) / K4[1] * z, z], 1)
    of, op, oxy = [], [], []
    for p in range(npoints):
        if p < npoints * 0.15:
            first, length = 0, int(rng.integers(2, 5))          # first pair: doubly observed
        else:
            first = int(rng.integers(1, nframes))
            length = 1 if rng.random() < single_share else int(rng.integers(2, 5))
        for f in range(first, min(nframes, first + length)):
            xy, depth = project(K4, ext[f], pts[p:p + 1])
            xy = xy[0] + rng.normal(0, noise, 2)
            if depth[0] <= 0.1 or not (0 <= xy[0] < width and 0 <= xy[1] < height):
                continue
            of.append(f)
            op.append(p)
            oxy.append(np.round(xy))
    out = dict(gt_K4=K4.copy(), gt_ext=ext.copy(), gt_pts=pts.copy(),
               obs_frame=np.array(of, np.int32), obs_point=np.array(op, np.int32),
               obs_xy=np.array(oxy, np.float64).reshape(-1, 2))
    if perturb:
        K4 = K4 * (1 + rng.normal(0, 0.005, 4))
        ext = ext.copy()
        ext[1:, :3] += rng.normal(0, math.radians(0.5), (nframes - 1, 3))
        ext[1:, 3:] += rng.normal(0, 0.01, (nframes - 1, 3))
        pts = pts + rng.normal(0, 0.02, pts.shape)
    out.update(K4=np.ascontiguousarray(K4), ext=np.ascontiguousarray(ext), pts=np.ascontiguousarray(pts))
    return out
