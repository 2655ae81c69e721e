"""GPU box: time solvePnPRansac / estimateTransformation calls (pipeline-sized inputs)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import slamhip
from test_oracle import pnp_scene

ctx = slamhip.Context(0)
for n, outl in ((1500, 0.3), (4000, 0.3)):
    K, rv, t, X, uv, out = pnp_scene(n, 3, outliers=outl)
    slamhip.solvePnPRansac(X, uv, K, None, ctx=ctx)
    t0 = time.perf_counter()
    for _ in range(10):
        slamhip.solvePnPRansac(X, uv, K, None, ctx=ctx)
    print(f"pnp n={n}: {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms")

# estimateTransformation (findEssentialMat RANSAC + recoverPose), 30 % outliers
rng = np.random.default_rng(3)
K = np.array([[1724.676, 0, 995.966], [0, 1730.482, 550.192], [0, 0, 1.0]])
for n in (2000, 10000):
    a = np.deg2rad(3.0)
    R2 = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    t2 = np.array([-0.2, 0.01, 0.02])
    X = np.stack([rng.uniform(-2, 2, n), rng.uniform(-1, 1, n), rng.uniform(3, 8, n)], 1)
    def proj(R, t):
        u = (X @ R.T + t) @ K.T
        return (u[:, :2] / u[:, 2:]).astype(np.float32)
    q1 = proj(np.eye(3), np.zeros(3)) + rng.normal(0, 0.5, (n, 2)).astype(np.float32)
    q2 = proj(R2, t2) + rng.normal(0, 0.5, (n, 2)).astype(np.float32)
    bad = rng.random(n) < 0.3
    q2[bad] = rng.uniform([0, 0], [1920, 1080], (int(bad.sum()), 2)).astype(np.float32)
    slamhip.estimateTransformation(q1, q2, K, ctx=ctx)
    t0 = time.perf_counter()
    for _ in range(5):
        slamhip.estimateTransformation(q1, q2, K, ctx=ctx)
    print(f"relative pose n={n}: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms")
