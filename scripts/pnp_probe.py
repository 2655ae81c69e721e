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
