"""solvePnPRansac alone on pipeline-sized inputs (1800 points, 3 % outliers):
per-call ms; with SLAMHIP_PNP_TIMING=1 the phases; under rocprofv3 the kernels
without a concurrent search.  Diagnostics only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import slamhip  # noqa: E402
from test_oracle import pnp_scene  # noqa: E402

ctx = slamhip.Context(0, priority=int(os.environ.get("PRIO", "0")))
if os.environ.get("SLAMHIP_PNP_SUMS"):
    from slamhip import _lib as L
    ctx.set_option(L.OPT_PNP_SUMS, int(os.environ["SLAMHIP_PNP_SUMS"]))
K, rv, t, X, uv, out = pnp_scene(1800, 3, outliers=0.03)
slamhip.solvePnPRansac(X, uv, K, None, ctx=ctx)
t0 = time.perf_counter()
reps = 20
for _ in range(reps):
    slamhip.solvePnPRansac(X, uv, K, None, ctx=ctx)
print(f"pnp n=1800 alone: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms per call")
