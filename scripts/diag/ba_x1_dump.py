"""GPU BA solutions after k = 1, 2, 3 LM iterations on the golden
framesBatchSize-210 windows (diagnostics: compared offline with the oracle's
iterates, scripts/diag/ba_x1_compare.py).  Writes gpurun_out/ba_x1.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))
import slamhip  # noqa: E402
from make_ba_b210 import load  # noqa: E402

ctx = slamhip.Context(0)
out = {}
for m in ("sift", "orb"):
    for wi, w in enumerate(load(os.path.join(ROOT, "tests", "golden", f"ba_b210_{m}.npz"))):
        for k in (0, 1, 2, 3):
            K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
            s = slamhip.bundle_adjust_arrays(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"], w["loss"],
                                             w["loss_param"], max_iters=k, ctx=ctx)
            key = f"{m}_w{wi}_k{k}"
            out[key + "_K4"], out[key + "_ext"], out[key + "_pts"] = K4, ext, pts
            out[key + "_summary"] = np.array([s.initial_cost, s.final_cost, s.iterations, s.successful_steps,
                                              s.termination], np.float64)
            print(key, s.initial_cost, s.final_cost, s.iterations, s.successful_steps, flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "ba_x1.npz"), **out)
