"""Every dumped searched-frame BA window (scripts/diag/ba_window_dump.sh) solved
again on the GPU and by oracle/ba.c with the 50-iteration cap and with 500
iterations: do the two meet once both have converged?  Diagnostics only."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))
import oracle_ffi as O  # noqa: E402
import slamhip  # noqa: E402

ctx = slamhip.Context(0)
for tag in ("sift", "orb"):
    f = os.path.join(ROOT, "gpurun_out", f"ba_windows_{tag}.npz")
    if not os.path.exists(f):
        continue
    z = np.load(f)
    k = 0
    while f"w{k}_summary" in z:
        w = {n[len(f"w{k}_in_"):]: z[n] for n in z.files if n.startswith(f"w{k}_in_")}
        nres = 2 * len(w["obs_frame"])
        rm = lambda c: math.sqrt(c / max(1, nres))
        for it in (50, 500):
            K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
            g = slamhip.bundle_adjust_arrays(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"],
                                             int(w["loss"]), float(w["loss_param"]), max_iters=it, ctx=ctx)
            o = O.ba(w["K4"], w["ext"], w["pts"], w["obs_frame"], w["obs_point"], w["obs_xy"], int(w["loss"]),
                     float(w["loss_param"]), max_iters=it)[3]
            print(f"{tag} w{k} iters<= {it}: gpu {g.final_cost:.10g} ({g.iterations} it, term {g.termination}) "
                  f"oracle {o.final_cost:.10g} ({o.iterations} it, term {o.termination}) "
                  f"rel {abs(g.final_cost - o.final_cost) / o.final_cost:.3g} rmse_px {abs(rm(g.final_cost) - rm(o.final_cost)):.3g}",
                  flush=True)
        k += 1
ctx.close()
