"""BA window timing (GPU): one synthetic BAMaxFramesCnt window, solved twice
(the first includes warm-up); prints ms per window and per LM iteration."""
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))


def main():
    import torch
    import slamhip
    from slamhip import synthba
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    npts = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    k4k = len(sys.argv) > 3 and sys.argv[3] == "4k"
    kw = dict(width=3840, height=2160, K4=synthba.K_4K) if k4k else {}
    ctx = slamhip.Context(0)
    w = synthba.make_window(nframes=nf, npoints=npts, seed=7, **kw)
    for rep in range(3):
        K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sm = slamhip.bundle_adjust_arrays(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"],
                                          slamhip.LOSS_HUBER, 4.0, ctx=ctx)
        el = time.perf_counter() - t0
    print(json.dumps({"frames": nf, "points": npts, "obs": int(len(w["obs_frame"])), "ms": el * 1e3,
                      "iters": int(sm.iterations), "ms_per_iter": el * 1e3 / max(1, sm.iterations),
                      "final_rmse": math.sqrt(sm.final_cost / sm.num_residuals)}))
    ctx.close()


if __name__ == "__main__":
    main()
