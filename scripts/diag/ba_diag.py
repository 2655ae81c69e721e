import sys
sys.path.insert(0, "slam-indoor-code_amd"); sys.path.insert(0, "tests")
import numpy as np
import oracle_ffi as O
import slamhip
from slamhip import synthba
ctx = slamhip.Context(0)
for loss, a in [(O.LOSS_TUKEY, 4.0), (O.LOSS_ARCTAN, 4.0)]:
    for nf, npnt, seed in [(5, 400, 3), (8, 2000, 7), (8, 10000, 7)]:
        w = synthba.make_window(nframes=nf, npoints=npnt, seed=seed)
        rK, rE, rP, rs = O.ba(w["K4"], w["ext"], w["pts"], w["obs_frame"], w["obs_point"], w["obs_xy"], loss, a)
        K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
        gs = slamhip.bundle_adjust_arrays(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"], loss, a, ctx=ctx)
        print(loss, nf, npnt, "ora", rs.initial_cost, rs.final_cost, rs.iterations, rs.successful_steps, rs.termination,
              "gpu", gs.initial_cost, gs.final_cost, gs.iterations, gs.successful_steps, gs.termination, flush=True)
        for it in (1, 2, 3, 5, 8):
            rK, rE, rP, rs = O.ba(w["K4"], w["ext"], w["pts"], w["obs_frame"], w["obs_point"], w["obs_xy"], loss, a, max_iters=it)
            K4, ext, pts = w["K4"].copy(), w["ext"].copy(), w["pts"].copy()
            gs = slamhip.bundle_adjust_arrays(K4, ext, pts, w["obs_frame"], w["obs_point"], w["obs_xy"], loss, a, max_iters=it, ctx=ctx)
            print("   it", it, rs.final_cost, gs.final_cost, rs.successful_steps, gs.successful_steps,
                  float(np.abs(pts - rP).max()), flush=True)
