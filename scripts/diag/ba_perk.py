"""Where does the GPU's BA leave the oracle's reordering spread?  (diagnostics)

For every golden framesBatchSize-210 window (tests/golden/ba_b210_*.npz) the
cost after k LM iterations, k = 1..K:
  * GPU: slam_ba capped at k iterations (one solve per k);
  * oracle/ba.c: one traced run per observation order (tests/ba_envelope.py
    orders: 0 = AddResidualBlock order, odd = shuffled inside frames, even =
    shuffled globally with the points relabelled), under each factorisation of
    --solvers (0 = the oracle's LL', 1 = Eigen SimplicialLDLT's arithmetic, the
    reference's solver; 2 = the GPU solve's arithmetic, diagnostics only).
A valid reordering stays inside the orders' [min, max] at every k; a
formula-level difference shows as a one-sided offset from an early k.

usage: python scripts/diag/ba_perk.py [--orders 16] [--kmax 50] [--solvers 0,1] [--no-gpu] [--out FILE]
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))
from ba_envelope import lm_path_envelope  # noqa: E402
from make_ba_b210 import load  # noqa: E402


def gpu_costs(w, ks, ctx):
    import slamhip
    out = []
    for k in ks:
        s = slamhip.bundle_adjust_arrays(w["K4"].copy(), w["ext"].copy(), w["pts"].copy(), w["obs_frame"],
                                         w["obs_point"], w["obs_xy"], w["loss"], w["loss_param"], max_iters=k,
                                         ctx=ctx)
        out.append((s.final_cost, int(s.iterations), int(s.termination)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--orders", type=int, default=16)
    ap.add_argument("--kmax", type=int, default=50)
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--solvers", default="0,1")
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ba_perk.json"))
    a = ap.parse_args()
    ctx = None
    if not a.no_gpu:
        import slamhip
        ctx = slamhip.Context(0)
    ks = list(range(1, a.kmax + 1))
    res = {}
    for m in ("sift", "orb"):
        for wi, w in enumerate(load(os.path.join(ROOT, "tests", "golden", f"ba_b210_{m}.npz"))):
            t0 = time.time()
            solvers = tuple(int(x) for x in a.solvers.split(","))
            lo, hi, tr = lm_path_envelope(w, a.kmax, a.orders, a.threads, solvers)
            o0 = tr[0][0]
            rec = {"observations": int(len(w["obs_frame"])), "k": ks, "oracle_order0": o0.tolist(),
                   "oracle_min": lo.tolist(), "oracle_max": hi.tolist(), "orders": a.orders,
                   "solvers": list(solvers)}
            if ctx is not None:
                g = gpu_costs(w, ks, ctx)
                gc = np.array([x[0] for x in g])
                rec["gpu"] = gc.tolist()
                rec["gpu_iterations"] = [x[1] for x in g]
                width = np.maximum(hi - lo, 1e-300)
                # signed distance outside the spread in units of its width (0 inside)
                out = np.where(gc > hi, (gc - hi) / width, np.where(gc < lo, (gc - lo) / width, 0.0))
                rec["gpu_outside_widths"] = out.tolist()
                rec["gpu_rel_to_order0"] = ((gc - o0) / o0).tolist()
                first = next((k for k, o in zip(ks, out) if o != 0.0), None)
                rec["first_k_outside"] = first
                rec["k_outside"] = [k for k, o in zip(ks, out) if o != 0.0]
            res[f"{m}_w{wi}"] = rec
            print(f"{m} w{wi}: {time.time() - t0:.1f}s", "first_k_outside", rec.get("first_k_outside"), flush=True)
            if ctx is not None:
                for k in (1, 2, 3, 5, 10, 20, 30, 40, 50):
                    if k <= a.kmax:
                        i = k - 1
                        print(f"   k={k:2d} gpu {rec['gpu'][i]:.10g} oracle [{lo[i]:.10g}, {hi[i]:.10g}] "
                              f"width_rel {(hi[i] - lo[i]) / o0[i]:.2e} outside {rec['gpu_outside_widths'][i]:+.2f} w",
                              flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
