"""Golden BA windows of the framesBatchSize-210 searched-frame pipelines (test data).

Source: bench.py's `pipeline_b210_leg` (slamMain at the reference's example
config, framesBatchSize 210, BA on, BAMaxFramesCnt 8, Huber 4; windows built by
mainCycle.cpp:193-210 from the frames the search selected) run on an MI355X
with SLAMHIP_BA_DUMP set (scripts/diag/ba_window_dump.sh), which wrote every
window's inputs and the GPU's solution to gpurun_out/ba_windows_{sift,orb}.npz.

This script keeps each window's INPUTS (K4, ext, pts, obs_frame, obs_point,
obs_xy, loss, loss_param) -- what bundleAdjustment (bundleAdjustment.cpp:73-129)
receives -- plus the round-4 GPU summary of the dump for provenance.  Every
point of the global array is kept (the solvers see the array the pipeline
passed).  The expected outputs are not stored: the checker is oracle/ba.c run
on the same inputs (tests/ba_envelope.py).

usage: python tests/golden/make_ba_b210.py [dump_prefix]   (default gpurun_out/ba_windows)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
KEYS = ("K4", "ext", "pts", "obs_frame", "obs_point", "obs_xy", "loss", "loss_param")


def convert(src, dst):
    z = np.load(src)
    out = {"kind": np.array("ba_windows")}
    k = 0
    while f"w{k}_in_K4" in z.files:
        for name in KEYS:
            out[f"w{k}_{name}"] = z[f"w{k}_in_{name}"]
        out[f"w{k}_r4_gpu_summary"] = z[f"w{k}_summary"]   # initial, final cost, iterations, residuals
        k += 1
    np.savez_compressed(dst, **out)
    return k


def load(path):
    """-> list of window input dicts"""
    z = np.load(path)
    ws = []
    k = 0
    while f"w{k}_K4" in z.files:
        w = {name: z[f"w{k}_{name}"] for name in KEYS}
        w["loss"] = int(w["loss"])
        w["loss_param"] = float(w["loss_param"])
        ws.append(w)
        k += 1
    return ws


if __name__ == "__main__":
    pre = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "..", "..", "gpurun_out", "ba_windows")
    for m in ("sift", "orb"):
        n = convert(f"{pre}_{m}.npz", os.path.join(HERE, f"ba_b210_{m}.npz"))
        print(m, n, "windows")
