"""bench.py's pipeline_b210 leg with the full scan and with tail-first early
exit at several chunk sizes: frames/s, candidates per search, and whether the
early-exit runs reproduce the full scan (winners, poses, points, BA windows).
usage: python3 scripts/diag/pipe_b210_ee.py [chunk ...]   (default 27 54)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import slamhip  # noqa: E402

chunks = [int(a) for a in sys.argv[1:]] or [27, 54]
ctx = slamhip.Context(0)
full = bench.pipeline_b210_leg(ctx, check=False)
a = full.pop("_result")
rows = {"full": {k: full.get(k) for k in ("frames_per_s", "candidates_per_search", "ms_per_search", "searches")}}
for c in chunks:
    r = bench.pipeline_b210_leg(ctx, check=False, early_exit=c)
    b = r.pop("_result")
    same = (a["searches"] == b["searches"] and len(a["poses"]) == len(b["poses"])
            and all(np.array_equal(x, y) for x, y in zip(a["poses"], b["poses"]))
            and np.array_equal(a["points"], b["points"]) and a["ba"] == b["ba"])
    rows[f"chunk{c}"] = {k: r.get(k) for k in ("frames_per_s", "candidates_per_search", "ms_per_search", "searches")}
    rows[f"chunk{c}"]["identical_to_full_scan"] = bool(same)
print(json.dumps(rows))
