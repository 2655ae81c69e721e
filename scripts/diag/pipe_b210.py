"""bench.py's pipeline_b210 leg alone (SIFT, or ORB with 'orb'): ms per search,
frames/s, and (check) the BA windows against the oracle.
usage: python3 scripts/diag/pipe_b210.py [orb] [check]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import slamhip  # noqa: E402

ctx = slamhip.Context(0)
r = bench.pipeline_b210_leg(ctx, check="check" in sys.argv, orb="orb" in sys.argv)
print(json.dumps({k: r.get(k) for k in ("frames_per_s", "candidate_frames_per_s", "ms_per_search", "searches",
                                         "parity_ok", "ba_north_star_ok")}))
