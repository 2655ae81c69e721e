"""cProfile of the main thread through bench.py's pipeline_b210 leg (SIFT): where
the host time between the searches goes.  Diagnostics only."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import slamhip  # noqa: E402

ctx = slamhip.Context(0)
bench.pipeline_b210_leg(ctx, check=False)          # warm
pr = cProfile.Profile()
pr.enable()
r = bench.pipeline_b210_leg(ctx, check=False)
pr.disable()
print("ms_per_search", r["ms_per_search"], "searches", r["searches"])
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
