"""cProfile of bench.py's pipeline leg (host-side time by function)"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))
import bench  # noqa: E402
import slamhip  # noqa: E402

ctx = slamhip.Context(0)
bench.pipeline_leg(ctx)                         # warm
pr = cProfile.Profile()
pr.enable()
p = bench.pipeline_leg(ctx)
pr.disable()
print("fps", p["frames_per_s"], p["ms_by_op"])
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(25)
