"""bench.py's 24-frame slamMain pipeline leg alone (timing, per-operation ms) and
its oracle check: python3 scripts/diag/pipe24.py [repeats]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import slamhip  # noqa: E402

ctx = slamhip.Context(0)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    r = bench.pipeline_leg(ctx)
    print(json.dumps({k: r[k] for k in ("frames_per_s", "ms_per_frame", "poses", "points", "ba_final_rmse",
                                        "ms_by_op")}), flush=True)
cpu = bench.pipeline_cpu_baseline(r["frames"])
chk = bench.pipeline_compare(r["_result"], cpu.pop("_result"))
print("cpu_frames_per_s", cpu.get("frames_per_s"))
print("oracle_check", json.dumps(chk, default=str)[:3000])
