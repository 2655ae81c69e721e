"""bench.py's pipeline leg alone: the resident GpuOps slamMain run on the 24-frame
1080p configs[2] sequence, timed, and compared with the oracle run of the same
sequence (poses, points, per-window BA RMSE)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))

import bench  # noqa: E402


def main():
    import slamhip
    ctx = slamhip.Context(0)
    p = bench.pipeline_leg(ctx)
    frames, res = p.pop("frames"), p.pop("_result")
    cpu = bench.pipeline_cpu_baseline(frames)
    p["oracle_check"] = bench.pipeline_compare(res, cpu.pop("_result"))
    p["cpu_baseline"] = cpu
    print(json.dumps(p))
    ctx.close()


if __name__ == "__main__":
    main()
