"""bench.py's pipeline_b210 leg alone (timing + its oracle checks): python3 scripts/diag/pipe210.py [nframes]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import slamhip  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3800
ctx = slamhip.Context(0)
r = bench.pipeline_b210_leg(ctx, nframes=n, check=True)
print(json.dumps(r))
