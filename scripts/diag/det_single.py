"""siftDetectAndCompute on single 1080p frames through host buffers (bench.py's
sift_detector leg), timed; SLAMHIP_DET_TIMING=1 prints the host phases.
Diagnostics only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))
import slamhip  # noqa: E402

ctx = slamhip.Context(0)
frames = slamhip.synth_frames(1920, 1080, 0, 3, seed=1234)
slamhip.siftDetectAndCompute(frames[0], ctx=ctx)
reps = int(os.environ.get("REPS", "6"))
t0 = time.perf_counter()
for r in range(reps):
    t1 = time.perf_counter()
    k, _ = slamhip.siftDetectAndCompute(frames[r % 3], ctx=ctx)
    print(f"frame {r}: {len(k)} kps {1e3 * (time.perf_counter() - t1):.3f} ms", file=sys.stderr)
el = time.perf_counter() - t0
print(f"single-frame detector: {reps / el:.1f} frames/s, {el / reps * 1e3:.3f} ms per frame")
ctx.close()
