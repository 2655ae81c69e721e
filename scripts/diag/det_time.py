"""The device-batch SIFT detector (slam_sift_detect_batch) over 16 resident
1080p frames, timed; for rocprofv3 --kernel-trace --stats (per-kernel split).
Diagnostics only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))
import torch  # noqa: E402
import slamhip  # noqa: E402

ctx = slamhip.Context(0)
nb = 16
dev = torch.from_numpy(slamhip.synth_frames(1920, 1080, 0, nb, seed=1234)).cuda()
slamhip.siftDetectAndComputeBatch(dev, ctx=ctx)
torch.cuda.synchronize()
t0 = time.perf_counter()
n = 0
reps = int(os.environ.get("REPS", "4"))
for _ in range(reps):
    n += int(slamhip.siftDetectAndComputeBatch(dev, ctx=ctx).counts.sum())
el = time.perf_counter() - t0
print(f"batch detector: {reps * nb / el:.1f} frames/s, {el / (reps * nb) * 1e3:.3f} ms per frame, {n / (reps * nb):.0f} kps")
ctx.close()
