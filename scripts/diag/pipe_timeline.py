"""Host-side timeline of bench.py's 24-frame slamMain pipeline leg: every GpuOps
call and the cycle module's per-frame helpers, with the thread that ran it
(main loop / post-search worker / BA worker), so the critical path between the
searches and the post-search work shows.

usage: python3 scripts/diag/pipe_timeline.py [repeats] [b210|ee]   (b210: the SIFT
pipeline_b210 leg instead, no oracle check; ee: its early-exit form)
prints per-thread busy time, the main thread's gaps, and per-name totals"""
import os
import sys
import threading
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import slamhip  # noqa: E402
from slamhip import cycle  # noqa: E402

EV = []


def traced(name, f):
    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            EV.append((threading.current_thread().name, name, t0, time.perf_counter()))
    return g


for fn in ("find_good_frame_from_batch", "fill_video_frame_batch", "old_spatial_points_and_new_coords",
           "push_new_spatial_points", "key_point_coords", "start_bundle_adjustment",
           "move_processed_data_to_global_struct"):
    setattr(cycle, fn, traced(fn, getattr(cycle, fn)))
from slamhip import batch as _batch  # noqa: E402
for meth in ("extract_match", "result", "export_desc", "fast", "keypoints"):
    setattr(_batch.DeviceBatch, meth, traced("db." + meth, getattr(_batch.DeviceBatch, meth)))
for meth in ("search", "solve_pnp", "reconstruct", "rodrigues", "ba_async", "fast", "ingest",
             "estimate_transformation", "fast_batch", "_query"):
    if hasattr(cycle.GpuOps, meth):
        setattr(cycle.GpuOps, meth, traced("ops." + meth, getattr(cycle.GpuOps, meth)))
MAIN_STARTS = []
_orig_main = cycle.slam_main


def _main(*a, **k):
    MAIN_STARTS.append(time.perf_counter())
    return _orig_main(*a, **k)


cycle.slam_main = _main
_orig_finish = cycle.PendingBA.finish
cycle.PendingBA.finish = traced("PendingBA.finish", _orig_finish)

ctx = slamhip.Context(0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 2
for r in range(reps):
    EV.clear()
    t0 = time.perf_counter()
    if "b210" in sys.argv or "ee" in sys.argv:
        res = bench.pipeline_b210_leg(ctx, check=False, early_exit=bench.EARLY_EXIT_CHUNK if "ee" in sys.argv else 0)
        print(f"rep {r}: frames_per_s {res['frames_per_s']:.1f} ms_per_search {res['ms_per_search']:.3f}")
    else:
        res = bench.pipeline_leg(ctx)
        print(f"rep {r}: frames_per_s {res['frames_per_s']:.1f} ms_per_frame {res['ms_per_frame']:.3f}")
# the timed slam_main is the last one the leg runs: keep the events after its start
ev = sorted((e for e in EV if e[2] >= MAIN_STARTS[-1]), key=lambda e: e[2])
T0, T1 = MAIN_STARTS[-1], max(e[3] for e in ev)
print(f"timed run: {len(ev)} events over {(T1 - T0) * 1e3:.2f} ms")
per_thread = defaultdict(list)
for th, n, a, b in ev:
    per_thread[th].append((a, b, n))


def union(iv):
    iv = sorted(iv)
    tot, cur = 0.0, None
    for a, b, _ in iv:
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        tot += cur[1] - cur[0]
    return tot


for th, iv in per_thread.items():
    print(f"thread {th:28s} busy {union(iv) * 1e3:8.2f} ms in {len(iv)} calls")
tot = defaultdict(lambda: [0, 0.0])
for th, n, a, b in ev:
    tot[(th, n)][0] += 1
    tot[(th, n)][1] += b - a
for (th, n), (c, s) in sorted(tot.items(), key=lambda x: -x[1][1]):
    print(f"  {th[:20]:20s} {n:40s} {c:4d} {s * 1e3:8.2f} ms")
print("main-thread sequence (ms from start):")
for th, n, a, b in ev:
    print(f"  {(a - T0) * 1e3:8.2f} {(b - T0) * 1e3:8.2f} {th[:16]:16s} {n}")
