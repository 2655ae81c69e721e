#!/bin/bash
# the SIFT and ORB searched-frame pipelines (bench.py pipeline_b210_leg) with
# every BA window's inputs and GPU solution dumped to gpurun_out/ba_windows_*.npz
set -o pipefail
mkdir -p gpurun_out
SLAMHIP_BA_DUMP=gpurun_out/ba_windows timeout -k 10 600 python -u -c "
import sys; sys.argv = ['bench.py']
import bench, slamhip
ctx = slamhip.Context(0)
for orb in (False, True):
    r = bench.pipeline_b210_leg(ctx, check=False, orb=orb)
    print('orb' if orb else 'sift', r['frames_per_s'], r['ba_windows'])
"
