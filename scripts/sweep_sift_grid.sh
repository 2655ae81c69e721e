#!/bin/bash
# GPU box: bench at several SIFT descriptor grid sizes (tuning sweep)
mkdir -p gpurun_out
for g in "$@"; do
    SLAMHIP_SIFT_GRID=$g timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sweep_$g.json 2>&1
    rc=$?
    echo "grid $g rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
exit 0
