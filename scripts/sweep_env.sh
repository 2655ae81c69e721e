#!/bin/bash
# GPU box: bench under several settings of one environment variable (tuning/ablation)
# usage: scripts/sweep_env.sh VAR value...
VAR=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sweep_${VAR}_$v.json 2>&1
    rc=$?
    echo "$VAR=$v rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
exit 0
