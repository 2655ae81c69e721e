#!/bin/bash
# BA window timing across camera-reduction workgroup counts (GPU box).
# usage: scripts/ba_sweep.sh TAG n1 n2 ...
TAG=$1; shift
mkdir -p gpurun_out
for n in "$@"; do
  SLAMHIP_BA_BLOCKS=$n timeout -k 10 120 python3 scripts/ba_bench.py > gpurun_out/${TAG}_ba_$n.json 2>/dev/null || exit $?
done
