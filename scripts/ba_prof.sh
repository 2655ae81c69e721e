#!/bin/bash
# BA kernel trace: W = 8 (1080p, 10k points) and W = 16 (4K, 40k points)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-ba}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/${TAG}_w8 -o run -- python3 $R/scripts/ba_bench.py 8 10000 > $O/${TAG}_w8.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/${TAG}_w16 -o run -- python3 $R/scripts/ba_bench.py 16 40000 4k > $O/${TAG}_w16.log 2>&1 || exit $?
tail -1 $O/${TAG}_w8.log; tail -1 $O/${TAG}_w16.log
