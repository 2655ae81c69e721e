#!/bin/bash
# kernel split of the batch SIFT detector (scripts/diag/det_time.py)
set -o pipefail
tag=${1:-det}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $GRAFT_REPO_ROOT/scripts/diag/det_time.py > $GRAFT_REPO_ROOT/gpurun_out/${tag}_time.txt 2>&1 || exit 1
cat $GRAFT_REPO_ROOT/gpurun_out/${tag}_time.txt | tail -1
REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/${tag}_kt -o run -- python3 $GRAFT_REPO_ROOT/scripts/diag/det_time.py > $GRAFT_REPO_ROOT/gpurun_out/${tag}_kt.log 2>&1 || exit 1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/${tag}_kt -name "*kernel_stats.csv" | head -1)
head -12 "$f" | cut -c1-160
