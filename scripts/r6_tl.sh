#!/bin/bash
# host timeline of the early-exit and full pipeline_b210 legs, then a kernel
# trace of the early-exit leg (device idle per search)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r6tl}
mkdir -p $O
timeout -k 10 300 python3 $R/scripts/diag/pipe_timeline.py 2 ee > $O/${tag}_ee.txt 2>&1 || exit $?
timeout -k 10 300 python3 $R/scripts/diag/pipe_timeline.py 2 b210 > $O/${tag}_full.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/${tag}_kt -o run -- python3 $R/scripts/diag/pipe_b210_ee.py 27 > $O/${tag}_kt.log 2>&1 || { echo "rc=$?"; tail -5 $O/${tag}_kt.log; exit 1; }
tail -1 $O/${tag}_kt.log
