#!/bin/bash
# round-5: device timeline of the SIFT pipeline_b210 leg (kernel trace) -- idle gaps per search
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5bt}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $O/${tag}_kt -o run -- python3 $R/scripts/diag/pipe_b210.py > $O/${tag}.log 2>&1 || { echo "rc=$?"; tail -5 $O/${tag}.log; exit 1; }
cd $R
tail -1 $O/${tag}.log
python3 scripts/diag/timeline.py $(find $O/${tag}_kt -name '*kernel_trace.csv' | head -1) sift_desc_band 6 10
