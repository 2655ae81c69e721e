#!/bin/bash
# kernel trace (+ memory copies) of the batch detector
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5detkt}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d $O/$tag -o run \
    -- python3 $R/scripts/diag/det_time.py > $O/$tag.log 2>&1 || { echo "kt failed"; tail $O/$tag.log; exit 1; }
for f in $(find $O/$tag -name '*stats.csv'); do echo "== $f"; cut -d, -f1-4 $f | sed 's/slamhip::(anonymous namespace):://g' | cut -c1-110; done
