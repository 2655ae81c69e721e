#!/bin/bash
# Round 6 detector A/B: the detector parity tests on the default build, then
# the 16-frame batch timing per environment variant (interleaved, twice), then
# one kernel trace of the default.
# usage: scripts/r6_det.sh TAG "" SLAMHIP_SD_DOG=1 SLAMHIP_SD_REFINE_BLOCKS=8192
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests -m gpu -q -x -k "sift_detect" --timeout 200 --timeout-method thread \
    > $O/${TAG}_tests.log 2>&1 || { tail -20 $O/${TAG}_tests.log; exit 1; }
tail -1 $O/${TAG}_tests.log
for rep in 1 2; do
    for e in "$@"; do
        echo -n "[${e:-default}] "
        env $e REPS=10 timeout -k 10 200 python3 $R/scripts/diag/det_time.py 2>&1 | tail -1 || exit 1
    done
done
cd /tmp && export TMPDIR=/tmp
REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/${TAG}_kt -o run -- python3 $R/scripts/diag/det_time.py > $O/${TAG}_kt.log 2>&1 || exit 1
f=$(find $O/${TAG}_kt -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for x in csv.DictReader(open('$f')): print(x['Name'][:50], x['Calls'], round(float(x['AverageNs'])/1e3,1), round(float(x['TotalDurationNs'])/1e6, 3))"
