#!/bin/bash
# sd_desc_staged blocks in XCD-contiguous order (SLAMHIP_SD_DESC_XCD) A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
SLAMHIP_SD_DESC_XCD=1 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "sift_detect or detector" -p no:cacheprovider \
    --timeout 200 --timeout-method thread > $O/dx_tests.log 2>&1 || { echo "tests failed"; tail -20 $O/dx_tests.log; exit 1; }
echo "tests (xcd) $(tail -1 $O/dx_tests.log)"
for v in 0 1 0 1; do
    SLAMHIP_SD_DESC_XCD=$v REPS=8 timeout -k 10 200 python3 $R/scripts/diag/det_time.py 2>&1 | tail -1 | sed "s/^/desc xcd $v: /" || exit 1
done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
    SLAMHIP_SD_DESC_XCD=$v REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/dx_kt$v -o run -- python3 $R/scripts/diag/det_time.py > $O/dx_kt$v.log 2>&1 || exit 1
    grep sd_desc_staged $(find $O/dx_kt$v -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4 | sed "s/^/desc xcd $v: /"
done
