#!/bin/bash
# round-5 detector descriptor A/B: sd_desc (SLAMHIP_SD_DESC=0) against the
# staged form at 1 / 2 / 4 rows per strip -- the detector parity tests under
# each, the batch detector's frames/s, and a kernel trace of each form
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5det}
mkdir -p $O
for v in "0 1 1" "1 1 1" "1 1 2"; do
    set -- $v
    export SLAMHIP_SD_DESC=$1 SLAMHIP_SD_STRIP=$2 SLAMHIP_SD_CPL=$3
    timeout -k 10 300 python -u -m pytest $R/tests -m gpu -q -x -k "sift_detect or detector" -p no:cacheprovider \
        --timeout 200 --timeout-method thread > $O/${tag}_$1_$2_$3.log 2>&1
    rc=$?
    echo "form $1 strip $2 cpl $3 tests rc=$rc $(tail -1 $O/${tag}_$1_$2_$3.log)"
    [ $rc -eq 0 ] || { tail -30 $O/${tag}_$1_$2_$3.log; exit 1; }
    timeout -k 10 200 python3 $R/scripts/diag/det_time.py 2>&1 | tail -1 || exit 1
done
export SLAMHIP_SD_DESC=0
timeout -k 10 200 python3 $R/scripts/diag/det_time.py 2>&1 | tail -1 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
    SLAMHIP_SD_CPL=2 SLAMHIP_SD_DESC=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/${tag}_kt$v -o run \
        -- python3 $R/scripts/diag/det_time.py > $O/${tag}_kt$v.log 2>&1 || { echo "kt $v failed"; exit 1; }
    f=$(find $O/${tag}_kt$v -name '*kernel_stats.csv' | head -1)
    grep -E "sd_desc|sd_refine|sd_extrema" $f | cut -c1-160
done
