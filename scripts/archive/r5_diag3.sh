#!/bin/bash
# round-5: FAST reuse parity + pipeline_b210 with / without it; detector sorted
# descriptor launch A/B; pipeline timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5d3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "reuses_fast or band_split or batch_pipeline or sift_detect" > $O/${tag}_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 $O/${tag}_tests.log; exit 1; }
echo "tests $(tail -1 $O/${tag}_tests.log)"
for v in 0 1 0 1; do
    SLAMHIP_SD_SORT=$v timeout -k 10 200 python3 -u scripts/diag/det_time.py > $O/${tag}_det_$v.txt 2>&1 \
        || { echo "det rc=$?"; tail -5 $O/${tag}_det_$v.txt; exit 1; }
    echo "sd_sort=$v $(tail -1 $O/${tag}_det_$v.txt)"
done
for v in 0 1; do
    SLAMHIP_FAST_REUSE=$v timeout -k 10 300 python3 -u scripts/diag/pipe_b210.py > $O/${tag}_b210_$v.txt 2>&1 \
        || { echo "b210 rc=$?"; tail -5 $O/${tag}_b210_$v.txt; exit 1; }
    echo "reuse=$v $(tail -1 $O/${tag}_b210_$v.txt)"
done
timeout -k 10 300 python3 -u scripts/diag/pipe_timeline.py 2 > $O/${tag}_ptl.txt 2>&1 || { echo "ptl rc=$?"; tail -5 $O/${tag}_ptl.txt; exit 1; }
head -30 $O/${tag}_ptl.txt
