#!/bin/bash
# sd_refine (64 candidates per wave-step) grid A/B: detector parity, batch timing, kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "sift_detect or detector" -p no:cacheprovider --timeout 200 \
    --timeout-method thread > $O/r5ref_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/r5ref_tests.log; exit 1; }
echo "tests $(tail -1 $O/r5ref_tests.log)"
for g in 4096 2048 8192 4096; do
    SLAMHIP_SD_REFINE_GRID=$g REPS=8 timeout -k 10 200 python3 $R/scripts/diag/det_time.py 2>&1 | tail -1 | sed "s/^/grid $g: /" || exit 1
done
cd /tmp && export TMPDIR=/tmp
REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/r5ref_kt -o run -- python3 $R/scripts/diag/det_time.py > $O/r5ref_kt.log 2>&1 || exit 1
cut -d, -f1-4 $(find $O/r5ref_kt -name '*kernel_stats.csv' | head -1) | sed 's/slamhip::(anonymous namespace):://g' | cut -c1-100 | head -6
