#!/bin/bash
# round-5: chunked essential-matrix RANSAC -- parity, timing, the 24-frame pipeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5ep}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_cycle.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "transformation or essential or cycle" > $O/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -20 $O/${tag}_tests.log; exit 1; }
echo "tests $(tail -1 $O/${tag}_tests.log)"
timeout -k 10 200 python3 -u scripts/pnp_probe.py > $O/${tag}_probe.txt 2>&1 || { echo "probe rc=$?"; tail -5 $O/${tag}_probe.txt; exit 1; }
grep -v amdgpu.ids $O/${tag}_probe.txt
timeout -k 10 300 python3 -u scripts/diag/pipe24.py 3 > $O/${tag}_p24.txt 2>&1 || { echo "p24 rc=$?"; exit 1; }
grep '"frames_per_s"' $O/${tag}_p24.txt | cut -c1-60
grep -o '"estimate_transformation": [0-9.]*' $O/${tag}_p24.txt
