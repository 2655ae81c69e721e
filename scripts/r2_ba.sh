#!/bin/bash
# BA: GPU parity tests, then timings and a kernel trace of W = 8 / W = 16
set -o pipefail
TAG=${1:-ba}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -v -k "ba or cycle" --maxfail=5 --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -8 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 60 python scripts/ba_bench.py 8 10000 > gpurun_out/${TAG}_w8.json || exit $?
timeout -k 10 60 python scripts/ba_bench.py 16 40000 4k > gpurun_out/${TAG}_w16.json || exit $?
cat gpurun_out/${TAG}_w8.json gpurun_out/${TAG}_w16.json
bash scripts/ba_prof.sh ${TAG}p
