#!/bin/bash
# Round-2 GPU check: the -m gpu suite, then the bench (default run).
# usage: scripts/r2_gpu.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r2}
shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
tail -c 600 gpurun_out/${TAG}_bench.json
