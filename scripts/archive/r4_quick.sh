#!/bin/bash
# round-4 quick GPU check: LDS microbenchmark, headline bench, the GPU tests touched this round
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r4}
timeout -k 10 120 ./scripts/diag/lds_add_bench > gpurun_out/${tag}_lds_add.txt 2>&1 || echo "lds bench rc=$?"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-extra > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench rc=$?"; tail -c 1500 gpurun_out/${tag}_bench.err; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "tiny_uniform or async_rematch or waits_for_torch or tukey_bench or pipelined_scan or fused" > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${tag}_tests.log
exit $rc
