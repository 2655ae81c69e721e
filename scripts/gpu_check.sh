#!/bin/bash
# GPU box check: parity tests, then a short bench.  Stops at the first step that
# crashed, aborted or timed out (never retries a GPU step).
# usage: scripts/gpu_check.sh TAG [pytest -k expr]
TAG=${1:-run}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider "${KARG[@]}" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/${TAG}_pytest.log
if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc2=$?
echo "pytest $rc bench $rc2"
exit $rc2
