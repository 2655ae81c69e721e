#!/bin/bash
# SIFT descriptor kernel: GPU parity (every SIFT test), then a short bench with kernel timings
set -o pipefail
TAG=${1:-sift}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v -k "sift or batch or real or smoke" --maxfail=5 --timeout 200 \
    --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
python3 - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_bench.json").read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3))
for k, v in d["kernels"].items(): print(k, round(v["avg_ms"], 4))
PY
