#!/bin/bash
# SIFT descriptor kernels: GPU parity (every SIFT test), then short benches of
# each FAST-keypoint kernel with kernel timings
set -o pipefail
TAG=${1:-sift}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v -k "sift or batch or real or smoke" --maxfail=5 --timeout 200 \
    --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
for k in pair band; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline --sift-kernel $k \
        > gpurun_out/${TAG}_bench_$k.json 2> gpurun_out/${TAG}_bench_$k.err || exit $?
    python3 - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_bench_$k.json").read().strip().splitlines()[-1])
print("$k", "value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3),
      {k: round(v["avg_ms"], 4) for k, v in d["kernels"].items()})
PY
done
