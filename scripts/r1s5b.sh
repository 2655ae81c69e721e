#!/bin/bash
# PnP / pipeline check: parity tests of the touched paths, then the bench legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "${1:-pnp or cycle or pipeline}" > gpurun_out/r1s5b_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r1s5b_pytest.log; exit 1; }
tail -2 gpurun_out/r1s5b_pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r1s5b_bench.json 2> gpurun_out/r1s5b_bench.err || exit 2
python - <<'PY'
import json
for line in open("gpurun_out/r1s5b_bench.json"):
    if line.startswith("{"):
        d = json.loads(line)
print("value", round(d["value"], 1), "pipeline", round(d["pipeline"]["frames_per_s"], 1), d["pipeline"]["ms_by_op"])
PY
