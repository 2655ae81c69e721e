#!/bin/bash
# subset parity + headline bench (no extra legs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "${1:-knn or batch or match}" > gpurun_out/r1s5f_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r1s5f_pytest.log; exit 1; }
tail -2 gpurun_out/r1s5f_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/r1s5f_bench.json 2>/dev/null || exit 2
python - <<'PY'
import json
for line in open("gpurun_out/r1s5f_bench.json"):
    if line.startswith("{"):
        d = json.loads(line)
print(round(d["value"], 1), round(d["ms_per_step"], 3), {k: round(v["avg_ms"], 3) for k, v in d["kernels"].items()})
PY
