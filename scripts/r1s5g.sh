#!/bin/bash
# kNN occupancy sweep (SLAMHIP_KNN_MINB), parity under the fastest
set -o pipefail
mkdir -p gpurun_out
for m in 3 4 2; do
    SLAMHIP_KNN_MINB=$m timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/r1s5g_m$m.json 2>/dev/null || exit 2
done
SLAMHIP_KNN_MINB=4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "knn or batch or match" > gpurun_out/r1s5g_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r1s5g_pytest.log; exit 1; }
tail -1 gpurun_out/r1s5g_pytest.log
python - <<'PY'
import json
for m in (3, 4, 2):
    for line in open(f"gpurun_out/r1s5g_m{m}.json"):
        if line.startswith("{"):
            d = json.loads(line)
    print(m, round(d["value"], 1), round(d["ms_per_step"], 3), {k: round(v["avg_ms"], 3) for k, v in d["kernels"].items()})
PY
