#!/bin/bash
# fused extract+match check: full GPU suite, then the bench both ways
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r1s5c_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r1s5c_pytest.log; exit 1; }
tail -2 gpurun_out/r1s5c_pytest.log
for v in fused two; do
    a=""; [ $v = two ] && a="--two-call"
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra $a > gpurun_out/r1s5c_$v.json 2> gpurun_out/r1s5c_$v.err || exit 2
done
python - <<'PY'
import json
for t in ("fused", "two"):
    for line in open(f"gpurun_out/r1s5c_{t}.json"):
        if line.startswith("{"):
            d = json.loads(line)
            print(t, round(d["value"], 1), round(d["ms_per_step"], 3), {k: round(v["avg_ms"], 3) for k, v in d.get("kernels", {}).items()})
PY
