#!/bin/bash
# kernel trace of the fused step + kNN split sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r1s5d_kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra > $R/gpurun_out/r1s5d_kt.log 2>&1 || exit 1
cd $R
for t in 10 14 20 30; do
    SLAMHIP_KNN_TSPLIT=$t timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/r1s5d_t$t.json 2>/dev/null || exit 2
done
python - <<'PY'
import json
for t in (10, 14, 20, 30):
    for line in open(f"gpurun_out/r1s5d_t{t}.json"):
        if line.startswith("{"):
            d = json.loads(line)
            print(t, round(d["value"], 1), round(d["ms_per_step"], 3), {k: round(v["avg_ms"], 3) for k, v in d.get("kernels", {}).items()})
PY
