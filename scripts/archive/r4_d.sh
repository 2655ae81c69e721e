#!/bin/bash
# round-4: the walk microbenchmark, the matcher parity tests, the headline step
set -o pipefail
tag=${1:-r4d}
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/diag/lds_walk_bench > gpurun_out/${tag}_walk.txt 2>&1 || echo "walk bench rc=$?"
grep "rep 2" gpurun_out/${tag}_walk.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_real_images.py -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "knn or match or batch or fused or rematch or sharded or pipelined" > gpurun_out/${tag}_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/${tag}_bench.json \
    2> gpurun_out/${tag}_bench.err || { echo "bench rc=$?"; tail -c 1500 gpurun_out/${tag}_bench.err; exit 1; }
python3 - gpurun_out/${tag}_bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("kernels_sequential") or d["kernels"]
print("value", round(d["value"]), "ms", round(d["ms_per_step"], 3), {k: round(v["avg_ms"], 3) for k, v in ks.items()},
      {k: round(v["frac"], 3) for k, v in d["rooflines"].items()})
PY
