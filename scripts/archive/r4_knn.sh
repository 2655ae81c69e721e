#!/bin/bash
# round-4 kNN check: parity of the matcher paths, then the headline step with the
# pipelined L2 kernel on and off (SLAMHIP_KNN_PIPE), and the LDS scatter microbenchmark
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r4knn}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "knn or batch or configs4 or pipelined or fused or rematch or sharded" > gpurun_out/${tag}_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
for pipe in 1 0; do
    SLAMHIP_KNN_PIPE=$pipe timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline \
        > gpurun_out/${tag}_bench_pipe${pipe}.json 2> gpurun_out/${tag}_bench_pipe${pipe}.err \
        || { echo "bench pipe=$pipe rc=$?"; tail -c 1500 gpurun_out/${tag}_bench_pipe${pipe}.err; exit 1; }
    python3 - gpurun_out/${tag}_bench_pipe${pipe}.json <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("kernels_sequential") or d["kernels"]
print(sys.argv[1], "value", round(d["value"]), "ms", round(d["ms_per_step"], 3), "mean_kps", round(d["config"]["mean_kps"]),
      "prev", d["config"]["prev_kps"], {k: round(v["avg_ms"], 3) for k, v in ks.items()},
      "knn_frac", round(d["rooflines"]["knn_mfma"]["frac"], 3))
EOF
done
timeout -k 10 120 ./scripts/diag/lds_add_bench > gpurun_out/${tag}_lds_add.txt 2>&1 || echo "lds bench rc=$?"
cat gpurun_out/${tag}_lds_add.txt
