#!/bin/bash
# round-4: the tree's GPU tests touched since r4b (batch detector with device
# outputs, pipeline / BA envelope), the full bench line, then timing variants
# (scripts/diag/lib_sift_*.so swapped in: base, blur row stride 80, kNN 128-row tiles)
set -o pipefail
tag=${1:-r4c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cycle.py -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "sift_detect or cycle or knn or fused or rematch" > gpurun_out/${tag}_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
    || { echo "bench rc=$?"; tail -c 2000 gpurun_out/${tag}_bench.err; exit 1; }
python3 - gpurun_out/${tag}_bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms", round(d["ms_per_step"], 3))
for leg in ("pipeline_b210", "pipeline_b210_orb"):
    v = d[leg]
    print(leg, round(v["frames_per_s"]), v["parity_ok"], [(c["ok"], round(c["final_cost_rel_diff"], 9), (c.get("envelope") or {}).get("orders")) for c in v["ba_window_checks"]])
print("detector", json.dumps(d["sift_detector"]["batch"]))
PY
TESTK="sift_1080p or sift_vga or batch_pipeline_sift or knn_sift" bash scripts/diag/sift_variant_check.sh base blur80 knn128
