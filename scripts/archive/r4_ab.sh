#!/bin/bash
# round-4 A/B check: parity of the SIFT / matcher paths with the new kernels, then
# the headline step with each new kernel on and off (SLAMHIP_SIFT_BAND4,
# SLAMHIP_KNN_PIPE; same results either way), and the LDS scatter microbenchmark
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r4ab}
K=${2:-"sift or knn or batch or configs4 or pipelined or fused or rematch or sharded or real"}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_real_images.py -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/${tag}_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
# the register-staged 16-keypoint kernel and the 32-keypoint one on the SIFT parity cases
for m in 1 0; do
    SLAMHIP_SIFT_BAND4=$m timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_real_images.py -x -q \
        --timeout 300 --timeout-method thread -p no:cacheprovider -k "sift_1080p or sift_vga or tiny or uniform or real or configs4" \
        > gpurun_out/${tag}_tests_band4_$m.log 2>&1 || { echo "band4=$m tests failed"; tail -30 gpurun_out/${tag}_tests_band4_$m.log; exit 1; }
    tail -1 gpurun_out/${tag}_tests_band4_$m.log
done
summ() {
    python3 - "$1" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("kernels_sequential") or d["kernels"]
c = d["config"]
print(sys.argv[1].split("/")[-1], "value", round(d["value"]), "ms", round(d["ms_per_step"], 3), "kps", round(c["mean_kps"]),
      c["min_kps"], c["max_kps"], "prev", c["prev_kps"], {k: round(v["avg_ms"], 3) for k, v in ks.items()},
      {k: round(v["frac"], 3) for k, v in d["rooflines"].items()})
EOF
}
for cfg in "2 1" "1 1" "0 1" "2 0"; do
    set -- $cfg
    name=b4_$1_pipe_$2
    SLAMHIP_SIFT_BAND4=$1 SLAMHIP_KNN_PIPE=$2 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-extra \
        --no-cpu-baseline > gpurun_out/${tag}_${name}.json 2> gpurun_out/${tag}_${name}.err \
        || { echo "bench $name rc=$?"; tail -c 1500 gpurun_out/${tag}_${name}.err; exit 1; }
    summ gpurun_out/${tag}_${name}.json
done
if [ -x scripts/diag/lds_add_bench ]; then
    timeout -k 10 120 ./scripts/diag/lds_add_bench > gpurun_out/${tag}_lds_add.txt 2>&1 || echo "lds bench rc=$?"
    cat gpurun_out/${tag}_lds_add.txt
fi
