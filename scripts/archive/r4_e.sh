#!/bin/bash
# round-4: SIFT band kernel with the slot-position plane (default) vs obin
# (SLAMHIP_SIFT_POSPLANE=0): SIFT parity cases, then the headline step each way
set -o pipefail
tag=${1:-r4e}
mkdir -p gpurun_out
K="sift or tiny or uniform or real or configs4 or batch or pipelined or fused or cycle"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_real_images.py -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/${tag}_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
SLAMHIP_SIFT_POSPLANE=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "sift_1080p or sift_vga or tiny or uniform" > gpurun_out/${tag}_tests_p0.log 2>&1 \
    || { echo "plane=0 tests failed"; tail -30 gpurun_out/${tag}_tests_p0.log; exit 1; }
tail -1 gpurun_out/${tag}_tests_p0.log
summ() {
    python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("kernels_sequential") or d["kernels"]
print(sys.argv[1].split("/")[-1], "value", round(d["value"]), "ms", round(d["ms_per_step"], 3),
      {k: round(v["avg_ms"], 3) for k, v in ks.items()}, {k: round(v["frac"], 3) for k, v in d["rooflines"].items()})
PY
}
for pl in 1 0; do
    SLAMHIP_SIFT_POSPLANE=$pl timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline \
        > gpurun_out/${tag}_plane$pl.json 2> gpurun_out/${tag}_plane$pl.err || { echo "bench plane=$pl rc=$?"; tail -c 1500 gpurun_out/${tag}_plane$pl.err; exit 1; }
    summ gpurun_out/${tag}_plane$pl.json
done
