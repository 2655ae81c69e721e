#!/bin/bash
# the in-tree library: the SIFT parity subset, then a short headline bench (sift kernel as given, default auto)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
TAG=${1:-sc}; K=${2:-auto}
timeout -k 10 300 python -u -m pytest $R/tests -m gpu -q -x -k "${TESTK:-sift_1080p or sift_vga or 4k_batch or real_sift or batch_pipeline_sift or forced_sift}" \
    --timeout 200 --timeout-method thread > $R/gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 $R/gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || { grep -E "Error|error|assert" $R/gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
for k in $K; do
timeout -k 10 120 python3 $R/bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline --sift-kernel $k > $R/gpurun_out/${TAG}_$k.json 2>$R/gpurun_out/${TAG}_$k.err || exit $?
python3 -c "
import json
d = json.loads(open('$R/gpurun_out/${TAG}_$k.json').read().strip().splitlines()[-1])
print('$k', 'sift_desc', round(d['kernels']['sift_desc']['avg_ms'], 4), 'step', round(d['ms_per_step'], 3), 'value', round(d['value']))"
done
