#!/bin/bash
# A/B of the one-keypoint-per-lane SIFT kernel (sift_desc_cols, SLAMHIP_SIFT_COLS=1)
# against sift_desc_band: the SIFT parity subset under the new kernel, then a
# short headline bench each way with the per-family launch times.
set -o pipefail
TAG=${1:-r6cols}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
SLAMHIP_SIFT_COLS=1 timeout -k 10 300 python -u -m pytest $R/tests -m gpu -q -x -k "${TESTK:-sift or real or batch_pipeline or fused or 4k}" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
echo "cols tests rc=$rc $(tail -1 $R/gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 0 1 0 1; do
    SLAMHIP_SIFT_COLS=$v timeout -k 10 120 python3 $R/bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline \
        > $R/gpurun_out/${TAG}_b$v.json 2>$R/gpurun_out/${TAG}_b$v.err || exit $?
    python3 -c "
import json
d = json.loads(open('$R/gpurun_out/${TAG}_b$v.json').read().strip().splitlines()[-1])
k = d.get('kernels_sequential') or d['kernels']
print('cols=$v', 'step', round(d['ms_per_step'], 3), 'fps', round(d['value']), {n: round(x['avg_ms'], 4) for n, x in k.items()})"
done
