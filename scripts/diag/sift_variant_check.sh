#!/bin/bash
# Each variant library (scripts/diag/lib_sift_<v>.so) swapped into the box's
# scratch copy of the package: the SIFT parity tests, then a short bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for v in "$@"; do
    cp $R/scripts/diag/lib_sift_$v.so $R/slam-indoor-code_amd/slamhip/libslamhip.so || exit 1
    timeout -k 10 300 python -u -m pytest $R/tests -m gpu -q -x -k "${TESTK:-sift_1080p or sift_vga or 4k_batch or real_sift or batch_pipeline_sift}" \
        --timeout 200 --timeout-method thread > $R/gpurun_out/svc_$v.log 2>&1
    rc=$?
    echo "$v tests rc=$rc $(tail -1 $R/gpurun_out/svc_$v.log)"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
    timeout -k 10 120 python3 $R/bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline > $R/gpurun_out/svc_$v.json 2>$R/gpurun_out/svc_$v.err || exit $?
    python3 -c "
import json
d = json.loads(open('$R/gpurun_out/svc_$v.json').read().strip().splitlines()[-1])
k = d.get('kernels_sequential') or d['kernels']
print('$v', 'step', round(d['ms_per_step'], 3), {n: round(x['avg_ms'], 4) for n, x in k.items()})"
done
