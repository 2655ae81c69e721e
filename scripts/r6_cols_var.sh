#!/bin/bash
# sift_desc_cols build variants (scripts/diag/lib_sift_<v>.so, SRC=sift_cols.hip):
# a SIFT parity subset under ENVV (default SLAMHIP_SIFT_COLS=1), then a short bench each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cp $R/slam-indoor-code_amd/slamhip/libslamhip.so /tmp/lib_base.so
for v in "$@"; do
    if [ "$v" = base ]; then cp /tmp/lib_base.so $R/slam-indoor-code_amd/slamhip/libslamhip.so
    else cp $R/scripts/diag/lib_sift_$v.so $R/slam-indoor-code_amd/slamhip/libslamhip.so || exit 1; fi
    env ${ENVV:-SLAMHIP_SIFT_COLS=1} timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -q -x -k "${TESTK:-sift_1080p or sift_vga or batch_pipeline_sift}" \
        --timeout 200 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/cv_$v.log 2>&1
    rc=$?
    echo "$v tests rc=$rc $(tail -1 $R/gpurun_out/cv_$v.log)"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
    env ${ENVV:-SLAMHIP_SIFT_COLS=1} timeout -k 10 120 python3 $R/bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline > $R/gpurun_out/cv_$v.json 2>$R/gpurun_out/cv_$v.err || exit $?
    python3 -c "
import json
d = json.loads(open('$R/gpurun_out/cv_$v.json').read().strip().splitlines()[-1])
k = d.get('kernels_sequential') or d['kernels']
print('$v', 'step', round(d['ms_per_step'], 3), 'sift', round(k['sift_desc']['avg_ms'], 3))"
done
cp /tmp/lib_base.so $R/slam-indoor-code_amd/slamhip/libslamhip.so
