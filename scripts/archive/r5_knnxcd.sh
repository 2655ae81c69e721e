#!/bin/bash
# knn_mfma_pk blocks in XCD-contiguous order (SLAMHIP_KNN_XCD) A/B: parity, step, FETCH
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
SLAMHIP_KNN_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "knn or configs4 or batch_extract_match or match or pipelined" > $O/kx_tests.log 2>&1 || { echo "tests failed"; tail -20 $O/kx_tests.log; exit 1; }
echo "tests (xcd) $(tail -1 $O/kx_tests.log)"
for b in 210 27; do
for v in 0 1 0 1; do
    SLAMHIP_KNN_XCD=$v timeout -k 10 200 python -u bench.py --batch $b --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $O/kx_$v.json 2>$O/kx.err || exit 1
    python3 -c "
import json
d=json.loads(open('$O/kx_$v.json').read().strip().splitlines()[-1])
ks=d.get('kernels_sequential') or d['kernels']
print('batch $b knn xcd $v', round(d['value']), round(d['ms_per_step'],3), 'knn', round(ks['knn_mfma']['avg_ms'],3))
"
done
done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
    SLAMHIP_KNN_XCD=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex knn_mfma -f csv -d $O/kx_f$v -o run -- python3 $R/bench.py --no-extra --no-cpu-baseline --steps 3 --warmup 1 > $O/kx_f$v.log 2>&1 || exit 1
    python3 - $(find $O/kx_f$v -name '*counter_collection.csv' | head -1) $v <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if "knn_mfma" in r["Kernel_Name"]]
print("knn xcd", sys.argv[2], "FETCH GB per launch", round(sum(v) / max(1, len(v)) * 1024 * 2 / 1e9, 3))
PY
done
