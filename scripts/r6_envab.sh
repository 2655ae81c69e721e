#!/bin/bash
# Environment A/B of the headline step: TESTENV's SIFT parity subset first (if
# set), then a short bench per environment string, each run twice interleaved.
# usage: TESTENV="SLAMHIP_X=1" scripts/r6_envab.sh TAG "A=0" "A=1" ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
if [ -n "$TESTENV" ]; then
    env $TESTENV timeout -k 10 300 python -u -m pytest $R/tests -m gpu -q -x -k "${TESTK:-sift or real or batch_pipeline or fused or 4k}" \
        --timeout 200 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/${TAG}_pytest.log 2>&1
    rc=$?
    echo "tests ($TESTENV) rc=$rc $(tail -1 $R/gpurun_out/${TAG}_pytest.log)"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
i=0
for rep in 1 2; do
    for e in "$@"; do
        i=$((i+1))
        env $e timeout -k 10 120 python3 $R/bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline ${BENCHARGS} \
            > $R/gpurun_out/${TAG}_$i.json 2>$R/gpurun_out/${TAG}_$i.err || exit $?
        python3 -c "
import json
d = json.loads(open('$R/gpurun_out/${TAG}_$i.json').read().strip().splitlines()[-1])
k = d.get('kernels_sequential') or d['kernels']
print('$e', 'step', round(d['ms_per_step'], 3), 'fps', round(d['value']), {n: round(x['avg_ms'], 4) for n, x in k.items()})"
    done
done
