#!/bin/bash
# ORB A/B: per variant (base = the in-tree build, else scripts/diag/lib_sift_<name>.so)
# the ORB parity tests, then scripts/diag/orb_pipe.py twice (interleaved), then
# one kernel trace of orb_pipe.py per variant
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
LIB=$R/slam-indoor-code_amd/slamhip/libslamhip.so
cp $LIB /tmp/lib_base.so
use() { if [ "$1" = base ]; then cp /tmp/lib_base.so $LIB; else cp $R/scripts/diag/lib_sift_$1.so $LIB; fi; }
fail() { cp /tmp/lib_base.so $LIB; exit 1; }
for v in "$@"; do
    use $v || fail
    timeout -k 10 300 python -u -m pytest $R/tests -m gpu -q -x -k "orb" --timeout 200 --timeout-method thread \
        > $O/${TAG}_${v}_tests.log 2>&1 || { tail -20 $O/${TAG}_${v}_tests.log; fail; }
    echo "$v: $(tail -1 $O/${TAG}_${v}_tests.log)"
done
for rep in 1 2; do
    for v in "$@"; do
        use $v || fail
        echo "[$v]"
        timeout -k 10 200 python3 $R/scripts/diag/orb_pipe.py 2>&1 | tail -4 || fail
    done
done
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
    use $v || fail
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/${TAG}_${v}_kt -o run -- python3 $R/scripts/diag/orb_pipe.py > $O/${TAG}_${v}_kt.log 2>&1 || fail
    f=$(find $O/${TAG}_${v}_kt -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv
for x in csv.DictReader(open('$f')):
    if 'orb' in x['Name']: print('$v', x['Name'].split('(')[0][-30:], x['Calls'], round(float(x['AverageNs']) / 1e3, 1), 'us')"
done
cp /tmp/lib_base.so $LIB
