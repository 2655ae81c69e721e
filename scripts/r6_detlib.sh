#!/bin/bash
# Detector library A/B: per variant (base = the in-tree build, else
# scripts/diag/lib_sift_<name>.so) the detector parity tests, then the 16-frame
# batch timing (interleaved, twice), then one kernel trace per variant.
# usage: scripts/r6_detlib.sh TAG base sdu2 sdu3
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
    timeout -k 10 300 python -u -m pytest $R/tests -m gpu -q -x -k "sift_detect" --timeout 200 --timeout-method thread \
        > $O/${TAG}_${v}_tests.log 2>&1 || { tail -20 $O/${TAG}_${v}_tests.log; fail; }
    echo "$v: $(tail -1 $O/${TAG}_${v}_tests.log)"
done
for rep in 1 2; do
    for v in "$@"; do
        use $v || fail
        echo -n "[$v] "
        REPS=10 timeout -k 10 200 python3 $R/scripts/diag/det_time.py 2>&1 | tail -1 || fail
    done
done
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
    use $v || fail
    REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/${TAG}_${v}_kt -o run -- python3 $R/scripts/diag/det_time.py > $O/${TAG}_${v}_kt.log 2>&1 || fail
    f=$(find $O/${TAG}_${v}_kt -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv
r = [(x['Name'].split('(')[0].split('::')[-1], float(x['AverageNs']) / 1e3, float(x['TotalDurationNs']) / 3e6) for x in csv.DictReader(open('$f'))]
print('$v', ' '.join(f'{n}:{a:.0f}us/{t:.2f}ms' for n, a, t in r[:8]))"
done
cp /tmp/lib_base.so $LIB
