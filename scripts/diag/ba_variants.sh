#!/bin/bash
# BA kernel timing of compile-time variants of ba.hip (-DBA_DIAG=k): each
# variant's library goes into its own copy of the package under /tmp.
# Timing only: variants skip work and give wrong results.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
    D=/tmp/bav_$v
    rm -rf $D && mkdir -p $D && cp -r $R/slam-indoor-code_amd/slamhip $D/
    cp $R/scripts/diag/lib_diag_$v.so $D/slamhip/libslamhip.so
    sed "s#sys.path.insert(0, os.path.join(ROOT, \"slam-indoor-code_amd\"))#sys.path.insert(0, \"$D\")#" $R/scripts/ba_bench.py > $D/ba_bench.py
    timeout -k 5 90 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/bav_$v -o run -- python3 $D/ba_bench.py 8 10000 > $R/gpurun_out/bav_$v.log 2>&1 || exit $?
    echo "variant $v"; grep '^{' $R/gpurun_out/bav_$v.log
    python3 - <<PY
import csv
r=list(csv.DictReader(open('$R/gpurun_out/bav_$v/run_kernel_stats.csv')))
for x in r[:5]: print(x['Name'][30:70], x['Calls'], round(float(x['AverageNs'])/1e3,2))
PY
done
