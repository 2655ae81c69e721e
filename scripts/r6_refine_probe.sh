#!/bin/bash
# sd_refine's time split: the -DSLAMHIP_DIAG build (scripts/diag/lib_sift_sddiag.so)
# under each SLAMHIP_SD_REFINE_DBG probe, one kernel trace each (REPS=2)
set -o pipefail
TAG=${1:-r6rp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
LIB=$R/slam-indoor-code_amd/slamhip/libslamhip.so
cp $LIB /tmp/lib_base.so
cp $R/scripts/diag/lib_sift_${VAR:-sddiag}.so $LIB || exit 1
cd /tmp && export TMPDIR=/tmp
for d in ${DBGS:-0 1 2 3 4}; do
    SLAMHIP_SD_REFINE_DBG=$d REPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/${TAG}_$d -o run -- \
        python3 $R/scripts/diag/det_time.py > $O/${TAG}_$d.log 2>&1 || { cp /tmp/lib_base.so $LIB; exit 1; }
    f=$(find $O/${TAG}_$d -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv
r = {x['Name'].split('(')[0].split('::')[-1]: float(x['AverageNs']) / 1e3 for x in csv.DictReader(open('$f'))}
print('dbg $d', {k: round(v, 1) for k, v in r.items() if 'refine' in k or 'desc' in k})"
done
cp /tmp/lib_base.so $LIB
