#!/bin/bash
# timing probes of the staged detector descriptor: full / no walk / no eval / neither
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5detdbg}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cpl in ${CPLS:-1 2}; do
for d in ${DBGS:-0 1 2 3}; do
    SLAMHIP_SD_CPL=$cpl SLAMHIP_SD_DBG=$d REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/${tag}_$cpl$d -o run \
        -- python3 $R/scripts/diag/det_time.py > $O/${tag}_$cpl$d.log 2>&1 || { echo "kt $d failed"; exit 1; }
    f=$(find $O/${tag}_$cpl$d -name '*kernel_stats.csv' | head -1)
    echo "cpl $cpl dbg $d: $(grep -E "sd_desc" $f | cut -d, -f4 | cut -c1-12)"
done
done
