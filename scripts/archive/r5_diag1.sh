#!/bin/bash
# round-5 diagnostics: the device timeline of the headline step at --batch 27
# (rocprofv3 kernel trace, scripts/diag/timeline.py) and the PnP phases of the
# 24-frame pipeline (SLAMHIP_PNP_TIMING=1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5d1}
mkdir -p $O
SLAMHIP_PNP_TIMING=1 timeout -k 10 300 python3 -u scripts/diag/pipe24.py 2 > $O/${tag}_pipe24.txt 2> $O/${tag}_pnp.txt \
    || { echo "pipe24 rc=$?"; tail -20 $O/${tag}_pnp.txt; exit 1; }
grep frames_per_s $O/${tag}_pipe24.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/${tag}_tl27 -o run -- python3 $R/bench.py --batch 27 --steps 20 \
    --warmup 3 --no-extra --no-cpu-baseline > $O/${tag}_tl27.log 2>&1 || { echo "tl27 rc=$?"; tail -5 $O/${tag}_tl27.log; exit 1; }
cd $R
python3 scripts/diag/timeline.py $(find $O/${tag}_tl27 -name '*kernel_trace.csv' | head -1) sift_desc_band 4
