#!/bin/bash
# Round 6 measurements beside the A/Bs: the strong-scaling shard (--batch 27)
# with sift_desc_colw (AUTO) and sift_desc_band (SLAMHIP_SIFT_COLW=0), and one
# SQ pass over fast_detect (LDS bank conflicts after the 18-group prefilter rows).
set -o pipefail
TAG=${1:-r6misc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for rep in 1 2; do
    for e in "SLAMHIP_SIFT_COLW=1" "SLAMHIP_SIFT_COLW=0"; do
        env $e timeout -k 10 120 python3 $R/bench.py --batch 27 --steps 60 --warmup 5 --no-extra --no-cpu-baseline \
            > $O/${TAG}_b27_${e##*=}_$rep.json 2> $O/${TAG}_b27_${e##*=}_$rep.err || exit $?
        python3 -c "
import json
d = json.loads(open('$O/${TAG}_b27_${e##*=}_$rep.json').read().strip().splitlines()[-1])
k = d.get('kernels_sequential') or d['kernels']
print('b27 $e', 'step', round(d['ms_per_step'], 3), 'fps', round(d['value']), {n: round(x['avg_ms'], 4) for n, x in k.items()})"
    done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-include-regex "fast_detect" -f csv -d $O/${TAG}_fastpmc -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $O/${TAG}_fastpmc.log 2>&1
rc=$?; echo "fast pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 $R/scripts/diag/pmc_sum.py fast_detect $O/${TAG}_fastpmc
