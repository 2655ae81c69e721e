#!/bin/bash
# SQ counters of the kNN MFMA kernel (knn_mfma_pk), one pass per run
# usage: scripts/diag/knn_pmc.sh TAG
TAG=${1:-knnpmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
i=0
for pass in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-include-regex "knn_mfma" -f csv -d $R/gpurun_out/${TAG}_p$i -o run -- \
        python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $R/gpurun_out/${TAG}_p$i.log 2>&1
    rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
