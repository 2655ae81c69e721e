#!/bin/bash
# SQ issue / stall / LDS counters of the SIFT descriptor band kernel, one pass per run
# usage: scripts/diag/sift_pmc.sh TAG
TAG=${1:-siftpmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_DATA_FIFO_FULL GRBM_GUI_ACTIVE"
P2="SQ_LDS_CMD_FIFO_FULL SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
i=0
for pass in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "sift_desc" -f csv -d $R/gpurun_out/${TAG}_p$i -o run -- \
        python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $R/gpurun_out/${TAG}_p$i.log 2>&1
    rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
