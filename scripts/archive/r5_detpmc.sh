#!/bin/bash
# SQ counter passes over the batch detector's descriptor kernels (both forms)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5detpmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
for v in 0 1; do
  i=0
  for pass in "$P1" "$P2"; do
    i=$((i+1))
    SLAMHIP_SD_CPL=${CPL:-1} SLAMHIP_SD_DESC=$v REPS=1 timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "sd_desc" -f csv -d $O/${tag}_${v}_p$i -o run -- \
        python3 $R/scripts/diag/det_time.py > $O/${tag}_${v}_p$i.log 2>&1 || { echo "pass $v $i failed"; exit 1; }
  done
done
cd $R
python3 - $O $tag <<'PY'
import csv, glob, sys
from collections import defaultdict
O, tag = sys.argv[1:]
for v in "01":
    tot = defaultdict(float)
    for f in glob.glob(f"{O}/{tag}_{v}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print("form", v, {k: f"{x:.4g}" for k, x in sorted(tot.items())})
PY
