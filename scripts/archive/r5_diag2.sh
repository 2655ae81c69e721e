#!/bin/bash
# round-5 diagnostics: kernel durations of the 24-frame pipeline (PnP, BA,
# triangulation kernels) from a rocprofv3 kernel trace + stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5d2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SLAMHIP_PNP_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/${tag}_p24 -o run -- \
    python3 $R/scripts/diag/pipe24.py 1 > $O/${tag}_p24.log 2>&1 || { echo "p24 rc=$?"; tail -5 $O/${tag}_p24.log; exit 1; }
cd $R
f=$(find $O/${tag}_p24 -name '*kernel_stats.csv' | head -1)
python3 - $f <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:40]:
    n = r["Name"].replace("slamhip::", "").replace("(anonymous namespace)::", "").replace("void ", "")
    print(f'{n.split("(")[0][:40]:40s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:9.1f} total_ms {float(r["TotalDurationNs"])/1e6:8.2f}')
PY
timeout -k 10 300 python3 -u scripts/diag/pipe_timeline.py 2 > $O/${tag}_ptl.txt 2>&1 || { echo "ptl rc=$?"; tail -5 $O/${tag}_ptl.txt; exit 1; }
head -40 $O/${tag}_ptl.txt
