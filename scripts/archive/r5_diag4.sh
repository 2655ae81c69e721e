#!/bin/bash
# round-5: PnP alone (phases + kernel trace) and the 24-frame pipeline with the
# post-search / BA contexts at normal or high stream priority
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5d4}
mkdir -p $O
SLAMHIP_PNP_TIMING=1 timeout -k 10 120 python3 -u scripts/diag/pnp_iso.py > $O/${tag}_pnp.txt 2>&1 || { echo "pnp rc=$?"; tail -5 $O/${tag}_pnp.txt; exit 1; }
tail -3 $O/${tag}_pnp.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/${tag}_pnpkt -o run -- python3 $R/scripts/diag/pnp_iso.py > $O/${tag}_pnpkt.log 2>&1 || { echo "pnpkt rc=$?"; exit 1; }
cd $R
python3 - $(find $O/${tag}_pnpkt -name '*kernel_stats.csv' | head -1) <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    n = r["Name"].replace("slamhip::", "").replace("(anonymous namespace)::", "").replace("void ", "")
    print(f'{n.split("(")[0][:30]:30s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:8.1f}')
PY
for v in 0 1 0 1; do
    SLAMHIP_POST_PRIO=$v timeout -k 10 300 python3 -u scripts/diag/pipe24.py 2 > $O/${tag}_p24_$v.txt 2>&1 || { echo "p24 rc=$?"; exit 1; }
    echo "prio=$v $(grep frames_per_s $O/${tag}_p24_$v.txt | tail -1 | cut -c1-80)"
done
