#!/bin/bash
# detector pyramid blurs in XCD-contiguous tile order (SLAMHIP_SD_XCD) A/B:
# detector parity under it, batch timing, blur kernel time, FETCH_SIZE
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
SLAMHIP_SD_XCD=1 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "sift_detect or detector" -p no:cacheprovider \
    --timeout 200 --timeout-method thread > $O/sdx_tests.log 2>&1 || { echo "tests failed"; tail -20 $O/sdx_tests.log; exit 1; }
echo "tests (xcd) $(tail -1 $O/sdx_tests.log)"
for v in 0 1 0 1; do
    SLAMHIP_SD_XCD=$v REPS=8 timeout -k 10 200 python3 $R/scripts/diag/det_time.py 2>&1 | tail -1 | sed "s/^/xcd $v: /" || exit 1
done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
    SLAMHIP_SD_XCD=$v REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/sdx_kt$v -o run -- python3 $R/scripts/diag/det_time.py > $O/sdx_kt$v.log 2>&1 || exit 1
    python3 - $(find $O/sdx_kt$v -name '*kernel_stats.csv' | head -1) $v <<'PY'
import csv, sys
t = {}
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "sd_blur" in n or "sd_extrema" in n or "sd_desc" in n or "sd_refine" in n:
        key = n.split("(")[0].replace("void ", "").split("::")[-1]
        t[key] = t.get(key, 0) + float(r["TotalDurationNs"]) / 4e6
print("xcd", sys.argv[2], {k: round(v, 3) for k, v in sorted(t.items())}, "blur sum", round(sum(v for k, v in t.items() if "blur" in k), 3))
PY
    SLAMHIP_SD_XCD=$v REPS=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/sdx_f$v -o run -- python3 $R/scripts/diag/det_time.py > $O/sdx_f$v.log 2>&1 || exit 1
    python3 - $(find $O/sdx_f$v -name '*counter_collection.csv' | head -1) $v <<'PY'
import csv, sys
tot = 0.0
for r in csv.DictReader(open(sys.argv[1])):
    if "sd_blur" in r["Kernel_Name"]:
        tot += float(r["Counter_Value"])
print("xcd", sys.argv[2], "blur FETCH GB per call (x2 corr, 2 calls)", round(tot * 1024 * 2 / 1e9 / 2, 3))
PY
done
