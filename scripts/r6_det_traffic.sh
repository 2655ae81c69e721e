#!/bin/bash
# HBM traffic of the batch detector's kernels (scripts/diag/det_time.py, REPS=1):
# one FETCH_SIZE pass and one WRITE_SIZE pass, summed per kernel and per call
set -o pipefail
TAG=${1:-r6dtr}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
    REPS=1 timeout -s KILL 200 rocprofv3 --pmc $c -f csv -d $O/${TAG}_$c -o run -- python3 $R/scripts/diag/det_time.py \
        > $O/${TAG}_$c.log 2>&1 || { echo "$c pass failed"; exit 1; }
done
python3 - <<PY
import csv, glob, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob("$O/${TAG}_" + c + "/**/*counter_collection.csv", recursive=True)[0]
    tot = collections.defaultdict(float); calls = collections.Counter()
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("slamhip::(anonymous namespace)::", "")
        tot[n] += float(r["Counter_Value"]); calls[n] += 1
    # 2 calls (warm-up + 1 timed): per call = half; KB -> GB
    print(c, {k: round(v / 2 / 1e6, 3) for k, v in sorted(tot.items(), key=lambda x: -x[1]) if v > 1e4}, "GB per 16-frame call")
PY
