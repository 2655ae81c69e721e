#!/bin/bash
# round-5 A/B: XCD-contiguous tile order in fast_detect / sift_blur_grad
# (SLAMHIP_XCD_TILES=0: the plain order) -- parity, step time, FETCH_SIZE
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5xcd}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "fast or sift_1080p or sift_vga or batch_pipeline or reuses_fast or gradient_border" > $O/${tag}_tests.log 2>&1 \
    || { echo "tests failed"; tail -20 $O/${tag}_tests.log; exit 1; }
echo "tests $(tail -1 $O/${tag}_tests.log)"
for v in 0 1 0 1; do
    SLAMHIP_XCD_TILES=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline > $O/${tag}_$v.json 2> $O/${tag}_$v.err \
        || { echo "bench $v rc=$?"; tail -c 800 $O/${tag}_$v.err; exit 1; }
    python3 - $O/${tag}_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("kernels_sequential") or d["kernels"]
print("xcd", sys.argv[2], "value", round(d["value"]), "ms", round(d["ms_per_step"], 3),
      {k: round(v["avg_ms"], 3) for k, v in ks.items()})
PY
done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
    SLAMHIP_XCD_TILES=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/${tag}_fetch$v -o run -- python3 $R/bench.py --no-extra --no-cpu-baseline --steps 3 --warmup 1 > $O/${tag}_fetch$v.log 2>&1 || { echo "fetch $v rc=$?"; exit 1; }
done
cd $R
for v in 0 1; do
python3 - $(find $O/${tag}_fetch$v -name '*counter_collection.csv' | head -1) $v <<'PY'
import csv, sys
from collections import defaultdict
tot = defaultdict(float); cnt = defaultdict(int)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    for k in ("fast_detect", "sift_blur_grad"):
        if k in n:
            tot[k] += float(r["Counter_Value"]); cnt[k] += 1
print("xcd", sys.argv[2], {k: round(tot[k] / max(1, cnt[k]) * 1024 * 2 / 1e9, 3) for k in tot}, "GB per launch (FETCH_SIZE x2)")
PY
done
