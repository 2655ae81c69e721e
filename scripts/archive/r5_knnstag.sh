#!/bin/bash
# round-5 kNN A/B: workgroup start stagger (KNN_STAGGER builds, scripts/diag/lib_sift_knnstag*.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5ks}
mkdir -p $O
cp slam-indoor-code_amd/slamhip/libslamhip.so /tmp/lib_base.so
for v in base 2 4 8 base 4; do
    if [ $v = base ]; then cp /tmp/lib_base.so slam-indoor-code_amd/slamhip/libslamhip.so
    else cp scripts/diag/lib_sift_knnstag$v.so slam-indoor-code_amd/slamhip/libslamhip.so; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline > $O/${tag}_$v.json 2> $O/${tag}_$v.err \
        || { echo "bench $v rc=$?"; tail -c 800 $O/${tag}_$v.err; exit 1; }
    python3 - $O/${tag}_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("kernels_sequential") or d["kernels"]
print("stagger", sys.argv[2], "value", round(d["value"]), "ms", round(d["ms_per_step"], 3), "knn", round(ks["knn_mfma"]["avg_ms"], 3),
      "frac", round(d["rooflines"]["knn_mfma"]["frac"], 3))
PY
done
cp /tmp/lib_base.so slam-indoor-code_amd/slamhip/libslamhip.so
