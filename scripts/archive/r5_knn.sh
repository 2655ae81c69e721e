#!/bin/bash
# round-5 kNN A/B: parity of the SIFT L2 matcher under each kernel variant
# (SLAMHIP_KNN_PIPE 0 = knn_mfma_pk QT 2, 2 = knn_pipe QT 1 at 4 waves/SIMD,
# 3 = knn_mfma_pk QT 1), then the headline step under each
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5knn}
shift
variants=${@:-0 2 3 0 2}
for v in $variants; do
    SLAMHIP_KNN_PIPE=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 \
        --timeout-method thread -p no:cacheprovider -k "knn or configs4 or batch_extract_match" \
        > gpurun_out/${tag}_tests_$v.log 2>&1 || { echo "tests v=$v failed"; tail -30 gpurun_out/${tag}_tests_$v.log; exit 1; }
    echo "v=$v $(tail -1 gpurun_out/${tag}_tests_$v.log)"
    SLAMHIP_KNN_PIPE=$v timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline \
        > gpurun_out/${tag}_bench_$v.json 2> gpurun_out/${tag}_bench_$v.err \
        || { echo "bench v=$v rc=$?"; tail -c 1500 gpurun_out/${tag}_bench_$v.err; exit 1; }
    python3 - gpurun_out/${tag}_bench_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("kernels_sequential") or d["kernels"]
print(sys.argv[1], "value", round(d["value"]), "ms", round(d["ms_per_step"], 3),
      {k: round(v["avg_ms"], 3) for k, v in ks.items()}, "knn_frac", round(d["rooflines"]["knn_mfma"]["frac"], 3))
PY
done
