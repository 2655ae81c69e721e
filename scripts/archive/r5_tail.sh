#!/bin/bash
# round-5 strong-scaling tail A/B of sift_desc_band: keypoint-group order
# (SLAMHIP_SIFT_BAND_ORDER=0: workgroup-major, the round-4 order; 1: wave-major)
# and the last partial round as part-walks (SLAMHIP_SIFT_BAND_SPLIT=0 off, 1
# auto; SLAMHIP_SIFT_BAND_PARTS=2 / 4 forces the part count); parity first, then
# the headline step at --batch 27 (configs[3]'s per-rank shard) and 210
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5tail}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "sift_1080p or sift_vga or fast_sift_4k or uniform_angle or tiny_uniform or batch_pipeline_sift or band_split" \
    > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
echo "tests $(tail -1 gpurun_out/${tag}_tests.log)"
run() {   # batch order split parts
    local n=${tag}_b$1_o$2s$3p$4
    SLAMHIP_SIFT_BAND_ORDER=$2 SLAMHIP_SIFT_BAND_SPLIT=$3 SLAMHIP_SIFT_BAND_PARTS=$4 timeout -k 10 300 python -u bench.py \
        --batch $1 --steps 20 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/$n.json 2> gpurun_out/$n.err \
        || { echo "bench $n rc=$?"; tail -c 1500 gpurun_out/$n.err; exit 1; }
    python3 - gpurun_out/$n.json "$*" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("kernels_sequential") or d["kernels"]
print("batch/order/split/parts", sys.argv[2], "value", round(d["value"]), "ms", round(d["ms_per_step"], 3),
      {k: round(v["avg_ms"], 3) for k, v in ks.items()})
PY
}
for rep in 1 2; do
    run 27 1 0 0 && run 27 1 1 2 && run 27 1 1 4 && run 27 1 1 0 || exit 1
done
for rep in 1 2; do
    run 210 0 0 0 && run 210 1 0 0 && run 210 1 1 0 || exit 1
done
