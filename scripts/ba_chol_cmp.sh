#!/bin/bash
# BA window timing for the two Cholesky variants at W = 8 / 10 / 16 (GPU box)
mkdir -p gpurun_out
for v in wave rows; do
  for cfg in "8 10000" "10 12000" "16 40000"; do
    SLAMHIP_BA_CHOL=$v timeout -k 10 120 python3 scripts/ba_bench.py $cfg > "gpurun_out/cholcmp_${v}_${cfg// /_}.json" 2>/dev/null || exit $?
  done
done
