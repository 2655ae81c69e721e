#!/bin/bash
# headline step per PipelinedScan overlap mode at the per-rank batch sizes of
# the strong-scaling layouts (210 / N): step ms, frames/s and per-family kernel ms
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for B in ${BATCHES:-210 27}; do
    for M in ${MODES:-knn desc_end desc_start}; do
        timeout -k 10 120 python3 $R/bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline --batch $B --overlap $M \
            > $R/gpurun_out/ov_${B}_$M.json 2> $R/gpurun_out/ov_${B}_$M.err || exit $?
        python3 -c "
import json
d = json.loads(open('$R/gpurun_out/ov_${B}_$M.json').read().strip().splitlines()[-1])
print($B, '$M', 'step_ms', round(d['ms_per_step'], 3), 'fps', round(d['value']), {k: round(v['avg_ms'], 3) for k, v in d['kernels'].items()})"
    done
done
