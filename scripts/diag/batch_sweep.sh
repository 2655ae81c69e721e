#!/bin/bash
# per-rank batch sizes of the strong-scaling layouts (210 / N) on one GPU: the headline step's time and kernels
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for B in ${@:-210 105 53 27}; do
    timeout -k 10 120 python3 $R/bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline --batch $B > $R/gpurun_out/bs_$B.json 2>$R/gpurun_out/bs_$B.err || exit $?
    python3 -c "
import json
d = json.loads(open('$R/gpurun_out/bs_$B.json').read().strip().splitlines()[-1])
print($B, 'step_ms', round(d['ms_per_step'], 3), 'fps', round(d['value']), {k: round(v['avg_ms'], 3) for k, v in d['kernels'].items()})"
done
