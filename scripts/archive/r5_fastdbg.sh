#!/bin/bash
# fast_detect timing probes (SLAMHIP_FAST_DBG: 1 no gray store, 2 no candidates,
# 4 no NMS; results wrong, timing only) on the headline batch
set -o pipefail
O=gpurun_out
mkdir -p $O
for d in 0 1 2 4 7 0; do
    SLAMHIP_FAST_DBG=$d timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline > $O/fdbg_$d.json 2>$O/fdbg_$d.err || { echo "d=$d failed"; tail -c 600 $O/fdbg_$d.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/fdbg_$d.json').read().strip().splitlines()[-1])
ks=d.get('kernels_sequential') or d['kernels']
print('dbg $d fast_detect', round(ks['fast_detect']['avg_ms'],3))
"
done
