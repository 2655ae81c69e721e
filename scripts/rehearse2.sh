#!/bin/bash
# multi-rank bench rehearsal on one card: N ranks (default 4: 210 candidates
# shard 53/53/52/52) share the GPU, gloo carries the device tensors; the
# headline loop and the with-BA leg (rank 0 solves, broadcasts) both run.
# The bench line itself always uses RCCL.
set -o pipefail
N=${1:-4}
mkdir -p gpurun_out
SLAMHIP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $N --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/rehearse$N.json 2> gpurun_out/rehearse$N.err || { echo "failed"; tail -20 gpurun_out/rehearse$N.err; exit 1; }
grep '^{' gpurun_out/rehearse$N.json | python -c "
import json,sys; d=json.loads(sys.stdin.read())
w=d['with_ba']
print(d['n_gpus'], round(d['value'],1), round(d['ms_per_step'],3), d['scaling'], 'with_ba', round(w['frames_per_s'],1), w.get('ba_final_rmse'), w.get('oracle', {}).get('parity_ok'))"
