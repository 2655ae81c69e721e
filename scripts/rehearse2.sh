#!/bin/bash
# multi-rank step rehearsal on one card: 2 ranks share the GPU, gloo carries the
# device tensors (the bench line itself always uses RCCL)
set -o pipefail
mkdir -p gpurun_out
SLAMHIP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-extra \
    > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err || { echo "failed"; tail -20 gpurun_out/rehearse2.err; exit 1; }
grep '^{' gpurun_out/rehearse2.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], round(d['value'],1), round(d['ms_per_step'],3))"
