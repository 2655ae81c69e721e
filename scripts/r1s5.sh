#!/bin/bash
# round-1 session-5 GPU check: parity suite, overlap on/off bench, 2-rank gloo
# rehearsal of the multi-rank step on one card.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r1s5_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r1s5_pytest.log; exit 1; }
tail -3 gpurun_out/r1s5_pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/r1s5_on.json 2> gpurun_out/r1s5_on.err || exit 2
SLAMHIP_OVERLAP=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/r1s5_off.json 2> gpurun_out/r1s5_off.err || exit 3
SLAMHIP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-extra \
    > gpurun_out/r1s5_gloo2.json 2> gpurun_out/r1s5_gloo2.err || { echo "gloo2 failed"; tail -20 gpurun_out/r1s5_gloo2.err; exit 4; }
python - <<'PY'
import json
for t in ("on", "off", "gloo2"):
    for line in open(f"gpurun_out/r1s5_{t}.json"):
        if line.startswith("{"):
            d = json.loads(line)
            print(t, round(d["value"], 1), round(d["ms_per_step"], 3), {k: round(v["avg_ms"], 3) for k, v in d.get("kernels", {}).items()})
PY
