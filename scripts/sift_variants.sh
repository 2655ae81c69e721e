#!/bin/bash
# GPU box: parity of the SIFT kernels, then bench the descriptor kernel variants (env-selected)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "sift_1080p or batch_pipeline_sift" > gpurun_out/var_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/var_pytest.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for v in "band:" "noload:SLAMHIP_SIFT_BAND_MODE=2" "tab:SLAMHIP_SIFT_KERNEL=tab"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/var_$name.json 2> gpurun_out/var_$name.err || { echo "$name failed"; tail -5 gpurun_out/var_$name.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/var_$name.json'));print('$name', round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()})"
done
