mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s4_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/s4_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/s4_bench.json 2> gpurun_out/s4_bench.err || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/s4_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: round(v['avg_ms'],3) for k,v in d['kernels'].items()})"
