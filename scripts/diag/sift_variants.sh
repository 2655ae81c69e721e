#!/bin/bash
# sift_desc timing of library variants (scripts/diag/lib_sift_<v>.so), each in
# its own copy of the package under /tmp.  Timing only: variants may be wrong.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for v in "$@"; do
    D=/tmp/sv_$v
    rm -rf $D && mkdir -p $D && cp -r $R/slam-indoor-code_amd/slamhip $D/ && cp $R/bench.py $D/
    cp $R/scripts/diag/lib_sift_$v.so $D/slamhip/libslamhip.so
    sed -i "s#sys.path.insert(0, os.path.join(ROOT, \"slam-indoor-code_amd\"))#sys.path.insert(0, \"$D\")#; s#^ROOT = .*#ROOT = \"$R\"#" $D/bench.py
    timeout -k 5 120 python3 $D/bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline > $R/gpurun_out/sv_$v.json 2>$R/gpurun_out/sv_$v.err || exit $?
    python3 -c "
import json
d = json.loads(open('$R/gpurun_out/sv_$v.json').read().strip().splitlines()[-1])
print('$v', 'sift_desc', round(d['kernels']['sift_desc']['avg_ms'], 4), 'step', round(d['ms_per_step'], 3))"
done
