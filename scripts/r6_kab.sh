#!/bin/bash
# Descriptor-kernel A/B at several batch sizes: each variant is LIB:ENV (LIB =
# base for the in-tree library or a scripts/diag/lib_sift_<LIB>.so build, ENV an
# environment assignment), each run twice, interleaved, short bench each.
# usage: BATCHES="210 27" scripts/r6_kab.sh TAG base:SLAMHIP_SIFT_COLW=1 base:SLAMHIP_SIFT_COLW=0 g1:X=1
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
LIB=$R/slam-indoor-code_amd/slamhip/libslamhip.so
cp $LIB /tmp/lib_base.so
for b in ${BATCHES:-210 27}; do
    steps=$(( b >= 100 ? 20 : 60 ))
    for rep in 1 2; do
        for v in "$@"; do
            l=${v%%:*}; e=${v#*:}
            if [ "$l" = base ]; then cp /tmp/lib_base.so $LIB; else cp $R/scripts/diag/lib_sift_$l.so $LIB || exit 1; fi
            f=$O/${TAG}_${b}_${l}_${e//[^A-Za-z0-9]/_}_$rep
            env $e timeout -k 10 120 python3 $R/bench.py --batch $b --steps $steps --warmup 3 --no-extra --no-cpu-baseline \
                > $f.json 2> $f.err || { cp /tmp/lib_base.so $LIB; exit 1; }
            python3 -c "
import json
d = json.loads(open('$f.json').read().strip().splitlines()[-1])
k = d.get('kernels_sequential') or d['kernels']
print('b$b $l $e', 'step', round(d['ms_per_step'], 3), 'fps', round(d['value']), 'sift', round(k['sift_desc']['avg_ms'], 3), d['config'].get('sift_desc_kernel'))"
        done
    done
done
cp /tmp/lib_base.so $LIB
