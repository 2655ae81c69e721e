#!/bin/bash
# GPU box: rocprofv3 kernel-trace summary + separate HBM-counter passes of the
# bench, then the full default bench line (with the CPU baseline).
# usage: scripts/profile.sh TAG      (outputs under gpurun_out/TAG_*)
set -o pipefail
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
step() {   # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $O/${TAG}_${name}.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
B="python3 $R/bench.py --no-cpu-baseline"
step kt 400 rocprofv3 --kernel-trace --stats -f csv -d $O/${TAG}_kt -o run -- $B --no-extra --steps 10 --warmup 3
step ktall 400 rocprofv3 --kernel-trace --stats -f csv -d $O/${TAG}_ktall -o run -- $B --steps 5 --warmup 2
step fetch 400 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/${TAG}_fetch -o run -- $B --no-extra --steps 3 --warmup 1
step write 400 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/${TAG}_write -o run -- $B --no-extra --steps 3 --warmup 1
cd $R
step bench 600 python3 bench.py
cp $O/${TAG}_bench.log $O/${TAG}_bench.json
if [ -n "$SQ" ]; then
    cd /tmp
    step sq 300 rocprofv3 --pmc $SQ -f csv -d $O/${TAG}_sq -o run -- $B --no-extra --steps 3 --warmup 1
fi
