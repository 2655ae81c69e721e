#!/bin/bash
# GPU box: separate rocprofv3 counter passes of a short bench, restricted to one kernel.
# usage: scripts/pmc_kernel.sh TAG KERNEL_REGEX "PASS1 COUNTERS" "PASS2 COUNTERS" ...
TAG=$1; RX=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "$@"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $pass --kernel-include-regex "$RX" -f csv -d $R/gpurun_out/${TAG}_p$i -o run -- \
        python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > $R/gpurun_out/${TAG}_p$i.log 2>&1
    rc=$?
    echo "pass $i ($pass) rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
exit 0
