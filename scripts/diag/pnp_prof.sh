#!/bin/bash
# kernel trace of pipeline-sized solvePnPRansac calls (scripts/pnp_probe.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/pnpprof -o run -- python3 $R/scripts/pnp_probe.py > $R/gpurun_out/pnpprof.log 2>&1
