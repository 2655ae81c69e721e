#!/bin/bash
# round-5: PnP parity (ordered bit-exact, pairwise within tolerance) with the
# level-parallel 12 x 12 Jacobi SVD in pnp_hyp; PnP alone; the 24-frame
# pipeline (worker-chained post-search work) with each sum mode
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5d5}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_cycle.py -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -m gpu -k "pnp or cycle_gpu" > $O/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/${tag}_tests.log; exit 1; }
echo "tests $(tail -1 $O/${tag}_tests.log)"
for v in 0 1; do
    SLAMHIP_PNP_SUMS=$v SLAMHIP_PNP_TIMING=1 timeout -k 10 120 python3 -u scripts/diag/pnp_iso.py > $O/${tag}_pnp_$v.txt 2>&1 || { echo "pnp rc=$?"; exit 1; }
    echo "sums=$v $(tail -1 $O/${tag}_pnp_$v.txt) $(grep 'pnp n' $O/${tag}_pnp_$v.txt | tail -1)"
done
for v in 0 1 0 1; do
    SLAMHIP_PNP_SUMS=$v timeout -k 10 300 python3 -u scripts/diag/pipe24.py 3 > $O/${tag}_p24_$v.txt 2>&1 || { echo "p24 rc=$?"; tail -5 $O/${tag}_p24_$v.txt; exit 1; }
    echo "sums=$v $(grep '"frames_per_s"' $O/${tag}_p24_$v.txt | cut -c17-22 | tr '\n' ' ')"
    grep -o '"pose_t_max_abs_diff": [^,]*\|"poses_before_first_ba_bitexact": [a-z]*\|"parity_ok": [a-z]*' $O/${tag}_p24_$v.txt | tr '\n' ' '; echo
done
