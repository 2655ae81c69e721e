#!/bin/bash
# round-5: PnP pairwise refinement sums -- parity (ordered bit-exact, pairwise
# within tolerance), PnP alone, and the 24-frame pipeline with each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
tag=${1:-r5d5}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "pnp" > $O/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/${tag}_tests.log; exit 1; }
echo "tests $(tail -1 $O/${tag}_tests.log)"
for v in 0 1; do
    SLAMHIP_PNP_SUMS=$v SLAMHIP_PNP_TIMING=1 timeout -k 10 120 python3 -u scripts/diag/pnp_iso.py > $O/${tag}_pnp_$v.txt 2>&1 || { echo "pnp rc=$?"; exit 1; }
    echo "sums=$v $(tail -1 $O/${tag}_pnp_$v.txt) $(grep 'pnp n' $O/${tag}_pnp_$v.txt | tail -1)"
done
for v in 0 1 0 1; do
    SLAMHIP_PNP_SUMS=$v timeout -k 10 300 python3 -u scripts/diag/pipe24.py 2 > $O/${tag}_p24_$v.txt 2>&1 || { echo "p24 rc=$?"; tail -5 $O/${tag}_p24_$v.txt; exit 1; }
    echo "sums=$v $(grep '"frames_per_s"' $O/${tag}_p24_$v.txt | cut -c1-40 | tr '\n' ' ')"
    grep -o '"pose_t_max_abs_diff": [^,]*\|"poses_before_first_ba_bitexact": [a-z]*\|"parity_ok": [a-z]*' $O/${tag}_p24_$v.txt | tr '\n' ' '; echo
done
