#!/bin/bash
# round-end evidence: full GPU parity suite, smoke(), then profile.sh (kernel
# trace, FETCH/WRITE passes, the default bench line with its CPU baseline)
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 2; }
tail -1 gpurun_out/${TAG}_smoke.log
SQ="${SQ:-SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE}" bash scripts/profile.sh ${TAG}
