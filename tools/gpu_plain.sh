#!/bin/bash
# Tables built by VALU (product) against the LDS-DMA copies (diag "old"): parity, then A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_tx_fcs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_plain.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/pytest_plain.log; exit 1; }
tail -2 gpurun_out/pytest_plain.log
CFGS=${CFGS:-c2} bash tools/gpu_abk.sh ${PAIRS:-old:4 base:4 old:5 base:5 old:4 base:4 old:5 base:5}
