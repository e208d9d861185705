#!/bin/bash
# 16-lane kernel check: wdebug sweep, parity suite, then A/B against the one-pass kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python tools/wdebug.py > gpurun_out/wdebug5.log 2>&1 || { echo "WDEBUG FAILED"; tail -20 gpurun_out/wdebug5.log; exit 1; }
grep -E "^[a-z]" gpurun_out/wdebug5.log | grep -v "bad=0" ; echo "wdebug done"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_tx_fcs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_w5.log 2>&1 || { echo "PARITY FAILED"; tail -30 gpurun_out/pytest_w5.log; exit 1; }
tail -1 gpurun_out/pytest_w5.log
STEPS=1000 WARM=500 bash tools/gpu_abk.sh base:1 base:3
